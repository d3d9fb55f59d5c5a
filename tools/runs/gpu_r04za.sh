# Round-4 call ZA: config C with few keys (2, 3, 4, 16, 1024): does the key-segmented path (chosen at
# >= 512 packets per row) put a large row's segment on one workgroup?
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04za}
mkdir -p $O
for k in 2 3 16 1024; do
  timeout -k 10 200 python3 bench.py --config c --keys $k --steps 3 --warmup 1 --warmup-seconds 0 --no-cpu-baseline > $O/c$k.json 2> $O/c$k.err || { tail $O/c$k.err; exit 1; }
  echo "keys $k $(python3 -c "import json,sys; d=json.loads([l for l in open('$O/c$k.json') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])")"
done
echo R04ZA_DONE
