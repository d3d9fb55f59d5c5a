# Round-4 call Q: config E with the ChaCha20 list on the persistent grid (product) against the
# one-shot grid (MQ_CC_LIST=0), both single-key; alternating runs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04q}
mkdir -p $O
for r in 1 2 3; do
  for v in persistent oneshot; do
    if [ $v = oneshot ]; then E="MQ_CC_LIST=0"; else E="MQ_CC_LIST=1"; fi
    env $E timeout -k 10 300 python3 bench.py --no-cpu-baseline --config e --steps 50 > $O/e_$v.$r.json 2> $O/e_$v.$r.err || { tail $O/e_$v.$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], r['seal_ms'], r['open_ms'])" $O/e_$v.$r.json
  done
done
echo R04Q_DONE
