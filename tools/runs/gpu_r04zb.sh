# Round-4 call ZB: key-segmented AES kernels claiming list slices (product) against whole-segment
# claims (prev.so): parity tests, config C over 2 / 3 / 16 / 1024 keys, A/B on C-1024.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04zb}
mkdir -p $O
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 2 3 16 1024; do
  timeout -k 10 200 python3 bench.py --config c --keys $k --steps 20 --warmup 5 --no-cpu-baseline > $O/c$k.json 2> $O/c$k.err || { tail $O/c$k.err; exit 1; }
  echo "keys $k $(python3 -c "import json,sys; d=json.loads([l for l in open('$O/c$k.json') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])")"
done
timeout -k 10 400 python3 tools/ab.py ck 1048576 milli_quic_amd/libmq_aead.so tools/ab_libs/prev.so > $O/ab_ck.txt 2>&1 || { tail $O/ab_ck.txt; exit 1; }
cat $O/ab_ck.txt
echo R04ZB_DONE
