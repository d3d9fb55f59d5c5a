# Round-4 call Z: config E with the key-segmented single-key AES kernels forced on (MQ_AES_SEG=1:
# 4096 Initial rows of ~64 packets each) against the multi-key kernel (product), alternating;
# mixed-batch tests with the forced path.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04z}
mkdir -p $O
echo "== tests (forced segmented) $(date +%T)"
MQ_AES_SEG=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  for v in product seg; do
    if [ $v = product ]; then E=""; else E="MQ_AES_SEG=1"; fi
    env $E timeout -k 10 200 python3 bench.py --config e --steps 20 --warmup 5 --no-cpu-baseline > $O/$v.$r.json 2> $O/$v.$r.err || { tail $O/$v.$r.err; exit 1; }
    echo "$v $r $(python3 -c "import json,sys; d=json.loads([l for l in open('$O/$v.$r.json') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])")"
  done
done
echo R04Z_DONE
