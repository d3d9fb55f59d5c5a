# resident per-packet path: its tests, then the latency tool
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-lat}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python tools/bench_latency.py > $O/latency.json 2> $O/latency.err || { tail $O/latency.err; exit 1; }
cat $O/latency.json
