# tests -> bench -> stamps (each step time-limited, stop at first failure)
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-v3}
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/tests_$TAG.log 2>&1; rc=$?
tail -5 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/tests_$TAG.log | head -30; exit $rc; }
timeout -k 10 400 python bench.py --cpu-sample 16384 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err; rc=$?
cat gpurun_out/bench_$TAG.json
[ $rc -eq 0 ] || { tail -20 gpurun_out/bench_$TAG.err; exit $rc; }
timeout -k 10 300 python bench.py --config c --no-cpu-baseline > gpurun_out/bench_${TAG}_c.json 2>&1 || exit $?
cat gpurun_out/bench_${TAG}_c.json
timeout -k 10 300 python bench.py --config e --no-cpu-baseline > gpurun_out/bench_${TAG}_e.json 2>&1 || exit $?
cat gpurun_out/bench_${TAG}_e.json
timeout -k 10 300 python tools/stamps.py b > gpurun_out/stamps_$TAG.txt 2>&1 || exit $?
cat gpurun_out/stamps_$TAG.txt
