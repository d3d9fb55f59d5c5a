# tests -> bench b/c/e -> phase costs (each step time-limited, stop at first failure)
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-v4}
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/tests_$TAG.log 2>&1; rc=$?
tail -5 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/tests_$TAG.log | head -30; exit $rc; }
for c in b c e; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err || { tail gpurun_out/bench_${TAG}_$c.err; exit 1; }
  cat gpurun_out/bench_${TAG}_$c.json
done
timeout -k 10 400 python tools/phase_cost.py b > gpurun_out/phase_${TAG}_b.log 2>&1; cat gpurun_out/phase_${TAG}_b.log
