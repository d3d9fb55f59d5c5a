# GPU round trip: parity tests, then the bench line (each step time-limited; stop at first failure)
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-run}
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/tests_$TAG.log 2>&1; rc=$?
tail -5 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || { echo "tests failed rc=$rc"; exit $rc; }
timeout -k 10 400 python bench.py ${BENCH_ARGS} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err; rc=$?
cat gpurun_out/bench_$TAG.json
[ $rc -eq 0 ] || { tail -20 gpurun_out/bench_$TAG.err; exit $rc; }
