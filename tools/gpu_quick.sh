# Quick GPU validation: parity tests, bench config B (with CPU baselines), the 2-rank launcher
# rehearsal on one GPU (gloo), per-packet latency. Every GPU step is time-limited; stops at the
# first failure.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-q}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python bench.py > $O/bench_b.json 2> $O/bench_b.err || { tail $O/bench_b.err; exit 1; }
cat $O/bench_b.json
MQ_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --no-cpu-baseline > $O/bench_b_2rank_gloo.json 2> $O/bench_b_2rank_gloo.err || { tail $O/bench_b_2rank_gloo.err; exit 1; }
cat $O/bench_b_2rank_gloo.json
timeout -k 10 300 python tools/bench_latency.py > $O/latency.json 2> $O/latency.err || { tail $O/latency.err; exit 1; }
cat $O/latency.json
echo QUICK_OK
