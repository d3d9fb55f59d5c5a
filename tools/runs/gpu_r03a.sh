# r03a: parity tests (incl. config-D shards, per-thread devices, two-stream mixed batches, the
# recv re-seal), then bench E (ChaCha list forked beside the AES kernels), C with 1024 keys, B,
# and the 2-rank gloo rehearsal of config E (per-rank parity). Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03a
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step ubench8
timeout -k 10 120 ./tools/ubench/ubench8 > $O/ubench8.txt 2>&1 || { cat $O/ubench8.txt; exit 1; }
cat $O/ubench8.txt
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
step bench_e
timeout -k 10 300 python bench.py --config e --no-cpu-baseline > $O/bench_e.json 2> $O/bench_e.err || { tail $O/bench_e.err; exit 1; }
cat $O/bench_e.json
step bench_e_nofork
MQ_FORK=0 timeout -k 10 300 python bench.py --config e --no-cpu-baseline > $O/bench_e_nofork.json 2> $O/bench_e_nofork.err || { tail $O/bench_e_nofork.err; exit 1; }
cat $O/bench_e_nofork.json
step bench_c_k1024
timeout -k 10 300 python bench.py --config c --keys 1024 --no-cpu-baseline > $O/bench_c_k1024.json 2> $O/bench_c_k1024.err || { tail $O/bench_c_k1024.err; exit 1; }
cat $O/bench_c_k1024.json
step bench_b
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_b.json 2> $O/bench_b.err || { tail $O/bench_b.err; exit 1; }
cat $O/bench_b.json
step gloo_2rank_e
MQ_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --config e --no-cpu-baseline > $O/bench_e_2rank_gloo.json 2> $O/bench_e_2rank_gloo.err || { tail $O/bench_e_2rank_gloo.err; exit 1; }
cat $O/bench_e_2rank_gloo.json
echo R03A_OK
