# Round artifacts in one gpurun call: parity tests, bench lines (B with CPU baselines, B end-to-end
# with the copy ceiling, C, E, the K = 1024-key variants), the 2-rank launcher rehearsal (gloo, one
# GPU), per-packet latency, OpenSSL scaling, rocprofv3 kernel-trace stats of B/C/E, aux components,
# PMC passes for B and C. Every GPU step is time-limited; the script stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r02}
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
step bench_b
timeout -k 10 400 python bench.py > $O/bench_b.json 2> $O/bench_b.err || { tail $O/bench_b.err; exit 1; }
cat $O/bench_b.json
step bench_b_e2e
timeout -k 10 600 python bench.py --no-cpu-baseline --e2e > $O/bench_b_e2e.json 2> $O/bench_b_e2e.err || { tail $O/bench_b_e2e.err; exit 1; }
cat $O/bench_b_e2e.json
for c in c e; do
  step bench_$c
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { tail $O/bench_$c.err; exit 1; }
  cat $O/bench_$c.json
done
for c in b c; do
  step bench_${c}_k1024
  timeout -k 10 300 python bench.py --config $c --keys 1024 --no-cpu-baseline > $O/bench_${c}_k1024.json 2> $O/bench_${c}_k1024.err || { tail $O/bench_${c}_k1024.err; exit 1; }
  cat $O/bench_${c}_k1024.json
done
step gloo_2rank
MQ_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --no-cpu-baseline > $O/bench_b_2rank_gloo.json 2> $O/bench_b_2rank_gloo.err || { tail $O/bench_b_2rank_gloo.err; exit 1; }
cat $O/bench_b_2rank_gloo.json
step latency
timeout -k 10 300 python tools/bench_latency.py > $O/latency.json 2> $O/latency.err || { tail $O/latency.err; exit 1; }
cat $O/latency.json
step ossl_scaling
{ for m in 1 2 4; do timeout -k 10 120 ./tools/ossl_scaling $m 0 64 || exit 1; done; timeout -k 10 120 ./tools/ossl_scaling 4 1 64; } > $O/ossl_scaling.txt 2>&1 || { cat $O/ossl_scaling.txt; exit 1; }
cat $O/ossl_scaling.txt
for c in b c e; do
  step prof_$c
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o run -- python3 bench.py --config $c --no-cpu-baseline > $O/prof_$c.json 2> $O/prof_$c.err || { tail $O/prof_$c.err; exit 1; }
done
step aux
timeout -k 10 300 python tools/bench_aux.py > $O/aux.json 2> $O/aux.err || { tail $O/aux.err; exit 1; }
cat $O/aux.json
step pmc
bash tools/gpu_pmc.sh b 1048576 && python3 tools/pmc_summary.py gpurun_out/pmc_b --tiles 131072 --json $O/pmc_traffic_b.json > $O/pmc_b.txt || exit 1
bash tools/gpu_pmc.sh c 1048576 && python3 tools/pmc_summary.py gpurun_out/pmc_c --tiles 131072 --json $O/pmc_traffic_c.json > $O/pmc_c.txt || exit 1
echo ROUND_OK
