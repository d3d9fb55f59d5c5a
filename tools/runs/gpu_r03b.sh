# r03b: tests, bench E (hot AES fork only), B with CPU baselines, C; rocprofv3 kernel stats of
# B/C/E; PMC passes of B and E (HBM traffic of the new seal composites). Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03b
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step tests_resident
timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py -x -v --timeout 120 --timeout-method thread > $O/tests_resident.log 2>&1 || { tail -40 $O/tests_resident.log; exit 1; }
tail -2 $O/tests_resident.log
step latency
timeout -k 10 300 python tools/bench_latency.py > $O/latency.json 2> $O/latency.err || { tail $O/latency.err; exit 1; }
cat $O/latency.json
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
step bench_e
timeout -k 10 300 python bench.py --config e --no-cpu-baseline > $O/bench_e.json 2> $O/bench_e.err || { tail $O/bench_e.err; exit 1; }
cat $O/bench_e.json
step bench_c
timeout -k 10 300 python bench.py --config c --no-cpu-baseline > $O/bench_c.json 2> $O/bench_c.err || { tail $O/bench_c.err; exit 1; }
cat $O/bench_c.json
step bench_b
timeout -k 10 400 python bench.py > $O/bench_b.json 2> $O/bench_b.err || { tail $O/bench_b.err; exit 1; }
cat $O/bench_b.json
for c in b c e; do
  step prof_$c
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o run -- python3 bench.py --config $c --no-cpu-baseline > $O/prof_$c.json 2> $O/prof_$c.err || { tail $O/prof_$c.err; exit 1; }
done
step pmc_b
bash tools/gpu_pmc.sh b 1048576 && python3 tools/pmc_summary.py gpurun_out/pmc_b --tiles 131072 --json $O/pmc_traffic_b.json > $O/pmc_b.txt || exit 1
step pmc_e
bash tools/gpu_pmc.sh e 1048576 && python3 tools/pmc_summary.py gpurun_out/pmc_e --json $O/pmc_traffic_e.json > $O/pmc_e.txt || exit 1
echo R03B_OK
