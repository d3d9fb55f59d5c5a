# r03c: resident latency (one round trip per request), mixed HP passes in descriptor order:
# tests, latency, bench E twice, PMC of E (traffic). Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03c
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
for k in 1 2; do
  step bench_e_$k
  timeout -k 10 300 python bench.py --config e --no-cpu-baseline > $O/bench_e_$k.json 2> $O/bench_e_$k.err || { tail $O/bench_e_$k.err; exit 1; }
  cat $O/bench_e_$k.json
done
step prof_e
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_e -o run -- python3 bench.py --config e --no-cpu-baseline > $O/prof_e.json 2> $O/prof_e.err || { tail $O/prof_e.err; exit 1; }
step pmc_e
bash tools/gpu_pmc.sh e 1048576 && python3 tools/pmc_summary.py gpurun_out/pmc_e --json $O/pmc_traffic_e.json > $O/pmc_e.txt || exit 1
echo R03C_OK
