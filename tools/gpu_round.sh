# Round artifacts: parity tests, bench lines (b with CPU baseline, b end-to-end, c, e),
# rocprofv3 kernel-trace stats of the bench, PMC passes for b and c. Every GPU step is
# time-limited and the script stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r01}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python bench.py > $O/bench_b.json 2> $O/bench_b.err || { tail $O/bench_b.err; exit 1; }
cat $O/bench_b.json
timeout -k 10 400 python bench.py --no-cpu-baseline --e2e > $O/bench_b_e2e.json 2> $O/bench_b_e2e.err || { tail $O/bench_b_e2e.err; exit 1; }
cat $O/bench_b_e2e.json
for c in c e; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { tail $O/bench_$c.err; exit 1; }
  cat $O/bench_$c.json
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b -o run -- python3 bench.py --no-cpu-baseline > $O/prof_b.json 2> $O/prof_b.err || { tail $O/prof_b.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c -o run -- python3 bench.py --config c --no-cpu-baseline > $O/prof_c.json 2> $O/prof_c.err || { tail $O/prof_c.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_e -o run -- python3 bench.py --config e --no-cpu-baseline > $O/prof_e.json 2> $O/prof_e.err || { tail $O/prof_e.err; exit 1; }
timeout -k 10 300 python tools/bench_aux.py > $O/aux.json 2> $O/aux.err || { tail $O/aux.err; exit 1; }
cat $O/aux.json
bash tools/gpu_pmc.sh b 1048576 && python3 tools/pmc_summary.py gpurun_out/pmc_b --tiles 131072 --json $O/pmc_traffic_b.json > $O/pmc_b.txt || exit 1
bash tools/gpu_pmc.sh c 1048576 && python3 tools/pmc_summary.py gpurun_out/pmc_c --tiles 131072 --json $O/pmc_traffic_c.json > $O/pmc_c.txt || exit 1
echo ROUND_OK
