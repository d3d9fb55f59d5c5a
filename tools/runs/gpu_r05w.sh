# r05w: partition with keyed ranks from the count kernel and code-driven scatter — parity tests,
# partition stamps (E, C/1024), bench E and C/1024, kernel stats of E. Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05w}
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
step stamps
timeout -k 10 150 python -u tools/part_count_stamps.py e > $O/part_e.txt 2>&1 || { tail $O/part_e.txt; exit 1; }
timeout -k 10 150 python -u tools/part_count_stamps.py ck > $O/part_ck.txt 2>&1 || { tail $O/part_ck.txt; exit 1; }
for a in "e --config e" "ck --config c --keys 1024"; do
  set -- $a; name=$1; shift
  step bench_$name
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/bench_$name.json 2> $O/bench_$name.err || { tail $O/bench_$name.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/bench_$name.json')); print('$name', d['value'], d['roofline']['seal_ms'], d['roofline']['open_ms'])"
done
step prof_e
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_e -o run -- python3 bench.py --no-cpu-baseline --config e > $O/prof_e.json 2> $O/prof_e.err || { tail $O/prof_e.err; exit 1; }
echo ALL_OK
