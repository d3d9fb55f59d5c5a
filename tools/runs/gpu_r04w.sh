# Round-4 call W: partition tiles sized by the batch's largest image per class — GPU tests, aux
# (protect / recv), config E, receive kernel stats.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04w}
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  step aux_$r
  timeout -k 10 300 python tools/bench_aux.py > $O/aux_$r.json 2> $O/aux_$r.err || { tail $O/aux_$r.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('derive', d['derive'], 'protect', d['protect'], 'recv', d['recv'])" $O/aux_$r.json
done
step bench_e
timeout -k 10 300 python3 bench.py --no-cpu-baseline --config e > $O/bench_e.json 2> $O/bench_e.err || { tail $O/bench_e.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], r['seal_ms'], r['open_ms'])" $O/bench_e.json
step prof_recv
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_recv -o run -- python3 tools/prof_aux.py recv 5 > $O/prof_recv.log 2>&1 || { tail $O/prof_recv.log; exit 1; }
grep -E "open_list|walk|gather" $O/prof_recv/run_kernel_stats.csv
echo R04W_DONE
