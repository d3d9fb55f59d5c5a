# Final tree after the resident mailbox fix: all GPU tests, the default bench line (B, with CPU
# baselines), E and C/1024 lines, per-packet latency, smoke. Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05final4}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python bench.py > $O/bench_b.json 2> $O/bench_b.err || { tail $O/bench_b.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --config e > $O/bench_e.json 2> $O/bench_e.err || { tail $O/bench_e.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --config c --keys 1024 > $O/bench_ck.json 2> $O/bench_ck.err || { tail $O/bench_ck.err; exit 1; }
python -c "import json; [print(n, json.load(open('$O/bench_'+n+'.json'))['value']) for n in ('b','e','ck')]"
timeout -k 10 300 python tools/bench_latency.py > $O/latency.json 2> $O/latency.err || { tail $O/latency.err; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo ROUND_OK
