# Round-4 call ZL: the final tree — all GPU tests, bench lines B (driver's command) and E, smoke.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04zl}
mkdir -p $O
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_b.json 2> $O/bench_b.err || { tail $O/bench_b.err; exit 1; }
grep '^{' $O/bench_b.json | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('B', d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 300 python3 bench.py --config e --no-cpu-baseline > $O/bench_e.json 2> $O/bench_e.err || { tail $O/bench_e.err; exit 1; }
grep '^{' $O/bench_e.json | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('E', d['value'], d['ms_per_step'])"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo R04ZL_DONE
