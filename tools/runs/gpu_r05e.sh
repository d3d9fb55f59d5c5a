# Round-5 call E: segmented receive walk (runs over several waves, verified chained starts,
# sequential fallback): receive tests first (long runs, full size), all GPU tests, bench_aux with
# few-connection receive runs, bench B and E.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05e}
mkdir -p $O
echo "== recv tests $(date +%T)"
timeout -k 10 800 python -u -m pytest tests/test_gpu_recv.py -x -v --timeout 300 --timeout-method thread > $O/tests_recv.log 2>&1 || { tail -40 $O/tests_recv.log; exit 1; }
grep -E "PASS|FAIL" $O/tests_recv.log | tail -20
echo "== aux $(date +%T)"
timeout -k 10 600 python3 tools/bench_aux.py 3 > $O/aux.json 2> $O/aux.err || { tail $O/aux.err; exit 1; }
cat $O/aux.json
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
echo "== bench $(date +%T)"
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_b.json 2> $O/bench_b.err || { tail $O/bench_b.err; exit 1; }
grep '^{' $O/bench_b.json | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('B', d['value'], d['ms_per_step'], d['roofline']['frac'])"
echo R05E_DONE
