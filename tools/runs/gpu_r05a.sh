# Round-5 call A: the round's first tree (ADVICE r04 fixes, stream-handle tests, e2e on separate copy
# streams): every GPU test, the driver's bench command with the end-to-end pipeline, a full length
# sweep of both suites (failures reported, not trimmed).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05a}
mkdir -p $O
echo "== narrow tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_narrow.py tests/test_gpu_streams.py -x -q --timeout 150 --timeout-method thread > $O/tests_narrow.log 2>&1 || { tail -40 $O/tests_narrow.log; exit 1; }
tail -1 $O/tests_narrow.log
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
echo "== bench $(date +%T)"
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --e2e > $O/bench_b.json 2> $O/bench_b.err || { tail $O/bench_b.err; exit 1; }
grep '^{' $O/bench_b.json | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('B', d['value'], d['ms_per_step'], d['roofline']['frac'], json.dumps(d['end_to_end']))"
echo "== sweep $(date +%T)"
timeout -k 10 400 python3 tools/len_sweep.py both 64 128 256 448 700 1200 1232 1280 1350 1452 1500 1600 2048 4096 > $O/len_sweep.txt 2>&1 || { tail $O/len_sweep.txt; exit 1; }
cat $O/len_sweep.txt
echo R05A_DONE
