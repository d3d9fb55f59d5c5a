# Round-5 call B: narrow regions of mixed batches' ChaCha20 lists: narrow tests first, every GPU test,
# the bench lines B and E, the length sweep.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05b}
mkdir -p $O
echo "== narrow tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_narrow.py tests/test_gpu_streams.py -x -q --timeout 150 --timeout-method thread > $O/tests_narrow.log 2>&1 || { tail -40 $O/tests_narrow.log; exit 1; }
tail -1 $O/tests_narrow.log
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
echo "== bench $(date +%T)"
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_b.json 2> $O/bench_b.err || { tail $O/bench_b.err; exit 1; }
timeout -k 10 300 python3 bench.py --config e --no-cpu-baseline > $O/bench_e.json 2> $O/bench_e.err || { tail $O/bench_e.err; exit 1; }
MQ_CC_NARROW=0 timeout -k 10 300 python3 bench.py --config e --no-cpu-baseline > $O/bench_e0.json 2> $O/bench_e0.err || { tail $O/bench_e0.err; exit 1; }
grep "^{" $O/bench_e0.json | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('E no-narrow', d['value'], d['ms_per_step'], d['roofline']['seal_ms'], d['roofline']['open_ms'])"
grep "^{" $O/bench_e.json | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('E', d['value'], d['ms_per_step'], d['roofline']['seal_ms'], d['roofline']['open_ms'])"
grep '^{' $O/bench_b.json | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('B', d['value'], d['ms_per_step'], d['roofline']['frac'])"
echo "== sweep $(date +%T)"
timeout -k 10 400 python3 tools/len_sweep.py c 64 128 256 448 700 1200 > $O/len_sweep.txt 2>&1 || { tail $O/len_sweep.txt; exit 1; }
cat $O/len_sweep.txt
echo R05B_DONE
