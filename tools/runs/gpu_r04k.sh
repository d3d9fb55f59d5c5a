# Round-4 call K: the wave-per-connection receive walk — receive GPU tests, aux (protect / recv)
# twice, kernel trace of the receive composite.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04k}
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 600 python -u -m pytest tests/test_gpu_recv.py tests/test_gpu_send.py -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  step aux_$r
  timeout -k 10 300 python tools/bench_aux.py > $O/aux_$r.json 2> $O/aux_$r.err || { tail $O/aux_$r.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('protect', d['protect'], 'recv', d['recv'])" $O/aux_$r.json
done
step prof_recv
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_recv -o run -- python3 tools/prof_aux.py recv 5 > $O/prof_recv.log 2>&1 || { tail $O/prof_recv.log; exit 1; }
grep -E "walk|open_list|aes_open1" $O/prof_recv/run_kernel_stats.csv
echo R04K_DONE
