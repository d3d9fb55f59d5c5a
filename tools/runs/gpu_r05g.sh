# Round-5 call G: arithmetic segment table + merged verify/fallback: debug runs, receive tests,
# receive A/B against MQ_RECV_SEG=0 (the r04 walk) on one box, kernel trace of the 4096-conn receive.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05g}
mkdir -p $O
MQ_RECV_TRACE=1 timeout -k 10 120 python3 tests/debug_recv_long.py 1 16384 0 > $O/dbg1.txt 2>&1 || { tail -20 $O/dbg1.txt; exit 1; }
grep -E "^n |recv" $O/dbg1.txt | head -8
MQ_RECV_TRACE=1 timeout -k 10 120 python3 tests/debug_recv_long.py 4 16384 1 > $O/dbg4.txt 2>&1 || { tail -20 $O/dbg4.txt; exit 1; }
grep -E "^n |recv" $O/dbg4.txt | head -8
echo "== recv tests $(date +%T)"
timeout -k 10 800 python -u -m pytest tests/test_gpu_recv.py -x -v --timeout 300 --timeout-method thread > $O/tests_recv.log 2>&1 || { tail -40 $O/tests_recv.log; exit 1; }
tail -1 $O/tests_recv.log
for i in 1 2; do
  timeout -k 10 300 python3 tools/bench_aux.py recv 10 4096 1024 64 4 1 > $O/recv_seg_$i.json 2> $O/recv_seg_$i.err || { tail $O/recv_seg_$i.err; exit 1; }
  cat $O/recv_seg_$i.json
  MQ_RECV_SEG=0 timeout -k 10 300 python3 tools/bench_aux.py recv 10 4096 1024 > $O/recv_noseg_$i.json 2> $O/recv_noseg_$i.err || { tail $O/recv_noseg_$i.err; exit 1; }
  cat $O/recv_noseg_$i.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o recv -- python3 tools/bench_aux.py recv 5 4096 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
grep -E "recv|Name" $O/prof/recv_kernel_stats.csv | cut -d, -f1-4
echo R05G_DONE
