# Round-5 call F: receive A/B on one box (segmented walk vs MQ_RECV_SEG=0, the r04 walk) at
# 4096 / 1024 / 64 / 1 connections, and a kernel trace of the 4096-connection receive.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05f}
mkdir -p $O
for i in 1 2; do
  echo "== seg $(date +%T)"
  timeout -k 10 300 python3 tools/bench_aux.py recv 10 4096 1024 64 1 > $O/recv_seg_$i.json 2> $O/recv_seg_$i.err || { tail $O/recv_seg_$i.err; exit 1; }
  cat $O/recv_seg_$i.json
  echo "== noseg $(date +%T)"
  MQ_RECV_SEG=0 timeout -k 10 300 python3 tools/bench_aux.py recv 10 4096 1024 > $O/recv_noseg_$i.json 2> $O/recv_noseg_$i.err || { tail $O/recv_noseg_$i.err; exit 1; }
  cat $O/recv_noseg_$i.json
done
echo "== trace $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o recv -- python3 tools/bench_aux.py recv 5 4096 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/recv4096_kernel_stats.csv
head -30 $O/recv4096_kernel_stats.csv | cut -d, -f1-8
echo R05F_DONE
