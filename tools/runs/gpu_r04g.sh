# Round-4 call G: the two new resident-server tests alone (co-residency timing, forced timeout),
# then the GPU suite, the schedule A/B and the driver-command bench lines (tools/gpu_r04d.sh).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04g}
mkdir -p $O
echo "== resident tests $(date +%T)"
timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py -x -v -s --timeout 150 --timeout-method thread -k "timeout_then or beside" > $O/resident.log 2>&1 || { tail -40 $O/resident.log; exit 1; }
grep -E "PASS|FAIL|beside the server|timeout outcomes|resident timeout test" $O/resident.log
bash tools/gpu_r04d.sh ${1:-r04g}
for a in protect recv; do
  echo "== prof_$a $(date +%T)"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$a -o run -- python3 tools/prof_aux.py $a 5 > $O/prof_$a.log 2>&1 || { tail $O/prof_$a.log; exit 1; }
  find $O/prof_$a -name "*kernel_stats.csv" -exec cut -c1-150 {} \;
done
