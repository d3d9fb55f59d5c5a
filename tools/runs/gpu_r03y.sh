# r03y: rocprof kernel stats of config E for the HEAD library and the mixed-HP-compaction build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03y
mkdir -p $O
for lib in base hpc; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$lib -o run -- python3 tools/phase_cost.py --child tools/ab_libs/$lib.so e 1048576 > $O/prof_$lib.log 2>&1 || { tail $O/prof_$lib.log; exit 1; }
  grep -E "part_|mixed_hp|Name" $O/prof_$lib/run_kernel_stats.csv | cut -d, -f1-4
done
echo R03Y_OK
