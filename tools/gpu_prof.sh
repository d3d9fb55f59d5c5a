# kernel-trace stats of the bench + PMC passes (config $2, default b). Summaries -> gpurun_out/
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r01}
CFG=${2:-b}
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --config $CFG --no-cpu-baseline > gpurun_out/prof_$TAG/bench.json 2> gpurun_out/prof_$TAG/bench.err || { tail gpurun_out/prof_$TAG/bench.err; exit 1; }
cat gpurun_out/prof_$TAG/bench.json
f=$(find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1); cat "$f" | cut -c1-220
bash tools/gpu_pmc.sh $CFG 1048576 && python3 tools/pmc_summary.py gpurun_out/pmc_$CFG --json gpurun_out/pmc_${CFG}_traffic.json
