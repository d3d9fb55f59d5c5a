set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/bench_r01.json 2> gpurun_out/bench_r01.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r01 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_r01.log 2>&1
echo rc=$?
cat gpurun_out/smoke.log; cat gpurun_out/bench_r01.json; tail -5 gpurun_out/bench_r01.err
