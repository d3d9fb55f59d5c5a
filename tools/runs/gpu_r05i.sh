# Round-5 call I: config-E state of the tree: bench E, cost split by part, kernel trace of E
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05i}
mkdir -p $O
timeout -k 10 300 python3 bench.py --config e --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_e.json 2> $O/bench_e.err || { tail $O/bench_e.err; exit 1; }
grep '^{' $O/bench_e.json | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('E', d['value'], d['ms_per_step'])"
timeout -k 10 300 python3 tools/e_parts.py > $O/e_parts.txt 2>&1 || { tail $O/e_parts.txt; exit 1; }
cat $O/e_parts.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_e -o run -- python3 tools/prof_driver.py e 1048576 5 > $O/prof_e.log 2>&1 || { tail $O/prof_e.log; exit 1; }
cut -d, -f1-4 $O/prof_e/run_kernel_stats.csv | head -30
echo R05I_DONE
