# Round-5 call K: partition without the single-workgroup scan kernel (class totals by atomics,
# the last count block lays the lists out, row totals counted directly): parity of the mixed and
# keyed paths, then E bench, parts and kernel timeline
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05k}
mkdir -p $O
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_narrow.py tests/test_gpu_config_d.py tests/test_gpu_recv.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 bench.py --config e --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_e.json 2> $O/bench_e.err || { tail $O/bench_e.err; exit 1; }
grep '^{' $O/bench_e.json | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('E', d['value'], d['ms_per_step'])"
timeout -k 10 300 python3 bench.py --config c --keys 1024 --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_ck.json 2> $O/bench_ck.err || { tail $O/bench_ck.err; exit 1; }
grep '^{' $O/bench_ck.json | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('C/1024', d['value'], d['ms_per_step'])"
timeout -k 10 200 python3 tools/e_parts.py > $O/e_parts.txt 2>&1 || { tail $O/e_parts.txt; exit 1; }
cat $O/e_parts.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_e -o run -- python3 tools/prof_driver.py e 1048576 5 > $O/prof_e.log 2>&1 || { tail $O/prof_e.log; exit 1; }
grep -E "part|hp" $O/prof_e/run_kernel_stats.csv | cut -d, -f1-4
echo R05K_DONE
