# Round-5 call L: open HP pre-pass forked beside the partition: A/B (MQ_HP_FORK=0), mixed parity
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05l}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_narrow.py tests/test_gpu_streams.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in 1 0; do
    MQ_HP_FORK=$v timeout -k 10 300 python3 bench.py --config e --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_e_$v.json 2> $O/bench_e_$v.err || { tail $O/bench_e_$v.err; exit 1; }
    grep '^{' $O/bench_e_$v.json | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('E hpfork=$v', d['value'], d['ms_per_step'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_e -o run -- python3 tools/prof_driver.py e 1048576 5 > $O/prof_e.log 2>&1 || { tail $O/prof_e.log; exit 1; }
echo R05L_DONE
