# Round-5 call U: config E list order A/B (MQ_LIST_ORDER=1: ChaCha20 list before the multi-key AES
# kernel on the caller's stream), alternating, plus a timeline of the alternative order
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05u}
mkdir -p $O
MQ_LIST_ORDER=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "mixed" --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  for v in 0 1; do
    MQ_LIST_ORDER=$v timeout -k 10 300 python3 bench.py --config e --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_e_$v$i.json 2> $O/bench_e_$v$i.err || { tail $O/bench_e_$v$i.err; exit 1; }
    grep '^{' $O/bench_e_$v$i.json | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); r=d['roofline']; print('E order=$v', d['value'], d['ms_per_step'], r['seal_ms'], r['open_ms'])"
  done
done
MQ_LIST_ORDER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_e -o run -- python3 tools/prof_driver.py e 1048576 3 > $O/prof_e.log 2>&1 || { tail $O/prof_e.log; exit 1; }
echo R05U_DONE
