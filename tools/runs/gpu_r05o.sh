# Round-5 call O: AES seal header mask from registers (no read-modify-write): parity, then A/B
# against the previous AES object (tools/ab_libs/prev.so) on C, C/1024 keys and E, alternating
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05o}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_send.py tests/test_gpu_records.py tests/test_gpu_config_d.py tests/test_gpu_narrow.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in new prev; do
    if [ $v = new ]; then L=""; else L=tools/ab_libs/prev.so; fi
    for a in "c --config c" "ck --config c --keys 1024" "e --config e"; do
      set -- $a; c=$1; shift
      MQ_LIB=$L timeout -k 10 300 python3 bench.py "$@" --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_${c}_$v$i.json 2> $O/bench_${c}_$v$i.err || { tail $O/bench_${c}_$v$i.err; exit 1; }
      grep '^{' $O/bench_${c}_$v$i.json | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); r=d['roofline']; print('$c $v', d['value'], d['ms_per_step'], r.get('seal_ms'), r.get('open_ms'))"
    done
  done
done
echo R05O_DONE
