# Round-5 call T: single-key AES GHASH through the conflict-free nibble half table of H^8
# (tools/ab_libs/nibble.so, MQ_AES_NIBBLE build) vs the byte-position table (product): C, C/1024, E
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05t}
mkdir -p $O
MQ_LIB=tools/ab_libs/nibble.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "aes or full_size or mixed" --timeout 200 --timeout-method thread > $O/tests_nibble.log 2>&1 || { tail -30 $O/tests_nibble.log; exit 1; }
tail -1 $O/tests_nibble.log
for i in 1 2; do
  for v in byte nibble; do
    if [ $v = byte ]; then L=""; else L=tools/ab_libs/nibble.so; fi
    for a in "c --config c" "ck --config c --keys 1024" "e --config e"; do
      set -- $a; c=$1; shift
      MQ_LIB=$L timeout -k 10 300 python3 bench.py "$@" --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_${c}_$v$i.json 2> $O/bench_${c}_$v$i.err || { tail $O/bench_${c}_$v$i.err; exit 1; }
      grep '^{' $O/bench_${c}_$v$i.json | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); r=d['roofline']; print('$c $v', d['value'], d['ms_per_step'], r.get('seal_ms'), r.get('open_ms'))"
    done
  done
done
echo R05T_DONE
