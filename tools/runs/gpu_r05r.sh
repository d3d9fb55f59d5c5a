# Round-5 call R: image gaps in the narrow ChaCha20 tiles too: parity, A/B against the no-gap build
# over short packet lengths, config E
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05r}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_narrow.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in pad nopad; do
  if [ $v = pad ]; then L=""; else L=tools/ab_libs/nopad.so; fi
  MQ_LIB=$L timeout -k 10 400 python3 tools/len_sweep.py c 64 96 128 192 256 320 384 448 512 640 > $O/sweep_$v.txt 2>&1 || { tail $O/sweep_$v.txt; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $O/sweep_$v.txt
done
for i in 1 2; do
  for v in pad nopad; do
    if [ $v = pad ]; then L=""; else L=tools/ab_libs/nopad.so; fi
    MQ_LIB=$L timeout -k 10 300 python3 bench.py --config e --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_e_$v$i.json 2> $O/bench_e_$v$i.err || { tail $O/bench_e_$v$i.err; exit 1; }
    grep '^{' $O/bench_e_$v$i.json | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('E $v', d['value'], d['ms_per_step'])"
  done
done
echo R05R_DONE
