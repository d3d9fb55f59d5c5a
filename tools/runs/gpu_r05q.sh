# Round-5 call Q: 16-B gaps between equal even-size ChaCha20 images (LDS bank stagger): parity,
# then A/B against the no-gap build (tools/ab_libs/nopad.so) over packet lengths, and config B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05q}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_narrow.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in pad nopad; do
  if [ $v = pad ]; then L=""; else L=tools/ab_libs/nopad.so; fi
  MQ_LIB=$L timeout -k 10 400 python3 tools/len_sweep.py c 768 1024 1152 1200 1280 1600 1800 2048 2400 > $O/sweep_$v.txt 2>&1 || { tail $O/sweep_$v.txt; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $O/sweep_$v.txt
done
for i in 1 2; do
  for v in pad nopad; do
    if [ $v = pad ]; then L=""; else L=tools/ab_libs/nopad.so; fi
    MQ_LIB=$L timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_b_$v$i.json 2> $O/bench_b_$v$i.err || { tail $O/bench_b_$v$i.err; exit 1; }
    grep '^{' $O/bench_b_$v$i.json | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('B $v', d['value'], d['ms_per_step'])"
    MQ_LIB=$L timeout -k 10 300 python3 bench.py --config e --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_e_$v$i.json 2> $O/bench_e_$v$i.err || { tail $O/bench_e_$v$i.err; exit 1; }
    grep '^{' $O/bench_e_$v$i.json | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('E $v', d['value'], d['ms_per_step'])"
  done
done
echo R05Q_DONE
