# Round-5 call P: 16-KiB image kernels in 2-wave workgroups (10 waves per CU) for flat ChaCha20
# batches of 1585-1952-B packets: parity, length sweep, config B unchanged
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05p}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_narrow.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python3 tools/len_sweep.py chacha 1584 1600 1700 1800 1900 1952 2000 2048 2400 > $O/len_sweep.txt 2>&1 || { tail $O/len_sweep.txt; exit 1; }
grep -v amdgpu.ids $O/len_sweep.txt
MQ_CC_LONG=2 timeout -k 10 400 python3 tools/len_sweep.py chacha 1600 1800 1952 > $O/len_sweep_20k.txt 2>&1 || { tail $O/len_sweep_20k.txt; exit 1; }
grep -v amdgpu.ids $O/len_sweep_20k.txt
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_b.json 2> $O/bench_b.err || { tail $O/bench_b.err; exit 1; }
grep '^{' $O/bench_b.json | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('B', d['value'], d['ms_per_step'])"
echo R05P_DONE
