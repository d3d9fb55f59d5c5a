# Round-4 call J: receive / send GPU tests, aux components with the product library and with the
# 4-chunk build batch (MQ_LIB), kernel stats of the receive / protect composites.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04j}
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 600 python -u -m pytest tests/test_gpu_recv.py tests/test_gpu_send.py tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  step aux_$r
  timeout -k 10 300 python tools/bench_aux.py > $O/aux_$r.json 2> $O/aux_$r.err || { tail $O/aux_$r.err; exit 1; }
  cat $O/aux_$r.json
  MQ_LIB=tools/ab_libs/bb4.so timeout -k 10 300 python tools/bench_aux.py > $O/aux_bb4_$r.json 2> $O/aux_bb4_$r.err || { tail $O/aux_bb4_$r.err; exit 1; }
  cat $O/aux_bb4_$r.json
done
step e2e
timeout -k 10 600 python3 bench.py --no-cpu-baseline --e2e > $O/bench_b_e2e.json 2> $O/bench_b_e2e.err || { tail $O/bench_b_e2e.err; exit 1; }
python3 -c "import json,sys; print(json.load(open(sys.argv[1]))[\"end_to_end\"])" $O/bench_b_e2e.json
for a in protect recv; do
  step prof_$a
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$a -o run -- python3 tools/prof_aux.py $a 5 > $O/prof_$a.log 2>&1 || { tail $O/prof_$a.log; exit 1; }
done
echo R04J_OK
