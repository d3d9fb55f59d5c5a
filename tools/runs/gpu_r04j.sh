# Round-4 call J: receive / send GPU tests, aux components with the fused ChaCha protect and with
# two-kernel composite (MQ_PROTECT_FUSED=0; and ChaCha lists on the one-shot grid, MQ_CC_LIST=0), kernel stats of the receive / protect composites.
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
  MQ_PROTECT_FUSED=0 MQ_CC_LIST=0 timeout -k 10 300 python tools/bench_aux.py > $O/aux_unfused_$r.json 2> $O/aux_unfused_$r.err || { tail $O/aux_unfused_$r.err; exit 1; }
  cat $O/aux_unfused_$r.json
done
step e2e
timeout -k 10 600 python3 bench.py --no-cpu-baseline --e2e > $O/bench_b_e2e.json 2> $O/bench_b_e2e.err || { tail $O/bench_b_e2e.err; exit 1; }
python3 -c "import json,sys; print(json.load(open(sys.argv[1]))[\"end_to_end\"])" $O/bench_b_e2e.json
for a in protect recv; do
  step prof_$a
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$a -o run -- python3 tools/prof_aux.py $a 5 > $O/prof_$a.log 2>&1 || { tail $O/prof_$a.log; exit 1; }
done

for a in "c --config c" "e --config e" "ck --config c --keys 1024"; do
  set -- $a; name=$1; shift
  step bench_$name
  timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > $O/bench_$name.json 2> $O/bench_$name.err || { tail $O/bench_$name.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], r['seal_ms'], r['open_ms'], r['frac'])" $O/bench_$name.json
done
step bench_e_oneshot
MQ_CC_LIST=0 timeout -k 10 300 python3 bench.py --no-cpu-baseline --config e > $O/bench_e_oneshot.json 2> $O/bench_e_oneshot.err || { tail $O/bench_e_oneshot.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], r['seal_ms'], r['open_ms'], r['frac'])" $O/bench_e_oneshot.json
step prof_e
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_e -o run -- python3 bench.py --no-cpu-baseline --config e > $O/prof_e.json 2> $O/prof_e.err || { tail $O/prof_e.err; exit 1; }
echo R04J_DONE
step prof_d20
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_d20 -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_d20.json 2> $O/prof_d20.err || { tail $O/prof_d20.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('prof_d20', d['value'], r['seal_ms'], r['open_ms'])" $O/prof_d20.json
grep -E "chacha_(seal|open)1" $O/prof_d20/run_kernel_stats.csv
echo R04J_ALL_DONE
