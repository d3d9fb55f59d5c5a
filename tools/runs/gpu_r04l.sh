# Round-4 call L: full GPU tests; receive (wave walk, gated empty passes, fused unmask), config E
# with the single-key ChaCha list kernels; kernel traces.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04l}
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
step aux
timeout -k 10 300 python tools/bench_aux.py > $O/aux.json 2> $O/aux.err || { tail $O/aux.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('protect', d['protect'], 'recv', d['recv'])" $O/aux.json
for a in "e1 --config e" "e2 --config e" "b --config b"; do
  set -- $a; name=$1; shift
  step bench_$name
  timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > $O/bench_$name.json 2> $O/bench_$name.err || { tail $O/bench_$name.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], r['seal_ms'], r['open_ms'], r['frac'])" $O/bench_$name.json
done
step prof_recv
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_recv -o run -- python3 tools/prof_aux.py recv 5 > $O/prof_recv.log 2>&1 || { tail $O/prof_recv.log; exit 1; }
step prof_e
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_e -o run -- python3 bench.py --no-cpu-baseline --config e --steps 20 > $O/prof_e.json 2> $O/prof_e.err || { tail $O/prof_e.err; exit 1; }
grep -E "chacha|aes_seal|aes_open|part_" $O/prof_e/run_kernel_stats.csv
echo R04L_DONE
