# r03p: tile-footprint probe (tools/scatter_probe.py), GPU tests, bench E with the one-pass keyed
# scan, rocprofv3 kernel stats of config E.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03p
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step scatter
timeout -k 10 400 python tools/scatter_probe.py > $O/scatter.json 2> $O/scatter.err || { tail $O/scatter.err; exit 1; }
cat $O/scatter.json
step tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  step bench_e_$r
  timeout -k 10 300 python bench.py --no-cpu-baseline --config e > $O/bench_e_$r.json 2> $O/bench_e_$r.err || { tail $O/bench_e_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_e_$r.json')); print(d['value'], d['roofline']['seal_ms'], d['roofline']['open_ms'])"
done
step prof_e
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_e -o run -- python3 bench.py --config e --no-cpu-baseline --steps 20 > $O/prof_e.json 2> $O/prof_e.err || { tail $O/prof_e.err; exit 1; }
echo R03P_OK
