# r03f: 4-wave resident workgroup, one-pass keyed scan; AES header protection of short packets inside the tile (no seal HP pass), the open HP
# pre-pass beside the partition, resident latency phases: GPU tests, benches B / C / E / 1024-key C, kernel trace of E.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03f
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step latency
timeout -k 10 300 python tools/bench_latency.py --calls 2000 > $O/latency.json 2> $O/latency.err || { tail $O/latency.err; exit 1; }
cat $O/latency.json
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # name, bench args
  local name=$1; shift
  step $name
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { tail $O/$name.err; exit 1; }
  cat $O/$name.json
}
run bench_e --config e
run bench_c --config c
run bench_b --config b
run bench_c_k1024 --config c --keys 1024
run bench_e2 --config e
step prof_e
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_e -o run -- python3 bench.py --config e --no-cpu-baseline --steps 20 > $O/prof_e.json 2> $O/prof_e.err || { tail $O/prof_e.err; exit 1; }
echo R03F_OK
