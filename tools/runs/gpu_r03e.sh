# r03e: keyed 16-wave multi-key AES kernels (partition lists in the keyed layout): GPU tests,
# resident latency with device-side phases, then config E and 1024-key config C with the keyed kernels on / off and the hot split on / off.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03e
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step latency
timeout -k 10 300 python tools/bench_latency.py --calls 2000 > $O/latency.json 2> $O/latency.err || { tail $O/latency.err; exit 1; }
cat $O/latency.json
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # name, env..., -- bench args
  local name=$1; shift
  step $name
  env "$@" > $O/$name.json 2> $O/$name.err || { tail $O/$name.err; exit 1; }
  cat $O/$name.json
}
run e_keyed_hot   MQ_AES_KEYED=1 MQ_AES_HOT=1 timeout -k 10 300 python bench.py --config e --no-cpu-baseline
run e_keyed_nohot MQ_AES_KEYED=1 MQ_AES_HOT=0 timeout -k 10 300 python bench.py --config e --no-cpu-baseline
run e_mixed       MQ_AES_KEYED=0 timeout -k 10 300 python bench.py --config e --no-cpu-baseline
run c1024_keyed   MQ_AES_KEYED=1 timeout -k 10 300 python bench.py --config c --keys 1024 --no-cpu-baseline
run c1024_mixed   MQ_AES_KEYED=0 timeout -k 10 300 python bench.py --config c --keys 1024 --no-cpu-baseline
step prof_e
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_e -o run -- python3 bench.py --config e --no-cpu-baseline --steps 20 > $O/prof_e.json 2> $O/prof_e.err || { tail $O/prof_e.err; exit 1; }
echo R03E_OK
