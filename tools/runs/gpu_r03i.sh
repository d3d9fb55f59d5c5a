# r03i: baseline of the restored tree: GPU tests, benches B / C / E.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03i
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # name, bench args
  local name=$1; shift
  step $name
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { tail $O/$name.err; exit 1; }
  cat $O/$name.json
}
run bench_b --config b
run bench_c --config c
run bench_e --config e
echo R03I_OK
