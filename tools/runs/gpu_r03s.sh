# r03s: empty-list AES workgroups leave before their tables, keyed bins merged per thread in the
# partition's count/scatter: GPU tests, benches C (1024 keys), E, C, B; kernel stats of 1024-key
# C; then ChaCha phase costs (tools/gpu_r03q.sh).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03s
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # name, bench args
  local name=$1; shift
  step $name
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { tail $O/$name.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/$name.json')); print('$name', d['value'], d['roofline']['seal_ms'], d['roofline']['open_ms'], d['parity']['match'])"
}
run ck --config c --keys 1024
run ck2 --config c --keys 1024
run e --config e
run c --config c
run b --config b
step prof_ck
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ck -o run -- python3 bench.py --config c --keys 1024 --no-cpu-baseline --steps 20 > $O/prof_ck.json 2> $O/prof_ck.err || { tail $O/prof_ck.err; exit 1; }
step phases
bash tools/gpu_r03q.sh || exit 1
echo R03S_OK
