# r03o (the keyed kernels measured here were rejected and removed; MQ_AES_KEYED no longer exists): 16-wave keyed AES kernels (key-uniform tiles of the partition's keyed layout) vs the 12-wave
# multi-key kernels (MQ_AES_KEYED=0): GPU tests, then configs E and C with 1024 keys, alternating.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03o
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # name, env, bench args
  local name=$1 envs=$2; shift 2
  step $name
  env $envs timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { tail $O/$name.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/$name.json')); print('$name', d['value'], d['roofline']['seal_ms'], d['roofline']['open_ms'])"
}
for r in 1 2; do
  run e_keyed_$r "MQ_AES_KEYED=1" --config e
  run e_multi_$r "MQ_AES_KEYED=0" --config e
  run ck_keyed_$r "MQ_AES_KEYED=1" --config c --keys 1024
  run ck_multi_$r "MQ_AES_KEYED=0" --config c --keys 1024
done
echo R03O_OK
