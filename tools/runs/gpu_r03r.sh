# r03r: key-segmented single-key AES kernels for keyed partitions with >= 512 packets per row
# (config C with 1024 keys) vs the hot split + multi-key kernel (MQ_AES_SEG=0): GPU tests, then
# C with 1024 keys and E (unchanged path) alternating, kernel stats of 1024-key C.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03r
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # name, env, bench args
  local name=$1 envs=$2; shift 2
  step $name
  env $envs timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { tail $O/$name.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/$name.json')); print('$name', d['value'], d['roofline']['seal_ms'], d['roofline']['open_ms'], d['parity']['match'])"
}
for r in 1 2; do
  run ck_seg_$r "MQ_AES_SEG=1" --config c --keys 1024
  run ck_multi_$r "MQ_AES_SEG=0" --config c --keys 1024
done
run e_1 "MQ_AES_SEG=1" --config e
run c_1 "MQ_AES_SEG=1" --config c
step prof_ck
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ck -o run -- python3 bench.py --config c --keys 1024 --no-cpu-baseline --steps 20 > $O/prof_ck.json 2> $O/prof_ck.err || { tail $O/prof_ck.err; exit 1; }
echo R03R_OK
