# r05zc: open header-protection masks fused into the partition's count kernel — all GPU tests, then
# E and C/1024 A/B against MQ_HP_FUSED=0 (alternating, 3 pairs), kernel trace of E.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05zc}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2 3; do
  for c in "e --config e" "ck --config c --keys 1024"; do
    set -- $c; name=$1; shift
    timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/${name}_fused_$i.json || exit 1
    MQ_HP_FUSED=0 timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/${name}_sep_$i.json || exit 1
    python -c "import json; a=json.load(open('$O/${name}_fused_$i.json')); b=json.load(open('$O/${name}_sep_$i.json')); print('$name fused', a['value'], a['roofline']['open_ms'], 'separate', b['value'], b['roofline']['open_ms'])"
  done
done
timeout -k 10 300 python tools/bench_latency.py > $O/latency.json 2> $O/latency.err || { tail $O/latency.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_e -o run -- python3 bench.py --no-cpu-baseline --config e --steps 20 > $O/prof_e.json 2> $O/prof_e.err || { tail $O/prof_e.err; exit 1; }
echo ALL_OK
