# r05zb: split open (HP pre-pass on the hot kernel's side stream, in-tile HP for the multi-key AES
# kernel) — all GPU tests, then E A/B against MQ_OPEN_HP_SPLIT=0 (alternating, 3 pairs), C/1024.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05zb}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --config e > $O/e_split_$i.json || exit 1
  MQ_OPEN_HP_SPLIT=0 timeout -k 10 120 python bench.py --no-cpu-baseline --config e > $O/e_join_$i.json || exit 1
  python -c "import json; a=json.load(open('$O/e_split_$i.json')); b=json.load(open('$O/e_join_$i.json')); print('split', a['value'], a['roofline']['open_ms'], 'join', b['value'], b['roofline']['open_ms'])"
done
timeout -k 10 120 python bench.py --no-cpu-baseline --config c --keys 1024 > $O/ck.json || exit 1
python -c "import json; a=json.load(open('$O/ck.json')); print('ck', a['value'], a['roofline']['open_ms'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_e -o run -- python3 bench.py --no-cpu-baseline --config e --steps 20 > $O/prof_e.json 2> $O/prof_e.err || { tail $O/prof_e.err; exit 1; }
echo ALL_OK
