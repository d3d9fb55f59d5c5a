# Round-4 call H: A/B of the interleaved-block dynamic schedule (product: blocks of 16, chunks <= 4)
# against the static stride, blocks of 1 / 64 and chunks <= 8, configs C, E, C/1024 keys; the
# driver's bench command (events recorded once during the warm-up, host enqueue times logged).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04h}
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
grep -E "beside the server|timeout outcomes" $O/tests.log
L=milli_quic_amd/libmq_aead.so
for c in c e ck; do
  step ab_$c
  timeout -k 10 600 python tools/ab.py $c 1048576 $L tools/ab_libs/static.so tools/ab_libs/b1.so tools/ab_libs/b64.so tools/ab_libs/cap8.so > $O/ab_$c.txt 2>&1 || { cat $O/ab_$c.txt; exit 1; }
  grep -v "^  " $O/ab_$c.txt
done
for r in 1 2; do
  step d20_$r
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/d20_$r.json 2> $O/d20_$r.err || { tail $O/d20_$r.err; exit 1; }
  step s100_$r
  timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/s100_$r.json 2> $O/s100_$r.err || { tail $O/s100_$r.err; exit 1; }
done
python3 - $O <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/[ds]*.json")):
    d = json.load(open(f)); r = d["roofline"]; p = r["per_step_ms"]
    print(os.path.basename(f), d["value"], r["seal_ms"], r["open_ms"], "seal", p["seal"]["min"], p["seal"]["median"], p["seal"]["max"], p["seal"]["first5"], "enq", r["host_enqueue_ms_first5"])
PY
step aux
timeout -k 10 300 python tools/bench_aux.py > $O/aux.json 2> $O/aux.err || { tail $O/aux.err; exit 1; }
cat $O/aux.json
for a in protect recv; do
  step prof_$a
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$a -o run -- python3 tools/prof_aux.py $a 5 > $O/prof_$a.log 2>&1 || { tail $O/prof_$a.log; exit 1; }
done
echo R04H_OK
