# Round-4 call D: GPU tests (incl. the resident timeout / co-residency tests); A/B of the dynamic
# tile schedule (product: deferred claims, chunk cap 16) against the static stride and chunk caps
# 4 / 32 on configs C, E, C/1024 keys; the driver's bench command with the r04 warm-up.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04d}
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
grep -E "timeout outcomes|beside the server" $O/tests.log
L=milli_quic_amd/libmq_aead.so
for c in c e ck; do
  step ab_$c
  timeout -k 10 600 python tools/ab.py $c 1048576 $L tools/ab_libs/static.so tools/ab_libs/cap4.so tools/ab_libs/cap32.so > $O/ab_$c.txt 2>&1 || { cat $O/ab_$c.txt; exit 1; }
  cat $O/ab_$c.txt
done
for r in 1 2; do
  step d20_$r
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/d20_$r.json 2> $O/d20_$r.err || { tail $O/d20_$r.err; exit 1; }
  step s100_$r
  timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/s100_$r.json 2> $O/s100_$r.err || { tail $O/s100_$r.err; exit 1; }
done
python3 - $O <<'EOF'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/[ds]*.json")):
    d = json.load(open(f)); r = d["roofline"]; p = r["per_step_ms"]
    print(os.path.basename(f), d["value"], d["warmup_extra"], r["seal_ms"], r["open_ms"], "seal", p["seal"]["min"], p["seal"]["median"], p["seal"]["max"], p["seal"]["first5"])
EOF
echo R04D_OK
step probe_null
timeout -k 5 60 python3 -u tools/resident_timeout_probe.py 1048576 --null > $O/probe_null.txt 2>&1; echo rc=$?; cat $O/probe_null.txt
