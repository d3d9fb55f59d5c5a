# Round-4 call C: per-step clock probe; GPU parity suite on the dynamic tile
# schedule; A/B of the static (MQ_SCHED=0) vs dynamic schedule on configs C, C/1024 keys, E, B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04c}
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step clock_probe
timeout -k 10 200 python3 tools/clock_probe.py 30 > $O/clock_probe.txt 2>&1 || { tail $O/clock_probe.txt; exit 1; }
grep -v "^{" $O/clock_probe.txt
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for cfg in "c --config c" "ck --config c --keys 1024" "e --config e"; do
    set -- $cfg; name=$1; shift
    for sch in 0 1; do
      step "${name}_s${sch}_$r"
      MQ_SCHED=$sch timeout -k 10 200 python3 bench.py --no-cpu-baseline "$@" > $O/${name}_s${sch}_$r.json 2> $O/${name}_s${sch}_$r.err || { tail $O/${name}_s${sch}_$r.err; exit 1; }
    done
  done
done
python3 - $O <<'EOF'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/*_s*_*.json")):
    d = json.load(open(f)); r = d["roofline"]
    print(os.path.basename(f), d["value"], r["seal_ms"], r["open_ms"], r["per_step_ms"]["seal"]["median"], r["per_step_ms"]["open"]["median"])
EOF
echo R04C_OK
