# Round-4 call A: the driver's exact bench command (--steps 20 --warmup 5)
# alternating with the 100-step default on one box, per-step event times in each line; the same
# 20-step command with a 1-s time-based warm-up; rocprofv3 kernel stats of the driver's command.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04a}
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
for r in 1 2 3; do
  step "d20_$r"
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/d20_$r.json 2> $O/d20_$r.err || { tail $O/d20_$r.err; exit 1; }
  step "s100_$r"
  timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/s100_$r.json 2> $O/s100_$r.err || { tail $O/s100_$r.err; exit 1; }
  step "w20_$r"
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --warmup-seconds 1 --no-cpu-baseline > $O/w20_$r.json 2> $O/w20_$r.err || { tail $O/w20_$r.err; exit 1; }
done
python3 - $O <<'EOF'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.load(open(f)); r = d["roofline"]; p = r["per_step_ms"]
    print(os.path.basename(f), d["value"], r["seal_ms"], r["open_ms"], "seal", p["seal"]["min"], p["seal"]["median"], p["seal"]["max"], p["seal"]["first5"], "open", p["open"]["first5"])
EOF
step prof_d20
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_d20 -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_d20.json 2> $O/prof_d20.err || { tail $O/prof_d20.err; exit 1; }
find $O/prof_d20 -name "*kernel_stats.csv" -exec cat {} \;
echo R04A_OK
