# r03t: config E with the open pre-pass beside the partition (MQ_PREPASS_FORK=1) vs after it,
# alternating; AES phase costs of config C (tools/phase_cost.py c: 16 no AES rounds, 2 no GHASH, 64 no
# final multiply) and per-phase instruction counts; the 2-rank launcher rehearsal on one GPU
# (gloo); smoke.
set -o pipefail
export TMPDIR=/tmp
export MQ_PROF_DIR=tools/ab_libs/prof
O=gpurun_out/r03t
mkdir -p $O
for r in 1 2; do
  for f in 1 0; do
    MQ_PREPASS_FORK=$f timeout -k 10 300 python bench.py --no-cpu-baseline --config e > $O/e_fork${f}_$r.json 2> $O/e_fork${f}_$r.err || { tail $O/e_fork${f}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/e_fork${f}_$r.json')); print('e fork=$f', d['value'], d['roofline']['seal_ms'], d['roofline']['open_ms'], d['parity']['match'])"
  done
done
timeout -k 10 300 python tools/phase_cost.py c > $O/phase_cost_c.txt 2>&1 || { cat $O/phase_cost_c.txt; exit 1; }
cat $O/phase_cost_c.txt
timeout -k 10 600 bash tools/phase_instr.sh c > $O/phase_instr_c.txt 2>&1 || { tail -20 $O/phase_instr_c.txt; exit 1; }
grep -E "aes_(seal|open)1" $O/phase_instr_c.txt
MQ_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --no-cpu-baseline > $O/bench_b_2rank_gloo.json 2> $O/bench_b_2rank_gloo.err || { tail $O/bench_b_2rank_gloo.err; exit 1; }
cat $O/bench_b_2rank_gloo.json
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
echo R03T_OK
