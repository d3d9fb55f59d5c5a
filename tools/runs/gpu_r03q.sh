# r03q: ChaCha phase costs of config B under full load (tools/phase_cost.py with the MQ_PROF_SKIP
# variants in tools/ab_libs/prof: 1 no rounds, 2 no MAC, 4 no store, 8 no staging) and their
# per-phase instruction counts (tools/phase_instr.sh: SQ_INSTS_* PMC per variant).
set -o pipefail
export TMPDIR=/tmp
export MQ_PROF_DIR=tools/ab_libs/prof
O=gpurun_out/r03q
mkdir -p $O
timeout -k 10 300 python tools/phase_cost.py b > $O/phase_cost_b.txt 2>&1 || { cat $O/phase_cost_b.txt; exit 1; }
cat $O/phase_cost_b.txt
timeout -k 10 600 bash tools/phase_instr.sh b > $O/phase_instr_b.txt 2>&1 || { tail -20 $O/phase_instr_b.txt; exit 1; }
cat $O/phase_instr_b.txt
echo R03Q_OK
