# Per-phase instruction counts: PMC (SQ_INSTS_*) of the product library and every MQ_PROF_SKIP
# variant on one workload; differences = what each phase issues per wave.
set -o pipefail
export TMPDIR=/tmp
CFG=${1:-b}
N=${2:-1048576}
O=gpurun_out/phase_instr_$CFG
mkdir -p $O
for lib in milli_quic_amd/libmq_aead.so ${MQ_PROF_DIR:-milli_quic_amd/prof}/prof_*.so; do
  name=$(basename $lib .so)
  timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $O/$name -o run -- python3 tools/phase_cost.py --child $lib $CFG $N > $O/$name.log 2>&1 || { echo "fail $name"; exit 1; }
done
python3 - "$O" <<'PY'
import sys, os, glob
sys.path.insert(0, "tools")
from pmc_summary import load
base = None
for d in sorted(glob.glob(os.path.join(sys.argv[1], "*/"))):
    r = load(d)
    name = os.path.basename(d.rstrip("/"))
    for k, c in sorted(r.items()):
        if ("seal" not in k and "open" not in k) or "hp_kernel" in k:
            continue
        w = c.get("SQ_WAVES", 1)
        if "aes" in k:  # persistent kernels: per tile (2^20 / 8 tiles), not per wave
            w = int(os.environ.get("N", "1048576")) / 8
        row = {x: c.get(x, 0) / w for x in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR")}
        print(f"{name:20s} {k:28s} " + " ".join(f"{x[9:]}={v:8.1f}" for x, v in row.items()))
PY
