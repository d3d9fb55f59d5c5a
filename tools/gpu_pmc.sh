# PMC passes (one counter group per rocprofv3 run, kernel-trace only; no sys/runtime trace)
set -o pipefail
export TMPDIR=/tmp
CFG=${1:-b}
N=${2:-1048576}
OUT=gpurun_out/pmc_${CFG}
mkdir -p $OUT
run() { name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- python3 tools/prof_driver.py $CFG $N 2 > $OUT/$name.log 2>&1 || { echo "pass $name failed"; return 1; }
}
run p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR && \
run p2 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU && \
run p3 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE && \
run p4 FETCH_SIZE && \
run p5 WRITE_SIZE
echo "pmc rc=$?"
