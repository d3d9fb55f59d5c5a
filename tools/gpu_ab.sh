# GPU tests, then A/B of library builds (tools/ab.py) for the given configs, then bench lines.
# Usage: bash tools/gpu_ab.sh TAG "CFG..." LIB_A LIB_B
set -o pipefail
export TMPDIR=/tmp
TAG=$1; CFGS=$2; shift 2
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for c in $CFGS; do
  timeout -k 10 600 python tools/ab.py $c 1048576 "$@" > $O/ab_$c.txt 2>&1 || { cat $O/ab_$c.txt; exit 1; }
  cat $O/ab_$c.txt
done
echo AB_OK
