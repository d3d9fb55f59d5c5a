# r03v: config-E upper bound of the Initial packets' multi-key cost (tools/e_probe.py) and the
# multi-key chunk A/B on the current tree.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03v
mkdir -p $O
timeout -k 10 300 python -u tools/e_probe.py > $O/e_probe.txt 2>&1 || { tail $O/e_probe.txt; exit 1; }
cat $O/e_probe.txt
timeout -k 10 500 python -u tools/ab.py e 1048576 tools/ab_libs/base.so tools/ab_libs/chunk2.so tools/ab_libs/chunk8.so > $O/ab_chunk.txt 2>&1 || { tail $O/ab_chunk.txt; exit 1; }
cat $O/ab_chunk.txt
echo R03V_OK
