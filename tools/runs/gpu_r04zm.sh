# Round-4 call ZM (diagnostic): where the long-packet rounds lose config B — product (no rounds)
# vs chk.so (the workgroup size check only) vs halves2.so (check + two inline rounds).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04zm}
mkdir -p $O
timeout -k 10 600 python3 tools/ab.py b 1048576 milli_quic_amd/libmq_aead.so tools/ab_libs/chk.so tools/ab_libs/halves2.so > $O/ab_b.txt 2>&1 || { tail $O/ab_b.txt; exit 1; }
cat $O/ab_b.txt
echo R04ZM_DONE
