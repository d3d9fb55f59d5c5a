# Round-4 call ZK: flat ChaCha20 workgroups with a tile over the LDS budget run two rounds (such a
# tile staged in halves) — product — vs the previous tree (prev.so): all GPU tests, length sweep,
# A/B on config B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04zk}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 tools/len_sweep.py c > $O/sweep_product.txt 2>&1 || { tail $O/sweep_product.txt; exit 1; }
grep chacha $O/sweep_product.txt
timeout -k 10 600 python3 tools/ab.py b 1048576 milli_quic_amd/libmq_aead.so tools/ab_libs/prev.so > $O/ab_b.txt 2>&1 || { tail $O/ab_b.txt; exit 1; }
cat $O/ab_b.txt
echo R04ZK_DONE
