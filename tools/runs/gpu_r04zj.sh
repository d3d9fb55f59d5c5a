# Round-4 call ZJ: rounds with the size check overlapped with the tile's descriptor loads
# (product) vs prev.so: ChaCha parity tests, sweep at 1200 / 1452, A/B on config B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04zj}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 tools/len_sweep.py c 1200 1452 > $O/sweep_product.txt 2>&1 || { tail $O/sweep_product.txt; exit 1; }
grep chacha $O/sweep_product.txt
timeout -k 10 400 python3 tools/ab.py b 1048576 milli_quic_amd/libmq_aead.so tools/ab_libs/prev.so > $O/ab_b.txt 2>&1 || { tail $O/ab_b.txt; exit 1; }
cat $O/ab_b.txt
echo R04ZJ_DONE
