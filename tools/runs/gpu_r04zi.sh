# Round-4 call ZI: flat ChaCha20 tiles over the LDS budget staged in rounds (product) vs the direct
# path (prev.so): all GPU tests, length sweep, A/B on config B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04zi}
mkdir -p $O
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 tools/len_sweep.py c > $O/sweep_product.txt 2>&1 || { tail $O/sweep_product.txt; exit 1; }
grep chacha $O/sweep_product.txt
timeout -k 10 400 python3 tools/ab.py b 1048576 milli_quic_amd/libmq_aead.so tools/ab_libs/prev.so > $O/ab_b.txt 2>&1 || { tail $O/ab_b.txt; exit 1; }
tail -2 $O/ab_b.txt
echo R04ZI_DONE
