# Round-4 call T: multi-key AES kernels at 8 waves / 195 VGPRs (m8.so: no spills) against the
# product (12 waves / 168, 15 spilled VGPRs) on config E; PMC HBM traffic of E with each.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04t}
mkdir -p $O
L=milli_quic_amd/libmq_aead.so
echo "== recv tests $(date +%T)"
timeout -k 10 300 python -u -m pytest tests/test_gpu_recv.py -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
echo "== ab_e $(date +%T)"
timeout -k 10 600 python tools/ab.py e 1048576 $L tools/ab_libs/m8.so > $O/ab_e.txt 2>&1 || { cat $O/ab_e.txt; exit 1; }
grep sum $O/ab_e.txt
for v in product m8; do
  if [ $v = product ]; then LIB=$L; else LIB=tools/ab_libs/$v.so; fi
  for pc in "p4 FETCH_SIZE" "p5 WRITE_SIZE"; do
    set -- $pc
    MQ_LIB=$LIB timeout -k 10 240 rocprofv3 --pmc $2 --output-format csv -d $O/pmc_$v/$1 -o run -- python3 tools/prof_driver.py e 1048576 2 > $O/pmc_${v}_$1.log 2>&1 || { echo "pmc $v $1 failed"; tail -5 $O/pmc_${v}_$1.log; exit 1; }
  done
  python tools/pmc_summary.py $O/pmc_$v > $O/pmc_traffic_$v.txt || exit 1
  echo "== traffic $v"; grep -A3 "aes_seal_kernel\|aes_open_kernel" $O/pmc_traffic_$v.txt | grep -E "==|HBM"
done
echo R04T_DONE
