# Round-4 call V: AES seal first-line deferral (product) against the build without it (nodefer.so):
# GPU parity tests, A/B on C, C/1024 keys, E, and PMC HBM traffic of C with each.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04v}
mkdir -p $O
L=milli_quic_amd/libmq_aead.so
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in c ck e; do
  echo "== ab_$c $(date +%T)"
  timeout -k 10 600 python tools/ab.py $c 1048576 $L tools/ab_libs/nodefer.so > $O/ab_$c.txt 2>&1 || { cat $O/ab_$c.txt; exit 1; }
  grep sum $O/ab_$c.txt
done
for v in product nodefer; do
  if [ $v = product ]; then LIB=$L; else LIB=tools/ab_libs/$v.so; fi
  for pc in "p4 FETCH_SIZE" "p5 WRITE_SIZE"; do
    set -- $pc
    MQ_LIB=$LIB timeout -k 10 240 rocprofv3 --pmc $2 --output-format csv -d $O/pmc_$v/$1 -o run -- python3 tools/prof_driver.py c 1048576 2 > $O/pmc_${v}_$1.log 2>&1 || { echo "pmc $v $1 failed"; tail -5 $O/pmc_${v}_$1.log; exit 1; }
  done
  python tools/pmc_summary.py $O/pmc_$v --tiles 131072 > $O/pmc_traffic_$v.txt || exit 1
  echo "== traffic $v"; grep -A3 "aes_seal1" $O/pmc_traffic_$v.txt | grep -E "==|HBM"
done
echo R04V_DONE
