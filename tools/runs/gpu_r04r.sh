# Round-4 call R: AES single-key kernels at 12 waves / 168 VGPRs (w12.so) and non-temporal packet
# streams (nt.so) against the product: A/B times on C, C/1024 keys, E, and PMC HBM traffic of C.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04r}
mkdir -p $O
L=milli_quic_amd/libmq_aead.so
for c in c e; do
  echo "== ab_$c $(date +%T)"
  timeout -k 10 600 python tools/ab.py $c 1048576 $L tools/ab_libs/w12.so tools/ab_libs/nt.so > $O/ab_$c.txt 2>&1 || { cat $O/ab_$c.txt; exit 1; }
  grep sum $O/ab_$c.txt
done
for v in product w12 nt; do
  if [ $v = product ]; then LIB=$L; else LIB=tools/ab_libs/$v.so; fi
  for pc in "p4 FETCH_SIZE" "p5 WRITE_SIZE"; do
    set -- $pc
    MQ_LIB=$LIB timeout -k 10 240 rocprofv3 --pmc $2 --output-format csv -d $O/pmc_$v/$1 -o run -- python3 tools/prof_driver.py c 1048576 2 > $O/pmc_${v}_$1.log 2>&1 || { echo "pmc $v $1 failed"; tail -5 $O/pmc_${v}_$1.log; exit 1; }
  done
  python tools/pmc_summary.py $O/pmc_$v --tiles 131072 > $O/pmc_traffic_$v.txt || exit 1
  echo "== traffic $v"; grep -A3 "aes_seal1\|aes_open1" $O/pmc_traffic_$v.txt | grep -E "==|HBM"
done
echo R04R_DONE
