# Round-4 call P: ChaCha20 pool with one own iteration per packet (MQ_CC_POOL_ITERS=1, own1.so)
# against the product (two) on configs E and B; A/B alternating child processes (tools/ab.py).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04p}
mkdir -p $O
L=milli_quic_amd/libmq_aead.so
for c in e b; do
  echo "== ab_$c $(date +%T)"
  timeout -k 10 600 python tools/ab.py $c 1048576 $L tools/ab_libs/own1.so > $O/ab_$c.txt 2>&1 || { cat $O/ab_$c.txt; exit 1; }
  cat $O/ab_$c.txt
done
echo R04P_DONE
