# Round-4 call N: phase costs of the fused ChaCha20 protect kernel — the product against builds
# without the edge chunks (pv256), without the frames loads (pv512) and without both (pv768);
# outputs of the diagnostic builds are garbage, only their times count.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04n}
mkdir -p $O
for r in 1 2; do
  for v in product pv256 pv512 pv768; do
    if [ $v = product ]; then L=""; else L="MQ_LIB=tools/ab_libs/$v.so"; fi
    echo "== $v $r"
    env $L timeout -k 10 120 python3 tools/prof_aux.py protect 10 > $O/$v.$r.txt 2>&1 || { tail $O/$v.$r.txt; exit 1; }
    tail -1 $O/$v.$r.txt
  done
done
echo R04N_DONE
