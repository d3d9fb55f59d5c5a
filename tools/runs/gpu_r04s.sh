# Round-4 call S: AES single-key wave counts — product (12 waves: stream and key-segmented
# kernels), seg16 (key-segmented kernels at 16), v16 (all single-key kernels at 16, r04 before) on
# configs C/1024 keys, C and E; tools/ab.py alternating child processes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04s}
mkdir -p $O
L=milli_quic_amd/libmq_aead.so
for c in ck c e; do
  echo "== ab_$c $(date +%T)"
  timeout -k 10 600 python tools/ab.py $c 1048576 $L tools/ab_libs/seg16.so tools/ab_libs/v16.so > $O/ab_$c.txt 2>&1 || { cat $O/ab_$c.txt; exit 1; }
  grep sum $O/ab_$c.txt
done
echo R04S_DONE
