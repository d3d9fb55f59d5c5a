# Round-4 call ZF: receive walk with the next chunk's inputs prefetched (product) against the
# previous walk (prev.so), alternating, at 4096 / 64 / 1 connections; receive tests.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04zf}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_recv.py -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in 4096 64 1; do
  for r in 1 2 3; do
    for v in product prev; do
      if [ $v = product ]; then L=""; else L="MQ_LIB=tools/ab_libs/$v.so"; fi
      env $L timeout -k 10 150 python3 tools/prof_aux.py recv 5 $c > $O/$v.$c.$r.txt 2>&1 || { tail $O/$v.$c.$r.txt; exit 1; }
      echo "$v conns $c $r $(tail -1 $O/$v.$c.$r.txt | sed 's/.*recv//')"
    done
  done
done
echo R04ZF_DONE
