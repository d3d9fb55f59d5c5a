# Round-4 call X: fused protect with the edge chunks and header bytes built first (product) against
# the previous order (prev.so); send tests; alternating protect timings.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04x}
mkdir -p $O
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_send.py -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  for v in product prev; do
    if [ $v = product ]; then L=""; else L="MQ_LIB=tools/ab_libs/$v.so"; fi
    env $L timeout -k 10 120 python3 tools/prof_aux.py protect 10 > $O/$v.$r.txt 2>&1 || { tail $O/$v.$r.txt; exit 1; }
    echo "$v $r $(tail -1 $O/$v.$r.txt)"
  done
done
echo R04X_DONE
