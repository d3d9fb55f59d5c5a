#!/bin/bash
# r06j: narrow AES kernels as the product for flat single-key batches <= 1792 B and the hot key's
# partition segment: whole GPU suite, A/B of C and E (narrow forced off vs product), sweep near the
# threshold
set -o pipefail
O=gpurun_out/r06j; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for m in 0 1; do
  MQ_AES_NARROW=$m timeout -k 10 300 python3 tools/len_sweep.py a 1600 1792 2048 > $O/sweep_$m.txt 2>&1 || { tail $O/sweep_$m.txt; exit 1; }
  echo "== MQ_AES_NARROW=$m"; cat $O/sweep_$m.txt
done
for c in c e; do
  timeout -k 10 600 python3 tools/ab_env.py $c 1048576 product:MQ_AES_NARROW=0 product > $O/ab_$c.txt 2>&1 || { tail $O/ab_$c.txt; exit 1; }
  cat $O/ab_$c.txt
done
