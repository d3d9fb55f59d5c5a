#!/bin/bash
# r06k: narrow tiles inside the key-segmented AES kernels (config C with 1024 keys): whole GPU
# suite, A/B of ck, c, e (narrow forced off vs product)
set -o pipefail
O=gpurun_out/r06k; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for c in ck c e; do
  timeout -k 10 600 python3 tools/ab_env.py $c 1048576 product:MQ_AES_NARROW=0 product > $O/ab_$c.txt 2>&1 || { tail $O/ab_$c.txt; exit 1; }
  cat $O/ab_$c.txt
done
