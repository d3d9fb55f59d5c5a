#!/bin/bash
# r06i: narrow AES tiles with the byte-position table of H^4: parity, length sweep forced off / on,
# config C A/B (octet vs narrow kernels on the same box, alternating)
set -o pipefail
O=gpurun_out/r06i; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_narrow.py -k aes > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for m in 0 1; do
  MQ_AES_NARROW=$m timeout -k 10 300 python3 tools/len_sweep.py a 64 256 448 700 900 1024 1200 1350 1500 2048 > $O/sweep_$m.txt 2>&1 || { tail $O/sweep_$m.txt; exit 1; }
  echo "== MQ_AES_NARROW=$m"; cat $O/sweep_$m.txt
done
timeout -k 10 600 python3 tools/ab_env.py c 1048576 product:MQ_AES_NARROW=0 product:MQ_AES_NARROW=1 > $O/ab_c.txt 2>&1 || { tail $O/ab_c.txt; exit 1; }
cat $O/ab_c.txt
