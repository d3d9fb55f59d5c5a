#!/bin/bash
# r06l: AES tiles of 32 packets on 2 lanes each (MQ_AES_NARROW=2) against the 16-packet narrow
# tiles: parity, length sweep, A/B of c, ck, e
set -o pipefail
O=gpurun_out/r06l; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_narrow.py -k aes > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for m in 1 2; do
  MQ_AES_NARROW=$m timeout -k 10 300 python3 tools/len_sweep.py a 64 128 256 448 700 1024 1200 1500 > $O/sweep_$m.txt 2>&1 || { tail $O/sweep_$m.txt; exit 1; }
  echo "== MQ_AES_NARROW=$m"; cat $O/sweep_$m.txt
done
for c in c ck e; do
  timeout -k 10 600 python3 tools/ab_env.py $c 1048576 product product:MQ_AES_NARROW=2 > $O/ab_$c.txt 2>&1 || { tail $O/ab_$c.txt; exit 1; }
  tail -2 $O/ab_$c.txt
done
