#!/bin/bash
# r06h: narrow AES-128-GCM tiles (16 packets per wave): parity vs the oracle, then the flat AES
# length sweep with the narrow kernels forced off / on / by the product choice
set -o pipefail
O=gpurun_out/r06h; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_narrow.py -k aes > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for m in 0 1; do
  MQ_AES_NARROW=$m timeout -k 10 300 python3 tools/len_sweep.py a 64 128 256 448 512 700 1200 > $O/sweep_$m.txt 2>&1 || { tail $O/sweep_$m.txt; exit 1; }
  echo "== MQ_AES_NARROW=$m"; cat $O/sweep_$m.txt
done
