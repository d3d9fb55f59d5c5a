#!/bin/bash
# r06u: flat single-key AES batches on the slice walk (MQ_AES_FLAT_SLICE=1): parity under the switch,
# A/B of C and of the short-packet sweep
set -o pipefail
O=gpurun_out/r06u; mkdir -p $O
MQ_AES_FLAT_SLICE=1 timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_narrow.py tests/test_gpu_parity.py -k "aes or config_c or full_size" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python3 tools/ab_env.py c 1048576 product product:MQ_AES_FLAT_SLICE=1 > $O/ab_c.txt 2>&1 || { tail $O/ab_c.txt; exit 1; }
tail -2 $O/ab_c.txt
for m in 0 1; do
  MQ_AES_FLAT_SLICE=$m timeout -k 10 300 python3 tools/len_sweep.py a 64 256 700 1200 > $O/sweep_$m.txt 2>&1 || { tail $O/sweep_$m.txt; exit 1; }
  echo "== MQ_AES_FLAT_SLICE=$m"; grep -v amdgpu $O/sweep_$m.txt
done
