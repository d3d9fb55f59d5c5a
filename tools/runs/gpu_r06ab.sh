#!/bin/bash
# r06ab: config E with the multi-key AES kernel after the hot segment on the side stream (ChaCha20
# list right after the partition on the caller's stream), A/B; parity of E under the switch
set -o pipefail
O=gpurun_out/r06ab; mkdir -p $O
MQ_AES_MULTI_HOT=1 timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_narrow.py tests/test_gpu_parity.py -k "partitioned or config_e or mixed" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 900 python3 tools/ab_env.py e 1048576 product product:MQ_AES_MULTI_HOT=1 > $O/ab_e.txt 2>&1 || { tail $O/ab_e.txt; exit 1; }
tail -2 $O/ab_e.txt
