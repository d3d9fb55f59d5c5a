#!/bin/bash
# r06s: multi-key AES kernels with 16-packet tiles (a tile over two keys as two octet tiles): GPU
# suite, E parts, A/B of E and C with 4096 keys against octet multi-key tiles
set -o pipefail
O=gpurun_out/r06s; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 tools/e_parts.py > $O/e_parts.txt 2>&1 || { tail $O/e_parts.txt; exit 1; }
grep -v amdgpu.ids $O/e_parts.txt
timeout -k 10 600 python3 tools/ab_env.py e 1048576 product:MQ_AES_MULTI_NARROW=0 product > $O/ab_e.txt 2>&1 || { tail $O/ab_e.txt; exit 1; }
tail -2 $O/ab_e.txt
