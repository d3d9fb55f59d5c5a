#!/bin/bash
# r06q: the partition's hot AES segment on the slice (key-segmented) kernel: GPU suite, E parts and
# an alternating A/B of E against the hot-split tile kernel (MQ_AES_HOT_SEG=0)
set -o pipefail
O=gpurun_out/r06q; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 tools/e_parts.py > $O/e_parts.txt 2>&1 || { tail $O/e_parts.txt; exit 1; }
grep -v amdgpu.ids $O/e_parts.txt
timeout -k 10 600 python3 tools/ab_env.py e 1048576 product:MQ_AES_HOT_SEG=0 product > $O/ab_e.txt 2>&1 || { tail $O/ab_e.txt; exit 1; }
tail -2 $O/ab_e.txt
