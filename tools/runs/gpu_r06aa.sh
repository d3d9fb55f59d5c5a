#!/bin/bash
# r06aa: multi-key AES kernels at 8 waves per CU (no spills) against 12 (A/B, config E)
set -o pipefail
O=gpurun_out/r06aa; mkdir -p $O
timeout -k 10 900 python3 tools/ab_env.py e 1048576 product tools/ab_libs/multi8.so > $O/ab_e.txt 2>&1 || { tail $O/ab_e.txt; exit 1; }
tail -2 $O/ab_e.txt
