#!/bin/bash
# r06x: mq_chacha.hip compiled with -amdgpu-sched-strategy=max-ilp (A/B, B, B/1024 keys, E)
set -o pipefail
O=gpurun_out/r06x; mkdir -p $O
for c in b e bk; do
  timeout -k 10 900 python3 tools/ab_env.py $c 1048576 product tools/ab_libs/cc_maxilp.so > $O/ab_$c.txt 2>&1 || { tail $O/ab_$c.txt; exit 1; }
  tail -2 $O/ab_$c.txt
done
