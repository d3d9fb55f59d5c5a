#!/bin/bash
# r06t: static tile stride (MQ_SCHED=0) against the dynamic schedule for the narrow AES kernels
set -o pipefail
O=gpurun_out/r06t; mkdir -p $O
for c in c e; do
  timeout -k 10 600 python3 tools/ab_env.py $c 1048576 product product:MQ_SCHED=0 > $O/ab_$c.txt 2>&1 || { tail $O/ab_$c.txt; exit 1; }
  tail -2 $O/ab_$c.txt
done
