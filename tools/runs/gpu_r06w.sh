#!/bin/bash
# r06w: LLVM AMDGPU scheduler strategies for the ChaCha20 and AES tile kernels (A/B, B and C)
set -o pipefail
O=gpurun_out/r06w; mkdir -p $O
L=tools/ab_libs
for c in b c; do
  timeout -k 10 900 python3 tools/ab_env.py $c 1048576 product $L/sched_max-ilp.so $L/sched_max-memory-clause.so $L/sched_iterative-ilp.so > $O/ab_$c.txt 2>&1 || { tail $O/ab_$c.txt; exit 1; }
  tail -4 $O/ab_$c.txt
done
