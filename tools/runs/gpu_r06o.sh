#!/bin/bash
# r06o: config E parts with 8 / 4 / 2 lanes per AES packet in the single-key kernels (alternating)
set -o pipefail
O=gpurun_out/r06o; mkdir -p $O
for r in 1 2; do for m in 0 1 2; do
  echo "== MQ_AES_NARROW=$m (round $r)"
  MQ_AES_NARROW=$m timeout -k 10 300 python3 tools/e_parts.py > $O/e_parts_$m.$r.txt 2>&1 || { tail $O/e_parts_$m.$r.txt; exit 1; }
  grep -v amdgpu.ids $O/e_parts_$m.$r.txt
done; done
