#!/bin/bash
# r06p: config E parts with the key-segmented AES kernels forced (MQ_AES_SEG=1) against the product
set -o pipefail
O=gpurun_out/r06p; mkdir -p $O
for r in 1 2; do for m in def 1; do
  echo "== MQ_AES_SEG=$m (round $r)"
  if [ $m = def ]; then timeout -k 10 300 python3 tools/e_parts.py > $O/e_parts_$m.$r.txt 2>&1 || { tail $O/e_parts_$m.$r.txt; exit 1; }
  else MQ_AES_SEG=$m timeout -k 10 300 python3 tools/e_parts.py > $O/e_parts_$m.$r.txt 2>&1 || { tail $O/e_parts_$m.$r.txt; exit 1; }; fi
  grep -v amdgpu.ids $O/e_parts_$m.$r.txt
done; done
