#!/bin/bash
# r06v: flat narrow AES open with header protection removed inside the tiles (no pre-pass), A/B
set -o pipefail
O=gpurun_out/r06v; mkdir -p $O
timeout -k 10 600 python3 tools/ab_env.py c 1048576 product product:MQ_AES_INTILE_HP=1 > $O/ab_c.txt 2>&1 || { tail $O/ab_c.txt; exit 1; }
tail -2 $O/ab_c.txt
for m in 0 1; do
  MQ_AES_INTILE_HP=$m timeout -k 10 300 python3 tools/len_sweep.py a 64 256 700 1200 > $O/sweep_$m.txt 2>&1 || { tail $O/sweep_$m.txt; exit 1; }
  echo "== MQ_AES_INTILE_HP=$m"; grep -v amdgpu $O/sweep_$m.txt
done
