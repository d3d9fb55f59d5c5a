#!/bin/bash
# r06r: config E with list 1 (ChaCha20) after the hot AES segment on its side stream, with the hot
# segment on the slice kernel or on the tile kernel (alternating A/B)
set -o pipefail
O=gpurun_out/r06r; mkdir -p $O
timeout -k 10 900 python3 tools/ab_env.py e 1048576 product product:MQ_LIST1_HOT=1 product:MQ_AES_HOT_SEG=0 product:MQ_AES_HOT_SEG=0,MQ_LIST1_HOT=1 > $O/ab_e.txt 2>&1 || { tail $O/ab_e.txt; exit 1; }
tail -4 $O/ab_e.txt
