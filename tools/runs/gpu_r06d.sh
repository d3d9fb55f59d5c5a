# r06d: config E with the ChaCha20 list beside the AES kernels (MQ_MIXED_CO=1) and multi-key AES
# kernels of 4 / 6 waves (room for a ChaCha20 workgroup on each CU), alternating A/B (tools/ab_env.py)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r06d}
mkdir -p $O
L=tools/ab_libs
timeout -k 10 900 python tools/ab_env.py e 1048576 product product:MQ_MIXED_CO=1 $L/aes6.so $L/aes6.so:MQ_MIXED_CO=1 $L/aes4.so:MQ_MIXED_CO=1 > $O/ab_e.txt 2>&1 || { cat $O/ab_e.txt; exit 1; }
cat $O/ab_e.txt
