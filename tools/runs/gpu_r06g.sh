# r06g: config E with the multi-key AES kernel's key-uniform tiles multiplying by H^8 through the
# integer (bit-holed) product instead of the wave's half table (LDS-bound vs VALU-bound), A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r06g}
mkdir -p $O
timeout -k 10 900 python tools/ab_env.py e 1048576 product tools/ab_libs/uprod.so > $O/ab_e.txt 2>&1 || { cat $O/ab_e.txt; exit 1; }
cat $O/ab_e.txt
