# Round-5 call N: phase cost of the AES seal's header-mask read-modify-write (diagnostic variant
# tools/ab_libs/prof_128.so skips it: garbage headers), product first, twice, on C and E
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05n}
mkdir -p $O
for i in 1 2; do
  for c in c e; do
    MQ_PROF_DIR=tools/ab_libs timeout -k 10 600 python3 tools/phase_cost.py $c > $O/phase_${c}_$i.txt 2>&1 || { tail $O/phase_${c}_$i.txt; exit 1; }
    echo "== $c $i"; grep -v amdgpu.ids $O/phase_${c}_$i.txt
  done
done
echo R05N_DONE
