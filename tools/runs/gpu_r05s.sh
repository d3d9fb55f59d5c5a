# Round-5 call S: config-C AES phase costs on the current tree (AES-only variants: 2 no GHASH
# Horner multiply, 16 no AES rounds, 64 no tag final multiply), twice
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05s}
mkdir -p $O
for i in 1 2; do
  MQ_PROF_DIR=tools/ab_libs timeout -k 10 600 python3 tools/phase_cost.py c > $O/phase_c_$i.txt 2>&1 || { tail $O/phase_c_$i.txt; exit 1; }
  grep -v amdgpu.ids $O/phase_c_$i.txt
done
echo R05S_DONE
