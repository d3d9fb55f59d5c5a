# Round-5 call J: config-E parts under AES phase-cost variants (2: no GHASH Horner multiply, 16: no
# AES rounds, 64: no tag final multiply), product library first
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05j}
mkdir -p $O
timeout -k 10 200 python3 tools/e_parts.py > $O/e_parts_prod.txt 2>&1 || { tail $O/e_parts_prod.txt; exit 1; }
cat $O/e_parts_prod.txt
for m in 2 16 64; do
  echo "== variant $m"
  E_NOCHECK=1 MQ_LIB=tools/ab_libs/prof_$m.so timeout -k 10 200 python3 tools/e_parts.py > $O/e_parts_$m.txt 2>&1 || { tail $O/e_parts_$m.txt; exit 1; }
  cat $O/e_parts_$m.txt
done
echo R05J_DONE
