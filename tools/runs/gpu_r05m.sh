# Round-5 call M: AES tile phase stamps (diagnostic build) over packet lengths
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05m}
mkdir -p $O
for c in a64 a256 a448 a700 c ak700; do
  echo "== $c"
  timeout -k 10 120 python3 tools/stamps.py $c > $O/stamps_$c.txt 2>&1 || { tail $O/stamps_$c.txt; exit 1; }
  grep -v amdgpu.ids $O/stamps_$c.txt
done
echo R05M_DONE
