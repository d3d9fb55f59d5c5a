# Round-4 call ZE: the send / receive composites at 2^20 packets over fewer connections (4096 is the
# aux bench): 1024, 64, 4, 1. The receive walk runs one wave per connection.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04ze}
mkdir -p $O
for c in 4096 1024 64 4 1; do
  timeout -k 10 150 python3 tools/prof_aux.py both 3 $c > $O/c$c.txt 2>&1 || { tail $O/c$c.txt; exit 1; }
  echo "conns $c $(tail -1 $O/c$c.txt)"
done
echo R04ZE_DONE
