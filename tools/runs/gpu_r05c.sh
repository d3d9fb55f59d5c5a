# Round-5 call C: config-E cost split (tools/e_parts.py), with and without the forked hot-key kernel
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05c}
mkdir -p $O
timeout -k 10 300 python3 tools/e_parts.py > $O/e_parts.txt 2>&1 || { tail $O/e_parts.txt; exit 1; }
cat $O/e_parts.txt
MQ_FORK=0 timeout -k 10 300 python3 tools/e_parts.py > $O/e_parts_nofork.txt 2>&1 || { tail $O/e_parts_nofork.txt; exit 1; }
cat $O/e_parts_nofork.txt
echo R05C_DONE
