# r06b: what a second AAD block costs (tools/aad_probe.py), config-E parts on the current tree
# (tools/e_parts.py), rocprofv3 kernel trace of E (per-kernel start/end for the overlap timeline).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r06b}
mkdir -p $O
timeout -k 10 400 python tools/aad_probe.py > $O/aad_probe.txt 2>&1 || { tail $O/aad_probe.txt; exit 1; }
cat $O/aad_probe.txt
timeout -k 10 400 python tools/e_parts.py > $O/e_parts.txt 2>&1 || { tail $O/e_parts.txt; exit 1; }
cat $O/e_parts.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_e -o run -- python3 bench.py --no-cpu-baseline --config e --steps 10 > $O/trace_e.json 2> $O/trace_e.err || { tail $O/trace_e.err; exit 1; }
echo ALL_OK
