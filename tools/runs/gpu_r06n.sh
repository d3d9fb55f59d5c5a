#!/bin/bash
# r06n: config E parts and kernel stats after the narrow AES tiles
set -o pipefail
O=gpurun_out/r06n; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python3 tools/e_parts.py > $O/e_parts.txt 2>&1 || { tail $O/e_parts.txt; exit 1; }
cat $O/e_parts.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_e -o run -- python3 bench.py --no-cpu-baseline --config e > $O/prof_e.json 2> $O/prof_e.err || { tail $O/prof_e.err; exit 1; }
python3 - <<'PY'
import csv,glob
f=glob.glob("gpurun_out/r06n/prof_e/**/run_kernel_stats.csv", recursive=True)[0]
rows=list(csv.DictReader(open(f)))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:14]: print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1),'us')
PY
