#!/bin/bash
# r06m: AES lanes per packet by length (2 / 4 / 8): whole GPU suite, bench lines C, C-1024, E, B,
# the AES length sweep
set -o pipefail
O=gpurun_out/r06m; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for a in "c --config c" "ck --config c --keys 1024" "e --config e" "b --config b"; do
  set -- $a; name=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/bench_$name.json 2> $O/bench_$name.err || { tail $O/bench_$name.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('$O/bench_$name.json'));r=d['roofline'];print('$name',d['value'],r['seal_ms'],r['open_ms'],r['frac'])"
done
timeout -k 10 300 python3 tools/len_sweep.py a 64 128 256 448 700 1200 2048 > $O/sweep.txt 2>&1 || { tail $O/sweep.txt; exit 1; }
cat $O/sweep.txt
