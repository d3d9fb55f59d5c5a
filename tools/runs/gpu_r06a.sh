# r06a: ADVICE r05 fixes (diagnostic switches as atomics, flat ChaCha kernel choice from the length
# hint, recv verify word, fallback attempt count) — all GPU tests, bench B / E / B end-to-end.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r06a}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_b.json || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --config e > $O/bench_e.json || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --e2e > $O/bench_b_e2e.json || exit 1
python - <<PY
import json
for k in ("b", "e", "b_e2e"):
    d = json.load(open("$O/bench_%s.json" % k))
    print(k, d["value"], d.get("roofline", {}).get("seal_ms"), d.get("end_to_end"))
PY
echo ALL_OK
