# r06f: pipelined persistent open pre-pass (mq_tile.h prepass_walk) — its parity tests and the full
# GPU suite, then configs B and C against r05's one-packet-per-thread pre-pass (MQ_HP_LOOP=0) and an
# 8-blocks-per-CU build, alternating (tools/ab_env.py), and a kernel trace of B's open
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r06f}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
L=tools/ab_libs
for c in b c; do
  timeout -k 10 600 python tools/ab_env.py $c 1048576 product product:MQ_HP_LOOP=0 $L/hp8.so > $O/ab_$c.txt 2>&1 || { cat $O/ab_$c.txt; exit 1; }
  cat $O/ab_$c.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b -o run -- python3 bench.py --no-cpu-baseline --steps 20 > $O/prof_b.json 2> $O/prof_b.err || { tail $O/prof_b.err; exit 1; }
echo ALL_OK
