# Round-6 final artifacts on the final tree, one gpurun call: parity tests; PMC HBM traffic of the
# bench configs (written into profiles/ first, so the bench lines' roofline.traffic reads them);
# bench lines B (with CPU baselines), B end-to-end, C, C/1024 keys, E, B/1024 keys; rocprofv3
# kernel stats of B, C, C/1024 keys, E; PMC instruction / LDS passes of B and C; the 2-rank
# launcher rehearsal (gloo); kernel stats of the driver's own bench command and of the receive /
# protect composites; per-packet latency; aux components; smoke. Every GPU step is time-limited;
# the script stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r06final2}
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
PART=${2:-1}
if [ "$PART" = 1 ]; then
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
step pmc_traffic
pmc() {  # cfg counter pass
  timeout -k 10 240 rocprofv3 --pmc $2 --output-format csv -d $O/pmc_$1/$3 -o run -- python3 tools/prof_driver.py $1 1048576 2 > $O/pmc_$1_$3.log 2>&1 || { echo "pmc $1 $2 failed"; tail -5 $O/pmc_$1_$3.log; return 1; }
}
for c in b c ck e; do pmc $c FETCH_SIZE p4 && pmc $c WRITE_SIZE p5 || exit 1; done
python tools/pmc_summary.py $O/pmc_b --tiles 131072 --json profiles/pmc_traffic_b.json > $O/pmc_traffic_b.txt || exit 1
python tools/pmc_summary.py $O/pmc_c --tiles 131072 --json profiles/pmc_traffic_c.json > $O/pmc_traffic_c.txt || exit 1
python tools/pmc_summary.py $O/pmc_ck --json profiles/pmc_traffic_c_k1024.json > $O/pmc_traffic_ck.txt || exit 1
python tools/pmc_summary.py $O/pmc_e --json profiles/pmc_traffic_e.json > $O/pmc_traffic_e.txt || exit 1
cp profiles/pmc_traffic_b.json profiles/pmc_traffic_c.json profiles/pmc_traffic_c_k1024.json profiles/pmc_traffic_e.json $O/
grep -hE "==|HBM" $O/pmc_traffic_*.txt
step bench_b
timeout -k 10 400 python bench.py > $O/bench_b.json 2> $O/bench_b.err || { tail $O/bench_b.err; exit 1; }
cat $O/bench_b.json
for a in "c --config c" "ck --config c --keys 1024" "e --config e" "bk --config b --keys 1024"; do
  set -- $a; name=$1; shift
  step bench_$name
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/bench_$name.json 2> $O/bench_$name.err || { tail $O/bench_$name.err; exit 1; }
  cat $O/bench_$name.json
done
step bench_b_e2e
timeout -k 10 600 python bench.py --no-cpu-baseline --e2e > $O/bench_b_e2e.json 2> $O/bench_b_e2e.err || { tail $O/bench_b_e2e.err; exit 1; }
cat $O/bench_b_e2e.json
echo PART1_OK
exit 0
fi
for a in "b --config b" "c --config c" "ck --config c --keys 1024" "e --config e"; do
  set -- $a; name=$1; shift
  step prof_$name
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$name -o run -- python3 bench.py --no-cpu-baseline "$@" > $O/prof_$name.json 2> $O/prof_$name.err || { tail $O/prof_$name.err; exit 1; }
done
step pmc_instr
for c in b c; do
  for p in "p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "p2 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
           "p3 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
    set -- $p; name=$1; shift
    timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d $O/pmc_$c/$name -o run -- python3 tools/prof_driver.py $c 1048576 2 > $O/pmc_${c}_$name.log 2>&1 || { echo "pmc $c $name failed"; exit 1; }
  done
  python tools/pmc_summary.py $O/pmc_$c --tiles 131072 > $O/pmc_$c.txt || exit 1
done
step prof_driver_cmd
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_d20 -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_d20.json 2> $O/prof_d20.err || { tail $O/prof_d20.err; exit 1; }
for a in protect recv; do
  step prof_$a
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$a -o run -- python3 tools/prof_aux.py $a 5 > $O/prof_$a.log 2>&1 || { tail $O/prof_$a.log; exit 1; }
done
step gloo_2rank
MQ_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --no-cpu-baseline > $O/bench_b_2rank_gloo.json 2> $O/bench_b_2rank_gloo.err || { tail $O/bench_b_2rank_gloo.err; exit 1; }
cat $O/bench_b_2rank_gloo.json
step latency
timeout -k 10 300 python tools/bench_latency.py > $O/latency.json 2> $O/latency.err || { tail $O/latency.err; exit 1; }
cat $O/latency.json
step aux
timeout -k 10 400 python tools/bench_aux.py > $O/aux.json 2> $O/aux.err || { tail $O/aux.err; exit 1; }
cat $O/aux.json
step sweep
timeout -k 10 400 python3 tools/len_sweep.py both 64 128 256 448 700 1200 1232 1350 1452 1584 1600 2048 2400 > $O/len_sweep.txt 2>&1 || { tail $O/len_sweep.txt; exit 1; }
cat $O/len_sweep.txt
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
echo ROUND_OK
