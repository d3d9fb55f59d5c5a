# Round-4 call M: config E kernels in isolation (MQ_FORK=0: the hot AES key, the other AES keys and
# the ChaCha list one after another on the caller's stream) against the forked schedule.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04m}
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step bench_e_nofork
MQ_FORK=0 timeout -k 10 300 python3 bench.py --no-cpu-baseline --config e > $O/bench_e_nofork.json 2> $O/bench_e_nofork.err || { tail $O/bench_e_nofork.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], r['seal_ms'], r['open_ms'], r['frac'])" $O/bench_e_nofork.json
step prof_e_nofork
MQ_FORK=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_e_nofork -o run -- python3 bench.py --no-cpu-baseline --config e --steps 20 > $O/prof_e_nofork.json 2> $O/prof_e_nofork.err || { tail $O/prof_e_nofork.err; exit 1; }
grep -E "chacha|aes_seal|aes_open|part_" $O/prof_e_nofork/run_kernel_stats.csv
echo R04M_DONE
