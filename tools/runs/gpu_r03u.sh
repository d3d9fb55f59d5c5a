# r03u: PMC HBM traffic (FETCH_SIZE, WRITE_SIZE passes) of configs E and C with 1024 keys on the
# current tree -> profiles/pmc_traffic_{e,c_k1024}.json (bench.py's roofline.traffic), then bench
# lines E and C/1024 keys with that traffic, and kernel stats of config E.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03u
mkdir -p $O
pmc() {  # cfg name counter
  timeout -k 10 240 rocprofv3 --pmc $3 --output-format csv -d $O/pmc_$1/$2 -o run -- python3 tools/prof_driver.py $1 1048576 2 > $O/pmc_$1_$2.log 2>&1 || { echo "pmc $1 $2 failed"; tail -5 $O/pmc_$1_$2.log; return 1; }
}
pmc e p4 FETCH_SIZE && pmc e p5 WRITE_SIZE && pmc ck p4 FETCH_SIZE && pmc ck p5 WRITE_SIZE || exit 1
python tools/pmc_summary.py $O/pmc_e --json profiles/pmc_traffic_e.json > $O/pmc_e.txt && cat $O/pmc_e.txt | grep -E "==|HBM"
python tools/pmc_summary.py $O/pmc_ck --json profiles/pmc_traffic_c_k1024.json > $O/pmc_ck.txt && cat $O/pmc_ck.txt | grep -E "==|HBM"
cp profiles/pmc_traffic_e.json profiles/pmc_traffic_c_k1024.json $O/
for a in "e --config e" "ck --config c --keys 1024"; do
  set -- $a; name=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/bench_$name.json 2> $O/bench_$name.err || { tail $O/bench_$name.err; exit 1; }
  cat $O/bench_$name.json
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_e -o run -- python3 bench.py --config e --no-cpu-baseline --steps 20 > $O/prof_e.json 2> $O/prof_e.err || { tail $O/prof_e.err; exit 1; }
echo R03U_OK
