set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02b
mkdir -p $O
timeout -k 10 120 ./tools/ubench/ubench4 new > $O/ubench_valu_r02.txt 2>&1 || { cat $O/ubench_valu_r02.txt; exit 1; }
cat $O/ubench_valu_r02.txt
timeout -k 10 300 python bench.py --keys 1024 --no-cpu-baseline > $O/bench_b_k1024.json 2> $O/bench_b_k1024.err || { tail $O/bench_b_k1024.err; exit 1; }
cat $O/bench_b_k1024.json
timeout -k 10 300 python bench.py --config c --keys 1024 --no-cpu-baseline > $O/bench_c_k1024.json 2> $O/bench_c_k1024.err || { tail $O/bench_c_k1024.err; exit 1; }
cat $O/bench_c_k1024.json
timeout -k 10 300 python bench.py --config c --no-cpu-baseline > $O/bench_c.json 2> $O/bench_c.err || { tail $O/bench_c.err; exit 1; }
cat $O/bench_c.json
timeout -k 10 300 python bench.py --config e --no-cpu-baseline > $O/bench_e.json 2> $O/bench_e.err || { tail $O/bench_e.err; exit 1; }
cat $O/bench_e.json
echo G2_OK
