#!/bin/bash
# Copy the judged artefacts of a tools/gpu_round.sh run (gpurun_out/TAG) into profiles/TAG_*.
set -e
T=$1; O=gpurun_out/$T
for f in bench_b bench_b_e2e bench_c bench_e bench_b_k1024 bench_c_k1024 bench_b_2rank_gloo; do cp $O/$f.json profiles/${T}_$f.json; done
cp $O/aux.json profiles/${T}_aux.json
cp $O/latency.json profiles/${T}_latency_per_packet.json
cp $O/ossl_scaling.txt profiles/${T}_ossl_scaling.txt
cp $O/pmc_b.txt profiles/${T}_pmc_b.txt; cp $O/pmc_c.txt profiles/${T}_pmc_c.txt
cp $O/pmc_traffic_b.json profiles/${T}_pmc_traffic_b.json; cp $O/pmc_traffic_c.json profiles/${T}_pmc_traffic_c.json
# the PMC traffic bench.py quotes as roofline.traffic
cp $O/pmc_traffic_b.json profiles/pmc_traffic_b.json; cp $O/pmc_traffic_c.json profiles/pmc_traffic_c.json
cp $O/tests.log profiles/${T}_gpu_tests.log
for c in b c e; do cp $O/prof_$c/run_kernel_stats.csv profiles/${T}_kernel_stats_$c.csv; done
ls profiles/${T}_* | wc -l
