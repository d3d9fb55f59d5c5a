# Round-5 call V: per-packet resident server with 4 lanes (mailboxes + resident workgroups): its
# tests, latency and multi-thread throughput, against 1 lane (MQ_RESIDENT_LANES=1)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05v}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_resident.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 tools/bench_latency.py --calls 2000 > $O/latency_4.json 2> $O/latency_4.err || { tail $O/latency_4.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/latency_4.json')); print('4 lanes', d['resident']['chacha20']['seal'], d['resident_throughput'])"
MQ_RESIDENT_LANES=1 timeout -k 10 300 python3 tools/bench_latency.py --calls 2000 > $O/latency_1.json 2> $O/latency_1.err || { tail $O/latency_1.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/latency_1.json')); print('1 lane ', d['resident']['chacha20']['seal'], d['resident_throughput'])"
echo R05V_DONE
