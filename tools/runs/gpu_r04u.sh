# Round-4 call U: config E with the ChaCha20 list launched before the AES lists on the caller's
# stream (MQ_MIXED_CHACHA_FIRST=1) against the product order; alternating runs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04u}
mkdir -p $O
for r in 1 2 3; do
  for v in product ccfirst; do
    if [ $v = ccfirst ]; then E="MQ_MIXED_CHACHA_FIRST=1"; else E="MQ_MIXED_CHACHA_FIRST=0"; fi
    env $E timeout -k 10 300 python3 bench.py --no-cpu-baseline --config e --steps 50 > $O/e_$v.$r.json 2> $O/e_$v.$r.err || { tail $O/e_$v.$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], r['seal_ms'], r['open_ms'], d['parity']['match'])" $O/e_$v.$r.json
  done
done
echo R04U_DONE
