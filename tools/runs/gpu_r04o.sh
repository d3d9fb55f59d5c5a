# Round-4 call O: send tests and the fused protect kernel's time (header bytes from row windows).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04o}
mkdir -p $O
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_send.py tests/test_gpu_recv.py -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3; do
  timeout -k 10 120 python3 tools/prof_aux.py protect 10 > $O/protect.$r.txt 2>&1 || { tail $O/protect.$r.txt; exit 1; }
  tail -1 $O/protect.$r.txt
done
echo R04O_DONE
