"""A/B timing of library builds on the same GPU: alternates child processes of
tools/phase_cost.py (seal + open medians) for each library, `rounds` times.
Usage: python tools/ab.py CFG N LIB_A LIB_B [...]"""
import subprocess
import sys

import numpy as np


def main():
    cfg, n, libs = sys.argv[1], sys.argv[2], sys.argv[3:]
    res = {lib: ([], []) for lib in libs}
    for _ in range(3):
        for lib in libs:
            out = subprocess.run([sys.executable, "tools/phase_cost.py", "--child", lib, cfg, n],
                                 capture_output=True, text=True, timeout=240)
            line = [x for x in out.stdout.splitlines() if x.startswith("RESULT")]
            if not line:
                print(lib, "FAILED", out.stderr[-400:])
                continue
            s, o = map(float, line[0].split()[1:])
            print(f"  {lib} seal {s:.4f} open {o:.4f}", flush=True)
            res[lib][0].append(s)
            res[lib][1].append(o)
    for lib, (s, o) in res.items():
        if s:
            print(f"{lib:60s} seal {np.median(s):.4f} ms  open {np.median(o):.4f} ms  sum {np.median(s) + np.median(o):.4f}",
                  flush=True)


if __name__ == "__main__":
    main()
