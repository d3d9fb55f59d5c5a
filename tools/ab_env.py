"""A/B of (library, environment) pairs on one GPU, alternating: each arm is a child process of
tools/phase_cost.py (seal + open medians). Diagnostic only.
Usage: python tools/ab_env.py CFG N ARM...   ARM = LIB[:VAR=VAL[,VAR=VAL...]] (LIB 'product' = the
in-tree library)"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    cfg, n, arms = sys.argv[1], sys.argv[2], sys.argv[3:]
    res = {a: ([], []) for a in arms}
    for _ in range(3):
        for a in arms:
            lib, _, envs = a.partition(":")
            lib = os.path.join(ROOT, "milli_quic_amd", "libmq_aead.so") if lib == "product" else lib
            env = dict(os.environ)
            for kv in filter(None, envs.split(",")):
                k, v = kv.split("=")
                env[k] = v
            out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "phase_cost.py"), "--child", lib, cfg, n],
                                 capture_output=True, text=True, timeout=240, env=env)
            line = [x for x in out.stdout.splitlines() if x.startswith("RESULT")]
            if not line:
                print(a, "FAILED", out.stderr[-600:], flush=True)
                continue
            s, o = map(float, line[0].split()[1:])
            print(f"  {a} seal {s:.4f} open {o:.4f}", flush=True)
            res[a][0].append(s)
            res[a][1].append(o)
    for a, (s, o) in res.items():
        if s:
            print(f"{a:70s} seal {np.median(s):.4f} ms  open {np.median(o):.4f} ms  sum {np.median(s) + np.median(o):.4f}",
                  flush=True)


if __name__ == "__main__":
    main()
