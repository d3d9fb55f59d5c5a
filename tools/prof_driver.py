"""Minimal profiling driver: `reps` seal+open passes of one workload (for rocprofv3 runs).

Usage: python tools/prof_driver.py [b|c|e|ck] [packets] [reps]   (ck: config C with 1024 keys)
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from milli_quic_amd import _lib, batch, workload  # noqa: E402
from milli_quic_amd.batch import KeyTable  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "b"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    assert _lib.load().mq_device_init(0) == 0
    w = {"b": workload.config_b, "c": workload.config_c, "e": workload.config_e,
         "ck": lambda m: workload.config_c(m, n_keys=1024)}[cfg](n)
    dev = torch.device("cuda", 0)
    kt = KeyTable(w.keys)
    arena = torch.from_numpy(w.arena).to(dev)
    sd = torch.from_numpy(w.seal_desc.view(np.uint8)).to(dev)
    od = torch.from_numpy(w.open_desc.view(np.uint8)).to(dev)
    st = torch.zeros(w.n, dtype=torch.uint8, device=dev)
    pn = torch.zeros(w.n, dtype=torch.int64, device=dev)
    ws = torch.empty(max(batch.workspace_bytes(w.n), 256), dtype=torch.uint8, device=dev)
    for _ in range(reps):
        batch.seal(kt, arena, sd, st, w.suite_hint, ws)
        batch.open_(kt, arena, od, st, pn, w.suite_hint, ws)
    torch.cuda.synchronize()
    print("failures", int((st != 0).sum()))


if __name__ == "__main__":
    main()
