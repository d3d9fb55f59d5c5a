"""Partition scan-kernel phase times (diagnostic): runs config E's seal with the -DMQ_PART_STAMPS
build (MQ_LIB=tools/ab_libs/part_stamps.so) and prints the scan kernel's phases from its
s_memrealtime stamps (100 MHz): hist scan, barrier, class layout, key scan pass 1, the rest.
Usage: MQ_LIB=... python tools/part_stamps.py [packets]"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from milli_quic_amd import _lib, batch, workload  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    lib = _lib.load()
    assert lib.mq_device_init(0) == 0
    w = workload.config_e(n)
    dev = torch.device("cuda", 0)
    kt = batch.KeyTable(w.keys)
    arena = torch.from_numpy(w.arena).to(dev)
    sd = torch.from_numpy(w.seal_desc.view(np.uint8)).to(dev)
    st = torch.zeros(w.n, dtype=torch.uint8, device=dev)
    ws = torch.empty(max(batch.workspace_bytes(w.n), 256), dtype=torch.uint8, device=dev)
    f = lib.mq_debug_part_stamps
    f.argtypes = [ctypes.c_void_p]
    buf = (ctypes.c_uint64 * 8)()
    names = ["hist scan", "barrier", "class layout", "key scan pass 1", "key scan rest"]
    for rep in range(4):
        batch.seal(kt, arena, sd, st, _lib.MQ_SUITE_MIXED, ws)
        torch.cuda.synchronize()
        assert f(buf) == 0
        t = list(buf)
        d = [(t[i + 1] - t[i]) / 100.0 for i in range(5)]
        print("rep", rep, " ".join(f"{nm} {x:.2f}" for nm, x in zip(names, d)), f"total {(t[5] - t[0]) / 100.0:.2f} us",
              flush=True)


if __name__ == "__main__":
    main()
