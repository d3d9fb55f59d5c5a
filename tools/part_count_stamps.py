"""Partition phase times (diagnostic): runs a mixed batch's seal with the -DMQ_STAMPS build
(libmq_aead_stamps.so) and prints the count and scatter kernels' phases from thread 0's
s_memrealtime stamps (100 MHz, one clock for the whole device), relative to each kernel's first
block start: median / max over blocks of each boundary, and the count kernel's last (layout) block.
Diagnostic only: never quote its times as kernel durations.
Usage: python tools/part_count_stamps.py [e|ck] [packets]"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from milli_quic_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(ROOT, "milli_quic_amd", "libmq_aead_stamps.so")
from milli_quic_amd import batch, workload  # noqa: E402

COUNT = ["entry", "fetched", "item atomics", "flushed", "done count", "layout end"]
SCATTER = ["entry", "fetched", "item ranks", "reservations", "end"]


def show(name, s, labels):
    ok = s[:, 0] > 0
    s = s[ok]
    t0 = s[:, 0].min()
    print(f"[{name}] blocks={len(s)}")
    for k, lab in enumerate(labels):
        v = s[:, k]
        v = v[v > 0]
        if len(v) == 0:
            continue
        r = (v - t0) / 100.0
        print(f"   {k}:{lab:14s} median={np.median(r):7.2f} us  max={r.max():7.2f} us  (blocks {len(v)})")


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "e"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
    lib = _lib.load()
    lib.mq_debug_set_part_stamps.argtypes = [ctypes.c_void_p]
    assert lib.mq_device_init(0) == 0
    if cfg == "ck":
        w = workload.uniform(n, _lib.MQ_SUITE_AES128GCM, n_keys=1024)
    else:
        w = workload.config_e(n)
    dev = torch.device("cuda", 0)
    kt = batch.KeyTable(w.keys)
    arena = torch.from_numpy(w.arena).to(dev)
    sd = torch.from_numpy(w.seal_desc.view(np.uint8)).to(dev)
    st = torch.zeros(w.n, dtype=torch.uint8, device=dev)
    ws = torch.empty(max(batch.workspace_bytes(w.n), 256), dtype=torch.uint8, device=dev)
    nb = (w.n + 4095) // 4096  # mq_partition.hip kPartBlock
    buf = torch.zeros(2 * nb * 8, dtype=torch.int64, device=dev)
    lib.mq_debug_set_part_stamps(ctypes.c_void_p(buf.data_ptr()))
    for rep in range(3):
        buf.zero_()
        batch.seal(kt, arena, sd, st, w.suite_hint, ws)
        torch.cuda.synchronize()
        if rep == 0:
            continue
        s = buf.cpu().numpy().reshape(2 * nb, 8).astype(np.int64)
        print(f"rep {rep} ({cfg}, {w.n} packets)")
        show("count", s[:nb], COUNT)
        show("scatter", s[nb:], SCATTER)
        gap = (s[nb:, 0][s[nb:, 0] > 0].min() - s[:nb, 5].max()) / 100.0
        print(f"   layout end -> first scatter block: {gap:.2f} us (keyed: the row blocks between)")
    print("failures", int((st != 0).sum()))


if __name__ == "__main__":
    main()
