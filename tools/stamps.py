"""Phase breakdown of the tile kernels from the diagnostic build (libmq_aead_stamps.so).

Each tile's lane 0 records s_memtime (shader clock) at: 0 start, 1 staged (table ready), 2 DMA
landed, 3/4/5 policy phases, 6 policy done, 7 stored. Reports the median / mean cycles of each
phase for seal and open, plus tiles resident per CU. Diagnostic only: never quote its times.
Usage: python tools/stamps.py [b|c|e|a<L>|ak<L>] [packets]   (a<L>: AES n x L B, ak<L>: with 1024 keys)
"""
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
from milli_quic_amd.batch import KeyTable  # noqa: E402

NAMES = {"seal": ["setup", "dma+blk0", "chacha", "poly+tag", "hp", "-", "store"],
         "open": ["setup", "dma", "hp+unmask", "blk0+poly+verify", "xor", "-", "store"]}
AES_NAMES = {"seal": ["setup", "iteration 0", "iterations 1+", "finish+tag", "late hp+mask", "-", "status"],
             "open": ["hp+setup", "iteration 0", "iterations 1+", "finish", "-", "-", "verify+restore+status"]}


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "b"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
    lib = _lib.load()
    lib.mq_debug_set_stamps.argtypes = [ctypes.c_void_p]
    assert lib.mq_device_init(0) == 0
    if cfg.startswith("a"):  # a<L>: AES-128-GCM, n x L bytes, one key; ak<L>: 1024 keys
        kk = 1024 if cfg.startswith("ak") else 1
        w = workload.uniform(n, _lib.MQ_SUITE_AES128GCM, L=int(cfg.lstrip("ak")), n_keys=kk)
    else:
        w = {"b": workload.config_b, "c": workload.config_c, "e": workload.config_e}[cfg](n)
    names = AES_NAMES if cfg[0] in "ca" else NAMES
    dev = torch.device("cuda", 0)
    kt = KeyTable(w.keys)
    arena = torch.from_numpy(w.arena).to(dev)
    sd = torch.from_numpy(w.seal_desc.view(np.uint8)).to(dev)
    od = torch.from_numpy(w.open_desc.view(np.uint8)).to(dev)
    st = torch.zeros(w.n, dtype=torch.uint8, device=dev)
    pn = torch.zeros(w.n, dtype=torch.int64, device=dev)
    tiles = (w.n + 7) // 8  # kPktsPerTile
    buf = torch.zeros(tiles * 8, dtype=torch.int64, device=dev)
    lib.mq_debug_set_stamps(ctypes.c_void_p(buf.data_ptr()))
    for rep in range(2):
        for which in ("seal", "open"):
            buf.zero_()
            if which == "seal":
                batch.seal(kt, arena, sd, st, w.suite_hint)
            else:
                batch.open_(kt, arena, od, st, pn, w.suite_hint)
            torch.cuda.synchronize()
            if rep == 0:
                continue
            s = buf.cpu().numpy().reshape(tiles, 8).astype(np.int64)
            t0 = s[:, 0].min()
            life = s[:, 7] - s[:, 0]
            print(f"[{which}] tiles={tiles} kernel span={s[:, 7].max() - t0} cycles, tile life median="
                  f"{int(np.median(life))} mean={int(life.mean())}")
            prev = s[:, 0]
            for k in range(1, 8):
                d = s[:, k] - prev
                ok = s[:, k] > 0
                if ok.sum() == 0:
                    continue
                print(f"   {k}:{names[which][k - 1]:18s} median={int(np.median(d[ok])):7d} mean={int(d[ok].mean()):7d}"
                      f"  ({100 * d[ok].mean() / life.mean():.1f}%)")
                prev = np.where(ok, s[:, k], prev)
            # concurrency: tiles alive at the midpoint of the kernel
            mid = t0 + (s[:, 7].max() - t0) // 2
            alive = ((s[:, 0] <= mid) & (s[:, 7] >= mid)).sum()
            print(f"   tiles alive at midpoint: {alive} ({alive / 256:.2f} per CU)")
    print("failures", int((st != 0).sum()))


if __name__ == "__main__":
    main()
