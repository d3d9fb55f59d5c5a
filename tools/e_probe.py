"""Config-E cost probe: seal / open medians of the mixed batch as generated, and with every
Initial packet moved onto the hot 1-RTT AES row (so every AES tile can use the H^8 table) —
the difference is what the multi-key GHASH costs. Diagnostic only.
Usage: python tools/e_probe.py [packets]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(n):
    import numpy as np
    import torch
    from milli_quic_amd import _lib
    from milli_quic_amd import batch, workload
    assert _lib.load().mq_device_init(0) == 0
    w = workload.config_e(n)
    dev = torch.device("cuda", 0)
    kt = batch.KeyTable(w.keys)
    init = w.seal_desc["key_id"] >= 2
    for variant in ("as generated", "Initial on hot row", "as generated"):
        sd_np, od_np = w.seal_desc.copy(), w.open_desc.copy()
        if variant == "Initial on hot row":
            sd_np["key_id"][init] = 1
            od_np["key_id"][init] = 1
        arena0 = torch.from_numpy(w.arena).to(dev)
        arena = arena0.clone()
        sd = torch.from_numpy(sd_np.view(np.uint8)).to(dev)
        od = torch.from_numpy(od_np.view(np.uint8)).to(dev)
        st = torch.zeros(w.n, dtype=torch.uint8, device=dev)
        pn = torch.zeros(w.n, dtype=torch.int64, device=dev)
        ws = torch.empty(max(batch.workspace_bytes(w.n), 256), dtype=torch.uint8, device=dev)
        res = {"seal": [], "open": []}
        for rep in range(10):
            arena.copy_(arena0)
            for which in ("seal", "open"):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                if which == "seal":
                    batch.seal(kt, arena, sd, st, w.suite_hint, ws)
                else:
                    batch.open_(kt, arena, od, st, pn, w.suite_hint, ws)
                e1.record()
                torch.cuda.synchronize()
                if which == "open":
                    assert int((st != 0).sum()) == 0, "open failed"
                if rep >= 2:
                    res[which].append(e0.elapsed_time(e1))
        print(f"{variant:22s} seal {np.median(res['seal']):.4f} ms  open {np.median(res['open']):.4f} ms", flush=True)


if __name__ == "__main__":
    run(int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20)
