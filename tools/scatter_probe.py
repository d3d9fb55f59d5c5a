"""Does a tile's memory footprint cost the AES kernels? Config C (2^20 x 1200-B AES-128-GCM
packets) sealed and opened through the flat single-key path (a) in descriptor order (a tile's 8
packets adjacent in the arena) and (b) with the descriptors permuted so that a tile's 8 packets lie
1024 packets (1.2 MB) apart — the footprint the partition's key-uniform tiles have in config C with
1024 keys (key_id = g mod 1024). Same packets, same kernel, same work; only the order differs.
Also (c) config C with 1024 keys through the partition (keyed layout). Prints one JSON line of
median seal / open milliseconds. Diagnostic only."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from milli_quic_amd import _lib, batch, workload  # noqa: E402


def timed(fn, reps=10):
    t = []
    for r in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        if r >= 2:
            t.append(e0.elapsed_time(e1))
    return round(float(np.median(t)), 4)


def run(w, order, hint):
    dev = torch.device("cuda", 0)
    kt = batch.KeyTable(w.keys)
    arena = torch.from_numpy(w.arena).to(dev)
    sd = torch.from_numpy(w.seal_desc[order].view(np.uint8)).to(dev)
    od = torch.from_numpy(w.open_desc[order].view(np.uint8)).to(dev)
    st = torch.zeros(w.n, dtype=torch.uint8, device=dev)
    pn = torch.zeros(w.n, dtype=torch.int64, device=dev)
    ws = torch.empty(max(batch.workspace_bytes(w.n), 256), dtype=torch.uint8, device=dev)
    seal = timed(lambda: batch.seal(kt, arena, sd, st, hint, ws))
    batch.seal(kt, arena, sd, st, hint, ws)
    opn = timed(lambda: (batch.open_(kt, arena, od, st, pn, hint, ws), batch.seal(kt, arena, sd, st, hint, ws)))
    seal_only = seal
    torch.cuda.synchronize()
    return {"seal_ms": seal_only, "open_plus_seal_ms": opn, "failures": int((st != 0).sum())}


def main():
    n = 1 << 20
    assert _lib.load().mq_device_init(0) == 0
    w = workload.config_c(n)
    ident = np.arange(n)
    stride = (ident % 1024) * 1024 + ident // 1024  # tile t: packets 1024 apart
    out = {"in_order": run(w, ident, w.suite_hint), "stride_1024": run(w, stride, w.suite_hint)}
    wk = workload.config_c(n, n_keys=1024)
    out["keys_1024_partition"] = run(wk, ident, wk.suite_hint)
    wb = workload.config_b(n)
    out["chacha_in_order"] = run(wb, ident, wb.suite_hint)
    out["chacha_stride_1024"] = run(wb, stride, wb.suite_hint)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
