"""Seal + open rate of flat single-key batches over packet lengths (both suites): finds length
cliffs (e.g. the ChaCha tile's 10-KiB LDS image: eight packets of more than ~1232 B take the direct
path). ~1.2 GB of packets per batch. Packets over the receive composite's 2048-B limit
(recv.rs:356-360) are opened with MQ_PKT_NO_RECV_LIMIT, else open answers BUFFER_TOO_SMALL by design
(the r04zg sweep's AssertionError: its L after 2048 was over the limit, and the flag was not set).
A failed packet is reported, never skipped. MQ_SWEEP_HINT=mixed runs the batches with the mixed
hint (device partition) instead of the single-suite hint.
Usage: python tools/len_sweep.py [c|a|both] [L ...]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from milli_quic_amd import _lib, batch, workload  # noqa: E402


def rate(suite, L, reps=6):
    n = int(min(1 << 22, (1200 << 20) // L))
    w = workload.uniform(n, suite, L=L)
    if L > _lib.MQ_RECV_MAX_PACKET:
        w.open_desc["flags"] |= _lib.MQ_PKT_NO_RECV_LIMIT
    hint = _lib.MQ_SUITE_MIXED if os.environ.get("MQ_SWEEP_HINT") == "mixed" else suite
    dev = torch.device("cuda", 0)
    kt = batch.KeyTable(w.keys)
    arena0 = torch.from_numpy(w.arena).to(dev)
    arena = arena0.clone()
    sd = torch.from_numpy(w.seal_desc.view(np.uint8)).to(dev)
    od = torch.from_numpy(w.open_desc.view(np.uint8)).to(dev)
    st = torch.zeros(n, dtype=torch.uint8, device=dev)
    st2 = torch.zeros(n, dtype=torch.uint8, device=dev)
    pn = torch.zeros(n, dtype=torch.int64, device=dev)
    ws = torch.empty(max(batch.workspace_bytes(n), 256), dtype=torch.uint8, device=dev)
    ts, to = [], []
    for rep in range(reps):
        arena.copy_(arena0)
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record()
        batch.seal(kt, arena, sd, st, hint, ws)
        e[1].record()
        batch.open_(kt, arena, od, st2, pn, hint, ws)
        e[2].record()
        torch.cuda.synchronize()
        bad = int((st != 0).sum()) + int((st2 != 0).sum())
        if bad:
            codes = sorted(set(st.cpu().numpy().tolist()) | set(st2.cpu().numpy().tolist()))
            raise SystemExit(f"L {L}: {bad} packets failed (statuses {codes})")
        if rep >= 2:
            ts.append(e[0].elapsed_time(e[1]))
            to.append(e[1].elapsed_time(e[2]))
    s, o = float(np.median(ts)), float(np.median(to))
    return n, s, o, 2 * n * L / ((s + o) * 1e-3) / 2 ** 30


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "both"
    Ls = [int(x) for x in sys.argv[2:]] or [64, 256, 700, 1200, 1232, 1280, 1350, 1452, 1500, 1584, 1600, 2048]
    assert _lib.load().mq_device_init(0) == 0
    suites = {"c": [_lib.MQ_SUITE_CHACHA20], "a": [_lib.MQ_SUITE_AES128GCM]}.get(
        which, [_lib.MQ_SUITE_CHACHA20, _lib.MQ_SUITE_AES128GCM])
    for suite in suites:
        for L in Ls:
            n, s, o, g = rate(suite, L)
            name = "chacha" if suite == _lib.MQ_SUITE_CHACHA20 else "aes"
            print(f"{name} L {L} n {n} seal {s:.4f} open {o:.4f} ms  {g:.1f} GiB/s", flush=True)


if __name__ == "__main__":
    main()
