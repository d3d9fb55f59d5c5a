"""Config-E cost split (diagnostic): seal / open medians of the whole mixed batch and of its parts
run on their own (E_NOCHECK=1: no status check, for MQ_LIB phase-cost variants) — the ChaCha20 packets, the hot 1-RTT AES key's packets, the Initial packets on
their 4096 per-connection keys, and the Initial packets moved onto the hot row (what the
per-connection keys cost). Every part goes through the same call the batch makes (mixed hint, the
device partition). MQ_* environment switches apply to every line (e.g. MQ_FORK=0).
Usage: python tools/e_parts.py [packets]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timeit(torch, batch, kt, w, sd_np, od_np, hint, reps=8):
    import numpy as np
    dev = torch.device("cuda", 0)
    n = len(sd_np)
    arena0 = torch.from_numpy(w.arena).to(dev)
    arena = arena0.clone()
    sd = torch.from_numpy(np.ascontiguousarray(sd_np).view(np.uint8)).to(dev)
    od = torch.from_numpy(np.ascontiguousarray(od_np).view(np.uint8)).to(dev)
    st = torch.zeros(n, dtype=torch.uint8, device=dev)
    pn = torch.zeros(n, dtype=torch.int64, device=dev)
    ws = torch.empty(max(batch.workspace_bytes(n), 256), dtype=torch.uint8, device=dev)
    res = {"seal": [], "open": []}
    for rep in range(reps + 2):
        arena.copy_(arena0)
        for which in ("seal", "open"):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if which == "seal":
                batch.seal(kt, arena, sd, st, hint, ws)
            else:
                batch.open_(kt, arena, od, st, pn, hint, ws)
            e1.record()
            torch.cuda.synchronize()
            bad = int((st != 0).sum())
            if bad and not os.environ.get("E_NOCHECK"):  # phase-cost variants (MQ_LIB) compute garbage
                raise SystemExit(f"{which}: {bad} packets failed")
            if rep >= 2:
                res[which].append(e0.elapsed_time(e1))
    return float(np.median(res["seal"])), float(np.median(res["open"]))


def run(n):
    import numpy as np
    import torch
    from milli_quic_amd import _lib, batch, workload
    assert _lib.load().mq_device_init(0) == 0
    w = workload.config_e(n)
    kt = batch.KeyTable(w.keys)
    kid = w.seal_desc["key_id"]
    parts = {
        "whole batch": np.ones(w.n, bool),
        "ChaCha20 1-RTT": kid == 0,
        "AES hot 1-RTT": kid == 1,
        "AES Initial (4096 keys)": kid >= 2,
        "AES (hot + Initial)": kid >= 1,
    }
    for name, m in parts.items():
        sd, od = w.seal_desc[m].copy(), w.open_desc[m].copy()
        s, o = timeit(torch, batch, kt, w, sd, od, _lib.MQ_SUITE_MIXED)
        wire = int(sd["len"].astype(np.int64).sum())
        print(f"{name:26s} packets {int(m.sum()):8d} seal {s:.4f} open {o:.4f} ms  "
              f"{2 * wire / ((s + o) * 1e-3) / 2 ** 30:7.1f} GiB/s  {(s + o) * 1e6 / max(int(m.sum()), 1):.3f} ns/pkt",
              flush=True)
    m = kid >= 2
    sd, od = w.seal_desc[m].copy(), w.open_desc[m].copy()
    sd["key_id"] = 1
    od["key_id"] = 1
    s, o = timeit(torch, batch, kt, w, sd, od, _lib.MQ_SUITE_MIXED)
    print(f"{'AES Initial on hot row':26s} packets {int(m.sum()):8d} seal {s:.4f} open {o:.4f} ms  "
          f"{(s + o) * 1e6 / int(m.sum()):.3f} ns/pkt", flush=True)


if __name__ == "__main__":
    run(int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20)
