"""Why config E's Initial packets cost more per packet than its 1-RTT AES packets (diagnostic).
Subsets of config E's 2^20-packet batch, all on ONE AES-128-GCM key (a one-row key table, the
hot 1-RTT key; flat AES hint: the single-key kernel alone, no partition), seal and open medians:
  initial      the Initial packets (long header, AAD 27-30 B, LONG_HEADER flag)
  initial-nf   the same packets with MQ_PKT_LONG_HEADER cleared (only the HP first-byte mask differs)
  1rtt         1-RTT AES packets, as many as the Initial ones
  1rtt-sorted  the same, descriptors sorted by length (as the partition's 64-B classes group them)
  initial-sorted  the Initial packets sorted by length
Usage: python tools/initial_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timeit(torch, batch, kt, arena_np, sd_np, od_np, hint, reps=10):
    import numpy as np
    dev = torch.device("cuda", 0)
    n = len(sd_np)
    a0 = torch.from_numpy(arena_np).to(dev)
    a = a0.clone()
    sd = torch.from_numpy(np.ascontiguousarray(sd_np).view(np.uint8)).to(dev)
    od = torch.from_numpy(np.ascontiguousarray(od_np).view(np.uint8)).to(dev)
    st = torch.zeros(n, dtype=torch.uint8, device=dev)
    pn = torch.zeros(n, dtype=torch.int64, device=dev)
    ws = torch.empty(max(batch.workspace_bytes(n), 256), dtype=torch.uint8, device=dev)
    res = {"seal": [], "open": []}
    for rep in range(reps + 2):
        a.copy_(a0)
        for which in ("seal", "open"):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if which == "seal":
                batch.seal(kt, a, sd, st, hint, ws)
            else:
                batch.open_(kt, a, od, st, pn, hint, ws)
            e1.record()
            torch.cuda.synchronize()
            assert int((st != 0).sum()) == 0, which
            if rep >= 2:
                res[which].append(e0.elapsed_time(e1))
    return float(np.median(res["seal"])), float(np.median(res["open"]))


def main():
    import numpy as np
    import torch
    from milli_quic_amd import _lib, batch, workload
    assert _lib.load().mq_device_init(0) == 0
    w = workload.config_e(1 << 20)
    kt = batch.KeyTable([w.keys[1]])  # the hot 1-RTT AES key as the only row
    kid = w.seal_desc["key_id"]
    ini = np.nonzero(kid >= 2)[0]
    one = np.nonzero(kid == 1)[0][: len(ini)]
    hint = _lib.MQ_SUITE_AES128GCM
    for name, sel, clear in (("initial", ini, False), ("initial-nf", ini, True), ("1rtt", one, False),
                             ("initial-sorted", ini[np.argsort(w.seal_desc["len"][ini], kind="stable")], False),
                             ("1rtt-sorted", one[np.argsort(w.seal_desc["len"][one], kind="stable")], False)):
        sd, od = w.seal_desc[sel].copy(), w.open_desc[sel].copy()
        sd["key_id"] = 0
        od["key_id"] = 0
        if clear:
            sd["flags"] &= ~np.uint8(_lib.MQ_PKT_LONG_HEADER)
            od["flags"] &= ~np.uint8(_lib.MQ_PKT_LONG_HEADER)
        s, o = timeit(torch, batch, kt, w.arena, sd, od, hint)
        wire = int(sd["len"].astype(np.int64).sum())
        print(f"{name:15s} packets {len(sel):7d} avg {wire / len(sel):6.1f} B  seal {s:.4f} open {o:.4f} ms  "
              f"{(s + o) * 1e6 / len(sel):.3f} ns/pkt  {2 * wire / ((s + o) * 1e-3) / 2 ** 30:6.1f} GiB/s", flush=True)


if __name__ == "__main__":
    main()
