"""What a second AAD block costs (diagnostic): single-key flat batches of n x L-byte short-header
packets whose DCID is 8 bytes (AAD 13 B: one GHASH / Poly1305 AAD block) or 20 bytes (AAD 25 B:
two blocks — the AES tiles then run an extra wave iteration, slot -1, for one block per packet),
both suites, seal and open medians (HIP events, 8 reps). Usage: python tools/aad_probe.py [n]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from milli_quic_amd import _lib, batch, workload
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    assert _lib.load().mq_device_init(0) == 0
    dev = torch.device("cuda", 0)
    for suite, name in ((_lib.MQ_SUITE_AES128GCM, "AES"), (_lib.MQ_SUITE_CHACHA20, "ChaCha")):
        for L in (300, 700, 1200):
            row = []
            for dl in (8, 20):
                w = workload.uniform(n, suite, L=L, dcid=bytes(range(1, dl + 1)))
                kt = batch.KeyTable(w.keys)
                a0 = torch.from_numpy(w.arena).to(dev)
                a = a0.clone()
                sd = torch.from_numpy(w.seal_desc.view(np.uint8)).to(dev)
                od = torch.from_numpy(w.open_desc.view(np.uint8)).to(dev)
                st = torch.zeros(n, dtype=torch.uint8, device=dev)
                pn = torch.zeros(n, dtype=torch.int64, device=dev)
                ws = torch.empty(batch.workspace_bytes(n), dtype=torch.uint8, device=dev)
                res = {"seal": [], "open": []}
                for rep in range(10):
                    a.copy_(a0)
                    for which in ("seal", "open"):
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        if which == "seal":
                            batch.seal(kt, a, sd, st, w.suite_hint, ws)
                        else:
                            batch.open_(kt, a, od, st, pn, w.suite_hint, ws)
                        e1.record()
                        torch.cuda.synchronize()
                        assert int((st != 0).sum()) == 0, (name, L, dl, which)
                        if rep >= 2:
                            res[which].append(e0.elapsed_time(e1))
                s, o = float(np.median(res["seal"])), float(np.median(res["open"]))
                row.append((s, o))
                print(f"{name:6s} L={L:5d} dcid={dl:2d} (AAD {1 + dl + 4} B) seal {s:.4f} open {o:.4f} ms  "
                      f"{2 * w.wire_bytes / ((s + o) * 1e-3) / 2 ** 30:7.1f} GiB/s", flush=True)
                del a, a0, ws
            print(f"{name:6s} L={L:5d} two AAD blocks / one: seal x{row[1][0] / row[0][0]:.3f} open x{row[1][1] / row[0][1]:.3f}",
                  flush=True)


if __name__ == "__main__":
    main()
