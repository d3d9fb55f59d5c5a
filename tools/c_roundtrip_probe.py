"""Diagnostic: config C (2^20 x 1200 B AES-128-GCM, one key, flat batch) seal + open round trips
with a given library; reports every byte that does not come back, and whether two seals of the
same input agree. Usage: python tools/c_roundtrip_probe.py LIB [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from milli_quic_amd import _lib
    _lib.LIB_PATH = sys.argv[1]
    from milli_quic_amd import batch, workload
    assert _lib.load().mq_device_init(0) == 0
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    w = workload.config_c(1 << 20)
    dev = torch.device("cuda", 0)
    kt = batch.KeyTable(w.keys)
    a0 = torch.from_numpy(w.arena).to(dev)
    sd = torch.from_numpy(w.seal_desc.view(np.uint8)).to(dev)
    od = torch.from_numpy(w.open_desc.view(np.uint8)).to(dev)
    st = torch.zeros(w.n, dtype=torch.uint8, device=dev)
    pn = torch.zeros(w.n, dtype=torch.int64, device=dev)
    ref = w.arena.reshape(w.n, 1200)[:, :1184]
    first = None
    for r in range(reps):
        a = a0.clone()
        batch.seal(kt, a, sd, st, w.suite_hint)
        torch.cuda.synchronize()
        sealed = a.cpu().numpy()
        s_bad = int((st != 0).sum())
        if first is None:
            first = sealed
        same = (sealed == first)
        batch.open_(kt, a, od, st, pn, w.suite_hint)
        torch.cuda.synchronize()
        o_bad = int((st != 0).sum())
        back = a.cpu().numpy().reshape(w.n, 1200)[:, :1184]
        diff = np.nonzero((back != ref).reshape(-1))[0]
        nd = np.nonzero(~same)[0]
        print(f"rep {r}: seal status!=0 {s_bad}, open status!=0 {o_bad}, round-trip byte diffs {len(diff)}, "
              f"sealed bytes differing from rep 0: {len(nd)}", flush=True)
        for x in diff[:12]:
            p, o = divmod(int(x), 1184)
            print(f"   packet {p} byte {o}: got {back.reshape(-1)[x]:#04x} want {ref.reshape(-1)[x]:#04x}")
        for x in nd[:12]:
            p, o = divmod(int(x), 1200)
            print(f"   sealed packet {p} byte {o}: {sealed[x]:#04x} vs {first[x]:#04x}")


if __name__ == "__main__":
    main()
