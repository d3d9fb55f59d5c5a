"""Phase costs under full load from the MQ_PROF_SKIP diagnostic builds (make prof-variants).

Times seal and open of one workload with the product library and with each variant that skips
one phase (1 ChaCha rounds, 2 MAC, 4 LDS->HBM store, 8 HBM->LDS staging, 16 AES rounds, 12 both
copies, 32 every tile on the direct path; 128: the ChaCha keystream XOR with a conflict-free
68-B block stride); the difference is what that phase costs.
MQ_PROF_DIR names the variants' directory (default milli_quic_amd/prof, which gpurun does not ship:
copy them under tools/ab_libs/ for a GPU run). Diagnostic only: variants compute garbage.
Usage: python tools/phase_cost.py [b|c|e|bk|ck] [packets]   (bk, ck: 1024 key rows)
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.environ.get("MQ_PROF_DIR", os.path.join(ROOT, "milli_quic_amd", "prof"))


def child(lib, cfg, n):
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch
    from milli_quic_amd import _lib
    _lib.LIB_PATH = lib
    from milli_quic_amd import batch, workload
    assert _lib.load().mq_device_init(0) == 0
    w = {"b": workload.config_b, "c": workload.config_c, "e": workload.config_e,
         "bk": lambda m: workload.config_b(m, n_keys=1024), "ck": lambda m: workload.config_c(m, n_keys=1024)}[cfg](n)
    dev = torch.device("cuda", 0)
    kt = batch.KeyTable(w.keys)
    arena0 = torch.from_numpy(w.arena).to(dev)
    arena = arena0.clone()
    sd = torch.from_numpy(w.seal_desc.view(np.uint8)).to(dev)
    od = torch.from_numpy(w.open_desc.view(np.uint8)).to(dev)
    st = torch.zeros(w.n, dtype=torch.uint8, device=dev)
    pn = torch.zeros(w.n, dtype=torch.int64, device=dev)
    ws = torch.empty(max(batch.workspace_bytes(w.n), 256), dtype=torch.uint8, device=dev)
    res = {"seal": [], "open": []}
    for rep in range(8):
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
            if rep >= 2:
                res[which].append(e0.elapsed_time(e1))
    print(f"RESULT {np.median(res['seal']):.4f} {np.median(res['open']):.4f}")


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        return child(sys.argv[2], sys.argv[3], int(sys.argv[4]))
    cfg = sys.argv[1] if len(sys.argv) > 1 else "b"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
    libs = [("product", os.path.join(ROOT, "milli_quic_amd", "libmq_aead.so"))]
    names = {1: "no chacha rounds", 2: "no MAC", 4: "no store", 8: "no staging", 16: "no AES rounds",
             12: "no store+staging", 32: "all direct", 64: "no AES final mul", 128: "ks stride 68 (ChaCha) / no AES header mask"}
    for m, nm in names.items():
        p = os.path.join(BUILD, f"prof_{m}.so")
        if os.path.exists(p):
            libs.append((nm, p))
    base = None
    for nm, lib in libs:
        out = subprocess.run([sys.executable, __file__, "--child", lib, cfg, str(n)], capture_output=True,
                             text=True, timeout=240)
        line = [x for x in out.stdout.splitlines() if x.startswith("RESULT")]
        if not line:
            print(nm, "FAILED", out.stderr[-500:])
            continue
        s, o = map(float, line[0].split()[1:])
        if base is None:
            base = (s, o)
        print(f"{nm:18s} seal {s:.4f} ms ({s - base[0]:+.4f})  open {o:.4f} ms ({o - base[1]:+.4f})", flush=True)


if __name__ == "__main__":
    main()
