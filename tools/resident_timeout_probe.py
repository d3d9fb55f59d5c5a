"""Diagnostic: the resident per-packet server's timeout path, step by step with timestamps (every
line flushed, so a hang shows where it stopped). A config-C batch holds every CU while a
per-packet call with a 100-us limit relaunches the idle server.
Usage: python tools/resident_timeout_probe.py [packets]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from milli_quic_amd import _lib, batch, crypto, workload  # noqa: E402
from milli_quic_amd.batch import KeyTable  # noqa: E402

T0 = time.perf_counter()


def log(*a):
    print(f"{time.perf_counter() - T0:8.3f}", *a, flush=True)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    null = "--null" in sys.argv  # the batch on the null stream, device-wide syncs (as the pytest does)
    lib = _lib.load()
    assert lib.mq_device_init(0) == 0
    dev = torch.device("cuda", 0)
    w = workload.config_c(n)
    kt = KeyTable(w.keys)
    arena = torch.from_numpy(w.arena.copy()).to(dev)
    sd = torch.from_numpy(w.seal_desc.view(np.uint8).copy()).to(dev)
    od = torch.from_numpy(w.open_desc.view(np.uint8).copy()).to(dev)
    st = torch.zeros(w.n, dtype=torch.uint8, device=dev)
    pn = torch.zeros(w.n, dtype=torch.int64, device=dev)
    ws = torch.empty(max(batch.workspace_bytes(w.n), 256), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream() if null else torch.cuda.Stream()
    sync = torch.cuda.synchronize if null else s.synchronize
    aead = crypto.ChaCha20Provider().aead(bytes(range(32)))
    buf = bytearray(100) + bytearray(16)
    aead.seal_in_place(bytes(12), b"h", buf, 100)
    log("warm call ok")
    for k in range(3):
        log(k, "sync")
        sync()
        time.sleep(0.05)
        log(k, "enqueue batch")
        with torch.cuda.stream(s):
            for _ in range(6):
                batch.seal(kt, arena, sd, st, w.suite_hint, ws, s.cuda_stream)
                batch.open_(kt, arena, od, st, pn, w.suite_hint, ws, s.cuda_stream)
        _lib.load().mq_debug_option(b"MQ_RESIDENT_TIMEOUT_US", 100)
        log(k, "call with a 100-us limit")
        buf = bytearray(100) + bytearray(16)
        try:
            aead.seal_in_place(bytes([k]) * 12, b"h", buf, 100)
            log(k, "served")
        except crypto.DeviceError as e:
            log(k, "timeout:", e)
        _lib.load().mq_debug_option(b"MQ_RESIDENT_TIMEOUT_US", -1)
        for q in range(3):
            buf = bytearray(100) + bytearray(16)
            aead.seal_in_place(bytes([k, q]) * 6, b"h", buf, 100)
            log(k, "next call", q, "ok")
        log(k, "sync")
        sync()
        log(k, "synced")
    log("device sync")
    torch.cuda.synchronize()
    log("done", int((st != 0).sum()))


if __name__ == "__main__":
    main()
