#!/usr/bin/env python3
"""Per-packet latency of the drop-in trait path: microseconds per call
of mq_aead_seal_in_place / mq_aead_open_in_place / mq_hp_mask on one 1200-B packet (13-B AAD,
1171-B payload), called through ctypes exactly as the reference calls Aead / HeaderProtection
once per packet (transmit.rs:713-719, recv.rs:416-421). Modes:
  resident   (default since r03) the device's resident wave serves the call from a mailbox in
             pinned host memory: no kernel launch (mq_resident.hip);
  zero_copy  (MQ_RESIDENT=0) a batch of one: one kernel launch on a pinned scratch mapped into the
             device, then a stream sync;
  copy       (MQ_RESIDENT=0 MQ_PER_PACKET_COPY=1) the same with H2D / D2H copies around it.
Prints one JSON line (median and p99 over `--calls` calls, after warm-up), both suites, all modes.
The batch API is the throughput path."""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=3000)
    args = ap.parse_args()
    from milli_quic_amd import _lib
    lib = _lib.load()
    assert lib.mq_device_init(0) == 0
    out = {"unit": "us per call", "packet": "1200 B (13 B AAD, 1171 B payload, 16 B tag)", "calls": args.calls}
    for mode in ("resident", "zero_copy", "copy"):
        lib.mq_debug_option(b"MQ_RESIDENT", 1 if mode == "resident" else 0)
        os.environ["MQ_PER_PACKET_COPY"] = "1" if mode == "copy" else "0"
        out[mode] = measure(lib, _lib, args.calls)
    lib.mq_debug_option(b"MQ_RESIDENT", -1)
    out["resident_throughput"] = throughput(lib, _lib)
    print(json.dumps(out), flush=True)


def throughput(lib, _lib, seconds=0.5):
    """Per-packet seal calls per second from T host threads at once (resident mode): each thread its
    own ChaCha20 context and 1200-B packet; ctypes drops the GIL during the call, so the calls meet
    in the library (r05: one server lane per thread up to MQ_RESIDENT_LANES)."""
    import threading
    res = {}
    for T in (1, 2, 4, 8):
        counts = [0] * T
        stop = threading.Event()

        def work(t):
            ctx = ctypes.c_void_p()
            assert lib.mq_aead_new(_lib.MQ_SUITE_CHACHA20, bytes(range(32)), 32, ctypes.byref(ctx)) == 0
            nonce = (ctypes.c_uint8 * 12)(*range(12))
            aad = (ctypes.c_uint8 * 13)(*range(13))
            buf = (ctypes.c_uint8 * 1200)()
            ol, nd = ctypes.c_size_t(), ctypes.c_size_t()
            while not stop.is_set():
                assert lib.mq_aead_seal_in_place(ctx, nonce, 12, aad, 13, buf, 1200, 1171, ctypes.byref(ol),
                                                 ctypes.byref(nd)) == 0
                counts[t] += 1
            lib.mq_aead_free(ctx)
        th = [threading.Thread(target=work, args=(t,)) for t in range(T)]
        for x in th:
            x.start()
        time.sleep(0.1)  # every lane's server up
        c0 = sum(counts)
        t0 = time.perf_counter()
        time.sleep(seconds)
        c1 = sum(counts)
        t1 = time.perf_counter()
        stop.set()
        for x in th:
            x.join()
        res[f"threads_{T}"] = round((c1 - c0) / (t1 - t0))
    res["unit"] = "seal calls per second (ChaCha20-Poly1305, 1200 B), all threads"
    return res


def measure(lib, _lib, calls):
    out = {}
    for suite, klen in ((_lib.MQ_SUITE_CHACHA20, 32), (_lib.MQ_SUITE_AES128GCM, 16)):
        ctx, hp = ctypes.c_void_p(), ctypes.c_void_p()
        assert lib.mq_aead_new(suite, bytes(range(klen)), klen, ctypes.byref(ctx)) == 0
        assert lib.mq_hp_new(suite, bytes(range(klen)), klen, ctypes.byref(hp)) == 0
        nonce = (ctypes.c_uint8 * 12)(*range(12))
        aad = (ctypes.c_uint8 * 13)(*range(13))
        buf = (ctypes.c_uint8 * 1200)()
        sample = (ctypes.c_uint8 * 16)(*range(16))
        mask = (ctypes.c_uint8 * 5)()
        ol, nd = ctypes.c_size_t(), ctypes.c_size_t()
        P = 1171

        def seal():
            return lib.mq_aead_seal_in_place(ctx, nonce, 12, aad, 13, buf, 1200, P, ctypes.byref(ol), ctypes.byref(nd))

        def open_():
            return lib.mq_aead_open_in_place(ctx, nonce, 12, aad, 13, buf, 1200, P + 16, ctypes.byref(ol))

        def pair():
            assert seal() == 0
            assert open_() == 0

        def hpm():
            return lib.mq_hp_mask(hp, sample, 16, mask)

        res = {}
        for name, fn in (("seal_open_pair", pair), ("hp_mask", hpm)):
            for _ in range(200):
                fn()
            t = np.empty(calls)
            for k in range(calls):
                t0 = time.perf_counter()
                fn()
                t[k] = time.perf_counter() - t0
            res[name] = {"median": round(float(np.median(t)) * 1e6, 2), "p99": round(float(np.quantile(t, 0.99)) * 1e6, 2)}
        # seal and open separately (open needs a sealed buffer: reseal before each timed open)
        ts, to = np.empty(calls), np.empty(calls)
        ph = (ctypes.c_uint32 * 9)()
        phs, pho = np.zeros((calls, 9)), np.zeros((calls, 9))
        for k in range(calls):
            t0 = time.perf_counter()
            assert seal() == 0
            t1 = time.perf_counter()
            if lib.mq_resident_phases(0, ph, 9) == 9:  # outside the timed calls
                phs[k] = list(ph)
            t1b = time.perf_counter()
            assert open_() == 0
            t2 = time.perf_counter()
            if lib.mq_resident_phases(0, ph, 9) == 9:
                pho[k] = list(ph)
            ts[k], to[k] = t1 - t0, t2 - t1b
        res["seal"] = {"median": round(float(np.median(ts)) * 1e6, 2), "p99": round(float(np.quantile(ts, 0.99)) * 1e6, 2)}
        res["open"] = {"median": round(float(np.median(to)) * 1e6, 2), "p99": round(float(np.quantile(to, 0.99)) * 1e6, 2)}
        if lib.mq_debug_option_get(b"MQ_RESIDENT") == 1:  # device-side phases (mq_resident_phases), median us
            names = ("header_broadcast", "first_half", "packet_wait", "second_half", "decrypt_applied", "written_back",
                     "host_request_written", "host_wait_done", "host_copy_out")
            res["phases_us"] = {
                op: {n: round(float(np.median(a[:, i])) / 1e3, 2) for i, n in enumerate(names)}
                for op, a in (("seal", phs), ("open", pho))}
        # ctypes call overhead alone (a call that returns at the argument checks)
        t = np.empty(calls)
        for k in range(calls):
            t0 = time.perf_counter()
            lib.mq_aead_seal_in_place(ctx, nonce, 11, aad, 13, buf, 1200, P, ctypes.byref(ol), ctypes.byref(nd))
            t[k] = time.perf_counter() - t0
        res["ctypes_overhead_median"] = round(float(np.median(t)) * 1e6, 3)
        out["chacha20" if suite == _lib.MQ_SUITE_CHACHA20 else "aes128gcm"] = res
        lib.mq_aead_free(ctx)
        lib.mq_hp_free(hp)
    return out


if __name__ == "__main__":
    main()
