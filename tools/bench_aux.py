"""Throughput of the SURVEY §8f components on one MI355X (device-resident, HIP events on the launch
stream; median of `reps`). Prints one JSON object; the round's copy lives in profiles/.

  derive   mq_batch_derive_initial: 2^20 client DCIDs (8 B) -> 2^21 key-table rows
  protect  mq_batch_protect: 2^20 x 1171-B frames -> 1200-B 1-RTT packets (ChaCha20, 4096 keys)
  recv     mq_batch_recv: the same 2^20 packets as one-packet datagrams of 4096 connections (and of
           1024, 64, 4, 1 connections); a 4096-datagram sample byte-checked against the oracle
  records  mq_batch_seal_records / open_records: 2^20 x 1200-B and 2^16 x 16 KiB TLS records
           (AES-128-GCM)
  hp_mask  mq_batch_hp_mask (SURVEY §8d "mask-only timing"): 2^20 16-B samples -> 5-B masks,
           AES-128 (config C keys) and ChaCha20 (config B keys)
Usage: python tools/bench_aux.py [reps]
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from milli_quic_amd import _lib, batch, recv, send, tls_record, workload  # noqa: E402
from milli_quic_amd.batch import KeyTable  # noqa: E402

DEV = torch.device("cuda", 0)


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).to(DEV)


def timed(fn, reps):
    out = []
    for _ in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1))
    return float(np.median(out[1:]))


def bench_derive(reps, n=1 << 20):
    kt = KeyTable([_lib.KeyMaterial() for _ in range(2 * n)])
    dc = t(workload.splitmix_bytes(20 * n, seed=9))
    ln = torch.full((n,), 8, dtype=torch.uint8, device=DEV)
    st = torch.zeros(n, dtype=torch.uint8, device=DEV)
    ms = timed(lambda: batch.derive_initial(kt, 0, dc, ln, st), reps)
    assert int((st != 0).sum()) == 0
    return {"connections": n, "ms": round(ms, 4), "connections_per_s": round(n / ms * 1e3)}


def bench_protect_recv(reps, n=1 << 20, n_conns=4096, only="both"):
    fl = 1171
    w = workload.uniform(64, _lib.MQ_SUITE_CHACHA20, n_keys=n_conns)
    kt = KeyTable(w.keys)
    conns = send.make_conns([workload.DCID8] * n_conns, [b""] * n_conns, [[k, k, k] for k in range(n_conns)])
    req = np.zeros(n, dtype=send.REQ_DTYPE)
    i = np.arange(n, dtype=np.uint64)
    req["frames_offset"], req["out_offset"] = i * np.uint64(fl), i * np.uint64(1200)
    req["pn"] = np.uint64(0x10000000) + i // np.uint64(n_conns)
    req["largest_acked"] = req["pn"] - np.uint64(1 << 24)
    req["frame_len"], req["out_cap"], req["level"] = fl, 1200, send.APPLICATION
    req["conn"] = (i % np.uint64(n_conns)).astype(np.uint32)
    frames = t(workload.splitmix_bytes(n * fl, seed=3))
    out = torch.zeros(n * 1200, dtype=torch.uint8, device=DEV)
    dc, dr = t(conns), t(req)
    st = torch.zeros(n, dtype=torch.uint8, device=DEV)
    ln = torch.zeros(n, dtype=torch.int32, device=DEV)
    ws = torch.empty(send.workspace_bytes(n), dtype=torch.uint8, device=DEV)
    ms_p = timed(lambda: send.protect(kt, dc, frames, out, dr, st, ln, _lib.MQ_SUITE_CHACHA20, ws),
                 reps if only != "recv" else 0)
    assert int((st != 0).sum()) == 0
    if only == "protect":
        return ({"ms": round(ms_p, 4)}, None)
    sealed = out.clone()
    rc = np.zeros(n_conns, dtype=recv.CONN_DTYPE)
    rc["app_row"][:, 1] = np.arange(n_conns)
    rc["dcid_len"], rc["flags"] = 8, recv.HAS_APP
    dg = np.zeros(n, dtype=recv.DGRAM_DTYPE)
    dg["offset"], dg["len"], dg["conn"] = i * np.uint64(1200), 1200, req["conn"]
    dgt = t(dg)
    pk = torch.zeros(n * 32, dtype=torch.uint8, device=DEV)
    cnt = torch.zeros(1, dtype=torch.int32, device=DEV)
    rws = torch.empty(recv.workspace_bytes(n, n, n_conns), dtype=torch.uint8, device=DEV)
    ct0 = t(rc)
    ct = ct0.clone()

    def one_recv():
        out.copy_(sealed)
        ct.copy_(ct0)
        recv.recv(kt, ct, out, dgt, pk, cnt, rws)
    copy_ms = timed(lambda: (out.copy_(sealed), ct.copy_(ct0)), reps)
    ms_r = timed(one_recv, reps) - copy_ms
    got = pk.cpu().numpy().view(recv.PKT_DTYPE)
    assert int(cnt[0]) == n and (got["status"] == 0).all()
    checked = sample_check(kt_rows=w.keys, rc=rc, sealed=sealed, opened=out, got=got, dg=dg)
    wire = n * 1200
    return ({"packets": n, "connections": n_conns, "ms": round(ms_p, 4),
             "GiB_per_s_wire": round(wire / ms_p * 1e3 / 2 ** 30, 1)},
            {"packets": n, "connections": n_conns, "ms": round(ms_r, 4),
             "GiB_per_s_wire": round(wire / ms_r * 1e3 / 2 ** 30, 1), "sample_checked": checked})


def sample_check(kt_rows, rc, sealed, opened, got, dg, k=4096, seed=12):
    """Byte check of a sample of the receive run: the oracle's receive composite
    (the checker) on k sampled datagrams, from the sealed bytes, must give the same records and
    the same opened bytes as the GPU's full run. The PNs are 4-byte encoded, so a sampled packet
    decodes the same without its connection's earlier packets."""
    from oracle import oracle
    oracle.load()
    rng = np.random.default_rng(seed)
    n = len(dg)
    idx = np.sort(rng.choice(n, size=min(k, n), replace=False))
    sd = dg[idx].copy()
    L = int(dg["len"][0])
    arena = np.zeros(len(idx) * L, dtype=np.uint8)
    sealed_np = sealed.cpu().numpy()
    opened_np = opened.cpu().numpy()
    for j, g in enumerate(idx):
        o = int(dg["offset"][g])
        arena[j * L:(j + 1) * L] = sealed_np[o:o + L]
    sd["offset"] = np.arange(len(idx), dtype=np.uint64) * np.uint64(L)
    o_pk, o_n = oracle.batch_recv(kt_rows, rc.copy(), arena, sd, len(idx), threads=16)
    assert o_n == len(idx) and (o_pk["status"] == 0).all(), "oracle sample failed"
    gp = got[idx]  # one packet per datagram: record index = datagram index
    assert (gp["pn"] == o_pk["pn"]).all() and (gp["status"] == o_pk["status"]).all()
    for j, g in enumerate(idx):
        o = int(dg["offset"][g])
        assert opened_np[o:o + L].tobytes() == arena[j * L:(j + 1) * L].tobytes(), f"datagram {g} differs"
    return len(idx)


def bench_records(reps, n, L):
    km = workload.key_material(_lib.MQ_SUITE_AES128GCM, workload.A1_SERVER_SECRET)
    kt = KeyTable([km])
    i = np.arange(n, dtype=np.uint64)
    a = t(workload.splitmix_bytes(n * L, seed=4))
    sd = t(tls_record.record_descs(i * np.uint64(L), L, 0, i, 23))
    od = t(tls_record.record_descs(i * np.uint64(L), L, 0, i))
    st = torch.zeros(n, dtype=torch.uint8, device=DEV)
    info = torch.zeros(n, dtype=torch.int64, device=DEV)
    ws = torch.empty(max(batch.workspace_bytes(n), 256), dtype=torch.uint8, device=DEV)
    ms_s = timed(lambda: batch.seal_records(kt, a, sd, st, _lib.MQ_SUITE_AES128GCM, ws), reps)
    assert int((st != 0).sum()) == 0
    ms_o = timed(lambda: (batch.seal_records(kt, a, sd, st, _lib.MQ_SUITE_AES128GCM, ws),
                          batch.open_records(kt, a, od, st, info, _lib.MQ_SUITE_AES128GCM, ws)), reps) - ms_s
    assert int((st != 0).sum()) == 0
    wire = n * L
    return {"records": n, "record_bytes": L, "seal_ms": round(ms_s, 4), "open_ms": round(ms_o, 4),
            "GiB_per_s_seal_open": round(2 * wire / (ms_s + ms_o) * 1e3 / 2 ** 30, 1)}


def bench_hp_mask(reps, suite, n=1 << 20):
    secret = workload.A1_SERVER_SECRET if suite == _lib.MQ_SUITE_AES128GCM else workload.A5_SECRET
    km = workload.key_material(suite, secret)
    kt = KeyTable([km])
    smp = workload.splitmix_bytes(16 * n, seed=11)
    s_d = t(smp)
    kid = torch.zeros(n, dtype=torch.int32, device=DEV)
    masks = torch.zeros(5 * n, dtype=torch.uint8, device=DEV)
    ms = timed(lambda: batch.hp_mask(kt, kid, s_d, masks), reps)  # parity: tests/test_gpu_parity.py
    return {"samples": n, "ms": round(ms, 4), "masks_per_s": round(n / ms * 1e3)}


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "recv":  # receive runs only: recv REPS CONNS...
        assert _lib.load().mq_device_init(0) == 0
        reps = int(sys.argv[2])
        res = {f"recv_{nc}_connections": bench_protect_recv(reps, n_conns=nc, only="recv")[1]
               for nc in map(int, sys.argv[3:])}
        print(json.dumps(res), flush=True)
        return
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    assert _lib.load().mq_device_init(0) == 0
    res = {"device": torch.cuda.get_device_name(0), "derive": bench_derive(reps)}
    res["protect"], res["recv"] = bench_protect_recv(reps)
    # the receive walk over few connections (r05: runs cut into segments of kSeg packets per wave)
    for nc in (1024, 64, 4, 1):
        res[f"recv_{nc}_connections"] = bench_protect_recv(reps, n_conns=nc, only="recv")[1]
    res["records_1200"] = bench_records(reps, 1 << 20, 1200)
    res["records_16k"] = bench_records(reps, 1 << 16, 16384 + 5 + 17)
    res["hp_mask_aes"] = bench_hp_mask(reps, _lib.MQ_SUITE_AES128GCM)
    res["hp_mask_chacha"] = bench_hp_mask(reps, _lib.MQ_SUITE_CHACHA20)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
