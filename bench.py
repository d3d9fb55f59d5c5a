#!/usr/bin/env python3
"""bench.py — device-resident AEAD seal+open throughput on MI355X (BASELINE.json metric).

One "step" = seal (AEAD + header protection) then open (HP removal + decode_pn + AEAD open) of
the whole per-GPU batch, in place in HBM. Default workload = BASELINE configs[1]: 2^20 x 1200-B
1-RTT packets, ChaCha20-Poly1305. With --gpus N (torch.distributed.run,
one rank per GPU) every rank protects its own 2^20-packet shard (config D; packets are
independent, so there is no data-path collective: scaling "weak").

  value  = sum over ranks of wire bytes x 2 / (t_seal + t_open) / 2^30   [GiB/s]
  roofline.achieved = algorithmic bytes of one seal launch (2 x L per packet: read + write) /
                      its average duration, from HIP events on the launch stream
  cpu_baseline = the C oracle (oracle/, "port") on a bounded sample, host threads stated;
  cpu_openssl  = OpenSSL EVP running the same composites on that sample (16 threads and 1)
Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config b|c|e] [--packets P]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="b", choices=["b", "c", "e"])
    ap.add_argument("--packets", type=int, default=1 << 20, help="packets per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=1 << 16, help="packets in the CPU baseline sample")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="minimum timed CPU baseline work")
    ap.add_argument("--e2e", action="store_true", help="also measure the host-resident (H2D+D2H) rate")
    return ap.parse_args()


def build_workload(cfg, n, rank):
    from milli_quic_amd import workload
    seed = workload.SEED ^ (rank * 0x9E3779B97F4A7C15 & 0xFFFFFFFFFFFFFFFF)
    if cfg == "b":
        return workload.config_b(n, seed=seed)
    if cfg == "c":
        return workload.config_c(n, seed=seed)
    return workload.config_e(n, seed=seed)


def cpu_baseline(w, sample, threads, min_seconds=10.0):
    """Time the CPU oracle (seal + open) on the first `sample` packets of the same workload,
    repeated until at least `min_seconds` of CPU work have been timed (bounded sample)."""
    from oracle import oracle
    oracle.load()
    n = min(sample, w.n)
    end = int(w.seal_desc["offset"][n - 1]) + int(w.seal_desc["len"][n - 1])
    arena = w.arena[:end].copy()
    sd, od = w.seal_desc[:n].copy(), w.open_desc[:n].copy()
    oracle.batch_seal(w.keys, arena.copy(), sd[: min(n, 256)].copy(), w.suite_hint, threads)  # warm
    reps, t_seal, t_open = 0, 0.0, 0.0
    while t_seal + t_open < min_seconds:
        t0 = time.perf_counter()
        st = oracle.batch_seal(w.keys, arena, sd, w.suite_hint, threads)
        t1 = time.perf_counter()
        st2, _ = oracle.batch_open(w.keys, arena, od, w.suite_hint, threads)
        t2 = time.perf_counter()
        assert (st == 0).all() and (st2 == 0).all(), "CPU oracle failed on its sample"
        reps, t_seal, t_open = reps + 1, t_seal + (t1 - t0), t_open + (t2 - t1)
    wire = int(sd["len"].astype(np.int64).sum())
    gibs = wire * 2 * reps / (t_seal + t_open) / 2 ** 30
    return {"value": round(gibs, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"{n} packets ({wire / 1e6:.1f} MB) of the same workload, seal+open repeated {reps}x "
                      f"(seal {t_seal:.1f}s + open {t_open:.1f}s), oracle/mq_oracle.c on {threads} host threads"}


def cpu_openssl(w, sample, threads, min_seconds=3.0):
    """OpenSSL 3 EVP (libcrypto.so.3, dlopen'ed; its AVX2/AVX-512/AES-NI code paths) running the
    same seal + open composites (oracle/ossl_baseline.c) on the same bounded sample, on `threads`
    host threads and on one: the like-for-like stand-in for the reference's RustCrypto backends
    (SURVEY §8d). None when libcrypto.so.3 is absent."""
    from oracle import oracle
    if not oracle.ossl_available():
        return None
    n = min(sample, w.n)
    end = int(w.seal_desc["offset"][n - 1]) + int(w.seal_desc["len"][n - 1])
    sd, od = w.seal_desc[:n].copy(), w.open_desc[:n].copy()
    wire = int(sd["len"].astype(np.int64).sum())
    out = {"unit": "GiB/s", "kind": "openssl-evp"}
    for key, thr in (("value", threads), ("value_1core", 1)):
        arena = w.arena[:end].copy()
        reps, t = 0, 0.0
        while t < min_seconds:
            t0 = time.perf_counter()
            st = oracle.ossl_batch(w.keys, arena, sd, False, thr)
            st2 = oracle.ossl_batch(w.keys, arena, od, True, thr)
            t += time.perf_counter() - t0
            assert (st == 0).all() and (st2 == 0).all(), "OpenSSL leg failed on its sample"
            reps += 1
        out[key] = round(wire * 2 * reps / t / 2 ** 30, 3)
    out["cores"] = threads
    out["sample"] = f"{n} packets ({wire / 1e6:.1f} MB) of the same workload, seal+open, {threads} threads and 1"
    return out


def end_to_end(torch, batch, kt, w, sd, od, dev, chunks=8, reps=3):
    """Host-resident rate (the path starts and ends in a socket buffer): pinned host arena ->
    H2D -> seal -> D2H, then H2D -> open -> D2H, pipelined over `chunks` descriptor ranges on
    two streams so copies overlap kernels. Returns GiB/s of wire bytes per direction."""
    n = w.n
    host = torch.from_numpy(w.arena).pin_memory()
    back = torch.empty_like(host).pin_memory()
    arena = torch.empty(host.numel(), dtype=torch.uint8, device=dev)
    st = torch.zeros(n, dtype=torch.uint8, device=dev)
    pn = torch.zeros(n, dtype=torch.int64, device=dev)
    per = (n + chunks - 1) // chunks
    wsl = [torch.empty(max(batch.workspace_bytes(per), 256), dtype=torch.uint8, device=dev) for _ in range(2)]
    offs = w.seal_desc["offset"].astype(np.int64)
    ends = offs + w.seal_desc["len"].astype(np.int64)
    bounds = [(n * k) // chunks for k in range(chunks + 1)]
    streams = [torch.cuda.Stream(device=dev) for _ in range(2)]

    def one_pass(desc, open_):
        for k in range(chunks):
            lo, hi = bounds[k], bounds[k + 1]
            if hi == lo:
                continue
            a, b = int(offs[lo:hi].min()), int(ends[lo:hi].max())
            s = streams[k % 2]
            with torch.cuda.stream(s):
                arena[a:b].copy_(host[a:b], non_blocking=True)
                if open_:
                    batch.open_(kt, arena, desc[32 * lo:32 * hi], st[lo:hi], pn[lo:hi], w.suite_hint,
                                wsl[k % 2], s.cuda_stream)
                else:
                    batch.seal(kt, arena, desc[32 * lo:32 * hi], st[lo:hi], w.suite_hint, wsl[k % 2],
                               s.cuda_stream)
                back[a:b].copy_(arena[a:b], non_blocking=True)
        torch.cuda.synchronize()

    res = {}
    for name, desc, open_ in (("seal", sd, False), ("open", od, True)):
        one_pass(desc, open_)  # warm
        t0 = time.perf_counter()
        for _ in range(reps):
            one_pass(desc, open_)
        dt = (time.perf_counter() - t0) / reps
        res[name] = round(w.wire_bytes / dt / 2 ** 30, 2)
        if not open_:
            host.copy_(back)  # the open pass starts from the sealed bytes
    return {"unit": "GiB/s of wire bytes, host-resident (pinned) in and out", "chunks": chunks,
            "seal": res["seal"], "open": res["open"]}


KERNELS = {"b": "mq_chacha_seal_kernel", "c": "mq_aes_seal_kernel", "e": None}


def seal_kernel(cfg, n_rows):
    """The seal kernel a single-suite batch launches: the "1" variant (key material in SGPRs)
    when the key table has a single row (launchers in mq_chacha.hip / mq_aes.hip)."""
    k = KERNELS.get(cfg)
    return k.replace("_seal_kernel", "_seal1_kernel") if k and n_rows == 1 else k


def load_traffic(cfg, kern):
    """HBM bytes per launch of the roofline kernel from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic_<cfg>.json, written by tools/pmc_summary.py: FETCH_SIZE x 2 + WRITE_SIZE),
    measured at the default 2^20 packets per GPU (reported only for that size)."""
    path = os.path.join(ROOT, "profiles", f"pmc_traffic_{cfg}.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return int(d["kernels"][kern]["hbm_bytes_per_launch"]) if kern else None
    except (OSError, ValueError, KeyError, TypeError):
        return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # MQ_BENCH_BACKEND=gloo with more ranks than GPUs rehearses the N-rank path on one GPU
    # (ranks then share devices: local % device_count); the driver's runs use RCCL, one GPU per rank
    backend = os.environ.get("MQ_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(local)

    from milli_quic_amd import _lib, batch
    from milli_quic_amd.batch import KeyTable
    lib = _lib.load()
    rc = lib.mq_device_init(local)
    if rc != 0:
        raise SystemExit(f"libmq_aead: no usable gfx950 device ({_lib.status_str(rc)})")

    w = build_workload(args.config, args.packets, rank)
    dev = torch.device("cuda", local)
    kt = KeyTable(w.keys)
    arena = torch.from_numpy(w.arena).to(dev)
    sd = torch.from_numpy(w.seal_desc.view(np.uint8)).to(dev)
    od = torch.from_numpy(w.open_desc.view(np.uint8)).to(dev)
    st = torch.zeros(w.n, dtype=torch.uint8, device=dev)
    pn = torch.zeros(w.n, dtype=torch.int64, device=dev)
    ws = torch.empty(max(batch.workspace_bytes(w.n), 256), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream

    def step(ev=None, i=0):
        if ev is not None:
            ev[3 * i].record(stream)
        batch.seal(kt, arena, sd, st, w.suite_hint, ws, sh)
        if ev is not None:
            ev[3 * i + 1].record(stream)
        batch.open_(kt, arena, od, st, pn, w.suite_hint, ws, sh)
        if ev is not None:
            ev[3 * i + 2].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # correctness gate before timing: the roundtrip must succeed for every packet
    fails = int((st != 0).sum())
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3 * args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(ev, i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    fails += int((st != 0).sum())
    seal_ms = float(np.mean([ev[3 * i].elapsed_time(ev[3 * i + 1]) for i in range(args.steps)]))
    open_ms = float(np.mean([ev[3 * i + 1].elapsed_time(ev[3 * i + 2]) for i in range(args.steps)]))

    wire = w.wire_bytes
    from milli_quic_amd.shard import reduce_totals
    tot = reduce_totals(elapsed, wire, fails, dist if world > 1 else None, dev)
    elapsed, fails, total_wire = tot.elapsed, tot.failures, float(tot.wire_bytes)
    ms_per_step = elapsed / args.steps * 1e3
    value = total_wire * 2 / (elapsed / args.steps) / 2 ** 30

    if rank == 0:
        # roofline kernel: seal — for configs b/c a single launch (mq_chacha_seal_kernel /
        # mq_aes_seal_kernel) timed by events on its stream; open = pre-pass + packet kernel
        algo_bytes = 2.0 * wire  # per launch: read + write of every wire byte
        achieved = algo_bytes / (seal_ms * 1e-3) / 1e9
        kern = seal_kernel(args.config, len(w.keys))
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": load_traffic(args.config, kern) if w.n == 1 << 20 else None,
                # north_star's "HBM-read roofline" fraction: wire bytes read per seal ÷ 8 TB/s
                "read_frac": round(wire / (seal_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "kernel": kern or "seal batch (partition + AES + ChaCha kernels)",
                "seal_ms": round(seal_ms, 4), "open_ms": round(open_ms, 4),
                "algorithmic_bytes_per_launch": int(algo_bytes)}
        cpu = ossl = None
        if world == 1 and not args.no_cpu_baseline:
            thr = min(16, os.cpu_count() or 1)
            cpu = cpu_baseline(w, args.cpu_sample, thr, args.cpu_seconds)
            ossl = cpu_openssl(w, args.cpu_sample, thr)
        names = {"b": "configs[1]: 1M x 1200B ChaCha20-Poly1305 seal+open, 1-RTT short header",
                 "c": "configs[2]: 1M x 1200B AES-128-GCM seal+open + header protection",
                 "e": "configs[4]: mixed 64-1350B batch, Initial + 1-RTT, ChaCha20/AES-GCM interleaved"}
        out = {
            "metric": "GiB/s device-resident AEAD seal+open, 1M×1200B QUIC packets, 1/2/4/8 GPU",
            "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
            "config": {"workload": names[args.config], "packets_per_gpu": w.n,
                       "wire_bytes_per_gpu": wire, "parallelism": f"dp{world} (independent packet shards)",
                       "seal_failures_or_open_failures": fails},
            "roofline": roof, "cpu_baseline": cpu,
        }
        if ossl is not None:
            out["cpu_openssl"] = ossl
        if args.e2e and world == 1:
            out["end_to_end"] = end_to_end(torch, batch, kt, w, sd, od, dev)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
