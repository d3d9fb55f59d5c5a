#!/usr/bin/env python3
"""bench.py — device-resident AEAD seal+open throughput on MI355X (BASELINE.json metric).

One "step" = seal (AEAD + header protection) then open (HP removal + decode_pn + AEAD open) of
the whole per-GPU batch, in place in HBM. Default workload = BASELINE configs[1]: 2^20 x 1200-B
1-RTT packets, ChaCha20-Poly1305.

N GPUs (config D): one process per GPU. `python bench.py --gpus N` launches the N
ranks itself (torch.distributed.run as a child process, started before anything touches the GPU);
under the driver's own `torch.distributed.run ... bench.py --gpus N` each rank just runs. The N
ranks hold ONE global batch of N x 2^20 packets: rank s owns packets [s 2^20, (s+1) 2^20) (global
index g -> pn 0x10000000 + g, key row g mod K, payload bytes [1200 g, 1200 (g+1)) of the SplitMix64
stream). Rank 0 derives the keys and broadcasts them (RCCL); packets are independent, so there is
no data-path collective ("weak" scaling). After the timed region the ranks all-reduce their
failure counts and tag checksums; rank 0 checks the checksum of a fixed sample of global indices
against the CPU oracle (the checker, outside the timed region).

  value  = sum over ranks of wire bytes x 2 / max-over-ranks(t_seal + t_open) / 2^30   [GiB/s]
  roofline.achieved = algorithmic bytes of one seal (2 x L per packet: read + write) / the seal
                      composite's average duration (tile kernel + HP pass), HIP events on its stream
  cpu_baseline = the C oracle (oracle/, "port") on a bounded sample (1 core, the box's CPU share,
                 all cores); cpu_openssl = OpenSSL EVP running the same composites
Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config b|c|e] [--packets P] [--keys K]
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)  # ~0.2-0.3 s timed: long enough for SMI samplers
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--warmup-seconds", type=float, default=0.25,
                    help="after the W warm-up steps, keep running untimed steps until this much time has passed "
                         "(the GPU's clocks ramp over ~20 ms of load after an idle of a few ms: tools/clock_probe.py)")
    ap.add_argument("--config", default="b", choices=["b", "c", "e"])
    ap.add_argument("--packets", type=int, default=1 << 20, help="packets per GPU")
    ap.add_argument("--keys", type=int, default=1, help="configs b/c: key rows, key_id = g mod K (SURVEY §8d)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=1 << 16, help="packets in the CPU baseline sample")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="minimum timed CPU work per thread count")
    ap.add_argument("--e2e", action="store_true", help="also measure the host-resident (H2D+D2H) rate")
    return ap.parse_args(argv)


# ---- launcher -------------------------------------------------------------------------------
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv, script=None):
    """Run `script` (this file) as n ranks under torch.distributed.run, one process per GPU, in a
    child process (this process never initialises the GPU; no exec). Returns the exit code."""
    script = script or os.path.abspath(__file__)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", script, *argv]
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    return subprocess.call(cmd, env=env)


def init_dist(backend):
    """One rank per GPU: (rank, world, local device index). backend "nccl" is RCCL on ROCm;
    "gloo" rehearses the N-rank path (on one GPU: ranks share device local % device_count)."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend == "gloo" and torch.cuda.device_count() > 0:
        local = local % torch.cuda.device_count()
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    return rank, world, local


# ---- workload ---------------------------------------------------------------------------------
def rank_keys(cfg, n_keys, dist, device):
    """Key rows: derived by rank 0 (HKDF from the RFC 9001 secrets), broadcast to every rank."""
    from milli_quic_amd import _lib, shard, workload
    if cfg == "e":
        return None  # config E derives its own per-connection keys on every rank
    rows = None
    if dist is None or not dist.is_initialized() or dist.get_rank() == 0:
        suite = _lib.MQ_SUITE_CHACHA20 if cfg == "b" else _lib.MQ_SUITE_AES128GCM
        rows = workload.uniform_keys(suite, n_keys)
    return shard.broadcast_keys(rows, dist, device)


def build_shard(cfg, n, rank, world, keys):
    """This rank's shard of ONE global batch of world x n packets. Configs b/c: global indices
    [rank n, (rank+1) n). Config e (mixed lengths): the range at byte quantiles of the global
    batch's packet lengths (shard.shard_range_bytes), so every rank gets about 1/world
    of the wire bytes. Returns (workload, first global index of the shard)."""
    from milli_quic_amd import _lib, shard, workload
    if cfg == "e":
        plan = workload.mixed_plan(n * world)
        lo, hi = shard.shard_range_bytes(plan.L, rank, world)
        return workload.config_e(n * world, lo=lo, hi=hi), lo
    suite = _lib.MQ_SUITE_CHACHA20 if cfg == "b" else _lib.MQ_SUITE_AES128GCM
    return workload.uniform(n, suite, start=rank * n, keys=keys), rank * n


def sample_for_rank(n_global, first, n_local):
    """(global sample indices, local positions of those in this rank's shard [first, first + n_local))."""
    from milli_quic_amd import shard
    g = shard.sample_indices(n_global)
    mine = g[(g >= first) & (g < first + n_local)]
    return g, mine - first


def parity_check(cfg, n_global, g_sample, keys, fails, csum, s_csum, pn_ok, dist=None, device=None):
    """Whole-job parity after the timed region (the checker, CPU oracle). Every config holds ONE
    global batch: the ranks all-reduce the checksum of the tags at the fixed global sample and
    rank 0's oracle seals exactly those packets. Returns the parity record (identical on every
    rank)."""
    from milli_quic_amd import shard
    world = dist.get_world_size() if dist is not None and dist.is_initialized() else 1
    rank = dist.get_rank() if world > 1 else 0
    fails_all, csum_all, s_csum_all, pn_bad = shard.reduce_sums(
        [fails, csum, s_csum, 0 if pn_ok else 1], dist, device)
    o_fail, o_csum = oracle_sample_checksum(cfg, n_global, g_sample, keys) if rank == 0 else (0, None)
    bad0 = int(rank == 0 and not (o_fail == 0 and o_csum == s_csum_all))
    match = shard.reduce_sums([bad0], dist, device)[0] == 0  # rank 0's verdict on every rank
    return {"failures": fails_all, "pn_mismatch_ranks": pn_bad, "tag_checksum": csum_all,
            "sample_packets": int(len(g_sample)), "sample_tag_checksum": s_csum_all,
            "oracle_sample_tag_checksum": o_csum, "sample_scope": f"global batch of {n_global}",
            "match": bool(match and fails_all == 0 and pn_bad == 0)}


def oracle_sample_checksum(cfg, n_global, g, keys):
    """CPU oracle (the checker) on the sampled global indices: the tag checksum the GPU run must
    reproduce."""
    from milli_quic_amd import _lib, shard, workload
    from oracle import oracle
    oracle.load()
    if cfg == "e":
        sw = workload.config_e_at(g, n_global)
    else:
        suite = _lib.MQ_SUITE_CHACHA20 if cfg == "b" else _lib.MQ_SUITE_AES128GCM
        sw = workload.uniform_at(g, suite, keys=keys)
    st = oracle.batch_seal(sw.keys, sw.arena, sw.seal_desc, sw.suite_hint, threads=min(16, os.cpu_count() or 1))
    return int((st != 0).sum()), shard.tag_checksum(sw.arena, sw.seal_desc)


# ---- CPU baselines (reported, not the target) -------------------------------------------------
def cpu_threads():
    """(1, the box's CPU share, every CPU the OS shows). The share is OMP_NUM_THREADS (16 per GPU
    on the GPU box) or the affinity mask."""
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if share <= 0:
        share = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return 1, share, os.cpu_count() or share


def _sample(w, sample):
    n = min(sample, w.n)
    end = int(w.seal_desc["offset"][n - 1]) + int(w.seal_desc["len"][n - 1])
    sd, od = w.seal_desc[:n].copy(), w.open_desc[:n].copy()
    return n, end, sd, od, int(sd["len"].astype(np.int64).sum())


# the box shows all its CPUs while this job's share is `cores`: a run on every visible CPU
# oversubscribes the share and measures thrashing, not capacity
ALL_CPUS_NOTE = ("threads = every CPU the box shows, many times this job's share: oversubscribed "
                 "(thrash), not a capacity figure; `value` (the share) is the baseline")


def cpu_baseline(w, sample, min_seconds=8.0):
    """The C oracle (oracle/mq_oracle.c, byte-wise scalar "port") timed on seal + open of the first
    `sample` packets of the same workload, repeated until min_seconds of work were timed, at 1
    thread, the CPU share and all CPUs. `value` is the CPU-share figure."""
    from oracle import oracle
    oracle.load()
    n, end, sd, od, wire = _sample(w, sample)
    one, share, allc = cpu_threads()
    res = {}
    for label, thr, secs in (("value_1core", one, min_seconds / 2), ("value", share, min_seconds),
                             ("value_all_cpus", allc, min_seconds / 2)):
        if label == "value_all_cpus" and allc == share:
            continue
        arena = w.arena[:end].copy()
        oracle.batch_seal(w.keys, arena.copy(), sd[: min(n, 256)].copy(), w.suite_hint, thr)  # warm
        reps, t = 0, 0.0
        while t < secs:
            t0 = time.perf_counter()
            st = oracle.batch_seal(w.keys, arena, sd, w.suite_hint, thr)
            st2, _ = oracle.batch_open(w.keys, arena, od, w.suite_hint, thr)
            t += time.perf_counter() - t0
            assert (st == 0).all() and (st2 == 0).all(), "CPU oracle failed on its sample"
            reps += 1
        res[label] = round(wire * 2 * reps / t / 2 ** 30, 3)
    return {"value": res["value"], "unit": "GiB/s", "cores": share, "kind": "port",
            "value_1core": res["value_1core"], "value_all_cpus": res.get("value_all_cpus"),
            "cpus_visible": allc,
            "value_all_cpus_note": ALL_CPUS_NOTE if res.get("value_all_cpus") is not None else None,
            "sample": f"{n} packets ({wire / 1e6:.1f} MB) of the same workload, seal+open repeated; "
                      f"oracle/mq_oracle.c on {share} threads (the box's CPU share), also 1 and {allc}"}


def cpu_openssl(w, sample, min_seconds=3.0):
    """OpenSSL 3 EVP (libcrypto.so.3, dlopen'ed; its AVX2/AVX-512/AES-NI code paths) running the
    same seal + open composites (oracle/ossl_baseline.c) on the same bounded sample, at 1 thread,
    the CPU share and all CPUs: the like-for-like stand-in for the reference's RustCrypto backends
    (SURVEY §8d). OpenSSL 3.0's per-packet EVP re-initialisation serialises across threads
    (tools/ossl_scaling.c), so value_1core x cores is its uncontended projection.
    None when libcrypto.so.3 is absent."""
    from oracle import oracle
    if not oracle.ossl_available():
        return None
    n, end, sd, od, wire = _sample(w, sample)
    one, share, allc = cpu_threads()
    out = {"unit": "GiB/s", "kind": "openssl-evp", "cores": share, "cpus_visible": allc}
    for label, thr in (("value_1core", one), ("value", share), ("value_all_cpus", allc)):
        if label == "value_all_cpus" and allc == share:
            continue
        arena = w.arena[:end].copy()
        reps, t = 0, 0.0
        while t < min_seconds:
            t0 = time.perf_counter()
            st = oracle.ossl_batch(w.keys, arena, sd, False, thr)
            st2 = oracle.ossl_batch(w.keys, arena, od, True, thr)
            t += time.perf_counter() - t0
            assert (st == 0).all() and (st2 == 0).all(), "OpenSSL leg failed on its sample"
            reps += 1
        out[label] = round(wire * 2 * reps / t / 2 ** 30, 3)
    out["uncontended_projection"] = round(out["value_1core"] * share, 3)
    if "value_all_cpus" in out:
        out["value_all_cpus_note"] = ALL_CPUS_NOTE
    out["sample"] = f"{n} packets ({wire / 1e6:.1f} MB) of the same workload, seal+open, 1/{share}/{allc} threads"
    return out


# ---- end-to-end (host-resident) ---------------------------------------------------------------
def end_to_end(torch, batch, kt, w, sd, od, dev, reps=3):
    """Host-resident rate (the path starts and ends in a socket buffer): pinned host arena ->
    H2D -> seal -> D2H, then H2D -> open -> D2H, pipelined over chunks of descriptor ranges. Since
    r05 the two copy directions run on copy streams of their own and the kernels on a third,
    joined by events, so chunk k's D2H runs beside chunk k + 1's H2D and chunk k's kernel (r02-r04
    ran each chunk's H2D, kernel and D2H on one stream: the directions barely overlapped, 0.60 of
    the one-way bound). Every wire byte crosses the link once each way, so the
    slower direction alone bounds the rate from above (`link_bound`); the same chunked pipeline
    with no kernel (chunk k + 1's H2D beside chunk k's D2H) is reported next to it as the duplex
    copy RATE — a measurement the kernels' pipeline can match or, by noise, exceed, not a bound
    (ADVICE r05). Each chunk's batch carries MQ_BATCH_LEN_HINT: its descriptors cover part of the
    whole arena, whose size would otherwise pick the long-packet kernel. Returns GiB/s
    of wire bytes."""
    from milli_quic_amd import _lib
    n = w.n
    host = torch.from_numpy(w.arena).pin_memory()
    back = torch.empty_like(host).pin_memory()
    arena = torch.empty(host.numel(), dtype=torch.uint8, device=dev)
    st = torch.zeros(n, dtype=torch.uint8, device=dev)
    pn = torch.zeros(n, dtype=torch.int64, device=dev)
    offs = w.seal_desc["offset"].astype(np.int64)
    ends = offs + w.seal_desc["len"].astype(np.int64)
    configs = (16, 32, 64)  # chunks per pass
    s_in, s_k, s_out = (torch.cuda.Stream(device=dev) for _ in range(3))
    ws = torch.empty(max(batch.workspace_bytes(n), 256), dtype=torch.uint8, device=dev)
    hint = w.suite_hint | _lib.MQ_BATCH_LEN_HINT(-(-w.wire_bytes // n))  # bytes per packet, rounded up

    def run(desc, mode, nch, nrep=reps):
        """mode: seal / open (copy in, kernel, copy out), duplex (both copies, no kernel), h2d, d2h"""
        bounds = [(n * k) // nch for k in range(nch + 1)]
        spans = [(int(offs[bounds[k]:bounds[k + 1]].min()), int(ends[bounds[k]:bounds[k + 1]].max()))
                 for k in range(nch) if bounds[k + 1] > bounds[k]]
        idx = [(bounds[k], bounds[k + 1]) for k in range(nch) if bounds[k + 1] > bounds[k]]

        def one_pass():
            prev_out = torch.cuda.Event()
            prev_out.record(s_out)
            for (a, b), (lo, hi) in zip(spans, idx):
                e_in, e_k = torch.cuda.Event(), torch.cuda.Event()
                if mode != "d2h":
                    with torch.cuda.stream(s_in):
                        arena[a:b].copy_(host[a:b], non_blocking=True)
                    e_in.record(s_in)
                else:
                    e_in.record(s_in)
                if mode in ("seal", "open"):
                    s_k.wait_event(e_in)
                    with torch.cuda.stream(s_k):
                        if mode == "open":
                            batch.open_(kt, arena, desc[32 * lo:32 * hi], st[lo:hi], pn[lo:hi], hint, ws,
                                        s_k.cuda_stream)
                        else:
                            batch.seal(kt, arena, desc[32 * lo:32 * hi], st[lo:hi], hint, ws, s_k.cuda_stream)
                    e_k.record(s_k)
                else:
                    e_k = e_in
                if mode != "h2d":
                    s_out.wait_event(e_k)  # duplex: chunk k goes out while chunk k + 1 comes in
                    with torch.cuda.stream(s_out):
                        back[a:b].copy_(arena[a:b], non_blocking=True)
            torch.cuda.synchronize()

        one_pass()  # warm
        best = None
        for _ in range(nrep):
            t0 = time.perf_counter()
            one_pass()
            dt = time.perf_counter() - t0
            best = dt if best is None or dt < best else best
        return best

    res, cfg_used = {}, {}
    for name, desc in (("seal", sd), ("open", od)):
        best_rate = 0.0
        for nch in configs:
            host.copy_(torch.from_numpy(w.arena) if name == "seal" else sealed)
            dt = run(desc, name, nch)
            r = w.wire_bytes / dt / 2 ** 30
            if r > best_rate:
                best_rate, cfg_used[name] = r, {"streams": "h2d + kernel + d2h", "chunks": nch}
            if name == "seal":
                sealed = back.clone()  # the open pass starts from the sealed bytes
        res[name] = round(best_rate, 2)
    link, link_cfg = {}, {}
    for mode in ("duplex", "h2d", "d2h"):
        rates = {nch: w.wire_bytes / run(None, mode, nch, 5) / 2 ** 30 for nch in configs}
        link_cfg[mode] = max(rates, key=rates.get)
        link[mode] = rates[link_cfg[mode]]
    bound = min(link["h2d"], link["d2h"])
    duplex = link["duplex"]
    return {"unit": "GiB/s of wire bytes, host-resident (pinned) in and out", "pipeline_config": cfg_used,
            "seal": res["seal"], "open": res["open"],
            "link_bound": round(bound, 2), "h2d_alone": round(link["h2d"], 2), "d2h_alone": round(link["d2h"], 2),
            "frac_of_link_bound": {"seal": round(res["seal"] / bound, 3), "open": round(res["open"] / bound, 3)},
            "duplex_copy_rate": round(duplex, 2), "duplex_chunks": link_cfg["duplex"],
            "frac_of_duplex_copy_rate": {"seal": round(res["seal"] / duplex, 3), "open": round(res["open"] / duplex, 3)},
            "bound_note": "every wire byte goes in and comes out: the slower direction alone bounds the rate; "
                          "the duplex copy rate is the same chunked pipeline with no kernel (H2D of chunk k+1 "
                          "beside D2H of chunk k), measured, not a bound",
            "len_hint": -(-w.wire_bytes // n),
            "device_resident_note": "never `value`: the device-resident rate is the metric"}


# ---- roofline bookkeeping ---------------------------------------------------------------------
# The seal composite of a single-suite, single-key batch is its tile kernel (the "1" variant: key
# material in SGPRs, n_rows == 1); the tiles apply header protection themselves (ChaCha20 and AES,
# r03), so no pass follows. seal_ms (HIP events around mq_batch_seal) spans the composite.
# A mixed batch (config E) or a multi-key AES batch goes through the partition (four launches
# since r05: the count kernel's last block lays the classes out, the row blocks the keyed rows),
# then list 0's AES tiles — the hot key's segment on the single-key kernel beside the multi-key
# kernel — then list 1 (ChaCha20, or the AES hint's leftovers on the multi-key kernel again).
# mq_host.cpp batch() makes the same launches.
PARTITION = ("mq_part_init_kernel", "mq_part_count_kernel", "mq_part_rows_kernel", "mq_part_scatter_kernel")
# single-key AES kernels by lanes per packet (r06 narrow tiles: mq_aes.hip aes_lanes)
AES_SEAL1 = {8: "mq_aes_seal1_kernel", 4: "mq_aes_seal1n_kernel", 2: "mq_aes_seal1n2_kernel"}
AES_SEALS = {8: "mq_aes_seals_kernel", 4: "mq_aes_sealsn_kernel", 2: "mq_aes_sealsn2_kernel"}


def aes_segment_kernel():
    """The kernel a partition's hot AES key segment runs on (mq_aes.hip mq_launch_aes): the slice
    kernel unless MQ_AES_HOT_SEG=0, with 4 lanes per packet unless MQ_AES_NARROW says otherwise."""
    from milli_quic_amd import _lib
    lib = _lib.load()
    f = lib.mq_debug_option_get(b"MQ_AES_NARROW")
    g = 4 if f < 0 else {0: 8, 2: 2}.get(f, 4)
    return (AES_SEAL1 if lib.mq_debug_option_get(b"MQ_AES_HOT_SEG") == 0 else AES_SEALS)[g], g


def seal_kernels(cfg, n_rows, n=1 << 20, non_aes_rows=None, arena_len=None):
    if cfg == "b":
        return ("mq_chacha_seal1_kernel",) if n_rows == 1 else ("mq_chacha_seal_kernel",)
    if cfg == "c":
        if n_rows == 1:
            from milli_quic_amd import _lib, batch
            return (AES_SEAL1[batch.aes_flat_kind(arena_len or 1200 * n, n, _lib.MQ_SUITE_AES128GCM)],)
        hot, g = aes_segment_kernel()
        if n >= 512 * n_rows:  # mq_host.cpp: keys with >= 512 packets each: the key-segmented kernel
            return PARTITION + (AES_SEALS[g], "mq_aes_seal_kernel")
        return PARTITION + (hot, "mq_aes_seal_kernel", "mq_aes_seal_kernel")
    if cfg == "e":
        # list 1 on the one-shot grid list kernels (mq_chacha.hip lgrid); a key table with one
        # non-AES row takes the single-key one
        hot, _ = aes_segment_kernel()
        return PARTITION + (hot, "mq_aes_seal_kernel",
                            "mq_chacha_seal_lgrid1_kernel" if non_aes_rows == 1 else "mq_chacha_seal_lgrid_kernel")
    return None


def kernel_key(name):
    """rocprofv3 kernel name -> the name KERNELS uses (argument list and 'void ' dropped)."""
    k = name.split("(")[0]
    return k[5:] if k.startswith("void ") else k


def load_traffic(cfg, kerns, keys=1):
    """HBM bytes per seal composite (sum over its kernels) from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic_<cfg>[_k<keys>].json, written by tools/pmc_summary.py: FETCH_SIZE x 2 +
    WRITE_SIZE), measured at the default 2^20 packets per GPU (reported only for that size)."""
    path = os.path.join(ROOT, "profiles", f"pmc_traffic_{cfg}.json" if keys == 1 else f"pmc_traffic_{cfg}_k{keys}.json")
    try:
        with open(path) as f:
            d = json.load(f)["kernels"]
        if not kerns:
            return None
        by_name = {kernel_key(k): v for k, v in d.items()}
        return int(sum(by_name[k]["hbm_bytes_per_launch"] for k in kerns))
    except (OSError, ValueError, KeyError, TypeError):
        return None


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # the N ranks are child processes; this one never touches the GPU
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    import torch
    import torch.distributed as dist

    backend = os.environ.get("MQ_BENCH_BACKEND", "nccl")
    rank, world, local = init_dist(backend)
    if world != args.gpus and rank == 0:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}; using {world} ranks", file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dd = dist if world > 1 else None

    from milli_quic_amd import _lib, batch, shard
    from milli_quic_amd.batch import KeyTable
    lib = _lib.load()
    rc = lib.mq_device_init(local)
    if rc != 0:
        raise SystemExit(f"libmq_aead: no usable gfx950 device ({_lib.status_str(rc)})")

    keys = rank_keys(args.config, args.keys, dd, dev)
    w, first = build_shard(args.config, args.packets, rank, world, keys)
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

    # Nothing that can idle the GPU for milliseconds may sit between the warm-up and the timed steps
    # (after an idle of a few ms the first ~5 steps run up to 40 % slower while the clocks ramp,
    # tools/clock_probe.py): the events are created and recorded once before the warm-up (r03 created
    # them in between), and host_enqueue_ms_first5 in the output shows the timed loop's own pace.
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3 * args.steps)]
    for e in ev:
        e.record(stream)
    for _ in range(args.warmup):
        step()
    # correctness gate: every packet of the warm-up's round trips succeeded (read after the timed
    # steps). Computed here, before the time-based warm-up: the first launch of a torch kernel in
    # the process loads its code object, milliseconds in which the GPU idles — after such a gap the
    # first ~5 steps run up to 40 % slower while the clocks ramp (tools/clock_probe.py,
    # profiles/r04b_clock_probe.txt), which is what slowed the driver's 20-step runs
    fails_warm = (st != 0).sum()
    if world > 1:  # ranks start the time-based warm-up together, so they also end it together
        dist.barrier()
    extra, tw = 0, time.perf_counter()
    while time.perf_counter() - tw < args.warmup_seconds:  # untimed, the same work: clock ramp
        step()
        torch.cuda.synchronize()  # per step: a rank overshoots the deadline by at most one step
        extra += 1
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host_t = []
    for i in range(args.steps):
        step(ev, i)
        host_t.append(time.perf_counter())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    fails = int(fails_warm) + int((st != 0).sum())
    seal_t = np.array([ev[3 * i].elapsed_time(ev[3 * i + 1]) for i in range(args.steps)])
    open_t = np.array([ev[3 * i + 1].elapsed_time(ev[3 * i + 2]) for i in range(args.steps)])
    seal_ms, open_ms = float(seal_t.mean()), float(open_t.mean())
    pn_ok = bool((pn.cpu().numpy().view(np.uint64) == w.pns).all())

    # cross-rank parity: after the steps every packet holds its plaintext and the tag the last seal
    # wrote; all-reduce failures and tag checksums (whole shard, and the fixed global sample)
    offs_t = torch.from_numpy(w.seal_desc["offset"].astype(np.int64)).to(dev)
    lens_t = torch.from_numpy(w.seal_desc["len"].astype(np.int64)).to(dev)
    g_sample, local_sample = sample_for_rank(args.packets * world, first, w.n)
    ls = torch.from_numpy(local_sample.astype(np.int64)).to(dev)
    csum = shard.tag_checksum_torch(arena, offs_t, lens_t)
    s_csum = shard.tag_checksum_torch(arena, offs_t[ls], lens_t[ls])
    parity = parity_check(args.config, args.packets * world, g_sample, keys, fails, csum, s_csum, pn_ok, dd, dev)
    fails_all = parity["failures"]

    wire = w.wire_bytes
    tot = shard.reduce_totals(elapsed, wire, 0, dd, dev)
    elapsed, total_wire = tot.elapsed, float(tot.wire_bytes)
    ms_per_step = elapsed / args.steps * 1e3
    value = total_wire * 2 / (elapsed / args.steps) / 2 ** 30

    if rank == 0:
        algo_bytes = 2.0 * wire  # per launch: read + write of every wire byte
        achieved = algo_bytes / (seal_ms * 1e-3) / 1e9
        non_aes = sum(1 for k in w.keys if int(k.suite) != 1)  # MQ_SUITE_AES128GCM = 1
        kerns = seal_kernels(args.config, len(w.keys), w.n, non_aes, len(w.arena))
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": load_traffic(args.config, kerns, args.keys) if w.n == 1 << 20 else None,
                # north_star's "HBM-read roofline" fraction: wire bytes read per seal ÷ 8 TB/s
                "read_frac": round(wire / (seal_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "kernel": ("seal composite: " if args.config != "e" else "seal batch: ") + " + ".join(kerns),
                "seal_ms": round(seal_ms, 4), "open_ms": round(open_ms, 4),
                "open_frac": round(algo_bytes / (open_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "algorithmic_bytes_per_launch": int(algo_bytes),
                # per-step HIP-event times of the timed steps
                "per_step_ms": {k: {"min": round(float(t.min()), 4), "median": round(float(np.median(t)), 4),
                                    "max": round(float(t.max()), 4),
                                    "first5": [round(float(x), 4) for x in t[:5]],
                                    "last5": [round(float(x), 4) for x in t[-5:]]}
                                for k, t in (("seal", seal_t), ("open", open_t))},
                # host time to enqueue each of the first timed steps (ms): a slow enqueue idles the GPU
                "host_enqueue_ms_first5": [round((b - a) * 1e3, 3) for a, b in zip([t0] + host_t[:4], host_t[:5])]}
        cpu = ossl = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(w, args.cpu_sample, args.cpu_seconds)
            ossl = cpu_openssl(w, args.cpu_sample)
        names = {"b": "configs[1]: 1M x 1200B ChaCha20-Poly1305 seal+open, 1-RTT short header",
                 "c": "configs[2]: 1M x 1200B AES-128-GCM seal+open + header protection",
                 "e": "configs[4]: mixed 64-1350B batch, Initial + 1-RTT, ChaCha20/AES-GCM interleaved"}
        workload_name = names[args.config]
        if world > 1 and args.config == "b":
            workload_name = (f"configs[3]: {world}x{args.packets // (1 << 20) or args.packets}M x 1200B "
                             f"ChaCha20-Poly1305 batch sharded across {world} GPUs")
        elif world > 1:
            workload_name += f" — one global batch of {world}x{args.packets} packets, " + \
                ("split at byte quantiles" if args.config == "e" else "contiguous shards") + f" over {world} GPUs"
        out = {
            "metric": "GiB/s device-resident AEAD seal+open, 1M×1200B QUIC packets, 1/2/4/8 GPU",
            # a run whose results differ from the oracle has no throughput (exit status 1 below)
            "value": round(value, 2) if parity["match"] else None,
            "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "warmup_extra": {"seconds": args.warmup_seconds, "steps": extra},
            "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
            "config": {"workload": workload_name, "packets_per_gpu": w.n, "key_rows": len(w.keys),
                       "wire_bytes_per_gpu": wire, "parallelism": f"dp{world} (independent packet shards)",
                       "collectives": "key broadcast + failure/checksum all-reduce + barriers (no data path)",
                       "backend": backend if world > 1 else None,
                       "seal_failures_or_open_failures": fails_all},
            "roofline": roof, "parity": parity, "cpu_baseline": cpu,
        }
        if ossl is not None:
            out["cpu_openssl"] = ossl
        if args.e2e and world == 1:
            out["end_to_end"] = end_to_end(torch, batch, kt, w, sd, od, dev)
        print(json.dumps(out), flush=True)
        if not parity["match"]:
            print("bench.py: PARITY CHECK FAILED " + json.dumps(parity), file=sys.stderr)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if not parity["match"]:
        sys.exit(1)


if __name__ == "__main__":
    main()
