"""Per-step seal / open times of config B around idle gaps (why the first timed steps
of bench.py run slow). Phases, each timed with HIP events per step on the bench's stream:
  cold:     after a 0.5-s idle, K steps enqueued back to back
  synced:   K steps with a host sync after each
  hot:      K steps back to back right after `synced` (only the sync's gap)
  gapX:     after an idle of X ms, K steps back to back
Usage: python tools/clock_probe.py [K]"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from milli_quic_amd import _lib, batch, workload  # noqa: E402
from milli_quic_amd.batch import KeyTable  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    lib = _lib.load()
    assert lib.mq_device_init(0) == 0
    dev = torch.device("cuda", 0)
    w = workload.uniform(1 << 20, _lib.MQ_SUITE_CHACHA20)
    kt = KeyTable(w.keys)
    arena = torch.from_numpy(w.arena).to(dev)
    sd = torch.from_numpy(w.seal_desc.view(np.uint8)).to(dev)
    od = torch.from_numpy(w.open_desc.view(np.uint8)).to(dev)
    st = torch.zeros(w.n, dtype=torch.uint8, device=dev)
    pn = torch.zeros(w.n, dtype=torch.int64, device=dev)
    ws = torch.empty(max(batch.workspace_bytes(w.n), 256), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3 * k)]

    def steps(sync_each):
        for i in range(k):
            ev[3 * i].record(stream)
            batch.seal(kt, arena, sd, st, w.suite_hint, ws, sh)
            ev[3 * i + 1].record(stream)
            batch.open_(kt, arena, od, st, pn, w.suite_hint, ws, sh)
            ev[3 * i + 2].record(stream)
            if sync_each:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        s = [round(ev[3 * i].elapsed_time(ev[3 * i + 1]), 3) for i in range(k)]
        o = [round(ev[3 * i + 1].elapsed_time(ev[3 * i + 2]), 3) for i in range(k)]
        return s, o

    for _ in range(3):  # first-use costs
        steps(False)
    out = {}
    time.sleep(0.5)
    out["cold"] = steps(False)
    out["synced"] = steps(True)
    out["hot"] = steps(False)
    for gap_ms in (0.2, 1, 5, 20, 100):
        steps(False)
        time.sleep(gap_ms / 1e3)
        out[f"gap{gap_ms}"] = steps(False)
    for name, (s, o) in out.items():
        print(f"{name:8s} seal first10 {s[:10]} median {np.median(s):.3f} | open first10 {o[:10]} median {np.median(o):.3f}",
              flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
