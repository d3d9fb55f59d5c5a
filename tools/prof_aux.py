"""Minimal driver of the SURVEY §8f composites for profiler runs (rocprofv3 --kernel-trace --stats):
mq_batch_protect and mq_batch_recv at 2^20 x 1200-B packets over 4096 connections, `reps` times
each (tools/bench_aux.py's workloads).
Usage: python tools/prof_aux.py [protect|recv|both] [reps] [connections]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench_aux  # noqa: E402


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "both"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    assert bench_aux._lib.load().mq_device_init(0) == 0
    n_conns = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
    p, r = bench_aux.bench_protect_recv(reps, n_conns=n_conns, only=which)
    print("protect", p, "recv", r, flush=True)


if __name__ == "__main__":
    main()
