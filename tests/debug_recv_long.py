"""Debugging aid for the segmented receive walk (test infrastructure): one long-run batch
(recv_traffic.long_runs) through mq_batch_recv and the oracle; prints the differing records with
their connection, index in the connection's run and neighbours. Usage (GPU box):
python tests/debug_recv_long.py [n_conns] [n_per_conn] [interleave]"""
import sys

import numpy as np

sys.path.insert(0, "tests"); sys.path.insert(0, ".")
from oracle import oracle as orc  # noqa: E402
orc.load()
from milli_quic_amd import _lib  # noqa: E402
from recv_traffic import long_runs  # noqa: E402
import test_gpu_recv as T  # noqa: E402

_lib.load().mq_device_init(0)
nc = int(sys.argv[1]) if len(sys.argv) > 1 else 4
npc = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
il = (sys.argv[3] != "0") if len(sys.argv) > 3 else True
keys, conns, arena, dgrams = long_runs(orc, nc, npc, seed=nc * 7 + npc, interleave=il)
oc, oa = conns.copy(), arena.copy()
o_pk, o_n = orc.batch_recv(keys, oc, oa, dgrams, len(dgrams), threads=8)
g_pk, g_n, gc, ga = T.gpu_recv(keys, conns, arena, dgrams, len(dgrams))
conn_of = dgrams["conn"][o_pk["dgram"]]
pos = np.zeros(len(o_pk), dtype=np.int64)
for c in range(nc):
    m = np.nonzero(conn_of == c)[0]
    pos[m] = np.arange(len(m))
bad = np.nonzero((g_pk["pn"] != o_pk["pn"]) | (g_pk["status"] != o_pk["status"]) | (g_pk["key_gen"] != o_pk["key_gen"]))[0]
print("n", o_n, g_n, "bad", len(bad), "statuses oracle", np.bincount(o_pk["status"]), "gpu", np.bincount(g_pk["status"]))
for i in bad[:10]:
    c = conn_of[i]
    m = np.nonzero(conn_of == c)[0]
    j = int(np.searchsorted(m, i))
    print(f"rec {i} conn {c} run pos {pos[i]} (segment {pos[i] // 1024}, offset {pos[i] % 1024})")
    for k in m[max(0, j - 3):j + 4]:
        print(f"   {k:6d} pos {pos[k]:6d} o st {o_pk['status'][k]} pn {o_pk['pn'][k]} gen {o_pk['key_gen'][k]} |"
              f" g st {g_pk['status'][k]} pn {g_pk['pn'][k]} gen {g_pk['key_gen'][k]}")
print("conn diff", [(f, np.nonzero(gc[f] != oc[f])[0][:5]) for f in gc.dtype.names if (gc[f] != oc[f]).any()])
print("arena equal", ga.tobytes() == oa.tobytes())
