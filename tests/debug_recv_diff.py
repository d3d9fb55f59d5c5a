"""Debugging aid for the receive composite (test infrastructure): runs one seeded traffic batch
through mq_batch_recv and the oracle and prints the first differing packets.
Usage (GPU box): python tests/debug_recv_diff.py"""
import sys, numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import torch
from oracle import oracle as orc
orc.load()
from milli_quic_amd import _lib, recv
from recv_traffic import assemble, build_traffic
import test_gpu_recv as T
_lib.load().mq_device_init(0)
keys, conns, scripts = build_traffic(orc, seed=11, n_conns=64, n_app=60)
arena, dgrams = assemble(orc, keys, conns, scripts, seed=11)
oc, oa = conns.copy(), arena.copy()
o_pk, o_n = orc.batch_recv(keys, oc, oa, dgrams, 1 << 16)
g_pk, g_n, gc, ga = T.gpu_recv(keys, conns, arena, dgrams, 1 << 16)
bad = np.nonzero((g_pk["pn"] != o_pk["pn"]) | (g_pk["status"] != o_pk["status"]))[0]
print("n", o_n, g_n, "bad", len(bad))
for i in bad[:12]:
    c = dgrams["conn"][o_pk["dgram"][i]]
    print(i, "conn", c, "lvl", o_pk["level"][i], "o", o_pk["status"][i], o_pk["pn"][i], o_pk["key_gen"][i], "g", g_pk["status"][i], g_pk["pn"][i], g_pk["key_gen"][i], "len", o_pk["len"][i])
print("conn diff", np.nonzero((gc != oc))[0][:10])
