"""Receive composite over raw UDP datagrams on the GPU.

Reference: Connection::recv (src/connection/recv.rs:189-265) — CoalescedPackets splitting
(src/packet/coalesce.rs:26-133), long-header parsing (long_header.rs:92-206), header-protection
removal, decode_pn against the running largest_recv_pn, the 1-RTT key-phase logic (current /
previous / next generation keys, recv.rs:410-509) and open — without frame dispatch. The
connection table (``CONN_DTYPE``, C ``mq_conn_recv``) holds the recv key rows and the state the
batch advances; datagrams (``DGRAM_DTYPE``) arrive in order; every packet found gets a record
(``PKT_DTYPE``) in arrival order. ``recv`` runs mq_batch_recv over device tensors.
"""
import ctypes

import numpy as np

from . import _lib
from .batch import _stream_ptr
from .crypto import InvalidArgument, _raise

HAS_INITIAL, HAS_HANDSHAKE, HAS_APP, HAS_PREV, HAS_NEXT = 0x01, 0x02, 0x04, 0x08, 0x10

DGRAM_DTYPE = np.dtype([("offset", "<u8"), ("len", "<u4"), ("conn", "<u4")])
CONN_DTYPE = np.dtype([
    ("initial_row", "<u4"), ("handshake_row", "<u4"), ("app_row", "<u4", 3), ("dcid_len", "u1"),
    ("key_phase", "u1"), ("flags", "u1"), ("key_updates", "u1"), ("largest_pn", "<u8", 3), ("reserved", "<u8", 2),
])
PKT_DTYPE = np.dtype([
    ("offset", "<u8"), ("pn", "<u8"), ("len", "<u4"), ("dgram", "<u4"), ("payload_offset", "<u2"),
    ("level", "u1"), ("status", "u1"), ("key_gen", "u1"), ("reserved", "u1", 3),
])
assert DGRAM_DTYPE.itemsize == 16 and CONN_DTYPE.itemsize == 64 and PKT_DTYPE.itemsize == 32


def workspace_bytes(n_dgrams, max_pkts, n_conns):
    return _lib.load().mq_batch_recv_workspace_size(n_dgrams, max_pkts, n_conns)


def recv(kt, conns, arena, dgrams, pkts, n_pkts, workspace, stream=None):
    """mq_batch_recv over device uint8 tensors (conns is updated in place; pkts holds
    max_pkts records; n_pkts is a device int32 tensor of one element)."""
    n_conns = conns.numel() // CONN_DTYPE.itemsize
    n_dgrams = dgrams.numel() // DGRAM_DTYPE.itemsize
    max_pkts = pkts.numel() // PKT_DTYPE.itemsize
    if workspace.numel() * workspace.element_size() < workspace_bytes(n_dgrams, max_pkts, n_conns):
        raise InvalidArgument("workspace too small")
    rc = _lib.load().mq_batch_recv(
        kt.handle, ctypes.c_void_p(conns.data_ptr()), n_conns, ctypes.c_void_p(arena.data_ptr()), arena.numel(),
        ctypes.c_void_p(dgrams.data_ptr()), n_dgrams, ctypes.c_void_p(pkts.data_ptr()), max_pkts,
        ctypes.c_void_p(n_pkts.data_ptr()), ctypes.c_void_p(workspace.data_ptr()), _stream_ptr(stream))
    _raise(rc)
