"""Send composite from plaintext frames on the GPU.

Reference: build_and_encrypt_initial_packet / build_and_encrypt_packet
(src/connection/transmit.rs:499-755): PN length, header + PN encode, PADDING, seal, header
protection. The connection supplies its CIDs, key phase and per-level send-key rows
(``CONN_DTYPE``, C ``mq_conn_send``); each packet is a request (``REQ_DTYPE``, C
``mq_send_req``): where its frames are, where the protected packet goes, its PN and the
largest PN that picks the PN length. ``protect`` runs mq_batch_protect over device tensors.
"""
import ctypes

import numpy as np

from . import _lib
from .batch import _stream_ptr
from .crypto import InvalidArgument, _raise

CONN_DTYPE = np.dtype([
    ("dcid_len", "u1"), ("scid_len", "u1"), ("key_phase", "u1"), ("reserved0", "u1"),
    ("dcid", "u1", 20), ("scid", "u1", 20), ("key_row", "<u4", 3), ("reserved1", "<u4", 2),
])
REQ_DTYPE = np.dtype([
    ("frames_offset", "<u8"), ("out_offset", "<u8"), ("pn", "<u8"), ("largest_acked", "<u8"),
    ("frame_len", "<u4"), ("out_cap", "<u4"), ("conn", "<u4"), ("level", "u1"), ("flags", "u1"),
    ("reserved", "<u2"),
])
assert CONN_DTYPE.itemsize == 64 and REQ_DTYPE.itemsize == 48

INITIAL, HANDSHAKE, APPLICATION = _lib.MQ_LEVEL_INITIAL, _lib.MQ_LEVEL_HANDSHAKE, _lib.MQ_LEVEL_APPLICATION
PAD_TO_MIN = _lib.MQ_SEND_PAD_TO_MIN
MAX_HEADER = 1 + 4 + 1 + 20 + 1 + 20 + 1 + 8  # Initial header with 20-B CIDs, empty token, 8-B Length


def make_conns(dcids, scids, key_rows, key_phase=0):
    """Connection rows: remote CID, local CID, key phase and [Initial, Handshake, 1-RTT] key rows."""
    n = len(dcids)
    c = np.zeros(n, dtype=CONN_DTYPE)
    for i in range(n):
        d, s = bytes(dcids[i]), bytes(scids[i])
        if len(d) > 20 or len(s) > 20:
            raise InvalidArgument("connection IDs are at most 20 bytes")
        c["dcid_len"][i], c["scid_len"][i] = len(d), len(s)
        c["dcid"][i, :len(d)] = np.frombuffer(d, dtype=np.uint8)
        c["scid"][i, :len(s)] = np.frombuffer(s, dtype=np.uint8)
    c["key_row"] = np.asarray(key_rows, dtype=np.uint32).reshape(n, 3)
    c["key_phase"] = key_phase
    return c


def max_packet_len(frame_len, level, pad_to_min=False):
    """An upper bound of the protected packet size (for out_cap / output arena planning)."""
    n = MAX_HEADER + 4 + max(frame_len, 3) + 16
    return max(n, 1201) if (level == INITIAL and pad_to_min) else n


def workspace_bytes(n):
    return _lib.load().mq_batch_protect_workspace_size(n)


def protect(kt, conns, frames, out, req, status, pkt_len, suite_hint, workspace, stream=None):
    """mq_batch_protect: build + seal + header-protect every request (device uint8 tensors)."""
    n = req.numel() // REQ_DTYPE.itemsize
    if status.numel() < n or pkt_len.numel() * pkt_len.element_size() < 4 * n:
        raise InvalidArgument("status needs 1 and pkt_len 4 bytes per packet")
    if workspace.numel() * workspace.element_size() < workspace_bytes(n):
        raise InvalidArgument(f"workspace needs {workspace_bytes(n)} bytes")
    rc = _lib.load().mq_batch_protect(
        kt.handle, ctypes.c_void_p(conns.data_ptr()), conns.numel() // CONN_DTYPE.itemsize,
        ctypes.c_void_p(frames.data_ptr()), frames.numel(), ctypes.c_void_p(out.data_ptr()), out.numel(),
        ctypes.c_void_p(req.data_ptr()), n, ctypes.c_void_p(status.data_ptr()), ctypes.c_void_p(pkt_len.data_ptr()),
        suite_hint, ctypes.c_void_p(workspace.data_ptr()), _stream_ptr(stream))
    _raise(rc)
