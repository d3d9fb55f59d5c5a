"""Device-resident batch API: the send / receive composites of the reference over a whole arena.

Reference composites reproduced per packet: send = build_and_encrypt_packet
(src/connection/transmit.rs:625-755, Initial twin :499-622); receive = recv_short /
decrypt_long_packet (src/connection/recv.rs:340-421, :953-1025). The reference processes one
packet per call; here a batch of packets sitting in one HBM arena is protected in one launch.
Torch supplies device memory and the stream only; the transforms are libmq_aead.so kernels.
"""
import ctypes

import numpy as np

from . import _lib
from . import crypto
from .crypto import _raise

DESC_DTYPE = np.dtype([
    ("offset", "<u8"), ("len", "<u4"), ("key_id", "<u4"), ("pn", "<u8"),
    ("pn_offset", "<u2"), ("pn_len", "u1"), ("flags", "u1"), ("reserved", "<u4"),
])
assert DESC_DTYPE.itemsize == 32


def make_descs(offsets, lens, key_ids, pns, pn_offsets, pn_lens, flags):
    """Build an mq_pkt_desc array (numpy structured, 32 B per packet)."""
    n = len(offsets)
    d = np.zeros(n, dtype=DESC_DTYPE)
    d["offset"] = offsets
    d["len"] = lens
    d["key_id"] = key_ids
    d["pn"] = pns
    d["pn_offset"] = pn_offsets
    d["pn_len"] = pn_lens
    d["flags"] = flags
    return d


class KeyTable:
    """Device key table (mq_keytable): AES schedules and GHASH powers expanded once on the host."""

    def __init__(self, rows):
        lib = _lib.load()
        arr = (_lib.KeyMaterial * max(len(rows), 1))(*rows)
        h = ctypes.c_void_p()
        _raise(lib.mq_keytable_create(arr, len(rows), ctypes.byref(h)))
        self._h = h
        self.rows = len(rows)

    @property
    def handle(self):
        return self._h

    def update(self, first_row, rows):
        arr = (_lib.KeyMaterial * len(rows))(*rows)
        _raise(_lib.load().mq_keytable_update(self._h, first_row, arr, len(rows)))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            _lib.load().mq_keytable_free(h)
            self._h = None


def _stream_ptr(stream):
    if stream is None:
        import torch
        return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    return ctypes.c_void_p(stream)


def workspace_bytes(n):
    return _lib.load().mq_batch_workspace_size(n)


def _ws_ptr(workspace, n):
    if workspace is None:
        return None
    if workspace.numel() * workspace.element_size() < workspace_bytes(n):
        raise crypto.InvalidArgument(f"workspace needs {workspace_bytes(n)} bytes for {n} packets")
    return ctypes.c_void_p(workspace.data_ptr())


def _check_out(status, pn_out, n):
    if status.numel() < n:
        raise crypto.InvalidArgument("status needs one byte per packet")
    if pn_out is not None and pn_out.numel() * pn_out.element_size() < 8 * n:
        raise crypto.InvalidArgument("pn_out needs 8 bytes per packet")


def seal(kt, arena, desc, status, suite_hint, workspace=None, stream=None):
    """Seal + header-protect every packet of `desc` in the device `arena` (torch uint8 tensors)."""
    n = desc.numel() // 32
    _check_out(status, None, n)
    ws = _ws_ptr(workspace, n)
    rc = _lib.load().mq_batch_seal(kt.handle, ctypes.c_void_p(arena.data_ptr()), arena.numel(),
                                   ctypes.c_void_p(desc.data_ptr()), n, ctypes.c_void_p(status.data_ptr()),
                                   suite_hint, ws, _stream_ptr(stream))
    _raise(rc)


def open_(kt, arena, desc, status, pn_out, suite_hint, workspace=None, stream=None):
    """Remove header protection, decode PNs and open every packet of `desc` in place."""
    n = desc.numel() // 32
    _check_out(status, pn_out, n)
    ws = _ws_ptr(workspace, n)
    pn = ctypes.c_void_p(pn_out.data_ptr()) if pn_out is not None else None
    rc = _lib.load().mq_batch_open(kt.handle, ctypes.c_void_p(arena.data_ptr()), arena.numel(),
                                   ctypes.c_void_p(desc.data_ptr()), n, ctypes.c_void_p(status.data_ptr()),
                                   pn, suite_hint, ws, _stream_ptr(stream))
    _raise(rc)


def derive_initial(kt, first_row, dcids, dcid_lens, status, km_out=None, stream=None):
    """Batched derive_initial (connection/keys.rs:181-212) on the GPU: for n client DCIDs
    (device uint8 tensors: dcids n x 20, dcid_lens n) write key-table rows first_row + 2i (client
    keys) and first_row + 2i + 1 (server keys); km_out (n x 2 x 88 bytes) gets the key material."""
    n = dcid_lens.numel()
    if dcids.numel() < 20 * n or status.numel() < n:
        raise crypto.InvalidArgument("dcids needs 20 bytes and status 1 byte per connection")
    if km_out is not None and km_out.numel() * km_out.element_size() < 2 * 88 * n:
        raise crypto.InvalidArgument("km_out needs 2 x 88 bytes per connection")
    rc = _lib.load().mq_batch_derive_initial(kt.handle, first_row, ctypes.c_void_p(dcids.data_ptr()),
                                             ctypes.c_void_p(dcid_lens.data_ptr()), n,
                                             ctypes.c_void_p(km_out.data_ptr()) if km_out is not None else None,
                                             ctypes.c_void_p(status.data_ptr()), _stream_ptr(stream))
    _raise(rc)


def seal_records(kt, arena, desc, status, suite_hint, workspace=None, stream=None):
    """Seal every TLS record of `desc` (MQ_PKT_TLS_RECORD rows, tls_record.record_descs) in place:
    writes each record header and inner content type, then seals (tcp_tls/record.rs:88-113)."""
    n = desc.numel() // 32
    _check_out(status, None, n)
    rc = _lib.load().mq_batch_seal_records(kt.handle, ctypes.c_void_p(arena.data_ptr()), arena.numel(),
                                           ctypes.c_void_p(desc.data_ptr()), n, ctypes.c_void_p(status.data_ptr()),
                                           suite_hint, _ws_ptr(workspace, n), _stream_ptr(stream))
    _raise(rc)


def open_records(kt, arena, desc, status, info, suite_hint, workspace=None, stream=None):
    """Open every record in place and find its inner content type (record.rs:122-143,
    connection.rs:546-556); info[i] = data_len | inner_type << 32 (tls_record.unpack_info)."""
    n = desc.numel() // 32
    _check_out(status, info, n)
    rc = _lib.load().mq_batch_open_records(kt.handle, ctypes.c_void_p(arena.data_ptr()), arena.numel(),
                                           ctypes.c_void_p(desc.data_ptr()), n, ctypes.c_void_p(status.data_ptr()),
                                           ctypes.c_void_p(info.data_ptr()), suite_hint, _ws_ptr(workspace, n),
                                           _stream_ptr(stream))
    _raise(rc)


def hp_mask(kt, key_ids, samples, masks, stream=None):
    """Batched HeaderProtection::mask: masks[i] = mask(row key_ids[i], samples[i])."""
    n = key_ids.numel()
    rc = _lib.load().mq_batch_hp_mask(kt.handle, ctypes.c_void_p(key_ids.data_ptr()),
                                      ctypes.c_void_p(samples.data_ptr()), ctypes.c_void_p(masks.data_ptr()),
                                      n, _stream_ptr(stream))
    _raise(rc)


def time_seal_open(kt, arena, desc, status, pn_out, suite_hint, iters, workspace=None, stream=None):
    """Back-to-back (seal, open) pairs timed with HIP events on the launch stream.
    Returns (seal_ms, open_ms) averaged per kernel pass."""
    n = desc.numel() // 32
    s_ms, o_ms = ctypes.c_float(), ctypes.c_float()
    ws = ctypes.c_void_p(workspace.data_ptr()) if workspace is not None else None
    rc = _lib.load().mq_batch_time_seal_open(
        kt.handle, ctypes.c_void_p(arena.data_ptr()), arena.numel(), ctypes.c_void_p(desc.data_ptr()), n,
        ctypes.c_void_p(status.data_ptr()), ctypes.c_void_p(pn_out.data_ptr()), suite_hint, ws,
        _stream_ptr(stream), iters, ctypes.byref(s_ms), ctypes.byref(o_ms))
    _raise(rc)
    return s_ms.value, o_ms.value


def flat_kind(arena_len, n, suite_hint):
    """The flat ChaCha20 kernel family a batch would run (mq_debug_chacha_flat_kind): 0 narrow,
    1 / 2 / 3 octet tiles over 10- / 13- / 20-KiB images."""
    return _lib.load().mq_debug_chacha_flat_kind(int(arena_len), int(n), int(suite_hint))


def aes_flat_kind(arena_len, n, suite_hint):
    """Lanes per packet of the flat single-key AES-128-GCM kernels a batch would run
    (mq_debug_aes_flat_kind): 2 (32 packets per wave), 4 (16) or 8 (octet tiles)."""
    return _lib.load().mq_debug_aes_flat_kind(int(arena_len), int(n), int(suite_hint))
