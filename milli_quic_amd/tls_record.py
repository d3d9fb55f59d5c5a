"""TLS 1.3 record protection over the same AEAD, mirroring the reference's record layer.

Reference (computer-whisperer/milli-quic): src/tcp_tls/record.rs:5-143 (ContentType, header
codec, build_nonce, seal_record, open_record) and src/tcp_tls/connection.rs:546-600
(find_inner_content_type, encrypt_into). This is the second caller of ``trait Aead`` besides
QUIC packet protection. seal/open run on the GPU through libmq_aead.so: per
record (``seal_record`` / ``open_record``, host buffers) or batched over a device arena
(``record_descs`` + ``batch.seal_records`` / ``batch.open_records``).
"""
import ctypes

import numpy as np

from . import _lib
from .batch import make_descs
from .crypto import BufferTooSmall, TlsError, _raise, nonce as _nonce

CHANGE_CIPHER_SPEC, ALERT, HANDSHAKE, APPLICATION_DATA = 20, 21, 22, 23  # record.rs:8-13
RECORD_HEADER_LEN = 5                     # record.rs:36
MAX_RECORD_PAYLOAD = 16384 + 256          # record.rs:39


def encode_record_header(content_type, length):
    """encode_record_header (record.rs:42-52): type, legacy version 0x0303, u16 length."""
    return bytes([content_type, 0x03, 0x03, (length >> 8) & 0xFF, length & 0xFF])


def decode_record_header(data):
    """decode_record_header (record.rs:55-67) -> (content_type, legacy_version, length)."""
    if len(data) < RECORD_HEADER_LEN:
        raise BufferTooSmall(RECORD_HEADER_LEN)
    if data[0] not in (CHANGE_CIPHER_SPEC, ALERT, HANDSHAKE, APPLICATION_DATA):
        raise TlsError("unknown content type")
    return data[0], (data[1] << 8) | data[2], (data[3] << 8) | data[4]


def build_nonce(iv, seq):
    """build_nonce (record.rs:70-78): iv XOR the big-endian sequence number in its last 8 bytes."""
    return _nonce(iv, seq)


def seal_record(aead, nonce, buf, payload_len, inner_content_type):
    """seal_record (record.rs:88-113): buf[:payload_len] plaintext -> ciphertext of
    plaintext || inner type, tag appended; returns payload_len + 1 + 16."""
    nonce = bytes(nonce)
    out, needed = ctypes.c_size_t(), ctypes.c_size_t()
    rc = _lib.load().mq_record_seal(aead._h, nonce, len(nonce), _lib.buf_ptr(buf), len(buf), payload_len,
                                    inner_content_type, ctypes.byref(out), ctypes.byref(needed))
    _raise(rc, needed.value)
    return out.value


def open_record(aead, nonce, buf, ciphertext_len, record_header_bytes):
    """open_record (record.rs:122-143) -> (data_len, inner content type)."""
    nonce, hdr = bytes(nonce), bytes(record_header_bytes)
    if len(hdr) != RECORD_HEADER_LEN:
        raise ValueError("record header is 5 bytes")
    dl, ct = ctypes.c_size_t(), ctypes.c_uint8()
    rc = _lib.load().mq_record_open(aead._h, nonce, len(nonce), _lib.buf_ptr(buf), len(buf), ciphertext_len,
                                    hdr, ctypes.byref(dl), ctypes.byref(ct))
    _raise(rc)
    return dl.value, ct.value


def record_descs(offsets, lens, key_ids, seqs, inner_types=0):
    """mq_pkt_desc rows for records: offset of the 5-byte header, total record length
    (5 + data + 1 + 16 to seal; 5 + the header's length field to open), sequence number,
    inner content type (seal)."""
    d = make_descs(offsets, lens, key_ids, seqs, RECORD_HEADER_LEN, 0, _lib.MQ_PKT_TLS_RECORD)
    d["reserved"] = np.asarray(inner_types, dtype=np.uint32) if np.ndim(inner_types) else inner_types
    return d


def unpack_info(info):
    """Per-record result of batch.open_records: (data_len, inner content type) arrays."""
    info = np.asarray(info, dtype=np.uint64)
    return (info & np.uint64(0xFFFFFFFF)).astype(np.int64), (info >> np.uint64(32)).astype(np.uint8)
