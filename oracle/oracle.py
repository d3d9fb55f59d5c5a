"""ctypes binding of the CPU oracle (oracle/build/liborc.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker / reported CPU baseline. The product (milli_quic_amd) never
imports this module. See mq_oracle.h for what the oracle restates and how it is pinned.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# MQ_ASAN=1 (tools/asan_cpu_tests.sh): the AddressSanitizer + UBSan builds of `make asan`
_BUILD = os.path.join(HERE, "build", "asan") if os.environ.get("MQ_ASAN") == "1" else os.path.join(HERE, "build")
LIB = os.path.join(_BUILD, "liborc.so")
OSSL_LIB = os.path.join(_BUILD, "libossl.so")

_lib = None
_ossl = None


def build():
    subprocess.run(["make", "-C", HERE, "-s"] + (["asan"] if _BUILD != os.path.join(HERE, "build") else []),
                   check=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
    return _lib


def _p(b):
    if b is None:
        return None
    if isinstance(b, bytes):
        return ctypes.c_char_p(b)
    if isinstance(b, np.ndarray):
        return ctypes.c_void_p(b.ctypes.data)
    return (ctypes.c_char * len(b)).from_buffer(b) if len(b) else None


def chacha20_block(key, counter, nonce):
    out = ctypes.create_string_buffer(64)
    load().orc_chacha20_block(_p(bytes(key)), ctypes.c_uint32(counter), _p(bytes(nonce)), out)
    return out.raw


def poly1305(key, msg):
    out = ctypes.create_string_buffer(16)
    msg = bytes(msg)
    load().orc_poly1305(_p(bytes(key)), _p(msg), ctypes.c_size_t(len(msg)), out)
    return out.raw


def aes128_encrypt(key, block):
    rk = (ctypes.c_uint32 * 44)()
    out = ctypes.create_string_buffer(16)
    load().orc_aes128_expand(_p(bytes(key)), rk)
    load().orc_aes128_encrypt(rk, _p(bytes(block)), out)
    return out.raw


def sha256(msg):
    out = ctypes.create_string_buffer(32)
    msg = bytes(msg)
    load().orc_sha256(_p(msg), ctypes.c_size_t(len(msg)), out)
    return out.raw


def aead_seal(suite, key, nonce, aad, pt, buf_len=None):
    """Returns (status, ciphertext||tag, needed)."""
    key, nonce, aad = bytes(key), bytes(nonce), bytes(aad)
    buf = bytearray(pt) + bytearray(16 if buf_len is None else max(0, buf_len - len(pt)))
    out, needed = ctypes.c_size_t(0), ctypes.c_size_t(0)
    rc = load().orc_aead_seal(ctypes.c_uint32(suite), _p(key), ctypes.c_size_t(len(key)), _p(nonce),
                              ctypes.c_size_t(len(nonce)), _p(aad), ctypes.c_size_t(len(aad)), _p(buf),
                              ctypes.c_size_t(len(buf)), ctypes.c_size_t(len(pt)), ctypes.byref(out),
                              ctypes.byref(needed))
    return rc, bytes(buf[:out.value]), needed.value


def aead_open(suite, key, nonce, aad, ct):
    key, nonce, aad = bytes(key), bytes(nonce), bytes(aad)
    buf = bytearray(ct)
    out = ctypes.c_size_t(0)
    rc = load().orc_aead_open(ctypes.c_uint32(suite), _p(key), ctypes.c_size_t(len(key)), _p(nonce),
                              ctypes.c_size_t(len(nonce)), _p(aad), ctypes.c_size_t(len(aad)), _p(buf),
                              ctypes.c_size_t(len(buf)), ctypes.c_size_t(len(buf)), ctypes.byref(out))
    return rc, bytes(buf[:out.value]) if rc == 0 else bytes(buf)


def hp_mask(suite, hp, sample):
    hp, sample = bytes(hp), bytes(sample)
    m = ctypes.create_string_buffer(5)
    rc = load().orc_hp_mask(ctypes.c_uint32(suite), _p(hp), ctypes.c_size_t(len(hp)), _p(sample),
                            ctypes.c_size_t(len(sample)), m)
    return rc, m.raw


def hkdf_expand_label(secret, label, ctx, length):
    out = ctypes.create_string_buffer(max(length, 1))
    secret, label, ctx = bytes(secret), bytes(label), bytes(ctx)
    rc = load().orc_hkdf_expand_label(_p(secret), ctypes.c_size_t(len(secret)), _p(label),
                                      ctypes.c_size_t(len(label)), _p(ctx), ctypes.c_size_t(len(ctx)), out,
                                      ctypes.c_size_t(length))
    return rc, out.raw[:length]


def derive_initial_secrets(dcid):
    c, s = ctypes.create_string_buffer(32), ctypes.create_string_buffer(32)
    dcid = bytes(dcid)
    load().orc_derive_initial_secrets(_p(dcid), ctypes.c_size_t(len(dcid)), c, s)
    return c.raw, s.raw


def decode_pn(truncated, pn_len, largest):
    f = load().orc_decode_pn
    f.restype = ctypes.c_uint64
    return f(ctypes.c_uint32(truncated), ctypes.c_size_t(pn_len), ctypes.c_uint64(largest))


def pn_length(full_pn, largest_acked):
    f = load().orc_pn_length
    f.restype = ctypes.c_size_t
    return f(ctypes.c_uint64(full_pn), ctypes.c_uint64(largest_acked))


def _rows(rows):
    # rows: sequence of milli_quic_amd._lib.KeyMaterial (identical layout to mq_key_material)
    if len(rows) and isinstance(rows[0], ctypes.Structure):
        arr = (type(rows[0]) * len(rows))(*rows)
        return arr, len(rows)
    raise TypeError("rows must be KeyMaterial structures")


def batch_seal(rows, arena, desc, suite_hint, threads=1):
    """Seal in place on the host copy `arena` (np.uint8); returns per-packet status."""
    arr, nr = _rows(rows)
    n = len(desc)
    status = np.zeros(n, dtype=np.uint8)
    load().orc_batch_seal(arr, ctypes.c_uint32(nr), _p(arena), ctypes.c_uint64(arena.size), _p(desc),
                          ctypes.c_uint32(n), _p(status), ctypes.c_uint32(suite_hint), ctypes.c_int(threads))
    return status


def batch_open(rows, arena, desc, suite_hint, threads=1):
    arr, nr = _rows(rows)
    n = len(desc)
    status = np.zeros(n, dtype=np.uint8)
    pn = np.zeros(n, dtype=np.uint64)
    load().orc_batch_open(arr, ctypes.c_uint32(nr), _p(arena), ctypes.c_uint64(arena.size), _p(desc),
                          ctypes.c_uint32(n), _p(status), _p(pn), ctypes.c_uint32(suite_hint),
                          ctypes.c_int(threads))
    return status, pn


def batch_protect(rows, conns, frames, out, req, suite_hint):
    """Send composite from frames (transmit.rs:499-755) into the host copy `out` (np.uint8);
    conns / req are numpy arrays of milli_quic_amd.send CONN_DTYPE / REQ_DTYPE."""
    arr, nr = _rows(rows)
    n = len(req)
    status = np.zeros(n, dtype=np.uint8)
    pkt_len = np.zeros(n, dtype=np.uint32)
    load().orc_batch_protect(arr, ctypes.c_uint32(nr), _p(conns), ctypes.c_uint32(len(conns)), _p(frames),
                             ctypes.c_uint64(frames.size), _p(out), ctypes.c_uint64(out.size), _p(req),
                             ctypes.c_uint32(n), _p(status), _p(pkt_len), ctypes.c_uint32(suite_hint))
    return status, pkt_len


def batch_recv(rows, conns, arena, dgrams, max_pkts, threads=1):
    """Receive composite over datagrams (recv.rs:189-510) on the host copies `arena` / `conns`
    (numpy, milli_quic_amd.recv dtypes; both updated in place); returns the packet records.
    threads > 1: connections split over threads (orc_batch_recv_mt, the same results)."""
    from milli_quic_amd.recv import PKT_DTYPE
    arr, nr = _rows(rows)
    out = np.zeros(max(max_pkts, 1), dtype=PKT_DTYPE)
    n = ctypes.c_uint32(0)
    args = (arr, ctypes.c_uint32(nr), _p(conns), ctypes.c_uint32(len(conns)), _p(arena), ctypes.c_uint64(arena.size),
            _p(dgrams), ctypes.c_uint32(len(dgrams)), _p(out), ctypes.c_uint32(max_pkts), ctypes.byref(n))
    if threads > 1:
        load().orc_batch_recv_mt(*args, ctypes.c_int(threads))
    else:
        load().orc_batch_recv(*args)
    return out[:min(n.value, max_pkts)], n.value


def _load_ossl():
    global _ossl
    if _ossl is None:
        if not os.path.exists(OSSL_LIB):
            build()
        _ossl = ctypes.CDLL(OSSL_LIB)
    return _ossl


def ossl_available():
    """True when libcrypto.so.3 can be dlopen'ed (OpenSSL EVP leg of the CPU baseline)."""
    return bool(_load_ossl().ossl_available())


def ossl_batch(rows, arena, desc, open_, threads=1):
    """OpenSSL EVP seal (open_=False) or open of `desc` in place on the host copy `arena`, with
    the same composites as the batch API (ossl_baseline.c); returns per-packet status or None when
    libcrypto.so.3 is absent."""
    arr, nr = _rows(rows)
    n = len(desc)
    status = np.zeros(n, dtype=np.uint8)
    rc = _load_ossl().ossl_batch(arr, ctypes.c_uint32(nr), _p(arena), ctypes.c_uint64(arena.size), _p(desc),
                                 ctypes.c_uint32(n), _p(status), ctypes.c_int(threads), ctypes.c_int(1 if open_ else 0))
    return None if rc != 0 else status
