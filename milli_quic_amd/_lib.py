"""ctypes binding of libmq_aead.so (C ABI declared in include/mq_aead.h).

The shared library is built in-tree by ``__graft_entry__.build()`` (milli_quic_amd/csrc/Makefile)
and is the only compute path: there is no Python or CPU fallback. ``load()`` raises if the
library is missing, and every packet transform returns ``MQ_ERR_NO_DEVICE`` without a gfx950.
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# MQ_ASAN=1 (tools/asan_cpu_tests.sh, CPU only): the build whose host code carries AddressSanitizer +
# UBSan (`make -C milli_quic_amd/csrc asan`); the kernels are the same
LIB_PATH = os.path.join(_HERE, "asan" if os.environ.get("MQ_ASAN") == "1" else "", "libmq_aead.so")
# diagnostic A/B of library builds (tools/ab_libs/*.so, tools/runs/gpu_r0*.sh); never set by the product
if os.environ.get("MQ_LIB"):
    LIB_PATH = os.environ["MQ_LIB"]
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "mq_aead.h")

MQ_OK = 0
MQ_ERR_CRYPTO = 1
MQ_ERR_BUFFER_TOO_SMALL = 2
MQ_ERR_INVALID_ARG = 3
MQ_ERR_PROTOCOL = 4
MQ_ERR_SUITE = 5
MQ_ERR_NO_DEVICE = 6
MQ_ERR_HIP = 7
MQ_ERR_TLS = 8
MQ_ERR_DEFERRED = 9

MQ_SUITE_AES128GCM = 1
MQ_SUITE_CHACHA20 = 2
MQ_SUITE_MIXED = 0xFF


def MQ_BATCH_LEN_HINT(length):
    """suite_hint bits: the batch's typical packet length (include/mq_aead.h)."""
    return min(int(length), 0xFFFF) << 16

MQ_PKT_LONG_HEADER = 0x01
MQ_PKT_NO_HP = 0x02
MQ_PKT_TLS_RECORD = 0x06  # implies MQ_PKT_NO_HP
MQ_PKT_NO_RECV_LIMIT = 0x08  # open: lift the reference's 2048-B receive limit (recv.rs:356-360)
MQ_RECV_MAX_PACKET = 2048

MQ_LEVEL_INITIAL, MQ_LEVEL_HANDSHAKE, MQ_LEVEL_APPLICATION = 0, 1, 2
MQ_SEND_PAD_TO_MIN = 0x01


class KeyMaterial(ctypes.Structure):
    """mq_key_material: what CryptoProvider::aead + ::header_protection consume."""

    _fields_ = [
        ("suite", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32),
        ("key", ctypes.c_uint8 * 32),
        ("iv", ctypes.c_uint8 * 12),
        ("pad", ctypes.c_uint8 * 4),
        ("hp", ctypes.c_uint8 * 32),
    ]


class PktDesc(ctypes.Structure):
    """mq_pkt_desc: one packet of a device batch (32 bytes)."""

    _fields_ = [
        ("offset", ctypes.c_uint64),
        ("len", ctypes.c_uint32),
        ("key_id", ctypes.c_uint32),
        ("pn", ctypes.c_uint64),
        ("pn_offset", ctypes.c_uint16),
        ("pn_len", ctypes.c_uint8),
        ("flags", ctypes.c_uint8),
        ("reserved", ctypes.c_uint32),
    ]


assert ctypes.sizeof(KeyMaterial) == 88
assert ctypes.sizeof(PktDesc) == 32

_u8p = ctypes.POINTER(ctypes.c_uint8)
_vp = ctypes.c_void_p
_sz = ctypes.c_size_t
_u32 = ctypes.c_uint32
_u64 = ctypes.c_uint64

# name -> (restype, argtypes); every function declared in include/mq_aead.h
SIGNATURES = {
    "mq_version": (ctypes.c_char_p, []),
    "mq_device_init": (ctypes.c_int, [ctypes.c_int]),
    "mq_device_current": (ctypes.c_int, []),
    "mq_keytable_device": (ctypes.c_int, [_vp]),
    "mq_stream_release": (None, [_vp]),
    "mq_resident_phases": (ctypes.c_int, [ctypes.c_int, _vp, ctypes.c_int]),
    "mq_status_str": (ctypes.c_char_p, [ctypes.c_int]),
    "mq_debug_option": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_long]),
    "mq_debug_option_get": (ctypes.c_long, [ctypes.c_char_p]),
    "mq_debug_chacha_flat_kind": (ctypes.c_int, [_u64, _u32, _u32]),
    "mq_debug_aes_flat_kind": (ctypes.c_int, [_u64, _u32, _u32]),
    "mq_aead_new": (ctypes.c_int, [_u32, _vp, _sz, ctypes.POINTER(_vp)]),
    "mq_aead_free": (None, [_vp]),
    "mq_aead_key_len": (_sz, [_u32]),
    "mq_aead_seal_in_place": (ctypes.c_int, [_vp, _vp, _sz, _vp, _sz, _vp, _sz, _sz,
                                             ctypes.POINTER(_sz), ctypes.POINTER(_sz)]),
    "mq_aead_open_in_place": (ctypes.c_int, [_vp, _vp, _sz, _vp, _sz, _vp, _sz, _sz,
                                             ctypes.POINTER(_sz)]),
    "mq_hp_new": (ctypes.c_int, [_u32, _vp, _sz, ctypes.POINTER(_vp)]),
    "mq_hp_free": (None, [_vp]),
    "mq_hp_mask": (ctypes.c_int, [_vp, _vp, _sz, _vp]),
    "mq_nonce": (None, [_vp, _u64, _vp]),
    "mq_hkdf_extract": (None, [_vp, _sz, _vp, _sz, _vp]),
    "mq_hkdf_expand": (ctypes.c_int, [_vp, _sz, _vp, _sz, _vp, _sz]),
    "mq_hkdf_expand_label": (ctypes.c_int, [_vp, _sz, _vp, _sz, _vp, _sz, _vp, _sz]),
    "mq_derive_initial_secrets": (ctypes.c_int, [_vp, _sz, _vp, _vp]),
    "mq_derive_key_material": (ctypes.c_int, [_u32, _vp, _sz, ctypes.POINTER(KeyMaterial)]),
    "mq_derive_next_secret": (ctypes.c_int, [_vp, _sz, _vp]),
    "mq_batch_derive_initial": (ctypes.c_int, [_vp, _u32, _vp, _vp, _u32, _vp, _vp, _vp]),
    "mq_batch_protect_workspace_size": (_sz, [_u32]),
    "mq_batch_protect": (ctypes.c_int, [_vp, _vp, _u32, _vp, _u64, _vp, _u64, _vp, _u32, _vp, _vp, _u32, _vp, _vp]),
    "mq_batch_recv_workspace_size": (_sz, [_u32, _u32, _u32]),
    "mq_batch_recv": (ctypes.c_int, [_vp, _vp, _u32, _vp, _u64, _vp, _u32, _vp, _u32, _vp, _vp, _vp]),
    "mq_keytable_create": (ctypes.c_int, [ctypes.POINTER(KeyMaterial), _u32, ctypes.POINTER(_vp)]),
    "mq_keytable_update": (ctypes.c_int, [_vp, _u32, ctypes.POINTER(KeyMaterial), _u32]),
    "mq_keytable_rows": (_u32, [_vp]),
    "mq_keytable_free": (None, [_vp]),
    "mq_batch_workspace_size": (_sz, [_u32]),
    "mq_batch_seal": (ctypes.c_int, [_vp, _vp, _u64, _vp, _u32, _vp, _u32, _vp, _vp]),
    "mq_batch_open": (ctypes.c_int, [_vp, _vp, _u64, _vp, _u32, _vp, _vp, _u32, _vp, _vp]),
    "mq_batch_hp_mask": (ctypes.c_int, [_vp, _vp, _vp, _vp, _u32, _vp]),
    "mq_record_seal": (ctypes.c_int, [_vp, _vp, _sz, _vp, _sz, _sz, ctypes.c_uint8, ctypes.POINTER(_sz),
                                      ctypes.POINTER(_sz)]),
    "mq_record_open": (ctypes.c_int, [_vp, _vp, _sz, _vp, _sz, _sz, _vp, ctypes.POINTER(_sz),
                                      ctypes.POINTER(ctypes.c_uint8)]),
    "mq_batch_seal_records": (ctypes.c_int, [_vp, _vp, _u64, _vp, _u32, _vp, _u32, _vp, _vp]),
    "mq_batch_open_records": (ctypes.c_int, [_vp, _vp, _u64, _vp, _u32, _vp, _vp, _u32, _vp, _vp]),
    "mq_batch_time_seal_open": (ctypes.c_int, [_vp, _vp, _u64, _vp, _u32, _vp, _vp, _u32, _vp, _vp,
                                               ctypes.c_int, ctypes.POINTER(ctypes.c_float),
                                               ctypes.POINTER(ctypes.c_float)]),
}

_lib = None
_lock = threading.Lock()


def load():
    """Load libmq_aead.so once; raise if it has not been built."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: run __graft_entry__.build() (make -C milli_quic_amd/csrc)")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


class option:
    """Context manager / setter of a diagnostic switch (mq_debug_option; None unsets it):
    ``with _lib.option("MQ_CC_NARROW", 0): ...`` restores the previous value on exit."""

    def __init__(self, name, value):
        self.name, self.value = name.encode(), -1 if value is None else int(value)
        self.old = None

    def __enter__(self):
        lib = load()
        self.old = lib.mq_debug_option_get(self.name)
        assert self.old != -2, self.name
        assert lib.mq_debug_option(self.name, self.value) == MQ_OK
        return self

    def __exit__(self, *exc):
        load().mq_debug_option(self.name, self.old)
        return False


def status_str(code):
    return load().mq_status_str(code).decode()


def buf_ptr(b):
    """Writable pointer into a bytearray / memoryview / ctypes array (no copy)."""
    if b is None:
        return None
    if isinstance(b, (bytes,)):
        return ctypes.cast(ctypes.c_char_p(b), _vp)
    return ctypes.cast((ctypes.c_char * len(b)).from_buffer(b), _vp) if len(b) else ctypes.c_void_p(0)
