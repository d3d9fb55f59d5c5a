"""QUIC v1 key schedule (RFC 9001 §5), mirroring src/crypto/key_schedule.rs.

Runs on the host through libmq_aead.so's HKDF-SHA256 (per connection / key update, never per
packet). ``key_material()`` produces the rows of a device key table.
"""
import ctypes

from . import _lib
from .crypto import CryptoError, DirectionalKeys, _raise

INITIAL_SALT_V1 = bytes.fromhex("38762cf7f55934b34d179ae6a4c80cadccbb7f0a")  # key_schedule.rs:10-13


def hkdf_expand_label(secret, label, context, length):
    """hkdf_expand_label (key_schedule.rs:23-55); Error::Crypto if the info exceeds 80 bytes."""
    secret, label, context = bytes(secret), bytes(label), bytes(context)
    out = (ctypes.c_uint8 * max(length, 1))()
    _raise(_lib.load().mq_hkdf_expand_label(secret, len(secret), label, len(label), context,
                                            len(context), out, length))
    return bytes(out)[:length]


def derive_initial_secrets(dcid):
    """derive_initial_secrets (key_schedule.rs:60-72) -> (client_secret, server_secret)."""
    dcid = bytes(dcid)
    c, s = (ctypes.c_uint8 * 32)(), (ctypes.c_uint8 * 32)()
    _raise(_lib.load().mq_derive_initial_secrets(dcid, len(dcid), c, s))
    return bytes(c), bytes(s)


def derive_packet_keys(secret, key_len, hp_len=None):
    """derive_packet_keys (key_schedule.rs:79-90) -> (key, iv, hp_key)."""
    hp_len = max(key_len, 16) if hp_len is None else hp_len
    return (hkdf_expand_label(secret, b"quic key", b"", key_len),
            hkdf_expand_label(secret, b"quic iv", b"", 12),
            hkdf_expand_label(secret, b"quic hp", b"", hp_len))


def derive_tls_record_keys(secret, key_len):
    """derive_tls_record_keys (key_schedule.rs:96-107) -> (key, iv)."""
    return hkdf_expand_label(secret, b"key", b"", key_len), hkdf_expand_label(secret, b"iv", b"", 12)


def derive_next_application_secret(current_secret):
    """derive_next_application_secret (key_schedule.rs:114-120), label "quic ku"."""
    out = (ctypes.c_uint8 * 32)()
    cur = bytes(current_secret)
    _raise(_lib.load().mq_derive_next_secret(cur, len(cur), out))
    return bytes(out)


def key_material(suite, secret):
    """derive_directional_keys' key/iv/hp (key_schedule.rs:123-151) as an mq_key_material row."""
    km = _lib.KeyMaterial()
    secret = bytes(secret)
    rc = _lib.load().mq_derive_key_material(suite, secret, len(secret), ctypes.byref(km))
    _raise(rc)
    return km


def make_key_material(suite, key, iv, hp):
    """An mq_key_material row from explicit key / iv / hp bytes."""
    km = _lib.KeyMaterial()
    km.suite = suite
    key, iv, hp = bytes(key), bytes(iv), bytes(hp)
    if len(iv) != 12 or len(key) > 32 or len(hp) > 32:
        raise CryptoError("bad key material lengths")
    ctypes.memmove(km.key, key, len(key))
    ctypes.memmove(km.iv, iv, 12)
    ctypes.memmove(km.hp, hp, len(hp))
    return km


def derive_directional_keys(provider, secret):
    """derive_directional_keys (key_schedule.rs:123-151) -> DirectionalKeys."""
    key_len = provider.Aead.KEY_LEN
    key, iv, hp = derive_packet_keys(secret, key_len, max(key_len, 16))
    return DirectionalKeys(provider.aead(key), provider.header_protection(hp), iv)
