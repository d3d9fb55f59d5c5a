"""milli_quic_amd — MI355X-native (gfx950) QUIC packet protection for milli-quic.

Drop-in for the reference's packet-protection path (src/crypto Aead / HeaderProtection /
CryptoProvider as applied by src/connection/{transmit,recv}.rs): ChaCha20-Poly1305 and
AES-128-GCM seal/open plus the header-protection mask, run as hand-written HIP kernels behind
the C ABI of include/mq_aead.h (libmq_aead.so, built in-tree).

(The directory is ``milli_quic_amd`` because a hyphenated name cannot be imported in Python.)
"""
from . import _lib  # noqa: F401
from .crypto import (Aes128GcmAead, Aes128GcmProvider, AesHeaderProtection, BufferTooSmall,  # noqa: F401
                     ChaCha20Poly1305Aead, ChaCha20Provider, ChaChaHeaderProtection, CryptoError,
                     DirectionalKeys, Error, HkdfSha256, InvalidArgument, ProtocolViolation, nonce)

__all__ = [
    "Aes128GcmAead", "Aes128GcmProvider", "AesHeaderProtection", "BufferTooSmall", "ChaCha20Poly1305Aead",
    "ChaCha20Provider", "ChaChaHeaderProtection", "CryptoError", "DirectionalKeys", "Error", "HkdfSha256",
    "InvalidArgument", "ProtocolViolation", "nonce",
]
