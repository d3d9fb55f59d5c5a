"""Host-side mirror of the reference's crypto trait surface, bound to the HIP kernels.

Reference (computer-whisperer/milli-quic):
  * ``trait Aead``             src/crypto/aead.rs:8-42
  * ``trait HeaderProtection`` src/crypto/header_protection.rs:6-13
  * ``trait Hkdf``             src/crypto/hkdf.rs:7-16
  * ``trait CryptoProvider``   src/crypto/mod.rs:38-51
  * ``DirectionalKeys``        src/crypto/mod.rs:54-75
  * RustCrypto adapters        src/crypto/rustcrypto.rs:9-287

Same names, argument meaning and error behaviour: ``Error::Crypto`` -> :class:`CryptoError`,
``Error::BufferTooSmall { needed }`` -> :class:`BufferTooSmall` (``.needed``); the reference's
panics (slice index out of range) -> :class:`InvalidArgument`. seal/open run on the GPU through
``libmq_aead.so`` (a batch of one); HKDF runs on the host, as in the reference (once per
connection, not per packet).
"""
import ctypes

from . import _lib
from ._lib import MQ_SUITE_AES128GCM, MQ_SUITE_CHACHA20


class Error(Exception):
    """crate::error::Error (src/error.rs:144-170), restricted to what this path raises."""


class CryptoError(Error):
    """Error::Crypto"""


class BufferTooSmall(Error):
    """Error::BufferTooSmall { needed }"""

    def __init__(self, needed):
        super().__init__(f"buffer too small, needed {needed}")
        self.needed = needed


class ProtocolViolation(Error):
    """Error::Transport(TransportError::ProtocolViolation)"""


class TlsError(Error):
    """Error::Tls (a TLS record without a valid inner content type, tcp_tls/connection.rs:546-556)"""


class InvalidArgument(Error):
    """Cases where the reference panics (index out of range) or a NULL argument."""


class DeviceError(Error):
    """No gfx950 device / HIP runtime failure (the library has no CPU fallback)."""


def _raise(rc, needed=None):
    if rc == _lib.MQ_OK:
        return
    if rc == _lib.MQ_ERR_CRYPTO:
        raise CryptoError("crypto")
    if rc == _lib.MQ_ERR_BUFFER_TOO_SMALL:
        raise BufferTooSmall(needed)
    if rc == _lib.MQ_ERR_PROTOCOL:
        raise ProtocolViolation("packet number exceeds 2^62-1")
    if rc == _lib.MQ_ERR_TLS:
        raise TlsError("no valid inner content type")
    if rc in (_lib.MQ_ERR_INVALID_ARG, _lib.MQ_ERR_SUITE):
        raise InvalidArgument(_lib.status_str(rc))
    raise DeviceError(_lib.status_str(rc))


class Aead:
    """trait Aead (src/crypto/aead.rs:8-42)."""

    KEY_LEN = 0
    NONCE_LEN = 12
    TAG_LEN = 16
    SUITE = 0

    def __init__(self, key):
        lib = _lib.load()
        key = bytes(key)
        h = ctypes.c_void_p()
        _raise(lib.mq_aead_new(self.SUITE, key, len(key), ctypes.byref(h)))
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            _lib.load().mq_aead_free(h)
            self._h = None

    def seal_in_place(self, nonce, aad, buf, payload_len):
        """Encrypt buf[:payload_len] in place and append the tag; returns payload_len + 16."""
        lib = _lib.load()
        nonce, aad = bytes(nonce), bytes(aad)
        out, needed = ctypes.c_size_t(), ctypes.c_size_t()
        rc = lib.mq_aead_seal_in_place(self._h, nonce, len(nonce), aad, len(aad), _lib.buf_ptr(buf),
                                       len(buf), payload_len, ctypes.byref(out), ctypes.byref(needed))
        _raise(rc, needed.value)
        return out.value

    def open_in_place(self, nonce, aad, buf, ciphertext_len):
        """Verify and decrypt buf[:ciphertext_len] in place; returns the plaintext length."""
        lib = _lib.load()
        nonce, aad = bytes(nonce), bytes(aad)
        out = ctypes.c_size_t()
        rc = lib.mq_aead_open_in_place(self._h, nonce, len(nonce), aad, len(aad), _lib.buf_ptr(buf),
                                       len(buf), ciphertext_len, ctypes.byref(out))
        _raise(rc)
        return out.value


class Aes128GcmAead(Aead):
    """rustcrypto.rs:27-95"""

    KEY_LEN = 16
    SUITE = MQ_SUITE_AES128GCM


class ChaCha20Poly1305Aead(Aead):
    """rustcrypto.rs:97-166"""

    KEY_LEN = 32
    SUITE = MQ_SUITE_CHACHA20


class HeaderProtection:
    """trait HeaderProtection (src/crypto/header_protection.rs:6-13)."""

    SUITE = 0
    KEY_LEN = 0

    def __init__(self, key):
        lib = _lib.load()
        key = bytes(key)
        h = ctypes.c_void_p()
        _raise(lib.mq_hp_new(self.SUITE, key, len(key), ctypes.byref(h)))
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            _lib.load().mq_hp_free(h)
            self._h = None

    def mask(self, sample):
        """5-byte mask from a 16-byte sample (shorter samples panic in the reference)."""
        sample = bytes(sample)
        m = (ctypes.c_uint8 * 5)()
        _raise(_lib.load().mq_hp_mask(self._h, sample, len(sample), m))
        return bytes(m)


class AesHeaderProtection(HeaderProtection):
    """rustcrypto.rs:168-186"""

    SUITE = MQ_SUITE_AES128GCM
    KEY_LEN = 16


class ChaChaHeaderProtection(HeaderProtection):
    """rustcrypto.rs:188-220"""

    SUITE = MQ_SUITE_CHACHA20
    KEY_LEN = 32


class HkdfSha256:
    """Hkdf trait impl (rustcrypto.rs:9-24; trait src/crypto/hkdf.rs:7-16)."""

    HASH_LEN = 32

    def extract(self, salt, ikm):
        salt, ikm = bytes(salt), bytes(ikm)
        prk = (ctypes.c_uint8 * 32)()
        _lib.load().mq_hkdf_extract(salt, len(salt), ikm, len(ikm), prk)
        return bytes(prk)

    def expand(self, prk, info, length):
        prk, info = bytes(prk), bytes(info)
        out = (ctypes.c_uint8 * max(length, 1))()
        _raise(_lib.load().mq_hkdf_expand(prk, len(prk), info, len(info), out, length))
        return bytes(out)[:length]


class CryptoProvider:
    """trait CryptoProvider (src/crypto/mod.rs:38-51)."""

    Aead = Aead
    HeaderProtection = HeaderProtection
    SUITE = 0

    def aead(self, key):
        if len(key) != self.Aead.KEY_LEN:  # rustcrypto.rs:234-236, 267-269
            raise CryptoError("bad key length")
        return self.Aead(key)

    def hkdf(self):
        return HkdfSha256()

    def header_protection(self, key):
        if len(key) != self.HeaderProtection.KEY_LEN:  # rustcrypto.rs:247-249, 280-282
            raise CryptoError("bad hp key length")
        return self.HeaderProtection(key)


class Aes128GcmProvider(CryptoProvider):
    """rustcrypto.rs:225-253"""

    Aead = Aes128GcmAead
    HeaderProtection = AesHeaderProtection
    SUITE = MQ_SUITE_AES128GCM


class ChaCha20Provider(CryptoProvider):
    """rustcrypto.rs:255-287"""

    Aead = ChaCha20Poly1305Aead
    HeaderProtection = ChaChaHeaderProtection
    SUITE = MQ_SUITE_CHACHA20


def nonce(iv, packet_number):
    """DirectionalKeys::nonce (src/crypto/mod.rs:66-74), via the C ABI."""
    iv = bytes(iv)
    if len(iv) != 12:
        raise InvalidArgument("iv must be 12 bytes")
    out = (ctypes.c_uint8 * 12)()
    _lib.load().mq_nonce(iv, packet_number, out)
    return bytes(out)


class DirectionalKeys:
    """src/crypto/mod.rs:54-75: AEAD + header protection + IV for one direction/level."""

    def __init__(self, aead, header_protection, iv):
        self.aead = aead
        self.header_protection = header_protection
        self.iv = bytes(iv)

    def nonce(self, packet_number):
        return nonce(self.iv, packet_number)
