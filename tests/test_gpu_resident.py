"""The resident per-packet path (mq_resident.hip): Aead::seal_in_place /
open_in_place and HeaderProtection::mask served by one resident wave per device polling a mailbox,
no kernel launch per call (reference call sites transmit.rs:713-718, recv.rs:416-421,
rustcrypto.rs:38-220). Bit-exact against the oracle and the golden vectors over sizes from an
empty payload to a 16-KiB TLS record, AAD from 0 to 300 B, tampering (Error::Crypto, buffer
untouched), the exit / relaunch handshake after idling, threads sharing the server, and equal to
the launch path (MQ_RESIDENT=0) call for call."""
import os
import threading
import time

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from milli_quic_amd import _lib, crypto  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _device(mqlib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert mqlib.mq_device_init(0) == 0
    os.environ.pop("MQ_RESIDENT", None)
    yield
    os.environ.pop("MQ_RESIDENT", None)


def provider(suite):
    return crypto.Aes128GcmProvider() if suite == _lib.MQ_SUITE_AES128GCM else crypto.ChaCha20Provider()


SUITES = [(_lib.MQ_SUITE_CHACHA20, 32), (_lib.MQ_SUITE_AES128GCM, 16)]


@pytest.mark.parametrize("suite,klen", SUITES)
def test_resident_sizes_vs_oracle(orc, suite, klen):
    rng = np.random.default_rng(suite)
    key = rng.bytes(klen)
    aead = provider(suite).aead(key)
    for P in (0, 1, 15, 16, 17, 63, 64, 65, 127, 1023, 1024, 1171, 1350, 4000, 16384):
        for A in (0, 5, 13, 64, 300):
            nonce, aad, pt = rng.bytes(12), rng.bytes(A), rng.bytes(P)
            rc, want, _ = orc.aead_seal(suite, key, nonce, aad, pt)
            assert rc == 0
            buf = bytearray(pt) + bytearray(16)
            assert aead.seal_in_place(nonce, aad, buf, P) == P + 16
            assert bytes(buf) == want, (suite, P, A)
            assert aead.open_in_place(nonce, aad, buf, P + 16) == P
            assert bytes(buf[:P]) == pt
            # tampered tag / ciphertext / AAD: Error::Crypto and the buffer left as it was
            sealed = bytearray(want)
            for where in ("tag", "ct", "aad"):
                b = bytearray(sealed)
                a = bytearray(aad)
                if where == "tag":
                    b[P] ^= 1
                elif where == "ct" and P:
                    b[P // 2] ^= 0x80
                elif where == "aad" and A:
                    a[A - 1] ^= 4
                else:
                    continue
                before = bytes(b)
                with pytest.raises(crypto.CryptoError):
                    aead.open_in_place(nonce, bytes(a), b, P + 16)
                assert bytes(b) == before


def test_resident_vectors_and_launch_path_agree(aead_vectors, hp_vectors):
    for mode in ("1", "0", "1"):
        os.environ["MQ_RESIDENT"] = mode
        for c in aead_vectors:
            key, nonce, aad, pt = (bytes.fromhex(c[k]) for k in ("key", "nonce", "aad", "pt"))
            aead = provider(c["suite"]).aead(key)
            buf = bytearray(pt) + bytearray(16)
            aead.seal_in_place(nonce, aad, buf, len(pt))
            assert bytes(buf).hex() == c["ct_tag"], (mode, c["suite"], len(pt))
            assert aead.open_in_place(nonce, aad, buf, len(buf)) == len(pt) and bytes(buf[:len(pt)]) == pt
        for c in hp_vectors:
            hp = provider(c["suite"]).header_protection(bytes.fromhex(c["hp"]))
            assert hp.mask(bytes.fromhex(c["sample"])).hex() == c["mask"], (mode, c)
    os.environ.pop("MQ_RESIDENT", None)


def test_resident_relaunch_after_idle(orc):
    # the resident wave leaves after 2 ms without a call; the next call relaunches it
    key = bytes(range(32))
    aead = crypto.ChaCha20Provider().aead(key)
    for k in range(6):
        nonce, pt = bytes([k]) * 12, bytes(range(200))
        buf = bytearray(pt) + bytearray(16)
        aead.seal_in_place(nonce, b"hdr", buf, len(pt))
        assert bytes(buf) == orc.aead_seal(2, key, nonce, b"hdr", pt)[1]
        time.sleep(0.001 * (k % 3) * 5)  # 0, 5, 10 ms: some calls find the kernel gone
    torch.cuda.synchronize()  # the resident kernel has left by itself


def test_resident_threads(orc):
    # several host threads share the device's resident server (calls serialise on its mailbox)
    errors = []

    def work(t):
        try:
            suite, klen = SUITES[t % 2]
            key = bytes((t * 7 + i) & 0xFF for i in range(klen))
            aead = provider(suite).aead(key)
            rng = np.random.default_rng(t)
            for k in range(150):
                nonce, aad, pt = rng.bytes(12), rng.bytes(13), rng.bytes(int(rng.integers(0, 1400)))
                buf = bytearray(pt) + bytearray(16)
                aead.seal_in_place(nonce, aad, buf, len(pt))
                if bytes(buf) != orc.aead_seal(suite, key, nonce, aad, pt)[1]:
                    errors.append((t, k))
                aead.open_in_place(nonce, aad, buf, len(buf))
                if bytes(buf[:len(pt)]) != pt:
                    errors.append((t, k, "open"))
        except Exception as e:  # noqa: BLE001
            errors.append((t, repr(e)))

    th = [threading.Thread(target=work, args=(t,)) for t in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors[:5]
