"""The resident per-packet path (mq_resident.hip): Aead::seal_in_place /
open_in_place and HeaderProtection::mask served by one resident wave per device polling a mailbox,
no kernel launch per call (reference call sites transmit.rs:713-718, recv.rs:416-421,
rustcrypto.rs:38-220). Bit-exact against the oracle and the golden vectors over sizes from an
empty payload to a 16-KiB TLS record, AAD from 0 to 300 B, tampering (Error::Crypto, buffer
untouched), the exit / relaunch handshake after idling, threads sharing the server, and equal to
the launch path (MQ_RESIDENT 0) call for call."""
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
    mqlib.mq_debug_option(b"MQ_RESIDENT", -1)
    yield
    mqlib.mq_debug_option(b"MQ_RESIDENT", -1)


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
        _lib.load().mq_debug_option(b"MQ_RESIDENT", int(mode))
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
    _lib.load().mq_debug_option(b"MQ_RESIDENT", -1)


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


def _batch_c(n, stream):
    """A config-C batch on the device (single-key AES-128-GCM: the persistent single-key kernels,
    one 16-wave workgroup per CU) and its seal / open closures on `stream`."""
    from milli_quic_amd import batch, workload
    from milli_quic_amd.batch import KeyTable
    w = workload.config_c(n)
    dev = torch.device("cuda", 0)
    kt = KeyTable(w.keys)
    arena = torch.from_numpy(w.arena.copy()).to(dev)
    sd = torch.from_numpy(w.seal_desc.view(np.uint8).copy()).to(dev)
    od = torch.from_numpy(w.open_desc.view(np.uint8).copy()).to(dev)
    st = torch.zeros(w.n, dtype=torch.uint8, device=dev)
    pn = torch.zeros(w.n, dtype=torch.int64, device=dev)
    ws = torch.empty(max(batch.workspace_bytes(w.n), 256), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()

    def seal():
        batch.seal(kt, arena, sd, st, w.suite_hint, ws, stream.cuda_stream)

    def open_():
        batch.open_(kt, arena, od, st, pn, w.suite_hint, ws, stream.cuda_stream)
    return w, arena, st, seal, open_


def _plaintext_back(arena, w):
    """After seal + open every 1200-B packet holds its header and plaintext again (the tag bytes
    stay). A plain bool: pytest's diff of two 1.26-GB byte strings would run for minutes."""
    got = arena.cpu().numpy().reshape(w.n, 1200)[:, :1184]
    return bool(np.array_equal(got, w.arena.reshape(w.n, 1200)[:, :1184]))


@pytest.mark.timeout(90)
def test_resident_timeout_then_recovers(orc):
    # a call that times out must not leave the server unable to serve (r03 waited for
    # done + 1 forever) nor a kernel that writes the mailbox during the next call. The timeout is
    # forced: the server has idled out, a long AES batch holds every CU (persistent grid, one
    # 160-KiB workgroup per CU), so the relaunched server cannot be placed within 100 us. The
    # batch runs on its own stream and only that stream is synchronised (a device-wide sync would
    # also wait for the resident kernel).
    s = torch.cuda.Stream()
    w, arena, st, seal, open_ = _batch_c(1 << 20, s)
    key = bytes(range(32))
    aead = crypto.ChaCha20Provider().aead(key)
    outcomes = []
    try:
        for k in range(3):
            s.synchronize()
            time.sleep(0.05)  # the server leaves after 2 ms without a call
            for _ in range(6):
                seal()
                open_()
            _lib.load().mq_debug_option(b"MQ_RESIDENT_TIMEOUT_US", 100)
            nonce, pt = bytes([k + 1]) * 12, bytes(range(256)) * 3
            buf = bytearray(pt) + bytearray(16)
            try:
                aead.seal_in_place(nonce, b"hdr", buf, len(pt))
                outcomes.append("served")
                assert bytes(buf) == orc.aead_seal(2, key, nonce, b"hdr", pt)[1]
            except crypto.DeviceError:
                outcomes.append("timeout")
            finally:
                _lib.load().mq_debug_option(b"MQ_RESIDENT_TIMEOUT_US", -1)
            print("resident timeout test: call", k, outcomes[-1], flush=True)
            # the next calls are served, byte-exact (both while the batch may still run and after)
            for q in range(4):
                nonce, pt = bytes([k + 1, q]) * 6, bytes((q * 31 + i) & 0xFF for i in range(1000))
                buf = bytearray(pt) + bytearray(16)
                aead.seal_in_place(nonce, b"hdr2", buf, len(pt))
                assert bytes(buf) == orc.aead_seal(2, key, nonce, b"hdr2", pt)[1], (k, q)
                assert aead.open_in_place(nonce, b"hdr2", buf, len(buf)) == len(pt)
                assert bytes(buf[:len(pt)]) == pt
            s.synchronize()
    finally:
        _lib.load().mq_debug_option(b"MQ_RESIDENT_TIMEOUT_US", -1)
    assert (st.cpu().numpy() == 0).all()
    assert _plaintext_back(arena, w)  # seal + open rounds: every packet's plaintext back
    print("timeout outcomes", outcomes)
    assert "timeout" in outcomes  # the path under test ran at least once


@pytest.mark.timeout(120)
def test_batch_beside_resident_server(orc):
    # per-packet calls (the resident server holds a CU) while a config-C batch runs.
    # The persistent AES grid has one workgroup per CU; under r03's static tile stride the workgroup
    # that found its CU taken started a whole kernel late (~2x). With the dynamic schedule the batch
    # stays within 1.15x of its time without the server, and its bytes equal the oracle's.
    s = torch.cuda.Stream()
    w, arena, st, seal, open_ = _batch_c(1 << 20, s)

    def timed(k):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * k)]
        for _ in range(10):  # untimed: clocks ramp up after an idle gap (tools/clock_probe.py)
            seal()
            open_()
        for i in range(k):
            ev[2 * i].record(s)
            seal()
            open_()
            ev[2 * i + 1].record(s)
        s.synchronize()
        return float(np.median([ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(k)]))

    for _ in range(3):
        seal()
        open_()
    s.synchronize()
    time.sleep(0.05)  # no server
    alone = timed(8)
    stop, calls, errors = threading.Event(), [0], []
    key = bytes(range(16))
    aead = crypto.Aes128GcmProvider().aead(key)

    def per_packet():
        try:
            k = 0
            while not stop.is_set():
                nonce, pt = k.to_bytes(12, "big"), bytes((k + i) & 0xFF for i in range(1171))
                buf = bytearray(pt) + bytearray(16)
                aead.seal_in_place(nonce, b"h" * 13, buf, len(pt))
                if k % 50 == 0 and bytes(buf) != orc.aead_seal(1, key, nonce, b"h" * 13, pt)[1]:
                    errors.append(k)
                calls[0] += 1
                k += 1
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = threading.Thread(target=per_packet)
    th.start()
    try:
        while calls[0] < 20 and th.is_alive():
            time.sleep(0.001)
        beside = timed(8)
        print(f"config C seal+open: alone {alone:.3f} ms, beside the server {beside:.3f} ms "
              f"({beside / alone:.3f}x, {calls[0]} per-packet calls so far)", flush=True)
        seal()  # the sealed bytes under the server, checked below
        s.synchronize()
        sealed = arena.cpu().numpy().copy()
        open_()
        s.synchronize()
    finally:
        stop.set()
        th.join()
    assert not errors, errors[:3]
    assert (st.cpu().numpy() == 0).all()
    assert _plaintext_back(arena, w)
    # every 256th packet of the sealed arena against the oracle
    idx = np.arange(0, w.n, 256)
    ref = w.arena.copy()
    sd = w.seal_desc[idx].copy()
    assert (orc.batch_seal(w.keys, ref, sd, w.suite_hint) == 0).all()
    for i in idx:
        o, L = int(w.seal_desc["offset"][i]), int(w.seal_desc["len"][i])
        assert sealed[o:o + L].tobytes() == ref[o:o + L].tobytes(), i
    assert calls[0] > 20
    assert beside <= 1.15 * alone, (alone, beside)
