"""The C-ABI library (no GPU needed): it loads, exports every symbol include/mq_aead.h declares,
its host-side key schedule matches RFC 9001 A.1 / A.5 and the oracle, and packet transforms
fail loudly (MQ_ERR_NO_DEVICE) instead of falling back to a CPU path when no GPU is present."""
import ctypes
import re
import subprocess

import pytest

from milli_quic_amd import _lib, key_schedule, packet


def header_functions():
    text = open(_lib.HEADER_PATH).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mq_[a-z0-9_]+)\s*\(", text)))


def test_header_matches_bindings():
    assert set(header_functions()) == set(_lib.SIGNATURES)


def test_library_exports_every_symbol(mqlib):
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (mq_[a-z0-9_]+)$", out, flags=re.M))
    missing = set(header_functions()) - exported
    assert not missing, missing
    for name in header_functions():
        assert hasattr(mqlib, name)


def test_struct_layouts():
    assert ctypes.sizeof(_lib.PktDesc) == 32 and ctypes.sizeof(_lib.KeyMaterial) == 88
    from milli_quic_amd.batch import DESC_DTYPE
    assert DESC_DTYPE.itemsize == 32
    for f in ("offset", "len", "key_id", "pn", "pn_offset", "pn_len", "flags"):
        assert DESC_DTYPE.fields[f][1] == getattr(_lib.PktDesc, f).offset


def test_host_key_schedule_rfc9001(mqlib, ref_fixtures, orc):
    a1 = ref_fixtures["rfc9001"]["a1"]
    c, s = key_schedule.derive_initial_secrets(bytes.fromhex(ref_fixtures["rfc9001"]["dcid"]))
    assert c.hex() == a1["client_initial_secret"] and s.hex() == a1["server_initial_secret"]
    k, iv, hp = key_schedule.derive_packet_keys(s, 16)
    assert (k.hex(), iv.hex(), hp.hex()) == (a1["server_key"], a1["server_iv"], a1["server_hp"])
    km = key_schedule.key_material(_lib.MQ_SUITE_CHACHA20, bytes.fromhex(ref_fixtures["rfc9001"]["a5"]["secret"]))
    assert bytes(km.key).hex() == "c6d98ff3441c3fe1b2182094f69caa2ed4b716b65488960a7a984979fb23e1c8"
    assert bytes(km.iv).hex() == "e0459b3474bdd0e44a41c144"
    assert bytes(km.hp).hex() == "25a282b9e82f06f21f488917a4fc8f1b73573685608597d0efcb076b0ab7a7a4"
    nxt = key_schedule.derive_next_application_secret(bytes.fromhex(ref_fixtures["rfc9001"]["a5"]["secret"]))
    assert nxt.hex() == "1223504755036d556342ee9361d253421a826c9ecdf3c7148684b36b714881f9"
    for label in (b"quic key", b"tls13x", b"", b"client in"):
        for ln in (1, 12, 16, 32, 48):
            assert key_schedule.hkdf_expand_label(c, label, b"ctx", ln) == orc.hkdf_expand_label(c, label, b"ctx", ln)[1]
    with pytest.raises(Exception):
        key_schedule.hkdf_expand_label(c, b"y" * 80, b"", 16)


def test_nonce(mqlib):
    from milli_quic_amd import crypto
    # RFC 9001 A.5: iv e0459b3474bdd0e44a41c144, pn 654360564 -> nonce e0459b3474bdd0e46d417eb0
    assert crypto.nonce(bytes.fromhex("e0459b3474bdd0e44a41c144"), 654360564).hex() == "e0459b3474bdd0e46d417eb0"


def test_pn_helpers(orc):
    import numpy as np
    rng = np.random.default_rng(1)
    for _ in range(2000):
        la = int(rng.integers(0, 1 << 40))
        full = la + int(rng.integers(0, 1 << 26))
        assert packet.pn_length(full, la) == orc.pn_length(full, la)
        enc = packet.encode_pn(full, la)
        assert packet.decode_pn(int.from_bytes(enc, "big"), len(enc), full - 1) == full
    hdr, off = packet.initial_header(bytes.fromhex("8394c8f03e515708"), b"", b"", 4, 1182)
    assert (hdr + (2).to_bytes(4, "big")).hex() == "c300000001088394c8f03e5157080000449e00000002"  # RFC 9001 A.2


def test_no_cpu_fallback_without_gpu(mqlib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    h = ctypes.c_void_p()
    rc = mqlib.mq_aead_new(_lib.MQ_SUITE_CHACHA20, bytes(32), 32, ctypes.byref(h))
    assert rc == _lib.MQ_ERR_NO_DEVICE
    from milli_quic_amd import crypto
    with pytest.raises(crypto.DeviceError):
        crypto.ChaCha20Provider().aead(bytes(32))


def test_flat_chacha_kernel_choice(mqlib):
    # a flat ChaCha20 batch picks its kernel family from the bytes per packet —
    # the caller's MQ_BATCH_LEN_HINT, else arena_len / n. A sub-range batch over a large arena
    # (bench.py --e2e chunks, ring buffers) with the hint gets the kernel of the same packets in a
    # tight arena; without it, the arena's size misleads the choice (the r05 e2e runs: config B's
    # 1200-B packets on the 20-KiB kernel).
    kind = mqlib.mq_debug_chacha_flat_kind
    C = _lib.MQ_SUITE_CHACHA20
    n_all, n_chunk = 1 << 20, 1 << 15
    tight = kind(1200 * n_chunk, n_chunk, C)
    assert tight == 1                                        # 10-KiB octet images (config B)
    assert kind(1200 * n_all, n_chunk, C) == 3               # the misled choice
    assert kind(1200 * n_all, n_chunk, C | _lib.MQ_BATCH_LEN_HINT(1200)) == tight
    for L, want in ((64, 0), (640, 0), (641, 1), (1216, 1), (1217, 2), (1584, 2), (1585, 3), (65535, 3), (1 << 20, 3)):
        assert kind(L * 1000, 1000, C) == want, L
        assert kind(1 << 40, 1000, C | _lib.MQ_BATCH_LEN_HINT(L)) == want, L
    assert kind(0, 0, C) == -1


def test_flat_aes_kernel_choice(mqlib):
    # r06: flat single-key AES-128-GCM batches run 2 lanes per packet up to 400 B per packet, 4 up
    # to 1536 B, else 8; MQ_AES_NARROW 0 / 1 / 2 forces 8 / 4 / 2
    kind = mqlib.mq_debug_aes_flat_kind
    A = _lib.MQ_SUITE_AES128GCM
    for L, want in ((21, 2), (64, 2), (400, 2), (401, 4), (1200, 4), (1536, 4), (1537, 8), (1 << 20, 8)):
        assert kind(L * 1000, 1000, A) == want, L
        assert kind(1 << 40, 1000, A | _lib.MQ_BATCH_LEN_HINT(L)) == want, L
    with _lib.option("MQ_AES_NARROW", 1):
        assert kind(4000 * 1000, 1000, A) == 4
    with _lib.option("MQ_AES_NARROW", 2):
        assert kind(4000 * 1000, 1000, A) == 2
    with _lib.option("MQ_AES_NARROW", 0):
        assert kind(64 * 1000, 1000, A) == 8
    assert kind(64 * 1000, 1000, A) == 2
    assert kind(0, 0, A) == -1


def test_debug_options(mqlib):
    # diagnostic switches: set, read back, unset; unknown names refused; a batch never reads the
    # environment on its hot path (mq_opts.h)
    assert mqlib.mq_debug_option_get(b"MQ_NO_SUCH") == -2
    assert mqlib.mq_debug_option(b"MQ_NO_SUCH", 1) == _lib.MQ_ERR_INVALID_ARG
    old = mqlib.mq_debug_option_get(b"MQ_RECV_SEG")
    with _lib.option("MQ_RECV_SEG", 256):
        assert mqlib.mq_debug_option_get(b"MQ_RECV_SEG") == 256
        with _lib.option("MQ_RECV_SEG", None):
            assert mqlib.mq_debug_option_get(b"MQ_RECV_SEG") == -1
        assert mqlib.mq_debug_option_get(b"MQ_RECV_SEG") == 256
    assert mqlib.mq_debug_option_get(b"MQ_RECV_SEG") == old
