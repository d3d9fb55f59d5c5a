"""Config A (BASELINE configs[0]): 4096 x 1200-B ChaCha20-Poly1305 seal+open on the host CPU —
the reference's CPU-runnable plumbing case. The reference's Rust src/crypto cannot be built here
(SURVEY §8c), so its stand-ins run it: the C oracle's batch composites (transmit.rs:625-755 /
recv.rs:340-421) and, where libcrypto is present, OpenSSL EVP. The batch result is pinned packet
by packet to the oracle's per-packet Aead::seal_in_place and HeaderProtection::mask
(rustcrypto.rs:111-135, 197-220; themselves pinned to RFC 8439 / RFC 9001 A.5 in
test_oracle_golden.py), and the GPU test runs the same batch through the C ABI."""
import numpy as np
import pytest

from milli_quic_amd import _lib, workload

N_A, L_A = 4096, 1200


def _config_a():
    return workload.config_b(N_A)


def _km(w):
    k = w.keys[0]
    return bytes(k.key)[:32], bytes(k.iv)[:12], bytes(k.hp)[:32]


def test_config_a_batch_matches_per_packet_calls(orc):
    w = _config_a()
    key, iv, hp = _km(w)
    sealed = w.arena.copy()
    st = orc.batch_seal(w.keys, sealed, w.seal_desc, w.suite_hint, threads=4)
    assert (st == 0).all()
    hdr = 1 + 8 + 4  # short header: first byte, 8-B DCID, 4-B PN (SURVEY §8 conventions)
    for i in list(range(0, N_A, 97)) + [N_A - 1]:
        o = int(w.seal_desc["offset"][i])
        pn = int(w.pns[i])
        nonce = bytes(a ^ b for a, b in zip(iv, b"\0" * 4 + pn.to_bytes(8, "big")))  # mod.rs:66-74
        aad = w.arena[o:o + hdr].tobytes()
        pt = w.arena[o + hdr:o + L_A - 16].tobytes()
        rc, ct, _ = orc.aead_seal(_lib.MQ_SUITE_CHACHA20, key, nonce, aad, pt)
        assert rc == 0 and sealed[o + hdr:o + L_A].tobytes() == ct
        smp = sealed[o + 9 + 4:o + 9 + 20].tobytes()  # sample at pn_offset + 4 (RFC 9001 §5.4.2)
        rc, mask = orc.hp_mask(_lib.MQ_SUITE_CHACHA20, hp, smp)
        assert rc == 0
        assert sealed[o] == aad[0] ^ (mask[0] & 0x1F)
        assert sealed[o + 9:o + 13].tobytes() == bytes(a ^ b for a, b in zip(aad[9:13], mask[1:5]))


def test_config_a_round_trip(orc):
    w = _config_a()
    a = w.arena.copy()
    assert (orc.batch_seal(w.keys, a, w.seal_desc, w.suite_hint, threads=4) == 0).all()
    tags = a.reshape(N_A, L_A)[:, L_A - 16:].copy()
    st, pn = orc.batch_open(w.keys, a, w.open_desc, w.suite_hint, threads=4)
    assert (st == 0).all() and (pn == w.pns).all()
    v, v0 = a.reshape(N_A, L_A), w.arena.reshape(N_A, L_A)
    assert v[:, :L_A - 16].tobytes() == v0[:, :L_A - 16].tobytes()  # header and plaintext restored
    assert v[:, L_A - 16:].tobytes() == tags.tobytes()  # open leaves the tag in place


def test_config_a_openssl_agrees(orc):
    if not orc.ossl_available():
        pytest.skip("libcrypto.so.3 not loadable")
    w = _config_a()
    a_orc, a_ssl = w.arena.copy(), w.arena.copy()
    assert (orc.batch_seal(w.keys, a_orc, w.seal_desc, w.suite_hint, threads=4) == 0).all()
    assert (orc.ossl_batch(w.keys, a_ssl, w.seal_desc, False, 4) == 0).all()
    assert a_orc.tobytes() == a_ssl.tobytes()


@pytest.mark.gpu
def test_config_a_on_gpu_vs_oracle(orc):
    import torch
    from milli_quic_amd import batch
    from milli_quic_amd.batch import KeyTable
    w = _config_a()
    dev = torch.device("cuda", 0)
    kt = KeyTable(w.keys)
    arena = torch.from_numpy(w.arena.copy()).to(dev)
    sd = torch.from_numpy(w.seal_desc.view(np.uint8)).to(dev)
    od = torch.from_numpy(w.open_desc.view(np.uint8)).to(dev)
    st = torch.full((N_A,), 0xEE, dtype=torch.uint8, device=dev)
    pn = torch.zeros(N_A, dtype=torch.int64, device=dev)
    ws = torch.empty(batch.workspace_bytes(N_A), dtype=torch.uint8, device=dev)
    batch.seal(kt, arena, sd, st, w.suite_hint, ws)
    torch.cuda.synchronize()
    ref = w.arena.copy()
    assert (orc.batch_seal(w.keys, ref, w.seal_desc, w.suite_hint, threads=4) == 0).all()
    assert (st.cpu().numpy() == 0).all()
    assert arena.cpu().numpy().tobytes() == ref.tobytes()
    batch.open_(kt, arena, od, st, pn, w.suite_hint, ws)
    torch.cuda.synchronize()
    st_o, pn_o = orc.batch_open(w.keys, ref, w.open_desc, w.suite_hint, threads=4)
    assert (st.cpu().numpy() == 0).all() and (st_o == 0).all()
    assert (pn.cpu().numpy().view(np.uint64) == pn_o).all()
    assert arena.cpu().numpy().tobytes() == ref.tobytes()
