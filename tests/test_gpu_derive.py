"""Batched Initial key derivation on the GPU: derive_initial
(reference src/connection/keys.rs:181-212) for many client DCIDs, bit-exact against the oracle's
HKDF (pinned to RFC 9001 A.1 in test_oracle_golden.py) and usable as key-table rows: packets
sealed with the device-derived rows equal the oracle's, and the reference's captured curl Initial
(src/connection/mod.rs:2210) opens with them."""
import ctypes

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from milli_quic_amd import _lib, batch, workload  # noqa: E402
from milli_quic_amd.batch import KeyTable, make_descs  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _device(mqlib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert mqlib.mq_device_init(0) == 0


def oracle_material(orc, dcid):
    c, s = orc.derive_initial_secrets(dcid)
    out = []
    for sec in (c, s):
        km = _lib.KeyMaterial()
        assert orc.load().orc_derive_key_material(ctypes.c_uint32(_lib.MQ_SUITE_AES128GCM), sec, ctypes.c_size_t(32), ctypes.byref(km)) == 0
        out.append(bytes(km))
    return out


def dcid_batch(ref_fixtures, n, seed=5):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 21, size=n).astype(np.uint8)
    dc = rng.integers(0, 256, size=(n, 20), dtype=np.uint8)
    a1 = bytes.fromhex(ref_fixtures["rfc9001"]["dcid"])
    curl = bytes.fromhex(ref_fixtures["curl_initial"]["hex"])
    curl_dcid = curl[6:6 + curl[5]]
    for i, d in ((0, a1), (1, curl_dcid)):
        lens[i] = len(d)
        dc[i, :] = 0
        dc[i, :len(d)] = np.frombuffer(d, dtype=np.uint8)
    lens[2], lens[3] = 0, 20
    return dc, lens


def run_derive(n_rows, first_row, dc, lens):
    kt = KeyTable([_lib.KeyMaterial() for _ in range(n_rows)])
    n = len(lens)
    st = torch.full((n,), 0xEE, dtype=torch.uint8, device=DEV)
    km = torch.zeros(2 * 88 * n, dtype=torch.uint8, device=DEV)
    batch.derive_initial(kt, first_row, torch.from_numpy(dc.reshape(-1).copy()).to(DEV),
                         torch.from_numpy(lens.copy()).to(DEV), st, km)
    torch.cuda.synchronize()
    return kt, st.cpu().numpy(), km.cpu().numpy().reshape(n, 2, 88)


def test_derive_matches_oracle(orc, ref_fixtures):
    n = 3000
    dc, lens = dcid_batch(ref_fixtures, n)
    _, st, km = run_derive(2 * n, 0, dc, lens)
    assert (st == 0).all()
    for i in range(n):
        want = oracle_material(orc, dc[i, :lens[i]].tobytes())
        assert km[i, 0].tobytes() == want[0] and km[i, 1].tobytes() == want[1], (i, lens[i])
    a1 = ref_fixtures["rfc9001"]["a1"]  # RFC 9001 A.1 client / server keys
    assert km[0, 0, 8:24].tobytes().hex() == a1["client_key"] and km[0, 1, 8:24].tobytes().hex() == a1["server_key"]
    assert km[0, 0, 40:52].tobytes().hex() == a1["client_iv"] and km[0, 1, 56:72].tobytes().hex() == a1["server_hp"]


def test_derived_rows_protect_like_oracle(orc, ref_fixtures):
    # rows written on the device (AES key schedules, GHASH H^1..H^8) seal and open exactly as the
    # oracle does with the oracle-derived key material; offset first_row exercises the row base
    n = 64
    dc, lens = dcid_batch(ref_fixtures, n, seed=9)
    kt, st, _ = run_derive(2 * n + 3, 3, dc, lens)
    assert (st == 0).all()
    w = workload.uniform(2 * n * 4, _lib.MQ_SUITE_AES128GCM, L=333, pn_len=2)
    sd, od = w.seal_desc.copy(), w.open_desc.copy()
    sd["key_id"] = 3 + np.arange(w.n) % (2 * n)
    od["key_id"] = sd["key_id"]
    a = torch.from_numpy(w.arena.copy()).to(DEV)
    d = torch.from_numpy(sd.view(np.uint8).copy()).to(DEV)
    s = torch.zeros(w.n, dtype=torch.uint8, device=DEV)
    batch.seal(kt, a, d, s, _lib.MQ_SUITE_AES128GCM)
    torch.cuda.synchronize()
    keys = [_lib.KeyMaterial() for _ in range(3)]
    for i in range(n):
        for m in oracle_material(orc, dc[i, :lens[i]].tobytes()):
            keys.append(_lib.KeyMaterial.from_buffer_copy(m))
    ref = w.arena.copy()
    o_st = orc.batch_seal(keys, ref, sd, _lib.MQ_SUITE_AES128GCM, threads=8)
    assert (s.cpu().numpy() == 0).all() and (o_st == 0).all()
    assert a.cpu().numpy().tobytes() == ref.tobytes()
    # the curl Initial (client keys of connection 1 = row 3 + 2) opens with the derived row
    from helpers import curl_desc_and_keys
    from milli_quic_amd import key_schedule
    data, dcid, pn_offset, length, _ = curl_desc_and_keys(None, ref_fixtures, key_schedule.derive_initial_secrets)
    arena = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).to(DEV)
    opn = make_descs([0], [pn_offset + length], [3 + 2], [0], [pn_offset], [0], [_lib.MQ_PKT_LONG_HEADER])
    st1 = torch.full((1,), 0xEE, dtype=torch.uint8, device=DEV)
    pn = torch.zeros(1, dtype=torch.int64, device=DEV)
    batch.open_(kt, arena, torch.from_numpy(opn.view(np.uint8).copy()).to(DEV), st1, pn, _lib.MQ_SUITE_AES128GCM)
    torch.cuda.synchronize()
    out = arena.cpu().numpy()
    assert int(st1[0]) == 0 and int(pn[0]) == 0 and out[pn_offset + 1] == 0x06


def test_derive_bounds(ref_fixtures):
    dc, lens = dcid_batch(ref_fixtures, 8)
    lens[4] = 21  # longer than a connection ID may be -> rejected, rows inert (suite 0)
    kt, st, _ = run_derive(16, 0, dc, lens)
    assert st[4] == _lib.MQ_ERR_INVALID_ARG and (np.delete(st, 4) == 0).all()
    with pytest.raises(Exception):  # first_row + 2n beyond the table: nothing launched
        run_derive(15, 0, dc, lens)
