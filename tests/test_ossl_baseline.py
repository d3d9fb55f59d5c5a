"""The OpenSSL EVP leg of bench.py's CPU baseline (oracle/ossl_baseline.c) computes the same
composites as the C oracle: sealed bytes, statuses and the round trip agree on samples of
configs B, C and E (short and long headers, both suites, per-connection Initial keys). CPU only;
skipped when libcrypto.so.3 is absent."""
import numpy as np
import pytest

from milli_quic_amd import workload


@pytest.mark.parametrize("cfg,n", [("b", 512), ("c", 512), ("e", 2048)])
def test_openssl_leg_matches_oracle(orc, cfg, n):
    if not orc.ossl_available():
        pytest.skip("libcrypto.so.3 not loadable")
    w = {"b": workload.config_b, "c": workload.config_c, "e": workload.config_e}[cfg](n)
    a_orc, a_ssl = w.arena.copy(), w.arena.copy()
    st_o = orc.batch_seal(w.keys, a_orc, w.seal_desc, w.suite_hint, 2)
    st_s = orc.ossl_batch(w.keys, a_ssl, w.seal_desc, False, 2)
    assert (st_o == 0).all() and (st_s == 0).all()
    assert a_orc.tobytes() == a_ssl.tobytes()
    st_s = orc.ossl_batch(w.keys, a_ssl, w.open_desc, True, 2)
    st_o, _ = orc.batch_open(w.keys, a_orc, w.open_desc, w.suite_hint, 2)
    assert (st_s == 0).all() and (st_o == 0).all()
    assert a_ssl.tobytes() == a_orc.tobytes()  # same plaintext, headers unmasked the same way


def test_openssl_leg_rejects_tamper(orc):
    if not orc.ossl_available():
        pytest.skip("libcrypto.so.3 not loadable")
    w = workload.config_b(16)
    a = w.arena.copy()
    orc.ossl_batch(w.keys, a, w.seal_desc, False, 1)
    off = int(w.seal_desc["offset"][3]) + 40
    a[off] ^= 1
    st = orc.ossl_batch(w.keys, a, w.open_desc, True, 1)
    assert st[3] != 0 and (np.delete(st, 3) == 0).all()
