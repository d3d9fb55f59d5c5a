import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (runs on the MI355X box)")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def aead_vectors():
    return load_golden("aead_vectors.json")["cases"]


@pytest.fixture(scope="session")
def hp_vectors():
    return load_golden("hp_vectors.json")["cases"]


@pytest.fixture(scope="session")
def packet_vectors():
    return load_golden("packet_vectors.json")["packets"]


@pytest.fixture(scope="session")
def ref_fixtures():
    return load_golden("ref_fixtures.json")


@pytest.fixture(scope="session")
def orc():
    from oracle import oracle
    oracle.load()
    return oracle


@pytest.fixture(scope="session")
def mqlib():
    """libmq_aead.so, built in-tree if missing (hipcc cross-compiles without a GPU)."""
    from milli_quic_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        import subprocess
        subprocess.run(["make", "-C", os.path.join(ROOT, "milli_quic_amd", "csrc"), "-s", "-j8"], check=True)
    return _lib.load()
