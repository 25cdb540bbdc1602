import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built HIP library")


@pytest.fixture(scope="session")
def golden():
    return GOLDEN


_ESA_CACHE = {}


def oracle_esa(name):
    """Oracle-built ESA of a golden FASTA, cached per session."""
    import oracle_lib as O
    if name not in _ESA_CACHE:
        text, _ = O.encode_fasta(os.path.join(GOLDEN, name))
        _ESA_CACHE[name] = O.Esa(text)
    return _ESA_CACHE[name]
