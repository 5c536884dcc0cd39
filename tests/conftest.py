import importlib
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")


@pytest.fixture(scope="session")
def hf():
    """The product package (HIP library behind the C ABI)."""
    return importlib.import_module("3fs_amd")


@pytest.fixture(scope="session")
def orc():
    """The CPU parity oracle (test infrastructure only)."""
    import oracle
    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(REPO, "tests", "golden", "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def bulk_golden():
    """Full-size digest table of bench.py's workload (tests/golden/make_bulk_golden.py)."""
    d = os.path.join(REPO, "tests", "golden")
    with open(os.path.join(d, "bulk_4MiB_digests.json")) as f:
        meta = json.load(f)
    import numpy as np
    table = np.fromfile(os.path.join(d, "bulk_4MiB_digests.bin"), dtype="<u4")
    return meta, table


@pytest.fixture
def opts(hf):
    """opts(name, value): set a library switch (hf3fs_crc_set_option) for this test only."""
    L = hf._lib
    saved = {}

    def set_(name, value):
        if name not in saved:
            saved[name] = L.get_option(name)
        L.set_option(name, value)

    yield set_
    for name, value in saved.items():
        L.set_option(name, value)
