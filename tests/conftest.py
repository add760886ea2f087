"""Shared fixtures.  `-m gpu` tests need an MI355X and the built
libgnark_mi355x.so; `-m "not gpu"` tests run on CPU (oracle, host logic, ABI)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("oracle", "gnark-icicle_amd", "tests"):
    p = os.path.join(ROOT, sub)
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU and the built HIP library")


@pytest.fixture(scope="session")
def oracle():
    import oracle_lib
    oracle_lib.build()
    return oracle_lib


@pytest.fixture(scope="session")
def gm_ctx():
    import gnark_mi355x as gm
    ctx = gm.Context(0)
    yield ctx
    ctx.close()
