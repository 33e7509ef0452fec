"""Shared test setup. `-m gpu` tests need an MI355X and the built libsgn.so; everything
else runs on the CPU (oracle, front end, ABI surface, gloo shard protocol)."""
import pathlib
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "shadow-gen_amd"))
sys.path.insert(0, str(ROOT / "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


@pytest.fixture(scope="session")
def oracle():
    import oracle_py
    oracle_py.load()
    return oracle_py


@pytest.fixture(scope="session")
def lib():
    import sgn
    return sgn.load()
