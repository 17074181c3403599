import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")
    config.addinivalue_line("markers", "slow: larger parity cases")


@pytest.fixture(scope="session")
def rmat22():
    """BASELINE C2 graph (RMAT scale 22, edge factor 16, 100 parts, e(p0, p1), no tags / in-edges) and
    the oracle loaded with it, shared by the C2 parity tests and the world-8 rehearsal."""
    from oracle import oracle
    from tests import fixtures
    ds = fixtures.RmatDataset(22, threads=16)
    o = oracle.Oracle()
    o.set_flags(threads=16)
    ds.load_oracle(o, threads=16)
    yield ds, o
    o.close()
    ds.rows.free()
