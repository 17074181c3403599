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
    """BASELINE C2 graph exactly as bench.py builds it at N = 1 (RMAT scale 22, edge factor 16, 100 parts,
    e(p0, p1), every out-edge also stored as its in-edge -e, no tags) and the oracle loaded with it,
    shared by the C2 parity tests and the world-8 rehearsal (which reads the out-edges only)."""
    from oracle import oracle
    from tests import fixtures
    ds = fixtures.RmatDataset(22, with_in=True, threads=16)
    o = oracle.Oracle()
    o.set_flags(threads=16, max_handlers=16, graph_threads=16)
    ds.load_oracle(o, threads=16)
    yield ds, o
    o.close()
    ds.rows.free()
