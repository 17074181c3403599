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


_CURRENT = {"node": "", "t0": 0.0}


def _uncaptured_fd(config):
    """The process's real stderr while pytest captures fd 2 (capture=fd saves the original with dup)."""
    try:
        cap = config.pluginmanager.getplugin("capturemanager")._global_capturing
        return cap.err.targetfd_save
    except Exception:
        return None


def pytest_sessionstart(session):
    """Long parity tests (the C2 oracle step and its fixture run minutes with nothing to print) write one
    line a minute to the uncaptured stderr and to gpurun_out/heartbeat.log when that directory exists, so
    a watchdog that reads output as liveness does not take them for hangs."""
    import threading
    import time
    _CURRENT["t0"] = time.monotonic()
    fd = _uncaptured_fd(session.config)
    beat_file = os.path.join(ROOT, "gpurun_out", "heartbeat.log")

    def beat():
        while True:
            time.sleep(60)
            line = f"[still running {time.monotonic() - _CURRENT['t0']:.0f} s] {_CURRENT['node']}\n"
            try:
                os.write(fd if fd is not None else 2, line.encode())
            except OSError:
                pass
            if os.path.isdir(os.path.dirname(beat_file)):
                with open(beat_file, "a") as f:
                    f.write(line)

    threading.Thread(target=beat, daemon=True).start()


def pytest_runtest_logstart(nodeid, location):
    _CURRENT["node"] = nodeid
