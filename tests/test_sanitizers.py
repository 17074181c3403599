"""Host AddressSanitizer + UndefinedBehaviorSanitizer run (CPU): the library's host-side C++ (KV ->
columnar exporter, snapshot reader / writer and its checks, expression decoder / pushdown rewrite /
compiler, synthetic generator) and the oracle, built with -fsanitize=address,undefined by
tools/san/Makefile into one driver (tools/san/san_driver.cpp). The driver exports an RMAT shard at
world 1 and 3, round-trips and damages the snapshot files, fuzzes the expression decoder and compiler
from the ExpressionTest encodings, and runs GO requests through the oracle. Any sanitizer report fails
the run (halt_on_error)."""
import json
import os
import subprocess

import pytest

from nebula_amd import datagen, ngql
from oracle import oracle
from tests.test_oracle_expr import CASES

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "tools", "san")

GO_QUERIES = [
    "GO FROM {S} OVER e YIELD e._dst, e.p0",
    "GO 2 STEPS FROM {S} OVER e WHERE e.p0 < 50 YIELD e._dst, e._rank, e.p1",
    "GO 2 STEPS FROM {S} OVER e REVERSELY WHERE $^.vt.v0 > 100 YIELD $^.vt.name, $$.vt.v0, e.p0 + e.p1",
    "GO 1 TO 3 STEPS FROM {S} OVER e BIDIRECT WHERE e.p0 > 80 YIELD DISTINCT e._dst, lower($$.vt.name)",
]


@pytest.fixture(scope="module")
def driver():
    r = subprocess.run(["make", "-s", "-j8"], cwd=SAN, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    return os.path.join(SAN, "build", "san_driver")


def test_host_code_under_asan_and_ubsan(driver, tmp_path):
    seeds = ", ".join(str(int(v)) for v in datagen.sample_vids(5, 1 << 10, 20))
    for i, q in enumerate(GO_QUERIES):
        (tmp_path / f"go_{i:02d}.bin").write_bytes(oracle.go_request(ngql.parse_go(q.replace("{S}", seeds))))
    for c in CASES:
        (tmp_path / f"expr_{c['line']:04d}.bin").write_bytes(ngql.parse_expr(c["expr"]).encode())
    for i, q in enumerate(["e.p0 > 3 && $^.vt.name == \"v1\" || $$.vt.v0 < 2", "udf_is_in(e.p1, 1, 2, 3)",
                           "(string)e.p0 + lpad($^.vt.name, 9, \"*\")", "$-.a + $var.b > 1 XOR e._rank == 0"]):
        (tmp_path / f"expr_x{i}.bin").write_bytes(ngql.parse_expr(q).encode())
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([driver, str(tmp_path), "10"], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-6000:])
    assert "OK (0 failures)" in r.stdout
    assert "oracle: 4 GO requests" in r.stdout
    assert "export == generator csr" in r.stdout
