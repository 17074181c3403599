"""The device's double -> string (nebula_amd/csrc/dtoa.h, `(string)` casts) compiled for the host and
checked against the oracle's rule — std::to_chars shortest digits formatted as Expression::toString
(oracle/orc_expr.cpp) — over special values, every power of two and ten with their neighbours, random
bit patterns (all exponents, subnormals, NaNs) and random short decimals (tools/dtoa_check.cpp)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shortest_double_strings_match_the_oracle(tmp_path):
    exe = str(tmp_path / "dtoa_check")
    r = subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(ROOT, "tools", "dtoa_check.cpp")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([exe, "300000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout[-2000:]
