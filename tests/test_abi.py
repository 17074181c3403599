"""The C-ABI boundary (include/nebula_gn.h): libnebula_gn.so loads on a CPU-only host and exports
every function the header declares, and nothing else (the version script keeps ngx_* only).
No compute calls are made here (no GPU)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "nebula_gn.h")
LIB = os.path.join(ROOT, "nebula_amd", "libnebula_gn.so")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\**\s*(ngx_[a-z0-9_]+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_the_boundary():
    names = declared()
    for must in ["ngx_open", "ngx_close", "ngx_add_space", "ngx_add_schema", "ngx_load_kv", "ngx_commit",
                 "ngx_get_neighbors", "ngx_gn_result_free", "ngx_go", "ngx_go_result_free", "ngx_last_error"]:
        assert must in names


def test_library_exports_every_declared_symbol():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "nebula_amd", "csrc")])
    L = ctypes.CDLL(LIB)
    missing = [n for n in declared() if not hasattr(L, n)]
    assert not missing, missing
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert exported == set(declared()), sorted(exported ^ set(declared()))


def test_hash_string_is_libstdcxx_hash():
    """ngx_hash_string is pure host code: std::hash<std::string> as the NBA fixture's vids use it
    (TraverseTestBase.h:122-126). GoTest's literal vid for "Tim Duncan" pins it (GoTest.cpp:335-337
    lists rows by hash)."""
    L = ctypes.CDLL(LIB)
    L.ngx_hash_string.restype = ctypes.c_int64
    L.ngx_hash_string.argtypes = [ctypes.c_char_p, ctypes.c_uint64]
    from nebula_amd import ngql
    for name in ["Tim Duncan", "Tony Parker", "LaMarcus Aldridge", ""]:
        b = name.encode()
        assert L.ngx_hash_string(b, len(b)) == ngql.nebula_hash(name)


def test_go_result_layout_matches_header(tmp_path):
    """The ctypes mirror of ngx_go_result (nebula_amd/engine.py) has the header's field offsets and size."""
    from nebula_amd.engine import GoResultC
    fields = [f[0] for f in GoResultC._fields_]
    prog = tmp_path / "layout.c"
    body = "".join(f'    printf("%s %zu\\n", "{f}", offsetof(ngx_go_result, {f}));\n' for f in fields)
    prog.write_text("#include <stddef.h>\n#include <stdio.h>\n#include \"nebula_gn.h\"\nint main(void) {\n" + body +
                    '    printf("sizeof %zu\\n", sizeof(ngx_go_result));\n    return 0;\n}\n')
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(prog), "-o", str(exe)])
    got = dict(line.split() for line in subprocess.check_output([str(exe)], text=True).splitlines())
    for f in fields:
        assert int(got[f]) == getattr(GoResultC, f).offset, f
    assert int(got["sizeof"]) == ctypes.sizeof(GoResultC)
