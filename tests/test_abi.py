"""The C-ABI library loads and exports every entry point include/*.h declares, and
the ctypes binding (the NIF stand-in) binds each of them.  No compute without a GPU."""

import ctypes
import os
import re
import subprocess

import pytest

from lasp_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    import glob
    src = "".join(open(h).read() for h in sorted(glob.glob(os.path.join(ROOT, "include", "*.h"))))
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(laspj_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from lasp_amd import build
    build.build()
    return _lib.load()


def test_header_parses():
    names = declared()
    assert "laspj_orset_join" in names and "laspj_orset_inflation" in names
    assert len(names) >= 40


def test_every_declared_symbol_is_exported(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (laspj_\w+)", out))
    missing = [n for n in declared() if n not in exported]
    assert not missing, missing
    for n in declared():
        assert hasattr(lib, n)


def test_binding_covers_header():
    assert sorted(_lib.SIGNATURES) == declared()


def test_integration_table_matches_header():
    """INTEGRATION.md §4 lists every entry point with the reference function it serves,
    as tools/abi_table.py generates it from the header (no entry point undocumented)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import abi_table
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    i = doc.index(abi_table.BEGIN) + len(abi_table.BEGIN)
    assert doc[i:doc.index(abi_table.END)].strip() == abi_table.table().strip()
    listed = set(re.findall(r"^\| `(laspj_\w+)`", doc, flags=re.M))
    assert listed == set(declared())


def test_abi_calls_without_gpu(lib):
    assert lib.laspj_abi_version() == 2
    assert lib.laspj_strerror(_lib.E_SHAPE) == b"shape mismatch"
    n = ctypes.c_int(-1)
    assert lib.laspj_device_count(ctypes.byref(n)) == 0
    assert n.value >= 0
    # null handles are rejected with LASPJ_E_INVAL, never a crash
    assert lib.laspj_orset_join(None, None, None, None) == _lib.E_INVAL
    assert lib.laspj_ctx_destroy(None) == _lib.E_INVAL
    assert lib.laspj_ctx_create(0, None) == _lib.E_INVAL
    if n.value == 0:
        h = ctypes.c_void_p()
        assert lib.laspj_ctx_create(0, ctypes.byref(h)) == _lib.E_DEVICE


def test_struct_layouts():
    assert ctypes.sizeof(_lib.Op) == 16
    assert ctypes.sizeof(_lib.BatchInfo) == 48


def test_engine_fails_loudly_without_library(monkeypatch):
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", "/nonexistent/liblaspj.so")
    with pytest.raises(_lib.LaspjUnavailable):
        _lib.load()


def _build_c_client(tmp_path):
    """Compile tests/c/laspj_c_client.c against include/laspj.h and liblaspj.so alone
    (the NIF's view of the boundary)."""
    import shutil
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    exe = str(tmp_path / "laspj_c_client")
    libdir = os.path.join(root, "lasp_amd")
    cmd = [cc, "-std=c11", "-O2", "-Wall", "-Werror", "-I", os.path.join(root, "include"),
           os.path.join(root, "tests", "c", "laspj_c_client.c"), "-L", libdir, "-llaspj",
           f"-Wl,-rpath,{libdir}", "-o", exe]
    res = subprocess.run(cmd, capture_output=True, text=True)
    assert res.returncode == 0, res.stderr
    return exe


def test_c_client_compiles_against_header(tmp_path):
    _build_c_client(tmp_path)


@pytest.mark.gpu
def test_c_client_runs(tmp_path):
    """merge / value / stats / inflation / update / error status from plain C."""
    import subprocess
    exe = _build_c_client(tmp_path)
    res = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert res.returncode == 0, res.stdout + res.stderr
    assert "laspj C client OK" in res.stdout
