"""CPU: liblira_hip.so loads, exports every symbol include/lira_hip.h declares,
and validates arguments before touching the GPU."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "lira_hip.h")
PKGDIR = os.path.join(ROOT, "lira-ann-search_amd")
LIB = os.path.join(PKGDIR, "lira_amd", "liblira_hip.so")


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-s", "-C", PKGDIR], check=True)
    from lira_amd import _lib
    return _lib.load()


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(lira_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_entry_points():
    fns = header_functions()
    assert "lira_scan_topk" in fns and "lira_rank_nearest" in fns and len(fns) >= 15


def test_every_declared_symbol_is_exported(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True,
                         check=True).stdout
    exported = set(l.split()[-1] for l in out.splitlines() if " T " in l)
    missing = [f for f in header_functions() if f not in exported]
    assert not missing, missing
    for f in header_functions():
        getattr(lib, f)  # resolvable through ctypes


def test_binding_covers_header():
    from lira_amd import _lib
    assert sorted(_lib.SIGNATURES) == header_functions()


def test_abi_version_and_errors(lib):
    assert lib.lira_abi_version() == 1
    h = ctypes.c_void_p()
    rc = lib.lira_index_create(0, 0, 0, ctypes.byref(h))
    assert rc == -1 and b"d must be" in lib.lira_last_error()
    rc = lib.lira_index_create(0, 16, 7, ctypes.byref(h))
    assert rc == -1 and b"metric" in lib.lira_last_error()
    sz = ctypes.c_size_t()
    assert lib.lira_scan_workspace_size(None, 1, 1, 10, 0, ctypes.byref(sz)) == -1
    assert lib.lira_scan_topk(None, None, 0, None, 1, 10, 0, None, None, None, None, 0, None) == -1
    assert lib.lira_rank_workspace_size(10, 64, ctypes.byref(sz)) == 0 and sz.value >= 10 * 64 * 4
    assert lib.lira_rank_nearest(None, 1, None, 64, 16, 0, None, None, 0, None) == -6
    assert lib.lira_select_probes(None, 1, 8, 9, 0.0, 4, None, None, None) == -1
    assert lib.lira_centroid_dist(None, 4, None, 8, 16, None, ctypes.c_void_p(1), None, None) == -1
    v = ctypes.c_int64()
    assert lib.lira_index_set_option(None, 1, 0) == -1
    assert lib.lira_index_get_option(None, 1, ctypes.byref(v)) == -1
    assert lib.lira_index_has_tiles(None, ctypes.byref(ctypes.c_int())) == -1


def test_option_names_match_header():
    from lira_amd import _lib
    txt = open(HEADER).read()
    keys = dict((m.lower(), int(v)) for m, v in re.findall(r"#define LIRA_OPT_([A-Z_]+) (\d+)", txt))
    assert keys == _lib.OPTIONS


def test_python_error_mapping(lib):
    from lira_amd import _lib
    with pytest.raises(_lib.LiraError, match="EINVAL"):
        _lib.call("lira_index_create", 0, -3, 0, ctypes.byref(ctypes.c_void_p()))


def test_no_fallback_when_library_missing(tmp_path):
    from lira_amd import _lib
    with pytest.raises(_lib.LiraError, match="no CPU fallback"):
        _lib.load(str(tmp_path / "missing.so"))
