"""The C-ABI library loads here (no GPU needed) and exports exactly the entry
points include/gk_capi.h declares; the ctypes binding covers every one; the
product package never touches oracle/ and fails loudly without a GPU."""
import ast
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gk_capi.h")
PKG = os.path.join(ROOT, "sketches-py_amd", "gkarray_amd")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gk_[a-z_]+)\s*\(", src)))


def test_header_declares_entry_points():
    names = declared()
    for must in ("gk_create", "gk_destroy", "gk_ingest", "gk_flush", "gk_quantiles", "gk_merge",
                 "gk_stats", "gk_export", "gk_import", "gk_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol(built_lib):
    import ctypes
    lib = ctypes.CDLL(built_lib)
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_matches_header(built_lib):
    from gkarray_amd import _lib
    assert sorted(_lib.SYMBOLS) == declared()
    h = _lib.load(built_lib)
    assert h.gk_version() == 100
    assert h.gk_last_error() == b""


def test_create_without_gpu_fails_loudly(built_lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from gkarray_amd import GKArray, GKBackendError, StreamSet
    with pytest.raises(GKBackendError):
        StreamSet(4, 0.01)
    with pytest.raises(GKBackendError):
        GKArray(0.01)


def test_product_package_does_not_import_oracle():
    for dirpath, _, files in os.walk(os.path.join(ROOT, "sketches-py_amd")):
        for f in files:
            if not f.endswith(".py"):
                continue
            tree = ast.parse(open(os.path.join(dirpath, f)).read())
            for node in ast.walk(tree):
                if isinstance(node, (ast.Import, ast.ImportFrom)):
                    mods = [a.name for a in node.names] if isinstance(node, ast.Import) else [node.module or ""]
                    assert not any("oracle" in m for m in mods), (f, mods)
            assert "gk_oracle" not in open(os.path.join(dirpath, f)).read(), f


def test_library_does_not_link_oracle(built_lib):
    data = open(built_lib, "rb").read()
    assert b"gko_" not in data and b"libgkoracle" not in data
