"""The C-ABI library loads and exports every symbol include/edverify.h
declares (no compute calls: this runs without a GPU)."""
import ctypes
import os
import re

from conftest import PKG, ROOT


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "edverify.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(edv_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_the_python_binding_table():
    from plenum_amd import _lib
    assert set(declared_symbols()) == set(_lib.SIGNATURES)


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(os.path.join(PKG, "libplenum_edverify.so"))
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_version_string():
    from plenum_amd import _lib
    lib = _lib.load()
    assert b"gfx950" in lib.edv_version()


def test_library_is_gfx950_code_object():
    data = open(os.path.join(PKG, "libplenum_edverify.so"), "rb").read()
    assert b"gfx950" in data
    assert b"edv_dsm_kernel" in data
