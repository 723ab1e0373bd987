"""CPU checks of the C ABI: the HIP library exists, loads without a GPU and
exports every function include/pmx_transfer.h declares (no compute calls)."""
import ctypes
import os
import re

from conftest import ROOT
from parmmg_amd import _native


def declared_functions():
    src = open(os.path.join(ROOT, "include", "pmx_transfer.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = set(re.findall(r"\b((?:pmx|PMX)_\w+)\s*\(", src))
    return sorted(names)


def test_header_declares_the_reference_seams():
    names = declared_functions()
    for n in ("PMX_interpMetricsAndFields", "PMX_copyMetricsAndFields_point", "pmx_run",
              "pmx_upload_background", "pmx_qualhisto", "pmx_prilen", "pmx_tetra_qual"):
        assert n in names


def test_library_exports_every_declared_symbol():
    assert os.path.exists(_native.LIB_PATH), "libpmx_transfer.so not built"
    lib = ctypes.CDLL(_native.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, f"missing exports: {missing}"


def test_binding_covers_header():
    assert set(declared_functions()) <= set(_native.SIGNATURES)
    _native.load()   # sets restype/argtypes for every symbol


def test_library_is_gfx950_code_object():
    data = open(_native.LIB_PATH, "rb").read()
    assert b"gfx950" in data
