"""CPU checks of the C ABI: the HIP library exists, loads without a GPU and
exports every function include/pmx_transfer.h declares (no compute calls)."""
import ctypes
import os
import re

import pytest

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


DEMO_SRC = os.path.join(ROOT, "tests", "c", "dropin_demo.c")
DEMO_BIN = os.path.join(ROOT, "tests", "c", "_build", "dropin_demo")


def build_dropin_demo() -> str:
    """gcc the C driver of the drop-in seam against the header and the HIP
    library (plain C, as ParMmg's own sources would be)."""
    import subprocess
    os.makedirs(os.path.dirname(DEMO_BIN), exist_ok=True)
    deps = [DEMO_SRC, os.path.join(ROOT, "include", "pmx_transfer.h"), _native.LIB_PATH]
    if (not os.path.exists(DEMO_BIN)
            or any(os.path.getmtime(DEMO_BIN) < os.path.getmtime(d) for d in deps if os.path.exists(d))):
        subprocess.run(["gcc", "-O2", "-Wall", "-Werror", "-std=c99", "-I",
                        os.path.join(ROOT, "include"), DEMO_SRC, "-o", DEMO_BIN, "-L",
                        os.path.dirname(_native.LIB_PATH), "-lpmx_transfer",
                        "-Wl,-rpath," + os.path.dirname(_native.LIB_PATH), "-lm"], check=True)
    return DEMO_BIN


ITER_SRC = os.path.join(ROOT, "tests", "c", "iteration_demo.c")
ITER_BIN = os.path.join(ROOT, "tests", "c", "_build", "iteration_demo")


def build_iteration_demo() -> str:
    """gcc the C driver of two resident iterations (+ the repository's mesh
    generator) against the header and the HIP library."""
    import subprocess
    os.makedirs(os.path.dirname(ITER_BIN), exist_ok=True)
    gen = os.path.join(ROOT, "parmmg_amd", "csrc", "meshgen.c")
    deps = [ITER_SRC, gen, os.path.join(ROOT, "include", "pmx_transfer.h"), _native.LIB_PATH]
    if (not os.path.exists(ITER_BIN)
            or any(os.path.getmtime(ITER_BIN) < os.path.getmtime(d) for d in deps if os.path.exists(d))):
        subprocess.run(["gcc", "-O2", "-Wall", "-Werror", "-Wno-unknown-pragmas", "-std=c99", "-I",
                        os.path.join(ROOT, "include"), ITER_SRC, gen, "-o", ITER_BIN, "-L", os.path.dirname(_native.LIB_PATH),
                        "-lpmx_transfer", "-Wl,-rpath," + os.path.dirname(_native.LIB_PATH), "-lm"],
                       check=True)
    return ITER_BIN


def test_iteration_demo_compiles_as_c():
    assert os.path.exists(build_iteration_demo())


@pytest.mark.gpu
def test_iteration_demo_runs():
    """Two ParMmg iterations from C with the background kept on the GPU, the
    new mesh's quality reduced over RCCL; bit-identical to a host upload."""
    import subprocess
    r = subprocess.run([build_iteration_demo()], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "iteration ok" in r.stdout


def test_dropin_demo_compiles_as_c():
    assert os.path.exists(build_dropin_demo())


@pytest.mark.gpu
def test_dropin_demo_runs():
    """The C driver: Mmg-style AoS records through strided views, adjacency
    rebuilt on the device, PMX_interpMetricsAndFields; linear fields exact,
    the MG_REQ point untouched."""
    import subprocess
    r = subprocess.run([build_dropin_demo()], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "dropin ok" in r.stdout


def test_integration_makefile_matches_the_build():
    """integration/Makefile (the Python-free build a ParMmg build links) lists
    the same HIP sources as parmmg_amd/build.py and the flags bit parity needs
    (-ffp-contract=off, gfx950); `make -n` resolves every rule."""
    import re
    import subprocess
    from parmmg_amd import build
    mk = open(os.path.join(ROOT, "integration", "Makefile")).read()
    m = re.search(r"^SOURCES\s*:=\s*((?:.*\\\n)*.*)$", mk, re.M)
    srcs = m.group(1).replace("\\\n", " ").split()
    assert srcs == build.HIP_SOURCES
    assert "-ffp-contract=off" in mk and "gfx950" in mk
    r = subprocess.run(["make", "-n", "-C", os.path.join(ROOT, "integration"), "OUT=/tmp/pmx_make_n"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert r.stdout.count("-c ") == len(srcs) and "libpmx_transfer.so" in r.stdout
