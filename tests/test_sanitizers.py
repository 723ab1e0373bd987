"""ASan/UBSan builds of the repository's CPU-side C.

* the oracle restatement (oracle/*.c) and the mesh generator
  (parmmg_amd/csrc/meshgen.c), driven end to end by tests/c/oracle_asan.c and
  run here (CPU): leaks, out-of-bounds accesses and undefined behaviour fail
  the test;
* the library's Medit I/O (parmmg_amd/csrc/pmx_medit.hip, host code) compiled
  with g++ and driven by tests/c/medit_asan.cpp (CPU);
* the C driver of the drop-in seam (tests/c/dropin_demo.c) built with the same
  flags (its host code instrumented, the HIP library as is); it runs on the
  GPU box (-m gpu), with leak checking off for the HIP runtime's allocations.
"""
import os
import subprocess

import pytest

from conftest import ROOT

BUILD = os.path.join(ROOT, "tests", "c", "_build")
SAN = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
       "-fno-sanitize-recover=undefined"]


def _gcc(srcs, out, extra=()):
    os.makedirs(BUILD, exist_ok=True)
    cmd = ["gcc", "-std=c99", "-Wall", *SAN, "-I", os.path.join(ROOT, "include"), "-I",
           os.path.join(ROOT, "oracle"), *srcs, "-o", out, *extra, "-lm"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    return out


def test_oracle_and_meshgen_under_asan_ubsan():
    srcs = [os.path.join(ROOT, "tests", "c", "oracle_asan.c"),
            os.path.join(ROOT, "parmmg_amd", "csrc", "meshgen.c")]
    srcs += sorted(os.path.join(ROOT, "oracle", f) for f in os.listdir(os.path.join(ROOT, "oracle"))
                   if f.endswith(".c"))
    exe = _gcc(srcs, os.path.join(BUILD, "oracle_asan"))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "oracle asan ok" in r.stdout


def test_medit_io_under_asan_ubsan(tmp_path):
    os.makedirs(BUILD, exist_ok=True)
    exe = os.path.join(BUILD, "medit_asan")
    cmd = ["g++", "-std=c++17", "-Wall", "-x", "c++", *SAN, "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "parmmg_amd", "csrc", "pmx_medit.hip"),
           os.path.join(ROOT, "tests", "c", "medit_asan.cpp"), "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "medit asan ok" in r.stdout


def _demo_asan():
    from parmmg_amd import _native
    libdir = os.path.dirname(_native.LIB_PATH)
    return _gcc([os.path.join(ROOT, "tests", "c", "dropin_demo.c")],
                os.path.join(BUILD, "dropin_demo_asan"),
                ["-L", libdir, "-lpmx_transfer", "-Wl,-rpath," + libdir])


def test_dropin_demo_builds_with_asan_ubsan():
    assert os.path.exists(_demo_asan())


@pytest.mark.gpu
def test_dropin_demo_runs_under_asan_ubsan():
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:protect_shadow_gap=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([_demo_asan()], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "dropin ok" in r.stdout


def test_compact_walk_records_roundtrip_under_asan_ubsan():
    """The walk's 24-B records (parmmg_amd/csrc/pmx_wrec.h, shared with the
    kernels) decode to the full tet record for every valid tet: packed deltas
    at and past their 20/24-bit limits, boundary faces, escapes, deleted tets."""
    os.makedirs(BUILD, exist_ok=True)
    exe = os.path.join(BUILD, "wrec_roundtrip")
    cmd = ["g++", "-std=c++17", "-Wall", *SAN, "-I", os.path.join(ROOT, "parmmg_amd", "csrc"),
           os.path.join(ROOT, "tests", "c", "wrec_roundtrip.cpp"), "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    env = dict(os.environ, UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "wrec roundtrip ok" in r.stdout
