"""Build recipes for the native parts of parmmg_amd (in-tree, no JIT cache).

* ``libpmx_transfer.so`` -- the product: HIP kernels for gfx950 + the C ABI of
  ``include/pmx_transfer.h``.  Built with ``-ffp-contract=off`` so that no
  multiply-add is fused and results match the x86-64 oracle bit for bit.
* ``libpmx_meshgen.so`` -- synthetic Kuhn-cube meshes / new points for tests and
  the bench (plain C + OpenMP, not on the product path).
* ``oracle/liboracle.so`` -- the CPU restatement used only as the checker
  (tests, smoke, bench cpu_baseline).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "parmmg_amd")
CSRC = os.path.join(PKG, "csrc")
INC = os.path.join(ROOT, "include")
ORACLE = os.path.join(ROOT, "oracle")

TRANSFER_SO = os.path.join(PKG, "libpmx_transfer.so")
MESHGEN_SO = os.path.join(PKG, "libpmx_meshgen.so")
ORACLE_SO = os.path.join(ORACLE, "liboracle.so")

HIP_SOURCES = ["pmx_capi.hip", "pmx_kernels.hip", "pmx_walk.hip", "pmx_bdy.hip", "pmx_stats.hip",
               "pmx_groups.hip", "pmx_topo.hip", "pmx_medit.hip"]
HIPCC_FLAGS = [
    "-O3", "--offload-arch=gfx950", "-std=c++17", "-fPIC", "-shared",
    "-ffp-contract=off", "-fno-fast-math", "-Wall", "-Wno-unused-function",
    "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib",
]


def _hipcc() -> str:
    for c in ("/opt/rocm/bin/hipcc", shutil.which("hipcc") or ""):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the HIP extension cannot be built")


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


class _locked:
    """Inter-process lock around a build step: the ranks of a multi-GPU job
    all call the build; one compiles, the others wait and find it fresh."""

    def __init__(self, name: str):
        self.path = os.path.join(PKG, f".{name}.lock")

    def __enter__(self):
        import fcntl
        self.f = open(self.path, "w")
        fcntl.flock(self.f, fcntl.LOCK_EX)
        return self

    def __exit__(self, *exc):
        import fcntl
        fcntl.flock(self.f, fcntl.LOCK_UN)
        self.f.close()
        return False


def _log(msg: str) -> None:
    """Timestamped progress on stderr: a rebuild (stale library on a fresh GPU
    box) compiles for minutes, and a silent one reads as a hang."""
    import time
    sys.stderr.write(f"[build {time.strftime('%H:%M:%S')}] {msg}\n")
    sys.stderr.flush()


def _run(cmd: list[str]) -> None:
    _log("run: " + " ".join(os.path.basename(c) if os.path.isabs(c) and c.endswith((".hip", ".c", ".so"))
                            else c for c in cmd[:1] + [c for c in cmd if c.endswith((".hip", ".c"))]))
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("build failed: " + " ".join(cmd))


def _jobs() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(8, n))


def build_transfer(force: bool = False) -> str:
    """One object per source file, compiled in parallel (the kernels and their
    launch functions share a file, so no relocatable device code is needed),
    then one link."""
    from concurrent.futures import ThreadPoolExecutor
    srcs = [os.path.join(CSRC, s) for s in HIP_SOURCES]
    hdrs = [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")]
    hdrs.append(os.path.join(INC, "pmx_transfer.h"))
    deps = srcs + hdrs
    if force or _stale(TRANSFER_SO, deps):
        with _locked("transfer"):
            if force or _stale(TRANSFER_SO, deps):
                odir = os.path.join(PKG, "build", "obj")
                os.makedirs(odir, exist_ok=True)
                cflags = [f for f in HIPCC_FLAGS if f not in ("-shared",) and not f.startswith(("-l", "-L", "-Wl"))]
                lflags = [f for f in HIPCC_FLAGS if f == "-shared" or f.startswith(("-l", "-L", "-Wl"))]

                def obj(src: str) -> str:
                    o = os.path.join(odir, os.path.basename(src) + ".o")
                    if force or _stale(o, [src] + hdrs):
                        tmp = o + f".{os.getpid()}.tmp"
                        _run([_hipcc(), *cflags, "-c", "-I", INC, "-I", CSRC, src, "-o", tmp])
                        os.replace(tmp, o)
                    return o

                with ThreadPoolExecutor(_jobs()) as ex:
                    objs = list(ex.map(obj, srcs))
                tmp = TRANSFER_SO + f".{os.getpid()}.tmp"
                _run([_hipcc(), "--offload-arch=gfx950", *objs, *lflags, "-o", tmp])
                os.replace(tmp, TRANSFER_SO)
    return TRANSFER_SO


def build_meshgen(force: bool = False) -> str:
    src = os.path.join(CSRC, "meshgen.c")
    if force or _stale(MESHGEN_SO, [src]):
        with _locked("meshgen"):
            if force or _stale(MESHGEN_SO, [src]):
                tmp = MESHGEN_SO + f".{os.getpid()}.tmp"
                _run(["gcc", "-O2", "-std=c99", "-fPIC", "-shared", "-fopenmp", src, "-o", tmp,
                      "-lm"])
                os.replace(tmp, MESHGEN_SO)
    return MESHGEN_SO


def build_oracle(force: bool = False) -> str:
    srcs = [os.path.join(ORACLE, f) for f in sorted(os.listdir(ORACLE)) if f.endswith(".c")]
    deps = srcs + [os.path.join(ORACLE, "pmx_oracle.h")]
    if force or _stale(ORACLE_SO, deps):
        with _locked("oracle"):
            if force or _stale(ORACLE_SO, deps):
                tmp = ORACLE_SO + f".{os.getpid()}.tmp"
                # x86-64 baseline (SSE2, no FMA), no contraction, -O3 as the
                # reference's Release build (CMakeLists.txt:100-116) without
                # -ffast-math: the CPU baseline is timed at the reference's level
                _run(["gcc", "-O3", "-std=c99", "-fPIC", "-shared", "-ffp-contract=off",
                      "-fno-fast-math", *srcs, "-o", tmp, "-lm"])
                os.replace(tmp, ORACLE_SO)
    return ORACLE_SO


def build_all(force: bool = False) -> None:
    build_meshgen(force)
    build_oracle(force)
    build_transfer(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
    print("built:", TRANSFER_SO, MESHGEN_SO, ORACLE_SO)
