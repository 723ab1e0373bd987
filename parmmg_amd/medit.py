"""Medit files through the C library (pmx_medit_*, include/pmx_transfer.h).

The wire format of the transfer path's inputs and outputs: ParMmg reads and
writes meshes and solutions through Mmg (reference src/inout_pmmg.c:440-991 ->
MMG3D_loadMesh / saveMesh / loadSol / saveSol).  ASCII ``.mesh``/``.sol`` and
binary ``.meshb``/``.solb`` by extension; arrays in Mmg's layout (1-based, row
0 unused, tensors (11,12,13,22,23,33)).
"""
from __future__ import annotations

import ctypes as C
import dataclasses

import numpy as np

from . import _native as N

_SIZE = {1: 1, 2: 3, 3: 6}
_TYPE = {1: 1, 3: 2, 6: 3}


def _err(what: str):
    raise RuntimeError(f"{what}: {N.load().pmx_medit_last_error().decode()}")


def _ip(a):
    return a.ctypes.data_as(N.iptr) if a is not None else None


@dataclasses.dataclass
class MeditMesh:
    xyz: np.ndarray        # (np+1, 3)
    vref: np.ndarray       # (np+1,)
    tet: np.ndarray        # (ne+1, 4)
    tetref: np.ndarray     # (ne+1,)
    tria: np.ndarray       # (nt+1, 3)
    triaref: np.ndarray    # (nt+1,)
    required: np.ndarray   # (nreq,) 1-based vertex indices
    version: int = 0


def read_mesh(path: str) -> MeditMesh:
    lib = N.load()
    info = N.MeditInfo()
    if not lib.pmx_medit_mesh_info(path.encode(), C.byref(info)):
        _err("pmx_medit_mesh_info")
    xyz = np.zeros((info.np + 1, 3))
    vref = np.zeros(info.np + 1, np.int32)
    tet = np.zeros((info.ne + 1, 4), np.int32)
    tetref = np.zeros(info.ne + 1, np.int32)
    tria = np.zeros((info.nt + 1, 3), np.int32)
    triaref = np.zeros(info.nt + 1, np.int32)
    req = np.zeros(max(info.nreq, 1), np.int32)
    if not lib.pmx_medit_mesh_read(path.encode(), C.byref(info), xyz.ctypes.data_as(N.dptr), _ip(vref), _ip(tet),
                                   _ip(tetref), _ip(tria), _ip(triaref), _ip(req)):
        _err("pmx_medit_mesh_read")
    return MeditMesh(xyz, vref, tet, tetref, tria, triaref, req[: info.nreq], info.version)


def write_mesh(path: str, xyz, tet, tria=None, required=None, vref=None, tetref=None, triaref=None):
    """xyz (np+1, 3), tet (ne+1, 4), tria (nt+1, 3): Mmg layout, row 0 unused."""
    lib = N.load()
    xyz = np.ascontiguousarray(xyz, np.float64)
    tet = np.ascontiguousarray(tet, np.int32)
    tria = np.ascontiguousarray(tria if tria is not None else np.zeros((1, 3)), np.int32)
    req = np.ascontiguousarray(required if required is not None else np.zeros(0), np.int32)
    refs = [None if r is None else np.ascontiguousarray(r, np.int32) for r in (vref, tetref, triaref)]
    if not lib.pmx_medit_mesh_write(path.encode(), xyz.shape[0] - 1, xyz.ctypes.data_as(N.dptr), _ip(refs[0]),
                                    tet.shape[0] - 1, _ip(tet), _ip(refs[1]), tria.shape[0] - 1, _ip(tria),
                                    _ip(refs[2]), len(req), _ip(req) if len(req) else None):
        _err("pmx_medit_mesh_write")


def read_sol(path: str) -> list[np.ndarray]:
    """-> list of (np+1, size) arrays (Mmg layout)."""
    lib = N.load()
    n = C.c_int64()
    nsol = C.c_int()
    types = (C.c_int * 8)()
    if not lib.pmx_medit_sol_info(path.encode(), C.byref(n), C.byref(nsol), types):
        _err("pmx_medit_sol_info")
    out = [np.zeros((n.value + 1, _SIZE[types[s]])) for s in range(nsol.value)]
    ptrs = (N.dptr * len(out))(*[a.ctypes.data_as(N.dptr) for a in out])
    if not lib.pmx_medit_sol_read(path.encode(), n, nsol, types, ptrs):
        _err("pmx_medit_sol_read")
    return out


def write_sol(path: str, sols: list[np.ndarray]):
    lib = N.load()
    arr = [np.ascontiguousarray(s, np.float64) for s in sols]
    n = arr[0].shape[0] - 1
    types = (C.c_int * len(arr))(*[_TYPE[a.shape[1]] for a in arr])
    ptrs = (N.dptr * len(arr))(*[a.ctypes.data_as(N.dptr) for a in arr])
    if not lib.pmx_medit_sol_write(path.encode(), n, len(arr), types, ptrs):
        _err("pmx_medit_sol_write")
