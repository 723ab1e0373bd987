"""ctypes wrapper of oracle/liboracle.so -- the CPU restatement of the reference
transfer path.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, always as the checker.  PARITY UNPINNED (see
pmx_oracle.h and DESIGN.md).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "liboracle.so")
_lib = None

vp, i64 = C.c_void_p, C.c_int64


class QualStats(C.Structure):
    _fields_ = [("ne", i64), ("max", C.c_double), ("min", C.c_double), ("avg", C.c_double),
                ("iel", i64), ("good", i64), ("med", i64), ("his", i64 * 5), ("nrid", i64)]


class LenStats(C.Structure):
    _fields_ = [("ned", i64), ("nullEdge", i64), ("avlen", C.c_double), ("lmin", C.c_double),
                ("lmax", C.c_double), ("amin", i64), ("bmin", i64), ("amax", i64), ("bmax", i64),
                ("hl", i64 * 9)]


class Surface(C.Structure):
    """orc_surface: Mmg's surface data (xTetra edge tags, point / xPoint normals)."""
    _fields_ = [("xt", C.c_void_p), ("xtag", C.c_void_p), ("n", C.c_void_p), ("xp", C.c_void_p),
                ("n1", C.c_void_p), ("n2", C.c_void_p)]


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            import sys
            sys.path.insert(0, os.path.dirname(_HERE))
            from parmmg_amd import build
            build.build_oracle()
        lib = C.CDLL(LIB)
        lib.orc_create.restype = vp
        lib.orc_create.argtypes = [i64, i64, i64, vp, vp, vp, vp, vp, C.c_double]
        lib.orc_destroy.argtypes = [vp]
        lib.orc_reset.argtypes = [vp]
        lib.orc_locate_vol.argtypes = [vp, vp, vp, vp, vp]
        lib.orc_locate_bdy.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp]
        lib.orc_tet_contains.argtypes = [vp, C.c_int, vp, vp]
        lib.orc_tria_contains.argtypes = [vp, C.c_int, vp]
        lib.orc_invmat.argtypes = [vp, vp]
        lib.orc_interp_points.argtypes = [vp, i64, vp, vp, vp, C.c_int, vp, vp, vp, C.c_int,
                                          vp, vp, C.c_int, vp, vp, vp, vp, vp]
        lib.orc_constant_size.argtypes = [i64, C.c_int, C.c_double, vp]
        lib.orc_tetra_qual.argtypes = [i64, vp, vp, vp, C.c_int, vp]
        lib.orc_tetra_qual_rid.argtypes = [i64, vp, vp, vp, C.c_int, vp, C.c_int, vp]
        lib.orc_qualhisto.argtypes = [i64, vp, vp, C.POINTER(QualStats)]
        lib.orc_qualhisto_tags.argtypes = [i64, vp, vp, vp, C.POINTER(QualStats)]
        lib.orc_prilen.restype = C.c_int
        lib.orc_prilen.argtypes = [i64, i64, vp, vp, vp, C.c_int, C.POINTER(LenStats)]
        lib.orc_prilen_full.restype = C.c_int
        lib.orc_prilen_full.argtypes = [i64, i64, vp, vp, vp, C.c_int, vp, C.c_int, C.POINTER(Surface), i64,
                                        vp, vp, vp, vp, C.c_int, C.c_int, C.POINTER(LenStats)]
        lib.orc_prilen_dist.restype = C.c_int
        lib.orc_prilen_dist.argtypes = [i64, i64, vp, vp, vp, C.c_int, vp, i64, vp, vp, vp, C.c_int,
                                        C.c_int, C.POINTER(LenStats)]
        _lib = lib
    return _lib


def _p(a):
    return C.c_void_p(a.ctypes.data) if a is not None else None


class Oracle:
    """Reference-semantics CPU transfer on one background group."""

    def __init__(self, mesh):
        self.lib = load()
        self.m = mesh
        self.ctx = self.lib.orc_create(mesh.np, mesh.ne, mesh.nt, _p(mesh.xyz), _p(mesh.tet),
                                       _p(mesh.adja), _p(mesh.tria) if mesh.nt else None,
                                       _p(mesh.adjt) if mesh.nt else None, mesh.hausd)

    def __del__(self):
        if getattr(self, "ctx", None):
            self.lib.orc_destroy(self.ctx)
            self.ctx = None

    def tet_contains(self, k: int, p) -> tuple[bool, float]:
        p = np.ascontiguousarray(p, np.float64)
        lm = np.zeros(1)
        r = self.lib.orc_tet_contains(self.ctx, int(k), _p(p), _p(lm))
        return bool(r), float(lm[0])

    def tria_contains(self, k: int, p) -> bool:
        p = np.ascontiguousarray(p, np.float64)
        return bool(self.lib.orc_tria_contains(self.ctx, int(k), _p(p)))

    def interp(self, xyz, tags, sols, imet=0, order=None, start_vol=None, start_bdy=None,
               fresh=False, init=None):
        """Returns (outs, elem, status, steps, edge, vertex); outs[s] is (npts, size)."""
        xyz = np.ascontiguousarray(xyz, np.float64)
        n = xyz.shape[0]
        tags = np.ascontiguousarray(tags if tags is not None else np.zeros(n), np.int32)
        sols = [np.ascontiguousarray(s, np.float64) for s in sols]
        sizes = np.array([s.shape[1] for s in sols], np.int32)
        outs = []
        for i, s in enumerate(sols):
            a = (np.array(init[i], np.float64, copy=True).reshape(n, s.shape[1]) if init is not None
                 else np.full((n, s.shape[1]), np.nan))
            outs.append(a)
        oldp = (C.c_void_p * max(len(sols), 1))(*[s.ctypes.data for s in sols])
        newp = (C.c_void_p * max(len(sols), 1))(*[a.ctypes.data for a in outs])
        elem = np.zeros(n, np.int32)
        status = np.zeros(n, np.int32)
        steps = np.zeros(n, np.int32)
        edge = np.full(n, -1, np.int32)
        vertex = np.full(n, -1, np.int32)
        od = np.ascontiguousarray(order, np.int64) if order is not None else None
        sv = np.ascontiguousarray(start_vol, np.int32) if start_vol is not None else None
        sb = np.ascontiguousarray(start_bdy, np.int32) if start_bdy is not None else None
        # order: the points to process, in that order (a subset is allowed)
        cnt = len(od) if od is not None else n
        self.lib.orc_interp_points(self.ctx, cnt, _p(xyz), _p(tags), _p(od), len(sols), _p(sizes),
                                   oldp, newp, imet if sols else -1, _p(sv), _p(sb), int(fresh),
                                   _p(elem), _p(status), _p(steps), _p(edge), _p(vertex))
        return outs, elem, status, steps, edge, vertex


def invmat(m):
    lib = load()
    m = np.ascontiguousarray(m, np.float64)
    mi = np.full(6, np.nan)
    ok = lib.orc_invmat(_p(m), _p(mi))
    return bool(ok), mi


def tetra_qual(mesh, met=None, tags=None, met_rid_typ=0):
    """MMG3D_tetraQual(mesh, met, metRidTyp); tags (np+1,) MMG5_Point.tag: the
    ridge points MMG5_moymet leaves out for metRidTyp 1 with a tensor metric."""
    lib = load()
    q = np.zeros(mesh.ne + 1)
    msize = met.shape[1] if met is not None else 0
    m = np.ascontiguousarray(met, np.float64) if met is not None else None
    t = None if tags is None else np.ascontiguousarray(tags, np.uint16)
    lib.orc_tetra_qual_rid(mesh.ne, _p(mesh.xyz), _p(mesh.tet), _p(m), msize, _p(t), int(met_rid_typ), _p(q))
    return q


def qualhisto(mesh, qual, tags=None):
    """MMG3D_computeInqua statistics; with point tags, MMG3D_computeOutqua's nrid."""
    lib = load()
    st = QualStats()
    t = None if tags is None else np.ascontiguousarray(tags, np.uint16)
    lib.orc_qualhisto_tags(mesh.ne, _p(mesh.tet), _p(np.ascontiguousarray(qual)), _p(t), C.byref(st))
    d = {f: getattr(st, f) for f, _ in QualStats._fields_}
    d["his"] = list(st.his)
    return d


def prilen(mesh, met, tags=None, par=None, met_rid_typ=0, surface=None):
    """PMMG_prilen: centralized (par None) or PMMG_computePrilen with parallel
    edges par = {"a", "b", "owner", "myrank", "exact_once", "tag" (optional)}.
    surface: Mmg's surface data {"xt" (ne+1,), "xtag" (nxt+1, 6), "n" (np+1, 3),
    "xp" (np+1,), "n1"/"n2" (nxp+1, 3)} (None: no xTetra, zero normals)."""
    lib = load()
    st = LenStats()
    m = np.ascontiguousarray(met, np.float64)
    t = None if tags is None else np.ascontiguousarray(tags, np.uint16)
    if par is None:
        pa = pb = po = pt = None
        npar, myrank, once = 0, 0, 0
    else:
        pa = np.ascontiguousarray(par["a"], np.int32)
        pb = np.ascontiguousarray(par["b"], np.int32)
        po = np.ascontiguousarray(par["owner"], np.int32)
        pt = None if par.get("tag") is None else np.ascontiguousarray(par["tag"], np.uint16)
        npar, myrank, once = len(pa), int(par.get("myrank", 0)), int(par.get("exact_once", 0))
    keep = []
    sp = None
    if surface is not None:
        sf = Surface()
        for f, dt in (("xt", np.int32), ("xtag", np.uint16), ("n", np.float64), ("xp", np.int32),
                      ("n1", np.float64), ("n2", np.float64)):
            a = surface.get(f)
            if a is not None:
                a = np.ascontiguousarray(a, dt)
                keep.append(a)
                setattr(sf, f, a.ctypes.data)
        sp = C.byref(sf)
    lib.orc_prilen_full(mesh.np, mesh.ne, _p(mesh.xyz), _p(mesh.tet), _p(m), m.shape[1], _p(t), met_rid_typ,
                        sp, npar, _p(pa), _p(pb), _p(po), _p(pt), myrank, once, C.byref(st))
    d = {f: getattr(st, f) for f, _ in LenStats._fields_}
    d["hl"] = list(st.hl)
    return d


def count_nodes(mesh, idx_ip, idx_comm, intvalues, base=1):
    """PMMG_count_nodes_par (reference src/quality_pmmg.c:33-80), restated in
    Python for small cases: intvalues updated in place; returns np."""
    flag = np.zeros(mesh.np + 1, bool)
    n = 0
    for ip, idx in zip(idx_ip, idx_comm):
        if not intvalues[idx]:
            intvalues[idx] = base
            n += 1
        flag[ip] = True
    for k in range(1, mesh.ne + 1):
        v = mesh.tet[k]
        if v[0] <= 0:
            continue
        for ip in v:
            if not flag[ip]:
                flag[ip] = True
                n += 1
    return n
