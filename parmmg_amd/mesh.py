"""Background-mesh container and synthetic inputs (Kuhn cubes, new points, fields).

Arrays follow Mmg's 1-based convention (row 0 unused), exactly what
``PMMG_create_oldGrp`` leaves in ``old_listgrp`` (reference
src/grpsplit_pmmg.c:207-418): tets, the tet adjacency ``adja``
(``adja[4*(k-1)+1+f] = 4*k'+f'``), boundary triangles and their adjacency
``adjt`` (``adjt[3*(k-1)+1+e] = 3*k'+e'``).

The generator and the Medit reader are test/bench utilities built in
``libpmx_meshgen.so``; they are not part of the transfer path.
"""
from __future__ import annotations

import ctypes as C
import dataclasses
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
MESHGEN_PATH = os.path.join(_HERE, "libpmx_meshgen.so")

TAG_REQ, TAG_BDY, TAG_NUL = 4, 16, 16384

# Mmg's point and tet records (MMG5_Point 72 B, MMG5_Tetra 48 B, libmmgtypes.h)
# for the AoS views of the binding
MMG_POINT = np.dtype([("c", "f8", 3), ("n", "f8", 3), ("ref", "i4"), ("xp", "i4"), ("tmp", "i4"),
                      ("flag", "i4"), ("s", "i4"), ("tag", "u2"), ("tagdel", "i1"), ("pad", "i1")])
MMG_TETRA = np.dtype([("qual", "f8"), ("v", "i4", 4), ("ref", "i4"), ("base", "i4"), ("mark", "i4"),
                      ("xt", "i4"), ("flag", "i4"), ("tag", "i2"), ("pad", "i2")])

_mg = None


def cpu_share() -> int:
    """CPUs this process may use: its affinity set capped by the cgroup v2
    quota (cpu.max; a GPU box: 16 of 256) -- the generator's OpenMP team."""
    try:
        k = len(os.sched_getaffinity(0))
    except AttributeError:
        k = os.cpu_count() or 1
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            k = min(k, max(1, -(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return max(1, k)


def _meshgen() -> C.CDLL:
    global _mg
    if _mg is None:
        if not os.path.exists(MESHGEN_PATH):
            from . import build
            build.build_meshgen()
        lib = C.CDLL(MESHGEN_PATH)
        i64, vp = C.c_int64, C.c_void_p
        lib.pmg_kuhn_counts.argtypes = [C.c_int, C.POINTER(i64), C.POINTER(i64), C.POINTER(i64)]
        lib.pmg_kuhn_cube.restype = i64
        lib.pmg_kuhn_cube.argtypes = [C.c_int, C.c_uint64, C.c_double, vp, vp, vp, vp, vp]
        lib.pmg_build_adja.restype = i64
        lib.pmg_build_adja.argtypes = [i64, vp, vp]
        lib.pmg_build_bdry.restype = i64
        lib.pmg_build_bdry.argtypes = [i64, vp, vp, vp, i64]
        lib.pmg_build_adjt.restype = C.c_int
        lib.pmg_build_adjt.argtypes = [i64, vp, vp]
        lib.pmg_new_points_count.restype = i64
        lib.pmg_new_points_count.argtypes = [C.c_int, C.c_int]
        lib.pmg_new_points.restype = i64
        lib.pmg_new_points.argtypes = [C.c_int, C.c_uint64, C.c_double, C.c_int, C.c_int, vp, vp]
        lib.pmg_count_inverted.restype = i64
        lib.pmg_count_inverted.argtypes = [i64, vp, vp]
        lib.pmg_set_threads.argtypes = [C.c_int]
        lib.pmg_set_threads(cpu_share())
        _mg = lib
    return _mg


def _p(a: np.ndarray) -> C.c_void_p:
    return C.c_void_p(a.ctypes.data)


@dataclasses.dataclass
class Mesh:
    xyz: np.ndarray            # (np+1, 3) float64
    tet: np.ndarray            # (ne+1, 4) int32
    adja: np.ndarray           # (4*ne+5,) int32
    tria: np.ndarray           # (nt+1, 3) int32
    adjt: np.ndarray           # (3*nt+4,) int32
    hausd: float = 0.01        # Mmg default hausd

    @property
    def np(self) -> int:
        return self.xyz.shape[0] - 1

    @property
    def ne(self) -> int:
        return self.tet.shape[0] - 1

    @property
    def nt(self) -> int:
        return self.tria.shape[0] - 1

    def centroids(self) -> np.ndarray:
        return self.xyz[self.tet[1:]].mean(axis=1)


def kuhn_cube(n: int, seed: int = 20250117, jitter: float = 0.15) -> Mesh:
    """Jittered Kuhn cube [0,1]^3 with n cells per axis (ne = 6 n^3)."""
    lib = _meshgen()
    np_, ne, nt = C.c_int64(), C.c_int64(), C.c_int64()
    lib.pmg_kuhn_counts(n, C.byref(np_), C.byref(ne), C.byref(nt))
    xyz = np.zeros((np_.value + 1, 3), np.float64)
    tet = np.zeros((ne.value + 1, 4), np.int32)
    adja = np.zeros(4 * ne.value + 5, np.int32)
    tria = np.zeros((nt.value + 1, 3), np.int32)
    adjt = np.zeros(3 * nt.value + 4, np.int32)
    r = lib.pmg_kuhn_cube(n, seed, jitter, _p(xyz), _p(tet), _p(adja), _p(tria), _p(adjt))
    if r != nt.value:
        raise RuntimeError("pmg_kuhn_cube failed")
    return Mesh(xyz, tet, adja, tria, adjt)


def from_tets(xyz1: np.ndarray, tet1: np.ndarray, hausd: float = 0.01) -> Mesh:
    """Build adja, boundary trias and adjt for an arbitrary tet mesh.
    xyz1 (np+1,3) and tet1 (ne+1,4) are 1-based (row 0 unused)."""
    lib = _meshgen()
    xyz = np.ascontiguousarray(xyz1, np.float64)
    tet = np.ascontiguousarray(tet1, np.int32)
    ne = tet.shape[0] - 1
    adja = np.zeros(4 * ne + 5, np.int32)
    if lib.pmg_build_adja(ne, _p(tet), _p(adja)) != 0:
        raise ValueError("non-manifold tet mesh")
    maxnt = 4 * ne
    tria = np.zeros((maxnt + 1, 3), np.int32)
    nt = lib.pmg_build_bdry(ne, _p(tet), _p(adja), _p(tria), maxnt)
    tria = np.ascontiguousarray(tria[: nt + 1])
    adjt = np.zeros(3 * nt + 4, np.int32)
    lib.pmg_build_adjt(nt, _p(tria), _p(adjt))
    return Mesh(xyz, tet, adja, tria, adjt, hausd)


def new_points(n: int, seed: int = 12345, jitter: float = 0.3, surface: bool = True,
               morton: bool = True) -> tuple[np.ndarray, np.ndarray]:
    """New vertices for an n-cube: jittered cell centres (volume, tag 0) and
    jittered face-cell centres on the 6 faces (tag MG_BDY), Morton ordered."""
    lib = _meshgen()
    cnt = lib.pmg_new_points_count(n, int(surface))
    xyz = np.zeros((cnt, 3), np.float64)
    tag = np.zeros(cnt, np.int32)
    r = lib.pmg_new_points(n, seed, jitter, int(surface), int(morton), _p(xyz), _p(tag))
    if r != cnt:
        raise RuntimeError("pmg_new_points failed")
    return xyz, tag.astype(np.uint16)


def new_point_tets(n: int, xyz: np.ndarray, tag: np.ndarray) -> np.ndarray:
    """Tets over the new points of new_points(n) in Mmg's layout ((ne+1, 4),
    1-based point indices, row 0 unused), for the reference's vertex loop
    over the new mesh's tets (src/interpmesh_pmmg.c:535-541): a Kuhn mesh of
    the lattice of cell-centre points (6 (n-1)^3 tets, cells in Morton order
    like the points: one space-filling numbering of both, as a Scotch
    renumbering gives) plus one tet per surface point joining it to the
    adjacent centres.
    Every point is in a tet (no orphans); the tets only enumerate vertices,
    they are not a conforming mesh of the surface layer."""
    x = np.asarray(xyz)
    ijk = np.clip(np.floor(x * n).astype(np.int64), 0, n - 1)
    bdy = (np.asarray(tag) & TAG_BDY) != 0
    vol = ~bdy
    idx = np.zeros((n, n, n), np.int64)
    vi = np.nonzero(vol)[0]
    idx[ijk[vi, 0], ijk[vi, 1], ijk[vi, 2]] = vi + 1
    c = np.arange(n - 1)
    I, J, K = np.meshgrid(c, c, c, indexing="ij")
    I, J, K = I.ravel(), J.ravel(), K.ravel()
    code = np.zeros(len(I), np.int64)
    for b in range(12):
        code |= (((I >> b) & 1) << (3 * b)) | (((J >> b) & 1) << (3 * b + 1)) | (((K >> b) & 1) << (3 * b + 2))
    o = np.argsort(code, kind="stable")
    I, J, K = I[o], J[o], K[o]
    e = np.eye(3, dtype=np.int64)
    tets = []
    for perm in ((0, 1, 2), (0, 2, 1), (1, 0, 2), (1, 2, 0), (2, 0, 1), (2, 1, 0)):
        p = np.stack([I, J, K], 1)
        vs = [idx[p[:, 0], p[:, 1], p[:, 2]]]
        for a in perm:
            p = p + e[a]
            vs.append(idx[p[:, 0], p[:, 1], p[:, 2]])
        tets.append(np.stack(vs, 1))
    kt = np.stack(tets, 1).reshape(-1, 4)          # the 6 tets of a cell together
    bi = np.nonzero(bdy)[0]
    b = ijk[bi]
    on = np.argmax((x[bi] == 0.0) | (x[bi] == 1.0), axis=1)   # the face's normal axis
    tt = [bi + 1]
    for d in range(3):
        p = b.copy()
        if d > 0:
            ax = (on + d) % 3
            r = np.arange(len(bi))
            p[r, ax] = np.where(p[r, ax] < n - 1, p[r, ax] + 1, p[r, ax] - 1)
        tt.append(idx[p[:, 0], p[:, 1], p[:, 2]])
    st = np.stack(tt, 1)
    out = np.zeros((1 + len(kt) + len(st), 4), np.int32)
    out[1:1 + len(kt)] = kt
    out[1 + len(kt):] = st
    return out


def count_inverted(m: Mesh) -> int:
    return int(_meshgen().pmg_count_inverted(m.ne, _p(m.xyz), _p(m.tet)))


# ---- analytic fields ----------------------------------

def renumber(m: Mesh, tperm: np.ndarray, vperm: np.ndarray | None = None):
    """The same mesh with its tets (and vertices) renumbered: tperm / vperm
    map new -> old (0-based over 1..ne / 1..np; vperm None: vertices kept).
    The adjacency is permuted, not rebuilt.  Returns (mesh, tinv) with
    tinv[old tet] = new tet."""
    ne, np_ = m.ne, m.np
    if vperm is None:
        vinv = np.arange(np_ + 1, dtype=np.int32)
        xyz = m.xyz
    else:
        vinv = np.zeros(np_ + 1, np.int32)
        vinv[vperm + 1] = np.arange(1, np_ + 1, dtype=np.int32)
        xyz = np.empty_like(m.xyz)
        xyz[0] = m.xyz[0]
        xyz[1:] = m.xyz[vperm + 1]
    tinv = np.zeros(ne + 1, np.int64)
    tinv[tperm + 1] = np.arange(1, ne + 1)
    tet = np.zeros_like(m.tet)
    tet[1:] = vinv[m.tet[tperm + 1]]
    old = m.adja[1:4 * ne + 1].reshape(ne, 4)[tperm]
    k, f = old >> 2, old & 3
    adja = np.zeros_like(m.adja)
    adja[1:4 * ne + 1] = np.where(old > 0, 4 * tinv[k] + f, 0).astype(np.int32).ravel()
    tria = vinv[m.tria]
    tria[0] = 0
    return Mesh(xyz, tet, adja, tria, m.adjt.copy(), m.hausd), tinv


def numbering(m: Mesh, kind: str, seed: int = 7, frac: float = 0.1):
    """Background tet numberings of the bench: "lex" the
    generator's cell-lexicographic order (a Scotch-renumbered Mmg mesh);
    "shuffle" the tets in random order (seed 7, vertices kept); "appended" 10 %
    of the tets, chosen at random, moved to the end in their order (what Mmg's
    insertions do to a numbering between renumberings; `frac` of them for
    the record-format A/B).  Returns (mesh, tinv or None)."""
    if kind == "lex":
        return m, None
    rng = np.random.default_rng(seed)
    if kind == "shuffle":
        tp = rng.permutation(m.ne)
    elif kind == "appended":
        moved = np.zeros(m.ne, bool)
        nmov = m.ne // 10 if frac == 0.1 else int(m.ne * frac)
        moved[rng.choice(m.ne, nmov, replace=False)] = True
        tp = np.concatenate([np.nonzero(~moved)[0], np.nonzero(moved)[0]])
    else:
        raise ValueError(f"unknown numbering {kind}")
    return renumber(m, tp)


def wrec_escapes(m: Mesh) -> int:
    """Tets whose walk record escapes whole (pmx_wrec.h): a vertex delta from
    v[0] outside [-2^19, 2^19); the walk reads those from the 32-B records."""
    t = m.tet[1:].astype(np.int64)
    valid = t[:, 0] > 0
    dv = t[:, 1:] - t[:, :1]
    esc = np.any((dv < -(1 << 19)) | (dv >= (1 << 19)), axis=1)
    return int(np.count_nonzero(esc & valid))


def wrec_far_fields(m: Mesh):
    """Neighbour fields of the walk records that escape alone (pmx_wrec.h): a
    delta from the tet index outside (-2^23 + 1, 2^23), the walk reading that
    neighbour from the 32-B record when it crosses the face.  Returns (far
    fields, tets with one or more)."""
    t = m.tet[1:].astype(np.int64)
    valid = t[:, 0] > 0
    nb = (m.adja[1:4 * m.ne + 1].reshape(m.ne, 4) >> 2).astype(np.int64)
    dn = nb - np.arange(1, m.ne + 1, dtype=np.int64)[:, None]
    far = (nb != 0) & ((dn <= -(1 << 23) + 1) | (dn >= (1 << 23))) & valid[:, None]
    return int(np.count_nonzero(far)), int(np.count_nonzero(far.any(axis=1)))


def iso_metric(x: np.ndarray) -> np.ndarray:
    """h(x) = 0.05 + 0.1 x0, shape (n, 1)."""
    return (0.05 + 0.1 * x[:, 0])[:, None]


def graded_iso_metric(n: int):
    """h(x) = (1.2 / n) exp(1.6 (x0 + x1 + x2 - 1.5)) on a Kuhn cube of n
    cells per axis: metric edge lengths l / h from about 0.04 to 20, so every
    bin of PMMG_prilen's histogram (bounds 0.3 ... 5) is populated -- a
    statistics workload that is not one bin (shape (n, 1))."""
    def f(x: np.ndarray) -> np.ndarray:
        return ((1.2 / n) * np.exp(1.6 * (x.sum(axis=1) - 1.5)))[:, None]
    return f


def shock_metric(x: np.ndarray) -> np.ndarray:
    """Anisotropic shock metric across the plane n.x = 0.5, n = (1,1,1)/sqrt(3);
    stored (m11, m12, m13, m22, m23, m33), shape (n, 6)."""
    nv = np.full(3, 1.0 / np.sqrt(3.0))
    d = x @ nv - 0.5
    hn = np.minimum(0.1, 0.002 + 0.2 * np.abs(d))
    ht = 0.05
    a = 1.0 / hn**2
    b = 1.0 / ht**2
    nn = np.outer(nv, nv)
    out = np.empty((x.shape[0], 6))
    idx = [(0, 0), (0, 1), (0, 2), (1, 1), (1, 2), (2, 2)]
    for j, (p, q) in enumerate(idx):
        out[:, j] = a * nn[p, q] + b * ((1.0 if p == q else 0.0) - nn[p, q])
    return out


def level_set(x: np.ndarray) -> np.ndarray:
    return (np.linalg.norm(x - 0.5, axis=1) - 0.3)[:, None]


def velocity(x: np.ndarray) -> np.ndarray:
    px, py = np.pi * x[:, 0], np.pi * x[:, 1]
    return np.stack([np.sin(px) * np.cos(py), -np.cos(px) * np.sin(py), np.zeros(x.shape[0])], axis=1)


def on_vertices(m: Mesh, f) -> np.ndarray:
    """Evaluate f on the mesh vertices; row 0 (unused) is zero."""
    v = f(m.xyz[1:])
    out = np.zeros((m.np + 1, v.shape[1]))
    out[1:] = v
    return out


# ---- Medit .mesh reader (fixtures) ----------------------------------------------

def read_medit(path: str, hausd: float = 0.01) -> Mesh:
    """Read Vertices and Tetrahedra of an ASCII Medit file and rebuild the
    background structures (adja, boundary trias, adjt)."""
    with open(path) as f:
        tok = f.read().split()
    i = 0
    xyz = tet = None
    while i < len(tok):
        t = tok[i]
        if t == "Vertices":
            n = int(tok[i + 1])
            a = np.array(tok[i + 2: i + 2 + 4 * n], dtype=np.float64).reshape(n, 4)
            xyz = np.zeros((n + 1, 3))
            xyz[1:] = a[:, :3]
            i += 2 + 4 * n
        elif t == "Tetrahedra":
            n = int(tok[i + 1])
            a = np.array(tok[i + 2: i + 2 + 5 * n], dtype=np.int64).reshape(n, 5)
            tet = np.zeros((n + 1, 4), np.int32)
            tet[1:] = a[:, :4]
            i += 2 + 5 * n
        else:
            i += 1
    if xyz is None or tet is None:
        raise ValueError(f"{path}: no Vertices/Tetrahedra")
    return from_tets(xyz, tet, hausd)


def read_medit_sol(path: str) -> list[np.ndarray]:
    """Read SolAtVertices of an ASCII .sol file -> list of (np+1, size) arrays
    (types 1 scalar, 2 vector, 3 tensor)."""
    with open(path) as f:
        tok = f.read().split()
    i = tok.index("SolAtVertices")
    n = int(tok[i + 1])
    nsol = int(tok[i + 2])
    types = [int(t) for t in tok[i + 3: i + 3 + nsol]]
    sizes = [{1: 1, 2: 3, 3: 6}[t] for t in types]
    vals = np.array(tok[i + 3 + nsol: i + 3 + nsol + n * sum(sizes)], dtype=np.float64)
    vals = vals.reshape(n, sum(sizes))
    out, off = [], 0
    for s in sizes:
        a = np.zeros((n + 1, s))
        a[1:] = vals[:, off: off + s]
        if s == 6:   # Medit (11,12,22,13,23,33) -> Mmg (11,12,13,22,23,33)
            a[1:, 2], a[1:, 3] = vals[:, off + 3], vals[:, off + 2]
        out.append(a)
        off += s
    return out


# ---- Medit writers (the wire format of ParMmg's
# src/inout_pmmg.c via Mmg's MMG3D_saveMesh / MMG3D_saveSol) ----------------------

_MEDIT_TYPE = {1: 1, 3: 2, 6: 3}     # solution size -> Medit type (scalar, vector, tensor)


def write_medit(path: str, m: Mesh, required=None) -> None:
    """ASCII Medit mesh: Vertices (ref 0), Tetrahedra (ref 0), the boundary
    Triangles and, if given, RequiredVertices (1-based indices; the MG_REQ
    points that the transfer copies instead of interpolating).  Coordinates
    in %.17g, so read_medit(write_medit(m)) is bit-identical."""
    with open(path, "w") as f:
        f.write("MeshVersionFormatted 2\n\nDimension 3\n\n")
        f.write(f"Vertices\n{m.np}\n")
        f.writelines(f"{x:.17g} {y:.17g} {z:.17g} 0\n" for x, y, z in m.xyz[1:])
        f.write(f"\nTetrahedra\n{m.ne}\n")
        f.writelines(f"{a} {b} {c} {d} 0\n" for a, b, c, d in m.tet[1:])
        if m.nt:
            f.write(f"\nTriangles\n{m.nt}\n")
            f.writelines(f"{a} {b} {c} 0\n" for a, b, c in m.tria[1:])
        if required is not None and len(required):
            f.write(f"\nRequiredVertices\n{len(required)}\n")
            f.writelines(f"{int(i)}\n" for i in required)
        f.write("\nEnd\n")


def read_medit_required(path: str) -> np.ndarray:
    """1-based indices listed under RequiredVertices (empty if none)."""
    with open(path) as f:
        tok = f.read().split()
    if "RequiredVertices" not in tok:
        return np.zeros(0, np.int64)
    i = tok.index("RequiredVertices")
    n = int(tok[i + 1])
    return np.array(tok[i + 2: i + 2 + n], dtype=np.int64)


def write_medit_sol(path: str, sols: list[np.ndarray]) -> None:
    """ASCII SolAtVertices of (np+1, size) arrays (row 0 unused, like
    read_medit_sol returns them); tensors from Mmg (11,12,13,22,23,33) to
    Medit (11,12,22,13,23,33) order."""
    n = sols[0].shape[0] - 1
    cols = []
    for s in sols:
        a = np.asarray(s, np.float64)[1:]
        if a.shape[1] == 6:
            a = a[:, [0, 1, 3, 2, 4, 5]]
        cols.append(a)
    vals = np.concatenate(cols, axis=1) if cols else np.zeros((n, 0))
    types = " ".join(str(_MEDIT_TYPE[s.shape[1]]) for s in sols)
    with open(path, "w") as f:
        f.write("MeshVersionFormatted 2\n\nDimension 3\n\n")
        f.write(f"SolAtVertices\n{n}\n{len(sols)} {types}\n")
        f.writelines(" ".join(f"{v:.17g}" for v in row) + "\n" for row in vals)
        f.write("\nEnd\n")
