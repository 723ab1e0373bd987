"""Shared case builders and parity checks for the transfer-path tests."""
from __future__ import annotations

import numpy as np

from parmmg_amd import mesh as M

# Parity tolerances (BASELINE.json north_star): located elements bit-exact except
# on documented ties; interpolated fields bit-exact when the element is the same
# (identical operation order, no FMA), and within TIE_TOL * local range when a
# documented tie put the point in a different (also containing) element:
# the barycentric inside test admits lambda_min > -1e-6, so two containing
# elements can differ by up to ~1e-6 of the field jump.
TIE_TOL = 4e-6


def lin_field(x):
    return (1.0 + 2.0 * x[:, 0] - 3.0 * x[:, 1] + 0.5 * x[:, 2])[:, None]


def cube_case(n: int, metric: str = "iso", surface: bool = True, fields: bool = True,
              seed_pts: int = 12345):
    m = M.kuhn_cube(n)
    x, t = M.new_points(n, seed=seed_pts, surface=surface)
    sols = []
    if metric == "iso":
        sols.append(M.on_vertices(m, M.iso_metric))
    elif metric == "ani":
        sols.append(M.on_vertices(m, M.shock_metric))
    if fields:
        sols += [M.on_vertices(m, M.level_set), M.on_vertices(m, M.velocity),
                 M.on_vertices(m, lin_field)]
    return m, x, t, sols


def split_partitions(m, cut: float = 0.5):
    """Two ParMmg partitions of a mesh (tets with centroid x < cut, the rest),
    each renumbered locally, and their parallel (interface) edges in local
    numbering: [(mesh_r, glob_r, par_r)] with par_r = {"a", "b", "owner"},
    owner = the lowest rank sharing the edge (0), orientation (min, max) of
    the global ids (the same edge on both sides)."""
    IARE = [(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)]
    c = m.centroids()
    sides = [np.nonzero(c[:, 0] < cut)[0] + 1, np.nonzero(c[:, 0] >= cut)[0] + 1]
    edges = []
    for ks in sides:
        t = m.tet[ks]
        e = np.concatenate([np.sort(t[:, [i, j]], axis=1) for i, j in IARE])
        edges.append(set(map(tuple, e)))
    shared = sorted(edges[0] & edges[1])
    out = []
    for r, ks in enumerate(sides):
        glob = np.unique(m.tet[ks].ravel())                  # local ip -> global, 0-based
        loc = np.zeros(m.np + 1, np.int32)
        loc[glob] = np.arange(1, len(glob) + 1)
        xyz = np.zeros((len(glob) + 1, 3))
        xyz[1:] = m.xyz[glob]
        tet = np.zeros((len(ks) + 1, 4), np.int32)
        tet[1:] = loc[m.tet[ks]]
        mr = M.from_tets(xyz, tet)
        par = {"a": np.array([loc[a] for a, b in shared], np.int32),
               "b": np.array([loc[b] for a, b in shared], np.int32),
               "owner": np.zeros(len(shared), np.int32), "myrank": r}
        out.append((mr, np.concatenate([[0], glob]), par))
    return out, len(shared)


def first_visit_order(tets_mmg: np.ndarray, npts: int) -> np.ndarray:
    """The order in which the reference's vertex loop reaches the new points
    (src/interpmesh_pmmg.c:535-544): new tets ie = 1..ne, valid ones only
    (MG_EOK: v[0] > 0), their vertices iloc = 0..3, each point at its first
    visit.  tets_mmg: (ne+1, 4), Mmg layout (1-based, row 0 unused); returns
    0-based point indices (points in no valid tet are not visited).  The
    oracle given this order runs the reference's sequential loop: the start
    tet / tria and the surface point flags carry over along it."""
    t = np.asarray(tets_mmg)[1:]
    flat = t[t[:, 0] > 0].ravel().astype(np.int64) - 1
    flat = flat[(flat >= 0) & (flat < npts)]
    _, first = np.unique(flat, return_index=True)
    return flat[np.sort(first)]


def bits_equal(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Row-wise bitwise equality of float64 arrays (NaN == NaN)."""
    a = np.ascontiguousarray(a, np.float64).view(np.int64)
    b = np.ascontiguousarray(b, np.float64).view(np.int64)
    return (a == b).reshape(a.shape[0], -1).all(axis=1)


def compare_volume(orc, x, tags, gpu, ref, sols):
    """gpu/ref: (outs, elem, status).  Returns dict of counts; asserts parity."""
    outs_g, elem_g, st_g = gpu
    outs_r, elem_r, st_r = ref
    vol = np.nonzero(tags == 0)[0]
    same = vol[elem_g[vol] == elem_r[vol]]
    diff = vol[elem_g[vol] != elem_r[vol]]
    for s in range(len(sols)):
        ok = bits_equal(outs_g[s][same], outs_r[s][same])
        assert ok.all(), f"sol {s}: {np.count_nonzero(~ok)} same-element points differ bitwise"
    # found-vs-closest is path independent
    assert np.array_equal(st_g[vol] != 0, st_r[vol] != 0), "found/closest status differs"
    ties = 0
    for i in diff:
        if st_r[i] == 0:
            raise AssertionError(f"point {i}: closest element differs ({elem_g[i]} vs {elem_r[i]})")
        cg, _ = orc.tet_contains(int(elem_g[i]), x[i])
        cr, _ = orc.tet_contains(int(elem_r[i]), x[i])
        assert cg and cr, f"point {i}: GPU tet {elem_g[i]} / oracle tet {elem_r[i]} not a tie"
        for s in range(len(sols)):
            rng = np.abs(sols[s][1:]).max() + 1e-300
            assert np.all(np.abs(outs_g[s][i] - outs_r[s][i]) <= TIE_TOL * rng + 1e-12 * rng)
        ties += 1
    return {"nvol": len(vol), "same": len(same), "ties": ties}


def compare_exact(gpu, ref, idx, nsol):
    """Bit-exact comparison of every per-point output on index set idx."""
    outs_g, elem_g, st_g, edge_g, vert_g = gpu
    outs_r, elem_r, st_r, edge_r, vert_r = ref
    assert np.array_equal(elem_g[idx], elem_r[idx]), \
        f"elements differ at {idx[elem_g[idx] != elem_r[idx]][:10]}"
    assert np.array_equal(st_g[idx], st_r[idx]), "status differs"
    assert np.array_equal(edge_g[idx], edge_r[idx]), "edge classification differs"
    assert np.array_equal(vert_g[idx], vert_r[idx]), "vertex classification differs"
    for s in range(nsol):
        ok = bits_equal(outs_g[s][idx], outs_r[s][idx])
        assert ok.all(), f"sol {s}: {np.count_nonzero(~ok)} points differ bitwise"


# Mmg tags (libmmgtypes.h, restated): MG_REF, MG_GEO, MG_REQ, MG_NOM, MG_BDY, MG_CRN
TAG_REF, TAG_GEO, TAG_REQ, TAG_NOM, TAG_BDY, TAG_CRN = 1, 2, 4, 8, 16, 32
IARE = [(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)]


def cube_surface(m, seed: int = 5, noise: float = 0.05, ridge_frac: float = 1.0):
    """Mmg-like surface data of a Kuhn mesh of the unit cube, the way
    MMG3D_analys leaves it (synthetic: the kernels only read it):

    * point tags: MG_BDY on the faces, MG_GEO on the 12 cube edges (ridges),
      MG_CRN | MG_REQ | MG_GEO at the 8 corners, a few ridge points MG_NOM
      (non-manifold: their metric is a plain tensor);
    * per tet an xTetra when it has a boundary face: tag[ia] = MG_BDY for the
      edges of its boundary faces, | MG_GEO for those along a cube edge;
    * per point p->n (the outward normal of a face point, the tangent of a
      ridge point) and an xPoint with n1 (face normal) / n1, n2 (the two face
      normals of a ridge point), all perturbed by `noise` and renormalised so
      that the curved-length formulas see non-trivial normals;
    * the metric in Mmg's ridge storage at the non-singular ridge points
      ((tangent, in-surface 1 / 2, normal 1 / 2) sizes^-2), a shock tensor
      elsewhere (ridge_frac < 1: only that fraction of the ridge points).

    Returns (tags (np+1,), surface dict for Transfer.upload_surface /
    oracle.prilen, met (np+1, 6))."""
    rng = np.random.default_rng(seed)
    x = m.xyz
    onb = np.stack([(x[:, a] == 0.0) | (x[:, a] == 1.0) for a in range(3)], 1)
    onb[0] = False
    cnt = onb.sum(1)
    tag = np.zeros(m.np + 1, np.uint16)
    tag[cnt >= 1] |= TAG_BDY
    tag[cnt >= 2] |= TAG_GEO
    tag[cnt == 3] |= TAG_CRN | TAG_REQ
    ridge = np.nonzero(cnt == 2)[0]
    tag[ridge[:: 17]] |= TAG_NOM

    def face_normal(ip, a):
        v = np.zeros(3)
        v[a] = 1.0 if x[ip, a] == 1.0 else -1.0
        return v

    def noisy(v):
        w = v + noise * rng.standard_normal(3)
        return w / np.sqrt((w * w).sum())

    n = np.zeros((m.np + 1, 3))
    xp = np.zeros(m.np + 1, np.int32)
    n1, n2 = [np.zeros(3)], [np.zeros(3)]
    for ip in np.nonzero((cnt == 1) | (cnt == 2))[0]:
        axes = np.nonzero(onb[ip])[0]
        a = face_normal(ip, axes[0])
        if cnt[ip] == 1:
            n[ip] = noisy(a)
            n1.append(noisy(a))
            n2.append(np.zeros(3))
        else:
            b = face_normal(ip, axes[1])
            n[ip] = noisy(np.cross(a, b))
            n1.append(noisy(a))
            n2.append(noisy(b))
        xp[ip] = len(n1) - 1
    # xTetras of the tets with a boundary face (face f opposite vertex f)
    ne = m.ne
    adj = m.adja[1:4 * ne + 1].reshape(ne, 4)
    xt = np.zeros(ne + 1, np.int32)
    xtag = [np.zeros(6, np.uint16)]
    for k in np.nonzero((adj == 0).any(1))[0] + 1:
        v = m.tet[k]
        t6 = np.zeros(6, np.uint16)
        for f in np.nonzero(adj[k - 1] == 0)[0]:
            for ia, (i, j) in enumerate(IARE):
                if f in (i, j):
                    continue
                t6[ia] |= TAG_BDY
                p, q = v[i], v[j]
                common = onb[p] & onb[q] & (x[p] == x[q])
                if common.sum() >= 2:
                    t6[ia] |= TAG_GEO
        xtag.append(t6)
        xt[k] = len(xtag) - 1
    met = M.on_vertices(m, M.shock_metric)
    rid = np.nonzero(((tag & TAG_GEO) != 0) & ((tag & (TAG_CRN | TAG_REQ | TAG_NOM)) == 0))[0]
    rid = rid[: int(len(rid) * ridge_frac)]
    h = rng.uniform(0.02, 0.2, size=(len(rid), 5))
    met[rid, :5] = 1.0 / (h * h)
    met[rid, 5] = 0.0
    surf = dict(xt=xt, xtag=np.array(xtag), n=n, xp=xp, n1=np.array(n1), n2=np.array(n2))
    return tag, surf, met
