"""GPU parity: the gfx950 transfer path (through the C ABI) against the oracle.

Volume points: located tets bit-exact except documented ties (several tets
contain the point within the reference's -1e-6 tolerance); fields bit-exact
where the tet is the same.  Surface points: bit-exact against the oracle run
with the device semantics (same start triangle, point flags as left by
PMMG_precompute_nodeTrias at every query) -- see DESIGN.md "Surface semantics".
"""
import os

import numpy as np
import pytest

from conftest import REF_INPUTS
from helpers import bits_equal, compare_exact, compare_volume, cube_case, lin_field
from oracle import oracle as O
from parmmg_amd import mesh as M

pytestmark = pytest.mark.gpu

from parmmg_amd import _native as N

SERIAL_BDY = N.RUN_SERIAL_SURFACE        # surface path on the main stream (no fork)
NOTIES = N.RUN_NO_INLINE_TIES            # every near-face point to the tie BFS
REFWALK = N.RUN_REFERENCE_WALK           # the reference-order walk k_walk instead of k_walks
FRESH = N.RUN_FRESH_BACKGROUND           # derived background data rebuilt by the step


def run_gpu(tr, m, x, t, sols, imet=0, hsiz=0.0, init=None, flags=0, tets=None):
    tr.upload_background(m, sols, imet)
    tr.upload_points(x, t, tets)
    tr.run(hsiz=hsiz, flags=flags, record_starts=True)
    r = tr.download(init=init)
    e, v = tr.border()
    return r, tr.starts(), e, v


@pytest.mark.parametrize("metric,n,flags", [("iso", 10, 0), ("ani", 9, 0), ("none", 7, 0),
                                            ("iso", 10, SERIAL_BDY), ("ani", 9, FRESH),
                                            ("iso", 10, NOTIES), ("ani", 9, REFWALK),
                                            ("iso", 10, REFWALK | NOTIES)])
def test_volume_parity(transfer, metric, n, flags):
    m, x, t, sols = cube_case(n, metric=metric, surface=False)
    imet = 0 if metric != "none" else -1
    r, starts, _, _ = run_gpu(transfer, m, x, t, sols, imet, flags=flags)
    o = O.Oracle(m)
    outs, elem, st, steps, e, v = o.interp(x, t, sols, imet=imet)
    c = compare_volume(o, x, t, (r.sols, r.elem, r.status), (outs, elem, st), sols)
    assert c["same"] >= c["nvol"] - max(3, c["nvol"] // 1000)
    assert np.all(r.status[t == 0] == 1)


def test_surface_parity_device_semantics(transfer):
    m, x, t, sols = cube_case(8, metric="iso")
    r, starts, edge, vert = run_gpu(transfer, m, x, t, sols, 0)
    o = O.Oracle(m)
    outs, elem, st, steps, e, v = o.interp(x, t, sols, imet=0, fresh=True,
                                           start_vol=starts, start_bdy=starts)
    bdy = np.nonzero(t == 16)[0]
    compare_exact((r.sols, r.elem, r.status, edge, vert), (outs, elem, st, e, v), bdy, len(sols))
    compare_volume(o, x, t, (r.sols, r.elem, r.status), (outs, elem, st), sols)


def test_surface_ani_metric_edges_and_vertices(transfer):
    """Surface points placed exactly on old boundary edges and vertices drive
    the interp2bar / copyMetrics branches (src/interpmesh_pmmg.c:564-575)."""
    m = M.kuhn_cube(6)
    sols = [M.on_vertices(m, M.shock_metric), M.on_vertices(m, M.level_set)]
    tr_ = m.tria[1:]
    mids = 0.5 * (m.xyz[tr_[:, 0]] + m.xyz[tr_[:, 1]])
    verts = m.xyz[np.unique(tr_.ravel())]
    x = np.concatenate([mids[::3], verts[::5]])
    t = np.full(len(x), 16, np.uint16)
    r, starts, edge, vert = run_gpu(transfer, m, x, t, sols, 0)
    o = O.Oracle(m)
    outs, elem, st, steps, e, v = o.interp(x, t, sols, imet=0, fresh=True, start_bdy=starts,
                                           start_vol=starts)
    idx = np.arange(len(x))
    compare_exact((r.sols, r.elem, r.status, edge, vert), (outs, elem, st, e, v), idx, len(sols))
    assert (e >= 0).sum() + (v >= 0).sum() > 0


def l_shaped(n):
    """Kuhn cube minus its upper octant: non-convex, exercises stuck walks."""
    m = M.kuhn_cube(n)
    c = m.centroids()
    keep = ~np.all(c > 0.5, axis=1)
    tet = np.concatenate([m.tet[:1], m.tet[1:][keep]])
    return M.from_tets(m.xyz, tet)


def test_nonconvex_exhaustive_and_closest(transfer):
    m = l_shaped(8)
    rng = np.random.default_rng(7)
    x = rng.uniform(-0.1, 1.1, size=(3000, 3))
    t = np.zeros(len(x), np.uint16)
    sols = [M.on_vertices(m, M.iso_metric), M.on_vertices(m, lin_field)]
    r, starts, _, _ = run_gpu(transfer, m, x, t, sols, 0)
    o = O.Oracle(m)
    outs, elem, st, steps, e, v = o.interp(x, t, sols, imet=0)
    assert (st == 0).sum() > 100
    c = compare_volume(o, x, t, (r.sols, r.elem, r.status), (outs, elem, st), sols)
    closest = np.nonzero(st == 0)[0]
    assert np.array_equal(r.elem[closest], elem[closest])
    stats = transfer.locate_stats()
    assert stats["nexhaust"] > 0 and stats["nclosest"] == len(closest)
    assert c["ties"] <= 3


def test_exhaustive_found_path(transfer):
    """Walk capped at one step: every point not in its hint tet goes through the
    LDS-staged exhaustive scan, whose answer (first containing tet in index
    order) must match the oracle's."""
    m, x, t, sols = cube_case(6, metric="ani", surface=False)
    transfer.upload_background(m, sols, 0)
    transfer.upload_points(x, t)
    transfer.run(max_walk=1)
    r = transfer.download()
    assert (r.status == -1).sum() > len(x) // 2
    o = O.Oracle(m)
    outs, elem, st, *_ = o.interp(x, t, sols, imet=0)
    compare_volume(o, x, t, (r.sols, r.elem, r.status), (outs, elem, st), sols)


def test_reference_wave_partition(transfer):
    """libexamples/adaptation_example1/wave.0.mesh: an unstructured partition
    (non-convex interface side) with points inside and outside."""
    m = M.read_medit(os.path.join(REF_INPUTS, "wave.0.mesh"))
    lo, hi = m.xyz[1:].min(0), m.xyz[1:].max(0)
    rng = np.random.default_rng(11)
    inside = m.centroids()[rng.choice(m.ne, 2000, replace=False)]
    x = np.concatenate([inside + rng.normal(0, 1e-3, inside.shape), rng.uniform(lo, hi, (500, 3))])
    t = np.zeros(len(x), np.uint16)
    f = lambda p: (np.sin(3 * p[:, 0]) + p[:, 1])[:, None]  # noqa: E731
    sols = [M.on_vertices(m, f), M.on_vertices(m, M.velocity)]
    r, starts, _, _ = run_gpu(transfer, m, x, t, sols, -1)
    o = O.Oracle(m)
    outs, elem, st, steps, e, v = o.interp(x, t, sols, imet=-1)
    compare_volume(o, x, t, (r.sols, r.elem, r.status), (outs, elem, st), sols)


def test_reference_cube_example(transfer):
    m = M.read_medit(os.path.join(REF_INPUTS, "cube.mesh"))
    met = M.read_medit_sol(os.path.join(REF_INPUTS, "cube-met.sol"))[0]
    flds = M.read_medit_sol(os.path.join(REF_INPUTS, "cube-solphys.sol"))
    rng = np.random.default_rng(3)
    x = rng.uniform(0, 1, (400, 3)) * np.array([1.0, 1.0, 1.0])
    t = np.zeros(len(x), np.uint16)
    sols = [met] + flds
    r, starts, _, _ = run_gpu(transfer, m, x, t, sols, 0)
    o = O.Oracle(m)
    outs, elem, st, *_ = o.interp(x, t, sols, imet=0)
    compare_volume(o, x, t, (r.sols, r.elem, r.status), (outs, elem, st), sols)


def test_constant_size_and_required_points(transfer):
    m, x, t, sols = cube_case(6, metric="iso")
    t = t.copy()
    t[::17] = 4                       # MG_REQ: skipped, copied elsewhere
    init = [np.full((len(x), s.shape[1]), -7.0) for s in sols]
    r, starts, _, _ = run_gpu(transfer, m, x, t, sols, 0, hsiz=0.05, init=init)
    assert np.all(r.sols[0][:, 0] == 0.05)          # MMG3D_Set_constantSize, all points
    req = t == 4
    for s in range(1, len(sols)):
        assert np.all(r.sols[s][req] == -7.0)
        assert not np.any(r.sols[s][~req] == -7.0)


def test_dropin_interp_metrics_and_fields(transfer):
    """PMX_interpMetricsAndFields on three groups in Mmg layout (1-based
    arrays): the groups alternate between two contexts (group 2 waits for
    group 0's download on the first)."""
    groups, refs = [], []
    for n, seed in ((6, 1), (7, 2), (5, 3)):
        m, x, t, sols = cube_case(n, metric="iso", seed_pts=seed)
        xyz1 = np.concatenate([np.zeros((1, 3)), x])
        tag1 = np.concatenate([np.zeros(1, np.uint16), t])
        met = np.zeros((len(xyz1), 1))
        fields = [np.zeros((len(xyz1), s.shape[1])) for s in sols[1:]]
        groups.append(dict(old_mesh=m, old_met=sols[0], old_fields=sols[1:], xyz=xyz1, tags=tag1,
                           met=met, fields=fields, hsiz=0.0))
        o = O.Oracle(m)
        refs.append((o, x, t, sols, o.interp(x, t, sols, imet=0)))
    assert transfer.interp_metrics_and_fields(groups, input_met=1) == 1
    for g, (o, x, t, sols, (outs, elem, st, *_)) in zip(groups, refs):
        got = [g["met"][1:]] + [f[1:] for f in g["fields"]]
        # the seam does not return elements: every volume point must be
        # bit-exact, or a documented tie (a containing tet on both sides,
        # fields within the tie tolerance) -- elements are taken from a
        # direct step on the same inputs
        r, *_ = run_gpu(transfer, g["old_mesh"], x, t, sols, 0)
        for s in range(len(sols)):
            assert bits_equal(got[s], r.sols[s]).all(), "seam differs from the direct step"
        c = compare_volume(o, x, t, (got, r.elem, r.status), (outs, elem, st), sols)
        assert c["same"] >= c["nvol"] - max(3, c["nvol"] // 1000)


def test_copy_required_points(transfer):
    m, x, t, sols = cube_case(5, metric="iso")
    otag = np.zeros(m.np + 1, np.uint16)
    otag[1::4] = 4
    perm = np.arange(m.np + 1, dtype=np.int32)[::-1].copy()
    perm = (m.np + 1 - np.arange(m.np + 1)).astype(np.int32)
    met = np.zeros((m.np + 2, 1))
    import ctypes as C
    from parmmg_amd import _native as N
    from parmmg_amd.transfer import mesh_view
    G = N.Group()
    G.old_mesh = mesh_view(m)
    sv_new, sv_old = N.SolView(), N.SolView()
    sv_new.size, sv_new.m = 1, met.ctypes.data_as(N.dptr)
    sv_old.size, sv_old.m = 1, sols[0].ctypes.data_as(N.dptr)
    G.met, G.old_met = C.pointer(sv_new), C.pointer(sv_old)
    G.nsols = 0
    r = transfer.lib.PMX_copyMetricsAndFields_point(transfer.ctx, C.byref(G),
                                                    otag.ctypes.data_as(N.u16ptr), 2,
                                                    perm.ctypes.data_as(N.iptr), 1, 1)
    assert r == 1
    for ip in range(1, m.np + 1):
        if otag[ip] & 4:
            assert met[perm[ip], 0] == sols[0][ip, 0]


@pytest.mark.parametrize("metric", ["iso", "ani"])
def test_quality_and_length_stats(transfer, metric):
    m, x, t, sols = cube_case(7, metric=metric, fields=False)
    transfer.upload_background(m, sols, 0)
    q = transfer.tetra_qual(m.ne)
    qo = O.tetra_qual(m, sols[0] if metric == "ani" else None)
    assert np.array_equal(q[1:], qo[1:]), "per-tet quality not bit-exact"
    h = transfer.qualhisto()
    ho = O.qualhisto(m, qo)
    assert h["his"] == ho["his"] and h["ne"] == ho["ne"] and h["iel"] == ho["iel"]
    assert h["good"] == ho["good"] and h["med"] == ho["med"]
    assert h["min"] == ho["min"] and h["max"] == ho["max"]
    assert abs(h["avg"] - ho["avg"]) <= 1e-12 * abs(ho["avg"])
    L = transfer.prilen()
    Lo = O.prilen(m, sols[0])
    assert L["ned"] == Lo["ned"] and L["nullEdge"] == Lo["nullEdge"]
    assert L["ned"] > 0
    # counts exact apart from lengths within a few ulp of a bin boundary
    assert L["hl"] == Lo["hl"]                         # glibc's log1p restated on the device (r06)
    assert abs(L["avlen"] - Lo["avlen"]) <= 1e-12 * abs(Lo["avlen"])
    assert L["lmin"] == Lo["lmin"] and L["lmax"] == Lo["lmax"]
    if L["lmin"] == Lo["lmin"]:
        assert (L["amin"], L["bmin"]) == (Lo["amin"], Lo["bmin"])
    if L["lmax"] == Lo["lmax"]:
        assert (L["amax"], L["bmax"]) == (Lo["amax"], Lo["bmax"])


def test_deterministic(transfer):
    """Located elements and fields are independent of the (racy) hint grid."""
    m, x, t, sols = cube_case(8, metric="ani")
    a, sa, ea, va = run_gpu(transfer, m, x, t, sols, 0)
    for stride in (1, 3, 7):
        transfer.run(hint_stride=stride)
        b = transfer.download()
        vol = t == 0
        assert np.array_equal(a.elem[vol], b.elem[vol])
        for s in range(len(sols)):
            assert bits_equal(a.sols[s][vol], b.sols[s][vol]).all()


@pytest.mark.parametrize("metric", ["iso", "ani"])
def test_slot_and_reference_walks_agree(transfer, metric):
    """The slot walk (k_walks, dense or Pt4 coordinates) and the
    reference-order walk (k_walk) are different paths to the same located tet:
    identical elements, statuses and bit-identical fields, ties included."""
    m, x, t, sols = cube_case(16, metric=metric, surface=False, fields=metric == "iso")
    P = m.xyz[m.tet[1::97]]
    x = np.concatenate([x, P[:, 0], 0.5 * (P[:, 0] + P[:, 1]), P[:, :3].mean(1)])
    t = np.zeros(len(x), np.uint16)
    a, *_ = run_gpu(transfer, m, x, t, sols, 0)
    for flags in (REFWALK, REFWALK | NOTIES, FRESH):
        b, *_ = run_gpu(transfer, m, x, t, sols, 0, flags=flags)
        assert np.array_equal(a.elem, b.elem)
        assert np.array_equal(a.status, b.status)
        for s in range(len(sols)):
            assert bits_equal(a.sols[s], b.sols[s]).all()


@pytest.mark.parametrize("flags", [0, NOTIES, REFWALK, NOTIES | REFWALK])
def test_tie_points_canonical(transfer, flags):
    """Old vertices, edge midpoints and face centroids (the tie suite of
    SURVEY.md 8(d)): the device returns the smallest index among all tets
    that contain the point by the reference predicate."""
    m = M.kuhn_cube(4)
    rng = np.random.default_rng(2)
    ks = rng.choice(np.arange(1, m.ne + 1), 60, replace=False)
    P = m.xyz[m.tet[ks]]
    x = np.concatenate([P[:, 0], 0.5 * (P[:, 0] + P[:, 1]), P[:, :3].mean(1), P.mean(1)])
    t = np.zeros(len(x), np.uint16)
    sols = [M.on_vertices(m, M.iso_metric)]
    r, starts, _, _ = run_gpu(transfer, m, x, t, sols, 0, flags=flags)
    o = O.Oracle(m)
    for i in range(len(x)):
        cont = [k for k in range(1, m.ne + 1) if o.tet_contains(k, x[i])[0]]
        assert cont and r.elem[i] == min(cont), (i, r.elem[i], cont)
    outs, elem, st, *_ = o.interp(x, t, sols, imet=0)
    c = compare_volume(o, x, t, (r.sols, r.elem, r.status), (outs, elem, st), sols)
    assert c["ties"] > 0


def test_large_size_properties(transfer):
    """n=60 (1.3M tets): size-independent properties -- every point found,
    linear fields reproduced, located tets contain their points."""
    m, x, t, sols = cube_case(60, metric="iso")
    r, starts, edge, vert = run_gpu(transfer, m, x, t, sols, 0)
    assert np.all(r.status != 0)
    vol = np.nonzero(t == 0)[0]
    # volume: linear fields are reproduced (barycentric interpolation)
    assert np.abs(r.sols[3][vol, 0] - lin_field(x[vol])[:, 0]).max() < 1e-12
    o = O.Oracle(m)
    rng = np.random.default_rng(5)
    for i in rng.choice(vol, 300, replace=False):
        assert o.tet_contains(int(r.elem[i]), x[i])[0]
    st = transfer.locate_stats()
    assert st["nexhaust"] == 0 and st["stepav"] < 4.0
    # surface: the reference's shadow-wedge / cone tests accept points within
    # hausd of a visited edge, so linear reproduction does not hold there;
    # check the surface points bit-exactly against the oracle instead
    outs, elem, sto, steps, e, v = o.interp(x, t, sols, imet=0, fresh=True, start_vol=starts,
                                            start_bdy=starts)
    bdy = np.nonzero(t == 16)[0]
    compare_exact((r.sols, r.elem, r.status, edge, vert), (outs, elem, sto, e, v), bdy, len(sols))


def _shuffled(m, seed=7):
    """Tets in a random order, local vertices rotated (orientation kept)."""
    rng = np.random.default_rng(seed)
    perm = rng.permutation(m.ne) + 1
    tet = np.zeros_like(m.tet)
    tet[1:] = m.tet[perm]
    even = np.array([[0, 1, 2, 3], [1, 0, 3, 2], [2, 3, 0, 1], [3, 2, 1, 0]])
    tet[1:] = np.take_along_axis(tet[1:], even[rng.integers(0, 4, m.ne)], axis=1)
    return M.from_tets(m.xyz, tet)


def test_shuffled_numbering_parity(transfer):
    """A background with no numbering locality (random tet order, SURVEY.md
    8(d) --shuffle-tets): same located tets and bit-exact fields as the oracle
    (ties: the documented canonical rule)."""
    m = _shuffled(M.kuhn_cube(10))
    x, t = M.new_points(10, seed=12345, surface=False)
    sols = [M.on_vertices(m, M.iso_metric), M.on_vertices(m, M.level_set),
            M.on_vertices(m, M.velocity)]
    r, *_ = run_gpu(transfer, m, x, t, sols, 0)
    o = O.Oracle(m)
    outs, elem, st, *_ = o.interp(x, t, sols, imet=0)
    c = compare_volume(o, x, t, (r.sols, r.elem, r.status), (outs, elem, st), sols)
    assert c["same"] >= c["nvol"] - max(3, c["nvol"] // 1000)
    assert np.all(r.status == 1)


def test_empty_and_single_point(transfer):
    """Ragged edge cases: no new vertex at all, then exactly one (volume) and
    one surface vertex."""
    m, x, t, sols = cube_case(5, metric="iso")
    r, *_ = run_gpu(transfer, m, x[:0], t[:0], sols, 0)
    assert len(r.elem) == 0 and all(s.shape[0] == 0 for s in r.sols)
    o = O.Oracle(m)
    for i in (int(np.nonzero(t == 0)[0][7]), int(np.nonzero(t == 16)[0][3])):
        xi, ti = x[i:i + 1], t[i:i + 1]
        r, starts, e, v = run_gpu(transfer, m, xi, ti, sols, 0)
        outs, elem, st, steps, e2, v2 = o.interp(xi, ti, sols, imet=0, fresh=True,
                                                 start_vol=starts, start_bdy=starts)
        assert r.elem[0] == elem[0] and r.status[0] == st[0]
        for s in range(len(sols)):
            assert bits_equal(r.sols[s], outs[s]).all()


def test_staging_arena_regrow_and_reuse(transfer):
    """The pinned host staging arena (pmx_capi.hip hstage) is grown and reused
    across uploads of different sizes: small -> large -> small background and
    point sets on one context give the oracle's results each time, and the
    last small step is bit-identical to the first."""
    first = None
    for n, metric in ((5, "iso"), (10, "ani"), (5, "iso")):
        m, x, t, sols = cube_case(n, metric=metric, surface=False)
        r, *_ = run_gpu(transfer, m, x, t, sols, 0)
        o = O.Oracle(m)
        outs, elem, st, steps, e, v = o.interp(x, t, sols, imet=0)
        c = compare_volume(o, x, t, (r.sols, r.elem, r.status), (outs, elem, st), sols)
        assert c["same"] >= c["nvol"] - max(3, c["nvol"] // 1000)
        assert np.all(r.status[t == 0] == 1)
        if first is None:
            first = r
    assert np.array_equal(first.elem, r.elem) and np.array_equal(first.status, r.status)
    for a, b in zip(first.sols, r.sols):
        assert bits_equal(a, b).all()


def test_download_into_existing_arrays(transfer):
    """download(into=...) writes the step's results in place (ParMmg's met->m /
    field->m exist before the step): bit-identical to a fresh download."""
    m, x, t, sols = cube_case(7, metric="ani")
    r, *_ = run_gpu(transfer, m, x, t, sols, 0)
    buf = transfer.download()
    for a in buf.sols:
        a.fill(np.nan)
    buf.elem.fill(-7)
    transfer.download(into=buf)
    assert np.array_equal(buf.elem, r.elem) and np.array_equal(buf.status, r.status)
    for a, b in zip(buf.sols, r.sols):
        assert bits_equal(a, b).all()
    with pytest.raises(ValueError):
        transfer.download(into=type(buf)(buf.sols[:0], buf.elem, buf.status, buf.steps))
