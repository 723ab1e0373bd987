"""GPU: PMX_RUN_SEQUENTIAL_SURFACE -- the reference's sequential surface
semantics, bit for bit against the oracle's sequential run.

The reference locates the boundary points one after the other in its vertex
loop's first-visit order through the new tets (src/interpmesh_pmmg.c:535-599):
each PMMG_locatePointBdy starts from the previous one's tria, mesh->base counts
every locate, and the shadow cone / wedge tests read and write MMG5_Point.flag
across queries (src/locate_pmmg.c:209-334,640-660).  The oracle given
``order=first_visit_order(tets)`` runs exactly that loop; the device in this
mode must return the same tria, edge / vertex classification, status and
interpolated fields for every surface point, and leave the volume points as
the default step does.  (The default step runs every query fresh from its hint
tria: see test_gpu_configs.py for how far apart the two semantics are.)
"""
import os

import numpy as np
import pytest

from conftest import ROOT
from helpers import bits_equal, compare_exact, cube_case, first_visit_order, lin_field
from oracle import oracle as O
from parmmg_amd import _native as N
from parmmg_amd import mesh as M

pytestmark = pytest.mark.gpu

REF_INPUTS = os.path.join(ROOT, "tests", "golden", "ref_inputs")
SEQ = N.RUN_SEQUENTIAL_SURFACE | N.RUN_SEQUENTIAL_VOLUME


def _run(tr, m, x, t, sols, tets, flags):
    tr.upload_background(m, sols, 0)
    tr.upload_points(x, t, tets_mmg=tets)
    tr.run(flags=flags)
    r = tr.download()
    e, v = tr.border()
    return r, e, v


def check_seq(tr, m, x, t, sols, tets):
    """Device sequential mode vs the oracle's sequential run on every point
    the reference visits; volume points as in the default step."""
    rd, ed, vd = _run(tr, m, x, t, sols, tets, 0)
    rs, es, vs = _run(tr, m, x, t, sols, tets, SEQ)
    st = tr.seq_surface_stats()
    fv = first_visit_order(tets, len(x))
    o = O.Oracle(m)
    qo, qe, qs, _, qed, qve = o.interp(x, t, sols, imet=0, order=fv)
    tt = np.asarray(t)
    live = np.zeros(len(x), bool)
    live[fv] = True
    live &= (tt < M.TAG_NUL) & ((tt & M.TAG_REQ) == 0)
    bdy = np.nonzero(live & ((tt & M.TAG_BDY) != 0))[0]
    vol = np.nonzero(live & ((tt & M.TAG_BDY) == 0))[0]
    assert st["nseq"] == len(bdy)
    compare_exact((rs.sols, rs.elem, rs.status, es, vs), (qo, qe, qs, qed, qve), bdy, len(sols))
    # the volume points too (PMX_RUN_SEQUENTIAL_VOLUME): the reference's own
    # walk from the previous volume point's tet -- ties included
    sv = tr.seq_volume_stats()
    assert sv["nseq"] == len(vol)
    assert np.array_equal(rs.elem[vol], qe[vol]), vol[rs.elem[vol] != qe[vol]][:10]
    assert np.array_equal(rs.status[vol], qs[vol])
    for a, b in zip(rs.sols, qo):
        assert bits_equal(a[vol], b[vol]).all()
    st["vol_nseq"], st["vol_nreplay"] = sv["nseq"], sv["nreplay"]
    # how far the device semantics are from the sequential run on this case
    ndiff = int(((rd.elem[bdy] != qe[bdy]) | (ed[bdy] != qed[bdy]) | (vd[bdy] != qve[bdy])).sum())
    st["vol_ndiff"] = int((rd.elem[vol] != qe[vol]).sum())
    return st, ndiff


@pytest.mark.parametrize("n,metric", [(6, "iso"), (11, "ani"), (18, "iso")])
def test_seq_surface_cube(transfer, n, metric):
    m, x, t, sols = cube_case(n, metric=metric)
    tets = M.new_point_tets(n, x, t)
    st, ndiff = check_seq(transfer, m, x, t, sols, tets)
    print(f"\nn={n}: {st['nseq']} surface points, {st['nreplay']} replayed, "
          f"{ndiff} differ in device semantics; volume {st['vol_nseq']} points, {st['vol_nreplay']} replayed, "
          f"{st['vol_ndiff']} differ")
    assert st["nreplay"] <= st["nseq"]


def test_seq_surface_shuffled_tets_req_nul_orphans(transfer):
    """The visit order from a shuffled new-tet numbering, frozen (REQ) and
    invalid (NUL) points that the loop skips without a locate (mesh->base not
    advanced), orphans never visited, deleted new tets ignored."""
    n = 12
    m, x, t, sols = cube_case(n, metric="iso")
    t = t.copy()
    tets = M.new_point_tets(n, x, t)
    rng = np.random.default_rng(8)
    body = tets[1:][rng.permutation(len(tets) - 1)]
    drop = rng.random(len(body)) < 0.03
    body[drop, 0] = -body[drop, 0]                   # deleted new tets (!MG_EOK)
    tets = np.concatenate([tets[:1], body]).astype(np.int32)
    t[5::37] |= M.TAG_REQ
    t[11::41] = M.TAG_NUL
    st, _ = check_seq(transfer, m, x, t, sols, tets)
    assert st["nseq"] > 0


def test_seq_surface_unstructured_wave(transfer):
    """libexamples/adaptation_example1/wave.0.mesh (an unstructured ParMmg
    partition, curved non-convex surface): the new points are its own vertices
    moved by 2e-4 (well inside hausd), the boundary ones tagged MG_BDY, the new
    tets its own tets in a shuffled order -- walks that meet visited trias run
    the shadow wedge / cone tests on the carried flags."""
    m = M.read_medit(os.path.join(REF_INPUTS, "wave.0.mesh"))
    rng = np.random.default_rng(4)
    x = m.xyz[1:] + rng.normal(0.0, 2e-4, (m.np, 3))
    onb = np.zeros(m.np + 1, bool)
    onb[m.tria[1:].ravel()] = True
    t = np.where(onb[1:], M.TAG_BDY, 0).astype(np.uint16)
    f = lambda p: (np.sin(3 * p[:, 0]) + p[:, 1])[:, None]  # noqa: E731
    sols = [M.on_vertices(m, M.iso_metric), M.on_vertices(m, f), M.on_vertices(m, lin_field)]
    order = rng.permutation(m.ne) + 1
    tets = np.concatenate([m.tet[:1], m.tet[order]]).astype(np.int32)
    st, ndiff = check_seq(transfer, m, x, t, sols, tets)
    print(f"\nwave.0: {st['nseq']} surface points, {st['nreplay']} replayed, {ndiff} differ in device semantics")


def test_seq_surface_stuck_replays(transfer):
    """Boundary points 0.05 off the cube (beyond hausd = 0.01 from every
    tria): their walks fail everywhere, run wedge tests and end stuck, so the
    replay hands them to the exhaustive scan (closest tria) and resumes."""
    n = 8
    m, x, t, sols = cube_case(n, metric="iso")
    x = x.copy()
    bi = np.nonzero(t == M.TAG_BDY)[0]
    off = bi[::29]
    x[off] += 0.05 * np.sign(x[off] - 0.5) * (np.abs(x[off] - 0.5) > 0.499)
    tets = M.new_point_tets(n, np.clip(x, 0, 1), t)
    st, _ = check_seq(transfer, m, x, t, sols, tets)
    assert st["nreplay"] >= len(off)


def test_seq_surface_needs_new_tets(transfer):
    m, x, t, sols = cube_case(5, metric="iso")
    transfer.upload_background(m, sols, 0)
    transfer.upload_points(x, t)
    with pytest.raises(RuntimeError, match="new tets"):
        transfer.run(flags=SEQ)


def test_seq_volume_ties_on_old_vertices_edges_faces(transfer):
    """Volume points ON the old mesh's vertices, edge midpoints and face
    centroids (ties of 2 to ~20 tets): the default step returns the canonical
    smallest-index tet, the sequential mode the tet the reference's own path
    reaches first -- bit for bit against the oracle's sequential run."""
    n = 7
    m, x, t, sols = cube_case(n, metric="ani")
    tets = M.new_point_tets(n, x, t)          # the vertex enumeration, before the points move
    x = x.copy()
    rng = np.random.default_rng(3)
    vol = np.nonzero(t == 0)[0]
    pick = rng.choice(vol, size=len(vol) // 3, replace=False)
    inner = np.nonzero(np.all((m.xyz[1:] > 0.01) & (m.xyz[1:] < 0.99), axis=1))[0] + 1
    third = len(pick) // 3
    x[pick[:third]] = m.xyz[rng.choice(inner, third)]                    # old vertices
    e = m.tet[rng.integers(1, m.ne + 1, third)]
    x[pick[third:2 * third]] = 0.5 * (m.xyz[e[:, 0]] + m.xyz[e[:, 1]])   # edge midpoints
    f = m.tet[rng.integers(1, m.ne + 1, len(pick) - 2 * third)]
    x[pick[2 * third:]] = (m.xyz[f[:, 0]] + m.xyz[f[:, 1]] + m.xyz[f[:, 2]]) / 3.0   # face centroids
    st, _ = check_seq(transfer, m, x, t, sols, tets)
    print(f"\nties: volume {st['vol_nseq']} points, {st['vol_nreplay']} replayed, {st['vol_ndiff']} differ "
          f"from the default step")
    assert st["vol_ndiff"] > 0


def test_seq_volume_walk_into_deleted_tets(transfer):
    """Deleted background tets (v[0] = 0) whose neighbours still point at them:
    the reference's walk that steps into one spins until step > ne and returns
    the closest tet it visited (status 0, src/locate_pmmg.c:809-811,846-851);
    the sequential mode does the same, bit for bit."""
    n = 6
    m, x, t, sols = cube_case(n, metric="iso")
    c = m.centroids()
    dead = np.nonzero(np.all(np.abs(c - 0.5) < 0.17, axis=1))[0] + 1
    tet = m.tet.copy()
    tet[dead, 0] = 0
    md = M.Mesh(m.xyz, tet, m.adja, m.tria, m.adjt, m.hausd)
    tets = M.new_point_tets(n, x, t)
    st, _ = check_seq(transfer, md, x, t, sols, tets)
    assert st["vol_nreplay"] > 0
