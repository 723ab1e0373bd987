"""GPU edge cases of the reference's transfer path, against the oracle.

* MG_NUL new points (``!MG_VOK``): never touched (src/interpmesh_pmmg.c:541).
* New points referenced by no valid new tet: never visited by the reference's
  vertex loop over the new tets (:535-541), left untouched here too; a
  constant-size metric is still written on them (MMG3D_Set_constantSize).
* Deleted background tets (``v[0] = 0``, !MG_EOK) carving a hole: stuck
  walks, exhaustive scan, closest element for points in the hole.
* A singular background metric: ``MMG5_invmat`` fails, the anisotropic
  interpolation returns 0 and leaves the output untouched (:258-267).
* Failure handling of the C ABI: a failed upload leaves no usable context,
  results of an earlier step are refused after new uploads, a fallback grid
  barrier that gives up makes the step fail instead of returning garbage.
* The threaded host gathers/scatters (PMX_HOST_THREADS_MIN) give the same
  bytes as the serial path.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT
from helpers import bits_equal, compare_volume, cube_case, lin_field
from oracle import oracle as O
from parmmg_amd import _native as N
from parmmg_amd import mesh as M

pytestmark = pytest.mark.gpu


def _run(tr, m, x, t, sols, init=None, imet=0, flags=0, tets=None, max_walk=0):
    tr.upload_background(m, sols, imet)
    tr.upload_points(x, t, tets)
    tr.run(flags=flags, max_walk=max_walk)
    return tr.download(init=init)


def test_nul_points_untouched(transfer):
    m, x, t, sols = cube_case(7, metric="ani")
    t = t.copy()
    t[::13] = M.TAG_NUL
    init = [np.full((len(x), s.shape[1]), -7.0) for s in sols]
    transfer.upload_background(m, sols, 0)
    transfer.upload_points(x, t)
    transfer.run()
    r = transfer.download(init=init)
    nul = t == M.TAG_NUL
    for s in range(len(sols)):
        assert np.all(r.sols[s][nul] == -7.0)
    o = O.Oracle(m)
    outs, elem, st, *_ = o.interp(x, t, sols, imet=0, init=init)
    vol = t == 0
    assert np.all(r.elem[nul] == 0)
    c = compare_volume(o, x, t, (r.sols, r.elem, r.status), (outs, elem, st), sols)
    assert c["same"] >= c["nvol"] - max(3, c["nvol"] // 1000)
    assert vol.sum() > 0


def test_orphan_points_untouched_and_constant_size(transfer):
    """Points outside every valid new tet are not located; with -hsiz the
    constant metric is still set on them."""
    m, x, t, sols = cube_case(6, metric="iso", surface=False)
    n = len(x)
    # new tets over the first 80 % of the points (0-based point indices)
    rng = np.random.default_rng(4)
    used = np.zeros(n, bool)
    used[: int(0.8 * n)] = True
    pool = np.nonzero(used)[0]
    ntet = len(pool)
    tets = np.zeros((ntet + 2, 4), np.int32)
    tets[1:ntet + 1] = rng.choice(pool, size=(ntet, 4))
    tets[1:ntet + 1, 0] = pool          # every pooled point in at least one tet
    orph = np.nonzero(~used)[0]
    tets[ntet + 1] = [-1, orph[0], orph[1], orph[2]]   # a deleted new tet (!MG_EOK) is ignored
    init = [np.full((n, s.shape[1]), -7.0) for s in sols]
    r = _run(transfer, m, x, t, sols, init, tets=tets)
    ref_t = t.copy()
    ref_t[~used] = M.TAG_NUL            # the oracle skips them too
    o = O.Oracle(m)
    outs, elem, st, *_ = o.interp(x, ref_t, sols, imet=0, init=init)
    for s in range(len(sols)):
        assert np.all(r.sols[s][~used] == -7.0)
    c = compare_volume(o, x, ref_t, (r.sols, r.elem, r.status), (outs, elem, st), sols)
    assert c["same"] >= c["nvol"] - max(3, c["nvol"] // 1000)
    # constant size: every valid point gets the metric, orphans included
    transfer.run(hsiz=0.05)
    r2 = transfer.download(init=init)
    assert np.all(r2.sols[0][:, 0] == 0.05)
    for s in range(1, len(sols)):
        assert np.all(r2.sols[s][~used] == -7.0)


@pytest.mark.parametrize("hsiz", [0.0, 0.05])
def test_eager_download_equals_download(transfer, hsiz):
    """PMX_RUN_EAGER_DOWNLOAD (the fields start down right after the step, the
    orphan reset applied on the host) gives pmx_download's bytes: orphans
    untouched (a constant-size metric still written on them), NUL points
    untouched, elem / status identical; a second download repeats them."""
    m, x, t, sols = cube_case(6, metric="iso", surface=True)
    n = len(x)
    t = t.copy()
    t[5::41] = M.TAG_NUL
    rng = np.random.default_rng(11)
    used = np.zeros(n, bool)
    used[: int(0.85 * n)] = True
    pool = np.nonzero(used)[0]
    tets = np.zeros((len(pool) + 1, 4), np.int32)
    tets[1:] = rng.choice(pool, size=(len(pool), 4))
    tets[1:, 0] = pool
    tets[0] = -1

    def go(flags):
        init = [np.full((n, s.shape[1]), -7.0) for s in sols]
        transfer.upload_background(m, sols, 0)
        transfer.upload_points(x, t, tets)
        transfer.run(flags=flags, hsiz=hsiz)
        a = transfer.download(init=init)
        b = transfer.download(init=[np.full((n, s.shape[1]), -7.0) for s in sols])
        return a, b

    ref, _ = go(0)
    eg, eg2 = go(N.RUN_EAGER_DOWNLOAD)
    for r in (eg, eg2):
        for s in range(len(sols)):
            assert bits_equal(r.sols[s], ref.sols[s]).all()
        assert np.array_equal(r.elem, ref.elem) and np.array_equal(r.status, ref.status)
        # (walk lengths are a diagnostic: the hint grid keeps whichever sampled
        # tet of a cell was stored last, so they vary from run to run)
    for s in range(1, len(sols)):
        assert np.all(eg.sols[s][~used] == -7.0)
    if hsiz > 0:
        assert np.all(eg.sols[0][t != M.TAG_NUL, 0] == hsiz)


def delete_tets(m, dead):
    """Mark tets `dead` as deleted (v[0] = 0, the rest of the record kept) and
    cut the adjacency to and from them: Mmg's state of a hole."""
    tet = m.tet.copy()
    adja = m.adja.copy()
    dead = np.asarray(sorted(set(int(k) for k in dead)))
    isdead = np.zeros(m.ne + 1, bool)
    isdead[dead] = True
    a = adja[1:4 * m.ne + 1].reshape(m.ne, 4)
    a[isdead[1:]] = 0
    nb = a // 4
    a[isdead[nb] & (nb > 0)] = 0
    tet[dead, 0] = 0
    return M.Mesh(m.xyz, tet, adja, m.tria, m.adjt, m.hausd)


def test_deleted_background_tets(transfer):
    m = M.kuhn_cube(8)
    c = m.centroids()
    hole = 1 + np.nonzero(np.linalg.norm(c - np.array([0.6, 0.45, 0.5]), axis=1) < 0.17)[0]
    hole = hole[hole > 1]
    md = delete_tets(m, hole)
    rng = np.random.default_rng(9)
    x = rng.uniform(0.02, 0.98, size=(3000, 3))
    t = np.zeros(len(x), np.uint16)
    sols = [M.on_vertices(md, M.shock_metric), M.on_vertices(md, lin_field)]
    r = _run(transfer, md, x, t, sols)
    o = O.Oracle(md)
    outs, elem, st, *_ = o.interp(x, t, sols, imet=0)
    assert (st == 0).sum() > 20, "points in the hole must fall back to the closest tet"
    assert np.all(md.tet[r.elem, 0] > 0), "a deleted tet was returned"
    cmp = compare_volume(o, x, t, (r.sols, r.elem, r.status), (outs, elem, st), sols)
    closest = np.nonzero(st == 0)[0]
    assert np.array_equal(r.elem[closest], elem[closest])
    assert cmp["ties"] <= 5


def test_singular_metric_leaves_output_untouched(transfer):
    m, x, t, sols = cube_case(6, metric="ani", surface=False, fields=False)
    met = sols[0].copy()
    # vertices with a singular, non-diagonal metric: MMG5_invmat fails
    bad = np.arange(1, m.np + 1, 17)
    met[bad] = [1.0, 1.0, 0.0, 1.0, 0.0, 1.0]
    sols = [met, M.on_vertices(m, lin_field)]
    init = [np.full((len(x), s.shape[1]), -7.0) for s in sols]
    r = _run(transfer, m, x, t, sols, init)
    o = O.Oracle(m)
    outs, elem, st, *_ = o.interp(x, t, sols, imet=0, init=init)
    untouched = np.all(r.sols[0] == -7.0, axis=1)
    assert untouched.sum() > 50, "some points must touch a singular vertex"
    # the linear field is interpolated regardless
    assert np.abs(r.sols[1][:, 0] - lin_field(x)[:, 0]).max() < 1e-12
    cmp = compare_volume(o, x, t, (r.sols, r.elem, r.status), (outs, elem, st), sols)
    assert cmp["same"] >= cmp["nvol"] - max(3, cmp["nvol"] // 1000)
    same = r.elem == elem
    assert np.array_equal(untouched[same], np.all(outs[0][same] == -7.0, axis=1))


def test_failed_upload_leaves_no_usable_context(transfer):
    """a good upload then a bad one must not leave sizes that
    disagree with the device buffers -- the next step is refused cleanly."""
    m, x, t, sols = cube_case(5, metric="iso")
    transfer.upload_background(m, sols, 0)
    transfer.upload_points(x, t)
    transfer.run()
    big = M.kuhn_cube(9)
    bad = M.Mesh(big.xyz, big.tet.copy(), big.adja, big.tria, big.adjt)
    bad.tet[3, 2] = big.np + 5                      # vertex index out of range
    with pytest.raises(RuntimeError, match="out of range"):
        transfer.upload_background(bad, [M.on_vertices(big, M.iso_metric)], 0)
    with pytest.raises(RuntimeError, match="upload background"):
        transfer.run()
    with pytest.raises(RuntimeError):
        transfer.download()
    # a good upload makes the context usable again
    r = _run(transfer, m, x, t, sols)
    assert np.all(r.status != 0)


def test_stale_results_refused_after_new_points(transfer):
    """results of a step are not downloadable once the points or
    the background changed (sizes would disagree)."""
    m, x, t, sols = cube_case(5, metric="iso")
    transfer.upload_background(m, sols, 0)
    transfer.upload_points(x[:10], t[:10])
    transfer.run()
    transfer.upload_points(x, t)                    # more points, no step yet
    with pytest.raises(RuntimeError, match="no step has run"):
        transfer.download()
    transfer.run()
    r = transfer.download()
    assert len(r.elem) == len(x) and np.all(r.status != 0)


def test_fallback_barrier_timeout_fails_loudly(transfer):
    """The fused fallback's grid barrier reports a timeout instead of
    proceeding: with the debug hook the barriers do not wait, and the step
    must fail (pmx_synchronize / pmx_download return 0)."""
    m, x, t, sols = cube_case(6, metric="ani", surface=False)
    transfer.upload_background(m, sols, 0)
    transfer.upload_points(x, t)
    transfer.run(max_walk=1, flags=N.RUN_DEBUG_BARRIER_TIMEOUT)   # stuck points: the fallback runs
    with pytest.raises(RuntimeError, match="grid barrier"):
        transfer.synchronize()
    with pytest.raises(RuntimeError, match="grid barrier"):
        transfer.download()
    # the next normal step is fine
    transfer.run(max_walk=1)
    r = transfer.download()
    o = O.Oracle(m)
    outs, elem, st, *_ = o.interp(x, t, sols, imet=0)
    compare_volume(o, x, t, (r.sols, r.elem, r.status), (outs, elem, st), sols)


_THREADED = r"""
import sys, numpy as np
sys.path.insert(0, {root!r})
sys.path.insert(0, {tests!r})
from helpers import cube_case
from parmmg_amd.transfer import Transfer
m, x, t, sols = cube_case(12, metric="ani")
tr = Transfer(0)
tr.upload_background(m, sols, 0)
tr.upload_points(x, t)
tr.run()
r = tr.download()
np.savez({out!r}, elem=r.elem, status=r.status, steps=r.steps, *[s for s in r.sols])
"""


def test_threaded_host_paths_bit_identical(tmp_path):
    """The host gathers/scatters split over threads (forced on a small case
    with PMX_HOST_THREADS_MIN=1) give the bytes of the serial path."""
    outs = []
    for mode, env in (("serial", {"PMX_HOST_THREADS": "1"}),
                      ("threaded", {"PMX_HOST_THREADS": "8", "PMX_HOST_THREADS_MIN": "1"})):
        out = str(tmp_path / f"{mode}.npz")
        code = _THREADED.format(root=ROOT, tests=os.path.join(ROOT, "tests"), out=out)
        e = dict(os.environ, **env)
        p = subprocess.run([sys.executable, "-c", code], env=e, capture_output=True, text=True,
                           timeout=300)
        assert p.returncode == 0, p.stdout + p.stderr
        outs.append(np.load(out))
    a, b = outs
    # walk step counts depend on which sampled tet won a hint cell (a racy
    # plain store); the results do not
    for k in a.files:
        if k != "steps":
            assert np.array_equal(a[k].view(np.uint8), b[k].view(np.uint8)), k


def test_orphan_locate_stats_and_rows(transfer):
    """Orphans (points in no valid new tet) are located by the step (their
    marks come with the new tets, after it) but then reset everywhere: kind,
    element, status, steps, start 0, edge / vertex -1 -- so the locate
    statistics count only the points the reference visits (an orphan outside
    the domain adds no exhaustive scan, no closest element), and the
    starts / border downloads show them as never visited.  New tets uploaded
    after such a points view replace its tets for the orphan marks too."""
    m, x, t, sols = cube_case(6, metric="iso", surface=True)
    n = len(x)
    x = x.copy()
    rng = np.random.default_rng(21)
    used = np.zeros(n, bool)
    used[: int(0.75 * n)] = True
    orph = np.nonzero(~used)[0]
    x[orph[:5]] = [2.0, 2.0, 2.0]              # orphans outside the domain
    pool = np.nonzero(used)[0]
    tets = np.zeros((len(pool) + 1, 4), np.int32)
    tets[1:] = rng.choice(pool, size=(len(pool), 4))
    tets[1:, 0] = pool
    tets[0] = -1
    transfer.upload_background(m, sols, 0)
    transfer.upload_points(x, t, tets)
    transfer.run(record_starts=True)
    st = transfer.locate_stats()
    live = used & (t != M.TAG_NUL) & ((t & M.TAG_REQ) == 0)
    bdy = (t & M.TAG_BDY) != 0
    assert st["nvol"] == int((live & ~bdy).sum())
    assert st["nbdy"] == int((live & bdy).sum())
    assert st["nclosest"] == 0 and st["nexhaust"] == 0
    starts = transfer.starts()
    edge, vert = transfer.border()
    r = transfer.download()
    assert np.all(starts[~used] == 0) and np.all(edge[~used] == -1) and np.all(vert[~used] == -1)
    assert np.all(r.elem[~used] == 0) and np.all(r.status[~used] == 0) and np.all(r.steps[~used] == 0)
    assert np.all(r.status[live] != 0)
    # the same points with the tets given afterwards (pmx_upload_new_tets
    # before the step): the same orphans
    transfer.upload_points(x, t, tets)
    transfer.upload_new_tets(tets)
    transfer.run()
    st2 = transfer.locate_stats()
    assert (st2["nvol"], st2["nbdy"], st2["nclosest"]) == (st["nvol"], st["nbdy"], 0)
    r2 = transfer.download()
    assert np.all(r2.elem[~used] == 0) and np.array_equal(r2.elem, r.elem)


def test_undersized_host_outputs_refused(transfer):
    """Every host-output call checks the caller's capacity before writing:
    an array one entry short returns 0 with the reason and stays untouched
    (r04: an output sized by a wrong tet count was written past)."""
    import ctypes as C
    m, x, t, sols = cube_case(5, metric="iso", surface=True)
    n = len(x)
    pool = np.arange(n)
    rng = np.random.default_rng(3)
    tets = np.zeros((n + 1, 4), np.int32)
    tets[1:] = rng.choice(pool, size=(n, 4))
    tets[1:, 0] = pool
    tets[0] = -1
    transfer.upload_background(m, sols, 0)
    transfer.upload_points(x, t, tets)
    transfer.run()
    lib, ctx = transfer.lib, transfer.ctx
    ip = lambda a: a.ctypes.data_as(N.iptr)
    dp = lambda a: a.ctypes.data_as(N.dptr)
    short = np.full(n - 1 + 8, -5, np.int32)        # room for n-1 (+ a guard)
    views = (N.SolView * len(sols))()
    arrs = [np.full((n - 1 + 8) * s.shape[1], -5.0) for s in sols]
    for i, (a, s) in enumerate(zip(arrs, sols)):
        views[i].size, views[i].m = s.shape[1], dp(a)

    def refused(rc, what):
        assert rc == 0, what
        err = lib.pmx_last_error(ctx).decode()
        assert "capacity" in err or "holds" in err, err

    refused(lib.pmx_download(ctx, views, n - 1, ip(short), None, None), "pmx_download")
    assert np.all(short == -5) and all(np.all(a == -5.0) for a in arrs)
    refused(lib.pmx_download_starts(ctx, ip(short), n - 1), "pmx_download_starts")
    refused(lib.pmx_download_border(ctx, ip(short), ip(short), n - 1), "pmx_download_border")
    assert np.all(short == -5)
    q = np.full(n + 8, -5.0)
    refused(lib.pmx_new_mesh_qual(ctx, None, 0, 0, N.INQUA, 0, dp(q), n, None), "pmx_new_mesh_qual")
    refused(lib.pmx_new_mesh_qual_synced(ctx, None, N.INQUA, 1, dp(q), 8, n, None), "pmx_new_mesh_qual_synced")
    assert np.all(q == -5.0)
    # the right sizes work
    full = np.zeros(n, np.int32)
    assert lib.pmx_download_starts(ctx, ip(full), n) == 1
    q2 = np.full(n + 1, -5.0)
    assert lib.pmx_new_mesh_qual(ctx, None, 0, 0, N.INQUA, 0, dp(q2), n + 1, None) == 1
    assert np.all(q2[1:] >= 0.0)             # (random tets: many inverted, quality 0)
    # the background's qualities
    qb = np.full(m.ne + 8, -5.0)
    refused(lib.pmx_tetra_qual(ctx, 0, dp(qb), m.ne), "pmx_tetra_qual")
    assert np.all(qb == -5.0)
    assert lib.pmx_tetra_qual(ctx, 0, dp(qb), m.ne + 1) == 1


def _surface_run(tr, m, x, t, sols):
    tr.upload_background(m, sols, 0)
    tr.upload_points(x, t)
    tr.run()
    r = tr.download()
    e, v = tr.border()
    return r.elem.copy(), r.status.copy(), [s.copy() for s in r.sols], e.copy(), v.copy()


@pytest.mark.parametrize("open_surface", [False, True])
def test_fans_by_rotation_equal_sorted_fans(transfer, monkeypatch, open_surface):
    """PMMG_precompute_nodeTrias two ways (pmx_bdy.hip): the fans walked
    through the tria adjacency (closed manifold surface, checked at the
    upload) and the sorted (vertex, tria) pairs (PMX_FAN_ROTATION=0, and
    whatever the upload's check refuses: here an edge without its neighbour
    opens the surface).  Same located trias, edges, vertices and fields, bit for bit."""
    m, x, t, sols = cube_case(10, metric="iso")
    if open_surface:                                 # one edge without its neighbour
        adjt = m.adjt.copy()
        k, i = 7, 0
        a = adjt[3 * (k - 1) + 1 + i]
        adjt[3 * (k - 1) + 1 + i] = 0
        adjt[3 * (a // 3 - 1) + 1 + a % 3] = 0
        m = M.Mesh(m.xyz, m.tet, m.adja, m.tria, adjt, m.hausd)
    monkeypatch.setenv("PMX_FAN_ROTATION", "0")
    a = _surface_run(transfer, m, x, t, sols)
    monkeypatch.delenv("PMX_FAN_ROTATION")
    b = _surface_run(transfer, m, x, t, sols)
    for u, w in zip(a[:2] + a[3:], b[:2] + b[3:]):
        assert np.array_equal(u, w)
    for u, w in zip(a[2], b[2]):
        assert np.array_equal(u.view(np.uint64), w.view(np.uint64))
    assert np.count_nonzero((t != 0) & (b[1] == 1)) > 0.9 * np.count_nonzero(t != 0)



def test_fans_at_a_pinched_vertex(transfer, monkeypatch):
    """Two cubes touching at one vertex (every surface edge manifold, two
    fans at the shared vertex): the upload's check (each fan holds all the
    vertex's trias) refuses the rotation, and surface points around the
    pinch are located and interpolated as with the sorted fans."""
    from test_fans import pinched_cubes
    m, ip = pinched_cubes(3)
    c = m.xyz[ip]
    rng = np.random.default_rng(5)
    pts = []
    for sgn in (-1.0, 1.0):                      # the two sheets' faces through the pinch
        for ax in range(3):
            for _ in range(40):
                p = c + sgn * rng.uniform(0.0, 0.15, 3)
                p[ax] = c[ax]
                pts.append(p)
    x = np.array(pts)
    t = np.full(len(x), 16, np.uint16)            # MG_BDY
    sols = [M.on_vertices(m, M.iso_metric), M.on_vertices(m, lin_field)]
    monkeypatch.setenv("PMX_FAN_ROTATION", "0")
    a = _surface_run(transfer, m, x, t, sols)
    monkeypatch.delenv("PMX_FAN_ROTATION")
    b = _surface_run(transfer, m, x, t, sols)
    for u, w in zip(a[:2] + a[3:], b[:2] + b[3:]):
        assert np.array_equal(u, w)
    for u, w in zip(a[2], b[2]):
        assert np.array_equal(u.view(np.uint64), w.view(np.uint64))


@pytest.mark.parametrize("records,sample,adja", [("", "0", True), ("compact", "2", True), ("", "0", False),
                                                 ("compact", "0", False)])
def test_fresh_step_equals_upload_step(transfer, monkeypatch, records, sample, adja):
    """PMX_RUN_FRESH_BACKGROUND redoes every device pass of the uploads inside
    the step (r06): the compact walk records and the owner hint sample when the
    upload built them, the device face matching of a background sent without
    Mmg's adjacency, the fan check, and the orphan marks of the new tets --
    the latter now BEFORE the classification, so orphans are never located
    instead of located and reset.  Same bytes as the plain step whose orphan
    rows fix_orphans resets: fields, write masks, elements, status, steps,
    starts, border, locate statistics; twice in a row."""
    if records:
        monkeypatch.setenv("PMX_WALK_RECORDS", records)
    monkeypatch.setenv("PMX_HINT_SAMPLE_ORDER", sample)
    m, x, t, sols = cube_case(7, metric="ani", surface=True)
    n = len(x)
    x = x.copy()
    t = t.copy()
    t[3::53] |= M.TAG_REQ
    rng = np.random.default_rng(5)
    used = np.zeros(n, bool)
    used[: int(0.8 * n)] = True
    x[np.nonzero(~used)[0][:4]] = [1.5, -0.5, 0.5]      # orphans outside the domain
    pool = np.nonzero(used)[0]
    tets = np.zeros((len(pool) + 1, 4), np.int32)
    tets[1:] = rng.choice(pool, size=(len(pool), 4))
    tets[1:, 0] = pool
    tets[0] = -1

    def go(flags):
        transfer.upload_background(m, sols, 0, adja=adja)
        transfer.upload_points(x, t, tets)
        res = []
        for _ in range(2):
            transfer.run(flags=flags, record_starts=True)
            init = [np.full((n, s.shape[1]), -7.0) for s in sols]
            r = transfer.download(init=init)
            res.append((r, transfer.starts().copy(), transfer.border(), transfer.locate_stats()))
        return res

    a, b = go(0), go(N.RUN_FRESH_BACKGROUND)
    # (the volume hint cells take whichever sampled tet lands last -- any is a
    # valid start, the located tet does not depend on it -- so the walks'
    # starts and step counts may differ from step to step; the surface hint
    # grid is deterministic)
    bdy = (t & M.TAG_BDY) != 0
    for (ra, sa, ba, la), (rb, sb, bb, lb) in zip(a + a, b + b[::-1]):
        assert np.array_equal(ra.elem, rb.elem) and np.array_equal(ra.status, rb.status)
        assert np.array_equal(ra.steps == 0, rb.steps == 0) and np.array_equal(ra.steps < 0, rb.steps < 0)
        assert np.array_equal(ra.steps[bdy], rb.steps[bdy]) and np.array_equal(sa[bdy], sb[bdy])
        for u, v in zip(ra.sols, rb.sols):
            assert np.array_equal(u.view(np.uint64), v.view(np.uint64))
        assert np.array_equal(ba[0], bb[0]) and np.array_equal(ba[1], bb[1])
        for f in ("nvol", "nbdy", "nexhaust", "nclosest"):
            assert la[f] == lb[f], f
    r = b[0][0]
    assert np.all(r.elem[~used] == 0) and np.all(r.status[~used] == 0)
    live = used & ((t & M.TAG_REQ) == 0)
    assert np.all(r.status[live] != 0)


def test_new_tets_after_a_step_must_match_the_view(transfer):
    """A step took its orphans from the points view's new tets (r05 advisor):
    pmx_upload_new_tets afterwards accepts the same tets (promotion needs
    them), refuses others -- the orphan rows could not be undone -- and the
    refusal leaves the context as it was."""
    m, x, t, sols = cube_case(5, metric="iso", surface=True)
    n = len(x)
    rng = np.random.default_rng(2)
    used = np.zeros(n, bool)
    used[: int(0.9 * n)] = True
    pool = np.nonzero(used)[0]
    tets = np.zeros((len(pool) + 1, 4), np.int32)
    tets[1:] = rng.choice(pool, size=(len(pool), 4))
    tets[1:, 0] = pool
    tets[0] = -1
    for flags in (0, N.RUN_FRESH_BACKGROUND):
        transfer.upload_background(m, sols, 0)
        transfer.upload_points(x, t, tets)
        transfer.run(flags=flags)
        r = transfer.download()
        other = tets.copy()
        other[1:, 1] = rng.choice(np.nonzero(~used)[0], size=len(pool))
        with pytest.raises(RuntimeError, match="other tets need another pmx_run"):
            transfer.upload_new_tets(other)
        transfer.upload_new_tets(tets)               # the same tets: accepted
        r2 = transfer.download()
        assert np.array_equal(r.elem, r2.elem) and np.all(r2.elem[~used] == 0)


@pytest.mark.parametrize("order", ["coherent", "scattered"])
def test_orphan_marks_window_and_far_vertices(transfer, order):
    """The orphan marks (k_mark_new_tets_win: an LDS byte window per chunk of
    new tets, flushed as word-wide atomicOr, vertices outside the window
    stored directly) at a size where the vertex ids span far more than one
    window: every point of a valid new tet is visited, every other one is an
    orphan -- at the upload (marks with the points) and inside a FRESH step
    (marks redone by the step), with deleted tets (v[0] <= 0) among them."""
    m, x, t, sols = cube_case(48, metric="iso", surface=False, fields=False)
    n = len(x)
    assert n > 4 * 16384
    rng = np.random.default_rng(7)
    used = rng.random(n) < 0.8
    pool = np.nonzero(used)[0] + 1                   # 1-based
    if order == "coherent":
        # tets over consecutive used points (each used point in >= 1 tet)
        tv = np.concatenate([pool, pool[: (-len(pool)) % 4]]).reshape(-1, 4)
        tv = np.concatenate([tv, np.sort(rng.choice(pool, size=(len(pool) // 2, 4)), axis=0)])
    else:
        tv = rng.choice(pool, size=(len(pool), 4))
        tv[: len(pool), 0] = rng.permutation(pool)
    tets = np.zeros((len(tv) + 1, 4), np.int32)
    tets[1:] = tv
    tets[0] = 0
    # deleted tets whose vertices are orphans: they must not mark them
    dead = rng.choice(len(tv), size=len(tv) // 50, replace=False) + 1
    orph = np.nonzero(~used)[0] + 1
    tets[dead, 1:] = rng.choice(orph, size=(len(dead), 3))
    tets[dead, 0] = 0
    covered = np.zeros(n + 1, bool)
    ok = tets[1:, 0] > 0
    covered[tets[1:][ok].ravel()] = True
    covered = covered[1:]
    assert (~covered).sum() > 1000 and covered.sum() > 4 * 16384
    transfer.upload_background(m, sols, 0)
    for flags in (0, N.RUN_FRESH_BACKGROUND):
        transfer.upload_points(x, t, tets_mmg=tets)      # 1-based, v[0] = 0 deleted
        transfer.run(flags=flags)
        r = transfer.download()
        assert np.all(r.status[~covered] == 0) and np.all(r.elem[~covered] == 0), flags
        assert np.all(r.status[covered] != 0), flags
        st = transfer.locate_stats()
        assert st["nvol"] == int(covered.sum()), flags
