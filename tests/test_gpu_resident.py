"""Device residency across ParMmg iterations (pmx_upload_new_tets +
pmx_promote_background) against a full host upload of the same background.

PMMG_update_oldGrps (reference src/libparmmg1.c:653) makes the group's current
mesh -- the last iteration's new mesh with its interpolated metric and fields --
the next iteration's background.  Promoting the device-resident new points and
results must give the same background as uploading that mesh from the host
(coordinates, downloaded fields, Mmg adjacency): the next step's elements,
statuses and fields are compared bit for bit.
"""
import numpy as np
import pytest

from helpers import bits_equal
from parmmg_amd import _native as N
from parmmg_amd import mesh as M
from parmmg_amd.transfer import Transfer

pytestmark = pytest.mark.gpu


def new_mesh(n, seed):
    """A "remeshed" group: a jittered Kuhn cube; its vertices are the new
    points (boundary vertices tagged MG_BDY), its tets the new tets."""
    m = M.kuhn_cube(n, seed=seed)
    x = m.xyz[1:].copy()
    onb = np.any((x == 0.0) | (x == 1.0), axis=1)
    t = np.where(onb, M.TAG_BDY, 0).astype(np.uint16)
    tets0 = m.tet.copy() - 1
    tets0[0] = -1
    return m, x, t, tets0


def fields(m):
    return [M.on_vertices(m, M.shock_metric), M.on_vertices(m, M.level_set),
            M.on_vertices(m, M.velocity)]


def mmg_layout(rows):
    out = np.zeros((rows.shape[0] + 1, rows.shape[1]))
    out[1:] = rows
    return out


def compare(a, b, nsol):
    assert np.array_equal(a.elem, b.elem)
    assert np.array_equal(a.status, b.status)
    for s in range(nsol):
        assert bits_equal(a.sols[s], b.sols[s]).all(), f"sol {s} differs"


@pytest.mark.parametrize("adja,residency", [(True, False), (False, False), (False, True),
                                             (True, True)])
def test_promoted_background_equals_host_upload(adja, residency):
    """residency: the next background's tet records are built on the device
    while the step runs (pmx_set_residency) and swapped in by the promotion."""
    m1 = M.kuhn_cube(7, seed=101)
    sols1 = fields(m1)
    m2, x2, t2, tets2 = new_mesh(8, 202)
    m3, x3, t3, tets3 = new_mesh(6, 303)
    # rows the step does not write keep "Mmg's" values (init)
    init2 = [np.full((len(x2), s.shape[1]), -3.0) for s in sols1]
    init2[0][::97] = 0.25                      # a few distinct values

    tr = Transfer(0)
    tr.set_residency(residency)
    tr.upload_background(m1, sols1, 0)
    tr.upload_points(x2, t2, tets2)
    tr.run()
    r2 = tr.download(init=init2)
    assert (r2.status != 0).any()
    # next iteration, resident: the new mesh (trias, adjacency) + results
    tr.promote_background(m2, r2.sols, adja=adja)
    tr.upload_points(x3, t3, tets3)
    tr.run()
    r3 = tr.download()

    ref = Transfer(0)
    ref.upload_background(m2, [mmg_layout(s) for s in r2.sols], 0)
    ref.upload_points(x3, t3, tets3)
    ref.run()
    r3ref = ref.download()
    compare(r3, r3ref, len(sols1))
    # and one more iteration on the promoted background of the promoted one
    tr.promote_background(m3, r3.sols, adja=adja)
    tr.upload_points(x2, t2, tets2)
    tr.run()
    r4 = tr.download()
    ref.upload_background(m3, [mmg_layout(s) for s in r3.sols], 0)
    ref.upload_points(x2, t2, tets2)
    ref.run()
    compare(r4, ref.download(), len(sols1))
    tr.close()
    ref.close()


def test_rows_not_written_come_from_the_caller():
    """Orphan (in no valid new tet) and NUL points are not located: their rows
    of the promoted background are the caller's values."""
    m1 = M.kuhn_cube(6, seed=11)
    sols1 = fields(m1)[:2]
    m2, x2, t2, tets2 = new_mesh(5, 22)
    t2 = t2.copy()
    t2[7] = M.TAG_NUL
    init = [np.full((len(x2), s.shape[1]), 0.5) for s in sols1]
    tr = Transfer(0)
    tr.upload_background(m1, sols1, 0)
    tr.upload_points(x2, t2, tets2)
    tr.upload_new_tets(tets2)
    tr.run()
    r2 = tr.download(init=init)
    assert np.all(r2.sols[0][7] == 0.5)
    tr.promote_background(m2, r2.sols)
    # the promoted background's statistics see the caller's row 7 (through
    # the quality of the tets around vertex 8 in the anisotropic metric)
    ref = Transfer(0)
    ref.upload_background(m2, [mmg_layout(s) for s in r2.sols], 0)
    assert np.array_equal(tr.tetra_qual(m2.ne), ref.tetra_qual(m2.ne))
    assert tr.prilen() == ref.prilen()
    tr.close()
    ref.close()


def test_promote_requires_step_and_tets():
    m1 = M.kuhn_cube(4, seed=1)
    m2, x2, t2, tets2 = new_mesh(4, 2)
    tr = Transfer(0)
    tr.upload_background(m1, fields(m1)[:1], 0)
    tr.upload_points(x2, t2)                      # no tets with the points
    with pytest.raises(RuntimeError, match="no step"):
        tr.promote_background(m2, None)
    tr.run()
    r = tr.download()
    with pytest.raises(RuntimeError, match="new tets"):
        tr.promote_background(m2, r.sols)
    tr.upload_new_tets(tets2)
    bad = M.kuhn_cube(5, seed=2)
    with pytest.raises(RuntimeError, match="sizes"):
        tr.promote_background(bad, r.sols)
    # an adjacency entry past the last face is refused before anything moves
    # (the walks would gather through it), and the step stays promotable
    saved = m2.adja.copy()
    m2.adja[4 * 3 + 2] = 4 * m2.ne + 4
    with pytest.raises(RuntimeError, match="adjacency entry out of range"):
        tr.promote_background(m2, r.sols)
    m2.adja[:] = saved
    tr.promote_background(m2, r.sols)
    with pytest.raises(RuntimeError, match="upload background and points"):
        tr.run()                                  # the points were consumed
    tr.close()


@pytest.mark.parametrize("use_perm,copy_metric", [(False, True), (True, True), (True, False)])
@pytest.mark.parametrize("eager", [False, True])
def test_copy_required_on_device(use_perm, copy_metric, eager):
    """pmx_copy_required: the frozen (MG_REQ) background points' values land
    in the rows of their new points that the step did not write -- the
    reference's PMMG_copySol_point (src/interpmesh_pmmg.c:311-358) before the
    interpolation, which then overwrites the rows it writes."""
    m1 = M.kuhn_cube(5, seed=31)
    sols1 = fields(m1)
    m2, x2, t2, tets2 = new_mesh(6, 32)
    np1, np2 = m1.np, len(x2)
    perm = np.zeros(np1 + 1, np.int32)
    perm[1:] = (np2 - np.arange(1, np1 + 1) + 1) if use_perm else np.arange(1, np1 + 1)
    tags1 = np.zeros(np1 + 1, np.uint16)
    req = np.array([3, 10, 27, 50, 51, 120, 200])
    tags1[req] = M.TAG_REQ
    t2 = t2.copy()
    frozen = req[req != 50]                       # old point 50's new point is not frozen
    t2[perm[frozen] - 1] |= M.TAG_REQ
    init = [np.full((np2, s.shape[1]), -9.0) for s in sols1]

    def step(copy):
        tr = Transfer(0)
        tr.upload_background(m1, sols1, 0)
        tr.upload_point_tags(tags1)
        tr.upload_points(x2, t2, tets2)
        # eager: the fields' copy started with the step is dropped by the copy
        tr.run(flags=N.RUN_EAGER_DOWNLOAD if eager else 0)
        if copy:
            tr.copy_required(perm if use_perm else None, copy_metric)
        r = tr.download(init=init)
        tr.close()
        return r

    r0, r1 = step(False), step(True)
    expect = [a.copy() for a in r0.sols]
    for s in range(len(sols1)):
        if s == 0 and not copy_metric:
            continue
        for ip in frozen:
            expect[s][perm[ip] - 1] = sols1[s][ip]
    for s in range(len(sols1)):
        assert bits_equal(r1.sols[s], expect[s]).all(), f"sol {s}"
    j50 = perm[50] - 1
    assert np.all(r1.sols[1][j50] == r0.sols[1][j50]) and r0.sols[1][j50][0] != -9.0
