"""C1 (unit cube, n = 20, 48k tets, -hsiz 0.05) through the
drop-in seam PMX_interpMetricsAndFields.

Reference (src/interpmesh_pmmg.c:497-512): with -hsiz the metric is
MMG3D_Set_constantSize's -- every MG_VOK point gets hsiz (iso) or
diag(1/hsiz^2) (ani), MG_NUL rows are untouched -- and when there is no field
nothing is located at all; with a field (the "+LS" variant) the fields are
interpolated as usual while the metric stays constant.
"""
import numpy as np
import pytest

from helpers import bits_equal, compare_exact, compare_volume
from oracle import oracle as O
from parmmg_amd import mesh as M

pytestmark = pytest.mark.gpu

N1 = 20
HSIZ = 0.05
SENT = -7.0


def c1_inputs(metric):
    m = M.kuhn_cube(N1)
    x, t = M.new_points(N1)
    t = t.copy()
    t[5::17] |= M.TAG_REQ                      # frozen (MG_REQ) points
    t[7::23] = M.TAG_NUL                       # !MG_VOK points
    size = 6 if metric == "ani" else 1
    old_met = M.on_vertices(m, M.shock_metric if metric == "ani" else M.iso_metric)
    xyz1 = np.concatenate([np.zeros((1, 3)), x])
    tag1 = np.concatenate([np.zeros(1, np.uint16), t])
    met = np.full((len(xyz1), size), SENT)
    return m, x, t, old_met, xyz1, tag1, met


def expected_constant(size):
    if size == 1:
        return np.array([HSIZ])
    v = 1.0 / (HSIZ * HSIZ)
    return np.array([v, 0.0, 0.0, v, 0.0, v])


@pytest.mark.parametrize("metric", ["iso", "ani"])
def test_c1_constant_size_no_fields(transfer, metric):
    """No field: MMG3D_Set_constantSize on every valid point, no locate."""
    m, x, t, old_met, xyz1, tag1, met = c1_inputs(metric)
    g = dict(old_mesh=m, old_met=old_met, old_fields=[], xyz=xyz1, tags=tag1, met=met, fields=[],
             hsiz=HSIZ)
    assert transfer.interp_metrics_and_fields([g], input_met=1) == 1
    got = met[1:]
    nul = t >= M.TAG_NUL
    assert np.all(got[nul] == SENT)                              # untouched
    assert np.all(got[~nul] == expected_constant(met.shape[1])[None, :])
    assert np.all(met[0] == SENT)                                # slot 0 untouched
    # nothing was located: no step ran on these points
    with pytest.raises(RuntimeError, match="no step has run"):
        transfer.locate_stats()


@pytest.mark.parametrize("metric", ["iso", "ani"])
def test_c1_constant_size_with_level_set(transfer, metric):
    """-hsiz + a level-set field: the constant metric on every valid point,
    the field interpolated (against the oracle: every volume point bit-exact
    or a verified tie), frozen and invalid rows untouched."""
    m, x, t, old_met, xyz1, tag1, met = c1_inputs(metric)
    ls = M.on_vertices(m, M.level_set)
    field = np.full((len(xyz1), 1), SENT)
    g = dict(old_mesh=m, old_met=old_met, old_fields=[ls], xyz=xyz1, tags=tag1, met=met,
             fields=[field], hsiz=HSIZ)
    assert transfer.interp_metrics_and_fields([g], input_met=1) == 1
    nul = t >= M.TAG_NUL
    req = ((t & M.TAG_REQ) != 0) & ~nul
    assert np.all(met[1:][nul] == SENT)
    assert np.all(met[1:][~nul] == expected_constant(met.shape[1])[None, :])
    f = field[1:]
    assert np.all(f[nul | req] == SENT)                          # not interpolated
    assert not np.any(f[~(nul | req)] == SENT)
    # the seam returns no elements: the same inputs through a direct step
    # give them; the seam's field must be that step's bit for bit
    transfer.upload_background(m, [ls], -1)
    transfer.upload_points(x, t)
    transfer.run(record_starts=True)
    r = transfer.download(init=[np.full((len(x), 1), SENT)])
    starts = transfer.starts()
    edge, vert = transfer.border()
    assert bits_equal(f, r.sols[0]).all()
    o = O.Oracle(m)
    outs, elem, st, *_ = o.interp(x, t, [ls], imet=-1, init=[np.full((len(x), 1), SENT)])
    c = compare_volume(o, x, t, ([f], r.elem, r.status), (outs, elem, st), [ls])
    assert c["nvol"] == int((t == 0).sum())
    assert c["same"] >= c["nvol"] - max(3, c["nvol"] // 1000)
    # surface points (frozen and invalid ones aside): bit-exact against the
    # oracle in device semantics -- each query from the device's start tria,
    # the point flags as PMMG_precompute_nodeTrias leaves them -- elements,
    # edge / vertex classification, status and the interpolated level set
    bdy = np.nonzero(((t & M.TAG_BDY) != 0) & ~(nul | req))[0]
    assert len(bdy) > 0
    so, se, ss, _, sed, sve = o.interp(x, t, [ls], imet=-1, order=bdy, fresh=True, start_vol=starts,
                                       start_bdy=starts, init=[np.full((len(x), 1), SENT)])
    compare_exact(([f], r.elem, r.status, edge, vert), (so, se, ss, sed, sve), bdy, 1)


def test_c1_constant_size_step_ani(transfer):
    """The device step's own -hsiz path (pmx_run hsiz > 0) with an ani metric
    and a field at n = 20: metric rows = diag(1/h^2) on every valid point."""
    m, x, t, old_met, *_ = c1_inputs("ani")
    ls = M.on_vertices(m, M.level_set)
    transfer.upload_background(m, [old_met, ls], 0)
    transfer.upload_points(x, t)
    transfer.run(hsiz=HSIZ)
    r = transfer.download(init=[np.full((len(x), 6), SENT), np.full((len(x), 1), SENT)])
    nul = t >= M.TAG_NUL
    assert np.all(r.sols[0][nul] == SENT)
    assert np.all(r.sols[0][~nul] == expected_constant(6)[None, :])
