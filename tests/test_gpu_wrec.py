"""GPU: the walk's compact 24-B records (WRec, parmmg_amd/csrc/pmx_device.h).

k_walks reads the tet records through a 24-B copy (vertex ids as deltas from
v[0], neighbours as deltas from the tet index); a tet whose deltas do not fit
is flagged and read from the 32-B records.  Both walks must locate and
interpolate bit for bit alike, with and without escaped records (the 32-B walk
is the one the oracle parity tests pin; run flag exp 6 selects it).
"""
import numpy as np
import pytest

from helpers import cube_case, lin_field
from parmmg_amd import _native as N
from parmmg_amd import mesh as M

pytestmark = pytest.mark.gpu

FULL_RECORDS = 6 << 16            # PMX_RUN_EXP_SHIFT: exp 6 = walk on the 32-B records


@pytest.fixture(autouse=True)
def _compact_records(monkeypatch):
    """Since r06 the walk reads the 32-B records unless the upload builds the
    compact ones (PMX_WALK_RECORDS=compact, read at every background upload):
    these tests pin that path against the 32-B walk."""
    monkeypatch.setenv("PMX_WALK_RECORDS", "compact")


def _both(tr, m, x, t, sols):
    tr.upload_background(m, sols, 0)
    tr.upload_points(x, t)
    out = []
    for flags in (0, FULL_RECORDS):
        tr.run(flags=flags)
        r = tr.download()
        out.append((r.elem.copy(), r.status.copy(), [s.copy() for s in r.sols]))
    return out


def _assert_same(a, b):
    assert np.array_equal(a[0], b[0])
    assert np.array_equal(a[1], b[1])
    for u, v in zip(a[2], b[2]):
        assert np.array_equal(u.view(np.uint64), v.view(np.uint64))


def test_compact_records_equal_full_records(transfer):
    m, x, t, sols = cube_case(24, metric="ani")
    a, b = _both(transfer, m, x, t, sols)
    _assert_same(a, b)
    assert np.count_nonzero(a[0]) > 0.9 * len(x)


def test_escaped_records(transfer):
    """Vertex ids scattered over > 2^19 (np = 83^3): most vertex deltas do not
    fit 20 bits, so most records take the escape path; the outer layer of
    vertices keeps its numbering so that escaped and packed records mix."""
    n = 82
    m0 = M.kuhn_cube(n)
    npts = m0.np
    assert npts > (1 << 19)
    rng = np.random.default_rng(7)
    perm = np.arange(npts + 1)
    inner = np.nonzero(np.all((m0.xyz[1:] > 0.1) & (m0.xyz[1:] < 0.9), axis=1))[0] + 1
    perm[inner] = rng.permutation(inner)          # old id -> new id
    xyz = np.empty_like(m0.xyz)
    xyz[perm] = m0.xyz
    m = M.Mesh(xyz, perm[m0.tet].astype(np.int32), m0.adja, perm[m0.tria].astype(np.int32), m0.adjt,
               m0.hausd)
    x, t = M.new_points(n, seed=5, surface=True)
    x, t = x[::4].copy(), t[::4].copy()
    sols = [M.on_vertices(m, M.iso_metric), M.on_vertices(m, lin_field)]
    a, b = _both(transfer, m, x, t, sols)
    _assert_same(a, b)
    vol = (t == 0) & (a[1] == 1)
    assert vol.sum() > 0.5 * (t == 0).sum()
    # located volume points reproduce the linear field (the interpolation
    # went through the right vertices of the escaped records)
    ref = lin_field(x[vol])[:, 0]
    assert np.max(np.abs(a[2][1][vol, 0] - ref)) < 1e-12


FAR_AS_WHOLE = 17 << 16           # exp 17: a record with a far field read whole (r04 rule, A/B)


def _gapped(m, gap):
    """m with its tets k > ne - ne // 10 moved up by `gap` indices (deleted
    tets in between): every neighbour delta across the gap is far."""
    ne = m.ne
    k0 = ne - ne // 10
    new = np.arange(ne + 1, dtype=np.int64)
    new[k0 + 1:] += gap
    tet = np.zeros((ne + gap + 1, 4), np.int32)
    tet[new[1:]] = m.tet[1:]
    old = m.adja[1:4 * ne + 1].reshape(ne, 4).astype(np.int64)
    adja = np.zeros(4 * (ne + gap) + 1, np.int32)
    rows = np.where(old > 0, 4 * new[old >> 2] + (old & 3), 0).astype(np.int32)
    adja[1:].reshape(ne + gap, 4)[new[1:] - 1] = rows
    return M.Mesh(m.xyz, tet, adja, m.tria, m.adjt, m.hausd), new


def test_far_neighbour_fields(transfer):
    """Mmg-appended numbering past the 24-bit neighbour field (r04 verdict
    item 7): 10 % of the tets moved to the end, more than 2^23 indices away
    (deleted tets in between).  Every face across the gap escapes alone
    (pmx_wrec.h WREC_FAR) and is resolved when a walk crosses it.  The
    compact walk, the 32-B walk and the whole-record rule of r04 (exp 17)
    locate and interpolate bit for bit alike, and equal the same mesh without
    the gap (tet indices shifted back)."""
    n = 16
    m0, _ = M.numbering(M.kuhn_cube(n), "appended")
    m, new = _gapped(m0, (1 << 23) + 5)
    nfar, ntf = M.wrec_far_fields(m)
    assert M.wrec_escapes(m) == 0 and ntf > 0.3 * m0.ne, (nfar, ntf)
    x, t = M.new_points(n, seed=9, surface=True)
    sols = [M.on_vertices(m0, M.iso_metric), M.on_vertices(m0, lin_field)]
    out = []
    transfer.upload_background(m, sols, 0)
    transfer.upload_points(x, t)
    for flags in (0, FULL_RECORDS, FAR_AS_WHOLE):
        transfer.run(flags=flags)
        r = transfer.download()
        out.append((r.elem.copy(), r.status.copy(), [s.copy() for s in r.sols]))
    _assert_same(out[0], out[1])
    _assert_same(out[0], out[2])
    transfer.upload_background(m0, sols, 0)
    transfer.upload_points(x, t)
    transfer.run()
    r = transfer.download()
    e = r.elem.astype(np.int64)
    vol = (t == 0) & (r.status == 1)
    assert vol.sum() > 0.9 * (t == 0).sum()
    assert np.array_equal(out[0][0][vol], new[e[vol]])
    for u, v in zip(out[0][2], r.sols):
        assert np.array_equal(u[vol].view(np.uint64), v[vol].view(np.uint64))
    ref = lin_field(x[vol])[:, 0]
    assert np.max(np.abs(out[0][2][1][vol, 0] - ref)) < 1e-12


def test_hint_sample_order(transfer, monkeypatch):
    """The hint samples of pmx_ctx::order_hint_samples -- every 4th tet in tet
    order, packed with the tet records (0, the default since r06), one owner
    tet per vertex (2) -- carry their tet indices: on an appended numbering the
    step locates and interpolates bit for bit alike, with walks as short, and
    a FRESH step (which rebuilds the owner sample) gives the same results."""
    m, _ = M.numbering(M.kuhn_cube(16), "appended")
    x, t = M.new_points(16, seed=3, surface=True)
    sols = [M.on_vertices(m, M.iso_metric), M.on_vertices(m, lin_field)]
    out = []
    for order in ("0", "2"):
        monkeypatch.setenv("PMX_HINT_SAMPLE_ORDER", order)
        transfer.upload_background(m, sols, 0)
        transfer.upload_points(x, t)
        for flags in (0, N.RUN_FRESH_BACKGROUND):
            transfer.run(record_starts=True, flags=flags)
            r = transfer.download()
            out.append((r.elem.copy(), r.status.copy(), [s.copy() for s in r.sols],
                        transfer.locate_stats()["stepav"], transfer.starts().copy()))
    for o in out[1:]:
        _assert_same(out[0], o)
    assert out[2][3] < 1.2 * out[0][3], (out[0][3], out[2][3])
    vol = (t == 0) & (out[0][1] == 1)
    assert not np.array_equal(out[0][4][vol], out[2][4][vol])       # other start tets
    assert np.array_equal(out[2][4], out[3][4])                     # the FRESH rebuild: same sample


COMPACT_FORCED = 18 << 16         # exp 18: compact records whatever their far fields


def test_record_format_switch_at_size(transfer):
    """An Mmg-appended numbering of 10.4 M tets (kuhn n = 120) with its moved
    tenth 2^23 indices further up: a fifth of the 18.8 M tet slots have a far
    neighbour field, above the 1/16 at which the walk takes the 32-B records
    (pmx_capi.hip fill_vol_args).  The default step, the
    compact records forced (exp 18: far fields resolved as crossed) and the
    32-B walk forced (exp 6) agree bit for bit."""
    n = 120
    m0, _ = M.numbering(M.kuhn_cube(n), "appended")
    m, _ = _gapped(m0, (1 << 23) + 5)
    far, ntf = M.wrec_far_fields(m)
    assert ntf * 16 > m.ne, (far, ntf, m.ne)
    x, t = M.new_points(n, seed=4, surface=True)
    x, t = x[::8].copy(), t[::8].copy()
    sols = [M.on_vertices(m0, M.iso_metric), M.on_vertices(m0, lin_field)]
    transfer.upload_background(m, sols, 0)
    transfer.upload_points(x, t)
    out = []
    for flags in (0, COMPACT_FORCED, FULL_RECORDS):
        transfer.run(flags=flags)
        r = transfer.download()
        out.append((r.elem.copy(), r.status.copy(), [s.copy() for s in r.sols]))
    _assert_same(out[0], out[1])
    _assert_same(out[0], out[2])
    vol = (t == 0) & (out[0][1] == 1)
    assert vol.sum() > 0.9 * (t == 0).sum()
    assert np.max(np.abs(out[0][2][1][vol, 0] - lin_field(x[vol])[:, 0])) < 1e-12
