"""GPU statistics (PMMG_qualhisto / PMMG_prilen / PMMG_tetraQual) against the oracle.

* ridge points (MMG5_Point.tag): the length loop's 4-ridge filter
  (reference src/quality_pmmg.c:509-517) and MMG3D_computeOutqua's nrid;
* PMMG_count_nodes_par (:33-80) against the oracle's restatement;
* the distributed prilen of a partition with parallel edges (:398-502), in the
  reference's semantics (interface edges counted by both ranks, :585-586) and
  exactly once;
* the quality of the NEW mesh right after the interpolation
  (src/libparmmg1.c:845): per-tet qualities bit-exact against the oracle's
  MMG3D_tetraQual on the new mesh with the same metric;
* the RCCL reduction with one rank equals the host fold of the same partial.

Sums (avg, avlen) are compared within 1e-12 relative: the device reduces in a
different order than the reference's sequential loop; everything else (counts,
histograms, minima/maxima and the elements realising them, per-tet qualities)
is exact.  Edge-length histogram bins may differ for lengths within an ulp of
a bin boundary (the length is the same formula but a different operation
order); the tests allow a couple of such edges.
"""
import numpy as np
import pytest
import torch

from helpers import compare_volume, cube_case, split_partitions
from oracle import oracle as O
from parmmg_amd import _native as N
from parmmg_amd import mesh as M
from parmmg_amd import shard
from parmmg_amd.transfer import Transfer, comm_unique_id

pytestmark = pytest.mark.gpu

GEO, REQ, NOM, CRN = 2, 4, 8, 32


def assert_len_equal(L, Lo, hl_slack=0):
    assert L["ned"] == Lo["ned"] and L["nullEdge"] == Lo["nullEdge"]
    assert sum(abs(a - b) for a, b in zip(L["hl"], Lo["hl"])) <= hl_slack
    assert abs(L["avlen"] - Lo["avlen"]) <= 1e-12 * abs(Lo["avlen"])
    assert L["lmin"] == Lo["lmin"] and L["lmax"] == Lo["lmax"]   # glibc's log1p restated (r06)
    if L["lmin"] == Lo["lmin"]:
        assert (L["amin"], L["bmin"]) == (Lo["amin"], Lo["bmin"])
    if L["lmax"] == Lo["lmax"]:
        assert (L["amax"], L["bmax"]) == (Lo["amax"], Lo["bmax"])


def assert_qual_equal(h, ho):
    for f in ("ne", "iel", "good", "med", "min", "max", "nrid"):
        assert h[f] == ho[f], f
    assert h["his"] == ho["his"]
    assert abs(h["avg"] - ho["avg"]) <= 1e-12 * abs(ho["avg"])


def ridge_tags(m, seed=3):
    """Ridge points on the x < 0.4 slab (mixed with singular / non-manifold
    ones that are NOT ridge points for the filter)."""
    rng = np.random.default_rng(seed)
    tags = np.zeros(m.np + 1, np.uint16)
    slab = np.nonzero(m.xyz[:, 0] < 0.4)[0]
    slab = slab[slab > 0]
    tags[slab] = GEO
    extra = rng.choice(slab, size=len(slab) // 6, replace=False)
    tags[extra[: len(extra) // 3]] |= REQ
    tags[extra[len(extra) // 3: 2 * len(extra) // 3]] |= NOM
    tags[extra[2 * len(extra) // 3:]] |= CRN
    return tags


@pytest.mark.parametrize("metric", ["iso", "ani"])
def test_ridge_filter_and_outqua(transfer, metric):
    m, x, t, sols = cube_case(7, metric=metric, fields=False)
    tags = ridge_tags(m)
    transfer.upload_background(m, sols, 0)
    transfer.upload_point_tags(tags)
    L = transfer.prilen()
    Lo = O.prilen(m, sols[0], tags=tags)
    Lall = O.prilen(m, sols[0])
    assert Lo["ned"] + Lo["nullEdge"] < Lall["ned"] + Lall["nullEdge"], "the filter must bite"
    assert_len_equal(L, Lo)
    met = sols[0] if metric == "ani" else None
    # OUTQUA: MMG3D_computeOutqua's MMG5_orcal (ridge-storage mean for a
    # tensor metric); INQUA: MMG3D_computeInqua's MMG5_caltet33_ani
    qr = O.tetra_qual(m, met, tags=tags, met_rid_typ=1)
    qo = O.tetra_qual(m, met)
    h = transfer.qualhisto(N.OUTQUA)
    ho = O.qualhisto(m, qr, tags=tags)
    assert ho["nrid"] > 0
    assert_qual_equal(h, ho)
    hin = transfer.qualhisto(N.INQUA)
    assert hin["nrid"] == 0 and hin["ne"] == ho["ne"]
    assert_qual_equal(hin, O.qualhisto(m, qo))
    # tags dropped: the filter is off again
    transfer.upload_point_tags(None)
    assert_len_equal(transfer.prilen(), Lall)


def test_count_nodes_matches_oracle(transfer):
    m = M.kuhn_cube(6)
    transfer.upload_background(m, [M.on_vertices(m, M.iso_metric)], 0)
    rng = np.random.default_rng(11)
    nitem = 60
    idx_ip = rng.choice(np.arange(1, m.np + 1), size=45, replace=False).astype(np.int32)
    idx_comm = rng.choice(nitem, size=45, replace=False).astype(np.int32)
    iv = np.zeros(nitem, np.int32)
    iv[rng.choice(nitem, size=20, replace=False)] = 1     # nodes another rank counts
    iv_o = iv.copy()
    n = transfer.count_nodes(idx_ip, idx_comm, iv, base=1)
    no = O.count_nodes(m, idx_ip, idx_comm, iv_o)
    assert n == no and np.array_equal(iv, iv_o)
    assert transfer.count_nodes() == m.np               # no communicator: touched points
    # the partial carries the count
    d = torch.zeros(shard.QUAL_WORDS, dtype=torch.float64, device="cuda:0")
    transfer.count_nodes(idx_ip, idx_comm, np.zeros(nitem, np.int32))
    transfer.qualhisto_device(d.data_ptr())
    transfer.synchronize()
    assert shard.fold_qual(d.cpu().numpy()[None])["np"] == O.count_nodes(
        m, idx_ip, idx_comm, np.zeros(nitem, np.int32))


@pytest.mark.parametrize("once", [0, 1])
def test_distributed_prilen_partitions(transfer, once):
    """Both partitions of a split cube: each rank's partial matches the
    oracle's PMMG_computePrilen, and the two partials add up to the whole
    cube's edges (plus the interface edges again in the reference's semantics)."""
    full = M.kuhn_cube(6)
    parts, nshared = split_partitions(full)
    tot = 0
    for rank, (mr, glob, par) in enumerate(parts):
        met = M.on_vertices(mr, M.shock_metric)
        p = dict(par, myrank=rank, owner=np.zeros(len(par["a"]), np.int32), exact_once=once)
        transfer.upload_background(mr, [met], 0)
        L = transfer.prilen(par=p)
        Lo = O.prilen(mr, met, par=p)
        assert_len_equal(L, Lo)
        tot += L["ned"] + L["nullEdge"]
    n = 6
    edges = 3 * n * (n + 1) ** 2 + 3 * n * n * (n + 1) + n ** 3
    assert tot == edges + (0 if once else nshared)


@pytest.mark.parametrize("metric", ["iso", "ani"])
def test_new_mesh_quality_after_interpolation(transfer, metric):
    """PMMG_tetraQual on the new mesh right after PMMG_interpMetricsAndFields:
    the new tets, the device-resident new points and interpolated metric."""
    m, _, _, sols = cube_case(6, metric=metric, fields=False)
    new = M.kuhn_cube(9, seed=77)                 # the "remeshed" group: another jittered cube
    x = new.xyz[1:].copy()
    t = np.zeros(len(x), np.uint16)
    tets0 = new.tet.copy() - 1                    # 0-based point indices
    tets0[0] = -1
    transfer.upload_background(m, sols, 0)
    transfer.upload_points(x, t, tets0)
    transfer.run()
    r = transfer.download()
    q = transfer.new_mesh_qual(tets0, N.INQUA)
    met = np.zeros((new.np + 1, sols[0].shape[1]))
    met[1:] = r.sols[0]
    qo = O.tetra_qual(new, met if metric == "ani" else None)
    assert np.array_equal(q[1:], qo[1:]), "new-mesh quality not bit-exact"
    # the partial of the new mesh (np = the points)
    d = torch.zeros(shard.QUAL_WORDS, dtype=torch.float64, device="cuda:0")
    transfer.new_mesh_qual(tets0, N.INQUA, d.data_ptr())
    transfer.synchronize()
    h = shard.fold_qual(d.cpu().numpy()[None])
    ho = O.qualhisto(new, qo)
    assert_qual_equal(dict(h, nrid=0), dict(ho, nrid=0))
    assert h["np"] == len(x)
    # the oracle's own interpolation (carry-over walk) gives the same metric
    # on all but documented ties, hence the same qualities on their tets
    o = O.Oracle(m)
    outs, elem, st, *_ = o.interp(x, t, sols, imet=0)
    same = np.all(outs[0].view(np.int64) == r.sols[0].view(np.int64), axis=1)
    mo = np.zeros_like(met)
    mo[1:] = outs[0]
    qo2 = O.tetra_qual(new, mo if metric == "ani" else None)
    c = compare_volume(o, x, t, (r.sols, r.elem, r.status), (outs, elem, st), sols)
    assert c["same"] + c["ties"] == len(x)
    # the new cube's boundary points lie on background faces: many ties there
    good = np.all(same[new.tet[1:] - 1], axis=1)
    assert good.mean() > 0.9
    assert np.array_equal(q[1:][good], qo2[1:][good])


def test_new_mesh_quality_deleted_tets_and_bad_index(transfer):
    m, _, _, sols = cube_case(5, metric="ani", fields=False)
    new = M.kuhn_cube(4, seed=5)
    x = new.xyz[1:].copy()
    tets0 = new.tet.copy() - 1
    tets0[0] = -1
    tets0[3, 0] = -1                               # deleted (!MG_EOK)
    transfer.upload_background(m, sols, 0)
    transfer.upload_points(x, np.zeros(len(x), np.uint16), tets0)
    transfer.run()
    r = transfer.download()
    q = transfer.new_mesh_qual(tets0)
    assert q[3] == 0.0 and np.all(q[4:] > 0)
    bad = tets0.copy()
    bad[2, 1] = len(x)                             # outside the uploaded points
    with pytest.raises(RuntimeError, match="outside"):
        transfer.new_mesh_qual(bad)


@pytest.mark.parametrize("metric", ["iso", "ani"])
def test_new_mesh_quality_synced_into_tetra_records(transfer, metric):
    """PMMG_tetraQual at :845 through pmx_new_mesh_qual_synced, the qualities
    written straight into MMG5_Tetra.qual (stride 48 B) for the valid tets
    only -- a deleted tet keeps its value, as MMG3D_tetraQual skips !MG_EOK --
    equal to the dense output and to the oracle.  Sizes past 2^20 tets run
    the chunked download (several chunks)."""
    m, _, _, sols = cube_case(6, metric=metric, fields=False)
    new = M.kuhn_cube(56, seed=3)                  # 56^3 * 6 = 1.05M tets: 2 chunks
    x = new.xyz[1:].copy()
    t = np.zeros(len(x), np.uint16)
    tv = new.tet.copy()
    tv[0] = 0
    tv[7, 0] = 0                                   # deleted (!MG_EOK)
    transfer.upload_background(m, sols, 0)
    transfer.upload_points(x, t, tets_mmg=tv)
    transfer.run()
    r = transfer.download()
    met = np.concatenate([np.zeros((1, sols[0].shape[1])), r.sols[0]])
    rec = np.zeros(tv.shape[0], M.MMG_TETRA)
    rec["v"] = tv
    rec["qual"] = -1.0
    transfer.new_mesh_qual_synced(met, out=rec)
    qd = transfer.new_mesh_qual_synced(met)
    qo = O.tetra_qual(M.Mesh(new.xyz, tv, new.adja, new.tria, new.adjt), met if metric == "ani" else None,
                      tags=np.zeros(new.np + 1, np.uint16), met_rid_typ=1)
    assert rec["qual"][7] == -1.0 and qd[7] == 0.0
    ok = np.arange(tv.shape[0]) != 7
    ok[0] = False
    assert np.array_equal(rec["qual"][ok], qd[ok])
    assert np.array_equal(qd.view(np.int64)[ok], qo.view(np.int64)[ok])


def test_new_tets_shuffled_numbering(transfer):
    """The points view's tets with a shuffled numbering of > 2^20 points (vertex
    indices of one tet far apart) and a deleted tet: the device's copy must be
    the caller's -- the new-mesh qualities (computed on it) bit-exact against
    the oracle's on the caller's tets -- and exactly the points in no valid
    tet are orphans (never visited)."""
    m, _, _, sols = cube_case(6, metric="iso", fields=False)
    n = 104
    x, t = M.new_points(n, surface=False)                # 1.12 M volume points
    tv = M.new_point_tets(n, x, t)
    perm = np.random.default_rng(3).permutation(len(x))  # new index of point j
    xs = np.empty_like(x)
    xs[perm] = x
    tvs = tv.copy()
    tvs[1:] = perm[tv[1:] - 1] + 1
    tvs[5, 0] = 0                                         # a deleted tet among them
    transfer.upload_background(m, sols, 0)
    transfer.upload_points(xs, np.zeros(len(x), np.uint16), tets_mmg=tvs)
    transfer.run()
    r = transfer.download()
    used = np.zeros(len(x), bool)
    used[tvs[1:][tvs[1:, 0] > 0].ravel() - 1] = True      # points of valid tets
    assert np.all(r.status[used] == 1) and np.all(r.status[~used] == 0)
    q = transfer.new_mesh_qual(None)
    xyz1 = np.concatenate([np.zeros((1, 3)), xs])
    qo = O.tetra_qual(M.Mesh(xyz1, tvs, None, np.zeros((1, 3), np.int32), None), None)
    assert q[5] == 0.0
    assert np.array_equal(q.view(np.int64)[1:], qo.view(np.int64)[1:])


def test_rccl_single_rank_equals_fold(transfer):
    """pmx_qualhisto_allreduce / pmx_prilen_allreduce over a 1-rank RCCL
    communicator: the all-gather + fold of the group partials equals the
    host fold of the same partials."""
    m, x, t, sols = cube_case(6, metric="ani", fields=False)
    transfer.upload_background(m, sols, 0)
    comm = transfer.comm_init(1, comm_unique_id(), 0)
    try:
        d = torch.zeros((2, shard.QUAL_WORDS), dtype=torch.float64, device="cuda:0")
        transfer.qualhisto_device(d[0].data_ptr())
        transfer.qualhisto_device(d[1].data_ptr())     # a second "group"
        dl = torch.zeros(shard.LEN_WORDS, dtype=torch.float64, device="cuda:0")
        transfer.prilen_device(dl.data_ptr())
        transfer.synchronize()
        rq = transfer.qualhisto_allreduce(comm, 1, d.data_ptr(), 2)
        rl = transfer.prilen_allreduce(comm, 1, dl.data_ptr())
    finally:
        transfer.comm_destroy(comm)
    fq = shard.fold_qual(d.cpu().numpy(), np.zeros(2, np.int32))
    fl = shard.fold_len(dl.cpu().numpy()[None])
    assert rq == fq and rl == fl
    assert rq["ne"] == 2 * m.ne and rq["cpu"] == 0 and rq["iel_grp"] == 0


@pytest.mark.parametrize("metric", ["iso", "ani"])
def test_tetra_qual_ridge_metric_storage(transfer, metric):
    """MMG3D_tetraQual(mesh, met, metRidTyp) (src/quality_pmmg.c:726; ParMmg's
    own call is PMMG_tetraQual(parmesh,1), src/libparmmg1.c:845): with a
    tensor metric, 1 averages it over the vertices that are not non-singular
    ridge points (MMG5_moymet; quality 0 when all 4 are), 0 over all 4
    (MMG5_caltet33_ani).  Bit-exact against the oracle's restatement, on the
    background and on the new mesh of a step (the points view's tags)."""
    m, x, t, sols = cube_case(7, metric=metric, fields=False)
    tags = ridge_tags(m)
    met = sols[0] if metric == "ani" else None
    transfer.upload_background(m, sols, 0)
    transfer.upload_point_tags(tags)
    q1, q0 = transfer.tetra_qual(m.ne, 1), transfer.tetra_qual(m.ne, 0)
    o1 = O.tetra_qual(m, met, tags=tags, met_rid_typ=1)
    o0 = O.tetra_qual(m, met)
    assert np.array_equal(q1.view(np.int64)[1:], o1.view(np.int64)[1:])
    assert np.array_equal(q0.view(np.int64)[1:], o0.view(np.int64)[1:])
    if metric == "ani":
        assert np.count_nonzero(q1 != q0) > 0, "the ridge points must change the mean metric"
        assert np.count_nonzero(o1[1:] == 0.0) > 0      # tets with 4 ridge points
    else:
        assert np.array_equal(q1, q0)
    # the new mesh of a step: a jittered Kuhn mesh whose points are located in
    # m, its tags the points view's
    nm = M.kuhn_cube(6, seed=77)
    ntags = ridge_tags(nm) & ~np.uint16(REQ)     # frozen points are not interpolated
    transfer.upload_points(nm.xyz[1:], ntags[1:], tets_mmg=nm.tet)
    transfer.run()
    r = transfer.download()
    qn = transfer.new_mesh_qual(None, met_rid_typ=1)
    metn = None
    if metric == "ani":
        metn = np.concatenate([np.zeros((1, 6)), r.sols[0]])
    on = O.tetra_qual(nm, metn, tags=ntags, met_rid_typ=1)
    assert np.array_equal(qn.view(np.int64)[1:], on.view(np.int64)[1:])


def assert_len_exact(L, Lo):
    """Tensor-metric lengths: sqrt and divisions correctly rounded on both
    sides, no log1p -- counts, bins, extrema and their endpoints bit for bit."""
    for f in ("ned", "nullEdge", "amin", "bmin", "amax", "bmax"):
        assert L[f] == Lo[f], (f, L[f], Lo[f])
    assert L["hl"] == Lo["hl"], (L["hl"], Lo["hl"])
    assert L["lmin"] == Lo["lmin"] and L["lmax"] == Lo["lmax"], (L, Lo)
    assert abs(L["avlen"] - Lo["avlen"]) <= 1e-12 * abs(Lo["avlen"])


@pytest.mark.parametrize("mrt", [0, 1])
@pytest.mark.parametrize("with_surface", [False, True])
def test_prilen_tensor_surface_and_ridge_storage(transfer, mrt, with_surface):
    """PMMG_prilen with a tensor metric, centralized (MMG3D_computePrilen):
    metRidTyp 0 = MMG5_lenedg33_ani, 1 = MMG5_lenedg_ani -- ParMmg's own output
    call PMMG_prilen(parmesh,1,0) (src/libparmmg1.c:964) -- with Mmg's surface
    data (xTetra edge tags, point / xPoint normals: MMG5_lenSurfEdg*_ani,
    MMG5_buildridmet) or without (no xTetra): bit-exact against the oracle's
    restatement."""
    from helpers import cube_surface
    m = M.kuhn_cube(9)
    tags, surf, met = cube_surface(m, noise=0.08)
    met = met * 0.01                       # lengths spread over the bins
    transfer.upload_background(m, [met], 0)
    transfer.upload_point_tags(tags)
    if with_surface:
        transfer.upload_surface(surf)
    L = transfer.prilen(met_rid_typ=mrt)
    Lo = O.prilen(m, met, tags=tags, met_rid_typ=mrt, surface=surf if with_surface else None)
    assert_len_exact(L, Lo)
    assert sum(1 for h in Lo["hl"] if h) >= 4


@pytest.mark.parametrize("mrt", [0, 1])
def test_distributed_prilen_tensor_surface(transfer, mrt):
    """The distributed PMMG_computePrilen with a tensor metric on two
    partitions: the owned parallel edges by MMG5_lenSurfEdg33_ani (isedg from
    the edge's hash tag) or, with metRidTyp 1, by MMG5_lenSurfEdg_iso on the
    metric array read as isotropic (src/quality_pmmg.c:462-466, as written),
    then the tet edges along the surface; every rank's partial bit-exact
    against the oracle, and the RCCL-free fold of both equals the oracle's."""
    from helpers import cube_surface
    full = M.kuhn_cube(7)
    parts, nshared = split_partitions(full)
    rng = np.random.default_rng(8)
    for rank, (mr, glob, par) in enumerate(parts):
        tags, surf, met = cube_surface(mr, noise=0.08, seed=rank + 1)
        met = np.abs(met) * 0.01 + 1e-3    # positive everywhere: the flat read stays finite
        met[0] = 1.0
        ptag = np.where(rng.random(len(par["a"])) < 0.3, 2, 0).astype(np.uint16)
        p = dict(par, myrank=rank, owner=np.zeros(len(par["a"]), np.int32), exact_once=0, tag=ptag)
        transfer.upload_background(mr, [met], 0)
        transfer.upload_point_tags(tags)
        transfer.upload_surface(surf)
        L = transfer.prilen(met_rid_typ=mrt, par=p)
        Lo = O.prilen(mr, met, tags=tags, par=p, met_rid_typ=mrt, surface=surf)
        assert_len_exact(L, Lo)


def test_prilen_ridge_storage_needs_tags(transfer):
    """metRidTyp 1 with a tensor metric reads the point tags (ridge points):
    without them the call is refused, not computed as if there were none."""
    m, x, t, sols = cube_case(5, metric="ani", fields=False)
    transfer.upload_background(m, sols, 0)
    with pytest.raises(RuntimeError, match="point tags"):
        transfer.prilen(met_rid_typ=1)
    with pytest.raises(RuntimeError, match="point tags"):
        transfer.tetra_qual(m.ne, 1)


_PB_SCRIPT = r'''
import json, sys
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[1] + "/tests")
import numpy as np
from helpers import split_partitions
from parmmg_amd import mesh as M
from parmmg_amd.transfer import Transfer
tr = Transfer(0)
out = []
for n, metric in ((9, "graded"), (8, "ani")):
    m = M.kuhn_cube(n)
    f = M.graded_iso_metric(n) if metric == "graded" else M.shock_metric
    tr.upload_background(m, [M.on_vertices(m, f)], 0)
    out.append(tr.prilen())
full = M.kuhn_cube(6)
parts, _ = split_partitions(full)
for rank, (mr, glob, par) in enumerate(parts):
    p = dict(par, myrank=rank, owner=np.zeros(len(par["a"]), np.int32), exact_once=1)
    tr.upload_background(mr, [M.on_vertices(mr, M.graded_iso_metric(6))], 0)
    out.append(tr.prilen(par={k: (v.tolist() if hasattr(v, "tolist") else v) for k, v in p.items()}))
print(json.dumps(out))
'''


def test_prilen_edge_buckets_equal_oracle():
    """The edge-bucket variant of PMMG_prilen (PMX_PRILEN_BUCKETS=1: unique
    edges by the buckets of their smaller endpoint instead of shell walks --
    the r04 verdict's alternative, measured in DESIGN.md section 7 r05) gives
    the oracle's statistics: iso graded and tensor metrics, and the two
    partitions of a distributed mesh (parallel edges excluded, exactly once)."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PMX_PRILEN_BUCKETS="1")
    r = subprocess.run([sys.executable, "-c", _PB_SCRIPT, root], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    got = json.loads(r.stdout.strip().splitlines()[-1])
    refs = []
    for n, metric in ((9, "graded"), (8, "ani")):
        m = M.kuhn_cube(n)
        f = M.graded_iso_metric(n) if metric == "graded" else M.shock_metric
        refs.append(O.prilen(m, M.on_vertices(m, f)))
    full = M.kuhn_cube(6)
    parts, _ = split_partitions(full)
    for rank, (mr, glob, par) in enumerate(parts):
        p = dict(par, myrank=rank, owner=np.zeros(len(par["a"]), np.int32), exact_once=1)
        refs.append(O.prilen(mr, M.on_vertices(mr, M.graded_iso_metric(6)), par=p))
    for L, Lo in zip(got, refs):
        assert_len_equal(L, Lo)
