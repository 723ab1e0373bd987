"""The BASELINE.json configurations on one GPU, against the oracle.

* C2 / C3 at their full benchmark sizes (the meshes bench.py builds): every
  volume point bit-exact vs the oracle's sequential run in the reference's
  own vertex order (first visit through the new tets) or a documented tie;
  every surface point bit-exact vs the oracle in device semantics;
  every surface point that differs from the reference's SEQUENTIAL run falls
  in a documented class (a containing tria, or a shadow wedge/cone acceptance
  within hausd of the returned edge/vertex).
* C4 per-GPU share: the bench's two 25M-tet groups in two contexts, steps
  overlapping on the device, each checked like C2 / C3; and two small
  non-convex groups whose fallback grid barriers run concurrently.
* C5 per-GPU share (n = 275, 124.8M tets): the statistics counts against the
  analytic Kuhn-cube counts, and the device partials of two groups reduced
  across two ranks (gloo) against the oracle on the union.
"""
import os
import socket

import numpy as np
import pytest

import bench
from helpers import bits_equal, compare_exact, compare_volume, first_visit_order, lin_field
from oracle import oracle as O
from parmmg_amd import _native as N
from parmmg_amd import mesh as M
from parmmg_amd.transfer import Transfer

pytestmark = pytest.mark.gpu


def _tria_dist_classes(m, x, idx, elem, edge, vert):
    """Distance of x[i] to the returned edge (edge >= 0) / vertex (vert >= 0)."""
    out = np.full(len(idx), np.inf)
    for j, i in enumerate(idx):
        tr = m.tria[elem[i]]
        p = x[i]
        if vert[i] >= 0:
            out[j] = np.linalg.norm(p - m.xyz[tr[vert[i]]])
        elif edge[i] >= 0:
            a, b = m.xyz[tr[(edge[i] + 1) % 3]], m.xyz[tr[(edge[i] + 2) % 3]]
            ab = b - a
            s = np.clip(np.dot(p - a, ab) / np.dot(ab, ab), 0.0, 1.0)
            out[j] = np.linalg.norm(p - (a + s * ab))
    return out


@pytest.mark.timeout(1100)
@pytest.mark.parametrize("cfg", ["C2", "C3", "C4"])
def test_full_size_parity(cfg):
    """Bench-size parity (the bench's own inputs, its new tets included, so the
    step's vertex enumeration and orphan marks run at full size).  C4 is the
    per-GPU share of the 8-GPU configuration: the bench's two 25M-tet groups
    in two contexts, their steps enqueued back to back so that they overlap on
    the device, each group checked on its own.

    The reference's sequential run is the oracle over the points in the order
    the reference's vertex loop reaches them -- first visit through the new
    tets (src/interpmesh_pmmg.c:535-544), the start tet / tria and the surface
    point flags carried along that order.

    Volume: every point bit-exact against that run or a verified tie.
    Surface (src/locate_pmmg.c:209-334,587-723, path dependent): bit-exact in
    device semantics on every surface point; against the sequential run,
    every point where the two differ is checked on BOTH sides -- each answer
    is a containing tria or a wedge/cone acceptance within hausd of its
    edge/vertex -- and where both contain the point a linear field is
    reproduced to 1e-12 by both."""
    conf = bench.CONFIGS[cfg]
    cases = [bench.build_case(conf, g) for g in range(conf.get("groups", 1))]
    trs, sols2 = [], []
    for m, x, t, sols, tv in cases:
        lin = (1.0 + 2.0 * m.xyz[:, 0] - 3.0 * m.xyz[:, 1] + 0.5 * m.xyz[:, 2])[:, None]
        sols2.append(sols + [lin])
        tr = Transfer(0)
        tr.upload_background(m, sols2[-1], 0)
        tr.upload_points(x, t, tets_mmg=tv)
        trs.append(tr)
    for tr in trs:                          # every group's step enqueued before any sync
        tr.run(record_starts=True)
    got = []
    for tr in trs:
        got.append((tr.download(), tr.starts(), tr.border(), tr.locate_stats()))
    # the reference's sequential surface semantics (PMX_RUN_SEQUENTIAL_SURFACE)
    seqr = []
    for tr in trs:
        import time
        t0 = time.perf_counter()
        tr.run(flags=N.RUN_SEQUENTIAL_SURFACE | N.RUN_SEQUENTIAL_VOLUME)
        tr.synchronize()
        dt = time.perf_counter() - t0
        sst = tr.seq_surface_stats()
        svt = tr.seq_volume_stats()
        sst.update({"vol_nseq": svt["nseq"], "vol_nreplay": svt["nreplay"]})
        seqr.append((tr.download(), tr.border(), sst, dt))
        tr.close()
    for g, ((m, x, t, sols, tv), s2, (r, starts, (edge, vert), st), (rq, (sqe, sqv), sst, sdt)) in enumerate(
            zip(cases, sols2, got, seqr)):
        o = O.Oracle(m)
        vol = np.nonzero(t == 0)[0]
        bdy = np.nonzero(t == M.TAG_BDY)[0]
        assert st["nvol"] == len(vol) and st["nbdy"] == len(bdy)
        fv = first_visit_order(tv, len(x))
        assert len(fv) == len(x)            # the bench's new mesh has no orphan point
        # the reference's sequential run, in its own order
        qo, qe, qs, _, qed, qve = o.interp(x, t, s2, imet=0, order=fv)
        c = compare_volume(o, x, t, (r.sols, r.elem, r.status), (qo, qe, qs), s2)
        print(f"\n{cfg} group {g}: {c['nvol']} volume points, {c['same']} identical elements, "
              f"{c['ties']} ties")
        assert c["same"] >= c["nvol"] - max(3, c["nvol"] // 1000)
        assert np.all(r.status[vol] == 1)
        # surface, the sequential mode: every surface point bit-exact against the
        # reference's sequential run
        compare_exact((rq.sols, rq.elem, rq.status, sqe, sqv), (qo, qe, qs, qed, qve), bdy, len(s2))
        # ... and every volume point (ties included) in the sequential volume mode
        assert np.array_equal(rq.elem[vol], qe[vol]) and np.array_equal(rq.status[vol], qs[vol])
        for a, b in zip(rq.sols, qo):
            assert bits_equal(a[vol], b[vol]).all()
        print(f"{cfg} group {g}: sequential modes: {len(bdy)} surface + {len(vol)} volume points bit-exact vs "
              f"the sequential run, {sst['nreplay']} + {sst['vol_nreplay']} replayed on the reference's state, "
              f"step {sdt * 1e3:.1f} ms")
        assert sst["nseq"] == len(bdy) and sst["vol_nseq"] == len(vol)
        # surface, device semantics (each query from the device's start tria, the
        # point flags as PMMG_precompute_nodeTrias leaves them): every surface point
        sample = bdy
        so, se, ss, _, sed, sve = o.interp(x, t, s2, imet=0, order=sample, fresh=True,
                                           start_vol=starts, start_bdy=starts)
        compare_exact((r.sols, r.elem, r.status, edge, vert), (so, se, ss, sed, sve), sample, len(s2))
        # surface, the reference's sequential run: where the answers differ, both
        # must be acceptable answers of PMMG_locatePointBdy
        diff = bdy[(r.elem[bdy] != qe[bdy]) | (edge[bdy] != qed[bdy]) | (vert[bdy] != qve[bdy])]

        def contains(el, ed, vx, stt):
            return np.array([ed[i] < 0 and vx[i] < 0 and stt[i] == 1 and o.tria_contains(int(el[i]), x[i])
                             for i in diff], bool)

        in_dev, in_ref = contains(r.elem, edge, vert, r.status), contains(qe, qed, qve, qs)
        sh_dev = _tria_dist_classes(m, x, diff, r.elem, edge, vert) <= m.hausd * (1 + 1e-12)
        sh_ref = _tria_dist_classes(m, x, diff, qe, qed, qve) <= m.hausd * (1 + 1e-12)
        print(f"{cfg} group {g}: {len(bdy)} surface points, {len(sample)} bit-exact in device semantics, "
              f"{len(diff)} differ from the sequential run (device: {int(in_dev.sum())} containing tria, "
              f"{int(sh_dev.sum())} wedge/cone within hausd; reference: {int(in_ref.sum())} / "
              f"{int(sh_ref.sum())})")
        # the interpolated metric where the answers differ:
        # relative difference device vs sequential run, by class
        rel = np.abs(r.sols[0][diff] - qo[0][diff]).max(axis=1) / np.abs(qo[0][diff]).max(axis=1)
        for name, sel in (("both containing", in_dev & in_ref), ("wedge/cone on a side", ~(in_dev & in_ref))):
            if sel.any():
                print(f"{cfg} group {g}: metric rel. difference, {name}: max {rel[sel].max():.3e}, "
                      f"median {np.median(rel[sel]):.3e} ({int(sel.sum())} points)")
        assert np.all(in_dev | sh_dev), diff[~(in_dev | sh_dev)][:10]
        assert np.all(in_ref | sh_ref), diff[~(in_ref | sh_ref)][:10]
        assert len(diff) <= 0.05 * len(bdy)
        both = diff[in_dev & in_ref]
        exact = 1.0 + 2.0 * x[both, 0] - 3.0 * x[both, 1] + 0.5 * x[both, 2]
        li = len(s2) - 1
        assert np.abs(r.sols[li][both, 0] - exact).max(initial=0.0) < 1e-12
        assert np.abs(qo[li][both, 0] - exact).max(initial=0.0) < 1e-12
        del o


def l_shaped(n, cut=(0.5, 0.5, 0.5)):
    m = M.kuhn_cube(n)
    c = m.centroids()
    keep = ~np.all(c > np.array(cut), axis=1)
    tet = np.concatenate([m.tet[:1], m.tet[1:][keep]])
    return M.from_tets(m.xyz, tet)


def test_c4_two_groups_concurrent_fallbacks():
    """C4's per-GPU share is two groups in two contexts on one GPU.  With the
    walk capped at one step and non-convex groups, both contexts' fallbacks
    (tie BFS, exhaustive scan, closest -- phases behind grid barriers) run at
    the same time; each group must still match the oracle."""
    rng = np.random.default_rng(17)
    cases = []
    for n, cut in ((8, (0.5, 0.5, 0.5)), (9, (0.4, 0.6, 0.3))):
        m = l_shaped(n, cut)
        x = rng.uniform(-0.05, 1.05, size=(2500, 3))
        t = np.zeros(len(x), np.uint16)
        sols = [M.on_vertices(m, M.shock_metric), M.on_vertices(m, lin_field)]
        cases.append((m, x, t, sols))
    trs = [Transfer(0), Transfer(0)]
    for tr, (m, x, t, sols) in zip(trs, cases):
        tr.upload_background(m, sols, 0)
        tr.upload_points(x, t)
    for _ in range(3):
        for tr in trs:                  # both steps enqueued before any sync
            tr.run(max_walk=1)
        res = [tr.download() for tr in trs]
        for r, (m, x, t, sols) in zip(res, cases):
            o = O.Oracle(m)
            outs, elem, st, *_ = o.interp(x, t, sols, imet=0)
            assert (r.status == -1).sum() > 500 and (r.status == 0).sum() > 50
            compare_volume(o, x, t, (r.sols, r.elem, r.status), (outs, elem, st), sols)
            closest = np.nonzero(st == 0)[0]
            assert np.array_equal(r.elem[closest], elem[closest])
    for tr in trs:
        tr.close()


def kuhn_edges(n):
    """Unique edges of the Kuhn cube: axis edges, one diagonal per square
    face, one body diagonal per cube."""
    return 3 * n * (n + 1) ** 2 + 3 * n * n * (n + 1) + n ** 3


@pytest.mark.timeout(900)
def test_c5_share_stats_counts():
    """C5's per-GPU share (1B tets over 8 GPUs, Kuhn n = 275 = 124.8M tets):
    counts exact against the analytic Kuhn-cube counts, and every statistic
    against the oracle's sequential restatement on the same mesh
    (tests/golden/c5share_stats.json, tools/make_c5_golden.py: MMG3D_tetraQual
    + computeInqua, MMG3D_computePrilen with its edge hash): the 5-bin
    histogram, good / med, min / max and the element of the min, and -- for
    the iso metric and a graded one that fills all nine bins -- ned, the
    length histogram, lmin / lmax and their endpoints.  Sums within 1e-12;
    the bins and extrema exact (r06: the device restates glibc's log1p; until
    r05 ocml's differed in the last ulp now and then)."""
    import json
    gold = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                       "c5share_stats.json")))
    n = 275
    m = M.kuhn_cube(n)
    assert (m.ne, m.np) == (gold["ne"], gold["np"])
    tr = Transfer(0)
    tr.upload_background(m, [M.on_vertices(m, M.iso_metric)], 0)
    q = tr.qualhisto()
    assert q["ne"] == 6 * n ** 3 and sum(q["his"]) == q["ne"]
    assert 0 < q["min"] <= q["max"] <= 1.0 + 1e-12
    g = gold["qualhisto"]
    for f in ("ne", "good", "med", "his", "min", "max", "iel"):
        assert q[f] == g[f], (f, q[f], g[f])
    assert abs(q["avg"] - g["avg"]) <= 1e-12 * g["avg"]
    L = tr.prilen()
    assert L["ned"] + L["nullEdge"] == kuhn_edges(n)
    assert sum(L["hl"]) == L["ned"]
    # deterministic: the same partials and the same fixed-order reduction
    for _ in range(3):
        assert tr.prilen() == L and tr.qualhisto() == q

    def same_len(L, g):
        assert (L["ned"], L["nullEdge"]) == (g["ned"], g["nullEdge"])
        assert L["hl"] == g["hl"], (L["hl"], g["hl"])   # glibc's log1p restated on the device (r06)
        assert abs(L["avlen"] - g["avlen"]) <= 1e-12 * g["avlen"]
        for e in ("lmin", "lmax"):
            assert L[e] == g[e], (e, L[e], g[e])
        if L["lmin"] == g["lmin"]:
            assert (L["amin"], L["bmin"]) == (g["amin"], g["bmin"])
        if L["lmax"] == g["lmax"]:
            assert (L["amax"], L["bmax"]) == (g["amax"], g["bmax"])
    same_len(L, gold["prilen_iso"])
    tr.upload_background(m, [M.on_vertices(m, M.graded_iso_metric(n))], 0)
    same_len(tr.prilen(), gold["prilen_graded"])
    tr.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _stats_rank(rank, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    from parmmg_amd import mesh as Mm
    from parmmg_amd import shard
    from parmmg_amd.transfer import Transfer as T
    dist.init_process_group("gloo", rank=rank, world_size=2)
    m = Mm.kuhn_cube(6 + 3 * rank, seed=300 + rank)
    met = Mm.on_vertices(m, Mm.iso_metric)
    tr = T(0)
    tr.upload_background(m, [met], 0)
    dq = torch.zeros(shard.QUAL_WORDS, dtype=torch.float64, device="cuda:0")
    dl = torch.zeros(shard.LEN_WORDS, dtype=torch.float64, device="cuda:0")
    tr.qualhisto_device(dq.data_ptr())
    tr.prilen_device(dl.data_ptr())
    tr.synchronize()
    rq = shard.reduce_qual(dq.cpu().reshape(1, -1), dist)
    rl = shard.reduce_len(dl.cpu(), dist)
    tr.close()
    q.put((rank, rq, rl))
    dist.destroy_process_group()


def test_c5_device_partials_reduced_across_two_ranks():
    """Two ranks (one GPU, gloo on CPU tensors) reduce their groups' device
    partials; the result equals the oracle's statistics of the union."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_stats_rank, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = sorted([q.get(timeout=300) for _ in ps], key=lambda e: e[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, rq0, rl0), (_, rq1, rl1) = out
    assert rq0 == rq1 and rl0 == rl1
    qs, ls = [], []
    for rank in range(2):
        m = M.kuhn_cube(6 + 3 * rank, seed=300 + rank)
        met = M.on_vertices(m, M.iso_metric)
        qo = O.tetra_qual(m)
        qs.append(O.qualhisto(m, qo))
        ls.append(O.prilen(m, met))
    assert rq0["ne"] == qs[0]["ne"] + qs[1]["ne"]
    assert rq0["his"] == [a + b for a, b in zip(qs[0]["his"], qs[1]["his"])]
    assert rq0["good"] == qs[0]["good"] + qs[1]["good"] and rq0["med"] == qs[0]["med"] + qs[1]["med"]
    assert rq0["max"] == max(qs[0]["max"], qs[1]["max"])
    w = 0 if qs[0]["min"] <= qs[1]["min"] else 1
    assert rq0["min"] == qs[w]["min"] and rq0["cpu"] == w and rq0["iel"] == qs[w]["iel"]
    assert abs(rq0["avg"] - (qs[0]["avg"] + qs[1]["avg"])) <= 1e-12 * abs(rq0["avg"])
    assert rl0["ned"] == ls[0]["ned"] + ls[1]["ned"]
    assert rl0["hl"] == [b + c for b, c in zip(ls[0]["hl"], ls[1]["hl"])]
    assert rl0["lmin"] == min(ls[0]["lmin"], ls[1]["lmin"])
    assert rl0["lmax"] == max(ls[0]["lmax"], ls[1]["lmax"])
