"""The statistics reduction across ranks (CPU: the host folds, world_size-2 gloo).

PMMG_qualhisto / PMMG_prilen reduce per-rank partials with MPI_Reduce and
custom operators (reference src/quality_pmmg.c:82-144, :265-307, :661-676).
The library replaces them with one all-gather of the partial records and the
reference's operators folded in rank order (pmx_qual_fold / pmx_len_fold);
on the GPU the all-gather is RCCL, here gloo on CPU tensors.  The partials
fed here come from the oracle (no GPU): two ParMmg partitions of one Kuhn
cube sharing an interface, so that node de-duplication (PMMG_count_nodes_par,
:33-80, 196-209) and parallel-edge ownership (:398-502) are exercised.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from parmmg_amd import _native as N
from parmmg_amd import shard

N_CUBE = 6


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def qual_record(st, np_, iel_grp=0):
    rec = N.QualPart()
    rec.avg, rec.max, rec.min = st["avg"], st["max"], st["min"]
    rec.iel, rec.ne, rec.np, rec.good, rec.med, rec.nrid = (st["iel"], st["ne"], np_, st["good"],
                                                            st["med"], st.get("nrid", 0))
    for i in range(5):
        rec.his[i] = st["his"][i]
    rec.iel_grp = iel_grp
    return np.frombuffer(bytes(rec), np.float64).copy()


def len_record(st):
    rec = N.LenPart()
    for f in ("avlen", "lmin", "lmax", "amin", "bmin", "amax", "bmax", "ned", "nullEdge"):
        setattr(rec, f, st[f])
    for i in range(9):
        rec.hl[i] = st["hl"][i]
    return np.frombuffer(bytes(rec), np.float64).copy()


def test_qual_fold_groups_then_ranks():
    """Groups of a rank as PMMG_qualhisto's loop (sums, strict min: first group
    on ties), then ranks with the min_iel operator (lowest rank on ties)."""
    def part(ne, mn, iel, mx, np_=10):
        return qual_record({"avg": 0.5 * ne, "max": mx, "min": mn, "iel": iel, "ne": ne, "good": ne,
                            "med": 1, "his": [0, 0, ne, 0, 0]}, np_)
    parts = np.stack([part(5, 0.3, 7, 0.9), part(6, 0.2, 3, 0.8),       # rank 0: groups 0, 1
                      part(4, 0.2, 9, 0.95),                            # rank 1: tie on min
                      part(3, 0.25, 1, 0.7), part(2, 0.1, 4, 0.6)])    # rank 2
    r = shard.fold_qual(parts, np.array([0, 0, 1, 2, 2], np.int32))
    assert r["ne"] == 20 and r["np"] == 50 and r["his"] == [0, 0, 20, 0, 0]
    assert r["max"] == 0.95 and r["min"] == 0.1
    assert (r["cpu"], r["iel_grp"], r["iel"]) == (2, 1, 4)
    r = shard.fold_qual(parts[:3], np.array([0, 0, 1], np.int32))
    assert (r["min"], r["cpu"], r["iel_grp"], r["iel"]) == (0.2, 0, 1, 3)   # tie: lowest rank
    m = shard.merge_groups(parts[3:])
    r = shard.fold_qual(np.stack([shard.merge_groups(parts[:2]), parts[2], m]))
    assert (r["min"], r["cpu"], r["iel_grp"], r["iel"]) == (0.1, 2, 1, 4)


def test_len_fold_reference_operator_quirk():
    """PMMG_compute_lenStats (:125-141): a strictly smaller lmin also takes the
    other rank's amax/bmax; ties keep the first (lowest) rank."""
    def part(lmin, a, lmax, A, ned):
        return len_record({"avlen": 1.0 * ned, "lmin": lmin, "lmax": lmax, "amin": a, "bmin": a + 1,
                           "amax": A, "bmax": A + 1, "ned": ned, "nullEdge": 1, "hl": [ned] + [0] * 8})
    r = shard.fold_len(np.stack([part(0.5, 10, 3.0, 20, 4), part(0.2, 30, 2.0, 40, 5)]))
    assert (r["lmin"], r["amin"], r["bmin"], r["cpu_min"]) == (0.2, 30, 31, 1)
    assert (r["lmax"], r["cpu_max"]) == (3.0, 0)
    assert (r["amax"], r["bmax"]) == (40, 41)          # the quirk: rank 1's amax/bmax
    assert r["ned"] == 9 and r["nullEdge"] == 2 and r["hl"][0] == 9
    r = shard.fold_len(np.stack([part(0.2, 10, 3.0, 20, 4), part(0.2, 30, 3.0, 40, 5)]))
    assert (r["amin"], r["cpu_min"], r["amax"], r["cpu_max"]) == (10, 0, 20, 0)


def _rank_partials(rank):
    """Oracle partials of partition `rank` of the split cube."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "tests"))
    from helpers import split_partitions
    from oracle import oracle as O
    from parmmg_amd import mesh as M
    parts, nshared = split_partitions(M.kuhn_cube(N_CUBE))
    mr, glob, par = parts[rank]
    met = M.on_vertices(mr, M.iso_metric)
    # interface nodes: the endpoints of the parallel edges, one int-comm slot
    # each; counted by the highest rank sharing them (:196-209)
    iface = np.unique(np.concatenate([par["a"], par["b"]]))
    idx_comm = np.arange(len(iface), dtype=np.int32)
    intvalues = np.zeros(len(iface), np.int32)
    if rank == 0:
        intvalues[:] = 1                     # shared with rank 1 > 0: rank 1 counts them
    np_ = O.count_nodes(mr, iface, idx_comm, intvalues)
    q = O.qualhisto(mr, O.tetra_qual(mr))
    lens = {once: O.prilen(mr, met, par=dict(par, exact_once=once)) for once in (0, 1)}
    return qual_record(q, np_), {k: len_record(v) for k, v in lens.items()}, nshared, q, lens


def _worker(rank, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    qrec, lrecs, nshared, qst, lst = _rank_partials(rank)
    rq = shard.reduce_qual(torch.from_numpy(qrec).reshape(1, -1), dist)
    rl = {once: shard.reduce_len(torch.from_numpy(lrecs[once]), dist) for once in (0, 1)}
    q.put((rank, rq, rl, nshared, qst, lst))
    dist.destroy_process_group()


def test_allreduce_two_partitions_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = sorted([q.get(timeout=180) for _ in ps], key=lambda e: e[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, rq0, rl0, nsh, q0, l0), (_, rq1, rl1, _, q1, l1) = out
    assert rq0 == rq1 and rl0 == rl1             # all-reduce: every rank has the result
    n = N_CUBE
    assert rq0["ne"] == 6 * n ** 3 and rq0["np"] == (n + 1) ** 3   # interface nodes counted once
    assert rq0["his"] == [a + b for a, b in zip(q0["his"], q1["his"])]
    w = 0 if q0["min"] <= q1["min"] else 1
    assert rq0["min"] == min(q0["min"], q1["min"]) and rq0["cpu"] == w
    assert rq0["iel"] == (q0, q1)[w]["iel"]
    edges = 3 * n * (n + 1) ** 2 + 3 * n * n * (n + 1) + n ** 3
    # exactly once: every edge of the cube once; the reference's semantics
    # count the parallel edges on both ranks (its warning, :585-586)
    assert rl0[1]["ned"] + rl0[1]["nullEdge"] == edges
    assert rl0[0]["ned"] + rl0[0]["nullEdge"] == edges + nsh
    assert rl0[0]["lmin"] == min(l0[0]["lmin"], l1[0]["lmin"])
    assert rl0[0]["lmax"] == max(l0[0]["lmax"], l1[0]["lmax"])


def test_groups_for_rank_partition():
    for ngrp in (1, 5, 16):
        for world in (1, 2, 3, 8):
            got = sum((shard.groups_for_rank(ngrp, r, world) for r in range(world)), [])
            assert got == list(range(ngrp))
