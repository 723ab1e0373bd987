"""world_size-2 gloo test of the multi-GPU statistics reduction (CPU tensors).

On the GPU the same code all-reduces device partials over RCCL; here each rank
feeds a partial computed by the oracle for its own group.
"""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from parmmg_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def qual_part(st):
    a = np.zeros(12, np.float64)
    a[:3] = [st["avg"], st["max"], st["min"]]
    a.view(np.int64)[3:] = [st["iel"], st["ne"], st["good"], st["med"], *st["his"]]
    return torch.from_numpy(a)


def len_part(st, kmin, kmax):
    a = np.zeros(16, np.float64)
    a[:3] = [st["avlen"], st["lmin"], st["lmax"]]
    a.view(np.int64)[3:] = [kmin, kmax, st["ned"], st["nullEdge"], *st["hl"]]
    return torch.from_numpy(a)


def _worker(rank, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import oracle as O
    from parmmg_amd import mesh as M
    m = M.kuhn_cube(4 + rank, seed=100 + rank)
    met = M.on_vertices(m, M.iso_metric)
    qo = O.tetra_qual(m)
    st = O.qualhisto(m, qo)
    res = shard.reduce_qual(qual_part(st), rank, 0, dist)
    ls = O.prilen(m, met)
    lres = shard.reduce_len(len_part(ls, 7 + rank, 9 + rank), rank, dist)
    q.put((rank, st, res, ls, lres))
    dist.destroy_process_group()


def test_allreduce_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort(key=lambda r: r[0])
    (_, s0, r0, l0, lr0), (_, s1, r1, l1, lr1) = out
    assert r0 == r1 and lr0 == lr1             # all-reduce: every rank has the result
    assert r0["ne"] == s0["ne"] + s1["ne"]
    assert r0["his"] == [a + b for a, b in zip(s0["his"], s1["his"])]
    assert r0["max"] == max(s0["max"], s1["max"])
    wmin = 0 if s0["min"] <= s1["min"] else 1
    assert r0["min"] == min(s0["min"], s1["min"]) and r0["min_rank"] == wmin
    assert r0["iel"] == (s0, s1)[wmin]["iel"]
    assert abs(r0["avg"] - (s0["avg"] + s1["avg"])) <= 1e-12 * abs(r0["avg"])
    assert lr0["ned"] == l0["ned"] + l1["ned"]
    assert lr0["hl"] == [a + b for a, b in zip(l0["hl"], l1["hl"])]
    assert lr0["lmin"] == min(l0["lmin"], l1["lmin"])
    assert lr0["lmax"] == max(l0["lmax"], l1["lmax"])


def test_groups_for_rank_partition():
    for ngrp in (1, 5, 16):
        for world in (1, 2, 3, 8):
            got = sum((shard.groups_for_rank(ngrp, r, world) for r in range(world)), [])
            assert got == list(range(ngrp))
