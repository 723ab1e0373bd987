"""Multi-GPU layout of the transfer path: one process per GPU, groups sharded.

ParMmg groups are interpolated independently (reference
src/interpmesh_pmmg.c:690-730), so the data path has no collective: each rank
(= one MPI rank of ParMmg, one GPU) transfers its own groups.  The only
exchange is the statistics reduction that PMMG_qualhisto / PMMG_prilen do with
MPI_Reduce and custom operators (src/quality_pmmg.c:82-144, :265-307,
:661-676).  RCCL has no user-defined operators, so the reduction is ONE
all-gather of the per-rank partial records (a few hundred bytes) followed by
the reference's operators folded in rank order by the library's host folds
(pmx_qual_fold / pmx_len_fold, the same code the C ABI's RCCL path runs):
deterministic, ties to the lowest rank, the prilen operator's quirk kept.
Here the all-gather is ``torch.distributed`` (backend "nccl" = RCCL on device
tensors, or gloo on CPU tensors in the tests); C callers use
pmx_qualhisto_allreduce / pmx_prilen_allreduce on an ncclComm_t directly.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _native as N

QUAL_WORDS = C.sizeof(N.QualPart) // 8     # 15
LEN_WORDS = C.sizeof(N.LenPart) // 8       # 18


def groups_for_rank(ngrp: int, rank: int, world: int) -> list[int]:
    """Contiguous block of groups per rank (ParMmg keeps a rank's groups local)."""
    per, rem = divmod(ngrp, world)
    lo = rank * per + min(rank, rem)
    return list(range(lo, lo + per + (1 if rank < rem else 0)))


def _gather(part: torch.Tensor, dist) -> np.ndarray:
    """All-gather of one float64 record per rank -> (world, words) host array."""
    world = dist.get_world_size()
    out = [torch.empty_like(part) for _ in range(world)]
    dist.all_gather(out, part.contiguous())
    return torch.stack(out).cpu().numpy().astype(np.float64, copy=False)


def _qdict(st) -> dict:
    d = {f: getattr(st, f) for f, _ in N.QualStats._fields_}
    d["his"] = list(st.his)
    return d


def _ldict(st) -> dict:
    d = {f: getattr(st, f) for f, _ in N.LenStats._fields_}
    d["hl"] = list(st.hl)
    return d


def fold_qual(parts: np.ndarray, ranks=None) -> dict:
    """parts: (n, 15) float64 words of pmx_qual_part records (groups of a rank
    consecutive, ranks nondecreasing in ``ranks``; None = one record per rank)."""
    a = np.ascontiguousarray(parts, np.float64).reshape(-1, QUAL_WORDS)
    r = None if ranks is None else np.ascontiguousarray(ranks, np.int32)
    st = N.QualStats()
    lib = N.load()
    if not lib.pmx_qual_fold(a.ctypes.data_as(C.POINTER(N.QualPart)),
                             r.ctypes.data_as(N.iptr) if r is not None else None, a.shape[0],
                             C.byref(st)):
        raise RuntimeError("pmx_qual_fold failed")
    return _qdict(st)


def fold_len(parts: np.ndarray) -> dict:
    """parts: (nranks, 18) float64 words of pmx_len_part records, rank order."""
    a = np.ascontiguousarray(parts, np.float64).reshape(-1, LEN_WORDS)
    st = N.LenStats()
    if not N.load().pmx_len_fold(a.ctypes.data_as(C.POINTER(N.LenPart)), a.shape[0], C.byref(st)):
        raise RuntimeError("pmx_len_fold failed")
    return _ldict(st)


def merge_groups(parts: np.ndarray) -> np.ndarray:
    """The rank's group partials merged into one record (PMMG_qualhisto's group
    loop, :216-261), iel_grp = the group of the minimum."""
    d = fold_qual(parts, np.zeros(len(parts), np.int32))
    rec = N.QualPart()
    for f, _ in N.QualPart._fields_:
        if f == "his":
            for i in range(5):
                rec.his[i] = d["his"][i]
        elif f == "iel_grp":
            rec.iel_grp = d["iel_grp"]
        else:
            setattr(rec, f, d[f])
    return np.frombuffer(bytes(rec), np.float64).copy()


def reduce_qual(group_parts, dist) -> dict:
    """group_parts: (ngrp, 15) records of this rank's groups (torch tensor on
    the device or the CPU, or numpy).  Returns the global statistics on every
    rank: PMMG_qualhisto's reduction (cpu = the rank of the minimum)."""
    p = group_parts.detach().cpu().numpy() if isinstance(group_parts, torch.Tensor) else group_parts
    mine = torch.from_numpy(merge_groups(np.asarray(p, np.float64).reshape(-1, QUAL_WORDS)))
    dev = group_parts.device if isinstance(group_parts, torch.Tensor) else torch.device("cpu")
    if dist.get_backend() == "nccl":
        mine = mine.to(dev)
    return fold_qual(_gather(mine, dist))


def reduce_len(part, dist) -> dict:
    """part: this rank's pmx_len_part record (one group per rank, as
    PMMG_prilen requires, :623-627)."""
    t = part if isinstance(part, torch.Tensor) else torch.from_numpy(np.asarray(part, np.float64))
    return fold_len(_gather(t.reshape(-1), dist))


def qualhisto_allreduce(tr, dist, local: int) -> dict:
    """Device partial of the uploaded group -> all-gather over the process group."""
    import time
    dev = torch.device("cuda", local)
    part = torch.zeros(QUAL_WORDS, dtype=torch.float64, device=dev)
    tr.qualhisto_device(part.data_ptr())
    tr.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = reduce_qual(part.reshape(1, -1), dist)
    torch.cuda.synchronize()
    res["allreduce_ms"] = (time.perf_counter() - t0) * 1e3
    return res


def binding_collectives(trs, dist, rank: int, world: int, local: int) -> dict:
    """The statistics reduction exactly as the ParMmg binding links it
    (integration/pmmg_pmx.c: PMMG_qualhisto / PMMG_prilen over
    pmx_qualhisto_allreduce / pmx_prilen_allreduce, reference
    src/quality_pmmg.c:275-306,629-678): an RCCL communicator of the C ABI
    (pmx_comm_unique_id on rank 0, the id broadcast over the torch process
    group as the binding broadcasts it over MPI, pmx_comm_init on every rank),
    this rank's group partials (PMMG_qualhisto OUTQUA over all groups,
    PMMG_prilen(parmesh,1,0) on group 0) all-gathered on the device and folded
    in rank order.  Every rank checks its result against the rank-ordered fold
    of the same partials gathered over the torch process group."""
    import time
    from .transfer import Transfer, comm_unique_id
    obj = [comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    tr0 = trs[0]
    comm = tr0.comm_init(world, obj[0], rank)
    dev = torch.device("cuda", local)
    ngrp = len(trs)
    qp = torch.zeros((ngrp, QUAL_WORDS), dtype=torch.float64, device=dev)
    lp = torch.zeros(LEN_WORDS, dtype=torch.float64, device=dev)
    for g, tr in enumerate(trs):
        tr.qualhisto_device(qp[g].data_ptr(), opt=N.OUTQUA)
    tr0.prilen_device(lp.data_ptr(), met_rid_typ=1)
    for tr in trs:
        tr.synchronize()
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    q = tr0.qualhisto_allreduce(comm, world, qp.data_ptr(), ngrp)
    ln = tr0.prilen_allreduce(comm, world, lp.data_ptr())
    ms = (time.perf_counter() - t0) * 1e3
    Transfer.comm_destroy(comm)
    # the check: the same partials over the torch process group, folded here
    allq = [None] * world
    alll = [None] * world
    dist.all_gather_object(allq, qp.cpu().numpy())
    dist.all_gather_object(alll, lp.cpu().numpy())
    ref_q = fold_qual(np.concatenate(allq), np.repeat(np.arange(world, dtype=np.int32), ngrp))
    ref_l = fold_len(np.stack(alll))
    for k, v in ref_q.items():
        if q[k] != v:
            raise AssertionError(f"rank {rank}: pmx_qualhisto_allreduce {k} = {q[k]}, fold = {v}")
    for k, v in ref_l.items():
        if ln[k] != v:
            raise AssertionError(f"rank {rank}: pmx_prilen_allreduce {k} = {ln[k]}, fold = {v}")
    return {"path": "C ABI RCCL (pmx_comm_init, pmx_qualhisto_allreduce, pmx_prilen_allreduce)",
            "ranks_checked": world, "allreduce_ms": ms, "qualhisto": q, "prilen": ln}
