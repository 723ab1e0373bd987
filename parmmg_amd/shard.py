"""Multi-GPU layout of the transfer path: one process per GPU, groups sharded.

ParMmg groups are interpolated independently (reference
src/interpmesh_pmmg.c:690-730), so the data path has no collective: each rank
(= one MPI rank of ParMmg, one GPU) transfers its own groups.  The only
exchange is the statistics reduction that PMMG_qualhisto / PMMG_prilen do with
MPI_Reduce and custom ops (src/quality_pmmg.c:82-144, :275-306, :664-675);
here it is an all-reduce over RCCL (``torch.distributed`` backend "nccl") of
device-resident partials -- or gloo on CPU tensors in the tests.

RCCL has no user-defined ops, so "min with location" is two reductions: MIN of
the value, then MIN of a packed (rank, group, element) key over the ranks
whose value equals the global minimum.
"""
from __future__ import annotations

import torch

KEY_MAX = (1 << 63) - 1

# layout of the device partial written by pmx_qualhisto_device (12 x 8 bytes)
QUAL_F64 = ("avg", "max", "min")
QUAL_I64 = ("iel", "ne", "good", "med", "his0", "his1", "his2", "his3", "his4")
# layout of the device partial written by pmx_prilen_device (16 x 8 bytes)
LEN_F64 = ("avlen", "lmin", "lmax")
LEN_I64 = ("kmin", "kmax", "ned", "nullEdge") + tuple(f"hl{i}" for i in range(9))


def groups_for_rank(ngrp: int, rank: int, world: int) -> list[int]:
    """Contiguous block of groups per rank (ParMmg keeps a rank's groups local)."""
    per, rem = divmod(ngrp, world)
    lo = rank * per + min(rank, rem)
    return list(range(lo, lo + per + (1 if rank < rem else 0)))


def pack_key(rank: int, grp: int, iel: int) -> int:
    return (rank << 48) | (grp << 36) | iel


def unpack_key(k: int) -> tuple[int, int, int]:
    return k >> 48, (k >> 36) & 0xFFF, k & ((1 << 36) - 1)


def _minloc(val: torch.Tensor, key: torch.Tensor, dist, op_min) -> tuple[float, int]:
    v = val.clone()
    dist.all_reduce(v, op=op_min)
    k = torch.where(val == v, key, torch.full_like(key, KEY_MAX))
    dist.all_reduce(k, op=op_min)
    return float(v.item()), int(k.item())


def reduce_qual(part: torch.Tensor, rank: int, grp: int, dist) -> dict:
    """part: float64 tensor of 12 entries laid out as QUAL_F64 + QUAL_I64
    (device or CPU).  Returns the global statistics on every rank."""
    f = part[:3].clone()
    i = part.view(torch.int64)[3:].clone()
    R = dist.ReduceOp
    sums = i[1:].clone()                      # ne, good, med, his[5]
    dist.all_reduce(sums, op=R.SUM)
    avg = f[0:1].clone()
    dist.all_reduce(avg, op=R.SUM)
    mx = f[1:2].clone()
    dist.all_reduce(mx, op=R.MAX)
    key = torch.tensor([pack_key(rank, grp, int(i[0].item()))], dtype=torch.int64, device=part.device)
    mn, k = _minloc(f[2:3], key, dist, R.MIN)
    s = sums.cpu().tolist()
    r, g, iel = unpack_key(k)
    return {"ne": s[0], "good": s[1], "med": s[2], "his": s[3:8], "avg": float(avg.item()),
            "max": float(mx.item()), "min": mn, "min_rank": r, "min_grp": g, "iel": iel}


def reduce_len(part: torch.Tensor, rank: int, dist) -> dict:
    """part: float64 tensor of 16 entries laid out as LEN_F64 + LEN_I64."""
    f = part[:3].clone()
    i = part.view(torch.int64)[3:].clone()
    R = dist.ReduceOp
    sums = i[2:].clone()                      # ned, nullEdge, hl[9]
    dist.all_reduce(sums, op=R.SUM)
    av = f[0:1].clone()
    dist.all_reduce(av, op=R.SUM)
    kmin = torch.tensor([(rank << 40) | int(i[0].item())], dtype=torch.int64, device=part.device)
    lmin, kmn = _minloc(f[1:2], kmin, dist, R.MIN)
    # lmax: MAX of value, then MIN key among the maximisers
    v = f[2:3].clone()
    dist.all_reduce(v, op=R.MAX)
    kmax = torch.tensor([(rank << 40) | int(i[1].item())], dtype=torch.int64, device=part.device)
    kk = torch.where(f[2:3] == v, kmax, torch.full_like(kmax, KEY_MAX))
    dist.all_reduce(kk, op=R.MIN)
    s = sums.cpu().tolist()
    return {"ned": s[0], "nullEdge": s[1], "hl": s[2:11], "avlen": float(av.item()),
            "lmin": lmin, "lmin_rank": kmn >> 40, "lmax": float(v.item()),
            "lmax_rank": int(kk.item()) >> 40}


def qualhisto_allreduce(tr, dist, local: int, grp: int = 0) -> dict:
    """Device partial of the uploaded group -> RCCL all-reduce."""
    dev = torch.device("cuda", local)
    part = torch.zeros(12, dtype=torch.float64, device=dev)
    tr.qualhisto_device(part.data_ptr())
    tr.synchronize()
    import time
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = reduce_qual(part, dist.get_rank(), grp, dist)
    torch.cuda.synchronize()
    res["allreduce_ms"] = (time.perf_counter() - t0) * 1e3
    return res
