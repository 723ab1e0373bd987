#!/usr/bin/env python3
"""Benchmark of the MI355X transfer path (locate + interpolate new vertices).

A step = one ParMmg iteration's PMMG_interpMetricsAndFields pass of one
background group on one GPU: every device pass of that iteration on the
uploaded raw arrays (PMX_RUN_FRESH_BACKGROUND, r06).  Per background: the
fixed-point grid coordinates of its vertices, the tria normals
(PMMG_precompute_triaNormals), the node -> trias fans with the upload's fan
check (PMMG_precompute_nodeTrias), and whatever layout the upload derived on
the device (none by default: the walk reads the 32-B tet records, the hint
sample is packed by the host with them; the device face matching when the
background came without Mmg's adjacency).  Per new mesh: the orphan marks
from the new tets (the reference's vertex loop over the new tets), the tag
dispatch and compaction of the new points.  Then the hint-grid build, the
adjacency-walk location of every new vertex (volume + surface), the fused
metric / field interpolation and the exhaustive fallback.  Inputs (the raw
background arrays -- tet records {v, adja}, vertices, solutions, boundary
trias -- and the new points and tets) are resident in HBM, uploaded before
the timed region; the host-staged (PCIe-inclusive) cycles are measured after
it and reported apart.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2|C3|C4]

The default workload is C3 (100M tets, metric + level set + velocity, the
north-star configuration of BASELINE.json, one GPU).

N > 1: launched by torch.distributed.run, one rank per GPU; every rank owns its
own group (ParMmg groups shard with no data-path collective: weak scaling);
RCCL all-reduces the quality histogram once after the timed loop.
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# SURVEY.md section 8 configurations (Kuhn cube with n cells per axis)
CONFIGS = {
    "C1": dict(n=20, metric="iso", fields=["ls"], desc="unit cube ~48k tets, iso metric + LS"),
    "C2": dict(n=119, metric="ani", fields=[], desc="10M-tet cube, anisotropic shock metric"),
    "C3": dict(n=255, metric="iso", fields=["ls", "vel"], desc="100M-tet cube, iso metric + LS + velocity"),
    # 400M tets = 16 ParMmg groups of ~25M (the group size cap,
    # src/parmmg.h:209) over 8 GPUs: 2 groups of 25M tets per GPU
    "C4": dict(n=161, groups=2, metric="iso", fields=["ls", "vel"],
               desc="per-GPU share of 400M tets over 8 GPUs (2 groups of 25M)"),
}
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)


def build_case(cfg: dict, rank: int):
    from parmmg_amd import mesh as M
    n = cfg["n"]
    m = M.kuhn_cube(n, seed=20250117 + rank)
    x, t = M.new_points(n, seed=12345 + rank)
    # the new mesh's tets over those points: the step enumerates the vertices
    # through them, as the reference's vertex loop does (orphan marks)
    tv = M.new_point_tets(n, x, t)
    sols = []
    if cfg["metric"] == "ani":
        sols.append(M.on_vertices(m, M.shock_metric))
    else:
        sols.append(M.on_vertices(m, M.iso_metric))
    if "ls" in cfg["fields"]:
        sols.append(M.on_vertices(m, M.level_set))
    if "vel" in cfg["fields"]:
        sols.append(M.on_vertices(m, M.velocity))
    return m, x, t, sols, tv


def alg_bytes(N: int, ne: int, np_: int, S: int) -> int:
    """compulsory bytes of locate+interp for one step."""
    return N * (24 + 8 * S + 4) + ne * 32 + np_ * (24 + 8 * S)


def profiled_traffic(config: str, kernel: str = "k_walks"):
    """HBM bytes per launch of the dominant kernel from the newest committed
    rocprofv3 PMC summary of this config (tools/profile.sh ->
    tools/prof_summary.py -> profiles/rNN_<config>_<tag>.json): 2*FETCH_SIZE +
    WRITE_SIZE per MI355X_MICROARCH.md section HBM.  None if not profiled."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{config.lower()}_*.json")))
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        for k, e in d.get("kernels", {}).items():
            if k.split("<")[0] == kernel and e.get("traffic"):
                return e["traffic"], os.path.relpath(f, ROOT)
    return None, None


_CPU_CASE = {}


def _cpu_rank(r: int):
    """One CPU 'rank' of the node baseline (forked child, no GPU state)."""
    m, x, t, sols, budget = _CPU_CASE["case"]
    res = cpu_baseline(m, x, t, sols, budget_s=budget)
    return res["value"], res["sample"]


def _physical_cores() -> int | None:
    """Physical cores of the machine (lscpu's CORE,SOCKET pairs), or None."""
    import subprocess
    try:
        out = subprocess.run(["lscpu", "-p=CORE,SOCKET"], capture_output=True, text=True, timeout=10).stdout
    except (OSError, subprocess.SubprocessError):
        return None
    pairs = {ln.strip() for ln in out.splitlines() if ln and not ln.startswith("#")}
    return len(pairs) or None


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_share() -> tuple[int, list[int]]:
    """The CPUs this process may use: its affinity set, capped by the cgroup
    quota (cpu.max "quota period"; a GPU box of this pool: 16 of 256)."""
    try:
        cpus = sorted(os.sched_getaffinity(0))
    except AttributeError:
        cpus = list(range(os.cpu_count() or 1))
    k = len(cpus)
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            k = min(k, max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return k, cpus


def mem_budget() -> float:
    """Bytes the CPU baseline may allocate: 75 % of min(MemAvailable, the
    cgroup's memory.max minus its current use)."""
    avail = None
    try:
        for line in open("/proc/meminfo"):
            if line.startswith("MemAvailable:"):
                avail = int(line.split()[1]) * 1024
    except OSError:
        pass
    try:
        mx = open("/sys/fs/cgroup/memory.max").read().strip()
        cur = int(open("/sys/fs/cgroup/memory.current").read().strip())
        if mx != "max":
            room = int(mx) - cur
            avail = room if avail is None else min(avail, room)
    except (OSError, ValueError):
        pass
    return 0.75 * (avail if avail is not None else 64e9)


def _cpu_rank_pinned(args):
    """A forked child pinned to one core of the share, then one oracle 'rank'."""
    r, core = args
    os.sched_setaffinity(0, {core})
    return _cpu_rank(r)


def cpu_baseline_node(m, x, t, sols, budget_s: float = 20.0) -> dict:
    """K concurrent single-core oracle processes on the same workload, the
    ParMmg model of one MPI rank per core: each measures its
    own step rate while the others run (shared memory bandwidth included);
    the node rate is their sum.  Forked BEFORE any GPU initialisation.  K =
    the process's CPU share (affinity and cgroup quota), each child pinned to
    its own core of it (os.sched_setaffinity, the `taskset` of SURVEY.md 8(d)),
    fewer only if the oracle's per-process memory (faceAreas & co., ~110 B
    per tet, the reference's own PMMG_precompute_faceAreas footprint) would not
    fit the memory left (MemAvailable, cgroup memory.max)."""
    import multiprocessing as mp
    share, cpus = cpu_share()
    # the oracle context's arrays (oracle/pmx_oracle.c orc_create: 12 face
    # normal components, volume and flag per tet; four int arrays per vertex)
    # plus its sample's outputs; the mesh itself is the parent's (copy on write)
    per_proc = max(1, m.ne * 110 + m.np * 24 + len(x) * 64)
    budget = mem_budget()
    K = max(1, min(share, len(cpus), int(budget // per_proc)))
    _CPU_CASE["case"] = (m, x, t, sols, budget_s)
    with mp.get_context("fork").Pool(K) as pool:
        res = pool.map(_cpu_rank_pinned, [(r, cpus[r % len(cpus)]) for r in range(K)])
    rates = [r[0] for r in res]
    return {"value": float(sum(rates)), "unit": "vertices/s", "cores": K, "kind": "port",
            "cpu_share": share, "pinning": f"one process per core, os.sched_setaffinity to cores "
                                           f"{cpus[:K][0]}..{cpus[:K][-1]} of the affinity set",
            "memory_bound": K < share, "mem_budget_GB": budget / 1e9, "per_process_GB": per_proc / 1e9,
            "per_core": float(np.mean(rates)), "cpu_model": _cpu_model(),
            "physical_cores": _physical_cores(),
            "sample": f"{K} concurrent processes, each: {res[0][1]}; node rate = sum of the "
                      f"{K} per-process rates (min {min(rates):.3g}, max {max(rates):.3g})"}


def cpu_baseline(m, x, t, sols, budget_s: float = 20.0) -> dict:
    """The oracle (CPU restatement of the reference, sequential carry-over
    walk, one core) on the same workload: the whole step when it fits the
    budget, else a Morton-contiguous prefix of the new points (the O(ne)
    precompute is always done in full and charged)."""
    from oracle import oracle as O
    t0 = time.perf_counter()
    o = O.Oracle(m)                       # faceAreas / triaNormals / nodeTrias
    t_pre = time.perf_counter() - t0
    n = len(x)
    S = min(n, 20000)
    t1 = time.perf_counter()
    o.interp(x[:S], t[:S], sols, imet=0)
    dt = time.perf_counter() - t1
    rate = S / max(dt, 1e-9)
    if dt * n / S + t_pre <= budget_s:
        S = n
        t1 = time.perf_counter()
        o.interp(x, t, sols, imet=0)
        dt = time.perf_counter() - t1
    else:
        S = int(min(n, max(S, rate * (budget_s - t_pre))))
        t1 = time.perf_counter()
        o.interp(x[:S], t[:S], sols, imet=0)
        dt = time.perf_counter() - t1
    t_step = t_pre + dt * n / S
    return {"value": n / t_step, "unit": "vertices/s", "cores": 1, "kind": "port",
            "sample": f"oracle/pmx_oracle.c (reference algorithm, gcc -O3, 1 thread): "
                      f"precompute over all {m.ne} tets {t_pre:.2f}s + {S}/{n} new vertices "
                      f"{dt:.2f}s, extrapolated to the full step"}


def pcie_inclusive(tr, m, x, t, sols, reps: int = 3) -> dict:
    """Wall-clock rate of the host-staged cycles of one group:
    points = upload new vertices + step + download fields/elements;
    full = also re-upload the background mesh and its solutions (SoA gather,
    device adjacency/boundary build when the mesh carries none);
    resident_cycle (added by the caller) = the iteration with the background
    kept on the device."""
    # the caller's output arrays exist before the step (ParMmg: met->m,
    # field->m), so they are allocated once, outside the window
    out = tr.download()

    def cyc(full: bool, adja: bool = True):
        best, phases = float("inf"), None
        for _ in range(reps):
            tr.synchronize()
            t0 = time.perf_counter()
            if full:
                tr.upload_background(m, sols, 0, adja=adja)
            t1 = time.perf_counter()
            tr.upload_points(x, t)
            t2 = time.perf_counter()
            tr.run()
            tr.synchronize()
            t3 = time.perf_counter()
            tr.download(into=out)
            t4 = time.perf_counter()
            if t4 - t0 < best:
                best = t4 - t0
                phases = {"background_ms": (t1 - t0) * 1e3, "points_ms": (t2 - t1) * 1e3,
                          "step_ms": (t3 - t2) * 1e3, "download_ms": (t4 - t3) * 1e3}
        return best, phases
    (tp, pp), (tf, pf), (td, pd) = cyc(False), cyc(True), cyc(True, adja=False)
    n = len(x)
    return {"unit": "vertices/s", "reps": reps, "timing": "best of reps, wall clock",
            "points_cycle": {"value": n / tp, "ms": tp * 1e3, "phases": pp},
            "full_cycle": {"value": n / tf, "ms": tf * 1e3, "phases": pf},
            # the same cycle with Mmg's adjacency left on the host: rebuilt by
            # device face matching (16 B/tet less over PCIe)
            "full_cycle_device_adjacency": {"value": n / td, "ms": td * 1e3, "phases": pd}}


def resident_cycle(m, sols, cfg: dict, local: int, iters: int = 4, warmup: int = 2) -> dict:
    """One ParMmg iteration with the background device resident (DESIGN.md §7,
    pmx_promote_background): upload the new mesh's points (+ its tets, same
    pass), step, download the fields into the caller's arrays, promote the new
    mesh + results to the next background (only its boundary trias and Mmg
    adjacency cross PCIe).  Two jittered Kuhn meshes of the config's size
    alternate as background and new mesh; wall clock per iteration."""
    from parmmg_amd import _native as N
    from parmmg_amd import mesh as M
    from parmmg_amd.transfer import Result, Transfer
    mb = M.kuhn_cube(cfg["n"], seed=777)

    def case(mm):
        x = mm.xyz[1:]
        onb = np.any((x == 0.0) | (x == 1.0), axis=1)
        t = np.where(onb, M.TAG_BDY, 0).astype(np.uint16)
        return mm, x, t, mm.tet            # Mmg layout: passed as is

    cases = [case(mb), case(m)]
    tr = Transfer(local)
    tr.set_residency(True)
    tr.upload_background(m, sols, 0)
    sizes = [s.shape[1] for s in sols]
    res = [Result([np.zeros((len(c[1]), sz)) for sz in sizes], *(np.zeros(len(c[1]), np.int32)
                                                                   for _ in range(3))) for c in cases]
    rows = []
    for it in range(warmup + iters):
        mm, x, t, tets1 = cases[it % 2]
        out = res[it % 2]
        tr.synchronize()
        t0 = time.perf_counter()
        tr.upload_points(x, t, tets_mmg=tets1)
        t1 = time.perf_counter()
        # the ParMmg seam's step: its fields always come down, so they start
        # down at once (overlapping the new tets' packing)
        tr.run(flags=N.RUN_EAGER_DOWNLOAD)
        tr.synchronize()
        t2 = time.perf_counter()
        tr.download(into=out, sols_only=True)
        t3 = time.perf_counter()
        tr.promote_background(mm, out.sols, adja=False)
        t4 = time.perf_counter()
        if it >= warmup:
            rows.append((t4 - t0, t1 - t0, t2 - t1, t3 - t2, t4 - t3, len(x)))
    tr.close()
    best = min(rows)
    mean = float(np.mean([r[0] for r in rows]))
    return {"value": best[5] / best[0], "ms": best[0] * 1e3, "mean_ms": mean * 1e3,
            "new_vertices": best[5], "new_tets": int(mb.ne),
            "phases": {"points_and_tets_ms": best[1] * 1e3, "step_ms": best[2] * 1e3,
                       "download_ms": best[3] * 1e3, "promote_ms": best[4] * 1e3},
            "timing": f"best of {iters} iterations after {warmup}, wall clock"}


from parmmg_amd.mesh import MMG_POINT, MMG_TETRA  # noqa: E402  (Mmg's AoS records)


def binding_cycle(m, x, t, tv, sols, local: int, iters: int = 3) -> dict:
    """The per-iteration device work of integration/pmmg_pmx.c at its two
    ParMmg seams, through the same C-ABI calls on Mmg-shaped AoS records
    (MMG5_Point 72 B, MMG5_Tetra 48 B, strided views): PMMG_interpMetricsAndFields
    (src/libparmmg1.c:829 -> PMX_interpMetricsAndFields_groups: new points +
    new tets up, background up with device face matching, step, fields down)
    then PMMG_tetraQual(parmesh, 1) (:845 -> pmx_new_mesh_qual_synced on the
    device-resident new mesh, qualities scattered into tetra[k].qual).
    `reupload_ms`: the r03 binding's :845 (the whole new mesh uploaded again,
    pmx_tetra_qual).  Wall clock, best of iters."""
    import ctypes as C
    from parmmg_amd import _native as N
    from parmmg_amd.transfer import Transfer
    n = len(x)
    op = np.zeros(m.np + 1, MMG_POINT)
    op["c"] = m.xyz
    ot = np.zeros(m.ne + 1, MMG_TETRA)
    ot["v"] = m.tet
    npnt = np.zeros(n + 1, MMG_POINT)
    npnt["c"][1:] = x
    npnt["tag"][1:] = t
    nt = np.zeros(tv.shape[0], MMG_TETRA)
    nt["v"] = tv
    olds = [np.ascontiguousarray(s) for s in sols]
    news = [np.full((n + 1, s.shape[1]), -7.0) for s in sols]
    tri = np.ascontiguousarray(m.tria, np.int32)
    adjt = np.ascontiguousarray(m.adjt, np.int32)

    def ptr(a, field=None, ct=C.c_double):
        base = a.ctypes.data + (a.dtype.fields[field][1] if field else 0)
        return C.cast(C.c_void_p(base), C.POINTER(ct))

    def sv(a):
        v = N.SolView()
        v.size, v.m = a.shape[1], a.ctypes.data_as(N.dptr)
        return v

    g = N.Group()
    g.mesh.np, g.mesh.ne = n, nt.shape[0] - 1
    g.mesh.point_c, g.mesh.point_stride = ptr(npnt, "c"), MMG_POINT.itemsize
    g.mesh.tetra_v, g.mesh.tetra_stride = ptr(nt, "v", C.c_int), MMG_TETRA.itemsize
    g.points.first, g.points.last = 1, n
    g.points.c, g.points.stride = ptr(npnt, "c"), MMG_POINT.itemsize
    g.points.tag, g.points.tag_stride = ptr(npnt, "tag", C.c_uint16), MMG_POINT.itemsize
    g.old_mesh.np, g.old_mesh.ne, g.old_mesh.nt = m.np, m.ne, m.nt
    g.old_mesh.point_c, g.old_mesh.point_stride = ptr(op, "c"), MMG_POINT.itemsize
    g.old_mesh.tetra_v, g.old_mesh.tetra_stride = ptr(ot, "v", C.c_int), MMG_TETRA.itemsize
    g.old_mesh.adja = None                     # the adapter's choice: device face matching
    g.old_mesh.tria_v, g.old_mesh.tria_stride = tri.ctypes.data_as(N.iptr), 12
    g.old_mesh.adjt = adjt.ctypes.data_as(N.iptr)
    g.old_mesh.hausd = m.hausd
    met, omet = sv(news[0]), sv(olds[0])
    fl = (N.SolView * max(1, len(sols) - 1))(*[sv(a) for a in news[1:]])
    ofl = (N.SolView * max(1, len(sols) - 1))(*[sv(a) for a in olds[1:]])
    g.met, g.old_met = C.pointer(met), C.pointer(omet)
    g.fields, g.old_fields = C.cast(fl, C.POINTER(N.SolView)), C.cast(ofl, C.POINTER(N.SolView))
    g.nsols = len(sols) - 1
    tr = Transfer(local)
    st = Transfer(local)                        # the adapter's statistics context
    lib = tr.lib
    ctxs = (C.c_void_p * 1)(tr.ctx)
    q = np.zeros(nt.shape[0])
    # :845 passes metRidTyp 1 (PMMG_tetraQual(parmesh,1))
    mrt = 1
    rows = []
    for it in range(iters + 1):
        t0 = time.perf_counter()
        if not lib.PMX_interpMetricsAndFields_groups(ctxs, 1, C.byref(g), None, 1):
            raise RuntimeError(lib.pmx_last_error(tr.ctx).decode())
        t1 = time.perf_counter()
        # straight into tetra[k].qual, as the binding does
        if not lib.pmx_new_mesh_qual_synced(tr.ctx, C.byref(met), N.INQUA, mrt, ptr(nt, "qual"),
                                            MMG_TETRA.itemsize, nt.shape[0], None):
            raise RuntimeError(lib.pmx_last_error(tr.ctx).decode())
        t2 = time.perf_counter()
        # the r03 binding's PMMG_tetraQual: the new mesh uploaded again
        mv = N.MeshView()
        mv.np, mv.ne = n, nt.shape[0] - 1
        mv.point_c, mv.point_stride = ptr(npnt, "c"), MMG_POINT.itemsize
        mv.tetra_v, mv.tetra_stride = ptr(nt, "v", C.c_int), MMG_TETRA.itemsize
        if not (lib.pmx_upload_background(st.ctx, C.byref(mv), 1, C.byref(met), 0) and
                lib.pmx_upload_point_tags(st.ctx, ptr(npnt, "tag", C.c_uint16), MMG_POINT.itemsize) and
                lib.pmx_tetra_qual(st.ctx, mrt, q.ctypes.data_as(N.dptr), q.shape[0])):
            raise RuntimeError(lib.pmx_last_error(st.ctx).decode())
        nt["qual"][1:] = q[1:]
        t3 = time.perf_counter()
        if it:
            rows.append((t2 - t0, t1 - t0, t2 - t1, t3 - t2))
    tr.close()
    st.close()
    best = min(rows)
    return {"value": n / best[0], "unit": "vertices/s", "ms": best[0] * 1e3,
            "phases": {"interp_ms": best[1] * 1e3, "tetra_qual_ms": best[2] * 1e3},
            "reupload_tetra_qual_ms": min(r[3] for r in rows) * 1e3,
            "timing": f"best of {iters} iterations, wall clock, Mmg-shaped AoS records "
                      f"({MMG_POINT.itemsize} / {MMG_TETRA.itemsize} B)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C3", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--no-pcie", action="store_true",
                    help="skip the host-staged (PCIe-inclusive) leg measured after the timed region")
    ap.add_argument("--no-new-tets", action="store_true",
                    help="ablation: upload the new points without the new mesh's tets (no vertex "
                         "enumeration through the tets / orphan marks in the step)")
    ap.add_argument("--numbering", default="lex", choices=["lex", "shuffle", "appended"],
                    help="background tet numbering (SURVEY.md 8(d)): lex = the generator's "
                         "cell-lexicographic order (Scotch-like), shuffle = random order (seed 7), "
                         "appended = 10%% of the tets moved to the end (Mmg insertions)")
    ap.add_argument("--no-seq", action="store_true",
                    help="skip the sequential-surface leg (PMX_RUN_SEQUENTIAL_SURFACE, measured after "
                         "the timed region)")
    ap.add_argument("--run-exp", type=int, default=0,
                    help="A/B measurement switch of the step (pmx_run flags bits 16-23, "
                         "parmmg_amd/csrc/pmx_capi.hip run_flags_valid)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="N>1 process group backend (nccl = RCCL; gloo only to rehearse "
                         "the multi-rank path, e.g. several ranks on one GPU)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        # PMX_BENCH_SAME_DEVICE=1 (rehearsal with gloo): every rank on GPU 0
        if os.environ.get("PMX_BENCH_SAME_DEVICE") == "1":
            local = 0
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    def phase(msg):
        print(f"[bench {time.strftime('%H:%M:%S')}] rank {rank}: {msg}", file=sys.stderr, flush=True)

    from parmmg_amd import build
    phase("build (libraries rebuilt only when stale)")
    build.build_meshgen()
    build.build_transfer()
    if rank == 0 and not args.no_cpu:
        build.build_oracle()

    cfg = CONFIGS[args.config]
    ngrp = cfg.get("groups", 1)
    phase(f"build_case {args.config}")
    cases = [build_case(cfg, rank * ngrp + g) for g in range(ngrp)]
    phase(f"{args.config} case built")
    if args.numbering != "lex":
        from parmmg_amd import mesh as M
        phase(f"numbering {args.numbering}")
        cases = [(M.numbering(c[0], args.numbering)[0],) + tuple(c[1:]) for c in cases]
        phase(f"{args.numbering} numbering done")
    # the CPU baseline first: its worker processes are forked before this
    # process touches the GPU
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        m, x, t, sols, _ = cases[0]
        phase("cpu baseline (forked oracle processes)")
        cpu = cpu_baseline_node(m, x, t, sols)
        phase("cpu baseline done")

    from parmmg_amd import _native as N
    from parmmg_amd import mesh as M
    from parmmg_amd.transfer import Transfer
    FRESH = N.RUN_FRESH_BACKGROUND | (args.run_exp << 16)
    # every group of this rank in its own context (own stream): the groups'
    # steps are enqueued back to back and may overlap on the device
    phase("uploads")
    trs = []
    for g in range(ngrp):
        m, x, t, sols, tv = cases[g]
        tr = Transfer(local)
        tr.upload_background(m, sols, 0)
        tr.upload_points(x, t, tets_mmg=None if args.no_new_tets else tv)
        trs.append(tr)
    m, x, t, sols, tv = cases[0]
    tr = trs[0]
    S = sum(s.shape[1] for s in sols)

    def step(timing=False, flags=FRESH):
        # FRESH: the background's derived data is rebuilt as in a new iteration
        for g in trs:
            g.run(timing=timing, flags=flags)

    def sync():
        for g in trs:
            g.synchronize()

    phase("warmup + timed steps")
    for _ in range(args.warmup):
        step()
    sync()

    def barrier():
        if dist is not None:
            import torch
            dist.barrier()
            torch.cuda.synchronize()

    barrier()
    sync()
    for g in trs:
        g.timing_reset()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(timing=True)
    sync()
    barrier()
    el = time.perf_counter() - t0
    k_ms = {name: tr.kernel_ms(i) for i, name in enumerate(["hint", "vol", "bdy", "exhaustive", "total",
                                                            "derive"])}
    st = tr.locate_stats()
    st["volume_waves"] = tr.wave_stats(0)
    from parmmg_amd import mesh as M
    st["wrec_escapes"] = M.wrec_escapes(m)
    st["wrec_far_fields"], st["wrec_tets_with_far_fields"] = M.wrec_far_fields(m)
    # the walk's record format (pmx_capi.hip fill_vol_args: 32-B records above
    # 1/16 of the tets with a far neighbour field)
    # (r06: the compact records only when the upload builds them,
    # PMX_WALK_RECORDS=compact; default the 32-B records, no per-background pass)
    compact = os.environ.get("PMX_WALK_RECORDS") == "compact"
    st["walk_records"] = "24-B compact" if compact and st["wrec_tets_with_far_fields"] * 16 <= m.ne else "32-B"
    # the same step on a background already prepared by an earlier step (what
    # repeated steps on one background cost; reported, never `value`)
    sync()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        step(flags=0)
    sync()
    resident_ms = (time.perf_counter() - t1) / args.steps * 1e3

    # the reference's sequential semantics (PMX_RUN_SEQUENTIAL_SURFACE |
    # _VOLUME, bit-exact against the oracle's sequential run in tests/): their
    # cost, and how many points the default step answers differently --
    # another tria / edge / vertex on the surface, another tet in the volume
    seq = None
    if world == 1 and not args.no_seq and not args.no_new_tets:
        phase("sequential-semantics step")
        sync()
        tr.run(flags=N.RUN_FRESH_BACKGROUND)
        r0 = tr.download()
        e0, v0 = tr.border()
        tr.synchronize()
        t2 = time.perf_counter()
        tr.run(flags=N.RUN_FRESH_BACKGROUND | N.RUN_SEQUENTIAL_SURFACE | N.RUN_SEQUENTIAL_VOLUME)
        tr.synchronize()
        seq_ms = (time.perf_counter() - t2) * 1e3
        r1 = tr.download()
        e1, v1 = tr.border()
        ss, sv = tr.seq_surface_stats(), tr.seq_volume_stats()
        b = (t & M.TAG_BDY) != 0
        ndiff = int(((r0.elem != r1.elem) | (e0 != e1) | (v0 != v1))[b].sum())
        vdiff = int((r0.elem != r1.elem)[~b].sum())
        seq = {"ms": seq_ms, "surface_points": ss["nseq"], "surface_replayed": ss["nreplay"],
               "default_mode_differs_on_surface": ndiff, "volume_points": sv["nseq"],
               "volume_replayed": sv["nreplay"], "default_mode_differs_in_volume": vdiff,
               "note": "one FRESH step with PMX_RUN_SEQUENTIAL_SURFACE | _VOLUME (the reference's sequential "
                       "semantics), wall clock incl. host syncs; the default step answers the differing points "
                       "with another tria / edge / vertex (surface) or tet (volume ties) than the reference's "
                       "sequential run"}

    # the shipped binding's configuration (integration/pmmg_pmx.c sends no
    # adjacency: 16 B/tet less over PCIe), where every FRESH step also runs the
    # device face matching of the background -- reported beside ms_per_step,
    # never `value`
    devadj = None
    if world == 1 and not args.no_pcie:
        phase("FRESH steps with device face matching")
        sync()
        tr.upload_background(m, sols, 0, adja=False)
        tr.run(flags=FRESH)
        tr.synchronize()
        t3 = time.perf_counter()
        nda = max(3, min(args.steps, 10))
        for _ in range(nda):
            tr.run(flags=FRESH)
        tr.synchronize()
        devadj = {"ms": (time.perf_counter() - t3) / nda * 1e3, "steps": nda,
                  "note": "group 0, background uploaded without Mmg's adjacency (the shipped binding's "
                          "choice): each FRESH step also rebuilds the face adjacency and the tet records "
                          "on the device (pmx_topo.hip face matching)"}
        tr.upload_background(m, sols, 0)
        tr.run(flags=FRESH)                    # the legs below read the last step's results
        tr.synchronize()

    # host-staged rate (ParMmg's adapter path: host buffers in and out), measured
    # after the timed region and never reported as `value`
    pcie = None
    if world == 1 and not args.no_pcie:
        phase("host-staged cycles")
        pcie = pcie_inclusive(tr, m, x, t, sols)
        pcie["resident_cycle"] = resident_cycle(m, sols, cfg, local)
        pcie["binding_cycle"] = binding_cycle(m, x, t, tv, sols, local)

    if dist is not None:
        import torch
        tt = torch.tensor([el], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
        # the statistics reduction, the path's only collective: with RCCL (the
        # driver's multi-GPU runs) through the C ABI's communicator and
        # pmx_qualhisto_allreduce / pmx_prilen_allreduce -- what the ParMmg
        # binding links -- checked on every rank against the rank-ordered fold;
        # the gloo rehearsal (several ranks on one GPU, where RCCL cannot run)
        # all-gathers over torch.distributed instead
        from parmmg_amd import shard
        if args.dist_backend == "nccl":
            qs = shard.binding_collectives(trs, dist, rank, world, local)
        else:
            qs = shard.qualhisto_allreduce(tr, dist, local)
            qs["path"] = "torch.distributed all-gather (gloo rehearsal)"
    npts = len(x)
    total_pts = sum(len(c[1]) for c in cases) * world * args.steps
    value = total_pts / el
    ms = el / args.steps * 1e3

    nvol = int((t == 0).sum())
    B = alg_bytes(npts, m.ne, m.np, S)
    # all groups of this rank (C4: 2 concurrent groups, one stream each)
    B_all = sum(alg_bytes(len(c[1]), c[0].ne, c[0].np, S) for c in cases)
    b_vol = B * nvol / npts
    achieved = b_vol / (k_ms["vol"] * 1e-3) / 1e9 if k_ms["vol"] > 0 else None
    traffic, traffic_src = profiled_traffic(args.config)

    out = {
        "metric": "new vertices located+interpolated/sec",
        "value": value,
        "unit": "vertices/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (jittered Kuhn cube, jittered Morton-ordered new vertices, analytic fields)",
        "config": {"workload": f"{args.config}: {cfg['desc']}", "n_cells": cfg["n"], "ne": m.ne,
                   "np": m.np, "nt": m.nt,
                   "new_vertices_per_gpu": sum(len(c[1]) for c in cases), "S": S,
                   "groups_per_gpu": ngrp, "parallelism": f"group-sharded x{world}",
                   "numbering": args.numbering},
        "roofline": {"bound": "hbm", "kernel": "k_walks",
                     "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                     "traffic": traffic, "traffic_source": traffic_src,
                     "alg_bytes_per_launch": b_vol, "avg_launch_ms": k_ms["vol"],
                     # >1: that many groups' walks run at once on separate
                     # streams, each launch's duration includes the others'
                     "concurrent_launches": ngrp,
                     # the whole step against the same peak (SURVEY 8(d)'s
                     # algorithmic bytes of the step / ms_per_step)
                     "step_frac": B_all / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS},
        "kernel_ms": k_ms,
        "per_iteration": {"ms": ms, "includes": (
            "every device pass of one PMMG_interpMetricsAndFields call on the raw uploaded arrays "
            "(PMX_RUN_FRESH_BACKGROUND): derived background data (grid coordinates, tria normals = "
            "PMMG_precompute_triaNormals), node -> trias fans with the upload's fan check "
            "(PMMG_precompute_nodeTrias), the layouts the upload derived on the device (none in the "
            "default configuration), "
            + ("orphan marks from the new tets (vertex loop over the new tets), " if not args.no_new_tets
               else "")
            + "tag dispatch + order-preserving compaction of the new points, hint grid, volume walk + "
            "interpolation, surface path, fallback"),
            "not_in_ms": "host packing and PCIe (pcie_inclusive); nothing the device runs per "
                         "upload is outside the step",
            "binding_configuration": devadj},
        "resident_background_ms_per_step": resident_ms,
        "step_alg_GBs": B_all / (ms * 1e-3) / 1e9,
        "locate": st,
    }
    if cpu is not None:
        if pcie is not None:
            # what ParMmg sees (the binding's two seams per iteration, host
            # buffers in and out) against the CPU node and one CPU core
            b = pcie["binding_cycle"]["value"]
            cpu["binding_cycle"] = {"vertices_per_s": b, "speedup_vs_node": b / cpu["value"],
                                    "speedup_vs_core": b / cpu["per_core"]}
        if cpu.get("physical_cores"):
            # an ESTIMATE, not a measurement: the per-core rate of the K measured
            # processes times the machine's physical cores (the reference run as
            # one MPI rank per core on the whole node, memory bandwidth assumed
            # to scale); what ParMmg gets from the GPU is binding_cycle
            est = cpu["per_core"] * cpu["physical_cores"]
            cpu["full_node_estimate"] = {
                "value": est, "unit": "vertices/s", "cores": cpu["physical_cores"], "kind": "estimate",
                "how": "per_core x physical cores (lscpu), not measured",
                "device_step_vs_estimate": value / est,
                "binding_cycle_vs_estimate": (pcie["binding_cycle"]["value"] / est) if pcie else None}
        out["cpu_baseline"] = cpu
    if pcie is not None:
        out["pcie_inclusive"] = pcie
    if seq is not None:
        out["sequential_surface"] = seq
    if dist is not None:
        out["qualhisto_allreduce"] = qs
        dist.destroy_process_group()
    if rank == 0:
        phase("done")
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
