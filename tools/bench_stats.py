#!/usr/bin/env python3
"""Quality histogram + metric edge-length statistics throughput (SURVEY.md 8
rows Q1-Q3; BASELINE.json configs[4] "C5": 1B tets over 2/4/8 GPUs, i.e.
~125M tets per GPU at 8 GPUs).

  python tools/bench_stats.py [--n 275] [--metric iso|ani] [--reps 10]

One rep = PMMG_tetraQual + PMMG_qualhisto's per-group pass (k_qual +
k_qual_final) and PMMG_prilen's per-group pass (k_prilen + k_prilen_final) on
the uploaded background, device partials only (the RCCL all-reduce of
parmmg_amd/shard.py is timed separately by bench.py at N > 1).  Prints one
JSON line: tets/s per statistic, algorithmic GB/s against SURVEY.md 8(d)
(ne*16 + np*(24 + 8*S_m) bytes per pass) and the HIP-event kernel times.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=275, help="Kuhn cube cells per axis (ne = 6 n^3)")
    ap.add_argument("--metric", default="iso", choices=["iso", "graded", "ani"],
                    help="iso: h = 0.05 + 0.1 x (every edge in bin 0); graded: lengths over all 9 bins")
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    import numpy as np
    import torch
    from parmmg_amd import build
    build.build_meshgen()
    build.build_transfer()
    from parmmg_amd import mesh as M
    from parmmg_amd.transfer import Transfer

    t0 = time.perf_counter()
    m = M.kuhn_cube(args.n)
    met = M.on_vertices(m, {"iso": M.iso_metric, "graded": M.graded_iso_metric(args.n),
                            "ani": M.shock_metric}[args.metric])
    tr = Transfer(0)
    tr.upload_background(m, [met], 0)
    t_setup = time.perf_counter() - t0
    dev = torch.device("cuda", 0)
    from parmmg_amd import shard
    qpart = torch.zeros(shard.QUAL_WORDS, dtype=torch.float64, device=dev)
    lpart = torch.zeros(shard.LEN_WORDS, dtype=torch.float64, device=dev)

    def timed(fn):
        fn()
        tr.synchronize()
        t = time.perf_counter()
        for _ in range(args.reps):
            fn()
        tr.synchronize()
        return (time.perf_counter() - t) / args.reps

    tq = timed(lambda: tr.qualhisto_device(qpart.data_ptr()))
    tl = timed(lambda: tr.prilen_device(lpart.data_ptr()))
    q = tr.qualhisto()
    ln = tr.prilen()
    S = met.shape[1]
    # compulsory bytes: the connectivity stream and one pass over the vertices
    # and their metric; the quality pass also stores every tet's quality
    # (MMG3D_tetraQual's pt->qual, 8 B per tet, read back by OUTQUA)
    B = m.ne * 16 + m.np * (24 + 8 * S)
    Bq = B + m.ne * 8
    out = {
        "metric": "tets/s (quality histogram, edge-length stats)",
        "config": {"workload": f"C5 per-GPU share: Kuhn cube n={args.n}", "ne": m.ne, "np": m.np,
                   "metric": args.metric, "S_m": S},
        "qualhisto": {"ms": tq * 1e3, "tets_per_s": m.ne / tq, "alg_GBs": Bq / tq / 1e9,
                      "frac_hbm_peak": Bq / tq / 8e12, "alg_bytes": Bq, "ne": q["ne"], "his": q["his"],
                      "min": q["min"], "max": q["max"]},
        "prilen": {"ms": tl * 1e3, "tets_per_s": m.ne / tl, "alg_GBs": B / tl / 1e9,
                   "frac_hbm_peak": B / tl / 8e12, "alg_bytes": B, "ned": ln["ned"], "hl": ln["hl"],
                   "sched": os.environ.get("PMX_PRILEN_SCHED", "0"),
                   **{k: ln[k] for k in ("avlen", "lmin", "lmax", "amin", "bmin", "amax", "bmax", "nullEdge")
                      if k in ln}},
        "setup_s": t_setup,
        "dtype": "f64", "data": "synthetic (jittered Kuhn cube, analytic metric)",
    }
    print(json.dumps(out), flush=True)
    tr.close()
    del np


if __name__ == "__main__":
    main()
