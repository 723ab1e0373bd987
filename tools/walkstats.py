#!/usr/bin/env python3
"""Walk diagnostics on a bench config (GPU): histogram of walk steps, distance
from the hint start, ties / stuck counts.

  python tools/walkstats.py --config C2 [--flags F] [--hint-stride S]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--flags", type=int, default=0)
    ap.add_argument("--hint-stride", type=int, default=0)
    args = ap.parse_args()
    import bench
    from parmmg_amd import build
    build.build_meshgen()
    build.build_transfer()
    from parmmg_amd.transfer import Transfer
    cfg = bench.CONFIGS[args.config]
    m, x, t, sols, _ = bench.build_case(cfg, 0)
    tr = Transfer(0)
    tr.upload_background(m, sols, 0)
    tr.upload_points(x, t)
    tr.run(flags=args.flags, hint_stride=args.hint_stride, record_starts=True)
    r = tr.download()
    st = tr.starts()
    vol = t == 0
    steps = r.steps[vol]
    h = np.bincount(np.clip(np.abs(steps), 0, 20))
    c = m.centroids()
    d = np.linalg.norm(c[st[vol] - 1] - x[vol], axis=1) * cfg["n"]
    ng = cfg["n"] ** 3
    grid = np.zeros(ng, np.int32)
    tr.lib.pmx_debug_hint_grid(tr.ctx, grid.ctypes.data, ng)
    # the cell of each sampled tet's centroid, recomputed on the host
    ks = np.arange(1, m.ne + 1, 4)
    cen = m.xyz[m.tet[ks]].mean(axis=1)
    cell = np.clip((cen * cfg["n"]).astype(np.int64), 0, cfg["n"] - 1)
    ci = cell[:, 0] + cfg["n"] * (cell[:, 1] + cfg["n"] * cell[:, 2])
    ok = np.zeros(ng, bool)
    gi = grid.astype(np.int64)
    nz = gi > 0
    # a cell's hint must be one of the samples whose centroid is in that cell
    samp_cell = np.full(m.ne + 1, -1, np.int64)
    samp_cell[ks] = ci
    ok[nz] = samp_cell[gi[nz]] == np.nonzero(nz)[0]
    out_grid = {"cells": ng, "empty": int((~nz).sum()), "wrong_cell": int((nz & ~ok).sum())}
    del cen, cell, ci, samp_cell
    out = {"grid": out_grid, "config": args.config, "n": cfg["n"], "nvol": int(vol.sum()),
           "steps_hist": {int(i): int(v) for i, v in enumerate(h) if v},
           "steps_mean": float(np.abs(steps).mean()),
           "start_dist_cells": {"mean": float(d.mean()), "p50": float(np.median(d)),
                                "p99": float(np.percentile(d, 99)), "max": float(d.max())},
           "status": {int(k): int(v) for k, v in zip(*np.unique(r.status[vol], return_counts=True))},
           "stats": tr.locate_stats()}
    # surface path: steps per point and per wave (64 consecutive list entries)
    bdy = np.nonzero(t == 16)[0]
    if len(bdy):
        bs = np.abs(r.steps[bdy]).astype(np.int64)
        pad = (-len(bs)) % 64
        wmax = np.concatenate([bs, np.zeros(pad, np.int64)]).reshape(-1, 64).max(1)
        out["bdy"] = {"n": int(len(bdy)), "steps_mean": float(bs.mean()),
                      "steps_hist": {int(i): int(v) for i, v in enumerate(np.bincount(np.clip(bs, 0, 40))) if v},
                      "wave_max_mean": float(wmax.mean()), "wave_max_max": int(wmax.max()),
                      "status": {int(k): int(v) for k, v in zip(*np.unique(r.status[bdy], return_counts=True))}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
