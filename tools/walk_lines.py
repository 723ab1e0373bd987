#!/usr/bin/env python3
"""Which 128-B lines the volume walk touches (CPU model, no GPU).

  python tools/walk_lines.py [--config C2] [--n N]

Replays the slot walk's path for every volume point on the CPU (hint grid
built as on the device: every 4th tet, fixed-point centroid cell, last
sample in index order wins; steps through the face of the most negative
barycentric among the interior, not recently visited neighbours) and counts
the distinct lines of the 32-B tet records, the 24-B vertex rows and the
solution rows it reads -- split into the lines only the hint record needs
and the lines the rest of the walk needs anyway.  Prints one JSON object.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def grid_dims(lo, hi, ne):
    ext = np.maximum(hi - lo, 1e-300)
    h = np.cbrt(np.prod(ext) / max(1.0, ne / 6.0))
    dim = np.clip(np.ceil(ext / h * (1.0 - 1e-9)).astype(np.int64), 1, 4096)
    qf = np.array([21 - int(np.ceil(np.log2(d))) if d > 1 else 21 for d in dim])
    return dim, dim / ext, qf


def lambdas(P, p):
    """Barycentrics of points p (n,3) in tets with vertex coordinates P (n,4,3)."""
    a, b, c, d = P[:, 0], P[:, 1], P[:, 2], P[:, 3]
    vol = np.einsum("ij,ij->i", b - a, np.cross(c - a, d - a))
    l1 = np.einsum("ij,ij->i", p - a, np.cross(c - a, d - a)) / vol
    l2 = np.einsum("ij,ij->i", b - a, np.cross(p - a, d - a)) / vol
    l3 = np.einsum("ij,ij->i", b - a, np.cross(c - a, p - a)) / vol
    return np.stack([1.0 - l1 - l2 - l3, l1, l2, l3], axis=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--n", type=int, default=0)
    args = ap.parse_args()
    import bench
    cfg = dict(bench.CONFIGS[args.config])
    if args.n:
        cfg["n"] = args.n
    m, x, t, sols, _ = bench.build_case(cfg, 0)
    S = sum(s.shape[1] for s in sols)
    ne = m.ne
    tet = m.tet.astype(np.int64)
    nb = np.zeros((ne + 1, 4), np.int64)
    nb[1:] = m.adja[1:4 * ne + 1].reshape(ne, 4) // 4
    xyz = m.xyz
    lo, hi = xyz[1:].min(axis=0), xyz[1:].max(axis=0)
    dim, inv, qf = grid_dims(lo, hi, ne)
    # fixed-point vertex coordinates and the sampled tets' centroid cells
    q = np.clip(((xyz - lo) * inv * (1 << qf)).astype(np.int64), 0, (dim << qf) - 1)
    ks = np.arange(1, ne + 1, 4)
    s4 = q[tet[ks]].sum(axis=1)
    cell = np.minimum(s4 >> (qf + 2), dim - 1)
    cid = cell[:, 0] + dim[0] * (cell[:, 1] + dim[1] * cell[:, 2])
    grid = np.zeros(int(np.prod(dim)), np.int64)
    grid[cid] = ks                                   # last sample in index order wins
    vol = t == 0
    p = x[vol]
    pc = np.clip(((p - lo) * inv).astype(np.int64), 0, dim - 1)
    start = grid[pc[:, 0] + dim[0] * (pc[:, 1] + dim[1] * pc[:, 2])]
    miss = start == 0
    start[miss] = 1                                  # empty cells: rare, any start
    n = len(p)
    cur = start.copy()
    ring = np.zeros((n, 4), np.int64)
    active = np.ones(n, bool)
    visited = [cur.copy()]
    steps = np.ones(n, np.int64)
    for it in range(64):
        idx = np.nonzero(active)[0]
        if len(idx) == 0:
            break
        lam = lambdas(xyz[tet[cur[idx]]], p[idx])
        done = lam.min(axis=1) > -1e-6
        active[idx[done]] = False
        idx = idx[~done]
        lam = lam[~done]
        nbs = nb[cur[idx]]
        seen = (nbs[:, :, None] == ring[idx][:, None, :]).any(axis=2)
        ok = (nbs != 0) & ~seen
        lam = np.where(ok, lam, np.inf)
        f = lam.argmin(axis=1)
        stuck = ~ok.any(axis=1)
        active[idx[stuck]] = False
        idx, f = idx[~stuck], f[~stuck]
        ring[idx, 1:] = ring[idx, :3]
        ring[idx, 0] = cur[idx]
        cur[idx] = nbs[~stuck][np.arange(len(idx)), f]
        steps[idx] += 1
        v = np.zeros(n, np.int64)
        v[idx] = cur[idx]
        visited.append(v)
    V = np.stack(visited, axis=1)                    # (n, steps) tets, 0 = none
    tline = lambda k: k // 4                         # 32-B records, 4 per line
    hint_lines = np.unique(tline(start))
    rest = V[:, 1:][V[:, 1:] > 0]
    rest_lines = np.unique(tline(rest))
    final = cur
    all_lines = np.union1d(hint_lines, rest_lines)
    only_hint = np.setdiff1d(hint_lines, rest_lines)
    # vertex rows (24 B) of every visited tet, solution rows of the final tet
    vt = tet[V[V > 0]]
    vrows = np.unique(vt)
    vlines = np.unique(np.concatenate([(24 * vrows) // 128, (24 * vrows + 23) // 128]))
    srows = np.unique(tet[final])
    slines = np.unique(np.concatenate([(8 * S * srows) // 128, (8 * S * srows + 8 * S - 1) // 128]))
    out = {
        "config": args.config, "n": cfg["n"], "ne": int(ne), "np": int(m.np), "volume_points": int(n),
        "mean_steps": float(steps.mean()), "empty_hint_cells": int(miss.sum()),
        "tet_lines_total": int(ne // 4 + 1),
        "tet_lines_touched": int(len(all_lines)),
        "tet_lines_hint": int(len(hint_lines)),
        "tet_lines_rest_of_walk": int(len(rest_lines)),
        "tet_lines_only_for_the_hint": int(len(only_hint)),
        "vertex_lines_touched": int(len(vlines)), "vertex_lines_total": int((24 * (m.np + 1)) // 128 + 1),
        "solution_lines_touched": int(len(slines)),
        "solution_lines_total": int((8 * S * (m.np + 1)) // 128 + 1),
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
