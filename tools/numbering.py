#!/usr/bin/env python3
"""Background numbering vs walk cost: the same mesh and new points with the
background's tets and vertices renumbered (interleaved A/B in one process).

  python tools/numbering.py --config C3 --variants lex,morton,random

lex    = the generator's numbering (cell-lexicographic tets, lexicographic
         vertices);
morton = tets by the Morton key of their centroid, vertices by their own key
         (what a device renumbering at upload would produce);
vmorton / tmorton = only the vertices / only the tets in Morton order;
random = both permuted at random (a numbering without spatial locality).
Prints per-variant median/min kernel times and checks that every variant
locates the same points (elements mapped back through the permutation).
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def morton_keys(x: np.ndarray, bits: int = 21) -> np.ndarray:
    lo, hi = x.min(axis=0), x.max(axis=0)
    q = ((x - lo) / np.maximum(hi - lo, 1e-300) * ((1 << bits) - 1)).astype(np.uint64)
    key = np.zeros(len(x), np.uint64)
    for b in range(bits):
        for d in range(3):
            key |= ((q[:, d] >> np.uint64(b)) & np.uint64(1)) << np.uint64(3 * b + d)
    return key


def renumber(m, tperm, vperm):
    from parmmg_amd.mesh import renumber as R
    return R(m, tperm, vperm)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variants", default="lex,morton,random")
    ap.add_argument("--n", type=int, default=0)
    args = ap.parse_args()
    import bench
    from parmmg_amd import build
    from parmmg_amd import _native as N
    build.build_meshgen()
    build.build_transfer()
    from parmmg_amd.transfer import Transfer
    cfg = dict(bench.CONFIGS[args.config])
    if args.n:
        cfg["n"] = args.n
    m, x, t, sols, _ = bench.build_case(cfg, 0)
    rng = np.random.default_rng(7)
    trs, back = {}, {}
    for v in args.variants.split(","):
        if v == "lex":
            mm, ss, tinv = m, sols, None
        else:
            if v == "morton":
                tp = np.argsort(morton_keys(m.centroids()), kind="stable")
                vp = np.argsort(morton_keys(m.xyz[1:]), kind="stable")
            elif v == "vmorton":                      # vertices only (tets keep their order)
                tp = np.arange(m.ne)
                vp = np.argsort(morton_keys(m.xyz[1:]), kind="stable")
            elif v == "tmorton":                      # tets only
                tp = np.argsort(morton_keys(m.centroids()), kind="stable")
                vp = np.arange(m.np)
            elif v == "random":
                tp, vp = rng.permutation(m.ne), rng.permutation(m.np)
            else:
                raise SystemExit(f"unknown variant {v}")
            mm, tinv = renumber(m, tp, vp)
            ss = [np.ascontiguousarray(np.concatenate([s[:1], s[1:][vp]])) if s.shape[0] == m.np + 1
                  else np.ascontiguousarray(s[vp]) for s in sols]
        tr = Transfer(0)
        tr.upload_background(mm, ss, 0)
        tr.upload_points(x, t)
        trs[v], back[v] = tr, tinv
        print(f"uploaded {v}", file=sys.stderr, flush=True)
    ref = None
    mism = {}
    for v, tr in trs.items():
        tr.run(flags=N.RUN_FRESH_BACKGROUND)
        r = tr.download()
        el = r.elem.astype(np.int64)
        if back[v] is not None:                       # new index -> lex index
            inv = np.zeros(m.ne + 1, np.int64)
            inv[back[v]] = np.arange(m.ne + 1)
            el = np.where((t == 0) & (el > 0), inv[np.maximum(el, 0)], el)
        if ref is None:
            ref = (el, r)
            continue
        vol = t == 0
        mism[v] = {"elem": int(np.count_nonzero(el[vol] != ref[0][vol])),
                   "sol_max_abs": float(max(np.max(np.abs(a[vol] - b[vol])) for a, b in
                                            zip(r.sols, ref[1].sols)))}
    names = ("hint", "vol", "bdy", "exhaustive", "total", "derive")
    res = {v: {k: [] for k in names} for v in trs}
    stats = {}
    for _ in range(args.rounds):
        for v, tr in trs.items():
            tr.run(flags=N.RUN_FRESH_BACKGROUND)
            tr.synchronize()
            tr.timing_reset()
            for _ in range(args.reps):
                tr.run(timing=True, flags=N.RUN_FRESH_BACKGROUND)
            for i, k in enumerate(names):
                res[v][k].append(tr.kernel_ms(i))
            stats[v] = tr.locate_stats()
    out = {}
    for v in trs:
        out[v] = {k: (float(np.median(a)), float(np.min(a))) for k, a in res[v].items()}
        out[v]["stepav"] = stats[v]["stepav"]
        out[v]["nexhaust"] = stats[v]["nexhaust"]
        if v in mism:
            out[v]["vs_lex"] = mism[v]
    print(json.dumps({"config": args.config, "n": cfg["n"], "npts": int(len(x)),
                      "ms(median,min)": out}, indent=1))
    for tr in trs.values():
        tr.close()


if __name__ == "__main__":
    main()
