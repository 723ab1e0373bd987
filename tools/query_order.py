#!/usr/bin/env python3
"""Order of the new points vs walk cost (interleaved A/B in one process):
the same background and points, uploaded in Morton order (the bench's),
lexicographic cell order (the background's own numbering) and at random.

  python tools/query_order.py --config C3
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
    ap.add_argument("--config", default="C3")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import bench
    from parmmg_amd import build
    from parmmg_amd import _native as N
    build.build_meshgen()
    build.build_transfer()
    from parmmg_amd.transfer import Transfer
    cfg = dict(bench.CONFIGS[args.config])
    m, x, t, sols, _ = bench.build_case(cfg, 0)
    n = cfg["n"]
    c = np.clip((x * n).astype(np.int64), 0, n - 1)
    orders = {"morton": np.arange(len(x)),
              "lex": np.lexsort((c[:, 0], c[:, 1], c[:, 2])),
              "random": np.random.default_rng(3).permutation(len(x))}
    tr = Transfer(0)
    tr.upload_background(m, sols, 0)
    names = ("hint", "vol", "bdy", "exhaustive", "total", "derive")
    res = {k: {nm: [] for nm in names} for k in orders}
    stats = {}
    for _ in range(args.rounds):
        for k, o in orders.items():
            tr.upload_points(np.ascontiguousarray(x[o]), np.ascontiguousarray(t[o]))
            tr.run(flags=N.RUN_FRESH_BACKGROUND)
            tr.synchronize()
            tr.timing_reset()
            for _ in range(args.reps):
                tr.run(timing=True, flags=N.RUN_FRESH_BACKGROUND)
            for i, nm in enumerate(names):
                res[k][nm].append(tr.kernel_ms(i))
            stats[k] = tr.locate_stats()
    out = {k: {nm: (float(np.median(a)), float(np.min(a))) for nm, a in v.items()} for k, v in res.items()}
    for k in out:
        out[k]["stepav"] = stats[k]["stepav"]
    print(json.dumps({"config": args.config, "npts": int(len(x)), "ms(median,min)": out}, indent=1))
    tr.close()


if __name__ == "__main__":
    main()
