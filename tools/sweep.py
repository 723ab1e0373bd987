#!/usr/bin/env python3
"""Interleaved A/B of run options in ONE process (cdna guide rule 24).

  python tools/sweep.py --config C2 --rounds 5 --opt hint_stride=1,2,4,8

Prints per-variant median/min kernel times (HIP events) and walk statistics.
"""
import argparse
import json
import os
import sys

import numpy as np

# the measurement switches (run flag exp 4 / 5) are refused without it
os.environ.setdefault("PMX_EXPERIMENTS", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--opt", default="hint_stride=1,4")
    ap.add_argument("--n", type=int, default=0, help="override the config's cells per axis")
    ap.add_argument("--numbering", default="lex",
                    help="background tet numbering (bench.py --numbering; appended:F moves "
                         "a fraction F of the tets)")
    ap.add_argument("--check", action="store_true",
                    help="compare every variant's results bit for bit with the first one's")
    args = ap.parse_args()
    import bench
    from parmmg_amd import build
    build.build_meshgen()
    build.build_transfer()
    from parmmg_amd.transfer import Transfer
    cfg = dict(bench.CONFIGS[args.config])
    if args.n:
        cfg["n"] = args.n
    m, x, t, sols, _ = bench.build_case(cfg, 0)
    if args.numbering != "lex":
        from parmmg_amd import mesh as M
        kind, _, frac = args.numbering.partition(":")
        m = M.numbering(m, kind, frac=float(frac) if frac else 0.1)[0]
        print("far fields, tets with one:", M.wrec_far_fields(m), "of", m.ne, flush=True)
    tr = Transfer(0)
    tr.upload_background(m, sols, 0)
    tr.upload_points(x, t)
    key, vals = args.opt.split("=")
    vals = [int(v) for v in vals.split(",")]
    res = {v: {k: [] for k in ("hint", "vol", "bdy", "exhaustive", "total")} for v in vals}
    stats = {}
    mism = {}
    if args.check:
        ref = None
        for v in vals:
            tr.run(**{key: v})
            r = tr.download()
            if ref is None:
                ref = r
                continue
            bad = int(np.count_nonzero(r.elem != ref.elem))
            bad += int(np.count_nonzero(r.status != ref.status))
            for a, b in zip(r.sols, ref.sols):
                bad += int(np.count_nonzero(a.view(np.uint64) != b.view(np.uint64)))
            mism[v] = bad
    for _ in range(args.rounds):
        for v in vals:
            kw = {key: v}
            tr.run(**kw)
            tr.synchronize()
            tr.timing_reset()
            for _ in range(args.reps):
                tr.run(timing=True, **kw)
            for i, k in enumerate(("hint", "vol", "bdy", "exhaustive", "total")):
                res[v][k].append(tr.kernel_ms(i))
            stats[v] = tr.locate_stats()
    out = {}
    for v in vals:
        out[v] = {k: (float(np.median(a)), float(np.min(a))) for k, a in res[v].items()}
        out[v]["stepav"] = stats[v]["stepav"]
        out[v]["nexhaust"] = stats[v]["nexhaust"]
        if v in mism:
            out[v]["mismatches"] = mism[v]
    print(json.dumps({"config": args.config, "n": cfg["n"], "npts": int(len(x)), "opt": key,
                      "numbering": args.numbering,
                      "ms(median,min)": out}, indent=1))


if __name__ == "__main__":
    main()
