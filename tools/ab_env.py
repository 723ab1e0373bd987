#!/usr/bin/env python3
"""Interleaved A/B of upload-time switches (environment variables read by
pmx_upload_background, e.g. PMX_HINT_SAMPLE_ORDER) in ONE process: one
context per value, each uploaded under its value, then timed in turn.

  python tools/ab_env.py --config C3 --env PMX_HINT_SAMPLE_ORDER=0,1,2

Prints per-value median/min kernel times (HIP events), walk statistics and
the number of results differing from the first value's (elem, status, fields
bit for bit).
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
    ap.add_argument("--env", required=True, help="NAME=v1,v2,...")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--flags", type=int, default=16, help="pmx_run flags (16: fresh background)")
    ap.add_argument("--numbering", default="lex")
    args = ap.parse_args()
    import bench
    from parmmg_amd import build
    build.build_meshgen()
    build.build_transfer()
    from parmmg_amd.transfer import Transfer
    cfg = dict(bench.CONFIGS[args.config])
    m, x, t, sols, _ = bench.build_case(cfg, 0)
    if args.numbering != "lex":
        from parmmg_amd import mesh as M
        kind, _, frac = args.numbering.partition(":")
        m = M.numbering(m, kind, frac=float(frac) if frac else 0.1)[0]
    name, vals = args.env.split("=")
    vals = vals.split(",")
    trs = {}
    for v in vals:
        os.environ[name] = v
        tr = Transfer(0)
        tr.upload_background(m, sols, 0)
        tr.upload_points(x, t)
        trs[v] = tr
        print(f"uploaded {name}={v}", flush=True)
    keys = ("hint", "vol", "bdy", "exhaustive", "total")
    res = {v: {k: [] for k in keys} for v in vals}
    ref, mism, stats = None, {}, {}
    for v in vals:
        trs[v].run(flags=args.flags)
        r = trs[v].download()
        if ref is None:
            ref = r
            continue
        bad = int(np.count_nonzero(r.elem != ref.elem)) + int(np.count_nonzero(r.status != ref.status))
        for a, b in zip(r.sols, ref.sols):
            bad += int(np.count_nonzero(a.view(np.uint64) != b.view(np.uint64)))
        mism[v] = bad
    for _ in range(args.rounds):
        for v in vals:
            tr = trs[v]
            tr.run(flags=args.flags)
            tr.synchronize()
            tr.timing_reset()
            for _ in range(args.reps):
                tr.run(timing=True, flags=args.flags)
            for i, k in enumerate(keys):
                res[v][k].append(tr.kernel_ms(i))
            stats[v] = tr.locate_stats()
        print("round done", flush=True)
    out = {}
    for v in vals:
        out[v] = {k: (float(np.median(a)), float(np.min(a))) for k, a in res[v].items()}
        out[v]["stepav"] = stats[v]["stepav"]
        if v in mism:
            out[v]["mismatches"] = mism[v]
    print(json.dumps({"config": args.config, "numbering": args.numbering, "env": name,
                      "ms(median,min)": out}, indent=1))


if __name__ == "__main__":
    main()
