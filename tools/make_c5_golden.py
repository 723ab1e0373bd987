#!/usr/bin/env python3
"""Golden statistics of C5's per-GPU share (Kuhn n = 275, 124.8M tets) from
the oracle (oracle/pmx_oracle_stats.c: MMG3D_tetraQual / computeInqua and
MMG3D_computePrilen restated), for test_gpu_configs.py::test_c5_share_stats_
against_oracle: the device statistics at full size compared with the
sequential restatement, not only with the analytic counts.

Runs on the CPU (about 20 GB of memory for the oracle's edge hash, a few
minutes); writes tests/golden/c5share_stats.json.

  python tools/make_c5_golden.py [--n 275]
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
    ap.add_argument("--n", type=int, default=275)
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "golden", "c5share_stats.json"))
    args = ap.parse_args()
    from parmmg_amd import build
    build.build_meshgen()
    build.build_oracle()
    from oracle import oracle as O
    from parmmg_amd import mesh as M
    t0 = time.time()
    m = M.kuhn_cube(args.n)
    out = {"n": args.n, "ne": int(m.ne), "np": int(m.np), "generator": "mesh.kuhn_cube(n), default seed"}
    q = O.tetra_qual(m)
    out["qualhisto"] = O.qualhisto(m, q)
    print(f"qualhisto {time.time() - t0:.1f}s", flush=True)
    for name, f in (("iso", M.iso_metric), ("graded", M.graded_iso_metric(args.n))):
        met = M.on_vertices(m, f)
        out[f"prilen_{name}"] = O.prilen(m, met)
        print(f"prilen {name} {time.time() - t0:.1f}s", flush=True)
        del met
    for k, v in list(out.items()):
        if isinstance(v, dict):
            out[k] = {kk: (list(map(int, vv)) if isinstance(vv, list) else vv) for kk, vv in v.items()}
    with open(args.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", args.out)


if __name__ == "__main__":
    main()
