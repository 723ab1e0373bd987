#!/usr/bin/env python3
"""Bit-compare a step's results under a run-flag experiment against the
default step (an A/B that must not change results):

  python tools/ab_exp_equal.py --exp 24 [--config C2]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--exp", type=int, required=True)
    ap.add_argument("--config", default="C2")
    args = ap.parse_args()
    import numpy as np
    import bench
    from parmmg_amd import _native as N
    from parmmg_amd.transfer import Transfer
    m, x, t, sols, tv = bench.build_case(bench.CONFIGS[args.config], 0)
    tr = Transfer(0)
    tr.upload_background(m, sols, 0)
    tr.upload_points(x, t, tets_mmg=tv)
    res = []
    for fl in (N.RUN_FRESH_BACKGROUND, N.RUN_FRESH_BACKGROUND | (args.exp << 16)):
        tr.run(flags=fl)
        r = tr.download()
        res.append((r, tr.border()))
    (a, ea), (b, eb) = res
    same = all(np.array_equal(np.asarray(x1).view(np.uint8), np.asarray(x2).view(np.uint8))
               for x1, x2 in zip(a.sols + [a.elem, a.status], b.sols + [b.elem, b.status]))
    same = same and np.array_equal(ea[0], eb[0]) and np.array_equal(ea[1], eb[1])
    print(f"exp {args.exp} on {args.config}: results {'bit-identical' if same else 'DIFFER'}")
    sys.exit(0 if same else 1)


if __name__ == "__main__":
    main()
