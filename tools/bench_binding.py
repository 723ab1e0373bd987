#!/usr/bin/env python3
"""The shipped binding's per-iteration cycle alone (bench.binding_cycle: the
two ParMmg seams on Mmg-shaped AoS records), for host-phase tracing:

  PMX_TRACE=1 python tools/bench_binding.py [--config C3] [--iters 3]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--iters", type=int, default=3)
    args = ap.parse_args()
    import bench
    cfg = bench.CONFIGS[args.config]
    m, x, t, sols, tv = bench.build_case(cfg, 0)
    print(json.dumps(bench.binding_cycle(m, x, t, tv, sols, 0, iters=args.iters)), flush=True)


if __name__ == "__main__":
    main()
