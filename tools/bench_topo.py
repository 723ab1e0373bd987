#!/usr/bin/env python3
"""Background topology throughput: GPU face matching
vs the CPU sort-based builder of parmmg_amd/csrc/meshgen.c (one core, qsort --
a stand-in for Mmg's hash-based MMG3D_hashTetra, which is absent here).

  python tools/bench_topo.py [--n 119] [--reps 3]
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
    ap.add_argument("--n", type=int, default=119)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cpu", action="store_true", help="also time the CPU builder")
    args = ap.parse_args()
    import numpy as np
    from parmmg_amd import build
    build.build_meshgen()
    build.build_transfer()
    from parmmg_amd import mesh as M
    from parmmg_amd.transfer import Transfer
    m = M.kuhn_cube(args.n)
    tr = Transfer(0)
    adja = tr.build_adja(m.tet, m.np)                     # warm-up
    assert np.array_equal(adja, m.adja)
    ta, tb, wa = [], [], []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        adja = tr.build_adja(m.tet, m.np)
        wa.append(time.perf_counter() - t0)
        ta.append(tr.topo_ms())
        tria, adjt = tr.build_bdry(m.tet, m.np, adja)
        tb.append(tr.topo_ms())
    assert np.array_equal(tria, m.tria) and np.array_equal(adjt, m.adjt)
    out = {"metric": "tets/s (face adjacency), device time", "config": {"n": args.n, "ne": m.ne,
                                                                        "np": m.np, "nt": m.nt},
           "adja_ms": min(ta), "adja_tets_per_s": m.ne / (min(ta) * 1e-3),
           "adja_wall_ms_incl_pcie": min(wa) * 1e3,
           "bdry_ms": min(tb), "exact_vs_cpu_builder": True}
    if args.cpu:
        lib = M._meshgen()
        a2 = np.zeros_like(adja)
        t0 = time.perf_counter()
        lib.pmg_build_adja(m.ne, M._p(m.tet), M._p(a2))
        out["cpu_qsort_adja_ms"] = (time.perf_counter() - t0) * 1e3
    print(json.dumps(out), flush=True)
    tr.close()


if __name__ == "__main__":
    main()
