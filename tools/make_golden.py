#!/usr/bin/env python3
"""Generate the committed regression fixtures under tests/golden/ from the
oracle (the CPU restatement of the reference algorithm).

These are regression vectors of the restatement, NOT pins against the
reference: the reference ships no golden vectors for this path and compiles
here only against stand-in Mmg headers (see DESIGN.md "Oracle").  Re-run after an intentional oracle
change:  python tools/make_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from helpers import cube_case  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main():
    n, metric = 6, "ani"
    m, x, t, sols = cube_case(n, metric=metric)
    o = O.Oracle(m)
    outs, elem, st, steps, e, v = o.interp(x, t, sols, imet=0)
    d = dict(n=n, metric=metric, xyz=x, tags=t, elem=elem, status=st, steps=steps, edge=e, vertex=v)
    for s, a in enumerate(outs):
        d[f"sol{s}"] = a
    path = os.path.join(ROOT, "tests", "golden", "oracle_kuhn.npz")
    np.savez_compressed(path, **d)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
