"""Diagnose FRESH vs plain step differences on the test_fresh_step_equals_upload_step case."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
from helpers import cube_case
from parmmg_amd import _native as N, mesh as M
from parmmg_amd.transfer import Transfer

m, x, t, sols = cube_case(7, metric="ani", surface=True)
n = len(x); x = x.copy(); t = t.copy(); t[3::53] |= M.TAG_REQ
rng = np.random.default_rng(5)
used = np.zeros(n, bool); used[: int(0.8 * n)] = True
x[np.nonzero(~used)[0][:4]] = [1.5, -0.5, 0.5]
pool = np.nonzero(used)[0]
tets = np.zeros((len(pool) + 1, 4), np.int32)
tets[1:] = rng.choice(pool, size=(len(pool), 4)); tets[1:, 0] = pool; tets[0] = -1
tr = Transfer(0)
def go(flags):
    tr.upload_background(m, sols, 0, adja=True)
    tr.upload_points(x, t, tets)
    out = []
    for _ in range(2):
        tr.run(flags=flags, record_starts=True)
        r = tr.download()
        out.append((r.steps.copy(), r.elem.copy(), tr.starts().copy()))
    return out
a, b = go(0), go(N.RUN_FRESH_BACKGROUND)
for name, u, v in (("a0 b0", a[0], b[0]), ("a1 b1", a[1], b[1]), ("a0 a1", a[0], a[1]), ("b0 b1", b[0], b[1])):
    d = np.nonzero(u[0] != v[0])[0]
    print(name, "steps differ at", len(d), "points; e.g.", [(int(i), int(t[i]), bool(used[i]), int(u[0][i]), int(v[0][i]), int(u[2][i]), int(v[2][i])) for i in d[:8]])
