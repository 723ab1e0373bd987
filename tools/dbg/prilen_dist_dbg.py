"""Debug: the distributed tensor prilen case of test_distributed_prilen_tensor_surface."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
from helpers import cube_surface, split_partitions
from parmmg_amd import mesh as M
from parmmg_amd.transfer import Transfer
from oracle import oracle as O
full = M.kuhn_cube(7)
parts, nshared = split_partitions(full)
rng = np.random.default_rng(8)
tr = Transfer(0)
for rank, (mr, glob, par) in enumerate(parts):
    tags, surf, met = cube_surface(mr, noise=0.08, seed=rank + 1)
    met = np.abs(met) * 0.01 + 1e-3
    met[0] = 1.0
    ptag = np.where(rng.random(len(par["a"])) < 0.3, 2, 0).astype(np.uint16)
    p = dict(par, myrank=rank, owner=np.zeros(len(par["a"]), np.int32), exact_once=0, tag=ptag)
    tr.upload_background(mr, [met], 0)
    tr.upload_point_tags(tags)
    tr.upload_surface(surf)
    for mrt in (0, 1):
        for pp in (p, None):
            L = tr.prilen(met_rid_typ=mrt, par=pp)
            Lo = O.prilen(mr, met, tags=tags, par=pp, met_rid_typ=mrt, surface=surf)
            print(rank, mrt, pp is not None)
            print("  dev", {k: L[k] for k in ("ned", "nullEdge", "lmin", "amin", "bmin", "lmax", "amax", "bmax", "avlen")}, L["hl"])
            print("  orc", {k: Lo[k] for k in ("ned", "nullEdge", "lmin", "amin", "bmin", "lmax", "amax", "bmax", "avlen")}, Lo["hl"])
