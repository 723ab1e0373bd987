#!/usr/bin/env python3
"""Host-staged phases of one group at a bench config (wall clock, best of reps):
points upload with / without the new tets, the tets alone, the step, the
download (fields only / everything), the promotion of the new mesh to the next
background (Mmg adjacency uploaded / built on the device).

  python tools/bench_upload.py [--config C2] [--reps 5]
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
    ap.add_argument("--config", default="C2")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import numpy as np
    import bench
    from parmmg_amd import mesh as M
    from parmmg_amd.transfer import Transfer
    cfg = bench.CONFIGS[args.config]
    m, _, _, sols, _ = bench.build_case(cfg, 0)
    mb = M.kuhn_cube(cfg["n"], seed=777)
    x = mb.xyz[1:]
    onb = np.any((x == 0.0) | (x == 1.0), axis=1)
    t = np.where(onb, M.TAG_BDY, 0).astype(np.uint16)
    tets1 = mb.tet                    # Mmg layout, passed as is
    tr = Transfer(0)
    tr.upload_background(m, sols, 0)
    out = {}

    def best(name, fn, pre=None):
        ts = []
        for _ in range(args.reps):
            if pre:
                pre()
            tr.synchronize()
            t0 = time.perf_counter()
            fn()
            tr.synchronize()
            ts.append(time.perf_counter() - t0)
        out[name] = min(ts) * 1e3
        print(name, round(out[name], 3), "ms", flush=True)

    best("upload_points", lambda: tr.upload_points(x, t))
    best("upload_points_with_tets", lambda: tr.upload_points(x, t, tets_mmg=tets1))
    best("run", lambda: tr.run())
    r = tr.download()
    best("download_all", lambda: tr.download(into=r))
    best("download_sols", lambda: tr.download(into=r, sols_only=True))

    def reset():
        tr.upload_background(m, sols, 0)
        tr.upload_points(x, t, tets_mmg=tets1)
        tr.run()
        tr.download(into=r, sols_only=True)
    best("promote_adja_host", lambda: tr.promote_background(mb, r.sols), pre=reset)
    best("promote_adja_device", lambda: tr.promote_background(mb, r.sols, adja=False), pre=reset)
    tr.set_residency(True)
    best("upload_points_with_tets_residency", lambda: tr.upload_points(x, t, tets_mmg=tets1))
    best("promote_prepared", lambda: tr.promote_background(mb, r.sols, adja=False), pre=reset)
    best("upload_background_full", lambda: tr.upload_background(m, sols, 0))
    out["config"] = args.config
    out["ne"], out["np_new"] = int(mb.ne), int(len(x))
    print(json.dumps(out), flush=True)
    tr.close()


if __name__ == "__main__":
    main()
