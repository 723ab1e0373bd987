#!/usr/bin/env python3
"""Summary of tools/walk_pmc.sh passes (+ the tools/sweep.py timings of the
same variants): per variant and kernel, physical read bytes (2 x FETCH_SIZE,
the calibration of DESIGN.md section 7 r03), written bytes, L2 hit rate, VALU
instructions per wave, fraction of wave cycles waiting.

  python tools/pmc_ab_summary.py gpurun_out/wpmc_<tag> [gpurun_out/<sweep>.log] > profiles/<out>.json
"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    d = sys.argv[1]
    sweep = None
    if len(sys.argv) > 2:
        s = open(sys.argv[2]).read()
        sweep = json.loads(s[s.index("{"):])["ms(median,min)"]
    variants = sorted({os.path.basename(p).split("_p")[0][1:] for p in glob.glob(os.path.join(d, "v*_p*"))
                       if os.path.isdir(p)}, key=int)
    out = {"source": d, "variants": {}}
    for v in variants:
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for f in glob.glob(os.path.join(d, f"v{v}_p*", "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                k = row["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
                agg[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
        ks = {}
        for k, c in agg.items():
            m = {n: sum(x) / len(x) for n, x in c.items()}
            waves = m.get("SQ_WAVES", 0) or 1
            ks[k] = {"read_GB": 2 * m.get("FETCH_SIZE", 0) * 1024 / 1e9,
                     "write_GB": m.get("WRITE_SIZE", 0) * 1024 / 1e9,
                     "l2_hit": m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
                     if m.get("TCC_HIT_sum") else None,
                     "tcp_tcc_reads": m.get("TCP_TCC_READ_REQ_sum"),
                     "valu_per_wave": m.get("SQ_INSTS_VALU", 0) / waves,
                     "vmem_rd_per_wave": m.get("SQ_INSTS_VMEM_RD", 0) / waves,
                     "wait_frac": m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"] if m.get("SQ_WAVE_CYCLES") else None}
        e = {"kernels": ks}
        if sweep and v in sweep:
            e["ms_median"] = {k: sweep[v][k][0] for k in ("hint", "vol", "bdy", "total")}
        out["variants"][v] = e
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
