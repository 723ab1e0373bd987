#!/usr/bin/env python3
"""Digest a tools/profile.sh run into a committed profiles/ summary.

  python tools/prof_summary.py gpurun_out/prof_<tag> profiles/<round>_<config>_<tag>

Writes <out>.json (per-kernel average duration from the kernel-trace stats,
per-dispatch PMC averages, HBM traffic per launch) and copies the rocprofv3
kernel stats CSV next to it as <out>_kernel_stats.csv.

HBM traffic per launch follows MI355X_MICROARCH.md section HBM: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts 64 B per 128-B line fetched
-- for wide streaming reads (the guide) and, calibrated by
tools/fetch_calib.hip (profiles/r03_fetch_calib.json), for 8/16/24/32/64/128-B
per-lane gathers alike -- so the read side is doubled ("traffic" = 2*FETCH +
WRITE); the raw sum is kept beside it ("traffic_raw").  Counts from separate --pmc
passes of the same command, averaged over that kernel's dispatches.
"""
import collections
import csv
import json
import os
import shutil
import sys


def short(name: str) -> str:
    n = name.split("(")[0]
    return n.replace("void ", "").strip()


def main():
    src, dst = sys.argv[1], sys.argv[2]
    stats_csv = os.path.join(src, "trace", "run_kernel_stats.csv")
    out = {"source": src, "kernels": {}}
    for r in csv.DictReader(open(stats_csv)):
        out["kernels"][short(r["Name"])] = {"calls": int(r["Calls"]),
                                            "avg_us": float(r["AverageNs"]) / 1e3,
                                            "min_us": float(r["MinNs"]) / 1e3,
                                            "max_us": float(r["MaxNs"]) / 1e3,
                                            "pct": float(r["Percentage"])}
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sorted(os.listdir(src)):
        f = os.path.join(src, d, "run_counter_collection.csv")
        if d.startswith("pmc") and os.path.exists(f):
            for r in csv.DictReader(open(f)):
                pmc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in pmc.items():
        e = out["kernels"].setdefault(k, {})
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        e["pmc"] = avg
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            e["traffic_raw"] = (avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024.0
            e["traffic"] = (2.0 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024.0
            if "avg_us" in e:
                e["traffic_GBs"] = e["traffic"] / (e["avg_us"] * 1e-6) / 1e9
        if "TCC_HIT_sum" in avg:
            h, m = avg["TCC_HIT_sum"], avg.get("TCC_MISS_sum", 0.0)
            e["l2_hit"] = h / max(h + m, 1.0)
        if "SQ_WAVE_CYCLES" in avg:
            wc = max(avg["SQ_WAVE_CYCLES"], 1.0)
            e["wave_share"] = {c: avg[c] / wc for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                                         "SQ_ACTIVE_INST_ANY") if c in avg}
            if "SQ_WAVES" in avg:
                e["valu_per_wave"] = avg.get("SQ_INSTS_VALU", 0) / max(avg["SQ_WAVES"], 1)
                e["vmem_rd_per_wave"] = avg.get("SQ_INSTS_VMEM_RD", 0) / max(avg["SQ_WAVES"], 1)
    log = os.path.join(src, "trace.log")
    if os.path.exists(log):
        for line in open(log):
            if line.startswith("{\"metric\""):
                out["bench"] = json.loads(line)
    with open(dst + ".json", "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    shutil.copy(stats_csv, dst + "_kernel_stats.csv")
    for k in ("k_locate_vol<1>", "k_locate_vol"):
        if k in out["kernels"]:
            e = out["kernels"][k]
            print(k, {x: e.get(x) for x in ("avg_us", "traffic", "traffic_GBs", "l2_hit")})


if __name__ == "__main__":
    main()
