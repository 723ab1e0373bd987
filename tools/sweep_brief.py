#!/usr/bin/env python3
"""One line per variant of a tools/sweep.py log and per bench.py line.

  python tools/sweep_brief.py gpurun_out/sw3.log gpurun_out/bench.log ...
"""
import json
import sys

for f in sys.argv[1:]:
    s = open(f).read()
    if '"ms(median,min)"' in s:
        d = json.loads(s[s.index("{"):])
        for k, v in d["ms(median,min)"].items():
            print(f, d["opt"], k, {kk: (round(vv[0], 4) if isinstance(vv, list) else vv) for kk, vv in v.items()})
        continue
    for line in s.splitlines():
        if line.startswith("{"):
            d = json.loads(line)
            rf = d.get("roofline") or {}
            print(f, d["config"]["workload"][:3], "%.3e" % d["value"], "ms/step %.4f" % d["ms_per_step"],
                  {k: round(v, 4) for k, v in d["kernel_ms"].items()}, "frac", rf.get("frac"))
