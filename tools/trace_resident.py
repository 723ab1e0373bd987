"""The bench's resident cycle alone, with the library's host phase trace
(PMX_TRACE=1: per-call phase timings on stderr).  Usage:
    python tools/trace_resident.py [C3|C2] [iters]
"""
import os
import sys

os.environ.setdefault("PMX_TRACE", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import json  # noqa: E402

import bench  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "C3"
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    cfg = bench.CONFIGS[name]
    m, x, t, sols, tv = bench.build_case(cfg, 0)
    r = bench.resident_cycle(m, sols, cfg, 0, iters=iters, warmup=1)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
