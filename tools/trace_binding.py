"""The bench's binding cycle alone (integration/pmmg_pmx.c's two seams on
Mmg-shaped AoS records), with the library's host phase trace (PMX_TRACE=1).
    python tools/trace_binding.py [C3|C2] [iters]
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
    r = bench.binding_cycle(m, x, t, tv, sols, 0, iters=iters)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
