#!/usr/bin/env python3
"""north_star's CPU reference run, measured rather than extrapolated: the single-threaded SCALED
restatement (oracle/ref_cpu.c, the reference's MP1Node tick per node) for 100 consecutive ticks at
one N, with the S-A schedule (warm start at t0 = 8, 1 % of the nodes crashed at tick 10). Writes
one JSON line per tick to --out (elapsed so far) so a long run can be read while it goes, and a
final summary line. Test/measurement infrastructure only: it runs the oracle, never libgm."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))

import oracle_py  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cluster", type=int, default=13722)
    ap.add_argument("--ticks", type=int, default=100)
    ap.add_argument("--out", default="-")
    a = ap.parse_args()
    out = sys.stdout if a.out == "-" else open(a.out, "w")
    n = a.cluster
    t_build = time.perf_counter()
    o = oracle_py.Oracle(n, oracle_py.OC_SCALED, rd_seed=7, init_mode=1, init_t0=8, init_seed=11,
                         crash_tick=10, crash_count=int(round(n * 0.01)), crash_seed=42)
    build_s = time.perf_counter() - t_build
    t0 = time.perf_counter()
    for k in range(a.ticks):
        w = time.perf_counter()
        o.tick()
        now = time.perf_counter()
        out.write(json.dumps({"tick": o.time - 1, "s": round(now - w, 3), "elapsed_s": round(now - t0, 1)}) + "\n")
        out.flush()
    el = time.perf_counter() - t0
    out.write(json.dumps({"summary": True, "n": n, "ticks": a.ticks, "seconds": el, "setup_s": build_s,
                          "node_ticks_per_s": n * a.ticks / el, "cores": 1,
                          "host": os.uname().nodename, "cpu": _cpu_model()}) + "\n")
    out.flush()


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


if __name__ == "__main__":
    main()
