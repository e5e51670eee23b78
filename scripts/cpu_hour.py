#!/usr/bin/env python3
"""north_star's CPU reference run, measured rather than extrapolated: the single-threaded SCALED
restatement (oracle/ref_cpu.c, the reference's MP1Node tick per node) for 100 consecutive ticks at
one N, with the S-A schedule (warm start at t0 = 8, 1 % of the nodes crashed at tick 10). Writes
one JSON line per tick to --out (elapsed so far) so a long run can be read while it goes, and a
final summary line. Test/measurement infrastructure only: it times the oracle, never libgm.

Segments (--start T, --ticks K): a GPU call on the pool is capped at 1,200 s, so the hour-sized run
is timed in segments. A segment gets the state before tick T from the HIP path (the SCALED tick is
bit-exact to the oracle: tests/test_gpu_scaled.py::test_oracle_continues_from_gpu_state) in
seconds, loads it into the oracle (oc_load_scaled) and times ticks T .. T+K-1 on one host core.
The per-tick times of consecutive segments add up to the continuous run's (the state at every
tick boundary is the same)."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "distributed-membership_amd"))

import oracle_py  # noqa: E402


def gpu_state(n, start, kw, ncrash):
    """(hb, ts, heartbeat, failed, targets, counts) before tick `start`, from the HIP path"""
    from membership import GM_MODE_SCALED, Simulator, crash_set
    sim = Simulator(n, GM_MODE_SCALED, rd_seed=kw["rd_seed"], init_mode=1, init_t0=kw["init_t0"],
                    init_seed=kw["init_seed"])
    sim.keep_events(0)
    crash = crash_set(n, ncrash, kw["crash_seed"])
    while sim.time < start:
        t = sim.time
        sim.tick()
        if t == kw["crash_tick"]:
            sim.set_failed(crash)
    hb, ts = sim.read_table()
    st = sim.read_nodes()
    tg, cnt = sim.read_targets()
    assert sim.tick_stats()["err"] == 0
    sim.close()
    return hb, ts, st[:, 3].copy(), st[:, 2].copy(), tg, cnt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cluster", type=int, default=13722)
    ap.add_argument("--ticks", type=int, default=100)
    ap.add_argument("--start", type=int, default=0, help="first timed tick (0: from the warm start, t0 + 1)")
    ap.add_argument("--out", default="-")
    a = ap.parse_args()
    out = sys.stdout if a.out == "-" else open(a.out, "a")
    n = a.cluster
    ncrash = int(round(n * 0.01))
    kw = dict(rd_seed=7, init_mode=1, init_t0=8, init_seed=11, crash_tick=10, crash_count=ncrash, crash_seed=42)
    t_build = time.perf_counter()
    o = oracle_py.Oracle(n, oracle_py.OC_SCALED, **kw)
    src = "oracle warm start"
    if a.start > o.time:
        state = gpu_state(n, a.start, kw, ncrash)
        o.load_state(a.start, *state)
        del state
        src = f"HIP-path state before tick {a.start} (gm_read_table / gm_read_nodes / gm_read_targets)"
    build_s = time.perf_counter() - t_build
    out.write(json.dumps({"segment": True, "n": n, "first_tick": o.time, "ticks": a.ticks, "state": src,
                          "setup_s": round(build_s, 1)}) + "\n")
    out.flush()
    t0 = time.perf_counter()
    for k in range(a.ticks):
        w = time.perf_counter()
        o.tick()
        now = time.perf_counter()
        out.write(json.dumps({"tick": o.time - 1, "s": round(now - w, 3), "elapsed_s": round(now - t0, 1)}) + "\n")
        out.flush()
    el = time.perf_counter() - t0
    out.write(json.dumps({"summary": True, "n": n, "first_tick": o.time - a.ticks, "ticks": a.ticks, "seconds": el,
                          "setup_s": build_s, "node_ticks_per_s": n * a.ticks / el, "cores": 1,
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
