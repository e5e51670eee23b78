#!/usr/bin/env python3
"""Diagnostics: per-tick gm_s_band time (HIP events) through the S-A schedule -- which ticks
(steady, crash-window escapes, TREMOVE removals) cost what. usage: tick_times.py [n] [ticks]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "distributed-membership_amd"))
from membership import GM_MODE_SCALED, Simulator, crash_set  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
last = int(sys.argv[2]) if len(sys.argv) > 2 else 48
sim = Simulator(n, GM_MODE_SCALED, rd_seed=7, init_mode=1, init_t0=8, init_seed=11)
sim.keep_events(0)
crash = crash_set(n, int(round(n * 0.01)), 42)
while sim.time <= last:
    t = sim.time
    sim.set_timing(1)
    sim.tick()
    sim.sync()
    print(f"t={t:3d} band {sim.last_kernel_ms():8.3f} ms  events {sim.event_counts()[0]}", flush=True)
    if t == 10:
        sim.set_failed(crash)
