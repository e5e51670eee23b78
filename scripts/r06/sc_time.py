#!/usr/bin/env python3
"""Diagnostics: S-C tick-kernel time (HIP events, gm_last_kernel_ms) of the library GM_LIBRARY
names, with no result checks -- for diagnostic builds whose results are wrong on purpose (e.g. list
loads redirected to a cache-resident block to see what the gathers' latency costs)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "distributed-membership_amd"))
from membership import GM_MODE_PARTIAL, Simulator, crash_set  # noqa: E402

n = 1 << 24
sim = Simulator(n, GM_MODE_PARTIAL, rd_seed=7, view=32, view_seed=5, init_mode=1, init_t0=8, init_seed=11,
                drop_pct=5, drop_from=0, drop_to=1 << 20, drop_seed=42)
sim.keep_events(0)
crash = crash_set(n, n // 100, 42)
while sim.time <= 14:
    t = sim.time
    sim.tick()
    if t == 10:
        sim.set_failed(crash)
# no gm_sync (it would latch a diagnostic build's error flags and stop the ticks): the timing
# events' waits are the only host waits
sim.set_timing(1)
sim.tick()
sim.last_kernel_ms()
t0 = time.perf_counter()
for _ in range(10):
    sim.tick()
k = sim.last_kernel_ms()
dt = (time.perf_counter() - t0) / 10
print(f"S-C ms per tick {dt * 1e3:.3f}, tick kernels {k:.3f} ms", flush=True)
