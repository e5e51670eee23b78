#!/usr/bin/env python3
"""Diagnostics: distribution of a present cell's heartbeat lag split as lag = L0 + age (L0 = the
lag its heartbeat had when it was last raised, constant while the entry ages) through the S-A
schedule -- which byte code ranges the stored cells need. usage: lag_hist.py [n] [rows]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "distributed-membership_amd"))
from membership import GM_MODE_SCALED, Simulator, crash_set  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 256
sim = Simulator(n, GM_MODE_SCALED, rd_seed=7, init_mode=1, init_t0=8, init_seed=11)
sim.keep_events(0)
crash = crash_set(n, int(round(n * 0.01)), 42)
crashed = np.zeros(n, bool)
crashed[crash] = True
r0 = n // 3
while sim.time <= 48:
    t = sim.time
    sim.tick()
    if t == 10:
        sim.set_failed(crash)
    if t in (9, 12, 16, 20, 24, 28, 32, 36, 40, 44, 48):
        hb, ts = sim.read_table(r0, rows)
        live_rows = ~crashed[r0:r0 + rows]
        hb, ts = hb[live_rows], ts[live_rows]
        pres = hb >= 0
        lag = (2 * t - 1 - hb) // 2
        age = t - ts
        l0 = lag - age
        for name, sel in (("live", pres & ~crashed[None, :]), ("crashed", pres & crashed[None, :])):
            if not sel.any():
                print(f"t={t} {name}: none", flush=True)
                continue
            lh = np.bincount(np.clip(l0[sel], -1, 30) + 1)
            ah = np.bincount(age[sel])
            print(f"t={t} {name}: cells {sel.sum()} L0 min {l0[sel].min()} max {l0[sel].max()} "
                  f"hist(L0=-1..) {lh.tolist()} age max {age[sel].max()} hist {ah.tolist()} "
                  f"even hb {(hb[sel] % 2 == 0).sum()}", flush=True)
