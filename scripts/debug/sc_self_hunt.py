"""Diagnostics for an intermittent GM_ERR_SELF seen once in the full-size S-C test: runs the
test's single-context configuration (optionally after an S-B context, as in the gate's test order),
and after every tick reads every view and reports the first rows whose list lacks the node itself,
together with the tick and the err word. usage: sc_self_hunt.py [reps] [sb_first]"""
import sys
import time

import numpy as np

from membership import GM_MODE_PARTIAL, GM_MODE_SCALED, Simulator, crash_set


def scan(sim, n, t, chunk=1 << 21):
    bad = []
    for r0 in range(0, n, chunk):
        v = sim.read_views(r0, min(chunk, n - r0))
        ids = (v >> np.uint64(32)).astype(np.int64)
        rows = np.arange(r0, r0 + v.shape[0], dtype=np.int64) + 1
        miss = ~(ids == rows[:, None]).any(axis=1)
        for r in np.nonzero(miss)[0][:4]:
            bad.append((r0 + int(r), v[r].tolist()))
    return bad


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    sb_first = len(sys.argv) > 2 and sys.argv[2] == "1"
    n, v = 1 << 24, 32
    kw = dict(rd_seed=7, view=v, view_seed=5, init_mode=1, init_t0=8, init_seed=11, drop_pct=5, drop_from=0,
              drop_to=1 << 20, drop_seed=42)
    crash = crash_set(n, int(round(n * 0.01)), 42)
    if sb_first:
        t0 = time.time()
        sb = Simulator(262144, GM_MODE_SCALED, rd_seed=7, init_mode=1, init_t0=8, init_seed=11)
        for _ in range(12):
            sb.tick()
        print("sb ticks done", sb.tick_stats(), f"{time.time() - t0:.1f}s", flush=True)
        sb.close()
        del sb
    for rep in range(reps):
        ref = Simulator(n, GM_MODE_PARTIAL, **kw)
        ref.keep_events(0)
        first = None
        while ref.time <= 30:
            t = ref.time
            ref.tick()
            if t == 10:
                ref.set_failed(crash)
            st = ref.tick_stats()
            bad = scan(ref, n, t)
            print(f"rep {rep} t={t} err={st['err']} self-missing rows={len(bad)}", flush=True)
            if bad and first is None:
                first = t
                for r, row in bad[:8]:
                    print("  row", r, "view", [(x >> 32, x & 0xFFFFFFFF) for x in row], flush=True)
            if st["err"] and first is None:
                first = t
        ref.close()
        del ref
        print(f"rep {rep}: first bad tick {first}", flush=True)


if __name__ == "__main__":
    main()
