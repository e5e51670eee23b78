"""SCALED parity: the HBM-bound HIP tick against the oracle's SCALED restatement.

Per tick: the full membership tables (dump digest), node state and the join /
remove event set, with a crash set and keyed message drops; then size-
independent invariants at a larger N that the oracle cannot finish quickly."""
import numpy as np
import pytest

import oracle_py
from golden_util import digest64, same_state
from membership import GM_EV_JOINED, GM_EV_REMOVED, GM_MODE_SCALED, Simulator, crash_set

pytestmark = pytest.mark.gpu


def run_pair(n, ticks, crash_tick, crash_count, drop_pct=0, drop_from=0, drop_to=0, rd_seed=7, seed=42, seen=None,
             init_mode=0, init_t0=0, band=0):
    init = dict(init_mode=init_mode, init_t0=init_t0, init_seed=seed + 1)
    ora = oracle_py.Oracle(n, oracle_py.OC_SCALED, rd_seed=rd_seed, crash_tick=crash_tick, crash_count=crash_count,
                           crash_seed=seed, drop_pct=drop_pct, drop_from=drop_from, drop_to=drop_to, drop_seed=seed,
                           **init)
    sim = Simulator(n, GM_MODE_SCALED, rd_seed=rd_seed, drop_pct=drop_pct, drop_from=drop_from, drop_to=drop_to,
                    drop_seed=seed, band=band, **init)
    crash = crash_set(n, crash_count, seed)
    assert np.array_equal(crash, oracle_py.crash_set(n, crash_count, seed))
    kinds = {GM_EV_JOINED: 1, GM_EV_REMOVED: 2}
    for _ in range(ticks):
        t = sim.time
        assert ora.time == t
        ora.tick()
        sim.tick()
        if t == crash_tick:
            sim.set_failed(crash)
        ev_g = [(e[0], e[1], kinds[e[2]], e[3]) for e in sim.drain_events()]
        assert ev_g == ora.events(), f"events differ at tick {t}"
        if seen is not None:
            for e in ev_g:
                seen[e[2]] = seen.get(e[2], 0) + 1
        assert same_state(sim, ora), f"tables differ at tick {t}"
    assert digest64(sim.dump_tables()) == digest64(ora.dump()), "text rendering differs"
    st = sim.tick_stats()
    assert st["err"] == 0
    return sim, ora


@pytest.mark.parametrize("n", [64, 300, 1024])
def test_scaled_matches_oracle(n):
    run_pair(n, 40, crash_tick=8, crash_count=max(1, n // 50))


@pytest.mark.parametrize("band", [64, 128, 256, 512, 1024])
def test_scaled_every_band_width_matches_oracle(band):
    # the band width changes only the tiling of gm_s_band / the rank-select of gm_s_pick
    run_pair(700, 36, crash_tick=9, crash_count=9, drop_pct=15, drop_from=4, drop_to=22, init_mode=1, init_t0=7,
             band=band)


@pytest.mark.parametrize("n", [200, 777])
def test_scaled_warm_start_matches_oracle(n):
    run_pair(n, 36, crash_tick=10, crash_count=max(1, n // 100), init_mode=1, init_t0=8)


@pytest.mark.parametrize("n", [128, 513])
def test_scaled_with_drops_matches_oracle(n):
    run_pair(n, 45, crash_tick=10, crash_count=3, drop_pct=20, drop_from=5, drop_to=30)


def test_scaled_heavy_drop_false_removals_match():
    # heavy loss makes entries go stale, get removed and re-join: exercises ADD events
    seen = {}
    run_pair(96, 60, crash_tick=-1, crash_count=0, drop_pct=85, drop_from=2, drop_to=60, seen=seen)
    assert seen.get(1, 0) > 0 and seen.get(2, 0) > 0, seen


@pytest.mark.parametrize("warm", [0, 1])
def test_scaled_invariants_large(warm):
    n, crash_tick, ncrash = 8192, 10, 82
    sim = Simulator(n, GM_MODE_SCALED, rd_seed=7, init_mode=warm, init_t0=8 if warm else 0, init_seed=3)
    crash = crash_set(n, ncrash, 42)
    crashed = np.zeros(n, bool)
    crashed[crash] = True
    removed = 0
    while sim.time <= 45:
        t = sim.time
        sim.tick()
        if t == crash_tick:
            sim.set_failed(crash)
        ev = sim.drain_events()
        for (_, logger, kind, subject) in ev:
            assert kind == GM_EV_REMOVED and crashed[subject - 1] and not crashed[logger]
        removed += len(ev)
    assert removed == (n - ncrash) * ncrash  # every live observer removed every crashed node, nothing else
    st = sim.tick_stats()
    assert st["err"] == 0 and st["live"] == n - ncrash
    for r in [0, 1, 4095, n - 1]:
        if crashed[r]:
            continue
        hb, ts = sim.read_row(r)
        assert np.all(hb[crashed] == -1)
        assert np.all(hb[~crashed] >= 0)
        assert np.all(sim.time - 1 - ts[~crashed] < 20)  # present => younger than TREMOVE


def _escaped_sends(dump, t):
    """Fresh entries of live rows whose payload value h' = 253 - 2t + hb falls outside the
    nibble range (h' < 226): sent through the escape plane at tick t (gm_scaled.h S_NIB_*)."""
    esc = 0
    for line in dump.decode().splitlines():
        f = line.split()
        if int(f[4]):
            continue
        for x in f[7:]:
            _, hb, ts = map(int, x.split(":"))
            esc += t - ts < 5 and 2 * t - hb > 27
    return esc


def test_scaled_escaped_payloads_match_oracle():
    # 80 % loss for ticks 6..23 lets fresh entries carry heartbeats more than 13 ticks old;
    # after the window the loss-free merge (nibble max + escape plane) must take them exactly
    n = 600
    kw = dict(rd_seed=7, drop_pct=80, drop_from=6, drop_to=24, drop_seed=42, init_mode=1, init_t0=5, init_seed=43)
    ora = oracle_py.Oracle(n, oracle_py.OC_SCALED, crash_tick=9, crash_count=6, crash_seed=42, **kw)
    sim = Simulator(n, GM_MODE_SCALED, **kw)
    crash = crash_set(n, 6, 42)
    kinds = {GM_EV_JOINED: 1, GM_EV_REMOVED: 2}
    esc_after_window = 0
    for _ in range(36):
        t = sim.time
        ora.tick()
        sim.tick()
        if t == 9:
            sim.set_failed(crash)
        assert [(e[0], e[1], kinds[e[2]], e[3]) for e in sim.drain_events()] == ora.events(), f"events t={t}"
        d = ora.dump()
        assert digest64(sim.dump_tables()) == digest64(d), f"tables differ at tick {t}"
        if t >= 24:
            esc_after_window += _escaped_sends(d, t)
    assert esc_after_window > 0  # the escape plane really carried loss-free deliveries
    assert sim.tick_stats()["err"] == 0


@pytest.mark.parametrize("drop", [0, 20])
def test_oracle_continues_from_gpu_state(drop):
    """The whole SCALED state between two ticks, read from the HIP path (gm_read_table,
    gm_read_nodes, gm_read_targets), loaded into the oracle (oc_load_scaled): the oracle's next
    ticks equal the HIP path's, events and tables. This is the hand-over scripts/cpu_hour.py uses
    to time a long CPU run in segments that start where the GPU got in seconds."""
    n = 300
    kw = dict(rd_seed=7, init_mode=1, init_t0=8, init_seed=11, drop_pct=drop, drop_from=0, drop_to=1000, drop_seed=5)
    sim = Simulator(n, GM_MODE_SCALED, **kw)
    crash = crash_set(n, 9, 42)
    while sim.time <= 24:
        t = sim.time
        sim.tick()
        if t == 10:
            sim.set_failed(crash)
    sim.drain_events()
    hb, ts = sim.read_table()
    st = sim.read_nodes()
    tg, cnt = sim.read_targets()
    ora = oracle_py.Oracle(n, oracle_py.OC_SCALED, crash_tick=10, crash_count=9, crash_seed=42, **kw)
    ora.load_state(sim.time, hb, ts, st[:, 3], st[:, 2], tg, cnt)
    assert digest64(ora.dump()) == digest64(sim.dump_tables())
    for _ in range(14):
        t = sim.time
        sim.tick()
        ora.tick()
        assert [(e[0], e[1], e[2], e[3]) for e in sim.drain_events()] == ora.events(), f"events t={t}"
        assert digest64(sim.dump_tables()) == digest64(ora.dump()), f"tables t={t}"
