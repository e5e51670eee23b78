"""SCALED join ramp: the full membership lifecycle at scale
instead of a converged start. Node i starts at tick (int)(0.25 i) (Application.cpp:130),
sends JOINREQ to the introducer, which adds it (hb 0), gossips to this tick's joiners
first (newNodes, MP1Node.cpp:458) and answers with JOINREP (MP1Node.cpp:226-251); the
joiner is in the group two ticks after its start. The HIP band/pick kernels (narrow
cells with a per-column heartbeat offset) against the oracle (oracle/ref_cpu.c SCALED,
init_mode 2), tick by tick: every table, node state (inited / inGroup / failed /
heartbeat) and the join/remove event set -- through the ramp, a crash set that hits
nodes before they start (nodeStart revives them, MP1Node.cpp:108), and the introducer
crashing mid-ramp (later starters never join)."""
import pytest

import oracle_py
from golden_util import digest64, same_state
from membership import GM_MODE_SCALED, Simulator, crash_set

pytestmark = pytest.mark.gpu


def seed_with(n, count, want):
    """a crash seed whose set contains `want` (node 0: the introducer)"""
    for seed in range(1, 10000):
        if want in set(crash_set(n, count, seed).tolist()):
            return seed
    raise AssertionError("no seed")


def run_ramp(n, ticks, crash_tick=-1, crash_count=0, crash_seed=42, band=0, drop_pct=0, every=1, ora_out=None):
    drops = dict(drop_pct=drop_pct, drop_from=0, drop_to=1 << 20, drop_seed=42)
    ora = oracle_py.Oracle(n, oracle_py.OC_SCALED, rd_seed=7, crash_tick=crash_tick, crash_count=crash_count,
                           crash_seed=crash_seed, init_mode=2, **drops)
    sim = Simulator(n, GM_MODE_SCALED, rd_seed=7, init_mode=2, band=band, **drops)
    if ora_out is not None:
        ora_out.append(ora)
    crash = crash_set(n, crash_count, crash_seed)
    ora.tick()  # tick 0: nodeStart of nodes 0-3 (the GPU context starts as of tick 0)
    assert sim.time == ora.time == 1
    assert digest64(sim.dump_tables()) == digest64(ora.dump()), "tick 0 state differs"
    joins = removes = 0
    for _ in range(ticks):
        t = sim.time
        ora.tick()
        sim.tick()
        if t == crash_tick:
            sim.set_failed(crash)
        ev = sim.drain_events()
        assert ev == ora.events(), f"events differ at tick {t}"
        joins += sum(e[2] == 1 for e in ev)
        removes += sum(e[2] == 2 for e in ev)
        if t % every == 0 or sim.time > ticks:
            assert same_state(sim, ora), f"tables differ at tick {t}"
    assert digest64(sim.dump_tables()) == digest64(ora.dump()), "final tables differ"
    assert sim.tick_stats()["err"] == 0
    return joins, removes


@pytest.mark.parametrize("n,band", [(64, 64), (300, 128), (1100, 0)])
def test_ramp_matches_oracle(n, band):
    joins, _ = run_ramp(n, n // 4 + 30, band=band)
    assert joins >= n * (n - 1)  # everyone learned everyone (plus re-joins)


def test_ramp_crash_before_start_and_removals():
    # crash at tick 20 of a 400-node ramp (starts run to tick 99): crashed starters revive
    joins, removes = run_ramp(400, 140, crash_tick=20, crash_count=40)
    assert removes > 0


def test_ramp_introducer_crash():
    n, cnt = 256, 8
    joins, removes = run_ramp(n, 110, crash_tick=30, crash_count=cnt, crash_seed=seed_with(n, cnt, 0))
    assert removes > 0


def test_ramp_at_scale_converges():
    """N = 16,384: the whole 4,096-tick ramp on the GPU (no oracle at this size; size-
    independent properties instead): every node joins, every live node ends up holding
    every node exactly once (n entries), each join event is logged once per (observer,
    subject) pair and nobody is removed in a crash-free run."""
    import numpy as np
    n = 16384
    sim = Simulator(n, GM_MODE_SCALED, rd_seed=7, init_mode=2)
    sim.keep_events(0)  # n^2 join records: counted on the device (gm_event_totals), not staged
    last = n // 4 + 40
    while sim.time <= last:
        sim.tick()
    tot = sim.event_totals()
    joins, removes = tot["joined"], tot["removed"]
    st = sim.tick_stats()
    assert st["err"] == 0 and st["live"] == n
    nodes = sim.read_nodes()
    assert (nodes[:, 0] == 1).all() and (nodes[:, 1] == 1).all()
    for r in (0, 1, n // 2, n - 1):  # spot rows: everyone present
        hb, ts = sim.read_row(r)
        assert (hb >= 0).all(), r
    assert removes == 0
    assert joins == n * n - 1  # everyone learns everyone (incl. itself); the introducer's own entry is not a join


@pytest.mark.parametrize("n,drop,band,every", [(300, 50, 128, 1), (1100, 10, 0, 4)])
def test_ramp_with_drops_matches_oracle(n, drop, band, every):
    """Keyed drops during the ramp: joiners miss their own entry in the lists they merge, so
    updateMyPos (MP1Node.cpp:308-322) takes the `&&` quirk -- the next larger id present takes
    the heartbeat and timestamp, and that id counts as "me" in the gossip draw (:459-470)."""
    keep = []
    joins, _ = run_ramp(n, n // 4 + 30, band=band, drop_pct=drop, every=every, ora_out=keep)
    fired, gap = keep[0].quirks()
    assert fired > 0 and gap == 0, (fired, gap)
    assert joins > 0


def test_ramp_with_drops_at_scale():
    """N = 16,384 ramp under 10 % keyed drops (no oracle at this size): the quirk path never
    meets a case the narrow cell cannot hold (err stays 0: gm_s_selfcheck, GM_ERR_LAG), and
    every node ends up in the group."""
    n = 16384
    sim = Simulator(n, GM_MODE_SCALED, rd_seed=7, init_mode=2, drop_pct=10, drop_from=0, drop_to=1 << 20,
                    drop_seed=42)
    sim.keep_events(0)
    while sim.time <= n // 4 + 40:
        sim.tick()
    st = sim.tick_stats()
    assert st["err"] == 0 and st["live"] == n
    nodes = sim.read_nodes()
    assert (nodes[:, 0] == 1).all() and (nodes[:, 1] == 1).all()
    assert sim.event_totals()["joined"] >= n * (n - 1)  # every other node joined (self may be appended, unlogged)
    for r in (0, 1, n // 2, n - 1):  # spot rows: everyone present
        hb, ts = sim.read_row(r)
        assert (hb >= 0).all(), r


@pytest.mark.parametrize("case", ["singlefailure_T1_R1", "multifailure_T42_R7", "n20_single", "n70_single"])
def test_ramp_equals_reference_fixtures(case):
    """HIP SCALED join ramp vs the seeded reference itself (no oracle in between): with no drops and
    N < 78 (EmulNet's buffer never fills) every tick's tables equal the golden FAITHFUL digests and
    the events the golden dbg.log's join/remove lines (tests/test_oracle_scaled_pin.py)."""
    from golden_util import load_case, parse_conf
    from test_oracle_scaled_pin import _canon, _parse_dbg

    m = load_case(case)
    n, _single, drop, _p = parse_conf(m["conf"])
    assert not drop
    ev, fails = _parse_dbg(m["dbg"])
    sim = Simulator(n, GM_MODE_SCALED, rd_seed=m["rd_seed"], init_mode=2)
    assert sim.time == 1  # the context starts as of tick 0
    assert digest64(sim.dump_tables()) == int(m["tick_digests"][0])
    for t in range(1, m["ticks"]):
        sim.tick()
        if fails.get(t):
            sim.set_failed(fails[t])
        got = [(e[1], e[2], e[3]) for e in sim.drain_events()]
        assert got == _canon(ev.get(t, [])), f"{case}: events differ at t={t}"
        assert digest64(sim.dump_tables()) == int(m["tick_digests"][t]), f"{case}: tables differ at t={t}"
    assert sim.tick_stats()["err"] == 0
