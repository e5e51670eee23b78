"""The BASELINE.json configurations that fit one GPU, at their full sizes, through
size-independent properties (the oracle cannot finish these sizes in seconds):

* S-A (configs[2]): N = 65,536 full membership, warm start, 1 % crash at tick 10 --
  exactly bench.py's schedule. Every live observer removes every crashed node exactly
  once (the TREMOVE sweep, /root/reference/MP1Node.cpp:429-444) and nothing else.
* S-B (configs[3]) on ONE GPU: N = 262,144, the same schedule (2,621 crashed nodes) -- the
  1-GPU point of the strong-scaling curve. 1 B of table + 1 B of payload nibbles per cell
  (137 GB) plus the bounded escape pools (gm_scaled.h) fit one 288 GB MI355X.
* S-C (configs[4], one GPU): N = 16,777,216, V = 32 partial views, 5 % keyed drops on
  every tick, 1 % crash at tick 10 -- bench.py --scenario S-C's schedule. Views stay
  full, id-sorted, self-present and fresh; crashed nodes leave every live view.

Plus the event-drain contract: records of several ticks survive until
drained, and the device-side cumulative counters agree with the drains."""
import numpy as np
import pytest

import oracle_py
from membership import GM_EV_JOINED, GM_EV_REMOVED, GM_MODE_PARTIAL, GM_MODE_SCALED, Simulator, crash_set

pytestmark = pytest.mark.gpu

TFAIL, TREMOVE = 5, 20


def test_sb_config_on_one_gpu_removes_exactly_the_crashed_nodes():
    n, crash_tick = 262144, 10
    ncrash = int(round(n * 0.01))
    sim = Simulator(n, GM_MODE_SCALED, rd_seed=7, init_mode=1, init_t0=8, init_seed=11)
    sim.keep_events(0)  # 687 M removal records: counted on the device (event totals), not staged
    crash = crash_set(n, ncrash, 42)
    while sim.time <= 48:
        t = sim.time
        sim.tick()
        if t == crash_tick:
            sim.set_failed(crash)
    sim.sync()
    st = sim.tick_stats()
    assert st["err"] == 0 and st["live"] == n - ncrash
    assert st["lists"] == 5 * (n - ncrash)
    tot = sim.event_totals()
    assert tot["removed"] == (n - ncrash) * ncrash and tot["joined"] == 0, tot
    crashed = np.zeros(n, bool)
    crashed[crash] = True
    t = sim.time - 1
    for r in (0, n // 2 + 1, n - 1):
        if crashed[r]:
            continue
        hb, ts = sim.read_row(r)
        assert np.all(hb[crashed] == -1) and np.all(hb[~crashed] >= 0)
        assert np.all(t - ts[~crashed] < TREMOVE)
        assert hb[r] == 2 * t - 1 and ts[r] == t
    sim.close()


def test_sa_bench_config_removes_exactly_the_crashed_nodes():
    n, crash_tick, ncrash = 65536, 10, 655
    sim = Simulator(n, GM_MODE_SCALED, rd_seed=7, init_mode=1, init_t0=8, init_seed=11)
    crash = crash_set(n, ncrash, 42)
    crashed = np.zeros(n + 1, bool)  # by node id
    crashed[crash + 1] = True
    live_idx = np.flatnonzero(~crashed[1:])
    n_live = n - ncrash
    per_subject = np.zeros(n + 1, np.int64)
    pairs = []
    last = 48  # bench.py: prologue to tick 25, 3 warmup + 20 timed ticks
    while sim.time <= last:
        t = sim.time
        sim.tick()
        if t == crash_tick:
            sim.set_failed(crash)
        ev = sim.drain_events_np()
        if len(ev):
            assert np.all(ev[:, 0] == t)
            assert np.all(ev[:, 2] == GM_EV_REMOVED), "a join in a converged cluster without drops"
            assert t >= crash_tick + TREMOVE, f"removal before TREMOVE at tick {t}"
            assert np.all(crashed[ev[:, 3]]), "a live node was removed"
            assert not np.any(crashed[ev[:, 1] + 1]), "a crashed node logged"
            per_subject += np.bincount(ev[:, 3], minlength=n + 1)
            pairs.append(ev[:, 1].astype(np.int64) * (n + 1) + ev[:, 3])
    allp = np.concatenate(pairs)
    assert len(allp) == n_live * ncrash
    assert len(np.unique(allp)) == len(allp), "an observer removed a node twice"
    assert np.all(per_subject[crash + 1] == n_live)
    tot = sim.event_totals()
    assert tot["removed"] == n_live * ncrash and tot["joined"] == 0, tot
    st = sim.tick_stats()
    assert st["err"] == 0 and st["live"] == n_live
    assert st["lists"] == 5 * n_live  # every live node gossips to 5 live targets once the crashed are gone
    t = sim.time - 1
    for r in [int(live_idx[0]), int(live_idx[len(live_idx) // 2]), int(live_idx[-1])]:
        hb, ts = sim.read_row(r)
        assert np.all(hb[crashed[1:]] == -1)
        assert np.all(hb[~crashed[1:]] >= 0)
        assert np.all(t - ts[~crashed[1:]] < TREMOVE)
        assert hb[r] == 2 * t - 1 and ts[r] == t  # own entry: heartbeat 2k-1 at the k-th nodeLoopOps


def _check_views(views, r0, t, crashed_id, v, after_crash):
    ids = (views >> np.uint64(32)).astype(np.int64)
    hb = (views & np.uint64(0xFFFFFFFF)).astype(np.int64)
    rows = np.arange(r0, r0 + len(views))
    live = ~crashed_id[rows + 1]
    ids, hb, rows = ids[live], hb[live], rows[live]
    assert np.all(ids > 0), "a live view is not full"
    assert np.all(np.diff(ids, axis=1) > 0), "a view is not strictly id-sorted"
    own = ids == (rows + 1)[:, None]
    assert np.all(own.sum(axis=1) == 1), "self missing from a view"
    assert np.all(hb[own] == 2 * t - 1)
    ts = (hb + 1) // 2
    assert np.all(t - ts < TREMOVE)
    if after_crash:
        assert not np.any(crashed_id[ids]), "a crashed node is still in a live view"
    assert ids.shape[1] == v


def test_sc_bench_config_views_stay_consistent():
    n, v, crash_tick = 1 << 24, 32, 10
    ncrash = int(round(n * 0.01))
    sim = Simulator(n, GM_MODE_PARTIAL, rd_seed=7, view=v, view_seed=5, init_mode=1, init_t0=8, init_seed=11,
                    drop_pct=5, drop_from=0, drop_to=1 << 20, drop_seed=42)
    sim.keep_events(0)  # ~24 view joins per node and tick: count them, do not stage them
    crash = crash_set(n, ncrash, 42)
    crashed_id = np.zeros(n + 1, bool)
    crashed_id[crash + 1] = True
    joins = 0
    while sim.time <= 36:
        t = sim.time
        sim.tick()
        if t == crash_tick:
            sim.set_failed(crash)
        c = sim.event_counts()
        assert c[GM_EV_REMOVED] == 0, f"removal at tick {t}: eviction keeps views fresh"
        joins += c[GM_EV_JOINED]
        if t in (12, 36):
            for r0 in (0, n // 2, n - (1 << 19)):
                _check_views(sim.read_views(r0, 1 << 19), r0, t, crashed_id, v, after_crash=t > crash_tick + TFAIL)
    st = sim.tick_stats()
    assert st["err"] == 0 and st["live"] == n - ncrash
    assert 4 * (n - ncrash) < st["lists"] <= 5 * (n - ncrash)  # 5 targets per live node, 5 % of lists... none lost
    assert joins > 0


@pytest.mark.parametrize("mode", [GM_MODE_SCALED, GM_MODE_PARTIAL])
def test_events_of_several_ticks_survive_until_drained(mode):
    n = 300
    crash_tick = 8 if mode == GM_MODE_SCALED else 12  # inside the window (first ticks 7 / 9)
    if mode == GM_MODE_SCALED:
        kw = dict(rd_seed=7, drop_pct=40, drop_from=3, drop_to=30, drop_seed=42, init_mode=1, init_t0=6, init_seed=43)
        ora = oracle_py.Oracle(n, oracle_py.OC_SCALED, crash_tick=crash_tick, crash_count=6, crash_seed=42, **kw)
        sim = Simulator(n, GM_MODE_SCALED, **kw)
    else:
        kw = dict(rd_seed=7, view_seed=5, init_t0=8, init_seed=11, drop_pct=10, drop_from=0, drop_to=100,
                  drop_seed=42)
        ora = oracle_py.PartialOracle(n, v=16, crash_tick=crash_tick, crash_count=6, crash_seed=42, **kw)
        sim = Simulator(n, GM_MODE_PARTIAL, view=16, init_mode=1, **kw)
    crash = crash_set(n, 6, 42)
    want = []
    kinds = {GM_EV_JOINED: 1, GM_EV_REMOVED: 2}
    for step in range(30):
        t = sim.time
        ora.tick()
        sim.tick()
        if t == crash_tick:
            sim.set_failed(crash)
        want += ora.events()
        if step % 3 == 2:  # drain every third tick: three ticks' records at once, in tick order
            got = [(e[0], e[1], kinds[e[2]], e[3]) for e in sim.drain_events()]
            assert got == want, f"drained records differ after tick {t}"
            want = []
    assert sim.tick_stats()["err"] == 0
    # event keeping off: a drain returns the last tick's records only
    sim.keep_events(0)
    ora.tick(), sim.tick()
    ora.events()
    ora.tick(), sim.tick()
    assert [(e[0], e[1], kinds[e[2]], e[3]) for e in sim.drain_events()] == ora.events()


def test_scaled_event_totals_match_drained_records():
    n = 500
    kw = dict(rd_seed=7, drop_pct=85, drop_from=2, drop_to=40, drop_seed=42)
    sim = Simulator(n, GM_MODE_SCALED, **kw)
    seen = {GM_EV_JOINED: 0, GM_EV_REMOVED: 0}
    for _ in range(45):
        sim.tick()
        for e in sim.drain_events():
            seen[e[2]] += 1
    tot = sim.event_totals()
    assert seen[GM_EV_JOINED] > 0 and seen[GM_EV_REMOVED] > 0
    assert tot["joined"] == seen[GM_EV_JOINED] and tot["removed"] == seen[GM_EV_REMOVED], (tot, seen)


def test_sa_half_cluster_crash_runs_clean():
    """The reference's multifailure schedule at S-A size: half the cluster fails at
    once (Application.cpp:188-195 fails nodes [s, s + N/2)). Every crashed node's entries escape
    the byte cells in the ~10 ticks before their removal -- the escape pools are dense-equivalent
    at N = 65,536 -- and ~550 M removal records of the peak tick overflow the per-(row, band)
    slots into the spill ring. Every live observer removes exactly the crashed half, no error."""
    n, crash_tick = 65536, 10
    s0 = 12345
    crash = np.arange(s0, s0 + n // 2, dtype=np.int32)
    sim = Simulator(n, GM_MODE_SCALED, rd_seed=7, init_mode=1, init_t0=8, init_seed=11)
    sim.keep_events(0)
    while sim.time <= 50:
        t = sim.time
        sim.tick()
        if t == crash_tick:
            sim.set_failed(crash)
    sim.sync()
    st = sim.tick_stats()
    n_live, ncrash = n - len(crash), len(crash)
    assert st["err"] == 0 and st["live"] == n_live, st
    tot = sim.event_totals()
    assert tot["removed"] == n_live * ncrash and tot["joined"] == 0, tot
    crashed = np.zeros(n, bool)
    crashed[crash] = True
    t = sim.time - 1
    for r in (0, n - 1):
        hb, ts = sim.read_row(r)
        assert np.all(hb[crashed] == -1) and np.all(hb[~crashed] >= 0)
        assert hb[r] == 2 * t - 1 and ts[r] == t
    sim.close()


def test_sa_cold_start_converges_without_false_removals():
    """init_mode 0 at S-A size: every cell starts at {hb 0, ts 0} (odd-heartbeat cells: ALL of them
    escape on the first ticks -- 4.3 G entries, held by the dense-equivalent pools). The epidemic
    raises every entry long before its TREMOVE age, so nothing is removed or joined, and after
    24 ticks every observer holds every subject with a raised heartbeat."""
    n = 65536
    sim = Simulator(n, GM_MODE_SCALED, rd_seed=7)
    sim.keep_events(0)
    while sim.time <= 24:
        sim.tick()
    sim.sync()
    st = sim.tick_stats()
    assert st["err"] == 0 and st["live"] == n, st
    tot = sim.event_totals()
    assert tot["removed"] == 0 and tot["joined"] == 0, tot
    t = sim.time - 1
    for r in (0, 4097, n - 1):
        hb, ts = sim.read_row(r)
        assert np.all(hb >= 1) and np.all(t - ts < TREMOVE)
        assert hb[r] == 2 * t - 1
    sim.close()
