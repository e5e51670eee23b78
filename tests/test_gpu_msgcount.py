"""msgcount analogue at scale (SURVEY §8(f) row 1 beyond FAITHFUL): EmulNet's per-node
sent_msgs / recv_msgs (EmulNet.cpp:111,172, one count per entry message) for the SCALED
and PARTIAL regimes, recorded on the device (gm_msgcount_record) and compared tick by tick
with the oracle's counts (oracle/ref_cpu.c oc_last_msgcount / op_last_msgcount): sent =
fresh entries x targets before loss, recv = delivered entries that survived the keyed loss."""
import numpy as np
import pytest

import oracle_py
from membership import GM_MODE_PARTIAL, GM_MODE_SCALED, GmError, Simulator, crash_set

pytestmark = pytest.mark.gpu

GM_ESTATE = -5


def compare(sim, ora, ticks, crash_tick, crash, tmax):
    """tick both; the device history's column t must equal the oracle's counts of tick t"""
    want = {}
    for _ in range(ticks):
        t = sim.time
        assert ora.time == t
        ora.tick()
        sim.tick()
        if t == crash_tick:
            sim.set_failed(crash)
        want[t] = ora.last_msgcount()
    sent, recv = sim.msgcount(tmax)
    for t, (ws, wr) in want.items():
        assert np.array_equal(sent[:, t], ws), f"sent differs at tick {t}"
        assert np.array_equal(recv[:, t], wr), f"recv differs at tick {t}"
    assert sim.tick_stats()["err"] == 0
    return sent, recv


@pytest.mark.parametrize("n,drop,band,init_mode", [(300, 0, 0, 1), (300, 25, 0, 1), (257, 40, 64, 1), (200, 0, 0, 0)])
def test_scaled_msgcount_matches_oracle(n, drop, band, init_mode):
    seed, ticks, crash_tick = 42, 30, 10
    t0 = 8 if init_mode == 1 else 0
    init = dict(init_mode=init_mode, init_t0=t0, init_seed=seed + 1)
    dkw = dict(drop_pct=drop, drop_from=5, drop_to=22, drop_seed=seed)
    ncrash = max(1, n // 50)
    ora = oracle_py.Oracle(n, oracle_py.OC_SCALED, rd_seed=7, crash_tick=crash_tick, crash_count=ncrash,
                           crash_seed=seed, **dkw, **init)
    sim = Simulator(n, GM_MODE_SCALED, rd_seed=7, band=band, **dkw, **init)
    tmax = sim.time + ticks
    sim.msgcount_record(tmax)
    sent, recv = compare(sim, ora, ticks, crash_tick, crash_set(n, ncrash, seed), tmax)
    assert sent.sum() > 0 and recv.sum() > 0
    if not drop:  # nothing lost in flight: every entry sent at t arrives at t+1 (live receivers)
        t1 = tmax - 1
        assert recv[:, t1].sum() <= sent[:, t1 - 1].sum()


def test_scaled_msgcount_join_ramp_matches_oracle():
    n, seed = 160, 42
    init = dict(init_mode=2, init_t0=0, init_seed=seed + 1)
    ora = oracle_py.Oracle(n, oracle_py.OC_SCALED, rd_seed=7, **init)
    sim = Simulator(n, GM_MODE_SCALED, rd_seed=7, **init)
    ora.tick()  # tick 0: nodeStart of nodes 0-3 (the GPU context starts as of tick 0)
    sim.msgcount_record(61)
    compare(sim, ora, 60, -1, [], 61)


@pytest.mark.parametrize("n,v,drop", [(1000, 32, 5), (300, 16, 30), (500, 32, 0)])
def test_partial_msgcount_matches_oracle(n, v, drop):
    seed, ticks, crash_tick = 42, 30, 12
    kw = dict(rd_seed=7, view_seed=5, init_t0=8, init_seed=11)
    dkw = dict(drop_pct=drop, drop_from=0, drop_to=1 << 20, drop_seed=seed)
    ncrash = max(1, n // 50)
    ora = oracle_py.PartialOracle(n, v=v, crash_tick=crash_tick, crash_count=ncrash, crash_seed=seed, **dkw, **kw)
    sim = Simulator(n, GM_MODE_PARTIAL, view=v, init_mode=1, **dkw, **kw)
    tmax = sim.time + ticks
    sim.msgcount_record(tmax)
    sent, recv = compare(sim, ora, ticks, crash_tick, crash_set(n, ncrash, seed), tmax)
    assert sent.sum() > 0 and recv.sum() > 0


def test_msgcount_record_contract():
    sim = Simulator(64, GM_MODE_SCALED, rd_seed=7, init_mode=1, init_t0=8, init_seed=1)
    with pytest.raises(GmError) as e:  # nothing recorded yet
        sim.msgcount(4)
    assert e.value.code == GM_ESTATE
    sim.tick()
    with pytest.raises(GmError) as e:  # the received counts need the tick before: only before the first tick
        sim.msgcount_record(20)
    assert e.value.code == GM_ESTATE
    sim.close()
    sim = Simulator(64, GM_MODE_PARTIAL, rd_seed=7, view=8, view_seed=5, init_mode=1, init_t0=8, init_seed=11)
    sim.msgcount_record(12)
    for _ in range(3):
        sim.tick()
    sent, recv = sim.msgcount(12)
    assert sent.shape == (64, 12) and not sent[:, :9].any() and sent[:, 9:12].any()
    sim.close()


@pytest.mark.parametrize("world,drop,rccl", [(2, 0, False), (3, 30, False), (1, 20, True)])
def test_column_shard_msgcount_matches_fused_kernel(world, drop, rccl, monkeypatch):
    """Column shards count their own columns' fresh entries (and kept entries on loss ticks);
    the SUM-allreduce gives every rank the whole rows' counts -- equal, tick by tick, to the
    single context's. rccl: one forced shard through ncclAllReduce, with the pending lists
    shrunk so rows finish in the host-driven rounds (msgcount waits for them)."""
    from membership.abi import comm_unique_id
    from membership.sharded import loopback_tick
    n, ticks, crash_tick = 611, 28, 9
    kw = dict(rd_seed=7, drop_pct=drop, drop_from=4, drop_to=20, drop_seed=42, init_mode=1, init_t0=6, init_seed=5)
    ref = Simulator(n, GM_MODE_SCALED, **kw)
    if rccl:
        monkeypatch.setenv("GM_FORCE_SHARD", "1")
        monkeypatch.setenv("GM_SHARD_SYNC", "0")
        monkeypatch.setenv("GM_PLIST_CAP", "4")
    shards = [Simulator(n, GM_MODE_SCALED, shard_rank=g, shard_count=world, **kw) for g in range(world)]
    for v in ("GM_FORCE_SHARD", "GM_SHARD_SYNC", "GM_PLIST_CAP"):
        monkeypatch.delenv(v, raising=False)
    if rccl:
        shards[0].comm_init(comm_unique_id(), 1, 0)
    tmax = ref.time + ticks
    for s in [ref] + shards:
        s.msgcount_record(tmax)
    crash = crash_set(n, 40, 42)
    for _ in range(ticks):
        t = ref.time
        ref.tick()
        if rccl:
            shards[0].tick()
        else:
            loopback_tick(shards)
        if t == crash_tick:
            for s in [ref] + shards:
                s.set_failed(crash)
    want = ref.msgcount(tmax)
    assert want[0].sum() > 0 and want[1].sum() > 0
    for s in shards:
        got = s.msgcount(tmax)
        for t in range(tmax - ticks, tmax):
            assert np.array_equal(got[0][:, t], want[0][:, t]), f"sent differs at tick {t}"
            assert np.array_equal(got[1][:, t], want[1][:, t]), f"recv differs at tick {t}"
        assert s.tick_stats()["err"] == 0
    if world == 1:
        assert shards[0].dump_tables() == ref.dump_tables()
