"""PARTIAL-view parity (scenario S-C semantics, oracle/ref_cpu.c "PARTIAL"): the HIP
V-entry-view tick against the oracle, tick by tick -- every node's list (dump),
node state and the join / remove event set -- with a crash set and keyed drops."""
import numpy as np
import pytest

import oracle_py
from golden_util import digest64
from membership import GM_EV_JOINED, GM_MODE_PARTIAL, Simulator, crash_set

pytestmark = pytest.mark.gpu


def run_pair(n, v, ticks, crash_tick=-1, crash_count=0, drop_pct=0, drop_from=0, drop_to=0, seed=42):
    run_pair.max_inbox = 0
    kw = dict(rd_seed=7, view_seed=5, init_t0=8, init_seed=11)
    ora = oracle_py.PartialOracle(n, v=v, crash_tick=crash_tick, crash_count=crash_count, crash_seed=seed,
                                  drop_pct=drop_pct, drop_from=drop_from, drop_to=drop_to, drop_seed=seed, **kw)
    sim = Simulator(n, GM_MODE_PARTIAL, rd_seed=7, view=v, view_seed=5, init_mode=1, init_t0=8, init_seed=11,
                    drop_pct=drop_pct, drop_from=drop_from, drop_to=drop_to, drop_seed=seed)
    crash = crash_set(n, crash_count, seed)
    assert sim.dump_tables() == ora.dump(), "initial views differ"
    joins = removes = 0
    for _ in range(ticks):
        t = sim.time
        assert ora.time == t
        ora.tick()
        sim.tick()
        if t == crash_tick:
            sim.set_failed(crash)
        ev = [(e[0], e[1], 1 if e[2] == GM_EV_JOINED else 2, e[3]) for e in sim.drain_events()]
        assert ev == ora.events(), f"events differ at tick {t}"
        joins += sum(e[2] == 1 for e in ev)
        removes += sum(e[2] == 2 for e in ev)
        assert digest64(sim.dump_tables()) == digest64(ora.dump()), f"views differ at tick {t}"
        run_pair.max_inbox = max(run_pair.max_inbox, sim.tick_stats()["max_inbox"])
    assert sim.tick_stats()["err"] == 0
    return joins, removes


@pytest.mark.parametrize("n,v", [(64, 8), (300, 16), (1000, 32)])
def test_partial_matches_oracle(n, v):
    joins, _ = run_pair(n, v, 36, crash_tick=12, crash_count=max(1, n // 50))
    assert joins > 0


def test_partial_with_drops_matches_oracle():
    run_pair(400, 32, 40, crash_tick=10, crash_count=8, drop_pct=30, drop_from=5, drop_to=30)
    # some node got more than P_KP = 16 lists in a tick: the huge-table kernel merged them all
    assert run_pair.max_inbox > 16, run_pair.max_inbox


def test_partial_sparse_views_remove_stale_entries():
    # heavy drops starve views of fresh entries: entries age past TREMOVE and are removed
    _, removes = run_pair(128, 4, 60, drop_pct=90, drop_from=2, drop_to=60)
    assert removes > 0


def test_partial_large_cluster_matches_oracle():
    # N = 131,072: ~0.2 % of the nodes receive more than P_KSMALL = 12 lists per tick
    # (the big-table kernel), ~2 per tick more than P_KP = 16 (the huge-table kernel, every list merged);
    # 5 % drops as in S-C, a crash set inside the window
    n, v = 131072, 32
    kw = dict(rd_seed=7, view_seed=5, init_t0=8, init_seed=11)
    ora = oracle_py.PartialOracle(n, v=v, crash_tick=10, crash_count=1311, crash_seed=42, drop_pct=5, drop_from=0,
                                  drop_to=1000, drop_seed=42, **kw)
    sim = Simulator(n, GM_MODE_PARTIAL, rd_seed=7, view=v, view_seed=5, init_mode=1, init_t0=8, init_seed=11,
                    drop_pct=5, drop_from=0, drop_to=1000, drop_seed=42)
    crash = crash_set(n, 1311, 42)
    for step in range(6):
        t = sim.time
        ora.tick()
        sim.tick()
        if t == 10:
            sim.set_failed(crash)
        ev = [(e[0], e[1], 1 if e[2] == GM_EV_JOINED else 2, e[3]) for e in sim.drain_events()]
        assert ev == ora.events(), f"events differ at tick {t}"
        if step in (2, 5):
            assert digest64(sim.dump_tables()) == digest64(ora.dump()), f"views differ at tick {t}"
    st = sim.tick_stats()
    assert st["err"] == 0 and st["max_inbox"] > 16, st  # the huge-table kernel merged all of them


@pytest.mark.parametrize("n,v,world,drop,chunks", [(300, 16, 2, 0, 4), (1000, 32, 3, 30, 1), (4099, 32, 4, 5, 4),
                                                   (2500, 32, 2, 5, 7)])
def test_row_shards_match_oracle(n, v, world, drop, chunks, monkeypatch):
    """S-C multi-GPU protocol on one device: G row-shard contexts exchange their
    outgoing (header, list) records -- chunk by chunk of their nodes, as the RCCL path
    pipelines them -- through device copies laid out exactly as the all-to-allv lays
    them out, and must reproduce the oracle tick for tick."""
    from membership.abi import partial_loopback_tick
    monkeypatch.setenv("GM_CHUNKS", str(chunks))
    kw = dict(rd_seed=7, view_seed=5, init_t0=8, init_seed=11)
    ora = oracle_py.PartialOracle(n, v=v, crash_tick=12, crash_count=max(1, n // 50), crash_seed=42, drop_pct=drop,
                                  drop_from=5, drop_to=30, drop_seed=42, **kw)
    shards = [Simulator(n, GM_MODE_PARTIAL, rd_seed=7, view=v, view_seed=5, init_mode=1, init_t0=8, init_seed=11,
                        drop_pct=drop, drop_from=5, drop_to=30, drop_seed=42, shard_rank=g, shard_count=world)
              for g in range(world)]
    lay = [s.shard_layout() for s in shards]
    assert lay[0][0] == 0 and sum(w for _, w in lay) == n
    crash = crash_set(n, max(1, n // 50), 42)
    assert b"".join(s.dump_tables() for s in shards) == ora.dump(), "initial views differ"
    for _ in range(36):
        t = shards[0].time
        ora.tick()
        partial_loopback_tick(shards)
        if t == 12:
            for s in shards:
                s.set_failed(crash)
        ev = sorted((e[0], e[1], 1 if e[2] == GM_EV_JOINED else 2, e[3]) for s in shards for e in s.drain_events())
        assert ev == sorted(ora.events()), f"events differ at tick {t}"
        assert b"".join(s.dump_tables() for s in shards) == ora.dump(), f"views differ at tick {t}"
    for s in shards:
        assert s.tick_stats()["err"] == 0


def test_rccl_single_rank_row_shard_matches_oracle(monkeypatch):
    """The RCCL exchange of the row-shard tick (per row chunk, two ncclAllToAllv of
    fixed-size blocks: record headers, then the lists' fresh entries) forced on with one
    rank: the multi-GPU call sequence on this box's one GPU (every target is local, so
    the blocks to other ranks are empty)."""
    from membership.abi import comm_unique_id
    n, v = 2000, 32
    kw = dict(rd_seed=7, view_seed=5, init_t0=8, init_seed=11)
    ora = oracle_py.PartialOracle(n, v=v, crash_tick=12, crash_count=40, crash_seed=42, drop_pct=5, drop_from=0,
                                  drop_to=100, drop_seed=42, **kw)
    monkeypatch.setenv("GM_FORCE_SHARD", "1")
    sim = Simulator(n, GM_MODE_PARTIAL, rd_seed=7, view=v, view_seed=5, init_mode=1, init_t0=8, init_seed=11,
                    drop_pct=5, drop_from=0, drop_to=100, drop_seed=42, shard_rank=0, shard_count=1)
    monkeypatch.delenv("GM_FORCE_SHARD")
    sim.comm_init(comm_unique_id(), 1, 0)
    crash = crash_set(n, 40, 42)
    for _ in range(24):
        t = sim.time
        ora.tick()
        sim.tick()
        if t == 12:
            sim.set_failed(crash)
        ev = [(e[0], e[1], 1 if e[2] == GM_EV_JOINED else 2, e[3]) for e in sim.drain_events()]
        assert ev == ora.events(), f"events differ at tick {t}"
        assert sim.dump_tables() == ora.dump(), f"views differ at tick {t}"
    assert sim.tick_stats()["err"] == 0


def block_caps(n, world, chunks, failed):
    """Python mirror of gm_host.hip xcap: capacity of every (sender shard g, chunk c, receiver q)
    block from the live nodes per shard -- f_q = max(n_q / n, live_q / live), address probability
    p = 1 - (1 - f_q)^5, capacity min(rows, ceil(rows p + 8 sqrt(rows p (1 - p)) + 64))."""
    import math
    b = [n * g // world for g in range(world + 1)]
    live = [int((~failed[b[g]:b[g + 1]]).sum()) for g in range(world)]
    tot = sum(live)
    pq = [1 - (1 - max((b[g + 1] - b[g]) / n, live[g] / tot)) ** 5 for g in range(world)]
    caps = {}
    for g in range(world):
        nl = b[g + 1] - b[g]
        for c in range(chunks):
            rows = nl * (c + 1) // chunks - nl * c // chunks
            for q in range(world):
                if q != g:
                    m = rows * pq[q] + 8 * math.sqrt(rows * pq[q] * (1 - pq[q])) + 64
                    caps[g, c, q] = min(rows, math.ceil(m))
    return caps


def test_row_shards_packed_blocks_match_oracle(monkeypatch):
    """The exchange sends each (chunk, peer) block packed to its records (gm_p_pack) and only the
    block's capacity travels: a binomial bound, 49 % of the slots at S-C (G = 8). At N = 16,384,
    G = 4, one chunk, a block has 4,096 slots whose records are ~Binomial(4096, 0.763) (mean 3,124,
    sigma 27): the capacity is mean + 8 sigma + 64 = 3,406 rows, 83 % of the slots, before the crash;
    after it the capacities follow the live nodes per shard (block_caps). Views, events and the
    oracle agree tick by tick, and each shard receives exactly the capacities' bytes."""
    from membership.abi import partial_loopback_tick
    n, v, world = 16384, 32, 4
    monkeypatch.setenv("GM_CHUNKS", "1")
    monkeypatch.delenv("GM_XCHG_CAP_FRAC", raising=False)
    kw = dict(rd_seed=7, view_seed=5, init_t0=8, init_seed=11)
    ora = oracle_py.PartialOracle(n, v=v, crash_tick=12, crash_count=n // 50, crash_seed=42, drop_pct=5,
                                  drop_from=5, drop_to=30, drop_seed=42, **kw)
    shards = [Simulator(n, GM_MODE_PARTIAL, rd_seed=7, view=v, view_seed=5, init_mode=1, init_t0=8, init_seed=11,
                        drop_pct=5, drop_from=5, drop_to=30, drop_seed=42, shard_rank=g, shard_count=world)
              for g in range(world)]
    crash = crash_set(n, n // 50, 42)
    for _ in range(22):
        t = shards[0].time
        ora.tick()
        partial_loopback_tick(shards)
        if t == 12:
            for s in shards:
                s.set_failed(crash)
        ev = sorted((e[0], e[1], 1 if e[2] == GM_EV_JOINED else 2, e[3]) for s in shards for e in s.drain_events())
        assert ev == sorted(ora.events()), f"events differ at tick {t}"
        if t % 3 == 0:
            assert digest64(b"".join(s.dump_tables() for s in shards)) == digest64(ora.dump()), f"views differ at tick {t}"
        if t == 11:  # before the crash: 3 peers x one block of capacity 3,406 rows
            for s in shards:
                assert s.exchange_bytes() == 3 * 3406 * (32 + 4 * v)
    failed = np.zeros(n, dtype=bool)
    failed[crash] = True
    caps = block_caps(n, world, 1, failed)
    for q, s in enumerate(shards):
        assert s.tick_stats()["err"] == 0
        assert s.exchange_bytes() == sum(caps[g, 0, q] for g in range(world) if g != q) * (32 + 4 * v)


def test_packed_block_overflow_fails_loudly(monkeypatch):
    """A packed exchange block too small for its records sets GM_ERR_XCHG: the tick returns
    GM_ERANGE instead of dropping lists (GM_XCHG_CAP_FRAC = 0.3 < the ~76 % of senders that
    address each peer at G = 4)."""
    from membership.abi import GmError, partial_loopback_tick
    monkeypatch.setenv("GM_XCHG_CAP_FRAC", "0.3")
    n, world = 2048, 4
    sh = [Simulator(n, GM_MODE_PARTIAL, rd_seed=7, view=32, view_seed=5, init_mode=1, init_t0=8, init_seed=11,
                    shard_rank=g, shard_count=world) for g in range(world)]
    with pytest.raises(GmError) as e:
        for _ in range(3):
            partial_loopback_tick(sh)
    assert e.value.code == -4


@pytest.mark.parametrize("chunks", [1, 4])
def test_row_shards_contiguous_half_crash_match_single_context(chunks, monkeypatch):
    """The reference's multifailure schedule crashes a contiguous half of the cluster
    (Application.cpp:188-195: nodes [r, r + N/2)), which takes out whole row shards: after TFAIL
    every survivor addresses each surviving shard with ~76 % at G = 8, far past the 49 % of evenly
    spread targets. The block capacities follow the live nodes per shard, so G = 8
    loopback row shards run the schedule without GM_ERANGE and equal the single context (itself
    oracle-pinned by the tests above) tick by tick: views, events, node state."""
    from membership.abi import partial_loopback_tick
    n, v, world, r = 16384, 32, 8, 3000
    monkeypatch.setenv("GM_CHUNKS", str(chunks))
    monkeypatch.delenv("GM_XCHG_CAP_FRAC", raising=False)
    kw = dict(rd_seed=7, view=v, view_seed=5, init_mode=1, init_t0=8, init_seed=11, drop_pct=5, drop_from=0,
              drop_to=1000, drop_seed=42)
    one = Simulator(n, GM_MODE_PARTIAL, **kw)
    shards = [Simulator(n, GM_MODE_PARTIAL, shard_rank=g, shard_count=world, **kw) for g in range(world)]
    crash = np.arange(r, r + n // 2, dtype=np.int32)
    failed = np.zeros(n, dtype=bool)
    failed[crash] = True
    caps = block_caps(n, world, chunks, failed)
    for _ in range(40):
        t = one.time
        one.tick()
        partial_loopback_tick(shards)
        if t == 10:
            one.set_failed(crash)
            for s in shards:
                s.set_failed(crash)
        ev1 = sorted(one.drain_events())
        evs = sorted(e for s in shards for e in s.drain_events())
        assert evs == ev1, f"events differ at tick {t}"
        if t % 4 == 0 or t in (15, 16, 31):
            assert b"".join(s.dump_tables() for s in shards) == one.dump_tables(), f"views differ at tick {t}"
    assert np.array_equal(np.concatenate([s.read_nodes() for s in shards]), one.read_nodes())
    for q, s in enumerate(shards):
        assert s.tick_stats()["err"] == 0
        want = sum(caps[g, c, q] for g in range(world) if g != q for c in range(chunks))
        assert s.exchange_bytes() == want * (32 + 4 * v), q
