"""Column-sharded SCALED ticks (the multi-GPU path) on one GPU: G shard contexts
in one process exchange through the in-process loopback collectives and must
reproduce the single-context fused kernel -- tables, node state and events --
tick for tick (crash set, keyed drops, converged-start transient included)."""
import numpy as np
import pytest

from membership import GM_MODE_SCALED, Simulator, crash_set
from membership.sharded import loopback_tick

pytestmark = pytest.mark.gpu


def merged_state(shards, owners):
    """Per-shard binary readbacks merged: (hb, ts) [n][n] by column concatenation (shards are
    ordered by rank = ascending column ranges) and each row's node state from the shard that
    owns the row's own column (only that shard bumps the row's self entry)."""
    tabs = [s.read_table() for s in shards]
    hb = np.concatenate([t[0] for t in tabs], axis=1)
    ts = np.concatenate([t[1] for t in tabs], axis=1)
    nodes = np.stack([s.read_nodes() for s in shards])  # [G][n][4]
    st = nodes[owners, np.arange(len(owners))]
    return hb, ts, st


def assert_same_state(shards, owners, ref, what):
    hb, ts, st = merged_state(shards, owners)
    rhb, rts = ref.read_table()
    assert np.array_equal(hb, rhb) and np.array_equal(ts, rts), f"tables differ {what}"
    assert np.array_equal(st, ref.read_nodes()), f"node state differs {what}"


def merge_dumps(dumps, owners):
    """Combine per-shard dumps (same rows, disjoint column ranges) into one dump."""
    per = [d.decode().splitlines() for d in dumps]
    out = []
    for i, lines in enumerate(zip(*per)):
        toks = [ln.split(" ") for ln in lines]
        head = toks[owners[i]][:6]
        n = sum(int(t[6]) for t in toks)
        ents = [e for t in toks for e in t[7:]]
        out.append(" ".join(head + [str(n)] + ents))
    return ("\n".join(out) + "\n").encode()


@pytest.mark.parametrize("n,world,drop,warm", [(256, 2, 0, 0), (600, 3, 0, 1), (512, 2, 25, 0), (1100, 4, 10, 1),
                                               (2048, 8, 10, 1), (21, 3, 30, 1)])
def test_shards_match_fused_kernel(n, world, drop, warm):
    # (21, 3): n < 8G, so shard starts 7 and 14 are odd -- the keyed loss hashes column pairs
    # that straddle a shard boundary (gm_scaled.hip s_keep_nibbles' per-cell path)
    kw = dict(rd_seed=7, drop_pct=drop, drop_from=3, drop_to=25, drop_seed=42, init_mode=warm,
              init_t0=6 if warm else 0, init_seed=5)
    ref = Simulator(n, GM_MODE_SCALED, **kw)
    shards = [Simulator(n, GM_MODE_SCALED, shard_rank=g, shard_count=world, **kw) for g in range(world)]
    owners = np.zeros(n, dtype=int)
    for g, s in enumerate(shards):
        c0, w = s.shard_layout()
        owners[c0:c0 + w] = g
    crash = crash_set(n, max(2, n // 64), 42)
    for _ in range(36):
        t = ref.time
        ref.tick()
        loopback_tick(shards)
        if t == 8:
            ref.set_failed(crash)
            for s in shards:
                s.set_failed(crash)
        assert all(s.time == ref.time for s in shards)
        ev = sorted(e for s in shards for e in s.drain_events())
        assert ev == sorted(ref.drain_events()), f"events differ at tick {t}"
        assert_same_state(shards, owners, ref, f"at tick {t}")
    assert merge_dumps([s.dump_tables() for s in shards], owners) == ref.dump_tables()  # the text rendering too
    for s in shards:
        st = s.tick_stats()
        assert st["err"] == 0
        assert st["lists"] == ref.tick_stats()["lists"]


@pytest.mark.parametrize("n,world,drop,chunks,pcap", [(2048, 8, 10, 4, 0), (1100, 3, 20, 3, 0), (600, 2, 0, 7, 0),
                                                      (4099, 4, 5, 2, 0), (2048, 8, 10, 4, 4), (4099, 4, 5, 2, 16)])
def test_pipelined_shards_match_fused_kernel(n, world, drop, chunks, pcap, monkeypatch):
    """The chunk order of the pipelined RCCL tick (per exchange row chunk: all-gather of the
    counts, round-0 draws, MAX-reduce of their statuses, acceptance -- on the comm stream while
    later chunks merge; then the bounded rounds) with G shard contexts on one device
    (gm_shard_loopback_tick, collectives by device copies): tick for tick equal to the fused
    kernel, and to the phase-API loopback shards. GM_SCHUNKS sets the exchange chunks (R rows,
    a power of two; the last chunk shorter). pcap > 0 shrinks the pending lists (GM_PLIST_CAP):
    in the warm-start transient and after the crash more rows stay pending than a list holds,
    and the rows each rank's atomics had put in an overflowing list would differ -- such a list
    is void on every rank and its rows take the host-driven rounds (the full-size S-B run at
    tick 15 found it: ranks MAX-reduced statuses of different rows)."""
    from membership.abi import shard_loopback_tick
    monkeypatch.setenv("GM_SCHUNKS", str(chunks))
    if pcap:
        monkeypatch.setenv("GM_PLIST_CAP", str(pcap))
    kw = dict(rd_seed=7, drop_pct=drop, drop_from=3, drop_to=25, drop_seed=42, init_mode=1, init_t0=6, init_seed=5)
    ref = Simulator(n, GM_MODE_SCALED, **kw)
    shards = [Simulator(n, GM_MODE_SCALED, shard_rank=g, shard_count=world, **kw) for g in range(world)]
    phase = [Simulator(n, GM_MODE_SCALED, shard_rank=g, shard_count=world, **kw) for g in range(world)]
    monkeypatch.delenv("GM_SCHUNKS")
    monkeypatch.delenv("GM_PLIST_CAP", raising=False)
    owners = np.zeros(n, dtype=int)
    for g, s in enumerate(shards):
        c0, w = s.shard_layout()
        owners[c0:c0 + w] = g
    crash = crash_set(n, max(2, n // 64), 42)
    for _ in range(34):
        t = ref.time
        ref.tick()
        shard_loopback_tick(shards)
        loopback_tick(phase)
        if t == 8:
            for s in [ref] + shards + phase:
                s.set_failed(crash)
        ev = sorted(ref.drain_events())
        assert sorted(e for s in shards for e in s.drain_events()) == ev, f"events differ at tick {t}"
        assert sorted(e for s in phase for e in s.drain_events()) == ev, f"phase-API events differ at tick {t}"
        assert_same_state(shards, owners, ref, f"at tick {t}")
    assert_same_state(phase, owners, ref, "(phase API) at the end")
    for s in shards:
        assert s.tick_stats()["err"] == 0


@pytest.mark.parametrize("n,drop,ncrash,rounds", [(777, 0, 12, "auto"), (2048, 20, 32, "auto"), (777, 0, 12, "sync"),
                                                  (777, 0, 388, "bounded"), (777, 0, 388, "overflow")])
def test_rccl_single_rank_matches_fused_kernel(n, drop, ncrash, rounds, monkeypatch):
    """The RCCL-driven sharded tick (gm_tick -> ncclAllGather / ncclAllReduce on the
    context stream) with one forced shard on the one GPU this box has: the exact
    collective calls the multi-GPU run makes, degenerate only in the rank count.
    "auto" takes the bounded, stream-ordered draw rounds here; "sync" the host-driven
    loop; "bounded" with half the cluster crashed forces the bounded path with many rows
    left pending after round 0, so round 1 (the sorted pending list) does real work;
    "overflow" shrinks both pending lists to 4 rows (GM_PLIST_CAP), so most pending rows
    overflow them and finish in the host-driven rounds, each from its own next round."""
    from membership.abi import comm_unique_id
    kw = dict(rd_seed=7, drop_pct=drop, drop_from=3, drop_to=25, drop_seed=42, init_mode=1, init_t0=6, init_seed=5)
    ref = Simulator(n, GM_MODE_SCALED, **kw)
    monkeypatch.setenv("GM_FORCE_SHARD", "1")
    if rounds != "auto":
        monkeypatch.setenv("GM_SHARD_SYNC", "1" if rounds == "sync" else "0")
    if rounds == "overflow":
        monkeypatch.setenv("GM_PLIST_CAP", "4")
    sh = Simulator(n, GM_MODE_SCALED, shard_rank=0, shard_count=1, **kw)
    monkeypatch.delenv("GM_FORCE_SHARD")
    monkeypatch.delenv("GM_SHARD_SYNC", raising=False)
    monkeypatch.delenv("GM_PLIST_CAP", raising=False)
    sh.comm_init(comm_unique_id(), 1, 0)
    crash = crash_set(n, ncrash, 42)
    for _ in range(32):
        t = ref.time
        ref.tick()
        sh.tick()
        if t == 8:
            ref.set_failed(crash)
            sh.set_failed(crash)
        assert sorted(sh.drain_events()) == sorted(ref.drain_events()), f"events differ at tick {t}"
        assert_same_state([sh], np.zeros(n, dtype=int), ref, f"at tick {t}")
    assert sh.dump_tables() == ref.dump_tables()
    assert sh.tick_stats()["err"] == 0


def _crash_seed_with(n, count, want):
    for seed in range(1, 10000):
        if want in set(crash_set(n, count, seed).tolist()):
            return seed
    raise AssertionError("no seed")


@pytest.mark.parametrize("n,world,drop,intro", [(400, 2, 0, False), (600, 3, 30, False), (1024, 4, 10, False),
                                                (256, 2, 0, True), (602, 3, 20, False), (1001, 4, 10, False)])
def test_ramp_shards_match_fused_kernel(n, world, drop, intro):
    """The join ramp (init_mode 2: JOINREQ / JOINREP / newNodes-first gossip) on G column
    shards equals the single context tick for tick: tables, node state, events. With keyed
    drops a joiner that misses its own entry takes updateMyPos's quirk path (MP1Node.cpp:316)
    on the shard owning its start group, which reports its "me" column to the draw; the
    introducer's joiners-first targets (MP1Node.cpp:458) are enqueued on every rank."""
    kw = dict(rd_seed=7, init_mode=2, drop_pct=drop, drop_from=0, drop_to=1 << 20, drop_seed=42)
    ref = Simulator(n, GM_MODE_SCALED, **kw)
    shards = [Simulator(n, GM_MODE_SCALED, shard_rank=g, shard_count=world, **kw) for g in range(world)]
    owners = np.zeros(n, dtype=int)
    for g, s in enumerate(shards):
        c0, w = s.shard_layout()
        owners[c0:c0 + w] = g
    cnt = max(2, n // 32)
    crash = crash_set(n, cnt, _crash_seed_with(n, cnt, 0) if intro else 42)
    crash_tick = n // 8  # mid-ramp: crashed starters revive at their nodeStart
    for _ in range(n // 4 + 30):
        t = ref.time
        ref.tick()
        loopback_tick(shards)
        if t == crash_tick:
            ref.set_failed(crash)
            for s in shards:
                s.set_failed(crash)
        ev = sorted(e for s in shards for e in s.drain_events())
        assert ev == sorted(ref.drain_events()), f"events differ at tick {t}"
        if t % 4 == 0:
            assert_same_state(shards, owners, ref, f"at tick {t}")
    assert merge_dumps([s.dump_tables() for s in shards], owners) == ref.dump_tables()
    for s in shards:
        assert s.tick_stats()["err"] == 0
    assert ref.tick_stats()["err"] == 0


def test_shard_boundaries_keep_start_groups_whole():
    """Column shard boundaries are multiples of 4 for any n >= 8G (n = 602, 1001: n*g/G is not), so
    no start group (ids 4g..4g+3) straddles two shards; a ramp whose tiny cluster cannot be cut that
    way (n < 8G) is refused."""
    from membership.abi import GmError
    for n, world in ((602, 3), (1001, 4), (4099, 8)):
        cols = [Simulator(n, GM_MODE_SCALED, rd_seed=7, init_mode=2, shard_rank=g, shard_count=world).shard_layout()
                for g in range(world)]
        assert [c0 for c0, _ in cols] == sorted(c0 for c0, _ in cols) and cols[0][0] == 0
        assert all(c0 % 4 == 0 for c0, _ in cols) and sum(w for _, w in cols) == n
        assert all(cols[g][0] + cols[g][1] == cols[g + 1][0] for g in range(world - 1))
        assert max(w for _, w in cols) - min(w for _, w in cols) <= 7
    with pytest.raises(GmError):
        Simulator(20, GM_MODE_SCALED, rd_seed=7, init_mode=2, shard_rank=0, shard_count=3)


def test_rccl_single_rank_ramp_matches_fused_kernel(monkeypatch):
    """The join ramp through gm_tick's RCCL-driven sharded tick (one forced shard):
    bounded draw rounds, joiners-first introducer targets, keyed drops."""
    from membership.abi import comm_unique_id
    n = 300
    kw = dict(rd_seed=7, init_mode=2, drop_pct=20, drop_from=0, drop_to=1 << 20, drop_seed=42)
    ref = Simulator(n, GM_MODE_SCALED, **kw)
    monkeypatch.setenv("GM_FORCE_SHARD", "1")
    sh = Simulator(n, GM_MODE_SCALED, shard_rank=0, shard_count=1, **kw)
    monkeypatch.delenv("GM_FORCE_SHARD")
    sh.comm_init(comm_unique_id(), 1, 0)
    crash = crash_set(n, 9, 42)
    for _ in range(n // 4 + 30):
        t = ref.time
        ref.tick()
        sh.tick()
        if t == 40:
            ref.set_failed(crash)
            sh.set_failed(crash)
        assert sorted(sh.drain_events()) == sorted(ref.drain_events()), f"events differ at tick {t}"
        assert_same_state([sh], np.zeros(n, dtype=int), ref, f"at tick {t}")
    assert sh.dump_tables() == ref.dump_tables()
    assert sh.tick_stats()["err"] == 0
