"""Multi-process (world_size 2, gloo, CPU) coverage of the N>1 path.

1. The sharded protocol itself: two processes each run a numpy model of their
   column shard (tests/shard_model.py) exchanging through gloo all-gather /
   MAX-allreduce exactly as libgm does through RCCL; their union must equal the
   unsharded oracle (tables and events every tick, crash + drops included).
2. The bench rendezvous: the RCCL unique id is broadcast over the gloo group
   (membership.sharded.rendezvous_uid) and every rank receives the same bytes.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _protocol_worker(rank, world, port, n, ticks, q):
    try:
        import sys
        here = os.path.dirname(os.path.abspath(__file__))
        sys.path.insert(0, here)
        import oracle_py
        from shard_model import ShardModel
        _init(rank, world, port)

        def all_gather(x):
            t = torch.from_numpy(np.ascontiguousarray(x))
            out = [torch.zeros_like(t) for _ in range(world)]
            dist.all_gather(out, t)
            return np.stack([o.numpy() for o in out])

        def all_reduce_max(x):
            t = torch.from_numpy(np.ascontiguousarray(x))
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return t.numpy()

        drop = dict(drop_pct=30, drop_from=4, drop_to=18, drop_seed=42, init_mode=1, init_t0=5, init_seed=9)
        m = ShardModel(n, rank, world, rd_seed=7, **drop)
        ora = oracle_py.Oracle(n, oracle_py.OC_SCALED, rd_seed=7, crash_tick=6, crash_count=3, crash_seed=42, **drop)
        crash = oracle_py.crash_set(n, 3, 42)
        for _ in range(ticks):
            t = m.t
            m.tick(all_gather, all_reduce_max)
            ora.tick()
            if t == 6:
                m.failed[crash] = True
            mine = sorted(e for e in ora.events() if m.c0 < e[3] <= m.c0 + m.w)
            assert sorted(m.events) == mine, f"rank {rank} events differ at tick {t}"
            for r in range(n):
                hb, ts = ora.row(r)
                mh, mt = m.row(r)
                assert np.array_equal(mh, hb[m.c0:m.c0 + m.w]), (rank, t, r)
                assert np.array_equal(mt, ts[m.c0:m.c0 + m.w]), (rank, t, r)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e)))


def _uid_worker(rank, world, port, q):
    try:
        import sys
        here = os.path.dirname(os.path.abspath(__file__))
        sys.path.insert(0, os.path.join(os.path.dirname(here), "distributed-membership_amd"))
        import membership.sharded as sh
        sh.comm_unique_id = lambda: bytes(range(128))  # no GPU here: a stand-in id, same plumbing
        _init(rank, world, port)
        uid = sh.rendezvous_uid(rank, world)
        t = torch.tensor(list(uid), dtype=torch.int64)
        ref = t.clone()
        dist.broadcast(ref, 0)
        assert torch.equal(t, ref) and len(uid) == 128
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))


def _run(target, *args, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=target, args=(r, world, port, *args, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    assert all(v == "ok" for _, v in res), res


def test_sharded_protocol_matches_oracle_gloo():
    _run(_protocol_worker, 48, 26)


def test_rccl_uid_rendezvous_gloo():
    _run(_uid_worker)
