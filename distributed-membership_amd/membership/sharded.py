"""Column-sharded SCALED ticks: multi-GPU (one rank per GPU, RCCL inside libgm)
or several shards of one device (in-process loopback collectives).

The N x N membership table is split by SUBJECT column: rank g owns columns
[c0_g, c0_g + w_g) of every observer row. The merge + sweep of a delivered
gossip list touches only local columns, so no gossip payload ever crosses a
GPU boundary. What does cross is the gossip-target draw of MP1Node.cpp:449-489,
which indexes the whole post-sweep row ("memberlist[ix]"). Per tick:

  1. every rank merges/sweeps its columns             (gm_shard_merge)
  2. all-gather of per-row (present, numfailed)       int32[G][N][2]
  3. every rank replays every row's S2 stream and resolves the draws landing
     in its columns                                   (gm_shard_draw)
  4. MAX-allreduce of the resolved draws              int32[N][D]
  5. every rank runs the acceptance loop identically  (gm_shard_accept);
     rows that ran out of draws repeat 3-5 with more draws
after which every rank holds identical inboxes for the next tick. With RCCL
attached (gm_comm_init) gm_tick runs all of this natively; loopback_tick
drives the same phases for G contexts living on one device.
"""
import os

from .abi import GM_MODE_SCALED, Simulator, comm_unique_id, shard_loopback

D_FIRST = 16        # must match GM_D_FIRST in gm_host.hip
D_MORE = 64         # must match GM_D_MORE
MAX_ROUNDS = 4096   # must match GM_MAX_ROUNDS: a row that never fills its targets


def loopback_tick(sims):
    """One tick of G in-process shard contexts (one device); returns the draw rounds used."""
    for s in sims:
        s.shard_merge()
    shard_loopback(sims, 0)
    if sims[0].msgcount_recording(sims[0].time):
        shard_loopback(sims, 2)  # msgcount: whole-row fresh counts on every shard
    rnd, d = 0, D_FIRST
    while True:
        for s in sims:
            s.shard_draw(rnd, d)
        shard_loopback(sims, 1, d)
        pend = [s.shard_accept(d) for s in sims]
        if any(p != pend[0] for p in pend):
            raise RuntimeError(f"shards disagree on pending rows: {pend}")
        if pend[0] == 0:
            break
        if rnd + 1 > MAX_ROUNDS:
            raise RuntimeError(f"{pend[0]} rows still drawing after {MAX_ROUNDS} rounds")
        rnd, d = rnd + 1, D_MORE
    for s in sims:
        s.shard_end_tick()
    return rnd + 1


def host_tick(sim, dist, group=None):
    """One tick of THIS process's column shard with the exchanges done by a host collective
    (torch.distributed, e.g. gloo between processes; gm_shard_export / gm_shard_import) in
    place of RCCL: the same phases as loopback_tick, one rank per process. Returns the draw
    rounds used."""
    import torch
    G = dist.get_world_size(group)
    sim.shard_merge()
    mine = torch.from_numpy(sim.shard_export(0))
    slots = [torch.empty_like(mine) for _ in range(G)]
    dist.all_gather(slots, mine, group=group)
    sim.shard_import(0, torch.cat(slots).numpy())
    if sim.msgcount_recording(sim.time):
        x = torch.from_numpy(sim.shard_export(2))
        dist.all_reduce(x, op=dist.ReduceOp.SUM, group=group)  # uint32 counts as int32: sums stay < 2^31
        sim.shard_import(2, x.numpy())
    rnd, d = 0, D_FIRST
    while True:
        sim.shard_draw(rnd, d)
        x = torch.from_numpy(sim.shard_export(1, d))
        dist.all_reduce(x, op=dist.ReduceOp.MAX, group=group)
        sim.shard_import(1, x.numpy(), d)
        pend = sim.shard_accept(d)
        both = torch.tensor([pend, -pend], dtype=torch.int64)
        dist.all_reduce(both, op=dist.ReduceOp.MAX, group=group)
        if int(both[0]) != -int(both[1]):
            raise RuntimeError(f"shards disagree on pending rows ({int(both[0])} vs {-int(both[1])})")
        if pend == 0:
            break
        if rnd + 1 > MAX_ROUNDS:
            raise RuntimeError(f"{pend} rows still drawing after {MAX_ROUNDS} rounds")
        rnd, d = rnd + 1, D_MORE
    sim.shard_end_tick()
    return rnd + 1


def rendezvous_uid(rank, world):
    """Share an RCCL unique id over the CPU (gloo) process group torchrun set up."""
    import torch.distributed as dist
    obj = [comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]


def distributed_shard(n, rank, world, local_rank, **kw):
    """This rank's column shard of an n-node cluster, with RCCL attached.

    Expects torch.distributed initialised with the gloo backend (CPU only: the
    GPU is driven by libgm alone, so torch never initialises HIP here). Every rank has a GPU of
    its own (device_share = 1: the escape pools take a quarter of that device's free HBM), unless
    the diagnostics env GM_DEVICE_OVERRIDE pins all ranks to one device."""
    share = world if "GM_DEVICE_OVERRIDE" in os.environ else 1
    kw.setdefault("device_share", share)
    sim = Simulator(n, GM_MODE_SCALED, shard_rank=rank, shard_count=world, device=local_rank, **kw)
    sim.comm_init(rendezvous_uid(rank, world), world, rank)
    return sim


def env_ranks():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))
