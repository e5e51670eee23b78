#!/usr/bin/env python3
"""Headline benchmark: simulated node-ticks/s (+ achieved HBM GB/s) of the
SCALED full-membership tick at N = 65,536 (BASELINE.json metric, SURVEY.md
§8(d) scenario S-A).

A "step" is one globaltime tick of the whole cluster (Application::mp1Run for
all N nodes: merge delivered gossip lists, heartbeat bump, TFAIL/TREMOVE sweep,
gossip-target draw, delivery to next tick's inboxes), state resident in HBM.

Scenario S-A: converged start (every observer holds every subject; the warm
variant of gm_abi.h init_mode 1 at t0 = 8, i.e. entries 0-3 ticks old as if the
cluster had been gossiping, so there is no mass-staleness transient), fanout 5,
TFAIL 5, TREMOVE 20, RD_SEED 7, 1% of the nodes (655) crash at the end of tick
10 (splitmix64-keyed crash set, seed 42), no drops. The prologue runs to tick
25 (T_warm of S-A); then W warmup ticks, then exactly K timed ticks, which
contain the crashed nodes' TREMOVE removals (~42 M events).

Multi-GPU (--gpus G via torch.distributed.run, one rank per GPU): the same
N = 65,536 cluster with its N x N table sharded by subject column, rank g
owning N/G columns of every row ("strong" scaling: total work fixed). libgm
runs the per-tick exchange (all-gather of per-row counts, MAX-allreduce of
resolved gossip draws) with RCCL on its own stream; torch.distributed is only
the CPU (gloo) rendezvous that hands every rank the RCCL unique id, plus the
barrier / max-over-ranks timing. See DESIGN.md §Multi-GPU.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "distributed-membership_amd"))

PEAK_HBM_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
LAYOUT_SA = "byte-band"  # profiles/traffic_n65536.json must describe this payload layout


class Roctx:
    """roctxProfilerPause/Resume around the timed region, so that
    `rocprofv3 --selected-regions --kernel-trace --stats -- python3 bench.py`
    traces exactly the K timed ticks (no-ops when not profiling)."""

    def __init__(self):
        import ctypes
        self.lib = None
        for name in ("librocprofiler-sdk-roctx.so.1", "libroctx64.so"):
            try:
                self.lib = ctypes.CDLL(name)
                break
            except OSError:
                continue

    def pause(self):
        if self.lib is not None:
            self.lib.roctxProfilerPause(0)

    def resume(self):
        if self.lib is not None:
            self.lib.roctxProfilerResume(0)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--scenario", choices=["S-A", "S-B", "S-C"], default="S-A",
                   help="S-A: full membership N=65,536 (headline); S-B: full membership N=262,144 (the "
                        "north_star scaling cluster); S-C: partial views V=32, N=16M, 5%% drop")
    p.add_argument("--dry-launch", action="store_true",
                   help="start the ranks (--gpus G), rendezvous over gloo, print one JSON line with every rank's "
                        "RANK / WORLD_SIZE / LOCAL_RANK and stop before libgm is loaded (no GPU call)")
    p.add_argument("--master-port", type=int, default=0, help="--gpus G > 1 launch: rendezvous port (0: a free one)")
    p.add_argument("--cluster", type=int, default=0, help="N, simulated nodes (0: the scenario's)")
    p.add_argument("--view", type=int, default=32, help="S-C view capacity V")
    p.add_argument("--prologue", type=int, default=25)
    p.add_argument("--t0", type=int, default=8, help="warm converged start at tick t0 (0: cold start)")
    p.add_argument("--crash-tick", type=int, default=10)
    p.add_argument("--crash-frac", type=float, default=0.01)
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--drop-pct", type=int, default=0,
                   help="diagnostics (S-A): keyed per-entry drops on every tick (the drop path of gm_s_band)")
    p.add_argument("--force-shard", action="store_true",
                   help="diagnostics: at N=1 run the column-shard protocol with RCCL over one rank")
    p.add_argument("--no-companion", dest="companion", action="store_false",
                   help="S-A only: skip the companion S-B run (N=262,144, same schedule and ranks) whose line "
                        "goes under \"companion\" -- the north_star scaling cluster measured by every --gpus G run")
    p.add_argument("--no-pmc", dest="pmc", action="store_false",
                   help="skip the live traffic measurement: by default (N=1) roofline.traffic is measured after "
                        "the timed run by two rocprofv3 --pmc passes of this workload (FETCH_SIZE, WRITE_SIZE; as "
                        "scripts/gpu.sh pmc_sa / pmc_sc), falling back to the committed profiles/traffic_*.json")
    p.add_argument("--pmc", dest="pmc", action="store_true", help=argparse.SUPPRESS)  # the default; kept for old callers
    return p.parse_args()


def live_traffic(kernel, layout, n, extra):
    """HBM bytes per launch of `kernel` measured now: this bench (5 ticks) under two rocprofv3
    PMC passes (each counter in a run of its own, --kernel-trace only), reduced by
    scripts/pmc_traffic.py (gfx950 FETCH_SIZE x2 correction). Child processes, so the
    measured run and this one never share a profiler."""
    import subprocess
    import tempfile
    d = tempfile.mkdtemp(prefix="gm_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    child = [sys.executable, os.path.abspath(__file__), "--no-cpu", "--no-pmc", "--steps", "5", "--warmup", "1"] + extra
    for ctr, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        cmd = ["rocprofv3", "--pmc", ctr, "--kernel-trace", "--output-format", "csv", "-d", os.path.join(d, sub),
               "-o", "p", "--"] + child
        subprocess.run(cmd, timeout=300, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    out = os.path.join(d, "traffic.json")
    subprocess.run([sys.executable, os.path.join(REPO, "scripts", "pmc_traffic.py"), "--kernel", kernel, "--fetch",
                    os.path.join(d, "fetch"), "--write", os.path.join(d, "write"), "--layout", layout, "--n", str(n),
                    "--out", out], timeout=120, check=True, stdout=subprocess.DEVNULL)
    with open(out) as f:
        tj = json.load(f)
    return tj["hbm_bytes_per_launch"], f"live: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this workload ({d})"


_JSON_FD = None


def host_cpu():
    """model name and logical CPU count of the host the CPU baseline ran on"""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return f"{model}, {os.cpu_count()} logical CPUs visible"


def quiet_stdout():
    """The bench's stdout carries exactly ONE JSON line: native libraries' own stdout
    (RCCL's version banner at communicator init, ...) goes to stderr instead."""
    global _JSON_FD
    if _JSON_FD is None:
        sys.stdout.flush()
        _JSON_FD = os.dup(1)
        os.dup2(2, 1)


def emit(out):
    line = (json.dumps(out) + "\n").encode()
    if _JSON_FD is None:
        sys.stdout.write(line.decode())
        sys.stdout.flush()
    else:
        os.write(_JSON_FD, line)


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(a):
    """`bench.py --gpus G` (G > 1) started as a plain process: run G ranks of this same
    command under torch.distributed.run (one rank per GPU, rendezvous on 127.0.0.1) as a
    CHILD process and return its exit code. Called before anything loads libgm or touches
    the GPU; the child's rank 0 prints the JSON line."""
    import subprocess
    port = a.master_port or free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this pool (RCCL across processes)
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def rank_env(a):
    """(rank, world, local_rank) of this process; exits non-zero when torch.distributed.run's
    WORLD_SIZE disagrees with --gpus (the bench would otherwise time a different job)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        sys.stderr.write(f"bench.py: WORLD_SIZE={world} but --gpus {a.gpus}\n")
        sys.exit(2)
    return int(os.environ.get("RANK", "0")), world, int(os.environ.get("LOCAL_RANK", "0"))


def gather_ranks(dist, info):
    """every rank's launch / RCCL facts, for rank 0's JSON line"""
    if dist is None:
        return [info]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, info)
    return out


def dry_launch(a):
    rank, world, local = rank_env(a)
    info = {"rank": rank, "world_size": world, "local_rank": local, "pid": os.getpid(),
            "master": f"{os.environ.get('MASTER_ADDR', '')}:{os.environ.get('MASTER_PORT', '')}"}
    dist = None
    if world > 1:
        import torch.distributed as tdist
        tdist.init_process_group("gloo")
        dist = tdist
    ranks = gather_ranks(dist, info)
    if rank == 0:
        emit({"dry_launch": True, "n_gpus": a.gpus, "scenario": a.scenario, "ranks": ranks,
              "companion": "S-B" if (a.companion and a.scenario == "S-A" and a.cluster in (0, 65536)
                                     and not a.drop_pct and not a.force_shard) else None})
    if dist is not None:
        dist.destroy_process_group()


def scaled_run(a, n, rank, world, local, dist, rtx, profiled):
    """One timed run of the SCALED tick at N = n on the S-A schedule (warm start at t0,
    a.crash_frac crashed at a.crash_tick, prologue to a.prologue, a.warmup untimed ticks,
    then exactly a.steps timed ticks between barriers), with the workload self-check
    after the window. profiled: the timed ticks are the roctx-selected region."""
    from membership import GM_MODE_SCALED, Simulator, crash_set
    from membership.sharded import distributed_shard
    ncrash = int(round(n * a.crash_frac))
    init = dict(init_mode=1 if a.t0 > 0 else 0, init_t0=a.t0, init_seed=11)
    if a.drop_pct:
        init.update(drop_pct=a.drop_pct, drop_from=0, drop_to=1 << 30, drop_seed=5)
    if world > 1:
        sim = distributed_shard(n, rank, world, local, rd_seed=7, **init)
    elif a.force_shard:
        os.environ["GM_FORCE_SHARD"] = "1"
        sim = Simulator(n, GM_MODE_SCALED, rd_seed=7, device=local, shard_rank=0, shard_count=1, **init)
        from membership.abi import comm_unique_id
        sim.comm_init(comm_unique_id(), 1, 0)
    else:
        sim = Simulator(n, GM_MODE_SCALED, rd_seed=7, device=local, **init)
    sim.keep_events(0)  # no per-tick staging of join/remove records; the device counts them (gm_event_totals)
    crash = crash_set(n, ncrash, 42)
    while sim.time <= a.prologue:
        t = sim.time
        sim.tick()
        if t == a.crash_tick:
            sim.set_failed(crash)
    for _ in range(a.warmup):
        sim.tick()
    sim.sync()

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    sim.sync()
    sim.set_timing(1)
    if profiled:
        rtx.resume()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        sim.tick()
    sim.sync()
    t1 = time.perf_counter()
    if profiled:
        rtx.pause()
    barrier()
    elapsed = t1 - t0
    if dist is not None:
        import torch
        x = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        elapsed = float(x.item())
    kernel_ms = sim.last_kernel_ms()
    st = sim.tick_stats()
    assert st["err"] == 0, st
    # self-check of the measured workload (outside the timed window): the window holds the
    # TREMOVE sweep of the crashed nodes (MP1Node.cpp:429-444) -- every live observer removed
    # every crashed node exactly once, nothing else was removed or joined (device counters)
    tot = sim.event_totals()
    # (a cold start too: its transient converges without false removals by t0 + 10,
    # test_sa_cold_start_converges_without_false_removals; profiles/r06/cold_start/)
    removed_ok = (a.prologue + a.warmup + a.steps >= a.crash_tick + 38
                  and not a.drop_pct)  # loss can remove live nodes too
    if removed_ok:
        c0, wl = sim.shard_layout() if world > 1 else (0, n)  # a column shard counts its own columns
        crash_here = int(((crash >= c0) & (crash < c0 + wl)).sum())
        assert tot["removed"] == (n - ncrash) * crash_here and tot["joined"] == 0, (tot, n - ncrash, crash_here)
    W = sim.shard_layout()[1] if world > 1 else n  # this rank's subject columns
    return dict(sim=sim, n=n, ncrash=ncrash, elapsed=elapsed, kernel_ms=kernel_ms, st=st, tot=tot,
                removed_ok=removed_ok, W=W, t0=t0, t1=t1)


def collective_bytes(n, world):
    """RCCL payload one rank contributes per column-shard tick (gm_host.hip tick_sharded): the
    all-gather of its per-row (present, numfailed) int32 pairs, the MAX-allreduce of the round-0
    draw statuses int32[n][16], and the bounded rounds' MAX-allreduces int32[cap1][64] +
    int32[256][256] (cap1 = min(4096, max(min(n, 1024), n / 16))). 0 on one GPU (no exchange)."""
    if world <= 1:
        return {"allgather_counts": 0, "allreduce_draws": 0, "allreduce_rounds": 0}
    cap1 = min(4096, max(min(n, 1024), n // 16))
    # the pipelined all-gather sends whole exchange chunks: xk chunks of R = 2^xlog rows (gm_host.hip:
    # xlog >= 6 is the least with R * K >= n, K = GM_SCHUNKS, default 2), padding included
    k = int(os.environ.get("GM_SCHUNKS", "2") or 2)
    xlog = 6
    while (1 << xlog) * k < n:
        xlog += 1
    R = 1 << xlog
    xk = (n + R - 1) // R
    return {"allgather_counts": 8 * xk * R, "allreduce_draws": 4 * 16 * n, "allreduce_rounds": 4 * (64 * cap1 + 256 * 256)}


def companion_sb(a, rank, world, local, dist, rtx):
    """The north_star scaling cluster measured beside the headline: the same schedule at
    N = 262,144 (S-B, BASELINE.json configs[3]) on the same G ranks, so that every
    `bench.py --gpus G` line of a 1/2/4/8-GPU sweep also carries the S-B curve. Not the
    headline value (that stays S-A); outside the roctx-selected region."""
    try:
        r = scaled_run(a, 262144, rank, world, local, dist, rtx, profiled=False)
    except (AssertionError, RuntimeError, OSError) as e:  # reported, not fatal to the headline line
        return {"scenario": "S-B", "error": f"{type(e).__name__}: {e}"}
    n = r["n"]
    st, W, kms = r["st"], r["W"], r["kernel_ms"]
    b_alg = (5 * st["live"] + st["lists"]) * W // 2  # rank 0's band kernels, as for S-A
    ach = b_alg / (kms * 1e-3) / 1e9 if kms > 0 else None
    out = {"scenario": "S-B", "metric": "simulated node-ticks/sec (S-B N=262,144 full membership)",
           "value": n * a.steps / r["elapsed"], "unit": "node-ticks/s", "n_gpus": world,
           "ms_per_step": r["elapsed"] / a.steps * 1e3, "kernel_ms_rank0": kms,
           "n": n, "crashed": r["ncrash"], "columns_per_gpu": W, "scaling": "strong",
           "roofline_rank0": {"bound": "hbm", "alg_bytes_per_launch": b_alg, "achieved": ach, "peak": PEAK_HBM_GBPS,
                              "unit": "GB/s", "frac": ach / PEAK_HBM_GBPS if ach else None},
           "collective_bytes_per_rank_tick": collective_bytes(n, world),
           "check": {"removed_rank0": r["tot"]["removed"], "joined_rank0": r["tot"]["joined"]}}
    r["sim"].close()
    return out


def main():
    a = parse()
    if a.gpus < 1:
        sys.stderr.write("bench.py: --gpus must be >= 1\n")
        sys.exit(2)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a))
    quiet_stdout()
    if a.dry_launch:
        return dry_launch(a)
    if a.scenario == "S-C":
        return main_partial(a)
    a.cluster = a.cluster or (262144 if a.scenario == "S-B" else 65536)
    rtx = Roctx()
    rtx.pause()
    rank, world, local = rank_env(a)
    if "GM_DEVICE_OVERRIDE" in os.environ:  # diagnostics only: pin every rank to one device
        local = int(os.environ["GM_DEVICE_OVERRIDE"])
    # libgm first: it binds the system ROCm HIP runtime and RCCL it was built
    # against before torch (CPU-only here) brings its own copies into the process
    from membership import load_library
    load_library()

    dist = None
    if world > 1:
        # CPU-only process group: rendezvous, barrier and max-over-ranks timing.
        # The GPU (and RCCL over xGMI) is driven by libgm alone.
        import torch.distributed as tdist
        tdist.init_process_group("gloo")
        dist = tdist

    r = scaled_run(a, a.cluster, rank, world, local, dist, rtx, profiled=True)
    sim, n, ncrash, elapsed, kernel_ms = r["sim"], r["n"], r["ncrash"], r["elapsed"], r["kernel_ms"]
    st, tot, removed_ok, W, t0, t1 = r["st"], r["tot"], r["removed_ok"], r["W"], r["t0"], r["t1"]
    n_live, m_lists = st["live"], st["lists"]
    # algorithmic bytes of one tick in this layout: per live row and
    # column 1 B cell read + 1 B cell write + 0.5 B payload write, plus 0.5 B per
    # delivered gossip list (payload read) -- the survey's formulation (SURVEY.md §8(d):
    # read and write the receiver's row once, read each delivered sender row once per
    # delivery) in this build's byte cell / 4-bit payload units (escaped cells' wide
    # plane traffic is not counted: it is the layout's overhead, seen by PMC traffic)
    b_alg = (5 * n_live + m_lists) * W // 2
    # the survey's int32 (hb, ts) formulation of the same work
    b_survey = 16 * n_live * W + 8 * m_lists * W
    achieved = b_alg / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else None
    # DRAM bytes the layout cannot avoid: the cell read + write and the payload write per
    # live cell, plus ONE read of each sender's payload (its ~5 re-reads are served by the
    # Infinity Cache while the band is in flight; FETCH_SIZE counts those hits too)
    dram_est = 3 * n_live * W
    frac_dram = (dram_est / (kernel_ms * 1e-3) / 1e9 / PEAK_HBM_GBPS) if kernel_ms > 0 else None
    traffic, traffic_src = None, None
    tpath_ok = world == 1
    tpath = os.path.join(REPO, "profiles", f"traffic_n{n}.json")
    if tpath_ok and os.path.exists(tpath):
        with open(tpath) as f:
            tj = json.load(f)
        if tj.get("layout") == LAYOUT_SA:
            traffic = tj.get("hbm_bytes_per_launch")
            traffic_src = f"profiles/traffic_n{n}.json ({tj.get('generated', 'r01')}, rocprofv3 --pmc passes by scripts/gpu.sh pmc_sa)"
    value = n * a.steps / elapsed
    ranks = gather_ranks(dist, {"rank": rank, "local_rank": local, **sim.comm_info(), "kernel_ms": kernel_ms,
                                "columns": W, "elapsed_s": t1 - t0})
    out = {
        "metric": ("simulated node-ticks/sec + achieved HBM GB/s at N=65,536 full-membership" if a.scenario == "S-A"
                   else "simulated node-ticks/sec (S-B N=262,144 full membership)"),
        "value": value,
        "unit": "node-ticks/s",
        "value_note": "all N simulated nodes per tick, the 1% crashed (frozen) ones included",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u8 cells (u16 escape lists) / 4-bit payload (integer)",
        "data": "synthetic (converged full-membership table, seeded crash set)",
        "config": {"workload": f"{a.scenario}: SCALED full membership, 1% crash at tick 10, fanout 5, TFAIL 5, TREMOVE 20"
                   + (f", DIAGNOSTIC keyed {a.drop_pct}% per-entry drops" if a.drop_pct else ""),
                   "n": n, "start": f"warm t0={a.t0}" if a.t0 > 0 else "cold", "prologue_to_tick": a.prologue, "crashed": ncrash, "live": n_live,
                   "lists_per_tick": m_lists, "parallelism": f"column-shard x{world}" if world > 1 else
                   ("column-shard x1 (RCCL, forced)" if a.force_shard else "single GPU")},
        "ranks": ranks,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                     "frac": (achieved / PEAK_HBM_GBPS) if achieved else None, "traffic": traffic,
                     "achieved_basis": "algorithmic bytes per launch / kernel time (contract field); NOT DRAM "
                                       "bandwidth: ~5 of every 6 payload reads are Infinity-Cache hits, see "
                                       "achieved_dram_est / frac_dram",
                     "achieved_algorithmic": achieved,
                     "achieved_dram_est": (dram_est / (kernel_ms * 1e-3) / 1e9) if kernel_ms > 0 else None,
                     "traffic_source": traffic_src,
                     "kernel": "gm_s_band" if a.drop_pct else "gm_s_band_fast + gm_s_band_listed",
                     "kernel_ms": kernel_ms,
                     "alg_bytes_per_launch": b_alg, "survey_int32_bytes_per_launch": b_survey,
                     "dram_bytes_est": dram_est, "frac_dram": frac_dram,
                     "columns_per_gpu": W},
        "collective_bytes_per_rank_tick": collective_bytes(n, world),
        "check": {"removed_rank0": tot["removed"], "joined_rank0": tot["joined"], "removed_all_expected":
                  (n - ncrash) * ncrash if removed_ok else None},
    }
    sim.close()  # the companion run and the PMC passes (child processes) need the device memory
    if a.companion and a.scenario == "S-A" and n == 65536 and not a.drop_pct and not a.force_shard:
        out["companion"] = companion_sb(a, rank, world, local, dist, rtx)
    if a.pmc and world == 1:
        try:
            out["roofline"]["traffic"], out["roofline"]["traffic_source"] = live_traffic(
                "gm_s_band", LAYOUT_SA, n, ["--cluster", str(n), "--no-companion"] +
                (["--drop-pct", str(a.drop_pct)] if a.drop_pct else []))
        except Exception as e:  # no profiler / counters on this host: the committed figure stands, said so
            out["roofline"]["traffic_source"] = f"{traffic_src} (live PMC passes failed: {type(e).__name__})"
    if rank == 0 and world == 1 and not a.no_cpu:
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import oracle_py  # the oracle is the CPU baseline here, never the measured path
        nodes, secs = oracle_py.bench_sample(n, lists=5, min_seconds=a.cpu_seconds)
        out["cpu_baseline"] = {"value": nodes / secs, "unit": "node-ticks/s", "cores": 1, "kind": "port",
                               "host": host_cpu(),
                               "sample": f"{nodes} node-ticks of the N={n} SCALED workload on one host core "
                                         f"({secs:.1f} s): per node-tick 5 gossip lists x {n} entries merged via "
                                         "updatelistCallBack + nodeLoopOps sweep/sort/draw (oracle/ref_cpu.c)"}
        hr = hour_run()
        if hr:
            out["cpu_baseline"]["hour_run"] = hr
    if rank == 0:
        emit(out)
    if dist is not None:
        dist.destroy_process_group()


HOUR_DIR = os.path.join(REPO, "profiles", "cpu_hour")  # (travels to the GPU box: not gpurun-ignored)


def hour_run():
    """The hour-sized CPU run, read from its committed segments
    (scripts/cpu_hour.py: the SCALED restatement at N = 13,722 on one host core of the GPU box,
    ticks 9..108 of the S-A schedule in 25-tick segments, each started from the GPU-reached state of
    its first tick, which gm_read_* hands to oc_load_scaled). Summed per tick, not re-run here:
    an hour of CPU is not a bench step. None when the segments are absent."""
    import glob
    ticks, host, n = {}, None, None
    for f in sorted(glob.glob(os.path.join(HOUR_DIR, "cpu_hour_seg*.jsonl"))):
        seg, fn = {}, None
        with open(f) as fh:
            for line in fh:
                try:
                    r = json.loads(line)
                except ValueError:  # a line cut off by an interrupted run
                    continue
                if "tick" in r:
                    seg[r["tick"]] = r["s"]
                elif r.get("segment") or r.get("summary"):
                    fn = r.get("n", fn)  # the segment header names n; the summary repeats it
                    host = r.get("cpu", host)
        if fn is None or (n is not None and fn != n):
            continue  # no header (or another cluster size): not part of the run
        n = fn
        ticks.update(seg)
    if not ticks or n is None:
        return None
    secs = sum(ticks.values())
    return {"value": n * len(ticks) / secs, "unit": "node-ticks/s", "cores": 1, "kind": "port", "n": n,
            "ticks": f"{min(ticks)}..{max(ticks)} ({len(ticks)} ticks)", "seconds": round(secs, 1),
            "host": host, "source": "profiles/cpu_hour/cpu_hour_seg*.jsonl (scripts/cpu_hour.py)",
            "stitched": "25-tick segments run in separate calls; each segment after the first starts from "
                        "the GPU-reached state of its first tick (gm_read_* -> oc_load_scaled), so the "
                        "100 ticks are not one CPU process: read the value as seconds per tick"}


def main_partial(a):
    """Scenario S-C (BASELINE.json configs[4]): N = 16,777,216 nodes
    with V = 32-entry partial views (GM_MODE_PARTIAL, oracle/ref_cpu.c "PARTIAL"),
    5 % per-entry message drop on every tick, the S-A crash schedule (1 % at tick 10).
    One step = one tick of gm_p_tick (+ the S2 precompute gm_p_mtgen)."""
    rtx = Roctx()
    rtx.pause()
    rank, world, local = rank_env(a)
    from membership import GM_MODE_PARTIAL, Simulator, crash_set, load_library
    from membership.abi import comm_unique_id
    from membership.sharded import rendezvous_uid
    load_library()
    dist = None
    if world > 1:  # row shards; RCCL all-to-all(v) inside libgm, gloo for rendezvous + timing
        import torch.distributed as tdist
        tdist.init_process_group("gloo")
        dist = tdist
    n = a.cluster or (1 << 24)
    V = a.view
    ncrash = int(round(n * a.crash_frac))
    t0 = max(a.t0, 5)
    kw = dict(rd_seed=7, view=V, view_seed=5, init_mode=1, init_t0=t0, init_seed=11,
              drop_pct=5, drop_from=0, drop_to=1 << 20, drop_seed=42)
    if a.force_shard and world == 1:  # diagnostics: the row-shard exchange with one RCCL rank
        os.environ["GM_FORCE_SHARD"] = "1"
    sim = Simulator(n, GM_MODE_PARTIAL, device=local, shard_rank=rank, shard_count=world, **kw)
    sim.keep_events(0)  # views churn ~V joins per node and tick: never staged in the bench
    if world > 1 or a.force_shard:
        sim.comm_init(rendezvous_uid(rank, world) if world > 1 else comm_unique_id(), world, rank)
    crash = crash_set(n, ncrash, 42)
    while sim.time <= a.prologue:
        t = sim.time
        sim.tick()
        if t == a.crash_tick:
            sim.set_failed(crash)
    for _ in range(a.warmup):
        sim.tick()
    sim.sync()
    if dist is not None:
        dist.barrier()
    sim.sync()
    sim.set_timing(1)
    rtx.resume()
    t_0 = time.perf_counter()
    for _ in range(a.steps):
        sim.tick()
    sim.sync()
    t_1 = time.perf_counter()
    rtx.pause()
    elapsed = t_1 - t_0
    kernel_ms = sim.last_kernel_ms()
    st = sim.tick_stats()
    assert st["err"] == 0, st
    n_live, m_lists = st["live"], st["lists"]
    ranks = gather_ranks(dist, {"rank": rank, "local_rank": local, **sim.comm_info(), "kernel_ms": kernel_ms,
                                "nodes": sim.shard_layout()[1], "elapsed_s": elapsed,
                                "exchange_bytes": sim.exchange_bytes() if (world > 1 or a.force_shard) else 0})
    if dist is not None:  # max time over ranks; this rank's kernel bytes, whole-cluster counts
        import torch
        dist.barrier()
        x = torch.tensor([elapsed, float(n_live), float(m_lists), float(st["max_inbox"])], dtype=torch.float64)
        y = x.clone()
        dist.all_reduce(x, op=dist.ReduceOp.SUM)
        dist.all_reduce(y, op=dist.ReduceOp.MAX)
        elapsed = float(y[0])
        st["max_inbox"] = int(y[3])
        n_live_all, m_lists_all = int(x[1]), int(x[2])
    else:
        n_live_all, m_lists_all = n_live, m_lists
    # algorithmic bytes of one gm_p_tick launch: per live node the own
    # list read + the new list written (2 x 8V B) + inbox/state/S2/targets/stat words (120 B);
    # per delivered list the sender's list (8V B) + its inbox word
    b_alg = n_live * (16 * V + 120) + m_lists * (8 * V + 4)
    achieved = b_alg / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else None
    traffic, traffic_src = None, None  # PMC FETCH_SIZE/WRITE_SIZE of the same tick (committed passes; N=16M, V=32 only)
    tpath = os.path.join(REPO, "profiles", f"traffic_sc_n{n}.json")
    if world == 1 and V == 32 and os.path.exists(tpath):
        with open(tpath) as f:
            tj = json.load(f)
        if tj.get("layout") == "partial-v32":
            traffic = tj.get("hbm_bytes_per_launch")
            traffic_src = f"profiles/traffic_sc_n{n}.json ({tj.get('generated', 'r01')}, rocprofv3 --pmc passes by scripts/gpu.sh pmc_sc)"
    out = {
        "metric": "simulated node-ticks/sec (S-C partial view)",
        "value": n * a.steps / elapsed,
        "unit": "node-ticks/s",
        "value_note": "all N simulated nodes per tick, the 1% crashed (frozen) ones included; "
                      "live-only rate = value * live / n",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u64 view entries (id<<32|hb, integer)",
        "data": "synthetic (warm random V-entry views, seeded crash set, keyed 5% drops)",
        "config": {"workload": f"S-C: PARTIAL V={V} views, 5% per-entry drop, 1% crash at tick {a.crash_tick}, "
                               "fanout 5, TFAIL 5, TREMOVE 20",
                   "n": n, "view": V, "start": f"warm t0={t0}", "prologue_to_tick": a.prologue, "crashed": ncrash,
                   "live": n_live_all, "lists_per_tick": m_lists_all, "max_inbox": st["max_inbox"],
                   "parallelism": f"row-shard x{world} (RCCL all-to-allv of lists)" if world > 1 else "single GPU"},
        "ranks": ranks,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                     "frac": (achieved / PEAK_HBM_GBPS) if achieved else None, "traffic": traffic,
                     "traffic_source": traffic_src,
                     "kernel": "gm_p_tick", "kernel_ms": kernel_ms, "alg_bytes_per_launch": b_alg,
                     "achieved_basis": "algorithmic bytes per launch / kernel time",
                     "note": "instruction-issue bound, not HBM bound (PMC SQ mix per node, "
                             "profiles/r05/gate_close/mix_sc_small_per_dispatch.txt; DESIGN.md PARTIAL); the "
                             "contract's bound field only offers hbm|mfma"},
    }
    if world > 1:
        out["roofline"]["note"] = "rank 0's local kernels (its n/G nodes)"
    if a.pmc and world == 1:
        sim.close()  # the PMC passes are child processes with their own context
        try:
            out["roofline"]["traffic"], out["roofline"]["traffic_source"] = live_traffic(
                "gm_p_tick", "partial-v32", n, ["--scenario", "S-C", "--cluster", str(n), "--view", str(V)])
        except Exception as e:  # no profiler / counters on this host: the committed figure stands, said so
            out["roofline"]["traffic_source"] = f"{traffic_src} (live PMC passes failed: {type(e).__name__})"
    if rank == 0 and world == 1 and not a.no_cpu:
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import oracle_py  # the oracle is the CPU baseline here, never the measured path
        ns = min(n, 1 << 17)
        ora = oracle_py.PartialOracle(ns, v=V, rd_seed=7, view_seed=5, init_t0=t0, init_seed=11,
                                      drop_pct=5, drop_from=0, drop_to=1 << 20, drop_seed=42)
        ora.tick()  # first tick: empty inboxes
        ora.tick()
        ticks, secs = 0, 0.0
        while secs < a.cpu_seconds and ticks < 8:
            c0 = time.perf_counter()
            ora.tick()
            secs += time.perf_counter() - c0
            ticks += 1
        out["cpu_baseline"] = {"value": ns * ticks / secs, "unit": "node-ticks/s", "cores": 1, "kind": "port",
                               "host": host_cpu(),
                               "sample": f"{ticks} steady ticks of an N={ns} S-C cluster (V={V}, 5% drop) on one host "
                                         f"core ({secs:.1f} s, oracle/ref_cpu.c op_tick)"}
    if rank == 0:
        emit(out)
    sim.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
