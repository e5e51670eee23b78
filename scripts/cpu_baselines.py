"""CPU baselines of BASELINE.md's plan (TEST INFRASTRUCTURE: times the oracle and the
seeded reference build, never the product path).

1. FAITHFUL, the three testcases + N = 70 (the largest cluster the reference keeps
   converged): 700 ticks of
     - oracle/_ref/Application_seeded  -- the reference's own sources, -O0, seed shim
       (oracle/Makefile.ref; kind "reference"),
     - oracle/build/ref_cpu            -- the clean-room restatement, -O2 (kind "port"),
     - ./Application                   -- this build on the GPU (only with --gpu).
2. SCALED: node-ticks/s of the restatement's full-membership tick on one host core at
   several N (oc_bench_sample: 5 delivered lists per node, merge + sweep + draw), the
   per-tick time 100 * N / rate fitted as a power law in N, and the largest N whose
   100 ticks fit in one hour -- then a confirming sample at that N.

Prints one JSON document (host CPU model and the cores used included).
Usage: python scripts/cpu_baselines.py [--gpu] [--out FILE]
"""
import argparse
import json
import math
import os
import platform
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))

CASES = {
    "singlefailure": "MAX_NNB: 10\nSINGLE_FAILURE: 1\nDROP_MSG: 0\nMSG_DROP_PROB: 0.1 \n",
    "multifailure": "MAX_NNB: 10\nSINGLE_FAILURE: 0\nDROP_MSG: 0\nMSG_DROP_PROB: 0.1 \n",
    "msgdropsinglefailure": "MAX_NNB: 10\nSINGLE_FAILURE: 1\nDROP_MSG: 1\nMSG_DROP_PROB: 0.1 \n",
    "n70_singlefailure": "MAX_NNB: 70\nSINGLE_FAILURE: 1\nDROP_MSG: 0\nMSG_DROP_PROB: 0.1 \n",
}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def time_binary(exe, conf, reps=3, env_extra=None):
    """Best-of-reps wall time of one 700-tick run of an ./Application-shaped binary."""
    best = None
    with tempfile.TemporaryDirectory() as td:
        cpath = os.path.join(td, "case.conf")
        with open(cpath, "w") as f:
            f.write(conf)
        env = dict(os.environ, TIME_SEED="1", RD_SEED="1", **(env_extra or {}))
        for _ in range(reps):
            t0 = time.perf_counter()
            subprocess.run([exe, cpath], cwd=td, env=env, check=True, stdout=subprocess.DEVNULL)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
    return best


def faithful(gpu):
    bins = {
        "reference": os.path.join(ROOT, "oracle", "_ref", "Application_seeded"),
        "port": os.path.join(ROOT, "oracle", "build", "ref_cpu"),
    }
    if gpu:
        bins["gpu_application"] = os.path.join(ROOT, "Application")
    out = {}
    for name, conf in CASES.items():
        row = {}
        for kind, exe in bins.items():
            if not os.path.exists(exe):
                row[kind] = None
                continue
            n = int(conf.split("\n")[0].split(":")[1])
            row[kind] = round(time_binary(exe, conf, reps=3 if n <= 10 else 1), 4)
        n = int(conf.split("\n")[0].split(":")[1])
        row["node_ticks"] = n * 700
        out[name] = row
    return out


def scaled(sizes, seconds):
    import oracle_py

    pts = []
    for n in sizes:
        nodes, secs = oracle_py.bench_sample(n, lists=5, min_seconds=seconds)
        rate = nodes / secs
        pts.append({"n": n, "node_ticks_per_s": round(rate, 2), "s_per_tick": round(n / rate, 3),
                    "sample": f"{nodes} node-ticks in {secs:.1f} s"})
    # power-law fit of s/tick over the two largest sizes (merge cost is ~N per node-tick)
    a, b = pts[-2], pts[-1]
    k = math.log(b["s_per_tick"] / a["s_per_tick"]) / math.log(b["n"] / a["n"])
    n_hour = int(b["n"] * (36.0 / b["s_per_tick"]) ** (1.0 / k))
    nodes, secs = oracle_py.bench_sample(n_hour, lists=5, min_seconds=seconds)
    rate = nodes / secs
    confirm = {"n": n_hour, "node_ticks_per_s": round(rate, 2), "s_per_tick": round(n_hour / rate, 2),
               "projected_100_ticks_s": round(100 * n_hour / rate, 0),
               "sample": f"{nodes} node-ticks in {secs:.1f} s"}
    return {"points": pts, "exponent": round(k, 3), "n_100_ticks_in_1h": confirm}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpu", action="store_true", help="also time this build's ./Application")
    ap.add_argument("--sizes", default="4096,8192,16384")
    ap.add_argument("--seconds", type=float, default=6.0)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    res = {
        "host": {"cpu_model": cpu_model(), "cpus_visible": len(os.sched_getaffinity(0)), "cores_used": 1},
        "faithful_700_ticks_s": faithful(a.gpu),
        "scaled_full_membership": scaled([int(x) for x in a.sizes.split(",")], a.seconds),
    }
    txt = json.dumps(res, indent=1)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
