"""ctypes binding of the oracle (oracle/ref_cpu.h) -- TEST INFRASTRUCTURE ONLY."""
import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
LIB = os.path.join(ORACLE_DIR, "build", "liboracle.so")
CLI = os.path.join(ORACLE_DIR, "build", "ref_cpu")
OC_FAITHFUL, OC_SCALED = 0, 1


class OcConfig(ctypes.Structure):
    _fields_ = [("mode", ctypes.c_int), ("n", ctypes.c_int), ("single_failure", ctypes.c_int),
                ("drop_msg", ctypes.c_int), ("drop_prob", ctypes.c_double), ("time_seed", ctypes.c_uint32),
                ("rd_seed", ctypes.c_uint64), ("crash_tick", ctypes.c_int), ("crash_count", ctypes.c_int),
                ("crash_seed", ctypes.c_uint64), ("drop_pct", ctypes.c_int), ("drop_from", ctypes.c_int),
                ("drop_to", ctypes.c_int), ("drop_seed", ctypes.c_uint64), ("init_mode", ctypes.c_int),
                ("init_t0", ctypes.c_int), ("init_seed", ctypes.c_uint64)]


class OpConfig(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("v", ctypes.c_int), ("rd_seed", ctypes.c_uint64),
                ("view_seed", ctypes.c_uint64), ("init_t0", ctypes.c_int), ("init_seed", ctypes.c_uint64),
                ("crash_tick", ctypes.c_int), ("crash_count", ctypes.c_int), ("crash_seed", ctypes.c_uint64),
                ("drop_pct", ctypes.c_int), ("drop_from", ctypes.c_int), ("drop_to", ctypes.c_int),
                ("drop_seed", ctypes.c_uint64)]


class OcEvent(ctypes.Structure):
    _fields_ = [("t", ctypes.c_int32), ("logger", ctypes.c_int32), ("kind", ctypes.c_int32),
                ("subject", ctypes.c_int32)]


_lib = None


def ensure_built():
    if not (os.path.exists(LIB) and os.path.exists(CLI)):
        subprocess.run(["make", "-C", ORACLE_DIR], check=True, capture_output=True)


def lib():
    global _lib
    if _lib is None:
        ensure_built()
        L = ctypes.CDLL(LIB)
        P = ctypes.POINTER
        L.oc_create.argtypes = [P(OcConfig)]
        L.oc_create.restype = ctypes.c_void_p
        L.oc_destroy.argtypes = [ctypes.c_void_p]
        L.oc_tick.argtypes = [ctypes.c_void_p]
        L.oc_time.argtypes = [ctypes.c_void_p]
        for f in ("oc_dbg_log", "oc_stdout", "oc_msgcount", "oc_dump"):
            getattr(L, f).argtypes = [ctypes.c_void_p, P(ctypes.c_size_t)]
            getattr(L, f).restype = ctypes.c_void_p
        L.oc_events.argtypes = [ctypes.c_void_p, P(P(OcEvent))]
        L.oc_events.restype = ctypes.c_size_t
        L.oc_row.argtypes = [ctypes.c_void_p, ctypes.c_int, P(ctypes.c_int32), P(ctypes.c_int32)]
        L.oc_node.argtypes = [ctypes.c_void_p, ctypes.c_int, P(ctypes.c_int32)]
        L.oc_quirks.argtypes = [ctypes.c_void_p, P(ctypes.c_int64)]
        L.oc_set_failed.argtypes = [ctypes.c_void_p, P(ctypes.c_int32), ctypes.c_int]
        L.oc_targets.argtypes = [ctypes.c_void_p, P(ctypes.c_int32), P(ctypes.c_int32)]
        L.oc_load_scaled.argtypes = [ctypes.c_void_p, ctypes.c_int] + [P(ctypes.c_int32)] * 6
        L.oc_last_msgcount.argtypes = [ctypes.c_void_p, P(ctypes.c_int32), P(ctypes.c_int32)]
        L.op_last_msgcount.argtypes = [ctypes.c_void_p, P(ctypes.c_int32), P(ctypes.c_int32)]
        L.op_last_msgcount.restype = None
        L.oc_quirks.restype = None
        L.oc_crash_set.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint64, P(ctypes.c_int32)]
        L.oc_srand.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        L.oc_rand_next.argtypes = [ctypes.c_void_p]
        L.oc_rand_next.restype = ctypes.c_int32
        L.oc_rd_seed.argtypes = [ctypes.c_uint64, ctypes.c_int32, ctypes.c_int32]
        L.oc_rd_seed.restype = ctypes.c_uint32
        L.oc_mt_uniform.argtypes = [ctypes.c_uint32, ctypes.c_int, ctypes.c_int, P(ctypes.c_int32)]
        L.op_create.argtypes = [P(OpConfig)]
        L.op_create.restype = ctypes.c_void_p
        L.op_destroy.argtypes = [ctypes.c_void_p]
        L.op_tick.argtypes = [ctypes.c_void_p]
        L.op_time.argtypes = [ctypes.c_void_p]
        L.op_dump.argtypes = [ctypes.c_void_p, P(ctypes.c_size_t)]
        L.op_dump.restype = ctypes.c_void_p
        L.op_events.argtypes = [ctypes.c_void_p, P(P(OcEvent))]
        L.op_events.restype = ctypes.c_size_t
        L.op_evict_key.argtypes = [ctypes.c_uint64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]
        L.op_evict_key.restype = ctypes.c_uint64
        _lib = L
    return _lib


def _i32p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))


class Oracle:
    def __init__(self, n, mode=OC_FAITHFUL, single_failure=1, drop_msg=0, drop_prob=0.1, time_seed=0, rd_seed=0,
                 crash_tick=-1, crash_count=0, crash_seed=0, drop_pct=0, drop_from=0, drop_to=0, drop_seed=0,
                 init_mode=0, init_t0=0, init_seed=0):
        self.L = lib()
        cfg = OcConfig(mode, n, single_failure, drop_msg, drop_prob, time_seed & 0xFFFFFFFF, rd_seed, crash_tick,
                       crash_count, crash_seed, drop_pct, drop_from, drop_to, drop_seed, init_mode, init_t0, init_seed)
        self.h = self.L.oc_create(ctypes.byref(cfg))
        if not self.h:
            raise ValueError("oc_create failed")
        self.n = n

    def close(self):
        if self.h:
            self.L.oc_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def tick(self):
        if self.L.oc_tick(self.h):
            raise RuntimeError("oc_tick")

    @property
    def time(self):
        return self.L.oc_time(self.h)

    def _buf(self, fn):
        n = ctypes.c_size_t()
        p = getattr(self.L, fn)(self.h, ctypes.byref(n))
        return ctypes.string_at(p, n.value) if n.value else b""

    def dump(self):
        return self._buf("oc_dump")

    def quirks(self):
        """(updateMyPos quirk firings so far, largest start-tick gap self -> rewritten entry)"""
        out = (ctypes.c_int64 * 2)()
        self.L.oc_quirks(self.h, out)
        return int(out[0]), int(out[1])

    def dbg(self):
        return self._buf("oc_dbg_log")

    def events(self):
        p = ctypes.POINTER(OcEvent)()
        n = self.L.oc_events(self.h, ctypes.byref(p))
        return [(p[k].t, p[k].logger, p[k].kind, p[k].subject) for k in range(n)]

    def row(self, r):
        hb = np.zeros(self.n, dtype=np.int32)
        ts = np.zeros(self.n, dtype=np.int32)
        self.L.oc_row(self.h, r, _i32p(hb), _i32p(ts))
        return hb, ts

    def table(self):
        """(hb, ts) int32 [n][n], -1 = absent: every observer's member list, dense"""
        hb = np.empty((self.n, self.n), dtype=np.int32)
        ts = np.empty((self.n, self.n), dtype=np.int32)
        for r in range(self.n):
            self.L.oc_row(self.h, r, _i32p(hb[r]), _i32p(ts[r]))
        return hb, ts

    def nodes(self):
        """[n][4] inited / inGroup / failed / heartbeat"""
        st = np.empty((self.n, 4), dtype=np.int32)
        for r in range(self.n):
            self.L.oc_node(self.h, r, _i32p(st[r]))
        return st

    def node(self, r):
        st = np.zeros(4, dtype=np.int32)
        self.L.oc_node(self.h, r, _i32p(st))
        return st

    def set_failed(self, idx):
        """SCALED: fail these nodes at the end of the tick just run"""
        a = np.ascontiguousarray(idx, dtype=np.int32)
        if self.L.oc_set_failed(self.h, _i32p(a), len(a)):
            raise ValueError("oc_set_failed")

    def targets(self):
        """SCALED: (targets int32 [n][5], counts [n]) drawn in the last tick"""
        tg = np.zeros((self.n, 5), dtype=np.int32)
        cnt = np.zeros(self.n, dtype=np.int32)
        if self.L.oc_targets(self.h, _i32p(tg), _i32p(cnt)):
            raise RuntimeError("oc_targets: SCALED only")
        return tg, cnt

    def load_state(self, t, hb, ts, heartbeat, failed, targets, counts):
        """SCALED (no join ramp): replace the state between ticks (oc_load_scaled); tick t runs next.
        hb / ts [n][n] (-1 absent), heartbeat / failed [n], targets [n][5], counts [n]."""
        arrs = [np.ascontiguousarray(a, dtype=np.int32) for a in (hb, ts, heartbeat, failed, targets, counts)]
        if self.L.oc_load_scaled(self.h, t, *[_i32p(a) for a in arrs]):
            raise ValueError("oc_load_scaled")

    def last_msgcount(self):
        """SCALED: per-node gossip entries sent (before loss) / received (after loss) last tick"""
        sent = np.zeros(self.n, dtype=np.int32)
        recv = np.zeros(self.n, dtype=np.int32)
        if self.L.oc_last_msgcount(self.h, _i32p(sent), _i32p(recv)):
            raise RuntimeError("oc_last_msgcount: SCALED only")
        return sent, recv


class PartialOracle:
    """PARTIAL mode (V-entry views, scenario S-C): the oracle IS the specification."""

    def __init__(self, n, v=32, rd_seed=7, view_seed=5, init_t0=8, init_seed=11, crash_tick=-1, crash_count=0,
                 crash_seed=42, drop_pct=0, drop_from=0, drop_to=0, drop_seed=0):
        self.L = lib()
        cfg = OpConfig(n, v, rd_seed, view_seed, init_t0, init_seed, crash_tick, crash_count, crash_seed, drop_pct,
                       drop_from, drop_to, drop_seed)
        self.h = self.L.op_create(ctypes.byref(cfg))
        if not self.h:
            raise ValueError("op_create failed")
        self.n = n

    def close(self):
        if self.h:
            self.L.op_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def tick(self):
        self.L.op_tick(self.h)

    @property
    def time(self):
        return self.L.op_time(self.h)

    def dump(self):
        n = ctypes.c_size_t()
        p = self.L.op_dump(self.h, ctypes.byref(n))
        return ctypes.string_at(p, n.value) if n.value else b""

    def events(self):
        p = ctypes.POINTER(OcEvent)()
        n = self.L.op_events(self.h, ctypes.byref(p))
        return [(p[k].t, p[k].logger, p[k].kind, p[k].subject) for k in range(n)]

    def last_msgcount(self):
        """per-node entries sent (before loss) / received (after loss) in the last tick"""
        sent = np.zeros(self.n, dtype=np.int32)
        recv = np.zeros(self.n, dtype=np.int32)
        self.L.op_last_msgcount(self.h, _i32p(sent), _i32p(recv))
        return sent, recv


def crash_set(n, count, seed):
    out = np.zeros(max(count, 1), dtype=np.int32)
    lib().oc_crash_set(n, count, seed, _i32p(out))
    return out[:count]


def glibc_rand(seed, k):
    L = lib()
    st = ctypes.create_string_buffer(256)
    L.oc_srand(st, seed)
    return np.array([L.oc_rand_next(st) for _ in range(k)], dtype=np.int32)


def mt_uniform(seed, n, k):
    out = np.zeros(k, dtype=np.int32)
    lib().oc_mt_uniform(seed, n, k, _i32p(out))
    return out


def run_cli(conf_text, time_seed, rd_seed, workdir, dump=False):
    """Run the oracle's ./Application-shaped CLI; returns (dbg, msgcount, stdout, dump)."""
    ensure_built()
    cpath = os.path.join(workdir, "case.conf")
    with open(cpath, "w") as f:
        f.write(conf_text)
    env = dict(os.environ, TIME_SEED=str(time_seed), RD_SEED=str(rd_seed))
    if dump:
        env["DUMP_FILE"] = os.path.join(workdir, "tables.txt")
    p = subprocess.run([CLI, cpath], cwd=workdir, env=env, capture_output=True, check=True)
    rd = lambda name: open(os.path.join(workdir, name), "rb").read()  # noqa: E731
    return rd("dbg.log"), rd("msgcount.log"), p.stdout, (rd("tables.txt") if dump else None)


def bench_sample(n, lists=5, max_nodes=1000000, min_seconds=10.0):
    """Time node-ticks of the SCALED workload on one host core (bench cpu_baseline leg)."""
    L = lib()
    L.oc_bench_sample.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                  ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_double)]
    nodes, secs = ctypes.c_int(), ctypes.c_double()
    if L.oc_bench_sample(n, lists, max_nodes, min_seconds, ctypes.byref(nodes), ctypes.byref(secs)):
        raise RuntimeError("oc_bench_sample")
    return nodes.value, secs.value
