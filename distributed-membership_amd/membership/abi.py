"""ctypes binding of include/gm_abi.h (libgm.so)."""
import ctypes
import os

import numpy as np

GM_ABI_VERSION = 2
GM_MODE_FAITHFUL, GM_MODE_SCALED, GM_MODE_PARTIAL = 0, 1, 2
GM_EV_JOINED, GM_EV_REMOVED, GM_EV_START_GROUP, GM_EV_TRY_JOIN, GM_EV_TIME_MARK = 1, 2, 3, 4, 5
GM_OK, GM_ERANGE = 0, -4

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def lib_path():
    return os.environ.get("GM_LIBRARY", os.path.join(_PKG, "lib", "libgm.so"))


class GmConfig(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_int32), ("mode", ctypes.c_int32), ("n", ctypes.c_int32),
                ("single_failure", ctypes.c_int32), ("drop_msg", ctypes.c_int32), ("drop_prob", ctypes.c_double),
                ("time_seed", ctypes.c_uint32), ("rd_seed", ctypes.c_uint64),
                ("drop_pct", ctypes.c_int32), ("drop_from", ctypes.c_int32), ("drop_to", ctypes.c_int32),
                ("drop_seed", ctypes.c_uint64),
                ("device", ctypes.c_int32), ("shard_rank", ctypes.c_int32), ("shard_count", ctypes.c_int32),
                ("init_mode", ctypes.c_int32), ("init_t0", ctypes.c_int32), ("init_seed", ctypes.c_uint64),
                ("band", ctypes.c_int32), ("view", ctypes.c_int32), ("view_seed", ctypes.c_uint64),
                ("device_share", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class GmEvent(ctypes.Structure):
    _fields_ = [("t", ctypes.c_int32), ("logger", ctypes.c_int32), ("kind", ctypes.c_int32),
                ("subject", ctypes.c_int32)]


EXPORTS = ["gm_parse_conf", "gm_create", "gm_destroy", "gm_tick", "gm_sync", "gm_time", "gm_rand", "gm_set_failed",
           "gm_set_dropmsg", "gm_drain_events", "gm_event_counts", "gm_msgcount", "gm_read_row", "gm_read_table", "gm_read_nodes",
           "gm_dump_tables", "gm_tick_stats", "gm_set_timing", "gm_last_kernel_ms", "gm_crash_set", "gm_strerror",
           "gm_comm_unique_id", "gm_comm_init", "gm_shard_layout", "gm_shard_merge", "gm_shard_draw",
           "gm_shard_accept", "gm_shard_end_tick", "gm_shard_loopback", "gm_partial_loopback_tick",
           "gm_shard_exchange_bytes", "gm_keep_events", "gm_event_totals", "gm_read_views", "gm_shard_stub",
           "gm_msgcount_record", "gm_comm_info", "gm_shard_export", "gm_shard_import", "gm_pool_info", "gm_shard_loopback_tick", "gm_read_targets"]

_lib = None


class GmError(RuntimeError):
    def __init__(self, code, what):
        self.code = code
        super().__init__(f"{what}: {load_library().gm_strerror(code).decode()} ({code})")


def load_library():
    """Load libgm.so (built in-tree by `make` / __graft_entry__.build()); raises if absent."""
    global _lib
    if _lib is not None:
        return _lib
    path = lib_path()
    if not os.path.exists(path):
        raise FileNotFoundError(f"libgm.so not built: {path} (run `make` at the repo root)")
    lib = ctypes.CDLL(path)
    P = ctypes.POINTER
    i32, u64, sz = ctypes.c_int32, ctypes.c_uint64, ctypes.c_size_t
    sig = {
        "gm_parse_conf": [ctypes.c_char_p, P(GmConfig)],
        "gm_create": [P(GmConfig), P(ctypes.c_void_p)],
        "gm_destroy": [ctypes.c_void_p], "gm_tick": [ctypes.c_void_p], "gm_sync": [ctypes.c_void_p],
        "gm_time": [ctypes.c_void_p, P(i32)], "gm_rand": [ctypes.c_void_p, P(i32)],
        "gm_set_failed": [ctypes.c_void_p, P(i32), i32], "gm_set_dropmsg": [ctypes.c_void_p, i32],
        "gm_drain_events": [ctypes.c_void_p, P(GmEvent), sz, P(sz)],
        "gm_event_counts": [ctypes.c_void_p, P(u64)], "gm_event_totals": [ctypes.c_void_p, P(u64)],
        "gm_keep_events": [ctypes.c_void_p, i32], "gm_shard_stub": [ctypes.c_void_p, i32], "gm_read_views": [ctypes.c_void_p, i32, i32, P(u64)],
        "gm_msgcount": [ctypes.c_void_p, i32, P(i32), P(i32)],
        "gm_msgcount_record": [ctypes.c_void_p, i32],
        "gm_read_row": [ctypes.c_void_p, i32, i32, i32, P(i32), P(i32)],
        "gm_read_table": [ctypes.c_void_p, i32, i32, P(i32), P(i32)],
        "gm_read_nodes": [ctypes.c_void_p, P(i32)], "gm_read_targets": [ctypes.c_void_p, P(i32), P(i32)],
        "gm_dump_tables": [ctypes.c_void_p, ctypes.c_char_p, sz, P(sz)],
        "gm_tick_stats": [ctypes.c_void_p, P(ctypes.c_int64)], "gm_pool_info": [ctypes.c_void_p, P(ctypes.c_int64)],
        "gm_set_timing": [ctypes.c_void_p, i32], "gm_last_kernel_ms": [ctypes.c_void_p, P(ctypes.c_float)],
        "gm_crash_set": [i32, i32, u64, P(i32)],
        "gm_comm_unique_id": [ctypes.c_char_p],
        "gm_comm_init": [ctypes.c_void_p, ctypes.c_char_p, i32, i32],
        "gm_comm_info": [ctypes.c_void_p, P(i32)],
        "gm_shard_export": [ctypes.c_void_p, i32, i32, ctypes.c_void_p, sz, P(sz)],
        "gm_shard_import": [ctypes.c_void_p, i32, i32, ctypes.c_void_p, sz],
        "gm_shard_layout": [ctypes.c_void_p, P(i32), P(i32)],
        "gm_shard_loopback": [P(ctypes.c_void_p), i32, i32, i32],
        "gm_partial_loopback_tick": [P(ctypes.c_void_p), i32], "gm_shard_loopback_tick": [P(ctypes.c_void_p), i32],
        "gm_shard_exchange_bytes": [ctypes.c_void_p, P(ctypes.c_int64)],
        "gm_shard_merge": [ctypes.c_void_p], "gm_shard_draw": [ctypes.c_void_p, i32, i32],
        "gm_shard_accept": [ctypes.c_void_p, i32, P(i32)], "gm_shard_end_tick": [ctypes.c_void_p],
    }
    # GM_AB_BUILD=1 (A/B scripts only): an older measurement build may lack newer entry points, which
    # are then left unbound. Otherwise every entry point must be present, whatever library GM_LIBRARY
    # names, so a stale libgm fails here and not at its first call of a missing symbol
    ab_build = os.environ.get("GM_AB_BUILD") == "1"
    for name, args in sig.items():
        if ab_build and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = ctypes.c_int
    lib.gm_strerror.argtypes = [ctypes.c_int]
    lib.gm_strerror.restype = ctypes.c_char_p
    _lib = lib
    return lib


def _ptr(a, ct=ctypes.c_int32):
    return a.ctypes.data_as(ctypes.POINTER(ct))


def crash_set(n, count, seed):
    lib = load_library()
    out = np.zeros(max(count, 1), dtype=np.int32)
    rc = lib.gm_crash_set(n, count, seed, _ptr(out))
    if rc:
        raise GmError(rc, "gm_crash_set")
    return out[:count]


class Simulator:
    """One libgm context: the whole cluster's MP1Node/EmulNet state on one GPU (or shard)."""

    def __init__(self, n, mode=GM_MODE_FAITHFUL, single_failure=1, drop_msg=0, drop_prob=0.1, time_seed=0,
                 rd_seed=0, drop_pct=0, drop_from=0, drop_to=0, drop_seed=0, device=0, shard_rank=0, shard_count=1,
                 init_mode=0, init_t0=0, init_seed=0, band=0, view=0, view_seed=0, device_share=0):
        self.lib = load_library()
        cfg = GmConfig()
        cfg.abi_version = GM_ABI_VERSION
        cfg.mode, cfg.n = mode, n
        cfg.single_failure, cfg.drop_msg, cfg.drop_prob = single_failure, drop_msg, drop_prob
        cfg.time_seed, cfg.rd_seed = time_seed & 0xFFFFFFFF, rd_seed
        cfg.drop_pct, cfg.drop_from, cfg.drop_to, cfg.drop_seed = drop_pct, drop_from, drop_to, drop_seed
        cfg.device, cfg.shard_rank, cfg.shard_count = device, shard_rank, shard_count
        cfg.init_mode, cfg.init_t0, cfg.init_seed = init_mode, init_t0, init_seed
        cfg.band = band
        cfg.view, cfg.view_seed = view, view_seed
        cfg.device_share = device_share
        self.cfg = cfg
        self.n = n
        self.mode = mode
        h = ctypes.c_void_p()
        self._call("gm_create", ctypes.byref(cfg), ctypes.byref(h))
        self.h = h

    def _call(self, name, *args):
        rc = getattr(self.lib, name)(*args)
        if rc != GM_OK:
            raise GmError(rc, name)
        return rc

    def close(self):
        if getattr(self, "h", None):
            self.lib.gm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def tick(self):
        self._call("gm_tick", self.h)

    def sync(self):
        self._call("gm_sync", self.h)

    @property
    def time(self):
        t = ctypes.c_int32()
        self._call("gm_time", self.h, ctypes.byref(t))
        return t.value

    def rand(self):
        v = ctypes.c_int32()
        self._call("gm_rand", self.h, ctypes.byref(v))
        return v.value

    def set_failed(self, idx):
        a = np.ascontiguousarray(np.asarray(idx, dtype=np.int32))
        self._call("gm_set_failed", self.h, _ptr(a), len(a))

    def set_dropmsg(self, on):
        self._call("gm_set_dropmsg", self.h, 1 if on else 0)

    def drain_events(self):
        n = ctypes.c_size_t()
        rc = self.lib.gm_drain_events(self.h, None, 0, ctypes.byref(n))
        if rc == GM_OK:
            return []
        if rc != GM_ERANGE:
            raise GmError(rc, "gm_drain_events")
        buf = (GmEvent * n.value)()
        self._call("gm_drain_events", self.h, buf, n.value, ctypes.byref(n))
        return [(e.t, e.logger, e.kind, e.subject) for e in buf[:n.value]]

    def drain_events_np(self):
        """gm_drain_events into an int32 array [n, 4] of (t, logger, kind, subject)."""
        n = ctypes.c_size_t()
        rc = self.lib.gm_drain_events(self.h, None, 0, ctypes.byref(n))
        if rc == GM_OK:
            return np.zeros((0, 4), dtype=np.int32)
        if rc != GM_ERANGE:
            raise GmError(rc, "gm_drain_events")
        buf = np.empty((n.value, 4), dtype=np.int32)
        self._call("gm_drain_events", self.h, buf.ctypes.data_as(ctypes.POINTER(GmEvent)), n.value, ctypes.byref(n))
        return buf[:n.value]

    def keep_events(self, on):
        self._call("gm_keep_events", self.h, 1 if on else 0)

    def event_total(self):
        c = (ctypes.c_uint64 * 6)()
        self._call("gm_event_counts", self.h, c)
        return int(c[0])

    def event_counts(self):
        """Records of the last tick: [total, joined, removed, ...] (per kind where the mode has it)."""
        c = (ctypes.c_uint64 * 6)()
        self._call("gm_event_counts", self.h, c)
        return [int(x) for x in c]

    def event_totals(self):
        """Records since gm_create: {kind: count} (FAITHFUL, SCALED)."""
        c = (ctypes.c_uint64 * 6)()
        self._call("gm_event_totals", self.h, c)
        return {"total": int(c[0]), "joined": int(c[GM_EV_JOINED]), "removed": int(c[GM_EV_REMOVED])}

    def read_views(self, r0, count):
        """PARTIAL: raw views (id << 32 | hb, 0 = empty) of nodes [r0, r0 + count), uint64 [count, V]."""
        v = self.cfg.view or 32
        out = np.zeros((count, v), dtype=np.uint64)
        self._call("gm_read_views", self.h, r0, count, _ptr(out, ctypes.c_uint64))
        return out

    def msgcount_record(self, tmax):
        """SCALED / PARTIAL: record per-node entry counts for ticks < tmax (before the first tick)"""
        self._call("gm_msgcount_record", self.h, tmax)
        self._mc_tmax = tmax

    def msgcount_recording(self, t):
        return t < getattr(self, "_mc_tmax", 0)

    def msgcount(self, t, rows=None):
        """[rows][t] sent / recv entry messages per node and tick (rows: this context's nodes)"""
        rows = self.n if rows is None else rows
        sent = np.zeros((rows, t), dtype=np.int32)
        recv = np.zeros((rows, t), dtype=np.int32)
        self._call("gm_msgcount", self.h, t, _ptr(sent), _ptr(recv))
        return sent, recv

    def read_row(self, r, c0=0, length=None):
        length = self.n if length is None else length
        hb = np.zeros(length, dtype=np.int32)
        ts = np.zeros(length, dtype=np.int32)
        self._call("gm_read_row", self.h, r, c0, length, _ptr(hb), _ptr(ts))
        return hb, ts

    def read_table(self, r0=0, count=None):
        """(hb, ts) int32 [count][w] of rows [r0, r0 + count) over this context's columns, -1 = absent."""
        count = self.n - r0 if count is None else count
        w = self.shard_layout()[1] if self.mode == GM_MODE_SCALED else self.n
        hb = np.zeros((count, w), dtype=np.int32)
        ts = np.zeros((count, w), dtype=np.int32)
        self._call("gm_read_table", self.h, r0, count, _ptr(hb), _ptr(ts))
        return hb, ts

    def read_nodes(self):
        rows = self.shard_layout()[1] if self.mode == GM_MODE_PARTIAL else self.n  # a row shard: its own nodes
        st = np.zeros((rows, 4), dtype=np.int32)
        self._call("gm_read_nodes", self.h, _ptr(st))
        return st

    def read_targets(self):
        """SCALED: (targets int32 [n][5], counts int32 [n]) of the last tick (gm_read_targets)"""
        tg = np.zeros((self.n, 5), dtype=np.int32)
        cnt = np.zeros(self.n, dtype=np.int32)
        self._call("gm_read_targets", self.h, _ptr(tg), _ptr(cnt))
        return tg, cnt

    def dump_tables(self):
        n = ctypes.c_size_t()
        rc = self.lib.gm_dump_tables(self.h, None, 0, ctypes.byref(n))
        if rc not in (GM_OK, GM_ERANGE):
            raise GmError(rc, "gm_dump_tables")
        buf = ctypes.create_string_buffer(n.value + 1)
        self._call("gm_dump_tables", self.h, buf, n.value + 1, ctypes.byref(n))
        return buf.raw[:n.value]

    def tick_stats(self):
        s = (ctypes.c_int64 * 4)()
        self._call("gm_tick_stats", self.h, s)
        return {"lists": int(s[0]), "live": int(s[1]), "max_inbox": int(s[2]), "err": int(s[3])}

    def pool_info(self):
        """SCALED escape storage as sized at create (gm_pool_info)"""
        v = (ctypes.c_int64 * 4)()
        self._call("gm_pool_info", self.h, v)
        return {"dense": bool(v[0]), "table_pool_entries": int(v[1]), "payload_pool_slots": int(v[2]),
                "event_spill_records": int(v[3])}

    def set_timing(self, on):
        self._call("gm_set_timing", self.h, 1 if on else 0)

    def last_kernel_ms(self):
        v = ctypes.c_float()
        self._call("gm_last_kernel_ms", self.h, ctypes.byref(v))
        return float(v.value)

    # ---- column shards (SCALED multi-GPU; see membership.sharded)
    def comm_init(self, uid, nranks, rank):
        self._call("gm_comm_init", self.h, uid, nranks, rank)

    def comm_info(self):
        """{"ranks", "rank", "rccl_device", "device"} of the attached RCCL communicator (ranks 0: none)"""
        v = (ctypes.c_int32 * 4)()
        self._call("gm_comm_info", self.h, v)
        return {"ranks": v[0], "rank": v[1], "rccl_device": v[2], "device": v[3]}

    def shard_layout(self):
        c0, w = ctypes.c_int32(), ctypes.c_int32()
        self._call("gm_shard_layout", self.h, ctypes.byref(c0), ctypes.byref(w))
        return c0.value, w.value

    def shard_merge(self):
        self._call("gm_shard_merge", self.h)

    def shard_draw(self, rnd, d):
        self._call("gm_shard_draw", self.h, rnd, d)

    def shard_accept(self, d):
        v = ctypes.c_int32()
        self._call("gm_shard_accept", self.h, d, ctypes.byref(v))
        return v.value

    def exchange_bytes(self):
        v = ctypes.c_int64()
        self._call("gm_shard_exchange_bytes", self.h, ctypes.byref(v))
        return v.value

    def shard_stub(self, on):
        """Diagnostics: tick this column shard alone on its device (gm_shard_stub)."""
        self._call("gm_shard_stub", self.h, 1 if on else 0)

    def shard_export(self, what, d=0):
        """the phase exchange buffer `what` of this shard (gm_shard_export) as a flat int32 array"""
        nb = ctypes.c_size_t()
        self._call("gm_shard_export", self.h, what, d, None, 0, ctypes.byref(nb))
        out = np.empty(nb.value // 4, dtype=np.int32)
        self._call("gm_shard_export", self.h, what, d, out.ctypes.data_as(ctypes.c_void_p), nb.value, ctypes.byref(nb))
        return out

    def shard_import(self, what, arr, d=0):
        a = np.ascontiguousarray(arr, dtype=np.int32)
        self._call("gm_shard_import", self.h, what, d, a.ctypes.data_as(ctypes.c_void_p), a.nbytes)

    def shard_end_tick(self):
        self._call("gm_shard_end_tick", self.h)


def comm_unique_id():
    """ncclGetUniqueId (RCCL) as 128 bytes, to broadcast to every rank."""
    buf = ctypes.create_string_buffer(128)
    rc = load_library().gm_comm_unique_id(buf)
    if rc:
        raise GmError(rc, "gm_comm_unique_id")
    return buf.raw


def shard_loopback(sims, what, d=0):
    arr = (ctypes.c_void_p * len(sims))(*[s.h for s in sims])
    rc = load_library().gm_shard_loopback(arr, len(sims), what, d)
    if rc:
        raise GmError(rc, "gm_shard_loopback")


def shard_loopback_tick(sims):
    """One column-shard tick of G contexts on one device in the pipelined tick's chunk order."""
    arr = (ctypes.c_void_p * len(sims))(*[s.h for s in sims])
    rc = load_library().gm_shard_loopback_tick(arr, len(sims))
    if rc:
        raise GmError(rc, "gm_shard_loopback_tick")


def partial_loopback_tick(sims):
    """One PARTIAL tick of G row-shard contexts on one device (exchange by device copies)."""
    arr = (ctypes.c_void_p * len(sims))(*[s.h for s in sims])
    rc = load_library().gm_partial_loopback_tick(arr, len(sims))
    if rc:
        raise GmError(rc, "gm_partial_loopback_tick")
