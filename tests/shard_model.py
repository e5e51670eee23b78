"""A numpy model of the column-sharded SCALED tick (membership/sharded.py,
gm_s_band / gm_s_draw / gm_s_accept) -- TEST INFRASTRUCTURE.

Each instance owns subject columns [c0, c0+w) of every row and talks to the
other shards only through the two collectives of the protocol (all-gather of
per-row (present, numfailed), MAX-allreduce of resolved draws), supplied as
callables -- torch.distributed gloo in the multi-process CPU test. The S2
stream is a pure-Python mt19937 checked against the oracle's mt19937 + Lemire
restatement (tests/test_rng_kat.py)."""
import numpy as np

import oracle_py

TFAIL, TREMOVE, FANOUT = 5, 20, 5
M64 = (1 << 64) - 1


def fmix32(h):
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & 0xFFFFFFFF
    return h ^ (h >> 16)


def mix64(z):
    z &= M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def mt19937_outputs(seed, k):
    """First k outputs of std::mt19937(seed) (the S2 stream before Lemire)."""
    x = [seed & 0xFFFFFFFF]
    for i in range(1, 624):
        x.append((1812433253 * (x[-1] ^ (x[-1] >> 30)) + i) & 0xFFFFFFFF)
    out, idx = [], 624
    while len(out) < k:
        if idx == 624:
            for i in range(624):
                y = (x[i] & 0x80000000) | (x[(i + 1) % 624] & 0x7FFFFFFF)
                x[i] = x[(i + 397) % 624] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
            idx = 0
        v = x[idx]
        idx += 1
        v ^= v >> 11
        v ^= (v << 7) & 0x9D2C5680
        v ^= (v << 15) & 0xEFC60000
        v ^= v >> 18
        out.append(v & 0xFFFFFFFF)
    return out


def lemire_draws(seed, size, k):
    """libstdc++-11 uniform_int_distribution<int>(0, size-1) over mt19937_outputs (test helper)."""
    thr = ((1 << 32) - size) % size
    out = []
    for x in mt19937_outputs(seed, 4 * k + 64):
        prod = x * size
        if (prod & 0xFFFFFFFF) >= thr:
            out.append(prod >> 32)
            if len(out) == k:
                break
    return out


class ShardModel:
    def __init__(self, n, rank, world, rd_seed=7, drop_pct=0, drop_from=0, drop_to=0, drop_seed=0,
                 init_mode=0, init_t0=0, init_seed=0):
        self.n, self.rank, self.world = n, rank, world
        self.c0 = n * rank // world
        self.w = n * (rank + 1) // world - self.c0
        self.hb = np.zeros((n, self.w), np.int64)
        self.ts = np.zeros((n, self.w), np.int64)         # cold converged start: all present at {0, 0}
        t0 = init_t0 if init_mode == 1 else 0
        if init_mode == 1:                                 # warm converged start (gm_abi.h init_mode)
            for r in range(n):
                for j in range(self.w):
                    c = self.c0 + j
                    if c == r:
                        self.hb[r, j], self.ts[r, j] = 2 * t0 - 1, t0
                    else:
                        a = (mix64(init_seed ^ (r << 32) ^ c) >> 40) % 4
                        self.hb[r, j], self.ts[r, j] = 2 * (t0 - 1 - a) - 1, t0 - a
        self.pay = np.full((n, self.w), -1, np.int64)     # payload plane of the previous tick
        self.inbox = [[] for _ in range(n)]
        self.hbctr = np.full(n, 2 * t0, np.int64)
        self.failed = np.zeros(n, bool)
        self.rd_seed, self.drop = rd_seed, (drop_pct, drop_from, drop_to, drop_seed)
        self.t = t0 + 1
        self.events = []

    def _dropped(self, t_send, s, r, col):
        pct, lo, hi, seed = self.drop
        if pct <= 0 or not (lo <= t_send < hi):
            return False
        pair = mix64(seed ^ (t_send << 48) ^ (s << 24) ^ r) & 0xFFFFFFFF
        thresh = 65536 if pct >= 100 else (pct * 65536 + 99) // 100  # gm_device.h gm_drop_thresh
        return ((fmix32(pair ^ (((col >> 1) * 0x9E3779B9) & 0xFFFFFFFF)) >> (16 * (col & 1))) & 0xFFFF) < thresh

    def tick(self, all_gather, all_reduce_max):
        n, t, w, c0 = self.n, self.t, self.w, self.c0
        present = self.ts >= 0
        new_pay = np.full((n, w), -1, np.int64)
        counts = np.zeros((n, 2), np.int64)
        fresh = np.zeros((n, w), bool)
        self.events = []
        for r in range(n):
            if self.failed[r]:
                continue
            key = np.full(w, -1, np.int64)
            for s in self.inbox[r]:
                for j in range(w):
                    v = self.pay[s, j]
                    if v >= 0 and not self._dropped(t - 1, s, r, c0 + j):
                        key[j] = max(key[j], v)
            for j in range(w):
                if key[j] >= 0:
                    if not present[r, j]:
                        self.hb[r, j], self.ts[r, j] = key[j], t
                        present[r, j] = True
                        self.events.append((t, r, 1, c0 + j + 1))
                    elif key[j] > self.hb[r, j]:
                        self.hb[r, j], self.ts[r, j] = key[j], t
            if c0 <= r < c0 + w:
                self.hbctr[r] += 1
                self.hb[r, r - c0], self.ts[r, r - c0] = self.hbctr[r], t
                self.hbctr[r] += 1
            nf = 0
            for j in range(w):
                if not present[r, j]:
                    continue
                age = t - self.ts[r, j]
                if age >= TFAIL:
                    nf += 1
                    if age >= TREMOVE:
                        present[r, j] = False
                        self.ts[r, j] = self.hb[r, j] = -1
                        self.events.append((t, r, 2, c0 + j + 1))
                        continue
                else:
                    fresh[r, j] = True
                    new_pay[r, j] = self.hb[r, j]
            counts[r] = (present[r].sum(), nf)
        allc = all_gather(counts)                       # [world][n][2]
        size = allc[:, :, 0].sum(0)
        numpot = size - 1 - allc[:, :, 1].sum(0)
        cols = [np.nonzero(present[r])[0] for r in range(n)]
        drawn = [r for r in range(n) if not self.failed[r] and numpot[r] > 0]
        acc = {r: [] for r in drawn}
        targets = {r: [] for r in range(n)}
        # rounds over the S2 OUTPUTS of each row's mt19937 (gm_s_draw): round 0 the first
        # 16, round q >= 1 the next 64; -2 marks an output Lemire rejects (no draw)
        off, d = 0, 16
        while drawn:
            status = np.full((n, d), -1, np.int64)
            for r in drawn:
                size_r = int(size[r])
                thr = ((1 << 32) - size_r) % size_r
                raw = mt19937_outputs(oracle_py.lib().oc_rd_seed(self.rd_seed, t, r + 1), off + d)[off:]
                for k, x in enumerate(raw):
                    prod = x * size_r
                    if (prod & 0xFFFFFFFF) < thr:
                        status[r, k] = -2
                        continue
                    ix = prod >> 32
                    pre = 0
                    for g in range(self.world):
                        if ix < pre + allc[g, r, 0]:
                            break
                        pre += allc[g, r, 0]
                    if g == self.rank:
                        j = cols[r][ix - pre]
                        status[r, k] = ((c0 + j) << 1) | int(fresh[r, j])
            status = all_reduce_max(status)
            done = []
            for r in drawn:
                for k in range(d):
                    v = int(status[r, k])
                    if v == -2:
                        continue
                    assert v >= 0
                    c = v >> 1
                    if c == r or not (v & 1) or c in acc[r]:
                        continue
                    acc[r].append(c)
                    if len(acc[r]) >= FANOUT or len(acc[r]) >= numpot[r]:
                        break
                if len(acc[r]) >= FANOUT or len(acc[r]) >= numpot[r]:
                    done.append(r)
            for r in done:
                targets[r] = acc.pop(r)
                drawn.remove(r)
            off, d = off + d, 64
        self.inbox = [[] for _ in range(n)]
        for r in range(n):
            for c in targets[r]:
                self.inbox[c].append(r)
        self.pay = new_pay
        self.t += 1

    def row(self, r):
        hb = np.where(self.ts[r] >= 0, self.hb[r], -1)
        return hb, self.ts[r].copy()
