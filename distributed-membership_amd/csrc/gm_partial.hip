// gm_partial.hip -- PARTIAL-view tick (scenario S-C: V-entry membership views).
//
// The reference is full-membership only; GM_MODE_PARTIAL caps every membership
// list at V entries with the semantics restated (and specified) by the oracle,
// oracle/ref_cpu.c "PARTIAL": entries carry their heartbeat's production tick
// (ts = (hb+1)/2), merge keeps the largest hb per id (updatelistCallBack,
// MP1Node.cpp:259-301), self bump, TFAIL/TREMOVE sweep (MP1Node.cpp:404-447),
// eviction to the V freshest (keyed tie-break), then the reference gossip draw
// over the final list (MP1Node.cpp:449-489) and sendMemberList of its fresh
// entries (MP1Node.cpp:360-395).
//
// One wave per node per tick (gm_p_tick), everything in the wave's LDS slice:
// an open-addressing table keyed by id (64-bit CAS insert + max-merge), a sweep
// over the table, radix selection of the V freshest, a 64-lane bitonic sort of
// the survivors by id, the draw, and the counting-sort append into the targets'
// inboxes. Lists are double-buffered by tick parity: a receiver reads its
// senders' lists of tick t-1 directly and keeps their fresh entries, so no
// separate payload copy is written.
#include "gm_device.h"
#include "gm_partial.h"

#define P_LDS_BYTES (P_H * 8 + P_H + 256 * 4 + 624 * 4 + P_KMAX * 4 + P_VMAX * 8 + P_VMAX * 4)

__device__ __forceinline__ void p_wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ uint32_t p_hash(uint32_t id) { return (id * 0x9E3779B1u) >> (32 - 10); }

// insert (id, hb) or raise the slot's hb to the max; returns the slot
__device__ __forceinline__ int p_insert(unsigned long long *tab, uint64_t key) {
  const uint32_t id = (uint32_t)(key >> 32);
  uint32_t h = p_hash(id);
  for (;;) {
    unsigned long long cur = tab[h];
    if (cur == 0) {
      cur = atomicCAS(&tab[h], 0ull, (unsigned long long)key);
      if (cur == 0) return (int)h;
    }
    if ((uint32_t)(cur >> 32) == id) {
      atomicMax(&tab[h], (unsigned long long)key);
      return (int)h;
    }
    h = (h + 1) & (P_H - 1);
  }
}

__device__ __forceinline__ int p_find(const unsigned long long *tab, uint32_t id) {
  uint32_t h = p_hash(id);
  for (int probe = 0; probe < P_H; probe++) {
    const unsigned long long cur = tab[h];
    if (cur == 0) return -1;
    if ((uint32_t)(cur >> 32) == id) return (int)h;
    h = (h + 1) & (P_H - 1);
  }
  return -1;
}

__device__ __forceinline__ uint64_t p_mix64(uint64_t z) { return gm_mix64(z); }

// eviction tie-break key (oracle op_evict_key): distinct ids give distinct keys
__device__ __forceinline__ uint64_t p_evict_key(uint64_t view_seed, int t, int obs, uint32_t id) {
  return p_mix64(p_mix64(view_seed ^ (uint64_t)(uint32_t)t) ^ (((uint64_t)(uint32_t)obs << 32) | id));
}

__device__ __forceinline__ int p_age(int t, uint32_t hb) { return t - (int)((hb + 1u) >> 1); }

// wave-wide inclusive scan of ints
__device__ __forceinline__ int p_scan(int v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(v, o, 64);
    if (lane >= o) v += y;
  }
  return v;
}

__global__ __launch_bounds__(256) void gm_p_tick(PState s, int t, const uint32_t *mtraw) {
  extern __shared__ __align__(16) unsigned char p_smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + wave;
  if (i >= s.n) return;  // whole wave; no workgroup barrier in this kernel
  unsigned char *base = p_smem + (size_t)wave * P_LDS_BYTES;
  unsigned long long *tab = (unsigned long long *)base;          // [P_H]
  uint8_t *flg = base + P_H * 8;                                 // [P_H] bit0 own, bit1 self
  uint32_t *hist = (uint32_t *)(flg + P_H);                      // [256]
  uint32_t *mts = hist + 256;                                    // [624]
  int32_t *snd = (int32_t *)(mts + 624);                         // [P_KMAX]
  uint64_t *fin = (uint64_t *)(snd + P_KMAX);                    // [P_VMAX]
  uint32_t *finf = (uint32_t *)(fin + P_VMAX);                   // [P_VMAX]
  const int V = s.V;
  const int par = t & 1;
  int32_t *stat = s.rowstat + (size_t)i * 4;
  int k = s.inbox_cnt[par][i];
  if (lane == 0) s.inbox_cnt[par][i] = 0;  // consumed; the append target of tick t+2
  if (s.failed[i]) {  // crashed: frozen (its list carried to this tick's buffer unchanged)
    if (lane < V) s.lists[((size_t)par * s.n + i) * V + lane] = s.lists[((size_t)(par ^ 1) * s.n + i) * V + lane];
    if (lane == 0) {
      stat[0] = stat[1] = stat[2] = stat[3] = 0;
      s.ev_cnt[i] = 0;
    }
    return;
  }
  if (k > P_KMAX) {
    if (lane == 0) atomicOr(s.err, GM_ERR_INBOX);
    k = P_KMAX;
  }
  const uint64_t *prev = s.lists + (size_t)(par ^ 1) * s.n * V;
  uint64_t *cur = s.lists + (size_t)par * s.n * V;
  for (int q = lane; q < P_H; q += 64) {
    tab[q] = 0;
    flg[q] = 0;
  }
  // senders of the delivered lists; with more than P_KP, the P_KP lowest indices
  int sv = lane < k ? s.inbox[par][(size_t)i * P_KMAX + lane] : 0x7FFFFFFF;
  if (k > P_KP) {  // bitonic sort of the (<= 64) sender indices across the wave
#pragma unroll
    for (int k2 = 2; k2 <= 64; k2 <<= 1)
#pragma unroll
      for (int j2 = k2 >> 1; j2 > 0; j2 >>= 1) {
        const int o = __shfl_xor(sv, j2, 64);
        const bool up = (lane & k2) == 0, lower = (lane & j2) == 0;
        sv = (lower == up) ? min(sv, o) : max(sv, o);
      }
  }
  snd[lane] = sv;
  const int kk = min(k, P_KP);
  p_wsync();
  // own entries (the row's list as of tick t-1)
  if (lane < V) {
    const uint64_t e = prev[(size_t)i * V + lane];
    if (e) flg[p_insert(tab, e)] = 1;
  }
  p_wsync();
  // delivered lists: each sender's list of tick t-1, fresh entries only (age < TFAIL at t-1)
  {
    const int per = 64 / V;  // senders per wave step
    const int l = lane % V, jo = lane / V;
    const uint32_t tfresh = (uint32_t)max(0, 2 * t - 11);  // hb >= 2t-11 <=> (t-1) - (hb+1)/2 < TFAIL
    for (int j0 = 0; j0 < kk; j0 += per) {
      const int j = j0 + jo;
      if (jo < per && j < kk) {
        const int sn = snd[j];
        const uint64_t e = prev[(size_t)sn * V + l];
        const uint32_t hb = (uint32_t)e, id = (uint32_t)(e >> 32);
        bool take = e != 0 && hb >= tfresh;
        if (take && s.drop_pct >= 0) {  // per-entry drops keyed by (t_send, src, dst, id-1)
          const uint64_t pair = p_mix64(s.drop_seed ^ ((uint64_t)(uint32_t)(t - 1) << 48) ^
                                        ((uint64_t)(uint32_t)sn << 24) ^ (uint64_t)(uint32_t)i);
          const uint32_t h = (uint32_t)(p_mix64(pair + (uint64_t)(id - 1)) >> 32);
          take = (int)(h % 100u) >= s.drop_pct;
        }
        if (take) (void)p_insert(tab, e);
      }
    }
  }
  p_wsync();
  // self bump (heartbeat++; myPos->setheartbeat(heartbeat++))
  if (lane == 0) {
    int h = p_find(tab, (uint32_t)(i + 1));
    if (h < 0) {
      atomicOr(s.err, GM_ERR_SELF);
      h = p_insert(tab, (uint64_t)(uint32_t)(i + 1) << 32 | 1u);
    }
    const int hb = s.hbctr[i] + 1;
    s.hbctr[i] = hb + 1;
    tab[h] = ((uint64_t)(uint32_t)(i + 1) << 32) | (uint32_t)hb;
    flg[h] |= 2;
  }
  p_wsync();
  // sweep: age >= TREMOVE removes; the rest are eviction candidates
  uint32_t alive = 0, removed_own = 0;
  int removed = 0;
  for (int u = 0; u < P_H / 64; u++) {
    const unsigned long long e = tab[lane + 64 * u];
    if (!e) continue;
    if (p_age(t, (uint32_t)e) >= GM_TREMOVE) {
      removed++;
      if (flg[lane + 64 * u] & 1) removed_own |= 1u << u;
      continue;
    }
    alive |= 1u << u;
  }
  int m = __builtin_popcount(alive);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    m += __shfl_xor(m, o, 64);
    removed += __shfl_xor(removed, o, 64);
  }
  uint32_t keep = alive;
  if (m > V) {
    // evict to V: self, then the freshest (largest hb = smallest age), ties by the
    // smallest eviction key. Age histogram (ages < TREMOVE) finds the cut age.
    if (lane < 32) hist[lane] = 0;
    p_wsync();
    for (int u = 0; u < P_H / 64; u++)
      if (((alive >> u) & 1) && !(flg[lane + 64 * u] & 2)) atomicAdd(&hist[p_age(t, (uint32_t)tab[lane + 64 * u])], 1u);
    p_wsync();
    const int need = V - 1;  // self is always kept
    const int hc = lane < 32 ? (int)hist[lane] : 0;
    const int inc = p_scan(hc, lane);
    const uint64_t over = __ballot(lane < 32 && inc >= need);
    const int acut = __builtin_ctzll(over);  // the cut age
    const int before = __shfl(inc - hc, acut, 64);
    uint32_t needb = (uint32_t)(need - before);
    uint32_t bucket = 0;
    keep = 0;
    uint64_t key[P_H / 64];
#pragma unroll
    for (int u = 0; u < P_H / 64; u++) {
      key[u] = 0;
      if (!((alive >> u) & 1)) continue;
      const unsigned long long e = tab[lane + 64 * u];
      const int a = p_age(t, (uint32_t)e);
      if ((flg[lane + 64 * u] & 2) || a < acut) keep |= 1u << u;
      else if (a == acut) {
        bucket |= 1u << u;
        key[u] = p_evict_key(s.view_seed, t, i, (uint32_t)(e >> 32));
      }
    }
    // radix select of the needb smallest keys in the cut bucket (distinct keys)
    uint64_t prefix = 0;
    for (int d = 7; d >= 0; d--) {
      p_wsync();
      for (int q = lane; q < 256; q += 64) hist[q] = 0;
      p_wsync();
      const uint64_t hmask = d == 7 ? 0ull : ~0ull << (8 * (d + 1));
#pragma unroll
      for (int u = 0; u < P_H / 64; u++)
        if (((bucket >> u) & 1) && ((key[u] ^ prefix) & hmask) == 0) atomicAdd(&hist[(key[u] >> (8 * d)) & 255u], 1u);
      p_wsync();
      uint32_t c4[4];
      int csum = 0;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        c4[q] = hist[4 * lane + q];
        csum += (int)c4[q];
      }
      const int cinc = p_scan(csum, lane);
      const uint64_t hit = __ballot(cinc >= (int)needb);
      const int ln = __builtin_ctzll(hit);
      int cb = __shfl(cinc - csum, ln, 64);  // count below lane ln's bins
      int bsel = 0;
      if (lane == ln) {
        int acc = cb;
        for (int q = 0; q < 4; q++) {
          if (acc + (int)c4[q] >= (int)needb) {
            bsel = 4 * lane + q;
            cb = acc;
            break;
          }
          acc += (int)c4[q];
        }
      }
      bsel = __shfl(bsel, ln, 64);
      cb = __shfl(cb, ln, 64);
      needb -= (uint32_t)cb;
      prefix |= (uint64_t)bsel << (8 * d);
    }
#pragma unroll
    for (int u = 0; u < P_H / 64; u++)
      if (((bucket >> u) & 1) && key[u] <= prefix) keep |= 1u << u;
  }
  // compact the kept entries, then sort them by id (bitonic across the wave)
  int kc = __builtin_popcount(keep);
  const int kinc = p_scan(kc, lane);
  int pos = kinc - kc;
  const int cnt = __shfl(kinc, 63, 64);
  for (int u = 0; u < P_H / 64; u++)
    if ((keep >> u) & 1) {
      fin[pos] = tab[lane + 64 * u];
      finf[pos] = flg[lane + 64 * u];
      pos++;
    }
  p_wsync();
  uint64_t x = lane < cnt ? fin[lane] : ~0ull;
  uint32_t f = lane < cnt ? finf[lane] : 0u;
#pragma unroll
  for (int k2 = 2; k2 <= 64; k2 <<= 1)
#pragma unroll
    for (int j2 = k2 >> 1; j2 > 0; j2 >>= 1) {
      const uint64_t ox = __shfl_xor(x, j2, 64);
      const uint32_t of = __shfl_xor(f, j2, 64);
      const bool up = (lane & k2) == 0, lower = (lane & j2) == 0;
      const bool take_min = lower == up;
      const bool swap = take_min ? (ox < x) : (ox > x);
      if (swap) {
        x = ox;
        f = of;
      }
    }
  // the final list (id order) of tick t: lane j holds entry j
  if (lane < V) cur[(size_t)i * V + lane] = lane < cnt ? x : 0ull;
  const bool valid = lane < cnt;
  const uint32_t hbx = (uint32_t)x;
  const bool stale = valid && p_age(t, hbx) >= GM_TFAIL;
  const bool joined = valid && !(f & 1u);
  int nstale = stale ? 1 : 0;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) nstale += __shfl_xor(nstale, o, 64);
  const int numfailed = removed + nstale;  // numfailed counts removed entries too (MP1Node.cpp:463)
  // events: joins (ascending id) then this row's own removed entries
  uint32_t *evr = s.ev + (size_t)i * 2 * V;
  const uint64_t jb = __ballot(joined);
  const int nj = __builtin_popcountll(jb);
  if (joined) evr[__builtin_popcountll(jb & ((1ull << lane) - 1))] = (P_EV_ADD << 30) | (uint32_t)(x >> 32);
  {
    const int rc = __builtin_popcount(removed_own);
    const int rinc = p_scan(rc, lane);
    int rp = nj + rinc - rc;
    for (int u = 0; u < P_H / 64; u++)
      if ((removed_own >> u) & 1) evr[rp++] = (P_EV_REMOVE << 30) | (uint32_t)(tab[lane + 64 * u] >> 32);
    if (lane == 63) s.ev_cnt[i] = nj + rinc;
  }
  // gossip draw over the final list (MP1Node.cpp:449-489)
  const int numpot = cnt - 1 - numfailed;
  const int target = min(GM_FANOUT, numpot);
  int n = 0, g0 = -1, g1 = -1, g2 = -1, g3 = -1, g4 = -1;
  if (numpot > 0) {
    const uint32_t size = (uint32_t)cnt;
    const uint32_t thr = (0u - size) % size;
    GmLazyMT mt;
    bool done = false;
    for (int batch = 0; !done; batch++) {
      if (batch > (1 << 16)) {
        if (lane == 0) atomicOr(s.err, GM_ERR_DRAWS);
        break;
      }
      uint32_t raw = 0;
      if (batch == 0) {
        if (lane < 16) raw = mtraw[(size_t)i * 16 + lane];
      } else {
        if (lane == 0 && batch == 1) {
          mt.seed(mts, gm_rd_seed(s.rd_seed, t, i + 1));
          for (int q = 0; q < 16; q++) (void)mt.next();
        }
        for (int q = 0; q < 16; q++) {
          uint32_t o = 0;
          if (lane == 0) o = mt.next();
          o = __shfl(o, 0, 64);
          if (lane == q) raw = o;
        }
      }
      const uint64_t prod = (uint64_t)raw * size;
      const bool ok = lane < 16 && (uint32_t)prod >= thr;
      const int ix = (int)(prod >> 32);
      uint64_t mk = __ballot(ok);
      while (mk && !done) {
        const int d = __builtin_ctzll(mk);
        mk &= mk - 1;
        const int ixd = __shfl(ix, d, 64);
        const uint64_t e = __shfl(x, ixd, 64);
        const int c = (int)(e >> 32) - 1;
        if (c == i) continue;                                    // "me"
        if (p_age(t, (uint32_t)e) >= GM_TFAIL) continue;          // age >= TFAIL
        if ((n > 0 && g0 == c) || (n > 1 && g1 == c) || (n > 2 && g2 == c) || (n > 3 && g3 == c)) continue;
        if (n == 0) g0 = c;
        else if (n == 1) g1 = c;
        else if (n == 2) g2 = c;
        else if (n == 3) g3 = c;
        else g4 = c;
        n++;
        if (n >= target) done = true;
      }
    }
  }
  if (lane == 0) {
    int32_t *cnt_out = s.inbox_cnt[par ^ 1];
    const int g[GM_FANOUT] = {g0, g1, g2, g3, g4};
    for (int q = 0; q < n; q++) {
      const int dst = g[q];
      s.targets[(size_t)i * GM_FANOUT + q] = dst;
      const int slot = atomicAdd(&cnt_out[dst], 1);
      if (slot < P_KMAX) s.inbox[par ^ 1][(size_t)dst * P_KMAX + slot] = i;
      else atomicOr(s.err, GM_ERR_INBOX);
    }
    stat[0] = kk;
    stat[1] = cnt;
    stat[2] = numfailed;
    stat[3] = n;
  }
}

// first 16 S2 outputs of every node for tick t (see gm_mt_first16)
__global__ __launch_bounds__(256) void gm_p_mtgen(PState s, int t, uint32_t *mtraw) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= s.n) return;
  uint32_t out[16];
  gm_mt_first16(gm_rd_seed(s.rd_seed, t, r + 1), out);
  uint4 *dst = (uint4 *)(mtraw + (size_t)r * 16);
#pragma unroll
  for (int q = 0; q < 4; q++) dst[q] = make_uint4(out[4 * q], out[4 * q + 1], out[4 * q + 2], out[4 * q + 3]);
}

// warm start at t0 (oracle op_create): self {2t0-1}, V-1 distinct peers chosen by
// mix64(view_seed ^ i<<32 ^ j) % n with hb 2(t0-1-a)-1, sorted by id; written to the
// parity of tick t0.
__global__ __launch_bounds__(64) void gm_p_init(PState s, int t0, uint64_t init_seed) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= s.n) return;
  const int V = s.V;
  uint64_t ent[P_VMAX];
  int cnt = 1;
  ent[0] = ((uint64_t)(uint32_t)(i + 1) << 32) | (uint32_t)(2 * t0 - 1);
  for (uint64_t j = 0; cnt < V; j++) {
    const int q = (int)(gm_mix64(s.view_seed ^ ((uint64_t)(uint32_t)i << 32) ^ j) % (uint64_t)s.n);
    bool dup = q == i;
    for (int a = 1; a < cnt && !dup; a++) dup = (int)(ent[a] >> 32) == q + 1;
    if (dup) continue;
    const int a = (int)((gm_mix64(init_seed ^ ((uint64_t)(uint32_t)i << 32) ^ (uint64_t)(uint32_t)q) >> 40) % 4);
    ent[cnt++] = ((uint64_t)(uint32_t)(q + 1) << 32) | (uint32_t)(2 * (t0 - 1 - a) - 1);
  }
  for (int a = 1; a < cnt; a++)
    for (int b = a; b > 0 && ent[b - 1] > ent[b]; b--) {
      const uint64_t x = ent[b];
      ent[b] = ent[b - 1];
      ent[b - 1] = x;
    }
  uint64_t *dst = s.lists + ((size_t)(t0 & 1) * s.n + i) * V;
  for (int a = 0; a < V; a++) dst[a] = a < cnt ? ent[a] : 0ull;
  s.hbctr[i] = 2 * t0;
}

hipError_t gm_launch_partial_tick(const PState &s, int t, uint32_t *mtraw, hipStream_t st, hipEvent_t k0,
                                  hipEvent_t k1) {
  hipLaunchKernelGGL(gm_p_mtgen, dim3((s.n + 255) / 256), dim3(256), 0, st, s, t, mtraw);
  if (k0) (void)hipEventRecord(k0, st);
  hipLaunchKernelGGL(gm_p_tick, dim3((s.n + 3) / 4), dim3(256), 4 * P_LDS_BYTES, st, s, t, (const uint32_t *)mtraw);
  if (k1) (void)hipEventRecord(k1, st);
  return hipGetLastError();
}

hipError_t gm_launch_partial_init(const PState &s, int t0, uint64_t init_seed, hipStream_t st) {
  hipLaunchKernelGGL(gm_p_init, dim3((s.n + 63) / 64), dim3(64), 0, st, s, t0, init_seed);
  return hipGetLastError();
}

size_t gm_partial_lds_bytes() { return 4 * (size_t)P_LDS_BYTES; }
