// gm_scaled.hip -- SCALED-mode tick: the HBM-bound full-membership hot path.
//
// One launch per globaltime tick; one 256-thread workgroup owns one observer
// row r (MP1Node of node r) and does, in a single streaming pass over the row:
//   1. merge: max-merge the gossip lists delivered to r this tick
//      (updatelistCallBack, MP1Node.cpp:259-301). A list is the sender's
//      post-sweep row of the previous tick reduced to 16-bit heartbeats of its
//      fresh entries (sendMemberList, MP1Node.cpp:360-395: entries with
//      t - ts < TFAIL), stored once per sender in a payload plane and read by
//      each of its <= ~5 receivers ("pull"; no atomics, commutative, order-free);
//   2. self heartbeat bump (nodeLoopOps, MP1Node.cpp:409-415);
//   3. failure sweep: age >= TFAIL -> numfailed, age >= TREMOVE -> removed
//      (MP1Node.cpp:426-444), with join/remove events appended to per-row slots;
//   4. writes the row back and the row's own payload plane for tick t+1;
//   5. builds presence / freshness bitmaps of the row in LDS, then one lane runs
//      the gossip-target draw (mt19937 + Lemire + rank-select, MP1Node.cpp:449-489)
//      and enqueues r into each target's inbox for the next tick -- the
//      counting sort by destination that replaces EmulNet's buffer scan.
// Bytes per live row per tick: 4W read + 4W write (table) + 2W write (payload)
// + 2W per delivered list (payload reads); nothing else touches HBM at scale.
#include "gm_device.h"
#include "gm_scaled.h"

typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u16x2 as_u16x2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }

// merge key of one payload word pair: hb+1, NONE (0xFFFF) -> 0
__device__ __forceinline__ u16x2 key2(uint32_t m) { return as_u16x2(m) + (u16x2)(1); }

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// 16-byte row-stream accesses, optionally non-temporal (A/B variant)
template <bool NT>
__device__ __forceinline__ uint4 ld(const uint4 *p) {
  u32x4 v = NT ? __builtin_nontemporal_load((const u32x4 *)p) : *(const u32x4 *)p;
  return make_uint4(v.x, v.y, v.z, v.w);
}
template <bool NT>
__device__ __forceinline__ void st(uint4 *p, uint4 v) {
  u32x4 w = {v.x, v.y, v.z, v.w};
  if (NT) __builtin_nontemporal_store(w, (u32x4 *)p);
  else *(u32x4 *)p = w;
}

template <bool SHARDED, bool NT>
__device__ __forceinline__ void gm_s_tick_body(SState &s, int t, int drop_pct) {
  extern __shared__ __align__(16) unsigned char s_smem[];
  const int wp = s.wp, nw = wp >> 6;
  uint64_t *s_pres = (uint64_t *)s_smem;               // [nw] present after the sweep
  uint64_t *s_fresh = s_pres + nw;                     // [nw] present and t - ts < TFAIL
  uint32_t *s_pre = (uint32_t *)(s_fresh + nw);        // [nw] exclusive prefix popcounts
  uint32_t *s_mt = s_pre + nw;                         // [624] mt19937 state
  int *s_send = (int *)(s_mt + 624);                   // [S_KMAX] senders of this tick's lists
  int *s_tmp = s_send + S_KMAX;                        // [16] scan scratch
  int *s_misc = s_tmp + 16;                            // [8]

  const int r = blockIdx.x, tid = threadIdx.x;
  const int par = t & 1;
  int32_t *cnt_in = s.inbox_cnt[par];
  if (tid == 0) {
    s_misc[0] = cnt_in[r];
    cnt_in[r] = 0;  // recycled as the append target of tick t+1
    s_misc[1] = 0;  // event slots used
  }
  __syncthreads();
  const int kin = s_misc[0];
  int32_t *stat = s.rowstat + (size_t)r * 4;
  if (s.failed[r]) {  // crashed node: frozen, receives and sends nothing
    if (tid == 0) {
      stat[0] = stat[1] = stat[2] = stat[3] = 0;
      s.ev_cnt[r] = 0;
      if (SHARDED) {
        int32_t *x = s.xcnt + ((size_t)s.shard_rank * s.n + r) * 2;
        x[0] = x[1] = 0;
      }
    }
    return;
  }
  const int k = kin < S_KMAX ? kin : S_KMAX;
  if (tid == 0 && kin > S_KMAX) atomicOr(s.err, GM_ERR_INBOX);
  for (int j = tid; j < k; j += S_THREADS) s_send[j] = s.inbox[par][(size_t)r * S_KMAX + j];
  __syncthreads();

  uint32_t *trow = s.table + (size_t)r * wp;
  uint16_t *mout = s.msg[par] + (size_t)r * s.mstride;
  const uint16_t *mprev = s.msg[par ^ 1];
  const size_t ms = s.mstride;
  const int selfc = (r >= s.c0 && r < s.c0 + s.w) ? r - s.c0 : -1;  // own column, if in this shard
  const uint32_t tt = (uint32_t)t;
  const int t_send = t - 1;
  int npres = 0, nfail = 0;

  for (int base = tid * S_COLS_PER_THREAD; base < wp; base += S_COLS_PER_STEP) {
    const uint4 ta = ld<NT>((const uint4 *)(trow + base));
    const uint4 tb = ld<NT>((const uint4 *)(trow + base + 4));
    u16x2 k0 = (u16x2)(0), k1 = (u16x2)(0), k2 = (u16x2)(0), k3 = (u16x2)(0);
    if (drop_pct < 0) {
      for (int j0 = 0; j0 < k; j0 += 8) {
        uint4 m[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
          if (j0 + u < k) m[u] = *(const uint4 *)(mprev + (size_t)s_send[j0 + u] * ms + base);
          else m[u] = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
          k0 = __builtin_elementwise_max(k0, key2(m[u].x));
          k1 = __builtin_elementwise_max(k1, key2(m[u].y));
          k2 = __builtin_elementwise_max(k2, key2(m[u].z));
          k3 = __builtin_elementwise_max(k3, key2(m[u].w));
        }
      }
    } else {
      // per-entry drops keyed by (t_send, src, dst, column) -- SCALED regime
      uint32_t kk[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int j = 0; j < k; j++) {
        const int snd = s_send[j];
        const uint4 m = *(const uint4 *)(mprev + (size_t)snd * ms + base);
        const uint32_t mw[4] = {m.x, m.y, m.z, m.w};
        const uint64_t pair = gm_mix64(s.drop_seed ^ ((uint64_t)(uint32_t)t_send << 48) ^
                                       ((uint64_t)(uint32_t)snd << 24) ^ (uint64_t)(uint32_t)r);
#pragma unroll
        for (int q = 0; q < 8; q++) {
          uint32_t hv = (mw[q >> 1] >> (16 * (q & 1))) & 0xFFFFu;
          uint32_t key = (hv + 1u) & 0xFFFFu;
          if (key == 0) continue;
          uint32_t h = (uint32_t)(gm_mix64(pair + (uint64_t)(s.c0 + base + q)) >> 32);
          if ((int)(h % 100u) < drop_pct) continue;
          kk[q] = kk[q] > key ? kk[q] : key;
        }
      }
      k0 = as_u16x2(kk[0] | (kk[1] << 16));
      k1 = as_u16x2(kk[2] | (kk[3] << 16));
      k2 = as_u16x2(kk[4] | (kk[5] << 16));
      k3 = as_u16x2(kk[6] | (kk[7] << 16));
    }
    uint32_t e[8] = {ta.x, ta.y, ta.z, ta.w, tb.x, tb.y, tb.z, tb.w};
    const uint32_t keys[4] = {as_u32(k0), as_u32(k1), as_u32(k2), as_u32(k3)};
    uint32_t out[4] = {0, 0, 0, 0};
    uint32_t pbits = 0, fbits = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int c = base + q;
      uint32_t en = e[q];
      const uint32_t key = (keys[q >> 1] >> (16 * (q & 1))) & 0xFFFFu;
      uint32_t ev = 0;
      if (key) {  // updatelistCallBack: insert, or raise hb and stamp ts = now
        const uint32_t hb = key - 1u;
        if (en == GM_ABSENT) { en = gm_pack(hb, tt); ev = S_EV_ADD; }
        else if (gm_hb(en) < hb) en = gm_pack(hb, tt);
      }
      if (c == selfc) {  // updateMyPos + heartbeat++ + myPos->setheartbeat(heartbeat++)
        if (en == GM_ABSENT) atomicOr(s.err, GM_ERR_SELF);
        const int hb = s.hbctr[r] + 1;
        s.hbctr[r] = hb + 1;
        en = gm_pack((uint32_t)hb, tt);
      }
      uint32_t o = GM_NONE16;
      if (en != GM_ABSENT) {
        const int age = t - (int)gm_ts(en);
        if (age >= GM_TFAIL) {
          nfail++;
          if (age >= GM_TREMOVE) { en = GM_ABSENT; ev = S_EV_REMOVE; }
        } else {
          o = gm_hb(en);
          fbits |= 1u << q;
        }
        if (en != GM_ABSENT) pbits |= 1u << q;
      }
      e[q] = en;
      out[q >> 1] |= o << (16 * (q & 1));
      if (ev) {
        const int slot = atomicAdd(&s_misc[1], 1);
        const uint32_t rec = (ev << 30) | (uint32_t)(s.c0 + c + 1);
        if (slot < s.evcap) {
          s.ev_rows[(size_t)r * s.evcap + slot] = rec;
        } else {
          const uint32_t sp = atomicAdd(s.ev_spill_cnt, 1u);
          if (sp < s.ev_spill_cap) s.ev_spill[sp] = ((uint64_t)(uint32_t)r << 32) | rec;
          else atomicOr(s.err, GM_ERR_EVENTS);
        }
      }
    }
    npres += __builtin_popcount(pbits);
    st<NT>((uint4 *)(trow + base), make_uint4(e[0], e[1], e[2], e[3]));
    st<NT>((uint4 *)(trow + base + 4), make_uint4(e[4], e[5], e[6], e[7]));
    st<NT>((uint4 *)(mout + base), make_uint4(out[0], out[1], out[2], out[3]));
    ((uint8_t *)s_pres)[base >> 3] = (uint8_t)pbits;
    ((uint8_t *)s_fresh)[base >> 3] = (uint8_t)fbits;
  }

  // row totals and rank-select prefix over the presence bitmap
  const int size = gm_block_sum(npres, s_tmp);
  const int numfailed = gm_block_sum(nfail, s_tmp);
  {
    const int per = (nw + S_THREADS - 1) / S_THREADS;
    const int w0 = tid * per, w1 = min(nw, w0 + per);
    int part = 0;
    for (int w = w0; w < w1; w++) part += __builtin_popcountll(s_pres[w]);
    int tot;
    int acc = gm_block_scan(part, s_tmp, &tot);
    for (int w = w0; w < w1; w++) {
      s_pre[w] = (uint32_t)acc;
      acc += __builtin_popcountll(s_pres[w]);
    }
  }
  __syncthreads();

  if (SHARDED) {
    // publish this shard's slice of the row: counts for the all-gather, bitmaps
    // and prefix for draw resolution (gm_s_draw); the draw itself needs the
    // whole row and runs after the exchange
    uint64_t *gp = s.gpres + (size_t)r * nw, *gf = s.gfresh + (size_t)r * nw;
    uint32_t *gq = s.gpre + (size_t)r * nw;
    for (int w = tid; w < nw; w += S_THREADS) {
      gp[w] = s_pres[w];
      gf[w] = s_fresh[w];
      gq[w] = s_pre[w];
    }
    if (tid == 0) {
      int32_t *x = s.xcnt + ((size_t)s.shard_rank * s.n + r) * 2;
      x[0] = size;
      x[1] = numfailed;
      stat[0] = k;
      s.ev_cnt[r] = s_misc[1];
    }
    return;
  }

  if (tid == 0) {
    // gossip-target draw on the post-sweep list (MP1Node.cpp:449-489); newNodes is
    // empty in the converged SCALED regime (no JOINREQ traffic)
    const int numpot = size - 1 - numfailed;
    int n = 0;
    int g[GM_FANOUT];
    if (numpot > 0) {
      GmLazyMT mt;
      mt.seed(s_mt, gm_rd_seed(s.rd_seed, t, r + 1));
      long guard = 0;
      while (n < GM_FANOUT && n < numpot) {
        if (++guard > (1l << 22)) { atomicOr(s.err, GM_ERR_DRAWS); break; }
        const int ix = mt.uniform((uint32_t)size);
        const int c = gm_rank_select(s_pres, s_pre, nw, (uint32_t)ix);
        if (c == selfc) continue;                                 // "me"
        if (!((s_fresh[c >> 6] >> (c & 63)) & 1ull)) continue;    // age >= TFAIL
        bool dup = false;
        for (int q = 0; q < n; q++) dup |= g[q] == c;
        if (!dup) g[n++] = c;
      }
    }
    int32_t *cnt_out = s.inbox_cnt[par ^ 1];
    for (int q = 0; q < n; q++) {
      const int dst = s.c0 + g[q];
      s.targets[(size_t)r * GM_FANOUT + q] = dst;
      const int slot = atomicAdd(&cnt_out[dst], 1);
      if (slot < S_KMAX) s.inbox[par ^ 1][(size_t)dst * S_KMAX + slot] = r;
      else atomicOr(s.err, GM_ERR_INBOX);
    }
    stat[0] = k;
    stat[1] = size;
    stat[2] = numfailed;
    stat[3] = n;
    s.ev_cnt[r] = s_misc[1];
  }
}

__global__ __launch_bounds__(S_THREADS) void gm_s_tick(SState s, int t, int drop_pct) {
  gm_s_tick_body<false, false>(s, t, drop_pct);
}
// same, with non-temporal table / payload-write streams (default; GM_NT=0 selects gm_s_tick)
__global__ __launch_bounds__(S_THREADS) void gm_s_tick_nt(SState s, int t, int drop_pct) {
  gm_s_tick_body<false, true>(s, t, drop_pct);
}

// Column-sharded phase A: merge + sweep of this shard's columns for every row.
__global__ __launch_bounds__(S_THREADS) void gm_s_tick_shard(SState s, int t, int drop_pct) {
  gm_s_tick_body<true, false>(s, t, drop_pct);
}

// Column-sharded phase B: each rank replays every live row's S2 stream (the
// same mt19937 + Lemire sequence on every rank), and resolves the draws whose
// rank lands in its own columns: status = (global column << 1) | fresh, else -1.
// round 0 seeds the generators and the acceptance state from the all-gathered
// per-shard (present, numfailed) counts.
__global__ __launch_bounds__(256) void gm_s_draw(SState s, int t, int round, int D) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= s.n) return;
  const int G = s.shard_count, nw = s.wp >> 6;
  int32_t *acc = s.acc + (size_t)r * 8;
  int32_t *mtk = s.mtk + (size_t)r * 3;
  if (round == 0) {
    int size = 0, nf = 0;
    for (int g = 0; g < G; g++) {
      size += s.xcnt[((size_t)g * s.n + r) * 2];
      nf += s.xcnt[((size_t)g * s.n + r) * 2 + 1];
    }
    const int numpot = size - 1 - nf;
    const bool live = !s.failed[r];
    acc[0] = 0;
    acc[6] = numpot;
    acc[7] = size;
    s.pending[r] = live && numpot > 0;
    int32_t *stat = s.rowstat + (size_t)r * 4;
    if (!live) stat[0] = 0;
    stat[1] = live ? size : 0;
    stat[2] = live ? nf : 0;
    stat[3] = 0;
    if (!s.pending[r]) return;
    GmLazyMT mt;
    mt.seed(s.mt + r, gm_rd_seed(s.rd_seed, t, r + 1), s.n);
    mtk[0] = mt.k;
    mtk[1] = mt.ninit;
    mtk[2] = 1;
  }
  if (!s.pending[r]) return;
  GmLazyMT mt;
  mt.x = s.mt + r;
  mt.stride = s.n;
  mt.k = mtk[0];
  mt.ninit = mtk[1];
  mt.first = mtk[2] != 0;
  const uint32_t size = (uint32_t)acc[7];
  int32_t *st = s.status + (size_t)r * D;
  for (int d = 0; d < D; d++) {
    const uint32_t ix = (uint32_t)mt.uniform(size);
    // which shard holds the ix-th present entry of row r (shards in column order)
    uint32_t pre = 0;
    int owner = G - 1;
    for (int g = 0; g < G; g++) {
      const uint32_t c = (uint32_t)s.xcnt[((size_t)g * s.n + r) * 2];
      if (ix < pre + c) { owner = g; break; }
      pre += c;
    }
    int32_t v = -1;
    if (owner == s.shard_rank) {
      const int cl = gm_rank_select(s.gpres + (size_t)r * nw, s.gpre + (size_t)r * nw, nw, ix - pre);
      const int fresh = (int)((s.gfresh[(size_t)r * nw + (cl >> 6)] >> (cl & 63)) & 1ull);
      v = ((s.c0 + cl) << 1) | fresh;
    }
    st[d] = v;
  }
  mtk[0] = mt.k;
  mtk[1] = mt.ninit;
  mtk[2] = mt.first ? 1 : 0;
}

// Column-sharded phase C: with every draw resolved (MAX-allreduced status), run
// the acceptance loop of MP1Node.cpp:466-489 (skip me, skip stale, skip
// duplicates) identically on every rank; finished rows enqueue themselves into
// their targets' inboxes for the next tick.
__global__ __launch_bounds__(256) void gm_s_accept(SState s, int t, int D) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= s.n || !s.pending[r]) return;
  int32_t *acc = s.acc + (size_t)r * 8;
  int n = acc[0];
  const int numpot = acc[6];
  int g[GM_FANOUT];
  for (int q = 0; q < n; q++) g[q] = acc[1 + q];
  const int32_t *st = s.status + (size_t)r * D;
  bool done = false;
  for (int d = 0; d < D && !done; d++) {
    const int32_t v = st[d];
    if (v < 0) { atomicOr(s.err, GM_ERR_DRAWS); done = true; break; }
    const int c = v >> 1;
    if (c == r) continue;        // "me"
    if (!(v & 1)) continue;      // age >= TFAIL (skipfailed: numpot > 0 here)
    bool dup = false;
    for (int q = 0; q < n; q++) dup |= g[q] == c;
    if (!dup) g[n++] = c;
    done = n >= GM_FANOUT || n >= numpot;
  }
  for (int q = 0; q < n; q++) acc[1 + q] = g[q];
  acc[0] = n;
  if (!done) {
    atomicAdd(s.npending, 1);
    return;
  }
  s.pending[r] = 0;
  const int par = t & 1;
  int32_t *cnt_out = s.inbox_cnt[par ^ 1];
  for (int q = 0; q < n; q++) {
    const int dst = g[q];
    s.targets[(size_t)r * GM_FANOUT + q] = dst;
    const int slot = atomicAdd(&cnt_out[dst], 1);
    if (slot < S_KMAX) s.inbox[par ^ 1][(size_t)dst * S_KMAX + slot] = r;
    else atomicOr(s.err, GM_ERR_INBOX);
  }
  s.rowstat[(size_t)r * 4 + 3] = n;
}

// SCALED initial state (gm_config.init_mode): every observer holds every subject.
// Cold: {hb 0, ts 0}. Warm at t0: own entry {2*t0-1, t0}; others {2*(t0-1-a)-1,
// t0-a}, a = splitmix64(seed ^ r<<32 ^ c) % 4 -- values as if the cluster had been
// gossiping, so the first ticks carry no mass-staleness transient. Padding absent.
__global__ void gm_s_init(SState s, int warm, int t0, uint64_t seed) {
  const int r = blockIdx.x;
  uint32_t *row = s.table + (size_t)r * s.wp;
  for (int j = threadIdx.x; j < s.wp; j += blockDim.x) {
    uint32_t e = GM_ABSENT;
    if (j < s.w) {
      const int c = s.c0 + j;
      if (!warm) e = gm_pack(0, 0);
      else if (c == r) e = gm_pack((uint32_t)(2 * t0 - 1), (uint32_t)t0);
      else {
        const int a = (int)((gm_mix64(seed ^ ((uint64_t)(uint32_t)r << 32) ^ (uint64_t)(uint32_t)c) >> 40) % 4);
        e = gm_pack((uint32_t)(2 * (t0 - 1 - a) - 1), (uint32_t)(t0 - a));
      }
    }
    row[j] = e;
  }
  if (threadIdx.x == 0) s.hbctr[r] = warm ? 2 * t0 : 0;
}
