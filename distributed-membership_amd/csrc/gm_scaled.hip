// gm_scaled.hip -- SCALED-mode tick: the HBM-bound full-membership hot path.
//
// One globaltime tick (Application::mp1Run for every node, Application.cpp:121-164)
// is three launches on the context stream:
//
//   gm_s_mtgen  thread per row: the first S_MT_RAW outputs of the row's S2 stream
//               (the mt19937 that nodeLoopOps seeds per call, MP1Node.cpp:450-452),
//               computed from 397+16 init words kept in registers.
//   gm_s_band   the merge / heartbeat / sweep pass over the N x W table, in COLUMN
//               BANDS: one wave per (band, 64 rows) streams the band's slice of its rows,
//               max-merges the slices of the gossip payloads delivered to each row
//               (updatelistCallBack, MP1Node.cpp:259-301), bumps the row's own entry
//               (MP1Node.cpp:409-415), runs the TFAIL/TREMOVE sweep (MP1Node.cpp:
//               426-444), writes the row slice back and the row's payload slice for
//               tick t+1 (the fresh entries' heartbeats, sendMemberList MP1Node.cpp:
//               360-395), and records per-(row, band) counts and events. Workgroups
//               are numbered band-major, so the chip sweeps one band of every row at a
//               time: a sender's payload slice is read by its ~5 receivers while that
//               band's payload slices (N x band x 2 B) are resident in the 256 MiB
//               Infinity Cache -- HBM sees each payload byte once instead of once per
//               delivery (band width sized so one band's traffic fits the cache).
//   gm_s_pick   wave per row: row totals from the band counts, the gossip-target draw
//               on the post-sweep list (MP1Node.cpp:449-489: Lemire over the S2
//               outputs, "memberlist[ix]" = rank-select over band prefix counts and one
//               table slice, skip me / stale / duplicates), and delivery: the row
//               appends itself to its targets' inboxes for tick t+1 (counting sort by
//               destination in place of EmulNet's buffer scan, EmulNet.cpp:144-177).
//
// Column-sharded ticks (multi-GPU) run gm_s_mtgen + gm_s_band on the shard's columns
// (which also accumulates the shard's per-row counts), exchange the counts, then
// gm_s_draw / gm_s_accept rounds.
#include "gm_device.h"
#include "gm_scaled.h"

#include <algorithm>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef uint8_t u8x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// ------------------------------------------------------------------ gm_s_mtgen
// Also zeroes the tick's counters (no fill launch of their own each tick): the event spill ring's
// count and the striped event totals (the last tick's records stay readable until here), and the
// fused draw's fallback-row count (gm_s_pick0 runs after the band kernels). Grid: max(n, 1 + S_EV_STRIPES).
// zero_draw (the pipelined column-shard tick): also the draw rounds' counters -- the pending lists'
// append counts and the rows left to the host-driven rounds (three fill launches a tick before)
__global__ __launch_bounds__(256) void gm_s_mtgen(SState s, int t, int zero_draw) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < 1 + S_EV_STRIPES) s.ev_spill_cnt[r] = 0;
  if (r == 0 && s.pk_cnt) *s.pk_cnt = 0;
  if (zero_draw && r == 0) {
    *s.plist_cnt[1] = 0;
    *s.plist_cnt[2] = 0;
    *s.npending = 0;
  }
  if (r >= s.n) return;
  uint32_t out[S_MT_RAW];
  gm_mt_first16(gm_rd_seed(s.rd_seed, t, r + 1), out);
  uint4 *dst = (uint4 *)(s.mtraw + (size_t)r * S_MT_RAW);
#pragma unroll
  for (int k = 0; k < S_MT_RAW / 4; k++) dst[k] = make_uint4(out[4 * k], out[4 * k + 1], out[4 * k + 2], out[4 * k + 3]);
}

// ------------------------------------------------------------------- gm_s_band
// One wave per work unit: unit u is (band u / U, rows [(u % U) * RPW, +RPW)),
// U = ceil(n / RPW) units per band, LPR = B/8 lanes per row, 8 columns per lane.
// Units are numbered band-major, so the waves in flight cover a few consecutive
// thousand rows of one band: the band's payload slab (n * B * 2 B per parity) is
// read ~5 times per sender slice while it sits in the Infinity Cache, and HBM sees
// each payload byte about once. Each wave issues its row's metadata (crash flag,
// inbox count, first S_SB sender ids) together with its table slice, then the
// payload slices, merges, sweeps, stores and exits (short-lived waves keep more
// bytes in flight than a persistent loop; measured with scripts/ubench).
template <int B>
struct RowMeta {
  int k;           // lists delivered to the row (-1: no such row, or a crashed node)
  int snd[S_SB];   // first S_SB senders
  uint32_t ebase;  // the (band, row) record's escape-list word of the last tick (S_EW_*, 0: no escaped cells)
  uint32_t bz;     // the record's count word of the last tick (S_BC_*: the slice's present cells as stored)
  uint64_t evc;    // EVC: the (row, band)'s cumulative events (evcum), read with the metadata
  uint32_t ebase2, bz2;  // band2 >= 0: the same words of the (band2, row) record
  uint64_t evc2;         // and its evcum cell (EVC)
};

// Every load of the row's metadata issues at once, none behind a branch on another (one
// memory round trip before the payload gathers can issue, not a chain of three).
// a load through a pointer known to be global memory (a pointer out of an asm statement is no
// longer known to be one, and a generic pointer's loads are never scalar)
template <typename T>
__device__ __forceinline__ T gld(const T *p) {
#if __HIP_DEVICE_COMPILE__
  return *(const __attribute__((address_space(1))) T *)p;
#else
  return *p;  // (host pass: never executed)
#endif
}
// band2 >= 0 (one row per wave): also the record and evcum cell of the row in band2 -- loaded here,
// before the empty asm statements below, which the compiler takes for memory writes (a load after
// them is not known unclobbered and becomes a vector load)
template <int B, bool UNI, bool EVC = false>
__device__ __forceinline__ RowMeta<B> row_meta(const SState &s, int r, int par, int t, size_t slab, int band,
                                               int band2 = -1) {
  RowMeta<B> m;
  const int rc = min(r, s.n - 1);  // r >= n (a partial unit): loads stay in bounds, k = -1
  const int32_t *ibase = par ? s.inbox[1] : s.inbox[0], *cbase = par ? s.inbox_cnt[1] : s.inbox_cnt[0];
  const int32_t *fbase = s.failed;
  const uint4 *rbase = s.brec;
  const uint64_t *ecbase = s.evcum;
  int ramp = s.ramp;
  // every kernel-argument word the row's loads need, in one batch: without this the compiler
  // interleaves these (scalar-cache) loads with the row's memory loads, and a wait for one of them
  // waits for all -- the evcum cell then issued only after the inbox had arrived (a second round trip
  // before the gathers). A plain asm statement (not volatile: no memory effect assumed).
  if (UNI) asm("" : "+s"(ibase), "+s"(cbase), "+s"(fbase), "+s"(rbase), "+s"(ecbase), "+s"(ramp));
  const int32_t *ib = ibase + (size_t)rc * S_KMAX;
  const i32x4 av = gld((const i32x4 *)ib), bv = gld((const i32x4 *)(ib + 4));
  int4 a = make_int4(av.x, av.y, av.z, av.w);
  int4 b = make_int4(bv.x, bv.y, bv.z, bv.w);
  int k = gld(cbase + rc);
  int failed = gld(fbase + rc);
  const u32x4 rv = gld((const u32x4 *)(rbase + slab + rc));
  const uint4 rec = make_uint4(rv.x, rv.y, rv.z, rv.w);
  m.ebase = rec.w;
  m.bz = rec.z;
  // the fast path (one row per wave): the unit is the only writer of its evcum cell this tick, so it is read
  // here (in flight with the rest) and written back plainly -- no device-scope atomic per unit with
  // events (at the TREMOVE peak ~4 M of them held the fast path's waves: +2 ms per tick)
  m.evc = EVC ? gld(ecbase + (size_t)rc * s.nb + band) : 0ull;
  if (band2 >= 0) {
    const u32x4 rec2 = gld((const u32x4 *)(rbase + (size_t)band2 * s.n + rc));
    m.ebase2 = rec2.w;
    m.bz2 = rec2.z;
    m.evc2 = EVC ? gld(ecbase + (size_t)rc * s.nb + band2) : 0ull;
  }
  // empty asm statements that read the values here: without them the compiler sinks the
  // inbox-count load into a branch on `failed` and the sender ids behind that, two more
  // round trips before the gathers (one row per wave: scalar registers)
  if (UNI) {
    asm volatile("" : "+s"(k), "+s"(failed), "+s"(a.x), "+s"(a.y), "+s"(a.z), "+s"(a.w));
    asm volatile("" : "+s"(b.x), "+s"(b.y), "+s"(b.z), "+s"(b.w));
  } else {
    asm volatile("" : "+v"(k), "+v"(failed));
  }
  m.snd[0] = a.x; m.snd[1] = a.y; m.snd[2] = a.z; m.snd[3] = a.w;
  m.snd[4] = b.x; m.snd[5] = b.y; m.snd[6] = b.z; m.snd[7] = b.w;
  // not in the group (join ramp) or crashed: untouched
  m.k = (r >= s.n || failed || !s_ingroup(ramp, s.intro_until, r, t)) ? -1 : k;
  if (r >= s.n) m.ebase = m.ebase2 = 0;
  return m;
}

// Buffer resource over [p, p + bytes) built from wave-uniform values (SGPRs): loads
// beyond `bytes` return 0 without touching memory, stores beyond it are dropped.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t gm_rsrc(const void *p, uint32_t bytes) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi << 32) | lo), (short)0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
#define GM_AUX_NT 2  // non-temporal (streamed once)
#define GM_OOB 0x80000000u

// Packed 16-bit lanes of a 32-bit register: two cells per VGPR, v_pk_* arithmetic.
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 pk(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ uint32_t unpk(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }
// payload bytes 0,1 / 2,3 of a dword, zero-extended into the two halves
// a += b per u16 half, opaque to the compiler: plain vector adds of the sweep's
// per-pair counts get re-associated into a tree that keeps every pair's term live
// (9 VGPR spills at occupancy 8); an in-order chain consumes each term at once
__device__ __forceinline__ u16x2 padd(u16x2 a, u16x2 b) {
  uint32_t r;
  asm("v_pk_add_u16 %0, %1, %2" : "=v"(r) : "v"(unpk(a)), "v"(unpk(b)));
  return pk(r);
}
// min(x, 1) per u16 half as ONE v_pk_min_u16: written as plain vector min the compiler
// lowers it to a compare + select per half (5 instructions instead of 1)
__device__ __forceinline__ u16x2 pmin1(u16x2 a) {
  uint32_t r;
  asm("v_pk_min_u16 %0, %1, 1 op_sel_hi:[1,0]" : "=v"(r) : "v"(unpk(a)));
  return pk(r);
}

// stored cell bytes 0,1 (hi = 0) or 2,3 (hi = 1) of a dword, zero-extended into the two u16 halves
__device__ __forceinline__ uint32_t byte_pair(uint32_t w, int hi) {
  return __builtin_amdgcn_perm(0u, w, hi ? 0x0c030c02u : 0x0c010c00u);
}
// s_widen of two stored bytes (nz = min(x, 1)); an escape byte gives garbage, replaced by its wide cell
// (h4 << 4 | a -> 7168 + (h4 << 6) + a = x + 3 (x & 0xF0) + 7168: two multiply-adds)
__device__ __forceinline__ u16x2 widen2(u16x2 x, u16x2 nz) {
  return nz * (u16x2)(7168) + ((x & (u16x2)(0xF0)) * (u16x2)(3) + x);
}

// wave-wide inclusive scan on DPP: row_shr 1/2/4/8 within each 16-lane row, row_bcast15 /
// row_bcast31 carry the row totals upward (lanes a DPP source does not reach add 0)
__device__ __forceinline__ int dpp_scan(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);  // row_shr:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
  return v;
}

// Stored bytes of two swept cells (pres = min(v2, 1)): tt = v2 - (S_CELL(230, 0) - 1) (wraps below
// h = 230) = (h - 230) << 5 | (age + 1); representable iff nothing above the h field (h <= 254, no
// wrap), h even (bit 5) and age <= 14 (bit 4 of age + 1) -> h4 << 4 | age (h4 = (h - 224) / 2 =
// the tt field + 3), else S_B_ESC (bad = 1); absent 0. gm_scaled.h: a stored byte is always one
// re-base away from another byte, which the fast path of gm_s_band relies on.
__device__ __forceinline__ u16x2 narrow2(u16x2 v2, u16x2 pres, u16x2 &bad) {
  const u16x2 tt = v2 - (u16x2)(S_CELL(S_H4_MIN_H, 0) - 1);
  bad = pmin1(tt & (u16x2)(0xFC30)) & pres;
  const uint32_t tu = unpk(tt);
  const u16x2 enc = pk((tu & 0x000F000Fu) | ((tu >> 2) & 0x00F000F0u)) + (u16x2)(0x2F);
  return enc * (pres - bad) + bad;
}

// The lane's escaped cells as a mask: bit 8j + i set where byte j of stored dword i (cell 4i + j)
// is the escape code S_B_ESC (the narrowing writes no other code below 16). x = w ^ 0x01010101 has
// a zero byte exactly there (carry-free SWAR zero-byte test); the four dwords' byte flags are
// merged by shifts alone (no quarter-rate 32-bit multiply to gather them). esc_cell maps a bit
// back to its cell; the list's entries carry their columns, so their order is not significant.
__device__ __forceinline__ uint32_t esc_mask16(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
  static_assert(S_B_ESC == 1u, "esc_mask16 tests for the byte 0x01");
  const uint32_t w[4] = {w0, w1, w2, w3};
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint32_t x = w[i] ^ 0x01010101u;
    const uint32_t e = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;  // bit 7 of each zero byte
    m |= e >> (7 - i);
  }
  return m;
}
__device__ __forceinline__ int esc_cell(int p) { return ((p & 7) << 2) | (p >> 3); }

// exclusive prefix of v over the LPR aligned lanes of this lane's row, and the row total;
// every lane of the row is active (the callers branch on row-uniform conditions only)
template <int LPR>
__device__ __forceinline__ int row_scan(int v, int li, int lane, int &total) {
  int x = v;
  if (LPR == 64) {
    x = dpp_scan(v);
    total = __builtin_amdgcn_readlane(x, 63);
  } else {
#pragma unroll
    for (int o = 1; o < LPR; o <<= 1) {
      const int y = __shfl_up(x, o, 64);
      if (li >= o) x += y;
    }
    total = __shfl(x, lane - li + LPR - 1, 64);
  }
  return x - v;
}

// any lane of this lane's row
template <int LPR>
__device__ __forceinline__ bool row_any(bool p, int sub) {
  const uint64_t b = __builtin_amdgcn_ballot_w64(p);
  return LPR == 64 ? b != 0 : ((b >> (sub * LPR)) & ((1ull << LPR) - 1)) != 0;
}

// stripe of the (band, row) list at slab + r (gm_scaled.h: striped pool allocation)
__device__ __forceinline__ int esc_stripe(const SState &s, size_t slab, int r) {
  return (int)((slab + (size_t)r) & (size_t)(s.esc_stripes - 1));
}
// The escape-list word of a (band, row) list of `total` escaped cells written at tick parity
// par: up to S_ESC_IN entries need no allocation; beyond, one reservation (the row's first lane)
// in its stripe's pool region, broadcast to the row -- 0 with GM_ERR_ESC if the region overflowed
// (the run is void). total is row-uniform.
template <int LPR>
__device__ __forceinline__ uint32_t row_alloc(const SState &s, int par, size_t slab, int r, int total, int li,
                                              int lane) {
  if (total <= S_ESC_IN) return (uint32_t)total;
  uint32_t w = 0;
  if (li == 0) {
    const int stripe = esc_stripe(s, slab, r);
    const unsigned long long need = (unsigned long long)(total - S_ESC_IN);
    const unsigned long long b = atomicAdd(s.tesc_cnt + par * s.esc_stripes + stripe, need);
    if (b + need <= (unsigned long long)s.tesc_region) w = (uint32_t)total | ((uint32_t)b << 11);
    else atomicOr(s.err, GM_ERR_ESC);
  }
  return LPR == 64 ? __builtin_amdgcn_readfirstlane(w) : (uint32_t)__shfl((int)w, lane - li, 64);
}
// a list's storage: entry i < S_ESC_IN in the inline slot, the rest in its stripe's pool region
struct EscList {
  uint32_t *inl, *pool;
  __device__ __forceinline__ uint32_t *at(int i) const { return i < S_ESC_IN ? inl + i : pool + (i - S_ESC_IN); }
};
__device__ __forceinline__ EscList esc_list(const SState &s, int par, size_t slab, int r, uint32_t word) {
  EscList l;
  l.inl = s.tesc_in[par] + (slab + (size_t)r) * S_ESC_IN;
  l.pool = s.tesc[par] + (size_t)esc_stripe(s, slab, r) * s.tesc_region + S_EW_OFF(word);
  return l;
}

// LDS of the band kernel: 32 B per lane (its 16 working cells), i.e. one wave's rows' cells in
// column order -- the meeting point of escape entries and the lanes holding their columns
#define S_LDS_WAVE_WORDS (64 * 8)
__device__ __forceinline__ void lds_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Reader: the row's list (tot entries, row-uniform) into the lanes' cells: every lane of the
// row parks its 16 cells in LDS, the row's lanes scatter the entries by column (lane li < 16
// has entry li prefetched in `ent`; entries beyond S_ESC_IN load here), then every lane takes
// its cells back. lds = this wave's area.
template <int LPR>
__device__ __forceinline__ void esc_apply(uint32_t *lds, int lane, int li, const EscList &l, int tot, uint32_t ent,
                                          u16x2 tw[8]) {
  u32x4 *mine = (u32x4 *)(lds + lane * 8);
  mine[0] = (u32x4){unpk(tw[0]), unpk(tw[1]), unpk(tw[2]), unpk(tw[3])};
  mine[1] = (u32x4){unpk(tw[4]), unpk(tw[5]), unpk(tw[6]), unpk(tw[7])};
  lds_wave_sync();
  uint16_t *row = (uint16_t *)(lds + (lane - li) * 8);  // the row's B cells in column order
  constexpr int P = LPR < S_ESC_IN ? LPR : S_ESC_IN;  // entries prefetched (one per lane)
  if (li < min(tot, P)) row[ent & 0xFFFFu] = (uint16_t)(ent >> 16);
  for (int i = P + li; i < tot; i += LPR) {  // rare: lists longer than the prefetch
    const uint32_t e = *l.at(i);
    row[e & 0xFFFFu] = (uint16_t)(e >> 16);
  }
  lds_wave_sync();
  const u32x4 a = mine[0], b = mine[1];
  tw[0] = pk(a.x); tw[1] = pk(a.y); tw[2] = pk(a.z); tw[3] = pk(a.w);
  tw[4] = pk(b.x); tw[5] = pk(b.y); tw[6] = pk(b.z); tw[7] = pk(b.w);
}

// Writer: the lane's 16 swept cells wait in its LDS slot (esc_park, right after the sweep, so
// they need no registers through the stores); its escaped cells (mask em, esc_mask16's bit order)
// become entries eoff, eoff + 1, ... of the list, a set bit's cell one dynamic LDS read (no
// register indexing).
// colb = the lane's first column in the band.
__device__ __forceinline__ void esc_park(uint32_t *lds, int lane, const uint32_t cw[8]) {
  u32x4 *mine = (u32x4 *)(lds + lane * 8);
  mine[0] = (u32x4){cw[0], cw[1], cw[2], cw[3]};
  mine[1] = (u32x4){cw[4], cw[5], cw[6], cw[7]};
}
// inl_only (row-uniform): the list fits its inline slot, so no entry needs the pool address.
// An escaped cell that is present with h < hmin (3: h <= 2, its next re-base would wrap) sets
// GM_ERR_LAG; only escaped cells can be that low (a stored byte holds h >= 226)
__device__ __forceinline__ void esc_emit(uint32_t *lds, int lane, const EscList &l, int eoff, uint32_t em, int colb,
                                         bool inl_only, uint32_t *err, int hmin) {
  if (!em) return;
  const uint16_t *cells = (const uint16_t *)(lds + lane * 8);
  int j = eoff;
  bool low = false;
  for (uint32_t m = em; m; m &= m - 1) {
    const int q = esc_cell(__builtin_ctz(m));
    const uint32_t c = cells[q];
    low |= c < (uint32_t)S_CELL(hmin, 0);
    *(inl_only ? l.inl + j : l.at(j)) = (uint32_t)(colb + q) | (c << 16);
    j++;
  }
  if (low) atomicOr(err, GM_ERR_LAG);
}

// Payload nibbles (gm_scaled.h S_NIB_*): dword w of a lane's 8-byte slice holds cells
// 8w..8w+7; cell 8w+2k sits in nibble 3-k of the low u16, cell 8w+2k+1 in nibble 3-k
// of the high u16. So v_pk_max_u16 of the dword shifted left by 4k leaves, in the top
// nibble of each u16, the max over lists of cells (8w+2k, 8w+2k+1) -- the table word
// 4w+k: max() of u16 lanes is decided by the top nibble whatever the bits below it.
__device__ __forceinline__ void nib_max(u16x2 acc[8], uint32_t x0, uint32_t x1) {
  const u16x2 a = pk(x0), b = pk(x1);
  acc[0] = __builtin_elementwise_max(acc[0], a);
  acc[1] = __builtin_elementwise_max(acc[1], a << (u16x2)(4));
  acc[2] = __builtin_elementwise_max(acc[2], a << (u16x2)(8));
  acc[3] = __builtin_elementwise_max(acc[3], a << (u16x2)(12));
  acc[4] = __builtin_elementwise_max(acc[4], b);
  acc[5] = __builtin_elementwise_max(acc[5], b << (u16x2)(4));
  acc[6] = __builtin_elementwise_max(acc[6], b << (u16x2)(8));
  acc[7] = __builtin_elementwise_max(acc[7], b << (u16x2)(12));
}
// nibble of lane cell q (0..15) in a lane slice (x0, x1)
__device__ __forceinline__ uint32_t nib_of(uint32_t x0, uint32_t x1, int q) {
  const uint32_t x = q < 8 ? x0 : x1;
  const int c = q & 7;
  return (x >> (16 * (c & 1) + 4 * (3 - (c >> 1)))) & 15u;
}
#define S_PESC_NONE 0xFFFFFFFFu  // payload escape record: no slots (overflow)
// escaped payload byte h' of lane li's cell q in sender sn's slice of tick parity pp: the
// sender's escaping lanes hold consecutive 16-byte slots from its record's base, in lane order
__device__ __forceinline__ uint32_t pesc_value(const SState &s, int pp, int band, int sn, int li, int q) {
  const uint4 rc = s.pesc_rec[pp][(size_t)band * s.n + sn];
  const uint64_t m = (uint64_t)rc.y | ((uint64_t)rc.z << 32);
  const uint32_t slot = rc.x + (uint32_t)__builtin_popcountll(m & ((1ull << li) - 1));
  return rc.x == S_PESC_NONE || slot >= s.pesc_cap ? 0u : (uint32_t)s.pesc[pp][(size_t)slot * 16 + q];
}
// payload value of a delivered cell: h' from its nibble, or from the sender's escape slots
__device__ __forceinline__ uint32_t nib_value(uint32_t nb, const SState &s, int pp, int band, int sn, int li, int q) {
  return nb == S_NIB_ESC ? pesc_value(s, pp, band, sn, li, q) : nb ? S_NIB_H(nb) : 0u;
}

// Keyed loss of the SCALED regime (build-defined; the reference drops whole messages with
// rand() % 100 < MSG_DROP_PROB * 100, EmulNet.cpp:90-94): the entry of global column c in the list
// src sent to dst at tick t_send is lost iff 16-bit half (c & 1) of fmix32(pair ^ (c >> 1) * phi) is
// below T = ceil(pct * 65536 / 100) (s_drop_thresh), pair = low word of mix64(seed ^ t_send << 48 ^
// src << 24 ^ dst): one 32-bit hash per column pair, whose halves are exactly the two u16 halves
// of the packed nibble layout (oracle/ref_cpu.c scaled_recv states the same function)
#define S_PHI 0x9E3779B9u
__device__ __forceinline__ uint32_t s_drop_pair(const SState &s, int t, int sn, int r) {
  return (uint32_t)gm_mix64(s.drop_seed ^ ((uint64_t)(uint32_t)(t - 1) << 48) ^ ((uint64_t)(uint32_t)sn << 24) ^
                            (uint64_t)(uint32_t)r);
}
__device__ __forceinline__ bool s_keep(const SState &s, int t, int sn, int r, int c, uint32_t T) {
  const uint32_t h = gm_fmix32(s_drop_pair(s, t, sn, r) ^ ((uint32_t)(c >> 1) * S_PHI));
  return ((h >> (16 * (c & 1))) & 0xFFFFu) >= T;
}
// payload nibble position of lane cell q (0..15) in its 8-byte slice (nib_max's order)
__device__ __forceinline__ constexpr int nib_pos(int q) { return 32 * (q >> 3) + 16 * (q & 1) + 4 * (3 - ((q & 7) >> 1)); }
// 0xF at the nibbles of the lane's kept cells in list sn -> row r (64 bits = the slice). Even c0:
// cells (2i, 2i+1) are a hash pair whose halves sit at the same nibble of the two u16 halves of
// dword i / 4 -- one fmix32 and four packed ops per pair; else one hash per cell (odd offsets)
__device__ __forceinline__ uint64_t s_keep_nibbles(const SState &s, int t, int sn, int r, int colb, uint32_t T,
                                                   bool agrp) {
  const uint32_t pair = s_drop_pair(s, t, sn, r);
  const int c = s.c0 + colb;
  if (T > 65535u) return 0;  // every entry lost
  if (agrp) {
    const u16x2 t2 = (u16x2)((uint16_t)T);
    uint32_t kw[2] = {0u, 0u};
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint32_t h = gm_fmix32(pair ^ ((uint32_t)((c >> 1) + i) * S_PHI));
      const u16x2 drop = pmin1(__builtin_elementwise_sub_sat(t2, pk(h)));  // 1 where the half is < T
      kw[i >> 2] |= unpk(((u16x2)(1) - drop) * (u16x2)(0xFu << (4 * (3 - (i & 3)))));
    }
    return (uint64_t)kw[0] | ((uint64_t)kw[1] << 32);
  }
  uint64_t km = 0;
  for (int q = 0; q < 16; q++) {
    const uint32_t h = gm_fmix32(pair ^ ((uint32_t)((c + q) >> 1) * S_PHI));
    if (((h >> (16 * ((c + q) & 1))) & 0xFFFFu) >= T) km |= 0xFull << nib_pos(q);
  }
  return km;
}
// bit 4i set where nibble i of x is non-zero
__device__ __forceinline__ uint32_t nz_nibble_bits(uint32_t x) { return (x | (x >> 1) | (x >> 2) | (x >> 3)) & 0x11111111u; }

// One work unit of the band sweep: unit u = (band u / U, rows [(u % U) * RPW, +RPW)).
// unit_load issues the row metadata and the table slice; unit_gather the payload slices
// (needs the sender ids); unit_finish merges, sweeps, stores and records the counts.
template <int B>
struct UnitIn {
  int band, r, k;  // k: lists delivered to this lane's row, -1 = not merged (crashed / absent / not in the group)
  int snd[S_SB];
  u32x4 ta;        // the row's 16 cell bytes of this lane (as loaded)
  uint32_t ebase;  // the row slice's escape list in the pool of tick t-1 (S_PESC_NONE: none)
  uint32_t bz;     // the (band, row) record's count word of tick t-1 (S_BC_PRES: present cells as loaded)
  uint64_t evc;    // evcum of the (row, band) as of tick t-1 (uni: read by unit_load)
  bool uni;        // the fast path's unit: its evcum cell is written back plainly, not by an atomic
  const uint8_t *msg;     // s.msg and the inline escape entries of tick t-1, read with the row's
  const uint32_t *tesc;   // kernel-argument words (unit_load)
};

// the unit's table slice (this lane's 16 cell bytes); r >= n: out of range -> zeros
template <int B>
__device__ __forceinline__ void unit_table(const SState &s, UnitIn<B> &in) {
  constexpr int LPR = B / S_COLS_PER_LANE, Q = S_COLS_PER_LANE;
  const int li = (threadIdx.x & 63) % LPR;
  const __amdgpu_buffer_rsrc_t trs = gm_rsrc(s.table + (size_t)in.band * s.n * B, (uint32_t)(s.n * B));
  in.ta = __builtin_amdgcn_raw_buffer_load_b128(trs, (uint32_t)(in.r * B + li * Q), 0, GM_AUX_NT);
}

// UNI: the row is wave-uniform and known to be (one row per wave, a grid-derived unit)
// in2 (one row per wave): the same row's unit in band2 -- the row's inbox, count and state are shared,
// its record words and evcum cell load with this unit's; its table slice issues later (unit_table)
template <int B, bool UNI = false, bool EVC = false, bool TWO = false>
__device__ __forceinline__ void unit_load(const SState &s, int t, int band, int ub, UnitIn<B> &in,
                                          UnitIn<B> &in2, int band2) {
  constexpr int LPR = B / S_COLS_PER_LANE, RPW = 64 / LPR;
  const int sub = (threadIdx.x & 63) / LPR;
  in.band = band;
  in.r = ub * RPW + sub;
  in.msg = s.msg;
  in.tesc = (t & 1) ? s.tesc_in[0] : s.tesc_in[1];
  if (UNI) asm("" : "+s"(in.msg), "+s"(in.tesc));
  const size_t slab = (size_t)in.band * s.n;
  // the table slice first: it is independent of the metadata, both in flight together
  unit_table<B>(s, in);
  const RowMeta<B> meta = row_meta<B, UNI, EVC>(s, in.r, t & 1, t, slab, band, TWO ? band2 : -1);
#pragma unroll
  for (int j = 0; j < S_SB; j++) in.snd[j] = meta.snd[j];
  in.k = meta.k;
  in.ebase = meta.ebase;
  in.bz = meta.bz;
  in.evc = meta.evc;
  in.uni = EVC;
  if (TWO) {
    in2.band = band2;
    in2.r = in.r;
#pragma unroll
    for (int j = 0; j < S_SB; j++) in2.snd[j] = meta.snd[j];
    in2.k = meta.k;
    in2.ebase = meta.ebase2;
    in2.bz = meta.bz2;
    in2.evc = meta.evc2;
    in2.uni = EVC;
    in2.msg = in.msg;
    in2.tesc = in.tesc;
  }
}
template <int B, bool UNI = false, bool EVC = false>
__device__ __forceinline__ void unit_load(const SState &s, int t, int band, int ub, UnitIn<B> &in) {
  unit_load<B, UNI, EVC, false>(s, t, band, ub, in, in, -1);
}


// every payload slice at once; slots j >= k read out of range (zeros = "not sent"); with them,
// lane li < 16 of a row whose slice held escaped cells fetches entry li of its list (ent)
template <int B, bool DROP>
__device__ __forceinline__ void unit_gather(const SState &s, int t, const UnitIn<B> &in, u32x2 m[S_SB], uint32_t &ent) {
  constexpr int LPR = B / S_COLS_PER_LANE;
  const int li = (threadIdx.x & 63) % LPR;
  ent = 0;
  if (li < (int)min(S_EW_TOT(in.ebase), (uint32_t)S_ESC_IN))
    ent = gld(in.tesc + ((size_t)in.band * s.n + in.r) * S_ESC_IN + li);
  const __amdgpu_buffer_rsrc_t prs = gm_rsrc(in.msg + (size_t)in.band * s.n * B, (uint32_t)(s.n * B));
  const uint32_t poff = (uint32_t)(((t & 1) ^ 1) * (B / 2) + li * 8);  // + sender * B
  const int k = min(in.k, S_KMAX);
#pragma unroll
  for (int j = 0; j < S_SB; j++)
    m[j] = __builtin_amdgcn_raw_buffer_load_b64(prs, j < k ? poff + (uint32_t)in.snd[j] * B : GM_OOB, 0, 0);
}

// The unit's commit, shared by both paths of unit_finish. unit_stores (a merged row's lanes): the
// swept slice's table bytes and payload nibbles, and its escape list; returns the list's word.
template <int B>
__device__ __forceinline__ uint32_t unit_stores(const SState &s, int t, const UnitIn<B> &in, const uint32_t bw[4],
                                                uint32_t ov0, uint32_t ov1, bool esc_row, uint32_t em, uint32_t *lds) {
  constexpr int LPR = B / S_COLS_PER_LANE;  // lanes per row
  constexpr int Q = S_COLS_PER_LANE;        // cells per lane
  const int lane = threadIdx.x & 63;
  const int par = t & 1;
  const int li = lane % LPR;
  const int band = in.band, r = in.r;
  const size_t slab = (size_t)band * s.n;
  const __amdgpu_buffer_rsrc_t trs = gm_rsrc(s.table + slab * B, (uint32_t)(s.n * B));
  const __amdgpu_buffer_rsrc_t prs = gm_rsrc(s.msg + slab * B, (uint32_t)(s.n * B));
  const uint32_t toff = (uint32_t)(r * B + li * Q);  // bytes
  uint32_t eb_out = 0;
  const u32x4 nb4 = {bw[0], bw[1], bw[2], bw[3]};
  __builtin_amdgcn_raw_buffer_store_b128(nb4, trs, toff, 0, GM_AUX_NT);
  const u32x2 ov = {ov0, ov1};
  __builtin_amdgcn_raw_buffer_store_b64(ov, prs, (uint32_t)(r * B + par * (B / 2) + li * 8), 0, GM_AUX_NT);
  if (band == 0 && li == 0) s.wtick[r] = t;
  if (esc_row) {  // the escaped cells as entries of this tick's list (the record's .w)
    int etot;
    const int eoff = row_scan<LPR>(__builtin_popcount(em), li, lane, etot);
    eb_out = row_alloc<LPR>(s, par, slab, r, etot, li, lane);
    if (eb_out != 0) esc_emit(lds, lane, esc_list(s, par, slab, r, eb_out), eoff, em, li * Q, etot <= S_ESC_IN, s.err, s.lag_hmin);
  }
  return eb_out;
}

// unit_records (every lane): the (band, row) record (rank-select chunk counts, the row's present /
// numfailed / event counts, the escape-list word eb_out), the events, a column shard's exchange
// slot. live: the row was merged and swept (else only its record is written).
// pre (one row per wave, the fast path): the chunk counts and row totals were reduced by the caller
// (row_counts), which needed the totals first -- piece_in / pf_in, not reduced again here
struct RowCounts {
  uint64_t piece;  // present cells per 128-column chunk, one byte each
  int pf;          // the row slice's present | numfailed << 16
};
// one row per wave: the present | numfailed counts per 8-lane chunk on DPP (xor 1, xor 2 by quad_perm,
// then + the mirrored lane of the other quad), the 8 chunk words by readlane on the scalar side
__device__ __forceinline__ RowCounts row_counts(int npres, int nfail) {
  int pf = npres | (nfail << 16);
  pf += __builtin_amdgcn_update_dpp(0, pf, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  pf += __builtin_amdgcn_update_dpp(0, pf, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  pf += __builtin_amdgcn_update_dpp(0, pf, 0x141, 0xF, 0xF, false);  // row_half_mirror
  RowCounts rc;
  rc.piece = 0;
  rc.pf = 0;
#pragma unroll
  for (int c = 0; c < 8; c++) {
    const int v = __builtin_amdgcn_readlane(pf, 8 * c);
    rc.piece |= (uint64_t)(v & 0xFF) << (8 * c);
    rc.pf += v;
  }
  return rc;
}
template <int B, bool DROP>
__device__ __forceinline__ void unit_records(const SState &s, int t, const UnitIn<B> &in, bool live, uint32_t eb_out,
                                             int npres, int nfail, int nev, uint32_t evk, int nkept,
                                             const RowCounts *pre = nullptr) {
  constexpr int LPR = B / S_COLS_PER_LANE;  // lanes per row
  constexpr int Q = S_COLS_PER_LANE;        // cells per lane
  const int lane = threadIdx.x & 63;
  const int sub = lane / LPR, li = lane % LPR;
  const int band = in.band, r = in.r;
  const int colb = band * B + li * Q;  // shard-local column of this lane's first cell
  const size_t slab = (size_t)band * s.n;
  if (DROP && s.mc_rdrop) {  // msgcount: the row's kept entries (wave-uniform test)
    int v = nkept;
#pragma unroll
    for (int o = 1; o < LPR; o <<= 1) v += __shfl_xor(v, o, 64);
    if (live && li == 0 && v) atomicAdd(&s.mc_rdrop[r], (uint32_t)v);
  }
  // present cells per 64-column chunk (4 lanes) for the draw's rank-select, gathered
  // into the row's first lane: bytes 0..B/64-1 of the (band, row) record
  constexpr int CH = S_CHUNK(B), LPC = CH / Q;  // columns / lanes per rank-select chunk
  // per-row reductions over the row's LPR lanes (aligned lane segments): counts packed
  // as present | numfailed << 16 (each <= B)
  int pf = npres | (nfail << 16);
  uint64_t piece = 0;
  if (LPR == 64 && LPC == 8 && pre) {
    piece = pre->piece;
    pf = pre->pf;
  } else if (LPR == 64 && LPC == 8) {
    const RowCounts rc = row_counts(npres, nfail);
    piece = rc.piece;
    pf = rc.pf;
  } else {
    int cc = npres;
#pragma unroll
    for (int o = 1; o < LPC; o <<= 1) cc += __shfl_xor(cc, o, 64);
#pragma unroll
    for (int c = 0; c < B / CH; c++) piece |= (uint64_t)(__shfl(cc, sub * LPR + LPC * c, 64) & 0xFF) << (8 * c);
#pragma unroll
    for (int o = LPR / 2; o >= 1; o >>= 1) pf += __shfl_xor(pf, o, 64);
  }
  int x = 0, tot = 0;
  if (__builtin_amdgcn_ballot_w64(nev != 0)) {  // wave-uniform: events anywhere in this wave
    // cumulative (joins, removals) of this (row, band): ADD kinds are 01, REMOVE kinds 10
    int jr = __builtin_popcount(evk & 0x55555555u) | (__builtin_popcount(evk & 0xAAAAAAAAu) << 16);
    x = nev;
    if (LPR == 64) {  // one row per wave: inclusive scans on DPP, totals from lane 63
      x = dpp_scan(x);
      jr = dpp_scan(jr);
      tot = __builtin_amdgcn_readlane(x, 63);
      jr = __builtin_amdgcn_readlane(jr, 63);
    } else {
#pragma unroll
      for (int o = 1; o < LPR; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (li >= o) x += y;
      }
      tot = __shfl(x, sub * LPR + LPR - 1, 64);
#pragma unroll
      for (int o = LPR / 2; o >= 1; o >>= 1) jr += __shfl_xor(jr, o, 64);
    }
    // single writer per (row, band): one row per wave writes back the value row_meta read; otherwise
    // a no-return atomic (no wave waits on a load)
    if (live && li == 0 && jr) {
      const unsigned long long add = (unsigned long long)(jr & 0xFFFF) | ((unsigned long long)(jr >> 16) << 32);
      if (in.uni) s.evcum[(size_t)r * s.nb + band] = in.evc + add;  // the only writer of the cell (row_meta)
      else atomicAdd((unsigned long long *)&s.evcum[(size_t)r * s.nb + band], add);
    }
  }
  const int E = s.evs;
  uint32_t sbase = 0;  // one spill-ring reservation per (row, band) that overflows its slots
  if (live && li == 0 && tot > E) sbase = atomicAdd(s.ev_spill_cnt, (uint32_t)(tot - E));
  if (live && li == 0 && tot)  // the tick's total (host staging), striped partial sums
    atomicAdd(s.ev_spill_cnt + 1 + ((slab + (size_t)r) & (S_EV_STRIPES - 1)), (uint32_t)tot);
  sbase = LPR == 64 ? __builtin_amdgcn_readfirstlane(sbase) : __shfl(sbase, sub * LPR, 64);
  if (live && nev) {
    int slot = x - nev;
    uint32_t *slots = s.ev_band + ((size_t)r * s.nb + band) * E;
    for (uint32_t ek = evk; ek; ek &= ek - 1) {
      const int bit = __builtin_ctz(ek);  // low bit of a set 2-bit kind field (ADD=1, REMOVE=2)
      const int q = bit >> 1;
      const uint32_t kind = (evk >> (2 * q)) & 3u;
      const uint32_t rec = (kind << 30) | (uint32_t)(s.c0 + colb + q + 1);
      if (slot < E) {
        slots[slot] = rec;
      } else {
        const uint32_t sp = sbase + (uint32_t)(slot - E);
        if (sp < s.ev_spill_cap) s.ev_spill[sp] = ((uint64_t)(uint32_t)r << 32) | rec;
        else atomicOr(s.err, GM_ERR_EVENTS);
      }
      slot++;
    }
  }
  if (li == 0 && r < s.n) {
    // one 16-byte record per (band, row), consecutive rows adjacent: whole-line writes
    const uint32_t bc = (uint32_t)(pf & 0xFFFF) | ((uint32_t)(pf >> 16) << 11) | ((uint32_t)min(tot, 1023) << 22);
    s.brec[slab + r] = live ? make_uint4((uint32_t)piece, (uint32_t)(piece >> 32), bc, eb_out)
                            : make_uint4(0u, 0u, 0u, eb_out);
    // (a column shard's row totals for the all-gather are summed from these records by gm_s_xrows)
  }
}

template <int B, bool DROP>
__device__ __forceinline__ void unit_finish(const SState &s, int t, int drop_pct, const UnitIn<B> &in,
                                            const u32x2 m[S_SB], uint32_t ent, uint32_t *lds) {
  constexpr int LPR = B / S_COLS_PER_LANE;  // lanes per row
  constexpr int RPW = 64 / LPR;             // rows per wave
  constexpr int Q = S_COLS_PER_LANE;        // cells per lane (8 packed pairs)
  const int lane = threadIdx.x & 63;
  const int par = t & 1;
  const int sub = lane / LPR, li = lane % LPR;
  const int band = in.band, r = in.r;
  const int colb = band * B + li * Q;  // shard-local column of this lane's first cell
  const size_t slab = (size_t)band * s.n;
  // this band's slabs: table [n][B] cell bytes, payload nibbles [n][2][B/2] bytes (32-bit offsets)
  const __amdgpu_buffer_rsrc_t trs = gm_rsrc(s.table + slab * B, (uint32_t)(s.n * B));
  const __amdgpu_buffer_rsrc_t prs = gm_rsrc(s.msg + slab * B, (uint32_t)(s.n * B));
  const uint32_t toff = (uint32_t)(r * B + li * Q);  // bytes
  const uint32_t poff = (uint32_t)((par ^ 1) * (B / 2) + li * 8);  // + sender * B
  int k = in.k;
  if (k > S_KMAX) {
    if (li == 0) atomicOr(s.err, GM_ERR_INBOX);
    k = S_KMAX;
  }
  const bool live = k >= 0;
  const u32x4 ta = in.ta;
  struct {
    int snd[S_SB];
  } meta;
#pragma unroll
  for (int j = 0; j < S_SB; j++) meta.snd[j] = in.snd[j];
  // lists to merge in this wave (uniform loop bound)
  int kw = 0;
  {
    const int kl = live ? k : 0;
#pragma unroll
    for (int w = 0; w < RPW; w++) kw = max(kw, __builtin_amdgcn_readlane(kl, w * LPR));
  }
  int npres = 0, nfail = 0, nev = 0;
  int nkept = 0;     // DROP: delivered entries this lane kept after the keyed loss (msgcount)
  uint32_t evk = 0;  // 2 bits per cell: event kind
  bool esc_st = false;  // this lane stored escaped cells
  uint32_t eb_out = 0;  // the row slice's escape-list word of this tick (the record's .w)
  if (!live && in.ebase != 0) {
    // a row not swept this tick (crashed, not yet in the group) keeps its cells as they are: its
    // escape list moves to this tick's storage (row-uniform branch; entries carry their columns)
    const int etot = (int)S_EW_TOT(in.ebase);
    eb_out = row_alloc<LPR>(s, par, slab, r, etot, li, lane);
    if (eb_out != 0) {
      const EscList src = esc_list(s, par ^ 1, slab, r, in.ebase), dst = esc_list(s, par, slab, r, eb_out);
      constexpr int P = LPR < S_ESC_IN ? LPR : S_ESC_IN;  // entries prefetched (one per lane)
      if (li < min(etot, P)) *dst.at(li) = ent;
      for (int i = P + li; i < etot; i += LPR) *dst.at(i) = *src.at(i);
    }
  }
  if (live) {
    // merge key per cell = the largest delivered payload h' (0 = nothing delivered), as
    // key5 = h' << 5 (the cell with age 0) in the u16 halves of each table word
    const int32_t *ib = s.inbox[par] + (size_t)r * S_KMAX;
    u16x2 key5[8];
    {
      // DROP (keyed loss on this tick's deliveries): a list's lost entries are cleared from its
      // nibbles before the max, per (list, lane) from 4 hashes of the pair key (s_keep_bits)
      const uint32_t T = DROP ? s_drop_thresh(drop_pct) : 0u;
      const bool agrp = ((s.c0 + colb) & 1) == 0;  // shard-uniform: the lane's cells are 8 whole hash pairs
      u16x2 acc[8];
#pragma unroll
      for (int i = 0; i < 8; i++) acc[i] = (u16x2)(0);
      auto merge_list = [&](int sn, uint32_t x0, uint32_t x1) {
        if (DROP) {
          if (!(x0 | x1)) return;
          const uint64_t km = s_keep_nibbles(s, t, sn, r, colb, T, agrp);
          x0 &= (uint32_t)km;
          x1 &= (uint32_t)(km >> 32);
          if (s.mc_rdrop) nkept += __builtin_popcount(nz_nibble_bits(x0)) + __builtin_popcount(nz_nibble_bits(x1));
        }
        nib_max(acc, x0, x1);
      };
#pragma unroll
      for (int j = 0; j < S_SB; j++)
        if (j < kw) merge_list(meta.snd[j], m[j].x, m[j].y);  // slots j >= k loaded zeros
      for (int j = S_SB; j < k; j++) {  // rare: more lists than prefetched ids
        const int sn = ib[j];
        const u32x2 mv = __builtin_amdgcn_raw_buffer_load_b64(prs, poff + (uint32_t)sn * B, 0, 0);
        merge_list(sn, mv.x, mv.y);
      }
      u16x2 nmax = (u16x2)(0);
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const u16x2 nb = acc[i] >> (u16x2)(12);
        nmax = __builtin_elementwise_max(nmax, nb);
        // h' = 224 + 2n for n >= 1: key5 = 7168 + 64 n, 0 for n = 0
        key5[i] = pmin1(nb) * (u16x2)(S_NIB_BASE << 5) + nb * (u16x2)(64);
      }
      if (__builtin_elementwise_max(nmax.x, nmax.y) == S_NIB_ESC) {
        // rare (cold start, JOINREQ entries, lag > 13 ticks): some list escaped a cell of
        // this lane; the exact key of those cells = max over the (kept) lists' decoded values
#pragma unroll
        for (int i = 0; i < 8; i++) {
          const u16x2 nb = acc[i] >> (u16x2)(12);
#pragma unroll
          for (int h = 0; h < 2; h++) {
            if (nb[h] != S_NIB_ESC) continue;
            const int q = 2 * i + h;
            uint32_t kv = 0;
            for (int j = 0; j < k; j++) {  // reloads (no dynamic register indexing: no scratch)
              const int sn = ib[j];
              if (DROP && !s_keep(s, t, sn, r, s.c0 + colb + q, T)) continue;
              const u32x2 mm = __builtin_amdgcn_raw_buffer_load_b64(prs, poff + (uint32_t)sn * B, 0, 0);
              kv = max(kv, nib_value(nib_of(mm.x, mm.y, q), s, par ^ 1, band, sn, li, q));
            }
            key5[i][h] = (uint16_t)(kv << 5);
          }
        }
      }
    }
    if (s.ramp && r == 0) {  // the introducer takes the JOINREQs of the nodes that started at t-1:
      // entry {hb 0, ts t} = stored heartbeat 2t (offset 2(t-1+1)) = h 255 (MP1Node.cpp:226-251)
#pragma unroll
      for (int q = 0; q < Q; q++) {
        const int c = s.c0 + colb + q;  // a real column of this shard (not row padding)
        if (c >= 1 && colb + q < s.w && s_start(c) == t - 1) key5[q >> 1][q & 1] = (uint16_t)(255u << 5);
      }
    }
    // widen the stored bytes to 16-bit cells; a row slice holding escaped cells (rare: a crashed
    // node's entries before their removal, cold-start / JOINREQ entries) takes those from its
    // list in the last tick's pool. npb: cells present as loaded (join detection below).
    const uint32_t tb4[4] = {ta.x, ta.y, ta.z, ta.w};
    u16x2 tw[8], npb = (u16x2)(0);
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const u16x2 x = pk(byte_pair(tb4[i >> 1], i & 1));
      const u16x2 nz = pmin1(x);
      npb = padd(npb, nz);
      tw[i] = widen2(x, nz);
    }
    if (in.ebase != 0)  // row-uniform: the row slice held escaped cells after the last tick
      esc_apply<LPR>(lds, lane, li, esc_list(s, par ^ 1, slab, r, in.ebase), (int)S_EW_TOT(in.ebase), ent, tw);
    // merge: re-base the cell to tick t (h -= 2, age += 1; absent stays 0), then max
    // with the delivered key (insert if absent; raise hb and stamp ts = t if newer)
    u16x2 mm[8];
#pragma unroll
    for (int i = 0; i < 8; i++)
      mm[i] = __builtin_elementwise_max(__builtin_elementwise_sub_sat(tw[i], (u16x2)(63)), key5[i]);
    const int selfc = (r >= s.c0 && r < s.c0 + s.w) ? r - s.c0 - colb : -1;
    int selfapp = -1;  // lane cell of an appended self entry: no join record (push_back, not logNodeAdd)
    if (selfc >= 0 && selfc < Q) {  // updateMyPos + heartbeat++ + myPos->setheartbeat(heartbeat++)
      const int hb = s.hbctr[r] + 1;
      s.hbctr[r] = hb + 1;
      // myPos = lower_bound(self) (MP1Node.cpp:308-322): self if present; else, by the `&&` at
      // :316, the next larger id if one is present -- that entry takes the heartbeat and ts
      // (the quirk); else self is appended. Nodes of one start tick (ids 4g..4g+3) share this
      // lane, and the quirk's target is always one of them in practice (gm_s_selfcheck turns
      // any other case into GM_ERR_SELF)
      int tq = selfc;
      uint32_t selfcell = 0;
#pragma unroll
      for (int q = 0; q < Q; q++)
        if (q == selfc) selfcell = (unpk(mm[q >> 1]) >> (16 * (q & 1))) & 0xFFFFu;
      if (selfcell == 0) {
        if (!s.ramp) {
          atomicOr(s.err, GM_ERR_SELF);
        } else {
#pragma unroll
          for (int q = Q - 1; q >= 0; q--)  // smallest present id above self in the group
            if (q > selfc && q <= (selfc | 3) && ((unpk(mm[q >> 1]) >> (16 * (q & 1))) & 0xFFFFu)) tq = q;
          if (tq == selfc) {  // appended: verify afterwards that no larger id was present
            selfapp = selfc;
            const uint32_t slot = atomicAdd(s.selfadd_cnt, 1u);
            if (slot < S_SELFADD_CAP) s.selfadd[slot] = r;
            else atomicOr(s.err, GM_ERR_SELF);
            // column shards: the other ranks check their (higher) columns in gm_s_draw
            if (s.sharded) atomicOr((uint32_t *)(s.xcnt + S_XC(s, s.shard_rank, r)), S_XC_SELFAPP);
          }
        }
      }
      if (s.ramp) s.mecol[r] = s.c0 + colb + tq;
      const int h = 255 - (2 * t - (hb + s_hbase(s.ramp, s.c0 + colb + tq)));
      if (h < s.lag_hmin || h > 255) atomicOr(s.err, GM_ERR_LAG);
#pragma unroll
      for (int i = 0; i < 8; i++) {
        if ((tq >> 1) != i) continue;
        uint32_t v = unpk(mm[i]);
        const int sh = 16 * (tq & 1);
        v = (v & ~(0xFFFFu << sh)) | ((uint32_t)S_CELL(h, 0) << sh);
        mm[i] = pk(v);
      }
    }
    // sweep (MP1Node.cpp:426-444), one packed pass: age >= TFAIL counts toward numfailed,
    // age >= TREMOVE removes; fresh entries (age < TFAIL) form the payload sent at tick t.
    // The swept cell is narrowed to its stored byte (S_B_ESC where the byte cannot hold it).
    // A fresh stored byte h4 << 4 | a sends h' = h - 2, i.e. the nibble h4 - 1 (>= 2: h4 >= 3);
    // escaped cells send the escape nibble 15 (their byte h' goes to the payload's wide plane).
    u16x2 np2 = (u16x2)(0), nf2 = (u16x2)(0), badv = (u16x2)(0), nmx = (u16x2)(0), amax = (u16x2)(0);
    u16x2 nwv[2] = {(u16x2)(0), (u16x2)(0)};
    uint32_t cw[8], bw[4], bprev = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const u16x2 v = mm[i];
      const u16x2 a = v & (u16x2)(31);
      const u16x2 stale = (a + (u16x2)(32 - GM_TFAIL)) >> (u16x2)(5);  // age >= TFAIL
      amax = __builtin_elementwise_max(amax, a);  // TREMOVE removals (rare) are applied below
      const u16x2 pres = pmin1(v);
      nf2 = padd(nf2, stale);
      np2 = padd(np2, pres);
      u16x2 bad;
      const u16x2 b = narrow2(v, pres, bad);
      // payload nibble of the fresh present cells: h4 - 1, or 15 where that is 0 (h4 <= 1)
      const u16x2 p = __builtin_elementwise_sub_sat(pres, stale);
      const u16x2 qn = __builtin_elementwise_sub_sat(b >> (u16x2)(4), (u16x2)(1));
      const u16x2 nib = p * (__builtin_elementwise_sub_sat((u16x2)(1), qn) * (u16x2)(S_NIB_ESC) + qn);
      nwv[i >> 2] = nwv[i >> 2] + nib * (u16x2)(1u << (4 * (3 - (i & 3))));
      badv |= bad;
      nmx = __builtin_elementwise_max(nmx, nib);
      cw[i] = unpk(v);
      if (i & 1) bw[i >> 1] = __builtin_amdgcn_perm(unpk(b), bprev, 0x06040200u);
      else bprev = unpk(b);
    }
    int ngone = 0;
    uint32_t gmask = 0;  // lane cells removed this tick (bit q = cell q)
    if (__builtin_elementwise_max(amax.x, amax.y) >= GM_TREMOVE) {
      // rare: age >= TREMOVE removes (MP1Node.cpp:429-444): the removed cells' stored bytes
      // become 0 (absent) and leave the present count. They sent nothing (stale: the nibbles
      // stand) and were escaped (age > 15), so the lane's escape flag is re-taken from the stored
      // bytes. cw keeps their old cells: only the escape mask's cells and fresh cells are read
      // from it afterwards
      u16x2 ng2 = (u16x2)(0);
      uint32_t gprev = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const u16x2 v = pk(cw[i]);
        const u16x2 gone = ((v & (u16x2)(31)) + (u16x2)(32 - GM_TREMOVE)) >> (u16x2)(5);
        gmask |= ((unpk(gone) & 1u) | ((unpk(gone) >> 15) & 2u)) << (2 * i);
        ng2 = padd(ng2, gone);
        const uint32_t gb = unpk(gone * (u16x2)(0xFF));  // 0xFF in the low byte of a removed cell's half
        if (i & 1) bw[i >> 1] &= ~__builtin_amdgcn_perm(gb, gprev, 0x06040200u);
        else gprev = gb;
      }
      np2 = np2 - ng2;
      ngone = (int)ng2.x + (int)ng2.y;
      badv = (u16x2)(esc_mask16(bw[0], bw[1], bw[2], bw[3]) != 0 ? 1 : 0);
    }
    esc_st = unpk(badv) != 0;
    const bool esc_row = row_any<LPR>(esc_st, sub);
    uint32_t em = 0;  // the lane's escaped cells (entries of this tick's list, emitted after the stores)
    if (esc_row) {  // rare: cells the byte cannot hold; the lane's cells wait in its LDS slot
      if (esc_st) {  // (a present cell with h <= 2 escapes: esc_emit flags it)
        em = esc_mask16(bw[0], bw[1], bw[2], bw[3]);
        esc_park(lds, lane, cw);
      }
    }
    const bool pesc = __builtin_elementwise_max(nmx.x, nmx.y) == S_NIB_ESC;
    if (row_any<LPR>(pesc, sub)) {
      // rare: the escaping lanes' 16 payload bytes h' into consecutive slots of this tick's payload
      // pool (read where a receiver meets nibble 15), one reservation per row
      const uint64_t bal = __builtin_amdgcn_ballot_w64(pesc);
      const uint64_t rm = LPR == 64 ? bal : (bal >> (sub * LPR)) & ((1ull << LPR) - 1);
      uint32_t pbase = S_PESC_NONE;
      if (li == 0) {
        const int ps = esc_stripe(s, slab, r);
        const unsigned long long b = atomicAdd(s.pesc_cnt + par * s.esc_stripes + ps, (unsigned long long)__builtin_popcountll(rm));
        if (b + (unsigned long long)__builtin_popcountll(rm) <= (unsigned long long)s.pesc_region)
          pbase = (uint32_t)ps * s.pesc_region + (uint32_t)b;
        else atomicOr(s.err, GM_ERR_ESC);
        s.pesc_rec[par][slab + r] = make_uint4(pbase, (uint32_t)rm, (uint32_t)(rm >> 32), 0u);
      }
      pbase = LPR == 64 ? __builtin_amdgcn_readfirstlane(pbase) : (uint32_t)__shfl((int)pbase, lane - li, 64);
      uint32_t pw[8];
#pragma unroll
      for (int i = 0; i < 8; i++) {  // removed cells send nothing: the swept cells suffice
        const u16x2 v = pk(cw[i]);
        const u16x2 stale = ((v & (u16x2)(31)) + (u16x2)(32 - GM_TFAIL)) >> (u16x2)(5);
        pw[i] = unpk(__builtin_elementwise_sub_sat(v >> (u16x2)(5), stale * (u16x2)(255) + (u16x2)(2)));
      }
      const u32x4 wv = {__builtin_amdgcn_perm(pw[1], pw[0], 0x06040200u), __builtin_amdgcn_perm(pw[3], pw[2], 0x06040200u),
                        __builtin_amdgcn_perm(pw[5], pw[4], 0x06040200u), __builtin_amdgcn_perm(pw[7], pw[6], 0x06040200u)};
      if (pesc && pbase != S_PESC_NONE)
        *(u32x4 *)(s.pesc[par] + ((size_t)pbase + __builtin_popcountll(rm & ((1ull << li) - 1))) * 16) = wv;
    }
    nfail = (int)nf2.x + (int)nf2.y;
    npres = (int)np2.x + (int)np2.y;
    // joins: present after the merge (npres + ngone) but not as loaded (npb) -- the merge never
    // deletes; removals: ngone. Rare: this lane's events, as 2-bit kinds per cell
    if (npres + ngone == (int)npb.x + (int)npb.y && ngone) {
      // removals only (the crash case): REMOVE kinds (10) at the removed cells
      uint32_t x = gmask;
      x = (x | (x << 8)) & 0x00FF00FFu;
      x = (x | (x << 4)) & 0x0F0F0F0Fu;
      x = (x | (x << 2)) & 0x33333333u;
      x = (x | (x << 1)) & 0x55555555u;
      evk = x << 1;
      nev = __builtin_popcount(gmask);
    } else if (npres + ngone != (int)npb.x + (int)npb.y) {
      // joins (and possibly removals): the bytes as loaded, re-read (still in memory: the
      // stores come below) rather than kept live through the sweep for this rare path
      const u32x4 ra = __builtin_amdgcn_raw_buffer_load_b128(trs, toff, 0, 0);
      const uint32_t tb0[4] = {ra.x, ra.y, ra.z, ra.w};
#pragma unroll
      for (int q = 0; q < Q; q++) {  // from the loaded and the swept cells only (the merge never deletes:
        // present before and absent after = removed; a cell inserted this tick has age 0)
        const uint32_t before = (tb0[q >> 2] >> (8 * (q & 3))) & 0xFFu;
        const uint32_t after = (bw[q >> 2] >> (8 * (q & 3))) & 0xFFu;  // stored byte: 0 = absent
        const uint32_t ev = !before ? (after && q != selfapp ? S_EV_ADD : 0u) : (!after ? S_EV_REMOVE : 0u);
        evk |= ev << (2 * q);
      }
      nev = __builtin_popcount((evk | (evk >> 1)) & 0x55555555u);
    }
    eb_out = unit_stores<B>(s, t, in, bw, unpk(nwv[0]), unpk(nwv[1]), esc_row, em, lds);
  }
  unit_records<B, DROP>(s, t, in, live, eb_out, npres, nfail, nev, evk, nkept);
}

// ------------------------------------------------------------ gm_s_band fast path
// Lane-mask bit p in esc_mask16's order is cell esc_cell(p); esc_bit is the inverse.
__device__ __forceinline__ int esc_bit(int q) { return ((q & 3) << 3) | (q >> 2); }
// set bits of a wave mask below this lane
__device__ __forceinline__ int p_lanes_below(uint64_t b) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
}
// One marked cell of the fast path, exactly (16-bit cell c: the merged byte y widened, or the escaped
// cell re-based and merged; the general path's arithmetic): its stored byte, payload nibble (high-
// nibble form), whether it is removed (TREMOVE) or needs the wide payload plane (bail), and the
// corrections of the SWAR pass's present / stale counts, which counted the byte y.
struct FastCell {
  uint32_t nbyte, nib, c;
  bool gone, bail;
  int dpres, dfail;
};
__device__ __forceinline__ FastCell fast_cell(const SState &s, int t, uint32_t y, uint32_t c, bool self, int hbself) {
  FastCell o;
  if (self) {  // heartbeat++; myPos->setheartbeat(heartbeat++) (MP1Node.cpp:412-415)
    if (c == 0) atomicOr(s.err, GM_ERR_SELF);  // converged start: the own entry is always present
    const int h = 255 - (2 * t - hbself);
    if (h < s.lag_hmin || h > 255) atomicOr(s.err, GM_ERR_LAG);
    c = (uint32_t)S_CELL(h, 0) & 0xFFFFu;
  }
  // branch-free (selects, not exec-mask branches: the scalar unit is what a divergent branch costs)
  const uint32_t age = c & 31u, h = c >> 5, hp = h - 2u;
  const bool pres = c != 0, stale = pres && age >= GM_TFAIL;
  o.gone = pres && age >= GM_TREMOVE;  // TREMOVE (MP1Node.cpp:429-444): absent; it sent nothing (stale)
  const bool keep = pres && !o.gone;
  const bool fits = h >= S_H4_MIN_H && !(h & 1u) && age <= S_AGE_MAX_B;  // s_narrow's test
  o.nbyte = keep ? (fits ? ((((h - 224u) >> 1) << 4) | age) : S_B_ESC) : 0u;
  // fresh: the nibble of h' = h - 2, or the wide plane (general path)
  const bool fresh = keep && !stale;
  const bool nibok = !(hp & 1u) && hp >= S_NIB_H(1) && hp <= S_NIB_H(14);
  o.bail = fresh && !nibok;
  o.nib = fresh && nibok ? ((hp - S_NIB_BASE) >> 1) << 4 : 0u;
  o.c = c;
  const bool fpres = y >= 16u, fstale = fpres && (y & 15u) >= GM_TFAIL;
  o.dpres = (int)(pres && !o.gone) - (int)fpres;
  o.dfail = (int)stale - (int)fstale;
  return o;
}
// gm_s_band's fast path (one row per wave; no keyed loss, no join ramp): the merge and the sweep on
// the stored bytes themselves. A stored byte x = h4 << 4 | a (h4 >= 3, a <= 14: gm_scaled.h) re-based
// by one tick is x - 15 (h4 - 1, a + 1) and a delivered nibble n is the byte n << 4 (h' = 224 + 2n,
// age 0); bytes order as their cells do, so the merge of updatelistCallBack (MP1Node.cpp:278-299) is
// max(sat(x - 15), n << 4), and the sweep's counts (MP1Node.cpp:426-444) and the payload nibbles of
// sendMemberList (MP1Node.cpp:360-395: the fresh cells' h4 - 1) come from SWAR over the packed
// result, four cells per instruction. The rare cells are marked and redone one by one with the 16-bit
// cell, as the general path computes them: escaped cells (their value is the row slice's escape
// list's), results a byte cannot hold (age 15, h4 <= 2: they escape, or are removed at TREMOVE), and
// the row's own cell (heartbeat bump). A delivered escape nibble, or a fresh cell whose payload needs
// the wide plane, sends the whole wave to the general path: the function then returns false before
// any global store. Returns true when the unit is done.
// nxt: called at most once, as soon as the payload words m are consumed (or not needed): the wave's
// next unit issues its table slice and payload gathers into m there, in flight under this unit's sweep
// (a unit handed to the general path may return before it: the caller then issues them).
template <int B, typename F>
__device__ __forceinline__ bool unit_fast(const SState &s, int t, const UnitIn<B> &in, const u32x2 m[S_SB],
                                          uint32_t ent, uint32_t *lds, uint32_t *park, F &&nxt) {
  static_assert(B / S_COLS_PER_LANE == 64, "the fast path takes one row per wave");
  constexpr int Q = S_COLS_PER_LANE;
  const int lane = threadIdx.x & 63, li = lane;
  const int par = t & 1;
  const int band = in.band, r = in.r;
  const int colb = band * B + li * Q;  // shard-local column of this lane's first cell
  const size_t slab = (size_t)band * s.n;
  const int k = in.k;  // wave-uniform
  if (k > S_KMAX || s.ramp) return false;  // inbox error / join ramp: general path (nxt: as for a bail)
  if (k < 0) {  // a row not merged this tick (crashed): its cells stay as they are, its escape list moves
    nxt();        // to this tick's storage (entries carry their columns), its record is written
    uint32_t eb_out = 0;
    if (in.ebase != 0) {
      const int etot = (int)S_EW_TOT(in.ebase);
      eb_out = row_alloc<64>(s, par, slab, r, etot, li, lane);
      if (eb_out != 0) {
        const EscList src = esc_list(s, par ^ 1, slab, r, in.ebase), dst = esc_list(s, par, slab, r, eb_out);
        if (li < min(etot, S_ESC_IN)) *dst.at(li) = ent;
        for (int i = S_ESC_IN + li; i < etot; i += 64) *dst.at(i) = *src.at(i);
      }
    }
    unit_records<B, false>(s, t, in, false, eb_out, 0, 0, 0, 0u, 0);
    return true;
  }
  // 1. the delivered lists: per cell pair the largest nibble, in the top nibble of each u16 (nib_max)
  u16x2 acc[8];
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = (u16x2)(0);
#pragma unroll
  for (int j = 0; j < S_SB; j++)
    if (j < k) nib_max(acc, m[j].x, m[j].y);  // slots j >= k loaded zeros
  if (k > S_SB) {  // more lists than prefetched ids (a Poisson tail: ~7 % of rows at fanout 5)
    const __amdgpu_buffer_rsrc_t prs = gm_rsrc(s.msg + slab * B, (uint32_t)(s.n * B));
    const uint32_t poff = (uint32_t)((par ^ 1) * (B / 2) + li * 8);
    const int32_t *ib = s.inbox[par] + (size_t)r * S_KMAX;
    for (int j = S_SB; j < k; j++) {
      const int sn = ib[j];
      const u32x2 mv = __builtin_amdgcn_raw_buffer_load_b64(prs, poff + (uint32_t)sn * B, 0, 0);
      nib_max(acc, mv.x, mv.y);
    }
  }
  {
    u16x2 amx = acc[0];
#pragma unroll
    for (int i = 1; i < 8; i++) amx = __builtin_elementwise_max(amx, acc[i]);
    if (__builtin_amdgcn_ballot_w64(__builtin_elementwise_max(amx.x, amx.y) >= (uint16_t)(S_NIB_ESC << 12)))
      return false;  // a delivered escape nibble: its value is in the sender's wide plane
  }
  // 2. re-base and merge, two cells per u16x2, packed back to bytes
  const uint32_t tb4[4] = {in.ta.x, in.ta.y, in.ta.z, in.ta.w};
  uint32_t bw[4], yprev = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const u16x2 x = pk(byte_pair(tb4[i >> 1], i & 1));
    const u16x2 kb = (acc[i] >> (u16x2)(8)) & (u16x2)(0xF0);
    const u16x2 y = __builtin_elementwise_max(__builtin_elementwise_sub_sat(x, (u16x2)(15)), kb);
    if (i & 1) bw[i >> 1] = __builtin_amdgcn_perm(unpk(y), yprev, 0x06040200u);
    else yprev = unpk(y);
  }
  // 3. SWAR over the merged bytes: present (h4 >= 1) and stale (age >= TFAIL) counts, payload nibbles
  // (fresh present cells: h4 - 1, in the byte's high nibble), and the cells to redo
  int npres = 0, nfail = 0;
  uint32_t nb[4], spm = 0;
#pragma unroll
  for (int w = 0; w < 4; w++) {
    const uint32_t v = bw[w];
    const uint32_t lo = v & 0x0F0F0F0Fu;
    const uint32_t st = (lo + 0x01010101u * (16 - GM_TFAIL)) & 0x10101010u;  // age >= TFAIL
    const uint32_t a15 = (lo + 0x01010101u) & 0x10101010u;                   // age 15: not a byte next tick
    const uint32_t hi = v & 0xF0F0F0F0u;
    const uint32_t hs = hi >> 1;
    const uint32_t pr = (hs + 0x78787878u) & 0x80808080u;  // h4 >= 1: present
    const uint32_t g3 = (hs + 0x68686868u) & 0x80808080u;  // h4 >= 3
    nfail += __builtin_popcount(st);
    npres += __builtin_popcount(pr);
    spm |= ((pr & ~g3) | (a15 << 3)) >> (7 - w);  // esc_mask16's bit order
    uint32_t st4 = st << 4;
    asm volatile("" : "+v"(st4));  // else (st << 4) - st becomes a quarter-rate multiply by 15
    nb[w] = (hi - (pr >> 3)) & ~(st4 - st);
  }
  const int selfc = (r >= s.c0 && r < s.c0 + s.w) ? r - s.c0 - colb : -1;
  const bool selflane = selfc >= 0 && selfc < Q;
  int hbself = 0;
  if (selflane) {
    spm |= 1u << esc_bit(selfc);
    hbself = s.hbctr[r] + 1;
  }
  // 4. the marked cells, exactly (fast_cell). The lane's merged bytes and nibble bytes wait in LDS
  // (park: 32 B per lane), so that a cell is one byte read and two byte writes there, not register
  // selects. Escaped cells go entry-parallel: lane j takes entry j of the row slice's escape list (the
  // entries carry their columns) and that column's parked byte, whichever lane holds it; what the
  // holding lane needs back (that its cell was escaped, its removal bits, its count corrections) meets
  // in that lane's three words `cor` (LDS or / add). The other marked cells (age 15, h4 <= 2, the own
  // cell) are taken one by one in their own lane. An escaped cell that stays escaped is this tick's
  // list entry straight from its entry lane (sv / sent: VALU issue is what these ticks spend, and
  // the wave pays every instruction of a per-lane loop at its longest lane); past 64 entries (a cold
  // start) they go through the row's 16-bit cells like the per-lane loop's new ones.
  int ngone = 0;
  uint32_t gmask = 0, em = 0, sent = 0;
  bool sv = false, epar = true;
  const bool eslice = in.ebase != 0;  // row-uniform
  // 4a. the crash window's common case, without the park: no other cell is marked, the list fits its
  // inline slot, every escaped cell is stale and no delivered list has a fresh entry at its column
  // (its merged byte is 0). Then an escaped cell is only re-based (c - 63): it stays escaped -- its
  // entry lane writes it to this tick's list -- or reaches TREMOVE (a removal: the uniform loop over
  // the gone entries), and its holding lane restores the escape byte and counts the cell present
  // and stale, as fast_cell would (y = 0: dpres = dfail = 1; removed: dpres = 0, dfail = 1).
  bool quick = false;
  if (eslice && S_EW_TOT(in.ebase) <= S_ESC_IN && !__builtin_amdgcn_ballot_w64(spm != 0)) {
    const int etot = (int)S_EW_TOT(in.ebase);
    // 0x80 in the bytes whose stored cell is escaped (byte == S_B_ESC), exact per byte (recomputed
    // below rather than held across the ballot: registers are what sets this kernel's occupancy);
    // an escaped column is loud when its merged byte (the delivered nibble << 4) has a nonzero high
    // nibble -- the SWAR pass's present test on bw, no multiply
    auto esc_bytes = [&](int w) {
      const uint32_t z = tb4[w] ^ (0x01010101u * S_B_ESC);
      return ~(((z & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | z) & 0x80808080u;
    };
    bool loud = false;
#pragma unroll
    for (int w = 0; w < 4; w++) loud |= ((((bw[w] >> 1) & 0x78787878u) + 0x78787878u) & esc_bytes(w)) != 0u;
    const bool ent_lane = li < etot;
    const uint32_t ev = ent_lane ? ent >> 16 : 0u;
    const uint32_t c = ev ? ev - 63u : 0u;  // the re-based cell (y = 0 delivers nothing)
    const bool gone = ent_lane && (c & 31u) >= GM_TREMOVE;
    const bool fresh = ent_lane && (c & 31u) < GM_TFAIL;
    if (!__builtin_amdgcn_ballot_w64(loud || fresh)) {
      quick = true;
      int ne = 0;
#pragma unroll
      for (int w = 0; w < 4; w++) {
        const uint32_t eb = esc_bytes(w);
        static_assert(S_B_ESC == 1u, "the escape byte is restored as the detection mask's low bit");
        bw[w] |= eb >> 7;  // the escape byte S_B_ESC = 1 back (the merged byte there was 0)
        ne += __builtin_popcount(eb);
      }
      npres += ne;
      nfail += ne;
      const uint32_t col = ent & 0xFFFFu;
      if (__builtin_amdgcn_ballot_w64(gone)) {
        // TREMOVE ticks: each gone entry's lane sets, in the holding lane's LDS words, its cell's removal
        // bit and a 0xFF over its byte (one scatter for all of them -- a uniform step per gone entry
        // cost ~6 VALU each, ~5 per unit at the peak); the holding lanes read their words back. The
        // wave's LDS is free here: the quick path parks nothing, and stores no escape bytes (em = 0)
        uint32_t *gw = lds;                    // [64] removal bits per lane (cell order)
        u32x4 *gbm = (u32x4 *)(lds + 64);      // [64][4] byte masks per lane (cell 4w + b: byte b of word w)
        gw[li] = 0u;
        gbm[li] = (u32x4){0u, 0u, 0u, 0u};
        lds_wave_sync();
        if (gone) {
          const uint32_t ol = col / Q, q = col % Q;
          atomicOr(gw + ol, 1u << q);
          atomicOr(lds + 64 + 4 * ol + (q >> 2), 0xFFu << (8 * (q & 3)));
        }
        lds_wave_sync();
        gmask = gw[li];
        const u32x4 bm = gbm[li];
        lds_wave_sync();  // read back before any later use of the wave's LDS
        ngone = __builtin_popcount(gmask);
        npres -= ngone;
        bw[0] &= ~bm.x;  // the removed cells' bytes to 0 (absent)
        bw[1] &= ~bm.y;
        bw[2] &= ~bm.z;
        bw[3] &= ~bm.w;
      }
      sv = ent_lane && !gone;
      sent = col | (c << 16);
    }
  }
  const bool slow = !quick && (eslice || __builtin_amdgcn_ballot_w64(spm != 0));
  if (slow) {
    uint16_t *row16 = (uint16_t *)lds;  // the wave's LDS: a 16-bit cell per column (lane li: [16 li, +16))
    u32x4 *pk4 = (u32x4 *)(park + li * 8);
    pk4[0] = (u32x4){bw[0], bw[1], bw[2], bw[3]};
    pk4[1] = (u32x4){nb[0], nb[1], nb[2], nb[3]};
    uint8_t *pall = (uint8_t *)park;  // lane l's cell q: byte 32 l + q, its nibble byte 32 l + 16 + q
    uint8_t *pb = pall + li * 32;
    // per lane: cor[li] = its escaped cells as loaded (esc order), cor[64 + li] = removal bits (cell
    // order), cor[128 + li] = the present / stale corrections, packed as dpres + dfail << 16
    uint32_t *cor = park + S_LDS_WAVE_WORDS;
    if (eslice) cor[li] = cor[64 + li] = cor[128 + li] = 0u;
    lds_wave_sync();
    bool bail = false;
    uint32_t escm = 0;  // this lane's escaped cells (esc order): the entry lanes took them
    if (eslice) {
      const int tot = (int)S_EW_TOT(in.ebase);
      epar = tot <= 64;
      const int selfb = r - s.c0 - band * B;  // the own column in the band (row-uniform), if in [0, B)
      const int hbs = (selfb >= 0 && selfb < B) ? __builtin_amdgcn_readlane(hbself, selfb / Q) : 0;
      const EscList l = esc_list(s, par ^ 1, slab, r, in.ebase);
      for (int j0 = 0; j0 < tot; j0 += 64) {
        const int j = j0 + li;
        if (j < tot) {
          const uint32_t e = j < S_ESC_IN ? ent : *l.at(j);  // lane li < S_ESC_IN prefetched entry li
          const int col = (int)(e & 0xFFFFu), q = col % Q, ol = col / Q;
          uint8_t *cb = pall + ol * 32 + q;
          const uint32_t y = cb[0];  // the merged byte of an escaped cell: the delivered key alone
          const uint32_t ev = e >> 16;
          const FastCell o = fast_cell(s, t, y, max(ev ? ev - 63u : 0u, s_widen(y)), col == selfb, hbs);
          bail |= o.bail;
          // the holding lane's words, unconditionally (LDS ops with zero operands, no branches)
          atomicOr(cor + ol, 1u << esc_bit(q));
          atomicOr(cor + 64 + ol, o.gone ? 1u << q : 0u);
          atomicAdd(cor + 128 + ol, (uint32_t)(o.dpres + o.dfail * 65536));
          cb[0] = (uint8_t)o.nbyte;
          cb[16] = (uint8_t)o.nib;
          const bool eout = o.nbyte == S_B_ESC;  // an entry of this tick's list
          if (epar) {
            sv = eout;
            sent = (uint32_t)col | (o.c << 16);
          } else if (eout) {
            row16[col] = (uint16_t)o.c;  // esc_emit reads it here (em: the escape bytes, below)
          }
        }
      }
      lds_wave_sync();
      escm = cor[li];
    }
    for (uint32_t mm = spm & ~escm; mm; mm &= mm - 1) {
      const int p = __builtin_ctz(mm), q = esc_cell(p);
      const uint32_t y = pb[q];  // the merged byte (exact: the stored cell did not escape)
      const FastCell o = fast_cell(s, t, y, s_widen(y), q == selfc, hbself);
      bail |= o.bail;
      if (o.gone) {
        gmask |= 1u << q;
        ngone++;
      }
      if (o.nbyte == S_B_ESC) {
        em |= 1u << p;
        row16[li * Q + q] = (uint16_t)o.c;
      }
      npres += o.dpres;
      nfail += o.dfail;
      pb[q] = (uint8_t)o.nbyte;
      pb[16 + q] = (uint8_t)o.nib;
    }
    if (__builtin_amdgcn_ballot_w64(bail)) return false;  // (nxt not called: the caller issues it)
    lds_wave_sync();  // other lanes' entries wrote into this lane's park and words
    if (eslice) {
      const uint32_t ge = cor[64 + li], cd = cor[128 + li];
      gmask |= ge;
      ngone += __builtin_popcount(ge);
      const int dp = (int)(int16_t)(cd & 0xFFFFu);
      npres += dp;
      nfail += ((int)cd - dp) >> 16;
    }
    const u32x4 b0 = pk4[0], b1 = pk4[1];
    bw[0] = b0.x; bw[1] = b0.y; bw[2] = b0.z; bw[3] = b0.w;
    nb[0] = b1.x; nb[1] = b1.y; nb[2] = b1.z; nb[3] = b1.w;
    if (!epar) em = esc_mask16(bw[0], bw[1], bw[2], bw[3]);  // every escape byte: row16 holds its cell
  }
  // payload words in nib_max's order: the high nibbles of cells [4, 0, 5, 1] | those of [6, 2, 7, 3]
  // shifted down, for cells 0..7 and likewise 8..15
  const uint32_t ov0 = __builtin_amdgcn_perm(nb[1], nb[0], 0x01050004u) | (__builtin_amdgcn_perm(nb[1], nb[0], 0x03070206u) >> 4);
  const uint32_t ov1 = __builtin_amdgcn_perm(nb[3], nb[2], 0x01050004u) | (__builtin_amdgcn_perm(nb[3], nb[2], 0x03070206u) >> 4);
  // 5. events: removals = gmask; joins = cells present now but absent as loaded -- there are some iff
  // the slice's present cells before the sweep (npres + ngone over the row) differ from the count
  // the record kept of the last tick (first tick after gm_s_init: no count kept, so the cells are
  // compared; they are always compared where any differ)
  int nev = 0;
  uint32_t evk = 0;
  // (the record's chunk counts and totals, reduced once here: their present total is the sweep's, and
  // the removals are added only where there are some)
  const RowCounts rcnt = row_counts(npres, nfail);
  int tot = rcnt.pf & 0xFFFF;
  if (__builtin_amdgcn_ballot_w64(ngone != 0)) {
    int g = ngone;
    g += __builtin_amdgcn_update_dpp(0, g, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    g += __builtin_amdgcn_update_dpp(0, g, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    g += __builtin_amdgcn_update_dpp(0, g, 0x141, 0xF, 0xF, false);  // row_half_mirror
    g += __builtin_amdgcn_update_dpp(0, g, 0x140, 0xF, 0xF, false);  // row_mirror
    tot += __builtin_amdgcn_readlane(g, 0) + __builtin_amdgcn_readlane(g, 16) + __builtin_amdgcn_readlane(g, 32) +
           __builtin_amdgcn_readlane(g, 48);
  }
  if (tot != (int)S_BC_PRES(in.bz)) {
#pragma unroll
    for (int q = 0; q < Q; q++) {
      const uint32_t before = (tb4[q >> 2] >> (8 * (q & 3))) & 0xFFu;
      const uint32_t after = (bw[q >> 2] >> (8 * (q & 3))) & 0xFFu;  // 0 = absent
      const uint32_t ev = !before ? (after ? S_EV_ADD : 0u) : (!after ? S_EV_REMOVE : 0u);
      evk |= ev << (2 * q);
    }
    nev = __builtin_popcount((evk | (evk >> 1)) & 0x55555555u);
  } else if (ngone) {  // removals only (the crash case): REMOVE kinds (10) at the removed cells
    uint32_t x = gmask;
    x = (x | (x << 8)) & 0x00FF00FFu;
    x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u;
    x = (x | (x << 1)) & 0x55555555u;
    evk = x << 1;
    nev = ngone;
  }
  // 6. commit: the table and payload stores (the general path's), then this tick's escape list --
  // the entry lanes' survivors first (ballot rank), the lanes' escape bytes after them (esc_emit)
  nxt();  // the next unit's loads: in flight under this unit's stores
  if (selflane) s.hbctr[r] = hbself + 1;
  uint32_t eb_out = unit_stores<B>(s, t, in, bw, ov0, ov1, false, 0u, lds);
  const uint64_t svb = __builtin_amdgcn_ballot_w64(sv);
  const bool emany = __builtin_amdgcn_ballot_w64(em != 0) != 0;
  if (svb || emany) {
    const int ns = __builtin_popcountll(svb);
    int etot = ns, eoff = 0;
    if (emany) {
      eoff = row_scan<64>(__builtin_popcount(em), li, lane, etot);
      etot += ns;
    }
    eb_out = row_alloc<64>(s, par, slab, r, etot, li, lane);
    if (eb_out != 0) {
      const EscList l = esc_list(s, par, slab, r, eb_out);
      if (sv) {
        *l.at(p_lanes_below(svb)) = sent;
        if ((sent >> 16) < (uint32_t)S_CELL(s.lag_hmin, 0)) atomicOr(s.err, GM_ERR_LAG);
      }
      if (emany) esc_emit(lds, lane, l, ns + eoff, em, li * Q, etot <= S_ESC_IN, s.err, s.lag_hmin);
    }
  }
  unit_records<B, false>(s, t, in, true, eb_out, npres, nfail, nev, evk, 0, &rcnt);
  return true;
}

#ifndef GM_DROP_MINW
#define GM_DROP_MINW 8  // the keyed-loss instantiation at 8 waves per SIMD (64 VGPRs + 20 B of spills: 7.39 ms vs 7.63 at its own 79 VGPRs)
#endif
// One unit of the general path (every band width, keyed loss, the join ramp, and the units the
// fast path hands back).
// UNI: the grid's own unit (its row metadata in scalar registers); the listed pass loads its units'
// rows through vector registers.
template <int B, bool DROP, bool UNI>
__device__ __forceinline__ void band_unit(const SState &s, int t, int drop_pct, int band, int ub, uint32_t *lds) {
  UnitIn<B> in;
  unit_load<B, UNI>(s, t, band, ub, in);
  u32x2 m[S_SB];
  uint32_t ent;
  unit_gather<B, DROP>(s, t, in, m, ent);
  unit_finish<B, DROP>(s, t, drop_pct, in, m, ent, lds);
}
// the pools of tick t+1 start empty (the tick t-1 lists in them are read through their bases,
// never through the counters), and so does the fast path's hand-back list of tick t+1 (whichever
// kernel ran tick t: a keyed-loss tick between two fast ticks must not leave a count behind); one
// wave of the tick's first band kernel
__device__ __forceinline__ void band_reset_pools(const SState &s, int t) {
  const int S = s.esc_stripes;
  for (int i = threadIdx.x; i < S; i += 64) {
    s.tesc_cnt[((t & 1) ^ 1) * S + i] = 0;
    s.pesc_cnt[((t & 1) ^ 1) * S + i] = 0;
  }
  if (s.fb_cnt && threadIdx.x == 0) s.fb_cnt[(t & 1) ^ 1] = 0;
}

template <int B, bool DROP>
#ifndef GM_BAND_MINW
#define GM_BAND_MINW 1
#endif
// grid (units of a band / 4, bands): blockIdx.y is the band, so workgroups still dispatch
// band-major, and the wave-uniform unit index needs no division
// units [u0, u1) of every band: a row chunk of the column-sharded pipeline, or all of them
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DROP ? GM_DROP_MINW : GM_BAND_MINW, 8))) void gm_s_band(SState s, int t, int drop_pct, int u0, int u1) {
  constexpr int RPW = 64 / (B / S_COLS_PER_LANE);
  const int ub = __builtin_amdgcn_readfirstlane(u0 + (int)blockIdx.x * 4 + (int)(threadIdx.x >> 6));
  if (ub >= u1) return;  // whole wave
  UnitIn<B> in;
  unit_load<B, RPW == 1>(s, t, (int)blockIdx.y, ub, in);
  u32x2 m[S_SB];
  uint32_t ent;
  unit_gather<B, DROP>(s, t, in, m, ent);
  __shared__ uint32_t lds_all[4 * S_LDS_WAVE_WORDS];  // escaped rows only (esc_apply / esc_emit)
  unit_finish<B, DROP>(s, t, drop_pct, in, m, ent, lds_all + (threadIdx.x >> 6) * S_LDS_WAVE_WORDS);
  if (ub == 0 && blockIdx.y == 0) band_reset_pools(s, t);
}

// The general path over the units gm_s_band_fast handed back this tick (s.fb_list): a fixed grid of
// waves striding over the list (rows through vector registers: the units come from memory).
// Only the units of rows [u0, u1) (one row per unit at B = 1024): the pipelined sharded tick runs it
// after each row chunk's fast pass, over the list so far.
template <int B>
__global__ __launch_bounds__(256) void gm_s_band_listed(SState s, int t, int u0, int u1) {
  __shared__ uint32_t lds_all[4 * S_LDS_WAVE_WORDS];
  uint32_t *lds = lds_all + (threadIdx.x >> 6) * S_LDS_WAVE_WORDS;
  const uint32_t cnt = s.fb_cnt[t & 1];
  const uint32_t nw = gridDim.x * 4;
  for (uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6); i < cnt; i += nw) {
    const int2 u = s.fb_list[i];
    const int ub = __builtin_amdgcn_readfirstlane(u.y);
    if (ub < u0 || ub >= u1) continue;
    band_unit<B, false, false>(s, t, -1, __builtin_amdgcn_readfirstlane(u.x), ub, lds);
  }
}

// The fast path's kernel (B = 1024, no keyed loss, no join ramp): every unit takes unit_fast; a
// unit it hands back (not merged, a delivered escape nibble, a payload for the wide plane) goes to
// s.fb_list for gm_s_band's listed pass right after, untouched. The list of tick t+1 starts empty.
// CH: a row chunk [u0, u1) of the pipelined column-shard tick; otherwise every row (no unit bounds
// among the kernel arguments: the wave's first loads issue as in round 4's codegen)
// Held to 7 waves per SIMD (72 VGPRs; the crash-window quick path alone would take 75, occupancy 6).
// BPW: bands per wave (blockIdx.y = a group of BPW bands). With 2, the wave's second unit is the same
// row in the next band: it shares the row's metadata (one round trip, not two), and its table slice
// and payload gathers issue as soon as the first unit's payload words are merged (nxt), so they are
// in flight under the first unit's sweep and stores -- one dependent round trip per unit instead of
// two (inbox, then gathers).
#ifndef GM_FAST_WG
#define GM_FAST_WG 1  // waves per workgroup of gm_s_band_fast (1: a finished wave frees its LDS slice at once;
                      // 4: 3.29 ms per S-A tick, 1: 3.22, profiles/r06/ab_fwg/)
#endif
template <int B, bool CH, int BPW>
#ifndef GM_FAST_MINW
#define GM_FAST_MINW 7  // gm_s_band_fast's waves per SIMD (72 VGPRs at 7)
#endif
__global__ __launch_bounds__(64 * GM_FAST_WG) __attribute__((amdgpu_waves_per_eu(GM_FAST_MINW, 8))) void gm_s_band_fast(SState s, int t, int u0, int u1) {
  if (!CH) {
    u0 = 0;
    u1 = s.n;
  }
  const int wv = GM_FAST_WG == 1 ? 0 : (int)(threadIdx.x >> 6);
  const int ub = __builtin_amdgcn_readfirstlane(u0 + (int)blockIdx.x * GM_FAST_WG + wv);
  if (ub >= u1) return;  // whole wave (one row per wave)
  // per wave: escape cells by column, the park, the per-lane words of the escaped cells' outcomes
  constexpr int W = 2 * S_LDS_WAVE_WORDS + 192;
  __shared__ uint32_t lds_all[GM_FAST_WG * W];
  uint32_t *lds = lds_all + wv * W;
  const int b0 = (int)blockIdx.y * BPW;
  const bool two = BPW == 2 && b0 + 1 < s.nb;  // wave-uniform
  UnitIn<B> in, in2;
  unit_load<B, true, true, BPW == 2>(s, t, b0, ub, in, in2, two ? b0 + 1 : b0);
  u32x2 m[S_SB];
  uint32_t ent, ent2 = 0;
  unit_gather<B, false>(s, t, in, m, ent);
  bool issued = false;  // wave-uniform
  const bool ok = unit_fast<B>(s, t, in, m, ent, lds, lds + S_LDS_WAVE_WORDS, [&]() {
    if (two) {
      unit_table<B>(s, in2);
      unit_gather<B, false>(s, t, in2, m, ent2);
    }
    issued = true;
  });
  if (!ok && (threadIdx.x & 63) == 0) {
    const uint32_t slot = atomicAdd(&s.fb_cnt[t & 1], 1u);  // < the units of a tick: the list's size
    s.fb_list[slot] = make_int2(b0, ub);
  }
  if (two) {
    if (!issued) {  // the first unit went to the general path before its payload words were consumed
      unit_table<B>(s, in2);
      unit_gather<B, false>(s, t, in2, m, ent2);
    }
    lds_wave_sync();  // the first unit's LDS reads are done before the second one's writes
    if (!unit_fast<B>(s, t, in2, m, ent2, lds, lds + S_LDS_WAVE_WORDS, []() {}) && (threadIdx.x & 63) == 0) {
      const uint32_t slot = atomicAdd(&s.fb_cnt[t & 1], 1u);
      s.fb_list[slot] = make_int2(b0 + 1, ub);
    }
  }
  if (ub == 0 && blockIdx.y == 0) band_reset_pools(s, t);
}

// --------------------------------------------------------------- gm_s_selfcheck
// Join ramp: rows that appended their own entry this tick (updateMyPos found no self and no
// larger id of its start group). The reference appends only if NO larger id is present
// after the merge (lower_bound == end); a larger id of a later group would have taken the
// quirk path with a heartbeat the narrow cell cannot hold. Verify, one wave per row: no
// cell above the group is present after the sweep, none was removed by it (events).
__global__ __launch_bounds__(256) void gm_s_selfcheck(SState s) {
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * 4;
  const uint32_t cnt = min(*s.selfadd_cnt, (uint32_t)S_SELFADD_CAP);
  for (uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6); i < cnt; i += nw) {
    const int r = s.selfadd[i];
    const int gend = (r | 3) - s.c0;  // last shard column of the row's start group
    const int b0 = (gend + 1) / s.band;
    bool bad = false;
    for (int b = b0 + 1 + lane; b < s.nb; b += 64) {  // whole bands above: nothing present, no events
      const uint32_t v = s.brec[(size_t)b * s.n + r].z;
      bad |= S_BC_PRES(v) != 0 || S_BC_NEV(v) != 0;
    }
    if (b0 < s.nb) {
      const uint8_t *cells = s.table + ((size_t)b0 * s.n + r) * s.band;
      for (int j = lane; j < s.band; j += 64)
        bad |= b0 * s.band + j > gend && cells[j] != 0;
      const uint32_t v = s.brec[(size_t)b0 * s.n + r].z;
      const int ne = min((int)S_BC_NEV(v), s.evs);
      const uint32_t *ev = s.ev_band + ((size_t)r * s.nb + b0) * s.evs;
      for (int q = lane; q < ne; q += 64) bad |= (int)(ev[q] & 0x3FFFFFFFu) - 1 - s.c0 > gend;
      if ((int)S_BC_NEV(v) > s.evs) {  // spilled records of this (row, band)
        const uint32_t ns = min(*s.ev_spill_cnt, s.ev_spill_cap);
        for (uint32_t q = lane; q < ns; q += 64) {
          const uint64_t e = s.ev_spill[q];
          bad |= (int)(e >> 32) == r && (int)((uint32_t)e & 0x3FFFFFFFu) - 1 - s.c0 > gend;
        }
      }
    }
    if (__ballot(bad) && lane == 0) atomicOr(s.err, GM_ERR_SELF);
  }
}

// ------------------------------------------------------- wave-per-row helpers
// LDS per wave of the draw kernels: chunk prefix [chunks + 1] u32 (S_CHUNK(B) columns per
// chunk), the fallback generator's state [624] u32.
__host__ __device__ __forceinline__ int gm_draw_chunks(int wp, int band) { return wp / S_CHUNK(band); }  // rank-select chunks per row
__host__ __device__ __forceinline__ size_t gm_draw_lds_words(int wp, int band) {
  return (size_t)gm_draw_chunks(wp, band) + 1 + 624;
}

// Row r of this shard: numfailed (band counts), size and the chunk prefix
// pre[c] = present cells in chunks [0, c) (pre[nc] = size), from the chunk counts.
// the lane's first (band, row) record of row r (all of them when nb <= 64), as gm_row_totals reads it
__device__ __forceinline__ uint4 gm_row_rec0(const SState &s, int r, int lane) {
  const int perb = (s.nb + 63) >> 6, b0 = lane * perb;
  return b0 < s.nb ? s.brec[(size_t)b0 * s.n + r] : make_uint4(0u, 0u, 0u, 0u);
}

// pre0: the lane's first record, when the caller loaded it already (gm_row_rec0)
template <int B>
__device__ __forceinline__ void gm_row_totals(const SState &s, int r, int lane, uint32_t *pre, uint32_t &size,
                                              uint32_t &nfail, const uint4 *pre0 = nullptr) {
  constexpr int CPB = B / S_CHUNK(B);  // rank-select chunks per band
  const int nb = s.nb, perb = (nb + 63) >> 6;
  const int b0 = min(nb, lane * perb), b1 = min(nb, b0 + perb);
  uint32_t fs = 0, ps = 0;
  uint4 rec0 = make_uint4(0u, 0u, 0u, 0u);  // the lane's first (band, row) record (all of them when nb <= 64)
  for (int b = b0; b < b1; b++) {
    const uint4 rc = (b == b0 && pre0) ? *pre0 : s.brec[(size_t)b * s.n + r];
    if (b == b0) rec0 = rc;
    fs += S_BC_FAIL(rc.z);
    ps += S_BC_PRES(rc.z);
  }
  // wave sums / prefix on DPP (no LDS round trips): inclusive scans, totals from lane 63
  nfail = (uint32_t)__builtin_amdgcn_readlane(dpp_scan((int)fs), 63);
  const uint32_t x = (uint32_t)dpp_scan((int)ps);
  size = (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
  if (pre) {
    uint32_t a = x - ps;
    for (int b = b0; b < b1; b++) {
      const uint2 pc = b == b0 ? make_uint2(rec0.x, rec0.y) : *(const uint2 *)&s.brec[(size_t)b * s.n + r];
      const uint64_t v = (uint64_t)pc.x | ((uint64_t)pc.y << 32);
#pragma unroll
      for (int c = 0; c < CPB; c++) {
        pre[b * CPB + c] = a;
        a += (uint32_t)(v >> (8 * c)) & 0xFFu;
      }
    }
    if (lane == 63) pre[nb * CPB] = a;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// Freshness (age < TFAIL) of the escaped cell (r, col) of tick t, from its (band, row) list of
// tick t (rare: a draw landing on an escaped cell)
__device__ __forceinline__ bool esc_fresh(const SState &s, int r, int col) {
  const int b = col / s.band, c = col % s.band;
  const size_t slab = (size_t)b * s.n;
  const uint32_t w = s.brec[slab + r].w;
  // the pools of the tick just swept: its parity is that of the row's last written tick
  const EscList l = esc_list(s, s.wtick[r] & 1, slab, r, w);
  for (int i = 0; i < (int)S_EW_TOT(w); i++) {
    const uint32_t e = *l.at(i);
    if ((e & 0xFFFFu) == (uint32_t)c) return S_AGE(e >> 16) < GM_TFAIL;
  }
  return false;
}

// Resolve up to 8 draws at once, one per 8-lane group: group g holds shard-local rank
// ix_g (valid iff act) of a present entry of row r. The chunk-word prefix finds the
// 64- or 128-column chunk; its cell bytes (8 or 16 per lane) give the column. Returns, to
// every lane, the shard-local column of each draw (-1 if none) and whether it is fresh.
template <int B>
__device__ __forceinline__ void gm_resolve8(const SState &s, int r, const uint32_t *pre, bool act, uint32_t ix, int lane,
                                            int col[8], int fresh[8]) {
  constexpr int CH = S_CHUNK(B), CPL = CH / 8;  // chunk columns, cells per lane of the 8-lane group
  const int gl = lane & 7;
  int cnt = 0, base = 0;
  uint32_t en[CPL];
#pragma unroll
  for (int v = 0; v < CPL; v++) en[v] = 0;
  uint32_t q = 0;
  if (act) {
    int lo = 0, hi = s.wp / CH - 1;  // largest chunk with pre[c] <= ix (a non-empty one)
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (pre[mid] <= ix) lo = mid;
      else hi = mid - 1;
    }
    q = ix - pre[lo];
    const int col0 = lo * CH + gl * CPL;  // this lane's cells
    base = col0;
    const uint8_t *cp = s.table + ((size_t)(col0 / B) * s.n + r) * B + (col0 % B);
#pragma unroll
    for (int h = 0; h < CPL / 8; h++) {
      const uint2 t2 = *(const uint2 *)(cp + 8 * h);
#pragma unroll
      for (int v = 0; v < 8; v++) en[8 * h + v] = ((v < 4 ? t2.x : t2.y) >> (8 * (v & 3))) & 0xFFu;
    }
#pragma unroll
    for (int v = 0; v < CPL; v++) cnt += en[v] != 0;
  }
  int x = cnt;
#pragma unroll
  for (int o = 1; o < 8; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (gl >= o) x += y;
  }
  const int excl = x - cnt;
  int mycol = -1, myfresh = 0;
  bool holder = false;
  if (act && (int)q >= excl && (int)q < excl + cnt) {
    holder = true;
    int need = (int)q - excl;
#pragma unroll
    for (int v = 0; v < CPL; v++) {
      if (en[v] != 0) {
        if (need == 0) {
          mycol = base + v;
          // the table is as of tick t; an escaped cell's age is in its (band, row) escape list
          myfresh = s_is_esc(en[v]) ? esc_fresh(s, r, mycol) : S_AGE(s_widen(en[v])) < GM_TFAIL;
        }
        need--;
      }
    }
  }
  const uint64_t hm = __ballot(holder);
#pragma unroll
  for (int g = 0; g < 8; g++) {
    const uint32_t seg = (uint32_t)(hm >> (8 * g)) & 0xFFu;
    const int src = seg ? 8 * g + __builtin_ctz(seg) : 0;
    col[g] = seg ? __shfl(mycol, src, 64) : -1;
    fresh[g] = seg ? __shfl(myfresh, src, 64) : 0;
  }
}

// S2 outputs of a row beyond the precomputed ones: lane 0 runs the lazy generator
// (state in this wave's LDS), `skip` outputs consumed already; lane q < cnt gets output q.
__device__ __forceinline__ uint32_t gm_mt_batch(GmLazyMT &mt, uint32_t *mts, uint32_t seed, bool fresh_gen, int skip,
                                                int cnt, int lane) {
  if (lane == 0 && fresh_gen) {
    mt.seed(mts, seed);
    for (int i = 0; i < skip; i++) (void)mt.next();
  }
  uint32_t raw = 0;
  for (int q = 0; q < cnt; q++) {
    uint32_t o = 0;
    if (lane == 0) o = mt.next();
    o = __shfl(o, 0, 64);
    if (lane == q) raw = o;
  }
  return raw;
}

// ------------------------------------------------------------------- gm_s_pick
// Single-context tick, phase 2: one wave per observer row.
template <int B>
__device__ __forceinline__ void pick_row(const SState &s, int t, int r, int wave, int lane);
template <int B>
// 6 waves per SIMD (80 VGPRs, no spills) rather than the compiler's 5 (89): the kernel waits on
// dependent loads, 141 -> 125 us per S-A tick (profiles/r04/pick_occupancy/)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6, 8))) void gm_s_pick(SState s, int t, int listed) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (!listed) {
    const int r = blockIdx.x * 4 + wave;
    if (r < s.n) pick_row<B>(s, t, r, wave, lane);  // whole wave; no workgroup barrier follows
    return;
  }
  // listed: the rows gm_s_pick0 left (its list, any order: each row's draw is its own), grid-stride
  const int cnt = (int)*s.pk_cnt;
  for (int i = blockIdx.x * 4 + wave; i < cnt; i += gridDim.x * 4) pick_row<B>(s, t, s.pk_list[i], wave, lane);
}
template <int B>
__device__ __forceinline__ void pick_row(const SState &s, int t, int r, int wave, int lane) {
  extern __shared__ __align__(16) uint32_t p_smem[];
  uint32_t *pre = p_smem + wave * gm_draw_lds_words(s.wp, B);
  uint32_t *mts = pre + gm_draw_chunks(s.wp, B) + 1;
  const int par = t & 1;
  int32_t *stat = s.rowstat + (size_t)r * 4;
  const int k = s.inbox_cnt[par][r];
  if (lane == 0) s.inbox_cnt[par][r] = 0;  // consumed by gm_s_band; the append target of tick t+2
  if (s.failed[r] || !s_ingroup(s.ramp, s.intro_until, r, t)) {
    if (lane == 0) stat[0] = stat[1] = stat[2] = stat[3] = 0;
    return;
  }
  uint32_t size, numfailed;
  gm_row_totals<B>(s, r, lane, pre, size, numfailed);
  const int me = s.ramp ? s.mecol[r] : r;
  const int numpot = (int)size - 1 - (int)numfailed;  // numfailed counts removed entries too (MP1Node.cpp:463)
  const int target = min(GM_FANOUT, numpot);
  int n = 0, g0 = -1, g1 = -1, g2 = -1, g3 = -1, g4 = -1;
  if (s.ramp && r == 0) {  // gossipnodes = newNodes first (MP1Node.cpp:458): this tick's joiners, ascending id
    for (int c = max(1, 4 * (t - 1)); c < min(s.n, 4 * t); c++) {
      if (n == 0) g0 = c;
      else if (n == 1) g1 = c;
      else if (n == 2) g2 = c;
      else g3 = c;
      n++;
    }
  }
  if (numpot > 0 && n < target) {
    const uint32_t thr = (0u - size) % size;  // Lemire rejection threshold (uniform_int_dist.h)
    GmLazyMT mt;
    bool done = false;
    for (int batch = 0; !done; batch++) {
      if (batch > (1 << 18)) {
        if (lane == 0) atomicOr(s.err, GM_ERR_DRAWS);
        break;
      }
      uint32_t raw = 0;
      if (batch == 0) {
        if (lane < S_MT_RAW) raw = s.mtraw[(size_t)r * S_MT_RAW + lane];
      } else {
        raw = gm_mt_batch(mt, mts, gm_rd_seed(s.rd_seed, t, r + 1), batch == 1, S_MT_RAW, S_MT_RAW, lane);
      }
      const uint64_t prod = (uint64_t)raw * size;
      const bool ok = lane < S_MT_RAW && (uint32_t)prod >= thr;
      const uint32_t ix = (uint32_t)(prod >> 32);
      uint64_t m = __ballot(ok);
      while (m && !done) {
        // the next (up to) 8 draws, in order: group g of 8 lanes takes the g-th
        const int grp = lane >> 3;
        uint64_t mm = m;
        int myd = 0, cnt = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
          if (mm) {
            if (grp == i) myd = __builtin_ctzll(mm);
            mm &= mm - 1;
            cnt++;
          }
        }
        m = mm;
        const uint32_t myix = __shfl(ix, myd, 64);
        int col[8], fr[8];
        gm_resolve8<B>(s, r, pre, grp < cnt, myix, lane, col, fr);
#pragma unroll
        for (int i = 0; i < 8; i++) {
          if (i >= cnt || done) continue;
          if (col[i] < 0) {  // a draw no chunk resolved: counts and cells disagree
            if (lane == 0) atomicOr(s.err, GM_ERR_DRAWS);
            done = true;
            continue;
          }
          const int c = s.c0 + col[i];
          if (c == me) continue;  // "me" = myPos's id (MP1Node.cpp:459-460,470)
          if (!fr[i]) continue;  // age >= TFAIL (MP1Node.cpp:471)
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
  }
  if (lane < n) {  // delivery: one target per lane, the n appends in flight together (the targets
                   // are wave-uniform; an inbox's order is free: the merge is a max)
    const int dst = lane == 0 ? g0 : lane == 1 ? g1 : lane == 2 ? g2 : lane == 3 ? g3 : g4;
    s.targets[(size_t)r * GM_FANOUT + lane] = dst;
    const int slot = atomicAdd(&s.inbox_cnt[par ^ 1][dst], 1);
    if (slot < s.kcap) s.inbox[par ^ 1][(size_t)dst * S_KMAX + slot] = r;
    else atomicOr(s.err, GM_ERR_INBOX);
  }
  if (lane == 0) {
    stat[0] = k;
    stat[1] = (int)size;
    stat[2] = (int)numfailed;
    stat[3] = n;
  }
}

__device__ __forceinline__ int row16_scan(int v) {  // inclusive scan within each 16-lane DPP row
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);  // row_shr:8
  return v;
}
// rows in pending list l this tick: its append count, or 0 when the appends overflowed its
// capacity (gm_s_plist_sort: such a list is void on every rank)
// gm_shard_stub (diagnostics): a draw landing in a peer's columns resolves to a fresh target spread
// evenly over the whole cluster -- rank ix of the row's `size` present entries stands for column
// ix * n / size. (Round 5 took column ix % n: the top ~1 % of the rows never received a list, their
// cells aged into escapes and removals, and the shard's band kernels grew ~25 % slower tick by tick.)
__device__ __forceinline__ int32_t stub_target(uint32_t ix, uint32_t size, int n) {
  return (int32_t)(((uint64_t)ix * (uint32_t)n / max(size, 1u)) << 1) | 1;
}
__device__ __forceinline__ int plist_len(const SState &s, int l) {
  const uint32_t c = *s.plist_cnt[l];
  return c > (uint32_t)s.plist_cap[l] ? 0 : (int)c;
}
__device__ __forceinline__ int row16_bcast(int v, int g, int q) { return __shfl(v, 16 * g + q, 64); }
__device__ __forceinline__ uint32_t row16_bits(uint64_t bal, int g) { return (uint32_t)(bal >> (16 * g)) & 0xFFFFu; }

// Single-context tick, phase 2, four rows per wave (16 lanes per row), B = 1024, no join ramp: the
// draw of MP1Node.cpp:449-489 over the row's first 16 S2 outputs (lane q: output q), each ok draw
// resolved in draw order by a 16-ary search of a band prefix in LDS, the band record's 8 chunk
// counts and one 128-cell chunk read by the row's 16 lanes, and accepted unless it is "me", stale or
// a repeat. Rows the 16 outputs do not finish go to s.pk_list for gm_s_pick (from output 0). Same
// results as gm_s_pick at a fraction of its instructions.
template <int B>
#ifndef GM_PICK_WG
#define GM_PICK_WG 4  // waves per workgroup of gm_s_pick0 (four rows per wave)
#endif
__global__ __launch_bounds__(64 * GM_PICK_WG) void gm_s_pick0(SState s, int t) {
  static_assert(B == 1024, "8 rank-select chunks of 128 columns per band");
  extern __shared__ __align__(16) uint32_t p_smem[];
  const int lane = threadIdx.x & 63, g = lane >> 4, q = lane & 15;
  const int slot = (int)(threadIdx.x >> 4);  // row slot of the workgroup (0 .. 4 GM_PICK_WG - 1)
  const int r = (int)blockIdx.x * (4 * GM_PICK_WG) + slot;
  const bool valid = r < s.n;
  const int rc = valid ? r : s.n - 1;
  const int nb = s.nb, perb = (nb + 15) >> 4, par = t & 1;
  uint32_t *bpre = p_smem + (size_t)slot * (nb + 1);
  // the band records' chunk counts in LDS too (read with the prefix's words, same lines): a draw then
  // waits for one load (its table chunk), not two
  uint2 *bcc = (uint2 *)(p_smem + 4 * GM_PICK_WG * (size_t)(nb + 1)) + (size_t)slot * nb;
  const int k = s.inbox_cnt[par][rc], failed = s.failed[rc];
  const uint32_t raw = s.mtraw[(size_t)rc * S_MT_RAW + q];
  uint32_t bp = 0, bf = 0;
  for (int kb = 0; kb < perb; kb++) {
    const int b = q * perb + kb;
    if (b < nb) {
      const uint4 rec = s.brec[(size_t)b * s.n + rc];
      bp += S_BC_PRES(rec.z);
      bf += S_BC_FAIL(rec.z);
      bcc[b] = make_uint2(rec.x, rec.y);
    }
  }
  const int bi = row16_scan((int)bp), fi = row16_scan((int)bf);
  const uint32_t size = (uint32_t)row16_bcast(bi, g, 15);
  const int numfailed = row16_bcast(fi, g, 15);  // counts removed entries too (MP1Node.cpp:463)
  {
    uint32_t a = (uint32_t)bi - bp;
    for (int kb = 0; kb < perb; kb++) {
      const int b = q * perb + kb;
      if (b < nb) {
        bpre[b] = a;
        a += S_BC_PRES(s.brec[(size_t)b * s.n + rc].z);
      }
    }
    if (q == 15) bpre[nb] = (uint32_t)bi;
  }
  const bool live = valid && !failed;
  const int numpot = (int)size - 1 - numfailed;
  const int target = min(GM_FANOUT, numpot);
  const bool pend = live && numpot > 0;
  const uint32_t sz = pend ? size : 1u;
  const uint32_t thr = (0u - sz) % sz;  // Lemire rejection threshold (uniform_int_dist.h)
  const uint64_t prod = (uint64_t)raw * sz;
  const uint32_t ix = (uint32_t)(prod >> 32);
  uint32_t okm = row16_bits(__ballot(pend && (uint32_t)prod >= thr), g);  // the row's draws, in order
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  int n = 0, g0 = -1, g1 = -1, g2 = -1, g3 = -1, g4 = -1;  // row-uniform (every lane of the row)
  bool done = !pend;
  while (__ballot(!done && okm != 0)) {
    const bool act = !done && okm != 0;
    const int d = act ? __builtin_ctz(okm) : 0;
    okm &= okm - 1;
    const uint32_t x = (uint32_t)row16_bcast((int)ix, g, d);
    int lo = 0, span = nb;
    while (__ballot(act && span > 1)) {  // 16-ary search: the band b with bpre[b] <= x < bpre[b + 1]
      const int step = (span + 15) >> 4;
      const bool le = act && q * step < span && bpre[lo + q * step] <= x;
      const int c = __builtin_popcount(row16_bits(__ballot(le), g));
      if (act && span > 1) {
        lo += (max(c, 1) - 1) * step;
        span = min(step, span - (max(c, 1) - 1) * step);
      }
    }
    const int band = lo;
    uint32_t rem = act ? x - bpre[band] : 0u;
    const uint2 rcc = act ? bcc[band] : make_uint2(0u, 0u);
    const uint64_t cc = (uint64_t)rcc.x | ((uint64_t)rcc.y << 32);
    int ch = 0;
#pragma unroll
    for (int kc = 0; kc < 7; kc++) {
      const uint32_t c8 = (uint32_t)(cc >> (8 * ch)) & 0xFFu;
      if (rem >= c8 && ch == kc) {
        rem -= c8;
        ch++;
      }
    }
    uint2 w = make_uint2(0u, 0u);
    if (act) w = *(const uint2 *)(s.table + ((size_t)band * s.n + rc) * B + ch * 128 + q * 8);
    auto nzb = [](uint32_t v) { return (v | (v >> 1) | (v >> 2) | (v >> 3) | (v >> 4) | (v >> 5) | (v >> 6) | (v >> 7)) & 0x01010101u; };
    const int cnt = __builtin_popcount(nzb(w.x)) + __builtin_popcount(nzb(w.y));
    const int incl = row16_scan(cnt);
    const int excl = incl - cnt;
    const bool holder = act && (int)rem >= excl && (int)rem < incl;
    int col = -1, fr = 0;
    if (holder) {  // the (rem - excl)-th present cell of the lane's 8
      int need = (int)rem - excl, pos = 0;
      uint32_t byte = 0;
#pragma unroll
      for (int v = 0; v < 8; v++) {
        const uint32_t bv = ((v < 4 ? w.x : w.y) >> (8 * (v & 3))) & 0xFFu;
        if (bv != 0) {
          if (need == 0) { pos = v; byte = bv; }
          need--;
        }
      }
      col = band * B + ch * 128 + q * 8 + pos;
      fr = s_is_esc(byte) ? esc_fresh(s, rc, col) : S_AGE(s_widen(byte)) < GM_TFAIL;
    }
    const uint32_t hm = row16_bits(__ballot(holder), g);
    const int src = hm ? __builtin_ctz(hm) : 0;
    const int c = row16_bcast(col, g, src);
    const int f = row16_bcast(fr, g, src);
    if (act) {
      if (!hm) {  // a draw no chunk resolved: counts and cells disagree
        if (q == 0) atomicOr(s.err, GM_ERR_DRAWS);
        done = true;
      } else if (c != r && f && !((n > 0 && g0 == c) || (n > 1 && g1 == c) || (n > 2 && g2 == c) || (n > 3 && g3 == c))) {
        if (n == 0) g0 = c;  // "me" (MP1Node.cpp:459-460,470), age >= TFAIL (:471), repeats skipped
        else if (n == 1) g1 = c;
        else if (n == 2) g2 = c;
        else if (n == 3) g3 = c;
        else g4 = c;
        n++;
        if (n >= target) done = true;
      }
    }
  }
  if (!valid) return;
  int32_t *stat = s.rowstat + (size_t)r * 4;
  if (!live) {
    if (q == 0) {
      s.inbox_cnt[par][r] = 0;
      stat[0] = stat[1] = stat[2] = stat[3] = 0;
    }
    return;
  }
  if (pend && n < target) {  // more than 16 outputs needed: gm_s_pick takes the row (it resets the inbox count)
    if (q == 0) s.pk_list[atomicAdd(s.pk_cnt, 1u)] = r;
    return;
  }
  if (q == 0) s.inbox_cnt[par][r] = 0;  // consumed by gm_s_band; the append target of tick t+2
  if (q < n) {  // delivery: one target per lane (an inbox's order is free: the merge is a max)
    const int dst = q == 0 ? g0 : q == 1 ? g1 : q == 2 ? g2 : q == 3 ? g3 : g4;
    s.targets[(size_t)r * GM_FANOUT + q] = dst;
    const int sl = atomicAdd(&s.inbox_cnt[par ^ 1][dst], 1);
    if (sl < s.kcap) s.inbox[par ^ 1][(size_t)dst * S_KMAX + sl] = r;
    else atomicOr(s.err, GM_ERR_INBOX);
  }
  if (q == 0) {
    stat[0] = k;
    stat[1] = (int)size;
    stat[2] = numfailed;
    stat[3] = n;
  }
}

// ------------------------------------------------------------ gm_s_msgcount
// msgcount analogue of tick t (gm_msgcount_record), in two phases:
//   gm_s_mcfresh (after gm_s_band, wave per row): fresh = the row's non-zero payload nibbles of
//     this tick in this context's columns (the entries it sends, MP1Node.cpp:372-375);
//     column shards SUM-allreduce it (and the DROP band kernel's per-row kept counts), so
//     every rank holds the whole row's counts;
//   gm_s_mcount (after the targets are final, thread per row): sent = fresh x targets;
//     received = the entries of the delivered lists -- the senders' fresh counts of tick t-1,
//     or on loss ticks the kept entries counted by the DROP band kernel.
__device__ __forceinline__ uint32_t nz_nibbles(uint32_t x) {
  return (uint32_t)__builtin_popcount((x | (x >> 1) | (x >> 2) | (x >> 3)) & 0x11111111u);
}
template <int B>
__global__ __launch_bounds__(256) void gm_s_mcfresh(SState s, int t) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= s.n) return;  // whole wave
  const int par = t & 1, half = B / 2, tot = s.nb * half;
  uint32_t f = 0;
  for (int off = lane * 16; off < tot; off += 64 * 16) {  // 16-byte pieces never straddle a band
    const int b = off / half, o = off % half;
    const uint4 v = *(const uint4 *)(s.msg + ((size_t)b * s.n + r) * B + par * half + o);
    f += nz_nibbles(v.x) + nz_nibbles(v.y) + nz_nibbles(v.z) + nz_nibbles(v.w);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) f += __shfl_xor(f, o, 64);
  if (lane == 0) s.mc_fresh[(size_t)par * s.n + r] = f;
}

__global__ __launch_bounds__(256) void gm_s_mcount(SState s, int t, int dropped) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= s.n) return;
  const int par = t & 1;
  const int32_t *stat = s.rowstat + (size_t)r * 4;
  uint32_t recv = 0;
  if (dropped) {
    recv = s.mc_rdrop[r];
    s.mc_rdrop[r] = 0;
  } else {
    const int k = min(stat[0], S_KMAX);  // 0 for rows not merged this tick
    for (int q = 0; q < k; q++) recv += s.mc_fresh[(size_t)(par ^ 1) * s.n + s.inbox[par][(size_t)r * S_KMAX + q]];
  }
  s.mc_sent[(size_t)t * s.n + r] = (uint32_t)stat[3] * s.mc_fresh[(size_t)par * s.n + r];
  s.mc_recv[(size_t)t * s.n + r] = recv;
}

// phase 0: fresh counts (gm_s_mcfresh); phase 1: sent / received (gm_s_mcount)
hipError_t gm_launch_msgcount(const SState &s, int t, bool dropped, int phase, hipStream_t st) {
  if (phase == 1) {
    hipLaunchKernelGGL(gm_s_mcount, dim3((s.n + 255) / 256), dim3(256), 0, st, s, t, dropped ? 1 : 0);
    return hipGetLastError();
  }
  const dim3 g((s.n + 3) / 4), b(256);
  switch (s.band) {
    case 64: hipLaunchKernelGGL(gm_s_mcfresh<64>, g, b, 0, st, s, t); break;
    case 128: hipLaunchKernelGGL(gm_s_mcfresh<128>, g, b, 0, st, s, t); break;
    case 256: hipLaunchKernelGGL(gm_s_mcfresh<256>, g, b, 0, st, s, t); break;
    case 512: hipLaunchKernelGGL(gm_s_mcfresh<512>, g, b, 0, st, s, t); break;
    case 1024: hipLaunchKernelGGL(gm_s_mcfresh<1024>, g, b, 0, st, s, t); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ---------------------------------------------------------- column-sharded mode
// Phase A (gm_s_band, sharded): merge / sweep of this shard's columns; each row's
// shard totals (present, numfailed) accumulate into xcnt[rank] for the all-gather.

// Phase A': this shard's per-row totals (present, numfailed) for the all-gather, summed over the
// row's band records (thread per row of [r0, r1): a wave reads 1 KB per band, coalesced) -- not a
// device-scope atomic per (row, band) inside the band kernel. The ramp's self-append flag, set by
// the band kernel, is kept.
__global__ __launch_bounds__(256) void gm_s_xrows(SState s, int r0, int r1) {
  const int r = r0 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (r >= r1) return;
  uint32_t p = 0, f = 0;
  for (int b = 0; b < s.nb; b++) {
    const uint32_t z = s.brec[(size_t)b * s.n + r].z;
    p += S_BC_PRES(z);
    f += S_BC_FAIL(z);
  }
  int32_t *x = s.xcnt + S_XC(s, s.shard_rank, r);
  // the join ramp's self-append flag (set by the band kernel, in a slot zeroed before it) is kept;
  // without the ramp the slot is written whole, so the tick needs no fill of xcnt
  x[0] = (s.ramp ? (int32_t)((uint32_t)x[0] & S_XC_SELFAPP) : 0) | (int32_t)p;
  x[1] = (int32_t)f;
}

hipError_t gm_launch_xrows(const SState &s, int r0, int r1, hipStream_t st) {
  if (r1 > r0) hipLaunchKernelGGL(gm_s_xrows, dim3((r1 - r0 + 255) / 256), dim3(256), 0, st, s, r0, r1);
  return hipGetLastError();
}

// Phase B, round 0, four rows per wave (16 lanes per row: lane q of a row holds S2 output q, the
// counts of rank q, this shard's bands [q * perb, +perb)). Same results as gm_s_draw's round 0 with
// a fraction of its instructions: per row the 16 Lemire draws, the rank range of this shard's
// entries, a band prefix in LDS, and for each draw landing in this shard's columns a 16-ary search
// of the bands, the band record's 8 chunk counts and one 128-cell chunk read by the row's 16 lanes
// (8 bytes each, SWAR counts, a DPP prefix). Not for the join ramp (gm_s_draw handles it); needs
// G <= 16 ranks and B = 1024 (8 rank-select chunks per band).
template <int B>
__global__ __launch_bounds__(256) void gm_s_draw0(SState s, int t, int r0, int r1) {
  static_assert(B == 1024, "8 rank-select chunks of 128 columns per band");
  extern __shared__ __align__(16) uint32_t p_smem[];
  const int lane = threadIdx.x & 63, g = lane >> 4, q = lane & 15;
  const int slot = (int)(threadIdx.x >> 4);  // row slot of the workgroup (0..15)
  const int r = r0 + (int)blockIdx.x * 16 + slot;
  const bool valid = r < r1;
  const int rc = valid ? r : r1 - 1;
  const int G = s.shard_count, nb = s.nb, perb = (nb + 15) >> 4, par = t & 1;
  uint32_t *bpre = p_smem + (size_t)slot * (nb + 1);  // band prefix of this shard's present cells
  // every load of the row at once
  const int failed = s.failed[rc], kin = s.inbox_cnt[par][rc];
  const uint32_t raw = s.mtraw[(size_t)rc * S_MT_RAW + q];
  const int xp = q < G ? s.xcnt[S_XC(s, q, rc)] & S_XC_COUNT : 0;
  const int xf = q < G ? s.xcnt[S_XC(s, q, rc) + 1] : 0;
  uint32_t bsum = 0;
  for (int k = 0; k < perb; k++) {
    const int b = q * perb + k;
    if (b < nb) bsum += S_BC_PRES(s.brec[(size_t)b * s.n + rc].z);
  }
  // row sums over the 16 lanes: size, numfailed, this shard's rank range [own_lo, own_lo + own_cnt)
  const int xpi = row16_scan(xp), xfi = row16_scan(xf), bi = row16_scan((int)bsum);
  const uint32_t size = (uint32_t)row16_bcast(xpi, g, 15);
  const int nf = row16_bcast(xfi, g, 15);
  const uint32_t own_lo = s.shard_rank > 0 ? (uint32_t)row16_bcast(xpi, g, s.shard_rank - 1) : 0u;
  const uint32_t own_cnt = (uint32_t)row16_bcast(xp, g, s.shard_rank);
  const int numpot = (int)size - 1 - nf;
  const bool live = valid && !failed;
  const bool pend = live && numpot > 0;
  if (valid && q == 0) {
    int32_t *acc = s.acc + (size_t)r * 8;
    acc[0] = 0;
    acc[6] = numpot;
    acc[7] = (int)size;
    s.pending[r] = pend;
    int32_t *stat = s.rowstat + (size_t)r * 4;
    stat[0] = live ? kin : 0;  // lists delivered this tick; consumed by gm_s_band, the append target of tick t+2
    stat[1] = live ? (int)size : 0;
    stat[2] = live ? nf : 0;
    stat[3] = 0;
    s.inbox_cnt[par][r] = 0;
  }
  // band prefix (exclusive) of this shard's row, in LDS
  {
    uint32_t a = (uint32_t)bi - bsum;
    for (int k = 0; k < perb; k++) {
      const int b = q * perb + k;
      if (b < nb) {
        bpre[b] = a;
        a += S_BC_PRES(s.brec[(size_t)b * s.n + rc].z);
      }
    }
    if (q == 15) bpre[nb] = (uint32_t)bi;
  }
  // Lemire on output q (uniform_int_distribution, MP1Node.cpp:466): rejection threshold 2^32 mod size
  const uint32_t sz = pend ? size : 1u;
  const uint32_t thr = (0u - sz) % sz;
  const uint64_t prod = (uint64_t)raw * sz;
  const bool ok = pend && (uint32_t)prod >= thr;
  const uint32_t ix = (uint32_t)(prod >> 32);
  const bool mine = ok && ix >= own_lo && ix < own_lo + own_cnt;
  int32_t *st = s.status + (size_t)rc * S_MT_RAW;  // round 0: D = the 16 precomputed outputs
  if (pend && !mine) st[q] = ok ? (s.stub ? stub_target(ix, size, s.n) : -1) : -2;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  uint32_t mm = row16_bits(__ballot(mine), g);  // this row's draws to resolve here
  const uint64_t any = __ballot(mm != 0);
  if (!any) return;
  const int me = r;
  int32_t myst = -1;  // status of this lane's draw (output q), when it lands in this shard's columns
  // up to DB of the row's draws per pass (a row has ~16/G in this shard's columns): their band
  // searches, then their band records' loads, then their chunk loads, each batch in flight together
  constexpr int DB = 4;
  while (__ballot(mm != 0)) {
    bool act[DB];
    int dj[DB], band[DB];
    uint32_t rem[DB];
#pragma unroll
    for (int j = 0; j < DB; j++) {
      act[j] = mm != 0;
      dj[j] = act[j] ? __builtin_ctz(mm) : 0;
      mm &= mm - 1;
      const uint32_t x = (uint32_t)row16_bcast((int)ix, g, dj[j]) - own_lo;  // rank among this shard's entries
      // 16-ary search: the band b with bpre[b] <= x < bpre[b + 1]
      int lo = 0, span = nb;
      while (__ballot(act[j] && span > 1)) {
        const int step = (span + 15) >> 4;
        const int idx = lo + q * step;
        const bool le = act[j] && q * step < span && bpre[idx] <= x;
        const int c = __builtin_popcount(row16_bits(__ballot(le), g));
        if (act[j] && span > 1) {
          lo += (max(c, 1) - 1) * step;
          span = min(step, span - (max(c, 1) - 1) * step);
        }
      }
      band[j] = lo;
      rem[j] = act[j] ? x - bpre[lo] : 0u;  // rank inside the band
    }
    // the band records' 8 chunk counts, then the chunks (128 cells: 8 bytes per lane of the row)
    uint4 rec[DB];
#pragma unroll
    for (int j = 0; j < DB; j++)
      rec[j] = act[j] ? s.brec[(size_t)band[j] * s.n + rc] : make_uint4(0u, 0u, 0u, 0u);
    int ch[DB];
    uint2 w[DB];
#pragma unroll
    for (int j = 0; j < DB; j++) {
      const uint64_t cc = (uint64_t)rec[j].x | ((uint64_t)rec[j].y << 32);
      ch[j] = 0;
#pragma unroll
      for (int k = 0; k < 7; k++) {
        const uint32_t c8 = (uint32_t)(cc >> (8 * ch[j])) & 0xFFu;
        if (rem[j] >= c8 && ch[j] == k) {
          rem[j] -= c8;
          ch[j]++;
        }
      }
      w[j] = make_uint2(0u, 0u);
      if (act[j]) w[j] = *(const uint2 *)(s.table + ((size_t)band[j] * s.n + rc) * B + ch[j] * 128 + q * 8);
    }
#pragma unroll
    for (int j = 0; j < DB; j++) {
      // present (non-zero) bytes of the lane's 8 cells
      auto nzb = [](uint32_t v) { return (v | (v >> 1) | (v >> 2) | (v >> 3) | (v >> 4) | (v >> 5) | (v >> 6) | (v >> 7)) & 0x01010101u; };
      const uint32_t m0 = nzb(w[j].x), m1 = nzb(w[j].y);
      const int cnt = __builtin_popcount(m0) + __builtin_popcount(m1);
      const int incl = row16_scan(cnt);
      const int excl = incl - cnt;
      const bool holder = act[j] && (int)rem[j] >= excl && (int)rem[j] < incl;
      int32_t val = -1;
      if (holder) {  // the (rem - excl)-th present cell of its 8
        int need = (int)rem[j] - excl, pos = 0;
        uint32_t byte = 0;
#pragma unroll
        for (int v = 0; v < 8; v++) {
          const uint32_t bv = ((v < 4 ? w[j].x : w[j].y) >> (8 * (v & 3))) & 0xFFu;
          if (bv != 0) {
            if (need == 0) { pos = v; byte = bv; }
            need--;
          }
        }
        const int col = band[j] * B + ch[j] * 128 + q * 8 + pos;  // shard-local column
        const bool fresh = s_is_esc(byte) ? esc_fresh(s, rc, col) : S_AGE(s_widen(byte)) < GM_TFAIL;
        val = ((s.c0 + col) << 1) | (int32_t)(fresh && s.c0 + col != me);
      }
      // lane d of the row takes draw d's status from its holder; a draw no lane holds (the record's
      // counts and the cells disagree) keeps -1, which the acceptance reports as GM_ERR_DRAWS if it
      // reaches it -- never an older tick's value left in the reused status buffer
      const uint32_t hm = row16_bits(__ballot(holder), g);
      const int32_t v = row16_bcast(val, g, hm ? __builtin_ctz(hm) : 0);
      if (act[j] && q == dj[j]) myst = hm ? v : -1;
    }
  }
  if (mine) st[q] = myst;
}

hipError_t gm_launch_draw0(const SState &s, int t, int r0, int r1, hipStream_t st) {
  if (r1 <= r0) return hipSuccess;
  const size_t smem = sizeof(uint32_t) * 16 * (size_t)(s.nb + 1);
  hipLaunchKernelGGL(gm_s_draw0<1024>, dim3((r1 - r0 + 15) / 16), dim3(256), smem, st, s, t, r0, r1);
  return hipGetLastError();
}
// true when gm_s_draw0 applies: B = 1024, no join ramp, <= 16 ranks, the band prefix fits LDS
bool gm_draw0_ok(const SState &s) {
  return s.band == 1024 && !s.ramp && s.shard_count <= 16 && sizeof(uint32_t) * 16 * (size_t)(s.nb + 1) <= 65536;
}

// Phase B: every rank replays every pending row's S2 stream (round 0: outputs
// [0, 16) from gm_s_mtgen; round q >= 1: [16 + 64(q-1), 16 + 64q) from the lazy
// generator) and resolves the draws whose rank lands in its own columns.
// status[r][d] = -2 for an output Lemire rejects (same on every rank),
// (global column << 1) | fresh on the owning rank, -1 elsewhere (MAX-allreduced).
template <int B>
__global__ __launch_bounds__(256) void gm_s_draw(SState s, int t, int round, int D, int listed, int r0, int r1) {
  extern __shared__ __align__(16) uint32_t p_smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // listed: the rows still pending after round 0, in ascending order (gm_s_plist_sort);
  // their statuses go to status1 by list position. Unlisted: rows [r0, r1) (a row chunk)
  const int i = (listed ? 0 : r0) + (int)blockIdx.x * 4 + wave;
  if (listed && i >= plist_len(s, listed)) return;
  const int r = listed ? s.plist[listed][i] : i;
  if (r >= (listed ? s.n : r1)) return;
  // round 0 has no lazy generator state (gm_launch_draw sizes its LDS to the chunk prefix)
  uint32_t *pre = p_smem + wave * (round == 0 ? (size_t)gm_draw_chunks(s.wp, B) + 1 : gm_draw_lds_words(s.wp, B));
  uint32_t *mts = pre + gm_draw_chunks(s.wp, B) + 1;
  const int G = s.shard_count;
  int32_t *acc = s.acc + (size_t)r * 8;
  // round 0: every load of the row issues at once -- crash flag, delivered-list count, the ranks'
  // counts, the 16 S2 outputs and this shard's first band record (for the chunk prefix; ~88 % of the
  // rows resolve a draw here) -- one memory round trip before the chunk search, not four
  uint32_t raw0 = 0;
  uint4 rec0 = make_uint4(0u, 0u, 0u, 0u);
  if (round == 0) {
    const int par = t & 1;
    int failed = s.failed[r], kin = s.inbox_cnt[par][r];
    int size = 0, nf = 0;
    bool selfapp = false;
    raw0 = lane < S_MT_RAW ? s.mtraw[(size_t)r * S_MT_RAW + lane] : 0u;
    rec0 = gm_row_rec0(s, r, lane);
    for (int g = 0; g < G; g++) {
      const int pr = s.xcnt[S_XC(s, g, r)];
      size += pr & S_XC_COUNT;
      selfapp |= (pr & S_XC_SELFAPP) != 0;
      nf += s.xcnt[S_XC(s, g, r) + 1];
    }
    asm volatile("" : "+v"(raw0), "+v"(rec0.x), "+v"(rec0.y), "+v"(rec0.z), "+v"(rec0.w));
    const bool live = !failed && s_ingroup(s.ramp, s.intro_until, r, t);  // else untouched
    if (lane == 0) {  // lists delivered this tick; consumed by gm_s_band, the append target of tick t+2
      s.rowstat[(size_t)r * 4] = live ? kin : 0;
      s.inbox_cnt[par][r] = 0;
    }
    if (selfapp && lane == 0) {
      // join ramp: row r appended its own entry (updateMyPos found no larger id in its start
      // group, gm_s_band); the reference appends only if no larger id is present at all --
      // the shards above the group must hold nothing of the row (present, or removed this tick)
      for (int g = 0; g < G; g++) {
        const int c0g = (int)((int64_t)s.n * g / G);
        if (c0g > (r | 3) && ((s.xcnt[S_XC(s, g, r)] & S_XC_COUNT) || s.xcnt[S_XC(s, g, r) + 1]))
          atomicOr(s.err, GM_ERR_SELF);
      }
    }
    const int numpot = size - 1 - nf;
    int nj = 0, jn[4] = {0, 0, 0, 0};
    if (s.ramp && r == 0 && live)  // gossipnodes = newNodes first (MP1Node.cpp:458): this tick's joiners, ascending id
      for (int c = max(1, 4 * (t - 1)); c < min(s.n, 4 * t); c++) jn[nj++] = c;
    const bool pend = live && numpot > 0 && nj < min(GM_FANOUT, numpot);
    if (lane == 0) {
      acc[0] = nj;
      for (int q = 0; q < 4; q++) acc[1 + q] = jn[q];
      acc[6] = numpot;
      acc[7] = size;
      s.pending[r] = pend;
      int32_t *stat = s.rowstat + (size_t)r * 4;
      stat[1] = live ? size : 0;
      stat[2] = live ? nf : 0;
      stat[3] = live && !pend ? nj : 0;
      if (live && !pend && nj) {  // the joiners alone (no draws): enqueue now, like gm_s_accept
        int32_t *cnt_out = s.inbox_cnt[(t & 1) ^ 1];
        for (int q = 0; q < nj; q++) {
          s.targets[(size_t)r * GM_FANOUT + q] = jn[q];
          const int slot = atomicAdd(&cnt_out[jn[q]], 1);
          if (slot < s.kcap) s.inbox[(t & 1) ^ 1][(size_t)jn[q] * S_KMAX + slot] = r;
          else atomicOr(s.err, GM_ERR_INBOX);
        }
      }
    }
    if (!pend) return;
  } else if (!s.pending[r]) {
    return;
  }
  // the round of this row's draws: the launch's for a bounded round over a pending list;
  // the row's own (pending[r] = its next round) in the host-driven loop, where rows that a
  // bounded round could not take continue from where they stopped
  const int rr = (round == 0 || listed) ? round : s.pending[r];
  const uint32_t size = (uint32_t)acc[7];
  uint32_t own_lo = 0;
  for (int g = 0; g < s.shard_rank; g++) own_lo += (uint32_t)s.xcnt[S_XC(s, g, r)] & S_XC_COUNT;
  const uint32_t own_cnt = (uint32_t)s.xcnt[S_XC(s, s.shard_rank, r)] & S_XC_COUNT;
  // "me" (myPos's id, MP1Node.cpp:459-460,470) is the row's own column, or in the join ramp
  // the quirk's target column; only the rank owning it knows it (mecol is -1 elsewhere), and
  // only that rank resolves a draw there: it reports "me" as not fresh, which the acceptance
  // skips the same way
  const int me = s.ramp ? s.mecol[r] : r;
  bool have_pre = false;  // this shard's chunk prefix of the row, built on first use
  const uint32_t thr = (0u - size) % size;
  GmLazyMT mt;
  int32_t *st = listed ? s.statusl[listed] + (size_t)i * D : s.status + (size_t)r * D;
  for (int d0 = 0; d0 < D; d0 += 64) {
    const int cnt = min(64, D - d0);
    uint32_t raw = 0;
    if (round == 0) {
      raw = raw0;  // D = 16: the one batch
    } else {  // round q >= 1 continues after 16 + 64 (q - 1) outputs (round 2 of the bounded tick: after 80)
      raw = gm_mt_batch(mt, mts, gm_rd_seed(s.rd_seed, t, r + 1), d0 == 0, S_MT_RAW + 64 * (rr - 1) + d0, cnt,
                        lane);
    }
    const uint64_t prod = (uint64_t)raw * size;
    const bool ok = lane < cnt && (uint32_t)prod >= thr;
    const uint32_t ix = (uint32_t)(prod >> 32);
    const bool mine = ok && ix >= own_lo && ix < own_lo + own_cnt;
    int32_t val = ok ? (s.stub ? stub_target(ix, size, s.n) : -1) : -2;
    uint64_t m = __ballot(mine);
    if (m && !have_pre) {
      uint32_t osz, onf;
      gm_row_totals<B>(s, r, lane, pre, osz, onf, round == 0 ? &rec0 : nullptr);
      have_pre = true;
    }
    while (m) {
      const int grp = lane >> 3;
      int myd = 0, c8 = 0, d[8];
#pragma unroll
      for (int i = 0; i < 8; i++) {
        d[i] = m ? __builtin_ctzll(m) : 64;
        if (m) {
          if (grp == i) myd = d[i];
          m &= m - 1;
          c8++;
        }
      }
      const uint32_t myix = __shfl(ix, myd, 64) - own_lo;
      int col[8], fr[8];
      gm_resolve8<B>(s, r, pre, grp < c8, myix, lane, col, fr);
#pragma unroll
      for (int i = 0; i < 8; i++)
        if (i < c8 && lane == d[i]) val = col[i] < 0 ? -1 : (((s.c0 + col[i]) << 1) | (fr[i] && s.c0 + col[i] != me));
    }
    if (lane < cnt) st[d0 + lane] = val;
  }
  if (rr > 0 && !listed && lane == 0) s.pending[r] = rr + 1;
}

// Phase C: with every draw resolved (MAX-allreduced status), run the acceptance loop
// of MP1Node.cpp:466-489 (skip me, skip stale, skip duplicates) identically on every
// rank; finished rows enqueue themselves into their targets' inboxes for tick t+1.
// mode 0: every row, statuses by row; rows left pending are counted (npending, host loop).
// mode 1: every row, and rows left pending are also appended to plist (bounded rounds).
// mode 2: the plist rows, statuses by list position; a row still pending sets GM_ERR_DRAWS.
// in_list 0: every row, statuses by row; 1 / 2: the rows of pending list 1 / 2, statuses by
// list position. Rows left pending go to: out -1 -> GM_ERR_DRAWS (bounded rounds exhausted),
// 0 -> the npending count (host-driven loop), 1 / 2 -> pending list 1 / 2 (next bounded round).
__global__ __launch_bounds__(256) void gm_s_accept(SState s, int t, int D, int in_list, int out, int r0, int r1) {
  const int i = (in_list ? 0 : r0) + (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (in_list && i >= plist_len(s, in_list)) return;
  const int r = in_list ? s.plist[in_list][i] : i;
  if (r >= (in_list ? s.n : r1) || !s.pending[r]) return;
  int32_t *acc = s.acc + (size_t)r * 8;
  // the row's accumulator (8 ints) and, in round 0 (D = 16), its 16 statuses by vector loads, all
  // in flight together: the draw loop below then runs on registers, not one load round trip per
  // draw (each row's words are its own 32 B / 64 B)
  const int4 a0 = ((const int4 *)acc)[0], a1 = ((const int4 *)acc)[1];
  int n = a0.x;
  const int numpot = a1.z;
  int g[GM_FANOUT] = {a0.y, a0.z, a0.w, a1.x, a1.y};
  static_assert(GM_FANOUT == 5, "acc = {n, g[0..4], numpot, size}");
  const int32_t *st = in_list ? s.statusl[in_list] + (size_t)i * D : s.status + (size_t)r * D;
  bool done = n >= GM_FANOUT || n >= numpot;
  auto take = [&](int32_t v) {  // one draw of MP1Node.cpp:466-489, in draw order
    if (done || v == -2) return;  // output rejected by Lemire: not a draw
    if (v < 0) {                  // a draw no shard resolved
      atomicOr(s.err, GM_ERR_DRAWS);
      done = true;
      return;
    }
    const int c = v >> 1;
    if (c == r) return;     // "me"
    if (!(v & 1)) return;   // age >= TFAIL
    bool dup = false;
#pragma unroll
    for (int q = 0; q < GM_FANOUT; q++) dup |= q < n && g[q] == c;
    if (!dup) {
#pragma unroll
      for (int q = 0; q < GM_FANOUT; q++)
        if (q == n) g[q] = c;
      n++;
    }
    done = n >= GM_FANOUT || n >= numpot;
  };
  if (D == 16) {
    int4 v4[4];
#pragma unroll
    for (int q = 0; q < 4; q++) v4[q] = ((const int4 *)st)[q];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      take(v4[q].x);
      take(v4[q].y);
      take(v4[q].z);
      take(v4[q].w);
    }
  } else {
    for (int d = 0; d < D && !done; d++) take(st[d]);
  }
  for (int q = 0; q < n; q++) acc[1 + q] = g[q];
  acc[0] = n;
  if (!done) {
    // pending[r] = the row's next round: host-driven rounds q >= 1 draw S2 outputs
    // [16 + 64(q-1), 16 + 64q), so bounded round 1 = host round 1 and bounded round 2 (outputs
    // [80, 336)) = host rounds 2..5. A row no bounded round takes (its list is full, or it is
    // still short after round 2) is counted in npending; the host finishes it with the
    // host-driven rounds before anything reads the tick (draw_settle, gm_host.hip)
    if (out == 0) {
      atomicAdd(s.npending, 1);  // gm_s_draw advanced pending[r]
    } else if (out > 0) {
      s.pending[r] = out;
      const uint32_t slot = atomicAdd(s.plist_cnt[out], 1u);
      if (slot < (uint32_t)s.plist_cap[out]) s.plist[out][slot] = r;
      else atomicAdd(s.npending, 1);
    } else {
      s.pending[r] = 1 + (GM_D_MORE_ROUND + GM_D_LAST_ROUND) / 64;
      atomicAdd(s.npending, 1);
    }
    return;
  }
  s.pending[r] = 0;
  const int par = t & 1;
  int32_t *cnt_out = s.inbox_cnt[par ^ 1];
  int slot[GM_FANOUT];
#pragma unroll
  for (int q = 0; q < GM_FANOUT; q++)  // the row's appends in flight together, then their stores
    if (q < n) slot[q] = atomicAdd(&cnt_out[g[q]], 1);
#pragma unroll
  for (int q = 0; q < GM_FANOUT; q++) {
    if (q >= n) continue;
    s.targets[(size_t)r * GM_FANOUT + q] = g[q];
    if (slot[q] < s.kcap) s.inbox[par ^ 1][(size_t)g[q] * S_KMAX + slot[q]] = r;
    else atomicOr(s.err, GM_ERR_INBOX);
  }
  s.rowstat[(size_t)r * 4 + 3] = n;
}

// SCALED initial state (gm_config.init_mode): every observer holds every subject.
// Cold: {hb 0, ts 0}. Warm at t0: own entry {2*t0-1, t0}; others {2*(t0-1-a)-1,
// t0-a}, a = splitmix64(seed ^ r<<32 ^ c) % 4 -- values as if the cluster had been
// gossiping, so the first ticks carry no mass-staleness transient. Padding absent.
// Cells are encoded relative to tick t0 (S_CELL: h = 255 - (2*t0 - hb), age = t0 - ts).
// Join ramp (warm = 2): nobody in any list but the introducer's own entry {hb 0, ts 0}
// (nodeStart of node 0 at tick 0, MP1Node.cpp:126-140); state as of tick 0.
// The band kernel's lane mapping (one wave per (band, rows) unit, 16 cells per lane), so the
// escaped cells (a cold start escapes them all: odd h) form the same per-(band, row) lists
// in the pool of tick t0 that gm_s_band writes, and every record's .w names its list.
template <int B>
__global__ __launch_bounds__(256) void gm_s_init(SState s, int warm, int t0, uint64_t seed) {
  constexpr int LPR = B / S_COLS_PER_LANE, RPW = 64 / LPR, Q = S_COLS_PER_LANE;
  const int U = (s.n + RPW - 1) / RPW;
  const int ub = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (ub >= U) return;  // whole wave
  const int lane = threadIdx.x & 63, li = lane % LPR;
  const int band = blockIdx.y, r = ub * RPW + lane / LPR;
  const bool row = r < s.n;
  uint32_t cw[8] = {0, 0, 0, 0, 0, 0, 0, 0}, bw[4] = {0, 0, 0, 0};
  if (row) {
#pragma unroll
    for (int q = 0; q < Q; q++) {
      const int j = band * B + li * Q + q;  // shard-local column
      uint32_t e = 0;                       // absent
      if (j < s.w && warm == 2) {
        if (r == 0 && s.c0 + j == 0) e = S_CELL(255u, 0u);
      } else if (j < s.w) {
        const int c = s.c0 + j;
        if (!warm) e = S_CELL(255u, 0u);  // hb 0 = 2*t0 at t0 = 0
        else if (c == r) e = S_CELL(254u, 0u);
        else {
          const int a = (int)((gm_mix64(seed ^ ((uint64_t)(uint32_t)r << 32) ^ (uint64_t)(uint32_t)c) >> 40) % 4);
          e = S_CELL((uint32_t)(252 - 2 * a), (uint32_t)a);
        }
      }
      cw[q >> 1] |= e << (16 * (q & 1));
      bw[q >> 2] |= s_narrow(e) << (8 * (q & 3));
    }
  }
  const uint32_t em = esc_mask16(bw[0], bw[1], bw[2], bw[3]);
  int etot;
  const int eoff = row_scan<LPR>(__builtin_popcount(em), li, lane, etot);
  const int par = t0 & 1;  // the state is "as of tick t0": tick t0 + 1 reads this pool
  const size_t slab = (size_t)band * s.n;
  const uint32_t base = row_alloc<LPR>(s, par, slab, min(r, s.n - 1), etot, li, lane);
  __shared__ uint32_t lds_all[4 * S_LDS_WAVE_WORDS];
  uint32_t *lds = lds_all + (threadIdx.x >> 6) * S_LDS_WAVE_WORDS;
  if (em) esc_park(lds, lane, cw);
  if (base != 0) esc_emit(lds, lane, esc_list(s, par, slab, r, base), eoff, em, li * Q, etot <= S_ESC_IN, s.err, s.lag_hmin);
  if (!row) return;
  *(u32x4 *)(s.table + (slab + r) * B + li * Q) = (u32x4){bw[0], bw[1], bw[2], bw[3]};
  if (li == 0) {
    s.brec[slab + r] = make_uint4(0u, 0u, 0u, base);
    if (band == 0) {
      s.hbctr[r] = warm == 1 ? 2 * t0 : 0;
      s.wtick[r] = t0;
    }
  }
}

// ------------------------------------------------------------ launch wrappers
// (template dispatch over the band width; called by gm_host.hip)
// the band kernels of rows [r0, r1) (r0, r1 multiples of the rows per unit, or r1 = n)
#ifndef GM_FAST_BPW
#define GM_FAST_BPW 2  // bands per wave of gm_s_band_fast (profiles/r05/ab4, ab5: 3.38 vs 3.48 ms at one)
#endif
template <int B>
static void launch_band_b(const SState &s, int t, int drop_pct, int r0, int r1, hipStream_t st) {
  constexpr int RPW = 64 / (B / S_COLS_PER_LANE);
  const int u0 = r0 / RPW, u1 = (r1 + RPW - 1) / RPW;
  if (u1 <= u0) return;
  const dim3 nblk((u1 - u0 + 3) / 4, s.nb);  // (units of the chunk in a band / 4, bands)
  if (drop_pct >= 0) {
    hipLaunchKernelGGL((gm_s_band<B, true>), dim3(nblk), dim3(256), 0, st, s, t, drop_pct, u0, u1);
  } else if (B == 1024 && !s.ramp && s.fb_list) {  // the fast path, then the units it handed back
    const dim3 nblk2((u1 - u0 + GM_FAST_WG - 1) / GM_FAST_WG, (s.nb + GM_FAST_BPW - 1) / GM_FAST_BPW);
    if (u0 == 0 && r1 == s.n)
      hipLaunchKernelGGL((gm_s_band_fast<B == 1024 ? B : 1024, false, GM_FAST_BPW>), nblk2, dim3(64 * GM_FAST_WG), 0,
                         st, s, t, u0, u1);
    else
      hipLaunchKernelGGL((gm_s_band_fast<B == 1024 ? B : 1024, true, GM_FAST_BPW>), nblk2, dim3(64 * GM_FAST_WG), 0,
                         st, s, t, u0, u1);
    hipLaunchKernelGGL((gm_s_band_listed<B == 1024 ? B : 1024>), dim3(S_FB_BLOCKS), dim3(256), 0, st, s, t, u0, u1);
  } else {
    hipLaunchKernelGGL((gm_s_band<B, false>), dim3(nblk), dim3(256), 0, st, s, t, drop_pct, u0, u1);
  }
}

// the per-tick work before the band kernels: event counters, the S2 precompute
hipError_t gm_launch_tick_prologue(const SState &s, int t, hipStream_t st, bool zero_draw) {
  // the event records of a tick (per-(row, band) slots + spill ring) stay readable until the next
  // tick: gm_s_mtgen zeroes their counters
  hipLaunchKernelGGL(gm_s_mtgen, dim3((std::max(s.n, 1 + S_EV_STRIPES) + 255) / 256), dim3(256), 0, st, s, t,
                     zero_draw ? 1 : 0);
  return hipGetLastError();
}

hipError_t gm_launch_band_rows(const SState &s, int t, int drop_pct, int r0, int r1, hipStream_t st) {
  switch (s.band) {
    case 64: launch_band_b<64>(s, t, drop_pct, r0, r1, st); break;
    case 128: launch_band_b<128>(s, t, drop_pct, r0, r1, st); break;
    case 256: launch_band_b<256>(s, t, drop_pct, r0, r1, st); break;
    case 512: launch_band_b<512>(s, t, drop_pct, r0, r1, st); break;
    case 1024: launch_band_b<1024>(s, t, drop_pct, r0, r1, st); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <int B>
static hipError_t launch_tick_b(const SState &s, int t, int drop_pct, hipStream_t st, hipEvent_t k0,
                                hipEvent_t k1, bool pick) {
  (void)gm_launch_tick_prologue(s, t, st, false);
  if (k0) (void)hipEventRecord(k0, st);
  launch_band_b<B>(s, t, drop_pct, 0, s.n, st);
  if (k1) (void)hipEventRecord(k1, st);
  if (s.ramp) {
    hipLaunchKernelGGL(gm_s_selfcheck, dim3(16), dim3(256), 0, st, s);
    (void)hipMemsetAsync(s.selfadd_cnt, 0, sizeof(uint32_t), st);
  }
  const size_t smem = sizeof(uint32_t) * 4 * gm_draw_lds_words(s.wp, s.band);
  if (pick && B == 1024 && s.pk_list && !s.ramp) {  // four rows per wave, then the rows it left (pk_cnt: 0 by gm_s_mtgen)
    constexpr int R = 4 * GM_PICK_WG;  // rows per workgroup
    hipLaunchKernelGGL((gm_s_pick0<B == 1024 ? B : 1024>), dim3((s.n + R - 1) / R), dim3(64 * GM_PICK_WG),
                       sizeof(uint32_t) * R * (size_t)(s.nb + 1) + sizeof(uint2) * R * (size_t)s.nb, st, s, t);
    hipLaunchKernelGGL((gm_s_pick<B>), dim3(256), dim3(256), smem, st, s, t, 1);
  } else if (pick) {
    hipLaunchKernelGGL((gm_s_pick<B>), dim3((s.n + 3) / 4), dim3(256), smem, st, s, t, 0);
  }
  return hipGetLastError();
}

hipError_t gm_launch_tick(const SState &s, int t, int drop_pct, hipStream_t st, hipEvent_t k0, hipEvent_t k1,
                          bool pick) {
  switch (s.band) {
    case 64: return launch_tick_b<64>(s, t, drop_pct, st, k0, k1, pick);
    case 128: return launch_tick_b<128>(s, t, drop_pct, st, k0, k1, pick);
    case 256: return launch_tick_b<256>(s, t, drop_pct, st, k0, k1, pick);
    case 512: return launch_tick_b<512>(s, t, drop_pct, st, k0, k1, pick);
    case 1024: return launch_tick_b<1024>(s, t, drop_pct, st, k0, k1, pick);
    default: return hipErrorInvalidValue;
  }
}

// rows [r0, r1) (unlisted) or the pending list `listed`. Round 0 draws only the 16 precomputed
// outputs: no lazy generator, so its waves take the chunk prefix's LDS alone.
hipError_t gm_launch_draw(const SState &s, int t, int round, int D, int listed, hipStream_t st, int r0, int r1) {
  if (r1 < 0) r1 = s.n;
  if (round == 0 && !listed && D == S_MT_RAW && gm_draw0_ok(s) && !(getenv("GM_DRAW0") && !atoi(getenv("GM_DRAW0"))))
    return gm_launch_draw0(s, t, r0, r1, st);  // four rows per wave
  const size_t words = round == 0 ? (size_t)gm_draw_chunks(s.wp, s.band) + 1 : gm_draw_lds_words(s.wp, s.band);
  const size_t smem = sizeof(uint32_t) * 4 * words;
  const int rows = listed ? s.plist_cap[listed] : r1 - r0;
  if (rows <= 0) return hipSuccess;
  const dim3 grid((rows + 3) / 4), blk(256);
  switch (s.band) {
    case 64: hipLaunchKernelGGL(gm_s_draw<64>, grid, blk, smem, st, s, t, round, D, listed, r0, r1); break;
    case 128: hipLaunchKernelGGL(gm_s_draw<128>, grid, blk, smem, st, s, t, round, D, listed, r0, r1); break;
    case 256: hipLaunchKernelGGL(gm_s_draw<256>, grid, blk, smem, st, s, t, round, D, listed, r0, r1); break;
    case 512: hipLaunchKernelGGL(gm_s_draw<512>, grid, blk, smem, st, s, t, round, D, listed, r0, r1); break;
    case 1024: hipLaunchKernelGGL(gm_s_draw<1024>, grid, blk, smem, st, s, t, round, D, listed, r0, r1); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t gm_launch_accept(const SState &s, int t, int D, int in_list, int out, hipStream_t st, int r0, int r1) {
  if (r1 < 0) r1 = s.n;
  const int rows = in_list ? s.plist_cap[in_list] : r1 - r0;
  if (rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(gm_s_accept, dim3((rows + 255) / 256), dim3(256), 0, st, s, t, D, in_list, out, r0, r1);
  return hipGetLastError();
}

// The pending rows of round 0 in ascending order: the list order (= status1 rows) must be
// the same on every rank, whatever order the atomics appended them in. A list that overflowed
// holds a subset that depends on that order, so it is void (plist_len 0) and all of its rows go
// to the host-driven rounds (every rank counts the same total, acceptance being identical).
__global__ __launch_bounds__(1024) void gm_s_plist_sort(SState s, int l) {
  __shared__ int32_t v[S_PLIST_CAP];
  int32_t *list = s.plist[l];
  if (*s.plist_cnt[l] > (uint32_t)s.plist_cap[l]) {  // the appends past cap were counted already
    if (threadIdx.x == 0) atomicAdd(s.npending, s.plist_cap[l]);
    return;
  }
  const int cnt = (int)*s.plist_cnt[l];
  if (cnt <= 1) return;
  int m = 1;
  while (m < cnt) m <<= 1;
  for (int k = threadIdx.x; k < m; k += blockDim.x) v[k] = k < cnt ? list[k] : 0x7FFFFFFF;
  __syncthreads();
  for (int size = 2; size <= m; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int k = threadIdx.x; k < m; k += blockDim.x) {
        const int o = k ^ stride;
        if (o > k) {
          const bool up = (k & size) == 0;
          const int a = v[k], b = v[o];
          if ((a > b) == up) {
            v[k] = b;
            v[o] = a;
          }
        }
      }
      __syncthreads();
    }
  for (int k = threadIdx.x; k < cnt; k += blockDim.x) list[k] = v[k];
}

hipError_t gm_launch_plist_sort(const SState &s, int l, hipStream_t st) {
  hipLaunchKernelGGL(gm_s_plist_sort, dim3(1), dim3(1024), 0, st, s, l);
  return hipGetLastError();
}

template <int B>
static hipError_t launch_init_b(const SState &s, int warm, int t0, uint64_t seed, hipStream_t st) {
  constexpr int RPW = 64 / (B / S_COLS_PER_LANE);
  const dim3 nblk((((s.n + RPW - 1) / RPW) + 3) / 4, s.nb);
  hipLaunchKernelGGL(gm_s_init<B>, nblk, dim3(256), 0, st, s, warm, t0, seed);
  return hipGetLastError();
}

hipError_t gm_launch_init(const SState &s, int warm, int t0, uint64_t seed, hipStream_t st) {
  switch (s.band) {
    case 64: return launch_init_b<64>(s, warm, t0, seed, st);
    case 128: return launch_init_b<128>(s, warm, t0, seed, st);
    case 256: return launch_init_b<256>(s, warm, t0, seed, st);
    case 512: return launch_init_b<512>(s, warm, t0, seed, st);
    case 1024: return launch_init_b<1024>(s, warm, t0, seed, st);
    default: return hipErrorInvalidValue;
  }
}
