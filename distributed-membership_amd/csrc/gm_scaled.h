// gm_scaled.h -- device state of the SCALED tick (see gm_scaled.hip).
#pragma once
#include <stdint.h>

#include "gm_device.h"

#define S_KMAX 64                // inbox capacity (gossip lists per receiver per tick)
#define S_COLS_PER_LANE 16       // 32 B of table + 16 B per sender payload per lane and row
#define S_ROW_ALIGN 512          // padded row width granule (a multiple of every band width up to 512)
#define S_CHUNK(B) ((B) >= 1024 ? 128 : 64)  // columns per rank-select chunk (<= 8 chunks per band)
#define S_SB 8                   // sender ids prefetched per row; payload loads in flight per lane
#define S_MT_RAW 16              // mt19937 outputs precomputed per row and tick (gm_s_mtgen)
#define S_SELFADD_CAP 65536      // join ramp: self appends verified per tick (gm_s_selfcheck)
#define S_PLIST_CAP 4096         // sharded tick: rows a second (bounded) draw round takes
#define S_FB_BLOCKS 2048         // workgroups (4 waves) of gm_s_band's pass over the fast path's handed-back units
#define GM_D_MORE_ROUND 64       // S2 outputs of bounded round 1 (= one host-driven round)
#define GM_D_LAST_ROUND 256      // S2 outputs of bounded round 2 (= host-driven rounds 2..5)

// SCALED cell (16 bits), relative to the tick w the row was last written at:
//   h = 255 - (2w - hb) (8 bits, the heartbeat; larger = newer), age = w - ts (5 bits);
//   cell = h << 5 | age, 0 = absent. Every tick rewrites every live cell, re-basing it
// to the new tick (h -= 2, age += 1: cell - 63). Ordering cells by value orders them
// by heartbeat first and, for equal heartbeats, keeps the older timestamp -- so the
// merge of updatelistCallBack is a max. In the SCALED regime a live node's heartbeat
// at tick t is 2t-1 (h = 254); h falls by 2 per tick of heartbeat lag, and a present
// entry lagging more than ~126 ticks sets GM_ERR_LAG instead of wrapping.
#define S_CELL(h, age) (((h) << 5) | (age))
// Stored table cell: ONE BYTE per (observer, subject). The 16-bit cell above is the
// working format in registers; in HBM a cell is
//   0             absent
//   h4 << 4 | a   h = 224 + 2 h4 (h4 in [3, 15]: even h in [230, 254], heartbeat lag <= 12
//                 ticks), age a <= 14 -- every live entry of a warm, steady cluster. The range
//                 is one short of the byte's at both ends, so that a stored byte re-based by one
//                 tick (h4 - 1, a + 1) is again a byte: gm_s_band's fast path merges and sweeps
//                 the stored bytes themselves and tests only its outputs
//   1 (S_B_ESC)   escaped: the exact 16-bit cell is an entry of the (band, row)'s escape list
//                 (codes 2..15, h4 = 0, are unused)
// Cells outside the byte's range (odd h of cold-start / JOINREQ entries, lag > 12 or age > 14,
// e.g. a crashed node's entries in the ticks before TREMOVE) escape. The pool is COMPACT: per
// (band, row) the escaped cells of the row's band slice (lane by lane; entries carry their columns,
// so the order is not significant), as consecutive u32
// ENTRIES of the tick that wrote them (tick parity: written at t, read at t+1), one u32 per
// escaped cell: its column in the band (low 16 bits) | its 16-bit cell << 16. The first S_ESC_IN
// entries sit in the list's fixed inline slot (no allocation: a crash window escapes ~1 % of a
// row's cells, ~10 per 1024-column band), the rest in the pool region of the list's stripe.
// The (band, row) record's .w is the list's word: entry count | offset in the stripe's region
// << 11 (0: no escapes), so a reader knows the list's extent with the row's metadata and
// prefetches the inline entries with the payload gathers; it scatters the entries into its
// row's cells through LDS (entries carry their columns: no per-cell search). Capacity is
// bounded (gm_host.hip: dense-equivalent for small clusters, a fraction of the cells beyond);
// an overflow sets GM_ERR_ESC (-> GM_ERANGE) -- never a silent divergence.
#define S_B_ESC 1u
#define S_H4_MIN_H 230u  // smallest h a stored byte holds (h4 = 3)
#define S_AGE_MAX_B 14u  // largest age a stored byte holds
#define S_ESC_IN 16                 // entries of a (band, row) list held inline (64 B per list)
#define S_EW_TOT(w) ((w) & 0x7FFu)  // escape-list word: entry count (<= band width)
#define S_EW_OFF(w) ((w) >> 11)     // offset of entries S_ESC_IN.. in the stripe's pool region
#define S_EW_REGION_MAX (1u << 21)  // pool entries per stripe the word can address
__host__ __device__ inline bool s_is_esc(uint32_t b) { return b != 0 && b < 16; }
__host__ __device__ inline uint32_t s_widen(uint32_t b) {  // byte -> 16-bit cell (escape codes: look in the pool)
  return b == 0 ? 0u : (7168u + ((b & 0xF0u) << 2) + (b & 0x0Fu));
}
__host__ __device__ inline uint32_t s_narrow(uint32_t c) {  // 16-bit cell -> byte (an escape code if not representable)
  if (c == 0) return 0u;
  const uint32_t h = c >> 5, a = c & 31u;
  if (h >= S_H4_MIN_H && !(h & 1) && a <= S_AGE_MAX_B) return (((h - 224) >> 1) << 4) | a;
  return S_B_ESC;
}
__host__ __device__ inline int s_start(int j) { return j >> 2; }  // (int)(0.25 * j) for j >= 0
__host__ __device__ inline int s_hbase(int ramp, int j) { return (ramp && j > 0) ? 2 * (s_start(j) + 1) : 0; }
__host__ __device__ inline bool s_ingroup(int ramp, int intro_until, int r, int t) {
  return !ramp || r == 0 || (t >= s_start(r) + 2 && s_start(r) + 1 <= intro_until);
}
// column shards: xcnt's per-(rank, row) present word carries a flag for a self append
#define S_XC_SELFAPP 0x40000000
// int32 index of (rank g, row r)'s present word in the chunk-major xcnt (numfailed follows it)
#define S_XC(s, g, r) \
  ((((((size_t)(r) >> (s).xlog) * (size_t)(s).shard_count + (size_t)(g)) << (s).xlog) + ((size_t)(r) & ((1u << (s).xlog) - 1))) * 2)
#define S_XC_COUNT 0x3FFFFFFF
#define S_H(c) ((c) >> 5)
#define S_AGE(c) ((c) & 31u)
// payload (sendMemberList's fresh entries, re-based to the receiving tick: h' = h - 2):
// one NIBBLE per cell, 0 = not sent, n in [1, 14] = h' = 224 + 2n (the even values
// [226, 252]: heartbeat lag <= 13 ticks -- every value of a warm, steady cluster), 15 =
// escape: the byte h' is in the wide plane (odd h' of cold-start / JOINREQ entries, or a
// larger lag). Larger nibble = larger h' = newer, so the merge maxes nibbles directly.
#define S_NIB_BASE 224u
#define S_NIB_ESC 15u
#define S_NIB_H(n) (S_NIB_BASE + 2u * (n))

// keyed loss threshold (gm_device.h gm_drop_thresh; gm_scaled.hip s_keep)
__host__ __device__ inline uint32_t s_drop_thresh(int pct) { return gm_drop_thresh(pct); }

#define S_EV_STRIPES 16384  // the tick's event total in partial sums (a TREMOVE tick adds ~4 M of them)
#define S_EV_ADD 1u
#define S_EV_REMOVE 2u

// bcnt word of one (row, band): present | numfailed << 11 | events << 22 (saturating)
#include <hip/hip_runtime.h>
#define S_BC_PRES(v) ((v) & 0x7FFu)
#define S_BC_FAIL(v) (((v) >> 11) & 0x7FFu)
#define S_BC_NEV(v) ((v) >> 22)

struct SState {
  int n;                   // observers (rows) = N
  int wp;                  // padded shard width (columns per row, multiple of S_ROW_ALIGN)
  int w;                   // real shard width
  int c0;                  // first global subject column of this shard
  int band;                // columns per band (64..512, divides wp)
  int nb;                  // bands per row = wp / band
  int evs;                 // event slots per (row, band) = band / 32; more spill to the ring
  uint32_t ev_spill_cap;
  uint64_t rd_seed, drop_seed;
  // Band-tiled layout: cell (r, c) of band b = c / band lives at ((b * n + r) * band + c % band),
  // so one band of all rows is one contiguous slab (the unit gm_s_band sweeps).
  uint8_t *table;          // [nb][n][band] stored cell bytes (s_narrow of S_CELL)
  uint32_t *tesc_in[2];    // [nb * n][S_ESC_IN] by tick parity: the first entries of each (band, row) list
  uint32_t *tesc[2];       // escape pools by tick parity: a list's entries beyond S_ESC_IN, from brec.w
  // Allocation is STRIPED: (band, row) list u allocates in stripe (band * n + row) & (stripes - 1),
  // a region of `region` entries with its own counter -- one global counter would serialise
  // every (band, row) of a crash-window tick on one address (4 M atomics at S-A: 25 ms)
  int esc_stripes;         // power of two
  unsigned long long *tesc_cnt;  // [2][esc_stripes] cells allocated per stripe this tick (zeroed a tick ahead)
  uint32_t tesc_region;    // entries per stripe
  size_t tesc_cap;         // entries per pool = esc_stripes * tesc_region
  uint8_t *msg;            // [nb][n][2][band/2] gossip payload nibbles, both tick parities of a (band, row) adjacent
  // escaped payload bytes (nibble 15): per (band, sender) of tick parity p the lanes holding escapes
  // write their 16 payload bytes h' into consecutive 16-byte slots of pesc[p] from the record's base,
  // in lane order (pesc_rec[p][band * n + sender] = {base, lane mask lo, lane mask hi, 0}, written
  // only by senders with escapes and read only where a receiver meets nibble 15)
  uint8_t *pesc[2];
  uint4 *pesc_rec[2];
  unsigned long long *pesc_cnt;  // [2][esc_stripes] slots allocated per stripe this tick
  uint32_t pesc_region;    // 16-byte slots per stripe
  uint32_t pesc_cap;       // 16-byte slots per pool
  int32_t *wtick;          // [n] tick each row's cells are relative to (last written)
  int32_t *inbox_cnt[2];   // [n] lists queued for each receiver, by delivery-tick parity
  int32_t *inbox[2];       // [n][S_KMAX] sender rows
  int32_t *hbctr;          // [n] MP1Node heartbeat counter (Member::heartbeat)
  int32_t *failed;         // [n] Member::bFailed
  uint4 *brec;             // [nb][n] per-(band, row) record after the sweep: .x/.y = present cells per 64-column
                           // chunk (band/64 bytes, rank-select), .z = bcnt word (S_BC_*), .w = the slice's escape-list
                           // word (S_EW_*, 0: none); rows adjacent = whole-line writes
  uint32_t *ev_band;       // [n][nb][evs] kind<<30 | subject id
  uint64_t *ev_spill;      // overflow: (logger<<32) | kind<<30 | subject id
  uint32_t *ev_spill_cnt;  // [1 + S_EV_STRIPES]: spill records, then the tick's total records in
                           // S_EV_STRIPES striped partial sums (one hot address would serialise)
  uint64_t *evcum;         // [n][nb] cumulative events since create: joins | removals << 32 (single writer per cell)
  uint32_t *mtraw;        // [n][S_MT_RAW] first mt19937 outputs of each row's S2 stream this tick
  int32_t *rowstat;        // [n][4]: lists delivered, present, numfailed, targets chosen
  int32_t *targets;        // [n][GM_FANOUT]
  uint32_t *err;
  // ---- column-sharded mode (shard_count > 1, or one shard forced by GM_FORCE_SHARD=1 to
  // rehearse the sharded protocol + RCCL on one GPU; see gm_s_draw / gm_s_accept)
  int shard_rank, shard_count;
  int sharded;
  int stub;                // diagnostics (gm_shard_stub): one shard alone on a device; draws landing in
                           // other shards' columns resolve to fresh column ix (a symmetric stand-in)
  // ---- join ramp (gm_config.init_mode 2, single context): node j starts at tick j/4
  // (Application.cpp:130, STEP_RATE 0.25) and is in the group from tick j/4 + 2 if the
  // introducer (node 0) answered its JOINREQ at j/4 + 1 (ran that tick: <= intro_until).
  // A column's heartbeats are stored offset by s_hbase(j) = 2(j/4 + 1) (0 for j = 0), so
  // every live node's own heartbeat still reads 2t-1 and the narrow cell applies.
  int ramp;
  int intro_until;
  int32_t *mecol;            // [n] ramp: myPos's column this tick (self, or the updateMyPos quirk's target)
  int32_t *selfadd;          // [S_SELFADD_CAP] ramp: rows that appended their own entry this tick
  uint32_t *selfadd_cnt;
  int32_t *xcnt;             // bound exchange buffer, chunk-major: [chunk][shard_count][2^xlog][2] (present,
                             //   numfailed) per shard and row (s_xc): a row chunk's slots of every rank are
                             //   contiguous, so each chunk's all-gather is one in-place ncclAllGather
  int32_t *status;           // bound exchange buffer [n][D]: resolved draws, MAX-allreduced
  int32_t *acc;              // [n][8]: targets so far, g[5], numpot, size
  int32_t *pending;          // [n] rows still drawing
  int32_t *npending;         // rows still drawing after the last accept round
  // bounded rounds (tick_sharded): pending list l = 1, 2 holds the rows left after round l-1
  // (ascending after gm_s_plist_sort: the same order on every rank); statusl[l] = the bound
  // exchange buffer [plist_cap[l]][D_l] of round l's draws, by list position. Index 0 unused.
  int plist_cap[3];
  int32_t *plist[3];
  uint32_t *plist_cnt[3];
  int32_t *statusl[3];
  // ---- msgcount analogue (gm_msgcount_record, single context; nullptr = off): per tick and
  // row, gossip entries sent (fresh entries x targets, before loss) and received (after loss),
  // EmulNet's sent_msgs / recv_msgs per entry message (EmulNet.cpp:111,172)
  uint32_t *mc_sent, *mc_recv;  // [mc_tmax][n]
  uint32_t *mc_fresh;           // [2][n] fresh entries of each row's payload, by tick parity
  uint32_t *mc_rdrop;           // [n] entries a row received after keyed loss (DROP band kernel)
  int mc_tmax;
  int kcap;                     // inbox slots used (S_KMAX; lowered only by the diagnostics env GM_INBOX_CAP)
  // fast path (B = 1024, gm_s_band_fast): the units it hands back to the general path this tick,
  // by tick parity (the count of tick t+1 is zeroed during tick t); nullptr: fast path off
  uint32_t *fb_cnt;             // [2]
  int2 *fb_list;                // [nb * n]: (band, row)
  int lag_hmin;                 // a present cell with h < lag_hmin sets GM_ERR_LAG: 3 (lag > 125 ticks, the
                                // encoding's limit); the diagnostics env GM_LAG_CAP=L (L >= 15) lowers it to lag > L
  // ---- round-5 fields, kept at the end: the band kernels are short-lived waves whose first scalar
  // loads come from this struct in the kernel arguments, and fields inserted above shifted their
  // offsets and the compiler's load grouping (S-A band kernels +7 %, profiles/r05/sa_regression/)
  int esc_dense;                // the pools are dense-equivalent (no run can overflow them); gm_pool_info
  int xlog;                     // column shards: log2 of the rows per exchange chunk (rows [c << xlog, (c + 1) << xlog))
  int xk;                       // exchange chunks = ceil(n / 2^xlog)
  // gm_s_pick0 (single context, B = 1024): rows whose first 16 S2 outputs do not finish their draw go
  // to this list, which gm_s_pick then takes from output 0 (nullptr: gm_s_pick takes every row)
  int32_t *pk_list;             // [n]
  uint32_t *pk_cnt;
};
