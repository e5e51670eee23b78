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
// One wave per node, everything in a ~4.8 KB LDS slice so 8 waves share a SIMD
// (the per-node work is short dependent-load chains + LDS atomics: latency is
// hidden by occupancy, and the instruction count per node is what bounds the
// kernel once it is):
//   1. loads issue together: the node's own list (one 8-byte entry per lane),
//      its inbox (sender indices), its 16 precomputed S2 outputs, then every
//      delivered list (V lanes per list, several lists per wave step);
//   2. merge into an open-addressing LDS table keyed by id (32-bit CAS claim +
//      ds_max of the heartbeat word), own entries first so they carry the
//      "own" bit, delivered entries filtered to fresh + not dropped;
//   3. self bump, then one sweep compacts the table in place into a dense
//      array (TREMOVE removals counted and logged on the way);
//   4. eviction to V only when the union exceeds V: an LDS histogram of the
//      heartbeat distance from the top finds the cut heartbeat; inside the cut
//      bucket a 6-bit radix histogram of the eviction keys and (rarely) an
//      exact min-selection pick the smallest keys -- no full sort;
//   5. the <= V kept entries are ranked by id (broadcast LDS compare) = the
//      id-sorted list, stored as one coalesced row; joins as a bit mask over it;
//   6. the gossip draw: the 16 precomputed S2 outputs resolved in parallel across
//      the wave (duplicates by shuffle-compares), the rare rest on scalars.
// Nodes with more than P_KSMALL delivered lists (Poisson tail, ~0.2 % at 12) do not fit
// the small table: the small kernel defers them to a worklist that the big
// kernel (1024-slot table) drains, and those with more than P_KP lists (~2e-5) to the
// huge kernel's (4096 slots): every delivered list is merged, as EmulNet delivers them all.
// Lists are double-buffered by tick parity: a receiver reads its senders' lists
// of tick t-1 directly, so no separate payload copy is written.
#include <algorithm>
#include <type_traits>
#include <cstdio>

#include "gm_device.h"
#include "gm_partial.h"

#define P_IDMASK 0x01FFFFFFu  // ids <= 2^25
#define P_OWN 0x80000000u     // table id-word flag: the id was in the node's own list
#define P_SELF 0x40000000u    // table id-word flag: the node's own entry
#define P_MISC_BYTES (64 * 4 + P_VMAX * 4 + P_VMAX * 4 + P_VMAX * 8)

// Lemire's rejection threshold 2^32 mod size for every list size 1..P_VMAX (a final list holds at
// most V <= P_VMAX entries), read by a scalar load instead of a 32-bit remainder per node
struct PThrTab {
  uint32_t v[P_VMAX + 1];
  constexpr PThrTab() : v() {
    for (uint32_t n = 1; n <= P_VMAX; n++) v[n] = (0u - n) % n;
  }
};
__constant__ PThrTab p_thr_tab = PThrTab();

template <int H>
struct PLds {
  static constexpr int bytes = H * 8 + P_MISC_BYTES;
};

// LDS hand-off between the lanes of ONE wave (every LDS region here is private to its wave):
// a wave's LDS instructions execute in issue order, so wavefront scope needs no lgkmcnt wait --
// only the compiler must not move LDS accesses across it (workgroup scope waited lgkmcnt(0)
// at each of the ~16 hand-offs of a node)
__device__ __forceinline__ void p_wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int p_age(int t, uint32_t hb) { return t - (int)((hb + 1u) >> 1); }
// p_age(t, hb) >= A as one compare: t - floor((hb+1)/2) >= A <=> hb < 2(t-A)+1 (heartbeats < 2^31)
__device__ __forceinline__ bool p_aged(int t, uint32_t hb, int A) { return (int)hb < 2 * (t - A) + 1; }

// eviction tie-break key (oracle op_evict_key): fmix32 of the id under a per-(tick, observer)
// seed -- a bijection, so distinct ids give distinct keys; oseed = (uint32)mix64(mix64(view_seed
// ^ t) ^ obs) is wave-uniform
__device__ __forceinline__ uint32_t p_evict_key(uint32_t oseed, uint32_t id) { return gm_fmix32(id ^ oseed); }

// wave-wide inclusive scan of ints on DPP: row_shr 1/2/4/8 scans each 16-lane row,
// row_bcast15 / row_bcast31 carry the row totals upward (lanes a DPP source does not
// reach keep the identity 0)
__device__ __forceinline__ int p_scan(int v, int) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);  // row_shr:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
  return v;
}

__device__ __forceinline__ int p_below(uint64_t bal) {  // set bits of bal below this lane
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
}

// exclusive wave prefix of small per-lane counts c < 2^BITS (ballot per bit + mbcnt)
template <int BITS>
__device__ __forceinline__ int p_excl(int c, int *total) {
  int pos = 0, tot = 0;
#pragma unroll
  for (int b = 0; b < BITS; b++) {
    const uint64_t bal = __ballot((c >> b) & 1);
    pos += p_below(bal) << b;
    tot += __builtin_popcountll(bal) << b;
  }
  *total = tot;
  return pos;
}

__device__ __forceinline__ uint64_t p_readlane64(uint64_t v, int l) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

// claim or find the slot of `id`, raise its heartbeat word. Every lane of the wave runs the probe
// loop (no divergent loop: its exec-mask bookkeeping was ~5 SALU per probe). A lane with nothing to
// insert (take false) points at its own word of the misc area (hist[lane], 2H words past tid),
// which holds P_TRASH while the lists merge: its CAS changes nothing and finds "its" id at once, and
// its max of 0 changes nothing (distinct words: no same-address serialisation). A lane that found
// its slot repeats an idempotent CAS. The merge claims bare ids (flags are ORed in after it), so one
// compare finds an id. Returns the slot (>= 2H for a lane that took nothing).
#define P_TRASH 0xFFFFFFFFu
template <int H>
__device__ __forceinline__ int p_insert(uint32_t *tid, bool take, uint32_t id, uint32_t hb, int lane) {
  // slot = low bits of id ^ id >> 9: view ids are uniform node indices, so this spreads them like a
  // multiplicative hash without its quarter-rate 32-bit multiply (the slot never shows in a result:
  // the table is compacted and ranked by id). Probing steps a byte offset: with the table at LDS
  // address 0 the slot's address is the offset
  const uint32_t idw = take ? id : P_TRASH;
  uint32_t a = take ? ((id ^ (id >> 9)) & (H - 1)) * 4 : 8 * H + 4 * lane;
  for (;;) {  // claim-or-compare in one LDS op
    const uint32_t cur = atomicCAS((uint32_t *)((unsigned char *)tid + a), 0u, idw);
    const bool more = cur != 0 && cur != idw;
    if (!__ballot(more)) break;
    if (more) a = (a + 4) & (4 * H - 1);
  }
  atomicMax((uint32_t *)((unsigned char *)tid + a + (take ? 4 * H : 0)), take ? hb : 0u);
  return (int)(a >> 2);
}

// owning row shard of node d: contiguous balanced ranges [n*g/G, n*(g+1)/G), boundaries
// in shard_n0[0..G]; a float estimate is off by at most one, two compares fix it
__device__ __forceinline__ int p_owner(const PState &s, int d) {
  int g = min(s.G - 1, max(0, (int)((float)d * (float)s.G / (float)s.n)));
  if (g + 1 < s.G && s.shard_n0[g + 1] <= d) g++;
  if (g > 0 && s.shard_n0[g] > d) g--;
  return g;
}

// A node's independent loads, issued together before any branch on them (one memory
// round trip instead of a chain): crash flag, inbox count, own list, inbox row, S2
// outputs, heartbeat counter. `nin` = inbox lanes to fetch (the kernel's list bound).
struct PPre {
  int failed, k, hbctr;
  uint64_t own;
  int sv;
  uint32_t raw0;  // S2 output d on lane roff + d
  int roff;
};
__device__ __forceinline__ PPre p_preload(const PState &s, int t, const uint32_t *mtraw, int li, int lane, int nin) {
  const int par = t & 1, V = s.V;
  PPre p;
  p.failed = s.failed[li];
  p.k = s.inbox[par][(size_t)li * P_KMAX];
  p.hbctr = s.hbctr[li];
  p.own = lane < V ? s.lists[((size_t)(par ^ 1) * s.rows + li) * V + lane] : 0ull;
  p.sv = lane < nin ? s.inbox[par][(size_t)li * P_KMAX + 1 + lane] : 0;
  p.raw0 = lane < 16 ? mtraw[(size_t)li * 16 + lane] : 0u;
  p.roff = 0;
  return p;
}

// The small kernel's next node, prefetched while the wave works on the current one: ONE
// packed word per lane -- inbox ids on lanes 0..15, S2 outputs on 16..31, crash flag / inbox
// count / heartbeat counter on lanes 32 / 33 / 34 -- by an LDS-DMA load (global_load_lds:
// no VGPR holds it across the node, and no register copy at the loop edge waits for it) into
// the wave's P_PF_BYTES area. The compiler does not see this load (inline asm): every node
// starts with vmcnt(0), which retires the DMA its predecessor issued.
#define P_PF_LANES 40
#define P_PF_BYTES (P_PF_LANES * 4)
__device__ __forceinline__ void p_prefetch(const PState &s, int t, const uint32_t *mtraw, int li, int lane,
                                           uint32_t lds) {
  const int par = t & 1;
  const uint32_t *a = lane < 16   ? (const uint32_t *)s.inbox[par] + (size_t)li * P_KMAX + 1 + lane
                      : lane < 32 ? mtraw + (size_t)li * 16 + (lane - 16)
                      : lane == 32 ? (const uint32_t *)s.failed + li
                      : lane == 33 ? (const uint32_t *)s.inbox[par] + (size_t)li * P_KMAX
                                   : (const uint32_t *)s.hbctr + li;
  if (lane < P_PF_LANES) {
    uint32_t keep;  // m0 = the LDS destination (lane l writes dword l); the reads of the area
                    // by the node before are waited for first
    asm volatile(
        "s_waitcnt lgkmcnt(0)\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
        "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(a), "s"(lds)
        : "memory");
  }
}
template <int VF>
__device__ __forceinline__ PPre p_unpack_next(const PState &s, int t, int li, uint32_t pv, int lane) {
  const int V = VF ? VF : s.V;
  PPre p;
  p.failed = (int)__builtin_amdgcn_readlane(pv, 32);
  p.k = (int)__builtin_amdgcn_readlane(pv, 33);
  p.hbctr = (int)__builtin_amdgcn_readlane(pv, 34);
  p.own = lane < V ? s.lists[((size_t)((t & 1) ^ 1) * s.rows + li) * V + lane] : 0ull;
  p.sv = lane < 16 ? (int)pv : 0;
  p.raw0 = pv;
  p.roff = 16;
  return p;
}

// One node's tick on one wave. li: the node's local row (global index n0 + li);
// pre.k: lists queued for it this tick.
// MC: the msgcount-recording instantiation (gm_msgcount_record); the others carry no trace of it
// RM: lists of other row shards may be delivered (sharded contexts); without, every sender is a
// local row and the list loads carry no branch
// VF: the view width when known at compile time (32: S-C), 0 = s.V at run time
template <int H, bool BIG, bool MC, bool RM = true, int VF = 0>
__device__ __forceinline__ void p_node(const PState &s, int t, const PPre &pre, int li, int lane, unsigned char *base,
                                       int chunk, int r0) {
  int k = pre.k;
  const int i = s.n0 + li;  // global node index (ids, keys, seeds, targets)
  constexpr int TS = H / 64;                          // table slots per lane
  constexpr int KK = H == P_HH ? P_KMAX : BIG ? P_KP : P_KSMALL;  // lists merged at most
  constexpr int DS = ((1 + KK) * P_VMAX + 63) / 64;   // dense entries per lane
  constexpr int NSTEP = (KK + 1) / 2;                 // list-load steps (>= 2 lists per step)
  using mask_t = typename std::conditional<(DS > 32), uint64_t, uint32_t>::type;  // one bit per dense slot
  uint32_t *tid = (uint32_t *)base;
  uint32_t *thb = tid + H;
  uint32_t *hist = thb + H;
  uint32_t *kid = hist + 64;
  uint32_t *khb = kid + P_VMAX;
  uint64_t *fin = (uint64_t *)(khb + P_VMAX);
  const int V = VF ? VF : s.V;
  const int par = t & 1;
  const uint64_t *prev = s.lists + (size_t)(par ^ 1) * s.rows * V;
  uint64_t *cur = s.lists + (size_t)par * s.rows * V;

  if (lane == 0) s.inbox[par][(size_t)li * P_KMAX] = 0;  // consumed; the append target of tick t+1
  const int kmax = min(KK, s.kcap);  // lists stored in the inbox row (the append counter may count more)
  if (k > kmax) {  // the huge kernel takes up to the inbox capacity; beyond it the tick is void
    if (lane == 0) atomicOr(s.err, GM_ERR_INBOX);
    k = kmax;  // never read sender slots that were not written
  }
  // ---- 1. loads (the independent ones arrived with `pre`)
  const uint64_t own = pre.own;
  int sv = lane < k ? pre.sv : 0x7FFFFFFF;  // list rows
  const uint32_t raw0 = pre.raw0;
  const int hbnew = pre.hbctr + 1;
  {  // clear the table (both word arrays are contiguous)
    uint4 *z = (uint4 *)tid;
#pragma unroll
    for (int q = 0; q < H / 128; q++) z[lane + 64 * q] = make_uint4(0, 0, 0, 0);
    tid[2 * H + lane] = P_TRASH;  // hist[lane]: the lane's trash word while the lists merge (p_insert)
  }
  const int kk = min(k, KK);
  // lists per load step (per), entry (l) and list slot (jo) of this lane; V = 32 (S-C) takes the
  // shifts instead of three integer divisions. The step's per-list values come by ds_bpermute
  // (the LDS port) rather than two readlanes + a select: VALU issue is what bounds this kernel
  const bool v32 = V == P_VMAX;
  int per, l, jo;
  if (v32) {
    per = 2;
    l = lane & 31;
    jo = lane >> 5;
  } else {
    per = 64 / V;
    l = lane % V;
    jo = lane / V;
  }
  auto step_val = [&](int v, int st) -> int { return __shfl(v, min(st * per + jo, 63), 64); };  // v of lane st * per + jo
  uint64_t dv[NSTEP];
#pragma unroll
  for (int st = 0; st < NSTEP; st++) {
    dv[st] = 0;
    if (st * per >= kk) continue;  // wave-uniform: no list in this step (k ~ 5 of up to 12 at S-C; -1.1 %,
                                   // profiles/r05/ab7/)
    const int j = st * per + jo;
    const bool ok = jo < per && j < kk;
    const int sn = step_val(sv, st);
    uint64_t e = 0;
    if (ok && (!RM || sn < s.nloc)) {
      e = prev[(size_t)sn * V + l];
    } else if (RM && ok) {  // a list another shard sent at t-1: wire entry id | (2(t-1)-1 - hb) << 25
      const uint32_t w = s.recv_list[par ^ 1][(size_t)(sn - s.nloc) * V + l];
      if (w) e = ((uint64_t)(w & ((1u << P_WIRE_IDBITS) - 1)) << 32) | (uint32_t)(2 * t - 3 - (int)(w >> P_WIRE_IDBITS));
    }
    dv[st] = e;
  }
  // global sender index of each list (the drop keys), after the list loads are in flight
  const int sg = lane < k ? (!RM || sv < s.nloc ? s.n0 + sv : s.rsrc[par ^ 1][sv - s.nloc]) : 0x7FFFFFFF;
  // drop keys: one (t_send, src, dst) hash per delivered list, lane j for list j
  const bool dropping = s.drop_pct >= 0;
  const bool mc = MC && t < s.mc_tmax;  // msgcount recording (wave-uniform)
  int nrecv = 0;                                           // delivered entries kept (msgcount)
  uint32_t pairv = 0;  // low word of mix64(seed ^ t_send << 48 ^ src << 24 ^ dst)
  if (dropping)
    pairv = (uint32_t)gm_mix64(s.drop_seed ^ ((uint64_t)(uint32_t)(t - 1) << 48) ^ ((uint64_t)(uint32_t)sg << 24) ^
                               (uint64_t)(uint32_t)i);
  const uint32_t dthr = gm_drop_thresh(s.drop_pct);
  p_wsync();
  // ---- 2. merge: own entries first (their slots get P_OWN after the merge), then the delivered lists
  int hslot = -1;
  const uint32_t self_id = (uint32_t)(i + 1);
  hslot = p_insert<H>(tid, own != 0, (uint32_t)(own >> 32), (uint32_t)own, lane);
  p_wsync();
  {
    const uint32_t tfresh = (uint32_t)max(0, 2 * t - 11);  // hb >= 2t-11 <=> (t-1) - (hb+1)/2 < TFAIL
#pragma unroll
    for (int st = 0; st < NSTEP; st++) {
      if (st * per >= kk) continue;  // wave-uniform
      const uint64_t e = dv[st];
      bool take = e != 0 && (uint32_t)e >= tfresh;
      const uint32_t id = (uint32_t)(e >> 32);
      if (dropping) {  // per-entry drops keyed by (t_send, src, dst, id-1): lost iff the top 16 bits of
        // fmix32(pair ^ (id-1)) are below the threshold
        const uint32_t pair = (uint32_t)step_val((int)pairv, st);
        take = take && (gm_fmix32(pair ^ (id - 1)) >> 16) >= dthr;
      }
      (void)p_insert<H>(tid, take, id, (uint32_t)e, lane);
      if (mc) nrecv += __builtin_popcountll(__ballot(take));
    }
  }
  atomicOr(&tid[hslot], own != 0 ? P_OWN : 0u);  // after the merge: its probes compare bare ids (a lane
                                                 // with no own entry ORs 0 into its trash word)
  p_wsync();
  // ---- 3. self bump (heartbeat++; myPos->setheartbeat(heartbeat++)), then sweep + compaction
  {
    const uint64_t sb = __ballot(own != 0 && (uint32_t)(own >> 32) == self_id);
    int hs;
    if (sb) {
      hs = __builtin_amdgcn_readlane(hslot, __builtin_ctzll(sb));
    } else {  // cannot happen for a live node (the oracle aborts): flag, and re-insert self
      hs = 0;
      if (lane == 0) {
        atomicOr(s.err, GM_ERR_SELF);
        hs = p_insert<H>(tid, true, self_id, 1u, lane);  // self is in no own slot: its id is bare
      }
      hs = __builtin_amdgcn_readfirstlane(hs);
    }
    if (lane == 0) {
      thb[hs] = (uint32_t)hbnew;
      tid[hs] |= P_SELF | P_OWN;
      s.hbctr[li] = hbnew + 1;
    }
  }
  p_wsync();
  uint32_t *evr = s.ev + (size_t)li * 2 * V;
  int m, removed, nrem;
  {
    uint32_t w[TS], hh[TS];
#pragma unroll
    for (int q = 0; q < TS / 4; q++) {
      const uint4 a = ((const uint4 *)tid)[lane * (TS / 4) + q];
      const uint4 b = ((const uint4 *)thb)[lane * (TS / 4) + q];
      w[4 * q] = a.x; w[4 * q + 1] = a.y; w[4 * q + 2] = a.z; w[4 * q + 3] = a.w;
      hh[4 * q] = b.x; hh[4 * q + 1] = b.y; hh[4 * q + 2] = b.z; hh[4 * q + 3] = b.w;
    }
    using tmask_t = typename std::conditional<(TS > 32), uint64_t, uint32_t>::type;  // one bit per table slot
    constexpr int CB = TS <= 8 ? 4 : TS <= 16 ? 5 : TS <= 32 ? 6 : 7;               // bits of a per-lane slot count
    // alive <=> present and not aged past TREMOVE <=> hb >= xa: every present entry has hb >= 1
    // (heartbeats start at 2t-1 >= 1; hb < 2^31) and an empty slot holds hb 0, so one compare per
    // slot gives the alive bit; removals = present - alive (rare: tested once per row)
    const uint32_t xa = (uint32_t)max(2 * (t - GM_TREMOVE) + 1, 1);
    // the alive count by compares whose results feed carry-ins (v_cmp + v_addc per slot), not by a
    // per-lane bit mask built and popcounted (~4 VALU per slot); the mask is built only in the rare
    // removal branch
    int rcount = 0, na = 0;
#pragma unroll
    for (int u = 0; u < TS; u++) {
      na += hh[u] >= xa;
      rcount += (int)min(w[u], 1u);
    }
    rcount -= na;
    int tot;
    removed = nrem = 0;
    if (__ballot(rcount != 0)) {  // rare: TREMOVE removals in this row
      tmask_t alive = 0, rown = 0;
#pragma unroll
      for (int u = 0; u < TS; u++) alive |= (tmask_t)(hh[u] >= xa) << u;
#pragma unroll
      for (int u = 0; u < TS; u++) rown |= (tmask_t)((w[u] >> 31) & (uint32_t)!((alive >> u) & 1)) << u;
      (void)p_excl<CB>(rcount, &removed);
      const int ro = __builtin_popcountll(rown);
      int rpos = p_excl<CB>(ro, &nrem);
      if (nrem) {  // REMOVE events of the node's own entries, from the back of its event row
#pragma unroll
        for (int u = 0; u < TS; u++)
          if ((rown >> u) & 1) evr[2 * V - 1 - rpos++] = (P_EV_REMOVE << 30) | (w[u] & P_IDMASK);
      }
    }
    // the alive slots' dense positions: an inclusive DPP scan of the per-lane counts (A/B on one box
    // against p_excl's ballot per count bit: -0.3 %, profiles/r04/sc_sweep/)
    const int incl = p_scan(na, lane);
    tot = __builtin_amdgcn_readlane(incl, 63);
    int pos = incl - na;
    m = tot;
    // every slot is stored: dead ones to a per-lane slot of [H-64, H), past the dense
    // range (m <= (1+KK)V+1 < H-64) and free of bank conflicts
#pragma unroll
    for (int u = 0; u < TS; u++) {
      const bool a = hh[u] >= xa;
      const int at = a ? pos : H - 64 + lane;
      tid[at] = w[u];
      thb[at] = hh[u];
      pos += a;
    }
  }
  p_wsync();
  // ---- 4. dense entries e = s*64 + lane; eviction to V
  // only the first dm = ceil(m / 64) of the DS per-lane slots hold entries (m is wave-uniform):
  // every per-slot loop below skips the rest with a scalar branch
  const int dm = (m + 63) >> 6;
  uint32_t dw[DS], dh[DS];
#pragma unroll
  for (int q = 0; q < DS; q++) {  // DS*64 < H: the reads stay inside the table
    dw[q] = dh[q] = 0u;
    if (q < dm) {
      const int e = q * 64 + lane;
      const uint32_t a = tid[e], b = thb[e];
      dw[q] = e < m ? a : 0u;
      dh[q] = e < m ? b : 0u;
    }
  }
  mask_t keep = 0;
  if (m <= V) {
#pragma unroll
    for (int q = 0; q < DS; q++)
      if (q < dm && dw[q]) keep |= (mask_t)1 << q;
  } else {
    // heartbeat distance from the top (2t-1 = this tick's self heartbeat); alive entries have
    // age < TREMOVE, i.e. distance <= 40; every heartbeat is odd (2k - 1, MP1Node.cpp:412-415), so the
    // distances are even. The cut class (the smallest distance whose cumulative count of candidates
    // -- self excluded -- reaches V - 1) is found by ballots, class by class: the candidates crowd into
    // ~4 classes, so a 64-bin LDS histogram took its atomics ~58 lanes to one address at a time
    // (serialised in the LDS pipe: ~4 ms of the S-C tick, profiles/r06/sc_sections/)
    const int top = 2 * t - 1;
    const int need = V - 1;  // self is always kept
    int dd[DS];              // the slot's distance class, 64 = no candidate (empty, or self)
    bool odd = false;
#pragma unroll
    for (int q = 0; q < DS; q++) {
      dd[q] = 64;
      if (q < dm && dw[q] && !(dw[q] & P_SELF)) dd[q] = min(max(top - (int)dh[q], 0), 63);
      odd |= dd[q] & 1;
    }
    if (__ballot(odd) && lane == 0) atomicOr(s.err, GM_ERR_PARITY);  // cannot happen: heartbeats are odd
    int dcut = 62, before = 0, bsz = 0;
    for (int d = 0; d <= 62; d += 2) {  // wave-uniform; ends within the populated classes (m - 1 > need)
      int c = 0;
#pragma unroll
      for (int q = 0; q < DS; q++)
        if (q < dm) c += __builtin_popcountll(__ballot(dd[q] == d));
      if (before + c >= need) {
        dcut = d;
        bsz = c;
        break;
      }
      before += c;
    }
    const int needb = need - before;  // 1 <= needb <= bsz
    mask_t bucket = 0;
#pragma unroll
    for (int q = 0; q < DS; q++) {
      if (q >= dm) continue;
      keep |= (mask_t)(((dw[q] & P_SELF) != 0) | (dd[q] < dcut)) << q;
      bucket |= (mask_t)(dd[q] == dcut) << q;
    }
    if (needb == bsz) {
      keep |= bucket;
    } else {
      // the needb smallest eviction keys of the bucket: 6-bit radix on the top bits,
      // then exact min-selection inside the cut bin
      const uint32_t oseed = (uint32_t)gm_mix64(gm_mix64(s.view_seed ^ (uint64_t)(uint32_t)t) ^ (uint64_t)(uint32_t)i);
      uint32_t key[DS];
#pragma unroll
      for (int q = 0; q < DS; q++) {
        key[q] = ~0u;
        if (q < dm && __ballot((bucket >> q) & 1)) key[q] = ((bucket >> q) & 1) ? p_evict_key(oseed, dw[q] & P_IDMASK) : ~0u;
      }
      p_wsync();
      hist[lane] = 0;
      p_wsync();
#pragma unroll
      for (int q = 0; q < DS; q++)
        if (q < dm) atomicAdd(((bucket >> q) & 1) ? &hist[key[q] >> 26] : &tid[H - 64 + lane], 1u);
      p_wsync();
      const int c = (int)hist[lane];
      const int inc = p_scan(c, lane);
      const uint64_t over2 = __ballot(inc >= needb);
      const int bcut = __builtin_ctzll(over2);
      const int before2 = __builtin_amdgcn_readlane(inc - c, bcut);
      const int bsz2 = __builtin_amdgcn_readlane(c, bcut);
      int needc = needb - before2;  // 1 <= needc <= bsz2
      mask_t cand = 0;
#pragma unroll
      for (int q = 0; q < DS; q++) {
        if (q >= dm) continue;
        const mask_t b = (bucket >> q) & 1;
        const int bin = (int)(key[q] >> 26);
        keep |= (b & (mask_t)(bin < bcut)) << q;
        cand |= (b & (mask_t)(bin == bcut)) << q;
      }
      if (needc == bsz2) {
        keep |= cand;
      } else {
        for (; needc > 0; needc--) {  // take the smallest remaining candidate key (keys are distinct)
          uint32_t mn = ~0u;
#pragma unroll
          for (int q = 0; q < DS; q++)
            if (q < dm && ((cand >> q) & 1)) mn = min(mn, key[q]);
#pragma unroll
          for (int o = 32; o >= 1; o >>= 1) mn = min(mn, (uint32_t)__shfl_xor((int)mn, o, 64));
#pragma unroll
          for (int q = 0; q < DS; q++)
            if (q < dm && ((cand >> q) & 1) && key[q] == mn) {
              keep |= (mask_t)1 << q;
              cand &= ~((mask_t)1 << q);
            }
        }
      }
    }
  }
  // ---- 5. compact the kept entries (<= V), rank them by id
  int cnt = 0;
  p_wsync();  // the eviction histogram is dead: it takes the stores of the entries not kept
#pragma unroll
  for (int q = 0; q < DS; q++) {
    if (q >= dm) break;
    const bool kq = (keep >> q) & 1;
    const uint64_t bal = __ballot(kq);
    const int p = cnt + p_below(bal);
    // id word rotated left by 2: id << 2 | own << 1 | self (ids < 2^25, bits 25..29 clear),
    // so the rank below compares whole words
    *(kq ? kid + p : hist + lane) = __builtin_amdgcn_alignbit(dw[q], dw[q], 30);
    *(kq ? khb + p : hist + lane) = dh[q];
    cnt += __builtin_popcountll(bal);
  }
  if (lane >= cnt && lane < P_VMAX) kid[lane] = ~0u;  // sentinels rank after every real entry
  p_wsync();
  {
    // entry e = lane % 32 on both half-waves; each half compares it against half of the
    // kept ids (cnt <= P_VMAX = 32), the two partial ranks add across the halves
    static_assert(P_VMAX == 32, "the id rank splits a wave into two half-waves of P_VMAX lanes");
    const int e = lane & (P_VMAX - 1);
    const uint32_t mw = e < cnt ? kid[e] : 0u, mh = e < cnt ? khb[e] : 0u;
    const uint32_t myid = mw >> 2;
    int rank = 0;
    const uint4 *kv = (const uint4 *)kid + (lane >> 5) * (P_VMAX / 8);
#pragma unroll
    for (int q = 0; q < P_VMAX / 8; q++) {  // broadcast reads, 4 ids each (ids are distinct)
      const uint4 v = kv[q];
      rank += (v.x < mw) + (v.y < mw) + (v.z < mw) + (v.w < mw);
    }
    rank += __shfl_xor(rank, 32, 64);
    p_wsync();
    if (lane < cnt) {
      fin[rank] = ((uint64_t)myid << 32) | mh;
      kid[rank] = mw;
    }
  }
  p_wsync();
  const uint64_t x = lane < cnt ? fin[lane] : 0ull;
  const uint32_t f = lane < cnt ? kid[lane] : 0u;
  if (lane < V) cur[(size_t)li * V + lane] = x;
  // joins (ascending id) from the front of the event row
  const uint64_t jb = __ballot(lane < cnt && !(f & 2u));  // rotated P_OWN
  const int nj = __builtin_popcountll(jb);
  // joins (ascending id): a mask over the final list (ev_jm)
  const int numfailed = removed + __builtin_popcountll(__ballot(lane < cnt && p_aged(t, (uint32_t)x, GM_TFAIL)));
  // ---- 6. gossip draw over the final list (MP1Node.cpp:449-489)
  const int numpot = cnt - 1 - numfailed;
  const int target = min(GM_FANOUT, numpot);
  int ng = 0;
  uint32_t *gl = hist;  // the chosen targets in draw order (hist is free after the compaction)
  if (numpot > 0) {
    const uint32_t size = (uint32_t)cnt;
    const uint32_t thr = p_thr_tab.v[size];  // size = cnt <= V <= P_VMAX
    {  // the 16 precomputed outputs in parallel, output d on lane d: it is taken iff Lemire
       // accepts it, the drawn entry is not "me" and not aged, and no earlier such output drew
       // the same id (that one was taken, or repeated a taken one) -- the reference's loop
      // every 16-lane group g evaluates all 16 outputs (output d = lane % 16) and tests
      // d against the earlier outputs q in [4g, 4g + 4); the groups' results are OR-ed
      const int d = lane & 15, g4 = (lane >> 4) * 4;
      const uint32_t rawd = __shfl(raw0, pre.roff + d, 64);
      const uint64_t prod = (uint64_t)rawd * size;
      const int ixv = (int)(prod >> 32);
      const uint32_t elo = __shfl((uint32_t)x, ixv, 64), ehi = __shfl((uint32_t)(x >> 32), ixv, 64);
      const int c = (int)ehi - 1;
      const bool okd = (uint32_t)prod >= thr && c != i && !p_aged(t, elo, GM_TFAIL);
      const int cv = okd ? c : -2;
      int dup = 0;
#pragma unroll
      for (int j = 0; j < 4; j++) dup |= (g4 + j < d) & (__shfl(cv, g4 + j, 64) == cv);
      uint64_t db = __ballot(dup);  // OR of the four groups' verdicts, bit d
      db |= db >> 32;
      db |= db >> 16;
      dup = (int)((uint32_t)db >> d) & 1;
      const bool ok = lane < 16 && okd;
      const bool acc = ok && !dup;
      const uint64_t ab = __ballot(acc);
      const int rk = p_below(ab);
      ng = min(__builtin_popcountll(ab), target);
      gl[acc && rk < target ? rk : 16 + lane] = (uint32_t)c;  // others: trash words past the targets
    }
    if (ng < target) {  // rare: more outputs, from the lazy generator in the (free) table region
      p_wsync();
      int g0 = -1, g1 = -1, g2 = -1, g3 = -1, g4 = -1;
      if (ng > 0) g0 = (int)__builtin_amdgcn_readfirstlane(gl[0]);
      if (ng > 1) g1 = (int)__builtin_amdgcn_readfirstlane(gl[1]);
      if (ng > 2) g2 = (int)__builtin_amdgcn_readfirstlane(gl[2]);
      if (ng > 3) g3 = (int)__builtin_amdgcn_readfirstlane(gl[3]);
      GmLazyMT mt;
      bool done = false;
      for (int batch = 1; !done; batch++) {
        if (batch > (1 << 16)) {
          if (lane == 0) atomicOr(s.err, GM_ERR_DRAWS);
          break;
        }
        if (lane == 0 && batch == 1) {
          mt.seed(tid, gm_rd_seed(s.rd_seed, t, i + 1));
          for (int q = 0; q < 16; q++) (void)mt.next();
        }
        uint32_t raw = 0;
        for (int q = 0; q < 16; q++) {
          uint32_t o = 0;
          if (lane == 0) o = mt.next();
          o = __builtin_amdgcn_readfirstlane(o);
          if (lane == q) raw = o;
        }
        const uint64_t prod = (uint64_t)raw * size;
        const int ix = (int)(prod >> 32);
        uint64_t mk = __ballot(lane < 16 && (uint32_t)prod >= thr);
        while (mk && !done) {
          const int d = __builtin_ctzll(mk);
          mk &= mk - 1;
          const int ixd = __builtin_amdgcn_readlane(ix, d);
          const uint64_t e = p_readlane64(x, ixd);
          const int c = (int)(e >> 32) - 1;
          if (c == i) continue;                                    // "me"
          if (p_aged(t, (uint32_t)e, GM_TFAIL)) continue;           // age >= TFAIL
          if ((ng > 0 && g0 == c) || (ng > 1 && g1 == c) || (ng > 2 && g2 == c) || (ng > 3 && g3 == c)) continue;
          if (ng == 0) g0 = c;
          else if (ng == 1) g1 = c;
          else if (ng == 2) g2 = c;
          else if (ng == 3) g3 = c;
          else g4 = c;
          ng++;
          if (ng >= target) done = true;
        }
      }
      p_wsync();
      if (lane < ng) gl[lane] = (uint32_t)(lane == 0 ? g0 : lane == 1 ? g1 : lane == 2 ? g2 : lane == 3 ? g3 : g4);
    }
  }
  p_wsync();
  // ---- sends: one parallel round of inbox appends, one lane per local target. A target owned by
  // another row shard is only recorded (targets / rowstat): gm_p_pack builds the exchange records from
  // them and this tick's list after the chunk (no record written per (sender, shard) here)
  const int dst = lane < ng ? (int)gl[lane] : 0;
  const int owner = (s.G > 1 && lane < ng) ? p_owner(s, dst) : s.rank;
  if (lane < ng) {
    s.targets[(size_t)li * GM_FANOUT + lane] = dst;
    if (owner == s.rank) {
      int32_t *row = s.inbox[par ^ 1] + (size_t)(dst - s.n0) * P_KMAX;  // count and slots share a line
      const int slot = atomicAdd(row, 1);
      if (slot < s.kcap) row[1 + slot] = li;
      else atomicOr(s.err, GM_ERR_INBOX);
    }
  }
  if (lane < 4) s.rowstat[(size_t)li * 4 + lane] = lane == 0 ? kk : lane == 1 ? cnt : lane == 2 ? numfailed : ng;
  if (lane == 0) s.ev_cnt[li] = nj | (nrem << 16);
  if (lane == 1) s.ev_jm[li] = (uint32_t)jb;  // lanes < cnt <= 32
  if (mc && lane == 0) {  // entries sent = fresh entries of the final list x targets (MP1Node.cpp:372-375)
    s.mc_sent[(size_t)t * s.nloc + li] = (uint32_t)(ng * (cnt - (numfailed - removed)));
    s.mc_recv[(size_t)t * s.nloc + li] = (uint32_t)nrecv;
  }
}

// crashed node: frozen (its list carried to this tick's buffer unchanged), inbox dropped
__device__ __forceinline__ void p_frozen(const PState &s, int t, int li, int lane) {
  const int par = t & 1, V = s.V;
  if (lane < V) s.lists[((size_t)par * s.rows + li) * V + lane] = s.lists[((size_t)(par ^ 1) * s.rows + li) * V + lane];
  if (lane < 4) s.rowstat[(size_t)li * 4 + lane] = 0;
  if (lane == 0) {
    s.inbox[par][(size_t)li * P_KMAX] = 0;
    s.ev_cnt[li] = 0;
    s.ev_jm[li] = 0;
  }
}

// rows [r0, r1) = chunk `chunk` of this shard's nodes
template <bool MC, bool RM, int VF>
__device__ __forceinline__ void p_small_node(const PState &s, int t, const PPre &pre, int li, int lane,
                                             unsigned char *base, int chunk, int r0) {
  if (pre.failed) {
    p_frozen(s, t, li, lane);
    return;
  }
  if (pre.k > P_KSMALL) {  // deferred to gm_p_tick_big (<= P_KP lists) or gm_p_tick_huge
    if (lane == 0) {
      if (pre.k <= P_KP) s.big[r0 + atomicAdd(&s.big_cnt[chunk], 1)] = li;
      else s.huge[r0 + atomicAdd(&s.huge_cnt[chunk], 1)] = li;
    }
    return;
  }
  p_node<P_HS, false, MC, RM, VF>(s, t, pre, li, lane, base, chunk, r0);
}

// P_NPW consecutive nodes per wave: each node's loads are prefetched during the node before it
// (p_prefetch), so a node starts with one global round trip (its delivered lists) instead of two.
// Held to 8 waves per SIMD (64 VGPRs; the loop keeps more live otherwise, and some SGPRs spill to
// VGPR lanes: ~40 more VALU per node, still faster than one node per wave: 26.1 vs 27.5 ms).
// P_SWG = 1 wave per workgroup: a finished wave releases its LDS slice at once (with 4 waves per
// workgroup the slice waited for the workgroup's last wave: 23.5 -> 22.8 ms)
template <bool MC, bool RM, int VF>
__global__ __launch_bounds__(64 * P_SWG) __attribute__((amdgpu_waves_per_eu(8, 8))) void gm_p_tick_small_pf(
    PState s, int t, const uint32_t *mtraw, int chunk, int r0, int r1, int npw) {
  // static LDS: its addresses are compile-time constants (offsets fold into the LDS instructions)
  __shared__ __align__(16) unsigned char p_smem[P_SWG * (PLds<P_HS>::bytes + P_PF_BYTES)];
  const int wave = P_SWG == 1 ? 0 : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int l0 = r0 + (blockIdx.x * P_SWG + wave) * npw;
  if (l0 >= r1) return;  // whole wave; no workgroup barrier in this kernel
  unsigned char *base = p_smem + (size_t)wave * PLds<P_HS>::bytes;
  const int l1 = min(r1, l0 + npw);
  uint32_t *pf = (uint32_t *)(p_smem + P_SWG * (size_t)PLds<P_HS>::bytes + (size_t)wave * P_PF_BYTES);
  const uint32_t pfa =
      __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(__attribute__((address_space(3))) uint32_t *)pf);
  p_prefetch(s, t, mtraw, l0, lane, pfa);
  for (int li = l0; li < l1; li++) {
    // the kernel arguments and the lane index pass through empty asm each node, so the
    // compiler re-derives what it needs per node instead of hoisting every address and
    // lane-dependent value out of the loop (that held 120 VGPRs live: occupancy 4).
    // (s is the first kernel argument: it sits at offset 0 of the kernarg segment)
    const __attribute__((address_space(4))) PState *ka =
        (const __attribute__((address_space(4))) PState *)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(ka));
    const PState &ss = *(const PState *)ka;
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int tt = t, cc = chunk, rr = r0;
    const uint32_t *mt = mtraw;
    // the node before is done except for its stores: retire them (and, for the compiler's
    // bookkeeping, every load it issued), so no stale pending load makes it wait on the DMA
    // issued next
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    asm volatile("" ::: "memory");       // the prefetch area is read only after the wait
    const uint32_t pv = ln < P_PF_LANES ? pf[ln] : 0u;
    if (li + 1 < l1) p_prefetch(ss, tt, mt, li + 1, ln, pfa);
    const PPre pre = p_unpack_next<VF>(ss, tt, li, pv, ln);
    p_small_node<MC, RM, VF>(ss, tt, pre, li, ln, base, cc, rr);
  }
}

// drains the worklist gm_p_tick_small filled (a fixed grid; every wave exits when the list is done)
template <bool MC>
__global__ __launch_bounds__(256, 3) void gm_p_tick_big(PState s, int t, const uint32_t *mtraw, int chunk, int r0) {
  extern __shared__ __align__(16) unsigned char p_smem[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int nbig = s.big_cnt[chunk];
  for (int w = blockIdx.x * 4 + wave; w < nbig; w += gridDim.x * 4) {
    const int li = s.big[r0 + w];
    const PPre pre = p_preload(s, t, mtraw, li, lane, P_KMAX - 1);
    p_node<P_HB, true, MC>(s, t, pre, li, lane, p_smem + (size_t)wave * PLds<P_HB>::bytes, chunk, r0);
  }
}

// drains the nodes with more than P_KP lists (Poisson tail: ~2e-5 of the nodes at S-C), one wave per
// workgroup for the 33 KB table
template <bool MC>
__global__ __launch_bounds__(64) void gm_p_tick_huge(PState s, int t, const uint32_t *mtraw, int chunk, int r0) {
  extern __shared__ __align__(16) unsigned char p_smem[];
  const int lane = threadIdx.x & 63;
  const int nh = s.huge_cnt[chunk];
  for (int w = blockIdx.x; w < nh; w += gridDim.x) {
    const int li = s.huge[r0 + w];
    const PPre pre = p_preload(s, t, mtraw, li, lane, P_KMAX - 1);
    p_node<P_HH, true, MC>(s, t, pre, li, lane, p_smem, chunk, r0);
  }
}

// first 16 S2 outputs of every node for tick t (see gm_mt_first16); resets the big
// worklist and the outgoing record counts
__global__ __launch_bounds__(256) void gm_p_mtgen(PState s, int t, uint32_t *mtraw, int reset) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (reset && r < s.nchunk) s.big_cnt[r] = s.huge_cnt[r] = 0;
  if (r >= s.nloc) return;
  uint32_t out[16];
  gm_mt_first16(gm_rd_seed(s.rd_seed, t, s.n0 + r + 1), out);
  uint4 *dst = (uint4 *)(mtraw + (size_t)r * 16);
#pragma unroll
  for (int q = 0; q < 4; q++) dst[q] = make_uint4(out[4 * q], out[4 * q + 1], out[4 * q + 2], out[4 * q + 3]);
}

// warm start at t0 (oracle op_create): self {2t0-1}, V-1 distinct peers chosen by
// mix64(view_seed ^ i<<32 ^ j) % n with hb 2(t0-1-a)-1, sorted by id; written to the
// parity of tick t0.
__global__ __launch_bounds__(64) void gm_p_init(PState s, int t0, uint64_t init_seed) {
  const int li = blockIdx.x * blockDim.x + threadIdx.x;
  if (li >= s.nloc) return;
  const int i = s.n0 + li;
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
  uint64_t *dst = s.lists + ((size_t)(t0 & 1) * s.rows + li) * V;
  for (int a = 0; a < V; a++) dst[a] = a < cnt ? ent[a] : 0ull;
  s.hbctr[li] = 2 * t0;
}

// received records of tick t (row shards): remote lists already sit in rows nloc + j of
// parity t&1; record each row's sender and append the row to its local targets' inboxes
__global__ __launch_bounds__(256) void gm_p_unpack(PState s, int t, int base, int nrecv) {
  const int j = base + blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= base + nrecv) return;
  const int par = t & 1;
  const int4 h0 = ((const int4 *)s.recv_hdr)[2 * (size_t)j];
  const int4 h1 = ((const int4 *)s.recv_hdr)[2 * (size_t)j + 1];
  if (h1.w != t) return;  // the sender's slot holds no record for this shard this tick (an older one, or none)
  s.rsrc[par][j] = h0.x;
  const int tg[GM_FANOUT] = {h0.z, h0.w, h1.x, h1.y, h1.z};
  for (int q = 0; q < h0.y && q < GM_FANOUT; q++) {
    const int d = tg[q] - s.n0;
    if (d < 0 || d >= s.nloc) {
      atomicOr(s.err, GM_ERR_INBOX);
      continue;
    }
    int32_t *row = s.inbox[par ^ 1] + (size_t)d * P_KMAX;
    const int slot = atomicAdd(row, 1);
    if (slot < s.kcap) row[1 + slot] = s.nloc + j;
    else atomicOr(s.err, GM_ERR_INBOX);
  }
}

// Row shards: the exchange records of chunk c (rows [r0, r1)), packed per peer q to the front of
// block (q, r0). A node with targets on q (its targets / rowstat of this tick) has one record for q:
// the header (sender, #targets on q, those targets in draw order, the tick as a stamp) and its final
// list of the tick (lists[t & 1]) in wire format -- the entries fresh at t, id | (2t-1 - hb) << 25.
// One workgroup per tile of 256 nodes and every peer: a node's distinct remote peers take their
// record slots in the tile by LDS atomics, ONE global atomic per (tile, peer) reserves each peer's
// run (the receivers' merge is order-free), and each node's list is read and converted once, by a
// half-wave, then written to each of its records. A block that would exceed its capacity (pk_cap,
// gm_host.hip xcap) sets GM_ERR_XCHG, never drops a record silently.
template <int VF>
__global__ __launch_bounds__(256) void gm_p_pack(PState s, int t, int c, int r0, int r1) {
  extern __shared__ int pk_sm[];  // [G] records per peer in this tile, then [G] the tile's run in each block
  const int G = s.G, V = VF ? VF : s.V;
  int *tcnt = pk_sm, *tbase = pk_sm + G;
  for (int q = threadIdx.x; q < G; q += 256) tcnt[q] = 0;
  __syncthreads();
  const int li = r0 + (int)blockIdx.x * 256 + (int)threadIdx.x;
  int tv[GM_FANOUT], tq[GM_FANOUT];
  const int ng = li < r1 ? min(s.rowstat[(size_t)li * 4 + 3], GM_FANOUT) : 0;
#pragma unroll
  for (int k = 0; k < GM_FANOUT; k++) {
    tv[k] = k < ng ? s.targets[(size_t)li * GM_FANOUT + k] : -1;
    tq[k] = k < ng ? p_owner(s, tv[k]) : -1;
  }
  // distinct remote peers in first-appearance order, each with its slot in the tile's run for that peer
  int pq[GM_FANOUT], ps[GM_FANOUT], np = 0;
#pragma unroll
  for (int k = 0; k < GM_FANOUT; k++) {
    bool fresh = tq[k] >= 0 && tq[k] != s.rank;
#pragma unroll
    for (int j = 0; j < k; j++) fresh = fresh && tq[j] != tq[k];
    if (fresh) {
      pq[np] = tq[k];
      ps[np] = atomicAdd(&tcnt[tq[k]], 1);
      np++;
    }
  }
  __syncthreads();
  for (int q = threadIdx.x; q < G; q += 256) tbase[q] = tcnt[q] ? atomicAdd(s.pk_cnt + (size_t)c * G + q, tcnt[q]) : 0;
  __syncthreads();
  // headers (the targets on q in draw order, -1 past nt); rec[j] = the record's row in block (pq[j], r0), -1 if over
  int rec[GM_FANOUT];
#pragma unroll
  for (int j = 0; j < GM_FANOUT; j++) {
    rec[j] = -1;
    if (j < np) {
      const int q = pq[j], d = tbase[q] + ps[j];
      if (d < s.pk_cap[(size_t)c * G + q]) {
        int h[GM_FANOUT], nt = 0;
#pragma unroll
        for (int k = 0; k < GM_FANOUT; k++) {
          h[k] = -1;
          if (tq[k] == q) h[nt++] = tv[k];
        }
        rec[j] = d;
        int4 *o = (int4 *)(s.pk_hdr + ((size_t)q * s.nloc + r0 + d) * 8);
        o[0] = make_int4(s.n0 + li, nt, h[0], h[1]);
        o[1] = make_int4(h[2], h[3], h[4], t);
      } else {
        atomicOr(s.err, GM_ERR_XCHG);
      }
    }
  }
  // lists: half-wave per node (entry e = lane & 31), two nodes of the wave per step; the node's
  // record rows and peers come from its own lane by shuffles
  const int lane = threadIdx.x & 63, e = lane & 31;
  const int wbase = r0 + (int)blockIdx.x * 256 + (int)(threadIdx.x & ~63u);
  const uint64_t *cur = s.lists + (size_t)(t & 1) * s.rows * V;
  const uint32_t tf = (uint32_t)(2 * t - 1);
  for (int it = 0; it < 32; it++) {
    const int src = 2 * it + (lane >> 5);  // the node's lane in this wave
    const int nnp = __shfl(np, src, 64);
    if (!__ballot(nnp > 0)) continue;
    const int node = wbase + src;
    uint32_t w = 0;
    if (nnp > 0 && e < V) {
      const uint64_t x = cur[(size_t)node * V + e];
      const uint32_t hb = (uint32_t)x;
      w = (x != 0 && !p_aged(t, hb, GM_TFAIL)) ? ((uint32_t)(x >> 32) | (tf - hb) << P_WIRE_IDBITS) : 0u;
    }
#pragma unroll
    for (int j = 0; j < GM_FANOUT; j++) {
      const int q = __shfl(pq[j], src, 64), d = __shfl(rec[j], src, 64);
      if (j < nnp && d >= 0 && e < V) s.pk_list[((size_t)q * s.nloc + r0 + d) * V + e] = w;
    }
  }
}

hipError_t gm_launch_partial_pack(const PState &s, int t, int c, hipStream_t st) {
  const int r0 = (int)((int64_t)s.nloc * c / s.nchunk), r1 = (int)((int64_t)s.nloc * (c + 1) / s.nchunk);
  if (r1 > r0 && s.G > 1) {
    const dim3 grid((r1 - r0 + 255) / 256);
    const size_t sm = sizeof(int) * 2 * (size_t)s.G;
    if (s.V == 32) hipLaunchKernelGGL(gm_p_pack<32>, grid, dim3(256), sm, st, s, t, c, r0, r1);
    else hipLaunchKernelGGL(gm_p_pack<0>, grid, dim3(256), sm, st, s, t, c, r0, r1);
  }
  return hipGetLastError();
}

#define P_BIG_GRID 1024
#define P_HUGE_GRID 256

// S2 precompute for every row + reset of the per-chunk worklists and record counts
hipError_t gm_launch_partial_mtgen(const PState &s, int t, uint32_t *mtraw, hipStream_t st, bool reset) {
  hipLaunchKernelGGL(gm_p_mtgen, dim3((std::max(s.nloc, s.nchunk * s.G) + 255) / 256), dim3(256), 0, st, s, t, mtraw,
                     reset ? 1 : 0);
  return hipGetLastError();
}

// the per-tick resets gm_p_mtgen does when the S2 outputs were prefetched without them
hipError_t gm_launch_partial_reset(const PState &s, hipStream_t st) {
  hipError_t e = hipMemsetAsync(s.big_cnt, 0, sizeof(int32_t) * s.nchunk, st);
  if (e == hipSuccess) e = hipMemsetAsync(s.huge_cnt, 0, sizeof(int32_t) * s.nchunk, st);
  return e;
}

// the node ticks of chunk c (rows [nloc*c/K, nloc*(c+1)/K))
hipError_t gm_launch_partial_chunk(const PState &s, int t, const uint32_t *mtraw, int c, hipStream_t st) {
  const int r0 = (int)((int64_t)s.nloc * c / s.nchunk), r1 = (int)((int64_t)s.nloc * (c + 1) / s.nchunk);
  const bool mc = s.mc_sent != nullptr && t < s.mc_tmax;
  if (r1 > r0) {
    const bool rm = s.rows != s.n || s.G > 1 || s.nloc != s.n;  // received lists possible
    // V = 32 (S-C) takes the instantiation with the view width folded in (shifts, not multiplies)
    auto *small = s.V == P_VMAX
                      ? (rm ? (mc ? gm_p_tick_small_pf<true, true, P_VMAX> : gm_p_tick_small_pf<false, true, P_VMAX>)
                            : (mc ? gm_p_tick_small_pf<true, false, P_VMAX> : gm_p_tick_small_pf<false, false, P_VMAX>))
                      : (rm ? (mc ? gm_p_tick_small_pf<true, true, 0> : gm_p_tick_small_pf<false, true, 0>)
                            : (mc ? gm_p_tick_small_pf<true, false, 0> : gm_p_tick_small_pf<false, false, 0>));
    // nodes per wave: P_NPW; a row shard's chunk (a few hundred thousand nodes per launch) takes
    // P_NPW_CHUNK, so the launch's last round of waves is a smaller share of it
    const int npw = s.nchunk > 1 ? P_NPW_CHUNK : P_NPW;
    hipLaunchKernelGGL(small, dim3((r1 - r0 + P_SWG * npw - 1) / (P_SWG * npw)), dim3(64 * P_SWG), 0, st, s, t, mtraw, c, r0, r1, npw);
  }
  hipLaunchKernelGGL(mc ? gm_p_tick_big<true> : gm_p_tick_big<false>, dim3(P_BIG_GRID), dim3(256),
                     4 * PLds<P_HB>::bytes, st, s, t, mtraw, c, r0);
  hipLaunchKernelGGL(mc ? gm_p_tick_huge<true> : gm_p_tick_huge<false>, dim3(P_HUGE_GRID), dim3(64),
                     PLds<P_HH>::bytes, st, s, t, mtraw, c, r0);
  return hipGetLastError();
}

hipError_t gm_launch_partial_tick(const PState &s, int t, uint32_t *mtraw, hipStream_t st, hipEvent_t k0,
                                  hipEvent_t k1) {
  hipError_t e = gm_launch_partial_mtgen(s, t, mtraw, st, true);
  if (e != hipSuccess) return e;
  if (k0) (void)hipEventRecord(k0, st);
  for (int c = 0; c < s.nchunk && e == hipSuccess; c++) e = gm_launch_partial_chunk(s, t, mtraw, c, st);
  if (k1) (void)hipEventRecord(k1, st);
  return e != hipSuccess ? e : hipGetLastError();
}

hipError_t gm_launch_partial_init(const PState &s, int t0, uint64_t init_seed, hipStream_t st) {
  hipLaunchKernelGGL(gm_p_init, dim3((s.nloc + 63) / 64), dim3(64), 0, st, s, t0, init_seed);
  return hipGetLastError();
}

hipError_t gm_launch_partial_unpack(const PState &s, int t, int base, int nrecv, hipStream_t st) {
  if (nrecv > 0) hipLaunchKernelGGL(gm_p_unpack, dim3((nrecv + 255) / 256), dim3(256), 0, st, s, t, base, nrecv);
  return hipGetLastError();
}

size_t gm_partial_lds_bytes() { return 4 * (size_t)PLds<P_HB>::bytes; }

