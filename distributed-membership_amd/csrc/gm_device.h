// gm_device.h -- device-side building blocks shared by the FAITHFUL and SCALED
// tick kernels (gfx950 / CDNA4, wave64).
//
//  * packed membership entry: one uint32 per (observer, subject) cell,
//    low 16 bits = heartbeat, high 16 bits = timestamp, 0xFFFFFFFF = absent.
//    Exact while globaltime < 32767 (hb <= 2t+1 < 65535), which gm_create
//    enforces. Replaces MemberListEntry {int id; short port; long hb; long ts}
//    (Member.h:62-81): id is the column, port is always 0 (EmulNet.cpp:75).
//  * the S2 stream: mt19937 seeded per (tick, node id) (MP1Node.cpp:450-452 under
//    the SURVEY Appendix B seed contract), twisted lazily in output order so a
//    node that needs k draws pays ~397+k init steps instead of 624 + a full twist,
//    and libstdc++-11 uniform_int_distribution<int> (Lemire) on top.
//  * rank-select over an LDS presence bitmap = "memberlist[ix]" of the sorted
//    std::vector the reference indexes (MP1Node.cpp:467-485).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define GM_TFAIL 5        // MP1Node.h:21
#define GM_TREMOVE 20     // MP1Node.h:20
#define GM_FANOUT 5       // MP1Node.cpp:456
#define GM_ABSENT 0xFFFFFFFFu
#define GM_NONE16 0xFFFFu

#define GM_ERR_INBOX 1u       // a receiver got more gossip lists than the inbox holds
#define GM_ERR_SELF 2u        // SCALED fast path: an observer lost its own entry
#define GM_ERR_EVENTS 4u      // event spill ring overflowed
#define GM_ERR_DRAWS 8u       // S1 draw table too small (FAITHFUL)
#define GM_ERR_BUFFER 16u     // FAITHFUL EmulNet buffer bookkeeping broke
#define GM_ERR_QUEUE 32u      // FAITHFUL per-node queue larger than the LDS stage
#define GM_ERR_LAG 64u        // SCALED: an entry heartbeat lag beyond the narrow cell encoding
#define GM_ERR_ESC 128u       // SCALED: an escape pool (compact wide cells / payload bytes) overflowed
#define GM_ERR_XCHG 256u      // PARTIAL row shards: a packed exchange block overflowed its capacity
#define GM_ERR_PARITY 512u    // PARTIAL: an even heartbeat distance (the odd-heartbeat invariant broke)

__device__ __forceinline__ uint32_t gm_pack(uint32_t hb, uint32_t ts) { return (ts << 16) | hb; }
__device__ __forceinline__ uint32_t gm_hb(uint32_t e) { return e & 0xFFFFu; }
__device__ __forceinline__ uint32_t gm_ts(uint32_t e) { return e >> 16; }

__device__ __forceinline__ uint64_t gm_mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

// murmur3 finalizer: a bijection of uint32 (distinct inputs -> distinct outputs), 2 multiplies
__host__ __device__ __forceinline__ uint32_t gm_fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  return h ^ (h >> 16);
}
// keyed-loss threshold on a 16-bit uniform chunk: lost iff chunk < ceil(pct * 65536 / 100)
// (probability pct % to within 1.5e-5; SCALED and PARTIAL, oracle/ref_cpu.c the same)
__host__ __device__ inline uint32_t gm_drop_thresh(int pct) {
  return pct <= 0 ? 0u : pct >= 100 ? 65536u : (uint32_t)((pct * 65536 + 99) / 100);
}

// random_device replacement of the seed contract
__device__ __forceinline__ uint32_t gm_rd_seed(uint64_t rd_seed, int32_t tick, int32_t id) {
  uint64_t z = rd_seed ^ (((uint64_t)(uint32_t)tick << 32) | (uint32_t)id);
  return (uint32_t)gm_mix64(z + 0x9E3779B97F4A7C15ULL);
}

// Lazily-twisted mt19937 whose 624-word state lives in LDS (one generator per
// workgroup, driven by a single lane). Twisting word k just before output k and
// storing it back is exactly the standard block twist, because word k's twist
// reads x[k+1] (old) and x[(k+397)%624] (old for k<227, already-new for k>=227).
// `stride` lets the 624 words live strided in global memory ([624][rows],
// coalesced across the rows of a launch) for generators that outlive a kernel.
struct GmLazyMT {
  uint32_t *x;     // 624 words (LDS, or global with a row stride)
  int stride;      // distance between consecutive state words
  int k;           // next output index within the current 624-block
  int ninit;       // init words computed so far (first block only)
  bool first;      // still in the first block (init words possibly incomplete)

  __device__ void seed(uint32_t *base, uint32_t s, int stride_ = 1) {
    x = base;
    stride = stride_;
    x[0] = s;
    ninit = 1;
    k = 0;
    first = true;
  }
  __device__ __forceinline__ uint32_t &w(int i) { return x[(size_t)i * stride]; }
  __device__ __forceinline__ void init_to(int upto) {  // make init words [0, upto] valid
    uint32_t v = w(ninit - 1);
    for (int i = ninit; i <= upto; i++) {
      v = 1812433253u * (v ^ (v >> 30)) + (uint32_t)i;
      w(i) = v;
    }
    if (upto + 1 > ninit) ninit = upto + 1;
  }
  __device__ uint32_t next() {
    if (k == 624) { k = 0; first = false; }
    if (first) {
      int need = k + 397 < 624 ? k + 397 : 623;
      if (k + 1 > need) need = k + 1 < 624 ? k + 1 : 623;
      if (need >= ninit) init_to(need);
    }
    uint32_t y = (w(k) & 0x80000000u) | (w(k + 1 < 624 ? k + 1 : 0) & 0x7fffffffu);
    uint32_t v = w(k + 397 < 624 ? k + 397 : k - 227) ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    w(k) = v;
    k++;
    v ^= v >> 11;
    v ^= (v << 7) & 0x9d2c5680u;
    v ^= (v << 15) & 0xefc60000u;
    v ^= v >> 18;
    return v;
  }
  // uniform_int_distribution<int>(0, range-1) (bits/uniform_int_dist.h, _S_nd)
  __device__ int uniform(uint32_t range) {
    uint64_t prod = (uint64_t)next() * range;
    uint32_t low = (uint32_t)prod;
    if (low < range) {
      uint32_t thr = (uint32_t)(0u - range) % range;
      while (low < thr) {
        prod = (uint64_t)next() * range;
        low = (uint32_t)prod;
      }
    }
    return (int)(prod >> 32);
  }
};

// The first 16 outputs of mt19937(seed): outputs 0..15 need init words x[0..16] and
// x[397..412] only (output k twists x[k], x[k+1], x[k+397], all still init words for
// k < 227), so 413 init steps in registers replace the 624-word state.
__device__ __forceinline__ void gm_mt_first16(uint32_t seed, uint32_t out[16]) {
  uint32_t lo[17], hi[16];
  uint32_t v = seed;
  lo[0] = v;
#pragma unroll
  for (int i = 1; i <= 16; i++) {
    v = 1812433253u * (v ^ (v >> 30)) + (uint32_t)i;
    lo[i] = v;
  }
#pragma unroll  // the constant i folds into one add (S-C's side-stream gm_p_mtgen: -0.6 % per tick,
                // profiles/r06/ab_sc_npw/)
  for (int i = 17; i < 397; i++) v = 1812433253u * (v ^ (v >> 30)) + (uint32_t)i;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    v = 1812433253u * (v ^ (v >> 30)) + (uint32_t)(397 + i);
    hi[i] = v;
  }
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const uint32_t y = (lo[k] & 0x80000000u) | (lo[k + 1] & 0x7fffffffu);
    uint32_t o = hi[k] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    o ^= o >> 11;
    o ^= (o << 7) & 0x9d2c5680u;
    o ^= (o << 15) & 0xefc60000u;
    out[k] = o ^ (o >> 18);
  }
}

// Index of the ix-th set bit (0-based) of a bitmap `bits` with exclusive
// per-word prefix popcounts `pre` (nw words). Caller guarantees ix < total.
__device__ __forceinline__ int gm_rank_select(const uint64_t *bits, const uint32_t *pre, int nw, uint32_t ix) {
  int lo = 0, hi = nw - 1;
  while (lo < hi) {  // largest w with pre[w] <= ix
    int mid = (lo + hi + 1) >> 1;
    if (pre[mid] <= ix) lo = mid; else hi = mid - 1;
  }
  uint64_t w = bits[lo];
  uint32_t r = ix - pre[lo];
  // select the r-th set bit of w
  uint32_t lo32 = (uint32_t)w, c = __builtin_popcount(lo32);
  int base = 0;
  if (r >= c) { r -= c; w >>= 32; base = 32; }
  uint32_t v = (uint32_t)w;
  for (int b = 0; b < 32; b++) {
    if (v & 1u) {
      if (r == 0) return lo * 64 + base + b;
      r--;
    }
    v >>= 1;
  }
  return -1;
}

// Block-wide exclusive scan of one int per thread (blockDim a multiple of 64,
// <= 1024); every thread of the block must call it. s_tmp: >= 16 ints of LDS.
__device__ __forceinline__ int gm_block_scan(int v, int *s_tmp, int *total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  int x = v;
  for (int o = 1; o < 64; o <<= 1) {
    int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_tmp[wid] = x;
  __syncthreads();
  if (wid == 0) {
    int w = lane < nw ? s_tmp[lane] : 0;
    for (int o = 1; o < 16; o <<= 1) {
      int y = __shfl_up(w, o, 64);
      if (lane >= o) w += y;
    }
    if (lane < nw) s_tmp[lane] = w;  // inclusive per-wave totals
  }
  __syncthreads();
  int base = wid ? s_tmp[wid - 1] : 0;
  *total = s_tmp[nw - 1];
  __syncthreads();
  return base + x - v;
}

// Block-wide sum (same calling rules as gm_block_scan).
__device__ __forceinline__ int gm_block_sum(int v, int *s_tmp) {
  int tot;
  (void)gm_block_scan(v, s_tmp, &tot);
  return tot;
}
