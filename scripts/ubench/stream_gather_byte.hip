// Microbenchmark (measurement tool, not product): the band tick's memory pattern with
// 8-BIT table cells (one byte per (observer, subject): 4-bit heartbeat lag class, 4-bit
// age) against round 2's 16-bit cells, both with 4-bit payload nibbles, 16 cells per lane:
//   W = 16: table slab stream 32 B/lane read + write (NT)        (gm_s_band today)
//   W = 8 : table slab stream 16 B/lane read + write (NT)
// plus payload write 8 B/lane and K gathered 8 B/lane payload reads of random rows of the
// band's payload slab (sender ids loaded from an inbox array first, as in the kernel).
// CONV = 1 adds the byte <-> packed-u16 widening and narrowing a byte table would cost
// (v_perm unpack, decode to the 16-bit cell, re-encode with a range check, v_perm pack).
// Prints ms per sweep of an N = 65,536 x 65,536 table.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16; return x;
}
__device__ __forceinline__ u16x2 pk(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ uint32_t unpk(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }

template <int B, int W, int K, int CONV>
__global__ __launch_bounds__(256) void kband(uint8_t *table, uint8_t *pay, const int *inbox, int n, int nb,
                                             uint32_t *sink) {
  constexpr int LPR = B / 16, RPW = 64 / LPR;
  const int lane = threadIdx.x & 63, sub = lane / LPR, li = lane % LPR;
  const int U = n / RPW;
  const int u = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (u >= U * nb) return;
  const int band = u / U, r = (u - band * U) * RPW + sub;
  const size_t slab = (size_t)band * n;
  uint8_t *tr = table + ((slab + r) * B + li * 16) * (W / 8);
  u32x4 a, b = {0, 0, 0, 0};
  a = __builtin_nontemporal_load((const u32x4 *)tr);
  if (W == 16) b = __builtin_nontemporal_load((const u32x4 *)(tr + 16));
  int snd[8];
  const int4 x = *(const int4 *)(inbox + (size_t)r * 8), y = *(const int4 *)(inbox + (size_t)r * 8 + 4);
  snd[0] = x.x; snd[1] = x.y; snd[2] = x.z; snd[3] = x.w; snd[4] = y.x; snd[5] = y.y; snd[6] = y.z; snd[7] = y.w;
  u32x2 m[K > 0 ? K : 1];
#pragma unroll
  for (int j = 0; j < K; j++) m[j] = *(const u32x2 *)(pay + (slab + snd[j]) * B + B / 2 + li * 8);
  u16x2 acc[8];
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = (u16x2)(0);
#pragma unroll
  for (int j = 0; j < K; j++) {
    acc[0] = __builtin_elementwise_max(acc[0], pk(m[j].x));
    acc[1] = __builtin_elementwise_max(acc[1], pk(m[j].x) << (u16x2)(4));
    acc[2] = __builtin_elementwise_max(acc[2], pk(m[j].x) << (u16x2)(8));
    acc[3] = __builtin_elementwise_max(acc[3], pk(m[j].x) << (u16x2)(12));
    acc[4] = __builtin_elementwise_max(acc[4], pk(m[j].y));
    acc[5] = __builtin_elementwise_max(acc[5], pk(m[j].y) << (u16x2)(4));
    acc[6] = __builtin_elementwise_max(acc[6], pk(m[j].y) << (u16x2)(8));
    acc[7] = __builtin_elementwise_max(acc[7], pk(m[j].y) << (u16x2)(12));
  }
  uint32_t tw[8];
  if (W == 16) {
    tw[0] = a.x; tw[1] = a.y; tw[2] = a.z; tw[3] = a.w; tw[4] = b.x; tw[5] = b.y; tw[6] = b.z; tw[7] = b.w;
  } else if (CONV) {  // bytes -> u16 halves, then cell16 = 7168 + (hi nibble << 6) + lo nibble for nonzero bytes
    const uint32_t s4[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
    for (int q = 0; q < 4; q++) {
      tw[2 * q] = __builtin_amdgcn_perm(0u, s4[q], 0x0c010c00u);
      tw[2 * q + 1] = __builtin_amdgcn_perm(0u, s4[q], 0x0c030c02u);
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const u16x2 v = pk(tw[i]);
      const u16x2 nz = __builtin_elementwise_min(v, (u16x2)(1));
      tw[i] = unpk(nz * (u16x2)(7168) + ((v & (u16x2)(0xF0)) << (u16x2)(2)) + (v & (u16x2)(0xF)));
    }
  } else {
    const uint32_t s4[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
    for (int q = 0; q < 4; q++) { tw[2 * q] = s4[q]; tw[2 * q + 1] = s4[q] >> 8; }
  }
  uint32_t cw[8];
  u16x2 bad = (u16x2)(0);
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const u16x2 nb = acc[i] >> (u16x2)(12);
    const u16x2 key5 = __builtin_elementwise_min(nb, (u16x2)(1)) * (u16x2)(7168) + (nb << (u16x2)(6));
    const u16x2 v = __builtin_elementwise_max(__builtin_elementwise_sub_sat(pk(tw[i]), (u16x2)(63)), key5);
    cw[i] = unpk(v);
    if (W == 8 && CONV) {  // re-encode: h even in [226, 254] and age <= 15, else escape
      const u16x2 h = v >> (u16x2)(5), ag = v & (u16x2)(31);
      const u16x2 h4 = __builtin_elementwise_sub_sat(h, (u16x2)(224)) >> (u16x2)(1);
      bad |= __builtin_elementwise_min((h4 * (u16x2)(2) + (u16x2)(224)) ^ h, (u16x2)(1)) |
             (ag >> (u16x2)(4));
      cw[i] = unpk((h4 << (u16x2)(4)) | (ag & (u16x2)(15)));
    }
  }
  uint32_t nib0 = cw[0] ^ cw[3], nib1 = cw[5] + cw[6];
  if (W == 16) {
    a = (u32x4){cw[0], cw[1], cw[2], cw[3]};
    b = (u32x4){cw[4], cw[5], cw[6], cw[7]};
    __builtin_nontemporal_store(a, (u32x4 *)tr);
    __builtin_nontemporal_store(b, (u32x4 *)(tr + 16));
  } else {
    a = (u32x4){__builtin_amdgcn_perm(cw[1], cw[0], 0x06040200u), __builtin_amdgcn_perm(cw[3], cw[2], 0x06040200u),
                __builtin_amdgcn_perm(cw[5], cw[4], 0x06040200u), __builtin_amdgcn_perm(cw[7], cw[6], 0x06040200u)};
    __builtin_nontemporal_store(a, (u32x4 *)tr);
  }
  const u32x2 o = {nib0, nib1};
  __builtin_nontemporal_store(o, (u32x2 *)(pay + (slab + r) * B + li * 8));
  if (unpk(bad) == 0x7b && r == 3) sink[0] = 1;
}

template <int B, int W, int K, int CONV>
float run(uint8_t *table, uint8_t *pay, const int *inbox, int n, int nb, uint32_t *sink, int reps) {
  constexpr int RPW = 64 / (B / 16);
  const int grid = ((n / RPW) * nb + 3) / 4;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL((kband<B, W, K, CONV>), dim3(grid), dim3(256), 0, 0, table, pay, inbox, n, nb, sink);
  hipEventRecord(e0);
  for (int i = 0; i < reps; i++)
    hipLaunchKernelGGL((kband<B, W, K, CONV>), dim3(grid), dim3(256), 0, 0, table, pay, inbox, n, nb, sink);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

__global__ void fill_inbox(int *inbox, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n * 8) inbox[i] = (int)(mix(i * 2654435761u) % (uint32_t)n);
}

int main() {
  const int n = 65536, wp = 65536;
  uint8_t *table, *pay; int *inbox; uint32_t *sink;
  hipMalloc(&table, (size_t)n * wp * 2);
  hipMalloc(&pay, (size_t)n * wp);
  hipMalloc(&inbox, (size_t)n * 8 * 4);
  hipMalloc(&sink, 64);
  hipMemset(table, 0, (size_t)n * wp * 2);
  hipMemset(pay, 0, (size_t)n * wp);
  hipLaunchKernelGGL(fill_inbox, dim3(n * 8 / 256), dim3(256), 0, 0, inbox, n);
  const double cells = (double)n * wp;
  auto rep = [&](int W, int B, int K, int conv, float ms) {
    const double dram = cells * (W / 8 * 2 + 1) / 1e9;  // table r+w + payload write + one payload read
    printf("cell%-2d B=%4d K=%d conv=%d  %6.3f ms  dram-min %5.1f GB %5.2f TB/s\n", W, B, K, conv, ms, dram,
           dram / ms / 1e3);
    fflush(stdout);
  };
#define RUN(B, W, K, C) rep(W, B, K, C, run<B, W, K, C>(table, pay, inbox, n, wp / B, sink, 5))
  RUN(1024, 16, 0, 0); RUN(1024, 16, 5, 0);
  RUN(1024, 8, 0, 0); RUN(1024, 8, 5, 0); RUN(1024, 8, 5, 1);
  RUN(512, 8, 5, 1); RUN(256, 8, 5, 1);
  RUN(1024, 16, 0, 0); RUN(1024, 8, 5, 1);
  return 0;
}
