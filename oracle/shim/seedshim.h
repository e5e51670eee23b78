/* seedshim.h -- TEST INFRASTRUCTURE ONLY (oracle/_ref build in this container).
 *
 * Force-included (g++ -include) when compiling the unmodified reference sources
 * that lie under /root/reference. It injects the build's seed contract so the
 * reference becomes bit-reproducible:
 *   S1 (glibc rand):   time() -> $TIME_SEED  (Application.cpp:50,96 srand(time(NULL)))
 *   S2 (mt19937 seed): random_device in nodeLoopOps (MP1Node.cpp:450) ->
 *                      low32(splitmix64((RD_SEED ^ (t<<32 | node_id)) + golden))
 * Nothing here is shipped or linked into the product.
 */
#pragma once
#include <random>
#include <cstdint>
#include <cstdlib>
struct SeededRDCtx {
  static long tick;
  static int id;
  SeededRDCtx(long t, int i) { tick = t; id = i; }
};
struct SeededRD {
  typedef unsigned int result_type;
  unsigned int operator()() {
    const char *s = getenv("RD_SEED");
    uint64_t z = (s ? strtoull(s, 0, 10) : 0);
    z ^= ((uint64_t)(uint32_t)SeededRDCtx::tick << 32) | (uint32_t)SeededRDCtx::id;
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z ^= z >> 31;
    return (unsigned int)z;
  }
};
/* MP1Node.cpp:450 `random_device rd;` becomes a (globaltime, own id) capture + SeededRD rd; */
#define random_device SeededRDCtx rd_ctx_(par->getcurrtime(), *(int *)(&memberNode->addr.addr[0])); SeededRD
