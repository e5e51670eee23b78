// gm_scaled.h -- device state of the SCALED tick (see gm_scaled.hip).
#pragma once
#include <stdint.h>

#define S_THREADS 256            // 4 waves per observer row
#define S_KMAX 64                // inbox capacity (gossip lists per receiver per tick)
#define S_COLS_PER_THREAD 8      // 32 B of table + 16 B per sender message per step
#define S_COLS_PER_STEP (S_THREADS * S_COLS_PER_THREAD)
#define S_ROW_ALIGN 512          // padded row width granule (one wave step, 8 bitmap words)

#define S_EV_ADD 1u
#define S_EV_REMOVE 2u

struct SState {
  int n;                   // observers (rows) = N
  int wp;                  // padded shard width (columns per row, multiple of S_ROW_ALIGN)
  int w;                   // real shard width
  int c0;                  // first global subject column of this shard
  int evcap;               // per-row event slots
  uint32_t ev_spill_cap;
  uint64_t rd_seed, drop_seed;
  uint32_t *table;         // [n][wp] packed {hb | ts<<16}, GM_ABSENT
  uint16_t *msg[2];        // gossip payload planes, indexed by tick parity; row r at msg[p] + r*mstride
  size_t mstride;          // row stride of the payload planes (2*wp: both parities of a row adjacent)
  int32_t *inbox_cnt[2];   // [n] lists queued for each receiver, by delivery-tick parity
  int32_t *inbox[2];       // [n][S_KMAX] sender rows
  int32_t *hbctr;          // [n] MP1Node heartbeat counter (Member::heartbeat)
  int32_t *failed;         // [n] Member::bFailed
  uint32_t *ev_rows;       // [n][evcap] kind<<30 | subject id
  int32_t *ev_cnt;         // [n]
  uint64_t *ev_spill;      // overflow: (logger<<32) | kind<<30 | subject id
  uint32_t *ev_spill_cnt;
  int32_t *rowstat;        // [n][4]: lists delivered, present, numfailed, targets chosen
  int32_t *targets;        // [n][GM_FANOUT]
  uint32_t *err;
  // ---- column-sharded mode (shard_count > 1; see gm_s_draw / gm_s_accept)
  int shard_rank, shard_count;
  uint64_t *gpres, *gfresh;  // [n][wp/64] post-sweep presence / freshness of this shard's columns
  uint32_t *gpre;            // [n][wp/64] exclusive prefix popcounts of gpres
  int32_t *xcnt;             // bound exchange buffer [shard_count][n][2]: (present, numfailed) per shard
  int32_t *status;           // bound exchange buffer [n][D]: resolved draws, MAX-allreduced
  uint32_t *mt;              // [624][n] per-row mt19937 state, strided
  int32_t *mtk;              // [n][3]: k, ninit, first of each row's generator
  int32_t *acc;              // [n][8]: targets so far, g[5], numpot, size
  int32_t *pending;          // [n] rows still drawing
  int32_t *npending;         // rows still drawing after the last accept round
};
