// gm_partial.h -- device state of the PARTIAL-view tick (see gm_partial.hip).
#pragma once
#include <stdint.h>

#define P_VMAX 32        // view capacity limit (a list is one half-wave of 8-byte entries)
#define P_KP 16          // gossip lists merged per node and tick (oracle OP_KP)
#define P_KSMALL 10      // nodes with <= P_KSMALL delivered lists take the small-table kernel
#define P_HS 512         // small kernel: LDS hash slots per wave (>= (1 + P_KSMALL) * P_VMAX / 0.69)
#define P_HB 1024        // big kernel: LDS hash slots per wave (>= (1 + P_KP) * P_VMAX / 0.53)
#define P_KMAX 64        // inbox capacity (lists queued per receiver per tick)
#define P_EV_ADD 1u
#define P_EV_REMOVE 2u

struct PState {
  int n;                 // nodes
  int V;                 // view capacity
  int drop_pct;          // per-entry drop percentage for this tick's deliveries (-1: none)
  uint64_t rd_seed, view_seed, drop_seed;
  uint64_t *lists;       // [2][n][V] entries (id << 32 | hb), 0 = empty, sorted by id; parity t&1 written at tick t
  int32_t *inbox_cnt[2]; // [n] lists queued for each receiver, by delivery-tick parity
  int32_t *inbox[2];     // [n][P_KMAX] sender indices
  int32_t *hbctr;        // [n] heartbeat counter
  int32_t *failed;       // [n]
  uint32_t *ev;          // [n][2V] kind<<30 | subject id: joins from the front (ascending id), removals from the back
  int32_t *ev_cnt;       // [n] joins | removals << 16
  int32_t *rowstat;      // [n][4]: lists merged, view size, numfailed, targets chosen
  int32_t *targets;      // [n][GM_FANOUT]
  int32_t *big;          // [n] worklist of nodes with > P_KSMALL lists (big-table kernel)
  int32_t *big_cnt;      // [1]
  uint32_t *err;
};
