// gm_partial.h -- device state of the PARTIAL-view tick (see gm_partial.hip).
#pragma once
#include <stdint.h>

#define P_VMAX 32        // view capacity limit (a list is one half-wave of 8-byte entries)
#define P_KSMALL 12      // nodes with <= P_KSMALL delivered lists take the small-table kernel
#define P_KP 16          // nodes with P_KSMALL < k <= P_KP lists take the big-table kernel, more the huge one
#define P_HS 512         // small kernel: LDS hash slots per wave (union <= (1 + P_KSMALL) * P_VMAX + 1 < P_HS - 64:
                         //   the sweep parks dead slots past the dense range; 12 lists = 0.2 % Poisson(5) tail left)
#define P_HB 1024        // big kernel: LDS hash slots per wave (>= (1 + P_KP) * P_VMAX / 0.53)
#define P_HH 4096        // huge kernel: LDS hash slots per wave (>= (1 + P_KMAX) * P_VMAX / 0.51)
#define P_KMAX 64        // inbox row: count + P_KMAX - 1 = 63 lists queued per receiver per tick; every list is merged
#ifndef P_NPW
#define P_NPW 16         // small kernel: consecutive nodes per wave, prefetching (one-box A/Bs: 16 -0.8 % vs 8, 32 -0.25 % vs 16)
#endif
#ifndef P_SWG
#define P_SWG 1          // small kernel: waves per workgroup (1: every wave's LDS starts at address 0)
#endif
#ifndef P_NPW_CHUNK
#define P_NPW_CHUNK 4    // the same for a row shard's chunk launches (fewer nodes per launch: a finer last round)
#endif
#define P_EV_ADD 1u
#define P_EV_REMOVE 2u
// Wire entry of an exchanged list: id | (2t-1 - hb) << 25, only entries fresh at the
// sender's tick t (the receiver drops the others anyway), 0 = none: 4 bytes instead of 8.
#define P_WIRE_IDBITS 25

static_assert((1 + P_KSMALL) * P_VMAX + 1 < P_HS - 64, "small table: the dense range must end below the trash slots");

struct PState {
  int n;                 // nodes of the whole cluster
  int V;                 // view capacity
  // row shard (multi-GPU S-C): this context owns nodes [n0, n0 + nloc); local row li = i - n0.
  // Single context: n0 = 0, nloc = n, G = 1.
  int n0, nloc, G, rank;
  int rows;              // list rows per parity (= nloc: received lists stay in recv_list, wire format)
  int nchunk;            // K: the node ticks run in K row chunks; a shard ships chunk c's records while c+1 runs
  int drop_pct;          // per-entry drop percentage for this tick's deliveries (-1: none)
  uint64_t rd_seed, view_seed, drop_seed;
  uint64_t *lists;       // [2][rows][V] entries (id << 32 | hb), 0 = empty, sorted by id; parity t&1 written at tick t
  int32_t *inbox[2];     // [nloc][P_KMAX] by delivery-tick parity: slot 0 = lists queued for the receiver (the
                         //   append counter: it shares a line with the first slots), slots 1.. = senders: local
                         //   row li, or nloc + j for received record j
  int32_t *rsrc[2];      // [n - nloc] global sender index of each received list row, by parity
  int32_t *hbctr;        // [nloc] heartbeat counter
  int32_t *failed;       // [nloc]
  uint32_t *ev;          // [nloc][2V] kind<<30 | subject id of the removals, from the back of the row
  int32_t *ev_cnt;       // [nloc] joins | removals << 16
  uint32_t *ev_jm;       // [nloc] joins as a mask over the node's final list of the tick (bit e: entry e is new;
                         //   the list is id-sorted, so the joins in ascending id order are its set bits)
  int32_t *rowstat;      // [nloc][4]: lists merged, view size, numfailed, targets chosen
  int32_t *targets;      // [nloc][GM_FANOUT] (global node indices)
  int32_t *big;          // [nloc] worklists of nodes with > P_KSMALL lists (big-table kernel), chunk c at rows r0_c..
  int32_t *big_cnt;      // [K]
  int32_t *huge;         // [nloc] worklists of nodes with > P_KP lists (huge-table kernel), chunk c at rows r0_c..
  int32_t *huge_cnt;     // [K]
  // outgoing lists to the other row shards (sharded only): after chunk c's node kernels, gm_p_pack
  // builds one record per (sender, remote shard) from the sender's targets and its final list of the
  // tick, packed per peer (below); the header's stamp (word 7 = the tick) tells the receiver which
  // rows of a block hold a record of this tick
  int32_t *recv_hdr;     // [n - nloc][8] received headers: chunk-major, source shard ascending
  uint32_t *recv_list[2]; // [n - nloc][V] received lists (wire format), by the parity of the tick that
                         //   sent them; the next tick's kernels decode them in place
  // packed exchange blocks (gm_p_pack): chunk c's records to shard q compacted to the front of the
  // rows [q * nloc + r0_c, +cap) of these buffers; only the block's first cap rows travel (cap: the
  // host's binomial bound from the live nodes per shard, gm_host.hip xcap); rows past the records
  // keep older stamps, so receivers need no count (gm_p_unpack takes the rows stamped t)
  int32_t *pk_hdr;       // [G][nloc][8]
  uint32_t *pk_list;     // [G][nloc][V]
  int32_t *pk_cnt;       // [K][G] records packed per (chunk, shard) this tick
  int32_t *pk_cap;       // [K][G] capacity of the block (chunk, shard) (host-written when the crash set changes)
  float xcap_frac;       // diagnostics (GM_XCHG_CAP_FRAC): block capacity = this fraction of the slots
  int32_t *shard_n0;     // [G+1] first node of every row shard (shard_n0[G] = n)
  uint32_t *err;
  // msgcount analogue (gm_msgcount_record; nullptr = off): per tick and local node, view
  // entries sent (fresh entries x targets, before loss) / received (after loss, lists merged)
  uint32_t *mc_sent, *mc_recv;  // [mc_tmax][nloc]
  int mc_tmax;
  int kcap;                     // inbox slots used (P_KMAX - 1; lowered only by the diagnostics env GM_INBOX_CAP)
};
