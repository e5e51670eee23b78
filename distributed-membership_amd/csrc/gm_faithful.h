// gm_faithful.h -- device state of the FAITHFUL tick (see gm_faithful.hip).
#pragma once
#include <stdint.h>

#define F_ENBUFFSIZE 30000  // EmulNet.h:12
#define F_MAX_NODES 1000    // EmulNet.h:10 (ENsend asserts src <= MAX_NODES)
#define F_MAX_TIME 3600     // EmulNet.h:11
#define F_RECV_LDS (160 * 1024)  // gm_f_recv dynamic LDS (the whole CU's)

enum { F_JOINREQ = 0, F_JOINREP = 1, F_LIST = 2 };  // MP1Node.h:30-35

// One EmulNet message (en_msg + payload, EmulNet.h:23-30; MP1Node.cpp:143-149,
// 246-250, 364-383): destination / source ids, type, the payload entry id
// (JOINREQ: the joiner; LIST: the gossiped member) and its heartbeat.
struct FMsg {
  int32_t to, from, type, subj, hb;
};

struct FEvent {
  int32_t t, logger, kind, subject, seq;
};

struct FState {
  int n, np, tmax;             // nodes, padded row width (x64), msgcount horizon
  int gstride;                 // gossip list stride (n + GM_FANOUT)
  int draw_cap;
  int drop_pct_now;            // (int)(MSG_DROP_PROB*100) while dropmsg, else -1
  uint64_t rd_seed;
  uint32_t *table;             // [n][np] packed (hb | ts<<16), GM_ABSENT
  int32_t *start;              // [n] (int)(STEP_RATE*i)
  int32_t *failed, *inited, *ingroup, *hbctr, *started_now;  // [n]
  FMsg *buf;                   // EmulNet buffer [F_ENBUFFSIZE]
  int32_t *bufsize;
  uint16_t *holepos;           // [2][F_ENBUFFSIZE] hole ranks + hit positions when they exceed gm_f_recv's LDS
  uint16_t *qidx;              // [F_ENBUFFSIZE] queue slot -> tick-start buffer index
  FMsg *buf2;                  // [F_ENBUFFSIZE] the other buffer: gm_f_recvout compacts the survivors into it
  uint16_t *bkey, *bkey2;      // [F_ENBUFFSIZE] destination key (strcmp prefix) of every buffered message
  uint16_t *sidx;              // [F_ENBUFFSIZE] survivors' tick-start indices (gm_f_recv -> gm_f_recvout)
  int32_t *rmeta;              // [2] messages delivered this tick, survivors
  FMsg *q;                     // this tick's queues, concatenated [F_ENBUFFSIZE]
  int32_t *q_off, *q_cnt;      // [n]
  int32_t *scount;             // sends per node this tick
  int32_t *jcnt, *gcnt, *fcnt; // JOINREPs, gossip targets, fresh entries per node
  int32_t *jrq;                // [n][n] JOINREP destinations (queue order)
  int32_t *gossip;             // [n][gstride] gossip target ids
  int32_t *fcols;              // [n][n] fresh columns ascending
  int32_t *s1;                 // glibc TYPE_3 state: 31 words + fptr + rptr
  int32_t *draws;              // [draw_cap]
  int32_t *sbase;              // [n] first send ordinal of node i (node-descending order)
  int32_t *smeta;              // [3] this tick's draw count S (-1: over draw_cap), S1 fptr at tick start, B0
  int32_t *spre;               // [draw_cap + 1] exclusive prefix count of kept sends
  uint32_t *s1mat;             // [64][31][32] P_q = R^(q+1), R = one 31-draw round of the S1 register
  uint32_t *s1vb;              // [draw_cap / 1984 + 2][32] S1 register at every 64th round
  int32_t *sent, *recv;        // [n + 1][tmax] (row = node id)
  FEvent *ev;
  unsigned long long *ev_count;
  int ev_cap;
  uint32_t *err;
};
