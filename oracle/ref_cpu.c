#define _POSIX_C_SOURCE 199309L
/* ref_cpu.c -- CPU restatement of the reference simulator (the parity oracle).
 *
 * TEST INFRASTRUCTURE ONLY; see ref_cpu.h for scope and the list of reference
 * functions restated. Data structures intentionally follow the reference
 * (sorted per-node member lists with lower_bound, a flat EmulNet message array
 * scanned from the end with swap-with-last removal) rather than the dense
 * SoA table of the HIP product, so the oracle shares no design decision with
 * the code it checks.
 */
#include "ref_cpu.h"

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define TFAIL 5            /* MP1Node.h:21 */
#define TREMOVE 20         /* MP1Node.h:20 */
#define FANOUT 5           /* MP1Node.cpp:456 maxneighbors */
#define ENBUFFSIZE 30000   /* EmulNet.h:12 */
#define MAX_MSG_SIZE 4000  /* Params.cpp:31 */
#define EN_MSG_HDR 16      /* sizeof(en_msg), EmulNet.h:23-30 */
#define MAX_TIME 3600      /* EmulNet.h:11 */
#define MAX_NODES 1000     /* EmulNet.h:10 */
#define LIST_SIZE 19       /* sizeof(MessageHdr)+6+8+1, MP1Node.cpp:143,364 */
#define JOINREP_SIZE 4     /* sizeof(MessageHdr), MP1Node.cpp:250 */

enum { JOINREQ = 0, JOINREP = 1, LIST = 2 }; /* MP1Node.h:30-35 */

/* ---------------------------------------------------------------- RNG S1 -- */
/* glibc TYPE_3 random_r/srandom_r (degree 31, separation 3), restated. */
void oc_srand(oc_rand *g, uint32_t seed) {
  if (seed == 0) seed = 1;
  int32_t word = (int32_t)seed;
  g->st[0] = word;
  for (int i = 1; i < 31; i++) {
    long hi = word / 127773, lo = word % 127773;
    word = (int32_t)(16807 * lo - 2836 * hi);
    if (word < 0) word += 2147483647;
    g->st[i] = word;
  }
  g->f = 3;
  g->r = 0;
  for (int k = 0; k < 310; k++) (void)oc_rand_next(g);
}

int32_t oc_rand_next(oc_rand *g) {
  uint32_t v = (uint32_t)g->st[g->f] + (uint32_t)g->st[g->r];
  g->st[g->f] = (int32_t)v;
  g->f = (g->f + 1) % 31;
  g->r = (g->r + 1) % 31;
  return (int32_t)(v >> 1);
}

/* ---------------------------------------------------------------- RNG S2 -- */
static uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

/* seed contract: one splitmix64 step over RD_SEED ^ (t<<32 | id) */
uint32_t oc_rd_seed(uint64_t rd_seed, int32_t tick, int32_t id) {
  uint64_t z = rd_seed ^ (((uint64_t)(uint32_t)tick << 32) | (uint32_t)id);
  return (uint32_t)mix64(z + 0x9E3779B97F4A7C15ULL);
}

typedef struct mt { uint32_t x[624]; int i; } mt;

static void mt_seed(mt *m, uint32_t s) {
  m->x[0] = s;
  for (int i = 1; i < 624; i++) m->x[i] = 1812433253u * (m->x[i - 1] ^ (m->x[i - 1] >> 30)) + (uint32_t)i;
  m->i = 624;
}

static uint32_t mt_next(mt *m) {
  if (m->i >= 624) {
    for (int k = 0; k < 624; k++) {
      uint32_t y = (m->x[k] & 0x80000000u) | (m->x[(k + 1) % 624] & 0x7fffffffu);
      m->x[k] = m->x[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    m->i = 0;
  }
  uint32_t y = m->x[m->i++];
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

/* libstdc++-11 uniform_int_distribution<int>(0, n-1) over a 32-bit engine: Lemire
 * (bits/uniform_int_dist.h _S_nd, downscaling branch). */
static int mt_uniform(mt *m, uint32_t range) {
  uint64_t prod = (uint64_t)mt_next(m) * range;
  uint32_t low = (uint32_t)prod;
  if (low < range) {
    uint32_t thr = (uint32_t)(-range) % range;
    while (low < thr) {
      prod = (uint64_t)mt_next(m) * range;
      low = (uint32_t)prod;
    }
  }
  return (int)(prod >> 32);
}

void oc_mt_uniform(uint32_t seed, int n, int k, int32_t *out) {
  mt m;
  mt_seed(&m, seed);
  for (int i = 0; i < k; i++) out[i] = mt_uniform(&m, (uint32_t)n);
}

/* ------------------------------------------------------------ containers -- */
typedef struct entry { int32_t id; int16_t port; int64_t hb, ts; } entry; /* MemberListEntry, Member.h:62-81 */
typedef struct elist { entry *v; int n, cap; } elist;
typedef struct msg { int32_t size, from, to, type, id; int16_t port; int64_t hb; } msg;
typedef struct mvec { msg *v; int n, cap; } mvec;
typedef struct sbuf { char *p; size_t n, cap; } sbuf;

static void el_push(elist *l, entry e) {
  if (l->n == l->cap) {
    l->cap = l->cap ? 2 * l->cap : 16;
    l->v = (entry *)realloc(l->v, sizeof(entry) * (size_t)l->cap);
  }
  l->v[l->n++] = e;
}

static void mv_push(mvec *l, const msg *m) {
  if (l->n == l->cap) {
    l->cap = l->cap ? 2 * l->cap : 64;
    l->v = (msg *)realloc(l->v, sizeof(msg) * (size_t)l->cap);
  }
  l->v[l->n++] = *m;
}

static void sb_put(sbuf *b, const char *s, size_t k) {
  if (b->n + k + 1 > b->cap) {
    b->cap = (b->n + k + 1) * 2;
    b->p = (char *)realloc(b->p, b->cap);
  }
  memcpy(b->p + b->n, s, k);
  b->n += k;
  b->p[b->n] = 0;
}

static void sb_printf(sbuf *b, const char *fmt, ...) {
  char tmp[512];
  va_list ap;
  va_start(ap, fmt);
  int k = vsnprintf(tmp, sizeof tmp, fmt, ap);
  va_end(ap);
  sb_put(b, tmp, (size_t)k);
}

/* MemberCompareLessThan, MP1Node.cpp:13-18 */
static int ent_less(const entry *a, int32_t id, int16_t port) {
  return a->id < id || (a->id == id && a->port < port);
}
static int ent_cmp(const void *x, const void *y) {
  const entry *a = (const entry *)x, *b = (const entry *)y;
  if (a->id != b->id) return a->id < b->id ? -1 : 1;
  if (a->port != b->port) return a->port < b->port ? -1 : 1;
  return 0;
}
static int lower_bound(const elist *l, int32_t id, int16_t port) {
  int lo = 0, hi = l->n;
  while (lo < hi) {
    int mid = (lo + hi) / 2;
    if (ent_less(&l->v[mid], id, port)) lo = mid + 1; else hi = mid;
  }
  return lo;
}
static void el_sort(elist *l) { qsort(l->v, (size_t)l->n, sizeof(entry), ent_cmp); }

/* ------------------------------------------------------------ simulation -- */
typedef struct node {
  int32_t id;
  int inited, in_group, failed;
  int64_t heartbeat;
  elist list;
  int mypos;
  mvec q;        /* mp1q */
} node;

typedef struct snap { int32_t *ids, *hbs; int n; } snap; /* SCALED: gossip payload snapshot */

struct oc_ctx {
  oc_config cfg;
  int n, t;
  node *nodes;
  oc_rand s1;
  int dropmsg;
  /* EmulNet */
  mvec buff;
  int32_t *sent, *recv; /* [MAX_NODES+1][MAX_TIME] in FAITHFUL */
  /* Log */
  sbuf dbg, out, tmp;
  int log_opened, log_first;
  /* SCALED network: snapshot + targets of every sender at the previous tick */
  snap *snaps, *snaps_next;
  int32_t *tgt, *ntgt, *tgt_next, *ntgt_next;
  oc_event *ev;
  size_t nev, evcap;
  int32_t *crash;
  /* SCALED join ramp (init_mode 2): the last tick the introducer ran */
  int intro_last;
  /* test telemetry: updateMyPos quirk firings and the largest start-tick gap self -> target */
  int64_t quirk_n, quirk_maxgap;
  /* SCALED msgcount analogue of the last tick (EmulNet.cpp:111,172 per entry message):
   * gossip entries node i put on the wire (fresh entries x targets) / received after loss */
  int32_t *mc_sent, *mc_recv;
};

static int is_scaled(const oc_ctx *c) { return c->cfg.mode == OC_SCALED; }

/* Address bytes: int32 id LE + int16 port (Member.h:29-55; EmulNet.cpp:74-75) */
static void addr_bytes(int32_t id, int16_t port, unsigned char b[6]) {
  memcpy(b, &id, 4);
  memcpy(b + 4, &port, 2);
}

/* strcmp(emsg->to.addr, myaddr->addr) == 0 (EmulNet.cpp:154): C-string compare of the 6 bytes */
static int addr_streq(int32_t a, int32_t b) {
  unsigned char x[7], y[7];
  addr_bytes(a, 0, x);
  addr_bytes(b, 0, y);
  x[6] = y[6] = 0;
  return strcmp((const char *)x, (const char *)y) == 0;
}

/* "%d.%d.%d.%d:%d" over signed char bytes (Log.cpp:73,118,129) */
static int fmt_addr(char *dst, int32_t id, int16_t port) {
  unsigned char b[6];
  addr_bytes(id, port, b);
  return sprintf(dst, "%d.%d.%d.%d:%d", (signed char)b[0], (signed char)b[1], (signed char)b[2],
                 (signed char)b[3], (int)port);
}

/* Log::LOG (Log.cpp:44-109): first record carries no address prefix; magic "131\n" once. */
static void log_line(oc_ctx *c, int32_t id, const char *text) {
  if (is_scaled(c)) return;
  char pre[64];
  pre[0] = 0;
  if (!c->log_opened) {
    c->log_opened = 1;
  } else {
    int k = fmt_addr(pre, id, 0);
    pre[k] = ' ';
    pre[k + 1] = 0;
  }
  if (!c->log_first) {
    int magic = 0;
    const char *m = "CS425";
    for (int i = 0; m[i]; i++) magic += m[i];
    sb_printf(&c->dbg, "%x\n", magic);
    c->log_first = 1;
  }
  sb_printf(&c->dbg, "\n %s", pre);
  sb_printf(&c->dbg, "[%d] ", c->t);
  sb_put(&c->dbg, text, strlen(text));
}

static void emit_event(oc_ctx *c, int32_t logger_idx, int kind, int32_t subject) {
  if (!is_scaled(c)) {
    char a[48], s[96];
    fmt_addr(a, subject, 0);
    sprintf(s, "Node %s %s at time %d", a, kind == OC_EV_ADD ? "joined" : "removed", c->t);
    log_line(c, c->nodes[logger_idx].id, s);
    return;
  }
  if (c->nev == c->evcap) {
    c->evcap = c->evcap ? 2 * c->evcap : 1024;
    c->ev = (oc_event *)realloc(c->ev, sizeof(oc_event) * c->evcap);
  }
  oc_event e = {c->t, logger_idx, kind, subject};
  c->ev[c->nev++] = e;
}

/* EmulNet::ENsend (EmulNet.cpp:87-118) */
static int en_send(oc_ctx *c, int32_t from, int32_t to, int type, int32_t id, int16_t port, int64_t hb, int size) {
  int draw = oc_rand_next(&c->s1) % 100;
  if (c->buff.n >= ENBUFFSIZE || size + EN_MSG_HDR >= MAX_MSG_SIZE ||
      (c->dropmsg && draw < (int)(c->cfg.drop_prob * 100)))
    return 0;
  msg m = {size, from, to, type, id, port, hb};
  mv_push(&c->buff, &m);
  c->sent[(size_t)from * MAX_TIME + (size_t)c->t]++;
  return size;
}

/* EmulNet::ENrecv (EmulNet.cpp:144-177): scan from the end, swap-with-last removal */
static void en_recv(oc_ctx *c, node *nd) {
  for (int i = c->buff.n - 1; i >= 0; i--) {
    if (addr_streq(c->buff.v[i].to, nd->id)) {
      msg m = c->buff.v[i];
      c->buff.v[i] = c->buff.v[c->buff.n - 1];
      c->buff.n--;
      mv_push(&nd->q, &m);
      c->recv[(size_t)nd->id * MAX_TIME + (size_t)c->t]++;
    }
  }
}

/* MP1Node::updateMyPos (MP1Node.cpp:308-322), including the `&&` quirk at :316 */
static void update_my_pos(oc_ctx *c, node *nd) {
  int p = lower_bound(&nd->list, nd->id, 0);
  if (p < nd->list.n && nd->list.v[p].id != nd->id) { /* the quirk fires: myPos = the next larger id */
    const int64_t gap = (int64_t)(int)(0.25 * (nd->list.v[p].id - 1)) - (int64_t)(int)(0.25 * (nd->id - 1));
    c->quirk_n++;
    if (gap > c->quirk_maxgap) c->quirk_maxgap = gap;
  }
  if (p == nd->list.n || (nd->list.v[p].id != nd->id && nd->list.v[p].port != 0)) {
    entry e = {nd->id, 0, nd->heartbeat, c->t};
    el_push(&nd->list, e);
    el_sort(&nd->list);
    p = lower_bound(&nd->list, nd->id, 0);
  }
  nd->mypos = p;
}

/* MP1Node::updatelistCallBack (MP1Node.cpp:259-301): returns 1 when inserted */
static int update_list(oc_ctx *c, int idx, int32_t id, int16_t port, int64_t hb) {
  node *nd = &c->nodes[idx];
  int p = lower_bound(&nd->list, id, port);
  if (p < nd->list.n && nd->list.v[p].id == id && nd->list.v[p].port == port) {
    if (nd->list.v[p].hb < hb) {
      nd->list.v[p].hb = hb;
      nd->list.v[p].ts = c->t;
    }
    return 0;
  }
  entry e = {id, port, hb, c->t};
  el_push(&nd->list, e);
  emit_event(c, idx, OC_EV_ADD, id);
  el_sort(&nd->list);
  return 1;
}

/* MP1Node::sendMemberList (MP1Node.cpp:360-395) */
static void send_member_list(oc_ctx *c, node *nd, int32_t to) {
  for (int k = 0; k < nd->list.n; k++) {
    entry *e = &nd->list.v[k];
    if (c->t - e->ts >= TFAIL) continue;
    en_send(c, nd->id, to, LIST, e->id, e->port, e->hb, LIST_SIZE);
  }
}

/* MP1Node::nodeLoopOps (MP1Node.cpp:404-495) */
static void node_loop_ops(oc_ctx *c, int idx, const entry *new_nodes, int n_new) {
  node *nd = &c->nodes[idx];
  int64_t now = c->t;
  update_my_pos(c, nd);
  nd->heartbeat++;
  nd->list.v[nd->mypos].hb = nd->heartbeat++;
  nd->list.v[nd->mypos].ts = now;
  entry me = nd->list.v[nd->mypos];
  int len = nd->list.n, numfailed = 0;
  for (int i = len - 1; i >= 0; --i) {
    int64_t diff = now - nd->list.v[i].ts;
    if (diff >= TFAIL) {
      numfailed++;
      if (diff >= TREMOVE) {
        int cur = nd->list.n;
        emit_event(c, idx, OC_EV_REMOVE, nd->list.v[i].id);
        entry tmp = nd->list.v[i];
        nd->list.v[i] = nd->list.v[cur - 1];
        nd->list.v[cur - 1] = tmp;
        nd->list.n--;
      }
    }
  }
  el_sort(&nd->list);
  nd->mypos = lower_bound(&nd->list, me.id, me.port);

  mt m;
  mt_seed(&m, oc_rd_seed(c->cfg.rd_seed, c->t, nd->id));
  uint32_t range = (uint32_t)nd->list.n; /* dist(0, size-1) */
  entry *gossip = (entry *)malloc(sizeof(entry) * (size_t)(n_new + FANOUT));
  int n = 0;
  for (int k = 0; k < n_new; k++) gossip[n++] = new_nodes[k];
  int32_t myid = nd->list.v[nd->mypos].id;
  int16_t myport = nd->list.v[nd->mypos].port;
  int numpot = nd->list.n - 1 - numfailed;
  int skipfailed = numpot > 0;
  while (n < FANOUT && n < numpot) {
    int ix = mt_uniform(&m, range);
    entry *e = &nd->list.v[ix];
    if (e->id != myid || e->port != myport) {
      if (skipfailed && (now - e->ts >= TFAIL)) continue;
      int found = 0;
      for (int k = 0; k < n; k++)
        if (gossip[k].id == e->id && gossip[k].port == e->port) { found = 1; break; }
      if (!found) gossip[n++] = *e;
    }
  }
  if (!is_scaled(c)) {
    for (int k = 0; k < n; k++) send_member_list(c, nd, gossip[k].id);
    free(gossip);
    return;
  }
  /* SCALED: one payload snapshot per sender (its fresh entries now), shared by every target */
  snap *s = &c->snaps_next[idx];
  s->n = 0;
  for (int k = 0; k < nd->list.n; k++) {
    entry *e = &nd->list.v[k];
    if (now - e->ts >= TFAIL) continue;
    s->ids[s->n] = e->id;
    s->hbs[s->n] = (int32_t)e->hb;
    s->n++;
  }
  c->ntgt_next[idx] = n;
  for (int k = 0; k < n; k++) c->tgt_next[(size_t)idx * FANOUT + k] = gossip[k].id - 1;
  if (c->mc_sent) c->mc_sent[idx] = s->n * n;  /* (oc_bench_sample's context counts nothing) */
  free(gossip);
}

/* MP1Node::nodeLoop + checkMessages + recvCallBack + joinreqCallBack (MP1Node.cpp:182-353) */
static void node_loop(oc_ctx *c, int idx) {
  node *nd = &c->nodes[idx];
  if (nd->failed) return;
  entry *newn = NULL;
  int n_new = 0, cap_new = 0;
  for (int k = 0; k < nd->q.n; k++) {
    msg *m = &nd->q.v[k];
    if (m->type == JOINREQ) {
      if (update_list(c, idx, m->id, m->port, m->hb)) {
        if (n_new == cap_new) {
          cap_new = cap_new ? 2 * cap_new : 8;
          newn = (entry *)realloc(newn, sizeof(entry) * (size_t)cap_new);
        }
        entry e = {m->id, m->port, m->hb, c->t};
        newn[n_new++] = e;
      }
      if (!is_scaled(c)) en_send(c, nd->id, m->id, JOINREP, 0, 0, 0, JOINREP_SIZE);
    } else if (m->type == JOINREP) {
      nd->in_group = 1;
    } else if (m->type == LIST) {
      update_list(c, idx, m->id, m->port, m->hb);
    }
  }
  nd->q.n = 0;
  if (nd->in_group) node_loop_ops(c, idx, newn, n_new);
  free(newn);
}

/* MP1Node::nodeStart -> initThisNode + introduceSelfToGroup (MP1Node.cpp:73-163) */
static void node_start(oc_ctx *c, int idx) {
  node *nd = &c->nodes[idx];
  nd->failed = 0;
  nd->inited = 1;
  nd->in_group = 0;
  nd->heartbeat = 0;
  nd->list.n = 0;
  if (nd->id == 1) { /* getJoinAddress() = 1:0 (MP1Node.cpp:511-519) */
    log_line(c, nd->id, "Starting up group...");
    update_my_pos(c, nd);
    nd->in_group = 1;
  } else {
    log_line(c, nd->id, "Trying to join...");
    /* SCALED: the introducer takes the JOINREQs of tick t-1 starters in mp1_run */
    if (!is_scaled(c)) en_send(c, nd->id, 1, JOINREQ, nd->id, 0, nd->heartbeat, LIST_SIZE);
  }
}

static uint32_t fmix32(uint32_t h) { /* murmur3 finalizer: a bijection of uint32 */
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  return h ^ (h >> 16);
}

/* SCALED keyed loss threshold: an entry is lost iff its 16-bit chunk < ceil(pct * 65536 / 100)
 * (gm_scaled.h s_drop_thresh) */
static uint32_t scaled_drop_thresh(int pct) {
  return pct <= 0 ? 0u : pct >= 100 ? 65536u : (uint32_t)((pct * 65536 + 99) / 100);
}

/* SCALED recv: every gossip list sent to this node at t-1, senders ascending,
 * entries ascending id, per-entry keyed drops. */
static void scaled_recv(oc_ctx *c, int idx) {
  for (int s = 0; s < c->n; s++) {
    for (int k = 0; k < c->ntgt[s]; k++) {
      if (c->tgt[(size_t)s * FANOUT + k] != idx) continue;
      snap *p = &c->snaps[s];
      int t_send = c->t - 1;
      int dropping = c->cfg.drop_pct > 0 && t_send >= c->cfg.drop_from && t_send < c->cfg.drop_to;
      uint32_t pair = (uint32_t)mix64(c->cfg.drop_seed ^ ((uint64_t)(uint32_t)t_send << 48) ^ ((uint64_t)s << 24) ^ (uint64_t)idx);
      for (int e = 0; e < p->n; e++) {
        if (dropping) { /* build-defined keyed loss: 16-bit half (col & 1) of one fmix32 per column pair */
          uint32_t col = (uint32_t)(p->ids[e] - 1);
          uint32_t v = (fmix32(pair ^ ((col >> 1) * 0x9E3779B9u)) >> (16 * (col & 1))) & 0xFFFFu;
          if (v < scaled_drop_thresh(c->cfg.drop_pct)) continue;
        }
        if (c->mc_recv) c->mc_recv[idx]++;
        update_list(c, idx, p->ids[e], 0, p->hbs[e]);
      }
    }
  }
}

static int ev_canon(const void *x, const void *y) {
  const oc_event *a = (const oc_event *)x, *b = (const oc_event *)y;
  if (a->logger != b->logger) return a->logger > b->logger ? -1 : 1; /* node phase: i descending */
  if (a->kind != b->kind) return a->kind < b->kind ? -1 : 1;         /* ADDs then REMOVEs */
  if (a->kind == OC_EV_ADD) return a->subject < b->subject ? -1 : (a->subject > b->subject);
  return a->subject > b->subject ? -1 : (a->subject < b->subject);
}

/* Application::mp1Run (Application.cpp:121-164) */
static void mp1_run(oc_ctx *c) {
  int t = c->t;
  if (!is_scaled(c)) {
    for (int i = 0; i < c->n; i++)
      if (t > (int)(0.25 * i) && !c->nodes[i].failed) en_recv(c, &c->nodes[i]);
    for (int i = c->n - 1; i >= 0; i--) {
      if (t == (int)(0.25 * i)) {
        node_start(c, i);
        sb_printf(&c->out, "%d-th introduced node is assigned with the address: %d:0\n", i, c->nodes[i].id);
      } else if (t > (int)(0.25 * i) && !c->nodes[i].failed) {
        node_loop(c, i);
        if (i == 0 && t % 500 == 0) {
          char s[64];
          sprintf(s, "@@time=%d", t);
          log_line(c, c->nodes[0].id, s);
        }
      }
    }
    return;
  }
  c->nev = 0;
  memset(c->mc_sent, 0, sizeof(int32_t) * (size_t)c->n);
  memset(c->mc_recv, 0, sizeof(int32_t) * (size_t)c->n);
  const int ramp = c->cfg.init_mode == 2;
  for (int i = c->n - 1; i >= 0; i--) {
    const int start = (int)(0.25 * i); /* Application.cpp:130,143 (STEP_RATE 0.25) */
    if (ramp && t == start) {
      node_start(c, i);
      if (i == 0) c->intro_last = t;
      continue;
    }
    if ((ramp && t < start) || c->nodes[i].failed) continue;
    scaled_recv(c, i);
    if (ramp) {
      node *nd = &c->nodes[i];
      if (i == 0) { /* JOINREQs of the nodes that started at t-1, ascending id (unbounded network) */
        for (int j = 1; j < c->n; j++) {
          if ((int)(0.25 * j) != t - 1) continue;
          msg m = {LIST_SIZE, j + 1, 1, JOINREQ, j + 1, 0, 0};
          mv_push(&nd->q, &m);
        }
      } else if (t == start + 2 && c->intro_last >= start + 1) { /* the introducer answered at start+1 */
        msg m = {JOINREP_SIZE, 1, i + 1, JOINREP, 0, 0, 0};
        mv_push(&nd->q, &m);
      }
    }
    node_loop(c, i);
    if (ramp && i == 0) c->intro_last = t;
  }
  qsort(c->ev, c->nev, sizeof(oc_event), ev_canon);
  snap *ts = c->snaps; c->snaps = c->snaps_next; c->snaps_next = ts;
  int32_t *tt = c->tgt; c->tgt = c->tgt_next; c->tgt_next = tt;
  tt = c->ntgt; c->ntgt = c->ntgt_next; c->ntgt_next = tt;
  memset(c->ntgt_next, 0, sizeof(int32_t) * (size_t)c->n);
}

/* Application::fail (Application.cpp:173-202) */
static void app_fail(oc_ctx *c) {
  int t = c->t;
  if (is_scaled(c)) {
    if (t == c->cfg.crash_tick)
      for (int k = 0; k < c->cfg.crash_count; k++) c->nodes[c->crash[k]].failed = 1;
    return;
  }
  char s[64];
  if (c->cfg.drop_msg && t == 50) c->dropmsg = 1;
  if (c->cfg.single_failure && t == 100) {
    int removed = oc_rand_next(&c->s1) % c->n;
    sprintf(s, "Node failed at time=%d", t);
    log_line(c, c->nodes[removed].id, s);
    c->nodes[removed].failed = 1;
  } else if (t == 100) {
    int removed = oc_rand_next(&c->s1) % c->n / 2;
    for (int i = removed; i < removed + c->n / 2; i++) {
      sprintf(s, "Node failed at time = %d", t);
      log_line(c, c->nodes[i].id, s);
      c->nodes[i].failed = 1;
    }
  }
  if (c->cfg.drop_msg && t == 300) c->dropmsg = 0;
}

typedef struct ck { uint64_t key; int32_t idx; } ck;
static int ck_cmp(const void *x, const void *y) {
  const ck *a = (const ck *)x, *b = (const ck *)y;
  if (a->key != b->key) return a->key < b->key ? -1 : 1;
  return a->idx - b->idx;
}
static int i32_cmp(const void *x, const void *y) { return *(const int32_t *)x - *(const int32_t *)y; }

int oc_crash_set(int n, int count, uint64_t seed, int32_t *out) {
  if (count < 0 || count > n) return -1;
  ck *k = (ck *)malloc(sizeof(ck) * (size_t)n);
  for (int i = 0; i < n; i++) {
    k[i].key = mix64(seed + 0x9E3779B97F4A7C15ULL * (uint64_t)(i + 1));
    k[i].idx = i;
  }
  qsort(k, (size_t)n, sizeof(ck), ck_cmp);
  for (int i = 0; i < count; i++) out[i] = k[i].idx;
  qsort(out, (size_t)count, sizeof(int32_t), i32_cmp);
  free(k);
  return 0;
}

oc_ctx *oc_create(const oc_config *cfg) {
  if (cfg->n <= 0) return NULL;
  if (cfg->mode == OC_SCALED && cfg->init_mode == 1 && cfg->init_t0 < 5) return NULL; /* hb >= 0 needs t0 >= 5 */
  /* the join ramp with keyed drops runs the updateMyPos quirk path (MP1Node.cpp:316) */
  if (cfg->mode == OC_FAITHFUL && cfg->n > MAX_NODES) return NULL; /* EmulNet.cpp:108 assert */
  oc_ctx *c = (oc_ctx *)calloc(1, sizeof(oc_ctx));
  c->cfg = *cfg;
  c->n = cfg->n;
  c->nodes = (node *)calloc((size_t)c->n, sizeof(node));
  for (int i = 0; i < c->n; i++) c->nodes[i].id = i + 1; /* ENinit: ids from 1 (EmulNet.cpp:74) */
  if (cfg->mode == OC_FAITHFUL) {
    c->sent = (int32_t *)calloc((size_t)(MAX_NODES + 1) * MAX_TIME, sizeof(int32_t));
    c->recv = (int32_t *)calloc((size_t)(MAX_NODES + 1) * MAX_TIME, sizeof(int32_t));
    for (int i = 0; i < c->n; i++) log_line(c, c->nodes[i].id, "APP"); /* Application.cpp:66 */
    oc_srand(&c->s1, cfg->time_seed); /* srand(time(NULL)), Application.cpp:50 and :96 */
    c->t = 0;
  } else {
    const int warm = cfg->init_mode == 1, ramp = cfg->init_mode == 2;
    const int t0 = warm ? cfg->init_t0 : 0;
    c->intro_last = -1;
    for (int i = 0; i < c->n; i++) {
      node *nd = &c->nodes[i];
      if (ramp) { /* join ramp: nobody started, empty lists (nodeStart at (int)(0.25 i)) */
        nd->list.v = (entry *)malloc(sizeof(entry) * (size_t)c->n);
        nd->list.cap = c->n;
        nd->list.n = 0;
        continue;
      }
      nd->inited = nd->in_group = 1;
      nd->heartbeat = warm ? 2 * t0 : 0;
      nd->list.v = (entry *)malloc(sizeof(entry) * (size_t)c->n);
      nd->list.cap = nd->list.n = c->n;
      for (int j = 0; j < c->n; j++) {
        entry e = {j + 1, 0, 0, 0};
        if (warm && j == i) {
          e.hb = 2 * t0 - 1;
          e.ts = t0;
        } else if (warm) {
          int a = (int)((mix64(cfg->init_seed ^ ((uint64_t)(uint32_t)i << 32) ^ (uint64_t)(uint32_t)j) >> 40) % 4);
          e.hb = 2 * (t0 - 1 - a) - 1;
          e.ts = t0 - a;
        }
        nd->list.v[j] = e;
      }
    }
    c->snaps = (snap *)calloc((size_t)c->n, sizeof(snap));
    c->snaps_next = (snap *)calloc((size_t)c->n, sizeof(snap));
    for (int i = 0; i < c->n; i++) {
      c->snaps[i].ids = (int32_t *)malloc(sizeof(int32_t) * (size_t)c->n);
      c->snaps[i].hbs = (int32_t *)malloc(sizeof(int32_t) * (size_t)c->n);
      c->snaps_next[i].ids = (int32_t *)malloc(sizeof(int32_t) * (size_t)c->n);
      c->snaps_next[i].hbs = (int32_t *)malloc(sizeof(int32_t) * (size_t)c->n);
    }
    c->tgt = (int32_t *)calloc((size_t)c->n * FANOUT, sizeof(int32_t));
    c->tgt_next = (int32_t *)calloc((size_t)c->n * FANOUT, sizeof(int32_t));
    c->ntgt = (int32_t *)calloc((size_t)c->n, sizeof(int32_t));
    c->ntgt_next = (int32_t *)calloc((size_t)c->n, sizeof(int32_t));
    c->mc_sent = (int32_t *)calloc((size_t)c->n, sizeof(int32_t));
    c->mc_recv = (int32_t *)calloc((size_t)c->n, sizeof(int32_t));
    c->crash = (int32_t *)calloc((size_t)(cfg->crash_count > 0 ? cfg->crash_count : 1), sizeof(int32_t));
    if (cfg->crash_count > 0 && oc_crash_set(c->n, cfg->crash_count, cfg->crash_seed, c->crash)) {
      oc_destroy(c);
      return NULL;
    }
    c->t = ramp ? 0 : t0 + 1; /* converged state is "as of tick t0"; the ramp starts at tick 0 */
  }
  return c;
}

void oc_destroy(oc_ctx *c) {
  if (!c) return;
  for (int i = 0; i < c->n; i++) {
    free(c->nodes[i].list.v);
    free(c->nodes[i].q.v);
    if (c->snaps) { free(c->snaps[i].ids); free(c->snaps[i].hbs); }
    if (c->snaps_next) { free(c->snaps_next[i].ids); free(c->snaps_next[i].hbs); }
  }
  free(c->snaps); free(c->snaps_next);
  free(c->tgt); free(c->tgt_next); free(c->ntgt); free(c->ntgt_next);
  free(c->mc_sent); free(c->mc_recv);
  free(c->crash); free(c->ev);
  free(c->nodes);
  free(c->buff.v);
  free(c->sent);
  free(c->recv);
  free(c->dbg.p); free(c->out.p); free(c->tmp.p);
  free(c);
}

int oc_tick(oc_ctx *c) {
  if (!is_scaled(c) && c->t >= MAX_TIME) return -1; /* EmulNet.cpp:109 assert */
  mp1_run(c);
  app_fail(c);
  c->t++;
  return 0;
}

int oc_time(const oc_ctx *c) { return c->t; }

const char *oc_dbg_log(oc_ctx *c, size_t *len) {
  *len = c->dbg.n;
  return c->dbg.p ? c->dbg.p : "";
}

const char *oc_stdout(oc_ctx *c, size_t *len) {
  *len = c->out.n;
  return c->out.p ? c->out.p : "";
}

/* EmulNet::ENcleanup (EmulNet.cpp:184-220), incl. the node-67 special case */
const char *oc_msgcount(oc_ctx *c, size_t *len) {
  c->tmp.n = 0;
  if (is_scaled(c)) { *len = 0; return ""; }
  for (int i = 1; i <= c->n; i++) {
    sb_printf(&c->tmp, "node %3d ", i);
    unsigned st = 0, rt = 0;
    for (int j = 0; j < c->t; j++) {
      int s = c->sent[(size_t)i * MAX_TIME + j], r = c->recv[(size_t)i * MAX_TIME + j];
      st += (unsigned)s;
      rt += (unsigned)r;
      if (i != 67) {
        sb_printf(&c->tmp, " (%4d, %4d)", s, r);
        if (j % 10 == 9) sb_printf(&c->tmp, "\n         ");
      } else {
        sb_printf(&c->tmp, "special %4d %4d %4d\n", j, s, r);
      }
    }
    sb_printf(&c->tmp, "\n");
    sb_printf(&c->tmp, "node %3d sent_total %6u  recv_total %6u\n\n", i, st, rt);
  }
  *len = c->tmp.n;
  return c->tmp.p;
}

/* SCALED: per-node gossip entries sent (fresh entries x targets, before loss) and received
 * (after loss) in the last tick; JOINREQ/JOINREP of the ramp are not counted */
int oc_last_msgcount(const oc_ctx *c, int32_t *sent, int32_t *recv) {
  if (!is_scaled(c)) return -1;
  memcpy(sent, c->mc_sent, sizeof(int32_t) * (size_t)c->n);
  memcpy(recv, c->mc_recv, sizeof(int32_t) * (size_t)c->n);
  return 0;
}

/* state of the tick just finished, in oracle/shim/dump_main.cpp's line format */
const char *oc_dump(oc_ctx *c, size_t *len) {
  c->tmp.n = 0;
  int t = c->t - 1;
  for (int i = 0; i < c->n; i++) {
    node *nd = &c->nodes[i];
    sb_printf(&c->tmp, "%d %d %d %d %d %ld %d", t, i, nd->inited, nd->in_group, nd->failed, (long)nd->heartbeat,
              nd->list.n);
    for (int k = 0; k < nd->list.n; k++)
      sb_printf(&c->tmp, " %d:%ld:%ld", nd->list.v[k].id, (long)nd->list.v[k].hb, (long)nd->list.v[k].ts);
    sb_put(&c->tmp, "\n", 1);
  }
  *len = c->tmp.n;
  return c->tmp.p ? c->tmp.p : "";
}

size_t oc_events(oc_ctx *c, const oc_event **ev) {
  *ev = c->ev;
  return c->nev;
}

int oc_row(oc_ctx *c, int r, int32_t *hb, int32_t *ts) {
  if (r < 0 || r >= c->n) return -1;
  for (int j = 0; j < c->n; j++) hb[j] = ts[j] = -1;
  node *nd = &c->nodes[r];
  for (int k = 0; k < nd->list.n; k++) {
    int j = nd->list.v[k].id - 1;
    if (j < 0 || j >= c->n) continue;
    hb[j] = (int32_t)nd->list.v[k].hb;
    ts[j] = (int32_t)nd->list.v[k].ts;
  }
  return 0;
}

/* SCALED: the gossip targets every node drew in the last tick (row-major [n][FANOUT], node indices)
 * and their counts -- the sends the next tick delivers */
int oc_targets(const oc_ctx *c, int32_t *tgt, int32_t *ntgt) {
  if (!is_scaled(c)) return -1;
  memcpy(tgt, c->tgt, sizeof(int32_t) * (size_t)c->n * FANOUT);
  memcpy(ntgt, c->ntgt, sizeof(int32_t) * (size_t)c->n);
  return 0;
}

/* SCALED (converged start, no join ramp): replace the whole state between two ticks by one read
 * from elsewhere -- the oracle's own oc_row / oc_node / oc_targets, or the HIP path's
 * gm_read_table / gm_read_nodes / gm_read_targets, which are bit-exact to them: every row's
 * members (hb / ts per column, -1 = absent; sorted by id as every tick leaves them), heartbeat
 * counters and crash flags, and the last tick's gossip targets. The payload each target receives
 * next (the sender's fresh entries at t - 1, node_loop_ops' snapshot) follows from the rows. `t`
 * is the next tick to run. Measurement infrastructure (scripts/cpu_hour.py): a long CPU run
 * continues from a state the GPU reached in seconds. */
int oc_load_scaled(oc_ctx *c, int t, const int32_t *hb, const int32_t *ts, const int32_t *heartbeat,
                   const int32_t *failed, const int32_t *tgt, const int32_t *ntgt) {
  if (!is_scaled(c) || c->cfg.init_mode == 2 || t < 1) return -1;
  const size_t n = (size_t)c->n;
  for (size_t i = 0; i < n; i++) {
    node *nd = &c->nodes[i];
    nd->list.n = 0;
    for (size_t j = 0; j < n; j++) {
      if (hb[i * n + j] < 0) continue;
      entry e = {(int32_t)j + 1, 0, hb[i * n + j], ts[i * n + j]};
      el_push(&nd->list, e);
    }
    nd->heartbeat = heartbeat[i];
    nd->failed = failed[i] != 0;
    nd->inited = nd->in_group = 1;
    nd->q.n = 0;
    snap *s = &c->snaps[i];  /* the sends of tick t - 1 (node_loop_ops) */
    s->n = 0;
    for (int k = 0; k < nd->list.n; k++) {
      const entry *e = &nd->list.v[k];
      if ((t - 1) - e->ts >= TFAIL) continue;
      s->ids[s->n] = e->id;
      s->hbs[s->n] = (int32_t)e->hb;
      s->n++;
    }
    if (ntgt[i] < 0 || ntgt[i] > FANOUT) return -1;
    c->ntgt[i] = ntgt[i];  /* a node failed at the end of t - 1 still sent in t - 1 */
    for (int k = 0; k < FANOUT; k++) c->tgt[i * FANOUT + k] = k < ntgt[i] ? tgt[i * FANOUT + k] : 0;
  }
  memset(c->ntgt_next, 0, sizeof(int32_t) * n);
  c->t = t;
  return 0;
}

/* SCALED: fail these nodes now, i.e. at the end of the tick just run (the host side of
 * Application::fail, Application.cpp:184-196, with the victims chosen by the caller) */
int oc_set_failed(oc_ctx *c, const int32_t *idx, int k) {
  if (!is_scaled(c)) return -1;
  for (int j = 0; j < k; j++) {
    if (idx[j] < 0 || idx[j] >= c->n) return -1;
    c->nodes[idx[j]].failed = 1;
  }
  return 0;
}

int oc_node(oc_ctx *c, int r, int32_t *st) {
  if (r < 0 || r >= c->n) return -1;
  node *nd = &c->nodes[r];
  st[0] = nd->inited;
  st[1] = nd->in_group;
  st[2] = nd->failed;
  st[3] = (int32_t)nd->heartbeat;
  return 0;
}

/* CPU baseline sample (bench.py cpu_baseline leg): time `nodes` node-ticks of the
 * SCALED full-membership workload at cluster size n through the same restated
 * code paths (updatelistCallBack per delivered entry, nodeLoopOps sweep + sort +
 * gossip draw), without materialising the other n - nodes member lists. Each
 * sampled observer holds all n subjects (converged regime) and receives `lists`
 * gossip lists of n fresh entries. Stops after min_seconds or max_nodes. */
int oc_bench_sample(int n, int lists, int max_nodes, double min_seconds, int *out_nodes, double *out_seconds) {
  if (n < 8 || lists < 0 || max_nodes <= 0) return -1;
  oc_config cfg = {0};
  cfg.mode = OC_SCALED;
  cfg.n = n;
  cfg.rd_seed = 7;
  oc_ctx *c = (oc_ctx *)calloc(1, sizeof(oc_ctx));
  c->cfg = cfg;
  c->n = n;
  c->t = 40;
  c->nodes = (node *)calloc((size_t)n, sizeof(node));
  for (int i = 0; i < n; i++) c->nodes[i].id = i + 1;
  c->snaps_next = (snap *)calloc((size_t)n, sizeof(snap));
  c->tgt_next = (int32_t *)calloc((size_t)n * FANOUT, sizeof(int32_t));
  c->ntgt_next = (int32_t *)calloc((size_t)n, sizeof(int32_t));
  /* sender payloads: every subject fresh, heartbeat a little ahead of the observer's */
  snap *pay = (snap *)calloc((size_t)(lists > 0 ? lists : 1), sizeof(snap));
  uint64_t z = 12345;
  for (int k = 0; k < lists; k++) {
    pay[k].ids = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
    pay[k].hbs = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
    pay[k].n = n;
    for (int j = 0; j < n; j++) {
      z = mix64(z + 1);
      pay[k].ids[j] = j + 1;
      pay[k].hbs[j] = 70 + (int32_t)(z % 4);
    }
  }
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  int done = 0;
  double el = 0;
  while (done < max_nodes) {
    int r = (int)(mix64((uint64_t)done * 7919 + 1) % (uint64_t)n);
    node *nd = &c->nodes[r];
    nd->inited = nd->in_group = 1;
    nd->heartbeat = 2 * c->t;
    nd->list.v = (entry *)malloc(sizeof(entry) * (size_t)n);
    nd->list.cap = nd->list.n = n;
    for (int j = 0; j < n; j++) {
      entry e = {j + 1, 0, 70, c->t - 1 - (j % 3)};
      nd->list.v[j] = e;
    }
    c->snaps_next[r].ids = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
    c->snaps_next[r].hbs = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
    /* the measured node-tick: merge every delivered list, then nodeLoopOps */
    for (int k = 0; k < lists; k++)
      for (int e = 0; e < pay[k].n; e++) update_list(c, r, pay[k].ids[e], 0, pay[k].hbs[e]);
    node_loop(c, r);
    free(nd->list.v);
    nd->list.v = NULL;
    nd->list.n = nd->list.cap = 0;
    free(c->snaps_next[r].ids);
    free(c->snaps_next[r].hbs);
    c->snaps_next[r].ids = c->snaps_next[r].hbs = NULL;
    done++;
    clock_gettime(CLOCK_MONOTONIC, &t1);
    el = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    if (el >= min_seconds) break;
  }
  *out_nodes = done;
  *out_seconds = el;
  for (int k = 0; k < lists; k++) { free(pay[k].ids); free(pay[k].hbs); }
  free(pay);
  free(c->snaps_next);
  free(c->tgt_next);
  free(c->ntgt_next);
  free(c->ev);
  free(c->nodes);
  free(c);
  return 0;
}

/* ===================================================================== PARTIAL
 * V-entry views (scenario S-C): the reference protocol with
 * every membership list capped at V entries. The reference is full-membership
 * only, so the semantics below are build-defined; each step cites the reference
 * rule it keeps. This restatement IS the specification of GM_MODE_PARTIAL.
 *
 *  - entry (id, hb); its timestamp is the tick the heartbeat was produced:
 *    every live node's self heartbeat at tick t is 2t-1 (MP1Node.cpp:412-415
 *    bumps twice per nodeLoopOps), so ts = (hb+1)/2 travels with the heartbeat
 *    (a bounded view churns: stamping ts = receive tick, as the full list does,
 *    would let a crashed node's entry circulate forever as "fresh");
 *  - merge (updatelistCallBack, MP1Node.cpp:259-301): per id keep the largest hb;
 *    absent ids are inserted; every list delivered to the node is merged (EmulNet.cpp:144-177);
 *  - self bump; sweep (MP1Node.cpp:426-444): age >= TFAIL counts toward numfailed,
 *    age >= TREMOVE removes (REMOVE event);
 *  - eviction to V: self first, then the largest hb (freshest), ties broken by a
 *    keyed bijective hash of the id (op_evict_key: view_seed, t, observer); evictions are silent; ids present
 *    after the tick and absent before are joins (ADD events);
 *  - numfailed = removed + stale entries of the final list; gossip draw over the
 *    final list in id order exactly as MP1Node.cpp:449-489; the sent list is the
 *    final list's fresh entries (sendMemberList, MP1Node.cpp:360-395);
 *  - drops keyed by (t_send, src, dst, id-1): top 16 bits of fmix32 of the pair hash ^ (id-1)
 *    below ceil(pct * 65536 / 100); crash set at the end
 *    of crash_tick; warm start at t0: self {2t0-1} plus V-1 distinct peers chosen by
 *    mix64(view_seed ^ i<<32 ^ j) % n, peer hb 2(t0-1-a)-1, a = mix64(init_seed ^
 *    i<<32 ^ p)>>40 % 4. */
typedef struct pnode { int32_t *ids, *hbs; int cnt; int32_t hbctr; int failed; } pnode;
struct op_ctx {
  op_config cfg;
  int n, t, V;
  pnode *nd;
  snap *snaps, *snaps_next;         /* sent lists of the previous / current tick */
  int32_t *tgt, *tgt_next, *ntgt, *ntgt_next;
  int32_t *crash;
  oc_event *ev;
  int nev, evcap;
  sbuf dump;
  /* per-receiver sender lists of this tick's deliveries, senders ascending (CSR) */
  int32_t *rcv_off, *rcv_src;
  /* scratch */
  int32_t *cid, *chb, *cown;
  int ccap;
  /* msgcount analogue of the last tick: entries put on the wire / received after loss */
  int32_t *mc_sent, *mc_recv;
};

static void op_emit(op_ctx *c, int logger, int kind, int32_t subject) {
  if (c->nev == c->evcap) {
    c->evcap = c->evcap ? 2 * c->evcap : 1024;
    c->ev = (oc_event *)realloc(c->ev, sizeof(oc_event) * (size_t)c->evcap);
  }
  oc_event e = {c->t, logger, kind, subject};
  c->ev[c->nev++] = e;
}

/* eviction tie-break: fmix32(id ^ (uint32)mix64(mix64(view_seed ^ t) ^ obs)) -- distinct ids,
 * distinct keys (fmix32 is a bijection) */
uint64_t op_evict_key(uint64_t view_seed, int32_t t, int32_t obs, int32_t id) {
  uint32_t s = (uint32_t)mix64(mix64(view_seed ^ (uint64_t)(uint32_t)t) ^ (uint64_t)(uint32_t)obs);
  return fmix32((uint32_t)id ^ s);
}

op_ctx *op_create(const op_config *cfg) {
  if (cfg->n < 2 || cfg->v < 2 || cfg->v > 64 || cfg->v > cfg->n || cfg->init_t0 < 5) return NULL;
  op_ctx *c = (op_ctx *)calloc(1, sizeof(op_ctx));
  c->cfg = *cfg;
  c->n = cfg->n;
  c->V = cfg->v;
  c->t = cfg->init_t0 + 1;
  const int n = c->n, V = c->V, t0 = cfg->init_t0;
  c->nd = (pnode *)calloc((size_t)n, sizeof(pnode));
  for (int i = 0; i < n; i++) {
    pnode *p = &c->nd[i];
    p->ids = (int32_t *)malloc(sizeof(int32_t) * (size_t)V);
    p->hbs = (int32_t *)malloc(sizeof(int32_t) * (size_t)V);
    p->hbctr = 2 * t0;
    p->ids[0] = i + 1;
    p->hbs[0] = 2 * t0 - 1;
    p->cnt = 1;
    for (uint64_t j = 0; p->cnt < V; j++) {
      int32_t q = (int32_t)(mix64(cfg->view_seed ^ ((uint64_t)(uint32_t)i << 32) ^ j) % (uint64_t)n);
      int dup = q == i;
      for (int k = 1; k < p->cnt && !dup; k++) dup = p->ids[k] == q + 1;
      if (dup) continue;
      int a = (int)((mix64(cfg->init_seed ^ ((uint64_t)(uint32_t)i << 32) ^ (uint64_t)(uint32_t)q) >> 40) % 4);
      p->ids[p->cnt] = q + 1;
      p->hbs[p->cnt] = 2 * (t0 - 1 - a) - 1;
      p->cnt++;
    }
    /* keep the list sorted by id (the reference's memberList order) */
    for (int a = 1; a < p->cnt; a++)
      for (int b = a; b > 0 && p->ids[b - 1] > p->ids[b]; b--) {
        int32_t x = p->ids[b]; p->ids[b] = p->ids[b - 1]; p->ids[b - 1] = x;
        x = p->hbs[b]; p->hbs[b] = p->hbs[b - 1]; p->hbs[b - 1] = x;
      }
  }
  c->snaps = (snap *)calloc((size_t)n, sizeof(snap));
  c->snaps_next = (snap *)calloc((size_t)n, sizeof(snap));
  for (int i = 0; i < n; i++) {
    c->snaps[i].ids = (int32_t *)malloc(sizeof(int32_t) * (size_t)V);
    c->snaps[i].hbs = (int32_t *)malloc(sizeof(int32_t) * (size_t)V);
    c->snaps_next[i].ids = (int32_t *)malloc(sizeof(int32_t) * (size_t)V);
    c->snaps_next[i].hbs = (int32_t *)malloc(sizeof(int32_t) * (size_t)V);
  }
  c->tgt = (int32_t *)calloc((size_t)n * FANOUT, sizeof(int32_t));
  c->tgt_next = (int32_t *)calloc((size_t)n * FANOUT, sizeof(int32_t));
  c->ntgt = (int32_t *)calloc((size_t)n, sizeof(int32_t));
  c->ntgt_next = (int32_t *)calloc((size_t)n, sizeof(int32_t));
  c->crash = (int32_t *)calloc((size_t)(cfg->crash_count > 0 ? cfg->crash_count : 1), sizeof(int32_t));
  if (cfg->crash_count > 0) oc_crash_set(n, cfg->crash_count, cfg->crash_seed, c->crash);
  c->rcv_off = (int32_t *)calloc((size_t)n + 1, sizeof(int32_t));
  c->rcv_src = (int32_t *)calloc((size_t)n * FANOUT + 1, sizeof(int32_t));
  c->mc_sent = (int32_t *)calloc((size_t)n, sizeof(int32_t));
  c->mc_recv = (int32_t *)calloc((size_t)n, sizeof(int32_t));
  return c;
}

void op_destroy(op_ctx *c) {
  if (!c) return;
  for (int i = 0; i < c->n; i++) {
    free(c->nd[i].ids); free(c->nd[i].hbs);
    free(c->snaps[i].ids); free(c->snaps[i].hbs);
    free(c->snaps_next[i].ids); free(c->snaps_next[i].hbs);
  }
  free(c->nd); free(c->snaps); free(c->snaps_next);
  free(c->tgt); free(c->tgt_next); free(c->ntgt); free(c->ntgt_next);
  free(c->crash); free(c->ev); free(c->dump.p);
  free(c->cid); free(c->chb); free(c->cown);
  free(c->rcv_off); free(c->rcv_src);
  free(c->mc_sent); free(c->mc_recv);
  free(c);
}

typedef struct pcand { int32_t id, hb, own; uint64_t key; } pcand;
static int pc_evict_cmp(const void *x, const void *y) { /* self first, hb desc, key asc */
  const pcand *a = (const pcand *)x, *b = (const pcand *)y;
  if (a->own != b->own && (a->own == 2 || b->own == 2)) return a->own == 2 ? -1 : 1;
  if (a->hb != b->hb) return a->hb > b->hb ? -1 : 1;
  return a->key < b->key ? -1 : (a->key > b->key);
}
static int pc_id_cmp(const void *x, const void *y) {
  const pcand *a = (const pcand *)x, *b = (const pcand *)y;
  return a->id - b->id;
}

static int pc_idown_cmp(const void *x, const void *y) { /* id asc, then hb desc */
  const pcand *a = (const pcand *)x, *b = (const pcand *)y;
  if (a->id != b->id) return a->id < b->id ? -1 : 1;
  return (a->hb < b->hb) - (a->hb > b->hb);
}

static void op_node(op_ctx *c, int i, pcand *m) {
  const int t = c->t, V = c->V;
  pnode *p = &c->nd[i];
  int cnt = 0;
  for (int k = 0; k < p->cnt; k++) { m[cnt].id = p->ids[k]; m[cnt].hb = p->hbs[k]; m[cnt].own = 1; cnt++; }
  /* lists delivered to i: every sender that targeted i at t-1 (BSP, order-free for the table) */
  const int t_send = t - 1;
  const int dropping = c->cfg.drop_pct > 0 && t_send >= c->cfg.drop_from && t_send < c->cfg.drop_to;
  const int nrcv = c->rcv_off[i + 1] - c->rcv_off[i];
  for (int q = 0; q < nrcv; q++) {
    const int s = c->rcv_src[c->rcv_off[i] + q];
    const snap *sp = &c->snaps[s];
    uint32_t pair = (uint32_t)mix64(c->cfg.drop_seed ^ ((uint64_t)(uint32_t)t_send << 48) ^ ((uint64_t)s << 24) ^ (uint64_t)i);
    for (int e = 0; e < sp->n; e++) {
      if (dropping) { /* lost iff the top 16 bits of fmix32(pair ^ (id-1)) fall below ceil(pct*65536/100) */
        uint32_t h = fmix32(pair ^ (uint32_t)(sp->ids[e] - 1));
        if ((h >> 16) < scaled_drop_thresh(c->cfg.drop_pct)) continue;
      }
      m[cnt].id = sp->ids[e]; m[cnt].hb = sp->hbs[e]; m[cnt].own = 0; cnt++;
      c->mc_recv[i]++;
    }
  }
  /* merge per id (updatelistCallBack): the largest hb; "own" if the id was in i's list */
  qsort(m, (size_t)cnt, sizeof(pcand), pc_idown_cmp);
  {
    int w = 0;
    for (int k = 0; k < cnt; k++) {
      if (w > 0 && m[w - 1].id == m[k].id) { m[w - 1].own |= m[k].own; continue; }
      m[w++] = m[k];
    }
    cnt = w;
  }
  /* self bump (heartbeat++; myPos->setheartbeat(heartbeat++)) */
  int selfk = -1;
  for (int k = 0; k < cnt; k++) if (m[k].id == i + 1) selfk = k;
  if (selfk < 0) { fprintf(stderr, "partial: node %d lost its own entry\n", i); abort(); }
  p->hbctr++;
  m[selfk].hb = p->hbctr++;
  m[selfk].own = 2;
  /* sweep */
  int removed = 0, w = 0;
  for (int k = 0; k < cnt; k++) {
    int age = t - (m[k].hb + 1) / 2;
    if (age >= TREMOVE) {
      removed++;
      if (m[k].own) op_emit(c, i, OC_EV_REMOVE, m[k].id);
      continue;
    }
    m[w++] = m[k];
  }
  cnt = w;
  /* evict to V */
  if (cnt > V) {
    for (int k = 0; k < cnt; k++) m[k].key = op_evict_key(c->cfg.view_seed, t, i, m[k].id);
    qsort(m, (size_t)cnt, sizeof(pcand), pc_evict_cmp);
    cnt = V;
  }
  qsort(m, (size_t)cnt, sizeof(pcand), pc_id_cmp);
  int nfail = removed;
  for (int k = 0; k < cnt; k++) {
    if (!m[k].own) op_emit(c, i, OC_EV_ADD, m[k].id);
    if (t - (m[k].hb + 1) / 2 >= TFAIL) nfail++;
  }
  p->cnt = cnt;
  for (int k = 0; k < cnt; k++) { p->ids[k] = m[k].id; p->hbs[k] = m[k].hb; }
  /* gossip draw (MP1Node.cpp:449-489) over the final list in id order */
  int numpot = cnt - 1 - nfail, ng = 0;
  int32_t g[FANOUT];
  if (numpot > 0) {
    mt r;
    mt_seed(&r, oc_rd_seed(c->cfg.rd_seed, t, i + 1));
    while (ng < FANOUT && ng < numpot) {
      int ix = mt_uniform(&r, (uint32_t)cnt);
      if (m[ix].id == i + 1) continue;
      if (t - (m[ix].hb + 1) / 2 >= TFAIL) continue;
      int dup = 0;
      for (int q = 0; q < ng; q++) dup |= g[q] == m[ix].id - 1;
      if (!dup) g[ng++] = m[ix].id - 1;
    }
  }
  c->ntgt_next[i] = ng;
  for (int q = 0; q < ng; q++) c->tgt_next[(size_t)i * FANOUT + q] = g[q];
  snap *sn = &c->snaps_next[i];
  sn->n = 0;
  for (int k = 0; k < cnt; k++)
    if (t - (m[k].hb + 1) / 2 < TFAIL) { sn->ids[sn->n] = m[k].id; sn->hbs[sn->n] = m[k].hb; sn->n++; }
  c->mc_sent[i] = sn->n * ng;
}

int op_tick(op_ctx *c) {
  const int n = c->n;
  c->nev = 0;
  memset(c->mc_sent, 0, sizeof(int32_t) * (size_t)n);
  memset(c->mc_recv, 0, sizeof(int32_t) * (size_t)n);
  /* counting sort of last tick's (sender, target) pairs by target, senders ascending */
  memset(c->rcv_off, 0, sizeof(int32_t) * (size_t)(n + 1));
  for (int s = 0; s < n; s++)
    for (int q = 0; q < c->ntgt[s]; q++) c->rcv_off[c->tgt[(size_t)s * FANOUT + q] + 1]++;
  for (int i = 0; i < n; i++) c->rcv_off[i + 1] += c->rcv_off[i];
  {
    int32_t *fill = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
    memcpy(fill, c->rcv_off, sizeof(int32_t) * (size_t)n);
    for (int s = 0; s < n; s++)
      for (int q = 0; q < c->ntgt[s]; q++) c->rcv_src[fill[c->tgt[(size_t)s * FANOUT + q]]++] = s;
    free(fill);
  }
  int kmax = 0; /* candidates of a node: its own list + every delivered list */
  for (int i = 0; i < n; i++) kmax = c->rcv_off[i + 1] - c->rcv_off[i] > kmax ? c->rcv_off[i + 1] - c->rcv_off[i] : kmax;
  pcand *m = (pcand *)malloc(sizeof(pcand) * (size_t)c->V * (size_t)(kmax + 2));
  for (int i = n - 1; i >= 0; i--) {
    c->ntgt_next[i] = 0;
    c->snaps_next[i].n = 0;
    if (c->nd[i].failed) continue;
    op_node(c, i, m);
  }
  free(m);
  qsort(c->ev, (size_t)c->nev, sizeof(oc_event), ev_canon);
  snap *ts = c->snaps; c->snaps = c->snaps_next; c->snaps_next = ts;
  int32_t *tt = c->tgt; c->tgt = c->tgt_next; c->tgt_next = tt;
  tt = c->ntgt; c->ntgt = c->ntgt_next; c->ntgt_next = tt;
  if (c->t == c->cfg.crash_tick)
    for (int k = 0; k < c->cfg.crash_count; k++) c->nd[c->crash[k]].failed = 1;
  c->t++;
  return 0;
}

int op_time(const op_ctx *c) { return c->t; }

/* per-node entries sent (fresh entries of the final list x targets, before loss) and
 * received (entries of the merged lists that survived the loss) in the last tick */
void op_last_msgcount(const op_ctx *c, int32_t *sent, int32_t *recv) {
  memcpy(sent, c->mc_sent, sizeof(int32_t) * (size_t)c->n);
  memcpy(recv, c->mc_recv, sizeof(int32_t) * (size_t)c->n);
}

size_t op_events(op_ctx *c, const oc_event **ev) {
  *ev = c->ev;
  return (size_t)c->nev;
}

const char *op_dump(op_ctx *c, size_t *len) {
  c->dump.n = 0;
  const int t = c->t - 1;
  for (int i = 0; i < c->n; i++) {
    const pnode *p = &c->nd[i];
    sb_printf(&c->dump, "%d %d 1 1 %d %d %d", t, i, p->failed, p->hbctr, p->cnt);
    for (int k = 0; k < p->cnt; k++) sb_printf(&c->dump, " %d:%d:%d", p->ids[k], p->hbs[k], (p->hbs[k] + 1) / 2);
    sb_put(&c->dump, "\n", 1);
  }
  *len = c->dump.n;
  return c->dump.p ? c->dump.p : "";
}

/* test telemetry: [0] = updateMyPos quirk firings so far, [1] = largest start-tick gap
 * between the node and the entry the quirk rewrote */
void oc_quirks(const oc_ctx *c, int64_t out[2]) {
  out[0] = c->quirk_n;
  out[1] = c->quirk_maxgap;
}
