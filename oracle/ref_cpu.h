/* ref_cpu.h -- CPU restatement of the reference gossip-membership simulator.
 *
 * TEST INFRASTRUCTURE ONLY (the parity oracle). Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product (libgm, ./Application)
 * never links it.
 *
 * Restates, in plain C, the single-threaded discrete-time simulator of
 * patour/distributed-membership:
 *   Application::run/mp1Run/fail      Application.cpp:90-202
 *   MP1Node (join, merge, sweep, gossip) MP1Node.cpp:73-495
 *   EmulNet (ENsend/ENrecv/ENcleanup) EmulNet.cpp:87-220
 *   Log (dbg.log byte contract)       Log.cpp:44-131
 *   Params::setparams                 Params.cpp:19-40
 * plus the seed contract of SURVEY.md Appendix B (S1 = glibc rand seeded with
 * TIME_SEED; S2 = mt19937 seeded per (tick, node id) from RD_SEED).
 *
 * Two modes:
 *   OC_FAITHFUL  the reference itself: EmulNet buffer cap 30000, per-entry
 *                messages, swap-with-last delivery order, S1 drop draws.
 *                Pinned bit-for-bit by tests/golden/ (generated from the
 *                seeded reference in oracle/_ref).
 *   OC_SCALED    the build-defined large-N regime: unbounded
 *                network, converged start, drops keyed by (tick,src,dst,col),
 *                binary event stream. Same protocol code paths otherwise.
 */
#ifndef GM_REF_CPU_H
#define GM_REF_CPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { OC_FAITHFUL = 0, OC_SCALED = 1 };
enum { OC_EV_ADD = 1, OC_EV_REMOVE = 2 };

typedef struct oc_config {
  int mode;
  int n;               /* EN_GPSZ (= MAX_NNB) */
  int single_failure;  /* SINGLE_FAILURE */
  int drop_msg;        /* DROP_MSG */
  double drop_prob;    /* MSG_DROP_PROB */
  uint32_t time_seed;  /* S1: srand(TIME_SEED) */
  uint64_t rd_seed;    /* S2: RD_SEED */
  /* SCALED only */
  int crash_tick;      /* tick at whose end the crash set fails (-1: none) */
  int crash_count;     /* size of the crash set */
  uint64_t crash_seed; /* crash-set selection seed */
  int drop_pct;        /* per-entry drop percentage in SCALED mode */
  int drop_from, drop_to; /* drops apply to sends at ticks in [drop_from, drop_to) */
  uint64_t drop_seed;
  int init_mode;       /* 0 cold converged start, 1 warm converged start at init_t0, 2 join ramp (gm_abi.h) */
  int init_t0;
  uint64_t init_seed;
} oc_config;

typedef struct oc_event { int32_t t, logger, kind, subject; } oc_event;

typedef struct oc_ctx oc_ctx;

oc_ctx *oc_create(const oc_config *cfg);
void oc_destroy(oc_ctx *c);
/* one globaltime tick: mp1Run() then fail() (Application.cpp:99-104) */
int oc_tick(oc_ctx *c);
int oc_time(const oc_ctx *c);
/* FAITHFUL outputs */
const char *oc_dbg_log(oc_ctx *c, size_t *len);
const char *oc_stdout(oc_ctx *c, size_t *len);
/* renders msgcount.log (EmulNet.cpp:184-220) into an internal buffer */
const char *oc_msgcount(oc_ctx *c, size_t *len);
/* per-tick table dump in oracle/shim/dump_main.cpp's line format */
const char *oc_dump(oc_ctx *c, size_t *len);
/* SCALED outputs: events of the last tick, in the build's canonical order */
size_t oc_events(oc_ctx *c, const oc_event **ev);
/* dense readback: hb/ts of row r (absent -> -1), len n */
int oc_row(oc_ctx *c, int r, int32_t *hb, int32_t *ts);
/* SCALED: per-node gossip entries sent (before loss) / received (after loss) in the last tick */
int oc_last_msgcount(const oc_ctx *c, int32_t *sent, int32_t *recv);
/* node state: inited, inGroup, bFailed, heartbeat counter */
int oc_node(oc_ctx *c, int r, int32_t *state4);
/* SCALED: fail nodes idx[0..k) at the end of the tick just run (host fail() with caller-chosen victims) */
int oc_set_failed(oc_ctx *c, const int32_t *idx, int k);
/* SCALED: the last tick's gossip targets [n][5] (node indices) and their counts [n] */
int oc_targets(const oc_ctx *c, int32_t *tgt, int32_t *ntgt);
/* SCALED (not the join ramp): load the state between ticks -- hb / ts [n][n] (-1 absent), heartbeat
 * counters, crash flags, the last tick's targets -- then tick t runs next (ref_cpu.c) */
int oc_load_scaled(oc_ctx *c, int t, const int32_t *hb, const int32_t *ts, const int32_t *heartbeat,
                   const int32_t *failed, const int32_t *tgt, const int32_t *ntgt);
/* test telemetry: [0] = updateMyPos quirk firings, [1] = largest start-tick gap self -> target */
void oc_quirks(const oc_ctx *c, int64_t out[2]);
/* the crash set the SCALED driver uses (host fault injection) */
int oc_crash_set(int n, int count, uint64_t seed, int32_t *out);

/* PARTIAL mode (V-entry views, scenario S-C; semantics in ref_cpu.c): */
typedef struct op_config {
  int n, v;              /* nodes, view capacity V (2..64) */
  uint64_t rd_seed;      /* S2 seed contract */
  uint64_t view_seed;    /* initial views, eviction tie-break */
  int init_t0;           /* warm start tick (>= 5) */
  uint64_t init_seed;    /* initial heartbeat lags */
  int crash_tick, crash_count;
  uint64_t crash_seed;
  int drop_pct, drop_from, drop_to;
  uint64_t drop_seed;
} op_config;
typedef struct op_ctx op_ctx;
op_ctx *op_create(const op_config *cfg);
void op_destroy(op_ctx *c);
int op_tick(op_ctx *c);
int op_time(const op_ctx *c);
size_t op_events(op_ctx *c, const oc_event **ev);
/* "t i 1 1 failed hbctr cnt id:hb:ts ..." per node, ts = (hb+1)/2 */
const char *op_dump(op_ctx *c, size_t *len);
/* per-node entries sent (before loss) / received (after loss) in the last tick */
void op_last_msgcount(const op_ctx *c, int32_t *sent, int32_t *recv);
uint64_t op_evict_key(uint64_t view_seed, int32_t t, int32_t obs, int32_t id);

/* CPU-baseline sample: time node-ticks of the SCALED workload at size n (see ref_cpu.c) */
int oc_bench_sample(int n, int lists, int max_nodes, double min_seconds, int *out_nodes, double *out_seconds);

/* RNG restatements, exported for the known-answer tests */
typedef struct oc_rand { int32_t st[31]; int f, r; } oc_rand;
void oc_srand(oc_rand *g, uint32_t seed);
int32_t oc_rand_next(oc_rand *g);
uint32_t oc_rd_seed(uint64_t rd_seed, int32_t tick, int32_t id);
/* mt19937(seed) + uniform_int_distribution<int>(0, n-1): k draws */
void oc_mt_uniform(uint32_t seed, int n, int k, int32_t *out);

#ifdef __cplusplus
}
#endif
#endif
