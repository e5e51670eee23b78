/* gm_abi.h -- C ABI of the MI355X-native gossip-membership simulator (libgm.so).
 *
 * The drop-in boundary. The reference's own plugin seam is the
 * Application <-> MP1Node <-> EmulNet API: the driver calls, per node and per
 * globaltime tick, MP1Node::recvLoop (-> EmulNet::ENrecv) and MP1Node::nodeStart /
 * nodeLoop (-> checkMessages, nodeLoopOps, sendMemberList -> EmulNet::ENsend),
 * then Application::fail pokes Member::bFailed / Params::dropmsg and draws from
 * rand(). Here the whole per-tick body of Application::mp1Run for ALL nodes is
 * one call, gm_tick(); fault injection keeps its host-side driver (gm_rand,
 * gm_set_failed, gm_set_dropmsg); dbg.log / msgcount.log content comes back as
 * plain records. Plain C types only; no HIP or torch types cross the boundary.
 *
 * Reference interface each entry point replaces (file:line in the reference):
 *   gm_create       Application::Application + EmulNet::EmulNet + ENinit + new MP1Node
 *                   (Application.cpp:47-70, EmulNet.cpp:12-27,72-77, MP1Node.cpp:25-34),
 *                   Params::setparams values in gm_config (Params.cpp:19-40)
 *   gm_tick         Application::mp1Run (Application.cpp:121-164): recvLoop/ENrecv for
 *                   i ascending, then nodeStart/nodeLoop (checkMessages, updatelistCallBack,
 *                   joinreqCallBack, nodeLoopOps, sendMemberList, ENsend) for i descending
 *                   (MP1Node.cpp:47-54,73-163,182-495; EmulNet.cpp:87-177)
 *   gm_rand         rand() in Application::fail (Application.cpp:182,189) -- the SAME S1
 *                   stream ENsend draws from (EmulNet.cpp:90)
 *   gm_set_failed   mp1[i]->getMemberNode()->bFailed = true (Application.cpp:186,194)
 *   gm_set_dropmsg  par->dropmsg = 0/1 (Application.cpp:178,199)
 *   gm_drain_events Log::LOG / logNodeAdd / logNodeRemove call sites inside the tick
 *                   (Log.cpp:44-131; MP1Node.cpp:135,153,295,437; Application.cpp:158)
 *   gm_msgcount     EmulNet::sent_msgs / recv_msgs as dumped by ENcleanup (EmulNet.cpp:184-220)
 *   gm_dump_tables  Member::memberList of every node (Member.h:89-122), for parity tests
 *   gm_destroy      Application::~Application / ENcleanup storage release
 *
 * Conventions: every function returns GM_OK (0) or a negative GM_E* code and never
 * throws; the context owns all device memory; output buffers are caller-owned;
 * one host thread per context. gm_tick enqueues the tick on the context's HIP
 * stream and returns (a tick is a BSP round: sends of tick t are consumed in
 * tick t+1); every read-back function and gm_sync wait for enqueued ticks.
 */
#ifndef GM_ABI_H
#define GM_ABI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GM_ABI_VERSION 2

enum gm_status {
  GM_OK = 0,
  GM_EINVAL = -1,     /* bad argument / config */
  GM_ENOMEM = -2,     /* device or host allocation failed */
  GM_EDEVICE = -3,    /* HIP runtime error */
  GM_ERANGE = -4,     /* a bounded resource overflowed (inbox, event ring, draw table) */
  GM_ESTATE = -5,     /* protocol invariant the fast path relies on was violated */
  GM_EUNSUPPORTED = -6,
  GM_ECOMM = -7       /* collective (RCCL) failure */
};

enum gm_mode {
  GM_MODE_FAITHFUL = 0, /* the reference: EmulNet cap 30000, per-entry messages, S1 drops */
  GM_MODE_SCALED = 1,   /* build-defined large-N regime: converged start, keyed drops */
  GM_MODE_PARTIAL = 2   /* build-defined V-entry membership views (scenario S-C; oracle/ref_cpu.c PARTIAL) */
};

enum gm_event_kind {
  GM_EV_JOINED = 1,        /* "Node a.b.c.d:p joined at time t"   (Log.cpp:116-120) */
  GM_EV_REMOVED = 2,       /* "Node a.b.c.d:p removed at time t"  (Log.cpp:127-131) */
  GM_EV_START_GROUP = 3,   /* "Starting up group..."              (MP1Node.cpp:135) */
  GM_EV_TRY_JOIN = 4,      /* "Trying to join..."                 (MP1Node.cpp:152-153) */
  GM_EV_TIME_MARK = 5      /* "@@time=t"                          (Application.cpp:156-160) */
};

typedef struct gm_config {
  int32_t abi_version;     /* = GM_ABI_VERSION */
  int32_t mode;            /* enum gm_mode */
  int32_t n;               /* EN_GPSZ (= MAX_NNB) */
  int32_t single_failure;  /* SINGLE_FAILURE (host-side fail() uses it; kept for completeness) */
  int32_t drop_msg;        /* DROP_MSG */
  double drop_prob;        /* MSG_DROP_PROB (FAITHFUL: drop iff rand()%100 < (int)(p*100)) */
  uint32_t time_seed;      /* S1: srand(TIME_SEED) */
  uint64_t rd_seed;        /* S2: per-(tick, id) mt19937 seed contract */
  /* SCALED only */
  int32_t drop_pct;        /* per-entry drop percentage */
  int32_t drop_from;       /* drops apply to sends at ticks in [drop_from, drop_to) */
  int32_t drop_to;
  uint64_t drop_seed;
  /* placement */
  int32_t device;          /* HIP device ordinal */
  int32_t shard_rank;      /* shard of this context: SCALED column shard / PARTIAL row shard; 0 */
  int32_t shard_count;     /* number of shards (GPUs); 1 */
  /* SCALED initial state: 0 = cold converged start (every cell {hb 0, ts 0},
   * first tick 1); 1 = warm converged start at t0: own entry {2*t0-1, t0},
   * others {2*(t0-1-a)-1, t0-a} with a = splitmix64(init_seed, r, c) % 4,
   * heartbeat counters 2*t0, first tick t0+1 (no mass-staleness transient);
   * 2 = join ramp (one context, no drops): node i starts at tick (int)(0.25*i)
   * (Application.cpp:130), JOINREQ -> introducer -> JOINREP + newNodes-first gossip
   * (MP1Node.cpp:126-163,226-251) over the unbounded network; state as of tick 0
   * (the introducer's own entry), first tick 1 */
  int32_t init_mode;
  int32_t init_t0;
  uint64_t init_seed;
  int32_t band;            /* SCALED columns per band of the tick kernel (64/128/256/512/1024; 0 = auto:
                              1024, the band fast path, whenever the row width allows it) */
  int32_t view;            /* PARTIAL view capacity V (2..32; 0 = 32) */
  uint64_t view_seed;      /* PARTIAL initial views and eviction tie-break */
  int32_t device_share;    /* SCALED: contexts of this cluster that share this context's device and
                              split its free HBM for the escape pools / event ring (0 = shard_count:
                              every shard on one device, as the loopback tests run them; 1 = a device
                              of its own, one RCCL rank per GPU) */
  int32_t reserved;
} gm_config;

/* one log record; gm_drain_events returns them already in reference log order (Log.cpp lines of a
 * tick: loggers descending, joins in dequeue / ascending id order, removals descending id) */
typedef struct gm_event {
  int32_t t;
  int32_t logger;          /* node index (id = logger + 1) whose LOG call it is */
  int32_t kind;            /* enum gm_event_kind */
  int32_t subject;         /* node id joined/removed; 0 otherwise */
} gm_event;

typedef struct gm_ctx gm_ctx;

/* Params::setparams equivalent: parse a reference testcase .conf
 * ("MAX_NNB: %d\nSINGLE_FAILURE: %d\nDROP_MSG: %d\nMSG_DROP_PROB: %lf"). */
int gm_parse_conf(const char *path, gm_config *cfg);

int gm_create(const gm_config *cfg, gm_ctx **out);
int gm_destroy(gm_ctx *ctx);

/* Enqueue one Application::mp1Run tick at the context's current globaltime,
 * then advance globaltime. Returns a latched device error from an earlier tick.
 * FAITHFUL ticks do not wait on the host either: their records and error flags
 * are collected by the next call that reads state (gm_drain_events, gm_sync,
 * gm_rand, gm_set_failed, gm_msgcount, gm_read_*, gm_event_*), or by gm_tick
 * itself once the device record buffer could fill; an error raised by tick t is
 * reported by that call. */
int gm_tick(gm_ctx *ctx);
int gm_sync(gm_ctx *ctx);
int gm_time(gm_ctx *ctx, int32_t *t);

/* Application::fail hooks (called between ticks, host order preserved) */
int gm_rand(gm_ctx *ctx, int32_t *out);
/* gm_set_failed: sharded contexts (column or row shards of one cluster) must all be given the
 * SAME crash set, as every rank of the reference run sees one Application::fail. Row shards derive
 * their exchange block sizes from it; they all-reduce a hash of the set at the next tick and return
 * GM_ESTATE when a rank disagrees. */
int gm_set_failed(gm_ctx *ctx, const int32_t *idx, int32_t n);
int gm_set_dropmsg(gm_ctx *ctx, int32_t on);

/* Drain every event produced since the last drain, in reference log order
 * (ticks ascending; node phase i descending; per node: start line or joins in
 * dequeue order, then removals by descending id, then @@time). If cap is too
 * small, *n receives the number pending and GM_ERANGE is returned (nothing drained).
 * SCALED / PARTIAL keep one tick's records on the device; with event keeping on
 * (the default) gm_tick first stages the previous tick's undrained records to host
 * memory (a readback per tick), so nothing is lost between drains. */
int gm_drain_events(gm_ctx *ctx, gm_event *out, size_t cap, size_t *n);
/* on = 1 (default): keep every tick's records until drained. on = 0 (benchmarks):
 * a tick overwrites the previous tick's undrained records (no per-tick readback);
 * gm_drain_events then returns the last tick's records only.
 * Limits: with on = 1 the host stages at most 2^27 records between drains (GM_ERANGE
 * beyond: a TREMOVE tick of S-B's 1 % crash removes ~687 M entries, of S-A's ~22 M);
 * clusters that large run with on = 0 and read the device totals (gm_event_totals). The
 * device keeps E = band/32 records per (row, band) plus a spill ring sized from free HBM
 * (>= 2^24 records; GM_ERR_EVENTS -> GM_ERANGE past it). */
int gm_keep_events(gm_ctx *ctx, int32_t on);
/* counts[0] = records produced in the last tick (SCALED / PARTIAL telemetry; PARTIAL
 * also splits them per kind in counts[kind]; FAITHFUL: records pending per kind) */
int gm_event_counts(gm_ctx *ctx, uint64_t counts[6]);
/* totals[k] = records of kind k produced since gm_create, totals[0] = their sum,
 * independent of draining (FAITHFUL, SCALED; SCALED counts on the device, per (row,
 * band) cell). PARTIAL: GM_EUNSUPPORTED (views churn ~V joins per node and tick). */
int gm_event_totals(gm_ctx *ctx, uint64_t totals[6]);

/* sent/recv message counts per node id 1..n for ticks [0, t): out arrays [n][t].
 * FAITHFUL: EmulNet's sent_msgs / recv_msgs (EmulNet.cpp:111,172), always recorded.
 * SCALED / PARTIAL: the same per-entry-message counts in the list-gossip regime, recorded
 * once gm_msgcount_record was called (GM_ESTATE otherwise): sent = entries a node put on
 * the wire (its fresh entries x its targets, before loss: the loss is decided in flight),
 * recv = entries of the lists delivered to it that survived the loss (PARTIAL: of every
 * delivered list; all are merged). Gossip LIST entries only (the ramp's JOINREQ / JOINREP are not counted).
 * A PARTIAL row shard reports its own nodes ([nloc][t]). */
int gm_msgcount(gm_ctx *ctx, int32_t t, int32_t *sent, int32_t *recv);
/* SCALED / PARTIAL: start recording the per-node counts of gm_msgcount for ticks < tmax
 * (device history of 8 * tmax bytes per node). Only before the first tick (GM_ESTATE
 * after); FAITHFUL: no-op. SCALED column shards count their own columns' fresh entries and
 * SUM-allreduce them (N x 4 B per tick, only while recording), so every rank returns the
 * whole cluster's counts, equal to the single-context ones. */
int gm_msgcount_record(gm_ctx *ctx, int32_t tmax);

/* Dense readback of observer row r: hb/ts per subject column (absent -> -1),
 * columns [c0, c0+len) of this context's shard (c0 relative to the shard start). */
int gm_read_row(gm_ctx *ctx, int32_t r, int32_t c0, int32_t len, int32_t *hb, int32_t *ts);
/* Dense readback of observer rows [r0, r0+count): hb/ts [count][w] over this context's
 * w columns (absent -> -1); one bulk copy of the table, for parity tests at larger N. */
int gm_read_table(gm_ctx *ctx, int32_t r0, int32_t count, int32_t *hb, int32_t *ts);
/* PARTIAL: the raw V-entry views (id << 32 | hb, 0 = empty, ascending id) of nodes
 * [r0, r0 + count) as of the last tick, [count][V]; a row shard reads its own nodes. */
int gm_read_views(gm_ctx *ctx, int32_t r0, int32_t count, uint64_t *out);
/* node state: inited, inGroup, bFailed, heartbeat counter (4 int32 per node) */
int gm_read_nodes(gm_ctx *ctx, int32_t *state4);
/* SCALED: the gossip targets every node drew in the last tick (the gossipnodes of nodeLoopOps,
 * MP1Node.cpp:449-489, as node indices; [n][5], unused slots 0) and their counts [n] -- with the
 * tables and node state, the whole state between two ticks */
int gm_read_targets(gm_ctx *ctx, int32_t *targets, int32_t *counts);
/* Render the membership lists of every node in the parity dump format
 * ("t i inited inGroup bFailed heartbeat n id:hb:ts ...\n" per node). */
int gm_dump_tables(gm_ctx *ctx, char *buf, size_t cap, size_t *len);

/* SCALED telemetry of the last tick: [0]=delivered gossip lists M, [1]=live nodes,
 * [2]=max inbox depth, [3]=error flags */
int gm_tick_stats(gm_ctx *ctx, int64_t stats[4]);
/* SCALED escape storage as sized at create: info = {1 if the pools are dense-equivalent (no run can
 * overflow them) else 0, table escape-pool entries, payload escape-pool 16-byte slots, event spill
 * ring records}; GM_EUNSUPPORTED for the other modes */
int gm_pool_info(gm_ctx *ctx, int64_t info[4]);
/* Mean per-tick duration (ms) of the tick kernel over the timing window, measured
 * with HIP events recorded on the context stream before the window's first
 * kernel and after its last. gm_set_timing(ctx, 1) opens a new window at the
 * next tick; 0 when nothing was timed. */
int gm_set_timing(gm_ctx *ctx, int32_t on);
int gm_last_kernel_ms(gm_ctx *ctx, float *ms);

/* ---- SCALED column sharding (multi-GPU). A context with shard_count = G > 1
 * owns subject columns [c0, c0 + w) of every observer row (one context per GPU).
 * Once RCCL is attached (gm_comm_init, same unique id on every rank), gm_tick
 * runs the sharded tick: merge/sweep own columns -> ncclAllGather of per-row
 * (present, numfailed) -> rounds of {draw + resolve own-column draws ->
 * ncclAllReduce(MAX) of resolved draws -> acceptance} until every row has its
 * gossip targets (stream-ordered bounded rounds; rows they cannot take finish in host-driven
 * rounds before the tick is read or the next one starts). No gossip payload crosses GPUs. The phase functions expose
 * the same steps for G contexts on one device (gm_shard_loopback collectives). */
int gm_comm_unique_id(uint8_t *out128);   /* ncclGetUniqueId, on one rank */
/* ncclCommInitRank, then an all-gather of the config words every rank must share (mode, n,
 * band, view, GM_CHUNKS, seeds, drop schedule, init state): GM_EINVAL if any rank differs.
 * The seam it replaces: every MP1Node shares one Params / EmulNet (Application.cpp:47-66). */
int gm_comm_init(gm_ctx *ctx, const uint8_t *id128, int32_t nranks, int32_t rank);
/* info = {ranks in the RCCL communicator (0 before gm_comm_init), this rank in it (-1),
 * the device RCCL bound (-1), the context's HIP device} */
int gm_comm_info(gm_ctx *ctx, int32_t info[4]);
int gm_shard_layout(gm_ctx *ctx, int32_t *c0, int32_t *w);
int gm_shard_merge(gm_ctx *ctx);
int gm_shard_draw(gm_ctx *ctx, int32_t round, int32_t D);
int gm_shard_accept(gm_ctx *ctx, int32_t D, int32_t *npending);
int gm_shard_end_tick(gm_ctx *ctx);
/* what = 0: all-gather the per-row counts; what = 1: MAX-allreduce the first n*D draws;
 * what = 2 (msgcount recording, after what = 0): SUM-allreduce this tick's fresh counts */
int gm_shard_loopback(gm_ctx **ctxs, int32_t G, int32_t what, int32_t D);
/* One whole tick of G column-shard contexts on one device in the chunk order of the pipelined
 * RCCL tick (per exchange row chunk: all-gather of the counts, round-0 draws, MAX-reduce, acceptance;
 * then the bounded rounds 1, 2), the collectives by device copies. Not for the join ramp or msgcount
 * recording (GM_EINVAL); rows the bounded rounds cannot take return GM_ERANGE (use the phase API). */
int gm_shard_loopback_tick(gm_ctx **ctxs, int32_t G);
/* Host-collective hook: the exchange buffers of ONE column-shard context as host arrays, so a
 * host-side collective (e.g. gloo between processes) can stand in for RCCL or gm_shard_loopback
 * between the phase calls. what = 0: export this rank's per-row counts int32[n][2], import all
 * G slots int32[G][n][2]; what = 1: export / import the draws int32[n][D] (import their MAX over
 * the ranks); what = 2 (msgcount recording): uint32[n] fresh counts (+ uint32[n] kept entries on
 * keyed-loss ticks), import their SUM. gm_shard_export with out = NULL returns the size in *bytes;
 * gm_shard_import requires exactly that many bytes. (The seam they replace is EmulNet's shared
 * in-process buffer, EmulNet.cpp:87-177, which the reference's single process never had to cross.) */
int gm_shard_export(gm_ctx *ctx, int32_t what, int32_t D, void *out, size_t cap, size_t *bytes);
int gm_shard_import(gm_ctx *ctx, int32_t what, int32_t D, const void *in, size_t bytes);
/* Diagnostics: tick ONE column shard alone on a device (no RCCL): peers' per-row counts
 * mirror this shard's and draws landing in peer columns resolve to fresh column ix --
 * the real kernels at the true shard shape, for measurement only (not a simulation). */
int gm_shard_stub(gm_ctx *ctx, int32_t on);

/* ---- PARTIAL row sharding (scenario S-C multi-GPU). A PARTIAL context with
 * shard_count = G > 1 owns nodes [n*g/G, n*(g+1)/G) (gm_shard_layout returns the
 * range; gm_read_nodes / gm_dump_tables / gm_drain_events / gm_tick_stats report
 * its own nodes, with global indices). With RCCL attached (gm_comm_init) gm_tick
 * runs the local kernels in row chunks and, per chunk on a second stream, two
 * ncclAllToAllv of fixed-size blocks (record headers stamped with the tick; the lists'
 * fresh entries, 4 bytes each, read in place by the next tick) -- sizes come from the
 * shard layout, so no host round trip -- then appends the received records to their
 * targets' inboxes. gm_partial_loopback_tick does one such tick for G contexts on one device. */
int gm_partial_loopback_tick(gm_ctx **ctxs, int32_t G);
/* bytes this shard received from the other shards in the last tick's exchange (whole blocks) */
int gm_shard_exchange_bytes(gm_ctx *ctx, int64_t *bytes);

/* Crash set of the SCALED fault schedule: `count` node indices, ascending,
 * chosen by a splitmix64-keyed permutation of [0, n) (host fault injection). */
int gm_crash_set(int32_t n, int32_t count, uint64_t seed, int32_t *out);

const char *gm_strerror(int code);

#ifdef __cplusplus
}
#endif
#endif /* GM_ABI_H */
