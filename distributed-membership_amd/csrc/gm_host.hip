// gm_host.cpp -- libgm: the C ABI of include/gm_abi.h on top of the HIP kernels.
//
// Owns the per-context device state, launches one tick per gm_tick on the
// context stream, and turns device event records into reference log order.
// Compiled by hipcc for gfx950 together with gm_faithful.hip / gm_scaled.hip.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gm_abi.h"
#include "gm_device.h"
#include "gm_faithful.h"
#include "gm_partial.h"
#include "gm_scaled.h"

__global__ void gm_f_recv(FState s, int t);
__global__ void gm_f_recvout(FState s, int t);
__global__ void gm_f_node(FState s, int t);
__global__ void gm_f_sendscan(FState s, int t);
__global__ void gm_f_sendemit(FState s);
__global__ void gm_f_sendprep(FState s);
__global__ void gm_f_s1expand(FState s);
hipError_t gm_launch_tick(const SState &s, int t, int drop_pct, hipStream_t st, hipEvent_t k0, hipEvent_t k1,
                          bool pick);
hipError_t gm_launch_tick_prologue(const SState &s, int t, hipStream_t st, bool zero_draw = false);
hipError_t gm_launch_band_rows(const SState &s, int t, int drop_pct, int r0, int r1, hipStream_t st);
hipError_t gm_launch_xrows(const SState &s, int r0, int r1, hipStream_t st);
hipError_t gm_launch_draw(const SState &s, int t, int round, int D, int listed, hipStream_t st, int r0 = 0, int r1 = -1);
hipError_t gm_launch_accept(const SState &s, int t, int D, int in_list, int out, hipStream_t st, int r0 = 0,
                            int r1 = -1);
hipError_t gm_launch_plist_sort(const SState &s, int l, hipStream_t st);
hipError_t gm_launch_init(const SState &s, int warm, int t0, uint64_t seed, hipStream_t st);
hipError_t gm_launch_partial_tick(const PState &s, int t, uint32_t *mtraw, hipStream_t st, hipEvent_t k0,
                                  hipEvent_t k1);
hipError_t gm_launch_partial_init(const PState &s, int t0, uint64_t init_seed, hipStream_t st);
hipError_t gm_launch_partial_unpack(const PState &s, int t, int base, int nrecv, hipStream_t st);
hipError_t gm_launch_partial_pack(const PState &s, int t, int c, hipStream_t st);
hipError_t gm_launch_partial_mtgen(const PState &s, int t, uint32_t *mtraw, hipStream_t st, bool reset);
hipError_t gm_launch_partial_reset(const PState &s, hipStream_t st);
hipError_t gm_launch_partial_chunk(const PState &s, int t, const uint32_t *mtraw, int c, hipStream_t st);
hipError_t gm_launch_msgcount(const SState &s, int t, bool dropped, int phase, hipStream_t st);
size_t gm_partial_lds_bytes();

#define GM_T_LIMIT 32766  // packed 16-bit hb/ts stay exact: hb <= 2t+1 < 0xFFFF
#define GM_F_MAILBOX 4096  // FAITHFUL events copied back with the count and error flags
#define GM_D_FIRST S_MT_RAW  // S2 outputs per row in the first round (steady state needs ~5-6)
#define GM_D_MORE GM_D_MORE_ROUND  // S2 outputs per row in later rounds (transients with many stale entries)
#define GM_MAX_ROUNDS 4096    // draw rounds per sharded tick (16 + 64 * 4096 S2 outputs per row)
#define GM_D_LAST GM_D_LAST_ROUND  // bounded rounds: S2 outputs of round 2 (outputs [80, 336))
#define GM_SIG_WORDS 17      // gm_comm_init: config words every rank must agree on

struct gm_ctx {
  gm_config cfg;
  hipStream_t stream = nullptr;
  int dmax = 0;                      // status exchange depth (sharded)
  ncclComm_t comm = nullptr;         // RCCL communicator across column shards
  hipEvent_t k0 = nullptr, k1 = nullptr;  // per-tick band-kernel events (sharded)
  std::vector<hipEvent_t> tev;            // per-tick band-kernel event pairs (single context)
  double kernel_ms_sum = 0;
  int shard_sync = -1;               // sharded tick draw rounds: 1 host-driven unbounded loop, 0 bounded
  int diag_zero_row = -1;            // diagnostics (GM_DIAG_ZERO_ROW, tests): the pipelined column-shard tick
                                     //   clears this row's cells after its band kernels, so its records'
                                     //   counts disagree with the cells and a draw finds no holder
                                     // stream-ordered, -1 auto (env GM_SHARD_SYNC)
  int64_t nfailed = 0;               // nodes with failed_h set (gm_set_failed; nodeStart clears it)
  // sharded bounded draw rounds: rows they could not finish (npending) copied back without a
  // wait; the next call that needs the tick finishes them with host-driven rounds (draw_settle)
  int32_t *draw_left_h = nullptr;    // pinned [2]: rows left to the host-driven rounds, rows pending after round 0
  bool draw_rounds = false;          // the pipelined tick deferred bounded rounds 1, 2 to draw_settle
  hipEvent_t draw_ev = nullptr;
  bool draw_check = false;
  int t = 0;
  int n = 0;
  int dropmsg = 0;
  int latched = GM_OK;
  bool timing = false;
  int64_t ticks_done = 0;  // gm_tick calls that enqueued a tick
  int timed_ticks = 0;  // ticks in the current timing window
  int ktimed = 0;       // band-kernel event pairs recorded in the window (ring slots in use: min(ktimed, GM_TEV_RING))
  hipEvent_t e0 = nullptr, e1 = nullptr;
  // events: the device keeps one tick's records; with keep_events (default) a tick's records
  // are staged to `pending` before the next tick overwrites them (gm_keep_events)
  bool keep_events = true;
  bool undrained = false;      // the device holds the last tick's records, not yet staged
  uint64_t ev_tot[6] = {0, 0, 0, 0, 0, 0};  // FAITHFUL: cumulative records per kind
  std::vector<void *> allocs;
  std::vector<int32_t> failed_h;
  std::vector<int32_t> fail_t;  // last tick a failed node ran (join ramp: its inGroup is frozen there)
  // FAITHFUL
  FState f{};
  size_t f_smem = 0;
  void *f_mail = nullptr;            // pinned host copy of the FAITHFUL tick mailbox
  int f_inflight = 0;                // FAITHFUL ticks enqueued since the last mailbox collection
  std::vector<gm_event> pending;
  // SCALED
  SState s{};
  // PARTIAL
  PState p{};
  uint32_t *p_mtraw = nullptr;        // [2][nloc][16] S2 outputs by tick parity
  hipStream_t p_side = nullptr;        // S2 outputs of tick t+1, computed while tick t runs
  hipEvent_t p_tickev[2] = {nullptr, nullptr};  // by parity: the tick that read that S2 buffer is done
  hipEvent_t p_mtev[2] = {nullptr, nullptr};    // by parity: the prefetched S2 outputs are written
  int p_mt_next = -1;                  // the tick whose S2 outputs were prefetched
  int64_t p_recv_last = 0;  // lists received from other row shards in the last tick
  bool p_sharded = false;   // row-shard exchange each tick (G > 1, or one rank forced by GM_FORCE_SHARD=1)
  hipStream_t p_comm = nullptr;        // row shards: RCCL exchange stream (overlaps the next chunk's kernels)
  std::vector<hipEvent_t> p_chev;      // per chunk: its node ticks are done (compute stream)
  hipEvent_t p_done = nullptr;         // the tick's exchange + unpacks are done (comm stream)
  std::vector<double> p_xq;            // per row shard q: probability that a sender addresses q (xcap)
  uint64_t p_crash_hash = 0;           // hash of the whole crash set the block capacities were derived from
  bool p_crash_check = false;          // agree it across the ranks at the next RCCL tick
  uint64_t *p_crash_dev = nullptr;     // [2] device words of that check
};

// Every copy and fill of a context goes through its own stream. That stream is non-blocking, so the
// legacy null stream that hipMemcpy / hipMemset use neither waits for its kernels nor is waited for by
// them: a fill at creation could still be running when the init kernel writes (seen as an own entry
// missing from an S-C view after a 8.6 GB fill of the lists), and a host-to-device copy may return
// before its DMA lands. Fills are enqueued in order; copies wait for the stream (the host buffers are
// the caller's).
static inline hipError_t ctx_memset(gm_ctx *c, void *p, int v, size_t n) { return hipMemsetAsync(p, v, n, c->stream); }
static inline hipError_t ctx_memcpy(gm_ctx *c, void *d, const void *src, size_t n, hipMemcpyKind k) {
  const hipError_t e = hipMemcpyAsync(d, src, n, k, c->stream);
  return e == hipSuccess ? hipStreamSynchronize(c->stream) : e;
}
static inline hipError_t ctx_memcpy2d(gm_ctx *c, void *d, size_t dpitch, const void *src, size_t spitch, size_t width,
                                      size_t height, hipMemcpyKind k) {
  const hipError_t e = hipMemcpy2DAsync(d, dpitch, src, spitch, width, height, k, c->stream);
  return e == hipSuccess ? hipStreamSynchronize(c->stream) : e;
}

static thread_local char g_errbuf[256];

#define HIPCHECK(x)                                                                   \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      snprintf(g_errbuf, sizeof g_errbuf, "%s:%d %s", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return GM_EDEVICE;                                                              \
    }                                                                                 \
  } while (0)
#define NCCLCHECK(x)                                                                 \
  do {                                                                               \
    ncclResult_t r_ = (x);                                                           \
    if (r_ != ncclSuccess) {                                                         \
      snprintf(g_errbuf, sizeof g_errbuf, "%s:%d RCCL %s", __FILE__, __LINE__, ncclGetErrorString(r_)); \
      return GM_ECOMM;                                                               \
    }                                                                                \
  } while (0)

// inbox slots per receiver: the compiled capacity; GM_INBOX_CAP (diagnostics, tests) lowers it
// to show that an overflow fails loudly (GM_ERR_INBOX -> GM_ERANGE), never silently
static int inbox_cap(int cap) {
  const char *e = getenv("GM_INBOX_CAP");
  return e ? std::max(1, std::min(cap, atoi(e))) : cap;
}

template <class T>
static int dalloc(gm_ctx *c, T **p, size_t count) {
  void *q = nullptr;
  size_t bytes = sizeof(T) * (count ? count : 1);
  if (hipMalloc(&q, bytes) != hipSuccess) {
    snprintf(g_errbuf, sizeof g_errbuf, "hipMalloc(%zu) failed", bytes);
    return GM_ENOMEM;
  }
  c->allocs.push_back(q);
  *p = (T *)q;
  return GM_OK;
}

#define TRY(x)              \
  do {                      \
    int r_ = (x);           \
    if (r_ != GM_OK) return r_; \
  } while (0)

extern "C" const char *gm_strerror(int code) {
  switch (code) {
    case GM_OK: return "ok";
    case GM_EINVAL: return "invalid argument";
    case GM_ENOMEM: return g_errbuf[0] ? g_errbuf : "out of memory";
    case GM_EDEVICE: return g_errbuf[0] ? g_errbuf : "HIP runtime error";
    case GM_ERANGE: return "bounded resource overflowed";
    case GM_ESTATE: return "protocol invariant violated";
    case GM_EUNSUPPORTED: return "unsupported configuration";
    case GM_ECOMM: return g_errbuf[0] ? g_errbuf : "collective failure";
    default: return "unknown error";
  }
}

// Params::setparams (Params.cpp:19-40): same fscanf key sequence
extern "C" int gm_parse_conf(const char *path, gm_config *cfg) {
  if (!path || !cfg) return GM_EINVAL;
  FILE *fp = fopen(path, "r");
  if (!fp) return GM_EINVAL;
  int n = 0, single = 0, drop = 0;
  double prob = 0;
  if (fscanf(fp, "MAX_NNB: %d", &n) != 1) n = 0;
  if (fscanf(fp, "\nSINGLE_FAILURE: %d", &single) != 1) single = 0;
  if (fscanf(fp, "\nDROP_MSG: %d", &drop) != 1) drop = 0;
  if (fscanf(fp, "\nMSG_DROP_PROB: %lf", &prob) != 1) prob = 0;
  fclose(fp);
  cfg->n = n;
  cfg->single_failure = single;
  cfg->drop_msg = drop;
  cfg->drop_prob = prob;
  return n > 0 ? GM_OK : GM_EINVAL;
}

// glibc srandom_r (TYPE_3) seeding of the S1 stream; the draws themselves are
// stepped on the device (gm_f_send) and by gm_rand.
static void s1_seed(uint32_t seed, int32_t st[33]) {
  if (seed == 0) seed = 1;
  int32_t word = (int32_t)seed;
  st[0] = word;
  for (int i = 1; i < 31; i++) {
    long hi = word / 127773, lo = word % 127773;
    word = (int32_t)(16807 * lo - 2836 * hi);
    if (word < 0) word += 2147483647;
    st[i] = word;
  }
  int f = 3, r = 0;
  for (int k = 0; k < 310; k++) {
    st[f] = (int32_t)((uint32_t)st[f] + (uint32_t)st[r]);
    f = (f + 1) % 31;
    r = (r + 1) % 31;
  }
  st[31] = f;
  st[32] = r;
}

// P_q = R^(q+1), q = 0..63, rows padded to 32 words: R is one 31-draw round of the S1
// register in fptr-rotated order, x[j] += x[(j + 28) % 31] for j ascending (gm_f_s1expand)
static std::vector<uint32_t> s1_round_powers() {
  // column i of P_q = the round applied q+1 times to basis vector e_i (31 adds per round)
  std::vector<uint32_t> P((size_t)64 * 31 * 32, 0u);
  for (int i = 0; i < 31; i++) {
    uint32_t x[31] = {0};
    x[i] = 1;
    for (int q = 0; q < 64; q++) {
      for (int j = 0; j < 31; j++) x[j] += x[(j + 28) % 31];
      for (int k = 0; k < 31; k++) P[((size_t)q * 31 + k) * 32 + i] = x[k];
    }
  }
  return P;
}

static void lap(const char *what);

static int create_faithful(gm_ctx *c) {
  const int n = c->n;
  if (n > F_MAX_NODES) return GM_EUNSUPPORTED;  // EmulNet.cpp:108 assert(src <= MAX_NODES)
  FState &f = c->f;
  f.n = n;
  f.np = (n + 63) / 64 * 64;
  f.tmax = F_MAX_TIME;
  f.gstride = n + GM_FANOUT;
  f.draw_cap = 5 * n * n + 2 * n + 1024;
  f.rd_seed = c->cfg.rd_seed;
  f.ev_cap = std::max(1 << 18, 4 * n * n + 64 * n);
  TRY(dalloc(c, &f.table, (size_t)n * f.np));
  TRY(dalloc(c, &f.start, n));
  TRY(dalloc(c, &f.failed, n));
  TRY(dalloc(c, &f.inited, n));
  TRY(dalloc(c, &f.ingroup, n));
  TRY(dalloc(c, &f.hbctr, n));
  TRY(dalloc(c, &f.started_now, n));
  TRY(dalloc(c, &f.buf, F_ENBUFFSIZE));
  TRY(dalloc(c, &f.bufsize, 1));
  TRY(dalloc(c, &f.holepos, 2 * F_ENBUFFSIZE));
  TRY(dalloc(c, &f.buf2, F_ENBUFFSIZE));
  TRY(dalloc(c, &f.bkey, F_ENBUFFSIZE));
  TRY(dalloc(c, &f.bkey2, F_ENBUFFSIZE));
  TRY(dalloc(c, &f.sidx, F_ENBUFFSIZE));
  TRY(dalloc(c, &f.rmeta, 2));
  TRY(dalloc(c, &f.q, F_ENBUFFSIZE));
  TRY(dalloc(c, &f.q_off, n));
  TRY(dalloc(c, &f.q_cnt, n));
  TRY(dalloc(c, &f.scount, n));
  TRY(dalloc(c, &f.jcnt, n));
  TRY(dalloc(c, &f.gcnt, n));
  TRY(dalloc(c, &f.fcnt, n));
  TRY(dalloc(c, &f.jrq, (size_t)n * n));
  TRY(dalloc(c, &f.gossip, (size_t)n * f.gstride));
  TRY(dalloc(c, &f.fcols, (size_t)n * n));
  TRY(dalloc(c, &f.s1, 33));
  TRY(dalloc(c, &f.draws, f.draw_cap));
  TRY(dalloc(c, &f.sbase, n));
  TRY(dalloc(c, &f.smeta, 3));
  TRY(dalloc(c, &f.spre, (size_t)f.draw_cap + 1));
  TRY(dalloc(c, &f.qidx, F_ENBUFFSIZE));
  TRY(dalloc(c, &f.s1mat, (size_t)64 * 31 * 32));
  TRY(dalloc(c, &f.s1vb, (size_t)(f.draw_cap / 1984 + 2) * 32));
  TRY(dalloc(c, &f.sent, (size_t)(n + 1) * f.tmax));  // rows 1..n: sent_msgs[id][time]
  TRY(dalloc(c, &f.recv, (size_t)(n + 1) * f.tmax));
  // one block = the tick's mailbox: event count, error flags, then the events, so that one
  // small copy per tick brings back all three (GM_F_MAILBOX events; more: a second copy)
  uint8_t *mb = nullptr;
  TRY(dalloc(c, &mb, 16 + sizeof(FEvent) * (size_t)f.ev_cap));
  f.ev_count = (unsigned long long *)mb;
  f.err = (uint32_t *)(mb + 8);
  f.ev = (FEvent *)(mb + 16);
  lap("faithful allocations");
  if (hipHostMalloc(&c->f_mail, 16 + sizeof(FEvent) * GM_F_MAILBOX, hipHostMallocDefault) != hipSuccess) return GM_ENOMEM;
  lap("pinned mailbox");
  HIPCHECK(ctx_memset(c, f.table, 0xFF, sizeof(uint32_t) * (size_t)n * f.np));
  std::vector<int32_t> start(n);
  for (int i = 0; i < n; i++) start[i] = (int)(0.25 * i);  // (int)(STEP_RATE*i), Application.cpp:143
  HIPCHECK(ctx_memcpy(c, f.start, start.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice));
  for (int32_t *p : {f.failed, f.inited, f.ingroup, f.hbctr, f.started_now, f.q_off, f.q_cnt,
                     f.scount, f.jcnt, f.gcnt, f.fcnt})
    HIPCHECK(ctx_memset(c, p, 0, sizeof(int32_t) * (size_t)n));
  HIPCHECK(ctx_memset(c, f.sent, 0, sizeof(int32_t) * (size_t)(n + 1) * f.tmax));
  HIPCHECK(ctx_memset(c, f.recv, 0, sizeof(int32_t) * (size_t)(n + 1) * f.tmax));
  HIPCHECK(ctx_memset(c, f.bufsize, 0, sizeof(int32_t)));
  HIPCHECK(ctx_memset(c, f.ev_count, 0, sizeof(unsigned long long)));
  HIPCHECK(ctx_memset(c, f.err, 0, sizeof(uint32_t)));
  int32_t st[33];
  s1_seed(c->cfg.time_seed, st);  // srand(time(NULL)) at Application.cpp:50 and :96
  HIPCHECK(ctx_memcpy(c, f.s1, st, sizeof st, hipMemcpyHostToDevice));
  lap("faithful memsets");
  const std::vector<uint32_t> pm = s1_round_powers();
  HIPCHECK(ctx_memcpy(c, f.s1mat, pm.data(), sizeof(uint32_t) * pm.size(), hipMemcpyHostToDevice));
  lap("S1 powers");
  HIPCHECK(hipFuncSetAttribute((const void *)gm_f_recv, hipFuncAttributeMaxDynamicSharedMemorySize, F_RECV_LDS));
  lap("kernel attributes");
  const int nw = f.np / 64;
  c->f_smem = (size_t)f.np * 8 + (size_t)nw * 8 * 3 + (size_t)nw * 4 + 624 * 4 + 48 * 4;
  return GM_OK;
}

// Band width of the SCALED tick: the largest of 512/256/128/64 columns (dividing
// the padded row) whose per-band traffic -- N rows x band x (2 B cell read + 2 B
// write + 1 B payload write + 1 B payload read) -- stays within ~210 MB, so a band's
// payload slab stays resident in the 256 MiB Infinity Cache across its ~5 readers
// per sender slice (gm_scaled.hip). gm_config.band / env GM_BAND override.
static int pick_band(const gm_ctx *c, int n, int wp) {
  int b = c->cfg.band;
  if (!b && getenv("GM_BAND")) b = atoi(getenv("GM_BAND"));
  if (b) return (b == 64 || b == 128 || b == 256 || b == 512 || b == 1024) && wp % b == 0 ? b : -1;
  // Measured (profiles/r02/): the widest band wins -- one row per wave at B = 1024 (no
  // max over two rows' list counts, half the per-(row, band) bookkeeping per cell), and a
  // payload gather stays whole lines; B = 128 gathers half a line per row. gm_s_band at
  // N = 65,536: 4.98 ms (B = 1024), 5.43 (512), 7.42 (128); the S-B shard (N = 262,144,
  // G = 8): 11.0 / 12.0 / 15.0 ms. Per-band traffic up to ~1.4 GB still keeps the gathered
  // payload slab (n x B/2 bytes) on-die.
  const double budget = 1.4e9;
  for (int cand : {1024, 512, 256, 128})
    if (wp % cand == 0 && 5.0 * n * cand <= budget) return cand;
  return 64;
}

// the chunk-major exchange buffer of a column shard (SState.xcnt, S_XC)
static size_t xcnt_bytes(const SState &s) {
  return sizeof(int32_t) * 2 * (size_t)s.xk * s.shard_count * ((size_t)1 << s.xlog);
}
static int xchunk_rows(const SState &s, int ch) {  // real rows of exchange chunk ch
  return (int)std::min<int64_t>((int64_t)1 << s.xlog, (int64_t)s.n - ((int64_t)ch << s.xlog));
}

static int create_scaled(gm_ctx *c) {
  const int n = c->n;
  const int G = c->cfg.shard_count > 0 ? c->cfg.shard_count : 1;
  const int rank = c->cfg.shard_rank;
  if (rank < 0 || rank >= G || G > n) return GM_EINVAL;
  SState &s = c->s;
  s.n = n;
  s.shard_rank = rank;
  s.shard_count = G;
  // one forced shard (diagnostics/tests): the sharded tick + RCCL with a single rank
  s.sharded = G > 1 || (getenv("GM_FORCE_SHARD") && atoi(getenv("GM_FORCE_SHARD")) == 1);
  // contiguous, balanced subject-column ranges whose boundaries are multiples of 4 (when n >= 8G):
  // a start group of the join ramp (ids 4g..4g+3, gm_s_band's updateMyPos quirk) never straddles two
  // shards, and the keyed loss's 4-column hash groups are whole on every shard
  auto col0 = [n, G](int g) {
    if (g >= G) return n;
    return n >= 8 * G ? 4 * (int)((int64_t)n * g / (4 * G)) : (int)((int64_t)n * g / G);
  };
  s.c0 = col0(rank);
  s.w = col0(rank + 1) - s.c0;
  s.wp = (s.w + S_ROW_ALIGN - 1) / S_ROW_ALIGN * S_ROW_ALIGN;
  s.band = pick_band(c, n, s.wp);
  if (s.band < 0) return GM_EINVAL;
  s.nb = s.wp / s.band;
  if ((size_t)n * s.band * 2 >= (1ull << 31)) return GM_EUNSUPPORTED;  // 32-bit buffer offsets per band slab
  s.evs = s.band / 32;
  // draw kernels' LDS: 4 waves x (chunk prefix + lazy MT state); N = 262,144 on one GPU: 42 KB
  if (sizeof(uint32_t) * 4 * ((size_t)(s.wp / S_CHUNK(s.band)) + 1 + 624) > 65536) return GM_EUNSUPPORTED;
  s.rd_seed = c->cfg.rd_seed;
  s.drop_seed = c->cfg.drop_seed;
  const size_t cells = (size_t)n * s.wp;
  TRY(dalloc(c, &s.table, cells));   // stored cell bytes
  s.kcap = inbox_cap(S_KMAX);
  s.lag_hmin = 3;  // h <= 2: the next re-base would wrap (lag > 125 ticks)
  if (getenv("GM_LAG_CAP")) {  // diagnostics (tests): fail at a lag > L ticks (h = 254 - 2 lag), L >= 15
    const int L = atoi(getenv("GM_LAG_CAP"));
    if (L < 15 || L > 125) return GM_EINVAL;
    s.lag_hmin = 254 - 2 * L;
  }
  c->shard_sync = getenv("GM_SHARD_SYNC") ? (atoi(getenv("GM_SHARD_SYNC")) ? 1 : 0) : -1;
  if (getenv("GM_DIAG_ZERO_ROW")) c->diag_zero_row = atoi(getenv("GM_DIAG_ZERO_ROW"));
  TRY(dalloc(c, &s.msg, cells));        // nibbles: 2 parities x band/2 bytes per (band, row)
  // Escape storage (gm_scaled.h), one set per tick parity: a 16-cell inline slot per (band, row)
  // list (1/32 B per cell at B = 1024) and the pools. The pools are DENSE-equivalent (every
  // list's whole slice fits its stripe's region: no run can overflow them) when that fits the
  // memory budget -- a quarter of the device's free HBM at create, split over the shard count
  // (G column shards of one cluster may share a device: the loopback tests) -- or always up
  // to 2^31 cells. S-A (N = 65,536): 43 GB of dense pools, so a crash of half the cluster (the
  // reference's multifailure schedule, Application.cpp:188-195) escapes every cell it needs.
  // Beyond the budget the pools take what it holds, at least 1/64 of the cells and 1/16 of the
  // payload lanes -- a warm cluster escapes only a crashed node's entries in the ticks before
  // their removal (~10 per list at a 1 % crash: inline) -- and an overflow fails loudly
  // (GM_ERR_ESC -> GM_ERANGE). GM_ESC_CAP (cells; diagnostics, tests) lowers the table pool.
  // Striped: >= 64 (band, row) lists per stripe (up to 1024 stripes), more stripes while a
  // stripe's region exceeds what the list word's offset field addresses (S_EW_REGION_MAX).
  const size_t lists = (size_t)n * s.nb;
  int S = 1024;
  while (S > 1 && lists / S < 64) S >>= 1;
  auto grow = [&](size_t per_stripe_cells_total) {  // stripes so that one region fits the offset field
    while ((per_stripe_cells_total + S - 1) / S > S_EW_REGION_MAX) S <<= 1;
  };
  const size_t dense_t = ((lists + 1023) / 1024) * 1024 * s.band;  // table-pool entries, dense (rounded per stripe)
  const size_t dense_p = dense_t / 16;                              // payload-pool 16-byte slots, dense
  const double dense_bytes = 2.0 * ((double)dense_t * 4 + (double)dense_p * 16);
  size_t free_b = 0, total_b = 0;
  HIPCHECK(hipMemGetInfo(&free_b, &total_b));
  // the free HBM is split over the contexts of this cluster on this device: every shard on one
  // device (loopback) unless the caller says each has its own GPU (device_share = 1, RCCL ranks)
  const int gdev = c->cfg.device_share > 0 ? std::min(c->cfg.device_share, G) : G;
  double budget = (double)free_b / 4 / gdev;
  if (getenv("GM_ESC_BUDGET_GB")) budget = atof(getenv("GM_ESC_BUDGET_GB")) * 1e9;  // diagnostics (tests)
  const bool dense = cells <= (1ull << 31) || dense_bytes <= budget;
  size_t tcells, pslots;
  if (dense) {
    while (((lists + S - 1) / S) * s.band > S_EW_REGION_MAX) S <<= 1;  // the list word's offset field
    const size_t per = (lists + S - 1) / S;  // lists per stripe (at most)
    tcells = per * s.band * S;
    pslots = per * (s.band / 16) * S;
  } else {
    // the table pool takes the fraction f of its dense size and the payload pool min(1, 4f) of its
    // dense count (cells / 16 slots), so at least 1/16 of the payload lanes at the floor f = 1/64
    // (a / 256 here gave 1/256); both parities together fit the budget:
    // 8 f cells + 2 min(1, 4f) cells bytes
    const double cb = (double)cells;
    double f = budget / (16.0 * cb);
    if (f > 0.25) f = (budget - 2.0 * cb) / (8.0 * cb);
    f = std::min(1.0, std::max(1.0 / 64, f));
    tcells = std::max<size_t>((size_t)(cb * f), 4 * (size_t)s.band * S);
    pslots = std::max<size_t>((size_t)(cb * std::min(1.0, 4 * f) / 16), 4 * (size_t)(s.band / 16) * S);
    grow(tcells);
  }
  s.esc_dense = dense ? 1 : 0;
  s.esc_stripes = S;
  size_t treg = std::min<size_t>((tcells + S - 1) / S, S_EW_REGION_MAX);
  size_t preg = std::min<size_t>((pslots + S - 1) / S, 0xFFFFFFF0ull / S);
  if (getenv("GM_ESC_CAP")) treg = std::max<size_t>(1, std::min<size_t>(atol(getenv("GM_ESC_CAP")) / S, treg));
  s.tesc_region = (uint32_t)treg;
  s.pesc_region = (uint32_t)preg;
  s.tesc_cap = treg * S;
  s.pesc_cap = (uint32_t)(preg * S);
  for (int p = 0; p < 2; p++) {
    TRY(dalloc(c, &s.tesc_in[p], lists * S_ESC_IN));
    TRY(dalloc(c, &s.tesc[p], s.tesc_cap));
    TRY(dalloc(c, &s.pesc[p], (size_t)s.pesc_cap * 16));
    TRY(dalloc(c, &s.pesc_rec[p], (size_t)n * s.nb));
  }
  TRY(dalloc(c, &s.tesc_cnt, 2 * (size_t)S));
  TRY(dalloc(c, &s.pesc_cnt, 2 * (size_t)S));
  HIPCHECK(ctx_memset(c, s.tesc_cnt, 0, 2 * S * sizeof(unsigned long long)));
  HIPCHECK(ctx_memset(c, s.pesc_cnt, 0, 2 * S * sizeof(unsigned long long)));
  for (int p = 0; p < 2; p++) {
    TRY(dalloc(c, &s.inbox_cnt[p], n));
    TRY(dalloc(c, &s.inbox[p], (size_t)n * S_KMAX));
  }
  TRY(dalloc(c, &s.hbctr, n));
  TRY(dalloc(c, &s.wtick, n));
  TRY(dalloc(c, &s.failed, n));
  TRY(dalloc(c, &s.brec, (size_t)n * s.nb));
  // the band kernel's fast path (B = 1024; gm_s_band_fast) and the list of units it hands back
  // (at most every unit of a tick). GM_BAND_FAST=0 (diagnostics, A/B against the general path:
  // tests/test_gpu_band_fast.py) leaves it off.
  s.fb_cnt = nullptr;
  s.fb_list = nullptr;
  if (s.band == 1024 && !(getenv("GM_BAND_FAST") && atoi(getenv("GM_BAND_FAST")) == 0)) {
    TRY(dalloc(c, &s.fb_cnt, 2));
    HIPCHECK(ctx_memset(c, s.fb_cnt, 0, 2 * sizeof(uint32_t)));
    TRY(dalloc(c, &s.fb_list, (size_t)n * s.nb));
  }
  // gm_s_pick0 (single context, B = 1024) and the list of rows it leaves to gm_s_pick
  s.pk_list = nullptr;
  s.pk_cnt = nullptr;
  // gm_s_pick0's LDS: per row of the workgroup's 16, the band prefix (nb + 1 words) and the bands'
  // chunk counts (nb x 8 bytes)
  if (s.band == 1024 && !s.sharded && 16 * (sizeof(uint32_t) * (size_t)(s.nb + 1) + sizeof(uint2) * (size_t)s.nb) <= 65536 &&
      !(getenv("GM_PICK0") && atoi(getenv("GM_PICK0")) == 0)) {
    TRY(dalloc(c, &s.pk_list, n));
    TRY(dalloc(c, &s.pk_cnt, 1));
  }
  TRY(dalloc(c, &s.ev_band, (size_t)n * s.nb * s.evs));
  {  // event spill ring (records past a (row, band)'s E slots): up to every cell of the shard, within a
     // 1/32 share of the free HBM (the loopback shards of one device split it); at least 2^24 records.
     // A half-cluster crash at S-A removes ~550 M entries in its peak tick (~420 M past the slots).
    HIPCHECK(hipMemGetInfo(&free_b, &total_b));
    const size_t want = std::min<size_t>((size_t)n * s.wp, free_b / 32 / gdev / sizeof(uint64_t));
    s.ev_spill_cap = (uint32_t)std::min<size_t>(std::max<size_t>(want, 1u << 24), 1ull << 31);
  }
  TRY(dalloc(c, &s.ev_spill, s.ev_spill_cap));
  TRY(dalloc(c, &s.ev_spill_cnt, 1 + S_EV_STRIPES));
  TRY(dalloc(c, &s.evcum, (size_t)n * s.nb));
  TRY(dalloc(c, &s.mtraw, (size_t)n * S_MT_RAW));
  TRY(dalloc(c, &s.rowstat, (size_t)n * 4));
  TRY(dalloc(c, &s.targets, (size_t)n * GM_FANOUT));
  TRY(dalloc(c, &s.err, 1));
  // converged start (cold or warm, gm_config.init_mode); padding columns absent
  const bool warm = c->cfg.init_mode == 1;
  const int t0 = warm ? c->cfg.init_t0 : 0;
  // join ramp (init_mode 2); with keyed drops a joiner can miss its own entry and take
  // updateMyPos's quirk path (MP1Node.cpp:316), handled in gm_s_band within the row's start
  // group (ids 4g..4g+3): column shards never split a group (col0 above)
  const bool ramp = c->cfg.init_mode == 2;
  if (c->cfg.init_mode < 0 || c->cfg.init_mode > 2 || (warm && (t0 < 5 || t0 > GM_T_LIMIT / 2))) return GM_EINVAL;
  if (ramp)
    for (int g = 1; g < G; g++)
      if (col0(g) % 4 != 0) return GM_EUNSUPPORTED;  // n < 8G only
  s.ramp = ramp ? 1 : 0;
  s.intro_until = 0x7FFFFFFF;
  if (ramp) {
    TRY(dalloc(c, &s.mecol, n));
    HIPCHECK(ctx_memset(c, s.mecol, 0xFF, sizeof(int32_t) * n));  // -1: written by the rank owning the row's column
    TRY(dalloc(c, &s.selfadd, S_SELFADD_CAP));
    TRY(dalloc(c, &s.selfadd_cnt, 1));
    HIPCHECK(ctx_memset(c, s.selfadd_cnt, 0, sizeof(uint32_t)));
  }
  HIPCHECK(ctx_memset(c, s.msg, 0, sizeof(uint8_t) * cells));
  for (int p = 0; p < 2; p++) HIPCHECK(ctx_memset(c, s.inbox_cnt[p], 0, sizeof(int32_t) * n));
  HIPCHECK(ctx_memset(c, s.failed, 0, sizeof(int32_t) * n));
  HIPCHECK(ctx_memset(c, s.err, 0, sizeof(uint32_t)));
  HIPCHECK(gm_launch_init(s, ramp ? 2 : warm ? 1 : 0, t0, c->cfg.init_seed, c->stream));  // table, records, pool
  HIPCHECK(hipStreamSynchronize(c->stream));
  uint32_t ierr = 0;
  HIPCHECK(ctx_memcpy(c, &ierr, s.err, sizeof ierr, hipMemcpyDeviceToHost));
  if (ierr) {  // a cold start escapes every cell: beyond the dense-pool size it does not fit
    snprintf(g_errbuf, sizeof g_errbuf, "initial state overflows the escape pool (%zu cells)", s.tesc_cap);
    return GM_ERANGE;
  }
  HIPCHECK(ctx_memset(c, s.ev_spill_cnt, 0, (1 + S_EV_STRIPES) * sizeof(uint32_t)));
  HIPCHECK(ctx_memset(c, s.evcum, 0, sizeof(uint64_t) * (size_t)n * s.nb));
  HIPCHECK(ctx_memset(c, s.rowstat, 0, sizeof(int32_t) * n * 4));
  if (s.sharded) {
    TRY(dalloc(c, &s.acc, (size_t)n * 8));
    TRY(dalloc(c, &s.pending, n));
    // npending, then the pending lists' append counts (plist_cnt[1], [2]): one word block, so the tick's
    // end reads the first two back in one copy
    TRY(dalloc(c, &s.npending, 4));
    s.plist_cnt[1] = (uint32_t *)(s.npending + 1);
    s.plist_cnt[2] = (uint32_t *)(s.npending + 2);
    c->dmax = 64;
    // the exchange's row chunks (tick_sharded pipelines band -> all-gather -> draw -> MAX-allreduce ->
    // acceptance chunk by chunk): 2^xlog rows each (>= 64: a multiple of every band width's rows per
    // unit), K = GM_SCHUNKS chunks, by default 2 (one-box A/B, profiles/r05/ab5: stub shard 7.64 vs 7.76 ms
    // at 4, G = 8 loopback 7.58 vs 7.79 ms per shard-tick)
    {
      int K = getenv("GM_SCHUNKS") ? atoi(getenv("GM_SCHUNKS")) : 2;
      if (K < 1 || K > 64) return GM_EINVAL;
      s.xlog = 6;
      while (((int64_t)1 << s.xlog) * K < n) s.xlog++;
      s.xk = (int)((n + (1 << s.xlog) - 1) >> s.xlog);
    }
    TRY(dalloc(c, &s.xcnt, (size_t)s.xk * G * ((size_t)1 << s.xlog) * 2));
    TRY(dalloc(c, &s.status, (size_t)n * c->dmax));
    // bounded rounds (tick_sharded): round 0 takes every row's first 16 S2 outputs, round 1
    // the next 64 for up to plist_cap rows left pending -- no host round trip per tick
    s.plist_cap[1] = std::min(S_PLIST_CAP, std::max(std::min(n, 1024), n / 16));  // round 1: 64 more outputs
    s.plist_cap[2] = 256;                                             // round 2: 256 more outputs
    if (getenv("GM_PLIST_CAP"))  // diagnostics (tests): smaller lists, so rows overflow to the host-driven rounds
      for (int l = 1; l <= 2; l++) s.plist_cap[l] = std::max(1, std::min(s.plist_cap[l], atoi(getenv("GM_PLIST_CAP"))));
    if (hipHostMalloc(&c->draw_left_h, 2 * sizeof(int32_t), hipHostMallocDefault) != hipSuccess) return GM_ENOMEM;
    c->draw_left_h[0] = c->draw_left_h[1] = 0;
    HIPCHECK(hipEventCreateWithFlags(&c->draw_ev, hipEventDisableTiming));
    for (int l = 1; l <= 2; l++) {
      TRY(dalloc(c, &s.plist[l], s.plist_cap[l]));
      TRY(dalloc(c, &s.statusl[l], (size_t)s.plist_cap[l] * (l == 1 ? GM_D_MORE : GM_D_LAST)));
    }
    HIPCHECK(ctx_memset(c, s.pending, 0, sizeof(int32_t) * n));
    HIPCHECK(ctx_memset(c, s.xcnt, 0, xcnt_bytes(s)));
    HIPCHECK(hipStreamCreateWithFlags(&c->p_comm, hipStreamNonBlocking));  // the pipelined exchange
    c->p_chev.assign(s.xk, nullptr);
    for (hipEvent_t &e : c->p_chev) HIPCHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIPCHECK(hipEventCreateWithFlags(&c->p_done, hipEventDisableTiming));
  }
  c->t = t0 + 1;  // the converged table is the state "as of tick t0"
  return GM_OK;
}

// PARTIAL: V-entry views (scenario S-C), warm start at init_t0 (oracle op_create).
// shard_count = G > 1: row shard `shard_rank` owns nodes [n*g/G, n*(g+1)/G) and
// exchanges the lists its nodes send to other shards every tick (gm_tick with RCCL
// attached: all-to-all of record counts + two all-to-allv; gm_partial_loopback for
// G contexts on one device).
static int partial_caps(gm_ctx *c);

static int create_partial(gm_ctx *c) {
  const int n = c->n;
  PState &p = c->p;
  p.n = n;
  p.V = c->cfg.view ? c->cfg.view : 32;
  // the per-wave LDS table holds the own list + P_KP delivered lists at <= 0.55 load
  if (p.V < 2 || p.V > 32 || p.V > n) return GM_EUNSUPPORTED;
  const int t0 = c->cfg.init_t0;
  if (c->cfg.init_mode != 1 || t0 < 5 || t0 > GM_T_LIMIT / 2) return GM_EINVAL;
  if (n > (1 << 25) - 1) return GM_EUNSUPPORTED;  // ids live in 25 bits of the LDS table words and wire entries
  const int G = c->cfg.shard_count > 0 ? c->cfg.shard_count : 1;
  const int rank = c->cfg.shard_rank;
  if (rank < 0 || rank >= G || G > n || G > 256) return GM_EINVAL;
  p.G = G;
  p.rank = rank;
  p.n0 = (int)((int64_t)n * rank / G);
  p.nloc = (int)((int64_t)n * (rank + 1) / G) - p.n0;
  p.rows = G > 1 ? p.nloc : n;  // own rows; received lists stay in recv_list (wire format)
  const int nl = p.nloc, R = n - nl;
  p.rd_seed = c->cfg.rd_seed;
  p.view_seed = c->cfg.view_seed;
  p.drop_seed = c->cfg.drop_seed;
  p.drop_pct = -1;
  TRY(dalloc(c, &p.lists, (size_t)2 * p.rows * p.V));
  for (int q = 0; q < 2; q++) {
    TRY(dalloc(c, &p.inbox[q], (size_t)nl * P_KMAX));
    HIPCHECK(ctx_memset(c, p.inbox[q], 0, sizeof(int32_t) * nl * P_KMAX));  // the counts (slot 0) start at 0
    if (G > 1) TRY(dalloc(c, &p.rsrc[q], R));
    if (G == 1) p.rsrc[q] = nullptr;
  }
  TRY(dalloc(c, &p.hbctr, nl));
  TRY(dalloc(c, &p.failed, nl));
  TRY(dalloc(c, &p.ev, (size_t)nl * 2 * p.V));
  TRY(dalloc(c, &p.ev_cnt, nl));
  TRY(dalloc(c, &p.ev_jm, nl));
  TRY(dalloc(c, &p.rowstat, (size_t)nl * 4));
  TRY(dalloc(c, &p.targets, (size_t)nl * GM_FANOUT));
  TRY(dalloc(c, &p.big, nl));
  TRY(dalloc(c, &p.huge, nl));
  TRY(dalloc(c, &p.err, 1));
  TRY(dalloc(c, &c->p_mtraw, (size_t)nl * 16 * 2));
  {  // the S2 prefetch for tick t+1 runs beside tick t's kernels: at the lowest stream priority it
     // takes the CUs the tick leaves idle instead of competing for them (GM_SIDE_PRIO=0: default)
    int lo = 0, hi = 0;
    HIPCHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    const bool low = !(getenv("GM_SIDE_PRIO") && !atoi(getenv("GM_SIDE_PRIO")));
    HIPCHECK(hipStreamCreateWithPriority(&c->p_side, hipStreamNonBlocking, low ? lo : 0));
  }
  for (int q = 0; q < 2; q++) {
    HIPCHECK(hipEventCreateWithFlags(&c->p_tickev[q], hipEventDisableTiming));
    HIPCHECK(hipEventCreateWithFlags(&c->p_mtev[q], hipEventDisableTiming));
  }
  c->p_sharded = G > 1 || (getenv("GM_FORCE_SHARD") && atoi(getenv("GM_FORCE_SHARD")) == 1);
  // row shards pipeline their exchange over K chunks of their nodes (GM_CHUNKS, default 4)
  p.nchunk = c->p_sharded ? (getenv("GM_CHUNKS") ? atoi(getenv("GM_CHUNKS")) : 4) : 1;
  p.kcap = inbox_cap(P_KMAX - 1);
  if (p.nchunk < 1 || p.nchunk > 64) return GM_EINVAL;
  TRY(dalloc(c, &p.big_cnt, p.nchunk));
  TRY(dalloc(c, &p.huge_cnt, p.nchunk));
  if (c->p_sharded) {
    HIPCHECK(hipStreamCreateWithFlags(&c->p_comm, hipStreamNonBlocking));
    c->p_chev.assign(p.nchunk, nullptr);
    for (hipEvent_t &e : c->p_chev) HIPCHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIPCHECK(hipEventCreateWithFlags(&c->p_done, hipEventDisableTiming));
    TRY(dalloc(c, &p.pk_hdr, (size_t)G * nl * 8));
    TRY(dalloc(c, &p.pk_list, (size_t)G * nl * p.V));
    HIPCHECK(ctx_memset(c, p.pk_hdr, 0xFF, sizeof(int32_t) * G * nl * 8));
    TRY(dalloc(c, &p.pk_cnt, (size_t)p.nchunk * G));
    TRY(dalloc(c, &p.pk_cap, (size_t)p.nchunk * G));
    p.xcap_frac = getenv("GM_XCHG_CAP_FRAC") ? (float)atof(getenv("GM_XCHG_CAP_FRAC")) : 0.f;
    if (p.xcap_frac < 0.f || p.xcap_frac > 1.f) return GM_EINVAL;
    TRY(dalloc(c, &p.recv_hdr, (size_t)std::max(R, 1) * 8));
    for (int q = 0; q < 2; q++) TRY(dalloc(c, &p.recv_list[q], (size_t)std::max(R, 1) * p.V));
    std::vector<int32_t> b(G + 1);
    for (int g = 0; g <= G; g++) b[g] = (int32_t)((int64_t)n * g / G);
    TRY(dalloc(c, &p.shard_n0, G + 1));
    HIPCHECK(ctx_memcpy(c, p.shard_n0, b.data(), sizeof(int32_t) * (G + 1), hipMemcpyHostToDevice));
    TRY(partial_caps(c));
  }
  HIPCHECK(ctx_memset(c, p.lists, 0, sizeof(uint64_t) * 2 * p.rows * p.V));
  HIPCHECK(ctx_memset(c, p.failed, 0, sizeof(int32_t) * nl));
  HIPCHECK(ctx_memset(c, p.ev_cnt, 0, sizeof(int32_t) * nl));
  HIPCHECK(ctx_memset(c, p.ev_jm, 0, sizeof(uint32_t) * nl));
  HIPCHECK(ctx_memset(c, p.rowstat, 0, sizeof(int32_t) * nl * 4));
  HIPCHECK(ctx_memset(c, p.err, 0, sizeof(uint32_t)));
  HIPCHECK(gm_launch_partial_init(p, t0, c->cfg.init_seed, c->stream));
  HIPCHECK(hipStreamSynchronize(c->stream));
  c->t = t0 + 1;
  return GM_OK;
}

// diagnostics (GM_CREATE_TIMING): where context creation time goes
static std::chrono::steady_clock::time_point g_ctime;
static void lap(const char *what) {
  if (!getenv("GM_CREATE_TIMING")) return;
  const auto t1 = std::chrono::steady_clock::now();
  fprintf(stderr, "[gm] create: %-24s %7.2f ms\n", what, std::chrono::duration<double, std::milli>(t1 - g_ctime).count());
  g_ctime = t1;
}

extern "C" int gm_create(const gm_config *cfg, gm_ctx **out) {
  if (!cfg || !out) return GM_EINVAL;
  *out = nullptr;
  if (cfg->abi_version != GM_ABI_VERSION) return GM_EINVAL;
  if (cfg->n <= 0 || (cfg->mode != GM_MODE_FAITHFUL && cfg->mode != GM_MODE_SCALED && cfg->mode != GM_MODE_PARTIAL))
    return GM_EINVAL;
  g_errbuf[0] = 0;
  gm_ctx *c = new gm_ctx();
  c->cfg = *cfg;
  c->n = cfg->n;
  c->failed_h.assign(cfg->n, 0);
  c->fail_t.assign(cfg->n, 0x7FFFFFFF);
  int rc = GM_OK;
  g_ctime = std::chrono::steady_clock::now();
  if (hipSetDevice(cfg->device) != hipSuccess) rc = GM_EDEVICE;
  lap("hipSetDevice");
  if (rc == GM_OK && hipFree(nullptr) != hipSuccess) rc = GM_EDEVICE;  // runtime + device init
  lap("runtime init");
  if (rc != GM_OK || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&c->e0) != hipSuccess || hipEventCreate(&c->e1) != hipSuccess ||
      hipEventCreate(&c->k0) != hipSuccess || hipEventCreate(&c->k1) != hipSuccess) {
    snprintf(g_errbuf, sizeof g_errbuf, "HIP device %d unavailable", cfg->device);
    rc = GM_EDEVICE;
  }
  lap("stream + events");
  if (rc == GM_OK)
    rc = cfg->mode == GM_MODE_FAITHFUL ? create_faithful(c) : cfg->mode == GM_MODE_SCALED ? create_scaled(c)
                                                                                        : create_partial(c);
  lap("mode state");
  if (rc != GM_OK) {
    gm_destroy(c);
    return rc;
  }
  *out = c;
  return GM_OK;
}

extern "C" int gm_destroy(gm_ctx *c) {
  if (!c) return GM_EINVAL;
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->p_side) (void)hipStreamSynchronize(c->p_side);  // the S2 prefetch of tick t+1 may still be writing
  if (c->p_comm) (void)hipStreamSynchronize(c->p_comm);
  if (c->comm) (void)ncclCommDestroy(c->comm);
  for (void *p : c->allocs) (void)hipFree(p);
  if (c->draw_left_h) (void)hipHostFree(c->draw_left_h);
  if (c->draw_ev) (void)hipEventDestroy(c->draw_ev);
  if (c->f_mail) (void)hipHostFree(c->f_mail);
  for (hipEvent_t e : {c->e0, c->e1, c->k0, c->k1})
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->tev) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->p_chev) (void)hipEventDestroy(e);
  if (c->p_done) (void)hipEventDestroy(c->p_done);
  if (c->p_comm) (void)hipStreamDestroy(c->p_comm);
  if (c->p_side) {
    (void)hipStreamSynchronize(c->p_side);
    (void)hipStreamDestroy(c->p_side);
  }
  for (int q = 0; q < 2; q++) {
    if (c->p_tickev[q]) (void)hipEventDestroy(c->p_tickev[q]);
    if (c->p_mtev[q]) (void)hipEventDestroy(c->p_mtev[q]);
  }
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return GM_OK;
}

static int check_err(gm_ctx *c) {
  uint32_t *errp = c->cfg.mode == GM_MODE_FAITHFUL ? c->f.err : c->cfg.mode == GM_MODE_SCALED ? c->s.err : c->p.err;
  uint32_t e = 0;
  HIPCHECK(hipMemcpyAsync(&e, errp, sizeof e, hipMemcpyDeviceToHost, c->stream));
  HIPCHECK(hipStreamSynchronize(c->stream));
  if (e) {
    snprintf(g_errbuf, sizeof g_errbuf, "device error flags 0x%x", e);
    c->latched = (e & (GM_ERR_SELF | GM_ERR_BUFFER)) ? GM_ESTATE : GM_ERANGE;
  }
  return c->latched;
}

static bool ev_order(const FEvent &a, const FEvent &b) {
  if (a.t != b.t) return a.t < b.t;
  if (a.logger != b.logger) return a.logger > b.logger;  // node phase: i descending
  return a.seq < b.seq;
}

// Records of a FAITHFUL tick can be at most n * (2n + 4): per node n joins, n removals and
// the start / join / time-mark lines.
static int64_t f_tick_event_bound(const gm_ctx *c) { return (int64_t)c->n * (2 * c->n + 4); }

// Collect the mailbox of every tick enqueued since the last collection: one copy of the
// count, the error flags and the first GM_F_MAILBOX records (more: a second copy), one
// wait; the records are staged to `pending` in the reference's order, the count reset in
// stream order.
static int f_collect(gm_ctx *c) {
  if (c->f_inflight == 0) return c->latched;
  c->f_inflight = 0;
  HIPCHECK(hipMemcpyAsync(c->f_mail, c->f.ev_count, 16 + sizeof(FEvent) * GM_F_MAILBOX, hipMemcpyDeviceToHost,
                          c->stream));
  HIPCHECK(hipStreamSynchronize(c->stream));
  const unsigned long long nev = *(const unsigned long long *)c->f_mail;
  const uint32_t e = *(const uint32_t *)((const uint8_t *)c->f_mail + 8);
  HIPCHECK(hipMemsetAsync(c->f.ev_count, 0, sizeof(unsigned long long), c->stream));
  if (nev > (unsigned long long)c->f.ev_cap) {
    c->latched = GM_ERANGE;
    return c->latched;
  }
  if (nev) {
    std::vector<FEvent> ev(nev);
    memcpy(ev.data(), (const uint8_t *)c->f_mail + 16, sizeof(FEvent) * std::min<size_t>(nev, GM_F_MAILBOX));
    if (nev > GM_F_MAILBOX) {
      HIPCHECK(ctx_memcpy(c, ev.data() + GM_F_MAILBOX, c->f.ev + GM_F_MAILBOX, sizeof(FEvent) * (nev - GM_F_MAILBOX),
                         hipMemcpyDeviceToHost));
    }
    std::sort(ev.begin(), ev.end(), ev_order);
    for (const FEvent &e : ev) {
      c->pending.push_back(gm_event{e.t, e.logger, e.kind, e.subject});
      if (e.kind > 0 && e.kind < 6) c->ev_tot[e.kind]++;
    }
  }
  if (e) {
    snprintf(g_errbuf, sizeof g_errbuf, "device error flags 0x%x", e);
    c->latched = (e & (GM_ERR_SELF | GM_ERR_BUFFER)) ? GM_ESTATE : GM_ERANGE;
  }
  return c->latched;
}

static int draw_settle(gm_ctx *c);

// Everything that reads the state (records, tables, counters, the S1 stream) or starts the
// next tick first completes the enqueued ticks: FAITHFUL collects its mailboxes; a column
// shard finishes the draws its bounded rounds left (rare).
static int f_settle(gm_ctx *c) {
  return c->cfg.mode == GM_MODE_FAITHFUL ? f_collect(c) : c->cfg.mode == GM_MODE_SCALED ? draw_settle(c) : GM_OK;
}

// FAITHFUL ticks are enqueued without a host wait: the records stay on the device until a
// call needs them (f_settle) or the next tick could overflow the record buffer.
static int tick_faithful(gm_ctx *c) {
  if (c->t >= F_MAX_TIME) return GM_ERANGE;  // EmulNet.cpp:109 assert(time < MAX_TIME)
  if ((c->f_inflight + 1) * f_tick_event_bound(c) > c->f.ev_cap) TRY(f_collect(c));
  // nodeStart of this tick's starters resets bFailed on the device (MP1Node.cpp:108-116); mirror it
  for (int i = 0; i < c->n; i++)
    if ((int)(0.25 * i) == c->t && c->failed_h[i]) {
      c->failed_h[i] = 0;
      c->fail_t[i] = 0x7FFFFFFF;
      c->nfailed--;
    }
  FState st = c->f;
  hipLaunchKernelGGL(gm_f_recv, dim3(1), dim3(1024), F_RECV_LDS, c->stream, st, c->t);
  hipLaunchKernelGGL(gm_f_recvout, dim3(64), dim3(256), 0, c->stream, st, c->t);
  std::swap(c->f.buf, c->f.buf2);  // gm_f_recvout compacted the survivors into buf2
  std::swap(c->f.bkey, c->f.bkey2);
  st = c->f;
  st.drop_pct_now = c->dropmsg ? (int)(c->cfg.drop_prob * 100) : -1;  // EmulNet.cpp:92
  hipLaunchKernelGGL(gm_f_node, dim3(c->n), dim3(256), c->f_smem, c->stream, st, c->t);
  hipLaunchKernelGGL(gm_f_sendprep, dim3(1), dim3(64), 0, c->stream, st);
  const int rounds = st.draw_cap / 31 + 1;
  hipLaunchKernelGGL(gm_f_s1expand, dim3(std::min(1024, (rounds + 7) / 8)), dim3(256), 0, c->stream, st);
  hipLaunchKernelGGL(gm_f_sendscan, dim3(1), dim3(1024), 0, c->stream, st, c->t);
  hipLaunchKernelGGL(gm_f_sendemit, dim3(std::min(1024, (st.draw_cap + 255) / 256)), dim3(256), 0, c->stream, st);
  HIPCHECK(hipGetLastError());
  c->f_inflight++;
  return c->latched;
}

static int tick_sharded(gm_ctx *c);
static int before_tick_events(gm_ctx *c);

// Tick-kernel timing: a ring of GM_TEV_RING event pairs on the context stream; a slot
// is folded into kernel_ms_sum when it is reused (its tick finished long before).
#define GM_TEV_RING 64
static int timing_slot(gm_ctx *c, hipEvent_t *k0, hipEvent_t *k1) {
  if (c->timed_ticks == 0) HIPCHECK(hipEventRecord(c->e0, c->stream));
  while (c->tev.size() < 2 * (size_t)GM_TEV_RING) {
    hipEvent_t e;
    HIPCHECK(hipEventCreate(&e));
    c->tev.push_back(e);
  }
  const int slot = c->ktimed % GM_TEV_RING;
  if (c->ktimed >= GM_TEV_RING) {
    float x = 0;
    HIPCHECK(hipEventSynchronize(c->tev[2 * slot + 1]));
    HIPCHECK(hipEventElapsedTime(&x, c->tev[2 * slot], c->tev[2 * slot + 1]));
    c->kernel_ms_sum += x;
  }
  *k0 = c->tev[2 * slot];
  *k1 = c->tev[2 * slot + 1];
  c->ktimed++;
  return GM_OK;
}

// Join ramp: nodeStart of this tick's starters clears bFailed (MP1Node.cpp:108)
static int ramp_starters(gm_ctx *c) {
  if (!c->s.ramp) return GM_OK;
  const int j0 = 4 * c->t, j1 = std::min(c->n, 4 * c->t + 4);
  for (int j = j0; j < j1; j++)
    if (c->failed_h[j]) {
      c->failed_h[j] = 0;
      c->fail_t[j] = 0x7FFFFFFF;
      c->nfailed--;
      HIPCHECK(hipMemcpyAsync(c->s.failed + j, c->failed_h.data() + j, sizeof(int32_t), hipMemcpyHostToDevice,
                              c->stream));
    }
  return GM_OK;
}

static int tick_scaled(gm_ctx *c) {
  if (c->t > GM_T_LIMIT) return GM_ERANGE;
  if (c->s.sharded) return tick_sharded(c);
  TRY(ramp_starters(c));
  const int t_send = c->t - 1;
  const bool drop = c->cfg.drop_pct > 0 && t_send >= c->cfg.drop_from && t_send < c->cfg.drop_to;
  hipEvent_t k0 = nullptr, k1 = nullptr;
  if (c->timing) TRY(timing_slot(c, &k0, &k1));
  HIPCHECK(gm_launch_tick(c->s, c->t, drop ? c->cfg.drop_pct : -1, c->stream, k0, k1, true));
  if (c->s.mc_sent && c->t < c->s.mc_tmax) {
    HIPCHECK(gm_launch_msgcount(c->s, c->t, drop, 0, c->stream));
    HIPCHECK(gm_launch_msgcount(c->s, c->t, drop, 1, c->stream));
  }
  if (c->timing) {
    HIPCHECK(hipEventRecord(c->e1, c->stream));
    c->timed_ticks++;
  }
  return GM_OK;
}

static int partial_exchange_chunk(gm_ctx *c, int q, int64_t *roff);

static int tick_partial(gm_ctx *c) {
  if (c->t > GM_T_LIMIT) return GM_ERANGE;
  if (c->p_sharded && !c->comm) return GM_EUNSUPPORTED;  // row shards need gm_comm_init (or gm_partial_loopback)
  const int t_send = c->t - 1;
  const bool drop = c->cfg.drop_pct > 0 && t_send >= c->cfg.drop_from && t_send < c->cfg.drop_to;
  PState st = c->p;
  st.drop_pct = drop ? c->cfg.drop_pct : -1;
  hipEvent_t k0 = nullptr, k1 = nullptr;
  if (c->timing) TRY(timing_slot(c, &k0, &k1));
  // S2 outputs of this tick: prefetched on the side stream while the last tick ran
  // (they depend only on (seed, t, id)), else computed here
  const int t = c->t, par = t & 1;
  uint32_t *mt = c->p_mtraw + (size_t)par * st.nloc * 16;
  if (c->p_mt_next == t) {
    HIPCHECK(hipStreamWaitEvent(c->stream, c->p_mtev[par], 0));
    HIPCHECK(gm_launch_partial_reset(st, c->stream));
  } else {
    HIPCHECK(gm_launch_partial_mtgen(st, t, mt, c->stream, true));
  }
  if (k0) HIPCHECK(hipEventRecord(k0, c->stream));
  if (!c->p_sharded) {
    HIPCHECK(gm_launch_partial_chunk(st, t, mt, 0, c->stream));
    if (k1) HIPCHECK(hipEventRecord(k1, c->stream));
  } else {
    if (c->p_crash_check) {
      // the block capacities (send counts of this rank, receive counts of its peers) derive from the
      // crash set each rank was given (gm_set_failed): a rank holding another set would size its
      // ncclAllToAllv differently and hang or corrupt it. One MAX-allreduce of (h, ~h) after each
      // change shows any disagreement, and the context latches GM_ESTATE instead.
      c->p_crash_check = false;
      if (!c->p_crash_dev) {
        HIPCHECK(hipMalloc(&c->p_crash_dev, 2 * sizeof(uint64_t)));
        c->allocs.push_back(c->p_crash_dev);
      }
      uint64_t hv[2] = {c->p_crash_hash, ~c->p_crash_hash}, mx[2] = {0, 0};
      HIPCHECK(hipMemcpyAsync(c->p_crash_dev, hv, sizeof hv, hipMemcpyHostToDevice, c->stream));
      NCCLCHECK(ncclAllReduce(c->p_crash_dev, c->p_crash_dev, 2, ncclUint64, ncclMax, c->comm, c->stream));
      HIPCHECK(hipMemcpyAsync(mx, c->p_crash_dev, sizeof mx, hipMemcpyDeviceToHost, c->stream));
      HIPCHECK(hipStreamSynchronize(c->stream));
      if (mx[0] != hv[0] || mx[1] != hv[1]) {
        c->latched = GM_ESTATE;
        return c->latched;
      }
    }
    // chunk pipeline: every chunk's node ticks queue on the compute stream; the exchange of
    // chunk q runs on the comm stream once q's kernels are done, while q+1.. still compute
    for (int q = 0; q < st.nchunk; q++) {
      HIPCHECK(gm_launch_partial_chunk(st, t, mt, q, c->stream));
      HIPCHECK(hipEventRecord(c->p_chev[q], c->stream));
    }
    if (k1) HIPCHECK(hipEventRecord(k1, c->stream));
    int64_t roff = 0;
    for (int q = 0; q < st.nchunk; q++) {
      HIPCHECK(hipStreamWaitEvent(c->p_comm, c->p_chev[q], 0));
      TRY(partial_exchange_chunk(c, q, &roff));
    }
    c->p_recv_last = roff;
    HIPCHECK(hipEventRecord(c->p_done, c->p_comm));
    HIPCHECK(hipStreamWaitEvent(c->stream, c->p_done, 0));  // the next tick reads the unpacked inboxes
  }
  // prefetch tick t+1's S2 outputs into the other parity buffer, last read by tick t-1
  HIPCHECK(hipEventRecord(c->p_tickev[par], c->stream));
  HIPCHECK(hipStreamWaitEvent(c->p_side, c->p_tickev[par ^ 1], 0));
  HIPCHECK(gm_launch_partial_mtgen(st, t + 1, c->p_mtraw + (size_t)(par ^ 1) * st.nloc * 16, c->p_side, false));
  HIPCHECK(hipEventRecord(c->p_mtev[par ^ 1], c->p_side));
  c->p_mt_next = t + 1;
  if (c->timing) {
    HIPCHECK(hipEventRecord(c->e1, c->stream));
    c->timed_ticks++;
  }
  return GM_OK;
}

extern "C" int gm_tick(gm_ctx *c) {
  if (!c) return GM_EINVAL;
  if (c->latched != GM_OK) return c->latched;
  if (c->cfg.mode == GM_MODE_SCALED) TRY(draw_settle(c));
  TRY(before_tick_events(c));
  int rc = c->cfg.mode == GM_MODE_FAITHFUL ? tick_faithful(c) : c->cfg.mode == GM_MODE_SCALED ? tick_scaled(c)
                                                                                             : tick_partial(c);
  if (rc == GM_OK) {
    c->t++;
    c->ticks_done++;
    c->undrained = c->cfg.mode != GM_MODE_FAITHFUL;
  }
  return rc;
}

extern "C" int gm_sync(gm_ctx *c) {
  if (!c) return GM_EINVAL;
  TRY(f_settle(c));
  if (c->cfg.mode == GM_MODE_SCALED) TRY(draw_settle(c));  // a sharded tick's remaining draw rounds
  HIPCHECK(hipStreamSynchronize(c->stream));
  return check_err(c);
}

extern "C" int gm_time(gm_ctx *c, int32_t *t) {
  if (!c || !t) return GM_EINVAL;
  *t = c->t;
  return GM_OK;
}

extern "C" int gm_rand(gm_ctx *c, int32_t *out) {
  if (!c || !out) return GM_EINVAL;
  if (c->cfg.mode != GM_MODE_FAITHFUL) return GM_EUNSUPPORTED;
  TRY(f_settle(c));
  int32_t st[33];
  HIPCHECK(hipMemcpyAsync(st, c->f.s1, sizeof st, hipMemcpyDeviceToHost, c->stream));
  HIPCHECK(hipStreamSynchronize(c->stream));
  int f = st[31], r = st[32];
  uint32_t v = (uint32_t)st[f] + (uint32_t)st[r];
  st[f] = (int32_t)v;
  st[31] = (f + 1) % 31;
  st[32] = (r + 1) % 31;
  HIPCHECK(ctx_memcpy(c, c->f.s1, st, sizeof st, hipMemcpyHostToDevice));
  *out = (int32_t)(v >> 1);
  return GM_OK;
}

extern "C" int gm_set_failed(gm_ctx *c, const int32_t *idx, int32_t n) {
  if (!c || n < 0 || (n > 0 && !idx)) return GM_EINVAL;
  for (int k = 0; k < n; k++)  // validate everything before any state changes
    if (idx[k] < 0 || idx[k] >= c->n) return GM_EINVAL;
  TRY(f_settle(c));
  for (int k = 0; k < n; k++) {
    c->nfailed += c->failed_h[idx[k]] == 0;
    if (!c->failed_h[idx[k]]) c->fail_t[idx[k]] = c->t - 1;
    c->failed_h[idx[k]] = 1;
    // join ramp: the introducer's last tick bounds who gets a JOINREP
    if (idx[k] == 0 && c->cfg.mode == GM_MODE_SCALED && c->s.ramp) c->s.intro_until = std::min(c->s.intro_until, c->t - 1);
  }
  int32_t *dst = c->cfg.mode == GM_MODE_FAITHFUL ? c->f.failed : c->cfg.mode == GM_MODE_SCALED ? c->s.failed : c->p.failed;
  const bool part = c->cfg.mode == GM_MODE_PARTIAL;  // a row shard holds its own nodes' flags only
  HIPCHECK(hipStreamSynchronize(c->stream));
  HIPCHECK(ctx_memcpy(c, dst, c->failed_h.data() + (part ? c->p.n0 : 0), sizeof(int32_t) * (part ? c->p.nloc : c->n),
                     hipMemcpyHostToDevice));
  if (part && c->p_sharded) TRY(partial_caps(c));  // the exchange blocks follow the live nodes per shard
  return GM_OK;
}

extern "C" int gm_set_dropmsg(gm_ctx *c, int32_t on) {
  if (!c) return GM_EINVAL;
  c->dropmsg = on ? 1 : 0;
  return GM_OK;
}

// The S_BC words of the last tick in (row, band) order (the device keeps [band][row] records).
static int read_bcnt(gm_ctx *c, std::vector<uint32_t> &bc) {
  const SState &s = c->s;
  const size_t n = (size_t)c->n, nrb = n * s.nb;
  std::vector<uint4> rec(nrb);
  HIPCHECK(hipMemcpyAsync(rec.data(), s.brec, sizeof(uint4) * nrb, hipMemcpyDeviceToHost, c->stream));
  HIPCHECK(hipStreamSynchronize(c->stream));
  bc.resize(nrb);
  for (size_t b = 0; b < (size_t)s.nb; b++)
    for (size_t r = 0; r < n; r++) bc[r * s.nb + b] = rec[b * n + r].z;
  return GM_OK;
}

// Host-side staging bound: records kept for gm_drain_events (a caller that never drains gets
// GM_ERANGE instead of unbounded host memory)
#define GM_PENDING_CAP (1ull << 27)

// The escape entries of one (band, row) list (k of them: inline slot, then pool) -> values by
// column of the row; GM_ESTATE if the record cannot hold them or an entry's column is no escape
static int place_entries(const SState &s, int b, const uint8_t *piece, const uint32_t *inl, const uint32_t *pool,
                         size_t k, uint16_t *esc_row) {
  for (size_t i = 0; i < k; i++) {
    const uint32_t e = i < S_ESC_IN ? inl[i] : pool[i - S_ESC_IN];
    const uint32_t col = e & 0xFFFFu;
    if (col >= (uint32_t)s.band || !s_is_esc(piece[col])) return GM_ESTATE;
    esc_row[(size_t)b * s.band + col] = (uint16_t)(e >> 16);
  }
  return GM_OK;
}

// SCALED: the last tick's join + remove records (the band kernel's striped partial sums) and
// how many of them spilled to the ring
static int tick_event_total(gm_ctx *c, uint64_t *total, uint32_t *spilled) {
  std::vector<uint32_t> cnt(1 + S_EV_STRIPES);
  HIPCHECK(hipMemcpyAsync(cnt.data(), c->s.ev_spill_cnt, sizeof(uint32_t) * cnt.size(), hipMemcpyDeviceToHost, c->stream));
  HIPCHECK(hipStreamSynchronize(c->stream));
  *spilled = cnt[0];
  *total = 0;
  for (int k = 1; k <= S_EV_STRIPES; k++) *total += cnt[k];
  return GM_OK;
}

static int drain_scaled(gm_ctx *c, std::vector<gm_event> &out) {
  const SState &s = c->s;
  const size_t nrb = (size_t)c->n * s.nb;
  std::vector<uint32_t> bc;
  uint64_t total = 0;
  uint32_t nsp = 0;
  TRY(tick_event_total(c, &total, &nsp));
  if (total == 0) return GM_OK;  // the common tick: nothing to stage, one 1 KB copy
  if (out.size() + total > GM_PENDING_CAP) return GM_ERANGE;
  TRY(read_bcnt(c, bc));
  const int t = c->t - 1;
  auto push = [&](int r, uint32_t rec) {
    out.push_back(gm_event{t, r, (int)(rec >> 30) == (int)S_EV_ADD ? GM_EV_JOINED : GM_EV_REMOVED,
                           (int32_t)(rec & 0x3FFFFFFFu)});
  };
  bool any = false;
  for (uint32_t v : bc) any |= S_BC_NEV(v) != 0;
  if (any) {
    std::vector<uint32_t> ev(nrb * s.evs);
    HIPCHECK(ctx_memcpy(c, ev.data(), s.ev_band, sizeof(uint32_t) * ev.size(), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < nrb; i++) {
      const int k = std::min<int>((int)S_BC_NEV(bc[i]), s.evs);
      for (int q = 0; q < k; q++) push((int)(i / s.nb), ev[i * s.evs + q]);
    }
  }
  nsp = std::min(nsp, s.ev_spill_cap);
  if (nsp) {
    std::vector<uint64_t> sp(nsp);
    HIPCHECK(ctx_memcpy(c, sp.data(), s.ev_spill, sizeof(uint64_t) * nsp, hipMemcpyDeviceToHost));
    for (uint64_t v : sp) push((int)(v >> 32), (uint32_t)v);
  }
  return GM_OK;
}

static void sort_canonical(std::vector<gm_event>::iterator b, std::vector<gm_event>::iterator e) {
  // canonical order of the build-defined modes: loggers descending; joins ascending id, then removals descending id
  std::sort(b, e, [](const gm_event &a, const gm_event &b) {
    if (a.logger != b.logger) return a.logger > b.logger;
    if (a.kind != b.kind) return a.kind < b.kind;
    return a.kind == GM_EV_JOINED ? a.subject < b.subject : a.subject > b.subject;
  });
}

static int drain_partial(gm_ctx *c, std::vector<gm_event> &out) {
  const PState &p = c->p;
  std::vector<int32_t> cnt(p.nloc);
  HIPCHECK(hipMemcpyAsync(cnt.data(), p.ev_cnt, sizeof(int32_t) * p.nloc, hipMemcpyDeviceToHost, c->stream));
  HIPCHECK(hipStreamSynchronize(c->stream));
  size_t tot = 0;
  for (int32_t v : cnt) tot += (size_t)(v & 0xFFFF) + (size_t)(v >> 16);
  if (!tot) return GM_OK;
  // joins: the set bits of each node's join mask over its final list of the tick (lists of parity t & 1,
  // intact until tick t + 2); removals: the records at the back of the node's event row
  const size_t row = 2 * (size_t)p.V;
  const int t = c->t - 1;
  std::vector<uint32_t> jm(p.nloc);
  HIPCHECK(ctx_memcpy(c, jm.data(), p.ev_jm, sizeof(uint32_t) * jm.size(), hipMemcpyDeviceToHost));
  // only the rows that hold events are copied: runs of such rows as async copies on the context
  // stream, one wait at the end -- not the whole list / event buffers (~4.3 GB of lists
  // per S-C context for a tick with any join). Gaps up to `gap` rows are bridged, so there are at
  // most ~4096 copies however the rows are spread.
  const int gap = std::max(64, p.nloc / 4096);
  auto copy_rows = [&](void *dst, const void *src, size_t rowb, int sel) -> hipError_t {
    int r = 0;
    while (r < p.nloc) {
      auto has = [&](int q) { return sel == 0 ? (cnt[q] & 0xFFFF) != 0 : (cnt[q] >> 16) != 0; };
      while (r < p.nloc && !has(r)) r++;
      if (r >= p.nloc) break;
      int e = r + 1, last = r;
      while (e < p.nloc && e - last <= gap) {
        if (has(e)) last = e;
        e++;
      }
      const hipError_t err = hipMemcpyAsync((uint8_t *)dst + (size_t)r * rowb, (const uint8_t *)src + (size_t)r * rowb,
                                            (size_t)(last + 1 - r) * rowb, hipMemcpyDeviceToHost, c->stream);
      if (err != hipSuccess) return err;
      r = last + 1;
    }
    return hipSuccess;
  };
  bool any_join = false, any_rem = false;
  for (int32_t v : cnt) {
    any_join |= (v & 0xFFFF) != 0;
    any_rem |= (v >> 16) != 0;
  }
  std::vector<uint64_t> lst;
  if (any_join) {
    lst.resize((size_t)p.nloc * p.V);
    HIPCHECK(copy_rows(lst.data(), p.lists + (size_t)(t & 1) * p.rows * p.V, sizeof(uint64_t) * p.V, 0));
  }
  std::vector<uint32_t> ev;
  if (any_rem) {
    ev.resize((size_t)p.nloc * row);
    HIPCHECK(copy_rows(ev.data(), p.ev, sizeof(uint32_t) * row, 1));
  }
  HIPCHECK(hipStreamSynchronize(c->stream));
  out.reserve(out.size() + tot);
  for (int r = 0; r < p.nloc; r++) {
    const int nj = cnt[r] & 0xFFFF, nr = cnt[r] >> 16;
    if (__builtin_popcount(jm[r]) != nj) return GM_ESTATE;
    for (uint32_t b = jm[r]; b; b &= b - 1)
      out.push_back(gm_event{t, p.n0 + r, GM_EV_JOINED, (int32_t)(lst[(size_t)r * p.V + __builtin_ctz(b)] >> 32)});
    for (int q = 0; q < nr; q++)
      out.push_back(gm_event{t, p.n0 + r, GM_EV_REMOVED, (int32_t)(ev[(size_t)r * row + row - 1 - q] & 0x3FFFFFFFu)});
  }
  return GM_OK;
}

// SCALED / PARTIAL: move the last tick's device records (one tick's worth is kept on the
// device, overwritten by the next tick) to the host list, in canonical order.
static int stage_events(gm_ctx *c) {
  TRY(f_settle(c));
  if (!c->undrained) return GM_OK;
  c->undrained = false;
  const size_t first = c->pending.size();
  if (c->cfg.mode == GM_MODE_SCALED) TRY(drain_scaled(c, c->pending));
  else if (c->cfg.mode == GM_MODE_PARTIAL) TRY(drain_partial(c, c->pending));
  sort_canonical(c->pending.begin() + first, c->pending.end());
  return GM_OK;
}

// Before a tick overwrites the device records: stage them (keep_events) or drop them.
static int before_tick_events(gm_ctx *c) {
  if (c->cfg.mode == GM_MODE_FAITHFUL) return GM_OK;
  if (c->keep_events) return stage_events(c);
  c->undrained = false;
  return GM_OK;
}

extern "C" int gm_keep_events(gm_ctx *c, int32_t on) {
  if (!c) return GM_EINVAL;
  c->keep_events = on != 0;
  return GM_OK;
}

extern "C" int gm_drain_events(gm_ctx *c, gm_event *out, size_t cap, size_t *n) {
  if (!c || !n) return GM_EINVAL;
  TRY(stage_events(c));
  *n = c->pending.size();
  if (c->pending.size() > cap) return GM_ERANGE;
  if (!c->pending.empty()) memcpy(out, c->pending.data(), sizeof(gm_event) * c->pending.size());
  c->pending.clear();
  return GM_OK;
}

extern "C" int gm_event_counts(gm_ctx *c, uint64_t counts[6]) {
  if (!c || !counts) return GM_EINVAL;
  TRY(f_settle(c));
  for (int k = 0; k < 6; k++) counts[k] = 0;
  if (c->cfg.mode == GM_MODE_SCALED) {
    uint32_t nsp = 0;
    TRY(tick_event_total(c, &counts[0], &nsp));  // join+remove records of the last tick (per-kind split needs a drain)
  } else if (c->cfg.mode == GM_MODE_PARTIAL) {
    std::vector<int32_t> cnt(c->p.nloc);
    HIPCHECK(hipMemcpyAsync(cnt.data(), c->p.ev_cnt, sizeof(int32_t) * c->p.nloc, hipMemcpyDeviceToHost, c->stream));
    HIPCHECK(hipStreamSynchronize(c->stream));
    for (int32_t v : cnt) {
      counts[GM_EV_JOINED] += (uint64_t)(v & 0xFFFF);
      counts[GM_EV_REMOVED] += (uint64_t)(v >> 16);
    }
    counts[0] = counts[GM_EV_JOINED] + counts[GM_EV_REMOVED];
  } else {
    for (const gm_event &e : c->pending) counts[e.kind]++;
  }
  return GM_OK;
}

extern "C" int gm_event_totals(gm_ctx *c, uint64_t totals[6]) {
  if (!c || !totals) return GM_EINVAL;
  TRY(f_settle(c));
  for (int k = 0; k < 6; k++) totals[k] = c->ev_tot[k];
  if (c->cfg.mode == GM_MODE_PARTIAL) return GM_EUNSUPPORTED;
  if (c->cfg.mode == GM_MODE_SCALED) {
    std::vector<uint64_t> cum((size_t)c->n * c->s.nb);
    HIPCHECK(hipMemcpyAsync(cum.data(), c->s.evcum, sizeof(uint64_t) * cum.size(), hipMemcpyDeviceToHost, c->stream));
    HIPCHECK(hipStreamSynchronize(c->stream));
    uint64_t j = 0, r = 0;
    for (uint64_t v : cum) {
      j += (uint32_t)v;
      r += v >> 32;
    }
    totals[GM_EV_JOINED] = j;
    totals[GM_EV_REMOVED] = r;
  }
  totals[0] = 0;
  for (int k = 1; k < 6; k++) totals[0] += totals[k];
  return GM_OK;
}

// SCALED / PARTIAL: per-tick, per-node entry counts from the next tick on, for ticks < tmax
// (FAITHFUL always counts, as EmulNet does)
extern "C" int gm_msgcount_record(gm_ctx *c, int32_t tmax) {
  if (!c || tmax <= 0 || tmax > GM_T_LIMIT + 1) return GM_EINVAL;
  if (c->cfg.mode == GM_MODE_FAITHFUL) return GM_OK;
  if (c->ticks_done) return GM_ESTATE;  // the received counts need the senders' counts of the tick before
  if (c->cfg.mode == GM_MODE_SCALED ? c->s.mc_sent != nullptr : c->p.mc_sent != nullptr) return GM_ESTATE;
  const size_t rows = c->cfg.mode == GM_MODE_SCALED ? (size_t)c->n : (size_t)c->p.nloc;
  uint32_t *ms = nullptr, *mr = nullptr;
  TRY(dalloc(c, &ms, (size_t)tmax * rows));
  TRY(dalloc(c, &mr, (size_t)tmax * rows));
  HIPCHECK(hipMemsetAsync(ms, 0, sizeof(uint32_t) * tmax * rows, c->stream));
  HIPCHECK(hipMemsetAsync(mr, 0, sizeof(uint32_t) * tmax * rows, c->stream));
  if (c->cfg.mode == GM_MODE_SCALED) {
    TRY(dalloc(c, &c->s.mc_fresh, 2 * rows));
    TRY(dalloc(c, &c->s.mc_rdrop, rows));
    HIPCHECK(hipMemsetAsync(c->s.mc_fresh, 0, sizeof(uint32_t) * 2 * rows, c->stream));
    HIPCHECK(hipMemsetAsync(c->s.mc_rdrop, 0, sizeof(uint32_t) * rows, c->stream));
    c->s.mc_sent = ms;
    c->s.mc_recv = mr;
    c->s.mc_tmax = tmax;
  } else {
    c->p.mc_sent = ms;
    c->p.mc_recv = mr;
    c->p.mc_tmax = tmax;
  }
  return GM_OK;
}

extern "C" int gm_msgcount(gm_ctx *c, int32_t t, int32_t *sent, int32_t *recv) {
  if (!c || !sent || !recv || t < 0) return GM_EINVAL;
  TRY(f_settle(c));  // a column shard's last tick may still owe its host-driven draw rounds
  if (c->cfg.mode != GM_MODE_FAITHFUL) {  // [nodes][t] of this context's nodes, from the recorded history
    const bool sc = c->cfg.mode == GM_MODE_SCALED;
    const uint32_t *ms = sc ? c->s.mc_sent : c->p.mc_sent, *mr = sc ? c->s.mc_recv : c->p.mc_recv;
    const int tmax = sc ? c->s.mc_tmax : c->p.mc_tmax;
    if (!ms) return GM_ESTATE;  // gm_msgcount_record was not called
    if (t > tmax) return GM_EINVAL;
    const size_t rows = sc ? (size_t)c->n : (size_t)c->p.nloc;
    HIPCHECK(hipStreamSynchronize(c->stream));
    std::vector<uint32_t> hs((size_t)t * rows), hr(hs.size());
    if (t > 0) {
      HIPCHECK(ctx_memcpy(c, hs.data(), ms, sizeof(uint32_t) * hs.size(), hipMemcpyDeviceToHost));
      HIPCHECK(ctx_memcpy(c, hr.data(), mr, sizeof(uint32_t) * hr.size(), hipMemcpyDeviceToHost));
    }
    for (size_t i = 0; i < rows; i++)
      for (int j = 0; j < t; j++) {
        sent[i * t + j] = (int32_t)hs[(size_t)j * rows + i];
        recv[i * t + j] = (int32_t)hr[(size_t)j * rows + i];
      }
    return GM_OK;
  }
  if (t > c->f.tmax) return GM_EINVAL;
  TRY(f_settle(c));
  HIPCHECK(hipStreamSynchronize(c->stream));
  std::vector<int32_t> hs((size_t)(c->n + 1) * c->f.tmax), hr(hs.size());
  HIPCHECK(ctx_memcpy(c, hs.data(), c->f.sent, sizeof(int32_t) * hs.size(), hipMemcpyDeviceToHost));
  HIPCHECK(ctx_memcpy(c, hr.data(), c->f.recv, sizeof(int32_t) * hr.size(), hipMemcpyDeviceToHost));
  for (int i = 0; i < c->n; i++)
    for (int j = 0; j < t; j++) {
      sent[(size_t)i * t + j] = hs[(size_t)(i + 1) * c->f.tmax + j];
      recv[(size_t)i * t + j] = hr[(size_t)(i + 1) * c->f.tmax + j];
    }
  return GM_OK;
}

// One row of stored bytes (column order) -> absolute (hb, ts), -1 = absent; escaped cells take
// their value from `esc` (per column, from the row's escape entries). Cells are relative to the
// row's last written tick wt.
static void decode_scaled_row(const gm_ctx *c, const uint8_t *row, const uint16_t *esc, int wt,
                              std::vector<int32_t> &hb, std::vector<int32_t> &ts) {
  const SState &s = c->s;
  hb.resize(s.w);
  ts.resize(s.w);
  for (int j = 0; j < s.w; j++) {
    const uint32_t e = s_is_esc(row[j]) ? (uint32_t)esc[j] : s_widen(row[j]);
    hb[j] = e == 0 ? -1 : 2 * wt - 255 + (int32_t)S_H(e) - s_hbase(s.ramp, s.c0 + j);
    ts[j] = e == 0 ? -1 : wt - (int32_t)S_AGE(e);
  }
}

// Row r of this context's table as absolute (hb, ts) per column, -1 = absent.
static int read_table_row(gm_ctx *c, int r, std::vector<int32_t> &hb, std::vector<int32_t> &ts, int &w) {
  if (c->cfg.mode == GM_MODE_FAITHFUL) {
    TRY(f_settle(c));
    w = c->n;
    std::vector<uint32_t> row(w);
    HIPCHECK(ctx_memcpy(c, row.data(), c->f.table + (size_t)r * c->f.np, sizeof(uint32_t) * w, hipMemcpyDeviceToHost));
    hb.resize(w);
    ts.resize(w);
    for (int j = 0; j < w; j++) {
      hb[j] = row[j] == GM_ABSENT ? -1 : (int32_t)(row[j] & 0xFFFF);
      ts[j] = row[j] == GM_ABSENT ? -1 : (int32_t)(row[j] >> 16);
    }
    return GM_OK;
  }
  if (c->cfg.mode == GM_MODE_PARTIAL) {  // the node's V-entry list as of the last tick
    const PState &p = c->p;
    if (r < p.n0 || r >= p.n0 + p.nloc) return GM_EINVAL;  // another row shard's node
    std::vector<uint64_t> lst(p.V);
    HIPCHECK(ctx_memcpy(c, lst.data(), p.lists + ((size_t)((c->t - 1) & 1) * p.rows + (r - p.n0)) * p.V,
                       sizeof(uint64_t) * p.V, hipMemcpyDeviceToHost));
    w = c->n;
    hb.assign(w, -1);
    ts.assign(w, -1);
    for (uint64_t e : lst) {
      if (!e) continue;
      const int id = (int)(e >> 32), h = (int)(uint32_t)e;
      if (id < 1 || id > c->n) return GM_ESTATE;
      hb[id - 1] = h;
      ts[id - 1] = (h + 1) / 2;
    }
    return GM_OK;
  }
  const SState &s = c->s;  // band-tiled: one B-cell piece of the row per band slab
  w = s.w;  // this context's columns
  std::vector<uint8_t> row(s.wp);
  std::vector<uint32_t> eb(s.nb);
  int32_t wt = 0;
  const size_t piece = s.band;  // bytes of one (band, row) piece of the stored cells
  HIPCHECK(ctx_memcpy2d(c, row.data(), piece, s.table + (size_t)r * s.band, piece * s.n, piece, s.nb,
                        hipMemcpyDeviceToHost));
  HIPCHECK(ctx_memcpy2d(c, eb.data(), sizeof(uint32_t), (const uint8_t *)(s.brec + r) + 12, sizeof(uint4) * s.n,
                        sizeof(uint32_t), s.nb, hipMemcpyDeviceToHost));
  HIPCHECK(ctx_memcpy(c, &wt, s.wtick + r, sizeof wt, hipMemcpyDeviceToHost));
  std::vector<uint16_t> esc(s.wp);  // escaped cells by column (the entries of the row's band lists)
  const int par = (c->t - 1) & 1;
  std::vector<uint32_t> ent;
  for (int b = 0; b < s.nb; b++) {
    const uint8_t *piece = row.data() + (size_t)b * s.band;
    size_t k = 0;
    for (int j = 0; j < s.band; j++) k += s_is_esc(piece[j]);
    if (!k) continue;
    const size_t in = std::min<size_t>(k, S_ESC_IN);
    if (S_EW_TOT(eb[b]) != k || S_EW_OFF(eb[b]) + (k - in) > s.tesc_region) return GM_ESTATE;
    ent.resize(k);
    HIPCHECK(ctx_memcpy(c, ent.data(), s.tesc_in[par] + ((size_t)b * s.n + r) * S_ESC_IN, sizeof(uint32_t) * in,
                       hipMemcpyDeviceToHost));
    const size_t stripe = ((size_t)b * s.n + r) & (size_t)(s.esc_stripes - 1);
    if (k > in)
      HIPCHECK(ctx_memcpy(c, ent.data() + in, s.tesc[par] + stripe * s.tesc_region + S_EW_OFF(eb[b]),
                         sizeof(uint32_t) * (k - in), hipMemcpyDeviceToHost));
    TRY(place_entries(s, b, piece, ent.data(), ent.data() + S_ESC_IN, k, esc.data()));
  }
  decode_scaled_row(c, row.data(), esc.data(), wt, hb, ts);
  return GM_OK;
}

extern "C" int gm_read_row(gm_ctx *c, int32_t r, int32_t c0, int32_t len, int32_t *hb, int32_t *ts) {
  if (!c || !hb || !ts || r < 0 || r >= c->n || c0 < 0 || len < 0) return GM_EINVAL;
  TRY(f_settle(c));
  HIPCHECK(hipStreamSynchronize(c->stream));
  std::vector<int32_t> rh, rt;
  int w;
  TRY(read_table_row(c, r, rh, rt, w));
  if (c0 + len > w) return GM_EINVAL;
  for (int j = 0; j < len; j++) {
    hb[j] = rh[c0 + j];
    ts[j] = rt[c0 + j];
  }
  return GM_OK;
}

// SCALED bulk readback: one copy of the table, the records, the row ticks and the last
// tick's escape entries (inline + each stripe's used pool part), decoded row by row.
struct ScaledSnapshot {
  std::vector<uint8_t> tab, row;
  std::vector<uint4> rec;
  std::vector<std::vector<uint32_t>> pool;  // per stripe: its used part of the region
  std::vector<uint32_t> inl;
  std::vector<uint16_t> esc;
  std::vector<int32_t> wts;
  int load(gm_ctx *c) {
    const SState &s = c->s;
    tab.resize((size_t)s.n * s.wp);
    rec.resize((size_t)s.n * s.nb);
    wts.resize(s.n);
    std::vector<unsigned long long> cnt(s.esc_stripes);
    HIPCHECK(ctx_memcpy(c, tab.data(), s.table, tab.size(), hipMemcpyDeviceToHost));
    HIPCHECK(ctx_memcpy(c, rec.data(), s.brec, sizeof(uint4) * rec.size(), hipMemcpyDeviceToHost));
    HIPCHECK(ctx_memcpy(c, wts.data(), s.wtick, sizeof(int32_t) * s.n, hipMemcpyDeviceToHost));
    const int par = (c->t - 1) & 1;
    HIPCHECK(ctx_memcpy(c, cnt.data(), s.tesc_cnt + (size_t)par * s.esc_stripes, sizeof(unsigned long long) * cnt.size(),
                       hipMemcpyDeviceToHost));
    inl.resize((size_t)s.n * s.nb * S_ESC_IN);
    HIPCHECK(ctx_memcpy(c, inl.data(), s.tesc_in[par], sizeof(uint32_t) * inl.size(), hipMemcpyDeviceToHost));
    pool.assign(s.esc_stripes, {});
    for (int k = 0; k < s.esc_stripes; k++) {
      const size_t used = std::min<unsigned long long>(cnt[k], s.tesc_region);
      pool[k].resize(used);
      if (used)
        HIPCHECK(ctx_memcpy(c, pool[k].data(), s.tesc[par] + (size_t)k * s.tesc_region, sizeof(uint32_t) * used,
                           hipMemcpyDeviceToHost));
    }
    row.resize(s.wp);
    esc.resize(s.wp);
    return GM_OK;
  }
  int decode(const gm_ctx *c, int i, std::vector<int32_t> &rh, std::vector<int32_t> &rt) {
    const SState &s = c->s;
    for (int b = 0; b < s.nb; b++) {
      const uint8_t *pc = tab.data() + ((size_t)b * s.n + i) * s.band;
      memcpy(row.data() + (size_t)b * s.band, pc, s.band);
      size_t k = 0;
      for (int j = 0; j < s.band; j++) k += s_is_esc(pc[j]);
      if (!k) continue;
      const uint32_t w = rec[(size_t)b * s.n + i].w;
      const size_t in = std::min<size_t>(k, S_ESC_IN);
      const size_t stripe = ((size_t)b * s.n + i) & (size_t)(s.esc_stripes - 1);
      if (S_EW_TOT(w) != k || S_EW_OFF(w) + (k - in) > pool[stripe].size()) return GM_ESTATE;
      TRY(place_entries(s, b, pc, inl.data() + ((size_t)b * s.n + i) * S_ESC_IN,
                        pool[stripe].data() + (k > in ? S_EW_OFF(w) : 0), k, esc.data()));
    }
    decode_scaled_row(c, row.data(), esc.data(), wts[i], rh, rt);
    return GM_OK;
  }
};

extern "C" int gm_read_table(gm_ctx *c, int32_t r0, int32_t count, int32_t *hb, int32_t *ts) {
  if (!c || r0 < 0 || count < 0 || r0 + (int64_t)count > c->n || (count > 0 && (!hb || !ts))) return GM_EINVAL;
  TRY(f_settle(c));
  HIPCHECK(hipStreamSynchronize(c->stream));
  std::vector<int32_t> rh, rt;
  ScaledSnapshot snap;
  if (c->cfg.mode == GM_MODE_SCALED) TRY(snap.load(c));
  for (int i = 0; i < count; i++) {
    int w;
    if (c->cfg.mode == GM_MODE_SCALED) {
      TRY(snap.decode(c, r0 + i, rh, rt));
      w = c->s.w;
    } else {
      TRY(read_table_row(c, r0 + i, rh, rt, w));
    }
    memcpy(hb + (size_t)i * w, rh.data(), sizeof(int32_t) * w);
    memcpy(ts + (size_t)i * w, rt.data(), sizeof(int32_t) * w);
  }
  return GM_OK;
}

extern "C" int gm_read_views(gm_ctx *c, int32_t r0, int32_t count, uint64_t *out) {
  if (!c || count < 0 || (count > 0 && !out)) return GM_EINVAL;
  if (c->cfg.mode != GM_MODE_PARTIAL) return GM_EUNSUPPORTED;
  const PState &p = c->p;
  if (r0 < p.n0 || r0 + (int64_t)count > (int64_t)p.n0 + p.nloc) return GM_EINVAL;  // this shard's nodes only
  HIPCHECK(hipStreamSynchronize(c->stream));
  if (count)
    HIPCHECK(ctx_memcpy(c, out, p.lists + ((size_t)((c->t - 1) & 1) * p.rows + (r0 - p.n0)) * p.V,
                       sizeof(uint64_t) * p.V * (size_t)count, hipMemcpyDeviceToHost));
  return GM_OK;
}

extern "C" int gm_read_nodes(gm_ctx *c, int32_t *st4) {
  if (!c || !st4) return GM_EINVAL;
  TRY(f_settle(c));
  HIPCHECK(hipStreamSynchronize(c->stream));
  const int n = c->cfg.mode == GM_MODE_PARTIAL ? c->p.nloc : c->n;  // a row shard reports its own nodes
  std::vector<int32_t> a(n), b(n), f(n), h(n);
  if (c->cfg.mode == GM_MODE_FAITHFUL) {
    HIPCHECK(ctx_memcpy(c, a.data(), c->f.inited, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
    HIPCHECK(ctx_memcpy(c, b.data(), c->f.ingroup, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
    HIPCHECK(ctx_memcpy(c, f.data(), c->f.failed, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
    HIPCHECK(ctx_memcpy(c, h.data(), c->f.hbctr, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
  } else {
    const bool part = c->cfg.mode == GM_MODE_PARTIAL;
    std::fill(a.begin(), a.end(), 1);
    std::fill(b.begin(), b.end(), 1);
    if (!part && c->s.ramp) {  // join ramp: started (inited) / in the group as of the last tick
      const int t = c->t - 1;
      for (int i = 0; i < n; i++) {
        a[i] = t >= s_start(i);
        // JOINREP is processed at start+2 only by a node still running then
        b[i] = i == 0 ? a[i] : s_ingroup(1, c->s.intro_until, i, t) && c->fail_t[i] >= s_start(i) + 2;
      }
    }
    HIPCHECK(ctx_memcpy(c, f.data(), part ? c->p.failed : c->s.failed, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
    HIPCHECK(ctx_memcpy(c, h.data(), part ? c->p.hbctr : c->s.hbctr, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
  }
  for (int i = 0; i < n; i++) {
    st4[4 * i] = a[i];
    st4[4 * i + 1] = b[i];
    st4[4 * i + 2] = f[i];
    st4[4 * i + 3] = h[i];
  }
  return GM_OK;
}

extern "C" int gm_dump_tables(gm_ctx *c, char *buf, size_t cap, size_t *len) {
  if (!c || !len) return GM_EINVAL;
  std::vector<int32_t> st(4 * (size_t)c->n);
  TRY(gm_read_nodes(c, st.data()));
  std::string out;
  char tmp[96];
  const int t = c->t - 1;
  if (c->cfg.mode == GM_MODE_PARTIAL) {  // the V-entry lists (id order) of the last tick, one copy
    const PState &p = c->p;          // a row shard renders its own nodes (global indices)
    std::vector<uint64_t> all((size_t)p.nloc * p.V);
    HIPCHECK(ctx_memcpy(c, all.data(), p.lists + (size_t)(t & 1) * p.rows * p.V, sizeof(uint64_t) * all.size(),
                       hipMemcpyDeviceToHost));
    for (int i = 0; i < p.nloc; i++) {
      const uint64_t *row = all.data() + (size_t)i * p.V;
      int cnt = 0;
      for (int j = 0; j < p.V; j++) cnt += row[j] != 0;
      snprintf(tmp, sizeof tmp, "%d %d %d %d %d %d %d", t, p.n0 + i, st[4 * i], st[4 * i + 1], st[4 * i + 2],
               st[4 * i + 3], cnt);
      out += tmp;
      for (int j = 0; j < p.V; j++) {
        if (!row[j]) continue;
        const int h = (int)(uint32_t)row[j];
        snprintf(tmp, sizeof tmp, " %d:%d:%d", (int)(row[j] >> 32), h, (h + 1) / 2);
        out += tmp;
      }
      out += "\n";
    }
    *len = out.size();
    if (!buf || cap < out.size()) return GM_ERANGE;
    memcpy(buf, out.data(), out.size());
    return GM_OK;
  }
  std::vector<int32_t> rh, rt;
  ScaledSnapshot snap;
  if (c->cfg.mode == GM_MODE_SCALED) TRY(snap.load(c));
  for (int i = 0; i < c->n; i++) {
    int w;
    if (c->cfg.mode == GM_MODE_SCALED) {
      TRY(snap.decode(c, i, rh, rt));
      w = c->s.w;
    } else {
      TRY(read_table_row(c, i, rh, rt, w));
    }
    int cnt = 0;
    const int c0 = c->cfg.mode == GM_MODE_SCALED ? c->s.c0 : 0;
    for (int j = 0; j < w; j++) cnt += rh[j] >= 0;
    snprintf(tmp, sizeof tmp, "%d %d %d %d %d %d %d", t, i, st[4 * i], st[4 * i + 1], st[4 * i + 2], st[4 * i + 3], cnt);
    out += tmp;
    for (int j = 0; j < w; j++) {
      if (rh[j] < 0) continue;
      snprintf(tmp, sizeof tmp, " %d:%d:%d", c0 + j + 1, rh[j], rt[j]);
      out += tmp;
    }
    out += "\n";
  }
  *len = out.size();
  if (!buf || cap < out.size()) return GM_ERANGE;
  memcpy(buf, out.data(), out.size());
  return GM_OK;
}

extern "C" int gm_read_targets(gm_ctx *c, int32_t *targets, int32_t *counts) {
  if (!c || !targets || !counts) return GM_EINVAL;
  if (c->cfg.mode != GM_MODE_SCALED) return GM_EUNSUPPORTED;
  TRY(draw_settle(c));
  const size_t n = (size_t)c->n;
  std::vector<int32_t> st(n * 4);
  HIPCHECK(ctx_memcpy(c, targets, c->s.targets, sizeof(int32_t) * n * GM_FANOUT, hipMemcpyDeviceToHost));
  HIPCHECK(ctx_memcpy(c, st.data(), c->s.rowstat, sizeof(int32_t) * n * 4, hipMemcpyDeviceToHost));
  for (size_t r = 0; r < n; r++) {
    counts[r] = st[r * 4 + 3];
    for (int q = counts[r]; q < GM_FANOUT; q++) targets[r * GM_FANOUT + q] = 0;
  }
  return check_err(c);
}

extern "C" int gm_tick_stats(gm_ctx *c, int64_t stats[4]) {
  if (!c || !stats) return GM_EINVAL;
  if (c->cfg.mode == GM_MODE_FAITHFUL) return GM_EUNSUPPORTED;
  const bool part = c->cfg.mode == GM_MODE_PARTIAL;
  const int rows = part ? c->p.nloc : c->n, r0 = part ? c->p.n0 : 0;  // a row shard reports its own nodes
  std::vector<int32_t> rs((size_t)rows * 4);
  uint32_t e = 0;
  HIPCHECK(hipMemcpyAsync(rs.data(), part ? c->p.rowstat : c->s.rowstat, sizeof(int32_t) * rs.size(),
                          hipMemcpyDeviceToHost, c->stream));
  HIPCHECK(hipMemcpyAsync(&e, part ? c->p.err : c->s.err, sizeof e, hipMemcpyDeviceToHost, c->stream));
  HIPCHECK(hipStreamSynchronize(c->stream));
  int64_t m = 0, live = 0, mx = 0;
  for (int r = 0; r < rows; r++) {
    m += rs[4 * r];
    mx = std::max<int64_t>(mx, rs[4 * r]);
    live += c->failed_h[r0 + r] ? 0 : 1;
  }
  stats[0] = m;
  stats[1] = live;
  stats[2] = mx;
  stats[3] = e;
  return GM_OK;
}

extern "C" int gm_pool_info(gm_ctx *c, int64_t info[4]) {
  if (!c || !info) return GM_EINVAL;
  if (c->cfg.mode != GM_MODE_SCALED) return GM_EUNSUPPORTED;
  info[0] = c->s.esc_dense;
  info[1] = (int64_t)c->s.tesc_cap;
  info[2] = (int64_t)c->s.pesc_cap;
  info[3] = (int64_t)c->s.ev_spill_cap;
  return GM_OK;
}

extern "C" int gm_set_timing(gm_ctx *c, int32_t on) {
  if (!c) return GM_EINVAL;
  c->timing = on != 0;
  c->timed_ticks = 0;  // (re)opens the timing window at the next tick
  c->ktimed = 0;
  c->kernel_ms_sum = 0;
  return GM_OK;
}

extern "C" int gm_last_kernel_ms(gm_ctx *c, float *ms) {
  if (!c || !ms) return GM_EINVAL;
  *ms = 0.f;
  if (!c->timing || c->cfg.mode == GM_MODE_FAITHFUL || c->timed_ticks == 0) return GM_OK;
  HIPCHECK(hipEventSynchronize(c->e1));
  double sum = c->kernel_ms_sum;  // folded ring slots + the pairs still in the ring
  for (int k = std::max(0, c->ktimed - GM_TEV_RING); k < c->ktimed; k++) {
    const int slot = k % GM_TEV_RING;
    float x = 0;
    HIPCHECK(hipEventElapsedTime(&x, c->tev[2 * slot], c->tev[2 * slot + 1]));
    sum += x;
  }
  *ms = c->ktimed ? (float)(sum / c->ktimed) : 0.f;
  return GM_OK;
}

static uint64_t mix64h(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

extern "C" int gm_crash_set(int32_t n, int32_t count, uint64_t seed, int32_t *out) {
  if (n <= 0 || count < 0 || count > n || (count && !out)) return GM_EINVAL;
  std::vector<std::pair<uint64_t, int32_t>> k(n);
  for (int i = 0; i < n; i++) k[i] = {mix64h(seed + 0x9E3779B97F4A7C15ULL * (uint64_t)(i + 1)), i};
  std::partial_sort(k.begin(), k.begin() + count, k.end());
  for (int i = 0; i < count; i++) out[i] = k[i].second;
  std::sort(out, out + count);
  return GM_OK;
}

// ------------------------------------------------------------ column shards
// A tick of a column shard: merge/sweep own columns, all-gather per-row counts,
// then rounds of {draw, MAX-allreduce of resolved draws, accept} until every row
// has its targets. Collectives are RCCL on the context stream (gm_comm_init),
// or in-process between contexts of one device (gm_shard_loopback, tests).


extern "C" int gm_comm_unique_id(uint8_t *out128) {
  if (!out128) return GM_EINVAL;
  ncclUniqueId id;
  NCCLCHECK(ncclGetUniqueId(&id));
  memcpy(out128, &id, sizeof id);
  return GM_OK;
}

extern "C" int gm_comm_init(gm_ctx *c, const uint8_t *id128, int32_t nranks, int32_t rank) {
  if (!c || !id128) return GM_EINVAL;
  if (c->cfg.mode == GM_MODE_SCALED ? (c->s.shard_count != nranks || c->s.shard_rank != rank)
      : c->cfg.mode == GM_MODE_PARTIAL ? (c->p.G != nranks || c->p.rank != rank) : true)
    return GM_EINVAL;
  if (c->comm) return GM_OK;
  ncclUniqueId id;
  memcpy(&id, id128, sizeof id);
  HIPCHECK(hipSetDevice(c->cfg.device));
  NCCLCHECK(ncclCommInitRank(&c->comm, nranks, id, rank));
  // Every rank must run the same cluster: the collectives' sizes follow from n, the band width
  // (column shards) and the chunk count (row shards, GM_CHUNKS), and the replayed draws from the
  // seeds. One all-gather of a config signature; a rank that disagrees fails here (GM_EINVAL)
  // instead of hanging or corrupting an all-to-allv later.
  const gm_config &g = c->cfg;
  const int64_t sig[GM_SIG_WORDS] = {g.mode, g.n, c->s.band, c->p.V, c->p.nchunk, (int64_t)g.rd_seed, g.drop_pct,
                                     g.drop_from, g.drop_to, (int64_t)g.drop_seed, g.init_mode, g.init_t0,
                                     (int64_t)g.init_seed, (int64_t)g.view_seed, c->p_sharded, GM_ABI_VERSION,
                                     (int64_t)(c->p.xcap_frac * 1e6f)};
  int64_t *dsig = nullptr;
  HIPCHECK(hipMalloc(&dsig, sizeof(int64_t) * GM_SIG_WORDS * (nranks + 1)));
  std::vector<int64_t> all((size_t)GM_SIG_WORDS * nranks);
  int rc = GM_OK;
  if (hipMemcpyAsync(dsig, sig, sizeof sig, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
      ncclAllGather(dsig, dsig + GM_SIG_WORDS, GM_SIG_WORDS, ncclInt64, c->comm, c->stream) != ncclSuccess ||
      hipMemcpyAsync(all.data(), dsig + GM_SIG_WORDS, sizeof(int64_t) * all.size(), hipMemcpyDeviceToHost,
                     c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess) {
    snprintf(g_errbuf, sizeof g_errbuf, "gm_comm_init: config all-gather failed");
    rc = GM_ECOMM;
  }
  (void)hipFree(dsig);
  for (int r = 0; rc == GM_OK && r < nranks; r++)
    for (int k = 0; k < GM_SIG_WORDS; k++)
      if (all[(size_t)r * GM_SIG_WORDS + k] != sig[k]) {
        snprintf(g_errbuf, sizeof g_errbuf, "gm_comm_init: rank %d disagrees on config word %d (%lld vs %lld)", r,
                 k, (long long)all[(size_t)r * GM_SIG_WORDS + k], (long long)sig[k]);
        rc = GM_EINVAL;
        break;
      }
  if (rc != GM_OK) {
    (void)ncclCommDestroy(c->comm);
    c->comm = nullptr;
  }
  return rc;
}

extern "C" int gm_comm_info(gm_ctx *c, int32_t info[4]) {
  if (!c || !info) return GM_EINVAL;
  if (!c->comm) {
    info[0] = 0, info[1] = -1, info[2] = -1, info[3] = c->cfg.device;
    return GM_OK;
  }
  int cnt = 0, rk = 0, dev = 0;
  NCCLCHECK(ncclCommCount(c->comm, &cnt));
  NCCLCHECK(ncclCommUserRank(c->comm, &rk));
  NCCLCHECK(ncclCommCuDevice(c->comm, &dev));
  info[0] = cnt, info[1] = rk, info[2] = dev, info[3] = c->cfg.device;
  return GM_OK;
}

extern "C" int gm_shard_layout(gm_ctx *c, int32_t *c0, int32_t *w) {
  if (c && c0 && w && c->cfg.mode == GM_MODE_PARTIAL) {  // row shard: nodes [n0, n0 + nloc)
    *c0 = c->p.n0;
    *w = c->p.nloc;
    return GM_OK;
  }
  if (!c || !c0 || !w || c->cfg.mode != GM_MODE_SCALED) return GM_EINVAL;
  *c0 = c->s.c0;
  *w = c->s.w;
  return GM_OK;
}

static bool drop_tick(const gm_ctx *c, int t) {  // keyed loss applies to the lists sent at t - 1
  return c->cfg.drop_pct > 0 && t - 1 >= c->cfg.drop_from && t - 1 < c->cfg.drop_to;
}
static bool mc_on(const gm_ctx *c, int t) { return c->s.mc_sent && t < c->s.mc_tmax; }

static int shard_ready(gm_ctx *c) {
  if (!c || c->cfg.mode != GM_MODE_SCALED || !c->s.sharded) return GM_EINVAL;
  if (c->latched != GM_OK) return c->latched;
  if (c->t > GM_T_LIMIT) return GM_ERANGE;
  return GM_OK;
}

extern "C" int gm_shard_merge(gm_ctx *c) {
  TRY(shard_ready(c));
  TRY(before_tick_events(c));
  TRY(ramp_starters(c));
  const int t_send = c->t - 1;
  const bool drop = c->cfg.drop_pct > 0 && t_send >= c->cfg.drop_from && t_send < c->cfg.drop_to;
  HIPCHECK(hipMemsetAsync(c->s.xcnt, 0, xcnt_bytes(c->s), c->stream));
  hipEvent_t k0 = nullptr, k1 = nullptr;
  if (c->timing) TRY(timing_slot(c, &k0, &k1));
  HIPCHECK(gm_launch_tick(c->s, c->t, drop ? c->cfg.drop_pct : -1, c->stream, k0, k1, false));
  HIPCHECK(gm_launch_xrows(c->s, 0, c->n, c->stream));  // this shard's row totals for the all-gather
  // msgcount: this shard's fresh counts (its columns), SUM-allreduced before the draws
  if (mc_on(c, c->t)) HIPCHECK(gm_launch_msgcount(c->s, c->t, drop, 0, c->stream));
  return GM_OK;
}

extern "C" int gm_shard_draw(gm_ctx *c, int32_t round, int32_t D) {
  TRY(shard_ready(c));
  // round 0 covers the precomputed S2 outputs [0, 16), round q >= 1 outputs [16 + 64(q-1), 16 + 64q)
  if (round < 0 || D != (round == 0 ? GM_D_FIRST : GM_D_MORE)) return GM_EINVAL;
  HIPCHECK(gm_launch_draw(c->s, c->t, round, D, 0, c->stream));
  return GM_OK;
}

extern "C" int gm_shard_accept(gm_ctx *c, int32_t D, int32_t *npending) {
  TRY(shard_ready(c));
  if (D <= 0 || D > c->dmax || !npending) return GM_EINVAL;
  HIPCHECK(hipMemsetAsync(c->s.npending, 0, sizeof(int32_t), c->stream));
  HIPCHECK(gm_launch_accept(c->s, c->t, D, 0, 0, c->stream));
  HIPCHECK(hipMemcpyAsync(npending, c->s.npending, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHECK(hipStreamSynchronize(c->stream));
  return GM_OK;
}

extern "C" int gm_shard_end_tick(gm_ctx *c) {
  TRY(shard_ready(c));
  // msgcount: sent / received once the targets are final (after draw_settle when bounded
  // rounds left rows to the host-driven loop)
  if (!c->draw_check && mc_on(c, c->t)) HIPCHECK(gm_launch_msgcount(c->s, c->t, drop_tick(c, c->t), 1, c->stream));
  if (c->timing) {  // band-kernel events are in the timing ring (no host wait here)
    HIPCHECK(hipEventRecord(c->e1, c->stream));
    c->timed_ticks++;
  }
  c->t++;
  c->ticks_done++;
  c->undrained = true;
  return GM_OK;
}

__global__ void gm_max_into(int32_t *dst, const int32_t *src, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = max(dst[i], src[i]);
}
__global__ void gm_add_into(uint32_t *dst, const uint32_t *src, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] += src[i];
}

// In-process collectives between the G shard contexts of one device:
// what = 0 all-gathers xcnt, what = 1 MAX-allreduces status[0, n*D), what = 2 SUM-allreduces
// the msgcount fresh counts of this tick (and the kept entries on a loss tick).
extern "C" int gm_shard_loopback(gm_ctx **ctxs, int32_t G, int32_t what, int32_t D) {
  if (!ctxs || G < 2) return GM_EINVAL;
  for (int g = 0; g < G; g++) {
    TRY(shard_ready(ctxs[g]));
    if (ctxs[g]->s.shard_count != G || ctxs[g]->s.shard_rank != g || ctxs[g]->n != ctxs[0]->n) return GM_EINVAL;
    HIPCHECK(hipStreamSynchronize(ctxs[g]->stream));
  }
  const size_t n = (size_t)ctxs[0]->n;
  hipStream_t st = ctxs[0]->stream;
  if (what == 0) {
    const SState &s0 = ctxs[0]->s;
    for (int g = 1; g < G; g++)
      if (ctxs[g]->s.xlog != s0.xlog) return GM_EINVAL;
    for (int dst = 0; dst < G; dst++)
      for (int src = 0; src < G; src++)
        for (int ch = 0; ch < s0.xk && src != dst; ch++) {
          const size_t o = S_XC(s0, src, (size_t)ch << s0.xlog);
          HIPCHECK(hipMemcpyAsync(ctxs[dst]->s.xcnt + o, ctxs[src]->s.xcnt + o, sizeof(int32_t) * 2 * xchunk_rows(s0, ch),
                                  hipMemcpyDeviceToDevice, st));
        }
  } else if (what == 2) {  // msgcount: SUM of the shards' fresh counts (and kept entries on loss ticks)
    const int t = ctxs[0]->t;
    if (!mc_on(ctxs[0], t)) return GM_ESTATE;
    const bool dropped = drop_tick(ctxs[0], t);
    for (int k = 0; k < (dropped ? 2 : 1); k++) {
      auto buf = [&](int g) { return k == 0 ? ctxs[g]->s.mc_fresh + (size_t)(t & 1) * n : ctxs[g]->s.mc_rdrop; };
      for (int g = 1; g < G; g++) hipLaunchKernelGGL(gm_add_into, dim3(64), dim3(256), 0, st, buf(0), buf(g), n);
      for (int g = 1; g < G; g++) HIPCHECK(hipMemcpyAsync(buf(g), buf(0), sizeof(uint32_t) * n, hipMemcpyDeviceToDevice, st));
    }
  } else {
    if (D <= 0 || D > ctxs[0]->dmax) return GM_EINVAL;
    const size_t cnt = n * (size_t)D;
    for (int g = 1; g < G; g++)
      hipLaunchKernelGGL(gm_max_into, dim3(256), dim3(256), 0, st, ctxs[0]->s.status, ctxs[g]->s.status, cnt);
    for (int g = 1; g < G; g++)
      HIPCHECK(hipMemcpyAsync(ctxs[g]->s.status, ctxs[0]->s.status, sizeof(int32_t) * cnt, hipMemcpyDeviceToDevice, st));
  }
  HIPCHECK(hipGetLastError());
  HIPCHECK(hipStreamSynchronize(st));
  return GM_OK;
}

// One PIPELINED column-shard tick (tick_sharded's chunk order) of G shard contexts living on one
// device, the collectives done by device copies / MAX kernels on one stream: per exchange chunk the
// all-gather of the counts, every shard's round-0 draws of the chunk's rows, the MAX-reduce of their
// statuses, every shard's acceptance; then the bounded rounds 1, 2 with their MAX-reduces. Tests
// compare it with the fused kernel and with the phase-API loopback (gm_shard_loopback); tick_sharded
// runs the same per-chunk steps with RCCL on the comm stream, overlapped with later chunks' merges.
extern "C" int gm_shard_loopback_tick(gm_ctx **ctxs, int32_t G) {
  if (!ctxs || G < 2) return GM_EINVAL;
  for (int g = 0; g < G; g++) {
    TRY(shard_ready(ctxs[g]));
    const SState &sg = ctxs[g]->s;
    if (sg.shard_count != G || sg.shard_rank != g || ctxs[g]->n != ctxs[0]->n || ctxs[g]->t != ctxs[0]->t ||
        sg.xlog != ctxs[0]->s.xlog || sg.ramp || mc_on(ctxs[g], ctxs[g]->t))
      return GM_EINVAL;
    TRY(draw_settle(ctxs[g]));
    TRY(before_tick_events(ctxs[g]));
    HIPCHECK(hipStreamSynchronize(ctxs[g]->stream));
  }
  hipStream_t ls = ctxs[0]->stream;
  const int t = ctxs[0]->t, t_send = t - 1;
  const SState &s0 = ctxs[0]->s;
  for (int g = 0; g < G; g++) {
    gm_ctx *c = ctxs[g];
    SState &s = c->s;
    const bool drop = c->cfg.drop_pct > 0 && t_send >= c->cfg.drop_from && t_send < c->cfg.drop_to;
    HIPCHECK(gm_launch_tick_prologue(s, t, ls, true));  // as tick_sharded: no fills
    for (int ch = 0; ch < s.xk; ch++) {
      const int r0 = ch << s.xlog;
      HIPCHECK(gm_launch_band_rows(s, t, drop ? c->cfg.drop_pct : -1, r0, r0 + xchunk_rows(s, ch), ls));
    }
  }
  auto max_reduce = [&](auto buf_of, size_t off, size_t cnt) -> int {  // MAX over the shards, into every shard
    if (!cnt) return GM_OK;
    for (int g = 1; g < G; g++)
      hipLaunchKernelGGL(gm_max_into, dim3(256), dim3(256), 0, ls, buf_of(0) + off, buf_of(g) + off, cnt);
    for (int g = 1; g < G; g++)
      HIPCHECK(hipMemcpyAsync(buf_of(g) + off, buf_of(0) + off, sizeof(int32_t) * cnt, hipMemcpyDeviceToDevice, ls));
    return GM_OK;
  };
  for (int ch = 0; ch < s0.xk; ch++) {
    const int r0 = ch << s0.xlog, r1 = r0 + xchunk_rows(s0, ch);
    for (int g = 0; g < G; g++) HIPCHECK(gm_launch_xrows(ctxs[g]->s, r0, r1, ls));
    for (int dst = 0; dst < G; dst++)  // the chunk's all-gather
      for (int src = 0; src < G; src++)
        if (src != dst) {
          const size_t o = S_XC(s0, src, (size_t)r0);
          HIPCHECK(hipMemcpyAsync(ctxs[dst]->s.xcnt + o, ctxs[src]->s.xcnt + o, sizeof(int32_t) * 2 * (r1 - r0),
                                  hipMemcpyDeviceToDevice, ls));
        }
    for (int g = 0; g < G; g++) HIPCHECK(gm_launch_draw(ctxs[g]->s, t, 0, GM_D_FIRST, 0, ls, r0, r1));
    TRY(max_reduce([&](int g) { return ctxs[g]->s.status; }, (size_t)r0 * GM_D_FIRST, (size_t)(r1 - r0) * GM_D_FIRST));
    for (int g = 0; g < G; g++) HIPCHECK(gm_launch_accept(ctxs[g]->s, t, GM_D_FIRST, 0, 1, ls, r0, r1));
  }
  for (int l = 1; l <= 2; l++) {
    const int D = l == 1 ? GM_D_MORE : GM_D_LAST;
    for (int g = 0; g < G; g++) {
      HIPCHECK(gm_launch_plist_sort(ctxs[g]->s, l, ls));
      HIPCHECK(gm_launch_draw(ctxs[g]->s, t, l, D, l, ls));
    }
    TRY(max_reduce([&](int g) { return ctxs[g]->s.statusl[l]; }, 0, (size_t)s0.plist_cap[l] * D));
    for (int g = 0; g < G; g++) HIPCHECK(gm_launch_accept(ctxs[g]->s, t, D, l, l == 1 ? 2 : -1, ls));
  }
  HIPCHECK(hipGetLastError());
  // rows the bounded rounds could not take (a pending list overflowed, or a row still short after
  // round 2): the host-driven rounds of draw_settle, each row from its own next round, with the
  // MAX-reduce by device kernels -- every shard must count the same rows
  for (int round = 0;; round++) {
    std::vector<int32_t> left(G, 0);
    for (int g = 0; g < G; g++)
      HIPCHECK(hipMemcpyAsync(&left[g], ctxs[g]->s.npending, sizeof(int32_t), hipMemcpyDeviceToHost, ls));
    HIPCHECK(hipStreamSynchronize(ls));
    for (int g = 1; g < G; g++)
      if (left[g] != left[0]) {
        snprintf(g_errbuf, sizeof g_errbuf, "pipelined loopback tick: shards disagree on pending rows (%d vs %d)",
                 left[g], left[0]);
        return GM_ESTATE;
      }
    if (!left[0]) break;
    if (round >= GM_MAX_ROUNDS) return GM_ERANGE;
    for (int g = 0; g < G; g++) HIPCHECK(gm_launch_draw(ctxs[g]->s, t, 1, GM_D_MORE, 0, ls));
    TRY(max_reduce([&](int g) { return ctxs[g]->s.status; }, 0, (size_t)ctxs[0]->n * GM_D_MORE));
    for (int g = 0; g < G; g++) {
      HIPCHECK(hipMemsetAsync(ctxs[g]->s.npending, 0, sizeof(int32_t), ls));
      HIPCHECK(gm_launch_accept(ctxs[g]->s, t, GM_D_MORE, 0, 0, ls));
    }
  }
  for (int g = 0; g < G; g++) TRY(gm_shard_end_tick(ctxs[g]));
  return GM_OK;
}

// Host-collective hook: the phase exchange buffers of ONE shard context as plain host arrays, so
// that any host-side collective (gloo across processes: membership.sharded.host_tick) can stand
// in for RCCL / gm_shard_loopback. Layouts (n = cluster size, G = shard count):
//   what 0  export: this rank's per-row (present, numfailed) int32[n][2]; import: all G slots
//           int32[G][n][2] (the all-gather's result)
//   what 1  export / import: the resolved draws int32[n][D]; import the MAX over the ranks
//   what 2  (msgcount recording) export / import: uint32[n] fresh counts, plus uint32[n] kept
//           entries on keyed-loss ticks; import the SUM over the ranks
static int shard_buf(gm_ctx *c, int what, int D, std::vector<std::pair<void *, size_t>> &parts, bool import) {
  const size_t n = (size_t)c->n;
  SState &s = c->s;
  parts.clear();
  if (what == 0) {  // host layout [n][2] (export) / [G][n][2] (import); device chunk-major (S_XC)
    for (int g = import ? 0 : s.shard_rank; g < (import ? s.shard_count : s.shard_rank + 1); g++)
      for (int ch = 0; ch < s.xk; ch++)
        parts.push_back({s.xcnt + S_XC(s, g, (size_t)ch << s.xlog), sizeof(int32_t) * 2 * xchunk_rows(s, ch)});
    (void)n;
  } else if (what == 1) {
    if (D <= 0 || D > c->dmax) return GM_EINVAL;
    parts.push_back({s.status, sizeof(int32_t) * n * D});
  } else if (what == 2) {
    if (!mc_on(c, c->t)) return GM_ESTATE;
    parts.push_back({s.mc_fresh + (size_t)(c->t & 1) * n, sizeof(uint32_t) * n});
    if (drop_tick(c, c->t)) parts.push_back({s.mc_rdrop, sizeof(uint32_t) * n});
  } else {
    return GM_EINVAL;
  }
  return GM_OK;
}

extern "C" int gm_shard_export(gm_ctx *c, int32_t what, int32_t D, void *out, size_t cap, size_t *bytes) {
  if (!c || !bytes) return GM_EINVAL;
  TRY(shard_ready(c));
  std::vector<std::pair<void *, size_t>> parts;
  TRY(shard_buf(c, what, D, parts, false));
  size_t tot = 0;
  for (auto &p : parts) tot += p.second;
  *bytes = tot;
  if (!out) return GM_OK;
  if (cap < tot) return GM_ERANGE;
  HIPCHECK(hipStreamSynchronize(c->stream));
  size_t off = 0;
  for (auto &p : parts) {
    HIPCHECK(ctx_memcpy(c, (uint8_t *)out + off, p.first, p.second, hipMemcpyDeviceToHost));
    off += p.second;
  }
  return GM_OK;
}

extern "C" int gm_shard_import(gm_ctx *c, int32_t what, int32_t D, const void *in, size_t bytes) {
  if (!c || !in) return GM_EINVAL;
  TRY(shard_ready(c));
  std::vector<std::pair<void *, size_t>> parts;
  TRY(shard_buf(c, what, D, parts, true));
  size_t tot = 0;
  for (auto &p : parts) tot += p.second;
  if (bytes != tot) return GM_EINVAL;
  HIPCHECK(hipStreamSynchronize(c->stream));
  size_t off = 0;
  for (auto &p : parts) {
    HIPCHECK(ctx_memcpy(c, p.first, (const uint8_t *)in + off, p.second, hipMemcpyHostToDevice));
    off += p.second;
  }
  return GM_OK;
}

// Diagnostics: one column shard alone on a device (no RCCL, no peers): the all-gather of
// per-row counts mirrors this shard's counts into every peer slot and the draw kernel
// resolves draws landing in peer columns as fresh column ix (SState.stub) -- a symmetric
// stand-in with the real kernels at the true shard shape (scripts/shard_profile.py --sb).
extern "C" int gm_shard_stub(gm_ctx *c, int32_t on) {
  if (!c || c->cfg.mode != GM_MODE_SCALED || !c->s.sharded) return GM_EINVAL;
  c->s.stub = on ? 1 : 0;
  return GM_OK;
}

__global__ void gm_xc_mirror(int32_t *chunk, int rank, int G, size_t words) {  // stub all-gather
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < words; i += (size_t)gridDim.x * blockDim.x) {
    const int32_t v = chunk[(size_t)rank * words + i];
    for (int g = 0; g < G; g++)
      if (g != rank) chunk[(size_t)g * words + i] = v;
  }
}

// the all-gather of this shard's per-row (present, numfailed) for exchange chunk ch (stub: mirrored
// into every peer slot), on stream st
static int xcnt_allgather(gm_ctx *c, int ch, hipStream_t st) {
  SState &s = c->s;
  const size_t R = (size_t)1 << s.xlog, r0 = (size_t)ch << s.xlog;
  int32_t *own = s.xcnt + S_XC(s, s.shard_rank, r0);
  if (s.stub) {  // one kernel mirrors the chunk's slot into every peer slot (the all-gather's local cost)
    hipLaunchKernelGGL(gm_xc_mirror, dim3(256), dim3(256), 0, st, s.xcnt + S_XC(s, 0, r0), s.shard_rank,
                       s.shard_count, (size_t)2 << s.xlog);
    HIPCHECK(hipGetLastError());
    return GM_OK;
  }
  // chunk-major: the chunk's G slots are contiguous, rank g's at g * R rows -- in place
  NCCLCHECK(ncclAllGather(own, s.xcnt + S_XC(s, 0, r0), R * 2, ncclInt32, c->comm, st));
  return GM_OK;
}

// Bounded rounds 1 and 2 of tick t over the rows round 0 left pending: their sorted list (identical on
// every rank) takes the next 64 S2 outputs, then up to 256 rows the next 256; a row still short sets
// GM_ERR_DRAWS. Rows the rounds could not take are counted in npending (draw_settle finishes them with
// host-driven rounds).
static int run_bounded(gm_ctx *c, int t) {
  SState &s = c->s;
  for (int l = 1; l <= 2; l++) {
    const int D = l == 1 ? GM_D_MORE : GM_D_LAST;
    HIPCHECK(gm_launch_plist_sort(s, l, c->stream));
    HIPCHECK(gm_launch_draw(s, t, l, D, l, c->stream));
    if (!s.stub)
      NCCLCHECK(ncclAllReduce(s.statusl[l], s.statusl[l], (size_t)s.plist_cap[l] * D, ncclInt32, ncclMax, c->comm,
                              c->stream));
    HIPCHECK(gm_launch_accept(s, t, D, l, l == 1 ? 2 : -1, c->stream));
  }
  if (getenv("GM_DEBUG_ROUNDS")) {  // diagnostics: rows left after round 0, error flags
    uint32_t pc1 = 0, pc2 = 0, e = 0;
    HIPCHECK(hipMemcpyAsync(&pc1, s.plist_cnt[1], sizeof pc1, hipMemcpyDeviceToHost, c->stream));
    HIPCHECK(hipMemcpyAsync(&pc2, s.plist_cnt[2], sizeof pc2, hipMemcpyDeviceToHost, c->stream));
    HIPCHECK(hipMemcpyAsync(&e, s.err, sizeof e, hipMemcpyDeviceToHost, c->stream));
    HIPCHECK(hipStreamSynchronize(c->stream));
    fprintf(stderr, "[gm] t=%d rows pending after round 0: %u (cap %d), after round 1: %u (cap %d), err 0x%x\n", t,
            pc1, s.plist_cap[1], pc2, s.plist_cap[2], e);
  }
  return GM_OK;
}

// The end of a sharded tick's device work: the counts of rows still drawing go to the host without
// a wait (draw_settle reads them before anything uses the tick). deferred (the pipelined tick):
// bounded rounds 1, 2 have not run; draw_settle runs them only when round 0 left rows pending -- in
// the steady state it leaves none, so a tick pays neither their six launches nor their two
// MAX-allreduces. Every rank takes the same decision (the acceptance is identical on all ranks), so
// the ranks' RCCL calls stay in step.
// ds: the stream whose work decides the counts (the pipelined tick's comm stream: the copy follows
// its last acceptance directly instead of behind a cross-stream join)
static int end_draws(gm_ctx *c, bool deferred, hipStream_t ds = nullptr) {
  SState &s = c->s;
  if (!deferred) TRY(run_bounded(c, c->t));
  if (!ds) ds = c->stream;
  HIPCHECK(hipMemcpyAsync(c->draw_left_h, s.npending, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, ds));
  HIPCHECK(hipEventRecord(c->draw_ev, ds));
  c->draw_rounds = deferred;
  c->t--;  // gm_tick advances globaltime
  c->draw_check = true;  // before end_tick: the msgcount phase waits for draw_settle
  TRY(gm_shard_end_tick(c));
  c->ticks_done--;  // gm_tick counts it
  return GM_OK;
}

// The column-shard tick, pipelined over the exchange's row chunks (north_star: the exchange
// overlapped with the local merge on a second stream). The compute stream runs the band kernels
// chunk after chunk; as soon as chunk ch's are done (event), the comm stream all-gathers the
// chunk's per-row counts, draws round 0 of its rows (every rank replays every row's first 16 S2
// outputs and resolves the draws landing in its columns), MAX-allreduces their statuses and runs
// the acceptance -- while the band kernels of chunks ch+1.. still run. A row's draws need only
// its own post-sweep row (in chunk ch) and the other ranks' counts of that row; the acceptance
// appends to the inboxes of tick t+1 (the other parity), which no band kernel of tick t reads.
// Then the bounded rounds 1, 2 on the compute stream. Ticks that record msgcount (their
// fresh-count all-reduce precedes every draw), the join ramp and the host-driven draw loop (mass
// failure, heavy loss) take the same steps unchunked.
static int tick_sharded(gm_ctx *c) {
  if (!c->comm && !c->s.stub) return GM_EUNSUPPORTED;  // multi-GPU ticks need gm_comm_init (or the phase API + loopback)
  SState &s = c->s;
  const size_t n = (size_t)c->n;
  const int64_t nfailed = c->nfailed;
  // mass failure or heavy loss leaves many entries stale, so rows need many draws: the
  // host-driven unbounded loop below (also GM_SHARD_SYNC=1)
  const bool sync = c->shard_sync == 1 || (c->shard_sync < 0 && (c->cfg.drop_pct >= 30 || 10 * nfailed > (int64_t)n));
  const bool pipe = !sync && !mc_on(c, c->t) && !s.ramp && !(getenv("GM_SHARD_PIPE") && !atoi(getenv("GM_SHARD_PIPE")));
  if (pipe) {
    TRY(shard_ready(c));
    TRY(before_tick_events(c));
    const int t = c->t, t_send = t - 1;
    const bool drop = c->cfg.drop_pct > 0 && t_send >= c->cfg.drop_from && t_send < c->cfg.drop_to;
    // no fills: gm_s_xrows writes this rank's xcnt slots whole (no join ramp here) and gm_s_mtgen
    // zeroes the draw rounds' counters
    HIPCHECK(gm_launch_tick_prologue(s, t, c->stream, true));
    hipEvent_t k0 = nullptr, k1 = nullptr;
    if (c->timing) TRY(timing_slot(c, &k0, &k1));
    if (k0) HIPCHECK(hipEventRecord(k0, c->stream));
    for (int ch = 0; ch < s.xk; ch++) {
      const int r0 = ch << s.xlog;
      HIPCHECK(gm_launch_band_rows(s, t, drop ? c->cfg.drop_pct : -1, r0, r0 + xchunk_rows(s, ch), c->stream));
      const int zr = c->diag_zero_row;
      if (zr >= r0 && zr < r0 + xchunk_rows(s, ch) && zr < c->n)
        for (int b = 0; b < s.nb; b++)
          HIPCHECK(hipMemsetAsync(s.table + ((size_t)b * n + zr) * s.band, 0, s.band, c->stream));
      HIPCHECK(hipEventRecord(c->p_chev[ch], c->stream));
    }
    if (k1) HIPCHECK(hipEventRecord(k1, c->stream));
    hipStream_t cs = c->p_comm;
    for (int ch = 0; ch < s.xk; ch++) {
      const int r0 = ch << s.xlog, r1 = r0 + xchunk_rows(s, ch);
      HIPCHECK(hipStreamWaitEvent(cs, c->p_chev[ch], 0));
      HIPCHECK(gm_launch_xrows(s, r0, r1, cs));
      TRY(xcnt_allgather(c, ch, cs));
      HIPCHECK(gm_launch_draw(s, t, 0, GM_D_FIRST, 0, cs, r0, r1));
      if (!s.stub)
        NCCLCHECK(ncclAllReduce(s.status + (size_t)r0 * GM_D_FIRST, s.status + (size_t)r0 * GM_D_FIRST,
                                (size_t)(r1 - r0) * GM_D_FIRST, ncclInt32, ncclMax, c->comm, cs));
      HIPCHECK(gm_launch_accept(s, t, GM_D_FIRST, 0, 1, cs, r0, r1));
    }
    HIPCHECK(hipEventRecord(c->p_done, cs));
    HIPCHECK(hipStreamWaitEvent(c->stream, c->p_done, 0));
    return end_draws(c, true, cs);
  }
  TRY(gm_shard_merge(c));
  for (int ch = 0; ch < s.xk; ch++) TRY(xcnt_allgather(c, ch, c->stream));
  if (!s.stub && mc_on(c, c->t)) {  // msgcount: whole-row fresh counts (and kept entries on loss ticks)
    NCCLCHECK(ncclAllReduce(s.mc_fresh + (size_t)(c->t & 1) * n, s.mc_fresh + (size_t)(c->t & 1) * n, n, ncclUint32,
                            ncclSum, c->comm, c->stream));
    if (drop_tick(c, c->t))
      NCCLCHECK(ncclAllReduce(s.mc_rdrop, s.mc_rdrop, n, ncclUint32, ncclSum, c->comm, c->stream));
  }
  if (!sync) {
    // bounded rounds, stream-ordered (no host round trip): round 0 = every row's first 16
    // S2 outputs; rows left pending go to a list (sorted: identical on every rank) that
    // round 1 serves with the next 64; a row still short after that sets GM_ERR_DRAWS
    for (int l = 1; l <= 2; l++) HIPCHECK(hipMemsetAsync(s.plist_cnt[l], 0, sizeof(uint32_t), c->stream));
    HIPCHECK(hipMemsetAsync(s.npending, 0, sizeof(int32_t), c->stream));
    HIPCHECK(gm_launch_draw(s, c->t, 0, GM_D_FIRST, 0, c->stream));
    if (!s.stub)
      NCCLCHECK(ncclAllReduce(s.status, s.status, n * GM_D_FIRST, ncclInt32, ncclMax, c->comm, c->stream));
    HIPCHECK(gm_launch_accept(s, c->t, GM_D_FIRST, 0, 1, c->stream));
    return end_draws(c, false);
  }
  int round = 0, D = GM_D_FIRST;
  for (;;) {
    TRY(gm_shard_draw(c, round, D));
    if (!s.stub)
      NCCLCHECK(ncclAllReduce(s.status, s.status, n * D, ncclInt32, ncclMax, c->comm, c->stream));
    int32_t pend = 0;
    TRY(gm_shard_accept(c, D, &pend));
    if (getenv("GM_DEBUG_ROUNDS")) fprintf(stderr, "[gm] t=%d round %d: %d rows still drawing\n", c->t, round, pend);
    if (pend == 0) break;
    if (++round > GM_MAX_ROUNDS) {  // a row that never finds its targets: same guard as gm_s_pick
      uint32_t e = GM_ERR_DRAWS;
      HIPCHECK(ctx_memcpy(c, s.err, &e, sizeof e, hipMemcpyHostToDevice));
      c->latched = GM_ERANGE;
      return c->latched;
    }
    D = GM_D_MORE;
  }
  c->t--;  // gm_tick advances globaltime
  TRY(gm_shard_end_tick(c));
  c->ticks_done--;  // gm_tick counts it
  return GM_OK;
}

// The rows the last sharded tick's bounded rounds left (a full pending list, or still short of
// targets after 336 S2 outputs): host-driven rounds, each row continuing from its own next round
// (gm_s_draw with round >= 1 reads it from pending[r]), until every row has its targets --
// tick t = c->t - 1 completes before anything reads it or the next tick starts.
static int draw_settle(gm_ctx *c) {
  if (!c->draw_check) return c->latched;
  c->draw_check = false;
  // the next tick's launches wait on these two counts: spin on the event rather than block (the
  // wait costs 2-18 us of GPU idle per pipelined tick, profiles/r06/stub_tail/). No work of the
  // next tick is enqueued before it: its S2 precompute zeroes the counts the copy reads
  hipError_t q;
  while ((q = hipEventQuery(c->draw_ev)) == hipErrorNotReady) {
  }
  HIPCHECK(q);
  int32_t pend = c->draw_left_h[0];
  const int t = c->t - 1;
  const size_t n = (size_t)c->n;
  if (c->draw_rounds) {  // the pipelined tick's bounded rounds, only if round 0 left rows pending
    c->draw_rounds = false;
    if (c->draw_left_h[1] > 0) {
      TRY(run_bounded(c, t));
      HIPCHECK(hipMemcpyAsync(&pend, c->s.npending, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
      HIPCHECK(hipStreamSynchronize(c->stream));
    }
  }
  for (int round = 0; pend > 0; round++) {
    if (getenv("GM_DEBUG_ROUNDS")) fprintf(stderr, "[gm] t=%d settle round %d: %d rows still drawing\n", t, round, pend);
    if (round >= GM_MAX_ROUNDS) {
      uint32_t e = GM_ERR_DRAWS;
      HIPCHECK(ctx_memcpy(c, c->s.err, &e, sizeof e, hipMemcpyHostToDevice));
      c->latched = GM_ERANGE;
      return c->latched;
    }
    HIPCHECK(gm_launch_draw(c->s, t, 1, GM_D_MORE, 0, c->stream));
    if (!c->s.stub)
      NCCLCHECK(ncclAllReduce(c->s.status, c->s.status, n * GM_D_MORE, ncclInt32, ncclMax, c->comm, c->stream));
    HIPCHECK(hipMemsetAsync(c->s.npending, 0, sizeof(int32_t), c->stream));
    HIPCHECK(gm_launch_accept(c->s, t, GM_D_MORE, 0, 0, c->stream));
    HIPCHECK(hipMemcpyAsync(&pend, c->s.npending, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHECK(hipStreamSynchronize(c->stream));
  }
  if (mc_on(c, t)) HIPCHECK(gm_launch_msgcount(c->s, t, drop_tick(c, t), 1, c->stream));
  return c->latched;
}

// ------------------------------------------------------------ PARTIAL row shards
// After chunk c's local kernels of tick t, gm_p_pack (on the comm stream) builds the records the
// chunk's nodes address to each other shard q -- from their targets and their final lists of the
// tick, no record written by the node kernels -- packed to the front of block (q, r0_c), whose
// capacity every rank knows (xcap). The exchange sends the blocks with two all-to-allv -- headers,
// then lists (wire format) into recv_list[t&1], where tick t+1 reads its senders' lists -- and
// gm_p_unpack appends each received record whose stamp is t to its targets' inboxes (rows of a block
// past its records keep older stamps), while later chunks compute. No host round trip.
// Capacity of a packed block (gm_p_pack): the records one chunk of `rows` senders addresses to
// shard q. A sender's five targets are drawn from its view; with a fraction f_q of the view's
// entries on shard q it addresses q with probability 1 - (1 - f_q)^5, so the block's record count is
// a sum of Bernoullis whose mean is at most rows * (1 - (1 - E f_q)^5) (the map is concave) and
// whose variance is at most the binomial's. E f_q: views follow the live nodes once the crashed
// ones are swept out, and hold the static shares before -- so f_q = max(n_q / n, live_q / live) (a
// crashed shard keeps its static share; ADVICE r4: a contiguous half-cluster crash, the
// reference's multifailure schedule, Application.cpp:189-192, leaves the survivors addressing each
// surviving shard with ~76 % at G = 8, past the static 49 %). The block holds the mean + 8 sigma +
// 64 (at most the slots); every rank derives the same capacities from the same crash set, and an
// overflow fails loudly (GM_ERR_XCHG).
static size_t xcap(const gm_ctx *c, size_t rows, int q) {
  const PState &p = c->p;
  if (p.xcap_frac > 0.f) return std::min(rows, (size_t)std::ceil((double)rows * p.xcap_frac));
  const double pq = c->p_xq[q];
  const double m = (double)rows * pq + 8.0 * std::sqrt((double)rows * pq * (1.0 - pq)) + 64.0;
  return std::min(rows, (size_t)std::ceil(m));
}
struct XChunk {  // the block layout of chunk ch (rows of shard g in chunk ch: [nloc_g ch / K, nloc_g (ch+1) / K))
  std::vector<size_t> sc, sd, rc, rd;  // send / receive record counts (block capacities) and row offsets per shard
  size_t rbase = 0, rrows = 0;         // this chunk's first received row, rows received
};
static XChunk xchunk(const gm_ctx *c, int ch) {
  const PState &p = c->p;
  const int G = p.G, K = p.nchunk;
  auto nloc_of = [&](int g) { return (int64_t)p.n * (g + 1) / G - (int64_t)p.n * g / G; };
  auto rows = [&](int g, int cc) { return (size_t)(nloc_of(g) * (cc + 1) / K - nloc_of(g) * cc / K); };
  XChunk x;
  x.sc.assign(G, 0); x.sd.assign(G, 0); x.rc.assign(G, 0); x.rd.assign(G, 0);
  for (int cc = 0; cc < ch; cc++)
    for (int g = 0; g < G; g++)
      if (g != p.rank) x.rbase += xcap(c, rows(g, cc), p.rank);
  const size_t r0 = (size_t)((int64_t)p.nloc * ch / K);
  size_t off = x.rbase;
  for (int q = 0; q < G; q++) {
    if (q == p.rank) continue;
    x.sc[q] = xcap(c, rows(p.rank, ch), q);
    x.sd[q] = (size_t)q * p.nloc + r0;  // the packed block (q, r0) of pk_hdr / pk_list
    x.rc[q] = xcap(c, rows(q, ch), p.rank);
    x.rd[q] = off;
    off += x.rc[q];
  }
  x.rrows = off - x.rbase;
  return x;
}

// the address probabilities per shard from the crash set (every rank holds the whole set), and the
// outgoing block capacities per (chunk, peer) on the device (gm_p_pack reads them)
static int partial_caps(gm_ctx *c) {
  const PState &p = c->p;
  const int G = p.G;
  std::vector<int64_t> live(G, 0);
  int64_t tot = 0;
  for (int g = 0; g < G; g++) {
    const int a = (int)((int64_t)p.n * g / G), b = (int)((int64_t)p.n * (g + 1) / G);
    for (int i = a; i < b; i++) live[g] += c->failed_h[i] ? 0 : 1;
    tot += live[g];
  }
  uint64_t h = 0x9E3779B97F4A7C15ull;  // the crash set every rank must hold (the capacities follow from it)
  for (int i = 0; i < p.n; i++)
    if (c->failed_h[i]) h = (h ^ (uint64_t)(uint32_t)i) * 0x100000001B3ull + 0x632BE59BD9B4E019ull;
  c->p_crash_hash = h;
  c->p_crash_check = true;
  c->p_xq.assign(G, 0.0);
  for (int g = 0; g < G; g++) {
    const double fs = (double)((int64_t)p.n * (g + 1) / G - (int64_t)p.n * g / G) / p.n;
    const double fl = tot > 0 ? (double)live[g] / tot : 0.0;
    c->p_xq[g] = 1.0 - std::pow(1.0 - std::max(fs, fl), (double)GM_FANOUT);
  }
  std::vector<int32_t> cap((size_t)p.nchunk * G, 0);
  for (int ch = 0; ch < p.nchunk; ch++) {
    const XChunk x = xchunk(c, ch);
    for (int q = 0; q < G; q++) cap[(size_t)ch * G + q] = (int32_t)x.sc[q];
  }
  HIPCHECK(ctx_memcpy(c, p.pk_cap, cap.data(), sizeof(int32_t) * cap.size(), hipMemcpyHostToDevice));
  return GM_OK;
}

static int partial_exchange_chunk(gm_ctx *c, int ch, int64_t *roff) {
  PState &p = c->p;
  const int G = p.G, V = p.V;
  hipStream_t cs = c->p_comm;
  const XChunk x = xchunk(c, ch);
  std::vector<size_t> hs(G), hsd(G), hr(G), hrd(G), ls(G), lsd(G), lr(G), lrd(G);
  for (int q = 0; q < G; q++) {
    hs[q] = x.sc[q] * 8;
    hsd[q] = x.sd[q] * 8;
    hr[q] = x.rc[q] * 8;
    hrd[q] = x.rd[q] * 8;
    ls[q] = x.sc[q] * V;
    lsd[q] = x.sd[q] * V;
    lr[q] = x.rc[q] * V;
    lrd[q] = x.rd[q] * V;
  }
  if (x.rbase + x.rrows > (size_t)(p.n - p.nloc)) return GM_ESTATE;
  if (ch == 0) HIPCHECK(hipMemsetAsync(p.pk_cnt, 0, sizeof(int32_t) * p.nchunk * G, cs));
  HIPCHECK(gm_launch_partial_pack(p, c->t, ch, cs));
  NCCLCHECK(ncclAllToAllv(p.pk_hdr, hs.data(), hsd.data(), p.recv_hdr, hr.data(), hrd.data(), ncclInt32, c->comm, cs));
  NCCLCHECK(ncclAllToAllv(p.pk_list, ls.data(), lsd.data(), p.recv_list[c->t & 1], lr.data(), lrd.data(), ncclUint32,
                          c->comm, cs));
  HIPCHECK(gm_launch_partial_unpack(p, c->t, (int)x.rbase, (int)x.rrows, cs));
  *roff = (int64_t)(x.rbase + x.rrows);
  return GM_OK;
}

// One PARTIAL tick of G row-shard contexts living on one device (tests): the local
// kernels of every shard, the exchange partial_exchange_chunk does by device copies (same layout),
// the unpack, and the globaltime advance gm_tick does.
extern "C" int gm_partial_loopback_tick(gm_ctx **ctxs, int32_t G) {
  if (!ctxs || G < 2) return GM_EINVAL;
  for (int g = 0; g < G; g++) {
    gm_ctx *c = ctxs[g];
    if (!c || c->cfg.mode != GM_MODE_PARTIAL || c->p.G != G || c->p.rank != g || c->t != ctxs[0]->t ||
        c->n != ctxs[0]->n || c->p.V != ctxs[0]->p.V)
      return GM_EINVAL;
    if (c->latched != GM_OK) return c->latched;
  }
  for (int g = 0; g < G; g++) TRY(before_tick_events(ctxs[g]));
  // every shard's kernels on ONE stream, shard after shard: the sum of the shards' own costs (8
  // concurrent streams on one device starve each other's small worklist kernels; on a node every
  // shard has its GPU to itself)
  for (int g = 0; g < G; g++) HIPCHECK(hipStreamSynchronize(ctxs[g]->stream));
  hipStream_t ls = ctxs[0]->stream;
  for (int g = 0; g < G; g++) {
    gm_ctx *c = ctxs[g];
    const int t_send = c->t - 1;
    const bool drop = c->cfg.drop_pct > 0 && t_send >= c->cfg.drop_from && t_send < c->cfg.drop_to;
    PState st = c->p;
    st.drop_pct = drop ? c->cfg.drop_pct : -1;
    HIPCHECK(gm_launch_partial_tick(st, c->t, c->p_mtraw, ls, nullptr, nullptr));
  }
  const int K = ctxs[0]->p.nchunk;
  for (int g = 0; g < G; g++)
    if (ctxs[g]->p.nchunk != K) return GM_EINVAL;
  // the blocks partial_exchange_chunk's all-to-allv moves, by device copies
  const int V = ctxs[0]->p.V;
  std::vector<size_t> roff(G, 0);
  for (int g = 0; g < G; g++) {  // every shard packs its records into its outgoing blocks (as on the comm stream)
    PState &pg = ctxs[g]->p;
    HIPCHECK(hipMemsetAsync(pg.pk_cnt, 0, sizeof(int32_t) * K * G, ls));
    for (int ch = 0; ch < K; ch++) HIPCHECK(gm_launch_partial_pack(pg, ctxs[g]->t, ch, ls));
  }
  for (int ch = 0; ch < K; ch++)
    for (int q = 0; q < G; q++) {
      PState &dq = ctxs[q]->p;
      hipStream_t st = ls;
      const XChunk xq = xchunk(ctxs[q], ch);
      for (int g = 0; g < G; g++) {
        if (g == q || !xq.rc[g]) continue;
        const XChunk xg = xchunk(ctxs[g], ch);
        const PState &sg = ctxs[g]->p;
        if (xg.sc[q] != xq.rc[g]) return GM_ESTATE;
        HIPCHECK(hipMemcpyAsync(dq.recv_hdr + xq.rd[g] * 8, sg.pk_hdr + xg.sd[q] * 8, sizeof(int32_t) * 8 * xq.rc[g],
                                hipMemcpyDeviceToDevice, st));
        HIPCHECK(hipMemcpyAsync(dq.recv_list[ctxs[q]->t & 1] + xq.rd[g] * V, sg.pk_list + xg.sd[q] * V,
                                sizeof(uint32_t) * V * xq.rc[g], hipMemcpyDeviceToDevice, st));
      }
      HIPCHECK(gm_launch_partial_unpack(dq, ctxs[q]->t, (int)xq.rbase, (int)xq.rrows, st));
      roff[q] = xq.rbase + xq.rrows;
    }
  for (int q = 0; q < G; q++) ctxs[q]->p_recv_last = (int64_t)roff[q];
  HIPCHECK(hipStreamSynchronize(ls));
  for (int g = 0; g < G; g++) {
    TRY(check_err(ctxs[g]));
    ctxs[g]->t++;
    ctxs[g]->ticks_done++;
    ctxs[g]->undrained = true;
  }
  return GM_OK;
}

extern "C" int gm_shard_exchange_bytes(gm_ctx *c, int64_t *bytes) {
  if (!c || !bytes) return GM_EINVAL;
  *bytes = 0;
  if (c->cfg.mode == GM_MODE_PARTIAL)  // record slots received in the last tick: 32 B header + the V-entry list
    *bytes = c->p_recv_last * (int64_t)(32 + 4 * c->p.V);
  return GM_OK;
}
