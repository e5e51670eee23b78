// gm_faithful.hip -- FAITHFUL-mode tick kernels (the reference's own regime:
// N <= 1000, EmulNet buffer cap 30000, per-entry messages, glibc-rand drops).
//
// One Application::mp1Run tick (Application.cpp:121-164) = three launches:
//   gm_f_recv   recv phase: EmulNet::ENrecv for receivers ascending
//               (EmulNet.cpp:144-177). One workgroup walks the receivers in
//               order; for each it matches the buffer in parallel, emits the
//               matches in descending buffer index (the order the reference's
//               backward scan dequeues them) and applies the swap-with-last
//               compaction in closed form: the i-th hole from the top is
//               filled from position B-i, following the chain through holes
//               that were themselves refilled earlier in the scan.
//   gm_f_node   node phase: nodeStart / nodeLoop for every node in parallel
//               (one workgroup per node; MP1Node.cpp:73-163,182-495). The
//               queue merge is commutative on the table (max heartbeat); the
//               order-dependent parts -- joined-event order and newNodes
//               order -- come from first-occurrence positions in the queue.
//               Sweep, self bump (incl. the updateMyPos `&&` quirk) and the
//               mt19937 + Lemire gossip-target draw run per node.
//   gm_f_send   EmulNet::ENsend for every send of the tick (EmulNet.cpp:87-118):
//               sends are ordered node-descending (the node-phase order), each
//               consumes the next glibc rand() draw of the S1 stream; the
//               30000 cap is a prefix count over the not-drop-drawn sends.
#include "gm_device.h"
#include "gm_abi.h"
#include "gm_faithful.h"

#define F_RECV_THREADS 1024
#define F_NODE_THREADS 256
#define F_SEND_THREADS 1024

__device__ __forceinline__ uint32_t f_strkey(int32_t id) {
  // strcmp over the 6 address bytes {id LE, port 0} compares up to the first
  // NUL byte (EmulNet.cpp:154): keep the bytes before the first zero byte.
  uint32_t u = (uint32_t)id, key = 0;
  for (int b = 0; b < 4; b++) {
    uint32_t byte = (u >> (8 * b)) & 0xFFu;
    if (byte == 0) break;
    key |= byte << (8 * b);
  }
  return key;
}

// ---------------------------------------------------------------- recv phase
__global__ __launch_bounds__(F_RECV_THREADS) void gm_f_recv(FState s, int t) {
  __shared__ int s_tmp[32];
  FMsg *buf = s.buf;
  int32_t *key = s.keys;  // strcmp key of every element's destination, moved with the element
  int B = *s.bufsize;
  for (int j = threadIdx.x; j < B; j += F_RECV_THREADS) key[j] = (int32_t)f_strkey(buf[j].to);
  __syncthreads();
  int qbase = 0;
  for (int i = 0; i < s.n; i++) {
    if (threadIdx.x == 0) { s.q_off[i] = qbase; s.q_cnt[i] = 0; }
    if (!(t > s.start[i] && !s.failed[i])) continue;  // Application.cpp:130
    const int32_t me = (int32_t)f_strkey(i + 1);
    const int L = (B + F_RECV_THREADS - 1) / F_RECV_THREADS;
    const int lo = min(B, (int)threadIdx.x * L), hi = min(B, lo + L);
    int c = 0;
    for (int j = lo; j < hi; j++) c += key[j] == me;
    int k;
    int before = gm_block_scan(c, s_tmp, &k);  // matches at index < lo
    if (k == 0) continue;
    const int Bn = B - k;
    // deliver in descending buffer index; tag the matches that sit in the
    // vacated tail [Bn, B) with their 1-based descending rank
    for (int j = max(lo, Bn); j < hi; j++) s.holepos[j - Bn] = 0;
    __syncthreads();
    if (c) {
      int r = before;
      for (int j = lo; j < hi; j++) {
        if (key[j] == me) {
          s.q[qbase + (k - 1 - r)] = buf[j];
          if (j >= Bn) s.holepos[j - Bn] = k - r;
          r++;
        }
      }
    }
    __syncthreads();
    // swap-with-last, closed form: the i-th hole (descending) receives what sits
    // at position B-i when it is processed; if B-i is itself an earlier hole h_m,
    // that is what h_m received from B-m -- follow the chain to an original element
    if (c && lo < Bn) {
      int r = before;
      for (int j = lo; j < min(hi, Bn); j++) {
        if (key[j] == me) {
          int x = B - (k - r);
          int guard = 0;
          while (s.holepos[x - Bn] > 0 && ++guard <= k) x = B - s.holepos[x - Bn];
          buf[j] = buf[x];  // x >= Bn: never overwritten in this pass
          key[j] = key[x];
          r++;
        }
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      s.q_cnt[i] = k;
      s.recv[(size_t)(i + 1) * s.tmax + t] += k;  // recv_msgs[dst][time] (EmulNet.cpp:172)
    }
    qbase += k;
    B = Bn;
  }
  if (threadIdx.x == 0) *s.bufsize = B;
}

// ---------------------------------------------------------------- node phase
__device__ void f_emit(FState &s, int t, int i, int seq, int kind, int subject) {
  unsigned long long slot = atomicAdd(s.ev_count, 1ull);
  if (slot < (unsigned long long)s.ev_cap) {
    FEvent e;
    e.t = t;
    e.logger = i;
    e.kind = kind;
    e.subject = subject;
    e.seq = seq;
    s.ev[slot] = e;
  } else {
    atomicOr(s.err, GM_ERR_EVENTS);
  }
}

__global__ __launch_bounds__(F_NODE_THREADS) void gm_f_node(FState s, int t) {
  extern __shared__ __align__(16) unsigned char f_smem[];
  const int i = blockIdx.x, tid = threadIdx.x;
  const int np = s.np;  // padded row width (multiple of 64)
  const int nw = np >> 6;
  int *s_first = (int *)f_smem;                       // [np]
  int *s_maxkey = s_first + np;                       // [np]
  uint64_t *s_pres = (uint64_t *)(s_maxkey + np);     // [nw]
  uint64_t *s_fresh = s_pres + nw;                    // [nw]
  uint64_t *s_rem = s_fresh + nw;                     // [nw]
  uint32_t *s_pre = (uint32_t *)(s_rem + nw);         // [nw]
  uint32_t *s_mt = s_pre + nw;                        // [624]
  int *s_tmp = (int *)(s_mt + 624);                   // [32]
  int *s_misc = s_tmp + 32;                           // [16]
  uint32_t *row = s.table + (size_t)i * np;

  if (tid == 0) s.scount[i] = 0;
  if (t == s.start[i]) {
    // nodeStart -> initThisNode + introduceSelfToGroup (MP1Node.cpp:101-163)
    for (int c = tid; c < np; c += F_NODE_THREADS) row[c] = GM_ABSENT;
    __syncthreads();
    if (tid == 0) {
      s.failed[i] = 0;
      s.inited[i] = 1;
      s.ingroup[i] = 0;
      s.hbctr[i] = 0;
      s.jcnt[i] = 0;
      s.gcnt[i] = 0;
      s.fcnt[i] = 0;
      if (i == 0) {  // id 1 == getJoinAddress(): updateMyPos adds self, inGroup
        f_emit(s, t, i, 0, GM_EV_START_GROUP, 0);
        row[0] = gm_pack(0, (uint32_t)t);
        s.ingroup[i] = 1;
        s.started_now[i] = 0;
      } else {       // JOINREQ {my addr, heartbeat 0} to 1:0
        f_emit(s, t, i, 0, GM_EV_TRY_JOIN, 0);
        s.scount[i] = 1;
        s.started_now[i] = 1;
      }
    }
    return;
  }
  if (tid == 0) s.started_now[i] = 0;
  if (!(t > s.start[i] && !s.failed[i])) return;

  // ---- checkMessages: merge the queue (MP1Node.cpp:208-353)
  for (int c = tid; c < np; c += F_NODE_THREADS) {
    s_first[c] = 0x7fffffff;
    s_maxkey[c] = 0;
  }
  if (tid == 0) { s_misc[0] = 0; s_misc[1] = 0; s_misc[2] = 0; }
  __syncthreads();
  const FMsg *q = s.q + s.q_off[i];
  const int Q = s.q_cnt[i];
  for (int p = tid; p < Q; p += F_NODE_THREADS) {
    FMsg m = q[p];
    int type = m.type;
    if (type == F_JOINREP) {
      s_misc[0] = 1;
    } else if (type == F_JOINREQ || type == F_LIST) {
      int c = m.subj - 1;
      if (c >= 0 && c < s.n) {
        atomicMin(&s_first[c], p);
        atomicMax(&s_maxkey[c], m.hb + 1);
      }
    }
  }
  __syncthreads();
  // joined events (first-occurrence order), newNodes (JOINREQ that inserted),
  // JOINREP destinations (every JOINREQ, queue order)
  int nadd = 0, nnew = 0, njr = 0;
  for (int base = 0; base < Q; base += F_NODE_THREADS) {
    int p = base + tid;
    int fadd = 0, fnew = 0, fjr = 0, subj = 0;
    if (p < Q) {
      FMsg m = q[p];
      subj = m.subj;
      if (m.type == F_JOINREQ || m.type == F_LIST) {
        int c = m.subj - 1;
        if (c >= 0 && c < s.n && row[c] == GM_ABSENT && s_first[c] == p) {
          fadd = 1;
          fnew = m.type == F_JOINREQ;
        }
      }
      fjr = m.type == F_JOINREQ;
    }
    int ta, tn, tj;
    int ra = gm_block_scan(fadd, s_tmp, &ta);
    int rn = gm_block_scan(fnew, s_tmp, &tn);
    int rj = gm_block_scan(fjr, s_tmp, &tj);
    if (fadd) f_emit(s, t, i, 1 + nadd + ra, GM_EV_JOINED, subj);
    if (fnew) s.gossip[(size_t)i * s.gstride + nnew + rn] = subj;
    if (fjr) s.jrq[(size_t)i * s.n + njr + rj] = subj;
    nadd += ta;
    nnew += tn;
    njr += tj;
  }
  // apply the merged table (absent -> insert {hb, t}; present -> max, ts = t on increase)
  for (int c = tid; c < np; c += F_NODE_THREADS) {
    int key = s_maxkey[c];
    if (key > 0) {
      uint32_t e = row[c];
      uint32_t hb = (uint32_t)(key - 1);
      if (e == GM_ABSENT || gm_hb(e) < hb) row[c] = gm_pack(hb, (uint32_t)t);
    }
  }
  __syncthreads();
  int ingroup = s.ingroup[i] | s_misc[0];
  if (tid == 0) {
    s.ingroup[i] = ingroup;
    s.jcnt[i] = njr;
    s.scount[i] = njr;  // JOINREPs are sent inside checkMessages (MP1Node.cpp:246-250)
    s.gcnt[i] = 0;
    s.fcnt[i] = 0;
  }
  if (!ingroup) return;

  // ---- nodeLoopOps (MP1Node.cpp:404-495)
  // updateMyPos: lower_bound(self); add self only when nothing >= self exists (`&&` quirk)
  if (tid == 0) s_misc[3] = 0x7fffffff;
  __syncthreads();
  for (int c = i + tid; c < s.n; c += F_NODE_THREADS)
    if (row[c] != GM_ABSENT) atomicMin(&s_misc[3], c);
  __syncthreads();
  int mypos = s_misc[3];
  if (tid == 0) {
    int hbc = s.hbctr[i];
    if (mypos == 0x7fffffff) {
      mypos = i;
      row[i] = gm_pack((uint32_t)hbc, (uint32_t)t);
    }
    hbc += 1;                                          // heartbeat++
    row[mypos] = gm_pack((uint32_t)hbc, (uint32_t)t);  // myPos->setheartbeat(heartbeat++)
    s.hbctr[i] = hbc + 1;
    s_misc[4] = mypos;
  }
  __syncthreads();
  mypos = s_misc[4];
  // sweep: age >= TFAIL counts toward numfailed, age >= TREMOVE removes (descending id)
  int nfail = 0, npres = 0;
  for (int w = tid; w < nw; w += F_NODE_THREADS) {
    uint64_t pres = 0, fresh = 0, rem = 0;
    for (int b = 0; b < 64; b++) {
      int c = w * 64 + b;
      uint32_t e = row[c];
      if (e == GM_ABSENT) continue;
      int age = t - (int)gm_ts(e);
      if (age >= GM_TFAIL) {
        nfail++;
        if (age >= GM_TREMOVE) { row[c] = GM_ABSENT; rem |= 1ull << b; continue; }
      } else {
        fresh |= 1ull << b;
      }
      pres |= 1ull << b;
    }
    s_pres[w] = pres;
    s_fresh[w] = fresh;
    s_rem[w] = rem;
    npres += __builtin_popcountll(pres);
  }
  int totfail, totpres;
  (void)gm_block_scan(nfail, s_tmp, &totfail);
  (void)gm_block_scan(npres, s_tmp, &totpres);
  // removal events: descending column order (MP1Node.cpp:429-444)
  {
    int nrem = 0;
    for (int top = np - 1; top >= 0; top -= F_NODE_THREADS) {
      int c = top - tid;
      int frem = 0;
      if (c >= 0) frem = (s_rem[c >> 6] >> (c & 63)) & 1ull;
      int tr;
      int rr = gm_block_scan(frem, s_tmp, &tr);
      if (frem) f_emit(s, t, i, 1 + nadd + nrem + rr, GM_EV_REMOVED, c + 1);
      nrem += tr;
    }
    if (tid == 0) s_misc[5] = nrem;
  }
  __syncthreads();
  // prefix popcounts for rank-select
  if (tid == 0) {
    uint32_t acc = 0;
    for (int w = 0; w < nw; w++) { s_pre[w] = acc; acc += (uint32_t)__builtin_popcountll(s_pres[w]); }
  }
  // fresh columns, ascending (sendMemberList iterates the sorted list: MP1Node.cpp:372-392)
  {
    int nf = 0;
    for (int base = 0; base < np; base += F_NODE_THREADS) {
      int c = base + tid;
      int ff = (c < np) && ((s_fresh[c >> 6] >> (c & 63)) & 1ull);
      int tf;
      int rf = gm_block_scan(ff, s_tmp, &tf);
      if (ff) s.fcols[(size_t)i * s.n + nf + rf] = c;
      nf += tf;
    }
    if (tid == 0) s_misc[6] = nf;
  }
  __syncthreads();
  if (tid == 0) {
    // gossip targets: newNodes first, then Lemire draws over the post-sweep list
    int size = totpres;
    int numpot = size - 1 - totfail;
    int *g = s.gossip + (size_t)i * s.gstride;
    int n = nnew;
    if (n < GM_FANOUT && n < numpot) {
      GmLazyMT mt;
      mt.seed(s_mt, gm_rd_seed(s.rd_seed, t, i + 1));
      long guard = 0;
      while (n < GM_FANOUT && n < numpot) {
        if (++guard > (1l << 22)) { atomicOr(s.err, GM_ERR_DRAWS); break; }
        int ix = mt.uniform((uint32_t)size);
        int c = gm_rank_select(s_pres, s_pre, nw, (uint32_t)ix);
        if (c == mypos) continue;
        if (!((s_fresh[c >> 6] >> (c & 63)) & 1ull)) continue;  // skipfailed (numpot > 0 here)
        bool found = false;
        for (int k = 0; k < n; k++)
          if (g[k] == c + 1) { found = true; break; }
        if (!found) g[n++] = c + 1;
      }
    }
    int nf = s_misc[6];
    s.gcnt[i] = n;
    s.fcnt[i] = nf;
    s.scount[i] = njr + n * nf;
    if (i == 0 && t % 500 == 0) f_emit(s, t, i, 1 + nadd + s_misc[5], GM_EV_TIME_MARK, 0);
  }
}

// ---------------------------------------------------------------- send phase
__global__ __launch_bounds__(F_SEND_THREADS) void gm_f_send(FState s, int t) {
  __shared__ int s_tmp[32];
  __shared__ int s_base[1024];
  __shared__ int s_total;
  // node-phase order is i descending: exclusive scan of scount over i = n-1..0
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int i = s.n - 1; i >= 0; i--) { s_base[i] = acc; acc += s.scount[i]; }
    s_total = acc;
  }
  __syncthreads();
  const int S = s_total;
  if (S > s.draw_cap) {
    if (threadIdx.x == 0) atomicOr(s.err, GM_ERR_DRAWS);
    return;
  }
  // S1: one glibc rand() draw per ENsend, in send order (EmulNet.cpp:90). glibc TYPE_3
  // keeps rptr 3 words behind fptr (mod 31), both advancing by one per draw; with the
  // ring rotated so that x[j] is the word fptr reaches at step j of each 31-step round,
  // step j is x[j] += x[(j + 28) % 31] -- static register indices in a fully unrolled
  // round, no dynamically indexed (scratch) state on the serial chain.
  if (threadIdx.x == 0) {
    const int f0 = s.s1[31];
    uint32_t x[31];
    for (int j = 0; j < 31; j++) x[j] = (uint32_t)s.s1[(f0 + j) % 31];
    int o = 0;
    for (; o + 31 <= S; o += 31) {
#pragma unroll
      for (int j = 0; j < 31; j++) {
        x[j] += x[(j + 28) % 31];
        s.draws[o + j] = (int32_t)(x[j] >> 1);
      }
    }
#pragma unroll
    for (int j = 0; j < 31; j++) {
      if (o + j < S) {
        x[j] += x[(j + 28) % 31];
        s.draws[o + j] = (int32_t)(x[j] >> 1);
      }
    }
    for (int j = 0; j < 31; j++) s.s1[(f0 + j) % 31] = (int32_t)x[j];
    const int f = (f0 + S) % 31;
    s.s1[31] = f;
    s.s1[32] = (f + 28) % 31;
  }
  __syncthreads();
  const int B0 = *s.bufsize;
  const int room = F_ENBUFFSIZE - B0;
  const int pct = s.drop_pct_now;  // (int)(MSG_DROP_PROB*100) while dropmsg, else -1
  int kept = 0;                    // not-drop-drawn sends so far
  for (int base = 0; base < S; base += F_SEND_THREADS) {
    int o = base + threadIdx.x;
    int keep = 0;
    if (o < S) keep = !(pct >= 0 && (s.draws[o] % 100) < pct);
    int tk;
    int rk = gm_block_scan(keep, s_tmp, &tk);
    int before = kept + rk;
    if (keep && before < room) {
      // locate the sender: s_base is non-increasing in i; the smallest i with
      // s_base[i] <= o is the node whose sends contain ordinal o
      int lo = 0, hi = s.n - 1, i = s.n - 1;
      while (lo <= hi) {
        int mid = (lo + hi) >> 1;
        if (s_base[mid] <= o) { i = mid; hi = mid - 1; } else lo = mid + 1;
      }
      int k = o - s_base[i];
      FMsg m;
      m.from = i + 1;
      if (s.started_now[i]) {
        m.to = 1;
        m.type = F_JOINREQ;
        m.subj = i + 1;
        m.hb = 0;
      } else if (k < s.jcnt[i]) {
        m.to = s.jrq[(size_t)i * s.n + k];
        m.type = F_JOINREP;
        m.subj = 0;
        m.hb = 0;
      } else {
        int kk = k - s.jcnt[i];
        int nf = s.fcnt[i];
        int g = kk / nf, e = kk % nf;
        int c = s.fcols[(size_t)i * s.n + e];
        m.to = s.gossip[(size_t)i * s.gstride + g];
        m.type = F_LIST;
        m.subj = c + 1;
        m.hb = (int)gm_hb(s.table[(size_t)i * s.np + c]);
      }
      s.buf[B0 + before] = m;
      atomicAdd(&s.sent[(size_t)(i + 1) * s.tmax + t], 1);  // sent_msgs[src][time]
    }
    kept += tk;
  }
  if (threadIdx.x == 0) *s.bufsize = B0 + min(kept, room);
}
