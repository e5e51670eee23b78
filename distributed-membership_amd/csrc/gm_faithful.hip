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
#include <type_traits>
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
// gm_f_recv (one workgroup) walks the receivers ascending on an LDS image of the buffer:
// one u32 per buffered message, its destination key << 16 | its index in the tick-start
// buffer (F_ENBUFFSIZE < 2^16; the key -- the strcmp prefix of the destination address,
// EmulNet.cpp:154 -- of ids 1..n is <= n; it is kept beside the buffer in bkey), message
// counts per (key, segment of `seg` slots, seg sized from n so the table stays ~24 KB),
// the receivers' active flags and two k-entry scratch arrays. Per receiver with k messages:
//   ranks  a DPP scan over the key's segment counts gives every segment's first rank;
//   scan   waves take the segments holding a match (and those of the vacated tail
//          [B-k, B)) round-robin; a match stores its position at hit[rank], every tail
//          slot gets its hole rank (1-based descending, 0 = no match);
//   fill   one thread per rank: queue slot k-1-rank (descending buffer index = the
//          reference's dequeue order) gets the message's tick-start index, and a match
//          below B-k is overwritten in closed form: the hole of descending rank i
//          receives what sits at B-i when it is processed, i.e. follow the chain
//          through earlier tail holes to an original element;
// with one LDS-only barrier after each. gm_f_recvout (many workgroups) then materialises
// the queues and compacts the survivors into the other buffer. Ranks over the LDS room
// use the same code on global scratch with full barriers.
#define F_EL_SLOTS ((F_ENBUFFSIZE + 255) / 256 * 256)  // el[] incl. the b128 overread pad
#define F_CW_BYTES 24576                               // count table budget
static_assert(4 * F_EL_SLOTS + F_CW_BYTES + 4 * (F_MAX_NODES + 1) + F_MAX_NODES + 4 * 1024 <= F_RECV_LDS,
              "gm_f_recv LDS budget");

__device__ __forceinline__ void lds_barrier() {
  // every wave's LDS traffic done, then the barrier; global stores stay in flight
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ int mbcnt(uint64_t m) {  // set bits of m in the lanes below
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

__device__ __forceinline__ int wave_incl_scan(int v) {  // DPP: rows by row_shr, then row_bcast
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);
  return v;
}

__global__ __launch_bounds__(F_RECV_THREADS) void gm_f_recv(FState s, int t) {
  extern __shared__ uint32_t s_lds[];
  const int n = s.n;
  // segment size: a multiple of 256 slots, (n + 1) x nseg u16 counts within F_CW_BYTES, nseg <= 128
  const int seg = max(256, (F_EL_SLOTS / min(128, F_CW_BYTES / 2 / (n + 1)) + 255) & ~255);
  const int nsw = ((F_EL_SLOTS + seg - 1) / seg + 1) >> 1;  // count words per key (2 segments each)
  uint32_t *el = s_lds;                                 // [F_EL_SLOTS]
  uint32_t *cw = s_lds + F_EL_SLOTS;                    // [n + 1][nsw]
  uint8_t *act = (uint8_t *)(cw + (n + 1) * nsw);       // [n], padded to 4
  uint16_t *scr = (uint16_t *)(act + ((n + 3) & ~3));   // [2][cap]: hole ranks, hit positions
  const int cap = (int)((F_RECV_LDS - ((uint8_t *)scr - (uint8_t *)s_lds)) / 4);
  int B = *s.bufsize;
  for (int j = threadIdx.x; j < (n + 1) * nsw; j += F_RECV_THREADS) cw[j] = 0;
  for (int i = threadIdx.x; i < n; i += F_RECV_THREADS)
    act[i] = t > s.start[i] && !s.failed[i];  // Application.cpp:130
  __syncthreads();
  for (int j0 = threadIdx.x; j0 < B; j0 += 8 * F_RECV_THREADS) {
    uint32_t kk[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int j = j0 + u * F_RECV_THREADS;
      kk[u] = j < B ? s.bkey[j] : 0u;
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int j = j0 + u * F_RECV_THREADS;
      if (j >= B) break;
      el[j] = kk[u] << 16 | (uint32_t)j;
      const int g = j / seg;
      atomicAdd(&cw[kk[u] * nsw + (g >> 1)], 1u << (16 * (g & 1)));
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int qbase = 0;
  for (int i = 0; i < n; i++) {
    if (threadIdx.x == 0) { s.q_off[i] = qbase; s.q_cnt[i] = 0; }
    if (!act[i]) continue;
    const uint32_t me = f_strkey(i + 1);
    // all of this key's messages go to its first active receiver; lane l holds the
    // counts of segments 2l, 2l+1 and the number of matches in the segments below 2l
    const uint32_t wd = lane < nsw ? cw[me * nsw + lane] : 0u;
    const int clo = (int)(wd & 0xFFFFu), chi = (int)(wd >> 16);
    const int incl = wave_incl_scan(clo + chi);
    const int k = __builtin_amdgcn_readlane(incl, 63);
    if (k == 0) continue;
    const int excl = incl - clo - chi;
    const int Bn = B - k;
    auto walk = [&](auto big_tag) {
      constexpr bool BIG = decltype(big_tag)::value;
      uint16_t *hp = BIG ? s.holepos : scr;
      uint16_t *hit = BIG ? s.holepos + F_ENBUFFSIZE : scr + cap;
      for (int g = wid; g * seg < B; g += F_RECV_THREADS / 64) {
        const int l = g >> 1;
        const int cg = (g & 1) ? __builtin_amdgcn_readlane(chi, l) : __builtin_amdgcn_readlane(clo, l);
        const int s0 = g * seg, s1 = min(B, s0 + seg);
        if (cg == 0 && s1 <= Bn) continue;
        int r = __builtin_amdgcn_readlane(excl, l) + ((g & 1) ? __builtin_amdgcn_readlane(clo, l) : 0);
        for (int j0 = cg ? s0 : max(s0, Bn & ~255); j0 < s1; j0 += 256) {
          const int jb = j0 + 4 * lane;
          const uint4 e4 = *(const uint4 *)&el[jb];
          const uint32_t e[4] = {e4.x, e4.y, e4.z, e4.w};
          bool h[4];
          uint64_t b[4];
          int rk = r;
#pragma unroll
          for (int q = 0; q < 4; q++) {
            h[q] = jb + q < s1 && (e[q] >> 16) == me;
            b[q] = __ballot(h[q]);
            rk += mbcnt(b[q]);
          }
#pragma unroll
          for (int q = 0; q < 4; q++) {
            const int j = jb + q;
            if (h[q]) hit[rk] = (uint16_t)j;
            if (j >= Bn && j < s1) hp[j - Bn] = h[q] ? (uint16_t)(k - rk) : (uint16_t)0;
            rk += h[q];
          }
          r += __popcll(b[0]) + __popcll(b[1]) + __popcll(b[2]) + __popcll(b[3]);
        }
      }
      if constexpr (BIG) __syncthreads(); else lds_barrier();
      for (int rk = threadIdx.x; rk < k; rk += F_RECV_THREADS) {
        const int j = hit[rk];
        s.qidx[qbase + (k - 1 - rk)] = (uint16_t)(el[j] & 0xFFFFu);
        if (j >= Bn) continue;
        int x = B - (k - rk);
        for (int guard = 0; guard < k; guard++) {
          const int hx = hp[x - Bn];
          if (hx == 0) break;
          x = B - hx;
        }
        const uint32_t mv = el[x];  // x >= Bn, not a match: never overwritten in this pass
        el[j] = mv;
        const int gx = x / seg, gj = j / seg;  // the moved message may change segment
        if (gx != gj) {
          const uint32_t kx = mv >> 16;
          atomicSub(&cw[kx * nsw + (gx >> 1)], 1u << (16 * (gx & 1)));
          atomicAdd(&cw[kx * nsw + (gj >> 1)], 1u << (16 * (gj & 1)));
        }
      }
      if (threadIdx.x < nsw) cw[me * nsw + threadIdx.x] = 0;
      if (threadIdx.x == 0) s.q_cnt[i] = k;
      if constexpr (BIG) __syncthreads(); else lds_barrier();
    };
    if (k > cap) walk(std::true_type{}); else walk(std::false_type{});
    qbase += k;
    B = Bn;
  }
  for (int j = threadIdx.x; j < B; j += F_RECV_THREADS) s.sidx[j] = (uint16_t)(el[j] & 0xFFFFu);
  if (threadIdx.x == 0) {
    s.rmeta[0] = qbase;
    s.rmeta[1] = B;
  }
}

// queues and survivors (grid-stride over both), recv_msgs counters
__global__ __launch_bounds__(256) void gm_f_recvout(FState s, int t) {
  const int Q = s.rmeta[0], B = s.rmeta[1];
  const int stride = gridDim.x * blockDim.x;
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  for (int p = tid; p < Q; p += stride) s.q[p] = s.buf[s.qidx[p]];
  for (int j = tid; j < B; j += stride) {
    const int x = s.sidx[j];
    s.buf2[j] = s.buf[x];
    s.bkey2[j] = s.bkey[x];
  }
  for (int i = tid; i < s.n; i += stride)
    s.recv[(size_t)(i + 1) * s.tmax + t] += s.q_cnt[i];  // recv_msgs[dst][time] (EmulNet.cpp:172)
  if (tid == 0) *s.bufsize = B;
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
// S1: one glibc rand() draw per ENsend, in send order (EmulNet.cpp:90). glibc TYPE_3 keeps
// rptr 3 words behind fptr (mod 31), both advancing by one per draw. With the ring rotated
// so that x[j] is the word fptr reaches at step j of a 31-step round, step j is
// x[j] += x[(j + 28) % 31] and its draw is x[j] >> 1: a round maps the register vector v
// linearly (mod 2^32) to v' = R v and its 31 draws are v' >> 1. So round m's draws are
// (R^(m+1) v0) >> 1, computed in parallel from precomputed powers: the prep kernel steps
// block states v_(64b) = (R^64)^b v0 serially (one 31x31 product per 1984 draws) and the
// expansion evaluates round 64b + q as R^(q+1) v_(64b), one output word per lane.

// node-phase order is i descending: exclusive scan of scount over i = n-1..0; S1 block states
__global__ __launch_bounds__(64) void gm_f_sendprep(FState s) {
  const int lane = threadIdx.x;
  int acc = 0;
  for (int top = s.n - 1; top >= 0; top -= 64) {
    const int i = top - lane;
    const int v = i >= 0 ? s.scount[i] : 0;
    int x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int y = __shfl_up(x, d);
      if (lane >= d) x += y;
    }
    if (i >= 0) s.sbase[i] = acc + x - v;
    acc += __shfl(x, 63);
  }
  const int S = acc;
  if (S > s.draw_cap) {
    if (lane == 0) {
      atomicOr(s.err, GM_ERR_DRAWS);
      s.smeta[0] = -1;
    }
    return;
  }
  const int f0 = s.s1[31];
  const int nb = S / 31 / 64 + 1;  // block states the expansion reads (rounds 0 .. S/31)
  const uint32_t *r64 = s.s1mat + (size_t)63 * 31 * 32;  // R^64 = P_63
  uint32_t row[31];
#pragma unroll
  for (int j = 0; j < 31; j++) row[j] = lane < 31 ? r64[lane * 32 + j] : 0u;
  uint32_t v = lane < 31 ? (uint32_t)s.s1[(f0 + lane) % 31] : 0u;
  for (int b = 0; b < nb; b++) {
    if (lane < 32) s.s1vb[(size_t)b * 32 + lane] = v;
    if (b + 1 < nb) {
      uint32_t a = 0;
#pragma unroll
      for (int j = 0; j < 31; j++) a += row[j] * (uint32_t)__builtin_amdgcn_readlane((int)v, j);
      v = a;
    }
  }
  if (lane == 0) {
    s.smeta[0] = S;
    s.smeta[1] = f0;
    const int f = (f0 + S) % 31;
    s.s1[31] = f;
    s.s1[32] = (f + 28) % 31;
  }
}

// the tick's S draws: round m (lanes 0..30 of a half-wave) = P_(m mod 64) v_(64 (m / 64));
// the rounds holding the last draw write the register back (words j < S mod 31 from round
// S/31, the rest from round S/31 - 1; none change when S < 31 for j >= S)
__global__ __launch_bounds__(256) void gm_f_s1expand(FState s) {
  const int S = s.smeta[0];
  if (S <= 0) return;
  const int f0 = s.smeta[1];
  const int full = S / 31, rem = S % 31;
  const int k = threadIdx.x & 31;
  const int hw = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 5), nhw = (int)((gridDim.x * blockDim.x) >> 5);
  if (k == 31) return;
  for (int m = hw; m <= full; m += nhw) {
    const uint4 *P = (const uint4 *)(s.s1mat + ((size_t)(m & 63) * 31 + k) * 32);
    const uint4 *vb = (const uint4 *)(s.s1vb + (size_t)(m >> 6) * 32);
    uint32_t a = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const uint4 p = P[j], x = vb[j];
      a += p.x * x.x + p.y * x.y + p.z * x.z + p.w * x.w;  // word 31 of both is 0
    }
    const int o = m * 31 + k;
    if (o < S) s.draws[o] = (int32_t)(a >> 1);
    if ((m == full && k < rem) || (m == full - 1 && k >= rem)) s.s1[(f0 + k) % 31] = (int32_t)a;
  }
}

// ENsend's drop draw and the 30000 cap (EmulNet.cpp:90-99): exclusive prefix count of the
// not-drop-drawn sends in send order (pre[o]); a send is buffered at B0 + pre[o] iff kept
// and pre[o] < room. One workgroup; thread t scans a contiguous run of ordinals.
__global__ __launch_bounds__(F_SEND_THREADS) void gm_f_sendscan(FState s, int t) {
  __shared__ int s_tmp[32];
  const int S = s.smeta[0];
  if (S < 0) return;  // draw cap exceeded (error latched by gm_f_sendprep)
  const int pct = s.drop_pct_now;  // (int)(MSG_DROP_PROB*100) while dropmsg, else -1
  const int L = (S + F_SEND_THREADS - 1) / F_SEND_THREADS;
  const int o0 = min(S, (int)threadIdx.x * L), o1 = min(S, o0 + L);
  int c = 0;
  for (int o = o0; o < o1; o++) c += !(pct >= 0 && (s.draws[o] % 100) < pct);
  int total;
  int p = gm_block_scan(c, s_tmp, &total);
  for (int o = o0; o < o1; o++) {
    s.spre[o] = p;
    p += !(pct >= 0 && (s.draws[o] % 100) < pct);
  }
  if (threadIdx.x == 0) s.spre[S] = total;
  __syncthreads();
  const int B0 = *s.bufsize;
  const int room = F_ENBUFFSIZE - B0;
  // sent_msgs[src][time]: node i's buffered sends are its kept ordinals below the cap
  for (int i = threadIdx.x; i < s.n; i += F_SEND_THREADS) {
    const int a = s.sbase[i], b = a + s.scount[i];
    const int k = min(s.spre[b], room) - min(s.spre[a], room);
    if (k) s.sent[(size_t)(i + 1) * s.tmax + t] += k;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    s.smeta[2] = B0;
    *s.bufsize = B0 + min(total, room);
  }
}

// materialise every buffered send (grid-stride over ordinals)
__global__ __launch_bounds__(256) void gm_f_sendemit(FState s) {
  __shared__ int s_base[F_MAX_NODES];
  const int S = s.smeta[0];
  if (S <= 0) return;
  const int B0 = s.smeta[2];
  const int room = F_ENBUFFSIZE - B0;
  const int pct = s.drop_pct_now;
  for (int i = threadIdx.x; i < s.n; i += blockDim.x) s_base[i] = s.sbase[i];
  __syncthreads();
  for (int o = blockIdx.x * blockDim.x + threadIdx.x; o < S; o += gridDim.x * blockDim.x) {
    const int before = s.spre[o];
    if (before >= room || (pct >= 0 && (s.draws[o] % 100) < pct)) continue;
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
    uint32_t key = f_strkey(m.to);
    if (key > (uint32_t)s.n) {  // destinations are node ids 1..n (ENsend asserts them)
      atomicOr(s.err, GM_ERR_BUFFER);
      key = s.n;
    }
    s.bkey[B0 + before] = (uint16_t)key;
  }
}
