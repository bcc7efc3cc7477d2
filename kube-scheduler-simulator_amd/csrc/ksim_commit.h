// ksim_commit.h — the batch commit shared by the P100 (ksim_batch.hip) and
// ADAPT (ksim_adapt.hip) batch paths.
#pragma once

#include "ksim_device.h"
#include "ksim_internal.h"
#include "ksim_wave.h"

namespace ksim {

// The batch's pod cap (DevState::bcap; kBatchPods when none) and its pods.
__device__ __forceinline__ int32_t batch_cap(const DevState* __restrict__ st) {
  const int32_t cap = st->bcap;
  return cap > 0 && cap < kBatchPods ? cap : kBatchPods;
}
__device__ __forceinline__ int32_t batch_pods(const DevState* __restrict__ st) {
  return min(batch_cap(st), st->end - st->cursor);
}

// Nodes of the circular scan window [s, s + len) of the cluster's n_total
// nodes that lie on this snapshot ([base, base + n)): the evaluations a shard
// ran for the window (all of them on an unsharded handle).
__device__ __forceinline__ int64_t window_local(const DevCluster& c, int32_t s, int64_t len) {
  const int64_t N = c.n_total, lo = c.base, hi = (int64_t)c.base + c.n;
  auto ov = [&](int64_t a, int64_t b) -> int64_t {   // |[a, b) n [lo, hi)|
    const int64_t x = a > lo ? a : lo, y = b < hi ? b : hi;
    return y > x ? y - x : 0;
  };
  if (s + len <= N) return ov(s, s + len);
  return ov(s, N) + ov(0, s + len - N);
}

// The resource columns of one node row and one pod's requests on them.
struct ResCols {
  int64_t cpu, mem, eph, nzc, nzm;
  int32_t pods;
};

// Validate the chain against M (pmax) and commit (one block of kBatchPods
// threads).  Its barriers hand off LDS only (lds_barrier): the row loads stay
// in flight across them and the row stores are not waited for (each committed
// pod's node has one writer; the next launch sees them).  Binds are applied by the shard that owns the node.  s_aw (ADAPT
// batch): per pod {scan start, cut offset or -1} (the awin pairs), staged in
// LDS by the caller from loads issued at kernel start, so neither the
// evaluation count nor nextStartNodeIndex waits for a global load after the
// cut is known; the evaluated counts and nextStartNodeIndex follow the
// committed pods' windows.  g_own / m_own: this thread's gkey / pmax entries,
// loaded by the caller at kernel start (before the state load they do not
// depend on).  inv_own (P100 generic runs, topology batches): this thread's
// pinv entry; the chain ends before the first flagged pod (pairs_block).
// nb_cap: the topology batch's pod count.
__device__ __forceinline__ void batch_commit(const DevCluster& c, const DevPods& P, DevState* __restrict__ st,
                                             uint64_t g_own, uint64_t m_own, const uint64_t* __restrict__ pmax,
                                             int32_t nchain, int32_t* __restrict__ chosen_out, int32_t* s_istar,
                                             int32_t* s_sched, int32_t* s_unsched,
                                             const int2* s_aw = nullptr, const int32_t* inv_own = nullptr,
                                             int32_t nb_cap = kBatchPods, int32_t* s_node = nullptr,
                                             bool adapt_cap = false) {
  __shared__ int32_t s_evals;
  __shared__ uint64_t s_m[kBatchPods];
  __shared__ ResCols s_req[kBatchPods];
  const int tid = threadIdx.x;
  if (inv_own) {                                   // block-uniform
    if (tid == 0) *s_istar = nchain;
    lds_barrier();
    block_first_min(s_istar, tid < nchain && *inv_own);
    lds_barrier();
    nchain = *s_istar;
    lds_barrier();                               // every read before s_istar is reused below
  }
  const int32_t base = st->cursor;
  const int32_t nb = min(nb_cap, st->end - base);   // the batch's pods (statistics: cut or truncated)
  const int64_t seq0 = st->pod_seq;
  // thread 0 rewrites the state whole at the end: its words loaded now, in
  // flight with the rest (no load round trip after the last barrier)
  constexpr int kStWords = (int)(sizeof(DevState) / 8);
  static_assert(sizeof(DevState) % 8 == 0, "DevState by words");
  uint64_t stw[kStWords];
  if (tid == 0) {
#pragma unroll
    for (int q = 0; q < kStWords; q++) stw[q] = reinterpret_cast<const uint64_t*>(st)[q];
  }
  const uint64_t gj = tid < nchain ? g_own : 0;
  const uint64_t mj = tid < nchain ? m_own : 0;
  // ahead of the cut: the row of the node this pod guessed (it binds there if
  // committed; bound nodes are distinct, so this thread is its only writer)
  // and the pod's requests (in LDS: pod i* may bind on another pod's node)
  const int32_t glocal = gj ? key_node(gj) - c.base : -1;
  const bool gown = glocal >= 0 && glocal < c.n;
  ResCols row{0, 0, 0, 0, 0, 0};
  if (gown) row = ResCols{c.req_cpu[glocal], c.req_mem[glocal], c.req_eph[glocal], c.nz_cpu[glocal], c.nz_mem[glocal],
                          c.num_pods[glocal]};
  if (tid < nchain) {
    const ksim_pod& p = P.pods[base + tid];
    s_req[tid] = ResCols{p.req_cpu, p.req_mem, p.req_eph, p.nz_cpu, p.nz_mem, 1};
  }
  s_m[tid] = mj;
  if (tid == 0) {
    *s_istar = nchain;
    *s_sched = 0;
    *s_unsched = 0;
    s_evals = 0;
  }
  lds_barrier();
  block_first_min(s_istar, tid < nchain && mj > gj);   // keys are unique per node: never equal unless 0
  lds_barrier();
  const int32_t istar = *s_istar;
  const int32_t committed = istar < nchain ? istar + 1 : nchain;
  const int32_t inode = istar < nchain ? key_node(s_m[istar]) : -1;
  // s_node (topology batches): each committed pod's local node (-1: none,
  // -2: not committed); the caller applies the class adds in parallel
  if (s_node && tid < nb_cap) s_node[tid] = tid >= committed ? -2 : tid == istar ? inode - c.base
                                                             : gj ? key_node(gj) - c.base : -1;
  if (tid < committed) {
    const int32_t node = tid == istar ? inode : (gj ? key_node(gj) : -1);     // global position
    if (chosen_out) chosen_out[base + tid] = node;
    atomicAdd(node >= 0 ? s_sched : s_unsched, 1);
    if (tid < istar && gown) {
      auto add = [&](const ResCols& q) {
        row.cpu += q.cpu;
        row.mem += q.mem;
        row.eph += q.eph;
        row.nzc += q.nzc;
        row.nzm += q.nzm;
        row.pods += q.pods;
      };
      add(s_req[tid]);
      if (!s_node) assume_pod_rest(c, P, P.pods[base + tid], glocal, 1);
      else assume_pod_cols(c, P.pods[base + tid], glocal);
      if (node == inode) {
        add(s_req[istar]);
        if (!s_node) assume_pod_rest(c, P, P.pods[base + istar], glocal, 1);
        else assume_pod_cols(c, P.pods[base + istar], glocal);
      }
      c.req_cpu[glocal] = row.cpu;
      c.req_mem[glocal] = row.mem;
      c.req_eph[glocal] = row.eph;
      c.nz_cpu[glocal] = row.nzc;
      c.nz_mem[glocal] = row.nzm;
      c.num_pods[glocal] = row.pods;
    }
  }
  if (s_aw && tid < committed) {
    const int2 w = s_aw[tid];
    atomicAdd(&s_evals, (int32_t)window_local(c, w.x, w.y >= 0 ? (int64_t)w.y + 1 : c.n_total));
  }
  lds_barrier();
  if (tid == 0) {
    DevState ns;
    __builtin_memcpy(&ns, stw, sizeof(ns));
    if (s_aw && committed > 0) {
      const int2 w = s_aw[committed - 1];
      ns.next_start = (int32_t)(((int64_t)w.x + (w.y >= 0 ? w.y : c.n_total)) % c.n_total);
      if (c.count_whole) ns.evals += s_evals;
    } else {
      ns.evals += (int64_t)committed * (c.eval_hi - c.eval_lo);   // the nodes this handle evaluated
    }
    ns.cursor = base + committed;
    ns.pod_seq = seq0 + committed;
    ns.scheduled += *s_sched;
    ns.unschedulable += *s_unsched;
    ns.batches += 1;
    if (committed < nb) {
      if (istar < nchain) ns.cuts += 1;
      else ns.truncations += 1;
    }
    if (adapt_cap) {
      // generic ADAPT: the next batch evaluates about twice what this one
      // committed (its mask and window launches scale with the pods), at
      // least 32, the whole batch again once a batch commits every pod
      const int32_t want = committed < nb ? 2 * committed : 2 * nb;
      const int32_t cap = min(kBatchPods, max(32, (want + 31) & ~31));
      ns.bcap = cap >= kBatchPods ? 0 : cap;
    }
    __builtin_memcpy(stw, &ns, sizeof(ns));
#pragma unroll
    for (int q = 0; q < kStWords; q++) reinterpret_cast<uint64_t*>(st)[q] = stw[q];
  }
}

// A lane's DefaultNormalizeScore maxima of a kPodNormVaries pod's raw
// TaintToleration / NodeAffinity scores over its S0-feasible nodes, and how
// many of its nodes hold each (raw scores are >= 0).
struct NormAcc {
  uint64_t lt = 0, la = 0;
  int32_t ct = 0, ca = 0;
  __device__ __forceinline__ void take(const NormRaw& v) {
    ct = (uint64_t)v.tt > lt ? 1 : ct + ((uint64_t)v.tt == lt ? 1 : 0);
    lt = umax64(lt, (uint64_t)v.tt);
    ca = (uint64_t)v.na > la ? 1 : ca + ((uint64_t)v.na == la ? 1 : 0);
    la = umax64(la, (uint64_t)v.na);
  }
};

// The block's maxima (returned to every thread) and their holder counts:
// thread 0 writes pnorm[4 j .. 4 j + 3] (the batch keeps pod j until every
// holder of a maximum has left its feasible set: pairs_block, k_adapt_pairs).
template <int kTopThreads>
__device__ __forceinline__ NormRaw norm_maxima(const NormAcc& n, int64_t* __restrict__ pnorm, int32_t j) {
  constexpr int kTopWaves = kTopThreads / 64;
  __shared__ uint64_t s_nmax[2][kTopWaves];
  __shared__ int32_t s_ncnt[2][kTopWaves];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t xt = wave_max_u64_dpp(n.lt), xa = wave_max_u64_dpp(n.la);
  if (lane == 0) {
    s_nmax[0][wv] = xt;
    s_nmax[1][wv] = xa;
  }
  __syncthreads();
#pragma unroll
  for (int w = 0; w < kTopWaves; w++) {
    xt = umax64(xt, s_nmax[0][w]);
    xa = umax64(xa, s_nmax[1][w]);
  }
  int32_t nt = n.lt == xt ? n.ct : 0, na = n.la == xa ? n.ca : 0;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    nt += __shfl_xor(nt, d, 64);
    na += __shfl_xor(na, d, 64);
  }
  if (lane == 0) {
    s_ncnt[0][wv] = nt;
    s_ncnt[1][wv] = na;
  }
  __syncthreads();
  const NormRaw mx{(int64_t)xt, (int64_t)xa};
  if (threadIdx.x == 0) {
    int32_t tt = 0, ta = 0;
    for (int w = 0; w < kTopWaves; w++) {
      tt += s_ncnt[0][w];
      ta += s_ncnt[1][w];
    }
    pnorm[4 * j] = mx.tt;
    pnorm[4 * j + 1] = mx.na;
    pnorm[4 * j + 2] = tt;
    pnorm[4 * j + 3] = ta;
  }
  return mx;
}

}  // namespace ksim
