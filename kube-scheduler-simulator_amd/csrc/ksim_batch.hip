// ksim_batch.hip — the speculative batch path of the scheduling cycle (gfx950).
//
// For B = kBatchPods consecutive pods of the queue that are "batchable" (P100,
// see pod_batchable in ksim_engine.cpp), placements equal running the cycle
// pod by pod (bit-exact with the oracle).  A batch is
//
//   k_batch_top          one block per pod: every pod x node pair against the
//                        batch-start snapshot S0 (static filters, Fit filter,
//                        LeastAllocated, BalancedAllocation, TB key) and the
//                        pod's provably exact top-T under S0;
//   k_batch_chain_pairs  one block per pod, every block running the greedy
//                        chain (pod i guesses the first entry of its list not
//                        guessed by an earlier pod of the batch; parallel
//                        relaxation, ksim_chain.h), then block j, thread k < j:
//                        key of pod j on pod k's guess after pod k is bound
//                        there; the block max M_j;
//   k_batch_commit       one block: validates the chain and commits
//
// or, on FAST runs of an unsharded handle, the deferred-commit form
// (k_batch_top_commit: batch i-1's commit inside batch i's top launch).
//
// Exactness: pods 0..i-1 took their guesses (distinct nodes), so before pod i
// only those nodes differ from S0.  Pod i's guess is the best node still at
// S0 (its list is the exact S0 top-T, minus nodes bound since), so pod i's
// exact choice is max(guess key, M_i).  The batch commits every pod up to the
// first i* with M_i* > guess key, and i* itself (it takes the node of M_i*).
// An exhausted incomplete list also ends the batch; the next batch starts at
// the first pod not committed.
#include "ksim_device.h"
#include <atomic>

#include "ksim_internal.h"
#include "ksim_wave.h"
#include "ksim_commit.h"
#include "ksim_chain.h"

namespace ksim {

// KEEP forms: on node ranges of at most kKeepPerLane * threads nodes every lane
// keeps all of its keys in registers (no insertion network; top_finish takes
// them unsorted)
constexpr int kKeepPerLane = 8;

// ---- k_batch_top: evaluation and the pod's top-T in one launch -------------------
// One block per pod of the batch (kTopThreads threads, kTopWaves waves: two per
// SIMD when every CU holds one block), the nodes strided over its lanes.  Each
// lane keeps its best kTileCand keys (and counts its feasible nodes); each wave
// extracts its provably exact top-T prefix from the lane lists; wave 0 merges
// the wave lists into the pod's top-T.  A list holds only its best keys: once a
// lane that had more feasible nodes than it kept has given up its last kept key,
// the next key of its wave cannot be proven, so the wave's prefix ends there
// (complete = 0); the block merge keeps the keys >= the last listed key of every
// incomplete wave (every key a wave did not list is below it).  complete = 1:
// every S0-feasible node is in the pod's list.

// The pod's top-T from the lanes' kept keys (a[]: the lane's best N keys,
// descending; nfeas: the lane's feasible nodes), written to topk[j] (and the
// sharded record xsend[j]).  Every thread of the block calls it.  !SORTED: a[]
// holds every key of the lane, in node order (nfeas <= N: nothing hidden).
template <int kTopThreads, int N = kTileCand, bool SORTED = true>
__device__ __forceinline__ void top_finish(uint64_t (&a)[N], int32_t nfeas, int32_t j,
                                           uint64_t* __restrict__ topk, int32_t* __restrict__ topk_cnt,
                                           int32_t* __restrict__ topk_complete, uint64_t* __restrict__ xsend,
                                           uint64_t* tclk = nullptr) {
  constexpr int kTopWaves = kTopThreads / 64;
  constexpr int kTopSlots = (kTopWaves * kTopT + 63) / 64;   // block-merge entries per lane
  __shared__ uint64_t s_list[kTopWaves][kTopT];
  __shared__ int32_t s_cnt[kTopWaves], s_complete[kTopWaves];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // ---- the pod's top-T by threshold ----------------------------------------
  // Provability: a lane that had more feasible nodes than it kept hides keys
  // below its last kept key, so every key >= thr (the largest such key over
  // the block; 0 when no lane overflowed) is in the exact order.  Pruning:
  // the T-th largest of the waves' maxima, L, is <= the T-th largest key, so
  // the pod's top-T lies among the kept keys >= cut = max(thr, L).  Those
  // candidates (a prefix of each lane's sorted list) go to LDS by prefix
  // sums, and one wave ranks them: no serial extraction rounds.  A block
  // with more than 64 candidates (a long L tie region cannot happen: keys
  // are unique) takes the round-by-round extraction below.
  {
    __shared__ uint64_t s_wmax[kTopWaves], s_wthr[kTopWaves];
    __shared__ int32_t s_wc[kTopWaves], s_wf[kTopWaves];
    __shared__ uint64_t s_cand[64];
    uint64_t lmax = a[0];
    if constexpr (!SORTED) {
#pragma unroll
      for (int q = 1; q < N; q++) lmax = umax64(lmax, a[q]);
    }
    const uint64_t u = SORTED && nfeas > N ? a[N - 1] : 0;
    const uint64_t wthr = wave_max_u64_dpp(u);
    const uint64_t wmax = wave_max_u64_dpp(lmax);
    const int32_t fsum = (int32_t)wave_sum_u32_dpp((uint32_t)nfeas);
    if (lane == 0) {
      s_wmax[wv] = wmax;
      s_wthr[wv] = wthr;
      s_wf[wv] = fsum;
    }
    lds_barrier();
#ifdef KSIM_TC_CLOCKS
    if (tclk && threadIdx.x == 0) tclk[0] = __builtin_amdgcn_s_memrealtime();
#endif
    uint64_t thr = 0, mine_w = lane < kTopWaves ? s_wmax[lane] : 0;
    int32_t total = 0, rank = 0;
#pragma unroll
    for (int w = 0; w < kTopWaves; w++) {
      const uint64_t o = s_wmax[w];               // LDS broadcast
      thr = umax64(thr, s_wthr[w]);
      total += s_wf[w];
      rank += o > mine_w;
    }
    const uint64_t at = __ballot(lane < kTopWaves && mine_w != 0 && rank == kTopT - 1);
    const uint64_t L = at ? readlane_u64(mine_w, __builtin_ctzll(at)) : 0;
    const uint64_t cut = umax64(umax64(thr, L), 1);   // keys are nonzero
    int32_t cl = 0;
#pragma unroll
    for (int q = 0; q < N; q++) cl += a[q] >= cut;   // SORTED: a prefix
    // inclusive wave scan of cl in [0, N]: by its bits' ballots
    constexpr int kBits = N < 4 ? 2 : N < 8 ? 3 : 4;
    static_assert(N < 16, "four ballots cover the count");
    int32_t pre = cl, wsum = 0;
#pragma unroll
    for (int bit = 0; bit < kBits; bit++) {
      const uint64_t cb = __ballot(cl & (1 << bit));
      pre += (int32_t)mask_below(cb) << bit;
      wsum += __popcll(cb) << bit;
    }
    if (lane == 0) s_wc[wv] = wsum;
    lds_barrier();
#ifdef KSIM_TC_CLOCKS
    if (tclk && threadIdx.x == 0) tclk[1] = __builtin_amdgcn_s_memrealtime();
#endif
    int32_t off = 0, C = 0;
#pragma unroll
    for (int w = 0; w < kTopWaves; w++) {
      const int32_t x = s_wc[w];
      off += w < wv ? x : 0;
      C += x;
    }
    if (C <= 64) {                                 // block-uniform
      const int32_t base_i = off + pre - cl;
      if constexpr (SORTED) {
#pragma unroll
        for (int q = 0; q < N; q++)
          if (q < cl) s_cand[base_i + q] = a[q];
      } else {
        int32_t w = base_i;
#pragma unroll
        for (int q = 0; q < N; q++)
          if (a[q] >= cut) s_cand[w++] = a[q];
      }
      lds_barrier();
#ifdef KSIM_TC_CLOCKS
      if (tclk && threadIdx.x == 0) tclk[2] = __builtin_amdgcn_s_memrealtime();
      if (tclk && threadIdx.x == 0) tclk[3] = C;
#endif
      if (wv != 0) return;
      const uint64_t c0 = lane < C ? s_cand[lane] : 0;
      int32_t r = 0;
      for (int j = 0; j < C; j++) r += readlane_u64(c0, j) > c0;   // keys are unique: ranks are distinct
      const int32_t n_out = C < kTopT ? C : kTopT;
      if (lane < C && r < kTopT) topk[(size_t)j * kTopT + r] = c0;
      if (lane >= n_out && lane < kTopT) topk[(size_t)j * kTopT + lane] = 0;
      const int32_t cmp = (thr == 0 && total <= kTopT) ? 1 : 0;
      if (lane == 0) {
        topk_cnt[j] = n_out;
        topk_complete[j] = cmp;
      }
      if (xsend) {                               // sharded: this shard's record for the all-gather
        uint64_t* x = xsend + (size_t)j * kXRec;
        if (lane < C && r < kTopT) x[r] = c0;
        if (lane >= n_out && lane < kTopT) x[lane] = 0;
        if (lane == 0) x[kTopT] = (uint64_t)(uint32_t)n_out | ((uint64_t)cmp << 32);
      }
      return;
    }
  }
  // the wave's provable top-T prefix (lane t keeps key t)
  uint64_t mine = 0;
  int32_t cnt = 0, complete = 0, popped = 0;
  for (int t = 0; t < kTopT; t++) {
    uint64_t lm = a[0];
    if constexpr (!SORTED) {
#pragma unroll
      for (int q = 1; q < N; q++) lm = umax64(lm, a[q]);
    }
    const uint64_t m = wave_max_u64_hi(lm);
    if (m == 0) { complete = 1; break; }
    if (lane == t) mine = m;
    cnt = t + 1;
    bool stop = false;
    if constexpr (SORTED) {
      if (a[0] == m) {                            // keys are unique (the node is in the key)
#pragma unroll
        for (int q = 0; q + 1 < N; q++) a[q] = a[q + 1];
        a[N - 1] = 0;
        stop = ++popped == N && nfeas > N;
      }
    } else {
#pragma unroll
      for (int q = 0; q < N; q++)
        if (a[q] == m) a[q] = 0;
    }
    if (__ballot(stop)) break;
  }
  if (lane < kTopT) s_list[wv][lane] = lane < cnt ? mine : 0;
  if (lane == 0) {
    s_cnt[wv] = cnt;
    s_complete[wv] = complete;
  }
  lds_barrier();
  if (wv != 0) return;
  // block merge: entry x = w * kTopT + e sits in lane x % 64, slot x / 64
  uint64_t key[kTopSlots], last = 0;
  bool incomplete = false;
#pragma unroll
  for (int q = 0; q < kTopSlots; q++) {
    const int x = q * 64 + lane, w = x / kTopT, e = x % kTopT;
    key[q] = 0;
    if (w < kTopWaves) {
      const int32_t n = s_cnt[w];
      if (e < n) key[q] = s_list[w][e];
      if (!s_complete[w] && n > 0 && e == n - 1) last = umax64(last, key[q]);
      if (!s_complete[w] && e == 0) incomplete = true;
    }
  }
  const uint64_t thr = wave_max_u64_dpp(last);   // the largest "last listed key" of an incomplete wave
  const bool all_complete = __ballot(incomplete) == 0;
  int32_t nvalid = 0;
#pragma unroll
  for (int q = 0; q < kTopSlots; q++) {
    if (key[q] < thr) key[q] = 0;                // not provably in the pod's order
    nvalid += __popcll(__ballot(key[q] != 0));
  }
  uint64_t out = 0;
  int32_t n_out = 0;
  for (int t = 0; t < kTopT; t++) {
    uint64_t best = key[0];
#pragma unroll
    for (int q = 1; q < kTopSlots; q++) best = umax64(best, key[q]);
    const uint64_t m = wave_max_u64_hi(best);
    if (m == 0) break;
    if (lane == t) out = m;
    n_out = t + 1;
#pragma unroll
    for (int q = 0; q < kTopSlots; q++)
      if (key[q] == m) key[q] = 0;
  }
  const int32_t cmp = (all_complete && nvalid <= kTopT) ? 1 : 0;
  if (lane < kTopT) topk[(size_t)j * kTopT + lane] = lane < n_out ? out : 0;
  if (lane == 0) {
    topk_cnt[j] = n_out;
    topk_complete[j] = cmp;
  }
  if (xsend) {                                   // sharded: this shard's record for the all-gather
    uint64_t* x = xsend + (size_t)j * kXRec;
    if (lane < kTopT) x[lane] = lane < n_out ? out : 0;
    if (lane == 0) x[kTopT] = (uint64_t)(uint32_t)n_out | ((uint64_t)cmp << 32);
  }
}

// The generic (non-FAST) keys of pod j = pi - cursor over the block's nodes:
// static filters, the resource key, and for kPodNormVaries pods the
// normalized TaintToleration / NodeAffinity parts.  ov(row) adds whatever the
// caller knows the snapshot lacks (the deferred commit's overlay); k_batch_top
// passes a no-op.
template <int kTopThreads, typename Ov>
__device__ __forceinline__ void generic_keys(const DevCluster& c, const DevPods& P, const ksim_profile& prof,
                                             const BatchProg& bp, const ksim_pod& p, int32_t pi, int32_t j,
                                             int64_t seq, bool trivial, int64_t* __restrict__ pnorm,
                                             uint64_t (&a)[kTileCand], int32_t& nfeas, Ov&& ov) {
  // kPodNormVaries: a first pass takes DefaultNormalizeScore's maxima of the
  // pod's TaintToleration / NodeAffinity raw scores over its S0-feasible
  // nodes (P100: every feasible node is scored), the keys then carry the
  // normalized scores (norm_part)
  const bool normv = (P.bflags[pi] & kPodNormVaries) != 0;   // block-uniform
  // a static class (DevPods::stab): the static verdict and raw scores are one
  // word per node, the row is the resource columns, and on a run_fast cluster
  // the key takes the FAST arithmetic (block-uniform)
  const int32_t scls = P.stab ? P.sclass[pi] : -1;
  const uint64_t* srow = scls >= 0 ? P.stab + (size_t)scls * c.n : nullptr;
  const bool fk = srow && P.stab_fast;
  const uint64_t hseed = prof.tiebreak_seed ^ ((uint64_t)seq << 20);
  auto tkey = [&](const NodeRow& r) -> uint64_t {   // table classes: the key of a row that passed
    if (fk) {
      const FastProg bq = fast_prog(bp);
      const uint32_t o8 = (uint32_t)r.node << 3;
      return dyn_key_fast(bq, fast_pod_fields(p), r, ld_off(c.inv_cpu, o8), ld_off(c.inv_mem, o8), hseed,
                          c.base + r.node);
    }
    return dyn_key(prof, bp, p, r, c.n_scalar, seq, c.base, c.fit_ignore);
  };
  NormRaw mx{0, 0};
  if (normv) {
    NormAcc acc;
    if (srow) {
#pragma unroll 1
      for (int32_t node = c.eval_lo + threadIdx.x; node < c.eval_hi; node += kTopThreads) {
        NodeRow r = load_res_row(c, node);
        ov(r);
        const uint64_t w = srow[node];
        if (stab_pass(w) && tkey(r)) acc.take(stab_raw(w, P, p));
      }
    } else {
#pragma unroll 1
      for (int32_t node = c.eval_lo + threadIdx.x; node < c.eval_hi; node += kTopThreads) {
        NodeRow r = load_row(c, node);
        ov(r);
        if (static_filters_pass(c, P, bp, p, r) && dyn_key(prof, bp, p, r, c.n_scalar, seq, c.base, c.fit_ignore))
          acc.take(norm_raw(c, P, p, r));
      }
    }
    mx = norm_maxima<kTopThreads>(acc, pnorm, j);
  }
  auto insert = [&](uint64_t kk) {
    nfeas += kk != 0;
    a[3] = umax64(a[3], kk);
    cswap_desc(a[2], a[3]);
    cswap_desc(a[1], a[2]);
    cswap_desc(a[0], a[1]);
  };
  if (srow) {
#pragma unroll 1
    for (int32_t node = c.eval_lo + threadIdx.x; node < c.eval_hi; node += kTopThreads) {
      NodeRow r = load_res_row(c, node);
      ov(r);
      const uint64_t w = srow[node];
      uint64_t kk = stab_pass(w) ? tkey(r) : 0;
      if (normv && kk) kk += (uint64_t)norm_part(bp, stab_raw(w, P, p), mx) << 44;
      insert(kk);
    }
    return;
  }
#pragma unroll 1
  for (int32_t node = c.eval_lo + threadIdx.x; node < c.eval_hi; node += kTopThreads) {
    uint64_t kk = 0;
    {
      NodeRow r = trivial && !normv ? load_res_row(c, node) : load_row(c, node);
      ov(r);
      if (trivial || static_filters_pass(c, P, bp, p, r)) kk = dyn_key(prof, bp, p, r, c.n_scalar, seq, c.base, c.fit_ignore);
      if (normv && kk) kk += (uint64_t)norm_part(bp, norm_raw(c, P, p, r), mx) << 44;
    }
    insert(kk);
  }
}

// The FAST keys of a static class's pod (STAB runs: every pod of the run has
// a class, the cluster meets run_fast's conditions): the FAST key, masked by
// the class's static verdict, plus for kPodNormVaries pods the normalized
// part (norm_part_fast) over the maxima of a first pass.  ov(row): as for
// generic_keys.
// KEEP: the range fits kKeepPerLane nodes per lane, every key stays in ak[]
// (node order), and a[] is not used.
template <int kTopThreads, bool DEF, bool KEEP, typename Ov>
__device__ __forceinline__ void stab_fast_keys(const DevCluster& c, const DevPods& P, const BatchProg& bp,
                                               const FastProg& bq, const ksim_pod& pf, int32_t pi, int32_t j,
                                               uint64_t hseed, int64_t* __restrict__ pnorm, uint64_t (&a)[kTileCand],
                                               uint64_t (&ak)[kKeepPerLane], int32_t& nfeas, Ov&& ov) {
  const uint64_t* srow = P.stab + (size_t)P.sclass[pi] * c.n;
  const bool normv = (P.bflags[pi] & kPodNormVaries) != 0;   // block-uniform
  const ksim_pod& pp = P.pods[pi];                           // its preferred terms (stab_raw)
  auto key = [&](int32_t node, uint64_t& w) -> uint64_t {
    const uint32_t o8 = (uint32_t)node << 3;
    NodeRow r = load_res_row_off(c, node);
    const double ic = ld_off(c.inv_cpu, o8), im = ld_off(c.inv_mem, o8);
    w = ld_off(srow, o8);
    ov(r);
    const uint64_t k = dyn_key_fast_t<DEF>(bq, pf, r, ic, im, hseed, c.base + node);
    return stab_pass(w) ? k : 0;
  };
  if constexpr (KEEP) {
    // the keys and static words in registers; for kPodNormVaries pods the
    // maxima over them, then the normalized parts added in place
    uint64_t wk[kKeepPerLane];
    NormAcc acc;
#pragma unroll
    for (int q = 0; q < kKeepPerLane; q++) {
      ak[q] = 0;
      wk[q] = 0;
    }
#pragma unroll
    for (int q = 0; q < kKeepPerLane; q++) {
      if (c.eval_lo + q * kTopThreads >= c.eval_hi) break;   // block-uniform
      const int32_t node = c.eval_lo + (int32_t)threadIdx.x + q * kTopThreads;
      if (node < c.eval_hi) {
        uint64_t w;
        const uint64_t k = key(node, w);
        ak[q] = k;
        wk[q] = w;
        if (normv && k) acc.take(stab_raw(w, P, pp));
      }
    }
    if (normv) {                                 // block-uniform
      const NormRaw mx = norm_maxima<kTopThreads>(acc, pnorm, j);
      const double y_tt = recip_or_zero(mx.tt), y_na = recip_or_zero(mx.na);
#pragma unroll
      for (int q = 0; q < kKeepPerLane; q++)
        if (ak[q]) ak[q] += (uint64_t)norm_part_fast(bp, stab_raw(wk[q], P, pp), mx, y_tt, y_na) << 44;
    }
#pragma unroll
    for (int q = 0; q < kKeepPerLane; q++) nfeas += ak[q] != 0;
    return;
  }
  // kPodNormVaries: the first pass keeps each node's key (without the
  // normalized part) in LDS when the range fits, so the second pass only adds
  // that part (each slot is written and read by the same thread: no barrier)
  constexpr int32_t kKeep = 8192;
  __shared__ uint64_t s_keep[kKeep];
  const bool keep = normv && c.eval_hi - c.eval_lo <= kKeep;   // block-uniform
  NormRaw mx{0, 0};
  double y_tt = 0, y_na = 0;
  if (normv) {
    NormAcc acc;
#pragma unroll 1
    for (int32_t node = c.eval_lo + threadIdx.x; node < c.eval_hi; node += kTopThreads) {
      uint64_t w;
      const uint64_t k = key(node, w);
      if (keep) s_keep[node - c.eval_lo] = k;
      if (k) acc.take(stab_raw(w, P, pp));
    }
    mx = norm_maxima<kTopThreads>(acc, pnorm, j);
    y_tt = recip_or_zero(mx.tt);
    y_na = recip_or_zero(mx.na);
  }
#pragma unroll 1
  for (int32_t node = c.eval_lo + threadIdx.x; node < c.eval_hi; node += kTopThreads) {
    uint64_t w;
    uint64_t k;
    if (keep) {
      k = s_keep[node - c.eval_lo];
      w = ld_off(srow, (uint32_t)node << 3);
    } else {
      k = key(node, w);
    }
    if (normv && k) k += (uint64_t)norm_part_fast(bp, stab_raw(w, P, pp), mx, y_tt, y_na) << 44;
    nfeas += k != 0;
    a[3] = umax64(a[3], k);
    cswap_desc(a[2], a[3]);
    cswap_desc(a[1], a[2]);
    cswap_desc(a[0], a[1]);
  }
}

// STAB (FAST only): a static-class run (stab_fast_keys).  DEF (FAST only): the
// default profile's key shape compiled in (fast_def).  KEEP (STAB only): every
// key of a lane kept (node ranges of at most kKeepPerLane * kTopThreads).
template <bool FAST, int kTopThreads, bool STAB = false, bool DEF = false, bool KEEP = false>
__global__ __launch_bounds__(kTopThreads) void k_batch_top(DevCluster c, DevPods P,
                                                           const ksim_profile* __restrict__ prof_p,
                                                           const BatchProg* __restrict__ bp_p,
                                                           const DevState* __restrict__ st,
                                                           uint64_t* __restrict__ topk, int32_t* __restrict__ topk_cnt,
                                                           int32_t* __restrict__ topk_complete,
                                                           uint64_t* __restrict__ xsend, int64_t* __restrict__ pnorm) {
  constexpr int kTopWaves = kTopThreads / 64;
  constexpr int kTopSlots = (kTopWaves * kTopT + 63) / 64;   // block-merge entries per lane
  static_assert(kTopSlots <= 4 && kTileCand == 4, "k_batch_top geometry");
  const ksim_profile& prof = *prof_p;   // device copies (ksim_set_profile): graphs outlive a weight change
  const BatchProg& bp = *bp_p;
  const int32_t base = st->cursor;
  const int32_t j = blockIdx.x;
  const int32_t pi = base + j;
  if (pi >= min(st->end, base + kBatchPods)) return;        // block-uniform
  const ksim_pod& p = P.pods[pi];
  const bool trivial = (P.bflags[pi] & kBatchStaticTrivial) != 0;   // block-uniform
  const int64_t seq = st->pod_seq + j;
  const uint64_t hseed = prof.tiebreak_seed ^ ((uint64_t)seq << 20);
  uint64_t a[kTileCand] = {0, 0, 0, 0};        // the lane's best keys, descending
  uint64_t ak[kKeepPerLane];                    // KEEP: every key of the lane, node order
  int32_t nfeas = 0;
  static_assert(!KEEP || STAB, "KEEP: static-class runs");
  if constexpr (FAST) {
    // the loop-invariant key inputs in registers (SGPRs): the profile's batch
    // program and the pod's request fields, loaded once
    const FastProg bq = fast_prog(bp);
    const ksim_pod pf = fast_pod_fields(p);
    if constexpr (STAB) {
      stab_fast_keys<kTopThreads, DEF, KEEP>(c, P, bp, bq, pf, pi, j, hseed, pnorm, a, ak, nfeas, [](NodeRow&) {});
    } else {
#pragma unroll 1
    for (int32_t node = c.eval_lo + threadIdx.x; node < c.eval_hi; node += kTopThreads) {
      const NodeRow r = load_res_row_off(c, node);
      const double ic = ld_off(c.inv_cpu, (uint32_t)node << 3), im = ld_off(c.inv_mem, (uint32_t)node << 3);
      __builtin_amdgcn_sched_barrier(0);      // the row in flight before the key
      const uint64_t k = dyn_key_fast_t<DEF>(bq, pf, r, ic, im, hseed, c.base + node);
      nfeas += k != 0;
      a[3] = umax64(a[3], k);
      cswap_desc(a[2], a[3]);
      cswap_desc(a[1], a[2]);
      cswap_desc(a[0], a[1]);
    }
    }
  }
  if constexpr (!FAST)                        // the generic loop is not compiled into FAST kernels
    generic_keys<kTopThreads>(c, P, prof, bp, p, pi, j, seq, trivial, pnorm, a, nfeas, [](NodeRow&) {});
  if constexpr (KEEP)
    top_finish<kTopThreads, kKeepPerLane, false>(ak, nfeas, j, topk, topk_cnt, topk_complete, xsend);
  else
    top_finish<kTopThreads>(a, nfeas, j, topk, topk_cnt, topk_complete, xsend);
}

// Sharded: merge the R shard records of pod j (all-gathered, [R][B][kXRec])
// into the pod's global top-T.  Entry x = s * T + e (shard s, entry e) sits in
// lane x % 64, slot x / 64.  A key is provably in the global order if it is
// >= the last listed key of every incomplete shard (every key a shard did not
// list is below its last listed one); the list is complete when every shard
// was and nothing was dropped.
__global__ __launch_bounds__(256) void k_batch_gmerge(const DevState* __restrict__ st,
                                                      const uint64_t* __restrict__ xrecv, int32_t world,
                                                      uint64_t* __restrict__ topk, int32_t* __restrict__ topk_cnt,
                                                      int32_t* __restrict__ topk_complete) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int32_t j = blockIdx.x * 4 + w;
  const int32_t base = st->cursor;
  if (base + j >= min(st->end, base + kBatchPods)) return;   // wave-uniform
  uint64_t key[kGmergeSlots], last = 0;
  bool valid[kGmergeSlots];
  bool incomplete_shard = false;
#pragma unroll
  for (int q = 0; q < kGmergeSlots; q++) {
    const int x = q * 64 + lane, sh = x / kTopT, e = x % kTopT;
    key[q] = 0;
    if (sh < world) {
      const uint64_t* rec = xrecv + ((size_t)sh * kBatchPods + j) * kXRec;
      const uint64_t meta = rec[kTopT];
      const int32_t cnt = (int32_t)(uint32_t)meta;
      const bool complete = (meta >> 32) != 0;
      if (e < cnt) key[q] = rec[e];
      if (!complete && cnt > 0 && e == cnt - 1) last = umax64(last, key[q]);
      if (!complete && e == 0) incomplete_shard = true;
    }
  }
  const uint64_t thr = wave_max_u64_dpp(last);     // the largest "last listed key" of an incomplete shard
  const bool all_complete = __ballot(incomplete_shard) == 0;
  int nvalid = 0;
  uint64_t vm[kGmergeSlots];
#pragma unroll
  for (int q = 0; q < kGmergeSlots; q++) {
    valid[q] = key[q] != 0 && key[q] >= thr;
    vm[q] = __ballot(valid[q]);
    nvalid += __popcll(vm[q]);
  }
  // rank of each valid key among the valid keys (keys are unique: one per node)
#pragma unroll
  for (int q = 0; q < kGmergeSlots; q++) {
    int rank = 0;
#pragma unroll
    for (int q2 = 0; q2 < kGmergeSlots; q2++)
      for (int l = 0; l < 64; l++) {
        const uint64_t o = readlane_u64(key[q2], l);
        if (((vm[q2] >> l) & 1ull) && o > key[q]) rank++;
      }
    if (valid[q] && rank < kTopT) topk[(size_t)j * kTopT + rank] = key[q];
  }
  const int n = nvalid < kTopT ? nvalid : kTopT;
  if (lane >= n && lane < kTopT) topk[(size_t)j * kTopT + lane] = 0;
  if (lane == 0) {
    topk_cnt[j] = n;
    topk_complete[j] = (all_complete && nvalid <= kTopT) ? 1 : 0;
  }
}

// Block j: pod j's pair keys on the guesses gk of threads k < j, max to pmax[j].
// FAST with pj / pk: pod j's and pod k's fields loaded by the caller.
// Generic runs also flag pod j in pinv[j] when every S0-feasible node that
// held one of its normalization maxima (kPodNormVaries) has left its feasible
// set: the maximum, and so its S0 keys, no longer hold, and the batch commits
// only the pods before it.
template <bool FAST, bool STAB = false, bool DEF = false>
__device__ __forceinline__ void pairs_block(const DevCluster& c, const DevPods& P, const ksim_profile& prof,
                                            const BatchProg& bp, const DevState* __restrict__ st, uint64_t gk,
                                            int32_t nchain, uint64_t* s_wmax, uint64_t* __restrict__ pmax,
                                            const ksim_pod* pj = nullptr, const ksim_pod* pk = nullptr,
                                            const int64_t* __restrict__ pnorm = nullptr,
                                            int32_t* __restrict__ pinv = nullptr, int32_t* s_winv = nullptr) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j = blockIdx.x, k = tid;
  const int32_t base = st->cursor;
  const int64_t seq0 = st->pod_seq;
  constexpr bool kInv = !FAST || STAB;               // pinv flags (kPodNormVaries pods)
  if (j >= nchain) {                                 // block-uniform
    if (tid == 0) {
      pmax[j] = 0;
      if (kInv) pinv[j] = 0;
    }
    return;
  }
  uint64_t v = 0;
  bool lost_t = false, lost_a = false;               // guess k held a maximum of pod j and left its feasible set
  if (k < j) {
    const int32_t local = gk ? key_node(gk) - c.base : -1;
    if (local >= 0 && local < c.n) {
      const ksim_pod& p = P.pods[base + j];
      if constexpr (FAST && STAB) {
        const int32_t bf = P.bflags[base + j];
        const bool normv = (bf & kPodNormVaries) != 0;
        const uint64_t w = P.stab[(size_t)P.sclass[base + j] * c.n + local];
        const double ic = c.inv_cpu[local], im = c.inv_mem[local];
        const uint64_t hseed = prof.tiebreak_seed ^ ((uint64_t)(seq0 + j) << 20);
        NodeRow r = load_res_row(c, local);
        const bool feas0 =
            normv && stab_pass(w) && dyn_key_fast_t<DEF>(fast_prog(bp), *pj, r, ic, im, hseed, c.base + local) != 0;
        row_add_pod(r, *pk, 1);
        v = stab_pass(w) ? dyn_key_fast_t<DEF>(fast_prog(bp), *pj, r, ic, im, hseed, c.base + local) : 0;
        if (normv && (v || feas0)) {
          const NormRaw mx{pnorm[4 * j], pnorm[4 * j + 1]};
          if (v) {
            v += (uint64_t)norm_part_fast(bp, stab_raw(w, P, p), mx, recip_or_zero(mx.tt), recip_or_zero(mx.na)) << 44;
          } else {
            const NormRaw x = stab_raw(w, P, p);
            lost_t = mx.tt > 0 && x.tt == mx.tt;
            lost_a = mx.na > 0 && x.na == mx.na;
          }
        }
      } else if constexpr (FAST) {
        NodeRow r = load_res_row(c, local);
        row_add_pod(r, pk ? *pk : P.pods[base + k], 1);
        v = dyn_key_fast_t<DEF>(fast_prog(bp), pj ? *pj : p, r, c.inv_cpu[local], c.inv_mem[local],
                         prof.tiebreak_seed ^ ((uint64_t)(seq0 + j) << 20), c.base + local);
      } else {
        const int32_t bf = P.bflags[base + j];
        const bool normv = (bf & kPodNormVaries) != 0;
        const int32_t scls = P.stab ? P.sclass[base + j] : -1;   // block-uniform (generic_keys)
        const uint64_t w = scls >= 0 ? P.stab[(size_t)scls * c.n + local] : 0;
        NodeRow r = scls >= 0 ? load_res_row(c, local) : load_row(c, local);
        auto key = [&](const NodeRow& x) -> uint64_t {
          if (scls >= 0 && P.stab_fast)
            return dyn_key_fast(bp, fast_pod_fields(p), x, c.inv_cpu[local], c.inv_mem[local],
                                prof.tiebreak_seed ^ ((uint64_t)(seq0 + j) << 20), c.base + local);
          return dyn_key(prof, bp, p, x, c.n_scalar, seq0 + j, c.base, c.fit_ignore);
        };
        const bool sp = scls >= 0 ? stab_pass(w) : ((bf & kBatchStaticTrivial) || static_filters_pass(c, P, bp, p, r));
        const bool feas0 = normv && sp && key(r) != 0;   // at S0
        row_add_pod(r, P.pods[base + k], 1);
        if (sp) v = key(r);
        if (normv && (v || feas0)) {
          const NormRaw mx{pnorm[4 * j], pnorm[4 * j + 1]};
          const NormRaw x = scls >= 0 ? stab_raw(w, P, p) : norm_raw(c, P, p, r);
          if (v) {
            v += (uint64_t)norm_part(bp, x, mx) << 44;
          } else {
            lost_t = mx.tt > 0 && x.tt == mx.tt;
            lost_a = mx.na > 0 && x.na == mx.na;
          }
        }
      }
    }
  }
  v = wave_max_u64_dpp(v);
  if (lane == 0) s_wmax[wave] = v;
  if (kInv) {                                        // holders lost per wave: TaintToleration | NodeAffinity << 16
    const int32_t nt = __popcll(__ballot(lost_t)), na = __popcll(__ballot(lost_a));
    if (lane == 0) s_winv[wave] = nt | (na << 16);
  }
  lds_barrier();
  if (tid == 0) {
    uint64_t m = 0;
    int32_t lt = 0, la = 0;
    for (int w = 0; w < kBatchPods / 64; w++) {
      m = umax64(m, s_wmax[w]);
      if (kInv) {
        lt += s_winv[w] & 0xffff;
        la += s_winv[w] >> 16;
      }
    }
    pmax[j] = m;
    // a maximum of pod j changes only once every S0-feasible node holding it
    // has left its feasible set (binds only shrink it; the raw scores are static)
    if (kInv) pinv[j] = (lt > 0 && lt >= pnorm[4 * j + 2]) || (la > 0 && la >= pnorm[4 * j + 3]);
  }
}

// The chain and the pair keys in one launch: every block of the pairs grid
// runs the (deterministic) chain itself, thread k ending with pod k's guess in
// a register, so the pairs need no chain launch and no gkey round trip.
// Block 0 also stores the guesses and the prefix length for k_batch_commit.
#if defined(KSIM_CP_CLOCKS) || defined(KSIM_TC_CLOCKS)
__device__ unsigned long long g_cp_dbg[8];
unsigned long long* cp_clock_buffer() {
  void* p = nullptr;
  (void)hipGetSymbolAddress(&p, HIP_SYMBOL(g_cp_dbg));
  return (unsigned long long*)p;
}
#else
unsigned long long* cp_clock_buffer() { return nullptr; }
#endif

// LAZY (deferred-commit batches): a batch with no pods marks its ring slot
// empty (chain_end = -1), so the next launch commits nothing for it.
// R: each pod's list is R slice records (the node-stationary evaluation).
// DEF (FAST pairs): the default profile's key shape compiled in.
template <bool FAST, bool LAZY = false, bool STAB = false, int R = 1, bool DEF = false>
__global__ __launch_bounds__(kBatchPods) void k_batch_chain_pairs(DevCluster c, DevPods P,
                                                                  const ksim_profile* __restrict__ prof_p,
                                                                  const BatchProg* __restrict__ bp_p,
                                                                  const DevState* __restrict__ st,
                                                                  const uint64_t* __restrict__ topk,
                                                                  const int32_t* __restrict__ topk_cnt,
                                                                  const int32_t* __restrict__ topk_complete,
                                                                  uint64_t* __restrict__ gkey,
                                                                  int32_t* __restrict__ chain_end,
                                                                  uint64_t* __restrict__ pmax,
                                                                  const int64_t* __restrict__ pnorm,
                                                                  int32_t* __restrict__ pinv) {
  __shared__ ChainLds L;
  __shared__ uint64_t s_wmax[kBatchPods / 64];
  __shared__ int32_t s_winv[kBatchPods / 64];
  // FAST: pod j's and pod k's request fields in flight during the chain
  ksim_pod pj, pk;
  if constexpr (FAST) {
    const int32_t base = st->cursor, nb = min(kBatchPods, st->end - base);
    const int32_t j = blockIdx.x, k = threadIdx.x;
    if (j < nb) pj = fast_pod_fields(P.pods[base + j]);
    if (k < nb) pk = fast_pod_fields(P.pods[base + k]);
  }
  uint64_t gk;
  int32_t nchain;
#ifdef KSIM_CP_CLOCKS
  // phase clocks of block 0 (KSIM_CP_CLOCKS builds, tools/cp_clocks.py): the
  // chain's setup / rounds / epilogue (dbg 0-2, launches 3, rounds 4), the
  // whole block (dbg 5)
  const uint64_t t_in = __builtin_amdgcn_s_memrealtime();
  unsigned long long* dbgc = blockIdx.x == 0 ? g_cp_dbg : nullptr;
#else
  unsigned long long* dbgc = nullptr;
#endif
  if (!chain_block<R>(L, st, topk, topk_cnt, topk_complete, &gk, &nchain, dbgc, kBatchPods, c.n_total)) {
    if (LAZY && blockIdx.x == 0 && threadIdx.x == 0) *chain_end = -1;
    return;
  }
  if (blockIdx.x == 0) {
    const int32_t nb = min(kBatchPods, st->end - st->cursor);
    if ((int)threadIdx.x < nb) gkey[threadIdx.x] = gk;
    if (threadIdx.x == 0) *chain_end = nchain;
  }
  pairs_block<FAST, STAB, DEF>(c, P, *prof_p, *bp_p, st, gk, nchain, s_wmax, pmax, FAST ? &pj : nullptr,
                          FAST ? &pk : nullptr, pnorm, pinv, s_winv);
#ifdef KSIM_CP_CLOCKS
  if (dbgc && threadIdx.x == 0) atomicAdd(&dbgc[5], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - t_in));
#endif
}

__global__ __launch_bounds__(kBatchPods) void k_batch_commit(DevCluster c, DevPods P, DevState* __restrict__ st,
                                                             const uint64_t* __restrict__ gkey,
                                                             const int32_t* __restrict__ chain_end,
                                                             const uint64_t* __restrict__ pmax,
                                                             int32_t* __restrict__ chosen_out,
                                                             const int32_t* __restrict__ pinv) {
  __shared__ int32_t s_istar, s_sched, s_unsched;
  const uint64_t g = gkey[threadIdx.x], m = pmax[threadIdx.x];   // in flight with the state loads
  const int32_t inv = pinv ? pinv[threadIdx.x] : 0;
  const int32_t nchain = *chain_end;
  if (min(kBatchPods, st->end - st->cursor) <= 0) return;
  batch_commit(c, P, st, g, m, pmax, nchain, chosen_out, &s_istar, &s_sched, &s_unsched, nullptr, pinv ? &inv : nullptr);
}

// ---- static classes (DevPods::stab) ------------------------------------------
// Row cls of the table: the static verdict and raw normalized scores of the
// class's representative pod rep[cls] on every node of the snapshot (grid
// x: nodes, y: classes).  Pure functions of the pod's static fields and the
// node's flags, taints and labels: built once per (pods, cluster, profile).
__global__ __launch_bounds__(256) void k_static_table(DevCluster c, DevPods P, const BatchProg* __restrict__ bp_p,
                                                      const int32_t* __restrict__ rep, uint64_t* __restrict__ stab) {
  const int32_t node = blockIdx.x * 256 + threadIdx.x;
  if (node >= c.n) return;
  const ksim_pod& p = P.pods[rep[blockIdx.y]];
  const NodeRow r = load_row(c, node);
  const bool pass = static_filters_pass(c, P, *bp_p, p, r);
  stab[(size_t)blockIdx.y * c.n + node] = stab_word(pass, count_intolerable_prefer(c, p, r), pref_term_mask(c, P, p, node));
}

void launch_static_table(const LaunchArgs& a, const int32_t* rep, int32_t n_cls, uint64_t* stab, hipStream_t stream) {
  if (n_cls <= 0 || a.c.n <= 0) return;
  k_static_table<<<dim3((a.c.n + 255) / 256, n_cls), 256, 0, stream>>>(a.c, a.P, a.dbp, rep, stab);
}

// ---- deferred commit: batch i-1's commit inside batch i's evaluation launch -----
// (ksim_internal.h "deferred-commit FAST batches").  Every block recomputes
// batch i-1's cut from its ring slot (the first pod whose pair maximum beats
// its guess, as batch_commit), so every block knows cursor_i and the nodes
// batch i-1 bound with the requests it bound there: an LDS overlay (a node
// bitmap, and a node -> entry hash for the nodes it marks).  A block keys its
// pod of batch i against X[p ^ 1] + overlay = S_i.  Block b also writes pod
// b's placement and S_i into X[p] at guess b of batches i-1 and i-2 (X[p] held
// S_{i-2}; a guess that was not bound keeps its value, so the superset is
// harmless); block 0 writes the state after the commit to st[p].  FLUSH: no
// evaluation, and slot i is marked empty.
constexpr int kLazyHash = 1 << kLazyHashBits;
constexpr int kLazyBitWords = kLazyMaxNodes / 32;
static_assert(kLazyHash >= 4 * kBatchPods && kBatchPods <= 1024, "overlay hash / block geometry");
// Clusters of at most kLazyDirect nodes index the overlay by node id (an int16
// entry per node, 64 KB of LDS): one LDS read per node instead of the bitmap
// test and the hash probe.
constexpr int kLazyDirect = 1 << 15;
static_assert(kBatchPods < 32767, "overlay entries are int16");

__device__ __forceinline__ uint32_t lazy_hash(int32_t node) {
  return ((uint32_t)node * 2654435761u) >> (32 - kLazyHashBits);
}

// the request fields a FAST pod's key reads
struct PodReq {
  int64_t cpu, mem, eph, nzc, nzm;
};

// DEF: the FAST key with the default profile's shape compiled in (fast_def).
// KEEP: the local node range is at most kKeepPerLane * 1024 nodes, so every
// lane keeps all of its keys (no insertion network; top_finish unsorted).
// NS: node-stationary blocks on larger ranges: block b keys the kNsPods pods
// kNsPods * (b / kNsSlices) + [0, kNsPods) over node slice b % kNsSlices, so
// a node's row, its overlay delta and the addressing are paid once for
// kNsPods keys; each block writes one list record per pod for its slice (rec
// = pod * kNsSlices + slice: the slice's provable top-T), which
// chain_block<kNsSlices> merges as it loads the pod's list.
constexpr int kNsSlices = 4;
constexpr int kNsPods = 4;
static_assert(kNsSlices == kNsPods && kBatchPods % kNsPods == 0, "NS grid: kBatchPods blocks");
static_assert(kNsSlices <= kMaxListRecords, "NS records: DevScratch::topk holds kMaxListRecords per pod");

// a wave-uniform 64-bit value as such (SGPRs)
__device__ __forceinline__ int64_t uni64(int64_t x) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)x >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

template <bool FLUSH, bool DIRECT, bool DEF = false, bool KEEP = false, bool NS = false>
__global__ __launch_bounds__(1024) void k_batch_top_commit(DevCluster c, DevPods P,
                                                           const ksim_profile* __restrict__ prof_p,
                                                           const BatchProg* __restrict__ bp_p, LazyStep L,
                                                           uint64_t* __restrict__ topk, int32_t* __restrict__ topk_cnt,
                                                           int32_t* __restrict__ topk_complete,
                                                           int32_t* __restrict__ chosen_out,
                                                           uint64_t* __restrict__ xsend) {
  constexpr int kThreads = 1024;
  static_assert(kThreads >= kBatchPods, "one thread per batch entry");
  // s_rq: batch i-1's pod requests, then each bound node's delta; entry
  // kBatchPods stays zero (DIRECT: the entry of every node batch i-1 did not bind)
  __shared__ ResCols s_rq[kBatchPods + 1];
  // pod cur0 + pod0 + t: this block's (first) pod of batch i is t = committed
  __shared__ PodReq s_pc[kBatchPods + (NS ? kNsPods : 1)];
  __shared__ __attribute__((aligned(16))) int16_t s_ent[DIRECT ? kLazyDirect : 1];   // node -> entry
  __shared__ int32_t s_hkey[DIRECT ? 1 : kLazyHash];   // overlay hash: local node or -1
  __shared__ int16_t s_hval[DIRECT ? 1 : kLazyHash];   // ... its entry
  __shared__ uint32_t s_bits[DIRECT ? 1 : kLazyBitWords];   // nodes batch i-1 bound
  __shared__ int32_t s_istar, s_inode, s_sched, s_unsched;
  const int tid = threadIdx.x;
  const int32_t b = blockIdx.x;
  const int32_t pod0 = NS ? (b / kNsSlices) * kNsPods : b;   // the block's first pod (batch i offset)
#ifdef KSIM_TC_CLOCKS
  // phase clocks of every block (KSIM_TC_CLOCKS builds, tools/tc_clocks.py),
  // thread 0's view, summed (see the end of the kernel)
  const uint64_t t_in = __builtin_amdgcn_s_memrealtime();
  uint64_t t_pro = 0, t_loop = 0, tclk[4] = {0, 0, 0, 0}, tp[3] = {0, 0, 0};
#endif
  // batch i-1's slot, batch i-2's guess b and the state batch i-1 started from
  // (independent loads)
  const int32_t e1 = *L.e1, e2 = *L.e2;
  uint64_t g1 = 0, m1 = 0, g2 = 0;
  if (tid < kBatchPods) {
    g1 = L.g1[tid];
    m1 = L.m1[tid];
  }
  if (tid == b) g2 = L.g2[b];
  const int32_t cur0 = L.st_in->cursor, end = L.st_in->end;
  const int64_t seq0 = L.st_in->pod_seq;
  // every pod record the commit may need, before the cut is known (they only
  // depend on cur0): pod tid of batch i-1 (its request, kept if committed) and
  // the candidates cur0 + pod0 + t for this block's pods of batch i
  ResCols rq{0, 0, 0, 0, 0, 0};
  for (int x = tid; x < 2 * kBatchPods + (NS ? kNsPods : 1); x += kThreads) {
    const int32_t q = x < kBatchPods ? cur0 + x : cur0 + pod0 + (x - kBatchPods);
    if (q < end) {
      const ksim_pod& y = P.pods[q];
      if (x < kBatchPods) {
        rq = ResCols{y.req_cpu, y.req_mem, y.req_eph, y.nz_cpu, y.nz_mem, 1};
      } else {
        s_pc[x - kBatchPods] = PodReq{y.req_cpu, y.req_mem, y.req_eph, y.nz_cpu, y.nz_mem};
      }
    }
  }
  if constexpr (DIRECT) {
    // every local node's entry = kBatchPods (the zero entry), 4 per store
    const uint64_t fill = 0x0001000100010001ull * (uint64_t)kBatchPods;
    for (int x = tid; x < (c.n + 3) >> 2; x += kThreads) reinterpret_cast<uint64_t*>(s_ent)[x] = fill;
  } else {
    const int nwords = (c.n + 31) >> 5;
    for (int x = tid; x < kLazyHash; x += kThreads) s_hkey[x] = -1;
    for (int x = tid; x < nwords; x += kThreads) s_bits[x] = 0;
  }
  const int32_t nchain = e1 > 0 ? e1 : 0;      // -1: no batch i-1 (run start, a flush, past the end)
  if (tid == 0) {
    s_istar = nchain;
    s_inode = -1;
    s_sched = 0;
    s_unsched = 0;
    s_rq[kBatchPods] = ResCols{0, 0, 0, 0, 0, 0};
  }
  lds_barrier();
#ifdef KSIM_TC_CLOCKS
  tp[0] = __builtin_amdgcn_s_memrealtime();
#endif
  block_first_min(&s_istar, tid < nchain && m1 > g1);   // keys are unique per node: never equal unless 0
  lds_barrier();
#ifdef KSIM_TC_CLOCKS
  tp[1] = __builtin_amdgcn_s_memrealtime();
#endif
  const int32_t istar = s_istar;
  const int32_t committed = istar < nchain ? istar + 1 : nchain;
  if (tid == istar && istar < nchain) s_inode = key_node(m1) - c.base;
  if (tid < committed) s_rq[tid] = rq;
  // this block's pod of batch i
  const int32_t base = cur0 + committed;
  const int32_t pi = base + pod0;
  const bool live = !FLUSH && pi < min(end, base + kBatchPods);   // block-uniform
  lds_barrier();
#ifdef KSIM_TC_CLOCKS
  tp[2] = __builtin_amdgcn_s_memrealtime();
#endif
  const int32_t inode = s_inode;
  // entry tid < i*: its guessed node takes pod tid, and pod i* when i* chose it
  const int32_t gnode = (tid < istar && g1) ? key_node(g1) - c.base : -1;
  if (gnode >= 0) {
    ResCols d = rq;
    if (gnode == inode) {
      const ResCols x = s_rq[istar];              // never overwritten: only entries < i* are
      d.cpu += x.cpu;
      d.mem += x.mem;
      d.eph += x.eph;
      d.nzc += x.nzc;
      d.nzm += x.nzm;
      d.pods += 1;
    }
    s_rq[tid] = d;
    if constexpr (DIRECT) {
      s_ent[gnode] = (int16_t)tid;                // guessed nodes are distinct
    } else {
      atomicOr(&s_bits[gnode >> 5], 1u << (gnode & 31));
      uint32_t h = lazy_hash(gnode);
      while (atomicCAS(&s_hkey[h], -1, gnode) != -1) h = (h + 1) & (kLazyHash - 1);   // guessed nodes are distinct
      s_hval[h] = (int16_t)tid;
    }
  }
  // batch i-1's placements and statistics (k_batch_commit's bookkeeping)
  const int32_t pnode = tid == istar ? inode + c.base : (g1 ? key_node(g1) : -1);
  if (tid == b && tid < committed && chosen_out) chosen_out[cur0 + b] = pnode;
  if (b == 0 && tid < committed) atomicAdd(pnode >= 0 ? &s_sched : &s_unsched, 1);
  // this block's two rows to materialize, loaded ahead of the node loop
  int32_t mn0 = -1, mn1 = -1;
  ResCols mr0{0, 0, 0, 0, 0, 0}, mr1{0, 0, 0, 0, 0, 0};
  if (tid == b) {
    if (b < nchain && g1) mn0 = key_node(g1) - c.base;
    if (b < e2 && g2) mn1 = key_node(g2) - c.base;   // thread b holds g2[b]
    if (mn0 >= 0) mr0 = ResCols{c.req_cpu[mn0], c.req_mem[mn0], c.req_eph[mn0], c.nz_cpu[mn0], c.nz_mem[mn0], c.num_pods[mn0]};
    if (mn1 >= 0) mr1 = ResCols{c.req_cpu[mn1], c.req_mem[mn1], c.req_eph[mn1], c.nz_cpu[mn1], c.nz_mem[mn1], c.num_pods[mn1]};
  }
  lds_barrier();
  // st[p] = st[p ^ 1] with the commit's updates, written whole by one thread
  // of block 0 off the critical path (a wave that is done before the top-T
  // merge): its words loaded together, no store-then-reload chain
  auto update_state = [&]() {
    static_assert(sizeof(DevState) % 8 == 0, "DevState by words");
    constexpr int kWords = (int)(sizeof(DevState) / 8);
    uint64_t w[kWords];
#pragma unroll
    for (int q = 0; q < kWords; q++) w[q] = reinterpret_cast<const uint64_t*>(L.st_in)[q];
    DevState ns;
    __builtin_memcpy(&ns, w, sizeof(ns));
    if (e1 > 0) {
      const int32_t nb = min(kBatchPods, end - cur0);
      ns.cursor = base;
      ns.pod_seq = seq0 + committed;
      ns.scheduled += s_sched;
      ns.unschedulable += s_unsched;
      ns.batches += 1;
      ns.cuts += (committed < nb && istar < nchain ? 1 : 0);
      ns.truncations += (committed < nb && istar >= nchain ? 1 : 0);
      ns.evals += (int64_t)committed * (c.eval_hi - c.eval_lo);
    }
    __builtin_memcpy(w, &ns, sizeof(ns));
#pragma unroll
    for (int q = 0; q < kWords; q++) reinterpret_cast<uint64_t*>(L.st_out)[q] = w[q];
    if (FLUSH) *L.e_self = -1;
  };
  const bool st_writer = b == 0 && tid == kThreads - 64;   // the last wave's first lane
  // the overlay delta of a node (zero when batch i-1 did not bind it)
  auto delta = [&](int32_t node) -> ResCols {
    if constexpr (DIRECT) {
      return s_rq[s_ent[node]];
    } else {
      ResCols d{0, 0, 0, 0, 0, 0};
      const uint32_t bw = s_bits[node >> 5], bit = 1u << (node & 31);
      if (bw & bit) {
        uint32_t h = lazy_hash(node);
        while (s_hkey[h] != node) h = (h + 1) & (kLazyHash - 1);   // present: the bit says so
        d = s_rq[s_hval[h]];
      }
      return d;
    }
  };
  auto materialize = [&]() {
    if (tid != b) return;
    if (mn0 >= 0) {
      const ResCols d = delta(mn0);
      L.w.req_cpu[mn0] = mr0.cpu + d.cpu;
      L.w.req_mem[mn0] = mr0.mem + d.mem;
      L.w.req_eph[mn0] = mr0.eph + d.eph;
      L.w.nz_cpu[mn0] = mr0.nzc + d.nzc;
      L.w.nz_mem[mn0] = mr0.nzm + d.nzm;
      L.w.num_pods[mn0] = mr0.pods + d.pods;
    }
    if (mn1 >= 0) {
      const ResCols d = delta(mn1);
      L.w.req_cpu[mn1] = mr1.cpu + d.cpu;
      L.w.req_mem[mn1] = mr1.mem + d.mem;
      L.w.req_eph[mn1] = mr1.eph + d.eph;
      L.w.nz_cpu[mn1] = mr1.nzc + d.nzc;
      L.w.nz_mem[mn1] = mr1.nzm + d.nzm;
      L.w.num_pods[mn1] = mr1.pods + d.pods;
    }
  };
  if (!live) {
    materialize();
    if (st_writer) update_state();
    return;
  }
  if constexpr (NS) {
    // pods pod0 + [0, kNsPods) of batch i against S_i over node slice s
    const int32_t s = b % kNsSlices;
    const int32_t len = c.eval_hi - c.eval_lo, S = (len + kNsSlices - 1) / kNsSlices;
    const int32_t slo = c.eval_lo + s * S, shi = min(c.eval_hi, slo + S);
    const FastProg bq = fast_prog(*bp_p);
    const int32_t cu = __builtin_amdgcn_readfirstlane(committed);
    ksim_pod pf[kNsPods];
    uint64_t hs[kNsPods];
    bool pv[kNsPods];
#pragma unroll
    for (int p = 0; p < kNsPods; p++) {
      const PodReq x = s_pc[cu + p];
      pf[p].req_cpu = uni64(x.cpu);
      pf[p].req_mem = uni64(x.mem);
      pf[p].req_eph = uni64(x.eph);
      pf[p].nz_cpu = uni64(x.nzc);
      pf[p].nz_mem = uni64(x.nzm);
#pragma unroll
      for (int k = 0; k < KSIM_MAX_SCALAR; k++) pf[p].scalar_req[k] = 0;   // FAST pods: no scalar requests
      hs[p] = prof_p->tiebreak_seed ^ ((uint64_t)(seq0 + cu + pod0 + p) << 20);
      pv[p] = pi + p < end;                      // block-uniform
    }
    uint64_t ap[kNsPods][kTileCand];
    int32_t nf[kNsPods];
#pragma unroll
    for (int p = 0; p < kNsPods; p++) {
      nf[p] = 0;
#pragma unroll
      for (int q = 0; q < kTileCand; q++) ap[p][q] = 0;
    }
#ifdef KSIM_TC_CLOCKS
    t_pro = __builtin_amdgcn_s_memrealtime();
#endif
#pragma unroll 1
    for (int32_t node = slo + tid; node < shi; node += kThreads) {
      NodeRow r = load_res_row_off(c, node);
      const double ic = ld_off(c.inv_cpu, (uint32_t)node << 3), im = ld_off(c.inv_mem, (uint32_t)node << 3);
      const ResCols d = delta(node);
      r.req_cpu += d.cpu;
      r.req_mem += d.mem;
      r.req_eph += d.eph;
      r.nz_cpu += d.nzc;
      r.nz_mem += d.nzm;
      r.num_pods += d.pods;
#pragma unroll
      for (int p = 0; p < kNsPods; p++) {
        const uint64_t k = pv[p] ? dyn_key_fast_t<DEF>(bq, pf[p], r, ic, im, hs[p], c.base + node) : 0;
        nf[p] += k != 0;
        ap[p][3] = umax64(ap[p][3], k);
        cswap_desc(ap[p][2], ap[p][3]);
        cswap_desc(ap[p][1], ap[p][2]);
        cswap_desc(ap[p][0], ap[p][1]);
      }
    }
#ifdef KSIM_TC_CLOCKS
    t_loop = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) {
      atomicAdd(&g_cp_dbg[0], (unsigned long long)(t_pro - t_in));
      atomicAdd(&g_cp_dbg[1], (unsigned long long)(t_loop - t_pro));
      atomicAdd(&g_cp_dbg[4], (unsigned long long)(tp[0] - t_in));
      atomicAdd(&g_cp_dbg[5], 1ull);
      atomicAdd(&g_cp_dbg[6], (unsigned long long)(tp[1] - tp[0]));
      atomicAdd(&g_cp_dbg[7], (unsigned long long)(tp[2] - tp[1]));
    }
#endif
    materialize();
    // the pods' slice records one after another (top_finish's LDS reused:
    // a barrier between them, which waits for the previous merge's wave)
#pragma unroll
    for (int p = 0; p < kNsPods; p++) {
      if (p) lds_barrier();
      top_finish<kThreads>(ap[p], nf[p], (pod0 + p) * kNsSlices + s, topk, topk_cnt, topk_complete, nullptr);
    }
#ifdef KSIM_TC_CLOCKS
    if (tid == 0) atomicAdd(&g_cp_dbg[3], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - t_loop));
#endif
    if (st_writer) update_state();
    return;
  } else {
  // pod b of batch i against S_i (k_batch_top's loops with the overlay)
  ksim_pod pf;
  {
    const PodReq x = s_pc[committed];
    pf.req_cpu = x.cpu;
    pf.req_mem = x.mem;
    pf.req_eph = x.eph;
    pf.nz_cpu = x.nzc;
    pf.nz_mem = x.nzm;
#pragma unroll
    for (int k = 0; k < KSIM_MAX_SCALAR; k++) pf.scalar_req[k] = 0;   // FAST pods: no scalar requests
  }
  uint64_t a[kTileCand] = {0, 0, 0, 0};
  int32_t nfeas = 0;
  const FastProg bq = fast_prog(*bp_p);
  const uint64_t hseed = prof_p->tiebreak_seed ^ ((uint64_t)(seq0 + committed + b) << 20);
#ifdef KSIM_TC_CLOCKS
  t_pro = __builtin_amdgcn_s_memrealtime();
#endif
  auto key_of = [&](int32_t node) -> uint64_t {
    NodeRow r = load_res_row_off(c, node);
    const double ic = ld_off(c.inv_cpu, (uint32_t)node << 3), im = ld_off(c.inv_mem, (uint32_t)node << 3);
    const ResCols d = delta(node);
    r.req_cpu += d.cpu;
    r.req_mem += d.mem;
    r.req_eph += d.eph;
    r.nz_cpu += d.nzc;
    r.nz_mem += d.nzm;
    r.num_pods += d.pods;
    return dyn_key_fast_t<DEF>(bq, pf, r, ic, im, hseed, c.base + node);
  };
  uint64_t ak[kKeepPerLane];                   // KEEP: the lane's keys, node order
  if constexpr (KEEP) {
#pragma unroll
    for (int q = 0; q < kKeepPerLane; q++) ak[q] = 0;
#pragma unroll
    for (int q = 0; q < kKeepPerLane; q++) {
      if (c.eval_lo + q * kThreads >= c.eval_hi) break;   // block-uniform
      const int32_t node = c.eval_lo + tid + q * kThreads;
      const uint64_t k = node < c.eval_hi ? key_of(node) : 0;
      nfeas += k != 0;
      ak[q] = k;
    }
  } else {
    auto insert = [&](uint64_t k) {
      nfeas += k != 0;
      a[3] = umax64(a[3], k);
      cswap_desc(a[2], a[3]);
      cswap_desc(a[1], a[2]);
      cswap_desc(a[0], a[1]);
    };
#pragma unroll 1
    for (int32_t node = c.eval_lo + tid; node < c.eval_hi; node += kThreads) insert(key_of(node));
  }
#ifdef KSIM_TC_CLOCKS
  t_loop = __builtin_amdgcn_s_memrealtime();
#endif
  materialize();
  // xsend (replicated handles): this replica's record of its node range, for the all-gather
#ifdef KSIM_TC_CLOCKS
  if constexpr (KEEP)
    top_finish<kThreads, kKeepPerLane, false>(ak, nfeas, b, topk, topk_cnt, topk_complete, xsend, tclk);
  else
    top_finish<kThreads>(a, nfeas, b, topk, topk_cnt, topk_complete, xsend, tclk);
  if (tid == 0) {
    // dbg: 0 prologue, 1 thread 0's node loop, 2 wait for the block's slowest
    // wave, 3 the finish after its first barrier, 4 prologue to the first
    // barrier (loads, LDS init), 5 blocks, 6 the cut, 7 the overlay
    const uint64_t t_out = __builtin_amdgcn_s_memrealtime();
    atomicAdd(&g_cp_dbg[0], (unsigned long long)(t_pro - t_in));
    atomicAdd(&g_cp_dbg[1], (unsigned long long)(t_loop - t_pro));
    atomicAdd(&g_cp_dbg[2], (unsigned long long)(tclk[0] - t_loop));
    atomicAdd(&g_cp_dbg[3], (unsigned long long)(t_out - tclk[0]));
    atomicAdd(&g_cp_dbg[4], (unsigned long long)(tp[0] - t_in));
    atomicAdd(&g_cp_dbg[5], 1ull);
    atomicAdd(&g_cp_dbg[6], (unsigned long long)(tp[1] - tp[0]));
    atomicAdd(&g_cp_dbg[7], (unsigned long long)(tp[2] - tp[1]));
  }
#else
  if constexpr (KEEP)
    top_finish<kThreads, kKeepPerLane, false>(ak, nfeas, b, topk, topk_cnt, topk_complete, xsend);
  else
    top_finish<kThreads>(a, nfeas, b, topk, topk_cnt, topk_complete, xsend);
#endif
  if (st_writer) update_state();              // waves past the first return from the merge early
  }
}

// Which instantiations of the evaluation launches a process has launched (or
// captured into a graph): bits 0..9 k_batch_top_commit (tc_variant), bits
// 16..21 k_batch_top (launch_eval_top).  ksim_get_diag out[25]; the variant
// tests assert every bit is reached.
static std::atomic<uint64_t> g_variant_reach{0};
uint64_t batch_variant_reach() { return g_variant_reach.load(std::memory_order_relaxed); }
static void note_variant(int bit) { g_variant_reach.fetch_or(1ull << bit, std::memory_order_relaxed); }

template <bool FLUSH, bool DIRECT, bool DEF, bool KEEP, bool NS>
constexpr int tc_variant() {
  if (FLUSH) return DIRECT ? 0 : 1;
  if (NS) return DIRECT ? 2 : 3;
  if (KEEP) return DEF ? 4 : 5;
  if (DIRECT) return DEF ? 6 : 7;
  return DEF ? 8 : 9;
}

// the evaluation launch of a deferred-commit batch (DIRECT overlay when the
// local node range fits kLazyDirect; DEF / KEEP as k_batch_top_commit says)
template <bool FLUSH, bool DIRECT, bool DEF, bool KEEP, bool NS = false>
static void launch_tc(const LazyBatch& z, uint64_t* xsend, hipStream_t stream) {
  const LaunchArgs& a = z.a;
  note_variant(tc_variant<FLUSH, DIRECT, DEF, KEEP, NS>());
  k_batch_top_commit<FLUSH, DIRECT, DEF, KEEP, NS><<<kBatchPods, 1024, 0, stream>>>(
      a.c, a.P, a.dprof, a.dbp, z.step, a.s.topk, a.s.topk_cnt, a.s.topk_complete, a.chosen, xsend);
}
// the node-stationary form (its records are merged by chain_block<kNsSlices>):
// unsharded launches of the default profile's shape past the KEEP range
static bool ns_eval(const LaunchArgs& a, const uint64_t* xsend) {
  const int32_t len = a.c.eval_hi - a.c.eval_lo;
  return !xsend && fast_def(a.bp) && len > kKeepPerLane * 1024;
}
template <bool FLUSH>
static void launch_top_commit(const LazyBatch& z, uint64_t* xsend, hipStream_t stream) {
  const LaunchArgs& a = z.a;
  const bool direct = a.c.n <= kLazyDirect;
  if constexpr (FLUSH) {
    if (direct) launch_tc<FLUSH, true, false, false>(z, xsend, stream);
    else launch_tc<FLUSH, false, false, false>(z, xsend, stream);
  } else {
    const bool def = fast_def(a.bp);
    const bool keep = direct && a.c.eval_hi - a.c.eval_lo <= kKeepPerLane * 1024;
    if (ns_eval(a, xsend)) {
      if (direct) launch_tc<FLUSH, true, true, false, true>(z, xsend, stream);
      else launch_tc<FLUSH, false, true, false, true>(z, xsend, stream);
    } else if (keep) {
      if (def) launch_tc<FLUSH, true, true, true>(z, xsend, stream);
      else launch_tc<FLUSH, true, false, true>(z, xsend, stream);
    } else if (direct) {
      if (def) launch_tc<FLUSH, true, true, false>(z, xsend, stream);
      else launch_tc<FLUSH, true, false, false>(z, xsend, stream);
    } else {
      if (def) launch_tc<FLUSH, false, true, false>(z, xsend, stream);
      else launch_tc<FLUSH, false, false, false>(z, xsend, stream);
    }
  }
}

const char* const kLazyKernelNames[kKernelsPerLazy] = {"k_batch_top_commit", "k_batch_chain_pairs"};

uint32_t launch_batch_lazy(const LazyBatch& z, hipStream_t stream, hipEvent_t* evs) {
  const LaunchArgs& a = z.a;
  if (evs) (void)hipEventRecord(evs[0], stream);
  launch_top_commit<false>(z, nullptr, stream);
  if (evs) (void)hipEventRecord(evs[1], stream);
  if (ns_eval(a, nullptr))                     // the slice records merged as the chain loads them
    k_batch_chain_pairs<true, true, false, kNsSlices, true><<<kBatchPods, kBatchPods, 0, stream>>>(
        z.cw, a.P, a.dprof, a.dbp, z.st, a.s.topk, a.s.topk_cnt, a.s.topk_complete, z.gkey, z.cend, z.pmax,
        a.s.pnorm, a.s.pinv);
  else if (fast_def(a.bp))
    k_batch_chain_pairs<true, true, false, 1, true><<<kBatchPods, kBatchPods, 0, stream>>>(
        z.cw, a.P, a.dprof, a.dbp, z.st, a.s.topk, a.s.topk_cnt, a.s.topk_complete, z.gkey, z.cend, z.pmax,
        a.s.pnorm, a.s.pinv);
  else
    k_batch_chain_pairs<true, true><<<kBatchPods, kBatchPods, 0, stream>>>(
        z.cw, a.P, a.dprof, a.dbp, z.st, a.s.topk, a.s.topk_cnt, a.s.topk_complete, z.gkey, z.cend, z.pmax,
        a.s.pnorm, a.s.pinv);
  if (evs) (void)hipEventRecord(evs[2], stream);
  return 0x3u;
}

void launch_lazy_top(const LazyBatch& z, hipStream_t stream) { launch_top_commit<false>(z, nullptr, stream); }

// Replicated handles (ksim_set_eval_range): the first launch keys the replica's
// node range and writes its record; after the records' all-gather, the global
// merge and the chain + pairs on X[p].
void launch_lazy_top_rep(const LazyBatch& z, uint64_t* xsend, hipStream_t stream) {
  launch_top_commit<false>(z, xsend, stream);
}

void launch_lazy_chain_rep(const LazyBatch& z, int32_t world, hipStream_t stream) {
  const LaunchArgs& a = z.a;
  k_batch_gmerge<<<kBatchPods / 4, 256, 0, stream>>>(z.st, a.s.xrecv, world, a.s.topk, a.s.topk_cnt,
                                                     a.s.topk_complete);
  k_batch_chain_pairs<true, true><<<kBatchPods, kBatchPods, 0, stream>>>(z.cw, a.P, a.dprof, a.dbp, z.st, a.s.topk,
                                                                            a.s.topk_cnt, a.s.topk_complete, z.gkey,
                                                                            z.cend, z.pmax, a.s.pnorm, a.s.pinv);
}

void launch_lazy_flush(const LazyBatch& z, hipStream_t stream) { launch_top_commit<true>(z, nullptr, stream); }

// In-process shard group: M = max over the group's pmax arrays, written back to each.
__global__ __launch_bounds__(kBatchPods) void k_group_max(GroupPtrs g) {
  const int j = threadIdx.x;
  uint64_t m = 0;
  for (int r = 0; r < g.n; r++) m = umax64(m, g.p[r][j]);
  for (int r = 0; r < g.n; r++) g.p[r][j] = m;
}

const char* const kBatchKernelNames[kKernelsPerBatch] = {"k_batch_top", "k_batch_chain_pairs", "k_batch_commit"};

// Evaluation and per-pod top-T (xsend: the sharded record, else null).
static void launch_eval_top(const LaunchArgs& a, uint64_t* xsend, hipStream_t stream) {
  const bool def = fast_def(a.bp);
  const bool keep = a.c.eval_hi - a.c.eval_lo <= kKeepPerLane * 1024;
  note_variant(a.stab && def && keep ? 16 : a.stab && def ? 17 : a.stab ? 18 : a.fast && def ? 19 : a.fast ? 20 : 21);
  if (a.stab && def && keep)
    k_batch_top<true, 1024, true, true, true><<<kBatchPods, 1024, 0, stream>>>(
        a.c, a.P, a.dprof, a.dbp, a.st, a.s.topk, a.s.topk_cnt, a.s.topk_complete, xsend, a.s.pnorm);
  else if (a.stab && def)   // static-class runs (unsharded handles only: run_stab)
    k_batch_top<true, 1024, true, true><<<kBatchPods, 1024, 0, stream>>>(
        a.c, a.P, a.dprof, a.dbp, a.st, a.s.topk, a.s.topk_cnt, a.s.topk_complete, xsend, a.s.pnorm);
  else if (a.stab)
    k_batch_top<true, 1024, true><<<kBatchPods, 1024, 0, stream>>>(a.c, a.P, a.dprof, a.dbp, a.st, a.s.topk,
                                                                    a.s.topk_cnt, a.s.topk_complete, xsend, a.s.pnorm);
  else if (a.fast && def)
    k_batch_top<true, 1024, false, true><<<kBatchPods, 1024, 0, stream>>>(
        a.c, a.P, a.dprof, a.dbp, a.st, a.s.topk, a.s.topk_cnt, a.s.topk_complete, xsend, a.s.pnorm);
  else if (a.fast)
    k_batch_top<true, 1024><<<kBatchPods, 1024, 0, stream>>>(a.c, a.P, a.dprof, a.dbp, a.st, a.s.topk, a.s.topk_cnt,
                                                              a.s.topk_complete, xsend, a.s.pnorm);
  else   // generic keys: 512 threads, so the full plugin chain's registers fit without spilling
    k_batch_top<false, 512><<<kBatchPods, 512, 0, stream>>>(a.c, a.P, a.dprof, a.dbp, a.st, a.s.topk, a.s.topk_cnt,
                                                             a.s.topk_complete, xsend, a.s.pnorm);
}

// The chain inside every pairs block (k_batch_chain_pairs).
static void launch_chain_pairs(const LaunchArgs& a, hipStream_t stream) {
  if (a.stab && fast_def(a.bp))
    k_batch_chain_pairs<true, false, true, 1, true><<<kBatchPods, kBatchPods, 0, stream>>>(
        a.c, a.P, a.dprof, a.dbp, a.st, a.s.topk, a.s.topk_cnt, a.s.topk_complete, a.s.gkey, a.s.chain_end, a.s.pmax,
        a.s.pnorm, a.s.pinv);
  else if (a.stab)
    k_batch_chain_pairs<true, false, true><<<kBatchPods, kBatchPods, 0, stream>>>(
        a.c, a.P, a.dprof, a.dbp, a.st, a.s.topk, a.s.topk_cnt, a.s.topk_complete, a.s.gkey, a.s.chain_end, a.s.pmax,
        a.s.pnorm, a.s.pinv);
  else if (a.fast)
    k_batch_chain_pairs<true><<<kBatchPods, kBatchPods, 0, stream>>>(a.c, a.P, a.dprof, a.dbp, a.st, a.s.topk,
                                                                     a.s.topk_cnt, a.s.topk_complete, a.s.gkey,
                                                                     a.s.chain_end, a.s.pmax, a.s.pnorm, a.s.pinv);
  else
    k_batch_chain_pairs<false><<<kBatchPods, kBatchPods, 0, stream>>>(a.c, a.P, a.dprof, a.dbp, a.st, a.s.topk,
                                                                      a.s.topk_cnt, a.s.topk_complete, a.s.gkey,
                                                                      a.s.chain_end, a.s.pmax, a.s.pnorm, a.s.pinv);
}

uint32_t launch_batch(const LaunchArgs& a, hipStream_t stream, hipEvent_t* evs) {
  if (evs) (void)hipEventRecord(evs[0], stream);
  launch_eval_top(a, nullptr, stream);
  if (evs) (void)hipEventRecord(evs[1], stream);
  launch_chain_pairs(a, stream);
  if (evs) (void)hipEventRecord(evs[2], stream);
  k_batch_commit<<<1, kBatchPods, 0, stream>>>(a.c, a.P, a.st, a.s.gkey, a.s.chain_end, a.s.pmax, a.chosen,
                                               (a.fast && !a.stab) ? nullptr : a.s.pinv);
  if (evs) (void)hipEventRecord(evs[3], stream);
  return 0x7u;
}

void launch_batch_eval_only(const LaunchArgs& a, hipStream_t stream) { launch_eval_top(a, nullptr, stream); }

void launch_shard_eval(const LaunchArgs& a, hipStream_t stream) { launch_eval_top(a, a.s.xsend, stream); }

void k_batch_gmerge_launch(const LaunchArgs& a, int32_t world, hipStream_t stream) {
  k_batch_gmerge<<<kBatchPods / 4, 256, 0, stream>>>(a.st, a.s.xrecv, world, a.s.topk, a.s.topk_cnt,
                                                     a.s.topk_complete);
}
void launch_shard_chain(const LaunchArgs& a, int32_t world, hipStream_t stream) {
  k_batch_gmerge_launch(a, world, stream);
  launch_chain_pairs(a, stream);
}

void launch_shard_commit(const LaunchArgs& a, hipStream_t stream) {
  k_batch_commit<<<1, kBatchPods, 0, stream>>>(a.c, a.P, a.st, a.s.gkey, a.s.chain_end, a.s.pmax, a.chosen, nullptr);
}

void launch_group_max(const GroupPtrs& g, hipStream_t stream) { k_group_max<<<1, kBatchPods, 0, stream>>>(g); }

}  // namespace ksim
