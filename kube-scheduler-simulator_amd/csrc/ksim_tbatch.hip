// ksim_tbatch.hip — the topology batch path (gfx950): pods with
// PodTopologySpread / InterPodAffinity uses, scheduled up to kTbPods at a time
// against the batch-start snapshot S0 (SURVEY §7 hard part 3; config 3).
//
// A pod's topology inputs are count classes (§5): the domain sums it reads
// come from the persistent tables of the classes its uses name, and a bind
// changes only the classes in the bound pod's adds.  The host cuts the queue
// into runs in which no pod reads a class an earlier pod of the run adds
// (DevPods.bflags >> kTlenShift, ksim_engine.cpp tbatch_runs).  Inside such a
// run every pod's filter verdicts, raw scores, normalization extrema and
// PodTopologySpread weights on every node are those of S0, except on the
// nodes earlier pods of the batch bound, and there only NodeResourcesFit and
// the two resource scores move.  So the P100 batch machinery applies: each
// pod's exact S0 top-T, the greedy chain, the pair keys of every pod on the
// earlier pods' nodes, and the commit up to the first pod whose choice
// differs.  One more way a pod's S0 keys can fail: a node that was feasible
// at S0 stops fitting after an earlier bind, which changes the feasible set
// the normalization and the spread weights were taken over; such a pod ends
// the batch before it (pinv), and the next batch starts from it.
//
// Zone variants (round 6, ksim_device.h TbVar): a run may also cross the
// class of a pod's DoNotSchedule spread constraint on a key of at most
// kVarDom domains (zones) when one earlier pod of the run adds to it.  That
// pod's bind moves one domain's count, which moves the skew verdict of whole
// domains (once an app's zones are level, almost every bind of the app does),
// so the pod is evaluated per reachable feasible-domain set: k_tb_filter
// passes the constraint's skew and keeps counters and extrema per domain,
// k_tb_select normalizes, keys and lists each distinct set (a slot) over its
// domains, and the chain takes the slot the earlier pod's guess lands in.
//
//   k_tb_filter      grid (node blocks, pods): RunFilterPlugins and the raw
//                    scores of pod j on every node (k_filter_score's plan
//                    chains), feasible / ignored counts and NormalizeScore
//                    extrema per pod (block_extrema; per domain for a variant
//                    pod), the critical paths and InterPodAffinity flags from
//                    the persistent tables; block 0 derives the pod's slots
//   k_tb_select      grid (node blocks, pods): normalized weighted totals (as
//                    k_select), TB keys, each block's exact top-T per pod and
//                    slot, and per node stat = total - (Fit + BalancedAllocation) part
//   k_tb_merge       one wave per pod and slot: its exact top-T from its blocks'
//   k_tb_chain_pairs the chain (tb_chain, one wave), then pod j on each earlier
//                    guess: stat + the resource part after that bind, or pinv
//   k_tb_commit      batch_commit, the committed pods' count-class adds and
//                    persistent-table updates as parallel atomics, and the
//                    window state re-zeroed for the next batch
#include "ksim_device.h"
#include "ksim_internal.h"
#include "ksim_wave.h"
#include "ksim_cycle.h"
#include "ksim_commit.h"

namespace ksim {

constexpr int32_t kStatNone = INT32_MIN;       // tb_stat: not feasible at S0
constexpr int32_t kStatOne = INT32_MIN + 1;    // tb_stat: the pod's only feasible node (chosen unscored)

// The batch's pod count: the conflict-free run from the cursor, capped.
// plain: the run without zone variants (replicated topology batches).
__device__ __forceinline__ int32_t tb_count(const DevState* __restrict__ st, const DevPods& P, int32_t plain) {
  const int32_t base = st->cursor;
  if (base >= st->end) return 0;
  const int32_t tlen = (P.bflags[base] >> (plain ? kTlenPlainShift : kTlenShift)) & kTlenMask;
  return min(min(kTbPods, st->end - base), max(tlen, 1));
}

// Pod j's slices of the topology batch scratch.
struct TbSlice {
  uint8_t* fail;
  uint8_t* ign;
  uint8_t* vdom;                                   // value ids: the pod's variant key | the run's variant column << 4
  int64_t* part;
  int64_t* raw;
  WinState* win;
};
__device__ __forceinline__ TbSlice tb_slice(const DevScratch& s, int32_t j, int32_t n) {
  const size_t N = (size_t)n;
  return TbSlice{s.tb_fail + j * N, s.tb_ign + j * N, s.tb_vdom + j * N, s.tb_part + j * N,
                 s.tb_raw + (size_t)j * KSIM_MAX_SCORE * N, s.tb_win + j};
}
// Pod j's list / stat / holder slot sl (0 for a pod without variants).
__device__ __forceinline__ size_t tb_pj(int32_t j, int32_t sl) { return (size_t)j * kVarSlots + sl; }

// KSIM_TB_CLOCKS builds (100 MHz realtime, summed into s.dbg, ksim_get_diag
// out[3..18]): k_tb_chain_pairs block 0 -- [0] chain prologue, [1] rounds,
// [2] rounds run, [3] chain + pairs, [4] launches; k_tb_filter every block --
// [5] start to the topology setup, [6] the filter and score plans, [7] the
// extrema and slots, [8] blocks; k_tb_select every block -- [9] start to the
// pod's inputs, [10] the slots, [11] blocks, [12] slots; k_tb_chain_pairs
// every block that keys pairs -- [13] start to the pair maxima, [14] blocks.
#ifdef KSIM_TB_CLOCKS
#define TB_CLOCK(var) const uint64_t var = __builtin_amdgcn_s_memrealtime()
#else
#define TB_CLOCK(var) do {} while (0)
#endif

// A variant pod's constraint skew passes on every node in k_tb_filter (the
// slots take the verdicts per domain): a critical-path minimum no count reaches.
constexpr int64_t kVarNoMin = 1ll << 50;

// The feasible / ignored counts of pod j's slot (mask mk; the pod's tb_win
// without variants).  Uniform.
__device__ __forceinline__ void tb_slot_counts(const DevScratch& s, int32_t j, const TbVar& V, uint32_t mk,
                                               int32_t& nf, int32_t& nign) {
  if (V.use < 0) {
    nf = s.tb_win[j].nfeas;
    nign = s.tb_win[j].nign;
    return;
  }
  nf = nign = 0;
#pragma unroll
  for (int d = 0; d < kVarDom; d++)
    if (d < V.ndom && ((mk >> d) & 1u)) {
      nf += s.tb_dom[(size_t)j * kVarDom + d].nfeas;
      nign += s.tb_dom[(size_t)j * kVarDom + d].nign;
    }
}

// One extremum word e of pod j's slot (mask mk) without materializing the
// slot's record (k_tb_select keeps its registers for the node loop).  Uniform.
__device__ __forceinline__ uint64_t tb_slot_ext(const DevScratch& s, int32_t j, const TbVar& V, uint32_t mk, int32_t nf,
                                                int e) {
  if (V.use < 0) return s.tb_win[j].ext[e];
  if ((V.zmask >> (e >> 1)) & 1u) return nf > 0 ? ((e & 1) ? min_image(0) : max_image(0)) : 0ull;
  uint64_t x = 0;
#pragma unroll
  for (int d = 0; d < kVarDom; d++)
    if (d < V.ndom && ((mk >> d) & 1u)) x = umax64(x, s.tb_dom[(size_t)j * kVarDom + d].ext[e]);
  return x;
}

// A variant pod's per-domain feasible / ignored counts and NormalizeScore
// extrema (block_extrema per domain of the variant key; zmask slots are set
// by tb_slot_ext).  dom: the node's value id of the key (1 .. nd when feasible).
__device__ __forceinline__ void tb_dom_extrema(const ksim_profile& prof, TbDom* __restrict__ out, int32_t nd,
                                               uint32_t zmask, bool feasible, bool ign, uint32_t dom,
                                               const uint64_t (&ix)[KSIM_MAX_SCORE],
                                               const uint64_t (&in)[KSIM_MAX_SCORE],
                                               uint64_t (*s_red)[kVarDom][2 * KSIM_MAX_SCORE],
                                               int32_t (*s_cnt)[kVarDom][2]) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int S = prof.n_score;
#pragma unroll 1
  for (int d = 0; d < nd; d++) {                  // one domain at a time (the loop body holds the VGPR peak)
    const bool on = feasible && dom == (uint32_t)(d + 1);
    const uint64_t fm = __ballot(on), im = __ballot(on && ign);
    if (lane == 0) {
      s_cnt[wv][d][0] = (int32_t)__popcll(fm);
      s_cnt[wv][d][1] = (int32_t)__popcll(im);
    }
#pragma unroll
    for (int k = 0; k < KSIM_MAX_SCORE; k++) {
      if (k >= S) break;
      if (norm_kind(prof.score[k]) == kNormNone || ((zmask >> k) & 1u)) continue;
      const uint64_t a = wave_max_u64_dpp(on ? ix[k] : 0), b = wave_max_u64_dpp(on ? in[k] : 0);
      if (lane == 0) {
        s_red[wv][d][2 * k] = a;
        s_red[wv][d][2 * k + 1] = b;
      }
    }
  }
  lds_barrier();
  if (tid < nd * 2 * KSIM_MAX_SCORE) {
    const int d = tid / (2 * KSIM_MAX_SCORE), e = tid % (2 * KSIM_MAX_SCORE), k = e >> 1;
    if (k < S && norm_kind(prof.score[k]) != kNormNone && !((zmask >> k) & 1u)) {
      uint64_t m = 0;
#pragma unroll
      for (int w = 0; w < 4; w++) m = umax64(m, s_red[w][d][e]);
      if (m) atomicMax(reinterpret_cast<unsigned long long*>(&out[d].ext[e]), (unsigned long long)m);
    }
  } else if (tid >= 128 && tid < 128 + 2 * nd) {
    const int d = (tid - 128) >> 1, q = (tid - 128) & 1;
    const int32_t v = s_cnt[0][d][q] + s_cnt[1][d][q] + s_cnt[2][d][q] + s_cnt[3][d][q];
    if (v) atomicAdd(q ? &out[d].nign : &out[d].nfeas, v);
  }
}

// Pod j's slots (one wave of block 0): the one earlier pod of the batch adding
// to the variant use's class (its adder: exactly one add entry in the batch,
// on the run's variant column), the S0 domain entries of the use's table, and
// per landing domain of the adder (0: it moves no count) the domains whose
// skew passes; equal sets share a slot.  The same verdict as pts_filter with
// topo_block_setup's critical path over the moved counts.
__device__ __forceinline__ void tb_var_setup(const DevCluster& c, const DevPods& P, const DevScratch& s,
                                          const DevState* __restrict__ st, int32_t j, int32_t vu, uint32_t zmask,
                                          int32_t vcol) {
  const int lane = threadIdx.x & 63;
  TbVar* out = s.tb_var + j;
  if (vu < 0) {
    if (lane == 0) {
      TbVar V{};
      V.use = -1;
      V.adder = -1;
      V.nslot = 1;
      V.col = -1;
      V.vcol = vcol;
      V.zmask = zmask;
      V.mask[0] = ~0u;
      *out = V;
    }
    return;
  }
  const int32_t base = st->cursor;
  const ksim_pod& p = P.pods[base + j];
  const ksim_topo_use u = load_use(P.uses + p.use_first, vu);
  const int32_t nd = c.col_nvals[u.col] - 1;        // 1 .. kVarDom (k_tb_filter)
  const uint32_t self = (P.plans[base + j].m.self_match >> vu) & 1u;
  int32_t ne = 0, cx = 0;
  if (lane < j) {
    const ksim_pod& pk = P.pods[base + lane];
    for (int a = 0; a < pk.add_count; a++) {
      const ksim_class_add x = P.adds[pk.add_first + a];
      if (x.cls == u.cls) {
        ne++;
        cx += x.count;
      }
    }
  }
  const int64_t e = lane <= nd ? P.ptab[u._pad + lane] : 0;
  const int32_t tot = (int32_t)wave_sum_u32_dpp((uint32_t)ne);
  const uint64_t who = __ballot(ne > 0);
  const int32_t adder = (tot == 1 && vcol == u.col) ? (int32_t)__builtin_ctzll(who) : -1;
  const int32_t x = __shfl(cx, adder >= 0 ? adder : 0, 64);
  int64_t cnt[kVarDom + 1];
  bool mk[kVarDom + 1];
#pragma unroll
  for (int v = 0; v <= kVarDom; v++) {
    const int64_t ev = (int64_t)readlane_u64((uint64_t)e, v);
    cnt[v] = ev & kDomCountMask;
    mk[v] = v <= nd && (ev >> kDomMarkShift) != 0;
  }
  if (lane != 0) return;
  TbVar V{};
  V.use = vu;
  V.adder = adder;
  V.ndom = nd;
  V.col = u.col;
  V.vcol = vcol;
  V.zmask = zmask;
  V.nslot = 0;
  const int32_t wmax = adder >= 0 ? nd : 0;
#pragma unroll
  for (int w = 0; w <= kVarDom; w++) {
    V.slot_of[w] = 0;
    if (w > wmax) continue;
    int64_t mn = 2147483647;                       // topo_block_setup's minimum over marked domains
#pragma unroll
    for (int v = 0; v <= kVarDom; v++)
      if (mk[v]) mn = min(mn, cnt[v] + (v == w && w > 0 ? x : 0));
    uint32_t m = 0;
#pragma unroll
    for (int d = 1; d <= kVarDom; d++) {
      if (d > nd) continue;
      const int64_t c = cnt[d] + (d == w ? x : 0);
      if (c + (int64_t)self - mn <= (int64_t)u.arg) m |= 1u << (d - 1);
    }
    int32_t q = 0;
    while (q < V.nslot && V.mask[q] != m) q++;
    if (q == V.nslot) V.mask[V.nslot++] = m;
    V.slot_of[w] = q;
  }
  *out = V;
}

// Three waves per SIMD (156 VGPRs, no spills) instead of the two its 176
// VGPRs allowed: the kernel waits on its table and row loads most of the time.
// KSIM_TB_FILTER_WAVES builds set another occupancy (A/B flavors).
#ifndef KSIM_TB_FILTER_WAVES
#define KSIM_TB_FILTER_WAVES 3
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(KSIM_TB_FILTER_WAVES))) void k_tb_filter(DevCluster c, DevPods P0, const ksim_profile* __restrict__ prof_p,
                                                   const BatchProg* __restrict__ bp, const DevState* __restrict__ st,
                                                   DevScratch s, int32_t plain) {
  __shared__ int64_t s_min[KSIM_MAX_USES];
  __shared__ uint64_t s_red[4][2 * KSIM_MAX_SCORE];
  __shared__ uint64_t s_dred[4][kVarDom][2 * KSIM_MAX_SCORE];
  __shared__ int32_t s_cnt[4][2];
  __shared__ int32_t s_dcnt[4][kVarDom][2];
  __shared__ uint32_t s_tf;
  TB_CLOCK(f0);
  const int32_t node = c.eval_lo + blockIdx.x * blockDim.x + threadIdx.x;   // replicas: their range
  const int32_t xr = node < c.eval_hi ? node : c.eval_hi - 1;
  // the node's row does not depend on the pod: its loads go out first
  const NodeRow r = load_row(c, xr);
  const double inv_c = c.inv_cpu[xr], inv_m = c.inv_mem[xr];
  const int32_t j = blockIdx.y;
  if (j >= tb_count(st, P0, plain)) return;         // block-uniform
  const ksim_profile& prof = *prof_p;
  const int32_t pi = st->cursor + j;
  const DevPods& P = P0;
  const ksim_pod& p = P0.pods[pi];
  const PodPlan pp = P0.plans[pi];
  const UseMasks& m = pp.m;
  const ksim_topo_use* U = P.uses + p.use_first;
  const TbSlice q = tb_slice(s, j, c.n);
  // the zone-variant use (plain launches and keys grown past kVarDom domains: none)
  int32_t vu = plain ? -1 : (int32_t)((pp.flags >> kPlanVuseShift) & 31u) - 1;
  const int32_t vcol = plain ? -1 : (int32_t)(P0.plans[st->cursor].flags >> kPlanVcolShift) - 1;
  int32_t nd = 0;
  uint32_t vdom = 0, rdom = 0;                     // the node's value ids of the variant key / the run's column
  if (vu >= 0) {
    const int32_t col = load_use(U, vu).col;
    nd = c.col_nvals[col] - 1;
    if (nd < 1 || nd > kVarDom) vu = -1;
    else vdom = c.labels[(size_t)col * c.n + xr];
  }
  if (vcol >= 0) rdom = c.labels[(size_t)vcol * c.n + xr];
  TopoRow t;
  load_topo_row(c, U, p.use_count, m, s, P0.ptab, xr, t);
  const bool pt = (pp.flags & kPlanPtab) != 0;      // the host admits only table-read pods (tbatch_admit)
  if (m.hard || (pt && (m.aff | m.score))) {
    topo_block_setup(c, P0, s, U, m, pt, true, s_min, &s_tf, &q.win->tflags);
    if (vu >= 0 && threadIdx.x == 0) s_min[vu] = kVarNoMin;   // after thread 0's critical paths
    lds_barrier();
  }
  TB_CLOCK(f1);
  const uint32_t tf = pt && (m.aff | m.score) ? s_tf : 0u;
  bool feasible = false, ign = false;
  RawScores rv{};
  int64_t soft_cnt = 0;
  const int soft = m.soft ? 31 - __builtin_clz(m.soft) : -1;   // the pod's one ScheduleAnyway use
  if (node < c.eval_hi) {
    uint32_t det;
    const uint8_t res = run_filter_plan(c, P, FilterPlan{bp->rank_lo, bp->rank_hi, pp.filter_en}, s_min, tf, p, r,
                                        U, m, t, det);
    q.fail[node] = res;
    if (vu >= 0 || vcol >= 0) q.vdom[node] = (uint8_t)(min(vdom, 15u) | (min(rdom, 15u) << 4));
    feasible = res == KSIM_PASSED;
    if (feasible) {
#pragma unroll
      for (int i = 0; i < KSIM_MAX_USES; i++) {
        if (((m.soft >> i) & 1u) && t.v[i] == 0 && !(p.topo_flags & KSIM_POD_PTS_SYSTEM_DEFAULT)) ign = true;
        if (i == soft) soft_cnt = t.x[i];
      }
      q.ign[node] = ign;
      const BatchProg* fast = (bp->fast_w && (c.cflags & kClusterNarrow)) ? bp : nullptr;
      // store_plain: the Fit / BalancedAllocation raw scores stay for k_tb_select's stat
      q.part[node] = run_score_plan(c, P, prof, ScorePlan{bp->slot, bp->slot_hi}, p, r, U, m, t, q.raw, true, rv,
                                    soft_cnt, fast, inv_c, inv_m);
    }
  }
  // feasible / ignored counts and the NormalizeScore extrema (k_filter_score's fuse_ext tail)
  const int lane = threadIdx.x & 63;
  const uint64_t fm = __ballot(feasible), im = __ballot(feasible && ign);
  TB_CLOCK(f2);
  if (lane == 0) {
    s_cnt[threadIdx.x >> 6][0] = (int32_t)__popcll(fm);
    s_cnt[threadIdx.x >> 6][1] = (int32_t)__popcll(im);
  }
  uint64_t ix[KSIM_MAX_SCORE], in[KSIM_MAX_SCORE];
#pragma unroll
  for (int k = 0; k < KSIM_MAX_SCORE; k++) {
    ix[k] = in[k] = 0;
    if (k >= prof.n_score || !feasible) continue;
    const int pl = (int)prof_score(prof, k);
    if (norm_kind(pl) == kNormNone) continue;
    int64_t v = 0;
    bool counted = true;
    if (pl == KSIM_PL_POD_TOPOLOGY_SPREAD) {
      counted = soft < 0 || !ign;                  // IgnoredNodes: not in min / max
      v = soft < 0 ? 0 : soft_cnt;
    } else {
      v = rv.of(pl);
    }
    if (counted) {
      ix[k] = max_image(v);
      in[k] = min_image(v);
    }
  }
  uint32_t zmask = 0;                              // slots constant 0 for this pod
#pragma unroll
  for (int k = 0; k < KSIM_MAX_SCORE; k++) {
    if (k >= prof.n_score) continue;
    const int pl = (int)prof_score(prof, k);
    const bool z = (pl == KSIM_PL_TAINT_TOLERATION && !(c.cflags & kClusterPreferTaints)) ||
                   (pl == KSIM_PL_NODE_AFFINITY && p.pref_term_count == 0) ||
                   (pl == KSIM_PL_INTER_POD_AFFINITY && m.score == 0) ||
                   (pl == KSIM_PL_POD_TOPOLOGY_SPREAD && soft < 0);
    if (z) zmask |= 1u << k;
  }
  if (vu < 0)
    block_extrema(prof, q.win, ix, in, s_red, zmask, s_cnt);
  else
    tb_dom_extrema(prof, s.tb_dom + (size_t)j * kVarDom, nd, zmask, feasible, ign, vdom, ix, in, s_dred, s_dcnt);
  if (blockIdx.x == 0 && threadIdx.x < 64) tb_var_setup(c, P0, s, st, j, vu, zmask, vcol);
#ifdef KSIM_TB_CLOCKS
  if (threadIdx.x == 0) {
    const uint64_t f3 = __builtin_amdgcn_s_memrealtime();
    atomicAdd(&s.dbg[5], (unsigned long long)(f1 - f0));
    atomicAdd(&s.dbg[6], (unsigned long long)(f2 - f1));
    atomicAdd(&s.dbg[7], (unsigned long long)(f3 - f2));
    atomicAdd(&s.dbg[8], 1ull);
  }
#endif
}

// Each block's exact top-T keys of pod j over its 256 nodes: every wave
// extracts its own top-T (kTopT rounds of DPP max), wave 0 ranks the 4 T
// candidates (keys are unique: ranks are distinct).  kd / out_dom (nullable):
// a byte carried with each key (the run-column value id of its node).
__device__ __forceinline__ void block_top_t(uint64_t key, uint32_t kd, uint64_t* s_cand, uint8_t* s_cdom,
                                            uint64_t* out, uint8_t* out_dom, int32_t* out_cnt) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t a = key;
#pragma unroll 1
  for (int e = 0; e < kTopT; e++) {
    const uint64_t mx = wave_max_u64_dpp(a);
    if (lane == 0) s_cand[wv * kTopT + e] = mx;
    if (a == mx && a != 0) s_cdom[wv * kTopT + e] = (uint8_t)kd;   // the one lane holding it
    if (a == mx) a = 0;                            // 0 stays 0: an exhausted wave lists zeros
  }
  lds_barrier();
  if (wv != 0) return;
  constexpr int kC = 4 * kTopT;
  static_assert(kC <= 64, "block_top_t geometry");
  const uint64_t c0 = lane < kC ? s_cand[lane] : 0;
  const uint8_t d0 = lane < kC ? s_cdom[lane] : 0;
  int32_t rank = 0;
#pragma unroll
  for (int x = 0; x < kC; x++) rank += s_cand[x] > c0;
  const int32_t n = __popcll(__ballot(c0 != 0));
  if (c0 != 0 && rank < kTopT) {
    out[rank] = c0;
    if (out_dom) out_dom[rank] = d0;
  }
  if (lane >= n && lane < kTopT) out[lane] = 0;
  if (lane == 0) *out_cnt = n < kTopT ? n : kTopT;
}

// The filter's per-node outputs, the pod's variant record and its counters /
// extrema (tb_win, or per domain tb_dom, staged in LDS) are read before the
// batch state: they do not depend on it, and a kernel that waited for the
// state first would pay one more global round trip (data the previous launch
// wrote sits in another XCD's L2).  Barriers are LDS-only (lds_barrier): the
// stat stores stay in flight across them.
__global__ __launch_bounds__(256) void k_tb_select(DevCluster c, DevPods P0, const ksim_profile* __restrict__ prof_p,
                                                   const BatchProg* __restrict__ bp, const DevState* __restrict__ st,
                                                   DevScratch s, int32_t plain) {
  __shared__ uint64_t s_cand[4 * kTopT];
  __shared__ uint8_t s_cdom[4 * kTopT];
  __shared__ int32_t s_hold[4][4];
  __shared__ TbDom s_dom[kVarDom + 1];             // the pod's domains; [kVarDom]: its tb_win counters / extrema
  TB_CLOCK(x0);
  const int32_t node = c.eval_lo + blockIdx.x * blockDim.x + threadIdx.x;
  const int32_t j = blockIdx.y;
  const int32_t sl = blockIdx.z;                   // one slot per block: a pod's slots run side by side
  if (sl > 0 && sl >= s.tb_var[j].nslot) return;   // slot 0 always runs: its loads need not wait for this
  const int32_t N = c.n;
  const TbSlice q = tb_slice(s, j, N);
  const bool live = node < c.eval_hi;
  const ksim_profile& prof = *prof_p;
  const int S = prof.n_score;
  const uint8_t fail = live ? q.fail[node] : (uint8_t)0;
  const uint8_t vd = live ? q.vdom[node] : (uint8_t)0;
  const bool ign0 = live && q.ign[node] != 0;
  const int64_t part = live ? q.part[node] : 0;
  int64_t raw[KSIM_MAX_SCORE];
#pragma unroll
  for (int k = 0; k < KSIM_MAX_SCORE; k++) raw[k] = (live && k < S) ? q.raw[(size_t)k * N + node] : 0;
  {
    constexpr int W = kVarDom * (int)(sizeof(TbDom) / 4);
    static_assert(sizeof(TbDom) % 4 == 0, "TbDom by words");
    const int32_t* src = reinterpret_cast<const int32_t*>(s.tb_dom + (size_t)j * kVarDom);
    int32_t* dst = reinterpret_cast<int32_t*>(s_dom);
    if (threadIdx.x < W) dst[threadIdx.x] = src[threadIdx.x];
    const int x = (int)threadIdx.x - W;
    if (x >= 0 && x < 2 * KSIM_MAX_SCORE) s_dom[kVarDom].ext[x] = q.win->ext[x];
    if (x == 2 * KSIM_MAX_SCORE) s_dom[kVarDom].nfeas = q.win->nfeas;
    if (x == 2 * KSIM_MAX_SCORE + 1) s_dom[kVarDom].nign = q.win->nign;
  }
  const TbVar& V = s.tb_var[j];
  const int32_t ns = V.nslot, vuse = V.use, vcol = V.vcol, vnd = V.ndom;
  const uint32_t vz = V.zmask;
  if (j >= tb_count(st, P0, plain) || sl >= ns) return;   // block-uniform
  const int32_t pi = st->cursor + j;
  const ksim_pod& p = P0.pods[pi];
  const UseMasks m = P0.plans[pi].m;
  const ksim_topo_use* U = P0.uses + p.use_first;
  const int soft = m.soft ? 31 - __builtin_clz(m.soft) : -1;
  int32_t ms = 0;                                  // topologyNormalizingWeight inputs (hostname keys only: tbatch_admit)
  bool soft_hn = false;
  if (soft >= 0) {
    const ksim_topo_use u = load_use(U, soft);
    soft_hn = (u.flags & KSIM_USEF_HOSTNAME) != 0;
    ms = u.arg;
  }
  const bool ipa_nonempty = (q.win->tflags & kTopoScoreNonEmpty) != 0;
  const ScorePlan sp{bp->slot, bp->slot_hi};
  const int k_fit = plan_slot(sp, KSIM_PL_NODE_RESOURCES_FIT), k_ba = plan_slot(sp, KSIM_PL_BALANCED_ALLOCATION);
  const uint64_t seed = prof.tiebreak_seed;
  const int64_t seq = st->pod_seq + j;
  const bool pass = live && fail == KSIM_PASSED;
  const uint32_t dom = vd & 15u, rdom = vd >> 4;
  const bool cross = (P0.bflags[st->cursor] & kPodTbCross) != 0;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  lds_barrier();                                   // s_dom
#ifdef KSIM_TB_CLOCKS
  const uint64_t x1 = (ms >= 0 && ipa_nonempty >= 0 && seq >= 0 && vd < 255) ? __builtin_amdgcn_s_memrealtime() : 0;
#endif
  {
    const uint32_t mk = vuse >= 0 ? V.mask[sl] : ~0u;
    // the slot's counters and extrema from the staged records
    int32_t nf = 0, nign = 0;
    uint64_t ext[2 * KSIM_MAX_SCORE];
    if (vuse < 0) {
      nf = s_dom[kVarDom].nfeas;
      nign = s_dom[kVarDom].nign;
#pragma unroll
      for (int e = 0; e < 2 * KSIM_MAX_SCORE; e++) ext[e] = s_dom[kVarDom].ext[e];
    } else {
#pragma unroll
      for (int e = 0; e < 2 * KSIM_MAX_SCORE; e++) ext[e] = 0;
#pragma unroll
      for (int d = 0; d < kVarDom; d++) {
        if (d >= vnd || !((mk >> d) & 1u)) continue;
        nf += s_dom[d].nfeas;
        nign += s_dom[d].nign;
#pragma unroll
        for (int e = 0; e < 2 * KSIM_MAX_SCORE; e++) ext[e] = umax64(ext[e], s_dom[d].ext[e]);
      }
      if (nf > 0) {                                // slots constant 0 (block_extrema's zmask)
#pragma unroll
        for (int k = 0; k < KSIM_MAX_SCORE; k++)
          if ((vz >> k) & 1u) {
            ext[2 * k] = max_image(0);
            ext[2 * k + 1] = min_image(0);
          }
      }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) s.tb_vnf[tb_pj(j, sl)] = nf;
    const bool has_soft = nf > 1 && soft >= 0;
    const double w_soft = has_soft ? c.topo_log[soft_hn ? nf - nign : 0] : 0.0;
    const bool feas = pass && (vuse < 0 || (dom >= 1 && dom <= (uint32_t)kVarDom && ((mk >> (dom - 1)) & 1u)));
    uint64_t key = 0;
    uint32_t hf = 0;                               // holds PTS max, PTS min, IPA max, IPA min
    if (live) {
      int32_t stat = kStatNone;
      if (feas) {
        if (nf > 1) {
          const bool ign = has_soft && ign0;
          int64_t tot = S == 0 ? 1 : part;
#pragma unroll
          for (int k = 0; k < KSIM_MAX_SCORE; k++) {
            if (k >= S) break;
            const int32_t kind = norm_kind(prof_score(prof, k));
            if (kind == kNormNone) continue;
            const uint64_t ex = ext[2 * k], en = ext[2 * k + 1];
            int64_t gmax = from_max_image(ex), gmin = from_min_image(en);
            const int64_t x = raw[k];
            if (kind == kNormIPA) {                // the holders of the extrema (k_tb_chain_pairs)
              hf |= (x == gmax ? 4u : 0u) | (x == gmin ? 8u : 0u);
            } else if (kind == kNormPTS && has_soft && !ign) {
              hf |= (x == gmax ? 1u : 0u) | (x == gmin ? 2u : 0u);
            }
            int64_t rv;
            if (kind == kNormPTS) {
              rv = 0;
              if (has_soft) {                      // counts -> scores (a non-decreasing map)
                if (!ign) rv = soft_score(x, w_soft, ms);
                if (ex) gmax = soft_score(gmax, w_soft, ms);
                if (en) gmin = soft_score(gmin, w_soft, ms);
              }
            } else {
              rv = x;
            }
            const int64_t nv = (kind == kNormPTS && ign) ? 0 : normalize_value(kind, rv, gmax, gmin, ipa_nonempty);
            tot += nv * prof_weight(prof, k);
          }
          int64_t dyn0 = 0;                        // the part a bind on this node moves
#pragma unroll
          for (int k = 0; k < KSIM_MAX_SCORE; k++) {
            if (k == k_fit) dyn0 += bp->w_fit * raw[k];
            if (k == k_ba) dyn0 += bp->w_ba * raw[k];
          }
          stat = (int32_t)(tot - dyn0);
          key = tb_key(tot, seed, seq, c.base + node);
        } else {                                   // one feasible node: schedulePod takes it unscored
          stat = kStatOne;
          key = tb_key(0, seed, seq, c.base + node);
        }
      }
      s.tb_stat[tb_pj(j, sl) * N + node] = stat;
    }
    // holder counts (runs that cross a class conflict): one popcount per wave,
    // one atomic per block and counter (after block_top_t's barrier)
    if (cross) {
#pragma unroll
      for (int h = 0; h < 4; h++) {
        const int32_t n = (int32_t)__popcll(__ballot((hf >> h) & 1u));
        if (lane == 0) s_hold[wv][h] = n;
      }
    }
    const size_t cb = tb_pj(j, sl) * kTbMaxBlocks + blockIdx.x;
    block_top_t(key, rdom, s_cand, s_cdom, s.tb_clist + cb * kTopT, vcol >= 0 ? s.tb_cdom + cb * kTopT : nullptr,
                s.tb_ccnt + cb);
    if (cross && threadIdx.x < 4) {
      int kp = -1, ki = -1;                        // the profile's slots (block-uniform)
      for (int k = 0; k < S; k++) {
        const int32_t kind = norm_kind(prof_score(prof, k));
        if (kind == kNormPTS) kp = k;
        if (kind == kNormIPA) ki = k;
      }
      const int h = threadIdx.x, k = h < 2 ? kp : ki;
      const int32_t n = s_hold[0][h] + s_hold[1][h] + s_hold[2][h] + s_hold[3][h];
      int32_t* hold = vuse >= 0 ? s.tb_vhold + tb_pj(j, sl) * 2 * KSIM_MAX_SCORE : q.win->hold;
      if (k >= 0 && n) atomicAdd(&hold[2 * k + (h & 1)], n);
    }
  }
#ifdef KSIM_TB_CLOCKS
  if (threadIdx.x == 0) {
    atomicAdd(&s.dbg[9], (unsigned long long)(x1 - x0));
    atomicAdd(&s.dbg[10], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - x1));
    atomicAdd(&s.dbg[11], 1ull);
    atomicAdd(&s.dbg[12], 1ull);
  }
#endif
}

// Pod j's exact top-T of slot sl from its blocks' exact lists (the pod's
// top-T lies in the union of the blocks' top-T): one wave, lane b holds block
// b's list (loaded before the batch state, as in k_tb_select), with the
// run-column value id of each key.  xsend (replicas, slot 0): the record
// [kTbPods][kTbXRec] of this replica's range (keys, count, holder counts)
// instead of the pod's lists.
__global__ __launch_bounds__(64) void k_tb_merge(DevCluster c, DevPods P, const DevState* __restrict__ st,
                                                 DevScratch s, uint64_t* __restrict__ xsend, int32_t plain) {
  const int lane = threadIdx.x;
  const int32_t j = blockIdx.x, sl = blockIdx.y;
  const size_t pj = tb_pj(j, sl);
  const int32_t nblk = (c.eval_hi - c.eval_lo + 255) / 256;
  const size_t cl = pj * kTbMaxBlocks + lane;
  uint64_t L[kTopT];
  uint32_t Ld = 0;                                 // value ids, 4 bits per entry
  int32_t cnt = 0;
  if (lane < nblk) {
    cnt = s.tb_ccnt[cl];
#pragma unroll
    for (int e = 0; e < kTopT; e++) L[e] = s.tb_clist[cl * kTopT + e];
    if (!plain) {
      const uint64_t db = *reinterpret_cast<const uint64_t*>(s.tb_cdom + cl * kTopT);
#pragma unroll
      for (int e = 0; e < kTopT; e++) Ld |= (uint32_t)((db >> (8 * e)) & 15u) << (4 * e);
    }
  }
  const int32_t nslot = s.tb_var[j].nslot, vcol = s.tb_var[j].vcol;
  const int32_t nf = s.tb_vnf[pj];
  if (j >= tb_count(st, P, plain)) return;
  if (sl >= nslot) return;
#pragma unroll
  for (int e = 0; e < kTopT; e++)
    if (e >= cnt) L[e] = 0;
  uint64_t mine = 0;
  uint32_t mdom = 0;
  int32_t n = 0;
#pragma unroll 1
  for (int e = 0; e < kTopT; e++) {
    const uint64_t mx = wave_max_u64_dpp(L[0]);
    if (mx == 0) break;
    const uint64_t own = __ballot(L[0] == mx);     // keys are unique: one lane
    const uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)(Ld & 15u), (int)__builtin_ctzll(own));
    if (lane == e) {
      mine = mx;
      mdom = d;
    }
    n = e + 1;
    if (L[0] == mx) {                              // pop the head (a register shift)
#pragma unroll
      for (int x = 0; x + 1 < kTopT; x++) L[x] = L[x + 1];
      L[kTopT - 1] = 0;
      Ld >>= 4;
    }
  }
  if (xsend) {
    uint64_t* r = xsend + (size_t)j * kTbXRec;
    if (lane < kTopT) r[lane] = lane < n ? mine : 0;
    if (lane == 0) r[kTopT] = (uint64_t)n;
    if (lane < KSIM_MAX_SCORE)
      r[kTopT + 1 + lane] = (uint64_t)(uint32_t)s.tb_win[j].hold[2 * lane] |
                            ((uint64_t)(uint32_t)s.tb_win[j].hold[2 * lane + 1] << 32);
    return;
  }
  if (lane < kTopT) {
    s.topk[pj * kTopT + lane] = lane < n ? mine : 0;
    if (vcol >= 0) s.tb_kdom[pj * kTopT + lane] = (uint8_t)(lane < n ? mdom : 0u);
  }
  if (lane == 0) {
    s.topk_cnt[pj] = n;
    s.topk_complete[pj] = nf <= kTopT ? 1 : 0;     // every feasible node listed
  }
}

// Replicas: pod j's counters and extrema over every replica's range (thread j).
__global__ __launch_bounds__(kTbPods) void k_tb_wmerge(DevScratch s, int32_t world) {
  const int32_t j = threadIdx.x;
  const WinState* w = reinterpret_cast<const WinState*>(s.tb_xrecv);
  WinState& o = s.tb_win[j];
  int32_t nf = 0, ni = 0;
  uint32_t tf = 0;
  uint64_t ext[2 * KSIM_MAX_SCORE];
#pragma unroll
  for (int x = 0; x < 2 * KSIM_MAX_SCORE; x++) ext[x] = 0;
  for (int32_t r = 0; r < world; r++) {
    const WinState& x = w[(size_t)r * kTbPods + j];
    nf += x.nfeas;
    ni += x.nign;
    tf |= x.tflags;                                // the same tables on every replica
#pragma unroll
    for (int e = 0; e < 2 * KSIM_MAX_SCORE; e++) ext[e] = umax64(ext[e], x.ext[e]);
  }
  o.nfeas = nf;
  o.nign = ni;
  o.tflags = tf;
#pragma unroll
  for (int e = 0; e < 2 * KSIM_MAX_SCORE; e++) o.ext[e] = ext[e];
}

// Replicas: pod j's exact global top-T from the replicas' exact range lists
// (one wave; lane l holds list entry l % T of replica l / T), and its holder
// counts summed.
__global__ __launch_bounds__(64) void k_tb_gmerge(DevPods P, const DevState* __restrict__ st, DevScratch s,
                                                  int32_t world) {
  static_assert(kTopT * kMaxShards <= 64, "k_tb_gmerge: one list entry per lane");
  const int lane = threadIdx.x;
  const int32_t j = blockIdx.x;
  if (j >= tb_count(st, P, 1)) return;
  const size_t pj = tb_pj(j, 0);
  const int32_t r = lane / kTopT, e = lane % kTopT;
  uint64_t key = 0;
  if (r < world) {
    const uint64_t* rec = s.xrecv + ((size_t)r * kTbPods + j) * kTbXRec;
    if ((uint64_t)e < rec[kTopT]) key = rec[e];
  }
  int32_t rank = 0;                                // keys are unique (node-specific) or 0
  for (int x = 0; x < 64; x++) {
    const uint64_t o = __shfl(key, x, 64);
    rank += o > key;
  }
  const int32_t n = __popcll(__ballot(key != 0));
  if (key != 0 && rank < kTopT) s.topk[pj * kTopT + rank] = key;
  if (lane >= n && lane < kTopT) s.topk[pj * kTopT + lane] = 0;
  if (lane == 0) {
    s.topk_cnt[pj] = n < kTopT ? n : kTopT;
    s.topk_complete[pj] = s.tb_win[j].nfeas <= kTopT ? 1 : 0;
  }
  if (lane < KSIM_MAX_SCORE) {
    uint32_t hmax = 0, hmin = 0;
    for (int32_t q = 0; q < world; q++) {
      const uint64_t h = s.xrecv[((size_t)q * kTbPods + j) * kTbXRec + kTopT + 1 + lane];
      hmax += (uint32_t)h;
      hmin += (uint32_t)(h >> 32);
    }
    s.tb_win[j].hold[2 * lane] = (int32_t)hmax;
    s.tb_win[j].hold[2 * lane + 1] = (int32_t)hmin;
  }
}

// A local change of one normalized raw score (PodTopologySpread counts,
// InterPodAffinity scores) on a node pod j keeps S0's extrema when the new
// value stays inside [gmin, gmax] and, if the node held an extremum, more nodes
// held it than the batch moves (at most j: one guessed node per earlier pod).
__device__ __forceinline__ bool tb_keeps_extrema(int64_t x0, int64_t x1, int64_t gmax, int64_t gmin, int32_t hmax,
                                                 int32_t hmin, int32_t j) {
  if (x1 > gmax || x1 < gmin) return false;
  if (x1 != x0 && x0 == gmax && hmax <= j) return false;
  if (x1 != x0 && x0 == gmin && hmin <= j) return false;
  return true;
}

// The topology batch's chain (tb_chain): node ids of the cluster index the
// guess table directly (tbatch_admit: at most kTbMaxBlocks x 256 nodes).
constexpr int kTbHoldSlots = kTbMaxBlocks * 256;
constexpr int kTbChainRounds = kTbPods + 2;        // pod i is exact after round i + 1
struct TbChainLds {
  uint32_t hold[kTbHoldSlots];                     // (round << 8) | (255 - pod): the lowest pod guessing the node
  uint64_t lst[kTbPods][kVarSlots][kTopT];         // each pod's lists per slot (the keys of the guesses)
  uint64_t gk[kTbPods];
  int32_t slot[kTbPods];
  int32_t nchain;
};


// The chain's inputs for lane i = pod i (every pod slot, every list slot:
// none of it waits for the batch state), in registers.
struct TbChainIn {
  uint64_t k0[kVarSlots][kTopT];                   // the lists' keys
  uint64_t dk[kVarSlots];                          // their run-column value ids, a byte each
  int32_t cnt[kVarSlots], comp[kVarSlots];
  int32_t nslot, adder;
  uint32_t sopk;                                   // slot_of, 3 bits per landing domain
};
__device__ __forceinline__ void tb_chain_load(TbChainIn& in, const DevScratch& s) {
  const int i = threadIdx.x;                       // wave 0
  in.nslot = 0;
  in.adder = -1;
  in.sopk = 0;
#pragma unroll
  for (int sl = 0; sl < kVarSlots; sl++) {
    in.cnt[sl] = in.comp[sl] = 0;
    in.dk[sl] = 0;
#pragma unroll
    for (int e = 0; e < kTopT; e++) in.k0[sl][e] = 0;
  }
  if (i >= kTbPods) return;
  const TbVar& V = s.tb_var[i];
  in.nslot = V.nslot;
  in.adder = V.adder;
#pragma unroll
  for (int w = 0; w < kVarSlots; w++) in.sopk |= (uint32_t)V.slot_of[w] << (3 * w);
#pragma unroll
  for (int sl = 0; sl < kVarSlots; sl++) {
    const size_t pj = tb_pj(i, sl);
    in.cnt[sl] = s.topk_cnt[pj];
    in.comp[sl] = s.topk_complete[pj];
    in.dk[sl] = *reinterpret_cast<const uint64_t*>(s.tb_kdom + pj * kTopT);
#pragma unroll
    for (int e = 0; e < kTopT; e++) in.k0[sl][e] = s.topk[pj * kTopT + e];
  }
}

// The greedy chain of one topology batch in one wave (lane i = pod i < nb):
// each pod takes the first entry of its current slot's list that no earlier
// pod guesses, its slot being the one its adder's current guess lands in
// (slot 0 without an adder).  Rounds run to the fixpoint: pod i depends only
// on pods before it, so pods [0, r) are exact after round r.  Then the exact
// prefix is cut before a pod whose incomplete list ran out.  The lists' node
// ids, value ids, counts and slot map stay in registers (a round is one LDS
// atomic, one lane exchange and one batch of independent guess-table reads).
// Writes L.gk (0: none or past the prefix), L.slot and L.nchain.
__device__ __forceinline__ void tb_chain(TbChainLds& L, const TbChainIn& in, int32_t nb, int32_t vcol,
                                         unsigned long long* __restrict__ dbg, uint64_t t0) {
  const int i = threadIdx.x;                       // wave 0
  const bool live = i < nb;
  const int32_t nslot = live ? in.nslot : 0, adder = live ? in.adder : -1;
  const uint32_t sopk = in.sopk;
  uint32_t cpk = 0, comp = 0;                      // counts (4 bits per slot), complete flags (1 bit per slot)
#pragma unroll
  for (int sl = 0; sl < kVarSlots; sl++)
    if (sl < nslot) {
      cpk |= (uint32_t)min(in.cnt[sl], kTopT) << (4 * sl);
      comp |= (in.comp[sl] ? 1u : 0u) << sl;
    }
  static_assert(kTopT <= 15 && 4 * kTopT <= 32, "tb_chain packing");
  int32_t nn[kVarSlots][kTopT];                    // node ids (-1 past the count)
  uint32_t dpk[kVarSlots];                         // value ids, 4 bits per entry
#pragma unroll
  for (int sl = 0; sl < kVarSlots; sl++) {
    dpk[sl] = 0;
    const int32_t cn = (int32_t)((cpk >> (4 * sl)) & 15u);
#pragma unroll
    for (int e = 0; e < kTopT; e++) {
      nn[sl][e] = e < cn ? key_node(in.k0[sl][e]) : -1;
      if (sl < nslot) L.lst[i][sl][e] = in.k0[sl][e];
      if (nn[sl][e] >= 0) {
        L.hold[nn[sl][e] & (kTbHoldSlots - 1)] = 0u;
        if (vcol >= 0) dpk[sl] |= (uint32_t)min((uint32_t)((in.dk[sl] >> (8 * e)) & 255u), (uint32_t)kVarDom) << (4 * e);
      }
    }
  }
  wave_lds_sync();
  TB_CLOCK(t1);
  int cs = 0, ca = (live && (cpk & 15u)) ? 0 : -1;  // current slot and entry
  int32_t gnode = ca >= 0 ? nn[0][0] : -1;
  int32_t gdom = ca >= 0 ? (int32_t)(dpk[0] & 15u) : 0;
  int32_t first = nb, rounds = 0;
  for (int32_t r = 1; r <= kTbChainRounds; r++) {
    rounds = r;
    if (gnode >= 0) atomicMax(&L.hold[gnode & (kTbHoldSlots - 1)], ((uint32_t)r << 8) | (uint32_t)(255 - i));
    wave_lds_sync();
    const int32_t ad = __shfl(gdom, adder >= 0 ? adder : 0, 64);
    const int ns = (live && adder >= 0) ? (int)((sopk >> (3 * ad)) & 7u) : 0;
    const int32_t cn = (int32_t)((cpk >> (4 * ns)) & 15u);
    int32_t sel[kTopT];
    uint32_t dsel = dpk[0];
#pragma unroll
    for (int e = 0; e < kTopT; e++) sel[e] = nn[0][e];
#pragma unroll
    for (int sl = 1; sl < kVarSlots; sl++) {
      const bool on = ns == sl;
      dsel = on ? dpk[sl] : dsel;
#pragma unroll
      for (int e = 0; e < kTopT; e++) sel[e] = on ? nn[sl][e] : sel[e];
    }
    uint32_t h[kTopT];                             // independent reads, one wait
#pragma unroll
    for (int e = 0; e < kTopT; e++) h[e] = L.hold[(sel[e] >= 0 ? sel[e] : 0) & (kTbHoldSlots - 1)];
    int na = -1;
#pragma unroll
    for (int e = kTopT - 1; e >= 0; e--) {
      const bool held = (h[e] >> 8) == (uint32_t)r && (int)(255 - (h[e] & 255u)) < i;
      if (e < cn && !held) na = e;
    }
    const uint64_t chg = __ballot(live && (ns != cs || na != ca));
    cs = ns;
    ca = na;
    int32_t g = -1;
#pragma unroll
    for (int e = 0; e < kTopT; e++) g = e == na ? sel[e] : g;
    gnode = g;
    gdom = na >= 0 ? (int32_t)((dsel >> (4 * na)) & 15u) : 0;
    if (!chg) {
      first = nb;
      break;
    }
    first = (int32_t)__builtin_ctzll(chg);
  }
  TB_CLOCK(t2);
  // exact prefix [0, first); an exhausted incomplete list inside it cuts the chain
  const uint64_t bad = __ballot(live && i < first && ca < 0 && !((comp >> cs) & 1u));
  const int32_t nchain = bad ? min(first, (int32_t)__builtin_ctzll(bad)) : first;
  if (i < kTbPods) {
    L.gk[i] = (i < nchain && ca >= 0) ? L.lst[i][cs][ca] : 0;
    L.slot[i] = cs;
  }
  if (i == 0) L.nchain = nchain;
#ifdef KSIM_TB_CLOCKS
  if (i == 0 && dbg && blockIdx.x == 0) {
    atomicAdd(&dbg[0], (unsigned long long)(t1 - t0));
    atomicAdd(&dbg[1], (unsigned long long)(t2 - t1));
    atomicAdd(&dbg[2], (unsigned long long)rounds);
    atomicAdd(&dbg[4], 1ull);
  }
#else
  (void)dbg;
  (void)t0;
  (void)rounds;
#endif
}

// Block j: the chain, then pod j's keys on the guesses of pods k < j after
// those binds (thread k: pod k's guess), or pinv[j] when pod j's S0 lists no
// longer describe it.  Pod k's bind moves pod j's inputs only on its guessed
// node g: the resources and, in a run that crosses a class conflict
// (kPodTbCross), the classes pod k adds through pod j's node-local uses (its
// zone-variant use aside: the slot holds that move).  The key on g is the
// slot's stat with the resource part and the changed PodTopologySpread /
// InterPodAffinity raw scores recomputed against the slot's extrema; pinv
// when a change would move an extremum, the feasible set (a node's verdict)
// or an emptiness flag.  What does not depend on the guesses (the lists, pod
// k's requests and add entries) is loaded before the chain runs.
// pp (replicas): pair maxima and pinv into pp[j] / pp[kTbPods + j], keyed
// only on the guesses in this replica's range (the all-reduce max combines).
constexpr int kPairAdds = 4;                       // pod k's add entries held in registers
__global__ __launch_bounds__(kBatchPods) void k_tb_chain_pairs(DevCluster c, DevPods P,
                                                               const ksim_profile* __restrict__ prof_p,
                                                               const BatchProg* __restrict__ bp_p,
                                                               const DevState* __restrict__ st, DevScratch s,
                                                               uint64_t* __restrict__ pp, int32_t plain) {
  __shared__ TbChainLds L;
  __shared__ uint64_t s_wmax[kBatchPods / 64];
  __shared__ int32_t s_winv[kBatchPods / 64];
  __shared__ TbDom s_dom[kVarDom + 1];             // pod j's domains; [kVarDom]: its tb_win counters / extrema
  __shared__ ksim_topo_use s_use[KSIM_MAX_USES];   // pod j's uses
  __shared__ UseMasks s_m;                         // ... and their roles
  __shared__ int32_t s_nu;
  uint64_t t0 = 0;
#ifdef KSIM_TB_CLOCKS
  t0 = __builtin_amdgcn_s_memrealtime();
#endif
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j = blockIdx.x, k = tid;
  TbChainIn in;
  if (threadIdx.x < 64) tb_chain_load(in, s);
  if (tid >= 64) {                                 // pod j's counters and extrema, staged while the chain runs
    constexpr int W = kVarDom * (int)(sizeof(TbDom) / 4);
    const int x = tid - 64;
    if (x < W) reinterpret_cast<int32_t*>(s_dom)[x] = reinterpret_cast<const int32_t*>(s.tb_dom + (size_t)j * kVarDom)[x];
    const int y = x - W;
    if (y >= 0 && y < 2 * KSIM_MAX_SCORE) s_dom[kVarDom].ext[y] = s.tb_win[j].ext[y];
    if (y == 2 * KSIM_MAX_SCORE) s_dom[kVarDom].nfeas = s.tb_win[j].nfeas;
    if (y == 2 * KSIM_MAX_SCORE + 1) s_dom[kVarDom].nign = s.tb_win[j].nign;
  }
  const int32_t nbt = tb_count(st, P, plain);
  if (nbt <= 0) return;                            // block-uniform
  const int32_t base = st->cursor;
  if (j < nbt && tid >= 128 && tid < 128 + KSIM_MAX_USES) {   // pod j's uses and roles, staged while the chain runs
    const ksim_pod& pj = P.pods[base + j];
    const int x = tid - 128;
    if (x < pj.use_count) s_use[x] = P.uses[pj.use_first + x];
    if (x == 0) {
      s_m = P.plans[base + j].m;
      s_nu = pj.use_count;
    }
  }
  // pod k's requests and first add entries (its pair's guess-independent inputs)
  const bool kin = k < j && k < nbt;
  ksim_pod pk{};
  int32_t acls[kPairAdds], acnt[kPairAdds];
#pragma unroll
  for (int a = 0; a < kPairAdds; a++) acls[a] = acnt[a] = 0;
  if (kin) {
    pk = P.pods[base + k];
#pragma unroll
    for (int a = 0; a < kPairAdds; a++)
      if (a < pk.add_count) {
        const ksim_class_add x = P.adds[pk.add_first + a];
        acls[a] = x.cls;
        acnt[a] = x.count;
      }
  }
  if (threadIdx.x < 64)
    tb_chain(L, in, nbt, plain ? -1 : (int32_t)(P.plans[base].flags >> kPlanVcolShift) - 1, s.dbg, t0);
  lds_barrier();
  const int32_t nchain = L.nchain;
  const uint64_t gk = k < nbt ? L.gk[k] : 0;
  if (j == 0) {
    if (tid < nbt) {
      s.gkey[tid] = gk;
      s.tb_slot[tid] = L.slot[tid];
    }
    if (tid == 0) *s.chain_end = nchain;
  }
  if (j >= nchain) {                               // block-uniform
    if (tid == 0) {
      if (pp) {
        pp[j] = 0;
        pp[kTbPods + j] = 0;
      } else {
        s.pmax[j] = 0;
        s.pinv[j] = 0;
      }
    }
    return;
  }
  const ksim_profile& prof = *prof_p;
  const BatchProg& bp = *bp_p;
  const int64_t seq0 = st->pod_seq;
  const int32_t N = c.n;
  const ksim_pod& p = P.pods[base + j];
  const bool cross = (P.bflags[base] & kPodTbCross) != 0;
  const int32_t sj = L.slot[j];
  const TbVar& Vj = s.tb_var[j];
  const int32_t vskip = Vj.adder >= 0 ? Vj.use : -1;   // the use the slot accounts for
  int kp = -1, ki = -1;                            // the profile's PodTopologySpread / InterPodAffinity slots
  for (int kk = 0; kk < prof.n_score; kk++) {
    const int32_t kind = norm_kind(prof_score(prof, kk));
    if (kind == kNormPTS) kp = kk;
    if (kind == kNormIPA) ki = kk;
  }
  UseMasks m{};
  const ksim_topo_use* U = s_use;                  // LDS
  const WinState* win = s.tb_win + j;
  uint32_t tf = 0;
  int soft = -1, nu = 0;
  if (cross) {
    m = s_m;
    nu = s_nu;
    tf = win->tflags;
    soft = m.soft ? 31 - __builtin_clz(m.soft) : -1;
  }
  uint64_t v = 0;
  bool inv = false;
  const int32_t local = (k < j && gk) ? key_node(gk) - c.base : -1;
  if (local >= 0 && local < N) {
    const bool own = local >= c.eval_lo && local < c.eval_hi;   // S0 values of g live on its replica
    // the guess's loads, all independent: stat, row, the uses' values, the raw scores
    const int32_t sv = own ? s.tb_stat[tb_pj(j, sj) * N + local] : kStatNone;
    NodeRow r{};
    if (own) r = load_row(c, local);
    uint32_t lv[KSIM_MAX_USES];
#pragma unroll
    for (int i = 0; i < KSIM_MAX_USES; i++) lv[i] = i < nu ? use_value(c, U[i], local) : 0u;
    const bool ign_g = own && soft >= 0 && s.tb_ign[(size_t)j * N + local] != 0;
    const int64_t xp0 = (own && kp >= 0) ? s.tb_raw[((size_t)j * KSIM_MAX_SCORE + kp) * N + local] : 0;
    const int64_t xi0 = (own && ki >= 0) ? s.tb_raw[((size_t)j * KSIM_MAX_SCORE + ki) * N + local] : 0;
    // what pod k's adds change for pod j on g = local (runs that cross only)
    int64_t d_soft = 0, d_ipa = 0;
    bool hit_anti = false, hit_aff = false, hit_score = false;
#pragma unroll
    for (int i = 0; i < KSIM_MAX_USES; i++) {
      if (i >= nu) break;
      if (i == vskip) continue;
      const ksim_topo_use u = U[i];
      if (u.cls < 0) continue;
      int32_t d = 0;
#pragma unroll
      for (int a = 0; a < kPairAdds; a++) d += acls[a] == u.cls && a < pk.add_count ? acnt[a] : 0;
      for (int a = kPairAdds; a < pk.add_count; a++) {
        const ksim_class_add x = P.adds[pk.add_first + a];
        if (x.cls == u.cls) d += x.count;
      }
      if (d == 0) continue;
      const uint32_t b = 1u << i;
      if ((m.node_count & b) && !(m.hard & b)) {   // g's own count
        if (lv[i] == 0) continue;                  // the use ignores a node without its key
        if ((m.anti | m.exist) & b) hit_anti = true;
        if (m.aff & b) hit_aff = true;
        if (m.score & b) {
          hit_score = true;
          d_ipa += ipa_coef(prof, u) * d;
        }
        if (i == soft) d_soft += d;
      } else {
        inv = true;                                // a domain-keyed use (the host ends runs there)
      }
    }
    if (hit_aff && !(tf & kTopoAffinityNonEmpty)) inv = true;   // len(affinityCounts) would change
    if (hit_score && !(tf & kTopoScoreNonEmpty)) inv = true;    // len(topologyScore) would change
    if (!own) {
    } else if (sv != kStatNone) {
      row_add_pod(r, pk, 1);
      if (hit_anti || (bp.has_fit_filter && fits_request(r, p, c.n_scalar, c.fit_ignore))) {
        inv = true;                                // a node of the slot's feasible set stops passing
      } else {
        int64_t tot = 0;
        if (sv != kStatOne) {
          tot = sv;
          if (d_soft || d_ipa) {                   // the changed topology scores, the slot's extrema
            // the slot's counters and extrema from the staged records
            const uint32_t mk = Vj.use >= 0 ? Vj.mask[sj] : ~0u;
            int32_t nf = 0, nign = 0;
            if (Vj.use < 0) {
              nf = s_dom[kVarDom].nfeas;
              nign = s_dom[kVarDom].nign;
            } else {
              for (int d = 0; d < kVarDom; d++)
                if (d < Vj.ndom && ((mk >> d) & 1u)) {
                  nf += s_dom[d].nfeas;
                  nign += s_dom[d].nign;
                }
            }
            auto ext_of = [&](int e) -> uint64_t {
              if (Vj.use < 0) return s_dom[kVarDom].ext[e];
              if ((Vj.zmask >> (e >> 1)) & 1u) return nf > 0 ? ((e & 1) ? min_image(0) : max_image(0)) : 0ull;
              uint64_t x = 0;
              for (int d = 0; d < kVarDom; d++)
                if (d < Vj.ndom && ((mk >> d) & 1u)) x = umax64(x, s_dom[d].ext[e]);
              return x;
            };
            const int32_t* hold = Vj.use >= 0 ? s.tb_vhold + tb_pj(j, sj) * 2 * KSIM_MAX_SCORE : win->hold;
            const bool ipa_ne = (tf & kTopoScoreNonEmpty) != 0;
            for (int h = 0; h < 2; h++) {          // PodTopologySpread, then InterPodAffinity
              const int kk = h == 0 ? kp : ki;
              const bool pts = h == 0 && kp >= 0 && d_soft != 0 && soft >= 0 && !ign_g;
              const bool ipa = h == 1 && ki >= 0 && d_ipa != 0;
              if (!pts && !ipa) continue;
              const int32_t kind = h == 0 ? kNormPTS : kNormIPA;
              const int64_t x0 = pts ? xp0 : xi0;
              const int64_t x1 = x0 + (pts ? d_soft : d_ipa);
              int64_t gmax = from_max_image(ext_of(2 * kk)), gmin = from_min_image(ext_of(2 * kk + 1));
              if (!tb_keeps_extrema(x0, x1, gmax, gmin, hold[2 * kk], hold[2 * kk + 1], j)) {
                inv = true;
                break;
              }
              int64_t r0 = x0, r1 = x1;
              if (pts) {                           // counts -> scores (topologyNormalizingWeight, hostname)
                const ksim_topo_use u = U[soft];
                const double wt = c.topo_log[(u.flags & KSIM_USEF_HOSTNAME) ? nf - nign : 0];
                r0 = soft_score(x0, wt, u.arg);
                r1 = soft_score(x1, wt, u.arg);
                gmax = soft_score(gmax, wt, u.arg);
                gmin = soft_score(gmin, wt, u.arg);
              }
              tot += prof_weight(prof, kk) *
                     (normalize_value(kind, r1, gmax, gmin, ipa_ne) - normalize_value(kind, r0, gmax, gmin, ipa_ne));
            }
          }
          if (bp.w_fit) tot += bp.w_fit * fit_score(r, prof, p, c.n_scalar);
          if (bp.w_ba) tot += bp.w_ba * balanced_allocation_score(r, prof, p, c.n_scalar);
        }
        if (!inv) v = tb_key(tot, prof.tiebreak_seed, seq0 + j, c.base + local);
      }
    } else if (hit_aff) {
      inv = true;                                  // required affinity may now pass on g
    }
  }
  v = wave_max_u64_dpp(v);
  const uint64_t b = __ballot(inv);
  if (lane == 0) {
    s_wmax[wave] = v;
    s_winv[wave] = b != 0;
  }
  lds_barrier();
  if (wave == 0) {
    if (tid == 0) {
      uint64_t mx = 0;
      int32_t any = 0;
      for (int w = 0; w < kBatchPods / 64; w++) {
        mx = umax64(mx, s_wmax[w]);
        any |= s_winv[w];
      }
      if (pp) {
        pp[j] = mx;
        pp[kTbPods + j] = (uint64_t)any;
      } else {
        s.pmax[j] = mx;
        s.pinv[j] = any;
      }
#ifdef KSIM_TB_CLOCKS
      if (j == 0) atomicAdd(&s.dbg[3], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - t0));
      atomicAdd(&s.dbg[13], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - t0));
      atomicAdd(&s.dbg[14], 1ull);
#endif
    }
  }
}

// batch_commit, then the committed pods' count-class adds and persistent
// table updates as parallel atomics (one (pod, add) / (pod, table) pair per
// thread; a pod and the pod i* that binds on its node may share entries).
constexpr int kTbAddSlots = 8;                     // adds / table updates per pod and pass
static_assert(kTbPods <= kBatchPods / kTbAddSlots, "k_tb_commit: one thread group per pod");
__global__ __launch_bounds__(kBatchPods) void k_tb_commit(DevCluster c, DevPods P, DevState* __restrict__ st,
                                                          DevScratch s, int32_t* __restrict__ chosen_out,
                                                          const uint64_t* __restrict__ pp, int32_t plain) {
  __shared__ int32_t s_istar, s_sched, s_unsched;
  __shared__ int32_t s_node[kTbPods];
  const int tid = threadIdx.x;
  const uint64_t g = s.gkey[tid];                  // in flight with the state loads
  const uint64_t m = pp ? (tid < kTbPods ? pp[tid] : 0) : s.pmax[tid];
  const int32_t inv = tid < kTbPods ? (pp ? (int32_t)(pp[kTbPods + tid] != 0) : s.pinv[tid]) : 0;
  const int32_t nchain = *s.chain_end;
  const int32_t vslot = tid < kTbPods ? s.tb_slot[tid] : 0;
  const int q = tid / kTbAddSlots, e = tid % kTbAddSlots;
  const uint64_t gq = s.gkey[q];                   // pod q's guess (its node unless q is the cut pod)
  const int32_t base = st->cursor;
  const int32_t nbt = tb_count(st, P, plain);
  if (nbt <= 0) return;
  // pod q's add / table-update entry e, and the table update's value on the
  // guessed node: none of it waits for the commit
  ksim_class_add x0{-1, 0};
  int4 t0{0, 0, 0, 0};
  uint32_t pfl = 0, v0 = 0;
  int32_t acount = 0, afirst = 0, tcount = 0, tfirst = 0;
  const int32_t gnode = gq ? key_node(gq) - c.base : -1;
  if (q < nbt) {
    const ksim_pod& pq = P.pods[base + q];
    const PodPlan& plq = P.plans[base + q];
    acount = pq.add_count;
    afirst = pq.add_first;
    pfl = plq.flags;
    tcount = plq.tadd_count;
    tfirst = plq.tadd_first;
    if (e < acount) x0 = P.adds[afirst + e];
    if ((pfl & kPlanTadds) && e < tcount) {
      t0 = P.ptab_padd[tfirst + e];
      if (gnode >= 0 && gnode < c.n) v0 = c.labels[(size_t)t0.y * c.n + gnode];
    }
  }
  batch_commit(c, P, st, g, m, s.pmax, nchain, chosen_out, &s_istar, &s_sched, &s_unsched, nullptr, &inv, nbt,
               s_node);
  lds_barrier();                                   // s_node
  const int32_t node = q < nbt ? s_node[q] : -1;
  if (node >= 0) {
    for (int a = e; a < acount; a += kTbAddSlots) {
      const ksim_class_add x = a == e ? x0 : P.adds[afirst + a];
      atomicAdd(&c.cnt[(size_t)x.cls * c.n + node], x.count);
      if (!(pfl & kPlanTadds)) ptab_add(c, P, x.cls, node, (int64_t)x.count);
    }
    if (pfl & kPlanTadds)
      for (int a = e; a < tcount; a += kTbAddSlots) {
        const int4 t = a == e ? t0 : P.ptab_padd[tfirst + a];
        const uint32_t v = (a == e && node == gnode) ? v0 : c.labels[(size_t)t.y * c.n + node];
        if (v) atomicAdd(reinterpret_cast<unsigned long long*>(P.ptab + t.x + (t.z == kPtabTotal ? 0u : v)),
                         (unsigned long long)(int64_t)t.w);
      }
  }
  // committed pods whose slot moved their zone verdicts (ksim_get_diag out[26])
  const uint64_t vb = __ballot(tid < nbt && s_node[tid < kTbPods ? tid : 0] != -2 && vslot != 0);
  if ((tid & 63) == 0 && vb) atomicAdd(s.tb_vpods, (unsigned long long)__popcll(vb));
  // the next batch's counters and extrema start from zero (the rows this batch used)
  for (int x = tid; x < kTbPods * (int)(sizeof(WinState) / 4); x += blockDim.x)
    reinterpret_cast<int32_t*>(s.tb_win)[x] = 0;
  for (int x = tid; x < nbt * kVarDom * (int)(sizeof(TbDom) / 4); x += blockDim.x)
    reinterpret_cast<int32_t*>(s.tb_dom)[x] = 0;
  for (int x = tid; x < nbt * kVarSlots * 2 * KSIM_MAX_SCORE; x += blockDim.x) s.tb_vhold[x] = 0;
}

const char* const kTbatchKernelNames[kKernelsPerTbatch] = {"k_tb_filter", "k_tb_select", "k_tb_merge",
                                                           "k_tb_chain_pairs", "k_tb_commit"};

uint32_t launch_tbatch(const LaunchArgs& a, hipStream_t stream, hipEvent_t* evs) {
  const dim3 grid((a.c.n + 255) / 256, kTbPods);
  if (evs) (void)hipEventRecord(evs[0], stream);
  k_tb_filter<<<grid, 256, 0, stream>>>(a.c, a.P, a.dprof, a.dbp, a.st, a.s, 0);
  if (evs) (void)hipEventRecord(evs[1], stream);
  k_tb_select<<<dim3(grid.x, kTbPods, kVarSlots), 256, 0, stream>>>(a.c, a.P, a.dprof, a.dbp, a.st, a.s, 0);
  if (evs) (void)hipEventRecord(evs[2], stream);
  k_tb_merge<<<dim3(kTbPods, kVarSlots), 64, 0, stream>>>(a.c, a.P, a.st, a.s, nullptr, 0);
  if (evs) (void)hipEventRecord(evs[3], stream);
  k_tb_chain_pairs<<<kTbPods, kBatchPods, 0, stream>>>(a.c, a.P, a.dprof, a.dbp, a.st, a.s, nullptr, 0);
  if (evs) (void)hipEventRecord(evs[4], stream);
  k_tb_commit<<<1, kBatchPods, 0, stream>>>(a.c, a.P, a.st, a.s, a.chosen, nullptr, 0);
  if (evs) (void)hipEventRecord(evs[5], stream);
  return (1u << kKernelsPerTbatch) - 1;
}

void launch_tb_rep_filter(const LaunchArgs& a, hipStream_t stream) {
  const dim3 grid((a.c.eval_hi - a.c.eval_lo + 255) / 256, kTbPods);
  k_tb_filter<<<grid, 256, 0, stream>>>(a.c, a.P, a.dprof, a.dbp, a.st, a.s, 1);
}

void launch_tb_rep_select(const LaunchArgs& a, int32_t world, hipStream_t stream) {
  const dim3 grid((a.c.eval_hi - a.c.eval_lo + 255) / 256, kTbPods);
  k_tb_wmerge<<<1, kTbPods, 0, stream>>>(a.s, world);
  k_tb_select<<<grid, 256, 0, stream>>>(a.c, a.P, a.dprof, a.dbp, a.st, a.s, 1);
  k_tb_merge<<<dim3(kTbPods, 1), 64, 0, stream>>>(a.c, a.P, a.st, a.s, a.s.xsend, 1);
}

void launch_tb_rep_pairs(const LaunchArgs& a, int32_t world, hipStream_t stream) {
  k_tb_gmerge<<<kTbPods, 64, 0, stream>>>(a.P, a.st, a.s, world);
  k_tb_chain_pairs<<<kTbPods, kBatchPods, 0, stream>>>(a.c, a.P, a.dprof, a.dbp, a.st, a.s, a.s.tb_pp, 1);
}

void launch_tb_rep_commit(const LaunchArgs& a, hipStream_t stream) {
  k_tb_commit<<<1, kBatchPods, 0, stream>>>(a.c, a.P, a.st, a.s, a.chosen, a.s.tb_pp, 1);
}

}  // namespace ksim
