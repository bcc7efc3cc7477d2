// ksim_kernels.hip — HIP kernels of the scheduling cycle (gfx950).
//
// Three execution paths produce identical placements (each bit-exact with the
// oracle):
//
// A. Per-pod path (compat mode, and pods the batch paths cannot take), one
//    cycle per pod:
//    k_topo_prefilter / k_topo_min  PodTopologySpread / InterPodAffinity
//                    PreFilter maps as domain sums (a27, a29)
//    k_filter_score  grid over nodes: RunFilterPlugins (SURVEY §8(a) a17, a22,
//                    a25-a29) and, for feasible nodes, every raw Score (a23-a30)
//    k_window        numFeasibleNodesToFind window by a block prefix scan (a16)
//                    and PTS PreScore (a28); not launched when K = N
//    k_extrema       NormalizeScore extrema (a31) and PTS raw scores
//    k_select        weighted totals (a18), selectHost as a packed-u64 argmax
//                    (a19, TB tie-break)
//    k_bind          NodeInfo.AddPod (a20) and the scheduler state
// B. Batch paths (pods whose normalized plugins are constant over nodes):
//    ksim_batch.hip (P100), ksim_adapt.hip (ADAPT).
// C. The node-sharded per-pod cycle (below).
#include "ksim_device.h"
#include "ksim_internal.h"
#include "ksim_wave.h"
#include "ksim_cycle.h"

namespace ksim {

// ---- wave64 / block reductions ------------------------------------------------
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    uint64_t o = shfl_xor_u64(v, m);
    v = o > v ? o : v;
  }
  return v;
}

__device__ __forceinline__ int64_t wave_max_i64(int64_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    int64_t o = (int64_t)shfl_xor_u64((uint64_t)v, m);
    v = o > v ? o : v;
  }
  return v;
}

// Block max over u64 for a block of NW waves (all threads get the result).
template <int NW>
__device__ uint64_t block_max_u64(uint64_t v, uint64_t* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_max_u64(v);
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  uint64_t r = sh[0];
#pragma unroll
  for (int i = 1; i < NW; i++) r = sh[i] > r ? sh[i] : r;
  return r;
}

constexpr int kFinalThreads = 1024;
constexpr int kFinalWaves = kFinalThreads / 64;

__device__ int64_t block_max_i64(int64_t v, int64_t* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_max_i64(v);
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  int64_t r = sh[0];
  for (int i = 1; i < kFinalWaves; i++) r = sh[i] > r ? sh[i] : r;
  return r;
}

__device__ int64_t block_min_i64(int64_t v, int64_t* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_min_i64(v);
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  int64_t r = sh[0];
  for (int i = 1; i < kFinalWaves; i++) r = sh[i] < r ? sh[i] : r;
  return r;
}

// Exclusive prefix sum over the block + total.
__device__ void block_scan_i32(int32_t v, int32_t& excl, int32_t& total, int32_t* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    int32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  __syncthreads();
  if (lane == 63) sh[w] = x;
  __syncthreads();
  int32_t base = 0, tot = 0;
  for (int i = 0; i < kFinalWaves; i++) {
    if (i < w) base += sh[i];
    tot += sh[i];
  }
  excl = base + x - v;
  total = tot;
}

// Block-wide min over NW waves (all threads get the result).
template <int NW>
__device__ int64_t block_min_i64_nw(int64_t v, int64_t* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_min_i64(v);
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  int64_t r = sh[0];
#pragma unroll
  for (int i = 1; i < NW; i++) r = sh[i] < r ? sh[i] : r;
  return r;
}

template <int NW>
__device__ int32_t block_sum_i32_nw(int32_t v, int32_t* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  int32_t r = 0;
#pragma unroll
  for (int i = 0; i < NW; i++) r += sh[i];
  return r;
}

// ==== A. per-pod path ===========================================================
constexpr int kLdsDom = 128;   // domain tables of key columns with <= kLdsDom value ids are LDS-staged

// PreFilter of PodTopologySpread / InterPodAffinity plus the domain sums their
// PreScore needs: one thread per node, adds into the pod's domain tables (the
// pod's plan says which uses have one; LDS-staged for small key vocabularies).
__global__ __launch_bounds__(256) void k_topo_prefilter(DevCluster c, DevPods P, ksim_profile prof,
                                                        DevState* __restrict__ st, DevScratch s) {
  __shared__ unsigned long long s_dom[KSIM_MAX_USES][kLdsDom];
  __shared__ uint32_t s_flags;
  const int32_t pi = st->cursor;
  if (pi >= st->end) return;
  const ksim_pod p = P.pods[pi];                  // block-uniform: scalar loads
  const int nu = p.use_count;
  if (nu == 0) return;
  const PodPlan pp = P.plans[pi];
  if (pp.flags & kPlanPtab) return;                // persistent tables: nothing to sum
  const UseMasks& m = pp.m;
  const ksim_topo_use* U = P.uses + p.use_first;
  uint32_t lds = 0;                                // uses whose table is staged in LDS
  for (uint32_t b = m.dom; b; b &= b - 1) {
    const int i = __builtin_ctz(b);
    if (c.col_nvals[load_use(U, i).col] <= kLdsDom) lds |= 1u << i;
  }
  const int tid = threadIdx.x;
  for (int x = tid; x < nu * kLdsDom; x += blockDim.x) s_dom[x / kLdsDom][x % kLdsDom] = 0;
  if (tid == 0) s_flags = 0;
  // the PTS pair-registration rows the no-window filter pass fills for this
  // pod start empty (k_bind used to clear them after the cycle)
  if (blockIdx.x == 0 && m.soft_val) {
    const uint32_t vwords = (uint32_t)(c.vmax + 31) >> 5;
    for (uint32_t b = m.soft_val; b; b &= b - 1) {
      const int i = __builtin_ctz(b);
      const int32_t words = (c.col_nvals[load_use(U, i).col] + 31) >> 5;
      for (int x = tid; x < words; x += blockDim.x) s.regbm[(size_t)i * vwords + x] = 0;
    }
  }
  __syncthreads();
  const int32_t node = blockIdx.x * blockDim.x + tid;
  uint32_t flags = 0;
  if (node < c.n) {
    uint32_t val[KSIM_MAX_USES];
    int64_t cnt[KSIM_MAX_USES];
#pragma unroll
    for (int i = 0; i < KSIM_MAX_USES; i++) {      // every load of the node first
      val[i] = 0;
      cnt[i] = 0;
      if (i < nu) {
        const ksim_topo_use u = load_use(U, i);
        if (u.col != KSIM_COL_NONE) val[i] = c.labels[(size_t)u.col * c.n + node];
        cnt[i] = class_count(c, u.cls, node);
      }
    }
    // requireAllTopologies is false for system-defaulted constraints (PreScore)
    const bool sysdef = (p.topo_flags & KSIM_POD_PTS_SYSTEM_DEFAULT) != 0;
    bool all_hard = true, all_soft = true;         // nodeLabelsMatchSpreadConstraints per kind
#pragma unroll
    for (int i = 0; i < KSIM_MAX_USES; i++) {
      if (((m.hard >> i) & 1u) && val[i] == 0) all_hard = false;
      if (((m.soft >> i) & 1u) && val[i] == 0) all_soft = false;
      if (((m.aff >> i) & 1u) && val[i] != 0 && cnt[i] > 0) flags |= kTopoAffinityNonEmpty;
      if (((m.score >> i) & 1u) && val[i] != 0 && cnt[i] != 0) flags |= kTopoScoreNonEmpty;
    }
    // matchNodeInclusionPolicies, once per node for every spread use
    const uint32_t spread = m.hard | m.soft_val;
    const bool aff_ok = (m.honor_aff & spread) ? required_node_affinity_match(c, P, p, node) : true;
    const bool taint_ok = (m.honor_taints & spread) ? !node_has_untolerated_taint(c, p, node) : true;
#pragma unroll
    for (int i = 0; i < KSIM_MAX_USES; i++) {
      const uint32_t v = val[i];
      // no table, or the node has no pair for this key (system defaults: the pair (key, ""))
      if (!((m.dom >> i) & 1u) || (v == 0 && !(sysdef && ((m.soft_val >> i) & 1u)))) continue;
      const bool incl = (!((m.honor_aff >> i) & 1u) || aff_ok) && (!((m.honor_taints >> i) & 1u) || taint_ok);
      int64_t add = cnt[i];
      if ((m.hard >> i) & 1u)                      // TpPairToMatchNum[pair] += count (+ presence mark)
        add = all_hard && incl ? add + (1ll << kDomMarkShift) : 0;
      else if ((m.soft_val >> i) & 1u)             // TopologyPairToPodCounts
        add = (all_soft || sysdef) && incl ? add : 0;
      if (add == 0) continue;
      if ((lds >> i) & 1u)
        atomicAdd(&s_dom[i][v], (unsigned long long)add);
      else
        atomicAdd(reinterpret_cast<unsigned long long*>(s.dom + (size_t)i * c.vmax + v), (unsigned long long)add);
    }
  }
  if (flags) atomicOr(&s_flags, flags);
  __syncthreads();
  for (int x = tid; x < nu * kLdsDom; x += blockDim.x) {
    if (!((lds >> (x / kLdsDom)) & 1u)) continue;
    const unsigned long long v = s_dom[x / kLdsDom][x % kLdsDom];
    if (v) atomicAdd(reinterpret_cast<unsigned long long*>(s.dom + (size_t)(x / kLdsDom) * c.vmax + x % kLdsDom), v);
  }
  if (tid == 0 && s_flags) atomicOr(&st->topo_flags, s_flags);
}

// TpKeyToCriticalPaths: per hard constraint, the minimum over its present pairs
// (math.MaxInt32 when no eligible node carries the key).
// Sharded (SHARDED): first unpack the all-reduced domain sums (s.xdom, packed by
// k_dom_pack) into the domain tables and re-derive the two topology flags from
// them (every class count is >= 0, so a domain sum is non-zero exactly when
// some node's count is).
template <bool SHARDED>
__global__ __launch_bounds__(256) void k_topo_min(DevCluster c, DevPods P, ksim_profile prof,
                                                  DevState* __restrict__ st, DevScratch s) {
  __shared__ int64_t sh[4];
  __shared__ uint32_t s_flags;
  const int32_t pi = st->cursor;
  if (pi >= st->end) return;
  const ksim_pod& p = P.pods[pi];
  if (SHARDED) {
    if (threadIdx.x == 0) s_flags = 0;
    __syncthreads();
    uint32_t flags = 0;
    int64_t off = 0;
    for (int i = 0; i < p.use_count; i++) {
      const ksim_topo_use u = P.uses[p.use_first + i];
      if (!use_needs_dom(u)) continue;
      const int32_t V = c.col_nvals[u.col];
      int64_t* d = s.dom + (size_t)i * c.vmax;
      const bool aff = u.kind == KSIM_USE_IPA_AFFINITY, sc = ipa_coef(prof, u) != 0;
      for (int32_t v = threadIdx.x; v < V; v += blockDim.x) {
        const int64_t x = s.xdom[off + v];
        d[v] = x;
        if (aff && x > 0) flags |= kTopoAffinityNonEmpty;
        if (sc && x != 0) flags |= kTopoScoreNonEmpty;
      }
      off += V;
    }
    if (flags) atomicOr(&s_flags, flags);
    __syncthreads();
    if (threadIdx.x == 0) st->topo_flags = s_flags;
  }
  for (int i = 0; i < p.use_count; i++) {
    const ksim_topo_use u = P.uses[p.use_first + i];
    if (u.kind != KSIM_USE_PTS_HARD) continue;
    int64_t mn = 2147483647;
    if (u.col != KSIM_COL_NONE) {
      const int32_t V = c.col_nvals[u.col];
      const int64_t* d = s.dom + (size_t)i * c.vmax;
      for (int32_t v = threadIdx.x; v < V; v += blockDim.x) {
        const int64_t x = d[v];
        if ((x >> kDomMarkShift) != 0) {
          const int64_t m = x & kDomCountMask;
          mn = m < mn ? m : mn;
        }
      }
    }
    mn = block_min_i64_nw<4>(mn, sh);
    if (threadIdx.x == 0) s.min_match[i] = mn;
  }
}

// NOWIN (K = N: every feasible node is kept, no cut): the filter pass also
// counts the feasible nodes and does PodTopologySpread's PreScore pair
// registration and IgnoredNodes count (wave-aggregated atomics), so the cycle
// needs no k_window.
// fuse_min: every hard spread constraint of the run keys a column of at most
// kFuseMinValues values, so each block derives the critical paths itself
// (k_topo_min's work, a few LDS reductions) instead of a separate launch.
// fuse_ext (NOWIN runs whose pods carry at most one ScheduleAnyway spread
// constraint): the NormalizeScore extrema are taken here, so the cycle needs
// no k_extrema.  PodTopologySpread's raw score is then a non-decreasing
// function of one count (round(count * w + maxSkew - 1), w > 0 known only
// after the pass), so its slots hold the count extrema and k_select maps them.

// Extrema are atomicMax over order-preserving u64 images of an int64 (max
// image x ^ 2^63, min image ~(x ^ 2^63); 0 is the identity of both:
// ksim_device.h).

// Wave max of (img, lo) pairs in lexicographic order (selectHost over full
// int64 totals): the max image first, then the max lo among the lanes holding it.
__device__ __forceinline__ void wave_best2(uint64_t& img, uint64_t& lo) {
  const uint64_t m = wave_max_u64_dpp(img);
  lo = wave_max_u64_dpp(img == m ? lo : 0ull);
  img = m;
}
__device__ __forceinline__ void best2_merge(uint64_t& img, uint64_t& lo, uint64_t img2, uint64_t lo2) {
  if (img2 > img || (img2 == img && lo2 > lo)) {
    img = img2;
    lo = lo2;
  }
}

// KSIM_FS_CLOCKS builds: per-block phase times of k_filter_score (thread 0,
// 100 MHz realtime) summed into s.dbg[8 + phase], s.dbg[15] = blocks.
#ifdef KSIM_FS_CLOCKS
#define FS_CLK(k)                                                          \
  do {                                                                     \
    if (threadIdx.x == 0) {                                                \
      const uint64_t _t = __builtin_amdgcn_s_memrealtime();                \
      if ((k) > 0) atomicAdd(&s.dbg[8 + (k) - 1], (unsigned long long)(_t - fs_t)); \
      fs_t = _t;                                                           \
    }                                                                      \
  } while (0)
#else
#define FS_CLK(k) do {} while (0)
#endif

template <bool COMPAT, bool NOWIN>
__global__ __launch_bounds__(256) void k_filter_score(DevCluster c, DevPods P0, ksim_profile prof,
                                                      const BatchProg* __restrict__ bp,
                                                      DevState* __restrict__ st, DevScratch s,
                                                      int32_t fuse_min, int32_t fuse_ext) {
  __shared__ int64_t s_min[KSIM_MAX_USES];
  __shared__ uint64_t s_red[4][2 * KSIM_MAX_SCORE];
  __shared__ int32_t s_cnt[4][2];
  __shared__ uint32_t s_tf;
#ifdef KSIM_FS_CLOCKS
  uint64_t fs_t = 0;
#endif
  FS_CLK(0);
  const int32_t node = blockIdx.x * blockDim.x + threadIdx.x;
  // the node's row does not depend on the cycle: its loads go out before the
  // state / pod / plan chain
  const int32_t xr = node < c.n ? node : c.n - 1;
  const NodeRow r = load_row(c, xr);
  const double inv_c = c.inv_cpu[xr], inv_m = c.inv_mem[xr];
  // a framework-driven pass mirrored to the host (m_head) runs pod 0 of its
  // single-pod set (ksim_fw_prefilter's begin job): no state load first
  const bool fwm = COMPAT && s.m_head != nullptr;
  const int32_t pi = fwm ? 0 : st->cursor;
  if (!fwm && pi >= st->end) return;
  // the pod record and its uses sit at a block-uniform address: scalar loads
  const DevPods& P = P0;
  const ksim_pod& p = P0.pods[pi];                // block-uniform address: scalar loads where used
  const PodPlan pp = P0.plans[pi];                 // block-uniform: scalar loads
  const UseMasks& m = pp.m;
  const ksim_topo_use* U = P.uses + p.use_first;
  FS_CLK(1);
  // the node's topology inputs depend on the pod's uses only: their loads go
  // out before the critical-path phase and its barrier
  TopoRow t;
  if (p.use_count) load_topo_row(c, U, p.use_count, m, s, P0.ptab, xr, t);
  const bool pt = (pp.flags & kPlanPtab) != 0;    // block-uniform: persistent tables
  if ((fuse_min && m.hard) || (pt && (m.aff | m.score))) {
    // k_select's normalization reads the flags from the state
    topo_block_setup(c, P0, s, U, m, pt, fuse_min != 0, s_min, &s_tf, &st->topo_flags);
    __syncthreads();
    if (fuse_min && m.hard) s.min_match = s_min;   // pts_filter reads the block's copy
  }
  FS_CLK(2);
  bool feasible = false, ign = false;
  RawScores rv{};                                  // normalized plugins' raw scores (fused extrema)
  int64_t soft_cnt = 0;                            // PodTopologySpread: the node's count for the soft use
  const int soft = m.soft ? 31 - __builtin_clz(m.soft) : -1;   // the pod's last ScheduleAnyway use
  bool scanned = true;
  if (p.flags & KSIM_POD_NODE_NAMES)              // block-uniform: NodeAffinity's PreFilterResult
    scanned = node < c.n && scan_pos(scan_set(c, P, p, st->next_start), c.base + node) >= 0;
  if (fwm && blockIdx.x == 0 && threadIdx.x == 0) s.m_head[0] = st->next_start;
  if (node < c.n && !scanned) {                   // never handed to Filter
    s.fail[node] = KSIM_NOT_EVALUATED;
    if (COMPAT) s.detail[node] = 0;
    if (COMPAT && s.m_fail) s.m_fail[node] = KSIM_NOT_EVALUATED;
    if (COMPAT && s.m_detail) s.m_detail[node] = 0;
  } else if (node < c.n) {
    const uint32_t tf = !p.use_count ? 0u : pt ? ((m.aff | m.score) ? s_tf : 0u) : st->topo_flags;
#ifdef KSIM_FS_CLOCKS
    __builtin_amdgcn_s_waitcnt(0);
    if (threadIdx.x == 0) {
      const uint64_t _t = __builtin_amdgcn_s_memrealtime();
      atomicAdd(&s.dbg[13], (unsigned long long)(_t - fs_t));
    }
#endif
    const FilterPlan fp{bp->rank_lo, bp->rank_hi, pp.filter_en};
#ifdef KSIM_FS_CLOCKS
    __builtin_amdgcn_s_waitcnt(0);
    if (threadIdx.x == 0) {
      const uint64_t _t = __builtin_amdgcn_s_memrealtime();
      atomicAdd(&s.dbg[14], (unsigned long long)(_t - fs_t));
    }
#endif
    uint32_t det;
    const uint8_t res = run_filter_plan(c, P, fp, s.min_match, tf, p, r, U, m, t, det);
    FS_CLK(3);
    s.fail[node] = res;
    if (COMPAT) s.detail[node] = det;
    if (COMPAT && s.m_fail) s.m_fail[node] = res;
    if (COMPAT && s.m_detail) s.m_detail[node] = det;
    feasible = res == KSIM_PASSED;
    if (feasible) {
      // PodTopologySpread IgnoredNodes candidates: feasible nodes missing a soft key
      // (none for system-defaulted constraints: requireAllTopologies false)
      const bool sysdef = (p.topo_flags & KSIM_POD_PTS_SYSTEM_DEFAULT) != 0;
#pragma unroll
      for (int i = 0; i < KSIM_MAX_USES; i++) {
        if (((m.soft >> i) & 1u) && t.v[i] == 0 && !sysdef) ign = true;
        if (i == soft) soft_cnt = t.x[i];          // soft_count: the node's own count or the domain sum
      }
      s.ign[node] = ign;
      const BatchProg* fast = (bp->fast_w && (c.cflags & kClusterNarrow)) ? bp : nullptr;
      s.part[node] = run_score_plan(c, P, prof, ScorePlan{bp->slot, bp->slot_hi}, p, r, U, m, t, s.raw, COMPAT, rv,
                                    soft_cnt, fast, inv_c, inv_m);
      if (COMPAT && s.m_raw) {                     // the feasible node's answers in the host's staging too:
        const size_t N = (size_t)c.n;                // node-major rows of S raw scores + the part, int32
        const int W = prof.n_score + 1;              // (m_head[1] = 1: a value did not fit)
        int32_t* row = s.m_raw + (size_t)node * W;
        bool wide = false;
        for (int k = 0; k < prof.n_score; k++) {
          const int64_t v = s.raw[(size_t)k * N + node];
          wide |= v != (int64_t)(int32_t)v;
          row[k] = (int32_t)v;
        }
        const int64_t v = s.part[node];
        wide |= v != (int64_t)(int32_t)v;
        row[prof.n_score] = (int32_t)v;
        if (wide) s.m_head[1] = 1;
      }
    }
  }
  FS_CLK(4);
  if (NOWIN) {
    const int lane = threadIdx.x & 63;
    WinState* win = s.win;
    const uint64_t fm = __ballot(feasible), im = __ballot(feasible && ign);
    if (!fuse_ext) {                               // block-uniform
      if (lane == 0 && fm) atomicAdd(&win->nfeas, (int32_t)__popcll(fm));
      if (lane == 0 && im) atomicAdd(&win->nign, (int32_t)__popcll(im));
    } else if (lane == 0) {                        // summed per block by block_extrema
      s_cnt[threadIdx.x >> 6][0] = (int32_t)__popcll(fm);
      s_cnt[threadIdx.x >> 6][1] = (int32_t)__popcll(im);
    }
    if (P.bflags[pi] & kPodRegistersValues) {
      const uint32_t vwords = (uint32_t)(c.vmax + 31) >> 5;
      for (uint32_t b = m.soft_val; b; b &= b - 1) {
        const int i = __builtin_ctz(b);
        const ksim_topo_use u = load_use(U, i);
        const bool reg = feasible && !ign && node < c.n;
        const uint32_t v = reg ? use_value(c, u, node) : 0u;
        uint32_t* bm = s.regbm + (size_t)i * vwords;
        if (c.col_nvals[u.col] <= 64) {            // few values: OR the wave's values first
          uint64_t bits = reg ? 1ull << v : 0ull;
#pragma unroll
          for (int d = 32; d >= 1; d >>= 1) bits |= __shfl_xor(bits, d, 64);
          if (lane == 0 && (uint32_t)bits) atomicOr(&bm[0], (uint32_t)bits);
          if (lane == 0 && (uint32_t)(bits >> 32)) atomicOr(&bm[1], (uint32_t)(bits >> 32));
        } else if (reg) {
          atomicOr(&bm[v >> 5], 1u << (v & 31));
        }
      }
    }
    if (fuse_ext) {                                // block-uniform
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
          counted = soft < 0 || !ign;              // IgnoredNodes: not in min / max
          v = soft < 0 ? 0 : soft_cnt;
        } else {
          v = rv.of(pl);
        }
        if (counted) {
          ix[k] = max_image(v);
          in[k] = min_image(v);
        }
      }
      uint32_t zmask = 0;                          // slots constant 0 for this pod
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
      block_extrema(prof, s.win, ix, in, s_red, zmask, s_cnt);
    }
  }
  FS_CLK(5);
#ifdef KSIM_FS_CLOCKS
  if (threadIdx.x == 0) atomicAdd(&s.dbg[15], 1ull);
#endif
}

constexpr int kBmWords = (KSIM_MAX_NODES + 1 + 31) / 32;   // value-id bitmap (PTS pair registration)


// The selection after the filters, as four launches (a single block cannot
// hide the latency of 10^4 nodes' loads):
//   k_window   1 block: numFeasibleNodesToFind window (block scan), the
//              PodTopologySpread PreScore (IgnoredNodes, pair registration,
//              topologyNormalizingWeight); resets the extrema / argmax slots
//   k_extrema  grid: PodTopologySpread raw scores, NormalizeScore extrema
//   k_select   grid: normalized weighted totals, TB argmax (atomicMax), and
//              the domain tables re-zeroed for the next pod
//   k_bind     1 wave: selectHost result, NodeInfo.AddPod, scheduler state
template <bool COMPAT>
__global__ __launch_bounds__(kFinalThreads) void k_window(DevCluster c, DevPods P, ksim_profile prof,
                                                          DevState* __restrict__ st, DevScratch s) {
  __shared__ int32_t sh32[kFinalWaves];
  __shared__ int32_t s_cut;
  __shared__ uint32_t s_bm[kBmWords];
  const int32_t pi = st->cursor;
  if (pi >= st->end) return;
  const int tid = threadIdx.x;
  const ksim_pod& p = P.pods[pi];
  // the scan (unsharded: global positions are local): every node, or the
  // PreFilterResult's nodes (KSIM_POD_NODE_NAMES)
  const ScanSet ss = scan_set(c, P, p, st->next_start);
  const int32_t NS = ss.n;
  const int32_t K = num_feasible_nodes_to_find(prof.percentage_of_nodes_to_score, NS);
  const int32_t chunk = (NS + kFinalThreads - 1) / kFinalThreads;
  const int32_t lo = min(NS, tid * chunk), hi = min(NS, lo + chunk);
  WinState* win = s.win;

  // Extender pass (s.ext_fail set, ksim_eval_pod_finish): the window of the
  // filter pass stands (nextStartNodeIndex moved before the extenders ran);
  // the kept nodes an extender dropped are marked and the list recounted.
  const bool ext = s.ext_fail != nullptr;
  const bool nb_filter_on = prof_has_filter(prof, KSIM_PL_NETWORK_BANDWIDTH);
  const bool nb_score_on = prof_has_score(prof, KSIM_PL_NETWORK_BANDWIDTH);
  int32_t cut, nf, error = 0;
  if (ext) {
    cut = win->cut;
    error = win->error;                            // the filter pass already failed
    const int32_t kend0 = cut < NS ? cut : NS;
    int32_t kept = 0;
    for (int32_t r = tid; r < kend0; r += kFinalThreads) {   // the stride the loops below use
      const int32_t node = scan_node(ss, r);
      if (s.fail[node] != KSIM_PASSED) continue;
      if (s.ext_fail[node]) {
        s.fail[node] = KSIM_FAIL_EXTENDER;
        if (COMPAT) s.detail[node] = 0;
      } else {
        kept++;
      }
    }
    nf = block_sum_i32_nw<kFinalWaves>(kept, sh32);
  } else {
    // feasible count per scan chunk, block scan, locate the (K+1)-th
    int32_t cnt = 0;
    for (int32_t r = lo; r < hi; r++) cnt += s.fail[scan_node(ss, r)] == KSIM_PASSED;
    int32_t excl, total;
    block_scan_i32(cnt, excl, total, sh32);
    if (tid == 0) s_cut = NS;
    __syncthreads();
    if (total > K && excl <= K && K < excl + cnt) {
      int32_t run = excl;
      for (int32_t r = lo; r < hi; r++) {
        if (s.fail[scan_node(ss, r)] == KSIM_PASSED) {
          if (run == K) { s_cut = r; break; }
          run++;
        }
      }
    }
    __syncthreads();
    cut = s_cut;
    nf = total < K ? total : K;
    if (nb_filter_on) {
      // the first node in scan order whose Filter status was an error; the
      // scan fails there if it comes before the (K+1)-th feasible node
      int64_t first = NS;
      for (int32_t r = lo; r < hi; r++) {
        if (fail_is_error(s.fail[scan_node(ss, r)])) { first = r; break; }
      }
      __shared__ int64_t sh64[kFinalWaves];
      const int32_t err = (int32_t)block_min_i64(first, sh64);
      if (err < (cut < NS ? cut + 1 : NS)) {
        error = kCycleErrorFilter;
        int32_t before = 0;                        // feasible nodes found before it
        for (int32_t r = lo; r < hi && r < err; r++) before += s.fail[scan_node(ss, r)] == KSIM_PASSED;
        nf = block_sum_i32_nw<kFinalWaves>(before, sh32);
        cut = err;                                 // processed = the nodes before it
      }
    }
    // NodeInfos().Get of a PreFilterResult name fails: framework.Error, nothing scanned
    if (p.flags & KSIM_POD_NODE_NAMES_UNKNOWN) error = kCycleErrorPrefilter;
  }
  const int32_t kend = cut < NS ? cut : NS;
  const int32_t evaluated = cut < NS ? cut + 1 : NS;
  if (COMPAT && !ext) {
    for (int32_t r = evaluated + tid; r < NS; r += kFinalThreads) {
      const int32_t node = scan_node(ss, r);
      s.fail[node] = KSIM_NOT_EVALUATED;
      s.detail[node] = 0;
    }
  }
  if (!error && nb_score_on && nf > 1) {
    int32_t bad = 0;                               // kept nodes whose Score returns Skip / Error
    for (int32_t r = tid; r < kend; r += kFinalThreads) {
      const int32_t node = scan_node(ss, r);
      bad += s.fail[node] == KSIM_PASSED && nb_score_error(c.flags[node]);
    }
    if (block_sum_i32_nw<kFinalWaves>(bad, sh32) > 0) error = kCycleErrorScore;
  }
  bool any_soft = false;
  for (int i = 0; i < p.use_count; i++) any_soft = any_soft || P.uses[p.use_first + i].kind == KSIM_USE_PTS_SOFT;
  const bool has_soft = !error && nf > 1 && any_soft;
  if (has_soft) {
    int32_t nign = 0;
    for (int32_t r = tid; r < kend; r += kFinalThreads) {
      const int32_t node = scan_node(ss, r);
      nign += s.fail[node] == KSIM_PASSED && s.ign[node];
    }
    nign = block_sum_i32_nw<kFinalWaves>(nign, sh32);
    for (int i = 0; i < p.use_count; i++) {
      const ksim_topo_use u = P.uses[p.use_first + i];
      if (u.kind != KSIM_USE_PTS_SOFT) continue;
      int32_t size;
      if (u.flags & KSIM_USEF_HOSTNAME) {
        size = nf - nign;
      } else {
        const int32_t words = u.col == KSIM_COL_NONE ? 1 : (c.col_nvals[u.col] + 31) / 32;
        for (int x = tid; x < words; x += kFinalThreads) s_bm[x] = 0;
        __syncthreads();
        for (int32_t r = tid; r < kend; r += kFinalThreads) {
          const int32_t node = scan_node(ss, r);
          if (s.fail[node] != KSIM_PASSED || s.ign[node]) continue;
          const uint32_t v = use_value(c, u, node);
          atomicOr(&s_bm[v >> 5], 1u << (v & 31));
        }
        __syncthreads();
        int32_t bits = 0;
        for (int x = tid; x < words; x += kFinalThreads) bits += __popc(s_bm[x]);
        size = block_sum_i32_nw<kFinalWaves>(bits, sh32);
      }
      if (tid == 0) win->w[i] = c.topo_log[size];
    }
  }
  if (tid < kExtWords) win->ext[tid] = 0;
  if (tid == 0) {
    win->cut = cut;
    win->kend = kend;
    win->nf = nf;
    win->evaluated = evaluated;
    win->has_soft = has_soft;
    win->k = K;
    win->error = error;
    win->nscan = NS;
  }
}

// Whether a (local) node is in the kept list: feasible and scanned before the cut.
__device__ __forceinline__ bool kept_node(const DevCluster& c, const DevScratch& s, const ScanSet& ss, int32_t node,
                                          int32_t kend) {
  if (s.fail[node] != KSIM_PASSED) return false;
  const int32_t r = scan_pos(ss, c.base + node);
  return r >= 0 && r < kend;
}

// NOWIN: the window state is derived here from k_filter_score's counters and
// registration bitmaps (every block alike; block 0 publishes it for k_select
// and k_bind).
template <bool NOWIN>
__global__ __launch_bounds__(256) void k_extrema(DevCluster c, DevPods P, ksim_profile prof,
                                                 const DevState* __restrict__ st, DevScratch s) {
  __shared__ uint64_t s_red[4][2 * KSIM_MAX_SCORE];
  __shared__ ksim_topo_use s_use[KSIM_MAX_USES];
  __shared__ double s_w[KSIM_MAX_USES];
  __shared__ int32_t sh32[4];
  const int32_t pi = st->cursor;
  if (pi >= st->end) return;
  WinState* win = s.win;
  const ksim_pod& p = P.pods[pi];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int nu = p.use_count;
  const ScanSet ss = scan_set(c, P, p, st->next_start);
  bool has_soft;
  if (NOWIN) {
    const int32_t nf = win->nfeas;
    bool any_soft = false;
    for (int i = 0; i < nu; i++) any_soft = any_soft || P.uses[p.use_first + i].kind == KSIM_USE_PTS_SOFT;
    has_soft = nf > 1 && any_soft;
    if (tid < nu) s_use[tid] = P.uses[p.use_first + tid];
    if (has_soft) {
      const uint32_t vwords = (uint32_t)(c.vmax + 31) >> 5;
      const int32_t nign = win->nign;
      for (int i = 0; i < nu; i++) {
        const ksim_topo_use u = P.uses[p.use_first + i];
        if (u.kind != KSIM_USE_PTS_SOFT) continue;
        int32_t size = 0;
        if (u.flags & KSIM_USEF_HOSTNAME) {
          size = nf - nign;
        } else if (u.col != KSIM_COL_NONE) {
          const int32_t words = (c.col_nvals[u.col] + 31) >> 5;
          int32_t bits = 0;
          for (int x = tid; x < words; x += blockDim.x) bits += __popc(s.regbm[(size_t)i * vwords + x]);
          size = block_sum_i32_nw<4>(bits, sh32);
        }
        if (tid == 0) s_w[i] = c.topo_log[size];
      }
    }
    if (blockIdx.x == 0 && tid == 0) {            // K = N: every scanned node is kept
      win->nf = nf;
      win->kend = ss.n;
      win->cut = ss.n;
      win->evaluated = ss.n;
      win->k = ss.n;
      win->nscan = ss.n;
      win->error = (p.flags & KSIM_POD_NODE_NAMES_UNKNOWN) ? kCycleErrorPrefilter : 0;
      win->has_soft = has_soft;
      for (int i = 0; i < nu; i++) win->w[i] = s_w[i];
    }
    __syncthreads();
    if (nf <= 1) return;                          // no scoring
  } else {
    if (win->nf <= 1 || win->error) return;       // no scoring
    has_soft = win->has_soft != 0;
    if (tid < nu) {
      s_use[tid] = P.uses[p.use_first + tid];
      s_w[tid] = win->w[tid];
    }
    __syncthreads();
  }
  const int32_t node = blockIdx.x * blockDim.x + tid;
  const int32_t N = c.n;
  const bool kept = node < N && kept_node(c, s, ss, node, NOWIN ? ss.n : win->kend);
  const int S = prof.n_score;
#pragma unroll
  for (int k = 0; k < KSIM_MAX_SCORE; k++) {
    if (k >= S) break;
    const int32_t kind = norm_kind(prof.score[k]);
    if (kind == kNormNone) continue;
    uint64_t ix = 0, in = 0;
    if (kept) {
      int64_t v;
      bool counted = true;
      if (kind == kNormPTS) {
        const bool ign = has_soft && s.ign[node];
        v = 0;
        if (has_soft && !ign) {                   // podtopologyspread Score
          double score = 0;
          for (int i = 0; i < nu; i++) {
            const ksim_topo_use& u = s_use[i];
            if (u.kind != KSIM_USE_PTS_SOFT) continue;
            const uint32_t val = use_value(c, u, node);
            if (val == 0) continue;
            const int64_t n_match = (u.flags & KSIM_USEF_HOSTNAME) ? class_count(c, u.cls, node)
                                                                    : s.dom[(size_t)i * c.vmax + val];
            score = score + ((double)n_match * s_w[i] + (double)(u.arg - 1));   // scoreForCount, unfused
          }
          v = (int64_t)round(score);              // math.Round
        }
        s.raw[(size_t)k * N + node] = v;
        counted = !ign;                           // invalidScore: not in min / max
      } else {
        v = s.raw[(size_t)k * N + node];
      }
      if (counted) {
        ix = max_image(v);
        in = min_image(v);
      }
    }
    ix = wave_max_u64_dpp(ix);
    in = wave_max_u64_dpp(in);
    if (lane == 0) {
      s_red[wv][2 * k] = ix;
      s_red[wv][2 * k + 1] = in;
    }
  }
  __syncthreads();
  if (tid < 2 * KSIM_MAX_SCORE && tid < 2 * S && norm_kind(prof.score[tid >> 1]) != kNormNone) {
    uint64_t m = 0;
#pragma unroll
    for (int w = 0; w < 4; w++) m = umax64(m, s_red[w][tid]);
    if (m) atomicMax(reinterpret_cast<unsigned long long*>(&win->ext[tid]), (unsigned long long)m);
  }
}

// fuse_ext: k_extrema did not run (see k_filter_score).  Every block derives
// the window state from the filter pass's counters, as k_extrema<true> does,
// and block 0 publishes it for k_bind; PodTopologySpread's raw scores and
// extrema come from the soft use's counts.
// The window scalars bind_cycle reads (see its ws argument).
struct WinScalars {
  int32_t nscan, nf, cut, evaluated, k, error;
};

// selectHost over k_select's per-block records (one wave): the winning TB lo
// word (0: no kept node).
__device__ __forceinline__ uint64_t reduce_block_best(const DevScratch& s, int32_t n_blocks) {
  const int lane = threadIdx.x & 63;
  uint64_t img = 0, lo = 0;
  for (int32_t b = lane; b < n_blocks; b += 64) best2_merge(img, lo, s.bbest[2 * b], s.bbest[2 * b + 1]);
  wave_best2(img, lo);
  return lo;
}

// The bind step of a per-pod cycle, by one wave: selectHost over k_select's
// block records, NodeInfo.AddPod on the chosen node (one column per lane) and
// the scheduler state (thread 0).  NOWIN also returns the counters and extrema
// slots to zero for the next cycle (k_window resets its own otherwise;
// k_topo_prefilter clears the registration rows).
__device__ __forceinline__ void bind_cycle(const DevCluster& c, const DevPods& P, DevState* __restrict__ st,
                                           const DevScratch& s, int32_t* __restrict__ chosen_out, int32_t pi,
                                           bool nowin, const PodPlan& pp, const WinScalars* ws = nullptr) {
  WinState* win = s.win;
  // the pod's persistent-table updates, loaded ahead of the selection they do not depend on
  const int lane = threadIdx.x & 63;
  const bool tadds = (pp.flags & kPlanTadds) != 0;
  int4 ta = make_int4(0, 0, 0, 0);
  if (tadds && lane < pp.tadd_count) ta = P.ptab_padd[pp.tadd_first + lane];
  ksim_class_add add0{};                           // this lane's first class add, likewise
  if (lane < P.pods[pi].add_count) add0 = P.adds[P.pods[pi].add_first + lane];
  // the window scalars and the scheduler state do not depend on the choice
  // either (the row stores below could alias them for the compiler: load first)
  // (ws: the launch's own block 0 writes them -- k_select fuse_ext -- and the
  // caller passes the values it derived itself instead of reading them back)
  const int32_t NS = ws ? ws->nscan : win->nscan, nf = ws ? ws->nf : win->nf, cut = ws ? ws->cut : win->cut,
                evaluated = ws ? ws->evaluated : win->evaluated, k = ws ? ws->k : win->k;
  DevState S = *st;                                // one read, one write back: no load-store chain
  const uint64_t best = reduce_block_best(s, (c.n + 255) / 256);   // every lane
  const int32_t error = ws ? ws->error : win->error;
  const int32_t chosen = best && !error ? key_node(best) : -1;   // unsharded: base == 0
  const ksim_pod p = P.pods[pi];
  if (chosen >= 0) {
    assume_pod_wave(c, P, p, chosen, 1, !tadds, &add0);         // NodeInfo.AddPod, one column per lane
    if (tadds)
      for (int32_t i = lane; i < pp.tadd_count; i += 64) {
        const int4 t = i == lane ? ta : P.ptab_padd[pp.tadd_first + i];
        const uint32_t v = c.labels[(size_t)t.y * c.n + chosen];
        if (v) atomicAdd(reinterpret_cast<unsigned long long*>(P.ptab + t.x + (t.z == kPtabTotal ? 0u : v)),
                         (unsigned long long)(int64_t)t.w);
      }
  }
  if (lane != 0) return;
  // nextStartNodeIndex = (nextStartNodeIndex + processed) % len(scanned nodes);
  // a pod PreFilter rejected scans nothing and leaves it
  const int32_t ns = NS > 0 ? (int32_t)(((int64_t)S.next_start + (cut < NS ? cut : NS)) % NS) : S.next_start;
  S.next_start = ns;
  if (c.count_whole) S.evals += evaluated;
  if (chosen >= 0) S.scheduled += 1;
  else S.unschedulable += 1;
  if (chosen_out) chosen_out[pi] = chosen >= 0 ? c.base + chosen : error ? KSIM_CHOSEN_ERROR : -1;
  S.chosen = chosen >= 0 ? chosen : error ? KSIM_CHOSEN_ERROR : -1;
  S.status = chosen >= 0 ? KSIM_STATUS_SCHEDULED : error ? KSIM_STATUS_ERROR : KSIM_STATUS_UNSCHEDULABLE;
  S.n_feasible = nf;
  S.n_evaluated = evaluated;
  S.n_processed = cut < NS ? cut : NS;
  S.k_to_find = k;
  S.next_start_after = ns;
  S.pod_seq += 1;
  S.topo_flags = 0;
  S.cursor = pi + 1;
  *st = S;
  win->error = 0;
  if (nowin) {
    win->nfeas = 0;
    win->nign = 0;
    for (int t = 0; t < kExtWords; t++) win->ext[t] = 0;
  }
}

// KSIM_SEL_CLOCKS builds: per-block phase times of k_select (thread 0, 100 MHz
// realtime) summed into s.dbg[phase - 1] (1 prologue, 2 totals, 3 block
// record, 4 arrival), s.dbg[4] = blocks, s.dbg[5] = the last block's bind,
// s.dbg[6] = bind steps.
#ifdef KSIM_SEL_CLOCKS
#define SEL_CLK(k)                                                         \
  do {                                                                     \
    if (threadIdx.x == 0) {                                                \
      const uint64_t _t = __builtin_amdgcn_s_memrealtime();                \
      if ((k) > 0) atomicAdd(&s.dbg[(k) - 1], (unsigned long long)(_t - sel_t)); \
      sel_t = _t;                                                          \
    }                                                                      \
  } while (0)
#else
#define SEL_CLK(k) do {} while (0)
#endif

template <bool COMPAT>
// bind_mode (unsharded cycles): 1 / 2 = the last block to finish runs the bind
// step (bind_cycle, windowed / NOWIN), which saves k_bind's launch.
__global__ __launch_bounds__(256) void k_select(DevCluster c, DevPods P0, ksim_profile prof,
                                                DevState* __restrict__ st, DevScratch s, DevEvalOut o,
                                                int32_t fuse_ext, int32_t bind_mode, int32_t* __restrict__ chosen_out) {
  __shared__ uint64_t s_best[8];
  __shared__ int32_t sh32[4];
#ifdef KSIM_SEL_CLOCKS
  uint64_t sel_t = 0;
#endif
  SEL_CLK(0);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int32_t node = blockIdx.x * blockDim.x + tid;
  const int32_t N = c.n;
  const int S = prof.n_score;
  const int32_t pi = st->cursor;
  if (pi >= st->end) return;
  WinState* win = s.win;
  const DevPods& P = P0;
  const ksim_pod p = P0.pods[pi];                 // block-uniform: scalar loads
  const PodPlan pp = P0.plans[pi];
  const UseMasks& m = pp.m;
  const ksim_topo_use* U = P.uses + p.use_first;
  int32_t nf, kend;
  bool has_soft;
  int soft = -1;
  double w_soft = 0;
  const ScanSet ss = scan_set(c, P, p, st->next_start);
  if (fuse_ext) {                                  // block-uniform
    nf = win->nfeas;
    kend = ss.n;
    soft = m.soft ? 31 - __builtin_clz(m.soft) : -1;   // the pod's one ScheduleAnyway use
    has_soft = nf > 1 && soft >= 0;
    if (has_soft) {                                // topologyNormalizingWeight of the one soft use
      const ksim_topo_use u = load_use(U, soft);
      int32_t size = 0;
      if (u.flags & KSIM_USEF_HOSTNAME) {
        size = nf - win->nign;
      } else if (u.col != KSIM_COL_NONE) {
        const uint32_t vwords = (uint32_t)(c.vmax + 31) >> 5;
        const int32_t words = (c.col_nvals[u.col] + 31) >> 5;
        int32_t bits = 0;
        for (int x = tid; x < words; x += blockDim.x) bits += __popc(s.regbm[(size_t)soft * vwords + x]);
        size = block_sum_i32_nw<4>(bits, sh32);
      }
      w_soft = c.topo_log[size];
    }
    if (blockIdx.x == 0 && tid == 0) {            // K = N: every scanned node is kept
      win->nf = nf;
      win->kend = ss.n;
      win->cut = ss.n;
      win->evaluated = ss.n;
      win->k = ss.n;
      win->nscan = ss.n;
      win->error = (p.flags & KSIM_POD_NODE_NAMES_UNKNOWN) ? kCycleErrorPrefilter : 0;
      win->has_soft = has_soft;
      if (soft >= 0) win->w[soft] = w_soft;
    }
  } else {
    nf = win->nf;
    kend = win->kend;
    has_soft = win->has_soft != 0;
  }
  SEL_CLK(1);
  uint64_t img = 0, tlo = 0;                       // this node's (total image, TB lo); tlo == 0: no key
  if (node < N) {
    const bool kept = nf >= 1 && !win->error && kept_node(c, s, ss, node, kend);
    if (kept && nf > 1) {
      const bool ign = has_soft && s.ign[node];
      const bool ipa_nonempty = (st->topo_flags & kTopoScoreNonEmpty) != 0;
      // prioritizeNodes: no score plugins and no extenders -> 1; the extenders'
      // combined scores are added to the plugin total
      int64_t tot = S == 0 ? (s.ext_score ? 0 : 1) : s.part[node];
      if (s.ext_score) tot += s.ext_score[node];
      for (int k = 0; k < S; k++) {
        const int32_t kind = norm_kind(prof_score(prof, k));
        int64_t raw, gmax = 0, gmin = 0;
        if (kind != kNormNone) {
          gmax = from_max_image(win->ext[2 * k]);
          gmin = from_min_image(win->ext[2 * k + 1]);
        }
        if (fuse_ext && kind == kNormPTS) {
          raw = 0;
          if (has_soft) {                          // counts -> scores (a non-decreasing map)
            const int32_t ms = load_use(U, soft).arg;
            // the filter pass left the node's count in the slot (the domain
            // tables are being re-zeroed by this kernel)
            if (!ign) raw = soft_score(s.raw[(size_t)k * N + node], w_soft, ms);
            if (win->ext[2 * k]) gmax = soft_score(gmax, w_soft, ms);
            if (win->ext[2 * k + 1]) gmin = soft_score(gmin, w_soft, ms);
          }
        } else {
          raw = s.raw[(size_t)k * N + node];
        }
        int64_t nv = raw;
        if (kind != kNormNone) {
          if (kind == kNormPTS && ign)
            nv = 0;
          else
            nv = normalize_value(kind, raw, gmax, gmin, ipa_nonempty);
          tot += nv * prof_weight(prof, k);
        }
        if (COMPAT) {
          o.raw[(size_t)k * N + node] = raw;
          o.norm[(size_t)k * N + node] = nv;
        }
      }
      if (COMPAT) {
        o.total[node] = tot;
        o.scored[node] = 1;
      }
      img = max_image(tot);
      tlo = tb_lo(prof.tiebreak_seed, st->pod_seq, c.base + node);
    } else {
      // one feasible node: schedulePod returns it without scoring
      if (kept) {
        img = max_image(0);
        tlo = tb_lo(prof.tiebreak_seed, st->pod_seq, c.base + node);
      }
      if (COMPAT) {
      o.total[node] = 0;
      o.scored[node] = 0;
      for (int k = 0; k < S; k++) {
        o.raw[(size_t)k * N + node] = 0;
        o.norm[(size_t)k * N + node] = 0;
      }
      }
    }
    // the domain tables are read no more this cycle: re-zero what this node's
    // values touched (every touched entry is some node's value); small tables
    // are cleared whole by block 0 below
    for (uint32_t b = m.dom & ~m.ptab; b; b &= b - 1) {
      const int i = __builtin_ctz(b);
      const ksim_topo_use u = load_use(U, i);
      if (c.col_nvals[u.col] > kLdsDom) s.dom[(size_t)i * c.vmax + use_value(c, u, node)] = 0;
    }
  }
  if (blockIdx.x == 0)
    for (uint32_t b = m.dom & ~m.ptab; b; b &= b - 1) {
      const int i = __builtin_ctz(b);
      const int32_t V = c.col_nvals[load_use(U, i).col];
      if (V <= kLdsDom && tid < V) s.dom[(size_t)i * c.vmax + tid] = 0;
    }
  SEL_CLK(2);
  // selectHost: the block's best (total, TB) pair -> its record (k_bind reduces the records)
  wave_best2(img, tlo);
  if (lane == 0) {
    s_best[2 * wv] = img;
    s_best[2 * wv + 1] = tlo;
  }
  __syncthreads();
  if (tid == 0) {
    uint64_t bi = s_best[0], bl = s_best[1];
#pragma unroll
    for (int w = 1; w < 4; w++) best2_merge(bi, bl, s_best[2 * w], s_best[2 * w + 1]);
    {
      s.bbest[2 * blockIdx.x] = bi;
      s.bbest[2 * blockIdx.x + 1] = bl;
    }
  }
  SEL_CLK(3);
  if (bind_mode) {
    __shared__ int32_t s_last;
    if (tid == 0) {
      // the last block: its acquire sees every block's record (and block 0's
      // window fields) released by their own increments
      const int32_t done = __hip_atomic_fetch_add(&win->done, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      s_last = done == (int32_t)gridDim.x - 1;
    }
    __syncthreads();
    SEL_CLK(4);
    if (s_last && tid < 64) {
      if (tid == 0) __hip_atomic_store(&win->done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // keeps the record loads below the ticket
      bind_cycle(c, P, st, s, chosen_out, pi, bind_mode == 2, pp, nullptr);
#ifdef KSIM_SEL_CLOCKS
      if (tid == 0) {
        atomicAdd(&s.dbg[5], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - sel_t));
        atomicAdd(&s.dbg[6], 1ull);
      }
#endif
    }
  }
#ifdef KSIM_SEL_CLOCKS
  if (tid == 0) atomicAdd(&s.dbg[4], 1ull);
#endif
}

// The persistent domain tables from the class counts (a queue's upload, a
// snapshot reset): one block per table, LDS sums over the column's values.
constexpr int kPtabLds = 2048;
__global__ __launch_bounds__(256) void k_ptab_init(DevCluster c, DevPods P) {
  __shared__ unsigned long long s_sum[kPtabLds];
  const int4 t = P.ptab_ent[blockIdx.x];
  const int32_t V = t.z == kPtabTotal ? 1 : c.col_nvals[t.y];
  int64_t* out = P.ptab + t.w;
  const bool lds = V <= kPtabLds;
  for (int32_t v = threadIdx.x; v < V; v += blockDim.x) {
    if (lds) s_sum[v] = 0;
    else out[v] = 0;
  }
  __syncthreads();
  const uint32_t* lab = c.labels + (size_t)t.y * c.n;
  for (int32_t n = threadIdx.x; n < c.n; n += blockDim.x) {
    const uint32_t v = lab[n];
    if (!v) continue;
    const int64_t add = (t.x >= 0 ? (int64_t)c.cnt[(size_t)t.x * c.n + n] : 0) + (t.z == kPtabMark ? (1ll << kDomMarkShift) : 0);
    const uint32_t x = t.z == kPtabTotal ? 0u : v;
    if (!add) continue;
    if (lds) atomicAdd(&s_sum[x], (unsigned long long)add);
    else atomicAdd(reinterpret_cast<unsigned long long*>(out + x), (unsigned long long)add);
  }
  __syncthreads();
  if (lds)
    for (int32_t v = threadIdx.x; v < V; v += blockDim.x) out[v] = (int64_t)s_sum[v];
}

void launch_ptab_init(const DevCluster& c, const DevPods& P, hipStream_t stream) {
  if (P.n_ptab > 0) k_ptab_init<<<P.n_ptab, 256, 0, stream>>>(c, P);
}

// ksim_reset_cluster's column copies and the state zeroing in one launch (one
// dispatch instead of nine copy / fill dispatches): segment k copies words[k]
// 32-bit words from src[k] to dst[k] (src null: zeroes), blocks strided over
// every segment in 16-byte units, the tails by word.
__global__ __launch_bounds__(256) void k_reset_copy(ResetList L) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const size_t t0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int k = 0; k < L.n; k++) {
    uint32_t* d = L.dst[k];
    const uint32_t* sp = L.src[k];
    const size_t n = L.words[k], n4 = n / 4;
    for (size_t i = t0; i < n4; i += stride) {
      const uint4 v = sp ? reinterpret_cast<const uint4*>(sp)[i] : make_uint4(0, 0, 0, 0);
      reinterpret_cast<uint4*>(d)[i] = v;
    }
    for (size_t i = 4 * n4 + t0; i < n; i += stride) d[i] = sp ? sp[i] : 0u;
  }
}

void launch_reset_copy(const ResetList& L, hipStream_t stream) {
  size_t most = 0;
  for (int k = 0; k < L.n; k++) most = L.words[k] > most ? L.words[k] : most;
  const int blocks = (int)std::min<size_t>(1024, std::max<size_t>(1, (most / 4 + 255) / 256));
  k_reset_copy<<<blocks, 256, 0, stream>>>(L);
}

__global__ void k_assume(DevCluster c, DevPods P, int32_t pod, int32_t node, int sign) {
  if (threadIdx.x == 0 && blockIdx.x == 0) assume_pod(c, P, P.pods[pod], node, sign);
}

// ==== C. node-sharded per-pod cycle ================================
// Each shard holds the nodes [c.base, c.base + c.n) of c.n_total.  A cycle is
// the unsharded one with exchanges at its grid-wide seams (the host issues
// them between these launches; ksim_engine.cpp shard_cycle):
//   k_topo_prefilter, k_dom_pack  -> all-reduce (sum) of the packed domain sums
//   k_topo_min<true>               unpack, flags, critical paths
//   k_filter_score, k_wcount_sh    -> all-gather of (feasible >= start, feasible < start)
//   k_window_sh                    global cut / kept rule / IgnoredNodes and pair
//                                  registrations -> all-reduce (sum) of s.xreg
//   k_wfinal_sh, k_extrema         -> all-reduce (max) of the extrema images + cut
//   k_select                       -> all-reduce (max) of the TB key
//   k_bind_sh                      the owner shard binds; every shard advances
// Scan order is the global rotated order, so a shard's nodes form at most two
// contiguous runs of it: "hi" (global index >= start) and "lo" (< start).

// Pack the domain rows a sharded exchange sums: use i's row (col_nvals entries)
// at the running offset, uses in order (the host sizes the exchange the same way).
__global__ __launch_bounds__(256) void k_dom_pack(DevCluster c, DevPods P, const DevState* __restrict__ st,
                                                  DevScratch s) {
  const int32_t pi = st->cursor;
  if (pi >= st->end) return;
  const ksim_pod& p = P.pods[pi];
  int64_t off = 0;
  for (int i = 0; i < p.use_count; i++) {
    const ksim_topo_use u = P.uses[p.use_first + i];
    if (!use_needs_dom(u)) continue;
    const int32_t V = c.col_nvals[u.col];
    const int64_t* d = s.dom + (size_t)i * c.vmax;
    for (int32_t v = threadIdx.x; v < V; v += blockDim.x) s.xdom[off + v] = d[v];
    off += V;
  }
}

// Local feasible counts of the two runs -> s.xsend[0..1]; zeroes s.xreg for k_window_sh.
__global__ __launch_bounds__(kFinalThreads) void k_wcount_sh(DevCluster c, DevPods P, const DevState* __restrict__ st,
                                                             DevScratch s) {
  __shared__ int32_t sh32[kFinalWaves];
  const int32_t pi = st->cursor;
  if (pi >= st->end) return;
  const int tid = threadIdx.x;
  const int32_t n = c.n;
  const int32_t split = min(n, max(0, st->next_start - c.base));   // local [split, n) is "hi"
  int32_t hi = 0, lo = 0;
  for (int32_t x = tid; x < n; x += kFinalThreads) {
    const bool f = s.fail[x] == KSIM_PASSED;
    if (x >= split) hi += f; else lo += f;
  }
  hi = block_sum_i32_nw<kFinalWaves>(hi, sh32);
  lo = block_sum_i32_nw<kFinalWaves>(lo, sh32);
  if (tid == 0) {
    s.xsend[0] = (uint64_t)hi;
    s.xsend[1] = (uint64_t)lo;
  }
  const ksim_pod& p = P.pods[pi];
  int64_t len = 1;
  for (int i = 0; i < p.use_count; i++) {
    const ksim_topo_use u = P.uses[p.use_first + i];
    if (use_registers_values(u)) len += c.col_nvals[u.col];
  }
  bool any_soft = false;
  for (int i = 0; i < p.use_count; i++) any_soft = any_soft || P.uses[p.use_first + i].kind == KSIM_USE_PTS_SOFT;
  if (any_soft)
    for (int64_t x = tid; x < len; x += kFinalThreads) s.xreg[x] = 0;
}

// The j-th (0-based) feasible node of local [lo, hi) in node order (block-wide).
__device__ int32_t block_nth_feasible(const uint8_t* __restrict__ fail, int32_t lo, int32_t hi, int32_t j,
                                      int32_t* sh32, int32_t* s_out) {
  const int tid = threadIdx.x;
  const int32_t len = hi - lo, chunk = (len + kFinalThreads - 1) / kFinalThreads;
  const int32_t a = lo + min(len, tid * chunk), b = min(hi, a + chunk);
  int32_t cnt = 0;
  for (int32_t x = a; x < b; x++) cnt += fail[x] == KSIM_PASSED;
  int32_t excl, total;
  block_scan_i32(cnt, excl, total, sh32);
  if (tid == 0) *s_out = -1;
  __syncthreads();
  if (excl <= j && j < excl + cnt) {
    int32_t run = excl;
    for (int32_t x = a; x < b; x++) {
      if (fail[x] == KSIM_PASSED) {
        if (run == j) {
          *s_out = x;
          break;
        }
        run++;
      }
    }
  }
  __syncthreads();
  return *s_out;
}

// Global numFeasibleNodesToFind window from the gathered counts (s.xrecv[world][2]):
// the cut is the K-th (0-based) feasible node of the global scan; this shard's
// kept rule is "scan position < win->kend".  Then this shard's IgnoredNodes
// count and pair registrations over its kept nodes -> s.xreg.
__global__ __launch_bounds__(kFinalThreads) void k_window_sh(DevCluster c, DevPods P, ksim_profile prof,
                                                             const DevState* __restrict__ st, DevScratch s,
                                                             int32_t rank, int32_t world) {
  __shared__ int32_t sh32[kFinalWaves];
  __shared__ int32_t s_out;
  const int32_t pi = st->cursor;
  if (pi >= st->end) return;
  const int tid = threadIdx.x;
  const ksim_pod& p = P.pods[pi];
  WinState* win = s.win;
  const int32_t N = c.n_total, n = c.n, base = c.base;
  const int32_t K = num_feasible_nodes_to_find(prof.percentage_of_nodes_to_score, N);
  const int32_t start = st->next_start;
  int64_t T = 0, all_hi = 0, bhi = 0, blo = 0, fhi = 0, flo = 0;
  for (int t = 0; t < world; t++) {
    const int64_t h = (int64_t)s.xrecv[2 * t], l = (int64_t)s.xrecv[2 * t + 1];
    T += h + l;
    all_hi += h;
    if (t < rank) {
      bhi += h;
      blo += l;
    }
    if (t == rank) {
      fhi = h;
      flo = l;
    }
  }
  blo += all_hi;
  const int32_t split = min(n, max(0, start - base));
  const ScanSet ss{nullptr, N, start};             // sharded cycles scan every node
  int32_t kend, cutslot = 0;
  if (T <= K) {
    kend = N;
  } else if (bhi <= K && K < bhi + fhi) {
    const int32_t x = block_nth_feasible(s.fail, split, n, (int32_t)(K - bhi), sh32, &s_out);
    kend = base + x - start;
    cutslot = kend + 1;
  } else if (blo <= K && K < blo + flo) {
    const int32_t x = block_nth_feasible(s.fail, 0, split, (int32_t)(K - blo), sh32, &s_out);
    kend = base + x - start + N;
    cutslot = kend + 1;
  } else if (blo + flo <= K) {
    kend = N;                                  // both runs before the cut
  } else if (bhi + fhi <= K && split < n) {
    kend = base + n - start;                   // the hi run before the cut, the lo run after
  } else {
    kend = 0;
  }
  const int32_t nf = (int32_t)(T < K ? T : K);
  bool any_soft = false;
  for (int i = 0; i < p.use_count; i++) any_soft = any_soft || P.uses[p.use_first + i].kind == KSIM_USE_PTS_SOFT;
  if (any_soft) {
    int32_t nign = 0;
    for (int32_t x = tid; x < n; x += kFinalThreads) {
      if (!kept_node(c, s, ss, x, kend)) continue;
      if (s.ign[x]) {
        nign++;
        continue;
      }
      int64_t off = 1;
      for (int i = 0; i < p.use_count; i++) {
        const ksim_topo_use u = P.uses[p.use_first + i];
        if (!use_registers_values(u)) continue;
        atomicAdd(reinterpret_cast<unsigned long long*>(s.xreg + off + use_value(c, u, x)), 1ull);
        off += c.col_nvals[u.col];
      }
    }
    nign = block_sum_i32_nw<kFinalWaves>(nign, sh32);
    if (tid == 0) atomicAdd(reinterpret_cast<unsigned long long*>(s.xreg), (unsigned long long)nign);
  }
  if (tid < kExtWords) win->ext[tid] = tid == kExtCut ? (uint64_t)cutslot : 0ull;
  if (tid == 0) {
    win->kend = kend;
    win->nf = nf;
    win->k = K;
    win->has_soft = nf > 1 && any_soft;
    win->nscan = N;
  }
}

// topologyNormalizingWeight from the all-reduced registrations.
__global__ __launch_bounds__(256) void k_wfinal_sh(DevCluster c, DevPods P, const DevState* __restrict__ st,
                                                   DevScratch s) {
  __shared__ int32_t sh32[4];
  const int32_t pi = st->cursor;
  if (pi >= st->end) return;
  WinState* win = s.win;
  if (!win->has_soft) return;
  const ksim_pod& p = P.pods[pi];
  const int64_t nign = (int64_t)s.xreg[0];
  int64_t off = 1;
  for (int i = 0; i < p.use_count; i++) {
    const ksim_topo_use u = P.uses[p.use_first + i];
    if (u.kind != KSIM_USE_PTS_SOFT) continue;
    int32_t size = 0;
    if (u.flags & KSIM_USEF_HOSTNAME) {
      size = (int32_t)(win->nf - nign);
    } else if (u.col != KSIM_COL_NONE) {
      const int32_t V = c.col_nvals[u.col];
      int32_t cnt = 0;
      // value 0 registers only for system-defaulted constraints: the pair (key, "")
      for (int32_t v = threadIdx.x; v < V; v += blockDim.x) cnt += s.xreg[off + v] > 0;
      size = block_sum_i32_nw<4>(cnt, sh32);
      off += V;
    }
    if (threadIdx.x == 0) win->w[i] = c.topo_log[size];
  }
}

// selectHost result (global), the owner shard's bind, scheduler state on every shard.
// This shard's best (total image, TB lo) over k_select's block records ->
// s.xsend[0..1], all-gathered (s.xrecv[world][2]) before k_bind_sh.
__global__ __launch_bounds__(64) void k_best_pack(DevCluster c, const DevState* __restrict__ st, DevScratch s) {
  if (st->cursor >= st->end) return;
  const int32_t n_blocks = (c.n + 255) / 256;
  const int lane = threadIdx.x;
  uint64_t img = 0, lo = 0;
  for (int32_t b = lane; b < n_blocks; b += 64) best2_merge(img, lo, s.bbest[2 * b], s.bbest[2 * b + 1]);
  wave_best2(img, lo);
  if (lane == 0) {
    s.xsend[0] = img;
    s.xsend[1] = lo;
  }
}

__global__ __launch_bounds__(256) void k_bind_sh(DevCluster c, DevPods P, DevState* __restrict__ st, DevScratch s,
                                                 int32_t world, int32_t* __restrict__ chosen_out) {
  const int32_t pi = st->cursor;
  if (pi >= st->end) return;
  const ksim_pod& p = P.pods[pi];
  // the exchanged domain rows hold other shards' values too: re-zero them whole
  for (int i = 0; i < p.use_count; i++) {
    const ksim_topo_use u = P.uses[p.use_first + i];
    if (!use_needs_dom(u)) continue;
    const int32_t V = c.col_nvals[u.col];
    for (int32_t v = threadIdx.x; v < V; v += blockDim.x) s.dom[(size_t)i * c.vmax + v] = 0;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  const WinState* win = s.win;
  const int32_t N = c.n_total, n = c.n, base = c.base, start = st->next_start;
  uint64_t bi = 0, bl = 0;                         // selectHost over the shards' records
  for (int32_t r = 0; r < world; r++) best2_merge(bi, bl, s.xrecv[2 * r], s.xrecv[2 * r + 1]);
  const int32_t chosen = bl ? key_node(bl) : -1;
  const int32_t local = chosen - base;
  const int64_t cs = (int64_t)win->ext[kExtCut];
  const int32_t processed = cs ? (int32_t)(cs - 1) : N;
  const int32_t evaluated = cs ? (int32_t)cs : N;
  // this shard's nodes among the evaluated scan prefix
  const int32_t split = min(n, max(0, start - base));
  auto in_prefix = [&](int32_t r0, int32_t len) { return min(max(evaluated - r0, 0), len); };
  const int32_t local_eval = in_prefix(base + split - start, n - split) + in_prefix(base - start + N, split);
  const int32_t ns = (int32_t)(((int64_t)start + processed) % N);
  st->next_start = ns;
  st->evals += local_eval;
  if (chosen >= 0 && local >= 0 && local < n) assume_pod(c, P, p, local, 1);
  if (chosen >= 0)
    st->scheduled += 1;
  else
    st->unschedulable += 1;
  if (chosen_out) chosen_out[pi] = chosen;
  st->chosen = chosen;
  st->status = chosen >= 0 ? KSIM_STATUS_SCHEDULED : KSIM_STATUS_UNSCHEDULABLE;
  st->n_feasible = win->nf;
  st->n_evaluated = evaluated;
  st->n_processed = processed;
  st->k_to_find = win->k;
  st->next_start_after = ns;
  st->pod_seq += 1;
  st->topo_flags = 0;
  st->cursor = pi + 1;
}

// In-process shard group exchanges (one device): element-wise sum / max over
// the group's buffers written back to every member, and the all-gather.
__global__ __launch_bounds__(256) void k_group_reduce(GroupPtrs g, int64_t count, int32_t op_max) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t acc = g.p[0][i];
    for (int r = 1; r < g.n; r++) acc = op_max ? umax64(acc, g.p[r][i]) : acc + g.p[r][i];
    for (int r = 0; r < g.n; r++) g.p[r][i] = acc;
  }
}

__global__ __launch_bounds__(256) void k_group_gather(GroupPtrs src, GroupPtrs dst, int32_t words) {
  const int32_t total = src.n * src.n * words;
  for (int32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int32_t r = i / (src.n * words), q = (i / words) % src.n, w = i % words;
    dst.p[r][q * words + w] = src.p[q][w];
  }
}

// ==== framework-driven compat cycle (ksim_fw_*) ====================================
// Under the simulator's own settings the upstream framework chooses which nodes
// Filter runs on, the feasible list PreScore / Score / NormalizeScore see and
// the node Reserve assumes (ksim_engine.h "Framework-driven compat mode").  The
// filter pass answers every node of the scan set (k_filter_score without the
// window); ksim_fw_score runs the extender-style finish with the framework's
// list as the kept set (k_window's ext branch: unlisted nodes out, PTS PreScore
// over the list), k_extrema and k_select without the bind.
//
// NormalizeScore of one score slot over an explicit (node, score) list, with
// the PreScore facts of the last ksim_fw_score: PodTopologySpread's
// IgnoredNodes (s.ign under win->has_soft) and InterPodAffinity's topologyScore
// emptiness (st->topo_flags).  One block: extrema as order-preserving images.
__global__ __launch_bounds__(kFinalThreads) void k_fw_normalize(ksim_profile prof, int32_t slot,
                                                                const DevState* __restrict__ st, DevScratch s,
                                                                const int32_t* __restrict__ nodes,
                                                                const int64_t* __restrict__ vals, int32_t n,
                                                                int64_t* __restrict__ out) {
  __shared__ uint64_t sh[kFinalWaves];
  const int32_t kind = norm_kind((int)prof_score(prof, slot));
  const bool soft = s.win->has_soft != 0;
  uint64_t ix = 0, in = 0;
  for (int32_t j = threadIdx.x; j < n; j += kFinalThreads) {
    const bool ign = kind == kNormPTS && soft && s.ign[nodes[j]];
    if (!ign) {
      ix = umax64(ix, max_image(vals[j]));
      in = umax64(in, min_image(vals[j]));
    }
  }
  const int64_t gmax = from_max_image(block_max_u64<kFinalWaves>(ix, sh));
  const int64_t gmin = from_min_image(block_max_u64<kFinalWaves>(in, sh));
  const bool ipa_nonempty = (st->topo_flags & kTopoScoreNonEmpty) != 0;
  for (int32_t j = threadIdx.x; j < n; j += kFinalThreads) {
    const int64_t v = vals[j];
    if (kind == kNormNone) out[j] = v;
    else if (kind == kNormPTS && soft && s.ign[nodes[j]]) out[j] = 0;
    else out[j] = normalize_value(kind, v, gmax, gmin, ipa_nonempty);
  }
}

// ---- launchers ----------------------------------------------------------------
const char* const kKernelNames[kKernelsPerCycle] = {"k_topo_prefilter", "k_topo_min", "k_filter_score",
                                                    "k_window", "k_extrema", "k_select", "k_bind"};

template <bool COMPAT, bool NOWIN>
uint32_t launch_cycle_t(const LaunchArgs& a, hipStream_t stream, bool topo, hipEvent_t* evs) {
  uint32_t mask = 0;
  const int blocks = (a.c.n + 255) / 256;
  if (evs) (void)hipEventRecord(evs[0], stream);
  const bool pre = topo && !a.ptab;                // persistent tables: no PreFilter pass
  if (pre) k_topo_prefilter<<<blocks, 256, 0, stream>>>(a.c, a.P, a.prof, a.st, a.s);
  if (pre) mask |= 1u << 0;
  if (evs) (void)hipEventRecord(evs[1], stream);
  if (topo && !a.fuse_min) k_topo_min<false><<<1, 256, 0, stream>>>(a.c, a.P, a.prof, a.st, a.s);
  if (topo && !a.fuse_min) mask |= 1u << 1;
  if (evs) (void)hipEventRecord(evs[2], stream);
  const int32_t fx = NOWIN && !COMPAT && a.fuse_ext;   // extrema in the filter pass, no k_extrema
  k_filter_score<COMPAT, NOWIN><<<blocks, 256, 0, stream>>>(a.c, a.P, a.prof, a.dbp, a.st, a.s, topo && a.fuse_min, fx);
  mask |= 1u << 2;
  if (evs) (void)hipEventRecord(evs[3], stream);
  if (!NOWIN) k_window<COMPAT><<<1, kFinalThreads, 0, stream>>>(a.c, a.P, a.prof, a.st, a.s);
  if (!NOWIN) mask |= 1u << 3;
  if (evs) (void)hipEventRecord(evs[4], stream);
  if (!fx) k_extrema<NOWIN><<<blocks, 256, 0, stream>>>(a.c, a.P, a.prof, a.st, a.s);
  if (!fx) mask |= 1u << 4;
  if (evs) (void)hipEventRecord(evs[5], stream);
  // the last k_select block binds (no k_bind launch)
  k_select<COMPAT><<<blocks, 256, 0, stream>>>(a.c, a.P, a.prof, a.st, a.s, a.o, fx, NOWIN ? 2 : 1, a.chosen);
  mask |= 1u << 5;
  if (evs) (void)hipEventRecord(evs[6], stream);
  if (evs) (void)hipEventRecord(evs[7], stream);
  return mask;
}

// K = N (percentageOfNodesToScore >= 100 or fewer than 100 nodes): no
// window, so the window state comes from the filter pass (no k_window).
// NetworkBandwidth's error statuses are resolved in k_window, so its profiles
// always take the windowed cycle.
uint32_t launch_cycle(const LaunchArgs& a, hipStream_t stream, bool compat, bool topo, hipEvent_t* evs) {
  const bool nowin = num_feasible_nodes_to_find(a.prof.percentage_of_nodes_to_score, a.c.n) >= a.c.n &&
                     !prof_has_filter(a.prof, KSIM_PL_NETWORK_BANDWIDTH) &&
                     !prof_has_score(a.prof, KSIM_PL_NETWORK_BANDWIDTH);
  if (compat) {
    return nowin ? launch_cycle_t<true, true>(a, stream, topo, evs) : launch_cycle_t<true, false>(a, stream, topo, evs);
  } else {
    return nowin ? launch_cycle_t<false, true>(a, stream, topo, evs) : launch_cycle_t<false, false>(a, stream, topo, evs);
  }
}

void launch_cycle_filter(const LaunchArgs& a, hipStream_t stream, bool topo) {
  const int blocks = (a.c.n + 255) / 256;
  if (topo) k_topo_prefilter<<<blocks, 256, 0, stream>>>(a.c, a.P, a.prof, a.st, a.s);
  if (topo) k_topo_min<false><<<1, 256, 0, stream>>>(a.c, a.P, a.prof, a.st, a.s);
  k_filter_score<true, false><<<blocks, 256, 0, stream>>>(a.c, a.P, a.prof, a.dbp, a.st, a.s, 0, 0);
  k_window<true><<<1, kFinalThreads, 0, stream>>>(a.c, a.P, a.prof, a.st, a.s);
}

void launch_cycle_finish(const LaunchArgs& a, hipStream_t stream) {
  const int blocks = (a.c.n + 255) / 256;
  k_window<true><<<1, kFinalThreads, 0, stream>>>(a.c, a.P, a.prof, a.st, a.s);
  k_extrema<false><<<blocks, 256, 0, stream>>>(a.c, a.P, a.prof, a.st, a.s);
  k_select<true><<<blocks, 256, 0, stream>>>(a.c, a.P, a.prof, a.st, a.s, a.o, 0, 1, a.chosen);
}

// Framework-driven compat cycle: Filter of every scanned node (no window, no
// scheduler-state change) ...
void launch_fw_filter(const LaunchArgs& a, hipStream_t stream, bool topo) {
  const int blocks = (a.c.n + 255) / 256;
  if (topo) k_topo_prefilter<<<blocks, 256, 0, stream>>>(a.c, a.P, a.prof, a.st, a.s);
  if (topo) k_topo_min<false><<<1, 256, 0, stream>>>(a.c, a.P, a.prof, a.st, a.s);
  k_filter_score<true, false><<<blocks, 256, 0, stream>>>(a.c, a.P, a.prof, a.dbp, a.st, a.s, 0, 0);
}

// ... then PreScore / Score / NormalizeScore over the framework's list
// (a.s.ext_fail: 1 = not in the list), no selectHost bind.
void launch_fw_score(const LaunchArgs& a, hipStream_t stream) {
  const int blocks = (a.c.n + 255) / 256;
  k_window<true><<<1, kFinalThreads, 0, stream>>>(a.c, a.P, a.prof, a.st, a.s);
  k_extrema<false><<<blocks, 256, 0, stream>>>(a.c, a.P, a.prof, a.st, a.s);
  k_select<true><<<blocks, 256, 0, stream>>>(a.c, a.P, a.prof, a.st, a.s, a.o, 0, 0, nullptr);
}

// Small copies to or from the handle's coherent pinned staging (its device
// address) as one kernel launch: the per-call uploads and result copies of
// the framework-driven calls, where a DMA copy per piece costs more than the
// bytes (up to kCopyPieces pieces; 16-byte accesses when a piece is at least
// 16 bytes, its addresses then 16-byte aligned; byte accesses for the tail).
__device__ __forceinline__ void fw_begin_block(DevState* __restrict__ st, WinState* __restrict__ win, int32_t first,
                                               int32_t end) {
  for (int x = threadIdx.x; x < (int)(sizeof(WinState) / 4); x += blockDim.x)
    reinterpret_cast<uint32_t*>(win)[x] = 0;
  if (threadIdx.x == 0) {
    st->cursor = first;
    st->end = end;
    st->topo_flags = 0;
  }
}

__global__ __launch_bounds__(256) void k_copy_list(CopyList l) {
  if (l.bst && blockIdx.x == 0 && blockIdx.y == 0) fw_begin_block(l.bst, l.bwin, l.bfirst, l.bend);
  if (l.anode >= 0 && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)
    assume_pod(l.ac, l.aP, l.aP.pods[0], l.anode, l.asign);
  const int q = blockIdx.y;
  const uint8_t* src = l.src[q];
  uint8_t* dst = l.dst[q];
  const uint32_t n = l.n[q], n16 = n >> 4;
  for (uint32_t x = blockIdx.x * 256 + threadIdx.x; x < n16; x += gridDim.x * 256)
    reinterpret_cast<uint4*>(dst)[x] = reinterpret_cast<const uint4*>(src)[x];
  if (blockIdx.x == 0 && threadIdx.x < (n & 15u)) dst[(n16 << 4) + threadIdx.x] = src[(n16 << 4) + threadIdx.x];
}

// ksim_update_node_rows: the static columns of updated nodes, one block per
// row, from packed records in mapped pinned memory: [pos, alloc cpu / mem /
// eph / pods, flags, nb_limit, inv_cpu, inv_mem, taints x8, alloc_scalar x S,
// labels x L] as 64-bit words.
__global__ __launch_bounds__(64) void k_node_rows(DevCluster c, const int64_t* __restrict__ rec, int32_t words) {
  const int64_t* r = rec + (size_t)blockIdx.x * words;
  const int32_t pos = (int32_t)r[0];
  const size_t N = (size_t)c.n;
  for (int32_t f = threadIdx.x; f < words - 1; f += 64) {
    const int64_t x = r[1 + f];
    if (f == 0) const_cast<int64_t*>(c.alloc_cpu)[pos] = x;
    else if (f == 1) const_cast<int64_t*>(c.alloc_mem)[pos] = x;
    else if (f == 2) const_cast<int64_t*>(c.alloc_eph)[pos] = x;
    else if (f == 3) const_cast<int32_t*>(c.alloc_pods)[pos] = (int32_t)x;
    else if (f == 4) const_cast<uint32_t*>(c.flags)[pos] = (uint32_t)x;
    else if (f == 5) const_cast<int64_t*>(c.nb_limit)[pos] = x;
    else if (f == 6) const_cast<int64_t*>(reinterpret_cast<const int64_t*>(c.inv_cpu))[pos] = x;
    else if (f == 7) const_cast<int64_t*>(reinterpret_cast<const int64_t*>(c.inv_mem))[pos] = x;
    else if (f < 8 + KSIM_MAX_NODE_TAINTS) const_cast<uint16_t*>(c.taints)[(size_t)(f - 8) * N + pos] = (uint16_t)x;
    else if (f < 8 + KSIM_MAX_NODE_TAINTS + c.n_scalar)
      const_cast<int64_t*>(c.alloc_scalar)[(size_t)(f - 8 - KSIM_MAX_NODE_TAINTS) * N + pos] = x;
    else
      const_cast<uint32_t*>(c.labels)[(size_t)(f - 8 - KSIM_MAX_NODE_TAINTS - c.n_scalar) * N + pos] = (uint32_t)x;
  }
}

void launch_node_rows(const DevCluster& c, const int64_t* rec, int32_t n, int32_t words, hipStream_t stream) {
  if (n > 0) k_node_rows<<<n, 64, 0, stream>>>(c, rec, words);
}

void launch_copy_list(const CopyList& l, int count, hipStream_t stream) {
  uint32_t mx = 0;
  for (int q = 0; q < count; q++) mx = l.n[q] > mx ? l.n[q] : mx;
  const uint32_t blocks = ((mx >> 4) + 255) / 256;
  CopyList x = l;
  if (count == 0) x.n[0] = 0;                    // the begin job alone: one block, nothing to copy
  k_copy_list<<<dim3(blocks < 1 ? 1 : blocks > 64 ? 64 : blocks, count > 0 ? count : 1), 256, 0, stream>>>(x);
}

// ksim_fw_score's answers for the listed nodes only: comp = [raw S x n][norm
// S x n][total n] (list order), then the scored flags (n bytes); the host
// copies n entries back instead of N (every unlisted node's answers are 0)
// win_out (nullable): the cycle's WinState copied there too (block 0); comp
// and win_out may be the pinned staging's device address.
__global__ __launch_bounds__(256) void k_fw_gather(DevEvalOut o, const int32_t* __restrict__ nodes, int32_t n,
                                                   int32_t N, int32_t S, int64_t* __restrict__ comp,
                                                   const WinState* __restrict__ win, uint32_t* __restrict__ win_out) {
  if (win_out && blockIdx.x == 0)
    for (int x = threadIdx.x; x < (int)(sizeof(WinState) / 4); x += blockDim.x)
      win_out[x] = reinterpret_cast<const uint32_t*>(win)[x];
  const int32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const int32_t x = nodes[j];
  for (int32_t k = 0; k < S; k++) {
    comp[(size_t)k * n + j] = o.raw[(size_t)k * N + x];
    comp[(size_t)(S + k) * n + j] = o.norm[(size_t)k * N + x];
  }
  comp[(size_t)2 * S * n + j] = o.total[x];
  reinterpret_cast<uint8_t*>(comp + (size_t)(2 * S + 1) * n)[j] = o.scored[x];
}

void launch_fw_gather(const DevEvalOut& o, const int32_t* nodes, int32_t n, int32_t N, int32_t S, int64_t* comp,
                      const WinState* win, void* win_out, hipStream_t stream) {
  k_fw_gather<<<n > 0 ? (n + 255) / 256 : 1, 256, 0, stream>>>(o, nodes, n, N, S, comp, win, (uint32_t*)win_out);
}

// A framework-driven filter pass's start: the run header, the topology flags
// and the window state, in one launch (set_run's copy and two memsets).
__global__ __launch_bounds__(256) void k_fw_begin(DevState* __restrict__ st, WinState* __restrict__ win,
                                                  int32_t first, int32_t end) {
  fw_begin_block(st, win, first, end);
}

void launch_fw_begin(DevState* st, WinState* win, int32_t first, int32_t end, hipStream_t stream) {
  k_fw_begin<<<1, 256, 0, stream>>>(st, win, first, end);
}

void launch_fw_normalize(const LaunchArgs& a, int32_t slot, const int32_t* nodes, const int64_t* vals, int32_t n,
                         int64_t* out, hipStream_t stream) {
  k_fw_normalize<<<1, kFinalThreads, 0, stream>>>(a.prof, slot, a.st, a.s, nodes, vals, n, out);
}

void launch_filter_only(const LaunchArgs& a, hipStream_t stream) {
  // the variant the cycle launches (launch_cycle_t); the no-window one adds
  // into the window counters, which the caller clears afterwards
  const int blocks = (a.c.n + 255) / 256;
  const bool nowin = num_feasible_nodes_to_find(a.prof.percentage_of_nodes_to_score, a.c.n) >= a.c.n &&
                     !prof_has_filter(a.prof, KSIM_PL_NETWORK_BANDWIDTH) &&
                     !prof_has_score(a.prof, KSIM_PL_NETWORK_BANDWIDTH);
  if (nowin)
    k_filter_score<false, true><<<blocks, 256, 0, stream>>>(a.c, a.P, a.prof, a.dbp, a.st, a.s, a.fuse_min, a.fuse_ext);
  else
    k_filter_score<false, false><<<blocks, 256, 0, stream>>>(a.c, a.P, a.prof, a.dbp, a.st, a.s, a.fuse_min, 0);
}

void launch_assume(const DevCluster& c, const DevPods& P, int32_t pod, int32_t node, int sign, hipStream_t stream) {
  k_assume<<<1, 64, 0, stream>>>(c, P, pod, node, sign);
}

void launch_pshard_topo(const LaunchArgs& a, hipStream_t stream) {
  const int blocks = (a.c.n + 255) / 256;
  k_topo_prefilter<<<blocks, 256, 0, stream>>>(a.c, a.P, a.prof, a.st, a.s);
  k_dom_pack<<<1, 256, 0, stream>>>(a.c, a.P, a.st, a.s);
}

void launch_pshard_filter(const LaunchArgs& a, bool topo, hipStream_t stream) {
  const int blocks = (a.c.n + 255) / 256;
  if (topo) k_topo_min<true><<<1, 256, 0, stream>>>(a.c, a.P, a.prof, a.st, a.s);
  k_filter_score<false, false><<<blocks, 256, 0, stream>>>(a.c, a.P, a.prof, a.dbp, a.st, a.s, 0, 0);
  k_wcount_sh<<<1, kFinalThreads, 0, stream>>>(a.c, a.P, a.st, a.s);
}

void launch_pshard_window(const LaunchArgs& a, int32_t rank, int32_t world, hipStream_t stream) {
  k_window_sh<<<1, kFinalThreads, 0, stream>>>(a.c, a.P, a.prof, a.st, a.s, rank, world);
}

void launch_pshard_extrema(const LaunchArgs& a, bool soft, hipStream_t stream) {
  const int blocks = (a.c.n + 255) / 256;
  if (soft) k_wfinal_sh<<<1, 256, 0, stream>>>(a.c, a.P, a.st, a.s);
  k_extrema<false><<<blocks, 256, 0, stream>>>(a.c, a.P, a.prof, a.st, a.s);
}

void launch_pshard_select(const LaunchArgs& a, hipStream_t stream) {
  const int blocks = (a.c.n + 255) / 256;
  k_select<false><<<blocks, 256, 0, stream>>>(a.c, a.P, a.prof, a.st, a.s, a.o, 0, 0, nullptr);
  k_best_pack<<<1, 64, 0, stream>>>(a.c, a.st, a.s);
}

void launch_pshard_bind(const LaunchArgs& a, int32_t world, hipStream_t stream) {
  k_bind_sh<<<1, 256, 0, stream>>>(a.c, a.P, a.st, a.s, world, a.chosen);
}

void launch_group_reduce(const GroupPtrs& g, int64_t count, bool op_max, hipStream_t stream) {
  if (count <= 0) return;
  const int blocks = (int)std::min<int64_t>((count + 255) / 256, 1024);
  k_group_reduce<<<blocks, 256, 0, stream>>>(g, count, op_max ? 1 : 0);
}

void launch_group_gather(const GroupPtrs& src, const GroupPtrs& dst, int32_t words, hipStream_t stream) {
  k_group_gather<<<1, 256, 0, stream>>>(src, dst, words);
}

}  // namespace ksim
