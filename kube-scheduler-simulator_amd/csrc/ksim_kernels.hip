// ksim_kernels.hip — HIP kernels of the scheduling cycle (gfx950).
//
// Two execution paths produce identical placements (both bit-exact with the
// oracle):
//
// A. Per-pod path (compat mode, and pods the batch path cannot take):
//    k_filter_score  grid over nodes: RunFilterPlugins (SURVEY §8(a) a17, a22,
//                    a25, a26) and, for feasible nodes, every raw Score (a23-a26).
//    k_finalize      one 1024-thread block: numFeasibleNodesToFind window by a
//                    block prefix scan (a16), NormalizeScore extrema (a31),
//                    weighted totals (a18), selectHost as a packed-u64 argmax
//                    (a19, TB tie-break), NodeInfo.AddPod (a20).
//
// B. Batch path (P100, pods whose normalized plugins are constant over
//    nodes): ksim_batch.hip.
#include "ksim_device.h"
#include "ksim_internal.h"

namespace ksim {

// ---- wave64 / block reductions ------------------------------------------------
__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  lo = (uint32_t)__shfl_xor((int)lo, m, 64);
  hi = (uint32_t)__shfl_xor((int)hi, m, 64);
  return ((uint64_t)hi << 32) | lo;
}

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

__device__ __forceinline__ int64_t wave_min_i64(int64_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    int64_t o = (int64_t)shfl_xor_u64((uint64_t)v, m);
    v = o < v ? o : v;
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

// ---- normalization ----------------------------------------------------------
// Extrema a slot needs, merged over the kept feasible list:
//   DefaultNormalizeScore: maxCount = max(0, max)          (helper/normalize_score.go)
//   PodTopologySpread:     maxScore = max(0, max), minScore = min
//   InterPodAffinity:      min / max (only when topologyScore is non-empty)
__device__ __forceinline__ int64_t normalize_value(int32_t kind, int64_t v, int64_t gmax, int64_t gmin) {
  switch (kind) {
    case kNormDefault: {
      int64_t m = gmax > 0 ? gmax : 0;
      return m == 0 ? v : (int64_t)kMaxNodeScore * v / m;
    }
    case kNormDefaultReverse: {
      int64_t m = gmax > 0 ? gmax : 0;
      return m == 0 ? (int64_t)kMaxNodeScore : (int64_t)kMaxNodeScore - (int64_t)kMaxNodeScore * v / m;
    }
    case kNormPTS: {
      int64_t mx = gmax > 0 ? gmax : 0;
      return mx == 0 ? (int64_t)kMaxNodeScore : (int64_t)kMaxNodeScore * (mx + gmin - v) / mx;
    }
    case kNormIPA:   // topologyScore empty for pods without terms: scores left unchanged
    default:
      return v;
  }
}

// ==== A. per-pod path ===========================================================
template <bool COMPAT>
__global__ __launch_bounds__(256) void k_filter_score(DevCluster c, DevPods P, ksim_profile prof,
                                                      const DevState* __restrict__ st, DevScratch s) {
  const int32_t pi = st->cursor;
  if (pi >= st->end) return;
  const int32_t node = blockIdx.x * blockDim.x + threadIdx.x;
  if (node >= c.n) return;
  const ksim_pod& p = P.pods[pi];
  const NodeRow r = load_row(c, node);
  uint32_t det;
  const uint8_t res = run_filter_plugins(c, P, prof, p, r, det);
  s.fail[node] = res;
  if (COMPAT) s.detail[node] = det;
  if (res != KSIM_PASSED) return;
  int64_t part = 0;
  for (int k = 0; k < prof.n_score; k++) {
    const int pl = prof.score[k];
    const int64_t v = score_plugin_raw(c, P, prof, p, pl, r);
    if (norm_kind(pl) == kNormNone) {
      const int64_t w = prof.score_weight[k] == 0 ? 1 : prof.score_weight[k];
      part += v * w;
      if (COMPAT) s.raw[(size_t)k * c.n + node] = v;
    } else {
      s.raw[(size_t)k * c.n + node] = v;
    }
  }
  s.part[node] = part;
}

template <bool COMPAT>
__global__ __launch_bounds__(kFinalThreads) void k_finalize(DevCluster c, DevPods P, ksim_profile prof,
                                                            DevState* __restrict__ st, DevScratch s,
                                                            DevEvalOut o, int32_t* __restrict__ chosen_out) {
  __shared__ int64_t sh64[kFinalWaves];
  __shared__ uint64_t shu[kFinalWaves];
  __shared__ int32_t sh32[kFinalWaves];
  __shared__ int32_t s_cut, s_single;
  __shared__ int64_t s_gmax[KSIM_MAX_SCORE], s_gmin[KSIM_MAX_SCORE];

  const int32_t pi = st->cursor;
  if (pi >= st->end) return;
  const int tid = threadIdx.x;
  const int32_t N = c.n;
  const int32_t K = num_feasible_nodes_to_find(prof.percentage_of_nodes_to_score, N);
  const int32_t start = st->next_start;
  const int64_t seq = st->pod_seq;
  const int32_t chunk = (N + kFinalThreads - 1) / kFinalThreads;
  const int32_t lo = min(N, tid * chunk), hi = min(N, lo + chunk);

  // Phase A: feasible count per rotated chunk, block scan, locate the (K+1)-th.
  int32_t cnt = 0;
  for (int32_t r = lo; r < hi; r++) {
    int32_t node = start + r;
    if (node >= N) node -= N;
    cnt += s.fail[node] == KSIM_PASSED;
  }
  int32_t excl, total;
  block_scan_i32(cnt, excl, total, sh32);
  if (tid == 0) { s_cut = N; s_single = -1; }
  __syncthreads();
  if (total > K && excl <= K && K < excl + cnt) {
    int32_t run = excl;
    for (int32_t r = lo; r < hi; r++) {
      int32_t node = start + r;
      if (node >= N) node -= N;
      if (s.fail[node] == KSIM_PASSED) {
        if (run == K) { s_cut = r; break; }
        run++;
      }
    }
  }
  __syncthreads();
  const int32_t cut = s_cut;                         // rotated position of the (K+1)-th feasible, or N
  const int32_t evaluated = cut < N ? cut + 1 : N;
  const int32_t nf = total < K ? total : K;
  const int32_t whi = min(hi, cut);
  const int S = prof.n_score;

  if (COMPAT) {
    for (int32_t r = lo; r < hi; r++) {
      int32_t node = start + r;
      if (node >= N) node -= N;
      if (r >= evaluated) s.fail[node] = KSIM_NOT_EVALUATED;
      o.scored[node] = 0;
      o.total[node] = 0;
      for (int k = 0; k < S; k++) {
        o.raw[(size_t)k * N + node] = 0;
        o.norm[(size_t)k * N + node] = 0;
      }
    }
  }

  int32_t chosen = -1;
  if (nf == 1) {
    for (int32_t r = lo; r < whi; r++) {
      int32_t node = start + r;
      if (node >= N) node -= N;
      if (s.fail[node] == KSIM_PASSED) s_single = node;
    }
    __syncthreads();
    chosen = s_single;
  } else if (nf > 1) {
    // Phase B: NormalizeScore extrema over the kept feasible list.
    for (int k = 0; k < S; k++) {
      const int32_t kind = norm_kind(prof.score[k]);
      if (kind == kNormNone) continue;
      int64_t mx = INT64_MIN, mn = INT64_MAX;
      for (int32_t r = lo; r < whi; r++) {
        int32_t node = start + r;
        if (node >= N) node -= N;
        if (s.fail[node] != KSIM_PASSED) continue;
        const int64_t v = s.raw[(size_t)k * N + node];
        mx = v > mx ? v : mx;
        mn = v < mn ? v : mn;
      }
      mx = block_max_i64(mx, sh64);
      mn = block_min_i64(mn, sh64);
      if (tid == 0) { s_gmax[k] = mx; s_gmin[k] = mn; }
    }
    __syncthreads();
    // Phase C: weighted totals and the tie-break argmax.
    uint64_t best = 0;
    for (int32_t r = lo; r < whi; r++) {
      int32_t node = start + r;
      if (node >= N) node -= N;
      if (s.fail[node] != KSIM_PASSED) continue;
      int64_t tot = S == 0 ? 1 : s.part[node];
      for (int k = 0; k < S; k++) {
        const int32_t kind = norm_kind(prof.score[k]);
        const int64_t raw = s.raw[(size_t)k * N + node];
        int64_t nv = raw;
        if (kind != kNormNone) {
          nv = normalize_value(kind, raw, s_gmax[k], s_gmin[k]);
          const int64_t w = prof.score_weight[k] == 0 ? 1 : prof.score_weight[k];
          tot += nv * w;
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
      const uint64_t key = tb_key(tot, prof.tiebreak_seed, seq, node);
      best = key > best ? key : best;
    }
    best = block_max_u64<kFinalWaves>(best, shu);
    chosen = key_node(best);
  }

  // Phase D: assume/bind + scheduler state.
  if (tid == 0) {
    const ksim_pod& p = P.pods[pi];
    int32_t ns = start + (cut < N ? cut : N);
    ns %= N;
    st->next_start = ns;
    st->evals += evaluated;
    if (chosen >= 0) {
      assume_pod(c, p, chosen, 1);
      st->scheduled += 1;
    } else {
      st->unschedulable += 1;
    }
    if (chosen_out) chosen_out[pi] = chosen;
    st->chosen = chosen;
    st->status = chosen >= 0 ? KSIM_STATUS_SCHEDULED : KSIM_STATUS_UNSCHEDULABLE;
    st->n_feasible = nf;
    st->n_evaluated = evaluated;
    st->n_processed = cut < N ? cut : N;
    st->k_to_find = K;
    st->next_start_after = ns;
    st->pod_seq = seq + 1;
    st->cursor = pi + 1;
  }
}

__global__ void k_assume(DevCluster c, ksim_pod p, int32_t node, int sign) {
  if (threadIdx.x == 0 && blockIdx.x == 0) assume_pod(c, p, node, sign);
}

// ---- launchers ----------------------------------------------------------------
const char* const kKernelNames[kKernelsPerCycle] = {"k_filter_score", "k_finalize"};

void launch_cycle(const LaunchArgs& a, hipStream_t stream, bool compat, hipEvent_t* evs) {
  const int blocks = (a.c.n + 255) / 256;
  if (evs) (void)hipEventRecord(evs[0], stream);
  if (compat)
    k_filter_score<true><<<blocks, 256, 0, stream>>>(a.c, a.P, a.prof, a.st, a.s);
  else
    k_filter_score<false><<<blocks, 256, 0, stream>>>(a.c, a.P, a.prof, a.st, a.s);
  if (evs) (void)hipEventRecord(evs[1], stream);
  if (compat)
    k_finalize<true><<<1, kFinalThreads, 0, stream>>>(a.c, a.P, a.prof, a.st, a.s, a.o, a.chosen);
  else
    k_finalize<false><<<1, kFinalThreads, 0, stream>>>(a.c, a.P, a.prof, a.st, a.s, a.o, a.chosen);
  if (evs) (void)hipEventRecord(evs[2], stream);
}

void launch_assume(const DevCluster& c, const ksim_pod& p, int32_t node, int sign, hipStream_t stream) {
  k_assume<<<1, 64, 0, stream>>>(c, p, node, sign);
}

}  // namespace ksim
