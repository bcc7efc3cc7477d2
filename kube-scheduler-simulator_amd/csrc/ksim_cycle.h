// ksim_cycle.h — block-level pieces of the per-pod cycle shared by its
// kernels (ksim_kernels.hip) and the topology batch (ksim_tbatch.hip).
#pragma once

#include "ksim_device.h"
#include "ksim_internal.h"
#include "ksim_wave.h"

namespace ksim {

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  lo = (uint32_t)__shfl_xor((int)lo, m, 64);
  hi = (uint32_t)__shfl_xor((int)hi, m, 64);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ int64_t wave_min_i64(int64_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    int64_t o = (int64_t)shfl_xor_u64((uint64_t)v, m);
    v = o < v ? o : v;
  }
  return v;
}

// Per-slot extrema images of this block's values -> one atomicMax per slot.
// zmask: slots whose raw score is 0 on every node for this pod; their extrema
// are (0, 0) whenever some node is feasible (and unread otherwise), so block 0
// stores them without a reduction.
// s_cnt (optional): per wave {feasible, ignored} counts, added to the window
// counters once per block after the barrier (one atomic per block, not per wave).
__device__ __forceinline__ void block_extrema(const ksim_profile& prof, WinState* win, const uint64_t (&ix)[KSIM_MAX_SCORE],
                                              const uint64_t (&in)[KSIM_MAX_SCORE], uint64_t (*s_red)[2 * KSIM_MAX_SCORE],
                                              uint32_t zmask = 0, const int32_t (*s_cnt)[2] = nullptr) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int S = prof.n_score;
#pragma unroll
  for (int k = 0; k < KSIM_MAX_SCORE; k++) {
    if (k >= S) break;
    if (norm_kind(prof.score[k]) == kNormNone || ((zmask >> k) & 1u)) continue;
    const uint64_t a = wave_max_u64_dpp(ix[k]), b = wave_max_u64_dpp(in[k]);
    if (lane == 0) {
      s_red[wv][2 * k] = a;
      s_red[wv][2 * k + 1] = b;
    }
  }
  lds_barrier();                                   // an LDS hand-off: the caller's stores stay in flight
  if (tid < 2 * KSIM_MAX_SCORE && tid < 2 * S && norm_kind(prof.score[tid >> 1]) != kNormNone) {
    uint64_t m = 0;
    if ((zmask >> (tid >> 1)) & 1u) {
      m = blockIdx.x == 0 ? ((tid & 1) ? ~(1ull << 63) : (1ull << 63)) : 0ull;   // min_image(0) / max_image(0)
    } else {
#pragma unroll
      for (int w = 0; w < 4; w++) m = umax64(m, s_red[w][tid]);
    }
    if (m) atomicMax(reinterpret_cast<unsigned long long*>(&win->ext[tid]), (unsigned long long)m);
  }
  if (s_cnt && (tid == 64 || tid == 65)) {
    const int q = tid - 64;
    const int32_t v = s_cnt[0][q] + s_cnt[1][q] + s_cnt[2][q] + s_cnt[3][q];
    if (v) atomicAdd(q ? &win->nign : &win->nfeas, v);
  }
}

// scoreForCount with a single constraint (k_extrema's sum from 0, unfused)
__device__ __forceinline__ int64_t soft_score(int64_t cnt, double w, int32_t max_skew) {
  double score = 0;
  score = score + ((double)cnt * w + (double)(max_skew - 1));
  return (int64_t)round(score);
}

// The block's PodTopologySpread critical paths (fuse_min: per hard use, the
// minimum match count over the domains with a presence marker, wave 0) into
// s_min, and (pt) the InterPodAffinity emptiness flags, len(affinityCounts) > 0
// / len(topologyScore) > 0, from the persistent tables (wave 1) into *s_tf;
// block x == 0 also stores the flags to *flags_out.  The caller's barrier
// publishes both.
__device__ __forceinline__ void topo_block_setup(const DevCluster& c, const DevPods& P0, const DevScratch& s,
                                                 const ksim_topo_use* U, const UseMasks& m, bool pt, bool fuse_min,
                                                 int64_t* s_min, uint32_t* s_tf, uint32_t* flags_out) {
  if (threadIdx.x < 64 && fuse_min) {              // the critical paths, one wave
    for (uint32_t b = m.hard; b; b &= b - 1) {
      const int i = __builtin_ctz(b);
      const ksim_topo_use u = load_use(U, i);
      int64_t mn = 2147483647;
      if (u.col != KSIM_COL_NONE) {
        const int32_t V = c.col_nvals[u.col];
        const int64_t* d = pt ? P0.ptab + u._pad : s.dom + (size_t)i * c.vmax;
        for (int32_t v = threadIdx.x; v < V; v += 64) {
          const int64_t x = d[v];
          if ((x >> kDomMarkShift) != 0) mn = min(mn, x & kDomCountMask);
        }
      }
      mn = wave_min_i64(mn);
      if (threadIdx.x == 0) s_min[i] = mn;
    }
  } else if (threadIdx.x >= 64 && threadIdx.x < 128 && pt) {
    // (k_topo_prefilter's flags): some node with the key and a count
    uint32_t f = 0;
    for (uint32_t b = m.aff | m.score; b; b &= b - 1) {
      const int i = __builtin_ctz(b);
      const ksim_topo_use u = load_use(U, i);
      if (u.col == KSIM_COL_NONE || u.cls < 0) continue;
      const bool total = (m.node_count >> i) & 1u;   // a kPtabTotal table
      const int32_t V = total ? 1 : c.col_nvals[u.col];
      const int64_t* d = P0.ptab + u._pad;
      bool nz = false;
      for (int32_t v = (int32_t)threadIdx.x - 64 + (total ? 0 : 1); v < V; v += 64) nz = nz || d[v] != 0;
      if (__ballot(nz))
        f |= (((m.aff >> i) & 1u) ? kTopoAffinityNonEmpty : 0u) | (((m.score >> i) & 1u) ? kTopoScoreNonEmpty : 0u);
    }
    if (threadIdx.x == 64) {
      *s_tf = f;
      if (blockIdx.x == 0) *flags_out = f;
    }
  }
}

}  // namespace ksim
