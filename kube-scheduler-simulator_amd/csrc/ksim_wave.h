// ksim_wave.h — wave64 primitives for gfx950.
//
// wave_max_u64_dpp64: the DPP reduction (quad_perm xor1, xor2, row_ror 4, 8
// inside each 16-lane row, then row_bcast15 / row_bcast31 across rows, result
// in lane 63, broadcast by readlane).  It never touches the LDS, unlike the
// __shfl_xor form (ds_bpermute) — on the repair kernel's single-wave critical
// path that difference is several hundred cycles per reduction.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ksim {

template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v) {
  const int lo = (int)(uint32_t)v, hi = (int)(uint32_t)(v >> 32);
  const int lo2 = __builtin_amdgcn_update_dpp(lo, lo, CTRL, ROW_MASK, 0xf, false);
  const int hi2 = __builtin_amdgcn_update_dpp(hi, hi, CTRL, ROW_MASK, 0xf, false);
  return ((uint64_t)(uint32_t)hi2 << 32) | (uint32_t)lo2;
}

__device__ __forceinline__ uint64_t umax64(uint64_t a, uint64_t b) { return a > b ? a : b; }

__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int lane) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane);
  return ((uint64_t)hi << 32) | lo;
}

// Wave max over u64 by 64-bit DPP steps; all 64 lanes must be active.
__device__ __forceinline__ uint64_t wave_max_u64_dpp64(uint64_t v) {
  v = umax64(v, dpp_u64<0xb1, 0xf>(v));    // quad_perm [1,0,3,2]
  v = umax64(v, dpp_u64<0x4e, 0xf>(v));    // quad_perm [2,3,0,1]
  v = umax64(v, dpp_u64<0x124, 0xf>(v));   // row_ror:4
  v = umax64(v, dpp_u64<0x128, 0xf>(v));   // row_ror:8
  v = umax64(v, dpp_u64<0x142, 0xa>(v));   // row_bcast:15 -> rows 1, 3
  v = umax64(v, dpp_u64<0x143, 0xc>(v));   // row_bcast:31 -> rows 2, 3
  return readlane_u64(v, 63);
}

template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp_max_u32(uint32_t v) {
  // old = 0 (the identity of unsigned max) for disabled rows and lanes, so the
  // move folds into v_max_u32 with a DPP operand
  const uint32_t w = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROW_MASK, 0xf, true);
  return v > w ? v : w;
}

// Wave max over u32; all 64 lanes must be active.
__device__ __forceinline__ uint32_t wave_max_u32_dpp(uint32_t v) {
  v = dpp_max_u32<0xb1, 0xf>(v);
  v = dpp_max_u32<0x4e, 0xf>(v);
  v = dpp_max_u32<0x124, 0xf>(v);
  v = dpp_max_u32<0x128, 0xf>(v);
  v = dpp_max_u32<0x142, 0xa>(v);
  v = dpp_max_u32<0x143, 0xc>(v);
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp_add_u32(uint32_t v) {
  // old = 0 for disabled rows and lanes (the identity of the sum)
  return v + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROW_MASK, 0xf, true);
}

// Wave sum over u32 by the same DPP steps as wave_max_u32_dpp (pairs, quads,
// rotations inside each 16-lane row, then rows 0+1 -> 1, 2+3 -> 3, 1 -> 2, 3;
// the total in lane 63); all 64 lanes must be active.
__device__ __forceinline__ uint32_t wave_sum_u32_dpp(uint32_t v) {
  v = dpp_add_u32<0xb1, 0xf>(v);
  v = dpp_add_u32<0x4e, 0xf>(v);
  v = dpp_add_u32<0x124, 0xf>(v);
  v = dpp_add_u32<0x128, 0xf>(v);
  v = dpp_add_u32<0x142, 0xa>(v);
  v = dpp_add_u32<0x143, 0xc>(v);
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// The number of set bits of m in the lanes below this one.
__device__ __forceinline__ uint32_t mask_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Wave max over u64 keys, high words first: one 32-bit reduction, and when a
// single lane holds the maximal high word (the common case for tie-break keys,
// whose high word carries hash bits) its low word by one readlane; otherwise a
// second 32-bit reduction over the low words of the lanes holding it.
__device__ __forceinline__ uint64_t wave_max_u64_hi(uint64_t v) {
  const uint32_t hi = (uint32_t)(v >> 32), lo = (uint32_t)v;
  const uint32_t mh = wave_max_u32_dpp(hi);
  const uint64_t tie = __ballot(hi == mh);
  uint32_t ml;
  if ((tie & (tie - 1)) == 0)
    ml = (uint32_t)__builtin_amdgcn_readlane((int)lo, __builtin_ctzll(tie));
  else
    ml = wave_max_u32_dpp(hi == mh ? lo : 0u);
  return ((uint64_t)mh << 32) | ml;
}

// Wave max over u64 (all 64 lanes active): the high-word-first form.
__device__ __forceinline__ uint64_t wave_max_u64_dpp(uint64_t v) { return wave_max_u64_hi(v); }

__device__ __forceinline__ void cswap_desc(uint64_t& a, uint64_t& b) {
  const uint64_t hi = a > b ? a : b, lo = a > b ? b : a;
  a = hi;
  b = lo;
}

// Order LDS accesses of one wave without a workgroup barrier (which would
// also wait for every outstanding global memory operation).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}


// A workgroup barrier for LDS hand-offs only: the fences are LDS-scoped, so
// the barrier waits for the wave's LDS operations (lgkmcnt) and not for its
// outstanding global loads and stores, as __syncthreads does (a load issued
// early for use after the barrier stays in flight across it; a store does not
// hold the barrier until it is acknowledged).  Not for hand-offs through
// global memory.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// *s = min(*s, the block's first thread with pred) for one-dimensional blocks:
// one LDS atomicMin per wave (its first set lane) instead of one per thread,
// which would all hit the same word.
__device__ __forceinline__ void block_first_min(int32_t* s, bool pred) {
  const uint64_t m = __ballot(pred);
  if (m && (threadIdx.x & 63) == 0) atomicMin(s, (int32_t)(threadIdx.x & ~63u) + __builtin_ctzll(m));
}

}  // namespace ksim
