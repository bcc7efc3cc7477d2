// ksim_match.hip — label-selector / affinity-term matching as an int8
// contraction on the matrix cores (BASELINE north_star).
//
// Upstream PodTopologySpread and InterPodAffinity run their selectors and
// terms against every existing pod in PreFilter / PreScore (podtopologyspread
// countPodsMatchSelector, interpodaffinity getExistingAntiAffinityCounts /
// getIncomingAffinityAntiAffinityCounts / processExistingPod, reached through
// scheduler/plugin/wrappedplugin.go:427-486).  The engine keeps those answers
// as count classes (ksim/topology.py); this file computes them on the device.
//
// The host reduces every matcher (namespace predicate AND label selector, or
// the conjunction of a pod's required affinity terms) to requirements over a
// feature vocabulary: ("ns", name), ("kv", key, value), ("key", key) — only
// features some requirement names.  A pod signature (namespace, labels) is a
// one-hot row over that vocabulary.  Then
//
//   hits[s][r] = sum_f A[s][f] * B[f][r]        (int8 MFMA, i32 accumulate)
//   sat[s][r]  = (hits > 0) XOR neg[r]          In / Exists: some feature hits
//                                               NotIn / DoesNotExist: none hits
//   match[s][m] = AND of sat[s][r] over the requirements r of matcher m
//
// In(k, V) names ("kv", k, v) for v in V; Exists(k) names ("key", k); the
// namespace predicate is In over ("ns", n); a nil selector is one positive
// requirement naming no feature (never satisfied).  The count classes are
// then cnt[c][node] = number of bound pods on node whose signature matches
// class c's matcher (k_match_count, one thread per bound pod).
//
// Operand maps of v_mfma_i32_16x16x64_i8: lane l supplies 16 bytes of row
// l & 15 of A (and of column l & 15 of B) from k-slice 16 * (l >> 4).  A and B
// take the same lane -> k assignment, so the sum over k is the same whatever
// order the instruction walks the 16 bytes in.  C/D: col = l & 15, row =
// 4 * (l >> 4) + i (the gfx950 C/D map is the same for every dtype).
#include "ksim_device.h"
#include "ksim_internal.h"

namespace ksim {

typedef int v4i __attribute__((ext_vector_type(4)));

// A [Sp][Fp] and Bt [Rp][Fp] one-hot rows from the CSR feature lists.
__global__ __launch_bounds__(256) void k_match_scatter(int8_t* __restrict__ rows, int32_t n_rows, int32_t fp,
                                                       const int32_t* __restrict__ off,
                                                       const int32_t* __restrict__ feat) {
  const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rows) return;
  int8_t* row = rows + (size_t)r * fp;
  for (int32_t j = off[r]; j < off[r + 1]; j++) row[feat[j]] = 1;
}

// One block per 16 signatures: the 16 x Rp hit tile on the matrix cores (4
// waves over the requirement column tiles), satisfied bits to LDS, then every
// matcher of the 16 rows as a ballot word.
__global__ __launch_bounds__(256) void k_match_mfma(DevMatch m) {
  __shared__ uint16_t sat[16][kMatchMaxReqs / 16];
  const int32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int32_t row0 = blockIdx.x * 16;
  const int32_t n_ct = m.rp / 16;
  const int8_t* arow = m.a + (size_t)(row0 + (lane & 15)) * m.fp + 16 * (lane >> 4);
  for (int32_t ct = wave; ct < n_ct; ct += 4) {
    const int32_t col = ct * 16 + (lane & 15);
    const int8_t* brow = m.bt + (size_t)col * m.fp + 16 * (lane >> 4);
    v4i acc = {0, 0, 0, 0};
    for (int32_t k0 = 0; k0 < m.fp; k0 += 64) {
      const v4i a = *reinterpret_cast<const v4i*>(arow + k0);
      const v4i b = *reinterpret_cast<const v4i*>(brow + k0);
      acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc, 0, 0, 0);
    }
    const bool neg = m.neg[col] != 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      // ballot bit 16 g + c: row 4 g + i, column ct * 16 + c
      const uint64_t w = __ballot((acc[i] > 0) != neg);
      if ((lane & 15) == 0) sat[4 * (lane >> 4) + i][ct] = (uint16_t)(w >> (lane & 48));
    }
  }
  __syncthreads();
  // matchers: wave w takes rows w, w + 4, ..; lane = matcher within a 64-chunk
  for (int32_t r = wave; r < 16; r += 4) {
    const int32_t s = row0 + r;
    if (s >= m.s) break;
    for (int32_t mb = 0; mb < m.m; mb += 64) {
      const int32_t mi = mb + lane;
      bool ok = mi < m.m;
      if (ok) {
        for (int32_t j = m.m_off[mi]; j < m.m_off[mi + 1]; j++) {
          const int32_t q = m.m_req[j];
          if (!((sat[r][q >> 4] >> (q & 15)) & 1)) {
            ok = false;
            break;
          }
        }
      }
      const uint64_t w = __ballot(ok);
      uint32_t* out = m.bits + (size_t)s * m.w + (mb >> 5);
      if (lane == 0) out[0] = (uint32_t)w;
      if (lane == 32 && (mb >> 5) + 1 < m.w) out[1] = (uint32_t)(w >> 32);
    }
  }
}

// Per signature: the classes whose matcher it satisfies, as bit words (one
// block per (signature, 256 classes), a 1-D grid: signatures may exceed the
// 65,536 blocks of a grid's y dimension).
__global__ __launch_bounds__(256) void k_match_classes(DevMatch m) {
  const int32_t chunks = (m.c + 255) / 256;
  const int32_t s = blockIdx.x / chunks;
  const int32_t c = (blockIdx.x % chunks) * blockDim.x + threadIdx.x;
  const bool hit = c < m.c && ((m.bits[(size_t)s * m.w + (m.cls_matcher[c] >> 5)] >> (m.cls_matcher[c] & 31)) & 1);
  const uint64_t w = __ballot(hit);
  const int32_t lane = threadIdx.x & 63;
  const int32_t word = c >> 5;
  if ((lane & 31) == 0 && word < m.cw) m.cls_bits[(size_t)s * m.cw + word] = (uint32_t)(w >> (lane & 32));
}

// One thread per bound pod: +1 on every class its signature matches.
__global__ __launch_bounds__(256) void k_match_count(DevMatch m) {
  const int32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= m.p) return;
  const int32_t s = m.pod_sig[p], node = m.pod_node[p];
  const uint32_t* cb = m.cls_bits + (size_t)s * m.cw;
  for (int32_t wd = 0; wd < m.cw; wd++) {
    uint32_t x = cb[wd];
    while (x) {
      const int32_t c = wd * 32 + __builtin_ctz(x);
      x &= x - 1;
      atomicAdd(m.cnt + (size_t)c * m.n + node, 1);
    }
  }
}

void launch_match(const DevMatch& m, hipStream_t stream) {
  k_match_scatter<<<(m.sp + 255) / 256, 256, 0, stream>>>(const_cast<int8_t*>(m.a), m.s, m.fp, m.sig_off, m.sig_feat);
  k_match_scatter<<<(m.rp + 255) / 256, 256, 0, stream>>>(const_cast<int8_t*>(m.bt), m.r, m.fp, m.req_off, m.req_feat);
  k_match_mfma<<<m.sp / 16, 256, 0, stream>>>(m);
  if (m.c > 0 && m.s > 0) {
    k_match_classes<<<m.s * ((m.c + 255) / 256), 256, 0, stream>>>(m);
    if (m.p > 0) k_match_count<<<(m.p + 255) / 256, 256, 0, stream>>>(m);
  }
}

}  // namespace ksim
