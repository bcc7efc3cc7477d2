// ksim_adapt.hip — the speculative batch path under ADAPT (gfx950).
//
// ADAPT is the simulator's forced default (percentageOfNodesToScore = 0): a pod
// scans nodes in nodeTree order from nextStartNodeIndex and keeps the first K =
// numFeasibleNodesToFind(N) feasible ones; the scan start of pod i+1 is pod i's
// start plus the nodes pod i processed.  For a batch of B
// batchable pods (same class of pods as ksim_batch.hip) five launches give the
// placements of the pod-by-pod cycle, bit-exact:
//
//   k_adapt_mask    grid (64-node words, pods): the S0 feasibility bitmap of
//                   every pod (static filters + Fit filter; one ballot per word).
//   k_adapt_window  one block, one thread per pod: the scan windows.  Pod i's
//                   start depends on every earlier pod's processed count, so the
//                   starts are found by relaxation: guess s_i = s_0 + i*K, let
//                   every pod find its cut (the K-th feasible node from s_i) in
//                   its bitmap, re-derive the starts as the prefix sum of the
//                   processed counts, repeat.  Pod 0's start is exact and each
//                   round extends the exact prefix; a fixpoint is exact.  The
//                   first round's cuts come from k_adapt_cut0 (a wave per pod).
//   k_adapt_top    one block per pod: TB keys of the kept nodes (the first K
//                   feasible of its window), the pod's exact top-T.
//   k_adapt_pairs   every block runs the greedy chain of ksim_batch.hip on those
//                   lists; then block j, thread k < j: pod j on pod k's guessed node once pod
//                   k is bound there, if the node lies in pod j's window: the key
//                   (M_j = max) and whether a node feasible under S0 became
//                   infeasible at or before the cut ("broken": pod j's window, and
//                   every later start, would shift).
//   k_adapt_commit  one block: the chain is cut at the first broken pod, then
//                   validated against M and committed as on the P100 path; the
//                   scheduler state advances to the start after the last committed pod.
//
// Exactness: binds only remove capacity, so feasibility under the current state
// is S0 feasibility minus flips on bound nodes (static filters never change).
// Bound nodes are the guesses of earlier pods of the batch.  Up to the first
// broken pod no window differs from the serial one; the chain argument of
// ksim_batch.hip then applies within each window.
#include "ksim_device.h"
#include "ksim_internal.h"
#include "ksim_wave.h"
#include "ksim_commit.h"
#include "ksim_chain.h"

namespace ksim {

// Filter outcome of a batchable pod on a node: static filters and Fit only.
// pi: the pod's queue index; a pod in a static class (DevPods::stab, built for
// the loaded queue) reads its static verdict from the class row instead of
// running the static filters (taints, node affinity: uniform loops the
// scalar unit runs per node and pod).
__device__ __forceinline__ bool batch_feasible(const DevCluster& c, const DevPods& P, const BatchProg& bp,
                                               const ksim_pod& p, const NodeRow& r, bool trivial, int32_t pi) {
  if (!trivial) {
    const int32_t scls = P.stab ? P.sclass[pi] : -1;   // uniform
    if (scls >= 0 ? !stab_pass(P.stab[(size_t)scls * c.n + r.node]) : !static_filters_pass(c, P, bp, p, r))
      return false;
  }
  return !bp.has_fit_filter || !fits_request(r, p, c.n_scalar, c.fit_ignore);
}

// The S0 feasibility bitmaps, node-stationary: a block of 256 threads holds
// one node per thread (its row loaded once) and sweeps mp <= 64 pods of the
// batch, one ballot per pod and 64-node word.  (A pod-per-block form re-reads
// every node row once per pod: B x the node table from L2 / MALL per batch,
// ~190 us at 100k nodes; here a row is read once per mp pods.)  mp shrinks on
// small clusters so the grid still fills the chip (mask_pods).
// (profiles/r04/maskdiv: with the LDS-staged pod loop, 1,280 in place of
// 2,560 blocks at 5,000 nodes: k_adapt_mask_commit 8.9 -> 7.9 us; at 100,000
// nodes the 2,048-block grid stays best, 15.8 against 16.6 us)
__host__ __device__ inline int32_t mask_pods(int32_t n_words) {
  const int32_t wb = (n_words + 3) / 4;            // 4 words (waves) per block
  const int32_t mp = wb / (n_words <= 256 ? 4 : 8);   // about 2,048 blocks over B pods (1,024 small)
  return mp < 1 ? 1 : mp > 64 ? 64 : mp;
}

__global__ __launch_bounds__(256) void k_adapt_mask_ns(DevCluster c, DevPods P, const BatchProg* __restrict__ bp_p,
                                                       const DevState* __restrict__ st, uint64_t* __restrict__ amask,
                                                       int32_t n_words, int32_t mp) {
  const BatchProg& bp = *bp_p;
  const int32_t base = st->cursor;
  const int32_t nb = batch_pods(st);
  const int32_t j0 = blockIdx.y * mp;
  if (j0 >= nb) return;                              // block-uniform
  const int lane = threadIdx.x & 63;
  const int32_t w = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= n_words) return;                          // wave-uniform
  const int32_t node = w * 64 + lane;
  const bool on = node < c.n;
  const int32_t x = on ? node : 0;
  const int32_t j1 = min(j0 + mp, nb);
  // The group's request fields, one pod per lane (mp <= 64), staged in the
  // wave's own LDS rows and read back per pod at a uniform address (as in
  // k_adapt_mask_commit).  Trivial pods only (every static filter host-proven
  // to pass; batchable pods request no scalar resources).
  __shared__ int64_t s_pq[4][64][4];
  __shared__ uint64_t s_mk[4][64];
  __shared__ int32_t s_cls[4][64];                 // static class, -2 trivial (static filters pass)
  const int wv = threadIdx.x >> 6;
  bool nontriv = false, generic = false;
  if (lane < j1 - j0) {
    const ksim_pod& q = P.pods[base + j0 + lane];
    // fits_request: a pod requesting nothing (and no scalar resources) needs
    // only a pod slot: its requests compare as INT64_MIN
    const bool none = q.req_cpu == 0 && q.req_mem == 0 && q.req_eph == 0 && !(q.flags & KSIM_POD_HAS_SCALAR);
    s_pq[wv][lane][0] = none ? INT64_MIN : q.req_cpu;
    s_pq[wv][lane][1] = none ? INT64_MIN : q.req_mem;
    s_pq[wv][lane][2] = none ? INT64_MIN : q.req_eph;
    nontriv = !(P.bflags[base + j0 + lane] & kBatchStaticTrivial);
    const int32_t cls = !nontriv ? -2 : P.stab ? P.sclass[base + j0 + lane] : -1;
    s_cls[wv][lane] = cls;
    generic = cls == -1 || (q.flags & KSIM_POD_HAS_SCALAR);
  }
  if (__ballot(nontriv) != 0 && __ballot(generic) == 0) {   // wave-uniform
    // static-class pods without scalar requests: each pod's verdict is its
    // class row's word at this node (batch_feasible), the Fit filter the
    // columns as below; eight pods' class words loaded before any is used
    const int32_t np = j1 - j0;
    const bool fit = bp.has_fit_filter != 0;
    const uint64_t room = fit ? __ballot(on && c.num_pods[x] + 1 <= c.alloc_pods[x]) : __ballot(on);
    const int64_t fc = c.alloc_cpu[x] - c.req_cpu[x];
    const int64_t fm = c.alloc_mem[x] - c.req_mem[x];
    const int64_t fe = c.alloc_eph[x] - c.req_eph[x];
#pragma unroll 1
    for (int32_t l0 = 0; l0 < np; l0 += 8) {
      int32_t cl[8];
      uint64_t sw[8];
#pragma unroll
      for (int t = 0; t < 8; t++) {
        cl[t] = l0 + t < np ? s_cls[wv][l0 + t] : -2;
        sw[t] = P.stab[(size_t)(cl[t] >= 0 ? cl[t] : 0) * c.n + x];
      }
#pragma unroll
      for (int t = 0; t < 8; t++) {
        const int32_t l = l0 + t;
        if (l >= np) break;                          // uniform
        const bool pass = cl[t] < 0 || stab_pass(sw[t]);
        const bool fits = !fit || ((s_pq[wv][l][0] <= fc) & (s_pq[wv][l][1] <= fm) & (s_pq[wv][l][2] <= fe));
        const uint64_t mk = room & __ballot(pass && fits);
        if (lane == 0) s_mk[wv][l] = mk;
      }
    }
    if (lane < np) amask[(size_t)(j0 + lane) * n_words + w] = s_mk[wv][lane];
    return;
  }
  if (__ballot(nontriv) == 0) {                    // wave-uniform
    // only the Fit filter's columns (the table is re-read once per pod group)
    uint64_t word;                                 // lane l: pod j0 + l's ballot
    if (bp.has_fit_filter == 0) {
      const uint64_t mk = __ballot(on);
      word = lane < j1 - j0 ? mk : 0ull;
    } else {
      const uint64_t room = __ballot(on && c.num_pods[x] + 1 <= c.alloc_pods[x]);
      const int64_t fc = c.alloc_cpu[x] - c.req_cpu[x];
      const int64_t fm = c.alloc_mem[x] - c.req_mem[x];
      const int64_t fe = c.alloc_eph[x] - c.req_eph[x];
      for (int32_t l = 0; l < j1 - j0; l++) {
        const int64_t c0 = s_pq[wv][l][0], m0 = s_pq[wv][l][1], e0 = s_pq[wv][l][2];
        const uint64_t mk = room & __ballot(c0 <= fc) & __ballot(m0 <= fm) & __ballot(e0 <= fe);
        if (lane == 0) s_mk[wv][l] = mk;
      }
      word = lane < j1 - j0 ? s_mk[wv][lane] : 0ull;
    }
    if (lane < j1 - j0) amask[(size_t)(j0 + lane) * n_words + w] = word;   // one store instruction per wave
    return;
  }
  const NodeRow r = load_row(c, x);
#pragma unroll 1
  for (int32_t j = j0; j < j1; j += 2) {           // two pods per step: both records' loads in flight
    const int32_t jb = j + 1 < j1 ? j + 1 : j;
    const bool ta = (P.bflags[base + j] & kBatchStaticTrivial) != 0;   // uniform
    const bool tb = (P.bflags[base + jb] & kBatchStaticTrivial) != 0;
    const bool fa = on && batch_feasible(c, P, bp, P.pods[base + j], r, ta, base + j);
    const bool fb = on && batch_feasible(c, P, bp, P.pods[base + jb], r, tb, base + jb);
    const uint64_t ma = __ballot(fa), mb = __ballot(fb);
    if (lane == 0) {
      amask[(size_t)j * n_words + w] = ma;
      if (jb != j) amask[(size_t)jb * n_words + w] = mb;
    }
  }
}

// Rotated offset of the K-th (0-based) set bit of `mask` counting from node s,
// or -1 when the bitmap holds at most K set bits.
// Eight word segments per step: their loads do not depend on the counts, so
// they go out together (one memory round trip per 512 nodes scanned instead of
// one per 64).
__device__ int32_t find_cut(const uint64_t* __restrict__ mask, int32_t s, int32_t n, int32_t k) {
  constexpr int kAhead = 8;                          // bitmap words per step (their loads are independent)
  int32_t need = k, off = 0, pos = s;
  while (off < n) {
    uint64_t bits[kAhead];
    int32_t len[kAhead];
    int32_t p = pos, o = off;
#pragma unroll
    for (int t = 0; t < kAhead; t++) {
      const int32_t w = p >> 6, b = p & 63;
      int32_t l = min((w + 1) * 64, n) - p;
      if (l > n - o) l = n - o;                     // back at s's word after the wrap (0: past the end)
      uint64_t x = mask[w] >> b;                     // p < n: w is in range
      if (l < 64) x &= (1ull << l) - 1;
      bits[t] = x;
      len[t] = l;
      o += l;
      p += l;
      if (p >= n) p = 0;
    }
#pragma unroll
    for (int t = 0; t < kAhead; t++) {
      const int cnt = __popcll(bits[t]);
      if (need < cnt) {
        uint64_t x = bits[t];
        for (int q = 0; q < need; q++) x &= x - 1;
        return off + __builtin_ctzll(x);
      }
      need -= cnt;
      off += len[t];
    }
    pos = p;
  }
  return -1;
}

constexpr int kWindowRounds = 48;
__device__ __forceinline__ int select_bit(uint64_t v, int32_t need) {   // position of set bit #need (0-based)
  int pos = 0;
#pragma unroll
  for (int wd = 32; wd >= 1; wd >>= 1) {
    const int32_t c = __popcll(v & ((1ull << wd) - 1));
    if (need >= c) {
      need -= c;
      v >>= wd;
      pos += wd;
    }
  }
  return pos;
}

constexpr int32_t kTopWideK = 4096;  // k_adapt_top with 1024 threads per pod from this window length

// The windows of one batch in one block of kBatchPods threads (thread j = pod
// j): *s_out = pod j's scan start, *cut_out = its cut offset (-1: no cut),
// *exact_out = pods with exact windows.  false: the batch is empty
// (block-uniform).  A pure function of the bitmaps and the state.
// NT threads (>= kBatchPods): thread j < nb is pod j, the others only join the barriers
template <int NT = kBatchPods>
__device__ __forceinline__ bool window_block(const DevState* __restrict__ st, const uint64_t* __restrict__ amask,
                                             int32_t n_words, int32_t n, int32_t k, int32_t* s_out,
                                             int32_t* cut_out, int32_t* exact_out,
                                             const int32_t* __restrict__ cut0 = nullptr,
                                             int32_t stop_after = kBatchPods) {
  static_assert(NT >= kBatchPods && NT % 64 == 0, "a thread per pod");
  __shared__ int64_t sh[NT / 64];
  __shared__ int32_t s_first;
  const int j = threadIdx.x, lane = j & 63, wv = j >> 6;
  const int32_t nb = batch_pods(st);
  if (nb <= 0) return false;
  const int32_t s0 = st->next_start;
  int32_t s = (int32_t)(((int64_t)s0 + (int64_t)j * k) % n);
  int32_t cut = -1, exact = 0;
  for (int round = 0; round < kWindowRounds; round++) {
    // cut0: the first round's cuts, from k_adapt_cut0 (a wave per pod)
    cut = j < nb ? (round == 0 && cut0 ? cut0[2 * j + 1] : find_cut(amask + (size_t)j * n_words, s, n, k)) : -1;
    const int64_t proc = j < nb ? (cut >= 0 ? cut : n) : 0;
    // exclusive prefix sum of the processed counts
    int64_t x = proc;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int64_t y = __shfl_up(x, d, 64);
      if (lane >= d) x += y;
    }
    if (lane == 63) sh[wv] = x;
    if (j == 0) s_first = kBatchPods;
    lds_barrier();
    int64_t before = 0;
    for (int w = 0; w < wv; w++) before += sh[w];
    const int32_t ns = (int32_t)(((int64_t)s0 + before + x - proc) % n);
    {                                                // the wave's first changed pod: one LDS atomic per wave
      const uint64_t chg = __ballot(j < nb && ns != s);
      if (chg && lane == 0) atomicMin(&s_first, (j & ~63) + __builtin_ctzll(chg));
    }
    lds_barrier();
    const int32_t f = s_first;
    lds_barrier();                                 // sh / s_first are rewritten next round
    if (f == kBatchPods) {                           // fixpoint: every window exact
      exact = nb;
      break;
    }
    exact = f;                                       // pods < f: start and cut exact
    if (j >= f) s = ns;                              // pods <= f now hold exact starts
    if (f > stop_after) break;                       // the caller's pod is exact: enough
  }
  *s_out = s;
  *cut_out = cut;
  *exact_out = exact;
  return true;
}

// The relaxation's first round over the whole chip: pod j's cut from its
// first guess s_j = s_0 + j K (mod N), one wave per pod, 128 bitmap words per
// step (each lane two, popcounts, a wave scan, the bit by halving), into
// acut[2j + 1].  window_block's walk is one thread per pod from one block,
// ~80 dependent words per pod at K = 5,000 (13.8 us per batch, config 4,
// where the first round is the fixpoint in every batch: profiles/r04/windbg);
// this launch takes the walk off the single block.
__global__ __launch_bounds__(256) void k_adapt_cut0(const DevState* __restrict__ st,
                                                    const uint64_t* __restrict__ amask, int32_t n_words, int32_t n,
                                                    int32_t k, int32_t* __restrict__ awin) {
  const int lane = threadIdx.x & 63;
  const int32_t j = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= batch_pods(st)) return;   // wave-uniform
  const int32_t s = (int32_t)(((int64_t)st->next_start + (int64_t)j * k) % n);
  const uint64_t* m = amask + (size_t)j * n_words;
  const int32_t ws = s >> 6;
  const uint64_t below = (1ull << (s & 63)) - 1;
  int32_t need = k, cut = -1;
  // virtual word v = 0 .. n_words: word (ws + v) mod n_words; v = 0 keeps the
  // bits from s on, v = n_words (ws again) the bits below s
  for (int32_t v0 = 0; v0 <= n_words; v0 += 128) {
    uint64_t b[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int32_t v = v0 + 2 * lane + h;
      int32_t w = ws + v;
      if (w >= n_words) w -= n_words;
      b[h] = v <= n_words ? m[w] : 0ull;
      if (v == 0) b[h] &= ~below;
      if (v == n_words) b[h] &= below;
    }
    const int32_t c0 = __popcll(b[0]), c = c0 + __popcll(b[1]);
    int32_t x = c;                                   // inclusive scan over the lanes
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int32_t y = __shfl_up(x, d, 64);
      if (lane >= d) x += y;
    }
    const uint64_t hit = __ballot(x > need);
    if (hit) {
      const int L = __builtin_ctzll(hit);
      if (lane == L) {
        int32_t r = need - (x - c);                  // set bit #r of the lane's two words
        const int h = r < c0 ? 0 : 1;
        if (h) r -= c0;
        const int32_t v = v0 + 2 * lane + h;
        int32_t w = ws + v;
        if (w >= n_words) w -= n_words;
        const int32_t node = w * 64 + select_bit(b[h], r);
        cut = node >= s ? node - s : node + n - s;
      }
      cut = __shfl(cut, L, 64);
      break;
    }
    need -= __shfl(x, 63, 64);
  }
  if (lane == 0) {
    awin[2 * j] = s;
    awin[2 * j + 1] = cut;
  }
}

// awin[2j] = scan start of pod j, awin[2j+1] = cut offset (-1: no cut, every
// feasible node kept and all N processed); *aexact = pods with exact windows.
// The first round's cuts are in acut (k_adapt_cut0).
__global__ __launch_bounds__(kBatchPods) void k_adapt_window(const DevState* __restrict__ st,
                                                             const uint64_t* __restrict__ amask, int32_t n_words,
                                                             int32_t n, int32_t k, const int32_t* __restrict__ acut,
                                                             int32_t* __restrict__ awin,
                                                             int32_t* __restrict__ aexact) {
  int32_t s, cut, exact;
  if (!window_block(st, amask, n_words, n, k, &s, &cut, &exact, acut)) return;
  const int j = threadIdx.x;
  if (j < batch_pods(st)) {
    awin[2 * j] = s;
    awin[2 * j + 1] = cut;
  }
  if (j == 0) *aexact = exact;
}

// Clusters of at most kWinSeqWords bitmap words take the exact windows of
// generic runs by doubling (below): a heterogeneous queue's feasible sets are
// sparse and uneven, so one pod's start error moves every later pod's and the
// relaxation converges slowly.  Pod j's scan stops at its (K+1)-th feasible
// node and pod j+1's scan starts there: s_{j+1} = F_j(s_j).  (Round 4 first
// walked this recurrence on one wave, 0.27 us per pod; profiles/r04/next1.)
constexpr int32_t kWinSeqWords = 128;

// The same windows by pointer doubling (clusters of at most kWinSeqWords
// bitmap words; the walk's function made parallel).  Pod j's step is a map
// F_j: start -> next start over the n starts (the (K+1)-th feasible node
// from the start, the start itself when at most K are feasible).  k_win_build
// tabulates every F_j (one block per pod: its ranks and the positions of its
// feasible nodes in LDS).  Two radix-8 rounds compose the prefixes
// (Q_j = F_j o ... o F_max(0, j-7), then strides of 8), each block staging
// the 8 source rows its pod reads in LDS; k_win_final composes the 64-pod
// prefixes at s_0 alone (stride 64), so pod j starts at
// (F_{j-1} o ... o F_0)(s_0).  Four launches of table lookups in place of the
// walk's 256 dependent steps on one wave (profiles/r04/winb: 21.0 us per
// batch; radix 16 over global gathers 30.1 us, radix 4 31.4 us, radix 8
// 30.3 us in profiles/r04/radix).
constexpr int kWinBuildThreads = 1024;
__global__ __launch_bounds__(kWinBuildThreads) void k_win_build(const DevState* __restrict__ st,
                                                   const uint64_t* __restrict__ amask, int32_t n_words, int32_t n,
                                                   int32_t k, uint16_t* __restrict__ tab0, int32_t* __restrict__ wtot) {
  __shared__ uint64_t s_w[kWinSeqWords];
  __shared__ int32_t s_pc[kWinSeqWords];
  __shared__ int32_t s_tot0;
  __shared__ uint16_t s_sel[kWinSeqWords * 64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int32_t j = blockIdx.x;
  if (j >= batch_pods(st)) return;   // block-uniform
  const uint64_t* m = amask + (size_t)j * n_words;
  if (tid < kWinSeqWords) {                        // the words' prefix counts, two waves
    const uint64_t w = tid < n_words ? m[tid] : 0ull;
    s_w[tid] = w;
    const int32_t c = (int32_t)__popcll(w);
    int32_t x = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int32_t y = __shfl_up(x, d, 64);
      if (lane >= d) x += y;
    }
    s_pc[tid] = x - c;
    if (tid == 63) s_tot0 = x;
  }
  lds_barrier();
  if (tid >= 64 && tid < kWinSeqWords) s_pc[tid] += s_tot0;
  lds_barrier();
  const int32_t total = s_pc[n_words - 1] + (int32_t)__popcll(s_w[n_words - 1]);
  for (int32_t x = tid; x < n; x += kWinBuildThreads) {         // the positions of the feasible nodes by rank
    const uint64_t w = s_w[x >> 6];
    const int b = x & 63;
    if ((w >> b) & 1ull) s_sel[s_pc[x >> 6] + (int32_t)__popcll(w & ((1ull << b) - 1ull))] = (uint16_t)x;
  }
  lds_barrier();
  uint16_t* out = tab0 + (size_t)j * n;
  for (int32_t x = tid; x < n; x += kWinBuildThreads) {
    const uint64_t w = s_w[x >> 6];
    int32_t t = s_pc[x >> 6] + (int32_t)__popcll(w & ((1ull << (x & 63)) - 1ull)) + k;   // the cut's rank
    if (t >= total) t -= total;
    out[x] = total > k ? s_sel[t] : (uint16_t)x;
  }
  if (tid == 0) wtot[j] = total;
}

// Round with stride d: Q'_j = Q_j o Q_{j-d} o Q_{j-2d} o Q_{j-3d} (terms with
// a negative index left out).
// D: the span of the prefixes in q (the last round, stride D, at s_0 alone).
template <int D>
__global__ __launch_bounds__(kBatchPods) void k_win_final(const DevState* __restrict__ st,
                                                          const uint16_t* __restrict__ tab0,
                                                          const uint16_t* __restrict__ q,
                                                          const int32_t* __restrict__ wtot, int32_t n, int32_t k,
                                                          int32_t* __restrict__ awin, int32_t* __restrict__ aexact) {
  const int32_t j = threadIdx.x;
  const int32_t nb = batch_pods(st);
  if (nb <= 0) return;
  if (j < nb) {
    const int32_t s0 = st->next_start, i = j - 1;
    int32_t s = s0;
#pragma unroll
    for (int t = kBatchPods / D - 1; t >= 0; t--)
      if (i - t * D >= 0) s = q[(size_t)(i - t * D) * n + s];
    const int32_t nx = tab0[(size_t)j * n + s];
    awin[2 * j] = s;
    awin[2 * j + 1] = wtot[j] <= k ? -1 : (nx > s ? nx - s : nx + n - s);
  }
  if (j == 0) *aexact = nb;
}

// A radix-R round with the R source rows a pod reads staged in LDS (one block
// per pod, rows of at most kWinSeqWords * 64 entries): R - 1 dependent LDS
// lookups per start instead of global gathers.
template <int R>
__global__ __launch_bounds__(1024) void k_win_round_lds(const DevState* __restrict__ st, int32_t n, int32_t d,
                                                        const uint16_t* __restrict__ src, uint16_t* __restrict__ dst) {
  __shared__ uint16_t s_rows[R][kWinSeqWords * 64];
  const int32_t j = blockIdx.x;
  if (j >= batch_pods(st)) return;   // block-uniform
  const int32_t words = (n + 7) >> 3;                  // 16-byte pieces per row (the row starts 16-byte aligned)
#pragma unroll
  for (int t = 0; t < R; t++) {
    const int32_t row = j - t * d;
    if (row < 0) continue;                              // block-uniform
    const uint16_t* in = src + (size_t)row * n;
    if ((n & 7) == 0) {
      for (int32_t x = threadIdx.x; x < words; x += 1024)
        reinterpret_cast<uint4*>(s_rows[t])[x] = reinterpret_cast<const uint4*>(in)[x];
    } else {
      for (int32_t x = threadIdx.x; x < n; x += 1024) s_rows[t][x] = in[x];
    }
  }
  __syncthreads();
  uint16_t* out = dst + (size_t)j * n;
  for (int32_t x = threadIdx.x; x < n; x += 1024) {
    int32_t v = x;
#pragma unroll
    for (int t = R - 1; t >= 1; t--)
      if (j - t * d >= 0) v = s_rows[t][v];
    out[x] = s_rows[0][v];
  }
}

static void launch_window_dbl(const LaunchArgs& a, int32_t n_words, int32_t k, hipStream_t stream) {
  const int32_t n = a.c.n;
  uint16_t* t0 = a.s.wtab;
  uint16_t* t1 = t0 + (size_t)kBatchPods * n;
  k_win_build<<<kBatchPods, kWinBuildThreads, 0, stream>>>(a.st, a.s.amask, n_words, n, k, t0, a.s.wtot);
  static_assert(kBatchPods == 256, "two radix-8 rounds and the stride-64 final cover 256 pods");
  uint16_t* t2 = t1 + (size_t)kBatchPods * n;
  k_win_round_lds<8><<<kBatchPods, 1024, 0, stream>>>(a.st, n, 1, t0, t1);
  k_win_round_lds<8><<<kBatchPods, 1024, 0, stream>>>(a.st, n, 8, t1, t2);
  k_win_final<64><<<1, kBatchPods, 0, stream>>>(a.st, t0, t2, a.s.wtot, n, k, a.s.awin, a.s.aexact);
}

// Clusters up to this many bitmap words run the window scan inside k_adapt_top
// (every block scans all B bitmaps: B x W words from L2 per block).
constexpr int32_t kWinFusedWords = 256;

// k_adapt_top's kept-node list (static-class FAST keys): windows with at most
// this many kept nodes are compacted into LDS before they are keyed.
constexpr int kAdaptList = 4096;
// The bits of nodes [a, b) within bitmap word w.
__device__ __forceinline__ uint64_t word_range(int32_t w, int32_t a, int32_t b) {
  const int32_t lo = max(a - w * 64, 0), hi = min(b - w * 64, 64);
  if (hi <= lo) return 0ull;
  const uint64_t up = hi >= 64 ? ~0ull : (1ull << hi) - 1ull;
  return up & ~((1ull << lo) - 1ull);
}

// One block (4 waves) per pod: the kept nodes' TB keys -> the pod's top-T
// (complete when it lists every kept node).  Each wave keeps its lanes' best T
// keys and extracts its own top-T; wave 0 merges the four lists.  Pods past
// the exact windows get an empty incomplete list, which ends the chain there.
// SH (node-sharded): amask / awin are global (n_total nodes); the block scores
// the kept nodes this shard holds and writes the pod's record (xsend: its T
// best keys and count | complete << 32) for the all-gather instead of topk.
// FAST: the narrow-arithmetic keys (dyn_key_fast; trivial cpu/memory pods, see
// ksim_batch.hip).
// NT threads per block: 256, or 1024 for long windows (K >= kTopWideK), so
// the block's waves fill their SIMDs (every CU holds one pod's block).
// WIN (NT = kBatchPods, unsharded): every block runs the window scan itself
// (window_block, thread i = pod i) instead of reading k_adapt_window's
// output; block 0 stores awin / aexact for the pairs and the commit.
// DEF (FAST only): the default profile's key shape compiled in (fast_def)
template <bool SH, bool FAST, int NT, int WIN = 0, bool DEF = false>
__global__ __launch_bounds__(NT) void k_adapt_top(DevCluster c, DevPods P, const ksim_profile* __restrict__ prof_p,
                                                   const BatchProg* __restrict__ bp_p,
                                                   const DevState* __restrict__ st,
                                                   const uint64_t* __restrict__ amask, int32_t n_words,
                                                   int32_t* __restrict__ awin,
                                                   int32_t* __restrict__ aexact, uint64_t* __restrict__ topk,
                                                   int32_t* __restrict__ topk_cnt,
                                                   int32_t* __restrict__ topk_complete,
                                                   uint64_t* __restrict__ xsend,
                                                   int64_t* __restrict__ pnorm = nullptr,
                                                   const int32_t* __restrict__ acut = nullptr) {
  const ksim_profile& prof = *prof_p;
  const BatchProg& bp = *bp_p;
  constexpr int W = NT / 64;
  constexpr int kSlots = (W * kTopT + 63) / 64;     // merge entries per lane
  __shared__ uint64_t s_top[W][kTopT];
  __shared__ int32_t s_kept[W];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int32_t j = blockIdx.x;
  const int32_t base = st->cursor;
  if (j >= batch_pods(st)) return;   // block-uniform
  int32_t win_s = 0, win_cut = -1, exact;
  if constexpr (WIN != 0) {
    // WIN 1: the whole relaxation in every block; WIN 2: from k_adapt_cut0's
    // first round (acut), so a batch at its fixpoint costs every block one
    // prefix sum over the batch's cuts
    static_assert(!SH && (WIN == 2 || NT == kBatchPods), "fused window: unsharded, one thread per pod");
    __shared__ int2 s_win;
    int32_t ws, wc;
    const int32_t kk = num_feasible_nodes_to_find(prof.percentage_of_nodes_to_score, c.n);
    // block 0 stores every window and the exact prefix: the whole relaxation;
    // block j stops once pod j's window is exact (rounds past the first,
    // a batch off its first-round fixpoint costs the later blocks
    // only the rounds their own pod needs)
    window_block<NT>(st, amask, n_words, c.n, kk, &ws, &wc, &exact, WIN == 2 ? acut : nullptr,
                     j == 0 ? kBatchPods : j);   // batch not empty (above)
    if (tid == j) s_win = make_int2(ws, wc);
    if (j == 0) {
      if (tid < batch_pods(st)) {
        awin[2 * tid] = ws;
        awin[2 * tid + 1] = wc;
      }
      if (tid == 0) *aexact = exact;
    }
    __syncthreads();
    win_s = s_win.x;
    win_cut = s_win.y;
  } else {
    exact = *aexact;
  }
  if (j >= exact) {
    if (SH) {
      if (tid <= kTopT) xsend[(size_t)j * kXRec + tid] = 0;   // empty, incomplete
    } else if (tid == 0) {
      topk_cnt[j] = 0;
      topk_complete[j] = 0;
    }
    return;
  }
  const int32_t n = SH ? c.n_total : c.n, s = WIN ? win_s : awin[2 * j], cut = WIN ? win_cut : awin[2 * j + 1];
  const int32_t kend = cut >= 0 ? cut : n;
  const int32_t pi = base + j;
  const ksim_pod& p = P.pods[pi];
  const int64_t seq = st->pod_seq + j;
  const uint64_t hseed = prof.tiebreak_seed ^ ((uint64_t)seq << 20);
  auto node_key = [&](int32_t local) -> uint64_t {
    const NodeRow r = load_res_row(c, local);       // scores read the resource columns only
    if constexpr (FAST)
      return dyn_key_fast_t<DEF>(fast_prog(bp), p, r, c.inv_cpu[local], c.inv_mem[local], hseed, c.base + local);
    return dyn_key(prof, bp, p, r, c.n_scalar, seq, c.base, c.fit_ignore);
  };
  const uint64_t* mask = amask + (size_t)j * n_words;
  uint64_t a[kTopT];
#pragma unroll
  for (int t = 0; t < kTopT; t++) a[t] = 0;
  int32_t kept = 0;
  if (SH) {
    // the window [s, s + kend) (circular, global) as two linear pieces, each
    // clipped to this shard's [base, base + c.n)
    const int32_t lo = c.base, hi = c.base + c.n;
    const int32_t e1 = s + kend <= n ? s + kend : n, e2 = s + kend <= n ? 0 : s + kend - n;
    const int32_t a0 = max(s, lo), a1 = min(e1, hi), b0 = max(0, lo), b1 = min(e2, hi);
    const int32_t len1 = a1 > a0 ? a1 - a0 : 0, len2 = b1 > b0 ? b1 - b0 : 0;
#pragma unroll 1
    for (int32_t i = tid; i < len1 + len2; i += NT) {
      const int32_t g = i < len1 ? a0 + i : b0 + (i - len1);
      if (!((mask[g >> 6] >> (g & 63)) & 1ull)) continue;
      kept++;
      a[kTopT - 1] = umax64(a[kTopT - 1], node_key(g - c.base));
#pragma unroll
      for (int t = kTopT - 1; t > 0; t--) cswap_desc(a[t - 1], a[t]);
    }
  } else if constexpr (FAST) {
    // two nodes per step, every load of both (bitmap words, rows) issued first
#pragma unroll 1
    for (int32_t off = tid; off < kend; off += 2 * NT) {
      int32_t n1 = s + off, n2 = s + off + NT;
      if (n1 >= n) n1 -= n;
      if (n2 >= n) n2 -= n;
      const bool v2 = off + NT < kend;
      if (!v2) n2 = n1;
      const uint64_t w1 = mask[n1 >> 6], w2 = mask[n2 >> 6];
      const NodeRow r1 = load_res_row_off(c, n1), r2 = load_res_row_off(c, n2);
      const double c1 = ld_off(c.inv_cpu, (uint32_t)n1 << 3), m1 = ld_off(c.inv_mem, (uint32_t)n1 << 3);
      const double c2 = ld_off(c.inv_cpu, (uint32_t)n2 << 3), m2 = ld_off(c.inv_mem, (uint32_t)n2 << 3);
      __builtin_amdgcn_sched_barrier(0);
      if ((w1 >> (n1 & 63)) & 1ull) {
        kept++;
        a[kTopT - 1] = umax64(a[kTopT - 1], dyn_key_fast_t<DEF>(fast_prog(bp), p, r1, c1, m1, hseed, c.base + n1));
#pragma unroll
        for (int t = kTopT - 1; t > 0; t--) cswap_desc(a[t - 1], a[t]);
      }
      if (v2 && ((w2 >> (n2 & 63)) & 1ull)) {
        kept++;
        a[kTopT - 1] = umax64(a[kTopT - 1], dyn_key_fast_t<DEF>(fast_prog(bp), p, r2, c2, m2, hseed, c.base + n2));
#pragma unroll
        for (int t = kTopT - 1; t > 0; t--) cswap_desc(a[t - 1], a[t]);
      }
    }
  } else {
    // kPodNormVaries (unsharded, pnorm given): DefaultNormalizeScore's maxima
    // over the pod's scored list -- the kept nodes of its window -- then keys
    // that carry the normalized part (norm_part).  The list stays the S0 list
    // while the window is not broken (k_adapt_pairs flags every kept node
    // that stops fitting for these pods), so the maxima hold for the batch.
    const bool normv = pnorm && (P.bflags[pi] & kPodNormVaries) != 0;   // block-uniform
    // a static class (DevPods::stab): the raw scores from the class row, and on
    // a run_fast cluster the FAST key arithmetic (block-uniform)
    const int32_t scls = P.stab ? P.sclass[pi] : -1;
    const uint64_t* srow = scls >= 0 ? P.stab + (size_t)scls * c.n : nullptr;
    const bool fk = srow && P.stab_fast;
    auto raw = [&](int32_t node) -> NormRaw {
      return srow ? stab_raw(srow[node], P, p) : norm_raw(c, P, p, load_row(c, node));
    };
    auto gkey = [&](int32_t node) -> uint64_t {
      if (fk) {
        const NodeRow r = load_res_row_off(c, node);
        const uint32_t o8 = (uint32_t)node << 3;
        return dyn_key_fast(bp, fast_pod_fields(p), r, ld_off(c.inv_cpu, o8), ld_off(c.inv_mem, o8), hseed,
                            c.base + node);
      }
      return node_key(node);
    };
    NormRaw mx{0, 0};
    if (fk) {
      // the FAST keys of a static class: two nodes per step with every load
      // of both (bitmap words, class words, rows) issued before the bit tests,
      // as the FAST loop above; the same nodes, maxima and keys as the loops below
      const ksim_pod pf = fast_pod_fields(p);
      const FastProg q = fast_prog(bp);
      // the window's kept nodes first compacted into LDS (one bitmap word per
      // thread, range-masked to the window's offsets [0, kend) from s), so a
      // thread keys at most ceil(kept / NT) nodes, each with all of its loads
      // in one round trip, instead of stepping over the window's whole span
      // (windows of at most 2 NT nodes take the stepping loop: one round trip
      // there, two here)
      __shared__ int32_t s_list[kAdaptList];
      __shared__ int32_t s_nl;
      int32_t nl = kAdaptList + 1;
      if (kend > 2 * NT) {                          // block-uniform
        if (tid == 0) s_nl = 0;
        lds_barrier();
        // the window's words only: piece 1 [s, b1), piece 2 [0, b2) after the wrap
        const bool wrap = s + kend > n;
        const int32_t b1 = wrap ? n : s + kend, b2 = wrap ? s + kend - n : 0;
        const int32_t c1 = ((b1 - 1) >> 6) - (s >> 6) + 1, c2 = b2 > 0 ? ((b2 - 1) >> 6) + 1 : 0;
        for (int32_t t = tid; t < c1 + c2; t += NT) {
          const int32_t w = t < c1 ? (s >> 6) + t : t - c1;
          uint64_t bits = mask[w] & (t < c1 ? word_range(w, s, b1) : word_range(w, 0, b2));
          const int32_t cnt = __popcll(bits);
          int32_t pos = cnt ? atomicAdd(&s_nl, cnt) : 0;
          for (; bits; bits &= bits - 1, pos++)
            if (pos < kAdaptList) s_list[pos] = w * 64 + __builtin_ctzll(bits);
        }
        lds_barrier();
        nl = s_nl;
      }
      if (nl <= NT) {                               // block-uniform: one kept node per thread at most
        const bool has = tid < nl;
        const int32_t nd = has ? s_list[tid] : 0;
        const uint64_t x = srow[nd];
        const NodeRow r = load_res_row_off(c, nd);
        const double ci = ld_off(c.inv_cpu, (uint32_t)nd << 3), mi = ld_off(c.inv_mem, (uint32_t)nd << 3);
        __builtin_amdgcn_sched_barrier(0);
        uint64_t k = has ? dyn_key_fast_t<false>(q, pf, r, ci, mi, hseed, c.base + nd) : 0;
        if (normv) {
          NormAcc acc;
          if (has) acc.take(stab_raw(x, P, p));
          mx = norm_maxima<NT>(acc, pnorm, j);
          if (k) k += (uint64_t)norm_part(bp, stab_raw(x, P, p), mx) << 44;
        }
        kept += has ? 1 : 0;
        a[kTopT - 1] = umax64(a[kTopT - 1], k);
#pragma unroll
        for (int t = kTopT - 1; t > 0; t--) cswap_desc(a[t - 1], a[t]);
      } else if (nl <= kAdaptList) {                // block-uniform
        if (normv) {
          NormAcc acc;
#pragma unroll 1
          for (int32_t i = tid; i < nl; i += NT) acc.take(stab_raw(srow[s_list[i]], P, p));
          mx = norm_maxima<NT>(acc, pnorm, j);
        }
#pragma unroll 1
        for (int32_t i = tid; i < nl; i += NT) {
          const int32_t nd = s_list[i];
          const uint64_t x = srow[nd];
          const NodeRow r = load_res_row_off(c, nd);
          const double ci = ld_off(c.inv_cpu, (uint32_t)nd << 3), mi = ld_off(c.inv_mem, (uint32_t)nd << 3);
          kept++;
          uint64_t k = dyn_key_fast_t<false>(q, pf, r, ci, mi, hseed, c.base + nd);
          if (normv && k) k += (uint64_t)norm_part(bp, stab_raw(x, P, p), mx) << 44;
          a[kTopT - 1] = umax64(a[kTopT - 1], k);
#pragma unroll
          for (int t = kTopT - 1; t > 0; t--) cswap_desc(a[t - 1], a[t]);
        }
      } else {
      if (normv) {
        NormAcc acc;
#pragma unroll 1
        for (int32_t off = tid; off < kend; off += 2 * NT) {
          int32_t n1 = s + off, n2 = s + off + NT;
          if (n1 >= n) n1 -= n;
          if (n2 >= n) n2 -= n;
          const bool v2 = off + NT < kend;
          if (!v2) n2 = n1;
          const uint64_t w1 = mask[n1 >> 6], w2 = mask[n2 >> 6], x1 = srow[n1], x2 = srow[n2];
          __builtin_amdgcn_sched_barrier(0);
          if ((w1 >> (n1 & 63)) & 1ull) acc.take(stab_raw(x1, P, p));
          if (v2 && ((w2 >> (n2 & 63)) & 1ull)) acc.take(stab_raw(x2, P, p));
        }
        mx = norm_maxima<NT>(acc, pnorm, j);
      }
#pragma unroll 1
      for (int32_t off = tid; off < kend; off += 2 * NT) {
        int32_t n1 = s + off, n2 = s + off + NT;
        if (n1 >= n) n1 -= n;
        if (n2 >= n) n2 -= n;
        const bool v2 = off + NT < kend;
        if (!v2) n2 = n1;
        const uint64_t w1 = mask[n1 >> 6], w2 = mask[n2 >> 6], x1 = srow[n1], x2 = srow[n2];
        const NodeRow r1 = load_res_row_off(c, n1), r2 = load_res_row_off(c, n2);
        const double c1 = ld_off(c.inv_cpu, (uint32_t)n1 << 3), m1 = ld_off(c.inv_mem, (uint32_t)n1 << 3);
        const double c2 = ld_off(c.inv_cpu, (uint32_t)n2 << 3), m2 = ld_off(c.inv_mem, (uint32_t)n2 << 3);
        __builtin_amdgcn_sched_barrier(0);
        if ((w1 >> (n1 & 63)) & 1ull) {
          kept++;
          uint64_t k = dyn_key_fast_t<false>(q, pf, r1, c1, m1, hseed, c.base + n1);
          if (normv && k) k += (uint64_t)norm_part(bp, stab_raw(x1, P, p), mx) << 44;
          a[kTopT - 1] = umax64(a[kTopT - 1], k);
#pragma unroll
          for (int t = kTopT - 1; t > 0; t--) cswap_desc(a[t - 1], a[t]);
        }
        if (v2 && ((w2 >> (n2 & 63)) & 1ull)) {
          kept++;
          uint64_t k = dyn_key_fast_t<false>(q, pf, r2, c2, m2, hseed, c.base + n2);
          if (normv && k) k += (uint64_t)norm_part(bp, stab_raw(x2, P, p), mx) << 44;
          a[kTopT - 1] = umax64(a[kTopT - 1], k);
#pragma unroll
          for (int t = kTopT - 1; t > 0; t--) cswap_desc(a[t - 1], a[t]);
        }
      }
      }
    } else {
    if (normv) {
      // the maxima over the kept nodes and how many kept nodes hold each
      // (pnorm[4 j + 2..3]): a window that scans every node never shifts, so
      // its pod stays exact until every holder of a maximum stops fitting
      // (k_adapt_pairs), as on the P100 path
      NormAcc acc;
#pragma unroll 1
      for (int32_t off = tid; off < kend; off += NT) {
        int32_t node = s + off;
        if (node >= n) node -= n;
        if (!((mask[node >> 6] >> (node & 63)) & 1ull)) continue;
        acc.take(raw(node));
      }
      mx = norm_maxima<NT>(acc, pnorm, j);
    }
#pragma unroll 1
    for (int32_t off = tid; off < kend; off += NT) {
      int32_t node = s + off;
      if (node >= n) node -= n;
      if (!((mask[node >> 6] >> (node & 63)) & 1ull)) continue;
      kept++;
      uint64_t k = gkey(node);
      if (normv && k) k += (uint64_t)norm_part(bp, raw(node), mx) << 44;
      a[kTopT - 1] = umax64(a[kTopT - 1], k);
#pragma unroll
      for (int t = kTopT - 1; t > 0; t--) cswap_desc(a[t - 1], a[t]);
    }
    }
  }
  // per wave: a lane can be popped at most T times and holds its T best, so
  // the wave's top-T is exact
  for (int t = 0; t < kTopT; t++) {
    const uint64_t m = wave_max_u64_hi(a[0]);
    if (lane == 0) s_top[wv][t] = m;
    if (m != 0 && a[0] == m) {
#pragma unroll
      for (int q = 0; q < kTopT - 1; q++) a[q] = a[q + 1];
      a[kTopT - 1] = 0;
    }
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) kept += __shfl_xor(kept, d, 64);
  if (lane == 0) s_kept[wv] = kept;
  lds_barrier();
  if (wv != 0) return;
  // merge: entry x = w * T + e (keys are unique per node) sits in lane x % 64, slot x / 64
  uint64_t key[kSlots];
#pragma unroll
  for (int q = 0; q < kSlots; q++) {
    const int x = q * 64 + lane;
    key[q] = x < W * kTopT ? s_top[x / kTopT][x % kTopT] : 0;
  }
  uint64_t mine = 0;
  int32_t cnt = 0;
  for (int t = 0; t < kTopT; t++) {
    uint64_t best = key[0];
#pragma unroll
    for (int q = 1; q < kSlots; q++) best = umax64(best, key[q]);
    const uint64_t m = wave_max_u64_hi(best);
    if (m == 0) break;
    if (lane == t) mine = m;
    cnt = t + 1;
#pragma unroll
    for (int q = 0; q < kSlots; q++)
      if (key[q] == m) key[q] = 0;
  }
  int32_t total = 0;
#pragma unroll
  for (int w = 0; w < W; w++) total += s_kept[w];
  if (SH) {
    uint64_t* x = xsend + (size_t)j * kXRec;
    if (lane < kTopT) x[lane] = lane < cnt ? mine : 0;
    if (lane == 0) x[kTopT] = (uint64_t)(uint32_t)cnt | ((uint64_t)(total <= kTopT ? 1 : 0) << 32);
    return;
  }
  if (lane < kTopT) topk[(size_t)j * kTopT + lane] = lane < cnt ? mine : 0;
  if (lane == 0) {
    topk_cnt[j] = cnt;
    topk_complete[j] = total <= kTopT ? 1 : 0;
  }
}

// SH: windows and bitmaps are global; a shard scores only the guesses on its
// own nodes; pmax[kBatchPods + j] carries the broken flag (all-reduced with M).
// Every block runs the chain itself from the top-T lists (as
// k_batch_chain_pairs on the P100 path); block 0 stores gkey / chain_end for
// the commit.
template <bool SH, bool LAZY = false>
__global__ __launch_bounds__(kBatchPods) void k_adapt_pairs(DevCluster c, DevPods P,
                                                            const ksim_profile* __restrict__ prof_p,
                                                            const BatchProg* __restrict__ bp_p,
                                                            const DevState* __restrict__ st,
                                                            const uint64_t* __restrict__ amask, int32_t n_words,
                                                            const int32_t* __restrict__ awin,
                                                            const uint64_t* __restrict__ topk,
                                                            const int32_t* __restrict__ topk_cnt,
                                                            const int32_t* __restrict__ topk_complete,
                                                            uint64_t* __restrict__ gkey,
                                                            int32_t* __restrict__ chain_end,
                                                            uint64_t* __restrict__ pmax,
                                                            int32_t* __restrict__ abroken,
                                                            const int64_t* __restrict__ pnorm = nullptr) {
  const ksim_profile& prof = *prof_p;
  const BatchProg& bp = *bp_p;
  __shared__ uint64_t s_wmax[kBatchPods / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int32_t base = st->cursor;
  const int32_t nb = batch_pods(st);
  if (nb <= 0) {
    if (LAZY && blockIdx.x == 0 && tid == 0) *chain_end = -1;   // deferred commit: an empty slot
    return;
  }
  const int j = blockIdx.x, k = tid;
  int32_t nchain;
  uint64_t gk;
  {
    __shared__ ChainLds L;
    if (!chain_block(L, st, topk, topk_cnt, topk_complete, &gk, &nchain, nullptr, batch_cap(st), c.n_total)) return;
    if (j == 0) {
      if (k < nb) gkey[k] = gk;
      if (k == 0) *chain_end = nchain;
    }
  }
  uint64_t v = 0;
  bool brk = false;
  bool lost_t = false, lost_a = false;           // guess k held a normalization maximum of pod j and stopped fitting
  if (j < nchain && k < j) {
    const int32_t node = gk ? key_node(gk) - c.base : -1;
    if (node >= 0 && node < c.n) {
      const int32_t g = node + c.base;              // global position (== node unsharded)
      const int32_t n = SH ? c.n_total : c.n, s = awin[2 * j], cut = awin[2 * j + 1];
      int32_t off = g - s;
      if (off < 0) off += n;
      const int32_t kend = cut >= 0 ? cut : n;
      if (off < kend || off == cut) {
        NodeRow r = load_row(c, node);
        // a static class (block-uniform): the raw normalized scores from its
        // row, and on a run_fast cluster the FAST key (as k_adapt_top's list keys)
        const int32_t scls = P.stab ? P.sclass[base + j] : -1;
        const uint64_t sw = scls >= 0 ? P.stab[(size_t)scls * c.n + node] : 0;
        row_add_pod(r, P.pods[base + k], 1);
        const ksim_pod& p = P.pods[base + j];
        auto raw = [&]() -> NormRaw { return scls >= 0 ? stab_raw(sw, P, p) : norm_raw(c, P, p, r); };
        const bool now = batch_feasible(c, P, bp, p, r, (P.bflags[base + j] & kBatchStaticTrivial) != 0, base + j);
        const bool was = (amask[(size_t)j * n_words + (g >> 6)] >> (g & 63)) & 1ull;
        // a window that stops before the ring's end shifts when a kept node
        // stops fitting; one that scans every node keeps its span, and for
        // kPodNormVaries pods (k_adapt_top's maxima) its scored list loses
        // the node: the maxima change once every holder has left
        const bool normv = pnorm && (P.bflags[base + j] & kPodNormVaries) != 0;
        if (was && !now) {
          if (cut >= 0) {
            brk = true;
          } else if (normv) {
            const NormRaw x = raw();
            lost_t = pnorm[4 * j] > 0 && x.tt == pnorm[4 * j];
            lost_a = pnorm[4 * j + 1] > 0 && x.na == pnorm[4 * j + 1];
          }
        }
        if (off < kend && now) {
          if (scls >= 0 && P.stab_fast)
            v = dyn_key_fast(bp, fast_pod_fields(p), r, c.inv_cpu[node], c.inv_mem[node],
                             prof.tiebreak_seed ^ ((uint64_t)(st->pod_seq + j) << 20), c.base + node);
          else
            v = dyn_key(prof, bp, p, r, c.n_scalar, st->pod_seq + j, c.base, c.fit_ignore);
        }
        if (normv && v) v += (uint64_t)norm_part(bp, raw(), NormRaw{pnorm[4 * j], pnorm[4 * j + 1]}) << 44;
      }
    }
  }
  __shared__ int32_t s_lost[2];
  if (tid < 2) s_lost[tid] = 0;
  lds_barrier();
  {
    const int32_t nt = __popcll(__ballot(lost_t)), na = __popcll(__ballot(lost_a));
    if (lane == 0 && nt) atomicAdd(&s_lost[0], nt);
    if (lane == 0 && na) atomicAdd(&s_lost[1], na);
  }
  lds_barrier();
  if (s_lost[0] > 0 && s_lost[0] >= pnorm[4 * j + 2]) brk = true;   // every holder of a maximum left
  if (s_lost[1] > 0 && s_lost[1] >= pnorm[4 * j + 3]) brk = true;
  const bool any_brk = __syncthreads_or(brk);
  v = wave_max_u64_dpp(v);
  if (lane == 0) s_wmax[wave] = v;
  lds_barrier();
  if (tid == 0) {
    uint64_t m = 0;
    for (int w = 0; w < kBatchPods / 64; w++) m = umax64(m, s_wmax[w]);
    pmax[j] = j < nchain ? m : 0;
    if (SH) pmax[kBatchPods + j] = j < nchain && any_brk ? 1 : 0;
    else abroken[j] = j < nchain && any_brk ? 1 : 0;
  }
}

#ifdef KSIM_ADAPT_DBG
// KSIM_ADAPT_DBG builds (tools/adapt_dbg.py): why ADAPT batches end short.
// dbg 0 batches, 1 the chain ended before the batch (an exhausted incomplete
// list), 2 a broken window before the chain's end, 3 sum of the chain's
// length, 4 sum of the prefix before the first broken window, 5 cut by a pair
// maximum, 6 sum of committed pods, 7 sum of the batch's pods
__device__ unsigned long long g_adapt_dbg[8];
unsigned long long* adapt_dbg_buffer() {
  void* p = nullptr;
  (void)hipGetSymbolAddress(&p, HIP_SYMBOL(g_adapt_dbg));
  return (unsigned long long*)p;
}
#else
unsigned long long* adapt_dbg_buffer() { return nullptr; }
#endif

// abroken null (sharded): the broken flags follow M in pmax[kBatchPods + j].
__global__ __launch_bounds__(kBatchPods) void k_adapt_commit(DevCluster c, DevPods P, DevState* __restrict__ st,
                                                             const uint64_t* __restrict__ gkey,
                                                             const int32_t* __restrict__ chain_end,
                                                             const uint64_t* __restrict__ pmax,
                                                             const int32_t* __restrict__ abroken,
                                                             const int32_t* __restrict__ awin,
                                                             int32_t* __restrict__ chosen_out) {
  __shared__ int32_t s_fb, s_istar, s_sched, s_unsched;
  __shared__ int2 s_aw[kBatchPods];
  const uint64_t g = gkey[threadIdx.x], m = pmax[threadIdx.x];   // in flight with the state loads
  const int32_t brk = abroken ? abroken[threadIdx.x] : (int32_t)pmax[kBatchPods + threadIdx.x];
  const int2 aw = reinterpret_cast<const int2*>(awin)[threadIdx.x];   // {scan start, cut}, likewise
  if (batch_pods(st) <= 0) return;
  const int32_t nchain0 = *chain_end;
  s_aw[threadIdx.x] = aw;
  if (threadIdx.x == 0) s_fb = nchain0;
  lds_barrier();
  block_first_min(&s_fb, (int32_t)threadIdx.x < nchain0 && brk);
  lds_barrier();
#ifdef KSIM_ADAPT_DBG
  const int32_t nb_dbg = batch_pods(st), fb_dbg = s_fb;
  const int32_t cur_dbg = st->cursor;
#endif
  batch_commit(c, P, st, g, m, pmax, s_fb, chosen_out, &s_istar, &s_sched, &s_unsched, s_aw, nullptr, batch_cap(st),
               nullptr, !abroken ? false : true);
#ifdef KSIM_ADAPT_DBG
  __syncthreads();
  if (threadIdx.x == 0) {
    const int32_t committed = st->cursor - cur_dbg;
    atomicAdd(&g_adapt_dbg[0], 1ull);
    if (nchain0 < nb_dbg) atomicAdd(&g_adapt_dbg[1], 1ull);
    if (fb_dbg < nchain0) atomicAdd(&g_adapt_dbg[2], 1ull);
    atomicAdd(&g_adapt_dbg[3], (unsigned long long)nchain0);
    atomicAdd(&g_adapt_dbg[4], (unsigned long long)fb_dbg);
    if (committed < fb_dbg) atomicAdd(&g_adapt_dbg[5], 1ull);
    atomicAdd(&g_adapt_dbg[6], (unsigned long long)committed);
    atomicAdd(&g_adapt_dbg[7], (unsigned long long)nb_dbg);
  }
#endif
}

// ---- deferred commit (ksim_internal.h): batch i-1's commit inside batch i's mask launch ----
// Every block recomputes batch i-1's cut from its ring slot (first broken
// window, then the first pod whose pair maximum beats its guess, as
// k_adapt_commit / batch_commit) and so knows cursor_i.  A block holds 256
// nodes, one per thread: the thread loads its row from X[p ^ 1], adds what
// batch i-1 bound there (the entries whose guess lies in the block, with their
// requests, in LDS), keys its node for the block's pods of batch i (the S_i
// feasibility bitmaps) and, in the blocks of the first pod group, writes the
// row to X[p] (every row: X[p] needs no older binds replayed).  Block b (flat
// index) writes placement b of batch i-1; block 0 writes the state after the
// commit to st[p].  FLUSH: the commit alone (rows written, no bitmaps).
// Trivial cpu/memory pods only (FAST runs).
template <bool FLUSH>
__global__ __launch_bounds__(256) void k_adapt_mask_commit(DevCluster c, DevPods P, const BatchProg* __restrict__ bp_p,
                                                           LazyStep L, const int32_t* __restrict__ b1,
                                                           const int32_t* __restrict__ w1, uint64_t* __restrict__ amask,
                                                           int32_t n_words, int32_t mp, int32_t* __restrict__ chosen_out) {
  static_assert(kBatchPods % 256 == 0, "k_adapt_mask_commit walks the batch in 256-pod chunks");
  constexpr int kChunks = kBatchPods / 256;
  __shared__ int32_t s_fb, s_istar, s_inode, s_sched, s_unsched, s_evals;
  __shared__ int16_t s_dn[256];                    // entry bound on this block's node tid, -1: none
  __shared__ ResCols s_rq[kBatchPods];             // those entries' deltas
  const int tid = threadIdx.x, lane = tid & 63;
  const int32_t nblocks = gridDim.x * gridDim.y, bl = blockIdx.y * gridDim.x + blockIdx.x;
  const int32_t nbase = blockIdx.x * 256;          // this block's first node (4 words of 64)
  const int32_t e1 = *L.e1;
  uint64_t g[kChunks], m[kChunks];
  int32_t brk[kChunks];
#pragma unroll
  for (int q = 0; q < kChunks; q++) {
    g[q] = L.g1[q * 256 + tid];
    m[q] = L.m1[q * 256 + tid];
    brk[q] = b1[q * 256 + tid];
  }
  const int32_t cur0 = L.st_in->cursor, end = L.st_in->end;
  const int64_t seq0 = L.st_in->pod_seq;
  const int32_t nchain0 = e1 > 0 ? e1 : 0;         // -1: no batch i-1
  s_dn[tid] = -1;
  if (tid == 0) {
    s_fb = nchain0;
    s_inode = -1;
    s_sched = 0;
    s_unsched = 0;
    s_evals = 0;
  }
  lds_barrier();
  // the chain ends before the first broken window
#pragma unroll
  for (int q = 0; q < kChunks; q++) {
    const uint64_t mm = __ballot(q * 256 + tid < nchain0 && brk[q]);
    if (mm && lane == 0) atomicMin(&s_fb, q * 256 + (tid & ~63) + __builtin_ctzll(mm));
  }
  lds_barrier();
  const int32_t nchain = s_fb;
  if (tid == 0) s_istar = nchain;
  lds_barrier();
#pragma unroll
  for (int q = 0; q < kChunks; q++) {
    const uint64_t mm = __ballot(q * 256 + tid < nchain && m[q] > g[q]);   // keys are unique per node
    if (mm && lane == 0) atomicMin(&s_istar, q * 256 + (tid & ~63) + __builtin_ctzll(mm));
  }
  lds_barrier();
  const int32_t istar = s_istar;
  const int32_t committed = istar < nchain ? istar + 1 : nchain;
#pragma unroll
  for (int q = 0; q < kChunks; q++)
    if (q * 256 + tid == istar && istar < nchain) s_inode = key_node(m[q]) - c.base;
  lds_barrier();
  const int32_t inode = s_inode;
  // the entries whose guessed node is in this block: pod t's requests (and pod
  // i*'s when i* took the same node)
#pragma unroll
  for (int q = 0; q < kChunks; q++) {
    const int32_t t = q * 256 + tid;
    const int32_t gn = (t < istar && g[q]) ? key_node(g[q]) - c.base : -1;
    if (gn >= nbase && gn < nbase + 256) {
      const ksim_pod& pt = P.pods[cur0 + t];
      ResCols d{pt.req_cpu, pt.req_mem, pt.req_eph, pt.nz_cpu, pt.nz_mem, 1};
      if (gn == inode) {
        const ksim_pod& pi = P.pods[cur0 + istar];
        d.cpu += pi.req_cpu;
        d.mem += pi.req_mem;
        d.eph += pi.req_eph;
        d.nzc += pi.nz_cpu;
        d.nzm += pi.nz_mem;
        d.pods += 1;
      }
      s_rq[t] = d;
      s_dn[gn - nbase] = (int16_t)t;
    }
  }
  // batch i-1's statistics and the state after its commit (block 0)
  if (bl == 0) {
#pragma unroll
    for (int q = 0; q < kChunks; q++) {
      const int32_t t = q * 256 + tid;
      if (t < committed) {
        const int32_t pn = t == istar ? inode + c.base : (g[q] ? key_node(g[q]) : -1);
        atomicAdd(pn >= 0 ? &s_sched : &s_unsched, 1);
        const int2 w = reinterpret_cast<const int2*>(w1)[t];
        atomicAdd(&s_evals, (int32_t)window_local(c, w.x, w.y >= 0 ? (int64_t)w.y + 1 : c.n_total));
      }
    }
  }
  // placements of batch i-1, one per block
  if (tid == 0)
    for (int32_t k = bl; k < committed; k += nblocks) {
      const uint64_t gk = L.g1[k];
      if (chosen_out) chosen_out[cur0 + k] = k == istar ? inode + c.base : (gk ? key_node(gk) : -1);
    }
  lds_barrier();
  if (bl == 0 && tid == 0) {
    // st[p] = st[p ^ 1] with the commit's updates, written whole: its words
    // loaded together, no store-then-reload chain (see k_batch_top_commit)
    constexpr int kWords = (int)(sizeof(DevState) / 8);
    uint64_t wd[kWords];
#pragma unroll
    for (int q = 0; q < kWords; q++) wd[q] = reinterpret_cast<const uint64_t*>(L.st_in)[q];
    DevState ns;
    __builtin_memcpy(&ns, wd, sizeof(ns));
    if (e1 > 0) {
      const int32_t nb = min(kBatchPods, end - cur0);
      ns.cursor = cur0 + committed;
      ns.pod_seq = seq0 + committed;
      ns.scheduled += s_sched;
      ns.unschedulable += s_unsched;
      ns.batches += 1;
      ns.cuts += (committed < nb && istar < nchain ? 1 : 0);
      ns.truncations += (committed < nb && istar >= nchain ? 1 : 0);
      if (committed > 0) {
        const int2 w = reinterpret_cast<const int2*>(w1)[committed - 1];
        ns.next_start = (int32_t)(((int64_t)w.x + (w.y >= 0 ? w.y : c.n_total)) % c.n_total);
        if (c.count_whole) ns.evals += s_evals;
      }
    }
    __builtin_memcpy(wd, &ns, sizeof(ns));
#pragma unroll
    for (int q = 0; q < kWords; q++) reinterpret_cast<uint64_t*>(L.st_out)[q] = wd[q];
    if (FLUSH) *L.e_self = -1;
  }
  // this thread's node: S_i row = X[p ^ 1] + delta; written to X[p] by the
  // first pod group's blocks
  const int32_t node = nbase + tid;
  const bool on = node < c.n;
  const int32_t x = on ? node : 0;
  const int32_t e = s_dn[tid];
  ResCols d{0, 0, 0, 0, 0, 0};
  if (on && e >= 0) d = s_rq[e];
  const int64_t rc = c.req_cpu[x] + d.cpu, rm = c.req_mem[x] + d.mem, re = c.req_eph[x] + d.eph;
  const int32_t np = c.num_pods[x] + d.pods;
  if (on && blockIdx.y == 0) {
    L.w.req_cpu[x] = rc;
    L.w.req_mem[x] = rm;
    L.w.req_eph[x] = re;
    L.w.nz_cpu[x] = c.nz_cpu[x] + d.nzc;
    L.w.nz_mem[x] = c.nz_mem[x] + d.nzm;
    L.w.num_pods[x] = np;
  }
  if (FLUSH) return;
  // the S_i feasibility bitmaps of pods [j0, j1) of batch i (k_adapt_mask_ns's trivial path)
  const int32_t base = cur0 + committed;
  const int32_t nb = min(kBatchPods, end - base);
  const int32_t j0 = blockIdx.y * mp;
  if (j0 >= nb) return;                              // block-uniform
  const int32_t w = blockIdx.x * 4 + (tid >> 6);
  if (w >= n_words) return;                          // wave-uniform
  const int32_t j1 = min(j0 + mp, nb);
  const BatchProg& bp = *bp_p;
  const bool fit = bp.has_fit_filter != 0;
  uint64_t word = 0;                               // lane l: pod j0 + l's ballot
  if (!fit) {                                      // every pod: the nodes that exist
    const uint64_t mk = __ballot(on);
    word = lane < j1 - j0 ? mk : 0ull;
  } else {
    // lane l's pod requests staged in the wave's own LDS rows (a wave reads
    // its own writes in order: no barrier), read back at a uniform address,
    // so each pod costs three 64-bit compares and one LDS row of ballots; a pod
    // with no requests (and no scalar ones) compares as INT64_MIN: it fits
    // wherever a pod slot is free
    __shared__ int64_t s_pq[4][64][4];
    const int wv = tid >> 6;
    if (lane < j1 - j0) {
      const ksim_pod& q = P.pods[base + j0 + lane];
      const bool none = q.req_cpu == 0 && q.req_mem == 0 && q.req_eph == 0 && !(q.flags & KSIM_POD_HAS_SCALAR);
      s_pq[wv][lane][0] = none ? INT64_MIN : q.req_cpu;
      s_pq[wv][lane][1] = none ? INT64_MIN : q.req_mem;
      s_pq[wv][lane][2] = none ? INT64_MIN : q.req_eph;
    }
    const uint64_t room = __ballot(on && np + 1 <= c.alloc_pods[x]);
    const int64_t fc = c.alloc_cpu[x] - rc, fm = c.alloc_mem[x] - rm, fe = c.alloc_eph[x] - re;
    __shared__ uint64_t s_mk[4][64];
#pragma unroll 4
    for (int32_t l = 0; l < j1 - j0; l++) {
      const int64_t c0 = s_pq[wv][l][0], m0 = s_pq[wv][l][1], e0 = s_pq[wv][l][2];
      const uint64_t mk = room & __ballot(c0 <= fc) & __ballot(m0 <= fm) & __ballot(e0 <= fe);
      if (lane == 0) s_mk[wv][l] = mk;
    }
    word = lane < j1 - j0 ? s_mk[wv][lane] : 0ull;
  }
  if (lane < j1 - j0) amask[(size_t)(j0 + lane) * n_words + w] = word;
}

const char* const kAdaptKernelNames[kKernelsPerAdapt] = {"k_adapt_mask", "k_adapt_window", "k_adapt_top",
                                                         "k_adapt_pairs", "k_adapt_commit"};

uint32_t launch_batch_adapt(const LaunchArgs& a, hipStream_t stream, hipEvent_t* evs) {
  const int32_t n_words = (a.c.n + 63) / 64;
  const int32_t k = num_feasible_nodes_to_find(a.prof.percentage_of_nodes_to_score, a.c.n);
  if (evs) (void)hipEventRecord(evs[0], stream);
  const int32_t mp = mask_pods(n_words);
  k_adapt_mask_ns<<<dim3((n_words + 3) / 4, (kBatchPods + mp - 1) / mp), 256, 0, stream>>>(a.c, a.P, a.dbp, a.st,
                                                                                          a.s.amask, n_words, mp);
  if (evs) (void)hipEventRecord(evs[1], stream);
  // generic runs on small clusters: the exact ordered walk as its own launch
  const bool win_seq = !a.fast && n_words <= kWinSeqWords;
  const bool win_fused = !win_seq && k < kTopWideK && n_words <= kWinFusedWords;
  if (win_seq)
    launch_window_dbl(a, n_words, k, stream);
  else if (!win_fused) {
    k_adapt_cut0<<<kBatchPods / 4, 256, 0, stream>>>(a.st, a.s.amask, n_words, a.c.n, k, a.s.acut);
    k_adapt_window<<<1, kBatchPods, 0, stream>>>(a.st, a.s.amask, n_words, a.c.n, k, a.s.acut, a.s.awin, a.s.aexact);
  }
  if (evs) (void)hipEventRecord(evs[2], stream);
#define TOP(F, NT, W) k_adapt_top<false, F, NT, W><<<kBatchPods, NT, 0, stream>>>(a.c, a.P, a.dprof, a.dbp, a.st, \
    a.s.amask, n_words, a.s.awin, a.s.aexact, a.s.topk, a.s.topk_cnt, a.s.topk_complete, nullptr, a.s.pnorm)
  // ordered-walk windows (generic runs): 1,024 threads per pod as for long windows
  if (k >= kTopWideK || win_seq) {
    if (a.fast) TOP(true, 1024, false);
    else TOP(false, 1024, false);
  } else if (win_fused) {
    if (a.fast) TOP(true, 256, true);
    else TOP(false, 256, true);
  } else {
    if (a.fast) TOP(true, 256, false);
    else TOP(false, 256, false);
  }
#undef TOP
  if (evs) (void)hipEventRecord(evs[3], stream);
  k_adapt_pairs<false><<<kBatchPods, kBatchPods, 0, stream>>>(
      a.c, a.P, a.dprof, a.dbp, a.st, a.s.amask, n_words, a.s.awin, a.s.topk, a.s.topk_cnt, a.s.topk_complete,
      a.s.gkey, a.s.chain_end, a.s.pmax, a.s.abroken, a.s.pnorm);
  if (evs) (void)hipEventRecord(evs[4], stream);
  k_adapt_commit<<<1, kBatchPods, 0, stream>>>(a.c, a.P, a.st, a.s.gkey, a.s.chain_end, a.s.pmax, a.s.abroken,
                                               a.s.awin, a.chosen);
  if (evs) (void)hipEventRecord(evs[5], stream);
  return win_fused ? 0x1du : 0x1fu;                 // fused: the window slot is an empty event pair
}

const char* const kLazyAdaptKernelNames[kKernelsPerLazyAdapt] = {"k_adapt_mask_commit", "k_adapt_cut0",
                                                                 "k_adapt_top", "k_adapt_pairs"};

static void launch_adapt_mask_commit(const LazyBatch& z, bool flush, hipStream_t stream) {
  const LaunchArgs& a = z.a;
  const int32_t n_words = (a.c.n + 63) / 64;
  const int32_t mp = mask_pods(n_words);
  const dim3 grid((n_words + 3) / 4, (kBatchPods + mp - 1) / mp);
  if (flush)
    k_adapt_mask_commit<true><<<grid, 256, 0, stream>>>(a.c, a.P, a.dbp, z.step, z.b1, z.w1, a.s.amask, n_words, mp,
                                                        a.chosen);
  else
    k_adapt_mask_commit<false><<<grid, 256, 0, stream>>>(a.c, a.P, a.dbp, z.step, z.b1, z.w1, a.s.amask, n_words, mp,
                                                         a.chosen);
}

uint32_t launch_batch_adapt_lazy(const LazyBatch& z, hipStream_t stream, hipEvent_t* evs) {
  const LaunchArgs& a = z.a;
  const int32_t n_words = (a.c.n + 63) / 64;
  const int32_t k = num_feasible_nodes_to_find(a.prof.percentage_of_nodes_to_score, a.c.n);
  if (evs) (void)hipEventRecord(evs[0], stream);
  launch_adapt_mask_commit(z, false, stream);
  if (evs) (void)hipEventRecord(evs[1], stream);
  const bool win_fused = k < kTopWideK && n_words <= kWinFusedWords;
  if (!win_fused) {
    // the fixpoint check inside the top (every block): no single-block launch
    k_adapt_cut0<<<kBatchPods / 4, 256, 0, stream>>>(z.st, a.s.amask, n_words, a.c.n, k, a.s.acut);
  }
  if (evs) (void)hipEventRecord(evs[2], stream);
  // every later launch reads X[p] (z.cw) and st[p]
#define TOP(NT, W, D) k_adapt_top<false, true, NT, W, D><<<kBatchPods, NT, 0, stream>>>(z.cw, a.P, a.dprof, a.dbp, \
    z.st, a.s.amask, n_words, z.awin, a.s.aexact, a.s.topk, a.s.topk_cnt, a.s.topk_complete, nullptr, nullptr, a.s.acut)
  const bool def = fast_def(a.bp);
  if (k >= kTopWideK) {
    if (def) TOP(1024, 2, true);
    else TOP(1024, 2, false);
  } else if (win_fused) {
    if (def) TOP(256, 1, true);
    else TOP(256, 1, false);
  } else {
    if (def) TOP(256, 2, true);
    else TOP(256, 2, false);
  }
#undef TOP
  if (evs) (void)hipEventRecord(evs[3], stream);
  k_adapt_pairs<false, true><<<kBatchPods, kBatchPods, 0, stream>>>(
      z.cw, a.P, a.dprof, a.dbp, z.st, a.s.amask, n_words, z.awin, a.s.topk, a.s.topk_cnt, a.s.topk_complete, z.gkey,
      z.cend, z.pmax, z.abroken);
  if (evs) (void)hipEventRecord(evs[4], stream);
  return win_fused ? 0xdu : 0xfu;
}

void launch_adapt_lazy_flush(const LazyBatch& z, hipStream_t stream) { launch_adapt_mask_commit(z, true, stream); }

// ---- node-sharded ADAPT batch -----------------------------------
// Shards hold 64-aligned node ranges (adapt_shard_chunk), so shard r's bitmap
// words are the global words [r * W, r * W + W).  Per batch: every shard's
// S0 bitmaps of its own nodes are all-gathered ([R][B][W] words) and unpacked
// into the global bitmap; the windows follow from it identically on every
// shard; each shard lists the top-T of the kept nodes it holds (a record as
// on the P100 path), the records are all-gathered and merged, the chain runs;
// each shard scores the guesses on its nodes (pair keys and broken flags),
// those are all-reduced (max) and every shard commits, binding its own nodes.
__global__ __launch_bounds__(256) void k_adapt_unpack(const DevState* __restrict__ st,
                                                      const uint64_t* __restrict__ recv, int32_t W, int32_t nw,
                                                      uint64_t* __restrict__ amask) {
  const int32_t j = blockIdx.y;
  const int32_t base = st->cursor;
  if (base + j >= min(st->end, base + kBatchPods)) return;   // block-uniform
  for (int32_t w = blockIdx.x * 256 + threadIdx.x; w < nw; w += gridDim.x * 256) {
    const int32_t r = w / W;
    amask[(size_t)j * nw + w] = recv[((size_t)r * kBatchPods + j) * W + (w - r * W)];
  }
}

void launch_adapt_sh_mask(const LaunchArgs& a, uint64_t* send, int32_t W, hipStream_t stream) {
  const int32_t mp = mask_pods(W);
  k_adapt_mask_ns<<<dim3((W + 3) / 4, (kBatchPods + mp - 1) / mp), 256, 0, stream>>>(a.c, a.P, a.dbp, a.st, send, W,
                                                                                     mp);
}

void launch_adapt_sh_window(const LaunchArgs& a, const uint64_t* recv, int32_t W, uint64_t* gmask,
                            hipStream_t stream) {
  const int32_t N = a.c.n_total, nw = (N + 63) / 64;
  const int32_t k = num_feasible_nodes_to_find(a.prof.percentage_of_nodes_to_score, N);
  k_adapt_unpack<<<dim3((nw + 255) / 256, kBatchPods), 256, 0, stream>>>(a.st, recv, W, nw, gmask);
  k_adapt_cut0<<<kBatchPods / 4, 256, 0, stream>>>(a.st, gmask, nw, N, k, a.s.acut);
  k_adapt_window<<<1, kBatchPods, 0, stream>>>(a.st, gmask, nw, N, k, a.s.acut, a.s.awin, a.s.aexact);
#define TOP(F, NT) k_adapt_top<true, F, NT><<<kBatchPods, NT, 0, stream>>>(a.c, a.P, a.dprof, a.dbp, a.st, gmask, \
    nw, a.s.awin, a.s.aexact, a.s.topk, a.s.topk_cnt, a.s.topk_complete, a.s.xsend)
  if (k >= kTopWideK) {
    if (a.fast) TOP(true, 1024);
    else TOP(false, 1024);
  } else {
    if (a.fast) TOP(true, 256);
    else TOP(false, 256);
  }
#undef TOP
}

void launch_adapt_sh_pairs(const LaunchArgs& a, const uint64_t* gmask, int32_t world, hipStream_t stream) {
  const int32_t nw = (a.c.n_total + 63) / 64;
  k_batch_gmerge_launch(a, world, stream);
  k_adapt_pairs<true><<<kBatchPods, kBatchPods, 0, stream>>>(a.c, a.P, a.dprof, a.dbp, a.st, gmask, nw, a.s.awin,
                                                              a.s.topk, a.s.topk_cnt, a.s.topk_complete, a.s.gkey,
                                                              a.s.chain_end, a.s.pmax, nullptr);
}

void launch_adapt_sh_commit(const LaunchArgs& a, hipStream_t stream) {
  k_adapt_commit<<<1, kBatchPods, 0, stream>>>(a.c, a.P, a.st, a.s.gkey, a.s.chain_end, a.s.pmax, nullptr, a.s.awin,
                                               a.chosen);
}

}  // namespace ksim
