// ksim_chain.h — the batch paths' greedy chain, run inside the chain + pairs
// launches of the P100, ADAPT and topology batches.
#pragma once
#include "ksim_device.h"
#include "ksim_internal.h"
#include "ksim_wave.h"

namespace ksim {

constexpr int kHashBits = kBatchPods * kTopT <= 2048 ? 12 : kBatchPods * kTopT <= 4096 ? 13 : 14;
constexpr int kHashSlots = 1 << kHashBits;     // >= 2 x the list entries (linear probing)
constexpr int kChainRounds = 64;               // exact prefix kept if not converged by then

// KSIM_CHAIN_DELAY builds (the race regression test, tests/test_gpu_chain_race.py):
// stretch the round boundary the per-parity flags protect.  The last wave
// sleeps before it reads the round's flag, so the fastest wave (thread 0's,
// which resets the flag slot) is a whole round ahead when it does; the
// pre-76f29c9 single flag reset at the top of a round would then be read as
// "every pod exact" by the sleeping wave.  s_sleep is a scalar ALU wait.
#ifdef KSIM_CHAIN_DELAY
#define CHAIN_DELAY(wave_sel)                                                      \
  do {                                                                             \
    if ((int)(threadIdx.x >> 6) == (wave_sel)) {                                   \
      __builtin_amdgcn_s_sleep(127);                                               \
      __builtin_amdgcn_s_sleep(127);                                               \
    }                                                                              \
  } while (0)
#else
#define CHAIN_DELAY(wave_sel) do {} while (0)
#endif
static_assert(kBatchPods * kTopT * 2 <= kHashSlots, "chain hash table too small");

// Clusters of at most kChainDirect nodes index the holders by node id (no hash
// probes while the lists are registered): config 2 7.03 -> 6.80 ms per step
// (profiles/r03/ab_chaindirect)
constexpr int kChainDirect = 8192;
constexpr int kChainHoldSlots = kHashSlots > kChainDirect ? kHashSlots : kChainDirect;
struct ChainLds {
  int32_t key[kHashSlots];                     // node id in the slot, -1 = empty (hash mode)
  int32_t hold[2][kChainHoldSlots];            // per round parity: lowest pod index holding the slot
  int16_t rep[kBatchPods][kTopT];              // slot of each list entry
  int32_t first[2], cut;                      // first: one slot per round parity (see the round loop)
};

// The chain of one batch in one block of kBatchPods threads (thread i = pod
// i; pods from nb_cap on take no part).  Returns false when the batch is empty (block-uniform); else *gk = pod
// i's guessed key (0: none, or i past the exact prefix) and *nchain = the
// prefix length.  A pure function of the lists: every block that runs it gets
// the same guesses.
// The top T of two descending lists, descending, into x: the elementwise max
// of x and y reversed is bitonic and holds the top T; a half-cleaner network
// sorts it.
__device__ __forceinline__ void merge_top(uint64_t (&x)[kTopT], const uint64_t (&y)[kTopT]) {
  static_assert((kTopT & (kTopT - 1)) == 0, "bitonic merge: T a power of two");
#pragma unroll
  for (int e = 0; e < kTopT; e++) x[e] = umax64(x[e], y[kTopT - 1 - e]);
#pragma unroll
  for (int h = kTopT / 2; h >= 1; h >>= 1)
#pragma unroll
    for (int e = 0; e < kTopT; e++)
      if ((e & h) == 0) cswap_desc(x[e], x[e + h]);
}

// R > 1: pod i's list is R records (i * R + r: a node slice's provable top-T,
// count, complete), merged here.  A key is provable when it is >= the last
// listed key of every incomplete record (a record hides only keys below its
// last); the merged list is complete when every record is and nothing was
// dropped.
template <int R = 1>
__device__ __forceinline__ bool chain_block(ChainLds& L, const DevState* __restrict__ st,
                                            const uint64_t* __restrict__ topk,
                                            const int32_t* __restrict__ topk_cnt,
                                            const int32_t* __restrict__ topk_complete, uint64_t* gk,
                                            int32_t* nchain_out, unsigned long long* __restrict__ dbg,
                                            int32_t nb_cap = kBatchPods, int32_t direct_n = 0) {
  int32_t* const s_key = L.key;
  int32_t& s_cut = L.cut;
  // phase clock (100 MHz realtime): dbg[0] setup, dbg[1] rounds, dbg[2] epilogue, dbg[3] launches, dbg[4] rounds run
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const int i = threadIdx.x;                   // one pod per thread
  // the pod's list, count and state in flight together (independent loads;
  // the buffers hold kBatchPods entries, so no bound check is needed yet)
  uint64_t lst[kTopT];
  int cnt0, complete0;
  if constexpr (R == 1) {
#pragma unroll
    for (int e = 0; e < kTopT; e++) lst[e] = topk[(size_t)i * kTopT + e];
    cnt0 = topk_cnt[i];
    complete0 = topk_complete[i];
  } else {
    uint64_t k[R][kTopT];
    int32_t rc[R], rp[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
#pragma unroll
      for (int e = 0; e < kTopT; e++) k[r][e] = topk[((size_t)i * R + r) * kTopT + e];
      rc[r] = topk_cnt[i * R + r];
      rp[r] = topk_complete[i * R + r];
    }
    uint64_t thr = 0;
    int32_t all_c = 1, csum = 0;
#pragma unroll
    for (int r = 0; r < R; r++) {
      uint64_t last = ~0ull;                     // an incomplete empty record proves nothing
#pragma unroll
      for (int e = 0; e < kTopT; e++) last = e == rc[r] - 1 ? k[r][e] : last;
      if (!rp[r]) thr = umax64(thr, last);
      all_c &= rp[r];
      csum += rc[r];
    }
#pragma unroll
    for (int r = 0; r < R; r++)
#pragma unroll
      for (int e = 0; e < kTopT; e++)
        if (k[r][e] < thr) k[r][e] = 0;          // a sorted suffix: the records stay sorted
#pragma unroll
    for (int e = 0; e < kTopT; e++) lst[e] = k[0][e];
#pragma unroll
    for (int r = 1; r < R; r++) merge_top(lst, k[r]);
    cnt0 = 0;
#pragma unroll
    for (int e = 0; e < kTopT; e++) cnt0 += lst[e] != 0;
    complete0 = all_c && csum <= kTopT;
  }
  const int32_t base = st->cursor;
  const int32_t nb = min(nb_cap, st->end - base);   // nb_cap: the topology batch's pod count
  if (nb <= 0) return false;
  const int cnt = i < nb ? cnt0 : 0;
  const bool incomplete = i < nb && !complete0;
  if (i < 2) L.first[i] = kBatchPods;
  // this pod's slots in registers (selects below, never a dynamic index)
  int32_t rep[kTopT];
  if (direct_n > 0 && direct_n <= kChainDirect) {   // block-uniform: the slot is the node id
#pragma unroll
    for (int e = 0; e < kTopT; e++) rep[e] = e < cnt ? key_node(lst[e]) : -1;
  } else {
    for (int x = i; x < kHashSlots; x += kBatchPods) s_key[x] = -1;
    lds_barrier();
#pragma unroll
    for (int e = 0; e < kTopT; e++) {
      int16_t slot = -1;
      if (e < cnt) {
        const int32_t node = key_node(lst[e]);
        uint32_t h = ((uint32_t)node * 2654435761u) >> (32 - kHashBits);
        while (true) {
          const int32_t prev = atomicCAS(&s_key[h], -1, node);
          if (prev == -1 || prev == node) break;
          h = (h + 1) & (kHashSlots - 1);
        }
        slot = (int16_t)h;
      }
      L.rep[i][e] = slot;
    }
    lds_barrier();
#pragma unroll
    for (int e = 0; e < kTopT; e++) rep[e] = L.rep[i][e];
  }
  // only the slots the lists name are ever read: each pod clears its own (a
  // slot shared by several lists is cleared by each, to the same value)
#pragma unroll
  for (int e = 0; e < kTopT; e++)
    if (e < cnt) L.hold[0][rep[e]] = L.hold[1][rep[e]] = kBatchPods;
  lds_barrier();
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  int a = cnt > 0 ? 0 : -1;                    // current guess (entry index) or -1
  int32_t pra = -1;                            // the slot this pod registered last round
  int first = kBatchPods, rounds = 0;
  for (; rounds < kChainRounds; rounds++) {
    // Round r registers in hold[r & 1] and reports in first[r & 1], with two
    // barriers.  The other parity's table and flag were last read in round
    // r - 1, by every thread before this round's first barrier, so they are
    // reset after it, for round r + 1 (resetting the current flag at the top
    // of the round raced with slower waves still reading the previous round's).
    const int par = rounds & 1;
    int32_t ra = 0;
#pragma unroll
    for (int e = 0; e < kTopT; e++) ra = e == a ? rep[e] : ra;
    if (a >= 0) atomicMin(&L.hold[par][ra], i);
    lds_barrier();
    CHAIN_DELAY(1);                            // a middle wave late after the first barrier
    if (pra >= 0) L.hold[par ^ 1][pra] = kBatchPods;
    if (i == 0) L.first[par ^ 1] = kBatchPods;
    // every entry's holder at once, then the first one not held by an earlier pod
    int32_t held[kTopT];
#pragma unroll
    for (int e = 0; e < kTopT; e++) held[e] = e < cnt ? L.hold[par][rep[e]] : 0;
    int na = -1;
#pragma unroll
    for (int e = kTopT - 1; e >= 0; e--)
      if (e < cnt && held[e] >= i) na = e;
    {                                          // the wave's first changed pod: one LDS atomic per wave
      const uint64_t chg = __ballot(na != a);
      if (chg && (threadIdx.x & 63) == 0) atomicMin(&L.first[par], (int)(threadIdx.x & ~63u) + __builtin_ctzll(chg));
    }
    pra = a >= 0 ? ra : -1;
    a = na;
    lds_barrier();
    CHAIN_DELAY((int)(blockDim.x >> 6) - 1);   // the last wave reads the flag late
    first = L.first[par];
    if (first == kBatchPods) break;            // a fixpoint: every pod exact
  }
  // exact prefix [0, first); an exhausted incomplete list inside it cuts the chain
  if (i == 0) s_cut = first < nb ? first : nb;
  lds_barrier();
  block_first_min(&s_cut, i < first && i < nb && a < 0 && incomplete);
  lds_barrier();
  const int32_t nchain = s_cut;
  const uint64_t t2 = __builtin_amdgcn_s_memrealtime();
  uint64_t ga = 0;
#pragma unroll
  for (int e = 0; e < kTopT; e++) ga = e == a ? lst[e] : ga;   // register select, no dynamic index
  *gk = (i < nchain && a >= 0) ? ga : 0;
  *nchain_out = nchain;
  if (i == 0 && dbg) {
    const uint64_t t3 = __builtin_amdgcn_s_memrealtime();
    atomicAdd(&dbg[0], (unsigned long long)(t1 - t0));
    atomicAdd(&dbg[1], (unsigned long long)(t2 - t1));
    atomicAdd(&dbg[2], (unsigned long long)(t3 - t2));
    atomicAdd(&dbg[3], 1ull);
    atomicAdd(&dbg[4], (unsigned long long)(rounds + 1));
  }
  return true;
}

}  // namespace ksim
