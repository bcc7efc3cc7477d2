// ksim_batch.hip — the speculative batch path of the scheduling cycle (gfx950).
//
// For B = 64 consecutive pods of the queue that are "batchable" (P100, every
// normalized score constant over nodes, no scalar requests; see
// pod_batchable in ksim_engine.cpp), placements equal running the cycle pod by
// pod (bit-exact with the oracle), in three launches per batch:
//
//   k_batch_eval    grid (node tiles, pods): every pod x node pair against the
//                   batch-start snapshot S0 — static filters, Fit filter,
//                   LeastAllocated, BalancedAllocation, TB key.  A wave tile is
//                   64 lanes x 4 nodes; each lane sorts its 4 keys and 4 rounds
//                   of DPP wave-max keep the tile's 4 best keys.
//   k_batch_merge   one wave per pod: merge the sorted tile lists into the
//                   pod's top-T under S0 (a prefix that is provably exact), and
//                   gather the S0 rows of those T nodes.
//   k_batch_repair  one 1024-thread block: the exact sequential replay by
//                   speculation rounds (greedy guesses validated in parallel
//                   against the nodes bound so far; see the kernel).  Only
//                   bound nodes differ from S0, hence exactness.  An exhausted
//                   list cuts the batch; the next batch restarts at that pod.
#include "ksim_device.h"
#include "ksim_internal.h"
#include "ksim_wave.h"

namespace ksim {

__global__ __launch_bounds__(256) void k_batch_eval(DevCluster c, DevPods P, ksim_profile prof, BatchProg bp,
                                                    const DevState* __restrict__ st, uint64_t* __restrict__ cand,
                                                    int32_t n_tiles) {
  const int32_t base = st->cursor;
  const int32_t end = min(st->end, base + kBatchPods);
  const int32_t j = blockIdx.y;                      // one pod of the batch per grid row
  const int32_t pi = base + j;
  if (pi >= end) return;
  const int lane = threadIdx.x & 63;
  const int32_t tile = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (tile >= n_tiles) return;                       // wave-uniform
  const ksim_pod& p = P.pods[pi];
  const int32_t nc = P.norm_const[pi];
  const int64_t seq = st->pod_seq + j;
  uint64_t a[kNodesPerLane];
#pragma unroll
  for (int k = 0; k < kNodesPerLane; k++) {
    const int32_t node = tile * kTileNodes + k * 64 + lane;
    uint64_t kk = 0;
    if (node < c.n) {
      const NodeRow r = load_row(c, node);
      if (static_filters_pass(c, P, bp, p, r)) kk = dyn_key(prof, bp, p, nc, r, c.n_scalar, seq);
    }
    a[k] = kk;
  }
  static_assert(kNodesPerLane == 4 && kTileCand == 4, "sorting network below is for 4 keys");
  cswap_desc(a[0], a[1]);
  cswap_desc(a[2], a[3]);
  cswap_desc(a[0], a[2]);
  cswap_desc(a[1], a[3]);
  cswap_desc(a[1], a[2]);
  uint64_t* out = cand + ((size_t)j * n_tiles + tile) * kTileCand;
#pragma unroll
  for (int t = 0; t < kTileCand; t++) {
    const uint64_t m = wave_max_u64_dpp(a[0]);
    if (lane == 0) out[t] = m;
    if (m != 0 && a[0] == m) {
      a[0] = a[1];
      a[1] = a[2];
      a[2] = a[3];
      a[3] = 0;
    }
  }
}

// A tile list holds only its best kTileCand keys: once one is fully consumed
// the merge can no longer prove the next key, so the prefix ends there
// (complete = 0).  complete = 1: every S0-feasible node is listed.
__global__ __launch_bounds__(256) void k_batch_merge(DevCluster c, const DevState* __restrict__ st,
                                                     const uint64_t* __restrict__ cand, int32_t n_tiles,
                                                     uint64_t* __restrict__ topk, int32_t* __restrict__ topk_cnt,
                                                     int32_t* __restrict__ topk_complete, BRow* __restrict__ rows) {
  extern __shared__ __attribute__((aligned(16))) uint64_t s_m[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int32_t j = blockIdx.x * 4 + w;
  const int32_t base = st->cursor;
  if (base + j >= min(st->end, base + kBatchPods)) return;   // wave-uniform; no block barrier below
  const int32_t per = n_tiles * kTileCand;
  uint64_t* lst = s_m + (size_t)w * (per + (n_tiles + 7) / 8);
  uint8_t* head = reinterpret_cast<uint8_t*>(lst + per);
  const uint64_t* src = cand + (size_t)j * per;
  for (int x = lane; x < per; x += 64) lst[x] = src[x];
  for (int l = lane; l < n_tiles; l += 64) head[l] = 0;
  wave_lds_sync();
  uint64_t mine = 0;                                 // lane t keeps merged key t
  int32_t cnt = 0, complete = 0;
  for (int t = 0; t < kTopT; t++) {
    uint64_t best = 0;
    int32_t bl = -1;
    for (int l = lane; l < n_tiles; l += 64) {
      const int h = head[l];
      const uint64_t v = h < kTileCand ? lst[l * kTileCand + h] : 0;
      if (v > best) { best = v; bl = l; }
    }
    const uint64_t m = wave_max_u64_dpp(best);
    if (m == 0) { complete = 1; break; }
    if (lane == t) mine = m;
    cnt = t + 1;
    bool stop = false;
    if (best == m) {
      const int h = ++head[bl];
      stop = h == kTileCand;
    }
    if (__ballot(stop)) break;
    wave_lds_sync();
  }
  if (lane < kTopT) topk[(size_t)j * kTopT + lane] = lane < cnt ? mine : 0;
  if (lane < cnt) rows[(size_t)j * kTopT + lane] = to_brow(load_row(c, key_node(mine)));
  if (lane == 0) {
    topk_cnt[j] = cnt;
    topk_complete[j] = complete;
  }
}

// Open-addressing set of node ids in LDS (bound + guessed nodes of a batch;
// at most 2 x kBatchPods live entries, so the load factor stays <= 1/2).
constexpr int kHashSlots = 256;

__device__ __forceinline__ uint32_t node_hash(int32_t nd) { return ((uint32_t)nd * 0x9E3779B1u) >> 24; }

__device__ __forceinline__ bool hash_has(const int32_t* hs, int32_t nd) {
  uint32_t h = node_hash(nd);
  while (true) {
    const int32_t v = hs[h];
    if (v == nd) return true;
    if (v < 0) return false;
    h = (h + 1) & (kHashSlots - 1);
  }
}

__device__ __forceinline__ void hash_insert(int32_t* hs, int32_t nd) {
  uint32_t h = node_hash(nd);
  while (true) {
    const int32_t prev = atomicCAS(&hs[h], -1, nd);
    if (prev == -1 || prev == nd) return;
    h = (h + 1) & (kHashSlots - 1);
  }
}

// Exact sequential replay of one batch by speculation rounds.  A round from
// pod s0 on:
//   A (wave 0, lane j = pod j)  greedy chain: pod i guesses the first entry of
//       its list whose node is neither bound nor guessed by an earlier pod of
//       the round; each guess opens a tentative slot (its S0 row + pod i).
//   B (all threads)  key of every later pod on every tentative slot.
//   C (wave 0)  pod i's exact choice is max(guess key, best key over the slots
//       of earlier pods): the guess is unbound so its S0 key is current, and
//       only slots differ from S0.  Pods up to the first mismatch i* commit;
//       i* itself takes its best slot (that slot's keys are recomputed for the
//       later pods) and the next round starts at i* + 1.
// An exhausted incomplete list cuts the batch (the next batch starts there).
__global__ __launch_bounds__(kRepairThreads) void k_batch_repair(
    DevCluster c, DevPods P, ksim_profile prof, BatchProg bp, DevState* __restrict__ st,
    const uint64_t* __restrict__ topk, const int32_t* __restrict__ topk_cnt,
    const int32_t* __restrict__ topk_complete, const BRow* __restrict__ rows, int32_t* __restrict__ chosen_out) {
  __shared__ __attribute__((aligned(16))) uint64_t s_top[kBatchPods][kTopT];  //  8 KB
  __shared__ uint64_t s_kc[kBatchPods][kBatchPods];   // 32 KB: [slot][pod] key of pod on the slot's row
  __shared__ BRow s_slot[kBatchPods];                 //  6 KB: current row of each slot
  __shared__ ksim_pod s_pod[kBatchPods];              // 12.5 KB
  __shared__ int32_t s_hash[kHashSlots];
  __shared__ int32_t s_nc[kBatchPods], s_owner[kBatchPods], s_gslot[kBatchPods], s_gptr[kBatchPods];
  __shared__ int32_t s_chosen[kBatchPods];
  __shared__ uint64_t s_gkey[kBatchPods];
  __shared__ int32_t s_ctl[8];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int32_t base = st->cursor;
  const int32_t nb = min(kBatchPods, st->end - base);
  if (nb <= 0) return;
  const int64_t seq0 = st->pod_seq;
  static_assert(sizeof(s_top) == 8 * 1024 && kRepairThreads >= 8 * 64, "one 1 KiB DMA chunk per wave");
  if (wave < 8)
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)(reinterpret_cast<const uint4*>(topk) + wave * 64 + lane),
        (__attribute__((address_space(3))) void*)(reinterpret_cast<uint4*>(&s_top[0][0]) + wave * 64), 16, 0, 0);
  {
    const uint32_t* gp = reinterpret_cast<const uint32_t*>(P.pods + base);
    uint32_t* lp = reinterpret_cast<uint32_t*>(s_pod);
    const int words = nb * (int)(sizeof(ksim_pod) / 4);
    for (int x = tid; x < words; x += kRepairThreads) lp[x] = gp[x];
  }
  if (tid < kBatchPods) s_nc[tid] = tid < nb ? P.norm_const[base + tid] : 0;
  for (int x = tid; x < kHashSlots; x += kRepairThreads) s_hash[x] = -1;
  const int32_t cnt = (wave == 0 && lane < nb) ? topk_cnt[lane] : 0;
  const int32_t complete = (wave == 0 && lane < nb) ? topk_complete[lane] : 1;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  int32_t s0 = 0, nslots = 0, committed = nb, rounds = 0;
  while (true) {
    rounds++;
    // ---- A: greedy chain (wave 0) ----
    if (wave == 0) {
      int ptr = 0;
      uint64_t cur = 0;
      const bool active = lane >= s0 && lane < nb;
      auto advance = [&]() {
        while (ptr < cnt && hash_has(s_hash, key_node(s_top[lane][ptr]))) ptr++;
        cur = ptr < cnt ? s_top[lane][ptr] : 0;
      };
      if (active) advance();
      int32_t nchain = nb, cut = -1, ntent = 0;
      for (int i = s0; i < nb; i++) {
        const uint64_t g = readlane_u64(cur, i);
        if (g == 0 && !__builtin_amdgcn_readlane(complete, i)) {
          nchain = cut = i;
          break;
        }
        const int32_t gnode = g ? key_node(g) : -1;
        if (lane == i) {
          s_gkey[i] = g;
          s_gptr[i] = ptr;
          s_gslot[i] = g ? nslots + ntent : -1;
          if (g) {
            s_owner[nslots + ntent] = i;
            hash_insert(s_hash, gnode);
          }
        }
        ntent += g ? 1 : 0;
        wave_lds_sync();
        if (g && active && lane > i && cur != 0 && key_node(cur) == gnode) advance();
      }
      if (lane == 0) {
        s_ctl[0] = nchain;
        s_ctl[1] = cut;
        s_ctl[2] = ntent;
      }
    }
    __syncthreads();
    const int32_t nchain = s_ctl[0], cut = s_ctl[1], ntent = s_ctl[2];
    // ---- B: tentative slot rows, then keys of later pods on them ----
    if (tid >= s0 && tid < nchain && s_gslot[tid] >= 0)
      brow_assign_add(s_slot[s_gslot[tid]], rows[(size_t)tid * kTopT + s_gptr[tid]], s_pod[tid]);
    __syncthreads();
    for (int idx = tid; idx < kBatchPods * kBatchPods; idx += kRepairThreads) {
      const int x = idx >> 6, i = idx & 63;
      if (x < nslots || x >= nslots + ntent || i >= nb || s_owner[x] >= i) continue;
      const ksim_pod& p = s_pod[i];
      const NodeRow rr = from_brow(s_slot[x]);
      s_kc[x][i] = static_filters_pass(c, P, bp, p, rr) ? dyn_key(prof, bp, p, s_nc[i], rr, c.n_scalar, seq0 + i) : 0;
    }
    __syncthreads();
    // ---- C: validate the chain (wave 0, lane i = pod i) ----
    if (wave == 0) {
      uint64_t m = 0;
      int32_t mx = -1;
      const bool inchain = lane >= s0 && lane < nchain;
      if (inchain)
        for (int x = 0; x < nslots + ntent; x++) {
          if (s_owner[x] >= lane) break;             // tentative slots are in pod order
          const uint64_t v = s_kc[x][lane];
          if (v > m) { m = v; mx = x; }
        }
      const uint64_t gk = inchain ? s_gkey[lane] : 0;
      const bool bad = inchain && m > gk;            // keys are unique per node: never equal unless 0
      const uint64_t badm = __ballot(bad);
      const int32_t istar = badm ? (int32_t)__builtin_ctzll(badm) : nchain;
      if (inchain && lane < istar) s_chosen[lane] = gk ? key_node(gk) : -1;
      // tentative slots of committed pods stay; later ones are dropped
      int32_t keep = ntent;
      for (int x = nslots; x < nslots + ntent; x++)
        if (s_owner[x] >= istar) { keep = x - nslots; break; }
      int32_t xs = -1;
      if (istar < nchain) {
        xs = __builtin_amdgcn_readlane(mx, istar);
        if (lane == istar) {
          brow_add_pod(s_slot[xs], s_pod[istar]);
          s_chosen[istar] = s_slot[xs].node;
        }
      }
      if (lane == 0) {
        s_ctl[3] = istar;
        s_ctl[4] = xs;
        s_ctl[5] = nslots + keep;
      }
    }
    __syncthreads();
    const int32_t istar = s_ctl[3], xs = s_ctl[4];
    nslots = s_ctl[5];
    if (istar >= nchain) {                            // the whole chain held
      if (cut >= 0) committed = cut;
      break;
    }
    s0 = istar + 1;
    if (s0 >= nb) break;
    // ---- D: pod i* changed slot xs: rekey it for the later pods; rebuild the set ----
    if (tid > istar && tid < nb) {
      const ksim_pod& p = s_pod[tid];
      const NodeRow rr = from_brow(s_slot[xs]);
      s_kc[xs][tid] = static_filters_pass(c, P, bp, p, rr) ? dyn_key(prof, bp, p, s_nc[tid], rr, c.n_scalar, seq0 + tid) : 0;
    }
    for (int x = tid; x < kHashSlots; x += kRepairThreads) s_hash[x] = -1;
    __syncthreads();
    if (tid < nslots) hash_insert(s_hash, s_slot[tid].node);
    __syncthreads();
  }
  // commit: placements, bound rows back to the HBM snapshot, scheduler state
  if (chosen_out)
    for (int x = tid; x < committed; x += kRepairThreads) chosen_out[base + x] = s_chosen[x];
  for (int x = tid; x < nslots; x += kRepairThreads) store_brow_dynamic(c, s_slot[x]);
  if (wave == 0) {
    const bool ok = lane < committed;
    const uint64_t sm = __ballot(ok && s_chosen[lane] >= 0), um = __ballot(ok && s_chosen[lane] < 0);
    if (lane == 0) {
      st->cursor = base + committed;
      st->pod_seq = seq0 + committed;
      st->evals += (int64_t)committed * c.n;
      st->scheduled += __builtin_popcountll(sm);
      st->unschedulable += __builtin_popcountll(um);
      st->batches += 1;
      if (committed < nb) st->truncations += 1;
      st->rounds += rounds;
    }
  }
}

const char* const kBatchKernelNames[kKernelsPerBatch] = {"k_batch_eval", "k_batch_merge", "k_batch_repair"};

void launch_batch(const LaunchArgs& a, hipStream_t stream, hipEvent_t* evs) {
  const int32_t n_tiles = (a.c.n + kTileNodes - 1) / kTileNodes;
  const dim3 g1((n_tiles + 3) / 4, kBatchPods);
  if (evs) (void)hipEventRecord(evs[0], stream);
  k_batch_eval<<<g1, 256, 0, stream>>>(a.c, a.P, a.prof, a.bp, a.st, a.s.cand, n_tiles);
  if (evs) (void)hipEventRecord(evs[1], stream);
  const size_t per_wave = (size_t)n_tiles * kTileCand * 8 + (size_t)((n_tiles + 7) / 8) * 8;
  k_batch_merge<<<kBatchPods / 4, 256, 4 * per_wave, stream>>>(a.c, a.st, a.s.cand, n_tiles, a.s.topk, a.s.topk_cnt,
                                                               a.s.topk_complete, a.s.rows);
  if (evs) (void)hipEventRecord(evs[2], stream);
  k_batch_repair<<<1, kRepairThreads, 0, stream>>>(a.c, a.P, a.prof, a.bp, a.st, a.s.topk, a.s.topk_cnt, a.s.topk_complete,
                                       a.s.rows, a.chosen);
  if (evs) (void)hipEventRecord(evs[3], stream);
}

}  // namespace ksim
