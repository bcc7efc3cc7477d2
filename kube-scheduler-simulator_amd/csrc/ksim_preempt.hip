// ksim_preempt.hip — PostFilter: DefaultPreemption's dry run on the device
// (upstream preemption.go / default_preemption.go, v1.26).
//
// After an unschedulable cycle, every node where preemption might help (the
// filter pass failed it at NodeResourcesFit) runs SelectVictimsOnNode on its
// own thread: remove every bound pod of lower priority, check the pod fits,
// then reprieve the removed pods most important first (priority desc, start
// time asc), keeping each one the pod still fits beside.  The bound pods are
// held per node in importance order (CSR), so the lower-priority pods are a
// suffix of the node's range.  One block then keeps the first numCandidates
// candidates in nodeTree order (upstream scans from a random offset; offset 0
// here) and picks one by pickOneNodeForPreemption's criteria.
#include "ksim_device.h"
#include "ksim_internal.h"
#include "ksim_wave.h"

namespace ksim {

__device__ __forceinline__ void row_add_req(NodeRow& r, const int64_t* q, int sign, int n_scalar) {
  r.req_cpu += sign * q[0];
  r.req_mem += sign * q[1];
  r.req_eph += sign * q[2];
#pragma unroll
  for (int k = 0; k < KSIM_MAX_SCALAR; k++)
    if (k < n_scalar) r.req_sc[k] += sign * q[3 + k];
  r.num_pods += sign;
}

// Per node: SelectVictimsOnNode.  res[node] = {candidate, victims, highest
// victim priority, sum of (priority + 2^31), earliest start among the
// highest-priority victims}; vflag marks the victims (CSR order).
__global__ __launch_bounds__(256) void k_preempt_nodes(DevCluster c, DevPods P, const DevState* __restrict__ st,
                                                       DevScratch s, DevPreempt pre, int32_t fit_index,
                                                       int32_t prio) {
  const int32_t node = blockIdx.x * blockDim.x + threadIdx.x;
  if (node >= c.n) return;
  PreemptNode out{};
  out.cand = 0;
  const bool potential = fit_index >= 0 && s.fail[node] == (uint8_t)fit_index;
  out.potential = potential;
  if (potential) {
    const ksim_pod& p = P.pods[st->cursor];
    const int32_t a = pre.off[node], b = pre.off[node + 1];
    int32_t j0 = a;
    while (j0 < b && pre.prio[j0] >= prio) j0++;       // lower priorities: the suffix [j0, b)
    for (int32_t j = a; j < j0; j++) pre.vflag[j] = 0;   // no stale flags from an earlier preemptor
    NodeRow r = load_row(c, node);
    if (pre.nslot && pre.nslot[node] >= 0) {              // the nominated pods stay (pass 1)
      const int64_t* q = pre.nreq + (size_t)pre.nslot[node] * (KSIM_PREEMPT_REQ + 1);
      row_add_req(r, q, 1, c.n_scalar);
      r.num_pods += (int32_t)q[KSIM_PREEMPT_REQ] - 1;
    }
    for (int32_t j = j0; j < b; j++) row_add_req(r, pre.req + (size_t)j * KSIM_PREEMPT_REQ, -1, c.n_scalar);
    if (fits_request(r, p, c.n_scalar, c.fit_ignore) == 0) {
      out.cand = 1;
      int32_t nv = 0, high = 0;
      int64_t sum = 0, early = INT64_MAX;
      for (int32_t j = j0; j < b; j++) {                 // reprievePod, most important first
        const int64_t* q = pre.req + (size_t)j * KSIM_PREEMPT_REQ;
        row_add_req(r, q, 1, c.n_scalar);
        const bool victim = fits_request(r, p, c.n_scalar, c.fit_ignore) != 0;
        pre.vflag[j] = victim;
        if (victim) {
          row_add_req(r, q, -1, c.n_scalar);
          if (nv == 0) high = pre.prio[j];
          sum += (int64_t)pre.prio[j] + ((int64_t)INT32_MAX + 1);
          if (pre.prio[j] == high && pre.start[j] < early) early = pre.start[j];   // GetEarliestPodStartTime
          nv++;
        }
      }
      out.nv = nv;
      out.high = nv ? high : INT32_MIN;
      out.sum = sum;
      out.early = early;
    } else {
      for (int32_t j = j0; j < b; j++) pre.vflag[j] = 0;
    }
  }
  pre.res[node] = out;
}

// pickOneNodeForPreemption order: a is better than b
__device__ __forceinline__ bool better(const PreemptNode& a, int32_t na, const PreemptNode& b, int32_t nb) {
  if (nb < 0) return na >= 0;
  if (na < 0) return false;
  if (a.high != b.high) return a.high < b.high;
  if (a.sum != b.sum) return a.sum < b.sum;
  if (a.nv != b.nv) return a.nv < b.nv;
  if (a.early != b.early) return a.early > b.early;
  return na < nb;                                        // the first candidate in scan order
}

constexpr int kPickThreads = 1024;

// min_pct / min_abs: DefaultPreemptionArgs (calculateNumCandidates)
__global__ __launch_bounds__(kPickThreads) void k_preempt_pick(DevCluster c, DevPreempt pre, int32_t min_pct,
                                                               int32_t min_abs) {
  __shared__ int32_t sh[kPickThreads / 64];
  __shared__ PreemptNode s_best[kPickThreads];
  __shared__ int32_t s_node[kPickThreads];
  const int tid = threadIdx.x;
  const int32_t N = c.n, chunk = (N + kPickThreads - 1) / kPickThreads;
  const int32_t lo = min(N, tid * chunk), hi = min(N, lo + chunk);
  int32_t npot = 0, ncand = 0;
  for (int32_t x = lo; x < hi; x++) {
    npot += pre.res[x].potential;
    ncand += pre.res[x].cand;
  }
  // GetOffsetAndNumCandidates over the potential nodes; candidates are kept
  // in nodeTree order until that many were found
  int32_t total_pot, cexcl, total_cand;
  {
    const int lane = tid & 63, w = tid >> 6;
    int32_t x = npot, y = ncand;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int32_t a = __shfl_up(x, d, 64), b = __shfl_up(y, d, 64);
      if (lane >= d) {
        x += a;
        y += b;
      }
    }
    __syncthreads();
    if (lane == 63) sh[w] = x;
    __syncthreads();
    int32_t base = 0, tot = 0;
    for (int i = 0; i < kPickThreads / 64; i++) {
      if (i < w) base += sh[i];
      tot += sh[i];
    }
    total_pot = tot;
    __syncthreads();
    if (lane == 63) sh[w] = y;
    __syncthreads();
    base = 0;
    tot = 0;
    for (int i = 0; i < kPickThreads / 64; i++) {
      if (i < w) base += sh[i];
      tot += sh[i];
    }
    cexcl = base + y - ncand;
    total_cand = tot;
  }
  int32_t want = total_pot * min_pct / 100;
  if (want < min_abs) want = min_abs;
  if (want > total_pot) want = total_pot;
  PreemptNode best{};
  int32_t best_node = -1, rank = cexcl;
  for (int32_t x = lo; x < hi; x++) {
    const PreemptNode& r = pre.res[x];
    if (!r.cand) continue;
    if (rank < want && better(r, x, best, best_node)) {
      best = r;
      best_node = x;
    }
    rank++;
  }
  s_best[tid] = best;
  s_node[tid] = best_node;
  __syncthreads();
  for (int stride = kPickThreads / 2; stride > 0; stride >>= 1) {
    if (tid < stride && better(s_best[tid + stride], s_node[tid + stride], s_best[tid], s_node[tid])) {
      s_best[tid] = s_best[tid + stride];
      s_node[tid] = s_node[tid + stride];
    }
    __syncthreads();
  }
  if (tid == 0) {
    pre.pick[0] = s_node[0];
    pre.pick[1] = s_node[0] >= 0 ? s_best[0].nv : 0;
    pre.pick[2] = total_pot;
    pre.pick[3] = total_cand < want ? total_cand : want;
  }
}

void launch_preempt(const LaunchArgs& a, const DevPreempt& pre, int32_t fit_index, int32_t prio,
                    hipStream_t stream, bool filter) {
  const int blocks = (a.c.n + 255) / 256;
  if (filter) launch_filter_only(a, stream);             // the filter statuses of every node
  k_preempt_nodes<<<blocks, 256, 0, stream>>>(a.c, a.P, a.st, a.s, pre, fit_index, prio);
  k_preempt_pick<<<1, kPickThreads, 0, stream>>>(a.c, pre, a.prof.preempt_min_pct, a.prof.preempt_min_abs);
}

}  // namespace ksim
