// ksim_device.h — device-side data layout and plugin arithmetic (gfx950).
//
// Each __device__ function restates the same upstream v1.26.2 function as the
// CPU oracle (oracle/ksim_oracle.c) does; the HIP kernels in ksim_kernels.hip
// compose them.  Compiled with -ffp-contract=off and no fast-math so float64
// division / sqrt are IEEE correctly rounded and nothing is fused (Go on
// GOAMD64=v1 never fuses), which makes BalancedAllocation bit-exact.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ksim_engine.h"

namespace ksim {

constexpr int kMaxNodeScore = 100;

// Node snapshot resident in HBM, structure-of-arrays (one column per field,
// node position = nodeTree order).  Static columns are read-only; the dynamic
// ones (requested / non-zero requested / pod count) are updated in place by
// the bind step of every cycle (NodeInfo.AddPod), never re-uploaded.
struct DevCluster {
  int32_t n, n_scalar, n_label_cols, n_taints;
  int32_t n_label_values, _pad[3];
  const int64_t* alloc_cpu;
  const int64_t* alloc_mem;
  const int64_t* alloc_eph;
  const int32_t* alloc_pods;
  const int64_t* alloc_scalar;   // [n_scalar][n]
  int64_t* req_cpu;
  int64_t* req_mem;
  int64_t* req_eph;
  int64_t* req_scalar;           // [n_scalar][n]
  int64_t* nz_cpu;
  int64_t* nz_mem;
  int32_t* num_pods;
  const uint32_t* flags;
  const uint16_t* taints;        // [KSIM_MAX_NODE_TAINTS][n]
  const uint32_t* labels;        // [n_label_cols][n]
  const uint8_t* taint_effect;
  const int32_t* label_col_offset;
  const int64_t* label_num;
  const uint8_t* label_num_ok;
};

struct DevPods {
  const ksim_pod* pods;
  const ksim_label_expr* exprs;
  const ksim_term* terms;
  int32_t n_pods, n_exprs, n_terms, _pad;
};

// Scheduler state that survives across cycles (sched.nextStartNodeIndex,
// the tie-break sequence) plus the run cursor and counters.
struct DevState {
  int32_t cursor;        // pod index of the next cycle
  int32_t end;           // one past the last pod of the current run
  int32_t next_start;    // nextStartNodeIndex
  int32_t _pad0;
  int64_t pod_seq;       // tie-break sequence (one per cycle)
  int64_t evals;         // pod x node filter evaluations
  int64_t scheduled;
  int64_t unschedulable;
  // scalars of the last cycle
  int32_t chosen, status, n_feasible, n_evaluated, n_processed, k_to_find, next_start_after, _pad1;
};

// Per-cycle scratch written by the filter/score kernel, read by finalize.
struct DevScratch {
  uint8_t* fail;         // [n] filter-order index of first failure or KSIM_PASSED
  uint32_t* detail;      // [n]
  int64_t* raw;          // [KSIM_MAX_SCORE][n] raw scores (normalized slots; all in compat)
  int64_t* part;         // [n] sum of weighted raw of slots without NormalizeScore
};

// Compat-mode outputs (ksim_eval_out), device copies.
struct DevEvalOut {
  uint8_t* scored;       // [n]
  int64_t* raw;          // [S][n]
  int64_t* norm;         // [S][n]
  int64_t* total;        // [n]
};

// Normalization kind of a score slot.
enum NormKind : int32_t { kNormNone = 0, kNormDefault = 1, kNormDefaultReverse = 2, kNormPTS = 3, kNormIPA = 4 };

__host__ __device__ inline int32_t norm_kind(int plugin) {
  switch (plugin) {
    case KSIM_PL_TAINT_TOLERATION: return kNormDefaultReverse;
    case KSIM_PL_NODE_AFFINITY: return kNormDefault;
    case KSIM_PL_POD_TOPOLOGY_SPREAD: return kNormPTS;
    case KSIM_PL_INTER_POD_AFFINITY: return kNormIPA;
    default: return kNormNone;
  }
}

// [upstream] schedule_one.go numFeasibleNodesToFind
__host__ __device__ inline int32_t num_feasible_nodes_to_find(int32_t pct, int32_t n) {
  if (n < 100 || pct >= 100) return n;
  int32_t a = pct;
  if (a <= 0) {
    a = 50 - n / 125;
    if (a < 5) a = 5;
  }
  int32_t k = n * a / 100;
  return k < 100 ? 100 : k;
}

__host__ __device__ inline uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// selectHost tie-break TB(seed): a single u64 max over (total, hash, node).
__host__ __device__ inline uint64_t tb_key(int64_t total, uint64_t seed, int64_t seq, int32_t node) {
  uint64_t h = splitmix64(seed ^ ((uint64_t)seq << 20) ^ (uint64_t)(uint32_t)node) >> 38;
  return ((uint64_t)total << 44) | (h << 18) | (uint64_t)((KSIM_MAX_NODES - 1) - node);
}

__device__ __forceinline__ int bit_set(const uint64_t* w, uint32_t id) {
  return (int)((w[id >> 6] >> (id & 63)) & 1ull);
}

// labels.Requirement.Matches / metadata.name field selector
__device__ inline bool label_req_matches(const DevCluster& c, const ksim_label_expr& e, int32_t node) {
  const uint8_t op = e.op;
  uint32_t v = 0;
  if (op <= KSIM_OP_LT) v = c.labels[(size_t)e.col * c.n + node];
  switch (op) {
    case KSIM_OP_IN: {
      if (!v) return false;
      for (int k = 0; k < e.nvals; k++) if (e.vals[k] == v) return true;
      return false;
    }
    case KSIM_OP_NOT_IN: {
      if (!v) return true;
      for (int k = 0; k < e.nvals; k++) if (e.vals[k] == v) return false;
      return true;
    }
    case KSIM_OP_EXISTS: return v != 0;
    case KSIM_OP_DOES_NOT_EXIST: return v == 0;
    case KSIM_OP_GT:
    case KSIM_OP_LT: {
      if (!v) return false;
      int32_t idx = c.label_col_offset[e.col] + (int32_t)v;
      if (idx < 0 || idx >= c.n_label_values || !c.label_num_ok[idx]) return false;
      return op == KSIM_OP_GT ? (c.label_num[idx] > e.num) : (c.label_num[idx] < e.num);
    }
    case KSIM_OP_FIELD_IN: {
      for (int k = 0; k < e.nvals; k++) if ((int32_t)e.vals[k] == node) return true;
      return false;
    }
    case KSIM_OP_FIELD_NOT_IN: {
      for (int k = 0; k < e.nvals; k++) if ((int32_t)e.vals[k] == node) return false;
      return true;
    }
    case KSIM_OP_TRUE: return true;
    default: return false;
  }
}

__device__ inline bool term_matches(const DevCluster& c, const DevPods& P, const ksim_term& t, int32_t node) {
  if (t.n_expr <= 0) return false;
  for (int i = 0; i < t.n_expr; i++)
    if (!label_req_matches(c, P.exprs[t.first_expr + i], node)) return false;
  return true;
}

// nodeaffinity RequiredNodeAffinity.Match
__device__ inline bool required_node_affinity_match(const DevCluster& c, const DevPods& P,
                                                    const ksim_pod& p, int32_t node) {
  for (int i = 0; i < p.sel_count; i++)
    if (!label_req_matches(c, P.exprs[p.sel_first + i], node)) return false;
  if (p.flags & KSIM_POD_HAS_REQUIRED_AFFINITY) {
    for (int i = 0; i < p.req_term_count; i++)
      if (term_matches(c, P, P.terms[p.req_term_first + i], node)) return true;
    return false;
  }
  return true;
}

// nodeaffinity PreferredSchedulingTerms.Score
__device__ inline int64_t preferred_node_affinity_score(const DevCluster& c, const DevPods& P,
                                                        const ksim_pod& p, int32_t node) {
  int64_t count = 0;
  for (int i = 0; i < p.pref_term_count; i++) {
    const ksim_term& t = P.terms[p.pref_term_first + i];
    if (t.weight == 0) continue;
    if (term_matches(c, P, t, node)) count += t.weight;
  }
  return count;
}

// v1helper.FindMatchingUntoleratedTaint (NoSchedule|NoExecute)
__device__ inline uint32_t find_matching_untolerated_taint(const DevCluster& c, const ksim_pod& p, int32_t node) {
  for (int k = 0; k < KSIM_MAX_NODE_TAINTS; k++) {
    uint32_t tid = c.taints[(size_t)k * c.n + node];
    if (!tid) break;
    uint8_t eff = c.taint_effect[tid];
    if ((eff == KSIM_EFFECT_NO_SCHEDULE || eff == KSIM_EFFECT_NO_EXECUTE) && !bit_set(p.tol_filter, tid))
      return tid;
  }
  return 0;
}

// tainttoleration countIntolerableTaintsPreferNoSchedule
__device__ inline int64_t count_intolerable_prefer(const DevCluster& c, const ksim_pod& p, int32_t node) {
  int64_t n = 0;
  for (int k = 0; k < KSIM_MAX_NODE_TAINTS; k++) {
    uint32_t tid = c.taints[(size_t)k * c.n + node];
    if (!tid) break;
    if (c.taint_effect[tid] != KSIM_EFFECT_PREFER_NO_SCHEDULE) continue;
    if (!bit_set(p.tol_prefer, tid)) n++;
  }
  return n;
}

// noderesources fitsRequest -> reason bits
__device__ inline uint32_t fits_request(const DevCluster& c, const ksim_pod& p, int32_t node) {
  uint32_t r = 0;
  if (c.num_pods[node] + 1 > c.alloc_pods[node]) r |= KSIM_FIT_TOO_MANY_PODS;
  if (p.req_cpu == 0 && p.req_mem == 0 && p.req_eph == 0 && !(p.flags & KSIM_POD_HAS_SCALAR)) return r;
  if (p.req_cpu > c.alloc_cpu[node] - c.req_cpu[node]) r |= KSIM_FIT_CPU;
  if (p.req_mem > c.alloc_mem[node] - c.req_mem[node]) r |= KSIM_FIT_MEMORY;
  if (p.req_eph > c.alloc_eph[node] - c.req_eph[node]) r |= KSIM_FIT_EPHEMERAL;
  for (int k = 0; k < c.n_scalar; k++) {
    int64_t q = p.scalar_req[k];
    if (q == 0) continue;
    size_t ix = (size_t)k * c.n + node;
    if (q > c.alloc_scalar[ix] - c.req_scalar[ix]) r |= (KSIM_FIT_SCALAR0 << k);
  }
  return r;
}

// resourceAllocationScorer.calculateResourceAllocatableRequest
__device__ inline void calc_alloc_req(const DevCluster& c, const ksim_pod& p, int32_t node, int32_t res,
                                      bool use_requested, int64_t& alloc, int64_t& req) {
  alloc = 0;
  req = 0;
  if (res == KSIM_RES_CPU) {
    alloc = c.alloc_cpu[node];
    req = (use_requested ? c.req_cpu[node] : c.nz_cpu[node]) + (use_requested ? p.req_cpu : p.nz_cpu);
  } else if (res == KSIM_RES_MEMORY) {
    alloc = c.alloc_mem[node];
    req = (use_requested ? c.req_mem[node] : c.nz_mem[node]) + (use_requested ? p.req_mem : p.nz_mem);
  } else if (res == KSIM_RES_EPHEMERAL) {
    alloc = c.alloc_eph[node];
    req = c.req_eph[node] + p.req_eph;
  } else {
    int k = res - KSIM_RES_SCALAR0;
    if (k < 0 || k >= c.n_scalar) return;
    int64_t pr = p.scalar_req[k];
    if (pr == 0) return;
    size_t ix = (size_t)k * c.n + node;
    alloc = c.alloc_scalar[ix];
    req = c.req_scalar[ix] + pr;
  }
}

// least_allocated.go leastRequestedScore
__device__ __forceinline__ int64_t least_requested_score(int64_t requested, int64_t capacity) {
  if (capacity == 0) return 0;
  if (requested > capacity) return 0;
  return ((capacity - requested) * kMaxNodeScore) / capacity;
}

__device__ inline int64_t fit_least_allocated_score(const DevCluster& c, const ksim_profile& prof,
                                                    const ksim_pod& p, int32_t node) {
  int64_t node_score = 0, weight_sum = 0;
  for (int i = 0; i < prof.fit_n_res; i++) {
    int64_t a, r;
    calc_alloc_req(c, p, node, prof.fit_res[i], false, a, r);
    if (a == 0) continue;
    node_score += least_requested_score(r, a) * prof.fit_res_weight[i];
    weight_sum += prof.fit_res_weight[i];
  }
  if (weight_sum == 0) return 0;
  return node_score / weight_sum;
}

// balanced_allocation.go balancedResourceScorer (float64, unfused)
__device__ inline int64_t balanced_allocation_score(const DevCluster& c, const ksim_profile& prof,
                                                    const ksim_pod& p, int32_t node) {
  double fr[KSIM_MAX_RES];
  int nf = 0;
  double total = 0;
  for (int i = 0; i < prof.ba_n_res && i < KSIM_MAX_RES; i++) {
    int64_t a, r;
    calc_alloc_req(c, p, node, prof.ba_res[i], true, a, r);
    if (a == 0) continue;
    double f = (double)r / (double)a;
    if (f > 1) f = 1;
    total += f;
    fr[nf++] = f;
  }
  double std = 0.0;
  if (nf == 2) {
    std = fabs((fr[0] - fr[1]) / 2);
  } else if (nf > 2) {
    double mean = total / (double)nf;
    double sum = 0;
    for (int i = 0; i < nf; i++) sum = sum + (fr[i] - mean) * (fr[i] - mean);
    std = sqrt(sum / (double)nf);
  }
  return (int64_t)((1 - std) * (double)kMaxNodeScore);
}

// frameworkImpl.RunFilterPlugins (stop at first failure)
__device__ inline uint8_t run_filter_plugins(const DevCluster& c, const DevPods& P, const ksim_profile& prof,
                                             const ksim_pod& p, int32_t node, uint32_t& detail) {
  detail = 0;
  for (int f = 0; f < prof.n_filter; f++) {
    switch (prof.filter[f]) {
      case KSIM_PL_NODE_UNSCHEDULABLE:
        if ((c.flags[node] & KSIM_NODE_UNSCHEDULABLE) && !(p.flags & KSIM_POD_TOLERATES_UNSCHEDULABLE))
          return (uint8_t)f;
        break;
      case KSIM_PL_NODE_NAME:
        if (p.node_name != -1 && p.node_name != node) return (uint8_t)f;
        break;
      case KSIM_PL_TAINT_TOLERATION: {
        uint32_t tid = find_matching_untolerated_taint(c, p, node);
        if (tid) { detail = tid; return (uint8_t)f; }
        break;
      }
      case KSIM_PL_NODE_AFFINITY:
        if (!required_node_affinity_match(c, P, p, node)) return (uint8_t)f;
        break;
      case KSIM_PL_NODE_RESOURCES_FIT: {
        uint32_t r = fits_request(c, p, node);
        if (r) { detail = r; return (uint8_t)f; }
        break;
      }
      default:
        break;
    }
  }
  return KSIM_PASSED;
}

__device__ inline int64_t score_plugin_raw(const DevCluster& c, const DevPods& P, const ksim_profile& prof,
                                           const ksim_pod& p, int plugin, int32_t node) {
  switch (plugin) {
    case KSIM_PL_NODE_RESOURCES_FIT: return fit_least_allocated_score(c, prof, p, node);
    case KSIM_PL_BALANCED_ALLOCATION: return balanced_allocation_score(c, prof, p, node);
    case KSIM_PL_TAINT_TOLERATION: return count_intolerable_prefer(c, p, node);
    case KSIM_PL_NODE_AFFINITY: return preferred_node_affinity_score(c, P, p, node);
    default: return 0;   // ImageLocality (no images), PTS/IPA without constraints/terms
  }
}

__device__ inline void assume_pod(const DevCluster& c, const ksim_pod& p, int32_t node, int sign) {
  c.req_cpu[node] += sign * p.req_cpu;
  c.req_mem[node] += sign * p.req_mem;
  c.req_eph[node] += sign * p.req_eph;
  for (int k = 0; k < c.n_scalar; k++) c.req_scalar[(size_t)k * c.n + node] += sign * p.scalar_req[k];
  c.nz_cpu[node] += sign * p.nz_cpu;
  c.nz_mem[node] += sign * p.nz_mem;
  c.num_pods[node] += sign;
}

}  // namespace ksim
