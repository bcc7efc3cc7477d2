// ksim_device.h — device-side data layout and plugin arithmetic (gfx950).
//
// Each __device__ function restates the same upstream v1.26.2 function as the
// CPU oracle (oracle/ksim_oracle.c) does; the HIP kernels in ksim_kernels.hip
// compose them.  Compiled with -ffp-contract=off and no fast-math so float64
// division / sqrt are IEEE correctly rounded and nothing is fused (Go on
// GOAMD64=v1 never fuses), which makes BalancedAllocation bit-exact.
//
// The per-node arithmetic works on a NodeRow held in registers: the node's
// NodeInfo aggregates, loaded once from the HBM columns (or from an LDS slot
// in the batch repair kernel), so one evaluation never re-reads a field.
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
  // node sharding: this snapshot holds global positions [base, base + n) of
  // n_total nodes.  Memory is indexed by the LOCAL position; tie-break keys,
  // spec.nodeName and metadata.name field selectors use the GLOBAL one.
  int32_t n_label_values, n_prefer_taints, base, n_total;
  // the nodes k_batch_top evaluates (local positions [eval_lo, eval_hi)): all
  // of them, except on replicated handles (ksim_set_eval_range), which hold
  // every node and evaluate one range of them
  int32_t eval_lo, eval_hi;
  // 0 on a replica that is not its group's first (rank 0): the runs every
  // replica executes whole (per-pod cycles, ADAPT batches) are counted in the
  // evaluation statistics once, by the first replica
  int32_t count_whole;
  // NodeResourcesFitArgs ignoredResources / ignoredResourceGroups (ksim_profile
  // fit_ignored_scalar): bit k = Fit's Filter skips scalar column k
  uint32_t fit_ignore;
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
  // PodTopologySpread / InterPodAffinity count classes (ksim_engine.h "Count classes")
  int32_t n_classes, n_topo_log, vmax;
  uint32_t cflags;               // kCluster*: facts the per-pod filter plan uses
  int32_t* cnt;                  // [n_classes][n], updated by every bind
  const double* topo_log;        // [n_topo_log] = log(size + 2), host-computed
  const int32_t* col_nvals;      // [n_label_cols] value ids per column (domain table sizes)
  const uint8_t* col_unique;     // [n_label_cols] every value on at most one node (e.g. hostname);
                                 // all zero on shard handles
  // NetworkBandwidth (milli-units): the node-limit annotation and the bound
  // pods' request annotations (getNodeAllocatedAmount), updated by every bind
  const int64_t* nb_limit;
  int64_t* nb_alloc;
  // RN(1 / allocatable) of cpu and memory (0 for allocatable 0), host-computed:
  // the FAST batch kernels divide by them (div_rn)
  const double* inv_cpu;
  const double* inv_mem;
};

// DevCluster.cflags
constexpr uint32_t kClusterUnschedulable = 1u;   // some node has spec.unschedulable
constexpr uint32_t kClusterHardTaints = 2u;      // some node has a NoSchedule / NoExecute taint
constexpr uint32_t kClusterPreferTaints = 4u;    // some node has a PreferNoSchedule taint
constexpr uint32_t kClusterNarrow = 8u;          // every allocatable cpu / memory in [0, 2^46) (fast quotients)

struct PodPlan;

struct DevPods {
  const ksim_pod* pods;
  const ksim_label_expr* exprs;
  const ksim_term* terms;
  const int32_t* nn;             // PreFilterResult.NodeNames positions (KSIM_POD_NODE_NAMES), sorted per pod
  const int32_t* bflags;         // [n_pods] batch path: kBatch* flags
  const ksim_topo_use* uses;
  const ksim_class_add* adds;
  const PodPlan* plans;          // [n_pods] per-pod cycle plans (host-compiled, see PodPlan)
  // Persistent domain tables: for the (count class, key column)
  // pairs the queue's topology uses read, the class's domain sums over the
  // column's values, built once per queue / reset (k_ptab_init) and kept by
  // every bind (ptab_add), so a pod whose plan carries kPlanPtab needs no
  // per-cycle PreFilter pass.  Null on shard handles.
  int64_t* ptab;                 // table entries; a use's table starts at its device copy's _pad
  const int4* ptab_ent;          // [n_ptab] {class, column, kind (kPtab*), first entry}
  const int32_t* ptab_cfirst;    // [n_classes + 1] the tables of each class: ptab_cidx[cfirst[c] .. cfirst[c+1])
  const int32_t* ptab_cidx;
  const int4* ptab_padd;         // per pod (PodPlan.tadd_*): {first entry, column, kind, count} of
                                 // every table its adds change, so a bind skips the class lookup
  int32_t n_pods, n_exprs, n_terms, n_uses, n_adds, n_nn, n_ptab, _pad;
  // Static classes (P100 batch keys of non-trivial and kPodNormVaries pods):
  // pods whose static-filter and normalized-score inputs are identical share a
  // class; stab[cls][node] holds the class's static verdict on the node and
  // its two raw normalized scores (stab_word).  Null: no table (the keys
  // evaluate every static plugin per node).  stab_fast: the handle meets
  // run_fast's cluster conditions, so the keys take the FAST arithmetic.
  const int32_t* sclass = nullptr;   // [n_pods] class or -1
  const uint64_t* stab = nullptr;    // [n_classes][c.n]
  int32_t stab_fast = 0, _pad2 = 0;
};

// A static-table word: bit 63 every static filter passes; bits 32..62
// countIntolerableTaintsPreferNoSchedule; bit k < 32: the pod's preferred
// node-affinity term k (weight != 0) matches the node.  The weights stay
// with the pod (a class is the terms' expressions, so pods that differ only
// in weights share it); stab_raw sums them.  The host admits a class only
// with at most 32 preferred terms, all weights >= 0.
__host__ __device__ __forceinline__ uint64_t stab_word(bool pass, int64_t tt, uint32_t match) {
  return (pass ? (1ull << 63) : 0ull) | ((uint64_t)(tt & 0x7fffffff) << 32) | (uint64_t)match;
}
__host__ __device__ __forceinline__ bool stab_pass(uint64_t w) { return (w >> 63) != 0; }

// Persistent table kinds (DevPods.ptab_ent .z)
constexpr int32_t kPtabPlain = 0;    // sum[v] = class count over the nodes with value v
constexpr int32_t kPtabMark = 1;     // plus one kDomMarkShift marker per node with value v (PTS hard)
constexpr int32_t kPtabTotal = 2;    // one entry: the class count over every node carrying the key

// Scheduler state that survives across cycles (sched.nextStartNodeIndex,
// the tie-break sequence) plus the run cursor and counters.
struct DevState {
  int32_t cursor;        // pod index of the next cycle
  int32_t end;           // one past the last pod of the current run
  int32_t next_start;    // nextStartNodeIndex
  int32_t truncations;   // batch path: batches cut short by an exhausted candidate list
  int64_t pod_seq;       // tie-break sequence (one per cycle)
  int64_t evals;         // pod x node filter evaluations
  int64_t scheduled;
  int64_t unschedulable;
  // scalars of the last cycle
  int32_t chosen, status, n_feasible, n_evaluated, n_processed, k_to_find, next_start_after, batches;
  // batch path: batches ended early because a pod's best node was one bound
  // earlier in the batch (its guess was not its exact choice)
  int64_t cuts;
  // per-pod topology flags of the current cycle (kTopo*), reset by k_bind
  uint32_t topo_flags;
  // generic ADAPT batches: the next batch's pod cap (0: the full batch), set
  // by k_adapt_commit from the last batch's committed pods, reset by set_run
  int32_t bcap;
};

// DevState.topo_flags
constexpr uint32_t kTopoAffinityNonEmpty = 1u;   // len(state.affinityCounts) > 0
constexpr uint32_t kTopoScoreNonEmpty = 2u;      // len(state.topologyScore) > 0

// PTS hard: a domain entry carries its pods in the low bits and one marker per
// eligible node above them (TpPairToMatchNum has the pair iff a marker is set).
constexpr int kDomMarkShift = 40;
constexpr int64_t kDomCountMask = (1ll << kDomMarkShift) - 1;

struct BRow;

// Topology batch zone variants (ksim_tbatch.hip): a pod whose one
// DoNotSchedule spread key has at most kVarDom domains is evaluated per
// feasible-domain set its batch can reach.  An earlier pod of the batch that
// adds to the constraint's count class (its adder) moves one domain's count by
// where it lands; each landing domain (or none) gives a set of domains whose
// skew passes, and each distinct set is a slot with its own normalization,
// top-T list and pair keys.  The chain takes the slot its adder's guess names.
constexpr int kVarDom = 4;
constexpr int kVarSlots = kVarDom + 1;
struct TbVar {
  int32_t use;                     // the variant use (-1: the pod's plain S0 path)
  int32_t adder;                   // batch index of the one earlier pod adding its class (-1: none, or several)
  int32_t nslot;                   // slots (1 without an adder)
  int32_t ndom;                    // domains of the key (value ids 1 .. ndom)
  int32_t col;                     // the key column
  int32_t vcol;                    // the run's variant column (PodPlan kPlanVcolShift of its first pod; -1: none)
  uint32_t zmask;                  // score slots constant 0 for the pod (k_tb_filter)
  int32_t slot_of[kVarSlots];      // slot by the adder's landing domain (0: it moves no count)
  uint32_t mask[kVarSlots];        // feasible domains per slot (bit d - 1)
};
struct TbDom {                     // per (pod, domain): nodes passing every filter but the variant skew
  int32_t nfeas, nign;
  uint64_t ext[2 * KSIM_MAX_SCORE];
};

// Selection state of one per-pod cycle (k_window -> k_extrema -> k_select -> k_bind).
// ext[kExtCut] (sharded cycles): 1 + the scan position of the cut node on the
// shard that holds it, 0 elsewhere; all-reduced (max) together with the extrema.
constexpr int kExtCut = 2 * KSIM_MAX_SCORE;
constexpr int kExtWords = kExtCut + 1;
struct WinState {
  int32_t cut, kend, nf, evaluated, k, has_soft;
  int32_t nfeas, nign;                   // no-window cycles (K = N): counted by k_filter_score
  int32_t error;                         // kCycleError*: the cycle fails with framework.Error
  int32_t nscan;                         // nodes the cycle scans (ScanSet.n): nextStartNodeIndex modulus
  double w[KSIM_MAX_USES];               // PTS soft: topologyNormalizingWeight per use
  uint64_t ext[kExtWords];               // per score slot: max image, min image (atomicMax); cut
  int32_t done;                          // k_select blocks finished (the last one binds; reset by it)
  uint32_t tflags;                       // topology batch: the pod's kTopo* flags (k_tb_filter block 0)
  int32_t hold[2 * KSIM_MAX_SCORE];      // topology batch: nodes holding each slot's max / min (k_tb_select)
};

// The nodes one cycle scans, in scan order: every node of
// the cluster in nodeTree order from nextStartNodeIndex, or only NodeAffinity's
// PreFilterResult.NodeNames (KSIM_POD_NODE_NAMES; [upstream] findNodesThatFitPod
// then scans that list from nextStartNodeIndex mod its length and advances
// nextStartNodeIndex mod its length).  Positions are global (sharded handles
// scan the whole cluster's order).
struct ScanSet {
  const int32_t* list;   // sorted global positions; nullptr: every one of n nodes
  int32_t n;             // scan length (0: PreFilter rejected the pod, nothing is scanned)
  int32_t start;         // first scan position's index (nextStartNodeIndex mod n)
};

__device__ __forceinline__ ScanSet scan_set(const DevCluster& c, const DevPods& P, const ksim_pod& p,
                                            int32_t next_start) {
  ScanSet s;
  if (p.flags & KSIM_POD_NODE_NAMES) {
    s.list = P.nn + p.nn_first;
    s.n = (p.flags & KSIM_POD_NODE_NAMES_UNKNOWN) ? 0 : p.nn_count;
  } else {
    s.list = nullptr;
    s.n = c.n_total;
  }
  s.start = s.n > 0 ? next_start % s.n : 0;
  return s;
}

// Global position of scan position r (0 <= r < s.n).
__device__ __forceinline__ int32_t scan_node(const ScanSet& s, int32_t r) {
  int32_t x = s.start + r;
  if (x >= s.n) x -= s.n;
  return s.list ? s.list[x] : x;
}

// Scan position of global node g, or -1 when the cycle does not scan it.
__device__ __forceinline__ int32_t scan_pos(const ScanSet& s, int32_t g) {
  int32_t idx = g;
  if (s.list) {
    int32_t lo = 0, hi = s.n;                      // lower_bound over the sorted list
    while (lo < hi) {
      const int32_t mid = (lo + hi) >> 1;
      if (s.list[mid] < g) lo = mid + 1;
      else hi = mid;
    }
    if (lo >= s.n || s.list[lo] != g) return -1;
    idx = lo;
  } else if (s.n == 0) {
    return -1;
  }
  const int32_t r = idx - s.start;
  return r < 0 ? r + s.n : r;
}

// Per-cycle scratch written by the filter/score kernel, read by the selection.
struct DevScratch {
  uint8_t* fail;         // [n] filter-order index of first failure or KSIM_PASSED
  uint8_t* ign;          // [n] feasible node missing a ScheduleAnyway spread key (IgnoredNodes)
  WinState* win;
  uint64_t* bbest;       // [2 * blocks] k_select: each block's best (max image of the total, TB lo word)
  uint64_t* amask;       // ADAPT batch: S0 feasibility bitmaps [kBatchPods][ceil(n / 64)]
  int32_t* awin;         // ADAPT batch: per pod {scan start, cut offset or -1}
  int32_t* aexact;       // ADAPT batch: pods whose windows are exact
  int32_t* acut;         // ADAPT batch: k_adapt_cut0's first-round {start, cut} per pod
  uint16_t* wtab;        // ADAPT windows by doubling (n <= 8192): [2][kBatchPods][n] start -> next-start tables
  int32_t* wtot;         // ADAPT windows by doubling: [kBatchPods] feasible nodes per pod
  int32_t* abroken;      // ADAPT batch: a bound node flipped feasibility inside the pod's window
  const uint8_t* ext_fail;   // extender pass only (else null): nodes an extender filtered out
  const int64_t* ext_score;  // extender pass only (else null): the extenders' combined scores
  uint32_t* regbm;       // no-window cycles: PTS pair registration bitmaps [KSIM_MAX_USES][(vmax + 31) / 32]
  int64_t* xdom;         // sharded cycle: packed domain sums (all-reduced, sum)
  int64_t* xreg;         // sharded cycle: IgnoredNodes count + per-value registrations (all-reduced, sum)
  uint32_t* detail;      // [n]
  int64_t* raw;          // [KSIM_MAX_SCORE][n] raw scores (normalized slots; all in compat)
  int64_t* part;         // [n] sum of weighted raw of slots without NormalizeScore
  uint64_t* topk;        // batch path: [B][T] merged top keys, descending
  int32_t* topk_cnt;     // batch path: [B] valid merged keys
  int32_t* topk_complete;// batch path: [B] 1 if every S0-feasible node is in the list
  uint64_t* gkey;        // batch path: [B] key of each pod's greedy guess (0: none)
  int32_t* chain_end;    // batch path: pods covered by the chain (an exhausted list cuts it)
  uint64_t* pmax;        // batch path: [B] best key of pod j over the guesses of pods k < j
  int64_t* pnorm;        // batch path: [B][4] kPodNormVaries pods' S0 maxima (TaintToleration, NodeAffinity raw)
                         // and the S0-feasible nodes holding each
  // topology batch path (ksim_tbatch.hip), per pod j of the batch: [kTbPods][n] slices
  uint8_t* tb_fail;      // filter result per node
  uint8_t* tb_ign;       // PodTopologySpread IgnoredNodes
  int64_t* tb_part;      // weighted raw scores of the slots without NormalizeScore
  int64_t* tb_raw;       // [kTbPods][KSIM_MAX_SCORE][n] raw scores
  int32_t* tb_stat;      // total - (w_fit LeastAllocated + w_ba BalancedAllocation) at S0; kStatNone / kStatOne
  WinState* tb_win;      // [kTbPods] counters, extrema, flags
  TbVar* tb_var;         // [kTbPods] zone variants of the pod (k_tb_filter block 0)
  TbDom* tb_dom;         // [kTbPods][kVarDom] variant pods: counters and extrema per domain of the variant key
  int32_t* tb_vhold;     // [kTbPods][kVarSlots][2 * KSIM_MAX_SCORE] variant pods: extremum holders per slot
  int32_t* tb_slot;      // [kTbPods] the slot the chain took per pod (k_tb_chain_pairs block 0)
  uint8_t* tb_vdom;      // [kTbPods][n] value ids: the pod's variant key (low nibble), the run's variant column (high)
  uint8_t* tb_cdom;      // [kTbPods][kVarSlots][kTbMaxBlocks][T] the block lists' run-column value ids
  uint8_t* tb_kdom;      // [kTbPods][kVarSlots][T] the merged lists' run-column value ids (the chain's slot map)
  int32_t* tb_vnf;       // [kTbPods][kVarSlots] feasible nodes per slot (k_tb_select block 0)
  unsigned long long* tb_vpods;   // [1] committed pods whose zone verdicts moved inside their batch (ksim_get_diag)
  uint64_t* tb_clist;    // [kTbPods][kTbMaxBlocks][T] each node block's exact top-T keys
  int32_t* tb_ccnt;      // [kTbPods][kTbMaxBlocks] their counts
  uint8_t* tb_xrecv;     // replicated topology batches: [world][kTbPods] WinState (the filter's counters)
  uint64_t* tb_pp;       // replicated topology batches: [2][kTbPods] pair maxima, pinv (all-reduced max)
  int32_t* pinv;         // batch path: [B] 1 = a maximum holder of pod j left its feasible set (batch ends before j)
  unsigned long long* dbg;   // [16] diagnostic accumulators (ksim_get_diag), e.g. chain phase times
  // framework-driven filter pass (ksim_fw_prefilter), pods without topology
  // uses: the answers written straight to the host's pinned staging (device
  // addresses; else null): next_start and a too-wide flag, the codes, the
  // details, each feasible node's row [n][S + 1] of its raw scores and
  // weighted part as int32 (one cache line per node for the host's reads)
  int32_t* m_head;
  uint8_t* m_fail;
  uint32_t* m_detail;
  int32_t* m_raw;
  uint64_t* xsend;       // sharded: [kBatchPods][kXRec] this shard's candidate records
  uint64_t* xrecv;       // sharded: [world][kBatchPods][kXRec] all shards' records
  int64_t* dom;          // [KSIM_MAX_USES][vmax] topology-pair sums of the current pod (zero between pods)
  int64_t* min_match;    // [KSIM_MAX_USES] PTS hard: critical-path minimum
};

// Compat-mode outputs (ksim_eval_out), device copies.
struct DevEvalOut {
  uint8_t* scored;       // [n]
  int64_t* raw;          // [S][n]
  int64_t* norm;         // [S][n]
  int64_t* total;        // [n]
};

// Normalization kind of a score slot.
enum NormKind : int32_t {
  kNormNone = 0, kNormDefault = 1, kNormDefaultReverse = 2, kNormPTS = 3, kNormIPA = 4,
  kNormMinMax = 5   // NetworkBandwidth: IPA's min-max form without the empty-state shortcut
};

__host__ __device__ __forceinline__ int32_t norm_kind(int plugin) {
  switch (plugin) {
    case KSIM_PL_TAINT_TOLERATION: return kNormDefaultReverse;
    case KSIM_PL_NODE_AFFINITY: return kNormDefault;
    case KSIM_PL_POD_TOPOLOGY_SPREAD: return kNormPTS;
    case KSIM_PL_INTER_POD_AFFINITY: return kNormIPA;
    case KSIM_PL_NETWORK_BANDWIDTH: return kNormMinMax;
    default: return kNormNone;
  }
}

// [upstream] schedule_one.go numFeasibleNodesToFind
__host__ __device__ __forceinline__ int32_t num_feasible_nodes_to_find(int32_t pct, int32_t n) {
  if (n < 100 || pct >= 100) return n;
  int32_t a = pct;
  if (a <= 0) {
    a = 50 - n / 125;
    if (a < 5) a = 5;
  }
  int32_t k = n * a / 100;
  return k < 100 ? 100 : k;
}

__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// selectHost tie-break TB(seed): the max of (total, hash26, node) in
// lexicographic order, total a full int64.  lo = hash26 << 18 | (mask - node)
// is the tie-break word; node < KSIM_MAX_NODES = KSIM_KEY_NODE_MASK keeps its
// low field >= 1, so a valid lo is never 0.
__host__ __device__ __forceinline__ uint64_t tb_lo(uint64_t seed, int64_t seq, int32_t node) {
  const uint64_t h = splitmix64(seed ^ ((uint64_t)seq << 20) ^ (uint64_t)(uint32_t)node) >> 38;
  return (h << 18) | (uint64_t)(KSIM_KEY_NODE_MASK - node);
}
// One-word key for a total known to lie in [0, 2^20) (kKeyTotalLimit): the
// batch paths key a pod's nodes by total minus a per-pod constant, which the
// host proves fits (pod_batchable); the order is the same as (total, lo).
constexpr int64_t kKeyTotalLimit = 1ll << 20;
__host__ __device__ __forceinline__ uint64_t tb_key(int64_t total, uint64_t seed, int64_t seq, int32_t node) {
  return ((uint64_t)total << 44) | tb_lo(seed, seq, node);
}
__host__ __device__ __forceinline__ int32_t key_node(uint64_t key) {
  return (int32_t)(KSIM_KEY_NODE_MASK - (int32_t)(key & KSIM_KEY_NODE_MASK));
}
// Order-preserving u64 image of an int64 (max image), so (total, lo) pairs
// compare as two u64 words; 0 is below every image of a real total > INT64_MIN.
__host__ __device__ __forceinline__ uint64_t max_image(int64_t x) { return (uint64_t)x ^ (1ull << 63); }
__host__ __device__ __forceinline__ int64_t from_max_image(uint64_t m) { return (int64_t)(m ^ (1ull << 63)); }
// Min image: order-reversing, so an atomicMax over images takes the minimum.
__host__ __device__ __forceinline__ uint64_t min_image(int64_t x) { return ~((uint64_t)x ^ (1ull << 63)); }
__host__ __device__ __forceinline__ int64_t from_min_image(uint64_t m) { return (int64_t)(~m ^ (1ull << 63)); }

// NodeInfo aggregates of one node, in registers.
struct NodeRow {
  int64_t alloc_cpu, alloc_mem, alloc_eph;
  int64_t req_cpu, req_mem, req_eph;
  int64_t nz_cpu, nz_mem;
  int64_t alloc_sc[KSIM_MAX_SCALAR], req_sc[KSIM_MAX_SCALAR];
  int32_t alloc_pods, num_pods;
  uint32_t flags;
  int32_t node;
  uint32_t taints[KSIM_MAX_NODE_TAINTS / 2];   // taint ids, two u16 per word, node.Spec.Taints order
};

__device__ __forceinline__ uint32_t row_taint(const NodeRow& r, int k) {
  return (r.taints[k >> 1] >> ((k & 1) * 16)) & 0xffffu;
}

// The resource columns only (what a batchable pod's Fit filter and scores
// read when its static filters are host-proven to pass): 10 loads, not 27.
__device__ __forceinline__ NodeRow load_res_row(const DevCluster& c, int32_t node) {
  NodeRow r;
  r.node = node;
  r.alloc_cpu = c.alloc_cpu[node];
  r.alloc_mem = c.alloc_mem[node];
  r.alloc_eph = c.alloc_eph[node];
  r.req_cpu = c.req_cpu[node];
  r.req_mem = c.req_mem[node];
  r.req_eph = c.req_eph[node];
  r.nz_cpu = c.nz_cpu[node];
  r.nz_mem = c.nz_mem[node];
  r.alloc_pods = c.alloc_pods[node];
  r.num_pods = c.num_pods[node];
  r.flags = 0;
#pragma unroll
  for (int k = 0; k < KSIM_MAX_SCALAR; k++) r.alloc_sc[k] = r.req_sc[k] = 0;
#pragma unroll
  for (int k = 0; k < KSIM_MAX_NODE_TAINTS / 2; k++) r.taints[k] = 0;
  return r;
}

// load_res_row by 32-bit byte offsets from the column bases (one shift per
// element size instead of a 64-bit address per column: the loads take the
// scalar-base + vector-offset form)
template <typename T>
__device__ __forceinline__ T ld_off(const T* base, uint32_t off) {
  return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + off);
}
__device__ __forceinline__ NodeRow load_res_row_off(const DevCluster& c, int32_t node) {
  const uint32_t o8 = (uint32_t)node << 3, o4 = (uint32_t)node << 2;
  NodeRow r;
  r.node = node;
  r.alloc_cpu = ld_off(c.alloc_cpu, o8);
  r.alloc_mem = ld_off(c.alloc_mem, o8);
  r.alloc_eph = ld_off(c.alloc_eph, o8);
  r.req_cpu = ld_off((const int64_t*)c.req_cpu, o8);
  r.req_mem = ld_off((const int64_t*)c.req_mem, o8);
  r.req_eph = ld_off((const int64_t*)c.req_eph, o8);
  r.nz_cpu = ld_off((const int64_t*)c.nz_cpu, o8);
  r.nz_mem = ld_off((const int64_t*)c.nz_mem, o8);
  r.alloc_pods = ld_off(c.alloc_pods, o4);
  r.num_pods = ld_off((const int32_t*)c.num_pods, o4);
  r.flags = 0;
#pragma unroll
  for (int k = 0; k < KSIM_MAX_SCALAR; k++) r.alloc_sc[k] = r.req_sc[k] = 0;
#pragma unroll
  for (int k = 0; k < KSIM_MAX_NODE_TAINTS / 2; k++) r.taints[k] = 0;
  return r;
}

__device__ __forceinline__ NodeRow load_row(const DevCluster& c, int32_t node) {
  NodeRow r;
  r.node = node;
  r.alloc_cpu = c.alloc_cpu[node];
  r.alloc_mem = c.alloc_mem[node];
  r.alloc_eph = c.alloc_eph[node];
  r.req_cpu = c.req_cpu[node];
  r.req_mem = c.req_mem[node];
  r.req_eph = c.req_eph[node];
  r.nz_cpu = c.nz_cpu[node];
  r.nz_mem = c.nz_mem[node];
  r.alloc_pods = c.alloc_pods[node];
  r.num_pods = c.num_pods[node];
  r.flags = c.flags[node];
#pragma unroll
  for (int k = 0; k < KSIM_MAX_SCALAR; k++) {
    const bool on = k < c.n_scalar;
    r.alloc_sc[k] = on ? c.alloc_scalar[(size_t)k * c.n + node] : 0;
    r.req_sc[k] = on ? c.req_scalar[(size_t)k * c.n + node] : 0;
  }
#pragma unroll
  for (int k = 0; k < KSIM_MAX_NODE_TAINTS / 2; k++)
    r.taints[k] = (uint32_t)c.taints[(size_t)(2 * k) * c.n + node] |
                  ((uint32_t)c.taints[(size_t)(2 * k + 1) * c.n + node] << 16);
  return r;
}

// floor(a / b) for a >= 0, b > 0.  Below 2^52 the correctly rounded f64
// quotient is within 1 of the true one, so one correction step makes it exact;
// this replaces the ~100-instruction 64-bit integer division sequence.
__device__ __forceinline__ int64_t div_floor_nonneg(int64_t a, int64_t b) {
  if (a >= (1ll << 52) || b >= (1ll << 52)) return a / b;
  int64_t q = (int64_t)((double)a / (double)b);
  if (q * b > a) q--;
  else if ((q + 1) * b <= a) q++;
  return q;
}

// a / b with Go / C truncation, b > 0 (NormalizeScore's quotients): the
// f64-quotient path of div_floor_nonneg on |a| (the integer division sequence
// only past 2^52).
__device__ __forceinline__ int64_t div_trunc_pos(int64_t a, int64_t b) {
  if (a >= 0) return div_floor_nonneg(a, b);
  if (a == INT64_MIN) return a / b;
  return -div_floor_nonneg(-a, b);
}

// ---- normalization ----------------------------------------------------------
// Extrema a slot needs, merged over the kept feasible list:
//   DefaultNormalizeScore: maxCount = max(0, max)          (helper/normalize_score.go)
//   PodTopologySpread:     maxScore = max(0, max), minScore = min, IgnoredNodes excluded
//   InterPodAffinity:      min / max, only when topologyScore is non-empty
__device__ __forceinline__ int64_t normalize_value(int32_t kind, int64_t v, int64_t gmax, int64_t gmin,
                                                   bool ipa_nonempty) {
  switch (kind) {
    case kNormDefault: {
      int64_t m = gmax > 0 ? gmax : 0;
      return m == 0 ? v : div_trunc_pos((int64_t)((uint64_t)kMaxNodeScore * (uint64_t)v), m);
    }
    case kNormDefaultReverse: {
      int64_t m = gmax > 0 ? gmax : 0;
      return m == 0 ? (int64_t)kMaxNodeScore
                    : (int64_t)kMaxNodeScore - div_trunc_pos((int64_t)((uint64_t)kMaxNodeScore * (uint64_t)v), m);
    }
    case kNormPTS: {
      int64_t mx = gmax > 0 ? gmax : 0;
      return mx == 0 ? (int64_t)kMaxNodeScore
                     : div_trunc_pos((int64_t)((uint64_t)kMaxNodeScore * (uint64_t)(mx + gmin - v)), mx);
    }
    case kNormIPA:
    case kNormMinMax: {
      if (kind == kNormIPA && !ipa_nonempty) return v;
      const int64_t diff = gmax - gmin;
      double f = 0;
      if (diff > 0) f = (double)kMaxNodeScore * ((double)(v - gmin) / (double)diff);
      return (int64_t)f;
    }
    default:
      return v;
  }
}


// floor(a / b) for 0 <= a <= 100 * b, b > 0 (a score-sized quotient): an f32
// reciprocal estimate is within 100 * 2^-20 of a / b, so its truncation is
// off by at most one, which one exact integer remainder test repairs.
__device__ __forceinline__ int64_t div_q100(int64_t a, int64_t b) {
  int32_t q = (int32_t)((float)a * __builtin_amdgcn_rcpf((float)b));
  const int64_t rem = a - (int64_t)q * b;
  q -= rem < 0;
  q += rem >= b;
  return q;
}

// Bit `id` of a KSIM_TAINT_WORDS-word set.  The word is picked with selects,
// never a runtime array index, so a pod record copied into registers stays in
// registers (a dynamic index would move it to scratch memory).
__device__ __forceinline__ int bit_set(const uint64_t (&w)[KSIM_TAINT_WORDS], uint32_t id) {
  static_assert(KSIM_TAINT_WORDS == 4, "bit_set assumes 4 words");
  const uint32_t q = id >> 6;
  const uint64_t x = q == 0 ? w[0] : q == 1 ? w[1] : q == 2 ? w[2] : w[3];
  return (int)((x >> (id & 63)) & 1ull);
}

// labels.Requirement.Matches / metadata.name field selector
__device__ __forceinline__ bool label_req_matches(const DevCluster& c, const ksim_label_expr& e, int32_t node) {
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
      for (int k = 0; k < e.nvals; k++) if ((int32_t)e.vals[k] == c.base + node) return true;
      return false;
    }
    case KSIM_OP_FIELD_NOT_IN: {
      for (int k = 0; k < e.nvals; k++) if ((int32_t)e.vals[k] == c.base + node) return false;
      return true;
    }
    case KSIM_OP_TRUE: return true;
    default: return false;
  }
}

__device__ __forceinline__ bool term_matches(const DevCluster& c, const DevPods& P, const ksim_term& t, int32_t node) {
  if (t.n_expr <= 0) return false;
  for (int i = 0; i < t.n_expr; i++)
    if (!label_req_matches(c, P.exprs[t.first_expr + i], node)) return false;
  return true;
}

// nodeaffinity RequiredNodeAffinity.Match
__device__ __forceinline__ bool required_node_affinity_match(const DevCluster& c, const DevPods& P,
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

// nodeaffinity.NodeAffinity.Filter: the profile's scheduler-enforced
// addedAffinity first (errReasonEnforced, detail KSIM_NA_ENFORCED), then the
// pod's selector and required terms (ErrReasonPod, detail 0).  Returns true
// when the node passes.
__device__ __forceinline__ bool node_affinity_filter(const DevCluster& c, const DevPods& P, const ksim_pod& p,
                                                     int32_t node, uint32_t& detail) {
  if (p.flags & KSIM_POD_ADDED_AFFINITY) {
    bool any = false;
    for (int i = 0; i < p.added_term_count && !any; i++) any = term_matches(c, P, P.terms[p.added_term_first + i], node);
    if (!any) {
      detail = KSIM_NA_ENFORCED;
      return false;
    }
  }
  detail = 0;
  return required_node_affinity_match(c, P, p, node);
}

// VolumeBinding / VolumeZone (ksim_engine.h "Volume groups"): terms
// [first, first + count) of the pod set in groups (ksim_term.weight = group
// index, non-decreasing); true iff every group has a matching term.
__device__ __forceinline__ bool volume_groups_match(const DevCluster& c, const DevPods& P, int32_t first,
                                                    int32_t count, int32_t node) {
  int32_t group = -1;
  bool ok = true;                                  // the current group has a match
  for (int i = 0; i < count; i++) {
    const ksim_term& t = P.terms[first + i];
    if (t.weight != group) {
      if (!ok) return false;
      group = t.weight;
      ok = false;
    }
    if (!ok && term_matches(c, P, t, node)) ok = true;
  }
  return ok;
}

// VolumeBinding: the reasons of the failing groups (KSIM_VB_NODE_CONFLICT for
// a bound-PV group, KSIM_VB_BIND_CONFLICT for an unbound-claim group); 0 = pass.
__device__ __forceinline__ uint32_t volume_binding_fails(const DevCluster& c, const DevPods& P, int32_t first,
                                                         int32_t count, int32_t node) {
  int32_t group = -1;
  bool ok = true;
  uint32_t why = 0;
  for (int i = 0; i < count; i++) {
    const ksim_term& t = P.terms[first + i];
    if (t.weight != group) {
      if (!ok) why |= (group & KSIM_VB_UNBOUND_GROUP) ? KSIM_VB_BIND_CONFLICT : KSIM_VB_NODE_CONFLICT;
      group = t.weight;
      ok = false;
    }
    if (!ok && term_matches(c, P, t, node)) ok = true;
  }
  if (!ok) why |= (group & KSIM_VB_UNBOUND_GROUP) ? KSIM_VB_BIND_CONFLICT : KSIM_VB_NODE_CONFLICT;
  return why;
}

// nodeaffinity PreferredSchedulingTerms.Score
__device__ __forceinline__ int64_t preferred_node_affinity_score(const DevCluster& c, const DevPods& P,
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
__device__ __forceinline__ uint32_t find_matching_untolerated_taint(const DevCluster& c, const ksim_pod& p, const NodeRow& r) {
#pragma unroll
  for (int k = 0; k < KSIM_MAX_NODE_TAINTS; k++) {
    uint32_t tid = row_taint(r, k);
    if (!tid) break;
    uint8_t eff = c.taint_effect[tid];
    if ((eff == KSIM_EFFECT_NO_SCHEDULE || eff == KSIM_EFFECT_NO_EXECUTE) && !bit_set(p.tol_filter, tid))
      return tid;
  }
  return 0;
}

// tainttoleration countIntolerableTaintsPreferNoSchedule
__device__ __forceinline__ int64_t count_intolerable_prefer(const DevCluster& c, const ksim_pod& p, const NodeRow& r) {
  int64_t n = 0;
#pragma unroll
  for (int k = 0; k < KSIM_MAX_NODE_TAINTS; k++) {
    uint32_t tid = row_taint(r, k);
    if (!tid) break;
    if (c.taint_effect[tid] != KSIM_EFFECT_PREFER_NO_SCHEDULE) continue;
    if (!bit_set(p.tol_prefer, tid)) n++;
  }
  return n;
}

// noderesources fitsRequest -> reason bits.  ignore: scalar columns the
// profile's ignoredResources / ignoredResourceGroups name (extended resources).
__device__ __forceinline__ uint32_t fits_request(const NodeRow& r, const ksim_pod& p, int n_scalar, uint32_t ignore) {
  uint32_t bits = 0;
  if (r.num_pods + 1 > r.alloc_pods) bits |= KSIM_FIT_TOO_MANY_PODS;
  if (p.req_cpu == 0 && p.req_mem == 0 && p.req_eph == 0 && !(p.flags & KSIM_POD_HAS_SCALAR)) return bits;
  if (p.req_cpu > r.alloc_cpu - r.req_cpu) bits |= KSIM_FIT_CPU;
  if (p.req_mem > r.alloc_mem - r.req_mem) bits |= KSIM_FIT_MEMORY;
  if (p.req_eph > r.alloc_eph - r.req_eph) bits |= KSIM_FIT_EPHEMERAL;
#pragma unroll
  for (int k = 0; k < KSIM_MAX_SCALAR; k++) {
    if (k >= n_scalar) break;
    const int64_t q = p.scalar_req[k];
    if (q != 0 && !((ignore >> k) & 1u) && q > r.alloc_sc[k] - r.req_sc[k]) bits |= (KSIM_FIT_SCALAR0 << k);
  }
  return bits;
}

// resourceAllocationScorer.calculateResourceAllocatableRequest
__device__ __forceinline__ void calc_alloc_req(const NodeRow& r, const ksim_pod& p, int32_t res, bool use_requested,
                                               int n_scalar, int64_t& alloc, int64_t& req) {
  alloc = 0;
  req = 0;
  if (res == KSIM_RES_CPU) {
    alloc = r.alloc_cpu;
    req = use_requested ? r.req_cpu + p.req_cpu : r.nz_cpu + p.nz_cpu;
  } else if (res == KSIM_RES_MEMORY) {
    alloc = r.alloc_mem;
    req = use_requested ? r.req_mem + p.req_mem : r.nz_mem + p.nz_mem;
  } else if (res == KSIM_RES_EPHEMERAL) {
    alloc = r.alloc_eph;
    req = r.req_eph + p.req_eph;
  } else {
#pragma unroll
    for (int k = 0; k < KSIM_MAX_SCALAR; k++) {
      if (res == KSIM_RES_SCALAR0 + k && k < n_scalar && p.scalar_req[k] != 0) {
        alloc = r.alloc_sc[k];
        req = r.req_sc[k] + p.scalar_req[k];
      }
    }
  }
}

// least_allocated.go leastRequestedScore.  (capacity - requested) * 100 is Go
// int64 arithmetic, which wraps for capacities past 2^56: the product is formed
// unsigned (defined wrap), and such a quotient is taken exactly (a / b).
__device__ __forceinline__ int64_t least_requested_score(int64_t requested, int64_t capacity) {
  if (capacity == 0) return 0;
  if (requested > capacity) return 0;
  const int64_t prod = (int64_t)((uint64_t)(capacity - requested) * (uint64_t)kMaxNodeScore);
  if (capacity < 0 || prod < 0) return prod / capacity;
  return div_floor_nonneg(prod, capacity);
}

// leastRequestedScore for 0 < capacity < 2^52 (no wrap; the quotient is in
// [0, 100]), the general form otherwise.
__device__ __forceinline__ int64_t least_requested_q100(int64_t requested, int64_t capacity) {
  if (capacity < 0 || capacity >= (1ll << 52)) return least_requested_score(requested, capacity);
  if (requested > capacity) return 0;
  return div_q100((capacity - requested) * kMaxNodeScore, capacity);
}

// most_allocated.go mostRequestedScore: requested clamped to capacity, Go
// int64 arithmetic (the product wraps as leastRequestedScore's does).
__device__ __forceinline__ int64_t most_requested_score(int64_t requested, int64_t capacity) {
  if (capacity == 0) return 0;
  if (requested > capacity) requested = capacity;
  const int64_t prod = (int64_t)((uint64_t)requested * (uint64_t)kMaxNodeScore);
  if (capacity < 0 || prod < 0) return prod / capacity;
  return div_floor_nonneg(prod, capacity);
}

// helper.BuildBrokenLinearFunction over the profile's RequestedToCapacityRatio
// shape (scores already x 10): the first point whose utilization is >= p, the
// segment before it interpolated in Go int64 (truncating) arithmetic.
// Constant indices only, so the shape stays in scalar registers.
__device__ __forceinline__ int64_t broken_linear(const ksim_profile& prof, int64_t p) {
  int64_t res = 0, pu = 0, ps = 0;
  bool done = false;
#pragma unroll
  for (int i = 0; i < KSIM_MAX_SHAPE; i++) {
    if (i < prof.fit_n_shape && !done) {
      const int64_t u = prof.fit_shape_util[i], sc = prof.fit_shape_score[i];
      if (p <= u) {
        res = i == 0 ? sc : ps + (sc - ps) * (p - pu) / (u - pu);
        done = true;
      }
      pu = u;
      ps = sc;
    }
  }
  return done ? res : ps;
}

// requested_to_capacity_ratio.go resourceScoringFunction
__device__ __forceinline__ int64_t rtcr_resource_score(const ksim_profile& prof, int64_t requested, int64_t capacity) {
  if (capacity == 0 || requested > capacity) return broken_linear(prof, 100);   // maxUtilization
  const int64_t prod = (int64_t)((uint64_t)requested * 100u);
  return broken_linear(prof, prod / capacity);
}

// NodeResourcesFit Score: resourceAllocationScorer.score with the profile's
// ScoringStrategy (useRequested = false: the non-zero requests).  Resources a
// node has no allocatable of (or an extended resource the pod does not
// request) are left out of the map, hence of the weight sum.
__device__ __forceinline__ int64_t fit_score(const NodeRow& r, const ksim_profile& prof, const ksim_pod& p,
                                             int n_scalar) {
  int64_t node_score = 0, weight_sum = 0;
  const int strat = prof.fit_strategy;
#pragma unroll
  for (int i = 0; i < KSIM_MAX_RES; i++) {      // constant indices only (no exit): prof stays in registers
    int64_t a = 0, q = 0;
    if (i < prof.fit_n_res) calc_alloc_req(r, p, prof.fit_res[i], false, n_scalar, a, q);
    if (a == 0) continue;
    const int64_t w = prof.fit_res_weight[i];
    if (strat == KSIM_FIT_REQUESTED_TO_CAPACITY_RATIO) {
      const int64_t rs = rtcr_resource_score(prof, q, a);
      if (rs > 0) {                             // only positive resource scores count
        node_score += rs * w;
        weight_sum += w;
      }
      continue;
    }
    node_score += (strat == KSIM_FIT_MOST_ALLOCATED ? most_requested_score(q, a) : least_requested_score(q, a)) * w;
    weight_sum += w;
  }
  if (weight_sum == 0) return 0;
  if (strat == KSIM_FIT_REQUESTED_TO_CAPACITY_RATIO)   // math.Round(float64(nodeScore) / float64(weightSum))
    return (int64_t)round((double)node_score / (double)weight_sum);
  if (node_score < 0 || weight_sum < 0) return node_score / weight_sum;
  return div_floor_nonneg(node_score, weight_sum);
}

// balanced_allocation.go balancedResourceScorer (float64, unfused).  The
// fractions are recomputed in the second pass instead of being stored in a
// dynamically indexed array (which would live in scratch memory); the
// recomputation is bitwise identical.
__device__ __forceinline__ int64_t balanced_allocation_score(const NodeRow& r, const ksim_profile& prof, const ksim_pod& p,
                                                    int n_scalar) {
  int nf = 0;
  double total = 0, f0 = 0, f1 = 0;
#pragma unroll
  for (int i = 0; i < KSIM_MAX_RES; i++) {
    int64_t a = 0, q = 0;
    if (i < prof.ba_n_res) calc_alloc_req(r, p, prof.ba_res[i], true, n_scalar, a, q);
    if (a == 0) continue;
    double f = (double)q / (double)a;
    if (f > 1) f = 1;
    total += f;
    if (nf == 0) f0 = f;
    else if (nf == 1) f1 = f;
    nf++;
  }
  double std = 0.0;
  if (nf == 2) {
    std = fabs((f0 - f1) / 2);
  } else if (nf > 2) {
    const double mean = total / (double)nf;
    double sum = 0;
#pragma unroll
    for (int i = 0; i < KSIM_MAX_RES; i++) {
      int64_t a = 0, q = 0;
      if (i < prof.ba_n_res) calc_alloc_req(r, p, prof.ba_res[i], true, n_scalar, a, q);
      if (a == 0) continue;
      double f = (double)q / (double)a;
      if (f > 1) f = 1;
      sum = sum + (f - mean) * (f - mean);
    }
    std = sqrt(sum / (double)nf);
  }
  return (int64_t)((1 - std) * (double)kMaxNodeScore);
}

// ---- NetworkBandwidth (simulator/scheduler/plugin/networkbandwidth/plugin.go) --
// A Filter status other than Success / Unschedulable (its Skip and Error
// returns) makes [upstream] RunFilterPlugins return framework.Error, and the
// cycle fails.  Such a node's fail code carries kFailError next to the plugin's
// filter index; the window decides whether the scan reached it.
constexpr uint8_t kFailError = 0x80;
constexpr int32_t kCycleErrorFilter = 1;   // an erroring node inside the scanned window
constexpr int32_t kCycleErrorScore = 2;    // Score returned Skip / Error for a kept node
constexpr int32_t kCycleErrorPrefilter = 3; // PreFilterResult names a node the snapshot lacks (KSIM_POD_NODE_NAMES_UNKNOWN)

__host__ __device__ __forceinline__ bool nb_error_detail(uint32_t d) { return d >= KSIM_NB_NO_LIMIT; }
__host__ __device__ __forceinline__ bool fail_is_error(uint8_t f) { return (f & kFailError) && f < KSIM_FAIL_EXTENDER; }
// Profile arrays at a runtime (uniform) index, extracted from packed words by
// shifts: a runtime index into the by-value kernel argument would compile to a
// select chain over every element at each access.
__device__ __forceinline__ uint32_t prof_filter(const ksim_profile& prof, int f) {
  uint64_t w0, w1;
  memcpy(&w0, prof.filter, 8);
  memcpy(&w1, prof.filter + 8, 8);
  return (uint32_t)(((f < 8 ? w0 : w1) >> (8 * (f & 7))) & 0xffu);
}
__device__ __forceinline__ uint32_t prof_score(const ksim_profile& prof, int k) {
  static_assert(KSIM_MAX_SCORE == 8 && KSIM_MAX_FILTER == 16, "packed profile words");
  uint64_t w;
  memcpy(&w, prof.score, 8);
  return (uint32_t)((w >> (8 * k)) & 0xffu);
}
// score_weight[k], 0 read as 1 (the framework's default weight)
__device__ __forceinline__ int64_t prof_weight(const ksim_profile& prof, int k) {
  uint64_t w[4];
  memcpy(w, prof.score_weight, 32);
  const int q = k >> 1;
  const uint64_t x = q == 0 ? w[0] : q == 1 ? w[1] : q == 2 ? w[2] : w[3];
  const int32_t v = (int32_t)(uint32_t)(x >> (32 * (k & 1)));
  return v == 0 ? 1 : v;
}

__host__ __device__ __forceinline__ bool prof_has_filter(const ksim_profile& prof, int plugin) {
  for (int f = 0; f < prof.n_filter; f++)
    if (prof.filter[f] == plugin) return true;
  return false;
}
__host__ __device__ __forceinline__ bool prof_has_score(const ksim_profile& prof, int plugin) {
  for (int k = 0; k < prof.n_score; k++)
    if (prof.score[k] == plugin) return true;
  return false;
}

// Filter, plugin.go:52-102, checks in its order (quantities in milli-units)
__device__ __forceinline__ uint32_t nb_filter(const DevCluster& c, const ksim_pod& p, uint32_t flags, int32_t node) {
  if (!(flags & KSIM_NODE_NB_LIMIT)) return KSIM_NB_NO_LIMIT;            // :54-57 Skip
  if (flags & KSIM_NODE_NB_LIMIT_BAD) return KSIM_NB_LIMIT_BAD;          // :58-61 Error
  if (p.nb_flags & KSIM_POD_NB_INGRESS_BAD) return KSIM_NB_INGRESS_BAD;  // :72-76 Error
  if (p.nb_flags & KSIM_POD_NB_EGRESS_BAD) return KSIM_NB_EGRESS_BAD;    // :84-88 Error
  if (p.nb_req == 0) return KSIM_NB_NO_REQUEST;                           // :92-94 Skip
  return c.nb_alloc[node] + p.nb_req > c.nb_limit[node] ? KSIM_NB_INSUFFICIENT : 0u;   // :97-99
}

// Score, plugin.go:128-149: (limit - allocated).Value(), resource.Quantity's
// integer value, which rounds a fraction away from zero
__device__ __forceinline__ int64_t nb_score(const DevCluster& c, int32_t node) {
  const int64_t d = c.nb_limit[node] - c.nb_alloc[node];
  return d >= 0 ? (d + 999) / 1000 : -((-d + 999) / 1000);
}

// Score returns Skip (no limit annotation) or Error (unparsable limit): the
// framework's RunScorePlugins fails the cycle
__host__ __device__ __forceinline__ bool nb_score_error(uint32_t flags) {
  return !(flags & KSIM_NODE_NB_LIMIT) || (flags & KSIM_NODE_NB_LIMIT_BAD);
}

// ---- PodTopologySpread / InterPodAffinity / NodePorts / ImageLocality inputs --
// Internal use flag, set only when a pod's uses are staged on the device (never
// in the ABI): the use's key column is unique per node (DevCluster.col_unique),
// so an InterPodAffinity domain sum is the node's own class count and needs no
// domain table.
constexpr uint8_t kUseUniqueCol = 0x80;

// The use's per-node number is the node's own class count (no domain table):
// PodTopologySpread ScheduleAnyway on hostname (upstream counts the node's
// pods), NodePorts, ImageLocality, and InterPodAffinity on a unique column.
__host__ __device__ __forceinline__ bool use_node_count(const ksim_topo_use& u) {
  return (u.kind == KSIM_USE_PTS_SOFT && (u.flags & KSIM_USEF_HOSTNAME)) || u.kind == KSIM_USE_NODE_PORT ||
         u.kind == KSIM_USE_IMAGE ||
         ((u.flags & kUseUniqueCol) && u.kind >= KSIM_USE_IPA_EXISTING_ANTI && u.kind <= KSIM_USE_IPA_SCORE_HARD);
}

// A use record as four dwords: one scalar load when its address is
// block-uniform (a sub-dword field read alone would take the vector memory
// path).  Layout: cls, arg, col | kind << 16 | flags << 24, pad.
static_assert(sizeof(ksim_topo_use) == 16, "ksim_topo_use is four dwords");
__device__ __forceinline__ ksim_topo_use load_use(const ksim_topo_use* U, int i) {
  const uint4 w = reinterpret_cast<const uint4*>(U)[i];
  ksim_topo_use u;
  u.cls = (int32_t)w.x;
  u.arg = (int32_t)w.y;
  u.col = (uint16_t)(w.z & 0xffffu);
  u.kind = (uint8_t)((w.z >> 16) & 0xffu);
  u.flags = (uint8_t)(w.z >> 24);
  u._pad = (int32_t)w.w;
  return u;
}

// The pod's uses by role, one bit per use (bit i = use i), built once per
// thread from scalar loads: the per-node code tests uniform bits instead of
// re-reading each use's kind inside every plugin.
struct UseMasks {
  uint32_t hard, soft, soft_val, aff, anti, exist, score, port, image, node_count, self_match;
  uint32_t dom;                  // k_topo_prefilter fills the use's domain table (use_needs_dom, and adds)
  uint32_t honor_aff, honor_taints;   // PTS nodeAffinityPolicy / nodeTaintsPolicy Honor
  uint32_t ptab;                 // dom uses read from a persistent table (kPlanPtab pods)
  uint32_t _pad;
};

// Per-pod plan of the per-pod cycle, compiled by the host when a pod set is
// uploaded (ksim_load_pods and the single-pod calls; a queue is uploaded again
// after every ksim_set_profile / ksim_set_cluster, so the plan may depend on
// both): the filter plugins that can fail for this pod on this cluster (the
// rest pass every node), and its topology uses by role.  The kernels read it
// with scalar loads instead of re-deriving it per node.
struct PodPlan {
  uint32_t filter_en;            // plugin ids to evaluate (1 << id), FilterPlan.en
  uint32_t flags;                // kPlan*
  UseMasks m;
  int32_t tadd_first, tadd_count;   // kPlanTadds: the pod's persistent-table updates (DevPods.ptab_padd)
};
// PodPlan.flags
// kPlanPtab: every domain sum the pod reads is a persistent table (its device
// use copies carry the table's first entry in _pad, DevPods.ptab), and so is
// every InterPodAffinity emptiness test (a kPtabTotal table for key columns
// unique per node): the cycle runs no k_topo_prefilter, and k_filter_score
// derives the topology flags from the tables.
constexpr uint32_t kPlanPtab = 1u;
// kPlanTadds: tadd_first / tadd_count list every persistent-table update of
// the pod's binds (queue pods; single uploads go through the class index).
constexpr uint32_t kPlanTadds = 2u;
// (flags >> kPlanVuseShift) & 31: 1 + the pod's zone-variant use (topology
// batches, TbVar: its first DoNotSchedule spread use read from a persistent
// table whose key has at most kVarDom domains), 0: none
constexpr int kPlanVuseShift = 8;
// (flags >> kPlanVcolShift) - 1: the key column of the zone variants of the
// topology batch run from this pod (-1: the run has none)
constexpr int kPlanVcolShift = 16;

// One node's inputs of every topology use of the cycle's pod, loaded up front:
// one round of label loads, then one of domain-table / class-count loads, so
// the plugins below read registers instead of a dependent load pair per use
// inside each plugin's loop.
struct TopoRow {
  uint32_t v[KSIM_MAX_USES];     // value id of the use's key column on the node (0: key absent)
  int64_t x[KSIM_MAX_USES];      // domain-table entry of that value, or the node's class count
};

// frameworkImpl.RunFilterPlugins (stop at first failure)
__device__ __forceinline__ uint32_t pts_filter(const ksim_topo_use* U, const UseMasks& m, const int64_t* min_match,
                                               const TopoRow& t);
__device__ __forceinline__ uint32_t ipa_filter(const UseMasks& m, const ksim_pod& p, uint32_t topo_flags,
                                               const TopoRow& t);
__device__ __forceinline__ int64_t ipa_score(const ksim_profile& prof, const ksim_topo_use* U, const UseMasks& m,
                                             const TopoRow& t);
__device__ __forceinline__ bool node_port_conflict(const UseMasks& m, const TopoRow& t);
__device__ __forceinline__ int64_t image_locality_score(const UseMasks& m, const TopoRow& t);

// U / m / t: the pod's uses (p.use_count of them), their masks and the node's TopoRow.
__device__ __forceinline__ uint8_t run_filter_plugins(const DevCluster& c, const DevPods& P, const ksim_profile& prof,
                                             const int64_t* min_match, uint32_t topo_flags, const ksim_pod& p,
                                             const NodeRow& r, const ksim_topo_use* U, const UseMasks& m,
                                             const TopoRow& t, uint32_t& detail) {
  detail = 0;
  const int32_t node = r.node;
  const int nu = p.use_count;
  for (int f = 0; f < prof.n_filter; f++) {
    switch (prof_filter(prof, f)) {
      case KSIM_PL_NODE_UNSCHEDULABLE:
        if ((r.flags & KSIM_NODE_UNSCHEDULABLE) && !(p.flags & KSIM_POD_TOLERATES_UNSCHEDULABLE))
          return (uint8_t)f;
        break;
      case KSIM_PL_NODE_NAME:
        if (p.node_name != -1 && p.node_name != c.base + node) return (uint8_t)f;
        break;
      case KSIM_PL_TAINT_TOLERATION: {
        uint32_t tid = find_matching_untolerated_taint(c, p, r);
        if (tid) { detail = tid; return (uint8_t)f; }
        break;
      }
      case KSIM_PL_NODE_AFFINITY: {
        uint32_t why;
        if (!node_affinity_filter(c, P, p, node, why)) { detail = why; return (uint8_t)f; }
        break;
      }
      case KSIM_PL_VOLUME_BINDING: {
        const uint32_t why = p.vb_count ? volume_binding_fails(c, P, p.vb_first, p.vb_count, node) : 0u;
        if (why) { detail = why; return (uint8_t)f; }
        break;
      }
      case KSIM_PL_VOLUME_ZONE:
        if (p.vz_count && !volume_groups_match(c, P, p.vz_first, p.vz_count, node)) return (uint8_t)f;
        break;
      case KSIM_PL_NODE_RESOURCES_FIT: {
        uint32_t bits = fits_request(r, p, c.n_scalar, c.fit_ignore);
        if (bits) { detail = bits; return (uint8_t)f; }
        break;
      }
      case KSIM_PL_NODE_PORTS:
        if (nu && node_port_conflict(m, t)) return (uint8_t)f;
        break;
      case KSIM_PL_POD_TOPOLOGY_SPREAD: {
        const uint32_t why = nu ? pts_filter(U, m, min_match, t) : 0;
        if (why) { detail = why; return (uint8_t)f; }
        break;
      }
      case KSIM_PL_INTER_POD_AFFINITY: {
        const uint32_t why = nu ? ipa_filter(m, p, topo_flags, t) : 0;
        if (why) { detail = why; return (uint8_t)f; }
        break;
      }
      case KSIM_PL_NETWORK_BANDWIDTH: {
        const uint32_t why = nb_filter(c, p, r.flags, node);
        if (why) {
          detail = why;
          return (uint8_t)(f | (nb_error_detail(why) ? kFailError : 0));
        }
        break;
      }
      default:
        break;
    }
  }
  return KSIM_PASSED;
}

// PodTopologySpread's raw score needs the feasible list (k_extrema computes it).
__device__ __forceinline__ int64_t score_plugin_raw(const DevCluster& c, const DevPods& P, const ksim_profile& prof,
                                           const ksim_pod& p, int plugin, const NodeRow& r,
                                           const ksim_topo_use* U, const UseMasks& m, const TopoRow& t) {
  switch (plugin) {
    case KSIM_PL_NODE_RESOURCES_FIT: return fit_score(r, prof, p, c.n_scalar);
    case KSIM_PL_BALANCED_ALLOCATION: return balanced_allocation_score(r, prof, p, c.n_scalar);
    case KSIM_PL_TAINT_TOLERATION: return count_intolerable_prefer(c, p, r);
    case KSIM_PL_NODE_AFFINITY: return preferred_node_affinity_score(c, P, p, r.node);
    case KSIM_PL_INTER_POD_AFFINITY: return p.use_count ? ipa_score(prof, U, m, t) : 0;
    case KSIM_PL_IMAGE_LOCALITY: return p.use_count ? image_locality_score(m, t) : 0;
    case KSIM_PL_NETWORK_BANDWIDTH: return nb_score_error(r.flags) ? 0 : nb_score(c, r.node);
    default: return 0;   // PodTopologySpread: k_extrema
  }
}

// ---- per-pod plans: the filter and score chains as straight-line code --------
// The per-node chain above is a runtime loop over the profile with a switch per
// plugin; on CDNA every iteration pays the dispatch branches and the spills
// around the inlined plugin bodies.  The plans below evaluate, in a fixed order,
// only the plugins that can matter for this pod on this cluster (uniform bits),
// then pick the first failure by profile position: the same result, because
// the filter plugins are pure.
struct FilterPlan {
  uint64_t rank_lo, rank_hi;   // profile position of each plugin id, 5 bits each (ids 0..11 | 12..)
  uint32_t en;                 // plugin ids to evaluate (1 << id)
};

__device__ __forceinline__ uint32_t plan_rank(const FilterPlan& fp, int pl) {
  return pl < 12 ? (uint32_t)((fp.rank_lo >> (5 * pl)) & 31u) : (uint32_t)((fp.rank_hi >> (5 * (pl - 12))) & 31u);
}

// FilterPlan.en for one pod (host, at upload): the profile's filter plugins
// that can fail for this pod on this cluster.  any_unschedulable / hard_taints:
// some node has spec.unschedulable / a NoSchedule or NoExecute taint.
inline uint32_t plan_filter_en(const ksim_profile& prof, const ksim_pod& p, const UseMasks& m, bool any_unschedulable,
                               bool hard_taints) {
  uint32_t en = 0;
  for (int f = 0; f < prof.n_filter; f++) {
    const int pl = prof.filter[f];
    bool on = false;
    switch (pl) {        // a plugin left out here passes every node for this pod
      case KSIM_PL_NODE_UNSCHEDULABLE:
        on = any_unschedulable && !(p.flags & KSIM_POD_TOLERATES_UNSCHEDULABLE);
        break;
      case KSIM_PL_NODE_NAME: on = p.node_name != -1; break;
      case KSIM_PL_TAINT_TOLERATION: on = hard_taints; break;
      case KSIM_PL_NODE_AFFINITY:
        on = p.sel_count > 0 || (p.flags & (KSIM_POD_HAS_REQUIRED_AFFINITY | KSIM_POD_ADDED_AFFINITY));
        break;
      case KSIM_PL_NODE_PORTS: on = m.port != 0; break;
      case KSIM_PL_NODE_RESOURCES_FIT: on = true; break;
      case KSIM_PL_POD_TOPOLOGY_SPREAD: on = m.hard != 0; break;
      case KSIM_PL_INTER_POD_AFFINITY: on = (m.aff | m.anti | m.exist) != 0; break;
      case KSIM_PL_NETWORK_BANDWIDTH: on = true; break;
      case KSIM_PL_VOLUME_BINDING: on = p.vb_count > 0; break;
      case KSIM_PL_VOLUME_ZONE: on = p.vz_count > 0; break;
      default: break;    // the other volume plugins pass (bound PVCs of unlimited kinds)
    }
    if (on) en |= 1u << pl;
  }
  return en;
}

// The profile's filter positions / score slots per plugin id (host, at
// ksim_set_profile; BatchProg carries them to the kernels).
inline void plan_profile(const ksim_profile& prof, uint64_t& rank_lo, uint64_t& rank_hi, uint64_t& slot,
                         uint32_t& slot_hi) {
  rank_lo = rank_hi = slot = 0;
  slot_hi = 0;
  for (int f = 0; f < prof.n_filter; f++) {
    const int pl = prof.filter[f];
    if (pl < 12) rank_lo |= (uint64_t)f << (5 * pl);
    else rank_hi |= (uint64_t)f << (5 * (pl - 12));
  }
  for (int k = 0; k < prof.n_score; k++) {
    const int pl = prof.score[k];
    if (pl < 16) slot |= (uint64_t)(k + 1) << (4 * pl);
    else slot_hi |= (uint32_t)(k + 1) << (4 * (pl - 16));
  }
}

// frameworkImpl.RunFilterPlugins over the plan: KSIM_PASSED or the profile
// position of the first failing plugin (| kFailError for an error status).
__device__ __forceinline__ uint8_t run_filter_plan(const DevCluster& c, const DevPods& P, const FilterPlan& fp,
                                                   const int64_t* min_match, uint32_t topo_flags, const ksim_pod& p,
                                                   const NodeRow& r, const ksim_topo_use* U, const UseMasks& m,
                                                   const TopoRow& t, uint32_t& detail) {
  uint32_t best = 0xffu, det = 0;
  bool err = false;
  auto take = [&](int pl, bool fails, uint32_t d, bool e) {
    const uint32_t rk = plan_rank(fp, pl);
    if (fails && rk < best) {
      best = rk;
      det = d;
      err = e;
    }
  };
  const int32_t node = r.node;
  if (fp.en & (1u << KSIM_PL_NODE_UNSCHEDULABLE))
    take(KSIM_PL_NODE_UNSCHEDULABLE, (r.flags & KSIM_NODE_UNSCHEDULABLE) != 0, 0, false);
  if (fp.en & (1u << KSIM_PL_NODE_NAME)) take(KSIM_PL_NODE_NAME, p.node_name != c.base + node, 0, false);
  if (fp.en & (1u << KSIM_PL_TAINT_TOLERATION)) {
    const uint32_t tid = find_matching_untolerated_taint(c, p, r);
    take(KSIM_PL_TAINT_TOLERATION, tid != 0, tid, false);
  }
  if (fp.en & (1u << KSIM_PL_NODE_AFFINITY)) {
    uint32_t why;
    const bool ok = node_affinity_filter(c, P, p, node, why);
    take(KSIM_PL_NODE_AFFINITY, !ok, why, false);
  }
  if (fp.en & (1u << KSIM_PL_VOLUME_BINDING))
  {
    const uint32_t why = volume_binding_fails(c, P, p.vb_first, p.vb_count, node);
    take(KSIM_PL_VOLUME_BINDING, why != 0, why, false);
  }
  if (fp.en & (1u << KSIM_PL_VOLUME_ZONE))
    take(KSIM_PL_VOLUME_ZONE, !volume_groups_match(c, P, p.vz_first, p.vz_count, node), 0, false);
  if (fp.en & (1u << KSIM_PL_NODE_RESOURCES_FIT)) {
    const uint32_t bits = fits_request(r, p, c.n_scalar, c.fit_ignore);
    take(KSIM_PL_NODE_RESOURCES_FIT, bits != 0, bits, false);
  }
  if (fp.en & (1u << KSIM_PL_NODE_PORTS)) take(KSIM_PL_NODE_PORTS, node_port_conflict(m, t), 0, false);
  if (fp.en & (1u << KSIM_PL_POD_TOPOLOGY_SPREAD)) {
    const uint32_t why = pts_filter(U, m, min_match, t);
    take(KSIM_PL_POD_TOPOLOGY_SPREAD, why != 0, why, false);
  }
  if (fp.en & (1u << KSIM_PL_INTER_POD_AFFINITY)) {
    const uint32_t why = ipa_filter(m, p, topo_flags, t);
    take(KSIM_PL_INTER_POD_AFFINITY, why != 0, why, false);
  }
  if (fp.en & (1u << KSIM_PL_NETWORK_BANDWIDTH)) {
    const uint32_t why = nb_filter(c, p, r.flags, node);
    take(KSIM_PL_NETWORK_BANDWIDTH, why != 0, why, nb_error_detail(why));
  }
  detail = best == 0xffu ? 0u : det;
  return best == 0xffu ? (uint8_t)KSIM_PASSED : (uint8_t)(best | (err ? kFailError : 0));
}

// The score slots of each plugin id: profile position + 1, 4 bits each (0: absent).
struct ScorePlan {
  uint64_t slot;               // plugin ids 0..15
  uint32_t slot_hi;            // plugin ids 16..
};

__device__ __forceinline__ int plan_slot(const ScorePlan& sp, int pl) {
  return pl < 16 ? (int)((sp.slot >> (4 * pl)) & 15u) - 1 : (int)((sp.slot_hi >> (4 * (pl - 16))) & 15u) - 1;
}

// The raw scores of the plugins with a NormalizeScore (PodTopologySpread's
// aside), kept in registers for the fused extrema.
struct RawScores {
  int64_t taint, aff, ipa, nb;
  __device__ __forceinline__ int64_t of(int pl) const {
    return pl == KSIM_PL_TAINT_TOLERATION ? taint : pl == KSIM_PL_NODE_AFFINITY ? aff
         : pl == KSIM_PL_INTER_POD_AFFINITY ? ipa : pl == KSIM_PL_NETWORK_BANDWIDTH ? nb : 0;
  }
};

// The score plugins' raw scores of one feasible node (PodTopologySpread's
// score needs the whole feasible list: its slot gets pts_count, the node's
// count for the pod's ScheduleAnyway use, which the fused k_select maps to
// the score; k_extrema overwrites it otherwise), stored per slot into raw
// ([slot][n]); returns the weighted sum of the slots without NormalizeScore.
// store_plain: also store the raw score of those slots (compat mode).
struct BatchProg;
// The FAST key's profile inputs as plain scalars, read once per kernel from the
// device copy of the BatchProg (a captured graph outlives a weight change):
// wave-uniform values the compiler keeps in SGPRs, so the key's conditions
// on them are scalar branches, never per-lane control flow.
struct FastProg {
  int32_t fit, w_fit, w_ba, w_eq, no_score;
  int64_t fw_cpu, fw_mem;
  double iw_cpu, iw_mem, iw_sum;
};
__device__ __forceinline__ FastProg fast_prog(const BatchProg& bp);
// DEF: the default profile's shape, known at compile time (fast_def below)
template <bool DEF = false>
__device__ __forceinline__ int32_t fast_least_allocated(const FastProg& q, const ksim_pod& p, const NodeRow& r,
                                                        double inv_c, double inv_m);
template <bool DEF = false>
__device__ __forceinline__ int32_t fast_balanced_allocation(const FastProg& q, const ksim_pod& p, const NodeRow& r,
                                                            double inv_c, double inv_m);

// fast (non-null): BatchProg::fast_w on a kClusterNarrow cluster, so the
// cpu / memory strategies take the host-reciprocal quotients (inv_c, inv_m).
__device__ __forceinline__ int64_t run_score_plan(const DevCluster& c, const DevPods& P, const ksim_profile& prof,
                                                  const ScorePlan& sp, const ksim_pod& p, const NodeRow& r,
                                                  const ksim_topo_use* U, const UseMasks& m, const TopoRow& t,
                                                  int64_t* raw, bool store_plain, RawScores& rv,
                                                  int64_t pts_count, const BatchProg* fast = nullptr,
                                                  double inv_c = 0, double inv_m = 0) {
  int64_t part = 0;
  const size_t n = (size_t)c.n;
  auto put = [&](int pl, int64_t v) {
    const int k = plan_slot(sp, pl);
    if (norm_kind(pl) == kNormNone) {
      part += v * prof_weight(prof, k);
      if (store_plain) raw[(size_t)k * n + r.node] = v;
    } else {
      raw[(size_t)k * n + r.node] = v;
    }
  };
#define KSIM_PUT(pl, dst, expr) \
  if (plan_slot(sp, pl) >= 0) { dst = (expr); put(pl, dst); }
  int64_t v;
  KSIM_PUT(KSIM_PL_NODE_RESOURCES_FIT, v, fast ? (int64_t)fast_least_allocated(fast_prog(*fast), p, r, inv_c, inv_m)
                                                : fit_score(r, prof, p, c.n_scalar));
  KSIM_PUT(KSIM_PL_BALANCED_ALLOCATION, v, fast ? (int64_t)fast_balanced_allocation(fast_prog(*fast), p, r, inv_c, inv_m)
                                                : balanced_allocation_score(r, prof, p, c.n_scalar));
  KSIM_PUT(KSIM_PL_TAINT_TOLERATION, rv.taint, (c.cflags & kClusterPreferTaints) ? count_intolerable_prefer(c, p, r) : 0);
  KSIM_PUT(KSIM_PL_NODE_AFFINITY, rv.aff, p.pref_term_count ? preferred_node_affinity_score(c, P, p, r.node) : 0);
  KSIM_PUT(KSIM_PL_INTER_POD_AFFINITY, rv.ipa, m.score ? ipa_score(prof, U, m, t) : 0);
  KSIM_PUT(KSIM_PL_IMAGE_LOCALITY, v, m.image ? image_locality_score(m, t) : 0);
  KSIM_PUT(KSIM_PL_NETWORK_BANDWIDTH, rv.nb, nb_score_error(r.flags) ? 0 : nb_score(c, r.node));
  KSIM_PUT(KSIM_PL_POD_TOPOLOGY_SPREAD, v, pts_count);   // k_extrema or k_select makes it a score
#undef KSIM_PUT
  return part;
}

// Sum of weighted raw scores of the slots without NormalizeScore.


// ---- PodTopologySpread / InterPodAffinity -------------
// Same structure as oracle/ksim_oracle.c: upstream's topology-pair maps are
// domain tables dom[u][value id of the use's key column] in HBM, filled by
// k_topo_prefilter (atomics, LDS-staged for small key vocabularies).
__device__ __forceinline__ uint32_t use_value(const DevCluster& c, const ksim_topo_use& u, int32_t node) {
  return u.col == KSIM_COL_NONE ? 0u : c.labels[(size_t)u.col * c.n + node];
}
__device__ __forceinline__ int64_t class_count(const DevCluster& c, int32_t cls, int32_t node) {
  return cls < 0 ? 0 : (int64_t)c.cnt[(size_t)cls * c.n + node];
}
__device__ __forceinline__ const int64_t* dom_of(const DevCluster& c, const DevScratch& s, int u) {
  return s.dom + (size_t)u * c.vmax;
}
// A use whose domain table k_topo_prefilter fills (use_node_count: the node's
// own count instead).
__host__ __device__ __forceinline__ bool use_needs_dom(const ksim_topo_use& u) {
  return u.col != KSIM_COL_NONE && !use_node_count(u);
}

// TopoRow of one node over the pod's uses U[0 .. nu) (block-uniform nu; the
// domain tables are the ones k_topo_prefilter filled for this cycle).
template <typename Scratch>
__device__ __forceinline__ void load_topo_row(const DevCluster& c, const ksim_topo_use* U, int nu,
                                              const UseMasks& m, const Scratch& s, const int64_t* ptab,
                                              int32_t node, TopoRow& t) {
#pragma unroll
  for (int i = 0; i < KSIM_MAX_USES; i++) {
    uint32_t v = 0;
    if (i < nu) {
      const uint16_t col = load_use(U, i).col;
      if (col != KSIM_COL_NONE) v = c.labels[(size_t)col * c.n + node];
    }
    t.v[i] = v;
  }
#pragma unroll
  for (int i = 0; i < KSIM_MAX_USES; i++) {
    int64_t x = 0;
    if (i < nu) {
      const ksim_topo_use u = load_use(U, i);
      x = ((m.node_count >> i) & 1u) ? class_count(c, u.cls, node)
          : ((m.ptab >> i) & 1u)     ? ptab[u._pad + t.v[i]]
                                     : s.dom[(size_t)i * c.vmax + t.v[i]];
    }
    t.x[i] = x;
  }
}
// A PTS soft use that registers its topology pairs by value (not hostname).
__host__ __device__ __forceinline__ bool use_registers_values(const ksim_topo_use& u) {
  return u.kind == KSIM_USE_PTS_SOFT && u.col != KSIM_COL_NONE && !(u.flags & KSIM_USEF_HOSTNAME);
}

__host__ __device__ __forceinline__ int64_t ipa_coef(const ksim_profile& prof, const ksim_topo_use& u);

// Host side (PodPlan): U is a host array.
__host__ __device__ __forceinline__ UseMasks use_masks(const ksim_profile& prof, const ksim_topo_use* U, int nu) {
  UseMasks m{};
  for (int i = 0; i < nu; i++) {
    const ksim_topo_use u = U[i];
    const uint32_t b = 1u << i;
    if (u.kind == KSIM_USE_PTS_HARD) m.hard |= b;
    if (u.kind == KSIM_USE_PTS_SOFT) m.soft |= b;
    if (use_registers_values(u)) m.soft_val |= b;
    if (u.kind == KSIM_USE_IPA_AFFINITY) m.aff |= b;
    if (u.kind == KSIM_USE_IPA_ANTI) m.anti |= b;
    if (u.kind == KSIM_USE_IPA_EXISTING_ANTI) m.exist |= b;
    if (ipa_coef(prof, u) != 0) m.score |= b;
    if (u.kind == KSIM_USE_NODE_PORT) m.port |= b;
    if (u.kind == KSIM_USE_IMAGE) m.image |= b;
    if (use_node_count(u)) m.node_count |= b;
    if (u.flags & KSIM_USEF_SELF_MATCH) m.self_match |= b;
    if (u.flags & KSIM_USEF_HONOR_AFFINITY) m.honor_aff |= b;
    if (u.flags & KSIM_USEF_HONOR_TAINTS) m.honor_taints |= b;
  }
  m.dom = (m.hard | m.soft_val | m.aff | m.anti | m.exist | m.score) & ~m.node_count;
  for (int i = 0; i < nu; i++)
    if (U[i].col == KSIM_COL_NONE) m.dom &= ~(1u << i);
  return m;
}

// FindMatchingUntoleratedTaint straight from the taint columns (no NodeRow).
__device__ __forceinline__ bool node_has_untolerated_taint(const DevCluster& c, const ksim_pod& p, int32_t node) {
#pragma unroll
  for (int k = 0; k < KSIM_MAX_NODE_TAINTS; k++) {
    const uint32_t tid = c.taints[(size_t)k * c.n + node];
    if (!tid) break;
    const uint8_t eff = c.taint_effect[tid];
    if ((eff == KSIM_EFFECT_NO_SCHEDULE || eff == KSIM_EFFECT_NO_EXECUTE) && !bit_set(p.tol_filter, tid)) return true;
  }
  return false;
}

// topologySpreadConstraint.matchNodeInclusionPolicies
__device__ __forceinline__ bool match_node_inclusion(const DevCluster& c, const DevPods& P, const ksim_pod& p,
                                                     const ksim_topo_use& u, int32_t node) {
  if ((u.flags & KSIM_USEF_HONOR_AFFINITY) && !required_node_affinity_match(c, P, p, node)) return false;
  if ((u.flags & KSIM_USEF_HONOR_TAINTS) && node_has_untolerated_taint(c, p, node)) return false;
  return true;
}

// nodeports Filter: HostPortInfo.CheckConflict of every wanted port, compiled
// by the host to "class of pods using a conflicting (ip, protocol, port) is
// empty on the node" (ksim/topology.py port classes)
__device__ __forceinline__ bool node_port_conflict(const UseMasks& m, const TopoRow& t) {
  bool hit = false;
#pragma unroll
  for (int i = 0; i < KSIM_MAX_USES; i++)
    if (((m.port >> i) & 1u) && t.x[i] > 0) hit = true;
  return hit;
}

// imagelocality Score: calculatePriority(sumImageScores) depends only on the
// node's static image list and the pod's container images, so the host
// compiles it per image signature to a static class (ksim/topology.py).
__device__ __forceinline__ int64_t image_locality_score(const UseMasks& m, const TopoRow& t) {
  int64_t r = 0;
#pragma unroll
  for (int i = KSIM_MAX_USES - 1; i >= 0; i--)     // the first image use wins
    if ((m.image >> i) & 1u) r = t.x[i];
  return r;
}

// podtopologyspread Filter -> 0 or KSIM_PTS_*
__device__ __forceinline__ uint32_t pts_filter(const ksim_topo_use* U, const UseMasks& m, const int64_t* min_match,
                                               const TopoRow& t) {
  uint32_t why = 0;                                               // the first failing constraint's reason
#pragma unroll
  for (int i = 0; i < KSIM_MAX_USES; i++) {
    if (why != 0 || !((m.hard >> i) & 1u)) continue;
    const int64_t self = (m.self_match >> i) & 1u;
    const int64_t match = t.x[i] & kDomCountMask;                  // absent pair: 0
    if (t.v[i] == 0) why = KSIM_PTS_MISSING_LABEL;
    else if (match + self - min_match[i] > (int64_t)load_use(U, i).arg) why = KSIM_PTS_SKEW;
  }
  return why;
}

// interpodaffinity Filter -> 0 or KSIM_IPA_*
__device__ __forceinline__ uint32_t ipa_filter(const UseMasks& m, const ksim_pod& p, uint32_t topo_flags,
                                               const TopoRow& t) {
  bool pods_exist = true, missing = false, anti = false, existing = false;
#pragma unroll
  for (int i = 0; i < KSIM_MAX_USES; i++) {
    const uint32_t v = t.v[i];
    if ((m.aff >> i) & 1u) {
      if (v == 0) missing = true;
      else if (t.x[i] <= 0) pods_exist = false;
    }
    if (((m.anti >> i) & 1u) && v != 0 && t.x[i] > 0) anti = true;
    if (((m.exist >> i) & 1u) && v != 0 && t.x[i] > 0) existing = true;
  }
  if (missing) return KSIM_IPA_AFFINITY;
  if (m.aff && !pods_exist &&
      !(!(topo_flags & kTopoAffinityNonEmpty) && (p.topo_flags & KSIM_POD_IPA_SELF_AFFINITY)))
    return KSIM_IPA_AFFINITY;
  if (anti) return KSIM_IPA_ANTI_AFFINITY;
  if (existing) return KSIM_IPA_EXISTING_ANTI;
  return 0;
}

__device__ __forceinline__ bool use_has_kind(const DevPods& P, const ksim_pod& p, int k0, int k1 = -1, int k2 = -1) {
  for (int i = 0; i < p.use_count; i++) {
    const int k = P.uses[p.use_first + i].kind;
    if (k == k0 || k == k1 || k == k2) return true;
  }
  return false;
}

__host__ __device__ __forceinline__ int64_t ipa_coef(const ksim_profile& prof, const ksim_topo_use& u) {
  if (u.kind == KSIM_USE_IPA_SCORE) return u.arg;
  if (u.kind == KSIM_USE_IPA_SCORE_HARD) return prof.hard_pod_affinity_weight > 0 ? prof.hard_pod_affinity_weight : 0;
  return 0;
}

// interpodaffinity Score
__device__ __forceinline__ int64_t ipa_score(const ksim_profile& prof, const ksim_topo_use* U, const UseMasks& m,
                                             const TopoRow& t) {
  int64_t sc = 0;
#pragma unroll
  for (int i = 0; i < KSIM_MAX_USES; i++)
    if (((m.score >> i) & 1u) && t.v[i] != 0) sc += ipa_coef(prof, load_use(U, i)) * t.x[i];
  return sc;
}

// The persistent domain tables of class cls follow a change of its count on
// node (concurrent binds of one batch may share a table entry: atomics).
__device__ __forceinline__ void ptab_add(const DevCluster& c, const DevPods& P, int32_t cls, int32_t node,
                                         int64_t delta) {
  if (!P.ptab_cfirst) return;
  const int32_t e1 = P.ptab_cfirst[cls + 1];
  for (int32_t e = P.ptab_cfirst[cls]; e < e1; e++) {
    const int4 t = P.ptab_ent[P.ptab_cidx[e]];
    const uint32_t v = c.labels[(size_t)t.y * c.n + node];
    if (v) atomicAdd(reinterpret_cast<unsigned long long*>(P.ptab + t.w + (t.z == kPtabTotal ? 0u : v)),
                     (unsigned long long)delta);
  }
}

// NodeInfo.AddPod / RemovePod on the count classes
__device__ __forceinline__ void apply_adds(const DevCluster& c, const DevPods& P, const ksim_pod& p, int32_t node,
                                           int sign) {
  for (int i = 0; i < p.add_count; i++) {
    const ksim_class_add a = P.adds[p.add_first + i];
    c.cnt[(size_t)a.cls * c.n + node] += sign * a.count;
    ptab_add(c, P, a.cls, node, (int64_t)sign * a.count);
  }
}

// ---- batch path: the profile compiled down to what batchable pods need -----
// Batchable pods (see pod_batchable in ksim_engine.cpp) pass every filter
// plugin except the ones listed here, and their normalized scores are a
// per-pod constant, so a key is
//   static filters (bind-invariant) -> Fit filter -> w_fit*LeastAllocated +
//   w_ba*BalancedAllocation + constant -> TB key.
struct BatchProg {
  int32_t n_static;                        // static (bind-invariant) filters, profile order
  uint8_t static_filter[KSIM_MAX_FILTER];
  int32_t has_fit_filter;
  int32_t cpu_mem;                         // both scoring strategies are exactly {cpu, memory}
  int64_t w_fit, w_ba;                     // summed profile weights of the Fit / BA score slots
  int64_t w_tt, w_na;                      // ... of the TaintToleration / NodeAffinity slots (norm_part)
  int64_t fit_w_cpu, fit_w_mem;            // cpu_mem: LeastAllocated resource weights
  int32_t fast_w;                          // cpu_mem with both LeastAllocated weights in [1, 2^31) (dyn_key_fast)
  int32_t no_score;                        // the profile has no score plugin: every total is 1
  int32_t fit_w_eq;                        // fast_w and fit_w_cpu == fit_w_mem: the mean is a halving
  int32_t _pad;
  double inv_w[3];                         // RN(1 / w) of fit_w_cpu, fit_w_mem, their sum (dyn_key_fast)
  // per-pod cycle (plan_profile): filter position / score slot per plugin id
  uint64_t rank_lo, rank_hi, slot;
  uint32_t slot_hi, _pad2;
};

// The FAST key with the default profile's shape compiled in (dyn_key_fast_t<true>):
// a Fit filter, equal LeastAllocated weights (fit_w_eq), a score plugin, and
// Fit / BA score weights in [0, 2^14) (24-bit multiplies).  The launch picks
// the kernel by it, so a profile change that flips it drops the batch graphs.
__host__ __device__ inline bool fast_def(const BatchProg& bp) {
  return bp.has_fit_filter && bp.fit_w_eq && !bp.no_score && bp.w_fit >= 0 && bp.w_fit < (1 << 14) &&
         bp.w_ba >= 0 && bp.w_ba < (1 << 14);
}

// DevPods.bflags (batch path, per pod)
constexpr int32_t kBatchStaticTrivial = 1; // every static filter passes on every node (host-proven)
constexpr int32_t kPodRegistersValues = 2; // has a ScheduleAnyway spread keyed by a non-hostname column
constexpr int32_t kPodNormVaries = 4;      // batch path: TaintToleration / NodeAffinity vary over nodes (norm_part)
constexpr int32_t kPodTopoBatch = 8;       // topology batch path (ksim_tbatch.hip)
constexpr int32_t kPodTbCross = 16;       // topology batch run from this pod crosses a class conflict (node-local)
constexpr int kTlenShift = 8;              // (bflags >> kTlenShift) & kTlenMask: topology batch run length from this pod
constexpr int kTlenPlainShift = 16;        // ... without zone variants (replicated topology batches)
constexpr int32_t kTlenMask = 255;

// Compact row for the batch repair's LDS staging: the NodeRow fields a
// batchable pod can read (batchable pods request no scalar resources and the
// scoring strategies use cpu / memory / ephemeral-storage only).  96 bytes.
struct BRow {
  int64_t alloc_cpu, alloc_mem, alloc_eph;
  int64_t req_cpu, req_mem, req_eph;
  int64_t nz_cpu, nz_mem;
  int32_t alloc_pods, num_pods;
  uint32_t flags;
  int32_t node;
  uint32_t taints[KSIM_MAX_NODE_TAINTS / 2];
};
static_assert(sizeof(BRow) == 96, "BRow layout");

__device__ __forceinline__ BRow to_brow(const NodeRow& r) {
  BRow b;
  b.alloc_cpu = r.alloc_cpu; b.alloc_mem = r.alloc_mem; b.alloc_eph = r.alloc_eph;
  b.req_cpu = r.req_cpu; b.req_mem = r.req_mem; b.req_eph = r.req_eph;
  b.nz_cpu = r.nz_cpu; b.nz_mem = r.nz_mem;
  b.alloc_pods = r.alloc_pods; b.num_pods = r.num_pods; b.flags = r.flags; b.node = r.node;
#pragma unroll
  for (int k = 0; k < KSIM_MAX_NODE_TAINTS / 2; k++) b.taints[k] = r.taints[k];
  return b;
}

__device__ __forceinline__ NodeRow from_brow(const BRow& b) {
  NodeRow r;
  r.alloc_cpu = b.alloc_cpu; r.alloc_mem = b.alloc_mem; r.alloc_eph = b.alloc_eph;
  r.req_cpu = b.req_cpu; r.req_mem = b.req_mem; r.req_eph = b.req_eph;
  r.nz_cpu = b.nz_cpu; r.nz_mem = b.nz_mem;
  r.alloc_pods = b.alloc_pods; r.num_pods = b.num_pods; r.flags = b.flags; r.node = b.node;
#pragma unroll
  for (int k = 0; k < KSIM_MAX_SCALAR; k++) { r.alloc_sc[k] = 0; r.req_sc[k] = 0; }
#pragma unroll
  for (int k = 0; k < KSIM_MAX_NODE_TAINTS / 2; k++) r.taints[k] = b.taints[k];
  return r;
}

__device__ __forceinline__ void brow_add_pod(BRow& r, const ksim_pod& p) {
  r.req_cpu += p.req_cpu;
  r.req_mem += p.req_mem;
  r.req_eph += p.req_eph;
  r.nz_cpu += p.nz_cpu;
  r.nz_mem += p.nz_mem;
  r.num_pods += 1;
}

// dst = src + pod (NodeInfo.AddPod), field by field (src may alias dst).
__device__ __forceinline__ void brow_assign_add(BRow& dst, const BRow& src, const ksim_pod& p) {
  const int64_t rc = src.req_cpu + p.req_cpu, rm = src.req_mem + p.req_mem, re = src.req_eph + p.req_eph;
  const int64_t zc = src.nz_cpu + p.nz_cpu, zm = src.nz_mem + p.nz_mem;
  const int64_t ac = src.alloc_cpu, am = src.alloc_mem, ae = src.alloc_eph;
  const int32_t ap = src.alloc_pods, np = src.num_pods + 1, nd = src.node;
  const uint32_t fl = src.flags, t0 = src.taints[0], t1 = src.taints[1], t2 = src.taints[2], t3 = src.taints[3];
  dst.alloc_cpu = ac; dst.alloc_mem = am; dst.alloc_eph = ae;
  dst.req_cpu = rc; dst.req_mem = rm; dst.req_eph = re;
  dst.nz_cpu = zc; dst.nz_mem = zm;
  dst.alloc_pods = ap; dst.num_pods = np; dst.flags = fl; dst.node = nd;
  dst.taints[0] = t0; dst.taints[1] = t1; dst.taints[2] = t2; dst.taints[3] = t3;
}

__device__ __forceinline__ void store_brow_dynamic(const DevCluster& c, const BRow& r) {
  const int32_t node = r.node;
  c.req_cpu[node] = r.req_cpu;
  c.req_mem[node] = r.req_mem;
  c.req_eph[node] = r.req_eph;
  c.nz_cpu[node] = r.nz_cpu;
  c.nz_mem[node] = r.nz_mem;
  c.num_pods[node] = r.num_pods;
}

__device__ __forceinline__ bool static_filters_pass(const DevCluster& c, const DevPods& P, const BatchProg& bp,
                                           const ksim_pod& p, const NodeRow& r) {
  for (int f = 0; f < bp.n_static; f++) {
    switch (bp.static_filter[f]) {
      case KSIM_PL_NODE_UNSCHEDULABLE:
        if ((r.flags & KSIM_NODE_UNSCHEDULABLE) && !(p.flags & KSIM_POD_TOLERATES_UNSCHEDULABLE)) return false;
        break;
      case KSIM_PL_NODE_NAME:
        if (p.node_name != -1 && p.node_name != c.base + r.node) return false;
        break;
      case KSIM_PL_TAINT_TOLERATION:
        if (find_matching_untolerated_taint(c, p, r)) return false;
        break;
      case KSIM_PL_NODE_AFFINITY: {
        uint32_t why;
        if (!node_affinity_filter(c, P, p, r.node, why)) return false;
        break;
      }
      default:
        break;
    }
  }
  return true;
}

// dyn_key for the default scoring strategies ({cpu, memory} for both
// LeastAllocated and BalancedAllocation; batchable pods request no scalars):
// the same arithmetic as the generic functions with the resource loops
// resolved, so the batch kernels stay small.  The key's total leaves out the
// pod's constant normalized scores (the same on every node), so it lies in
// [0, 100 * (w_fit + w_ba)] < kKeyTotalLimit (pod_batchable checks the bound).
__device__ __forceinline__ uint64_t dyn_key_cpu_mem(const ksim_profile& prof, const BatchProg& bp,
                                                    const ksim_pod& p, const NodeRow& r,
                                                    int64_t seq, int32_t base) {
  if (bp.has_fit_filter) {
    if (r.num_pods + 1 > r.alloc_pods) return 0;
    if (p.req_cpu != 0 || p.req_mem != 0 || p.req_eph != 0) {
      if (p.req_cpu > r.alloc_cpu - r.req_cpu || p.req_mem > r.alloc_mem - r.req_mem ||
          p.req_eph > r.alloc_eph - r.req_eph)
        return 0;
    }
  }
  int64_t tot = 0;
  if (bp.w_fit) {                              // leastResourceScorer over {cpu, memory}
    int64_t ns = 0, ws = 0;
    if (r.alloc_cpu != 0) {
      ns += least_requested_q100(r.nz_cpu + p.nz_cpu, r.alloc_cpu) * bp.fit_w_cpu;
      ws += bp.fit_w_cpu;
    }
    if (r.alloc_mem != 0) {
      ns += least_requested_q100(r.nz_mem + p.nz_mem, r.alloc_mem) * bp.fit_w_mem;
      ws += bp.fit_w_mem;
    }
    // the weighted mean of scores in [0, 100] is a score-sized quotient (a
    // wrapped leastRequestedScore of a capacity past 2^56 may leave that range)
    const int64_t la = ws == 0 ? 0 : (ns < 0 || ws <= 0 || ns > kMaxNodeScore * ws) ? ns / ws : div_q100(ns, ws);
    tot += bp.w_fit * la;
  }
  if (bp.w_ba) {                               // balancedResourceScorer over {cpu, memory}
    double f0 = 0, f1 = 0;
    int nf = 0;
    if (r.alloc_cpu != 0) {
      double f = (double)(r.req_cpu + p.req_cpu) / (double)r.alloc_cpu;
      f0 = f > 1 ? 1 : f;
      nf++;
    }
    if (r.alloc_mem != 0) {
      double f = (double)(r.req_mem + p.req_mem) / (double)r.alloc_mem;
      if (nf == 0) f0 = f > 1 ? 1 : f;
      else f1 = f > 1 ? 1 : f;
      nf++;
    }
    const double std = nf == 2 ? fabs((f0 - f1) / 2) : 0.0;
    tot += bp.w_ba * (int64_t)((1 - std) * (double)kMaxNodeScore);
  }
  if (prof.n_score == 0) tot = 1;
  return tb_key(tot, prof.tiebreak_seed, seq, base + r.node);
}

// The correctly rounded quotient n / d (the IEEE division's result) from
// y = RN(1 / d): q0 = RN(n y) is within an ulp of n / d, the FMA residual
// n - q0 d is exact, and one FMA correction rounds correctly (Markstein's
// theorem; operands here are integers far from overflow and underflow).  The
// FMAs are explicit: they emulate a division, they do not contract any of the
// plugins' own float64 expressions (-ffp-contract=off still holds for those).
__device__ __forceinline__ double div_rn(double n, double d, double y) {
  const double q0 = n * y;
  const double e = __builtin_fma(-q0, d, n);
  return __builtin_fma(e, y, q0);
}

// The FAST key (k_batch_top<true>, k_batch_chain_pairs<true>): trivial pods (every
// static filter host-proven to pass), {cpu, memory} strategies with
// LeastAllocated weights in [1, 2^31) (BatchProg::fast_w), allocatable cpu and
// memory in [0, 2^46) on every node (checked at ksim_set_cluster).  Then each
// leastRequestedScore quotient n / d has integers n < 2^53, 0 < d < 2^46, and
// the truncation of the correctly rounded float64 quotient IS the integer
// quotient: an integer quotient is exact, any other lies at least 1/d > 2^-46
// below the next integer while the rounding error of a quotient below 128 is
// at most 2^-47.  The same bound covers the weighted mean (n < 2^40, d < 2^32).
// Each division is div_rn with the host's RN(1 / d) (DevCluster inv_cpu /
// inv_mem, BatchProg inv_w): three float64 operations instead of a 64-bit division and
// its correction steps, and for BalancedAllocation bit for bit the float64
// quotient Go computes.  hseed = seed ^ (seq << 20), the pod's part of the
// tie-break hash.
// An integer in [0, 2^52) as a double, exactly: the bits of 2^52 + x minus
// 2^52 (one OR and one add, where the general int64 conversion takes two
// conversions, a scale and an add).  Every value the FAST keys convert is
// below 2^46 (kClusterNarrow allocatables; sums bounded by them, see callers).
__device__ __forceinline__ double u52_to_f64(int64_t x) {
  return __longlong_as_double(x | 0x4330000000000000LL) - 4503599627370496.0;
}

// leastResourceScorer over {cpu, memory} (BatchProg::fast_w, kClusterNarrow).
// (alloc - requested) * 100 is an integer below 2^53, so the double product of
// the converted difference and 100 is exact, as the int64 product converted is.
// Branch-free: every quotient is computed and the plugin's conditions select
// (a quotient of a zero or overdrawn capacity is garbage that is never
// selected; v_cvt_i32_f64 does not trap).  The batch kernels keep their lanes
// convergent this way: no exec-mask branches, no per-branch SALU work.
__device__ __forceinline__ FastProg fast_prog(const BatchProg& bp) {
  FastProg f;
  f.fit = bp.has_fit_filter;
  f.w_fit = (int32_t)bp.w_fit;
  f.w_ba = (int32_t)bp.w_ba;
  f.w_eq = bp.fit_w_eq;
  f.no_score = bp.no_score;
  f.fw_cpu = bp.fit_w_cpu;
  f.fw_mem = bp.fit_w_mem;
  f.iw_cpu = bp.inv_w[0];
  f.iw_mem = bp.inv_w[1];
  f.iw_sum = bp.inv_w[2];
  return f;
}

template <bool DEF>
__device__ __forceinline__ int32_t fast_least_allocated(const FastProg& q, const ksim_pod& p, const NodeRow& r,
                                                        double inv_c, double inv_m) {
  const bool hc = r.alloc_cpu != 0, hm = r.alloc_mem != 0;
  const int64_t dc = r.alloc_cpu - (r.nz_cpu + p.nz_cpu), dm = r.alloc_mem - (r.nz_mem + p.nz_mem);
  const double ac = u52_to_f64(r.alloc_cpu), am = u52_to_f64(r.alloc_mem);
  const int32_t qc = (int32_t)div_rn(u52_to_f64(dc) * (double)kMaxNodeScore, ac, inv_c);
  const int32_t qm = (int32_t)div_rn(u52_to_f64(dm) * (double)kMaxNodeScore, am, inv_m);
  const int32_t sc = (hc && dc >= 0) ? qc : 0;   // requested > capacity scores 0
  const int32_t sm = (hm && dm >= 0) ? qm : 0;
  if (DEF || q.w_eq) return (hc && hm) ? (sc + sm) >> 1 : hc ? sc : sm;   // (sc w + sm w) / (2 w)
  // selects of values (a select of the struct members' lvalues becomes an
  // address select, and the struct a per-lane copy in LDS)
  const int64_t fwc = q.fw_cpu, fwm = q.fw_mem;
  const double iws = q.iw_sum, iwc = q.iw_cpu, iwm = q.iw_mem;
  const int64_t wc = hc ? fwc : 0, wm = hm ? fwm : 0;
  const double inv = (hc && hm) ? iws : hc ? iwc : iwm;
  const int32_t v = (int32_t)div_rn((double)(sc * wc + sm * wm), (double)(wc + wm), inv);
  return (hc || hm) ? v : 0;
}

// balancedResourceScorer over {cpu, memory}: the float64 quotients Go computes.
// With a Fit filter in the profile it passed, so requested + request <=
// allocatable < 2^46 and the short conversion is exact (without one the sums
// are unbounded and take the general conversion).  With one resource missing
// the standard deviation is 0 (score 100), as with both present and equal.
template <bool DEF>
__device__ __forceinline__ int32_t fast_balanced_allocation(const FastProg& q, const ksim_pod& p, const NodeRow& r,
                                                            double inv_c, double inv_m) {
  const bool hc = r.alloc_cpu != 0, hm = r.alloc_mem != 0;
  const int64_t qc = r.req_cpu + p.req_cpu, qm = r.req_mem + p.req_mem;
  const bool fit = DEF || q.fit;
  const double fc = fmin(div_rn(fit ? u52_to_f64(qc) : (double)qc, u52_to_f64(r.alloc_cpu), inv_c), 1.0);
  const double fm = fmin(div_rn(fit ? u52_to_f64(qm) : (double)qm, u52_to_f64(r.alloc_mem), inv_m), 1.0);
  const int32_t b = (int32_t)((1 - fabs((fc - fm) / 2)) * (double)kMaxNodeScore);
  return (hc && hm) ? b : kMaxNodeScore;
}

// DEF (fast_def(bp) on the host): a Fit filter, equal LeastAllocated weights,
// at least one score plugin and both score weights below 2^14, so the key's
// shape is compiled in: no uniform branches in the node loop, and the weights
// scale the scores by 24-bit multiplies (w * 100 < 2^21) instead of 32-bit ones.
template <bool DEF>
__device__ __forceinline__ uint64_t dyn_key_fast_t(const FastProg& q, const ksim_pod& p, const NodeRow& r,
                                                   double inv_c, double inv_m, uint64_t hseed, int32_t gnode) {
  // the Fit filter with non-short-circuit operators: one select, no branches
  // (the request's zero test is uniform across the wave)
  const bool any = (p.req_cpu | p.req_mem | p.req_eph) != 0;
  const bool fits = (p.req_cpu <= r.alloc_cpu - r.req_cpu) & (p.req_mem <= r.alloc_mem - r.req_mem) &
                    (p.req_eph <= r.alloc_eph - r.req_eph);
  const bool ok = !(DEF || q.fit) | ((r.num_pods < r.alloc_pods) & (!any | fits));
  int32_t tot = 0;
  if constexpr (DEF) {
    // the masks change no value (weights < 2^14, scores in [0, 100]); they let
    // the compiler prove both factors narrow and pick v_mul_u32_u24
    const uint32_t la = (uint32_t)fast_least_allocated<true>(q, p, r, inv_c, inv_m) & 0xffffu;
    const uint32_t ba = (uint32_t)fast_balanced_allocation<true>(q, p, r, inv_c, inv_m) & 0xffffu;
    tot = (int32_t)(((uint32_t)q.w_fit & 0x3fffu) * la + ((uint32_t)q.w_ba & 0x3fffu) * ba);
  } else {
    if (q.w_fit) tot += q.w_fit * fast_least_allocated(q, p, r, inv_c, inv_m);
    if (q.w_ba) tot += q.w_ba * fast_balanced_allocation(q, p, r, inv_c, inv_m);
    if (q.no_score) tot = 1;
  }
  const uint64_t h = splitmix64(hseed ^ (uint64_t)(uint32_t)gnode) >> 38;
  const uint64_t key = ((uint64_t)(uint32_t)tot << 44) | (h << 18) | (uint64_t)(KSIM_KEY_NODE_MASK - gnode);
  return ok ? key : 0;
}

__device__ __forceinline__ uint64_t dyn_key_fast(const FastProg& q, const ksim_pod& p, const NodeRow& r,
                                                 double inv_c, double inv_m, uint64_t hseed, int32_t gnode) {
  return dyn_key_fast_t<false>(q, p, r, inv_c, inv_m, hseed, gnode);
}

// The request fields the FAST pair key reads (pod j's and the bound pod k's),
// as a local ksim_pod: a caller can load them before it knows the guesses.
__device__ __forceinline__ ksim_pod fast_pod_fields(const ksim_pod& g) {
  ksim_pod p;
  p.req_cpu = g.req_cpu;
  p.req_mem = g.req_mem;
  p.req_eph = g.req_eph;
  p.nz_cpu = g.nz_cpu;
  p.nz_mem = g.nz_mem;
#pragma unroll
  for (int k = 0; k < KSIM_MAX_SCALAR; k++) p.scalar_req[k] = 0;   // trivial pods: no scalar requests
  return p;
}

__device__ __forceinline__ uint64_t dyn_key_fast(const BatchProg& bp, const ksim_pod& p, const NodeRow& r,
                                                 double inv_c, double inv_m, uint64_t hseed, int32_t gnode) {
  return dyn_key_fast(fast_prog(bp), p, r, inv_c, inv_m, hseed, gnode);
}

// Key of a batchable pod on a row whose static filters passed (0 = infeasible).
// Pods with scalar requests take the generic functions (their Fit filter
// checks the scalar columns).
__device__ __forceinline__ uint64_t dyn_key(const ksim_profile& prof, const BatchProg& bp, const ksim_pod& p,
                                            const NodeRow& r, int n_scalar, int64_t seq, int32_t base,
                                            uint32_t ignore) {
  if (bp.cpu_mem && !(p.flags & KSIM_POD_HAS_SCALAR)) return dyn_key_cpu_mem(prof, bp, p, r, seq, base);
  if (bp.has_fit_filter && fits_request(r, p, n_scalar, ignore)) return 0;
  int64_t tot = 0;
  if (bp.w_fit) tot += bp.w_fit * fit_score(r, prof, p, n_scalar);
  if (bp.w_ba) tot += bp.w_ba * balanced_allocation_score(r, prof, p, n_scalar);
  if (prof.n_score == 0) tot = 1;
  return tb_key(tot, prof.tiebreak_seed, seq, base + r.node);
}

// kPodNormVaries pods (P100 batch path): the raw scores of the two normalized
// plugins that can vary over nodes for a batchable pod.  Both depend on the
// node's taints and labels only, never on what is bound there.
struct NormRaw {
  int64_t tt, na;   // countIntolerableTaintsPreferNoSchedule, preferred NodeAffinity weight sum
};
// The raw normalized scores of pod p from a static-table word of its class
// (DevPods::stab): the taint count, and the weights of the matching terms
// (preferred_node_affinity_score; the term count and weights are uniform).
__device__ __forceinline__ NormRaw stab_raw(uint64_t w, const DevPods& P, const ksim_pod& p) {
  int64_t na = 0;
  for (int k = 0; k < p.pref_term_count; k++)
    na += ((w >> k) & 1ull) ? (int64_t)P.terms[p.pref_term_first + k].weight : 0;
  return NormRaw{(int64_t)((w >> 32) & 0x7fffffffull), na};
}
// The static-table word's match bits of pod p's preferred terms on a node.
__device__ __forceinline__ uint32_t pref_term_mask(const DevCluster& c, const DevPods& P, const ksim_pod& p,
                                                   int32_t node) {
  uint32_t m = 0;
  for (int k = 0; k < p.pref_term_count && k < 32; k++) {
    const ksim_term& t = P.terms[p.pref_term_first + k];
    if (t.weight != 0 && term_matches(c, P, t, node)) m |= 1u << k;
  }
  return m;
}
__device__ __forceinline__ NormRaw norm_raw(const DevCluster& c, const DevPods& P, const ksim_pod& p,
                                            const NodeRow& r) {
  return NormRaw{count_intolerable_prefer(c, p, r), p.pref_term_count ? preferred_node_affinity_score(c, P, p, r.node) : 0};
}
// Their weighted NormalizeScore over the pod's S0 maxima (mx): added to the
// batch key's total.  Exact while the maxima hold: a node's raw scores never
// change with binds, and the maxima only change when a node holding one
// leaves the pod's feasible set (pairs_block flags that pod, pinv).
__device__ __forceinline__ int64_t norm_part(const BatchProg& bp, const NormRaw& v, const NormRaw& mx) {
  return bp.w_tt * normalize_value(kNormDefaultReverse, v.tt, mx.tt, 0, false) +
         bp.w_na * normalize_value(kNormDefault, v.na, mx.na, 0, false);
}

// norm_part of a static-table word for the FAST keys of a static class
// (at most 32 terms of weights in [0, 2^31), so both raw scores lie in
// [0, 2^36)): each quotient 100 v / m through div_rn with y = RN(1 / m).
// n = 100 v < 2^43 and 0 < m < 2^36, so the truncated correctly rounded
// quotient is the integer quotient (as for the FAST key's quotients: a
// non-integer quotient lies at least 1 / m below the next integer, the
// rounding error of one below 128 is at most 2^-45).  y_tt / y_na: the caller's RN(1 / mx.tt), RN(1 / mx.na).
__device__ __forceinline__ int64_t norm_part_fast(const BatchProg& bp, const NormRaw& v, const NormRaw& mx,
                                                  double y_tt, double y_na) {
  const int64_t qt = (int64_t)div_rn((double)(kMaxNodeScore * v.tt), (double)mx.tt, y_tt);
  const int64_t qa = (int64_t)div_rn((double)(kMaxNodeScore * v.na), (double)mx.na, y_na);
  const int64_t nt = mx.tt > 0 ? (int64_t)kMaxNodeScore - qt : (int64_t)kMaxNodeScore;
  const int64_t na = mx.na > 0 ? qa : v.na;
  return bp.w_tt * nt + bp.w_na * na;
}
__device__ __forceinline__ double recip_or_zero(int64_t m) { return m > 0 ? 1.0 / (double)m : 0.0; }

__device__ __forceinline__ void row_add_pod(NodeRow& r, const ksim_pod& p, int sign) {
  r.req_cpu += sign * p.req_cpu;
  r.req_mem += sign * p.req_mem;
  r.req_eph += sign * p.req_eph;
#pragma unroll
  for (int k = 0; k < KSIM_MAX_SCALAR; k++) r.req_sc[k] += sign * p.scalar_req[k];
  r.nz_cpu += sign * p.nz_cpu;
  r.nz_mem += sign * p.nz_mem;
  r.num_pods += sign;
}

__device__ __forceinline__ void assume_pod(const DevCluster& c, const DevPods& P, const ksim_pod& p, int32_t node,
                                           int sign) {
  apply_adds(c, P, p, node, sign);
  c.req_cpu[node] += sign * p.req_cpu;
  c.req_mem[node] += sign * p.req_mem;
  c.req_eph[node] += sign * p.req_eph;
  for (int k = 0; k < c.n_scalar; k++) c.req_scalar[(size_t)k * c.n + node] += sign * p.scalar_req[k];
  c.nz_cpu[node] += sign * p.nz_cpu;
  c.nz_mem[node] += sign * p.nz_mem;
  c.num_pods[node] += sign;
  if (p.nb_add) c.nb_alloc[node] += sign * p.nb_add;
}

// assume_pod without the six resource columns (the batch commit updates those
// from a row it loaded ahead): class adds, scalar resources, bandwidth.
__device__ __forceinline__ void assume_pod_rest(const DevCluster& c, const DevPods& P, const ksim_pod& p, int32_t node,
                                                int sign) {
  apply_adds(c, P, p, node, sign);
  for (int k = 0; k < c.n_scalar; k++) c.req_scalar[(size_t)k * c.n + node] += sign * p.scalar_req[k];
  if (p.nb_add) c.nb_alloc[node] += sign * p.nb_add;
}

// assume_pod_rest without the class adds (a topology batch commit applies
// those for all its pods at once): scalar resources, bandwidth.
__device__ __forceinline__ void assume_pod_cols(const DevCluster& c, const ksim_pod& p, int32_t node) {
  for (int k = 0; k < c.n_scalar; k++) c.req_scalar[(size_t)k * c.n + node] += p.scalar_req[k];
  if (p.nb_add) c.nb_alloc[node] += p.nb_add;
}

// Returnless 64-bit atomic add (two's complement: wraps as the plain add does).
__device__ __forceinline__ void atomic_add_i64(int64_t* x, int64_t v) {
  atomicAdd(reinterpret_cast<unsigned long long*>(x), (unsigned long long)v);
}

// assume_pod by one wave (every lane calls it): one lane per column, each a
// returnless atomic add (one writer per column: the same result as a
// read-modify-write, without waiting for the read; the per-pod bind at the end
// of k_select: 26.9 -> 26.3 us per pod on config 3, same-box A/B.  The batch
// commit's one-thread-per-pod binds keep plain read-modify-writes: atomics
// there cost 9.23 -> 9.86 ms per config-2 step).  A pod's class adds name
// distinct classes.  ``add0``: this lane's first class add (lane < add_count),
// loaded by the caller ahead of the node choice.
__device__ __forceinline__ void assume_pod_wave(const DevCluster& c, const DevPods& P, const ksim_pod& p, int32_t node,
                                                int sign, bool tables = true, const ksim_class_add* add0 = nullptr) {
  const int lane = threadIdx.x & 63;
  if (lane == 0) atomic_add_i64(&c.req_cpu[node], sign * p.req_cpu);
  if (lane == 1) atomic_add_i64(&c.req_mem[node], sign * p.req_mem);
  if (lane == 2) atomic_add_i64(&c.req_eph[node], sign * p.req_eph);
  if (lane == 3) atomic_add_i64(&c.nz_cpu[node], sign * p.nz_cpu);
  if (lane == 4) atomic_add_i64(&c.nz_mem[node], sign * p.nz_mem);
  if (lane == 5) atomicAdd(&c.num_pods[node], sign);
  if (lane == 6 && p.nb_add) atomic_add_i64(&c.nb_alloc[node], sign * p.nb_add);
  if (lane >= 8 && lane < 8 + c.n_scalar) {
    const int k = lane - 8;
    int64_t q = 0;
#pragma unroll
    for (int j = 0; j < KSIM_MAX_SCALAR; j++)
      if (j == k) q = p.scalar_req[j];
    atomic_add_i64(&c.req_scalar[(size_t)k * c.n + node], sign * q);
  }
  for (int i = lane; i < p.add_count; i += 64) {
    const ksim_class_add a = (add0 && i == lane) ? *add0 : P.adds[p.add_first + i];
    atomicAdd(&c.cnt[(size_t)a.cls * c.n + node], sign * a.count);
    if (tables) ptab_add(c, P, a.cls, node, (int64_t)sign * a.count);
  }
}

__device__ __forceinline__ void store_row_dynamic(const DevCluster& c, const NodeRow& r) {
  const int32_t node = r.node;
  c.req_cpu[node] = r.req_cpu;
  c.req_mem[node] = r.req_mem;
  c.req_eph[node] = r.req_eph;
  for (int k = 0; k < c.n_scalar; k++) c.req_scalar[(size_t)k * c.n + node] = r.req_sc[k];
  c.nz_cpu[node] = r.nz_cpu;
  c.nz_mem[node] = r.nz_mem;
  c.num_pods[node] = r.num_pods;
}

}  // namespace ksim
