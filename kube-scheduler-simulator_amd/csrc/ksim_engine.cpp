// ksim_engine.cpp — host runtime behind the C ABI (include/ksim_engine.h).
//
// Owns the HBM-resident snapshot (SoA node columns, vocabularies), the pod
// queue, the per-cycle scratch and one HIP stream.  Batch runs are split into
// maximal runs of pods the speculative batch path can take (P100 and no
// node-varying normalized score) and runs that need the per-pod path; each
// path is a captured hipGraph replayed until the run's cursor is consumed.
// Every input is validated on the host before any kernel sees it (a bad index
// must never reach the device), copied during the call, never retained.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <tuple>
#include <unordered_map>
#include <type_traits>
#include <vector>

#include "ksim_internal.h"

using namespace ksim;

namespace {

constexpr int kGraphCycles = 128;      // per-pod cycles per captured graph

// RCCL, resolved at run time: the process may already hold torch's librccl
// (RTLD_NOLOAD finds it first, so both share one RCCL and one HIP runtime).
struct Rccl {
  bool ok = false;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
};

const Rccl& rccl() {
  static Rccl r = [] {
    Rccl x;
    void* lib = nullptr;
    for (const char* name : {"librccl.so", "librccl.so.1"})
      if (!lib) lib = dlopen(name, RTLD_NOW | RTLD_NOLOAD);
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
      if (!lib) lib = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
    if (!lib) return x;
    x.get_unique_id = (decltype(x.get_unique_id))dlsym(lib, "ncclGetUniqueId");
    x.comm_init_rank = (decltype(x.comm_init_rank))dlsym(lib, "ncclCommInitRank");
    x.comm_destroy = (decltype(x.comm_destroy))dlsym(lib, "ncclCommDestroy");
    x.all_gather = (decltype(x.all_gather))dlsym(lib, "ncclAllGather");
    x.all_reduce = (decltype(x.all_reduce))dlsym(lib, "ncclAllReduce");
    x.error_string = (decltype(x.error_string))dlsym(lib, "ncclGetErrorString");
    x.ok = x.get_unique_id && x.comm_init_rank && x.comm_destroy && x.all_gather && x.all_reduce && x.error_string;
    return x;
  }();
  return r;
}
constexpr int kGraphBatches = 16;      // speculative batches per captured graph

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

// A device buffer reused across calls, grown (never shrunk) on demand: the
// per-call uploads of the framework-driven calls (one pod, its terms and uses)
// without a hipMalloc / hipFree pair per call.
struct DevArena {
  void* p = nullptr;
  size_t cap = 0;
};

}  // namespace

// One pod (re-based) as a device pod set of its own, packed the way it is
// uploaded: every piece at a 64-byte aligned offset of one blob.
struct PodBlob {
  std::vector<char> bytes;
  size_t off[8];
  int32_t n_nn, n_exprs, n_terms, n_uses, n_adds;
};

struct ksim_handle {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  std::string err;

  bool has_profile = false;
  ksim_profile prof{};
  BatchProg bp{};
  // device copies of prof / bp, read by the batch-path kernels: a captured
  // batch graph then survives a weight change (ksim_set_profile)
  ksim_profile* d_prof = nullptr;
  BatchProg* d_bp = nullptr;
  std::vector<size_t> pod_buf_bytes;    // sizes of pod_bufs (ksim_load_pods reuses same-sized buffers)

  bool has_cluster = false;
  DevCluster dc{};
  std::vector<DevBuf> cluster_bufs;
  std::vector<uint8_t> taint_effect;    // host copy (batchability analysis)
  std::vector<uint16_t> hard_taints;    // taint ids with effect NoSchedule/NoExecute on some node
  bool any_unschedulable = false;       // some node has spec.unschedulable
  bool alloc_narrow = false;            // every allocatable cpu / memory in [0, 2^46) (dyn_key_fast)

  // device copy of the uploaded dynamic columns (ksim_reset_cluster)
  struct {
    int64_t *req_cpu, *req_mem, *req_eph, *req_scalar, *nz_cpu, *nz_mem;
    int32_t *num_pods, *cnt;
    int64_t* nb_alloc;
  } init{};
  std::vector<int32_t> col_nvals;       // host copy (pod validation)
  std::vector<uint8_t> col_unique;      // host copy of DevCluster.col_unique (kUseUniqueCol on upload)
  std::vector<uint8_t> col_total;       // per label column: every node carries the key

  DevScratch sc{};
  DevEvalOut eo{};
  std::vector<DevBuf> scratch_bufs;

  DevState* st = nullptr;
  int32_t run_hdr[2] = {0, 0};

  // loaded pod queue (batch mode)
  DevPods dp{};
  int32_t* d_chosen = nullptr;
  std::vector<DevBuf> pod_bufs;
  std::vector<uint8_t> batchable;       // per loaded pod
  std::vector<uint8_t> topo;            // per loaded pod: 0 no topology uses, 1 uses (k_topo_prefilter), 2 uses
                                        // read from persistent tables (kPlanPtab)
  std::vector<uint8_t> trivial;         // per loaded pod: kBatchStaticTrivial
  std::vector<uint8_t> noadd;           // per loaded pod: no count-class adds (deferred-commit batches)
  std::vector<uint8_t> noscalar;        // ... and no scalar requests (generic deferred-commit batches)
  // static classes (DevPods::stab, ensure_stab): per loaded pod its class or
  // -1 (d_sclass), each class's representative pod (d_srep); the table is
  // rebuilt after any change of pods, cluster or profile (stab_dirty)
  int32_t* d_sclass = nullptr;
  int32_t* d_srep = nullptr;
  int32_t stab_ncls = 0;
  bool stab_dirty = true, stab_ready = false;
  std::vector<DevBuf> stab_bufs;
  size_t stab_bytes = 0;
  std::vector<int32_t> sclass;          // host copy of d_sclass
  std::vector<uint8_t> hard_small;      // per loaded pod: every hard spread key column has <= kFuseMinValues values
  std::vector<uint8_t> soft_le1;        // per loaded pod: at most one ScheduleAnyway spread constraint
  std::vector<int32_t> tlen;            // per loaded pod: topology batch run length from it (tbatch_runs)
  std::vector<int32_t> tlen_plain;      // ... without zone variants (replicated topology batches)
  std::vector<int64_t> xdom_len;        // per loaded pod: sharded cycle, packed domain words
  std::vector<int64_t> xreg_len;        // per loaded pod: sharded cycle, registration words (0: no soft spread)

  // compat-mode single pod
  DevArena pod1_arena;                  // the single-pod uploads (upload_single)
  DevArena nom_arena;                   // a nominated pod (ksim_fw_filter_nominated)
  // Reserve / Unreserve calls that arrive while a framework cycle sits between
  // its PreFilter and Score (the binding goroutine's Unreserve):
  // upstream's running cycle keeps its snapshot, so the engine applies them
  // once that cycle has scored (flush_deferred_binds), in call order
  struct DeferredBind {
    ksim_pod pod;
    std::vector<ksim_label_expr> ex;
    std::vector<ksim_term> tm;
    std::vector<ksim_topo_use> us;
    std::vector<ksim_class_add> ad;
    std::vector<int32_t> nn;
    int32_t node;
    int sign;
  };
  std::vector<DeferredBind> deferred_binds;
  // pinned, coherent host staging for the per-call uploads / results, and the
  // device's addresses of it (copy kernels read / write it directly)
  void* pin = nullptr;
  void* pin_d = nullptr;
  size_t pin_cap = 0;
  // the last pod upload's copy out of the staging (upload_blob waits on it
  // instead of the whole stream); the pod last uploaded into pod1_arena (its
  // bytes and device address: a Reserve / Unreserve of the same pod binds
  // from there, no upload)
  // upload_blob's pinned staging ring: consecutive pod uploads (an informer's
  // pod deltas, another pod's Reserve, the next cycle's pod) do not wait for
  // each other's copies; a slot is reused once its copy has run (its event)
  struct PinSlot {
    void* p = nullptr;
    void* d = nullptr;
    size_t cap = 0;
    hipEvent_t ev = nullptr;
    bool pending = false;
  };
  static constexpr int kPinRing = 4;
  PinSlot ring[kPinRing];
  int ring_next = 0;
  std::vector<char> pod1_blob;
  char* pod1_base = nullptr;
  // build_pod_blob's pieces and the framework-driven pass's blob, kept so the
  // per-cycle calls reuse their capacity
  std::vector<ksim_label_expr> bs_ex;
  std::vector<ksim_term> bs_tm;
  std::vector<ksim_topo_use> bs_us;
  std::vector<ksim_class_add> bs_ad;
  std::vector<int32_t> bs_nn;
  PodBlob fw_blob;
  // the framework-driven filter passes alternate two arenas, so the Reserve of
  // cycle i (binding from cycle i's arena) can wait, queued, and run inside
  // cycle i+1's upload launch (pend_bind); any other call launches it first
  DevArena fw_arena[2];
  int fw_flip = 0;
  struct PendBind {
    bool on = false;
    DevPods P{};
    int32_t node = 0;
    int sign = 0;
  } pend_bind;
  int64_t pend_reuse = 0;                      // upload_blob found the queued Reserve's arena reused (flushed)
  void* pout = nullptr;
  void* pout_d = nullptr;
  size_t pout_cap = 0;
  // DefaultPreemption: bound pods per node in importance order
  std::vector<DevBuf> pre_bufs;
  std::vector<DevBuf> pre_nom_bufs;     // ksim_preempt_nominated's group requests
  DevPreempt pre{};
  std::vector<int32_t> pre_index;       // CSR position -> bound-pod table index
  int32_t pre_n = 0;
  // extender round trip (ksim_eval_pod_filter -> ksim_eval_pod_finish)
  DevPods pod1{};
  bool ext_pending = false;
  uint8_t* ext_fail = nullptr;     // device [n]
  int64_t* ext_score = nullptr;    // device [n]
  // framework-driven compat cycle (ksim_fw_prefilter -> ksim_fw_score ->
  // ksim_fw_normalize): the pod in h->pod1, its filter pass on the host for
  // list validation, the scan-set size
  bool fw_pending = false, fw_scored = false, fw_dom_dirty = false, fw_topo = false;
  int32_t fw_ns = 0;
  std::vector<uint8_t> fw_fail;
  // ksim_fw_score's list and answers, host side: a NormalizeScore over that
  // list with the raw scores it returned is answered from here
  std::vector<int32_t> fw_list;
  std::vector<int64_t> fw_raw, fw_norm;         // [slot][list position]
  // host-answered Score (fw_host): ksim_fw_prefilter also copies every node's
  // raw scores, the weighted sum of the plugins without NormalizeScore and the
  // topology flags into pinned memory, and ksim_fw_score normalizes over the
  // framework's list on the host (no second device round trip) when no
  // PreScore of the pod depends on that list
  bool fw_host = false;
  int64_t fw_counts[4] = {0, 0, 0, 0};   // Score on the host / device, NormalizeScore cached / device
  std::vector<uint8_t> fw_seen;    // list validation (all zero between calls)
  std::vector<int64_t> fw_tot;
  void* fwh = nullptr;             // pinned: [S][n] raw, [n] part
  void* fwh_d = nullptr;
  size_t fwh_cap = 0;
  uint32_t fw_tflags = 0;
  size_t fw_oraw = 0, fw_opart = 0;  // fwh offsets of the raw scores and the weighted part
  bool fw_raw32 = false;             // ... as int32 (the filter kernel's own copy) or int64 (a copy launch)
  int32_t* fw_nodes = nullptr;     // device [n]
  int64_t* fw_vals = nullptr;      // device [n]
  int64_t* fw_out = nullptr;       // device [n]

  // node sharding: this handle holds [shard_base, shard_base + n) of shard_total
  int32_t shard_base = 0, shard_total = 0;
  // replicated handle (ksim_set_eval_range): holds every node, evaluates
  // [eval_lo, eval_hi) in the P100 batch top-T and keeps its replica by
  // binding every placement: one exchange per batch (the records' all-gather)
  bool replicated = false;
  int32_t eval_lo = 0, eval_hi = 0;
  bool rep_primary = true;              // replicated: this replica counts the whole-run evaluations
  int32_t rank = 0, world = 1;
  ncclComm_t comm = nullptr;

  // per-pod cycles, by variant: topology kernels (1) | critical paths in the
  // filter pass (2) | NormalizeScore extrema in the filter pass (4)
  hipGraphExec_t graph_cycle[16] = {};   // | persistent tables (8)
  hipGraphExec_t graph_batch = nullptr;
  hipGraphExec_t graph_batch_fast = nullptr;   // k_batch_top<true> runs
  hipGraphExec_t graph_batch_stab = nullptr;   // static-class runs (LaunchArgs::stab)
  hipGraphExec_t graph_tbatch = nullptr;       // topology batches (ksim_tbatch.hip)
  // deferred-commit FAST batches (ksim_internal.h): the second snapshot buffer
  // X[1] and state st[1], the ring of chain + pairs outputs, kGraphBatches
  // batches as one graph (starting at a batch index divisible by kLazySlots)
  std::vector<DevBuf> lazy_bufs;
  int32_t lazy_n = -1;
  DynCols lazy_x1{};
  DevState* lazy_st1 = nullptr;
  uint64_t *lazy_g = nullptr, *lazy_m = nullptr;   // [kLazySlots][kBatchPods]
  int32_t* lazy_e = nullptr;                        // [kLazySlots] prefix length, -1 = empty slot
  int32_t *lazy_ab = nullptr, *lazy_aw = nullptr;   // ADAPT: [kLazySlots][kBatchPods] broken flags, [..][2 B] windows
  hipGraphExec_t graph_lazy = nullptr;
  hipGraphExec_t graph_lazy_adapt = nullptr;
  // node-sharded ADAPT batch: this shard's bitmaps, the all-gathered ones and
  // the global bitmap (allocated at the first such run)
  std::vector<DevBuf> ash_bufs;
  uint64_t *ash_send = nullptr, *ash_recv = nullptr, *ash_gmask = nullptr;
  int32_t ash_world = 0, ash_w = 0;
  int64_t graph_captures = 0;                  // graphs captured since ksim_create (ksim_get_diag)
  // node-sharded per-pod cycles (group leader): graphs of kGraphCycles cycles
  // per shape (topology, exchange lengths), valid while every handle of the
  // group keeps the graph generation it had at capture
  int64_t graph_gen = 0;                       // bumped whenever this handle's cycle graphs are dropped
  std::vector<std::pair<const ksim_handle*, int64_t>> sg_sig;
  std::map<std::tuple<bool, int64_t, int64_t>, hipGraphExec_t> sg_graphs;
  bool sg_off = false;                         // capture failed once (e.g. a collective that cannot be captured)
  int64_t match_ns = 0;                        // device time of the last ksim_match_terms (HIP events)
};

namespace {

int set_err(ksim_handle* h, int code, const std::string& msg) {
  if (h) h->err = msg;
  return code;
}

int hip_fail(ksim_handle* h, hipError_t e, const char* what) {
  int code = (e == hipErrorOutOfMemory) ? KSIM_E_OOM : KSIM_E_DEVICE;
  return set_err(h, code, std::string(what) + ": " + hipGetErrorString(e));
}

#define HIPCHK(h, expr)                                    \
  do {                                                     \
    hipError_t _e = (expr);                                \
    if (_e != hipSuccess) return hip_fail((h), _e, #expr); \
  } while (0)

// Blocking copies on the handle's own non-blocking stream.  A hipMemcpy on the
// legacy stream is refused while another host thread captures a graph (several
// engines in one process: bench config 5's concurrent sweep), and stream order
// is the order the engine relies on anyway.
static hipError_t hcopy(ksim_handle* h, void* dst, const void* src, size_t bytes, hipMemcpyKind kind) {
  const hipError_t e = hipMemcpyAsync(dst, src, bytes, kind, h->stream);
  return e != hipSuccess ? e : hipStreamSynchronize(h->stream);
}

static hipError_t hzero(ksim_handle* h, void* dst, size_t bytes) {
  const hipError_t e = hipMemsetAsync(dst, 0, bytes, h->stream);
  return e != hipSuccess ? e : hipStreamSynchronize(h->stream);
}

void free_bufs(std::vector<DevBuf>& v) {
  for (auto& b : v)
    if (b.p) (void)hipFree(b.p);
  v.clear();
}

// Allocate + copy (src may be null: zero-filled).
int upload(ksim_handle* h, std::vector<DevBuf>& owner, const void* src, size_t bytes, void** out) {
  void* p = nullptr;
  size_t alloc = bytes ? bytes : 16;
  hipError_t e = hipMalloc(&p, alloc);
  if (e != hipSuccess) return hip_fail(h, e, "hipMalloc");
  owner.push_back({p, alloc});
  if (src && bytes) {
    e = hipMemcpyAsync(p, src, bytes, hipMemcpyHostToDevice, h->stream);
  } else {
    e = hipMemsetAsync(p, 0, alloc, h->stream);
  }
  if (e != hipSuccess) return hip_fail(h, e, "upload copy");
  *out = p;
  return KSIM_OK;
}

// The per-pod cycle graphs (their kernels take the profile by value).
void drop_cycle_graphs(ksim_handle* h) {
  for (auto& g : h->graph_cycle) {
    if (g) (void)hipGraphExecDestroy(g);
    g = nullptr;
  }
  for (auto& kv : h->sg_graphs) (void)hipGraphExecDestroy(kv.second);
  h->sg_graphs.clear();
  h->graph_gen++;
}

void drop_graphs(ksim_handle* h) {
  drop_cycle_graphs(h);
  if (h->graph_batch) (void)hipGraphExecDestroy(h->graph_batch);
  if (h->graph_batch_fast) (void)hipGraphExecDestroy(h->graph_batch_fast);
  if (h->graph_batch_stab) (void)hipGraphExecDestroy(h->graph_batch_stab);
  h->graph_batch_stab = nullptr;
  if (h->graph_tbatch) (void)hipGraphExecDestroy(h->graph_tbatch);
  if (h->graph_lazy) (void)hipGraphExecDestroy(h->graph_lazy);
  if (h->graph_lazy_adapt) (void)hipGraphExecDestroy(h->graph_lazy_adapt);
  h->graph_lazy_adapt = nullptr;
  h->graph_batch_fast = nullptr;
  h->graph_batch = nullptr;
  h->graph_tbatch = nullptr;
  h->graph_lazy = nullptr;
}

bool plugin_supported(int id) { return id >= 0 && id < KSIM_PL_COUNT; }
bool is_sharded(const ksim_handle* h);

int validate_pod(ksim_handle* h, const ksim_pod_set* ps, int32_t i) {
  const ksim_pod& p = ps->pods[i];
  const DevCluster& c = h->dc;
  if (p.flags & (KSIM_POD_HAS_HOST_PORTS | KSIM_POD_HAS_VOLUMES))
    return set_err(h, KSIM_E_UNSUPPORTED, "pod " + std::to_string(i) + ": host ports / volumes not supported by the engine");
  if (p.node_name < -2 || p.node_name >= c.n_total)
    return set_err(h, KSIM_E_INVALID, "pod " + std::to_string(i) + ": node_name out of range");
  auto check_expr = [&](int32_t e) -> bool {
    if (e < 0 || e >= ps->n_exprs) return false;
    const ksim_label_expr& x = ps->exprs[e];
    if (x.nvals > KSIM_EXPR_VALS || x.op > KSIM_OP_TRUE) return false;
    if (x.op <= KSIM_OP_LT && x.col >= c.n_label_cols) return false;
    return true;
  };
  auto check_terms = [&](int32_t first, int32_t count) -> bool {
    if (count < 0 || (count > 0 && (first < 0 || first + count > ps->n_terms))) return false;
    for (int32_t t = 0; t < count; t++) {
      const ksim_term& tm = ps->terms[first + t];
      if (tm.n_expr < 0) return false;
      for (int32_t k = 0; k < tm.n_expr; k++)
        if (!check_expr(tm.first_expr + k)) return false;
    }
    return true;
  };
  if (p.sel_count < 0) return set_err(h, KSIM_E_INVALID, "bad sel_count");
  for (int32_t k = 0; k < p.sel_count; k++)
    if (!check_expr(p.sel_first + k)) return set_err(h, KSIM_E_INVALID, "pod " + std::to_string(i) + ": bad nodeSelector expr");
  if (!check_terms(p.req_term_first, p.req_term_count) || !check_terms(p.pref_term_first, p.pref_term_count))
    return set_err(h, KSIM_E_INVALID, "pod " + std::to_string(i) + ": bad affinity term range");
  if ((p.flags & KSIM_POD_ADDED_AFFINITY) && (p.added_term_count <= 0 || !check_terms(p.added_term_first, p.added_term_count)))
    return set_err(h, KSIM_E_INVALID, "pod " + std::to_string(i) + ": bad addedAffinity term range");
  const std::string who = "pod " + std::to_string(i) + ": ";
  for (const auto& vl : {std::make_pair(p.vb_first, p.vb_count), std::make_pair(p.vz_first, p.vz_count)}) {
    if (vl.second == 0) continue;
    if (!check_terms(vl.first, vl.second)) return set_err(h, KSIM_E_INVALID, who + "bad volume term range");
    for (int32_t k = 0; k < vl.second; k++) {   // group indices: non-negative, non-decreasing
      const int32_t g = ps->terms[vl.first + k].weight;
      if (g < 0 || (k > 0 && g < ps->terms[vl.first + k - 1].weight))
        return set_err(h, KSIM_E_INVALID, who + "volume term groups must be non-decreasing");
    }
  }
  if (p.use_count < 0 || p.use_count > KSIM_MAX_USES ||
      (p.use_count > 0 && (!ps->uses || p.use_first < 0 || p.use_first + p.use_count > ps->n_uses)))
    return set_err(h, KSIM_E_INVALID, who + "bad topology use range");
  for (int32_t k = 0; k < p.use_count; k++) {
    const ksim_topo_use& u = ps->uses[p.use_first + k];
    if (u.kind > KSIM_USE_IMAGE) return set_err(h, KSIM_E_INVALID, who + "bad topology use kind");
    if (u.cls < -1 || u.cls >= c.n_classes) return set_err(h, KSIM_E_INVALID, who + "topology use class out of range");
    if (u.col != KSIM_COL_NONE && u.col >= c.n_label_cols)
      return set_err(h, KSIM_E_INVALID, who + "topology key column out of range");
    if (u.kind == KSIM_USE_PTS_SOFT && c.n_topo_log < c.n + 1)
      return set_err(h, KSIM_E_INVALID, who + "ScheduleAnyway spread needs topo_log[0..n_nodes]");
  }
  if (p.add_count < 0 || (p.add_count > 0 && (!ps->adds || p.add_first < 0 || p.add_first + p.add_count > ps->n_adds)))
    return set_err(h, KSIM_E_INVALID, who + "bad class add range");
  for (int32_t k = 0; k < p.add_count; k++)
    if (ps->adds[p.add_first + k].cls < 0 || ps->adds[p.add_first + k].cls >= c.n_classes)
      return set_err(h, KSIM_E_INVALID, who + "class add out of range");
  if (p.flags & KSIM_POD_NODE_NAMES) {
    if (p.nn_count < 0 || (p.nn_count > 0 && (!ps->nn || p.nn_first < 0 ||
                                              (int64_t)p.nn_first + p.nn_count > (int64_t)ps->n_nn)))
      return set_err(h, KSIM_E_INVALID, who + "bad PreFilterResult node range");
    for (int32_t k = 0; k < p.nn_count; k++) {
      const int32_t v = ps->nn[p.nn_first + k];
      if (v < 0 || v >= c.n_total || (k > 0 && v <= ps->nn[p.nn_first + k - 1]))
        return set_err(h, KSIM_E_INVALID, who + "PreFilterResult nodes must be increasing node positions");
    }
    if (is_sharded(h))
      return set_err(h, KSIM_E_UNSUPPORTED, who + "a PreFilterResult node restriction runs on unsharded handles");
  }
  return KSIM_OK;
}

// Batch-path eligibility of a pod and the constant it adds to every total.
// The batch path needs P100 (every feasible node is kept, so no window) and
// every normalized plugin constant over nodes:
//   TaintToleration: no PreferNoSchedule taint the pod does not tolerate ->
//                    all raw 0 -> DefaultNormalizeScore(reverse) = 100
//   NodeAffinity:    no preferred terms -> raw 0 -> 0
//   PodTopologySpread: no constraints -> 100
//   InterPodAffinity:  no uses -> topologyScore empty -> 0
// A pod with topology uses reads the count classes, which binds of earlier
// pods of a batch change, so it always takes the per-pod path.
// Every static filter of the batch path passes on every node for this pod:
// no spec.nodeName, no nodeSelector / required node affinity, every
// NoSchedule/NoExecute taint in the cluster tolerated, no unschedulable node
// (or tolerated).  The batch kernels then skip the static filters.
bool static_trivial(const ksim_handle* h, const ksim_pod& p) {
  if (p.node_name != -1 || p.sel_count > 0 || (p.flags & (KSIM_POD_HAS_REQUIRED_AFFINITY | KSIM_POD_ADDED_AFFINITY)))
    return false;
  if (h->any_unschedulable && !(p.flags & KSIM_POD_TOLERATES_UNSCHEDULABLE)) return false;
  for (uint16_t id : h->hard_taints)
    if (!((p.tol_filter[id >> 6] >> (id & 63)) & 1ull)) return false;
  return true;
}

bool is_sharded(const ksim_handle* h) { return h->comm != nullptr || h->shard_total != 0; }

// The FAST batch kernels (dyn_key_fast): trivial pods, {cpu, memory}
// strategies with weights in [1, 2^31), allocatable cpu / memory below 2^46.
bool run_fast(const ksim_handle* h, int32_t a, int32_t b) {
  if (!h->bp.cpu_mem || !h->bp.fast_w || !h->alloc_narrow) return false;
  for (int32_t i = a; i < b; i++)
    if (!h->trivial[i] || h->batchable[i] == 2) return false;
  return true;
}

// ---- static classes (DevPods::stab) -------------------------------------------
constexpr int32_t kStabMaxClasses = 4096;
constexpr size_t kStabMaxEntries = (size_t)1 << 26;   // 512 MB of table

// The static inputs of a batch pod's keys, as bytes: what static_filters_pass
// (NodeUnschedulable, NodeName, TaintToleration, NodeAffinity) and norm_raw
// read of the pod, the selector and affinity expressions expanded, the
// preferred terms without their weights (two pods with equal signatures have
// equal verdicts, taint counts and preferred-term matches on every node;
// stab_word).  False past 32 preferred terms or for a negative weight.
bool stab_signature(const ksim_pod_set* ps, const ksim_pod& q, std::string& s) {
  s.clear();
  auto put = [&](const void* p, size_t n) { s.append((const char*)p, n); };
  auto put_expr = [&](int32_t e) {
    const ksim_label_expr& x = ps->exprs[e];
    put(&x.num, sizeof x.num);
    put(&x.col, sizeof x.col);
    put(&x.op, sizeof x.op);
    put(&x.nvals, sizeof x.nvals);
    put(x.vals, sizeof(uint32_t) * std::min<int>(x.nvals, KSIM_EXPR_VALS));
  };
  auto put_term = [&](int32_t t, bool preferred) {
    const ksim_term& x = ps->terms[t];
    if (preferred) s.push_back(x.weight != 0 ? 1 : 0);   // a zero weight never counts
    put(&x.n_expr, sizeof x.n_expr);
    for (int32_t k = 0; k < x.n_expr; k++) put_expr(x.first_expr + k);
  };
  const uint32_t fl = q.flags & (KSIM_POD_TOLERATES_UNSCHEDULABLE | KSIM_POD_HAS_REQUIRED_AFFINITY |
                                 KSIM_POD_ADDED_AFFINITY);
  put(&fl, sizeof fl);
  if (q.flags & KSIM_POD_ADDED_AFFINITY) {
    put(&q.added_term_count, sizeof q.added_term_count);
    for (int32_t k = 0; k < q.added_term_count; k++) put_term(q.added_term_first + k, false);
  }
  put(&q.node_name, sizeof q.node_name);
  put(q.tol_filter, sizeof q.tol_filter);
  put(q.tol_prefer, sizeof q.tol_prefer);
  put(&q.sel_count, sizeof q.sel_count);
  for (int32_t k = 0; k < q.sel_count; k++) put_expr(q.sel_first + k);
  put(&q.req_term_count, sizeof q.req_term_count);
  for (int32_t k = 0; k < q.req_term_count; k++) put_term(q.req_term_first + k, false);
  if (q.pref_term_count > 32) return false;
  put(&q.pref_term_count, sizeof q.pref_term_count);
  for (int32_t k = 0; k < q.pref_term_count; k++) {
    put_term(q.pref_term_first + k, true);
    if (ps->terms[q.pref_term_first + k].weight < 0) return false;   // raw scores >= 0 (norm_part_fast)
  }
  return true;
}

// The "ab" flavor: no table (the keys evaluate the static plugins per node).
bool stab_enabled() {
  constexpr bool off = ab(kAbStab);
  return !off;
}

LaunchArgs make_args(ksim_handle* h, const DevPods& P, int32_t* chosen);

// The static table of the loaded queue's classes on the current snapshot and
// profile, rebuilt in place when stale (in stream order: a graph captured with
// the table replays on the new contents, so a weight sweep keeps its graphs);
// graphs that may hold the table's old address, or a table that no longer
// exists, drop.
int ensure_stab(ksim_handle* h) {
  if (!h->stab_dirty) return KSIM_OK;
  h->stab_dirty = false;
  const bool was_ready = h->stab_ready;
  h->stab_ready = false;
  const size_t entries = (size_t)h->stab_ncls * (size_t)std::max(h->dc.n, 0);
  if (!stab_enabled() || !h->dp.pods || entries == 0 || entries > kStabMaxEntries) {
    if (was_ready) {
      HIPCHK(h, hipStreamSynchronize(h->stream));
      drop_graphs(h);
    }
    return KSIM_OK;
  }
  if (h->stab_bytes < 8 * entries) {
    HIPCHK(h, hipStreamSynchronize(h->stream));
    drop_graphs(h);
    free_bufs(h->stab_bufs);
    h->stab_bytes = 0;
    void* p = nullptr;
    int rc;
    if ((rc = upload(h, h->stab_bufs, nullptr, 8 * entries, &p))) return rc;
    h->stab_bytes = 8 * entries;
  } else if (!was_ready) {
    HIPCHK(h, hipStreamSynchronize(h->stream));
    drop_graphs(h);                              // captured without the table
  }
  launch_static_table(make_args(h, h->dp, nullptr), h->d_srep, h->stab_ncls, (uint64_t*)h->stab_bufs[0].p, h->stream);
  HIPCHK(h, hipGetLastError());
  h->stab_ready = true;
  return KSIM_OK;
}

// ADAPT: the profile keeps fewer than all nodes (K < N over the whole cluster).
bool adapt_mode(const ksim_handle* h) {
  return num_feasible_nodes_to_find(h->prof.percentage_of_nodes_to_score, h->dc.n_total) < h->dc.n_total;
}

// The STAB batch kernels (LaunchArgs::stab): every pod of the P100 run in a
// static class, run_fast's cluster conditions, an unsharded handle and the
// default launch forms.
bool run_stab(const ksim_handle* h, int32_t a, int32_t b) {
  if (!h->stab_ready || h->stab_dirty || adapt_mode(h) || is_sharded(h) || h->replicated) return false;
  if (!h->bp.cpu_mem || !h->bp.fast_w || !h->alloc_narrow) return false;
  for (int32_t i = a; i < b; i++)
    if (h->sclass[(size_t)i] < 0) return false;
  return true;
}

// The key kernels of a batch run: FAST, FAST with the static table, or generic.
void pick_keys(const ksim_handle* h, int32_t a, int32_t b, LaunchArgs& la) {
  la.fast = run_fast(h, a, b);
  la.stab = !la.fast && run_stab(h, a, b);
  la.fast = la.fast || la.stab;
}

// NetworkBandwidth in the profile (Filter or Score)
bool profile_nb(const ksim_profile& p) {
  return prof_has_filter(p, KSIM_PL_NETWORK_BANDWIDTH) || prof_has_score(p, KSIM_PL_NETWORK_BANDWIDTH);
}

// The batch keys carry a pod's total minus its constant normalized part in
// 20 bits (tb_key): 100 * (w_fit + w_ba), plus w_tt + w_na for the pods
// whose normalized scores vary, must stay below kKeyTotalLimit, or the pods
// take the per-pod path, whose (total, TB) pairs are exact for any int64 total.  Pods that NodeAffinity's PreFilterResult
// restricts scan a node list of their own: per-pod path.
// Returns 0 (per-pod path), 1 (every batch path) or 2 (the unsharded P100
// batch path only): pods whose TaintToleration / NodeAffinity scores vary
// over nodes (kPodNormVaries: the keys carry them, normalized over the pod's
// S0 maxima) and pods with scalar requests (the ADAPT repair's compact rows
// carry no scalars).
int pod_batchable(const ksim_handle* h, const ksim_pod& p, bool* norm_varies = nullptr) {
  const ksim_profile& prof = h->prof;
  if (norm_varies) *norm_varies = false;
  if (p.use_count > 0) return 0;
  if (p.flags & KSIM_POD_NODE_NAMES) return 0;
  if (p.vb_count > 0 || p.vz_count > 0) return 0;       // volume groups: the per-pod filter chain
  // NetworkBandwidth runs on the per-pod path (its error statuses end cycles),
  // and so do pods that add to a node's allocated bandwidth
  if (profile_nb(prof) || p.nb_add != 0) return 0;
  const int64_t w_dyn = h->bp.w_fit + h->bp.w_ba;
  if ((int64_t)kMaxNodeScore * w_dyn >= kKeyTotalLimit) return 0;
  int cls = (p.flags & KSIM_POD_HAS_SCALAR) ? 2 : 1;
  bool varies = false;
  for (int k = 0; k < prof.n_score; k++) {
    switch (norm_kind(prof.score[k])) {
      case kNormDefaultReverse:                         // varies when some PreferNoSchedule taint is not tolerated
        for (size_t t = 1; t < h->taint_effect.size(); t++)
          if (h->taint_effect[t] == KSIM_EFFECT_PREFER_NO_SCHEDULE && !((p.tol_prefer[t >> 6] >> (t & 63)) & 1ull))
            varies = true;
        break;                                          // else every node 100
      case kNormDefault:
        if (p.pref_term_count > 0) varies = true;        // else every node 0
        break;
      default:                                          // PodTopologySpread 100, InterPodAffinity 0
        break;
    }
  }
  if (varies && (int64_t)kMaxNodeScore * (w_dyn + h->bp.w_tt + h->bp.w_na) >= kKeyTotalLimit) return 0;
  if (varies) cls = 2;
  if (norm_varies) *norm_varies = varies;
  return cls;
}

// Whether loaded pod i runs on this handle's batch path (see pod_batchable):
// class 2 needs the unsharded P100 path over the whole node table.
// Class 2 under ADAPT: pods whose normalized scores vary (k_adapt_top's
// maxima over the window's kept nodes), without scalar requests, on an
// unsharded handle (the "ab" flavor: the per-pod path).
bool pod_on_batch(const ksim_handle* h, int32_t i) {
  constexpr bool adapt_norm = !ab(kAbAdaptNorm);
  const uint8_t b = h->batchable[i];
  if (b != 2 && b != 3) return b != 0;
  if (h->replicated) return b == 3 && !adapt_mode(h);   // class 3: replicated topology batches (shard_run_tbatch)
  if (is_sharded(h)) return false;
  if (!adapt_mode(h)) return true;
  return b == 2 && adapt_norm && h->noscalar[(size_t)i];
}

// Topology pods the topology batch path takes (class 3; ksim_tbatch.hip): the
// per-pod path's fused no-window cycle would run them (at most one
// ScheduleAnyway spread constraint, keyed by hostname or by no node's key;
// hard spread keys of <= kFuseMinValues values) with every domain sum read
// from a persistent table, no port / volume / bandwidth inputs and no
// PreFilterResult node list, totals inside the batch key's 20 bits, and a
// cluster of at most kTbMaxBlocks node blocks.  The "ab" flavor: per-pod path.
bool tbatch_admit(const ksim_handle* h, const ksim_pod& p, const PodPlan& pl, bool hard_small, bool soft_le1) {
  constexpr bool off = ab(kAbTbatch);
  if (off || p.use_count <= 0) return false;
  if (h->dc.n > kTbMaxBlocks * 256) return false;
  if (p.flags & KSIM_POD_NODE_NAMES) return false;
  if (p.vb_count > 0 || p.vz_count > 0 || profile_nb(h->prof) || p.nb_add != 0) return false;
  const UseMasks& m = pl.m;
  if (m.port || m.soft_val || !hard_small || !soft_le1) return false;
  const bool pt = (pl.flags & kPlanPtab) != 0;
  if ((m.dom & ~(pt ? m.ptab : 0u)) != 0) return false;     // a domain sum k_topo_prefilter would build
  if ((m.aff | m.score) != 0 && !pt) return false;         // the InterPodAffinity flags come from the tables
  int64_t wsum = 0;
  for (int k = 0; k < h->prof.n_score; k++) wsum += h->prof.score_weight[k] == 0 ? 1 : h->prof.score_weight[k];
  return (int64_t)kMaxNodeScore * wsum < kKeyTotalLimit;
}

// A framework-driven cycle left behind by another entry point: its PreFilter
// domain sums were never re-zeroed by a k_select (no ksim_fw_score ran), and
// its pod / scratch state is about to be replaced.
int fw_abandon(ksim_handle* h) {
  if (h->fw_dom_dirty && h->sc.dom)
    HIPCHK(h, hipMemsetAsync(h->sc.dom, 0, 8 * (size_t)KSIM_MAX_USES * h->dc.vmax, h->stream));
  h->fw_dom_dirty = h->fw_pending = h->fw_scored = false;
  h->fw_list.clear();
  h->fw_raw.clear();
  return KSIM_OK;
}

}  // namespace
static int flush_deferred_binds(ksim_handle* h);
static int flush_idle(ksim_handle* h);
// The queued Reserve of the last framework cycle (pend_bind), launched now.
static int flush_pend_bind(ksim_handle* h) {
  if (!h || !h->pend_bind.on) return KSIM_OK;
  h->pend_bind.on = false;
  HIPCHK(h, hipSetDevice(h->device));
  launch_assume(h->dc, h->pend_bind.P, 0, h->pend_bind.node, h->pend_bind.sign, h->stream);
  HIPCHK(h, hipGetLastError());
  return KSIM_OK;
}
namespace {

int ensure_ready(ksim_handle* h, bool fw = false, bool keep_pend = false) {
  if (!h) return KSIM_E_INVALID;
  if (!keep_pend) {
    const int rc = flush_pend_bind(h);
    if (rc) return rc;
  }
  if (!fw && (h->fw_pending || h->fw_scored || h->fw_dom_dirty)) {
    const int rc = fw_abandon(h);
    if (rc) return rc;
  }
  if (!h->has_profile) return set_err(h, KSIM_E_INVALID, "profile not set");
  if (!h->has_cluster) return set_err(h, KSIM_E_INVALID, "cluster not set");
  if (h->dc.n <= 0) return set_err(h, KSIM_E_INVALID, "no nodes available");
  if (!h->fw_pending && !h->deferred_binds.empty()) return flush_deferred_binds(h);
  return KSIM_OK;
}

LaunchArgs make_args(ksim_handle* h, const DevPods& P, int32_t* chosen) {
  LaunchArgs a;
  a.c = h->dc;
  a.c.eval_lo = 0;                       // every node (replicated shard batches narrow it, shard_batch)
  a.c.eval_hi = a.c.n;
  a.c.count_whole = (!h->replicated || h->rep_primary) ? 1 : 0;
  a.P = P;
  if (h->stab_ready && !h->stab_dirty && P.pods == h->dp.pods) {   // the loaded queue's static classes
    a.P.sclass = h->d_sclass;
    a.P.stab = (const uint64_t*)h->stab_bufs[0].p;
    a.P.stab_fast = (h->bp.cpu_mem && h->bp.fast_w && h->alloc_narrow) ? 1 : 0;
  }
  a.prof = h->prof;
  a.bp = h->bp;
  a.dprof = h->d_prof;
  a.dbp = h->d_bp;
  a.st = h->st;
  a.s = h->sc;
  a.o = h->eo;
  a.chosen = chosen;
  return a;
}

int set_run(ksim_handle* h, int32_t first, int32_t end) {
  h->run_hdr[0] = first;
  h->run_hdr[1] = end;
  HIPCHK(h, hipMemcpyAsync(h->st, h->run_hdr, sizeof(h->run_hdr), hipMemcpyHostToDevice, h->stream));
  // a run starts with full batches (generic ADAPT batches cap the next one, DevState::bcap)
  HIPCHK(h, hipMemsetAsync(&h->st->bcap, 0, sizeof(int32_t), h->stream));
  // per-cycle selection state starts from zero (the no-window cycle keeps it
  // zero between its own cycles; other paths leave extrema behind)
  HIPCHK(h, hipMemsetAsync(h->sc.win, 0, sizeof(WinState), h->stream));
  return KSIM_OK;
}

int read_state(ksim_handle* h, DevState& st) {
  HIPCHK(h, hipMemcpyAsync(&st, h->st, sizeof(st), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return KSIM_OK;
}

int capture(ksim_handle* h, bool batch, bool topo, hipGraphExec_t* out, bool fast = false, bool fuse_min = false,
            bool fuse_ext = false, bool ptab = false, bool stab = false) {
  HIPCHK(h, hipStreamSynchronize(h->stream));
  LaunchArgs a = make_args(h, h->dp, h->d_chosen);
  a.fast = fast;
  a.stab = stab;
  a.fuse_min = fuse_min;
  a.fuse_ext = fuse_ext;
  a.ptab = ptab;
  hipGraph_t g = nullptr;
  HIPCHK(h, hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
  if (batch)
    for (int i = 0; i < kGraphBatches; i++) {
      if (adapt_mode(h))
        launch_batch_adapt(a, h->stream);
      else
        launch_batch(a, h->stream);
    }
  else
    for (int i = 0; i < kGraphCycles; i++) launch_cycle(a, h->stream, false, topo);
  hipError_t e = hipStreamEndCapture(h->stream, &g);
  if (e != hipSuccess) return hip_fail(h, e, "hipStreamEndCapture");
  e = hipGraphInstantiate(out, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (e != hipSuccess) return hip_fail(h, e, "hipGraphInstantiate");
  h->graph_captures++;
  return KSIM_OK;
}


// A run of topology batch pods [a, b) (set_run done).  The host knows each
// batch's pod count (the conflict-free run from its first pod, capped) and a
// batch commits at most that many, so launching the batches the counts predict
// never passes the end; a batch that commits fewer (a cut, an exhausted list,
// pinv) leaves pods for the next round.
int run_tbatch(ksim_handle* h, int32_t a, int32_t b, const LaunchArgs& la) {
  int rc;
  HIPCHK(h, hipMemsetAsync(h->sc.tb_win, 0, sizeof(WinState) * kTbPods, h->stream));
  HIPCHK(h, hipMemsetAsync(h->sc.tb_dom, 0, sizeof(TbDom) * kTbPods * kVarDom, h->stream));
  HIPCHK(h, hipMemsetAsync(h->sc.tb_vhold, 0, 4 * (size_t)kTbPods * kVarSlots * 2 * KSIM_MAX_SCORE, h->stream));
  if (!h->graph_tbatch) {
    HIPCHK(h, hipStreamSynchronize(h->stream));
    hipGraph_t g = nullptr;
    HIPCHK(h, hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < kGraphBatches; i++) launch_tbatch(la, h->stream);
    hipError_t e = hipStreamEndCapture(h->stream, &g);
    if (e != hipSuccess) return hip_fail(h, e, "hipStreamEndCapture");
    e = hipGraphInstantiate(&h->graph_tbatch, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (e != hipSuccess) {
      h->graph_tbatch = nullptr;
      return hip_fail(h, e, "hipGraphInstantiate");
    }
    h->graph_captures++;
  }
  int32_t cursor = a;
  while (cursor < b) {
    int32_t nbat = 0;
    for (int32_t i = cursor; i < b; nbat++) i += std::min(std::min(kTbPods, b - i), std::max(h->tlen[i], 1));
    int32_t done = 0;
    for (; done + kGraphBatches <= nbat; done += kGraphBatches) HIPCHK(h, hipGraphLaunch(h->graph_tbatch, h->stream));
    for (; done < nbat; done++) launch_tbatch(la, h->stream);
    HIPCHK(h, hipGetLastError());
    DevState st;
    if ((rc = read_state(h, st))) return rc;
    if (st.cursor <= cursor) return set_err(h, KSIM_E_DEVICE, "topology batch path made no progress");
    cursor = st.cursor;
  }
  return KSIM_OK;
}

// ---- deferred-commit FAST batches (ksim_internal.h, ksim_batch.hip) ----------
// The "ab" flavor: the three-launch batches (parity of both forms).
bool lazy_enabled() {
  constexpr bool off = ab(kAbLazy);
  return !off;
}

// A FAST run [a, b) whose pods add to no count class (the overlay carries the
// resource columns only), on a cluster the overlay's LDS node bitmap covers.
// Generic runs and static-class runs keep the three launches: the deferred
// commit measured slower for both (config 1 scaled, profiles/r03/ab_lazy_gen:
// 46.8 against 35.3 ms per step for generic keys, whose loop with the overlay
// held 205 VGPRs; profiles/r03/ab_stab: 13.3 against 12.7 ms for the
// static-class keys, whose overlay lookups in both passes cost more than the
// commit launch).
bool lazy_ok(const ksim_handle* h, int32_t a, int32_t b, bool fast, bool stab = false) {
  if (!lazy_enabled() || !fast || stab) return false;
  // ADAPT runs whole on a replica (no exchange); replicated P100 batches take
  // shard_run_lazy (lazy_rep_ok)
  if (adapt_mode(h) ? (is_sharded(h) && !h->replicated) : (is_sharded(h) || h->replicated)) return false;
  if (h->dc.base != 0 || h->dc.n > kLazyMaxNodes || h->dc.n <= 0) return false;
  for (int32_t i = a; i < b; i++)
    if (!h->noadd[i]) return false;
  return true;
}

int alloc_lazy(ksim_handle* h) {
  if (h->lazy_n == h->dc.n) return KSIM_OK;
  HIPCHK(h, hipStreamSynchronize(h->stream));
  if (h->graph_lazy) (void)hipGraphExecDestroy(h->graph_lazy);
  if (h->graph_lazy_adapt) (void)hipGraphExecDestroy(h->graph_lazy_adapt);
  h->graph_lazy = h->graph_lazy_adapt = nullptr;
  free_bufs(h->lazy_bufs);
  h->lazy_n = -1;
  const size_t n = (size_t)h->dc.n;
  int rc;
  void* p = nullptr;
  int64_t** cols[5] = {&h->lazy_x1.req_cpu, &h->lazy_x1.req_mem, &h->lazy_x1.req_eph, &h->lazy_x1.nz_cpu,
                       &h->lazy_x1.nz_mem};
  for (auto* c : cols) {
    if ((rc = upload(h, h->lazy_bufs, nullptr, 8 * n, &p))) return rc;
    *c = (int64_t*)p;
  }
  if ((rc = upload(h, h->lazy_bufs, nullptr, 4 * n, &p))) return rc;
  h->lazy_x1.num_pods = (int32_t*)p;
  if ((rc = upload(h, h->lazy_bufs, nullptr, sizeof(DevState), &p))) return rc;
  h->lazy_st1 = (DevState*)p;
  if ((rc = upload(h, h->lazy_bufs, nullptr, 8 * (size_t)kLazySlots * kBatchPods, &p))) return rc;
  h->lazy_g = (uint64_t*)p;
  if ((rc = upload(h, h->lazy_bufs, nullptr, 8 * (size_t)kLazySlots * kBatchPods, &p))) return rc;
  h->lazy_m = (uint64_t*)p;
  if ((rc = upload(h, h->lazy_bufs, nullptr, 4 * (size_t)kLazySlots, &p))) return rc;
  h->lazy_e = (int32_t*)p;
  if ((rc = upload(h, h->lazy_bufs, nullptr, 4 * (size_t)kLazySlots * kBatchPods, &p))) return rc;
  h->lazy_ab = (int32_t*)p;
  if ((rc = upload(h, h->lazy_bufs, nullptr, 8 * (size_t)kLazySlots * kBatchPods, &p))) return rc;
  h->lazy_aw = (int32_t*)p;
  h->lazy_n = h->dc.n;
  return KSIM_OK;
}

DynCols dyn_cols(const DevCluster& c) {
  return DynCols{c.req_cpu, c.req_mem, c.req_eph, c.nz_cpu, c.nz_mem, c.num_pods};
}

DevCluster with_cols(DevCluster c, const DynCols& d) {
  c.req_cpu = d.req_cpu;
  c.req_mem = d.req_mem;
  c.req_eph = d.req_eph;
  c.nz_cpu = d.nz_cpu;
  c.nz_mem = d.nz_mem;
  c.num_pods = d.num_pods;
  return c;
}

// The launch arguments of deferred-commit batch i of a run.
LazyBatch lazy_batch(const ksim_handle* h, const LaunchArgs& la, int64_t i) {
  const int p = (int)(i & 1), q = (int)(i & 3), q1 = (int)((i + 3) & 3), q2 = (int)((i + 2) & 3);
  const DynCols x[2] = {dyn_cols(h->dc), h->lazy_x1};
  DevState* st[2] = {h->st, h->lazy_st1};
  LazyBatch z;
  z.a = la;
  z.a.c = with_cols(la.c, x[p ^ 1]);
  z.cw = with_cols(la.c, x[p]);
  z.step.w = x[p];
  z.step.st_in = st[p ^ 1];
  z.step.st_out = st[p];
  z.step.g1 = h->lazy_g + (size_t)q1 * kBatchPods;
  z.step.m1 = h->lazy_m + (size_t)q1 * kBatchPods;
  z.step.e1 = h->lazy_e + q1;
  z.step.g2 = h->lazy_g + (size_t)q2 * kBatchPods;
  z.step.e2 = h->lazy_e + q2;
  z.step.e_self = h->lazy_e + q;
  z.st = st[p];
  z.gkey = h->lazy_g + (size_t)q * kBatchPods;
  z.pmax = h->lazy_m + (size_t)q * kBatchPods;
  z.cend = h->lazy_e + q;
  z.b1 = h->lazy_ab + (size_t)q1 * kBatchPods;
  z.w1 = h->lazy_aw + (size_t)q1 * 2 * kBatchPods;
  z.abroken = h->lazy_ab + (size_t)q * kBatchPods;
  z.awin = h->lazy_aw + (size_t)q * 2 * kBatchPods;
  return z;
}

// Start of a deferred-commit run (set_run done): X[1] = X[0], st[1] = st[0],
// every ring slot empty.
int lazy_begin(ksim_handle* h) {
  int rc;
  if ((rc = alloc_lazy(h))) return rc;
  const size_t n = (size_t)h->dc.n;
  const DynCols x0 = dyn_cols(h->dc), x1 = h->lazy_x1;
  HIPCHK(h, hipMemcpyAsync(x1.req_cpu, x0.req_cpu, 8 * n, hipMemcpyDeviceToDevice, h->stream));
  HIPCHK(h, hipMemcpyAsync(x1.req_mem, x0.req_mem, 8 * n, hipMemcpyDeviceToDevice, h->stream));
  HIPCHK(h, hipMemcpyAsync(x1.req_eph, x0.req_eph, 8 * n, hipMemcpyDeviceToDevice, h->stream));
  HIPCHK(h, hipMemcpyAsync(x1.nz_cpu, x0.nz_cpu, 8 * n, hipMemcpyDeviceToDevice, h->stream));
  HIPCHK(h, hipMemcpyAsync(x1.nz_mem, x0.nz_mem, 8 * n, hipMemcpyDeviceToDevice, h->stream));
  HIPCHK(h, hipMemcpyAsync(x1.num_pods, x0.num_pods, 4 * n, hipMemcpyDeviceToDevice, h->stream));
  HIPCHK(h, hipMemcpyAsync(h->lazy_st1, h->st, sizeof(DevState), hipMemcpyDeviceToDevice, h->stream));
  HIPCHK(h, hipMemsetAsync(h->lazy_e, 0xff, 4 * kLazySlots, h->stream));
  return KSIM_OK;
}

// After the flush of batch index f: the snapshot and state are in X[f & 1],
// st[f & 1]; bring them to the handle's own buffers.
int lazy_end(ksim_handle* h, int64_t f) {
  if ((f & 1) == 0) return KSIM_OK;
  const size_t n = (size_t)h->dc.n;
  const DynCols x0 = dyn_cols(h->dc), x1 = h->lazy_x1;
  HIPCHK(h, hipMemcpyAsync(x0.req_cpu, x1.req_cpu, 8 * n, hipMemcpyDeviceToDevice, h->stream));
  HIPCHK(h, hipMemcpyAsync(x0.req_mem, x1.req_mem, 8 * n, hipMemcpyDeviceToDevice, h->stream));
  HIPCHK(h, hipMemcpyAsync(x0.req_eph, x1.req_eph, 8 * n, hipMemcpyDeviceToDevice, h->stream));
  HIPCHK(h, hipMemcpyAsync(x0.nz_cpu, x1.nz_cpu, 8 * n, hipMemcpyDeviceToDevice, h->stream));
  HIPCHK(h, hipMemcpyAsync(x0.nz_mem, x1.nz_mem, 8 * n, hipMemcpyDeviceToDevice, h->stream));
  HIPCHK(h, hipMemcpyAsync(x0.num_pods, x1.num_pods, 4 * n, hipMemcpyDeviceToDevice, h->stream));
  HIPCHK(h, hipMemcpyAsync(h->st, h->lazy_st1, sizeof(DevState), hipMemcpyDeviceToDevice, h->stream));
  return KSIM_OK;
}

int read_state_at(ksim_handle* h, const DevState* src, DevState& st) {
  HIPCHK(h, hipMemcpyAsync(&st, src, sizeof(st), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return KSIM_OK;
}

// A run of pods [a, b) as deferred-commit batches (lazy_ok; set_run done).
// Batch i commits batch i - 1; each stretch of launches ends with a flush, whose
// state tells the host where the run stands.  A batch commits 1..kBatchPods
// pods, so ceil(left / kBatchPods) batches never start past the end.
uint32_t lazy_launch(const ksim_handle* h, const LazyBatch& z, hipStream_t stream, hipEvent_t* evs = nullptr) {
  return adapt_mode(h) ? launch_batch_adapt_lazy(z, stream, evs) : launch_batch_lazy(z, stream, evs);
}

void lazy_flush(const ksim_handle* h, const LazyBatch& z, hipStream_t stream) {
  if (adapt_mode(h)) launch_adapt_lazy_flush(z, stream);
  else launch_lazy_flush(z, stream);
}

int run_lazy(ksim_handle* h, int32_t a, int32_t b, const LaunchArgs& la) {
  int rc;
  if ((rc = lazy_begin(h))) return rc;
  hipGraphExec_t& graph = adapt_mode(h) ? h->graph_lazy_adapt : h->graph_lazy;
  if (!graph) {
    HIPCHK(h, hipStreamSynchronize(h->stream));
    hipGraph_t g = nullptr;
    HIPCHK(h, hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < kGraphBatches; i++) lazy_launch(h, lazy_batch(h, la, i), h->stream);
    hipError_t e = hipStreamEndCapture(h->stream, &g);
    if (e != hipSuccess) return hip_fail(h, e, "hipStreamEndCapture");
    e = hipGraphInstantiate(&graph, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (e != hipSuccess) {
      graph = nullptr;
      return hip_fail(h, e, "hipGraphInstantiate");
    }
    h->graph_captures++;
  }
  static_assert(kGraphBatches % kLazySlots == 0, "lazy graphs keep the ring phase");
  int64_t i = 0;
  int32_t cursor = a;
  while (cursor < b) {
    int32_t nb = (b - cursor + kBatchPods - 1) / kBatchPods;
    const int32_t align = (int32_t)((kLazySlots - (i & 3)) & 3);
    if (nb >= align + kGraphBatches) {
      for (int32_t r = 0; r < align; r++, i++, nb--) lazy_launch(h, lazy_batch(h, la, i), h->stream);
      for (int32_t r = 0; r < nb / kGraphBatches; r++, i += kGraphBatches) HIPCHK(h, hipGraphLaunch(graph, h->stream));
    } else {
      for (int32_t r = 0; r < nb; r++, i++) lazy_launch(h, lazy_batch(h, la, i), h->stream);
    }
    lazy_flush(h, lazy_batch(h, la, i), h->stream);
    HIPCHK(h, hipGetLastError());
    DevState st;
    if ((rc = read_state_at(h, (i & 1) ? h->lazy_st1 : h->st, st))) return rc;
    if (st.cursor <= cursor) return set_err(h, KSIM_E_DEVICE, "deferred-commit batch path made no progress");
    cursor = st.cursor;
    i++;
  }
  return lazy_end(h, i - 1);
}

// Run pods [a, b) on one path (all of them share the path).
int run_range(ksim_handle* h, int32_t a, int32_t b, bool batch, bool topo) {
  int rc;
  if ((rc = set_run(h, a, b))) return rc;
  // No launch is ever issued past the end of the run (a launch there would
  // exit at once and skew per-kernel averages): whole graphs while they fit,
  // then single launches for the remainder.
  LaunchArgs la = make_args(h, h->dp, h->d_chosen);
  if (!batch) {
    la.fuse_min = topo;
    for (int32_t i = a; i < b && la.fuse_min; i++) la.fuse_min = h->hard_small[i] != 0;
    la.fuse_ext = true;
    for (int32_t i = a; i < b && la.fuse_ext; i++) la.fuse_ext = h->soft_le1[i] != 0;
    la.ptab = h->topo[a] == 2;                     // runs are uniform in topo (for_each_run)
    hipGraphExec_t& g =
        h->graph_cycle[(topo ? 1 : 0) | (la.fuse_min ? 2 : 0) | (la.fuse_ext ? 4 : 0) | (la.ptab ? 8 : 0)];
    if (!g && (rc = capture(h, false, topo, &g, false, la.fuse_min, la.fuse_ext, la.ptab))) return rc;
    int32_t done = a;
    for (; done + kGraphCycles <= b; done += kGraphCycles) HIPCHK(h, hipGraphLaunch(g, h->stream));
    for (; done < b; done++) launch_cycle(la, h->stream, false, topo);
    HIPCHK(h, hipGetLastError());
    return KSIM_OK;
  }
  if (topo) return run_tbatch(h, a, b, la);
  // the FAST evaluation kernel when every pod of the run is trivial with
  // cpu/memory scoring, or is in a static class (STAB)
  pick_keys(h, a, b, la);
  if (lazy_ok(h, a, b, la.fast, la.stab)) return run_lazy(h, a, b, la);
  hipGraphExec_t& gb = la.stab ? h->graph_batch_stab : la.fast ? h->graph_batch_fast : h->graph_batch;
  if (!gb && (rc = capture(h, true, false, &gb, la.fast, false, false, false, la.stab))) return rc;
  // every batch commits between 1 and kBatchPods pods: a graph of
  // kGraphBatches batches never overshoots while left >= kBatchPods * kGraphBatches,
  // and ceil(left / kBatchPods) single batches never overshoot either
  int32_t cursor = a;
  while (cursor < b) {
    const int32_t left = b - cursor;
    if (left >= kBatchPods * kGraphBatches) {
      const int reps = left / (kBatchPods * kGraphBatches);
      for (int r = 0; r < reps; r++) HIPCHK(h, hipGraphLaunch(gb, h->stream));
    } else {
      const int n1 = (left + kBatchPods - 1) / kBatchPods;
      for (int r = 0; r < n1; r++) {
        if (adapt_mode(h))
          launch_batch_adapt(la, h->stream);
        else
          launch_batch(la, h->stream);
      }
      HIPCHK(h, hipGetLastError());
    }
    DevState st;
    if ((rc = read_state(h, st))) return rc;
    if (st.cursor <= cursor) return set_err(h, KSIM_E_DEVICE, "batch path made no progress");
    cursor = st.cursor;
  }
  return KSIM_OK;
}

// Split [first, first+count) into maximal same-path runs (batch / per-pod,
// per-pod runs further by whether a pod carries topology uses).
// adapt_sharded: sharded handles whose shards follow adapt_shard_chunk, so
// ADAPT may take the sharded batch path (otherwise it runs cycle by cycle).
template <typename F>
int for_each_run(ksim_handle* h, int32_t first, int32_t count, F&& fn, bool adapt_sharded = false) {
  int32_t i = first;
  const int32_t end = first + count;
  while (i < end) {
    const bool batch_ok = !(adapt_mode(h) && is_sharded(h)) || adapt_sharded;
    const bool b = batch_ok && pod_on_batch(h, i);
    const bool t = h->topo[i] != 0;
    int32_t j = i + 1;
    while (j < end && (batch_ok && pod_on_batch(h, j)) == b && h->topo[j] == h->topo[i]) j++;
    int rc = fn(i, j, b, t);
    if (rc) return rc;
    i = j;
  }
  return KSIM_OK;
}

// ---- node-sharded batch path ----------------------------------
// One batch on every shard of a group, phases separated by the two exchanges:
// all-gather of the per-shard candidate records, all-reduce (max) of the pair
// keys.  `hs` is either {this rank's handle} with an RCCL communicator (one
// process per GPU) or an in-process group of shard handles on one device
// (exchanges by device copies).  Everything runs on `stream`, asynchronously.
// Replicated handles hold every node: each evaluates its range, and the pair
// keys and binds of every guess are local, so the pair-key all-reduce is not
// needed (one exchange per batch).
LaunchArgs shard_args(ksim_handle* h, bool fast) {
  LaunchArgs la = make_args(h, h->dp, h->d_chosen);
  la.fast = fast;
  if (h->replicated) {
    la.c.eval_lo = h->eval_lo;
    la.c.eval_hi = h->eval_hi;
  }
  return la;
}

int shard_batch(const std::vector<ksim_handle*>& hs, hipStream_t stream, bool fast) {
  const int R = (int)hs.size();
  ksim_handle* h0 = hs[0];
  const size_t rec = (size_t)kBatchPods * kXRec;            // u64 per shard
  for (auto* h : hs) launch_shard_eval(shard_args(h, fast), stream);
  if (h0->comm) {
    const ncclResult_t r = rccl().all_gather(h0->sc.xsend, h0->sc.xrecv, rec, ncclUint64, h0->comm, stream);
    if (r != ncclSuccess) return set_err(h0, KSIM_E_RCCL, std::string("ncclAllGather: ") + rccl().error_string(r));
  } else {
    for (int src = 0; src < R; src++)
      for (int dst = 0; dst < R; dst++)
        HIPCHK(h0, hipMemcpyAsync(hs[dst]->sc.xrecv + (size_t)src * rec, hs[src]->sc.xsend, 8 * rec,
                                  hipMemcpyDeviceToDevice, stream));
  }
  const int32_t world = h0->comm ? h0->world : R;
  for (auto* h : hs) launch_shard_chain(shard_args(h, fast), world, stream);
  if (h0->replicated) {
    // every guess is local: the pair maxima are complete on every handle
  } else if (h0->comm) {
    const ncclResult_t r =
        rccl().all_reduce(h0->sc.pmax, h0->sc.pmax, kBatchPods, ncclUint64, ncclMax, h0->comm, stream);
    if (r != ncclSuccess) return set_err(h0, KSIM_E_RCCL, std::string("ncclAllReduce: ") + rccl().error_string(r));
  } else if (R > 1) {
    GroupPtrs g{};
    g.n = R;
    for (int i = 0; i < R; i++) g.p[i] = hs[i]->sc.pmax;
    launch_group_max(g, stream);
  }
  for (auto* h : hs) launch_shard_commit(shard_args(h, fast), stream);
  HIPCHK(h0, hipGetLastError());
  return KSIM_OK;
}

hipGraphExec_t shard_batch_graph(const std::vector<ksim_handle*>& hs, bool fast, bool adapt);

// ---- replicated deferred-commit batches (ksim_internal.h) -----------------------
// Replicated handles of a FAST P100 run: batch i is k_batch_top_commit over the
// replica's node range (the commit of batch i-1 included, every replica binds
// every placement), the records' all-gather, the global merge and the chain +
// pairs: one exchange and three launches per batch instead of four.
bool lazy_rep_ok(const std::vector<ksim_handle*>& hs, int32_t a, int32_t b, bool fast) {
  if (!fast || !lazy_enabled()) return false;
  for (auto* h : hs) {
    if (!h->replicated || h->dc.base != 0 || h->dc.n > kLazyMaxNodes || h->dc.n <= 0) return false;
    for (int32_t i = a; i < b; i++)
      if (!h->noadd[i]) return false;
  }
  return true;
}

int shard_batch_lazy(const std::vector<ksim_handle*>& hs, hipStream_t stream, int64_t i) {
  const int R = (int)hs.size();
  ksim_handle* h0 = hs[0];
  const size_t rec = (size_t)kBatchPods * kXRec;
  for (auto* h : hs) launch_lazy_top_rep(lazy_batch(h, shard_args(h, true), i), h->sc.xsend, stream);
  if (h0->comm) {
    const ncclResult_t r = rccl().all_gather(h0->sc.xsend, h0->sc.xrecv, rec, ncclUint64, h0->comm, stream);
    if (r != ncclSuccess) return set_err(h0, KSIM_E_RCCL, std::string("ncclAllGather: ") + rccl().error_string(r));
  } else {
    for (int src = 0; src < R; src++)
      for (int dst = 0; dst < R; dst++)
        HIPCHK(h0, hipMemcpyAsync(hs[dst]->sc.xrecv + (size_t)src * rec, hs[src]->sc.xsend, 8 * rec,
                                  hipMemcpyDeviceToDevice, stream));
  }
  const int32_t world = h0->comm ? h0->world : R;
  for (auto* h : hs) launch_lazy_chain_rep(lazy_batch(h, shard_args(h, true), i), world, stream);
  HIPCHK(h0, hipGetLastError());
  return KSIM_OK;
}

hipGraphExec_t shard_lazy_graph(const std::vector<ksim_handle*>& hs) {
  ksim_handle* h0 = hs[0];
  if (h0->sg_off || ab(kAbShardGraph)) return nullptr;
  std::vector<std::pair<const ksim_handle*, int64_t>> sig;
  for (auto* h : hs) sig.emplace_back(h, h->graph_gen);
  if (sig != h0->sg_sig) {
    for (auto& kv : h0->sg_graphs) (void)hipGraphExecDestroy(kv.second);
    h0->sg_graphs.clear();
    h0->sg_sig = sig;
  }
  const auto key = std::make_tuple(true, (int64_t)-3, (int64_t)-1);
  auto it = h0->sg_graphs.find(key);
  if (it != h0->sg_graphs.end()) return it->second;
  hipStream_t stream = h0->stream;
  if (hipStreamSynchronize(stream) != hipSuccess) return nullptr;
  hipGraph_t g = nullptr;
  hipGraphExec_t ge = nullptr;
  bool ok = hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal) == hipSuccess;
  for (int i = 0; ok && i < kGraphBatches; i++) ok = shard_batch_lazy(hs, stream, i) == KSIM_OK;
  const hipError_t e = hipStreamEndCapture(stream, &g);
  ok = ok && e == hipSuccess && g && hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) == hipSuccess;
  if (g) (void)hipGraphDestroy(g);
  (void)hipGetLastError();
  if (!ok) {
    h0->sg_off = true;
    h0->err.clear();
    return nullptr;
  }
  h0->graph_captures++;
  h0->sg_graphs.emplace(key, ge);
  return ge;
}

// set_run done on every handle.  As run_lazy, on the group's stream.
int shard_run_lazy(const std::vector<ksim_handle*>& hs, int32_t a, int32_t b) {
  ksim_handle* h0 = hs[0];
  hipStream_t stream = h0->stream;
  int rc;
  for (auto* h : hs) {
    if ((rc = lazy_begin(h))) return rc;
    HIPCHK(h, hipStreamSynchronize(h->stream));
  }
  const hipGraphExec_t g = b - a >= kBatchPods * kGraphBatches ? shard_lazy_graph(hs) : nullptr;
  int64_t i = 0;
  int32_t cursor = a;
  while (cursor < b) {
    int32_t nb = (b - cursor + kBatchPods - 1) / kBatchPods;
    const int32_t align = (int32_t)((kLazySlots - (i & 3)) & 3);
    if (g && nb >= align + kGraphBatches) {
      for (int32_t r = 0; r < align; r++, i++, nb--)
        if ((rc = shard_batch_lazy(hs, stream, i))) return rc;
      for (int32_t r = 0; r < nb / kGraphBatches; r++, i += kGraphBatches) HIPCHK(h0, hipGraphLaunch(g, stream));
    } else {
      for (int32_t r = 0; r < nb; r++, i++)
        if ((rc = shard_batch_lazy(hs, stream, i))) return rc;
    }
    for (auto* h : hs) launch_lazy_flush(lazy_batch(h, shard_args(h, true), i), stream);
    HIPCHK(h0, hipGetLastError());
    DevState st;
    HIPCHK(h0, hipMemcpyAsync(&st, (i & 1) ? h0->lazy_st1 : h0->st, sizeof(st), hipMemcpyDeviceToHost, stream));
    HIPCHK(h0, hipStreamSynchronize(stream));
    if (st.cursor <= cursor) return set_err(h0, KSIM_E_DEVICE, "replicated deferred-commit batches made no progress");
    cursor = st.cursor;
    i++;
  }
  for (auto* h : hs) {
    if ((rc = lazy_end(h, i - 1))) return rc;
    HIPCHK(h, hipStreamSynchronize(h->stream));
  }
  return KSIM_OK;
}

// Pods [a, b) on the sharded batch path (every pod must be batchable).  No
// batch is ever issued past the run's end (each commits 1..kBatchPods pods):
// whole graphs of kGraphBatches batches while at least kBatchPods *
// kGraphBatches pods are left, then left / kBatchPods single batches.
int shard_run(const std::vector<ksim_handle*>& hs, int32_t a, int32_t b) {
  ksim_handle* h0 = hs[0];
  hipStream_t stream = h0->stream;
  bool fast = run_fast(h0, a, b);                      // every shard of an in-process group alike
  for (auto* h : hs) fast = fast && h->alloc_narrow;
  for (auto* h : hs) {
    int rc;
    if ((rc = set_run(h, a, b))) return rc;
    HIPCHK(h, hipStreamSynchronize(h->stream));
  }
  if (lazy_rep_ok(hs, a, b, fast)) return shard_run_lazy(hs, a, b);
  const hipGraphExec_t g = b - a >= kBatchPods * kGraphBatches ? shard_batch_graph(hs, fast, false) : nullptr;
  int32_t cursor = a;
  while (cursor < b) {
    const int32_t left = b - cursor;
    if (g && left >= kBatchPods * kGraphBatches) {
      const int reps = left / (kBatchPods * kGraphBatches);
      for (int r = 0; r < reps; r++) HIPCHK(h0, hipGraphLaunch(g, stream));
    } else {
      const int32_t n = std::max(1, left / kBatchPods);
      for (int32_t i = 0; i < n; i++) {
        int rc = shard_batch(hs, stream, fast);
        if (rc) return rc;
      }
    }
    DevState st;
    HIPCHK(h0, hipMemcpyAsync(&st, h0->st, sizeof(st), hipMemcpyDeviceToHost, stream));
    HIPCHK(h0, hipStreamSynchronize(stream));
    if (st.cursor <= cursor) return set_err(h0, KSIM_E_DEVICE, "sharded batch path made no progress");
    cursor = st.cursor;
  }
  return KSIM_OK;
}

// ---- replicated topology batches (ksim_tbatch.hip launch_tb_rep_*) -------------
template <typename F>
int x_allreduce(const std::vector<ksim_handle*>& hs, F&& ptr, int64_t count, bool op_max, hipStream_t stream);

// All-gather of `bytes` per handle: src(h) -> dst(h) + rank * bytes.
template <typename S, typename D>
int x_allgather_bytes(const std::vector<ksim_handle*>& hs, S&& src, D&& dst, size_t bytes, hipStream_t stream) {
  ksim_handle* h0 = hs[0];
  if (h0->comm) {
    const ncclResult_t r = rccl().all_gather(src(h0), dst(h0), bytes, ncclUint8, h0->comm, stream);
    if (r != ncclSuccess) return set_err(h0, KSIM_E_RCCL, std::string("ncclAllGather: ") + rccl().error_string(r));
    return KSIM_OK;
  }
  for (size_t a = 0; a < hs.size(); a++)
    for (size_t b = 0; b < hs.size(); b++)
      HIPCHK(h0, hipMemcpyAsync((char*)dst(hs[b]) + a * bytes, src(hs[a]), bytes, hipMemcpyDeviceToDevice, stream));
  return KSIM_OK;
}

// One topology batch on every replica of a group: each evaluates its node
// range; three exchanges (the filter's per-pod counters and extrema, the
// per-pod top-T records with the extremum holder counts, the pair maxima and
// pinv); every replica commits every placement.
int shard_tbatch(const std::vector<ksim_handle*>& hs, hipStream_t stream) {
  ksim_handle* h0 = hs[0];
  const int32_t world = h0->comm ? h0->world : (int32_t)hs.size();
  int rc;
  for (auto* h : hs) launch_tb_rep_filter(shard_args(h, false), stream);
  if ((rc = x_allgather_bytes(hs, [](ksim_handle* h) { return (void*)h->sc.tb_win; },
                              [](ksim_handle* h) { return (void*)h->sc.tb_xrecv; }, sizeof(WinState) * kTbPods, stream)))
    return rc;
  for (auto* h : hs) launch_tb_rep_select(shard_args(h, false), world, stream);
  if ((rc = x_allgather_bytes(hs, [](ksim_handle* h) { return (void*)h->sc.xsend; },
                              [](ksim_handle* h) { return (void*)h->sc.xrecv; }, 8 * (size_t)kTbPods * kTbXRec,
                              stream)))
    return rc;
  for (auto* h : hs) launch_tb_rep_pairs(shard_args(h, false), world, stream);
  if ((rc = x_allreduce(hs, [](ksim_handle* h) { return h->sc.tb_pp; }, 2 * kTbPods, true, stream))) return rc;
  for (auto* h : hs) launch_tb_rep_commit(shard_args(h, false), stream);
  HIPCHK(h0, hipGetLastError());
  return KSIM_OK;
}

// Topology batch pods [a, b) on the replicas of a group (as run_tbatch: the
// batches the run lengths predict, then the state).
int shard_run_tbatch(const std::vector<ksim_handle*>& hs, int32_t a, int32_t b) {
  ksim_handle* h0 = hs[0];
  hipStream_t stream = h0->stream;
  int rc;
  for (auto* h : hs) {
    if ((rc = set_run(h, a, b))) return rc;
    HIPCHK(h, hipMemsetAsync(h->sc.tb_win, 0, sizeof(WinState) * kTbPods, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
  }
  int32_t cursor = a;
  while (cursor < b) {
    int32_t nbat = 0;
    for (int32_t i = cursor; i < b; nbat++) i += std::min(std::min(kTbPods, b - i), std::max(h0->tlen_plain[i], 1));
    for (int32_t i = 0; i < nbat; i++)
      if ((rc = shard_tbatch(hs, stream))) return rc;
    DevState st;
    HIPCHK(h0, hipMemcpyAsync(&st, h0->st, sizeof(st), hipMemcpyDeviceToHost, stream));
    HIPCHK(h0, hipStreamSynchronize(stream));
    if (st.cursor <= cursor) return set_err(h0, KSIM_E_DEVICE, "replicated topology batches made no progress");
    cursor = st.cursor;
  }
  return KSIM_OK;
}

// ---- node-sharded per-pod cycle (C1 extrema, C2 argmax, C3 window) ----
// Element-wise all-reduce of a per-handle device buffer of `count` 8-byte words:
// sum (int64) or max (uint64).  RCCL across processes, a group kernel in-process.
template <typename F>
int x_allreduce(const std::vector<ksim_handle*>& hs, F&& ptr, int64_t count, bool op_max, hipStream_t stream) {
  if (count <= 0) return KSIM_OK;
  ksim_handle* h0 = hs[0];
  if (h0->comm) {
    void* b = (void*)ptr(h0);
    const ncclResult_t r = rccl().all_reduce(b, b, (size_t)count, op_max ? ncclUint64 : ncclInt64,
                                             op_max ? ncclMax : ncclSum, h0->comm, stream);
    if (r != ncclSuccess) return set_err(h0, KSIM_E_RCCL, std::string("ncclAllReduce: ") + rccl().error_string(r));
  } else if (hs.size() > 1) {
    GroupPtrs g{};
    g.n = (int32_t)hs.size();
    for (size_t i = 0; i < hs.size(); i++) g.p[i] = (uint64_t*)ptr(hs[i]);
    launch_group_reduce(g, count, op_max, stream);
  }
  return KSIM_OK;
}

// All-gather of two words per shard: s.xsend[0..1] -> s.xrecv[world][2].
int x_allgather2(const std::vector<ksim_handle*>& hs, hipStream_t stream) {
  ksim_handle* h0 = hs[0];
  if (h0->comm) {
    const ncclResult_t r = rccl().all_gather(h0->sc.xsend, h0->sc.xrecv, 2, ncclUint64, h0->comm, stream);
    if (r != ncclSuccess) return set_err(h0, KSIM_E_RCCL, std::string("ncclAllGather: ") + rccl().error_string(r));
    return KSIM_OK;
  }
  GroupPtrs src{}, dst{};
  src.n = dst.n = (int32_t)hs.size();
  for (size_t i = 0; i < hs.size(); i++) {
    src.p[i] = hs[i]->sc.xsend;
    dst.p[i] = hs[i]->sc.xrecv;
  }
  launch_group_gather(src, dst, 2, stream);
  return KSIM_OK;
}

// One per-pod cycle (the pod at the shards' common cursor) across node shards,
// with exchanges of xdom / xreg words (at least the pod's own lengths: words
// past them are summed but never read).
int shard_cycle(const std::vector<ksim_handle*>& hs, bool topo, int64_t xdom, int64_t xreg, hipStream_t stream) {
  ksim_handle* h0 = hs[0];
  const int R = (int)hs.size();
  const int32_t world = h0->comm ? h0->world : R;
  int rc;
  if (topo) {
    for (auto* h : hs) launch_pshard_topo(make_args(h, h->dp, h->d_chosen), stream);
    if ((rc = x_allreduce(hs, [](ksim_handle* h) { return h->sc.xdom; }, xdom, false, stream))) return rc;
  }
  for (auto* h : hs) launch_pshard_filter(make_args(h, h->dp, h->d_chosen), topo, stream);
  if ((rc = x_allgather2(hs, stream))) return rc;      // C3: feasible counts per shard
  for (int i = 0; i < R; i++)
    launch_pshard_window(make_args(hs[i], hs[i]->dp, hs[i]->d_chosen), h0->comm ? h0->rank : i, world, stream);
  if ((rc = x_allreduce(hs, [](ksim_handle* h) { return h->sc.xreg; }, xreg, false, stream))) return rc;
  for (auto* h : hs) launch_pshard_extrema(make_args(h, h->dp, h->d_chosen), xreg > 0, stream);
  if ((rc = x_allreduce(hs, [](ksim_handle* h) { return h->sc.win->ext; }, kExtWords, true, stream))) return rc;
  for (auto* h : hs) launch_pshard_select(make_args(h, h->dp, h->d_chosen), stream);
  if ((rc = x_allgather2(hs, stream))) return rc;      // C2: every shard's (total, TB) best
  for (auto* h : hs) launch_pshard_bind(make_args(h, h->dp, h->d_chosen), world, stream);
  HIPCHK(h0, hipGetLastError());
  return KSIM_OK;
}

int shard_cycle(const std::vector<ksim_handle*>& hs, int32_t pod, hipStream_t stream) {
  const ksim_handle* h0 = hs[0];
  return shard_cycle(hs, h0->topo[pod] != 0, h0->xdom_len[pod], h0->xreg_len[pod], stream);
}

// kGraphCycles sharded cycles of one shape as a graph on the leader (its
// stream carries every shard's kernels and the collectives), or nullptr when
// capture is off or fails (the caller runs the cycles eagerly).
hipGraphExec_t shard_graph(const std::vector<ksim_handle*>& hs, bool topo, int64_t xdom, int64_t xreg) {
  ksim_handle* h0 = hs[0];
  if (h0->sg_off || ab(kAbShardGraph)) return nullptr;
  std::vector<std::pair<const ksim_handle*, int64_t>> sig;
  for (auto* h : hs) sig.emplace_back(h, h->graph_gen);
  if (sig != h0->sg_sig) {                     // another group, or some handle dropped its graphs
    for (auto& kv : h0->sg_graphs) (void)hipGraphExecDestroy(kv.second);
    h0->sg_graphs.clear();
    h0->sg_sig = sig;
  }
  const auto key = std::make_tuple(topo, xdom, xreg);
  auto it = h0->sg_graphs.find(key);
  if (it != h0->sg_graphs.end()) return it->second;
  hipStream_t stream = h0->stream;
  if (hipStreamSynchronize(stream) != hipSuccess) return nullptr;
  hipGraph_t g = nullptr;
  hipGraphExec_t ge = nullptr;
  bool ok = hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal) == hipSuccess;
  for (int i = 0; ok && i < kGraphCycles; i++) ok = shard_cycle(hs, topo, xdom, xreg, stream) == KSIM_OK;
  const hipError_t e = hipStreamEndCapture(stream, &g);   // ends a capture even after a failed launch
  ok = ok && e == hipSuccess && g && hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) == hipSuccess;
  if (g) (void)hipGraphDestroy(g);
  (void)hipGetLastError();
  if (!ok) {
    h0->sg_off = true;
    h0->err.clear();
    return nullptr;
  }
  h0->graph_captures++;
  h0->sg_graphs.emplace(key, ge);
  return ge;
}

// kGraphBatches sharded batches (every shard's kernels and the exchanges on
// the leader's stream, RCCL collectives included) as a graph, cached with the
// per-pod shard graphs; nullptr when capture is off or fails (eager batches).
int shard_batch_adapt(const std::vector<ksim_handle*>& hs, hipStream_t stream, bool fast);

hipGraphExec_t shard_batch_graph(const std::vector<ksim_handle*>& hs, bool fast, bool adapt) {
  ksim_handle* h0 = hs[0];
  if (h0->sg_off || ab(kAbShardGraph)) return nullptr;
  std::vector<std::pair<const ksim_handle*, int64_t>> sig;
  for (auto* h : hs) sig.emplace_back(h, h->graph_gen);
  if (sig != h0->sg_sig) {
    for (auto& kv : h0->sg_graphs) (void)hipGraphExecDestroy(kv.second);
    h0->sg_graphs.clear();
    h0->sg_sig = sig;
  }
  const auto key = std::make_tuple(fast, (int64_t)(adapt ? -2 : -1), (int64_t)-1);   // per-pod keys: lengths >= 0
  auto it = h0->sg_graphs.find(key);
  if (it != h0->sg_graphs.end()) return it->second;
  hipStream_t stream = h0->stream;
  if (hipStreamSynchronize(stream) != hipSuccess) return nullptr;
  hipGraph_t g = nullptr;
  hipGraphExec_t ge = nullptr;
  bool ok = hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal) == hipSuccess;
  for (int i = 0; ok && i < kGraphBatches; i++)
    ok = (adapt ? shard_batch_adapt(hs, stream, fast) : shard_batch(hs, stream, fast)) == KSIM_OK;
  const hipError_t e = hipStreamEndCapture(stream, &g);
  ok = ok && e == hipSuccess && g && hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) == hipSuccess;
  if (g) (void)hipGraphDestroy(g);
  (void)hipGetLastError();
  if (!ok) {
    h0->sg_off = true;
    h0->err.clear();
    return nullptr;
  }
  h0->graph_captures++;
  h0->sg_graphs.emplace(key, ge);
  return ge;
}

// Pods [a, b) on the sharded per-pod path, one cycle each: whole graphs of
// kGraphCycles cycles shaped for the run's largest exchanges, then single
// cycles for the rest.
int shard_run_perpod(const std::vector<ksim_handle*>& hs, int32_t a, int32_t b) {
  ksim_handle* h0 = hs[0];
  hipStream_t stream = h0->stream;
  for (auto* h : hs) {
    int rc;
    if ((rc = set_run(h, a, b))) return rc;
    HIPCHK(h, hipStreamSynchronize(h->stream));
  }
  int32_t i = a;
  if (b - a >= kGraphCycles) {
    const bool topo = h0->topo[a] != 0;          // runs are uniform in topo (for_each_run)
    int64_t xdom = 0, xreg = 0;
    for (int32_t k = a; k < b; k++) {
      xdom = std::max(xdom, h0->xdom_len[k]);
      xreg = std::max(xreg, h0->xreg_len[k]);
    }
    if (hipGraphExec_t g = shard_graph(hs, topo, xdom, xreg))
      for (; i + kGraphCycles <= b; i += kGraphCycles) HIPCHK(h0, hipGraphLaunch(g, stream));
  }
  for (; i < b; i++) {
    int rc = shard_cycle(hs, i, stream);
    if (rc) return rc;
  }
  return KSIM_OK;
}

// ---- node-sharded ADAPT batch path (ksim_adapt.hip "node-sharded ADAPT batch") ----
// The shard layout it needs: R shards of chunk = ceil(ceil(N / R) / 64) * 64
// nodes each (the last one the rest, non-empty), in order (ksim/shard.py
// partition follows it whenever it can).
int32_t adapt_shard_chunk(int32_t n_total, int32_t world) {
  const int32_t q = (n_total + world - 1) / world;
  return (q + 63) / 64 * 64;
}

bool adapt_shard_layout(const std::vector<ksim_handle*>& hs) {
  const ksim_handle* h0 = hs[0];
  const int32_t world = h0->comm ? h0->world : (int32_t)hs.size();
  const int32_t N = h0->dc.n_total, chunk = adapt_shard_chunk(N, world);
  if ((int64_t)(world - 1) * chunk >= N) return false;
  for (size_t i = 0; i < hs.size(); i++) {
    const int32_t r = h0->comm ? h0->rank : (int32_t)i;
    const int32_t base = r * chunk, n = std::min(chunk, N - base);
    if (hs[i]->dc.base != base || hs[i]->dc.n != n) return false;
  }
  return true;
}

int adapt_shard_buffers(ksim_handle* h, int32_t world, int32_t W) {
  if (h->ash_world == world && h->ash_w == W) return KSIM_OK;
  HIPCHK(h, hipStreamSynchronize(h->stream));
  drop_cycle_graphs(h);                           // shard batch graphs captured over the old buffers
  free_bufs(h->ash_bufs);
  const size_t nw = (size_t)(h->dc.n_total + 63) / 64;
  void* p = nullptr;
  int rc;
  if ((rc = upload(h, h->ash_bufs, nullptr, 8 * (size_t)kBatchPods * W, &p))) return rc;
  h->ash_send = (uint64_t*)p;
  if ((rc = upload(h, h->ash_bufs, nullptr, 8 * (size_t)world * kBatchPods * W, &p))) return rc;
  h->ash_recv = (uint64_t*)p;
  if ((rc = upload(h, h->ash_bufs, nullptr, 8 * (size_t)kBatchPods * nw, &p))) return rc;
  h->ash_gmask = (uint64_t*)p;
  h->ash_world = world;
  h->ash_w = W;
  return KSIM_OK;
}

// One ADAPT batch on every shard of a group (exchanges: bitmaps, records, M).
int shard_batch_adapt(const std::vector<ksim_handle*>& hs, hipStream_t stream, bool fast) {
  auto args = [&](ksim_handle* h) {
    LaunchArgs la = make_args(h, h->dp, h->d_chosen);
    la.fast = fast;
    return la;
  };
  const int R = (int)hs.size();
  ksim_handle* h0 = hs[0];
  const int32_t world = h0->comm ? h0->world : R;
  const int32_t W = adapt_shard_chunk(h0->dc.n_total, world) / 64;
  const size_t mw = (size_t)kBatchPods * W;                   // bitmap words per shard
  for (auto* h : hs) launch_adapt_sh_mask(args(h), h->ash_send, W, stream);
  if (h0->comm) {
    const ncclResult_t r = rccl().all_gather(h0->ash_send, h0->ash_recv, mw, ncclUint64, h0->comm, stream);
    if (r != ncclSuccess) return set_err(h0, KSIM_E_RCCL, std::string("ncclAllGather: ") + rccl().error_string(r));
  } else {
    for (int src = 0; src < R; src++)
      for (int dst = 0; dst < R; dst++)
        HIPCHK(h0, hipMemcpyAsync(hs[dst]->ash_recv + (size_t)src * mw, hs[src]->ash_send, 8 * mw,
                                  hipMemcpyDeviceToDevice, stream));
  }
  for (auto* h : hs) launch_adapt_sh_window(args(h), h->ash_recv, W, h->ash_gmask, stream);
  const size_t rec = (size_t)kBatchPods * kXRec;
  if (h0->comm) {
    const ncclResult_t r = rccl().all_gather(h0->sc.xsend, h0->sc.xrecv, rec, ncclUint64, h0->comm, stream);
    if (r != ncclSuccess) return set_err(h0, KSIM_E_RCCL, std::string("ncclAllGather: ") + rccl().error_string(r));
  } else {
    for (int src = 0; src < R; src++)
      for (int dst = 0; dst < R; dst++)
        HIPCHK(h0, hipMemcpyAsync(hs[dst]->sc.xrecv + (size_t)src * rec, hs[src]->sc.xsend, 8 * rec,
                                  hipMemcpyDeviceToDevice, stream));
  }
  for (auto* h : hs) launch_adapt_sh_pairs(args(h), h->ash_gmask, world, stream);
  int rc;
  if ((rc = x_allreduce(hs, [](ksim_handle* h) { return h->sc.pmax; }, 2 * kBatchPods, true, stream))) return rc;
  for (auto* h : hs) launch_adapt_sh_commit(args(h), stream);
  HIPCHK(h0, hipGetLastError());
  return KSIM_OK;
}

// Pods [a, b) on the sharded ADAPT batch path.
int shard_run_adapt(const std::vector<ksim_handle*>& hs, int32_t a, int32_t b) {
  ksim_handle* h0 = hs[0];
  hipStream_t stream = h0->stream;
  const int32_t world = h0->comm ? h0->world : (int32_t)hs.size();
  const int32_t W = adapt_shard_chunk(h0->dc.n_total, world) / 64;
  bool fast = run_fast(h0, a, b);                      // every shard alike
  for (auto* h : hs) fast = fast && h->alloc_narrow;
  for (auto* h : hs) {
    int rc;
    if ((rc = adapt_shard_buffers(h, world, W))) return rc;
    if ((rc = set_run(h, a, b))) return rc;
    HIPCHK(h, hipStreamSynchronize(h->stream));
  }
  const hipGraphExec_t g = b - a >= kBatchPods * kGraphBatches ? shard_batch_graph(hs, fast, true) : nullptr;
  int32_t cursor = a;
  while (cursor < b) {
    const int32_t left = b - cursor;
    if (g && left >= kBatchPods * kGraphBatches) {   // as shard_run
      const int reps = left / (kBatchPods * kGraphBatches);
      for (int r = 0; r < reps; r++) HIPCHK(h0, hipGraphLaunch(g, stream));
    } else {
      const int32_t n = std::max(1, left / kBatchPods);
      for (int32_t i = 0; i < n; i++) {
        int rc = shard_batch_adapt(hs, stream, fast);
        if (rc) return rc;
      }
    }
    DevState st;
    HIPCHK(h0, hipMemcpyAsync(&st, h0->st, sizeof(st), hipMemcpyDeviceToHost, stream));
    HIPCHK(h0, hipStreamSynchronize(stream));
    if (st.cursor <= cursor) return set_err(h0, KSIM_E_DEVICE, "sharded ADAPT batch path made no progress");
    cursor = st.cursor;
  }
  return KSIM_OK;
}

// A sharded run: batchable stretches on the batch protocol, the rest cycle by cycle.
int shard_schedule(const std::vector<ksim_handle*>& hs, int32_t first, int32_t count) {
  if (profile_nb(hs[0]->prof))
    return set_err(hs[0], KSIM_E_UNSUPPORTED, "NetworkBandwidth profiles run on unsharded handles");
  if (hs[0]->replicated) {
    // P100 batch stretches on the replicated exchange; everything else runs
    // whole on every replica (the same cycles, so the replicas stay equal)
    const bool adapt = adapt_mode(hs[0]);
    return for_each_run(hs[0], first, count, [&](int32_t a, int32_t b, bool batch, bool topo) {
      if (batch && !adapt) return topo ? shard_run_tbatch(hs, a, b) : shard_run(hs, a, b);
      for (auto* h : hs) {
        int rc = run_range(h, a, b, batch, topo);
        if (rc) return rc;
      }
      return (int)KSIM_OK;
    }, true);
  }
  const bool adapt = adapt_mode(hs[0]);
  const bool adapt_batch = adapt && adapt_shard_layout(hs);
  return for_each_run(hs[0], first, count, [&](int32_t a, int32_t b, bool batch, bool) {
    if (!batch) return shard_run_perpod(hs, a, b);
    return adapt ? shard_run_adapt(hs, a, b) : shard_run(hs, a, b);
  }, adapt_batch);
}



int reset_counters(ksim_handle* h, hipStream_t stream) {
  HIPCHK(h, hipMemsetAsync(&h->st->truncations, 0, 4, stream));
  HIPCHK(h, hipMemsetAsync(&h->st->evals, 0, 3 * sizeof(int64_t), stream));
  HIPCHK(h, hipMemsetAsync(&h->st->batches, 0, 4, stream));
  HIPCHK(h, hipMemsetAsync(&h->st->cuts, 0, 8, stream));
  return KSIM_OK;
}

}  // namespace

extern "C" {

int ksim_abi_version(void) { return KSIM_ABI_VERSION; }

size_t ksim_abi_sizeof(int which) {
  switch (which) {
    case 0: return sizeof(ksim_node_table);
    case 1: return sizeof(ksim_vocab);
    case 2: return sizeof(ksim_label_expr);
    case 3: return sizeof(ksim_term);
    case 4: return sizeof(ksim_pod);
    case 5: return sizeof(ksim_pod_set);
    case 6: return sizeof(ksim_profile);
    case 7: return sizeof(ksim_eval_out);
    case 8: return sizeof(ksim_batch_stats);
    case 9: return sizeof(ksim_topo_use);
    case 10: return sizeof(ksim_class_add);
    case 11: return sizeof(ksim_match_problem);
    case 12: return sizeof(ksim_k8s_kv);
    case 13: return sizeof(ksim_k8s_taint);
    case 14: return sizeof(ksim_k8s_toleration);
    case 15: return sizeof(ksim_k8s_requirement);
    case 16: return sizeof(ksim_k8s_selector_term);
    case 17: return sizeof(ksim_k8s_preferred_term);
    case 18: return sizeof(ksim_k8s_label_selector);
    case 19: return sizeof(ksim_k8s_pod_term);
    case 20: return sizeof(ksim_k8s_spread);
    case 21: return sizeof(ksim_k8s_port);
    case 22: return sizeof(ksim_k8s_container);
    case 23: return sizeof(ksim_k8s_image);
    case 24: return sizeof(ksim_k8s_volume_group);
    case 25: return sizeof(ksim_k8s_node);
    case 26: return sizeof(ksim_k8s_pod);
    case 27: return sizeof(ksim_k8s_namespace);
    case 28: return sizeof(ksim_k8s_service);
    case 29: return sizeof(ksim_k8s_controller);
    case 30: return sizeof(ksim_k8s_pool);
    case 31: return sizeof(ksim_encode_nodes_opts);
    case 32: return sizeof(ksim_encode_pods_opts);
    case 33: return sizeof(ksim_encoder_info);
    default: return 0;
  }
}

int ksim_create(int device, ksim_handle** out) {
  if (!out) return KSIM_E_INVALID;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return KSIM_E_DEVICE;
  if (device < 0 || device >= ndev) return KSIM_E_INVALID;
  auto* h = new ksim_handle();
  h->device = device;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&h->ev0) != hipSuccess || hipEventCreate(&h->ev1) != hipSuccess ||
      hipMalloc(&h->st, sizeof(DevState)) != hipSuccess || hipMemset(h->st, 0, sizeof(DevState)) != hipSuccess ||
      // written only by ksim_set_profile, on the engine's stream (a null-stream
      // memset here would not be ordered before that copy)
      hipMalloc(&h->d_prof, sizeof(ksim_profile)) != hipSuccess ||
      hipMalloc(&h->d_bp, sizeof(BatchProg)) != hipSuccess) {
    delete h;
    return KSIM_E_DEVICE;
  }
  *out = h;
  return KSIM_OK;
}

void ksim_destroy(ksim_handle* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  drop_graphs(h);
  if (h->comm && rccl().ok) (void)rccl().comm_destroy(h->comm);
  free_bufs(h->cluster_bufs);
  free_bufs(h->scratch_bufs);
  free_bufs(h->ash_bufs);
  free_bufs(h->lazy_bufs);
  free_bufs(h->stab_bufs);
  free_bufs(h->pod_bufs);
  if (h->pod1_arena.p) (void)hipFree(h->pod1_arena.p);
  if (h->nom_arena.p) (void)hipFree(h->nom_arena.p);
  for (auto& a : h->fw_arena)
    if (a.p) (void)hipFree(a.p);
  if (h->fwh) (void)hipHostFree(h->fwh);
  if (h->pin) (void)hipHostFree(h->pin);
  if (h->pout) (void)hipHostFree(h->pout);
  free_bufs(h->pre_bufs);
  free_bufs(h->pre_nom_bufs);
  if (h->d_chosen) (void)hipFree(h->d_chosen);
  if (h->st) (void)hipFree(h->st);
  if (h->d_prof) (void)hipFree(h->d_prof);
  if (h->d_bp) (void)hipFree(h->d_bp);
  for (auto& r : h->ring) {
    if (r.p) (void)hipHostFree(r.p);
    if (r.ev) (void)hipEventDestroy(r.ev);
  }
  if (h->ev0) (void)hipEventDestroy(h->ev0);
  if (h->ev1) (void)hipEventDestroy(h->ev1);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
}

const char* ksim_last_error(const ksim_handle* h) { return h ? h->err.c_str() : "null handle"; }

int ksim_set_profile(ksim_handle* h, const ksim_profile* p) {
  if (const int prc = flush_pend_bind(h)) return prc;   // a queued Reserve lands first
  if (!h || !p) return KSIM_E_INVALID;
  h->stab_dirty = true;                     // DevPods::stab: the static filter list may change
  if (p->n_filter < 0 || p->n_filter > KSIM_MAX_FILTER || p->n_score < 0 || p->n_score > KSIM_MAX_SCORE)
    return set_err(h, KSIM_E_INVALID, "plugin count out of range");
  for (int i = 0; i < p->n_filter; i++) {
    if (!plugin_supported(p->filter[i])) return set_err(h, KSIM_E_INVALID, "unknown filter plugin id");
    for (int j = 0; j < i; j++)
      if (p->filter[j] == p->filter[i]) return set_err(h, KSIM_E_INVALID, "filter plugin listed twice");
  }
  for (int i = 0; i < p->n_score; i++) {
    if (!plugin_supported(p->score[i])) return set_err(h, KSIM_E_INVALID, "unknown score plugin id");
    for (int j = 0; j < i; j++)
      if (p->score[j] == p->score[i]) return set_err(h, KSIM_E_INVALID, "score plugin listed twice");
    if (p->score_weight[i] < 0) return set_err(h, KSIM_E_INVALID, "negative score weight");
  }
  if (p->fit_n_res < 0 || p->fit_n_res > KSIM_MAX_RES || p->ba_n_res < 0 || p->ba_n_res > KSIM_MAX_RES)
    return set_err(h, KSIM_E_INVALID, "scoring resources out of range");
  // NodeResourcesFitArgs / DefaultPreemptionArgs as validation.ValidateNodeResourcesFitArgs /
  // ValidateDefaultPreemptionArgs accept them (the plugin constructors refuse anything else)
  if (p->fit_strategy < KSIM_FIT_LEAST_ALLOCATED || p->fit_strategy > KSIM_FIT_REQUESTED_TO_CAPACITY_RATIO)
    return set_err(h, KSIM_E_INVALID, "unknown NodeResourcesFit scoring strategy");
  if (p->fit_strategy == KSIM_FIT_REQUESTED_TO_CAPACITY_RATIO) {
    if (p->fit_n_shape < 1 || p->fit_n_shape > KSIM_MAX_SHAPE)
      return set_err(h, KSIM_E_INVALID, "RequestedToCapacityRatio shape: 1..16 points");
    for (int i = 0; i < p->fit_n_shape; i++) {
      if (p->fit_shape_util[i] < 0 || p->fit_shape_util[i] > 100 || (i > 0 && p->fit_shape_util[i] <= p->fit_shape_util[i - 1]))
        return set_err(h, KSIM_E_INVALID, "RequestedToCapacityRatio shape: utilization strictly increasing in [0, 100]");
      if (p->fit_shape_score[i] < 0 || p->fit_shape_score[i] > 100 || p->fit_shape_score[i] % 10 != 0)
        return set_err(h, KSIM_E_INVALID, "RequestedToCapacityRatio shape: score x 10 in [0, 100]");
    }
  }
  if (p->fit_ignored_scalar >> KSIM_MAX_SCALAR) return set_err(h, KSIM_E_INVALID, "fit_ignored_scalar past the scalar columns");
  if (p->preempt_min_pct < 0 || p->preempt_min_pct > 100 || p->preempt_min_abs < 0 ||
      (p->preempt_min_pct == 0 && p->preempt_min_abs == 0))
    return set_err(h, KSIM_E_INVALID, "DefaultPreemptionArgs: minCandidateNodesPercentage in [0, 100], "
                                      "minCandidateNodesAbsolute >= 0, not both 0");
  // the profile compiled for batchable pods (see BatchProg in ksim_device.h)
  BatchProg bp{};
  // the FAST / cpu-memory keys implement LeastAllocated; the other strategies
  // take the generic keys (fit_score)
  bp.cpu_mem = p->fit_strategy == KSIM_FIT_LEAST_ALLOCATED && p->fit_n_res == 2 && p->fit_res[0] == KSIM_RES_CPU &&
               p->fit_res[1] == KSIM_RES_MEMORY && p->ba_n_res == 2 && p->ba_res[0] == KSIM_RES_CPU &&
               p->ba_res[1] == KSIM_RES_MEMORY;
  bp.fit_w_cpu = p->fit_res_weight[0];
  bp.fit_w_mem = p->fit_res_weight[1];
  bp.fast_w = bp.cpu_mem && bp.fit_w_cpu >= 1 && bp.fit_w_cpu < (1ll << 31) && bp.fit_w_mem >= 1 &&
              bp.fit_w_mem < (1ll << 31);
  bp.no_score = p->n_score == 0;
  bp.fit_w_eq = bp.fast_w && bp.fit_w_cpu == bp.fit_w_mem;
  if (bp.fast_w) {                                    // RN(1 / w): IEEE division on the host
    bp.inv_w[0] = 1.0 / (double)bp.fit_w_cpu;
    bp.inv_w[1] = 1.0 / (double)bp.fit_w_mem;
    bp.inv_w[2] = 1.0 / (double)(bp.fit_w_cpu + bp.fit_w_mem);
  }
  for (int i = 0; i < p->n_filter; i++) {
    const int f = p->filter[i];
    if (f == KSIM_PL_NODE_UNSCHEDULABLE || f == KSIM_PL_NODE_NAME || f == KSIM_PL_TAINT_TOLERATION ||
        f == KSIM_PL_NODE_AFFINITY)
      bp.static_filter[bp.n_static++] = (uint8_t)f;
    if (f == KSIM_PL_NODE_RESOURCES_FIT) bp.has_fit_filter = 1;
  }
  for (int k = 0; k < p->n_score; k++) {
    const int64_t w = p->score_weight[k] == 0 ? 1 : p->score_weight[k];
    if (p->score[k] == KSIM_PL_NODE_RESOURCES_FIT) bp.w_fit += w;
    if (p->score[k] == KSIM_PL_BALANCED_ALLOCATION) bp.w_ba += w;
    if (p->score[k] == KSIM_PL_TAINT_TOLERATION) bp.w_tt += w;
    if (p->score[k] == KSIM_PL_NODE_AFFINITY) bp.w_na += w;
  }
  plan_profile(*p, bp.rank_lo, bp.rank_hi, bp.slot, bp.slot_hi);
  HIPCHK(h, hipSetDevice(h->device));
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  // the batch graphs read the profile from d_prof / d_bp; only the ADAPT
  // window size K is captured by value (from percentageOfNodesToScore)
  // and the Fit filter's ignored scalar columns (DevCluster::fit_ignore); the
  // launch picks the evaluation kernel by the FAST key's shape (fast_def)
  const bool keep_batch_graphs = h->has_profile &&
                                 h->prof.percentage_of_nodes_to_score == p->percentage_of_nodes_to_score &&
                                 h->dc.fit_ignore == p->fit_ignored_scalar && fast_def(h->bp) == fast_def(bp);
  // batchability depends on the profile: a loaded queue must be reloaded (its
  // buffers stay allocated for ksim_load_pods to reuse)
  h->dp = DevPods{};
  h->batchable.clear();
  // device copies first: if one fails the handle holds no profile at all (never
  // a host profile the device copies and the kept graphs disagree with)
  hipError_t e = hipMemcpyAsync(h->d_prof, p, sizeof(ksim_profile), hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(h->d_bp, &bp, sizeof(BatchProg), hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  if (e != hipSuccess) {
    drop_graphs(h);
    h->has_profile = false;
    return hip_fail(h, e, "profile upload");
  }
  h->prof = *p;
  h->bp = bp;
  h->dc.fit_ignore = p->fit_ignored_scalar;
  h->has_profile = true;
  if (keep_batch_graphs)
    drop_cycle_graphs(h);
  else
    drop_graphs(h);
  return KSIM_OK;
}

int ksim_set_cluster(ksim_handle* h, const ksim_node_table* t, const ksim_vocab* v) {
  if (const int prc = flush_pend_bind(h)) return prc;   // a queued Reserve lands first
  if (!h || !t || !v) return KSIM_E_INVALID;
  h->stab_dirty = true;
  HIPCHK(h, hipSetDevice(h->device));
  const int32_t n = t->n_nodes;
  if (n < 0 || n > KSIM_MAX_NODES) return set_err(h, KSIM_E_INVALID, "n_nodes out of range");
  if (t->n_scalar < 0 || t->n_scalar > KSIM_MAX_SCALAR) return set_err(h, KSIM_E_INVALID, "n_scalar out of range");
  if (t->n_label_cols < 0 || t->n_label_cols > KSIM_MAX_LABEL_COLS)
    return set_err(h, KSIM_E_INVALID, "n_label_cols out of range");
  if (v->n_taints < 1 || v->n_taints > 64 * KSIM_TAINT_WORDS || !v->taint_effect)
    return set_err(h, KSIM_E_INVALID, "n_taints out of range");
  if (n > 0 && (!t->alloc_cpu || !t->alloc_mem || !t->alloc_eph || !t->alloc_pods || !t->req_cpu || !t->req_mem ||
                !t->req_eph || !t->nz_cpu || !t->nz_mem || !t->num_pods || !t->flags || !t->taints ||
                (t->n_label_cols > 0 && !t->labels) || (t->n_scalar > 0 && (!t->alloc_scalar || !t->req_scalar))))
    return set_err(h, KSIM_E_INVALID, "null node column");
  for (size_t i = 0; i < (size_t)n * KSIM_MAX_NODE_TAINTS; i++)
    if (t->taints[i] >= v->n_taints) return set_err(h, KSIM_E_INVALID, "taint id out of vocabulary");
  if (t->n_label_cols > 0 && (!v->label_col_offset || (v->n_label_values > 0 && (!v->label_num || !v->label_num_ok))))
    return set_err(h, KSIM_E_INVALID, "null label vocabulary");
  // value ids per label column: every label id must index its column's domain
  // tables (device atomics use it as an address)
  std::vector<int32_t> col_nvals((size_t)t->n_label_cols, 0);
  int32_t vmax = 1;
  for (int k = 0; k < t->n_label_cols; k++) {
    const int32_t end = k + 1 < t->n_label_cols ? v->label_col_offset[k + 1] : v->n_label_values;
    col_nvals[k] = end - v->label_col_offset[k];
    if (v->label_col_offset[k] < 0 || col_nvals[k] < 1 || end > v->n_label_values)
      return set_err(h, KSIM_E_INVALID, "label_col_offset not increasing within n_label_values");
    if (col_nvals[k] > KSIM_MAX_NODES + 1) return set_err(h, KSIM_E_INVALID, "label column vocabulary too large");
    vmax = std::max(vmax, col_nvals[k]);
    for (int32_t i = 0; i < n; i++)
      if (t->labels[(size_t)k * n + i] >= (uint32_t)col_nvals[k])
        return set_err(h, KSIM_E_INVALID, "label value id out of its column's vocabulary");
  }
  if (t->n_classes < 0 || t->n_classes > KSIM_MAX_CLASSES || (t->n_classes > 0 && n > 0 && !t->class_count))
    return set_err(h, KSIM_E_INVALID, "n_classes out of range / null class_count");
  if (v->n_topo_log < 0 || (v->n_topo_log > 0 && !v->topo_log))
    return set_err(h, KSIM_E_INVALID, "bad topo_log");
  (void)hipStreamSynchronize(h->stream);
  // the inputs are valid: the old snapshot goes, and with it the evaluation
  // range (a replica calls ksim_set_eval_range again)
  h->replicated = false;
  drop_graphs(h);
  free_bufs(h->cluster_bufs);
  free_bufs(h->scratch_bufs);
  free_bufs(h->ash_bufs);
  free_bufs(h->lazy_bufs);
  h->lazy_n = -1;
  h->ash_send = h->ash_recv = h->ash_gmask = nullptr;
  h->ash_world = h->ash_w = 0;
  free_bufs(h->pod_bufs);
  h->pod_buf_bytes.clear();
  h->dp = DevPods{};
  h->batchable.clear();
  h->topo.clear();
  h->has_cluster = false;
  // node positions of the old snapshot: the bound-pod table and a pending
  // extender round trip do not carry over
  free_bufs(h->pre_bufs);
  free_bufs(h->pre_nom_bufs);
  h->pre = DevPreempt{};
  h->pre_index.clear();
  h->pre_n = 0;
  h->ext_pending = false;
  h->fw_pending = h->fw_scored = h->fw_dom_dirty = false;   // fresh scratch below
  h->deferred_binds.clear();           // Reserve / Unreserve queued against the old node positions

  const int32_t n_total = h->shard_total ? h->shard_total : n;
  if (h->shard_base < 0 || h->shard_base + n > n_total || n_total > KSIM_MAX_NODES)
    return set_err(h, KSIM_E_INVALID, "shard range outside the cluster (ksim_set_shard)");
  DevCluster c{};
  c.count_whole = 1;
  c.base = h->shard_base;
  c.n_total = n_total;
  c.n_classes = t->n_classes;
  c.n_topo_log = v->n_topo_log;
  c.vmax = vmax;
  c.n = n;
  c.n_scalar = t->n_scalar;
  c.n_label_cols = t->n_label_cols;
  c.n_taints = v->n_taints;
  c.n_label_values = v->n_label_values;
  const size_t N = (size_t)n;
  int rc;
#define UP(field, src, bytes)                                                         \
  do {                                                                                \
    void* _p = nullptr;                                                               \
    if ((rc = upload(h, h->cluster_bufs, (src), (bytes), &_p)) != KSIM_OK) return rc; \
    c.field = reinterpret_cast<decltype(c.field)>(_p);                                \
  } while (0)
  UP(alloc_cpu, t->alloc_cpu, 8 * N);
  UP(alloc_mem, t->alloc_mem, 8 * N);
  UP(alloc_eph, t->alloc_eph, 8 * N);
  UP(alloc_pods, t->alloc_pods, 4 * N);
  UP(alloc_scalar, t->alloc_scalar, 8 * N * t->n_scalar);
  UP(req_cpu, t->req_cpu, 8 * N);
  UP(req_mem, t->req_mem, 8 * N);
  UP(req_eph, t->req_eph, 8 * N);
  UP(req_scalar, t->req_scalar, 8 * N * t->n_scalar);
  UP(nz_cpu, t->nz_cpu, 8 * N);
  UP(nz_mem, t->nz_mem, 8 * N);
  UP(num_pods, t->num_pods, 4 * N);
  UP(flags, t->flags, 4 * N);
  UP(taints, t->taints, 2 * N * KSIM_MAX_NODE_TAINTS);
  UP(labels, t->labels, 4 * N * t->n_label_cols);
  UP(taint_effect, v->taint_effect, (size_t)v->n_taints);
  UP(label_col_offset, v->label_col_offset, 4 * (size_t)t->n_label_cols);
  UP(label_num, v->label_num, 8 * (size_t)std::max(v->n_label_values, 0));
  UP(label_num_ok, v->label_num_ok, (size_t)std::max(v->n_label_values, 0));
  UP(cnt, t->class_count, 4 * N * (size_t)t->n_classes);
  UP(topo_log, v->topo_log, 8 * (size_t)v->n_topo_log);
  UP(col_nvals, col_nvals.data(), 4 * col_nvals.size());
  {
    // label columns whose every value sits on at most one node (hostname):
    // InterPodAffinity reads the node's own count there (kUseUniqueCol); off
    // on shard handles, whose domain sums are exchanged as tables
    std::vector<uint8_t> uniq((size_t)t->n_label_cols, 0);
    if (!h->shard_total) {
      std::vector<uint8_t> seen;
      for (int k = 0; k < t->n_label_cols; k++) {
        seen.assign((size_t)col_nvals[k], 0);
        bool u = true;
        for (int32_t i = 0; i < n && u; i++) {
          const uint32_t v = t->labels[(size_t)k * n + i];
          if (v && seen[v]++) u = false;
        }
        uniq[k] = u;
      }
    }
    UP(col_unique, uniq.data(), uniq.size());
    h->col_unique = uniq;
    h->col_total.assign((size_t)t->n_label_cols, 1);
    for (int k = 0; k < t->n_label_cols; k++)
      for (int32_t i = 0; i < n && h->col_total[k]; i++)
        if (!t->labels[(size_t)k * n + i]) h->col_total[k] = 0;
  }
  UP(nb_limit, t->nb_limit, 8 * N);                      // zeros when no node has the annotation
  UP(nb_alloc, t->nb_alloc, 8 * N);
  {
    std::vector<double> ic(N), im(N);                  // RN(1 / allocatable): IEEE division on the host
    for (size_t i = 0; i < N; i++) {
      ic[i] = t->alloc_cpu[i] ? 1.0 / (double)t->alloc_cpu[i] : 0.0;
      im[i] = t->alloc_mem[i] ? 1.0 / (double)t->alloc_mem[i] : 0.0;
    }
    UP(inv_cpu, ic.data(), 8 * N);
    UP(inv_mem, im.data(), 8 * N);
  }
#undef UP
  h->col_nvals = col_nvals;
  c.fit_ignore = h->has_profile ? h->prof.fit_ignored_scalar : 0u;
  h->dc = c;
  h->taint_effect.assign(v->taint_effect, v->taint_effect + v->n_taints);
  {
    std::vector<uint8_t> seen((size_t)v->n_taints, 0);
    for (size_t i = 0; i < (size_t)n * KSIM_MAX_NODE_TAINTS; i++) seen[t->taints[i]] = 1;
    h->hard_taints.clear();
    for (int id = 1; id < v->n_taints; id++)
      if (seen[id] && (v->taint_effect[id] == KSIM_EFFECT_NO_SCHEDULE || v->taint_effect[id] == KSIM_EFFECT_NO_EXECUTE))
        h->hard_taints.push_back((uint16_t)id);
    h->any_unschedulable = false;
    for (int32_t i = 0; i < n; i++) h->any_unschedulable = h->any_unschedulable || (t->flags[i] & KSIM_NODE_UNSCHEDULABLE);
    c.cflags = h->any_unschedulable ? kClusterUnschedulable : 0u;
    if (!h->hard_taints.empty()) c.cflags |= kClusterHardTaints;
    for (size_t i = 0; i < (size_t)n * KSIM_MAX_NODE_TAINTS; i++)
      if (t->taints[i] && v->taint_effect[t->taints[i]] == KSIM_EFFECT_PREFER_NO_SCHEDULE) c.cflags |= kClusterPreferTaints;
    h->dc.cflags = c.cflags;
    h->alloc_narrow = true;
    for (int32_t i = 0; i < n; i++)
      h->alloc_narrow = h->alloc_narrow && t->alloc_cpu[i] >= 0 && t->alloc_cpu[i] < (1ll << 46) &&
                        t->alloc_mem[i] >= 0 && t->alloc_mem[i] < (1ll << 46);
    if (h->alloc_narrow) h->dc.cflags |= kClusterNarrow;
  }
  {
    void* q = nullptr;
#define SNAP(field, bytes)                                                                 \
  do {                                                                                     \
    if ((rc = upload(h, h->cluster_bufs, nullptr, (bytes), &q)) != KSIM_OK) return rc;     \
    h->init.field = reinterpret_cast<decltype(h->init.field)>(q);                          \
    HIPCHK(h, hipMemcpyAsync(q, c.field, (bytes), hipMemcpyDeviceToDevice, h->stream));     \
  } while (0)
    SNAP(req_cpu, 8 * N);
    SNAP(req_mem, 8 * N);
    SNAP(req_eph, 8 * N);
    SNAP(req_scalar, 8 * N * t->n_scalar);
    SNAP(nz_cpu, 8 * N);
    SNAP(nz_mem, 8 * N);
    SNAP(num_pods, 4 * N);
    SNAP(cnt, 4 * N * (size_t)t->n_classes);
    SNAP(nb_alloc, 8 * N);
#undef SNAP
  }

  DevScratch s{};
  DevEvalOut o{};
  void* p = nullptr;
#define SCR(dst, type, bytes)                                                         \
  do {                                                                                \
    if ((rc = upload(h, h->scratch_bufs, nullptr, (bytes), &p)) != KSIM_OK) return rc; \
    dst = (type)p;                                                                    \
  } while (0)
  SCR(s.fail, uint8_t*, N);
  SCR(s.ign, uint8_t*, N);
  SCR(s.win, WinState*, sizeof(WinState));
  SCR(s.bbest, uint64_t*, 16 * ((N + 255) / 256));
  SCR(s.regbm, uint32_t*, 4 * (size_t)KSIM_MAX_USES * ((vmax + 31) / 32));
  SCR(h->ext_fail, uint8_t*, N);
  SCR(h->ext_score, int64_t*, 8 * N);
  SCR(h->fw_nodes, int32_t*, 4 * N);
  SCR(h->fw_vals, int64_t*, 8 * N);
  SCR(h->fw_out, int64_t*, 8 * N);
  SCR(s.detail, uint32_t*, 4 * N);
  SCR(s.raw, int64_t*, 8 * N * KSIM_MAX_SCORE);
  SCR(s.part, int64_t*, 8 * N);
  // [B][kMaxListRecords] list records: the node-stationary evaluation writes one per node slice
  SCR(s.topk, uint64_t*, 8 * (size_t)kBatchPods * kMaxListRecords * kTopT);
  SCR(s.topk_cnt, int32_t*, 4 * (size_t)kBatchPods * kMaxListRecords);
  SCR(s.topk_complete, int32_t*, 4 * (size_t)kBatchPods * kMaxListRecords);
  SCR(s.gkey, uint64_t*, 8 * (size_t)kBatchPods);
  SCR(s.chain_end, int32_t*, 4);
  SCR(s.pmax, uint64_t*, 8 * 2 * (size_t)kBatchPods);   // [M | sharded ADAPT broken flags]
  SCR(s.pnorm, int64_t*, 8 * 4 * (size_t)kBatchPods);
  const size_t NT = N <= (size_t)kTbMaxBlocks * 256 ? N : 0;   // topology batches (tbatch_admit)
  SCR(s.tb_fail, uint8_t*, (size_t)kTbPods * NT);
  SCR(s.tb_ign, uint8_t*, (size_t)kTbPods * NT);
  SCR(s.tb_part, int64_t*, 8 * (size_t)kTbPods * NT);
  SCR(s.tb_raw, int64_t*, 8 * (size_t)kTbPods * KSIM_MAX_SCORE * NT);
  SCR(s.tb_stat, int32_t*, 4 * (size_t)kTbPods * kVarSlots * NT);   // per zone-variant slot
  SCR(s.tb_win, WinState*, sizeof(WinState) * (size_t)kTbPods);
  SCR(s.tb_var, TbVar*, sizeof(TbVar) * (size_t)kTbPods);
  SCR(s.tb_dom, TbDom*, sizeof(TbDom) * (size_t)kTbPods * kVarDom);
  SCR(s.tb_vhold, int32_t*, 4 * (size_t)kTbPods * kVarSlots * 2 * KSIM_MAX_SCORE);
  SCR(s.tb_slot, int32_t*, 4 * (size_t)kTbPods);
  SCR(s.tb_vdom, uint8_t*, (size_t)kTbPods * NT);
  SCR(s.tb_cdom, uint8_t*, (size_t)kTbPods * kVarSlots * kTbMaxBlocks * kTopT);
  SCR(s.tb_kdom, uint8_t*, (size_t)kTbPods * kVarSlots * kTopT);
  SCR(s.tb_vnf, int32_t*, 4 * (size_t)kTbPods * kVarSlots);
  SCR(s.tb_vpods, unsigned long long*, 8);
  SCR(s.tb_clist, uint64_t*, 8 * (size_t)kTbPods * kVarSlots * kTbMaxBlocks * kTopT);
  SCR(s.tb_ccnt, int32_t*, 4 * (size_t)kTbPods * kVarSlots * kTbMaxBlocks);
  SCR(s.tb_xrecv, uint8_t*, sizeof(WinState) * (size_t)kMaxShards * kTbPods);
  SCR(s.tb_pp, uint64_t*, 8 * 2 * (size_t)kTbPods);
  SCR(s.pinv, int32_t*, 4 * (size_t)kBatchPods);
  SCR(s.dom, int64_t*, 8 * (size_t)KSIM_MAX_USES * vmax);
  SCR(s.dbg, unsigned long long*, 8 * 16);
  SCR(s.xsend, uint64_t*, 8 * (size_t)kBatchPods * kXRec);
  SCR(s.xrecv, uint64_t*, 8 * (size_t)kMaxShards * kBatchPods * kXRec);
  SCR(s.min_match, int64_t*, 8 * (size_t)KSIM_MAX_USES);
  SCR(s.xdom, int64_t*, 8 * (size_t)KSIM_MAX_USES * vmax);
  SCR(s.amask, uint64_t*, 8 * (size_t)kBatchPods * ((N + 63) / 64));
  SCR(s.awin, int32_t*, 4 * 2 * (size_t)kBatchPods);
  SCR(s.aexact, int32_t*, 4);
  SCR(s.acut, int32_t*, 4 * 2 * (size_t)kBatchPods);
  {                                      // the doubling window's tables (clusters of <= 128 bitmap words)
    const size_t NW = (N + 63) / 64 <= 128 ? N : 0;
    SCR(s.wtab, uint16_t*, 2 * 3 * (size_t)kBatchPods * std::max<size_t>(NW, 1));
    SCR(s.wtot, int32_t*, 4 * (size_t)kBatchPods);
  }
  SCR(s.abroken, int32_t*, 4 * (size_t)kBatchPods);
  SCR(s.xreg, int64_t*, 8 * (1 + (size_t)KSIM_MAX_USES * vmax));
  SCR(o.scored, uint8_t*, N);
  SCR(o.raw, int64_t*, 8 * N * KSIM_MAX_SCORE);
  SCR(o.norm, int64_t*, 8 * N * KSIM_MAX_SCORE);
  SCR(o.total, int64_t*, 8 * N);
#undef SCR
  h->sc = s;
  h->eo = o;
  DevState zero{};
  HIPCHK(h, hipMemcpyAsync(h->st, &zero, sizeof(zero), hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  h->has_cluster = true;
  if (h->d_chosen) (void)hipFree(h->d_chosen);
  h->d_chosen = nullptr;
  return KSIM_OK;
}

// Node informer deltas: the new table in nodeTree order, old_pos[i] = the
// current position of new node i or -1 (added).  The table is the new
// snapshot (static columns, vocabulary and the dynamic columns of the bound
// pods); on a kept node the binds the cycles made since the last snapshot
// (device column - snapshot column at old_pos) are replayed on top of it, for
// every scalar column / count class the handle already has.  nextStartNodeIndex
// carries over mod the new node count (upstream keeps the index and scans
// nodes[(index + i) % numAllNodes]), and so does the tie-break sequence.
// Loaded pods, the bound-pod table and captured graphs are dropped (node
// positions changed).
int ksim_upsert_nodes(ksim_handle* h, const ksim_node_table* t, const ksim_vocab* v, const int32_t* old_pos) {
  if (const int prc = flush_pend_bind(h)) return prc;   // a queued Reserve lands first
  // (a replica keeps its flag when the delta is refused; the new snapshot
  // below clears it: ksim_set_eval_range again)
  if (!h || !t || !v) return KSIM_E_INVALID;
  h->stab_dirty = true;
  if (!h->has_cluster) return set_err(h, KSIM_E_INVALID, "ksim_upsert_nodes before ksim_set_cluster");
  if (h->shard_total || h->world > 1) return set_err(h, KSIM_E_UNSUPPORTED, "ksim_upsert_nodes on a shard handle");
  HIPCHK(h, hipSetDevice(h->device));
  const int32_t n = t->n_nodes, n0 = h->dc.n;
  if (n < 0 || n > KSIM_MAX_NODES) return set_err(h, KSIM_E_INVALID, "n_nodes out of range");
  if (n > 0 && !old_pos) return set_err(h, KSIM_E_INVALID, "null old_pos");
  const int32_t s0 = h->dc.n_scalar, c0 = h->dc.n_classes;
  if (t->n_scalar < s0 || t->n_scalar > KSIM_MAX_SCALAR)
    return set_err(h, KSIM_E_INVALID, "scalar columns may only be appended");
  if (t->n_classes < c0 || t->n_classes > KSIM_MAX_CLASSES)
    return set_err(h, KSIM_E_INVALID, "count classes may only be appended");
  if (n > 0 && (!t->req_cpu || !t->req_mem || !t->req_eph || !t->nz_cpu || !t->nz_mem || !t->num_pods ||
                (t->n_scalar > 0 && !t->req_scalar) || (t->n_classes > 0 && !t->class_count)))
    return set_err(h, KSIM_E_INVALID, "null node column");
  {
    std::vector<uint8_t> seen((size_t)n0, 0);
    for (int32_t i = 0; i < n; i++) {
      const int32_t op = old_pos[i];
      if (op < -1 || op >= n0 || (op >= 0 && seen[op]++))
        return set_err(h, KSIM_E_INVALID, "old_pos: out of range or repeated");
    }
  }
  HIPCHK(h, hipStreamSynchronize(h->stream));
  DevState st{};
  HIPCHK(h, hcopy(h, &st, h->st, sizeof(st), hipMemcpyDeviceToHost));
  const size_t N = (size_t)n, N0 = (size_t)n0;
  // out = table + (device - snapshot) at old_pos, rows of n0 -> rows of n
  auto replay = [&](auto& out, const auto* dev, const auto* snap, const auto* tab, int rows, int rows0) -> int {
    using T = typename std::remove_reference<decltype(out)>::type::value_type;
    std::vector<T> a(N0 * (size_t)rows0), b(N0 * (size_t)rows0);
    if (!a.empty()) {
      HIPCHK(h, hcopy(h, a.data(), dev, sizeof(T) * a.size(), hipMemcpyDeviceToHost));
      HIPCHK(h, hcopy(h, b.data(), snap, sizeof(T) * b.size(), hipMemcpyDeviceToHost));
    }
    out.assign(N * (size_t)rows, 0);
    for (int k = 0; k < rows; k++)
      for (size_t i = 0; i < N; i++) {
        T x = tab ? tab[k * N + i] : 0;
        if (k < rows0 && old_pos[i] >= 0) x += a[k * N0 + old_pos[i]] - b[k * N0 + old_pos[i]];
        out[k * N + i] = x;
      }
    return KSIM_OK;
  };
  std::vector<int64_t> rc_, rm, re, rs, zc, zm, nb;
  std::vector<int32_t> np, cnt;
  int rc;
  const DevCluster& c = h->dc;
  if ((rc = replay(rc_, c.req_cpu, h->init.req_cpu, t->req_cpu, 1, 1)) ||
      (rc = replay(rm, c.req_mem, h->init.req_mem, t->req_mem, 1, 1)) ||
      (rc = replay(re, c.req_eph, h->init.req_eph, t->req_eph, 1, 1)) ||
      (rc = replay(rs, c.req_scalar, h->init.req_scalar, t->req_scalar, t->n_scalar, s0)) ||
      (rc = replay(zc, c.nz_cpu, h->init.nz_cpu, t->nz_cpu, 1, 1)) ||
      (rc = replay(zm, c.nz_mem, h->init.nz_mem, t->nz_mem, 1, 1)) ||
      (rc = replay(nb, c.nb_alloc, h->init.nb_alloc, t->nb_alloc, 1, 1)) ||
      (rc = replay(np, c.num_pods, h->init.num_pods, t->num_pods, 1, 1)) ||
      (rc = replay(cnt, c.cnt, h->init.cnt, t->class_count, t->n_classes, c0)))
    return rc;
  // the table becomes the snapshot (ksim_set_cluster copies it to h->init)
  if ((rc = ksim_set_cluster(h, t, v)) != KSIM_OK) return rc;
  const DevCluster& d = h->dc;
  auto put = [&](void* dst, const void* src, size_t bytes) -> int {
    if (bytes) HIPCHK(h, hcopy(h, dst, src, bytes, hipMemcpyHostToDevice));
    return KSIM_OK;
  };
  if ((rc = put(d.req_cpu, rc_.data(), 8 * N)) || (rc = put(d.req_mem, rm.data(), 8 * N)) ||
      (rc = put(d.req_eph, re.data(), 8 * N)) || (rc = put(d.req_scalar, rs.data(), 8 * rs.size())) ||
      (rc = put(d.nz_cpu, zc.data(), 8 * N)) || (rc = put(d.nz_mem, zm.data(), 8 * N)) ||
      (rc = put(d.num_pods, np.data(), 4 * N)) || (rc = put(d.cnt, cnt.data(), 4 * cnt.size())) ||
      (rc = put(d.nb_alloc, nb.data(), 8 * N)))
    return rc;
  DevState s2{};
  s2.next_start = n > 0 ? st.next_start % n : 0;
  s2.pod_seq = st.pod_seq;
  HIPCHK(h, hcopy(h, h->st, &s2, sizeof(s2), hipMemcpyHostToDevice));
  return KSIM_OK;
}

// DeleteNode: the node at `pos` leaves; later positions move down by one.  The
// table handed to ksim_upsert_nodes is the current snapshot without it, so the
// replay keeps every other node's state.
static int pin_reserve(ksim_handle* h, size_t bytes);

// UpdateNode in place: the changed rows' static columns through one launch
// from the pinned staging; the cluster facts the filter plans read (hard
// taints, unschedulable nodes, narrow allocatable, unique / total label
// columns) recomputed from the whole table on the host.
int ksim_update_node_rows(ksim_handle* h, const ksim_node_table* t, const ksim_vocab* v, const int32_t* rows,
                          int32_t n_rows) {
  if (const int prc = flush_pend_bind(h)) return prc;   // a queued Reserve lands first
  if (!h || !t || !v || n_rows < 0 || (n_rows > 0 && !rows)) return KSIM_E_INVALID;
  if (!h->has_cluster) return set_err(h, KSIM_E_INVALID, "ksim_update_node_rows before ksim_set_cluster");
  if (h->shard_total || h->world > 1) return set_err(h, KSIM_E_UNSUPPORTED, "ksim_update_node_rows on a shard handle");
  const DevCluster& c = h->dc;
  const int32_t n = c.n;
  if (t->n_nodes != n || t->n_scalar != c.n_scalar || t->n_label_cols != c.n_label_cols ||
      t->n_classes != c.n_classes || v->n_taints != c.n_taints || v->n_label_values != c.n_label_values)
    return set_err(h, KSIM_E_INVALID, "ksim_update_node_rows: the table's layout or vocabulary differs (ksim_upsert_nodes)");
  if (n > 0 && (!t->alloc_cpu || !t->alloc_mem || !t->alloc_eph || !t->alloc_pods || !t->flags || !t->taints ||
                (t->n_label_cols > 0 && !t->labels) || (t->n_scalar > 0 && !t->alloc_scalar)))
    return set_err(h, KSIM_E_INVALID, "null node column");
  for (int k = 0; k < c.n_label_cols; k++)
    if (!v->label_col_offset || (k + 1 < c.n_label_cols ? v->label_col_offset[k + 1] : v->n_label_values) -
                                        v->label_col_offset[k] != h->col_nvals[k])
      return set_err(h, KSIM_E_INVALID, "ksim_update_node_rows: a label column's vocabulary changed (ksim_upsert_nodes)");
  if (!v->taint_effect || !std::equal(h->taint_effect.begin(), h->taint_effect.end(), v->taint_effect))
    return set_err(h, KSIM_E_INVALID, "ksim_update_node_rows: the taint vocabulary changed (ksim_upsert_nodes)");
  const size_t N = (size_t)n;
  std::vector<uint8_t> seen_row((size_t)n, 0);
  for (int32_t q = 0; q < n_rows; q++) {
    const int32_t r = rows[q];
    if (r < 0 || r >= n || seen_row[r]++) return set_err(h, KSIM_E_INVALID, "rows: out of range or repeated");
    for (int k = 0; k < KSIM_MAX_NODE_TAINTS; k++)
      if (t->taints[(size_t)k * N + r] >= v->n_taints) return set_err(h, KSIM_E_INVALID, "taint id out of vocabulary");
    for (int k = 0; k < c.n_label_cols; k++)
      if (t->labels[(size_t)k * N + r] >= (uint32_t)h->col_nvals[k])
        return set_err(h, KSIM_E_INVALID, "label value id out of its column's vocabulary");
  }
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(h->stream));     // the pinned staging is free
  const int32_t words = 1 + 8 + KSIM_MAX_NODE_TAINTS + c.n_scalar + c.n_label_cols;
  int rc;
  if ((rc = pin_reserve(h, 8 * (size_t)words * (size_t)std::max(n_rows, 1)))) return rc;
  int64_t* rec = (int64_t*)h->pin;
  for (int32_t q = 0; q < n_rows; q++) {
    const int32_t r = rows[q];
    int64_t* w = rec + (size_t)q * words;
    const double ic = t->alloc_cpu[r] ? 1.0 / (double)t->alloc_cpu[r] : 0.0;   // as ksim_set_cluster
    const double im = t->alloc_mem[r] ? 1.0 / (double)t->alloc_mem[r] : 0.0;
    w[0] = r;
    w[1] = t->alloc_cpu[r];
    w[2] = t->alloc_mem[r];
    w[3] = t->alloc_eph[r];
    w[4] = t->alloc_pods[r];
    w[5] = t->flags[r];
    w[6] = t->nb_limit ? t->nb_limit[r] : 0;
    std::memcpy(&w[7], &ic, 8);
    std::memcpy(&w[8], &im, 8);
    for (int k = 0; k < KSIM_MAX_NODE_TAINTS; k++) w[9 + k] = t->taints[(size_t)k * N + r];
    for (int k = 0; k < c.n_scalar; k++) w[9 + KSIM_MAX_NODE_TAINTS + k] = t->alloc_scalar[(size_t)k * N + r];
    for (int k = 0; k < c.n_label_cols; k++)
      w[9 + KSIM_MAX_NODE_TAINTS + c.n_scalar + k] = t->labels[(size_t)k * N + r];
  }
  launch_node_rows(c, (const int64_t*)h->pin_d, n_rows, words, h->stream);
  HIPCHK(h, hipGetLastError());
  // the cluster facts, from the whole table (as ksim_set_cluster)
  {
    std::vector<uint8_t> seen((size_t)v->n_taints, 0);
    for (size_t i = 0; i < N * KSIM_MAX_NODE_TAINTS; i++) seen[t->taints[i]] = 1;
    h->hard_taints.clear();
    for (int id = 1; id < v->n_taints; id++)
      if (seen[id] && (h->taint_effect[id] == KSIM_EFFECT_NO_SCHEDULE || h->taint_effect[id] == KSIM_EFFECT_NO_EXECUTE))
        h->hard_taints.push_back((uint16_t)id);
    h->any_unschedulable = false;
    for (int32_t i = 0; i < n; i++) h->any_unschedulable = h->any_unschedulable || (t->flags[i] & KSIM_NODE_UNSCHEDULABLE);
    uint32_t cf = h->any_unschedulable ? kClusterUnschedulable : 0u;
    if (!h->hard_taints.empty()) cf |= kClusterHardTaints;
    for (size_t i = 0; i < N * KSIM_MAX_NODE_TAINTS; i++)
      if (t->taints[i] && h->taint_effect[t->taints[i]] == KSIM_EFFECT_PREFER_NO_SCHEDULE) cf |= kClusterPreferTaints;
    h->alloc_narrow = true;
    for (int32_t i = 0; i < n; i++)
      h->alloc_narrow = h->alloc_narrow && t->alloc_cpu[i] >= 0 && t->alloc_cpu[i] < (1ll << 46) &&
                        t->alloc_mem[i] >= 0 && t->alloc_mem[i] < (1ll << 46);
    if (h->alloc_narrow) cf |= kClusterNarrow;
    h->dc.cflags = cf;
    std::vector<uint8_t> uniq((size_t)c.n_label_cols, 0);
    std::vector<uint8_t> vs;
    for (int k = 0; k < c.n_label_cols; k++) {
      vs.assign((size_t)h->col_nvals[k], 0);
      bool u = true;
      for (int32_t i = 0; i < n && u; i++) {
        const uint32_t x = t->labels[(size_t)k * N + i];
        if (x && vs[x]++) u = false;
      }
      uniq[k] = u;
      h->col_total[k] = 1;
      for (int32_t i = 0; i < n && h->col_total[k]; i++)
        if (!t->labels[(size_t)k * N + i]) h->col_total[k] = 0;
    }
    if (uniq != h->col_unique && c.n_label_cols > 0) {
      HIPCHK(h, hcopy(h, const_cast<uint8_t*>(c.col_unique), uniq.data(), uniq.size(), hipMemcpyHostToDevice));
      h->col_unique = uniq;
    }
  }
  // what was compiled against the old rows: graphs, the static-class table, loaded pods
  drop_graphs(h);
  h->stab_dirty = true;
  free_bufs(h->pod_bufs);
  h->pod_buf_bytes.clear();
  h->dp = DevPods{};
  h->batchable.clear();
  h->topo.clear();
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return KSIM_OK;
}

int ksim_remove_node(ksim_handle* h, int32_t pos) {
  if (const int prc = flush_pend_bind(h)) return prc;   // a queued Reserve lands first
  if (!h || !h->has_cluster) return set_err(h, KSIM_E_INVALID, "cluster not set");
  h->stab_dirty = true;
  if (h->shard_total || h->world > 1) return set_err(h, KSIM_E_UNSUPPORTED, "ksim_remove_node on a shard handle");
  const int32_t n0 = h->dc.n;
  if (pos < 0 || pos >= n0) return set_err(h, KSIM_E_INVALID, "node position out of range");
  h->replicated = false;                        // a new snapshot: ksim_set_eval_range again
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  const DevCluster& c = h->dc;
  const int32_t n = n0 - 1;
  const size_t N0 = (size_t)n0;
  // the static columns and vocabulary, read back and compacted
  auto pull = [&](auto& out, const auto* dev, size_t rows) -> int {
    using T = typename std::remove_reference<decltype(out)>::type::value_type;
    std::vector<T> all(N0 * rows);
    if (!all.empty()) HIPCHK(h, hcopy(h, all.data(), dev, sizeof(T) * all.size(), hipMemcpyDeviceToHost));
    out.clear();
    for (size_t k = 0; k < rows; k++)
      for (size_t i = 0; i < N0; i++)
        if ((int32_t)i != pos) out.push_back(all[k * N0 + i]);
    return KSIM_OK;
  };
  std::vector<int64_t> ac, am, ae, as, rc_, rm, re, rs, zc, zm, nbl, nba;
  std::vector<int32_t> ap, np, cnt;
  std::vector<uint32_t> fl, lb;
  std::vector<uint16_t> tn;
  int rc;
  if ((rc = pull(ac, c.alloc_cpu, 1)) || (rc = pull(am, c.alloc_mem, 1)) || (rc = pull(ae, c.alloc_eph, 1)) ||
      (rc = pull(as, c.alloc_scalar, (size_t)c.n_scalar)) || (rc = pull(ap, c.alloc_pods, 1)) ||
      (rc = pull(rc_, h->init.req_cpu, 1)) || (rc = pull(rm, h->init.req_mem, 1)) ||
      (rc = pull(re, h->init.req_eph, 1)) || (rc = pull(rs, h->init.req_scalar, (size_t)c.n_scalar)) ||
      (rc = pull(zc, h->init.nz_cpu, 1)) || (rc = pull(zm, h->init.nz_mem, 1)) ||
      (rc = pull(np, h->init.num_pods, 1)) || (rc = pull(fl, c.flags, 1)) ||
      (rc = pull(tn, c.taints, KSIM_MAX_NODE_TAINTS)) || (rc = pull(lb, c.labels, (size_t)c.n_label_cols)) ||
      (rc = pull(cnt, h->init.cnt, (size_t)c.n_classes)) || (rc = pull(nbl, c.nb_limit, 1)) ||
      (rc = pull(nba, h->init.nb_alloc, 1)))
    return rc;
  std::vector<uint8_t> te(h->taint_effect);
  std::vector<int32_t> lco((size_t)c.n_label_cols);
  std::vector<int64_t> lnum((size_t)std::max(c.n_label_values, 0));
  std::vector<uint8_t> lok((size_t)std::max(c.n_label_values, 0));
  std::vector<double> tlog((size_t)c.n_topo_log);
  if (!lco.empty()) HIPCHK(h, hcopy(h, lco.data(), c.label_col_offset, 4 * lco.size(), hipMemcpyDeviceToHost));
  if (!lnum.empty()) {
    HIPCHK(h, hcopy(h, lnum.data(), c.label_num, 8 * lnum.size(), hipMemcpyDeviceToHost));
    HIPCHK(h, hcopy(h, lok.data(), c.label_num_ok, lok.size(), hipMemcpyDeviceToHost));
  }
  if (!tlog.empty()) HIPCHK(h, hcopy(h, tlog.data(), c.topo_log, 8 * tlog.size(), hipMemcpyDeviceToHost));
  ksim_node_table t{};
  t.n_nodes = n;
  t.n_scalar = c.n_scalar;
  t.n_label_cols = c.n_label_cols;
  t.alloc_cpu = ac.data();
  t.alloc_mem = am.data();
  t.alloc_eph = ae.data();
  t.alloc_pods = ap.data();
  t.alloc_scalar = as.data();
  t.req_cpu = rc_.data();
  t.req_mem = rm.data();
  t.req_eph = re.data();
  t.req_scalar = rs.data();
  t.nz_cpu = zc.data();
  t.nz_mem = zm.data();
  t.num_pods = np.data();
  t.flags = fl.data();
  t.taints = tn.data();
  t.labels = lb.data();
  t.n_classes = c.n_classes;
  t.class_count = cnt.data();
  t.nb_limit = nbl.data();
  t.nb_alloc = nba.data();
  ksim_vocab v{};
  v.n_taints = (int32_t)te.size();
  v.n_label_values = c.n_label_values;
  v.taint_effect = te.data();
  v.label_col_offset = lco.data();
  v.label_num = lnum.data();
  v.label_num_ok = lok.data();
  v.n_topo_log = c.n_topo_log;
  v.topo_log = tlog.data();
  std::vector<int32_t> old_pos((size_t)std::max(n, 1));
  for (int32_t i = 0; i < n; i++) old_pos[i] = i < pos ? i : i + 1;
  return ksim_upsert_nodes(h, &t, &v, old_pos.data());
}

int ksim_get_node_state(ksim_handle* h, int64_t* req_cpu, int64_t* req_mem, int64_t* req_eph, int64_t* nz_cpu,
                        int64_t* nz_mem, int32_t* num_pods) {
  if (!h || !h->has_cluster) return set_err(h, KSIM_E_INVALID, "cluster not set");
  if (int rc = flush_idle(h)) return rc;
  HIPCHK(h, hipSetDevice(h->device));
  const size_t N = (size_t)h->dc.n;
  HIPCHK(h, hipStreamSynchronize(h->stream));
  if (req_cpu) HIPCHK(h, hcopy(h, req_cpu, h->dc.req_cpu, 8 * N, hipMemcpyDeviceToHost));
  if (req_mem) HIPCHK(h, hcopy(h, req_mem, h->dc.req_mem, 8 * N, hipMemcpyDeviceToHost));
  if (req_eph) HIPCHK(h, hcopy(h, req_eph, h->dc.req_eph, 8 * N, hipMemcpyDeviceToHost));
  if (nz_cpu) HIPCHK(h, hcopy(h, nz_cpu, h->dc.nz_cpu, 8 * N, hipMemcpyDeviceToHost));
  if (nz_mem) HIPCHK(h, hcopy(h, nz_mem, h->dc.nz_mem, 8 * N, hipMemcpyDeviceToHost));
  if (num_pods) HIPCHK(h, hcopy(h, num_pods, h->dc.num_pods, 4 * N, hipMemcpyDeviceToHost));
  return KSIM_OK;
}

int ksim_get_nb_alloc(ksim_handle* h, int64_t* out) {
  if (!h || !h->has_cluster || !out) return set_err(h, KSIM_E_INVALID, "cluster not set / null out");
  if (int rc = flush_idle(h)) return rc;
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  HIPCHK(h, hcopy(h, out, h->dc.nb_alloc, 8 * (size_t)h->dc.n, hipMemcpyDeviceToHost));
  return KSIM_OK;
}

int ksim_get_class_count(ksim_handle* h, int32_t* out) {
  if (!h || !h->has_cluster || !out) return set_err(h, KSIM_E_INVALID, "cluster not set / null out");
  if (int rc = flush_idle(h)) return rc;
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  if (h->dc.n_classes)
    HIPCHK(h, hcopy(h, out, h->dc.cnt, 4 * (size_t)h->dc.n * h->dc.n_classes, hipMemcpyDeviceToHost));
  return KSIM_OK;
}

int ksim_get_next_start(ksim_handle* h, int32_t* next_start) {
  if (const int prc = flush_pend_bind(h)) return prc;   // a queued Reserve lands first
  if (!h || !next_start) return KSIM_E_INVALID;
  HIPCHK(h, hipStreamSynchronize(h->stream));
  HIPCHK(h, hcopy(h, next_start, &h->st->next_start, 4, hipMemcpyDeviceToHost));
  return KSIM_OK;
}

int ksim_set_next_start(ksim_handle* h, int32_t next_start) {
  if (const int prc = flush_pend_bind(h)) return prc;   // a queued Reserve lands first
  if (!h) return KSIM_E_INVALID;
  if (h->has_cluster && (next_start < 0 || next_start >= std::max(h->dc.n, 1)))
    return set_err(h, KSIM_E_INVALID, "next_start out of range");
  HIPCHK(h, hipStreamSynchronize(h->stream));
  HIPCHK(h, hcopy(h, &h->st->next_start, &next_start, 4, hipMemcpyHostToDevice));
  return KSIM_OK;
}

int ksim_set_pod_seq(ksim_handle* h, int64_t seq) {
  if (const int prc = flush_pend_bind(h)) return prc;   // a queued Reserve lands first
  if (!h) return KSIM_E_INVALID;
  HIPCHK(h, hipStreamSynchronize(h->stream));
  HIPCHK(h, hcopy(h, &h->st->pod_seq, &seq, 8, hipMemcpyHostToDevice));
  return KSIM_OK;
}

// Device copies of topology uses carry kUseUniqueCol when their key column is
// unique per node (ksim_device.h use_node_count).
static void mark_unique(const ksim_handle* h, ksim_topo_use* u, size_t n) {
  for (size_t i = 0; i < n; i++)
    if (u[i].col != KSIM_COL_NONE && u[i].col < h->col_unique.size() && h->col_unique[u[i].col])
      u[i].flags |= kUseUniqueCol;
}

// The pod's PodPlan against the current profile and cluster (uses: its device
// copies, kUseUniqueCol marked).
static PodPlan make_plan(const ksim_handle* h, const ksim_pod& p, const ksim_topo_use* uses) {
  PodPlan pl{};
  pl.m = use_masks(h->prof, uses, p.use_count);
  pl.filter_en = plan_filter_en(h->prof, p, pl.m, h->any_unschedulable, !h->hard_taints.empty());
  return pl;
}

// Re-based copy of one pod with only the expressions/terms it references.
static void single_pod_set(const ksim_pod_set* ps, int32_t i, ksim_pod& pod, std::vector<ksim_label_expr>& ex,
                           std::vector<ksim_term>& tm, std::vector<ksim_topo_use>& us,
                           std::vector<ksim_class_add>& ad, std::vector<int32_t>& nn) {
  pod = ps->pods[i];
  us.assign(ps->uses + pod.use_first, ps->uses + pod.use_first + pod.use_count);
  ad.assign(ps->adds + pod.add_first, ps->adds + pod.add_first + pod.add_count);
  if ((pod.flags & KSIM_POD_NODE_NAMES) && pod.nn_count > 0)
    nn.assign(ps->nn + pod.nn_first, ps->nn + pod.nn_first + pod.nn_count);
  pod.use_first = 0;
  pod.add_first = 0;
  pod.nn_first = 0;
  int32_t sel0 = (int32_t)ex.size();
  for (int32_t k = 0; k < pod.sel_count; k++) ex.push_back(ps->exprs[pod.sel_first + k]);
  pod.sel_first = sel0;
  auto copy_terms = [&](int32_t& first, int32_t count) {
    int32_t t0 = (int32_t)tm.size();
    for (int32_t t = 0; t < count; t++) {
      ksim_term x = ps->terms[first + t];
      int32_t e0 = (int32_t)ex.size();
      for (int32_t k = 0; k < x.n_expr; k++) ex.push_back(ps->exprs[x.first_expr + k]);
      x.first_expr = e0;
      tm.push_back(x);
    }
    first = t0;
  };
  copy_terms(pod.req_term_first, pod.req_term_count);
  copy_terms(pod.pref_term_first, pod.pref_term_count);
  copy_terms(pod.added_term_first, pod.added_term_count);
  copy_terms(pod.vb_first, pod.vb_count);
  copy_terms(pod.vz_first, pod.vz_count);
}

static int arena_reserve(ksim_handle* h, DevArena& a, size_t bytes) {
  if (bytes <= a.cap) return KSIM_OK;
  if (a.p) (void)hipFree(a.p);
  a.p = nullptr;
  a.cap = 0;
  const size_t cap = std::max<size_t>(bytes * 2, 1 << 16);
  const hipError_t e = hipMalloc(&a.p, cap);
  if (e != hipSuccess) return hip_fail(h, e, "hipMalloc (arena)");
  a.cap = cap;
  return KSIM_OK;
}

// The handle's pinned staging (the stream must be idle: a copy from it may be
// in flight otherwise).
static int pin_reserve(ksim_handle* h, size_t bytes) {
  if (bytes <= h->pin_cap) return KSIM_OK;
  if (h->pin) (void)hipHostFree(h->pin);
  h->pin = h->pin_d = nullptr;
  h->pin_cap = 0;
  const size_t cap = std::max<size_t>(bytes * 2, 1 << 16);
  hipError_t e = hipHostMalloc(&h->pin, cap, hipHostMallocCoherent | hipHostMallocMapped);
  if (e != hipSuccess) return hip_fail(h, e, "hipHostMalloc (staging)");
  if ((e = hipHostGetDevicePointer(&h->pin_d, h->pin, 0)) != hipSuccess) return hip_fail(h, e, "hipHostGetDevicePointer");
  h->pin_cap = cap;
  return KSIM_OK;
}

// Copies to / from the pinned staging by one kernel (launch_copy_list).
struct Copies {
  CopyList l{};
  int n = 0;
  Copies() { l.anode = -1; }
  void add(const void* src, void* dst, size_t bytes) {
    if (!bytes) return;
    l.src[n] = (const uint8_t*)src;
    l.dst[n] = (uint8_t*)dst;
    l.n[n] = (uint32_t)bytes;
    n++;
  }
  // a framework-driven filter pass's start in the same launch (launch_fw_begin)
  void begin(DevState* st, WinState* win, int32_t first, int32_t end) {
    l.bst = st;
    l.bwin = win;
    l.bfirst = first;
    l.bend = end;
  }
  // a queued bind in the same launch
  void bind(const DevCluster& c, const DevPods& P, int32_t node, int sign) {
    l.ac = c;
    l.aP = P;
    l.anode = node;
    l.asign = sign;
  }
  int run(ksim_handle* h) {
    if (n || l.bst || l.anode >= 0) launch_copy_list(l, n, h->stream);
    HIPCHK(h, hipGetLastError());
    return KSIM_OK;
  }
};

// The results' pinned staging (callers sync before reading it).
static int pout_reserve(ksim_handle* h, size_t bytes) {
  if (bytes <= h->pout_cap) return KSIM_OK;
  HIPCHK(h, hipStreamSynchronize(h->stream));
  if (h->pout) (void)hipHostFree(h->pout);
  h->pout = h->pout_d = nullptr;
  h->pout_cap = 0;
  const size_t cap = std::max<size_t>(bytes * 2, 1 << 16);
  hipError_t e = hipHostMalloc(&h->pout, cap, hipHostMallocCoherent | hipHostMallocMapped);
  if (e != hipSuccess) return hip_fail(h, e, "hipHostMalloc (results)");
  if ((e = hipHostGetDevicePointer(&h->pout_d, h->pout, 0)) != hipSuccess) return hip_fail(h, e, "hipHostGetDevicePointer");
  h->pout_cap = cap;
  return KSIM_OK;
}

static void build_pod_blob(ksim_handle* h, const ksim_pod_set* ps, int32_t pod_index, PodBlob& b) {
  ksim_pod pod;
  std::vector<ksim_label_expr>& ex = h->bs_ex;
  std::vector<ksim_term>& tm = h->bs_tm;
  std::vector<ksim_topo_use>& us = h->bs_us;
  std::vector<ksim_class_add>& ad = h->bs_ad;
  std::vector<int32_t>& nn = h->bs_nn;
  ex.clear();                              // single_pod_set appends
  tm.clear();
  nn.clear();
  single_pod_set(ps, pod_index, pod, ex, tm, us, ad, nn);
  mark_unique(h, us.data(), us.size());
  int32_t bflag[4] = {0, 0, 0, 0};
  for (const auto& u : us)
    if (use_registers_values(u)) bflag[0] |= kPodRegistersValues;
  const PodPlan plan = make_plan(h, pod, us.data());
  struct Piece {
    const void* src;
    size_t bytes;
  };
  const Piece pc[8] = {{&pod, sizeof(pod)},
                       {ex.data(), ex.size() * sizeof(ksim_label_expr)},
                       {tm.data(), tm.size() * sizeof(ksim_term)},
                       {nn.data(), 4 * nn.size()},
                       {bflag, sizeof(bflag)},
                       {&plan, sizeof(plan)},
                       {us.data(), us.size() * sizeof(ksim_topo_use)},
                       {ad.data(), ad.size() * sizeof(ksim_class_add)}};
  size_t total = 0;
  for (int q = 0; q < 8; q++) {
    b.off[q] = total;
    total += (std::max<size_t>(pc[q].bytes, 16) + 63) & ~(size_t)63;
  }
  b.bytes.assign(total, 0);                // zero padding: blobs of one pod compare equal (capacity reused)
  for (int q = 0; q < 8; q++)
    if (pc[q].bytes) std::memcpy(b.bytes.data() + b.off[q], pc[q].src, pc[q].bytes);
  b.n_nn = (int32_t)nn.size();
  b.n_exprs = (int32_t)ex.size();
  b.n_terms = (int32_t)tm.size();
  b.n_uses = (int32_t)us.size();
  b.n_adds = (int32_t)ad.size();
}

// The device pod set of a blob uploaded at d.
static DevPods blob_pods(const ksim_handle* h, const PodBlob& b, char* d) {
  DevPods P{};
  P.pods = (const ksim_pod*)(d + b.off[0]);
  P.exprs = (const ksim_label_expr*)(d + b.off[1]);
  P.terms = (const ksim_term*)(d + b.off[2]);
  P.nn = (const int32_t*)(d + b.off[3]);
  P.n_nn = b.n_nn;
  P.bflags = (const int32_t*)(d + b.off[4]);
  P.plans = (const PodPlan*)(d + b.off[5]);
  P.uses = (const ksim_topo_use*)(d + b.off[6]);
  P.adds = (const ksim_class_add*)(d + b.off[7]);
  P.n_pods = 1;
  P.n_exprs = b.n_exprs;
  P.n_terms = b.n_terms;
  // this pod's binds keep the loaded queue's persistent tables (its plan reads
  // none of them: no kPlanPtab on single uploads)
  P.ptab = h->dp.ptab;
  P.ptab_ent = h->dp.ptab_ent;
  P.ptab_cfirst = h->dp.ptab_cfirst;
  P.ptab_cidx = h->dp.ptab_cidx;
  P.n_uses = b.n_uses;
  P.n_adds = b.n_adds;
  return P;
}

// The blob into the pinned staging and, by one copy kernel, into the arena
// (valid until the arena's next upload).  The staging is reused once the last
// upload's copy has run (its event), not after the whole stream drains; a
// growing staging or arena drains the stream first.  begin_win: a
// framework-driven filter pass's start in the same launch.
// The next slot of the upload ring, free (its last copy has run) and at least
// `bytes` large.
static int ring_slot(ksim_handle* h, size_t bytes, ksim_handle::PinSlot** out) {
  ksim_handle::PinSlot& sl = h->ring[h->ring_next];
  h->ring_next = (h->ring_next + 1) % ksim_handle::kPinRing;
  if (sl.pending) HIPCHK(h, hipEventSynchronize(sl.ev));   // this slot's last reader (four uploads ago)
  sl.pending = false;
  if (bytes > sl.cap) {
    if (sl.p) (void)hipHostFree(sl.p);
    sl.p = sl.d = nullptr;
    sl.cap = 0;
    const size_t cap = std::max<size_t>(bytes * 2, 1 << 14);
    hipError_t e = hipHostMalloc(&sl.p, cap, hipHostMallocCoherent | hipHostMallocMapped);
    if (e != hipSuccess) return hip_fail(h, e, "hipHostMalloc (upload ring)");
    if ((e = hipHostGetDevicePointer(&sl.d, sl.p, 0)) != hipSuccess) return hip_fail(h, e, "hipHostGetDevicePointer");
    sl.cap = cap;
  }
  *out = &sl;
  return KSIM_OK;
}

static int upload_blob(ksim_handle* h, const PodBlob& b, DevArena& arena, DevPods& P,
                       WinState* begin_win = nullptr, bool record = false, bool synced = false) {
  const size_t total = b.bytes.size();
  if (h->pend_bind.on && arena.p && (const char*)h->pend_bind.P.pods >= (const char*)arena.p &&
      (const char*)h->pend_bind.P.pods < (const char*)arena.p + arena.cap) {
    // the queued Reserve reads this arena (every caller alternates arenas, so
    // this does not happen today): land it before the arena is grown or overwritten
    h->pend_reuse++;
    if (const int prc = flush_pend_bind(h)) return prc;
  }
  if (total > arena.cap) {
    HIPCHK(h, hipStreamSynchronize(h->stream));   // the arena is reallocated: nothing may read it
    for (auto& r : h->ring) r.pending = false;
  }
  ksim_handle::PinSlot* slp = nullptr;
  int rc;
  if ((rc = ring_slot(h, total, &slp))) return rc;
  ksim_handle::PinSlot& sl = *slp;
  if ((rc = arena_reserve(h, arena, total))) return rc;
  std::memcpy(sl.p, b.bytes.data(), total);
  Copies cp;
  cp.add(sl.d, arena.p, total);
  if (begin_win) cp.begin(h->st, begin_win, 0, 1);
  if (record && h->pend_bind.on) {         // the last cycle's queued Reserve, ahead of this pass
    cp.bind(h->dc, h->pend_bind.P, h->pend_bind.node, h->pend_bind.sign);
    h->pend_bind.on = false;
  }
  if ((rc = cp.run(h))) return rc;
  if (!synced) {                           // synced: the caller drains the stream before returning
    if (!sl.ev) HIPCHK(h, hipEventCreateWithFlags(&sl.ev, hipEventDisableTiming));
    HIPCHK(h, hipEventRecord(sl.ev, h->stream));
    sl.pending = true;
  }
  P = blob_pods(h, b, (char*)arena.p);
  if (record || &arena == &h->pod1_arena) {   // what a Reserve of this pod binds from
    h->pod1_blob = b.bytes;
    h->pod1_base = (char*)arena.p;
  }
  return KSIM_OK;
}

// Upload one pod (re-based) as a device pod set of its own.
static int upload_single(ksim_handle* h, const ksim_pod_set* ps, int32_t pod_index, DevPods& P, DevArena& arena) {
  PodBlob b;
  build_pod_blob(h, ps, pod_index, b);
  return upload_blob(h, b, arena, P);
}

static int upload_single(ksim_handle* h, const ksim_pod_set* ps, int32_t pod_index, DevPods& P) {
  return upload_single(h, ps, pod_index, P, h->pod1_arena);
}

// Copy one compat cycle's per-node outputs and scalars to the caller.
// The device marks a node whose Filter status was an error with kFailError
// next to the plugin index; the ABI reports the plugin index alone (the cycle
// status says the cycle failed).
static void strip_fail_errors(uint8_t* f, size_t n) {
  for (size_t i = 0; i < n; i++)
    if (fail_is_error(f[i])) f[i] &= (uint8_t)~kFailError;
}

static int copy_eval_out(ksim_handle* h, ksim_eval_out* out) {
  const size_t N = (size_t)h->dc.n;
  const int S = h->prof.n_score;
  if (out->fail_plugin) {
    HIPCHK(h, hcopy(h, out->fail_plugin, h->sc.fail, N, hipMemcpyDeviceToHost));
    strip_fail_errors(out->fail_plugin, N);
  }
  if (out->fail_detail) HIPCHK(h, hcopy(h, out->fail_detail, h->sc.detail, 4 * N, hipMemcpyDeviceToHost));
  if (out->scored) HIPCHK(h, hcopy(h, out->scored, h->eo.scored, N, hipMemcpyDeviceToHost));
  if (out->raw && S) HIPCHK(h, hcopy(h, out->raw, h->eo.raw, 8 * N * S, hipMemcpyDeviceToHost));
  if (out->norm && S) HIPCHK(h, hcopy(h, out->norm, h->eo.norm, 8 * N * S, hipMemcpyDeviceToHost));
  if (out->total) HIPCHK(h, hcopy(h, out->total, h->eo.total, 8 * N, hipMemcpyDeviceToHost));
  DevState st;
  HIPCHK(h, hcopy(h, &st, h->st, sizeof(st), hipMemcpyDeviceToHost));
  out->chosen = st.chosen;
  out->status = st.status;
  out->n_feasible = st.n_feasible;
  out->n_evaluated = st.n_evaluated;
  out->n_processed = st.n_processed;
  out->k_to_find = st.k_to_find;
  out->next_start = st.next_start_after;
  if (out->scored && out->n_feasible <= 1) std::memset(out->scored, 0, N);
  return KSIM_OK;
}

int ksim_eval_pod(ksim_handle* h, const ksim_pod_set* ps, int32_t pod_index, ksim_eval_out* out) {
  int rc = ensure_ready(h);
  if (rc) return rc;
  if (!ps || !out || pod_index < 0 || pod_index >= ps->n_pods || !ps->pods)
    return set_err(h, KSIM_E_INVALID, "bad pod set / index");
  if ((rc = validate_pod(h, ps, pod_index))) return rc;
  if (is_sharded(h) && profile_nb(h->prof))
    return set_err(h, KSIM_E_UNSUPPORTED, "NetworkBandwidth profiles run on unsharded handles");
  HIPCHK(h, hipSetDevice(h->device));
  h->ext_pending = false;
  DevPods P;
  if ((rc = upload_single(h, ps, pod_index, P))) return rc;
  if ((rc = set_run(h, 0, 1))) return rc;
  launch_cycle(make_args(h, P, nullptr), h->stream, true, ps->pods[pod_index].use_count > 0);
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return copy_eval_out(h, out);
}

int ksim_eval_pod_filter(ksim_handle* h, const ksim_pod_set* ps, int32_t pod_index, ksim_eval_out* out) {
  int rc = ensure_ready(h);
  if (rc) return rc;
  if (!ps || !out || pod_index < 0 || pod_index >= ps->n_pods || !ps->pods)
    return set_err(h, KSIM_E_INVALID, "bad pod set / index");
  if (is_sharded(h)) return set_err(h, KSIM_E_UNSUPPORTED, "extender cycles run on unsharded handles");
  if ((rc = validate_pod(h, ps, pod_index))) return rc;
  HIPCHK(h, hipSetDevice(h->device));
  if ((rc = upload_single(h, ps, pod_index, h->pod1))) return rc;
  if ((rc = set_run(h, 0, 1))) return rc;
  launch_cycle_filter(make_args(h, h->pod1, nullptr), h->stream, ps->pods[pod_index].use_count > 0);
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipStreamSynchronize(h->stream));
  const size_t N = (size_t)h->dc.n;
  if (out->fail_plugin) {
    HIPCHK(h, hcopy(h, out->fail_plugin, h->sc.fail, N, hipMemcpyDeviceToHost));
    strip_fail_errors(out->fail_plugin, N);
  }
  if (out->fail_detail) HIPCHK(h, hcopy(h, out->fail_detail, h->sc.detail, 4 * N, hipMemcpyDeviceToHost));
  WinState w;
  DevState st;
  HIPCHK(h, hcopy(h, &w, h->sc.win, sizeof(w), hipMemcpyDeviceToHost));
  HIPCHK(h, hcopy(h, &st, h->st, sizeof(st), hipMemcpyDeviceToHost));
  const int32_t ns = w.nscan;                      // nodes scanned (PreFilterResult: its node count)
  const int32_t processed = w.cut < ns ? w.cut : ns;
  out->chosen = w.error ? KSIM_CHOSEN_ERROR : -1;
  out->status = w.error ? KSIM_STATUS_ERROR : 0;
  out->n_feasible = w.nf;
  out->n_evaluated = w.evaluated;
  out->n_processed = processed;
  out->k_to_find = w.k;
  out->next_start = ns > 0 ? (int32_t)(((int64_t)st.next_start + processed) % ns) : st.next_start;
  h->ext_pending = true;
  return KSIM_OK;
}

int ksim_eval_pod_finish(ksim_handle* h, const uint8_t* ext_fail, const int64_t* ext_score, ksim_eval_out* out) {
  int rc = ensure_ready(h);
  if (rc) return rc;
  if (!out) return set_err(h, KSIM_E_INVALID, "out is null");
  if (!h->ext_pending) return set_err(h, KSIM_E_INVALID, "ksim_eval_pod_finish without ksim_eval_pod_filter");
  h->ext_pending = false;
  HIPCHK(h, hipSetDevice(h->device));
  const size_t N = (size_t)h->dc.n;
  if (ext_fail)
    HIPCHK(h, hipMemcpyAsync(h->ext_fail, ext_fail, N, hipMemcpyHostToDevice, h->stream));
  else
    HIPCHK(h, hipMemsetAsync(h->ext_fail, 0, N, h->stream));
  if (ext_score)
    HIPCHK(h, hipMemcpyAsync(h->ext_score, ext_score, 8 * N, hipMemcpyHostToDevice, h->stream));
  else
    HIPCHK(h, hipMemsetAsync(h->ext_score, 0, 8 * N, h->stream));
  LaunchArgs a = make_args(h, h->pod1, nullptr);
  a.s.ext_fail = h->ext_fail;
  a.s.ext_score = h->ext_score;
  launch_cycle_finish(a, h->stream);
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return copy_eval_out(h, out);
}

// ---- framework-driven compat mode (SURVEY §8(b) compat mode) -------------------
// The simulator runs upstream's framework with parallelism 16 and
// percentageOfNodesToScore 0 (simulator/scheduler/scheduler.go:149,153,231-241):
// the framework, not the engine, decides which nodes Filter runs on, the list
// PreScore / Score / NormalizeScore see and the node Reserve records
// (wrappedplugin.go:356-375, 491-516, 583-584).  These entry points answer the
// engine-backed plugins under those choices.
int ksim_fw_prefilter(ksim_handle* h, const ksim_pod_set* ps, int32_t pod_index, ksim_eval_out* out) {
  // a queued Reserve of the last cycle runs inside this pass's upload launch;
  // with Unreserves queued behind it (deferred_binds) it is launched first
  if (h && h->pend_bind.on && !h->deferred_binds.empty()) {
    const int prc = flush_pend_bind(h);
    if (prc) return prc;
  }
  int rc = ensure_ready(h, false, true);   // abandons any framework cycle in flight
  if (rc) return rc;
  if (!ps || !out || pod_index < 0 || pod_index >= ps->n_pods || !ps->pods)
    return set_err(h, KSIM_E_INVALID, "bad pod set / index");
  if (is_sharded(h)) return set_err(h, KSIM_E_UNSUPPORTED, "framework-driven cycles run on unsharded handles");
  if ((rc = validate_pod(h, ps, pod_index))) return rc;
  HIPCHK(h, hipSetDevice(h->device));
  h->ext_pending = false;
  h->fw_list.clear();                // a new cycle: no normalization answered from the last one
  h->fw_raw.clear();
  const ksim_pod& p = ps->pods[pod_index];
  const size_t N = (size_t)h->dc.n;
  const int S = h->prof.n_score;
  // Score on the host (ksim_fw_score) unless a PreScore reads the framework's
  // list: PodTopologySpread's ScheduleAnyway constraints (IgnoredNodes, pair
  // counts over the list); NetworkBandwidth's Score may fail the cycle
  bool host = S > 0 && !profile_nb(h->prof) && !(p.flags & KSIM_POD_NODE_NAMES_UNKNOWN);
  for (int32_t u = 0; host && u < p.use_count; u++)
    if (ps->uses[p.use_first + u].kind == KSIM_USE_PTS_SOFT) host = false;
  h->fw_host = host;
  // a pod without topology uses: the filter kernel writes its answers straight
  // to the pinned staging (fwh), no copy launch; with uses, the topology flags
  // are the PreFilter pass's, copied after it
  const bool mirror = p.use_count == 0;
  // fwh: [head 64][fail N][detail 4N][raw S x N][part N], 64-byte aligned pieces
  const size_t o_fail = 64, o_det = o_fail + ((N + 63) & ~(size_t)63),
               o_raw = o_det + ((4 * N + 63) & ~(size_t)63), o_part = o_raw + ((8 * (size_t)S * N + 63) & ~(size_t)63),
               need = o_part + 8 * N;
  if (need > h->fwh_cap) {
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (h->fwh) (void)hipHostFree(h->fwh);
    h->fwh = h->fwh_d = nullptr;
    h->fwh_cap = 0;
    hipError_t e = hipHostMalloc(&h->fwh, need, hipHostMallocCoherent | hipHostMallocMapped);
    if (e != hipSuccess) return hip_fail(h, e, "hipHostMalloc (fw answers)");
    if ((e = hipHostGetDevicePointer(&h->fwh_d, h->fwh, 0)) != hipSuccess)
      return hip_fail(h, e, "hipHostGetDevicePointer");
    h->fwh_cap = need;
  }
  char* fo = (char*)h->fwh;
  char* fd = (char*)h->fwh_d;
  // the pod, and the run header / window state / topology flags reset, in one
  // launch (upload_blob's begin job)
  build_pod_blob(h, ps, pod_index, h->fw_blob);
  h->fw_flip ^= 1;
  if ((rc = upload_blob(h, h->fw_blob, h->fw_arena[h->fw_flip], h->pod1, h->sc.win, true, true))) return rc;
  LaunchArgs a = make_args(h, h->pod1, nullptr);
  if (mirror) {
    a.s.m_head = (int32_t*)fd;
    a.s.m_fail = (uint8_t*)(fd + o_fail);
    a.s.m_detail = out->fail_detail ? (uint32_t*)(fd + o_det) : nullptr;
    a.s.m_raw = host ? (int32_t*)(fd + o_raw) : nullptr;
    reinterpret_cast<int32_t*>(fo)[1] = 0;        // the kernel's too-wide flag
  }
  launch_fw_filter(a, h->stream, p.use_count > 0);
  HIPCHK(h, hipGetLastError());
  h->fw_dom_dirty = p.use_count > 0;
  h->fw_topo = p.use_count > 0;
  h->fw_fail.resize(N);
  if (!mirror) {
    // the results into the same staging, one copy launch: next_start, the
    // topology flags, the filter codes, the details (and the raw scores)
    Copies cp;
    cp.add(&h->st->next_start, fd, sizeof(int32_t));
    cp.add(&h->st->topo_flags, fd + 4, sizeof(uint32_t));
    cp.add(h->sc.fail, fd + o_fail, N);
    if (out->fail_detail) cp.add(h->sc.detail, fd + o_det, 4 * N);
    if (host) {
      cp.add(h->sc.raw, fd + o_raw, 8 * (size_t)S * N);
      cp.add(h->sc.part, fd + o_part, 8 * N);
    }
    if ((rc = cp.run(h))) return rc;
  }
  HIPCHK(h, hipStreamSynchronize(h->stream));
  std::memcpy(h->fw_fail.data(), fo + o_fail, N);
  if (out->fail_detail) std::memcpy(out->fail_detail, fo + o_det, 4 * N);
  int32_t ns = h->dc.n;
  if (p.flags & KSIM_POD_NODE_NAMES) ns = (p.flags & KSIM_POD_NODE_NAMES_UNKNOWN) ? 0 : p.nn_count;
  int32_t nf = 0;
  for (size_t i = 0; i < N; i++) nf += h->fw_fail[i] == KSIM_PASSED;
  if (out->fail_plugin) {
    std::memcpy(out->fail_plugin, h->fw_fail.data(), N);
    strip_fail_errors(out->fail_plugin, N);
  }
  int32_t next = 0;
  std::memcpy(&next, fo, sizeof(next));
  h->fw_tflags = 0;
  if (!mirror) std::memcpy(&h->fw_tflags, fo + 4, sizeof(uint32_t));
  h->fw_oraw = o_raw;
  h->fw_opart = o_part;
  h->fw_raw32 = mirror;
  if (mirror && host && reinterpret_cast<const int32_t*>(fo)[1] != 0)
    h->fw_host = false;                  // a raw score past int32: ksim_fw_score on the device
  const bool unknown = (p.flags & KSIM_POD_NODE_NAMES_UNKNOWN) != 0;
  out->chosen = unknown ? KSIM_CHOSEN_ERROR : -1;
  out->status = unknown ? KSIM_STATUS_ERROR : 0;
  out->n_feasible = nf;
  out->n_evaluated = ns;
  out->n_processed = 0;
  out->k_to_find = num_feasible_nodes_to_find(h->prof.percentage_of_nodes_to_score, ns);
  out->next_start = next;
  h->fw_ns = ns;
  h->fw_pending = !unknown;
  return KSIM_OK;
}

// The cycle's filter pass again, on the current dynamic state: the PreFilter
// domain sums start from zero, the topology flags too (ksim_fw_prefilter).
static int fw_filter_pass(ksim_handle* h) {
  if (h->fw_topo && h->sc.dom)
    HIPCHK(h, hipMemsetAsync(h->sc.dom, 0, 8 * (size_t)KSIM_MAX_USES * h->dc.vmax, h->stream));
  launch_fw_begin(h->st, h->sc.win, 0, 1, h->stream);
  launch_fw_filter(make_args(h, h->pod1, nullptr), h->stream, h->fw_topo);
  HIPCHK(h, hipGetLastError());
  return KSIM_OK;
}

// RunFilterPluginsWithNominatedPods' first pass: for each listed node, the
// cycle's pod against that node with its nominated pods added (addNominatedPods:
// NodeInfo.AddPodInfo and the PreFilterExtensions' AddPod of PodTopologySpread
// and InterPodAffinity, which for +1 updates equal a PreFilter over the state
// with the pods bound there).  Each node's pods are assumed, the filter pass
// re-run, the node's verdict read, the pods forgotten; a last pass restores the
// cycle's own PreFilter state for ksim_fw_score.
int ksim_fw_filter_nominated(ksim_handle* h, const ksim_pod_set* nps, int32_t n_nodes, const int32_t* nodes,
                             const int32_t* first, const int32_t* count, uint8_t* fail_plugin,
                             uint32_t* fail_detail) {
  int rc = ensure_ready(h, true);
  if (rc) return rc;
  if (!h->fw_pending) return set_err(h, KSIM_E_INVALID, "ksim_fw_filter_nominated without ksim_fw_prefilter");
  if (n_nodes < 0 || (n_nodes > 0 && (!nodes || !first || !count || !nps || !nps->pods || !fail_plugin)))
    return set_err(h, KSIM_E_INVALID, "bad nominated-node groups");
  for (int32_t k = 0; k < n_nodes; k++) {
    if (nodes[k] < 0 || nodes[k] >= h->dc.n) return set_err(h, KSIM_E_INVALID, "nominated node out of range");
    if (count[k] < 0 || first[k] < 0 || first[k] + count[k] > nps->n_pods)
      return set_err(h, KSIM_E_INVALID, "nominated pod range out of the pod set");
    for (int32_t j = first[k]; j < first[k] + count[k]; j++)
      if ((rc = validate_pod(h, nps, j))) return rc;
  }
  if (n_nodes == 0) return KSIM_OK;
  HIPCHK(h, hipSetDevice(h->device));
  auto bind_all = [&](int32_t k, int sign) -> int {
    for (int32_t j = first[k]; j < first[k] + count[k]; j++) {
      DevPods P;
      int r;
      if ((r = upload_single(h, nps, j, P, h->nom_arena))) return r;
      launch_assume(h->dc, P, 0, nodes[k], sign, h->stream);
      HIPCHK(h, hipGetLastError());
    }
    return KSIM_OK;
  };
  for (int32_t k = 0; k < n_nodes; k++) {
    if ((rc = bind_all(k, 1))) return rc;
    if ((rc = fw_filter_pass(h))) return rc;
    uint8_t f = 0;
    uint32_t d = 0;
    HIPCHK(h, hcopy(h, &f, h->sc.fail + nodes[k], 1, hipMemcpyDeviceToHost));
    HIPCHK(h, hcopy(h, &d, h->sc.detail + nodes[k], 4, hipMemcpyDeviceToHost));
    if (fail_is_error(f)) f &= (uint8_t)~kFailError;
    fail_plugin[k] = f;
    if (fail_detail) fail_detail[k] = d;
    if ((rc = bind_all(k, -1))) return rc;
  }
  if ((rc = fw_filter_pass(h))) return rc;                 // the cycle's own PreFilter state again
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return KSIM_OK;
}

// NormalizeScore of one value on the host (ksim_device.h normalize_value, the
// same integer and float64 expressions; -ffp-contract=off holds for this file)
static int64_t host_normalize(int32_t kind, int64_t v, int64_t gmax, int64_t gmin, bool ipa_nonempty) {
  switch (kind) {
    case kNormDefault: {
      const int64_t m = gmax > 0 ? gmax : 0;
      return m == 0 ? v : (int64_t)((uint64_t)kMaxNodeScore * (uint64_t)v) / m;
    }
    case kNormDefaultReverse: {
      const int64_t m = gmax > 0 ? gmax : 0;
      return m == 0 ? (int64_t)kMaxNodeScore : (int64_t)kMaxNodeScore - (int64_t)((uint64_t)kMaxNodeScore * (uint64_t)v) / m;
    }
    case kNormPTS: {
      const int64_t mx = gmax > 0 ? gmax : 0;
      return mx == 0 ? (int64_t)kMaxNodeScore : (int64_t)((uint64_t)kMaxNodeScore * (uint64_t)(mx + gmin - v)) / mx;
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

// ksim_fw_score answered on the host (fw_host): PreScore / Score were the
// filter pass's (no list-dependent PreScore), NormalizeScore, the weights and
// the totals over the framework's list, as k_window / k_extrema / k_select
// compute them (k_select: one listed node is not scored).
static int fw_score_host(ksim_handle* h, const int32_t* nodes, int32_t n, ksim_eval_out* out) {
  const size_t N = (size_t)h->dc.n;
  const int S = h->prof.n_score;
  std::vector<uint8_t>& seen = h->fw_seen;
  if (seen.size() != N) seen.assign(N, 0);
  for (int32_t j = 0; j < n; j++) {
    const int32_t x = nodes[j];
    if (x < 0 || (size_t)x >= N || h->fw_fail[x] != KSIM_PASSED || seen[x]) {
      for (int32_t q = 0; q < j; q++) seen[nodes[q]] = 0;
      return set_err(h, KSIM_E_INVALID, "node list: not a feasible node of the filter pass, or repeated");
    }
    seen[x] = 1;
  }
  for (int32_t j = 0; j < n; j++) seen[nodes[j]] = 0;
  // the filter pass's answers: node-major int32 rows [n][S + 1] (the kernel's
  // own copy), or slot-major int64 [S][n] and [n] (a copy launch)
  const char* rawb = (const char*)h->fwh + h->fw_oraw;
  const char* partb = (const char*)h->fwh + h->fw_opart;
  const bool w32 = h->fw_raw32;
  const size_t W = (size_t)S + 1;
  auto raw_at = [&](int k, size_t node) -> int64_t {
    return w32 ? (int64_t)reinterpret_cast<const int32_t*>(rawb)[node * W + (size_t)k]
               : reinterpret_cast<const int64_t*>(rawb)[(size_t)k * N + node];
  };
  auto part_at = [&](size_t node) -> int64_t {
    return w32 ? (int64_t)reinterpret_cast<const int32_t*>(rawb)[node * W + (size_t)S]
               : reinterpret_cast<const int64_t*>(partb)[node];
  };
  const bool scored = n > 1;
  const bool ipa_nonempty = (h->fw_tflags & kTopoScoreNonEmpty) != 0;
  h->fw_list.assign(nodes, nodes + n);
  h->fw_raw.assign((size_t)S * n, 0);
  h->fw_norm.assign((size_t)S * n, 0);
  std::vector<int64_t>& tot = h->fw_tot;
  tot.assign(n, 0);
  if (scored) {
    if (w32) {                             // one row (a cache line) per listed node
      const int32_t* rows = reinterpret_cast<const int32_t*>(rawb);
      int64_t* fr = h->fw_raw.data();
      for (int32_t j = 0; j < n; j++) {
        const int32_t* row = rows + (size_t)nodes[j] * W;
        for (int k = 0; k < S; k++) fr[(size_t)k * n + j] = row[k];
        tot[j] = row[S];
      }
    } else {
      for (int32_t j = 0; j < n; j++) tot[j] = part_at((size_t)nodes[j]);
      for (int k = 0; k < S; k++)
        for (int32_t j = 0; j < n; j++) h->fw_raw[(size_t)k * n + j] = raw_at(k, (size_t)nodes[j]);
    }
    for (int k = 0; k < S; k++) {
      int64_t* r = h->fw_raw.data() + (size_t)k * n;
      int64_t* nv = h->fw_norm.data() + (size_t)k * n;
      const int32_t kind = norm_kind(h->prof.score[k]);
      if (kind == kNormNone) {
        std::memcpy(nv, r, 8 * (size_t)n);
        continue;
      }
      int64_t gmax = INT64_MIN, gmin = INT64_MAX;
      for (int32_t j = 0; j < n; j++) {
        gmax = std::max(gmax, r[j]);
        gmin = std::min(gmin, r[j]);
      }
      const int64_t w = h->prof.score_weight[k] == 0 ? 1 : h->prof.score_weight[k];
      // a list's raw scores take few distinct values: each value's normalized
      // score once (a 64-entry direct-mapped memo), not a division per node
      int64_t mk[64], mv[64];
      bool mset[64] = {};
      for (int32_t j = 0; j < n; j++) {
        const int64_t v = r[j];
        const uint32_t e = (uint32_t)((uint64_t)v * 0x9E3779B97F4A7C15ull >> 58);
        if (!mset[e] || mk[e] != v) {
          mset[e] = true;
          mk[e] = v;
          mv[e] = host_normalize(kind, v, gmax, gmin, ipa_nonempty);
        }
        nv[j] = mv[e];
        tot[j] += mv[e] * w;
      }
    }
  }
  if (out->scored)
    for (int32_t j = 0; j < n; j++) out->scored[nodes[j]] = scored ? 1 : 0;
  for (int k = 0; k < S; k++) {
    if (out->raw) {
      int64_t* r = out->raw + (size_t)k * N;
      for (int32_t j = 0; j < n; j++) r[nodes[j]] = h->fw_raw[(size_t)k * n + j];
    }
    if (out->norm) {
      int64_t* r = out->norm + (size_t)k * N;
      for (int32_t j = 0; j < n; j++) r[nodes[j]] = h->fw_norm[(size_t)k * n + j];
    }
  }
  if (out->total)
    for (int32_t j = 0; j < n; j++) out->total[nodes[j]] = tot[j];
  if (out->fail_plugin) {                  // the filter pass, unchanged
    std::memcpy(out->fail_plugin, h->fw_fail.data(), N);
    strip_fail_errors(out->fail_plugin, N);
  }
  out->n_feasible = n;
  out->n_evaluated = h->fw_ns;
  out->n_processed = 0;
  out->k_to_find = num_feasible_nodes_to_find(h->prof.percentage_of_nodes_to_score, h->fw_ns);
  out->chosen = -1;
  out->status = 0;
  h->fw_pending = false;                   // the domain sums stay for fw_abandon (no k_select ran)
  h->fw_scored = true;
  return KSIM_OK;
}

int ksim_fw_score(ksim_handle* h, const int32_t* nodes, int32_t n, ksim_eval_out* out) {
  int rc = ensure_ready(h, true);
  if (rc) return rc;
  if (!out || n < 0 || (n > 0 && !nodes)) return set_err(h, KSIM_E_INVALID, "bad node list");
  if (!h->fw_pending) return set_err(h, KSIM_E_INVALID, "ksim_fw_score without ksim_fw_prefilter");
  h->fw_counts[h->fw_host ? 0 : 1]++;
  if (h->fw_host) return fw_score_host(h, nodes, n, out);
  const size_t N = (size_t)h->dc.n;
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(h->stream));    // the upload staging is free again
  const size_t o_list = (64 + N + 63) & ~(size_t)63;
  if ((rc = pin_reserve(h, o_list + 4 * (size_t)n))) return rc;
  // the list: feasible nodes of the filter pass, each once (the mask in staging)
  uint8_t* out_of_list = (uint8_t*)h->pin + 64;
  std::memset(out_of_list, 1, N);
  for (int32_t j = 0; j < n; j++) {
    const int32_t x = nodes[j];
    if (x < 0 || (size_t)x >= N || h->fw_fail[x] != KSIM_PASSED || !out_of_list[x])
      return set_err(h, KSIM_E_INVALID, "node list: not a feasible node of the filter pass, or repeated");
    out_of_list[x] = 0;
  }
  std::memcpy((char*)h->pin + o_list, nodes, 4 * (size_t)n);
  // the window of the filter pass covers the whole scan set (k_window's
  // extender branch keeps it and drops the unlisted nodes)
  std::memcpy(h->pin, &h->fw_ns, sizeof(int32_t));
  {
    Copies cp;
    cp.add((char*)h->pin_d + 64, h->ext_fail, N);
    cp.add(h->pin_d, &h->sc.win->cut, sizeof(int32_t));
    cp.add((char*)h->pin_d + o_list, h->fw_nodes, 4 * (size_t)n);
    if ((rc = cp.run(h))) return rc;
  }
  LaunchArgs a = make_args(h, h->pod1, nullptr);
  a.s.ext_fail = h->ext_fail;
  a.s.ext_score = nullptr;
  launch_fw_score(a, h->stream);
  const int S = h->prof.n_score;
  // the listed nodes' answers and the window state gathered straight into
  // the pinned staging, one synchronization; the caller's entries of
  // unlisted nodes are left as they are (ksim_engine.h)
  const size_t o_comp = (sizeof(WinState) + 63) & ~(size_t)63, nb = (16 * (size_t)S + 9) * n;
  if ((rc = pout_reserve(h, o_comp + nb))) return rc;
  char* po = (char*)h->pout;
  launch_fw_gather(h->eo, h->fw_nodes, n, (int32_t)N, S, (int64_t*)((char*)h->pout_d + o_comp), h->sc.win,
                   h->pout_d, h->stream);
  HIPCHK(h, hipGetLastError());
  h->fw_pending = false;
  h->fw_dom_dirty = false;                 // k_select re-zeroed the domain sums
  h->fw_scored = true;
  HIPCHK(h, hipStreamSynchronize(h->stream));
  const int64_t* craw = (const int64_t*)(po + o_comp);
  const int64_t* cnorm = craw + (size_t)S * n;
  const int64_t* ctot = cnorm + (size_t)S * n;
  const uint8_t* csc = (const uint8_t*)(ctot + n);
  if (out->scored)
    for (int32_t j = 0; j < n; j++) out->scored[nodes[j]] = csc[j];
  for (int k = 0; k < S; k++) {
    if (out->raw) {
      int64_t* r = out->raw + (size_t)k * N;
      for (int32_t j = 0; j < n; j++) r[nodes[j]] = craw[(size_t)k * n + j];
    }
    if (out->norm) {
      int64_t* r = out->norm + (size_t)k * N;
      for (int32_t j = 0; j < n; j++) r[nodes[j]] = cnorm[(size_t)k * n + j];
    }
  }
  if (out->total)
    for (int32_t j = 0; j < n; j++) out->total[nodes[j]] = ctot[j];
  // kept for ksim_fw_normalize over the same list
  h->fw_list.assign(nodes, nodes + n);
  h->fw_raw.assign(craw, craw + (size_t)S * n);
  h->fw_norm.assign(cnorm, cnorm + (size_t)S * n);
  WinState w;
  std::memcpy(&w, po, sizeof(w));
  if (out->fail_plugin) {                  // the filter pass, unchanged
    std::memcpy(out->fail_plugin, h->fw_fail.data(), N);
    strip_fail_errors(out->fail_plugin, N);
  }
  out->n_feasible = w.nf;
  out->n_evaluated = h->fw_ns;
  out->n_processed = 0;
  out->k_to_find = num_feasible_nodes_to_find(h->prof.percentage_of_nodes_to_score, h->fw_ns);
  out->chosen = w.error ? KSIM_CHOSEN_ERROR : -1;
  out->status = w.error ? KSIM_STATUS_ERROR : 0;
  if (out->scored && w.nf <= 1)
    for (int32_t j = 0; j < n; j++) out->scored[nodes[j]] = 0;
  return KSIM_OK;
}

int ksim_fw_normalize(ksim_handle* h, int32_t score_slot, const int32_t* nodes, const int64_t* scores, int32_t n,
                      int64_t* out) {
  int rc = ensure_ready(h, true);
  if (rc) return rc;
  if (!h->fw_scored) return set_err(h, KSIM_E_INVALID, "ksim_fw_normalize without ksim_fw_score");
  if (score_slot < 0 || score_slot >= h->prof.n_score) return set_err(h, KSIM_E_INVALID, "bad score slot");
  const size_t N = (size_t)h->dc.n;
  if (n < 0 || (size_t)n > N || (n > 0 && (!nodes || !scores || !out)))
    return set_err(h, KSIM_E_INVALID, "bad score list");
  for (int32_t j = 0; j < n; j++)
    if (nodes[j] < 0 || (size_t)nodes[j] >= N) return set_err(h, KSIM_E_INVALID, "bad node in score list");
  if (n == 0) return KSIM_OK;
  // the framework's NormalizeScore hands over exactly ksim_fw_score's list
  // and the raw scores it returned: that normalization is already computed
  if ((size_t)n == h->fw_list.size() && h->fw_raw.size() == (size_t)h->prof.n_score * n) {
    const int64_t* raw = h->fw_raw.data() + (size_t)score_slot * n;
    bool same = std::equal(nodes, nodes + n, h->fw_list.begin());
    for (int32_t j = 0; same && j < n; j++) same = scores[j] == raw[j];
    if (same) {
      h->fw_counts[2]++;
      std::memcpy(out, h->fw_norm.data() + (size_t)score_slot * n, 8 * (size_t)n);
      return KSIM_OK;
    }
  }
  h->fw_counts[3]++;
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(h->stream));    // the staging is free again
  const size_t o_vals = (4 * (size_t)n + 63) & ~(size_t)63;
  if ((rc = pin_reserve(h, o_vals + 8 * (size_t)n)) || (rc = pout_reserve(h, 8 * (size_t)n))) return rc;
  std::memcpy(h->pin, nodes, 4 * (size_t)n);
  std::memcpy((char*)h->pin + o_vals, scores, 8 * (size_t)n);
  {
    Copies cp;
    cp.add(h->pin_d, h->fw_nodes, 4 * (size_t)n);
    cp.add((char*)h->pin_d + o_vals, h->fw_vals, 8 * (size_t)n);
    if ((rc = cp.run(h))) return rc;
  }
  launch_fw_normalize(make_args(h, h->pod1, nullptr), score_slot, h->fw_nodes, h->fw_vals, n, h->fw_out, h->stream);
  HIPCHK(h, hipGetLastError());
  {
    Copies cp;
    cp.add(h->fw_out, h->pout_d, 8 * (size_t)n);
    if ((rc = cp.run(h))) return rc;
  }
  HIPCHK(h, hipStreamSynchronize(h->stream));
  std::memcpy(out, h->pout, 8 * (size_t)n);
  return KSIM_OK;
}

// Reserve / Unreserve (wrappedplugin.go:583-584, 617), uploaded through their
// own arena (never the cycle's pod).  Unreserve never abandons a framework
// cycle in flight: between that cycle's PreFilter and Score it is queued and
// applied once the cycle has scored (ensure_ready), as upstream's cycle keeps
// the snapshot it started from while the cache takes the binding goroutine's
// ForgetPod.  Reserve is the end of a cycle (after Score, or with one
// feasible node, which the framework does not score): it closes the cycle,
// applies what was queued, then assumes.
static int apply_bind(ksim_handle* h, const ksim_pod_set* ps, int32_t pod_index, int32_t node, int sign) {
  DevPods P;
  int rc;
  if ((rc = flush_pend_bind(h))) return rc;
  PodBlob b;
  build_pod_blob(h, ps, pod_index, b);
  if (h->pod1_base && b.bytes == h->pod1_blob) {
    // the pod the last filter pass uploaded (the framework's Reserve of the
    // cycle's pod): bind from its arena copy, queued (pend_bind) until the
    // next call: the next framework-driven pass runs it inside its upload
    // launch (into the other arena), any other call launches it first
    h->pend_bind.P = blob_pods(h, b, h->pod1_base);
    h->pend_bind.node = node;
    h->pend_bind.sign = sign;
    h->pend_bind.on = true;
    return KSIM_OK;
  }
  // another pod's Reserve / Unreserve (an informer's pod delta, a forget): the
  // bind reads the pod straight from a pinned ring slot (mapped host memory):
  // one launch, no arena copy
  ksim_handle::PinSlot* sl = nullptr;
  if ((rc = ring_slot(h, b.bytes.size(), &sl))) return rc;
  std::memcpy(sl->p, b.bytes.data(), b.bytes.size());
  P = blob_pods(h, b, (char*)sl->d);
  launch_assume(h->dc, P, 0, node, sign, h->stream);
  HIPCHK(h, hipGetLastError());
  if (!sl->ev) HIPCHK(h, hipEventCreateWithFlags(&sl->ev, hipEventDisableTiming));
  HIPCHK(h, hipEventRecord(sl->ev, h->stream));
  sl->pending = true;
  // no synchronization: every later call is ordered after it on the stream
  return KSIM_OK;
}

// the queued Unreserves, when no framework cycle sits between PreFilter and
// Score (the state getters read the cache's view)
static int flush_idle(ksim_handle* h) {
  int rc = flush_pend_bind(h);
  if (rc) return rc;
  return (!h->fw_pending && !h->deferred_binds.empty()) ? flush_deferred_binds(h) : KSIM_OK;
}

static int flush_deferred_binds(ksim_handle* h) {
  std::vector<ksim_handle::DeferredBind> q;
  q.swap(h->deferred_binds);
  HIPCHK(h, hipSetDevice(h->device));
  for (auto& d : q) {
    ksim_pod_set v{};
    v.n_pods = 1;
    v.pods = &d.pod;
    v.n_exprs = (int32_t)d.ex.size();
    v.exprs = d.ex.data();
    v.n_terms = (int32_t)d.tm.size();
    v.terms = d.tm.data();
    v.n_uses = (int32_t)d.us.size();
    v.uses = d.us.data();
    v.n_adds = (int32_t)d.ad.size();
    v.adds = d.ad.data();
    v.n_nn = (int32_t)d.nn.size();
    v.nn = d.nn.data();
    const int rc = apply_bind(h, &v, 0, d.node, d.sign);
    if (rc) return rc;
  }
  return KSIM_OK;
}

static int assume_common(ksim_handle* h, const ksim_pod_set* ps, int32_t pod_index, int32_t node, int sign) {
  int rc = ensure_ready(h, sign < 0);
  if (rc) return rc;
  if (!ps || !ps->pods || pod_index < 0 || pod_index >= ps->n_pods || node < 0 || node >= h->dc.n)
    return set_err(h, KSIM_E_INVALID, "bad pod / node");
  if ((rc = validate_pod(h, ps, pod_index))) return rc;
  if (h->fw_pending) {                     // Unreserve, a cycle between PreFilter and Score: queued
    ksim_handle::DeferredBind d;
    single_pod_set(ps, pod_index, d.pod, d.ex, d.tm, d.us, d.ad, d.nn);
    d.node = node;
    d.sign = sign;
    h->deferred_binds.push_back(std::move(d));
    return KSIM_OK;
  }
  HIPCHK(h, hipSetDevice(h->device));
  return apply_bind(h, ps, pod_index, node, sign);
}

int ksim_assume(ksim_handle* h, const ksim_pod_set* ps, int32_t pod_index, int32_t node) {
  return assume_common(h, ps, pod_index, node, 1);
}

int ksim_forget(ksim_handle* h, const ksim_pod_set* ps, int32_t pod_index, int32_t node) {
  return assume_common(h, ps, pod_index, node, -1);
}

// Persistent domain tables of a queue: which pods read every
// domain sum from a table kept by the binds, and the tables they need.
struct PtabRegistry {
  std::vector<int4> ent;                 // {class, column, kind, first entry}
  std::vector<int32_t> cfirst, cidx;     // CSR by class
  int64_t len = 0;                       // int64 entries
  std::vector<uint8_t> pod;              // per pod: kPlanPtab
  std::vector<uint32_t> mask;            // per pod: UseMasks.ptab
  std::vector<int4> padd;                // per pod: the table updates of its adds
  std::vector<int32_t> padd_first, padd_count;
};

// uses: the queue's device use copies (kUseUniqueCol marked); their _pad
// becomes the first entry of the use's table.  A pod qualifies when each of
// its domain sums is independent of the pod beyond (class, column): PTS hard
// constraints on keys every node carries with nodeInclusionPolicies that
// filter nothing here, InterPodAffinity terms; value-keyed ScheduleAnyway
// constraints keep k_topo_prefilter (k_extrema reads their sums).  Shard
// handles exchange per-cycle sums and build no tables.
static void build_ptab(const ksim_handle* h, const ksim_pod_set* ps, std::vector<ksim_topo_use>& uses,
                       PtabRegistry& R) {
  R = PtabRegistry{};
  R.pod.assign((size_t)ps->n_pods, 0);
  R.mask.assign((size_t)ps->n_pods, 0);
  // replicas (RCCL ones included) hold every node: their tables are whole
  if ((is_sharded(h) && !h->replicated) || ab(kAbPtab)) return;   // A/B form: per-cycle PreFilter sums
  std::map<std::tuple<int32_t, int32_t, int32_t>, int32_t> index;
  for (int32_t i = 0; i < ps->n_pods; i++) {
    const ksim_pod& p = ps->pods[i];
    if (p.use_count <= 0) continue;
    ksim_topo_use* U = uses.data() + p.use_first;
    const UseMasks m = use_masks(h->prof, U, p.use_count);
    const bool pod_aff = p.sel_count > 0 || (p.flags & KSIM_POD_HAS_REQUIRED_AFFINITY);
    int32_t kind[KSIM_MAX_USES];
    bool ok = true;
    for (int k = 0; k < p.use_count && ok; k++) {
      const ksim_topo_use& u = U[k];
      const uint32_t b = 1u << k;
      kind[k] = -1;
      if (u.col == KSIM_COL_NONE) continue;
      if (use_node_count(u)) {                   // the node's own count; a total for the emptiness test
        if ((m.aff | m.score) & b && u.cls >= 0) kind[k] = kPtabTotal;
        continue;
      }
      if (u.kind == KSIM_USE_PTS_SOFT) {
        ok = false;
      } else if (u.kind == KSIM_USE_PTS_HARD) {
        ok = h->col_total[u.col] && h->col_nvals[u.col] <= kFuseMinValues &&
             !((u.flags & KSIM_USEF_HONOR_AFFINITY) && pod_aff) &&
             !((u.flags & KSIM_USEF_HONOR_TAINTS) && !h->hard_taints.empty());
        kind[k] = kPtabMark;
      } else {
        ok = !((m.aff | m.score) & b) || h->col_nvals[u.col] <= kFuseMinValues;   // emptiness scans
        kind[k] = kPtabPlain;
      }
    }
    if (!ok) continue;
    for (int k = 0; k < p.use_count; k++) {
      if (kind[k] < 0) continue;
      ksim_topo_use& u = U[k];
      const auto key = std::make_tuple(u.cls, (int32_t)u.col, kind[k]);
      auto it = index.find(key);
      if (it == index.end()) {
        it = index.emplace(key, (int32_t)R.ent.size()).first;
        R.ent.push_back(make_int4(u.cls, (int32_t)u.col, kind[k], (int32_t)R.len));
        R.len += kind[k] == kPtabTotal ? 1 : h->col_nvals[u.col];
      }
      u._pad = R.ent[(size_t)it->second].w;
      if (kind[k] != kPtabTotal) R.mask[i] |= 1u << k;
    }
    R.pod[i] = 1;
  }
  R.padd_first.assign((size_t)ps->n_pods, 0);
  R.padd_count.assign((size_t)ps->n_pods, 0);
  if (R.ent.empty()) return;
  const int32_t C = h->dc.n_classes;
  R.cfirst.assign((size_t)C + 1, 0);
  for (const int4& e : R.ent)
    if (e.x >= 0) R.cfirst[(size_t)e.x + 1]++;
  for (int32_t c = 0; c < C; c++) R.cfirst[(size_t)c + 1] += R.cfirst[(size_t)c];
  R.cidx.assign((size_t)R.cfirst[(size_t)C], 0);
  std::vector<int32_t> fill(R.cfirst.begin(), R.cfirst.end() - 1);
  for (size_t e = 0; e < R.ent.size(); e++)
    if (R.ent[e].x >= 0) R.cidx[(size_t)fill[(size_t)R.ent[e].x]++] = (int32_t)e;
  for (int32_t i = 0; i < ps->n_pods; i++) {
    const ksim_pod& p = ps->pods[i];
    R.padd_first[(size_t)i] = (int32_t)R.padd.size();
    for (int32_t a = 0; a < p.add_count; a++) {
      const ksim_class_add& ad = ps->adds[p.add_first + a];
      for (int32_t e = R.cfirst[(size_t)ad.cls]; e < R.cfirst[(size_t)ad.cls + 1]; e++) {
        const int4& t = R.ent[(size_t)R.cidx[(size_t)e]];
        R.padd.push_back(make_int4(t.w, t.y, t.z, ad.count));
      }
    }
    R.padd_count[(size_t)i] = (int32_t)R.padd.size() - R.padd_first[(size_t)i];
  }
}

// A use of a topology batch pod that may read a class an earlier pod of its
// run adds (ksim_tbatch.hip k_tb_chain_pairs): a node-local one (the guessed
// node's own count, re-keyed there).  A domain-keyed use ends the run: pod
// k's bind moves a whole domain for pod j.  Re-checking DoNotSchedule domain
// verdicts per batch was built and measured on config 3 (profiles/r04/tbcap):
// once an app's zones are level, nearly every bind of the app flips a zone's
// verdict, so the crossing pods were cut (pinv) after their evaluation was
// paid for (61.6 ms per step without crossing, 68.6-81.4 ms with).
static bool tbatch_conflict_ok(const ksim_topo_use& u) {
  return use_node_count(u) && u.kind != KSIM_USE_PTS_HARD && u.kind != KSIM_USE_NODE_PORT &&
         u.kind != KSIM_USE_IMAGE;
}

// The zone-variant use of a topology batch pod (ksim_device.h TbVar), or -1:
// its first DoNotSchedule spread use, read from a persistent table, keyed by a
// column of at most kVarDom domains (value ids 1 .. col_nvals - 1).
int32_t tbatch_vuse(const ksim_handle* h, const ksim_pod& p, const PodPlan& pl, const ksim_topo_use* U) {
  if (!(pl.flags & kPlanPtab)) return -1;
  for (int32_t i = 0; i < p.use_count && i < KSIM_MAX_USES; i++) {
    const ksim_topo_use& u = U[i];
    if (u.kind != KSIM_USE_PTS_HARD) continue;
    if (!((pl.m.hard >> i) & 1u) || !((pl.m.ptab >> i) & 1u) || u.col == KSIM_COL_NONE || u.cls < 0) return -1;
    if (u.col >= (1 << (32 - kPlanVcolShift)) - 1) return -1;
    const int32_t nd = h->col_nvals[u.col] - 1;
    return nd >= 1 && nd <= kVarDom ? i : -1;
  }
  return -1;
}

// Topology batch runs (class 3 pods, ksim_tbatch.hip): tlen[i] = the number
// of consecutive class-3 pods from i (at most kTbPods) none of which reads a
// count class an earlier one of them adds through a use tbatch_conflict_ok
// refuses; cross[i]: the run crosses a conflict.  0 for the other pods.
// variants: a pod may also read such a class through its zone-variant use
// (tbatch_vuse) when exactly one earlier pod of the run adds the class and the
// use's column is the run's variant column vcol[i] (the first such use's;
// -1: none), so the chain names its slot by where that pod lands.
// uses: the queue's device use copies.
void tbatch_runs(const ksim_pod_set* ps, const std::vector<ksim_topo_use>& uses,
                 const std::vector<uint8_t>& batchable, const std::vector<PodPlan>& plans, bool variants,
                 std::vector<int32_t>& tlen, std::vector<uint8_t>& cross, std::vector<int32_t>& vcol) {
  const int32_t n = ps->n_pods;
  tlen.assign((size_t)std::max(n, 0), 0);
  cross.assign((size_t)std::max(n, 0), 0);
  vcol.assign((size_t)std::max(n, 0), -1);
  int32_t n_cls = 0;
  for (int32_t k = 0; k < ps->n_adds; k++) n_cls = std::max(n_cls, ps->adds[k].cls + 1);
  std::vector<int32_t> stamp((size_t)n_cls, -1);   // class -> the window start that added it
  std::vector<int32_t> nadd((size_t)n_cls, 0);     // ... and how many pods of that run add it
  for (int32_t i = 0; i < n; i++) {
    if (batchable[i] != 3) continue;
    int32_t L = 0, vc = -1;
    bool crossed = false;
    for (int32_t j = i; j < n && L < kTbPods && batchable[j] == 3; j++, L++) {
      const ksim_pod& p = ps->pods[j];
      const ksim_topo_use* U = uses.data() + p.use_first;
      const int32_t vu = variants ? (int32_t)((plans[(size_t)j].flags >> kPlanVuseShift) & 31u) - 1 : -1;
      bool clash = false, hit = false;
      for (int32_t u = 0; u < p.use_count && !clash; u++) {
        const int32_t c = U[u].cls;
        if (c < 0 || c >= n_cls || stamp[c] != i) continue;
        hit = true;
        if (tbatch_conflict_ok(U[u])) continue;
        clash = !(u == vu && nadd[c] == 1 && (vc < 0 || vc == U[u].col));
        if (!clash) vc = U[u].col;
      }
      if (clash) break;
      crossed = crossed || hit;
      for (int32_t a = 0; a < p.add_count; a++) {
        const int32_t c = ps->adds[p.add_first + a].cls;
        if (stamp[c] != i) {
          stamp[c] = i;
          nadd[c] = 0;
        }
        nadd[c]++;   // per add entry: a pod listing the class twice counts as two adders
      }
    }
    tlen[i] = std::max(L, 1);
    cross[i] = crossed;
    vcol[i] = vc;
  }
}

int ksim_load_pods(ksim_handle* h, const ksim_pod_set* ps) {
  int rc = ensure_ready(h);
  if (rc) return rc;
  if (!ps || ps->n_pods < 0 || (ps->n_pods > 0 && !ps->pods) || ps->n_exprs < 0 || ps->n_terms < 0 ||
      ps->n_uses < 0 || ps->n_adds < 0 || ps->n_nn < 0)
    return set_err(h, KSIM_E_INVALID, "bad pod set");
  for (int32_t i = 0; i < ps->n_pods; i++)
    if ((rc = validate_pod(h, ps, i))) return rc;
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  // The handle holds no queue until every buffer below is in place: a failure
  // part-way leaves it empty, never with pointers to freed or half-written
  // buffers (or graphs captured over them).
  h->dp = DevPods{};
  h->batchable.clear();
  // A queue with the same array sizes as the loaded one (a policy sweep
  // reloading its pods under each profile) is copied into the same buffers:
  // the device pointers, and so every captured graph, stay valid.  Every count
  // a graph captures by value (n_pods, n_exprs, n_terms, n_uses, n_adds,
  // n_nn) is a byte size over a fixed element size, so equal sizes mean equal
  // captured values.
  const size_t np1 = (size_t)std::max(ps->n_pods, 1);
  std::vector<ksim_topo_use> uses(ps->uses, ps->uses + std::max(ps->n_uses, 0));
  mark_unique(h, uses.data(), uses.size());
  PtabRegistry R;
  build_ptab(h, ps, uses, R);
  const std::vector<size_t> bytes = {sizeof(ksim_pod) * (size_t)ps->n_pods,
                                     sizeof(int4) * R.ent.size(), 4 * R.cfirst.size(), 4 * R.cidx.size(),
                                     8 * (size_t)R.len, sizeof(int4) * R.padd.size(),
                                     sizeof(ksim_label_expr) * (size_t)ps->n_exprs,
                                     sizeof(ksim_term) * (size_t)ps->n_terms,
                                     4 * (size_t)ps->n_nn,
                                     4 * np1,
                                     sizeof(ksim_topo_use) * (size_t)ps->n_uses,
                                     sizeof(PodPlan) * (size_t)ps->n_pods,
                                     sizeof(ksim_class_add) * (size_t)ps->n_adds,
                                     4 * np1, 4 * np1};
  const bool reuse = h->d_chosen && h->pod_buf_bytes == bytes;
  auto drop_queue = [&](int code) {
    drop_graphs(h);
    free_bufs(h->pod_bufs);
    h->pod_buf_bytes.clear();
    if (h->d_chosen) (void)hipFree(h->d_chosen);
    h->d_chosen = nullptr;
    return code;
  };
  if (!reuse) drop_queue(KSIM_OK);
  size_t next_buf = 0;
  auto put = [&](const void* src, size_t nbytes, void** out) -> int {
    if (!reuse) return upload(h, h->pod_bufs, src, nbytes, out);
    DevBuf& b = h->pod_bufs[next_buf++];
    const hipError_t e = (src && nbytes) ? hipMemcpyAsync(b.p, src, nbytes, hipMemcpyHostToDevice, h->stream)
                                         : hipMemsetAsync(b.p, 0, b.bytes, h->stream);
    if (e != hipSuccess) return hip_fail(h, e, "pod upload");
    *out = b.p;
    return KSIM_OK;
  };
  std::vector<int32_t> bf(np1, 0);
  std::vector<uint8_t> batchable((size_t)ps->n_pods, 0);
  h->topo.assign((size_t)ps->n_pods, 0);
  h->xdom_len.assign((size_t)ps->n_pods, 0);
  h->trivial.assign((size_t)ps->n_pods, 0);
  h->noadd.assign((size_t)ps->n_pods, 0);
  h->noscalar.assign((size_t)ps->n_pods, 0);
  h->hard_small.assign((size_t)ps->n_pods, 1);
  h->soft_le1.assign((size_t)ps->n_pods, 1);
  h->xreg_len.assign((size_t)ps->n_pods, 0);
  for (int32_t i = 0; i < ps->n_pods; i++) {
    bool nv = false;
    batchable[i] = (uint8_t)pod_batchable(h, ps->pods[i], &nv);
    if (nv) bf[i] |= kPodNormVaries;
    h->topo[i] = ps->pods[i].use_count > 0 ? (R.pod[i] ? 2 : 1) : 0;
    // sharded-cycle exchange sizes, laid out as k_dom_pack / k_window_sh do
    bool soft = false;
    int n_soft = 0;
    int64_t xr = 1;
    for (int32_t k = 0; k < ps->pods[i].use_count; k++) {
      const ksim_topo_use& u = ps->uses[ps->pods[i].use_first + k];
      if (use_needs_dom(u)) h->xdom_len[i] += h->col_nvals[u.col];
      if (u.kind == KSIM_USE_PTS_HARD && u.col != KSIM_COL_NONE && h->col_nvals[u.col] > kFuseMinValues) h->hard_small[i] = 0;
      if (use_registers_values(u)) {
        xr += h->col_nvals[u.col];
        bf[i] |= kPodRegistersValues;
      }
      soft = soft || u.kind == KSIM_USE_PTS_SOFT;
      n_soft += u.kind == KSIM_USE_PTS_SOFT ? 1 : 0;
    }
    h->soft_le1[i] = n_soft <= 1 ? 1 : 0;
    h->xreg_len[i] = soft ? xr : 0;
    // class-2 pods (pod_batchable) read full rows: taints, labels, scalar columns
    if (static_trivial(h, ps->pods[i]) && batchable[i] != 2) bf[i] |= kBatchStaticTrivial;
    h->trivial[i] = (bf[i] & kBatchStaticTrivial) ? 1 : 0;
    h->noadd[i] = ps->pods[i].add_count == 0 ? 1 : 0;
    h->noscalar[i] = (ps->pods[i].flags & KSIM_POD_HAS_SCALAR) == 0 ? 1 : 0;
  }
  // static classes (DevPods::stab): the batch pods without scalar requests
  // (trivial ones too, so a run mixing them with static-plugin pods takes
  // the STAB kernels)
  std::vector<int32_t> scls(np1, -1), srep(np1, 0);
  int32_t ncls = 0;
  {
    std::unordered_map<std::string, int32_t> ids;
    std::string sig;
    for (int32_t i = 0; i < ps->n_pods; i++) {
      const ksim_pod& q = ps->pods[i];
      if (batchable[i] != 1 && batchable[i] != 2) continue;
      if ((q.flags & KSIM_POD_HAS_SCALAR) || !stab_signature(ps, q, sig)) continue;
      auto it = ids.find(sig);
      if (it == ids.end()) {
        if (ncls >= kStabMaxClasses) continue;
        it = ids.emplace(sig, ncls).first;
        srep[(size_t)ncls++] = i;
      }
      scls[(size_t)i] = it->second;
    }
  }
  std::vector<PodPlan> plans((size_t)ps->n_pods);
  for (int32_t i = 0; i < ps->n_pods; i++) {
    plans[i] = make_plan(h, ps->pods[i], uses.data() + std::max(ps->pods[i].use_first, 0));
    if (R.pod[i]) {
      plans[i].flags |= kPlanPtab;
      plans[i].m.ptab = R.mask[i];
    }
    if (!R.padd_first.empty()) {   // the table updates of its binds, listed
      plans[i].flags |= kPlanTadds;
      plans[i].tadd_first = R.padd_first[(size_t)i];
      plans[i].tadd_count = R.padd_count[(size_t)i];
    }
    if (batchable[i] == 0 && tbatch_admit(h, ps->pods[i], plans[i], h->hard_small[i] != 0, h->soft_le1[i] != 0)) {
      batchable[i] = 3;
      bf[i] |= kPodTopoBatch;
      const int32_t vu = tbatch_vuse(h, ps->pods[i], plans[i], uses.data() + std::max(ps->pods[i].use_first, 0));
      if (vu >= 0) plans[i].flags |= (uint32_t)(vu + 1) << kPlanVuseShift;
    }
  }
  std::vector<uint8_t> tcross, c2;
  std::vector<int32_t> tvcol, v2;
  tbatch_runs(ps, uses, batchable, plans, !ab(kAbTbVar), h->tlen, tcross, tvcol);
  tbatch_runs(ps, uses, batchable, plans, false, h->tlen_plain, c2, v2);   // replicated handles
  for (int32_t i = 0; i < ps->n_pods; i++) {
    // a run crosses with variants when it does without (a prefix of it)
    bf[i] |= (std::min(h->tlen[i], kTlenMask) << kTlenShift) | (std::min(h->tlen_plain[i], kTlenMask) << kTlenPlainShift) |
             (tcross[(size_t)i] ? kPodTbCross : 0);
    plans[i].flags |= (uint32_t)(tvcol[(size_t)i] + 1) << kPlanVcolShift;
  }
  DevPods P{};
  void* p = nullptr;
  if ((rc = put(ps->pods, sizeof(ksim_pod) * ps->n_pods, &p))) return drop_queue(rc);
  P.pods = (const ksim_pod*)p;
  if ((rc = put(ps->exprs, sizeof(ksim_label_expr) * ps->n_exprs, &p))) return drop_queue(rc);
  P.exprs = (const ksim_label_expr*)p;
  if ((rc = put(ps->terms, sizeof(ksim_term) * ps->n_terms, &p))) return drop_queue(rc);
  P.terms = (const ksim_term*)p;
  if ((rc = put(ps->nn, 4 * (size_t)ps->n_nn, &p))) return drop_queue(rc);
  P.nn = (const int32_t*)p;
  if ((rc = put(bf.data(), 4 * bf.size(), &p))) return drop_queue(rc);
  P.bflags = (const int32_t*)p;
  if ((rc = put(uses.data(), sizeof(ksim_topo_use) * uses.size(), &p))) return drop_queue(rc);
  P.uses = (const ksim_topo_use*)p;
  if ((rc = put(plans.data(), sizeof(PodPlan) * plans.size(), &p))) return drop_queue(rc);
  P.plans = (const PodPlan*)p;
  if ((rc = put(ps->adds, sizeof(ksim_class_add) * (size_t)ps->n_adds, &p))) return drop_queue(rc);
  P.adds = (const ksim_class_add*)p;
  if ((rc = put(scls.data(), 4 * np1, &p))) return drop_queue(rc);
  h->d_sclass = (int32_t*)p;
  if ((rc = put(srep.data(), 4 * np1, &p))) return drop_queue(rc);
  h->d_srep = (int32_t*)p;
  h->stab_ncls = ncls;
  h->sclass.assign(scls.begin(), scls.begin() + ps->n_pods);
  h->stab_dirty = true;
  if ((rc = put(R.ent.data(), sizeof(int4) * R.ent.size(), &p))) return drop_queue(rc);
  P.ptab_ent = (const int4*)p;
  if ((rc = put(R.cfirst.data(), 4 * R.cfirst.size(), &p))) return drop_queue(rc);
  P.ptab_cfirst = R.cfirst.empty() ? nullptr : (const int32_t*)p;
  if ((rc = put(R.cidx.data(), 4 * R.cidx.size(), &p))) return drop_queue(rc);
  P.ptab_cidx = (const int32_t*)p;
  if ((rc = put(nullptr, 8 * (size_t)R.len, &p))) return drop_queue(rc);   // filled by k_ptab_init
  P.ptab = (int64_t*)p;
  P.n_ptab = (int32_t)R.ent.size();
  if ((rc = put(R.padd.data(), sizeof(int4) * R.padd.size(), &p))) return drop_queue(rc);
  P.ptab_padd = (const int4*)p;
  P.n_uses = ps->n_uses;
  P.n_adds = ps->n_adds;
  P.n_nn = ps->n_nn;
  P.n_pods = ps->n_pods;
  P.n_exprs = ps->n_exprs;
  P.n_terms = ps->n_terms;
  hipError_t e = hipSuccess;
  if (!reuse) {
    e = hipMalloc(&h->d_chosen, 4 * np1);
    if (e != hipSuccess) {
      h->d_chosen = nullptr;
      return drop_queue(hip_fail(h, e, "hipMalloc"));
    }
    h->pod_buf_bytes = bytes;
  }
  if ((e = hipMemsetAsync(h->d_chosen, 0xff, 4 * np1, h->stream)) != hipSuccess ||
      (e = hipStreamSynchronize(h->stream)) != hipSuccess)
    return drop_queue(hip_fail(h, e, "pod queue setup"));
  h->batchable = std::move(batchable);
  h->dp = P;
  launch_ptab_init(h->dc, P, h->stream);
  if ((e = hipGetLastError()) != hipSuccess || (e = hipStreamSynchronize(h->stream)) != hipSuccess) {
    h->dp = DevPods{};
    return drop_queue(hip_fail(h, e, "persistent tables"));
  }
  return KSIM_OK;
}

int ksim_schedule_loaded(ksim_handle* h, int32_t first, int32_t count, int32_t* chosen, ksim_batch_stats* stats) {
  int rc = ensure_ready(h);
  if (rc) return rc;
  if (!h->dp.pods && count > 0) return set_err(h, KSIM_E_INVALID, "no pods loaded");
  if (first < 0 || count < 0 || first + count > h->dp.n_pods) return set_err(h, KSIM_E_INVALID, "range out of loaded pods");
  HIPCHK(h, hipSetDevice(h->device));
  if ((rc = ensure_stab(h))) return rc;
  if ((rc = reset_counters(h, h->stream))) return rc;
  int64_t perpod = 0;
  HIPCHK(h, hipEventRecord(h->ev0, h->stream));
  if (is_sharded(h)) {
    for (int32_t i = first; i < first + count; i++) perpod += pod_on_batch(h, i) ? 0 : 1;
    rc = shard_schedule({h}, first, count);
  } else {
    rc = for_each_run(h, first, count, [&](int32_t a, int32_t b, bool batch, bool topo) {
      if (!batch) perpod += b - a;
      return run_range(h, a, b, batch, topo);
    });
  }
  if (rc) return rc;
  HIPCHK(h, hipEventRecord(h->ev1, h->stream));
  HIPCHK(h, hipEventSynchronize(h->ev1));
  HIPCHK(h, hipGetLastError());
  if (chosen && count) HIPCHK(h, hcopy(h, chosen, h->d_chosen + first, 4 * (size_t)count, hipMemcpyDeviceToHost));
  if (stats) {
    DevState st;
    if ((rc = read_state(h, st))) return rc;
    float ms = 0;
    HIPCHK(h, hipEventElapsedTime(&ms, h->ev0, h->ev1));
    stats->pods = count;
    stats->scheduled = st.scheduled;
    stats->unschedulable = st.unschedulable;
    stats->evals = st.evals;
    stats->device_ms = ms;
    stats->batches = st.batches;
    stats->truncations = st.truncations;
    stats->perpod_cycles = perpod;
  }
  return KSIM_OK;
}

int ksim_set_shard(ksim_handle* h, int32_t node_base, int32_t n_total) {
  if (const int prc = flush_pend_bind(h)) return prc;   // a queued Reserve lands first
  if (!h) return KSIM_E_INVALID;
  h->stab_dirty = true;
  if (node_base < 0 || n_total < 0 || n_total > KSIM_MAX_NODES || node_base > n_total)
    return set_err(h, KSIM_E_INVALID, "bad shard range");
  if (h->has_cluster) return set_err(h, KSIM_E_INVALID, "ksim_set_shard must precede ksim_set_cluster");
  h->shard_base = node_base;
  h->shard_total = n_total;
  return KSIM_OK;
}

int ksim_set_eval_range(ksim_handle* h, int32_t eval_lo, int32_t eval_hi) {
  if (const int prc = flush_pend_bind(h)) return prc;   // a queued Reserve lands first
  if (!h) return KSIM_E_INVALID;
  if (!h->has_cluster) return set_err(h, KSIM_E_INVALID, "ksim_set_eval_range needs the cluster (ksim_set_cluster)");
  if (h->shard_total != 0) return set_err(h, KSIM_E_INVALID, "a node-shard handle holds only its nodes: no eval range");
  if (eval_lo < 0 || eval_hi < eval_lo || eval_hi > h->dc.n) return set_err(h, KSIM_E_INVALID, "bad eval range");
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  drop_cycle_graphs(h);                        // shard batch graphs captured with the old range
  h->replicated = true;
  h->eval_lo = eval_lo;
  h->eval_hi = eval_hi;
  return KSIM_OK;
}

int ksim_comm_unique_id(uint8_t* id) {
  if (!id) return KSIM_E_INVALID;
  if (!rccl().ok) return KSIM_E_RCCL;
  ncclUniqueId u;
  if (rccl().get_unique_id(&u) != ncclSuccess) return KSIM_E_RCCL;
  std::memcpy(id, u.internal, KSIM_COMM_ID_BYTES);
  return KSIM_OK;
}

int ksim_comm_init(ksim_handle* h, int32_t rank, int32_t world, const uint8_t* id) {
  if (const int prc = flush_pend_bind(h)) return prc;   // a queued Reserve lands first
  if (!h || !id) return KSIM_E_INVALID;
  if (world < 1 || world > kMaxShards || rank < 0 || rank >= world)
    return set_err(h, KSIM_E_INVALID, "world must be 1.." + std::to_string(kMaxShards));
  if (!rccl().ok) return set_err(h, KSIM_E_RCCL, "librccl not found");
  HIPCHK(h, hipSetDevice(h->device));
  if (h->comm) (void)rccl().comm_destroy(h->comm);
  h->comm = nullptr;
  ncclUniqueId u;
  std::memcpy(u.internal, id, KSIM_COMM_ID_BYTES);
  const ncclResult_t r = rccl().comm_init_rank(&h->comm, world, u, rank);
  if (r != ncclSuccess) {
    h->comm = nullptr;
    return set_err(h, KSIM_E_RCCL, std::string("ncclCommInitRank: ") + rccl().error_string(r));
  }
  h->rank = rank;
  h->world = world;
  if (h->rep_primary != (rank == 0)) {
    drop_graphs(h);                        // captured with the other counting flag
    h->rep_primary = rank == 0;
  }
  return KSIM_OK;
}

int ksim_group_schedule_loaded(ksim_handle** hs, int32_t n, int32_t first, int32_t count, int32_t* chosen,
                               ksim_batch_stats* stats) {
  if (!hs || n < 1 || n > kMaxShards) return KSIM_E_INVALID;
  ksim_handle* h0 = hs[0];
  std::vector<ksim_handle*> v(hs, hs + n);
  int32_t expect = 0;
  for (auto* h : v) {
    int rc = ensure_ready(h);
    if (rc) return rc;
    if (h->comm) return set_err(h0, KSIM_E_INVALID, "group handles must not hold a communicator");
    if (h->device != h0->device) return set_err(h0, KSIM_E_INVALID, "group handles must share one device");
    if (!h->dp.pods || h->dp.n_pods != h0->dp.n_pods) return set_err(h0, KSIM_E_INVALID, "pods not loaded alike");
    if (h->replicated != h0->replicated) return set_err(h0, KSIM_E_INVALID, "mixed replicated / shard handles");
    if (h->replicated) {                       // replicas: whole clusters, eval ranges tiling it in order
      if (h->dc.n != h0->dc.n || h->eval_lo != expect)
        return set_err(h0, KSIM_E_INVALID, "eval ranges must tile the cluster in order");
      expect = h->eval_hi;
      if (h->rep_primary != (h == h0)) {       // the first replica counts whole-run evaluations
        (void)hipStreamSynchronize(h->stream);
        drop_graphs(h);
        h->rep_primary = h == h0;
      }
      continue;
    }
    if (h->dc.n_total != h0->dc.n_total || h->dc.base != expect)
      return set_err(h0, KSIM_E_INVALID, "shards must tile the cluster in order");
    expect += h->dc.n;
  }
  if (expect != h0->dc.n_total) return set_err(h0, KSIM_E_INVALID, "shards must tile the cluster");
  if (first < 0 || count < 0 || first + count > h0->dp.n_pods) return set_err(h0, KSIM_E_INVALID, "range out of loaded pods");
  HIPCHK(h0, hipSetDevice(h0->device));
  int rc;
  for (auto* h : v)
    if ((rc = ensure_stab(h)) || (rc = reset_counters(h, h->stream))) return rc;
  HIPCHK(h0, hipEventRecord(h0->ev0, h0->stream));
  if (count && (rc = shard_schedule(v, first, count))) return rc;
  HIPCHK(h0, hipEventRecord(h0->ev1, h0->stream));
  HIPCHK(h0, hipEventSynchronize(h0->ev1));
  if (chosen && count) HIPCHK(h0, hcopy(h0, chosen, h0->d_chosen + first, 4 * (size_t)count, hipMemcpyDeviceToHost));
  if (stats) {
    std::memset(stats, 0, sizeof(*stats));
    for (auto* h : v) {
      DevState st;
      if ((rc = read_state(h, st))) return rc;
      stats->evals += st.evals;                // each shard counts its own nodes
      if (h == h0) {
        stats->scheduled = st.scheduled;
        stats->unschedulable = st.unschedulable;
        stats->batches = st.batches;
        stats->truncations = st.truncations;
      }
    }
    float ms = 0;
    HIPCHK(h0, hipEventElapsedTime(&ms, h0->ev0, h0->ev1));
    stats->pods = count;
    stats->device_ms = ms;
  }
  return KSIM_OK;
}

int ksim_schedule_batch(ksim_handle* h, const ksim_pod_set* ps, int32_t* chosen, ksim_batch_stats* stats) {
  int rc = ksim_load_pods(h, ps);
  if (rc) return rc;
  return ksim_schedule_loaded(h, 0, ps->n_pods, chosen, stats);
}

int ksim_reset_cluster(ksim_handle* h) {
  if (const int prc = flush_pend_bind(h)) return prc;   // a queued Reserve lands first
  if (!h || !h->has_cluster) return set_err(h, KSIM_E_INVALID, "cluster not set");
  h->stab_dirty = true;
  HIPCHK(h, hipSetDevice(h->device));
  const size_t N = (size_t)h->dc.n;
  const DevCluster& c = h->dc;
  // the dynamic columns from their snapshot copies and the run state zeroed,
  // in one launch (every buffer is a hipMalloc allocation: 16-byte aligned)
  ResetList L;
  hipError_t fe = hipSuccess;
  auto put = [&](void* d, const void* s, size_t bytes) {   // an entry the launch cannot take: its own copy
    if (L.add(d, s, bytes) || fe != hipSuccess) return;
    fe = s ? hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, h->stream) : hipMemsetAsync(d, 0, bytes, h->stream);
  };
  put(c.req_cpu, h->init.req_cpu, 8 * N);
  put(c.req_mem, h->init.req_mem, 8 * N);
  put(c.req_eph, h->init.req_eph, 8 * N);
  if (c.n_scalar) put(c.req_scalar, h->init.req_scalar, 8 * N * c.n_scalar);
  put(c.nz_cpu, h->init.nz_cpu, 8 * N);
  put(c.nz_mem, h->init.nz_mem, 8 * N);
  put(c.num_pods, h->init.num_pods, 4 * N);
  if (c.n_classes) put(c.cnt, h->init.cnt, 4 * N * c.n_classes);
  put(c.nb_alloc, h->init.nb_alloc, 8 * N);
  static_assert(sizeof(DevState) % 4 == 0, "DevState by words");
  put(h->st, nullptr, sizeof(DevState));
  HIPCHK(h, fe);
  if (L.n) launch_reset_copy(L, h->stream);
  launch_ptab_init(h->dc, h->dp, h->stream);        // the queue's persistent tables follow the counts
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return KSIM_OK;
}

int ksim_time_eval(ksim_handle* h, int32_t first, int32_t reps, double* avg_ms, int32_t* kernel) {
  int rc = ensure_ready(h);
  if (rc) return rc;
  if (!avg_ms || reps < 1 || !h->dp.pods || first < 0 || first >= h->dp.n_pods)
    return set_err(h, KSIM_E_INVALID, "bad ksim_time_eval arguments");
  const bool batch = pod_on_batch(h, first) && !is_sharded(h);
  if (batch && h->batchable[first] == 3)
    return set_err(h, KSIM_E_UNSUPPORTED, "topology batch evaluations span two kernels");
  if (batch && adapt_mode(h)) return set_err(h, KSIM_E_UNSUPPORTED, "ADAPT batch evaluations span two kernels");
  HIPCHK(h, hipSetDevice(h->device));
  if ((rc = ensure_stab(h))) return rc;
  // two batches' pods: the deferred-commit timing below keys batch 1 (a full
  // batch whatever batch 0 commits)
  const int32_t end = batch ? std::min(h->dp.n_pods, first + 2 * kBatchPods) : first + 1;
  if ((rc = set_run(h, first, end))) return rc;
  LaunchArgs a = make_args(h, h->dp, h->d_chosen);
  if (batch) pick_keys(h, first, end, a);
  a.fuse_min = !batch && h->topo[first] && h->hard_small[first];
  a.fuse_ext = !batch && h->soft_le1[first];
  a.ptab = !batch && h->topo[first] == 2;
  if (batch && a.fast && lazy_ok(h, first, end, true, a.stab)) {
    // the deferred-commit evaluation launch as the run issues it: batch 0 of
    // the run (both launches), then batch 1's k_batch_top_commit repeated
    // (idempotent: it reads X[0], st[0] and slot 0, and writes X[1], st[1],
    // the lists and batch 0's placements); the handle's own buffers keep
    // their contents
    if ((rc = lazy_begin(h))) return rc;
    launch_batch_lazy(lazy_batch(h, a, 0), h->stream);
    const LazyBatch z = lazy_batch(h, a, 1);
    launch_lazy_top(z, h->stream);
    HIPCHK(h, hipEventRecord(h->ev0, h->stream));
    for (int32_t i = 0; i < reps; i++) launch_lazy_top(z, h->stream);
    HIPCHK(h, hipEventRecord(h->ev1, h->stream));
    HIPCHK(h, hipEventSynchronize(h->ev1));
    HIPCHK(h, hipGetLastError());
    float ms = 0;
    HIPCHK(h, hipEventElapsedTime(&ms, h->ev0, h->ev1));
    *avg_ms = ms / reps;
    if (kernel) *kernel = kKernelsPerCycle + kKernelsPerBatch + kKernelsPerAdapt + kKernelsPerTbatch;
    return KSIM_OK;
  }
  auto launch = [&] {
    if (batch) launch_batch_eval_only(a, h->stream);
    else launch_filter_only(a, h->stream);
  };
  launch();                                          // warm (code object, caches)
  HIPCHK(h, hipEventRecord(h->ev0, h->stream));
  for (int32_t i = 0; i < reps; i++) launch();
  HIPCHK(h, hipEventRecord(h->ev1, h->stream));
  HIPCHK(h, hipEventSynchronize(h->ev1));
  HIPCHK(h, hipGetLastError());
  float ms = 0;
  HIPCHK(h, hipEventElapsedTime(&ms, h->ev0, h->ev1));
  *avg_ms = ms / reps;
  // the timed no-window filter passes added into the window counters
  if (!batch) HIPCHK(h, hzero(h, h->sc.win, sizeof(WinState)));
  if (kernel) *kernel = batch ? kKernelsPerCycle : 2;   // k_batch_top / k_filter_score
  return KSIM_OK;
}

const char* ksim_kernel_name(int32_t k) {
  if (k >= 0 && k < kKernelsPerCycle) return kKernelNames[k];
  k -= kKernelsPerCycle;
  if (k >= 0 && k < kKernelsPerBatch) return kBatchKernelNames[k];
  k -= kKernelsPerBatch;
  if (k >= 0 && k < kKernelsPerAdapt) return kAdaptKernelNames[k];
  k -= kKernelsPerAdapt;
  if (k >= 0 && k < kKernelsPerTbatch) return kTbatchKernelNames[k];
  k -= kKernelsPerTbatch;
  if (k >= 0 && k < kKernelsPerLazy) return kLazyKernelNames[k];
  k -= kKernelsPerLazy;
  if (k >= 0 && k < kKernelsPerLazyAdapt) return kLazyAdaptKernelNames[k];
  return nullptr;
}

int ksim_time_kernels(ksim_handle* h, int32_t first, int32_t count, double* avg_ms, int64_t* launches, int32_t cap) {
  int rc = ensure_ready(h);
  if (rc) return rc;
  constexpr int kKinds = kKernelsPerCycle + kKernelsPerBatch + kKernelsPerAdapt + kKernelsPerTbatch + kKernelsPerLazy +
                         kKernelsPerLazyAdapt;
  if (!avg_ms || cap < kKinds) return set_err(h, KSIM_E_INVALID, "avg_ms too small");
  if (!h->dp.pods || first < 0 || count <= 0 || first + count > h->dp.n_pods)
    return set_err(h, KSIM_E_INVALID, "range out of loaded pods");
  HIPCHK(h, hipSetDevice(h->device));
  if ((rc = ensure_stab(h))) return rc;
  double sum[kKinds] = {0};
  int64_t n[kKinds] = {0};
  LaunchArgs a = make_args(h, h->dp, h->d_chosen);
  rc = for_each_run(h, first, count, [&](int32_t lo, int32_t hi, bool batch, bool topo) -> int {
    int r;
    if ((r = set_run(h, lo, hi))) return r;
    const bool adapt = batch && adapt_mode(h);
    const bool tb = batch && topo;                 // topology batch runs (class 3)
    // the same kernel variants the run itself would launch
    a.fast = a.stab = false;
    if (batch) pick_keys(h, lo, hi, a);
    a.fuse_min = !batch && topo;
    for (int32_t i = lo; i < hi && a.fuse_min; i++) a.fuse_min = h->hard_small[i] != 0;
    a.fuse_ext = !batch;
    for (int32_t i = lo; i < hi && a.fuse_ext; i++) a.fuse_ext = h->soft_le1[i] != 0;
    a.ptab = !batch && h->topo[lo] == 2;
    const int per = tb ? kKernelsPerTbatch : adapt ? kKernelsPerAdapt : batch ? kKernelsPerBatch : kKernelsPerCycle;
    const int base = tb      ? kKernelsPerCycle + kKernelsPerBatch + kKernelsPerAdapt
                     : adapt ? kKernelsPerCycle + kKernelsPerBatch
                     : batch ? kKernelsPerCycle : 0;
    if (tb) {
      HIPCHK(h, hipMemsetAsync(h->sc.tb_win, 0, sizeof(WinState) * kTbPods, h->stream));
      HIPCHK(h, hipMemsetAsync(h->sc.tb_dom, 0, sizeof(TbDom) * kTbPods * kVarDom, h->stream));
      HIPCHK(h, hipMemsetAsync(h->sc.tb_vhold, 0, 4 * (size_t)kTbPods * kVarSlots * 2 * KSIM_MAX_SCORE, h->stream));
    }
    if (batch && !tb && a.fast && lazy_ok(h, lo, hi, true, a.stab)) {
      // deferred-commit batches: two (P100) or three to four (ADAPT) launches
      // each, a flush (untimed) before every state read
      const int lper = adapt ? kKernelsPerLazyAdapt : kKernelsPerLazy;
      const int lbase = kKernelsPerCycle + kKernelsPerBatch + kKernelsPerAdapt + kKernelsPerTbatch +
                        (adapt ? kKernelsPerLazy : 0);
      HIPCHK(h, hipMemsetAsync(&h->st->batches, 0, 4, h->stream));
      if ((r = lazy_begin(h))) return r;
      int64_t i = 0;
      int32_t cursor = lo, done_batches = 0;
      while (cursor < hi) {
        const int32_t iters = std::min(64, (hi - cursor + kBatchPods - 1) / kBatchPods);
        std::vector<hipEvent_t> evs((size_t)iters * (lper + 1));
        for (auto& e : evs) HIPCHK(h, hipEventCreate(&e));
        uint32_t launched = 0;
        for (int32_t t = 0; t < iters; t++, i++)
          launched = lazy_launch(h, lazy_batch(h, a, i), h->stream, &evs[(size_t)t * (lper + 1)]);
        lazy_flush(h, lazy_batch(h, a, i), h->stream);
        HIPCHK(h, hipGetLastError());
        DevState st;
        if ((r = read_state_at(h, (i & 1) ? h->lazy_st1 : h->st, st))) return r;
        const int32_t did = std::min<int32_t>(iters, st.batches - done_batches);
        done_batches = st.batches;
        for (int32_t t = 0; t < did; t++)
          for (int k = 0; k < lper; k++) {
            if (!((launched >> k) & 1u)) continue;   // an empty event pair (the window fused into the top)
            float ms = 0;
            const size_t e0 = (size_t)t * (lper + 1);
            HIPCHK(h, hipEventElapsedTime(&ms, evs[e0 + k], evs[e0 + k + 1]));
            sum[lbase + k] += ms;
            n[lbase + k] += 1;
          }
        for (auto& e : evs) (void)hipEventDestroy(e);
        if (st.cursor <= cursor) return set_err(h, KSIM_E_DEVICE, "no progress while timing");
        cursor = st.cursor;
        i++;
      }
      return lazy_end(h, i - 1);
    }
    int32_t cursor = lo;
    uint32_t launched = (1u << per) - 1;         // batch paths launch every kernel of a batch
    while (cursor < hi) {
      int32_t iters = batch ? std::min(64, (hi - cursor + kBatchPods - 1) / kBatchPods) : std::min(512, hi - cursor);
      if (tb) {                                  // the batches the host's run lengths predict (run_tbatch)
        iters = 0;
        for (int32_t i = cursor; i < hi && iters < 64; iters++) i += std::min(std::min(kTbPods, hi - i), std::max(h->tlen[i], 1));
      }
      std::vector<hipEvent_t> evs((size_t)iters * (per + 1));
      for (auto& e : evs) HIPCHK(h, hipEventCreate(&e));
      if (batch) HIPCHK(h, hipMemsetAsync(&h->st->batches, 0, 4, h->stream));
      for (int32_t i = 0; i < iters; i++) {
        if (tb)
          launched = launch_tbatch(a, h->stream, &evs[(size_t)i * (per + 1)]);
        else if (adapt)
          launched = launch_batch_adapt(a, h->stream, &evs[(size_t)i * (per + 1)]);
        else if (batch)
          launched = launch_batch(a, h->stream, &evs[(size_t)i * (per + 1)]);
        else
          launched = launch_cycle(a, h->stream, false, topo, &evs[(size_t)i * (per + 1)]);
      }
      HIPCHK(h, hipGetLastError());
      DevState st;
      if ((r = read_state(h, st))) return r;
      // iterations past the end exit at once; count only those that did work
      const int32_t did = batch ? std::min<int32_t>(iters, st.batches) : std::min(iters, st.cursor - cursor);
      for (int32_t i = 0; i < did; i++)
        for (int k = 0; k < per; k++) {
          if (!((launched >> k) & 1u)) continue;   // an empty event pair, not a kernel
          float ms = 0;
          const size_t b = (size_t)i * (per + 1);
          HIPCHK(h, hipEventElapsedTime(&ms, evs[b + k], evs[b + k + 1]));
          sum[base + k] += ms;
          n[base + k] += 1;
        }
      for (auto& e : evs) (void)hipEventDestroy(e);
      if (st.cursor <= cursor) return set_err(h, KSIM_E_DEVICE, "no progress while timing");
      cursor = st.cursor;
    }
    return KSIM_OK;
  });
  if (rc) return rc;
  for (int k = 0; k < kKinds; k++) {
    avg_ms[k] = n[k] ? sum[k] / n[k] : 0.0;
    if (launches) launches[k] = n[k];
  }
  return kKinds;
}

}  // extern "C"

extern "C" int ksim_get_diag(ksim_handle* h, int64_t* out, int32_t n) {
  if (!h || !out || n < 0) return KSIM_E_INVALID;
  DevState st;
  int rc = read_state(h, st);
  if (rc) return rc;
  int64_t v[3 + 16 + 2 + 4 + 2] = {st.batches, st.truncations, st.cuts};
  if (h->has_cluster) HIPCHK(h, hcopy(h, v + 3, h->sc.dbg, 8 * 16, hipMemcpyDeviceToHost));
  if (unsigned long long* cp = cp_clock_buffer())   // KSIM_CP_CLOCKS builds: the chain + pairs phase clocks
    HIPCHK(h, hcopy(h, v + 3, cp, 8 * 8, hipMemcpyDeviceToHost));
  if (unsigned long long* ad = adapt_dbg_buffer())  // KSIM_ADAPT_DBG builds: ADAPT batch ends
    HIPCHK(h, hcopy(h, v + 3, ad, 8 * 8, hipMemcpyDeviceToHost));
  v[19] = h->graph_captures;
  v[20] = h->match_ns;
  for (int k = 0; k < 4; k++) v[21 + k] = h->fw_counts[k];
  v[25] = (int64_t)batch_variant_reach();
  if (h->has_cluster && h->sc.tb_vpods) HIPCHK(h, hcopy(h, v + 26, h->sc.tb_vpods, 8, hipMemcpyDeviceToHost));
  const int32_t m = n < 27 ? n : 27;
  for (int32_t i = 0; i < m; i++) out[i] = v[i];
  return m;
}

extern "C" int ksim_batch_geometry(int32_t* out, int32_t n) {
  if (!out || n < 0) return KSIM_E_INVALID;
  const int32_t v[4] = {kBatchPods, kTopT, kTopThreads, kTileCand};
  const int32_t m = n < 4 ? n : 4;
  for (int32_t i = 0; i < m; i++) out[i] = v[i];
  return m;
}


// ---- PostFilter: DefaultPreemption (ksim_preempt.hip) ------------------------------
extern "C" int ksim_set_bound_pods(ksim_handle* h, const ksim_bound_pods* b) {
  int rc = ensure_ready(h);
  if (rc) return rc;
  if (!b || b->n < 0 || (b->n > 0 && (!b->node || !b->priority || !b->start_time || !b->req)))
    return set_err(h, KSIM_E_INVALID, "bad bound-pod table");
  const int32_t N = h->dc.n, n = b->n;
  for (int32_t i = 0; i < n; i++)
    if (b->node[i] < 0 || b->node[i] >= N) return set_err(h, KSIM_E_INVALID, "bound pod on a node out of range");
  // per node, util.MoreImportantPod order (priority desc, start asc), then table order
  std::vector<int32_t> ix((size_t)n);
  for (int32_t i = 0; i < n; i++) ix[i] = i;
  std::sort(ix.begin(), ix.end(), [&](int32_t x, int32_t y) {
    if (b->node[x] != b->node[y]) return b->node[x] < b->node[y];
    if (b->priority[x] != b->priority[y]) return b->priority[x] > b->priority[y];
    if (b->start_time[x] != b->start_time[y]) return b->start_time[x] < b->start_time[y];
    return x < y;
  });
  std::vector<int32_t> off((size_t)N + 1, 0), prio((size_t)std::max(n, 1));
  std::vector<int64_t> start((size_t)std::max(n, 1)), req((size_t)std::max(n, 1) * KSIM_PREEMPT_REQ);
  for (int32_t i = 0; i < n; i++) off[b->node[i] + 1]++;
  for (int32_t v = 0; v < N; v++) off[v + 1] += off[v];
  for (int32_t k = 0; k < n; k++) {
    const int32_t i = ix[k];
    prio[k] = b->priority[i];
    start[k] = b->start_time[i];
    for (int q = 0; q < KSIM_PREEMPT_REQ; q++) req[(size_t)k * KSIM_PREEMPT_REQ + q] = b->req[(size_t)i * KSIM_PREEMPT_REQ + q];
  }
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  free_bufs(h->pre_bufs);
  DevPreempt d{};
  void* p = nullptr;
  if ((rc = upload(h, h->pre_bufs, off.data(), 4 * off.size(), &p))) return rc;
  d.off = (const int32_t*)p;
  if ((rc = upload(h, h->pre_bufs, prio.data(), 4 * prio.size(), &p))) return rc;
  d.prio = (const int32_t*)p;
  if ((rc = upload(h, h->pre_bufs, start.data(), 8 * start.size(), &p))) return rc;
  d.start = (const int64_t*)p;
  if ((rc = upload(h, h->pre_bufs, req.data(), 8 * req.size(), &p))) return rc;
  d.req = (const int64_t*)p;
  if ((rc = upload(h, h->pre_bufs, nullptr, (size_t)std::max(n, 1), &p))) return rc;
  d.vflag = (uint8_t*)p;
  if ((rc = upload(h, h->pre_bufs, nullptr, sizeof(PreemptNode) * (size_t)N, &p))) return rc;
  d.res = (PreemptNode*)p;
  if ((rc = upload(h, h->pre_bufs, nullptr, 16, &p))) return rc;
  d.pick = (int32_t*)p;
  if ((rc = upload(h, h->pre_bufs, nullptr, 4 * (size_t)std::max(N, 1), &p))) return rc;
  d.nslot = (int32_t*)p;
  HIPCHK(h, hipMemsetAsync(d.nslot, 0xff, 4 * (size_t)std::max(N, 1), h->stream));   // -1: no group
  d.nreq = nullptr;
  HIPCHK(h, hipStreamSynchronize(h->stream));
  h->pre = d;
  h->pre_index = ix;
  h->pre_n = n;
  return KSIM_OK;
}

extern "C" int ksim_preempt(ksim_handle* h, const ksim_pod_set* ps, int32_t pod_index, int32_t priority,
                            ksim_preempt_out* out) {
  return ksim_preempt_nominated(h, ps, pod_index, priority, nullptr, 0, nullptr, nullptr, nullptr, out);
}

extern "C" int ksim_preempt_nominated(ksim_handle* h, const ksim_pod_set* ps, int32_t pod_index, int32_t priority,
                                      const ksim_pod_set* nps, int32_t n_groups, const int32_t* gnodes,
                                      const int32_t* first, const int32_t* count, ksim_preempt_out* out) {
  int rc = ensure_ready(h);
  if (rc) return rc;
  if (!ps || !out || pod_index < 0 || pod_index >= ps->n_pods || !ps->pods)
    return set_err(h, KSIM_E_INVALID, "bad pod set / index");
  if (n_groups < 0 || (n_groups > 0 && (!nps || !nps->pods || !gnodes || !first || !count)))
    return set_err(h, KSIM_E_INVALID, "bad nominated-node groups");
  {
    std::vector<uint8_t> seen((size_t)std::max(h->dc.n, 1), 0);
    for (int32_t k = 0; k < n_groups; k++) {
      if (gnodes[k] < 0 || gnodes[k] >= h->dc.n || seen[gnodes[k]])
        return set_err(h, KSIM_E_INVALID, "nominated node out of range or repeated");
      seen[gnodes[k]] = 1;
      if (count[k] < 0 || first[k] < 0 || first[k] + count[k] > nps->n_pods)
        return set_err(h, KSIM_E_INVALID, "nominated pod range out of the pod set");
      for (int32_t j = first[k]; j < first[k] + count[k]; j++)
        if ((rc = validate_pod(h, nps, j))) return rc;
    }
  }
  if (!h->pre.off) return set_err(h, KSIM_E_INVALID, "ksim_set_bound_pods first");
  if (is_sharded(h)) return set_err(h, KSIM_E_UNSUPPORTED, "preemption runs on unsharded handles");
  if (prof_has_filter(h->prof, KSIM_PL_NETWORK_BANDWIDTH))
    return set_err(h, KSIM_E_UNSUPPORTED, "preemption dry runs re-run Fit only, not NetworkBandwidth");
  if (ps->pods[pod_index].use_count > 0)
    return set_err(h, KSIM_E_UNSUPPORTED, "preemption for pods with topology / port / image uses");
  if (ps->pods[pod_index].flags & KSIM_POD_NODE_NAMES)
    return set_err(h, KSIM_E_UNSUPPORTED, "preemption for pods a PreFilterResult restricts");
  if ((rc = validate_pod(h, ps, pod_index))) return rc;
  int32_t fit = -1;
  for (int f = 0; f < h->prof.n_filter; f++)
    if (h->prof.filter[f] == KSIM_PL_NODE_RESOURCES_FIT) fit = f;
  HIPCHK(h, hipSetDevice(h->device));
  DevPods P;
  if ((rc = upload_single(h, ps, pod_index, P))) return rc;
  if ((rc = set_run(h, 0, 1))) return rc;
  const LaunchArgs a = make_args(h, P, nullptr);
  DevPreempt pre = h->pre;
  std::vector<uint8_t> gfail((size_t)std::max(n_groups, 1), KSIM_PASSED);
  std::vector<int64_t> nreq((size_t)std::max(n_groups, 1) * (KSIM_PREEMPT_REQ + 1), 0);
  auto bind_group = [&](int32_t k, int sign) -> int {
    for (int32_t j = first[k]; j < first[k] + count[k]; j++) {
      DevPods Q;
      int r;
      if ((r = upload_single(h, nps, j, Q, h->nom_arena))) return r;
      launch_assume(h->dc, Q, 0, gnodes[k], sign, h->stream);
      HIPCHK(h, hipGetLastError());
    }
    return KSIM_OK;
  };
  for (int32_t k = 0; k < n_groups; k++) {                // pass 1 of each grouped node
    if ((rc = bind_group(k, 1))) return rc;
    launch_filter_only(a, h->stream);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hcopy(h, &gfail[k], h->sc.fail + gnodes[k], 1, hipMemcpyDeviceToHost));
    if ((rc = bind_group(k, -1))) return rc;
    int64_t* q = nreq.data() + (size_t)k * (KSIM_PREEMPT_REQ + 1);
    for (int32_t j = first[k]; j < first[k] + count[k]; j++) {
      const ksim_pod& x = nps->pods[j];
      q[0] += x.req_cpu;
      q[1] += x.req_mem;
      q[2] += x.req_eph;
      for (int c = 0; c < KSIM_MAX_SCALAR; c++) q[3 + c] += x.scalar_req[c];
    }
    q[KSIM_PREEMPT_REQ] = count[k];
  }
  launch_filter_only(a, h->stream);                        // every node as is
  HIPCHK(h, hipGetLastError());
  if (n_groups > 0) {
    free_bufs(h->pre_nom_bufs);
    void* p = nullptr;
    if ((rc = upload(h, h->pre_nom_bufs, nreq.data(), 8 * nreq.size(), &p))) return rc;
    pre.nreq = (const int64_t*)p;
    for (int32_t k = 0; k < n_groups; k++) {
      // a grouped node's status: pass 1's unless it passed (then pass 2's, as is)
      if (gfail[k] != KSIM_PASSED) {
        gfail[k] &= (uint8_t)~kFailError;
        HIPCHK(h, hipMemcpyAsync(h->sc.fail + gnodes[k], &gfail[k], 1, hipMemcpyHostToDevice, h->stream));
      }
      HIPCHK(h, hipMemcpyAsync(pre.nslot + gnodes[k], &k, 4, hipMemcpyHostToDevice, h->stream));
      HIPCHK(h, hipStreamSynchronize(h->stream));        // k and gfail[k] are host stack / vector slots
    }
  }
  launch_preempt(a, pre, fit, priority, h->stream, false);
  HIPCHK(h, hipGetLastError());
  if (n_groups > 0) {
    static const int32_t kNoGroup = -1;
    for (int32_t k = 0; k < n_groups; k++)
      HIPCHK(h, hipMemcpyAsync(pre.nslot + gnodes[k], &kNoGroup, 4, hipMemcpyHostToDevice, h->stream));
  }
  int32_t pick[4];
  HIPCHK(h, hipMemcpyAsync(pick, h->pre.pick, sizeof(pick), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  out->nominated = pick[0];
  out->n_victims = pick[1];
  out->n_potential = pick[2];
  out->n_candidates = pick[3];
  if (pick[0] >= 0 && out->victims && out->victims_cap > 0) {
    std::vector<int32_t> off(2);
    HIPCHK(h, hcopy(h, off.data(), h->pre.off + pick[0], 8, hipMemcpyDeviceToHost));
    std::vector<uint8_t> flag((size_t)std::max(off[1] - off[0], 1));
    if (off[1] > off[0])
      HIPCHK(h, hcopy(h, flag.data(), h->pre.vflag + off[0], (size_t)(off[1] - off[0]), hipMemcpyDeviceToHost));
    int32_t k = 0;
    for (int32_t j = off[0]; j < off[1] && k < out->victims_cap; j++)
      if (flag[j - off[0]]) out->victims[k++] = h->pre_index[j];
  }
  return KSIM_OK;
}

// ---- selector / affinity-term matching (ksim_match.hip) ------
extern "C" int ksim_match_terms(ksim_handle* h, const ksim_match_problem* mp, uint32_t* match_bits, int32_t* counts) {
  if (const int prc = flush_pend_bind(h)) return prc;   // a queued Reserve lands first
  if (!h || !mp || !match_bits) return set_err(h, KSIM_E_INVALID, "null argument");
  const ksim_match_problem& q = *mp;
  if (q.n_sigs < 0 || q.n_feat < 0 || q.n_reqs < 0 || q.n_matchers < 0 || q.n_pods < 0 || q.n_nodes < 0 ||
      q.n_classes < 0)
    return set_err(h, KSIM_E_INVALID, "negative size");
  if (q.n_reqs > kMatchMaxReqs || q.n_feat > kMatchMaxFeat)
    return set_err(h, KSIM_E_UNSUPPORTED, "match problem exceeds 4096 requirements or 65536 features");
  if (q.n_classes > 0 && !counts) return set_err(h, KSIM_E_INVALID, "counts buffer missing");
  if (!q.sig_feat_off || !q.req_feat_off || (!q.req_neg && q.n_reqs > 0) || !q.m_req_off)
    return set_err(h, KSIM_E_INVALID, "null CSR");
  // host validation: every index the kernels follow is in range
  auto csr_ok = [](const int32_t* off, int32_t rows, const int32_t* v, int32_t bound) {
    if (off[0] != 0) return false;
    for (int32_t i = 0; i < rows; i++)
      if (off[i + 1] < off[i]) return false;
    if (off[rows] > 0 && !v) return false;
    for (int32_t j = 0; j < off[rows]; j++)
      if (v[j] < 0 || v[j] >= bound) return false;
    return true;
  };
  if (!csr_ok(q.sig_feat_off, q.n_sigs, q.sig_feat, q.n_feat) ||
      !csr_ok(q.req_feat_off, q.n_reqs, q.req_feat, q.n_feat) ||
      !csr_ok(q.m_req_off, q.n_matchers, q.m_req, q.n_reqs))
    return set_err(h, KSIM_E_INVALID, "feature / requirement index out of range");
  if (q.n_classes > 0) {
    if (!q.class_matcher) return set_err(h, KSIM_E_INVALID, "class_matcher missing");
    for (int32_t c = 0; c < q.n_classes; c++)
      if (q.class_matcher[c] < 0 || q.class_matcher[c] >= q.n_matchers)
        return set_err(h, KSIM_E_INVALID, "class matcher out of range");
    if (q.n_pods > 0 && (!q.pod_sig || !q.pod_node)) return set_err(h, KSIM_E_INVALID, "bound pod arrays missing");
    for (int32_t p = 0; p < q.n_pods; p++)
      if (q.pod_sig[p] < 0 || q.pod_sig[p] >= q.n_sigs || q.pod_node[p] < 0 || q.pod_node[p] >= q.n_nodes)
        return set_err(h, KSIM_E_INVALID, "bound pod signature / node out of range");
  }
  if (q.n_sigs == 0) {                         // no signature: no bound pod either (pod_sig < n_sigs)
    if (q.n_classes > 0 && q.n_nodes > 0) std::memset(counts, 0, (size_t)q.n_classes * q.n_nodes * 4);
    return KSIM_OK;
  }
  HIPCHK(h, hipSetDevice(h->device));
  DevMatch m{};
  m.s = q.n_sigs;
  m.sp = (q.n_sigs + 15) / 16 * 16;
  m.fp = std::max(64, (q.n_feat + 63) / 64 * 64);
  m.r = q.n_reqs;
  m.rp = std::max(16, (q.n_reqs + 15) / 16 * 16);
  m.m = q.n_matchers;
  m.w = (q.n_matchers + 31) / 32;
  m.c = q.n_classes;
  m.cw = (q.n_classes + 31) / 32;
  m.p = q.n_classes > 0 ? q.n_pods : 0;
  m.n = q.n_nodes;
  std::vector<DevBuf> bufs;
  struct Guard {
    std::vector<DevBuf>& b;
    ~Guard() { free_bufs(b); }
  } guard{bufs};
  int rc;
  void* p;
  std::vector<uint8_t> neg((size_t)m.rp, 0);
  std::copy(q.req_neg, q.req_neg + q.n_reqs, neg.begin());
  if ((rc = upload(h, bufs, nullptr, (size_t)m.sp * m.fp, &p))) return rc;
  m.a = (int8_t*)p;
  if ((rc = upload(h, bufs, nullptr, (size_t)m.rp * m.fp, &p))) return rc;
  m.bt = (int8_t*)p;
  if ((rc = upload(h, bufs, neg.data(), neg.size(), &p))) return rc;
  m.neg = (uint8_t*)p;
  auto put = [&](const int32_t* src, int64_t n, const int32_t** dst) {
    void* d;
    int r = upload(h, bufs, src, (size_t)std::max<int64_t>(n, 0) * 4, &d);
    *dst = (const int32_t*)d;
    return r;
  };
  if ((rc = put(q.sig_feat_off, q.n_sigs + 1, &m.sig_off)) || (rc = put(q.sig_feat, q.sig_feat_off[q.n_sigs], &m.sig_feat)) ||
      (rc = put(q.req_feat_off, q.n_reqs + 1, &m.req_off)) || (rc = put(q.req_feat, q.req_feat_off[q.n_reqs], &m.req_feat)) ||
      (rc = put(q.m_req_off, q.n_matchers + 1, &m.m_off)) || (rc = put(q.m_req, q.m_req_off[q.n_matchers], &m.m_req)))
    return rc;
  if ((rc = upload(h, bufs, nullptr, (size_t)m.s * std::max(m.w, 1) * 4, &p))) return rc;
  m.bits = (uint32_t*)p;
  if (m.c > 0) {
    if ((rc = put(q.class_matcher, m.c, &m.cls_matcher)) || (rc = put(q.pod_sig, m.p, &m.pod_sig)) ||
        (rc = put(q.pod_node, m.p, &m.pod_node)))
      return rc;
    if ((rc = upload(h, bufs, nullptr, (size_t)m.s * m.cw * 4, &p))) return rc;
    m.cls_bits = (uint32_t*)p;
    if ((rc = upload(h, bufs, nullptr, (size_t)m.c * std::max(m.n, 1) * 4, &p))) return rc;
    m.cnt = (int32_t*)p;
  }
  HIPCHK(h, hipEventRecord(h->ev0, h->stream));
  launch_match(m, h->stream);
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipEventRecord(h->ev1, h->stream));
  if (m.w > 0)
    HIPCHK(h, hipMemcpyAsync(match_bits, m.bits, (size_t)m.s * m.w * 4, hipMemcpyDeviceToHost, h->stream));
  if (m.c > 0 && m.n > 0)
    HIPCHK(h, hipMemcpyAsync(counts, m.cnt, (size_t)m.c * m.n * 4, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  float ms = 0.f;
  HIPCHK(h, hipEventElapsedTime(&ms, h->ev0, h->ev1));
  h->match_ns = (int64_t)(ms * 1e6);
  return KSIM_OK;
}
