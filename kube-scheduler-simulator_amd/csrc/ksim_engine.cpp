// ksim_engine.cpp — host runtime behind the C ABI (include/ksim_engine.h).
//
// Owns the HBM-resident snapshot (SoA node columns, vocabularies), the pod
// queue, the per-cycle scratch, one HIP stream and a captured hipGraph of G
// back-to-back cycles that is replayed for batch runs.  Every input is
// validated on the host before any kernel sees it (a bad index must never
// reach the device), copied during the call, and never retained (cgo rule).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "ksim_internal.h"

using namespace ksim;

namespace {

constexpr int kGraphCycles = 128;   // cycles per captured graph

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

}  // namespace

struct ksim_handle {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  std::string err;

  bool has_profile = false;
  ksim_profile prof{};

  bool has_cluster = false;
  DevCluster dc{};
  std::vector<DevBuf> cluster_bufs;

  DevScratch sc{};
  DevEvalOut eo{};
  std::vector<DevBuf> scratch_bufs;

  DevState* st = nullptr;
  int32_t run_hdr[2] = {0, 0};

  // loaded pod queue (batch mode)
  DevPods dp{};
  int32_t* d_chosen = nullptr;
  std::vector<DevBuf> pod_bufs;

  // compat-mode single pod
  DevPods dp1{};
  std::vector<DevBuf> pod1_bufs;

  hipGraph_t graph = nullptr;
  hipGraphExec_t graph_exec = nullptr;
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

#define HIPCHK(h, expr)                                   \
  do {                                                    \
    hipError_t _e = (expr);                               \
    if (_e != hipSuccess) return hip_fail((h), _e, #expr); \
  } while (0)

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

void drop_graph(ksim_handle* h) {
  if (h->graph_exec) (void)hipGraphExecDestroy(h->graph_exec);
  if (h->graph) (void)hipGraphDestroy(h->graph);
  h->graph_exec = nullptr;
  h->graph = nullptr;
}

bool plugin_supported(int id) { return id >= 0 && id < KSIM_PL_COUNT; }

int validate_pod(ksim_handle* h, const ksim_pod_set* ps, int32_t i) {
  const ksim_pod& p = ps->pods[i];
  const DevCluster& c = h->dc;
  if (p.flags & (KSIM_POD_HAS_HOST_PORTS | KSIM_POD_HAS_VOLUMES))
    return set_err(h, KSIM_E_UNSUPPORTED, "pod " + std::to_string(i) + ": host ports / volumes not supported by the engine");
  if (p.node_name < -2 || p.node_name >= c.n)
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
  return KSIM_OK;
}

int ensure_ready(ksim_handle* h) {
  if (!h) return KSIM_E_INVALID;
  if (!h->has_profile) return set_err(h, KSIM_E_INVALID, "profile not set");
  if (!h->has_cluster) return set_err(h, KSIM_E_INVALID, "cluster not set");
  if (h->dc.n <= 0) return set_err(h, KSIM_E_INVALID, "no nodes available");
  return KSIM_OK;
}

LaunchArgs make_args(ksim_handle* h, const DevPods& P, int32_t* chosen) {
  LaunchArgs a;
  a.c = h->dc;
  a.P = P;
  a.prof = h->prof;
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
  if (hipSetDevice(device) != hipSuccess ||
      hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&h->ev0) != hipSuccess || hipEventCreate(&h->ev1) != hipSuccess ||
      hipMalloc(&h->st, sizeof(DevState)) != hipSuccess ||
      hipMemset(h->st, 0, sizeof(DevState)) != hipSuccess) {
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
  drop_graph(h);
  free_bufs(h->cluster_bufs);
  free_bufs(h->scratch_bufs);
  free_bufs(h->pod_bufs);
  free_bufs(h->pod1_bufs);
  if (h->d_chosen) (void)hipFree(h->d_chosen);
  if (h->st) (void)hipFree(h->st);
  if (h->ev0) (void)hipEventDestroy(h->ev0);
  if (h->ev1) (void)hipEventDestroy(h->ev1);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
}

const char* ksim_last_error(const ksim_handle* h) { return h ? h->err.c_str() : "null handle"; }

int ksim_set_profile(ksim_handle* h, const ksim_profile* p) {
  if (!h || !p) return KSIM_E_INVALID;
  if (p->n_filter < 0 || p->n_filter > KSIM_MAX_FILTER || p->n_score < 0 || p->n_score > KSIM_MAX_SCORE)
    return set_err(h, KSIM_E_INVALID, "plugin count out of range");
  for (int i = 0; i < p->n_filter; i++)
    if (!plugin_supported(p->filter[i])) return set_err(h, KSIM_E_INVALID, "unknown filter plugin id");
  for (int i = 0; i < p->n_score; i++) {
    if (!plugin_supported(p->score[i])) return set_err(h, KSIM_E_INVALID, "unknown score plugin id");
    if (p->score_weight[i] < 0) return set_err(h, KSIM_E_INVALID, "negative score weight");
  }
  if (p->fit_n_res < 0 || p->fit_n_res > KSIM_MAX_RES || p->ba_n_res < 0 || p->ba_n_res > KSIM_MAX_RES)
    return set_err(h, KSIM_E_INVALID, "scoring resources out of range");
  h->prof = *p;
  h->has_profile = true;
  drop_graph(h);
  return KSIM_OK;
}

int ksim_set_cluster(ksim_handle* h, const ksim_node_table* t, const ksim_vocab* v) {
  if (!h || !t || !v) return KSIM_E_INVALID;
  HIPCHK(h, hipSetDevice(h->device));
  const int32_t n = t->n_nodes;
  if (n < 0 || n > KSIM_MAX_NODES) return set_err(h, KSIM_E_INVALID, "n_nodes out of range");
  if (t->n_scalar < 0 || t->n_scalar > KSIM_MAX_SCALAR) return set_err(h, KSIM_E_INVALID, "n_scalar out of range");
  if (t->n_label_cols < 0 || t->n_label_cols > KSIM_MAX_LABEL_COLS)
    return set_err(h, KSIM_E_INVALID, "n_label_cols out of range");
  if (v->n_taints < 1 || v->n_taints > 64 * KSIM_TAINT_WORDS) return set_err(h, KSIM_E_INVALID, "n_taints out of range");
  if (n > 0 && (!t->alloc_cpu || !t->alloc_mem || !t->alloc_eph || !t->alloc_pods || !t->req_cpu ||
                !t->req_mem || !t->req_eph || !t->nz_cpu || !t->nz_mem || !t->num_pods || !t->flags ||
                !t->taints || (t->n_label_cols > 0 && !t->labels) ||
                (t->n_scalar > 0 && (!t->alloc_scalar || !t->req_scalar))))
    return set_err(h, KSIM_E_INVALID, "null node column");
  for (size_t i = 0; i < (size_t)n * KSIM_MAX_NODE_TAINTS; i++)
    if (t->taints[i] >= v->n_taints) return set_err(h, KSIM_E_INVALID, "taint id out of vocabulary");
  if (t->n_label_cols > 0 && (!v->label_col_offset || (v->n_label_values > 0 && (!v->label_num || !v->label_num_ok))))
    return set_err(h, KSIM_E_INVALID, "null label vocabulary");
  (void)hipStreamSynchronize(h->stream);
  drop_graph(h);
  free_bufs(h->cluster_bufs);
  free_bufs(h->scratch_bufs);
  h->has_cluster = false;

  DevCluster c{};
  c.n = n;
  c.n_scalar = t->n_scalar;
  c.n_label_cols = t->n_label_cols;
  c.n_taints = v->n_taints;
  c.n_label_values = v->n_label_values;
  const size_t N = (size_t)n;
  int rc;
#define UP(field, src, bytes)                                                       \
  do {                                                                              \
    void* _p = nullptr;                                                             \
    if ((rc = upload(h, h->cluster_bufs, (src), (bytes), &_p)) != KSIM_OK) return rc; \
    c.field = reinterpret_cast<decltype(c.field)>(_p);                              \
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
#undef UP
  h->dc = c;

  DevScratch s{};
  DevEvalOut o{};
  void* p = nullptr;
  if ((rc = upload(h, h->scratch_bufs, nullptr, N, &p))) return rc;
  s.fail = (uint8_t*)p;
  if ((rc = upload(h, h->scratch_bufs, nullptr, 4 * N, &p))) return rc;
  s.detail = (uint32_t*)p;
  if ((rc = upload(h, h->scratch_bufs, nullptr, 8 * N * KSIM_MAX_SCORE, &p))) return rc;
  s.raw = (int64_t*)p;
  if ((rc = upload(h, h->scratch_bufs, nullptr, 8 * N, &p))) return rc;
  s.part = (int64_t*)p;
  if ((rc = upload(h, h->scratch_bufs, nullptr, N, &p))) return rc;
  o.scored = (uint8_t*)p;
  if ((rc = upload(h, h->scratch_bufs, nullptr, 8 * N * KSIM_MAX_SCORE, &p))) return rc;
  o.raw = (int64_t*)p;
  if ((rc = upload(h, h->scratch_bufs, nullptr, 8 * N * KSIM_MAX_SCORE, &p))) return rc;
  o.norm = (int64_t*)p;
  if ((rc = upload(h, h->scratch_bufs, nullptr, 8 * N, &p))) return rc;
  o.total = (int64_t*)p;
  h->sc = s;
  h->eo = o;
  DevState zero{};
  HIPCHK(h, hipMemcpyAsync(h->st, &zero, sizeof(zero), hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  h->has_cluster = true;
  // a loaded pod queue was validated against the previous cluster
  free_bufs(h->pod_bufs);
  h->dp = DevPods{};
  if (h->d_chosen) (void)hipFree(h->d_chosen);
  h->d_chosen = nullptr;
  return KSIM_OK;
}

int ksim_get_node_state(ksim_handle* h, int64_t* req_cpu, int64_t* req_mem, int64_t* req_eph,
                        int64_t* nz_cpu, int64_t* nz_mem, int32_t* num_pods) {
  if (!h || !h->has_cluster) return set_err(h, KSIM_E_INVALID, "cluster not set");
  HIPCHK(h, hipSetDevice(h->device));
  const size_t N = (size_t)h->dc.n;
  HIPCHK(h, hipStreamSynchronize(h->stream));
  if (req_cpu) HIPCHK(h, hipMemcpy(req_cpu, h->dc.req_cpu, 8 * N, hipMemcpyDeviceToHost));
  if (req_mem) HIPCHK(h, hipMemcpy(req_mem, h->dc.req_mem, 8 * N, hipMemcpyDeviceToHost));
  if (req_eph) HIPCHK(h, hipMemcpy(req_eph, h->dc.req_eph, 8 * N, hipMemcpyDeviceToHost));
  if (nz_cpu) HIPCHK(h, hipMemcpy(nz_cpu, h->dc.nz_cpu, 8 * N, hipMemcpyDeviceToHost));
  if (nz_mem) HIPCHK(h, hipMemcpy(nz_mem, h->dc.nz_mem, 8 * N, hipMemcpyDeviceToHost));
  if (num_pods) HIPCHK(h, hipMemcpy(num_pods, h->dc.num_pods, 4 * N, hipMemcpyDeviceToHost));
  return KSIM_OK;
}

int ksim_get_next_start(ksim_handle* h, int32_t* next_start) {
  if (!h || !next_start) return KSIM_E_INVALID;
  HIPCHK(h, hipStreamSynchronize(h->stream));
  HIPCHK(h, hipMemcpy(next_start, &h->st->next_start, 4, hipMemcpyDeviceToHost));
  return KSIM_OK;
}

int ksim_set_next_start(ksim_handle* h, int32_t next_start) {
  if (!h) return KSIM_E_INVALID;
  if (h->has_cluster && (next_start < 0 || next_start >= std::max(h->dc.n, 1)))
    return set_err(h, KSIM_E_INVALID, "next_start out of range");
  HIPCHK(h, hipStreamSynchronize(h->stream));
  HIPCHK(h, hipMemcpy(&h->st->next_start, &next_start, 4, hipMemcpyHostToDevice));
  return KSIM_OK;
}

int ksim_set_pod_seq(ksim_handle* h, int64_t seq) {
  if (!h) return KSIM_E_INVALID;
  HIPCHK(h, hipStreamSynchronize(h->stream));
  HIPCHK(h, hipMemcpy(&h->st->pod_seq, &seq, 8, hipMemcpyHostToDevice));
  return KSIM_OK;
}

// Re-based copy of one pod with only the expressions/terms it references.
static void single_pod_set(const ksim_pod_set* ps, int32_t i, ksim_pod& pod, std::vector<ksim_label_expr>& ex,
                           std::vector<ksim_term>& tm) {
  pod = ps->pods[i];
  auto copy_expr = [&](int32_t e) { ex.push_back(ps->exprs[e]); };
  int32_t sel0 = (int32_t)ex.size();
  for (int32_t k = 0; k < pod.sel_count; k++) copy_expr(pod.sel_first + k);
  pod.sel_first = sel0;
  auto copy_terms = [&](int32_t& first, int32_t count) {
    int32_t t0 = (int32_t)tm.size();
    for (int32_t t = 0; t < count; t++) {
      ksim_term x = ps->terms[first + t];
      int32_t e0 = (int32_t)ex.size();
      for (int32_t k = 0; k < x.n_expr; k++) copy_expr(x.first_expr + k);
      x.first_expr = e0;
      tm.push_back(x);
    }
    first = t0;
  };
  copy_terms(pod.req_term_first, pod.req_term_count);
  copy_terms(pod.pref_term_first, pod.pref_term_count);
}

int ksim_eval_pod(ksim_handle* h, const ksim_pod_set* ps, int32_t pod_index, ksim_eval_out* out) {
  int rc = ensure_ready(h);
  if (rc) return rc;
  if (!ps || !out || pod_index < 0 || pod_index >= ps->n_pods || !ps->pods)
    return set_err(h, KSIM_E_INVALID, "bad pod set / index");
  if ((rc = validate_pod(h, ps, pod_index))) return rc;
  HIPCHK(h, hipSetDevice(h->device));
  ksim_pod pod;
  std::vector<ksim_label_expr> ex;
  std::vector<ksim_term> tm;
  single_pod_set(ps, pod_index, pod, ex, tm);
  HIPCHK(h, hipStreamSynchronize(h->stream));
  free_bufs(h->pod1_bufs);
  DevPods P{};
  void* p = nullptr;
  if ((rc = upload(h, h->pod1_bufs, &pod, sizeof(pod), &p))) return rc;
  P.pods = (const ksim_pod*)p;
  if ((rc = upload(h, h->pod1_bufs, ex.data(), ex.size() * sizeof(ksim_label_expr), &p))) return rc;
  P.exprs = (const ksim_label_expr*)p;
  if ((rc = upload(h, h->pod1_bufs, tm.data(), tm.size() * sizeof(ksim_term), &p))) return rc;
  P.terms = (const ksim_term*)p;
  P.n_pods = 1;
  P.n_exprs = (int32_t)ex.size();
  P.n_terms = (int32_t)tm.size();
  h->dp1 = P;
  if ((rc = set_run(h, 0, 1))) return rc;
  launch_cycle(make_args(h, P, nullptr), h->stream, true);
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipStreamSynchronize(h->stream));
  const size_t N = (size_t)h->dc.n;
  const int S = h->prof.n_score;
  if (out->fail_plugin) HIPCHK(h, hipMemcpy(out->fail_plugin, h->sc.fail, N, hipMemcpyDeviceToHost));
  if (out->fail_detail) HIPCHK(h, hipMemcpy(out->fail_detail, h->sc.detail, 4 * N, hipMemcpyDeviceToHost));
  if (out->scored) HIPCHK(h, hipMemcpy(out->scored, h->eo.scored, N, hipMemcpyDeviceToHost));
  if (out->raw && S) HIPCHK(h, hipMemcpy(out->raw, h->eo.raw, 8 * N * S, hipMemcpyDeviceToHost));
  if (out->norm && S) HIPCHK(h, hipMemcpy(out->norm, h->eo.norm, 8 * N * S, hipMemcpyDeviceToHost));
  if (out->total) HIPCHK(h, hipMemcpy(out->total, h->eo.total, 8 * N, hipMemcpyDeviceToHost));
  DevState st;
  HIPCHK(h, hipMemcpy(&st, h->st, sizeof(st), hipMemcpyDeviceToHost));
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

static int assume_common(ksim_handle* h, const ksim_pod_set* ps, int32_t pod_index, int32_t node, int sign) {
  int rc = ensure_ready(h);
  if (rc) return rc;
  if (!ps || pod_index < 0 || pod_index >= ps->n_pods || node < 0 || node >= h->dc.n)
    return set_err(h, KSIM_E_INVALID, "bad pod / node");
  HIPCHK(h, hipSetDevice(h->device));
  launch_assume(h->dc, ps->pods[pod_index], node, sign, h->stream);
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return KSIM_OK;
}

int ksim_assume(ksim_handle* h, const ksim_pod_set* ps, int32_t pod_index, int32_t node) {
  return assume_common(h, ps, pod_index, node, 1);
}

int ksim_forget(ksim_handle* h, const ksim_pod_set* ps, int32_t pod_index, int32_t node) {
  return assume_common(h, ps, pod_index, node, -1);
}

int ksim_load_pods(ksim_handle* h, const ksim_pod_set* ps) {
  int rc = ensure_ready(h);
  if (rc) return rc;
  if (!ps || ps->n_pods < 0 || (ps->n_pods > 0 && !ps->pods) || ps->n_exprs < 0 || ps->n_terms < 0)
    return set_err(h, KSIM_E_INVALID, "bad pod set");
  for (int32_t i = 0; i < ps->n_pods; i++)
    if ((rc = validate_pod(h, ps, i))) return rc;
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  drop_graph(h);
  free_bufs(h->pod_bufs);
  if (h->d_chosen) (void)hipFree(h->d_chosen);
  h->d_chosen = nullptr;
  DevPods P{};
  void* p = nullptr;
  if ((rc = upload(h, h->pod_bufs, ps->pods, sizeof(ksim_pod) * ps->n_pods, &p))) return rc;
  P.pods = (const ksim_pod*)p;
  if ((rc = upload(h, h->pod_bufs, ps->exprs, sizeof(ksim_label_expr) * ps->n_exprs, &p))) return rc;
  P.exprs = (const ksim_label_expr*)p;
  if ((rc = upload(h, h->pod_bufs, ps->terms, sizeof(ksim_term) * ps->n_terms, &p))) return rc;
  P.terms = (const ksim_term*)p;
  P.n_pods = ps->n_pods;
  P.n_exprs = ps->n_exprs;
  P.n_terms = ps->n_terms;
  HIPCHK(h, hipMalloc(&h->d_chosen, 4 * (size_t)std::max(ps->n_pods, 1)));
  HIPCHK(h, hipMemsetAsync(h->d_chosen, 0xff, 4 * (size_t)std::max(ps->n_pods, 1), h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  h->dp = P;
  return KSIM_OK;
}

static int build_graph(ksim_handle* h) {
  drop_graph(h);
  LaunchArgs a = make_args(h, h->dp, h->d_chosen);
  HIPCHK(h, hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < kGraphCycles; i++) launch_cycle(a, h->stream, false);
  hipError_t e = hipStreamEndCapture(h->stream, &h->graph);
  if (e != hipSuccess) return hip_fail(h, e, "hipStreamEndCapture");
  HIPCHK(h, hipGraphInstantiate(&h->graph_exec, h->graph, nullptr, nullptr, 0));
  return KSIM_OK;
}

int ksim_schedule_loaded(ksim_handle* h, int32_t first, int32_t count, int32_t* chosen, ksim_batch_stats* stats) {
  int rc = ensure_ready(h);
  if (rc) return rc;
  if (!h->dp.pods && count > 0) return set_err(h, KSIM_E_INVALID, "no pods loaded");
  if (first < 0 || count < 0 || first + count > h->dp.n_pods) return set_err(h, KSIM_E_INVALID, "range out of loaded pods");
  HIPCHK(h, hipSetDevice(h->device));
  if (!h->graph_exec && (rc = build_graph(h))) return rc;
  if ((rc = set_run(h, first, first + count))) return rc;
  HIPCHK(h, hipMemsetAsync(&h->st->evals, 0, 3 * sizeof(int64_t), h->stream));
  HIPCHK(h, hipEventRecord(h->ev0, h->stream));
  for (int32_t done = 0; done < count; done += kGraphCycles) HIPCHK(h, hipGraphLaunch(h->graph_exec, h->stream));
  HIPCHK(h, hipEventRecord(h->ev1, h->stream));
  HIPCHK(h, hipEventSynchronize(h->ev1));
  HIPCHK(h, hipGetLastError());
  if (chosen && count) HIPCHK(h, hipMemcpy(chosen, h->d_chosen + first, 4 * (size_t)count, hipMemcpyDeviceToHost));
  if (stats) {
    DevState st;
    HIPCHK(h, hipMemcpy(&st, h->st, sizeof(st), hipMemcpyDeviceToHost));
    float ms = 0;
    HIPCHK(h, hipEventElapsedTime(&ms, h->ev0, h->ev1));
    stats->pods = count;
    stats->scheduled = st.scheduled;
    stats->unschedulable = st.unschedulable;
    stats->evals = st.evals;
    stats->device_ms = ms;
  }
  return KSIM_OK;
}

int ksim_schedule_batch(ksim_handle* h, const ksim_pod_set* ps, int32_t* chosen, ksim_batch_stats* stats) {
  int rc = ksim_load_pods(h, ps);
  if (rc) return rc;
  return ksim_schedule_loaded(h, 0, ps->n_pods, chosen, stats);
}

}  // extern "C"
