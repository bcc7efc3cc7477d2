/*
 * ksim_oracle.c — CPU restatement (ORACLE) of the per-pod scheduling cycle.
 *
 * TEST INFRASTRUCTURE ONLY (see ksim_oracle.h): the checker for the HIP engine
 * and the CPU baseline timed by bench.py.  Never linked by libksim_engine.so.
 *
 * Every function names the upstream k8s.io/kubernetes v1.26.2 function it
 * restates ([upstream] path, absent from /root/reference; pinned at
 * simulator/go.mod:53) and the SURVEY.md §8(a) row it covers.  Simulator-side
 * behaviour cites /root/reference files directly.
 *
 * Build: gcc -O2 -fPIC -shared -fopenmp -ffp-contract=off (oracle/Makefile).
 * -ffp-contract=off matches Go on GOAMD64=v1 (simulator/Dockerfile:1 golang:1.19),
 * which never fuses float64 multiply-add.
 */
#include "ksim_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define MAX_NODE_SCORE 100   /* framework.MaxNodeScore */
#define MIN_NODE_SCORE 0     /* framework.MinNodeScore */
#define MIN_FEASIBLE_NODES_TO_FIND 100            /* schedule_one.go minFeasibleNodesToFind */
#define MIN_FEASIBLE_NODES_PERCENTAGE_TO_FIND 5   /* schedule_one.go minFeasibleNodesPercentageToFind */

#define ORACLE_MAX_THREADS 256

struct ksim_oracle {
  /* ksim_oracle_schedule's per-thread partials (one cache line apart) */
  int32_t th_cnt[ORACLE_MAX_THREADS * 16], th_err[ORACLE_MAX_THREADS * 16], th_pre[ORACLE_MAX_THREADS * 16];
  int32_t th_node[ORACLE_MAX_THREADS * 16], th_stop;
  int64_t th_mn[ORACLE_MAX_THREADS * 8], th_mx[ORACLE_MAX_THREADS * 8];
  uint64_t th_lo[ORACLE_MAX_THREADS * 8];
  int64_t th_ext[ORACLE_MAX_THREADS * 2 * KSIM_MAX_SCORE];
  ksim_profile prof;
  int32_t n, n_scalar, n_label_cols;
  /* static node columns */
  int64_t *alloc_cpu, *alloc_mem, *alloc_eph, *alloc_scalar;
  int32_t *alloc_pods;
  uint32_t *flags;
  uint16_t *taints;
  uint32_t *labels;
  /* dynamic node columns (NodeInfo.Requested / NonZeroRequested / Pods) */
  int64_t *req_cpu, *req_mem, *req_eph, *req_scalar, *nz_cpu, *nz_mem;
  int32_t *num_pods;
  /* vocab */
  int32_t n_taints, n_label_values;
  uint8_t *taint_effect;
  int32_t *label_col_offset;
  int64_t *label_num;
  uint8_t *label_num_ok;
  /* PodTopologySpread / InterPodAffinity count classes (ksim_engine.h) */
  int32_t n_classes;
  int32_t *cnt;         /* [n_classes][n] dynamic */
  int32_t n_topo_log;
  double *topo_log;
  int32_t *col_nvals;   /* value ids per label column */
  int32_t vmax;
  /* NetworkBandwidth: node limit (static) and allocated amount (dynamic), milli-units */
  int64_t *nb_limit, *nb_alloc;
  /* the dynamic columns as given at create / upsert (ksim_oracle_upsert_nodes) */
  int64_t *s_req_cpu, *s_req_mem, *s_req_eph, *s_req_scalar, *s_nz_cpu, *s_nz_mem, *s_nb_alloc;
  int32_t *s_num_pods, *s_cnt;
  /* scheduler state */
  int32_t next_start;   /* sched.nextStartNodeIndex */
  int64_t pod_seq;      /* tie-break sequence */
  /* scratch */
  uint8_t *fail;
  uint32_t *detail;
  int32_t *flist;
  int64_t *raw;         /* [KSIM_MAX_SCORE][n] */
  int64_t *dom;         /* [KSIM_MAX_USES][vmax] topology-pair sums */
  uint8_t *present;     /* [KSIM_MAX_USES][vmax] pair present (PTS) / registered (PTS soft) */
  uint8_t *ignored;     /* [n] PTS IgnoredNodes */
  /* framework-driven compat mode (ksim_oracle_fw_*): the PreFilter state of
   * the pod in flight and the PreScore facts NormalizeScore reads */
  struct topo_ctx *fw_tc;
  int fw_active, fw_scored;
};

/* ------------------------------------------------------------------------ */
static void* dupbuf(const void* src, size_t bytes) {
  void* p = malloc(bytes ? bytes : 1);
  if (p && src && bytes) memcpy(p, src, bytes);
  else if (p) memset(p, 0, bytes ? bytes : 1);
  return p;
}

ksim_oracle* ksim_oracle_create(const ksim_node_table* t, const ksim_vocab* v,
                                const ksim_profile* prof) {
  if (!t || !v || !prof || t->n_nodes < 0 || t->n_nodes > KSIM_MAX_NODES) return NULL;
  ksim_oracle* o = (ksim_oracle*)calloc(1, sizeof(*o));
  size_t n = (size_t)t->n_nodes;
  o->prof = *prof;
  o->n = t->n_nodes;
  o->n_scalar = t->n_scalar;
  o->n_label_cols = t->n_label_cols;
  o->alloc_cpu = dupbuf(t->alloc_cpu, n * 8);
  o->alloc_mem = dupbuf(t->alloc_mem, n * 8);
  o->alloc_eph = dupbuf(t->alloc_eph, n * 8);
  o->alloc_pods = dupbuf(t->alloc_pods, n * 4);
  o->alloc_scalar = dupbuf(t->alloc_scalar, n * 8 * (size_t)t->n_scalar);
  o->req_cpu = dupbuf(t->req_cpu, n * 8);
  o->req_mem = dupbuf(t->req_mem, n * 8);
  o->req_eph = dupbuf(t->req_eph, n * 8);
  o->req_scalar = dupbuf(t->req_scalar, n * 8 * (size_t)t->n_scalar);
  o->nz_cpu = dupbuf(t->nz_cpu, n * 8);
  o->nz_mem = dupbuf(t->nz_mem, n * 8);
  o->num_pods = dupbuf(t->num_pods, n * 4);
  o->flags = dupbuf(t->flags, n * 4);
  o->taints = dupbuf(t->taints, n * 2 * KSIM_MAX_NODE_TAINTS);
  o->labels = dupbuf(t->labels, n * 4 * (size_t)t->n_label_cols);
  o->n_taints = v->n_taints;
  o->n_label_values = v->n_label_values;
  o->taint_effect = dupbuf(v->taint_effect, (size_t)v->n_taints);
  o->label_col_offset = dupbuf(v->label_col_offset, 4 * (size_t)t->n_label_cols);
  o->label_num = dupbuf(v->label_num, 8 * (size_t)v->n_label_values);
  o->label_num_ok = dupbuf(v->label_num_ok, (size_t)v->n_label_values);
  o->fail = malloc(n + 1);
  o->detail = malloc(4 * n + 4);
  o->flist = malloc(4 * n + 4);
  o->raw = malloc(8 * n * KSIM_MAX_SCORE + 8);
  o->n_classes = t->n_classes;
  o->cnt = dupbuf(t->class_count, 4 * n * (size_t)(t->n_classes > 0 ? t->n_classes : 0));
  o->n_topo_log = v->n_topo_log;
  o->topo_log = dupbuf(v->topo_log, 8 * (size_t)(v->n_topo_log > 0 ? v->n_topo_log : 0));
  o->col_nvals = malloc(4 * (size_t)t->n_label_cols + 4);
  o->vmax = 1;
  for (int k = 0; k < t->n_label_cols; k++) {
    int32_t end = (k + 1 < t->n_label_cols) ? v->label_col_offset[k + 1] : v->n_label_values;
    o->col_nvals[k] = end - v->label_col_offset[k];
    if (o->col_nvals[k] > o->vmax) o->vmax = o->col_nvals[k];
  }
  o->dom = malloc(8 * (size_t)KSIM_MAX_USES * o->vmax);
  o->present = malloc((size_t)KSIM_MAX_USES * o->vmax);
  o->ignored = malloc(n + 1);
  o->nb_limit = dupbuf(t->nb_limit, n * 8);
  o->nb_alloc = dupbuf(t->nb_alloc, n * 8);
  o->s_req_cpu = dupbuf(o->req_cpu, n * 8);
  o->s_req_mem = dupbuf(o->req_mem, n * 8);
  o->s_req_eph = dupbuf(o->req_eph, n * 8);
  o->s_req_scalar = dupbuf(o->req_scalar, n * 8 * (size_t)t->n_scalar);
  o->s_nz_cpu = dupbuf(o->nz_cpu, n * 8);
  o->s_nz_mem = dupbuf(o->nz_mem, n * 8);
  o->s_nb_alloc = dupbuf(o->nb_alloc, n * 8);
  o->s_num_pods = dupbuf(o->num_pods, n * 4);
  o->s_cnt = dupbuf(o->cnt, 4 * n * (size_t)(t->n_classes > 0 ? t->n_classes : 0));
  return o;
}

void ksim_oracle_destroy(ksim_oracle* o) {
  if (!o) return;
  void* ps[] = {o->alloc_cpu, o->alloc_mem, o->alloc_eph, o->alloc_pods, o->alloc_scalar,
                o->req_cpu, o->req_mem, o->req_eph, o->req_scalar, o->nz_cpu, o->nz_mem,
                o->num_pods, o->flags, o->taints, o->labels, o->taint_effect,
                o->label_col_offset, o->label_num, o->label_num_ok, o->fail, o->detail,
                o->flist, o->raw, o->cnt, o->topo_log, o->col_nvals, o->dom, o->present,
                o->ignored, o->nb_limit, o->nb_alloc, o->s_req_cpu, o->s_req_mem, o->s_req_eph,
                o->s_req_scalar, o->s_nz_cpu, o->s_nz_mem, o->s_nb_alloc, o->s_num_pods, o->s_cnt, o->fw_tc};
  for (size_t i = 0; i < sizeof(ps) / sizeof(ps[0]); i++) free(ps[i]);
  free(o);
}

/* Node informer deltas (ksim_engine.h ksim_upsert_nodes): the table is the
 * new snapshot; on a kept node the binds since the last snapshot (live -
 * snapshot at old_pos) are replayed on top of it for the scalar columns /
 * classes the oracle already has.  nextStartNodeIndex mod the new node count,
 * the pod sequence carries over. */
#define REPLAY(T, out, live, snap, tab, rows, rows0)                                    \
  do {                                                                                 \
    out = (T*)malloc(sizeof(T) * n * (size_t)(rows) + sizeof(T));                      \
    for (int k = 0; k < (rows); k++)                                                   \
      for (size_t i = 0; i < n; i++) {                                                 \
        T x = (tab) ? (tab)[k * n + i] : 0;                                            \
        if (k < (rows0) && old_pos[i] >= 0)                                            \
          x += (live)[k * n0 + (size_t)old_pos[i]] - (snap)[k * n0 + (size_t)old_pos[i]]; \
        out[k * n + i] = x;                                                            \
      }                                                                                \
  } while (0)

int ksim_oracle_upsert_nodes(ksim_oracle* o, const ksim_node_table* t, const ksim_vocab* v,
                             const int32_t* old_pos) {
  if (!o || !t || !v || t->n_nodes < 0 || t->n_nodes > KSIM_MAX_NODES) return -1;
  if (t->n_scalar < o->n_scalar || t->n_classes < o->n_classes || (t->n_nodes > 0 && !old_pos)) return -1;
  const size_t n = (size_t)t->n_nodes, n0 = (size_t)o->n;
  for (size_t i = 0; i < n; i++)
    if (old_pos[i] < -1 || old_pos[i] >= o->n) return -1;
  ksim_oracle* q = ksim_oracle_create(t, v, &o->prof);     /* snapshot = the table */
  if (!q) return -1;
  int64_t *rc, *rm, *re, *zc, *zm, *nb, *rs;
  int32_t *np, *cnt;
  REPLAY(int64_t, rc, o->req_cpu, o->s_req_cpu, t->req_cpu, 1, 1);
  REPLAY(int64_t, rm, o->req_mem, o->s_req_mem, t->req_mem, 1, 1);
  REPLAY(int64_t, re, o->req_eph, o->s_req_eph, t->req_eph, 1, 1);
  REPLAY(int64_t, zc, o->nz_cpu, o->s_nz_cpu, t->nz_cpu, 1, 1);
  REPLAY(int64_t, zm, o->nz_mem, o->s_nz_mem, t->nz_mem, 1, 1);
  REPLAY(int64_t, nb, o->nb_alloc, o->s_nb_alloc, t->nb_alloc, 1, 1);
  REPLAY(int64_t, rs, o->req_scalar, o->s_req_scalar, t->req_scalar, t->n_scalar, o->n_scalar);
  REPLAY(int32_t, np, o->num_pods, o->s_num_pods, t->num_pods, 1, 1);
  REPLAY(int32_t, cnt, o->cnt, o->s_cnt, t->class_count, t->n_classes, o->n_classes);
  free(q->req_cpu); q->req_cpu = rc;
  free(q->req_mem); q->req_mem = rm;
  free(q->req_eph); q->req_eph = re;
  free(q->nz_cpu); q->nz_cpu = zc;
  free(q->nz_mem); q->nz_mem = zm;
  free(q->nb_alloc); q->nb_alloc = nb;
  free(q->req_scalar); q->req_scalar = rs;
  free(q->num_pods); q->num_pods = np;
  free(q->cnt); q->cnt = cnt;
  q->next_start = n > 0 ? o->next_start % (int32_t)n : 0;
  q->pod_seq = o->pod_seq;   /* a framework cycle in flight does not survive a node delta */
  ksim_oracle swap = *o;
  *o = *q;
  *q = swap;
  ksim_oracle_destroy(q);
  return 0;
}
#undef REPLAY

/* ---- tie-break TB(seed), SURVEY §8(b) "Determinism modes" ---------------- */
static uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* selectHost picks the max of (total, lo) in lexicographic order, total the
 * full int64; lo = hash26<<18 | (2^18-1-node).  This replaces the reservoir
 * sampling of [upstream] schedule_one.go selectHost (global math/rand). */
uint64_t ksim_oracle_tb_lo(uint64_t seed, int64_t pod_seq, int32_t node) {
  uint64_t h = splitmix64(seed ^ ((uint64_t)pod_seq << 20) ^ (uint64_t)(uint32_t)node) >> 38;
  return (h << 18) | (uint64_t)(KSIM_KEY_NODE_MASK - node);
}

/* The same order packed into one u64 for a total in [0, 2^20): total<<44 | lo. */
uint64_t ksim_oracle_tb_key(int64_t total, uint64_t seed, int64_t pod_seq, int32_t node) {
  return ((uint64_t)total << 44) | ksim_oracle_tb_lo(seed, pod_seq, node);
}

/* (total, lo) > (best_total, best_lo) */
static int tb_better(int64_t total, uint64_t lo, int64_t best_total, uint64_t best_lo) {
  return total > best_total || (total == best_total && lo > best_lo);
}

/* The nodes findNodesThatFitPod scans (a16): every node, or NodeAffinity's
 * PreFilterResult.NodeNames (a5: ksim_engine.h KSIM_POD_NODE_NAMES), in
 * increasing position from nextStartNodeIndex mod their count. */
typedef struct scan_set {
  const int32_t* list;   /* NULL: every node */
  int32_t n, start;
} scan_set;

static scan_set pod_scan_set(const ksim_oracle* o, const ksim_pod_set* ps, const ksim_pod* p) {
  scan_set s;
  s.list = NULL;
  s.n = o->n;
  if (p->flags & KSIM_POD_NODE_NAMES) {
    s.list = ps->nn + p->nn_first;
    s.n = (p->flags & KSIM_POD_NODE_NAMES_UNKNOWN) ? 0 : p->nn_count;
  }
  s.start = s.n > 0 ? o->next_start % s.n : 0;
  return s;
}

static int32_t scan_node_at(const scan_set* s, int32_t i) {
  const int32_t x = (s->start + i) % s->n;
  return s->list ? s->list[x] : x;
}

/* [upstream] schedule_one.go (*Scheduler).numFeasibleNodesToFind — §8(a) a16 */
int32_t ksim_oracle_num_feasible_nodes_to_find(int32_t percentage, int32_t num_all_nodes) {
  if (num_all_nodes < MIN_FEASIBLE_NODES_TO_FIND || percentage >= 100) return num_all_nodes;
  int32_t adaptive = percentage;
  if (adaptive <= 0) {
    adaptive = 50 - num_all_nodes / 125;
    if (adaptive < MIN_FEASIBLE_NODES_PERCENTAGE_TO_FIND) adaptive = MIN_FEASIBLE_NODES_PERCENTAGE_TO_FIND;
  }
  int32_t num = num_all_nodes * adaptive / 100;
  if (num < MIN_FEASIBLE_NODES_TO_FIND) return MIN_FEASIBLE_NODES_TO_FIND;
  return num;
}

/* ---- NodeAffinity (component-helpers nodeaffinity + apimachinery labels) - */
static inline uint32_t node_label(const ksim_oracle* o, int col, int32_t node) {
  return o->labels[(size_t)col * o->n + node];
}

/* labels.Requirement.Matches / fields selector for metadata.name — §8(a) a26 */
static int label_req_matches(const ksim_oracle* o, const ksim_label_expr* e, int32_t node) {
  uint32_t v = (e->op <= KSIM_OP_LT) ? node_label(o, e->col, node) : 0;
  switch (e->op) {
    case KSIM_OP_IN:
      if (!v) return 0;
      for (int k = 0; k < e->nvals; k++) if (e->vals[k] == v) return 1;
      return 0;
    case KSIM_OP_NOT_IN:
      if (!v) return 1;
      for (int k = 0; k < e->nvals; k++) if (e->vals[k] == v) return 0;
      return 1;
    case KSIM_OP_EXISTS: return v != 0;
    case KSIM_OP_DOES_NOT_EXIST: return v == 0;
    case KSIM_OP_GT:
    case KSIM_OP_LT: {
      if (!v) return 0;
      int32_t idx = o->label_col_offset[e->col] + (int32_t)v;
      if (idx < 0 || idx >= o->n_label_values || !o->label_num_ok[idx]) return 0;
      return e->op == KSIM_OP_GT ? (o->label_num[idx] > e->num) : (o->label_num[idx] < e->num);
    }
    case KSIM_OP_FIELD_IN:
      for (int k = 0; k < e->nvals; k++) if ((int32_t)e->vals[k] == node) return 1;
      return 0;
    case KSIM_OP_FIELD_NOT_IN:
      for (int k = 0; k < e->nvals; k++) if ((int32_t)e->vals[k] == node) return 0;
      return 1;
    case KSIM_OP_TRUE: return 1;
    default: return 0;
  }
}

/* nodeSelectorTerm.match: empty term matches nothing; AND of requirements. */
static int term_matches(const ksim_oracle* o, const ksim_pod_set* ps, const ksim_term* t,
                        int32_t node) {
  if (t->n_expr <= 0) return 0;
  for (int i = 0; i < t->n_expr; i++)
    if (!label_req_matches(o, &ps->exprs[t->first_expr + i], node)) return 0;
  return 1;
}

/* VolumeBinding (binder.go checkBoundClaims -> volumeutil.CheckNodeAffinity,
 * one group per bound PV with required node affinity) and VolumeZone
 * (volume_zone.go Filter, one group per PV topology label): every group of
 * terms [first, first + count) (ksim_term.weight = group index) has a
 * matching term.  The groups are compiled by ksim/encode.py (see the header). */
static int volume_groups_match(const ksim_oracle* o, const ksim_pod_set* ps, int32_t first, int32_t count,
                               int32_t node) {
  int32_t group = -1;
  int ok = 1;
  for (int32_t i = 0; i < count; i++) {
    const ksim_term* t = &ps->terms[first + i];
    if (t->weight != group) {
      if (!ok) return 0;
      group = t->weight;
      ok = 0;
    }
    if (!ok && term_matches(o, ps, t, node)) ok = 1;
  }
  return ok;
}

/* VolumeBinding: KSIM_VB_NODE_CONFLICT if a bound-PV group fails,
 * KSIM_VB_BIND_CONFLICT if an unbound-claim group (group index with
 * KSIM_VB_UNBOUND_GROUP) fails -- FindPodVolumes' reasons; 0 = pass. */
static uint32_t volume_binding_fails(const ksim_oracle* o, const ksim_pod_set* ps, int32_t first, int32_t count,
                                     int32_t node) {
  uint32_t why = 0;
  int32_t i = 0;
  while (i < count) {
    const int32_t g = ps->terms[first + i].weight;
    int ok = 0;
    for (; i < count && ps->terms[first + i].weight == g; i++)
      if (!ok && term_matches(o, ps, &ps->terms[first + i], node)) ok = 1;
    if (!ok) why |= (g & KSIM_VB_UNBOUND_GROUP) ? KSIM_VB_BIND_CONFLICT : KSIM_VB_NODE_CONFLICT;
  }
  return why;
}

/* RequiredNodeAffinity.Match: nodeSelector (labels.SelectorFromSet) AND
 * (OR of required terms) — [upstream] nodeaffinity.Filter, §8(a) a26 */
static int required_node_affinity_match(const ksim_oracle* o, const ksim_pod_set* ps,
                                        const ksim_pod* p, int32_t node) {
  for (int i = 0; i < p->sel_count; i++)
    if (!label_req_matches(o, &ps->exprs[p->sel_first + i], node)) return 0;
  if (p->flags & KSIM_POD_HAS_REQUIRED_AFFINITY) {
    for (int i = 0; i < p->req_term_count; i++)
      if (term_matches(o, ps, &ps->terms[p->req_term_first + i], node)) return 1;
    return 0;
  }
  return 1;
}

/* nodeaffinity.NodeAffinity.Filter (v1.26): the profile's addedAffinity
 * (NodeAffinityArgs, addedNodeSelector.Match) first -> errReasonEnforced,
 * then the pod's RequiredNodeAffinity -> ErrReasonPod.  Returns 1 on pass. */
static int node_affinity_filter(const ksim_oracle* o, const ksim_pod_set* ps, const ksim_pod* p, int32_t node,
                                uint32_t* detail) {
  *detail = 0;
  if (p->flags & KSIM_POD_ADDED_AFFINITY) {
    int any = 0;
    for (int i = 0; i < p->added_term_count && !any; i++)
      any = term_matches(o, ps, &ps->terms[p->added_term_first + i], node);
    if (!any) {
      *detail = KSIM_NA_ENFORCED;
      return 0;
    }
  }
  return required_node_affinity_match(o, ps, p, node);
}

/* PreferredSchedulingTerms.Score — [upstream] nodeaffinity.Score */
static int64_t preferred_node_affinity_score(const ksim_oracle* o, const ksim_pod_set* ps,
                                             const ksim_pod* p, int32_t node) {
  int64_t count = 0;
  for (int i = 0; i < p->pref_term_count; i++) {
    const ksim_term* t = &ps->terms[p->pref_term_first + i];
    if (t->weight == 0) continue;
    if (term_matches(o, ps, t, node)) count += t->weight;
  }
  return count;
}

/* ---- TaintToleration ---------------------------------------------------- */
static inline int bit_set(const uint64_t* w, uint32_t id) {
  return (int)((w[id >> 6] >> (id & 63)) & 1u);
}

/* v1helper.FindMatchingUntoleratedTaint with DoNotScheduleTaintsFilterFunc —
 * [upstream] tainttoleration.Filter, §8(a) a25.  Returns taint id or 0. */
static uint32_t find_matching_untolerated_taint(const ksim_oracle* o, const ksim_pod* p,
                                                int32_t node) {
  for (int k = 0; k < KSIM_MAX_NODE_TAINTS; k++) {
    uint32_t tid = o->taints[(size_t)k * o->n + node];
    if (!tid) break;
    uint8_t eff = o->taint_effect[tid];
    if ((eff == KSIM_EFFECT_NO_SCHEDULE || eff == KSIM_EFFECT_NO_EXECUTE) &&
        !bit_set(p->tol_filter, tid))
      return tid;
  }
  return 0;
}

/* countIntolerableTaintsPreferNoSchedule — [upstream] tainttoleration.Score */
static int64_t count_intolerable_prefer_no_schedule(const ksim_oracle* o, const ksim_pod* p,
                                                    int32_t node) {
  int64_t c = 0;
  for (int k = 0; k < KSIM_MAX_NODE_TAINTS; k++) {
    uint32_t tid = o->taints[(size_t)k * o->n + node];
    if (!tid) break;
    if (o->taint_effect[tid] != KSIM_EFFECT_PREFER_NO_SCHEDULE) continue;
    if (!bit_set(p->tol_prefer, tid)) c++;
  }
  return c;
}

/* ---- NodeResourcesFit --------------------------------------------------- */
/* fitsRequest — [upstream] noderesources/fit.go, §8(a) a22.  Reason bits in
 * the order upstream appends them (pods, cpu, memory, ephemeral, scalars). */
static uint32_t fits_request(const ksim_oracle* o, const ksim_pod* p, int32_t node) {
  uint32_t r = 0;
  if (o->num_pods[node] + 1 > o->alloc_pods[node]) r |= KSIM_FIT_TOO_MANY_PODS;
  if (p->req_cpu == 0 && p->req_mem == 0 && p->req_eph == 0 && !(p->flags & KSIM_POD_HAS_SCALAR))
    return r;
  if (p->req_cpu > o->alloc_cpu[node] - o->req_cpu[node]) r |= KSIM_FIT_CPU;
  if (p->req_mem > o->alloc_mem[node] - o->req_mem[node]) r |= KSIM_FIT_MEMORY;
  if (p->req_eph > o->alloc_eph[node] - o->req_eph[node]) r |= KSIM_FIT_EPHEMERAL;
  for (int k = 0; k < o->n_scalar; k++) {
    int64_t q = p->scalar_req[k];
    if (q == 0) continue;
    /* NodeResourcesFitArgs ignoredResources / ignoredResourceGroups (extended resources) */
    if ((o->prof.fit_ignored_scalar >> k) & 1u) continue;
    size_t ix = (size_t)k * o->n + node;
    if (q > o->alloc_scalar[ix] - o->req_scalar[ix]) r |= (KSIM_FIT_SCALAR0 << k);
  }
  return r;
}

/* resourceAllocationScorer.calculateResourceAllocatableRequest — a23/a24.
 * use_requested: BalancedAllocation (true) vs Fit LeastAllocated (false). */
static void calc_alloc_req(const ksim_oracle* o, const ksim_pod* p, int32_t node, int32_t res,
                           int use_requested, int64_t* alloc, int64_t* req) {
  *alloc = 0; *req = 0;
  switch (res) {
    case KSIM_RES_CPU: {
      int64_t pr = use_requested ? p->req_cpu : p->nz_cpu;
      *alloc = o->alloc_cpu[node];
      *req = (use_requested ? o->req_cpu[node] : o->nz_cpu[node]) + pr;
      return;
    }
    case KSIM_RES_MEMORY: {
      int64_t pr = use_requested ? p->req_mem : p->nz_mem;
      *alloc = o->alloc_mem[node];
      *req = (use_requested ? o->req_mem[node] : o->nz_mem[node]) + pr;
      return;
    }
    case KSIM_RES_EPHEMERAL:
      *alloc = o->alloc_eph[node];
      *req = o->req_eph[node] + p->req_eph;   /* always nodeInfo.Requested */
      return;
    default: {
      int k = res - KSIM_RES_SCALAR0;
      if (k < 0 || k >= o->n_scalar) return;
      int64_t pr = p->scalar_req[k];
      if (pr == 0) return;                    /* scalar not requested: bypass */
      size_t ix = (size_t)k * o->n + node;
      *alloc = o->alloc_scalar[ix];
      *req = o->req_scalar[ix] + pr;
      return;
    }
  }
}

/* leastRequestedScore — [upstream] noderesources/least_allocated.go */
int64_t ksim_oracle_least_requested_score(int64_t requested, int64_t capacity) {
  if (capacity == 0) return 0;
  if (requested > capacity) return 0;
  /* Go's int64 product wraps (capacities past 2^56); C's signed one must not overflow */
  const int64_t prod = (int64_t)((uint64_t)(capacity - requested) * (uint64_t)MAX_NODE_SCORE);
  return prod / capacity;
}

/* mostRequestedScore — [upstream] noderesources/most_allocated.go */
int64_t ksim_oracle_most_requested_score(int64_t requested, int64_t capacity) {
  if (capacity == 0) return 0;
  if (requested > capacity) requested = capacity;   /* pods with no requests get minimum values */
  const int64_t prod = (int64_t)((uint64_t)requested * (uint64_t)MAX_NODE_SCORE);
  return prod / capacity;
}

/* helper.BuildBrokenLinearFunction (scores already x MaxNodeScore / MaxCustomPriorityScore) */
int64_t ksim_oracle_broken_linear(const ksim_profile* prof, int64_t p) {
  for (int i = 0; i < prof->fit_n_shape; i++) {
    if (p <= prof->fit_shape_util[i]) {
      if (i == 0) return prof->fit_shape_score[0];
      const int64_t s0 = prof->fit_shape_score[i - 1], s1 = prof->fit_shape_score[i];
      const int64_t u0 = prof->fit_shape_util[i - 1], u1 = prof->fit_shape_util[i];
      return s0 + (s1 - s0) * (p - u0) / (u1 - u0);
    }
  }
  return prof->fit_shape_score[prof->fit_n_shape - 1];
}

/* requested_to_capacity_ratio.go buildRequestedToCapacityRatioScorerFunction's
 * resourceScoringFunction (maxUtilization = 100) */
static int64_t rtcr_resource_score(const ksim_profile* prof, int64_t requested, int64_t capacity) {
  if (capacity == 0 || requested > capacity) return ksim_oracle_broken_linear(prof, 100);
  const int64_t prod = (int64_t)((uint64_t)requested * 100u);
  return ksim_oracle_broken_linear(prof, prod / capacity);
}

/* NodeResourcesFit.Score: resourceAllocationScorer.score with the profile's
 * ScoringStrategy (leastResourceScorer / mostResourceScorer /
 * requestedToCapacityRatioScorer) — a23 */
static int64_t fit_score(const ksim_oracle* o, const ksim_pod* p, int32_t node) {
  const ksim_profile* prof = &o->prof;
  int64_t node_score = 0, weight_sum = 0;
  for (int i = 0; i < prof->fit_n_res; i++) {
    int64_t a, r;
    calc_alloc_req(o, p, node, prof->fit_res[i], 0, &a, &r);
    if (a == 0) continue;                      /* only non-zero allocatable enters the map */
    const int64_t w = prof->fit_res_weight[i];
    switch (prof->fit_strategy) {
      case KSIM_FIT_MOST_ALLOCATED:
        node_score += ksim_oracle_most_requested_score(r, a) * w;
        weight_sum += w;
        break;
      case KSIM_FIT_REQUESTED_TO_CAPACITY_RATIO: {
        const int64_t rs = rtcr_resource_score(prof, r, a);
        if (rs > 0) {
          node_score += rs * w;
          weight_sum += w;
        }
        break;
      }
      default:
        node_score += ksim_oracle_least_requested_score(r, a) * w;
        weight_sum += w;
        break;
    }
  }
  if (weight_sum == 0) return 0;
  if (prof->fit_strategy == KSIM_FIT_REQUESTED_TO_CAPACITY_RATIO)
    return (int64_t)round((double)node_score / (double)weight_sum);   /* math.Round: half away from zero */
  return node_score / weight_sum;
}

/* balancedResourceScorer — [upstream] noderesources/balanced_allocation.go, a24 */
int64_t ksim_oracle_balanced_score(int32_t n, const int64_t* requested, const int64_t* allocatable) {
  double fr[KSIM_MAX_RES];
  int nf = 0;
  double total = 0;
  for (int i = 0; i < n && i < KSIM_MAX_RES; i++) {
    if (allocatable[i] == 0) continue;
    double f = (double)requested[i] / (double)allocatable[i];
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
  return (int64_t)((1 - std) * (double)MAX_NODE_SCORE);
}

static int64_t balanced_allocation_score(const ksim_oracle* o, const ksim_pod* p, int32_t node) {
  int64_t req[KSIM_MAX_RES], alloc[KSIM_MAX_RES];
  int m = 0;
  for (int i = 0; i < o->prof.ba_n_res && i < KSIM_MAX_RES; i++) {
    int64_t a, r;
    calc_alloc_req(o, p, node, o->prof.ba_res[i], 1, &a, &r);
    if (a == 0) continue;
    alloc[m] = a; req[m] = r; m++;
  }
  return ksim_oracle_balanced_score(m, req, alloc);
}

/* ---- helper.DefaultNormalizeScore — a31 ---------------------------------- */
void ksim_oracle_default_normalize(int64_t max_priority, int reverse, int32_t n, int64_t* s) {
  int64_t max_count = 0;
  for (int i = 0; i < n; i++) if (s[i] > max_count) max_count = s[i];
  if (max_count == 0) {
    if (reverse) for (int i = 0; i < n; i++) s[i] = max_priority;
    return;
  }
  for (int i = 0; i < n; i++) {
    int64_t v = max_priority * s[i] / max_count;
    if (reverse) v = max_priority - v;
    s[i] = v;
  }
}

/* ---- PodTopologySpread / InterPodAffinity (a27-a30) ---------------------- */
/* The host compiled every selector / term into count classes (ksim_engine.h
 * "Count classes"); upstream's topology-pair maps become arrays indexed by the
 * label value id of the use's key column:  pair (key, value) -> dom[u][value]. */
typedef struct topo_ctx {
  int n;                                 /* uses of the pod */
  const ksim_topo_use* u[KSIM_MAX_USES];
  int64_t min_match[KSIM_MAX_USES];      /* PTS hard: TpKeyToCriticalPaths[key][0].MatchNum */
  double weight[KSIM_MAX_USES];          /* PTS soft: TopologyNormalizingWeight */
  int has_hard, has_soft, has_ipa_filter, has_ipa_score;
  int affinity_counts_empty;             /* len(state.affinityCounts) == 0 */
  int topology_score_empty;              /* len(state.topologyScore) == 0 */
} topo_ctx;

static inline int64_t* dom_of(const ksim_oracle* o, int u) { return o->dom + (size_t)u * o->vmax; }
static inline uint8_t* present_of(const ksim_oracle* o, int u) { return o->present + (size_t)u * o->vmax; }

static inline uint32_t use_value(const ksim_oracle* o, const ksim_topo_use* u, int32_t node) {
  return u->col == KSIM_COL_NONE ? 0u : node_label(o, u->col, node);   /* 0 = key absent */
}
static inline int64_t class_count(const ksim_oracle* o, int32_t cls, int32_t node) {
  return cls < 0 ? 0 : o->cnt[(size_t)cls * o->n + node];
}

/* nodeports fitsPorts: HostPortInfo.CheckConflict(ip, protocol, port) of each
 * wanted port; the host compiled each check to the classes of pods holding a
 * conflicting (ip, protocol, port) on a node (0.0.0.0 conflicts with every ip). */
static int node_port_conflict(const ksim_oracle* o, const ksim_pod_set* ps, const ksim_pod* p, int32_t node) {
  for (int32_t i = 0; i < p->use_count; i++) {
    const ksim_topo_use* u = &ps->uses[p->use_first + i];
    if (u->kind == KSIM_USE_NODE_PORT && class_count(o, u->cls, node) > 0) return 1;
  }
  return 0;
}

static int required_node_affinity_match(const ksim_oracle* o, const ksim_pod_set* ps,
                                        const ksim_pod* p, int32_t node);
static uint32_t find_matching_untolerated_taint(const ksim_oracle* o, const ksim_pod* p, int32_t node);

/* topologySpreadConstraint.matchNodeInclusionPolicies */
static int match_node_inclusion_policies(const ksim_oracle* o, const ksim_pod_set* ps, const ksim_pod* p,
                                         const ksim_topo_use* u, int32_t node) {
  if ((u->flags & KSIM_USEF_HONOR_AFFINITY) && !required_node_affinity_match(o, ps, p, node)) return 0;
  if ((u->flags & KSIM_USEF_HONOR_TAINTS) && find_matching_untolerated_taint(o, p, node)) return 0;
  return 1;
}

/* nodeLabelsMatchSpreadConstraints over the uses of one kind */
static int node_has_all_keys(const ksim_oracle* o, const topo_ctx* t, int kind, int32_t node) {
  for (int i = 0; i < t->n; i++)
    if (t->u[i]->kind == kind && use_value(o, t->u[i], node) == 0) return 0;
  return 1;
}

/* PreFilter of PodTopologySpread (calPreFilterState) and InterPodAffinity
 * (getExistingAntiAffinityCounts, getIncomingAffinityAntiAffinityCounts). */
static void topo_prefilter(ksim_oracle* o, const ksim_pod_set* ps, const ksim_pod* p, topo_ctx* t) {
  memset(t, 0, sizeof(*t));
  t->n = p->use_count;
  for (int i = 0; i < t->n; i++) {
    t->u[i] = &ps->uses[p->use_first + i];
    int k = t->u[i]->kind;
    if (k == KSIM_USE_PTS_HARD) t->has_hard = 1;
    else if (k == KSIM_USE_PTS_SOFT) t->has_soft = 1;
    else if (k == KSIM_USE_IPA_EXISTING_ANTI || k == KSIM_USE_IPA_AFFINITY || k == KSIM_USE_IPA_ANTI) t->has_ipa_filter = 1;
    else t->has_ipa_score = 1;
    memset(dom_of(o, i), 0, 8 * (size_t)o->vmax);
    memset(present_of(o, i), 0, (size_t)o->vmax);
  }
  t->affinity_counts_empty = 1;
  for (int32_t node = 0; node < o->n; node++) {
    int all_hard = t->has_hard ? node_has_all_keys(o, t, KSIM_USE_PTS_HARD, node) : 0;
    for (int i = 0; i < t->n; i++) {
      const ksim_topo_use* u = t->u[i];
      uint32_t v = use_value(o, u, node);
      switch (u->kind) {
        case KSIM_USE_PTS_HARD:
          if (!all_hard || !match_node_inclusion_policies(o, ps, p, u, node)) break;
          dom_of(o, i)[v] += class_count(o, u->cls, node);      /* TpPairToMatchNum[pair] += count */
          present_of(o, i)[v] = 1;
          break;
        case KSIM_USE_IPA_EXISTING_ANTI:
        case KSIM_USE_IPA_AFFINITY:
        case KSIM_USE_IPA_ANTI:
          if (v == 0) break;                                     /* topologyToMatchedTermCount.update */
          dom_of(o, i)[v] += class_count(o, u->cls, node);
          if (u->kind == KSIM_USE_IPA_AFFINITY && class_count(o, u->cls, node) > 0) t->affinity_counts_empty = 0;
          break;
        default:
          break;
      }
    }
  }
  /* TpKeyToCriticalPaths: the minimum over the key's pairs (math.MaxInt32 if none) */
  for (int i = 0; i < t->n; i++) {
    if (t->u[i]->kind != KSIM_USE_PTS_HARD) continue;
    int64_t mn = 2147483647;
    for (int32_t v = 0; v < o->vmax; v++)
      if (present_of(o, i)[v] && dom_of(o, i)[v] < mn) mn = dom_of(o, i)[v];
    t->min_match[i] = mn;
  }
}

/* podtopologyspread Filter -> 0 or KSIM_PTS_* */
static uint32_t pts_filter(const ksim_oracle* o, const topo_ctx* t, int32_t node) {
  for (int i = 0; i < t->n; i++) {
    const ksim_topo_use* u = t->u[i];
    if (u->kind != KSIM_USE_PTS_HARD) continue;
    uint32_t v = use_value(o, u, node);
    if (v == 0) return KSIM_PTS_MISSING_LABEL;
    int64_t self = (u->flags & KSIM_USEF_SELF_MATCH) ? 1 : 0;
    int64_t match = present_of(o, i)[v] ? dom_of(o, i)[v] : 0;
    int64_t skew = match + self - t->min_match[i];
    if (skew > (int64_t)u->arg) return KSIM_PTS_SKEW;
  }
  return 0;
}

/* interpodaffinity Filter -> 0 or KSIM_IPA_* */
static uint32_t ipa_filter(const ksim_oracle* o, const ksim_pod* p, const topo_ctx* t, int32_t node) {
  /* satisfyPodAffinity */
  int pods_exist = 1, any_aff = 0;
  for (int i = 0; i < t->n; i++) {
    const ksim_topo_use* u = t->u[i];
    if (u->kind != KSIM_USE_IPA_AFFINITY) continue;
    any_aff = 1;
    uint32_t v = use_value(o, u, node);
    if (v == 0) return KSIM_IPA_AFFINITY;            /* all topology labels must exist */
    if (dom_of(o, i)[v] <= 0) pods_exist = 0;
  }
  if (any_aff && !pods_exist &&
      !(t->affinity_counts_empty && (p->topo_flags & KSIM_POD_IPA_SELF_AFFINITY)))
    return KSIM_IPA_AFFINITY;
  /* satisfyPodAntiAffinity */
  for (int i = 0; i < t->n; i++) {
    const ksim_topo_use* u = t->u[i];
    if (u->kind != KSIM_USE_IPA_ANTI) continue;
    uint32_t v = use_value(o, u, node);
    if (v != 0 && dom_of(o, i)[v] > 0) return KSIM_IPA_ANTI_AFFINITY;
  }
  /* satisfyExistingPodsAntiAffinity */
  for (int i = 0; i < t->n; i++) {
    const ksim_topo_use* u = t->u[i];
    if (u->kind != KSIM_USE_IPA_EXISTING_ANTI) continue;
    uint32_t v = use_value(o, u, node);
    if (v != 0 && dom_of(o, i)[v] > 0) return KSIM_IPA_EXISTING_ANTI;
  }
  return 0;
}

/* PreScore of PodTopologySpread (initPreScoreState + PreScore) and
 * InterPodAffinity (processExistingPod over all nodes), over the feasible list. */
static void topo_prescore(ksim_oracle* o, const ksim_pod_set* ps, const ksim_pod* p, const int32_t* flist,
                          int32_t nf, topo_ctx* t) {
  /* PTS: IgnoredNodes = feasible nodes missing a soft key; pair registration; topoSize */
  int32_t n_ignored = 0;
  for (int i = 0; i < t->n; i++)
    if (t->u[i]->kind == KSIM_USE_PTS_SOFT) {
      memset(dom_of(o, i), 0, 8 * (size_t)o->vmax);
      memset(present_of(o, i), 0, (size_t)o->vmax);
    }
  /* requireAllTopologies = len(pod constraints) > 0 || !systemDefaulted */
  const int require_all = !(p->topo_flags & KSIM_POD_PTS_SYSTEM_DEFAULT);
  if (t->has_soft) {
    int32_t size[KSIM_MAX_USES] = {0};
    for (int32_t j = 0; j < nf; j++) {
      int32_t node = flist[j];
      o->ignored[node] = require_all && !node_has_all_keys(o, t, KSIM_USE_PTS_SOFT, node);
      if (o->ignored[node]) { n_ignored++; continue; }
      for (int i = 0; i < t->n; i++) {
        const ksim_topo_use* u = t->u[i];
        if (u->kind != KSIM_USE_PTS_SOFT || (u->flags & KSIM_USEF_HOSTNAME)) continue;
        uint32_t v = use_value(o, u, node);
        if (!present_of(o, i)[v]) { present_of(o, i)[v] = 1; size[i]++; }
      }
    }
    for (int i = 0; i < t->n; i++) {
      const ksim_topo_use* u = t->u[i];
      if (u->kind != KSIM_USE_PTS_SOFT) continue;
      int32_t sz = (u->flags & KSIM_USEF_HOSTNAME) ? nf - n_ignored : size[i];
      t->weight[i] = o->topo_log[sz];                 /* topologyNormalizingWeight(sz) = log(sz + 2) */
    }
    for (int32_t node = 0; node < o->n; node++) {     /* processAllNode */
      if (require_all && !node_has_all_keys(o, t, KSIM_USE_PTS_SOFT, node)) continue;
      for (int i = 0; i < t->n; i++) {
        const ksim_topo_use* u = t->u[i];
        if (u->kind != KSIM_USE_PTS_SOFT || (u->flags & KSIM_USEF_HOSTNAME)) continue;
        if (!match_node_inclusion_policies(o, ps, p, u, node)) continue;
        uint32_t v = use_value(o, u, node);
        if (!present_of(o, i)[v]) continue;           /* pair not associated with a candidate node */
        dom_of(o, i)[v] += class_count(o, u->cls, node);
      }
    }
  }
  /* IPA: topologyScore[key][value] = sum of weighted counts over the nodes of the pair */
  t->topology_score_empty = 1;
  for (int i = 0; i < t->n; i++) {
    const ksim_topo_use* u = t->u[i];
    if (u->kind != KSIM_USE_IPA_SCORE && u->kind != KSIM_USE_IPA_SCORE_HARD) continue;
    memset(dom_of(o, i), 0, 8 * (size_t)o->vmax);
    if (u->kind == KSIM_USE_IPA_SCORE_HARD && o->prof.hard_pod_affinity_weight <= 0) continue;
    for (int32_t node = 0; node < o->n; node++) {
      uint32_t v = use_value(o, u, node);
      int64_t c = class_count(o, u->cls, node);
      if (v == 0 || c == 0) continue;
      dom_of(o, i)[v] += c;
      t->topology_score_empty = 0;
    }
  }
}

/* podtopologyspread Score (before NormalizeScore); ignored nodes score 0 */
static int64_t pts_score(const ksim_oracle* o, const topo_ctx* t, int32_t node) {
  if (!t->has_soft || o->ignored[node]) return 0;
  double score = 0;
  for (int i = 0; i < t->n; i++) {
    const ksim_topo_use* u = t->u[i];
    if (u->kind != KSIM_USE_PTS_SOFT) continue;
    uint32_t v = use_value(o, u, node);
    if (v == 0) continue;
    int64_t cnt = (u->flags & KSIM_USEF_HOSTNAME) ? class_count(o, u->cls, node) : dom_of(o, i)[v];
    score += (double)cnt * t->weight[i] + (double)(u->arg - 1);   /* scoreForCount, unfused */
  }
  return (int64_t)round(score);                                   /* math.Round: half away from zero */
}

/* interpodaffinity Score */
static int64_t ipa_score(const ksim_oracle* o, const topo_ctx* t, int32_t node) {
  int64_t s = 0;
  for (int i = 0; i < t->n; i++) {
    const ksim_topo_use* u = t->u[i];
    int64_t coef;
    if (u->kind == KSIM_USE_IPA_SCORE) coef = u->arg;
    else if (u->kind == KSIM_USE_IPA_SCORE_HARD) coef = o->prof.hard_pod_affinity_weight;
    else continue;
    if (coef == 0) continue;
    uint32_t v = use_value(o, u, node);
    if (v != 0) s += coef * dom_of(o, i)[v];
  }
  return s;
}

/* ---- framework: RunFilterPlugins — a17 ---------------------------------- */
/* ---- NetworkBandwidth, the simulator's out-of-tree plugin -----------------
 * simulator/scheduler/plugin/networkbandwidth/plugin.go.  Quantities are
 * milli-units (the host rejects finer ones).  Filter's Skip / Error returns are
 * neither Success nor Unschedulable, so [upstream] RunFilterPlugins turns them
 * into framework.Error and the scheduling cycle fails (nb_error). */
static uint32_t nb_filter(const ksim_oracle* o, const ksim_pod* p, int32_t node) {
  const uint32_t fl = o->flags[node];
  if (!(fl & KSIM_NODE_NB_LIMIT)) return KSIM_NB_NO_LIMIT;               /* :54-57 Skip */
  if (fl & KSIM_NODE_NB_LIMIT_BAD) return KSIM_NB_LIMIT_BAD;             /* :58-61 Error */
  if (p->nb_flags & KSIM_POD_NB_INGRESS_BAD) return KSIM_NB_INGRESS_BAD; /* :72-76 Error */
  if (p->nb_flags & KSIM_POD_NB_EGRESS_BAD) return KSIM_NB_EGRESS_BAD;   /* :84-88 Error */
  if (p->nb_req == 0) return KSIM_NB_NO_REQUEST;                          /* :92-94 Skip */
  return o->nb_alloc[node] + p->nb_req > o->nb_limit[node] ? KSIM_NB_INSUFFICIENT : 0; /* :97-99 */
}
static int nb_error(const ksim_oracle* o, uint8_t r, uint32_t detail) {
  return r != KSIM_PASSED && o->prof.filter[r] == KSIM_PL_NETWORK_BANDWIDTH && detail >= KSIM_NB_NO_LIMIT;
}
/* Score :128-149: (limit - allocated).Value(), rounding a fraction away from zero */
static int64_t nb_score(const ksim_oracle* o, int32_t node) {
  const int64_t d = o->nb_limit[node] - o->nb_alloc[node];
  return d >= 0 ? (d + 999) / 1000 : -((-d + 999) / 1000);
}
/* Score returns Skip (no limit annotation) or Error (limit does not parse) */
static int nb_score_fails(const ksim_oracle* o, int32_t node) {
  return !(o->flags[node] & KSIM_NODE_NB_LIMIT) || (o->flags[node] & KSIM_NODE_NB_LIMIT_BAD);
}
static int has_score_plugin(const ksim_oracle* o, int plugin) {
  for (int k = 0; k < o->prof.n_score; k++)
    if (o->prof.score[k] == plugin) return 1;
  return 0;
}
/* RunScorePlugins fails when NetworkBandwidth's Score fails on a kept node */
static int nb_score_error(const ksim_oracle* o, const int32_t* flist, int32_t nf) {
  if (nf <= 1 || !has_score_plugin(o, KSIM_PL_NETWORK_BANDWIDTH)) return 0;
  for (int32_t j = 0; j < nf; j++)
    if (nb_score_fails(o, flist[j])) return 1;
  return 0;
}

/* Runs the profile's filter plugins in order and stops at the first failure
 * (runAllFilters=false).  Returns the filter-order index of the failing plugin
 * or KSIM_PASSED; *detail gets the reason payload. */
static uint8_t run_filter_plugins(const ksim_oracle* o, const ksim_pod_set* ps, const ksim_pod* p,
                                  const topo_ctx* t, int32_t node, uint32_t* detail) {
  *detail = 0;
  for (int f = 0; f < o->prof.n_filter; f++) {
    switch (o->prof.filter[f]) {
      case KSIM_PL_NODE_UNSCHEDULABLE:   /* nodeunschedulable.Filter */
        if ((o->flags[node] & KSIM_NODE_UNSCHEDULABLE) &&
            !(p->flags & KSIM_POD_TOLERATES_UNSCHEDULABLE))
          return (uint8_t)f;
        break;
      case KSIM_PL_NODE_NAME:            /* nodename.Filter */
        if (p->node_name != -1 && p->node_name != node) return (uint8_t)f;
        break;
      case KSIM_PL_TAINT_TOLERATION: {
        uint32_t tid = find_matching_untolerated_taint(o, p, node);
        if (tid) { *detail = tid; return (uint8_t)f; }
        break;
      }
      case KSIM_PL_NODE_AFFINITY: {
        uint32_t why;
        if (!node_affinity_filter(o, ps, p, node, &why)) { *detail = why; return (uint8_t)f; }
        break;
      }
      case KSIM_PL_VOLUME_BINDING: {     /* bound claims' PV node affinity, unbound claims' matches */
        uint32_t r = volume_binding_fails(o, ps, p->vb_first, p->vb_count, node);
        if (r) { *detail = r; return (uint8_t)f; }
        break;
      }
      case KSIM_PL_VOLUME_ZONE:          /* bound claims: PV topology labels */
        if (!volume_groups_match(o, ps, p->vz_first, p->vz_count, node)) return (uint8_t)f;
        break;
      case KSIM_PL_NODE_RESOURCES_FIT: {
        uint32_t r = fits_request(o, p, node);
        if (r) { *detail = r; return (uint8_t)f; }
        break;
      }
      case KSIM_PL_POD_TOPOLOGY_SPREAD: {
        uint32_t r = t->has_hard ? pts_filter(o, t, node) : 0;
        if (r) { *detail = r; return (uint8_t)f; }
        break;
      }
      case KSIM_PL_INTER_POD_AFFINITY: {
        uint32_t r = t->has_ipa_filter ? ipa_filter(o, p, t, node) : 0;
        if (r) { *detail = r; return (uint8_t)f; }
        break;
      }
      case KSIM_PL_NODE_PORTS:           /* nodeports.Filter -> fitsPorts */
        if (node_port_conflict(o, ps, p, node)) return (uint8_t)f;
        break;
      case KSIM_PL_NETWORK_BANDWIDTH: {
        uint32_t r = nb_filter(o, p, node);
        if (r) { *detail = r; return (uint8_t)f; }
        break;
      }
      /* the other volume plugins: bound claims of unlimited kinds pass. */
      default:
        break;
    }
  }
  return KSIM_PASSED;
}

static int64_t score_plugin_raw(const ksim_oracle* o, const ksim_pod_set* ps, const ksim_pod* p,
                                const topo_ctx* t, int plugin, int32_t node) {
  switch (plugin) {
    case KSIM_PL_NODE_RESOURCES_FIT: return fit_score(o, p, node);
    case KSIM_PL_BALANCED_ALLOCATION: return balanced_allocation_score(o, p, node);
    case KSIM_PL_TAINT_TOLERATION: return count_intolerable_prefer_no_schedule(o, p, node);
    case KSIM_PL_NODE_AFFINITY: return preferred_node_affinity_score(o, ps, p, node);
    case KSIM_PL_POD_TOPOLOGY_SPREAD: return pts_score(o, t, node);
    case KSIM_PL_INTER_POD_AFFINITY: return t->has_ipa_score ? ipa_score(o, t, node) : 0;
    case KSIM_PL_IMAGE_LOCALITY: {     /* imagelocality.Score, compiled per image signature */
      for (int32_t i = 0; i < p->use_count; i++) {
        const ksim_topo_use* u = &ps->uses[p->use_first + i];
        if (u->kind == KSIM_USE_IMAGE) return class_count(o, u->cls, node);
      }
      return 0;
    }
    case KSIM_PL_NETWORK_BANDWIDTH: return nb_score_fails(o, node) ? 0 : nb_score(o, node);
    default: return 0;
  }
}

/* NormalizeScore of each plugin over the scored list (in place).  ign[j]:
 * node j of the list is in PodTopologySpread's IgnoredNodes. */
static void normalize_plugin(int plugin, const topo_ctx* t, const uint8_t* ign, int32_t n, int64_t* s) {
  switch (plugin) {
    case KSIM_PL_TAINT_TOLERATION:        /* tainttoleration.NormalizeScore (reverse) */
      ksim_oracle_default_normalize(MAX_NODE_SCORE, 1, n, s);
      return;
    case KSIM_PL_NODE_AFFINITY:           /* nodeaffinity.NormalizeScore */
      ksim_oracle_default_normalize(MAX_NODE_SCORE, 0, n, s);
      return;
    case KSIM_PL_POD_TOPOLOGY_SPREAD: {   /* podtopologyspread.NormalizeScore */
      int64_t mn = INT64_MAX, mx = 0;
      for (int i = 0; i < n; i++) {
        if (ign[i]) continue;               /* invalidScore: excluded from min / max */
        if (s[i] < mn) mn = s[i];
        if (s[i] > mx) mx = s[i];
      }
      for (int i = 0; i < n; i++) {
        if (ign[i]) s[i] = 0;
        else s[i] = (mx == 0) ? MAX_NODE_SCORE : MAX_NODE_SCORE * (mx + mn - s[i]) / mx;
      }
      return;
    }
    case KSIM_PL_INTER_POD_AFFINITY:      /* interpodaffinity.NormalizeScore */
    case KSIM_PL_NETWORK_BANDWIDTH: {     /* networkbandwidth NormalizeScore, plugin.go:159-186 */
      if (plugin == KSIM_PL_INTER_POD_AFFINITY && t->topology_score_empty) return;
      int64_t mn = INT64_MAX, mx = INT64_MIN;
      for (int i = 0; i < n; i++) { if (s[i] > mx) mx = s[i]; if (s[i] < mn) mn = s[i]; }
      int64_t diff = mx - mn;
      for (int i = 0; i < n; i++) {
        double f = 0;
        if (diff > 0) f = (double)MAX_NODE_SCORE * ((double)(s[i] - mn) / (double)diff);
        s[i] = (int64_t)f;
      }
      return;
    }
    default:
      return;                              /* Fit / BalancedAllocation / ImageLocality: none */
  }
}

/* normalize_plugin's map of one score given the list's extrema (the timing
 * path reduces the extrema across threads first) */
static int64_t normalize_one(int plugin, uint8_t ign, int64_t mn, int64_t mx, int64_t v) {
  switch (plugin) {
    case KSIM_PL_TAINT_TOLERATION:
    case KSIM_PL_NODE_AFFINITY: {         /* DefaultNormalizeScore: mx = maxCount */
      const int reverse = plugin == KSIM_PL_TAINT_TOLERATION;
      if (mx == 0) return reverse ? MAX_NODE_SCORE : v;
      const int64_t x = MAX_NODE_SCORE * v / mx;
      return reverse ? MAX_NODE_SCORE - x : x;
    }
    case KSIM_PL_POD_TOPOLOGY_SPREAD:
      if (ign) return 0;
      return (mx == 0) ? MAX_NODE_SCORE : MAX_NODE_SCORE * (mx + mn - v) / mx;
    case KSIM_PL_INTER_POD_AFFINITY:
    case KSIM_PL_NETWORK_BANDWIDTH: {
      const int64_t diff = mx - mn;
      double f = 0;
      if (diff > 0) f = (double)MAX_NODE_SCORE * ((double)(v - mn) / (double)diff);
      return (int64_t)f;
    }
  }
  return v;
}

static int has_normalize(int plugin) {
  return plugin == KSIM_PL_TAINT_TOLERATION || plugin == KSIM_PL_NODE_AFFINITY ||
         plugin == KSIM_PL_POD_TOPOLOGY_SPREAD || plugin == KSIM_PL_INTER_POD_AFFINITY ||
         plugin == KSIM_PL_NETWORK_BANDWIDTH;
}

/* NodeInfo.AddPod restricted to the aggregates the plugins read — a20 */
static void assume_pod(ksim_oracle* o, const ksim_pod_set* ps, const ksim_pod* p, int32_t node, int sign) {
  o->req_cpu[node] += sign * p->req_cpu;
  o->req_mem[node] += sign * p->req_mem;
  o->req_eph[node] += sign * p->req_eph;
  for (int k = 0; k < o->n_scalar; k++) o->req_scalar[(size_t)k * o->n + node] += sign * p->scalar_req[k];
  o->nz_cpu[node] += sign * p->nz_cpu;
  o->nz_mem[node] += sign * p->nz_mem;
  o->num_pods[node] += sign;
  o->nb_alloc[node] += sign * p->nb_add;
  for (int i = 0; i < p->add_count; i++) {            /* pod counts / carried terms */
    const ksim_class_add* a = &ps->adds[p->add_first + i];
    o->cnt[(size_t)a->cls * o->n + node] += sign * a->count;
  }
}

/* ---- schedulePod: findNodesThatFitPod + prioritizeNodes + selectHost ----- */
/* Sequential (parallelism 1) semantics of [upstream] schedule_one.go — a15-a19. */
int ksim_oracle_cycle(ksim_oracle* o, const ksim_pod_set* ps, int32_t pi, ksim_eval_out* out) {
  return ksim_oracle_cycle_ext(o, ps, pi, NULL, NULL, out);
}

/* The cycle with extenders (schedule_one.go findNodesThatPassExtenders and the
 * extender part of prioritizeNodes): ext_fail[node] nonzero removes a kept
 * node after the window (nextStartNodeIndex has already advanced);
 * ext_score[node] (the extenders' combined weighted scores) is added to the
 * plugin total before selectHost.  Either may be NULL. */
int ksim_oracle_cycle_ext(ksim_oracle* o, const ksim_pod_set* ps, int32_t pi, const uint8_t* ext_fail,
                          const int64_t* ext_score, ksim_eval_out* out) {
  if (!o || !ps || pi < 0 || pi >= ps->n_pods || !out) return KSIM_E_INVALID;
  const ksim_pod* p = &ps->pods[pi];
  const int32_t N = o->n;
  if (N == 0) return KSIM_E_INVALID;                      /* ErrNoNodesAvailable */
  const int64_t seq = o->pod_seq++;
  const scan_set ss = pod_scan_set(o, ps, p);
  const int32_t NS = ss.n;
  const int32_t K = ksim_oracle_num_feasible_nodes_to_find(o->prof.percentage_of_nodes_to_score, NS);
  const int S = o->prof.n_score;

  if (out->fail_plugin) memset(out->fail_plugin, KSIM_NOT_EVALUATED, (size_t)N);
  if (out->fail_detail) memset(out->fail_detail, 0, 4 * (size_t)N);
  if (out->scored) memset(out->scored, 0, (size_t)N);
  if (out->raw) memset(out->raw, 0, 8 * (size_t)N * S);
  if (out->norm) memset(out->norm, 0, 8 * (size_t)N * S);
  if (out->total) memset(out->total, 0, 8 * (size_t)N);

  /* PreFilter (PodTopologySpread / InterPodAffinity state), then findNodesThatPassFilters */
  topo_ctx tc;
  topo_prefilter(o, ps, p, &tc);
  int32_t nf = 0, nfailed = 0, evaluated = 0, error = 0;
  /* NodeInfos().Get of a PreFilterResult name the snapshot lacks: the cycle
   * fails with an error before any Filter call */
  if (p->flags & KSIM_POD_NODE_NAMES_UNKNOWN) error = 1;
  for (int32_t i = 0; i < NS; i++) {
    int32_t node = scan_node_at(&ss, i);
    uint32_t det;
    uint8_t r = run_filter_plugins(o, ps, p, &tc, node, &det);
    evaluated++;
    if (out->fail_plugin) out->fail_plugin[node] = r;
    if (out->fail_detail) out->fail_detail[node] = det;
    if (nb_error(o, r, det)) {     /* checkNode: errCh.SendErrorWithCancel; not in the status map */
      error = 1;
      break;
    }
    if (r == KSIM_PASSED) {
      if (nf == K) break;          /* the (K+1)-th feasible node: recorded, not kept */
      o->flist[nf++] = node;
    } else {
      nfailed++;
    }
  }
  int32_t processed = nf + nfailed;
  if (NS > 0) o->next_start = (int32_t)(((int64_t)o->next_start + processed) % NS);
  if (ext_fail) {                  /* findNodesThatPassExtenders over the kept list */
    int32_t m = 0;
    for (int32_t j = 0; j < nf; j++) {
      const int32_t node = o->flist[j];
      if (ext_fail[node]) {
        if (out->fail_plugin) out->fail_plugin[node] = KSIM_FAIL_EXTENDER;
      } else {
        o->flist[m++] = node;
      }
    }
    nf = m;
  }

  out->k_to_find = K;
  out->n_feasible = nf;
  out->n_evaluated = evaluated;
  out->n_processed = processed;
  out->next_start = o->next_start;

  if (error || nb_score_error(o, o->flist, nf)) {   /* the cycle fails with framework.Error */
    out->chosen = KSIM_CHOSEN_ERROR;
    out->status = KSIM_STATUS_ERROR;
    return KSIM_OK;
  }
  if (nf == 0) {
    out->chosen = -1;
    out->status = KSIM_STATUS_UNSCHEDULABLE;
    return KSIM_OK;
  }
  int32_t chosen;
  if (nf == 1) {
    chosen = o->flist[0];          /* single feasible node: no scoring at all */
  } else {
    /* RunScorePlugins: raw scores, NormalizeScore per plugin, weights */
    int64_t* tmp = (int64_t*)malloc(8 * (size_t)nf);
    int64_t* totals = (int64_t*)calloc((size_t)nf, 8);
    uint8_t* ign = (uint8_t*)calloc((size_t)nf, 1);
    topo_prescore(o, ps, p, o->flist, nf, &tc);
    if (tc.has_soft) for (int32_t j = 0; j < nf; j++) ign[j] = o->ignored[o->flist[j]];
    for (int s = 0; s < S; s++) {
      int pl = o->prof.score[s];
      for (int32_t j = 0; j < nf; j++) tmp[j] = score_plugin_raw(o, ps, p, &tc, pl, o->flist[j]);
      if (out->raw) for (int32_t j = 0; j < nf; j++) out->raw[(size_t)s * N + o->flist[j]] = tmp[j];
      if (has_normalize(pl)) normalize_plugin(pl, &tc, ign, nf, tmp);
      int64_t w = o->prof.score_weight[s] == 0 ? 1 : o->prof.score_weight[s];
      for (int32_t j = 0; j < nf; j++) {
        if (out->norm) out->norm[(size_t)s * N + o->flist[j]] = tmp[j];
        totals[j] += tmp[j] * w;
      }
    }
    /* prioritizeNodes: no score plugins and no extenders -> every node scores 1 */
    if (S == 0 && !ext_score) for (int32_t j = 0; j < nf; j++) totals[j] = 1;
    if (ext_score) for (int32_t j = 0; j < nf; j++) totals[j] += ext_score[o->flist[j]];
    int64_t best_total = 0;
    uint64_t best_lo = 0;
    chosen = -1;
    for (int32_t j = 0; j < nf; j++) {
      int32_t node = o->flist[j];
      if (out->total) out->total[node] = totals[j];
      if (out->scored) out->scored[node] = 1;
      const uint64_t lo = ksim_oracle_tb_lo(o->prof.tiebreak_seed, seq, node);
      if (chosen < 0 || tb_better(totals[j], lo, best_total, best_lo)) {
        best_total = totals[j];
        best_lo = lo;
        chosen = node;
      }
    }
    free(tmp);
    free(totals);
    free(ign);
  }
  out->chosen = chosen;
  out->status = KSIM_STATUS_SCHEDULED;
  assume_pod(o, ps, p, chosen, 1);
  return KSIM_OK;
}

/* ---- framework-driven compat mode (ksim_engine.h ksim_fw_*) -------------- */
/* Under the simulator's own settings (parallelism 16, percentageOfNodesToScore
 * 0: simulator/scheduler/scheduler.go:149,153,231-241) the [upstream]
 * framework, not the plugins, decides which nodes Filter runs on (16 racing
 * Parallelizer workers, first numFeasibleNodesToFind feasible), the feasible
 * list PreScore / Score / NormalizeScore see, and the node selectHost's
 * reservoir picks for Reserve.  The plugin answers are functions of those
 * choices alone:
 *   Filter(node)        the PreFilter state and the snapshot (every node of
 *                       the scan set answered here);
 *   PreScore(list)      PodTopologySpread's IgnoredNodes, pair registration
 *                       and topologyNormalizingWeight over the list
 *                       (initPreScoreState); InterPodAffinity's topologyScore
 *                       over all nodes (processExistingPod);
 *   NormalizeScore(ls)  the plugin's normalization over exactly the list it
 *                       is handed (wrappedplugin.go:356-375).
 * Reserve / Unreserve are ksim_oracle_assume with sign +1 / -1. */
int ksim_oracle_fw_filter(ksim_oracle* o, const ksim_pod_set* ps, int32_t pi, ksim_eval_out* out) {
  if (!o || !ps || pi < 0 || pi >= ps->n_pods || !out || o->n == 0) return KSIM_E_INVALID;
  const ksim_pod* p = &ps->pods[pi];
  const int32_t N = o->n;
  const scan_set ss = pod_scan_set(o, ps, p);
  if (!o->fw_tc) o->fw_tc = (topo_ctx*)calloc(1, sizeof(topo_ctx));
  topo_prefilter(o, ps, p, o->fw_tc);
  if (out->fail_plugin) memset(out->fail_plugin, KSIM_NOT_EVALUATED, (size_t)N);
  if (out->fail_detail) memset(out->fail_detail, 0, 4 * (size_t)N);
  int32_t nf = 0;
  const int unknown = (p->flags & KSIM_POD_NODE_NAMES_UNKNOWN) != 0;
  for (int32_t i = 0; i < ss.n; i++) {
    const int32_t node = scan_node_at(&ss, i);
    uint32_t det;
    const uint8_t r = run_filter_plugins(o, ps, p, o->fw_tc, node, &det);
    if (out->fail_plugin) out->fail_plugin[node] = r;
    if (out->fail_detail) out->fail_detail[node] = det;
    nf += r == KSIM_PASSED;
  }
  out->chosen = unknown ? KSIM_CHOSEN_ERROR : -1;
  out->status = unknown ? KSIM_STATUS_ERROR : 0;
  out->n_feasible = nf;
  out->n_evaluated = ss.n;
  out->n_processed = 0;
  out->k_to_find = ksim_oracle_num_feasible_nodes_to_find(o->prof.percentage_of_nodes_to_score, ss.n);
  out->next_start = o->next_start;
  o->fw_active = 1;
  o->fw_scored = 0;
  return KSIM_OK;
}

/* RunFilterPluginsWithNominatedPods' first pass (addNominatedPods): for each
 * group, the nominated pods added to the node (NodeInfo.AddPodInfo; the
 * PreFilterExtensions' AddPod of PodTopologySpread / InterPodAffinity, which
 * for +1 updates equal the PreFilter state over the snapshot with them bound),
 * the node's Filter, the pods removed again; the cycle's PreFilter state is
 * recomputed at the end. */
int ksim_oracle_fw_filter_nominated(ksim_oracle* o, const ksim_pod_set* ps, int32_t pi, const ksim_pod_set* nps,
                                    int32_t n_nodes, const int32_t* nodes, const int32_t* first, const int32_t* count,
                                    uint8_t* fail_plugin, uint32_t* fail_detail) {
  if (!o || !o->fw_active || !ps || pi < 0 || pi >= ps->n_pods || n_nodes < 0) return KSIM_E_INVALID;
  if (n_nodes == 0) return KSIM_OK;
  if (!nps || !nodes || !first || !count || !fail_plugin) return KSIM_E_INVALID;
  const ksim_pod* p = &ps->pods[pi];
  for (int32_t k = 0; k < n_nodes; k++) {
    if (nodes[k] < 0 || nodes[k] >= o->n || first[k] < 0 || count[k] < 0 || first[k] + count[k] > nps->n_pods)
      return KSIM_E_INVALID;
  }
  topo_ctx tc;
  for (int32_t k = 0; k < n_nodes; k++) {
    for (int32_t j = first[k]; j < first[k] + count[k]; j++) assume_pod(o, nps, &nps->pods[j], nodes[k], 1);
    topo_prefilter(o, ps, p, &tc);
    uint32_t det;
    fail_plugin[k] = run_filter_plugins(o, ps, p, &tc, nodes[k], &det);
    if (fail_detail) fail_detail[k] = det;
    for (int32_t j = first[k]; j < first[k] + count[k]; j++) assume_pod(o, nps, &nps->pods[j], nodes[k], -1);
  }
  topo_prefilter(o, ps, p, o->fw_tc);            /* the cycle's own PreFilter state */
  return KSIM_OK;
}

/* PreScore + Score + NormalizeScore + weights over exactly `nodes` (the
 * framework's feasible list, any order).  No selectHost, no bind. */
int ksim_oracle_fw_score(ksim_oracle* o, const ksim_pod_set* ps, int32_t pi, const int32_t* nodes, int32_t n,
                         ksim_eval_out* out) {
  if (!o || !o->fw_active || !ps || pi < 0 || pi >= ps->n_pods || !out || n < 0 || (n > 0 && !nodes))
    return KSIM_E_INVALID;
  const ksim_pod* p = &ps->pods[pi];
  const int32_t N = o->n;
  const int S = o->prof.n_score;
  for (int32_t j = 0; j < n; j++) {
    if (nodes[j] < 0 || nodes[j] >= N) return KSIM_E_INVALID;
    o->flist[j] = nodes[j];
  }
  if (out->scored) memset(out->scored, 0, (size_t)N);
  if (out->raw) memset(out->raw, 0, 8 * (size_t)N * S);
  if (out->norm) memset(out->norm, 0, 8 * (size_t)N * S);
  if (out->total) memset(out->total, 0, 8 * (size_t)N);
  topo_ctx* tc = o->fw_tc;
  out->chosen = -1;
  out->n_feasible = n;
  if (nb_score_error(o, o->flist, n)) {
    out->status = KSIM_STATUS_ERROR;
    out->chosen = KSIM_CHOSEN_ERROR;
    return KSIM_OK;
  }
  out->status = 0;
  topo_prescore(o, ps, p, o->flist, n, tc);
  o->fw_scored = 1;
  int64_t* tmp = (int64_t*)malloc(8 * (size_t)(n ? n : 1));
  int64_t* totals = (int64_t*)calloc((size_t)(n ? n : 1), 8);
  uint8_t* ign = (uint8_t*)calloc((size_t)(n ? n : 1), 1);
  if (tc->has_soft) for (int32_t j = 0; j < n; j++) ign[j] = o->ignored[o->flist[j]];
  for (int s = 0; s < S; s++) {
    const int pl = o->prof.score[s];
    for (int32_t j = 0; j < n; j++) tmp[j] = score_plugin_raw(o, ps, p, tc, pl, o->flist[j]);
    if (out->raw) for (int32_t j = 0; j < n; j++) out->raw[(size_t)s * N + o->flist[j]] = tmp[j];
    if (has_normalize(pl)) normalize_plugin(pl, tc, ign, n, tmp);
    const int64_t w = o->prof.score_weight[s] == 0 ? 1 : o->prof.score_weight[s];
    for (int32_t j = 0; j < n; j++) {
      if (out->norm) out->norm[(size_t)s * N + o->flist[j]] = tmp[j];
      totals[j] += tmp[j] * w;
    }
  }
  if (S == 0) for (int32_t j = 0; j < n; j++) totals[j] = 1;
  for (int32_t j = 0; j < n; j++) {
    if (out->total) out->total[o->flist[j]] = totals[j];
    if (out->scored) out->scored[o->flist[j]] = 1;
  }
  free(tmp);
  free(totals);
  free(ign);
  return KSIM_OK;
}

/* NormalizeScore of the plugin at profile score slot `slot` over an explicit
 * (node, score) list, with the PreScore state of the last ksim_oracle_fw_score
 * (PodTopologySpread's IgnoredNodes, InterPodAffinity's topologyScore). */
int ksim_oracle_fw_normalize(ksim_oracle* o, int32_t slot, const int32_t* nodes, const int64_t* scores, int32_t n,
                             int64_t* out) {
  if (!o || !o->fw_scored || slot < 0 || slot >= o->prof.n_score || n < 0 || (n > 0 && (!nodes || !scores || !out)))
    return KSIM_E_INVALID;
  const int pl = o->prof.score[slot];
  uint8_t* ign = (uint8_t*)calloc((size_t)(n ? n : 1), 1);
  for (int32_t j = 0; j < n; j++) {
    if (nodes[j] < 0 || nodes[j] >= o->n) { free(ign); return KSIM_E_INVALID; }
    ign[j] = o->fw_tc->has_soft && o->ignored[nodes[j]];
    out[j] = scores[j];
  }
  if (has_normalize(pl)) normalize_plugin(pl, o->fw_tc, ign, n, out);
  free(ign);
  return KSIM_OK;
}

/* NodeInfo.AddPod / RemovePod of a pod on a node: Reserve / Unreserve
 * (wrappedplugin.go:583-584, 617), informer pod add / delete. */
int ksim_oracle_assume(ksim_oracle* o, const ksim_pod_set* ps, int32_t pi, int32_t node, int sign) {
  if (!o || !ps || pi < 0 || pi >= ps->n_pods || node < 0 || node >= o->n || (sign != 1 && sign != -1))
    return KSIM_E_INVALID;
  assume_pod(o, ps, &ps->pods[pi], node, sign);
  return KSIM_OK;
}

/* ---- timing mode: same cycle, node loop fanned out (Parallelizer analogue) */
/* One OpenMP region for the whole run (no fork / join per pod).  Per pod:
 * every thread filters its slice of the scan and counts it; one thread places
 * the stop; every thread lists its slice's feasible nodes at its offset and
 * (no PreScore state, no NetworkBandwidth score check: `fused`) scores them,
 * keeping per-plugin extrema; after a barrier, NormalizeScore, the totals and
 * selectHost's best of its part; one thread combines the bests, binds, and
 * sets up the next pod.  Four barriers a pod on the fused path. */
int ksim_oracle_schedule(ksim_oracle* o, const ksim_pod_set* ps, int32_t first, int32_t count,
                         int32_t* chosen_out, int nthreads, ksim_batch_stats* st) {
  if (!o || !ps || first < 0 || count < 0 || first + count > ps->n_pods) return KSIM_E_INVALID;
  const int32_t N = o->n;
  if (N == 0) return KSIM_E_INVALID;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > ORACLE_MAX_THREADS) nthreads = ORACLE_MAX_THREADS;
  const int S = o->prof.n_score;
  int64_t evals = 0, sched = 0, unsched = 0;
  uint8_t* feas = o->fail;   /* 1 = passed all filters */
  int64_t* raw = o->raw;     /* [S][N] */
  int64_t* totals = (int64_t*)malloc(8 * (size_t)N);
  uint8_t* ign_buf = (uint8_t*)malloc((size_t)N);
  const int nb_score = has_score_plugin(o, KSIM_PL_NETWORK_BANDWIDTH);
  /* the pod in flight (shared; written by one thread between barriers) */
  const ksim_pod* p = NULL;
  int64_t seq = 0;
  scan_set ss;
  int32_t NS = 0, K = 0, nf = 0, nfailed = 0, evaluated = 0, error = 0, chosen = -1, fused = 0;
  topo_ctx tc;
#define POD_SETUP(cc)                                                                                 \
  do {                                                                                                \
    p = &ps->pods[first + (cc)];                                                                      \
    seq = o->pod_seq++;                                                                               \
    ss = pod_scan_set(o, ps, p);                                                                      \
    NS = ss.n;                                                                                        \
    K = ksim_oracle_num_feasible_nodes_to_find(o->prof.percentage_of_nodes_to_score, NS);             \
    nf = nfailed = evaluated = 0;                                                                     \
    error = (p->flags & KSIM_POD_NODE_NAMES_UNKNOWN) ? 1 : 0;                                         \
    chosen = -1;                                                                                      \
    topo_prefilter(o, ps, p, &tc);                                                                    \
    fused = tc.n == 0 && !nb_score;                                                                   \
  } while (0)
  if (count > 0) POD_SETUP(0);

#pragma omp parallel num_threads(nthreads) if (nthreads > 1)
  {
    const int T = omp_get_num_threads(), tid = omp_get_thread_num();
    for (int32_t c = 0; c < count; c++) {
      /* findNodesThatPassFilters: this thread's slice of the scan from
       * nextStartNodeIndex, its feasible nodes counted up to its first error */
      const int32_t a = (int32_t)((int64_t)NS * tid / T), b = (int32_t)((int64_t)NS * (tid + 1) / T);
      int32_t cnt = 0, err_at = NS;
      for (int32_t i = a; i < b; i++) {
        const int32_t node = scan_node_at(&ss, i);
        uint32_t det;
        const uint8_t r = run_filter_plugins(o, ps, p, &tc, node, &det);
        const uint8_t f = r == KSIM_PASSED ? 1 : nb_error(o, r, det) ? 2 : 0;
        feas[node] = f;
        if (err_at == NS) {
          if (f == 2) err_at = i;
          else cnt += f;
        }
      }
      o->th_cnt[tid * 16] = cnt;
      o->th_err[tid * 16] = err_at;
#pragma omp barrier
#pragma omp single
      {
        /* the stop: the (K+1)-th feasible node or the first error, both evaluated */
        int32_t pre = 0, stop = NS, before = -1;
        for (int t = 0; t < T; t++) {
          const int32_t ta = (int32_t)((int64_t)NS * t / T), tb = (int32_t)((int64_t)NS * (t + 1) / T);
          o->th_pre[t * 16] = pre;
          if (pre + o->th_cnt[t * 16] > K) {            /* the (K+1)-th feasible node is in this slice */
            int32_t c2 = pre;
            for (int32_t i = ta; i < tb; i++)
              if (feas[scan_node_at(&ss, i)] == 1 && ++c2 == K + 1) {
                stop = i;
                break;
              }
            before = K;
            break;
          }
          pre += o->th_cnt[t * 16];
          if (o->th_err[t * 16] < NS) {                 /* an error before it */
            stop = o->th_err[t * 16];
            error = 1;
            before = pre;
            break;
          }
        }
        nf = before < 0 ? pre : before;
        evaluated = stop < NS ? stop + 1 : NS;
        nfailed = (stop < NS ? stop : NS) - nf;
        o->th_stop = stop;
      }
      const int32_t w0 = o->th_pre[tid * 16];
      int32_t w1 = w0;
      {
        const int32_t e = b < o->th_stop ? b : o->th_stop;
        for (int32_t i = a; i < e; i++) {
          const int32_t node = scan_node_at(&ss, i);
          if (feas[node] == 1) o->flist[w1++] = node;
        }
      }
      o->th_node[tid * 16] = -1;
      if (fused && nf > 1 && !error) {
        /* prioritizeNodes over this thread's part of the list: raw scores and
         * the per-plugin extrema NormalizeScore reads */
        int64_t* mn = &o->th_ext[tid * 2 * KSIM_MAX_SCORE];
        int64_t* mx = mn + KSIM_MAX_SCORE;
        for (int s2 = 0; s2 < S; s2++) {
          const int pl = o->prof.score[s2];
          mn[s2] = INT64_MAX;
          mx[s2] = (pl == KSIM_PL_INTER_POD_AFFINITY || pl == KSIM_PL_NETWORK_BANDWIDTH) ? INT64_MIN : 0;
        }
        for (int32_t j = w0; j < w1; j++)
          for (int s2 = 0; s2 < S; s2++) {
            const int64_t v = score_plugin_raw(o, ps, p, &tc, o->prof.score[s2], o->flist[j]);
            raw[(size_t)s2 * N + j] = v;
            if (v < mn[s2]) mn[s2] = v;
            if (v > mx[s2]) mx[s2] = v;
          }
#pragma omp barrier
        int64_t gmn[KSIM_MAX_SCORE], gmx[KSIM_MAX_SCORE];
        for (int s2 = 0; s2 < S; s2++) {
          gmn[s2] = mn[s2];
          gmx[s2] = mx[s2];
          for (int t = 0; t < T; t++) {
            const int64_t* tm = &o->th_ext[t * 2 * KSIM_MAX_SCORE];
            if (tm[s2] < gmn[s2]) gmn[s2] = tm[s2];
            if (tm[KSIM_MAX_SCORE + s2] > gmx[s2]) gmx[s2] = tm[KSIM_MAX_SCORE + s2];
          }
        }
        /* NormalizeScore, the weighted totals and selectHost's best (TB) on this part */
        int64_t bt = 0;
        uint64_t bl = 0;
        int32_t bn = -1;
        for (int32_t j = w0; j < w1; j++) {
          int64_t tot = S == 0 ? 1 : 0;
          for (int s2 = 0; s2 < S; s2++) {
            const int pl = o->prof.score[s2];
            int64_t v = raw[(size_t)s2 * N + j];
            if (has_normalize(pl) && !(pl == KSIM_PL_INTER_POD_AFFINITY && tc.topology_score_empty))
              v = normalize_one(pl, 0, gmn[s2], gmx[s2], v);
            tot += v * (o->prof.score_weight[s2] == 0 ? 1 : o->prof.score_weight[s2]);
          }
          const uint64_t lo = ksim_oracle_tb_lo(o->prof.tiebreak_seed, seq, o->flist[j]);
          if (bn < 0 || tb_better(tot, lo, bt, bl)) {
            bt = tot;
            bl = lo;
            bn = o->flist[j];
          }
        }
        o->th_mn[tid * 8] = bt;
        o->th_lo[tid * 8] = bl;
        o->th_node[tid * 16] = bn;
      } else {
#pragma omp barrier
#pragma omp single
        if (!error && nb_score_error(o, o->flist, nf)) error = 1;
        if (nf > 1 && !error) {
#pragma omp single
          topo_prescore(o, ps, p, o->flist, nf, &tc);
#pragma omp for schedule(static)
          for (int32_t j = 0; j < nf; j++) {
            totals[j] = (S == 0) ? 1 : 0;
            ign_buf[j] = tc.has_soft ? o->ignored[o->flist[j]] : 0;
            for (int s2 = 0; s2 < S; s2++)
              raw[(size_t)s2 * N + j] = score_plugin_raw(o, ps, p, &tc, o->prof.score[s2], o->flist[j]);
          }
          /* NormalizeScore per plugin: per-thread extrema, combined, then the map */
          for (int s2 = 0; s2 < S; s2++) {
            const int pl = o->prof.score[s2];
            if (!has_normalize(pl) || (pl == KSIM_PL_INTER_POD_AFFINITY && tc.topology_score_empty)) continue;
            int64_t* v = raw + (size_t)s2 * N;
            int64_t mn = INT64_MAX, mx = (pl == KSIM_PL_INTER_POD_AFFINITY || pl == KSIM_PL_NETWORK_BANDWIDTH)
                                             ? INT64_MIN : 0;
#pragma omp for schedule(static)
            for (int32_t j = 0; j < nf; j++) {
              if (pl == KSIM_PL_POD_TOPOLOGY_SPREAD && ign_buf[j]) continue;
              if (v[j] < mn) mn = v[j];
              if (v[j] > mx) mx = v[j];
            }
            o->th_mn[tid * 8] = mn;
            o->th_mx[tid * 8] = mx;
#pragma omp barrier
            for (int t = 0; t < T; t++) {
              if (o->th_mn[t * 8] < mn) mn = o->th_mn[t * 8];
              if (o->th_mx[t * 8] > mx) mx = o->th_mx[t * 8];
            }
#pragma omp for schedule(static)
            for (int32_t j = 0; j < nf; j++) v[j] = normalize_one(pl, ign_buf[j], mn, mx, v[j]);
          }
          /* the weighted totals and selectHost (TB): per thread */
          int64_t bt = 0;
          uint64_t bl = 0;
          int32_t bn = -1;
#pragma omp for schedule(static)
          for (int32_t j = 0; j < nf; j++) {
            for (int s2 = 0; s2 < S; s2++) {
              const int64_t w = o->prof.score_weight[s2] == 0 ? 1 : o->prof.score_weight[s2];
              totals[j] += raw[(size_t)s2 * N + j] * w;
            }
            const uint64_t lo = ksim_oracle_tb_lo(o->prof.tiebreak_seed, seq, o->flist[j]);
            if (bn < 0 || tb_better(totals[j], lo, bt, bl)) {
              bt = totals[j];
              bl = lo;
              bn = o->flist[j];
            }
          }
          o->th_mn[tid * 8] = bt;
          o->th_lo[tid * 8] = bl;
          o->th_node[tid * 16] = bn;
        }
      }
#pragma omp barrier
#pragma omp single
      {
        /* selectHost over the threads' bests, the bind, the next pod */
        if (nf > 1 && !error) {
          int64_t bt = 0;
          uint64_t bl = 0;
          for (int t = 0; t < T; t++) {
            const int32_t n2 = o->th_node[t * 16];
            if (n2 >= 0 && (chosen < 0 || tb_better(o->th_mn[t * 8], o->th_lo[t * 8], bt, bl))) {
              bt = o->th_mn[t * 8];
              bl = o->th_lo[t * 8];
              chosen = n2;
            }
          }
        }
        if (nf == 1 && !error) chosen = o->flist[0];
        if (NS > 0) o->next_start = (int32_t)(((int64_t)o->next_start + nf + nfailed) % NS);
        evals += evaluated;
        if (chosen >= 0) {
          assume_pod(o, ps, p, chosen, 1);
          sched++;
        } else {
          unsched++;
        }
        if (chosen_out) chosen_out[c] = error ? KSIM_CHOSEN_ERROR : chosen;
        if (c + 1 < count) POD_SETUP(c + 1);
      }
    }
  }
#undef POD_SETUP
  free(totals);
  free(ign_buf);
  if (st) {
    st->pods = count;
    st->scheduled = sched;
    st->unschedulable = unsched;
    st->evals = evals;
    st->device_ms = 0;
  }
  return KSIM_OK;
}

int ksim_oracle_get_node_state(const ksim_oracle* o, int64_t* req_cpu, int64_t* req_mem,
                               int64_t* req_eph, int64_t* nz_cpu, int64_t* nz_mem,
                               int32_t* num_pods) {
  if (!o) return KSIM_E_INVALID;
  size_t n = (size_t)o->n;
  if (req_cpu) memcpy(req_cpu, o->req_cpu, 8 * n);
  if (req_mem) memcpy(req_mem, o->req_mem, 8 * n);
  if (req_eph) memcpy(req_eph, o->req_eph, 8 * n);
  if (nz_cpu) memcpy(nz_cpu, o->nz_cpu, 8 * n);
  if (nz_mem) memcpy(nz_mem, o->nz_mem, 8 * n);
  if (num_pods) memcpy(num_pods, o->num_pods, 4 * n);
  return KSIM_OK;
}

int ksim_oracle_get_nb_alloc(const ksim_oracle* o, int64_t* out) {
  if (!o || !out) return KSIM_E_INVALID;
  memcpy(out, o->nb_alloc, 8 * (size_t)o->n);
  return KSIM_OK;
}

int32_t ksim_oracle_next_start(const ksim_oracle* o) { return o->next_start; }
void ksim_oracle_set_next_start(ksim_oracle* o, int32_t s) { o->next_start = s; }
void ksim_oracle_set_pod_seq(ksim_oracle* o, int64_t seq) { o->pod_seq = seq; }

int ksim_oracle_get_class_count(const ksim_oracle* o, int32_t* out) {
  if (!o || !out) return KSIM_E_INVALID;
  memcpy(out, o->cnt, 4 * (size_t)o->n * (size_t)(o->n_classes > 0 ? o->n_classes : 0));
  return KSIM_OK;
}


/* ---- PostFilter: DefaultPreemption (preemption.go / default_preemption.go,
 * v1.26), deterministic: offset 0, candidates in nodeTree order. ----------- */
typedef struct { int32_t idx, prio; int64_t start; } victim_rec;

static int victim_cmp(const void* a, const void* b) {       /* util.MoreImportantPod, then index */
  const victim_rec* x = (const victim_rec*)a;
  const victim_rec* y = (const victim_rec*)b;
  if (x->prio != y->prio) return x->prio > y->prio ? -1 : 1;
  if (x->start != y->start) return x->start < y->start ? -1 : 1;
  return x->idx - y->idx;
}

/* fitsRequest with the node's requested aggregates adjusted by delta[] / dpods */
static int fits_adjusted(const ksim_oracle* o, const ksim_pod* p, int32_t node, const int64_t* delta, int64_t dpods) {
  if (o->num_pods[node] + dpods + 1 > o->alloc_pods[node]) return 0;
  if (p->req_cpu == 0 && p->req_mem == 0 && p->req_eph == 0 && !(p->flags & KSIM_POD_HAS_SCALAR)) return 1;
  if (p->req_cpu > o->alloc_cpu[node] - (o->req_cpu[node] + delta[0])) return 0;
  if (p->req_mem > o->alloc_mem[node] - (o->req_mem[node] + delta[1])) return 0;
  if (p->req_eph > o->alloc_eph[node] - (o->req_eph[node] + delta[2])) return 0;
  for (int k = 0; k < o->n_scalar; k++) {
    const int64_t q = p->scalar_req[k];
    const size_t ix = (size_t)k * o->n + node;
    if (q != 0 && q > o->alloc_scalar[ix] - (o->req_scalar[ix] + delta[3 + k])) return 0;
  }
  return 1;
}

/* SelectVictimsOnNode: 1 + victims written to vout (importance order), or 0 */
static int32_t select_victims(const ksim_oracle* o, const ksim_pod* p, int32_t prio, const ksim_bound_pods* b,
                              int32_t node, const int64_t* nom, victim_rec* buf, int32_t* vout) {
  int32_t m = 0;
  for (int32_t i = 0; i < b->n; i++)
    if (b->node[i] == node && b->priority[i] < prio) {
      buf[m].idx = i;
      buf[m].prio = b->priority[i];
      buf[m].start = b->start_time[i];
      m++;
    }
  qsort(buf, (size_t)m, sizeof(victim_rec), victim_cmp);
  int64_t delta[KSIM_PREEMPT_REQ];
  for (int k = 0; k < KSIM_PREEMPT_REQ; k++) delta[k] = nom[k];
  for (int32_t j = 0; j < m; j++)
    for (int k = 0; k < KSIM_PREEMPT_REQ; k++) delta[k] -= b->req[(size_t)buf[j].idx * KSIM_PREEMPT_REQ + k];
  int64_t dpods = nom[KSIM_PREEMPT_REQ] - m;
  if (!fits_adjusted(o, p, node, delta, dpods)) return 0;
  int32_t nv = 0;
  for (int32_t j = 0; j < m; j++) {                      /* reprievePod, most important first */
    const int64_t* r = b->req + (size_t)buf[j].idx * KSIM_PREEMPT_REQ;
    for (int k = 0; k < KSIM_PREEMPT_REQ; k++) delta[k] += r[k];
    dpods++;
    if (!fits_adjusted(o, p, node, delta, dpods)) {
      for (int k = 0; k < KSIM_PREEMPT_REQ; k++) delta[k] -= r[k];
      dpods--;
      vout[nv++] = buf[j].idx;
    }
  }
  return 1 + nv;
}

int ksim_oracle_preempt(ksim_oracle* o, const ksim_pod_set* ps, int32_t pi, int32_t prio, const ksim_bound_pods* b,
                        ksim_preempt_out* out) {
  return ksim_oracle_preempt_nominated(o, ps, pi, prio, b, NULL, 0, NULL, NULL, NULL, out);
}

/* With the PodNominator's pods (ksim_engine.h ksim_preempt_nominated): a
 * grouped node's status is RunFilterPluginsWithNominatedPods' (pass 1 with the
 * group's pods assumed; pass 2 as is only when pass 1 passed), and
 * SelectVictimsOnNode keeps the group's requests on the node. */
int ksim_oracle_preempt_nominated(ksim_oracle* o, const ksim_pod_set* ps, int32_t pi, int32_t prio,
                                  const ksim_bound_pods* b, const ksim_pod_set* nps, int32_t n_groups,
                                  const int32_t* gnodes, const int32_t* first, const int32_t* count,
                                  ksim_preempt_out* out) {
  if (!o || !ps || !b || !out || pi < 0 || pi >= ps->n_pods || n_groups < 0) return KSIM_E_INVALID;
  if (n_groups > 0 && (!nps || !gnodes || !first || !count)) return KSIM_E_INVALID;
  for (int32_t k = 0; k < n_groups; k++)
    if (gnodes[k] < 0 || gnodes[k] >= o->n || first[k] < 0 || count[k] < 0 || first[k] + count[k] > nps->n_pods)
      return KSIM_E_INVALID;
  const ksim_pod* p = &ps->pods[pi];
  if (p->use_count > 0) return KSIM_E_UNSUPPORTED;
  const int32_t N = o->n;
  int fit = -1;
  for (int f = 0; f < o->prof.n_filter; f++)           /* the dry run re-runs Fit only */
    if (o->prof.filter[f] == KSIM_PL_NETWORK_BANDWIDTH) return KSIM_E_UNSUPPORTED;
  for (int f = 0; f < o->prof.n_filter; f++)
    if (o->prof.filter[f] == KSIM_PL_NODE_RESOURCES_FIT) fit = f;
  int32_t* group = (int32_t*)malloc(sizeof(int32_t) * (size_t)(N > 0 ? N : 1));
  uint8_t* gfail = (uint8_t*)malloc((size_t)(n_groups > 0 ? n_groups : 1));
  for (int32_t node = 0; node < N; node++) group[node] = -1;
  topo_ctx tc;
  for (int32_t k = 0; k < n_groups; k++) {               /* pass 1 of each grouped node */
    group[gnodes[k]] = k;
    for (int32_t j = first[k]; j < first[k] + count[k]; j++) assume_pod(o, nps, &nps->pods[j], gnodes[k], 1);
    topo_prefilter(o, ps, p, &tc);
    uint32_t det;
    gfail[k] = run_filter_plugins(o, ps, p, &tc, gnodes[k], &det);
    for (int32_t j = first[k]; j < first[k] + count[k]; j++) assume_pod(o, nps, &nps->pods[j], gnodes[k], -1);
  }
  topo_prefilter(o, ps, p, &tc);
  int32_t* potential = (int32_t*)malloc(sizeof(int32_t) * (size_t)(N > 0 ? N : 1));
  int32_t np = 0;
  for (int32_t node = 0; node < N; node++) {            /* nodesWherePreemptionMightHelp */
    uint32_t det;
    uint8_t f = run_filter_plugins(o, ps, p, &tc, node, &det);
    if (group[node] >= 0 && gfail[group[node]] != KSIM_PASSED) f = gfail[group[node]];
    if (fit >= 0 && f == (uint8_t)fit) potential[np++] = node;
  }
  int32_t want = np * o->prof.preempt_min_pct / 100;    /* GetOffsetAndNumCandidates / calculateNumCandidates */
  if (want < o->prof.preempt_min_abs) want = o->prof.preempt_min_abs;
  if (want > np) want = np;
  victim_rec* buf = (victim_rec*)malloc(sizeof(victim_rec) * (size_t)(b->n > 0 ? b->n : 1));
  int32_t* vic = (int32_t*)malloc(sizeof(int32_t) * (size_t)(b->n > 0 ? b->n : 1));
  int32_t* best_v = (int32_t*)malloc(sizeof(int32_t) * (size_t)(b->n > 0 ? b->n : 1));
  int32_t ncand = 0, best = -1, best_nv = 0;
  int32_t best_high = 0;
  int64_t best_sum = 0, best_start = 0;
  for (int32_t i = 0; i < np && ncand < want; i++) {
    const int32_t node = potential[i];
    int64_t nom[KSIM_PREEMPT_REQ + 1] = {0};            /* the group's requests and pod count */
    if (group[node] >= 0) {
      const int32_t k = group[node];
      for (int32_t j = first[k]; j < first[k] + count[k]; j++) {
        const ksim_pod* q = &nps->pods[j];
        nom[0] += q->req_cpu;
        nom[1] += q->req_mem;
        nom[2] += q->req_eph;
        for (int s2 = 0; s2 < KSIM_MAX_SCALAR; s2++) nom[3 + s2] += q->scalar_req[s2];
      }
      nom[KSIM_PREEMPT_REQ] = count[k];
    }
    const int32_t r = select_victims(o, p, prio, b, node, nom, buf, vic);
    if (r == 0) continue;
    ncand++;
    const int32_t nv = r - 1;
    /* pickOneNodeForPreemption criteria (no PDBs: no violations anywhere) */
    const int32_t high = nv ? b->priority[vic[0]] : INT32_MIN;
    int64_t sum = 0, early = INT64_MAX;
    for (int32_t j = 0; j < nv; j++) sum += (int64_t)b->priority[vic[j]] + ((int64_t)INT32_MAX + 1);
    for (int32_t j = 0; j < nv; j++)                    /* GetEarliestPodStartTime */
      if (b->priority[vic[j]] == high && b->start_time[vic[j]] < early) early = b->start_time[vic[j]];
    int better = best < 0;
    if (!better) {
      if (high != best_high) better = high < best_high;
      else if (sum != best_sum) better = sum < best_sum;
      else if (nv != best_nv) better = nv < best_nv;
      else if (early != best_start) better = early > best_start;
    }
    if (better) {
      best = node; best_nv = nv; best_high = high; best_sum = sum; best_start = early;
      memcpy(best_v, vic, sizeof(int32_t) * (size_t)nv);
    }
  }
  out->nominated = best;
  out->n_victims = best >= 0 ? best_nv : 0;
  out->n_potential = np;
  out->n_candidates = ncand;
  if (out->victims)
    for (int32_t j = 0; j < out->n_victims && j < out->victims_cap; j++) out->victims[j] = best_v[j];
  free(potential); free(buf); free(vic); free(best_v); free(group); free(gfail);
  return KSIM_OK;
}
