/* fwdrive.c — the drop-in's framework-driven cycle driven from C, as a cgo
 * host makes the calls (integration/go/engine/plugins.go, encoder.go): per
 * pod ksim_encode_pods + ksim_encoder_pods (its v1 pod's flat pool against
 * the snapshot), ksim_fw_prefilter (Filter of every node), the framework's
 * feasible list (the sequential worker's first K nodes in scan order from
 * nextStartNodeIndex), ksim_fw_score over it, ksim_fw_normalize per
 * NormalizeScore plugin with the raw scores Score returned, the highest total
 * (first in list order), ksim_assume.  bench.py --mode fw times the same
 * sequence from Python; this measures it without the ctypes glue.
 *
 * fwdrive_run_deltas adds what the Go host's incremental snapshot does around
 * the same cycle (integration/go/engine/encoder.go NativeEncoder, ABI 11):
 * the pod's flat pool copied into one fresh C allocation (the host's
 * pool.build), the encoder's membership bind after each Reserve, and informer
 * deltas between cycles -- external bound pods added (encode, ksim_assume,
 * ksim_encoder_bind) and deleted (encode, ksim_encoder_unbind, ksim_forget),
 * node updates (ksim_encoder_update_nodes, ksim_encoder_old_pos,
 * ksim_upsert_nodes) -- with the re-send check after every compile.
 *
 * Benchmark harness, not product code: the engine's entry points come in as
 * function pointers (the library variant bench.py loaded), and only the
 * public C-ABI of include/ksim_engine.h is used. */
#define _POSIX_C_SOURCE 199309L
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "ksim_engine.h"

typedef struct fwdrive_fns {
  int (*encode_pods)(ksim_encoder*, const ksim_k8s_pool*, const ksim_encode_pods_opts*);
  int (*encoder_pods)(const ksim_encoder*, ksim_pod_set*);
  int (*prefilter)(ksim_handle*, const ksim_pod_set*, int32_t, ksim_eval_out*);
  int (*score)(ksim_handle*, const int32_t*, int32_t, ksim_eval_out*);
  int (*normalize)(ksim_handle*, int32_t, const int32_t*, const int64_t*, int32_t, int64_t*);
  int (*assume)(ksim_handle*, const ksim_pod_set*, int32_t, int32_t);
} fwdrive_fns;

/* per-call seconds: encode, prefilter, score, normalize, assume; cycles with
 * a bind; total seconds */
typedef struct fwdrive_result {
  double sec[5];
  double total;
  int64_t bound;
  int64_t cycles;
} fwdrive_result;

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

/* Runs cycles over pools[0 .. n_pods).  n_nodes: the snapshot's nodes; k:
 * numFeasibleNodesToFind; nslots: the NormalizeScore plugins' score slots;
 * n_score: the profile's score plugins.  Returns 0 or the first failing
 * call's code. */
int fwdrive_run(const fwdrive_fns* f, ksim_handle* h, ksim_encoder* enc, const ksim_k8s_pool* const* pools,
                int32_t n_pods, const ksim_encode_pods_opts* opts, int32_t n_nodes, int32_t k, const int32_t* nslots,
                int32_t n_nslots, int32_t n_score, fwdrive_result* res) {
  const size_t N = (size_t)n_nodes;
  uint8_t* fail = (uint8_t*)malloc(N);
  int64_t* raw = (int64_t*)calloc((size_t)(n_score > 0 ? n_score : 1) * N, 8);
  int64_t* total = (int64_t*)calloc(N, 8);
  int32_t* list = (int32_t*)malloc(4 * N);
  int64_t* scores = (int64_t*)malloc(8 * N);
  int64_t* nout = (int64_t*)malloc(8 * N);
  int rc = 0;
  if (!fail || !raw || !total || !list || !scores || !nout) {
    rc = KSIM_E_INVALID;
    goto done;
  }
  memset(res, 0, sizeof(*res));
  ksim_eval_out fo, so;
  memset(&fo, 0, sizeof(fo));
  memset(&so, 0, sizeof(so));
  fo.fail_plugin = fail;
  so.raw = raw;
  so.total = total;
  int32_t ns = 0;
  const double t_start = now();
  for (int32_t i = 0; i < n_pods; i++) {
    ksim_pod_set ps;
    double t0 = now();
    if ((rc = f->encode_pods(enc, pools[i], opts)) || (rc = f->encoder_pods(enc, &ps))) goto done;
    double t1 = now();
    if ((rc = f->prefilter(h, &ps, 0, &fo))) goto done;
    double t2 = now();
    res->sec[0] += t1 - t0;
    res->sec[1] += t2 - t1;
    /* the framework's list: the first k feasible nodes in scan order */
    int32_t n = 0, proc = (int32_t)N;
    for (int32_t j = 0; j < (int32_t)N; j++) {
      const int32_t x = (int32_t)(((size_t)ns + (size_t)j) % N);
      if (fail[x] != KSIM_PASSED) continue;
      if (n == k) {
        proc = j;
        break;
      }
      list[n++] = x;
    }
    ns = (int32_t)(((size_t)ns + (size_t)proc) % N);
    if (n == 0) continue;
    int32_t node = list[0];
    if (n > 1) {
      t0 = now();
      if ((rc = f->score(h, list, n, &so))) goto done;
      t1 = now();
      for (int32_t q = 0; q < n_nslots; q++) {
        const int64_t* r = raw + (size_t)nslots[q] * N;
        for (int32_t j = 0; j < n; j++) scores[j] = r[list[j]];
        if ((rc = f->normalize(h, nslots[q], list, scores, n, nout))) goto done;
      }
      t2 = now();
      res->sec[2] += t1 - t0;
      res->sec[3] += t2 - t1;
      int64_t best = total[list[0]];
      for (int32_t j = 1; j < n; j++)
        if (total[list[j]] > best) {
          best = total[list[j]];
          node = list[j];
        }
    }
    t0 = now();
    if ((rc = f->assume(h, &ps, 0, node))) goto done;
    res->sec[4] += now() - t0;
    res->bound++;
  }
  res->total = now() - t_start;
  res->cycles = n_pods;
done:
  free(fail);
  free(raw);
  free(total);
  free(list);
  free(scores);
  free(nout);
  return rc;
}

/* ---- the incremental-snapshot cycle ------------------------------------------------ */
typedef struct fwdrive_delta_fns {
  int (*encoder_bind)(ksim_encoder*, int32_t, int32_t);
  int (*encoder_unbind)(ksim_encoder*, const char*, const char*, int32_t*);
  int (*encoder_update_nodes)(ksim_encoder*, const ksim_k8s_pool*, const int32_t*, int32_t);
  int (*encoder_old_pos)(const ksim_encoder*, int32_t*);
  int (*encoder_cluster)(const ksim_encoder*, ksim_node_table*, ksim_vocab*);
  int (*encoder_info)(const ksim_encoder*, ksim_encoder_info*);
  int (*upsert_nodes)(ksim_handle*, const ksim_node_table*, const ksim_vocab*, const int32_t*);
  int (*forget)(ksim_handle*, const ksim_pod_set*, int32_t, int32_t);
  int (*encoder_changed_rows)(const ksim_encoder*, int32_t*, int32_t);
  int (*update_node_rows)(ksim_handle*, const ksim_node_table*, const ksim_vocab*, const int32_t*, int32_t);
} fwdrive_delta_fns;

typedef struct fwdrive_deltas {
  const ksim_k8s_pool* const* ext;        /* bound pods an informer adds (spec.nodeName set) */
  const char* const* ext_ns;
  const char* const* ext_name;
  const int32_t* ext_node;                /* their node positions */
  int32_t n_ext, ext_every, lag;          /* an add every ext_every cycles; the add `lag` adds back is deleted */
  const ksim_k8s_pool* const* node_upd;   /* one updated node each */
  int32_t n_node_upd, node_every;
} fwdrive_deltas;

/* sec: encode, prefilter, score, normalize, assume (+ bind), deltas, pool build */
typedef struct fwdrive_delta_result {
  double sec[7];
  double total;
  int64_t bound, cycles, pod_adds, pod_deletes, node_updates, resends, node_rows_in_place;
} fwdrive_delta_result;

/* the host's pool.build (encoder.go): the flat pool into one fresh C allocation */
static ksim_k8s_pool* copy_pool(const ksim_k8s_pool* s) {
  size_t sizes[22], total = sizeof(ksim_k8s_pool);
  const void* src[22];
  int k = 0;
#define PART(ptr, n, one) do { src[k] = (ptr); sizes[k] = (size_t)(n) * (one); total += (sizes[k] + 15) & ~(size_t)15; k++; } while (0)
  PART(s->strings, s->n_strings ? s->str_off[s->n_strings] : 0, 1);
  PART(s->str_off, s->n_strings + 1, 8);
  PART(s->str_list, s->n_str_list, 4);
  PART(s->kv, s->n_kv, sizeof(ksim_k8s_kv));
  PART(s->taints, s->n_taints, sizeof(ksim_k8s_taint));
  PART(s->tolerations, s->n_tolerations, sizeof(ksim_k8s_toleration));
  PART(s->reqs, s->n_reqs, sizeof(ksim_k8s_requirement));
  PART(s->terms, s->n_terms, sizeof(ksim_k8s_selector_term));
  PART(s->preferred, s->n_preferred, sizeof(ksim_k8s_preferred_term));
  PART(s->selectors, s->n_selectors, sizeof(ksim_k8s_label_selector));
  PART(s->pod_terms, s->n_pod_terms, sizeof(ksim_k8s_pod_term));
  PART(s->spread, s->n_spread, sizeof(ksim_k8s_spread));
  PART(s->ports, s->n_ports, sizeof(ksim_k8s_port));
  PART(s->containers, s->n_containers, sizeof(ksim_k8s_container));
  PART(s->images, s->n_images, sizeof(ksim_k8s_image));
  PART(s->volume_groups, s->n_volume_groups, sizeof(ksim_k8s_volume_group));
  PART(s->nodes, s->n_nodes, sizeof(ksim_k8s_node));
  PART(s->pods, s->n_pods, sizeof(ksim_k8s_pod));
  PART(s->namespaces, s->n_namespaces, sizeof(ksim_k8s_namespace));
  PART(s->services, s->n_services, sizeof(ksim_k8s_service));
  PART(s->controllers, s->n_controllers, sizeof(ksim_k8s_controller));
#undef PART
  char* base = (char*)malloc(total);
  if (!base) return NULL;
  ksim_k8s_pool* d = (ksim_k8s_pool*)base;
  *d = *s;
  void* dst[22];
  size_t at = sizeof(ksim_k8s_pool);
  for (int i = 0; i < k; i++) {
    dst[i] = sizes[i] ? base + at : NULL;
    if (sizes[i]) memcpy(dst[i], src[i], sizes[i]);
    at += (sizes[i] + 15) & ~(size_t)15;
  }
  d->strings = (const char*)dst[0];
  d->str_off = (const int64_t*)dst[1];
  d->str_list = (const int32_t*)dst[2];
  d->kv = (const ksim_k8s_kv*)dst[3];
  d->taints = (const ksim_k8s_taint*)dst[4];
  d->tolerations = (const ksim_k8s_toleration*)dst[5];
  d->reqs = (const ksim_k8s_requirement*)dst[6];
  d->terms = (const ksim_k8s_selector_term*)dst[7];
  d->preferred = (const ksim_k8s_preferred_term*)dst[8];
  d->selectors = (const ksim_k8s_label_selector*)dst[9];
  d->pod_terms = (const ksim_k8s_pod_term*)dst[10];
  d->spread = (const ksim_k8s_spread*)dst[11];
  d->ports = (const ksim_k8s_port*)dst[12];
  d->containers = (const ksim_k8s_container*)dst[13];
  d->images = (const ksim_k8s_image*)dst[14];
  d->volume_groups = (const ksim_k8s_volume_group*)dst[15];
  d->nodes = (const ksim_k8s_node*)dst[16];
  d->pods = (const ksim_k8s_pod*)dst[17];
  d->namespaces = (const ksim_k8s_namespace*)dst[18];
  d->services = (const ksim_k8s_service*)dst[19];
  d->controllers = (const ksim_k8s_controller*)dst[20];
  return d;
}

typedef struct dstate {
  const fwdrive_fns* f;
  const fwdrive_delta_fns* g;
  ksim_handle* h;
  ksim_encoder* enc;
  const ksim_encode_pods_opts* opts;
  int32_t layout[2];
  int32_t* keep;
  int32_t n_nodes;
  fwdrive_delta_result* res;
} dstate;

/* the compile grew the label columns or classes: the table again, every node kept */
static int resend(dstate* s) {
  ksim_encoder_info in;
  int rc = s->g->encoder_info(s->enc, &in);
  if (rc) return rc;
  if (in.n_label_cols == s->layout[0] && in.n_classes == s->layout[1]) return 0;
  ksim_node_table t;
  ksim_vocab v;
  if ((rc = s->g->encoder_cluster(s->enc, &t, &v))) return rc;
  for (int32_t i = 0; i < t.n_nodes; i++) s->keep[i] = i;
  if ((rc = s->g->upsert_nodes(s->h, &t, &v, s->keep))) return rc;
  s->layout[0] = in.n_label_cols;
  s->layout[1] = in.n_classes;
  s->res->resends++;
  return 0;
}

static int pod_add(dstate* s, const ksim_k8s_pool* pool, int32_t node) {
  ksim_pod_set ps;
  int rc;
  if ((rc = s->f->encode_pods(s->enc, pool, s->opts)) || (rc = s->f->encoder_pods(s->enc, &ps)) || (rc = resend(s)))
    return rc;
  if ((rc = s->f->encoder_pods(s->enc, &ps)) || (rc = s->f->assume(s->h, &ps, 0, node))) return rc;
  if ((rc = s->g->encoder_bind(s->enc, 0, node))) return rc;
  s->res->pod_adds++;
  return 0;
}

static int pod_delete(dstate* s, const ksim_k8s_pool* pool, const char* ns, const char* name) {
  ksim_pod_set ps;
  int32_t pos = -1;
  int rc;
  if ((rc = s->f->encode_pods(s->enc, pool, s->opts)) || (rc = resend(s))) return rc;
  if ((rc = s->f->encoder_pods(s->enc, &ps)) || (rc = s->g->encoder_unbind(s->enc, ns, name, &pos))) return rc;
  if ((rc = s->g->forget(s->h, &ps, 0, pos))) return rc;
  s->res->pod_deletes++;
  return 0;
}

static int node_update(dstate* s, const ksim_k8s_pool* pool, int32_t* old_pos) {
  int rc;
  if ((rc = s->g->encoder_update_nodes(s->enc, pool, NULL, 0))) return rc;
  ksim_node_table t;
  ksim_vocab v;
  if ((rc = s->g->encoder_cluster(s->enc, &t, &v))) return rc;
  int32_t rows[8];
  const int k = s->g->encoder_changed_rows(s->enc, rows, 8);
  if (k >= 0 && k <= 8) {                      /* in place: the updated rows only */
    if ((rc = s->g->update_node_rows(s->h, &t, &v, rows, k))) return rc;
    s->res->node_rows_in_place++;
  } else {
    if ((rc = s->g->encoder_old_pos(s->enc, old_pos)) || (rc = s->g->upsert_nodes(s->h, &t, &v, old_pos))) return rc;
  }
  s->res->node_updates++;
  return 0;
}

int fwdrive_run_deltas(const fwdrive_fns* f, const fwdrive_delta_fns* g, ksim_handle* h, ksim_encoder* enc,
                       const ksim_k8s_pool* const* pools, int32_t n_pods, const ksim_encode_pods_opts* opts,
                       int32_t n_nodes, int32_t k, const int32_t* nslots, int32_t n_nslots, int32_t n_score,
                       const fwdrive_deltas* dl, fwdrive_delta_result* res) {
  const size_t N = (size_t)n_nodes;
  uint8_t* fail = (uint8_t*)malloc(N);
  int64_t* raw = (int64_t*)calloc((size_t)(n_score > 0 ? n_score : 1) * N, 8);
  int64_t* total = (int64_t*)calloc(N, 8);
  int32_t* list = (int32_t*)malloc(4 * N);
  int64_t* scores = (int64_t*)malloc(8 * N);
  int64_t* nout = (int64_t*)malloc(8 * N);
  int32_t* keep = (int32_t*)malloc(4 * N);
  int32_t* old_pos = (int32_t*)malloc(4 * N);
  int rc = 0;
  memset(res, 0, sizeof(*res));
  dstate s = {f, g, h, enc, opts, {0, 0}, keep, n_nodes, res};
  if (!fail || !raw || !total || !list || !scores || !nout || !keep || !old_pos) {
    rc = KSIM_E_INVALID;
    goto done;
  }
  {
    ksim_encoder_info in;
    if ((rc = g->encoder_info(enc, &in))) goto done;
    s.layout[0] = in.n_label_cols;
    s.layout[1] = in.n_classes;
  }
  ksim_eval_out fo, so;
  memset(&fo, 0, sizeof(fo));
  memset(&so, 0, sizeof(so));
  fo.fail_plugin = fail;
  so.raw = raw;
  so.total = total;
  int32_t ns = 0, adds = 0, nupd = 0;
  const double t_start = now();
  for (int32_t i = 0; i < n_pods; i++) {
    double t0 = now();
    /* the informer events queued since the last cycle (Snapshot) */
    if (dl && dl->ext_every > 0 && i % dl->ext_every == 0 && adds < dl->n_ext) {
      if ((rc = pod_add(&s, dl->ext[adds], dl->ext_node[adds]))) goto done;
      if (adds >= dl->lag) {
        const int32_t j = adds - dl->lag;
        if ((rc = pod_delete(&s, dl->ext[j], dl->ext_ns[j], dl->ext_name[j]))) goto done;
      }
      adds++;
    }
    if (dl && dl->node_every > 0 && i % dl->node_every == dl->node_every - 1 && dl->n_node_upd > 0) {
      if ((rc = node_update(&s, dl->node_upd[nupd % dl->n_node_upd], old_pos))) goto done;
      nupd++;
    }
    double t1 = now();
    res->sec[5] += t1 - t0;
    ksim_k8s_pool* own = copy_pool(pools[i]);
    if (!own) {
      rc = KSIM_E_OOM;
      goto done;
    }
    double t2 = now();
    res->sec[6] += t2 - t1;
    ksim_pod_set ps;
    rc = f->encode_pods(enc, own, opts);
    free(own);
    if (rc || (rc = f->encoder_pods(enc, &ps)) || (rc = resend(&s)) || (rc = f->encoder_pods(enc, &ps))) goto done;
    double t3 = now();
    if ((rc = f->prefilter(h, &ps, 0, &fo))) goto done;
    double t4 = now();
    res->sec[0] += t3 - t2;
    res->sec[1] += t4 - t3;
    int32_t n = 0, proc = (int32_t)N;
    for (int32_t j = 0; j < (int32_t)N; j++) {
      const int32_t x = (int32_t)(((size_t)ns + (size_t)j) % N);
      if (fail[x] != KSIM_PASSED) continue;
      if (n == k) {
        proc = j;
        break;
      }
      list[n++] = x;
    }
    ns = (int32_t)(((size_t)ns + (size_t)proc) % N);
    if (n == 0) continue;
    int32_t node = list[0];
    if (n > 1) {
      t0 = now();
      if ((rc = f->score(h, list, n, &so))) goto done;
      t1 = now();
      for (int32_t q = 0; q < n_nslots; q++) {
        const int64_t* r = raw + (size_t)nslots[q] * N;
        for (int32_t j = 0; j < n; j++) scores[j] = r[list[j]];
        if ((rc = f->normalize(h, nslots[q], list, scores, n, nout))) goto done;
      }
      t2 = now();
      res->sec[2] += t1 - t0;
      res->sec[3] += t2 - t1;
      int64_t best = total[list[0]];
      for (int32_t j = 1; j < n; j++)
        if (total[list[j]] > best) {
          best = total[list[j]];
          node = list[j];
        }
    }
    t0 = now();
    if ((rc = f->assume(h, &ps, 0, node)) || (rc = g->encoder_bind(enc, 0, node))) goto done;
    res->sec[4] += now() - t0;
    res->bound++;
  }
  res->total = now() - t_start;
  res->cycles = n_pods;
done:
  free(fail);
  free(raw);
  free(total);
  free(list);
  free(scores);
  free(nout);
  free(keep);
  free(old_pos);
  return rc;
}
