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
