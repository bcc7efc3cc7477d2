/*
 * ksim_oracle.h — CPU restatement (ORACLE) of the per-pod scheduling cycle.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load libksim_oracle.so, and only as the
 * checker / reported CPU baseline.  The product path (libksim_engine.so) never
 * links, loads or falls back to it.
 *
 * Parity status: the plugin arithmetic lives in the third-party module
 * k8s.io/kubernetes v1.26.2 (simulator/go.mod:53), which is absent from the
 * reference checkout and cannot be fetched (no Go toolchain, no network).
 * This restatement follows SURVEY.md Appendix A; it is pinned by the
 * hand-derived known-answer vectors in tests/golden/ and the reference's own
 * contract tests restated in tests/, NOT by outputs of the Go plugins:
 * "parity unpinned vs Go" for the arithmetic.
 */
#ifndef KSIM_ORACLE_H
#define KSIM_ORACLE_H

#include "../include/ksim_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ksim_oracle ksim_oracle;

ksim_oracle* ksim_oracle_create(const ksim_node_table* nodes, const ksim_vocab* vocab,
                                const ksim_profile* profile);
void ksim_oracle_destroy(ksim_oracle* o);
/* ksim_engine.h ksim_upsert_nodes on the oracle's snapshot (0 on success). */
int ksim_oracle_upsert_nodes(ksim_oracle* o, const ksim_node_table* t, const ksim_vocab* v,
                             const int32_t* old_pos);

/* One scheduling cycle with full per-node outputs, sequential semantics
 * (parallelism 1), then assume/bind of the chosen node. */
int ksim_oracle_cycle(ksim_oracle* o, const ksim_pod_set* pods, int32_t pod_index,
                      ksim_eval_out* out);
int ksim_oracle_preempt(ksim_oracle* o, const ksim_pod_set* pods, int32_t pod_index, int32_t priority,
                        const ksim_bound_pods* b, ksim_preempt_out* out);
/* ksim_engine.h ksim_preempt_nominated. */
int ksim_oracle_preempt_nominated(ksim_oracle* o, const ksim_pod_set* ps, int32_t pi, int32_t prio,
                                  const ksim_bound_pods* b, const ksim_pod_set* nps, int32_t n_groups,
                                  const int32_t* nodes, const int32_t* first, const int32_t* count,
                                  ksim_preempt_out* out);
int ksim_oracle_cycle_ext(ksim_oracle* o, const ksim_pod_set* pods, int32_t pod_index, const uint8_t* ext_fail,
                          const int64_t* ext_score, ksim_eval_out* out);

/* Cycles for pods [first, first+count) without per-node outputs.
 * nthreads > 1 fans the node loop out over a thread pool (timing mode; results
 * identical to nthreads == 1). */
int ksim_oracle_schedule(ksim_oracle* o, const ksim_pod_set* pods, int32_t first,
                         int32_t count, int32_t* chosen, int nthreads,
                         ksim_batch_stats* stats);

/* Framework-driven compat mode (ksim_engine.h ksim_fw_*): Filter of every
 * node of the scan set, PreScore / Score / NormalizeScore over the
 * framework's list, NormalizeScore over an explicit list, assume / forget. */
int ksim_oracle_fw_filter(ksim_oracle* o, const ksim_pod_set* pods, int32_t pod_index, ksim_eval_out* out);
int ksim_oracle_fw_score(ksim_oracle* o, const ksim_pod_set* pods, int32_t pod_index, const int32_t* nodes,
                         int32_t n, ksim_eval_out* out);
int ksim_oracle_fw_normalize(ksim_oracle* o, int32_t slot, const int32_t* nodes, const int64_t* scores, int32_t n,
                             int64_t* out);
/* ksim_engine.h ksim_fw_filter_nominated for the framework cycle of pod pi of ps. */
int ksim_oracle_fw_filter_nominated(ksim_oracle* o, const ksim_pod_set* ps, int32_t pi, const ksim_pod_set* nps,
                                    int32_t n_nodes, const int32_t* nodes, const int32_t* first, const int32_t* count,
                                    uint8_t* fail_plugin, uint32_t* fail_detail);
int ksim_oracle_assume(ksim_oracle* o, const ksim_pod_set* pods, int32_t pod_index, int32_t node, int sign);
int ksim_oracle_get_node_state(const ksim_oracle* o, int64_t* req_cpu, int64_t* req_mem,
                               int64_t* req_eph, int64_t* nz_cpu, int64_t* nz_mem,
                               int32_t* num_pods);
int ksim_oracle_get_class_count(const ksim_oracle* o, int32_t* out);
int ksim_oracle_get_nb_alloc(const ksim_oracle* o, int64_t* out);
int32_t ksim_oracle_next_start(const ksim_oracle* o);
void ksim_oracle_set_next_start(ksim_oracle* o, int32_t s);
void ksim_oracle_set_pod_seq(ksim_oracle* o, int64_t seq);

/* Building blocks exported for known-answer tests. */
int32_t ksim_oracle_num_feasible_nodes_to_find(int32_t percentage, int32_t num_all_nodes);
int64_t ksim_oracle_least_requested_score(int64_t requested, int64_t capacity);
int64_t ksim_oracle_balanced_score(int32_t n, const int64_t* requested, const int64_t* allocatable);
int64_t ksim_oracle_most_requested_score(int64_t requested, int64_t capacity);
int64_t ksim_oracle_broken_linear(const ksim_profile* prof, int64_t p);
void    ksim_oracle_default_normalize(int64_t max_priority, int reverse, int32_t n, int64_t* scores);
uint64_t ksim_oracle_tb_key(int64_t total, uint64_t seed, int64_t pod_seq, int32_t node);
uint64_t ksim_oracle_tb_lo(uint64_t seed, int64_t pod_seq, int32_t node);

#ifdef __cplusplus
}
#endif
#endif
