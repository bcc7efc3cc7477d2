// ksim_internal.h — launcher interface between the host runtime
// (ksim_engine.cpp) and the kernels (ksim_kernels.hip).
#pragma once

#include "ksim_device.h"

namespace ksim {

// A/B forms of the same runs, chosen at compile time (csrc/Makefile "ab":
// libksim_engine_ab.so, every alternative form on; tests/test_gpu_ab_switches.py
// runs it against the oracle).  The product library has none of them.
// KSIM_AB_FORMS is a bitmask of the alternative forms (csrc/Makefile "ab":
// 127, every one on; "abforms": one form each, checked against the product's
// other forms):
constexpr unsigned kAbStab = 1;      // per-node static plugins (no static-class table)
constexpr unsigned kAbLazy = 2;      // three-launch batches (commit as its own launch)
constexpr unsigned kAbAdaptNorm = 4; // ADAPT normalized-score pods on the per-pod path
constexpr unsigned kAbTbatch = 8;    // topology pods on the per-pod path
constexpr unsigned kAbShardGraph = 16;   // eager shard cycles (no shard-group graphs)
constexpr unsigned kAbPtab = 32;     // per-cycle PreFilter domain sums (no persistent tables)
constexpr unsigned kAbTbVar = 64;    // topology batches end at a zone-keyed class conflict (no zone variants)
#ifdef KSIM_AB_FORMS
constexpr unsigned kAbMask = KSIM_AB_FORMS;
#else
constexpr unsigned kAbMask = 0;
#endif
constexpr bool ab(unsigned form) { return (kAbMask & form) != 0; }


// Batch path geometry.
// Compile-time overridable for A/B builds (-DKSIM_BATCH_PODS=512 -DKSIM_TOP_T=16).
#ifndef KSIM_BATCH_PODS
#define KSIM_BATCH_PODS 256
#endif
#ifndef KSIM_TOP_T
#define KSIM_TOP_T 8
#endif
constexpr int kBatchPods = KSIM_BATCH_PODS;   // B: pods per speculative batch
constexpr int kTopT = KSIM_TOP_T;             // T: candidate keys kept per pod
constexpr int kMaxListRecords = 4;            // list records per pod (ksim_batch.hip kNsSlices)
static_assert(kBatchPods % 64 == 0 && kBatchPods <= 1024 && kTopT <= 64, "batch geometry");
constexpr int kTopThreads = 1024;  // threads per pod of the batch top
constexpr int kTileCand = 4;       // best keys each lane of the batch top keeps per pod
constexpr int kXRec = kTopT + 1;   // sharded exchange record per pod: T keys + (count | complete << 32)
#ifndef KSIM_MAX_SHARDS
#define KSIM_MAX_SHARDS 8
#endif
constexpr int kMaxShards = KSIM_MAX_SHARDS;   // shards of one simulation (one per GPU of a node)
constexpr int kGmergeSlots = (kTopT * kMaxShards + 63) / 64;   // list entries per lane in k_batch_gmerge
static_assert(kGmergeSlots <= 2, "gmerge geometry");

// In-process shard group (one device): the pmax arrays of up to kMaxShards handles.
struct GroupPtrs {
  uint64_t* p[kMaxShards];
  int32_t n;
};

struct LaunchArgs {
  DevCluster c;
  DevPods P;
  ksim_profile prof;
  BatchProg bp;
  DevState* st;
  DevScratch s;
  DevEvalOut o;
  int32_t* chosen;   // [n_pods] device, may be null
  const ksim_profile* dprof = nullptr;   // device copies of prof / bp (the batch kernels read these)
  const BatchProg* dbp = nullptr;
  bool fast = false; // batch runs: every pod trivial and cpu/memory scoring (k_batch_top<true>)
  bool stab = false; // ... or (with fast) every pod in a static class (DevPods::stab; the STAB kernels)
  bool fuse_min = false;  // per-pod topology runs: every hard spread key has <= 256 values
  bool fuse_ext = false;  // per-pod runs: every pod has <= 1 ScheduleAnyway spread constraint (K = N: no k_extrema)
  bool ptab = false;      // per-pod topology runs: every pod carries kPlanPtab (no k_topo_prefilter)
};

constexpr int kKernelsPerCycle = 7;
constexpr int kFuseMinValues = 256;   // k_filter_score computes the PTS critical paths itself up to this many values
extern const char* const kKernelNames[kKernelsPerCycle];
constexpr int kKernelsPerBatch = 3;
extern const char* const kBatchKernelNames[kKernelsPerBatch];
constexpr int kKernelsPerAdapt = 5;
extern const char* const kAdaptKernelNames[kKernelsPerAdapt];
// Topology batch path (ksim_tbatch.hip): at most kTbPods pods per batch (the
// host's runs, bflags >> kTlenShift), clusters of at most kTbMaxBlocks node
// blocks of 256.  A run may cross a class an earlier pod of it adds when every
// use that reads it is node-local (tbatch_conflict_ok; the pairs step re-keys
// the guessed node; the run's first pod carries kPodTbCross).
constexpr int kTbPods = 32;
constexpr int kTbMaxBlocks = 64;
constexpr int kKernelsPerTbatch = 5;
extern const char* const kTbatchKernelNames[kKernelsPerTbatch];
uint32_t launch_tbatch(const LaunchArgs& a, hipStream_t stream, hipEvent_t* evs = nullptr);
// Replicated topology batches (every replica holds the whole snapshot and
// evaluates its node range [c.eval_lo, c.eval_hi)); the caller exchanges
// between the phases:
//   launch_tb_rep_filter   filter + raw scores + per-pod counters / extrema
//                          (all-gather s.tb_win -> s.tb_xrecv [world][kTbPods])
//   launch_tb_rep_select   merged counters, totals + keys, holders, the
//                          replica's per-pod top-T record
//                          (all-gather s.xsend -> s.xrecv [world][kTbPods][kTbXRec])
//   launch_tb_rep_pairs    global top-T, chain, pair keys of the guesses this
//                          replica evaluated (all-reduce max s.tb_pp)
//   launch_tb_rep_commit   commit on every replica (every bind, every class add)
constexpr int kTbXRec = kTopT + 1 + KSIM_MAX_SCORE;   // T keys, count, holder counts (2 x int32 per slot)
void launch_tb_rep_filter(const LaunchArgs& a, hipStream_t stream);
void launch_tb_rep_select(const LaunchArgs& a, int32_t world, hipStream_t stream);
void launch_tb_rep_pairs(const LaunchArgs& a, int32_t world, hipStream_t stream);
void launch_tb_rep_commit(const LaunchArgs& a, hipStream_t stream);

// One scheduling cycle for the pod at st->cursor (no-op once cursor >= end).
// evs (nullable, kKernelsPerCycle + 1 events) are recorded around each kernel.
// topo: the pod may carry PodTopologySpread / InterPodAffinity uses (adds the
// two topology kernels; they exit at once for a pod without uses).
// Returns the kernel slots it launched (bit k: kernel k of the cycle), so a
// timing run counts only those.
uint32_t launch_cycle(const LaunchArgs& a, hipStream_t stream, bool compat, bool topo, hipEvent_t* evs = nullptr);
// One speculative batch of up to kBatchPods pods from st->cursor (>= 1 committed).
// Returns the mask of kernel slots launched (bit k: kBatchKernelNames[k]).
unsigned long long* adapt_dbg_buffer();  // KSIM_ADAPT_DBG builds: why ADAPT batches end short (else null)
unsigned long long* cp_clock_buffer();   // KSIM_CP_CLOCKS builds: chain + pairs phase clocks (else null)
uint32_t launch_batch(const LaunchArgs& a, hipStream_t stream, hipEvent_t* evs = nullptr);
// The same under ADAPT (K < N): windows by relaxation, see ksim_adapt.hip.
uint32_t launch_batch_adapt(const LaunchArgs& a, hipStream_t stream, hipEvent_t* evs = nullptr);

// ---- deferred-commit FAST batches (ksim_batch.hip k_batch_top_commit) ---------
// Batch i's commit runs inside batch i+1's evaluation launch: two launches per
// batch instead of three.  The dynamic node columns are double-buffered: batch
// i evaluates the snapshot X[p ^ 1] (p = i & 1) that batch i-1 evaluated, plus
// batch i-1's binds as an overlay, and writes S_i into X[p] for the nodes batch
// i-1 or i-2 bound (X[p] held S_{i-2}); its chain + pairs then read X[p].  The
// chain + pairs outputs (guess keys, pair maxima, prefix length) live in a
// ring of kLazySlots slots, slot i & 3.  X[0] and st[0] are the handle's own.
constexpr int kLazySlots = 4;
constexpr int kLazyMaxNodes = 1 << 17;   // the overlay's LDS node bitmap (16 KB)
constexpr int kLazyHashBits = 10;        // overlay hash: node -> entry, >= 4 x kBatchPods slots
struct DynCols {
  int64_t *req_cpu, *req_mem, *req_eph, *nz_cpu, *nz_mem;
  int32_t* num_pods;
};
struct LazyStep {
  DynCols w;                                       // X[p]: receives S_i
  const DevState* st_in;                           // st[p ^ 1]: the state batch i-1 started from
  DevState* st_out;                                // st[p]: after batch i-1's commit
  const uint64_t* g1; const uint64_t* m1; const int32_t* e1;   // batch i-1's slot: guesses, pair maxima, prefix
  const uint64_t* g2; const int32_t* e2;                       // batch i-2's slot: guesses, prefix
  int32_t* e_self;                                 // batch i's slot (a flush marks it empty: -1)
};
struct LazyBatch {
  LaunchArgs a;        // a.c: static columns + X[p ^ 1]
  DevCluster cw;       // static columns + X[p]
  LazyStep step;
  DevState* st;        // st[p]
  uint64_t* gkey;      // batch i's slot
  uint64_t* pmax;
  int32_t* cend;
  // ADAPT: batch i-1's broken-window flags and windows, batch i's slot of them
  const int32_t* b1;
  const int32_t* w1;
  int32_t* abroken;
  int32_t* awin;
};
constexpr int kKernelsPerLazy = 2;
extern const char* const kLazyKernelNames[kKernelsPerLazy];
// ADAPT (ksim_adapt.hip): k_adapt_mask_commit (commit of i-1, the S_i bitmaps
// of i, every row written to X[p]), the window scan when not fused into the
// top, the top, the chain + pairs.  X[p] is written whole, so only batch i-1's
// slot is read.
constexpr int kKernelsPerLazyAdapt = 4;
extern const char* const kLazyAdaptKernelNames[kKernelsPerLazyAdapt];
uint32_t launch_batch_adapt_lazy(const LazyBatch& z, hipStream_t stream, hipEvent_t* evs = nullptr);
void launch_adapt_lazy_flush(const LazyBatch& z, hipStream_t stream);
// batch i: k_batch_top_commit (commit of i-1, evaluation of i), then the
// chain + pairs of i.  A flush is the first launch alone with no evaluation:
// it commits batch i-1 and leaves slot i empty.
// DevPods::stab rows of classes [0, n_cls) (ksim_batch.hip k_static_table)
void launch_static_table(const LaunchArgs& a, const int32_t* rep, int32_t n_cls, uint64_t* stab, hipStream_t stream);
uint32_t launch_batch_lazy(const LazyBatch& z, hipStream_t stream, hipEvent_t* evs = nullptr);
void launch_lazy_flush(const LazyBatch& z, hipStream_t stream);
// the evaluation-launch instantiations launched so far (ksim_get_diag out[25])
uint64_t batch_variant_reach();
void launch_lazy_top(const LazyBatch& z, hipStream_t stream);   // the first launch alone (ksim_time_eval)
// replicated handles: the first launch with the replica's record (xsend), then,
// after the records' all-gather into a.s.xrecv, the global merge + chain + pairs
void launch_lazy_top_rep(const LazyBatch& z, uint64_t* xsend, hipStream_t stream);
void launch_lazy_chain_rep(const LazyBatch& z, int32_t world, hipStream_t stream);
// Compat cycle around the host's extender round trip (ksim_eval_pod_filter / _finish):
// the filter pass + window, then (a.s.ext_fail / ext_score set) the rest.
void launch_cycle_filter(const LaunchArgs& a, hipStream_t stream, bool topo);
void launch_cycle_finish(const LaunchArgs& a, hipStream_t stream);
// Framework-driven compat cycle (ksim_fw_*): Filter of every scanned node; then
// PreScore / Score / NormalizeScore over the framework's list (a.s.ext_fail =
// 1 for unlisted nodes), no bind; NormalizeScore of one slot over an explicit list.
void launch_fw_filter(const LaunchArgs& a, hipStream_t stream, bool topo);
void launch_fw_score(const LaunchArgs& a, hipStream_t stream);
constexpr int kCopyPieces = 8;
struct CopyList {
  const uint8_t* src[kCopyPieces];
  uint8_t* dst[kCopyPieces];
  uint32_t n[kCopyPieces];
  // optional (bst non-null): a framework-driven filter pass's start in the same
  // launch (launch_fw_begin's work, by block (0, 0))
  DevState* bst;
  WinState* bwin;
  int32_t bfirst, bend;
  // optional (anode >= 0): a queued Reserve / Unreserve (assume_pod of pod 0 of
  // aP on node anode, sign asign) in the same launch, by block (0, 0)
  int32_t anode, asign;
  DevCluster ac;
  DevPods aP;
};
void launch_copy_list(const CopyList& l, int count, hipStream_t stream);
// ksim_update_node_rows: packed static-column records of n rows (words int64 each)
void launch_node_rows(const DevCluster& c, const int64_t* rec, int32_t n, int32_t words, hipStream_t stream);
void launch_fw_gather(const DevEvalOut& o, const int32_t* nodes, int32_t n, int32_t N, int32_t S, int64_t* comp,
                      const WinState* win, void* win_out, hipStream_t stream);
void launch_fw_begin(DevState* st, WinState* win, int32_t first, int32_t end, hipStream_t stream);
void launch_fw_normalize(const LaunchArgs& a, int32_t slot, const int32_t* nodes, const int64_t* vals, int32_t n,
                         int64_t* out, hipStream_t stream);
// DefaultPreemption dry run (ksim_preempt.hip): the bound pods per node in
// importance order (CSR over nodes), per-node results, the pick.
struct PreemptNode {
  int32_t potential, cand, nv, high;   // potential node, candidate, victims, highest victim priority
  int64_t sum, early;                  // sum of (priority + 2^31), earliest start of the highest-priority victims
};
struct DevPreempt {
  const int32_t* off;                  // [n + 1]
  const int32_t* prio;                 // [n_bound] CSR order
  const int64_t* start;                // [n_bound]
  const int64_t* req;                  // [n_bound][KSIM_PREEMPT_REQ]
  uint8_t* vflag;                      // [n_bound] victim of its node's dry run
  PreemptNode* res;                    // [n]
  int32_t* pick;                       // [4] nominated, victims, potential, candidates
  int32_t* nslot;                      // [n] nominated group of the node, -1: none
  const int64_t* nreq;                 // [groups][KSIM_PREEMPT_REQ + 1] requests, pod count
};
// filter = false: s.fail already holds the statuses (ksim_preempt_nominated)
void launch_preempt(const LaunchArgs& a, const DevPreempt& pre, int32_t fit_index, int32_t prio, hipStream_t stream,
                    bool filter = true);

// The evaluation kernels alone (ksim_time_eval).
void launch_batch_eval_only(const LaunchArgs& a, hipStream_t stream);
void launch_filter_only(const LaunchArgs& a, hipStream_t stream);
// Sharded batch (node shards; the caller exchanges between the phases):
//   launch_shard_eval    batch top; writes this shard's records to s.xsend
//   (all-gather s.xsend -> s.xrecv [world][kBatchPods][kXRec])
//   launch_shard_chain   global merge + chain + pair keys of owned guesses -> s.pmax
//   (all-reduce max s.pmax)
//   launch_shard_commit  validate + commit (owner shard binds)
void launch_shard_eval(const LaunchArgs& a, hipStream_t stream);
// records all-gathered in s.xrecv ([world][kBatchPods][kXRec]) -> per-pod global top-T
void k_batch_gmerge_launch(const LaunchArgs& a, int32_t world, hipStream_t stream);
// node-sharded ADAPT batch (ksim_adapt.hip): shard bitmaps of W words per pod
// -> all-gather -> windows + this shard's records -> all-gather -> chain +
// pairs (s.pmax: [M | broken]) -> all-reduce (max) -> commit
void launch_adapt_sh_mask(const LaunchArgs& a, uint64_t* send, int32_t W, hipStream_t stream);
void launch_adapt_sh_window(const LaunchArgs& a, const uint64_t* recv, int32_t W, uint64_t* gmask, hipStream_t stream);
void launch_adapt_sh_pairs(const LaunchArgs& a, const uint64_t* gmask, int32_t world, hipStream_t stream);
void launch_adapt_sh_commit(const LaunchArgs& a, hipStream_t stream);
void launch_shard_chain(const LaunchArgs& a, int32_t world, hipStream_t stream);
void launch_shard_commit(const LaunchArgs& a, hipStream_t stream);
void launch_group_max(const GroupPtrs& g, hipStream_t stream);
// Sharded per-pod cycle (node shards; the caller exchanges between the phases,
// see ksim_kernels.hip §C):
//   launch_pshard_topo     prefilter + pack           (all-reduce sum s.xdom)
//   launch_pshard_filter   [topo min] + filter + counts (all-gather s.xsend[2] -> s.xrecv[world][2])
//   launch_pshard_window   cut / kept / registrations (all-reduce sum s.xreg; pods with soft spread)
//   launch_pshard_extrema  weights + extrema            (all-reduce max win->ext[kExtWords])
//   launch_pshard_select   totals + TB pair, shard best  (all-gather s.xsend[2] -> s.xrecv[world][2])
//   launch_pshard_bind     selectHost over the shards, owner binds
void launch_pshard_topo(const LaunchArgs& a, hipStream_t stream);
void launch_pshard_filter(const LaunchArgs& a, bool topo, hipStream_t stream);
void launch_pshard_window(const LaunchArgs& a, int32_t rank, int32_t world, hipStream_t stream);
void launch_pshard_extrema(const LaunchArgs& a, bool soft, hipStream_t stream);
void launch_pshard_select(const LaunchArgs& a, hipStream_t stream);
void launch_pshard_bind(const LaunchArgs& a, int32_t world, hipStream_t stream);
void launch_group_reduce(const GroupPtrs& g, int64_t count, bool op_max, hipStream_t stream);
void launch_group_gather(const GroupPtrs& src, const GroupPtrs& dst, int32_t words, hipStream_t stream);
// Persistent domain tables of a loaded queue (DevPods.ptab) from the class counts.
void launch_ptab_init(const DevCluster& c, const DevPods& P, hipStream_t stream);
// ksim_reset_cluster: copies (or zeroes, src null) of 16-byte-aligned buffers in one launch
struct ResetList {
  static constexpr int kMax = 12;
  int n = 0;
  uint32_t* dst[kMax];
  const uint32_t* src[kMax];
  size_t words[kMax];
  // Takes the entry when k_reset_copy can (a slot left, whole words, both
  // pointers 16-byte aligned: it moves uint4 words); false: the caller copies
  // it itself.
  [[nodiscard]] bool add(void* d, const void* s, size_t bytes) {
    if (n >= kMax || bytes % 4 != 0 || ((uintptr_t)d & 15) != 0 || ((uintptr_t)s & 15) != 0) return false;
    dst[n] = (uint32_t*)d;
    src[n] = (const uint32_t*)s;
    words[n] = bytes / 4;
    n++;
    return true;
  }
};
void launch_reset_copy(const ResetList& L, hipStream_t stream);

// Selector / term matching as an int8 contraction (ksim_match.hip, ksim_match_terms).
constexpr int kMatchMaxReqs = 4096;     // requirement columns (LDS: 16 rows x 4096 bits)
constexpr int kMatchMaxFeat = 65536;    // feature vocabulary (K of the contraction)
struct DevMatch {
  const int8_t* a;          // [sp][fp] signature one-hot rows (zeroed before the scatter)
  const int8_t* bt;         // [rp][fp] requirement rows (B transposed)
  const uint8_t* neg;       // [rp] 1: satisfied when no feature hits
  const int32_t *sig_off, *sig_feat, *req_off, *req_feat;   // CSR feature lists
  const int32_t *m_off, *m_req;                               // CSR requirement lists per matcher
  const int32_t *pod_sig, *pod_node, *cls_matcher;
  uint32_t* bits;           // [s][w] matcher bits per signature
  uint32_t* cls_bits;       // [s][cw] class bits per signature
  int32_t* cnt;             // [c][n] class counts over the bound pods (zeroed)
  int32_t s, sp, fp, r, rp, m, w, c, cw, p, n;
};
void launch_match(const DevMatch& m, hipStream_t stream);
void launch_assume(const DevCluster& c, const DevPods& P, int32_t pod, int32_t node, int sign, hipStream_t stream);

}  // namespace ksim
