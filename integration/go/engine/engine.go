// Package engine is the cgo binding of libksim_engine.so (include/ksim_engine.h)
// that a maintainer would add to the simulator as simulator/scheduler/engine,
// next to the plugin factory it serves (simulator/scheduler/plugin/plugins.go:75-87:
// the closure builds the original in-tree plugin `p` and wraps it with
// NewWrappedPlugin; an engine-backed plugin takes the place of `p`).
//
// NOT BUILT HERE: the build container has no Go toolchain.  The declarations
// follow the C header one to one; INTEGRATION.md describes the call sequence.
//
// Every call copies its inputs before returning and keeps no Go pointer, which
// satisfies the cgo pointer-passing rules.  CGO_ENABLED=0 in
// simulator/Dockerfile:5 must become 1, and libamdhip64.so must be present
// next to libksim_engine.so.
package engine

/*
#cgo CFLAGS: -I${SRCDIR}/../../../include
#cgo LDFLAGS: -L${SRCDIR}/../../../kube-scheduler-simulator_amd/ksim -lksim_engine -Wl,-rpath,${SRCDIR}/../../../kube-scheduler-simulator_amd/ksim
#include <stdlib.h>
#include "ksim_engine.h"
*/
import "C"

import (
	"fmt"
	"sync"
	"unsafe"
)

// ABIVersion is the header version this binding was written against.
const ABIVersion = 11

// Engine owns one device handle (one GPU, or one node shard of a cluster).
// A handle is not reentrant: the framework's 16 Filter goroutines (nominated
// first passes), the binding goroutine (Unreserve) and the next scheduling
// cycle reach it concurrently, so every call holds mu.
type Engine struct {
	h  *C.ksim_handle
	mu sync.Mutex
}

// locked runs one C call under the handle's mutex.
func (e *Engine) locked(f func() C.int) error {
	e.mu.Lock()
	rc := f()
	err := e.err(rc)
	e.mu.Unlock()
	return err
}

// New opens the engine on a HIP device; it fails when no GPU is present (the
// engine has no CPU fallback).
func New(device int) (*Engine, error) {
	if v := int(C.ksim_abi_version()); v != ABIVersion {
		return nil, fmt.Errorf("libksim_engine ABI %d, binding %d", v, ABIVersion)
	}
	var h *C.ksim_handle
	if rc := C.ksim_create(C.int(device), &h); rc != C.KSIM_OK {
		return nil, fmt.Errorf("ksim_create: %d", int(rc))
	}
	return &Engine{h: h}, nil
}

// Close releases the handle and its device memory.
func (e *Engine) Close() { C.ksim_destroy(e.h) }

func (e *Engine) err(rc C.int) error {
	if rc == C.KSIM_OK {
		return nil
	}
	return fmt.Errorf("ksim %d: %s", int(rc), C.GoString(C.ksim_last_error(e.h)))
}

// SetProfile installs the converted KubeSchedulerProfile
// (convertConfigurationForSimulator, simulator/scheduler/scheduler.go:199-249).
func (e *Engine) SetProfile(p *C.ksim_profile) error {
	return e.locked(func() C.int { return C.ksim_set_profile(e.h, p) })
}

// SetCluster uploads the whole snapshot in nodeTree order (resets
// nextStartNodeIndex).  t's column pointers point into Go memory pinned for
// the call only.
func (e *Engine) SetCluster(t *C.ksim_node_table, v *C.ksim_vocab) error {
	return e.locked(func() C.int { return C.ksim_set_cluster(e.h, t, v) })
}

// UpsertNodes applies node informer events (AddNode / UpdateNode / RemoveNode)
// without losing the binds the cycles made: t is the new snapshot, oldPos[i]
// the previous position of new node i or -1.  Reload the pod queue afterwards.
func (e *Engine) UpsertNodes(t *C.ksim_node_table, v *C.ksim_vocab, oldPos []int32) error {
	var p *C.int32_t
	if len(oldPos) > 0 {
		p = (*C.int32_t)(unsafe.Pointer(&oldPos[0]))
	}
	return e.locked(func() C.int { return C.ksim_upsert_nodes(e.h, t, v, p) })
}

// UpdateNodeRows applies an in-place UpdateNode (ABI 11): the static columns
// of rows from t, whose layout and vocabulary are the handle's (the encoder's
// ksim_encoder_changed_rows says when a delta qualifies).
func (e *Engine) UpdateNodeRows(t *C.ksim_node_table, v *C.ksim_vocab, rows []int32) error {
	var p *C.int32_t
	if len(rows) > 0 {
		p = (*C.int32_t)(unsafe.Pointer(&rows[0]))
	}
	return e.locked(func() C.int { return C.ksim_update_node_rows(e.h, t, v, p, C.int32_t(len(rows))) })
}

// RemoveNode removes the node at position pos (later nodes move down by one).
func (e *Engine) RemoveNode(pos int) error {
	return e.locked(func() C.int { return C.ksim_remove_node(e.h, C.int32_t(pos)) })
}

// SetEvalRange makes this handle a replica (whole snapshot) that evaluates
// nodes [lo, hi) in the batch top-T; the ranks' ranges tile the cluster.
func (e *Engine) SetEvalRange(lo, hi int) error {
	return e.locked(func() C.int { return C.ksim_set_eval_range(e.h, C.int32_t(lo), C.int32_t(hi)) })
}

// MatchTerms answers every (signature, matcher) pair of the count classes'
// selectors and terms on the device (the existing-pod scans of
// PodTopologySpread / InterPodAffinity PreFilter and PreScore):
// bits[s*words+m/32] bit m%32 = signature s matches matcher m, and
// counts[c*nNodes+node] = bound pods on node whose signature matches
// classMatcher[c] (counts may be empty when mp.n_classes == 0).
func (e *Engine) MatchTerms(mp *C.ksim_match_problem, bits []uint32, counts []int32) error {
	var cp *C.int32_t
	if len(counts) > 0 {
		cp = (*C.int32_t)(unsafe.Pointer(&counts[0]))
	}
	return e.locked(func() C.int { return C.ksim_match_terms(e.h, mp, (*C.uint32_t)(unsafe.Pointer(&bits[0])), cp) })
}

// EvalPod runs one full cycle for pod idx of ps (PreFilter .. bind) and fills
// the per-node outputs the wrapped plugins record (out's slices are Go-owned:
// n_nodes entries, n_score x n_nodes for the score matrices).
func (e *Engine) EvalPod(ps *C.ksim_pod_set, idx int, out *C.ksim_eval_out) error {
	return e.locked(func() C.int { return C.ksim_eval_pod(e.h, ps, C.int32_t(idx), out) })
}

// EvalPodFilter / EvalPodFinish split a cycle around the host's extender
// round trip (findNodesThatPassExtenders, the extender part of prioritizeNodes).
func (e *Engine) EvalPodFilter(ps *C.ksim_pod_set, idx int, out *C.ksim_eval_out) error {
	return e.locked(func() C.int { return C.ksim_eval_pod_filter(e.h, ps, C.int32_t(idx), out) })
}

func (e *Engine) EvalPodFinish(extFail []uint8, extScore []int64, out *C.ksim_eval_out) error {
	var f *C.uint8_t
	var s *C.int64_t
	if len(extFail) > 0 {
		f = (*C.uint8_t)(unsafe.Pointer(&extFail[0]))
	}
	if len(extScore) > 0 {
		s = (*C.int64_t)(unsafe.Pointer(&extScore[0]))
	}
	return e.locked(func() C.int { return C.ksim_eval_pod_finish(e.h, f, s, out) })
}

// Framework-driven compat mode (plugins.go uses these through cgo directly):
// FwPreFilter answers Filter for every node of the pod's scan set, FwScore
// runs PreScore / Score / NormalizeScore over the framework's list,
// FwNormalize normalizes one score slot over an explicit list.
func (e *Engine) FwPreFilter(ps *C.ksim_pod_set, idx int, out *C.ksim_eval_out) error {
	return e.locked(func() C.int { return C.ksim_fw_prefilter(e.h, ps, C.int32_t(idx), out) })
}

func (e *Engine) FwScore(nodes []int32, out *C.ksim_eval_out) error {
	var p *C.int32_t
	if len(nodes) > 0 {
		p = (*C.int32_t)(unsafe.Pointer(&nodes[0]))
	}
	return e.locked(func() C.int { return C.ksim_fw_score(e.h, p, C.int32_t(len(nodes)), out) })
}

func (e *Engine) FwNormalize(slot int, nodes []int32, scores, out []int64) error {
	if len(nodes) == 0 {
		return nil
	}
	return e.locked(func() C.int {
		return C.ksim_fw_normalize(e.h, C.int32_t(slot), (*C.int32_t)(unsafe.Pointer(&nodes[0])),
			(*C.int64_t)(unsafe.Pointer(&scores[0])), C.int32_t(len(nodes)), (*C.int64_t)(unsafe.Pointer(&out[0])))
	})
}

// SetBoundPods / Preempt: DefaultPreemption's dry run over the bound pods.
func (e *Engine) SetBoundPods(b *C.ksim_bound_pods) error {
	return e.locked(func() C.int { return C.ksim_set_bound_pods(e.h, b) })
}

func (e *Engine) Preempt(ps *C.ksim_pod_set, idx int, priority int32, out *C.ksim_preempt_out) error {
	return e.locked(func() C.int { return C.ksim_preempt(e.h, ps, C.int32_t(idx), C.int32_t(priority), out) })
}

// PreemptNominated: the dry run with the PodNominator's pods; group k is
// nominated[first[k] : first[k]+count[k]] on node position nodes[k].
func (e *Engine) PreemptNominated(ps *C.ksim_pod_set, idx int, priority int32, nominated *C.ksim_pod_set,
	nodes, first, count []int32, out *C.ksim_preempt_out) error {
	var n, f, c *C.int32_t
	if len(nodes) > 0 {
		n = (*C.int32_t)(unsafe.Pointer(&nodes[0]))
		f = (*C.int32_t)(unsafe.Pointer(&first[0]))
		c = (*C.int32_t)(unsafe.Pointer(&count[0]))
	}
	return e.locked(func() C.int {
		return C.ksim_preempt_nominated(e.h, ps, C.int32_t(idx), C.int32_t(priority), nominated,
			C.int32_t(len(nodes)), n, f, c, out)
	})
}

// FwFilterNominated: RunFilterPluginsWithNominatedPods' first pass of the
// cycle in flight on the grouped nodes (plugins.go calls it per node).
func (e *Engine) FwFilterNominated(nominated *C.ksim_pod_set, nodes, first, count []int32, fail []uint8,
	detail []uint32) error {
	if len(nodes) == 0 {
		return nil
	}
	return e.locked(func() C.int {
		return C.ksim_fw_filter_nominated(e.h, nominated, C.int32_t(len(nodes)), (*C.int32_t)(unsafe.Pointer(&nodes[0])),
			(*C.int32_t)(unsafe.Pointer(&first[0])), (*C.int32_t)(unsafe.Pointer(&count[0])),
			(*C.uint8_t)(unsafe.Pointer(&fail[0])), (*C.uint32_t)(unsafe.Pointer(&detail[0])))
	})
}

// Assume / Forget: NodeInfo.AddPod / RemovePod of a bound pod (informer pod
// events, Unreserve), count classes included.
func (e *Engine) Assume(ps *C.ksim_pod_set, idx, node int) error {
	return e.locked(func() C.int { return C.ksim_assume(e.h, ps, C.int32_t(idx), C.int32_t(node)) })
}

func (e *Engine) Forget(ps *C.ksim_pod_set, idx, node int) error {
	return e.locked(func() C.int { return C.ksim_forget(e.h, ps, C.int32_t(idx), C.int32_t(node)) })
}

// LoadPods uploads a pending queue in PrioritySort order for ScheduleLoaded.
func (e *Engine) LoadPods(ps *C.ksim_pod_set) error {
	return e.locked(func() C.int { return C.ksim_load_pods(e.h, ps) })
}

// ScheduleLoaded schedules loaded pods [first, first+count) on the device
// (batch, ADAPT batch or per-pod cycles; placements identical to cycle by
// cycle).  chosen[i] receives the node position of pod first+i, or -1.
func (e *Engine) ScheduleLoaded(first, count int, chosen []int32) (C.ksim_batch_stats, error) {
	var st C.ksim_batch_stats
	var p *C.int32_t
	if len(chosen) > 0 {
		p = (*C.int32_t)(unsafe.Pointer(&chosen[0]))
	}
	err := e.locked(func() C.int { return C.ksim_schedule_loaded(e.h, C.int32_t(first), C.int32_t(count), p, &st) })
	return st, err
}

// ResetCluster restores the snapshot of the last SetCluster / UpsertNodes.
func (e *Engine) ResetCluster() error {
	return e.locked(func() C.int { return C.ksim_reset_cluster(e.h) })
}

// NextStart is the scheduler's nextStartNodeIndex.
func (e *Engine) NextStart() (int, error) {
	var v C.int32_t
	err := e.locked(func() C.int { return C.ksim_get_next_start(e.h, &v) })
	return int(v), err
}

// Multi-GPU: one process per GPU.  SetShard (before SetCluster) gives this
// handle the contiguous node range [base, base+count) of nTotal; rank 0 makes
// the communicator id with CommUniqueID, the ranks share it over any side
// channel, and each calls CommInit.
func (e *Engine) SetShard(base, nTotal int) error {
	return e.locked(func() C.int { return C.ksim_set_shard(e.h, C.int32_t(base), C.int32_t(nTotal)) })
}

func CommUniqueID() ([C.KSIM_COMM_ID_BYTES]byte, error) {
	var id [C.KSIM_COMM_ID_BYTES]byte
	if rc := C.ksim_comm_unique_id((*C.uint8_t)(unsafe.Pointer(&id[0]))); rc != C.KSIM_OK {
		return id, fmt.Errorf("ksim_comm_unique_id: %d", int(rc))
	}
	return id, nil
}

func (e *Engine) CommInit(rank, world int, id [C.KSIM_COMM_ID_BYTES]byte) error {
	return e.locked(func() C.int { return C.ksim_comm_init(e.h, C.int32_t(rank), C.int32_t(world), (*C.uint8_t)(unsafe.Pointer(&id[0]))) })
}
