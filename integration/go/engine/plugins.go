// Engine-backed framework plugins: what takes the place of the original
// in-tree plugin `p` in the simulator's factory closure
// (simulator/scheduler/plugin/plugins.go:75-87):
//
//	factory := func(configuration runtime.Object, f framework.Handle) (framework.Plugin, error) {
//		p, err := r(configuration, f)
//		...
//		p = engine.Backed(pl.Name, p, f)          // <- the one added line
//		return NewWrappedPlugin(store, p, WithWeightOption(&weight)), nil
//	}
//
// NewWrappedPlugin, the result store and the annotations stay unchanged: the
// wrapper calls these plugins exactly as it calls the originals and records
// what they return (wrappedplugin.go:356-516, 583-612).
//
// The simulator runs upstream's framework with parallelism 16 and
// percentageOfNodesToScore 0 (simulator/scheduler/scheduler.go:149,153,
// 231-241), so the FRAMEWORK decides which nodes Filter runs on, the feasible
// list PreScore / Score / NormalizeScore see and the node Reserve records.
// The plugins answer under those choices through the engine's
// framework-driven calls (include/ksim_engine.h, "framework-driven compat
// mode"):
//
//	PreFilter       the first engine-backed PreFilter of a cycle encodes the pod
//	                and calls ksim_fw_prefilter: Filter of every node of the
//	                pod's scan set on the GPU; the answers live in CycleState.
//	Filter          a read: plugin k of the profile's Filter order fails on the
//	                node iff the engine's chain stopped at k.
//	PreScore        the first engine-backed PreScore calls ksim_fw_score with the
//	                framework's list.
//	Score           raw[slot][node].
//	NormalizeScore  ksim_fw_normalize over the NodeScoreList it is handed.
//	Reserve         KsimAssume (an unwrapped Reserve plugin the host appends to
//	                every profile's Reserve set, so no annotation changes):
//	                ksim_assume on the framework's node; Unreserve ksim_forget.
//	                This is the scheduler cache's AssumePod for the engine's
//	                device-resident snapshot.
//	PostFilter      DefaultPreemption: ksim_preempt's dry run picks the node
//	                and victims; victims are deleted as prepareCandidate does.
//
// A pod the engine refuses (KSIM_E_UNSUPPORTED: e.g. unbound PVCs) is answered
// by the original plugin for the whole cycle: the engine has no CPU fallback,
// the reference plugins are the answer outside its scope.
//
// NOT BUILT HERE (no Go toolchain in the build container).  The node / pod
// encoders (Encoder) are the Go counterparts of ksim/encode.py and
// ksim/topology.py; ksim/fwplugins.py is the Python mirror of this file and
// tests/test_gpu_fw.py drives it under a racing-framework mirror.
package engine

/*
#include <stdlib.h>
#include "ksim_engine.h"
*/
import "C"

import (
	"context"
	"fmt"
	"sync"
	"unsafe"

	v1 "k8s.io/api/core/v1"
	metav1 "k8s.io/apimachinery/pkg/apis/meta/v1"
	"k8s.io/apimachinery/pkg/util/sets"
	"k8s.io/kubernetes/pkg/scheduler/framework"
)

// Encoder is the host side of the snapshot: NodeInfo -> SoA node table in
// nodeTree order, Pod -> ksim_pod_set (requests, tolerations, selector terms,
// topology uses / adds, PreFilterResult.NodeNames), as ksim/encode.py does.
type Encoder interface {
	// Snapshot brings the engine's device snapshot up to the framework's
	// (UpdateSnapshot: node informer deltas through Engine.UpsertNodes).
	Snapshot(e *Engine, f framework.Handle) error
	// Pod encodes one pod; the returned set stays valid until the next call.
	Pod(pod *v1.Pod) (*C.ksim_pod_set, error)
	// NodeNames are the node names in nodeTree order (engine positions).
	NodeNames() []string
	// Position of a node name in the engine's snapshot.
	Position(name string) (int, bool)
	// FilterMessage builds Status.Message() of a failing Filter
	// (ksim/wrapped.py filter_message).
	FilterMessage(plugin string, detail uint32, node string, pod *v1.Pod) string
	// PreFilterNodeNames is NodeAffinity's PreFilterResult.NodeNames (nil: all).
	PreFilterNodeNames(pod *v1.Pod) sets.String
	// Priority and victims bookkeeping for DefaultPreemption.
	BoundPod(index int) *v1.Pod
}

// Profile is the engine-side view of one framework profile.
type Profile struct {
	Engine      *Engine
	Enc         Encoder
	FilterOrder []string // the profile's Filter plugins in order (original names)
	ScoreOrder  []string // the profile's Score plugins in order
}

var (
	profilesMu sync.Mutex
	profiles   = map[framework.Handle]*Profile{}
)

// Register attaches an engine to the framework handle of one profile (the
// host does this when it builds the scheduler, scheduler.go:141-155).
func Register(f framework.Handle, p *Profile) {
	profilesMu.Lock()
	defer profilesMu.Unlock()
	profiles[f] = p
}

func profileOf(f framework.Handle) *Profile {
	profilesMu.Lock()
	defer profilesMu.Unlock()
	return profiles[f]
}

// cycleKey holds the engine's answers for the pod in flight.
const cycleKey framework.StateKey = "ksim.io/cycle"

type cycle struct {
	ps       *C.ksim_pod_set
	podIndex int
	refused  bool // KSIM_E_UNSUPPORTED: the original plugins answer
	nn       sets.String
	status   int32
	fail     []uint8
	detail   []uint32
	scored   bool
	raw      []int64 // [score slot][node]
	nNodes   int
}

func (c *cycle) Clone() framework.StateData { return c }

func readCycle(state *framework.CycleState) *cycle {
	d, err := state.Read(cycleKey)
	if err != nil {
		return nil
	}
	return d.(*cycle)
}

// ensureFilter runs the engine's PreFilter + Filter pass once per cycle.
func (p *Profile) ensureFilter(state *framework.CycleState, pod *v1.Pod, f framework.Handle) (*cycle, error) {
	if c := readCycle(state); c != nil {
		return c, nil
	}
	if err := p.Enc.Snapshot(p.Engine, f); err != nil {
		return nil, err
	}
	ps, err := p.Enc.Pod(pod)
	c := &cycle{nNodes: len(p.Enc.NodeNames())}
	if err != nil {
		c.refused = true
		state.Write(cycleKey, c)
		return c, nil
	}
	c.ps = ps
	c.nn = p.Enc.PreFilterNodeNames(pod)
	n := c.nNodes
	c.fail = make([]uint8, n)
	c.detail = make([]uint32, n)
	var out C.ksim_eval_out
	out.fail_plugin = (*C.uint8_t)(unsafe.Pointer(&c.fail[0]))
	out.fail_detail = (*C.uint32_t)(unsafe.Pointer(&c.detail[0]))
	rc := C.ksim_fw_prefilter(p.Engine.h, ps, 0, &out)
	if rc == C.KSIM_E_UNSUPPORTED {
		c.refused = true
	} else if err := p.Engine.err(rc); err != nil {
		return nil, err
	}
	c.status = int32(out.status)
	state.Write(cycleKey, c)
	return c, nil
}

// Backed returns the engine-backed plugin for an in-tree / out-of-tree plugin
// name, or the original when the engine does not replace it.
func Backed(name string, original framework.Plugin, f framework.Handle) framework.Plugin {
	b := &base{name: name, orig: original, f: f}
	switch name {
	case "NodeUnschedulable", "NodeName":
		return &filterOnly{b}
	case "NodeResourcesFit", "NodePorts":
		return &preFilterFilterScore{filterOnly{b}}
	case "TaintToleration", "NodeAffinity", "PodTopologySpread", "InterPodAffinity", "NetworkBandwidth":
		return &fullPlugin{preFilterFilterScore{filterOnly{b}}}
	case "NodeResourcesBalancedAllocation", "ImageLocality":
		return &scoreOnly{b}
	case "DefaultPreemption":
		return &postFilter{b}
	}
	return original
}

type base struct {
	name string
	orig framework.Plugin
	f    framework.Handle
}

func (b *base) Name() string { return b.name }

func (b *base) prof() *Profile { return profileOf(b.f) }

func index(xs []string, x string) int {
	for i, y := range xs {
		if y == x {
			return i
		}
	}
	return -1
}

// ---- Filter -------------------------------------------------------------------
type filterOnly struct{ *base }

func (p *filterOnly) Filter(ctx context.Context, state *framework.CycleState, pod *v1.Pod,
	nodeInfo *framework.NodeInfo) *framework.Status {
	pr := p.prof()
	c, err := pr.ensureFilter(state, pod, p.f)
	if err != nil {
		return framework.AsStatus(err)
	}
	if c.refused {
		return p.orig.(framework.FilterPlugin).Filter(ctx, state, pod, nodeInfo)
	}
	pos, ok := pr.Enc.Position(nodeInfo.Node().Name)
	if !ok {
		return framework.AsStatus(fmt.Errorf("node %s not in the engine snapshot", nodeInfo.Node().Name))
	}
	k := index(pr.FilterOrder, p.name)
	r := int(c.fail[pos])
	if r == C.KSIM_PASSED || r != k {
		return nil
	}
	d := c.detail[pos]
	return framework.NewStatus(filterCode(p.name, d), pr.Enc.FilterMessage(p.name, d, nodeInfo.Node().Name, pod))
}

// filterCode: the framework.Code upstream v1.26 plugins return on failure
// (ksim/fwplugins.py filter_code).
func filterCode(plugin string, detail uint32) framework.Code {
	switch plugin {
	case "NetworkBandwidth":
		if detail == C.KSIM_NB_INSUFFICIENT {
			return framework.Unschedulable
		}
		return framework.Error
	case "PodTopologySpread":
		if detail == C.KSIM_PTS_MISSING_LABEL {
			return framework.UnschedulableAndUnresolvable
		}
		return framework.Unschedulable
	case "InterPodAffinity":
		if detail == C.KSIM_IPA_AFFINITY {
			return framework.UnschedulableAndUnresolvable
		}
		return framework.Unschedulable
	case "NodeUnschedulable", "NodeName", "TaintToleration", "NodeAffinity", "VolumeBinding", "VolumeZone":
		return framework.UnschedulableAndUnresolvable
	}
	return framework.Unschedulable
}

// ---- PreFilter + Filter + Score ---------------------------------------------------
type preFilterFilterScore struct{ filterOnly }

func (p *preFilterFilterScore) PreFilter(ctx context.Context, state *framework.CycleState,
	pod *v1.Pod) (*framework.PreFilterResult, *framework.Status) {
	c, err := p.prof().ensureFilter(state, pod, p.f)
	if err != nil {
		return nil, framework.AsStatus(err)
	}
	if c.refused {
		return p.orig.(framework.PreFilterPlugin).PreFilter(ctx, state, pod)
	}
	if p.name == "NodeAffinity" && c.nn != nil {
		if c.nn.Len() == 0 {
			return nil, framework.NewStatus(framework.UnschedulableAndUnresolvable, "pod affinity terms conflict")
		}
		return &framework.PreFilterResult{NodeNames: c.nn}, nil
	}
	return nil, nil
}

func (p *preFilterFilterScore) PreFilterExtensions() framework.PreFilterExtensions { return nil }

func (p *preFilterFilterScore) Score(ctx context.Context, state *framework.CycleState, pod *v1.Pod,
	nodeName string) (int64, *framework.Status) {
	return score(p.base, ctx, state, pod, nodeName)
}

func (p *preFilterFilterScore) ScoreExtensions() framework.ScoreExtensions { return nil }

// ---- PreScore + Score + NormalizeScore ---------------------------------------------
type fullPlugin struct{ preFilterFilterScore }

func (p *fullPlugin) PreScore(ctx context.Context, state *framework.CycleState, pod *v1.Pod,
	nodes []*v1.Node) *framework.Status {
	c := readCycle(state)
	if c == nil || c.refused {
		return p.orig.(framework.PreScorePlugin).PreScore(ctx, state, pod, nodes)
	}
	if c.scored {
		return nil
	}
	pr := p.prof()
	list := make([]int32, len(nodes))
	for i, n := range nodes {
		pos, ok := pr.Enc.Position(n.Name)
		if !ok {
			return framework.AsStatus(fmt.Errorf("node %s not in the engine snapshot", n.Name))
		}
		list[i] = int32(pos)
	}
	c.raw = make([]int64, len(pr.ScoreOrder)*c.nNodes)
	var out C.ksim_eval_out
	if len(c.raw) > 0 {
		out.raw = (*C.int64_t)(unsafe.Pointer(&c.raw[0]))
	}
	var lp *C.int32_t
	if len(list) > 0 {
		lp = (*C.int32_t)(unsafe.Pointer(&list[0]))
	}
	if err := pr.Engine.err(C.ksim_fw_score(pr.Engine.h, lp, C.int32_t(len(list)), &out)); err != nil {
		return framework.AsStatus(err)
	}
	c.scored = true
	if out.status == C.KSIM_STATUS_ERROR {
		return framework.AsStatus(fmt.Errorf("NetworkBandwidth Score failed on a listed node"))
	}
	return nil
}

func (p *fullPlugin) ScoreExtensions() framework.ScoreExtensions { return p }

func (p *fullPlugin) NormalizeScore(ctx context.Context, state *framework.CycleState, pod *v1.Pod,
	scores framework.NodeScoreList) *framework.Status {
	c := readCycle(state)
	if c == nil || c.refused {
		return p.orig.(framework.ScorePlugin).ScoreExtensions().NormalizeScore(ctx, state, pod, scores)
	}
	pr := p.prof()
	n := len(scores)
	if n == 0 {
		return nil
	}
	nodes := make([]int32, n)
	vals := make([]int64, n)
	for i, s := range scores {
		pos, _ := pr.Enc.Position(s.Name)
		nodes[i] = int32(pos)
		vals[i] = s.Score
	}
	out := make([]int64, n)
	slot := index(pr.ScoreOrder, p.name)
	rc := C.ksim_fw_normalize(pr.Engine.h, C.int32_t(slot), (*C.int32_t)(unsafe.Pointer(&nodes[0])),
		(*C.int64_t)(unsafe.Pointer(&vals[0])), C.int32_t(n), (*C.int64_t)(unsafe.Pointer(&out[0])))
	if err := pr.Engine.err(rc); err != nil {
		return framework.AsStatus(err)
	}
	for i := range scores {
		scores[i].Score = out[i]
	}
	return nil
}

// ---- Score only (BalancedAllocation, ImageLocality) -----------------------------
type scoreOnly struct{ *base }

func (p *scoreOnly) Score(ctx context.Context, state *framework.CycleState, pod *v1.Pod,
	nodeName string) (int64, *framework.Status) {
	return score(p.base, ctx, state, pod, nodeName)
}

func (p *scoreOnly) ScoreExtensions() framework.ScoreExtensions { return nil }

func score(b *base, ctx context.Context, state *framework.CycleState, pod *v1.Pod,
	nodeName string) (int64, *framework.Status) {
	c := readCycle(state)
	if c == nil || c.refused || !c.scored {
		// no engine pass for this cycle (refused pod, or a profile whose
		// PreScore set holds no engine-backed plugin): the original answers
		return b.orig.(framework.ScorePlugin).Score(ctx, state, pod, nodeName)
	}
	pr := b.prof()
	pos, ok := pr.Enc.Position(nodeName)
	if !ok {
		return 0, framework.AsStatus(fmt.Errorf("node %s not in the engine snapshot", nodeName))
	}
	return c.raw[index(pr.ScoreOrder, b.name)*c.nNodes+pos], nil
}

// ---- KsimAssume: the engine snapshot's AssumePod ----------------------------------
// An unwrapped Reserve plugin the host appends to every profile's Reserve set
// (after ConvertForSimulator, so the wrapped set and its annotations are
// unchanged).  Reserve records nothing; it assumes the pod on the framework's
// node (selectHost's pick, ties included) in the device snapshot.
type KsimAssume struct{ f framework.Handle }

func NewKsimAssume(_ interface{}, f framework.Handle) (framework.Plugin, error) {
	return &KsimAssume{f: f}, nil
}

func (p *KsimAssume) Name() string { return "KsimAssume" }

func (p *KsimAssume) Reserve(ctx context.Context, state *framework.CycleState, pod *v1.Pod,
	nodeName string) *framework.Status {
	c := readCycle(state)
	if c == nil || c.refused {
		return nil // the engine snapshot picks the pod up from the informer (Engine.Assume)
	}
	pr := profileOf(p.f)
	pos, ok := pr.Enc.Position(nodeName)
	if !ok {
		return framework.AsStatus(fmt.Errorf("node %s not in the engine snapshot", nodeName))
	}
	return framework.AsStatus(pr.Engine.err(C.ksim_assume(pr.Engine.h, c.ps, 0, C.int32_t(pos))))
}

func (p *KsimAssume) Unreserve(ctx context.Context, state *framework.CycleState, pod *v1.Pod, nodeName string) {
	c := readCycle(state)
	if c == nil || c.refused {
		return
	}
	pr := profileOf(p.f)
	if pos, ok := pr.Enc.Position(nodeName); ok {
		_ = C.ksim_forget(pr.Engine.h, c.ps, 0, C.int32_t(pos))
	}
}

// ---- DefaultPreemption --------------------------------------------------------------
type postFilter struct{ *base }

func (p *postFilter) PostFilter(ctx context.Context, state *framework.CycleState, pod *v1.Pod,
	m framework.NodeToStatusMap) (*framework.PostFilterResult, *framework.Status) {
	c := readCycle(state)
	if c == nil || c.refused {
		return p.orig.(framework.PostFilterPlugin).PostFilter(ctx, state, pod, m)
	}
	pr := p.prof()
	victims := make([]int32, 1024)
	var out C.ksim_preempt_out
	out.victims = (*C.int32_t)(unsafe.Pointer(&victims[0]))
	out.victims_cap = C.int32_t(len(victims))
	prio := int32(0)
	if pod.Spec.Priority != nil {
		prio = *pod.Spec.Priority
	}
	rc := C.ksim_preempt(pr.Engine.h, c.ps, 0, C.int32_t(prio), &out)
	if rc == C.KSIM_E_UNSUPPORTED {
		return p.orig.(framework.PostFilterPlugin).PostFilter(ctx, state, pod, m)
	}
	if err := pr.Engine.err(rc); err != nil {
		return nil, framework.AsStatus(err)
	}
	if out.nominated < 0 {
		return nil, framework.NewStatus(framework.Unschedulable, "preemption: no candidate node")
	}
	// prepareCandidate: delete the victims (PodDisruptionBudgets are out of
	// the engine's scope, DESIGN.md §8)
	cs := p.f.ClientSet()
	for i := 0; i < int(out.n_victims) && i < len(victims); i++ {
		v := pr.Enc.BoundPod(int(victims[i]))
		if err := cs.CoreV1().Pods(v.Namespace).Delete(ctx, v.Name, metav1.DeleteOptions{}); err != nil {
			return nil, framework.AsStatus(err)
		}
	}
	name := pr.Enc.NodeNames()[int(out.nominated)]
	return &framework.PostFilterResult{NominatingInfo: &framework.NominatingInfo{
		NominatedNodeName: name, NominatingMode: framework.ModeOverride}}, nil
}
