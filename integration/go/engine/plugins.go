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
//	PostFilter      DefaultPreemption: PodEligibleToPreemptOthers on the host,
//	                then ksim_preempt_nominated's dry run (the PodNominator's
//	                pods of priority >= the preemptor stay on each candidate)
//	                picks the node and victims; prepareCandidate's side effects
//	                (DisruptionTarget condition, delete, lower-priority
//	                nominations cleared) on the host.
//	AddPod          PreFilterExtensions on the CycleState clone that
//	                RunFilterPluginsWithNominatedPods builds: the clone carries
//	                the nominated pods, and Filter on it answers from
//	                ksim_fw_filter_nominated (pass 1), once per node and cycle.
//
// Concurrency: the framework's 16 Filter goroutines, the binding goroutine
// (Unreserve) and the next scheduling cycle reach the handle concurrently;
// every engine call holds Engine.mu, and a cycle's first engine pass is made
// once under Profile.mu.
//
// A pod the engine refuses (KSIM_E_UNSUPPORTED: e.g. unbound PVCs) is answered
// by the original plugin for the whole cycle: the engine has no CPU fallback,
// the reference plugins are the answer outside its scope.
//
// NOT BUILT HERE (no Go toolchain in the build container).  The Encoder is
// NativeEncoder (encoder.go) over the engine's native snapshot encoder
// (ksim_encode_nodes / ksim_encode_pods, byte-equal to ksim/encode.py);
// ksim/fwplugins.py is the Python mirror of this file and tests/test_gpu_fw.py
// drives it under a racing-framework mirror.
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
	"k8s.io/apimachinery/pkg/util/sets"
	utilfeature "k8s.io/apiserver/pkg/util/feature"
	"k8s.io/client-go/tools/cache"
	corev1helpers "k8s.io/component-helpers/scheduling/corev1"
	"k8s.io/klog/v2"
	apipod "k8s.io/kubernetes/pkg/api/v1/pod"
	"k8s.io/kubernetes/pkg/features"
	"k8s.io/kubernetes/pkg/scheduler/framework"
	schedutil "k8s.io/kubernetes/pkg/scheduler/util"
)

// Encoder is the host side of the snapshot: NodeInfo -> SoA node table in
// nodeTree order, Pod -> ksim_pod_set (requests, tolerations, selector terms,
// topology uses / adds, PreFilterResult.NodeNames), as ksim/encode.py does.
// NativeEncoder (encoder.go) implements it over ksim_encode_nodes / _pods.
type Encoder interface {
	// Snapshot brings the engine's device snapshot up to the cluster at a
	// cycle start (UpdateSnapshot): the whole snapshot once, then the queued
	// informer events as deltas (Engine.UpsertNodes, ksim_assume / ksim_forget).
	Snapshot(e *Engine, f framework.Handle) error
	// Pod encodes one pod; the returned set stays valid until the next call.
	Pod(pod *v1.Pod) (*C.ksim_pod_set, error)
	// Resync re-sends the node table when Pod added label columns or count
	// classes (keys / selectors no earlier pod referenced).
	Resync(e *Engine) error
	// NodeNames are the node names in nodeTree order (engine positions).
	NodeNames() []string
	// Position of a node name in the engine's snapshot.
	Position(name string) (int, bool)
	// FilterMessage builds Status.Message() of a failing Filter
	// (ksim/wrapped.py filter_message).
	FilterMessage(plugin string, detail uint32, node string, pod *v1.Pod) string
	// PreFilterNodeNames is NodeAffinity's PreFilterResult.NodeNames (nil: all).
	PreFilterNodeNames(pod *v1.Pod) sets.String
	// Priority and victims bookkeeping for DefaultPreemption: the bound-pod
	// table row index -> pod (the table follows the snapshot, SetBoundPods).
	BoundPod(index int) *v1.Pod
	// Pods encodes a list of pods into a set the caller owns (C memory) until
	// release: the nominated pods of a first pass / dry run.
	Pods(pods []*v1.Pod) (ps *C.ksim_pod_set, release func(), err error)
	// Assume / Forget: the cycle's pod enters / leaves the device snapshot and
	// the encoder's membership (KsimAssume's Reserve / Unreserve).
	Assume(e *Engine, pod *v1.Pod, node int) error
	Forget(e *Engine, pod *v1.Pod) error
	// BoundTable re-sends DefaultPreemption's bound-pod table when it is stale.
	BoundTable(e *Engine) error
}

// informerFed is an Encoder that follows the cluster through informer event
// handlers (NativeEncoder.Handlers).
type informerFed interface {
	Handlers() (pods, nodes cache.ResourceEventHandlerFuncs)
}

// Profile is the engine-side view of one framework profile.
type Profile struct {
	Engine      *Engine
	Enc         Encoder
	FilterOrder []string // the profile's Filter plugins in order (original names)
	ScoreOrder  []string // the profile's Score plugins in order
	mu          sync.Mutex
}

var (
	profilesMu sync.Mutex
	profiles   = map[framework.Handle]*Profile{}
)

// Register attaches an engine to the framework handle of one profile (the
// host does this when it builds the scheduler, scheduler.go:141-155) and
// feeds the encoder the pod and node informers' events (the deltas the next
// cycle start applies).
func Register(f framework.Handle, p *Profile) {
	profilesMu.Lock()
	defer profilesMu.Unlock()
	profiles[f] = p
	if fed, ok := p.Enc.(informerFed); ok {
		pods, nodes := fed.Handlers()
		f.SharedInformerFactory().Core().V1().Pods().Informer().AddEventHandler(pods)
		f.SharedInformerFactory().Core().V1().Nodes().Informer().AddEventHandler(nodes)
	}
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
	// added: the nominated pods addNominatedPods put on this clone of the
	// CycleState (PreFilterExtensions.AddPod); empty on the cycle's own state
	added []*v1.Pod
	sh    *cycleShared
}

// cycleShared is what every clone of one cycle's state shares.
type cycleShared struct {
	mu      sync.Mutex
	nom     map[int]nomAnswer // node position -> pass-1 answer
	assumed bool              // KsimAssume's Reserve succeeded and was not undone
	node    int
}

type nomAnswer struct {
	fail   uint8
	detail uint32
}

// Clone: RunFilterPluginsWithNominatedPods clones the state before AddPod, so
// the added list is per clone; the engine's answers are shared.
func (c *cycle) Clone() framework.StateData {
	d := *c
	d.added = append([]*v1.Pod(nil), c.added...)
	return &d
}

func readCycle(state *framework.CycleState) *cycle {
	d, err := state.Read(cycleKey)
	if err != nil {
		return nil
	}
	return d.(*cycle)
}

// ensureFilter runs the engine's PreFilter + Filter pass once per cycle.  A
// profile without an engine-backed PreFilter reaches it first from the 16
// Filter goroutines, hence Profile.mu around the check and the pass.
func (p *Profile) ensureFilter(state *framework.CycleState, pod *v1.Pod, f framework.Handle) (*cycle, error) {
	if c := readCycle(state); c != nil {
		return c, nil
	}
	p.mu.Lock()
	defer p.mu.Unlock()
	if c := readCycle(state); c != nil {
		return c, nil
	}
	if err := p.Enc.Snapshot(p.Engine, f); err != nil {
		return nil, err
	}
	ps, err := p.Enc.Pod(pod)
	if err == nil {
		err = p.Enc.Resync(p.Engine)
	}
	c := &cycle{nNodes: len(p.Enc.NodeNames()), sh: &cycleShared{nom: map[int]nomAnswer{}}}
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
	// the error text is read under the handle's mutex (another goroutine's
	// call may set the handle's last error right after this one)
	p.Engine.mu.Lock()
	rc := C.ksim_fw_prefilter(p.Engine.h, ps, 0, &out)
	err = p.Engine.err(rc)
	p.Engine.mu.Unlock()
	if rc == C.KSIM_E_UNSUPPORTED {
		c.refused = true
	} else if err != nil {
		return nil, err
	}
	c.status = int32(out.status)
	state.Write(cycleKey, c)
	return c, nil
}

// nominatedAnswer: pass 1 of RunFilterPluginsWithNominatedPods on node pos,
// the clone's added pods on the node (ksim_fw_filter_nominated), once per
// node and cycle (the 15 Filter plugins of the clone all read it).
func (p *Profile) nominatedAnswer(c *cycle, pos int) (nomAnswer, error) {
	c.sh.mu.Lock()
	defer c.sh.mu.Unlock()
	if a, ok := c.sh.nom[pos]; ok {
		return a, nil
	}
	nps, release, err := p.Enc.Pods(c.added)
	if err != nil {
		return nomAnswer{}, err
	}
	defer release()
	node, first, count := C.int32_t(pos), C.int32_t(0), C.int32_t(len(c.added))
	var fp C.uint8_t
	var fd C.uint32_t
	if err := p.Engine.locked(func() C.int {
		return C.ksim_fw_filter_nominated(p.Engine.h, nps, 1, &node, &first, &count, &fp, &fd)
	}); err != nil {
		return nomAnswer{}, err
	}
	a := nomAnswer{fail: uint8(fp), detail: uint32(fd)}
	c.sh.nom[pos] = a
	return a, nil
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
	r, d := int(c.fail[pos]), c.detail[pos]
	if len(c.added) > 0 { // the clone carrying the node's nominated pods (pass 1)
		a, err := pr.nominatedAnswer(c, pos)
		if err != nil {
			return framework.AsStatus(err)
		}
		r, d = int(a.fail), a.detail
	}
	if r == C.KSIM_PASSED || r != k {
		return nil
	}
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

// PreFilterExtensions: AddPod / RemovePod record the nominated pods on the
// CycleState clone (every engine-backed PreFilter plugin gets the call; the
// pod is added once).  Refused cycles forward to the original's extensions.
func (p *preFilterFilterScore) PreFilterExtensions() framework.PreFilterExtensions { return p }

func (p *preFilterFilterScore) AddPod(ctx context.Context, state *framework.CycleState, podToSchedule *v1.Pod,
	podInfoToAdd *framework.PodInfo, nodeInfo *framework.NodeInfo) *framework.Status {
	c := readCycle(state)
	if c == nil || c.refused {
		if ext := p.orig.(framework.PreFilterPlugin).PreFilterExtensions(); ext != nil {
			return ext.AddPod(ctx, state, podToSchedule, podInfoToAdd, nodeInfo)
		}
		return nil
	}
	for _, q := range c.added {
		if q.UID == podInfoToAdd.Pod.UID {
			return nil
		}
	}
	c.added = append(c.added, podInfoToAdd.Pod)
	return nil
}

func (p *preFilterFilterScore) RemovePod(ctx context.Context, state *framework.CycleState, podToSchedule *v1.Pod,
	podInfoToRemove *framework.PodInfo, nodeInfo *framework.NodeInfo) *framework.Status {
	c := readCycle(state)
	if c == nil || c.refused {
		if ext := p.orig.(framework.PreFilterPlugin).PreFilterExtensions(); ext != nil {
			return ext.RemovePod(ctx, state, podToSchedule, podInfoToRemove, nodeInfo)
		}
		return nil
	}
	for i, q := range c.added {
		if q.UID == podInfoToRemove.Pod.UID {
			c.added = append(c.added[:i], c.added[i+1:]...)
			return nil
		}
	}
	// removing a bound pod from the clone happens only in the original
	// DefaultPreemption's dry run, which the engine-backed PostFilter replaces
	return framework.AsStatus(fmt.Errorf("RemovePod of a bound pod on an engine-backed cycle"))
}

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
	if err := pr.Engine.locked(func() C.int {
		return C.ksim_fw_score(pr.Engine.h, lp, C.int32_t(len(list)), &out)
	}); err != nil {
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
	if err := pr.Engine.locked(func() C.int {
		return C.ksim_fw_normalize(pr.Engine.h, C.int32_t(slot), (*C.int32_t)(unsafe.Pointer(&nodes[0])),
			(*C.int64_t)(unsafe.Pointer(&vals[0])), C.int32_t(n), (*C.int64_t)(unsafe.Pointer(&out[0])))
	}); err != nil {
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
// An unwrapped Reserve + PostBind plugin the host appends to every profile
// (after ConvertForSimulator, so the wrapped set and its annotations are
// unchanged).  Reserve records nothing; it assumes the pod on the framework's
// node (selectHost's pick, ties included) in the device snapshot and in the
// encoder's membership (Encoder.Assume), so the next cycle starts from it
// without a re-encode; the informer's later report of the bound pod is a
// no-op.  Unreserve -- from a later Reserve plugin's failure, Permit, PreBind
// or Bind, possibly on the binding goroutine after the next cycle started --
// forgets it only if this Reserve assumed it (upstream cache.ForgetPod is
// likewise a no-op for a pod never assumed).
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
	if err := pr.Enc.Assume(pr.Engine, pod, pos); err != nil {
		return framework.AsStatus(err)
	}
	c.sh.mu.Lock()
	c.sh.assumed, c.sh.node = true, pos
	c.sh.mu.Unlock()
	return nil
}

func (p *KsimAssume) Unreserve(ctx context.Context, state *framework.CycleState, pod *v1.Pod, nodeName string) {
	c := readCycle(state)
	if c == nil || c.refused {
		return
	}
	pr := profileOf(p.f)
	c.sh.mu.Lock()
	defer c.sh.mu.Unlock()
	if !c.sh.assumed {
		return
	}
	if err := pr.Enc.Forget(pr.Engine, pod); err != nil {
		klog.ErrorS(err, "ksim: Unreserve", "pod", klog.KObj(pod))
	}
	c.sh.assumed = false
}

// PostBind: the pod is bound; the snapshot keeps it (the informer's report of
// the binding finds it assumed already).
func (p *KsimAssume) PostBind(ctx context.Context, state *framework.CycleState, pod *v1.Pod, nodeName string) {}

// ---- DefaultPreemption --------------------------------------------------------------
type postFilter struct{ *base }

// PostFilter restates DefaultPreemption.PostFilter / Evaluator.Preempt (v1.26
// default_preemption.go, preemption.go) around the engine's dry run.
func (p *postFilter) PostFilter(ctx context.Context, state *framework.CycleState, pod *v1.Pod,
	m framework.NodeToStatusMap) (*framework.PostFilterResult, *framework.Status) {
	c := readCycle(state)
	if c == nil || c.refused {
		return p.orig.(framework.PostFilterPlugin).PostFilter(ctx, state, pod, m)
	}
	pr := p.prof()
	// 0) the latest version of the pod (its nominatedNodeName)
	if latest, err := p.f.SharedInformerFactory().Core().V1().Pods().Lister().Pods(pod.Namespace).Get(pod.Name); err == nil {
		pod = latest
	} else {
		return nil, framework.AsStatus(err)
	}
	prio := corev1helpers.PodPriority(pod)
	// 1) PodEligibleToPreemptOthers
	if pod.Spec.PreemptionPolicy != nil && *pod.Spec.PreemptionPolicy == v1.PreemptNever {
		return nil, framework.NewStatus(framework.Unschedulable, "preemption: not eligible due to preemptionPolicy=Never.")
	}
	if nom := pod.Status.NominatedNodeName; nom != "" && m[nom].Code() != framework.UnschedulableAndUnresolvable {
		if ni, err := p.f.SnapshotSharedLister().NodeInfos().Get(nom); err == nil {
			for _, q := range ni.Pods {
				if q.Pod.DeletionTimestamp != nil && corev1helpers.PodPriority(q.Pod) < prio {
					return nil, framework.NewStatus(framework.Unschedulable,
						"preemption: not eligible due to a terminating pod on the nominated node.")
				}
			}
		}
	}
	// 2) the dry run, with the PodNominator's pods of priority >= the pod's
	// (SelectVictimsOnNode filters through RunFilterPluginsWithNominatedPods)
	var noms []*v1.Pod
	var gnodes, first, count []C.int32_t
	for pos, name := range pr.Enc.NodeNames() {
		k := 0
		for _, q := range p.f.NominatedPodsForNode(name) {
			if q.Pod.UID != pod.UID && corev1helpers.PodPriority(q.Pod) >= prio {
				noms = append(noms, q.Pod)
				k++
			}
		}
		if k > 0 {
			gnodes = append(gnodes, C.int32_t(pos))
			first = append(first, C.int32_t(len(noms)-k))
			count = append(count, C.int32_t(k))
		}
	}
	var nps *C.ksim_pod_set
	var gn, gf, gc *C.int32_t
	if len(noms) > 0 {
		set, release, err := pr.Enc.Pods(noms)
		if err != nil {
			return nil, framework.AsStatus(err)
		}
		defer release()
		nps, gn, gf, gc = set, &gnodes[0], &first[0], &count[0]
	}
	if err := pr.Enc.BoundTable(pr.Engine); err != nil {
		return nil, framework.AsStatus(err)
	}
	victims := make([]int32, 1024)
	var out C.ksim_preempt_out
	out.victims = (*C.int32_t)(unsafe.Pointer(&victims[0]))
	out.victims_cap = C.int32_t(len(victims))
	pr.Engine.mu.Lock()
	rc := C.ksim_preempt_nominated(pr.Engine.h, c.ps, 0, C.int32_t(prio), nps, C.int32_t(len(gnodes)), gn, gf, gc, &out)
	perr := pr.Engine.err(rc) // under the mutex: the handle's last error is this call's
	pr.Engine.mu.Unlock()
	if rc == C.KSIM_E_UNSUPPORTED {
		return p.orig.(framework.PostFilterPlugin).PostFilter(ctx, state, pod, m)
	}
	if perr != nil {
		return nil, framework.AsStatus(perr)
	}
	if out.nominated < 0 {
		// no candidate: ModeOverride "" clears the pod's nomination
		return framework.NewPostFilterResultWithNominatedNode(""),
			framework.NewStatus(framework.Unschedulable, "preemption: no candidate node")
	}
	// 5) prepareCandidate (PodDisruptionBudgets are out of the engine's scope,
	// DESIGN.md §8): reject waiting victims, else patch the DisruptionTarget
	// condition (PodDisruptionConditions, beta in v1.26; upstream builds the
	// new status from the preemptor's own status, restated as is) and delete
	// with the default grace period; then clear the nominations of
	// lower-priority pods nominated on the node.
	cs := p.f.ClientSet()
	for i := 0; i < int(out.n_victims) && i < len(victims); i++ {
		v := pr.Enc.BoundPod(int(victims[i]))
		if wp := p.f.GetWaitingPod(v.UID); wp != nil {
			wp.Reject("DefaultPreemption", "preempted")
			continue
		}
		if utilfeature.DefaultFeatureGate.Enabled(features.PodDisruptionConditions) {
			cond := &v1.PodCondition{Type: v1.DisruptionTarget, Status: v1.ConditionTrue,
				Reason:  v1.PodReasonPreemptionByScheduler,
				Message: fmt.Sprintf("%s: preempting to accommodate a higher priority pod", pod.Spec.SchedulerName)}
			st := pod.Status.DeepCopy()
			if apipod.UpdatePodCondition(st, cond) {
				if err := schedutil.PatchPodStatus(ctx, cs, v, st); err != nil {
					return nil, framework.AsStatus(err)
				}
			}
		}
		if err := schedutil.DeletePod(ctx, cs, v); err != nil {
			return nil, framework.AsStatus(err)
		}
		p.f.EventRecorder().Eventf(v, pod, v1.EventTypeNormal, "Preempted", "Preempting",
			"Preempted by a pod on node %v", pr.Enc.NodeNames()[int(out.nominated)])
	}
	name := pr.Enc.NodeNames()[int(out.nominated)]
	var lower []*v1.Pod
	for _, q := range p.f.NominatedPodsForNode(name) {
		if corev1helpers.PodPriority(q.Pod) < prio {
			lower = append(lower, q.Pod)
		}
	}
	if len(lower) > 0 {
		if err := schedutil.ClearNominatedNodeName(ctx, cs, lower...); err != nil {
			klog.ErrorS(err, "Cannot clear 'NominatedNodeName' field")
		}
	}
	return framework.NewPostFilterResultWithNominatedNode(name), framework.NewStatus(framework.Success)
}
