// Command ksimgo runs the Go-harness fixtures (tests/golden/go/<case>.json.gz)
// through the upstream in-tree scheduler plugins of k8s.io/kubernetes v1.26.2,
// the module the reference builds its scheduler from (simulator/go.mod:53), and
// writes <case>.go.json.gz next to each fixture.  tests/test_go_fixtures.py then
// compares those cycles with the ones the restatement recorded: that is the
// only route to pinning the engine's plugin arithmetic against the reference
// (SURVEY §8(c), golden vectors item 4).
//
// TEST INFRASTRUCTURE, NOT BUILT HERE: the build container has no Go toolchain
// and no module cache, so this file has never been compiled.  The framework
// API it calls is v1.26's as recalled (SURVEY Appendix C); fix what the
// compiler reports before trusting a run.
//
// What it mirrors (the reference's wrapped plugins call the original plugins
// one by one and record each result, wrappedplugin.go:346-516):
//   - the plugins are built from plugins.NewInTreeRegistry() with the default
//     profile's args, as newPluginFactories does (plugins.go:46-92);
//   - PreFilter, then Filter over the nodes in nodeTree order from
//     nextStartNodeIndex, first failing plugin per node, sequential scan
//     (parallelism 1) stopping at the (K+1)-th feasible node, K =
//     numFeasibleNodesToFind (SURVEY §8(b) ADAPT / P100);
//   - PreScore, Score, NormalizeScore, weights (0 -> 1), and selectHost by the
//     fixed-seed tie-break TB(seed) of SURVEY §8(b) instead of the global
//     math/rand reservoir;
//   - the chosen node's NodeInfo.AddPod (assume).
//
// Round 5 cases (tools/make_go_fixtures.py "optional inputs"):
//   - profile.pluginConfig: the v1beta2 args decoded over the defaults,
//     defaulted and converted (NewPluginConfig, plugins.go:103-179);
//   - services / replicaSets / statefulSets / replicationControllers and pvs /
//     pvcs: created in the fake clientset before the informers sync (the
//     listers PodTopologySpread's DefaultSelector and VolumeBinding read);
//   - nominatedPods / cycleInputs: the PodNominator of each cycle:
//     RunFilterPluginsWithNominatedPods (pass 1 on a clone carrying the node's
//     nominated pods of priority >= the pod's, PreFilterExtensions.AddPod, then
//     pass 2) and evaluateNominatedNode (schedule_one.go v1.26);
//   - preemption: after an unschedulable cycle, DefaultPreemption's dry run
//     with the candidate search from offset 0 (the deterministic stand-in for
//     GetOffsetAndNumCandidates' random offset): potential nodes are those whose
//     status is Unschedulable, SelectVictimsOnNode per node, the first
//     numCandidates candidates, pickOneNodeForPreemption restated below.
//
//	cd oracle/go && go run . ../../tests/golden/go/*.json.gz
package main

import (
	"compress/gzip"
	"context"
	"encoding/json"
	"fmt"
	"math"
	"os"
	"sort"
	"strings"
	"time"

	appsv1 "k8s.io/api/apps/v1"
	v1 "k8s.io/api/core/v1"
	metav1 "k8s.io/apimachinery/pkg/apis/meta/v1"
	"k8s.io/apimachinery/pkg/runtime"
	"k8s.io/client-go/informers"
	clientsetfake "k8s.io/client-go/kubernetes/fake"
	configv1beta2 "k8s.io/kube-scheduler/config/v1beta2"
	"k8s.io/kubernetes/pkg/scheduler/apis/config"
	"k8s.io/kubernetes/pkg/scheduler/apis/config/scheme"
	"k8s.io/kubernetes/pkg/scheduler/framework"
	"k8s.io/kubernetes/pkg/scheduler/framework/plugins"
	"k8s.io/kubernetes/pkg/scheduler/framework/plugins/defaultpreemption"
	frameworkruntime "k8s.io/kubernetes/pkg/scheduler/framework/runtime"
	corev1helpers "k8s.io/component-helpers/scheduling/corev1"
)

// The simulator's default profile (scheduler_test.go:388-437).
var (
	preFilterOrder = []string{"NodeResourcesFit", "NodePorts", "VolumeRestrictions", "PodTopologySpread",
		"InterPodAffinity", "VolumeBinding", "NodeAffinity"}
	filterOrder = []string{"NodeUnschedulable", "NodeName", "TaintToleration", "NodeAffinity", "NodePorts",
		"NodeResourcesFit", "VolumeRestrictions", "EBSLimits", "GCEPDLimits", "NodeVolumeLimits",
		"AzureDiskLimits", "VolumeBinding", "VolumeZone", "PodTopologySpread", "InterPodAffinity"}
	preScoreOrder = []string{"InterPodAffinity", "PodTopologySpread", "TaintToleration", "NodeAffinity"}
	scoreOrder    = []string{"NodeResourcesBalancedAllocation", "ImageLocality", "InterPodAffinity",
		"NodeResourcesFit", "NodeAffinity", "PodTopologySpread", "TaintToleration"}
	scoreWeight = map[string]int64{"NodeResourcesBalancedAllocation": 1, "ImageLocality": 1,
		"InterPodAffinity": 1, "NodeResourcesFit": 1, "NodeAffinity": 1, "PodTopologySpread": 2,
		"TaintToleration": 1}
)

type fixture struct {
	Name                  string                       `json:"name"`
	Pct                   int32                        `json:"percentageOfNodesToScore"`
	Seed                  uint64                       `json:"tiebreakSeed"`
	HardPodAffinityWeight int32                        `json:"hardPodAffinityWeight"`
	Namespaces            map[string]map[string]string `json:"namespaces"`
	Nodes                 []v1.Node                    `json:"nodes"`
	BoundPods             []v1.Pod                     `json:"boundPods"`
	Pods                  []v1.Pod                     `json:"pods"`
	// round 5 (optional)
	Profile                *configv1beta2.KubeSchedulerProfile `json:"profile"`
	Services               []v1.Service                        `json:"services"`
	ReplicaSets            []appsv1.ReplicaSet                 `json:"replicaSets"`
	StatefulSets           []appsv1.StatefulSet                `json:"statefulSets"`
	ReplicationControllers []v1.ReplicationController          `json:"replicationControllers"`
	PVs                    []v1.PersistentVolume               `json:"pvs"`
	PVCs                   []v1.PersistentVolumeClaim          `json:"pvcs"`
	NominatedPods          []v1.Pod                            `json:"nominatedPods"`
	CycleInputs            []struct {
		Nominator         map[string][]string `json:"nominator"`
		NominatedNodeName *string             `json:"nominatedNodeName"`
	} `json:"cycleInputs"`
	Preemption bool `json:"preemption"`
}

// assumedStart: status.startTime of queue pod i once assumed (seconds after
// 2022-01-01T00:00:00Z; tools/make_go_fixtures.py ASSUMED_START)
const assumedStart = 20000

// One cycle in the schema of tests/golden/go (tools/make_go_fixtures.py).
type cycle struct {
	Pod        string                      `json:"pod"`
	Chosen     *string                     `json:"chosen"`
	NextStart  int                         `json:"nextStartNodeIndex"`
	NFeasible  int                         `json:"nFeasible"`
	Filter     map[string]interface{}      `json:"filter"`
	Score      map[string]map[string]int64 `json:"score"`
	Normalized map[string]map[string]int64 `json:"normalized"`
	Total      map[string]int64            `json:"total"`
	PostFilter *postFilter                 `json:"postFilter,omitempty"`
}

type postFilter struct {
	NominatedNode *string  `json:"nominatedNode"`
	Victims       []string `json:"victims"`
}

// snapshot is the framework.SharedLister the plugins read: NodeInfos in
// nodeTree order (the fixture's node order), mutated in place by assume.
type snapshot struct {
	list   []*framework.NodeInfo
	byName map[string]*framework.NodeInfo
}

func (s *snapshot) NodeInfos() framework.NodeInfoLister       { return s }
func (s *snapshot) StorageInfos() framework.StorageInfoLister { return s }
func (s *snapshot) List() ([]*framework.NodeInfo, error)      { return s.list, nil }
func (s *snapshot) IsPVCUsedByPods(string) bool               { return false }

func (s *snapshot) HavePodsWithAffinityList() ([]*framework.NodeInfo, error) {
	var out []*framework.NodeInfo
	for _, ni := range s.list {
		if len(ni.PodsWithAffinity) > 0 {
			out = append(out, ni)
		}
	}
	return out, nil
}

func (s *snapshot) HavePodsWithRequiredAntiAffinityList() ([]*framework.NodeInfo, error) {
	var out []*framework.NodeInfo
	for _, ni := range s.list {
		if len(ni.PodsWithRequiredAntiAffinity) > 0 {
			out = append(out, ni)
		}
	}
	return out, nil
}

func (s *snapshot) Get(name string) (*framework.NodeInfo, error) {
	if ni, ok := s.byName[name]; ok {
		return ni, nil
	}
	return nil, fmt.Errorf("nodeinfo not found for node name %q", name)
}

func newSnapshot(f *fixture) *snapshot {
	s := &snapshot{byName: map[string]*framework.NodeInfo{}}
	// cache.addNodeImageStates: size from the first node listing the name,
	// NumNodes = nodes listing it
	type img struct {
		size  int64
		nodes map[string]bool
	}
	images := map[string]*img{}
	for i := range f.Nodes {
		n := &f.Nodes[i]
		for _, im := range n.Status.Images {
			for _, name := range im.Names {
				if images[name] == nil {
					images[name] = &img{im.SizeBytes, map[string]bool{}}
				}
				images[name].nodes[n.Name] = true
			}
		}
	}
	for i := range f.Nodes {
		n := &f.Nodes[i]
		ni := framework.NewNodeInfo()
		ni.SetNode(n)
		for _, im := range n.Status.Images {
			for _, name := range im.Names {
				ni.ImageStates[name] = &framework.ImageStateSummary{Size: images[name].size,
					NumNodes: len(images[name].nodes)}
			}
		}
		s.list = append(s.list, ni)
		s.byName[n.Name] = ni
	}
	for i := range f.BoundPods {
		p := &f.BoundPods[i]
		if ni, ok := s.byName[p.Spec.NodeName]; ok {
			ni.AddPod(p)
		}
	}
	return s
}

// numFeasibleNodesToFind (schedule_one.go) with the simulator's parallelism-1 scan.
func numFeasibleNodesToFind(pct int32, n int32) int32 {
	if n < 100 || pct >= 100 {
		return n
	}
	adaptive := pct
	if adaptive <= 0 {
		adaptive = 50 - n/125
		if adaptive < 5 {
			adaptive = 5
		}
	}
	num := n * adaptive / 100
	if num < 100 {
		return 100
	}
	return num
}

func splitmix64(x uint64) uint64 {
	z := x + 0x9E3779B97F4A7C15
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9
	z = (z ^ (z >> 27)) * 0x94D049BB133111EB
	return z ^ (z >> 31)
}

// tbLo is the tie-break word of SURVEY §8(b)'s TB(seed) (ksim_oracle_tb_lo):
// selectHost takes the max of (total, tbLo) in lexicographic order.
func tbLo(seed uint64, seq int64, node int) uint64 {
	const nodeMask = (1 << 18) - 1
	h := splitmix64(seed^(uint64(seq)<<20)^uint64(node)) >> 38
	return h<<18 | uint64(nodeMask-node)
}

// defaultArgs: the v1beta2 defaults the simulator starts from
// (NewPluginConfig, plugins.go:103-179), with the fixture profile's
// pluginConfig decoded over them, converted to the internal types.
func defaultArgs(hardW int32, prof *configv1beta2.KubeSchedulerProfile) (map[string]runtime.Object, error) {
	versioned := &configv1beta2.KubeSchedulerConfiguration{}
	if prof != nil {
		versioned.Profiles = []configv1beta2.KubeSchedulerProfile{*prof.DeepCopy()}
	}
	scheme.Scheme.Default(versioned)
	var internal config.KubeSchedulerConfiguration
	if err := scheme.Scheme.Convert(versioned, &internal, nil); err != nil {
		return nil, err
	}
	args := map[string]runtime.Object{}
	for _, pc := range internal.Profiles[0].PluginConfig {
		args[pc.Name] = pc.Args
	}
	if a, ok := args["InterPodAffinity"].(*config.InterPodAffinityArgs); ok && hardW > 0 && prof == nil {
		a.HardPodAffinityWeight = hardW
	}
	return args, nil
}

func run(f *fixture) ([]cycle, error) {
	ctx := context.Background()
	stop := make(chan struct{})
	defer close(stop)

	client := clientsetfake.NewSimpleClientset()
	for ns, labels := range f.Namespaces {
		if _, err := client.CoreV1().Namespaces().Create(ctx,
			&v1.Namespace{ObjectMeta: metav1.ObjectMeta{Name: ns, Labels: labels}}, metav1.CreateOptions{}); err != nil {
			return nil, err
		}
	}
	for i := range f.Services {
		if _, err := client.CoreV1().Services(f.Services[i].Namespace).Create(ctx, &f.Services[i], metav1.CreateOptions{}); err != nil {
			return nil, err
		}
	}
	for i := range f.ReplicationControllers {
		rc := &f.ReplicationControllers[i]
		if _, err := client.CoreV1().ReplicationControllers(rc.Namespace).Create(ctx, rc, metav1.CreateOptions{}); err != nil {
			return nil, err
		}
	}
	for i := range f.ReplicaSets {
		rs := &f.ReplicaSets[i]
		if _, err := client.AppsV1().ReplicaSets(rs.Namespace).Create(ctx, rs, metav1.CreateOptions{}); err != nil {
			return nil, err
		}
	}
	for i := range f.StatefulSets {
		ss := &f.StatefulSets[i]
		if _, err := client.AppsV1().StatefulSets(ss.Namespace).Create(ctx, ss, metav1.CreateOptions{}); err != nil {
			return nil, err
		}
	}
	for i := range f.PVs {
		if _, err := client.CoreV1().PersistentVolumes().Create(ctx, &f.PVs[i], metav1.CreateOptions{}); err != nil {
			return nil, err
		}
	}
	for i := range f.PVCs {
		c := &f.PVCs[i]
		if _, err := client.CoreV1().PersistentVolumeClaims(c.Namespace).Create(ctx, c, metav1.CreateOptions{}); err != nil {
			return nil, err
		}
	}
	informerFactory := informers.NewSharedInformerFactory(client, 0)
	snap := newSnapshot(f)
	args, err := defaultArgs(f.HardPodAffinityWeight, f.Profile)
	if err != nil {
		return nil, err
	}
	profile := &config.KubeSchedulerProfile{SchedulerName: v1.DefaultSchedulerName, Plugins: &config.Plugins{}}
	registry := plugins.NewInTreeRegistry()
	fwk, err := frameworkruntime.NewFramework(registry, profile, stop,
		frameworkruntime.WithClientSet(client),
		frameworkruntime.WithInformerFactory(informerFactory),
		frameworkruntime.WithSnapshotSharedLister(snap),
		frameworkruntime.WithParallelism(1))
	if err != nil {
		return nil, err
	}
	// the original plugins, built as the simulator's factories build them
	// (plugins.go:76: r(configuration, f)), with the framework as their Handle
	pl := map[string]framework.Plugin{}
	names := append(append(append([]string{}, filterOrder...), scoreOrder...), preFilterOrder...)
	if f.Preemption {
		names = append(names, "DefaultPreemption")
	}
	for _, name := range names {
		if pl[name] != nil {
			continue
		}
		p, err := registry[name](args[name], fwk)
		if err != nil {
			return nil, fmt.Errorf("plugin %s: %w", name, err)
		}
		pl[name] = p
	}
	informerFactory.Start(stop)
	informerFactory.WaitForCacheSync(stop)

	index := map[string]int{}
	for i, ni := range snap.list {
		index[ni.Node().Name] = i
	}
	nominatedByName := map[string]*v1.Pod{}
	for i := range f.NominatedPods {
		nominatedByName[f.NominatedPods[i].Name] = &f.NominatedPods[i]
	}
	// RunFilterPlugins: the first failing plugin (name, status) or nil
	runFilters := func(state *framework.CycleState, pod *v1.Pod, ni *framework.NodeInfo) (string, *framework.Status) {
		for _, name := range filterOrder {
			if st := pl[name].(framework.FilterPlugin).Filter(ctx, state, pod, ni); !st.IsSuccess() {
				return name, st
			}
		}
		return "", nil
	}
	// RunFilterPluginsWithNominatedPods (framework/runtime/framework.go v1.26)
	filterWithNominated := func(seq int, state *framework.CycleState, pod *v1.Pod, ni *framework.NodeInfo) (string, *framework.Status) {
		var add []*v1.Pod
		if seq < len(f.CycleInputs) {
			for _, n := range f.CycleInputs[seq].Nominator[ni.Node().Name] {
				q := nominatedByName[n]
				if q != nil && corev1helpers.PodPriority(q) >= corev1helpers.PodPriority(pod) && q.UID != pod.UID &&
					q.Name != pod.Name {
					add = append(add, q)
				}
			}
		}
		if len(add) > 0 {
			stateOut := state.Clone()
			niOut := ni.Clone()
			for _, q := range add {
				pi := framework.NewPodInfo(q)
				niOut.AddPodInfo(pi)
				for _, name := range preFilterOrder {
					if p, ok := pl[name].(framework.PreFilterPlugin); ok && p.PreFilterExtensions() != nil {
						if st := p.PreFilterExtensions().AddPod(ctx, stateOut, pod, pi, niOut); !st.IsSuccess() {
							return name, st
						}
					}
				}
			}
			if name, st := runFilters(stateOut, pod, niOut); st != nil {
				return name, st
			}
		}
		return runFilters(state, pod, ni)
	}
	startOf := map[string]time.Time{}
	base := time.Date(2022, 1, 1, 0, 0, 0, 0, time.UTC)
	for i := range f.BoundPods {
		if st := f.BoundPods[i].Status.StartTime; st != nil {
			startOf[f.BoundPods[i].Name] = st.Time
		}
	}
	nextStart := 0
	var out []cycle
	for seq := range f.Pods {
		pod := f.Pods[seq].DeepCopy()
		c := cycle{Pod: pod.Name, Filter: map[string]interface{}{}, Score: map[string]map[string]int64{},
			Normalized: map[string]map[string]int64{}, Total: map[string]int64{}}
		state := framework.NewCycleState()
		var preRes *framework.PreFilterResult
		for _, name := range preFilterOrder {
			if p, ok := pl[name].(framework.PreFilterPlugin); ok {
				r, st := p.PreFilter(ctx, state, pod)
				if !st.IsSuccess() {
					return nil, fmt.Errorf("pod %s: PreFilter %s: %s (not modelled)", pod.Name, name, st.Message())
				}
				preRes = preRes.Merge(r)
			}
		}
		// findNodesThatFitPod: a PreFilterResult restricts the scan to its nodes,
		// taken in nodeTree order (upstream ranges over the set in Go map order)
		scan := snap.list
		if !preRes.AllNodes() {
			scan = nil
			for _, ni := range snap.list {
				if preRes.NodeNames.Has(ni.Node().Name) {
					scan = append(scan, ni)
				}
			}
			if len(scan) != len(preRes.NodeNames) {
				return nil, fmt.Errorf("pod %s: PreFilterResult names a node outside the snapshot (not modelled)", pod.Name)
			}
		}
		N := len(scan)
		if N == 0 {
			return nil, fmt.Errorf("pod %s: empty PreFilterResult (not modelled)", pod.Name)
		}
		statuses := map[string]*framework.Status{}
		var chosen *framework.NodeInfo
		var feasible []*framework.NodeInfo
		failed := map[string]bool{}
		nominatedPass := false
		// evaluateNominatedNode (schedule_one.go v1.26): the pod's nominated node
		// first; passing, it is the only feasible node and nextStartNodeIndex
		// stays; failing, its status stays in the diagnosis
		if seq < len(f.CycleInputs) && f.CycleInputs[seq].NominatedNodeName != nil {
			if ni, ok := snap.byName[*f.CycleInputs[seq].NominatedNodeName]; ok {
				name, st := filterWithNominated(seq, state, pod, ni)
				if st == nil {
					c.Filter[ni.Node().Name] = "passed"
					feasible, nominatedPass = []*framework.NodeInfo{ni}, true
				} else {
					if st.Code() == framework.Error {
						return nil, fmt.Errorf("pod %s: Filter %s: %s", pod.Name, name, st.Message())
					}
					c.Filter[ni.Node().Name] = []interface{}{name, st.Message()}
					statuses[ni.Node().Name] = st
					failed[ni.Node().Name] = true
				}
			}
		}
		if !nominatedPass {
			K := int(numFeasibleNodesToFind(f.Pct, int32(N)))
			// findNodesThatPassFilters, parallelism 1
			for i := 0; i < N; i++ {
				ni := scan[(nextStart+i)%N]
				var rec interface{} = "passed"
				if name, st := filterWithNominated(seq, state, pod, ni); st != nil {
					if st.Code() == framework.Error {
						return nil, fmt.Errorf("pod %s: Filter %s on %s: %s", pod.Name, name, ni.Node().Name, st.Message())
					}
					rec = []interface{}{name, st.Message()}
					statuses[ni.Node().Name] = st
				}
				c.Filter[ni.Node().Name] = rec
				if rec == "passed" {
					if len(feasible) == K {
						break // the (K+1)-th feasible node: recorded, not kept
					}
					feasible = append(feasible, ni)
				} else {
					failed[ni.Node().Name] = true
				}
			}
			nextStart = (nextStart + len(feasible) + len(failed)) % N
		}
		c.NextStart = nextStart
		c.NFeasible = len(feasible)
		switch {
		case len(feasible) == 0:
		case len(feasible) == 1:
			chosen = feasible[0] // schedulePod returns it without scoring
		default:
			nodes := make([]*v1.Node, len(feasible))
			for j, ni := range feasible {
				nodes[j] = ni.Node()
			}
			for _, name := range preScoreOrder {
				if p, ok := pl[name].(framework.PreScorePlugin); ok {
					if st := p.PreScore(ctx, state, pod, nodes); !st.IsSuccess() {
						return nil, fmt.Errorf("pod %s: PreScore %s: %s", pod.Name, name, st.Message())
					}
				}
			}
			totals := make([]int64, len(feasible))
			for _, name := range scoreOrder {
				p := pl[name].(framework.ScorePlugin)
				list := make(framework.NodeScoreList, len(feasible))
				raw := map[string]int64{}
				for j, n := range nodes {
					s, st := p.Score(ctx, state, pod, n.Name)
					if !st.IsSuccess() {
						return nil, fmt.Errorf("pod %s: Score %s: %s", pod.Name, name, st.Message())
					}
					list[j] = framework.NodeScore{Name: n.Name, Score: s}
					raw[n.Name] = s
				}
				if ext := p.ScoreExtensions(); ext != nil {
					if st := ext.NormalizeScore(ctx, state, pod, list); !st.IsSuccess() {
						return nil, fmt.Errorf("pod %s: NormalizeScore %s: %s", pod.Name, name, st.Message())
					}
				}
				norm := map[string]int64{}
				w := scoreWeight[name]
				if w == 0 {
					w = 1
				}
				for j, ns := range list {
					norm[ns.Name] = ns.Score
					totals[j] += ns.Score * w
				}
				c.Score[name] = raw
				c.Normalized[name] = norm
			}
			best := -1
			var bestTotal int64
			var bestLo uint64
			for j, n := range nodes {
				c.Total[n.Name] = totals[j]
				lo := tbLo(f.Seed, int64(seq), index[n.Name])
				if best < 0 || totals[j] > bestTotal || (totals[j] == bestTotal && lo > bestLo) {
					best, bestTotal, bestLo = j, totals[j], lo
				}
			}
			chosen = feasible[best]
		}
		if chosen != nil {
			name := chosen.Node().Name
			c.Chosen = &name
			pod.Spec.NodeName = name
			if f.Preemption {
				st := metav1.NewTime(base.Add(time.Duration(assumedStart+seq) * time.Second))
				pod.Status.StartTime = &st
				startOf[pod.Name] = st.Time
			}
			chosen.AddPod(pod) // assume
		} else if f.Preemption {
			pf, err := preempt(ctx, pl["DefaultPreemption"].(*defaultpreemption.DefaultPreemption), state, pod,
				snap, statuses, args, startOf)
			if err != nil {
				return nil, fmt.Errorf("pod %s: preemption: %w", pod.Name, err)
			}
			c.PostFilter = pf
		}
		out = append(out, c)
	}
	return out, nil
}

// preempt: DefaultPreemption's dry run (preemption.Evaluator.findCandidates +
// SelectCandidate, v1.26) with the candidate search from offset 0.  Potential
// nodes: status Unschedulable (nodesWherePreemptionMightHelp drops
// UnschedulableAndUnresolvable), in nodeTree order; SelectVictimsOnNode is
// the plugin's own; pickOneNodeForPreemption is restated (unexported upstream).
func preempt(ctx context.Context, dp *defaultpreemption.DefaultPreemption, state *framework.CycleState, pod *v1.Pod,
	snap *snapshot, statuses map[string]*framework.Status, args map[string]runtime.Object,
	startOf map[string]time.Time) (*postFilter, error) {
	var potential []*framework.NodeInfo
	for _, ni := range snap.list {
		if st, ok := statuses[ni.Node().Name]; ok && st.Code() == framework.Unschedulable {
			potential = append(potential, ni)
		}
	}
	pa := args["DefaultPreemption"].(*config.DefaultPreemptionArgs)
	// GetOffsetAndNumCandidates (default_preemption.go v1.26)
	want := len(potential) * int(pa.MinCandidateNodesPercentage) / 100
	if want < int(pa.MinCandidateNodesAbsolute) {
		want = int(pa.MinCandidateNodesAbsolute)
	}
	if want > len(potential) {
		want = len(potential)
	}
	type cand struct {
		node    string
		victims []*v1.Pod
	}
	var cands []cand
	for _, ni := range potential {
		if len(cands) >= want {
			break
		}
		victims, _, st := dp.SelectVictimsOnNode(ctx, state.Clone(), pod, ni.Clone(), nil)
		if st.IsSuccess() {
			cands = append(cands, cand{ni.Node().Name, victims})
		}
	}
	none := &postFilter{Victims: []string{}}
	if len(cands) == 0 {
		return none, nil
	}
	// pickOneNodeForPreemption (preemption.go v1.26): lowest highest-victim
	// priority, lowest sum of (priority + MaxInt32 + 1), fewest victims, latest
	// earliest start time of the highest-priority victims, first candidate
	start := func(p *v1.Pod) time.Time { return startOf[p.Name] }
	best := 0
	key := func(c cand) (int32, int64, int, time.Time) {
		if len(c.victims) == 0 {
			return math.MinInt32, 0, 0, time.Time{}
		}
		hi := corev1helpers.PodPriority(c.victims[0])
		var sum int64
		earliest := start(c.victims[0])
		for _, v := range c.victims {
			pr := corev1helpers.PodPriority(v)
			if pr > hi {
				hi = pr
			}
			sum += int64(pr) + int64(math.MaxInt32) + 1
		}
		for _, v := range c.victims {
			if corev1helpers.PodPriority(v) == hi && start(v).Before(earliest) {
				earliest = start(v)
			}
		}
		return hi, sum, len(c.victims), earliest
	}
	for i := 1; i < len(cands); i++ {
		h0, s0, n0, t0 := key(cands[best])
		h1, s1, n1, t1 := key(cands[i])
		switch {
		case h1 != h0:
			if h1 < h0 {
				best = i
			}
		case s1 != s0:
			if s1 < s0 {
				best = i
			}
		case n1 != n0:
			if n1 < n0 {
				best = i
			}
		case !t1.Equal(t0):
			if t1.After(t0) {
				best = i
			}
		}
	}
	// the victims in MoreImportantPod order (SelectVictimsOnNode's result order)
	vs := cands[best].victims
	sort.SliceStable(vs, func(a, b int) bool {
		pa, pb := corev1helpers.PodPriority(vs[a]), corev1helpers.PodPriority(vs[b])
		if pa != pb {
			return pa > pb
		}
		return start(vs[a]).Before(start(vs[b]))
	})
	names := make([]string, len(vs))
	for i, v := range vs {
		names[i] = v.Name
	}
	node := cands[best].node
	return &postFilter{NominatedNode: &node, Victims: names}, nil
}

func main() {
	if len(os.Args) < 2 {
		fmt.Fprintln(os.Stderr, "usage: ksimgo <fixture.json.gz>...")
		os.Exit(2)
	}
	for _, path := range os.Args[1:] {
		if strings.HasSuffix(path, ".go.json.gz") {
			continue
		}
		fh, err := os.Open(path)
		if err != nil {
			panic(err)
		}
		zr, err := gzip.NewReader(fh)
		if err != nil {
			panic(err)
		}
		var f fixture
		if err := json.NewDecoder(zr).Decode(&f); err != nil {
			panic(fmt.Errorf("%s: %w", path, err))
		}
		fh.Close()
		cycles, err := run(&f)
		if err != nil {
			panic(fmt.Errorf("%s: %w", path, err))
		}
		outPath := strings.TrimSuffix(path, ".json.gz") + ".go.json.gz"
		of, err := os.Create(outPath)
		if err != nil {
			panic(err)
		}
		zw := gzip.NewWriter(of)
		if err := json.NewEncoder(zw).Encode(map[string]interface{}{"name": f.Name, "cycles": cycles}); err != nil {
			panic(err)
		}
		zw.Close()
		of.Close()
		fmt.Printf("%s: %d cycles -> %s\n", path, len(cycles), outPath)
	}
}
