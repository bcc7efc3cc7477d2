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
//	cd oracle/go && go run . ../../tests/golden/go/*.json.gz
package main

import (
	"compress/gzip"
	"context"
	"encoding/json"
	"fmt"
	"os"
	"strings"

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
	frameworkruntime "k8s.io/kubernetes/pkg/scheduler/framework/runtime"
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
}

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
// (NewPluginConfig, plugins.go:103-179), converted to the internal types.
func defaultArgs(hardW int32) (map[string]runtime.Object, error) {
	versioned := &configv1beta2.KubeSchedulerConfiguration{}
	scheme.Scheme.Default(versioned)
	var internal config.KubeSchedulerConfiguration
	if err := scheme.Scheme.Convert(versioned, &internal, nil); err != nil {
		return nil, err
	}
	args := map[string]runtime.Object{}
	for _, pc := range internal.Profiles[0].PluginConfig {
		args[pc.Name] = pc.Args
	}
	if a, ok := args["InterPodAffinity"].(*config.InterPodAffinityArgs); ok && hardW > 0 {
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
	informerFactory := informers.NewSharedInformerFactory(client, 0)
	snap := newSnapshot(f)
	args, err := defaultArgs(f.HardPodAffinityWeight)
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
		K := int(numFeasibleNodesToFind(f.Pct, int32(N)))
		// findNodesThatPassFilters, parallelism 1
		var feasible []*framework.NodeInfo
		failed := 0
		for i := 0; i < N; i++ {
			ni := scan[(nextStart+i)%N]
			var rec interface{} = "passed"
			for _, name := range filterOrder {
				st := pl[name].(framework.FilterPlugin).Filter(ctx, state, pod, ni)
				if !st.IsSuccess() {
					if st.Code() == framework.Error {
						return nil, fmt.Errorf("pod %s: Filter %s on %s: %s", pod.Name, name, ni.Node().Name, st.Message())
					}
					rec = []interface{}{name, st.Message()}
					break
				}
			}
			c.Filter[ni.Node().Name] = rec
			if rec == "passed" {
				if len(feasible) == K {
					break // the (K+1)-th feasible node: recorded, not kept
				}
				feasible = append(feasible, ni)
			} else {
				failed++
			}
		}
		nextStart = (nextStart + len(feasible) + failed) % N
		c.NextStart = nextStart
		c.NFeasible = len(feasible)
		var chosen *framework.NodeInfo
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
			chosen.AddPod(pod) // assume
		}
		out = append(out, c)
	}
	return out, nil
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
