// The Encoder of the engine-backed plugins (plugins.go) over the engine's
// native snapshot encoder (include/ksim_engine.h, "native snapshot encoder";
// csrc/ksim_encode.cpp): v1.Node / v1.Pod objects are laid out as one flat
// ksim_k8s_pool (a string table and arrays of plain C structs: no Go pointer
// ever reaches C memory), and ksim_encode_nodes / ksim_encode_pods compile
// them into the engine's node table and pod sets exactly as ksim/encode.py
// does (tests/test_native_encode.py checks the C++ encoder byte for byte
// against it).
//
// The device snapshot is encoded whole once and then follows the informers'
// events and the framework's Reserve / Unreserve as deltas (ABI 11, "snapshot
// deltas"): NativeEncoder below; ksim/fwsnapshot.py is its Python mirror.
//
// NOT BUILT HERE (no Go toolchain in the build container).
package engine

/*
#include <stdlib.h>
#include <string.h>
#include "ksim_engine.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"sort"
	"strings"
	"sync"
	"unsafe"

	v1 "k8s.io/api/core/v1"
	"k8s.io/apimachinery/pkg/api/equality"
	"k8s.io/apimachinery/pkg/api/resource"
	metav1 "k8s.io/apimachinery/pkg/apis/meta/v1"
	"k8s.io/apimachinery/pkg/util/sets"
	"k8s.io/client-go/tools/cache"
	"k8s.io/kubernetes/pkg/scheduler/framework"
)

// ---- the flat pool --------------------------------------------------------------

type pool struct {
	ids         map[string]int32
	blob        []byte
	off         []int64
	strList     []int32
	kv          []C.ksim_k8s_kv
	taints      []C.ksim_k8s_taint
	tols        []C.ksim_k8s_toleration
	reqs        []C.ksim_k8s_requirement
	terms       []C.ksim_k8s_selector_term
	preferred   []C.ksim_k8s_preferred_term
	selectors   []C.ksim_k8s_label_selector
	podTerms    []C.ksim_k8s_pod_term
	spread      []C.ksim_k8s_spread
	ports       []C.ksim_k8s_port
	containers  []C.ksim_k8s_container
	images      []C.ksim_k8s_image
	groups      []C.ksim_k8s_volume_group
	nodes       []C.ksim_k8s_node
	pods        []C.ksim_k8s_pod
	namespaces  []C.ksim_k8s_namespace
	services    []C.ksim_k8s_service
	controllers []C.ksim_k8s_controller
}

func newPool() *pool { return &pool{ids: map[string]int32{}, off: []int64{0}} }

func (p *pool) s(x string) C.int32_t {
	if i, ok := p.ids[x]; ok {
		return C.int32_t(i)
	}
	i := int32(len(p.off) - 1)
	p.ids[x] = i
	p.blob = append(p.blob, x...)
	p.off = append(p.off, int64(len(p.blob)))
	return C.int32_t(i)
}

func (p *pool) strs(xs []string) (C.int32_t, C.int32_t) {
	first := len(p.strList)
	for _, x := range xs {
		p.strList = append(p.strList, int32(p.s(x)))
	}
	return C.int32_t(first), C.int32_t(len(xs))
}

// Go maps have no order: keys are laid out sorted (the compile's outputs do not
// depend on the order; only label-column creation order follows it)
func sortedKeys[V any](m map[string]V) []string {
	ks := make([]string, 0, len(m))
	for k := range m {
		ks = append(ks, k)
	}
	sort.Strings(ks)
	return ks
}

func (p *pool) kvMap(m map[string]string) (C.int32_t, C.int32_t) {
	first := len(p.kv)
	for _, k := range sortedKeys(m) {
		p.kv = append(p.kv, C.ksim_k8s_kv{key: p.s(k), value: p.s(m[k])})
	}
	return C.int32_t(first), C.int32_t(len(m))
}

func (p *pool) resources(rl v1.ResourceList) (C.int32_t, C.int32_t) {
	first := len(p.kv)
	keys := make([]string, 0, len(rl))
	for k := range rl {
		keys = append(keys, string(k))
	}
	sort.Strings(keys)
	for _, k := range keys {
		q := rl[v1.ResourceName(k)]
		p.kv = append(p.kv, C.ksim_k8s_kv{key: p.s(k), value: p.s(q.String())})
	}
	return C.int32_t(first), C.int32_t(len(keys))
}

func (p *pool) nodeReqs(rs []v1.NodeSelectorRequirement) (C.int32_t, C.int32_t) {
	first := len(p.reqs)
	for _, r := range rs {
		vf, vc := p.strs(r.Values)
		p.reqs = append(p.reqs, C.ksim_k8s_requirement{key: p.s(r.Key), op: p.s(string(r.Operator)),
			values_first: vf, values_count: vc})
	}
	return C.int32_t(first), C.int32_t(len(rs))
}

func (p *pool) term(t v1.NodeSelectorTerm) C.int32_t {
	ef, ec := p.nodeReqs(t.MatchExpressions)
	ff, fc := p.nodeReqs(t.MatchFields)
	p.terms = append(p.terms, C.ksim_k8s_selector_term{exprs_first: ef, exprs_count: ec, fields_first: ff,
		fields_count: fc})
	return C.int32_t(len(p.terms) - 1)
}

func (p *pool) termList(ts []v1.NodeSelectorTerm) (C.int32_t, C.int32_t) {
	if len(ts) == 0 {
		return 0, 0
	}
	first := p.term(ts[0])
	for _, t := range ts[1:] {
		p.term(t)
	}
	return first, C.int32_t(len(ts))
}

func (p *pool) preferredTerms(ts []v1.PreferredSchedulingTerm) (C.int32_t, C.int32_t) {
	idx := make([]C.int32_t, len(ts))
	for i, t := range ts {
		idx[i] = p.term(t.Preference)
	}
	first := len(p.preferred)
	for i, t := range ts {
		p.preferred = append(p.preferred, C.ksim_k8s_preferred_term{weight: C.int32_t(t.Weight), term: idx[i]})
	}
	return C.int32_t(first), C.int32_t(len(ts))
}

func (p *pool) selector(s *metav1.LabelSelector) C.int32_t {
	if s == nil {
		return -1
	}
	lf, lc := p.kvMap(s.MatchLabels)
	ef := len(p.reqs)
	for _, r := range s.MatchExpressions {
		vf, vc := p.strs(r.Values)
		p.reqs = append(p.reqs, C.ksim_k8s_requirement{key: p.s(r.Key), op: p.s(string(r.Operator)),
			values_first: vf, values_count: vc})
	}
	p.selectors = append(p.selectors, C.ksim_k8s_label_selector{labels_first: lf, labels_count: lc,
		exprs_first: C.int32_t(ef), exprs_count: C.int32_t(len(s.MatchExpressions))})
	return C.int32_t(len(p.selectors) - 1)
}

func (p *pool) podTerm(t v1.PodAffinityTerm, weight int32) C.ksim_k8s_pod_term {
	nf, nc := p.strs(t.Namespaces)
	return C.ksim_k8s_pod_term{topology_key: p.s(t.TopologyKey), selector: p.selector(t.LabelSelector),
		ns_first: nf, ns_count: nc, ns_selector: p.selector(t.NamespaceSelector), weight: C.int32_t(weight)}
}

func (p *pool) podTerms(ts []v1.PodAffinityTerm) (C.int32_t, C.int32_t) {
	built := make([]C.ksim_k8s_pod_term, len(ts))
	for i, t := range ts {
		built[i] = p.podTerm(t, 0)
	}
	first := len(p.podTerms)
	p.podTerms = append(p.podTerms, built...)
	return C.int32_t(first), C.int32_t(len(ts))
}

func (p *pool) weightedTerms(ts []v1.WeightedPodAffinityTerm) (C.int32_t, C.int32_t) {
	built := make([]C.ksim_k8s_pod_term, len(ts))
	for i, t := range ts {
		built[i] = p.podTerm(t.PodAffinityTerm, t.Weight)
	}
	first := len(p.podTerms)
	p.podTerms = append(p.podTerms, built...)
	return C.int32_t(first), C.int32_t(len(ts))
}

func (p *pool) spreads(cs []v1.TopologySpreadConstraint) (C.int32_t, C.int32_t) {
	built := make([]C.ksim_k8s_spread, len(cs))
	for i, c := range cs {
		na, nt := C.int32_t(-1), C.int32_t(-1)
		if c.NodeAffinityPolicy != nil {
			na = p.s(string(*c.NodeAffinityPolicy))
		}
		if c.NodeTaintsPolicy != nil {
			nt = p.s(string(*c.NodeTaintsPolicy))
		}
		built[i] = C.ksim_k8s_spread{max_skew: C.int32_t(c.MaxSkew), topology_key: p.s(c.TopologyKey),
			when_unsatisfiable: p.s(string(c.WhenUnsatisfiable)), selector: p.selector(c.LabelSelector),
			node_affinity_policy: na, node_taints_policy: nt}
	}
	first := len(p.spread)
	p.spread = append(p.spread, built...)
	return C.int32_t(first), C.int32_t(len(cs))
}

func (p *pool) containerList(cs []v1.Container) (C.int32_t, C.int32_t) {
	built := make([]C.ksim_k8s_container, len(cs))
	for i, c := range cs {
		rf, rc := p.resources(c.Resources.Requests)
		pf := len(p.ports)
		for _, port := range c.Ports {
			p.ports = append(p.ports, C.ksim_k8s_port{host_port: C.int32_t(port.HostPort),
				protocol: p.s(string(port.Protocol)), host_ip: p.s(port.HostIP)})
		}
		built[i] = C.ksim_k8s_container{requests_first: rf, requests_count: rc, ports_first: C.int32_t(pf),
			ports_count: C.int32_t(len(c.Ports)), image: p.s(c.Image)}
	}
	first := len(p.containers)
	p.containers = append(p.containers, built...)
	return C.int32_t(first), C.int32_t(len(cs))
}

func (p *pool) node(n *v1.Node) {
	lf, lc := p.kvMap(n.Labels)
	tf := len(p.taints)
	for _, t := range n.Spec.Taints {
		p.taints = append(p.taints, C.ksim_k8s_taint{key: p.s(t.Key), value: p.s(t.Value), effect: p.s(string(t.Effect))})
	}
	af, ac := p.resources(n.Status.Allocatable)
	nf, nc := p.kvMap(n.Annotations)
	imf := len(p.images)
	for _, im := range n.Status.Images {
		f, c := p.strs(im.Names)
		p.images = append(p.images, C.ksim_k8s_image{names_first: f, names_count: c, size_bytes: C.int64_t(im.SizeBytes)})
	}
	unsched := C.int32_t(0)
	if n.Spec.Unschedulable {
		unsched = 1
	}
	p.nodes = append(p.nodes, C.ksim_k8s_node{name: p.s(n.Name), unschedulable: unsched, labels_first: lf,
		labels_count: lc, taints_first: C.int32_t(tf), taints_count: C.int32_t(len(n.Spec.Taints)),
		alloc_first: af, alloc_count: ac, annotations_first: nf, annotations_count: nc,
		images_first: C.int32_t(imf), images_count: C.int32_t(len(n.Status.Images))})
}

// volume sources the engine does not model (ksim/model.py _VOLUME_SOURCES):
// the pod is refused (KSIM_POD_HAS_VOLUMES) and the original plugins answer
func refusedVolumes(pod *v1.Pod) bool {
	for _, v := range pod.Spec.Volumes {
		s := v.VolumeSource
		if s.PersistentVolumeClaim != nil || s.GCEPersistentDisk != nil || s.AWSElasticBlockStore != nil ||
			s.AzureDisk != nil || s.CSI != nil || s.RBD != nil || s.ISCSI != nil || s.Cinder != nil || s.Ephemeral != nil {
			return true
		}
	}
	return false
}

func (p *pool) pod(pod *v1.Pod) {
	spec := &pod.Spec
	rec := C.ksim_k8s_pod{name: p.s(pod.Name), namespace_: p.s(pod.Namespace), node_name: p.s(spec.NodeName),
		owner_api_version: -1, owner_kind: -1, owner_name: -1, required_first: -1}
	rec.labels_first, rec.labels_count = p.kvMap(pod.Labels)
	rec.annotations_first, rec.annotations_count = p.kvMap(pod.Annotations)
	rec.containers_first, rec.containers_count = p.containerList(spec.Containers)
	rec.init_first, rec.init_count = p.containerList(spec.InitContainers)
	rec.overhead_first, rec.overhead_count = p.resources(spec.Overhead)
	rec.selector_first, rec.selector_count = p.kvMap(spec.NodeSelector)
	if a := spec.Affinity; a != nil {
		if na := a.NodeAffinity; na != nil {
			if req := na.RequiredDuringSchedulingIgnoredDuringExecution; req != nil {
				rec.required_first, rec.required_count = p.termList(req.NodeSelectorTerms)
			}
			rec.preferred_first, rec.preferred_count = p.preferredTerms(na.PreferredDuringSchedulingIgnoredDuringExecution)
		}
		if pa := a.PodAffinity; pa != nil {
			rec.aff_req_first, rec.aff_req_count = p.podTerms(pa.RequiredDuringSchedulingIgnoredDuringExecution)
			rec.aff_pref_first, rec.aff_pref_count = p.weightedTerms(pa.PreferredDuringSchedulingIgnoredDuringExecution)
		}
		if paa := a.PodAntiAffinity; paa != nil {
			rec.anti_req_first, rec.anti_req_count = p.podTerms(paa.RequiredDuringSchedulingIgnoredDuringExecution)
			rec.anti_pref_first, rec.anti_pref_count = p.weightedTerms(paa.PreferredDuringSchedulingIgnoredDuringExecution)
		}
	}
	tf := len(p.tols)
	for _, t := range spec.Tolerations {
		p.tols = append(p.tols, C.ksim_k8s_toleration{key: p.s(t.Key), op: p.s(string(t.Operator)),
			value: p.s(t.Value), effect: p.s(string(t.Effect))})
	}
	rec.tolerations_first, rec.tolerations_count = C.int32_t(tf), C.int32_t(len(spec.Tolerations))
	rec.spread_first, rec.spread_count = p.spreads(spec.TopologySpreadConstraints)
	if ref := metav1.GetControllerOf(pod); ref != nil {
		rec.owner_api_version, rec.owner_kind, rec.owner_name = p.s(ref.APIVersion), p.s(ref.Kind), p.s(ref.Name)
	}
	rec.volumes = C.KSIM_K8S_VOLUMES_NONE
	if refusedVolumes(pod) {
		rec.volumes = C.KSIM_K8S_VOLUMES_REFUSE
	}
	p.pods = append(p.pods, rec)
}

// build copies the pool into one C allocation: the ksim_k8s_pool struct and
// every array it points to.  free releases it.
func (p *pool) build() (cp *C.ksim_k8s_pool, free func()) {
	type part struct {
		src unsafe.Pointer
		n   uintptr
	}
	sz := func(n int, one uintptr) uintptr { return uintptr(n) * one }
	ptr := func(n int, first unsafe.Pointer) unsafe.Pointer {
		if n == 0 {
			return nil
		}
		return first
	}
	first := func(b []byte) unsafe.Pointer {
		if len(b) == 0 {
			return nil
		}
		return unsafe.Pointer(&b[0])
	}
	var z C.ksim_k8s_pool
	parts := []part{
		{ptr(len(p.blob), first(p.blob)), uintptr(len(p.blob))},
		{unsafe.Pointer(&p.off[0]), sz(len(p.off), 8)},
	}
	add := func(n int, base unsafe.Pointer, one uintptr) { parts = append(parts, part{ptr(n, base), sz(n, one)}) }
	add(len(p.strList), unsafe.Pointer(unsafe.SliceData(p.strList)), 4)
	add(len(p.kv), unsafe.Pointer(unsafe.SliceData(p.kv)), unsafe.Sizeof(C.ksim_k8s_kv{}))
	add(len(p.taints), unsafe.Pointer(unsafe.SliceData(p.taints)), unsafe.Sizeof(C.ksim_k8s_taint{}))
	add(len(p.tols), unsafe.Pointer(unsafe.SliceData(p.tols)), unsafe.Sizeof(C.ksim_k8s_toleration{}))
	add(len(p.reqs), unsafe.Pointer(unsafe.SliceData(p.reqs)), unsafe.Sizeof(C.ksim_k8s_requirement{}))
	add(len(p.terms), unsafe.Pointer(unsafe.SliceData(p.terms)), unsafe.Sizeof(C.ksim_k8s_selector_term{}))
	add(len(p.preferred), unsafe.Pointer(unsafe.SliceData(p.preferred)), unsafe.Sizeof(C.ksim_k8s_preferred_term{}))
	add(len(p.selectors), unsafe.Pointer(unsafe.SliceData(p.selectors)), unsafe.Sizeof(C.ksim_k8s_label_selector{}))
	add(len(p.podTerms), unsafe.Pointer(unsafe.SliceData(p.podTerms)), unsafe.Sizeof(C.ksim_k8s_pod_term{}))
	add(len(p.spread), unsafe.Pointer(unsafe.SliceData(p.spread)), unsafe.Sizeof(C.ksim_k8s_spread{}))
	add(len(p.ports), unsafe.Pointer(unsafe.SliceData(p.ports)), unsafe.Sizeof(C.ksim_k8s_port{}))
	add(len(p.containers), unsafe.Pointer(unsafe.SliceData(p.containers)), unsafe.Sizeof(C.ksim_k8s_container{}))
	add(len(p.images), unsafe.Pointer(unsafe.SliceData(p.images)), unsafe.Sizeof(C.ksim_k8s_image{}))
	add(len(p.groups), unsafe.Pointer(unsafe.SliceData(p.groups)), unsafe.Sizeof(C.ksim_k8s_volume_group{}))
	add(len(p.nodes), unsafe.Pointer(unsafe.SliceData(p.nodes)), unsafe.Sizeof(C.ksim_k8s_node{}))
	add(len(p.pods), unsafe.Pointer(unsafe.SliceData(p.pods)), unsafe.Sizeof(C.ksim_k8s_pod{}))
	add(len(p.namespaces), unsafe.Pointer(unsafe.SliceData(p.namespaces)), unsafe.Sizeof(C.ksim_k8s_namespace{}))
	add(len(p.services), unsafe.Pointer(unsafe.SliceData(p.services)), unsafe.Sizeof(C.ksim_k8s_service{}))
	add(len(p.controllers), unsafe.Pointer(unsafe.SliceData(p.controllers)), unsafe.Sizeof(C.ksim_k8s_controller{}))
	total := unsafe.Sizeof(z)
	for _, x := range parts {
		total += (x.n + 15) &^ 15
	}
	base := C.malloc(C.size_t(total))
	addr := make([]unsafe.Pointer, len(parts))
	at := unsafe.Sizeof(z)
	for i, x := range parts {
		addr[i] = unsafe.Add(base, at)
		if x.n > 0 {
			C.memcpy(addr[i], x.src, C.size_t(x.n))
		}
		at += (x.n + 15) &^ 15
	}
	cp = (*C.ksim_k8s_pool)(base)
	*cp = C.ksim_k8s_pool{}
	cp.strings = (*C.char)(addr[0])
	cp.str_off = (*C.int64_t)(addr[1])
	cp.n_strings = C.int64_t(len(p.off) - 1)
	cp.str_list, cp.n_str_list = (*C.int32_t)(addr[2]), C.int64_t(len(p.strList))
	cp.kv, cp.n_kv = (*C.ksim_k8s_kv)(addr[3]), C.int64_t(len(p.kv))
	cp.taints, cp.n_taints = (*C.ksim_k8s_taint)(addr[4]), C.int64_t(len(p.taints))
	cp.tolerations, cp.n_tolerations = (*C.ksim_k8s_toleration)(addr[5]), C.int64_t(len(p.tols))
	cp.reqs, cp.n_reqs = (*C.ksim_k8s_requirement)(addr[6]), C.int64_t(len(p.reqs))
	cp.terms, cp.n_terms = (*C.ksim_k8s_selector_term)(addr[7]), C.int64_t(len(p.terms))
	cp.preferred, cp.n_preferred = (*C.ksim_k8s_preferred_term)(addr[8]), C.int64_t(len(p.preferred))
	cp.selectors, cp.n_selectors = (*C.ksim_k8s_label_selector)(addr[9]), C.int64_t(len(p.selectors))
	cp.pod_terms, cp.n_pod_terms = (*C.ksim_k8s_pod_term)(addr[10]), C.int64_t(len(p.podTerms))
	cp.spread, cp.n_spread = (*C.ksim_k8s_spread)(addr[11]), C.int64_t(len(p.spread))
	cp.ports, cp.n_ports = (*C.ksim_k8s_port)(addr[12]), C.int64_t(len(p.ports))
	cp.containers, cp.n_containers = (*C.ksim_k8s_container)(addr[13]), C.int64_t(len(p.containers))
	cp.images, cp.n_images = (*C.ksim_k8s_image)(addr[14]), C.int64_t(len(p.images))
	cp.volume_groups, cp.n_volume_groups = (*C.ksim_k8s_volume_group)(addr[15]), C.int64_t(len(p.groups))
	cp.nodes, cp.n_nodes = (*C.ksim_k8s_node)(addr[16]), C.int64_t(len(p.nodes))
	cp.pods, cp.n_pods = (*C.ksim_k8s_pod)(addr[17]), C.int64_t(len(p.pods))
	cp.namespaces, cp.n_namespaces = (*C.ksim_k8s_namespace)(addr[18]), C.int64_t(len(p.namespaces))
	cp.services, cp.n_services = (*C.ksim_k8s_service)(addr[19]), C.int64_t(len(p.services))
	cp.controllers, cp.n_controllers = (*C.ksim_k8s_controller)(addr[20]), C.int64_t(len(p.controllers))
	return cp, func() { C.free(base) }
}

// copyPodSet deep-copies a ksim_pod_set into one C allocation the caller owns.
func copyPodSet(ps *C.ksim_pod_set) (*C.ksim_pod_set, func()) {
	sizes := []uintptr{
		uintptr(ps.n_pods) * unsafe.Sizeof(C.ksim_pod{}), uintptr(ps.n_exprs) * unsafe.Sizeof(C.ksim_label_expr{}),
		uintptr(ps.n_terms) * unsafe.Sizeof(C.ksim_term{}), uintptr(ps.n_uses) * unsafe.Sizeof(C.ksim_topo_use{}),
		uintptr(ps.n_adds) * unsafe.Sizeof(C.ksim_class_add{}), uintptr(ps.n_nn) * 4}
	srcs := []unsafe.Pointer{unsafe.Pointer(ps.pods), unsafe.Pointer(ps.exprs), unsafe.Pointer(ps.terms),
		unsafe.Pointer(ps.uses), unsafe.Pointer(ps.adds), unsafe.Pointer(ps.nn)}
	total := unsafe.Sizeof(C.ksim_pod_set{})
	for _, n := range sizes {
		total += (n + 15) &^ 15
	}
	base := C.malloc(C.size_t(total))
	out := (*C.ksim_pod_set)(base)
	*out = *ps
	at := unsafe.Sizeof(C.ksim_pod_set{})
	dst := make([]unsafe.Pointer, len(sizes))
	for i, n := range sizes {
		dst[i] = nil
		if n > 0 {
			dst[i] = unsafe.Add(base, at)
			C.memcpy(dst[i], srcs[i], C.size_t(n))
		}
		at += (n + 15) &^ 15
	}
	out.pods = (*C.ksim_pod)(dst[0])
	out.exprs = (*C.ksim_label_expr)(dst[1])
	out.terms = (*C.ksim_term)(dst[2])
	out.uses = (*C.ksim_topo_use)(dst[3])
	out.adds = (*C.ksim_class_add)(dst[4])
	out.nn = (*C.int32_t)(dst[5])
	return out, func() { C.free(base) }
}

// ---- the Encoder ------------------------------------------------------------------

// NativeEncoder implements Encoder (plugins.go) over ksim_encode_nodes /
// ksim_encode_pods and the encoder's snapshot deltas (ABI 11).  The host sets
// the profile's plugin args before the first cycle (NewPluginConfig's merged
// args, plugins.go:103-179) and registers Handlers() on the pod and node
// informers (plugins.go Register does both).
//
// The snapshot is encoded whole once, at the first cycle.  From then on the
// informers' events queue here and the next cycle start applies them
// (Snapshot), as the scheduler cache applies them before UpdateSnapshot
// (simulator/scheduler/scheduler.go:160-167 runs the scheduler off informers):
//
//	node added / updated / removed  ksim_encoder_update_nodes, then
//	                                ksim_upsert_nodes (one per cycle start;
//	                                the engine replays its binds on kept nodes)
//	bound pod added                 ksim_encode_pods, the table re-sent if the
//	                                compile grew it, ksim_assume, ksim_encoder_bind
//	bound pod deleted               ksim_encode_pods, ksim_forget, ksim_encoder_unbind
//	Reserve / Unreserve             Assume / Forget: the same, for the cycle's pod
//
// A pod the engine assumed and the informer then reports bound on the same
// node is already in the snapshot (a no-op).  A full re-encode (of the host's
// record of nodes and bound pods, ksim_set_cluster) happens again only when a
// delta cannot be encoded (a vocabulary or class limit): Stats.FullEncodes.
type NativeEncoder struct {
	// NetworkBandwidthArgs annotation names ("" = the plugin's defaults)
	NodeLimitAnnotation, IngressRequestAnnotation, EgressRequestAnnotation string
	// NodeAffinityArgs.addedAffinity (nil: none)
	AddedAffinity *v1.NodeAffinity
	// PodTopologySpreadArgs.defaultingType: "" or "System" (upstream's default,
	// SetDefaults_PodTopologySpreadArgs), "List" (with DefaultConstraints), or
	// "None" (no default constraints at all: an explicit opt-out)
	SpreadDefaulting   string
	DefaultConstraints []v1.TopologySpreadConstraint
	// Namespaces (namespaceSelector terms), Services and controllers
	// (helper.DefaultSelector) the host's listers return
	Namespaces      func() []*v1.Namespace
	Services        func() []*v1.Service
	ReplicaSets     func() []metav1.Object
	ControllerOf    func(obj metav1.Object) (kind string, rcSelector map[string]string, selector *metav1.LabelSelector)

	Stats struct{ FullEncodes, NodeDeltas, PodAdds, PodDeletes, Resends int }

	mu       sync.Mutex
	enc      *C.ksim_encoder
	encoded  bool
	names    []string
	pos      map[string]int
	podCopy  func() // Pod's set (C memory), freed by the next Pod call
	layout   [2]int32

	// the host's record of the snapshot: nodes in informer add order, bound
	// pods by namespace/name (with their node) in bind order
	nodes     map[string]*v1.Node
	nodeOrder []string
	bound     map[string]boundPod
	waiting   map[string]*v1.Pod // bound to a node the snapshot does not hold yet
	boundRows []*v1.Pod          // the bound-pod table rows (DefaultPreemption)
	boundBufs func()
	tableOld  bool

	evMu   sync.Mutex
	events []event
}

type boundPod struct {
	pod  *v1.Pod
	node string
	seq  uint64 // bind order
}

type eventKind int

const (
	evNode eventKind = iota
	evNodeGone
	evPod
	evPodGone
)

type event struct {
	kind eventKind
	node *v1.Node
	name string
	pod  *v1.Pod
}

func podKey(p *v1.Pod) string { return p.Namespace + "/" + p.Name }

func (n *NativeEncoder) queue(ev ...event) {
	n.evMu.Lock()
	n.events = append(n.events, ev...)
	n.evMu.Unlock()
}

// Handlers are the informer event handlers (pods, nodes) that feed the deltas.
func (n *NativeEncoder) Handlers() (pods, nodes cache.ResourceEventHandlerFuncs) {
	asPod := func(obj interface{}) *v1.Pod {
		switch t := obj.(type) {
		case *v1.Pod:
			return t
		case cache.DeletedFinalStateUnknown:
			p, _ := t.Obj.(*v1.Pod)
			return p
		}
		return nil
	}
	asNode := func(obj interface{}) *v1.Node {
		switch t := obj.(type) {
		case *v1.Node:
			return t
		case cache.DeletedFinalStateUnknown:
			nd, _ := t.Obj.(*v1.Node)
			return nd
		}
		return nil
	}
	pods = cache.ResourceEventHandlerFuncs{
		AddFunc: func(obj interface{}) {
			if p := asPod(obj); p != nil && p.Spec.NodeName != "" {
				n.queue(event{kind: evPod, pod: p})
			}
		},
		UpdateFunc: func(oldObj, newObj interface{}) {
			o, p := asPod(oldObj), asPod(newObj)
			if o == nil || p == nil {
				return
			}
			if o.Spec.NodeName != "" && o.Spec.NodeName == p.Spec.NodeName && samePlacementInputs(o, p) {
				return // status / metadata churn the plugins do not read
			}
			if o.Spec.NodeName != "" {
				n.queue(event{kind: evPodGone, pod: o})
			}
			if p.Spec.NodeName != "" {
				n.queue(event{kind: evPod, pod: p})
			}
		},
		DeleteFunc: func(obj interface{}) {
			if p := asPod(obj); p != nil {
				n.queue(event{kind: evPodGone, pod: p})
			}
		},
	}
	nodes = cache.ResourceEventHandlerFuncs{
		AddFunc: func(obj interface{}) {
			if nd := asNode(obj); nd != nil {
				n.queue(event{kind: evNode, node: nd})
			}
		},
		UpdateFunc: func(_, newObj interface{}) {
			if nd := asNode(newObj); nd != nil {
				n.queue(event{kind: evNode, node: nd})
			}
		},
		DeleteFunc: func(obj interface{}) {
			if nd := asNode(obj); nd != nil {
				n.queue(event{kind: evNodeGone, name: nd.Name})
			}
		},
	}
	return pods, nodes
}

// samePlacementInputs: what the encoder reads of a bound pod (labels, the
// NetworkBandwidth annotations, the spec) did not change.
func samePlacementInputs(a, b *v1.Pod) bool {
	return equality.Semantic.DeepEqual(a.Labels, b.Labels) && equality.Semantic.DeepEqual(a.Annotations, b.Annotations) &&
		equality.Semantic.DeepEqual(a.Spec, b.Spec)
}

func (n *NativeEncoder) ensure() error {
	if n.enc != nil {
		return nil
	}
	var e *C.ksim_encoder
	if rc := C.ksim_encoder_create(&e); rc != C.KSIM_OK {
		return fmt.Errorf("ksim_encoder_create: %d", int(rc))
	}
	n.enc = e
	return nil
}

// encodeError marks a delta the encoder refused (a limit): the record is re-encoded whole.
type encodeError struct{ err error }

func (x *encodeError) Error() string { return x.err.Error() }

func (n *NativeEncoder) errOf(rc C.int) error {
	if rc == C.KSIM_OK {
		return nil
	}
	return &encodeError{fmt.Errorf("ksim encoder %d: %s", int(rc), C.GoString(C.ksim_encoder_last_error(n.enc)))}
}

func (n *NativeEncoder) info() C.ksim_encoder_info {
	var in C.ksim_encoder_info
	C.ksim_encoder_get_info(n.enc, &in)
	return in
}

// Snapshot brings the device snapshot up to the cluster at a cycle start: the
// whole snapshot at the first cycle, the queued informer events afterwards.
func (n *NativeEncoder) Snapshot(e *Engine, f framework.Handle) error {
	n.mu.Lock()
	defer n.mu.Unlock()
	if err := n.ensure(); err != nil {
		return err
	}
	n.evMu.Lock()
	ev := n.events
	n.events = nil
	n.evMu.Unlock()
	if !n.encoded {
		// the framework's snapshot is the record; events queued before it are
		// in it already (an add of a pod the record holds is a no-op)
		infos, err := f.SnapshotSharedLister().NodeInfos().List()
		if err != nil {
			return err
		}
		n.nodes, n.bound, n.waiting = map[string]*v1.Node{}, map[string]boundPod{}, map[string]*v1.Pod{}
		n.nodeOrder = nil
		var seq uint64
		for _, ni := range infos {
			if ni.Node() == nil {
				continue
			}
			n.nodes[ni.Node().Name] = ni.Node()
			n.nodeOrder = append(n.nodeOrder, ni.Node().Name)
			for _, pi := range ni.Pods {
				seq++
				n.bound[podKey(pi.Pod)] = boundPod{pi.Pod, ni.Node().Name, seq}
			}
		}
		return n.encodeRecord(e)
	}
	if err := n.apply(e, ev); err != nil {
		var ee *encodeError
		if errors.As(err, &ee) {
			return n.encodeRecord(e)
		}
		return err
	}
	return nil
}

// encodeRecord: the whole record, one ksim_encode_nodes and ksim_set_cluster.
func (n *NativeEncoder) encodeRecord(e *Engine) error {
	p := newPool()
	for _, name := range n.nodeOrder {
		p.node(n.nodes[name])
	}
	for _, b := range n.sortedBound() {
		q := b.pod
		if q.Spec.NodeName != b.node {
			q = q.DeepCopy() // assumed by the engine: the framework's node
			q.Spec.NodeName = b.node
		}
		p.pod(q)
	}
	if n.Namespaces != nil {
		for _, ns := range n.Namespaces() {
			lf, lc := p.kvMap(ns.Labels)
			p.namespaces = append(p.namespaces, C.ksim_k8s_namespace{name: p.s(ns.Name), labels_first: lf, labels_count: lc})
		}
	}
	opts := C.ksim_encode_nodes_opts{nb_node_limit: -1, nb_ingress_request: -1, nb_egress_request: -1}
	if n.NodeLimitAnnotation != "" {
		opts.nb_node_limit = p.s(n.NodeLimitAnnotation)
	}
	if n.IngressRequestAnnotation != "" {
		opts.nb_ingress_request = p.s(n.IngressRequestAnnotation)
	}
	if n.EgressRequestAnnotation != "" {
		opts.nb_egress_request = p.s(n.EgressRequestAnnotation)
	}
	if n.encoded {
		opts.keep_previous = 1 // class ids of pods encoded earlier stay valid
	}
	cp, free := p.build()
	defer free()
	if err := n.errOf(C.ksim_encode_nodes(n.enc, cp, &opts)); err != nil {
		return err
	}
	n.readNames()
	n.encoded = true
	n.Stats.FullEncodes++
	var t C.ksim_node_table
	var v C.ksim_vocab
	if err := n.errOf(C.ksim_encoder_cluster(n.enc, &t, &v)); err != nil {
		return err
	}
	ns, _ := e.NextStart()
	if err := e.SetCluster(&t, &v); err != nil {
		return err
	}
	if len(n.names) > 0 {
		_ = e.locked(func() C.int { return C.ksim_set_next_start(e.h, C.int32_t(ns%len(n.names))) })
	}
	n.noteLayout()
	n.tableOld = true
	return nil
}

func (n *NativeEncoder) sortedBound() []boundPod {
	out := make([]boundPod, 0, len(n.bound))
	for _, b := range n.bound {
		out = append(out, b)
	}
	sort.Slice(out, func(i, j int) bool { return out[i].seq < out[j].seq })
	return out
}

func (n *NativeEncoder) readNames() {
	in := n.info()
	names := make([]string, int(in.n_nodes))
	pos := make(map[string]int, len(names))
	for i := range names {
		names[i] = C.GoString(C.ksim_encoder_string(n.enc, C.KSIM_ENC_STR_NODE_NAME, C.int32_t(i), 0))
		pos[names[i]] = i
	}
	n.names, n.pos = names, pos
}

func (n *NativeEncoder) noteLayout() {
	in := n.info()
	n.layout = [2]int32{int32(in.n_label_cols), int32(in.n_classes)}
}

// apply: the node events in one update, then the pod events in order.
func (n *NativeEncoder) apply(e *Engine, ev []event) error {
	var upd []*v1.Node
	var gone []string
	seen := map[string]int{}
	for _, x := range ev {
		switch x.kind {
		case evNode:
			if i, ok := seen[x.node.Name]; ok {
				upd[i] = x.node
			} else {
				seen[x.node.Name] = len(upd)
				upd = append(upd, x.node)
			}
		case evNodeGone:
			if i, ok := seen[x.name]; ok {
				upd = append(upd[:i], upd[i+1:]...)
				delete(seen, x.name)
				for k, j := range seen {
					if j > i {
						seen[k] = j - 1
					}
				}
			}
			if _, ok := n.nodes[x.name]; ok {
				gone = append(gone, x.name)
			}
		}
	}
	if len(upd) > 0 || len(gone) > 0 {
		if err := n.applyNodes(e, upd, gone); err != nil {
			return err
		}
	}
	for _, x := range ev {
		var err error
		switch x.kind {
		case evPod:
			err = n.podAdded(e, x.pod)
		case evPodGone:
			err = n.podDeleted(e, x.pod)
		}
		if err != nil {
			return err
		}
	}
	for key, p := range n.waiting {
		if _, ok := n.pos[p.Spec.NodeName]; ok {
			delete(n.waiting, key)
			if err := n.podAdded(e, p); err != nil {
				return err
			}
		}
	}
	return nil
}

func (n *NativeEncoder) applyNodes(e *Engine, upd []*v1.Node, gone []string) error {
	// the record first (nodeTree.updateNode re-adds a node whose zone moved)
	for _, name := range gone {
		delete(n.nodes, name)
		for key, b := range n.bound {
			if b.node == name {
				delete(n.bound, key)
			}
		}
	}
	order := n.nodeOrder[:0:0]
	for _, name := range n.nodeOrder {
		if _, ok := n.nodes[name]; ok {
			order = append(order, name)
		}
	}
	for _, nd := range upd {
		if old, ok := n.nodes[nd.Name]; ok && zoneKey(old) != zoneKey(nd) {
			for i, x := range order {
				if x == nd.Name {
					order = append(order[:i], order[i+1:]...)
					break
				}
			}
			order = append(order, nd.Name)
		} else if !ok {
			order = append(order, nd.Name)
		}
		n.nodes[nd.Name] = nd
	}
	n.nodeOrder = order
	p := newPool()
	for _, nd := range upd {
		p.node(nd)
	}
	removed := make([]C.int32_t, len(gone)+1)
	for i, name := range gone {
		removed[i] = p.s(name)
	}
	cp, free := p.build()
	defer free()
	if err := n.errOf(C.ksim_encoder_update_nodes(n.enc, cp, &removed[0], C.int32_t(len(gone)))); err != nil {
		return err
	}
	n.readNames()
	var t C.ksim_node_table
	var v C.ksim_vocab
	if err := n.errOf(C.ksim_encoder_cluster(n.enc, &t, &v)); err != nil {
		return err
	}
	n.Stats.NodeDeltas++
	// in place (no node moved, no new vocabulary): the updated rows only
	rows := make([]int32, len(upd)+1)
	if k := int(C.ksim_encoder_changed_rows(n.enc, (*C.int32_t)(unsafe.Pointer(&rows[0])), C.int32_t(len(rows)))); k >= 0 {
		return e.UpdateNodeRows(&t, &v, rows[:k])
	}
	oldPos := make([]int32, len(n.names)+1)
	if err := n.errOf(C.ksim_encoder_old_pos(n.enc, (*C.int32_t)(unsafe.Pointer(&oldPos[0])))); err != nil {
		return err
	}
	if err := e.UpsertNodes(&t, &v, oldPos[:len(n.names)]); err != nil {
		return err
	}
	n.noteLayout()
	n.tableOld = true // the engine dropped the bound-pod table (positions moved)
	return nil
}

// zoneKey: utilnode.GetZoneKey (region and zone labels, GA then beta)
func zoneKey(nd *v1.Node) string {
	l := nd.Labels
	zone, region := l[v1.LabelTopologyZone], l[v1.LabelTopologyRegion]
	if zone == "" {
		zone = l[v1.LabelFailureDomainBetaZone]
	}
	if region == "" {
		region = l[v1.LabelFailureDomainBetaRegion]
	}
	if zone == "" && region == "" {
		return ""
	}
	return region + ":\x00:" + zone
}

// resend: the compile added label columns or count classes; the table again
// with every node kept (ksim_upsert_nodes replays the device's binds), before
// any bind the new rows do not count.
func (n *NativeEncoder) resend(e *Engine) error {
	in := n.info()
	if int32(in.n_label_cols) == n.layout[0] && int32(in.n_classes) == n.layout[1] {
		return nil
	}
	var t C.ksim_node_table
	var v C.ksim_vocab
	if err := n.errOf(C.ksim_encoder_cluster(n.enc, &t, &v)); err != nil {
		return err
	}
	keep := make([]int32, len(n.names)+1)
	for i := range n.names {
		keep[i] = int32(i)
	}
	if err := e.UpsertNodes(&t, &v, keep[:len(n.names)]); err != nil {
		return err
	}
	n.noteLayout()
	n.tableOld = true
	n.Stats.Resends++
	return nil
}

// podAdded: a bound pod enters the snapshot (informer Add / Update).
func (n *NativeEncoder) podAdded(e *Engine, p *v1.Pod) error {
	key := podKey(p)
	if b, ok := n.bound[key]; ok {
		if b.node == p.Spec.NodeName {
			return nil // assumed by the engine's Reserve already
		}
		if err := n.podDeleted(e, b.pod); err != nil {
			return err
		}
	}
	pos, ok := n.pos[p.Spec.NodeName]
	if !ok {
		n.waiting[key] = p
		return nil
	}
	if err := n.encodeQueue([]*v1.Pod{p}); err != nil {
		return err
	}
	if err := n.resend(e); err != nil {
		return err
	}
	if err := e.Assume(n.encodedSet(), 0, pos); err != nil {
		return err
	}
	if err := n.errOf(C.ksim_encoder_bind(n.enc, 0, C.int32_t(pos))); err != nil {
		return err
	}
	n.bind(key, p, p.Spec.NodeName)
	n.Stats.PodAdds++
	return nil
}

func (n *NativeEncoder) bind(key string, p *v1.Pod, node string) {
	var seq uint64
	for _, b := range n.bound {
		if b.seq > seq {
			seq = b.seq
		}
	}
	n.bound[key] = boundPod{p, node, seq + 1}
	n.tableOld = true
}

// podDeleted: a bound pod leaves the snapshot (informer Delete, Unreserve).
// The pod is compiled again as it was bound: its adds include the classes
// registered since its bind, which count it.
func (n *NativeEncoder) podDeleted(e *Engine, p *v1.Pod) error {
	key := podKey(p)
	delete(n.waiting, key)
	b, ok := n.bound[key]
	if !ok {
		return nil
	}
	if err := n.encodeQueue([]*v1.Pod{b.pod}); err != nil {
		return err
	}
	if err := n.resend(e); err != nil {
		return err
	}
	ns, name := C.CString(b.pod.Namespace), C.CString(b.pod.Name)
	defer C.free(unsafe.Pointer(ns))
	defer C.free(unsafe.Pointer(name))
	var pos C.int32_t
	if err := n.errOf(C.ksim_encoder_unbind(n.enc, ns, name, &pos)); err != nil {
		return err
	}
	if err := e.Forget(n.encodedSet(), 0, int(pos)); err != nil {
		return err
	}
	delete(n.bound, key)
	n.tableOld = true
	n.Stats.PodDeletes++
	return nil
}

// Assume is KsimAssume.Reserve: the cycle's pod on the framework's node, on
// the device and in the snapshot's membership.
func (n *NativeEncoder) Assume(e *Engine, pod *v1.Pod, node int) error {
	n.mu.Lock()
	defer n.mu.Unlock()
	if err := n.encodeQueue([]*v1.Pod{pod}); err != nil {
		return err
	}
	if err := n.resend(e); err != nil {
		return err
	}
	if err := e.Assume(n.encodedSet(), 0, node); err != nil {
		return err
	}
	if err := n.errOf(C.ksim_encoder_bind(n.enc, 0, C.int32_t(node))); err != nil {
		return err
	}
	n.bind(podKey(pod), pod, n.names[node])
	return nil
}

// Forget is KsimAssume.Unreserve (possibly on the binding goroutine while the
// next cycle runs: the engine queues it behind that cycle's PreFilter).
func (n *NativeEncoder) Forget(e *Engine, pod *v1.Pod) error {
	n.mu.Lock()
	defer n.mu.Unlock()
	return n.podDeleted(e, pod)
}

// BoundTable re-sends DefaultPreemption's bound-pod table when binds, deletes
// or node deltas changed it since the last dry run (ksim_set_bound_pods:
// node, priority, start time, requests as NodeInfo's Requested,
// ksim/preemption.py bound_table).
func (n *NativeEncoder) BoundTable(e *Engine) error {
	n.mu.Lock()
	defer n.mu.Unlock()
	if !n.tableOld {
		return nil
	}
	if n.boundBufs != nil {
		n.boundBufs()
		n.boundBufs = nil
	}
	in := n.info()
	scalars := make([]string, int(in.n_scalar))
	for k := range scalars {
		scalars[k] = C.GoString(C.ksim_encoder_string(n.enc, C.KSIM_ENC_STR_SCALAR, C.int32_t(k), 0))
	}
	n.boundRows = n.boundRows[:0]
	var nodes []int
	for _, b := range n.sortedBound() {
		if q, ok := n.pos[b.node]; ok {
			n.boundRows = append(n.boundRows, b.pod)
			nodes = append(nodes, q)
		}
	}
	rows := len(n.boundRows)
	node := (*[1 << 30]C.int32_t)(C.malloc(C.size_t(4*rows + 4)))[: rows+1 : rows+1]
	prio := (*[1 << 30]C.int32_t)(C.malloc(C.size_t(4*rows + 4)))[: rows+1 : rows+1]
	start := (*[1 << 30]C.int64_t)(C.malloc(C.size_t(8*rows + 8)))[: rows+1 : rows+1]
	req := (*[1 << 30]C.int64_t)(C.malloc(C.size_t(8*rows*C.KSIM_PREEMPT_REQ + 8)))[: rows*C.KSIM_PREEMPT_REQ+1 : rows*C.KSIM_PREEMPT_REQ+1]
	n.boundBufs = func() {
		C.free(unsafe.Pointer(&node[0]))
		C.free(unsafe.Pointer(&prio[0]))
		C.free(unsafe.Pointer(&start[0]))
		C.free(unsafe.Pointer(&req[0]))
	}
	for i, b := range n.boundRows {
		node[i] = C.int32_t(nodes[i])
		if b.Spec.Priority != nil {
			prio[i] = C.int32_t(*b.Spec.Priority)
		} else {
			prio[i] = 0
		}
		start[i] = 0
		if b.Status.StartTime != nil {
			start[i] = C.int64_t(b.Status.StartTime.UnixNano())
		}
		r := podRequests(b)
		row := req[i*C.KSIM_PREEMPT_REQ : (i+1)*C.KSIM_PREEMPT_REQ]
		for k := range row {
			row[k] = 0
		}
		row[0], row[1], row[2] = C.int64_t(r[v1.ResourceCPU]), C.int64_t(r[v1.ResourceMemory]),
			C.int64_t(r[v1.ResourceEphemeralStorage])
		for k, s := range scalars {
			row[3+k] = C.int64_t(r[v1.ResourceName(s)])
		}
	}
	bp := C.ksim_bound_pods{n: C.int32_t(rows), node: &node[0], priority: &prio[0], start_time: &start[0], req: &req[0]}
	if err := e.SetBoundPods(&bp); err != nil {
		return err
	}
	n.tableOld = false
	return nil
}

// podRequests: computePodResourceRequest (sum of containers, max of each init
// container, + overhead), cpu in millicores (ksim/encode.py pod_requests).
func podRequests(p *v1.Pod) map[v1.ResourceName]int64 {
	val := func(name v1.ResourceName, q resource.Quantity) int64 {
		if name == v1.ResourceCPU {
			return q.MilliValue()
		}
		return q.Value()
	}
	out := map[v1.ResourceName]int64{}
	for _, c := range p.Spec.Containers {
		for k, q := range c.Resources.Requests {
			out[k] += val(k, q)
		}
	}
	for _, c := range p.Spec.InitContainers {
		for k, q := range c.Resources.Requests {
			if v := val(k, q); v > out[k] {
				out[k] = v
			}
		}
	}
	for k, q := range p.Spec.Overhead {
		out[k] += val(k, q)
	}
	return out
}

// encodeQueue compiles pods against the snapshot (the profile's args).
func (n *NativeEncoder) encodeQueue(pods []*v1.Pod) error {
	p := newPool()
	for _, pod := range pods {
		p.pod(pod)
	}
	opts := C.ksim_encode_pods_opts{added_required_first: -1}
	if a := n.AddedAffinity; a != nil {
		if req := a.RequiredDuringSchedulingIgnoredDuringExecution; req != nil {
			opts.added_required_first, opts.added_required_count = p.termList(req.NodeSelectorTerms)
		}
		opts.added_preferred_first, opts.added_preferred_count = p.preferredTerms(a.PreferredDuringSchedulingIgnoredDuringExecution)
	}
	switch n.SpreadDefaulting {
	case "", "System": // PodTopologySpreadArgs.defaultingType defaults to System
		opts.spread_defaults = C.KSIM_SPREAD_DEFAULTS_SYSTEM
	case "List":
		if len(n.DefaultConstraints) > 0 {
			opts.spread_defaults = C.KSIM_SPREAD_DEFAULTS_LIST
			opts.spread_first, opts.spread_count = p.spreads(n.DefaultConstraints)
		}
	case "None":
	default:
		return fmt.Errorf("ksim: PodTopologySpread defaultingType %q not supported", n.SpreadDefaulting)
	}
	if opts.spread_defaults != C.KSIM_SPREAD_DEFAULTS_NONE {
		if n.Services != nil {
			for _, s := range n.Services() {
				rec := C.ksim_k8s_service{namespace_: p.s(s.Namespace), selector_first: -1}
				if s.Spec.Selector != nil {
					rec.selector_first, rec.selector_count = p.kvMap(s.Spec.Selector)
				}
				p.services = append(p.services, rec)
			}
		}
		if n.ReplicaSets != nil && n.ControllerOf != nil {
			for _, obj := range n.ReplicaSets() {
				kind, rcSel, sel := n.ControllerOf(obj)
				rec := C.ksim_k8s_controller{kind: p.s(kind), namespace_: p.s(obj.GetNamespace()), name: p.s(obj.GetName()),
					rc_selector_first: -1, selector: p.selector(sel)}
				if rcSel != nil {
					rec.rc_selector_first, rec.rc_selector_count = p.kvMap(rcSel)
				}
				p.controllers = append(p.controllers, rec)
			}
		}
	}
	cp, free := p.build()
	defer free()
	return n.errOf(C.ksim_encode_pods(n.enc, cp, &opts))
}

func (n *NativeEncoder) encodedSet() *C.ksim_pod_set {
	var ps C.ksim_pod_set
	C.ksim_encoder_pods(n.enc, &ps)
	return &ps
}

// layoutGrew: the compile added label columns or count classes (keys or
// selectors no pod referenced before): the device needs the table again.
func (n *NativeEncoder) layoutGrew() bool {
	in := n.info()
	return int32(in.n_label_cols) != n.layout[0] || int32(in.n_classes) != n.layout[1]
}

// Pod encodes the cycle's pod; the set stays valid until the next Pod call.
// A pod that references new label keys or selectors re-sends the table (the
// framework snapshot, which Snapshot just matched, is the truth).
func (n *NativeEncoder) Pod(pod *v1.Pod) (*C.ksim_pod_set, error) {
	n.mu.Lock()
	defer n.mu.Unlock()
	if err := n.encodeQueue([]*v1.Pod{pod}); err != nil {
		return nil, err
	}
	if n.podCopy != nil {
		n.podCopy()
		n.podCopy = nil
	}
	set, free := copyPodSet(n.encodedSet())
	n.podCopy = free
	return set, nil
}

// Pods encodes pods into a set the caller owns until release.
func (n *NativeEncoder) Pods(pods []*v1.Pod) (*C.ksim_pod_set, func(), error) {
	n.mu.Lock()
	defer n.mu.Unlock()
	if err := n.encodeQueue(pods); err != nil {
		return nil, nil, err
	}
	if n.layoutGrew() {
		// a nominated pod nobody encoded before, mid-cycle: the engine's
		// table cannot change under the cycle in flight; the original plugins answer
		return nil, nil, fmt.Errorf("ksim: pods reference label keys or selectors the device snapshot lacks")
	}
	set, free := copyPodSet(n.encodedSet())
	return set, free, nil
}

// Resync re-sends the table after Pod grew the layout (call before the cycle's
// ksim_fw_prefilter; plugins.go ensureFilter does): every node kept, the
// device's binds replayed on the grown table.
func (n *NativeEncoder) Resync(e *Engine) error {
	n.mu.Lock()
	defer n.mu.Unlock()
	return n.resend(e)
}

func (n *NativeEncoder) NodeNames() []string { return n.names }

func (n *NativeEncoder) Position(name string) (int, bool) {
	p, ok := n.pos[name]
	return p, ok
}

func (n *NativeEncoder) BoundPod(index int) *v1.Pod { return n.boundRows[index] }

// PreFilterNodeNames: NodeAffinity's PreFilterResult.NodeNames (nil: all
// nodes; empty: conflicting terms), ksim/encode.py prefilter_node_names.
func (n *NativeEncoder) PreFilterNodeNames(pod *v1.Pod) sets.String {
	a := pod.Spec.Affinity
	if a == nil || a.NodeAffinity == nil || a.NodeAffinity.RequiredDuringSchedulingIgnoredDuringExecution == nil {
		return nil
	}
	terms := a.NodeAffinity.RequiredDuringSchedulingIgnoredDuringExecution.NodeSelectorTerms
	if len(terms) == 0 {
		return nil
	}
	var names sets.String
	for _, t := range terms {
		var tn sets.String
		for _, r := range t.MatchFields {
			if r.Key == "metadata.name" && r.Operator == v1.NodeSelectorOpIn {
				vals := sets.NewString(r.Values...)
				if tn == nil {
					tn = vals
				} else {
					tn = tn.Intersection(vals)
				}
			}
		}
		if tn == nil {
			return nil
		}
		if names == nil {
			names = sets.NewString()
		}
		names = names.Union(tn)
	}
	return names
}

// FilterMessage is Status.Message() of a failing Filter (ksim/wrapped.py
// filter_message).
func (n *NativeEncoder) FilterMessage(plugin string, detail uint32, node string, pod *v1.Pod) string {
	switch plugin {
	case "NodeUnschedulable":
		return "node(s) were unschedulable"
	case "NodeName":
		return "node(s) didn't match the requested node name"
	case "TaintToleration":
		k := C.GoString(C.ksim_encoder_string(n.enc, C.KSIM_ENC_STR_TAINT_KEY, C.int32_t(detail), 0))
		v := C.GoString(C.ksim_encoder_string(n.enc, C.KSIM_ENC_STR_TAINT_VALUE, C.int32_t(detail), 0))
		return fmt.Sprintf("node(s) had untolerated taint {%s: %s}", k, v)
	case "NodeAffinity":
		if detail == C.KSIM_NA_ENFORCED {
			return "node(s) didn't match scheduler-enforced node affinity"
		}
		return "node(s) didn't match Pod's node affinity/selector"
	case "NodePorts":
		return "node(s) didn't have free ports for the requested pod ports"
	case "NodeResourcesFit":
		var reasons []string
		if detail&C.KSIM_FIT_TOO_MANY_PODS != 0 {
			reasons = append(reasons, "Too many pods")
		}
		if detail&C.KSIM_FIT_CPU != 0 {
			reasons = append(reasons, "Insufficient cpu")
		}
		if detail&C.KSIM_FIT_MEMORY != 0 {
			reasons = append(reasons, "Insufficient memory")
		}
		if detail&C.KSIM_FIT_EPHEMERAL != 0 {
			reasons = append(reasons, "Insufficient ephemeral-storage")
		}
		in := n.info()
		for k := 0; k < int(in.n_scalar); k++ {
			if detail&(C.KSIM_FIT_SCALAR0<<uint(k)) != 0 {
				reasons = append(reasons, "Insufficient "+C.GoString(C.ksim_encoder_string(n.enc, C.KSIM_ENC_STR_SCALAR,
					C.int32_t(k), 0)))
			}
		}
		return strings.Join(reasons, ", ")
	case "PodTopologySpread":
		if detail == C.KSIM_PTS_MISSING_LABEL {
			return "node(s) didn't match pod topology spread constraints (missing required label)"
		}
		return "node(s) didn't match pod topology spread constraints"
	case "InterPodAffinity":
		switch detail {
		case C.KSIM_IPA_AFFINITY:
			return "node(s) didn't match pod affinity rules"
		case C.KSIM_IPA_ANTI_AFFINITY:
			return "node(s) didn't match pod anti-affinity rules"
		default:
			return "node(s) didn't satisfy existing pods anti-affinity rules"
		}
	case "NetworkBandwidth":
		return networkBandwidthMessage(detail, node, pod, n)
	}
	return plugin + " failed"
}

// networkBandwidthMessage: networkbandwidth/plugin.go:56,60,75,87,93,98.
func networkBandwidthMessage(detail uint32, node string, pod *v1.Pod, n *NativeEncoder) string {
	limit, ingress, egress := n.NodeLimitAnnotation, n.IngressRequestAnnotation, n.EgressRequestAnnotation
	if limit == "" {
		limit = "node.kubernetes.io/network-limit"
	}
	if ingress == "" {
		ingress = "kubernetes.io/ingress-request"
	}
	if egress == "" {
		egress = "kubernetes.io/egress-request"
	}
	switch detail {
	case C.KSIM_NB_INSUFFICIENT:
		return fmt.Sprintf("Node %s does not have enough network bandwidth capacity to schedule pod", node)
	case C.KSIM_NB_NO_LIMIT:
		return fmt.Sprintf("Node %s does not have %s annotation present", node, limit)
	case C.KSIM_NB_LIMIT_BAD:
		return fmt.Sprintf("Node %s has an incorrect quantity in %s annotation present", node, limit)
	case C.KSIM_NB_INGRESS_BAD:
		return fmt.Sprintf("Could not parse quantity from pod %s %s annotations", pod.Name, ingress)
	case C.KSIM_NB_EGRESS_BAD:
		return fmt.Sprintf("Could not parse quantity from pod %s %s annotations", pod.Name, egress)
	}
	return fmt.Sprintf("Pod %s does not have network bandwidth request annotations set. (Missing %s or %s)",
		pod.Name, ingress, egress)
}
