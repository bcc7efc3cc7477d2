"""Plugin args beyond the defaults (NewPluginConfig merges a
profile's pluginConfig over the defaults, /root/reference/simulator/scheduler/
plugin/plugins.go:103-179): NodeResourcesFit MostAllocated and
RequestedToCapacityRatio scoring (extended resources included),
ignoredResources / ignoredResourceGroups, NodeAffinity addedAffinity,
DefaultPreemption's candidate counts.

CPU only: known-answer vectors hand-derived from the upstream formulas, the C
oracle cycle by cycle against the object-level restatement (oracle/objref.py)
under each arg, and the ingest's decoding (fields decoded over the default
object; anything the engine does not implement refused, never dropped).
Parity against the Go plugins stays unpinned (no Go toolchain here)."""
import ctypes

import numpy as np
import pytest

from ksim import abi, ingest, profile
from ksim.encode import encode_cluster, encode_pods
from ksim.model import Container, Node, NodeSelectorTerm, Pod, PreferredTerm, Requirement, Taint
from ksim.wrapped import filter_message
from oracle.objref import ObjScheduler
from oracle.oracle import Oracle, lib

SCORE_NAMES = ["NodeResourcesBalancedAllocation", "ImageLocality", "InterPodAffinity", "NodeResourcesFit",
               "NodeAffinity", "PodTopologySpread", "TaintToleration"]
GPU, NV, HP = "example.com/gpu", "nvidia.com/gpu", "hugepages-2Mi"


# ---- known answers ------------------------------------------------------------------
def test_most_requested_score_kat():
    """mostRequestedScore: requested * 100 / capacity, requested clamped to capacity."""
    f = lib().ksim_oracle_most_requested_score
    assert f(0, 4000) == 0
    assert f(1000, 4000) == 25
    assert f(3999, 4000) == 99           # truncation
    assert f(5000, 4000) == 100          # clamped
    assert f(7, 0) == 0                  # capacity 0


def _shape_profile(points):
    p = abi.Profile()
    p.fit_strategy = abi.FIT_REQUESTED_TO_CAPACITY_RATIO
    p.fit_n_shape = len(points)
    for i, (u, s) in enumerate(points):
        p.fit_shape_util[i], p.fit_shape_score[i] = u, s * 10
    return p


@pytest.mark.parametrize("points,cases", [
    # bin packing (0, 0) -> (100, 10): score = utilization
    ([(0, 0), (100, 10)], [(0, 0), (37, 37), (100, 100), (120, 100)]),
    # spreading (0, 10) -> (100, 0): a decreasing segment truncates toward zero
    ([(0, 10), (100, 0)], [(0, 100), (1, 99), (33, 67), (100, 0)]),
    # three points; below the first point its score, past the last its score
    ([(20, 2), (50, 8), (80, 3)], [(0, 20), (20, 20), (35, 50), (49, 78), (50, 80), (51, 79), (79, 32), (80, 30),
                                   (95, 30)]),
])
def test_broken_linear_kat(points, cases):
    """helper.BuildBrokenLinearFunction on shape scores x 10 (MaxNodeScore /
    MaxCustomPriorityScore): s_{i-1} + (s_i - s_{i-1}) * (p - u_{i-1}) / (u_i - u_{i-1})
    in Go int64 (truncating) arithmetic."""
    prof = _shape_profile(points)
    f = lib().ksim_oracle_broken_linear
    for p, want in cases:
        assert f(ctypes.byref(prof), p) == want, (points, p)


# ---- oracle vs objref under each arg -----------------------------------------------
def _nodes(n=24, seed=1):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        alloc = {"cpu": str(int(rng.choice([4, 8, 16]))), "memory": f"{int(rng.choice([16, 32, 64]))}Gi",
                 "pods": "110"}
        if i % 3:
            alloc[GPU] = str(int(rng.integers(1, 5)))
        if i % 4 == 1:
            alloc[NV] = str(int(rng.integers(1, 3)))
        if i % 5 != 2:
            alloc[HP] = f"{int(rng.integers(1, 8)) * 64}Mi"
        labels = {"kubernetes.io/hostname": f"n{i}", "topology.kubernetes.io/zone": f"z{i % 3}",
                  "pool": "ab"[i % 2]}
        taints = [Taint("spot", "true", "PreferNoSchedule")] if i % 7 == 3 else []
        out.append(Node(f"n{i}", labels, taints, alloc))
    return out


def _pods(n=70, seed=2, scalars=True):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        req = {"cpu": f"{int(rng.integers(1, 30)) * 100}m", "memory": f"{int(rng.integers(1, 24)) * 256}Mi"}
        if scalars and i % 3 == 0:
            req[GPU] = str(int(rng.integers(1, 3)))
        if scalars and i % 7 == 1:
            req[NV] = "1"
        if scalars and i % 5 == 3:
            req[HP] = "128Mi"
        if i % 11 == 4:
            req = {}                                      # no requests: the non-zero defaults score it
        p = Pod(f"p{i}", containers=[Container(req)])
        if i % 6 == 5:
            p.preferred_terms = [PreferredTerm(int(rng.integers(1, 60)),
                                               NodeSelectorTerm([Requirement("pool", "In", ["a"])]))]
        if i % 8 == 7:
            p.node_selector = {"topology.kubernetes.io/zone": "z1"}
        out.append(p)
    return out


def run_both(nodes, pods, sp: profile.SchedulerProfile, bound=()):
    """Every cycle of ``pods`` on the C oracle and on objref: filter outcomes and
    messages, raw / normalized scores, totals, placements."""
    cluster, _ = encode_cluster(nodes, list(bound), extra_scalar=[GPU, NV, HP])
    enc = encode_pods(cluster, pods, added_affinity=sp.node_affinity)
    prof = profile.compile_profile(sp, cluster.scalar_names)
    ora = Oracle(cluster, prof)
    ref = ObjScheduler(nodes, list(bound), pct=sp.percentage_of_nodes_to_score, seed=sp.tiebreak_seed,
                       fit=sp.fit, node_affinity=sp.node_affinity, preemption=sp.preemption)
    ref.scalar_order = list(cluster.scalar_names)
    forder = sp.filter_order()
    names = cluster.node_names
    chosen = []
    for i, pod in enumerate(pods):
        o = ora.cycle(enc, i)
        r = ref.cycle(pod)
        where = f"pod {i} ({pod.name})"
        for pos, name in enumerate(names):
            fp = int(o["fail_plugin"][pos])
            if fp == abi.NOT_EVALUATED:
                assert name not in r["filter"], f"{where}: {name} evaluated only by objref"
                continue
            pl, msg = r["filter"][name]
            if fp == abi.PASSED:
                assert pl is None, f"{where}: {name} oracle passed, objref {pl}: {msg}"
            else:
                assert pl == forder[fp], f"{where}: {name} oracle {forder[fp]} objref {pl}"
                assert msg == filter_message(cluster, forder[fp], int(o["fail_detail"][pos])), (where, name, msg)
        assert o["n_feasible"] == r["n_feasible"], where
        if o["n_feasible"] > 1:
            for k, pl in enumerate(SCORE_NAMES):
                for pos in np.nonzero(o["scored"])[0]:
                    name = names[pos]
                    assert o["raw"][k][pos] == r["raw"][pl][name], f"{where}: raw {pl} on {name}"
                    assert o["norm"][k][pos] == r["norm"][pl][name], f"{where}: norm {pl} on {name}"
                    assert o["total"][pos] == r["total"][name], f"{where}: total on {name}"
        got = names[o["chosen"]] if o["chosen"] >= 0 else None
        assert got == r["chosen"], f"{where}: oracle {got} objref {r['chosen']}"
        chosen.append(got)
    return chosen


FIT_CASES = {
    "most": profile.FitArgs("MostAllocated"),
    "most_weighted": profile.FitArgs("MostAllocated", [("cpu", 2), ("memory", 1), (GPU, 3)]),
    "rtcr_pack": profile.FitArgs("RequestedToCapacityRatio", [("cpu", 1), ("memory", 1)], [(0, 0), (100, 10)]),
    "rtcr_spread": profile.FitArgs("RequestedToCapacityRatio", [("cpu", 3), ("memory", 1), (GPU, 2)],
                                   [(0, 10), (100, 0)]),
    "rtcr_three": profile.FitArgs("RequestedToCapacityRatio", [("cpu", 1), (NV, 5), (HP, 2)],
                                  [(20, 2), (50, 8), (80, 3)]),
    "least_scalar": profile.FitArgs("LeastAllocated", [("cpu", 1), ("memory", 1), (GPU, 4), ("memory", 7)]),
    "ignored": profile.FitArgs(ignored_resources=[GPU, HP]),           # hugepages are native: not ignorable
    "ignored_group": profile.FitArgs("MostAllocated", [("cpu", 1), (NV, 1)], ignored_resource_groups=["nvidia.com"]),
}


@pytest.mark.parametrize("pct", [0, 100])
@pytest.mark.parametrize("case", sorted(FIT_CASES))
def test_fit_args_oracle_vs_objref(case, pct):
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=pct, fit=FIT_CASES[case])
    chosen = run_both(_nodes(), _pods(), sp)
    assert sum(c is not None for c in chosen) > 20


def test_ignored_resources_admit_oversubscribed_pods():
    """With example.com/gpu ignored, pods asking for more GPUs than any node
    holds still fit (and the binds still count them); without it they do not."""
    nodes = _nodes(12)
    pods = [Pod(f"g{i}", containers=[Container({"cpu": "100m", GPU: "9"})]) for i in range(6)]
    base = run_both(nodes, pods, profile.SchedulerProfile(percentage_of_nodes_to_score=100))
    assert base == [None] * 6
    ign = run_both(nodes, pods, profile.SchedulerProfile(percentage_of_nodes_to_score=100,
                                                         fit=profile.FitArgs(ignored_resources=[GPU])))
    assert all(c is not None for c in ign)


def _added(required=True, preferred=True):
    return profile.NodeAffinityArgs(
        [NodeSelectorTerm([Requirement("topology.kubernetes.io/zone", "In", ["z0", "z2"])]),
         NodeSelectorTerm([Requirement("kubernetes.io/hostname", "In", ["n4"])])] if required else None,
        [PreferredTerm(40, NodeSelectorTerm([Requirement("pool", "In", ["b"])])),
         PreferredTerm(7, NodeSelectorTerm([Requirement("topology.kubernetes.io/zone", "In", ["z2"])]))]
        if preferred else [])


@pytest.mark.parametrize("pct", [0, 100])
@pytest.mark.parametrize("req,pref", [(True, True), (True, False), (False, True)])
def test_added_affinity_oracle_vs_objref(req, pref, pct):
    """NodeAffinityArgs.addedAffinity: the enforced selector fails first with
    errReasonEnforced; the added preferred terms add to the pod's own score.
    Pods with a zone z1 nodeSelector can only land on n4 (the second added term)."""
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=pct, node_affinity=_added(req, pref))
    chosen = run_both(_nodes(), _pods(scalars=False), sp)
    zones = {f"n{i}": f"z{i % 3}" for i in range(24)}
    if req:
        assert all(c is None or zones[c] in ("z0", "z2") or c == "n4" for c in chosen)


def test_added_affinity_message():
    nodes = _nodes(6)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=100, node_affinity=_added(True, False))
    cluster, _ = encode_cluster(nodes, extra_scalar=[GPU, NV, HP])
    enc = encode_pods(cluster, [Pod("x", containers=[Container({"cpu": "1"})])], added_affinity=sp.node_affinity)
    assert enc.pods["flags"][0] & abi.POD_ADDED_AFFINITY
    o = Oracle(cluster, profile.compile_profile(sp, cluster.scalar_names)).cycle(enc, 0)
    forder = sp.filter_order()
    msgs = {cluster.node_names[i]: filter_message(cluster, forder[o["fail_plugin"][i]], int(o["fail_detail"][i]))
            for i in range(6) if o["fail_plugin"][i] < len(forder)}
    # zones z0 z1 z2 z0 z1 z2: n1 fails, n4 passes by the second (hostname) term
    assert msgs == {"n1": "node(s) didn't match scheduler-enforced node affinity"}


@pytest.mark.parametrize("pct_abs", [(10, 100), (50, 1), (0, 3), (100, 0)])
def test_preemption_candidate_args(pct_abs):
    """DefaultPreemptionArgs minCandidateNodesPercentage / Absolute bound the
    dry run's candidates (calculateNumCandidates) on the C oracle and objref."""
    from test_preemption import crowded
    from ksim.preemption import bound_table
    nodes, bound, start, order = crowded(n_nodes=40, seed=4)
    cluster, _ = encode_cluster(nodes, bound)
    table = bound_table(cluster, bound, start)
    rng = np.random.default_rng(104)
    pods = [Pod(f"p{i}", priority=int(rng.choice([0, 5, 50, 500, 5000])),
                containers=[Container({"cpu": f"{int(rng.integers(10, 400)) * 100}m",
                                       "memory": f"{int(rng.integers(4, 40))}Gi"})]) for i in range(30)]
    enc = encode_pods(cluster, pods)
    pa = profile.PreemptionArgs(*pct_abs)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=100, preemption=pa)
    ora = Oracle(cluster, profile.compile_profile(sp))
    ref = ObjScheduler(nodes, bound, pct=100, seed=sp.tiebreak_seed, preemption=pa)
    cands = set()
    for i, pod in enumerate(pods):
        node, victims, n_pot, n_cand = ora.preempt(enc, i, pod.priority, table)
        rnode, rvictims = ref.preempt(pod, pod.priority, start, order)
        assert (cluster.node_names[node] if node >= 0 else None) == rnode, f"pod {i}"
        assert [bound[v].name for v in victims] == rvictims, f"pod {i}"
        want = min(max(n_pot * pa.min_candidate_nodes_percentage // 100, pa.min_candidate_nodes_absolute), n_pot)
        assert n_cand <= want
        cands.add(n_cand)
    assert len(cands) > 1 or pct_abs == (10, 100)


# ---- ingest: decoding over the defaults, refusals ------------------------------------
def _profile(plugin_config):
    return ingest.profile_from_config({"schedulerName": "s", "pluginConfig": plugin_config})


def test_ingest_fit_args_merge_over_defaults():
    sp = _profile([{"name": "NodeResourcesFit", "args": {"scoringStrategy": {"type": "MostAllocated"}}}])
    assert sp.fit.strategy == "MostAllocated" and sp.fit.resources == [("cpu", 1), ("memory", 1)]
    sp = _profile([{"name": "NodeResourcesFit", "args": {
        "ignoredResources": [GPU], "ignoredResourceGroups": ["nvidia.com"],
        "scoringStrategy": {"type": "RequestedToCapacityRatio", "resources": [{"name": "cpu", "weight": 0},
                                                                              {"name": GPU, "weight": 5}],
                            "requestedToCapacityRatio": {"shape": [{"utilization": 0, "score": 0},
                                                                   {"utilization": 100, "score": 10}]}}}}])
    assert sp.fit.strategy == "RequestedToCapacityRatio" and sp.fit.resources == [("cpu", 1), (GPU, 5)]
    assert sp.fit.shape == [(0, 0), (100, 10)]
    p = profile.compile_profile(sp, [HP, GPU, NV])
    assert p.fit_strategy == abi.FIT_REQUESTED_TO_CAPACITY_RATIO and p.fit_n_shape == 2
    assert list(p.fit_shape_score[:2]) == [0, 100]
    assert p.fit_ignored_scalar == 0b110                 # hugepages (column 0) is native


def test_ingest_other_args():
    sp = _profile([
        {"name": "NodeAffinity", "args": {"addedAffinity": {
            "requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": [
                {"matchExpressions": [{"key": "pool", "operator": "In", "values": ["a"]}]}]},
            "preferredDuringSchedulingIgnoredDuringExecution": [
                {"weight": 3, "preference": {"matchExpressions": [{"key": "zone", "operator": "Exists"}]}}]}}},
        {"name": "DefaultPreemption", "args": {"minCandidateNodesPercentage": 30}},
        {"name": "VolumeBinding", "args": {"bindTimeoutSeconds": 30}},
        {"name": "PodTopologySpread", "args": {"defaultingType": "List", "defaultConstraints": [
            {"maxSkew": 2, "topologyKey": "topology.kubernetes.io/zone", "whenUnsatisfiable": "DoNotSchedule"}]}}])
    assert sp.node_affinity.required[0].match_expressions[0].values == ["a"]
    assert sp.node_affinity.preferred[0].weight == 3
    assert (sp.preemption.min_candidate_nodes_percentage, sp.preemption.min_candidate_nodes_absolute) == (30, 100)
    assert sp.spread.defaulting_type == "List" and sp.spread.default_constraints[0].max_skew == 2


@pytest.mark.parametrize("pc,exc", [
    ({"name": "NodeResourcesFit", "args": {"scoringStrategy": {"type": "Balanced"}}}, ValueError),
    ({"name": "NodeResourcesFit", "args": {"scoringStrategy": {"type": "RequestedToCapacityRatio"}}}, ValueError),
    ({"name": "NodeResourcesFit", "args": {"scoringStrategy": {"resources": [{"name": "cpu", "weight": 101}]}}},
     ValueError),
    ({"name": "NodeResourcesFit", "args": {"ignoredResourceGroups": ["a/b"]}}, ValueError),
    ({"name": "NodeResourcesFit", "args": {"somethingNew": 1}}, ingest.UnsupportedArgs),
    ({"name": "InterPodAffinity", "args": {"ignorePreferredTermsOfExistingPods": True}}, ingest.UnsupportedArgs),
    ({"name": "NodeAffinity", "args": {"addedAffinity": {
        "requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": []}}}}, ValueError),
    ({"name": "PodTopologySpread", "args": {"defaultConstraints": [
        {"maxSkew": 1, "topologyKey": "zone", "whenUnsatisfiable": "ScheduleAnyway"}]}}, ValueError),  # System
    ({"name": "PodTopologySpread", "args": {"defaultingType": "List", "defaultConstraints": [
        {"maxSkew": 1, "topologyKey": "zone", "whenUnsatisfiable": "ScheduleAnyway",
         "labelSelector": {"matchLabels": {"a": "b"}}}]}}, ValueError),
    ({"name": "DefaultPreemption", "args": {"minCandidateNodesPercentage": 0, "minCandidateNodesAbsolute": 0}},
     ValueError),
    ({"name": "TaintToleration", "args": {"x": 1}}, ingest.UnsupportedArgs),
])
def test_ingest_refuses(pc, exc):
    with pytest.raises(exc):
        sp = _profile([pc])
        profile.compile_profile(sp)
