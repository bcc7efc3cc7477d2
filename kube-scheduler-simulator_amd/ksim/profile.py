"""Profile handling: the simulator's plugin-set conversion and the engine profile.

Mirrors, name for name:
  * config.InTree*PluginSet / RegisteredScorePlugins — simulator/scheduler/config/plugin.go:12-273
  * plugin.ConvertForSimulator / applyPluingSet / mergePluginSet — simulator/scheduler/plugin/plugins.go:185-288
  * plugin.registeredPlugins — plugins.go:293-357
  * the store's default score weights — plugins.go:22-34
  * default plugin args — pinned by plugins_test.go:901-1119
and compiles the converted profile into the engine's ``ksim_profile``.
"""
from __future__ import annotations

import copy
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import re

from . import abi
from .model import NodeSelectorTerm, PreferredTerm, TopologySpreadConstraint
from .netbw import NetworkBandwidthArgs

SUFFIX = "Wrapped"                    # wrappedplugin.go:239 pluginSuffix


def plugin_name(name: str) -> str:    # wrappedplugin.go:242-244
    return name + SUFFIX


def original_name(name: str) -> str:
    return name[: -len(SUFFIX)] if name.endswith(SUFFIX) else name


@dataclass
class Plugin:
    name: str
    weight: Optional[int] = None


@dataclass
class PluginSet:
    enabled: List[Plugin] = field(default_factory=list)
    disabled: List[Plugin] = field(default_factory=list)


EXTENSION_POINTS = ["preFilter", "filter", "postFilter", "preScore", "score", "reserve",
                    "permit", "preBind", "bind", "postBind"]


def _ps(*names, weights=None) -> PluginSet:
    w = weights or {}
    return PluginSet([Plugin(n, w.get(n)) for n in names])


# v1beta2 defaults of k8s v1.26 (DefaultSchedulerConfig, config/config.go:9-15);
# order and weights pinned by scheduler_test.go:380-437.
def default_plugins() -> Dict[str, PluginSet]:
    return {
        "preFilter": _ps("NodeResourcesFit", "NodePorts", "VolumeRestrictions", "PodTopologySpread",
                         "InterPodAffinity", "VolumeBinding", "NodeAffinity"),
        "filter": _ps("NodeUnschedulable", "NodeName", "TaintToleration", "NodeAffinity", "NodePorts",
                      "NodeResourcesFit", "VolumeRestrictions", "EBSLimits", "GCEPDLimits",
                      "NodeVolumeLimits", "AzureDiskLimits", "VolumeBinding", "VolumeZone",
                      "PodTopologySpread", "InterPodAffinity"),
        "postFilter": _ps("DefaultPreemption"),
        "preScore": _ps("InterPodAffinity", "PodTopologySpread", "TaintToleration", "NodeAffinity"),
        "score": _ps("NodeResourcesBalancedAllocation", "ImageLocality", "InterPodAffinity",
                     "NodeResourcesFit", "NodeAffinity", "PodTopologySpread", "TaintToleration",
                     weights={"NodeResourcesBalancedAllocation": 1, "ImageLocality": 1,
                              "InterPodAffinity": 1, "NodeResourcesFit": 1, "NodeAffinity": 1,
                              "PodTopologySpread": 2, "TaintToleration": 1}),
        "reserve": _ps("VolumeBinding"),
        "permit": _ps(),
        "preBind": _ps("VolumeBinding"),
        "bind": _ps("DefaultBinder"),
        "postBind": _ps(),
    }


# out-of-tree plugins registered by the fork (config/plugin.go:214-221,266-273)
OUT_OF_TREE = {"filter": [Plugin("NetworkBandwidth")], "score": [Plugin("NetworkBandwidth")]}


def registered_plugins(ext: str) -> List[Plugin]:
    """config.Registered<Ext>Plugins: in-tree defaults + OutOfTree<Ext>Plugins."""
    return copy.deepcopy(default_plugins()[ext].enabled) + copy.deepcopy(OUT_OF_TREE.get(ext, []))


def default_score_weights() -> Dict[str, int]:
    """Weights the result store applies (plugins.go:22-34): registry default,
    0 for plugins without one."""
    return {p.name: (p.weight if p.weight is not None else 0) for p in registered_plugins("score")}


def all_registered_plugins() -> List[Plugin]:
    """plugins.go registeredPlugins(): score, bind, postBind, preBind, reserve,
    permit, preFilter, preScore, filter, postFilter — de-duplicated by name."""
    out, seen = [], set()
    for ext in ["score", "bind", "postBind", "preBind", "reserve", "permit", "preFilter",
                "preScore", "filter", "postFilter"]:
        for p in registered_plugins(ext):
            if p.name not in seen:
                seen.add(p.name)
                out.append(p)
    return out


def merge_plugin_set(in_tree: PluginSet, out_of_tree: PluginSet) -> PluginSet:
    """mergePluginSet (plugins.go:246-288, copied upstream from v1beta2 default_config.go)."""
    disabled = {p.name for p in out_of_tree.disabled}
    custom = {p.name: (i, p) for i, p in enumerate(out_of_tree.enabled)}
    replaced = set()
    enabled: List[Plugin] = []
    if "*" not in disabled:
        for p in in_tree.enabled:
            if p.name in disabled:
                continue
            if p.name in custom:
                i, cp = custom[p.name]
                p = cp
                replaced.add(i)
            enabled.append(copy.deepcopy(p))
    for i, p in enumerate(out_of_tree.enabled):
        if i not in replaced:
            enabled.append(copy.deepcopy(p))
    return PluginSet(enabled)


def convert_for_simulator(plugins: Optional[Dict[str, PluginSet]]) -> Dict[str, PluginSet]:
    """ConvertForSimulator + applyPluingSet (plugins.go:185-242): merge the
    user's set over the in-tree defaults, rename to <Name>Wrapped, Disabled=[*]."""
    plugins = plugins or {}
    d = default_plugins()
    out = {}
    for ext in EXTENSION_POINTS:
        merged = merge_plugin_set(d[ext], plugins.get(ext, PluginSet()))
        out[ext] = PluginSet([Plugin(plugin_name(p.name), p.weight) for p in merged.enabled],
                             [Plugin("*")])
    return out


@dataclass
class FitArgs:                   # NodeResourcesFitArgs, LeastAllocated cpu:1 memory:1
    strategy: str = "LeastAllocated"
    resources: List[tuple] = field(default_factory=lambda: [("cpu", 1), ("memory", 1)])
    # scoringStrategy.requestedToCapacityRatio.shape: (utilization, score 0..10); None = absent
    shape: Optional[List[tuple]] = None
    ignored_resources: List[str] = field(default_factory=list)
    ignored_resource_groups: List[str] = field(default_factory=list)


@dataclass
class NodeAffinityArgs:          # NodeAffinityArgs.addedAffinity (nil by default)
    required: Optional[List[NodeSelectorTerm]] = None    # requiredDuringScheduling...nodeSelectorTerms
    preferred: List[PreferredTerm] = field(default_factory=list)


@dataclass
class PodTopologySpreadArgs:     # PodTopologySpreadArgs (defaultingType System)
    defaulting_type: str = "System"
    default_constraints: List[TopologySpreadConstraint] = field(default_factory=list)

    def constraints(self) -> List[TopologySpreadConstraint]:
        """The constraints buildDefaultConstraints filters (v1.26
        podtopologyspread.New: System -> systemDefaultConstraints, List -> the args')."""
        if self.defaulting_type == "System":
            return [TopologySpreadConstraint(3, "kubernetes.io/hostname", "ScheduleAnyway"),
                    TopologySpreadConstraint(5, "topology.kubernetes.io/zone", "ScheduleAnyway")]
        return list(self.default_constraints)


@dataclass
class PreemptionArgs:            # DefaultPreemptionArgs
    min_candidate_nodes_percentage: int = 10
    min_candidate_nodes_absolute: int = 100


@dataclass
class BalancedAllocationArgs:    # NodeResourcesBalancedAllocationArgs cpu:1 memory:1
    resources: List[tuple] = field(default_factory=lambda: [("cpu", 1), ("memory", 1)])


@dataclass
class SchedulerProfile:
    """The converted profile the engine runs (one KubeSchedulerProfile)."""
    plugins: Dict[str, PluginSet] = field(default_factory=lambda: convert_for_simulator(None))
    fit: FitArgs = field(default_factory=FitArgs)
    balanced: BalancedAllocationArgs = field(default_factory=BalancedAllocationArgs)
    hard_pod_affinity_weight: int = 1
    node_affinity: NodeAffinityArgs = field(default_factory=NodeAffinityArgs)
    spread: PodTopologySpreadArgs = field(default_factory=PodTopologySpreadArgs)
    preemption: PreemptionArgs = field(default_factory=PreemptionArgs)
    network_bandwidth: NetworkBandwidthArgs = field(default_factory=NetworkBandwidthArgs)
    percentage_of_nodes_to_score: int = 0      # simulator forces the default (scheduler.go:231-241)
    tiebreak_seed: int = 0x4B53494D

    def filter_order(self) -> List[str]:
        return [original_name(p.name) for p in self.plugins["filter"].enabled]

    def score_plugins(self) -> List[Plugin]:
        return [Plugin(original_name(p.name), p.weight) for p in self.plugins["score"].enabled]

    def with_weights(self, weights: Dict[str, int]) -> "SchedulerProfile":
        p = copy.deepcopy(self)
        for pl in p.plugins["score"].enabled:
            n = original_name(pl.name)
            if n in weights:
                pl.weight = weights[n]
        return p


def _res_id(name: str, scalar_names: List[str]) -> int:
    if name == "cpu":
        return abi.RES_CPU
    if name == "memory":
        return abi.RES_MEMORY
    if name == "ephemeral-storage":
        return abi.RES_EPHEMERAL
    if name in scalar_names:
        return abi.RES_SCALAR0 + scalar_names.index(name)
    return -1


_QUALIFIED_NAME = re.compile(r"^([A-Za-z0-9]([-A-Za-z0-9_.]*[A-Za-z0-9])?)$")
_DNS_SUBDOMAIN = re.compile(r"^[a-z0-9]([-a-z0-9]*[a-z0-9])?(\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*$")


def _qualified_name(s: str) -> bool:
    """k8s.io/apimachinery validation.IsQualifiedName."""
    parts = s.split("/")
    if len(parts) == 1:
        name = parts[0]
    elif len(parts) == 2:
        prefix, name = parts
        if not prefix or len(prefix) > 253 or not _DNS_SUBDOMAIN.match(prefix):
            return False
    else:
        return False
    return 0 < len(name) <= 63 and bool(_QUALIFIED_NAME.match(name))


def is_extended_resource_name(name: str) -> bool:
    """v1helper.IsExtendedResourceName: not native (no "/", or in the
    kubernetes.io/ namespace), not "requests."-prefixed, and a qualified name
    once prefixed with "requests."."""
    if "/" not in name or "kubernetes.io/" in name or name.startswith("requests."):
        return False
    return _qualified_name("requests." + name)


def fit_ignored_scalar(fit: "FitArgs", scalar_names: List[str]) -> int:
    """NodeResourcesFit fitsRequest's skip set over the cluster's scalar columns:
    bit k when column k is an extended resource named in ignoredResources or
    whose group (the part before "/") is in ignoredResourceGroups."""
    mask = 0
    ign, groups = set(fit.ignored_resources), set(fit.ignored_resource_groups)
    for k, name in enumerate(scalar_names):
        if is_extended_resource_name(name) and (name in ign or name.split("/")[0] in groups):
            mask |= 1 << k
    return mask


def validate_fit_args(fit: "FitArgs") -> None:
    """validation.ValidateNodeResourcesFitArgs (NewFit refuses the plugin -- and
    the scheduler does not start -- on any of these)."""
    for r in fit.ignored_resources:
        if not _qualified_name(r):
            raise ValueError(f"NodeResourcesFitArgs.ignoredResources: {r!r} is not a valid label name")
    for g in fit.ignored_resource_groups:
        if "/" in g or not _qualified_name(g):
            raise ValueError(f"NodeResourcesFitArgs.ignoredResourceGroups: {g!r} is not a valid group name")
    if fit.strategy not in abi.FIT_STRATEGY_ID:
        raise ValueError(f"NodeResourcesFitArgs.scoringStrategy.type {fit.strategy!r} not supported")
    for name, w in fit.resources:
        if w <= 0 or w > 100:
            raise ValueError(f"resource weight of {name} not in valid range (0, 100]")
    if fit.shape is not None:
        if not fit.shape:
            raise ValueError("requestedToCapacityRatio.shape: at least one point must be specified")
        for i in range(1, len(fit.shape)):
            if fit.shape[i - 1][0] >= fit.shape[i][0]:
                raise ValueError("requestedToCapacityRatio.shape: utilization should be greater than prior element")
        for u, sc in fit.shape:
            if not 0 <= u <= 100 or not 0 <= sc <= 10:
                raise ValueError("requestedToCapacityRatio.shape: utilization in [0, 100], score in [0, 10]")
    if fit.strategy == "RequestedToCapacityRatio" and fit.shape is None:
        # NewFit dereferences the nil RequestedToCapacityRatio: no scheduler
        raise ValueError("RequestedToCapacityRatio scoring strategy without requestedToCapacityRatio")


def validate_spread_args(a: "PodTopologySpreadArgs") -> None:
    """validation.ValidatePodTopologySpreadArgs (v1.26)."""
    if a.defaulting_type not in ("System", "List"):
        raise ValueError(f"PodTopologySpreadArgs.defaultingType {a.defaulting_type!r} not supported")
    if a.defaulting_type == "System" and a.default_constraints:
        raise ValueError('when .defaultingType is "System", .defaultConstraints must be empty')
    seen = set()
    for c in a.default_constraints:
        if c.max_skew <= 0:
            raise ValueError("defaultConstraints: maxSkew must be greater than zero")
        if not c.topology_key or not _qualified_name(c.topology_key):
            raise ValueError(f"defaultConstraints: invalid topologyKey {c.topology_key!r}")
        if c.when_unsatisfiable not in ("DoNotSchedule", "ScheduleAnyway"):
            raise ValueError(f"defaultConstraints: whenUnsatisfiable {c.when_unsatisfiable!r} not supported")
        if c.label_selector is not None:
            raise ValueError("defaultConstraints: constraint must not define a selector, as they deduced for each pod")
        if (c.topology_key, c.when_unsatisfiable) in seen:
            raise ValueError("defaultConstraints: duplicate (topologyKey, whenUnsatisfiable) pair")
        seen.add((c.topology_key, c.when_unsatisfiable))


SUPPORTED_FILTER = set(abi.PLUGINS)
SUPPORTED_SCORE = {"NodeResourcesBalancedAllocation", "ImageLocality", "InterPodAffinity",
                   "NodeResourcesFit", "NodeAffinity", "PodTopologySpread", "TaintToleration",
                   "NetworkBandwidth"}


def compile_profile(prof: SchedulerProfile, scalar_names: List[str] = ()) -> abi.Profile:
    """SchedulerProfile -> ksim_profile.  Unknown plugins raise (the engine
    covers the in-tree default set; out-of-tree plugins keep their own path)."""
    p = abi.Profile()
    fo = prof.filter_order()
    if len(fo) > abi.MAX_FILTER:
        raise ValueError("too many filter plugins")
    for i, n in enumerate(fo):
        if n not in SUPPORTED_FILTER:
            raise ValueError(f"filter plugin {n} not supported by the engine")
        p.filter[i] = abi.PLUGIN_ID[n]
    p.n_filter = len(fo)
    sp = prof.score_plugins()
    if len(sp) > abi.MAX_SCORE:
        raise ValueError("too many score plugins")
    for i, pl in enumerate(sp):
        if pl.name not in SUPPORTED_SCORE:
            raise ValueError(f"score plugin {pl.name} not supported by the engine")
        p.score[i] = abi.PLUGIN_ID[pl.name]
        p.score_weight[i] = pl.weight or 0
    p.n_score = len(sp)
    p.percentage_of_nodes_to_score = prof.percentage_of_nodes_to_score
    scal = list(scalar_names)
    validate_fit_args(prof.fit)
    # resourcesToWeightMap: a name listed twice keeps its last weight
    fw: Dict[str, int] = {}
    for r, w in prof.fit.resources:
        fw.pop(r, None)
        fw[r] = w
    fr = list(fw.items())
    if len(fr) > abi.MAX_RES:
        raise ValueError(f"NodeResourcesFit scoring over {len(fr)} resources (the engine keeps {abi.MAX_RES})")
    p.fit_strategy = abi.FIT_STRATEGY_ID[prof.fit.strategy]
    if prof.fit.strategy == "RequestedToCapacityRatio":
        if len(prof.fit.shape) > abi.MAX_SHAPE:
            raise ValueError(f"requestedToCapacityRatio.shape: more than {abi.MAX_SHAPE} points")
        p.fit_n_shape = len(prof.fit.shape)
        for i, (u, sc) in enumerate(prof.fit.shape):
            p.fit_shape_util[i] = u
            p.fit_shape_score[i] = sc * 10      # x MaxNodeScore / MaxCustomPriorityScore
    p.fit_ignored_scalar = fit_ignored_scalar(prof.fit, scal)
    p.fit_n_res = len(fr)
    for i, (r, w) in enumerate(fr):
        p.fit_res[i] = _res_id(r, scal)
        p.fit_res_weight[i] = w
    br = [(r, w) for r, w in prof.balanced.resources]
    p.ba_n_res = len(br)
    for i, (r, w) in enumerate(br):
        p.ba_res[i] = _res_id(r, scal)
        p.ba_res_weight[i] = w
    p.hard_pod_affinity_weight = prof.hard_pod_affinity_weight
    pa = prof.preemption
    if not (0 <= pa.min_candidate_nodes_percentage <= 100) or pa.min_candidate_nodes_absolute < 0 or \
            (pa.min_candidate_nodes_percentage == 0 and pa.min_candidate_nodes_absolute == 0):
        raise ValueError("DefaultPreemptionArgs: minCandidateNodesPercentage in [0, 100], "
                         "minCandidateNodesAbsolute >= 0, not both 0")
    p.preempt_min_pct = pa.min_candidate_nodes_percentage
    p.preempt_min_abs = pa.min_candidate_nodes_absolute
    p.tiebreak_seed = prof.tiebreak_seed & (2 ** 64 - 1)
    return p


def num_feasible_nodes_to_find(n: int, pct: int) -> int:
    """numFeasibleNodesToFind (upstream schedule_one.go): the
    feasible nodes a cycle keeps.  pct 0 is the adaptive default."""
    if n < 100 or pct >= 100:
        return n
    p = pct if pct > 0 else max(5, 50 - n // 125)
    return max(n * p // 100, 100)
