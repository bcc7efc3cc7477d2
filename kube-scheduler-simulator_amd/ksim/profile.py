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

from . import abi
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
    fr = [(r, w) for r, w in prof.fit.resources]
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
    p.tiebreak_seed = prof.tiebreak_seed & (2 ** 64 - 1)
    return p


def num_feasible_nodes_to_find(n: int, pct: int) -> int:
    """numFeasibleNodesToFind (upstream schedule_one.go): the
    feasible nodes a cycle keeps.  pct 0 is the adaptive default."""
    if n < 100 or pct >= 100:
        return n
    p = pct if pct > 0 else max(5, 50 - n // 125)
    return max(n * p // 100, 100)
