"""Restated contract tests of the simulator's profile handling.

Sources (reference tests restated against the host mirror, same inputs and
expected values):
  * converted default profile, plugin order and weights — simulator/scheduler/scheduler_test.go:380-437
  * ConvertForSimulator cases — simulator/scheduler/plugin/plugins_test.go:14-548
  * registered plugins — plugins_test.go:852-899 (the fork appends NetworkBandwidth,
    simulator/scheduler/config/plugin.go:214-221,266-273, so that test is stale
    as written; here the fork's actual list is asserted)
  * store default weights — simulator/scheduler/plugin/plugins.go:22-34
"""
from ksim import abi
from ksim.profile import (Plugin, PluginSet, SchedulerProfile, all_registered_plugins,
                          compile_profile, convert_for_simulator, default_score_weights,
                          merge_plugin_set)


def names(ps):
    return [(p.name, p.weight) for p in ps.enabled]


def test_converted_default_profile_matches_scheduler_test():
    got = convert_for_simulator(None)
    assert names(got["preFilter"]) == [(n + "Wrapped", None) for n in [
        "NodeResourcesFit", "NodePorts", "VolumeRestrictions", "PodTopologySpread",
        "InterPodAffinity", "VolumeBinding", "NodeAffinity"]]
    assert names(got["filter"]) == [(n + "Wrapped", None) for n in [
        "NodeUnschedulable", "NodeName", "TaintToleration", "NodeAffinity", "NodePorts",
        "NodeResourcesFit", "VolumeRestrictions", "EBSLimits", "GCEPDLimits", "NodeVolumeLimits",
        "AzureDiskLimits", "VolumeBinding", "VolumeZone", "PodTopologySpread", "InterPodAffinity"]]
    assert names(got["postFilter"]) == [("DefaultPreemptionWrapped", None)]
    assert names(got["reserve"]) == [("VolumeBindingWrapped", None)]
    assert names(got["preBind"]) == [("VolumeBindingWrapped", None)]
    assert names(got["bind"]) == [("DefaultBinderWrapped", None)]
    assert names(got["preScore"]) == [(n + "Wrapped", None) for n in [
        "InterPodAffinity", "PodTopologySpread", "TaintToleration", "NodeAffinity"]]
    assert names(got["score"]) == [
        ("NodeResourcesBalancedAllocationWrapped", 1), ("ImageLocalityWrapped", 1),
        ("InterPodAffinityWrapped", 1), ("NodeResourcesFitWrapped", 1),
        ("NodeAffinityWrapped", 1), ("PodTopologySpreadWrapped", 2),
        ("TaintTolerationWrapped", 1)]
    for ext, ps in got.items():
        assert [p.name for p in ps.disabled] == ["*"], ext


def test_convert_for_simulator_disable_most_plugins():
    """plugins_test.go:26-198 'success'."""
    star = PluginSet([], [Plugin("*")])
    arg = {
        "preFilter": star, "preScore": star, "reserve": star, "permit": star, "preBind": star,
        "bind": star, "postBind": star,
        "filter": PluginSet([], [Plugin(n) for n in [
            "EBSLimits", "NodeUnschedulable", "NodeName", "TaintToleration", "NodeAffinity",
            "GCEPDLimits", "NodeVolumeLimits", "AzureDiskLimits", "VolumeBinding", "VolumeZone",
            "NodePorts", "NodeResourcesFit", "VolumeRestrictions"]]),
        "postFilter": PluginSet([], [Plugin("DefaultPreemption")]),
        "score": PluginSet([], [Plugin(n) for n in [
            "NodeResourcesFit", "NodeResourcesBalancedAllocation", "ImageLocality",
            "InterPodAffinity", "NodeAffinity"]]),
    }
    got = convert_for_simulator(arg)
    for ext in ("preFilter", "preScore", "reserve", "permit", "preBind", "bind", "postBind",
                "postFilter"):
        assert names(got[ext]) == [], ext
    assert names(got["filter"]) == [("PodTopologySpreadWrapped", None), ("InterPodAffinityWrapped", None)]
    assert names(got["score"]) == [("PodTopologySpreadWrapped", 2), ("TaintTolerationWrapped", 1)]


def test_convert_for_simulator_non_in_tree_plugins():
    """plugins_test.go:359-548 'success with non in-tree plugins'."""
    star = PluginSet([], [Plugin("*")])
    arg = {
        "preFilter": star, "preScore": star, "reserve": star, "permit": star, "preBind": star,
        "bind": star, "postBind": star,
        "filter": PluginSet([Plugin("CustomPlugin1")], [Plugin("*")]),
        "postFilter": PluginSet([Plugin("CustomPlugin1")], [Plugin("*")]),
        "score": PluginSet([Plugin("CustomPlugin1")], [Plugin(n) for n in [
            "NodeResourcesFit", "NodeResourcesBalancedAllocation", "ImageLocality",
            "InterPodAffinity", "NodeAffinity"]]),
    }
    got = convert_for_simulator(arg)
    assert names(got["filter"]) == [("CustomPlugin1Wrapped", None)]
    assert names(got["postFilter"]) == [("CustomPlugin1Wrapped", None)]
    assert names(got["score"]) == [("PodTopologySpreadWrapped", 2), ("TaintTolerationWrapped", 1),
                                   ("CustomPlugin1Wrapped", None)]


def test_merge_plugin_set_replaces_in_place():
    """A re-configured default plugin keeps its position (mergePluginSet)."""
    base = PluginSet([Plugin("A", 1), Plugin("B", 1), Plugin("C", 1)])
    user = PluginSet([Plugin("X", 3), Plugin("B", 5)], [Plugin("C")])
    got = merge_plugin_set(base, user)
    assert [(p.name, p.weight) for p in got.enabled] == [("A", 1), ("B", 5), ("X", 3)]


def test_registered_plugins_and_default_weights():
    got = [(p.name, p.weight) for p in all_registered_plugins()]
    assert got == [
        ("NodeResourcesBalancedAllocation", 1), ("ImageLocality", 1), ("InterPodAffinity", 1),
        ("NodeResourcesFit", 1), ("NodeAffinity", 1), ("PodTopologySpread", 2),
        ("TaintToleration", 1), ("NetworkBandwidth", None), ("DefaultBinder", None),
        ("VolumeBinding", None), ("NodePorts", None), ("VolumeRestrictions", None),
        ("NodeUnschedulable", None), ("NodeName", None), ("EBSLimits", None),
        ("GCEPDLimits", None), ("NodeVolumeLimits", None), ("AzureDiskLimits", None),
        ("VolumeZone", None), ("DefaultPreemption", None)]
    assert default_score_weights() == {
        "NodeResourcesBalancedAllocation": 1, "ImageLocality": 1, "InterPodAffinity": 1,
        "NodeResourcesFit": 1, "NodeAffinity": 1, "PodTopologySpread": 2, "TaintToleration": 1,
        "NetworkBandwidth": 0}


def test_compile_profile_default():
    p = compile_profile(SchedulerProfile())
    assert [abi.PLUGINS[x] for x in p.filter[:p.n_filter]] == SchedulerProfile().filter_order()
    assert [abi.PLUGINS[x] for x in p.score[:p.n_score]] == [
        "NodeResourcesBalancedAllocation", "ImageLocality", "InterPodAffinity", "NodeResourcesFit",
        "NodeAffinity", "PodTopologySpread", "TaintToleration"]
    assert list(p.score_weight[:p.n_score]) == [1, 1, 1, 1, 1, 2, 1]
    assert p.percentage_of_nodes_to_score == 0          # simulator forces the default
    assert (p.fit_n_res, list(p.fit_res[:2]), list(p.fit_res_weight[:2])) == (2, [0, 1], [1, 1])
    assert (p.ba_n_res, list(p.ba_res[:2]), list(p.ba_res_weight[:2])) == (2, [0, 1], [1, 1])
    assert p.hard_pod_affinity_weight == 1


def test_with_weights_sweep_vector():
    sp = SchedulerProfile().with_weights({"PodTopologySpread": 7, "NodeResourcesFit": 3})
    p = compile_profile(sp)
    assert list(p.score_weight[:p.n_score]) == [1, 1, 1, 3, 1, 7, 1]
