"""Engine-backed plugins behind the simulator's wrapper contract.

``record_cycle`` replays one engine cycle into a result Store exactly as the
simulator's wrappedPlugin records the original plugins during that cycle
(simulator/scheduler/plugin/wrappedplugin.go):

  PreFilter      -> AddPreFilterResult(plugin, "success"|msg, result)   :459-486
  Filter         -> AddFilterResult(node, plugin, "passed"|msg)          :491-516
                    (only plugins the framework ran: up to the first failure)
  PostFilter     -> AddPostFilterResult(nominated, plugin, nodes)        :518-544
  PreScore       -> AddPreScoreResult(plugin, "success"|msg)             :427-454
  Score          -> AddScoreResult(node, plugin, raw)                    :388-413
  NormalizeScore -> AddNormalizedScoreResult(node, plugin, normalized)   :356-383
  Reserve        -> AddSelectedNode(node) + AddReserveResult             :583-612
  PreBind/Bind   -> AddPreBindResult / AddBindResult
Keys are the ORIGINAL plugin names (wrappedplugin.go:374,406,447,479,510).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

from . import abi
from .encode import EncodedCluster
from .profile import SchedulerProfile, original_name
from .resultstore import PASSED_FILTER_MESSAGE, SUCCESS_MESSAGE, Store

# Plugins with a ScoreExtensions (NormalizeScore) in v1.26.
HAS_NORMALIZE = {"TaintToleration", "NodeAffinity", "PodTopologySpread", "InterPodAffinity", "NetworkBandwidth"}

# Upstream error reasons.
ERR_UNSCHEDULABLE = "node(s) were unschedulable"                        # nodeunschedulable
ERR_NODE_NAME = "node(s) didn't match the requested node name"          # nodename
ERR_NODE_AFFINITY = "node(s) didn't match Pod's node affinity/selector"  # nodeaffinity ErrReasonPod
ERR_NODE_AFFINITY_ENFORCED = "node(s) didn't match scheduler-enforced node affinity"   # errReasonEnforced
ERR_NODE_PORTS = "node(s) didn't have free ports for the requested pod ports"     # nodeports.ErrReason
ERR_PTS = "node(s) didn't match pod topology spread constraints"        # podtopologyspread ErrReasonConstraintsNotMatch
ERR_PTS_LABEL = ERR_PTS + " (missing required label)"                   # ErrReasonNodeLabelNotMatch
ERR_NODE_AFFINITY_CONFLICT = "pod affinity terms conflict"              # nodeaffinity errReasonConflict (PreFilter)
ERR_IPA = {abi.IPA_AFFINITY: "node(s) didn't match pod affinity rules",
           abi.IPA_ANTI_AFFINITY: "node(s) didn't match pod anti-affinity rules",
           abi.IPA_EXISTING_ANTI: "node(s) didn't satisfy existing pods anti-affinity rules"}


def filter_message(cluster: EncodedCluster, plugin: str, detail: int, node: str = "", pod: str = "") -> str:
    """framework.Status.Message() of a failing Filter (NetworkBandwidth's name
    the node and the pod)."""
    if plugin == "NetworkBandwidth":
        from .netbw import filter_message as nb_message
        return nb_message(detail, node, pod, cluster.nb_args)
    if plugin == "NodeUnschedulable":
        return ERR_UNSCHEDULABLE
    if plugin == "NodeName":
        return ERR_NODE_NAME
    if plugin == "TaintToleration":
        t = cluster.taint_vocab[detail]
        return f"node(s) had untolerated taint {{{t.key}: {t.value}}}"
    if plugin == "NodeAffinity":
        return ERR_NODE_AFFINITY_ENFORCED if detail == abi.NA_ENFORCED else ERR_NODE_AFFINITY
    if plugin == "NodePorts":
        return ERR_NODE_PORTS
    if plugin == "NodeResourcesFit":
        reasons = []
        if detail & abi.FIT_TOO_MANY_PODS:
            reasons.append("Too many pods")
        if detail & abi.FIT_CPU:
            reasons.append("Insufficient cpu")
        if detail & abi.FIT_MEMORY:
            reasons.append("Insufficient memory")
        if detail & abi.FIT_EPHEMERAL:
            reasons.append("Insufficient ephemeral-storage")
        for k, name in enumerate(cluster.scalar_names):
            if detail & (abi.FIT_SCALAR0 << k):
                reasons.append(f"Insufficient {name}")
        return ", ".join(reasons)
    if plugin == "PodTopologySpread":
        return ERR_PTS_LABEL if detail == abi.PTS_MISSING_LABEL else ERR_PTS
    if plugin == "InterPodAffinity":
        return ERR_IPA[detail]
    if plugin == "VolumeBinding":
        from .volumes import binding_message
        return binding_message(detail)
    if plugin == "VolumeZone":
        from .volumes import MSG_VOLUME_ZONE
        return MSG_VOLUME_ZONE
    return f"{plugin} failed"


def record_cycle(store: Store, cluster: EncodedCluster, prof: SchedulerProfile, ns: str, name: str,
                 res: Dict, prefilter_names: Optional[List[str]] = None, nominated: int = -1,
                 rejection: Optional[Tuple[str, str]] = None) -> None:
    """Feed ``store`` with one compat-mode cycle result (engine or oracle).
    ``prefilter_names``: the pod's NodeAffinity PreFilterResult.NodeNames
    (EncodedPods.prefilter_names; None = all nodes, [] = conflicting terms).
    ``nominated``: DefaultPreemption's nominated node of an unschedulable cycle
    (ksim_preempt; -1 none), which wrappedPlugin.PostFilter records as
    "preemption victim" (wrappedplugin.go:529-538, store.go:437-452).
    ``rejection``: (plugin, message) of a PreFilter that rejects the pod
    (EncodedPods.rejection: VolumeBinding's UnschedulableAndUnresolvable)."""
    names = cluster.node_names
    conflict = prefilter_names is not None and len(prefilter_names) == 0
    stopped = False
    for p in prof.plugins["preFilter"].enabled:
        plugin = original_name(p.name)
        if rejection is not None and plugin == rejection[0]:
            store.add_pre_filter_result(ns, name, plugin, rejection[1], None)
            stopped = True
            break                              # RunPreFilterPlugins stops at a failing plugin
        if plugin == "NodeAffinity" and prefilter_names is not None:
            # wrappedPlugin.PreFilter records the status and result.NodeNames.List()
            store.add_pre_filter_result(ns, name, plugin, ERR_NODE_AFFINITY_CONFLICT if conflict else SUCCESS_MESSAGE,
                                        None if conflict else list(prefilter_names))
            if conflict:
                stopped = True
                break
        else:
            store.add_pre_filter_result(ns, name, plugin, SUCCESS_MESSAGE, None)
    if stopped:
        # findNodesThatFitPod: every node gets the PreFilter status; no Filter runs
        for p in prof.plugins["postFilter"].enabled:
            store.add_post_filter_result(ns, name, "", original_name(p.name), list(names))
        return
    forder = prof.filter_order()
    fp, fd = res["fail_plugin"], res["fail_detail"]
    for node in range(cluster.n_nodes):
        r = int(fp[node])
        if r == abi.NOT_EVALUATED:
            continue
        last = len(forder) if r == abi.PASSED else r + 1
        for f in range(last):
            if f == r:
                store.add_filter_result(ns, name, names[node], forder[f],
                                        filter_message(cluster, forder[f], int(fd[node]), names[node], name))
            else:
                store.add_filter_result(ns, name, names[node], forder[f], PASSED_FILTER_MESSAGE)
    if res["status"] == abi.STATUS_ERROR:
        # framework.Error: a PreFilterResult node missing from the snapshot ends
        # the cycle before any Filter; a Filter error ends the scan; a Score
        # error ends the cycle after PreScore (which partial Score records
        # survive the cancelled parallel run is not deterministic upstream:
        # none are kept)
        if prefilter_names is not None and res["n_evaluated"] == 0:
            return
        filter_error = any(int(fp[i]) < len(forder) and forder[int(fp[i])] == "NetworkBandwidth" and
                           int(fd[i]) >= abi.NB_NO_LIMIT for i in range(cluster.n_nodes))
        if not filter_error:
            for p in prof.plugins["preScore"].enabled:
                store.add_pre_score_result(ns, name, original_name(p.name), SUCCESS_MESSAGE)
        return
    if res["status"] == abi.STATUS_UNSCHEDULABLE:
        failed = [names[i] for i in range(cluster.n_nodes) if fp[i] not in (abi.PASSED, abi.NOT_EVALUATED)]
        for p in prof.plugins["postFilter"].enabled:
            nom = names[nominated] if nominated >= 0 and original_name(p.name) == "DefaultPreemption" else ""
            store.add_post_filter_result(ns, name, nom, original_name(p.name), failed)
        return
    if res["n_feasible"] > 1:
        for p in prof.plugins["preScore"].enabled:
            store.add_pre_score_result(ns, name, original_name(p.name), SUCCESS_MESSAGE)
        scored = [i for i in range(cluster.n_nodes) if res["scored"][i]]
        splugins = prof.score_plugins()
        for i in scored:
            for k, pl in enumerate(splugins):
                store.add_score_result(ns, name, names[i], pl.name, int(res["raw"][k][i]))
        for k, pl in enumerate(splugins):
            if pl.name in HAS_NORMALIZE:
                for i in scored:
                    store.add_normalized_score_result(ns, name, names[i], pl.name, int(res["norm"][k][i]))
    chosen = names[res["chosen"]]
    for p in prof.plugins["reserve"].enabled:
        store.add_selected_node(ns, name, chosen)
        store.add_reserve_result(ns, name, original_name(p.name), SUCCESS_MESSAGE)
    for p in prof.plugins["preBind"].enabled:
        store.add_pre_bind_result(ns, name, original_name(p.name), SUCCESS_MESSAGE)
    for p in prof.plugins["bind"].enabled:
        store.add_bind_result(ns, name, original_name(p.name), SUCCESS_MESSAGE)


def compat_cycle(backend, store: Store, cluster: EncodedCluster, prof: SchedulerProfile, pods, index: int,
                 priority: int = 0, bound=None) -> Dict:
    """One deterministic compat cycle as the wrapped plugins see it: the cycle
    (ksim_eval_pod), then for an unschedulable pod DefaultPreemption's
    PostFilter dry run (ksim_preempt over the bound-pod table set with
    set_bound_pods) when the profile enables it, recorded into ``store``.
    ``backend`` is an Engine (or the oracle, whose preempt takes ``bound``)."""
    res = backend.eval_pod(pods, index) if hasattr(backend, "eval_pod") else backend.cycle(pods, index)
    nominated = -1
    post = [original_name(p.name) for p in prof.plugins["postFilter"].enabled]
    if res["status"] == abi.STATUS_UNSCHEDULABLE and "DefaultPreemption" in post and pods.rejection(index) is None:
        names = pods.prefilter_names[index] if pods.prefilter_names else None
        if not (names is not None and len(names) == 0):
            out = backend.preempt(pods, index, priority) if bound is None else \
                backend.preempt(pods, index, priority, bound)
            nominated = int(out[0])
    res["nominated"] = nominated
    ns, name = pods.names[index]
    record_cycle(store, cluster, prof, ns, name, res,
                 pods.prefilter_names[index] if pods.prefilter_names else None, nominated, pods.rejection(index))
    return res


def emit_cycle_annotations(cluster: EncodedCluster, prof: SchedulerProfile, res: Dict,
                           score_plugin_weight: Dict[str, int], pod_name: str = "") -> Dict[str, str]:
    """The three large annotation values of one cycle from the native emitter
    (ksim_emit_cycle_json): what record_cycle + Store.add_stored_result_to_pod
    produce for them, without building the maps."""
    import numpy as np
    from . import engine
    from .resultstore import FILTER_RESULT, FINALSCORE_RESULT, SCORE_RESULT
    forder = prof.filter_order()
    fp = np.asarray(res["fail_plugin"], np.uint8)
    fd = np.asarray(res["fail_detail"])
    failed = (fp != abi.PASSED) & (fp != abi.NOT_EVALUATED)
    names = cluster.node_names
    # one message per (plugin, detail); NetworkBandwidth's also name the node
    keys = [(int(fp[i]), int(fd[i]), names[i] if int(fp[i]) < len(forder) and forder[fp[i]] == "NetworkBandwidth" else "")
            for i in np.nonzero(failed)[0]]
    pairs = sorted(set(keys))
    index = {pr: k for k, pr in enumerate(pairs)}
    messages = [filter_message(cluster, forder[a], b, nd, pod_name) for a, b, nd in pairs]
    msg_id = np.zeros(cluster.n_nodes, np.int32)
    for i, key in zip(np.nonzero(failed)[0], keys):
        msg_id[i] = index[key]
    splugins = prof.score_plugins()
    snames = [p.name for p in splugins]
    scored = np.asarray(res["scored"], np.uint8) if res["n_feasible"] > 1 else np.zeros(cluster.n_nodes, np.uint8)
    if res["status"] in (abi.STATUS_UNSCHEDULABLE, abi.STATUS_ERROR):
        scored = np.zeros(cluster.n_nodes, np.uint8)
    raw = np.asarray(res["raw"], np.int64).reshape(len(snames), cluster.n_nodes) if snames else \
        np.zeros((0, cluster.n_nodes), np.int64)
    norm = np.asarray(res["norm"], np.int64).reshape(len(snames), cluster.n_nodes) if snames else raw
    f, s, g = engine.emit_cycle_json(
        cluster.node_names, forder, snames, [int(score_plugin_weight.get(n, 0)) for n in snames],
        [1 if n in HAS_NORMALIZE else 0 for n in snames], fp, msg_id, messages, scored, raw, norm)
    return {FILTER_RESULT: f, SCORE_RESULT: s, FINALSCORE_RESULT: g}
