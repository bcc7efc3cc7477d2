"""NetworkBandwidth, the simulator's out-of-tree plugin (SURVEY §8(f) 4;
simulator/scheduler/plugin/networkbandwidth/plugin.go).

CPU side: the host's quantity / annotation handling, the encoder's node and
pod columns, and the C oracle against the object-level restatement (which
sums the nodes' allocated amounts from their pods with exact Fractions, as
getNodeAllocatedAmount does), cycle by cycle, including the cycles that fail
with framework.Error.  The GPU engine is checked against the oracle in
tests/test_gpu_parity.py.

Parity unpinned against Go: the reference ships no test for this plugin; the
expected values follow plugin.go and upstream v1.26 RunFilterPlugins /
RunScorePlugins status handling.
"""
import numpy as np
import pytest

from ksim import abi, gen, netbw, profile
from ksim.encode import EncodeError, encode_cluster, encode_pods
from ksim.model import Node, Pod
from ksim.profile import Plugin, PluginSet, SchedulerProfile, convert_for_simulator
from ksim.wrapped import filter_message
from oracle.objref import ObjScheduler
from oracle.oracle import Oracle


def nb_profile(pct=0, filt=True, score=True, weight=3) -> SchedulerProfile:
    """A profile enabling NetworkBandwidth as a user config does (merged after the in-tree plugins)."""
    user = {}
    if filt:
        user["filter"] = PluginSet([Plugin("NetworkBandwidth")])
    if score:
        user["score"] = PluginSet([Plugin("NetworkBandwidth", weight)])
    return SchedulerProfile(plugins=convert_for_simulator(user), percentage_of_nodes_to_score=pct)


@pytest.mark.parametrize("s,want", [
    ("10G", 10 ** 13), ("1Gi", 2 ** 30 * 1000), ("1500m", 1500), ("0.5G", 5 * 10 ** 11), ("1e8", 10 ** 11),
    ("+2k", 2 * 10 ** 6), (".5", 500), ("5.", 5000), ("-3M", -3 * 10 ** 9), ("0", 0),
    ("abc", None), ("", None), (" 1G", None), ("1G ", None), ("1GB", None), ("1e", None), ("--1", None)])
def test_quantity_milli(s, want):
    assert netbw.milli(s) == want


@pytest.mark.parametrize("s", ["1u", "1n", "0.0001"])
def test_quantity_finer_than_milli_refused(s):
    with pytest.raises(netbw.QuantityError):
        netbw.milli(s)


def test_pod_request_fallbacks_and_allocated_share():
    a = netbw.NetworkBandwidthArgs()
    ann = {netbw.INGRESS_BANDWIDTH: "100M", a.egress_request_annotation: "50M"}
    assert netbw.pod_request(ann, a) == (0, 150 * 10 ** 9)
    assert netbw.pod_allocated(ann, a) == 50 * 10 ** 9        # the fallback is not an allocated amount
    ann = {a.ingress_request_annotation: "1M", netbw.INGRESS_BANDWIDTH: "9M"}
    assert netbw.pod_request(ann, a) == (0, 10 ** 9)          # the request annotation wins
    assert netbw.pod_request({a.ingress_request_annotation: "x"}, a)[0] == abi.POD_NB_INGRESS_BAD
    assert netbw.pod_request({netbw.EGRESS_BANDWIDTH: "x"}, a)[0] == abi.POD_NB_EGRESS_BAD
    assert netbw.pod_allocated({a.ingress_request_annotation: "x", a.egress_request_annotation: "2"}, a) == 2000
    assert netbw.pod_request({}, a) == (0, 0)


def test_args_from_config_keep_defaults():
    a = netbw.NetworkBandwidthArgs.from_config({"nodeLimitAnnotation": "example.com/limit"})
    assert a.node_limit_annotation == "example.com/limit"
    assert a.ingress_request_annotation == "kubernetes.io/ingress-request"
    assert a.egress_request_annotation == "kubernetes.io/egress-request"


def test_encoder_columns():
    a = netbw.NetworkBandwidthArgs()
    nodes = [Node("n0", annotations={a.node_limit_annotation: "1G"}), Node("n1"),
             Node("n2", annotations={a.node_limit_annotation: "fast"})]
    for n in nodes:
        n.allocatable = {"cpu": "4", "memory": "8Gi", "pods": "10"}
    bound = [Pod("b0", node_name="n0", annotations={a.ingress_request_annotation: "100M",
                                                      a.egress_request_annotation: "?",
                                                      netbw.EGRESS_BANDWIDTH: "7M"}),
             Pod("b1", node_name="n0", annotations={a.egress_request_annotation: "1500m"})]
    c, order = encode_cluster(nodes, bound)
    pos = {n: i for i, n in enumerate(c.node_names)}
    assert c.flags[pos["n0"]] == abi.NODE_NB_LIMIT and c.nb_limit[pos["n0"]] == 10 ** 12
    assert c.flags[pos["n1"]] == 0
    assert c.flags[pos["n2"]] == abi.NODE_NB_LIMIT | abi.NODE_NB_LIMIT_BAD
    assert c.nb_alloc[pos["n0"]] == 10 ** 11 + 1500
    pods = encode_pods(c, [Pod("p", annotations={netbw.INGRESS_BANDWIDTH: "2M", a.egress_request_annotation: "3M"})])
    rec = pods.pods[0]
    assert (rec["nb_flags"], rec["nb_req"], rec["nb_add"]) == (0, 5 * 10 ** 9, 3 * 10 ** 9)
    with pytest.raises(EncodeError):
        encode_pods(c, [Pod("q", annotations={a.ingress_request_annotation: "1n"})])


def test_profile_compiles_network_bandwidth_last():
    sp = nb_profile(weight=4)
    assert sp.filter_order()[-1] == "NetworkBandwidth"
    p = profile.compile_profile(sp)
    assert p.filter[p.n_filter - 1] == abi.PL_NETWORK_BANDWIDTH
    assert p.score[p.n_score - 1] == abi.PL_NETWORK_BANDWIDTH and p.score_weight[p.n_score - 1] == 4


def run_both(nodes, bound, pending, sp, filt=True, score=True, weight=3):
    cluster, _ = encode_cluster(nodes, bound, nb_args=sp.network_bandwidth)
    enc = encode_pods(cluster, pending)
    ora = Oracle(cluster, profile.compile_profile(sp))
    w = {p.name: p.weight for p in sp.score_plugins()}
    ref = ObjScheduler(nodes, bound, pct=sp.percentage_of_nodes_to_score, seed=sp.tiebreak_seed,
                       network_bandwidth=sp.network_bandwidth, nb_filter=filt, nb_score=score, weights=w)
    forder = sp.filter_order()
    snames = [p.name for p in sp.score_plugins()]
    names = cluster.node_names
    stats = {"scheduled": 0, "unschedulable": 0, "error": 0, "insufficient": 0}
    for i, pod in enumerate(pending):
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
                got = filter_message(cluster, forder[fp], int(o["fail_detail"][pos]), name, pod.name)
                assert got == msg, (where, name)
                stats["insufficient"] += pl == "NetworkBandwidth" and int(o["fail_detail"][pos]) == abi.NB_INSUFFICIENT
        assert o["n_feasible"] == r["n_feasible"], where
        assert (o["status"] == abi.STATUS_ERROR) == (r["error"] is not None), where
        if o["status"] == abi.STATUS_ERROR:
            assert o["chosen"] == abi.CHOSEN_ERROR
            stats["error"] += 1
        elif o["n_feasible"] > 1:
            for k, pl in enumerate(snames):
                for pos in np.nonzero(o["scored"])[0]:
                    nm = names[pos]
                    assert o["raw"][k][pos] == r["raw"][pl][nm], f"{where}: raw {pl} on {nm}"
                    assert o["norm"][k][pos] == r["norm"][pl][nm], f"{where}: norm {pl} on {nm}"
            for pos in np.nonzero(o["scored"])[0]:
                assert o["total"][pos] == r["total"][names[pos]], where
        got = names[o["chosen"]] if o["chosen"] >= 0 else None
        assert got == r["chosen"], f"{where}: oracle {got} objref {r['chosen']}"
        if o["status"] != abi.STATUS_ERROR:
            stats["scheduled" if got else "unschedulable"] += 1
        assert ora.next_start == ref.next_start, where
    alloc = ora.nb_alloc()
    for pos, name in enumerate(names):
        ni = ref.by_name[name]
        assert alloc[pos] == int(ref._nb_allocated(ni) * 1000), name
    return stats


@pytest.mark.parametrize("pct", [0, 100])
def test_clean_cluster_vs_objref(pct):
    nodes, bound, pending = gen.netbw_objects(n_nodes=120, n_pods=500)
    st = run_both(nodes, bound, pending, nb_profile(pct))
    assert st["scheduled"] > 100 and st["insufficient"] > 0 and st["error"] == 0


@pytest.mark.parametrize("pct", [0, 100])
def test_error_statuses_vs_objref(pct):
    nodes, bound, pending = gen.netbw_objects(n_nodes=120, n_pods=250, node_errors=True, pod_errors=True)
    st = run_both(nodes, bound, pending, nb_profile(pct))
    assert st["error"] > 0 and st["scheduled"] > 0


def test_score_only_and_filter_only_vs_objref():
    nodes, bound, pending = gen.netbw_objects(n_nodes=110, n_pods=150, node_errors=True)
    st = run_both(nodes, bound, pending, nb_profile(0, filt=False), filt=False)
    assert st["error"] > 0                              # kept nodes without a limit fail Score
    nodes, bound, pending = gen.netbw_objects(n_nodes=110, n_pods=150, pod_errors=True)
    st = run_both(nodes, bound, pending, nb_profile(100, score=False), score=False)
    assert st["error"] > 0 and st["scheduled"] > 0


def test_oracle_timing_mode_matches_cycles():
    nodes, bound, pending = gen.netbw_objects(n_nodes=120, n_pods=200, node_errors=True, pod_errors=True)
    sp = nb_profile(0)
    cluster, _ = encode_cluster(nodes, bound, nb_args=sp.network_bandwidth)
    enc = encode_pods(cluster, pending)
    a = Oracle(cluster, profile.compile_profile(sp))
    want = np.array([a.cycle(enc, i)["chosen"] for i in range(enc.n_pods)], np.int32)
    b = Oracle(cluster, profile.compile_profile(sp))
    got, st = b.schedule(enc, nthreads=4)
    assert np.array_equal(got, want)
    assert (want == abi.CHOSEN_ERROR).any()
    assert np.array_equal(a.nb_alloc(), b.nb_alloc()) and a.next_start == b.next_start
