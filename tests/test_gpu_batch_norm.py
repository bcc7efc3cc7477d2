"""The P100 batch path for pods whose normalized scores vary over nodes
(kPodNormVaries: PreferNoSchedule taints the pod does not tolerate, preferred
node affinity; ksim_batch.hip k_batch_top / pairs_block, ksim_engine.cpp
pod_batchable) and for pods with scalar requests, against the one-by-one
oracle.  The keys carry the pod's TaintToleration / NodeAffinity scores
normalized over its S0 maxima (DefaultNormalizeScore, the reverse form for
TaintToleration: /root/reference/simulator/scheduler/plugin/wrappedplugin.go
runs the upstream plugins' NormalizeScore over the scored list); a batch ends
before a pod one of whose maxima holders stopped fitting."""
import numpy as np
import pytest

from ksim import gen, profile
from ksim.encode import encode_cluster, encode_pods
from ksim.engine import Engine
from ksim.model import Container, Node, NodeSelectorTerm, Pod, PreferredTerm, Requirement, Taint
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu


def _run(cluster, pods, pct=100, weights=None):
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=pct)
    if weights:
        sp = sp.with_weights(weights)
    prof = profile.compile_profile(sp)
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(cluster)
    chosen, st = eng.schedule_batch(pods)
    ora = Oracle(cluster, prof)
    ochosen, ost = ora.schedule(pods, nthreads=8)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals and st.scheduled == ost.scheduled
    assert eng.next_start == ora.next_start
    es, os_ = eng.node_state(), ora.node_state()
    for k in es:
        np.testing.assert_array_equal(es[k], os_[k], err_msg=k)
    return st


@pytest.mark.parametrize("n_nodes,n_pods", [(100, 1000), (1200, 4000), (5000, 6000)])
def test_config1_distribution_batched(n_nodes, n_pods):
    """Config 1's objects (taints incl. PreferNoSchedule, tolerations, required
    and preferred node affinity), scaled: every pod on the batch path."""
    nodes, pods = gen.config1_objects(n_nodes=n_nodes, n_pods=n_pods)
    cluster, _ = encode_cluster(nodes)
    st = _run(cluster, encode_pods(cluster, pods))
    assert st.perpod_cycles == 0 and st.batches > 0


@pytest.mark.parametrize("n_nodes,n_pods", [(400, 1500), (1200, 4000), (3000, 6000)])
def test_config1_distribution_adapt_batched(n_nodes, n_pods):
    """ADAPT (K < N), the simulator's own mode: the varying-normalization pods
    (on config 1's distribution nearly every pod varies: 20 % of the nodes
    carry a PreferNoSchedule taint, 30 % of the pods prefer node labels) take
    the ADAPT batch path, their keys normalized over the window's kept nodes
    (ksim_adapt.hip k_adapt_top), a kept node that stops fitting ending the
    batch (k_adapt_pairs)."""
    nodes, pods = gen.config1_objects(n_nodes=n_nodes, n_pods=n_pods)
    cluster, _ = encode_cluster(nodes)
    st = _run(cluster, encode_pods(cluster, pods), pct=0)
    assert st.perpod_cycles == 0 and st.batches > 0


def _holder_cluster(n_nodes, n_small, big_weight):
    """Most nodes roomy and plain; a few small nodes are the only ones labeled
    disk=ssd (the preferred-affinity maximum) and the only ones without the
    PreferNoSchedule taint most pods do not tolerate (the reverse maximum is
    held by the rest).  The small nodes fill up inside batches."""
    nodes = []
    for i in range(n_nodes):
        small = i % (n_nodes // n_small) == 0
        nodes.append(Node(
            name=f"n{i:05d}",
            labels={"kubernetes.io/hostname": f"n{i:05d}", "disk": "ssd" if small else "hdd",
                    "pool": "a" if i % 2 else "b"},
            taints=[] if small else [Taint("spot", "true", "PreferNoSchedule")],
            allocatable={"cpu": "2" if small else "64", "memory": "4Gi" if small else "256Gi", "pods": "110"}))
    rng = np.random.default_rng(7)
    pods = []
    for j in range(3000):
        p = Pod(f"p{j:05d}", containers=[Container({"cpu": f"{int(rng.integers(2, 9)) * 100}m",
                                                    "memory": f"{int(rng.integers(1, 5)) * 256}Mi"})])
        if j % 3:
            p.preferred_terms = [PreferredTerm(big_weight, NodeSelectorTerm([Requirement("disk", "In", ["ssd"])])),
                                 PreferredTerm(7, NodeSelectorTerm([Requirement("pool", "In", ["a"])]))]
        pods.append(p)
    return nodes, pods


@pytest.mark.parametrize("n_nodes,n_small", [(300, 30), (2000, 8)])
def test_maxima_holders_fill_up(n_nodes, n_small):
    """The nodes holding a pod's NodeAffinity maximum stop fitting inside a
    batch: the batch must end before the pod (pinv) and the next batch
    re-normalizes; placements stay the oracle's."""
    nodes, pods = _holder_cluster(n_nodes, n_small, big_weight=100)
    cluster, _ = encode_cluster(nodes)
    st = _run(cluster, encode_pods(cluster, pods))
    assert st.perpod_cycles == 0
    assert st.truncations > 0


def test_weights_and_key_bound():
    """Heavy TaintToleration / NodeAffinity weights (still inside the 20-bit
    key field) and past it (the pods fall back to the per-pod path)."""
    nodes, pods = gen.config1_objects(n_nodes=600, n_pods=1500)
    cluster, _ = encode_cluster(nodes)
    enc = encode_pods(cluster, pods)
    st = _run(cluster, enc, weights={"TaintToleration": 4000, "NodeAffinity": 3000})
    assert st.perpod_cycles == 0
    st = _run(cluster, enc, weights={"TaintToleration": 6000, "NodeAffinity": 5000})
    assert st.perpod_cycles > 0


def test_scalar_requests_batched():
    """Pods requesting an extended resource (scalar columns: Fit filter and
    LeastAllocated over cpu / memory) on the P100 batch path."""
    rng = np.random.default_rng(3)
    nodes = [Node(name=f"g{i:04d}", labels={"kubernetes.io/hostname": f"g{i:04d}"},
                  allocatable={"cpu": "32", "memory": "128Gi", "pods": "110",
                               "example.com/gpu": str(int(rng.integers(0, 5)))}) for i in range(700)]
    pods = []
    for j in range(2500):
        req = {"cpu": f"{int(rng.integers(1, 8)) * 250}m", "memory": f"{int(rng.integers(1, 8))}Gi"}
        if j % 2:
            req["example.com/gpu"] = str(int(rng.integers(1, 3)))
        pods.append(Pod(f"s{j:05d}", containers=[Container(req)]))
    cluster, _ = encode_cluster(nodes)
    st = _run(cluster, encode_pods(cluster, pods))
    assert st.perpod_cycles == 0 and st.unschedulable > 0
