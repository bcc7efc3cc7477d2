"""DefaultPreemption PostFilter: the C oracle's dry run
(ksim_oracle_preempt) against the object-level restatement (oracle/objref.py
ObjScheduler.preempt) on crowded clusters with mixed priorities."""
import numpy as np
import pytest

from ksim import gen
from ksim.encode import encode_cluster, encode_pods
from ksim.model import Container, Pod
from ksim.preemption import bound_table
from ksim import profile
from oracle.objref import ObjScheduler
from oracle.oracle import Oracle


def crowded(n_nodes=40, per_node=6, seed=3):
    """Config-1 nodes, each holding bound pods of mixed priorities and start times."""
    rng = np.random.default_rng(seed)
    nodes, _ = gen.config1_objects(n_nodes=n_nodes, n_pods=1)
    bound, start, order = [], {}, {}
    for ni, n in enumerate(nodes):
        for k in range(per_node):
            name = f"b{ni}-{k}"
            p = Pod(name, node_name=n.name, priority=int(rng.choice([0, 10, 100, 1000])),
                    containers=[Container({"cpu": f"{int(rng.integers(2, 12)) * 100}m",
                                           "memory": f"{int(rng.integers(1, 6))}Gi"})])
            bound.append(p)
            start[name] = int(rng.integers(0, 50))       # ties on purpose
            order[name] = len(order)
    return nodes, bound, start, order


@pytest.mark.parametrize("seed", [3, 4, 5])
def test_preempt_oracle_vs_objref(seed):
    nodes, bound, start, order = crowded(seed=seed)
    cluster, _ = encode_cluster(nodes, bound)
    table = bound_table(cluster, bound, start)
    rng = np.random.default_rng(seed + 100)
    pods = [Pod(f"p{i}", priority=int(rng.choice([0, 5, 50, 500, 5000])),
                containers=[Container({"cpu": f"{int(rng.integers(10, 400)) * 100}m",
                                       "memory": f"{int(rng.integers(4, 40))}Gi"})]) for i in range(30)]
    enc = encode_pods(cluster, pods)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=100)
    ora = Oracle(cluster, profile.compile_profile(sp))
    ref = ObjScheduler(nodes, bound, pct=100, seed=sp.tiebreak_seed)
    nominated = 0
    for i, pod in enumerate(pods):
        node, victims, n_pot, n_cand = ora.preempt(enc, i, pod.priority, table)
        rnode, rvictims = ref.preempt(pod, pod.priority, start, order)
        got = cluster.node_names[node] if node >= 0 else None
        assert got == rnode, f"pod {i}"
        assert [bound[v].name for v in victims] == rvictims, f"pod {i}"
        nominated += node >= 0
    assert 0 < nominated < len(pods)


def test_postfilter_records_nominated_node():
    """wrappedPlugin.PostFilter records the nominated node of DefaultPreemption
    as "preemption victim" and "" otherwise (wrappedplugin.go:529-538,
    store.go:437-452): compat_cycle feeds ksim_preempt's pick into the store."""
    import json
    from ksim.resultstore import POSTFILTER_RESULT, POST_FILTER_NOMINATED_MESSAGE, Store
    from ksim.wrapped import compat_cycle
    nodes, bound, start, order = crowded(seed=4)
    cluster, _ = encode_cluster(nodes, bound)
    table = bound_table(cluster, bound, start)
    rng = np.random.default_rng(104)
    pods = [Pod(f"p{i}", priority=int(rng.choice([0, 5, 50, 500, 5000])),
                containers=[Container({"cpu": f"{int(rng.integers(10, 400)) * 100}m",
                                       "memory": f"{int(rng.integers(4, 40))}Gi"})]) for i in range(30)]
    enc = encode_pods(cluster, pods)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=100)
    ora = Oracle(cluster, profile.compile_profile(sp))
    ref = Oracle(cluster.copy_state(), profile.compile_profile(sp))
    store = Store(profile.default_score_weights())
    seen = 0
    for i, pod in enumerate(pods):
        res = compat_cycle(ora, store, cluster, sp, enc, i, pod.priority, table)
        ann = {}
        store.add_stored_result_to_pod(*enc.names[i], ann)
        if res["status"] != 1:
            ref.cycle(enc, i)
            continue
        want, _, _, _ = ref.preempt(enc, i, pod.priority, table)
        ref.cycle(enc, i)
        assert res["nominated"] == want
        post = json.loads(ann[POSTFILTER_RESULT])
        marked = [n for n, v in post.items() if v.get("DefaultPreemption") == POST_FILTER_NOMINATED_MESSAGE]
        assert marked == ([cluster.node_names[want]] if want >= 0 else [])
        seen += want >= 0
    assert seen > 0
