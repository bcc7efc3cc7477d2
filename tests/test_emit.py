"""Native result emission: ksim_emit_cycle_json against the
result-store mirror (ksim/wrapped.py record_cycle + ksim/resultstore.py, the
restatement of store.go's maps and encoding/json), cycle by cycle on oracle
outputs.  Host code only: runs without a GPU."""
import pytest

from ksim import abi, gen, profile
from ksim.resultstore import FILTER_RESULT, FINALSCORE_RESULT, SCORE_RESULT, Store
from ksim.wrapped import emit_cycle_annotations, record_cycle
from oracle.oracle import Oracle


def _check(cluster, pods, pct, n=None):
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=pct)
    weights = profile.default_score_weights()
    ora = Oracle(cluster, profile.compile_profile(sp))
    seen = set()
    for i in range(pods.n_pods if n is None else n):
        res = ora.cycle(pods, i)
        store = Store(weights)
        ns, name = pods.names[i] if pods.names else ("default", f"p{i}")
        record_cycle(store, cluster, sp, ns, name, res)
        want = {}
        store.add_stored_result_to_pod(ns, name, want)
        got = emit_cycle_annotations(cluster, sp, res, weights)
        for k in (FILTER_RESULT, SCORE_RESULT, FINALSCORE_RESULT):
            assert got[k] == want[k], f"pod {i} {k}"
        seen.add(int(res["status"]))
    return seen


@pytest.mark.parametrize("pct", [0, 100])
def test_emit_config1(pct):
    cluster, pods = gen.config1()
    _check(cluster, pods, pct, n=300)


def test_emit_config3_topology_messages():
    cluster, pods = gen.config3(n_nodes=120, pods_per_node=10, n_incoming=150, seed=5, zone_anti_every=20)
    _check(cluster, pods, 0)


def test_emit_unschedulable_and_escaping():
    """Pods that fit nowhere (every node records a reason) and a node name that
    needs JSON escaping."""
    cluster, pods = gen.config1(n_nodes=100, n_pods=1)
    cluster.node_names = list(cluster.node_names)
    cluster.node_names[3] = "n<&>\\\"x"
    pods.pods["req_cpu"][0] = 10 ** 9
    seen = _check(cluster, pods, 100)
    assert abi.STATUS_UNSCHEDULABLE in seen
