"""Framework-driven compat mode on the CPU (oracle side): the framework mirror
(tests/fwmirror.py) driving the oracle's ksim_oracle_fw_* answers.

* With parallelism 1 and the TB tie-break the framework's choices are the
  engine's deterministic ones, so the cycle must equal ksim_oracle_cycle's:
  placements, nextStartNodeIndex, the node state and every annotation.
* With 16 racing workers and reservoir ties the framework's bookkeeping
  invariants hold (feasible list <= K, nextStartNodeIndex advance, evaluated
  nodes recorded), over configs with topology, PreFilterResult and preemption.
"""
import numpy as np
import pytest

from ksim import abi, gen, profile
from ksim.encode import encode_cluster, encode_pods
from ksim.fwplugins import EnginePlugins
from ksim.resultstore import Store
from ksim.wrapped import record_cycle
from oracle.oracle import Oracle

from fwmirror import Framework, OracleBackend, annotations


def _setup(kind: str, pct: int = 0):
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=pct)
    if kind == "config1":
        cluster, pods = gen.config1(n_nodes=300, n_pods=240)
    elif kind == "prefilter":
        nodes, pods_o = gen.prefilter_objects(n_nodes=300, n_pods=200)
        cluster, _ = encode_cluster(nodes, [])
        pods = encode_pods(cluster, pods_o)
    elif kind == "config3":
        nodes, bound, incoming = gen.config3_objects(n_nodes=240, pods_per_node=3, n_incoming=160)
        cluster, _ = encode_cluster(nodes, bound)
        pods = encode_pods(cluster, incoming)
    else:
        raise ValueError(kind)
    return cluster, pods, sp


@pytest.mark.parametrize("kind", ["config1", "prefilter", "config3"])
def test_sequential_framework_equals_oracle_cycle(kind):
    cluster, pods, sp = _setup(kind)
    prof = profile.compile_profile(sp)
    weights = profile.default_score_weights()
    # the framework mirror, one worker, TB ties, over the oracle's fw answers
    o1 = Oracle(cluster.copy_state(), prof)
    s1 = Store(weights)
    fw = Framework(EnginePlugins(OracleBackend(o1), cluster, sp), sp, s1, parallelism=1, tie="tb",
                   tb_seed=sp.tiebreak_seed)
    # the oracle's own deterministic cycle, recorded by record_cycle
    o2 = Oracle(cluster.copy_state(), prof)
    s2 = Store(weights)
    for i in range(pods.n_pods):
        rec = fw.schedule_one(pods, i)
        res = o2.cycle(pods, i)
        ns, name = pods.names[i]
        record_cycle(s2, cluster, sp, ns, name, res,
                     pods.prefilter_names[i] if pods.prefilter_names else None)
        assert rec["chosen"] == res["chosen"], i
        assert fw.next_start == o2.next_start, i
        assert annotations(s1, pods, i) == annotations(s2, pods, i), i
    a, b = o1.node_state(), o2.node_state()
    for k in a:
        np.testing.assert_array_equal(a[k], b[k])
    np.testing.assert_array_equal(o1.class_count(), o2.class_count())


@pytest.mark.parametrize("kind", ["config1", "prefilter", "config3"])
def test_racing_framework_invariants(kind):
    cluster, pods, sp = _setup(kind)
    prof = profile.compile_profile(sp)
    o = Oracle(cluster.copy_state(), prof)
    s = Store(profile.default_score_weights())
    fw = Framework(EnginePlugins(OracleBackend(o), cluster, sp), sp, s, seed=7)
    raced = 0
    for i in range(pods.n_pods):
        before = fw.next_start
        rec = fw.schedule_one(pods, i)
        if "feasible" not in rec:
            continue
        names = pods.prefilter_names[i] if pods.prefilter_names else None
        n = cluster.n_nodes if names is None else len(names)
        k = profile.num_feasible_nodes_to_find(n, sp.percentage_of_nodes_to_score)
        f, failed, ev = rec["feasible"], rec["failed"], rec["evaluated"]
        assert len(f) <= k and len(set(f)) == len(f) and len(set(ev)) == len(ev)
        assert set(f) <= set(ev) and set(failed) <= set(ev) and not set(f) & set(failed)
        # nextStartNodeIndex advances by feasible + failed; feasible nodes found
        # after the K-th were evaluated (and recorded) but count in neither
        assert fw.next_start == (before + len(f) + len(failed)) % n
        raced += len(ev) > len(f) + len(failed)
        if rec["status"] == abi.STATUS_SCHEDULED:
            assert rec["chosen"] in f
    assert raced > 0, "no cycle evaluated a feasible node past the K-th"
