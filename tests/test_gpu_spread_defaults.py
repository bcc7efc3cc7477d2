"""PodTopologySpread default constraints on the GPU (KSIM_POD_PTS_SYSTEM_DEFAULT:
PreScore's requireAllTopologies = false; defaultingType List): the HIP engine
against the C oracle (tests/test_spread_defaults.py pins the oracle to objref's
own buildDefaultConstraints / DefaultSelector) on clusters where some nodes
lack the zone or hostname label: compat cycles field by field, loaded runs
(per-pod path, P100 and ADAPT) and node-sharded groups."""
import numpy as np
import pytest

from ksim import abi, profile
from ksim.encode import encode_cluster, encode_pods
from ksim.engine import Engine, group_schedule_loaded
from ksim.model import TopologySpreadConstraint
from ksim.topology import SpreadDefaults
from oracle.oracle import Oracle
from test_spread_defaults import HOST, WORKLOADS, ZONE, mixed_nodes, workload_pods

pytestmark = pytest.mark.gpu

FIELDS = ("chosen", "status", "n_feasible", "n_evaluated", "n_processed", "k_to_find", "next_start")
LIST_ARGS = profile.PodTopologySpreadArgs("List", [
    TopologySpreadConstraint(2, ZONE, "DoNotSchedule"),
    TopologySpreadConstraint(1, HOST, "ScheduleAnyway", node_taints_policy="Honor"),
    TopologySpreadConstraint(4, "pool", "ScheduleAnyway", node_affinity_policy="Ignore")])


def _encode(n_nodes, n_bound, n_pods, args, seed=5):
    nodes = mixed_nodes(n_nodes, seed=3)
    bound = workload_pods(n_bound, seed=11, bound_nodes=[n.name for n in nodes])
    pods = workload_pods(n_pods, seed=seed)
    cluster, _ = encode_cluster(nodes, bound)
    enc = encode_pods(cluster, pods, spread=SpreadDefaults(args, *WORKLOADS))
    return cluster, enc


@pytest.mark.parametrize("pct", [0, 100])
@pytest.mark.parametrize("kind", ["system", "list"])
def test_compat_cycles(kind, pct):
    args = profile.PodTopologySpreadArgs() if kind == "system" else LIST_ARGS
    cluster, enc = _encode(400, 800, 400, args)
    if kind == "system":
        assert (enc.pods["topo_flags"] & abi.POD_PTS_SYSTEM_DEFAULT).any()
    prof = profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=pct, spread=args))
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(cluster)
    ora = Oracle(cluster, prof)
    for i in range(enc.n_pods):
        e, o = eng.eval_pod(enc, i), ora.cycle(enc, i)
        for f in FIELDS:
            assert e[f] == o[f], f"pod {i}: {f} engine={e[f]} oracle={o[f]}"
        for k in ("fail_plugin", "fail_detail", "scored", "raw", "norm", "total"):
            np.testing.assert_array_equal(e[k], o[k], err_msg=f"pod {i} {k}")
    np.testing.assert_array_equal(eng.class_count(), ora.class_count())


@pytest.mark.parametrize("pct", [0, 100])
@pytest.mark.parametrize("kind", ["system", "list"])
def test_loaded_runs(kind, pct):
    args = profile.PodTopologySpreadArgs() if kind == "system" else LIST_ARGS
    cluster, enc = _encode(2000, 4000, 2500, args, seed=8)
    prof = profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=pct, spread=args))
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(cluster)
    chosen, st = eng.schedule_batch(enc)
    ora = Oracle(cluster, prof)
    ochosen, ost = ora.schedule(enc, nthreads=8)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals and st.scheduled == ost.scheduled and eng.next_start == ora.next_start
    es, os_ = eng.node_state(), ora.node_state()
    for k in es:
        np.testing.assert_array_equal(es[k], os_[k], err_msg=k)
    np.testing.assert_array_equal(eng.class_count(), ora.class_count())


@pytest.mark.parametrize("pct,world", [(0, 2), (100, 3)])
def test_sharded_group_system_defaults(pct, world):
    """The sharded per-pod cycle: domain sums (the (key, "") pair included)
    exchanged, pair registrations over the global kept list, no IgnoredNodes."""
    from ksim.shard import partition
    args = profile.PodTopologySpreadArgs()
    cluster, enc = _encode(600, 1200, 500, args, seed=9)
    prof = profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=pct, spread=args))
    engines = []
    for base, cnt in partition(cluster.n_nodes, world):
        e = Engine(0)
        e.set_shard(base, cluster.n_nodes)
        e.set_profile(prof)
        e.set_cluster(cluster.shard(base, cnt))
        e.load_pods(enc)
        engines.append(e)
    chosen, st = group_schedule_loaded(engines, 0, enc.n_pods)
    ora = Oracle(cluster, prof)
    ochosen, ost = ora.schedule(enc, nthreads=8)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals and st.scheduled == ost.scheduled
