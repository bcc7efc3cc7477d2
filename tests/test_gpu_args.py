"""GPU parity under plugin args beyond the defaults (ABI 8):
NodeResourcesFit MostAllocated / RequestedToCapacityRatio scoring with
extended resources, ignoredResources / ignoredResourceGroups, NodeAffinity
addedAffinity, DefaultPreemption's candidate counts.  The HIP engine through
the C ABI against the C oracle (tests/test_plugin_args.py pins the oracle to
objref under the same args): compat cycles field by field, loaded runs (the
batch paths: generic keys, the static-class table, ADAPT) placement by
placement with the node state after the run."""
import numpy as np
import pytest

from ksim import abi, gen, profile
from ksim.encode import encode_cluster, encode_pods
from ksim.engine import Engine
from oracle.oracle import Oracle
from test_plugin_args import FIT_CASES, GPU, HP, NV, _added, _nodes, _pods

pytestmark = pytest.mark.gpu

FIELDS = ("chosen", "status", "n_feasible", "n_evaluated", "n_processed", "k_to_find", "next_start")


def _compare_cycle(e, o, where):
    for f in FIELDS:
        assert e[f] == o[f], f"{where}: {f} engine={e[f]} oracle={o[f]}"
    for k in ("fail_plugin", "fail_detail", "scored", "raw", "norm", "total"):
        np.testing.assert_array_equal(e[k], o[k], err_msg=f"{where} {k}")


def _setup(nodes, pods, sp):
    cluster, _ = encode_cluster(nodes, extra_scalar=[GPU, NV, HP])
    enc = encode_pods(cluster, pods, added_affinity=sp.node_affinity)
    prof = profile.compile_profile(sp, cluster.scalar_names)
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(cluster)
    return cluster, enc, prof, eng, Oracle(cluster, prof)


def _check_state(eng, ora):
    es, os_ = eng.node_state(), ora.node_state()
    for k in es:
        np.testing.assert_array_equal(es[k], os_[k], err_msg=k)


@pytest.mark.parametrize("pct", [0, 100])
@pytest.mark.parametrize("case", sorted(FIT_CASES))
def test_fit_args_compat_cycles(case, pct):
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=pct, fit=FIT_CASES[case])
    _, enc, _, eng, ora = _setup(_nodes(300), _pods(500), sp)
    for i in range(enc.n_pods):
        _compare_cycle(eng.eval_pod(enc, i), ora.cycle(enc, i), f"{case} pod {i}")
    _check_state(eng, ora)


@pytest.mark.parametrize("pct", [0, 100])
@pytest.mark.parametrize("case", sorted(FIT_CASES))
def test_fit_args_loaded_runs(case, pct):
    """The loaded queue: pods without scalar requests and with constant
    normalized scores take the batch paths with the generic keys (the FAST
    cpu / memory keys implement LeastAllocated only), the rest per pod."""
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=pct, fit=FIT_CASES[case])
    _, enc, _, eng, ora = _setup(_nodes(1200), _pods(3000, scalars=case.startswith(("ignored", "least"))), sp)
    chosen, st = eng.schedule_batch(enc)
    ochosen, ost = ora.schedule(enc, nthreads=8)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals and st.scheduled == ost.scheduled
    assert eng.next_start == ora.next_start
    _check_state(eng, ora)


@pytest.mark.parametrize("pct", [0, 100])
@pytest.mark.parametrize("req,pref", [(True, True), (True, False), (False, True)])
def test_added_affinity_vs_oracle(req, pref, pct):
    """addedAffinity: compat cycles (errReasonEnforced detail) and a loaded run
    (the static-class table keys the added terms with the pod's own)."""
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=pct, node_affinity=_added(req, pref))
    _, enc, _, eng, ora = _setup(_nodes(240), _pods(300, scalars=False), sp)
    enforced = 0
    for i in range(enc.n_pods):
        e, o = eng.eval_pod(enc, i), ora.cycle(enc, i)
        _compare_cycle(e, o, f"pod {i}")
        enforced += int(np.sum(o["fail_detail"][o["fail_plugin"] == 3] == abi.NA_ENFORCED))
    assert (enforced > 0) == req
    _, enc, _, eng, ora = _setup(_nodes(1500), _pods(4000, scalars=False), sp)
    chosen, st = eng.schedule_batch(enc)
    ochosen, ost = ora.schedule(enc, nthreads=8)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals and eng.next_start == ora.next_start
    _check_state(eng, ora)


def test_ignored_group_and_rtcr_weight_sweep():
    """One engine across profiles: the Fit filter's ignored scalar columns are
    captured by value in the batch graphs, so a profile that changes them must
    not replay old graphs."""
    nodes, pods = _nodes(800), _pods(2000)
    cluster, _ = encode_cluster(nodes, extra_scalar=[GPU, NV, HP])
    enc = encode_pods(cluster, pods)
    eng = Engine(0)
    eng.set_cluster(cluster)
    for fit in (profile.FitArgs(), profile.FitArgs(ignored_resources=[GPU]), profile.FitArgs(),
                profile.FitArgs("RequestedToCapacityRatio", [("cpu", 1), (GPU, 3)], [(0, 0), (100, 10)],
                                ignored_resource_groups=["nvidia.com", "example.com"])):
        prof = profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=100, fit=fit),
                                       cluster.scalar_names)
        eng.set_profile(prof)
        eng.reset_cluster()
        chosen, st = eng.schedule_batch(enc)
        ochosen, ost = Oracle(cluster, prof).schedule(enc, nthreads=8)
        np.testing.assert_array_equal(chosen, ochosen)


@pytest.mark.parametrize("pct_abs", [(50, 1), (0, 3)])
def test_preemption_candidate_args_vs_oracle(pct_abs):
    from test_preemption import crowded
    from ksim.model import Container, Pod
    from ksim.preemption import bound_table
    nodes, bound, start, order = crowded(n_nodes=300, seed=9)
    cluster, _ = encode_cluster(nodes, bound)
    table = bound_table(cluster, bound, start)
    rng = np.random.default_rng(5)
    pods = [Pod(f"p{i}", priority=int(rng.choice([0, 5, 50, 500, 5000])),
                containers=[Container({"cpu": f"{int(rng.integers(10, 400)) * 100}m",
                                       "memory": f"{int(rng.integers(4, 40))}Gi"})]) for i in range(20)]
    enc = encode_pods(cluster, pods)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=100, preemption=profile.PreemptionArgs(*pct_abs))
    prof = profile.compile_profile(sp)
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(cluster)
    eng.set_bound_pods(table)
    ora = Oracle(cluster, prof)
    for i, pod in enumerate(pods):
        got = eng.preempt(enc, i, pod.priority)
        want = ora.preempt(enc, i, pod.priority, table)
        assert got == want, f"pod {i}: engine {got[:1]} {got[2:]} oracle {want[:1]} {want[2:]}"
