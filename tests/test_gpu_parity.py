"""GPU parity: the HIP engine (through the C ABI) vs the CPU oracle, bit-exact."""
import numpy as np
import pytest

from ksim import abi, gen, profile
from ksim.engine import Engine
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu

FIELDS = ("chosen", "status", "n_feasible", "n_evaluated", "n_processed", "k_to_find", "next_start")


def _prof(pct=0, seed=0x4B53494D):
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=pct, tiebreak_seed=seed)
    return profile.compile_profile(sp)


def _compare_cycle(e, o, where):
    for f in FIELDS:
        assert e[f] == o[f], f"{where}: {f} engine={e[f]} oracle={o[f]}"
    np.testing.assert_array_equal(e["fail_plugin"], o["fail_plugin"], err_msg=f"{where} fail_plugin")
    np.testing.assert_array_equal(e["fail_detail"], o["fail_detail"], err_msg=f"{where} fail_detail")
    np.testing.assert_array_equal(e["scored"], o["scored"], err_msg=f"{where} scored")
    np.testing.assert_array_equal(e["raw"], o["raw"], err_msg=f"{where} raw")
    np.testing.assert_array_equal(e["norm"], o["norm"], err_msg=f"{where} norm")
    np.testing.assert_array_equal(e["total"], o["total"], err_msg=f"{where} total")


@pytest.mark.parametrize("pct", [0, 100])
def test_config1_compat_cycles(pct):
    """Config 1 (100 nodes x 1,000 pods): every per-node filter code, raw and
    normalized score, total and placement equal the oracle's."""
    cluster, pods = gen.config1()
    prof = _prof(pct)
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(cluster)
    ora = Oracle(cluster, prof)
    for i in range(pods.n_pods):
        _compare_cycle(eng.eval_pod(pods, i), ora.cycle(pods, i), f"pod {i}")
    es, os_ = eng.node_state(), ora.node_state()
    for k in es:
        np.testing.assert_array_equal(es[k], os_[k])


@pytest.mark.parametrize("pct", [0, 100])
def test_config1_batch(pct):
    cluster, pods = gen.config1()
    prof = _prof(pct)
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(cluster)
    chosen, st = eng.schedule_batch(pods)
    ora = Oracle(cluster, prof)
    ochosen, ost = ora.schedule(pods)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals and st.scheduled == ost.scheduled
    assert eng.next_start == ora.next_start


@pytest.mark.parametrize("pct", [0, 100])
def test_config2_slice_batch(pct):
    """Config 2 cluster (5,000 nodes), first 2,000 pods: placements equal."""
    cluster, pods = gen.config2(n_pods=2000)
    prof = _prof(pct)
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(cluster)
    chosen, st = eng.schedule_batch(pods)
    ora = Oracle(cluster, prof)
    ochosen, ost = ora.schedule(pods, nthreads=8)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals
    es, os_ = eng.node_state(), ora.node_state()
    for k in es:
        np.testing.assert_array_equal(es[k], os_[k])
