"""The oracle's timing path (ksim_oracle_schedule) fans every phase of the
cycle out over threads -- the filter loop, findNodesThatPassFilters' scan
(per-thread slices, one stop), the scores, NormalizeScore (per-thread
extrema), the totals and selectHost (per-thread best, combined) -- for the CPU
baseline (bench.py cpu_baseline).  Its placements, evaluation counts,
nextStartNodeIndex and final state must not depend on the thread count, and
must equal the per-pod compat cycle (ksim_oracle_cycle), a separate serial
restatement."""
import numpy as np
import pytest

from ksim import gen, profile
from ksim.encode import encode_cluster, encode_pods
from oracle.oracle import Oracle


def _case(kind):
    if kind == "config1_p100":
        c, p = gen.config1(n_nodes=300, n_pods=400)
        return c, p, profile.compile_profile(profile.SchedulerProfile())
    if kind == "config1_adapt":
        c, p = gen.config1(n_nodes=300, n_pods=400)
        return c, p, profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=0))
    if kind == "config2_adapt":
        c, p = gen.config2(n_nodes=700, n_pods=900)
        return c, p, profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=0))
    if kind == "config3":
        nodes, bound, inc = gen.config3_objects(n_nodes=240, pods_per_node=3, n_incoming=200)
        c, _ = encode_cluster(nodes, bound)
        return c, encode_pods(c, inc), profile.compile_profile(profile.SchedulerProfile())
    if kind == "netbw_errors":
        import test_netbw
        nodes, bound, pending = gen.netbw_objects(n_nodes=150, n_pods=300, node_errors=True, pod_errors=True)
        sp = test_netbw.nb_profile(0)
        c, _ = encode_cluster(nodes, bound, nb_args=sp.network_bandwidth)
        return c, encode_pods(c, pending), profile.compile_profile(sp)
    raise KeyError(kind)


@pytest.mark.parametrize("kind", ["config1_p100", "config1_adapt", "config2_adapt", "config3", "netbw_errors"])
def test_schedule_independent_of_threads(kind):
    cluster, pods, prof = _case(kind)
    runs = []
    for nt in (1, 3, 8, 16):
        o = Oracle(cluster.copy_state(), prof)
        chosen, st = o.schedule(pods, nthreads=nt)
        runs.append((nt, chosen, st.evals, st.scheduled, o.next_start, o.node_state(), o.class_count()))
    ref = Oracle(cluster.copy_state(), prof)
    want = np.array([ref.cycle(pods, i)["chosen"] for i in range(pods.n_pods)], np.int32)
    for nt, chosen, evals, sched, ns, state, cls in runs:
        np.testing.assert_array_equal(chosen, want, err_msg=f"{kind} threads={nt}")
        assert (evals, sched, ns) == runs[0][2:5], (kind, nt)
        for k in state:
            np.testing.assert_array_equal(state[k], runs[0][5][k], err_msg=f"{kind} threads={nt} {k}")
        np.testing.assert_array_equal(cls, runs[0][6])
    assert ref.next_start == runs[0][4]
