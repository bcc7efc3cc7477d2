"""The batch path's runtime-chosen kernel instantiations at their thresholds.

launch_top_commit / launch_eval_top (csrc/ksim_batch.hip) pick a template
instantiation per launch from the node count and the profile: KEEP while a
handle's node range fits kKeepPerLane * 1024 = 8,192 nodes, the direct overlay
while the cluster fits kLazyDirect = 32,768 nodes, node-stationary evaluation
past 8,192 nodes for the default profile's key shape (DEF), the generic key
for any other shape (unequal resource weights here), the static-class (STAB)
and FAST forms of the three-launch batches, and the generic keys.  Each case
runs at 8,192 / 8,193 and 32,768 / 32,769 nodes (P100 and ADAPT) against the
oracle, and the last test asserts through ksim_get_diag out[25] that every
instantiation ran in this process."""
import numpy as np
import pytest

from ksim import gen, profile
from ksim.engine import Engine, group_schedule_loaded
from ksim.shard import partition
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu

SIZES = [8192, 8193, 32768, 32769]
ALL_BITS = set(range(10)) | set(range(16, 22))
SEEN = {}


def _sp(pct, shape):
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=pct)
    if shape == "generic":                      # unequal resource weights: not the compiled-in shape
        sp.fit = profile.FitArgs(resources=[("cpu", 2), ("memory", 1)])
    return sp


def _bits(e):
    m = e.diag()["variants"]
    return {b for b in range(64) if m >> b & 1}


def _check(cluster, pods, prof, tag):
    e = Engine(0)
    e.set_profile(prof)
    e.set_cluster(cluster.copy_state())
    before = _bits(e)
    chosen, st = e.schedule_batch(pods)
    ora = Oracle(cluster.copy_state(), prof)
    ochosen, ost = ora.schedule(pods, nthreads=16)
    np.testing.assert_array_equal(chosen, ochosen, err_msg=tag)
    assert (st.evals, st.scheduled) == (ost.evals, ost.scheduled), tag
    assert e.next_start == ora.next_start, tag
    es, os_ = e.node_state(), ora.node_state()
    for k in es:
        np.testing.assert_array_equal(es[k], os_[k], err_msg=f"{tag} {k}")
    SEEN[tag] = sorted(_bits(e) - before)
    e.close()


@pytest.mark.parametrize("shape", ["default", "generic"])
@pytest.mark.parametrize("pct", [100, 0])
@pytest.mark.parametrize("n_nodes", SIZES)
def test_bare_pods_at_thresholds(n_nodes, pct, shape):
    """Config-2 pods (FAST, no count classes: the deferred-commit batches)."""
    cluster, pods = gen.config2(n_nodes=n_nodes, n_pods=700)
    _check(cluster, pods, profile.compile_profile(_sp(pct, shape)), f"bare {n_nodes} {pct} {shape}")


@pytest.mark.parametrize("shape", ["default", "generic"])
@pytest.mark.parametrize("n_nodes", [8192, 8193])
def test_config1_pods_at_keep_threshold(n_nodes, shape):
    """Config-1 pods (taints, node affinity: static-class and generic keys,
    the three-launch batches) on both sides of the KEEP range."""
    cluster, pods = gen.config1(n_nodes=n_nodes, n_pods=500)
    _check(cluster, pods, profile.compile_profile(_sp(100, shape)), f"config1 {n_nodes} {shape}")


@pytest.mark.parametrize("n_nodes", [3000, 8193])
def test_generic_keys(n_nodes):
    """A scoring strategy over ephemeral-storage as well as cpu and memory:
    neither the FAST nor the static-class keys, the generic key (512 threads)."""
    cluster, pods = gen.config1(n_nodes=n_nodes, n_pods=500)
    sp = _sp(100, "default")
    sp.fit = profile.FitArgs(resources=[("cpu", 1), ("memory", 1), ("ephemeral-storage", 1)])
    _check(cluster, pods, profile.compile_profile(sp), f"generic keys {n_nodes}")


def _shards(cluster, pods, prof, world, replicated):
    engines = []
    for base, cnt in partition(cluster.n_nodes, world):
        e = Engine(0)
        if replicated:
            e.set_profile(prof)
            e.set_cluster(cluster)
            e.set_eval_range(base, base + cnt)
        else:
            e.set_shard(base, cluster.n_nodes)
            e.set_profile(prof)
            e.set_cluster(cluster.shard(base, cnt))
        e.load_pods(pods)
        engines.append(e)
    return engines


@pytest.mark.parametrize("shape", ["default", "generic"])
@pytest.mark.parametrize("n_nodes,replicated", [(3000, False), (20000, True), (40000, True)])
def test_group_forms(n_nodes, replicated, shape):
    """Sharded groups (the FAST three-launch form with the candidate exchange)
    and replicated groups past the KEEP range and past the direct overlay
    (each replica keys its range and sends its record)."""
    cluster, pods = gen.config2(n_nodes=n_nodes, n_pods=600)
    prof = profile.compile_profile(_sp(100, shape))
    engines = _shards(cluster, pods, prof, 2, replicated)
    before = _bits(engines[0])
    chosen, st = group_schedule_loaded(engines, 0, pods.n_pods)
    ora = Oracle(cluster, prof)
    ochosen, ost = ora.schedule(pods, nthreads=16)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals and st.scheduled == ost.scheduled
    SEEN[f"group {n_nodes} {replicated} {shape}"] = sorted(_bits(engines[0]) - before)
    for e in engines:
        e.close()


def test_every_instantiation_reached():
    """Run after the cases above (file order): every k_batch_top_commit and
    k_batch_top instantiation was launched by this process."""
    cluster, _ = gen.config2(n_nodes=64, n_pods=1)
    e = Engine(0)
    e.set_profile(profile.compile_profile(profile.SchedulerProfile()))
    e.set_cluster(cluster)
    got = _bits(e)
    e.close()
    missing = sorted(ALL_BITS - got)
    assert not missing, f"instantiations never launched: {missing}; per case: {SEEN}"
