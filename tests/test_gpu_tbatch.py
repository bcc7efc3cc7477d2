"""The topology batch path (ksim_tbatch.hip; class-3 pods of pod_batchable /
tbatch_admit in ksim_engine.cpp) against the one-by-one oracle: pods with
PodTopologySpread and InterPodAffinity uses read from the persistent domain
tables, scheduled up to kTbPods at a time over runs that cross a class an
earlier pod of the run adds only through node-local uses the pairs step
re-keys (tbatch_conflict_ok).  Placements, evaluation counts,
node rows and count classes must equal the oracle's (config 3 shapes:
/root/reference/simulator/scheduler/scheduler.go runs the upstream
scheduler's per-pod cycle; the restatement is oracle/ksim_oracle.c)."""
import numpy as np
import pytest

from ksim import gen, profile
from ksim.encode import encode_cluster, encode_pods
from ksim.engine import Engine
from ksim.model import Container, LabelSelector, Pod
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu


def _run(cluster, pods, weights=None):
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=100)
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
    np.testing.assert_array_equal(eng.class_count(), ora.class_count())
    es, os_ = eng.node_state(), ora.node_state()
    for k in es:
        np.testing.assert_array_equal(es[k], os_[k], err_msg=k)
    return eng, st


@pytest.mark.parametrize("n_nodes,per_node,n_inc,zone_every", [(300, 4, 800, 50), (1000, 10, 2500, 1000),
                                                               (257, 3, 700, 7)])
def test_config3_shapes(n_nodes, per_node, n_inc, zone_every):
    """Config 3's objects: zone DoNotSchedule + hostname ScheduleAnyway spread
    on the pod's app, preferred anti-affinity to it, existing pods' required
    anti-affinity (hostname, and zone-wide for tier=critical) and preferred
    affinity terms.  Every pod on the topology batch path."""
    cluster, pods = gen.config3(n_nodes=n_nodes, pods_per_node=per_node, n_incoming=n_inc, seed=n_nodes,
                                zone_anti_every=zone_every)
    eng, st = _run(cluster, pods)
    assert st.perpod_cycles == 0 and st.batches > 0
    assert st.batches < pods.n_pods                  # batches of several pods


def test_nodes_fill_up():
    """Small nodes: guesses stop fitting for later pods of a batch (pinv ends
    the batch before them) and pods become unschedulable."""
    nodes, bound, inc = gen.config3_objects(n_nodes=120, pods_per_node=2, n_incoming=1500, seed=5)
    for n in nodes:
        n.allocatable = {"cpu": "2", "memory": "4Gi", "pods": "110"}
    cluster, _ = encode_cluster(nodes, bound)
    eng, st = _run(cluster, encode_pods(cluster, inc))
    assert st.perpod_cycles == 0 and st.unschedulable > 0 and st.truncations > 0


def test_one_app_serializes():
    """Every pod spreads over the same selector: each pod reads the zone
    DoNotSchedule counts the earlier ones add.  A run holds two pods (the
    second's zone variant is taken by where the first lands, ksim_device.h
    TbVar); a third reads a class two earlier pods add and starts the next
    run.  Still exact."""
    nodes, bound, inc = gen.config3_objects(n_nodes=200, pods_per_node=3, n_incoming=200, seed=9)
    for p in inc:
        p.labels["app"] = "a7"
        for c in p.topology_spread:
            c.label_selector = LabelSelector({"app": "a7"})
        for w in p.pod_anti_affinity_preferred:
            w.term.label_selector = LabelSelector({"app": "a7"})
    cluster, _ = encode_cluster(nodes, bound)
    eng, st = _run(cluster, encode_pods(cluster, inc))
    assert st.perpod_cycles == 0 and 100 <= st.batches < 200
    assert eng.diag()["tb_variant_pods"] > 0


def _few_apps(inc, n_apps, rng, zone=True):
    """Incoming pods relabelled to n_apps apps (selectors follow): most pods of
    a batch read classes earlier ones add.  zone=False drops the zone
    DoNotSchedule constraint (a domain-keyed use ends a run; the hostname
    spread and the preferred anti-affinity are node-local and runs cross them)."""
    for p in inc:
        app = f"a{int(rng.integers(0, n_apps))}"
        p.labels["app"] = app
        if not zone:
            p.topology_spread = [c for c in p.topology_spread if c.when_unsatisfiable == "ScheduleAnyway"]
        for c in p.topology_spread:
            c.label_selector = LabelSelector({"app": app})
        for w in p.pod_anti_affinity_preferred:
            w.term.label_selector = LabelSelector({"app": app})
    return inc


@pytest.mark.parametrize("n_apps,per_node,zone", [(2, 4, False), (6, 4, False), (6, 0, False), (6, 4, True)])
def test_cross_class_runs(n_apps, per_node, zone):
    """Runs that cross class conflicts (tbatch_conflict_ok): pods of few apps
    re-key the guessed nodes (hostname spread counts, preferred anti-affinity
    scores, the holders of the extrema).  With no existing pods the
    InterPodAffinity topologyScore starts empty (the emptiness flag flips).
    With the zone DoNotSchedule constraint runs end at the conflicts."""
    nodes, bound, inc = gen.config3_objects(n_nodes=600, pods_per_node=per_node, n_incoming=1500, seed=31 + n_apps)
    inc = _few_apps(inc, n_apps, np.random.default_rng(n_apps), zone=zone)
    cluster, _ = encode_cluster(nodes, bound)
    eng, st = _run(cluster, encode_pods(cluster, inc))
    # few apps over 3 zones even out quickly: many zone verdicts flip (pinv)
    print(f"apps {n_apps}: {len(inc)} pods in {st.batches} batches, {st.truncations} truncated")
    assert st.perpod_cycles == 0 and st.batches < len(inc)


def test_cross_class_required_terms():
    """Required anti-affinity (hostname, against the pod's own app) on some
    pods and required affinity (hostname, to an app) on others: a guessed node
    stops passing for a later pod of the app (pinv) or may start passing."""
    from ksim.model import PodAffinityTerm
    nodes, bound, inc = gen.config3_objects(n_nodes=400, pods_per_node=3, n_incoming=1200, seed=41)
    rng = np.random.default_rng(41)
    inc = _few_apps(inc, 5, rng, zone=False)
    for k, p in enumerate(inc):
        if k % 4 == 1:
            p.pod_anti_affinity_required = [PodAffinityTerm("kubernetes.io/hostname",
                                                            LabelSelector({"app": p.labels["app"]}))]
        elif k % 9 == 2:
            p.pod_affinity_required = [PodAffinityTerm("kubernetes.io/hostname",
                                                       LabelSelector({"app": f"a{int(rng.integers(0, 5))}"}))]
    cluster, _ = encode_cluster(nodes, bound)
    _run(cluster, encode_pods(cluster, inc))


def test_mixed_with_plain_pods():
    """Spread pods (topology batches) interleaved with plain pods carrying the
    same app labels (P100 batches whose binds add to the spread selectors'
    classes): the runs alternate and hand the snapshot on."""
    nodes, bound, inc = gen.config3_objects(n_nodes=500, pods_per_node=4, n_incoming=900, seed=17)
    plain = [Pod(f"plain-{k}", labels={"app": f"a{k % 64}", "tier": "web"},
                 containers=[Container({"cpu": "300m", "memory": "512Mi"})]) for k in range(900)]
    queue = []
    for k in range(900):
        queue.append(inc[k])
        if k % 3 == 0:
            queue.extend(plain[k:k + 3])
    cluster, _ = encode_cluster(nodes, bound)
    _run(cluster, encode_pods(cluster, queue))


def test_weights_and_soft_only():
    """Score weights from a config-5 style vector, and pods with only a
    ScheduleAnyway hostname spread (no hard constraint)."""
    nodes, bound, inc = gen.config3_objects(n_nodes=400, pods_per_node=5, n_incoming=900, seed=21)
    for k, p in enumerate(inc):
        if k % 2:
            p.topology_spread = [c for c in p.topology_spread if c.when_unsatisfiable == "ScheduleAnyway"]
    cluster, _ = encode_cluster(nodes, bound)
    w = {"NodeResourcesFit": 3, "NodeResourcesBalancedAllocation": 7, "PodTopologySpread": 5,
         "InterPodAffinity": 9, "TaintToleration": 1, "NodeAffinity": 2}
    _run(cluster, encode_pods(cluster, inc), weights=w)


def test_kernel_timing_names():
    """ksim_time_kernels times the topology batch kernels under their names."""
    cluster, pods = gen.config3(n_nodes=300, pods_per_node=4, n_incoming=300, seed=3)
    prof = profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=100))
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(cluster)
    eng.load_pods(pods)
    kt = eng.time_kernels(0, pods.n_pods)
    for k in ("k_tb_filter", "k_tb_select", "k_tb_merge", "k_tb_chain_pairs", "k_tb_commit"):
        assert k in kt and kt[k][1] > 0, (k, kt)


# ---- zone variants (round 6): runs that cross the zone DoNotSchedule class ----
def _zone_objects(n_nodes, per_node, n_inc, seed, zones=3, zone_every=1000, max_skew=1):
    """config3_objects with the nodes spread round-robin over ``zones`` zones
    and the incoming pods' zone constraint at ``max_skew``."""
    nodes, bound, inc = gen.config3_objects(n_nodes=n_nodes, pods_per_node=per_node, n_incoming=n_inc, seed=seed,
                                            zone_anti_every=zone_every)
    for i, n in enumerate(nodes):
        n.labels["topology.kubernetes.io/zone"] = f"z{i % zones}"
    for p in inc:
        for c in p.topology_spread:
            if c.when_unsatisfiable == "DoNotSchedule":
                c.max_skew = max_skew
    return nodes, bound, inc


def _batches_without_variants(cluster, pods):
    """The same queue on the flavor without zone variants (libksim_engine_ab64.so):
    runs end at a zone-keyed class conflict."""
    prof = profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=100))
    eng = Engine(0, variant="ab64")
    eng.set_profile(prof)
    eng.set_cluster(cluster)
    chosen, st = eng.schedule_batch(pods)
    assert eng.diag()["tb_variant_pods"] == 0
    eng.close()
    return chosen, st


@pytest.mark.parametrize("n_nodes,per_node,n_inc,zone_every,seed", [(900, 6, 2400, 1000, 3), (600, 4, 1600, 50, 4),
                                                                     (5000, 10, 3000, 1000, 5)])
def test_zone_variants_config3(n_nodes, per_node, n_inc, zone_every, seed):
    """Config 3's queue: a pod whose app already has one pod earlier in the run
    is evaluated per feasible-zone set that pod's landing zone gives (its
    slots), and the chain takes the slot its guess names.  Placements equal
    the oracle's; batches are longer than the flavor without variants, which
    places the same pods."""
    cluster, pods = gen.config3(n_nodes=n_nodes, pods_per_node=per_node, n_incoming=n_inc, seed=seed,
                                zone_anti_every=zone_every)
    eng, st = _run(cluster, pods)
    vp = eng.diag()["tb_variant_pods"]
    chosen0, st0 = _batches_without_variants(cluster, pods)
    print(f"{n_inc} pods: {st.batches} batches ({vp} pods on a moved zone verdict), {st0.batches} without variants")
    assert st.perpod_cycles == 0 and vp > 0
    assert st.batches < st0.batches


@pytest.mark.parametrize("zones,max_skew", [(2, 1), (4, 1), (4, 2), (5, 1), (3, 3)])
def test_zone_variants_domains(zones, max_skew):
    """Keys of 2 and 4 zones (kVarDom = 4: the slots of every landing zone),
    5 zones (more domains than slots: no variants, runs end at the conflict),
    and a wider maxSkew (fewer verdicts move)."""
    nodes, bound, inc = _zone_objects(700, 4, 1500, seed=50 + zones, zones=zones, zone_every=70, max_skew=max_skew)
    cluster, _ = encode_cluster(nodes, bound)
    eng, st = _run(cluster, encode_pods(cluster, inc))
    vp = eng.diag()["tb_variant_pods"]
    print(f"zones {zones} maxSkew {max_skew}: {st.batches} batches, {vp} variant pods")
    assert st.perpod_cycles == 0
    if zones > 4:
        assert vp == 0
    elif max_skew == 1:
        assert vp > 0


def test_zone_variants_few_apps_and_full_nodes():
    """Two apps on small nodes: most pods have an adder, guesses stop fitting
    (pinv), adders become unschedulable (no count moves: slot 0)."""
    nodes, bound, inc = _zone_objects(150, 2, 1800, seed=61)
    for n in nodes:
        n.allocatable = {"cpu": "4", "memory": "8Gi", "pods": "110"}
    inc = _few_apps(inc, 2, np.random.default_rng(61))
    cluster, _ = encode_cluster(nodes, bound)
    eng, st = _run(cluster, encode_pods(cluster, inc))
    assert st.perpod_cycles == 0 and st.unschedulable > 0


def test_zone_variants_foreign_selector_and_two_keys():
    """Pods whose zone constraint selects another app (they add nothing to the
    class they read: self match 0, the adders are that app's pods), pods with a
    second DoNotSchedule constraint on a region key (a second zone-keyed
    conflict ends the run), and pods whose required node affinity leaves one
    zone out (the per-pod path takes those: tbatch_admit)."""
    from ksim.model import LabelSelector as LS, NodeSelectorTerm, Requirement, TopologySpreadConstraint
    nodes, bound, inc = _zone_objects(600, 4, 1500, seed=71, zone_every=60)
    for i, n in enumerate(nodes):
        n.labels["topology.kubernetes.io/region"] = f"r{(i // 7) % 2}"
    rng = np.random.default_rng(71)
    for k, p in enumerate(inc):
        if k % 5 == 1:
            other = f"a{int(rng.integers(0, 64))}"
            for c in p.topology_spread:
                if c.when_unsatisfiable == "DoNotSchedule":
                    c.label_selector = LS({"app": other})
        elif k % 5 == 2:
            p.topology_spread = list(p.topology_spread) + [
                TopologySpreadConstraint(1, "topology.kubernetes.io/region", "DoNotSchedule",
                                         LS({"app": p.labels["app"]}))]
        elif k % 5 == 3:
            p.required_terms = [NodeSelectorTerm([Requirement("topology.kubernetes.io/zone", "NotIn", ["z2"])])]
    cluster, _ = encode_cluster(nodes, bound)
    eng, st = _run(cluster, encode_pods(cluster, inc))
    assert st.perpod_cycles == sum(1 for p in inc if p.required_terms) and eng.diag()["tb_variant_pods"] > 0
