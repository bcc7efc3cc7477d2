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


def _batch_vs_oracle(cluster, pods, pct=100, seed=0x4B53494D, nthreads=None):
    prof = _prof(pct, seed)
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(cluster)
    chosen, st = eng.schedule_batch(pods)
    ora = Oracle(cluster, prof)
    ochosen, ost = ora.schedule(pods) if nthreads is None else ora.schedule(pods, nthreads=nthreads)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals and st.scheduled == ost.scheduled
    assert eng.next_start == ora.next_start
    es, os_ = eng.node_state(), ora.node_state()
    for k in es:
        np.testing.assert_array_equal(es[k], os_[k])
    return st


# ---- ADAPT batch path (ksim_adapt.hip): windows by relaxation, broken windows ----

@pytest.mark.parametrize("n_nodes", [101, 150, 257, 1000])
def test_adapt_batch_until_full(n_nodes):
    """K < N; nodes fill up (feasibility flips inside windows, unschedulable pods)."""
    cluster, _ = gen.config2(n_nodes=n_nodes, n_pods=1)
    pods = gen.bare_pods(n_nodes * 60 + 37, seed=31)
    st = _batch_vs_oracle(cluster, pods, pct=0)
    assert st.perpod_cycles == 0 and st.batches > 0


def test_adapt_batch_config2_and_pct():
    cluster, pods = gen.config2(n_nodes=5000, n_pods=6000)
    _batch_vs_oracle(cluster, pods, pct=0)
    cluster, pods = gen.config2(n_nodes=3000, n_pods=4000, seed=77)
    _batch_vs_oracle(cluster, pods, pct=30)


@pytest.mark.parametrize("pct,n_pods", [(0, 45000), (30, 20000)])
def test_adapt_batch_group_counts(pct, n_pods):
    """Lazy ADAPT windows on more than 256 bitmap words (k_adapt_cut0, then
    the relaxation inside k_adapt_top from those cuts): 17,000 nodes, pods at
    16x config 2's requests fill them, so the feasibility bitmaps turn sparse,
    the windows wrap and ~2,000 pods find no node; K = 850 (pct 0) and
    K = 5,100 (pct 30, the wide top)."""
    cluster, _ = gen.config2(n_nodes=17000, n_pods=1)
    pods = gen.bare_pods(n_pods, seed=41)
    for col in ("req_cpu", "req_mem", "nz_cpu", "nz_mem"):
        pods.pods[col] *= 16
    st = _batch_vs_oracle(cluster, pods, pct=pct, nthreads=16)
    assert st.perpod_cycles == 0 and st.batches > 0


def test_adapt_batch_mixed_runs():
    """Config-1 objects on 400 nodes (K = 100 < N): batch and per-pod runs
    interleave and hand nextStartNodeIndex to each other (every fifth pod
    carries a ScheduleAnyway zone spread constraint: the per-pod path)."""
    from ksim.encode import encode_cluster, encode_pods
    from ksim.model import LabelSelector, TopologySpreadConstraint
    nodes, pods = gen.config1_objects(n_nodes=400, n_pods=2000)
    for n in nodes:
        n.taints = [t for t in n.taints if t.effect != "PreferNoSchedule"]
    for k, p in enumerate(pods):
        p.labels = {"app": f"a{k % 3}"}
        if k % 5 == 4:
            p.topology_spread = [TopologySpreadConstraint(1, "topology.kubernetes.io/zone", "ScheduleAnyway",
                                                          LabelSelector({"app": p.labels["app"]}))]
    cluster, _ = encode_cluster(nodes)
    st = _batch_vs_oracle(cluster, encode_pods(cluster, pods), pct=0)
    assert st.perpod_cycles > 0 and st.batches > 0


@pytest.mark.parametrize("n_nodes", [1, 7, 64, 65, 300])
def test_batch_small_clusters(n_nodes):
    """Ragged node counts (partial wave tiles, single node), pod count not a
    multiple of the batch size, and pods that stop fitting (unschedulable)."""
    cluster, _ = gen.config2(n_nodes=n_nodes, n_pods=1)
    pods = gen.bare_pods(n_nodes * 40 + 37, seed=99)
    st = _batch_vs_oracle(cluster, pods)
    assert st.perpod_cycles == 0 and st.batches > 0


def test_batch_truncation_identical_pods():
    """Identical pods on identical nodes: every pod's top-T overlaps the nodes
    already bound in the batch, forcing truncated batches; placements must still
    equal the one-by-one oracle."""
    cluster, _ = gen.config2(n_nodes=40, n_pods=1)
    cluster.alloc_cpu[:] = 64000
    cluster.alloc_mem[:] = 256 << 30
    pods = gen.bare_pods(3000, seed=5, cpu_steps=1, mem_steps=1)
    prof = _prof(100)
    st = _batch_vs_oracle(cluster, pods)
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(cluster)
    eng.schedule_batch(pods)
    assert st.truncations + eng.diag()["cuts"] > 0 and st.batches > pods.n_pods // 256


def test_batch_mixed_runs_config1_p100():
    """Config-1 pods on config-1 nodes without PreferNoSchedule taints: pods
    with preferred node affinity carry their normalized NodeAffinity scores in
    the batch keys (kPodNormVaries), so every pod takes the batch path.
    Pods with spec.nodeName (a static filter) stay batchable."""
    from ksim.encode import encode_cluster, encode_pods
    nodes, pods = gen.config1_objects()
    for n in nodes:
        n.taints = [t for t in n.taints if t.effect != "PreferNoSchedule"]
    cluster, _ = encode_cluster(nodes)
    st = _batch_vs_oracle(cluster, encode_pods(cluster, pods))
    assert st.perpod_cycles == 0 and st.batches > 0
    for i in range(0, len(pods), 97):
        pods[i].node_name = nodes[i % len(nodes)].name
    st = _batch_vs_oracle(cluster, encode_pods(cluster, pods))
    assert st.perpod_cycles == 0 and st.batches > 0


def test_batch_weights_sweep():
    """Config-5 style weight vectors over a config-2 slice."""
    cluster, pods = gen.config2(n_nodes=1000, n_pods=3000)
    ws = gen.config5_weights()[:3]
    for w in ws:
        sp = profile.SchedulerProfile(percentage_of_nodes_to_score=100)
        names = [p.name for p in sp.score_plugins()]
        prof = profile.compile_profile(sp.with_weights({n: int(x) for n, x in zip(names, w)}))
        eng = Engine(0)
        eng.set_profile(prof)
        eng.set_cluster(cluster)
        chosen, _ = eng.schedule_batch(pods)
        ochosen, _ = Oracle(cluster, prof).schedule(pods)
        np.testing.assert_array_equal(chosen, ochosen)


def test_batch_cuts_balanced_heavy():
    """BalancedAllocation-heavy weights with skewed pods: binding a pod can
    raise a node's balance score for a later pod of the same batch, so some
    pods' exact choice is a node bound earlier in the batch (a cut).  The cut
    path must stay exact."""
    cluster, _ = gen.config2(n_nodes=300, n_pods=1)
    pods = gen.bare_pods(4000, seed=17, cpu_steps=20, mem_steps=2)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=100)
    names = [p.name for p in sp.score_plugins()]
    w = {n: (10 if n == "NodeResourcesBalancedAllocation" else 1) for n in names}
    prof = profile.compile_profile(sp.with_weights(w))
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(cluster)
    chosen, st = eng.schedule_batch(pods)
    ora = Oracle(cluster, prof)
    ochosen, ost = ora.schedule(pods)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals and st.scheduled == ost.scheduled
    d = eng.diag()
    print("diag", d)
    assert d["cuts"] > 0


# ---- PodTopologySpread + InterPodAffinity (config 3 shapes) ----------------------
def _engine(cluster, prof):
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(cluster)
    return eng


@pytest.mark.parametrize("pct", [0, 100])
def test_config3_compat_cycles(pct):
    """Per-node outputs of every cycle (filter codes incl. PTS / IPA details,
    raw + normalized scores, totals) and the count classes afterwards."""
    cluster, pods = gen.config3(n_nodes=300, pods_per_node=10, n_incoming=300, seed=11, zone_anti_every=50)
    prof = _prof(pct)
    eng, ora = _engine(cluster, prof), Oracle(cluster, prof)
    for i in range(pods.n_pods):
        _compare_cycle(eng.eval_pod(pods, i), ora.cycle(pods, i), f"pod {i}")
    np.testing.assert_array_equal(eng.class_count(), ora.class_count())


@pytest.mark.parametrize("pct", [0, 100])
def test_config3_batch(pct):
    cluster, pods = gen.config3(n_nodes=1000, pods_per_node=10, n_incoming=1500, seed=12)
    prof = _prof(pct)
    eng = _engine(cluster, prof)
    chosen, st = eng.schedule_batch(pods)
    ora = Oracle(cluster, prof)
    ochosen, ost = ora.schedule(pods, nthreads=8)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals and st.scheduled == ost.scheduled
    np.testing.assert_array_equal(eng.class_count(), ora.class_count())
    es, os_ = eng.node_state(), ora.node_state()
    for k in es:
        np.testing.assert_array_equal(es[k], os_[k])


def test_topology_mixed_with_batchable_pods():
    """Bare pods carrying app labels (batch path; their binds add to the
    spread constraints' selector classes) interleaved with spread pods
    (topology batch path).  No pod carries an affinity term, so the bare pods have
    no topology uses of their own and stay batchable."""
    from ksim.encode import encode_cluster, encode_pods
    from ksim.model import Container, Pod
    nodes, bound, inc = gen.config3_objects(n_nodes=400, pods_per_node=5, n_incoming=600, seed=13)
    for p in bound:
        p.pod_anti_affinity_required, p.pod_affinity_preferred = [], []
    for p in inc:
        p.pod_anti_affinity_preferred = []
    bare = [Pod(f"bare-{k}", labels={"app": f"a{k % 64}", "tier": "web"},
                containers=[Container({"cpu": "200m", "memory": "512Mi"})]) for k in range(1200)]
    queue = []
    for k in range(600):
        queue.append(inc[k])
        queue.extend(bare[2 * k:2 * k + 2])
    cluster, _ = encode_cluster(nodes, bound)
    pods = encode_pods(cluster, queue)
    prof = _prof(100)
    eng = _engine(cluster, prof)
    chosen, st = eng.schedule_batch(pods)
    ora = Oracle(cluster, prof)
    ochosen, _ = ora.schedule(pods, nthreads=8)
    np.testing.assert_array_equal(chosen, ochosen)
    np.testing.assert_array_equal(eng.class_count(), ora.class_count())
    assert st.perpod_cycles == 0 and st.batches > 0      # spread pods: topology batches (ksim_tbatch.hip)


def test_topology_hand_cases_vs_oracle():
    """The object-level cases of tests/test_topology.py through the engine."""
    import test_topology as tt
    from ksim.encode import encode_cluster, encode_pods
    cases = []
    nodes = [tt._node(i, f"z{i % 3}") for i in range(9)]
    term = tt.PodAffinityTerm("topology.kubernetes.io/zone", tt.LabelSelector({"app": "db"}))
    cases.append((nodes, [], [tt._pod(f"db{i}", {"app": "db"}, pod_affinity_required=[term]) for i in range(4)]))
    nodes2 = [tt._node(i, f"z{i % 2}") for i in range(6)]
    bound2 = [tt._pod("e0", {"app": "x"}, node="n0", pod_anti_affinity_required=[
        tt.PodAffinityTerm("topology.kubernetes.io/zone", tt.LabelSelector({"app": "y"}))])]
    cases.append((nodes2, bound2, [tt._pod("y0", {"app": "y"}), tt._pod("x1", {"app": "z"}, pod_anti_affinity_required=[
        tt.PodAffinityTerm("kubernetes.io/hostname", tt.LabelSelector({"app": "x"}))])]))
    for nodes, bound, pods in cases:
        cluster, _ = encode_cluster(nodes, bound)
        enc = encode_pods(cluster, pods)
        for pct in (0, 100):
            prof = _prof(pct)
            eng, ora = _engine(cluster, prof), Oracle(cluster, prof)
            for i in range(enc.n_pods):
                _compare_cycle(eng.eval_pod(enc, i), ora.cycle(enc, i), f"pod {i}")


@pytest.mark.parametrize("pct", [0, 100])
def test_node_ports_vs_oracle(pct):
    """NodePorts on the device: per-node codes of every cycle, then a batch run
    mixing port pods (per-pod path) and batchable pods."""
    from ksim.encode import encode_cluster, encode_pods
    from ksim.model import ContainerPort
    nodes, pods = gen.config1_objects(n_nodes=150, n_pods=900)
    for i, p in enumerate(pods):
        if i % 3 == 0:
            p.containers[0].ports = [ContainerPort(8000 + i % 7, "TCP" if i % 4 else "UDP",
                                                   "" if i % 2 else "10.1.0.%d" % (i % 4))]
    cluster, _ = encode_cluster(nodes)
    enc = encode_pods(cluster, pods)
    prof = _prof(pct)
    eng, ora = _engine(cluster, prof), Oracle(cluster, prof)
    for i in range(300):
        _compare_cycle(eng.eval_pod(enc, i), ora.cycle(enc, i), f"pod {i}")
    _batch_vs_oracle(cluster, enc, pct=pct)


@pytest.mark.parametrize("pct", [0, 100])
def test_image_locality_vs_oracle(pct):
    """ImageLocality on the device: nodes with image lists, pods with container
    images (per-pod path) mixed with image-less batchable pods."""
    from ksim.encode import encode_cluster, encode_pods
    mb = 1024 * 1024
    nodes, pods = gen.config1_objects(n_nodes=160, n_pods=800)
    for i, n in enumerate(nodes):
        n.images = [(["app:%d" % (i % 4)], (60 + 90 * (i % 5)) * mb)]
        if i % 7 == 0:
            n.images.append((["base/os"], 1500 * mb))
    for i, p in enumerate(pods):
        if i % 2 == 0:
            p.containers[0].image = "app:%d" % (i % 5)
        if i % 6 == 0:
            p.containers[0].image = "base/os:latest"
    cluster, _ = encode_cluster(nodes)
    enc = encode_pods(cluster, pods)
    prof = _prof(pct)
    eng, ora = _engine(cluster, prof), Oracle(cluster, prof)
    for i in range(200):
        _compare_cycle(eng.eval_pod(enc, i), ora.cycle(enc, i), f"pod {i}")
    _batch_vs_oracle(cluster, enc, pct=pct)


def test_ingested_template_cluster():
    """The reference's import document + UI templates through ksim.ingest, on the device."""
    import test_ingest
    from ksim import ingest
    snap = ingest.load(test_ingest._template_cluster(n_nodes=160, n_pods=2000))
    cluster, enc, _ = ingest.encode(snap)
    _batch_vs_oracle(cluster, enc, pct=0)


@pytest.mark.parametrize("pct", [0, 100])
def test_extender_cycles_vs_oracle(pct):
    """ksim_eval_pod_filter / _finish around a deterministic extender, cycle by
    cycle against the oracle's extender cycle (configs 1 and 3 shapes)."""
    import test_extender
    for cluster, pods in (gen.config1(n_nodes=160, n_pods=120),
                          gen.config3(n_nodes=200, pods_per_node=10, n_incoming=80, seed=3, zone_anti_every=20)):
        fail, score = test_extender.extender_model(cluster.node_names)
        prof = _prof(pct)
        eng, ora = _engine(cluster, prof), Oracle(cluster, prof)
        seen = set()

        def ext(filtered):
            kept = filtered["fail_plugin"] == abi.PASSED
            seen.add(int(kept.sum()))
            return fail, score

        for i in range(pods.n_pods):
            _compare_cycle(eng.eval_pod_extenders(pods, i, ext), ora.cycle(pods, i, fail, score), f"pod {i}")
        es, os_ = eng.node_state(), ora.node_state()
        for k in es:
            np.testing.assert_array_equal(es[k], os_[k])


@pytest.mark.parametrize("n_nodes", [40, 1500])
def test_preemption_vs_oracle(n_nodes):
    """DefaultPreemption dry run on the device (ksim_preempt) against the oracle:
    nominated node, victims in reprieve order, potential nodes, candidates kept
    (1,500 nodes: more than 100 candidates, so numCandidates cuts the scan)."""
    import test_preemption
    from ksim.encode import encode_cluster, encode_pods
    from ksim.model import Container, Pod
    from ksim.preemption import bound_table
    nodes, bound, start, order = test_preemption.crowded(n_nodes=n_nodes, seed=7)
    cluster, _ = encode_cluster(nodes, bound)
    table = bound_table(cluster, bound, start)
    rng = np.random.default_rng(11)
    pods = [Pod(f"p{i}", priority=int(rng.choice([0, 5, 50, 500, 5000])),
                containers=[Container({"cpu": f"{int(rng.integers(10, 400)) * 100}m",
                                       "memory": f"{int(rng.integers(4, 40))}Gi"})]) for i in range(40)]
    enc = encode_pods(cluster, pods)
    prof = _prof(100)
    eng, ora = _engine(cluster, prof), Oracle(cluster, prof)
    eng.set_bound_pods(table)
    many = 0
    for i, pod in enumerate(pods):
        got = eng.preempt(enc, i, pod.priority)
        want = ora.preempt(enc, i, pod.priority, table)
        assert got == want, f"pod {i}: engine {got[:1]} {got[2:]} oracle {want[:1]} {want[2:]}"
        many += want[3] >= 100
    if n_nodes > 1000:
        assert many > 0


# ---- NetworkBandwidth (the simulator's out-of-tree plugin) -------------------------
def _nb_case(pct, node_errors, pod_errors, filt=True, score=True, n_nodes=150, n_pods=300):
    import test_netbw
    from ksim.encode import encode_cluster, encode_pods
    nodes, bound, pending = gen.netbw_objects(n_nodes=n_nodes, n_pods=n_pods, node_errors=node_errors,
                                              pod_errors=pod_errors)
    sp = test_netbw.nb_profile(pct, filt=filt, score=score)
    cluster, _ = encode_cluster(nodes, bound, nb_args=sp.network_bandwidth)
    return cluster, encode_pods(cluster, pending), profile.compile_profile(sp)


@pytest.mark.parametrize("pct", [0, 100])
@pytest.mark.parametrize("errors", [False, True])
def test_network_bandwidth_compat_cycles(pct, errors):
    cluster, pods, prof = _nb_case(pct, errors, errors)
    eng, ora = _engine(cluster, prof), Oracle(cluster, prof)
    statuses = set()
    for i in range(pods.n_pods):
        e, o = eng.eval_pod(pods, i), ora.cycle(pods, i)
        _compare_cycle(e, o, f"pod {i}")
        statuses.add(o["status"])
    np.testing.assert_array_equal(eng.nb_alloc(), ora.nb_alloc())
    assert (abi.STATUS_ERROR in statuses) == errors


@pytest.mark.parametrize("pct", [0, 100])
def test_network_bandwidth_batch_and_score_only(pct):
    for filt, score in ((True, True), (False, True), (True, False)):
        cluster, pods, prof = _nb_case(pct, True, True, filt, score, n_nodes=300, n_pods=600)
        eng, ora = _engine(cluster, prof), Oracle(cluster, prof)
        chosen, st = eng.schedule_batch(pods)
        want, ost = ora.schedule(pods)
        np.testing.assert_array_equal(chosen, want, err_msg=f"filter={filt} score={score}")
        assert st.evals == ost.evals and eng.next_start == ora.next_start
        assert (chosen == abi.CHOSEN_ERROR).any()
        np.testing.assert_array_equal(eng.nb_alloc(), ora.nb_alloc())


def test_network_bandwidth_extender_cycles():
    import test_extender
    cluster, pods, prof = _nb_case(0, True, True, n_pods=120)
    fail, score = test_extender.extender_model(cluster.node_names)
    eng, ora = _engine(cluster, prof), Oracle(cluster, prof)
    for i in range(pods.n_pods):
        _compare_cycle(eng.eval_pod_extenders(pods, i, lambda f: (fail, score)), ora.cycle(pods, i, fail, score),
                       f"pod {i}")
