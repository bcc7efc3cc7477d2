"""GPU parity, round-2 cases: the HIP engine (through the C ABI) against the
oracle, bit-exact.

- NodeAffinity's PreFilterResult restricting the scan;
- selectHost over full int64 totals: large weights (the batch paths' 20-bit
  key gate) and extender scores far outside a 20-bit field;
- a policy sweep on ONE handle exactly as bench.py runs config 5
  (ksim_set_profile keeping the captured batch graphs, ksim_load_pods reusing
  the pod buffers);
- resource edge cases (allocatable 0, overcommitted nodes, quantities past
  2^52 and 2^56, weight 0);
- every BASELINE config at full size: config 2 (50,000 pods, both modes),
  config 3 (10,000 nodes, 100,000 existing pods), config 4 (100,000 nodes as
  an in-process 8-shard group), config 5 (16 weight vectors);
- the Go-harness fixtures (tests/golden/go) through the engine.
"""
import gzip
import json
import os

import numpy as np
import pytest

from ksim import abi, gen, profile
from ksim.encode import encode_cluster, encode_pods
from ksim.engine import Engine, group_schedule_loaded
from ksim.shard import partition
from oracle.oracle import Oracle
from test_gpu_parity import _batch_vs_oracle, _compare_cycle, _prof

pytestmark = pytest.mark.gpu

BIG_W = {"NodeResourcesBalancedAllocation": 900001, "ImageLocality": 1, "InterPodAffinity": 7,
         "NodeResourcesFit": 1234567, "NodeAffinity": 40000, "PodTopologySpread": 2, "TaintToleration": 3}


def _engine(cluster, prof):
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(cluster)
    return eng


def _same_state(eng, ora):
    es, os_ = eng.node_state(), ora.node_state()
    for k in es:
        np.testing.assert_array_equal(es[k], os_[k], err_msg=k)


# ---- NodeAffinity PreFilterResult ---------------------------------------------------
@pytest.mark.parametrize("pct", [0, 100])
def test_prefilter_node_names_compat(pct):
    nodes, pods = gen.prefilter_objects(n_nodes=300, n_pods=360)
    cluster, _ = encode_cluster(nodes)
    enc = encode_pods(cluster, pods)
    prof = _prof(pct)
    eng, ora = _engine(cluster, prof), Oracle(cluster, prof)
    statuses = set()
    for i in range(enc.n_pods):
        e, o = eng.eval_pod(enc, i), ora.cycle(enc, i)
        _compare_cycle(e, o, f"pod {i}")
        statuses.add(o["status"])
    _same_state(eng, ora)
    assert {abi.STATUS_SCHEDULED, abi.STATUS_UNSCHEDULABLE, abi.STATUS_ERROR} <= statuses


@pytest.mark.parametrize("pct", [0, 100])
def test_prefilter_node_names_batch(pct):
    """Restricted pods (per-pod path) interleaved with batchable ones: the
    restricted scans move nextStartNodeIndex mod their length."""
    nodes, pods = gen.prefilter_objects(n_nodes=1200, n_pods=2400)
    for n in nodes:
        n.taints = [t for t in n.taints if t.effect != "PreferNoSchedule"]
    cluster, _ = encode_cluster(nodes)
    enc = encode_pods(cluster, pods)
    st = _batch_vs_oracle(cluster, enc, pct=pct)
    assert st.perpod_cycles > 0 and st.batches > 0


# ---- selectHost over full int64 totals ---------------------------------------------
@pytest.mark.parametrize("pct", [0, 100])
def test_large_weights_compat(pct):
    cluster, pods = gen.config1(n_nodes=120, n_pods=200)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=pct).with_weights(BIG_W)
    prof = profile.compile_profile(sp)
    eng, ora = _engine(cluster, prof), Oracle(cluster, prof)
    top = 0
    for i in range(pods.n_pods):
        e, o = eng.eval_pod(pods, i), ora.cycle(pods, i)
        _compare_cycle(e, o, f"pod {i}")
        top = max(top, int(o["total"].max()))
    assert top >= 1 << 20


@pytest.mark.parametrize("pct", [0, 100])
def test_large_weights_batch_gate(pct):
    """100 x (w_fit + w_ba) >= 2^20: the pods leave the batch path for the
    per-pod path (exact for any total); just below the bound they stay."""
    cluster, pods = gen.config2(n_nodes=1500, n_pods=2500)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=pct)
    for w, batched in ((BIG_W, False), ({"NodeResourcesFit": 5000, "NodeResourcesBalancedAllocation": 5485}, True)):
        prof = profile.compile_profile(sp.with_weights(w))
        eng = _engine(cluster, prof)
        chosen, st = eng.schedule_batch(pods)
        ora = Oracle(cluster, prof)
        ochosen, ost = ora.schedule(pods, nthreads=8)
        np.testing.assert_array_equal(chosen, ochosen)
        assert st.evals == ost.evals and eng.next_start == ora.next_start
        assert (st.perpod_cycles == 0) == batched and (st.batches > 0) == batched


@pytest.mark.parametrize("pct", [0, 100])
def test_extender_scores_beyond_key_field(pct):
    import test_extender
    cluster, pods = gen.config1(n_nodes=160, n_pods=150)
    fail, score = test_extender.extender_model(cluster.node_names)
    score = (score - 150) * 10000 * 37                   # weights x 10^4, both signs
    prof = _prof(pct)
    eng, ora = _engine(cluster, prof), Oracle(cluster, prof)
    for i in range(pods.n_pods):
        _compare_cycle(eng.eval_pod_extenders(pods, i, lambda f: (fail, score)), ora.cycle(pods, i, fail, score),
                       f"pod {i}")
    _same_state(eng, ora)


# ---- policy sweep on one handle (config 5 as bench.py runs it) ---------------------
@pytest.mark.parametrize("case", ["fast", "generic", "adapt"])
def test_sweep_one_engine_reuses_graphs(case):
    """set_profile(w_k) -> load_pods (same queue, same buffers) ->
    reset_cluster -> schedule_loaded, on ONE engine: the batch graphs captured
    under the first vector replay under every later one (kernels read the
    profile from device memory) and the placements equal the oracle's."""
    cluster, pods = gen.config2(n_nodes=1500, n_pods=9000)
    pct = 0 if case == "adapt" else 100
    base = profile.SchedulerProfile(percentage_of_nodes_to_score=pct)
    if case == "generic":                                # bp.cpu_mem off: the generic evaluation kernel
        base.fit.resources = [("cpu", 2), ("memory", 1), ("ephemeral-storage", 1)]
    names = [p.name for p in base.score_plugins()]
    vectors = gen.config5_weights(6)
    eng = Engine(0)
    eng.set_profile(profile.compile_profile(base))
    eng.set_cluster(cluster)
    caps = None
    for k, v in enumerate(vectors):
        prof = profile.compile_profile(base.with_weights({n: int(x) for n, x in zip(names, v)}))
        eng.set_profile(prof)
        eng.load_pods(pods)
        eng.reset_cluster()
        chosen, st = eng.schedule_loaded(0, pods.n_pods)
        ochosen, ost = Oracle(cluster, prof).schedule(pods, nthreads=8)
        np.testing.assert_array_equal(chosen, ochosen, err_msg=f"vector {k}")
        assert st.evals == ost.evals and st.perpod_cycles == 0
        if k == 0:
            caps = eng.diag()["graph_captures"]
        else:
            assert eng.diag()["graph_captures"] == caps, "set_profile / load_pods dropped the batch graphs"


def test_config5_sweep_as_bench():
    """bench.py's config-5 loop on the config-5 cluster: 16 vectors, one engine."""
    cluster, pods = gen.config2(5000, 4500)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=100)
    names = [p.name for p in sp.score_plugins()]
    eng = Engine(0)
    eng.set_profile(profile.compile_profile(sp))
    eng.set_cluster(cluster)
    for k, v in enumerate(gen.config5_weights(16)):
        prof = profile.compile_profile(sp.with_weights({n: int(x) for n, x in zip(names, v)}))
        eng.set_profile(prof)
        eng.load_pods(pods)
        eng.reset_cluster()
        chosen, _ = eng.schedule_loaded(0, pods.n_pods)
        np.testing.assert_array_equal(chosen, Oracle(cluster, prof).schedule(pods, nthreads=16)[0],
                                      err_msg=f"vector {k}")


# ---- resource edge cases -----------------------------------------------------------
@pytest.mark.parametrize("pct", [0, 100])
def test_edge_quantities(pct):
    nodes, bound, pods = gen.edge_objects()
    cluster, _ = encode_cluster(nodes, bound)
    enc = encode_pods(cluster, pods)
    w0 = {"NodeResourcesBalancedAllocation": 0, "ImageLocality": 0, "InterPodAffinity": 0,
          "NodeResourcesFit": 3, "NodeAffinity": 0, "PodTopologySpread": 0, "TaintToleration": 0}
    for sp in (profile.SchedulerProfile(percentage_of_nodes_to_score=pct),
               profile.SchedulerProfile(percentage_of_nodes_to_score=pct).with_weights(w0)):
        prof = profile.compile_profile(sp)
        eng, ora = _engine(cluster, prof), Oracle(cluster, prof)
        for i in range(enc.n_pods):
            _compare_cycle(eng.eval_pod(enc, i), ora.cycle(enc, i), f"pod {i}")
        _same_state(eng, ora)
        _batch_vs_oracle(cluster, enc, pct=pct)


# ---- every BASELINE config at full size ----------------------------------------------
@pytest.mark.parametrize("pct", [100, 0])
def test_config2_full(pct):
    """Config 2 exactly as bench.py runs it: 5,000 nodes x 50,000 pods."""
    cluster, pods = gen.config2()
    prof = _prof(pct)
    eng = _engine(cluster, prof)
    chosen, st = eng.schedule_batch(pods)
    ora = Oracle(cluster, prof)
    ochosen, ost = ora.schedule(pods, nthreads=16)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals and st.scheduled == ost.scheduled and eng.next_start == ora.next_start
    _same_state(eng, ora)


def test_config3_full():
    """Config 3 at BASELINE size (10,000 nodes, 3 zones, 100,000 existing pods
    with anti-affinity terms): per-node outputs of the first 300 cycles, then
    placements and count classes over the next 1,700."""
    cluster, pods = gen.config3(n_incoming=2000)
    prof = _prof(100)
    eng, ora = _engine(cluster, prof), Oracle(cluster, prof)
    for i in range(300):
        _compare_cycle(eng.eval_pod(pods, i), ora.cycle(pods, i), f"pod {i}")
    rest = pods.subset(300, pods.n_pods - 300)
    chosen, st = eng.schedule_batch(rest)
    ochosen, ost = ora.schedule(rest, nthreads=16)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals
    np.testing.assert_array_equal(eng.class_count(), ora.class_count())
    _same_state(eng, ora)


@pytest.mark.parametrize("n_nodes,n_pods", [(100000, 3000), (20000, 6000)])
def test_node_stationary_p100(n_nodes, n_pods):
    """P100 batches past 8,192 nodes on one handle: the node-stationary
    evaluation (4 pods x a quarter of the nodes per block, the slice lists
    merged by the chain) on config 4's cluster (hash overlay) and on a
    20,000-node config-2 cluster (overlay indexed by node id)."""
    if n_nodes == 100000:
        cluster, pods = gen.config4(n_pods=n_pods)
    else:
        cluster, pods = gen.config2(n_nodes=n_nodes, n_pods=n_pods, seed=5)
    prof = _prof(100)
    eng = _engine(cluster, prof)
    chosen, st = eng.schedule_batch(pods)
    ora = Oracle(cluster, prof)
    ochosen, ost = ora.schedule(pods, nthreads=16)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals and st.scheduled == ost.scheduled
    assert st.perpod_cycles == 0 and st.batches > 0
    _same_state(eng, ora)


def test_config4_group8():
    """Config 4's cluster (100,000 nodes) as an in-process 8-shard group, the
    node-sharded exchange protocol on one device, for 20,000 pods."""
    cluster, pods = gen.config4(n_pods=20000)
    prof = _prof(100)
    engines = []
    for base, cnt in partition(cluster.n_nodes, 8):
        e = Engine(0)
        e.set_shard(base, cluster.n_nodes)
        e.set_profile(prof)
        e.set_cluster(cluster.shard(base, cnt))
        e.load_pods(pods)
        engines.append(e)
    chosen, st = group_schedule_loaded(engines, 0, pods.n_pods)
    ora = Oracle(cluster, prof)
    ochosen, ost = ora.schedule(pods, nthreads=16)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals and st.scheduled == ost.scheduled


@pytest.mark.parametrize("world", [1, 8])
def test_config4_adapt(world):
    """Config 4's cluster in the simulator's own mode (percentageOfNodesToScore
    0: K = 5,000 of 100,000, the wide k_adapt_top), 6,000 pods, on one handle
    and as an in-process 8-shard group (the node-sharded ADAPT batch protocol)."""
    cluster, pods = gen.config4(n_pods=6000)
    prof = _prof(0)
    if world == 1:
        eng = _engine(cluster, prof)
        chosen, st = eng.schedule_batch(pods)
        starts = [eng.next_start]
    else:
        engines = []
        for base, cnt in partition(cluster.n_nodes, world):
            e = Engine(0)
            e.set_shard(base, cluster.n_nodes)
            e.set_profile(prof)
            e.set_cluster(cluster.shard(base, cnt))
            e.load_pods(pods)
            engines.append(e)
        chosen, st = group_schedule_loaded(engines, 0, pods.n_pods)
        starts = [e.next_start for e in engines]
    ora = Oracle(cluster, prof)
    ochosen, ost = ora.schedule(pods, nthreads=16)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals and st.scheduled == ost.scheduled
    assert all(s == ora.next_start for s in starts)
    assert st.perpod_cycles == 0                     # every pod on the ADAPT batch path


def test_sweep_concurrent_engines():
    """bench.py config 5's concurrent form: weight vectors split over engines
    driven from host threads (own streams, own graphs); every vector's
    placements equal the sequential one-engine sweep's."""
    from concurrent.futures import ThreadPoolExecutor
    cluster, pods = gen.config2(n_nodes=1000, n_pods=2000)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=100)
    names = [p.name for p in sp.score_plugins()]
    profs = [profile.compile_profile(sp.with_weights({n: int(x) for n, x in zip(names, w)}))
             for w in gen.config5_weights(16)]
    ref = _engine(cluster, profs[0])
    want = []
    for pr in profs:
        ref.set_profile(pr)
        want.append(ref.schedule_batch(pods)[0])
        ref.reset_cluster()
    engs = [_engine(cluster, profs[0]) for _ in range(4)]

    def run(j):
        out = {}
        for v in range(j, len(profs), len(engs)):
            engs[j].set_profile(profs[v])
            engs[j].load_pods(pods)
            engs[j].reset_cluster()
            out[v] = engs[j].schedule_loaded(0, pods.n_pods)[0]
        return out

    got = {}
    with ThreadPoolExecutor(len(engs)) as ex:
        for part in ex.map(run, range(len(engs))):
            got.update(part)
    for v in range(len(profs)):
        np.testing.assert_array_equal(got[v], want[v], err_msg=f"vector {v}")


def test_persistent_tables_under_assume_forget():
    """The persistent domain tables follow binds made outside the loaded queue
    (ksim_assume / ksim_forget of single uploads: the class-index update path)
    and snapshot resets: an engine reading the tables must place every later
    pod exactly as one that recomputes the domain sums per cycle
    (k_topo_prefilter: the "ab" flavor), and both as the oracle before the binds."""
    cluster, pods = gen.config3(n_nodes=800, pods_per_node=6, n_incoming=900, seed=31, zone_anti_every=40)
    extra = pods.subset(800, 60)                     # same encoding: their adds name this cluster's classes
    prof = _prof(100)
    a = _engine(cluster, prof)
    a.load_pods(pods)
    b = Engine(0, variant="ab")
    b.set_profile(prof)
    b.set_cluster(cluster)
    b.load_pods(pods)
    ca, _ = a.schedule_loaded(0, 300)
    cb, _ = b.schedule_loaded(0, 300)
    np.testing.assert_array_equal(ca, cb)
    np.testing.assert_array_equal(ca, Oracle(cluster, prof).schedule(pods.subset(0, 300))[0])
    nodes = [(i * 37) % cluster.n_nodes for i in range(extra.n_pods)]
    for e in (a, b):
        for i, n in enumerate(nodes):
            e.assume(extra, i, n)
        for i in range(0, extra.n_pods, 3):
            e.forget(extra, i, nodes[i])
    ca, _ = a.schedule_loaded(300, pods.n_pods - 300)
    cb, _ = b.schedule_loaded(300, pods.n_pods - 300)
    np.testing.assert_array_equal(ca, cb)
    np.testing.assert_array_equal(a.class_count(), b.class_count())
    # a reset rebuilds the tables from the snapshot counts: the run repeats
    for e in (a, b):
        e.reset_cluster()
    ca2, _ = a.schedule_loaded(0, pods.n_pods)
    cb2, _ = b.schedule_loaded(0, pods.n_pods)
    np.testing.assert_array_equal(ca2, cb2)
    np.testing.assert_array_equal(ca2, Oracle(cluster, prof).schedule(pods)[0])


# ---- the Go-harness fixtures through the engine --------------------------------------
GO = sorted(p for p in __import__("glob").glob(os.path.join(os.path.dirname(__file__), "golden", "go", "*.json.gz"))
            if not p.endswith(".go.json.gz"))


@pytest.mark.parametrize("path", GO, ids=[os.path.basename(p).split(".")[0] for p in GO])
def test_go_fixtures_through_engine(path):
    """The recorded cycles of each fixture reproduced by the device: filter
    outcomes and messages, scores, totals, placement, nextStartNodeIndex.  The
    recorded cycles are oracle/objref.py's (objref regression pins, see
    tests/test_go_fixtures.py), not the Go plugins'."""
    import gofixture
    from ksim.wrapped import filter_message
    with gzip.open(path, "rb") as f:
        doc = json.loads(f.read())
    if not gofixture.plain(doc):
        pytest.skip("PodNominator / PostFilter cycles (objref replays them on the CPU)")
    cluster, enc, sp, prof = gofixture.encode(doc, encode_cluster, encode_pods)
    eng = _engine(cluster, prof)
    forder, names = sp.filter_order(), cluster.node_names
    snames = [p.name for p in sp.score_plugins()]
    for i, exp in enumerate(doc["expected"]):
        e = eng.eval_pod(enc, i)
        where = f"{os.path.basename(path)}: pod {exp['pod']}"
        for pos, name in enumerate(names):
            fp = int(e["fail_plugin"][pos])
            if fp == abi.NOT_EVALUATED:
                assert name not in exp["filter"], where
            elif fp == abi.PASSED:
                assert exp["filter"][name] == "passed", (where, name)
            else:
                assert exp["filter"][name] == [forder[fp], filter_message(cluster, forder[fp],
                                                                          int(e["fail_detail"][pos]))], (where, name)
        assert e["n_feasible"] == exp["nFeasible"] and e["next_start"] == exp["nextStartNodeIndex"], where
        if exp["nFeasible"] > 1:
            for k, pl in enumerate(snames):
                for name, raw in exp["score"][pl].items():
                    assert e["raw"][k][names.index(name)] == raw, (where, pl, name)
                    assert e["norm"][k][names.index(name)] == exp["normalized"][pl][name], (where, pl, name)
            for name, tot in exp["total"].items():
                assert e["total"][names.index(name)] == tot, (where, name)
        got = names[e["chosen"]] if e["chosen"] >= 0 else None
        assert got == exp["chosen"], where
