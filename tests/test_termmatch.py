"""Selector / affinity-term matching as an int8 contraction (SURVEY §2.3 K8,
ksim/termmatch.py, csrc/ksim_match.hip).

The host class compiler (ksim/topology.py, pinned against the object-level
restatement oracle/objref.py by tests/test_topology.py) is the checker: an
encoding whose classes were matched through ``ksim_match_terms`` must equal
the host-matched encoding array for array (class counts, uses, adds, pod
records).  On the CPU a numpy restatement of the contraction stands in for the
device (it checks the requirement / feature compilation); the ``gpu`` tests
run the HIP kernels through the C ABI."""
import numpy as np
import pytest

from ksim import gen
from ksim.encode import encode_cluster, encode_pods
from ksim.model import (Container, LabelSelector, Node, Pod, PodAffinityTerm, Requirement,
                        TopologySpreadConstraint, WeightedPodAffinityTerm)
from ksim.termmatch import MatchProblem, expand_rows, unpack_bits


class NumpyMatcher:
    """The contraction of csrc/ksim_match.hip restated with numpy (checker)."""

    def __init__(self):
        self.calls = 0

    def match(self, mp: MatchProblem):
        self.calls += 1
        nf = max(len(mp.feat), 1)
        a = np.zeros((mp.n_sigs, nf), np.int32)
        for s in range(mp.n_sigs):
            a[s, mp.sig_feat[mp.sig_off[s]:mp.sig_off[s + 1]]] = 1
        b = np.zeros((nf, len(mp.req_neg)), np.int32)
        for r in range(len(mp.req_neg)):
            b[mp.req_feat[mp.req_off[r]:mp.req_off[r + 1]], r] = 1
        sat = (a @ b > 0) != mp.neg.astype(bool)[None, :]
        hit = np.ones((mp.n_sigs, mp.n_matchers), bool)
        for m in range(mp.n_matchers):
            for r in mp.m_req[mp.m_off[m]:mp.m_off[m + 1]]:
                hit[:, m] &= sat[:, r]
        counts = np.zeros((mp.class_matcher.size, mp.n_nodes), np.int32)
        for c, m in enumerate(mp.class_matcher):
            np.add.at(counts[c], mp.pod_node[hit[mp.pod_sig, m]], 1)
        return expand_rows(mp, hit), counts


def encode_both(nodes, bound, pods, matcher, namespaces=None):
    ch, _ = encode_cluster(nodes, bound, namespaces=namespaces)
    eh = encode_pods(ch, pods)
    cd, _ = encode_cluster(nodes, bound, namespaces=namespaces, matcher=matcher)
    ed = encode_pods(cd, pods)
    return (ch, eh), (cd, ed)


def assert_same(host, dev):
    (ch, eh), (cd, ed) = host, dev
    assert ch.topo.keys == cd.topo.keys
    np.testing.assert_array_equal(ch.class_count, cd.class_count)
    np.testing.assert_array_equal(eh.uses, ed.uses)
    np.testing.assert_array_equal(eh.adds, ed.adds)
    np.testing.assert_array_equal(eh.pods, ed.pods)


LABEL_KEYS = ["app", "tier", "team", "env", "track"]
LABEL_VALS = ["a", "b", "c", "d"]


def _labels(rng):
    return {k: LABEL_VALS[rng.integers(4)] for k in LABEL_KEYS if rng.random() < 0.6}


def _selector(rng):
    """Random LabelSelector with every operator, or None (nil) / {} (everything)."""
    x = rng.random()
    if x < 0.05:
        return None
    if x < 0.1:
        return LabelSelector()
    ml = {LABEL_KEYS[rng.integers(5)]: LABEL_VALS[rng.integers(4)] for _ in range(rng.integers(0, 2))}
    ex = []
    for _ in range(rng.integers(0, 3)):
        k = LABEL_KEYS[rng.integers(5)]
        op = ["In", "NotIn", "Exists", "DoesNotExist"][rng.integers(4)]
        vals = list(rng.choice(LABEL_VALS + ["zz"], size=rng.integers(1, 3), replace=False)) if op in ("In", "NotIn") else []
        ex.append(Requirement(k, op, vals))
    return LabelSelector(ml, ex)


def _term(rng, namespaces):
    key = ["kubernetes.io/hostname", "topology.kubernetes.io/zone"][rng.integers(2)]
    x = rng.random()
    if x < 0.2:
        return PodAffinityTerm(key, _selector(rng), namespaces=list(rng.choice(namespaces, size=2, replace=False)))
    if x < 0.3:
        return PodAffinityTerm(key, _selector(rng), namespace_selector=LabelSelector())
    if x < 0.4:
        return PodAffinityTerm(key, _selector(rng), namespace_selector=LabelSelector({"env": "prod"}))
    return PodAffinityTerm(key, _selector(rng))


def random_scenario(seed, n_nodes=40, n_bound=300, n_pods=80, n_terms=4, p_term=0.2):
    rng = np.random.default_rng(seed)
    namespaces = {"default": {"env": "prod"}, "web": {"env": "prod"}, "batch": {"env": "dev"}, "ops": {}}
    ns_names = list(namespaces)
    nodes = [Node(name=f"n{i:03d}", labels={"kubernetes.io/hostname": f"n{i:03d}",
                                            "topology.kubernetes.io/zone": f"z{i % 3}"},
                  allocatable={"cpu": "64", "memory": "256Gi", "pods": "110"}) for i in range(n_nodes)]

    # a pool of terms (a pod's topology uses are capped at 16: carried terms of
    # other pods that match it count too)
    pool = [_term(rng, ns_names) for _ in range(n_terms)]

    def term():
        return pool[rng.integers(n_terms)]

    def pod(name, node=""):
        p = Pod(name=name, namespace=ns_names[rng.integers(4)], labels=_labels(rng),
                containers=[Container({"cpu": "100m", "memory": "128Mi"})], node_name=node)
        if rng.random() < p_term:
            p.pod_anti_affinity_required = [term()]
        if rng.random() < p_term:
            p.pod_affinity_required = [term() for _ in range(rng.integers(1, 3))]
        if rng.random() < p_term:
            p.pod_affinity_preferred = [WeightedPodAffinityTerm(int(rng.integers(1, 100)), term())]
        if rng.random() < p_term:
            p.pod_anti_affinity_preferred = [WeightedPodAffinityTerm(int(rng.integers(1, 100)), term())]
        return p

    bound = [pod(f"b{j}", nodes[rng.integers(n_nodes)].name) for j in range(n_bound)]
    pods = []
    for j in range(n_pods):
        p = pod(f"p{j}")
        if rng.random() < 0.5:
            p.topology_spread = [TopologySpreadConstraint(1 + int(rng.integers(2)), "topology.kubernetes.io/zone",
                                                          "DoNotSchedule", _selector(rng))]
        pods.append(p)
    return nodes, bound, pods, namespaces


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_numpy_contraction_random_selectors(seed):
    nodes, bound, pods, ns = random_scenario(seed)
    m = NumpyMatcher()
    host, dev = encode_both(nodes, bound, pods, m, namespaces=ns)
    assert m.calls == 2                      # encode_cluster + encode_pods
    assert_same(host, dev)


def test_numpy_contraction_config3_small():
    nodes, bound, pods = gen.config3_objects(n_nodes=300, pods_per_node=4, n_incoming=200, zone_anti_every=50)
    host, dev = encode_both(nodes, bound, pods, NumpyMatcher())
    assert_same(host, dev)


def test_unpack_bits():
    w = np.array([[0x80000001, 0x2]], np.uint32)
    b = unpack_bits(w, 34)
    assert list(np.flatnonzero(b[0])) == [0, 31, 33]


# ---- device --------------------------------------------------------------------
@pytest.fixture(scope="module")
def engine():
    from ksim.engine import Engine
    e = Engine(0)
    yield e
    e.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_device_match_random_selectors(engine, seed):
    from ksim.termmatch import DeviceMatcher
    nodes, bound, pods, ns = random_scenario(seed, n_nodes=64, n_bound=2000, n_pods=300, n_terms=3, p_term=0.15)
    m = DeviceMatcher(engine)
    host, dev = encode_both(nodes, bound, pods, m, namespaces=ns)
    assert m.calls == 2
    assert_same(host, dev)


@pytest.mark.gpu
def test_device_match_config3_full(engine):
    """BASELINE config 3 at full size: 10,000 nodes, 100,000 bound pods with
    anti-affinity terms, 10,000 incoming pods."""
    from ksim.termmatch import DeviceMatcher
    nodes, bound, pods = gen.config3_objects()
    host, dev = encode_both(nodes, bound, pods, DeviceMatcher(engine))
    assert_same(host, dev)


@pytest.mark.gpu
def test_device_match_many_requirements(engine):
    """More requirement column tiles than waves and a feature axis of several
    k-steps: 600 distinct In selectors over 600 label values."""
    from ksim.termmatch import DeviceMatcher
    nodes = [Node(name=f"n{i}", labels={"kubernetes.io/hostname": f"n{i}"},
                  allocatable={"cpu": "64", "memory": "64Gi", "pods": "110"}) for i in range(50)]
    bound = [Pod(name=f"b{j}", labels={"app": f"v{j % 600}", "x": f"{j % 7}"},
                 containers=[Container({"cpu": "10m"})], node_name=f"n{j % 50}") for j in range(3000)]
    pods = [Pod(name=f"p{j}", labels={"app": f"v{(7 * j) % 600}"}, containers=[Container({"cpu": "10m"})],
                pod_anti_affinity_preferred=[WeightedPodAffinityTerm(5, PodAffinityTerm(
                    "kubernetes.io/hostname", LabelSelector(match_expressions=[
                        Requirement("app", "In", [f"v{j % 600}", f"v{(j + 1) % 600}"]),
                        Requirement("x", "NotIn", [f"{j % 7}"])])))])
            for j in range(600)]
    host, dev = encode_both(nodes, bound, pods, DeviceMatcher(engine))
    assert_same(host, dev)


def _exists_problem(n_sigs, n_keys=17, seed=0):
    """Signatures labelled with the keys of the bits of their index (distinct
    feature sets), matchers Exists(a) AND DoesNotExist(b) over key pairs."""
    from ksim.topology import Matcher
    rng = np.random.default_rng(seed)
    keys = [f"k{i}" for i in range(n_keys)]
    sigs = [("default", tuple(sorted((keys[b], "v") for b in range(n_keys) if (s >> b) & 1))) for s in range(n_sigs)]
    ms = []
    for a in range(n_keys):
        b = (a * 5 + 3) % n_keys
        sel = LabelSelector(match_expressions=[Requirement(keys[a], "Exists", []), Requirement(keys[b], "DoesNotExist", [])])
        ms.append(Matcher(frozenset(["default"]), False, sel.key()))
    mp = MatchProblem(None, ms, sigs)
    n_pods, n_nodes = 4 * n_sigs, 50
    mp.set_counts(rng.integers(0, n_sigs, n_pods), rng.integers(0, n_nodes, n_pods), n_nodes, np.arange(len(ms)))
    return mp, sigs, ms


def test_signatures_with_equal_features_share_a_row():
    """Labels no requirement names do not split a signature's row."""
    from ksim.topology import Matcher
    sel = LabelSelector({"app": "a"})
    ms = [Matcher(frozenset(["default"]), False, sel.key())]
    sigs = [("default", (("app", "a"), ("pod", f"x{i}"))) for i in range(100)] + [("default", (("app", "b"),))]
    mp = MatchProblem(None, ms, sigs)
    assert mp.n_sigs == 2 and list(mp.sig_row[:3]) == [0, 0, 0] and mp.sig_row[100] == 1
    mp.set_counts(np.arange(101), np.zeros(101, np.int64), 1, [0])
    hit, counts = NumpyMatcher().match(mp)
    assert hit.shape == (101, 1) and hit[:100, 0].all() and not hit[100, 0]
    assert counts.tolist() == [[100]]


@pytest.mark.gpu
def test_device_match_more_rows_than_grid_y(engine):
    """70,000 distinct signature rows (more than the 65,536 blocks of a grid's
    y dimension) and 280,000 bound pods: bits and class counts vs numpy."""
    from ksim.termmatch import DeviceMatcher
    mp, _, _ = _exists_problem(70000)
    assert mp.n_sigs == 70000
    hd, cd = DeviceMatcher(engine).match(mp)
    hn, cn = NumpyMatcher().match(mp)
    np.testing.assert_array_equal(hd, hn)
    np.testing.assert_array_equal(cd, cn)
