"""Host encoder: Quantity parsing, request sums, nodeTree order, tolerations,
node-selector compilation — the per-pod precomputation upstream does in
PreFilter/PreScore (computePodResourceRequest, GetNonzeroRequests,
nodeTree.list, ToleratesTaint, nodeSelectorRequirementsAsSelector)."""
import numpy as np
import pytest

from ksim import abi
from ksim.encode import (encode_cluster, encode_pods, node_tree_order, pod_nonzero_requests,
                         pod_requests, zone_key)
from ksim.model import (Container, Node, NodeSelectorTerm, Pod, Requirement, Taint, Toleration,
                        node_from_dict, parse_quantity, pod_from_dict, quantity_milli_value,
                        quantity_value)


@pytest.mark.parametrize("q,value,milli", [
    ("100m", 1, 100), ("1", 1, 1000), ("1.5", 2, 1500), ("16Gi", 16 << 30, (16 << 30) * 1000),
    ("128Mi", 128 << 20, (128 << 20) * 1000), ("1k", 1000, 10 ** 6), ("1e3", 1000, 10 ** 6),
    ("0.5", 1, 500), ("250m", 1, 250), ("2", 2, 2000),
])
def test_quantity(q, value, milli):
    assert quantity_value(q) == value
    assert quantity_milli_value(q) == milli


def test_quantity_invalid():
    with pytest.raises(ValueError):
        parse_quantity("12Q")


def test_pod_requests_init_max_and_overhead():
    p = Pod("p", containers=[Container({"cpu": "100m", "memory": "1Gi"}), Container({"cpu": "200m"})],
            init_containers=[Container({"cpu": "500m", "memory": "512Mi"})],
            overhead={"cpu": "10m", "memory": "1Mi"})
    r = pod_requests(p)
    assert r["cpu"] == 500 + 10                       # max(300, 500) + overhead
    assert r["memory"] == (1 << 30) + (1 << 20)       # max(1Gi, 512Mi) + overhead
    cpu, mem = pod_nonzero_requests(p)
    assert cpu == 500 + 10                            # max(100+200, 500) + overhead
    assert mem == max((1 << 30) + 200 * 1024 * 1024, 512 << 20) + (1 << 20)


def test_nonzero_defaults_for_missing_requests():
    p = Pod("p", containers=[Container({}), Container({"cpu": "0"})])
    assert pod_requests(p).get("cpu", 0) == 0
    cpu, mem = pod_nonzero_requests(p)
    assert cpu == 100 + 0                             # unset -> 100m, explicit 0 stays 0
    assert mem == 2 * 200 * 1024 * 1024


def test_zone_key_and_node_tree_order():
    labels = [{"topology.kubernetes.io/zone": "a"}, {"topology.kubernetes.io/zone": "a"},
              {"topology.kubernetes.io/zone": "b"}, {}, {"topology.kubernetes.io/zone": "b"},
              {"topology.kubernetes.io/zone": "a"}]
    keys = [zone_key(l) for l in labels]
    assert keys[0] == ":\x00:a" and keys[3] == ""
    # zones in insertion order: a, b, ""; round-robin, insertion order within a zone
    assert node_tree_order(keys) == [0, 2, 3, 1, 4, 5]


def test_tolerations():
    t = Taint("k", "v", "NoSchedule")
    assert Toleration("k", "Equal", "v", "NoSchedule").tolerates(t)
    assert Toleration("k", "", "v", "").tolerates(t)
    assert not Toleration("k", "Equal", "w", "").tolerates(t)
    assert Toleration("k", "Exists", "", "").tolerates(t)
    assert Toleration("", "Exists", "", "").tolerates(t)
    assert not Toleration("k", "Exists", "", "NoExecute").tolerates(t)


def _cluster():
    nodes = [
        Node("n0", {"zone": "a", "size": "10"}, [Taint("spot", "true", "PreferNoSchedule")],
             {"cpu": "4", "memory": "8Gi", "pods": "110"}),
        Node("n1", {"zone": "b", "size": "x"}, [Taint("dedicated", "gpu", "NoSchedule")],
             {"cpu": "8", "memory": "16Gi", "pods": "110", "example.com/gpu": "2"}),
    ]
    return encode_cluster(nodes)[0]


def test_encode_cluster_vocab():
    c = _cluster()
    assert c.n_nodes == 2 and c.scalar_names == ["example.com/gpu"]
    assert list(c.alloc_cpu) == [4000, 8000]
    assert list(c.alloc_scalar[0]) == [0, 2]
    assert [t.key for t in c.taint_vocab[1:]] == ["spot", "dedicated"]
    assert list(c.taint_effect) == [0, abi.EFFECT_PREFER_NO_SCHEDULE, abi.EFFECT_NO_SCHEDULE]
    col = c.label_col("size")
    nums = c.label_num[c.label_col_offset[col]:]
    oks = c.label_num_ok[c.label_col_offset[col]:]
    assert nums[c.value_id(col, "10")] == 10 and oks[c.value_id(col, "10")] == 1
    assert oks[c.value_id(col, "x")] == 0


def test_encode_pod_expressions():
    c = _cluster()
    p = Pod("p", containers=[Container({"cpu": "1", "example.com/gpu": "1"})],
            node_selector={"zone": "b"},
            required_terms=[NodeSelectorTerm([Requirement("size", "Gt", ["5"])]),
                            NodeSelectorTerm([Requirement("zone", "NotIn", ["zz"])]),
                            NodeSelectorTerm([Requirement("missing", "DoesNotExist")]),
                            NodeSelectorTerm([Requirement("zone", "In", [])]),
                            NodeSelectorTerm([])],
            tolerations=[Toleration("dedicated", "Exists")])
    e = encode_pods(c, [p])
    rec = e.pods[0]
    assert rec["flags"] & abi.POD_HAS_REQUIRED_AFFINITY and rec["flags"] & abi.POD_HAS_SCALAR
    assert rec["scalar_req"][0] == 1 and rec["req_cpu"] == 1000
    ops = [int(x["op"]) for x in e.exprs]
    assert ops == [abi.OP_IN, abi.OP_GT, abi.OP_TRUE, abi.OP_TRUE, abi.OP_FALSE]
    assert [int(t["n_expr"]) for t in e.terms] == [1, 1, 1, 1, 0]
    assert int(rec["tol_filter"][0]) == 0b100        # tolerates taint id 2 only
    assert int(rec["tol_prefer"][0]) == 0b100        # effect "" also counts for PreferNoSchedule


def test_from_dict_roundtrip():
    n = node_from_dict({"metadata": {"name": "n", "labels": {"a": "b"}},
                        "spec": {"taints": [{"key": "k", "value": "v", "effect": "NoSchedule"}],
                                 "unschedulable": True},
                        "status": {"allocatable": {"cpu": "4", "memory": "32Gi", "pods": "110"}}})
    assert n.unschedulable and n.taints[0].key == "k" and n.allocatable["cpu"] == "4"
    p = pod_from_dict({"metadata": {"name": "p", "namespace": "ns"},
                       "spec": {"containers": [{"resources": {"requests": {"cpu": "100m"}},
                                                "ports": [{"containerPort": 80, "hostPort": 8080}]}],
                                "affinity": {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
                                    "nodeSelectorTerms": [{"matchExpressions": [
                                        {"key": "a", "operator": "In", "values": ["b"]}]}]}}},
                                "volumes": [{"name": "x", "persistentVolumeClaim": {"claimName": "c"}}]}})
    assert p.required_terms[0].match_expressions[0].values == ["b"]
    assert p.containers[0].host_ports == [8080] and p.pvc_claims == ["c"] and not p.has_volumes
    c, _ = encode_cluster([n])
    e = encode_pods(c, [p])
    rec = e.pods[0]
    # host ports compile to a NodePorts use (class of pods on 0.0.0.0:8080/TCP); a claim without a
    # VolumeIndex (no PVs / PVCs given) stays unsupported
    assert not rec["flags"] & abi.POD_HAS_HOST_PORTS and rec["flags"] & abi.POD_HAS_VOLUMES
    assert rec["use_count"] == 1 and e.uses[rec["use_first"]]["kind"] == abi.USE_NODE_PORT


def test_bound_pods_fill_node_info():
    nodes = [Node("n0", {}, [], {"cpu": "4", "memory": "8Gi", "pods": "110"})]
    bound = [Pod("b", containers=[Container({"cpu": "250m"})], node_name="n0")]
    c, _ = encode_cluster(nodes, bound)
    assert c.req_cpu[0] == 250 and c.req_mem[0] == 0
    assert c.nz_cpu[0] == 250 and c.nz_mem[0] == 200 * 1024 * 1024 and c.num_pods[0] == 1
