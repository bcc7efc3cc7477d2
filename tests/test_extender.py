"""Extenders: findNodesThatPassExtenders after the window and
the extenders' scores added before selectHost.  The C oracle (ext arrays per
node) against the object-level restatement (an extender callback on the kept
list), cycle by cycle; the GPU two-phase API is in tests/test_gpu_parity.py."""
import zlib

import numpy as np
import pytest

from ksim import abi, gen, profile
from ksim.encode import encode_cluster, encode_pods
from oracle.objref import ObjScheduler
from oracle.oracle import Oracle


def extender_model(names):
    """A deterministic extender: drops ~1/5 of the nodes, scores 0..10 x weight 3 x (100 / 10)."""
    h = np.array([zlib.crc32(n.encode()) for n in names], np.uint64)
    fail = (h % 5 == 0).astype(np.uint8)
    score = ((h // 7) % 11).astype(np.int64) * 3 * 10
    return fail, score


@pytest.mark.parametrize("pct", [0, 100])
def test_extender_cycles_vs_objref(pct):
    nodes, pods = gen.config1_objects(n_nodes=160, n_pods=200)
    cluster, _ = encode_cluster(nodes)
    enc = encode_pods(cluster, pods)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=pct)
    ora = Oracle(cluster, profile.compile_profile(sp))
    ref = ObjScheduler(nodes, [], pct=pct, seed=sp.tiebreak_seed)
    fail, score = extender_model(cluster.node_names)
    by_name = {n: (int(f), int(s)) for n, f, s in zip(cluster.node_names, fail, score)}

    def ext(kept):
        return {n for n in kept if by_name[n][0]}, {n: by_name[n][1] for n in kept}

    filtered = 0
    for i, pod in enumerate(pods):
        o = ora.cycle(enc, i, fail, score)
        r = ref.cycle(pod, extender=ext)
        assert o["n_feasible"] == r["n_feasible"], i
        got = cluster.node_names[o["chosen"]] if o["chosen"] >= 0 else None
        assert got == r["chosen"], i
        for pos in np.nonzero(o["scored"])[0]:
            assert o["total"][pos] == r["total"][cluster.node_names[pos]], (i, pos)
        ext_out = np.nonzero(o["fail_plugin"] == abi.FAIL_EXTENDER)[0]
        assert all(r["filter"][cluster.node_names[p]][0] == "extender" for p in ext_out)
        filtered += len(ext_out)
    assert filtered > 0
