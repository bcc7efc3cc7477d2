"""The native snapshot encoder's outputs (ksim_encode_nodes / ksim_encode_pods)
drive the engine directly: configs 1 and 3 compiled natively, scheduled on
the GPU in both modes, placements and node state bit-exact against the C
oracle on the same arrays (tests/test_native_encode.py pins the arrays
byte for byte to the Python compile on the CPU)."""
import numpy as np
import pytest

from ksim import gen, nativeenc, profile
from ksim.engine import Engine
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("pct", [100, 0])
@pytest.mark.parametrize("kind", ["config1", "config3"])
def test_native_encoded_runs(kind, pct):
    if kind == "config1":
        nodes, pods_o = gen.config1_objects(n_nodes=600, n_pods=3000)
        bound = []
    else:
        nodes, bound, pods_o = gen.config3_objects(n_nodes=900, pods_per_node=4, n_incoming=600)
    cluster, pods = nativeenc.encode(nodes, bound, pods_o)
    prof = profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=pct))
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(cluster.copy_state())
    chosen, st = eng.schedule_batch(pods)
    ora = Oracle(cluster.copy_state(), prof)
    ochosen, ost = ora.schedule(pods)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals
    es, os_ = eng.node_state(), ora.node_state()
    for k in es:
        np.testing.assert_array_equal(es[k], os_[k], err_msg=k)
    np.testing.assert_array_equal(eng.class_count(), ora.class_count())
