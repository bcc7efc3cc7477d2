"""The node-split batch top (k_batch_top_ns, ksim_batch.hip; opt-in, measured
and not kept: the "ns4" flavor, libksim_engine_ns4.so, selects it) against the oracle:
P100 placements and evaluation counts, on cluster sizes around the chunk
thresholds (2 chunks from 2,048 nodes, 4 from 4,096, ragged chunks) and on
clusters shaped to reach every branch of its top-T: identical nodes (every
total tied, the hash decides), nearly full nodes (few feasible, complete
lists), and the best nodes packed into one wave's lanes (a wave with more
than T candidates, the capped extraction)."""
import os

import numpy as np
import pytest

from ksim import engine, gen, profile
from ksim.engine import Engine
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu

VARIANT = "ns4"


def _run(cluster, pods):
    path = os.path.join(os.path.dirname(engine.LIB_PATH), f"libksim_engine_{VARIANT}.so")
    if not os.path.exists(path):
        pytest.fail(f"{path} missing: __graft_entry__.build() builds it")
    prof = profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=100))
    eng = Engine(0, variant=VARIANT)
    eng.set_profile(prof)
    eng.set_cluster(cluster)
    chosen, st = eng.schedule_batch(pods)
    ochosen, ost = Oracle(cluster, prof).schedule(pods)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals and st.scheduled == ost.scheduled
    assert st.batches > 1
    return st


@pytest.mark.parametrize("n_nodes", [2048, 3001, 4096, 4099, 9000])
def test_sizes(n_nodes):
    cluster, pods = gen.config2(n_nodes, 3000)
    _run(cluster, pods)


def test_identical_nodes():
    cluster, pods = gen.config2(5000, 3000)
    cluster.alloc_cpu[:] = 32000
    cluster.alloc_mem[:] = 128 * 1024 ** 3
    _run(cluster, pods)


def test_nearly_full_nodes():
    cluster, pods = gen.config2(4500, 1500)
    # most nodes hold almost all their cpu: a pod fits on few of them
    cluster.req_cpu[:] = cluster.alloc_cpu - 300
    cluster.nz_cpu[:] = cluster.req_cpu
    cluster.req_cpu[::97] = 0
    cluster.nz_cpu[::97] = 0
    _run(cluster, pods)


def test_best_nodes_in_one_wave():
    cluster, pods = gen.config2(6000, 2000)
    # nodes whose position mod 1024 is below 64 (one wave's lanes in every
    # chunk) are the roomiest by far: their keys crowd the pods' top-T
    idx = np.arange(cluster.n_nodes)
    big = (idx % 1024) < 64
    cluster.alloc_cpu[big] = 512000
    cluster.alloc_mem[big] = 2048 * 1024 ** 3
    _run(cluster, pods)
