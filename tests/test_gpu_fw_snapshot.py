"""The drop-in's incremental snapshot on the GPU (ABI 11): the engine follows
informer events -- bound pods added and deleted, pod relabels, nodes added,
updated, moved between zones and removed -- through ksim_encoder_update_nodes
/ ksim_upsert_nodes and ksim_assume / ksim_forget with the encoder's
membership (ksim/fwsnapshot.py, the mirror of the Go adapter's NativeEncoder),
interleaved with framework-driven cycles under the racing framework mirror.
The engine, the oracle fed the same deltas, and an oracle that re-encodes and
re-sends its whole record every cycle make the same choices and annotations;
no full re-encode after the first."""
import numpy as np
import pytest

from fwdeltas import drive, make_runs, objects, same_node_state
from fwmirror import EngineBackend, OracleBackend
from ksim import profile
from ksim.engine import Engine
from ksim.nativeenc import encode
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu


def _specs(nodes, bound, prof):
    eng = Engine(0)
    eng.set_profile(prof)
    cluster, _ = encode(nodes, bound, [])
    return eng, [("engine", EngineBackend(eng), False),
                 ("oracle", OracleBackend(Oracle(cluster, prof)), False),
                 ("full", OracleBackend(Oracle(cluster, prof)), True)]


@pytest.mark.parametrize("seed", [21, 22])
def test_engine_snapshot_deltas_vs_oracle(seed):
    nodes, bound, incoming = objects(n_nodes=300, pods_per_node=3, n_incoming=260)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=0)
    prof = profile.compile_profile(sp)
    eng, specs = _specs(nodes, bound, prof)
    runs = make_runs(specs, nodes, bound, sp, seed)

    def check(i):
        if i % 37 == 36:                            # the device's count classes equal the oracle's
            np.testing.assert_array_equal(eng.class_count(), runs[1].b.o.class_count())
    events = drive(runs, nodes, bound, incoming, seed=seed, on_step=check)
    assert events > 100
    same_node_state(runs)
    np.testing.assert_array_equal(eng.class_count(), runs[1].b.o.class_count())
    st = runs[0].sync.stats
    assert st["full_encodes"] == 1, st
    assert st["node_deltas"] > 20 and st["pod_adds"] > 40 and st["pod_deletes"] > 40, st
    d = eng.diag()
    assert d["fw_score_host"] + d["fw_score_device"] > 100, d
