"""The A/B forms of the same runs live in a flavor build, not behind runtime
switches (csrc/Makefile "ab": libksim_engine_ab.so, KSIM_AB_FORMS): the
three-launch P100 / ADAPT batches (commit as its own launch) instead of the
deferred commit, the static plugins evaluated per node instead of the
static-class table, ADAPT normalized-score and topology pods on the per-pod
path, per-cycle PreFilter domain sums, eager shard cycles, topology batch
runs that end at a zone-keyed class conflict (no zone variants).  A child process
loads that library (KSIM_LIB_VARIANT=ab), schedules P100 and ADAPT batches
and checks them against the oracle (the product forms run in every other GPU
test)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))

CHILD = r'''
import numpy as np
from ksim import gen, profile
from ksim.engine import Engine
from oracle.oracle import Oracle
for pct, n_nodes, n_pods in ((100, 2000, 3000), (0, 2000, 3000), (0, 300, 300 * 60 + 11)):
    cluster, pods = gen.config2(n_nodes=n_nodes, n_pods=n_pods, seed=5)
    prof = profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=pct))
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(cluster)
    chosen, st = eng.schedule_batch(pods)
    ora = Oracle(cluster, prof)
    ochosen, ost = ora.schedule(pods, nthreads=8)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals and eng.next_start == ora.next_start
    assert st.batches > 0
    eng.close()
from ksim.encode import encode_cluster, encode_pods
nodes, objs = gen.config1_objects(n_nodes=1200, n_pods=4000)
cluster, _ = encode_cluster(nodes)
pods = encode_pods(cluster, objs)
prof = profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=100))
eng = Engine(0)
eng.set_profile(prof)
eng.set_cluster(cluster)
chosen, st = eng.schedule_batch(pods)
ochosen, ost = Oracle(cluster, prof).schedule(pods, nthreads=8)
np.testing.assert_array_equal(chosen, ochosen)
assert st.evals == ost.evals and st.perpod_cycles == 0 and st.batches > 0
eng.close()
cluster, pods = gen.config3(n_nodes=700, pods_per_node=4, n_incoming=1500, seed=700, zone_anti_every=60)
eng = Engine(0)
eng.set_profile(prof)
eng.set_cluster(cluster)
chosen, st = eng.schedule_batch(pods)
ora = Oracle(cluster, prof)
ochosen, ost = ora.schedule(pods, nthreads=8)
np.testing.assert_array_equal(chosen, ochosen)
assert st.evals == ost.evals and eng.next_start == ora.next_start
np.testing.assert_array_equal(eng.class_count(), ora.class_count())
eng.close()
print("ok")
'''


@pytest.mark.parametrize("flavor", ["ab", "ab1", "ab2", "ab64"])
def test_ab_forms_vs_oracle(flavor):
    """ab: every alternative form at once; ab1: only the static-class table
    off (deferred commit kept); ab2: only the three-launch batches (the table
    kept); ab64: only the topology batches' zone variants off -- each form
    alone against the product's others."""
    lib = os.path.join(ROOT, "kube-scheduler-simulator_amd", "ksim", f"libksim_engine_{flavor}.so")
    assert os.path.exists(lib), "build the ab flavors: make -C kube-scheduler-simulator_amd/csrc ab abforms"
    env = dict(os.environ)
    env["KSIM_LIB_VARIANT"] = flavor
    env["PYTHONPATH"] = os.pathsep.join([ROOT, os.path.join(ROOT, "kube-scheduler-simulator_amd"),
                                         env.get("PYTHONPATH", "")])
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout[-2000:] + r.stderr[-2000:]
