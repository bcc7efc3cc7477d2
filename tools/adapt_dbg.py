"""Why config 1's ADAPT batches end short (KSIM_ADAPT_DBG flavor, the
non-deferred ADAPT path's commit): exhausted lists vs broken windows vs pair
cuts.  Run: KSIM_LIB_VARIANT=adbg python3 tools/adapt_dbg.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kube-scheduler-simulator_amd")]
from ksim import gen, profile  # noqa: E402
from ksim.engine import Engine  # noqa: E402
from ksim.nativeenc import encode  # noqa: E402

nodes, pobjs_all = gen.config1_objects(n_nodes=5000, n_pods=50000)
for n_pods in (5000, 15000, 30000, 50000):
    cluster, pods = encode(nodes, [], pobjs_all[:n_pods])
    eng = Engine(0)
    eng.set_profile(profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=0)))
    eng.set_cluster(cluster)
    eng.load_pods(pods)
    d0 = eng.diag()["dbg"]
    _, st = eng.schedule_loaded(0, pods.n_pods, want_chosen=False)
    d = [a - b for a, b in zip(eng.diag()["dbg"], d0)]
    n = max(d[0], 1)
    print(f"{n_pods} pods: batches {d[0]} (truncations {st.truncations}, scheduled {st.scheduled}): chain shorter "
          f"than the batch {d[1]}, broken window inside the chain {d[2]}, pair-max cuts {d[5]}; mean chain "
          f"{d[3] / n:.1f}, mean prefix before a broken window {d[4] / n:.1f}, mean committed {d[6] / n:.1f} of "
          f"{d[7] / n:.1f}; device {st.device_ms:.1f} ms", flush=True)
    eng.close()
