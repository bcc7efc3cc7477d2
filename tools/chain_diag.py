"""Phase clock of k_batch_chain (setup / relaxation rounds / epilogue) on config 2 P100."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kube-scheduler-simulator_amd")]
from ksim import gen, profile  # noqa: E402
from ksim.engine import Engine  # noqa: E402

cluster, pods = gen.config2(5000, 50000)
for pct in (100, 0):
    e = Engine(0)
    e.set_profile(profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=pct)))
    e.set_cluster(cluster)
    e.load_pods(pods)
    _, st = e.schedule_loaded(0, pods.n_pods, want_chosen=False)
    print(pct, f"batches={st.batches} truncations={st.truncations} ms={st.device_ms:.2f}", e.diag())
