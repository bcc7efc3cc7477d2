"""Drive the batch path on a config-2 slice (for rocprofv3 counter passes)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kube-scheduler-simulator_amd")]
from ksim import gen, profile  # noqa: E402
from ksim.engine import Engine  # noqa: E402

n_pods = int(sys.argv[1]) if len(sys.argv) > 1 else 6400
cluster, pods = gen.config2(n_pods=n_pods)
e = Engine(0)
e.set_profile(profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=100)))
e.set_cluster(cluster)
e.load_pods(pods)
_, st = e.schedule_loaded(0, pods.n_pods, want_chosen=False)
print(f"pods={pods.n_pods} batches={st.batches} trunc={st.truncations} device_ms={st.device_ms:.2f}")
print("diag", e.diag())
print("time_kernels", e.time_kernels(0, min(pods.n_pods, 8192)) if False else "")
