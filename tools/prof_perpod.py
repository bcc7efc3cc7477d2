"""Per-kernel times of the per-pod path (ADAPT config 2, config 3)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kube-scheduler-simulator_amd")]
from ksim import gen, profile  # noqa: E402
from ksim.engine import Engine  # noqa: E402

for name, (cluster, pods), pct in (("adapt", gen.config2(5000, 3000), 0),
                                   ("c3", gen.config3(n_nodes=10000, n_incoming=1000), 100)):
    e = Engine(0)
    e.set_profile(profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=pct)))
    e.set_cluster(cluster)
    e.load_pods(pods)
    _, st = e.schedule_loaded(0, pods.n_pods, want_chosen=False)
    print(name, f"pods={pods.n_pods} device_ms={st.device_ms:.1f} per_pod_us={st.device_ms * 1e3 / pods.n_pods:.1f}")
    e.set_cluster(cluster)
    e.load_pods(pods)
    print(name, e.time_kernels(0, min(pods.n_pods, 300)))
