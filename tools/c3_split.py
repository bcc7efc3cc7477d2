"""Config 3 per-pod path: where k_filter_score's time goes (full profile vs
filters only vs scores only vs no topology plugins)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kube-scheduler-simulator_amd")]
from ksim import gen, profile  # noqa: E402
from ksim.engine import Engine  # noqa: E402
from ksim.profile import Plugin, PluginSet, SchedulerProfile, convert_for_simulator  # noqa: E402

cluster, pods = gen.config3(n_nodes=10000, n_incoming=400)
star = PluginSet([], [Plugin("*")])
variants = {
    "full": SchedulerProfile(percentage_of_nodes_to_score=100),
    "no_score": SchedulerProfile(plugins=convert_for_simulator({"score": star}), percentage_of_nodes_to_score=100),
    "no_topo_filter": SchedulerProfile(plugins=convert_for_simulator(
        {"filter": PluginSet([], [Plugin("PodTopologySpread"), Plugin("InterPodAffinity")])}),
        percentage_of_nodes_to_score=100),
    "fit_only": SchedulerProfile(plugins=convert_for_simulator(
        {"filter": PluginSet([Plugin("NodeResourcesFit")], [Plugin("*")]), "score": star}),
        percentage_of_nodes_to_score=100),
}
for name, sp in variants.items():
    e = Engine(0)
    e.set_profile(profile.compile_profile(sp))
    e.set_cluster(cluster)
    e.load_pods(pods)
    t = e.time_kernels(0, 300)
    print(name, {k: round(v[0] * 1e3, 2) for k, v in t.items()}, flush=True)
