"""Round 4: where one config-5 weight vector's time goes on one engine
(set_profile, load_pods, reset_cluster, schedule_loaded), wall clock."""
import sys
import time

sys.path[:0] = [".", "kube-scheduler-simulator_amd"]
import numpy as np  # noqa: E402

from ksim import engine, gen, profile  # noqa: E402

cluster, pods = gen.config2(5000, 10000)
sp = profile.SchedulerProfile(percentage_of_nodes_to_score=100)
names = [p.name for p in sp.score_plugins()]
weights = gen.config5_weights(16)
profs = [profile.compile_profile(sp.with_weights({n: int(x) for n, x in zip(names, w)})) for w in weights]
e = engine.Engine(0)
e.set_profile(profs[0])
e.set_cluster(cluster)
e.load_pods(pods)
e.schedule_loaded(0, pods.n_pods)
t = {"set_profile": 0.0, "load_pods": 0.0, "reset_cluster": 0.0, "schedule": 0.0}
for pr in profs:
    a = time.perf_counter()
    e.set_profile(pr)
    b = time.perf_counter()
    e.load_pods(pods)
    c = time.perf_counter()
    e.reset_cluster()
    d = time.perf_counter()
    chosen, st = e.schedule_loaded(0, pods.n_pods)
    f = time.perf_counter()
    t["set_profile"] += b - a
    t["load_pods"] += c - b
    t["reset_cluster"] += d - c
    t["schedule"] += f - d
print({k: round(v / len(profs) * 1e3, 3) for k, v in t.items()}, "ms per vector", "device_ms", round(st.device_ms, 3))
