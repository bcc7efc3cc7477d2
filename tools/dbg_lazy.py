import os, sys
sys.path[:0] = ['/root/repo', '/root/repo/kube-scheduler-simulator_amd']
import numpy as np
from ksim import gen, profile, engine
from ksim.engine import Engine
cluster, pods = gen.config2(5000, 50000)
prof = profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=100))
eng = Engine(0); eng.set_profile(prof); eng.set_cluster(cluster); eng.load_pods(pods)
for r in range(4):
    eng.reset_cluster()
    ch, st = eng.schedule_loaded(0, pods.n_pods)
    print("run", r, "batches", st.batches, "trunc", st.truncations, "sched", st.scheduled, "evals", st.evals, "sum", int(ch.astype(np.int64).sum()), flush=True)
print("diag", eng.diag() if hasattr(eng, "diag") else None)
