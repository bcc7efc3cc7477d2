"""The CPU restatement's 1 -> 16 thread scaling on the box under OpenMP
runtime settings (each setting in a child process: the runtime reads them
once).  Config 2's sample, as bench.py's cpu_baseline times it.  Two runs on
two boxes (16 vs 1 thread): default 5.64x; OMP_WAIT_POLICY=active 5.65x;
active + PROC_BIND close + PLACES cores 8.78x, then 6.77x; PROC_BIND spread
5.38x.  Pinning the team inside the oracle (thread t on the t-th allowed CPU)
gave 3.83x at 16 threads and 6.6x at 8 on the second box: the host's other
tenants share the first CPUs, so the baseline stays unpinned."""
import json
import os
import subprocess
import sys

CHILD = r'''
import sys, time, json
sys.path[:0] = [".", "kube-scheduler-simulator_amd"]
from ksim import gen, profile
from oracle.oracle import Oracle
cluster, pods = gen.config2(n_nodes=5000, n_pods=50000)
prof = profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=100))
out = {}
for t in (1, 8, 16):
    o = Oracle(cluster.copy_state(), prof)
    o.schedule(pods, 0, 100, nthreads=t)
    n = 3000 if t > 1 else 800
    t0 = time.perf_counter()
    _, st = o.schedule(pods, 100, n, nthreads=t)
    out[t] = st.evals / (time.perf_counter() - t0)
print(json.dumps(out))
'''
settings = [{}, {"OMP_WAIT_POLICY": "active"}, {"OMP_WAIT_POLICY": "active", "OMP_PROC_BIND": "close", "OMP_PLACES": "cores"},
            {"OMP_PROC_BIND": "spread", "OMP_PLACES": "cores"}]
for extra in settings:
    env = dict(os.environ, **extra)
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-500:]
    try:
        d = json.loads(line)
        print(extra or "default", {k: f"{v:.3e}" for k, v in d.items()},
              "16 vs 1: %.2f" % (d["16"] / d["1"]), flush=True)
    except Exception:
        print(extra, "failed:", line, flush=True)
