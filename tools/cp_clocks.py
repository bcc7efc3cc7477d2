"""Phase clocks of the chain + pairs launch (KSIM_CP_CLOCKS flavor, block 0 of
every launch): chain setup (list loads, hash), chain rounds, chain epilogue,
the whole block; config 2, P100, deferred-commit batches.
Run: KSIM_LIB_VARIANT=cpclk python3 tools/cp_clocks.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kube-scheduler-simulator_amd")]
from ksim import gen, profile  # noqa: E402
from ksim.engine import Engine  # noqa: E402

cluster, pods = gen.config2(5000, 50000)
for pct in (100, 0):
    eng = Engine(0)
    eng.set_profile(profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=pct)))
    eng.set_cluster(cluster)
    eng.load_pods(pods)
    eng.schedule_loaded(0, pods.n_pods, want_chosen=False)
    d0 = eng.diag()["dbg"]
    eng.reset_cluster()
    _, st = eng.schedule_loaded(0, pods.n_pods, want_chosen=False)
    d = [a - b for a, b in zip(eng.diag()["dbg"], d0)]
    n = max(d[3], 1)
    us = lambda x: round(x / n * 0.01, 3)   # s_memrealtime: 100 MHz
    print(f"pct {pct}: launches {d[3]} rounds/launch {d[4] / n:.2f} setup {us(d[0])} us rounds {us(d[1])} us "
          f"epilogue {us(d[2])} us block {us(d[5])} us; batches {st.batches} device {st.device_ms:.2f} ms")
    eng.close()
