"""Phase clocks of the deferred-commit evaluation launch (k_batch_top_commit,
KSIM_TC_CLOCKS flavor, thread 0 of every block): prologue (ring slot, cut,
overlay build, state copy), node loop, top-T finish; config 2, P100.
Run: KSIM_LIB_VARIANT=tcclk python3 tools/tc_clocks.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kube-scheduler-simulator_amd")]
from ksim import gen, profile  # noqa: E402
from ksim.engine import Engine  # noqa: E402

cluster, pods = gen.config2(5000, 50000)
eng = Engine(0)
eng.set_profile(profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=100)))
eng.set_cluster(cluster)
eng.load_pods(pods)
eng.schedule_loaded(0, pods.n_pods, want_chosen=False)
d0 = eng.diag()["dbg"]
eng.reset_cluster()
_, st = eng.schedule_loaded(0, pods.n_pods, want_chosen=False)
d = [a - b for a, b in zip(eng.diag()["dbg"], d0)]
n = max(d[5], 1)
us = lambda x: round(x / n * 0.01, 3)   # s_memrealtime: 100 MHz
print(f"blocks {d[5]} per block: prologue {us(d[0])} us (to the first barrier {us(d[4])}, cut {us(d[6])}, "
      f"overlay {us(d[7])}), thread 0's node loop {us(d[1])} us, wait for the slowest wave {us(d[2])} us, "
      f"finish {us(d[3])} us; batches {st.batches} device {st.device_ms:.2f} ms", flush=True)
eng.close()
