"""Phase clocks of the ADAPT ordered-walk window (KSIM_WIN_CLOCKS flavor):
staging (bitmaps + prefix counts into LDS), the walk, the whole kernel per
launch; config 1 scaled under ADAPT.  Run: KSIM_LIB_VARIANT=winclk python3 tools/win_clocks.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kube-scheduler-simulator_amd")]
from ksim import gen, profile  # noqa: E402
from ksim.engine import Engine  # noqa: E402

cluster, pods = gen.config1(n_nodes=5000, n_pods=20000)
eng = Engine(0)
eng.set_profile(profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=0)))
eng.set_cluster(cluster)
eng.load_pods(pods)
d0 = eng.diag()["dbg"]
_, st = eng.schedule_loaded(0, pods.n_pods, want_chosen=False)
d = [a - b for a, b in zip(eng.diag()["dbg"], d0)]
n = max(d[2], 1)
us = lambda x: round(x / n * 0.01, 3)   # s_memrealtime: 100 MHz
print(f"launches {d[2]} pods/launch {d[4] / n:.1f} staging {us(d[0])} us walk {us(d[1])} us kernel {us(d[3])} us; "
      f"batches {st.batches} device {st.device_ms:.2f} ms", flush=True)
