"""Config-3 per-pod cycle with the KSIM_SEL_CLOCKS build: mean per-block phase
times of k_select and the last block's bind.  Run with KSIM_LIB_VARIANT=selclk
on the GPU box (make -C kube-scheduler-simulator_amd/csrc flavor TAG=selclk
DEFS=-DKSIM_SEL_CLOCKS)."""
import sys
import time

sys.path.insert(0, "kube-scheduler-simulator_amd")
from ksim import gen, profile  # noqa: E402
from ksim.engine import Engine  # noqa: E402

n_pods = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
cluster, pods = gen.config3(n_incoming=n_pods)
prof = profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=100))
eng = Engine(0)
eng.set_profile(prof)
eng.set_cluster(cluster)
eng.load_pods(pods)
eng.schedule_loaded(0, 500)
d0 = eng.diag()["dbg"]
t = time.perf_counter()
_, st = eng.schedule_loaded(500, n_pods - 500)
dt = time.perf_counter() - t
d1 = eng.diag()["dbg"]
blocks = d1[4] - d0[4]
binds = d1[6] - d0[6]
print(f"{(n_pods - 500) / dt:.0f} pods/s, {dt / (n_pods - 500) * 1e6:.1f} us/pod, blocks {blocks}, binds {binds}")
for k, nm in enumerate(["prologue", "totals", "block record", "arrival"]):
    print(f"  {nm:14s} {(d1[k] - d0[k]) / max(blocks, 1) * 10 / 1000:.2f} us per block")
print(f"  {'bind (last)':14s} {(d1[5] - d0[5]) / max(binds, 1) * 10 / 1000:.2f} us per cycle")
