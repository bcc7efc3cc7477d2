"""Probe: HIP runtime sharing between torch and libksim_engine.so in one process."""
import os, sys, subprocess
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kube-scheduler-simulator_amd")]
order = sys.argv[1] if len(sys.argv) > 1 else "torch_first"
if order == "torch_first":
    import torch
    print("torch", torch.__version__, torch.cuda.is_available(), torch.cuda.device_count(), flush=True)
    x = torch.ones(4, device="cuda"); torch.cuda.synchronize(); print("torch tensor ok", x.sum().item(), flush=True)
from ksim import engine, gen, profile
import numpy as np
from oracle.oracle import Oracle
c, p = gen.config1(n_nodes=100, n_pods=50)
prof = profile.compile_profile(profile.SchedulerProfile())
e = engine.Engine(0); e.set_profile(prof); e.set_cluster(c)
ch, st = e.schedule_batch(p)
o, _ = Oracle(c, prof).schedule(p)
print(order, "engine parity", np.array_equal(ch, o), flush=True)
if order != "torch_first":
    import torch
    print("torch after engine", torch.cuda.is_available(), flush=True)
    torch.cuda.synchronize(); print("sync ok", flush=True)
with open("/proc/self/maps") as f:
    libs = sorted({l.split()[-1] for l in f if "amdhip64" in l})
print("hip runtime mapped:", libs, flush=True)
