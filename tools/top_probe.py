import sys, os, time
sys.path.insert(0, "kube-scheduler-simulator_amd")
from ksim import gen, profile, engine
from ksim.engine import Engine
cluster, pods = gen.config2()
prof = profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=100))
e = Engine(0); e.set_profile(prof); e.set_cluster(cluster); e.load_pods(pods)
for rep in range(3):
    name, ms = e.time_eval(0, 200)
    print(os.environ.get("KSIM_LIB_VARIANT", "base"), name, "%.2f us" % (ms * 1000))
