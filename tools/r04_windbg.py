"""Config 4 ADAPT once with the KSIM_WIN_DEBUG build (printf per window launch);
summarises rounds and phase times (wall clock ticks at 100 MHz)."""
import collections, os, re, subprocess, sys

if len(sys.argv) > 1 and sys.argv[1] == "run":
    sys.path.insert(0, "kube-scheduler-simulator_amd")
    sys.path.insert(0, "tests")
    sys.path.insert(0, ".")
    from ksim import gen
    from ksim.engine import Engine
    from test_gpu_parity import _prof
    cluster, pods = gen.config4()
    eng = Engine(0)
    eng.set_profile(_prof(0))
    eng.set_cluster(cluster)
    chosen, st = eng.schedule_batch(pods)
    print("DONE", st.batches, st.scheduled, flush=True)
    sys.exit(0)

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/windbg"
os.makedirs(out, exist_ok=True)
for tag, env in (("gc", {}), ("walk", {"KSIM_NO_WIN_GC": "1"})):
    e = dict(os.environ, KSIM_LIB_VARIANT="windbg", **env)
    r = subprocess.run([sys.executable, "-u", __file__, "run"], env=e, capture_output=True, text=True, timeout=300)
    open(f"{out}/{tag}.txt", "w").write(r.stdout[-200000:] + r.stderr[-5000:])
    rounds, build, relax = collections.Counter(), [], []
    for line in r.stdout.splitlines():
        m = re.search(r"rounds=(\d+).*build=(\d+) relax=(\d+)", line)
        if m:
            rounds[int(m.group(1))] += 1
            build.append(int(m.group(2)))
            relax.append(int(m.group(3)))
        m = re.search(r"WINDBG0 exact=\d+ relax=(\d+)", line)
        if m:
            relax.append(int(m.group(1)))
    n = max(len(relax), 1)
    print(tag, r.returncode, "launches", len(relax), "rounds", sorted(rounds.items())[:30],
          "build_us %.2f" % (sum(build) / max(len(build), 1) / 100), "relax_us %.2f" % (sum(relax) / n / 100),
          [l for l in r.stdout.splitlines() if l.startswith("DONE")])
    if r.returncode:
        sys.exit(r.returncode)
