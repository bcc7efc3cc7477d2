"""Config 3 (full size) on the product library, the clocked flavor
(KSIM_TB_CLOCKS: chain + pairs phases of k_tb_chain_pairs) and the flavor
without zone variants: ms per step, batches, and the chain phase clocks."""
import sys
import time

sys.path[:0] = [".", "kube-scheduler-simulator_amd"]
import numpy as np  # noqa: E402

from ksim import gen, profile  # noqa: E402
from ksim.engine import Engine  # noqa: E402

cluster, pods = gen.config3()
prof = profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=100))
ref = None
for variant in [None, "tbclk", "ab64"]:
    eng = Engine(0, variant=variant)
    eng.set_profile(prof)
    eng.set_cluster(cluster)
    eng.load_pods(pods)
    eng.schedule_loaded(0, pods.n_pods)
    ts = []
    for _ in range(3):
        eng.reset_cluster()
        d0 = eng.diag()
        t = time.perf_counter()
        chosen, st = eng.schedule_loaded(0, pods.n_pods)
        ts.append(time.perf_counter() - t)
    d = eng.diag()
    if ref is None:
        ref = chosen
    assert np.array_equal(chosen, ref), variant
    line = f"{variant or 'product'}: {1e3 * min(ts):.2f} ms, batches {st.batches}, variant pods {d['tb_variant_pods']}"
    if variant == "tbclk":
        db = [d["dbg"][k] - d0["dbg"][k] for k in range(5)]
        n = max(db[4], 1)
        line += (f"; chain prologue {db[0] / n / 100:.2f} us, rounds {db[1] / n / 100:.2f} us"
                 f" ({db[2] / n:.1f} rounds), block 0 chain+pairs {db[3] / n / 100:.2f} us")
        fb = [d["dbg"][k] - d0["dbg"][k] for k in range(5, 9)]
        nb = max(fb[3], 1)
        line += (f"; filter blocks {fb[3] / n:.0f} per launch: setup {fb[0] / nb / 100:.2f} us,"
                 f" plans {fb[1] / nb / 100:.2f} us, extrema {fb[2] / nb / 100:.2f} us")
        sb = [d["dbg"][k] - d0["dbg"][k] for k in range(9, 13)]
        ns = max(sb[2], 1)
        line += (f"; select blocks {sb[2] / n:.0f} per launch: inputs {sb[0] / ns / 100:.2f} us,"
                 f" slots {sb[1] / ns / 100:.2f} us ({sb[3] / ns:.2f} slots per block)")
        cb = [d["dbg"][k] - d0["dbg"][k] for k in (13, 14)]
        line += f"; chain_pairs blocks {cb[1] / n:.1f} per launch, {cb[0] / max(cb[1], 1) / 100:.2f} us each"

    print(line, flush=True)
    if variant in (None, "ab64"):
        eng.reset_cluster()
        kt = eng.time_kernels(0, pods.n_pods)
        print("   kernels (us per launch):",
              {k: round(1e3 * v[0], 2) for k, v in kt.items() if k.startswith("k_tb")}, flush=True)
    eng.close()
