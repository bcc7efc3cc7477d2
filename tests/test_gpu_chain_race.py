"""Regression test of the chain round-flag race (fixed in 76f29c9;
tests/test_chain_protocol.py models it): the KSIM_CHAIN_DELAY build
(libksim_engine_chaindelay.so, csrc/Makefile "flavor") makes one wave sleep
right before it reads each round's flag and another after the round's first
barrier, so the fastest wave is a round ahead whenever the chain runs more
than one round.  With the per-parity flags the placements stay the oracle's;
with the pre-76f29c9 single flag reset at the top of a round the sleeping wave
would leave the relaxation early (the model shows the interleaving)."""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from ksim import engine, gen, profile
from ksim.engine import Engine
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu

VARIANT = "chaindelay"


def _need_flavor():
    path = os.path.join(os.path.dirname(engine.LIB_PATH), f"libksim_engine_{VARIANT}.so")
    if not os.path.exists(path):
        pytest.fail(f"{path} missing: __graft_entry__.build() builds it")


@pytest.mark.parametrize("pct", [100, 0])
def test_delayed_chain_matches_oracle(pct):
    _need_flavor()
    cluster, pods = gen.config2(n_nodes=1500, n_pods=6000)
    prof = profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=pct))
    eng = Engine(0, variant=VARIANT)
    eng.set_profile(prof)
    eng.set_cluster(cluster)
    chosen, st = eng.schedule_batch(pods)
    ochosen, ost = Oracle(cluster, prof).schedule(pods)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.batches > 10 and st.evals == ost.evals


def test_delayed_chain_concurrent_sweep():
    """The interleaving the race first showed in: several engines sweeping
    weight vectors concurrently (config 5's shape, small)."""
    _need_flavor()
    cluster, pods = gen.config2(n_nodes=1000, n_pods=3000)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=100)
    names = [p.name for p in sp.score_plugins()]
    weights = gen.config5_weights(8)
    profs = [profile.compile_profile(sp.with_weights({n: int(x) for n, x in zip(names, w)})) for w in weights]
    engs = []
    for _ in range(4):
        e = Engine(0, variant=VARIANT)
        e.set_profile(profs[0])
        e.set_cluster(cluster)
        e.load_pods(pods)
        engs.append(e)

    def part(j):
        out = []
        for pr in profs[j::len(engs)]:
            engs[j].set_profile(pr)
            engs[j].load_pods(pods)
            engs[j].reset_cluster()
            out.append((pr, engs[j].schedule_loaded(0, pods.n_pods)[0]))
        return out

    with ThreadPoolExecutor(len(engs)) as pool:
        results = [r for rs in pool.map(part, range(len(engs))) for r in rs]
    for pr, chosen in results:
        np.testing.assert_array_equal(chosen, Oracle(cluster, pr).schedule(pods)[0])
