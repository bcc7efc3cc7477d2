"""Generate the committed golden vectors in tests/golden/.

kat.json: known-answer vectors whose expected values come from an independent
  Python restatement of the upstream formulas (integer leastRequestedScore;
  float64 balancedResourceScorer — Python floats are IEEE binary64 and never
  fuse multiply-add, matching Go on GOAMD64=v1).  NOT produced by the oracle.
config1_placements.npz: config-1 placements (100 nodes x 1,000 pods, seed
  0x4B53494D0001) produced by the CPU oracle in ADAPT (pct 0) and P100 modes:
  "self-consistent, unpinned vs Go" — they freeze the oracle's behaviour so a
  regression in it (or in the generator) is caught.

Run from the repo root:  python tests/golden/make_golden.py
"""
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kube-scheduler-simulator_amd")]

OUT = os.path.dirname(os.path.abspath(__file__))


def least_requested(req, cap):
    if cap == 0 or req > cap:
        return 0
    return ((cap - req) * 100) // cap


def balanced(req, alloc):
    fr = []
    for r, a in zip(req, alloc):
        if a == 0:
            continue
        f = float(r) / float(a)
        fr.append(1.0 if f > 1 else f)
    std = 0.0
    if len(fr) == 2:
        std = abs((fr[0] - fr[1]) / 2)
    elif len(fr) > 2:
        mean = sum(fr) / len(fr)
        s = 0.0
        for f in fr:
            s = s + (f - mean) * (f - mean)
        std = math.sqrt(s / len(fr))
    return int((1 - std) * 100)


def main():
    rng = np.random.default_rng(20250225)
    lr = []
    for _ in range(200):
        cap = int(rng.integers(0, 1 << 42))
        req = int(rng.integers(0, cap + 2)) if cap else 5
        lr.append({"req": req, "cap": cap, "score": least_requested(req, cap)})
    ba = []
    for _ in range(300):
        n = int(rng.integers(1, 5))
        alloc = [int(x) for x in rng.integers(0, 1 << 40, n)]
        req = [int(x) for x in rng.integers(0, 1 << 40, n)]
        ba.append({"req": req, "alloc": alloc, "score": balanced(req, alloc)})
    with open(os.path.join(OUT, "kat.json"), "w") as f:
        json.dump({"least_requested": lr, "balanced": ba}, f)

    from ksim import gen, profile
    from oracle.oracle import Oracle
    cluster, pods = gen.config1()
    out = {}
    for pct in (0, 100):
        sp = profile.SchedulerProfile(percentage_of_nodes_to_score=pct)
        chosen, _ = Oracle(cluster, profile.compile_profile(sp)).schedule(pods)
        out[f"pct{pct}"] = chosen
    np.savez_compressed(os.path.join(OUT, "config1_placements.npz"), **out)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
