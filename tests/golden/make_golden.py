"""Generate the committed golden fixtures (run in the build container, not on the GPU box).

GTSAM (the reference optimiser's arithmetic) is absent and the reference holds
no tests or fixtures for this path, so the fixtures are the
output of the CPU restatements:

* C1, C1-nn, C2, KAT square/chain -- oracle/pgo_numpy.py (numpy + scipy SuperLU/COLAMD),
  independent of the C oracle, which tests/test_oracle.py checks against them;
* C3 (100k poses) -- oracle/pgo_oracle.c (the numpy twin is too slow at this size):
  final error, iteration counts, the error trace and every 100th final pose.

Each fixture also records a SHA-256 of the generated inputs so a change of the
generator is detected instead of silently comparing different graphs.

    python tests/golden/make_golden.py [C1 C1-nn C2 C3 ...]
"""
from __future__ import annotations

import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from graphslam_amd import datasets  # noqa: E402


def input_digest(g):
    h = hashlib.sha256()
    for a in (g.initial, g.edge_k1, g.edge_k2, g.edge_z, g.edge_cov, g.prior_keys, g.prior_pose, g.prior_cov):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def graph_for(name):
    if name == "square":
        return datasets.square_loop()
    if name == "chain":
        return datasets.straight_chain()
    return datasets.make(name)


def numpy_fixture(name):
    from oracle import pgo_numpy as tw
    g = graph_for(name)
    r = tw.optimize_graph(g)
    tr = np.array([[t["iteration"], t["lam"], t["new_error"], float(t["accepted"])] for t in r.trace])
    np.savez_compressed(os.path.join(HERE, f"golden_{name}.npz"), source="pgo_numpy", digest=input_digest(g),
                        initial=g.initial if g.num_poses <= 1000 else np.zeros((0, 3)), final=r.xyt(), trace=tr, final_error=r.error,
                        initial_error=r.initial_error, iterations=r.iterations,
                        inner_iterations=r.inner_iterations)
    print(name, "err", r.error, "it", r.iterations)


def oracle_fixture(name, stride=100):
    from oracle.oracle import Oracle
    g = graph_for(name)
    o = Oracle(g)
    r = o.optimize()
    s = r.stats
    idx = np.arange(0, g.num_poses, stride)
    tr = r.trace[:, [0, 1, 4, 6]]
    np.savez_compressed(os.path.join(HERE, f"golden_{name}.npz"), source="pgo_oracle.c", digest=input_digest(g),
                        sample_index=idx, final_sample=r.poses[idx], trace=tr,
                        final_error=s["final_error"], initial_error=s["initial_error"],
                        iterations=s["iterations"], inner_iterations=s["inner_iterations"],
                        linearizations=s["linearizations"])
    print(name, "err", s["final_error"], "it", s["iterations"], "t", s["t_total"])


if __name__ == "__main__":
    names = sys.argv[1:] or ["square", "chain", "C1", "C1-nn", "C2", "C3"]
    for n in names:
        if n == "C3":
            oracle_fixture(n)
        else:
            numpy_fixture(n)
