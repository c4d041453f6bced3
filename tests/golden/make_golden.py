"""Generate the committed golden fixtures (run in the build container, not on the GPU box).

GTSAM (the reference optimiser's arithmetic) is absent and the reference holds
no tests or fixtures for this path, so the fixtures are the
output of the CPU restatements:

* C1, C1-nn, C2, KAT square/chain -- oracle/pgo_numpy.py (numpy + scipy SuperLU/COLAMD),
  independent of the C oracle, which tests/test_oracle.py checks against them;
* C3 (100k poses) -- oracle/pgo_oracle.c for the whole trajectory: final
  error, iteration counts, the error trace and every 100th final pose;
* C3-numpy -- the numpy twin's whole C3 trajectory (24 tries, 8
  linearisations; ~40 min single-threaded SuperLU), so the headline size is
  also pinned end to end by a source independent of the C code that provides
  the CPU baseline: trace, error and every 100th pose; C3-numpy2 -- its first 2
  linearisations (max_outer = 2);
* C3-gn -- the C oracle's Gauss-Newton run of C3 (error per step, final error,
  every 100th final pose);
* C5 -- the C oracle's first linearisation, first Cholesky step and first LM
  linearisation (sampled); C5-numpy -- the numpy twin's first linearisation
  (0.5 chi^2, sampled gradient and H diagonal blocks), a second source;
  C5-lm5, C5-lm25, C5-lm100 -- the C oracle's first 5 / 25 / 100 LM linearisations of C5
  (every lambda try, the error after them, a 1000-pose sample of the values;
  round 6).

Each fixture also records a SHA-256 of the generated inputs so a change of the
generator is detected instead of silently comparing different graphs.

    python tests/golden/make_golden.py [C1 C1-nn C2 C3 C3-gn C3-numpy C5 C5-numpy C5-lm5 C5-lm25 C5-lm100 ...]
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


def numpy_truncated_fixture(name, max_outer=2, stride=100):
    """The numpy twin's trajectory of a large graph, sampled: max_outer = 2 ->
    golden_<name>-numpy2.npz; max_outer = 0 -> the whole GTSAM-default run,
    golden_<name>-numpy.npz (round 5: C3's 8 linearisations / 24 tries, so the
    headline trajectory is pinned end to end by a source independent of the C
    oracle, which is also the CPU baseline)."""
    from oracle import pgo_numpy as tw
    import time
    g = graph_for(name)
    t0 = time.time()
    r = tw.optimize_graph(g, tw.LMParams(max_outer=max_outer))
    tr = np.array([[t["iteration"], t["lam"], t["new_error"], float(t["accepted"])] for t in r.trace])
    idx = np.arange(0, g.num_poses, stride)
    fname = f"golden_{name}-numpy{max_outer}.npz" if max_outer else f"golden_{name}-numpy.npz"
    np.savez_compressed(os.path.join(HERE, fname), source="pgo_numpy",
                        digest=input_digest(g), max_outer=max_outer, sample_index=idx, final_sample=r.xyt()[idx],
                        trace=tr, final_error=r.error, initial_error=r.initial_error, iterations=r.iterations,
                        inner_iterations=r.inner_iterations)
    print(name, "numpy max_outer", max_outer, "err", r.error, "it", r.iterations, "t", time.time() - t0)


def c5_fixture(stride=1000):
    """C5 (1M poses / 5M edges) is too big for a full trajectory fixture: the
    C oracle's first linearisation (error, gradient and H diagonal blocks at
    every 1000th pose), the first lambda try's Cholesky step (sampled, plus its
    2-norm) and the state after max_outer = 1 (trace, error, sampled poses).
    The oracle factorises on the GPU plan's nested-dissection ordering
    (pgo_debug_ordering, host-only; AMD's fill would not fit this container's
    memory) -- the ordering changes rounding only."""
    import time
    from graphslam_amd.pose_graph import PoseGraph
    from oracle.oracle import Oracle
    g = graph_for("C5")
    pg = PoseGraph.from_dataset(g)
    order = pg.debug_ordering()
    pg.close()
    t0 = time.time()
    o = Oracle(g, order=order)
    hd, _, grad, err0 = o.linearize()
    idx = np.arange(0, g.num_poses, stride)
    rc, delta = o.solve(1e-5)
    assert rc == 0
    r = o.optimize(max_outer=1)
    s = r.stats
    np.savez_compressed(os.path.join(HERE, "golden_C5.npz"), source="pgo_oracle.c", digest=input_digest(g),
                        sample_index=idx, initial_error=err0, grad_sample=grad[idx], hdiag_sample=hd[idx],
                        delta_lambda=1e-5, delta_sample=delta[idx], delta_norm=np.linalg.norm(delta),
                        trace=r.trace[:, [0, 1, 4, 6]], error_after=s["final_error"],
                        poses_after_sample=r.poses[idx], factor_flops=s["factor_flops"], nnz_l=s["nnz_l"])
    print("C5 err0", err0, "after 1 linearisation", s["final_error"], "tries", s["inner_iterations"],
          "GFLOP", s["factor_flops"] / 1e9, "t", time.time() - t0)


def c5_trajectory_fixture(max_outer=5, stride=1000):
    """C5 past its first linearisation (round 6): the C oracle's first
    `max_outer` LM linearisations -- every lambda try (iteration, lambda,
    candidate error, accept decision), the error after each linearisation and
    a 1000-pose sample of the values after the last -- on the GPU plan's
    nested-dissection ordering, so a -m gpu test can walk the same tries
    (golden_C5-lm<max_outer>.npz)."""
    import time
    from graphslam_amd.pose_graph import PoseGraph
    from oracle.oracle import Oracle
    g = graph_for("C5")
    pg = PoseGraph.from_dataset(g)
    order = pg.debug_ordering()
    pg.close()
    t0 = time.time()
    o = Oracle(g, order=order)
    r = o.optimize(max_outer=max_outer)
    s = r.stats
    idx = np.arange(0, g.num_poses, stride)
    np.savez_compressed(os.path.join(HERE, f"golden_C5-lm{max_outer}.npz"), source="pgo_oracle.c",
                        digest=input_digest(g), max_outer=max_outer, sample_index=idx,
                        trace=r.trace[:, [0, 1, 4, 6]], initial_error=s["initial_error"],
                        final_error=s["final_error"], iterations=s["iterations"],
                        inner_iterations=s["inner_iterations"], linearizations=s["linearizations"],
                        final_sample=r.poses[idx])
    print("C5 max_outer", max_outer, "err", s["initial_error"], "->", s["final_error"], "tries",
          s["inner_iterations"], "it", s["iterations"], "t", time.time() - t0)


def c5_numpy_fixture(stride=1000):
    """C5's first linearisation pinned by the numpy twin (independent of the C
    oracle that made golden_C5.npz): 0.5 chi^2 at the dead-reckoned values, and
    at every 1000th pose the gradient g = J' Omega e and the diagonal block
    H_ii = sum J' Omega J (oracle/pgo_numpy.py's residuals and Jacobians,
    accumulated with np.add.at -- no sparse matrix at this size)."""
    import time
    from oracle import pgo_numpy as tw
    g = graph_for("C5")
    t0 = time.time()
    prob = tw.problem_from_graph(g)
    poses = tw.from_xyt(g.initial)
    ee, ep, p1, p2, hx = tw.residuals(prob, poses)
    J1 = tw.between_jacobian(p1, p2, hx)
    om = prob.eom
    B = np.einsum("eki,ekl->eil", J1, om)
    D = np.zeros((g.num_poses, 3, 3))
    np.add.at(D, prob.ei, np.einsum("eil,elj->eij", B, J1))
    np.add.at(D, prob.ej, om)
    np.add.at(D, prob.pi, prob.pom)
    G = np.zeros((g.num_poses, 3))
    np.add.at(G, prob.ei, np.einsum("eil,el->ei", B, ee))
    np.add.at(G, prob.ej, np.einsum("eil,el->ei", om, ee))
    np.add.at(G, prob.pi, np.einsum("pij,pj->pi", prob.pom, ep))
    err0 = 0.5 * (np.einsum("ei,eij,ej->", ee, om, ee) + np.einsum("ei,eij,ej->", ep, prob.pom, ep))
    idx = np.arange(0, g.num_poses, stride)
    np.savez_compressed(os.path.join(HERE, "golden_C5-numpy.npz"), source="pgo_numpy", digest=input_digest(g),
                        sample_index=idx, initial_error=err0, grad_sample=G[idx],
                        hdiag_sample=D[idx].reshape(-1, 9))
    print("C5 numpy err0", err0, "t", time.time() - t0)


def gn_fixture(name, stride=100):
    """GTSAM's GaussNewtonOptimizer (PGO_ALG_GN) from the dead-reckoned values:
    the C oracle's error after every step, the iteration count, the final error
    and every 100th final pose (the GPU plan's nested-dissection ordering)."""
    from graphslam_amd.pose_graph import PoseGraph
    from oracle.oracle import Oracle
    g = graph_for(name)
    pg = PoseGraph.from_dataset(g)
    order = pg.debug_ordering()
    pg.close()
    o = Oracle(g, order=order)
    r = o.optimize(algorithm=1)
    s = r.stats
    idx = np.arange(0, g.num_poses, stride)
    np.savez_compressed(os.path.join(HERE, f"golden_{name}-gn.npz"), source="pgo_oracle.c", digest=input_digest(g),
                        sample_index=idx, final_sample=r.poses[idx], errors=r.trace[:, 4],
                        final_error=s["final_error"], initial_error=s["initial_error"],
                        iterations=s["iterations"], linearizations=s["linearizations"])
    print(name, "GN err", s["final_error"], "it", s["iterations"], "t", s["t_total"])


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
        if n == "C5":
            c5_fixture()
        elif n.startswith("C5-lm"):
            c5_trajectory_fixture(int(n[len("C5-lm"):]))
        elif n == "C5-numpy":
            c5_numpy_fixture()
        elif n.endswith("-gn"):
            gn_fixture(n[: -len("-gn")])
        elif n.endswith("-numpy2"):
            numpy_truncated_fixture(n[: -len("-numpy2")], 2)
        elif n.endswith("-numpy"):
            numpy_truncated_fixture(n[: -len("-numpy")], 0)
        elif n == "C3":
            oracle_fixture(n)
        else:
            numpy_fixture(n)
