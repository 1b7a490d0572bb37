"""Golden fixtures for Fabrik.calculate on chains outside the unrolled 2..8
joints (1, 9, 13 and 24 joints, unequal links), by importing the reference.

Run in the build container only (see make_golden.py for the keras stub and
the iteration counter; the reference never travels to the GPU box):

    python tests/golden/make_golden_chains.py

Writes tests/golden/fabrik_calc_chains.npz: per chain length nj the keys
links_<nj>, init_<nj>, goals_<nj>, joints_<nj>, iters_<nj>, plus tol / max_iter.
"""
from __future__ import annotations

import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_golden as MG  # noqa: E402  (imports the reference, stubs keras)

CHAINS = (1, 9, 13, 24)
N_GOALS = 120
TOL, MAX_ITER = 1e-4, 150


def main():
    rng = np.random.default_rng(29)
    out = {"tol": np.float64(TOL), "max_iter": np.int32(MAX_ITER)}
    for nj in CHAINS:
        # equal links converge (the reference's backward pass spans dists[:-1] and
        # its forward pass dists[1:], fabrik.py:24,37); 13 joints keep unequal ones
        links = rng.uniform(0.3, 1.5, nj) if nj == 13 else np.full(nj, 0.7)
        init = np.zeros((N_GOALS, nj, 3))
        for k in range(1, nj):
            init[:, k, 2] = init[:, k - 1, 2] + links[k - 1]
        if nj > 1:
            init[:, 1:, :2] += rng.normal(0, 0.05, (N_GOALS, nj - 1, 2))
        reach = links[:-1].sum() if nj > 1 else 1.0
        goals = rng.normal(0, 0.25 * reach, (N_GOALS, 3)) + np.array([0.0, 0.0, 0.4 * reach])
        fab = MG.fabrik.Fabrik(list(links), TOL, MAX_ITER)
        jo, it = [], []
        for i in range(N_GOALS):
            MG._count["n"] = 0
            r = fab.calculate([MG.inverse.Point(list(q)) for q in init[i]], list(goals[i]))
            jo.append([list(q) for q in r])
            it.append(MG._count["n"])
        out.update({f"links_{nj}": links, f"init_{nj}": init, f"goals_{nj}": goals,
                    f"joints_{nj}": np.array(jo), f"iters_{nj}": np.array(it, np.int32)})
        print(f"nj={nj}: mean iters {np.mean(it):.1f}, capped {int((np.array(it) >= MAX_ITER).sum())}")
    np.savez_compressed(os.path.join(MG.OUT, "fabrik_calc_chains.npz"), **out)


if __name__ == "__main__":
    main()
