"""Generate tests/golden/shapes.json: the reference's TrainingDataGenerator
shapes (robot/position_generator.py) on the CLI's example arguments, with the
global random states seeded, by importing the reference.  Build container only:

    python tests/golden/make_shapes.py

`random` calls sklearn's minmax_scale with the limits list as its feature_range;
sklearn >= 1.2 (1.7 here) refuses a list there (the reference pins 1.0.2, which
takes it), so for that shape the fixture runs the same draws through
minmax_scale with the tuple -- the reference's arithmetic, its argument type
adjusted.  Only inputs and outputs are stored.
"""
from __future__ import annotations

import json
import os
import random
import sys

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def main():
    sys.path.insert(0, REF)
    import robot.position_generator as pg  # noqa: E402
    from sklearn.preprocessing import minmax_scale
    G = pg.TrainingDataGenerator
    lim = {"x": [0.0, 3.0], "y": [0.0, 4.0], "z": [0.0, 5.0]}
    cases = []

    def add(name, args, pts, seed=None):
        cases.append({"shape": name, "args": args, "seed": seed,
                      "points": [[float(v) for v in p] for p in pts]})

    add("circle", [3.0, 20, [1.0, 5.0, 2.0]], G.circle(3.0, 20, [1.0, 5.0, 2.0]))
    add("circle", [0.5, 7, [0.0, 0.0, 0.0]], G.circle(0.5, 7, [0.0, 0.0, 0.0]))
    add("cube", [0.75, 2.0, 3.0, 4.0, [1.0, 2.0, 3.0]], G.cube(0.75, 2.0, 3.0, 4.0, [1.0, 2.0, 3.0]))
    add("cube", [0.3, 1.0, 0.7, 0.9, [0.0, -1.0, 0.5]], G.cube(0.3, 1.0, 0.7, 0.9, [0.0, -1.0, 0.5]))
    np.random.seed(7)
    add("cube_random", [0.75, 2.0, 3.0, 4.0, [1.0, 2.0, 3.0]],
        G.cube_random(0.75, 2.0, 3.0, 4.0, [1.0, 2.0, 3.0]), seed=7)
    add("spring", [50, 2.0, 3.0, 6.0], G.spring(50, 2.0, 3.0, 6.0))
    add("spring", [20, 2.0, 3.0, 6.0], G.spring(20, 2.0, 3.0, 6.0))
    np.random.seed(11)
    pts = list(zip(*[minmax_scale(np.random.randn(20), tuple(lim[a])) for a in ("x", "y", "z")]))
    add("random", [20, lim], pts, seed=11)
    for dist, seed in (("normal", 5), ("uniform", 3), ("random", 9)):
        np.random.seed(seed)
        random.seed(seed)
        add("random_dist", [100, lim, dist, 0.35], G.random_distribution(100, lim, dist, 0.35),
            seed=seed)
    with open(os.path.join(OUT, "shapes.json"), "w") as f:
        json.dump(cases, f, indent=0)
    print(f"wrote {len(cases)} cases")


if __name__ == "__main__":
    main()
