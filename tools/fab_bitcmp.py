"""Hash of FABRIK solves' outputs, for bit-identity checks between library builds
(IKHIP_LIB=... python tools/fab_bitcmp.py): 1M random_dist seed-0 points at tol
1e-3 / 100 and 1e-5 / 200 (angles, iterations, FK errors), each solved twice (the
second call runs on the learned work order).  Two builds that claim the same
arithmetic print the same lines."""
import hashlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    from inversekinematicsann_amd import _native
    from inversekinematicsann_amd.robot.position_generator import random_dist
    ctx = _native.Context(0)
    pts = random_dist(1_000_000, seed=0)
    for tol, mi in ((1e-3, 100), (1e-5, 200)):
        for call in range(2):
            ang, it, err, _ = ctx.fabrik_solve_fk(pts, tol, mi)
            h = hashlib.sha256(ang.tobytes() + it.tobytes() + err.tobytes()).hexdigest()[:16]
            if os.environ.get("FAB_BITCMP_SPLIT"):  # angles + iterations apart from the FK errors
                hai = hashlib.sha256(ang.tobytes() + it.tobytes()).hexdigest()[:16]
                ok = err == err
                print(f"tol {tol:g} call {call} iters {int(it.sum())} max_err {err[ok].max():.17g} "
                      f"sum_err {err[ok].sum():.17g} angles+iters {hai}")
            else:
                print(f"tol {tol:g} call {call} iters {int(it.sum())} {h}")


if __name__ == "__main__":
    main()
