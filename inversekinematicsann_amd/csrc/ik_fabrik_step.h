// ik_fabrik_step.h -- one FABRIK iteration of the 4-joint chain in its three
// arithmetic forms (general, core sequences, core + reused distances), shared
// by the FABRIK kernels (ik_fabrik.hip) and the iteration microbenchmark
// (tools/ubench.hip).  Bit-exactness notes: DESIGN.md "FABRIK".
#pragma once

#include "ik_common.h"

namespace ikhip {

// One FABRIK iteration for the 4-joint chain (fabrik.py:57-64): backward pass
// from the goal (dists[2], dists[1], dists[0]), start error, forward pass from
// the start (dists[1], dists[2], dists[3]), goal error.  cur[0] is always start.
// The two errors are returned SQUARED (the radicands of get_distance_between):
// they are only compared with tol (fabrik.py:57), and sqrt(x) > tol <=> x > t
// for t = tol_threshold(tol) exactly, sqrt being correctly rounded and monotonic.
__device__ __forceinline__ void fabrik_step4(const d3 start, d3 &c1, d3 &c2, d3 &c3,
                                             const d3 g, const double *L, double &se2,
                                             double &ge2, int &st) {
  d3 b2 = point_between(g, c2, L[2], st);
  d3 b1 = point_between(b2, c1, L[1], st);
  d3 b0 = point_between(b1, start, L[0], st);
  se2 = dist3_sq(b0, start);
  c1 = point_between(start, b1, L[1], st);
  c2 = point_between(c1, b2, L[2], st);
  c3 = point_between(c2, g, L[3], st);
  ge2 = dist3_sq(c3, g);
}

// fabrik_step4 through point_between_core: the same bits wherever dom comes back
// below kCoreDom (then no ZeroDivisionError is possible either).  The six radicands are
// checked against sqrt_core's domain instead of carrying the general sqrt /
// division's range handling: ~22 % fewer instructions per iteration.
__device__ __forceinline__ void fabrik_step4_core(const d3 start, d3 &c1, d3 &c2, d3 &c3,
                                                  const d3 g, const double *L, double &se2,
                                                  double &ge2, uint32_t &dom) {
  d3 b2 = point_between_core(g, c2, L[2], dom);
  d3 b1 = point_between_core(b2, c1, L[1], dom);
  d3 b0 = point_between_core(b1, start, L[0], dom);
  se2 = dist3_sq(b0, start);
  c1 = point_between_core(start, b1, L[1], dom);
  c2 = point_between_core(c1, b2, L[2], dom);
  c3 = point_between_core(c2, g, L[3], dom);
  ge2 = dist3_sq(c3, g);
}

// fabrik_step4_core with the two distances the reference computes twice taken once
// (links L0 == L1 and L2 == L3, bitwise; the host checks):
//  * b0 = pb(b1, start, L0) and c1 = pb(start, b1, L1) share |b1 - start| (the
//    radicand squares start - b1 = -(b1 - start) exactly) and, with L0 == L1, the
//    quotient, so c1 = start + q*(b1 - start) = start - q*(start - b1);
//  * this iteration's c3 = pb(c2, g, L3) and the next one's b2 = pb(g, c2, L2) share
//    |c2 - g| and, with L2 == L3, the quotient: the lane carries (cq, cd = g - c2)
//    into the next iteration, whose b2 = g + cq*(c2 - g) = g - cq*cd.
// Every value is the one the reference computes (IEEE: a + (-b) == a - b and
// q*(-d) == -(q*d)), so the bits do not change; two of the six square roots and
// divisions per iteration go.  cdom is the carried radicand's domain value: it joins
// dom so that the wave-uniform fallback still sees it.
__device__ __forceinline__ void fabrik_step4_reuse(const d3 start, d3 &c1, d3 &c2, d3 &c3,
                                                   const d3 g, const double *L, double &se2,
                                                   double &ge2, double &cq, d3 &cd,
                                                   uint32_t &cdom, uint32_t &dom) {
  dom = cdom;
  const d3 b2 = {g.x - cq * cd.x, g.y - cq * cd.y, g.z - cq * cd.z};
  const d3 b1 = point_between_core(b2, c1, L[1], dom);
  const double dx = start.x - b1.x, dy = start.y - b1.y, dz = start.z - b1.z;
  const double x = sq(dx) + sq(dy) + sq(dz);
  dom = max(dom, sqrt_core_dom(x));
  const double q = div_core(L[0], sqrt_core(x));
  const d3 b0 = {b1.x + (q * dx), b1.y + (q * dy), b1.z + (q * dz)};
  se2 = dist3_sq(b0, start);
  c1 = {start.x - (q * dx), start.y - (q * dy), start.z - (q * dz)};
  c2 = point_between_core(c1, b2, L[2], dom);
  const double ex = g.x - c2.x, ey = g.y - c2.y, ez = g.z - c2.z;
  const double x3 = sq(ex) + sq(ey) + sq(ez);
  cdom = sqrt_core_dom(x3);
  dom = max(dom, cdom);
  cq = div_core(L[3], sqrt_core(x3));
  c3 = {c2.x + (cq * ex), c2.y + (cq * ey), c2.z + (cq * ez)};
  cd = {ex, ey, ez};
  ge2 = dist3_sq(c3, g);
}

// The carry of fabrik_step4_reuse for a chain whose c2 did not come from it (a
// refilled lane's seed pose, or the general step of a fallback), through the
// core sequences: inside sqrt_core's domain they are the general sqrt / division's
// bits, and outside it cdom sends the next iteration to the fallback, which
// recomputes everything without reading cq (so the value is never used there).
__device__ __forceinline__ void reuse_carry(const d3 c2, const d3 g, double L3, double &cq,
                                            d3 &cd, uint32_t &cdom) {
  cd = {g.x - c2.x, g.y - c2.y, g.z - c2.z};
  const double x = sq(cd.x) + sq(cd.y) + sq(cd.z);
  cdom = sqrt_core_dom(x);
  cq = div_core(L3, sqrt_core(x));
}

}  // namespace ikhip

namespace ikhip {

// ---- the loop condition without the start and goal errors' own arithmetic ----
// fabrik.py:57-64 continues while se > tol or ge > tol, se = |B0 - start| and
// ge = |F3 - goal| (squared here, against tol2).  b0 lies at L0 from b1 towards
// start, and start at sqrt(x) from b1: se = |sqrt(x) - L0| up to roundings (r06;
// r05 took |1 - q| sqrt(x), one multiply more and after the division), and the
// goal error is |sqrt(x3) - L3| with x3 the carried quotient's radicand.  The
// reference's own se2 / ge2 (b0, F3 = c3 and their differences, 25 VALU) are
// computed only when an approximation falls inside the launch's band [lo, hi]
// (ErrBand): outside it the comparison with tol2 provably comes out the same.
//
// The band: with u = 2^-53, every rounding of b0 = b1 + q (start - b1), B0 - start,
// the squares and the root moves |B0 - start| by at most
//   1.03 u (3 |goal| + 2 |start| + 3 sum L)
// from |1 - q| |start - b1| (the backward points lie within sum L of the goal, the
// forward ones within sum L of the start; the same bound with the roles swapped
// covers the goal error).  The approximation s - L0 (s = RN(sqrt(x))) is that value
// up to |s - |start - b1|| <= 2.5 u |start - b1| <= 2.5 u (n1 + sum L) and
// |q s - L0| <= 3.5 u L0 (x's three roundings, the root's, the quotient's), and
// rounds itself (relative u).  So with n1 = |start|_1 + |goal|_1 the distance of
// sea = |s - L0| from the reference's error is at most u (5.6 n1 + 7.4 sum L) + u sea;
// D is twice the absolute part, D = 2^-52 (6 n1max + 8 sum L + 1), and the relative
// part (< 2^-52) sits far inside the band's 2^-36.  With T = sqrt(tol2) (real):
//   sea > hi = (D + T) (1 + 2^-36)        =>  se2 > tol2
//   sea < lo = (T - D) (1 - 2^-36)        =>  se2 <= tol2   (only if D <= T / 2)
// (tests/test_band_cpu.py checks the bound along real iterations.)  The band is one
// per launch (fabrik_band on the host): n1max bounds |start|_1 + |goal|_1 (L1 norms
// bound the Euclidean ones), with T's bounds tol_lo <= T <= tol_hi.  A lane past
// n1max (or with a non-finite goal) never runs this step: the iteration kernel hands
// it to the retire step's general re-solve (r06; r05 made its comparisons exact).
struct ErrBand {
  double lo, hi;
};

__host__ __forceinline__ ErrBand fabrik_band(double tol2, double n1max, double sum_l) {
  // tol2 <= 0 (tol = 0, or a negative tol): a band that decides nothing, every
  // comparison exact.  (hi = 0 would call any sea > 0 "above", but at tol = 0 the
  // reference stops where b0 rounds onto start exactly, se2 == 0, while s is
  // L0 +- 1 ulp and sea > 0: ADVICE r05.)
  ErrBand b = {-1.0, INFINITY};
  if (!(tol2 > 0.0)) return b;
  const double T = std::sqrt(tol2);
  const double tol_lo = T * (1.0 - 0x1p-50), tol_hi = T * (1.0 + 0x1p-50);
  const double d = 0x1p-52 * (6.0 * n1max + 8.0 * sum_l + 1.0);
  b.hi = (d + tol_hi) * (1.0 + 0x1p-36);
  b.lo = (d <= 0.5 * tol_lo) ? (tol_lo - d) * (1.0 - 0x1p-36) : -1.0;
  return b;
}

// The core domain from the quotients (r06): a radicand x outside sqrt_core's
// domain (0, tiny, inf, NaN) gives a quotient L / sqrt_core(x) that is NaN or
// larger in magnitude than |L| 2^382 (tools/dom_check.hip, every binade below
// 2^-767 and the specials on gfx950), and an in-domain one a quotient at most
// |L| 2^383.5.  So |q1| + |q| + |q2| + |cq| <= qmax = min |L| 2^382 (fabrik_qmax)
// implies every radicand of the iteration is >= 2^-764 and finite: in the
// domain.  Lanes that fail it (the true out-of-domain ones and any in
// [2^-767, 2^-764)) are re-solved in the general arithmetic (kStRedo): the same
// bits either way.  3 adds and a compare instead of four exponent extractions,
// their maximum and a compare.
__host__ __forceinline__ double fabrik_qmax(const double *L) {
  double m = std::fabs(L[0]);
  for (int k = 1; k < 4; ++k) m = std::fmin(m, std::fabs(L[k]));
  return m * 0x1p382;
}

// fabrik_step4_reuse with the loop condition cont = (se2 > tol2) || (ge2 > tol2)
// decided through the band, the core domain from the quotients, and F3 (c3 = c2 +
// cq cd, the reference's get_point_between(c2, goal, L3) from the carry) left to
// the caller.  The exact se2 / ge2 run in a wave-uniform branch when any lane's
// approximation is uncertain (and for the goal error only where the start error
// has not already decided).  Returns whether the iteration's radicands were all
// in the core domain.  (The masks are formed right before their branches: held
// longer, or with the wave's exec taken once, they went to VGPRs, r06.)
__device__ __forceinline__ bool fabrik_step4_lazy(const d3 start, d3 &c1, d3 &c2, const d3 g,
                                                  const double *L, const ErrBand band,
                                                  double tol2, double qmax,
                                                  bool &cont, double &cq, d3 &cd) {
  const d3 b2 = {g.x - cq * cd.x, g.y - cq * cd.y, g.z - cq * cd.z};
  const double ux = c1.x - b2.x, uy = c1.y - b2.y, uz = c1.z - b2.z;
  const double q1 = div_core(L[1], sqrt_core(sq(ux) + sq(uy) + sq(uz)));
  const d3 b1 = {b2.x + (q1 * ux), b2.y + (q1 * uy), b2.z + (q1 * uz)};
  const double dx = start.x - b1.x, dy = start.y - b1.y, dz = start.z - b1.z;
  const double sx = sqrt_core(sq(dx) + sq(dy) + sq(dz));
  const double q = div_core(L[0], sx);
  const double qx = q * dx, qy = q * dy, qz = q * dz;
  // the decisions as lane masks (ballots of the compares): the band tests, the
  // merges with the exact results and the uncertainty are scalar-ALU operations
  const uint64_t ex = __builtin_amdgcn_read_exec();
  const double sea = fabs(sx - L[0]);  // |B0 - start| up to the band
  uint64_t gt = __builtin_amdgcn_ballot_w64(sea > band.hi);
  uint64_t unc = ex & ~(gt | __builtin_amdgcn_ballot_w64(sea < band.lo));
  if (__builtin_expect(unc != 0, 0)) {  // (a NaN is uncertain)
    const d3 b0 = {b1.x + qx, b1.y + qy, b1.z + qz};
    const double se2 = dist3_sq(b0, start);
    gt = (gt & ~unc) | (__builtin_amdgcn_ballot_w64(se2 > tol2) & unc);
  }
  c1 = {start.x - qx, start.y - qy, start.z - qz};
  const double vx = b2.x - c1.x, vy = b2.y - c1.y, vz = b2.z - c1.z;
  const double q2 = div_core(L[2], sqrt_core(sq(vx) + sq(vy) + sq(vz)));
  c2 = {c1.x + (q2 * vx), c1.y + (q2 * vy), c1.z + (q2 * vz)};
  const double ex3 = g.x - c2.x, ey3 = g.y - c2.y, ez3 = g.z - c2.z;
  const double sx3 = sqrt_core(sq(ex3) + sq(ey3) + sq(ez3));
  cq = div_core(L[3], sx3);
  cd = {ex3, ey3, ez3};
  const double gea = fabs(sx3 - L[3]);  // |F3 - goal| up to the band
  uint64_t gt3 = __builtin_amdgcn_ballot_w64(gea > band.hi);
  // (the goal error only matters where the start error has not decided already)
  uint64_t unc3 =
      ex & ~(gt3 | __builtin_amdgcn_ballot_w64(gea < band.lo) | gt);
  if (__builtin_expect(unc3 != 0, 0)) {
    const d3 c3 = {c2.x + (cq * ex3), c2.y + (cq * ey3), c2.z + (cq * ez3)};
    const double ge2 = dist3_sq(c3, g);
    gt3 = (gt3 & ~unc3) | (__builtin_amdgcn_ballot_w64(ge2 > tol2) & unc3);
  }
  cont = __builtin_amdgcn_inverse_ballot_w64(gt | gt3);
  return (fabs(q1) + fabs(q)) + (fabs(q2) + fabs(cq)) <= qmax;
}

}  // namespace ikhip
