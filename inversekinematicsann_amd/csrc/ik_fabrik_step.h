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
