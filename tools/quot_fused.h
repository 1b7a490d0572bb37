// quot_fused.h -- the r05 candidate that tools/quot_check.hip and
// tools/quot_fab_check.hip test (measured -4 / -8 % and DROPPED: not bit-identical,
// profiles/r05/quot_check.txt): d / sqrt(x) with the divisor's reciprocal seeded
// from sqrt_core's own refined half reciprocal root h (2h ~ 1 / sqrt(x)) and one
// Newton step, instead of v_rcp_f64 and two (div_core).  Kept with the tools so
// that the record can be reproduced; the product never used it.
#pragma once

#include "../inversekinematicsann_amd/csrc/ik_common.h"

namespace ikhip {

__device__ __forceinline__ double quot_sqrt_core(double a, double x) {
  // sqrt_core's sequence (ik_common.h), keeping h
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y;
  double h = y * 0.5;
  const double r = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, r, g);
  h = __builtin_fma(h, r, h);
  double e = __builtin_fma(-g, g, x);
  g = __builtin_fma(e, h, g);
  e = __builtin_fma(-g, g, x);
  const double s = __builtin_fma(e, h, g);
  // 1 / s from 2h, one Newton step; then div_core's quotient and correction
  double rc = h + h;
  const double t = __builtin_fma(-s, rc, 1.0);
  rc = __builtin_fma(rc, t, rc);
  const double q = a * rc;
  const double res = __builtin_fma(-s, q, a);
  return __builtin_fma(res, rc, q);
}

}  // namespace ikhip
