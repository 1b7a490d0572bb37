// ik_common.h -- device helpers shared by the FK / FABRIK / ANN kernels.
//
// Float64 arithmetic here follows the reference's operation order exactly and
// the whole library is compiled with -ffp-contract=off (CPython never fuses a
// multiply-add), so that FABRIK iteration counts match the reference bit for
// bit.  The one deliberate difference: the reference squares with pow(v, 2)
// (glibc pow, kinematics/point.py:27-29, inverse.py:79,90,98), here v*v, the
// correctly rounded square; glibc pow differs from it in the last ulp on a
// small fraction of inputs.  See DESIGN.md "Numerics".
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>
#include <vector>

#include "../../include/ikhip.h"

namespace ikhip {

constexpr double kPi = 3.141592653589793;  // math.pi

// Device-side accumulators of one call (reset by reset_stats_kernel).  The
// batch sums are sharded: each workgroup reduces in registers/LDS and adds to
// shard blockIdx % kStatShards, so no single word takes more than a few
// hundred atomics per launch; the host folds the shards.
constexpr int kStatShards = 64;
constexpr int kOrdClasses = 16;  // FABRIK work-order cost classes (queue order: hardest first)
constexpr int kOrdShards = 16;   // ... and the counter shards per class (blocks b % kOrdShards)
// Work-queue heads of the persistent FABRIK kernel: one returning device-scope
// atomicAdd on a single word saturates near 88 grabs/us (MI355X_MICROARCH.md,
// "dequeue"), which 2048 waves grabbing 64-point chunks reach; a head per XCD
// (blocks b % 8 share one) divides that contention by 8.
constexpr int kQueueHeads = 8;
struct DevStats {
  unsigned long long first_oob;      // atomicMin of point index
  unsigned long long first_err_key;  // atomicMin of (index << 8) | code
  unsigned long long unseen;         // FABRIK classify: points whose goal cell the cost table has not seen
  // FABRIK work order: points per (cost class, block shard), and the scatter's
  // cursor inside each (class, shard) region of the queue
  unsigned int cls_tot[kOrdClasses][kOrdShards];
  unsigned int cls_cur[kOrdClasses][kOrdShards];
  unsigned long long sum_iters[kStatShards];
  unsigned long long n_capped[kStatShards];
  unsigned long long max_fk_err_bits[kStatShards];  // atomicMax on non-negative double bits
  double sum_fk_err[kStatShards];
  int max_iters[kStatShards];
  // the FABRIK iteration kernel's work queue: kQueueHeads heads, one 128-B line
  // each, head h handing out the queue's chunks h, h + kQueueHeads, ...
  alignas(128) unsigned long long heads[kQueueHeads][16];
};

struct d3 {
  double x, y, z;
};

// The FK-error histogram bin of e (ikhip.h IK_FKHIST_BINS): 16 bins per octave
// from the float64 exponent and top 4 mantissa bits, monotonic in e; -1 for NaN,
// inf and negative values (not counted, like the max / sum stats).
__host__ __device__ inline int fkhist_bin(double e) {
  if (!(e >= 0.0) || e > 1.7976931348623157e308) return -1;
  uint64_t b;
  __builtin_memcpy(&b, &e, sizeof(b));
  b &= 0x7fffffffffffffffull;
  const int k = ((int)(b >> 52) - (1023 - 64)) * 16 + (int)((b >> 48) & 15);
  return k < 0 ? 0 : (k >= IK_FKHIST_BINS ? IK_FKHIST_BINS - 1 : k);
}

// The reference's pow(v, 2).
__device__ __forceinline__ double sq(double v) { return v * v; }

// kinematics/point.py:25-29 get_distance_between, and its radicand
__device__ __forceinline__ double dist3_sq(d3 a, d3 b) {
  return sq(a.x - b.x) + sq(a.y - b.y) + sq(a.z - b.z);
}
__device__ __forceinline__ double dist3(d3 a, d3 b) { return sqrt(dist3_sq(a, b)); }

__device__ __forceinline__ void set_err(int &st, int code) {
  if (st == IK_OK) st = code;
}

// kinematics/point.py:32-45 get_point_between: s_c + ((d / |s-e|) * (e_c - s_c)).
// |s-e| == 0 raises ZeroDivisionError in the reference.  The differences are
// formed once: the distance squares s_c - e_c and fl(s_c - e_c) = -fl(e_c - s_c)
// exactly, so squaring e_c - s_c gives the same radicand bit for bit.
__device__ __forceinline__ d3 point_between(d3 s, d3 e, double d, int &st) {
  const double dx = e.x - s.x, dy = e.y - s.y, dz = e.z - s.z;
  double n = sqrt(sq(dx) + sq(dy) + sq(dz));
  if (n == 0.0) set_err(st, IK_E_ZERODIV);
  double q = d / n;
  d3 r;
  r.x = s.x + (q * dx);
  r.y = s.y + (q * dy);
  r.z = s.z + (q * dz);
  return r;
}

// The compiler's correctly rounded float64 sqrt and division (the AMDGPU
// lowerings of llvm.sqrt.f64 and fdiv double) are a Newton sequence wrapped in
// range handling: sqrt scales radicands below 2^-767 by 2^256 and patches 0/inf
// with v_cmp_class + selects; division pre/post-scales with v_div_scale /
// v_div_fmas and patches specials with v_div_fixup.  Where none of that fires
// the result is the bare sequence below, instruction for instruction, so these
// give the same bits as sqrt() / operator/ on their domains:
//   sqrt_core(x): 2^-767 <= x < 2^1024 (the high word of x in [hi(2^-767),
//     hi(+inf)), which also rejects 0, negatives and NaN);
//   div_core(a, b): b = sqrt_core(x) for such an x and 2^-100 <= |a| <= 2^100
//   (no v_div_scale case: exponent gap < 768, quotient and 1/b normal, a not tiny).
__device__ __forceinline__ double sqrt_core(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y;
  double h = y * 0.5;
  const double r = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, r, g);
  h = __builtin_fma(h, r, h);
  double e = __builtin_fma(-g, g, x);
  g = __builtin_fma(e, h, g);
  e = __builtin_fma(-g, g, x);
  return __builtin_fma(e, h, g);
}
__device__ __forceinline__ double div_core(double a, double b) {
  double r = __builtin_amdgcn_rcp(b);
  double e = __builtin_fma(-b, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-b, r, 1.0);
  r = __builtin_fma(r, e, r);
  const double q = a * r;
  const double res = __builtin_fma(-b, q, a);
  return __builtin_fma(res, r, q);
}

// point_between through sqrt_core / div_core.  dom accumulates the radicands'
// distance from sqrt_core's domain (sqrt_core_dom: max over calls < kCoreDom
// <=> all in the domain); d must be in div_core's (checked once on the host).
// Where the domain holds the result equals point_between's and no error is
// possible.
constexpr uint32_t kCoreDom = 0x6FF00000u;
__device__ __forceinline__ uint32_t sqrt_core_dom(double x) {
  return (uint32_t)__double2hiint(x) - 0x10000000u;
}
__device__ __forceinline__ d3 point_between_core(d3 s, d3 e, double d, uint32_t &dom) {
  const double dx = e.x - s.x, dy = e.y - s.y, dz = e.z - s.z;
  const double x = sq(dx) + sq(dy) + sq(dz);
  dom = max(dom, sqrt_core_dom(x));
  const double q = div_core(d, sqrt_core(x));
  d3 r;
  r.x = s.x + (q * dx);
  r.y = s.y + (q * dy);
  r.z = s.z + (q * dz);
  return r;
}

// CPython round(v, 8): exact value of v rounded half-even to 8 decimals, then
// the nearest double.  v*1e8 = p + e exactly; e breaks a tie at p = k + 1/2.
__device__ __forceinline__ double py_round8(double v) {
  const double s = 1e8;
  double p = v * s;
  if (!isfinite(p)) return v;
  double e = fma(v, s, -p);
  double fl = floor(p);
  double k;
  if (p - fl == 0.5) {
    k = (e > 0) ? fl + 1.0 : ((e < 0) ? fl : rint(p));
  } else {
    k = rint(p);
  }
  double r = k / s;
  if (r == 0.0) r = copysign(0.0, v);
  return r;
}

// math.acos: ValueError('math domain error') outside [-1, 1]; nan passes.
__device__ __forceinline__ double py_acos(double v, int &st) {
  if (v > 1.0 || v < -1.0) set_err(st, IK_E_DOMAIN);
  return acos(v);
}

// float division: ZeroDivisionError when the divisor is zero.
__device__ __forceinline__ double py_div(double a, double b, int &st) {
  if (b == 0.0) set_err(st, IK_E_ZERODIV);
  return a / b;
}

// ---------------------------------------------------------------- FK ----
// kinematics/forward.py:21-94.  A_i = Rz(theta)*Tz(d)*Tx(a)*Rx(alpha) and the
// chain M_{i+1} = M_i * A_{i+1}, each 4x4 product an FMA chain in k order from
// 0 (what numpy's dgemm does; pinned bit-exact by the oracle tests).
__device__ __forceinline__ void mm4(const double *A, const double *B, double *C) {
  double T[16];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k < 4; ++k) acc = fma(A[i * 4 + k], B[k * 4 + j], acc);
      T[i * 4 + j] = acc;
    }
#pragma unroll
  for (int i = 0; i < 16; ++i) C[i] = T[i];
}

__device__ __forceinline__ void ident4(double *M) {
#pragma unroll
  for (int i = 0; i < 16; ++i) M[i] = (i % 5 == 0) ? 1.0 : 0.0;
}

// sin and cos of |x| <= 2 pi (the reference's FK angle range, forward.py:23-25):
// Cody-Waite reduction by pi/2 in three parts, then fdlibm's __kernel_sin /
// __kernel_cos polynomials on [-pi/4, pi/4].  Absolute error <= 1.2e-16 against
// glibc over [-2 pi, 2 pi] (1 ulp for |result| >= 0.5; 2e7 samples, gcc restatement);
// ~40 instructions against ocml's general sincos.  Outside the range the result is
// finite garbage (the FK kernel reports those points as out of range).
__device__ __forceinline__ void sincos_fk(double x, double *sp, double *cp) {
  const double k = __builtin_rint(x * 0.63661977236758134308);
  double r = __builtin_fma(-k, 1.57079632673412561417e+00, x);
  r = __builtin_fma(-k, 6.07710050650619224932e-11, r);
  r = r + (-k * 2.02226624879595063154e-21);
  const double z = r * r;
  const double ps = __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, __builtin_fma(z,
                    __builtin_fma(z, 1.58969099521155010221e-10, -2.50507602534068634195e-08),
                    2.75573137070700676789e-06), -1.98412698298579493134e-04),
                    8.33333333332248946124e-03), -1.66666666666666324348e-01);
  const double sn = __builtin_fma(r * z, ps, r);
  const double pc = __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, __builtin_fma(z,
                    __builtin_fma(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09),
                    -2.75573143513906633035e-07), 2.48015872894767294178e-05),
                    -1.38888888888741095749e-03), 4.16666666666666019037e-02);
  const double hz = 0.5 * z, w = 1.0 - hz;
  const double cs = w + (((1.0 - w) - hz) + z * z * pc);
  const int q = (int)k;
  const double ss = (q & 1) ? cs : sn, cc = (q & 1) ? sn : cs;
  *sp = (q & 2) ? -ss : ss;
  *cp = ((q + 1) & 2) ? -cc : cc;
}

__device__ __forceinline__ bool angle_ok(double a) { return !((a < -2 * kPi) || (a > 2 * kPi)); }

__device__ __forceinline__ void dh_transform(double th, double eps, double a, double al,
                                             double *A) {
  double R[16], T1[16], T2[16], X[16];
  double c = cos(th), s = sin(th);
  ident4(R);
  R[0] = c; R[1] = -s; R[4] = s; R[5] = c;
  ident4(T1);
  T1[11] = eps;
  ident4(T2);
  T2[3] = a;
  double ca = cos(al), sa = sin(al);
  ident4(X);
  X[5] = ca; X[6] = -sa; X[9] = sa; X[10] = ca;
  mm4(R, T1, A);
  mm4(A, T2, A);
  mm4(A, X, A);
}

// dh: rows thetas(unused here), d, a, alpha; th: the 4 joint angles.
// Writes the translations of M_1..M_4.  Returns IK_OK or IK_E_ANGLE_RANGE.
__device__ __forceinline__ int fk_chain(const double *dh, const double th[4], d3 J[4]) {
  int st = IK_OK;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (!angle_ok(th[i]) || !angle_ok(dh[12 + i])) st = IK_E_ANGLE_RANGE;
  double M[16], A[16];
  dh_transform(th[0], dh[4], dh[8], dh[12], M);
  J[0].x = M[3]; J[0].y = M[7]; J[0].z = M[11];
#pragma unroll
  for (int i = 1; i < 4; ++i) {
    dh_transform(th[i], dh[4 + i], dh[8 + i], dh[12 + i], A);
    mm4(M, A, M);
    J[i].x = M[3]; J[i].y = M[7]; J[i].z = M[11];
  }
  return st;
}

// The per-robot constants of the FABRIK seed pose and of the FK round trip
// (RobotConstDev), computed once per robot by robot_const_kernel.
struct RobotConstDev {
  double lim[6];    // workspace limits (inverse.py:26-35)
  double jc[16];    // fk_error's per-joint constants (fk_trip_consts)
  double P[4][3];   // the seed chain's joints at theta_1 = 0 (seed_closed)
  int alpha_bad;
  int st;           // fk_chain's angle check of the constant angles
};
// The robot constants through the constant address space: wave-uniform
// s_load_dwordx* into SGPRs instead of vector loads per lane.
typedef const RobotConstDev __attribute__((address_space(4))) *RcConst;

// The seed pose in closed form.  theta_1 enters the DH chain only through the
// leftmost factor, A_1 = Rz(theta_1) C_1 (forward.py:63-70), so every seed joint
// is J_k = Rz(theta_1) P_k with P_k the chain's joint k at theta_1 = 0 (a robot
// constant), and cos / sin(atan2(y, x)) = (x, y) / |(x, y)|: one reciprocal root
// and four products per joint instead of atan2, cos, sin and three 3 x 4 matrix
// products (r05: ~530 VALU per prepared batch entry).  The joints differ from the
// reference's chain in the last bits of their x / y (for SixDOFRobot those are
// ~1e-16 in size, P_k = (~1e-16, ~1e-16, 2k + 2)): no FABRIK iteration count
// changed over 24M goals at tol 1e-3 .. 1e-8, random_dist and uniform box
// (tools/seed_form_check.c against the oracle's chain).  Goals on the z axis or
// with x^2 + y^2 outside the normal range (and NaN) take cos / sin of atan2 itself
// in a wave-uniform branch.  Returns the robot's constant status.
__device__ __forceinline__ int seed_closed(const RobotConstDev *rc, d3 g, d3 J[4]) {
  const RcConst k = (RcConst)rc;
  const double t = g.x * g.x + g.y * g.y;
  const bool fast = t >= 0x1p-1000 && t <= 0x1p1000;
  // 1 / sqrt(t): the hardware estimate and two coupled Newton steps (sqrt_core's
  // g / h iteration: h -> 1 / (2 sqrt(t)) within a few ulps)
  const double y0 = __builtin_amdgcn_rsq(t);
  double h = 0.5 * y0, gg = t * y0;
  double e = __builtin_fma(-h, gg, 0.5);
  h = __builtin_fma(h, e, h);
  gg = __builtin_fma(gg, e, gg);
  e = __builtin_fma(-h, gg, 0.5);
  h = __builtin_fma(h, e, h);
  double c = g.x * (2.0 * h), s = g.y * (2.0 * h);
  if (__builtin_expect(__any(!fast), 0)) {
    if (!fast) {
      const double th = atan2(g.y, g.x);
      c = cos(th);
      s = sin(th);
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const double px = k->P[j][0], py = k->P[j][1];
    J[j].x = __builtin_fma(c, px, -(s * py));
    J[j].y = __builtin_fma(s, px, c * py);
    J[j].z = k->P[j][2];
  }
  return k->st;
}

// The FK round trip of one point (cli.py:54-61 + the distance to the target),
// register-lean: the effector is Rz(t1) B1 Rz(t2) B2 Rz(t3) B3 Rz(t4) B4 e4
// with B_i = Tz(d_i) Tx(a_i) Rx(alpha_i) (forward.py:63-70 regrouped),
// applied right to left to a vector; jc[i] = {a_i, d_i, cos alpha_i, sin alpha_i}
// from the host (fk_trip_consts).  Same value as fk_chain up to rounding (~1e-15).
// The chain of fk_error from the angles' cosines and sines (c[i], s[i]) and
// whether every angle passed forward.py:23-25's range check (ok).
__device__ __forceinline__ double fk_error_cs(const double *jc, const double c[4],
                                              const double s[4], bool ok, double px, double py,
                                              double pz) {
  double x = jc[12], y = 0.0, z = jc[13];  // B4 e4 = (a4, 0, d4)
#pragma unroll
  for (int i = 3; i >= 0; --i) {
    double xr = c[i] * x - s[i] * y, yr = s[i] * x + c[i] * y;  // Rz(t_i)
    x = xr;
    y = yr;
    if (i > 0) {  // B_{i} (1-based), i.e. jc[i - 1]
      const double *b = jc + 4 * (i - 1);
      double yb = b[2] * y - b[3] * z, zb = b[3] * y + b[2] * z + b[1];
      x = x + b[0];
      y = yb;
      z = zb;
    }
  }
  d3 e = {x, y, z}, p = {px, py, pz};
  return ok ? dist3(e, p) : __builtin_nan("");
}

__device__ __forceinline__ double fk_error(const double *jc, const double th[4], double px,
                                           double py, double pz, int alpha_bad) {
  bool ok = !alpha_bad;
  double c[4], s[4];
#pragma unroll
  for (int i = 3; i >= 0; --i) {
    ok = ok && angle_ok(th[i]);
    sincos_fk(th[i], &s[i], &c[i]);  // |th| <= 2 pi here (ok); outside, the result is NaN anyway
  }
  return fk_error_cs(jc, c, s, ok, px, py, pz);
}

// Same chain, writing all four cumulative transforms (row-major 4x4 each).
__device__ __forceinline__ int fk_chain_mats(const double *dh, const double th[4], double *out) {
  int st = IK_OK;
  for (int i = 0; i < 4; ++i)
    if (!angle_ok(th[i]) || !angle_ok(dh[12 + i])) st = IK_E_ANGLE_RANGE;
  double M[16], A[16];
  dh_transform(th[0], dh[4], dh[8], dh[12], M);
  for (int k = 0; k < 16; ++k) out[k] = M[k];
  for (int i = 1; i < 4; ++i) {
    dh_transform(th[i], dh[4 + i], dh[8 + i], dh[12 + i], A);
    mm4(M, A, M);
    for (int k = 0; k < 16; ++k) out[16 * i + k] = M[k];
  }
  return st;
}

// ------------------------------------------------------------- stats ----
__device__ __forceinline__ void record_error(DevStats *S, int64_t idx, int code) {
  unsigned long long key = ((unsigned long long)idx << 8) | (unsigned long long)code;
  atomicMin(&S->first_err_key, key);
}

__device__ __forceinline__ bool outside(const double *lim, double x, double y, double z) {
  // kinematics/inverse.py:26-35: inclusive bounds, dict order x, y, z
  return (x < lim[0] || x > lim[1]) || (y < lim[2] || y > lim[3]) || (z < lim[4] || z > lim[5]);
}

// 64-lane wave sum of a 64-bit value.
__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ int wave_max_i32(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = max(v, __shfl_xor(v, off, 64));
  return v;
}

__device__ __forceinline__ double wave_max_f64(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
  return v;
}

__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Block-wide FABRIK iteration stats (blockDim 256): one atomic per counter per
// block, into the block's shard.  Every thread of the block must call it.
// s / c / m: this thread's iteration sum, capped-point count and largest count.
__device__ __forceinline__ void block_iter_stats_acc(DevStats *S, unsigned long long s,
                                                     unsigned long long c, int m) {
  __shared__ unsigned long long red_s[4], red_c[4];
  __shared__ int red_m[4];
  s = wave_sum_u64(s);
  c = wave_sum_u64(c);
  m = wave_max_i32(m);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red_s[w] = s;
    red_c[w] = c;
    red_m[w] = m;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nw = (blockDim.x + 63) >> 6;
    for (int i = 1; i < nw; ++i) {
      s += red_s[i];
      c += red_c[i];
      m = max(m, red_m[i]);
    }
    const int sh = blockIdx.x % kStatShards;
    if (s) atomicAdd(&S->sum_iters[sh], s);
    if (c) atomicAdd(&S->n_capped[sh], c);
    if (m) atomicMax(&S->max_iters[sh], m);
  }
}

__device__ __forceinline__ void block_iter_stats(DevStats *S, bool valid, int it, int max_iter) {
  block_iter_stats_acc(S, valid ? (unsigned long long)it : 0ull,
                       (valid && it >= max_iter) ? 1ull : 0ull, valid ? it : 0);
}

// FK round-trip error stats: one atomic pair per wave into the block's shard.
// mx / sm: this lane's largest and summed finite errors.  The whole wave calls it.
__device__ __forceinline__ void wave_fk_stats(DevStats *S, double mx, double sm) {
  mx = wave_max_f64(mx);
  sm = wave_sum_f64(sm);
  if ((threadIdx.x & 63) == 0) {
    const int sh = blockIdx.x % kStatShards;
    atomicMax(&S->max_fk_err_bits[sh], (unsigned long long)__double_as_longlong(mx));
    atomicAdd(&S->sum_fk_err[sh], sm);
  }
}

}  // namespace ikhip

// Launchers implemented in the .hip files and called by ik_api.cpp.
namespace ikhip {
struct RobotDev {
  double dh[16];
  double links[4];
  double lim[6];
};

// Host: the per-joint constants of fk_error, {a_i, d_i, cos alpha_i, sin alpha_i},
// and whether some |alpha_i| > 2 pi (then FK raises for every point, forward.py:23-25).
inline void fk_trip_consts(const RobotDev &r, double jc[16], int *alpha_bad) {
  *alpha_bad = 0;
  for (int i = 0; i < 4; ++i) {
    const double al = r.dh[12 + i];
    jc[4 * i + 0] = r.dh[8 + i];
    jc[4 * i + 1] = r.dh[4 + i];
    jc[4 * i + 2] = std::cos(al);
    jc[4 * i + 3] = std::sin(al);
    if (al < -2 * kPi || al > 2 * kPi) *alpha_bad = 1;
  }
}

// Optional per-kernel HIP-event timing of the current call (ik_ctx_set_timing):
// launchers bracket every kernel with kt_begin / IK_LAUNCH / kt_end.  The kernel's
// events are handed to hipExtLaunchKernel, so the dispatch itself stamps its own
// start and end: neither the kernels ahead of it on the stream nor the host's
// launch latency fall inside the interval.  Spans that are not
// one kernel (the RCCL gather) use kt_span_begin: stream markers.
void kt_begin(const char *name, hipStream_t st);
void kt_span_begin(const char *name, hipStream_t st);
void kt_end(hipStream_t st);
// the armed slot's events for the kernel about to launch (false: timing is off)
bool kt_take_events(hipEvent_t *beg, hipEvent_t *end);
}  // namespace ikhip
#include <hip/hip_ext.h>
namespace ikhip {
#define IK_LAUNCH(K, G, B, SH, ST, ...)                                             \
  do {                                                                              \
    hipEvent_t ik_kb_ = nullptr, ik_ke_ = nullptr;                                  \
    if (::ikhip::kt_take_events(&ik_kb_, &ik_ke_))                                  \
      hipExtLaunchKernelGGL(K, G, B, SH, ST, ik_kb_, ik_ke_, 0u, __VA_ARGS__);      \
    else                                                                            \
      hipLaunchKernelGGL(K, G, B, SH, ST, __VA_ARGS__);                             \
  } while (0)

void launch_reset_stats(DevStats *S, hipStream_t st);
void launch_check_limits(const RobotDev &r, const double *pts, int64_t n, DevStats *S,
                         hipStream_t st);
void launch_fk(const RobotDev &r, const double *ang, int64_t n, double *xyz, double *mats,
               DevStats *S, hipStream_t st);
// FK of a chain of nj (2..kFkMaxJoints) joints; dh: device 4 x nj, mats nullable
// n x nj x 16 (2..8 unrolled, longer chains a run-time joint loop).
constexpr int kFkMaxJoints = 1024;
// Fabrik.calculate's chain length bound (ik_fabrik_calc).  Chains past 8 joints
// run one goal per lane with the chain in its output row, so a goal costs about
// nj * max_iter * 2 dependent point_between steps (~0.4 us each, an L2 round
// trip): 4096 joints at 100 iterations is ~0.3 s for a launch of any width
// (tests/test_gpu_parity.py::test_fabrik_calc_longest_chain), well inside the
// GPU's hang detection; longer chains are refused.
constexpr int kCalcMaxJoints = 4096;
void launch_fk_n(int nj, const double *dh, const double *ang, int64_t n, double *xyz,
                 double *mats, DevStats *S, hipStream_t st);
// FABRIK work order (ik_fabrik.hip "Work order"): per context, the largest
// iteration count recorded in each goal cell (distance x elevation from the
// shoulder) on the context's earlier calls decides which points start first.
constexpr int kOrdCellsR = 64, kOrdCellsE = 16, kOrdCells = kOrdCellsR * kOrdCellsE;
constexpr int kOrdSample = 256;           // 1 point in 256 is recorded ...
constexpr int kOrdMaxSample = 1 << 14;    // ... up to this many per call
struct FabOrderDev {
  unsigned int key[kOrdCells];  // 1 + largest recorded iterations per cell, 0 = unseen
  unsigned int sample[kOrdMaxSample];  // (cell << 16 | iterations) records of the call
};

// FABRIK ikine.  scratch must hold fabrik_scratch_bytes(n).  ord: the
// context's cost table (zero-initialised once), or null for queue order =
// point order.  fk_err (nullable): |FK(theta) - p| per point, max/sum into S.
size_t fabrik_scratch_bytes(int64_t n);
void launch_fabrik_ikine(const RobotDev &r, const double *pts, int64_t n, double tol,
                         int max_iter, double *ang, int32_t *iters, double *joints,
                         double *fk_err, bool check_limits, void *scratch, DevStats *S, hipStream_t st,
                         int variant, int core, FabOrderDev *ord, const RobotConstDev *rc,
                         unsigned long long *dbg, int bpc = 0, bool prior = false);
constexpr size_t kFabrikDebugWords = 64 + 24 * 4096;  // diagnostic build: totals + per-wave records
// Per-robot seed constants (RobotConstDev) into device memory, on stream st.
void launch_robot_const(const RobotDev &r, RobotConstDev *rc, hipStream_t st);
// The robot constants of the last launch_robot_const, for an unchanged robot.
bool robot_const_current(const RobotDev &r);
void launch_fabrik_calc(int nj, const double *dists, const double *init, bool init_shared,
                        const double *goals, int64_t n, double tol, int max_iter,
                        double *joints, int32_t *iters, DevStats *S, hipStream_t st);

constexpr int kAnnMaxLayers = 24;
constexpr int kAnnMaxWidth = 1024;  // > 512: the wide build (ik_ann_w.hip), fp32 only
struct AnnModelDev {
  int n_layers;
  int kp[kAnnMaxLayers];  // padded in-dim (multiple of 8)
  int np[kAnnMaxLayers];  // padded out-dim (multiple of 32)
  int act[kAnnMaxLayers];
  const float4 *wp[kAnnMaxLayers];  // packed weights (see ik_ann.hip)
  const void *wx[kAnnMaxLayers];    // split modes: the layer's weight operand, else null
  float xinv[kAnnMaxLayers];        // fp16x3: 2^-k, k the layer's weight pre-scale exponent
  int xmode;                        // 0 fp32, 1 bf16x6, 2 fp16x3 (IK_ANN_*)
  const float *bias[kAnnMaxLayers];
  double xm[3], xs[3], ym[4], ys[4];
};
size_t ann_packed_floats(int k, int n);  // floats of one packed layer
void ann_pack_layer(const float *W, int k, int n, float *dst);  // host-side packing
size_t ann_x_bytes(int k, int n);  // bytes of one layer's bf16x6 weight operand
void ann_pack_layer_x(const float *W, int k, int n, void *dst);
size_t ann_h_bytes(int k, int n);  // bytes of one layer's fp16x3 weight operand
int ann_h_scale_exp(const float *W, int k, int n);  // the weight pre-scale exponent k
void ann_pack_layer_h(const float *W, int k, int n, int scale_exp, void *dst);
size_t ann_debug_words();  // u64 slots of the diagnostic stamp buffer
void launch_ann(const AnnModelDev &m, const RobotDev &r, const double *pts, int64_t n,
                float *ang, double *fk_err, bool check_limits, DevStats *S, hipStream_t st,
                unsigned long long *dbg);
void launch_ann_wide(const AnnModelDev &m, const RobotDev &r, const double *pts, int64_t n,
                     float *ang, double *fk_err, bool check_limits, DevStats *S, hipStream_t st,
                     unsigned long long *dbg);

// Models outside the fused kernel's caps (more than kAnnMaxLayers layers or a
// layer wider than kAnnMaxWidth): layer at a time through HBM (ik_ann_big.hip),
// fp32, or bf16x6 for the hidden layers after the first in a split mode.  Bounds:
constexpr int kAnnBigMaxLayers = 4096;
constexpr int kAnnBigMaxWidth = 16384;
struct AnnBigLayer {
  int kp, np, act;   // padded in-dim (multiple of 8), padded out-dim (multiple of 32)
  const float *wp;   // packed weights (ann_pack_layer order)
  const float *bias; // np floats, zero past the layer's width
  const uint16_t *wx = nullptr;  // bf16x6 planes (ann_big_pack_x), hidden layers only
};
struct AnnBigModel {
  std::vector<AnnBigLayer> layers;
  double xm[3], xs[3], ym[4], ys[4];
};
// floats per activation row (the widest padded layer, at least 8)
size_t ann_big_ld(const AnnBigModel &m);
// the layered path's bf16x6 weight planes: [plane][ceil(k / 32)][n rounded up to
// 128][32] bf16, ann_big_x_bytes(k, n) bytes
size_t ann_big_x_bytes(int k, int n);
void ann_big_pack_x(const float *W, int k, int n, void *dst);
// rows per chunk that fit two activation buffers in act_bytes (multiple of 128)
int64_t ann_big_rows(const AnnBigModel &m, size_t act_bytes);
// act: 2 * chunk_rows * ann_big_ld(m) floats
void launch_ann_big(const AnnBigModel &m, const RobotDev &r, const double *pts, int64_t n,
                    float *ang, double *fk_err, bool check_limits, DevStats *S, hipStream_t st,
                    float *act, int64_t chunk_rows, int xmode = 0);
}  // namespace ikhip
