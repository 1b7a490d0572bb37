// ik_fabrik.hip -- batched FABRIK inverse kinematics for gfx950.
//
// Restates, one goal point per lane in float64, the reference's
//   FabrikInverseKinematics.ikine   kinematics/inverse.py:115-139
//   Fabrik.calculate / __backward / __forward   kinematics/fabrik.py:19-67
//   __get_angles                    kinematics/inverse.py:54-112
// with the same operation order, so iteration counts are bit-exact.
//
// Two pipelines (DESIGN.md "FABRIK"):
//  * fused (default): classify + scatter (the hard-first work order, 6 bytes
//    per point) -> iter_kernel: persistent; each wave prepares batches of seed
//    poses into its LDS batch, refills the lanes whose points converged from it
//    (so a wave does not wait for its slowest lane), parks finished lanes in an
//    LDS ring and runs the angles step + FK round trip + batch stats on them in
//    batches -> fold (the samples into the cost table).  Seed poses and final
//    joints never touch HBM.
//  * simple: everything in one kernel, one point per lane, no refill.
// Per point the state is 4 joints + goal (15 doubles) held in VGPRs.
#include <atomic>
#include <cmath>

#include "ik_common.h"
#include "ik_fabrik_step.h"

namespace ikhip {

// div_core's domain for the link lengths (the numerators): 2^-100 <= |L| <= 2^100.
static bool links_core_ok(const double *L, int n) {
  for (int k = 0; k < n; ++k) {
    const double v = std::fabs(L[k]);
    if (!(v >= 0x1p-100 && v <= 0x1p100)) return false;
  }
  return true;
}

// The largest x with fl(sqrt(x)) <= tol (NaN for a NaN tol, -inf for a
// negative one), so that the reference's `sqrt(x) > tol` is `x > t` bit for
// bit.  The loop's initial errors of 1.0 stay 1.0 (sqrt(1) = 1 exactly).
static double tol_threshold(double tol) {
  if (std::isnan(tol)) return NAN;
  if (tol < 0) return -INFINITY;
  if (std::isinf(tol)) return INFINITY;
  double t = tol * tol;
  while (std::sqrt(t) > tol) t = std::nextafter(t, -INFINITY);
  for (;;) {
    const double u = std::nextafter(t, INFINITY);
    if (std::sqrt(u) <= tol) t = u;
    else break;
  }
  return t;
}

// kinematics/inverse.py:54-112 __get_angles; J = FABRIK joints B, C, D, E.
__device__ __forceinline__ void get_angles(const d3 J[4], double th[4], int &st) {
  const d3 A = {0.0, 0.0, 0.0};
  const d3 B = J[0], C = J[1], D = J[2], E = J[3];
  th[0] = atan2(E.y, E.x);
  double ab = dist3(A, B), bc = dist3(B, C), cd = dist3(C, D), de = dist3(D, E);
  double ac = dist3(A, C);
  double num = (sq(ab) + sq(bc)) - sq(ac);
  double den = 2 * ab * bc;
  double a2 = py_acos(py_round8(py_div(num, den, st)), st);
  th[1] = (C.x * D.x < 0) ? ((3 * kPi / 2) - a2) : -(kPi / 2 - a2);
  double bd = dist3(B, D);
  num = (sq(bc) + sq(cd)) - sq(bd);
  den = 2 * bc * cd;
  double a3 = py_acos(py_round8(py_div(num, den, st)), st);
  th[2] = -(kPi - a3);
  double ce = dist3(C, E);
  num = (sq(cd) + sq(de)) - sq(ce);
  den = 2 * cd * de;
  double a4 = py_acos(py_round8(py_div(num, den, st)), st);
  d3 m = point_between(C, E, dist3(C, E) / 2, st);
  double da = dist3(B, m);
  double db = dist3(B, D);
  th[3] = (db > da) ? -(kPi - a4) : (kPi - a4);
}

// ---- the angles step through cheaper sequences ------------
// Everything __get_angles compares or rounds -- the distances, the law-of-
// cosines quotients, round(., 8), the C.x D.x and |B - D| > |B - m| tests -- must
// keep the reference's bits (a different round(., 8) moves an angle by up to
// 1e-4 near a straight joint).  sqrt_core / div_core give those bits on their
// domains (ik_common.h).  Only the final math.acos / math.atan2 values leave
// the kernel, and those need not be glibc's last bit (ocml's never were): the
// angles are held to 1e-9 of the oracle (the north star's tolerance is 1e-5).
// acos_fast / atan2_fast: polynomials fitted against mpmath (asin on [0, 1/2],
// degree 11 in u^2, <= 2.1 ulp; atan on [0, tan(pi/8)], degree 10, <= 1 ulp), the
// usual reductions, pi split in two parts.  ~40 VALU instructions each against
// ~100 (ocml acos) and ~114 (ocml atan2).
constexpr double kPio2Hi = 0x1.921fb54442d18p0, kPio2Lo = 0x1.1a62633145c07p-54;
constexpr double kPio4Hi = 0x1.921fb54442d18p-1, kPio4Lo = 0x1.1a62633145c07p-55;
constexpr double kPiHi = 0x1.921fb54442d18p1, kPiLo = 0x1.1a62633145c07p-53;

// asin(u) for u in [0, 1/2]: u + u z P(z), z = u^2 (z passed in)
__device__ __forceinline__ double asin_small(double u, double z) {
  double p = 0x1.c4e4e17088d7fp-6;
  p = __builtin_fma(p, z, -0x1.478579af5a664p-7);
  p = __builtin_fma(p, z, 0x1.fe14951c32a4cp-7);
  p = __builtin_fma(p, z, 0x1.0524bf7ebc431p-7);
  p = __builtin_fma(p, z, 0x1.83eb350c10662p-7);
  p = __builtin_fma(p, z, 0x1.c89fb23c062d2p-7);
  p = __builtin_fma(p, z, 0x1.1c5717f04e8d6p-6);
  p = __builtin_fma(p, z, 0x1.6e8b4bd3059d9p-6);
  p = __builtin_fma(p, z, 0x1.f1c71e76e5bd8p-6);
  p = __builtin_fma(p, z, 0x1.6db6db6aaeb82p-5);
  p = __builtin_fma(p, z, 0x1.3333333335124p-4);
  p = __builtin_fma(p, z, 0x1.555555555555fp-3);
  return __builtin_fma(u * z, p, u);
}

// atan(t) for |t| <= tan(pi/8): t + t s P(s), s = t^2
__device__ __forceinline__ double atan_small(double t) {
  const double s = t * t;
  double p = -0x1.f318cc05bca37p-7;
  p = __builtin_fma(p, s, 0x1.2487560b8b924p-5);
  p = __builtin_fma(p, s, -0x1.959b5ed0b32b2p-5);
  p = __builtin_fma(p, s, 0x1.dd91ab8788317p-5);
  p = __builtin_fma(p, s, -0x1.10d3fc8f710cbp-4);
  p = __builtin_fma(p, s, 0x1.3b0f4916f8726p-4);
  p = __builtin_fma(p, s, -0x1.745ce3b26915fp-4);
  p = __builtin_fma(p, s, 0x1.c71c705fa87fap-4);
  p = __builtin_fma(p, s, -0x1.24924921fc848p-3);
  p = __builtin_fma(p, s, 0x1.99999999958a3p-3);
  p = __builtin_fma(p, s, -0x1.5555555555541p-2);
  return __builtin_fma(t * s, p, t);
}

// math.acos on [-1, 1] (NaN outside, and for NaN): |x| <= 1/2 as pi/2 -+ asin|x|,
// else 2 asin(sqrt((1 - |x|) / 2)) (x > 0) or pi minus it; 1 - |x| is exact there.
__device__ __forceinline__ double acos_fast(double x) {
  const double ax = fabs(x);
  const bool small = ax <= 0.5;
  const double zl = (1.0 - ax) * 0.5;  // 0 or >= 2^-54: sqrt_core's domain or 0
  const double z = small ? x * x : zl;
  const double u = small ? ax : (zl > 0.0 ? sqrt_core(zl) : 0.0);
  const double p = asin_small(u, z);
  const double r_small = x >= 0.0 ? kPio2Hi - (p - kPio2Lo) : kPio2Hi + (p + kPio2Lo);
  const double r_large = x > 0.0 ? 2.0 * p : kPiHi - (2.0 * p - kPiLo);
  const double r = small ? r_small : r_large;
  return ax <= 1.0 ? r : __builtin_nan("");
}

// math.atan2 where both |x| and |y| are in [2^-100, 2^100] (div_core's domain);
// the caller sends zeros, non-finite and extreme values to the library's atan2.
__device__ __forceinline__ double atan2_fast(double y, double x) {
  const double ax = fabs(x), ay = fabs(y);
  const bool swap = ay > ax;
  const double r = div_core(swap ? ax : ay, swap ? ay : ax);  // [0, 1]
  const bool red = r > 0x1.a827999fcef32p-2;  // tan(pi/8): atan r = pi/4 + atan((r-1)/(r+1))
  const double t = red ? div_core(r - 1.0, r + 1.0) : r;
  double a = atan_small(t);
  a = red ? kPio4Hi + (a + kPio4Lo) : a;
  a = swap ? kPio2Hi - (a - kPio2Lo) : a;
  a = x < 0.0 ? kPiHi - (a - kPiLo) : a;
  return copysign(a, y);
}

__device__ __forceinline__ bool in_div_domain(double v) {
  const double a = fabs(v);
  return a >= 0x1p-100 && a <= 0x1p100;
}

// dist3 through sqrt_core (same bits where dom stays below kCoreDom)
__device__ __forceinline__ double dist3c(d3 a, d3 b, uint32_t &dom) {
  const double x = dist3_sq(a, b);
  dom = max(dom, sqrt_core_dom(x));
  return sqrt_core(x);
}

// round(v, 8) (py_round8) with the final k / 1e8 through div_core
__device__ __forceinline__ double py_round8_core(double v, bool &ok) {
  const double s = 1e8;
  const double p = v * s;
  if (!isfinite(p)) return v;
  const double e = fma(v, s, -p);
  const double fl = floor(p);
  double k;
  if (p - fl == 0.5) {
    k = (e > 0) ? fl + 1.0 : ((e < 0) ? fl : rint(p));
  } else {
    k = rint(p);
  }
  ok = ok && (k == 0.0 || in_div_domain(k));
  double r = div_core(k, s);
  if (r == 0.0) r = copysign(0.0, v);
  return r;
}

// sqrt(1 - v^2) = sin(acos(v)) for |v| <= 1 (the FK round trip's sines): 1 - v^2
// in one rounding (fma), its root from the hardware estimate and one coupled
// Newton step -- a few ulps, far inside the round trip's 1e-12 (its value is only
// reported, never compared: tests/test_gpu_parity.py
// ::test_fabrik_fk_err_equals_standalone_fk).
__device__ __forceinline__ double sin_of_acos(double v) {
  const double t = __builtin_fma(-v, v, 1.0);
  const double y = __builtin_amdgcn_rsq(t);
  const double h = 0.5 * y, g = t * y;
  const double e = __builtin_fma(-h, g, 0.5);
  return t > 0.0 ? __builtin_fma(g, e, g) : 0.0;
}

// __get_angles (inverse.py:54-112) through the core sequences; returns false
// (and the caller runs get_angles) when some radicand or quotient leaves their
// domains -- coincident joints, a zero divisor, non-finite joints -- or the
// effector's x or y is zero or extreme (atan2's special cases).
// cs / sn: the angles' cosines and sines for the FK round trip (cli.py:54-61),
// from the values the angles come from instead of sin / cos of the angles:
// theta_1 = atan2(E.y, E.x) gives (E.x, E.y) / |(E.x, E.y)|, and every other angle
// is +-(k pi / 2 -+ acos(v)) of a law-of-cosines value v, so its cosine and sine
// are +-v and +-sqrt(1 - v^2).  They differ from sin / cos of the rounded angles
// by a few ulps (the rounding of the angles themselves), not 4 x 40 instructions.
__device__ __forceinline__ bool get_angles_core(const d3 J[4], double th[4], int &st,
                                                double cs[4], double sn[4]) {
  const d3 A = {0.0, 0.0, 0.0};
  const d3 B = J[0], C = J[1], D = J[2], E = J[3];
  uint32_t dom = 0;
  bool ok = in_div_domain(E.x) && in_div_domain(E.y);
  const double ab = dist3c(A, B, dom), bc = dist3c(B, C, dom), cd = dist3c(C, D, dom),
               de = dist3c(D, E, dom);
  const double ac = dist3c(A, C, dom);
  auto quot = [&](double num, double den) {
    ok = ok && (num == 0.0 || in_div_domain(num)) && in_div_domain(den);
    return div_core(num, den);
  };
  auto acos_py = [&](double v) {
    if (v > 1.0 || v < -1.0) set_err(st, IK_E_DOMAIN);
    return acos_fast(v);
  };
  double num = (sq(ab) + sq(bc)) - sq(ac);
  double den = 2 * ab * bc;
  const double v2 = py_round8_core(quot(num, den), ok);
  const double a2 = acos_py(v2);
  const bool up = C.x * D.x < 0;
  th[1] = up ? ((3 * kPi / 2) - a2) : -(kPi / 2 - a2);
  const double w2 = sin_of_acos(v2);
  cs[1] = up ? -w2 : w2;  // cos(3 pi / 2 - a) = -sin a, cos(a - pi / 2) = sin a
  sn[1] = -v2;            // sin of either is -cos a
  const double bd = dist3c(B, D, dom);
  num = (sq(bc) + sq(cd)) - sq(bd);
  den = 2 * bc * cd;
  const double v3 = py_round8_core(quot(num, den), ok);
  const double a3 = acos_py(v3);
  th[2] = -(kPi - a3);
  cs[2] = -v3;  // a - pi
  sn[2] = -sin_of_acos(v3);
  const double ce = dist3c(C, E, dom);
  num = (sq(cd) + sq(de)) - sq(ce);
  den = 2 * cd * de;
  const double v4 = py_round8_core(quot(num, den), ok);
  const double a4 = acos_py(v4);
  // get_point_between(C, E, |C - E| / 2): |C - E| is ce again (the radicand squares
  // E - C = -(C - E) exactly) and (ce / 2) / ce is exactly 0.5 for a ce in the domain
  const d3 m = {C.x + (0.5 * (E.x - C.x)), C.y + (0.5 * (E.y - C.y)), C.z + (0.5 * (E.z - C.z))};
  const double da = dist3c(B, m, dom);
  th[3] = (bd > da) ? -(kPi - a4) : (kPi - a4);  // db = |B - D| = bd
  cs[3] = -v4;  // a - pi or pi - a
  const double w4 = sin_of_acos(v4);
  sn[3] = (bd > da) ? -w4 : w4;
  // th[0] = atan2_fast(E.y, E.x): by the caller, after the fallback pass; its
  // cosine and sine from E (E.x, E.y in the division domain: t is normal)
  {
    const double t = E.x * E.x + E.y * E.y;
    const double y = __builtin_amdgcn_rsq(t);
    const double h = 0.5 * y, g = t * y;
    const double e = __builtin_fma(-h, g, 0.5);
    const double yi = __builtin_fma(y, e, y);
    cs[0] = E.x * yi;
    sn[0] = E.y * yi;
  }
  return ok && dom < kCoreDom;
}

// Seed pose, inverse.py:123-130: FK of [atan2(y, x), thetas[1:]] (the
// reference writes theta_1 into dh_matrix[0][0] and runs fkine on that row), in
// closed form from the per-robot constants (seed_closed, ik_common.h; r05 and
// before: seed_chain, the DH chain's own products).
__device__ __forceinline__ int seed_pose(const RobotConstDev *rc, d3 g, d3 J[4]) {
  return seed_closed(rc, g, J);
}

// The per-robot constants (RobotConstDev).  jc / alpha_bad come from the host
// (fk_trip_consts: the values the ANN kernel's round trip uses too).
struct FkTrip {
  double jc[16];
  int alpha_bad;
};

__global__ void robot_const_kernel(RobotDev r, FkTrip t, RobotConstDev *rc) {
  if (threadIdx.x != 0) return;
  int st = IK_OK;
  for (int k = 1; k < 4; ++k)
    if (!angle_ok(r.dh[k])) st = IK_E_ANGLE_RANGE;
  for (int k = 0; k < 4; ++k)
    if (!angle_ok(r.dh[12 + k])) st = IK_E_ANGLE_RANGE;
  for (int k = 0; k < 6; ++k) rc->lim[k] = r.lim[k];
  for (int k = 0; k < 16; ++k) rc->jc[k] = t.jc[k];
  rc->alpha_bad = t.alpha_bad;
  rc->st = st;
  // seed_closed's P_k: the seed chain at theta_1 = 0 (Rz(0) = I exactly)
  {
    const double th[4] = {0.0, r.dh[1], r.dh[2], r.dh[3]};
    d3 P[4];
    (void)fk_chain(r.dh, th, P);
    for (int j = 0; j < 4; ++j) {
      rc->P[j][0] = P[j].x;
      rc->P[j][1] = P[j].y;
      rc->P[j][2] = P[j].z;
    }
  }
}

void launch_robot_const(const RobotDev &r, RobotConstDev *rc, hipStream_t stream) {
  FkTrip t;
  fk_trip_consts(r, t.jc, &t.alpha_bad);
  IK_LAUNCH(robot_const_kernel, dim3(1), dim3(64), 0, stream, r, t, rc);
}

__device__ __forceinline__ void store_joints(double *dst, int64_t i, const d3 J[4]) {
  double *p = dst + 12 * i;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    p[3 * k] = J[k].x;
    p[3 * k + 1] = J[k].y;
    p[3 * k + 2] = J[k].z;
  }
}

__device__ __forceinline__ void load_joints(const double *src, int64_t i, d3 J[4]) {
  const double2 *p = reinterpret_cast<const double2 *>(src + 12 * i);
  double2 v0 = p[0], v1 = p[1], v2 = p[2], v3 = p[3], v4 = p[4], v5 = p[5];
  J[0] = {v0.x, v0.y, v1.x};
  J[1] = {v1.y, v2.x, v2.y};
  J[2] = {v3.x, v3.y, v4.x};
  J[3] = {v4.y, v5.x, v5.y};
}


struct FabArgs {
  RobotDev r;
  const RobotConstDev *rc;  // seed constants (robot_const_kernel)
  const double *pts;
  int64_t n;
  double tol;      // fabrik.py:57 err_margin, as given
  double tol2;     // tol_threshold(tol): the loop compares squared errors with it
  ErrBand band;    // the lazy errors' band (fabrik_band) for lanes with |J0|_1 + |goal|_1 <= band_n1
  double band_n1;
  double qmax;     // the core-domain test on the quotients (fabrik_qmax)
  int max_iter;
  int check_limits;
  double *ang;
  int32_t *iters;   // nullable
  double *joints;   // final joints n x 12 (nullable)
  double *fk_err;   // |FK(theta) - p| per point (nullable; max/sum into S)
  DevStats *S;
  int chunk;        // work-queue grab size of the persistent iteration kernel (1..64)
  // hard-first ordering (see "Work order" below); unused when perm is null
  int32_t *perm;    // queue position -> point index
  uint16_t *cell;   // per point: goal cell (bits 0-9) | cost class << 10
  FabOrderDev *ord; // context-owned cost table
  int prior_gate;   // the table is a built-in prior no call has taught yet (see scatter)
  unsigned long long *dbg;  // diagnostic build only: iteration-kernel counters
};

// Diagnostic counters of the iteration kernel (-DIKHIP_DIAG, libikhip_diag.so,
// tools/fabrik_diag.py): per wave, summed into dbg[0..7], and per wave w at
// dbg[64 + 4w ..]: s_memrealtime (100 MHz) at start, when the queue ran dry
// for it and at the end, and the steps it ran after the queue ran dry.
enum { kDiagLoops, kDiagSteps, kDiagLaneSteps, kDiagRefills, kDiagGrabs, kDiagFallbacks,
       kDiagWaves, kDiagFlushes, kDiagFlushTicks, kDiagPrepTicks, kDiagRefillTicks,
       kDiagParkTicks, kDiagStageTicks, kDiagCount };
// per-wave record (kDiagWords): the counters above, then s_memrealtime stamps
enum { kDiagTStart = kDiagCount, kDiagTDry, kDiagTLast, kDiagStepsDry, kDiagTDrain, kDiagTEnd,
       kDiagTRefill, kDiagTSub, kDiagDrainN, kDiagTDrain2, kDiagHwId, kDiagWords = 24 };
#ifdef IKHIP_DIAG
constexpr int kDiagWaveMax = 4096;  // = (kFabrikDebugWords - 64) / kDiagWords (24)
#endif

// Phase marks for the instruction census (tools/isa_phases.py): an analysis build
// with -DIKHIP_PHASE_MARKS puts an assembly comment at each phase boundary of the
// iteration kernel; the production build has none.
#ifdef IKHIP_PHASE_MARKS
#define IKHIP_MARK(s) asm volatile(";@phase " s)
#else
#define IKHIP_MARK(s) ((void)0)
#endif

static int env_int(const char *name, int dflt) {
  const char *v = getenv(name);
  return (v && *v) ? atoi(v) : dflt;
}

// The angles step of one finished point (inverse.py:136 __get_angles) and what
// the call reports about it: angles, iterations, joints, the FK round trip
// (cli.py:54-61) and the per-lane sums of the batch stats.
struct LaneAcc {
  unsigned long long sum_it = 0, capped = 0;
  int max_it = 0;
  double fk_max = 0.0, fk_sum = 0.0;
};

// The robot constants' pointer made opaque to the compiler: loads through it are
// issued where they are used (s_load, scalar cache) instead of hoisted out of the
// persistent loop into SGPRs, where the seed and angles steps' ~100 constants
// spilled and the iteration paid for their reloads (v_readlane) every step.
__device__ __forceinline__ RcConst opaque_rc(const RobotConstDev *p) {
  asm volatile("" : "+s"(p));
  return (RcConst)p;
}

__device__ __forceinline__ bool outside_rc(RcConst k, d3 g) {
  const double lim[6] = {k->lim[0], k->lim[1], k->lim[2], k->lim[3], k->lim[4], k->lim[5]};
  return outside(lim, g.x, g.y, g.z);
}

// What the call reports about one finished point once its angles are known:
// angles, iterations, joints, the FK round trip (cli.py:54-61) and the per-lane
// sums of the batch stats.
__device__ __forceinline__ void commit_point(const FabArgs &a, int64_t i, const d3 J[4], d3 g,
                                             int it, int st, const double th[4],
                                             const double cs[4], const double sn[4],
                                             LaneAcc &acc) {
  if (st != IK_OK) record_error(a.S, i, st);
  double2 *o = reinterpret_cast<double2 *>(a.ang + 4 * i);
  o[0] = make_double2(th[0], th[1]);
  o[1] = make_double2(th[2], th[3]);
  if (a.iters) a.iters[i] = it;
  if (a.joints) store_joints(a.joints, i, J);
  acc.sum_it += (unsigned long long)it;
  acc.capped += (it >= a.max_iter) ? 1ull : 0ull;
  acc.max_it = max(acc.max_it, it);
  if (a.fk_err) {
    double e = __builtin_nan("");
    IKHIP_MARK("commit.fk");
    if (st == IK_OK) {
      const RcConst k = opaque_rc(a.rc);
      double jc[16];
#pragma unroll
      for (int e2 = 0; e2 < 16; ++e2) jc[e2] = k->jc[e2];
      // (the angles' own range, forward.py:23-25: always within 2 pi here)
      bool ok = !k->alpha_bad;
#pragma unroll
      for (int e2 = 0; e2 < 4; ++e2) ok = ok && angle_ok(th[e2]);
      e = fk_error_cs(jc, cs, sn, ok, g.x, g.y, g.z);
    }
    IKHIP_MARK("commit.fk_end");
    a.fk_err[i] = e;
    if (e == e) {
      acc.fk_max = fmax(acc.fk_max, e);
      acc.fk_sum += e;
    }
  }
}

// The angles step of one finished point (inverse.py:136 __get_angles): the core
// sequences (get_angles_core); a lane outside their domains is flagged (redo)
// and the whole wave then runs the general get_angles for the flagged lanes in
// a pass of its own, so the general code's registers are never live beside the
// fast path's.  has: the lane holds a point; st: its status so far.
template <class Joints>
__device__ __forceinline__ void angles_step(bool has, Joints joints, int &st, double th[4],
                                            double cs[4], double sn[4]) {
#pragma unroll
  for (int k = 0; k < 4; ++k) th[k] = cs[k] = sn[k] = __builtin_nan("");
  bool redo = false, fast = false;
  if (has && st == IK_OK) {
    d3 J[4];
    joints(J);
    int sf = IK_OK;
    fast = get_angles_core(J, th, sf, cs, sn);
    redo = !fast;
    if (fast) st = sf;
  }
  IKHIP_MARK("angles.general");
  if (__any(redo)) {  // wave-uniform and rare: coincident joints, zero divisors, x = 0 or y = 0
    if (redo) {
      d3 J[4];
      joints(J);
      get_angles(J, th, st);
#pragma unroll
      for (int k = 0; k < 4; ++k) sincos_fk(th[k], &sn[k], &cs[k]);
    }
  }
  // theta_1 (inverse.py:60) last: kept out of the fast pass, whose registers
  // then fit beside the general pass's without spilling
  IKHIP_MARK("angles.atan2");
  if (fast) {
    d3 J[4];
    joints(J);
    th[0] = atan2_fast(J[3].y, J[3].x);
  }
  IKHIP_MARK("angles.end");
}

// ------------------------------------------------------------- simple ----
// One point per lane, no refill: the test variant (IKHIP_FABRIK_VARIANT=0) and
// the solves whose loop runs no iteration at all (max_iter 0, tol >= 1) or whose
// robot FK rejects (its own DH angles out of range: every seed raises).
__global__ __launch_bounds__(256) void fabrik_simple_kernel(FabArgs a) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  LaneAcc acc;
  d3 g = {0.0, 0.0, 0.0}, J[4] = {};
  int st = IK_OK, it = 0;
  if (i < a.n) {
    g = {a.pts[3 * i], a.pts[3 * i + 1], a.pts[3 * i + 2]};
    if (a.check_limits && outside(a.r.lim, g.x, g.y, g.z))
      atomicMin(&a.S->first_oob, (unsigned long long)i);
    st = seed_pose(a.rc, g, J);
    double se = 1.0, ge = 1.0;
    if (st == IK_OK) {
      while (((se > a.tol2) || (ge > a.tol2)) && (a.max_iter > it)) {
        fabrik_step4(J[0], J[1], J[2], J[3], g, a.r.links, se, ge, st);
        ++it;
        if (st != IK_OK) break;
      }
    }
  }
  double th[4], cs[4], sn[4];
  angles_step(i < a.n, [&](d3 *o) {
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = J[k];
  }, st, th, cs, sn);
  if (i < a.n) commit_point(a, i, J, g, it, st, th, cs, sn, acc);
  block_iter_stats_acc(a.S, acc.sum_it, acc.capped, acc.max_it);
  if (a.fk_err) wave_fk_stats(a.S, acc.fk_max, acc.fk_sum);
}

// The whole FABRIK solve of one goal in the general arithmetic (the simple
// kernel's loop: fabrik.py:44-67 from the seed pose, inverse.py:123-133): the
// iteration kernel's retire step re-solves the rare lanes whose core sequences
// left their domain (kStRedo) with it.
__device__ __forceinline__ void solve_general(const FabArgs &a, d3 g, d3 J[4], int &it,
                                              int &st) {
  st = seed_pose(a.rc, g, J);
  it = 0;
  double se = 1.0, ge = 1.0;
  if (st != IK_OK) return;
  while (((se > a.tol2) || (ge > a.tol2)) && (a.max_iter > it)) {
    fabrik_step4(J[0], J[1], J[2], J[3], g, a.r.links, se, ge, st);
    ++it;
    if (st != IK_OK) break;
  }
}
// A lane of the iteration kernel whose core sequences left their domain
// (coincident joints, non-finite or extreme coordinates: sqrt_core / div_core
// would not give the general sequences' bits) stops with this status; the retire
// step re-solves its goal with solve_general (r06: no copy of the pre-step state
// is kept for an in-loop redo).
constexpr int kStRedo = 0x40;

// ---------------------------------------------------------- Work order ----
// The persistent iteration kernel hands points out in queue order.  In point
// order a 100-iteration point can be picked up just before the queue runs dry
// and set the launch length alone (≈ 1.4x the lane-iterations / lanes bound
// at 1M random_dist points).  Handing out the expensive points first removes
// most of that tail.  The cost of a point is predicted from its goal cell --
// distance from the shoulder (the seed's first joint) in 64 bins up to the reach
// of links 1..3, and the sine of the elevation in 16 bins -- by the LARGEST
// iteration count the context recorded in that cell on earlier calls (1 point
// in kOrdSample; the old key decays by 1/8 when new records arrive).  The
// largest, not the mean: what sets the tail is a long point starting late, and
// long points (9 % of random_dist points take >= 80 of 100 iterations) sit in
// cells of every mean.  A list-scheduling simulation of 131k lanes on 1M
// reference iteration counts (tol 1e-3 / 1e-5): point order 1.29x / 1.34x the
// lane-iterations / lanes bound, cells by mean 1.15x / 1.23x, cells by sampled
// max 1.04x / 1.03x, exact longest-first 1.01x.  Unseen cells count as hard.
// Costs map to 16 classes; a counting sort (class-major, hardest first; order
// inside a class is whatever the atomics give) yields the queue -> point
// permutation.  Results do not depend on the order: every point is still
// solved by the same arithmetic on its own.
//
// Launches: classify (cell + class per point from the goal alone, class totals)
// -> scatter (class region starts from the totals, one cursor per class: the
// queue -> point permutation) -> iterate (records 1 point in kOrdSample) -> fold
// (one block: this call's records into the table for the next call).
// 16 at 1M points: classify + scatter 28.8 us against 34.2 for 8 (table reads early)
// and 49.0 for 4 (same box)
#ifndef IKHIP_ORD_PPT
#define IKHIP_ORD_PPT 16
#endif
constexpr int kOrdPPT = IKHIP_ORD_PPT;  // points per thread of the classify / scatter blocks
// (r04: classify and scatter in one launch, the queue in per-class regions of n
// entries: the launch takes 17.8 us against 13.5 + 9.8, but its queue order inside a
// cost class makes the iteration kernel 4 % slower at tol 1e-3 with the same learned
// table; dropped, profiles/r04/ab/fabrik_fused_scatter.txt)
// (r04: spreading a block's class run over its slots -- slot r * 4099 mod run length --
// so that a grab's points come from the whole block: iteration kernel +0.9 %, scatter
// +3 us; profiles/r04/ab/fabrik_order_spread_dropped.txt)

// The shoulder (the seed's first joint, the translation of A_1) is
// (a1 cos t1, a1 sin t1, d1) with t1 the goal's own azimuth: its distance from the
// goal needs no trigonometry.
__device__ __forceinline__ int goal_cell(const RobotDev &r, d3 g) {
  const double rxy = sqrt(g.x * g.x + g.y * g.y) - r.dh[8];
  const double dz = g.z - r.dh[4];
  const double dist = sqrt(rxy * rxy + dz * dz);
  const double reach = r.links[1] + r.links[2] + r.links[3];
  int rb = (int)(dist / reach * kOrdCellsR);
  rb = rb < 0 ? 0 : (rb >= kOrdCellsR ? kOrdCellsR - 1 : rb);
  int eb = dist > 0.0 ? (int)((dz / dist + 1.0) * (0.5 * kOrdCellsE)) : kOrdCellsE / 2;
  eb = eb < 0 ? 0 : (eb >= kOrdCellsE ? kOrdCellsE - 1 : eb);
  return rb * kOrdCellsE + eb;
}

__device__ __forceinline__ int key_class(unsigned int key, int max_iter) {
  // key: 1 + largest recorded iterations, 0 = unseen
  if (key == 0) return kOrdClasses - 1;
  const int k = (int)((long long)(key - 1) * kOrdClasses / (max_iter + 1));
  return k < 0 ? 0 : (k >= kOrdClasses ? kOrdClasses - 1 : k);
}


// Fold ns records into the table: per cell, the largest recorded iteration
// count of the call, or the decayed old key if larger.  One block.
__device__ void order_fold(FabOrderDev *T, unsigned int ns) {
  __shared__ unsigned int lm[kOrdCells];
  const int t = threadIdx.x;
  for (int c = t; c < kOrdCells; c += blockDim.x) lm[c] = 0;
  __syncthreads();
  constexpr int kFoldBatch = 8;  // independent loads in flight
  for (unsigned int k0 = t; k0 < ns; k0 += blockDim.x * kFoldBatch) {
    unsigned int v[kFoldBatch];
#pragma unroll
    for (int j = 0; j < kFoldBatch; ++j) {
      const unsigned int k = k0 + blockDim.x * j;
      v[j] = k < ns ? T->sample[k] : 0xffffffffu;
    }
#pragma unroll
    for (int j = 0; j < kFoldBatch; ++j)
      if (v[j] != 0xffffffffu) atomicMax(&lm[v[j] >> 16], (v[j] & 0xffffu) + 1u);
  }
  __syncthreads();
  for (int c = t; c < kOrdCells; c += blockDim.x) {
    if (lm[c]) {
      const unsigned int old = T->key[c];
      const unsigned int dec = old - (old >> 3);
      T->key[c] = lm[c] > dec ? lm[c] : dec;
    }
  }
}

// 1. classify: the goal's cell and cost class per point (2 bytes), and the
// class totals (one atomic per class and block, into the block's shard: one
// address per class took ~1k same-address atomics per launch at 1M points).
// The cell -> class map of this call is built in LDS first.
__global__ __launch_bounds__(256) void fabrik_classify_kernel(FabArgs a) {
  __shared__ unsigned int cnt[kOrdClasses], unseen;
  __shared__ uint8_t cls[kOrdCells];  // the cell's class, 0xff: unseen (the hardest class)
  const int t = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * (256 * kOrdPPT);
  d3 g[kOrdPPT];
#pragma unroll
  for (int j = 0; j < kOrdPPT; ++j) {  // all loads in flight before the first use
    const int64_t i = b0 + j * 256 + t;
    if (i < a.n) g[j] = {a.pts[3 * i], a.pts[3 * i + 1], a.pts[3 * i + 2]};
  }
  if (t < kOrdClasses) cnt[t] = 0;
  if (t == 0) unseen = 0;
  // the cell -> class map's table reads, in flight with the goals'
  static_assert(kOrdCells % 256 == 0, "whole table rows per thread");
  unsigned int key[kOrdCells / 256];
#pragma unroll
  for (int q = 0; q < kOrdCells / 256; ++q) key[q] = a.ord->key[t + 256 * q];
#pragma unroll
  for (int q = 0; q < kOrdCells / 256; ++q)
    cls[t + 256 * q] = key[q] ? (uint8_t)key_class(key[q], a.max_iter) : (uint8_t)0xff;
  __syncthreads();
  unsigned int nu = 0;
#pragma unroll
  for (int j = 0; j < kOrdPPT; ++j) {
    const int64_t i = b0 + j * 256 + t;
    if (i < a.n) {
      const int cell = goal_cell(a.r, g[j]);
      int k = cls[cell];
      nu += k == 0xff ? 1u : 0u;
      k = k == 0xff ? kOrdClasses - 1 : k;
      a.cell[i] = (uint16_t)(cell | (k << 10));
      atomicAdd(&cnt[k], 1u);
    }
  }
  // (only the prior's gate reads the count: the first call of a context; a
  // wave sum, then one LDS atomic per wave -- one per thread cost 2 us a launch)
  if (a.prior_gate) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) nu += __shfl_xor(nu, off, 64);
    if ((t & 63) == 0 && nu) atomicAdd(&unseen, nu);
  }
  __syncthreads();
  if (t < kOrdClasses && cnt[t]) atomicAdd(&a.S->cls_tot[t][blockIdx.x % kOrdShards], cnt[t]);
  if (t == 0 && unseen) atomicAdd(&a.S->unseen, (unsigned long long)unseen);
}

// The built-in prior's gate: a table no call has taught yet is
// the prior learned on random_dist batches (ik_fabrik_prior.h).  On a batch of
// another distribution many goals fall in cells it has never seen (uniform box:
// the unreachable far cells; a spring trajectory: the far end of its curve), and
// ordering by it measured slower than point order (r06 lease: uniform box +1.5 %,
// spring +2.3 %).  When more than 1 / kPriorUnseenDiv of the batch lands in unseen
// cells, the first call keeps point order; the call's records then teach the
// table as usual.
constexpr unsigned kPriorUnseenDiv = 50;

// 2. scatter: perm[queue position] = point.  The queue is class-major (hardest
// first), then shard: region (c, s) starts after every harder class and every
// lower shard of class c.  Block b covers the points classify's block b counted
// into shard b % kOrdShards, claims its run inside its region with one atomic
// per class and hands the slots out through LDS atomics.
__global__ __launch_bounds__(256) void fabrik_scatter_kernel(FabArgs a) {
  static_assert(kOrdClasses * kOrdShards == 256, "one total per thread");
  // the prior does not describe this batch (see above): every point in the last
  // class, i.e. the order an empty table gives (block shards, point order inside)
  const bool gated = a.prior_gate && a.S->unseen * kPriorUnseenDiv > (unsigned long long)a.n;
  __shared__ unsigned int cnt[kOrdClasses], base[kOrdClasses];
  __shared__ unsigned int tot[kOrdClasses][kOrdShards], ctot[kOrdClasses];
  const int t = threadIdx.x;
  const int sh = blockIdx.x % kOrdShards;
  if (t < kOrdClasses) cnt[t] = 0;
  // the 256 (class, shard) totals, one load per thread, in flight with the cells
  tot[t / kOrdShards][t % kOrdShards] = (&a.S->cls_tot[0][0])[t];
  const int64_t b0 = (int64_t)blockIdx.x * (256 * kOrdPPT);
  uint16_t cl[kOrdPPT];
#pragma unroll
  for (int j = 0; j < kOrdPPT; ++j) {
    const int64_t i = b0 + j * 256 + t;
    cl[j] = i < a.n ? a.cell[i] : (uint16_t)0xffff;
    if (gated && cl[j] != 0xffff) cl[j] |= (uint16_t)((kOrdClasses - 1) << 10);
  }
  __syncthreads();
  if (gated) {  // (uniform) the shards' totals all in the last class
    unsigned int col = 0;
    if (t < kOrdShards)
      for (int c = 0; c < kOrdClasses; ++c) col += tot[c][t];
    __syncthreads();
    if (t < kOrdShards)
      for (int c = 0; c < kOrdClasses; ++c) tot[c][t] = c == kOrdClasses - 1 ? col : 0u;
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < kOrdPPT; ++j)
    if (cl[j] != 0xffff) atomicAdd(&cnt[cl[j] >> 10], 1u);
  if (t < kOrdClasses) {
    unsigned int c = 0;
#pragma unroll
    for (int q = 0; q < kOrdShards; ++q) c += tot[t][q];
    ctot[t] = c;
  }
  __syncthreads();
  if (t < kOrdClasses) {
    // region (t, sh) starts after every harder class and the lower shards of t
    unsigned int start = 0;
    for (int c = kOrdClasses - 1; c > t; --c) start += ctot[c];
    for (int q = 0; q < sh; ++q) start += tot[t][q];
    base[t] = start + (cnt[t] ? atomicAdd(&a.S->cls_cur[t][sh], cnt[t]) : 0u);
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kOrdPPT; ++j) {
    if (cl[j] != 0xffff) {
      const unsigned int pos = atomicAdd(&base[cl[j] >> 10], 1u);
      a.perm[pos] = (int32_t)(b0 + j * 256 + t);
    }
  }
}

// 3. persistent iteration with per-lane refill, seed and angles in batches.
//
// A lane whose point converged is refilled from the wave's batch of prepared
// points: a wave grabs a.chunk queue positions at once and each lane prepares one
// of them -- the goal, the limits check and the seed pose (inverse.py:123-130) --
// into the wave's LDS batch, at full SIMD width; a refill then hands entries to
// the free lanes (LDS reads), with no memory round trip.
// A finished lane parks its final joints in the wave's LDS ring at the next
// refill; when the ring would overflow, and at the end, the whole wave runs the
// angles step on it, one entry per lane (finish_point).  So the seed pose and
// the joints never travel through HBM, and neither step runs at the width of
// the handful of lanes that finish together.
// A parked point is one 144-byte record per slot, written and read as nine
// 16-byte words (ds_write_b128 / ds_read_b128): the joints, the goal (for the FK
// round trip, not read from HBM again) and {index, iterations, status}.  The
// 36-dword slot stride puts 16 lanes' words on 64 distinct banks.
struct RetireRing {
  double2 w[64][9];
};

__device__ __forceinline__ void ring_put(RetireRing &R, int s, const d3 &J0, const d3 &J1,
                                         const d3 &J2, const d3 &J3, const d3 &g, int64_t idx,
                                         int it, int st) {
  double2 *w = R.w[s];
  w[0] = {J0.x, J0.y};
  w[1] = {J0.z, J1.x};
  w[2] = {J1.y, J1.z};
  w[3] = {J2.x, J2.y};
  w[4] = {J2.z, J3.x};
  w[5] = {J3.y, J3.z};
  w[6] = {g.x, g.y};
  w[7] = {g.z, 0.0};
  w[8] = {__longlong_as_double(idx),
          __longlong_as_double((long long)(((uint64_t)(uint32_t)st << 32) | (uint32_t)it))};
}

__device__ __forceinline__ void ring_joints(const RetireRing &R, int s, d3 *J) {
  const double2 *w = R.w[s];
  const double2 w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4], w5 = w[5];
  J[0] = {w0.x, w0.y, w1.x};
  J[1] = {w1.y, w2.x, w2.y};
  J[2] = {w3.x, w3.y, w4.x};
  J[3] = {w4.y, w5.x, w5.y};
}

// The angles step over the ring's first cnt entries (the whole wave calls it).
// ORD: 1 in kOrdSample points records (cell, iterations) for the cost table.
// IKHIP_FAB_PRIO: the angles step and the seed preparation run at a raised wave
// priority.  Two waves share a SIMD and, at equal priority, the older one's VALU
// wins every issue arbitration (MI355X_MICROARCH.md, "Two waves per SIMD"): a
// younger wave's angles step -- long dependent chains, few instructions ready at
// a time -- then gets only the slots its iterating partner leaves and took 10-50 us
// instead of 2.5 for one wave in ten at the end of the launch.  Raised, it issues
// whenever it has an instruction ready and the partner's issue-bound iteration
// fills the rest.
#ifndef IKHIP_FAB_PRIO
#define IKHIP_FAB_PRIO 2
#endif
__device__ __forceinline__ void prio_raise() {
  if (IKHIP_FAB_PRIO) __builtin_amdgcn_s_setprio(IKHIP_FAB_PRIO);
}
__device__ __forceinline__ void prio_drop() {
  if (IKHIP_FAB_PRIO) __builtin_amdgcn_s_setprio(0);
}

template <bool ORD>
__device__ __forceinline__ void ring_flush(const FabArgs &a, RetireRing &R, int cnt, int lane,
                                           LaneAcc &acc) {
  prio_raise();
  IKHIP_MARK("flush.angles");
  __builtin_amdgcn_wave_barrier();
  const bool has = lane < cnt;
  // the joints from the ring each time they are needed (LDS reads are cheap; the
  // barrier keeps the compiler from holding them in registers across the step)
  auto joints = [&](d3 *J) {
    asm volatile("" ::: "memory");
    ring_joints(R, lane, J);
  };
  double2 meta = R.w[lane][8];
  uint64_t itst = (uint64_t)__double_as_longlong(meta.y);
  int st = has ? (int)(itst >> 32) : IK_OK;
  if (__builtin_expect(__any(has && st == kStRedo), 0)) {  // wave-uniform, rare
    if (has && st == kStRedo) {
      const double2 g01 = R.w[lane][6], g2 = R.w[lane][7];
      d3 J[4];
      int it2;
      solve_general(a, {g01.x, g01.y, g2.x}, J, it2, st);
      ring_put(R, lane, J[0], J[1], J[2], J[3], {g01.x, g01.y, g2.x},
               __double_as_longlong(meta.x), it2, st);
      itst = ((uint64_t)(uint32_t)st << 32) | (uint32_t)it2;
    }
    __builtin_amdgcn_wave_barrier();
  }
  double th[4], cs[4], sn[4];
  angles_step(has, joints, st, th, cs, sn);
  IKHIP_MARK("flush.commit");
  if (has) {
    d3 J[4];
    joints(J);
    const int64_t i = __double_as_longlong(meta.x);
    const int it = (int)(uint32_t)itst;
    const double2 g01 = R.w[lane][6], g2 = R.w[lane][7];
    commit_point(a, i, J, {g01.x, g01.y, g2.x}, it, st, th, cs, sn, acc);
    if constexpr (ORD) {
      if (i % kOrdSample == 0 && i / kOrdSample < kOrdMaxSample) {
        const uint32_t lo = (uint32_t)(it < 0xffff ? it : 0xffff);
        a.ord->sample[i / kOrdSample] = ((uint32_t)(a.cell[i] & (kOrdCells - 1)) << 16) | lo;
      }
    }
  }
  IKHIP_MARK("flush.end");
  __builtin_amdgcn_wave_barrier();
  prio_drop();
}


// ORD: the queue is a.perm (work order above), else point order.  CORE: 0
// general sqrt / division, 1 sqrt_core / div_core, 2 the same with the repeated
// distances taken once and the loop condition from the band (fabrik_step4_lazy;
// needs L0 == L1 and L2 == L3).
// Every solve reaching this kernel runs at least one iteration (the host sends
// the others to fabrik_simple_kernel), so the seed's last joint is never needed.
#ifndef IKHIP_FAB_REFILL  // free lanes that trigger a refill (r05: 12 against 6 / 8 / 16 / 20 / 24 / 32; 12 since the dry waves' raised priority; r06 on the 142-VALU loop: 8 +1.5-4 %, 16 even-+1.4 %)
#define IKHIP_FAB_REFILL 12
#endif
#ifndef IKHIP_ITER_WAVES
#define IKHIP_ITER_WAVES 2
#endif
// The refill (park, stage, hand-out) runs at raised wave priority, like the seed and
// angles steps: its dependent chains issue when ready instead of in the partner's
// leftover slots.  r04, same box: iteration kernel -1.7 % at tol 1e-3, -1.3 % at 1e-5
// (rocprof windows, 3 / 2 runs each), -1.0 / -1.3 % per bench step in another lease.
// (r04: taking the seed's carried quotient in the prepare step instead of at the
// hand-out measured slower, profiles/r04/ab/fabrik_refill_prio_prep_carry.txt; r06
// takes it there as part of a bundle that measured faster, DESIGN_HISTORY.md.)
constexpr int kIterWaves = IKHIP_ITER_WAVES;  // waves per SIMD = blocks per CU
template <int REFILL_MIN, bool ORD, int CORE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kIterWaves, kIterWaves))) void
fabrik_iter_kernel(FabArgs a) {
  __shared__ RetireRing rings[4];
  const int lane = threadIdx.x & 63;
  RetireRing &R = rings[threadIdx.x >> 6];
  const unsigned long long lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  // the loop condition's operands held in VGPRs: as wave-uniform values they
  // compete for the SGPRs the nested exec masks need, and the compiler then
  // re-read tol2 from the kernel arguments (s_load + wait) every iteration
  double tol2 = a.tol2;
  int max_iter = a.max_iter;
  asm volatile("" : "+v"(tol2), "+v"(max_iter));
  // the goal error's threshold as an opaque second copy: with one value on both
  // compares, (se > t) || (ge > t) becomes max(se, ge) > t, three v_max_f64 (two
  // canonicalizing) and a compare instead of two compares
  double tol2g = tol2;
  asm volatile("" : "+v"(tol2g));
  double qmax = a.qmax;  // (CORE 2: fabrik_step4_lazy's domain test, also in a VGPR)
  asm volatile("" : "+v"(qmax));
  double L[4] = {a.r.links[0], a.r.links[1], a.r.links[2], a.r.links[3]};

  // prepared points: the batch's entry j in slot j of the wave's LDS batch
  // (wave-uniform count / cursor); a refilled lane reads its entry from there
  struct PrepBatch {  // per entry seven 16-byte words: seed joints 0..2, goal, {meta, cq}
    double2 w[64][7];
  };
  // an entry's meta word: the point index, and (CORE 2, bit 62) whether the point
  // goes straight to the retire step's general re-solve: the seed's carried
  // radicand outside the core domain, or a start / goal past the launch's error
  // band (|J0|_1 + |goal|_1 > band_n1, or not finite) -- the carry itself
  // (reuse_carry) and the band test are taken at full width in the preparation,
  // not per refill (r06)
  constexpr uint64_t kMetaRedo = 1ull << 62;
  __shared__ PrepBatch batches[4];
  PrepBatch &PB = batches[threadIdx.x >> 6];
  int pcount = 0, pptr = 0;
  // the next batch, fetched in stages while the current one is handed out (so
  // that no stage waits for memory): 0 none, 1 queue grab issued (na), 2 its
  // permutation entries loaded (nperm), 3 its goals loaded (ng, ni); -1 the queue is dry
  int nstage = 0, ncount = 0;
  int64_t nbase = 0;
  // the queue head this wave grabs from (its block's, blockIdx % kQueueHeads,
  // until that one runs dry; then the next one its block has not seen dry)
  __shared__ unsigned int dry_heads;  // the heads this block found dry
  if (threadIdx.x == 0) dry_heads = 0;
  __syncthreads();
  int head = (int)(blockIdx.x % kQueueHeads);
  unsigned long long na = 0;
  // (nperm as loaded, 32 bits, widened by the stage that uses it, and the goal as
  // three separate loads: each lands in the register the preparation reads, so no
  // copy waits for a load right after its issue)
  int32_t nperm = 0;
  int64_t ni = 0;
  d3 ng = {0, 0, 0};
  bool dry = false;   // the queue and the batch are exhausted
  int rcnt = 0;       // entries in the retire ring
  LaneAcc acc;

  bool active = false, pending = false;  // solving / finished but not yet parked
  int64_t out = 0;                       // the lane's point index
  // J3: the effector; CORE 2 keeps it only from a fallback iteration (the fast
  // step leaves it to the carry: effector() below)
  d3 J0 = {0, 0, 0}, J1 = J0, J2 = J0, J3 = J0, g = J0;
  bool cont = true;  // the reference's loop condition after the lane's last iteration
  int st = IK_OK;
  // the lane's iteration count as step - max_iter (mod 2^32): the increment's
  // carry is the cap (fabrik.py:57 iteration < max_iter), folded into cont, so
  // the loop's run test needs no compare of its own (r06)
  uint32_t kst = 0;
  auto steps = [&]() -> int { return (int)(kst + (uint32_t)max_iter); };
  double cq = 0.0;  // CORE == 2: the carried quotient and offset
  d3 cd = J0;
  bool cbad = false;  // CORE == 2: the taken entry goes to the retire step's re-solve
  // the effector F3 = get_point_between(F2, goal, L3): CORE 2 from the carry (cq,
  // cd = goal - F2; a lane whose radicands left the core domain is re-solved at
  // retire, kStRedo), else the step's J3
  auto effector = [&]() -> d3 {
    if constexpr (CORE == 2) return {J2.x + (cq * cd.x), J2.y + (cq * cd.y), J2.z + (cq * cd.z)};
    return J3;
  };

#ifdef IKHIP_DIAG
  // counters and stamps live in LDS (lane 0 writes), so that the diagnostic
  // build keeps the production kernel's registers and occupancy
  __shared__ unsigned long long dgs[4][kDiagWords];
  unsigned long long *dg = dgs[threadIdx.x >> 6];
  if (lane < kDiagWords) dg[lane] = 0;
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) dg[kDiagTStart] = __builtin_amdgcn_s_memrealtime();
  // where the wave runs: XCC_ID (hwreg 20) << 32 | HW_ID (hwreg 4: wave 3:0, SIMD 5:4, CU 11:8, SE 14:13)
  if (lane == 0)
    dg[kDiagHwId] = ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |
                    (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4);
#define IKHIP_DG(k, v) \
  do {                 \
    if (lane == 0) dg[k] += (v); \
  } while (0)
#define IKHIP_DT(k) \
  do {              \
    if (lane == 0) dg[k] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define IKHIP_DT_ACC(k, k0) \
  do {                      \
    if (lane == 0) dg[k] += __builtin_amdgcn_s_memrealtime() - dg[k0]; \
  } while (0)
#else
#define IKHIP_DG(k, v) ((void)0)
#define IKHIP_DT(k) ((void)0)
#define IKHIP_DT_ACC(k, k0) ((void)0)
#endif
  while (true) {
    const unsigned long long freem = __ballot(!active);
    const int nfree = __popcll(freem);
    if (dry && nfree == 64) break;
    IKHIP_DG(kDiagLoops, 1);
    if (!dry && (nfree >= REFILL_MIN || nfree == 64)) {
      prio_raise();
      IKHIP_MARK("refill.park");
      IKHIP_DG(kDiagRefills, 1);
      IKHIP_DT(kDiagTRefill);  // refill time, less the flushes and preparations in it
      IKHIP_DT(kDiagTSub);
      // park the lanes that finished since the last refill
      const unsigned long long pm = __ballot(pending);
      const int np = __popcll(pm);
      if (np) {
        if (rcnt + np > 64) {
          IKHIP_DG(kDiagFlushes, 1);
          IKHIP_DT_ACC(kDiagParkTicks, kDiagTSub);  // (the park's time excludes the flush)
          IKHIP_DT(kDiagTEnd);  // (scratch slot: the flush's start)
          ring_flush<ORD>(a, R, rcnt, lane, acc);
          prio_raise();  // (the flush dropped it)
          IKHIP_DT_ACC(kDiagFlushTicks, kDiagTEnd);
          IKHIP_DT_ACC(kDiagTRefill, kDiagTEnd);  // (not refill time)
          IKHIP_DT(kDiagTSub);
          rcnt = 0;
        }
        if (pending)
          ring_put(R, rcnt + __popcll(pm & lt_mask), J0, J1, J2, effector(), g, out, steps(), st);
        pending = false;
        rcnt += np;
      }
      IKHIP_DT_ACC(kDiagParkTicks, kDiagTSub);
      IKHIP_DT(kDiagTSub);
      IKHIP_MARK("refill.handout");
      // the next batch's three stages (called below: one per refill ahead of time,
      // or back to back just before a preparation)
      auto stage1 = [&]() {
        if (lane == 0) na = atomicAdd(&a.S->heads[head][0], 1ull);
        nstage = 1;
      };
      auto stage2 = [&]() {
        // the grab's chunk: head h's k-th is the queue's (k * kQueueHeads + h)-th
        // (lane 0's value read into SGPRs: a shuffle would leave the batch's count,
        // cursor and the hand-out divergent in the compiler's eyes)
        const uint64_t na0 =
            ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(na >> 32), 0) << 32) |
            (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)na, 0);
        nbase = ((int64_t)na0 * kQueueHeads + head) * a.chunk;
        if (nbase >= a.n) {  // this head is dry: on to one the block has not seen dry
          if (lane == 0) atomicOr(&dry_heads, 1u << head);
          const unsigned m =
              __builtin_amdgcn_readfirstlane(__hip_atomic_load(&dry_heads, __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_WORKGROUP)) |
              (1u << head);
          if (m == (1u << kQueueHeads) - 1) {
            nstage = -1;
            return;
          }
          int h = head;
          do h = (h + 1) % kQueueHeads;
          while ((m >> h) & 1u);
          head = h;
          nstage = 0;
          return;
        }
        ncount = (int)min((int64_t)a.chunk, a.n - nbase);
        if (lane < ncount) {
          if (ORD) nperm = a.perm[nbase + lane];
        }
        nstage = 2;
      };
      auto stage3 = [&]() {
        if (lane < ncount) {
          const int64_t ip = ORD ? (int64_t)nperm : nbase + lane;
          int64_t iy = 3 * ip + 1, iz = 3 * ip + 2;
          asm volatile("" : "+v"(iy), "+v"(iz));  // (three loads, not a merged x4 + x2)
          ng = {a.pts[3 * ip], a.pts[iy], a.pts[iz]};
          ni = ip;
        }
        nstage = 3;
      };
      // hand prepared points to the free lanes: first what the batch holds, then, if
      // the batch runs out, from the next one.  Straight-line code with one call
      // site per stage: each stage's loads land in the registers the next stage
      // reads, with no merge copies that would wait for them right after issue.
      const bool wasfree = !active;
      const int rank = __popcll(freem & lt_mask);
      const int avail = pcount - pptr;
      const int take1 = min(nfree, avail);
      const bool prep = nfree > avail;  // the batch runs out: prepare the next one
      bool mine = wasfree && rank < take1;
      auto take_entry = [&](int src) {
        const double2 *w = PB.w[src];
        const double2 w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4], w5 = w[5];
        J0 = {w0.x, w0.y, w1.x};
        J1 = {w1.y, w2.x, w2.y};
        J2 = {w3.x, w3.y, w4.x};
        g = {w4.y, w5.x, w5.y};
        const double2 w6 = w[6];
        const uint64_t meta = (uint64_t)__double_as_longlong(w6.x);
        out = (int64_t)(meta & (kMetaRedo - 1));
        if constexpr (CORE == 2) {
          // the seed's carry (reuse_carry): cd = goal - J2, exact, as it computes it
          cq = w6.y;
          cd = {g.x - J2.x, g.y - J2.y, g.z - J2.z};
          cbad = (meta & kMetaRedo) != 0;
        }
      };
      // (read before a preparation overwrites the batch)
      if (mine) take_entry(pptr + rank);
      pptr += take1;
      // the next batch's stages: while the batch is down to its last 24 / 16 / 8
      // entries, one per refill (a stage consumes what the one before loaded, so the
      // loads are long done); before a preparation, the stages still missing.  No
      // loop: when stage 2 finds its head dry (back to stage 1 on another), the free
      // lanes stay free, the inner loop returns at once and the next refill goes on.
      // (diagnostic build: before a preparation the stages count as preparation time,
      // as the r04 / r05 breakdowns did, so that staging is the lookahead's cost)
      IKHIP_MARK("refill.stages");
      if (prep) IKHIP_DT(kDiagTDrain);  // (scratch slot: the preparation's start)
      bool more = true;
      if (nstage == 0 && (prep || avail <= 24)) { stage1(); more = prep; }
      if (more && nstage == 1 && (prep || avail <= 16)) { stage2(); more = prep; }
      if (more && nstage == 2 && (prep || avail <= 8)) stage3();
      if (!prep) IKHIP_DT_ACC(kDiagStageTicks, kDiagTSub);
      if (prep && nstage == 3) {
        IKHIP_DG(kDiagGrabs, 1);
        // prepare: limits check and seed pose of the batch, one entry per lane
        pcount = ncount;
        nstage = 0;
        prio_raise();
        IKHIP_MARK("refill.prepare");
        if (lane < pcount) {
          const RcConst k = opaque_rc(a.rc);
          if (a.check_limits && outside_rc(k, ng))
            atomicMin(&a.S->first_oob, (unsigned long long)ni);
          d3 Js[4];
          (void)seed_pose((const RobotConstDev *)k, ng, Js);
          uint64_t meta = (uint64_t)ni;
          double pcq = 0.0;
          if constexpr (CORE == 2) {
            d3 pcd;
            uint32_t pcdom;
            reuse_carry(Js[2], ng, L[3], pcq, pcd, pcdom);
            const bool pbok = fabs(Js[0].x) + fabs(Js[0].y) + fabs(Js[0].z) + fabs(ng.x) +
                                  fabs(ng.y) + fabs(ng.z) <=
                              a.band_n1;
            meta |= (pcdom < kCoreDom && pbok) ? 0ull : kMetaRedo;
          }
          double2 *w = PB.w[lane];
          w[0] = {Js[0].x, Js[0].y};
          w[1] = {Js[0].z, Js[1].x};
          w[2] = {Js[1].y, Js[1].z};
          w[3] = {Js[2].x, Js[2].y};
          w[4] = {Js[2].z, ng.x};
          w[5] = {ng.y, ng.z};
          w[6] = {__longlong_as_double((long long)meta), pcq};
        }
#ifdef IKHIP_DIAG
        // (the seed's loads are consumed before the stamp)
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the batch's LDS writes landed
#endif
        IKHIP_DT_ACC(kDiagPrepTicks, kDiagTDrain);
        IKHIP_DT_ACC(kDiagTRefill, kDiagTDrain);  // (not refill time)
        // the rest of the free lanes from the new batch (a short last chunk may leave
        // some free until the next refill)
        IKHIP_MARK("refill.handout2");
        const int take2 = min(nfree - take1, pcount);
        const bool mine2 = wasfree && rank >= take1 && rank < take1 + take2;
        __builtin_amdgcn_wave_barrier();  // the batch's LDS writes before the reads
        if (mine2) take_entry(rank - take1);
        pptr = take2;
        mine = mine || mine2;
      }
      IKHIP_MARK("refill.start");
      if (mine) {
        st = IK_OK;
        cont = true;  // the loop's initial errors of 1.0 (fabrik.py:53-54) exceed tol
        kst = 0u - (uint32_t)max_iter;
        active = true;
        // (CORE 2: the carry came with the entry, take_entry; an entry the
        // preparation sent to the re-solve -- its carry outside the core domain,
        // or its goal past the band -- stops before its first iteration, for the
        // retire step's solve_general)
        if constexpr (CORE == 2) {
          if (cbad) {
            st = kStRedo;
            cont = false;
          }
        }
      }
      IKHIP_MARK("refill.end");
      dry = nstage < 0 && pptr >= pcount;
      IKHIP_DT_ACC(kDiagRefillTicks, kDiagTRefill);
      // a dry wave's last lanes are the launch's tail: they iterate at priority 1,
      // ahead of a SIMD partner that still hands out its batch (r05, three boxes:
      // iteration kernel -0.7..-1.0 % at tol 1e-3, -0.8..-1.8 % at 1e-5; priority 3,
      // above the partner's refill and angles steps, and refilling at 4 / 8 free
      // lanes once the queue is dry both measured slower: profiles/r05/lease_dry/)
      if (dry) __builtin_amdgcn_s_setprio(1);
      else prio_drop();
    }
    // iterate until a refill is due (REFILL_MIN lanes free) or, once the queue is
    // dry, until every lane has stopped: the refill's scalar state stays out of
    // this loop, so its SGPRs are not reloaded from their spill lanes per iteration
    IKHIP_MARK("loop");
    const int need = __builtin_amdgcn_readfirstlane(dry ? 64 : REFILL_MIN);  // (an SGPR)
    // (r06: the loop's control as uint64 wave masks instead of these lane bools
    // measured worse in the ISA: the masks, updated inside the divergent step,
    // went to VGPRs and took ~25 VALU per iteration; the bools live in SGPR lane
    // masks already, and only ballot(!run) costs a v_cndmask + v_cmp -- also
    // written as exec & ~ballot(run), and with the band flag as a wave mask taken
    // at the refill, which put the wave's exec in VGPRs)
    while (true) {
#ifdef IKHIP_DIAG
    {
      const unsigned long long sm =
          __ballot(active && st == IK_OK && cont);
      IKHIP_DG(kDiagSteps, sm ? 1 : 0);
      IKHIP_DG(kDiagLaneSteps, __popcll(sm));
      if (dry) {  // the queue and the wave's batch are exhausted
        if (lane == 0 && dg[kDiagTDry] == 0) dg[kDiagTDry] = __builtin_amdgcn_s_memrealtime();
        IKHIP_DG(kDiagStepsDry, sm ? 1 : 0);
      }
      if (sm) IKHIP_DT(kDiagTLast);
    }
#endif
    {
      // one divergent region per iteration: lanes that stop here become pending
      // (parked at the next refill) without a branch of their own.  (No st test:
      // every step that sets an error status also clears cont -- the general
      // step's errors give NaN errors, whose comparisons are false, and the core
      // step's kStRedo clears it explicitly.)
      const bool run = active && cont;  // (cont holds the cap: kst)
      pending = pending || (active && !run);
      active = run;
      if (__popcll(__builtin_amdgcn_ballot_w64(!run)) >= need) break;  // (a bool: no VGPR round trip)
      if (run) {
        if constexpr (CORE == 2) {
          // in place: a lane whose radicands leave the core domain stops with
          // kStRedo and the retire step re-solves it in the general arithmetic
          // (solve_general), so no copy of the pre-step state is kept (r06: the
          // wave-wide in-loop redo needed one, 7 register moves per iteration)
          if (!fabrik_step4_lazy(J0, J1, J2, g, L, a.band, tol2, qmax, cont, cq, cd)) {
            st = kStRedo;
            cont = false;
          }
        } else if constexpr (CORE == 1) {
          // wave-uniform fallback: when any lane's radicand leaves sqrt_core's
          // domain (coincident joints, non-finite input) the wave redoes the
          // iteration with the general sqrt / division (and their errors)
          uint32_t dom = 0;
          d3 n1 = J1, n2 = J2, n3 = J3;
          double se, ge;
          fabrik_step4_core(J0, n1, n2, n3, g, L, se, ge, dom);
          if (__all(dom < kCoreDom)) {
            J1 = n1; J2 = n2; J3 = n3;
          } else {
            IKHIP_DG(kDiagFallbacks, 1);
            fabrik_step4(J0, J1, J2, J3, g, L, se, ge, st);
          }
          cont = (se > tol2) || (ge > tol2g);
        } else {
          double se, ge;
          fabrik_step4(J0, J1, J2, J3, g, L, se, ge, st);
          cont = (se > tol2) || (ge > tol2g);
        }
        if (__builtin_add_overflow(kst, 1u, &kst)) cont = false;  // max_iter reached
      }
    }
    }
  }
  // drain: park the last finished lanes, then the angles step on the ring
  IKHIP_MARK("drain");
  IKHIP_DT(kDiagTDrain);
  {
    const unsigned long long pm = __ballot(pending);
    const int np = __popcll(pm);
    IKHIP_DG(kDiagDrainN, rcnt + np);
    if (rcnt + np > 64) {
      ring_flush<ORD>(a, R, rcnt, lane, acc);
      rcnt = 0;
    }
    IKHIP_DT(kDiagTDrain2);
    if (pending)
      ring_put(R, rcnt + __popcll(pm & lt_mask), J0, J1, J2, effector(), g, out, steps(), st);
    rcnt += np;
    IKHIP_DG(kDiagFlushes, 1);
    IKHIP_DT(kDiagTEnd);
    ring_flush<ORD>(a, R, rcnt, lane, acc);
    IKHIP_DT_ACC(kDiagFlushTicks, kDiagTEnd);
  }
#ifdef IKHIP_DIAG
  IKHIP_DT(kDiagTEnd);
  IKHIP_DG(kDiagWaves, 1);
  __builtin_amdgcn_wave_barrier();
  if (a.dbg) {
    const int w = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    if (lane < kDiagCount) atomicAdd(&a.dbg[lane], dg[lane]);
    if (w < kDiagWaveMax && lane < kDiagWords) a.dbg[64 + kDiagWords * w + lane] = dg[lane];
  }
#endif
#undef IKHIP_DG
#undef IKHIP_DT
#undef IKHIP_DT_ACC
  block_iter_stats_acc(a.S, acc.sum_it, acc.capped, acc.max_it);
  if (a.fk_err) wave_fk_stats(a.S, acc.fk_max, acc.fk_sum);
  // (ORD: the cost table is folded by fabrik_fold_kernel, launched next on the
  // same stream: the kernel boundary publishes the sample stores, so no block
  // fences them here -- a release per wave, and later one per block, wrote the
  // XCD's L2 back while the last waves were still draining, r03)
}

// The cost-table fold after an ordered solve (one block): this call's samples
// (the retire steps' stores, published by the kernel boundary) into the table
// the next call's classify reads.
__global__ __launch_bounds__(256) void fabrik_fold_kernel(FabArgs a) {
  const int64_t ns = (a.n + kOrdSample - 1) / kOrdSample;
  order_fold(a.ord, (unsigned int)(ns < kOrdMaxSample ? ns : kOrdMaxSample));
}

static size_t up256(size_t b) { return (b + 255) & ~(size_t)255; }

size_t fabrik_scratch_bytes(int64_t n) {
  // work order: perm n int32, cell n uint16
  return up256((size_t)n * 4) + up256((size_t)n * 2) + 1024;
}

// CUs of the current device, cached per device index (relaxed atomics: every
// writer stores the same value)
static int num_cus() {
  static std::atomic<int> cache[64];
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::atomic<int> *slot = (dev >= 0 && dev < 64) ? &cache[dev] : nullptr;
  int v = slot ? slot->load(std::memory_order_relaxed) : 0;
  if (v <= 0) {
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        v <= 0)
      v = 256;
    if (slot) slot->store(v, std::memory_order_relaxed);
  }
  return v;
}

template <int REFILL_MIN, bool ORD>
static void launch_iter(int core, unsigned grid, hipStream_t stream, const FabArgs &a) {
  if (core == 2)
    IK_LAUNCH((fabrik_iter_kernel<REFILL_MIN, ORD, 2>), dim3(grid), dim3(256), 0,
                       stream, a);
  else if (core == 1)
    IK_LAUNCH((fabrik_iter_kernel<REFILL_MIN, ORD, 1>), dim3(grid), dim3(256), 0,
                       stream, a);
  else
    IK_LAUNCH((fabrik_iter_kernel<REFILL_MIN, ORD, 0>), dim3(grid), dim3(256), 0,
                       stream, a);
}

void launch_fabrik_ikine(const RobotDev &r, const double *pts, int64_t n, double tol,
                         int max_iter, double *ang, int32_t *iters, double *joints,
                         double *fk_err, bool check_limits, void *scratch, DevStats *S,
                         hipStream_t stream, int variant, int core_req, FabOrderDev *ord,
                         const RobotConstDev *rc, unsigned long long *dbg, int bpc_req,
                         bool prior) {
  if (n <= 0) return;
  FabArgs a;
  a.r = r;
  a.rc = rc;
  a.dbg = dbg;
  a.pts = pts;
  a.n = n;
  a.tol = tol;
  a.tol2 = tol_threshold(tol);
  // the band covers goals well past the reach: 64 (1 + |d1| + |a1| + sum L)
  {
    const double sum_l = std::fabs(r.links[0]) + std::fabs(r.links[1]) + std::fabs(r.links[2]) +
                         std::fabs(r.links[3]);
    a.band_n1 = 64.0 * (1.0 + std::fabs(r.dh[4]) + std::fabs(r.dh[8]) + sum_l);
    if (!std::isfinite(a.band_n1)) a.band_n1 = -1.0;  // (no lane: every comparison exact)
    a.band = fabrik_band(a.tol2, a.band_n1, sum_l);
    a.qmax = fabrik_qmax(r.links);
  }
  a.max_iter = max_iter;
  a.check_limits = check_limits ? 1 : 0;
  a.ang = ang;
  a.iters = iters;
  a.joints = joints;
  a.fk_err = fk_err;
  a.S = S;
  a.chunk = 64;
  a.perm = nullptr;
  a.cell = nullptr;
  a.ord = ord;
  a.prior_gate = prior ? 1 : 0;
  // the seed's own angles (robot_const_kernel's check, forward.py:23-25)
  bool robot_ok = true;
  for (int k = 1; k < 4; ++k)
    if (r.dh[k] < -2 * kPi || r.dh[k] > 2 * kPi) robot_ok = false;
  for (int k = 0; k < 4; ++k)
    if (r.dh[12 + k] < -2 * kPi || r.dh[12 + k] > 2 * kPi) robot_ok = false;
  const unsigned grid = (unsigned)((n + 255) / 256);
  // no iteration at all when the loop's initial errors of 1.0 already pass
  if (variant == 0 || max_iter <= 0 || !(1.0 > a.tol2) || !robot_ok) {
    kt_begin("fabrik_simple_kernel", stream);
    IK_LAUNCH(fabrik_simple_kernel, dim3(grid), dim3(256), 0, stream, a);
    kt_end(stream);
    return;
  }
  static const int order_on = env_int("IKHIP_FABRIK_ORDER", 1);
  const bool ordered = ord && order_on && n < (int64_t)1 << 31;
  if (ordered) {
    char *p = static_cast<char *>(scratch);
    const unsigned ogrid = (unsigned)((n + 256 * kOrdPPT - 1) / (256 * kOrdPPT));
    a.perm = reinterpret_cast<int32_t *>(p);
    p += up256((size_t)n * 4);
    a.cell = reinterpret_cast<uint16_t *>(p);
    kt_begin("fabrik_classify_kernel", stream);
    IK_LAUNCH(fabrik_classify_kernel, dim3(ogrid), dim3(256), 0, stream, a);
    kt_end(stream);
    kt_begin("fabrik_scatter_kernel", stream);
    IK_LAUNCH(fabrik_scatter_kernel, dim3(ogrid), dim3(256), 0, stream, a);
    kt_end(stream);
  }
  // persistent grid: blocks_per_cu 256-thread blocks per CU (= waves per SIMD)
  // measured on MI355X (tools/sweep_fabrik.py): at 1M points 2 blocks/CU with
  // 64-point grabs beats 4 and 8 by 10-30 % (more lanes = fewer points per lane
  // = a longer divergent tail); 2 and 3 are within noise at 1-1.25M points, and
  // from 4M points on 3 wins by ~5 % at every tolerance (the tail matters less
  // than the latency a third wave per SIMD hides), and so it does at 1M points
  // with tol 1e-5 (56 iterations per point against 33 at 1e-3).
  // (4M / 10M points at tol 1e-3: 4 per CU is 2 % ahead of 3; at 1e-5 they are even)
  // bpc_req: the context's IKHIP_FABRIK_BPC (0 = this rule)
  // The fused kernel keeps the batch of prepared points and the angles step's
  // temporaries beside the loop state: ~250 VGPRs, two waves per SIMD at most.
  const int bpc = bpc_req > 0 ? (bpc_req < kIterWaves ? bpc_req : kIterWaves) : kIterWaves;
  static const int chunk = env_int("IKHIP_FABRIK_CHUNK", 64);
  a.chunk = (chunk > 0 && chunk <= 64) ? chunk : 64;
  unsigned pgrid = (unsigned)num_cus() * (unsigned)(bpc > 0 ? bpc : 8);
  int64_t waves_needed = (n + 63) / 64;
  if ((int64_t)pgrid * 4 > waves_needed)
    pgrid = (unsigned)((waves_needed + 3) / 4 > 0 ? (waves_needed + 3) / 4 : 1);
  // the iteration through sqrt_core / div_core (same bits, fewer instructions)
  // unless the link lengths are outside div_core's domain, and with the repeated
  // distances taken once (core 2) when L0 == L1 and L2 == L3.  core_req (context's
  // IKHIP_FABRIK_CORE) 0 forces the general sqrt / division, 1 the core sequences
  // without the reuse.
  const double *Lk = a.r.links;
  int core = links_core_ok(Lk, 4) ? core_req : 0;
  if (core == 2 && !(Lk[0] == Lk[1] && Lk[2] == Lk[3])) core = 1;
#ifdef IKHIP_DIAG
  if (a.dbg) (void)hipMemsetAsync(a.dbg, 0, kFabrikDebugWords * 8, stream);
#endif
  kt_begin("fabrik_iter_kernel", stream);
  if (variant == 2) {
    if (ordered) launch_iter<1, true>(core, pgrid, stream, a);
    else launch_iter<1, false>(core, pgrid, stream, a);
  } else {
    if (ordered) launch_iter<IKHIP_FAB_REFILL, true>(core, pgrid, stream, a);
    else launch_iter<IKHIP_FAB_REFILL, false>(core, pgrid, stream, a);
  }
  kt_end(stream);
  if (ordered) {
    kt_begin("fabrik_fold_kernel", stream);
    IK_LAUNCH(fabrik_fold_kernel, dim3(1), dim3(256), 0, stream, a);
    kt_end(stream);
  }
}

// ------------------------------------------------------ Fabrik.calculate ----
template <int NJ>
__global__ __launch_bounds__(256) void fabrik_calc_kernel(const double *dists_in,
                                                          const double *init, int shared,
                                                          const double *goals, int64_t n,
                                                          double tol2, int max_iter,
                                                          double *joints, int32_t *iters,
                                                          DevStats *S) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool valid = i < n;
  int it = 0;
  if (valid) {
    double L[NJ];
#pragma unroll
    for (int k = 0; k < NJ; ++k) L[k] = dists_in[k];
    const double *ip = shared ? init : init + (size_t)i * NJ * 3;
    d3 cur[NJ], B[NJ];
#pragma unroll
    for (int k = 0; k < NJ; ++k) cur[k] = {ip[3 * k], ip[3 * k + 1], ip[3 * k + 2]};
    d3 g = {goals[3 * i], goals[3 * i + 1], goals[3 * i + 2]};
    const d3 start = cur[0];
    double se = 1.0, ge = 1.0;
    int st = IK_OK;
    while (((se > tol2) || (ge > tol2)) && (max_iter > it)) {  // squared errors
      B[NJ - 1] = g;
#pragma unroll
      for (int k = NJ - 2; k >= 0; --k) B[k] = point_between(B[k + 1], cur[k], L[k], st);
      se = dist3_sq(B[0], start);
      cur[0] = start;
#pragma unroll
      for (int k = 1; k < NJ; ++k) cur[k] = point_between(cur[k - 1], B[k], L[k], st);
      ge = dist3_sq(cur[NJ - 1], g);
      ++it;
      if (st != IK_OK) break;
    }
    if (st != IK_OK) record_error(S, i, st);
    double *o = joints + (size_t)i * NJ * 3;
#pragma unroll
    for (int k = 0; k < NJ; ++k) {
      o[3 * k] = cur[k].x;
      o[3 * k + 1] = cur[k].y;
      o[3 * k + 2] = cur[k].z;
    }
    if (iters) iters[i] = it;
  }
  block_iter_stats(S, valid, it, max_iter);
}

// Any chain length (1 joint up, fabrik.py:44-67 takes any len(init) ==
// len(dists)): the chain lives in the lane's output row instead of registers.
// The backward pass writes B[k] over cur[k] (cur[k] is read only to form B[k]),
// and the forward pass writes the new cur[k] over B[k] (read only to form it),
// so one nj x 3 row per point holds both passes.  Same point_between calls in the
// same order as the unrolled kernel: the same bits.
__global__ __launch_bounds__(256) void fabrik_calc_any_kernel(int nj, const double *dists,
                                                              const double *init, int shared,
                                                              const double *goals, int64_t n,
                                                              double tol2, int max_iter,
                                                              double *joints, int32_t *iters,
                                                              DevStats *S) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = i < n;
  int it = 0;
  if (valid) {
    const double *ip = shared ? init : init + (size_t)i * nj * 3;
    double *row = joints + (size_t)i * nj * 3;
    auto ld = [&](const double *p, int k) -> d3 { return {p[3 * k], p[3 * k + 1], p[3 * k + 2]}; };
    auto stj = [&](int k, d3 v) {
      row[3 * k] = v.x;
      row[3 * k + 1] = v.y;
      row[3 * k + 2] = v.z;
    };
    for (int k = 0; k < nj; ++k) stj(k, ld(ip, k));
    const d3 g = {goals[3 * i], goals[3 * i + 1], goals[3 * i + 2]};
    const d3 start = ld(ip, 0);
    double se = 1.0, ge = 1.0;
    int st = IK_OK;
    while (((se > tol2) || (ge > tol2)) && (max_iter > it)) {  // squared errors
      d3 b = g;  // B[nj - 1]
      stj(nj - 1, b);
      for (int k = nj - 2; k >= 0; --k) {
        b = point_between(b, ld(row, k), dists[k], st);
        stj(k, b);
      }
      se = dist3_sq(b, start);  // B[0]
      d3 f = start;
      stj(0, f);
      for (int k = 1; k < nj; ++k) {
        f = point_between(f, ld(row, k), dists[k], st);
        stj(k, f);
      }
      ge = dist3_sq(f, g);
      ++it;
      if (st != IK_OK) break;
    }
    if (st != IK_OK) record_error(S, i, st);
    if (iters) iters[i] = it;
  }
  block_iter_stats(S, valid, it, max_iter);
}

void launch_fabrik_calc(int nj, const double *dists, const double *init, bool init_shared,
                        const double *goals, int64_t n, double tol, int max_iter,
                        double *joints, int32_t *iters, DevStats *S, hipStream_t st) {
  if (n <= 0) return;
  unsigned grid = (unsigned)((n + 255) / 256);
  int sh = init_shared ? 1 : 0;
  const double tol2 = tol_threshold(tol);
#define IK_CALC_CASE(K)                                                                      \
  case K:                                                                                    \
    IK_LAUNCH(fabrik_calc_kernel<K>, dim3(grid), dim3(256), 0, st, dists, init, sh, \
                       goals, n, tol2, max_iter, joints, iters, S);                          \
    break;
  kt_begin("fabrik_calc_kernel", st);
  switch (nj) {
    IK_CALC_CASE(2)
    IK_CALC_CASE(3)
    IK_CALC_CASE(4)
    IK_CALC_CASE(5)
    IK_CALC_CASE(6)
    IK_CALC_CASE(7)
    IK_CALC_CASE(8)
    default:
      IK_LAUNCH(fabrik_calc_any_kernel, dim3(grid), dim3(256), 0, st, nj, dists, init,
                         sh, goals, n, tol2, max_iter, joints, iters, S);
      break;
  }
  kt_end(st);
#undef IK_CALC_CASE
}

}  // namespace ikhip
