/*
 * ik_oracle.c -- CPU restatement of the reference FABRIK / FK / angle path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP
 * kernels in inversekinematicsann_amd/csrc.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load libikoracle.so.  The product path
 * never links or calls it.
 *
 * It restates, scalar and in float64 with the reference's exact operation
 * order, the functions of lstar93/InverseKinematicsANN listed below.  It is
 * built with -ffp-contract=off and -fno-builtin so that
 *   - no multiply-add is fused (CPython never fuses), and
 *   - pow(x, 2) calls glibc pow exactly as CPython's float.__pow__ does
 *     (glibc pow is not always bit-identical to x*x).
 * With the same glibc it reproduces the reference bit for bit; the pinning is
 * done by tests/test_oracle_golden.py against the tests/golden fixtures, which were
 * produced by importing the reference itself (tests/golden/make_golden.py).
 *
 * Reference functions restated (file:line in /root/reference):
 *   dist()            kinematics/point.py:25-29   get_distance_between
 *   point_between()   kinematics/point.py:32-45   get_point_between
 *   backward/forward  kinematics/fabrik.py:19-42
 *   fabrik_calc()     kinematics/fabrik.py:44-67  Fabrik.calculate
 *   fk_chain()        kinematics/forward.py:21-94 ForwardKinematics.fkine
 *   get_angles()      kinematics/inverse.py:54-112
 *   fabrik_ikine()    kinematics/inverse.py:115-139
 *   check_limits()    kinematics/inverse.py:26-35
 *   round_nd()        CPython round(x, 8) (Objects/floatobject.c double_round)
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define IKO_PI 3.141592653589793 /* math.pi */
#define IKO_OK 0
#define IKO_E_OUT_OF_REACH 1
#define IKO_E_DOMAIN 2
#define IKO_E_ZERODIV 3
#define IKO_E_ANGLE_RANGE 4

/* pow through a volatile exponent: keeps gcc from folding pow(x,2) -> x*x. */
static volatile double k_two = 2.0;
static double sq(double v) { return pow(v, k_two); }

typedef struct { double x, y, z; } pt3;

/* point.py:25-29: sqrt(pow(dx,2) + pow(dy,2) + pow(dz,2)), summed left to right */
static double dist(pt3 a, pt3 b) {
  return sqrt(sq(a.x - b.x) + sq(a.y - b.y) + sq(a.z - b.z));
}

/* point.py:32-45: s_c + ((d / |s-e|) * (e_c - s_c)); |s-e| == 0 -> ZeroDivisionError */
static pt3 point_between(pt3 s, pt3 e, double d, int *st) {
  pt3 r;
  double n = dist(s, e);
  if (n == 0.0) {
    if (*st == IKO_OK) *st = IKO_E_ZERODIV;
    r.x = r.y = r.z = NAN;
    return r;
  }
  r.x = s.x + ((d / n) * (e.x - s.x));
  r.y = s.y + ((d / n) * (e.y - s.y));
  r.z = s.z + ((d / n) * (e.z - s.z));
  return r;
}

/*
 * CPython round(v, nd) for nd >= 0: the exact binary value of v rounded
 * half-even to nd decimals, then the nearest double of that decimal.
 * v*10^nd = p + e exactly (fma residual); p decides unless it sits exactly on
 * a half-integer, where the sign of e breaks the tie.
 */
double iko_round_nd(double v, int nd) {
  if (!isfinite(v)) return v;
  double s = 1.0;
  for (int i = 0; i < nd; ++i) s *= 10.0;
  double p = v * s;
  if (!isfinite(p)) return v;
  double e = fma(v, s, -p);
  double fl = floor(p);
  double k;
  if (p - fl == 0.5) {
    if (e > 0) k = fl + 1.0;
    else if (e < 0) k = fl;
    else k = nearbyint(p); /* exact tie: half-even */
  } else {
    k = nearbyint(p);
  }
  double r = k / s;
  if (r == 0.0) r = copysign(0.0, v);
  return r;
}

/* Python math.acos: ValueError outside [-1, 1]; nan passes through. */
static double py_acos(double v, int *st) {
  if (v > 1.0 || v < -1.0) {
    if (*st == IKO_OK) *st = IKO_E_DOMAIN;
    return NAN;
  }
  return acos(v);
}

static double py_div(double a, double b, int *st) {
  if (b == 0.0) {
    if (*st == IKO_OK) *st = IKO_E_ZERODIV;
    return NAN;
  }
  return a / b;
}

/* ---------------------------------------------------------------- FK ---- */
/* forward.py:21-70 builds A_i = Rz(t)*Tz(d)*Tx(a)*Rx(al) with numpy 4x4 dots;
 * every entry of A_i is a single product, so its value does not depend on the
 * summation order.  The chain M_{i+1} = M_i * A_{i+1} (forward.py:85-92) does:
 * numpy hands it to OpenBLAS dgemm, whose kernels accumulate in k order with
 * fused multiply-add starting from 0.  mm4() restates that (FMA chain, k order). */
static void mm4(const double A[16], const double B[16], double C[16], int fma_chain) {
  double T[16];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) {
      double acc = 0.0;
      for (int k = 0; k < 4; ++k) {
        if (fma_chain) acc = fma(A[i * 4 + k], B[k * 4 + j], acc);
        else acc = acc + A[i * 4 + k] * B[k * 4 + j];
      }
      T[i * 4 + j] = acc;
    }
  memcpy(C, T, sizeof(T));
}

static int g_fma_chain = 1;
void iko_set_fma_chain(int on) { g_fma_chain = on; }

static void rot(char axis, double ang, double M[16]) {
  double c = cos(ang), s = sin(ang);
  for (int i = 0; i < 16; ++i) M[i] = (i % 5 == 0) ? 1.0 : 0.0;
  if (axis == 'z') {
    M[0] = c; M[1] = -s; M[4] = s; M[5] = c;
  } else { /* 'x' */
    M[5] = c; M[6] = -s; M[9] = s; M[10] = c;
  }
}

static void trans(double vx, double vy, double vz, double M[16]) {
  for (int i = 0; i < 16; ++i) M[i] = (i % 5 == 0) ? 1.0 : 0.0;
  M[3] = vx; M[7] = vy; M[11] = vz;
}

static int angle_ok(double a) { return !((a < -2 * IKO_PI) || (a > 2 * IKO_PI)); }

/* forward.py:63-70 */
static void dh_transform(double th, double eps, double a, double al, double A[16]) {
  double R[16], T1[16], T2[16], X[16];
  rot('z', th, R);
  trans(0.0, 0.0, eps, T1);
  trans(a, 0.0, 0.0, T2);
  rot('x', al, X);
  mm4(R, T1, A, g_fma_chain);
  mm4(A, T2, A, g_fma_chain);
  mm4(A, X, A, g_fma_chain);
}

/* forward.py:73-94: all four cumulative transforms; joints[k] = M_k[:3,3] */
static int fk_chain(const double dh[16], const double th[4], pt3 joints[4], double Mout[16]) {
  /* dh rows: thetas, epsilons(d), ais(a), alphas */
  for (int i = 0; i < 4; ++i)
    if (!angle_ok(th[i]) || !angle_ok(dh[12 + i])) return IKO_E_ANGLE_RANGE;
  double M[16], A[16];
  dh_transform(th[0], dh[4], dh[8], dh[12], M);
  joints[0].x = M[3]; joints[0].y = M[7]; joints[0].z = M[11];
  for (int i = 1; i < 4; ++i) {
    dh_transform(th[i], dh[4 + i], dh[8 + i], dh[12 + i], A);
    mm4(M, A, M, g_fma_chain);
    joints[i].x = M[3]; joints[i].y = M[7]; joints[i].z = M[11];
  }
  if (Mout) memcpy(Mout, M, sizeof(M));
  return IKO_OK;
}

/* Batch FK: ang n x 4 -> xyz n x 3 (effector), joints n x 4 x 3 (nullable). */
void iko_fk(const double *dh, const double *ang, int64_t n, double *xyz, double *joints,
            int32_t *status) {
  for (int64_t i = 0; i < n; ++i) {
    pt3 J[4];
    int st = fk_chain(dh, ang + 4 * i, J, 0);
    status[i] = st;
    if (st != IKO_OK) {
      for (int c = 0; c < 3; ++c) xyz[3 * i + c] = NAN;
      continue;
    }
    xyz[3 * i + 0] = J[3].x; xyz[3 * i + 1] = J[3].y; xyz[3 * i + 2] = J[3].z;
    if (joints)
      for (int k = 0; k < 4; ++k) {
        joints[12 * i + 3 * k + 0] = J[k].x;
        joints[12 * i + 3 * k + 1] = J[k].y;
        joints[12 * i + 3 * k + 2] = J[k].z;
      }
  }
}

/* ------------------------------------------------------------ FABRIK ---- */
/* fabrik.py:44-67 for a chain of nj (>= 1) joints; returns iterations run.
 * B / F: nj points of caller-provided scratch each. */
static int fabrik_calc(int nj, const double *dists, pt3 *cur, pt3 goal, double tol, int max_iter,
                       int *st, pt3 *B, pt3 *F) {
  pt3 start = cur[0];
  double se = 1.0, ge = 1.0;
  int step = 0;
  while (((se > tol) || (ge > tol)) && (max_iter > step)) {
    /* __backward, fabrik.py:19-29 */
    B[nj - 1] = goal;
    for (int k = nj - 2; k >= 0; --k) B[k] = point_between(B[k + 1], cur[k], dists[k], st);
    se = dist(B[0], start);
    /* __forward, fabrik.py:32-42 (note dists[1:], not dists[:-1]) */
    F[0] = start;
    for (int k = 1; k < nj; ++k) F[k] = point_between(F[k - 1], B[k], dists[k], st);
    ge = dist(F[nj - 1], goal);
    for (int k = 0; k < nj; ++k) cur[k] = F[k];
    step++;
    if (*st != IKO_OK) break; /* the reference raises here; nothing after matters */
  }
  return step;
}

/* Batch Fabrik.calculate with one init chain per point (init: n x nj x 3), any
 * nj >= 1 (fabrik.py takes any length with len(init) == len(dists)).  Returns 0,
 * or -1 when nj < 1 or the scratch cannot be allocated. */
int iko_fabrik_calc(int nj, const double *dists, const double *init, const double *goals,
                    int64_t n, double tol, int max_iter, double *out_joints, int32_t *iters,
                    int32_t *status) {
  if (nj < 1) return -1;
  pt3 *cur = (pt3 *)malloc(sizeof(pt3) * 3 * (size_t)nj);
  if (!cur) return -1;
  pt3 *B = cur + nj, *F = cur + 2 * nj;
  for (int64_t i = 0; i < n; ++i) {
    for (int k = 0; k < nj; ++k) {
      cur[k].x = init[(i * nj + k) * 3 + 0];
      cur[k].y = init[(i * nj + k) * 3 + 1];
      cur[k].z = init[(i * nj + k) * 3 + 2];
    }
    pt3 g = {goals[3 * i], goals[3 * i + 1], goals[3 * i + 2]};
    int st = IKO_OK;
    int it = fabrik_calc(nj, dists, cur, g, tol, max_iter, &st, B, F);
    iters[i] = it;
    status[i] = st;
    for (int k = 0; k < nj; ++k) {
      out_joints[(i * nj + k) * 3 + 0] = cur[k].x;
      out_joints[(i * nj + k) * 3 + 1] = cur[k].y;
      out_joints[(i * nj + k) * 3 + 2] = cur[k].z;
    }
  }
  free(cur);
  return 0;
}

/* inverse.py:54-112 */
static void get_angles(const pt3 J[4], double th[4], int *st) {
  const double pi = IKO_PI;
  pt3 A = {0.0, 0.0, 0.0};
  pt3 B = J[0], C = J[1], D = J[2], E = J[3];
  th[0] = atan2(E.y, E.x);
  double ab = dist(A, B), bc = dist(B, C), cd = dist(C, D), de = dist(D, E);
  double ac = dist(A, C);
  double num = (sq(ab) + sq(bc)) - sq(ac);
  double den = 2 * ab * bc;
  double a2 = py_acos(iko_round_nd(py_div(num, den, st), 8), st);
  if (C.x * D.x < 0) th[1] = (3 * pi / 2) - a2;
  else th[1] = -(pi / 2 - a2);
  double bd = dist(B, D);
  num = (sq(bc) + sq(cd)) - sq(bd);
  den = 2 * bc * cd;
  double a3 = py_acos(iko_round_nd(py_div(num, den, st), 8), st);
  th[2] = -(pi - a3);
  double ce = dist(C, E);
  num = (sq(cd) + sq(de)) - sq(ce);
  den = 2 * cd * de;
  double a4 = py_acos(iko_round_nd(py_div(num, den, st), 8), st);
  pt3 m = point_between(C, E, dist(C, E) / 2, st);
  double da = dist(B, m);
  double db = dist(B, D);
  if (db > da) th[3] = -(pi - a4);
  else th[3] = pi - a4;
}

/* inverse.py:26-35: inclusive bounds, dict order x, y, z. lim = {xlo,xhi,ylo,yhi,zlo,zhi} */
int64_t iko_check_limits(const double *lim, const double *pts, int64_t n) {
  for (int64_t i = 0; i < n; ++i)
    for (int c = 0; c < 3; ++c) {
      double v = pts[3 * i + c];
      if (v < lim[2 * c] || v > lim[2 * c + 1]) return i;
    }
  return -1;
}

/*
 * inverse.py:115-139 per point (limits are checked separately, as the
 * reference does before its loop).  dh: 4x4 row-major DH matrix (thetas,
 * d, a, alpha); the seed uses [atan2(y,x), dh[0][1], dh[0][2], dh[0][3]].
 */
void iko_fabrik_ikine(const double *dh, const double *links, const double *pts, int64_t n,
                      double tol, int max_iter, double *ang, int32_t *iters, double *joints,
                      int32_t *status) {
  for (int64_t i = 0; i < n; ++i) {
    pt3 g = {pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]};
    double th[4] = {atan2(g.y, g.x), dh[1], dh[2], dh[3]};
    pt3 cur[4];
    int st = fk_chain(dh, th, cur, 0);
    int it = 0;
    double a[4] = {NAN, NAN, NAN, NAN};
    pt3 B[4], F[4];
    if (st == IKO_OK) it = fabrik_calc(4, links, cur, g, tol, max_iter, &st, B, F);
    if (st == IKO_OK) get_angles(cur, a, &st);
    status[i] = st;
    iters[i] = it;
    for (int k = 0; k < 4; ++k) ang[4 * i + k] = a[k];
    if (joints)
      for (int k = 0; k < 4; ++k) {
        joints[12 * i + 3 * k + 0] = cur[k].x;
        joints[12 * i + 3 * k + 1] = cur[k].y;
        joints[12 * i + 3 * k + 2] = cur[k].z;
      }
  }
}
