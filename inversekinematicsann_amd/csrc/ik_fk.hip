// ik_fk.hip -- batched forward kinematics and workspace check.
//
// fk_kernel restates ForwardKinematics.fkine (kinematics/forward.py:73-94)
// for a batch: one point per lane, the DH chain in float64 (ik_common.h).
// HBM traffic per point: 32 B angles in + 24 B xyz out (+96 B joints if asked).
#include <cmath>

#include "ik_common.h"

namespace ikhip {

__global__ void reset_stats_kernel(DevStats *S) {
  const int t = threadIdx.x;
  if (t == 0) {
    S->first_oob = ~0ull;
    S->first_err_key = ~0ull;
    S->unseen = 0;
  }
  if (t < kQueueHeads) S->heads[t][0] = 0;
  for (int e = t; e < kOrdClasses * kOrdShards; e += blockDim.x) {
    (&S->cls_tot[0][0])[e] = 0;
    (&S->cls_cur[0][0])[e] = 0;
  }
  if (t < kStatShards) {
    S->sum_iters[t] = 0;
    S->n_capped[t] = 0;
    S->max_fk_err_bits[t] = 0;
    S->sum_fk_err[t] = 0.0;
    S->max_iters[t] = 0;
  }
}

void launch_reset_stats(DevStats *S, hipStream_t st) {
  IK_LAUNCH(reset_stats_kernel, dim3(1), dim3(64), 0, st, S);
}

// kinematics/inverse.py:26-35 InverseKinematics.check_limits
__global__ __launch_bounds__(256) void check_limits_kernel(RobotDev r, const double *pts,
                                                            int64_t n, DevStats *S) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double x = pts[3 * i], y = pts[3 * i + 1], z = pts[3 * i + 2];
  if (outside(r.lim, x, y, z)) atomicMin(&S->first_oob, (unsigned long long)i);
}

void launch_check_limits(const RobotDev &r, const double *pts, int64_t n, DevStats *S,
                         hipStream_t st) {
  if (n <= 0) return;
  unsigned grid = (unsigned)((n + 255) / 256);
  kt_begin("check_limits_kernel", st);
  IK_LAUNCH(check_limits_kernel, dim3(grid), dim3(256), 0, st, r, pts, n, S);
  kt_end(st);
}

// The effector from the closed form of each DH matrix,
// A_k = [[c, -s ca, s sa, a c], [s, c ca, -c sa, a s], [0, sa, ca, d]] (row 3 is
// [0, 0, 0, 1]), with cos / sin(alpha_k) per robot (host, launch_fk).  Every
// entry is the single product the reference's ((Rz Tz) Tx) Rx chain reduces to
// (its other terms multiply exact zeros and ones), so A_k agrees with fk_chain's
// up to the cos / sin(alpha) rounding and signed zeros: three 4x4 products and
// two cos / sin pairs fewer per joint.  cos / sin(theta) come from sincos_fk
// (|error| <= 1.2e-16; the positions stay within 1e-15 of fk_chain's).
struct FkConst {
  double ca[4], sa[4];
};

// The effector of the chain from the closed-form A_k: rows 0-2 of the cumulative
// products, each element the reference's k-ordered FMA chain with the terms that
// multiply A_k's exact zeros dropped (they add a signed zero to a finite sum) and
// its exact one kept as the add it is; the last product forms column 3 only.
__device__ __forceinline__ int fk_effector(const double *dh, const FkConst &k,
                                           const double th[4], d3 &E) {
  int st = IK_OK;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (!angle_ok(th[i]) || !angle_ok(dh[12 + i])) st = IK_E_ANGLE_RANGE;
  double M[12];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    double s, c;
    sincos_fk(th[i], &s, &c);
    const double ca = k.ca[i], sa = k.sa[i], a = dh[8 + i], d = dh[4 + i];
    // A_k rows 0-2: [[c, -s ca, s sa, a c], [s, c ca, -c sa, a s], [0, sa, ca, d]]
    const double A00 = c, A01 = -s * ca, A02 = s * sa, A03 = a * c;
    const double A10 = s, A11 = c * ca, A12 = -c * sa, A13 = a * s;
    const double A21 = sa, A22 = ca, A23 = d;
    if (i == 0) {
      M[0] = A00; M[1] = A01; M[2] = A02;  M[3] = A03;
      M[4] = A10; M[5] = A11; M[6] = A12;  M[7] = A13;
      M[8] = 0.0; M[9] = A21; M[10] = A22; M[11] = A23;
    } else {
      double T[12];
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const double m0 = M[4 * r], m1 = M[4 * r + 1], m2 = M[4 * r + 2], m3 = M[4 * r + 3];
        T[4 * r + 3] = __builtin_fma(m2, A23, __builtin_fma(m1, A13, m0 * A03)) + m3;
        if (i < 3) {
          T[4 * r] = __builtin_fma(m1, A10, m0 * A00);
          T[4 * r + 1] = __builtin_fma(m2, A21, __builtin_fma(m1, A11, m0 * A01));
          T[4 * r + 2] = __builtin_fma(m2, A22, __builtin_fma(m1, A12, m0 * A02));
        }
      }
#pragma unroll
      for (int e = 0; e < 12; ++e) M[e] = T[e];
    }
  }
  E = {M[3], M[7], M[11]};
  return st;
}

// mats (nullable): the four cumulative 4x4 transforms M_1..M_4 of each point,
// the second return value of fkine (forward.py:94), through fk_chain_mats.
__global__ __launch_bounds__(256) void fk_mats_kernel(RobotDev r, const double *__restrict__ ang,
                                                       int64_t n, double *__restrict__ xyz,
                                                       double *__restrict__ mats, DevStats *S) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double th[4] = {ang[4 * i], ang[4 * i + 1], ang[4 * i + 2], ang[4 * i + 3]};
  double *o = mats + 64 * i;
  const int st = fk_chain_mats(r.dh, th, o);
  d3 e = {o[51], o[55], o[59]};
  if (st != IK_OK) {
    record_error(S, i, st);
    e.x = e.y = e.z = __builtin_nan("");
  }
  xyz[3 * i] = e.x;
  xyz[3 * i + 1] = e.y;
  xyz[3 * i + 2] = e.z;
}

// The effector only: a grid-stride loop over the points whose next angles are
// loaded before the current point's chain runs, so the HBM round trip of one
// point hides under the arithmetic of the one before (one point per lane and
// launch left most of the kernel waiting on its loads at 4 waves per SIMD).
__global__ __launch_bounds__(256) void fk_kernel(RobotDev r, FkConst kc,
                                                  const double *__restrict__ ang,
                                                  int64_t n, double *__restrict__ xyz,
                                                  DevStats *S) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // (8-byte loads: a caller's device pointer need not be 16-byte aligned)
  double p0 = ang[4 * i], p1 = ang[4 * i + 1], p2 = ang[4 * i + 2], p3 = ang[4 * i + 3];
  for (; i < n; i += stride) {
    const double th[4] = {p0, p1, p2, p3};
    const int64_t nx = i + stride;
    if (nx < n) {
      p0 = ang[4 * nx];
      p1 = ang[4 * nx + 1];
      p2 = ang[4 * nx + 2];
      p3 = ang[4 * nx + 3];
    }
    d3 e;
    const int st = fk_effector(r.dh, kc, th, e);
    if (st != IK_OK) {
      record_error(S, i, st);
      e.x = e.y = e.z = __builtin_nan("");
    }
    xyz[3 * i] = e.x;
    xyz[3 * i + 1] = e.y;
    xyz[3 * i + 2] = e.z;
  }
}

// ForwardKinematics.fkine for a chain of NJ joints (forward.py:11-94 accepts any
// number of features >= 3; 4 is the robot's own): dh is 4 x NJ row-major (thetas,
// d, a, alpha), ang n x NJ.  The reference builds NJ x NJ matrices whose
// upper-left 4 x 4 block is the usual DH transform and whose remaining rows and
// columns are the identity, so every product is that block's product: the
// kernel forms the 4 x 4 chain (dh_transform + mm4, the same as fk_chain) and
// the host embeds it.  Angles are checked joint by joint, theta then alpha
// (forward.py:23-25 raises on the first).
template <int NJ>
__global__ __launch_bounds__(256) void fk_n_kernel(const double *__restrict__ dh,
                                                    const double *__restrict__ ang, int64_t n,
                                                    double *__restrict__ xyz,
                                                    double *__restrict__ mats, DevStats *S) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int st = IK_OK;
  double M[16], A[16];
#pragma unroll
  for (int k = 0; k < NJ; ++k) {
    const double th = ang[(size_t)i * NJ + k];
    if (!angle_ok(th) || !angle_ok(dh[3 * NJ + k])) st = IK_E_ANGLE_RANGE;
    dh_transform(th, dh[NJ + k], dh[2 * NJ + k], dh[3 * NJ + k], k == 0 ? M : A);
    if (k > 0) mm4(M, A, M);
    if (mats) {
      double *o = mats + ((size_t)i * NJ + k) * 16;
#pragma unroll
      for (int e = 0; e < 16; ++e) o[e] = M[e];
    }
  }
  d3 e = {M[3], M[7], M[11]};
  if (st != IK_OK) {
    record_error(S, i, st);
    e.x = e.y = e.z = __builtin_nan("");
  }
  xyz[3 * i] = e.x;
  xyz[3 * i + 1] = e.y;
  xyz[3 * i + 2] = e.z;
}

// The same chain for any number of joints (longer than the unrolled builds
// above): the joint loop runs at run time, the arithmetic is fk_n_kernel's.
__global__ __launch_bounds__(256) void fk_any_kernel(int nj, const double *__restrict__ dh,
                                                     const double *__restrict__ ang, int64_t n,
                                                     double *__restrict__ xyz,
                                                     double *__restrict__ mats, DevStats *S) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int st = IK_OK;
  double M[16], A[16];
  for (int k = 0; k < nj; ++k) {
    const double th = ang[(size_t)i * nj + k];
    if (!angle_ok(th) || !angle_ok(dh[3 * nj + k])) st = IK_E_ANGLE_RANGE;
    dh_transform(th, dh[nj + k], dh[2 * nj + k], dh[3 * nj + k], k == 0 ? M : A);
    if (k > 0) mm4(M, A, M);
    if (mats) {
      double *o = mats + ((size_t)i * nj + k) * 16;
#pragma unroll
      for (int e = 0; e < 16; ++e) o[e] = M[e];
    }
  }
  d3 e = {M[3], M[7], M[11]};
  if (st != IK_OK) {
    record_error(S, i, st);
    e.x = e.y = e.z = __builtin_nan("");
  }
  xyz[3 * i] = e.x;
  xyz[3 * i + 1] = e.y;
  xyz[3 * i + 2] = e.z;
}

void launch_fk_n(int nj, const double *dh, const double *ang, int64_t n, double *xyz,
                 double *mats, DevStats *S, hipStream_t st) {
  if (n <= 0) return;
  const unsigned grid = (unsigned)((n + 255) / 256);
  kt_begin("fk_n_kernel", st);
#define IK_FKN(K)                                                                           \
  case K:                                                                                   \
    IK_LAUNCH(fk_n_kernel<K>, dim3(grid), dim3(256), 0, st, dh, ang, n, xyz, mats, S); \
    break;
  switch (nj) {
    IK_FKN(2)
    IK_FKN(3)
    IK_FKN(4)
    IK_FKN(5)
    IK_FKN(6)
    IK_FKN(7)
    IK_FKN(8)
    default:
      IK_LAUNCH(fk_any_kernel, dim3(grid), dim3(256), 0, st, nj, dh, ang, n, xyz, mats, S);
      break;
  }
#undef IK_FKN
  kt_end(st);
}

static int fk_cus() {
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0)
    cus = 256;
  return cus;
}

void launch_fk(const RobotDev &r, const double *ang, int64_t n, double *xyz, double *joints,
               DevStats *S, hipStream_t st) {
  if (n <= 0) return;
  const unsigned grid_all = (unsigned)((n + 255) / 256);
  kt_begin("fk_kernel", st);
  if (joints) {
    IK_LAUNCH(fk_mats_kernel, dim3(grid_all), dim3(256), 0, st, r, ang, n, xyz,
                       joints, S);
  } else {
    FkConst kc;
    for (int i = 0; i < 4; ++i) {
      kc.ca[i] = std::cos(r.dh[12 + i]);
      kc.sa[i] = std::sin(r.dh[12 + i]);
    }
    // resident blocks only (8 per CU): every lane walks several points
    // (2, 4, 6, 8 blocks per CU or one point per lane all measured 17.0-17.3 us per
    // 1M points: at that size the launch's fixed cost, ~6 us, is a third of it)
    const unsigned cap = (unsigned)fk_cus() * 8;
    const unsigned grid = grid_all < cap ? grid_all : cap;
    IK_LAUNCH(fk_kernel, dim3(grid), dim3(256), 0, st, r, kc, ang, n, xyz, S);
  }
  kt_end(st);
}

}  // namespace ikhip
