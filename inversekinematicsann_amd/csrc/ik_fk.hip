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
    S->queue = 0;
    S->pad0 = 0;
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
  hipLaunchKernelGGL(reset_stats_kernel, dim3(1), dim3(64), 0, st, S);
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
  hipLaunchKernelGGL(check_limits_kernel, dim3(grid), dim3(256), 0, st, r, pts, n, S);
  kt_end(st);
}

// The translations of M_1..M_4 from the closed form of each DH matrix,
// A_k = [[c, -s ca, s sa, a c], [s, c ca, -c sa, a s], [0, sa, ca, d]] (row 3 is
// [0, 0, 0, 1]), with cos / sin(alpha_k) per robot (host, launch_fk).  Every
// entry is the single product the reference's ((Rz Tz) Tx) Rx chain reduces to
// (its other terms multiply exact zeros and ones), so A_k and the cumulative
// rows-0..2 products (mm4_r3: the reference's k-ordered FMA chains) agree with
// fk_chain to the last bits up to the cos / sin(alpha) rounding: three 4x4
// products and two cos / sin pairs fewer per joint.
struct FkConst {
  double ca[4], sa[4];
};

__device__ __forceinline__ int fk_chain_closed(const double *dh, const FkConst &k,
                                               const double th[4], d3 J[4]) {
  int st = IK_OK;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (!angle_ok(th[i]) || !angle_ok(dh[12 + i])) st = IK_E_ANGLE_RANGE;
  double M[12], A[16];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    double s, c;
    sincos(th[i], &s, &c);
    const double ca = k.ca[i], sa = k.sa[i], a = dh[8 + i], d = dh[4 + i];
    A[0] = c;   A[1] = -s * ca; A[2] = s * sa;  A[3] = a * c;
    A[4] = s;   A[5] = c * ca;  A[6] = -c * sa; A[7] = a * s;
    A[8] = 0.0; A[9] = sa;      A[10] = ca;     A[11] = d;
    A[12] = 0.0; A[13] = 0.0;   A[14] = 0.0;    A[15] = 1.0;
    if (i == 0) {
#pragma unroll
      for (int e = 0; e < 12; ++e) M[e] = A[e];
    } else {
      mm4_r3(M, A, M);
    }
    J[i].x = M[3]; J[i].y = M[7]; J[i].z = M[11];
  }
  return st;
}

// mats (nullable): the four cumulative 4x4 transforms M_1..M_4 of each point,
// the second return value of fkine (forward.py:94).
__global__ __launch_bounds__(256) void fk_kernel(RobotDev r, FkConst kc,
                                                  const double *__restrict__ ang,
                                                  int64_t n, double *__restrict__ xyz,
                                                  double *__restrict__ mats, DevStats *S) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double th[4] = {ang[4 * i], ang[4 * i + 1], ang[4 * i + 2], ang[4 * i + 3]};
  d3 J[4];
  int st;
  if (mats) {
    double *o = mats + 64 * i;
    st = fk_chain_mats(r.dh, th, o);
    for (int k = 0; k < 4; ++k) J[k] = {o[16 * k + 3], o[16 * k + 7], o[16 * k + 11]};
  } else {
    st = fk_chain_closed(r.dh, kc, th, J);
  }
  if (st != IK_OK) {
    record_error(S, i, st);
    J[3].x = J[3].y = J[3].z = __builtin_nan("");
  }
  xyz[3 * i] = J[3].x;
  xyz[3 * i + 1] = J[3].y;
  xyz[3 * i + 2] = J[3].z;
}

void launch_fk(const RobotDev &r, const double *ang, int64_t n, double *xyz, double *joints,
               DevStats *S, hipStream_t st) {
  if (n <= 0) return;
  unsigned grid = (unsigned)((n + 255) / 256);
  FkConst kc;
  for (int i = 0; i < 4; ++i) {
    kc.ca[i] = std::cos(r.dh[12 + i]);
    kc.sa[i] = std::sin(r.dh[12 + i]);
  }
  kt_begin("fk_kernel", st);
  hipLaunchKernelGGL(fk_kernel, dim3(grid), dim3(256), 0, st, r, kc, ang, n, xyz, joints, S);
  kt_end(st);
}

}  // namespace ikhip
