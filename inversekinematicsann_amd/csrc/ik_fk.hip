// ik_fk.hip -- batched forward kinematics and workspace check.
//
// fk_kernel restates ForwardKinematics.fkine (kinematics/forward.py:73-94)
// for a batch: one point per lane, the DH chain in float64 (ik_common.h).
// HBM traffic per point: 32 B angles in + 24 B xyz out (+96 B joints if asked).
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

// mats (nullable): the four cumulative 4x4 transforms M_1..M_4 of each point,
// the second return value of fkine (forward.py:94).
__global__ __launch_bounds__(256) void fk_kernel(RobotDev r, const double *__restrict__ ang,
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
    st = fk_chain(r.dh, th, J);
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
  kt_begin("fk_kernel", st);
  hipLaunchKernelGGL(fk_kernel, dim3(grid), dim3(256), 0, st, r, ang, n, xyz, joints, S);
  kt_end(st);
}

}  // namespace ikhip
