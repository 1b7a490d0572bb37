// ik_ann.hip -- fused ANN inverse kinematics for gfx950 (fp32 MFMA).
//
// Restates ANN.predict (kinematics/ann.py:70-76) for a batch in ONE launch:
//   x = f32((p - x_mean) / x_scale)            StandardScaler.transform, float64
//   h_{l+1} = act_l(h_l @ W_l + b_l)           Keras Dense layers, ann.py:46-56
//   y = f32(f32(y * y_scale) + y_mean)         StandardScaler.inverse_transform
// plus, in the epilogue, the cli.py:54-61 FK round trip |FK(y) - p|_2 and the
// inverse.py:26-35 workspace check.
//
// Layout (DESIGN.md "ANN"): a workgroup of 4 waves owns a tile of 64 points
// and carries it through every layer with the activations resident in LDS
// (64 x 516 fp32, 129 KiB; the 516 stride makes the ds_read_b128 A-fragment
// reads bank-conflict free).  Each wave computes a 64 x (32*NR) slab of the
// layer output with v_mfma_f32_32x32x2_f32 (exact fp32, 2x4 accumulator tiles
// in AGPR/VGPR), streaming its weight columns straight from L2 into registers
// in a pre-packed "MFMA fragment" order (one 1 KiB dwordx4 load per 8-deep K
// group and column tile), prefetched one K group ahead.  Bias + activation
// are applied on the accumulators and written back over the tile in LDS.
// The grid is persistent: one workgroup per CU walks the point tiles.
#include "ik_common.h"

namespace ikhip {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kBM = 64;    // points per tile
constexpr int kLd = 516;   // LDS row stride in floats (>= 512 + 4)
constexpr int kWaves = 4;  // waves per workgroup

struct AnnArgs {
  AnnModelDev m;
  RobotDev r;
  const double *pts;
  int64_t n;
  float *ang;
  double *fk_err;
  int check_limits;
  DevStats *S;
};

// tanh(x) = sign(x) (1 - e) / (1 + e), e = exp(-2|x|); abs error ~1e-7.
template <int ACT>
__device__ __forceinline__ float act_apply(float v) {
  if constexpr (ACT == IK_ACT_TANH) {
    float e = __expf(-2.0f * fabsf(v));
    float t = __fdividef(1.0f - e, 1.0f + e);
    return copysignf(t, v);
  } else if constexpr (ACT == IK_ACT_RELU) {
    return fmaxf(v, 0.0f);
  } else if constexpr (ACT == IK_ACT_SIGMOID) {
    return __fdividef(1.0f, 1.0f + __expf(-v));
  } else {
    return v;
  }
}

// Operands of one 8-deep K group: A fragments of the two 32-row tiles (LDS)
// and the B fragments of the wave's NR column tiles (global, packed).
template <int NR>
struct Frag {
  f32x4 a0, a1;
  f32x4 b[NR];
};

template <int NR>
__device__ __forceinline__ void load_group(Frag<NR> &f, const float *a0p, const float *a1p,
                                           const f32x4 *const (&bp)[NR], int g) {
  f.a0 = *reinterpret_cast<const f32x4 *>(a0p + 8 * g);
  f.a1 = *reinterpret_cast<const f32x4 *>(a1p + 8 * g);
#pragma unroll
  for (int j = 0; j < NR; ++j) f.b[j] = bp[j][(size_t)g * 64];
}

template <int NR>
__device__ __forceinline__ void mma_group(const Frag<NR> &f, f32x16 (&acc)[2][NR]) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      acc[0][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f.a0[s], f.b[j][s], acc[0][j], 0, 0, 0);
      acc[1][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f.a1[s], f.b[j][s], acc[1][j], 0, 0, 0);
    }
  }
}

// One layer, one wave: out[64 x 32*NR] for the wave's column tiles
// nt_j = wave + kWaves * j.  G = padded K / 8.  Operands are triple-buffered:
// the loads of group g+2 are issued before the MFMAs of group g (a scheduling
// barrier keeps the compiler from sinking them), so ~2 groups (4k cycles of
// MFMA) cover the L2 / MALL latency of the weight stream.
template <int NR>
__device__ __forceinline__ void layer_gemm(const float *H, const f32x4 *__restrict__ wp, int G,
                                           int wave, int lane, f32x16 (&acc)[2][NR]) {
  const int r = lane & 31, h = lane >> 5;
  const float *a0p = H + r * kLd + 4 * h;
  const float *a1p = H + (32 + r) * kLd + 4 * h;
  const f32x4 *bp[NR];
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    bp[j] = wp + (size_t)(wave + kWaves * j) * G * 64 + lane;
#pragma unroll
    for (int m = 0; m < 2; ++m) acc[m][j] = (f32x16)(0.0f);
  }
  const int last = G - 1;
  Frag<NR> f0, f1, f2;
  load_group(f0, a0p, a1p, bp, 0);
  load_group(f1, a0p, a1p, bp, min(1, last));
  int g = 0;
  for (; g + 3 <= G; g += 3) {
    load_group(f2, a0p, a1p, bp, min(g + 2, last));
    __builtin_amdgcn_sched_barrier(0);
    mma_group(f0, acc);
    __builtin_amdgcn_sched_barrier(0);
    load_group(f0, a0p, a1p, bp, min(g + 3, last));
    __builtin_amdgcn_sched_barrier(0);
    mma_group(f1, acc);
    __builtin_amdgcn_sched_barrier(0);
    load_group(f1, a0p, a1p, bp, min(g + 4, last));
    __builtin_amdgcn_sched_barrier(0);
    mma_group(f2, acc);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (g < G) mma_group(f0, acc);
  if (g + 1 < G) mma_group(f1, acc);
}

template <int NR, int ACT>
__device__ __forceinline__ void layer_store(float *H, const float *__restrict__ bias, int wave,
                                            int lane, const f32x16 (&acc)[2][NR]) {
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const int col = (wave + kWaves * j) * 32 + r;
    const float bv = bias[col];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int row = m * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
        H[row * kLd + col] = act_apply<ACT>(acc[m][j][q] + bv);
      }
  }
}

template <int NR>
__device__ __forceinline__ void run_layer(float *H, const f32x4 *wp, const float *bias, int act,
                                          int G, int wave, int lane) {
  f32x16 acc[2][NR];
  layer_gemm<NR>(H, wp, G, wave, lane, acc);
  __syncthreads();  // every wave has finished reading the layer input
  switch (act) {
    case IK_ACT_TANH: layer_store<NR, IK_ACT_TANH>(H, bias, wave, lane, acc); break;
    case IK_ACT_RELU: layer_store<NR, IK_ACT_RELU>(H, bias, wave, lane, acc); break;
    case IK_ACT_SIGMOID: layer_store<NR, IK_ACT_SIGMOID>(H, bias, wave, lane, acc); break;
    default: layer_store<NR, IK_ACT_LINEAR>(H, bias, wave, lane, acc); break;
  }
}

__global__ __launch_bounds__(256, 1) void ann_fused_kernel(AnnArgs a) {
  __shared__ __attribute__((aligned(16))) float H[kBM * kLd];
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int64_t ntiles = (a.n + kBM - 1) / kBM;

  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t pt = tile * kBM + tid;
    double px = 0.0, py = 0.0, pz = 0.0;
    // ---- input: workspace check + StandardScaler.transform (float64) -> fp32
    if (tid < kBM) {
      float x0 = 0.0f, x1 = 0.0f, x2 = 0.0f;
      if (pt < a.n) {
        px = a.pts[3 * pt];
        py = a.pts[3 * pt + 1];
        pz = a.pts[3 * pt + 2];
        if (a.check_limits && outside(a.r.lim, px, py, pz))
          atomicMin(&a.S->first_oob, (unsigned long long)pt);
        x0 = (float)((px - a.m.xm[0]) / a.m.xs[0]);
        x1 = (float)((py - a.m.xm[1]) / a.m.xs[1]);
        x2 = (float)((pz - a.m.xm[2]) / a.m.xs[2]);
      }
      f32x4 *row = reinterpret_cast<f32x4 *>(H + tid * kLd);
      row[0] = f32x4{x0, x1, x2, 0.0f};
      row[1] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    }
    __syncthreads();
    // ---- Dense layers
    for (int l = 0; l < a.m.n_layers; ++l) {
      const int G = a.m.kp[l] >> 3;
      const int NT = a.m.np[l] >> 5;
      const int cnt = (wave < NT) ? (NT - wave + kWaves - 1) / kWaves : 0;
      const f32x4 *wp = reinterpret_cast<const f32x4 *>(a.m.wp[l]);
      const float *bias = a.m.bias[l];
      const int act = a.m.act[l];
      switch (cnt) {
        case 4: run_layer<4>(H, wp, bias, act, G, wave, lane); break;
        case 3: run_layer<3>(H, wp, bias, act, G, wave, lane); break;
        case 2: run_layer<2>(H, wp, bias, act, G, wave, lane); break;
        case 1: run_layer<1>(H, wp, bias, act, G, wave, lane); break;
        default: __syncthreads(); break;  // idle wave still joins the barrier
      }
      __syncthreads();
    }
    // ---- output: StandardScaler.inverse_transform (in-place fp32, fp64 ops) + FK
    if (tid < kBM) {
      bool valid = pt < a.n;
      double err = 0.0;
      if (valid) {
        const float *row = H + tid * kLd;
        float y[4];
        double th[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          float t = (float)((double)row[c] * a.m.ys[c]);
          y[c] = (float)((double)t + a.m.ym[c]);
          th[c] = (double)y[c];
        }
        *reinterpret_cast<f32x4 *>(a.ang + 4 * pt) = f32x4{y[0], y[1], y[2], y[3]};
        if (a.fk_err) {
          d3 J[4];
          int st = fk_chain(a.r.dh, th, J);
          d3 p = {px, py, pz};
          err = (st == IK_OK) ? dist3(J[3], p) : __builtin_nan("");
          a.fk_err[pt] = err;
        }
      }
      if (a.fk_err) {
        double e = (valid && err == err) ? err : 0.0;
        double mx = wave_max_f64(e);
        double sm = wave_sum_f64(e);
        if (lane == 0) {
          atomicMax(&a.S->max_fk_err_bits, (unsigned long long)__double_as_longlong(mx));
          atomicAdd(&a.S->sum_fk_err, sm);
        }
      }
    }
    __syncthreads();  // the next tile's staging overwrites H
  }
}

size_t ann_packed_floats(int k, int n) {
  int kp = (k + 7) / 8 * 8, np = (n + 31) / 32 * 32;
  return (size_t)kp * np;
}

// dst[((nt*G + g)*64 + lane)*4 + s] = W[8g + 4*(lane>>5) + s][nt*32 + (lane&31)]
// -- the B fragment of v_mfma_f32_32x32x2_f32 for K-step s of group g, with the
// K order inside a group permuted to match the A fragment read (ds_read_b128 of
// 4 consecutive activations per lane half).
void ann_pack_layer(const float *W, int k, int n, float *dst) {
  int kp = (k + 7) / 8 * 8, np = (n + 31) / 32 * 32;
  int G = kp / 8, NT = np / 32;
  for (int nt = 0; nt < NT; ++nt)
    for (int g = 0; g < G; ++g)
      for (int lane = 0; lane < 64; ++lane)
        for (int s = 0; s < 4; ++s) {
          int kk = 8 * g + 4 * (lane >> 5) + s;
          int c = nt * 32 + (lane & 31);
          dst[(((size_t)nt * G + g) * 64 + lane) * 4 + s] =
              (kk < k && c < n) ? W[(size_t)kk * n + c] : 0.0f;
        }
}

void launch_ann(const AnnModelDev &m, const RobotDev &r, const double *pts, int64_t n,
                float *ang, double *fk_err, bool check_limits, DevStats *S, hipStream_t st) {
  if (n <= 0) return;
  AnnArgs a;
  a.m = m;
  a.r = r;
  a.pts = pts;
  a.n = n;
  a.ang = ang;
  a.fk_err = fk_err;
  a.check_limits = check_limits ? 1 : 0;
  a.S = S;
  int dev = 0, cus = 256;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0)
    cus = 256;
  int64_t ntiles = (n + kBM - 1) / kBM;
  unsigned grid = (unsigned)(ntiles < cus ? ntiles : cus);
  kt_begin("ann_fused_kernel", st);
  hipLaunchKernelGGL(ann_fused_kernel, dim3(grid), dim3(256), 0, st, a);
  kt_end(st);
}

}  // namespace ikhip
