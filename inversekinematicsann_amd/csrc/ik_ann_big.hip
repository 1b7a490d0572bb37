// ik_ann_big.hip -- ANN.predict for models outside the fused kernel's caps.
//
// Restates ANN.predict (kinematics/ann.py:70-76) for a Keras Dense stack of any
// depth and width (ann.py:46-56,78-85 loads any Sequential): more than
// kAnnMaxLayers layers, or a layer wider than kAnnMaxWidth.  The fused kernel
// (ik_ann.hip) keeps a tile's activations in LDS through every layer, which
// bounds the width by LDS and the depth by its kernel arguments; here the
// activations go through HBM, one launch per layer, over chunks of points:
//   annb_in_kernel     workspace check + StandardScaler.transform (float64) -> fp32
//                      rows of 8 (x, y, z, 0...)
//   annb_gemm_kernel   Y = act(X @ W + b), exact-fp32 v_mfma_f32_32x32x2_f32;
//                      128 x 128 output tiles, 4 waves each 64 x 64, the X tile
//                      double-buffered through LDS 32 deep in K, the weights read
//                      straight from L2 in the fused kernel's packed fragment order
//                      (ann_pack_layer: one 16-byte load per lane per 8-deep group)
//   annb_out_kernel    StandardScaler.inverse_transform (in-place fp32, float64
//                      ops) + the cli.py:54-61 FK round trip + stats, as the fused
//                      kernel's epilogue does
// A chunk's activations alternate between two buffers of rows x ld floats (ld the
// widest padded layer); the chunk's row count keeps both within the context's
// activation budget.  Still one library call (ik_ann_solve): the chunk loop is
// host code on the context's stream.
#include <cmath>

#include "ik_common.h"

namespace ikhip {
namespace annb {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kBM = 128;      // output rows per workgroup
constexpr int kBN = 128;      // output columns per workgroup (4 column tiles of 32)
constexpr int kBK = 32;       // K per LDS stage (4 groups of 8)
constexpr int kLdA = kBK + 4; // LDS row stride in floats (= 4 mod 32: conflict-free b128 reads)

// The fused kernel's activations (ik_ann.hip act_apply): same forms, same bits.
__device__ __forceinline__ float act_apply(int act, float v) {
  switch (act) {
    case IK_ACT_TANH: {
      const float e = __builtin_amdgcn_exp2f(2.885390081777927f * v);
      return __builtin_fmaf(-2.0f, __builtin_amdgcn_rcpf(1.0f + e), 1.0f);
    }
    case IK_ACT_RELU:
      return fmaxf(v, 0.0f);
    case IK_ACT_SIGMOID:
      return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * v));
    default:
      return v;
  }
}

// Input rows: x = f32((p - x_mean) / x_scale) in columns 0..2 of an 8-float row
// (columns 3..7 zero: the first layer's packed weights are zero there too).
__global__ __launch_bounds__(256) void annb_in_kernel(const double *__restrict__ pts, int64_t p0,
                                                      int64_t rows, double xm0, double xm1,
                                                      double xm2, double xs0, double xs1,
                                                      double xs2, RobotDev r, int check_limits,
                                                      float *__restrict__ X, DevStats *S) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows) return;
  const int64_t pt = p0 + i;
  const double px = pts[3 * pt], py = pts[3 * pt + 1], pz = pts[3 * pt + 2];
  if (check_limits && outside(r.lim, px, py, pz)) atomicMin(&S->first_oob, (unsigned long long)pt);
  f32x4 *row = reinterpret_cast<f32x4 *>(X + 8 * i);
  row[0] = f32x4{(float)((px - xm0) / xs0), (float)((py - xm1) / xs1), (float)((pz - xm2) / xs2),
                 0.0f};
  row[1] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
}

// One Dense layer over `rows` rows: C[rows x NT*32] = act(A[rows x 8G] @ W + b).
// A: row stride lda floats (a multiple of 4, >= 8G; columns past the layer's
// real inputs hold finite values, multiplied by the packed weights' zero rows).
// wp: ann_pack_layer order, dst[((nt*G + g)*64 + lane)*4 + s] =
// W[8g + 4(lane>>5) + s][32nt + (lane&31)]; the A fragment is read in the same
// permuted K order (4 consecutive activations per lane half), so each MFMA step
// s pairs the same k on both operands.  Output columns past the layer's width
// get act(0 + 0): finite, and the next layer's packed weights are zero there.
__global__ __launch_bounds__(256) void annb_gemm_kernel(const float *__restrict__ A, int lda,
                                                        int64_t rows,
                                                        const f32x4 *__restrict__ wp, int G,
                                                        int NT, const float *__restrict__ bias,
                                                        int act, float *__restrict__ C,
                                                        int ldc) {
  __shared__ __attribute__((aligned(16))) float As[2][kBM * kLdA];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware tile order: workgroups are dealt round-robin over the 8 XCDs, so
  // workgroup b runs on XCD b % 8; XCD x takes row panels x, x + 8, ... and every
  // column block of a panel in turn, so a panel's A tile is read from HBM once into
  // that XCD's L2 and reused by all its column blocks
  const int nCB = (NT + kBN / 32 - 1) / (kBN / 32);
  const unsigned b = blockIdx.x, xcd = b & 7u, k = b >> 3;
  const int64_t rb = (int64_t)(k / (unsigned)nCB) * 8 + xcd;
  const int cb = (int)(k % (unsigned)nCB);
  if (rb * kBM >= rows) return;  // the grid's last panel row is padded to 8
  const int64_t row0 = rb * kBM;
  const int nt0 = cb * (kBN / 32) + wn * 2;  // this wave's two column tiles
  const int r = lane & 31, h = lane >> 5;
  f32x16 acc[2][2];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[m][j] = (f32x16)(0.0f);

  // the A tile of one stage: 128 rows x 32 floats, 4 x 16 bytes per thread, loaded
  // two stages ahead into one of two register sets (the loads' HBM latency under
  // load outlasts one stage of MFMAs) and written to the LDS buffer of its stage at
  // the end of the stage before
  const int nst = (G + 3) / 4;
  f32x4 ra0[4], ra1[4];
  auto load_a = [&](f32x4 (&ra)[4], int s) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + 256 * i;
      const int row = idx >> 3, c4 = idx & 7;
      const int64_t gr = row0 + row;
      const int kk = s * kBK + 4 * c4;
      ra[i] = (s < nst && gr < rows && kk < lda)
                  ? *reinterpret_cast<const f32x4 *>(A + gr * (int64_t)lda + kk)
                  : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    }
  };
  auto store_a = [&](const f32x4 (&ra)[4], int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + 256 * i;
      const int row = idx >> 3, c4 = idx & 7;
      *reinterpret_cast<f32x4 *>(&As[buf][row * kLdA + 4 * c4]) = ra[i];
    }
  };
  // the weight fragments of stage s (zero for column tiles past the layer), loaded one
  // stage ahead so that their L2 latency hides under the stage before's MFMAs
  auto load_b = [&](f32x4 (&b)[4][2], int s) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int g = s * 4 + u, nt = nt0 + j;
        b[u][j] = (g < G && nt < NT) ? wp[((size_t)nt * G + g) * 64 + lane]
                                     : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      }
  };
  // stage s: the next stage's weights and the A tile two ahead go out, the MFMAs of
  // this stage run, then the A tile of stage s + 1 (loaded one stage ago) goes to LDS
  auto stage = [&](int s, f32x4 (&bn)[4][2], f32x4 (&ra_fill)[4], const f32x4 (&ra_next)[4]) {
    const int buf = s & 1;
    f32x4 b[4][2];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 2; ++j) b[u][j] = bn[u][j];
    if (s + 1 < nst) load_b(bn, s + 1);
    if (s + 2 < nst) load_a(ra_fill, s + 2);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (s * 4 + u >= G) break;
      f32x4 a[2];
#pragma unroll
      for (int m = 0; m < 2; ++m)
        a[m] = *reinterpret_cast<const f32x4 *>(
            &As[buf][(wm * 64 + m * 32 + r) * kLdA + 8 * u + 4 * h]);
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int m = 0; m < 2; ++m)
            acc[m][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[m][q], b[u][j][q], acc[m][j], 0, 0, 0);
    }
    if (s + 1 < nst) store_a(ra_next, buf ^ 1);
    __syncthreads();
  };
  f32x4 bn[4][2];
  load_b(bn, 0);
  load_a(ra0, 0);
  load_a(ra1, 1);
  store_a(ra0, 0);
  __syncthreads();
  // even stages fill ra0 (stage s + 2) and store ra1 (stage s + 1); odd ones the reverse
  for (int s = 0; s < nst; s += 2) {
    stage(s, bn, ra0, ra1);
    if (s + 1 < nst) stage(s + 1, bn, ra1, ra0);
  }
  // bias (after the dot product, as Keras adds it) + activation, stored per
  // accumulator element: lane (r, h) holds column r of rows (q&3) + 8(q>>2) + 4h
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int nt = nt0 + j;
    if (nt >= NT) continue;
    const int col = nt * 32 + r;
    const float bv = bias[col];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int64_t row = row0 + wm * 64 + m * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
        if (row < rows) C[row * (int64_t)ldc + col] = act_apply(act, acc[m][j][q] + bv);
      }
  }
}

// Output: StandardScaler.inverse_transform (in-place fp32 with float64 operands,
// as the fused kernel's epilogue) + the FK round trip and its batch stats.
struct OutArgs {
  double ym[4], ys[4];
  double jc[16];
  int alpha_bad;
};

__global__ __launch_bounds__(256) void annb_out_kernel(const float *__restrict__ Y, int ldy,
                                                       const double *__restrict__ pts,
                                                       int64_t p0, int64_t rows, OutArgs o,
                                                       float *__restrict__ ang,
                                                       double *__restrict__ fk_err,
                                                       DevStats *S) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double e = 0.0;
  if (i < rows) {
    const int64_t pt = p0 + i;
    const float *row = Y + i * (int64_t)ldy;
    float y[4];
    double th[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float t = (float)((double)row[c] * o.ys[c]);
      y[c] = (float)((double)t + o.ym[c]);
      th[c] = (double)y[c];
    }
    *reinterpret_cast<f32x4 *>(ang + 4 * pt) = f32x4{y[0], y[1], y[2], y[3]};
    if (fk_err) {
      const double err = fk_error(o.jc, th, pts[3 * pt], pts[3 * pt + 1], pts[3 * pt + 2],
                                  o.alpha_bad);
      fk_err[pt] = err;
      e = (err == err) ? err : 0.0;
    }
  }
  if (fk_err) wave_fk_stats(S, e, e);
}

}  // namespace annb

size_t ann_big_ld(const AnnBigModel &m) {
  int ld = 8;
  for (const AnnBigLayer &L : m.layers) ld = L.np > ld ? L.np : ld;
  return (size_t)ld;
}

int64_t ann_big_rows(const AnnBigModel &m, size_t act_bytes) {
  const size_t per_row = 2 * ann_big_ld(m) * sizeof(float);
  int64_t rows = (int64_t)(act_bytes / per_row) / annb::kBM * annb::kBM;
  return rows;
}

void launch_ann_big(const AnnBigModel &m, const RobotDev &r, const double *pts, int64_t n,
                    float *ang, double *fk_err, bool check_limits, DevStats *S, hipStream_t st,
                    float *act, int64_t chunk_rows) {
  using namespace annb;
  if (n <= 0 || chunk_rows <= 0) return;
  const int ld = (int)ann_big_ld(m);
  float *buf[2] = {act, act + (size_t)chunk_rows * ld};
  OutArgs o;
  for (int c = 0; c < 4; ++c) {
    o.ym[c] = m.ym[c];
    o.ys[c] = m.ys[c];
  }
  fk_trip_consts(r, o.jc, &o.alpha_bad);
  for (int64_t p0 = 0; p0 < n; p0 += chunk_rows) {
    const int64_t rows = (n - p0) < chunk_rows ? (n - p0) : chunk_rows;
    const unsigned g1 = (unsigned)((rows + 255) / 256);
    kt_begin("annb_in_kernel", st);
    hipLaunchKernelGGL(annb_in_kernel, dim3(g1), dim3(256), 0, st, pts, p0, rows, m.xm[0],
                       m.xm[1], m.xm[2], m.xs[0], m.xs[1], m.xs[2], r, check_limits ? 1 : 0,
                       buf[0], S);
    kt_end(st);
    int cur = 0, lda = 8;
    for (const AnnBigLayer &L : m.layers) {
      const int G = L.kp / 8, NT = L.np / 32;
      const int64_t nRB = (rows + kBM - 1) / kBM;
      const dim3 grid((unsigned)((nRB + 7) / 8 * 8 * ((NT + 3) / 4)));
      kt_begin("annb_gemm_kernel", st);
      hipLaunchKernelGGL(annb_gemm_kernel, grid, dim3(256), 0, st, buf[cur], lda, rows,
                         reinterpret_cast<const f32x4 *>(L.wp), G, NT, L.bias, L.act,
                         buf[cur ^ 1], L.np);
      kt_end(st);
      cur ^= 1;
      lda = L.np;
    }
    kt_begin("annb_out_kernel", st);
    hipLaunchKernelGGL(annb_out_kernel, dim3(g1), dim3(256), 0, st, buf[cur], lda, pts, p0, rows,
                       o, ang, fk_err, S);
    kt_end(st);
  }
}

}  // namespace ikhip
