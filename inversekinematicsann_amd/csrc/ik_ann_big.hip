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
//                      128 x 128 output tiles, 4 waves each 64 x 64, the X tile and
//                      the weights (the fused kernel's packed fragment order,
//                      ann_pack_layer) double-buffered through LDS 32 deep in K
//   annb_gemm_x6_kernel  the same layer in the bf16x6 mode (IK_ANN_BF16X6): six
//                      bf16 products per fp32 one on v_mfma_f32_16x16x32_bf16
//   annb_out_kernel    StandardScaler.inverse_transform (in-place fp32, float64
//                      ops) + the cli.py:54-61 FK round trip + stats, as the fused
//                      kernel's epilogue does
// A chunk's activations alternate between two buffers of rows x ld floats (ld the
// widest padded layer); the chunk's row count keeps both within the context's
// activation budget.  Still one library call (ik_ann_solve): the chunk loop is
// host code on the context's stream.
#include <cmath>
#include <cstring>
#include <type_traits>

#include "ik_common.h"

namespace ikhip {
namespace annb {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kBM = 128;      // chunk granularity of the activation buffers (rows)
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
//
// Workgroup tile 128 rows x 128 columns, 4 waves (one per SIMD) of 64 x 64 (2 x 2
// accumulators of v_mfma_f32_32x32x2_f32), two workgroups per CU so that one's
// barrier and stage turnover run under the other's MFMAs; K in stages of 32 (4
// groups of 8).  Both operands go through LDS, double-buffered: the stage's A tile
// (128 x 32 floats, 18 KiB with the row pad, from HBM) and its B tile (the block's
// 4 column tiles x 4 groups, 16 KiB of packed fragments, from L2 / MALL) are loaded
// once per workgroup and read by the two waves that need each.  Both are loaded
// two stages ahead into one of two register sets and written to the stage's
// buffer at the start of the stage before (their loads are a stage old by then);
// inside a stage the next group's fragments are read from LDS before the current
// group's MFMAs are issued.  One barrier per stage.  (r04's kernel read B straight
// from L2 in every wave and stored A after the MFMAs: 0.67-0.73 of the fp32 MFMA
// peak, MFMA busy 76 %; 256 x 128 tiles, one workgroup per CU: the same.)
// WN: waves along the columns (2: 2 x 2 waves of 64 x 64, 128 columns; 1: the
// layer has a single column tile -- the 4-angle output layer -- and the 4 waves
// take 32 rows x 32 columns each, so no wave multiplies 96 padding columns).
constexpr int kBM2 = 128;  // output rows per workgroup
template <int WN>
__global__ __launch_bounds__(256, 2) void annb_gemm_kernel(const float *__restrict__ A, int lda,
                                                           int64_t rows,
                                                           const f32x4 *__restrict__ wp, int G,
                                                           int NT, const float *__restrict__ bias,
                                                           int act, float *__restrict__ C,
                                                           int ldc) {
  constexpr int WM = 4 / WN;          // waves along the rows
  constexpr int MT = kBM2 / 32 / WM;  // 32-row tiles per wave
  constexpr int JT = WN == 2 ? 2 : 1; // 32-column tiles per wave
  constexpr int NTB = WN * JT;        // column tiles per workgroup
  __shared__ __attribute__((aligned(16))) float As[2][kBM2 * kLdA];  // 2 x 18 KiB
  __shared__ __attribute__((aligned(16))) f32x4 Bs[2][NTB * 4 * 64];  // 2 x NTB x 4 KiB
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;
  // XCD-aware tile order in 2-D groups: workgroups are dealt round-robin over the 8
  // XCDs (workgroup b runs on XCD b % 8), and each XCD's consecutive workgroups --
  // the ones resident together -- cover a group of BH row panels x BW column blocks
  // (BW = 8, BH = 8 for layers of >= 1024 columns), so every stage's A tile is read
  // into the XCD's L2 once for BW workgroups and every B tile once for BH of them.
  // (Panel-major order, all column blocks of two panels at a time, re-read the
  // weights from MALL for every panel pair: L2 hit 52 %.)
  const int nCB = (NT + NTB - 1) / NTB;
  const int64_t nRB = (rows + kBM2 - 1) / kBM2;
  const int BW = nCB < 8 ? nCB : 8, BH = 64 / BW, per = BH * BW;
  const int nBC = (nCB + BW - 1) / BW;
  const unsigned b = blockIdx.x, xcd = b & 7u, kx = b >> 3;
  const int64_t grp = (int64_t)(kx / (unsigned)per) * 8 + xcd;
  const int inb = (int)(kx % (unsigned)per);
  const int64_t rb = (grp / nBC) * BH + inb / BW;
  const int cb = (int)(grp % nBC) * BW + inb % BW;
  if (rb >= nRB || cb >= nCB) return;  // the grid is padded to whole groups
  const int64_t row0 = rb * kBM2;
  const int ntb = cb * NTB;  // the block's first column tile
  const int r = lane & 31, h = lane >> 5;
  f32x16 acc[MT][JT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int j = 0; j < JT; ++j) acc[m][j] = (f32x16)(0.0f);

  // Operand loads through buffer descriptors, branch-free: a load past a
  // descriptor's range returns zeros, so rows past the chunk, columns past the
  // layer and K groups past the layer read 0 with no per-load branch (which made
  // the compiler wait for every outstanding load before each LDS write, and copy
  // the accumulators between the branches' register sets: 128 moves a stage).
  // A: the panel's rows from row0 on; B: the block's column tiles from ntb on.
  const uint32_t kOOB = 0x80000000u;  // an offset past any range below
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float *>(A) + row0 * (int64_t)lda, 0,
      (int)((rows - row0 < kBM2 ? rows - row0 : kBM2) * (int64_t)lda * 4), 0x00020000);
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<f32x4 *>(wp) + (size_t)ntb * G * 64, 0,
      (int)((NT - ntb < NTB ? NT - ntb : NTB) * G * 1024), 0x00020000);
  const int nst = (G + 3) / 4;
  // A tile of stage s: 128 rows x 32 floats, 4 x 16 bytes per thread (row idx >> 3,
  // columns 4 (idx & 7) ..), zero past the row's lda floats
  auto load_a = [&](f32x4 (&ra)[4], int s) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + 256 * i;
      const int kk = s * kBK + 4 * (idx & 7);
      const uint32_t off = kk < lda ? (uint32_t)(((idx >> 3) * lda + kk) * 4) : kOOB;
      ra[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsA, off, 0, 0));
    }
  };
  // B tile of stage s: block (ntl, u) = the packed fragments of column tile ntb + ntl,
  // group 4s + u; NTB x 16 bytes per thread, lane-linear in LDS
  auto load_b = [&](f32x4 (&rbv)[NTB], int s) {
#pragma unroll
    for (int i = 0; i < NTB; ++i) {
      const int idx = tid + 256 * i;
      const int blk = idx >> 6, g = s * 4 + (blk & 3);
      const uint32_t off = g < G ? (uint32_t)((((blk >> 2) * G + g) * 64 + (idx & 63)) * 16) : kOOB;
      rbv[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsB, off, 0, 0));
    }
  };
  auto store = [&](const f32x4 (&ra)[4], const f32x4 (&rbv)[NTB], int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + 256 * i;
      *reinterpret_cast<f32x4 *>(&As[buf][(idx >> 3) * kLdA + 4 * (idx & 7)]) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < NTB; ++i) Bs[buf][tid + 256 * i] = rbv[i];
  };
  struct Frag {
    f32x4 a[MT], b[JT];
  };
  auto read_frag = [&](Frag &f, int buf, int u) {
#pragma unroll
    for (int m = 0; m < MT; ++m)
      f.a[m] = *reinterpret_cast<const f32x4 *>(
          &As[buf][(wm * MT * 32 + m * 32 + r) * kLdA + 8 * u + 4 * h]);
#pragma unroll
    for (int j = 0; j < JT; ++j) f.b[j] = Bs[buf][((wn * JT + j) * 4 + u) * 64 + lane];
  };
  auto mma = [&](const Frag &f) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int j = 0; j < JT; ++j)
#pragma unroll
        for (int m = 0; m < MT; ++m)
          acc[m][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f.a[m][q], f.b[j][q], acc[m][j], 0, 0, 0);
  };
  // stage s (reading buffer s & 1): stage s + 1's tiles (loaded two stages ago) go
  // to the other buffer, stage s + 3's loads go out into the freed registers, then
  // the stage's 4 groups with the next group's fragments read ahead (a group past
  // the layer's K multiplies zero weights)
  auto stage = [&](int s, f32x4 (&ra)[4], f32x4 (&rbv)[NTB]) {
    const int buf = s & 1;
    store(ra, rbv, buf ^ 1);  // (past the last stage: zeros, never read)
    load_b(rbv, s + 3);
    load_a(ra, s + 3);
    Frag f0, f1;
    read_frag(f0, buf, 0);
    read_frag(f1, buf, 1);
    mma(f0);
    read_frag(f0, buf, 2);
    mma(f1);
    read_frag(f1, buf, 3);
    mma(f0);
    mma(f1);
    __syncthreads();
  };
  // prologue: stage 0 into buffer 0; stage 1's loads into set 1, stage 2's into set 0
  f32x4 ra0[4], ra1[4], rb0[NTB], rb1[NTB];
  load_b(rb0, 0);
  load_a(ra0, 0);
  load_b(rb1, 1);
  load_a(ra1, 1);
  store(ra0, rb0, 0);
  load_b(rb0, 2);
  load_a(ra0, 2);
  __syncthreads();
  // even stages store set 1 (stage s + 1) and refill it with stage s + 3; odd ones
  // set 0.  Stages in pairs, both unconditional (an odd count gets a stage of zero
  // weights): a conditional second stage left the loop head's wait for the first
  // store at vmcnt(0) instead of vmcnt(8), one stage of load latency lost.
  const int nst2 = (nst + 1) & ~1;
  for (int s = 0; s < nst2; s += 2) {
    stage(s, ra1, rb1);
    stage(s + 1, ra0, rb0);
  }
  // bias (after the dot product, as Keras adds it) + activation, stored per
  // accumulator element: lane (r, h) holds column r of rows (q&3) + 8(q>>2) + 4h;
  // one store instruction writes two 128-byte row segments.  Stores through a
  // descriptor over the panel's valid rows (past it they are dropped: no per-element
  // branch), the activation chosen once per workgroup.
  const auto rsC = __builtin_amdgcn_make_buffer_rsrc(
      C + row0 * (int64_t)ldc, 0,
      (int)((rows - row0 < kBM2 ? rows - row0 : kBM2) * (int64_t)ldc * 4), 0x00020000);
  auto epilogue = [&](auto actc) {
    constexpr int ACT = decltype(actc)::value;
#pragma unroll
    for (int j = 0; j < JT; ++j) {
      const int nt = ntb + wn * JT + j;
      if (nt >= NT) continue;
      const int col = nt * 32 + r;
      const float bv = bias[col];
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int row = wm * MT * 32 + m * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
          __builtin_amdgcn_raw_buffer_store_b32(
              __builtin_bit_cast(uint32_t, act_apply(ACT, acc[m][j][q] + bv)), rsC,
              (uint32_t)((row * ldc + col) * 4), 0, 0);
        }
    }
  };
  switch (act) {
    case IK_ACT_TANH: epilogue(std::integral_constant<int, IK_ACT_TANH>{}); break;
    case IK_ACT_RELU: epilogue(std::integral_constant<int, IK_ACT_RELU>{}); break;
    case IK_ACT_SIGMOID: epilogue(std::integral_constant<int, IK_ACT_SIGMOID>{}); break;
    default: epilogue(std::integral_constant<int, IK_ACT_LINEAR>{}); break;
  }
}

// ---------------------------------------------------------------- bf16x6 ----
// The layer in the split mode (IK_ANN_BF16X6, as the fused kernel's, ik_ann.hip
// "split-bf16"): x = hi + mid + lo in bf16 (each residual exact in fp32) for both
// operands, and the six products above 2^-24 -- W.hi X.lo, W.mid X.mid, W.lo X.hi,
// W.hi X.mid, W.mid X.hi, W.hi X.hi, smallest first -- accumulated in fp32 by
// v_mfma_f32_16x16x32_bf16 (exact bf16 products): fp32-level results at 6 bf16
// MFMAs (96 cycles) per 16 x 16 x 32 block instead of 16 fp32 ones (256).
//
// Tile 256 points x 128 features, 8 waves of 64 x 64 (4 x 4 accumulators of 16 x
// 16), one workgroup per CU (two waves per SIMD).  The weights are the MFMA's A
// operand (16 features x 32 k) and the activations its B operand (32 k x 16
// points), so a lane's accumulator holds 4 consecutive features of one point: one
// 16-byte store.  Stages of 32 in K, double-buffered through LDS (activations and
// weights, three planes each, 2 x 72 KiB), one barrier per stage: the activations
// arrive fp32 from HBM and are split as they are written to LDS, the weights arrive
// split (ann_big_pack_x: [plane][K / 32][features][32] bf16).  (A 128 x 128 tile with
// one LDS buffer, two barriers a stage and two workgroups per CU: MFMA busy 58 %.)
// LDS rows of 32 bf16 (64 B), the 16-byte block kb of row r at position
// kb ^ (2 ((r >> 3) & 1)): each of ds_read_b128's four 16-lane groups ({0-3, 12-15,
// 20-27}, {4-11, 16-19, 28-31}, and the same + 32; MI355X_MICROARCH.md "LDS") then
// covers the 64 banks once when a fragment read takes 16 rows x one block, and
// ds_write_b128's 8-lane groups (banks mod 32) take 2 rows x 4 blocks without a
// conflict.  (An 80-byte row pad: 50 % of LDS-active cycles in conflicts; the
// swizzle kb ^ ((r >> 2) & 3), right for contiguous 16-lane groups: 33 %.)
__device__ __forceinline__ int xoff(int r, int kb) { return r * 32 + 8 * (kb ^ (((r >> 3) & 1) << 1)); }

struct Split3 {
  bf16x8 hi, mid, lo;
};

__device__ __forceinline__ Split3 split3(f32x4 a, f32x4 b) {
  const float x[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  u32x4 h, m, l;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f32x2 v = {x[2 * i], x[2 * i + 1]};
    const uint32_t ph = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
    const f32x2 vh = {__builtin_bit_cast(float, ph << 16),
                      __builtin_bit_cast(float, ph & 0xffff0000u)};
    const f32x2 r1 = v - vh;
    const uint32_t pm = __builtin_bit_cast(uint32_t, __builtin_convertvector(r1, bf16x2));
    const f32x2 vm = {__builtin_bit_cast(float, pm << 16),
                      __builtin_bit_cast(float, pm & 0xffff0000u)};
    const f32x2 r2 = r1 - vm;
    h[i] = ph;
    m[i] = pm;
    l[i] = __builtin_bit_cast(uint32_t, __builtin_convertvector(r2, bf16x2));
  }
  return {__builtin_bit_cast(bf16x8, h), __builtin_bit_cast(bf16x8, m),
          __builtin_bit_cast(bf16x8, l)};
}

constexpr int kBMX = 256;  // bf16x6 tile: points per workgroup
__global__ __launch_bounds__(512, 1) void annb_gemm_x6_kernel(
    const float *__restrict__ A, int lda, int64_t rows, const uint16_t *__restrict__ wx, int KG,
    int NP, const float *__restrict__ bias, int act, float *__restrict__ C, int ldc) {
  // two stages: [stage][plane][rows x 32 bf16]; 96 + 48 KiB
  __shared__ __attribute__((aligned(16))) uint16_t Xs[2][3][kBMX * 32];
  __shared__ __attribute__((aligned(16))) uint16_t Ws[2][3][128 * 32];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;  // 4 x 2 waves of 64 points x 64 features
  // the fp32 kernel's XCD-aware 2-D tile groups (128 features = 4 column tiles)
  const int NT = NP / 32;
  const int nCB = (NT + 3) / 4;
  const int64_t nRB = (rows + kBMX - 1) / kBMX;
  const int BW = nCB < 8 ? nCB : 8, BH = 64 / BW, per = BH * BW;
  const int nBC = (nCB + BW - 1) / BW;
  const unsigned b = blockIdx.x, xcd = b & 7u, kx = b >> 3;
  const int64_t grp = (int64_t)(kx / (unsigned)per) * 8 + xcd;
  const int inb = (int)(kx % (unsigned)per);
  const int64_t rb = (grp / nBC) * BH + inb / BW;
  const int cb = (int)(grp % nBC) * BW + inb % BW;
  if (rb >= nRB || cb >= nCB) return;  // the grid is padded to whole groups
  const int64_t row0 = rb * kBMX;
  const int vrows = (int)(rows - row0 < kBMX ? rows - row0 : kBMX);
  const int n0 = cb * 128;  // the block's first feature
  f32x4 acc[4][4];          // [point subtile][feature subtile]
#pragma unroll
  for (int pm = 0; pm < 4; ++pm)
#pragma unroll
    for (int fm = 0; fm < 4; ++fm) acc[pm][fm] = (f32x4)(0.0f);

  const auto rsA = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float *>(A) + row0 * (int64_t)lda, 0, (int)(vrows * (int64_t)lda * 4), 0x00020000);
  // the planes' feature rows are padded to whole 128-feature blocks (zeros), so
  // no load needs a range check: a prefetch past the last stage reads the next
  // plane's stages, the next rows or past the end (zeros), and is never read back
  const int NPp = (NP + 127) / 128 * 128;
  const auto rsW = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t *>(wx), 0, (int)((size_t)3 * KG * NPp * 64), 0x00020000);
  // stage s: activations, 8 k of point (b >> 2) at k block (b & 3) for b = tid,
  // tid + 512 (two 16-byte loads each); weights, plane i, 16 bytes of feature row
  // (tid >> 2) at k block (tid & 3)
  auto load = [&](f32x4 (&ra)[4], u32x4 (&rw)[3], int s) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int bb = tid + 512 * i, p = bb >> 2, kb = bb & 3;
      const uint32_t off = (uint32_t)((p * lda + s * 32 + 8 * kb) * 4);
      ra[2 * i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsA, off, 0, 0));
      ra[2 * i + 1] =
          __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsA, off + 16, 0, 0));
    }
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) {
      const int n = tid >> 2, kb = tid & 3;
      const uint32_t off = (uint32_t)(((((size_t)pl * KG + s) * NPp + n0 + n) * 32 + 8 * kb) * 2);
      rw[pl] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsW, off, 0, 0));
    }
  };
  auto store = [&](const f32x4 (&ra)[4], const u32x4 (&rw)[3], int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int bb = tid + 512 * i, p = bb >> 2, kb = bb & 3;
      const Split3 x = split3(ra[2 * i], ra[2 * i + 1]);
      *reinterpret_cast<bf16x8 *>(&Xs[buf][0][xoff(p, kb)]) = x.hi;
      *reinterpret_cast<bf16x8 *>(&Xs[buf][1][xoff(p, kb)]) = x.mid;
      *reinterpret_cast<bf16x8 *>(&Xs[buf][2][xoff(p, kb)]) = x.lo;
    }
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
      *reinterpret_cast<u32x4 *>(&Ws[buf][pl][xoff(tid >> 2, tid & 3)]) = rw[pl];
  };
  const int fr = lane & 15, fkb = lane >> 4;
  auto compute = [&](int buf) {
    bf16x8 xf[4][3];
#pragma unroll
    for (int pm = 0; pm < 4; ++pm)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        xf[pm][pl] =
            *reinterpret_cast<const bf16x8 *>(&Xs[buf][pl][xoff(wm * 64 + pm * 16 + fr, fkb)]);
    // the next feature subtile's weight fragments are read before this one's MFMAs
    bf16x8 wf[2][3];
    auto read_w = [&](bf16x8 (&w)[3], int fm) {
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        w[pl] = *reinterpret_cast<const bf16x8 *>(&Ws[buf][pl][xoff(wn * 64 + fm * 16 + fr, fkb)]);
    };
    read_w(wf[0], 0);
#pragma unroll
    for (int fm = 0; fm < 4; ++fm) {
      if (fm < 3) read_w(wf[(fm + 1) & 1], fm + 1);
      const bf16x8(&w)[3] = wf[fm & 1];
#pragma unroll
      for (int pm = 0; pm < 4; ++pm) {
        f32x4 c = acc[pm][fm];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], xf[pm][2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[1], xf[pm][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[2], xf[pm][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], xf[pm][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[1], xf[pm][0], c, 0, 0, 0);
        acc[pm][fm] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], xf[pm][0], c, 0, 0, 0);
      }
    }
  };
  // double-buffered stages, one barrier each: at stage s the registers hold stage
  // s + 1 (loaded a stage ago), which goes to the other buffer (last read at stage
  // s - 1, before the barrier), stage s + 2's loads go out, then stage s's MFMAs
  f32x4 ra[4];
  u32x4 rw[3];
  load(ra, rw, 0);
  store(ra, rw, 0);
  load(ra, rw, 1);
  __syncthreads();
  for (int s = 0; s < KG; ++s) {
    store(ra, rw, (s + 1) & 1);  // (past the last stage: never read)
    load(ra, rw, s + 2);
    __builtin_amdgcn_sched_barrier(0);
    compute(s & 1);
    __syncthreads();
  }
  // bias + activation: lane (fr, lane >> 4) of accumulator (pm, fm) holds features
  // 4 (lane >> 4) .. + 3 of feature subtile fm for point fr of point subtile pm
  const auto rsC = __builtin_amdgcn_make_buffer_rsrc(
      C + row0 * (int64_t)ldc, 0, (int)(vrows * (int64_t)ldc * 4), 0x00020000);
  auto epilogue = [&](auto actc) {
    constexpr int ACT = decltype(actc)::value;
#pragma unroll
    for (int fm = 0; fm < 4; ++fm) {
      const int f = n0 + wn * 64 + fm * 16;  // (NP is a multiple of 32: whole subtiles)
      if (f >= NP) continue;
      const int col = f + 4 * (lane >> 4);
      const f32x4 bv = *reinterpret_cast<const f32x4 *>(bias + col);
#pragma unroll
      for (int pm = 0; pm < 4; ++pm) {
        const int p = wm * 64 + pm * 16 + fr;
        f32x4 v;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = act_apply(ACT, acc[pm][fm][i] + bv[i]);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rsC,
                                               (uint32_t)((p * ldc + col) * 4), 0, 0);
      }
    }
  };
  switch (act) {
    case IK_ACT_TANH: epilogue(std::integral_constant<int, IK_ACT_TANH>{}); break;
    case IK_ACT_RELU: epilogue(std::integral_constant<int, IK_ACT_RELU>{}); break;
    case IK_ACT_SIGMOID: epilogue(std::integral_constant<int, IK_ACT_SIGMOID>{}); break;
    default: epilogue(std::integral_constant<int, IK_ACT_LINEAR>{}); break;
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
// (annb_gemm_kernel's buffer offsets are 32-bit: a panel's A is at most 128 rows of
// 16384 floats, 8 MiB, and a block's weights 4 tiles x 2048 groups x 1 KiB, 8 MiB)

// (host) round to nearest even, as v_cvt_pk_bf16_f32 does on the device
static uint16_t bf16_rne_h(float x) {
  uint32_t u;
  std::memcpy(&u, &x, 4);
  if ((u & 0x7f800000u) == 0x7f800000u) return (uint16_t)(u >> 16);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
static float bf16_f32_h(uint16_t h) {
  const uint32_t u = (uint32_t)h << 16;
  float x;
  std::memcpy(&x, &u, 4);
  return x;
}

size_t ann_big_x_bytes(int k, int n) {
  return (size_t)3 * ((k + 31) / 32) * ((n + 127) / 128 * 128) * 32 * 2;
}

void ann_big_pack_x(const float *W, int k, int n, void *dst) {
  const int KG = (k + 31) / 32, NP = (n + 127) / 128 * 128;  // (whole 128-feature blocks)
  uint16_t *d = static_cast<uint16_t *>(dst);
  const size_t plane = (size_t)KG * NP * 32;
  for (int g = 0; g < KG; ++g)
    for (int c = 0; c < NP; ++c)
      for (int kk = 0; kk < 32; ++kk) {
        const int kr = 32 * g + kk;
        const float x = (kr < k && c < n) ? W[(size_t)kr * n + c] : 0.0f;
        const uint16_t h = bf16_rne_h(x);
        const float r1 = x - bf16_f32_h(h);
        const uint16_t m = bf16_rne_h(r1);
        const float r2 = r1 - bf16_f32_h(m);
        const size_t at = ((size_t)g * NP + c) * 32 + kk;
        d[at] = h;
        d[plane + at] = m;
        d[2 * plane + at] = bf16_rne_h(r2);
      }
}

void launch_ann_big(const AnnBigModel &m, const RobotDev &r, const double *pts, int64_t n,
                    float *ang, double *fk_err, bool check_limits, DevStats *S, hipStream_t st,
                    float *act, int64_t chunk_rows, int xmode) {
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
    IK_LAUNCH(annb_in_kernel, dim3(g1), dim3(256), 0, st, pts, p0, rows, m.xm[0],
                       m.xm[1], m.xm[2], m.xs[0], m.xs[1], m.xs[2], r, check_limits ? 1 : 0,
                       buf[0], S);
    kt_end(st);
    int cur = 0, lda = 8;
    for (const AnnBigLayer &L : m.layers) {
      const int G = L.kp / 8, NT = L.np / 32;
      // whole groups of BH x BW tiles, a multiple of 8 groups (annb_gemm_kernel)
      const int64_t nRB = (rows + kBM2 - 1) / kBM2;
      const int ntb = NT == 1 ? 1 : 4;  // column tiles per workgroup
      const int nCB = (NT + ntb - 1) / ntb, BW = nCB < 8 ? nCB : 8, BH = 64 / BW;
      const int64_t groups = (nRB + BH - 1) / BH * ((nCB + BW - 1) / BW);
      const dim3 grid((unsigned)((groups + 7) / 8 * 8 * BH * BW));
      if (xmode != IK_ANN_FP32 && L.wx && NT > 1 && lda % 32 == 0) {
        // bf16x6 (the layer's split planes exist: a hidden layer after the first),
        // 256-row tiles of 512 threads
        const int64_t xRB = (rows + kBMX - 1) / kBMX;
        const int64_t xgroups = (xRB + BH - 1) / BH * ((nCB + BW - 1) / BW);
        const dim3 xgrid((unsigned)((xgroups + 7) / 8 * 8 * BH * BW));
        kt_begin("annb_gemm_x6_kernel", st);
        IK_LAUNCH(annb_gemm_x6_kernel, xgrid, dim3(512), 0, st, buf[cur], lda, rows,
                           L.wx, lda / 32, L.np, L.bias, L.act, buf[cur ^ 1], L.np);
        kt_end(st);
        cur ^= 1;
        lda = L.np;
        continue;
      }
      kt_begin("annb_gemm_kernel", st);
      if (NT == 1)
        IK_LAUNCH(annb_gemm_kernel<1>, grid, dim3(256), 0, st, buf[cur], lda, rows,
                           reinterpret_cast<const f32x4 *>(L.wp), G, NT, L.bias, L.act,
                           buf[cur ^ 1], L.np);
      else
        IK_LAUNCH(annb_gemm_kernel<2>, grid, dim3(256), 0, st, buf[cur], lda, rows,
                           reinterpret_cast<const f32x4 *>(L.wp), G, NT, L.bias, L.act,
                           buf[cur ^ 1], L.np);
      kt_end(st);
      cur ^= 1;
      lda = L.np;
    }
    kt_begin("annb_out_kernel", st);
    IK_LAUNCH(annb_out_kernel, dim3(g1), dim3(256), 0, st, buf[cur], lda, pts, p0, rows,
                       o, ang, fk_err, S);
    kt_end(st);
  }
}

}  // namespace ikhip
