// ik_ann.hip -- fused ANN inverse kinematics for gfx950 (fp32 MFMA).
//
// Restates ANN.predict (kinematics/ann.py:70-76) for a batch in ONE launch:
//   x = f32((p - x_mean) / x_scale)            StandardScaler.transform, float64
//   h_{l+1} = act_l(h_l @ W_l + b_l)           Keras Dense layers, ann.py:46-56
//   y = f32(f32(y * y_scale) + y_mean)         StandardScaler.inverse_transform
// plus, in the epilogue, the cli.py:54-61 FK round trip |FK(y) - p|_2 and the
// inverse.py:26-35 workspace check.
//
// Layout (DESIGN.md "ANN"): a workgroup of 4 waves owns a tile of BM = 32*MR
// points and carries it through every layer with the activations resident in
// LDS (BM x 516 fp32; the 516 stride makes the ds_read_b128 A-fragment reads
// bank-conflict free).  Each wave computes a BM x (32*NR) slab of the layer
// output with v_mfma_f32_32x32x2_f32 (exact fp32; MR x NR accumulator tiles),
// streaming its weight columns straight from L2 into registers in a
// pre-packed "MFMA fragment" order (one 1 KiB dwordx4 load per 8-deep K group
// and column tile), triple-buffered two K groups ahead.  Bias + activation are
// applied on the accumulators and written back over the tile in LDS.
//   MR = 2: 64-point tiles, 129 KiB LDS, one workgroup per CU (max weight reuse;
//           the split modes' default);
//   MR = 1: 32-point tiles, 64.5 KiB LDS, two workgroups per CU, so one
//           workgroup's barrier / epilogue overlaps the other's MFMAs (fp32 default).
// The grid is persistent: workgroups walk the point tiles.
#include <cmath>
#include <cstring>
#include <type_traits>

#include "ik_common.h"

namespace ikhip {
// The device code is compiled twice: for widths <= 512 (this TU and ik_ann_x.hip,
// namespace ann) and for widths <= 1024 (ik_ann_w.hip, IKHIP_ANN_WIDE, namespace
// annw: 1028-float rows, 32-point tiles, up to 8 column tiles per wave).  The
// inline device functions of the two builds differ (kLd), hence the namespaces.
#ifdef IKHIP_ANN_WIDE
namespace annw {
#else
namespace ann {
#endif

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#ifdef IKHIP_ANN_WIDE
constexpr int kLd = 1028;  // LDS row stride in floats (>= 1024 + 4)
constexpr bool kWide = true;
#else
constexpr int kLd = 516;   // LDS row stride in floats (>= 512 + 4)
constexpr bool kWide = false;
#endif
constexpr int kWaves = 4;  // waves per workgroup
constexpr int kHPad = 64;  // floats past the last activation row (see layer_gemm)

// Row layout of the activation tile H (LY).  0: row r at r kLd floats (kLd = 516:
// row r starts one 16-byte slot after row r - 1).  1, the bf16x6 kernel's: a stride
// of kLdX = 520 floats (130 slots, 2 mod 16) and rows 4..11 of every 16 one slot
// further, so row r starts at slot 2r + [r mod 16 in 4..11] (mod 16): rows 0-3 and
// 12-15 of a 16-row block on even slots, rows 4-11 on odd ones.  Its K loop
// (layer_gemm_x16) reads with ds_read_b128, lane (row lane & 15, k-block lane >> 4),
// in the 16-lane groups {0-3, 12-15, 20-27}, {4-11, 16-19, 28-31}, ...
// (MI355X_MICROARCH.md §LDS): a group takes rows 0-3, 12-15 of one k-block and rows
// 4-11 of the next (2 slots on), 16 distinct slots; with kLd = 516 rows r and r + 2
// of neighbouring k-blocks collided in every group (2-way, 39 % of LDS-active
// cycles in the r05 profile).  Its epilogue stores (ds_write_b128, 8-lane groups of
// 8 consecutive rows, banks mod 32 dwords = 8 slots) land on 8 distinct slots too,
// and so do the fp32 GEMM's A reads of its first and last layers.  Row offsets that
// are multiples of 16 rows add a multiple of 16 kLdX, so the per-lane bases stay
// additive.
constexpr int kLdX = kLd + 4;
template <int LY>
constexpr int ld_of() { return LY ? kLdX : kLd; }
template <int LY>
__device__ __forceinline__ int hrow(int r) {
  if constexpr (LY != 0) return r * kLdX + ((((r + 4) >> 3) & 1) << 2);
  else return r * kLd;
}

struct AnnArgs {
  AnnModelDev m;
  RobotDev r;
  const double *pts;
  int64_t n;
  float *ang;
  double *fk_err;
  int check_limits;
  DevStats *S;
  unsigned long long *dbg;  // diagnostic s_memtime stamps (ik_ctx_set_debug), normally null
  double jc[16];            // per joint {a, d, cos alpha, sin alpha} for the FK round trip
  int alpha_bad;            // some |alpha| > 2 pi: FK raises for every point (forward.py:23-25)
};

constexpr int kStampSlots = 32;  // per (tile, wave): see ann_fused_kernel
constexpr int kStampTiles = 4;
// Stamps exist only in the diagnostic build (-DIKHIP_DIAG, libikhip_diag.so):
// their pointers cost registers the production main loop does not have.
__device__ __forceinline__ void stamp(unsigned long long *p) {
#ifdef IKHIP_DIAG
  if (p) *p = __builtin_amdgcn_s_memtime();
#else
  (void)p;
#endif
}

// Activations with the hardware exp2 / reciprocal (1 ulp each).  tanh is
// 1 - 2 / (1 + e), e = exp2(2 log2(e) v): one exp, one add, one reciprocal and one
// fma per element, absolute error <= ~2.5e-7 (tests/test_gpu_parity.py
// ::test_ann_tanh_accuracy); the limits come out exactly (e = inf -> 1, e = 0 ->
// -1) and NaN propagates.  The r02 form sign(v) (1 - e') / (1 + e'), e' =
// exp2(-2 log2(e) |v|), needs a subtraction, a multiply and a sign copy more:
// tools/ubench.hip `act` measured 39.0 -> 35.5 cycles per element slot (-9 %), and
// exp2 from a degree-6 polynomial on the full-rate pipe (v_pk_fma_f32) instead of
// v_exp_f32 58.5 (+50 %: v_exp_f32 issues in 8 cycles, the polynomial's range
// reduction, six packed fmas and exponent insert in more) -- profiles/r03/ubench.
template <int ACT>
__device__ __forceinline__ float act_apply(float v) {
  if constexpr (ACT == IK_ACT_TANH) {
    const float e = __builtin_amdgcn_exp2f(2.885390081777927f * v);
    return __builtin_fmaf(-2.0f, __builtin_amdgcn_rcpf(1.0f + e), 1.0f);
  } else if constexpr (ACT == IK_ACT_RELU) {
    return fmaxf(v, 0.0f);
  } else if constexpr (ACT == IK_ACT_SIGMOID) {
    return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * v));
  } else {
    return v;
  }
}

// Two elements at once: the adds / multiplies / fmas become packed-fp32
// instructions (v_pk_mul_f32 / v_pk_add_f32 / v_pk_fma_f32).
typedef float f32x2 __attribute__((ext_vector_type(2)));
template <int ACT>
__device__ __forceinline__ f32x2 act_apply2(f32x2 v) {
  if constexpr (ACT == IK_ACT_TANH) {
    f32x2 e = v * 2.885390081777927f;
    e.x = __builtin_amdgcn_exp2f(e.x);
    e.y = __builtin_amdgcn_exp2f(e.y);
    e = 1.0f + e;
    e.x = __builtin_amdgcn_rcpf(e.x);
    e.y = __builtin_amdgcn_rcpf(e.y);
    return __builtin_elementwise_fma(e, f32x2{-2.0f, -2.0f}, f32x2{1.0f, 1.0f});
  } else {
    f32x2 t;
    t.x = act_apply<ACT>(v.x);
    t.y = act_apply<ACT>(v.y);
    return t;
  }
}

// Four pairs at once, phase by phase (see layer_store): the dependent exp / rcp
// chains of the eight elements overlap.
// pre: a power-of-two scale still to be applied to v (the fp16x3 weight
// pre-scale, 1 elsewhere); for tanh it folds into exp2's argument scale, which
// rounds the same way (pre * 2 log2(e) is exact, and v * pre would be).
template <int ACT>
__device__ __forceinline__ void act_apply2x4(f32x2 (&v)[4], float pre = 1.0f) {
  if constexpr (ACT == IK_ACT_TANH) {
    f32x2 e[4];
    const float k2 = 2.885390081777927f * pre;
#pragma unroll
    for (int k = 0; k < 4; ++k) e[k] = v[k] * k2;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      e[k].x = __builtin_amdgcn_exp2f(e[k].x);
      e[k].y = __builtin_amdgcn_exp2f(e[k].y);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) e[k] = 1.0f + e[k];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      e[k].x = __builtin_amdgcn_rcpf(e[k].x);
      e[k].y = __builtin_amdgcn_rcpf(e[k].y);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      v[k] = __builtin_elementwise_fma(e[k], f32x2{-2.0f, -2.0f}, f32x2{1.0f, 1.0f});
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = act_apply2<ACT>(v[k] * pre);
  }
}

// Operands of one 8-deep K group: A fragments of the MR 32-row tiles (LDS)
// and the B fragments of the wave's NR column tiles (global, packed).
template <int MR, int NR>
struct Frag {
  f32x4 a[MR];
  f32x4 b[NR];
};

// A wave's weight stream over one layer operand through a buffer descriptor
// (wave-uniform base and size): each load is one buffer_load_dwordx4 with the
// lane's column-tile offset in a VGPR fixed for the layer and the 1 KiB block
// index in soffset -- no per-load 64-bit address arithmetic, whose issue cost
// beside the MFMAs is what the loop overhead mostly was (DESIGN.md "ANN").
// Blocks past the operand's end read zeros (range check), so prefetches need
// no clamp; blocks past a tile's K range read the next tile, never multiplied.
template <int NR>
struct WStream {
  __amdgpu_buffer_rsrc_t rs;
  int vo[NR];
};

template <int NR>
__device__ __forceinline__ WStream<NR> make_wstream(const void *base, int bytes, int nt0,
                                                    int nt_stride, int blocks_per_tile,
                                                    int lane) {
  WStream<NR> w;
  const uint64_t bi = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)bi);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(bi >> 32));
  w.rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(((uint64_t)hi << 32) | lo),
                                           0, __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
#pragma unroll
  for (int j = 0; j < NR; ++j) w.vo[j] = ((nt0 + nt_stride * j) * blocks_per_tile * 64 + lane) * 16;
  return w;
}

template <typename T, int NR>
__device__ __forceinline__ T wload(const WStream<NR> &w, int j, int blk) {
  return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b128(w.rs, w.vo[j], blk * 1024, 0));
}

// The 4 K steps of one group: C layout, a lane owns column lane & 31 of every
// tile, rows (q & 3) + 8 (q >> 2) + 4 (lane >> 5) (layer_store_c).
template <int MR, int NR>
__device__ __forceinline__ void mma_group(const Frag<MR, NR> &f, f32x16 (&acc)[MR][NR]) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
#pragma unroll
    for (int j = 0; j < NR; ++j) {
#pragma unroll
      for (int m = 0; m < MR; ++m)
        acc[m][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f.a[m][s], f.b[j][s], acc[m][j], 0, 0, 0);
    }
  }
}

// One layer, one wave: out[BM x 32*NR] for column tiles nt0 + nt_stride*j over
// K groups [g0, g1).  A ring of kRing operand buffers: the loads of group
// g + kRing - 1 are issued before the MFMAs of group g (scheduling barriers
// keep the compiler from sinking them), so kRing - 1 groups of MFMA (2 k
// cycles each at MR = 2, NR = 4) cover the L2 / Infinity-cache latency of the
// weight stream.  kRing = 4 measured 3.4 % faster than 3 (the 3 % of weight
// reads that miss the XCD's L2 outlast two groups) and, at MR = 2, allocates
// without the spills the 3-deep ring had.
#ifndef IKHIP_ANN_RING
#define IKHIP_ANN_RING 4
#endif
constexpr int kRing = IKHIP_ANN_RING;

template <int MR, int NR, int LY = 0>
__device__ __forceinline__ void layer_gemm(const float *H, const f32x4 *__restrict__ wp, int G,
                                           int wbytes, int g0, int g1, int nt0, int nt_stride,
                                           int lane, f32x16 (&acc)[MR][NR],
                                           unsigned long long *st_first = nullptr) {
  const int r = lane & 31, h = lane >> 5;
  const float *ap = H + hrow<LY>(r) + 4 * h;
#pragma unroll
  for (int j = 0; j < NR; ++j)
#pragma unroll
    for (int m = 0; m < MR; ++m) acc[m][j] = (f32x16)(0.0f);
  if (g1 <= g0) return;
  Frag<MR, NR> f[kRing];
  const WStream<NR> ws = make_wstream<NR>(wp, wbytes, nt0, nt_stride, G, lane);
  auto load_b = [&](Frag<MR, NR> &fr, int gbase, int u) {
#pragma unroll
    for (int j = 0; j < NR; ++j) fr.b[j] = wload<f32x4>(ws, j, gbase + u);
  };
  // A fragments: one base address per ring pass, the slot in the ds_read
  // immediate offset.  Reads run up to kRing - 1 groups past the K range
  // (into the next row, or the pad at the end of H), never multiplied.
  auto load_a = [&](Frag<MR, NR> &fr, const float *a0, int u) {
#pragma unroll
    for (int m = 0; m < MR; ++m)
      fr.a[m] = *reinterpret_cast<const f32x4 *>(a0 + m * 32 * ld_of<LY>() + 8 * u);
  };
#pragma unroll
  for (int u = 0; u < kRing - 1; ++u) {  // group by group, as the loop issues them
    load_a(f[u], ap + 8 * g0, u);
    load_b(f[u], g0, u);
    __builtin_amdgcn_sched_barrier(0);
  }
  int g = g0;
  for (; g + kRing <= g1; g += kRing) {
    const float *a0 = ap + 8 * (g + kRing - 1);
#pragma unroll
    for (int u = 0; u < kRing; ++u) {
      load_a(f[(u + kRing - 1) % kRing], a0, u);
      load_b(f[(u + kRing - 1) % kRing], g + kRing - 1, u);
      __builtin_amdgcn_sched_barrier(0);
      mma_group<MR, NR>(f[u], acc);
      __builtin_amdgcn_sched_barrier(0);
      if (u == 0 && g == g0) stamp(st_first);  // diagnostic: first K group done
    }
  }
#pragma unroll
  for (int u = 0; u < kRing - 1; ++u)
    if (g + u < g1) mma_group<MR, NR>(f[u], acc);
}

// fp16x3 activation planes.  A layer whose successor runs in fp16x3 stores its
// activations already split, x = hi + lo in fp16 (the residual exact in fp32),
// row r of H holding the 512 hi halves in bytes [0, 1024) and the 512 lo halves
// in [1024, 2048) of its 2064: the next layer's K loop then reads its operands
// with no conversion, and each activation is split once by the wave that wrote it
// instead of once by every wave that reads it (4x), in the MFMA loop.
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ _Float16 *hplane(float *H, int row) {
  return reinterpret_cast<_Float16 *>(H + row * kLd);
}

// Plane swizzle: rows 4..11 of every 16 hold their 16-byte k-blocks
// pairwise swapped (half index col ^ 8).  The 16x16x32 loop's ds_read_b128 of a K step
// (lane: row lane & 15, k-block lane >> 4; kLd = 516 floats puts row r one 16-byte slot
// after row r - 1) then lands each of the instruction's four 16-lane bank groups on 16
// distinct slots; unswizzled, every group has one 2-way collision (rows 11 and 12 of
// consecutive k-blocks), i.e. 8 LDS cycles instead of 4 (SQ_LDS_BANK_CONFLICT = 47 % of
// SQ_LDS_IDX_ACTIVE in the r04 fp16x3 profile).  Writers (store_h4 / store_h1) and
// readers apply the same XOR; it touches only bit 3 of the half index, so K-step and
// row-group offsets (multiples of 16 halves / 16 rows) pass through unchanged.
__device__ __forceinline__ int hswz(int row) { return (((row + 4) >> 3) & 1) << 3; }

__device__ __forceinline__ void store_h4(float *H, int row, int col, f32x4 v) {
  const f32x2 v01 = {v[0], v[1]}, v23 = {v[2], v[3]};
  const f16x2 h01 = __builtin_convertvector(v01, f16x2), h23 = __builtin_convertvector(v23, f16x2);
  const f16x2 l01 = __builtin_convertvector(v01 - __builtin_convertvector(h01, f32x2), f16x2);
  const f16x2 l23 = __builtin_convertvector(v23 - __builtin_convertvector(h23, f32x2), f16x2);
  _Float16 *p = hplane(H, row) + (col ^ hswz(row));
  *reinterpret_cast<f16x4 *>(p) = f16x4{h01[0], h01[1], h23[0], h23[1]};
  *reinterpret_cast<f16x4 *>(p + 512) = f16x4{l01[0], l01[1], l23[0], l23[1]};
}

__device__ __forceinline__ void store_h1(float *H, int row, int col, float v) {
  const _Float16 h = (_Float16)v;
  _Float16 *p = hplane(H, row) + (col ^ hswz(row));
  p[0] = h;
  p[512] = (_Float16)(v - (float)h);
}

// Epilogue of a full-width fp32 layer (C layout: column lane & 31, rows
// (q & 3) + 8 (q >> 2) + 4 (lane >> 5)).  bv[j]: the bias of the lane's column
// in tile j, loaded before the GEMM (a load issued here, after the barrier,
// would put a memory round trip on every layer's critical path).  The
// transposed form below (bias in the accumulators, b128 stores) measured
// 0.6 k cycles per layer slower here: its 5.9 k-cycle epilogue saves 0.7 k,
// its GEMM loses 1.3 k (bias loads ahead of the first MFMA).
// HOUT: 0 fp32 rows (in the LY layout), 1 fp16x3 split planes.
template <int MR, int NR, int ACT, int HOUT = 0, int W = kWaves, int LY = 0>
__device__ __forceinline__ void layer_store_c(float *H, const float (&bv)[NR], int wave, int lane,
                                              f32x16 (&acc)[MR][NR], unsigned long long *st) {
  const int r = lane & 31, h = lane >> 5;
  stamp(st);
  __syncthreads();  // every wave has finished reading the layer input
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const int col = (wave + W * j) * 32 + r;
#pragma unroll
    for (int m = 0; m < MR; ++m)
#pragma unroll
      for (int q0 = 0; q0 < 16; q0 += 8) {
        f32x2 t[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          t[k] = f32x2{acc[m][j][q0 + 2 * k], acc[m][j][q0 + 2 * k + 1]} + bv[j];
        act_apply2x4<ACT>(t);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int q = q0 + 2 * k;
          const int row = m * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;  // row of q + 1 is row + 1
          if constexpr (HOUT == 1) {
            store_h1(H, row, col, t[k].x);
            store_h1(H, row + 1, col, t[k].y);
          } else {
            H[hrow<LY>(row) + col] = t[k].x;
            H[hrow<LY>(row + 1) + col] = t[k].y;
          }
        }
      }
  }
}

// ------------------------------------------------ split-bf16 (bf16x6) mode ----
// Opt-in (IK_ANN_MODE_BF16X6): fp32 operands are split into three bf16 parts,
// x = hi + mid + lo (each residual exact in fp32), and the six products whose
// order is above 2^-24 -- lo*hi, mid*mid, hi*lo, mid*hi, hi*mid, hi*hi -- are
// accumulated in fp32 by v_mfma_f32_16x16x32_bf16 (exact bf16 products;
// layer_gemm_x16 below).  The result is fp32-accurate (max |d| vs a float64
// forward ~1e-7 on the reference architecture, tests/test_gpu_parity.py) at 6
// bf16 MFMAs per 32x32x16 block of work instead of 8 fp32 ones (192 against 512
// cycles).  Weights are split on
// the host into three fragment-ordered planes; activations are split in VALU
// as they are read from LDS, in the MFMA issue gaps.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct Split3 {
  bf16x8 hi, mid, lo;
};

__device__ __forceinline__ Split3 split3(f32x8 x) {
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
  Split3 s;
  s.hi = __builtin_bit_cast(bf16x8, h);
  s.mid = __builtin_bit_cast(bf16x8, m);
  s.lo = __builtin_bit_cast(bf16x8, l);
  return s;
}

// Compile-time loop: f(std::integral_constant<int, 0>) .. f(<N - 1>).
template <int I, int N, typename F>
__device__ __forceinline__ void static_for_(F &&f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for_<I + 1, N>(f);
  }
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F &&f) {
  static_for_<0, N>(f);
}

// ------------------------------------------------- split-fp16 (fp16x3) mode ----
// Opt-in (IK_ANN_FP16X3): x = hi + lo in fp16 (round to nearest; the residual
// is exact in fp32), weights pre-scaled by 2^k so their largest is ~2^14, and
// the three products above 2^-22 -- lo*hi, hi*lo, hi*hi -- accumulated in fp32
// by v_mfma_f32_16x16x32_f16 (layer_gemm_h16); fp16 products are exact in fp32.  The result is scaled back by 2^-k (exact).  3 MFMAs (96
// cycles) per 32x32x16 block against 6 for bf16x6 and 8 fp32 ones (512
// cycles), 4 B per weight from L2.  Only for
// layers whose input is bounded (the layer before is tanh or sigmoid): fp16's
// range ends at 65504.  Accuracy on the reference architecture: max |d| to a
// float64 forward 3.6e-7, the same as numpy's float32 forward (test_gpu_parity).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

struct Split2 {
  f16x8 hi, lo;
};

// fp16x3 on v_mfma_f32_16x16x32_f16.  The same products and cycles per FLOP as
// the 32x32x16 shape (r01-r03's loop, history §3), but the chip holds a higher
// clock under the power cap on the 16x16 shape (MI355X_MICROARCH.md, "Shape").  A wave's 32x32 tile (m, j) is four 16x16 sub-tiles s = 2 fh + ph
// (feature half fh, point half ph), each in elements [4s, 4s + 4) of the f32x16
// accumulator: lane l holds point 16 ph + (l & 15), features 32 nt + 16 fh +
// 4 (l >> 4) + 0..3.  One K step is 32 deep: weights of plane p, feature half
// fh at block ((g * 2 + fh) * 2 + p) of the tile (ann_pack_layer_h), and the
// activations one ds_read_b128 per plane and point half.
// weight-step buffers of the 16x16x32 loop (kH16Ring - 1 steps of 32 ahead)
#ifndef IKHIP_ANN_H16_RING
#define IKHIP_ANN_H16_RING 2
#endif
constexpr int kH16Ring = IKHIP_ANN_H16_RING;

template <int NR>
struct WStepH16 {
  f16x8 p[NR][2][2];  // [tile][feature half][plane]
};

template <int NR>
__device__ __forceinline__ void load_wh16(WStepH16<NR> &w, const WStream<NR> &ws, int g) {
#pragma unroll
  for (int j = 0; j < NR; ++j)
#pragma unroll
    for (int fh = 0; fh < 2; ++fh)
#pragma unroll
      for (int p = 0; p < 2; ++p)
        w.p[j][fh][p] = wload<f16x8>(ws, j, g * 4 + fh * 2 + p);
}

// lane l: point 16 ph + (l & 15) of row group m, k 32 g + 8 (l >> 4) + 0..7
template <int MR>
__device__ __forceinline__ void load_ah16(Split2 (&a)[MR][2], const _Float16 *ap, int g) {
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) {
      const _Float16 *q = ap + (m * 32 + 16 * ph) * 2 * kLd + 32 * g;
      a[m][ph].hi = *reinterpret_cast<const f16x8 *>(q);
      a[m][ph].lo = *reinterpret_cast<const f16x8 *>(q + 512);
    }
}

template <int MR, int NR, int GI>
__device__ __forceinline__ void step_h16(Split2 (&sa)[MR][2], const WStepH16<NR> &w,
                                         WStepH16<NR> &fill, const WStream<NR> &ws,
                                         const _Float16 *ab, int g, f32x4 (&acc)[MR][NR][4]) {
  __builtin_amdgcn_sched_barrier(0);
  load_wh16(fill, ws, g + kH16Ring - 1);
  Split2 sn[MR][2];
  load_ah16(sn, ab, GI + 1);  // step g + 1; ab is the pass base (step g - GI)
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int j = 0; j < NR; ++j)
#pragma unroll
      for (int fh = 0; fh < 2; ++fh)
#pragma unroll
        for (int ph = 0; ph < 2; ++ph) {
          f32x4 c = acc[m][j][2 * fh + ph];
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(w.p[j][fh][0], sa[m][ph].lo, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(w.p[j][fh][1], sa[m][ph].hi, c, 0, 0, 0);
          acc[m][j][2 * fh + ph] =
              __builtin_amdgcn_mfma_f32_16x16x32_f16(w.p[j][fh][0], sa[m][ph].hi, c, 0, 0, 0);
        }
  // one weight load, one LDS read per two MFMAs from the start of the step (with
  // 4 waves: 13.49 ms against 13.65 for 8 waves in the compiler's order, 13.82 for
  // 4 waves in it, 13.88 with the loads first)
#pragma unroll
  for (int i = 0; i < 4 * NR; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    if (i < 4 * MR) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) sa[m][ph] = sn[m][ph];
}

template <int MR, int NR, int W = kWaves>
__device__ __forceinline__ void layer_gemm_h16(const float *H, const f16x8 *__restrict__ wx,
                                               int G32, int xbytes, float xinv, int wave, int lane,
                                               const float *bias, f32x16 (&acc)[MR][NR],
                                               unsigned long long *st_first = nullptr) {
  const _Float16 *ap =
      hplane(const_cast<float *>(H), lane & 15) + ((8 * (lane >> 4)) ^ hswz(lane & 15));
  // the bias loads go out before the first weight step's: vmcnt counts in issue
  // order, so the accumulators' start (bias x scale) then waits for the bias
  // alone and the first MFMAs for their own weight blocks, not for all of the
  // step's
  f32x4 bl[NR][2];
#pragma unroll
  for (int j = 0; j < NR; ++j)
#pragma unroll
    for (int fh = 0; fh < 2; ++fh)
      bl[j][fh] = *reinterpret_cast<const f32x4 *>(bias + (wave + W * j) * 32 + 16 * fh +
                                                   4 * (lane >> 4));
  __builtin_amdgcn_sched_barrier(0);
  const WStream<NR> ws = make_wstream<NR>(wx, xbytes, wave, W, G32 * 4, lane);
  WStepH16<NR> w[kH16Ring];
#pragma unroll
  for (int u = 0; u < kH16Ring - 1; ++u) load_wh16(w[u], ws, u);
  f32x4 c4[MR][NR][4];
  const float scale = 1.0f / xinv;  // exact: xinv is 2^-k
#pragma unroll
  for (int j = 0; j < NR; ++j)
#pragma unroll
    for (int fh = 0; fh < 2; ++fh) {
      const f32x4 b = bl[j][fh] * scale;
#pragma unroll
      for (int m = 0; m < MR; ++m) c4[m][j][2 * fh] = c4[m][j][2 * fh + 1] = b;
    }
  Split2 sa[MR][2];
  load_ah16(sa, ap, 0);
  int g = 0;
  for (; g + kH16Ring <= G32; g += kH16Ring) {
    const _Float16 *ab = ap + 32 * g;
    static_for<kH16Ring>([&](auto u) {
      step_h16<MR, NR, u.value>(sa, w[u.value], w[(u.value + kH16Ring - 1) % kH16Ring], ws, ab,
                                g + u.value, c4);
      if (u.value == 0 && g == 0) stamp(st_first);  // diagnostic: first K step done
    });
  }
  const _Float16 *ab = ap + 32 * g;
  static_for<kH16Ring - 1>([&](auto u) {
    if (g + u.value < G32)
      step_h16<MR, NR, u.value>(sa, w[u.value], w[(u.value + kH16Ring - 1) % kH16Ring], ws, ab,
                                g + u.value, c4);
  });
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int j = 0; j < NR; ++j)
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[m][j][4 * s + i] = c4[m][j][s][i];
  (void)xinv;  // the epilogue applies it (layer_store_h16's pre)
}

// Epilogue of an fp16x3 layer in the 16x16 sub-tile layout above: per lane and
// sub-tile four consecutive features of one point, one 8-byte store per plane
// (or one ds_write_b128 of fp32).
template <int MR, int NR, int ACT, int HOUT = 0, int W = kWaves, int LY = 0>
__device__ __forceinline__ void layer_store_h16(float *H, int wave, int lane,
                                                f32x16 (&acc)[MR][NR], unsigned long long *st,
                                                float pre = 1.0f) {
  stamp(st);
  __syncthreads();  // every wave has finished reading the layer input
#pragma unroll
  for (int j = 0; j < NR; ++j)
#pragma unroll
    for (int fh = 0; fh < 2; ++fh) {
      const int col = (wave + W * j) * 32 + 16 * fh + 4 * (lane >> 4);
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        f32x2 t[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int q = 4 * (2 * fh + (k >> 1)) + 2 * (k & 1);
          t[k] = f32x2{acc[m][j][q], acc[m][j][q + 1]};
        }
        act_apply2x4<ACT>(t, pre);
#pragma unroll
        for (int ph = 0; ph < 2; ++ph) {
          const int row = m * 32 + 16 * ph + (lane & 15);
          const f32x4 v = {t[2 * ph].x, t[2 * ph].y, t[2 * ph + 1].x, t[2 * ph + 1].y};
          if constexpr (HOUT == 1) store_h4(H, row, col, v);
          else *reinterpret_cast<f32x4 *>(H + hrow<LY>(row) + col) = v;
        }
      }
    }
}

// bf16x6 on v_mfma_f32_16x16x32_bf16: the same six products in
// the 16x16 sub-tile layout of layer_gemm_h16 (epilogue layer_store_h16), the
// activations split in VALU as they are read: lane l reads point 16 ph + (l & 15)
// of row group m, k 32 g + 8 (l >> 4) + 0..7 (two ds_read_b128).  Weights: plane p
// of feature half fh at block ((g * 2 + fh) * 3 + p) of the tile (ann_pack_layer_x).
// Same box: 26.26 -> 24.12 ms per 1M points with the loads first (pattern 1, 40
// VGPRs spilled outside the loop); 25.18 in the compiler's order (0, no spills);
// weight loads spread: 23.5 against 23.1 with them first on another box.

template <int NR>
struct WStepX16 {
  bf16x8 p[NR][2][3];  // [tile][feature half][plane]
};

template <int NR>
__device__ __forceinline__ void load_wx16(WStepX16<NR> &w, const WStream<NR> &ws, int g) {
#pragma unroll
  for (int j = 0; j < NR; ++j)
#pragma unroll
    for (int fh = 0; fh < 2; ++fh)
#pragma unroll
      for (int p = 0; p < 3; ++p) w.p[j][fh][p] = wload<bf16x8>(ws, j, (g * 2 + fh) * 3 + p);
}

template <int MR>
__device__ __forceinline__ void load_ax16(f32x8 (&a)[MR][2], const float *ap, int g) {
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) {
      const f32x4 *q = reinterpret_cast<const f32x4 *>(ap + (m * 32 + 16 * ph) * kLdX + 32 * g);
      const f32x4 lo4 = q[0], hi4 = q[1];
      a[m][ph] = f32x8{lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
    }
}

template <int MR, int NR, int GI>
__device__ __forceinline__ void step_x16(Split3 (&sa)[MR][2], const WStepX16<NR> &w,
                                         WStepX16<NR> &fill, const WStream<NR> &ws,
                                         const float *ab, int g, f32x4 (&acc)[MR][NR][4]) {
  __builtin_amdgcn_sched_barrier(0);
  load_wx16(fill, ws, g + 1);
  f32x8 an[MR][2];
  load_ax16(an, ab, GI + 1);  // step g + 1; ab is the pass base (step g - GI)
  Split3 sn[MR][2];
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) sn[m][ph] = split3(an[m][ph]);
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int j = 0; j < NR; ++j)
#pragma unroll
      for (int fh = 0; fh < 2; ++fh)
#pragma unroll
        for (int ph = 0; ph < 2; ++ph) {
          const bf16x8 *wp = w.p[j][fh];
          const Split3 &x = sa[m][ph];
          f32x4 c = acc[m][j][2 * fh + ph];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wp[0], x.lo, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wp[1], x.mid, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wp[2], x.hi, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wp[0], x.mid, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wp[1], x.hi, c, 0, 0, 0);
          acc[m][j][2 * fh + ph] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wp[0], x.hi, c, 0, 0, 0);
        }
  // the loads, a few MFMAs to cover the LDS latency, then the split VALU two
  // instructions per MFMA gap
  constexpr int kMfma = 24 * MR * NR, kLead = 6;
  __builtin_amdgcn_sched_group_barrier(0x020, 6 * NR, 0);  // VMEM reads, all first
  __builtin_amdgcn_sched_group_barrier(0x100, 4 * MR, 0);  // DS reads
  __builtin_amdgcn_sched_group_barrier(0x008, kLead, 0);   // MFMA
#pragma unroll
  for (int i = 0; i < kMfma - kLead; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);  // VALU
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) sa[m][ph] = sn[m][ph];
}

template <int MR, int NR, int W = kWaves>
__device__ __forceinline__ void layer_gemm_x16(const float *H, const bf16x8 *__restrict__ wx,
                                               int G32, int xbytes, int wave, int lane,
                                               const float *bias, f32x16 (&acc)[MR][NR]) {
  // (the bf16x6 kernel's tile layout, LY 1)
  const float *ap = H + hrow<1>(lane & 15) + 8 * (lane >> 4);
  f32x4 bl[NR][2];  // before the weights (layer_gemm_h16)
#pragma unroll
  for (int j = 0; j < NR; ++j)
#pragma unroll
    for (int fh = 0; fh < 2; ++fh)
      bl[j][fh] = *reinterpret_cast<const f32x4 *>(bias + (wave + W * j) * 32 + 16 * fh +
                                                   4 * (lane >> 4));
  __builtin_amdgcn_sched_barrier(0);
  const WStream<NR> ws = make_wstream<NR>(wx, xbytes, wave, W, G32 * 6, lane);
  WStepX16<NR> w[2];
  load_wx16(w[0], ws, 0);
  f32x4 c4[MR][NR][4];
#pragma unroll
  for (int j = 0; j < NR; ++j)
#pragma unroll
    for (int fh = 0; fh < 2; ++fh) {
      const f32x4 b = bl[j][fh];
#pragma unroll
      for (int m = 0; m < MR; ++m) c4[m][j][2 * fh] = c4[m][j][2 * fh + 1] = b;
    }
  Split3 sa[MR][2];
  {
    f32x8 a0[MR][2];
    load_ax16(a0, ap, 0);
#pragma unroll
    for (int m = 0; m < MR; ++m)
#pragma unroll
      for (int ph = 0; ph < 2; ++ph) sa[m][ph] = split3(a0[m][ph]);
  }
  int g = 0;
  for (; g + 2 <= G32; g += 2) {
    const float *ab = ap + 32 * g;
    step_x16<MR, NR, 0>(sa, w[0], w[1], ws, ab, g, c4);
    step_x16<MR, NR, 1>(sa, w[1], w[0], ws, ab, g + 1, c4);
  }
  if (g < G32) step_x16<MR, NR, 0>(sa, w[0], w[1], ws, ap + 32 * g, g, c4);
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int j = 0; j < NR; ++j)
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[m][j][4 * s + i] = c4[m][j][s][i];
}

// One Dense layer for a wave with NR column tiles.  X: 0 fp32, 1 bf16x6,
// 2 fp16x3; wx: the layer's split weight operand in that mode, or nullptr for
// a layer that stays fp32.  HX: the kernel runs fp16x3 layers, so hout (the next
// layer is one) stores the activations as split planes.
template <int ACT, int HOUT, int W, int X, int LY, int MR, int NR>
__device__ __forceinline__ void store_any(bool tr, float *H, const float (&bv)[NR], int wave,
                                          int lane, f32x16 (&acc)[MR][NR],
                                          unsigned long long *st, float pre) {
  if (tr) {
    if constexpr (X != 0) layer_store_h16<MR, NR, ACT, HOUT, W, LY>(H, wave, lane, acc, st, pre);
  } else {
    layer_store_c<MR, NR, ACT, HOUT, W, LY>(H, bv, wave, lane, acc, st);
  }
}

// pre: the fp16x3 16x16x32 GEMM's accumulators still carry the weight pre-scale
// (layer_gemm_h16); 1 for every other layer.
template <int HOUT, int W, int X, int LY, int MR, int NR>
__device__ __forceinline__ void store_act(int act, bool tr, float *H, const float (&bv)[NR],
                                          int wave, int lane, f32x16 (&acc)[MR][NR],
                                          unsigned long long *st, float pre = 1.0f) {
  switch (act) {
    case IK_ACT_TANH: store_any<IK_ACT_TANH, HOUT, W, X, LY>(tr, H, bv, wave, lane, acc, st, pre); break;
    case IK_ACT_RELU: store_any<IK_ACT_RELU, HOUT, W, X, LY>(tr, H, bv, wave, lane, acc, st, pre); break;
    case IK_ACT_SIGMOID: store_any<IK_ACT_SIGMOID, HOUT, W, X, LY>(tr, H, bv, wave, lane, acc, st, pre); break;
    default: store_any<IK_ACT_LINEAR, HOUT, W, X, LY>(tr, H, bv, wave, lane, acc, st, pre); break;
  }
}

template <int MR, int NR, int X = 0, int HX = 0, int W = kWaves, int LY = 0>
__device__ __forceinline__ void run_layer(float *H, const f32x4 *wp, const float *bias, int act,
                                          int G, int wbytes, int wave, int lane, unsigned long long *st,
                                          unsigned long long *st_first,
                                          const void *wx = nullptr, int G32 = 0,
                                          float xinv = 1.0f, bool hout = false) {
  f32x16 acc[MR][NR];
  const int NT = wbytes / (G * 1024);  // column tiles of the layer
  float bv[NR];
  const bool tr = X != 0 && wx;  // split GEMM: transposed tile, bias in the accumulators
  if (tr) {
    if (X == 1)  // G32: 32-deep K steps
      layer_gemm_x16<MR, NR, W>(H, static_cast<const bf16x8 *>(wx), G32, NT * G32 * 6 * 1024,
                                wave, lane, bias, acc);
    else
      layer_gemm_h16<MR, NR, W>(H, static_cast<const f16x8 *>(wx), G32, NT * G32 * 4 * 1024,
                                xinv, wave, lane, bias, acc, st_first);
  } else {
#pragma unroll
    for (int j = 0; j < NR; ++j) bv[j] = bias[(wave + W * j) * 32 + (lane & 31)];
    layer_gemm<MR, NR, LY>(H, wp, G, wbytes, 0, G, wave, W, lane, acc, st_first);
  }
  const float pre = (X == 2 && tr) ? xinv : 1.0f;
  if (HX && hout) store_act<HX, W, X, LY>(act, tr, H, bv, wave, lane, acc, st, pre);
  else store_act<0, W, X, LY>(act, tr, H, bv, wave, lane, acc, st, pre);
}

// HOUT 1: the next layer runs fp16x3, so the result goes out as split planes
// (bytes [0, 64) and [1024, 1088) of the row: clear of the partials at floats
// 32..159, which other threads of the block are still reading).
template <int BM, int ACT, int HOUT = 0, int W = kWaves, int LY = 0>
__device__ __forceinline__ void splitk_finish(float *H, const float *__restrict__ bias, int tid) {
  for (int o = tid; o < BM * 32; o += W * 64) {
    const int row = o >> 5, col = o & 31;
    const float *p = H + hrow<LY>(row) + 32 + col;
    float v = ((p[0] + p[32]) + p[64]) + p[96];  // fixed order: deterministic
    const float y = act_apply<ACT>(v + bias[col]);
    if constexpr (HOUT == 1) store_h1(H, row, col, y);
    else H[hrow<LY>(row) + col] = y;
  }
}

// A layer with a single 32-column output tile (e.g. the 4-angle output layer,
// ann.py:56): the K range is split over the 4 waves, the partial BM x 32 tiles
// go to LDS columns 32..159 (never read by this or the next layer) and are
// summed in a fixed order, so no wave idles.
template <int MR, int HX = 0, int W = kWaves, int LY = 0>
__device__ __forceinline__ void run_layer_splitk(float *H, const f32x4 *wp, const float *bias,
                                                 int act, int G, int wave, int lane, int tid,
                                                 unsigned long long *st, bool hout = false) {
  constexpr int BM = 32 * MR;
  f32x16 acc[MR][1];
  // K split over the first four waves (their partials fill columns 32..159; any
  // further waves only join the barriers)
  const int ws = wave < 4 ? wave : 4;
  const int g0 = (G * ws) / 4, g1 = wave < 4 ? (G * (wave + 1)) / 4 : g0;
  layer_gemm<MR, 1, LY>(H, wp, G, G * 1024, g0, g1, 0, 0, lane, acc);
  stamp(st);
  __syncthreads();
  const int r = lane & 31, h = lane >> 5;
  if (wave < 4)
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int row = m * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
      H[hrow<LY>(row) + 32 + wave * 32 + r] = acc[m][0][q];
    }
  __syncthreads();
  switch (act) {
    case IK_ACT_TANH:
      if (HX && hout) splitk_finish<BM, IK_ACT_TANH, HX, W, LY>(H, bias, tid);
      else splitk_finish<BM, IK_ACT_TANH, 0, W, LY>(H, bias, tid);
      break;
    case IK_ACT_RELU:
      if (HX && hout) splitk_finish<BM, IK_ACT_RELU, HX, W, LY>(H, bias, tid);
      else splitk_finish<BM, IK_ACT_RELU, 0, W, LY>(H, bias, tid);
      break;
    case IK_ACT_SIGMOID:
      if (HX && hout) splitk_finish<BM, IK_ACT_SIGMOID, HX, W, LY>(H, bias, tid);
      else splitk_finish<BM, IK_ACT_SIGMOID, 0, W, LY>(H, bias, tid);
      break;
    default:
      if (HX && hout) splitk_finish<BM, IK_ACT_LINEAR, HX, W, LY>(H, bias, tid);
      else splitk_finish<BM, IK_ACT_LINEAR, 0, W, LY>(H, bias, tid);
      break;
  }
}

// X: 0 fp32; 1 bf16x6, 2 fp16x3 -- layers whose split weight operand exists
// (a.m.wx[l]) take the split GEMM; the others (input layer, split-K output
// layer, fp16x3-ineligible layers) stay fp32.
// Waves per workgroup: 4, one per SIMD (NR column tiles each, 4 at full width).
// IKHIP_ANN_XWAVES for the fp16x3 kernel at 64-point tiles: 4 (its loads spread
// over the MFMAs: 13.34 against 13.59 ms for 8).
#ifndef IKHIP_ANN_BWAVES  // bf16x6: 8 waves measured 27.5 vs 25.6 ms (27 VGPR spills)
#define IKHIP_ANN_BWAVES 4
#endif
#ifndef IKHIP_ANN_FWAVES  // fp32 at 64-point tiles (IKHIP_ANN_MR=2): 8 waves 40.9 ms, 4 41.6, MR=1 40.2
#define IKHIP_ANN_FWAVES 4
#endif
#ifndef IKHIP_ANN_XWAVES
#define IKHIP_ANN_XWAVES 4
#endif
template <int MR, int X>
constexpr int ann_waves() {
  return (X == 2 && MR == 2)   ? IKHIP_ANN_XWAVES
         : (X == 1 && MR == 2) ? IKHIP_ANN_BWAVES
         : (X == 0 && MR == 2 && !kWide) ? IKHIP_ANN_FWAVES
                                         : kWaves;
}

// Tiles after the first are claimed from a launch-wide counter (a static stride
// ends on the slowest workgroup's share: 0.7 % slower, profiles/r04/ab/
// ann_dyn_traffic.txt).  The claim is issued by the workgroup's last wave after
// the tile's last GEMM, when that wave has no memory wait left in the tile (point
// I/O is wave 0's), so the atomic's latency hides under the output epilogue.
// Issued by thread 0 at the tile's start instead (r02-r03), its returning atomic
// was older than wave 0's first weight loads and vmcnt (counted in issue order)
// made them wait for it: same box, bit-identical, 39.44 -> 39.17 ms, HBM traffic
// 33.6 -> 23.2 GB per launch, L2 hit 80.7 -> 86.2 % (profiles/r04/ab/ann_claim_late.txt).
template <int MR, int X>
__global__ __launch_bounds__((64 * ann_waves<MR, X>()), (MR == 2 || kWide) ? 1 : 2) void
ann_fused_kernel(AnnArgs a) {
  constexpr int BM = 32 * MR;
  constexpr int W = ann_waves<MR, X>();
  // how a layer stores activations its split-GEMM successor reads (HOUT: fp16x3
  // planes), and the tile's row layout (LY 1 for bf16x6)
  constexpr int HK = X == 2 ? 1 : 0;
  constexpr int LY = X == 1 ? 1 : 0;
  // + kHPad: the fp32 GEMM's operand ring reads up to 3 K groups past a row's end
  __shared__ __attribute__((aligned(16))) float H[BM * ld_of<LY>() + kHPad];
  const int tid = threadIdx.x;
  // wave index in an SGPR: the per-wave column-tile count (cnt) and the paths it
  // selects are uniform branches, not exec-masked regions
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int64_t ntiles = (a.n + BM - 1) / BM;
  double blk_max = 0.0, blk_sum = 0.0;  // FK round-trip error of this lane's points

  // tiles after the first are claimed from a launch-wide counter (DevStats heads[0],
  // zeroed by the stats reset before every solve): a workgroup that runs faster
  // (an XCD at a higher clock, a CU whose partner workgroup has finished) takes more
  // tiles, so the launch does not end on the slowest workgroup's static share.  Two
  // slots, so the next claim never overwrites the one the others are still reading.
  __shared__ long long next_tile[2];
  unsigned long long *const tile_ctr = &a.S->heads[0][0];
  int64_t it_local = 0;  // this workgroup's tile counter
  for (int64_t tile = blockIdx.x; tile < ntiles; ++it_local) {
    const int64_t pt = tile * BM + tid;
    // diagnostic stamps (block 0, first tiles, lane 0 of each wave): slot 0 tile
    // start, 1 staged, 2+2l layer l GEMM done, 3+2l layer l done, 31 tile done
    unsigned long long *stp = nullptr;
    if (a.dbg && blockIdx.x == 0 && lane == 0 && it_local < kStampTiles && wave < kWaves)
      stp = a.dbg + ((size_t)it_local * kWaves + wave) * kStampSlots;
    stamp(stp);
    double px = 0.0, py = 0.0, pz = 0.0;
    // ---- input: workspace check + StandardScaler.transform (float64) -> fp32
    if (tid < BM) {
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
      f32x4 *row = reinterpret_cast<f32x4 *>(H + hrow<LY>(tid));
      row[0] = f32x4{x0, x1, x2, 0.0f};
      row[1] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    }
    __syncthreads();
    stamp(stp ? stp + 1 : nullptr);
    // ---- Dense layers
    for (int l = 0; l < a.m.n_layers; ++l) {
      // an opaque (always 0) uniform offset on the LDS tile per layer: the layer
      // functions' per-lane LDS addresses are recomputed per layer instead of being
      // hoisted out of the tile loop and held in registers across it (fp16x3 kernel:
      // 503 -> 396 registers; bf16x6 -1.2 %, the others even)
      int hz = 0;
      asm volatile("" : "+s"(hz));
      float *const HL = H + hz;
      const int G = a.m.kp[l] >> 3;
      const int NT = a.m.np[l] >> 5;
      const f32x4 *wp = reinterpret_cast<const f32x4 *>(a.m.wp[l]);
      const float *bias = a.m.bias[l];
      const int act = a.m.act[l];
      unsigned long long *sl = (stp && l < 14) ? stp + 2 + 2 * l : nullptr;
      unsigned long long *sf = (stp && l == 5) ? stp + 30 : nullptr;  // layer 5's first group
      const void *wx = X ? a.m.wx[l] : nullptr;
      // fp16x3: the next layer reads split planes when it runs the split GEMM
      const bool hout = X == 2 && l + 1 < a.m.n_layers && a.m.wx[l + 1] &&
                        (a.m.np[l + 1] >> 5) > 1;
      if (NT == 1) {
        run_layer_splitk<MR, HK, W, LY>(HL, wp, bias, act, G, wave, lane, tid, sl, hout);
      } else if (X && wx) {
        const float xinv = a.m.xinv[l];
        const int G32 = (a.m.kp[l] + 31) >> 5;  // 32-deep K steps of the split GEMM
        const int cnt = (wave < NT) ? (NT - wave + W - 1) / W : 0;
        switch (cnt) {
          case 4:
            if constexpr (W * 4 <= 16) run_layer<MR, 4, X, HK, W, LY>(HL, wp, bias, act, G, G * NT * 1024, wave, lane, sl, sf, wx, G32, xinv, hout);
            break;
          case 3:
            if constexpr (W * 3 <= 16) run_layer<MR, 3, X, HK, W, LY>(HL, wp, bias, act, G, G * NT * 1024, wave, lane, sl, sf, wx, G32, xinv, hout);
            break;
          case 2: run_layer<MR, 2, X, HK, W, LY>(HL, wp, bias, act, G, G * NT * 1024, wave, lane, sl, sf, wx, G32, xinv, hout); break;
          case 1: run_layer<MR, 1, X, HK, W, LY>(HL, wp, bias, act, G, G * NT * 1024, wave, lane, sl, sf, wx, G32, xinv, hout); break;
          default: __syncthreads(); break;
        }
      } else {
        const int cnt = (wave < NT) ? (NT - wave + W - 1) / W : 0;
        switch (cnt) {
          case 4:
            if constexpr (W * 4 <= 16) run_layer<MR, 4, 0, HK, W, LY>(HL, wp, bias, act, G, G * NT * 1024, wave, lane, sl, sf, nullptr, 0, 1.0f, hout);
            break;
          case 3:
            if constexpr (W * 3 <= 16) run_layer<MR, 3, 0, HK, W, LY>(HL, wp, bias, act, G, G * NT * 1024, wave, lane, sl, sf, nullptr, 0, 1.0f, hout);
            break;
          case 2: run_layer<MR, 2, 0, HK, W, LY>(HL, wp, bias, act, G, G * NT * 1024, wave, lane, sl, sf, nullptr, 0, 1.0f, hout); break;
          case 1: run_layer<MR, 1, 0, HK, W, LY>(HL, wp, bias, act, G, G * NT * 1024, wave, lane, sl, sf, nullptr, 0, 1.0f, hout); break;
#ifdef IKHIP_ANN_WIDE
          case 8: run_layer<MR, 8>(HL, wp, bias, act, G, G * NT * 1024, wave, lane, sl, sf); break;
          case 7: run_layer<MR, 7>(HL, wp, bias, act, G, G * NT * 1024, wave, lane, sl, sf); break;
          case 6: run_layer<MR, 6>(HL, wp, bias, act, G, G * NT * 1024, wave, lane, sl, sf); break;
          case 5: run_layer<MR, 5>(HL, wp, bias, act, G, G * NT * 1024, wave, lane, sl, sf); break;
#endif
          default: __syncthreads(); break;  // idle wave still joins the barrier
        }
      }
      __syncthreads();
      stamp(sl ? sl + 1 : nullptr);
    }
    if (tid == W * 64 - 64)  // the last wave, after the tile's last GEMM
      next_tile[it_local & 1] = (long long)atomicAdd(tile_ctr, 1ull) + (long long)gridDim.x;
    // ---- output: StandardScaler.inverse_transform (in-place fp32, fp64 ops) + FK
    if (tid < BM) {
      bool valid = pt < a.n;
      double err = 0.0;
      if (valid) {
        const float *row = H + hrow<LY>(tid);
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
          err = fk_error(a.jc, th, px, py, pz, a.alpha_bad);
          a.fk_err[pt] = err;
        }
      }
      if (a.fk_err) {
        double e = (valid && err == err) ? err : 0.0;
        blk_max = fmax(blk_max, e);
        blk_sum += e;
      }
    }
    __syncthreads();  // the next tile's staging overwrites H
    stamp(stp ? stp + kStampSlots - 1 : nullptr);
    tile = (int64_t)next_tile[it_local & 1];
  }
  // per-block FK-error stats: one atomic pair per wave holding points, into its shard.
  // The whole wave reduces (lanes >= BM hold zeros): at MR = 1 the upper half of
  // wave 0 holds no points but its registers take part in the shuffles.
  if (a.fk_err && wave * 64 < BM) wave_fk_stats(a.S, blk_max, blk_sum);
}

// The bf16x6 kernels are instantiated in a translation unit of their own
// (ik_ann_x.hip defines IKHIP_ANN_X_TU and includes this file): in one module
// with the fp32 kernel they change the latter's register allocation (29 -> 51
// spilled VGPRs at MR = 2, -Rpass-analysis=kernel-resource-usage).
void launch_ann_kernel_x(int mr, int xmode, unsigned grid, hipStream_t st, const AnnArgs &a);

}  // namespace ann / annw

#if defined(IKHIP_ANN_WIDE)

// Models wider than 512 (up to 1024): fp32 only, 32-point tiles (132 KiB of
// LDS: one workgroup per CU).
void launch_ann_wide(const AnnModelDev &m, const RobotDev &r, const double *pts, int64_t n,
                     float *ang, double *fk_err, bool check_limits, DevStats *S, hipStream_t st,
                     unsigned long long *dbg) {
  using namespace annw;
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
  a.dbg = dbg;
  fk_trip_consts(r, a.jc, &a.alpha_bad);
  int dev = 0, cus = 256;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0)
    cus = 256;
  const int64_t ntiles = (n + 31) / 32;
  const unsigned grid = (unsigned)(ntiles < cus ? ntiles : cus);
  kt_begin("ann_fused_kernel_wide", st);
  IK_LAUNCH((ann_fused_kernel<1, 0>), dim3(grid), dim3(256), 0, st, a);
  kt_end(st);
}

#elif !defined(IKHIP_ANN_X_TU)
using namespace ann;

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

size_t ann_x_bytes(int k, int n) {
  const int k32 = (k + 31) / 32 * 32, np = (n + 31) / 32 * 32;
  return (size_t)k32 * np * 6;
}

static uint16_t bf16_rne(float x) {
  uint32_t u;
  std::memcpy(&u, &x, 4);
  if ((u & 0x7f800000u) == 0x7f800000u) return (uint16_t)(u >> 16);  // inf / nan (none expected)
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

static float bf16_to_f32(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float x;
  std::memcpy(&x, &u, 4);
  return x;
}

// The bf16x6 weight operand: three bf16 planes p (0 hi, 1 mid, 2 lo) of the B
// fragment of v_mfma_f32_16x16x32_bf16 for K step g (32 deep) of feature half fh
// of column tile nt, element j (0..7) of lane l being
// W[32g + 8*(l>>4) + j][32nt + 16fh + (l&15)]:
// dst[((((nt*G32 + g)*2 + fh)*3 + p)*64 + l)*8 + j], split here by
// round-to-nearest-even exactly as split3() splits the activations on the GPU.
// (An fp32 layout split in the kernel reads 4 B per weight instead of 6 but
// measured slower at 64-point tiles: 30.5 vs 27.3 ms per 1M points, the VALU
// being the dearer.)
void ann_pack_layer_x(const float *W, int k, int n, void *dst) {
  const int np = (n + 31) / 32 * 32, NT = np / 32, G32 = (k + 31) / 32;
  uint16_t *d16 = static_cast<uint16_t *>(dst);
  for (int nt = 0; nt < NT; ++nt)
    for (int g = 0; g < G32; ++g)
      for (int fh = 0; fh < 2; ++fh)
        for (int lane = 0; lane < 64; ++lane)
          for (int j = 0; j < 8; ++j) {
            const int kk = 32 * g + 8 * (lane >> 4) + j;
            const int c = nt * 32 + 16 * fh + (lane & 15);
            const float x = (kk < k && c < n) ? W[(size_t)kk * n + c] : 0.0f;
            const uint16_t h = bf16_rne(x);
            const float r1 = x - bf16_to_f32(h);
            const uint16_t m = bf16_rne(r1);
            const float r2 = r1 - bf16_to_f32(m);
            const size_t base =
                ((((size_t)nt * G32 + g) * 2 + fh) * 3) * 64 * 8 + (size_t)lane * 8 + j;
            d16[base] = h;
            d16[base + 64 * 8] = m;
            d16[base + 2 * 64 * 8] = bf16_rne(r2);
          }
}

size_t ann_h_bytes(int k, int n) {
  const int k32 = (k + 31) / 32 * 32, np = (n + 31) / 32 * 32;
  return (size_t)k32 * np * 4;
}

// The power of two that brings the layer's largest |weight| to [2^13, 2^14):
// the fp16 planes then keep their full 11 bits down to weights ~2^-10 of the
// largest, and nothing comes near fp16's 65504.
int ann_h_scale_exp(const float *W, int k, int n) {
  float mx = 0.0f;
  for (size_t i = 0; i < (size_t)k * n; ++i) mx = std::fmax(mx, std::fabs(W[i]));
  if (!(mx > 0.0f) || !std::isfinite(mx)) return 0;
  int e = 0;
  std::frexp(mx, &e);  // mx in [2^(e-1), 2^e)
  int s = 14 - e;
  return s < -60 ? -60 : (s > 60 ? 60 : s);
}

// The fp16x3 weight operand: planes p (0 hi, 1 lo) of W * 2^scale_exp in the
// B-fragment order of v_mfma_f32_16x16x32_f16 (32-deep K steps):
// dst[((((nt*G32 + g)*2 + fh)*2 + p)*64 + l)*8 + j] = plane p of
// W[32g + 8*(l>>4) + j][32nt + 16fh + (l&15)] * 2^scale_exp, each plane rounded
// to nearest (the scaled weight and its residual are exact in fp32).
void ann_pack_layer_h(const float *W, int k, int n, int scale_exp, void *dst) {
  const int np = (n + 31) / 32 * 32, NT = np / 32, G32 = (k + 31) / 32;
  _Float16 *d = static_cast<_Float16 *>(dst);
  for (int nt = 0; nt < NT; ++nt)
    for (int g = 0; g < G32; ++g)
      for (int fh = 0; fh < 2; ++fh)
        for (int lane = 0; lane < 64; ++lane)
          for (int j = 0; j < 8; ++j) {
            const int kk = 32 * g + 8 * (lane >> 4) + j;
            const int c = nt * 32 + 16 * fh + (lane & 15);
            const float x =
                (kk < k && c < n) ? std::ldexp(W[(size_t)kk * n + c], scale_exp) : 0.0f;
            const _Float16 h = (_Float16)x;
            const size_t base =
                ((((size_t)nt * G32 + g) * 2 + fh) * 2) * 64 * 8 + (size_t)lane * 8 + j;
            d[base] = h;
            d[base + 64 * 8] = (_Float16)(x - (float)h);
          }
}

// Tile rows per workgroup: 32 * MR points.  fp32: MR = 1 (two 32-point
// workgroups per CU, one's barrier and epilogue under the other's MFMAs)
// measured 39.8 ms against 41.3 ms for MR = 2 (1M points, 3-12x500-4,
// tools/sweep_ann.py and bench.py, same box; round 1's GEMM loop measured the
// opposite, 49.0 vs 44.9 ms).  The split modes keep MR = 2: their GEMM is bound
// by the weight stream from L2, which 64-point tiles halve (bf16x6 25.1 vs
// 33.8 ms, fp16x3 15.2 vs 19.6 ms).  IKHIP_ANN_MR overrides.
static int ann_tile_rows(int xmode) {
  static int forced = -1;
  if (forced < 0) {
    const char *v = getenv("IKHIP_ANN_MR");
    forced = (v && (atoi(v) == 1 || atoi(v) == 2)) ? atoi(v) : 0;
  }
  return forced ? forced : (xmode ? 2 : 1);
}

size_t ann_debug_words() { return (size_t)kStampTiles * kWaves * kStampSlots; }

void launch_ann(const AnnModelDev &m, const RobotDev &r, const double *pts, int64_t n,
                float *ang, double *fk_err, bool check_limits, DevStats *S, hipStream_t st,
                unsigned long long *dbg) {
  if (n <= 0) return;
  for (int l = 0; l < m.n_layers; ++l)
    if (m.np[l] > 512 || m.kp[l] > 512) {
      launch_ann_wide(m, r, pts, n, ang, fk_err, check_limits, S, st, dbg);
      return;
    }
  AnnArgs a;
  a.m = m;
  a.r = r;
  a.pts = pts;
  a.n = n;
  a.ang = ang;
  a.fk_err = fk_err;
  a.check_limits = check_limits ? 1 : 0;
  a.S = S;
  a.dbg = dbg;
  fk_trip_consts(r, a.jc, &a.alpha_bad);
  int dev = 0, cus = 256;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0)
    cus = 256;
  bool x = false;
  for (int l = 0; l < m.n_layers; ++l) x = x || m.wx[l] != nullptr;
  const int xmode = x ? m.xmode : 0;
  const int mr = ann_tile_rows(xmode);
  const int64_t bm = 32 * mr;
  const int64_t ntiles = (n + bm - 1) / bm;
  const int64_t slots = (int64_t)cus * (mr == 2 ? 1 : 2);  // resident workgroups
  unsigned grid = (unsigned)(ntiles < slots ? ntiles : slots);
  kt_begin(xmode == 1 ? "ann_fused_kernel_bf16x6"
                      : xmode == 2 ? "ann_fused_kernel_fp16x3" : "ann_fused_kernel",
           st);
  if (xmode)
    launch_ann_kernel_x(mr, xmode, grid, st, a);
  else if (mr == 2)
    IK_LAUNCH((ann_fused_kernel<2, 0>), dim3(grid), dim3(64 * ann_waves<2, 0>()), 0, st,
                       a);
  else
    IK_LAUNCH((ann_fused_kernel<1, 0>), dim3(grid), dim3(256), 0, st, a);
  kt_end(st);
}

#else  // IKHIP_ANN_X_TU

void ann::launch_ann_kernel_x(int mr, int xmode, unsigned grid, hipStream_t st,
                              const AnnArgs &a) {
#define IK_X(M, X) \
  IK_LAUNCH((ann_fused_kernel<M, X>), dim3(grid), dim3(64 * ann_waves<M, X>()), 0, st, a)
  if (mr == 2) {
    if (xmode == 2) IK_X(2, 2); else IK_X(2, 1);
  } else {
    if (xmode == 2) IK_X(1, 2); else IK_X(1, 1);
  }
#undef IK_X
}

#endif  // IKHIP_ANN_X_TU

}  // namespace ikhip
