// ubench.hip -- microbenchmarks behind two design decisions:
//
//  iter  W ILP  the FABRIK iteration (fabrik_step4_reuse, the production
//               arithmetic from csrc/ik_fabrik_step.h) at W waves per SIMD and ILP
//               independent chains per lane, with the production kernel's
//               per-iteration wave-uniform domain vote: is the iteration
//               latency-bound (more waves / chains help) or issue-bound?
//  iterl W      the r06 step (fabrik_step4_lazy) at W waves per SIMD: the loop's own rate
//  act   V W    the tanh epilogue of the ANN split modes, 8 elements per lane in
//               flight like act_apply2x4: V 0 = sign (1-e)/(1+e) (r02), 1 = 1 - 2/(1+e),
//               2 = 1 - 2/(1+e) with e = exp2 from a degree-6 polynomial on the
//               full-rate pipe (the VERDICT r02 proposal) instead of v_exp_f32.
//  lat   K      dependent-chain latency of one instruction kind (K 0 v_fma_f64,
//               1 v_rcp_f64, 2 v_rsq_f64, 3 v_fma_f32, 4 v_exp_f32), one wave per SIMD.
//  mfma  Z F32  full-chip MFMA issue rate and the clock the chip holds under it.
//  kloop V      the fp16x3 layer's K loop alone, with / without its loads, and over
//               a 12 MiB weight set (V 4; V 5 with each workgroup at its own layer).
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/ubench tools/ubench.hip
// Prints one JSON line per case: times from HIP events, cycles from s_memtime
// (shader clock ticks) in block 0.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../inversekinematicsann_amd/csrc/ik_fabrik_step.h"

using namespace ikhip;

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                     \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

template <int ILP>
__global__ __launch_bounds__(256) void iter_bench(int iters, const double *goals, int ng,
                                                  double *out, unsigned long long *clk) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  const d3 start = {0.0, 0.0, 2.0};
  const double L[4] = {2.0, 2.0, 2.0, 2.0};
  d3 J1[ILP], J2[ILP], J3[ILP], g[ILP], cd[ILP];
  double cq[ILP];
  uint32_t cdom[ILP];
#pragma unroll
  for (int k = 0; k < ILP; ++k) {
    const int i = (tid * ILP + k) % ng;
    g[k] = {goals[3 * i], goals[3 * i + 1], goals[3 * i + 2]};
    J1[k] = {1e-16, 0.0, 4.0};
    J2[k] = {2e-16, 0.0, 6.0};
    J3[k] = {3e-16, 0.0, 8.0};
    reuse_carry(J2[k], g[k], L[3], cq[k], cd[k], cdom[k]);
  }
  double acc = 0.0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < ILP; ++k) {
      uint32_t dom = 0, cdom_n = cdom[k];
      d3 n1 = J1[k], n2 = J2[k], n3 = J3[k], cd_n = cd[k];
      double se, ge, cq_n = cq[k];
      fabrik_step4_reuse(start, n1, n2, n3, g[k], L, se, ge, cq_n, cd_n, cdom_n, dom);
      if (__all(dom < kCoreDom)) {  // the production kernel's per-iteration vote
        J1[k] = n1; J2[k] = n2; J3[k] = n3;
        cq[k] = cq_n; cd[k] = cd_n; cdom[k] = cdom_n;
        acc += se + ge;
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = acc;
#pragma unroll
  for (int k = 0; k < ILP; ++k) s += J3[k].x + J3[k].y + J3[k].z;
  out[tid] = s;
  if (tid == 0) clk[0] = t1 - t0;
}

// iterl: the r06 production step (fabrik_step4_lazy: errors from the roots, the
// quotient domain test, the band decisions as ballots) with the kernel's stop rule
// (a lane that stops keeps its state; the wave goes on while any lane runs), every
// lane iterating the same goal set: the loop's own issue rate, against which the
// iteration kernel's wave-iterations per SIMD cycle are compared.
__global__ __launch_bounds__(256) void iter_lazy_bench(int iters, const double *goals, int ng,
                                                       double *out, unsigned long long *clk,
                                                       ErrBand band, double tol2, double qmax) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  const d3 start = {0.0, 0.0, 2.0};
  const double L[4] = {2.0, 2.0, 2.0, 2.0};
  const int i = tid % ng;
  const d3 g = {goals[3 * i], goals[3 * i + 1], goals[3 * i + 2]};
  d3 J1 = {1e-16, 0.0, 4.0}, J2 = {2e-16, 0.0, 6.0}, cd;
  double cq;
  uint32_t cdom;
  reuse_carry(J2, g, L[3], cq, cd, cdom);
  double acc = 0.0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    bool cont = true;
    if (!fabrik_step4_lazy(start, J1, J2, g, L, band, tol2, qmax, cont, cq, cd)) acc += 1.0;
    acc += cont ? 1.0 : 0.0;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[tid] = acc + J2.x + J2.y + J2.z + cq;
  if (tid == 0) clk[0] = t1 - t0;
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int V>
__device__ __forceinline__ void tanh8(f32x2 (&v)[4]) {
  if constexpr (V == 0) {  // r02: sign(v) (1 - e) / (1 + e), e = exp2(-2|v| log2 e)
    f32x2 e[4], d[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) e[k] = v[k] * 2.885390081777927f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      e[k].x = __builtin_amdgcn_exp2f(-fabsf(e[k].x));
      e[k].y = __builtin_amdgcn_exp2f(-fabsf(e[k].y));
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) d[k] = 1.0f + e[k];
#pragma unroll
    for (int k = 0; k < 4; ++k) e[k] = 1.0f - e[k];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      d[k].x = __builtin_amdgcn_rcpf(d[k].x);
      d[k].y = __builtin_amdgcn_rcpf(d[k].y);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) e[k] = e[k] * d[k];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[k].x = copysignf(e[k].x, v[k].x);
      v[k].y = copysignf(e[k].y, v[k].y);
    }
  } else {  // 1 - 2 / (1 + exp2(2 v log2 e)); V == 2: exp2 by polynomial
    f32x2 e[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) e[k] = v[k] * 2.885390081777927f;
    if constexpr (V == 1) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        e[k].x = __builtin_amdgcn_exp2f(e[k].x);
        e[k].y = __builtin_amdgcn_exp2f(e[k].y);
      }
    } else {
      // 2^u = 2^n * p(f), n = rint(u) (magic-number rounding), f in [-0.5, 0.5],
      // p the degree-6 Taylor/minimax polynomial, 2^n inserted into the exponent
      const f32x2 magic = {12582912.0f, 12582912.0f};  // 1.5 * 2^23
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        f32x2 u = __builtin_elementwise_min(__builtin_elementwise_max(e[k], f32x2{-126.f, -126.f}),
                                            f32x2{126.f, 126.f});
        const f32x2 t = u + magic;
        const f32x2 n = t - magic;
        const f32x2 f = u - n;
        const auto F = [](f32x2 a, f32x2 b, float c) {
          return __builtin_elementwise_fma(a, b, f32x2{c, c});  // v_pk_fma_f32
        };
        f32x2 p = F(f, f32x2{1.5403530393381609e-4f, 1.5403530393381609e-4f},
                    1.3333558146428443e-3f);
        p = F(p, f, 9.6181291076284772e-3f);
        p = F(p, f, 5.5504108664821580e-2f);
        p = F(p, f, 2.4022650695910071e-1f);
        p = F(p, f, 6.9314718055994531e-1f);
        p = F(p, f, 1.0f);
        const int nx = __builtin_bit_cast(int, t.x) - 0x4B400000;
        const int ny = __builtin_bit_cast(int, t.y) - 0x4B400000;
        e[k].x = __builtin_bit_cast(float, __builtin_bit_cast(int, p.x) + (nx << 23));
        e[k].y = __builtin_bit_cast(float, __builtin_bit_cast(int, p.y) + (ny << 23));
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) e[k] = 1.0f + e[k];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      e[k].x = __builtin_amdgcn_rcpf(e[k].x);
      e[k].y = __builtin_amdgcn_rcpf(e[k].y);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = 1.0f - 2.0f * e[k];
  }
}

template <int V>
__global__ __launch_bounds__(256) void act_bench(int iters, float *out, unsigned long long *clk) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  f32x2 v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = f32x2{0.01f * (tid % 97) - 0.3f * k, 0.02f * k - 0.4f};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = v[k] * 1.7f + 0.05f;  // the bias add's slot
    tanh8<V>(v);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[tid] = v[0].x + v[1].y + v[2].x + v[3].y;
  if (tid == 0) clk[0] = t1 - t0;
}

template <int K>
__global__ __launch_bounds__(64) void lat_bench(int iters, float *out, unsigned long long *clk) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  double x = 1.0 + 1e-9 * tid;
  float y = 1.0f + 1e-6f * tid;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if constexpr (K == 0) x = __builtin_fma(x, 0.999999, 1e-7);
    else if constexpr (K == 1) x = __builtin_amdgcn_rcp(x);
    else if constexpr (K == 2) x = __builtin_amdgcn_rsq(x) * 1.0000001;
    else if constexpr (K == 3) y = __builtin_fmaf(y, 0.999f, 1e-4f);
    else y = __builtin_amdgcn_exp2f(y) * 0.25f;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[tid] = (float)x + y;
  if (tid == 0) clk[0] = t1 - t0;
}

// Full-chip MFMA issue rate (one wave per SIMD, 4 waves per CU, every CU): steps
// of 96 v_mfma_f32_16x16x32_f16 on 16 accumulators (in-place asm) from register
// operands, no memory.  Z: operands all zero (1) or
// random (0): the operand bits set the power drawn.  F32: the fp32 kernel's
// v_mfma_f32_32x32x2_f32 on 8 accumulators instead (32 per step).
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
template <int Z, int F32>
__global__ __launch_bounds__(256) void mfma_bench(int iters, float *out, unsigned long long *clk) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  const float base = Z ? 0.0f : 0.001f * (tid % 89) + 0.1f;
  if constexpr (!F32) {
    h8 a[4], b[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        a[k][e] = (_Float16)(base * (e + 1) - 0.3f * k);
        b[k][e] = (_Float16)(base * (7 - e) + 0.2f * k);
      }
    f4 c[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) c[q] = f4{0, 0, 0, 0};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int q = 0; q < 16; ++q)
          // (asm: dst = srcC in place; the builtin let the allocator rotate the
          // accumulators through the loop with ~90 AGPR moves per 96 MFMAs)
          asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0"
                       : "+a"(c[q]) : "v"(a[(q + r) & 3]), "v"(b[(q >> 2) & 3]));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float acc = 0.0f;
#pragma unroll
    for (int q = 0; q < 16; ++q) acc += (c[q][0] + c[q][1]) + (c[q][2] + c[q][3]);
    out[tid] = acc;
    if (tid == 0) clk[0] = t1 - t0;
  } else {
    f4 a[2], b[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      a[k] = f4{base, base * 2, base * 3 - 0.1f * k, base * 0.5f};
      b[k] = f4{base * 5, base - 0.2f * k, base * 0.25f, base * 4};
    }
    f16v c[8];
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int e = 0; e < 16; ++e) c[q][e] = 0.0f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 8; ++q)
          c[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[(q + r) & 1][r], b[((q >> 1) + r) & 1][r], c[q], 0, 0, 0);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float acc = 0.0f;
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc += c[q][e];
    out[tid] = acc;
    if (tid == 0) clk[0] = t1 - t0;
  }
}

// The fp16x3 layer's K loop alone (ik_ann.hip layer_gemm_h16 / step_h16,
// restated: 4 waves per CU, MR = 2 x NR = 4 tiles of 16x16x32 sub-tiles, the weight
// stream through a buffer descriptor from a 1 MiB L2-resident operand, a 2-step
// ring, the activations from LDS split planes, pattern 2), LAYERS x 16 steps with
// no epilogue: V 0 as production, 1 without the weight loads (the ring's registers
// reused), 2 without the LDS reads, 3 without either.  cycles per K step per wave.
typedef float kf4 __attribute__((ext_vector_type(4)));
struct KSplit2 {
  h8 hi, lo;
};
struct KW {
  h8 p[4][2][2];  // [tile][feature half][plane]
};
constexpr int kKLd = 516;  // floats per LDS row (ik_ann.hip kLd)
// V 4: as V 0, but layer l reads weight slice l % 12 of a 12 MiB operand (the
// reference model's 11 hidden layers do not fit one XCD's 4 MB L2); V 5: each
// workgroup starts at its own slice (blockIdx % 12), as drifted workgroups are.
template <int V>
__global__ __launch_bounds__(256) void kloop_bench(int layers, const h8 *wx0, int xbytes,
                                                   float *out, unsigned long long *clk) {
  __shared__ float H[64 * kKLd];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 64 * kKLd; i += 256) H[i] = 0.001f * (i % 251);
  __syncthreads();
  constexpr int G32 = 16, W = 4;
  const _Float16 *ap = reinterpret_cast<const _Float16 *>(H + (lane & 15) * kKLd) + 8 * (lane >> 4);
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<h8 *>(wx0), 0, xbytes, 0x00020000);
  int vo[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) vo[j] = ((wave + W * j) * G32 * 4 * 64 + lane) * 16;
  auto load_w = [&](KW &w, int g) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int fh = 0; fh < 2; ++fh)
#pragma unroll
        for (int p = 0; p < 2; ++p)
          w.p[j][fh][p] = __builtin_bit_cast(
              h8, __builtin_amdgcn_raw_buffer_load_b128(rs, vo[j], (g * 4 + fh * 2 + p) * 1024, 0));
  };
  auto load_a = [&](KSplit2 (&a)[2][2], const _Float16 *base, int g) {
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int ph = 0; ph < 2; ++ph) {
        const _Float16 *q = base + (m * 32 + 16 * ph) * 2 * kKLd + 32 * g;
        a[m][ph].hi = *reinterpret_cast<const h8 *>(q);
        a[m][ph].lo = *reinterpret_cast<const h8 *>(q + 512);
      }
  };
  kf4 acc[2][4][4];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int s = 0; s < 4; ++s) acc[m][j][s] = kf4{0, 0, 0, 0};
  KW w[2];
  load_w(w[0], 0);
  load_w(w[1], 1);
  KSplit2 sa[2][2];
  load_a(sa, ap, 0);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int l = 0; l < layers; ++l) {
    if (V >= 4) {  // 5: each workgroup at its own layer phase (blockIdx % 12)
      const h8 *wl = wx0 + (size_t)((l + (V == 5 ? blockIdx.x : 0)) % 12) * (xbytes / 16);
      rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<h8 *>(wl), 0, xbytes, 0x00020000);
    }
    for (int g = 0; g < G32; g += 2) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        __builtin_amdgcn_sched_barrier(0);
        if (V == 0 || V == 2 || V >= 4) load_w(w[(u + 1) % 2], g + u + 1);
        KSplit2 sn[2][2];
        if (V == 0 || V == 1 || V >= 4) load_a(sn, ap + 32 * g, u + 1);
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int fh = 0; fh < 2; ++fh)
#pragma unroll
              for (int ph = 0; ph < 2; ++ph) {
                const KW &ww = w[u];
                kf4 c = acc[m][j][2 * fh + ph];
                c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ww.p[j][fh][0], sa[m][ph].lo, c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ww.p[j][fh][1], sa[m][ph].hi, c, 0, 0, 0);
                acc[m][j][2 * fh + ph] =
                    __builtin_amdgcn_mfma_f32_16x16x32_f16(ww.p[j][fh][0], sa[m][ph].hi, c, 0, 0, 0);
              }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          if (V == 0 || V == 2 || V >= 4) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          if ((V == 0 || V == 1 || V >= 4) && i < 8) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (V == 0 || V == 1 || V >= 4)
#pragma unroll
          for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int ph = 0; ph < 2; ++ph) sa[m][ph] = sn[m][ph];
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float r = 0.0f;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) r += (acc[m][j][q][0] + acc[m][j][q][1]) + (acc[m][j][q][2] + acc[m][j][q][3]);
  out[blockIdx.x * 256 + threadIdx.x] = r;
  if (blockIdx.x == 0 && threadIdx.x == 0) clk[0] = t1 - t0;
}

static int num_cus() {
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  return cus;
}

template <class F>
static void timed(const char *name, F launch, unsigned long long *dclk, double work_units,
                  double per_simd_units, const char *extra) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  launch();  // warm-up
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  launch();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0.0f;
  CK(hipEventElapsedTime(&ms, a, b));
  unsigned long long clk = 0;
  CK(hipMemcpy(&clk, dclk, 8, hipMemcpyDeviceToHost));
  printf("{\"case\": \"%s\", %s, \"ms\": %.4f, \"units_per_ns\": %.4f, "
         "\"cycles_per_unit_per_simd\": %.2f}\n",
         name, extra, ms, work_units / (ms * 1e6), (double)clk / per_simd_units);
  fflush(stdout);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
}

int main(int argc, char **argv) {
  const int cus = num_cus();
  double *dout = nullptr, *dgoals = nullptr;
  unsigned long long *dclk = nullptr;
  CK(hipMalloc(&dout, (size_t)cus * 8 * 256 * 8));
  CK(hipMalloc(&dclk, 8));
  // reachable goals around the robot (random_dist-like)
  const int ng = 4096;
  std::vector<double> g(3 * ng);
  unsigned s = 12345;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (s >> 8) * (1.0 / 16777216.0); };
  for (int i = 0; i < ng; ++i) {
    g[3 * i] = 0.2 + 1.5 * rnd();
    g[3 * i + 1] = -1.0 + 2.0 * rnd();
    g[3 * i + 2] = -0.5 + 2.0 * rnd();
  }
  CK(hipMalloc(&dgoals, g.size() * 8));
  CK(hipMemcpy(dgoals, g.data(), g.size() * 8, hipMemcpyHostToDevice));
  const char *what = argc > 1 ? argv[1] : "all";
  char extra[128];
  if (!strcmp(what, "all") || !strcmp(what, "iter")) {
    const int iters = 200;
    for (int ilp = 1; ilp <= 2; ++ilp)
      for (int W = 1; W <= (ilp == 1 ? 6 : 3); ++W) {
        const unsigned blocks = (unsigned)cus * W;
        snprintf(extra, sizeof extra, "\"waves_per_simd\": %d, \"ilp\": %d", W, ilp);
        const double lane_it = (double)blocks * 256 * ilp * iters;
        const double simd_wave_it = (double)W * ilp * iters;  // per SIMD: W waves
        auto L = [&]() {
          if (ilp == 1)
            hipLaunchKernelGGL(iter_bench<1>, dim3(blocks), dim3(256), 0, 0, iters, dgoals, ng,
                               dout, dclk);
          else
            hipLaunchKernelGGL(iter_bench<2>, dim3(blocks), dim3(256), 0, 0, iters, dgoals, ng,
                               dout, dclk);
        };
        timed("iter", L, dclk, lane_it, simd_wave_it, extra);
      }
  }
  if (!strcmp(what, "all") || !strcmp(what, "iterl")) {
    const int iters = 400;
    const double tol2 = 1e-6;  // tol 1e-3 (the threshold's exact value does not matter here)
    const ErrBand band = fabrik_band(tol2, 64.0 * 11.0, 8.0);
    const double Ls[4] = {2.0, 2.0, 2.0, 2.0};
    const double qmax = fabrik_qmax(Ls);
    for (int W = 1; W <= 3; ++W) {
      const unsigned blocks = (unsigned)cus * W;
      snprintf(extra, sizeof extra, "\"waves_per_simd\": %d", W);
      const double lane_it = (double)blocks * 256 * iters;
      const double simd_wave_it = (double)W * iters;
      auto L = [&]() {
        hipLaunchKernelGGL(iter_lazy_bench, dim3(blocks), dim3(256), 0, 0, iters, dgoals, ng,
                           dout, dclk, band, tol2, qmax);
      };
      timed("iterl", L, dclk, lane_it, simd_wave_it, extra);
    }
  }
  if (!strcmp(what, "all") || !strcmp(what, "act")) {
    const int iters = 2000;
    for (int V = 0; V <= 2; ++V)
      for (int W = 1; W <= 2; ++W) {
        const unsigned blocks = (unsigned)cus * W;
        snprintf(extra, sizeof extra, "\"variant\": %d, \"waves_per_simd\": %d", V, W);
        const double elems = (double)blocks * 256 * 8 * iters;
        const double simd_elems = (double)W * 8 * iters * 64;  // per SIMD: lanes x elements
        float *fo = reinterpret_cast<float *>(dout);
        auto L = [&]() {
          if (V == 0) hipLaunchKernelGGL(act_bench<0>, dim3(blocks), dim3(256), 0, 0, iters, fo, dclk);
          else if (V == 1) hipLaunchKernelGGL(act_bench<1>, dim3(blocks), dim3(256), 0, 0, iters, fo, dclk);
          else hipLaunchKernelGGL(act_bench<2>, dim3(blocks), dim3(256), 0, 0, iters, fo, dclk);
        };
        timed("act", L, dclk, elems, simd_elems / 64.0, extra);  // cycles per element-slot of a wave
      }
  }
  if (!strcmp(what, "all") || !strcmp(what, "lat")) {
    const int iters = 4096;
    const char *names[5] = {"v_fma_f64", "v_rcp_f64", "v_rsq_f64", "v_fma_f32", "v_exp_f32"};
    for (int K = 0; K < 5; ++K) {
      snprintf(extra, sizeof extra, "\"instr\": \"%s\"", names[K]);
      float *fo = reinterpret_cast<float *>(dout);
      auto L = [&]() {
        switch (K) {
          case 0: hipLaunchKernelGGL(lat_bench<0>, dim3(cus * 4), dim3(64), 0, 0, iters, fo, dclk); break;
          case 1: hipLaunchKernelGGL(lat_bench<1>, dim3(cus * 4), dim3(64), 0, 0, iters, fo, dclk); break;
          case 2: hipLaunchKernelGGL(lat_bench<2>, dim3(cus * 4), dim3(64), 0, 0, iters, fo, dclk); break;
          case 3: hipLaunchKernelGGL(lat_bench<3>, dim3(cus * 4), dim3(64), 0, 0, iters, fo, dclk); break;
          default: hipLaunchKernelGGL(lat_bench<4>, dim3(cus * 4), dim3(64), 0, 0, iters, fo, dclk); break;
        }
      };
      timed("lat", L, dclk, (double)cus * 4 * 64 * iters, (double)iters, extra);
    }
  }
  if (!strcmp(what, "all") || !strcmp(what, "mfma")) {
    // cycles per MFMA per SIMD (s_memtime) and the clock the chip held (s_memtime
    // cycles of wave 0 over the launch's event time)
    // ~40-60 ms per launch (the clock settles under load), each variant twice,
    // interleaved
    const int iters = 50000;
    for (int rep = 0; rep < 2; ++rep)
    for (int F32 = 0; F32 <= 1; ++F32)
      for (int Z = 0; Z <= 1; ++Z) {
        const unsigned blocks = (unsigned)cus;
        const double per_wave = (double)iters * (F32 ? 32 : 96);
        snprintf(extra, sizeof extra, "\"instr\": \"%s\", \"zeros\": %d",
                 F32 ? "v_mfma_f32_32x32x2_f32" : "v_mfma_f32_16x16x32_f16", Z);
        float *fo = reinterpret_cast<float *>(dout);
        auto L = [&]() {
          if (F32) {
            if (Z) hipLaunchKernelGGL((mfma_bench<1, 1>), dim3(blocks), dim3(256), 0, 0, iters, fo, dclk);
            else hipLaunchKernelGGL((mfma_bench<0, 1>), dim3(blocks), dim3(256), 0, 0, iters, fo, dclk);
          } else {
            if (Z) hipLaunchKernelGGL((mfma_bench<1, 0>), dim3(blocks), dim3(256), 0, 0, iters, fo, dclk);
            else hipLaunchKernelGGL((mfma_bench<0, 0>), dim3(blocks), dim3(256), 0, 0, iters, fo, dclk);
          }
        };
        timed("mfma", L, dclk, (double)blocks * 4 * per_wave, per_wave, extra);
      }
  }
  if (!strcmp(what, "all") || !strcmp(what, "kloop")) {
    const int layers = 400;
    const int xbytes = 16 * 16 * 4 * 1024;  // 16 column tiles x 16 K steps x 4 blocks
    h8 *wx = nullptr;
    CK(hipMalloc(&wx, (size_t)xbytes * 12));
    {
      std::vector<_Float16> hw((size_t)xbytes * 12 / 2);
      for (size_t i = 0; i < hw.size(); ++i) hw[i] = (_Float16)(0.01f * (float)((i * 37) % 101) - 0.5f);
      CK(hipMemcpy(wx, hw.data(), (size_t)xbytes * 12, hipMemcpyHostToDevice));
    }
    float *fo = reinterpret_cast<float *>(dout);
    for (int rep = 0; rep < 2; ++rep)
      for (int V = 0; V <= 5; ++V) {
        snprintf(extra, sizeof extra, "\"variant\": %d", V);
        const double steps = (double)layers * 16;
        auto L = [&]() {
          switch (V) {
            case 0: hipLaunchKernelGGL(kloop_bench<0>, dim3(cus), dim3(256), 0, 0, layers, wx, xbytes, fo, dclk); break;
            case 1: hipLaunchKernelGGL(kloop_bench<1>, dim3(cus), dim3(256), 0, 0, layers, wx, xbytes, fo, dclk); break;
            case 2: hipLaunchKernelGGL(kloop_bench<2>, dim3(cus), dim3(256), 0, 0, layers, wx, xbytes, fo, dclk); break;
            case 3: hipLaunchKernelGGL(kloop_bench<3>, dim3(cus), dim3(256), 0, 0, layers, wx, xbytes, fo, dclk); break;
            case 4: hipLaunchKernelGGL(kloop_bench<4>, dim3(cus), dim3(256), 0, 0, layers, wx, xbytes, fo, dclk); break;
            default: hipLaunchKernelGGL(kloop_bench<5>, dim3(cus), dim3(256), 0, 0, layers, wx, xbytes, fo, dclk); break;
          }
        };
        timed("kloop", L, dclk, (double)cus * 4 * steps * 96, steps, extra);  // units: MFMAs
      }
    CK(hipFree(wx));
  }
  CK(hipFree(dout));
  CK(hipFree(dgoals));
  CK(hipFree(dclk));
  return 0;
}
