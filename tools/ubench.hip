// ubench.hip -- microbenchmarks behind two design decisions:
//
//  iter  W ILP  the FABRIK iteration (fabrik_step4_reuse, the production
//               arithmetic from csrc/ik_fabrik_step.h) at W waves per SIMD and ILP
//               independent chains per lane, with the production kernel's
//               per-iteration wave-uniform domain vote: is the iteration
//               latency-bound (more waves / chains help) or issue-bound?
//  act   V W    the tanh epilogue of the ANN split modes, 8 elements per lane in
//               flight like act_apply2x4: V 0 = sign (1-e)/(1+e) (r02), 1 = 1 - 2/(1+e),
//               2 = 1 - 2/(1+e) with e = exp2 from a degree-6 polynomial on the
//               full-rate pipe (the VERDICT r02 proposal) instead of v_exp_f32.
//  lat   K      dependent-chain latency of one instruction kind (K 0 v_fma_f64,
//               1 v_rcp_f64, 2 v_rsq_f64, 3 v_fma_f32, 4 v_exp_f32), one wave per SIMD.
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
  CK(hipFree(dout));
  CK(hipFree(dgoals));
  CK(hipFree(dclk));
  return 0;
}
