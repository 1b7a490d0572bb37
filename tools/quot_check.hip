// quot_check.hip -- is quot_sqrt_core(a, x) (tools/quot_fused.h: the quotient
// a / sqrt(x) with the divisor's reciprocal seeded from sqrt_core's own
// refined 1/(2 sqrt(x)) instead of v_rcp_f64) bit-identical to
// div_core(a, sqrt_core(x)) and to the compiler's a / sqrt(x)?  Counts
// mismatches over N random (a, x) pairs per distribution, on the GPU.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/quot_check tools/quot_check.hip
//   tools/quot_check [log2 pairs per case, default 36]
//
// Distributions: 0 FABRIK-like (x log-uniform in [2^-20, 2^8], a = 2), 1 x
// log-uniform over sqrt_core's whole domain [2^-767, 2^1023), a log-uniform in
// [2^-100, 2^100] with either sign, 2 x uniform mantissa in [1, 4) (every binade
// pair), a uniform in [1, 2); 3 near-midpoint reciprocals: x within 3 ulps of root^2 for
// roots within 2^15 ulps of a power of two, a with 4 mantissa bits in [2^-4, 2^4].
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../inversekinematicsann_amd/csrc/ik_common.h"
#include "quot_fused.h"

using namespace ikhip;

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ double from_bits(uint64_t b) { return __longlong_as_double((long long)b); }

__global__ __launch_bounds__(256) void check(int dist, uint64_t per_thread, uint64_t seed,
                                             unsigned long long *cnt, double *first) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long bad_fused = 0, bad_core = 0;
  for (uint64_t k = 0; k < per_thread; ++k) {
    const uint64_t r = mix(seed ^ (tid * 0x100000001b3ull + k));
    const uint64_t r2 = mix(r);
    double x, a;
    const uint64_t mant = r & 0xfffffffffffffull;
    if (dist == 0) {
      const uint64_t e = 1023 - 20 + ((r >> 52) % 28);
      x = from_bits((e << 52) | mant);
      a = 2.0;
    } else if (dist == 1) {
      const uint64_t e = 256 + ((r >> 52) % (2046 - 256));  // 2^-767 .. 2^1022
      x = from_bits((e << 52) | mant);
      const uint64_t ea = 1023 - 100 + ((r2 >> 52) % 201);
      a = from_bits(((r2 >> 63) << 63) | (ea << 52) | (r2 & 0xfffffffffffffull));
    } else if (dist == 2) {
      x = from_bits(((uint64_t)(1023 + ((r >> 52) & 1)) << 52) | mant);
      a = from_bits((1023ull << 52) | (r2 & 0xfffffffffffffull));
    } else {
      // hard cases: x within a few ulps of the square of a root just below or above a
      // power of two (1/root then sits near a rounding midpoint), or of an exact
      // square of a short-mantissa root; a a link-like length (few mantissa bits)
      const int64_t j = (int64_t)(r & 0xffff) - 0x8000;            // root offset in ulps
      const int e = (int)((r >> 16) % 64) - 32;                    // root binade
      const double root = ldexp(1.0 + (double)j * 0x1p-52, e);
      const double x0 = root * root;
      const int64_t dx = (int64_t)((r >> 24) & 7) - 3;             // +-3 ulps
      x = from_bits((uint64_t)(__double_as_longlong(x0) + dx));
      const uint64_t am = (r2 & 0xfull) << 48;                     // 4 mantissa bits
      a = from_bits(((uint64_t)(1023 - 4 + (int)((r2 >> 8) % 9)) << 52) | am);
    }
    const double q_ref = a / sqrt(x);
    const double q_core = div_core(a, sqrt_core(x));
    const double q_fused = quot_sqrt_core(a, x);
    const bool bf = __double_as_longlong(q_fused) != __double_as_longlong(q_ref);
    const bool bc = __double_as_longlong(q_core) != __double_as_longlong(q_ref);
    bad_fused += bf;
    bad_core += bc;
    if (bf && atomicAdd(&cnt[2], 1ull) == 0) {
      first[0] = a;
      first[1] = x;
      first[2] = q_ref;
      first[3] = q_fused;
    }
  }
  atomicAdd(&cnt[0], bad_fused);
  atomicAdd(&cnt[1], bad_core);
}

int main(int argc, char **argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 36;
  const unsigned blocks = 8192, threads = 256;
  const uint64_t total = 1ull << lg;
  const uint64_t per_thread = total / ((uint64_t)blocks * threads);
  unsigned long long *cnt;
  double *first;
  hipMalloc(&cnt, 4 * sizeof(unsigned long long));
  hipMalloc(&first, 4 * sizeof(double));
  int rc = 0;
  for (int dist = 0; dist < 4; ++dist) {
    hipMemset(cnt, 0, 4 * sizeof(unsigned long long));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(check, dim3(blocks), dim3(threads), 0, 0, dist, per_thread,
                       0x5eed0000ull + dist, cnt, first);
    hipEventRecord(e1);
    if (hipDeviceSynchronize() != hipSuccess) {
      fprintf(stderr, "kernel failed\n");
      return 2;
    }
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[4];
    double f[4];
    hipMemcpy(h, cnt, sizeof h, hipMemcpyDeviceToHost);
    hipMemcpy(f, first, sizeof f, hipMemcpyDeviceToHost);
    printf("{\"dist\": %d, \"pairs\": %llu, \"fused_vs_ref_mismatch\": %llu, "
           "\"core_vs_ref_mismatch\": %llu, \"ms\": %.1f",
           dist, (unsigned long long)(per_thread * blocks * threads), h[0], h[1], ms);
    if (h[0]) printf(", \"first\": [%.17g, %.17g, %.17g, %.17g]", f[0], f[1], f[2], f[3]);
    printf("}\n");
    if (h[0] || h[1]) rc = 1;
  }
  return rc;
}
