// quot_fab_check.hip -- the (d, x) pairs of real FABRIK solves (general
// arithmetic, fabrik_step4's order) against quot_sqrt_core: for every
// get_point_between of every iteration of every goal in a raw float64 n x 3 file,
// is quot_sqrt_core(d, x) == d / sqrt(x) == div_core(d, sqrt_core(x)) where x is
// in sqrt_core's domain?  Prints mismatch counts and the first few pairs.
//   tools/quot_fab_check goals.f64 tol max_iter
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../inversekinematicsann_amd/csrc/ik_common.h"
#include "quot_fused.h"

using namespace ikhip;

struct Mis {
  double d, x, q_gen, q_fused, q_core;
};

__device__ void chk(double d, double x, unsigned long long *cnt, Mis *m) {
  if (sqrt_core_dom(x) >= kCoreDom) return;
  const double qg = d / sqrt(x), qf = quot_sqrt_core(d, x), qc = div_core(d, sqrt_core(x));
  const bool bf = __double_as_longlong(qf) != __double_as_longlong(qg);
  const bool bc = __double_as_longlong(qc) != __double_as_longlong(qg);
  atomicAdd(&cnt[0], 1ull);
  if (bf) {
    const unsigned long long k = atomicAdd(&cnt[1], 1ull);
    if (k < 16) m[k] = {d, x, qg, qf, qc};
  }
  if (bc) atomicAdd(&cnt[2], 1ull);
}

__device__ d3 pb(d3 s, d3 e, double d, unsigned long long *cnt, Mis *m) {
  const double dx = e.x - s.x, dy = e.y - s.y, dz = e.z - s.z;
  const double x = sq(dx) + sq(dy) + sq(dz);
  chk(d, x, cnt, m);
  const double q = d / sqrt(x);
  return {s.x + (q * dx), s.y + (q * dy), s.z + (q * dz)};
}

__global__ void run(const double *g3, int n, double tol2, int max_iter, unsigned long long *cnt,
                    Mis *m) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const d3 g = {g3[3 * i], g3[3 * i + 1], g3[3 * i + 2]};
  // seed: straight up from the shoulder (0, 0, 2), joints at 2 / 4 / 6 above it,
  // rotated to the goal's azimuth (the seed's exact bits do not matter here)
  const double t1 = atan2(g.y, g.x), c = cos(t1), s = sin(t1);
  const d3 start = {0.0, 0.0, 2.0};
  d3 c1 = {1e-16 * c, 1e-16 * s, 4.0}, c2 = {2e-16 * c, 2e-16 * s, 6.0},
     c3 = {3e-16 * c, 3e-16 * s, 8.0};
  double se = 1.0, ge = 1.0;
  for (int it = 0; it < max_iter && (se > tol2 || ge > tol2); ++it) {
    d3 b2 = pb(g, c2, 2.0, cnt, m);
    d3 b1 = pb(b2, c1, 2.0, cnt, m);
    d3 b0 = pb(b1, start, 2.0, cnt, m);
    se = dist3_sq(b0, start);
    c1 = pb(start, b1, 2.0, cnt, m);
    c2 = pb(c1, b2, 2.0, cnt, m);
    c3 = pb(c2, g, 2.0, cnt, m);
    ge = dist3_sq(c3, g);
  }
}

int main(int argc, char **argv) {
  if (argc < 4) return 2;
  FILE *f = fopen(argv[1], "rb");
  if (!f) return 2;
  std::vector<double> h;
  double v;
  while (fread(&v, 8, 1, f) == 1) h.push_back(v);
  fclose(f);
  const int n = (int)(h.size() / 3);
  const double tol = atof(argv[2]);
  const int mi = atoi(argv[3]);
  double *dg;
  unsigned long long *cnt;
  Mis *m;
  (void)hipMalloc(&dg, h.size() * 8);
  (void)hipMalloc(&cnt, 3 * 8);
  (void)hipMalloc(&m, 16 * sizeof(Mis));
  (void)hipMemcpy(dg, h.data(), h.size() * 8, hipMemcpyHostToDevice);
  (void)hipMemset(cnt, 0, 24);
  hipLaunchKernelGGL(run, dim3((n + 255) / 256), dim3(256), 0, 0, dg, n, tol * tol, mi, cnt, m);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  unsigned long long c[3];
  Mis hm[16];
  (void)hipMemcpy(c, cnt, 24, hipMemcpyDeviceToHost);
  (void)hipMemcpy(hm, m, sizeof hm, hipMemcpyDeviceToHost);
  printf("{\"goals\": %d, \"tol\": %g, \"pairs\": %llu, \"fused_mismatch\": %llu, \"core_mismatch\": %llu}\n",
         n, tol, c[0], c[1], c[2]);
  for (unsigned long long k = 0; k < c[1] && k < 16; ++k)
    printf("  d %.17g x %a q_gen %a q_fused %a q_core %a\n", hm[k].d, hm[k].x, hm[k].q_gen,
           hm[k].q_fused, hm[k].q_core);
  return 0;
}
