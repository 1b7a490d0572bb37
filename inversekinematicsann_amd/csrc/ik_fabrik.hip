// ik_fabrik.hip -- batched FABRIK inverse kinematics for gfx950.
//
// Restates, one goal point per lane in float64, the reference's
//   FabrikInverseKinematics.ikine   kinematics/inverse.py:115-139
//   Fabrik.calculate / __backward / __forward   kinematics/fabrik.py:19-67
//   __get_angles                    kinematics/inverse.py:54-112
// with the same operation order, so iteration counts are bit-exact.
//
// Two pipelines (DESIGN.md "FABRIK"):
//  * split (default): seed_kernel (limits + FK seed pose) -> iter_kernel
//    (persistent; a lane whose point converged is refilled from a per-wave
//    chunk of a global work queue, so a wave no longer waits for its slowest
//    lane) -> angles_kernel (law of cosines + per-batch stats).
//  * simple: everything in one kernel, one point per lane, no refill.
// Per point the state is 4 joints + goal (15 doubles) held in VGPRs.
#include <atomic>
#include <cmath>

#include "ik_common.h"

namespace ikhip {

// One FABRIK iteration for the 4-joint chain (fabrik.py:57-64): backward pass
// from the goal (dists[2], dists[1], dists[0]), start error, forward pass from
// the start (dists[1], dists[2], dists[3]), goal error.  cur[0] is always start.
// The two errors are returned SQUARED (the radicands of get_distance_between):
// they are only compared with tol (fabrik.py:57), and sqrt(x) > tol <=> x > t
// for t = tol_threshold(tol) exactly, sqrt being correctly rounded and monotonic.
__device__ __forceinline__ void fabrik_step4(const d3 start, d3 &c1, d3 &c2, d3 &c3,
                                             const d3 g, const double *L, double &se2,
                                             double &ge2, int &st) {
  d3 b2 = point_between(g, c2, L[2], st);
  d3 b1 = point_between(b2, c1, L[1], st);
  d3 b0 = point_between(b1, start, L[0], st);
  se2 = dist3_sq(b0, start);
  c1 = point_between(start, b1, L[1], st);
  c2 = point_between(c1, b2, L[2], st);
  c3 = point_between(c2, g, L[3], st);
  ge2 = dist3_sq(c3, g);
}

// fabrik_step4 through point_between_core: the same bits wherever dom comes back
// below kCoreDom (then no ZeroDivisionError is possible either).  The six radicands are
// checked against sqrt_core's domain instead of carrying the general sqrt /
// division's range handling: ~22 % fewer instructions per iteration.
__device__ __forceinline__ void fabrik_step4_core(const d3 start, d3 &c1, d3 &c2, d3 &c3,
                                                  const d3 g, const double *L, double &se2,
                                                  double &ge2, uint32_t &dom) {
  d3 b2 = point_between_core(g, c2, L[2], dom);
  d3 b1 = point_between_core(b2, c1, L[1], dom);
  d3 b0 = point_between_core(b1, start, L[0], dom);
  se2 = dist3_sq(b0, start);
  c1 = point_between_core(start, b1, L[1], dom);
  c2 = point_between_core(c1, b2, L[2], dom);
  c3 = point_between_core(c2, g, L[3], dom);
  ge2 = dist3_sq(c3, g);
}

// fabrik_step4_core with the two distances the reference computes twice taken once
// (links L0 == L1 and L2 == L3, bitwise; the host checks):
//  * b0 = pb(b1, start, L0) and c1 = pb(start, b1, L1) share |b1 - start| (the
//    radicand squares start - b1 = -(b1 - start) exactly) and, with L0 == L1, the
//    quotient, so c1 = start + q*(b1 - start) = start - q*(start - b1);
//  * this iteration's c3 = pb(c2, g, L3) and the next one's b2 = pb(g, c2, L2) share
//    |c2 - g| and, with L2 == L3, the quotient: the lane carries (cq, cd = g - c2)
//    into the next iteration, whose b2 = g + cq*(c2 - g) = g - cq*cd.
// Every value is the one the reference computes (IEEE: a + (-b) == a - b and
// q*(-d) == -(q*d)), so the bits do not change; two of the six square roots and
// divisions per iteration go.  cdom is the carried radicand's domain value: it joins
// dom so that the wave-uniform fallback still sees it.
__device__ __forceinline__ void fabrik_step4_reuse(const d3 start, d3 &c1, d3 &c2, d3 &c3,
                                                   const d3 g, const double *L, double &se2,
                                                   double &ge2, double &cq, d3 &cd,
                                                   uint32_t &cdom, uint32_t &dom) {
  dom = cdom;
  const d3 b2 = {g.x - cq * cd.x, g.y - cq * cd.y, g.z - cq * cd.z};
  const d3 b1 = point_between_core(b2, c1, L[1], dom);
  const double dx = start.x - b1.x, dy = start.y - b1.y, dz = start.z - b1.z;
  const double x = sq(dx) + sq(dy) + sq(dz);
  dom = max(dom, sqrt_core_dom(x));
  const double q = div_core(L[0], sqrt_core(x));
  const d3 b0 = {b1.x + (q * dx), b1.y + (q * dy), b1.z + (q * dz)};
  se2 = dist3_sq(b0, start);
  c1 = {start.x - (q * dx), start.y - (q * dy), start.z - (q * dz)};
  c2 = point_between_core(c1, b2, L[2], dom);
  const double ex = g.x - c2.x, ey = g.y - c2.y, ez = g.z - c2.z;
  const double x3 = sq(ex) + sq(ey) + sq(ez);
  cdom = sqrt_core_dom(x3);
  dom = max(dom, cdom);
  cq = div_core(L[3], sqrt_core(x3));
  c3 = {c2.x + (cq * ex), c2.y + (cq * ey), c2.z + (cq * ez)};
  cd = {ex, ey, ez};
  ge2 = dist3_sq(c3, g);
}

// The carry of fabrik_step4_reuse for a chain whose c2 did not come from it (a
// refilled lane's seed pose, or the general step of a fallback), through the
// general sqrt / division: the same bits inside sqrt_core's domain, and outside it
// cdom sends the next iteration to the fallback, which recomputes everything.
__device__ __forceinline__ void reuse_carry(const d3 c2, const d3 g, double L3, double &cq,
                                            d3 &cd, uint32_t &cdom) {
  cd = {g.x - c2.x, g.y - c2.y, g.z - c2.z};
  const double x = sq(cd.x) + sq(cd.y) + sq(cd.z);
  cdom = sqrt_core_dom(x);
  cq = L3 / sqrt(x);
}

// div_core's domain for the link lengths (the numerators): 2^-100 <= |L| <= 2^100.
static bool links_core_ok(const double *L, int n) {
  for (int k = 0; k < n; ++k) {
    const double v = std::fabs(L[k]);
    if (!(v >= 0x1p-100 && v <= 0x1p100)) return false;
  }
  return true;
}

// The largest x with fl(sqrt(x)) <= tol (NaN for a NaN tol, -inf for a
// negative one), so that the reference's `sqrt(x) > tol` is `x > t` bit for
// bit.  The loop's initial errors of 1.0 stay 1.0 (sqrt(1) = 1 exactly).
static double tol_threshold(double tol) {
  if (std::isnan(tol)) return NAN;
  if (tol < 0) return -INFINITY;
  if (std::isinf(tol)) return INFINITY;
  double t = tol * tol;
  while (std::sqrt(t) > tol) t = std::nextafter(t, -INFINITY);
  for (;;) {
    const double u = std::nextafter(t, INFINITY);
    if (std::sqrt(u) <= tol) t = u;
    else break;
  }
  return t;
}

// kinematics/inverse.py:54-112 __get_angles; J = FABRIK joints B, C, D, E.
__device__ __forceinline__ void get_angles(const d3 J[4], double th[4], int &st) {
  const d3 A = {0.0, 0.0, 0.0};
  const d3 B = J[0], C = J[1], D = J[2], E = J[3];
  th[0] = atan2(E.y, E.x);
  double ab = dist3(A, B), bc = dist3(B, C), cd = dist3(C, D), de = dist3(D, E);
  double ac = dist3(A, C);
  double num = (sq(ab) + sq(bc)) - sq(ac);
  double den = 2 * ab * bc;
  double a2 = py_acos(py_round8(py_div(num, den, st)), st);
  th[1] = (C.x * D.x < 0) ? ((3 * kPi / 2) - a2) : -(kPi / 2 - a2);
  double bd = dist3(B, D);
  num = (sq(bc) + sq(cd)) - sq(bd);
  den = 2 * bc * cd;
  double a3 = py_acos(py_round8(py_div(num, den, st)), st);
  th[2] = -(kPi - a3);
  double ce = dist3(C, E);
  num = (sq(cd) + sq(de)) - sq(ce);
  den = 2 * cd * de;
  double a4 = py_acos(py_round8(py_div(num, den, st)), st);
  d3 m = point_between(C, E, dist3(C, E) / 2, st);
  double da = dist3(B, m);
  double db = dist3(B, D);
  th[3] = (db > da) ? -(kPi - a4) : (kPi - a4);
}

// Seed pose, inverse.py:123-130: FK of [atan2(y, x), thetas[1:]] (the
// reference writes theta_1 into dh_matrix[0][0] and runs fkine on that row),
// through the per-robot constants (seed_chain; same bits as fk_chain).
__device__ __forceinline__ int seed_pose(const RobotDev &r, const RobotConstDev *rc, d3 g,
                                         d3 J[4]) {
  return seed_chain(r.dh, rc, atan2(g.y, g.x), J);
}

__global__ void robot_const_kernel(RobotDev r, RobotConstDev *rc) {
  if (threadIdx.x != 0) return;
  int st = IK_OK;
  for (int k = 1; k < 4; ++k) {
    dh_transform(r.dh[k], r.dh[4 + k], r.dh[8 + k], r.dh[12 + k], rc->A[k - 1]);
    if (!angle_ok(r.dh[k])) st = IK_E_ANGLE_RANGE;
  }
  for (int k = 0; k < 4; ++k)
    if (!angle_ok(r.dh[12 + k])) st = IK_E_ANGLE_RANGE;
  const double al = r.dh[12];
  rc->ca1 = cos(al);
  rc->sa1 = sin(al);
  rc->st = st;
}

void launch_robot_const(const RobotDev &r, RobotConstDev *rc, hipStream_t stream) {
  hipLaunchKernelGGL(robot_const_kernel, dim3(1), dim3(64), 0, stream, r, rc);
}

__device__ __forceinline__ void store_joints(double *dst, int64_t i, const d3 J[4]) {
  double *p = dst + 12 * i;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    p[3 * k] = J[k].x;
    p[3 * k + 1] = J[k].y;
    p[3 * k + 2] = J[k].z;
  }
}

__device__ __forceinline__ void load_joints(const double *src, int64_t i, d3 J[4]) {
  const double2 *p = reinterpret_cast<const double2 *>(src + 12 * i);
  double2 v0 = p[0], v1 = p[1], v2 = p[2], v3 = p[3], v4 = p[4], v5 = p[5];
  J[0] = {v0.x, v0.y, v1.x};
  J[1] = {v1.y, v2.x, v2.y};
  J[2] = {v3.x, v3.y, v4.x};
  J[3] = {v4.y, v5.x, v5.y};
}


struct FabArgs {
  RobotDev r;
  const RobotConstDev *rc;  // seed constants (robot_const_kernel)
  const double *pts;
  int64_t n;
  double tol;      // fabrik.py:57 err_margin, as given
  double tol2;     // tol_threshold(tol): the loop compares squared errors with it
  int max_iter;
  int check_limits;
  double *ang;
  int32_t *iters;
  double *joints;  // final joints (n x 12); never null in the split pipeline
  double *seeds;   // split pipeline scratch (n x 12)
  uint8_t *status; // split pipeline scratch (n)
  DevStats *S;
  int chunk;       // work-queue grab size of the persistent iteration kernel
  // hard-first ordering (see "Work order" below); unused when perm is null
  int32_t *perm;            // queue position -> point index
  uint8_t *status_in;       // ordered: the seed status by point
  uint16_t *cell;           // per point: goal cell (bits 0-9) | cost class << 10
  FabOrderDev *ord;         // context-owned cost table and class histogram
  int nseg, seg_blocks;     // histogram segments, and blocks per segment
  unsigned long long *dbg;  // diagnostic build only: iteration-kernel counters
};

// Diagnostic counters of the iteration kernel (-DIKHIP_DIAG, libikhip_diag.so,
// tools/fabrik_diag.py): per wave, summed into dbg[0..7], and per wave w at
// dbg[64 + 4w ..]: s_memrealtime (100 MHz) at start, when the queue ran dry
// for it and at the end, and the steps it ran after the queue ran dry.
enum { kDiagLoops, kDiagSteps, kDiagLaneSteps, kDiagRefills, kDiagGrabs, kDiagFallbacks,
       kDiagWaves, kDiagCount };
#ifdef IKHIP_DIAG
constexpr int kDiagWaveMax = 4000;  // = (kFabrikDebugWords - 64) / 4
#endif

static int env_int(const char *name, int dflt) {
  const char *v = getenv(name);
  return (v && *v) ? atoi(v) : dflt;
}

// ------------------------------------------------------------- simple ----
__global__ __launch_bounds__(256) void fabrik_simple_kernel(FabArgs a) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool valid = i < a.n;
  int it = 0;
  if (valid) {
    d3 g = {a.pts[3 * i], a.pts[3 * i + 1], a.pts[3 * i + 2]};
    if (a.check_limits && outside(a.r.lim, g.x, g.y, g.z))
      atomicMin(&a.S->first_oob, (unsigned long long)i);
    d3 J[4];
    int st = seed_pose(a.r, a.rc, g, J);
    double se = 1.0, ge = 1.0;
    if (st == IK_OK) {
      while (((se > a.tol2) || (ge > a.tol2)) && (a.max_iter > it)) {
        fabrik_step4(J[0], J[1], J[2], J[3], g, a.r.links, se, ge, st);
        ++it;
        if (st != IK_OK) break;
      }
    }
    double th[4] = {__builtin_nan(""), __builtin_nan(""), __builtin_nan(""), __builtin_nan("")};
    if (st == IK_OK) get_angles(J, th, st);
    if (st != IK_OK) record_error(a.S, i, st);
    double2 *o = reinterpret_cast<double2 *>(a.ang + 4 * i);
    o[0] = make_double2(th[0], th[1]);
    o[1] = make_double2(th[2], th[3]);
    if (a.iters) a.iters[i] = it;
    if (a.joints) store_joints(a.joints, i, J);
  }
  block_iter_stats(a.S, valid, it, a.max_iter);
}

// -------------------------------------------------------------- split ----
// 1. limits + seed pose (uniform work, one point per lane).  ORD (work order
// below): also the goal's cell and the per-segment counts of its cost class.
template <bool ORD>
__global__ __launch_bounds__(256) void fabrik_seed_kernel(FabArgs a);

// ---------------------------------------------------------- Work order ----
// The persistent iteration kernel hands points out in queue order.  In point
// order a 100-iteration point can be picked up just before the queue runs dry
// and set the launch length alone (≈ 1.4x the lane-iterations / lanes bound
// at 1M random_dist points).  Handing out the expensive points first removes
// most of that tail.  The cost of a point is predicted from its goal cell --
// distance from the shoulder (the first joint) in 64 bins up to the reach of
// links 1..3, and the sine of the elevation in 16 bins -- by the LARGEST
// iteration count the context recorded in that cell on earlier calls (1 point
// in kOrdSample; the old key decays by 1/8 when new records arrive).  The
// largest, not the mean: what sets the tail is a long point starting late, and
// long points (9 % of random_dist points take >= 80 of 100 iterations) sit in
// cells of every mean.  A list-scheduling simulation of 131k lanes on 1M
// reference iteration counts (tol 1e-3 / 1e-5): point order 1.29x / 1.34x the
// lane-iterations / lanes bound, cells by mean 1.15x / 1.23x, cells by sampled
// max 1.04x / 1.03x, exact longest-first 1.01x.  Unseen cells count as hard.
// Costs map to 16 classes; a counting sort (class-major, hardest first; order
// inside a class is whatever the atomics give) yields the queue -> point
// permutation.  Results do not depend on the order: every point is still
// solved by the same arithmetic on its own.
//
// Launches: seed (+ class counts) -> scan (1 block; + folds the previous
// call's records into the table) -> scatter -> iterate -> angles (+ records,
// + clears the class counts).  (Doing the one-block steps in the last block of
// the kernel before, found with a ticket counter, measured 0.6 ms: 4k
// same-address returning atomics.)
constexpr int kOrdSegBlocksMin = 16;  // histogram segment: >= 16 blocks of 256 points

__device__ __forceinline__ int goal_cell(const RobotDev &r, d3 g, d3 shoulder) {
  const double dx = g.x - shoulder.x, dy = g.y - shoulder.y, dz = g.z - shoulder.z;
  const double dist = sqrt(dx * dx + dy * dy + dz * dz);
  const double reach = r.links[1] + r.links[2] + r.links[3];
  int rb = (int)(dist / reach * kOrdCellsR);
  rb = rb < 0 ? 0 : (rb >= kOrdCellsR ? kOrdCellsR - 1 : rb);
  int eb = dist > 0.0 ? (int)((dz / dist + 1.0) * (0.5 * kOrdCellsE)) : kOrdCellsE / 2;
  eb = eb < 0 ? 0 : (eb >= kOrdCellsE ? kOrdCellsE - 1 : eb);
  return rb * kOrdCellsE + eb;
}

__device__ __forceinline__ int cost_class(const FabOrderDev *T, int cell, int max_iter) {
  const unsigned int key = T->key[cell];  // 1 + largest recorded iterations, 0 = unseen
  if (key == 0) return kOrdClasses - 1;
  const int k = (int)((long long)(key - 1) * kOrdClasses / (max_iter + 1));
  return k < 0 ? 0 : (k >= kOrdClasses ? kOrdClasses - 1 : k);
}

// Exclusive scan of the class counts in queue order (hardest class first,
// then segment), in place: hist becomes the per-(class, segment) cursors the
// scatter advances.  One block.
__device__ void order_scan(FabOrderDev *T, int nseg) {
  __shared__ uint32_t part[256];
  const int t = threadIdx.x;
  const int E = kOrdClasses * nseg;
  const int per = (E + 255) / 256, b0 = t * per, b1 = min(E, b0 + per);
  // scan position e = class (kOrdClasses-1 - e / nseg), segment e % nseg
  auto at = [&](int e) { return (kOrdClasses - 1 - e / nseg) * nseg + e % nseg; };
  // the counts are read kScanBatch at a time with independent loads (a plain
  // loop waits out one memory latency per entry: 15 us per call at 1M points)
  constexpr int kScanBatch = 16;
  uint32_t s = 0;
  for (int e0 = b0; e0 < b1; e0 += kScanBatch) {
    uint32_t v[kScanBatch];
#pragma unroll
    for (int j = 0; j < kScanBatch; ++j) v[j] = (e0 + j < b1) ? T->hist[at(e0 + j)] : 0u;
#pragma unroll
    for (int j = 0; j < kScanBatch; ++j) s += v[j];
  }
  part[t] = s;
  __syncthreads();
  for (int d = 1; d < 256; d <<= 1) {  // inclusive Hillis-Steele scan
    const uint32_t v = (t >= d) ? part[t - d] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - s;
  for (int e0 = b0; e0 < b1; e0 += kScanBatch) {
    uint32_t v[kScanBatch];
#pragma unroll
    for (int j = 0; j < kScanBatch; ++j) v[j] = (e0 + j < b1) ? T->hist[at(e0 + j)] : 0u;
#pragma unroll
    for (int j = 0; j < kScanBatch; ++j) {
      if (e0 + j < b1) T->hist[at(e0 + j)] = run;
      run += v[j];
    }
  }
}

// Fold the records into the table: per cell, the largest recorded iteration
// count of the call, or the decayed old key if larger.  One block.
__device__ void order_fold(FabOrderDev *T) {
  __shared__ unsigned int lm[kOrdCells];
  const int t = threadIdx.x;
  for (int c = t; c < kOrdCells; c += 256) lm[c] = 0;
  __syncthreads();
  const unsigned int ns = T->nsample < kOrdMaxSample ? T->nsample : kOrdMaxSample;
  constexpr int kFoldBatch = 8;  // independent loads in flight (as in order_scan)
  for (unsigned int k0 = t; k0 < ns; k0 += 256 * kFoldBatch) {
    unsigned int v[kFoldBatch];
#pragma unroll
    for (int j = 0; j < kFoldBatch; ++j) {
      const unsigned int k = k0 + 256u * j;
      v[j] = k < ns ? T->sample[k] : 0xffffffffu;
    }
#pragma unroll
    for (int j = 0; j < kFoldBatch; ++j)
      if (v[j] != 0xffffffffu) atomicMax(&lm[v[j] >> 16], (v[j] & 0xffffu) + 1u);
  }
  __syncthreads();
  for (int c = t; c < kOrdCells; c += 256) {
    if (lm[c]) {
      const unsigned int old = T->key[c];
      const unsigned int dec = old - (old >> 3);
      T->key[c] = lm[c] > dec ? lm[c] : dec;
    }
  }
  if (t == 0) T->nsample = 0;
}

// One block: this call's class counts -> cursors, then the previous call's
// records -> the table (which the next call's seed kernel reads: the table
// lags one call, which costs nothing but saves a launch).
__global__ __launch_bounds__(256) void fabrik_order_scan_kernel(FabOrderDev *T, int nseg) {
  order_scan(T, nseg);
  __syncthreads();
  order_fold(T);
}

template <bool ORD>
__global__ __launch_bounds__(256) void fabrik_seed_kernel(FabArgs a) {
  __shared__ unsigned int cnt[kOrdClasses];
  const int t = threadIdx.x;
  if (ORD) {
    if (t < kOrdClasses) cnt[t] = 0;
    __syncthreads();
  }
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + t;
  if (i < a.n) {
    d3 g = {a.pts[3 * i], a.pts[3 * i + 1], a.pts[3 * i + 2]};
    if (a.check_limits && outside(a.r.lim, g.x, g.y, g.z))
      atomicMin(&a.S->first_oob, (unsigned long long)i);
    d3 J[4];
    int st = seed_pose(a.r, a.rc, g, J);
    store_joints(a.seeds, i, J);
    if constexpr (ORD) {
      a.status_in[i] = (uint8_t)st;
      const int cell = goal_cell(a.r, g, J[0]);
      const int k = cost_class(a.ord, cell, a.max_iter);
      a.cell[i] = (uint16_t)(cell | (k << 10));  // the scatter must see this very class
      atomicAdd(&cnt[k], 1u);
    } else {
      a.status[i] = (uint8_t)st;
    }
  }
  if constexpr (ORD) {
    __syncthreads();
    if (t < kOrdClasses && cnt[t])
      atomicAdd(&a.ord->hist[t * a.nseg + blockIdx.x / a.seg_blocks], cnt[t]);
  }
}

// scatter: perm[cursor] = point (one point per lane; one atomic per class
// and block claims the block's range of each class in its segment)
__global__ __launch_bounds__(256) void fabrik_order_scatter_kernel(FabArgs a) {
  __shared__ uint32_t wcnt[4][kOrdClasses], base[kOrdClasses];
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + t;
  const int k = (i < a.n) ? (a.cell[i] >> 10) : -1;
  const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  int rank = 0;
#pragma unroll
  for (int c = 0; c < kOrdClasses; ++c) {
    const unsigned long long m = __ballot(k == c);
    if (k == c) rank = __popcll(m & lt);
    if (lane == 0) wcnt[w][c] = (uint32_t)__popcll(m);
  }
  __syncthreads();
  if (t < kOrdClasses) {
    const uint32_t tot = wcnt[0][t] + wcnt[1][t] + wcnt[2][t] + wcnt[3][t];
    base[t] = tot ? atomicAdd(&a.ord->hist[t * a.nseg + blockIdx.x / a.seg_blocks], tot) : 0u;
  }
  __syncthreads();
  if (k >= 0) {
    uint32_t pos = base[k] + rank;
    for (int v = 0; v < w; ++v) pos += wcnt[v][k];
    a.perm[pos] = (int32_t)i;
  }
}

// 2. persistent iteration with per-lane refill.
// a.chunk: points a wave takes from the global queue at once (tuning knob,
// IKHIP_FABRIK_CHUNK; small enough that every wave gets work at 1M points).

// ORD: the queue is a.perm (work order above): a refilled lane gathers its
// point's seed pose and goal and keeps the point's index, where its results go
// (so the angles kernel reads them in point order, coalesced).
// CORE: 0 general sqrt / division, 1 sqrt_core / div_core, 2 the same with the
// repeated distances taken once (fabrik_step4_reuse; needs L0 == L1 and L2 == L3).
template <int REFILL_MIN, bool ORD, int CORE>
__global__ __launch_bounds__(256) void fabrik_iter_kernel(FabArgs a) {
  const int lane = threadIdx.x & 63;
  const unsigned long long lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const double tol2 = a.tol2;
  const int max_iter = a.max_iter;
  double L[4] = {a.r.links[0], a.r.links[1], a.r.links[2], a.r.links[3]};

  int64_t qnext = 0, qend = 0;  // wave-uniform: indices not yet handed out
  bool exhausted = false;
  bool active = false;
  int64_t idx = 0;  // queue position (= the point index unless ORD)
  int64_t out = 0;  // the point index: where the lane's results go
  d3 J0 = {0, 0, 0}, J1 = J0, J2 = J0, J3 = J0, g = J0;
  double se = 1.0, ge = 1.0;
  int step = 0, st = IK_OK;
  double cq = 0.0;  // CORE == 2: the carried quotient, offset and domain value
  d3 cd = J0;
  uint32_t cdom = 0;

#ifdef IKHIP_DIAG
  unsigned long long dg[kDiagCount] = {};
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
  unsigned long long t_dry = 0, steps_dry = 0;
#define IKHIP_DG(k, v) (dg[k] += (v))
#else
#define IKHIP_DG(k, v) ((void)0)
#endif
  while (true) {
    unsigned long long freem = __ballot(!active);
    int nfree = __popcll(freem);
    if (exhausted && nfree == 64) break;
    IKHIP_DG(kDiagLoops, 1);
    if (!exhausted && (nfree >= REFILL_MIN || nfree == 64)) {
      IKHIP_DG(kDiagRefills, 1);
      int rank = __popcll(freem & lt_mask);
      int64_t mine = -1;
      int handed = 0;
      while (handed < nfree) {
        if (qnext >= qend) {
          IKHIP_DG(kDiagGrabs, 1);
          unsigned long long old = 0;
          if (lane == 0) old = atomicAdd(&a.S->queue, (unsigned long long)a.chunk);
          old = __shfl(old, 0, 64);
          if ((int64_t)old >= a.n) {
            exhausted = true;
            break;
          }
          qnext = (int64_t)old;
          qend = min((int64_t)old + a.chunk, a.n);
        }
        int take = (int)min((int64_t)(nfree - handed), qend - qnext);
        if (!active && rank >= handed && rank < handed + take) mine = qnext + (rank - handed);
        qnext += take;
        handed += take;
      }
      if (mine >= 0) {
        idx = mine;
        d3 Jn[4];
        if constexpr (ORD) {
          const int64_t p = a.perm[idx];
          st = a.status_in[p];
          load_joints(a.seeds, p, Jn);
          g = {a.pts[3 * p], a.pts[3 * p + 1], a.pts[3 * p + 2]};
          out = p;
        } else {
          st = a.status[idx];
          load_joints(a.seeds, idx, Jn);
          g = {a.pts[3 * idx], a.pts[3 * idx + 1], a.pts[3 * idx + 2]};
          out = idx;
        }
        // consume the gathered operands here: left pending, their loads made the
        // compiler put an s_waitcnt vmcnt(0) at the top of every step (the join
        // of the refill and no-refill paths), which also waited out the result
        // stores of the lanes that finished the step before
        asm volatile("" ::"v"(st), "v"(Jn[0].x), "v"(Jn[0].y), "v"(Jn[0].z), "v"(Jn[1].x),
                     "v"(Jn[1].y), "v"(Jn[1].z), "v"(Jn[2].x), "v"(Jn[2].y), "v"(Jn[2].z));
        asm volatile("" ::"v"(Jn[3].x), "v"(Jn[3].y), "v"(Jn[3].z), "v"(g.x), "v"(g.y),
                     "v"(g.z));
        J0 = Jn[0]; J1 = Jn[1]; J2 = Jn[2]; J3 = Jn[3];
        if constexpr (CORE == 2) reuse_carry(J2, g, L[3], cq, cd, cdom);
        se = 1.0;
        ge = 1.0;
        step = 0;
        active = true;
      }
    }
#ifdef IKHIP_DIAG
    {
      const unsigned long long sm =
          __ballot(active && st == IK_OK && ((se > tol2) || (ge > tol2)) && (max_iter > step));
      dg[kDiagSteps] += sm ? 1 : 0;
      dg[kDiagLaneSteps] += __popcll(sm);
      if (exhausted) {
        if (!t_dry) t_dry = __builtin_amdgcn_s_memrealtime();
        steps_dry += sm ? 1 : 0;
      }
    }
#endif
    if (active) {
      if (st == IK_OK && ((se > tol2) || (ge > tol2)) && (max_iter > step)) {
        if constexpr (CORE == 2) {
          uint32_t dom = 0, cdom_n = cdom;
          d3 n1 = J1, n2 = J2, n3 = J3, cd_n = cd;
          double se_n, ge_n, cq_n = cq;
          fabrik_step4_reuse(J0, n1, n2, n3, g, L, se_n, ge_n, cq_n, cd_n, cdom_n, dom);
          if (__all(dom < kCoreDom)) {
            J1 = n1; J2 = n2; J3 = n3;
            se = se_n;
            ge = ge_n;
            cq = cq_n;
            cd = cd_n;
            cdom = cdom_n;
          } else {
            IKHIP_DG(kDiagFallbacks, 1);
            fabrik_step4(J0, J1, J2, J3, g, L, se, ge, st);
            reuse_carry(J2, g, L[3], cq, cd, cdom);
          }
        } else if constexpr (CORE == 1) {
          // wave-uniform fallback: when any lane's radicand leaves sqrt_core's
          // domain (coincident joints, non-finite input) the wave redoes the
          // iteration with the general sqrt / division (and their errors)
          uint32_t dom = 0;
          d3 n1 = J1, n2 = J2, n3 = J3;
          double se_n, ge_n;
          fabrik_step4_core(J0, n1, n2, n3, g, L, se_n, ge_n, dom);
          if (__all(dom < kCoreDom)) {
            J1 = n1; J2 = n2; J3 = n3;
            se = se_n;
            ge = ge_n;
          } else {
            IKHIP_DG(kDiagFallbacks, 1);
            fabrik_step4(J0, J1, J2, J3, g, L, se, ge, st);
          }
        } else {
          fabrik_step4(J0, J1, J2, J3, g, L, se, ge, st);
        }
        ++step;
      } else {
        d3 J[4] = {J0, J1, J2, J3};
        store_joints(a.joints, out, J);
        a.iters[out] = step;
        a.status[out] = (uint8_t)st;
        active = false;
      }
    }
  }
#ifdef IKHIP_DIAG
  if (a.dbg && lane == 0) {
    dg[kDiagWaves] = 1;
    for (int k = 0; k < kDiagCount; ++k) atomicAdd(&a.dbg[k], dg[k]);
    const int w = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    if (w < kDiagWaveMax) {
      a.dbg[64 + 4 * w] = t_start;
      a.dbg[65 + 4 * w] = t_dry;
      a.dbg[66 + 4 * w] = __builtin_amdgcn_s_memrealtime();
      a.dbg[67 + 4 * w] = steps_dry;
    }
  }
#endif
#undef IKHIP_DG
}

// 3. angles + stats (uniform work, one point per lane).  ORD: 1 in kOrdSample
// points records (cell, iterations) for the next call's cost table.
template <bool ORD>
__global__ __launch_bounds__(256) void fabrik_angles_kernel(FabArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool valid = i < a.n;
  int it = 0;
  if (valid) {
    int st = a.status[i];
    it = a.iters[i];
    d3 J[4];
    double th[4] = {__builtin_nan(""), __builtin_nan(""), __builtin_nan(""), __builtin_nan("")};
    if (st == IK_OK) load_joints(a.joints, i, J);
    if (st == IK_OK) get_angles(J, th, st);
    if (st != IK_OK) record_error(a.S, i, st);
    double2 *o = reinterpret_cast<double2 *>(a.ang + 4 * i);
    o[0] = make_double2(th[0], th[1]);
    o[1] = make_double2(th[2], th[3]);
    if constexpr (ORD) {
      if (i % kOrdSample == 0 && i / kOrdSample < kOrdMaxSample)
        a.ord->sample[i / kOrdSample] =
            ((uint32_t)(a.cell[i] & (kOrdCells - 1)) << 16) |
            (uint32_t)(it < 0xffff ? it : 0xffff);
    }
  }
  if constexpr (ORD) {
    if (i == 0) {
      const int64_t ns = (a.n + kOrdSample - 1) / kOrdSample;
      a.ord->nsample = (uint32_t)(ns < kOrdMaxSample ? ns : kOrdMaxSample);
    }
    if (i < (int64_t)kOrdClasses * a.nseg) a.ord->hist[i] = 0;  // for the next call
  }
  block_iter_stats(a.S, valid, it, a.max_iter);
}

static size_t up256(size_t b) { return (b + 255) & ~(size_t)255; }

size_t fabrik_scratch_bytes(int64_t n) {
  // seeds n*12 doubles, joints n*12 doubles, iters n int32, status n bytes;
  // work order: perm n int32, cell n uint16, seed status n bytes
  size_t b = 0;
  b += up256((size_t)n * 96);
  b += up256((size_t)n * 96);
  b += up256((size_t)n * 4);
  b += up256((size_t)n);
  b += up256((size_t)n * 4) + up256((size_t)n * 2) + up256((size_t)n);
  return b + 1024;
}

// CUs of the current device, cached per device index (relaxed atomics: every
// writer stores the same value)
static int num_cus() {
  static std::atomic<int> cache[64];
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::atomic<int> *slot = (dev >= 0 && dev < 64) ? &cache[dev] : nullptr;
  int v = slot ? slot->load(std::memory_order_relaxed) : 0;
  if (v <= 0) {
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        v <= 0)
      v = 256;
    if (slot) slot->store(v, std::memory_order_relaxed);
  }
  return v;
}

template <int REFILL_MIN, bool ORD>
static void launch_iter(int core, unsigned grid, hipStream_t stream, const FabArgs &a) {
  if (core == 2)
    hipLaunchKernelGGL((fabrik_iter_kernel<REFILL_MIN, ORD, 2>), dim3(grid), dim3(256), 0,
                       stream, a);
  else if (core == 1)
    hipLaunchKernelGGL((fabrik_iter_kernel<REFILL_MIN, ORD, 1>), dim3(grid), dim3(256), 0,
                       stream, a);
  else
    hipLaunchKernelGGL((fabrik_iter_kernel<REFILL_MIN, ORD, 0>), dim3(grid), dim3(256), 0,
                       stream, a);
}

void launch_fabrik_ikine(const RobotDev &r, const double *pts, int64_t n, double tol,
                         int max_iter, double *ang, int32_t *iters, double *joints,
                         bool check_limits, void *scratch, DevStats *S, hipStream_t stream,
                         int variant, int core_req, FabOrderDev *ord,
                         const RobotConstDev *rc, unsigned long long *dbg, int bpc_req) {
  if (n <= 0) return;
  FabArgs a;
  a.r = r;
  a.rc = rc;
  a.dbg = dbg;
  a.pts = pts;
  a.n = n;
  a.tol = tol;
  a.tol2 = tol_threshold(tol);
  a.max_iter = max_iter;
  a.check_limits = check_limits ? 1 : 0;
  a.ang = ang;
  a.iters = iters;
  a.joints = joints;
  a.S = S;
  a.chunk = 64;
  a.perm = nullptr;
  a.status_in = nullptr;
  a.cell = nullptr;
  a.ord = ord;
  a.nseg = 0;
  a.seg_blocks = 1;
  unsigned grid = (unsigned)((n + 255) / 256);
  if (variant == 0) {
    a.seeds = nullptr;
    a.status = nullptr;
    kt_begin("fabrik_simple_kernel", stream);
    hipLaunchKernelGGL(fabrik_simple_kernel, dim3(grid), dim3(256), 0, stream, a);
    kt_end(stream);
    return;
  }
  char *p = static_cast<char *>(scratch);
  a.seeds = reinterpret_cast<double *>(p);
  p += up256((size_t)n * 96);
  double *jtmp = reinterpret_cast<double *>(p);
  p += up256((size_t)n * 96);
  int32_t *itmp = reinterpret_cast<int32_t *>(p);
  p += up256((size_t)n * 4);
  a.status = reinterpret_cast<uint8_t *>(p);
  p += up256((size_t)n);
  static const int order_on = env_int("IKHIP_FABRIK_ORDER", 1);
  const bool ordered = ord && order_on && n < (int64_t)1 << 31;
  if (ordered) {
    // the iteration kernel writes its results by point index (a lane keeps its
    // point's index from the refill gather), straight into the caller's
    // (nullable) iterations / joints buffers
    a.perm = reinterpret_cast<int32_t *>(p);
    p += up256((size_t)n * 4);
    a.cell = reinterpret_cast<uint16_t *>(p);
    p += up256((size_t)n * 2);
    a.status_in = reinterpret_cast<uint8_t *>(p);
    a.seg_blocks = (int)((grid + kOrdMaxSeg - 1) / kOrdMaxSeg);
    if (a.seg_blocks < kOrdSegBlocksMin) a.seg_blocks = kOrdSegBlocksMin;
    a.nseg = (int)((grid + a.seg_blocks - 1) / a.seg_blocks);
    if (!a.joints) a.joints = jtmp;
    if (!a.iters) a.iters = itmp;
    kt_begin("fabrik_seed_kernel", stream);
    hipLaunchKernelGGL(fabrik_seed_kernel<true>, dim3(grid), dim3(256), 0, stream, a);
    kt_end(stream);
    kt_begin("fabrik_order_scan_kernel", stream);
    hipLaunchKernelGGL(fabrik_order_scan_kernel, dim3(1), dim3(256), 0, stream, ord, a.nseg);
    kt_end(stream);
    kt_begin("fabrik_order_scatter_kernel", stream);
    hipLaunchKernelGGL(fabrik_order_scatter_kernel, dim3(grid), dim3(256), 0, stream, a);
    kt_end(stream);
  } else {
    if (!a.joints) a.joints = jtmp;
    if (!a.iters) a.iters = itmp;
    kt_begin("fabrik_seed_kernel", stream);
    hipLaunchKernelGGL(fabrik_seed_kernel<false>, dim3(grid), dim3(256), 0, stream, a);
    kt_end(stream);
  }
  // persistent grid: blocks_per_cu 256-thread blocks per CU (= waves per SIMD)
  // measured on MI355X (tools/sweep_fabrik.py): at 1M points 2 blocks/CU with
  // 64-point grabs beats 4 and 8 by 10-30 % (more lanes = fewer points per lane
  // = a longer divergent tail); 2 and 3 are within noise at 1-1.25M points, and
  // from 4M points on 3 wins by ~5 % at every tolerance (the tail matters less
  // than the latency a third wave per SIMD hides), and so it does at 1M points
  // with tol 1e-5 (56 iterations per point against 33 at 1e-3: 0.559 vs 0.586 ms
  // per launch with the reuse iteration; at 1e-3 2 stays ahead, 0.386 vs 0.395).
  // (4M / 10M points at tol 1e-3: 4 per CU is 2 % ahead of 3; at 1e-5 they are even)
  // bpc_req: the context's IKHIP_FABRIK_BPC (0 = this rule)
  const int bpc = bpc_req > 0 ? bpc_req
                              : (n >= 4000000 && tol >= 1e-4) ? 4
                                                              : ((n >= 2000000 || tol < 1e-4) ? 3 : 2);
  static const int chunk = env_int("IKHIP_FABRIK_CHUNK", 64);
  a.chunk = chunk > 0 ? chunk : 64;
  unsigned pgrid = (unsigned)num_cus() * (unsigned)(bpc > 0 ? bpc : 8);
  int64_t waves_needed = (n + 63) / 64;
  if ((int64_t)pgrid * 4 > waves_needed)
    pgrid = (unsigned)((waves_needed + 3) / 4 > 0 ? (waves_needed + 3) / 4 : 1);
  // the iteration through sqrt_core / div_core (same bits, fewer instructions)
  // unless the link lengths are outside div_core's domain, and with the repeated
  // distances taken once (core 2) when L0 == L1 and L2 == L3.  core_req (context's
  // IKHIP_FABRIK_CORE) 0 forces the general sqrt / division, 1 the core sequences
  // without the reuse.
  const double *Lk = a.r.links;
  int core = links_core_ok(Lk, 4) ? core_req : 0;
  if (core == 2 && !(Lk[0] == Lk[1] && Lk[2] == Lk[3])) core = 1;
#ifdef IKHIP_DIAG
  if (a.dbg) (void)hipMemsetAsync(a.dbg, 0, kFabrikDebugWords * 8, stream);
#endif
  kt_begin("fabrik_iter_kernel", stream);
  if (variant == 2) {
    if (ordered) launch_iter<1, true>(core, pgrid, stream, a);
    else launch_iter<1, false>(core, pgrid, stream, a);
  } else {
    if (ordered) launch_iter<8, true>(core, pgrid, stream, a);
    else launch_iter<8, false>(core, pgrid, stream, a);
  }
  kt_end(stream);
  kt_begin("fabrik_angles_kernel", stream);
  if (ordered)
    hipLaunchKernelGGL(fabrik_angles_kernel<true>, dim3(grid), dim3(256), 0, stream, a);
  else
    hipLaunchKernelGGL(fabrik_angles_kernel<false>, dim3(grid), dim3(256), 0, stream, a);
  kt_end(stream);

}

// ------------------------------------------------------ Fabrik.calculate ----
template <int NJ>
__global__ __launch_bounds__(256) void fabrik_calc_kernel(const double *dists_in,
                                                          const double *init, int shared,
                                                          const double *goals, int64_t n,
                                                          double tol2, int max_iter,
                                                          double *joints, int32_t *iters,
                                                          DevStats *S) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool valid = i < n;
  int it = 0;
  if (valid) {
    double L[NJ];
#pragma unroll
    for (int k = 0; k < NJ; ++k) L[k] = dists_in[k];
    const double *ip = shared ? init : init + (size_t)i * NJ * 3;
    d3 cur[NJ], B[NJ];
#pragma unroll
    for (int k = 0; k < NJ; ++k) cur[k] = {ip[3 * k], ip[3 * k + 1], ip[3 * k + 2]};
    d3 g = {goals[3 * i], goals[3 * i + 1], goals[3 * i + 2]};
    const d3 start = cur[0];
    double se = 1.0, ge = 1.0;
    int st = IK_OK;
    while (((se > tol2) || (ge > tol2)) && (max_iter > it)) {  // squared errors
      B[NJ - 1] = g;
#pragma unroll
      for (int k = NJ - 2; k >= 0; --k) B[k] = point_between(B[k + 1], cur[k], L[k], st);
      se = dist3_sq(B[0], start);
      cur[0] = start;
#pragma unroll
      for (int k = 1; k < NJ; ++k) cur[k] = point_between(cur[k - 1], B[k], L[k], st);
      ge = dist3_sq(cur[NJ - 1], g);
      ++it;
      if (st != IK_OK) break;
    }
    if (st != IK_OK) record_error(S, i, st);
    double *o = joints + (size_t)i * NJ * 3;
#pragma unroll
    for (int k = 0; k < NJ; ++k) {
      o[3 * k] = cur[k].x;
      o[3 * k + 1] = cur[k].y;
      o[3 * k + 2] = cur[k].z;
    }
    if (iters) iters[i] = it;
  }
  block_iter_stats(S, valid, it, max_iter);
}

void launch_fabrik_calc(int nj, const double *dists, const double *init, bool init_shared,
                        const double *goals, int64_t n, double tol, int max_iter,
                        double *joints, int32_t *iters, DevStats *S, hipStream_t st) {
  if (n <= 0) return;
  unsigned grid = (unsigned)((n + 255) / 256);
  int sh = init_shared ? 1 : 0;
  const double tol2 = tol_threshold(tol);
#define IK_CALC_CASE(K)                                                                      \
  case K:                                                                                    \
    hipLaunchKernelGGL(fabrik_calc_kernel<K>, dim3(grid), dim3(256), 0, st, dists, init, sh, \
                       goals, n, tol2, max_iter, joints, iters, S);                          \
    break;
  kt_begin("fabrik_calc_kernel", st);
  switch (nj) {
    IK_CALC_CASE(2)
    IK_CALC_CASE(3)
    IK_CALC_CASE(4)
    IK_CALC_CASE(5)
    IK_CALC_CASE(6)
    IK_CALC_CASE(7)
    IK_CALC_CASE(8)
    default:
      break;
  }
  kt_end(st);
#undef IK_CALC_CASE
}

}  // namespace ikhip
