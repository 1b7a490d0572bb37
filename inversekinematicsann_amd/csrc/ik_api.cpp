// ik_api.cpp -- the C ABI of libikhip.so (declared in include/ikhip.h).
//
// Owns per-context state: the HIP stream, the device-side stats block, a
// grow-only device scratch buffer (host-pointer calls stage through it), the
// robot constants and the packed ANN weights.  No allocation happens inside a
// solve call once the scratch is large enough, so IK_F_DEVICE|IK_F_ASYNC calls
// can be captured in a hipGraph.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "ik_fabrik_prior.h"
#include "ik_internal.h"

using namespace ikhip;

namespace {

thread_local std::string g_last_error;

const double kDefaultDh[16] = {0.0, kPi / 2, 0.0, 0.0, 2.0, 0.0, 0.0, 0.0,
                               0.0, 2.0,     2.0, 2.0, kPi / 2, 0.0, 0.0, 0.0};
const double kDefaultLinks[4] = {2.0, 2.0, 2.0, 2.0};
const double kDefaultLimits[6] = {0.0, 6.0, -6.0, 6.0, -3.0, 6.0};

thread_local KTimer *g_kt = nullptr;

static_assert(sizeof(FabPrior::key) == sizeof(FabOrderDev::key), "prior = one cost table");

// The FABRIK work order's built-in tables (ik_fabrik_prior.h) describe
// SixDOFRobot's chain (robot/robot.py:38-42): dh rows d, a, alpha and thetas[1:],
// and the links.  theta_1 (dh[0]) is never read on the device.
bool default_chain(const RobotDev &r) {
  return std::memcmp(r.dh + 1, kDefaultDh + 1, 15 * sizeof(double)) == 0 &&
         std::memcmp(r.links, kDefaultLinks, sizeof(kDefaultLinks)) == 0;
}

// The built-in table for a solve's (tol, max_iter): the nearest in log10(tol),
// then max_iter; -1 without one.
int prior_for(double tol, int max_iter) {
  int best = -1;
  double bd = 0.0;
  for (int k = 0; k < kFabPriors; ++k) {
    const double lt = tol > 0.0 ? std::log10(tol) : -30.0;
    const double d = std::fabs(lt - std::log10(kFabPrior[k].tol)) * 1000.0 +
                     std::fabs((double)(max_iter - kFabPrior[k].max_iter));
    if (best < 0 || d < bd) {
      best = k;
      bd = d;
    }
  }
  return best;
}

}  // namespace

namespace ikapi {

// A fresh table for the context's robot: the built-in one that suits (tol,
// max_iter) when the chain is SixDOFRobot's, else empty (point order).
int seed_order(ik_ctx *c, double tol, int max_iter) {
  const int w = (c->fab_priors && default_chain(c->robot)) ? prior_for(tol, max_iter) : -1;
  if (w >= 0)
    IK_HIP(hipMemcpyAsync(c->fab_ord->key, c->fab_priors + (size_t)w * kOrdCells,
                          sizeof(c->fab_ord->key), hipMemcpyDeviceToDevice, c->stream));
  else
    IK_HIP(hipMemsetAsync(c->fab_ord->key, 0, sizeof(c->fab_ord->key), c->stream));
  c->fab_prior = w;
  return IK_OK;
}

}  // namespace ikapi

namespace ikhip {
void kt_begin(const char *name, hipStream_t) {
  if (!g_kt || !g_kt->on || g_kt->n >= kMaxTimed) return;
  g_kt->name[g_kt->n] = name;
  g_kt->state = 1;
}
void kt_span_begin(const char *name, hipStream_t st) {
  if (!g_kt || !g_kt->on || g_kt->n >= kMaxTimed) return;
  g_kt->name[g_kt->n] = name;
  g_kt->state = 3;
  (void)hipEventRecord(g_kt->beg[g_kt->n], st);
}
bool kt_take_events(hipEvent_t *beg, hipEvent_t *end) {
  if (!g_kt || !g_kt->on || g_kt->n >= kMaxTimed || g_kt->state != 1) return false;
  *beg = g_kt->beg[g_kt->n];
  *end = g_kt->end[g_kt->n];
  g_kt->state = 2;
  return true;
}
void kt_end(hipStream_t st) {
  if (!g_kt || !g_kt->on || g_kt->n >= kMaxTimed) return;
  if (g_kt->state == 3) (void)hipEventRecord(g_kt->end[g_kt->n], st);
  // a slot armed without a stamped launch (no kernel ran) is dropped
  if (g_kt->state == 2 || g_kt->state == 3) g_kt->n++;
  g_kt->state = 0;
}
}  // namespace ikhip

namespace ikapi {

int fail(int code, const std::string &msg) {
  g_last_error = msg;
  return code;
}

KtScope::KtScope(ik_ctx *c) : c_(c) {
  g_kt = &c->kt;
  if (!c->kt.acc) c->kt.n = 0;  // (accumulating: slots fill across calls, up to kMaxTimed)
  c->kt.state = 0;
  // calls on one context share its stats block and work-queue words: a call on
  // another stream than the last one starts after that one's work
  if (c->call_done_set && c->last_stream && c->last_stream != c->stream)
    (void)hipStreamWaitEvent(c->stream, c->call_done, 0);
  c->last_stream = c->stream;  // every enqueueing entry point opens one
  c->last_piped = false;
}
KtScope::~KtScope() {
  g_kt = nullptr;
  if (c_->call_done && hipEventRecord(c_->call_done, c_->stream) == hipSuccess)
    c_->call_done_set = true;
}

int ensure_scratch(ik_ctx *c, size_t bytes) {
  if (bytes <= c->scratch_bytes) return IK_OK;
  IK_HIP(hipStreamSynchronize(c->stream));
  if (c->scratch) IK_HIP(hipFree(c->scratch));
  c->scratch = nullptr;
  c->scratch_bytes = 0;
  size_t want = bytes + bytes / 4 + (1 << 20);
  IK_HIP(hipMalloc(&c->scratch, want));
  c->scratch_bytes = want;
  return IK_OK;
}

int set_dev(ik_ctx *c) {
  IK_HIP(hipSetDevice(c->device));
  return IK_OK;
}

void stats_from_dev(const DevStats &d, ik_stats *s) {
  std::memset(s, 0, sizeof(*s));
  s->first_oob = (d.first_oob == ~0ull) ? -1 : (int64_t)d.first_oob;
  if (d.first_err_key == ~0ull) {
    s->first_err = -1;
    s->first_err_code = IK_OK;
  } else {
    s->first_err = (int64_t)(d.first_err_key >> 8);
    s->first_err_code = (int32_t)(d.first_err_key & 0xff);
  }
  for (int i = 0; i < kStatShards; ++i) {
    s->max_iters = d.max_iters[i] > s->max_iters ? d.max_iters[i] : s->max_iters;
    s->sum_iters += (int64_t)d.sum_iters[i];
    s->n_capped += (int64_t)d.n_capped[i];
    double mx;
    std::memcpy(&mx, &d.max_fk_err_bits[i], sizeof(mx));
    s->max_fk_err = mx > s->max_fk_err ? mx : s->max_fk_err;
    s->sum_fk_err += d.sum_fk_err[i];
  }
}

int finish(ik_ctx *c, int flags, ik_stats *stats) {
  c->last_sharded = false;
  if (flags & IK_F_ASYNC) return IK_OK;
  IK_HIP(hipMemcpyAsync(c->h_stats, c->d_stats, sizeof(DevStats), hipMemcpyDeviceToHost,
                        c->stream));
  IK_HIP(hipStreamSynchronize(c->stream));
  if (stats) stats_from_dev(*c->h_stats, stats);
  return IK_OK;
}

}  // namespace ikapi

using namespace ikapi;

namespace ikapi {

// Device pointers only, on the context's stream: stats reset + the kernels.
int fabrik_launch(ik_ctx *c, const double *dp, int64_t n, double tol, int max_iter, double *da,
                  int32_t *di, double *dj, double *dfe, bool limits, void *work, DevStats *S) {
  if (!S) S = c->d_stats;
  // a table still holding a built-in prior takes the one for this call's
  // tolerance; the solve then folds its own records in (learned from here on)
  const bool prior = c->fab_prior >= 0 && n > 0;
  if (prior) {
    if (prior_for(tol, max_iter) != c->fab_prior) {
      const int rc = seed_order(c, tol, max_iter);
      if (rc) return rc;
    }
    c->fab_prior = -1;
  }
  launch_reset_stats(S, c->stream);
  launch_fabrik_ikine(c->robot, dp, n, tol, max_iter, da, di, dj, dfe, limits, work, S,
                      c->stream, c->fabrik_variant, c->fabrik_core, c->fab_ord, c->rconst,
                      c->dbg, c->fabrik_bpc, prior);
  IK_HIP(hipGetLastError());
  return IK_OK;
}

int ann_launch(ik_ctx *c, const double *dp, int64_t n, float *da, double *de, bool limits,
               DevStats *S) {
  if (!S) S = c->d_stats;
  launch_reset_stats(S, c->stream);
  if (c->ann_big) {
    // two activation buffers of chunk x ld floats within IKHIP_ANN_ACT_MB (default
    // 1024 MiB; at least one 128-row tile), grown on demand
    if (n <= 0) return IK_OK;
    const char *bv = getenv("IKHIP_ANN_ACT_MB");  // (read per call: tests shrink it)
    long long budget_mb = (bv && *bv) ? atoll(bv) : 1024;
    if (budget_mb <= 0) budget_mb = 1024;
    const size_t ld = ann_big_ld(c->ann_bigm);
    int64_t rows = ann_big_rows(c->ann_bigm, (size_t)budget_mb << 20);
    if (rows < 128) rows = 128;
    const int64_t n128 = (n + 127) / 128 * 128;
    if (rows > n128) rows = n128;
    if (2 * (size_t)rows * ld * sizeof(float) > c->ann_act_bytes) {
      IK_HIP(hipStreamSynchronize(c->stream));
      if (c->ann_act) IK_HIP(hipFree(c->ann_act));
      c->ann_act = nullptr;
      c->ann_act_bytes = 0;
      // the budget's rows, or fewer (down to one 128-row tile, which ik_ann_load
      // checked would fit) when the device has less free
      for (;;) {
        const size_t bytes = 2 * (size_t)rows * ld * sizeof(float);
        const hipError_t e = hipMalloc(&c->ann_act, bytes);
        if (e == hipSuccess) {
          c->ann_act_bytes = bytes;
          break;
        }
        (void)hipGetLastError();
        if (e != hipErrorOutOfMemory || rows <= 128) IK_HIP(e);
        rows = (rows / 2 + 127) / 128 * 128;
      }
    }
    // the rows the buffers hold (a smaller earlier allocation limits the chunk)
    const int64_t fit = (int64_t)(c->ann_act_bytes / (2 * ld * sizeof(float))) / 128 * 128;
    if (rows > fit) rows = fit;
    // (both split modes run bf16x6 here: fp16x3's bounded-input planes are the
    // fused kernel's)
    launch_ann_big(c->ann_bigm, c->robot, dp, n, da, de, limits, S, c->stream,
                   static_cast<float *>(c->ann_act), rows, c->ann_mode);
    IK_HIP(hipGetLastError());
    return IK_OK;
  }
  AnnModelDev m = c->ann;
  m.xmode = c->ann_mode;
  for (int l = 0; l < m.n_layers; ++l) {
    m.wx[l] = c->ann_mode == IK_ANN_BF16X6   ? c->ann_wx[l]
              : c->ann_mode == IK_ANN_FP16X3 ? c->ann_wh[l]
                                             : nullptr;
    m.xinv[l] = c->ann_hinv[l];
  }
  launch_ann(m, c->robot, dp, n, da, de, limits, S, c->stream, c->dbg);
  IK_HIP(hipGetLastError());
  return IK_OK;
}

}  // namespace ikapi

extern "C" {

const char *ik_last_error(void) { return g_last_error.c_str(); }
const char *ik_version(void) { return "ikhip 0.1 gfx950"; }

int ik_ctx_create(int device, ik_ctx **out) {
  if (!out) return fail(IK_E_BADARG, "ik_ctx_create: out is NULL");
  *out = nullptr;
  int ndev = 0;
  IK_HIP(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev)
    return fail(IK_E_BADARG, "ik_ctx_create: device " + std::to_string(device) +
                                 " out of range (" + std::to_string(ndev) + " devices)");
  ik_ctx *c = new ik_ctx();
  c->device = device;
  int rc = set_dev(c);
  if (rc) {
    delete c;
    return rc;
  }
  hipError_t e = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMalloc(&c->d_stats, sizeof(DevStats));
  if (e == hipSuccess) e = hipHostMalloc(&c->h_stats, sizeof(DevStats), hipHostMallocDefault);
  if (e == hipSuccess) e = hipMalloc(&c->fab_ord, sizeof(FabOrderDev));
  if (e == hipSuccess) e = hipMemset(c->fab_ord, 0, sizeof(FabOrderDev));
  if (e == hipSuccess && kFabPriors > 0) {
    e = hipMalloc(&c->fab_priors, sizeof(FabPrior::key) * kFabPriors);
    for (int k = 0; k < kFabPriors && e == hipSuccess; ++k)
      e = hipMemcpy(c->fab_priors + (size_t)k * kOrdCells, kFabPrior[k].key, sizeof(FabPrior::key),
                    hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) e = hipMalloc(&c->rconst, sizeof(RobotConstDev));
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->call_done, hipEventDisableTiming);
  c->stream = c->own_stream;
  if (e != hipSuccess) {
    (void)ik_ctx_destroy(c);  // frees whatever was allocated
    return fail(IK_E_HIP, std::string("ik_ctx_create: ") + hipGetErrorString(e));
  }
  std::memcpy(c->robot.dh, kDefaultDh, sizeof(kDefaultDh));
  std::memcpy(c->robot.links, kDefaultLinks, sizeof(kDefaultLinks));
  std::memcpy(c->robot.lim, kDefaultLimits, sizeof(kDefaultLimits));
  launch_robot_const(c->robot, c->rconst, c->stream);
  // a fresh context's work order: SixDOFRobot's built-in table for the
  // reference's defaults (tol 1e-3, 100 iterations; FabrikInverseKinematics)
  if (seed_order(c, 1e-3, 100) != IK_OK) e = hipErrorUnknown;
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e == hipSuccess) e = hipGetLastError();
  if (e != hipSuccess) {
    (void)ik_ctx_destroy(c);
    return fail(IK_E_HIP, std::string("ik_ctx_create: ") + hipGetErrorString(e));
  }
  if (const char *v = std::getenv("IKHIP_FABRIK_VARIANT")) c->fabrik_variant = std::atoi(v);
  if (const char *v = std::getenv("IKHIP_FABRIK_CORE")) c->fabrik_core = std::atoi(v);
  if (const char *v = std::getenv("IKHIP_FABRIK_BPC")) c->fabrik_bpc = std::atoi(v);
  if (const char *v = std::getenv("IKHIP_ANN_MODE"))
    c->ann_mode = std::strcmp(v, "bf16x6") == 0   ? IK_ANN_BF16X6
                  : std::strcmp(v, "fp16x3") == 0 ? IK_ANN_FP16X3
                                                  : IK_ANN_FP32;
  *out = c;
  return IK_OK;
}

int ik_ctx_destroy(ik_ctx *c) {
  if (!c) return IK_OK;
  (void)hipSetDevice(c->device);
  // the communicator first: a live one's last call is waited for with its
  // deadline; an aborted one whose work has not drained leaves the context's
  // device memory to the process's end rather than block on it
  if (!comm_release(c)) return fail(IK_E_RCCL, "ik_ctx_destroy: aborted collective work has not "
                                               "drained; the context is left to the process's end");
  (void)hipStreamSynchronize(c->stream);
  if (c->scratch) (void)hipFree(c->scratch);
  if (c->ann_buf) (void)hipFree(c->ann_buf);
  if (c->ann_act) (void)hipFree(c->ann_act);
  if (c->d_stats) (void)hipFree(c->d_stats);
  if (c->dbg) (void)hipFree(c->dbg);
  if (c->fab_ord) (void)hipFree(c->fab_ord);
  if (c->fab_priors) (void)hipFree(c->fab_priors);
  if (c->rconst) (void)hipFree(c->rconst);
  if (c->h_stats) (void)hipHostFree(c->h_stats);
  pipe_release(c);
  if (c->call_done) (void)hipEventDestroy(c->call_done);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  for (int i = 0; i < kMaxTimed; ++i) {
    if (c->kt.beg[i]) (void)hipEventDestroy(c->kt.beg[i]);
    if (c->kt.end[i]) (void)hipEventDestroy(c->kt.end[i]);
  }
  delete c;
  return IK_OK;
}

int ik_ctx_set_stream(ik_ctx *c, void *stream) {
  if (!c) return fail(IK_E_BADARG, "ik_ctx_set_stream: NULL context");
  c->stream = stream ? static_cast<hipStream_t>(stream) : c->own_stream;
  return IK_OK;
}

void *ik_ctx_get_stream(ik_ctx *c) { return c ? static_cast<void *>(c->stream) : nullptr; }

int ik_set_robot(ik_ctx *c, const double *dh, const double *links, const double *limits) {
  if (!c) return fail(IK_E_BADARG, "ik_set_robot: NULL context");
  const RobotDev old = c->robot;
  if (dh) std::memcpy(c->robot.dh, dh, sizeof(c->robot.dh));
  if (links) std::memcpy(c->robot.links, links, sizeof(c->robot.links));
  if (limits) std::memcpy(c->robot.lim, limits, sizeof(c->robot.lim));
  // dh[0] (theta_1) is never read on the device: every solve takes the point's
  // own azimuth (inverse.py:123-125 writes it into the table per point), so a
  // drop-in caller re-sending the table with the last point's theta_1 changes
  // nothing.  The FABRIK cost table describes one chain (dh[1..15], links):
  // forget it only when that changes; the seed / limit constants follow any
  // change of those or of the limits.
  const bool chain = std::memcmp(old.dh + 1, c->robot.dh + 1, 15 * sizeof(double)) ||
                     std::memcmp(old.links, c->robot.links, sizeof(old.links));
  const bool lim = std::memcmp(old.lim, c->robot.lim, sizeof(old.lim)) != 0;
  if (chain || lim) {
    int rc = set_dev(c);
    if (rc) return rc;
    if (chain) {  // another chain's costs: its own (built-in for SixDOFRobot's), or empty
      const int rc = seed_order(c, 1e-3, 100);
      if (rc) return rc;
    }
    launch_robot_const(c->robot, c->rconst, c->stream);
    IK_HIP(hipGetLastError());
    // synchronous: later calls may run on another stream (ik_ctx_set_stream)
    IK_HIP(hipStreamSynchronize(c->stream));
  }
  return IK_OK;
}

int ik_ctx_set_timing(ik_ctx *c, int on) {
  if (!c) return fail(IK_E_BADARG, "ik_ctx_set_timing: NULL context");
  int rc = set_dev(c);
  if (rc) return rc;
  if (on && !c->kt.beg[0]) {
    for (int i = 0; i < kMaxTimed; ++i) {
      IK_HIP(hipEventCreate(&c->kt.beg[i]));
      IK_HIP(hipEventCreate(&c->kt.end[i]));
    }
  }
  c->kt.on = on != 0;
  c->kt.acc = on == 2;
  c->kt.n = 0;
  c->kt.state = 0;
  return IK_OK;
}

int ik_kernel_times(ik_ctx *c, int max, float *ms, char *names, int name_len) {
  if (!c || max < 0 || (max > 0 && !ms)) return -IK_E_BADARG;
  if (!c->kt.on) return 0;
  if (set_dev(c)) return -IK_E_HIP;
  int n = c->kt.n < max ? c->kt.n : max;
  for (int i = 0; i < n; ++i) {
    if (hipEventSynchronize(c->kt.end[i]) != hipSuccess) return -IK_E_HIP;
    float t = 0.0f;
    if (hipEventElapsedTime(&t, c->kt.beg[i], c->kt.end[i]) != hipSuccess) return -IK_E_HIP;
    ms[i] = t;
    if (names && name_len > 0) {
      std::strncpy(names + (size_t)i * name_len, c->kt.name[i], (size_t)name_len - 1);
      names[(size_t)i * name_len + name_len - 1] = 0;
    }
  }
  return n;
}

// the diagnostic buffer: ANN stamps or FABRIK iteration-kernel counters
static size_t debug_words() {
  return ann_debug_words() > kFabrikDebugWords ? ann_debug_words() : kFabrikDebugWords;
}

int ik_ctx_set_debug(ik_ctx *c, int on) {
  if (!c) return fail(IK_E_BADARG, "ik_ctx_set_debug: NULL context");
  int rc = set_dev(c);
  if (rc) return rc;
  IK_HIP(hipStreamSynchronize(c->stream));
  if (on && !c->dbg) {
    IK_HIP(hipMalloc(&c->dbg, debug_words() * 8));
    IK_HIP(hipMemset(c->dbg, 0, debug_words() * 8));
  } else if (!on && c->dbg) {
    IK_HIP(hipFree(c->dbg));
    c->dbg = nullptr;
  }
  return IK_OK;
}

int ik_debug_read(ik_ctx *c, uint64_t *out, int max) {
  if (!c || !out || max < 0) return -IK_E_BADARG;
  if (!c->dbg) return 0;
  if (set_dev(c)) return -IK_E_HIP;
  int n = (int)debug_words() < max ? (int)debug_words() : max;
  if (hipStreamSynchronize(c->stream) != hipSuccess) return -IK_E_HIP;
  if (hipMemcpy(out, c->dbg, (size_t)n * 8, hipMemcpyDeviceToHost) != hipSuccess)
    return -IK_E_HIP;
  return n;
}

int ik_ctx_sync(ik_ctx *c) {
  if (!c) return fail(IK_E_BADARG, "ik_ctx_sync: NULL context");
  int rc = set_dev(c);
  if (rc) return rc;
  if (c->last_piped) return IK_OK;  // a chunked host pipeline returns complete
  if (!c->call_done_set) return IK_OK;
  // with a communicator the wait is bounded (its deadline and async errors)
  rc = comm_wait(c, c->call_done, "the last call");
  if (rc) return rc;
  // an IK_F_ASYNC sharded call is validated here as ik_stats_fetch would: every
  // rank planned the same (n, chunks, method), else the gathered rows belong to
  // another plan
  if (c->last_sharded) return sharded_stats(c, nullptr);
  return IK_OK;
}

int ik_stats_fetch(ik_ctx *c, ik_stats *stats) {
  if (!c) return fail(IK_E_BADARG, "ik_stats_fetch: NULL context");
  int rc = set_dev(c);
  if (rc) return rc;
  // the stats of the last call live on the stream it ran on (ik_ctx_set_stream may
  // have switched since)
  if (c->last_piped) {  // a chunked host pipeline: merged when it returned
    if (stats) *stats = c->piped_stats;
    return IK_OK;
  }
  hipStream_t cur = c->stream;
  if (c->last_stream) c->stream = c->last_stream;
  rc = c->last_sharded ? sharded_stats(c, stats) : finish(c, 0, stats);
  c->stream = cur;
  return rc;
}

int ik_check_limits(ik_ctx *c, const double *pts, int64_t n, int flags, ik_stats *stats) {
  if (!c || n < 0 || (n > 0 && !pts)) return fail(IK_E_BADARG, "ik_check_limits: bad args");
  if ((flags & IK_F_ASYNC) && !(flags & IK_F_DEVICE))
    return fail(IK_E_BADARG, "IK_F_ASYNC requires IK_F_DEVICE");
  int rc = set_dev(c);
  if (rc) return rc;
  KtScope kts(c);
  const double *dp = pts;
  if (!(flags & IK_F_DEVICE)) {
    if ((rc = ensure_scratch(c, (size_t)n * 24 + 256))) return rc;
    IK_HIP(hipMemcpyAsync(c->scratch, pts, (size_t)n * 24, hipMemcpyHostToDevice, c->stream));
    dp = static_cast<const double *>(c->scratch);
  }
  launch_reset_stats(c->d_stats, c->stream);
  launch_check_limits(c->robot, dp, n, c->d_stats, c->stream);
  IK_HIP(hipGetLastError());
  return finish(c, flags, stats);
}

int ik_fk(ik_ctx *c, const double *ang, int64_t n, double *xyz, double *mats, int flags,
          ik_stats *stats) {
  double *joints = mats;  // n x 4 x 16
  if (!c || n < 0 || (n > 0 && (!ang || !xyz))) return fail(IK_E_BADARG, "ik_fk: bad args");
  if ((flags & IK_F_ASYNC) && !(flags & IK_F_DEVICE))
    return fail(IK_E_BADARG, "IK_F_ASYNC requires IK_F_DEVICE");
  int rc = set_dev(c);
  if (rc) return rc;
  KtScope kts(c);
  const double *da = ang;
  double *dx = xyz, *dj = joints;
  if (!(flags & IK_F_DEVICE)) {
    size_t b_in = Stage::up((size_t)n * 32), b_x = Stage::up((size_t)n * 24),
           b_j = joints ? Stage::up((size_t)n * 512) : 0;
    if ((rc = ensure_scratch(c, b_in + b_x + b_j))) return rc;
    char *s = static_cast<char *>(c->scratch);
    IK_HIP(hipMemcpyAsync(s, ang, (size_t)n * 32, hipMemcpyHostToDevice, c->stream));
    da = reinterpret_cast<double *>(s);
    dx = reinterpret_cast<double *>(s + b_in);
    dj = joints ? reinterpret_cast<double *>(s + b_in + b_x) : nullptr;
  }
  launch_reset_stats(c->d_stats, c->stream);
  launch_fk(c->robot, da, n, dx, dj, c->d_stats, c->stream);
  IK_HIP(hipGetLastError());
  if (!(flags & IK_F_DEVICE) && n > 0) {
    IK_HIP(hipMemcpyAsync(xyz, dx, (size_t)n * 24, hipMemcpyDeviceToHost, c->stream));
    if (joints)
      IK_HIP(hipMemcpyAsync(joints, dj, (size_t)n * 512, hipMemcpyDeviceToHost, c->stream));
  }
  return finish(c, flags, stats);
}

int ik_fk_chain(ik_ctx *c, int nj, const double *dh, const double *ang, int64_t n,
                double *xyz, double *mats, int flags, ik_stats *stats) {
  if (!c || nj < 2 || nj > kFkMaxJoints || !dh || n < 0 || (n > 0 && (!ang || !xyz)))
    return fail(IK_E_BADARG, "ik_fk_chain: bad args (nj must be 2.." +
                                 std::to_string(kFkMaxJoints) + ")");
  if ((flags & IK_F_ASYNC) && !(flags & IK_F_DEVICE))
    return fail(IK_E_BADARG, "IK_F_ASYNC requires IK_F_DEVICE");
  int rc = set_dev(c);
  if (rc) return rc;
  KtScope kts(c);
  const bool dev = flags & IK_F_DEVICE;
  const size_t b_dh = Stage::up((size_t)nj * 32);
  const size_t b_in = dev ? 0 : Stage::up((size_t)n * nj * 8);
  const size_t b_x = dev ? 0 : Stage::up((size_t)n * 24);
  const size_t b_m = (dev || !mats) ? 0 : Stage::up((size_t)n * nj * 128);
  if ((rc = ensure_scratch(c, b_dh + b_in + b_x + b_m))) return rc;
  char *s = static_cast<char *>(c->scratch);
  // the DH table always travels from host memory
  IK_HIP(hipMemcpyAsync(s, dh, (size_t)nj * 32, hipMemcpyHostToDevice, c->stream));
  const double *dd = reinterpret_cast<const double *>(s);
  const double *da = ang;
  double *dx = xyz, *dm = mats;
  if (!dev) {
    char *q = s + b_dh;
    IK_HIP(hipMemcpyAsync(q, ang, (size_t)n * nj * 8, hipMemcpyHostToDevice, c->stream));
    da = reinterpret_cast<const double *>(q);
    dx = reinterpret_cast<double *>(q + b_in);
    dm = mats ? reinterpret_cast<double *>(q + b_in + b_x) : nullptr;
  }
  launch_reset_stats(c->d_stats, c->stream);
  launch_fk_n(nj, dd, da, n, dx, dm, c->d_stats, c->stream);
  IK_HIP(hipGetLastError());
  if (!dev && n > 0) {
    IK_HIP(hipMemcpyAsync(xyz, dx, (size_t)n * 24, hipMemcpyDeviceToHost, c->stream));
    if (mats)
      IK_HIP(hipMemcpyAsync(mats, dm, (size_t)n * nj * 128, hipMemcpyDeviceToHost, c->stream));
  }
  // dh came from a host buffer that may go away: always complete before return
  if (flags & IK_F_ASYNC) IK_HIP(hipStreamSynchronize(c->stream));
  return finish(c, flags, stats);
}

int ik_fabrik_solve(ik_ctx *c, const double *pts, int64_t n, double tol, int32_t max_iter,
                    double *ang, int32_t *iters, double *joints, int flags, ik_stats *stats) {
  return ik_fabrik_solve_fk(c, pts, n, tol, max_iter, ang, iters, joints, nullptr, flags, stats);
}

int ik_fabrik_solve_fk(ik_ctx *c, const double *pts, int64_t n, double tol, int32_t max_iter,
                       double *ang, int32_t *iters, double *joints, double *fk_err, int flags,
                       ik_stats *stats) {
  if (!c || n < 0 || (n > 0 && (!pts || !ang)) || max_iter < 0)
    return fail(IK_E_BADARG, "ik_fabrik_solve: bad args");
  if ((flags & IK_F_ASYNC) && !(flags & IK_F_DEVICE))
    return fail(IK_E_BADARG, "IK_F_ASYNC requires IK_F_DEVICE");
  if ((flags & IK_F_DEVICE) && (reinterpret_cast<uintptr_t>(ang) & 15))
    return fail(IK_E_BADARG, "ik_fabrik_solve: device ang must be 16-byte aligned");
  int rc = set_dev(c);
  if (rc) return rc;
  KtScope kts(c);
  const bool dev = flags & IK_F_DEVICE;
  if (!dev && pipeline_wanted(c, n, {pts, ang, iters, joints, fk_err}))
    return fabrik_host_pipeline(c, pts, n, tol, max_iter, ang, iters, joints, fk_err, flags,
                                stats);
  size_t b_work = Stage::up(fabrik_scratch_bytes(n));
  size_t b_in = dev ? 0 : Stage::up((size_t)n * 24);
  size_t b_ang = dev ? 0 : Stage::up((size_t)n * 32);
  size_t b_it = (dev || !iters) ? 0 : Stage::up((size_t)n * 4);
  size_t b_jo = (dev || !joints) ? 0 : Stage::up((size_t)n * 96);
  size_t b_fe = (dev || !fk_err) ? 0 : Stage::up((size_t)n * 8);
  if ((rc = ensure_scratch(c, b_work + b_in + b_ang + b_it + b_jo + b_fe))) return rc;
  char *s = static_cast<char *>(c->scratch);
  void *work = s;
  const double *dp = pts;
  double *da = ang, *dj = joints, *dfe = fk_err;
  int32_t *di = iters;
  if (!dev) {
    char *q = s + b_work;
    dp = reinterpret_cast<double *>(q);
    IK_HIP(hipMemcpyAsync(q, pts, (size_t)n * 24, hipMemcpyHostToDevice, c->stream));
    q += b_in;
    da = reinterpret_cast<double *>(q);
    q += b_ang;
    di = iters ? reinterpret_cast<int32_t *>(q) : nullptr;
    q += b_it;
    dj = joints ? reinterpret_cast<double *>(q) : nullptr;
    q += b_jo;
    dfe = fk_err ? reinterpret_cast<double *>(q) : nullptr;
  }
  rc = fabrik_launch(c, dp, n, tol, max_iter, da, di, dj, dfe, !(flags & IK_F_NO_LIMITS), work);
  if (rc) return rc;
  if (!dev && n > 0) {
    IK_HIP(hipMemcpyAsync(ang, da, (size_t)n * 32, hipMemcpyDeviceToHost, c->stream));
    if (iters)
      IK_HIP(hipMemcpyAsync(iters, di, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
    if (joints)
      IK_HIP(hipMemcpyAsync(joints, dj, (size_t)n * 96, hipMemcpyDeviceToHost, c->stream));
    if (fk_err)
      IK_HIP(hipMemcpyAsync(fk_err, dfe, (size_t)n * 8, hipMemcpyDeviceToHost, c->stream));
  }
  return finish(c, flags, stats);
}

int ik_fabrik_reset_order(ik_ctx *c) {
  if (!c) return fail(IK_E_BADARG, "ik_fabrik_reset_order: NULL context");
  int rc = set_dev(c);
  if (rc) return rc;
  KtScope kts(c);  // ordered after the context's earlier calls, whatever their stream
  return seed_order(c, 1e-3, 100);
}

int ik_fabrik_order_get(ik_ctx *c, uint32_t *key, int n) {
  if (!c || !key || n < kOrdCells) return -fail(IK_E_BADARG, "ik_fabrik_order_get: bad args");
  if (set_dev(c)) return -IK_E_HIP;
  // the last call's end, waited for with the communicator's deadline when one is
  // bound (a dead peer ends the wait with IK_E_RCCL instead of hanging it)
  if (c->call_done_set) {
    const int rc = comm_wait(c, c->call_done, "the last call");
    if (rc) return -rc;
  } else if (hipStreamSynchronize(c->stream) != hipSuccess) {
    return -fail(IK_E_HIP, "ik_fabrik_order_get: stream synchronize failed");
  }
  if (hipMemcpy(key, c->fab_ord->key, sizeof(c->fab_ord->key), hipMemcpyDeviceToHost) != hipSuccess)
    return -fail(IK_E_HIP, "ik_fabrik_order_get: copy failed");
  return kOrdCells;
}

int ik_fabrik_order_set(ik_ctx *c, const uint32_t *key, int n) {
  if (!c || (key && n != kOrdCells)) return fail(IK_E_BADARG, "ik_fabrik_order_set: bad args");
  int rc = set_dev(c);
  if (rc) return rc;
  KtScope kts(c);
  IK_HIP(hipStreamSynchronize(c->stream));  // key may be a short-lived host buffer
  if (key)
    IK_HIP(hipMemcpy(c->fab_ord->key, key, sizeof(c->fab_ord->key), hipMemcpyHostToDevice));
  else
    IK_HIP(hipMemset(c->fab_ord->key, 0, sizeof(c->fab_ord->key)));
  c->fab_prior = -1;
  return IK_OK;
}

int ik_fabrik_calc(ik_ctx *c, int nj, const double *dists, const double *init,
                   int init_shared, const double *goals, int64_t n, double tol,
                   int32_t max_iter, double *joints, int32_t *iters, int flags,
                   ik_stats *stats) {
  if (!c || nj < 1 || nj > kCalcMaxJoints || !dists || n < 0 ||
      (n > 0 && (!init || !goals || !joints)) || max_iter < 0)
    return fail(IK_E_BADARG, "ik_fabrik_calc: bad args (nj must be 1.." +
                                 std::to_string(kCalcMaxJoints) + ")");
  if ((flags & IK_F_ASYNC) && !(flags & IK_F_DEVICE))
    return fail(IK_E_BADARG, "IK_F_ASYNC requires IK_F_DEVICE");
  int rc = set_dev(c);
  if (rc) return rc;
  KtScope kts(c);
  const bool dev = flags & IK_F_DEVICE;
  size_t b_d = Stage::up((size_t)nj * 8);
  size_t n_init = init_shared ? (size_t)nj * 3 : (size_t)n * nj * 3;
  size_t b_init = dev ? 0 : Stage::up(n_init * 8);
  size_t b_g = dev ? 0 : Stage::up((size_t)n * 24);
  size_t b_jo = dev ? 0 : Stage::up((size_t)n * nj * 24);
  size_t b_it = (dev || !iters) ? 0 : Stage::up((size_t)n * 4);
  if ((rc = ensure_scratch(c, b_d + b_init + b_g + b_jo + b_it))) return rc;
  char *s = static_cast<char *>(c->scratch);
  // the link distances always travel from host memory
  IK_HIP(hipMemcpyAsync(s, dists, (size_t)nj * 8, hipMemcpyHostToDevice, c->stream));
  const double *dd = reinterpret_cast<double *>(s);
  const double *di = init, *dg = goals;
  double *djo = joints;
  int32_t *dit = iters;
  if (!dev) {
    char *q = s + b_d;
    IK_HIP(hipMemcpyAsync(q, init, n_init * 8, hipMemcpyHostToDevice, c->stream));
    di = reinterpret_cast<double *>(q);
    q += b_init;
    IK_HIP(hipMemcpyAsync(q, goals, (size_t)n * 24, hipMemcpyHostToDevice, c->stream));
    dg = reinterpret_cast<double *>(q);
    q += b_g;
    djo = reinterpret_cast<double *>(q);
    q += b_jo;
    dit = iters ? reinterpret_cast<int32_t *>(q) : nullptr;
  }
  launch_reset_stats(c->d_stats, c->stream);
  launch_fabrik_calc(nj, dd, di, init_shared != 0, dg, n, tol, max_iter, djo, dit, c->d_stats,
                     c->stream);
  IK_HIP(hipGetLastError());
  if (!dev && n > 0) {
    IK_HIP(hipMemcpyAsync(joints, djo, (size_t)n * nj * 24, hipMemcpyDeviceToHost, c->stream));
    if (iters)
      IK_HIP(hipMemcpyAsync(iters, dit, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
  }
  // dists came from a host buffer that may go away: always complete before return
  if (flags & IK_F_ASYNC) IK_HIP(hipStreamSynchronize(c->stream));
  return finish(c, flags, stats);
}

int ik_ann_load(ik_ctx *c, int n_layers, const int32_t *dims, const int32_t *acts,
                const float *const *W, const float *const *b, const double *x_mean,
                const double *x_scale, const double *y_mean, const double *y_scale) {
  if (!c || n_layers < 1 || n_layers > kAnnBigMaxLayers || !dims || !acts || !W || !b ||
      !x_mean || !x_scale || !y_mean || !y_scale)
    return fail(IK_E_BADARG, "ik_ann_load: bad args (1.." + std::to_string(kAnnBigMaxLayers) +
                                 " layers)");
  if (dims[0] != 3 || dims[n_layers] != 4)
    return fail(IK_E_BADARG, "ik_ann_load: the model must map 3 inputs to 4 outputs");
  for (int l = 0; l <= n_layers; ++l)
    if (dims[l] < 1 || dims[l] > kAnnBigMaxWidth)
      return fail(IK_E_BADARG, "ik_ann_load: layer widths must be 1.." +
                                   std::to_string(kAnnBigMaxWidth));
  // past the fused kernel's caps: the layered path (fp32, activations through HBM)
  bool big = n_layers > kAnnMaxLayers;
  for (int l = 0; l <= n_layers; ++l) big = big || dims[l] > kAnnMaxWidth;
  for (int l = 0; l < n_layers; ++l)
    if (acts[l] < IK_ACT_LINEAR || acts[l] > IK_ACT_SIGMOID)
      return fail(IK_E_BADARG, "ik_ann_load: unsupported activation code");
  int rc = set_dev(c);
  if (rc) return rc;
  // one device buffer: per layer packed weights, padded bias and -- for the
  // hidden layers that can take the bf16x6 mode (not the input layer, not a
  // single-column-tile output layer) -- the split bf16 planes
  std::vector<size_t> woff(n_layers), boff(n_layers), xoff(n_layers, 0), hoff(n_layers, 0);
  std::vector<int> hexp(n_layers, 0);
  // models wider than 512 run the wide fp32 kernel only: no split operands; the
  // layered path (big) has its own bf16x6 planes (ann_big_pack_x)
  bool wide = big;
  for (int l = 0; l <= n_layers; ++l) wide = wide || dims[l] > 512;
  bool planes = true;  // (dropped below when only the fp32 operands fit the device)
  auto splittable = [&](int l) {
    return planes && (!wide || big) && l > 0 && (dims[l + 1] + 31) / 32 > 1;
  };
  // fp16x3 also needs a bounded layer input: the layer before is tanh or sigmoid
  auto halvable = [&](int l) {
    return !big && splittable(l) &&
           (acts[l - 1] == IK_ACT_TANH || acts[l - 1] == IK_ACT_SIGMOID);
  };
  size_t total = 0;
  auto layout = [&]() {
    total = 0;
    for (int l = 0; l < n_layers; ++l) {
      woff[l] = total;
      total += ann_packed_floats(dims[l], dims[l + 1]) * 4;
      total = (total + 255) & ~(size_t)255;
      boff[l] = total;
      total += (size_t)((dims[l + 1] + 31) / 32 * 32) * 4;
      total = (total + 255) & ~(size_t)255;
      if (splittable(l)) {
        xoff[l] = total;
        total += big ? ann_big_x_bytes(dims[l], dims[l + 1]) : ann_x_bytes(dims[l], dims[l + 1]);
        total = (total + 255) & ~(size_t)255;
      }
      if (halvable(l)) {
        hoff[l] = total;
        total += ann_h_bytes(dims[l], dims[l + 1]);
        total = (total + 255) & ~(size_t)255;
      }
    }
  };
  layout();
  // (the widths and depth are capped above, so `total` stays far below 2^64: at
  // most 4096 layers of a 16384 x 16384 product, ~4.4 TB -- but that may not fit
  // the device, and the host staging must not be one buffer of that size)
  IK_HIP(hipStreamSynchronize(c->stream));
  if (c->ann_buf) IK_HIP(hipFree(c->ann_buf));
  c->ann_buf = nullptr;
  c->ann_loaded = false;
  size_t dev_free = 0, dev_total = 0;
  IK_HIP(hipMemGetInfo(&dev_free, &dev_total));
  // the layered path's first solve also needs its two activation buffers: at
  // least one 128-row tile of the widest padded layer (ann_launch takes up to
  // IKHIP_ANN_ACT_MB and falls back to fewer rows when that much is not free;
  // ADVICE r05), less what a previous model's buffers already hold
  size_t act_min = 0;
  if (big) {
    size_t ld = 8;
    for (int l = 0; l < n_layers; ++l) {
      const size_t np = (size_t)(dims[l + 1] + 31) / 32 * 32;
      ld = np > ld ? np : ld;
    }
    act_min = 2 * 128 * ld * sizeof(float);
    act_min = act_min > c->ann_act_bytes ? act_min - c->ann_act_bytes : 0;
  }
  if (total + act_min > dev_free) {  // without the split planes (the split modes then run fp32)?
    planes = false;
    layout();
  }
  if (total + act_min > dev_free)
    return fail(IK_E_HIP, "ik_ann_load: the packed model needs " + std::to_string(total) +
                              " bytes of device memory (+ " + std::to_string(act_min) +
                              " for its activations), " + std::to_string(dev_free) +
                              " are free");
  // (without the planes a split mode runs fp32: ik_ann_effective_mode says so)
  IK_HIP(hipMalloc(&c->ann_buf, total));
  char *base = static_cast<char *>(c->ann_buf);
  // pack and upload one layer's section at a time: the host holds
  // at most the largest layer's packed bytes, and an allocation failure is an
  // error code, not an exception leaving the C ABI
  try {
    std::vector<char> host;
    for (int l = 0; l < n_layers; ++l) {
      const size_t end = l + 1 < n_layers ? woff[l + 1] : total;
      host.assign(end - woff[l], 0);
      char *h = host.data();  // the section starts at woff[l] in the model buffer
      ann_pack_layer(W[l], dims[l], dims[l + 1], reinterpret_cast<float *>(h));
      std::memcpy(h + (boff[l] - woff[l]), b[l], (size_t)dims[l + 1] * 4);
      if (splittable(l)) {
        if (big) ann_big_pack_x(W[l], dims[l], dims[l + 1], h + (xoff[l] - woff[l]));
        else ann_pack_layer_x(W[l], dims[l], dims[l + 1], h + (xoff[l] - woff[l]));
      }
      if (halvable(l)) {
        hexp[l] = ann_h_scale_exp(W[l], dims[l], dims[l + 1]);
        ann_pack_layer_h(W[l], dims[l], dims[l + 1], hexp[l], h + (hoff[l] - woff[l]));
      }
      IK_HIP(hipMemcpy(base + woff[l], host.data(), host.size(), hipMemcpyHostToDevice));
    }
  } catch (const std::bad_alloc &) {
    (void)hipFree(c->ann_buf);
    c->ann_buf = nullptr;
    return fail(IK_E_HIP, "ik_ann_load: out of host memory staging the packed weights");
  }
  c->ann_big = big;
  c->ann_bigm.layers.clear();
  if (big) {
    AnnBigModel &bm = c->ann_bigm;
    for (int l = 0; l < n_layers; ++l)
      bm.layers.push_back({(dims[l] + 7) / 8 * 8, (dims[l + 1] + 31) / 32 * 32, acts[l],
                           reinterpret_cast<const float *>(base + woff[l]),
                           reinterpret_cast<const float *>(base + boff[l]),
                           splittable(l) ? reinterpret_cast<const uint16_t *>(base + xoff[l])
                                         : nullptr});
    for (int i = 0; i < 3; ++i) {
      bm.xm[i] = x_mean[i];
      bm.xs[i] = x_scale[i];
    }
    for (int i = 0; i < 4; ++i) {
      bm.ym[i] = y_mean[i];
      bm.ys[i] = y_scale[i];
    }
    std::memset(&c->ann, 0, sizeof(c->ann));
    c->ann_loaded = true;
    return IK_OK;
  }
  AnnModelDev &m = c->ann;
  std::memset(&m, 0, sizeof(m));
  m.n_layers = n_layers;
  for (int l = 0; l < n_layers; ++l) {
    m.kp[l] = (dims[l] + 7) / 8 * 8;
    m.np[l] = (dims[l + 1] + 31) / 32 * 32;
    m.act[l] = acts[l];
    m.wp[l] = reinterpret_cast<const float4 *>(base + woff[l]);
    m.bias[l] = reinterpret_cast<const float *>(base + boff[l]);
    c->ann_wx[l] = splittable(l) ? base + xoff[l] : nullptr;
    c->ann_wh[l] = halvable(l) ? base + hoff[l] : nullptr;
    c->ann_hinv[l] = std::ldexp(1.0f, -hexp[l]);
  }
  for (int i = 0; i < 3; ++i) {
    m.xm[i] = x_mean[i];
    m.xs[i] = x_scale[i];
  }
  for (int i = 0; i < 4; ++i) {
    m.ym[i] = y_mean[i];
    m.ys[i] = y_scale[i];
  }
  c->ann_loaded = true;
  return IK_OK;
}

int ik_ann_set_mode(ik_ctx *c, int mode) {
  if (!c) return fail(IK_E_BADARG, "ik_ann_set_mode: NULL context");
  if (mode != IK_ANN_FP32 && mode != IK_ANN_BF16X6 && mode != IK_ANN_FP16X3)
    return fail(IK_E_BADARG, "ik_ann_set_mode: unknown mode");
  c->ann_mode = mode;
  return IK_OK;
}

int ik_ann_get_mode(ik_ctx *c) { return c ? c->ann_mode : -IK_E_BADARG; }

int ik_ann_effective_mode(ik_ctx *c) {
  if (!c) return -IK_E_BADARG;
  if (!c->ann_loaded) return -fail(IK_E_NOMODEL, "ik_ann_effective_mode: no model loaded");
  if (c->ann_mode == IK_ANN_FP32) return IK_ANN_FP32;
  if (c->ann_big) {  // both split modes run bf16x6 there
    for (const AnnBigLayer &L : c->ann_bigm.layers)
      if (L.wx) return IK_ANN_BF16X6;
    return IK_ANN_FP32;
  }
  const void *const *ops = c->ann_mode == IK_ANN_BF16X6 ? c->ann_wx : c->ann_wh;
  for (int l = 0; l < c->ann.n_layers; ++l)
    if (ops[l]) return c->ann_mode;
  return IK_ANN_FP32;
}

int ik_ann_solve(ik_ctx *c, const double *pts, int64_t n, float *ang, double *fk_err,
                 int flags, ik_stats *stats) {
  if (!c || n < 0 || (n > 0 && (!pts || !ang))) return fail(IK_E_BADARG, "ik_ann_solve: bad args");
  if (!c->ann_loaded) return fail(IK_E_NOMODEL, "ik_ann_solve: no model loaded (ik_ann_load)");
  if ((flags & IK_F_ASYNC) && !(flags & IK_F_DEVICE))
    return fail(IK_E_BADARG, "IK_F_ASYNC requires IK_F_DEVICE");
  if ((flags & IK_F_DEVICE) && (reinterpret_cast<uintptr_t>(ang) & 15))
    return fail(IK_E_BADARG, "ik_ann_solve: device ang must be 16-byte aligned");
  int rc = set_dev(c);
  if (rc) return rc;
  KtScope kts(c);
  const bool dev = flags & IK_F_DEVICE;
  // (no chunked pipeline for ANN: its copies are ~2 % of the call and splitting
  // the launch into chunks costs more tile-quantisation tail than the overlap
  // saves -- 41.6 vs 41.1 ms per 1M points measured)
  const double *dp = pts;
  float *da = ang;
  double *de = fk_err;
  if (!dev) {
    size_t b_in = Stage::up((size_t)n * 24), b_a = Stage::up((size_t)n * 16),
           b_e = fk_err ? Stage::up((size_t)n * 8) : 0;
    if ((rc = ensure_scratch(c, b_in + b_a + b_e))) return rc;
    char *s = static_cast<char *>(c->scratch);
    IK_HIP(hipMemcpyAsync(s, pts, (size_t)n * 24, hipMemcpyHostToDevice, c->stream));
    dp = reinterpret_cast<double *>(s);
    da = reinterpret_cast<float *>(s + b_in);
    de = fk_err ? reinterpret_cast<double *>(s + b_in + b_a) : nullptr;
  }
  rc = ann_launch(c, dp, n, da, de, !(flags & IK_F_NO_LIMITS));
  if (rc) return rc;
  if (!dev && n > 0) {
    IK_HIP(hipMemcpyAsync(ang, da, (size_t)n * 16, hipMemcpyDeviceToHost, c->stream));
    if (fk_err)
      IK_HIP(hipMemcpyAsync(fk_err, de, (size_t)n * 8, hipMemcpyDeviceToHost, c->stream));
  }
  return finish(c, flags, stats);
}

}  // extern "C"
