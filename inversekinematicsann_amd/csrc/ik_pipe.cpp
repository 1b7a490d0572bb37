// ik_pipe.cpp -- host-pointer solves over PCIe with copy / compute overlap.
//
// A host-pointer call otherwise copies all its points in, solves, and copies all
// its results out, one after the other; for FABRIK (0.45 ms of kernels per 1M
// points against 24 MB in and 36 MB out) the copies are most of the call.  When
// every host array of the call is pinned (ik_host_alloc, or any hipHostMalloc'd
// memory) and the batch is large, the batch is cut into chunks and each chunk
// runs H2D (copy-in stream) -> solve (the context's stream) -> D2H (copy-out
// stream), chained by events, so the kernels of one chunk run under the copies
// of the others (the box's PCIe does not overlap its two directions,
// tools/pcie_probe.py: ~55 GB/s either way, 55.5 GB/s both at once).  Each
// chunk has its own stats block; the call's stats merge them with the chunks'
// offsets (ik_tail_reduce: lowest global failing index, sums, max).
// Pageable arrays keep the one-shot path (the driver stages those itself).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>

#include "ik_internal.h"

using namespace ikhip;

namespace {

bool is_pinned(const void *p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // pageable memory: clear the sticky error
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

int64_t pipe_min_points() {
  static int64_t v = -1;
  if (v < 0) {
    const char *e = std::getenv("IKHIP_PIPE_MIN");  // 0 disables the pipeline
    v = (e && *e) ? std::atoll(e) : 131072;
  }
  return v;
}

int64_t pipe_chunk_points() {
  static int64_t v = -1;
  if (v < 0) {
    const char *e = std::getenv("IKHIP_PIPE_CHUNK");  // points per chunk
    v = (e && *e && std::atoll(e) > 0) ? std::atoll(e) : 262144;
  }
  return v;
}

int chunks_for(int64_t n) {
  // ~250k points per chunk (1M points: 4), 2..8 chunks
  const int64_t c = pipe_chunk_points();
  int64_t k = (n + c - 1) / c;
  return (int)(k < 2 ? 2 : (k > kPipeMaxChunks ? kPipeMaxChunks : k));
}

}  // namespace

namespace ikapi {

bool pipeline_wanted(ik_ctx *c, int64_t n, std::initializer_list<const void *> ptrs) {
  (void)c;
  const int64_t lim = pipe_min_points();
  if (lim <= 0 || n < lim) return false;
  for (const void *p : ptrs)
    if (p && !is_pinned(p)) return false;
  return true;
}

static int pipe_ready(ik_ctx *c, size_t bytes) {
  IkPipe &p = c->pipe;
  if (!p.s_in) {
    IK_HIP(hipStreamCreateWithFlags(&p.s_in, hipStreamNonBlocking));
    IK_HIP(hipStreamCreateWithFlags(&p.s_out, hipStreamNonBlocking));
    for (int k = 0; k < kPipeMaxChunks; ++k) {
      IK_HIP(hipEventCreateWithFlags(&p.ev_in[k], hipEventDisableTiming));
      IK_HIP(hipEventCreateWithFlags(&p.ev_done[k], hipEventDisableTiming));
    }
    IK_HIP(hipEventCreateWithFlags(&p.ev_out, hipEventDisableTiming));
    IK_HIP(hipMalloc(&p.d_stats, sizeof(DevStats) * kPipeMaxChunks));
    IK_HIP(hipHostMalloc(reinterpret_cast<void **>(&p.h_stats),
                         sizeof(DevStats) * kPipeMaxChunks, hipHostMallocDefault));
  }
  if (bytes > p.buf_bytes) {
    IK_HIP(hipStreamSynchronize(c->stream));
    IK_HIP(hipStreamSynchronize(p.s_in));
    IK_HIP(hipStreamSynchronize(p.s_out));
    if (p.buf) IK_HIP(hipFree(p.buf));
    p.buf = nullptr;
    p.buf_bytes = 0;
    IK_HIP(hipMalloc(&p.buf, bytes));
    p.buf_bytes = bytes;
  }
  return IK_OK;
}

void pipe_release(ik_ctx *c) {
  IkPipe &p = c->pipe;
  if (p.s_in) (void)hipStreamSynchronize(p.s_in);
  if (p.s_out) (void)hipStreamSynchronize(p.s_out);
  for (int k = 0; k < kPipeMaxChunks; ++k) {
    if (p.ev_in[k]) (void)hipEventDestroy(p.ev_in[k]);
    if (p.ev_done[k]) (void)hipEventDestroy(p.ev_done[k]);
  }
  if (p.ev_out) (void)hipEventDestroy(p.ev_out);
  if (p.d_stats) (void)hipFree(p.d_stats);
  if (p.h_stats) (void)hipHostFree(p.h_stats);
  if (p.buf) (void)hipFree(p.buf);
  if (p.s_in) (void)hipStreamDestroy(p.s_in);
  if (p.s_out) (void)hipStreamDestroy(p.s_out);
  p = IkPipe();
}

// The chunks' stats -> the call's (indices made global).
static int merge_chunk_stats(ik_ctx *c, int K, const int64_t *begin, ik_stats *stats) {
  IK_HIP(hipStreamSynchronize(c->pipe.s_out));
  IK_HIP(hipStreamSynchronize(c->stream));
  c->last_sharded = false;
  ik_shard_tail t[kPipeMaxChunks];
  for (int k = 0; k < K; ++k) {
    ik_stats s;
    stats_from_dev(c->pipe.h_stats[k], &s);
    t[k].first_oob = s.first_oob >= 0 ? s.first_oob + begin[k] : -1;
    t[k].first_err = s.first_err >= 0 ? s.first_err + begin[k] : -1;
    t[k].first_err_code = s.first_err_code;
    t[k].max_iters = s.max_iters;
    t[k].sum_iters = s.sum_iters;
    t[k].n_capped = s.n_capped;
    t[k].max_fk_err = s.max_fk_err;
    t[k].sum_fk_err = s.sum_fk_err;
    t[k].rows = begin[k + 1] - begin[k];
  }
  // kept on the context: ik_stats_fetch after this call returns them (the
  // context's own stats block holds no part of a pipelined call)
  int rc = ik_tail_reduce(t, K, &c->piped_stats);
  if (rc) return rc;
  c->last_piped = true;
  if (stats) *stats = c->piped_stats;
  return IK_OK;
}

// One output region: row_bytes per point, host base, device base.
struct Region {
  size_t row;
  char *host;
  char *dev;
};

// H2D of chunk k on s_in, then the solve (launch) on the context's stream, then
// the chunk's rows of every output region and its stats block D2H on s_out.
template <class Launch>
static int run_chunks(ik_ctx *c, int K, const int64_t *begin, const double *pts, double *d_pts,
                      Region *outs, int nout, Launch launch) {
  IkPipe &p = c->pipe;
  // the copy streams start after whatever the context's stream already holds
  IK_HIP(hipEventRecord(p.ev_out, c->stream));
  IK_HIP(hipStreamWaitEvent(p.s_in, p.ev_out, 0));
  IK_HIP(hipStreamWaitEvent(p.s_out, p.ev_out, 0));
  for (int k = 0; k < K; ++k) {
    const int64_t b = begin[k], m = begin[k + 1] - begin[k];
    IK_HIP(hipMemcpyAsync(d_pts + 3 * b, pts + 3 * b, (size_t)m * 24, hipMemcpyHostToDevice,
                          p.s_in));
    IK_HIP(hipEventRecord(p.ev_in[k], p.s_in));
    IK_HIP(hipStreamWaitEvent(c->stream, p.ev_in[k], 0));
    int rc = launch(k, b, m);
    if (rc) return rc;
    IK_HIP(hipEventRecord(p.ev_done[k], c->stream));
    IK_HIP(hipStreamWaitEvent(p.s_out, p.ev_done[k], 0));
    // every D2H on the copy-out stream (the compute stream issues no copies)
    IK_HIP(hipMemcpyAsync(&p.h_stats[k], &p.d_stats[k], sizeof(DevStats), hipMemcpyDeviceToHost,
                          p.s_out));
    for (int r = 0; r < nout; ++r)
      if (outs[r].host)
        IK_HIP(hipMemcpyAsync(outs[r].host + b * outs[r].row, outs[r].dev + b * outs[r].row,
                              (size_t)m * outs[r].row, hipMemcpyDeviceToHost, p.s_out));
  }
  return IK_OK;
}

int fabrik_host_pipeline(ik_ctx *c, const double *pts, int64_t n, double tol, int max_iter,
                         double *ang, int32_t *iters, double *joints, double *fk_err, int flags,
                         ik_stats *stats) {
  const int K = chunks_for(n);
  int64_t begin[kPipeMaxChunks + 1];
  for (int k = 0; k <= K; ++k) begin[k] = n * k / K;
  const size_t b_pts = Stage::up((size_t)n * 24), b_ang = Stage::up((size_t)n * 32);
  const size_t b_it = iters ? Stage::up((size_t)n * 4) : 0;
  const size_t b_jo = joints ? Stage::up((size_t)n * 96) : 0;
  const size_t b_fe = fk_err ? Stage::up((size_t)n * 8) : 0;
  const size_t b_work = Stage::up(fabrik_scratch_bytes(begin[1] + 1));  // chunks differ by <= 1
  int rc = pipe_ready(c, b_pts + b_ang + b_it + b_jo + b_fe + b_work);
  if (rc) return rc;
  char *q = static_cast<char *>(c->pipe.buf);
  double *d_pts = reinterpret_cast<double *>(q);
  q += b_pts;
  Region outs[4] = {{32, reinterpret_cast<char *>(ang), q}, {4, nullptr, nullptr},
                    {96, nullptr, nullptr}, {8, nullptr, nullptr}};
  q += b_ang;
  if (iters) outs[1] = {4, reinterpret_cast<char *>(iters), q};
  q += b_it;
  if (joints) outs[2] = {96, reinterpret_cast<char *>(joints), q};
  q += b_jo;
  if (fk_err) outs[3] = {8, reinterpret_cast<char *>(fk_err), q};
  q += b_fe;
  void *work = q;
  const bool limits = !(flags & IK_F_NO_LIMITS);
  rc = run_chunks(c, K, begin, pts, d_pts, outs, 4, [&](int k, int64_t b, int64_t m) {
    return fabrik_launch(
        c, d_pts + 3 * b, m, tol, max_iter, reinterpret_cast<double *>(outs[0].dev) + 4 * b,
        iters ? reinterpret_cast<int32_t *>(outs[1].dev) + b : nullptr,
        joints ? reinterpret_cast<double *>(outs[2].dev) + 12 * b : nullptr,
        fk_err ? reinterpret_cast<double *>(outs[3].dev) + b : nullptr, limits, work,
        &c->pipe.d_stats[k]);
  });
  if (rc) return rc;
  return merge_chunk_stats(c, K, begin, stats);
}

}  // namespace ikapi

extern "C" {

int ik_host_alloc(size_t bytes, void **out) {
  if (!out) return ikapi::fail(IK_E_BADARG, "ik_host_alloc: out is NULL");
  *out = nullptr;
  IK_HIP(hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault));
  return IK_OK;
}

int ik_host_free(void *p) {
  if (p) IK_HIP(hipHostFree(p));
  return IK_OK;
}

}  // extern "C"
