// ik_internal.h -- the context behind the C ABI and the helpers its
// translation units share (ik_api.cpp: single-device calls; ik_comm.cpp: the
// RCCL-sharded calls).  Not installed; include/ikhip.h is the interface.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <initializer_list>
#include <string>

#include "ik_common.h"

namespace ikhip {
constexpr int kMaxTimed = 64;  // kernels timed per call (the layered ANN path launches one per layer)
struct KTimer {
  bool on = false;
  bool acc = false;  // ik_ctx_set_timing(ctx, 2): the calls' kernels accumulate
  int n = 0;
  // slot n's state: 1 = armed by kt_begin (the next IK_LAUNCH takes its events),
  // 2 = stamped by that dispatch, 3 = a marker span (kt_span_begin)
  int state = 0;
  hipEvent_t beg[kMaxTimed] = {};
  hipEvent_t end[kMaxTimed] = {};
  const char *name[kMaxTimed] = {};
};
}  // namespace ikhip

// What a rank planned its sharded call with; every rank's must agree (a rank
// that planned another batch or chunk count gathered other rows).
struct IkPlanHdr {
  int64_t n;
  int32_t chunks, method;
  uint32_t magic, pad;
};
constexpr uint32_t kPlanMagic = 0x494b5348u;  // "IKSH"

// One rank's tail block as gathered: the stats record, the plan, then its
// FK-error histogram.
struct IkTailBlock {
  ik_shard_tail t;
  IkPlanHdr plan;
  uint32_t hist[IK_FKHIST_BINS];
};

// One RCCL communicator of a context (ik_comm_init) and the state of the
// chunked in-place all-gathers of the sharded solves (ik_shard.hip), grow-only
// like the scratch.
struct IkComm {
  void *comm = nullptr;  // ncclComm_t (a non-null sentinel for a loopback communicator)
  bool loopback = false;  // ik_comm_init_loopback (test-only): no RCCL, see ik_shard.hip
  int nranks = 0, rank = -1;
  int chunks_req = 0;    // ik_comm_set_chunks (0 = automatic)
  int last_chunks = 0;   // all-gathers of the last sharded call (its plan's chunks)
  int last_req = 0;      // the chunk count that plan was made with (ik_comm_info)
  bool last_hist = false;  // the last sharded call gathered FK-error histograms
  hipStream_t cs = nullptr;  // the gathers' stream
  void *stage = nullptr;     // the ragged last chunk's rows (all regions)
  size_t stage_bytes = 0;
  IkTailBlock *tail_send = nullptr;  // device: this rank's tail block
  IkTailBlock *tail_recv = nullptr;  // device: every rank's
  IkTailBlock *h_tails = nullptr;    // pinned: every rank's
  int tails_n = 0;
  ikhip::DevStats *d_cstats = nullptr;  // one stats block per chunk
  hipEvent_t ev_solved[IK_MAX_GATHER_CHUNKS] = {};  // chunk k's rows written (solve stream)
  hipEvent_t ev_gs[IK_MAX_GATHER_CHUNKS] = {}, ev_ge[IK_MAX_GATHER_CHUNKS] = {};  // gather k
  hipEvent_t ev_done = nullptr;  // the call's last gather / copy on cs
  // Bounded waits (ik_shard.hip comm_wait): every host wait on the collective
  // polls the communicator's async error against this deadline and aborts the
  // communicator when it passes, so a dead or stuck peer ends in IK_E_RCCL
  // instead of a hang.  0 = IKHIP_RCCL_TIMEOUT_S, else 120 s.
  double timeout_s = 0.0;
  bool broken = false;   // aborted (deadline, async error, mid-call failure): calls refuse
  std::string why;       // ... and why
  hipEvent_t ev_end = nullptr;  // the last sharded call's end on its solve stream
  bool ev_end_set = false;
  // ik_comm_loopback_stall (test-only): the loopback all-gathers spin on this
  // pinned flag until the deadline's abort sets it (or their own 30 s cap)
  int *stall_flag = nullptr;
  bool stall = false;
};

// The chunked host-pointer pipeline (ik_pipe.cpp): copy streams, per-chunk
// events and stats blocks, device staging; created on first use.
constexpr int kPipeMaxChunks = 8;
struct IkPipe {
  hipStream_t s_in = nullptr, s_out = nullptr;
  hipEvent_t ev_in[kPipeMaxChunks] = {}, ev_done[kPipeMaxChunks] = {}, ev_out = nullptr;
  ikhip::DevStats *d_stats = nullptr;  // kPipeMaxChunks blocks
  ikhip::DevStats *h_stats = nullptr;  // pinned copies
  void *buf = nullptr;
  size_t buf_bytes = 0;
};

struct ik_ctx {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  ikhip::DevStats *d_stats = nullptr;
  ikhip::DevStats *h_stats = nullptr;  // pinned
  void *scratch = nullptr;
  size_t scratch_bytes = 0;
  ikhip::RobotDev robot;
  bool ann_loaded = false;
  ikhip::AnnModelDev ann;
  void *ann_buf = nullptr;
  const void *ann_wx[ikhip::kAnnMaxLayers] = {};  // bf16x6 weight operand of each layer
  const void *ann_wh[ikhip::kAnnMaxLayers] = {};  // fp16x3 weight operand of each layer
  float ann_hinv[ikhip::kAnnMaxLayers] = {};      // fp16x3: 2^-(weight pre-scale exponent)
  int ann_mode = IK_ANN_FP32;
  // a model outside the fused kernel's caps runs layer at a time (ik_ann_big.hip)
  bool ann_big = false;
  ikhip::AnnBigModel ann_bigm;  // its layers (pointers into ann_buf)
  void *ann_act = nullptr;      // its activation buffers, grow-only
  size_t ann_act_bytes = 0;
  int fabrik_variant = 1;
  int fabrik_bpc = 0;   // IKHIP_FABRIK_BPC: iteration-kernel blocks per CU (0 = size rule)
  int fabrik_core = 2;  // IKHIP_FABRIK_CORE: 2 core + reuse, 1 sqrt_core / div_core, 0 general
  ikhip::KTimer kt;
  unsigned long long *dbg = nullptr;     // diagnostic stamp buffer (ik_ctx_set_debug)
  ikhip::FabOrderDev *fab_ord = nullptr;  // FABRIK work-order cost table (learned per robot)
  unsigned int *fab_priors = nullptr;     // device copies of the built-in tables (ik_fabrik_prior.h)
  int fab_prior = -1;  // the built-in table fab_ord holds untouched (index), -1 learned / empty
  ikhip::RobotConstDev *rconst = nullptr;  // FABRIK seed-pose constants of the robot
  IkComm comm;
  IkPipe pipe;
  hipStream_t last_stream = nullptr;  // the stream the last solve was enqueued on
  hipEvent_t call_done = nullptr;     // recorded on last_stream at the end of every call
  bool call_done_set = false;
  bool last_sharded = false;  // the last call's stats are in comm.h_tails
  // the gathered tails of the last sharded call (for IK_F_ASYNC + ik_stats_fetch)
  int64_t last_n = 0;
  bool last_piped = false;  // the last call was a chunked host pipeline: its stats are piped_stats
  ik_stats piped_stats = {};
};

namespace ikapi {

int fail(int code, const std::string &msg);

#define IK_HIP(call)                                                                 \
  do {                                                                               \
    hipError_t e_ = (call);                                                          \
    if (e_ != hipSuccess)                                                            \
      return ::ikapi::fail(IK_E_HIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)

// One enqueueing call: per-kernel HIP-event timing of it (ik_ctx_set_timing),
// and the context's one sequence of device work -- on entry the call's stream
// waits for the previous call's end event when that call ran on another stream;
// on exit the call records its own.
struct KtScope {
  explicit KtScope(ik_ctx *c);
  ~KtScope();
  ik_ctx *c_;
};

struct Stage {
  static size_t up(size_t b) { return (b + 255) & ~(size_t)255; }
};

int ensure_scratch(ik_ctx *c, size_t bytes);
int set_dev(ik_ctx *c);
void stats_from_dev(const ikhip::DevStats &d, ik_stats *s);
int finish(ik_ctx *c, int flags, ik_stats *stats);
// Device pointers only, on the context's stream: stats reset + the solve's kernels.
// work: fabrik_scratch_bytes(n) of device memory.
// S: the stats block (null: the context's).
int fabrik_launch(ik_ctx *c, const double *dp, int64_t n, double tol, int max_iter, double *da,
                  int32_t *di, double *dj, double *dfe, bool limits, void *work,
                  ikhip::DevStats *S = nullptr);
int ann_launch(ik_ctx *c, const double *dp, int64_t n, float *da, double *de, bool limits,
               ikhip::DevStats *S = nullptr);
// The FABRIK work order of a fresh table (ik_api.cpp): the built-in prior for
// (tol, max_iter) when the robot is SixDOFRobot's chain, else empty.
int seed_order(ik_ctx *c, double tol, int max_iter);
// FABRIK host-pointer solves whose arrays are all pinned (ik_host_alloc) and large enough:
// chunked H2D / solve / D2H on three streams (ik_pipe.cpp).
bool pipeline_wanted(ik_ctx *c, int64_t n, std::initializer_list<const void *> ptrs);
int fabrik_host_pipeline(ik_ctx *c, const double *pts, int64_t n, double tol, int max_iter,
                         double *ang, int32_t *iters, double *joints, double *fk_err, int flags,
                         ik_stats *stats);
void pipe_release(ik_ctx *c);
// The batch stats of the last sharded call, from the gathered tails (waits).
int sharded_stats(ik_ctx *c, ik_stats *stats);
// Releases the communicator; false when aborted work has not drained (its
// buffers are then left to the process's end).
bool comm_release(ik_ctx *c);
// Waits for `ev` with the communicator's deadline and async-error polling when
// the context holds a live communicator (else a plain hipEventSynchronize).
int comm_wait(ik_ctx *c, hipEvent_t ev, const char *what);

}  // namespace ikapi
