// ik_shard.hip -- the batch sharded over GPUs, gathered in place over RCCL in
// chunks that overlap the solve (include/ikhip.h "multi-GPU").
//
// The reference scales by competing consumers (rpc_broker.py:55-68): each worker
// takes whole requests.  Here the points of one batch are independent, so the
// batch is split over the ranks (one process per GPU) in C chunks of g parts:
// rank r owns part (c, r) = rows [(c g + r) S, (c g + r + 1) S) of every chunk c,
// S = ceil(n / (C g)).  Each chunk is contiguous in the caller's arrays and every
// rank's part of it sits at rank offset r S, which is exactly ncclAllGather's
// in-place layout (sendbuf = recvbuf + r count): the solve writes its rows at
// their global position and the all-gather of chunk c fills in the other ranks'
// rows, on a second stream, while the solve stream runs chunk c + 1.  There is no
// pack and no unpack kernel; only the ragged last chunk (when C g S > n) is
// gathered through a staging buffer of g S rows and copied out (its rows are in
// global order there too, truncated at n).
//
// What is gathered per row is what the reference returns: the angles (and the
// FABRIK iteration counts, the bit-exact integer result).  The per-point FK
// error stays on its rank; the batch's FK-error max / sum and a 2048-bin
// histogram (quantiles) travel in a per-rank tail block with the last chunk,
// beside first_oob / first_err (lowest GLOBAL index: the reference's sequential
// exception precedence), the iteration sum and the capped count.  No all_reduce.
//
// RCCL is loaded at run time (dlopen): a librccl the process already holds
// (torch ships one, built against the HIP runtime the process uses; found by
// walking the loaded objects), else librccl.so.1 from the ROCm install.
#include <dlfcn.h>
#include <link.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>

#include "ik_internal.h"

using namespace ikhip;
using namespace ikapi;

namespace {

// ---- RCCL entry points (rccl.h, loaded by name) ---------------------------
typedef int (*GetUniqueIdFn)(void *id);
// ncclUniqueId: a 128-byte struct passed by value (same ABI as this one)
struct IdBlob {
  char b[IK_COMM_ID_BYTES];
};
// ncclConfig_t as rccl.h (ncclConfig_v22700) lays it out.  RCCL copies
// min(size, its own sizeof) bytes of it, so an older librccl (torch's 2.26)
// reads the prefix it knows; NCCL_CONFIG_INITIALIZER's values, blocking = 0.
struct NcclConfig {
  size_t size = sizeof(NcclConfig);
  unsigned int magic = 0xcafebeefu;
  unsigned int version = 22707;  // NCCL_VERSION(2, 27, 7)
  int blocking = 0;              // non-blocking: init and group ends return ncclInProgress
  int cga_cluster_size = INT32_MIN, min_ctas = INT32_MIN, max_ctas = INT32_MIN;
  const char *net_name = nullptr;
  int split_share = INT32_MIN, traffic_class = INT32_MIN;
  const char *comm_name = nullptr;
  int collnet_enable = INT32_MIN, cta_policy = INT32_MIN, shrink_share = INT32_MIN,
      nvls_ctas = INT32_MIN;
};
typedef int (*CommInitRankBlobFn)(void **comm, int nranks, IdBlob id, int rank);
typedef int (*CommInitRankConfigFn)(void **comm, int nranks, IdBlob id, int rank,
                                    NcclConfig *config);
typedef int (*CommFn)(void *comm);
typedef int (*CommAsyncErrorFn)(void *comm, int *result);
typedef int (*AllGatherFn)(const void *send, void *recv, size_t count, int dtype, void *comm,
                           hipStream_t stream);
typedef int (*GroupFn)();
typedef const char *(*GetErrorStringFn)(int);
constexpr int kNcclUint8 = 1;       // ncclDataType_t ncclUint8
constexpr int kNcclInProgress = 7;  // ncclResult_t ncclInProgress

struct Rccl {
  void *lib = nullptr;
  GetUniqueIdFn get_unique_id = nullptr;
  CommInitRankBlobFn comm_init_rank = nullptr;
  CommInitRankConfigFn comm_init_rank_config = nullptr;  // non-blocking init (may be absent)
  CommFn comm_destroy = nullptr, comm_abort = nullptr;
  CommAsyncErrorFn comm_async_error = nullptr;
  AllGatherFn all_gather = nullptr;
  GroupFn group_start = nullptr, group_end = nullptr;
  GetErrorStringFn error_string = nullptr;
  std::string where;
  // the bounded-wait path needs all three; else the communicator is blocking
  bool nonblocking() const { return comm_init_rank_config && comm_abort && comm_async_error; }
};

std::mutex g_rccl_mu;
Rccl g_rccl;

// The path of a librccl*.so* already mapped into the process (torch's bundled
// copy may carry another soname than librccl.so.1), or "".
int find_loaded_rccl(struct dl_phdr_info *info, size_t, void *data) {
  const char *p = info->dlpi_name;
  if (!p || !*p) return 0;
  const char *base = std::strrchr(p, '/');
  base = base ? base + 1 : p;
  if (std::strncmp(base, "librccl", 7) == 0 && std::strstr(base, ".so")) {
    *static_cast<std::string *>(data) = p;
    return 1;
  }
  return 0;
}

int load_rccl(Rccl **out) {
  std::lock_guard<std::mutex> lk(g_rccl_mu);
  if (!g_rccl.lib) {
    const char *over = std::getenv("IKHIP_RCCL_LIB");
    void *h = nullptr;
    std::string where;
    if (over && *over) {
      h = dlopen(over, RTLD_NOW | RTLD_LOCAL);
      where = over;
    } else {
      // a librccl the process already holds (torch's), then the ROCm one
      std::string loaded;
      dl_iterate_phdr(find_loaded_rccl, &loaded);
      if (!loaded.empty()) {
        h = dlopen(loaded.c_str(), RTLD_NOW | RTLD_NOLOAD);
        where = loaded + " (already loaded)";
      }
      for (const char *nm : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1"}) {
        if (h) break;
        h = dlopen(nm, RTLD_NOW | RTLD_LOCAL);
        where = nm;
      }
    }
    if (!h) {
      const char *e = dlerror();
      return fail(IK_E_RCCL, std::string("RCCL not found: ") + (e ? e : "dlopen failed"));
    }
    Rccl r;
    r.lib = h;
    r.where = where;
    r.get_unique_id = reinterpret_cast<GetUniqueIdFn>(dlsym(h, "ncclGetUniqueId"));
    r.comm_init_rank = reinterpret_cast<CommInitRankBlobFn>(dlsym(h, "ncclCommInitRank"));
    r.comm_init_rank_config =
        reinterpret_cast<CommInitRankConfigFn>(dlsym(h, "ncclCommInitRankConfig"));
    r.comm_destroy = reinterpret_cast<CommFn>(dlsym(h, "ncclCommDestroy"));
    r.comm_abort = reinterpret_cast<CommFn>(dlsym(h, "ncclCommAbort"));
    r.comm_async_error = reinterpret_cast<CommAsyncErrorFn>(dlsym(h, "ncclCommGetAsyncError"));
    r.all_gather = reinterpret_cast<AllGatherFn>(dlsym(h, "ncclAllGather"));
    r.group_start = reinterpret_cast<GroupFn>(dlsym(h, "ncclGroupStart"));
    r.group_end = reinterpret_cast<GroupFn>(dlsym(h, "ncclGroupEnd"));
    r.error_string = reinterpret_cast<GetErrorStringFn>(dlsym(h, "ncclGetErrorString"));
    if (!r.get_unique_id || !r.comm_init_rank || !r.comm_destroy || !r.all_gather ||
        !r.group_start || !r.group_end)
      return fail(IK_E_RCCL, "RCCL at " + where + " lacks ncclGetUniqueId / ncclCommInitRank / "
                                                  "ncclCommDestroy / ncclAllGather / ncclGroup*");
    g_rccl = r;
  }
  *out = &g_rccl;
  return IK_OK;
}

int rccl_fail(const Rccl *r, const char *what, int res) {
  const char *msg = (r && r->error_string) ? r->error_string(res) : "?";
  return fail(IK_E_RCCL, std::string(what) + ": " + msg + " (" + std::to_string(res) + ")");
}

// ---- bounded waits -----------------------------------------------------------
using Clock = std::chrono::steady_clock;

double since(Clock::time_point t0) {
  return std::chrono::duration<double>(Clock::now() - t0).count();
}

// One poll's back-off: yield for the first ~2000 polls (a few ms), then sleep 50 us.
void backoff(int &spins) {
  if (++spins < 2000)
    std::this_thread::yield();
  else
    std::this_thread::sleep_for(std::chrono::microseconds(50));
}

double comm_timeout(const IkComm &m) {
  if (m.timeout_s > 0.0) return m.timeout_s;
  static double env = -1.0;
  if (env < 0.0) {
    const char *e = std::getenv("IKHIP_RCCL_TIMEOUT_S");
    const double v = (e && *e) ? std::atof(e) : 0.0;
    env = v > 0.0 ? v : 120.0;
  }
  return env;
}

std::string rank_tag(const IkComm &m) {
  return "rank " + std::to_string(m.rank) + " of " + std::to_string(m.nranks);
}

std::string secs_str(double s) {
  char b[32];
  std::snprintf(b, sizeof(b), "%.3g", s);
  return b;
}

// A non-blocking communicator's pending operation (init, a group end, a lone
// collective): poll its async state until it leaves ncclInProgress or the
// deadline passes.  Returns the final ncclResult_t, or -1 on timeout.
int rccl_settle(Rccl *r, void *comm, double timeout) {
  if (!r->comm_async_error) return 0;
  const Clock::time_point t0 = Clock::now();
  int spins = 0;
  for (;;) {
    int st = 0;
    const int q = r->comm_async_error(comm, &st);
    if (q != 0) return q;
    if (st != kNcclInProgress) return st;
    if (since(t0) > timeout) return -1;
    backoff(spins);
  }
}

// Marks the communicator unusable and stops its collectives: ncclCommAbort (the
// RCCL kernels poll its abort flag and exit), or for the loopback the stall
// flag; then lets `drain` complete for up to 10 s.  Returns IK_E_RCCL(why).
int comm_abort(ik_ctx *c, hipEvent_t drain, const std::string &why) {
  IkComm &m = c->comm;
  if (!m.broken) {
    m.broken = true;
    m.why = why;
    if (m.loopback) {
      if (m.stall_flag) __atomic_store_n(m.stall_flag, 1, __ATOMIC_SEQ_CST);
    } else {
      Rccl *r = nullptr;
      if (load_rccl(&r) == IK_OK && r->comm_abort) (void)r->comm_abort(m.comm);
    }
  }
  if (drain) {
    const Clock::time_point t0 = Clock::now();
    int spins = 0;
    while (hipEventQuery(drain) == hipErrorNotReady && since(t0) < 10.0) backoff(spins);
  }
  return fail(IK_E_RCCL, why);
}

// Whether the communicator's streams hold no pending work (after an abort).
bool comm_drained(const IkComm &m) {
  if (m.cs && hipStreamQuery(m.cs) == hipErrorNotReady) return false;
  if (m.ev_end_set && hipEventQuery(m.ev_end) == hipErrorNotReady) return false;
  return true;
}

bool plan_args_ok(int64_t n, int nranks, int chunks) {
  return n >= 0 && n < ((int64_t)1 << 48) && nranks >= 1 && nranks <= 1024 && chunks >= 1 &&
         chunks <= IK_MAX_GATHER_CHUNKS;
}

// S = ceil(n / (C g)); the chunks that hold rows; the rows of the full ones.
void make_plan(int64_t n, int g, int C, ik_shard_plan *p) {
  std::memset(p, 0, sizeof(*p));
  p->n = n;
  p->nranks = g;
  const int64_t cg = (int64_t)C * g;
  p->part_rows = n > 0 ? (n + cg - 1) / cg : 0;
  const int64_t per_chunk = p->part_rows * g;
  p->chunks = n > 0 ? (int)((n + per_chunk - 1) / per_chunk) : 0;
  p->full_rows = per_chunk > 0 ? (n / per_chunk) * per_chunk : 0;
}

void part_of(const ik_shard_plan &p, int r, int c, int64_t *b, int64_t *e) {
  const int64_t S = p.part_rows;
  const int64_t lo = ((int64_t)c * p.nranks + r) * S, hi = lo + S;
  *b = lo < p.n ? lo : p.n;
  *e = hi < p.n ? hi : p.n;
}

}  // namespace

namespace ikhip {

// The rank's FK errors of one part into its tail block's histogram.
__global__ __launch_bounds__(256) void fk_hist_kernel(const double *err, int64_t n,
                                                      uint32_t *hist) {
  __shared__ uint32_t h[IK_FKHIST_BINS];
  for (int i = threadIdx.x; i < IK_FKHIST_BINS; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int b = fkhist_bin(err[i]);
    if (b >= 0) atomicAdd(&h[b], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < IK_FKHIST_BINS; i += blockDim.x)
    if (h[i]) atomicAdd(&hist[i], h[i]);
}

// The rank's tail: its chunks' DevStats merged, indices made global (the
// chunks are in increasing global order, so the first chunk holding a failure
// holds the rank's lowest failing index).
struct TailArgs {
  const DevStats *S;  // K blocks
  int K;
  int64_t base[IK_MAX_GATHER_CHUNKS];  // global row of each chunk's part's first row
  int64_t rows;
  IkPlanHdr plan;  // what this rank planned the call with
};

__global__ void pack_tail_kernel(TailArgs a, IkTailBlock *blk) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  blk->plan = a.plan;
  ik_shard_tail *t = &blk->t;
  ik_shard_tail o;
  o.first_oob = -1;
  o.first_err = -1;
  o.first_err_code = IK_OK;
  o.max_iters = 0;
  o.sum_iters = 0;
  o.n_capped = 0;
  o.max_fk_err = 0.0;
  o.sum_fk_err = 0.0;
  for (int k = 0; k < a.K; ++k) {
    const DevStats *S = a.S + k;
    if (o.first_oob < 0 && S->first_oob != ~0ull) o.first_oob = (int64_t)S->first_oob + a.base[k];
    if (o.first_err < 0 && S->first_err_key != ~0ull) {
      o.first_err = (int64_t)(S->first_err_key >> 8) + a.base[k];
      o.first_err_code = (int32_t)(S->first_err_key & 0xff);
    }
    for (int s = 0; s < kStatShards; ++s) {  // the shard order of stats_from_dev
      o.max_iters = S->max_iters[s] > o.max_iters ? S->max_iters[s] : o.max_iters;
      o.sum_iters += (int64_t)S->sum_iters[s];
      o.n_capped += (int64_t)S->n_capped[s];
      const double mx = __longlong_as_double((long long)S->max_fk_err_bits[s]);
      o.max_fk_err = mx > o.max_fk_err ? mx : o.max_fk_err;
      o.sum_fk_err += S->sum_fk_err[s];
    }
  }
  o.rows = a.rows;
  *t = o;
}

// ik_comm_init_loopback's all-gather (test-only): one GPU plays rank `me` of g.
// The other ranks' slots of the receive buffer get a fixed byte pattern of
// (slot, byte offset), ik_loopback_byte, so a test can check where the plan put
// every foreign row (in place and through the stage); tail blocks (replicate)
// get a copy of this rank's.
__host__ __device__ inline uint8_t loopback_byte(int slot, uint64_t o) {
  return (uint8_t)(((uint32_t)slot * 29u + (uint32_t)o * 13u + (uint32_t)(o >> 7)) ^ 0xA5u);
}

// stall (ik_comm_loopback_stall, test-only): a pinned host flag; every block
// first waits for it to turn non-zero -- a peer that never arrives -- or for
// cap_ticks of the 100 MHz wall clock, so the grid always drains.
__global__ __launch_bounds__(256) void loopback_gather_kernel(const uint8_t *send, uint8_t *recv,
                                                              uint64_t cnt, int g, int me,
                                                              int replicate, const int *stall,
                                                              long long cap_ticks) {
  if (stall) {
    if (threadIdx.x == 0) {
      const long long t0 = wall_clock64();
      while (__hip_atomic_load(stall, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0 &&
             wall_clock64() - t0 < cap_ticks)
        __builtin_amdgcn_s_sleep(127);
    }
    __syncthreads();
  }
  const uint64_t tot = cnt * (uint64_t)g;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < tot;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const int s = (int)(i / cnt);
    const uint64_t o = i - (uint64_t)s * cnt;
    recv[i] = (s == me || replicate) ? send[o] : loopback_byte(s, o);  // in place: same byte
  }
}

}  // namespace ikhip

namespace {

int env_chunks() {
  static int env = -1;
  if (env < 0) {
    const char *e = std::getenv("IKHIP_GATHER_CHUNKS");
    env = (e && *e) ? std::atoi(e) : 0;
  }
  return env;
}

int auto_chunks(ik_ctx *c, int method, int64_t n) {
  const IkComm &m = c->comm;
  int C = m.chunks_req;
  if (C <= 0) C = env_chunks();
  // automatic: one chunk for both methods.  ANN's gather is ~0.5 % of the solve;
  // FABRIK's 32-byte rows gather in about the solve's time at 8 ranks, and two
  // chunks would overlap chunk 0's gather with chunk 1's solve (DESIGN.md §5's
  // model: 0.93 against 1.06 ms a step for configs[4] at 8 ranks), but the
  // chunked gather has run bit-checked only through the loopback communicator,
  // never across real RCCL ranks, so it stays opt-in (ik_comm_set_chunks /
  // IKHIP_GATHER_CHUNKS) until an N >= 2 run records its gather check (ADVICE
  // r05).  The plan depends only on (n, g, method) and the explicit setting, so
  // every rank makes the same one (ik_comm_init checks the environment's, every
  // call's tail its plan); bench.py's gather check compares the gathered rows
  // with a plain re-solve bit for bit on every N > 1 run.
  (void)n;
  (void)method;
  if (C <= 0) C = 1;
  return C > IK_MAX_GATHER_CHUNKS ? IK_MAX_GATHER_CHUNKS : C;
}

int ensure_comm_state(ik_ctx *c, size_t stage) {
  IkComm &m = c->comm;
  if (!m.cs) {
    IK_HIP(hipStreamCreateWithFlags(&m.cs, hipStreamNonBlocking));
    for (int k = 0; k < IK_MAX_GATHER_CHUNKS; ++k) {
      IK_HIP(hipEventCreateWithFlags(&m.ev_solved[k], hipEventDisableTiming));
      IK_HIP(hipEventCreate(&m.ev_gs[k]));
      IK_HIP(hipEventCreate(&m.ev_ge[k]));
    }
    IK_HIP(hipEventCreateWithFlags(&m.ev_done, hipEventDisableTiming));
    IK_HIP(hipEventCreateWithFlags(&m.ev_end, hipEventDisableTiming));
    IK_HIP(hipMalloc(&m.d_cstats, sizeof(DevStats) * IK_MAX_GATHER_CHUNKS));
    IK_HIP(hipMalloc(&m.tail_send, sizeof(IkTailBlock)));
  }
  // the previous sharded call's gathers finished before its solve stream did
  // (it waited for ev_done), so its end frees every buffer below; waited for
  // with the deadline (a stuck peer aborts the communicator, not this thread)
  if ((stage > m.stage_bytes || m.tails_n < m.nranks) && m.ev_end_set) {
    const int rc = comm_wait(c, m.ev_end, "the previous sharded call");
    if (rc) return rc;
  }
  if (stage > m.stage_bytes) {
    if (m.stage) IK_HIP(hipFree(m.stage));
    m.stage = nullptr;
    m.stage_bytes = 0;
    IK_HIP(hipMalloc(&m.stage, stage));
    m.stage_bytes = stage;
  }
  if (m.tails_n < m.nranks) {
    if (m.tail_recv) IK_HIP(hipFree(m.tail_recv));
    if (m.h_tails) IK_HIP(hipHostFree(m.h_tails));
    m.tail_recv = nullptr;
    m.h_tails = nullptr;
    m.tails_n = 0;
    IK_HIP(hipMalloc(&m.tail_recv, sizeof(IkTailBlock) * (size_t)m.nranks));
    IK_HIP(hipHostMalloc(reinterpret_cast<void **>(&m.h_tails),
                         sizeof(IkTailBlock) * (size_t)m.nranks, hipHostMallocDefault));
    m.tails_n = m.nranks;
  }
  return IK_OK;
}

// One gathered output: row bytes, the caller-visible device rows (n of them;
// the caller's array, or device scratch for host pointers), the staging rows of
// the ragged chunk.
struct Region {
  int rb;
  char *out;
  char *stage;
};

// The solve of one part: rows [b, b + m) of the batch; `at(q)` is where
// region q's first row goes; fk_err (device, nullable) the part's FK errors;
// S the chunk's stats block.
struct PartJob {
  int64_t b, m;
  char *at[2];
  double *fk_err;
  DevStats *S;
};

// The whole sharded call after argument checks: per chunk, the solve of this
// rank's part on the context's stream, then the in-place all-gather of the
// chunk on the comm stream; the tail block with the last chunk; the ragged
// chunk's rows out of the stage; the solve stream waits for the gathers.
template <class Solve>
int sharded_enqueue(ik_ctx *c, int method, const ik_shard_plan &P, Region *R, int nreg,
                    double *fk_err_dev, Solve solve, int *gathers) {
  IkComm &m = c->comm;
  Rccl *r = nullptr;
  int rc = m.loopback ? IK_OK : load_rccl(&r);
  if (rc) return rc;
  const int g = m.nranks, me = m.rank, C = P.chunks;
  const double T = comm_timeout(m);
  long long cap_ticks = 0;
  if (m.loopback && m.stall) {
    int khz = 0;
    IK_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device));
    cap_ticks = (long long)(khz > 0 ? khz : 100000) * 1000 * 30;  // 30 s
  }
  // one all-gather of cnt bytes per rank on the comm stream (inside a group);
  // a non-blocking communicator may answer ncclInProgress (settled at the group end)
  auto gather = [&](const void *send, void *recv, size_t cnt, bool replicate) -> int {
    ++*gathers;
    if (m.loopback) {
      const uint64_t tot = (uint64_t)cnt * g, blocks = (tot + 255) / 256;
      if (tot)
        IK_LAUNCH(loopback_gather_kernel, dim3((unsigned)(blocks < 1024 ? blocks : 1024)),
                           dim3(256), 0, m.cs, static_cast<const uint8_t *>(send),
                           static_cast<uint8_t *>(recv), (uint64_t)cnt, g, me, replicate ? 1 : 0,
                           m.stall ? m.stall_flag : nullptr, cap_ticks);
      IK_HIP(hipGetLastError());
      return IK_OK;
    }
    const int res = r->all_gather(send, recv, cnt, kNcclUint8, m.comm, m.cs);
    return (res && res != kNcclInProgress) ? rccl_fail(r, "ncclAllGather", res) : IK_OK;
  };
  // the group end of a non-blocking communicator enqueues asynchronously: wait
  // (bounded) until the kernels are on the comm stream before recording its events
  auto group = [&](bool start) -> int {
    if (m.loopback) return IK_OK;
    int res = start ? r->group_start() : r->group_end();
    if (!start && res == kNcclInProgress) {
      res = rccl_settle(r, m.comm, T);
      if (res < 0)
        return fail(IK_E_RCCL, "ncclGroupEnd did not settle within " + secs_str(T) + " s");
    }
    return res ? rccl_fail(r, start ? "ncclGroupStart" : "ncclGroupEnd", res) : IK_OK;
  };
  const int64_t S = P.part_rows;
  m.last_chunks = C;
  m.last_hist = fk_err_dev != nullptr;
  // the tail block: zeroed (histogram) before any part adds to it
  IK_HIP(hipMemsetAsync(m.tail_send, 0, sizeof(IkTailBlock), c->stream));
  TailArgs ta;
  std::memset(&ta, 0, sizeof(ta));
  ta.S = m.d_cstats;
  ta.K = C;
  ta.plan.n = P.n;
  ta.plan.chunks = C;
  ta.plan.method = method;
  ta.plan.magic = kPlanMagic;
  for (int k = 0; k < C; ++k) {
    int64_t b, e;
    part_of(P, me, k, &b, &e);
    const int64_t cb = (int64_t)k * g * S;  // the chunk's first row
    const bool staged = cb + g * S > P.n;  // the ragged last chunk
    PartJob j;
    j.b = b;
    j.m = e - b;
    for (int q = 0; q < 2; ++q)
      j.at[q] = q < nreg ? (staged ? R[q].stage + (int64_t)me * S * R[q].rb
                                   : R[q].out + b * R[q].rb)
                         : nullptr;
    j.fk_err = fk_err_dev ? fk_err_dev + b : nullptr;
    j.S = m.d_cstats + k;
    ta.base[k] = b;
    ta.rows += j.m;
    if (j.m > 0) {
      if ((rc = solve(j))) return rc;
      if (j.fk_err) {
        const int64_t want = (j.m + 2047) / 2048;
        kt_begin("fk_hist_kernel", c->stream);
        IK_LAUNCH(fk_hist_kernel, dim3((unsigned)(want < 512 ? want : 512)), dim3(256),
                           0, c->stream, j.fk_err, j.m, m.tail_send->hist);
        kt_end(c->stream);
      }
    } else {
      launch_reset_stats(j.S, c->stream);  // an empty part: zero stats for the tail
    }
    const bool last = k == C - 1;
    if (last) {
      IK_LAUNCH(pack_tail_kernel, dim3(1), dim3(64), 0, c->stream, ta, m.tail_send);
    }
    IK_HIP(hipGetLastError());
    IK_HIP(hipEventRecord(m.ev_solved[k], c->stream));
    IK_HIP(hipStreamWaitEvent(m.cs, m.ev_solved[k], 0));
    // chunk k's rows of every rank, in place (+ every rank's tail block with the last)
    kt_span_begin("rccl_all_gather", m.cs);
    IK_HIP(hipEventRecord(m.ev_gs[k], m.cs));
    if ((rc = group(true))) return rc;
    for (int q = 0; q < nreg && !rc; ++q) {
      char *base = staged ? R[q].stage : R[q].out + cb * R[q].rb;
      const size_t cnt = (size_t)S * R[q].rb;
      rc = gather(base + (size_t)me * cnt, base, cnt, false);
    }
    if (last && !rc) rc = gather(m.tail_send, m.tail_recv, sizeof(IkTailBlock), true);
    if (rc) {
      (void)group(false);
      return rc;
    }
    if ((rc = group(false))) return rc;
    IK_HIP(hipEventRecord(m.ev_ge[k], m.cs));
    kt_end(m.cs);
    if (staged && cb < P.n)  // the ragged chunk: its rows are in global order in the stage
      for (int q = 0; q < nreg; ++q)
        IK_HIP(hipMemcpyAsync(R[q].out + cb * R[q].rb, R[q].stage, (size_t)(P.n - cb) * R[q].rb,
                              hipMemcpyDeviceToDevice, m.cs));
  }
  if (C == 0) {  // an empty batch: every rank still exchanges its (empty) tail
    launch_reset_stats(m.d_cstats, c->stream);
    ta.K = 1;
    IK_LAUNCH(pack_tail_kernel, dim3(1), dim3(64), 0, c->stream, ta, m.tail_send);
    IK_HIP(hipGetLastError());
    IK_HIP(hipEventRecord(m.ev_solved[0], c->stream));
    IK_HIP(hipStreamWaitEvent(m.cs, m.ev_solved[0], 0));
    IK_HIP(hipEventRecord(m.ev_gs[0], m.cs));
    if ((rc = group(true))) return rc;
    rc = gather(m.tail_send, m.tail_recv, sizeof(IkTailBlock), true);
    if (rc) {
      (void)group(false);
      return rc;
    }
    if ((rc = group(false))) return rc;
    IK_HIP(hipEventRecord(m.ev_ge[0], m.cs));
    m.last_chunks = 1;
  }
  // the call ends on the solve stream: it waits for the gathers, then the tails
  // go to the host
  IK_HIP(hipEventRecord(m.ev_done, m.cs));
  IK_HIP(hipStreamWaitEvent(c->stream, m.ev_done, 0));
  IK_HIP(hipMemcpyAsync(m.h_tails, m.tail_recv, sizeof(IkTailBlock) * (size_t)g,
                        hipMemcpyDeviceToHost, c->stream));
  IK_HIP(hipEventRecord(m.ev_end, c->stream));
  m.ev_end_set = true;
  c->last_sharded = true;
  c->last_n = P.n;
  return IK_OK;
}

// sharded_enqueue, and on a failure part-way (a solve launch, a collective call,
// the group end's deadline) the solve stream still ends after whatever reached
// the comm stream, and the communicator is aborted: this rank's sequence of
// collectives no longer matches its peers', so no later call may use it
// (ADVICE r03).
template <class Solve>
int sharded_run(ik_ctx *c, int method, const ik_shard_plan &P, Region *R, int nreg,
                double *fk_err_dev, Solve solve) {
  IkComm &m = c->comm;
  if (m.broken) return fail(IK_E_RCCL, "communicator aborted earlier (" + m.why +
                                           "); ik_comm_destroy and ik_comm_init again");
  int gathers = 0;
  const int rc = sharded_enqueue(c, method, P, R, nreg, fk_err_dev, solve, &gathers);
  if (rc == IK_OK) return IK_OK;
  const std::string msg = ik_last_error();
  if (hipEventRecord(m.ev_done, m.cs) == hipSuccess)
    (void)hipStreamWaitEvent(c->stream, m.ev_done, 0);
  c->last_sharded = false;
  return comm_abort(c, m.ev_done, rank_tag(m) + ": sharded call failed after " +
                                      std::to_string(gathers) + " all-gather(s) (" + msg +
                                      "); communicator aborted");
}

}  // namespace

namespace ikapi {

int comm_wait(ik_ctx *c, hipEvent_t ev, const char *what) {
  IkComm &m = c->comm;
  if (!m.comm) {
    IK_HIP(hipEventSynchronize(ev));
    return IK_OK;
  }
  if (m.broken)  // already aborted: at most a bounded drain, then the old reason
    return comm_abort(c, ev, "communicator aborted earlier (" + m.why + ")");
  Rccl *r = nullptr;
  if (!m.loopback && load_rccl(&r) != IK_OK) r = nullptr;
  const double T = comm_timeout(m);
  const Clock::time_point t0 = Clock::now();
  int spins = 0;
  for (;;) {
    const hipError_t e = hipEventQuery(ev);
    if (e == hipSuccess) return IK_OK;
    if (e != hipErrorNotReady)
      return fail(IK_E_HIP, std::string("waiting for ") + what + ": " + hipGetErrorString(e));
    if (r && r->comm_async_error) {
      int st = 0;
      if (r->comm_async_error(m.comm, &st) == 0 && st != 0 && st != kNcclInProgress) {
        const char *msg = r->error_string ? r->error_string(st) : "?";
        return comm_abort(c, ev, rank_tag(m) + ": " + what + ": RCCL async error " + msg + " (" +
                                     std::to_string(st) + "); communicator aborted");
      }
    }
    if (since(t0) > T)
      return comm_abort(c, ev, rank_tag(m) + ": " + what + " did not complete within " +
                                   secs_str(T) +
                                   " s (IKHIP_RCCL_TIMEOUT_S / ik_comm_set_timeout): a peer "
                                   "rank stopped or is in another collective; communicator "
                                   "aborted");
    backoff(spins);
  }
}

int sharded_stats(ik_ctx *c, ik_stats *stats) {
  IkComm &m = c->comm;
  int rc = comm_wait(c, m.ev_end, "the sharded call");
  if (rc) return rc;
  // every rank planned the same call (same batch size, chunk count, method):
  // else the rows it gathered belong to another plan
  const IkPlanHdr &h0 = m.h_tails[0].plan;
  for (int r = 0; r < m.nranks; ++r) {
    const IkPlanHdr &h = m.h_tails[r].plan;
    if (h.magic != kPlanMagic || h.n != h0.n || h.chunks != h0.chunks || h.method != h0.method)
      return comm_abort(
          c, nullptr,
          rank_tag(m) + ": rank " + std::to_string(r) + " planned (n " + std::to_string(h.n) +
              ", chunks " + std::to_string(h.chunks) + ", method " + std::to_string(h.method) +
              ") but rank 0 (n " + std::to_string(h0.n) + ", chunks " +
              std::to_string(h0.chunks) + ", method " + std::to_string(h0.method) +
              "): every rank must pass the same batch and chunk setting; communicator aborted");
  }
  if (!stats) return IK_OK;
  ik_shard_tail t[1024];
  for (int r = 0; r < m.nranks; ++r) t[r] = m.h_tails[r].t;
  rc = ik_tail_reduce(t, m.nranks, stats);
  if (rc) return rc;
  float tot = 0.0f;
  for (int k = 0; k < m.last_chunks; ++k) {
    float ms = 0.0f;
    if (hipEventElapsedTime(&ms, m.ev_gs[k], m.ev_ge[k]) == hipSuccess) tot += ms;
  }
  stats->gather_ms = tot;
  return IK_OK;
}

bool comm_release(ik_ctx *c) {
  IkComm &m = c->comm;
  // a live communicator's last call first ends, or is aborted at the deadline
  if (m.comm && !m.broken && m.ev_end_set) (void)comm_wait(c, m.ev_end, "the last sharded call");
  if (m.broken && !comm_drained(m)) {
    // aborted work still queued: freeing its buffers would block on it, so
    // they are left to the process's end (the communicator is unusable anyway)
    const int keep_chunks = m.chunks_req;
    const double keep_t = m.timeout_s;
    m = IkComm();
    m.chunks_req = keep_chunks;
    m.timeout_s = keep_t;
    c->last_sharded = false;
    return false;
  }
  if (m.cs) (void)hipStreamSynchronize(m.cs);
  if (m.comm && !m.loopback && !m.broken) {  // (ncclCommAbort already freed an aborted one)
    Rccl *r = nullptr;
    if (load_rccl(&r) == IK_OK) (void)r->comm_destroy(m.comm);
  }
  if (m.stage) (void)hipFree(m.stage);
  if (m.tail_send) (void)hipFree(m.tail_send);
  if (m.tail_recv) (void)hipFree(m.tail_recv);
  if (m.h_tails) (void)hipHostFree(m.h_tails);
  if (m.d_cstats) (void)hipFree(m.d_cstats);
  if (m.stall_flag) (void)hipHostFree(m.stall_flag);
  for (int k = 0; k < IK_MAX_GATHER_CHUNKS; ++k) {
    if (m.ev_solved[k]) (void)hipEventDestroy(m.ev_solved[k]);
    if (m.ev_gs[k]) (void)hipEventDestroy(m.ev_gs[k]);
    if (m.ev_ge[k]) (void)hipEventDestroy(m.ev_ge[k]);
  }
  if (m.ev_done) (void)hipEventDestroy(m.ev_done);
  if (m.ev_end) (void)hipEventDestroy(m.ev_end);
  if (m.cs) (void)hipStreamDestroy(m.cs);
  const int keep_chunks = m.chunks_req;
  const double keep_t = m.timeout_s;
  m = IkComm();
  m.chunks_req = keep_chunks;
  m.timeout_s = keep_t;
  c->last_sharded = false;
  return true;
}

}  // namespace ikapi

namespace {

// The first collective of a new communicator: one all-gather of a 64-byte
// record per rank, waited for with the deadline.  It checks the communicator
// end to end before any solve relies on it, and that the ranks agree on what
// their plans depend on (rank numbering, size, IKHIP_GATHER_CHUNKS, library).
struct Hello {
  uint32_t magic;
  int32_t rank, nranks, env_chunks;
  char version[48];
};
static_assert(sizeof(Hello) == 64, "Hello is one 64-byte slot");

int comm_hello(ik_ctx *c, Rccl *r) {
  IkComm &m = c->comm;
  const int g = m.nranks;
  int rc = ensure_comm_state(c, sizeof(Hello) * (size_t)g);
  if (rc) return rc;
  char *dev = static_cast<char *>(m.stage);
  Hello *h = reinterpret_cast<Hello *>(m.h_tails);  // pinned, >= g slots of 64 B
  Hello me;
  std::memset(&me, 0, sizeof(me));
  me.magic = kPlanMagic;
  me.rank = m.rank;
  me.nranks = g;
  me.env_chunks = env_chunks();
  std::snprintf(me.version, sizeof(me.version), "%s", ik_version());
  h[m.rank] = me;
  IK_HIP(hipMemcpyAsync(dev + (size_t)m.rank * sizeof(Hello), &h[m.rank], sizeof(Hello),
                        hipMemcpyHostToDevice, m.cs));
  int res = r->all_gather(dev + (size_t)m.rank * sizeof(Hello), dev, sizeof(Hello), kNcclUint8,
                          m.comm, m.cs);
  if (res == kNcclInProgress) res = rccl_settle(r, m.comm, comm_timeout(m));
  if (res < 0) return comm_abort(c, nullptr, rank_tag(m) + ": the first all-gather did not settle");
  if (res) {
    rccl_fail(r, "ncclAllGather (first)", res);
    return comm_abort(c, nullptr, rank_tag(m) + ": " + ik_last_error());
  }
  IK_HIP(hipMemcpyAsync(h, dev, sizeof(Hello) * (size_t)g, hipMemcpyDeviceToHost, m.cs));
  IK_HIP(hipEventRecord(m.ev_end, m.cs));
  m.ev_end_set = true;
  if ((rc = comm_wait(c, m.ev_end, "the communicator's first all-gather"))) return rc;
  for (int q = 0; q < g; ++q) {
    const Hello &o = h[q];
    std::string bad;
    if (o.magic != kPlanMagic || o.rank != q || o.nranks != g)
      bad = "slot " + std::to_string(q) + " holds rank " + std::to_string(o.rank) + " of " +
            std::to_string(o.nranks);
    else if (o.env_chunks != me.env_chunks)
      bad = "rank " + std::to_string(q) + " has IKHIP_GATHER_CHUNKS " +
            std::to_string(o.env_chunks) + ", this rank " + std::to_string(me.env_chunks);
    else if (std::strncmp(o.version, me.version, sizeof(me.version)) != 0)
      bad = "rank " + std::to_string(q) + " runs " + std::string(o.version, strnlen(o.version, 47));
    if (!bad.empty())
      return comm_abort(c, nullptr, rank_tag(m) + ": ranks disagree: " + bad +
                                        "; communicator aborted");
  }
  return IK_OK;
}

}  // namespace

extern "C" {

int ik_comm_unique_id(uint8_t *id) {
  if (!id) return fail(IK_E_BADARG, "ik_comm_unique_id: id is NULL");
  Rccl *r = nullptr;
  int rc = load_rccl(&r);
  if (rc) return rc;
  IdBlob b;
  const int res = r->get_unique_id(&b);
  if (res != 0) return rccl_fail(r, "ncclGetUniqueId", res);
  std::memcpy(id, b.b, IK_COMM_ID_BYTES);
  return IK_OK;
}

int ik_comm_init(ik_ctx *c, int nranks, int rank, const uint8_t *id) {
  if (!c || !id || nranks < 1 || nranks > 1024 || rank < 0 || rank >= nranks)
    return fail(IK_E_BADARG, "ik_comm_init: bad args");
  int rc = set_dev(c);
  if (rc) return rc;
  Rccl *r = nullptr;
  if ((rc = load_rccl(&r))) return rc;
  if (!comm_release(c)) return fail(IK_E_RCCL, "ik_comm_init: the aborted communicator's work "
                                               "has not drained");
  (void)hipStreamSynchronize(c->stream);
  IdBlob b;
  std::memcpy(b.b, id, IK_COMM_ID_BYTES);
  void *comm = nullptr;
  c->comm.nranks = nranks;
  c->comm.rank = rank;
  const double T = comm_timeout(c->comm);
  if (r->nonblocking()) {
    // non-blocking: ncclCommInitRankConfig returns at once and the rendezvous
    // with the other ranks is polled against the deadline
    NcclConfig cfg;
    int res = r->comm_init_rank_config(&comm, nranks, b, rank, &cfg);
    if (res != 0 && res != kNcclInProgress) return rccl_fail(r, "ncclCommInitRankConfig", res);
    res = rccl_settle(r, comm, T);
    if (res != 0) {
      if (comm) (void)r->comm_abort(comm);
      if (res < 0)
        return fail(IK_E_RCCL, rank_tag(c->comm) + ": ncclCommInitRankConfig did not complete "
                                                   "within " + secs_str(T) +
                                   " s (IKHIP_RCCL_TIMEOUT_S): a rank missing or another "
                                   "unique id?");
      return rccl_fail(r, "ncclCommInitRankConfig", res);
    }
  } else {  // an RCCL without the non-blocking API: a blocking init
    const int res = r->comm_init_rank(&comm, nranks, b, rank);
    if (res != 0) return rccl_fail(r, "ncclCommInitRank", res);
  }
  c->comm.comm = comm;
  return comm_hello(c, r);
}

int ik_comm_init_loopback(ik_ctx *c, int nranks, int rank) {
  if (!c || nranks < 1 || nranks > 1024 || rank < 0 || rank >= nranks)
    return fail(IK_E_BADARG, "ik_comm_init_loopback: bad args");
  int rc = set_dev(c);
  if (rc) return rc;
  if (!comm_release(c)) return fail(IK_E_RCCL, "ik_comm_init_loopback: the aborted "
                                               "communicator's work has not drained");
  (void)hipStreamSynchronize(c->stream);
  c->comm.comm = &c->comm;  // a sentinel: never passed to RCCL
  c->comm.loopback = true;
  c->comm.nranks = nranks;
  c->comm.rank = rank;
  return IK_OK;
}

int ik_comm_loopback_stall(ik_ctx *c, int on) {
  if (!c || !c->comm.comm || !c->comm.loopback)
    return fail(IK_E_BADARG, "ik_comm_loopback_stall: needs a loopback communicator");
  IkComm &m = c->comm;
  if (!m.stall_flag)
    IK_HIP(hipHostMalloc(reinterpret_cast<void **>(&m.stall_flag), sizeof(int),
                         hipHostMallocCoherent | hipHostMallocMapped));
  __atomic_store_n(m.stall_flag, 0, __ATOMIC_SEQ_CST);
  m.stall = on != 0;
  return IK_OK;
}

int ik_comm_set_timeout(ik_ctx *c, double seconds) {
  if (!c || !(seconds >= 0.0)) return fail(IK_E_BADARG, "ik_comm_set_timeout: bad args");
  c->comm.timeout_s = seconds;
  return IK_OK;
}

int ik_loopback_byte(int slot, int64_t offset) { return loopback_byte(slot, (uint64_t)offset); }

int ik_comm_destroy(ik_ctx *c) {
  if (!c) return fail(IK_E_BADARG, "ik_comm_destroy: NULL context");
  int rc = set_dev(c);
  if (rc) return rc;
  if (!comm_release(c))
    return fail(IK_E_RCCL, "ik_comm_destroy: the aborted communicator's work has not drained "
                           "(its buffers are left to the process's end)");
  (void)hipStreamSynchronize(c->stream);
  return IK_OK;
}

int ik_comm_info(ik_ctx *c, int *nranks, int *rank, int *last_chunks) {
  if (!c) return fail(IK_E_BADARG, "ik_comm_info: NULL context");
  if (nranks) *nranks = c->comm.comm ? c->comm.nranks : 0;
  if (rank) *rank = c->comm.comm ? c->comm.rank : -1;
  if (last_chunks) *last_chunks = c->comm.last_req;
  return IK_OK;
}

int ik_comm_set_chunks(ik_ctx *c, int chunks) {
  if (!c || chunks < 0 || chunks > IK_MAX_GATHER_CHUNKS)
    return fail(IK_E_BADARG, "ik_comm_set_chunks: chunks must be 0.." +
                                 std::to_string(IK_MAX_GATHER_CHUNKS));
  c->comm.chunks_req = chunks;
  return IK_OK;
}

int ik_shard_plan_of(int64_t n, int nranks, int chunks, ik_shard_plan *out) {
  if (!out || !plan_args_ok(n, nranks, chunks)) return fail(IK_E_BADARG, "ik_shard_plan_of: bad args");
  make_plan(n, nranks, chunks, out);
  return IK_OK;
}

int ik_shard_part(const ik_shard_plan *p, int rank, int chunk, int64_t *begin, int64_t *end) {
  if (!p || !begin || !end || rank < 0 || rank >= p->nranks || chunk < 0 ||
      chunk >= IK_MAX_GATHER_CHUNKS)
    return fail(IK_E_BADARG, "ik_shard_part: bad args");
  part_of(*p, rank, chunk, begin, end);
  return IK_OK;
}

int ik_shard_range(int64_t n, int nranks, int rank, int64_t *begin, int64_t *end) {
  if (!plan_args_ok(n, nranks, 1) || rank < 0 || rank >= nranks || !begin || !end)
    return fail(IK_E_BADARG, "ik_shard_range: bad args");
  ik_shard_plan p;
  make_plan(n, nranks, 1, &p);
  part_of(p, rank, 0, begin, end);
  return IK_OK;
}

// Rank order, as one process would meet the points: the lowest global failing
// index wins, sums add up, FK-error max over ranks.
int ik_tail_reduce(const ik_shard_tail *t, int nranks, ik_stats *s) {
  if (!t || !s || nranks < 1) return fail(IK_E_BADARG, "ik_tail_reduce: bad args");
  std::memset(s, 0, sizeof(*s));
  s->first_oob = -1;
  s->first_err = -1;
  s->first_err_code = IK_OK;
  for (int r = 0; r < nranks; ++r) {
    if (t[r].first_oob >= 0 && (s->first_oob < 0 || t[r].first_oob < s->first_oob))
      s->first_oob = t[r].first_oob;
    if (t[r].first_err >= 0 && (s->first_err < 0 || t[r].first_err < s->first_err)) {
      s->first_err = t[r].first_err;
      s->first_err_code = t[r].first_err_code;
    }
    s->max_iters = t[r].max_iters > s->max_iters ? t[r].max_iters : s->max_iters;
    s->sum_iters += t[r].sum_iters;
    s->n_capped += t[r].n_capped;
    s->max_fk_err = t[r].max_fk_err > s->max_fk_err ? t[r].max_fk_err : s->max_fk_err;
    s->sum_fk_err += t[r].sum_fk_err;
  }
  return IK_OK;
}

int ik_fkhist_bin(double e) { return fkhist_bin(e); }

double ik_fkhist_upper(int bin) {
  if (bin < 0 || bin >= IK_FKHIST_BINS - 1) return bin < 0 ? 0.0 : HUGE_VAL;
  return std::ldexp(1.0 + (double)(bin % 16 + 1) / 16.0, bin / 16 - 64);
}

int ik_fk_err_quantile(ik_ctx *c, double q, double *out) {
  if (!c || !out || !(q > 0.0 && q <= 1.0)) return fail(IK_E_BADARG, "ik_fk_err_quantile: bad args");
  if (!c->last_sharded || !c->comm.last_hist)
    return fail(IK_E_BADARG, "ik_fk_err_quantile: the last call was not a sharded solve with fk_err");
  int rc = set_dev(c);
  if (rc) return rc;
  if ((rc = comm_wait(c, c->comm.ev_end, "the last sharded call"))) return rc;
  const IkComm &m = c->comm;
  uint64_t tot = 0;
  for (int r = 0; r < m.nranks; ++r)
    for (int b = 0; b < IK_FKHIST_BINS; ++b) tot += m.h_tails[r].hist[b];
  *out = NAN;
  if (tot == 0) return IK_OK;
  const uint64_t want = (uint64_t)std::ceil(q * (double)tot);
  uint64_t cum = 0;
  for (int b = 0; b < IK_FKHIST_BINS; ++b) {
    for (int r = 0; r < m.nranks; ++r) cum += m.h_tails[r].hist[b];
    if (cum >= (want ? want : 1)) {
      *out = ik_fkhist_upper(b);
      break;
    }
  }
  return IK_OK;
}

static int sharded_common(ik_ctx *c, int flags, const char *who) {
  if (!c) return fail(IK_E_BADARG, std::string(who) + ": NULL context");
  if (!c->comm.comm) return fail(IK_E_BADARG, std::string(who) + ": no communicator (ik_comm_init)");
  if ((flags & IK_F_ASYNC) && !(flags & IK_F_DEVICE))
    return fail(IK_E_BADARG, "IK_F_ASYNC requires IK_F_DEVICE");
  return set_dev(c);
}

// Host pointers: device scratch holds the points (the rank's parts, at their
// global rows), the gathered outputs (n rows each) and the FK errors.
struct HostStage {
  char *pts, *out[2], *fk;
};

static int host_stage(ik_ctx *c, const ik_shard_plan &P, int64_t n, const int *rb, int nreg,
                      bool fk, size_t extra, HostStage *h, char **extra_at) {
  const size_t b_pts = Stage::up((size_t)n * 24);
  size_t b_out[2] = {0, 0};
  for (int q = 0; q < nreg; ++q) b_out[q] = Stage::up((size_t)n * rb[q]);
  const size_t b_fk = fk ? Stage::up((size_t)n * 8) : 0;
  int rc = ensure_scratch(c, extra + b_pts + b_out[0] + b_out[1] + b_fk);
  if (rc) return rc;
  char *s = static_cast<char *>(c->scratch);
  *extra_at = s;
  s += extra;
  h->pts = s;
  s += b_pts;
  for (int q = 0; q < 2; ++q) {
    h->out[q] = q < nreg ? s : nullptr;
    s += b_out[q];
  }
  h->fk = fk ? s : nullptr;
  (void)P;
  return IK_OK;
}

// The rank's parts of the points, host -> scratch at their global rows.
static int host_points_in(ik_ctx *c, const ik_shard_plan &P, const double *pts, char *dst) {
  for (int k = 0; k < P.chunks; ++k) {
    int64_t b, e;
    part_of(P, c->comm.rank, k, &b, &e);
    if (e > b)
      IK_HIP(hipMemcpyAsync(dst + b * 24, pts + 3 * b, (size_t)(e - b) * 24,
                            hipMemcpyHostToDevice, c->stream));
  }
  return IK_OK;
}

// After the call: the gathered rows (all n) and this rank's FK errors to the host.
static int host_results_out(ik_ctx *c, const ik_shard_plan &P, const Region *R, int nreg,
                            char *const *host_out, const char *dfk, double *hfk) {
  for (int q = 0; q < nreg; ++q)
    if (host_out[q] && P.n > 0)
      IK_HIP(hipMemcpyAsync(host_out[q], R[q].out, (size_t)P.n * R[q].rb, hipMemcpyDeviceToHost,
                            c->stream));
  if (hfk)
    for (int k = 0; k < P.chunks; ++k) {
      int64_t b, e;
      part_of(P, c->comm.rank, k, &b, &e);
      if (e > b)
        IK_HIP(hipMemcpyAsync(hfk + b, dfk + b * 8, (size_t)(e - b) * 8, hipMemcpyDeviceToHost,
                              c->stream));
    }
  return IK_OK;
}

int ik_ann_solve_sharded(ik_ctx *c, const double *pts, int64_t n, float *ang, double *fk_err,
                         int flags, ik_stats *stats) {
  int rc = sharded_common(c, flags, "ik_ann_solve_sharded");
  if (rc) return rc;
  if (n < 0 || n >= ((int64_t)1 << 48) || (n > 0 && (!pts || !ang)))
    return fail(IK_E_BADARG, "ik_ann_solve_sharded: bad args");
  if ((flags & IK_F_DEVICE) && (reinterpret_cast<uintptr_t>(ang) & 15))
    return fail(IK_E_BADARG, "ik_ann_solve_sharded: device ang must be 16-byte aligned");
  if (!c->ann_loaded) return fail(IK_E_NOMODEL, "ik_ann_solve_sharded: no model loaded");
  KtScope kts(c);
  const bool dev = flags & IK_F_DEVICE;
  const int g = c->comm.nranks;
  ik_shard_plan P;
  if (c->comm.broken)
    return fail(IK_E_RCCL, "ik_ann_solve_sharded: communicator aborted earlier (" +
                               c->comm.why + ")");
  c->comm.last_req = auto_chunks(c, IK_METHOD_ANN, n);
  make_plan(n, g, c->comm.last_req, &P);
  const size_t stage = Stage::up((size_t)P.part_rows * g * 16);
  if ((rc = ensure_comm_state(c, stage))) return rc;
  Region R[1] = {{16, reinterpret_cast<char *>(ang), static_cast<char *>(c->comm.stage)}};
  const double *dp = pts;
  double *dfk = fk_err;
  HostStage hs;
  if (!dev) {
    // pageable host copies wait for the stream: the previous call's end first
    if (c->comm.ev_end_set && (rc = comm_wait(c, c->comm.ev_end, "the previous sharded call")))
      return rc;
    const int rb[1] = {16};
    char *unused = nullptr;
    if ((rc = host_stage(c, P, n, rb, 1, fk_err != nullptr, 0, &hs, &unused))) return rc;
    if ((rc = host_points_in(c, P, pts, hs.pts))) return rc;
    dp = reinterpret_cast<const double *>(hs.pts);
    R[0].out = hs.out[0];
    dfk = reinterpret_cast<double *>(hs.fk);
  }
  const bool limits = !(flags & IK_F_NO_LIMITS);
  rc = sharded_run(c, IK_METHOD_ANN, P, R, 1, dfk, [&](const PartJob &j) {
    return ann_launch(c, dp + 3 * j.b, j.m, reinterpret_cast<float *>(j.at[0]), j.fk_err, limits,
                      j.S);
  });
  if (rc) return rc;
  if (!dev) {
    // copies into pageable host memory block the thread until the stream
    // reaches them: first the bounded wait for the gathers
    if ((rc = comm_wait(c, c->comm.ev_end, "the sharded call"))) return rc;
    char *ho[1] = {reinterpret_cast<char *>(ang)};
    if ((rc = host_results_out(c, P, R, 1, ho, hs.fk, fk_err))) return rc;
  }
  if (flags & IK_F_ASYNC) return IK_OK;
  return sharded_stats(c, stats);
}

int ik_fabrik_solve_sharded(ik_ctx *c, const double *pts, int64_t n, double tol,
                            int32_t max_iter, double *ang, int32_t *iters, double *fk_err,
                            int flags, ik_stats *stats) {
  int rc = sharded_common(c, flags, "ik_fabrik_solve_sharded");
  if (rc) return rc;
  if (n < 0 || n >= ((int64_t)1 << 48) || (n > 0 && (!pts || !ang)) || max_iter < 0)
    return fail(IK_E_BADARG, "ik_fabrik_solve_sharded: bad args");
  if ((flags & IK_F_DEVICE) && (reinterpret_cast<uintptr_t>(ang) & 15))
    return fail(IK_E_BADARG, "ik_fabrik_solve_sharded: device ang must be 16-byte aligned");
  KtScope kts(c);
  const bool dev = flags & IK_F_DEVICE;
  const int g = c->comm.nranks;
  ik_shard_plan P;
  if (c->comm.broken)
    return fail(IK_E_RCCL, "ik_fabrik_solve_sharded: communicator aborted earlier (" +
                               c->comm.why + ")");
  c->comm.last_req = auto_chunks(c, IK_METHOD_FABRIK, n);
  make_plan(n, g, c->comm.last_req, &P);
  const int nreg = iters ? 2 : 1;
  const size_t b_ang_st = Stage::up((size_t)P.part_rows * g * 32);
  const size_t stage = b_ang_st + (iters ? Stage::up((size_t)P.part_rows * g * 4) : 0);
  if ((rc = ensure_comm_state(c, stage))) return rc;
  char *st = static_cast<char *>(c->comm.stage);
  Region R[2] = {{32, reinterpret_cast<char *>(ang), st},
                 {4, reinterpret_cast<char *>(iters), st + b_ang_st}};
  const size_t b_work = Stage::up(fabrik_scratch_bytes(P.part_rows));
  const double *dp = pts;
  double *dfk = fk_err;
  char *work = nullptr;
  HostStage hs;
  if (!dev) {
    if (c->comm.ev_end_set && (rc = comm_wait(c, c->comm.ev_end, "the previous sharded call")))
      return rc;
    const int rb[2] = {32, 4};
    if ((rc = host_stage(c, P, n, rb, nreg, fk_err != nullptr, b_work, &hs, &work))) return rc;
    if ((rc = host_points_in(c, P, pts, hs.pts))) return rc;
    dp = reinterpret_cast<const double *>(hs.pts);
    R[0].out = hs.out[0];
    if (iters) R[1].out = hs.out[1];
    dfk = reinterpret_cast<double *>(hs.fk);
  } else {
    if ((rc = ensure_scratch(c, b_work))) return rc;
    work = static_cast<char *>(c->scratch);
  }
  const bool limits = !(flags & IK_F_NO_LIMITS);
  rc = sharded_run(c, IK_METHOD_FABRIK, P, R, nreg, dfk, [&](const PartJob &j) {
    return fabrik_launch(c, dp + 3 * j.b, j.m, tol, max_iter, reinterpret_cast<double *>(j.at[0]),
                         iters ? reinterpret_cast<int32_t *>(j.at[1]) : nullptr, nullptr,
                         j.fk_err, limits, work, j.S);
  });
  if (rc) return rc;
  if (!dev) {
    if ((rc = comm_wait(c, c->comm.ev_end, "the sharded call"))) return rc;
    char *ho[2] = {reinterpret_cast<char *>(ang), reinterpret_cast<char *>(iters)};
    if ((rc = host_results_out(c, P, R, nreg, ho, hs.fk, fk_err))) return rc;
  }
  if (flags & IK_F_ASYNC) return IK_OK;
  return sharded_stats(c, stats);
}

}  // extern "C"
