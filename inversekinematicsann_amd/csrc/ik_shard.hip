// ik_shard.hip -- the batch sharded over GPUs with one RCCL all-gather
// (include/ikhip.h "multi-GPU").
//
// The reference scales by competing consumers (rpc_broker.py:55-68): each worker
// takes whole requests.  Here the points of one batch are independent, so the
// batch is split contiguously over the ranks (one process per GPU), every rank
// solves its rows into one block of a send buffer -- the rows of each output,
// then a 64-byte tail with its stats -- and ONE ncclAllGather over xGMI hands
// every rank every block.  The rows go to the caller's arrays in point order
// (one unpack kernel, or per-rank D2H copies for host arrays) and the stats are
// reduced on the host from the gathered tails, so no all_reduce is needed: the
// lowest global failing index, iteration sums and FK-error max/sum all come from
// the same collective.
//
// RCCL is loaded at run time (dlopen): the process's own librccl when one is
// already loaded (torch ships one, built against the HIP runtime the process
// uses), else librccl.so.1 from the ROCm install.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

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
typedef int (*CommInitRankBlobFn)(void **comm, int nranks, IdBlob id, int rank);
typedef int (*CommDestroyFn)(void *comm);
typedef int (*AllGatherFn)(const void *send, void *recv, size_t count, int dtype, void *comm,
                           hipStream_t stream);
typedef const char *(*GetErrorStringFn)(int);
constexpr int kNcclUint8 = 1;  // ncclDataType_t ncclUint8

struct Rccl {
  void *lib = nullptr;
  GetUniqueIdFn get_unique_id = nullptr;
  CommInitRankBlobFn comm_init_rank = nullptr;
  CommDestroyFn comm_destroy = nullptr;
  AllGatherFn all_gather = nullptr;
  GetErrorStringFn error_string = nullptr;
  std::string where;
};

std::mutex g_rccl_mu;
Rccl g_rccl;

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
      for (const char *nm : {"librccl.so", "librccl.so.1"}) {
        h = dlopen(nm, RTLD_NOW | RTLD_NOLOAD);
        if (h) {
          where = std::string(nm) + " (already loaded)";
          break;
        }
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
    r.comm_destroy = reinterpret_cast<CommDestroyFn>(dlsym(h, "ncclCommDestroy"));
    r.all_gather = reinterpret_cast<AllGatherFn>(dlsym(h, "ncclAllGather"));
    r.error_string = reinterpret_cast<GetErrorStringFn>(dlsym(h, "ncclGetErrorString"));
    if (!r.get_unique_id || !r.comm_init_rank || !r.comm_destroy || !r.all_gather)
      return fail(IK_E_RCCL, "RCCL at " + where + " lacks ncclGetUniqueId / ncclCommInitRank / "
                                                  "ncclCommDestroy / ncclAllGather");
    g_rccl = r;
  }
  *out = &g_rccl;
  return IK_OK;
}

int rccl_fail(const Rccl *r, const char *what, int res) {
  const char *msg = (r && r->error_string) ? r->error_string(res) : "?";
  return fail(IK_E_RCCL, std::string(what) + ": " + msg + " (" + std::to_string(res) + ")");
}

// floor(r n / g); exact in 64 bits for n g < 2^63 (ik_shard_range checks n < 2^48)
int64_t shard_begin(int64_t n, int g, int r) { return n * r / g; }

int64_t up64(int64_t b) { return (b + 63) & ~(int64_t)63; }

}  // namespace

namespace ikhip {

// The tail of this rank: the shard's DevStats reduced, indices made global.
__global__ void pack_tail_kernel(const DevStats *S, int64_t begin, int64_t rows,
                                 ik_shard_tail *t) {
  __shared__ unsigned long long s_it[kStatShards], s_cap[kStatShards], s_mx[kStatShards];
  __shared__ double s_sum[kStatShards];
  __shared__ int s_mi[kStatShards];
  const int i = threadIdx.x;
  if (i < kStatShards) {
    s_it[i] = S->sum_iters[i];
    s_cap[i] = S->n_capped[i];
    s_mx[i] = S->max_fk_err_bits[i];
    s_sum[i] = S->sum_fk_err[i];
    s_mi[i] = S->max_iters[i];
  }
  __syncthreads();
  if (i != 0) return;
  ik_shard_tail o;
  o.first_oob = S->first_oob == ~0ull ? -1 : (int64_t)S->first_oob + begin;
  if (S->first_err_key == ~0ull) {
    o.first_err = -1;
    o.first_err_code = IK_OK;
  } else {
    o.first_err = (int64_t)(S->first_err_key >> 8) + begin;
    o.first_err_code = (int32_t)(S->first_err_key & 0xff);
  }
  o.max_iters = 0;
  o.sum_iters = 0;
  o.n_capped = 0;
  o.max_fk_err = 0.0;
  o.sum_fk_err = 0.0;
  for (int k = 0; k < kStatShards; ++k) {  // the shard order of stats_from_dev
    o.max_iters = s_mi[k] > o.max_iters ? s_mi[k] : o.max_iters;
    o.sum_iters += (int64_t)s_it[k];
    o.n_capped += (int64_t)s_cap[k];
    const double mx = __longlong_as_double((long long)s_mx[k]);
    o.max_fk_err = mx > o.max_fk_err ? mx : o.max_fk_err;
    o.sum_fk_err += s_sum[k];
  }
  o.rows = rows;
  *t = o;
}

// Gathered blocks -> the caller's arrays in point order: row i belongs to rank
// r = ceil((i + 1) g / n) - 1 (the r with floor(r n / g) <= i < floor((r + 1) n / g)).
struct Unpack {
  const char *recv;
  int64_t block, n;
  int g, nreg;
  int64_t off[3];
  int words[3];  // 4-byte words per row of each region
  char *dst[3];
};

__global__ __launch_bounds__(256) void gather_unpack_kernel(Unpack u) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < u.n; i += stride) {
    const int r = (int)(((i + 1) * u.g + u.n - 1) / u.n) - 1;
    const int64_t local = i - u.n * r / u.g;
    const char *blk = u.recv + (int64_t)r * u.block;
    for (int q = 0; q < u.nreg; ++q) {
      const uint32_t *s =
          reinterpret_cast<const uint32_t *>(blk + u.off[q]) + local * u.words[q];
      uint32_t *d = reinterpret_cast<uint32_t *>(u.dst[q]) + i * u.words[q];
      if (u.words[q] == 4) {
        *reinterpret_cast<uint4 *>(d) = *reinterpret_cast<const uint4 *>(s);
      } else if (u.words[q] == 8) {
        reinterpret_cast<uint4 *>(d)[0] = reinterpret_cast<const uint4 *>(s)[0];
        reinterpret_cast<uint4 *>(d)[1] = reinterpret_cast<const uint4 *>(s)[1];
      } else {
        for (int w = 0; w < u.words[q]; ++w) d[w] = s[w];
      }
    }
  }
}

}  // namespace ikhip

namespace {

// Bytes of the regions: angles first (16-byte aligned rows for the kernels'
// 16-byte stores), then iterations / FK errors, each region 64-byte aligned.
void layout(int method, int64_t n, int g, bool with_iters, bool with_fk, ik_gather_layout *L) {
  std::memset(L, 0, sizeof(*L));
  const int64_t S = g > 0 ? (n + g - 1) / g : 0;  // >= the largest floor-split shard
  L->shard = S;
  int k = 0;
  int64_t off = 0;
  auto add = [&](int rb) {
    L->row_bytes[k] = rb;
    L->offset[k] = off;
    off = up64(off + S * rb);
    ++k;
  };
  add(method == IK_METHOD_ANN ? 16 : 32);
  if (with_iters) add(4);
  if (with_fk) add(8);
  L->nregion = k;
  L->tail_offset = off;
  L->block_bytes = up64(off + (int64_t)sizeof(ik_shard_tail));
}

int ensure_comm_buffers(ik_ctx *c, size_t send, size_t recv) {
  IkComm &m = c->comm;
  if (send > m.send_bytes || recv > m.recv_bytes || m.h_tails_n < m.nranks) {
    IK_HIP(hipStreamSynchronize(c->stream));
  }
  if (send > m.send_bytes) {
    if (m.send) IK_HIP(hipFree(m.send));
    m.send = nullptr;
    m.send_bytes = 0;
    IK_HIP(hipMalloc(&m.send, send));
    m.send_bytes = send;
  }
  if (recv > m.recv_bytes) {
    if (m.recv) IK_HIP(hipFree(m.recv));
    m.recv = nullptr;
    m.recv_bytes = 0;
    IK_HIP(hipMalloc(&m.recv, recv));
    m.recv_bytes = recv;
  }
  if (m.h_tails_n < m.nranks) {
    if (m.h_tails) IK_HIP(hipHostFree(m.h_tails));
    m.h_tails = nullptr;
    IK_HIP(hipHostMalloc(reinterpret_cast<void **>(&m.h_tails),
                         sizeof(ik_shard_tail) * (size_t)m.nranks, hipHostMallocDefault));
    m.h_tails_n = m.nranks;
  }
  if (!m.g0) IK_HIP(hipEventCreate(&m.g0));
  if (!m.g1) IK_HIP(hipEventCreate(&m.g1));
  return IK_OK;
}

// After the solve wrote this rank's rows into its send block: the tail, the
// all-gather, the rows to the caller's arrays, the tails to the host.
int gather_and_unpack(ik_ctx *c, const ik_gather_layout &L, int64_t n, int64_t begin,
                      int64_t rows, char *const dst[3], bool dev) {
  IkComm &m = c->comm;
  Rccl *r = nullptr;
  int rc = load_rccl(&r);
  if (rc) return rc;
  char *send = static_cast<char *>(m.send);
  char *recv = static_cast<char *>(m.recv);
  hipLaunchKernelGGL(pack_tail_kernel, dim3(1), dim3(64), 0, c->stream, c->d_stats, begin, rows,
                     reinterpret_cast<ik_shard_tail *>(send + L.tail_offset));
  IK_HIP(hipGetLastError());
  kt_begin("rccl_all_gather", c->stream);
  IK_HIP(hipEventRecord(m.g0, c->stream));
  const int res = r->all_gather(send, recv, (size_t)L.block_bytes, kNcclUint8, m.comm, c->stream);
  if (res != 0) return rccl_fail(r, "ncclAllGather", res);
  IK_HIP(hipEventRecord(m.g1, c->stream));
  kt_end(c->stream);
  if (dev) {
    Unpack u;
    std::memset(&u, 0, sizeof(u));
    u.recv = recv;
    u.block = L.block_bytes;
    u.n = n;
    u.g = m.nranks;
    u.nreg = 0;
    for (int q = 0; q < L.nregion; ++q) {
      if (!dst[q]) continue;
      u.off[u.nreg] = L.offset[q];
      u.words[u.nreg] = L.row_bytes[q] / 4;
      u.dst[u.nreg] = dst[q];
      ++u.nreg;
    }
    if (u.nreg && n > 0) {
      int cus = 256, dv = 0;
      (void)hipGetDevice(&dv);
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dv);
      const int64_t want = (n + 255) / 256, cap = (int64_t)(cus > 0 ? cus : 256) * 8;
      kt_begin("gather_unpack_kernel", c->stream);
      hipLaunchKernelGGL(gather_unpack_kernel, dim3((unsigned)(want < cap ? want : cap)),
                         dim3(256), 0, c->stream, u);
      kt_end(c->stream);
      IK_HIP(hipGetLastError());
    }
  } else {
    for (int rr = 0; rr < m.nranks; ++rr) {
      const int64_t b = shard_begin(n, m.nranks, rr), e = shard_begin(n, m.nranks, rr + 1);
      if (e <= b) continue;
      for (int q = 0; q < L.nregion; ++q) {
        if (!dst[q]) continue;
        IK_HIP(hipMemcpyAsync(dst[q] + b * L.row_bytes[q],
                              recv + (int64_t)rr * L.block_bytes + L.offset[q],
                              (size_t)(e - b) * L.row_bytes[q], hipMemcpyDeviceToHost,
                              c->stream));
      }
    }
  }
  // every rank's tail to the host (the stats; read by sharded_stats)
  IK_HIP(hipMemcpy2DAsync(m.h_tails, sizeof(ik_shard_tail), recv + L.tail_offset,
                          (size_t)L.block_bytes, sizeof(ik_shard_tail), (size_t)m.nranks,
                          hipMemcpyDeviceToHost, c->stream));
  c->last_sharded = true;
  c->last_n = n;
  return IK_OK;
}

}  // namespace

namespace ikapi {

int sharded_stats(ik_ctx *c, ik_stats *stats) {
  IK_HIP(hipStreamSynchronize(c->stream));
  if (!stats) return IK_OK;
  int rc = ik_tail_reduce(c->comm.h_tails, c->comm.nranks, stats);
  if (rc) return rc;
  float ms = 0.0f;
  if (hipEventElapsedTime(&ms, c->comm.g0, c->comm.g1) == hipSuccess) stats->gather_ms = ms;
  return IK_OK;
}

void comm_release(ik_ctx *c) {
  IkComm &m = c->comm;
  if (m.comm) {
    Rccl *r = nullptr;
    if (load_rccl(&r) == IK_OK) (void)r->comm_destroy(m.comm);
  }
  if (m.send) (void)hipFree(m.send);
  if (m.recv) (void)hipFree(m.recv);
  if (m.h_tails) (void)hipHostFree(m.h_tails);
  if (m.g0) (void)hipEventDestroy(m.g0);
  if (m.g1) (void)hipEventDestroy(m.g1);
  m = IkComm();
  c->last_sharded = false;
}

}  // namespace ikapi

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
  if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks)
    return fail(IK_E_BADARG, "ik_comm_init: bad args");
  int rc = set_dev(c);
  if (rc) return rc;
  Rccl *r = nullptr;
  if ((rc = load_rccl(&r))) return rc;
  comm_release(c);
  IdBlob b;
  std::memcpy(b.b, id, IK_COMM_ID_BYTES);
  void *comm = nullptr;
  const int res = r->comm_init_rank(&comm, nranks, b, rank);
  if (res != 0) return rccl_fail(r, "ncclCommInitRank", res);
  c->comm.comm = comm;
  c->comm.nranks = nranks;
  c->comm.rank = rank;
  return IK_OK;
}

int ik_comm_destroy(ik_ctx *c) {
  if (!c) return fail(IK_E_BADARG, "ik_comm_destroy: NULL context");
  int rc = set_dev(c);
  if (rc) return rc;
  (void)hipStreamSynchronize(c->stream);
  comm_release(c);
  return IK_OK;
}

int ik_shard_range(int64_t n, int nranks, int rank, int64_t *begin, int64_t *end) {
  if (n < 0 || n >= ((int64_t)1 << 48) || nranks < 1 || nranks > 1024 || rank < 0 ||
      rank >= nranks || !begin || !end)
    return fail(IK_E_BADARG, "ik_shard_range: bad args");
  *begin = shard_begin(n, nranks, rank);
  *end = shard_begin(n, nranks, rank + 1);
  return IK_OK;
}

int ik_gather_layout_of(int method, int64_t n, int nranks, int with_iters, int with_fk_err,
                        ik_gather_layout *out) {
  if (!out || n < 0 || n >= ((int64_t)1 << 48) || nranks < 1 || nranks > 1024 || (method != IK_METHOD_ANN && method != IK_METHOD_FABRIK) ||
      (method == IK_METHOD_ANN && with_iters))
    return fail(IK_E_BADARG, "ik_gather_layout_of: bad args");
  layout(method, n, nranks, with_iters != 0, with_fk_err != 0, out);
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

static int sharded_common(ik_ctx *c, int flags, const char *who) {
  if (!c) return fail(IK_E_BADARG, std::string(who) + ": NULL context");
  if (!c->comm.comm) return fail(IK_E_BADARG, std::string(who) + ": no communicator (ik_comm_init)");
  if (c->comm.nranks > 1024) return fail(IK_E_BADARG, std::string(who) + ": more than 1024 ranks");
  if ((flags & IK_F_ASYNC) && !(flags & IK_F_DEVICE))
    return fail(IK_E_BADARG, "IK_F_ASYNC requires IK_F_DEVICE");
  return set_dev(c);
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
  const int g = c->comm.nranks, me = c->comm.rank;
  ik_gather_layout L;
  layout(IK_METHOD_ANN, n, g, false, fk_err != nullptr, &L);
  const int64_t b = shard_begin(n, g, me), rows = shard_begin(n, g, me + 1) - b;
  if ((rc = ensure_comm_buffers(c, (size_t)L.block_bytes, (size_t)L.block_bytes * g))) return rc;
  char *send = static_cast<char *>(c->comm.send);
  const double *dp = pts + 3 * b;
  if (!dev) {
    if ((rc = ensure_scratch(c, Stage::up((size_t)rows * 24) + 256))) return rc;
    if (rows > 0)
      IK_HIP(hipMemcpyAsync(c->scratch, dp, (size_t)rows * 24, hipMemcpyHostToDevice, c->stream));
    dp = static_cast<const double *>(c->scratch);
  }
  // this rank's rows straight into its send block
  float *da = reinterpret_cast<float *>(send + L.offset[0]);
  double *de = fk_err ? reinterpret_cast<double *>(send + L.offset[1]) : nullptr;
  if ((rc = ann_launch(c, dp, rows, da, de, !(flags & IK_F_NO_LIMITS)))) return rc;
  char *dst[3] = {reinterpret_cast<char *>(ang), reinterpret_cast<char *>(fk_err), nullptr};
  if ((rc = gather_and_unpack(c, L, n, b, rows, dst, dev))) return rc;
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
  const int g = c->comm.nranks, me = c->comm.rank;
  ik_gather_layout L;
  layout(IK_METHOD_FABRIK, n, g, iters != nullptr, fk_err != nullptr, &L);
  const int64_t b = shard_begin(n, g, me), rows = shard_begin(n, g, me + 1) - b;
  if ((rc = ensure_comm_buffers(c, (size_t)L.block_bytes, (size_t)L.block_bytes * g))) return rc;
  char *send = static_cast<char *>(c->comm.send);
  const size_t b_work = Stage::up(fabrik_scratch_bytes(rows));
  const size_t b_in = dev ? 0 : Stage::up((size_t)rows * 24);
  if ((rc = ensure_scratch(c, b_work + b_in))) return rc;
  char *s = static_cast<char *>(c->scratch);
  const double *dp = pts + 3 * b;
  if (!dev) {
    if (rows > 0)
      IK_HIP(hipMemcpyAsync(s + b_work, dp, (size_t)rows * 24, hipMemcpyHostToDevice, c->stream));
    dp = reinterpret_cast<const double *>(s + b_work);
  }
  int q = 0;
  double *da = reinterpret_cast<double *>(send + L.offset[q++]);
  int32_t *di = iters ? reinterpret_cast<int32_t *>(send + L.offset[q++]) : nullptr;
  double *dfe = fk_err ? reinterpret_cast<double *>(send + L.offset[q++]) : nullptr;
  if ((rc = fabrik_launch(c, dp, rows, tol, max_iter, da, di, nullptr, dfe,
                          !(flags & IK_F_NO_LIMITS), s)))
    return rc;
  char *dst[3] = {reinterpret_cast<char *>(ang), nullptr, nullptr};
  q = 1;
  if (iters) dst[q++] = reinterpret_cast<char *>(iters);
  if (fk_err) dst[q++] = reinterpret_cast<char *>(fk_err);
  if ((rc = gather_and_unpack(c, L, n, b, rows, dst, dev))) return rc;
  if (flags & IK_F_ASYNC) return IK_OK;
  return sharded_stats(c, stats);
}

}  // extern "C"
