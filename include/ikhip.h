/*
 * ikhip.h -- C ABI of libikhip.so, the MI355X (gfx950) batched inverse-kinematics
 * engine.  Plain pointers and sizes only; no torch or HIP types in the
 * signatures (streams are passed as void*, a hipStream_t underneath).
 *
 * Each entry point replaces one function of the reference
 * (lstar93/InverseKinematicsANN, file:line below).  The reference is pure
 * Python and has no FFI of its own; the binding a maintainer would add on the
 * reference side is a ctypes stub, shown in INTEGRATION.md.
 *
 * Pointer convention: by default every array argument is a HOST pointer and the
 * call blocks until results are back in host memory.  With IK_F_DEVICE the
 * array arguments are device pointers (e.g. torch tensors' data_ptr()) on the
 * context's device, and with IK_F_ASYNC the call only enqueues work on the
 * context's stream (stats are then read with ik_stats_fetch()).
 *
 * Error convention: every call returns an ik_status.  Per-point failures of the
 * reference (its exceptions) are NOT call failures: they are reported in
 * ik_stats (first_oob / first_err / first_err_code) so that the host can raise
 * the reference's exception for the lowest failing index, exactly as the
 * reference's sequential loop would.  Calls on one context are not re-entrant.
 */
#ifndef IKHIP_H
#define IKHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum ik_status {
  IK_OK = 0,
  IK_E_OUT_OF_REACH = 1, /* OutOfRobotReachException, kinematics/inverse.py:32 */
  IK_E_DOMAIN = 2,       /* ValueError('math domain error'), acos in inverse.py:81,92,100 */
  IK_E_ZERODIV = 3,      /* ZeroDivisionError, kinematics/point.py:40, inverse.py:81,92,100 */
  IK_E_ANGLE_RANGE = 4,  /* OutOfRobotReachException, kinematics/forward.py:23-25 */
  IK_E_BADARG = 16,      /* invalid argument (shape/size/order of calls) */
  IK_E_HIP = 17,         /* HIP runtime failure (see ik_last_error) */
  IK_E_NOMODEL = 18,     /* ik_ann_solve before ik_ann_load */
  IK_E_RCCL = 19         /* RCCL missing or a collective failed (see ik_last_error) */
} ik_status;

enum {
  IK_F_DEVICE = 1,    /* array arguments are device pointers */
  IK_F_ASYNC = 2,     /* enqueue only; requires IK_F_DEVICE */
  IK_F_NO_LIMITS = 4  /* skip the workspace check (ANN.predict has none, ann.py:70-76) */
};

enum { IK_ACT_LINEAR = 0, IK_ACT_TANH = 1, IK_ACT_RELU = 2, IK_ACT_SIGMOID = 3 };

typedef struct ik_ctx ik_ctx;

typedef struct ik_stats {
  int64_t first_oob;      /* lowest index outside the workspace limits, -1 if none */
  int64_t first_err;      /* lowest index whose solve raised, -1 if none */
  int32_t first_err_code; /* ik_status of first_err */
  int32_t max_iters;      /* FABRIK: max iterations over the batch */
  int64_t sum_iters;      /* FABRIK: total iterations */
  int64_t n_capped;       /* FABRIK: points that hit max_iter */
  double max_fk_err;      /* max |FK(theta) - p|_2 over the batch (if requested) */
  double sum_fk_err;      /* sum of |FK(theta) - p|_2 */
  double gather_ms;       /* sharded calls: the RCCL all-gather's duration (HIP events), else 0 */
} ik_stats;

/* ---- context ----------------------------------------------------------- */
/* One context per device; owns a stream, device scratch and model weights. */
int ik_ctx_create(int device, ik_ctx **out);
int ik_ctx_destroy(ik_ctx *ctx);
/* Use an external stream (e.g. torch.cuda.current_stream().cuda_stream);
 * NULL restores the context's own stream.  A context's device work is one
 * sequence whatever the streams: a call enqueued on another stream than the
 * previous call first waits (hipStreamWaitEvent) for the previous call's work,
 * so two calls never share the context's stats / work-queue words at once.
 * Host threads must still not call into one context concurrently. */
int ik_ctx_set_stream(ik_ctx *ctx, void *stream);
void *ik_ctx_get_stream(ik_ctx *ctx);
const char *ik_last_error(void); /* thread-local message of the last failure */
const char *ik_version(void);

/* ---- robot ---------------------------------------------------------------
 * robot/robot.py:38-42 SixDOFRobot: dh is the 4x4 row-major DH matrix
 * (rows thetas, d, a, alpha), links the 4 joint distances, limits
 * {x_lo, x_hi, y_lo, y_hi, z_lo, z_hi} (inclusive).  Defaults are SixDOFRobot's. */
int ik_set_robot(ik_ctx *ctx, const double *dh, const double *links, const double *limits);

/* ---- workspace check ----------------------------------------------------
 * InverseKinematics.check_limits, kinematics/inverse.py:26-35. */
int ik_check_limits(ik_ctx *ctx, const double *pts, int64_t n, int flags, ik_stats *stats);

/* ---- forward kinematics --------------------------------------------------
 * ForwardKinematics.fkine, kinematics/forward.py:73-94, batched: ang n x 4
 * (float64) -> effector xyz n x 3 and, if mats is not NULL, the four
 * cumulative transforms M_1..M_4 (n x 4 x 4 x 4, row-major; fkine's second
 * return value).  Angles outside [-2pi, 2pi] give IK_E_ANGLE_RANGE in stats. */
int ik_fk(ik_ctx *ctx, const double *ang, int64_t n, double *xyz, double *mats, int flags,
          ik_stats *stats);

/* ForwardKinematics(dh).fkine for a DH table of nj (2..1024) joints (the reference
 * takes any nj >= 3, forward.py:13-19): dh host 4 x nj row-major (thetas, d, a,
 * alpha), ang n x nj -> effector xyz n x 3 and, if mats is not NULL, the nj
 * cumulative 4 x 4 transforms (n x nj x 16; the reference's nj x nj matrices
 * are these embedded in the identity). */
int ik_fk_chain(ik_ctx *ctx, int nj, const double *dh, const double *ang, int64_t n, double *xyz,
                double *mats, int flags, ik_stats *stats);

/* ---- FABRIK ---------------------------------------------------------------
 * FabrikInverseKinematics.ikine, kinematics/inverse.py:115-139 (+ check_limits,
 * Fabrik.calculate fabrik.py:44-67, __get_angles inverse.py:54-112), batched:
 * pts n x 3 -> ang n x 4 (float64), iters n (nullable), final joint positions
 * n x 4 x 3 (nullable).  tol/max_iter: Fabrik(err_margin, max_iter_num).
 * With IK_F_DEVICE, ang must be 16-byte aligned (else IK_E_BADARG). */
int ik_fabrik_solve(ik_ctx *ctx, const double *pts, int64_t n, double tol, int32_t max_iter,
                    double *ang, int32_t *iters, double *joints, int flags, ik_stats *stats);

/* ik_fabrik_solve plus the --verbose round trip of the reference CLI
 * (cli.py:54-72, IkineCommand, the base of both --method commands): fk_err
 * (nullable) n float64 |FK(ang) - p|_2, computed in the same launch as the
 * angles; its max/sum over the finite values go to stats (max_fk_err,
 * sum_fk_err).  A point whose solve raised has fk_err NaN. */
int ik_fabrik_solve_fk(ik_ctx *ctx, const double *pts, int64_t n, double tol, int32_t max_iter,
                       double *ang, int32_t *iters, double *joints, double *fk_err, int flags,
                       ik_stats *stats);

/* Forget the context's learned FABRIK work order (the per-goal-cell cost table
 * the solves keep to start the hardest points first; DESIGN.md "Work order"):
 * the table goes back to a fresh context's -- for SixDOFRobot's chain the
 * library's built-in one (learned on random_dist batches at tol 1e-3 / 100 and
 * 1e-5 / 200; the first solve picks the one nearest its tolerance), for other
 * chains empty, i.e. point order.  Results never depend on it; only the
 * launch's tail does. */
int ik_fabrik_reset_order(ik_ctx *ctx);
/* The work-order table itself: n = 1024 cells, 1 + the largest recorded
 * iteration count per goal cell (0 = unseen).  get waits for the context's last
 * call and returns the count copied (or -ik_status); set with key NULL empties it
 * (point order). */
int ik_fabrik_order_get(ik_ctx *ctx, uint32_t *key, int n);
int ik_fabrik_order_set(ik_ctx *ctx, const uint32_t *key, int n);

/* Fabrik.calculate, kinematics/fabrik.py:44-67, batched over n goals for a chain
 * of nj (1..4096) joints: init is n x nj x 3 (or nj x 3 shared by all goals when
 * init_shared != 0), goals n x 3 -> joints n x nj x 3, iters n (nullable).
 * 2..8 joints run with the chain in registers; other lengths keep it in the
 * joints output row (same arithmetic, same bits) at about nj * max_iter * 2
 * dependent steps of ~0.4 us per goal (4096 joints x 100 iterations: ~0.3 s). */
int ik_fabrik_calc(ik_ctx *ctx, int nj, const double *dists, const double *init,
                   int init_shared, const double *goals, int64_t n, double tol,
                   int32_t max_iter, double *joints, int32_t *iters, int flags,
                   ik_stats *stats);

/* ---- ANN ----------------------------------------------------------------
 * ANN.load_model, kinematics/ann.py:78-85, with the decoded model: n_layers
 * Dense layers, dims[0..n_layers] (dims[0] == 3, dims[n_layers] == 4), acts[l]
 * one of IK_ACT_*, W[l] host float32 [dims[l]][dims[l+1]] row-major (the Keras
 * kernel layout, x @ W + b), b[l] host float32 [dims[l+1]], and the two
 * StandardScalers (ann.py:83-84).  Up to 4096 layers of widths up to 16384.
 * Up to 24 layers of widths up to 1024 run the fused kernel (one launch, the
 * activations in LDS); models wider than 512 there run its fp32 build whatever
 * ik_ann_set_mode says.  Deeper or wider models run layer at a time with the
 * activations in HBM (fp32 MFMA, one launch per layer and chunk of points,
 * still one ik_ann_solve call; ik_ann_set_mode does not apply), in chunks whose
 * two activation buffers fit IKHIP_ANN_ACT_MB (default 1024 MiB). */
int ik_ann_load(ik_ctx *ctx, int n_layers, const int32_t *dims, const int32_t *acts,
                const float *const *W, const float *const *b, const double *x_mean,
                const double *x_scale, const double *y_mean, const double *y_scale);

/* ANN.predict, kinematics/ann.py:70-76 (+ check_limits for AnnInverseKinematics.ikine,
 * inverse.py:152-155 unless IK_F_NO_LIMITS): pts n x 3 float64 -> ang n x 4
 * float32.  fk_err (nullable) n float64: |FK(ang) - p|_2, the cli.py:54-61
 * round trip, fused into the same launch; its max/sum go to stats.  With
 * IK_F_DEVICE, ang must be 16-byte aligned (else IK_E_BADARG). */
int ik_ann_solve(ik_ctx *ctx, const double *pts, int64_t n, float *ang, double *fk_err,
                 int flags, ik_stats *stats);

/* Arithmetic of the hidden-layer GEMMs.  IK_ANN_FP32 (default): fp32 MFMA
 * (v_mfma_f32_32x32x2_f32), a fp32 dot product like the reference's TF/Keras
 * CPU float32 forward.  IK_ANN_BF16X6: every fp32 operand split into three bf16
 * parts and six bf16 MFMA products accumulated in fp32 -- fp32-level accuracy
 * (tested within 1e-6 of a float64 forward, the fp32 mode's own distance from
 * it) at ~2.7x the MFMA rate.  IK_ANN_FP16X3: two fp16 parts (weights
 * pre-scaled by a power of two) and three fp16 MFMA products, on layers whose
 * input is tanh/sigmoid-bounded (others stay fp32); as close to a float64
 * forward as numpy's float32 one on the tested networks, at ~5x the MFMA rate.
 * The input layer and a one-tile output layer stay fp32 in every mode.  Models
 * wider than 512 on the fused kernel stay fp32; models past its caps (the
 * layered path) run bf16x6 in either split mode.
 * Environment default: IKHIP_ANN_MODE=bf16x6|fp16x3. */
enum { IK_ANN_FP32 = 0, IK_ANN_BF16X6 = 1, IK_ANN_FP16X3 = 2 };
int ik_ann_set_mode(ik_ctx *ctx, int mode);
int ik_ann_get_mode(ik_ctx *ctx); /* the mode, or -ik_status */
/* The arithmetic the next ik_ann_solve runs for the loaded model (or
 * -ik_status; -IK_E_NOMODEL before ik_ann_load): the set mode, or IK_ANN_FP32
 * when no layer of the model can take it (a fused model wider than 512, or the
 * split planes left out at load because only the fp32 operands fit the
 * device), or IK_ANN_BF16X6 for IK_ANN_FP16X3 on the layered path. */
int ik_ann_effective_mode(ik_ctx *ctx);

/* Per-kernel timing with HIP events: when on, every kernel a call launches
 * goes through hipExtLaunchKernel with a start and a stop event, which the
 * dispatch itself stamps (the kernel's own start and end: not the kernels ahead
 * of it on the stream, not the host's launch latency); the RCCL gather of a
 * sharded call is bracketed by stream markers.  on = 1: ik_kernel_times
 * returns the last call's kernels; on = 2: the calls' kernels accumulate, in
 * launch order, up to 64, until the next ik_ctx_set_timing (back-to-back calls
 * timed with no host sync between them).  ik_kernel_times waits for the events
 * and returns how many kernels were timed, their durations in ms and (if names
 * != NULL) their names, name_len bytes each; a negative value is -ik_status. */
int ik_ctx_set_timing(ik_ctx *ctx, int on);
int ik_kernel_times(ik_ctx *ctx, int max, float *ms, char *names, int name_len);

/* Diagnostics: when on, the ANN kernel's workgroup 0 records s_memtime stamps
 * (shader clock ticks) per wave for its first 4 tiles: 32 slots per
 * (tile, wave) -- 0 tile start, 1 input staged, 2+2l layer l GEMM done,
 * 3+2l layer l done, 31 tile done.  ik_debug_read copies them out (returns the
 * count, or -ik_status). */
int ik_ctx_set_debug(ik_ctx *ctx, int on);
int ik_debug_read(ik_ctx *ctx, uint64_t *out, int max);

/* Pinned host memory (hipHostMalloc).  A host-pointer FABRIK solve whose arrays
 * are all pinned and that has at least 131072 points (IKHIP_PIPE_MIN; 0
 * disables) is cut into chunks whose H2D copies, kernels and D2H copies overlap
 * on three streams; pageable arrays take the one-shot path. */
int ik_host_alloc(size_t bytes, void **out);
int ik_host_free(void *p);

/* After IK_F_ASYNC calls: wait for the stream and read the accumulated stats
 * of the last call. */
int ik_stats_fetch(ik_ctx *ctx, ik_stats *stats);
/* Wait for the context's last call.  With a communicator bound (ik_comm_init)
 * the wait is bounded: it polls RCCL's async error and, past the deadline
 * (ik_comm_set_timeout), aborts the communicator and returns IK_E_RCCL -- so an
 * IK_F_ASYNC caller (e.g. a benchmark loop) never hangs on a dead peer. */
int ik_ctx_sync(ik_ctx *ctx);

/* ---- multi-GPU: RCCL over xGMI ------------------------------
 * The reference scales by competing consumers of one RabbitMQ queue
 * (rpc_broker.py:55-68); here one process per GPU shares the batch instead.
 * Every rank calls the sharded solve with the same whole batch (n points, host
 * or device pointer).  The batch is cut into C chunks of g parts each
 * (ik_shard_plan): rank r solves part (c, r) = rows [(c g + r) S, (c g + r + 1) S)
 * of every chunk c (S = ceil(n / (C g)), clipped to n), writing the results at
 * their global rows of the caller's arrays, and chunk c's rows are all-gathered
 * IN PLACE (ncclAllGather with sendbuf = recvbuf + r S rows) while chunk c + 1 is
 * solved: no pack, no unpack, no padding except in the one ragged last chunk
 * (gathered through a staging buffer and copied out).  Gathered per row: the
 * angles and, for FABRIK, the iteration counts.  The per-point FK error stays
 * local: only the rank's own rows of fk_err are written; the batch's FK-error
 * max / sum / quantiles come from a 64-byte tail record (ik_shard_tail) and a
 * histogram that ride with the last chunk's all-gather, as do first_oob /
 * first_err (the lowest GLOBAL indices: the reference's sequential exception
 * precedence).  With a device pointer only the rank's own rows of pts are read.
 * RCCL is loaded at ik_comm_init (the process's librccl if already loaded --
 * torch ships one --, else librccl.so.1; IKHIP_RCCL_LIB overrides). */
#define IK_COMM_ID_BYTES 128
#define IK_MAX_GATHER_CHUNKS 8
/* FK-error histogram of a rank (uint32 counts, gathered with the tail): finite
 * e >= 0 falls in bin 16 (E - 959) + m, E the biased float64 exponent and m the top
 * 4 mantissa bits, clamped to [0, 2047] (2^-64 .. 2^64, 1/16 octave per bin). */
#define IK_FKHIST_BINS 2048

/* The stats of one rank's shard as gathered (64 bytes). */
typedef struct ik_shard_tail {
  int64_t first_oob, first_err; /* GLOBAL indices, -1 if none */
  int32_t first_err_code, max_iters;
  int64_t sum_iters, n_capped;
  double max_fk_err, sum_fk_err;
  int64_t rows; /* rows the rank solved */
} ik_shard_tail;

/* How a batch of n rows is split over nranks ranks in chunks (host only). */
typedef struct ik_shard_plan {
  int64_t n;         /* rows of the batch */
  int32_t nranks;    /* g */
  int32_t chunks;    /* C: chunks that hold rows (<= the requested count) */
  int64_t part_rows; /* S: rows of one rank's part of one chunk */
  int64_t full_rows; /* rows of the chunks gathered in place (the rest is staged) */
} ik_shard_plan;

enum { IK_METHOD_ANN = 0, IK_METHOD_FABRIK = 1 };

/* One rank creates the id and hands it to the others (any transport). */
int ik_comm_unique_id(uint8_t *id /* IK_COMM_ID_BYTES */);
/* Collective over the nranks processes: binds the context to an RCCL
 * communicator (one GPU per rank).  The communicator is non-blocking
 * (ncclCommInitRankConfig, blocking = 0): every host wait on it -- the
 * rendezvous, group ends, a synchronous call's end, ik_ctx_sync,
 * ik_stats_fetch -- polls ncclCommGetAsyncError against a deadline
 * (IKHIP_RCCL_TIMEOUT_S, default 120 s; ik_comm_set_timeout) and on an error or
 * timeout calls ncclCommAbort and returns IK_E_RCCL naming the rank and the
 * wait.  An aborted communicator (also after any failure part-way through a
 * sharded call) refuses later calls until ik_comm_destroy + ik_comm_init.  Its
 * first act is one all-gather of a 64-byte record per rank that checks the
 * ranks agree (numbering, IKHIP_GATHER_CHUNKS, library version). */
int ik_comm_init(ik_ctx *ctx, int nranks, int rank, const uint8_t *id);
/* The deadline of the communicator's waits in seconds (0: IKHIP_RCCL_TIMEOUT_S
 * or 120).  Kept across ik_comm_init. */
int ik_comm_set_timeout(ik_ctx *ctx, double seconds);
/* TEST-ONLY: a communicator without RCCL, so that one GPU can run the sharded
 * path as rank `rank` of `nranks` (the placement of every part, the ragged
 * chunk's stage, the tail reduction).  Its all-gather writes byte o of rank
 * s's slot as ik_loopback_byte(s, o) for every s != rank, and copies this
 * rank's tail block into every rank's. */
int ik_comm_init_loopback(ik_ctx *ctx, int nranks, int rank);
/* TEST-ONLY: with on != 0 the loopback communicator's all-gathers wait for a
 * peer that never comes (each block spins on a pinned flag, at most 30 s), so a
 * test can drive the deadline path: the wait times out, the abort releases the
 * flag, the GPU drains, the call returns IK_E_RCCL. */
int ik_comm_loopback_stall(ik_ctx *ctx, int on);
int ik_loopback_byte(int slot, int64_t offset);
int ik_comm_destroy(ik_ctx *ctx);
/* The communicator as the library holds it: ranks, this rank, and the chunk
 * count the last sharded call was planned with (ik_shard_plan_of's chunks; 0
 * before one), so a caller can find its own rows with ik_shard_part. */
int ik_comm_info(ik_ctx *ctx, int *nranks, int *rank, int *last_chunks);
/* Chunks per sharded call (1..IK_MAX_GATHER_CHUNKS), or 0 = automatic: one
 * chunk for both methods (one in-place all-gather after the solve; C >= 2
 * overlaps chunk c's gather with chunk c + 1's solve, opt-in until a real
 * N >= 2 run has bit-checked it).  Every rank must use the same value:
 * each call's tail carries its plan (n, chunks, method) and a rank whose plan
 * differs from rank 0's fails the call with IK_E_RCCL.  Environment default:
 * IKHIP_GATHER_CHUNKS (checked equal on every rank by ik_comm_init). */
int ik_comm_set_chunks(ik_ctx *ctx, int chunks);
/* Host-only helpers of the protocol (no device needed). */
int ik_shard_plan_of(int64_t n, int nranks, int chunks, ik_shard_plan *out);
/* Rank's part of chunk c: rows [begin, end) (empty when begin == end). */
int ik_shard_part(const ik_shard_plan *plan, int rank, int chunk, int64_t *begin, int64_t *end);
/* = ik_shard_part of the one-chunk plan: rank's rows [r S, (r + 1) S) clipped, S = ceil(n / g). */
int ik_shard_range(int64_t n, int nranks, int rank, int64_t *begin, int64_t *end);
int ik_tail_reduce(const ik_shard_tail *tails, int nranks, ik_stats *out);
/* The bin of an FK error (see IK_FKHIST_BINS; -1 for NaN / inf / negative) and
 * the upper edge of a bin. */
int ik_fkhist_bin(double e);
double ik_fkhist_upper(int bin);
/* q-quantile (0 < q <= 1) of the FK errors of the last sharded call, from the
 * gathered histograms: the upper edge of the bin holding the ceil(q m)-th
 * smallest of the m finite errors (an upper bound, within 1/16 octave).  Needs
 * fk_err in that call; waits for it. */
int ik_fk_err_quantile(ik_ctx *ctx, double q, double *out);

/* AnnInverseKinematics.ikine / ANN.predict (see ik_ann_solve) over the ranks:
 * ang n x 4 float32 of the WHOLE batch; fk_err (nullable) n float64, of which
 * only this rank's rows are written. */
int ik_ann_solve_sharded(ik_ctx *ctx, const double *pts, int64_t n, float *ang, double *fk_err,
                         int flags, ik_stats *stats);
/* FabrikInverseKinematics.ikine (see ik_fabrik_solve_fk) over the ranks: ang n x 4
 * float64 and iters (nullable) n int32 of the whole batch, fk_err (nullable) n
 * float64 of this rank's rows. */
int ik_fabrik_solve_sharded(ik_ctx *ctx, const double *pts, int64_t n, double tol,
                            int32_t max_iter, double *ang, int32_t *iters, double *fk_err,
                            int flags, ik_stats *stats);

#ifdef __cplusplus
}
#endif
#endif /* IKHIP_H */
