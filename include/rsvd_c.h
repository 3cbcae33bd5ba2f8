/*
 * rsvd_c.h -- C ABI of the MI355X-native randomized-SVD engine (librsvd_hip.so).
 *
 * Plain pointers and sizes only: no torch, Eigen or HIP types cross this boundary (streams are
 * passed as `void*` = hipStream_t).  Every entry point returns an rsvd_status_t and never throws.
 *
 * Boundary mapping (reference = AMSC22-23/rSVD_Kamaneh_Raganato_Terrana @ 2024-10-08):
 *   rsvd_run / rsvd_run_host_f64    <- void rSVD(Mat_m& A, Mat_m& U, Vec_v& S, Mat_m& V, int l,
 *                                          SVDMethod)             include/rSVD.hpp:14, src/rSVD.cpp:72-133
 *   rsvd_range_finder              <- void intermediate_step(const Mat_m& A, Mat_m& Q,
 *                                          const Mat_m& Omega, int l, int q)
 *                                                                  include/rSVD.hpp:13, src/rSVD.cpp:57-70
 *   rsvd_generate_omega            <- Mat_m generateOmega(int n, int l)
 *                                                                  include/rSVD.hpp:15, src/rSVD.cpp:12-55
 *   rsvd_qr (full = 0 / 1)         <- void qr_decomposition_reduced/full(const Mat_m& A, Mat_m& Q,
 *                                          Mat_m& R)              include/QR.hpp:15-16, src/QR.cpp:22-80
 *   rsvd_svd                       <- template<SVDMethod> SVD::compute()/getU/getS/getV
 *                                                                  include/SVD_class.hpp:35-71,79-180
 * The C++ drop-in headers include/rSVD.hpp, include/QR.hpp, include/SVD_class.hpp sit on top of
 * these symbols with the reference's exact signatures.
 *
 * Layouts: every matrix is COLUMN-major (Eigen's default) with an explicit leading dimension.
 * Device-pointer entry points are asynchronous on the handle's stream; *_host_* variants copy
 * host buffers in and out and synchronise.
 */
#ifndef RSVD_C_H
#define RSVD_C_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RSVD_ABI_VERSION 6

typedef enum {
    RSVD_OK = 0,
    RSVD_ERR_INVALID_ARG = 1,    /* bad sizes / pointers (Eigen would assert)                      */
    RSVD_ERR_UNSUPPORTED = 2,    /* e.g. SVD method not available; maps to std::invalid_argument     */
    RSVD_ERR_HIP = 3,            /* a HIP runtime / launch error (see rsvd_last_error)              */
    RSVD_ERR_NO_DEVICE = 4,
    RSVD_ERR_NUMERICAL = 5,      /* non-finite result                                              */
    RSVD_ERR_COMM = 6            /* the distributed all-reduce callback failed                      */
} rsvd_status_t;

/* Storage / compute type of A.  F64: fp64 end to end (the reference's arithmetic class).
 * F32: fp32 MFMA projections and fp32 panels; Grams accumulated in fp64 (f64 MFMA), the panel
 * products by R^-1 in fp64, Cholesky factor and small Jacobi SVD in fp32.
 * BF16 / FP8_E4M3 (OCP e4m3fn): A stored in that type (A = a_scale * stored value), projections
 * on the bf16 MFMA with a hi/lo-split fp32 skinny operand, fp32 panels, fp64 Grams / Cholesky /
 * small SVD; Omega is the Philox Gaussian rounded to bf16 (resp. e4m3); U, S, V, Omega and Q are
 * fp32 at the ABI. */
typedef enum { RSVD_F64 = 0, RSVD_F32 = 1, RSVD_BF16 = 2, RSVD_FP8_E4M3 = 3 } rsvd_dtype_t;

/* Mirrors enum class SVDMethod { Jacobi, Power, ParallelJacobi } (include/SVD_class.hpp:28-32).
 * RSVD_SVD_POWER_IC (rsvd_run / rsvd_range_finder only) is image_compression's power-method small
 * SVD behind its 5-argument rSVD (image_compression/src/SVD.cpp:30-55, PowerMethod.cpp:3-43): B is
 * recomputed as A^T A of the deflated matrix after every triplet and there is no sigma < 1e-12 stop
 * (a triplet with sigma == 0, where the reference divides by zero, ends it); V in columns. */
typedef enum {
    RSVD_SVD_JACOBI = 0,
    RSVD_SVD_POWER = 1,
    RSVD_SVD_PARALLEL_JACOBI = 2,
    RSVD_SVD_POWER_IC = 3
} rsvd_svd_method_t;

/* Orthonormalisation of the tall-skinny panels.  AUTO = CholeskyQR (one pass for fp32 power-
 * iteration intermediates, two otherwise) with a predicated Gram-Schmidt (CGS2) re-
 * orthonormalisation of the panel when a Cholesky pivot breaks down (rank-deficient or too
 * ill-conditioned sketch).  GS2 = always the CGS2 path (single-GPU panels).
 * CHOLQR2 = two CholeskyQR passes on every panel. */
typedef enum { RSVD_QR_AUTO = 0, RSVD_QR_GS2 = 1, RSVD_QR_CHOLQR2 = 2 } rsvd_qr_mode_t;

/* rsvd_desc_t.flags.  LOWP_INTERMEDIATES (bf16 / e4m3 A, q >= 2): the two projections of power
 * iterations 1 .. q-1 take the fp32 skinny operand as its bf16 rounding alone (one MFMA pass
 * instead of the hi + lo pair); the last iteration, B^T = A^T Q and the outputs keep 16-bit
 * operands.  An error injected there is damped by the later iterations by about
 * (sigma_{l+1} / sigma_{l/2})^2 each: on spectra that decay across the sketch (e.g. 0.985^i at
 * l = 256) the results stay within 1e-5 of the full-precision path, on flat ones (0.999^i) they
 * drift to ~5e-3.  Off by default. */
#define RSVD_FLAG_LOWP_INTERMEDIATES 1
/* Test/diagnostic flag (ABI 6): run the n-side sharded code path (reduce-scatter / all-gather
 * through the handle's collectives) even at world 1, so a one-GPU box exercises the exact RCCL
 * calls an N-GPU run makes.  Requires collectives (rsvd_set_collectives or rsvd_comm_init). */
#define RSVD_FLAG_FORCE_NSHARD 2

typedef struct {
    int64_t m, n;              /* A is m x n                                                   */
    int64_t lda;               /* >= m                                                         */
    int32_t l;                 /* sketch width k + p (the reference's `l`)                     */
    int32_t q;                 /* power iterations; the reference hard-codes 2 (src/rSVD.cpp:83) */
    int32_t dtype;             /* rsvd_dtype_t                                                 */
    int32_t method;            /* rsvd_svd_method_t                                            */
    int32_t qr_mode;           /* rsvd_qr_mode_t                                               */
    int32_t flags;             /* RSVD_FLAG_* (ABI 5; the former reserved word, 0 = defaults)  */
    uint64_t seed;             /* Philox key for Omega when no Omega is supplied               */
    double a_scale;            /* A = a_scale * (stored A); 0 means 1 (any dtype; S scales by
                                  |a_scale|, V flips sign when a_scale < 0)                        */
} rsvd_desc_t;

/* Diagnostics of the last run on a handle. */
typedef struct {
    int32_t cholqr_fallbacks;  /* panels re-orthonormalised by the CGS2 fallback                 */
    int32_t jacobi_sweeps;     /* sweeps of the small SVD                                      */
    int32_t splits_nn, splits_tn; /* K splits chosen for the projections                         */
    int32_t power_kept;        /* SVDMethod::Power: triplets found before sigma < 1e-12 (else 0)  */
    int32_t n_shard_rows;      /* n-side rows per rank of a sharded n side (ABI 5), 0: replicated */
} rsvd_info_t;

typedef struct rsvd_handle_s *rsvd_handle_t;

/* Distributed exchange hook: sum `count` elements of `dtype` at device pointer `buf` over all
 * ranks, in place, ordered after the work already enqueued on `stream`.  Return 0 on success.
 * (The Python front end binds it to torch.distributed.all_reduce over RCCL.) */
typedef int (*rsvd_allreduce_fn)(void *buf, int64_t count, int32_t dtype, void *stream, void *user);

/* Collective hook of the n-side sharding (ABI 5).  op RSVD_COLL_REDUCE_SCATTER: `send` holds
 * world x count elements, rank r receives the sum over ranks of elements [r count, (r + 1) count)
 * in `recv` (recv may alias send + rank count, in place).  op RSVD_COLL_ALL_GATHER: every rank
 * contributes `count` elements at `send` and receives all world x count, rank r's at
 * recv + r count (send may alias recv + rank count).  dtype: RSVD_F64, RSVD_F32 or RSVD_BF16.
 * Ordered after the work enqueued on `stream`; return 0 on success.  (The Python front end binds
 * it to torch.distributed.reduce_scatter_tensor / all_gather_into_tensor over RCCL.) */
typedef int (*rsvd_collective_fn)(int32_t op, void *send, void *recv, int64_t count, int32_t dtype, void *stream,
                                  void *user);
#define RSVD_COLL_REDUCE_SCATTER 1
#define RSVD_COLL_ALL_GATHER 2

const char *rsvd_status_string(int status);
int rsvd_abi_version(void);

int rsvd_create(int device, rsvd_handle_t *out);
int rsvd_destroy(rsvd_handle_t h);
int rsvd_set_stream(rsvd_handle_t h, void *hip_stream);
const char *rsvd_last_error(rsvd_handle_t h);
/* Synchronise the handle's stream and report what the queued runs could not report at enqueue
 * time: RSVD_ERR_HIP for an in-kernel hand-off or grid barrier that timed out,
 * RSVD_ERR_NUMERICAL for a rank-deficient panel the repair pass could not complete or for
 * non-finite singular values.  These conditions are sticky on the handle until reported (by this
 * call or rsvd_get_info), so one rsvd_sync after several asynchronous rsvd_run calls checks them
 * all.  The *_host_* entry points end with it. */
int rsvd_sync(rsvd_handle_t h);
/* rsvd_sync, then the diagnostics of the last run. */
int rsvd_get_info(rsvd_handle_t h, rsvd_info_t *info);
/* Row-sharded runs: this handle owns rows [offset, offset + m_local) of a global m x n A; the
 * hook sums the n x l partial products A_g^T Q_g and the l x l Grams across ranks. */
int rsvd_set_comm(rsvd_handle_t h, int rank, int world, rsvd_allreduce_fn fn, void *user);
/* Optional (ABI 5), after rsvd_set_comm: with a collective hook the wide engine (bf16 / e4m3 A,
 * or l > 64) also shards the n side -- rank r owns rows [r c, (r + 1) c) of the
 * n x l panels, c = n / world rounded up to 32: A^T Q is reduce-scattered instead of all-reduced,
 * each rank orthonormalises its rows (CholeskyQR with the l x l Gram all-reduced), the next
 * skinny operand and the final V are all-gathered.  fn = NULL switches back to the replicated
 * n side.  SVDMethod::Power runs keep the replicated n side.  rsvd_workspace_bytes covers the
 * padded n-side panels of any world up to 64; past 64 ranks the n side stays replicated. */
int rsvd_set_collectives(rsvd_handle_t h, rsvd_collective_fn fn, void *user);

/* Library-owned RCCL (ABI 6): the handle creates and owns an RCCL communicator over the ranks'
 * GPUs (one process per GPU, as the reference's MPI ranks, src/rSVD.cpp:15,20-23) and issues
 * ncclAllReduce / ncclReduceScatter / ncclAllGather on its own stream -- no hooks, no Python.
 * rsvd_comm_unique_id fills RSVD_COMM_ID_BYTES bytes (ncclGetUniqueId) on ONE rank; the caller
 * broadcasts them (e.g. MPI_Bcast, where the reference Bcasts Omega, src/rSVD.cpp:52) and every
 * rank calls rsvd_comm_init with its rank.  shard_n != 0 also shards the n side (as
 * rsvd_set_collectives).  rsvd_set_comm / rsvd_set_collectives afterwards replace it;
 * rsvd_comm_destroy (or rsvd_destroy) releases it.  librccl is loaded on first use
 * (RSVD_ERR_UNSUPPORTED when it cannot be). */
#define RSVD_COMM_ID_BYTES 128
int rsvd_comm_unique_id(void *id);
int rsvd_comm_init(rsvd_handle_t h, const void *id, int rank, int world, int shard_n);
int rsvd_comm_destroy(rsvd_handle_t h);

/* Row partition of src/rSVD.cpp:20-23 / src/PM.cpp:31-35: rows of rank `rank` out of `world`.
 * Host-only arithmetic (no device needed).  Returns the local row count, *offset = first row. */
int64_t rsvd_row_partition(int64_t rows, int world, int rank, int64_t *offset);

/* Device workspace bytes rsvd_run needs for `desc` (allocated lazily by the handle). */
int rsvd_workspace_bytes(const rsvd_desc_t *desc, size_t *bytes);
/* Timing mode (benchmarking): hipEvent pairs bracket every projection GEMM kernel launch
 * (A*X and A^T*Q; not their slab reductions).  rsvd_set_timing resets the accumulators;
 * rsvd_get_timing synchronises the stream and returns totals since the reset. */
typedef struct {
    int32_t nn_launches, tn_launches;
    double nn_ms, tn_ms;
    int32_t sketch_launches, reserved; /* the sketch Y = A Omega alone (also counted in nn_*): e4m3 A runs
                                          it on the fp8 MFMA, every other product on the bf16 / fp32 one */
    double sketch_ms;
} rsvd_timing_t;
int rsvd_set_timing(rsvd_handle_t h, int enable);
int rsvd_get_timing(rsvd_handle_t h, rsvd_timing_t *t);
/* Use caller-owned device memory as the workspace (NULL reverts to handle-owned memory). */
int rsvd_set_workspace(rsvd_handle_t h, void *ptr, size_t bytes);

/* ---- device-pointer entry points (asynchronous on the handle stream) ---------------------- */

/* rSVD: U (m x d, ldu), S (d), V (n x d, ldv), d = min(l, n); element type = desc->dtype (fp32
 * for BF16 / FP8_E4M3).  method POWER (src/rSVD.cpp:106-113): the reference's power method with
 * deflation on B = Q^T A (start vectors: Philox stream (seed ^ 0x504F574552) + i, the reference's
 * s(n) iterations); V's columns are the right singular vectors (the reference returns them as the
 * rows of an n x n V_ -- include/SVD_class.hpp rebuilds that layout); triplets past an early stop
 * (sigma < 1e-12) are zero and rsvd_get_info reports how many were kept.  omega: optional n x l column-major (ld = ldo) sketch in that element
 * type (rounded to bf16 / e4m3 for the low-precision types); NULL => Philox(desc->seed).
 * l <= 512 on the wide engine; 512 < l <= 4096 (the reference has no cap, src/rSVD.cpp:72) on one GPU
 * through dense_big.cpp's column-major blocks (MFMA GEMM products, block CGS2 + CholeskyQR3, the
 * block Jacobi small SVD -- or, for Power, the power method in the coordinates of Q_B on a persistent
 * grid; bf16 / e4m3 A widened to fp32 once), also row-sharded (RSVD_ERR_UNSUPPORTED for
 * RSVD_SVD_POWER_IC and past 4096). */
int rsvd_run(rsvd_handle_t h, const rsvd_desc_t *desc, const void *A, const void *omega, int64_t ldo,
             void *U, int64_t ldu, void *S, void *V, int64_t ldv);

/* intermediate_step: Q (m x l, ldq) orthonormal basis of the range of (A A^T)^q A Omega. */
int rsvd_range_finder(rsvd_handle_t h, const rsvd_desc_t *desc, const void *A, const void *omega, int64_t ldo,
                      void *Q, int64_t ldq);

/* generateOmega: n x l N(0,1), column-major (ld = n), element (i,j) = Philox stream element i+n*j.
 * dtype BF16 / FP8_E4M3: the same values rounded to bf16 / e4m3 (round half to even; e4m3
 * saturates at +-448), written as fp32 -- the Omega the low-precision rsvd_run draws. */
int rsvd_generate_omega(rsvd_handle_t h, int64_t n, int32_t l, uint64_t seed, int32_t dtype, void *omega);

/* QR() boundary <- qr_decomposition_reduced / qr_decomposition_full (include/QR.hpp:15-16,
 * src/QR.cpp:22-80).  full = 0: Q m x n (ldq), R n x n (ldr), requires m >= n (src/QR.cpp:78);
 * full = 1: Q m x m, R m x n (upper trapezoidal).  dtype F64 / F32.  Q has orthonormal columns
 * and A = Q R; R(j,j) >= 0 except on the leading columns of A whose sub-diagonal is already zero,
 * where R(j,j) = A(j,j) as the Givens sweep leaves them.  For full-rank A this is the unique QR,
 * i.e. the reference's; the complement Q[:, n:] of a full QR is an orthonormal completion
 * (identity columns for an A with trailing zero rows).  Up to 512 columns (of A, or of Q for the
 * full form) one shifted-CholeskyQR3 pass; past that, 512-column blocks by block CGS2 + CholeskyQR3
 * (dense_big.cpp), bounded only by device memory. */
int rsvd_qr(rsvd_handle_t h, int64_t m, int64_t n, const void *A, int64_t lda, int32_t dtype, int32_t full, void *Q,
            int64_t ldq, void *R, int64_t ldr);

/* SVD<method>::compute() boundary (include/SVD_class.hpp:35-97).  Jacobi / ParallelJacobi
 * (:100-180, :223-333): U m x k (ldu), S k (descending, >= 0), V n x k (ldv), k = min(m, n)
 * <= 4096 (past 512: block Jacobi directly on the columns of A or A^T, RSVD_ERR_UNSUPPORTED
 * above 4096); dtype F64 / F32.  Power (:183-219 with PM, src/PM.cpp): dtype F64, any n,
 * dim = r ? r : min(m, n) deflation steps, start vectors Philox(seed + i); stops at the first
 * sigma < 1e-12 (:198-208); *kept = triplets written (U, S, V columns 0..kept-1; V's columns are
 * the right singular vectors -- the reference's row layout is rebuilt by include/SVD_class.hpp).
 * Jacobi sets *kept = k without synchronising; Power synchronises the stream. */
int rsvd_svd(rsvd_handle_t h, int64_t m, int64_t n, const void *A, int64_t lda, int32_t dtype, int32_t method,
             int32_t r, uint64_t seed, void *U, int64_t ldu, void *S, void *V, int64_t ldv, int32_t *kept);
/* Device workspace bytes of rsvd_qr / rsvd_svd (for rsvd_set_workspace callers). */
int rsvd_qr_workspace_bytes(int64_t m, int64_t n, int32_t dtype, int32_t full, size_t *bytes);
int rsvd_svd_workspace_bytes(int64_t m, int64_t n, int32_t dtype, int32_t method, size_t *bytes);

/* ---- host-pointer fp64 entry points used by the C++ drop-in headers (synchronous) --------- */
int rsvd_run_host_f64(rsvd_handle_t h, int64_t m, int64_t n, const double *A, int64_t lda, int32_t l,
                      int32_t q, int32_t method, const double *omega /* nullable, n x l, ld n */,
                      uint64_t seed, double *U /* m x d */, double *S /* d */, double *V /* n x d */);
int rsvd_range_finder_host_f64(rsvd_handle_t h, int64_t m, int64_t n, const double *A, int64_t lda,
                               const double *omega /* n x l, ld n */, int32_t l, int32_t q,
                               double *Q /* m x l */);
int rsvd_generate_omega_host_f64(rsvd_handle_t h, int64_t n, int32_t l, uint64_t seed, double *omega);
/* Q: m x (full ? m : n), ld m; R: (full ? m : n) x n, ld = its rows. */
int rsvd_qr_host_f64(rsvd_handle_t h, int64_t m, int64_t n, const double *A, int64_t lda, int32_t full, double *Q,
                     double *R);
/* U: m x min(m,n), S: min(m,n), V: n x min(m,n) buffers (ld m, n); *kept columns are written. */
int rsvd_svd_host_f64(rsvd_handle_t h, int64_t m, int64_t n, const double *A, int64_t lda, int32_t method, int32_t r,
                      uint64_t seed, double *U, double *S, double *V, int32_t *kept);

#ifdef __cplusplus
}
#endif
#endif /* RSVD_C_H */
