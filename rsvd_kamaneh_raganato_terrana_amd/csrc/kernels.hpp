// kernels.hpp -- host-side launch wrappers for the gfx950 rSVD kernels (one per .hip file).
// Every wrapper enqueues on `stream` and returns hipSuccess or the launch error; none of them
// allocates or synchronises (so the driver can be captured into a hipGraph).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rsvd {

enum class DType : int { F64 = 0, F32 = 1, BF16 = 2, FP8_E4M3 = 3 };

// ---- util.hip --------------------------------------------------------------------------------
// Omega (n x l, N(0,1) Philox4x32-10, stream element i + n*j) into a row-major n x LP panel.
template <typename T>
hipError_t launch_philox_omega(T* out, int64_t n, int l, int LP, uint64_t seed, hipStream_t s);
// col-major (ld) m x l  ->  row-major m x LP panel (zero-padded)
template <typename T>
hipError_t launch_colmajor_to_panel(const T* in, int64_t ld, int64_t m, int l, int LP, T* out, hipStream_t s);
// Sum `nslab` slabs of `count` elements (stride slab_stride) into out.
template <typename T>
hipError_t launch_sum_slabs(const T* slabs, int64_t slab_stride, int nslab, int64_t count, T* out, hipStream_t s);
// row-major m x LP panel (first `cols` columns)  ->  col-major (ld) m x cols
template <typename T>
hipError_t launch_panel_to_colmajor(const T* in, int64_t m, int cols, int LP, T* out, int64_t ld, hipStream_t s);

// X (col-major rows x cols, ld) *= f
template <typename T>
hipError_t launch_scale_cols(T* X, int64_t rows, int cols, int64_t ld, double f, hipStream_t s);
// *flag |= 1 when any of x[0..n) is not finite
template <typename T>
hipError_t launch_check_finite(const T* x, int n, int* flag, hipStream_t s);
// *cnt = v (one fp64 word; the row count a sharded run sums with its first m-side Gram all-reduce)
hipError_t launch_set_count(double* cnt, int64_t v, hipStream_t s);
// *flag = 1 when *cnt (the summed global row count) is below l
hipError_t launch_check_rows(const double* cnt, int l, int* flag, hipStream_t s);

// Fallback re-orthonormalisation of P into Q (CGS2 + deterministic random completion) when
// *flag != 0; returns immediately otherwise.  One workgroup.
template <typename T>
hipError_t launch_robust_orth(const T* P, int64_t rows, int l, int LP, T* Q, const int* flag, uint64_t seed,
                              hipStream_t s);

// ---- proj.hip: the projections (MFMA) ----------------------------------------------------------
struct ProjPlan {
    int splits;      // K-splits (slabs); 1 => written straight into the output panel
    int64_t chunk;   // K range per workgroup
    int blocks;      // output row/col blocks
};
// Y (m x LP panel) = A (m x n, col-major) * X (n x LP panel)        [src/rSVD.cpp:59,66]
template <typename T>
ProjPlan plan_proj_nn(int64_t m, int64_t n, int LP);
// `done` (optional) is recorded right after the GEMM kernel, before the slab reduction.
template <typename T>
hipError_t launch_proj_nn(const T* A, int64_t lda, int64_t m, int64_t n, const T* X, int LP,
                          const ProjPlan& p, T* slabs, T* Y, hipStream_t s, hipEvent_t done = nullptr);
// Z (n x LP panel) = A^T * Q (m x LP panel)                           [src/rSVD.cpp:63,89]
template <typename T>
ProjPlan plan_proj_tn(int64_t m, int64_t n, int LP);
template <typename T>
hipError_t launch_proj_tn(const T* A, int64_t lda, int64_t m, int64_t n, const T* Q, int LP,
                          const ProjPlan& p, T* slabs, T* Z, hipStream_t s, hipEvent_t done = nullptr);

// ---- qr.hip: CholeskyQR with fp64 Gram ----------------------------------------------------------
// Workgroups for the partial Gram of a `rows`-row panel; Gram tiles (16x16) per slab.
int plan_gram_blocks(int64_t rows);
int gram_tiles(int LP, int cross);
// One launch: partial Grams of P (rows x LP) -> nb slabs -> per-tile reductions (fixed order)
// -> mode 1: R = chol(G) (upper, LP x LP zero-padded) and Rinv = R^-1, factored in fp32 when
// compute_f32 else fp64; mode 0: the summed Gram to Gsum (distributed path).  flag[0] += 1 on a
// bad pivot.  ctr[0..1] are run-cumulative arrival counters (zeroed per run): t0 = ctr[0] after
// this launch's nb arrivals, t1 = ctr[1] after its tile reducers (gram_tiles(LP, 0)).
// pred (nullable): the whole launch is skipped unless *pred != 0 (give such a launch counters of its
// own).  tmo: the sticky timeout word (a bounded hand-off spin that expired sets it).  refine (nullable, mode 1): set to 1 when cond_F(R) > 2e4 or a pivot broke down -- the
// predicate of an optional second CholeskyQR pass.
template <typename T>
hipError_t launch_gram_chol(const T* P, int64_t rows, int LP, int nb, double* slabs, double* tiles, unsigned* ctr,
                            unsigned t0, unsigned t1, int mode, int compute_f32, double* Gsum, int l, double* R,
                            double* Rinv, int* flag, int* tmo, hipStream_t s, const int* pred = nullptr,
                            int* refine = nullptr);
// Cross-Gram Gout = P^T P2 (LP x LP fp64, zero outside l x l); t1 advances by gram_tiles(LP, 1).
template <typename T>
hipError_t launch_cross_gram(const T* P, const T* P2, int64_t rows, int LP, int nb, double* slabs, double* tiles,
                             unsigned* ctr, unsigned t0, unsigned t1, double* Gout, int l, int* tmo, hipStream_t s);
// Factor an already-summed Gram G (LP x LP) -- same outputs as mode 1 above.
hipError_t launch_chol(const double* G, int l, int LP, int compute_f32, double* R, double* Rinv, int* flag,
                       hipStream_t s);
// Out (rows x LP) = In (rows x LP) * M (LP x LP, fp64, applied in T precision).
// out_colmajor: write Out's first `cols` columns col-major with leading dim ld instead.
template <typename T>
hipError_t launch_panel_small(const T* In, int64_t rows, int LP, const double* M, T* Out,
                              int out_colmajor, int cols, int64_t ld, hipStream_t s, const int* pred = nullptr);

// ---- jacobi.hip: small SVD of W = R^T (l x l) ---------------------------------------------------
// One-sided Jacobi (round-robin order) in fp64 on one workgroup.  Outputs U_w, V_w (LP x LP
// fp64, zero padded), S (l, descending) in the requested precision.  Returns sweeps in *info.
template <typename T>
hipError_t launch_small_svd(const double* R, int l, int LP, double* Uw, double* Vw, T* S, int* info,
                            hipStream_t s);

}  // namespace rsvd
