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

// ---- proj.hip: the projections (MFMA) ----------------------------------------------------------
struct ProjPlan {
    int splits;      // K-splits (slabs); 1 => written straight into the output panel
    int64_t chunk;   // K range per workgroup
    int blocks;      // output row/col blocks
};
// Y (m x LP panel) = A (m x n, col-major) * X (n x LP panel)        [src/rSVD.cpp:59,66]
template <typename T>
ProjPlan plan_proj_nn(int64_t m, int64_t n, int LP);
template <typename T>
hipError_t launch_proj_nn(const T* A, int64_t lda, int64_t m, int64_t n, const T* X, int LP,
                          const ProjPlan& p, T* slabs, T* Y, hipStream_t s);
// Z (n x LP panel) = A^T * Q (m x LP panel)                           [src/rSVD.cpp:63,89]
template <typename T>
ProjPlan plan_proj_tn(int64_t m, int64_t n, int LP);
template <typename T>
hipError_t launch_proj_tn(const T* A, int64_t lda, int64_t m, int64_t n, const T* Q, int LP,
                          const ProjPlan& p, T* slabs, T* Z, hipStream_t s);

// ---- qr.hip: CholeskyQR2 with fp64 Gram / Cholesky ----------------------------------------------
// Partial Gram slabs of the first l columns of a rows x LP panel; returns slab count via plan.
int plan_gram_blocks(int64_t rows);
template <typename T>
hipError_t launch_gram_partial(const T* P, int64_t rows, int LP, int nblk, double* gslabs, hipStream_t s);
// G = sum of slabs; R = chol(G) (upper, l x l, LP-padded);  Rinv = R^-1; Racc = R * Racc_in
// (if accumulate).  Sets *flag |= 1 when a pivot is not safely positive (breakdown / rank loss).
hipError_t launch_chol_inv(const double* gslabs, int nslab, int l, int LP, double* R, double* Rinv,
                           double* Racc, int accumulate, int* flag, hipStream_t s);
// Out (rows x LP) = In (rows x LP) * M (LP x LP, fp64, applied in T precision).
// out_colmajor: write Out's first `cols` columns col-major with leading dim ld instead.
template <typename T>
hipError_t launch_panel_small(const T* In, int64_t rows, int LP, const double* M, T* Out,
                              int out_colmajor, int cols, int64_t ld, hipStream_t s);

// ---- jacobi.hip: small SVD of W = R^T (l x l) ---------------------------------------------------
// One-sided Jacobi (round-robin order) in fp64 on one workgroup.  Outputs U_w, V_w (LP x LP
// fp64, zero padded), S (l, descending) in the requested precision.  Returns sweeps in *info.
template <typename T>
hipError_t launch_small_svd(const double* R, int l, int LP, double* Uw, double* Vw, T* S, int* info,
                            hipStream_t s);

}  // namespace rsvd
