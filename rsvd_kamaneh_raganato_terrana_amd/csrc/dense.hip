// dense.hip -- kernels of the dense drop-ins next to rSVD: QR() (src/QR.cpp:22-80) and the
// stand-alone SVD<method> (include/SVD_class.hpp:79-219).  The heavy lifting reuses the wide
// engine's CholeskyQR / Gram / panel-product / Jacobi kernels (wide_qr.hip, wide_svd.hip,
// jacobi.hip); this file adds the layout helpers and the power method.
//
//   transpose_to_panel   A (m x n col-major) -> A^T as an n x LP row-major panel: the panel row j
//                        is column j of A, so reads and writes are both unit-stride.
//   upper_to_colmajor    R = Q^T A (LP x LP fp64 row-major) -> the caller's column-major R with the
//                        strictly lower part set to 0 (Givens R is upper triangular / trapezoidal).
//   shift_diag           G += s I, s = 11 (rows l + l (l + 1)) u tr(G): the shift of shifted
//                        CholeskyQR3, which keeps the first pass positive definite up to
//                        cond(A) ~ 1/u (Fukaya et al., SIAM J. Sci. Comput. 2020).
//   power_svd_kernel     SVD<Power> (SVD_class.hpp:183-219 + src/PM.cpp:4-81): for i < dim, a
//                        fixed number `s` of power iterations x <- B x / |B x| on the deflated
//                        B = A^T A, v = x, sigma = |A_i v|, u = A_i v / sigma, stop when
//                        sigma < 1e-12, deflate B -= sigma^2 (u.u) v v^T.  A_i = A - sum_j<i
//                        sigma_j u_j v_j^T is applied implicitly (A v - sum_j sigma_j (v_j.v) u_j),
//                        so A is never rewritten.  One workgroup; B lives in LDS when LP <= 128.
#include "common.hpp"
#include "dense.hpp"

namespace rsvd {

namespace {

constexpr int kPowThreads = 1024;

template <typename T>
__global__ void transpose_to_panel_kernel(const T* __restrict__ A, int64_t lda, int64_t m, int64_t n, int LP,
                                          T* __restrict__ P) {
    const int64_t total = n * LP;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = e / LP;
        const int64_t i = e - j * LP;
        P[e] = (i < m) ? A[i + j * lda] : T(0);
    }
}

template <typename T>
__global__ void unit_columns_kernel(T* __restrict__ P, int LP, int c0, int c1) {
    const int j = c0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (j < c1) P[(int64_t)j * LP + j] = T(1);
}

// One workgroup: nz[j] = column j of A has a non-zero below the diagonal; the leading run of
// columns with nz[j] == 0 saw no Givens rotation in the reference, so R(j,j) = A(j,j).
template <typename T>
__global__ __launch_bounds__(256) void qr_signs_kernel(const T* __restrict__ A, int64_t lda, int64_t m, int n,
                                                       T* __restrict__ Qp, int LP) {
    __shared__ int nz[512];
    __shared__ int run;
    const int kmin = (int)(m < n ? m : n);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int j = w; j < kmin; j += 4) {
        int any = 0;
        for (int64_t i = j + 1 + lane; i < m; i += 64) any |= A[i + j * lda] != T(0);
        any = __any(any);
        if (lane == 0) nz[j] = any;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        while (t < kmin && !nz[t]) ++t;
        run = t;
    }
    __syncthreads();
    for (int j = 0; j < run; ++j) {
        if (!(A[j + j * lda] < T(0))) continue;
        for (int64_t i = threadIdx.x; i < m; i += 256) Qp[i * LP + j] = -Qp[i * LP + j];
    }
}

// Out = In R^-1 by forward substitution per row (R upper, LP x LP fp64): q R = a solved row by
// row is backward stable, |a - q R| <= O(u) |q| |R|, however ill-conditioned R is -- the explicit
// R^-1 product of the rSVD panels (wide_qr.hip panel_gemm) loses u * cond(R), which a QR() caller
// would see as A != Q R for rank-deficient A.  One thread per row; the R columns of a 32-wide
// chunk are staged in LDS (rows 0 .. c0 + 32), earlier outputs of the row are re-read from Out.
template <typename T>
__global__ __launch_bounds__(256) void trsm_rows_kernel(const T* __restrict__ In, int64_t rows, int k, int LP,
                                                        const double* __restrict__ R, T* __restrict__ Out,
                                                        const int* __restrict__ pred) {
    if (pred && *pred == 0) return;
    extern __shared__ double Rs[];  // [c0 + 32][32]
    const int tid = threadIdx.x;
    const int64_t row = blockIdx.x * 256ll + tid;
    const bool live = row < rows;
    for (int c0 = 0; c0 < LP; c0 += 32) {
        const int cw = (LP - c0 < 32) ? LP - c0 : 32;
        __syncthreads();
        for (int e = tid; e < (c0 + cw) * 32; e += 256) {
            const int t = e >> 5, j = e & 31;
            Rs[e] = (j < cw) ? R[(int64_t)t * LP + c0 + j] : 0.0;
        }
        __syncthreads();
        if (!live) continue;
        double x[32];
#pragma unroll
        for (int j = 0; j < 32; ++j) x[j] = (c0 + j < k) ? (double)In[row * LP + c0 + j] : 0.0;
        for (int t = 0; t < c0; ++t) {
            const double q = (double)Out[row * LP + t];
#pragma unroll
            for (int j = 0; j < 32; ++j) x[j] -= q * Rs[t * 32 + j];
        }
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            const int c = c0 + j;
            if (c < k) {
                x[j] /= Rs[c * 32 + j];
#pragma unroll
                for (int jj = j + 1; jj < 32; ++jj) x[jj] -= x[j] * Rs[c * 32 + jj];
            } else {
                x[j] = 0.0;
            }
        }
#pragma unroll
        for (int j = 0; j < 32; ++j)
            if (j < cw) Out[row * LP + c0 + j] = (T)x[j];
    }
}

// det(Q) of a square Q (m x m in a row-major LP panel) by LU with partial pivoting in W (LP x LP
// fp64 scratch, L2-resident); when det(Q) < 0 column m-1 of Q is negated.  The reference's Q is a
// product of Givens rotations (det +1) and its last column is never rotated on its own
// (src/QR.cpp:31-32: no row below it), so R(m-1, m-1) carries whatever sign makes det(Q) = +1.
template <typename T>
__global__ __launch_bounds__(1024) void det_sign_kernel(T* __restrict__ Qp, int m, int LP, double* __restrict__ W) {
    __shared__ double bv[16];
    __shared__ int bi[16];
    __shared__ int piv;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    for (int e = tid; e < m * m; e += 1024) {
        const int i = e / m, j = e - i * m;
        W[(int64_t)i * LP + j] = (double)Qp[(int64_t)i * LP + j];
    }
    __syncthreads();
    int sign = 1;
    for (int k = 0; k < m; ++k) {
        double v = -1.0;
        int vi = k;
        for (int i = k + tid; i < m; i += 1024) {
            const double a = fabs(W[(int64_t)i * LP + k]);
            if (a > v) {
                v = a;
                vi = i;
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const double ov = __shfl_xor(v, o);
            const int oi = __shfl_xor(vi, o);
            if (ov > v || (ov == v && oi < vi)) {
                v = ov;
                vi = oi;
            }
        }
        if (lane == 0) {
            bv[w] = v;
            bi[w] = vi;
        }
        __syncthreads();
        if (tid == 0) {
            double b = bv[0];
            int p = bi[0];
            for (int t = 1; t < 16; ++t)
                if (bv[t] > b || (bv[t] == b && bi[t] < p)) {
                    b = bv[t];
                    p = bi[t];
                }
            piv = p;
        }
        __syncthreads();
        const int p = piv;
        if (p != k) {
            for (int j = k + tid; j < m; j += 1024) {
                const double t = W[(int64_t)k * LP + j];
                W[(int64_t)k * LP + j] = W[(int64_t)p * LP + j];
                W[(int64_t)p * LP + j] = t;
            }
            sign = -sign;
            __syncthreads();
        }
        const double d = W[(int64_t)k * LP + k];
        if (!(d != 0.0)) {  // singular (cannot happen for an orthonormal Q): leave Q as is
            sign = 1;
            break;
        }
        if (d < 0.0) sign = -sign;
        const int rem = m - k - 1;
        for (int e = tid; e < rem * rem; e += 1024) {
            const int i = k + 1 + e / rem, j = k + 1 + e % rem;
            W[(int64_t)i * LP + j] -= (W[(int64_t)i * LP + k] / d) * W[(int64_t)k * LP + j];
        }
        __syncthreads();
    }
    if (sign < 0)
        for (int i = tid; i < m; i += 1024) Qp[(int64_t)i * LP + m - 1] = -Qp[(int64_t)i * LP + m - 1];
}

template <typename T>
__global__ void upper_to_colmajor_kernel(const double* __restrict__ Rf, int LP, int nr, int nc, T* __restrict__ R,
                                         int64_t ldr) {
    const int64_t total = (int64_t)nr * nc;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int j = (int)(e / nr), i = (int)(e - (int64_t)j * nr);
        R[i + j * ldr] = (i <= j) ? (T)Rf[(int64_t)i * LP + j] : T(0);
    }
}

__global__ __launch_bounds__(256) void shift_diag_kernel(double* __restrict__ G, int LP, int l, int64_t rows,
                                                         double u) {
    __shared__ double part[256];
    double t = 0.0;
    for (int i = threadIdx.x; i < l; i += 256) t += G[(int64_t)i * LP + i];
    part[threadIdx.x] = t;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
        __syncthreads();
    }
    const double sh = 11.0 * ((double)rows * l + (double)l * (l + 1)) * u * part[0];
    for (int i = threadIdx.x; i < l; i += 256) G[(int64_t)i * LP + i] += sh;
}

// Sum over the workgroup (kPowThreads threads); every thread gets the total.  `red` >= 17 doubles.
__device__ __forceinline__ double block_sum(double v, double* red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    __syncthreads();  // `red` may still be read from the previous call
    if (lane == 0) red[w] = v;
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int i = 0; i < kPowThreads / 64; ++i) t += red[i];
    return t;
}

// y = B x for symmetric B (row-major, ld LP): TPR consecutive threads share a row and stride the
// columns, so a row is read with unit stride; partial sums combined with lane shuffles.
template <bool LDSB>
__device__ __forceinline__ void sym_matvec(const double* __restrict__ B, int n, int LP, int tpr,
                                           const double* __restrict__ x, double* __restrict__ y) {
    const int sub = threadIdx.x % tpr;
    for (int r0 = threadIdx.x / tpr; r0 < n; r0 += kPowThreads / tpr) {
        const double* row = B + (int64_t)r0 * LP;
        double acc = 0.0;
        for (int c = sub; c < n; c += tpr) acc += row[c] * x[c];
        for (int o = tpr >> 1; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
        if (sub == 0) y[r0] = acc;
    }
}

template <typename T, bool LDSB>
__global__ __launch_bounds__(kPowThreads) void power_svd_kernel(const T* __restrict__ P, int64_t m, int n, int LP,
                                                                double* __restrict__ Bg, int dim, uint64_t seed,
                                                                int iters, T* __restrict__ Up, double* __restrict__ Vr,
                                                                double* __restrict__ S, int* __restrict__ kept,
                                                                const double* __restrict__ x0, int rsvd_mode) {
    extern __shared__ double lds[];
    double* x = lds;            // LP
    double* y = x + LP;         // LP
    double* coef = y + LP;      // LP
    double* red = coef + LP;    // 32
    double* B = LDSB ? red + 32 : Bg;
    const int tid = threadIdx.x;
    if (LDSB) {
        for (int e = tid; e < LP * LP; e += kPowThreads) B[e] = Bg[e];
        __syncthreads();
    }
    int tpr = 1;
    while (tpr < 16 && n * tpr * 2 <= kPowThreads) tpr *= 2;
    int k = dim;
    for (int i = 0; i < dim; ++i) {
        // x0 = N(0,1) Philox stream (seed + i), normalised (src/PM.cpp:15-22)
        double sq = 0.0;
        for (int c = tid; c < n; c += kPowThreads) {
            const double g = x0 ? x0[(int64_t)i * LP + c] : gauss_elem((uint64_t)c, seed + (uint64_t)i);
            x[c] = g;
            sq += g * g;
        }
        double nrm = sqrt(block_sum(sq, red));
        for (int c = tid; c < n; c += kPowThreads) x[c] /= nrm;
        __syncthreads();
        for (int it = 0; it < iters; ++it) {  // x0 = B x0 ; x0.normalize()  (src/PM.cpp:40-69)
            sym_matvec<LDSB>(B, n, LP, tpr, x, y);
            __syncthreads();
            sq = 0.0;
            for (int c = tid; c < n; c += kPowThreads) sq += y[c] * y[c];
            nrm = sqrt(block_sum(sq, red));
            for (int c = tid; c < n; c += kPowThreads) x[c] = y[c] / nrm;
            __syncthreads();
        }
        sq = 0.0;  // v = x0.normalized() (:72-73)
        for (int c = tid; c < n; c += kPowThreads) sq += x[c] * x[c];
        nrm = sqrt(block_sum(sq, red));
        for (int c = tid; c < n; c += kPowThreads) x[c] /= nrm;
        // coef_j = sigma_j (v_j . v): the deflations A_i = A - sum_j sigma_j u_j v_j^T applied to v
        {
            const int lane = tid & 63, w = tid >> 6;
            __syncthreads();
            for (int j = w; j < i; j += kPowThreads / 64) {
                double d = 0.0;
                for (int c = lane; c < n; c += 64)
                    d += Vr[rsvd_mode ? (int64_t)c * LP + j : (int64_t)j * LP + c] * x[c];
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) d += __shfl_xor(d, o);
                if (lane == 0) coef[j] = S[j] * d;
            }
            __syncthreads();
        }
        // w = A_i v (:76,79); written into column i of the U panel, normalised below
        sq = 0.0;
        for (int64_t r = tid; r < m; r += kPowThreads) {
            const T* row = P + r * LP;
            double acc = 0.0;
            for (int c = 0; c < n; ++c) acc += (double)row[c] * x[c];
            const T* urow = Up + r * LP;
            for (int j = 0; j < i; ++j) acc -= coef[j] * (double)urow[j];
            Up[r * LP + i] = (T)acc;
            sq += acc * acc;
        }
        const double sigma = sqrt(block_sum(sq, red));
        // SVD_class.hpp:198-208 stops at sigma < 1e-12; image_compression's SVD (rsvd_mode 2,
        // image_compression/src/SVD.cpp:44-51) has no stop -- it only ends here at sigma == 0, where
        // the reference would divide by zero (u = A v / sigma, PowerMethod.cpp:42)
        if (rsvd_mode == 2 ? !(sigma > 0.0) : sigma < 1e-12) {
            k = i;
            break;
        }
        sq = 0.0;
        for (int64_t r = tid; r < m; r += kPowThreads) {
            const double u = (double)Up[r * LP + i] / sigma;
            Up[r * LP + i] = (T)u;
            sq += u * u;
        }
        const double f = sigma * sigma * block_sum(sq, red);
        if (rsvd_mode == 2) {
            // image_compression recomputes B = A_{i+1}^T A_{i+1} after A_{i+1} = A_i - sigma u v^T
            // (SVD.cpp:47-48): B' = B - sigma (w v^T + v w^T) + sigma^2 (u.u) v v^T with w = A_i^T u,
            // A_i = P - sum_j sigma_j u_j v_j^T (the deflations so far)
            {
                const int lane = tid & 63, w = tid >> 6;
                for (int j = w; j < i; j += kPowThreads / 64) {  // coef_j = sigma_j (u_j . u)
                    double d = 0.0;
                    for (int64_t r = lane; r < m; r += 64) d += (double)Up[r * LP + j] * (double)Up[r * LP + i];
#pragma unroll
                    for (int o = 32; o > 0; o >>= 1) d += __shfl_xor(d, o);
                    if (lane == 0) coef[j] = S[j] * d;
                }
                __syncthreads();
            }
            for (int c = tid; c < n; c += kPowThreads) {  // y <- w
                double acc = 0.0;
                for (int64_t r = 0; r < m; ++r) acc += (double)P[r * LP + c] * (double)Up[r * LP + i];
                for (int j = 0; j < i; ++j) acc -= coef[j] * Vr[rsvd_mode ? (int64_t)c * LP + j : (int64_t)j * LP + c];
                y[c] = acc;
            }
            __syncthreads();
            for (int e = tid; e < n * n; e += kPowThreads) {
                const int r = e / n, c = e - r * n;
                B[(int64_t)r * LP + c] += f * (x[r] * x[c]) - sigma * (y[r] * x[c] + x[r] * y[c]);
            }
        } else {
            for (int e = tid; e < n * n; e += kPowThreads) {  // B -= update^T update (:212)
                const int r = e / n, c = e - r * n;
                B[(int64_t)r * LP + c] -= f * (x[r] * x[c]);
            }
        }
        for (int c = tid; c < n; c += kPowThreads)  // V_.row(i) = v (:214); rsvd mode: column i
            Vr[rsvd_mode ? (int64_t)c * LP + i : (int64_t)i * LP + c] = x[c];
        if (tid == 0) S[i] = sigma;
        __syncthreads();
    }
    if (rsvd_mode) {  // triplets past an early stop are zero (the reference drops them)
        for (int i = k; i < dim; ++i) {
            for (int64_t r = tid; r < m; r += kPowThreads) Up[r * LP + i] = T(0);
            for (int c = tid; c < n; c += kPowThreads) Vr[(int64_t)c * LP + i] = 0.0;
            if (tid == 0) S[i] = 0.0;
        }
    }
    if (tid == 0) *kept = k;
}

// rSVD with SVDMethod::Power (src/rSVD.cpp:106-113) in the coordinates of Q_B: B = R^T Q_B^T with
// R = Q_B^T B^T (LP x LP, R[i][j] = q_i . b_j).  The power iteration x <- B^T B x of the reference
// stays in span(Q_B) after its first product, so with x = Q_B y it is y <- (R R^T) y, sigma =
// |R^T y|, u = R^T y / sigma, and the deflation of B is R^T -= sigma u y^T.  This kernel writes
// P = R^T (row-major, the power kernel's "A"), Bpm = R R^T, and the start vectors
// X0s[i] = Q_B^T x0_i from Y0 = Q_B^T X0 (Y0[c][i] = q_c . x0_i).  One workgroup.
__global__ __launch_bounds__(1024) void power_prep_kernel(const double* __restrict__ R, const double* __restrict__ Y0,
                                                          int l, int LP, double* __restrict__ P,
                                                          double* __restrict__ X0s, double* __restrict__ Bpm) {
    const int tid = threadIdx.x;
    for (int e = tid; e < LP * LP; e += 1024) {
        const int i = e / LP, j = e - i * LP;
        const bool in = i < l && j < l;
        P[e] = in ? R[(int64_t)j * LP + i] : 0.0;
        X0s[e] = in ? Y0[(int64_t)j * LP + i] : 0.0;
        double acc = 0.0;
        if (in)
            for (int c = 0; c < l; ++c) acc += R[(int64_t)i * LP + c] * R[(int64_t)j * LP + c];
        Bpm[e] = acc;
    }
}

// X0 (rows x LP, row-major): X0[r][i] = N(0,1) Philox element r of stream (seed + i), i < l --
// the reference's random start vector of the i-th power-method triplet (src/PM.cpp:15-21).
template <typename T>
__global__ void power_start_kernel(T* __restrict__ X0, int64_t rows, int l, int LP, uint64_t seed) {
    const int64_t total = rows * LP;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = e / LP;
        const int i = (int)(e - r * LP);
        X0[e] = (i < l) ? (T)gauss_elem((uint64_t)r, seed + (uint64_t)i) : T(0);
    }
}

inline int grid_of(int64_t work) {
    int64_t g = (work + 255) / 256;
    return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

}  // namespace

template <typename T>
hipError_t launch_transpose_to_panel(const T* A, int64_t lda, int64_t m, int64_t n, int LP, T* P, hipStream_t s) {
    hipLaunchKernelGGL((transpose_to_panel_kernel<T>), dim3(grid_of(n * LP)), dim3(256), 0, s, A, lda, m, n, LP, P);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_unit_columns(T* P, int LP, int c0, int c1, hipStream_t s) {
    if (c1 <= c0) return hipSuccess;
    hipLaunchKernelGGL((unit_columns_kernel<T>), dim3((c1 - c0 + 255) / 256), dim3(256), 0, s, P, LP, c0, c1);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_qr_signs(const T* A, int64_t lda, int64_t m, int n, T* Qp, int LP, hipStream_t s) {
    if ((m < n ? m : n) > 512) return hipErrorInvalidValue;
    hipLaunchKernelGGL((qr_signs_kernel<T>), dim3(1), dim3(256), 0, s, A, lda, m, n, Qp, LP);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_trsm_rows(const T* In, int64_t rows, int k, int LP, const double* R, T* Out, const int* pred,
                            hipStream_t s) {
    if (LP % 16 || LP > 512 || k > LP) return hipErrorInvalidValue;
    const size_t lds = (size_t)(LP + 32) * 32 * sizeof(double);
    hipLaunchKernelGGL((trsm_rows_kernel<T>), dim3((unsigned)((rows + 255) / 256)), dim3(256), lds, s, In, rows, k, LP,
                       R, Out, pred);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_det_sign(T* Qp, int m, int LP, double* W, hipStream_t s) {
    if (m > LP) return hipErrorInvalidValue;
    hipLaunchKernelGGL((det_sign_kernel<T>), dim3(1), dim3(1024), 0, s, Qp, m, LP, W);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_upper_to_colmajor(const double* Rf, int LP, int nr, int nc, T* R, int64_t ldr, hipStream_t s) {
    hipLaunchKernelGGL((upper_to_colmajor_kernel<T>), dim3(grid_of((int64_t)nr * nc)), dim3(256), 0, s, Rf, LP, nr,
                       nc, R, ldr);
    return hipGetLastError();
}

hipError_t launch_shift_diag(double* G, int LP, int l, int64_t rows, double u, hipStream_t s) {
    hipLaunchKernelGGL(shift_diag_kernel, dim3(1), dim3(256), 0, s, G, LP, l, rows, u);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// SVD<Power> for large n (n > 512: B = A^T A no longer fits the one-workgroup kernel above).
//
// gram_cm_kernel: B = A^T A (n x n fp64, symmetric, stored in full) from the column-major A, one
// 64 x 64 tile of B per 256-thread workgroup (upper tiles only, mirrored), fp64 MFMA 16x16x4 with
// the k order permuted inside each 16-row step so a lane reads 4 consecutive rows of one column
// (32 contiguous bytes) per fragment.
namespace {

constexpr int kPgThreads = 256;  // four waves (power_grid_kernel's quarter sums assume it)

__global__ __launch_bounds__(256) void gram_cm_kernel(const double* __restrict__ A, int64_t lda, int64_t m, int64_t n,
                                                      double* __restrict__ B) {
    typedef Mfma<double> MD;
    const int nt = (int)((n + 63) / 64);
    // upper-triangular tile index -> (ti, tj), ti <= tj
    int t = blockIdx.x, ti = 0;
    while (t >= nt - ti) {
        t -= nt - ti;
        ++ti;
    }
    const int tj = ti + t;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 15, h = lane >> 4;
    const int64_t ca = (int64_t)ti * 64 + 16 * w + r;  // this lane's A-operand column
    f64x4 acc[4] = {MD::zero(), MD::zero(), MD::zero(), MD::zero()};
    for (int64_t k0 = 0; k0 < m; k0 += 16) {
        const int64_t kr = k0 + 4 * h;
        double a[4], b[4][4];
#pragma unroll
        for (int j = 0; j < 4; ++j) a[j] = (ca < n && kr + j < m) ? A[ca * lda + kr + j] : 0.0;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int64_t cb = (int64_t)tj * 64 + 16 * g + r;
#pragma unroll
            for (int j = 0; j < 4; ++j) b[g][j] = (cb < n && kr + j < m) ? A[cb * lda + kr + j] : 0.0;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g) acc[g] = MD::mma(a[j], b[g][j], acc[g]);
    }
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t row = (int64_t)ti * 64 + 16 * w + MD::row(h, j), col = (int64_t)tj * 64 + 16 * g + r;
            if (row < n && col < n) {
                B[row * n + col] = acc[g][j];
                B[col * n + row] = acc[g][j];
            }
        }
}

// Grid barrier of the power kernel below (counter form, MI355X_MICROARCH.md "Workgroup dispatch
// ... inter-workgroup visibility": drained stores -> workgroup barrier -> agent release -> relaxed
// counter add; relaxed poll -> agent acquire).  Bounded: a timeout sets the abort word.
__device__ bool pg_barrier(unsigned* sync, unsigned target) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    __shared__ int ok;
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int good = 1;
        long spins = 0;
        while (__hip_atomic_load(sync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(1);
            if ((++spins & 1023) == 0 &&
                (__hip_atomic_load(sync + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 || spins > (1l << 27))) {
                __hip_atomic_store(sync + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                good = 0;
                break;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        ok = good;
    }
    __syncthreads();
    return ok != 0;
}

__device__ __forceinline__ double pg_block_sum(double v, double* red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int i = 0; i < kPgThreads / 64; ++i) t += red[i];
    return t;
}

// Row range of workgroup g out of G for `rows` rows: the reference's split (src/PM.cpp:31-35).
__device__ __forceinline__ void pg_rows(int64_t rows, int G, int g, int64_t& r0, int64_t& r1) {
    const int64_t per = rows / G, rem = rows % G;
    r0 = g * per + (g < rem ? g : rem);
    r1 = r0 + per + (g < rem ? 1 : 0);
}

// The power method with deflation (SVD_class.hpp:183-219, src/PM.cpp:4-81) on a persistent grid:
// workgroup g owns rows pg_rows(n, G, g) of B for the matvecs x <- B x (the reference's MPI row
// partition of B, PM.cpp:31-35, with the Gatherv + Bcast of each iterate replaced by one grid
// barrier: every workgroup reads the whole iterate from the L2) and rows pg_rows(m, G, g) of A for
// u = A_i v.  The iterate is normalised on the fly: y_{t+1} = B y_t / |y_t|.  A_i = A - sum_j
// sigma_j u_j v_j^T is applied implicitly (the coefficients sigma_j (v_j . v) are reduced over the
// grid); B is deflated explicitly, B -= sigma^2 (u.u) v v^T (:212).  Outputs: U (m x dim, ldu),
// V (n x dim, ldv, v_i in column i), S (dim), *kept.  Work: Y (2 n), part (G (dim + 2)), sync (8).
// General layouts (PowerGridIO): A(r, c) = A[r ar + c ac], B row r at B + r ldb, U(r, i) = U[r + i ldu],
// V(c, i) = V[c + i ldv]; x0 (optional): start vector i is x0[i ldx0 + c] instead of the Philox
// stream; zero_tail: the triplets past an early stop are written as zeros (the rSVD's layout).
struct PowerGridIO {
    int64_t ar, ac, ldb, ldu, ldv, ldx0;
    const double* x0;
    int zero_tail;
};

__global__ __launch_bounds__(kPgThreads) void power_grid_kernel(const double* __restrict__ A, PowerGridIO io, int64_t m,
                                                                int64_t n, double* __restrict__ B, int dim, uint64_t seed,
                                                                int iters, double* __restrict__ U,
                                                                double* __restrict__ V,
                                                                double* __restrict__ S, double* __restrict__ Y,
                                                                double* __restrict__ part, unsigned* __restrict__ sync,
                                                                int* __restrict__ kept, int* __restrict__ tmo) {
    const int64_t ldu = io.ldu, ldv = io.ldv, ldb = io.ldb;
    __shared__ double red[kPgThreads / 64];
    __shared__ double coef_s[64];
    __shared__ double qsum[kPgThreads / 64][64];
    const int G = gridDim.x, g = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    int64_t b0, b1, a0, a1;
    pg_rows(n, G, g, b0, b1);
    pg_rows(m, G, g, a0, a1);
    const int P = dim + 2;  // partial slots per workgroup
    unsigned bar = 0;
    auto barrier = [&]() -> bool {
        if (pg_barrier(sync, (unsigned)G * ++bar)) return true;
        if (g == 0 && tid == 0) atomicOr(tmo, 1);
        return false;
    };
    // Fixed-order sum of the workgroups' partials in `slot`, called by every thread: each wave loads the
    // G partials across its lanes (all in flight) and folds them by a butterfly, so every lane of every
    // workgroup gets the same bits (a serial loop over G cross-XCD loads per thread cost ~G L2-miss
    // latencies per iteration: ADVICE r05, l = 2048 took 19 s).
    auto grid_sum = [&](int slot) {
        double t = 0.0;
        for (int q = lane; q < G; q += 64) t += part[(size_t)q * P + slot];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
        return t;
    };
    double* y0 = Y;
    double* y1 = Y + n;
    int k = dim;
    for (int i = 0; i < dim; ++i) {
        // x0 = N(0,1) Philox stream (seed + i) (src/PM.cpp:15-22), or the given start; |x0| over the grid
        double sq = 0.0;
        for (int64_t c = b0 + tid; c < b1; c += kPgThreads) {
            const double v = io.x0 ? io.x0[(int64_t)i * io.ldx0 + c] : gauss_elem((uint64_t)c, seed + (uint64_t)i);
            y0[c] = v;
            sq += v * v;
        }
        sq = pg_block_sum(sq, red);
        if (tid == 0) part[(size_t)g * P + dim] = sq;
        if (!barrier()) return;
        double nrm = sqrt(grid_sum(dim));
        // s iterations x <- B x / |B x| (:40-69): y_{t+1} = B (y_t / |y_t|)
        for (int it = 0; it < iters; ++it) {
            const double inv = 1.0 / nrm;
            double sq2 = 0.0;
            for (int64_t row = b0 + w; row < b1; row += kPgThreads / 64) {
                const double* br = B + row * ldb;
                double a4[4] = {0.0, 0.0, 0.0, 0.0};  // four loads in flight per lane
                int64_t c = lane;
                for (; c + 192 < n; c += 256) {
#pragma unroll
                    for (int u = 0; u < 4; ++u) a4[u] += br[c + 64 * u] * y0[c + 64 * u];
                }
                if (c < n) a4[0] += br[c] * y0[c];  // (at most three 64-column steps remain)
                if (c + 64 < n) a4[1] += br[c + 64] * y0[c + 64];
                if (c + 128 < n) a4[2] += br[c + 128] * y0[c + 128];
                double acc = (a4[0] + a4[1]) + (a4[2] + a4[3]);
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
                acc *= inv;
                if (lane == 0) y1[row] = acc;
                sq2 += (lane == 0) ? acc * acc : 0.0;
            }
            sq2 = pg_block_sum(sq2, red);
            if (tid == 0) part[(size_t)g * P + dim + ((it + 1) & 1)] = sq2;
            if (!barrier()) return;
            nrm = sqrt(grid_sum(dim + ((it + 1) & 1)));
            double* t = y0;
            y0 = y1;
            y1 = t;
        }
        // v = x0.normalized() (:72-73); coef_j = sigma_j (v_j . v) for the implicit deflation of A
        // (thread (quarter w, slot lane): its quarter of this workgroup's rows, the quarters summed in
        // order through LDS -- all 64 slots of a chunk at once instead of one wave-wide dot per slot)
        const double vs = 1.0 / nrm;
        for (int j0 = 0; j0 < i; j0 += 64) {
            const int jn = (i - j0) < 64 ? (i - j0) : 64;
            double d = 0.0;
            if (lane < jn) {
                const double* vj = V + (size_t)(j0 + lane) * ldv;
                for (int64_t c = b0 + w; c < b1; c += kPgThreads / 64) d += vj[c] * y0[c];
            }
            __syncthreads();
            qsum[w][lane] = d;
            __syncthreads();
            if (tid < jn) part[(size_t)g * P + j0 + tid] = ((qsum[0][tid] + qsum[1][tid]) + (qsum[2][tid] + qsum[3][tid])) * vs;
        }
        if (!barrier()) return;
        // u = A_i v = A v - sum_j coef_j u_j over this workgroup's rows of A; |u| over the grid.
        // A v: row-major A (ac = 1: the rSVD's R^T, ar = l) takes a wave per row, lanes along the
        // row and a shuffle sum (a thread per row left l / 256 threads of a workgroup
        // busy on serial l-long dots); otherwise (column-major A, ar = 1) a thread per row, whose
        // loads are coalesced down each column.
        if (io.ac == 1) {
            for (int64_t row = a0 + w; row < a1; row += kPgThreads / 64) {
                const double* arow = A + row * io.ar;
                double acc = 0.0;
                for (int64_t c = lane; c < n; c += 64) acc += arow[c] * (y0[c] * vs);
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
                if (lane == 0) U[row + (size_t)i * ldu] = acc;
            }
        } else {
            for (int64_t row = a0 + tid; row < a1; row += kPgThreads) {
                double acc = 0.0;
                for (int64_t c = 0; c < n; ++c) acc += A[row * io.ar + c * io.ac] * (y0[c] * vs);
                U[row + (size_t)i * ldu] = acc;
            }
        }
        double su = 0.0;
        for (int j0 = 0; j0 < i; j0 += 64) {  // coefficients in chunks of 64 (LDS)
            const int jn = (i - j0) < 64 ? (i - j0) : 64;
            // coefficient j0 + lane summed over the workgroups: quarter w takes every fourth partial
            double cq = 0.0;
            if (lane < jn) {
#pragma unroll 8
                for (int q = w; q < G; q += kPgThreads / 64) cq += part[(size_t)q * P + j0 + lane];
            }
            __syncthreads();  // (also orders the A v stores before the reads below)
            qsum[w][lane] = cq;
            __syncthreads();
            if (tid < jn) coef_s[tid] = S[j0 + tid] * ((qsum[0][tid] + qsum[1][tid]) + (qsum[2][tid] + qsum[3][tid]));
            __syncthreads();
            for (int64_t row = a0 + tid; row < a1; row += kPgThreads) {
                double acc = U[row + (size_t)i * ldu];
                for (int jj = 0; jj < jn; ++jj) acc -= coef_s[jj] * U[row + (size_t)(j0 + jj) * ldu];
                U[row + (size_t)i * ldu] = acc;
            }
        }
        __syncthreads();
        for (int64_t row = a0 + tid; row < a1; row += kPgThreads) {
            const double u = U[row + (size_t)i * ldu];
            su += u * u;
        }
        su = pg_block_sum(su, red);
        if (tid == 0) part[(size_t)g * P + dim] = su;
        if (!barrier()) return;
        const double sigma = sqrt(grid_sum(dim));
        if (sigma < 1e-12) {  // SVD_class.hpp:198-208
            k = i;
            break;
        }
        // u /= sigma; B -= sigma^2 (u.u) v v^T (:210-212) with u.u = 1; V(:, i) = v; S[i] = sigma
        for (int64_t row = a0 + tid; row < a1; row += kPgThreads) U[row + (size_t)i * ldu] /= sigma;
        const double f = sigma * sigma * vs * vs;  // sigma^2 (u.u) with u.u = 1, v = y0 vs
        for (int64_t row = b0 + w; row < b1; row += kPgThreads / 64) {
            const double xr = y0[row];
            double* br = B + row * ldb;
            for (int64_t c = lane; c < n; c += 64) br[c] -= f * xr * y0[c];
        }
        for (int64_t c = b0 + tid; c < b1; c += kPgThreads) V[c + (size_t)i * ldv] = y0[c] * vs;
        if (g == 0 && tid == 0) S[i] = sigma;
        if (!barrier()) return;
    }
    if (io.zero_tail) {  // (rSVD layout) triplets past an early stop are zero, as the one-workgroup kernel's
        for (int i = k; i < dim; ++i) {
            for (int64_t row = a0 + tid; row < a1; row += kPgThreads) U[row + (size_t)i * ldu] = 0.0;
            for (int64_t c = b0 + tid; c < b1; c += kPgThreads) V[c + (size_t)i * ldv] = 0.0;
            if (g == 0 && tid == 0) S[i] = 0.0;
        }
    }
    if (g == 0 && tid == 0) *kept = k;
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// SVD<ParallelJacobi> with the reference's own iteration (SVD_class.hpp:223-333,
// JacobiOperations.cpp:120-203): two-sided Jacobi on the d x d triangle W with, per sweep, the
// list of pairs whose weight W(p,q)^2 + W(q,p)^2 exceeds max(1e-12, 1e-12 maxDiag) (:253-254,
// 266-282), sorted by decreasing weight (ties by decreasing p, then q: std::greater on the tuple,
// :286) and applied IN THAT ORDER -- each rotation after the previous one (the _par helpers only
// parallelise inside a rotation), skipping blocks already diagonal to maxDiag eps (:89-103); the
// right rotation is dropped when deno = 2|m01| < 1e-10 (:168).  This is a sequential algorithm,
// so one workgroup runs it: rows / columns of a rotation are updated in parallel, W, Jl, Jr live
// in global memory (L2), the pair list is built by an atomic counter and bitonic-sorted.  tri > 0
// (< 0): W is upper (lower) triangular, the other triangle read as exact zeros.  Jl / Jr
// accumulate the left / right rotations (U = Q_U Jl, V = Q_V Jr are formed afterwards); then the
// sign fix (:307-312) and the selection sort (:314-330).  W(p, q) = Win[p * sp + q * sq].
namespace {

constexpr int kPjThreads = 1024;

struct PjEntry {
    double w;
    int key;  // p * 65536 + q
    int pad;
};

__device__ __forceinline__ bool pj_before(const PjEntry& a, const PjEntry& b) {  // descending (w, p, q)
    return a.w > b.w || (a.w == b.w && a.key > b.key);
}

template <typename TI>
__global__ __launch_bounds__(kPjThreads) void pjacobi_ref_kernel(const TI* __restrict__ Win, int64_t sp, int64_t sq,
                                                                 int tri, int d, int LP, double* __restrict__ W,
                                                                 double* __restrict__ Jl, double* __restrict__ Jr,
                                                                 double* __restrict__ S, PjEntry* __restrict__ list,
                                                                 int* __restrict__ info) {
    __shared__ double rot[4];
    __shared__ double maxd_s;
    __shared__ int cnt_s, skip_s[2], flag_s;  // skip_s double-buffered: thread 0 writes the next
                                              // one while slower waves still read this one
    const int tid = threadIdx.x;
    for (int e = tid; e < d * d; e += kPjThreads) {
        const int p = e / d, q = e % d;
        const bool zero = (tri > 0 && p > q) || (tri < 0 && p < q);  // the triangle's exact zeros
        W[(int64_t)p * LP + q] = zero ? 0.0 : (double)Win[(int64_t)p * sp + (int64_t)q * sq];
        Jl[(int64_t)p * LP + q] = (p == q) ? 1.0 : 0.0;
        Jr[(int64_t)p * LP + q] = (p == q) ? 1.0 : 0.0;
    }
    __syncthreads();
    if (tid == 0) {
        double md = 0.0;
        for (int i = 0; i < d; ++i) md = fmax(md, fabs(W[(int64_t)i * LP + i]));
        maxd_s = md;
    }
    __syncthreads();
    const double eps = 2.220446049250313e-16;
    int sweeps = 0;
    for (; sweeps < 200; ++sweeps) {
        // weights above the threshold (:266-282)
        if (tid == 0) cnt_s = 0;
        __syncthreads();
        const double threshold = fmax(1e-12, 1e-12 * maxd_s);
        for (int e = tid; e < d * d; e += kPjThreads) {
            const int p = e / d, q = e % d;
            if (q < p) {
                const double a = W[(int64_t)p * LP + q], b = W[(int64_t)q * LP + p];
                const double wgt = a * a + b * b;
                if (wgt > threshold) {
                    const int at = atomicAdd(&cnt_s, 1);
                    list[at].w = wgt;
                    list[at].key = p * 65536 + q;
                }
            }
        }
        __syncthreads();
        const int cnt = cnt_s;
        if (cnt == 0) break;
        // bitonic sort of the first npow2 entries (padding w = -1 sorts last)
        int np2 = 1;
        while (np2 < cnt) np2 <<= 1;
        for (int e = cnt + tid; e < np2; e += kPjThreads) {
            list[e].w = -1.0;
            list[e].key = -1;
        }
        __syncthreads();
        for (int kk = 2; kk <= np2; kk <<= 1)
            for (int j = kk >> 1; j > 0; j >>= 1) {
                for (int e = tid; e < np2; e += kPjThreads) {
                    const int x = e ^ j;
                    if (x > e) {
                        const PjEntry a = list[e], b = list[x];
                        const bool up = (e & kk) == 0;  // this run sorted "descending-first"
                        if (up ? pj_before(b, a) : pj_before(a, b)) {
                            list[e] = b;
                            list[x] = a;
                        }
                    }
                }
                __syncthreads();
            }
        // the rotations, in order (:288-303)
        for (int e = 0; e < cnt; ++e) {
            const int key = list[e].key, p = key >> 16, q = key & 0xFFFF;
            if (tid == 0) {
                const double m00 = W[(int64_t)p * LP + p], m01 = W[(int64_t)p * LP + q];
                const double m10 = W[(int64_t)q * LP + p], m11 = W[(int64_t)q * LP + q];
                const double md = maxd_s;
                const int skip = (fabs(m01) < md * eps && fabs(m10) < md * eps) ? 1 : 0;  // :96-101
                skip_s[e & 1] = skip;
                if (!skip) {  // real_2x2_jacobi_svd_par (:140-202)
                    const double t = m00 + m11, dd = m10 - m01;
                    double c1 = 1.0, s1 = 0.0;
                    if (dd != 0.0) {
                        const double u = t / dd, tmp = sqrt(1.0 + u * u);
                        s1 = 1.0 / tmp;
                        c1 = u / tmp;
                    }
                    const double n00 = c1 * m00 + s1 * m10, n01 = c1 * m01 + s1 * m11;
                    const double n11 = -s1 * m01 + c1 * m11;
                    const double deno = 2.0 * fabs(n01);
                    double cr = 1.0, sr = 0.0;
                    if (deno >= 1e-10) {
                        const double tau = (n00 - n11) / deno, w = sqrt(tau * tau + 1.0);
                        const double t2 = tau > 0.0 ? 1.0 / (tau + w) : 1.0 / (tau - w);
                        const double segno = t2 > 0.0 ? 1.0 : -1.0;
                        const double nn = 1.0 / sqrt(t2 * t2 + 1.0);
                        sr = -segno * (n01 / fabs(n01)) * fabs(t2) * nn;
                        cr = nn;
                    }
                    rot[0] = c1 * cr + s1 * sr;     // c_left
                    rot[1] = c1 * (-sr) + s1 * cr;  // s_left
                    rot[2] = cr;
                    rot[3] = sr;
                }
            }
            __syncthreads();
            if (skip_s[e & 1]) continue;  // uniform
            const double cl = rot[0], sl = rot[1], cr = rot[2], sr = rot[3];
            for (int i = tid; i < d; i += kPjThreads) {
                // applyOnTheLeft_par(W, p, q, cl, sl) (:120-128)
                const double xi = W[(int64_t)p * LP + i], yi = W[(int64_t)q * LP + i];
                W[(int64_t)p * LP + i] = cl * xi + sl * yi;
                W[(int64_t)q * LP + i] = -sl * xi + cl * yi;
                // applyOnTheRight_par(U_, p, q, cl, -sl) (:130-138)
                const double ui = Jl[(int64_t)i * LP + p], vi = Jl[(int64_t)i * LP + q];
                Jl[(int64_t)i * LP + p] = cl * ui + sl * vi;
                Jl[(int64_t)i * LP + q] = -sl * ui + cl * vi;
            }
            __syncthreads();
            for (int i = tid; i < d; i += kPjThreads) {
                // applyOnTheRight_par(W, p, q, cr, sr); applyOnTheRight_par(V_, p, q, cr, sr)
                const double xi = W[(int64_t)i * LP + p], yi = W[(int64_t)i * LP + q];
                W[(int64_t)i * LP + p] = cr * xi - sr * yi;
                W[(int64_t)i * LP + q] = sr * xi + cr * yi;
                const double ui = Jr[(int64_t)i * LP + p], vi = Jr[(int64_t)i * LP + q];
                Jr[(int64_t)i * LP + p] = cr * ui - sr * vi;
                Jr[(int64_t)i * LP + q] = sr * ui + cr * vi;
            }
            __syncthreads();
            if (tid == 0)  // :298-299
                maxd_s = fmax(maxd_s, fmax(fabs(W[(int64_t)p * LP + p]), fabs(W[(int64_t)q * LP + q])));
        }
        __syncthreads();
    }
    // S = |diag|, negative diagonal flips the U column (:307-312)
    for (int i = tid; i < d; i += kPjThreads) {
        const double a = W[(int64_t)i * LP + i];
        S[i] = fabs(a);
        if (a < 0.0)
            for (int r = 0; r < d; ++r) Jl[(int64_t)r * LP + i] = -Jl[(int64_t)r * LP + i];
    }
    __syncthreads();
    // selection sort, first maximum (:314-330)
    for (int i = 0; i < d; ++i) {
        if (tid == 0) {
            int pos = i;
            double mx = S[i];
            for (int t = i + 1; t < d; ++t)
                if (S[t] > mx) {
                    mx = S[t];
                    pos = t;
                }
            flag_s = (mx == 0.0) ? -1 : pos;
        }
        __syncthreads();
        const int pos = flag_s;
        if (pos < 0) break;
        if (pos != i) {
            if (tid == 0) {
                const double ts = S[i];
                S[i] = S[pos];
                S[pos] = ts;
            }
            for (int r = tid; r < d; r += kPjThreads) {
                double x = Jl[(int64_t)r * LP + pos];
                Jl[(int64_t)r * LP + pos] = Jl[(int64_t)r * LP + i];
                Jl[(int64_t)r * LP + i] = x;
                x = Jr[(int64_t)r * LP + pos];
                Jr[(int64_t)r * LP + pos] = Jr[(int64_t)r * LP + i];
                Jr[(int64_t)r * LP + i] = x;
            }
        }
        __syncthreads();
    }
    if (tid == 0) info[0] = sweeps;
}

}  // namespace

size_t pjacobi_ref_list_bytes(int d) {
    int64_t pairs = (int64_t)d * (d - 1) / 2, np2 = 1;
    while (np2 < pairs) np2 <<= 1;
    return (size_t)np2 * sizeof(PjEntry);
}

template <typename TI>
hipError_t launch_pjacobi_ref(const TI* Win, int64_t sp, int64_t sq, int tri, int d, int LP, double* W, double* Jl,
                              double* Jr, double* S, void* list, int* info, hipStream_t s) {
    hipLaunchKernelGGL(pjacobi_ref_kernel<TI>, dim3(1), dim3(kPjThreads), 0, s, Win, sp, sq, tri, d, LP, W, Jl, Jr, S,
                       reinterpret_cast<PjEntry*>(list), info);
    return hipGetLastError();
}
template hipError_t launch_pjacobi_ref<double>(const double*, int64_t, int64_t, int, int, int, double*, double*, double*,
                                               double*, void*, int*, hipStream_t);
template hipError_t launch_pjacobi_ref<float>(const float*, int64_t, int64_t, int, int, int, double*, double*, double*,
                                              double*, void*, int*, hipStream_t);

hipError_t launch_gram_colmajor(const double* A, int64_t lda, int64_t m, int64_t n, double* B, hipStream_t s) {
    const int64_t nt = (n + 63) / 64;
    hipLaunchKernelGGL(gram_cm_kernel, dim3((unsigned)(nt * (nt + 1) / 2)), dim3(256), 0, s, A, lda, m, n, B);
    return hipGetLastError();
}

int power_grid_size(int64_t n) {
    int64_t g = (n + 15) / 16;
    return (int)(g > 256 ? 256 : (g < 1 ? 1 : g));
}

hipError_t launch_power_grid(const double* A, int64_t lda, int64_t m, int64_t n, double* B, int dim, uint64_t seed,
                             int iters, double* U, int64_t ldu, double* V, int64_t ldv, double* S, double* Y,
                             double* part, unsigned* sync, int* kept, int* tmo, hipStream_t s) {
    hipError_t e = hipMemsetAsync(sync, 0, 8 * sizeof(unsigned), s);
    if (e != hipSuccess) return e;
    const PowerGridIO io{1, lda, n, ldu, ldv, 0, nullptr, 0};
    return launch_coresident(power_grid_kernel, dim3(power_grid_size(n)), dim3(kPgThreads), 0, s, A, io, m, n, B, dim,
                             seed, iters, U, V, S, Y, part, sync, kept, tmo);
}

hipError_t launch_power_grid_rsvd(const double* R, int l, double* B, const double* X0s, int iters, double* Up,
                                  double* Vc, double* S, double* Y, double* part, unsigned* sync, int* kept, int* tmo,
                                  hipStream_t s) {
    hipError_t e = hipMemsetAsync(sync, 0, 8 * sizeof(unsigned), s);
    if (e != hipSuccess) return e;
    // P = R^T (P(r, c) = R[c + r l]); B, U_p, V_c, X0s all l x l with ld l
    const PowerGridIO io{l, 1, l, l, l, l, X0s, 1};
    return launch_coresident(power_grid_kernel, dim3(power_grid_size(l)), dim3(kPgThreads), 0, s, R, io, (int64_t)l,
                             (int64_t)l, B, l, (uint64_t)0, iters, Up, Vc, S, Y, part, sync, kept, tmo);
}

int power_iterations(int64_t n) {
    // s = ceil(log(4 log(2 n / delta) / (eps delta)) / (2 lambda)), src/PM.cpp:25-28
    const double eps = 1.e-10, delta = 0.05, lambda = 0.1;
    return (int)ceil(log(4.0 * log(2.0 * (double)n / delta) / (eps * delta)) / (2.0 * lambda));
}

hipError_t launch_power_svd(const double* P, int64_t m, int n, int LP, double* B, int dim, uint64_t seed, int iters,
                            double* Up, double* Vr, double* S, int* kept, hipStream_t s, const double* x0,
                            int rsvd_mode) {
    if (n > LP || LP > 512 || dim > n) return hipErrorInvalidValue;
    const size_t small = (size_t)(3 * LP + 32) * sizeof(double);
    if (LP <= 128) {
        const size_t lds = small + (size_t)LP * LP * sizeof(double);
        hipLaunchKernelGGL((power_svd_kernel<double, true>), dim3(1), dim3(kPowThreads), lds, s, P, m, n, LP, B, dim,
                           seed, iters, Up, Vr, S, kept, x0, rsvd_mode);
    } else {
        hipLaunchKernelGGL((power_svd_kernel<double, false>), dim3(1), dim3(kPowThreads), small, s, P, m, n, LP, B,
                           dim, seed, iters, Up, Vr, S, kept, x0, rsvd_mode);
    }
    return hipGetLastError();
}

hipError_t launch_power_prep(const double* R, const double* Y0, int l, int LP, double* P, double* X0s, double* Bpm,
                             hipStream_t s) {
    hipLaunchKernelGGL(power_prep_kernel, dim3(1), dim3(1024), 0, s, R, Y0, l, LP, P, X0s, Bpm);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_power_start(T* X0, int64_t rows, int l, int LP, uint64_t seed, hipStream_t s) {
    hipLaunchKernelGGL((power_start_kernel<T>), dim3(grid_of(rows * LP)), dim3(256), 0, s, X0, rows, l, LP, seed);
    return hipGetLastError();
}

uint64_t power_seed(uint64_t seed) { return seed ^ 0x504F574552ull; }

#define RSVD_INST(T)                                                                                         \
    template hipError_t launch_transpose_to_panel<T>(const T*, int64_t, int64_t, int64_t, int, T*, hipStream_t); \
    template hipError_t launch_upper_to_colmajor<T>(const double*, int, int, int, T*, int64_t, hipStream_t); \
    template hipError_t launch_unit_columns<T>(T*, int, int, int, hipStream_t);                               \
    template hipError_t launch_det_sign<T>(T*, int, int, double*, hipStream_t);                               \
    template hipError_t launch_power_start<T>(T*, int64_t, int, int, uint64_t, hipStream_t);                   \
    template hipError_t launch_trsm_rows<T>(const T*, int64_t, int, int, const double*, T*, const int*, hipStream_t); \
    template hipError_t launch_qr_signs<T>(const T*, int64_t, int64_t, int, T*, int, hipStream_t);
RSVD_INST(float)
RSVD_INST(double)
#undef RSVD_INST

}  // namespace rsvd
