// gemm.hip -- column-major dense building blocks for the QR() / SVD<> drop-ins past the 512-column
// panels of the rSVD engine (dense_big.cpp): a general GEMM on the MFMA, the Givens sign rule and
// the determinant sign of a square Q for any size.
//
//   C = alpha op(A) op(B) + beta C     (fp64 on v_mfma_f64_16x16x4f64, fp32 on v_mfma_f32_16x16x4f32)
//
// 64 x 64 output tile per 256-thread workgroup (4 waves, 32 x 32 each = 2 x 2 MFMA tiles), the
// 64 x 16 slices of op(A) and op(B) staged through LDS k-major (As[k][i], Bs[k][j]: the MFMA operand
// of lane (r, h) at k-step kk is As[4 kk + h][row r], one bank-conflict-free read).  Global loads
// run along the contiguous dimension of each operand (i for A N, k for A T / B N, j for B T).
// Sizes are arbitrary (edges zero-filled); beta == 0 never reads C.
#include <algorithm>
#include <utility>

#include "common.hpp"
#include "dense.hpp"

namespace rsvd {

namespace {

constexpr int GT = 64, GK = 16, GP = GT + 4;  // tile, k slice, LDS pitch

template <typename T>
__global__ __launch_bounds__(256) void gemm_kernel(int ta, int tb, int64_t M, int64_t N, int64_t K, T alpha,
                                                   const T* __restrict__ A, int64_t lda, const T* __restrict__ B,
                                                   int64_t ldb, T beta, T* __restrict__ C, int64_t ldc) {
    typedef Mfma<T> MM;
    __shared__ T As[GK][GP];
    __shared__ T Bs[GK][GP];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 15, h = lane >> 4;
    const int64_t i0 = (int64_t)blockIdx.x * GT, j0 = (int64_t)blockIdx.y * GT;
    const int wi = (w >> 1) * 32, wj = (w & 1) * 32;
    typename MM::acc_t acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = MM::zero();
    for (int64_t k0 = 0; k0 < K; k0 += GK) {
        // op(A)(i, k): N -> A[i + k lda] (threads along i), T -> A[k + i lda] (threads along k)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = tid + 256 * u;
            int ii, kk;
            if (!ta) { ii = e & 63; kk = e >> 6; } else { kk = e & 15; ii = e >> 4; }
            const int64_t gi = i0 + ii, gk = k0 + kk;
            T v = T(0);
            if (gi < M && gk < K) v = ta ? A[gk + gi * lda] : A[gi + gk * lda];
            As[kk][ii] = v;
        }
        // op(B)(k, j): N -> B[k + j ldb] (threads along k), T -> B[j + k ldb] (threads along j)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = tid + 256 * u;
            int jj, kk;
            if (!tb) { kk = e & 15; jj = e >> 4; } else { jj = e & 63; kk = e >> 6; }
            const int64_t gj = j0 + jj, gk = k0 + kk;
            T v = T(0);
            if (gj < N && gk < K) v = tb ? B[gj + gk * ldb] : B[gk + gj * ldb];
            Bs[kk][jj] = v;
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < GK / 4; ++kk) {
            const T a0 = As[4 * kk + h][wi + r], a1 = As[4 * kk + h][wi + 16 + r];
            const T b0 = Bs[4 * kk + h][wj + r], b1 = Bs[4 * kk + h][wj + 16 + r];
            acc[0][0] = MM::mma(a0, b0, acc[0][0]);
            acc[0][1] = MM::mma(a0, b1, acc[0][1]);
            acc[1][0] = MM::mma(a1, b0, acc[1][0]);
            acc[1][1] = MM::mma(a1, b1, acc[1][1]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int64_t gi = i0 + wi + 16 * a + MM::row(h, q), gj = j0 + wj + 16 * b + r;
                if (gi < M && gj < N) {
                    T* c = C + gi + gj * ldc;
                    const T v = alpha * acc[a][b][q];
                    *c = (beta == T(0)) ? v : v + beta * *c;
                }
            }
}

// The Givens sign rule (src/QR.cpp:31-39) on a column-major Q (m x kq): the leading columns of A
// whose sub-diagonal is already zero get no rotation, so R(j, j) keeps the sign of A(j, j); flip
// those columns of Q where A(j, j) < 0 (R = Q^T A is formed afterwards).
template <typename T>
__global__ __launch_bounds__(256) void qr_signs_cm_kernel(const T* __restrict__ A, int64_t lda, int64_t m, int64_t n,
                                                          T* __restrict__ Q, int64_t ldq) {
    __shared__ int run;
    const int64_t kmin = m < n ? m : n;
    if (threadIdx.x == 0) run = (int)kmin;
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int64_t j = w; j < kmin; j += 4) {
        if (j >= run) break;
        int any = 0;
        for (int64_t i = j + 1 + lane; i < m; i += 64) any |= A[i + j * lda] != T(0);
        any = __any(any);
        if (lane == 0 && any) atomicMin(&run, (int)j);
    }
    __syncthreads();
    const int rn = run;
    for (int j = 0; j < rn; ++j) {
        if (!(A[j + j * lda] < T(0))) continue;
        for (int64_t i = threadIdx.x; i < m; i += 256) Q[i + j * ldq] = -Q[i + j * ldq];
    }
}

// One step k of Gaussian elimination with partial pivoting on the m x m fp64 W (column-major,
// double-buffered: Win -> Wout, rows >= k), tracking sign(det): every workgroup finds the same
// pivot (max |W(i, k)|, i >= k, lowest index on ties), then rewrites its rows i > k of the trailing
// block from the swapped source row.  sgn[0] accumulates the sign (workgroup 0, thread 0).
__global__ __launch_bounds__(256) void lu_sign_step_kernel(const double* __restrict__ Win, double* __restrict__ Wout,
                                                           int m, int k, int* __restrict__ sgn) {
    __shared__ double bv[4];
    __shared__ int bi[4];
    __shared__ int piv;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    double v = -1.0;
    int vi = k;
    for (int i = k + tid; i < m; i += 256) {
        const double a = fabs(Win[i + (int64_t)k * m]);
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
        for (int t = 1; t < 4; ++t)
            if (bv[t] > b || (bv[t] == b && bi[t] < p)) {
                b = bv[t];
                p = bi[t];
            }
        piv = p;
        if (blockIdx.x == 0) {
            const double d = Win[p + (int64_t)k * m];
            int s = sgn[0];
            if (p != k) s = -s;
            if (d < 0.0) s = -s;
            if (!(d != 0.0)) s = 0;  // singular: no sign (Q is orthonormal, so this does not happen)
            sgn[0] = s;
        }
    }
    __syncthreads();
    const int p = piv;
    const double d = Win[p + (int64_t)k * m];
    // rows k+1 .. m-1 of the new W: row i comes from source row (i == p ? k : i)
    const int rem = m - k - 1;
    const int64_t tot = (int64_t)rem * rem;
    for (int64_t e = blockIdx.x * 256 + tid; e < tot; e += (int64_t)gridDim.x * 256) {
        const int j = k + 1 + (int)(e / rem), i = k + 1 + (int)(e % rem);  // i fastest: coalesced columns
        const int src = (i == p) ? k : i;
        const double f = (d != 0.0) ? Win[src + (int64_t)k * m] / d : 0.0;
        Wout[i + (int64_t)j * m] = Win[src + (int64_t)j * m] - f * Win[p + (int64_t)j * m];
    }
}

template <typename T>
__global__ void to_f64_square_kernel(const T* __restrict__ Q, int64_t ldq, int m, double* __restrict__ W) {
    const int64_t tot = (int64_t)m * m;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = e % m, j = e / m;
        W[e] = (double)Q[i + j * ldq];
    }
}

template <typename T>
__global__ void flip_last_if_negative_kernel(T* __restrict__ Q, int64_t ldq, int m, int col, const int* __restrict__ sgn) {
    if (sgn[0] >= 0) return;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
        Q[i + (int64_t)col * ldq] = -Q[i + (int64_t)col * ldq];
}

template <typename T>
__global__ void identity_cols_kernel(T* __restrict__ Y, int64_t ldy, int64_t rows, int cols, int64_t e0) {
    const int64_t tot = rows * cols;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = e % rows, j = e / rows;
        Y[i + j * ldy] = (i == e0 + j) ? T(1) : T(0);
    }
}

template <typename T>
__global__ void zero_below_kernel(T* __restrict__ R, int64_t ldr, int64_t rows, int64_t cols) {
    const int64_t tot = rows * cols;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = e % rows, j = e / rows;
        if (i > j) R[i + j * ldr] = T(0);
    }
}

__global__ void set_one_kernel(int* p) { *p = 1; }

template <typename T>
__global__ void widen_kernel(const T* __restrict__ A, int64_t lda, int64_t m, int64_t n, double* __restrict__ D) {
    const int64_t tot = m * n;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x)
        D[e] = (double)A[(e % m) + (e / m) * lda];
}

inline unsigned grid_for(int64_t n) { return (unsigned)std::min<int64_t>((n + 255) / 256, 4096); }

// OCP e4m3fn -> fp32 (exact): 1 sign, 4 exponent (bias 7), 3 mantissa bits; S.1111.111 is NaN
__device__ __forceinline__ float e4m3_to_f32(uint32_t b) {
    const uint32_t e = (b >> 3) & 15u, mt = b & 7u;
    float v;
    if (e == 15u && mt == 7u) v = __builtin_nanf("");
    else if (e == 0u) v = (float)mt * 0x1p-9f;
    else v = __uint_as_float(((e + 120u) << 23) | (mt << 20));
    return (b & 0x80u) ? -v : v;
}

// bf16 / e4m3 A (column-major, ld lda) -> fp32 (column-major, ld m)
__global__ void lowp_to_f32_kernel(const void* __restrict__ A, int64_t lda, int64_t m, int64_t n, int fp8,
                                   float* __restrict__ D) {
    const int64_t tot = m * n;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t o = (e % m) + (e / m) * lda;
        D[e] = fp8 ? e4m3_to_f32(reinterpret_cast<const uint8_t*>(A)[o])
                   : __uint_as_float((uint32_t)reinterpret_cast<const uint16_t*>(A)[o] << 16);
    }
}

// bf16 row-major panel (rows x LP) -> fp32 column-major (rows x cols, ld)
__global__ void bf16_panel_to_f32_kernel(const uint16_t* __restrict__ P, int64_t rows, int cols, int LP,
                                         float* __restrict__ D, int64_t ld) {
    const int64_t tot = rows * cols;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = e % rows, j = e / rows;
        D[i + j * ld] = __uint_as_float((uint32_t)P[i * LP + j] << 16);
    }
}

}  // namespace

hipError_t launch_lowp_to_f32(const void* A, int64_t lda, int64_t m, int64_t n, int fp8, float* D, hipStream_t s) {
    hipLaunchKernelGGL(lowp_to_f32_kernel, dim3(grid_for(m * n)), dim3(256), 0, s, A, lda, m, n, fp8, D);
    return hipGetLastError();
}

hipError_t launch_bf16_panel_to_f32(const uint16_t* P, int64_t rows, int cols, int LP, float* D, int64_t ld,
                                    hipStream_t s) {
    hipLaunchKernelGGL(bf16_panel_to_f32_kernel, dim3(grid_for(rows * cols)), dim3(256), 0, s, P, rows, cols, LP, D, ld);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_gemm(int ta, int tb, int64_t M, int64_t N, int64_t K, T alpha, const T* A, int64_t lda, const T* B,
                       int64_t ldb, T beta, T* C, int64_t ldc, hipStream_t s) {
    if (M <= 0 || N <= 0) return hipSuccess;
    const dim3 grid((unsigned)((M + GT - 1) / GT), (unsigned)((N + GT - 1) / GT));
    hipLaunchKernelGGL((gemm_kernel<T>), grid, dim3(256), 0, s, ta, tb, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_qr_signs_cm(const T* A, int64_t lda, int64_t m, int64_t n, T* Q, int64_t ldq, hipStream_t s) {
    hipLaunchKernelGGL((qr_signs_cm_kernel<T>), dim3(1), dim3(256), 0, s, A, lda, m, n, Q, ldq);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_det_sign_cm(T* Q, int64_t ldq, int m, double* W, int* sgn, hipStream_t s) {
    // W: 2 m^2 doubles (double buffer); sgn: one int
    hipLaunchKernelGGL(set_one_kernel, dim3(1), dim3(1), 0, s, sgn);
    double* W0 = W;
    double* W1 = W + (size_t)m * m;
    hipLaunchKernelGGL((to_f64_square_kernel<T>), dim3(grid_for((int64_t)m * m)), dim3(256), 0, s, Q, ldq, m, W0);
    for (int k = 0; k < m; ++k) {
        const int64_t rem = (int64_t)(m - k - 1) * (m - k - 1);
        const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((rem + 255) / 256, 1024));
        hipLaunchKernelGGL(lu_sign_step_kernel, dim3(g), dim3(256), 0, s, W0, W1, m, k, sgn);
        std::swap(W0, W1);
    }
    hipLaunchKernelGGL((flip_last_if_negative_kernel<T>), dim3(grid_for(m)), dim3(256), 0, s, Q, ldq, m, m - 1, sgn);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_identity_cols(T* Y, int64_t ldy, int64_t rows, int cols, int64_t e0, hipStream_t s) {
    hipLaunchKernelGGL((identity_cols_kernel<T>), dim3(grid_for(rows * cols)), dim3(256), 0, s, Y, ldy, rows, cols, e0);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_zero_below(T* R, int64_t ldr, int64_t rows, int64_t cols, hipStream_t s) {
    hipLaunchKernelGGL((zero_below_kernel<T>), dim3(grid_for(rows * cols)), dim3(256), 0, s, R, ldr, rows, cols);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_widen(const T* A, int64_t lda, int64_t m, int64_t n, double* D, hipStream_t s) {
    hipLaunchKernelGGL((widen_kernel<T>), dim3(grid_for(m * n)), dim3(256), 0, s, A, lda, m, n, D);
    return hipGetLastError();
}

#define RSVD_GEMM_INST(T)                                                                                          \
    template hipError_t launch_gemm<T>(int, int, int64_t, int64_t, int64_t, T, const T*, int64_t, const T*,        \
                                       int64_t, T, T*, int64_t, hipStream_t);                                      \
    template hipError_t launch_qr_signs_cm<T>(const T*, int64_t, int64_t, int64_t, T*, int64_t, hipStream_t);      \
    template hipError_t launch_det_sign_cm<T>(T*, int64_t, int, double*, int*, hipStream_t);                       \
    template hipError_t launch_identity_cols<T>(T*, int64_t, int64_t, int, int64_t, hipStream_t);                  \
    template hipError_t launch_zero_below<T>(T*, int64_t, int64_t, int64_t, hipStream_t);                          \
    template hipError_t launch_widen<T>(const T*, int64_t, int64_t, int64_t, double*, hipStream_t);
RSVD_GEMM_INST(float)
RSVD_GEMM_INST(double)
#undef RSVD_GEMM_INST

}  // namespace rsvd
