// util.hip -- Omega generation, panel layout conversions, slab reduction.
//
// Omega: the reference draws an n x l Gaussian from std::mt19937(random_device()+rank)
// (src/rSVD.cpp:26-37) and ships it with MPI_Gatherv + MPI_Bcast (:49,52).  Here every GPU
// regenerates the identical matrix from a counter-based Philox4x32-10 stream keyed by the
// seed, so Omega needs no communication and the CPU oracle (oracle/rsvd_oracle.c,
// orc_philox_gaussian) can draw the same numbers.  Element (i, j) is stream element i + n*j.
#include <algorithm>

#include "common.hpp"
#include "kernels.hpp"

namespace rsvd {

namespace {

template <typename T>
__global__ void philox_omega_kernel(T* __restrict__ out, int64_t n, int l, int LP, uint64_t seed) {
    const int64_t total = n * LP;
    for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = idx / LP;
        const int j = (int)(idx - i * LP);
        out[idx] = (j < l) ? (T)gauss_elem((uint64_t)(i + n * (int64_t)j), seed) : T(0);
    }
}

template <typename T>
__global__ void colmajor_to_panel_kernel(const T* __restrict__ in, int64_t ld, int64_t m, int l, int LP,
                                         T* __restrict__ out) {
    const int64_t total = m * LP;
    for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = idx / LP;
        const int j = (int)(idx - i * LP);
        out[idx] = (j < l) ? in[i + (int64_t)j * ld] : T(0);
    }
}

template <typename T>
__global__ void panel_to_colmajor_kernel(const T* __restrict__ in, int64_t m, int cols, int LP,
                                         T* __restrict__ out, int64_t ld) {
    const int64_t total = m * cols;
    for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = idx / m;
        const int64_t i = idx - j * m;
        out[i + j * ld] = in[i * LP + j];
    }
}

template <typename T>
__global__ void sum_slabs_kernel(const T* __restrict__ slabs, int64_t stride, int nslab, int64_t count,
                                 T* __restrict__ out) {
    typedef typename Vec16<T>::type V;
    constexpr int VW = Vec16<T>::N;
    const int64_t nv = count / VW;
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < nv;
         v += (int64_t)gridDim.x * blockDim.x) {
        V acc = *reinterpret_cast<const V*>(slabs + v * VW);
        T* a = reinterpret_cast<T*>(&acc);
        for (int s = 1; s < nslab; ++s) {
            const V o = *reinterpret_cast<const V*>(slabs + s * stride + v * VW);
            const T* b = reinterpret_cast<const T*>(&o);
#pragma unroll
            for (int t = 0; t < VW; ++t) a[t] += b[t];
        }
        *reinterpret_cast<V*>(out + v * VW) = acc;
    }
}

template <typename T>
__global__ void scale_cols_kernel(T* __restrict__ X, int64_t rows, int cols, int64_t ld, double f) {
    const int64_t total = rows * cols;
    for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = idx / rows, i = idx - j * rows;
        X[i + j * ld] = (T)((double)X[i + j * ld] * f);
    }
}

template <typename T>
__global__ void check_finite_kernel(const T* __restrict__ x, int n, int* __restrict__ flag) {
    bool bad = false;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        bad = bad || !isfinite((double)x[i]);
    if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

// The global row count of a row-sharded A: *cnt = this rank's rows, summed by the
// first m-side Gram all-reduce; the check flags l > m_global (every rank sees the same sum).
__global__ void set_count_kernel(double* __restrict__ cnt, double v) { *cnt = v; }
__global__ void check_rows_kernel(const double* __restrict__ cnt, int l, int* __restrict__ flag) {
    if (*cnt + 0.5 < (double)l) *flag = 1;
}

inline int grid_for(int64_t work, int block) {
    int64_t g = (work + block - 1) / block;
    if (g > 4096) g = 4096;
    if (g < 1) g = 1;
    return (int)g;
}

}  // namespace

template <typename T>
hipError_t launch_philox_omega(T* out, int64_t n, int l, int LP, uint64_t seed, hipStream_t s) {
    hipLaunchKernelGGL((philox_omega_kernel<T>), dim3(grid_for(n * LP, 256)), dim3(256), 0, s, out, n, l, LP,
                       seed);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_colmajor_to_panel(const T* in, int64_t ld, int64_t m, int l, int LP, T* out, hipStream_t s) {
    hipLaunchKernelGGL((colmajor_to_panel_kernel<T>), dim3(grid_for(m * LP, 256)), dim3(256), 0, s, in, ld, m,
                       l, LP, out);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_panel_to_colmajor(const T* in, int64_t m, int cols, int LP, T* out, int64_t ld, hipStream_t s) {
    hipLaunchKernelGGL((panel_to_colmajor_kernel<T>), dim3(grid_for(m * cols, 256)), dim3(256), 0, s, in, m,
                       cols, LP, out, ld);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_sum_slabs(const T* slabs, int64_t slab_stride, int nslab, int64_t count, T* out,
                            hipStream_t s) {
    // count and slab_stride are multiples of LP (>= 16) -> multiples of the 16-B vector width.
    hipLaunchKernelGGL((sum_slabs_kernel<T>), dim3(grid_for(count / Vec16<T>::N, 256)), dim3(256), 0, s, slabs,
                       slab_stride, nslab, count, out);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_scale_cols(T* X, int64_t rows, int cols, int64_t ld, double f, hipStream_t s) {
    hipLaunchKernelGGL((scale_cols_kernel<T>), dim3(grid_for(rows * cols, 256)), dim3(256), 0, s, X, rows, cols, ld, f);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_check_finite(const T* x, int n, int* flag, hipStream_t s) {
    hipLaunchKernelGGL((check_finite_kernel<T>), dim3(std::min(64, (n + 255) / 256)), dim3(256), 0, s, x, n, flag);
    return hipGetLastError();
}

hipError_t launch_set_count(double* cnt, int64_t v, hipStream_t s) {
    hipLaunchKernelGGL(set_count_kernel, dim3(1), dim3(1), 0, s, cnt, (double)v);
    return hipGetLastError();
}

hipError_t launch_check_rows(const double* cnt, int l, int* flag, hipStream_t s) {
    hipLaunchKernelGGL(check_rows_kernel, dim3(1), dim3(1), 0, s, cnt, l, flag);
    return hipGetLastError();
}

#define RSVD_INST(T)                                                                                    \
    template hipError_t launch_scale_cols<T>(T*, int64_t, int, int64_t, double, hipStream_t);           \
    template hipError_t launch_check_finite<T>(const T*, int, int*, hipStream_t);                       \
    template hipError_t launch_philox_omega<T>(T*, int64_t, int, int, uint64_t, hipStream_t);           \
    template hipError_t launch_colmajor_to_panel<T>(const T*, int64_t, int64_t, int, int, T*, hipStream_t); \
    template hipError_t launch_panel_to_colmajor<T>(const T*, int64_t, int, int, T*, int64_t, hipStream_t); \
    template hipError_t launch_sum_slabs<T>(const T*, int64_t, int, int64_t, T*, hipStream_t);
RSVD_INST(float)
RSVD_INST(double)
#undef RSVD_INST

}  // namespace rsvd

// ================================================================================================
// Robust re-orthonormalisation (fallback for a panel whose CholeskyQR flagged a bad pivot:
// rank-deficient or too ill-conditioned Y).  Predicated on *flag: one early-exit launch otherwise.
// One workgroup, classical Gram-Schmidt with re-orthogonalisation ("twice is enough", a third pass
// when a column lost more than half its norm) on the ORIGINAL panel P.  A column whose residual is
// at the rounding-noise level (relative 1e-13 fp64 / 1e-6 fp32) is replaced by a Philox Gaussian
// vector and orthogonalised: like the reference's Householder Q (src/rSVD.cpp:60-61), the result is
// an orthonormal basis of span(Y) completed by arbitrary orthonormal directions.
// ================================================================================================
namespace rsvd {
namespace {

constexpr int kRobustThreads = 256;

__device__ __forceinline__ double block_sum(double v, double* red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    double s = 0.0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
    return s;
}

template <typename T>
__global__ __launch_bounds__(kRobustThreads) void robust_orth_kernel(const T* __restrict__ P, int64_t rows, int l,
                                                                    int LP, T* __restrict__ Q,
                                                                    const int* __restrict__ flag, uint64_t seed) {
    if (*flag == 0) return;
    __shared__ double dots[64 + 8];
    __shared__ double red[8];
    const int tid = threadIdx.x, nt = blockDim.x;
    const double tiny = sizeof(T) == 4 ? 1e-6 : 1e-13;
    // zero the padding columns, copy P into Q (columns are orthogonalised in place)
    for (int64_t e = tid; e < rows * LP; e += nt) Q[e] = ((e % LP) < l) ? P[e] : T(0);
    __syncthreads();
    for (int j = 0; j < l; ++j) {
        double n0 = 0.0;
        for (int64_t r = tid; r < rows; r += nt) n0 += (double)Q[r * LP + j] * (double)Q[r * LP + j];
        n0 = sqrt(block_sum(n0, red));
        bool replaced = false;
        for (int attempt = 0; attempt < 2; ++attempt) {
            double nprev = n0;
            for (int pass = 0; pass < 3; ++pass) {
                // d_i = <q_i, v>, i < j  (256 threads x up to 64 partial sums, reduced per i)
                for (int i = 0; i < j; ++i) {
                    double d = 0.0;
                    for (int64_t r = tid; r < rows; r += nt) d += (double)Q[r * LP + i] * (double)Q[r * LP + j];
                    d = block_sum(d, red);
                    if (tid == 0) dots[i] = d;
                }
                __syncthreads();
                double nn = 0.0;
                for (int64_t r = tid; r < rows; r += nt) {
                    double x = (double)Q[r * LP + j];
                    for (int i = 0; i < j; ++i) x -= dots[i] * (double)Q[r * LP + i];
                    Q[r * LP + j] = (T)x;
                    nn += x * x;
                }
                nn = sqrt(block_sum(nn, red));
                const bool again = nn < 0.5 * nprev;
                nprev = nn;
                if (pass >= 1 && !again) break;
            }
            if (nprev > tiny * n0 && nprev > 0.0 && isfinite(nprev)) {
                const double inv = 1.0 / nprev;
                for (int64_t r = tid; r < rows; r += nt) Q[r * LP + j] = (T)((double)Q[r * LP + j] * inv);
                __syncthreads();
                break;
            }
            // rounding-noise residual: replace by a deterministic Gaussian vector and retry
            replaced = true;
            for (int64_t r = tid; r < rows; r += nt) {
                uint32_t x[4];
                philox4x32_10((uint64_t)r * 64 + j, seed ^ 0xC0FFEE1234ull, x);
                Q[r * LP + j] = (T)((double)x[0] * 2.3283064365386963e-10 - 0.5);
            }
            __syncthreads();
            n0 = 0.0;
            for (int64_t r = tid; r < rows; r += nt) n0 += (double)Q[r * LP + j] * (double)Q[r * LP + j];
            n0 = sqrt(block_sum(n0, red));
        }
        (void)replaced;
        __syncthreads();
    }
}

}  // namespace

template <typename T>
hipError_t launch_robust_orth(const T* P, int64_t rows, int l, int LP, T* Q, const int* flag, uint64_t seed,
                              hipStream_t s) {
    hipLaunchKernelGGL((robust_orth_kernel<T>), dim3(1), dim3(kRobustThreads), 0, s, P, rows, l, LP, Q, flag, seed);
    return hipGetLastError();
}

template hipError_t launch_robust_orth<float>(const float*, int64_t, int, int, float*, const int*, uint64_t, hipStream_t);
template hipError_t launch_robust_orth<double>(const double*, int64_t, int, int, double*, const int*, uint64_t,
                                               hipStream_t);

}  // namespace rsvd
