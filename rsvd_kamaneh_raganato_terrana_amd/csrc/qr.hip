// qr.hip -- tall-skinny orthonormalisation by CholeskyQR2 with an fp64 Gram, plus the
// "panel x small matrix" MFMA kernel used for Q = Y R^-1 and the back-projections
// U = Q * U_w (src/rSVD.cpp:128) and V = Q_B * V_w.
//
// The reference orthonormalises with Eigen::HouseholderQR + householderQ()*Identity
// (src/rSVD.cpp:60-61,64-65,67-68).  rSVD's outputs depend only on span(Q), so
// any numerically orthonormal basis of span(Y) is a drop-in.  CholeskyQR2 needs two streaming
// passes over the panel and an l x l Cholesky:
//     G = Y^T Y (fp64, exact products of f32/f64 entries), R1 = chol(G), Q1 = Y R1^-1,
//     G' = Q1^T Q1, R2 = chol(G'), Q = Q1 R2^-1, R = R2 R1.
// It is accurate while cond(Y) << 1/sqrt(u_64); the Cholesky raises a device flag when a pivot
// falls below 1e-10 of its original diagonal (cond(Y) >~ 1e5 or rank loss), and the driver then
// re-runs that panel through the Householder TSQR path (tsqr.hip).
#include "common.hpp"
#include "kernels.hpp"

namespace rsvd {

namespace {

constexpr int kGramWaves = 4;

// Partial Gram of the panel rows [b*chunk, (b+1)*chunk): f64 MFMA on (exactly) up-converted
// entries.  Lane (r, h) holds P[i0 + h][16 g + r] for every column group g; that value is both
// the A operand (P^T[16 g1 + r][i0 + h]) and the B operand (P[i0 + h][16 g2 + r]).
template <typename T, int LP>
__global__ __launch_bounds__(kWave* kGramWaves) void gram_partial_kernel(const T* __restrict__ P,
                                                                        int64_t rows, int64_t chunk,
                                                                        double* __restrict__ gslabs) {
    constexpr int G = LP / 16;
    typedef Mfma<double> M;
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    double* red = reinterpret_cast<double*>(smem_raw);  // [kGramWaves][LP][LP]
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = lane & 15, h = lane >> 4;
    const int64_t rbeg = (int64_t)blockIdx.x * chunk;
    const int64_t rend = (rbeg + chunk < rows) ? rbeg + chunk : rows;

    f64x4 acc[G][G];
#pragma unroll
    for (int a = 0; a < G; ++a)
#pragma unroll
        for (int b = 0; b < G; ++b) acc[a][b] = M::zero();

    for (int64_t i0 = rbeg + 4 * w; i0 < rend; i0 += 4 * kGramWaves) {
        const int64_t i = i0 + h;
        double y[G];
#pragma unroll
        for (int g = 0; g < G; ++g) y[g] = (i < rend) ? (double)P[i * LP + 16 * g + r] : 0.0;
#pragma unroll
        for (int a = 0; a < G; ++a)
#pragma unroll
            for (int b = a; b < G; ++b) acc[a][b] = M::mma(y[a], y[b], acc[a][b]);
    }
    double* mine = red + (size_t)w * LP * LP;
#pragma unroll
    for (int a = 0; a < G; ++a)
#pragma unroll
        for (int b = a; b < G; ++b)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int row = 16 * a + M::row(h, j), col = 16 * b + r;
                mine[row * LP + col] = acc[a][b][j];
            }
    __syncthreads();
    double* dst = gslabs + (size_t)blockIdx.x * LP * LP;
    for (int e = threadIdx.x; e < LP * LP; e += blockDim.x) {
        const int row = e / LP, col = e % LP;
        const int a = row / 16, b = col / 16;
        // only the upper tile blocks were produced; mirror the lower ones
        const int src = (a <= b) ? e : col * LP + row;
        double s = 0.0;
#pragma unroll
        for (int ww = 0; ww < kGramWaves; ++ww) s += red[(size_t)ww * LP * LP + src];
        dst[e] = s;
    }
}

// One workgroup: G = sum(slabs); R = chol(G) upper; Rinv = R^-1; Racc = R * Racc (optional).
__global__ __launch_bounds__(256) void chol_inv_kernel(const double* __restrict__ gslabs, int nslab, int l,
                                                       int LP, double* __restrict__ Rout,
                                                       double* __restrict__ Rinv_out, double* __restrict__ Racc,
                                                       int accumulate, int* __restrict__ flag) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    double* Gs = reinterpret_cast<double*>(smem_raw);  // [LP][LP]
    double* Ri = Gs + LP * LP;                          // [LP][LP]
    double* d0 = Ri + LP * LP;                          // [LP] original diagonal
    int& bad = *reinterpret_cast<int*>(d0 + LP);        // kept in the dynamic region (Guideline 17)
    const int tid = threadIdx.x, nt = blockDim.x;
    if (tid == 0) bad = 0;
    for (int e = tid; e < LP * LP; e += nt) {
        double s = 0.0;
        for (int b = 0; b < nslab; ++b) s += gslabs[(size_t)b * LP * LP + e];
        Gs[e] = s;
        Ri[e] = 0.0;
    }
    __syncthreads();
    for (int k = tid; k < l; k += nt) d0[k] = Gs[k * LP + k];
    __syncthreads();
    // right-looking Cholesky on the upper triangle
    for (int k = 0; k < l; ++k) {
        if (tid == 0) {
            double d = Gs[k * LP + k];
            const double ref = d0[k];
            if (!(d > 1e-10 * ref) || !(ref > 0.0) || !isfinite(d)) {
                bad = 1;
                d = (ref > 0.0 && isfinite(ref)) ? ref : 1.0;  // keep going without NaNs; result flagged
            }
            Gs[k * LP + k] = sqrt(d);
        }
        __syncthreads();
        const double inv = 1.0 / Gs[k * LP + k];
        for (int j = k + 1 + tid; j < l; j += nt) Gs[k * LP + j] *= inv;
        __syncthreads();
        const int rem = l - k - 1;
        for (int e = tid; e < rem * rem; e += nt) {
            const int i = k + 1 + e / rem, j = k + 1 + e % rem;
            if (j >= i) Gs[i * LP + j] -= Gs[k * LP + i] * Gs[k * LP + j];
        }
        __syncthreads();
    }
    // Rinv: bottom-up rows, Rinv[i][j] = -(1/R_ii) * sum_{p=i+1..j} R[i][p] Rinv[p][j]
    for (int i = l - 1; i >= 0; --i) {
        const double rii = Gs[i * LP + i];
        for (int j = i + tid; j < l; j += nt) {
            if (j == i) {
                Ri[i * LP + i] = 1.0 / rii;
            } else {
                double s = 0.0;
                for (int p = i + 1; p <= j; ++p) s += Gs[i * LP + p] * Ri[p * LP + j];
                Ri[i * LP + j] = -s / rii;
            }
        }
        __syncthreads();
    }
    // outputs (zero the strictly-lower part and the padding)
    for (int e = tid; e < LP * LP; e += nt) {
        const int i = e / LP, j = e % LP;
        const bool in = (i < l && j < l && j >= i);
        Rout[e] = in ? Gs[e] : 0.0;
        Rinv_out[e] = in ? Ri[e] : 0.0;
    }
    if (accumulate) {
        // Racc <- R * Racc  (both upper triangular); stage old Racc in Ri (Rinv already written)
        __syncthreads();
        for (int e = tid; e < LP * LP; e += nt) Ri[e] = Racc[e];
        __syncthreads();
        for (int e = tid; e < LP * LP; e += nt) {
            const int i = e / LP, j = e % LP;
            double s = 0.0;
            if (i < l && j < l && j >= i)
                for (int p = i; p <= j; ++p) s += Gs[i * LP + p] * Ri[p * LP + j];
            Racc[e] = s;
        }
    }
    __syncthreads();
    if (tid == 0 && bad) atomicOr(flag, 1);
}

// Out = In * M: 16 rows per wave, 4 waves per workgroup; In tile and M staged in LDS.
template <typename T, int LP>
__global__ __launch_bounds__(256) void panel_small_kernel(const T* __restrict__ In, int64_t rows,
                                                          const double* __restrict__ Mg, T* __restrict__ Out,
                                                          int out_colmajor, int cols, int64_t ld) {
    typedef Mfma<T> M;
    typedef typename M::acc_t acc_t;
    constexpr int G = LP / 16;
    constexpr int RPB = 64;  // rows per block
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    T* Ms = reinterpret_cast<T*>(smem_raw);  // [LP][LP]
    T* Is = Ms + LP * LP;                    // [RPB][LP + 1] (padded: fragment reads are column-wise)
    constexpr int IS = LP + 1;
    const int tid = threadIdx.x;
    const int lane = tid & 63, w = tid >> 6;
    const int r = lane & 15, h = lane >> 4;
    const int64_t row0 = (int64_t)blockIdx.x * RPB;
    for (int e = tid; e < LP * LP; e += blockDim.x) Ms[e] = (T)Mg[e];
    for (int e = tid; e < RPB * LP; e += blockDim.x) {
        const int lr = e / LP, c = e % LP;
        Is[lr * IS + c] = (row0 + lr < rows) ? In[(row0 + lr) * LP + c] : T(0);
    }
    __syncthreads();
    acc_t acc[G];
#pragma unroll
    for (int g = 0; g < G; ++g) acc[g] = M::zero();
    const int lr0 = w * 16;
#pragma unroll
    for (int k0 = 0; k0 < LP; k0 += 4) {
        const T a = Is[(lr0 + r) * IS + k0 + h];
#pragma unroll
        for (int g = 0; g < G; ++g) acc[g] = M::mma(a, Ms[(k0 + h) * LP + 16 * g + r], acc[g]);
    }
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t row = row0 + lr0 + M::row(h, j);
            const int col = 16 * g + r;
            if (row < rows) {
                if (!out_colmajor)
                    Out[row * LP + col] = acc[g][j];
                else if (col < cols)
                    Out[row + (int64_t)col * ld] = acc[g][j];
            }
        }
}

}  // namespace

int plan_gram_blocks(int64_t rows) {
    int64_t blocks = (rows + 1023) / 1024;  // >= 1024 rows per workgroup
    if (blocks > 64) blocks = 64;
    if (blocks < 1) blocks = 1;
    return (int)blocks;
}

template <typename T>
hipError_t launch_gram_partial(const T* P, int64_t rows, int LP, int nblk, double* gslabs, hipStream_t s) {
    const int64_t chunk = (rows + nblk - 1) / nblk;
    const size_t lds = (size_t)kGramWaves * LP * LP * sizeof(double);
    switch (LP) {
#define CASE(L)                                                                                            \
    case L:                                                                                                \
        hipLaunchKernelGGL((gram_partial_kernel<T, L>), dim3(nblk), dim3(kWave * kGramWaves), lds, s, P, rows, \
                           chunk, gslabs);                                                                 \
        break;
        CASE(16) CASE(32) CASE(48) CASE(64)
#undef CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_chol_inv(const double* gslabs, int nslab, int l, int LP, double* R, double* Rinv, double* Racc,
                           int accumulate, int* flag, hipStream_t s) {
    const size_t lds = (size_t)(2 * LP * LP + LP) * sizeof(double) + 16;
    hipLaunchKernelGGL(chol_inv_kernel, dim3(1), dim3(256), lds, s, gslabs, nslab, l, LP, R, Rinv, Racc,
                       accumulate, flag);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_panel_small(const T* In, int64_t rows, int LP, const double* Mat, T* Out, int out_colmajor,
                              int cols, int64_t ld, hipStream_t s) {
    const int blocks = (int)((rows + 63) / 64);
    const size_t lds = (size_t)(LP * LP + 64 * (LP + 1)) * sizeof(T);
    switch (LP) {
#define CASE(L)                                                                                          \
    case L:                                                                                              \
        hipLaunchKernelGGL((panel_small_kernel<T, L>), dim3(blocks), dim3(256), lds, s, In, rows, Mat, Out, \
                           out_colmajor, cols, ld);                                                      \
        break;
        CASE(16) CASE(32) CASE(48) CASE(64)
#undef CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

#define RSVD_INST(T)                                                                                       \
    template hipError_t launch_gram_partial<T>(const T*, int64_t, int, int, double*, hipStream_t);         \
    template hipError_t launch_panel_small<T>(const T*, int64_t, int, const double*, T*, int, int, int64_t, \
                                              hipStream_t);
RSVD_INST(float)
RSVD_INST(double)
#undef RSVD_INST

}  // namespace rsvd
