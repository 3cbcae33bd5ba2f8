// jacobi.hip -- the small SVD of the rSVD (SVD<Jacobi>::compute on B, include/SVD_class.hpp:100-180).
//
// The reference QR-preconditions the wide B (l x n): B^T = Q_B R, W = R^T (l x l), then runs a
// cyclic two-sided Jacobi on W, applying every rotation to the n x l V_ directly (:145-148),
// takes |diag| with a sign fix (:158-162) and selection-sorts descending (:164-178).
// Here the same decomposition W = U_w diag(S) V_w^T is computed on ONE workgroup by
// one-sided (Hestenes) Jacobi with the round-robin (circle-method) pair ordering, so the l/2
// disjoint rotations of a round run in parallel (TPP threads per pair, wavefront-level
// shuffle reductions for the three dot products).  Rotations accumulate into the l x l V_w,
// and the driver forms V = Q_B V_w and U = Q U_w with one MFMA panel product each instead of
// rotating n x l / m x l matrices column pair by column pair.
// The converged factorisation is the same SVD as the reference's up to the sign of each
// (u_i, v_i) pair (and the basis inside exactly repeated singular values), which is how the
// parity tests compare it.
#include "common.hpp"
#include "kernels.hpp"

namespace rsvd {

namespace {

__device__ __forceinline__ void rr_pair(int round, int k, int N, int& p, int& q) {
    if (k == 0) {
        p = round;
        q = N - 1;
    } else {
        p = (round + k) % (N - 1);
        q = (round - k + (N - 1)) % (N - 1);
    }
}

template <typename T>
__global__ __launch_bounds__(256) void small_svd_kernel(const double* __restrict__ R, int l, int LP,
                                                        double* __restrict__ Uw, double* __restrict__ Vw,
                                                        T* __restrict__ S, int* __restrict__ info) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    const int CS = LP + 1;                                  // padded column stride
    double* X = reinterpret_cast<double*>(smem_raw);        // [LP][CS]   X[c*CS + i]
    double* J = X + LP * CS;                                // [LP][CS]
    double* sig = J + LP * CS;                              // [LP]
    double* v = sig + LP;                                   // [LP] completion scratch
    int* rank = reinterpret_cast<int*>(v + LP);             // [LP]
    int* flags = rank + LP;                                 // [4]
    const int tid = threadIdx.x, nt = blockDim.x;

    // X = W = R^T  (column c of W is row c of R), J = I
    for (int e = tid; e < LP * LP; e += nt) {
        const int c = e / LP, i = e % LP;
        X[c * CS + i] = (c < l && i < l) ? R[c * LP + i] : 0.0;  // W[i][c] = R[c][i]
        J[c * CS + i] = (c == i && c < l) ? 1.0 : 0.0;
    }
    const int N = (l & 1) ? l + 1 : l;       // dummy zero column when l is odd (l < LP then)
    const int npairs = N / 2;
    int TPP = 1;
    while (TPP * 2 * npairs <= nt && TPP < 64) TPP *= 2;
    const int pi = tid / TPP, sub = tid % TPP;
    const bool active = pi < npairs;
    const double tol = (double)l * 2.220446049250313e-16;
    int sweeps = 0;
    __syncthreads();
    for (; sweeps < 64; ++sweeps) {
        if (tid == 0) flags[0] = 0;
        __syncthreads();
        for (int round = 0; round < N - 1; ++round) {
            if (active) {
                int p, q;
                rr_pair(round, pi, N, p, q);
                double a = 0.0, b = 0.0, c = 0.0;
                for (int i = sub; i < l; i += TPP) {
                    const double xp = X[p * CS + i], xq = X[q * CS + i];
                    a += xp * xp;
                    b += xq * xq;
                    c += xp * xq;
                }
                for (int o = TPP >> 1; o > 0; o >>= 1) {
                    a += __shfl_xor(a, o, 64);
                    b += __shfl_xor(b, o, 64);
                    c += __shfl_xor(c, o, 64);
                }
                if (c != 0.0 && fabs(c) > tol * sqrt(a) * sqrt(b)) {
                    const double zeta = (b - a) / (2.0 * c);
                    const double t = (zeta >= 0.0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                    const double cs = 1.0 / sqrt(1.0 + t * t), sn = cs * t;
                    for (int i = sub; i < LP; i += TPP) {
                        const double xp = X[p * CS + i], xq = X[q * CS + i];
                        X[p * CS + i] = cs * xp - sn * xq;
                        X[q * CS + i] = sn * xp + cs * xq;
                        const double jp = J[p * CS + i], jq = J[q * CS + i];
                        J[p * CS + i] = cs * jp - sn * jq;
                        J[q * CS + i] = sn * jp + cs * jq;
                    }
                    if (sub == 0) flags[0] = 1;
                }
            }
            __syncthreads();
        }
        if (flags[0] == 0) break;
        __syncthreads();
    }
    // singular values = column norms
    for (int c = tid; c < LP; c += nt) {
        double s2 = 0.0;
        if (c < l)
            for (int i = 0; i < l; ++i) s2 += X[c * CS + i] * X[c * CS + i];
        sig[c] = sqrt(s2);
    }
    __syncthreads();
    // descending rank (stable on ties)
    for (int c = tid; c < l; c += nt) {
        int rk = 0;
        const double sc = sig[c];
        for (int d = 0; d < l; ++d) rk += (sig[d] > sc) || (sig[d] == sc && d < c);
        rank[c] = rk;
    }
    __syncthreads();
    for (int e = tid; e < LP * LP; e += nt) {
        Uw[e] = 0.0;
        Vw[e] = 0.0;
    }
    __syncthreads();
    for (int e = tid; e < l * l; e += nt) {
        const int c = e / l, i = e % l;
        const int k = rank[c];
        const double sc = sig[c];
        Uw[i * LP + k] = (sc > 0.0) ? X[c * CS + i] / sc : 0.0;
        Vw[i * LP + k] = J[c * CS + i];
    }
    for (int c = tid; c < l; c += nt) S[rank[c]] = (T)sig[c];
    __syncthreads();
    // Exactly-zero singular values: complete U_w to an orthonormal basis (the reference's U is a
    // product of rotations, hence always orthonormal).  Rare path, one thread.
    if (tid == 0) {
        int nz = 0;
        for (int c = 0; c < l; ++c) nz += (sig[c] > 0.0);
        for (int k = nz; k < l; ++k) {
            for (int cand = 0; cand < l; ++cand) {
                for (int i = 0; i < l; ++i) v[i] = (i == cand) ? 1.0 : 0.0;
                for (int pass = 0; pass < 2; ++pass)
                    for (int j = 0; j < k; ++j) {
                        double d = 0.0;
                        for (int i = 0; i < l; ++i) d += Uw[i * LP + j] * v[i];
                        for (int i = 0; i < l; ++i) v[i] -= d * Uw[i * LP + j];
                    }
                double nv = 0.0;
                for (int i = 0; i < l; ++i) nv += v[i] * v[i];
                nv = sqrt(nv);
                if (nv > 0.5) {
                    for (int i = 0; i < l; ++i) Uw[i * LP + k] = v[i] / nv;
                    break;
                }
            }
        }
        info[0] = sweeps + 1;
    }
}

}  // namespace

template <typename T>
hipError_t launch_small_svd(const double* R, int l, int LP, double* Uw, double* Vw, T* S, int* info,
                            hipStream_t s) {
    if (l > 256 || LP > 256) return hipErrorInvalidValue;
    const size_t lds = (size_t)(2 * LP * (LP + 1) + 2 * LP) * sizeof(double) + (size_t)(LP + 4) * sizeof(int);
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    hipLaunchKernelGGL((small_svd_kernel<T>), dim3(1), dim3(256), lds, s, R, l, LP, Uw, Vw, S, info);
    return hipGetLastError();
}

template hipError_t launch_small_svd<float>(const double*, int, int, double*, double*, float*, int*, hipStream_t);
template hipError_t launch_small_svd<double>(const double*, int, int, double*, double*, double*, int*, hipStream_t);

}  // namespace rsvd
