// jacobi.hip -- the small SVD of the rSVD (SVD<Jacobi>::compute on B, include/SVD_class.hpp:100-180).
//
// The reference QR-preconditions the wide B (l x n): B^T = Q_B R, W = R^T (l x l), then runs a
// cyclic two-sided Jacobi on W, applying every rotation to the n x l V_ directly (:145-148),
// takes |diag| with a sign fix (:158-162) and selection-sorts descending (:164-178).
// Here W = U_w diag(S) V_w^T is computed on ONE workgroup by one-sided (Hestenes) Jacobi with the
// round-robin (circle-method) pair ordering, so the l/2 disjoint rotations of a round run in
// parallel (TPP threads per pair, DPP reductions for the dot product).  Rotations accumulate into
// the l x l V_w, and the driver forms V = Q_B V_w and U = Q U_w with one MFMA panel product each
// instead of rotating n x l / m x l matrices column pair by column pair.  The input is given as
// R with W[i][c] = R[c][i] (the driver passes R = Q_B^T B^T from the cross-Gram, so W need not be
// triangular).  Compute type C: fp64 on the fp64 path; fp32 on the fp32 path (one-sided Jacobi
// is relatively accurate, and fp32 halves the dependent-latency chains that bound a round).
// The converged factorisation is the same SVD as the reference's up to the sign of each
// (u_i, v_i) pair (and the basis inside exactly repeated singular values), which is how the
// parity tests compare it.
#include "common.hpp"
#include "kernels.hpp"

namespace rsvd {

namespace {

// Sum over aligned groups of 8 (TPP = 8) or 16 (TPP = 16) lanes with DPP moves (no LDS traffic):
// quad_perm [1,0,3,2] and [2,3,0,1] sum quads, row_half_mirror joins the two quads of 8 lanes,
// row_mirror joins the two halves of 16.
template <int CTRL>
__device__ __forceinline__ double dpp_c(double v) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)u, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), CTRL, 0xF, 0xF, false);
    return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
template <int CTRL>
__device__ __forceinline__ float dpp_c(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
template <int TPP, typename C>
__device__ __forceinline__ C group_sum(C v) {
    v += dpp_c<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp_c<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dpp_c<0x141>(v);  // row_half_mirror
    if (TPP == 16) v += dpp_c<0x140>(v);  // row_mirror
    return v;
}

__device__ __forceinline__ double rsqrt_c(double d) {
    const double y = __builtin_amdgcn_rsq(d);
    return y * (1.5 - 0.5 * d * y * y);
}
__device__ __forceinline__ float rsqrt_c(float d) {
    const float y = __builtin_amdgcn_rsqf(d);
    return y * (1.5f - 0.5f * d * y * y);
}
__device__ __forceinline__ double rcp_c(double d) {
    double y = __builtin_amdgcn_rcp(d);
    y = y * (2.0 - d * y);
    return y * (2.0 - d * y);
}
__device__ __forceinline__ float rcp_c(float d) {
    const float y = __builtin_amdgcn_rcpf(d);
    return y * (2.0f - d * y);
}

template <typename C> struct Eps;
template <> struct Eps<double> {
    static constexpr double eps = 2.220446049250313e-16;
    static constexpr double quad2 = 1e-16;  // (1e-8)^2: rotation ratios below 1e-8 => converged next sweep
    static constexpr double lo = 1e-290, hi = 1e290;  // safe range of d^2 + 4 g^2
};
template <> struct Eps<float> {
    static constexpr double eps = 1.1920928955078125e-07;
    static constexpr double quad2 = 1e-8;   // (1e-4)^2
    static constexpr double lo = 1e-35, hi = 1e35;
};

template <typename C> struct Two;
template <> struct Two<double> { typedef double2 type; };
template <> struct Two<float> { typedef float2 type; };
// LDS vector of the column accesses: up to 16 B per lane, N elements dividing the CH rows a
// thread owns (so every access stays aligned)
template <typename C, int N> struct VecT { typedef C type; };
template <> struct VecT<float, 2> { typedef float2 type; };
template <> struct VecT<float, 4> { typedef float4 type; };
template <> struct VecT<double, 2> { typedef double2 type; };
template <typename C, int CH>
struct JVec {
    static constexpr int W = 16 / (int)sizeof(C);
    static constexpr int N = (CH % W == 0) ? W : ((CH % 2 == 0) ? 2 : 1);
    typedef typename VecT<C, N>::type type;
};

__device__ __forceinline__ void rr_pair(int round, int k, int N, int& p, int& q) {
    if (k == 0) {
        p = round;
        q = N - 1;
    } else {  // (round + k) mod (N - 1), (round - k) mod (N - 1) without an integer division
        p = round + k;
        p -= (p >= N - 1) ? N - 1 : 0;
        q = round - k + (N - 1);
        q -= (q >= N - 1) ? N - 1 : 0;
    }
}

// Thread layout: TPP threads per column pair, thread `sub` of a pair owns the CH = LP / TPP
// contiguous rows sub * CH .. (vector LDS accesses); columns are CS apart.
template <typename C, int LP>
struct JacobiShape {
    static constexpr int TPP = 16;  // threads per column pair (the round is issue-bound: more threads, shorter chains)
    static constexpr int CH = LP / TPP;                                // rows per thread (even)
    static constexpr int CS = LP + 16 / (int)sizeof(C);                // column stride: 16-B aligned, staggered banks
    static constexpr int NTHR = (LP / 2) * TPP;                        // one pair per TPP threads
};

template <typename C, int LP>
constexpr size_t svd_lds_bytes() {
    // X, J (C) -- later reused as the fp64 LP x LP U_w image -- then sig, v, nrm, rank, flags
    const size_t xj = (size_t)2 * LP * JacobiShape<C, LP>::CS * sizeof(C);
    const size_t ud = (size_t)LP * LP * sizeof(double);
    return (xj > ud ? xj : ud) + (size_t)3 * LP * sizeof(double) + (size_t)(LP + 4) * sizeof(int) + 64;
}

template <typename T, typename C, int LP>
__global__ __launch_bounds__((JacobiShape<C, LP>::NTHR)) void small_svd_kernel(const double* __restrict__ R, int l,
                                                        double* __restrict__ Uw, double* __restrict__ Vw,
                                                        T* __restrict__ S, int* __restrict__ info) {
    typedef JacobiShape<C, LP> SH;
    constexpr int TPP = SH::TPP, CH = SH::CH, CS = SH::CS;
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    C* X = reinterpret_cast<C*>(smem_raw);                  // [LP][CS]   X[c*CS + i]
    C* J = X + LP * CS;                                     // [LP][CS]
    constexpr size_t xj_bytes = (size_t)2 * LP * CS * sizeof(C);
    constexpr size_t ud_bytes = (size_t)LP * LP * sizeof(double);
    double* sig = reinterpret_cast<double*>(smem_raw + (xj_bytes > ud_bytes ? xj_bytes : ud_bytes));  // [LP]
    double* v = sig + LP;                                   // [LP] completion scratch
    C* nrm = reinterpret_cast<C*>(v + LP);                  // [LP] squared column norms
    int* rank = reinterpret_cast<int*>(nrm + LP);           // [LP]
    int* flags = rank + LP;                                 // [4]
    const int tid = threadIdx.x, nt = blockDim.x;

    // X = W (W[i][c] = R[c][i]), J = I
    for (int e = tid; e < LP * LP; e += nt) {
        const int c = e / LP, i = e % LP;
        X[c * CS + i] = (c < l && i < l) ? (C)R[c * LP + i] : C(0);
        J[c * CS + i] = (c == i && c < l) ? C(1) : C(0);
    }
    const int N = (l & 1) ? l + 1 : l;       // dummy zero column when l is odd (l < LP then)
    const int npairs = N / 2;
    const int pi = tid / TPP, sub = tid % TPP;
    const bool active = pi < npairs;
    const C tol = (C)((double)l * Eps<C>::eps);
    const C tol2 = tol * tol;
    int sweeps = 0;
    C negl = C(0);
    __syncthreads();
    for (; sweeps < 40; ++sweeps) {
        // exact squared norms at the start of every sweep (the rounds update them incrementally):
        // all LP columns before sweep 0 (negl below reads them); later sweeps take them in round 0,
        // whose pairs cover every live column, by the same DPP group sums as the dot products
        if (sweeps == 0)
            for (int c = tid; c < LP; c += nt) {
                C s2 = C(0);
                for (int i = 0; i < LP; ++i) s2 += X[c * CS + i] * X[c * CS + i];
                nrm[c] = s2;
            }
        if (tid == 0) {
            flags[0] = 0;
            flags[1] = 0;
        }
        __syncthreads();
        if (sweeps == 0) {  // ||W||_F^2 -> columns below (l eps)^2 ||W||_F^2 are numerically zero
            C f = C(0);
            for (int c = 0; c < LP; ++c) f += nrm[c];
            negl = f * (C)((double)l * l * Eps<C>::eps * Eps<C>::eps);
        }
        for (int round = 0; round < N - 1; ++round) {
            if (active) {
                int p, q;
                rr_pair(round, pi, N, p, q);
                // every LDS operand of the round is requested up front: one exposed latency
                C xp[CH], xq[CH], jp[CH], jq[CH];
                const int i0 = sub * CH;
                typedef typename JVec<C, CH>::type CV;
                constexpr int NV = JVec<C, CH>::N;
#pragma unroll
                for (int t = 0; t < CH; t += NV) {
                    const CV a4 = *reinterpret_cast<const CV*>(X + p * CS + i0 + t);
                    const CV b4 = *reinterpret_cast<const CV*>(X + q * CS + i0 + t);
                    const CV c4 = *reinterpret_cast<const CV*>(J + p * CS + i0 + t);
                    const CV d4 = *reinterpret_cast<const CV*>(J + q * CS + i0 + t);
                    const C* ap = reinterpret_cast<const C*>(&a4);
                    const C* bp = reinterpret_cast<const C*>(&b4);
                    const C* cp = reinterpret_cast<const C*>(&c4);
                    const C* dp = reinterpret_cast<const C*>(&d4);
#pragma unroll
                    for (int v = 0; v < NV; ++v) {
                        xp[t + v] = ap[v];
                        xq[t + v] = bp[v];
                        jp[t + v] = cp[v];
                        jq[t + v] = dp[v];
                    }
                }
                C a, b;
                if (round == 0 && sweeps > 0) {
                    C a0 = C(0), b0 = C(0);
#pragma unroll
                    for (int t = 0; t < CH; ++t) {
                        a0 += xp[t] * xp[t];
                        b0 += xq[t] * xq[t];
                    }
                    a = group_sum<TPP>(a0);
                    b = group_sum<TPP>(b0);
                    if (sub == 0) {  // kept when the pair does not rotate
                        nrm[p] = a;
                        nrm[q] = b;
                    }
                } else {
                    a = nrm[p];
                    b = nrm[q];
                }
                C g0 = C(0), g1 = C(0);
#pragma unroll
                for (int t = 0; t < CH; ++t) {
                    if (t & 1) g1 += xp[t] * xq[t];
                    else g0 += xp[t] * xq[t];
                }
                const C g = group_sum<TPP>(g0 + g1);
                const C gg = g * g, ab = a * b;
                if (g != C(0) && gg > tol2 * ab && a > negl && b > negl) {
                    // t = sign(zeta) / (|zeta| + sqrt(1 + zeta^2)), zeta = (b - a) / (2 g), written as
                    // t = sign(d g) |2g| / (|d| + sqrt(d^2 + 4 g^2)) with d = b - a (no overflow for small g)
                    const C d = b - a, g2 = C(2) * g;
                    const C hyp2 = d * d + g2 * g2;
                    C tmag;
                    if (hyp2 > (C)Eps<C>::lo && hyp2 < (C)Eps<C>::hi) {
                        const C hyp = hyp2 * rsqrt_c(hyp2);
                        tmag = fabs(g2) * rcp_c(fabs(d) + hyp);
                    } else {  // d^2 + 4 g^2 under/overflows: same formula on scaled operands
                        const C sc = fmax(fabs(d), fabs(g2));
                        const C ds = fabs(d) / sc, gs = fabs(g2) / sc;
                        tmag = gs / (ds + sqrt(ds * ds + gs * gs));
                    }
                    const C t = ((d >= C(0)) == (g >= C(0))) ? tmag : -tmag;
                    const C cs = rsqrt_c(C(1) + t * t), sn = cs * t;
#pragma unroll
                    for (int u = 0; u < CH; u += NV) {
                        CV np, nq, mp, mq;
                        C* npp = reinterpret_cast<C*>(&np);
                        C* nqp = reinterpret_cast<C*>(&nq);
                        C* mpp = reinterpret_cast<C*>(&mp);
                        C* mqp = reinterpret_cast<C*>(&mq);
#pragma unroll
                        for (int v = 0; v < NV; ++v) {
                            npp[v] = cs * xp[u + v] - sn * xq[u + v];
                            nqp[v] = sn * xp[u + v] + cs * xq[u + v];
                            mpp[v] = cs * jp[u + v] - sn * jq[u + v];
                            mqp[v] = sn * jp[u + v] + cs * jq[u + v];
                        }
                        *reinterpret_cast<CV*>(X + p * CS + i0 + u) = np;
                        *reinterpret_cast<CV*>(X + q * CS + i0 + u) = nq;
                        *reinterpret_cast<CV*>(J + p * CS + i0 + u) = mp;
                        *reinterpret_cast<CV*>(J + q * CS + i0 + u) = mq;
                    }
                    if (sub == 0) {
                        nrm[p] = a - t * g;
                        nrm[q] = b + t * g;
                        flags[0] = 1;
                        if (gg > (C)Eps<C>::quad2 * ab) flags[1] = 1;  // not yet in the quadratic regime
                    }
                }
            }
            __syncthreads();
        }
        // Stop when a sweep rotated nothing, or when every rotation of the sweep was already
        // tiny (cyclic Jacobi converges quadratically: the next sweep would fall under tol).
        if (flags[0] == 0 || flags[1] == 0) {
            ++sweeps;
            break;
        }
        __syncthreads();
    }
    // singular values = column norms (accumulated in fp64); negligible or non-finite -> 0 (then
    // completed to an orthonormal U_w below)
    for (int c = tid; c < LP; c += nt) {
        double s2 = 0.0;
        if (c < l)
            for (int i = 0; i < LP; ++i) s2 += (double)X[c * CS + i] * (double)X[c * CS + i];
        const double sv = sqrt(s2);
        sig[c] = (isfinite(sv) && s2 > (double)negl) ? sv : 0.0;
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
    // U_w (fp64) is assembled in LDS over the X/J area: Ud[k][i] = u_k[i] (column k contiguous)
    double* Ud = reinterpret_cast<double*>(smem_raw);  // [LP][LP], reuses X/J after a copy of J
    for (int e = tid; e < LP * LP; e += nt) Vw[e] = 0.0;
    __syncthreads();
    for (int e = tid; e < l * l; e += nt) {
        const int c = e / l, i = e % l;
        Vw[i * LP + rank[c]] = (double)J[c * CS + i];
    }
    // stash the normalised columns in registers before Ud overwrites X/J
    constexpr int PER = (LP * LP + SH::NTHR - 1) / SH::NTHR;
    double ureg[PER];
    int kreg[PER];
#pragma unroll
    for (int t = 0; t < PER; ++t) {
        const int e = tid + SH::NTHR * t;
        const int c = e / LP, i = e % LP;
        kreg[t] = -1;
        ureg[t] = 0.0;
        if (e < LP * LP && c < l && i < l && sig[c] > 0.0) {
            kreg[t] = rank[c] * LP + i;
            ureg[t] = (double)X[c * CS + i] / sig[c];
        }
    }
    __syncthreads();
    for (int e = tid; e < LP * LP; e += nt) Ud[e] = 0.0;
    __syncthreads();
#pragma unroll
    for (int t = 0; t < PER; ++t)
        if (kreg[t] >= 0) Ud[kreg[t]] = ureg[t];
    for (int c = tid; c < l; c += nt) S[rank[c]] = (T)sig[c];
    __syncthreads();
    // Exactly-zero singular values (rank-deficient or zero input): complete U_w to an orthonormal
    // basis, as the reference's U (a product of rotations) always is.  For each missing column k,
    // take the unit vector e_i least covered by the columns so far (its residual norm^2 is at
    // least (l - k) / l) and orthogonalise it twice -- O(l k) parallel work per column.
    int nz = 0;
    for (int c = 0; c < l; ++c) nz += (sig[c] > 0.0);
    for (int k = nz; k < l; ++k) {
        // coverage of row i by columns 0..k-1, argmin over i (rank tie-break by index)
        for (int i = tid; i < LP; i += nt) {
            double cov = 0.0;
            for (int j = 0; j < k; ++j) cov += Ud[j * LP + i] * Ud[j * LP + i];
            v[i] = (i < l) ? cov : 1e300;
        }
        __syncthreads();
        if (tid == 0) {
            int best = 0;
            for (int i = 1; i < l; ++i)
                if (v[i] < v[best]) best = i;
            flags[2] = best;
        }
        __syncthreads();
        const int cand = flags[2];
        for (int i = tid; i < LP; i += nt) Ud[k * LP + i] = (i == cand) ? 1.0 : 0.0;
        __syncthreads();
        for (int pass = 0; pass < 2; ++pass) {
            // dots d_j = <u_j, u_k> (one thread per j), then u_k -= sum_j d_j u_j (one thread per i)
            for (int j = tid; j < k; j += nt) {
                double d = 0.0;
                for (int i = 0; i < l; ++i) d += Ud[j * LP + i] * Ud[k * LP + i];
                v[j] = d;
            }
            __syncthreads();
            for (int i = tid; i < l; i += nt) {
                double x = Ud[k * LP + i];
                for (int j = 0; j < k; ++j) x -= v[j] * Ud[j * LP + i];
                Ud[k * LP + i] = x;
            }
            __syncthreads();
        }
        if (tid == 0) {
            double nv = 0.0;
            for (int i = 0; i < l; ++i) nv += Ud[k * LP + i] * Ud[k * LP + i];
            v[0] = 1.0 / sqrt(nv);
        }
        __syncthreads();
        const double sc = v[0];
        for (int i = tid; i < l; i += nt) Ud[k * LP + i] *= sc;
        __syncthreads();
    }
    for (int e = tid; e < LP * LP; e += nt) {
        const int i = e / LP, k = e % LP;
        Uw[e] = Ud[k * LP + i];  // Uw row-major [i][k]
    }
    if (tid == 0) info[0] = sweeps;
}

}  // namespace

template <typename T>
hipError_t launch_small_svd(const double* R, int l, int LP, double* Uw, double* Vw, T* S, int* info,
                            hipStream_t s) {
    typedef T C;  // compute in the panel precision: fp32 path -> fp32 Jacobi, fp64 path -> fp64
    switch (LP) {
#define CASE(L)                                                                                              \
    case L:                                                                                                  \
        hipLaunchKernelGGL((small_svd_kernel<T, C, L>), dim3(1), dim3(JacobiShape<C, L>::NTHR), (svd_lds_bytes<C, L>()), s, R, l, Uw, Vw, \
                           S, info);                                                                         \
        break;
        CASE(16) CASE(32) CASE(48) CASE(64)
#undef CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template hipError_t launch_small_svd<float>(const double*, int, int, double*, double*, float*, int*, hipStream_t);
template hipError_t launch_small_svd<double>(const double*, int, int, double*, double*, double*, int*, hipStream_t);

}  // namespace rsvd
