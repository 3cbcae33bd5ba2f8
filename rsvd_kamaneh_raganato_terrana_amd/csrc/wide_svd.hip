// wide_svd.hip -- the small SVD of the rSVD for sketch widths 128..512 (SVD<Jacobi>::compute on B,
// include/SVD_class.hpp:100-180).
//
// As in jacobi.hip, W = R^T (R = Q_B^T B^T, so B = W Q_B^T) is diagonalised by one-sided
// (Hestenes) Jacobi: X = W, J = I, rotate column pairs until the columns of X are orthogonal;
// then S = column norms (descending, the reference's selection sort :164-178), U_w = X / S,
// V_w = J.  For l > 64 the l x l problem no longer fits one workgroup, so the columns are cut
// into NB = LP/16 blocks of 16 and paired round-robin (NB/2 disjoint block pairs per round,
// NB - 1 rounds per sweep) over a persistent grid of NB/2 workgroups:
//   1. Gp = X_pair^T X_pair (32 x 32, fp64 MFMA over the LP rows; exact column dot products, the
//      same quantities the one-sided rotation angles use);
//   2. the 32 x 32 symmetric eigenproblem of Gp by cyclic Jacobi in LDS (16 disjoint rotations
//      per inner round, accumulated into Jp) -- each inner rotation is the one-sided rotation of
//      the corresponding column pair of X, with the same angle formula as jacobi.hip;
//   3. X_pair <- X_pair Jp, J_pair <- J_pair Jp (fp64 MFMA), into the other half of a double
//      buffer (every column is owned by exactly one pair per round).
// Rounds are separated by an agent-scope grid barrier (MI355X_MICROARCH.md "Workgroup dispatch
// ... inter-workgroup visibility": plain stores -> vmcnt(0) -> barrier -> release fence -> relaxed
// counter; acquire fence after the poll).  The grid (<= 16 workgroups) is always co-resident;
// every spin is bounded and reports a timeout instead of hanging.  A sweep in which no pair has
// an off-diagonal |g| > l eps sqrt(a b) (or only rotations already in the quadratic regime)
// ends the iteration, as in jacobi.hip.
#include "common.hpp"
#include "kernels.hpp"
#include "wide.hpp"

namespace rsvd {

namespace {

typedef Mfma<double> MD;
constexpr double kEps = 2.220446049250313e-16;
constexpr int kMaxSweeps = 30;
// sync layout (unsigned): [0] barrier counter, [1] abort, [2] final parity, [4 + s] sweep s rotated,
// [36 + s] sweep s had rotations outside the quadratic regime
constexpr int kSyncWords = 72;

__device__ __forceinline__ void rr_pair(int round, int k, int N, int& p, int& q) {
    if (k == 0) {
        p = round;
        q = N - 1;
    } else {
        p = (round + k) % (N - 1);
        q = (round - k + (N - 1)) % (N - 1);
    }
}

// Returns false on timeout (then every workgroup bails out through the abort word).
__device__ bool grid_barrier(unsigned* sync, unsigned target) {
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
            __builtin_amdgcn_s_sleep(2);
            if ((++spins & 1023) == 0 &&
                (__hip_atomic_load(sync + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 || spins > (1l << 26))) {
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

// Rotation of the pair (a = |x_p|^2, b = |x_q|^2, g = x_p.x_q): x_p' = c x_p - s x_q, x_q' = s x_p + c x_q
// zeroes the cross term (jacobi.hip formula).
__device__ __forceinline__ void jacobi_angle(double a, double b, double g, double& c, double& s) {
    const double d = b - a, g2 = 2.0 * g;
    const double sc = fmax(fabs(d), fabs(g2));
    const double ds = fabs(d) / sc, gs = fabs(g2) / sc;
    const double tmag = gs / (ds + sqrt(ds * ds + gs * gs));
    const double t = ((d >= 0.0) == (g >= 0.0)) ? tmag : -tmag;
    c = 1.0 / sqrt(1.0 + t * t);
    s = c * t;
}

constexpr int GS = 33;  // LDS pitch of the 32 x 32 blocks

__global__ __launch_bounds__(256) void block_jacobi_kernel(const double* __restrict__ R, int l, int LP,
                                                           double* __restrict__ Xb, double* __restrict__ Jb,
                                                           unsigned* __restrict__ sync, int* __restrict__ info) {
    __shared__ double Gs[32 * GS], Jp[32 * GS];
    __shared__ double cs_[16], sn_[16];
    __shared__ int flags[4];
    __shared__ double fro;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 15, h = lane >> 4;
    const int nwg = gridDim.x, wg = blockIdx.x;
    const int NB = LP / 16;
    const int64_t L2 = (int64_t)LP * LP;
    const double tol = (double)l * kEps, tol2 = tol * tol, quad2 = 1e-16;

    // X (column-major, X[c][i] = W[i][c] = R[c][i]) and J = I into buffer 0: rows of this workgroup
    for (int64_t e = (int64_t)wg * 256 + tid; e < L2; e += (int64_t)nwg * 256) {
        const int c = (int)(e / LP), i = (int)(e % LP);
        Xb[e] = (c < l && i < l) ? R[e] : 0.0;
        Jb[e] = (c == i && c < l) ? 1.0 : 0.0;
    }
    // ||W||_F^2 (every workgroup, same order) -> negligible-column threshold
    if (tid == 0) fro = 0.0;
    __syncthreads();
    {
        double part = 0.0;
        for (int64_t e = tid; e < L2; e += 256) {
            const int c = (int)(e / LP), i = (int)(e % LP);
            const double v = (c < l && i < l) ? R[e] : 0.0;
            part += v * v;
        }
        part = warp_sum(part);
        if (lane == 0) atomicAdd(&fro, part);
    }
    __syncthreads();
    const double negl = fro * (double)l * l * kEps * kEps;
    unsigned bar = 0;
    if (!grid_barrier(sync, (unsigned)nwg * ++bar)) {
        if (tid == 0) info[2] = 1;
        return;
    }

    int par = 0, sweeps = 0;
    for (int sweep = 0; sweep < kMaxSweeps; ++sweep) {
        for (int round = 0; round < NB - 1; ++round) {
            int P, Q;
            rr_pair(round, wg, NB, P, Q);
            const double* Xs = Xb + (size_t)par * L2;
            const double* Js = Jb + (size_t)par * L2;
            double* Xd = Xb + (size_t)(1 - par) * L2;
            double* Jd = Jb + (size_t)(1 - par) * L2;
            auto col = [&](int k) { return k < 16 ? 16 * P + k : 16 * Q + k - 16; };
            // 1. Gp = X_pair^T X_pair: wave w -> 16 x 16 tile (w >> 1, w & 1)
            {
                const int ta = w >> 1, tb = w & 1;
                const double* xa = Xs + (int64_t)col(16 * ta + r) * LP;
                const double* xb = Xs + (int64_t)col(16 * tb + r) * LP;
                f64x4 acc = MD::zero();
                for (int i0 = 0; i0 < LP; i0 += 4) acc = MD::mma(xa[i0 + h], xb[i0 + h], acc);
#pragma unroll
                for (int j = 0; j < 4; ++j) Gs[(16 * ta + MD::row(h, j)) * GS + 16 * tb + r] = acc[j];
            }
            if (tid < 4) flags[tid] = 0;
            for (int e = tid; e < 32 * 32; e += 256) Jp[(e / 32) * GS + e % 32] = (e / 32 == e % 32) ? 1.0 : 0.0;
            __syncthreads();
            // 2. convergence test on the fresh Gram: any pair above threshold?
            for (int e = tid; e < 32 * 32; e += 256) {
                const int i = e / 32, j = e % 32;
                if (i < j) {
                    const double a = Gs[i * GS + i], b = Gs[j * GS + j], g = Gs[i * GS + j];
                    if (g != 0.0 && g * g > tol2 * a * b && a > negl && b > negl) {
                        flags[0] = 1;
                        if (g * g > quad2 * a * b) flags[1] = 1;
                    }
                }
            }
            __syncthreads();
            const bool work = flags[0] != 0;
            if (work) {
                if (tid == 0) {
                    __hip_atomic_store(sync + 4 + sweep, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (flags[1]) __hip_atomic_store(sync + 36 + sweep, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                // 3. cyclic Jacobi on Gp (two-sided updates), accumulated into Jp
                for (int isw = 0; isw < 4; ++isw) {
                    if (tid == 0) flags[2] = 0;
                    __syncthreads();
                    for (int ir = 0; ir < 31; ++ir) {
                        if (tid < 16) {
                            int p, q;
                            rr_pair(ir, tid, 32, p, q);
                            const double a = Gs[p * GS + p], b = Gs[q * GS + q], g = Gs[p * GS + q];
                            double c = 1.0, s = 0.0;
                            if (g != 0.0 && g * g > tol2 * a * b && a > negl && b > negl) {
                                jacobi_angle(a, b, g, c, s);
                                flags[2] = 1;
                            }
                            cs_[tid] = c;
                            sn_[tid] = s;
                        }
                        __syncthreads();
                        // columns p, q of Gs and Jp
                        for (int e = tid; e < 16 * 32; e += 256) {
                            const int k = e / 32, i = e % 32;
                            const double c = cs_[k], s = sn_[k];
                            if (s == 0.0) continue;
                            int p, q;
                            rr_pair(ir, k, 32, p, q);
                            const double gp = Gs[i * GS + p], gq = Gs[i * GS + q];
                            Gs[i * GS + p] = c * gp - s * gq;
                            Gs[i * GS + q] = s * gp + c * gq;
                            const double jp = Jp[i * GS + p], jq = Jp[i * GS + q];
                            Jp[i * GS + p] = c * jp - s * jq;
                            Jp[i * GS + q] = s * jp + c * jq;
                        }
                        __syncthreads();
                        // rows p, q of Gs
                        for (int e = tid; e < 16 * 32; e += 256) {
                            const int k = e / 32, i = e % 32;
                            const double c = cs_[k], s = sn_[k];
                            if (s == 0.0) continue;
                            int p, q;
                            rr_pair(ir, k, 32, p, q);
                            const double gp = Gs[p * GS + i], gq = Gs[q * GS + i];
                            Gs[p * GS + i] = c * gp - s * gq;
                            Gs[q * GS + i] = s * gp + c * gq;
                        }
                        __syncthreads();
                    }
                    if (flags[2] == 0) break;
                }
                // 4. X_pair Jp, J_pair Jp -> destination buffer (wave w: row tiles w, w+4, ...)
                for (int mtx = 0; mtx < 2; ++mtx) {
                    const double* S = mtx ? Js : Xs;
                    double* D = mtx ? Jd : Xd;
                    for (int it = w; it < LP / 16; it += 4) {
                        const int i0 = 16 * it;
                        f64x4 acc[2] = {MD::zero(), MD::zero()};
#pragma unroll
                        for (int kk = 0; kk < 8; ++kk) {
                            const double a = S[(int64_t)col(4 * kk + h) * LP + i0 + r];
                            acc[0] = MD::mma(a, Jp[(4 * kk + h) * GS + r], acc[0]);
                            acc[1] = MD::mma(a, Jp[(4 * kk + h) * GS + 16 + r], acc[1]);
                        }
#pragma unroll
                        for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                            for (int j = 0; j < 4; ++j) D[(int64_t)col(16 * ct + r) * LP + i0 + MD::row(h, j)] = acc[ct][j];
                    }
                }
            } else {
                for (int e = tid; e < 32 * LP; e += 256) {
                    const int64_t o = (int64_t)col(e / LP) * LP + e % LP;
                    Xd[o] = Xs[o];
                    Jd[o] = Js[o];
                }
            }
            par = 1 - par;
            if (!grid_barrier(sync, (unsigned)nwg * ++bar)) {
                if (tid == 0) info[2] = 1;
                return;
            }
        }
        ++sweeps;
        const unsigned rot = __hip_atomic_load(sync + 4 + sweep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned big = __hip_atomic_load(sync + 36 + sweep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (rot == 0 || big == 0) break;
    }
    if (wg == 0 && tid == 0) {
        sync[2] = (unsigned)par;
        info[0] = sweeps;
    }
}

// S, U_w = X / S (sorted descending, completed to orthonormal where S = 0), V_w = J.  One
// workgroup; Uw / Vw row-major [row][col], LP x LP.
template <typename T>
__global__ __launch_bounds__(1024) void block_jacobi_finish_kernel(const double* __restrict__ Xb,
                                                                   const double* __restrict__ Jb, int l, int LP,
                                                                   const unsigned* __restrict__ sync,
                                                                   double* __restrict__ Uw, double* __restrict__ Vw,
                                                                   T* __restrict__ S) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    double* sig = reinterpret_cast<double*>(smem_raw);  // [LP]
    double* v = sig + LP;                               // [LP]
    int* rank = reinterpret_cast<int*>(v + LP);         // [LP]
    int* misc = rank + LP;                              // [4]
    const int tid = threadIdx.x, nt = blockDim.x;
    const int64_t L2 = (int64_t)LP * LP;
    const int par = (int)sync[2];
    const double* X = Xb + (size_t)par * L2;
    const double* J = Jb + (size_t)par * L2;
    if (tid == 0) v[0] = 0.0;
    __syncthreads();
    for (int c = tid; c < LP; c += nt) {
        double s2 = 0.0;
        if (c < l)
            for (int i = 0; i < LP; ++i) s2 += X[(int64_t)c * LP + i] * X[(int64_t)c * LP + i];
        sig[c] = s2;
    }
    __syncthreads();
    if (tid == 0) {
        double f = 0.0;
        for (int c = 0; c < l; ++c) f += sig[c];
        misc[1] = 0;
        v[0] = f * (double)l * l * kEps * kEps;  // negligible column norm^2
    }
    __syncthreads();
    const double negl = v[0];
    __syncthreads();
    for (int c = tid; c < LP; c += nt) {
        const double s2 = sig[c];
        const double sv = sqrt(s2);
        sig[c] = (c < l && isfinite(sv) && s2 > negl) ? sv : 0.0;
    }
    __syncthreads();
    for (int c = tid; c < l; c += nt) {
        int rk = 0;
        const double sc = sig[c];
        for (int d = 0; d < l; ++d) rk += (sig[d] > sc) || (sig[d] == sc && d < c);
        rank[c] = rk;
    }
    __syncthreads();
    for (int64_t e = tid; e < L2; e += nt) {
        Uw[e] = 0.0;
        Vw[e] = 0.0;
    }
    __syncthreads();
    for (int64_t e = tid; e < (int64_t)l * LP; e += nt) {
        const int c = (int)(e / LP), i = (int)(e % LP);
        if (i < l) {
            Vw[(int64_t)i * LP + rank[c]] = J[(int64_t)c * LP + i];
            if (sig[c] > 0.0) Uw[(int64_t)i * LP + rank[c]] = X[(int64_t)c * LP + i] / sig[c];
        }
    }
    for (int c = tid; c < l; c += nt) S[rank[c]] = (T)sig[c];
    __syncthreads();
    // complete U_w for zero singular values (as jacobi.hip): least-covered unit vector, CGS2
    int nz = 0;
    for (int c = 0; c < l; ++c) nz += (sig[c] > 0.0);
    for (int k = nz; k < l; ++k) {
        for (int i = tid; i < LP; i += nt) {
            double cov = 0.0;
            for (int j = 0; j < k; ++j) cov += Uw[(int64_t)i * LP + j] * Uw[(int64_t)i * LP + j];
            v[i] = (i < l) ? cov : 1e300;
        }
        __syncthreads();
        if (tid == 0) {
            int best = 0;
            for (int i = 1; i < l; ++i)
                if (v[i] < v[best]) best = i;
            misc[0] = best;
        }
        __syncthreads();
        const int cand = misc[0];
        for (int i = tid; i < LP; i += nt) Uw[(int64_t)i * LP + k] = (i == cand) ? 1.0 : 0.0;
        __syncthreads();
        for (int pass = 0; pass < 2; ++pass) {
            for (int j = tid; j < k; j += nt) {
                double d = 0.0;
                for (int i = 0; i < l; ++i) d += Uw[(int64_t)i * LP + j] * Uw[(int64_t)i * LP + k];
                v[j] = d;
            }
            __syncthreads();
            for (int i = tid; i < l; i += nt) {
                double x = Uw[(int64_t)i * LP + k];
                for (int j = 0; j < k; ++j) x -= v[j] * Uw[(int64_t)i * LP + j];
                Uw[(int64_t)i * LP + k] = x;
            }
            __syncthreads();
        }
        if (tid == 0) {
            double nv = 0.0;
            for (int i = 0; i < l; ++i) nv += Uw[(int64_t)i * LP + k] * Uw[(int64_t)i * LP + k];
            v[0] = 1.0 / sqrt(nv);
        }
        __syncthreads();
        const double sc = v[0];
        for (int i = tid; i < l; i += nt) Uw[(int64_t)i * LP + k] *= sc;
        __syncthreads();
    }
}

}  // namespace

template <typename T>
hipError_t launch_block_jacobi(const double* R, int l, int LP, double* X, double* J, double* Uw, double* Vw, T* S,
                               unsigned* sync, int* info, hipStream_t s) {
    if (LP % 32 || LP < 64 || LP > 512) return hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(sync, 0, kSyncWords * sizeof(unsigned), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(block_jacobi_kernel, dim3(LP / 32), dim3(256), 0, s, R, l, LP, X, J, sync, info);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    const size_t lds = (size_t)LP * 8 * 2 + (size_t)LP * 4 + 64;
    hipLaunchKernelGGL((block_jacobi_finish_kernel<T>), dim3(1), dim3(1024), lds, s, X, J, l, LP, sync, Uw, Vw, S);
    return hipGetLastError();
}

template hipError_t launch_block_jacobi<float>(const double*, int, int, double*, double*, double*, double*, float*,
                                               unsigned*, int*, hipStream_t);
template hipError_t launch_block_jacobi<double>(const double*, int, int, double*, double*, double*, double*, double*,
                                                unsigned*, int*, hipStream_t);

}  // namespace rsvd
