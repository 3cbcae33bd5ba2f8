// proj.hip -- the rSVD projections on MFMA (gfx950).
//
//   proj_nn:  Y = A * X      (A m x n col-major, X n x LP row-major panel)   src/rSVD.cpp:59,66
//   proj_tn:  Z = A^T * Q    (Q m x LP panel, Z n x LP panel)                src/rSVD.cpp:63,89
//                                                                           (B = Q^T A is taken
//                                                                            as B^T = A^T Q)
// Both stream A exactly once per launch; the skinny panel (<= a few MB) is re-read from L2.
// Arithmetic intensity is 2*l flop per A element, i.e. l/2 flop/B for f32 A: MFMA-bound for
// l >= 64 on fp32 inputs (ridge 157.3 TF / 8 TB/s = 19.7 flop/B), HBM-bound for narrow panels.
//
// Tiling (16x16x4 MFMA, f32 or f64 in; operand maps in common.hpp):
//  * NN: lane (r, h) loads one 16-B vector A[i0 + VW*r .. +VW-1][k0 + h] (VW = 4 f32 / 2 f64),
//    i.e. 16 lanes read 256 contiguous bytes of one A column.  Vector element t feeds MFMA t,
//    whose tile row r is global row i0 + VW*r + t (a row permutation undone in the epilogue).
//    A wave owns WR = 16*VW rows x LP columns; the 4 waves of a workgroup interleave the K
//    steps and are summed through LDS at the end; K is further split over workgroups into
//    fp-T slabs that launch_sum_slabs (util.hip) adds up (deterministic order).
//  * TN: lane (r, h) loads A[i0 + VW*h .. +VW-1][j0 + r] (the reduction index i is the
//    contiguous one), element t is k-slot h of MFMA t; the wave owns 16*JT output rows
//    (columns of A) x LP.  Same wave/LDS/slab reduction over the m rows.
#include "common.hpp"
#include "kernels.hpp"

namespace rsvd {

namespace {

constexpr int kWaves = 4;
#ifndef RSVD_PDTN
#define RSVD_PDTN 8
#endif
// k-steps of A kept in flight per wave (register prefetch ring); measured on C2 (kernel_lab):
// NN 8 with the loads issued before the step's MFMAs, TN 8 (its steps are twice as wide)
constexpr int kPrefetchNN = 8;
constexpr int kPrefetchTN = RSVD_PDTN;

template <typename T>
__device__ __forceinline__ typename Vec16<T>::type load_vec_guarded(const T* __restrict__ col, int64_t i,
                                                                  int64_t lim, bool vec_ok) {
    typedef typename Vec16<T>::type V;
    constexpr int VW = Vec16<T>::N;
    V v;
    T* e = reinterpret_cast<T*>(&v);
    if (vec_ok && i + VW <= lim) {
        v = *reinterpret_cast<const V*>(col + i);
    } else {
#pragma unroll
        for (int t = 0; t < VW; ++t) e[t] = (i + t < lim) ? col[i + t] : T(0);
    }
    return v;
}

// ------------------------------------------------------------------------------------------------
template <typename T, int LP>
__global__ __launch_bounds__(kWave* kWaves) void proj_nn_kernel(
    const T* __restrict__ A, int64_t lda, int64_t m, int64_t n, const T* __restrict__ X,
    T* __restrict__ out, int64_t slab_stride, int64_t kchunk, int nrowblk, int vec_ok, int ldp) {
    typedef Mfma<T> M;
    typedef typename M::acc_t acc_t;
    typedef typename Vec16<T>::type V;
    constexpr int VW = Vec16<T>::N;
    constexpr int WR = 16 * VW;
    constexpr int G = LP / 16;
    // PERM (fp32, LP = 64): MFMA tile g, column r holds panel column 4r + g, so a lane's four
    // B values of a k are one 16-B load; the epilogue maps the columns back.
    constexpr bool PERM = sizeof(T) == 4 && G == 4;
    auto pcol = [](int rr, int g) { return PERM ? 4 * rr + g : 16 * g + rr; };
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    T* red = reinterpret_cast<T*>(smem_raw);  // [kWaves][WR][LP]

    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = lane & 15, h = lane >> 4;
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int rb = bid % nrowblk, s = bid / nrowblk;
    const int64_t i0 = (int64_t)rb * WR;
    const int64_t kbeg = (int64_t)s * kchunk;
    const int64_t kend = (kbeg + kchunk < n) ? kbeg + kchunk : n;
    const int64_t row = i0 + VW * r;

    acc_t acc[VW][G];
#pragma unroll
    for (int t = 0; t < VW; ++t)
#pragma unroll
        for (int g = 0; g < G; ++g) acc[t][g] = M::zero();

    // This wave's k-steps (4 k each, interleaved with the other waves), register-prefetched PD
    // steps ahead so that enough A bytes are in flight per CU to cover HBM latency.  Steps whose
    // 4 k values are all in range (and the row tile full, vector loads legal) run a branch-free
    // ring with pointer-bumped loads; the remaining steps take the guarded path.
    constexpr int PD = kPrefetchNN;
    const int64_t kstep = 4 * kWaves, kfirst = kbeg + 4 * w;
    const int nst = (kfirst < kend) ? (int)((kend - kfirst + kstep - 1) / kstep) : 0;
    const bool fast_rows = vec_ok && i0 + WR <= m;  // wave-uniform: MFMAs need every lane on one path
    const int nfull = (fast_rows && kfirst + 3 < kend) ? (int)((kend - kfirst - 4) / kstep) + 1 : 0;
    auto mma_step = [&](const V& a, const T* b) {
#pragma unroll
        for (int t = 0; t < VW; ++t) {
            const T at = Vec16<T>::get(a, t);
#pragma unroll
            for (int g = 0; g < G; ++g) acc[t][g] = M::mma(at, b[g], acc[t][g]);
        }
    };
    int st = 0;
    if (nfull >= PD) {
        V pa[PD];
        T pb[PD][G];
        const int64_t astride = kstep * lda, xstride = kstep * ldp;
        const T* ap = A + (kfirst + h) * lda + row;
        const T* xp = X + (kfirst + h) * ldp + (PERM ? 4 * r : r);
        auto load_fast = [&](V& a, T* b) {
            a = *reinterpret_cast<const V*>(ap);
            if constexpr (PERM) {
                const float4 x4 = *reinterpret_cast<const float4*>(xp);
                b[0] = x4.x; b[1] = x4.y; b[2] = x4.z; b[3] = x4.w;
            } else {
#pragma unroll
                for (int g = 0; g < G; ++g) b[g] = xp[16 * g];
            }
            ap += astride;
            xp += xstride;
        };
#pragma unroll
        for (int u = 0; u < PD; ++u) load_fast(pa[u], pb[u]);
        for (; st + 2 * PD <= nfull; st += PD) {
#pragma unroll
            for (int u = 0; u < PD; ++u) {
                const V a = pa[u];  // next load issued before this step's MFMAs
                T b[G];
#pragma unroll
                for (int g = 0; g < G; ++g) b[g] = pb[u][g];
                load_fast(pa[u], pb[u]);
                mma_step(a, b);
            }
        }
#pragma unroll
        for (int u = 0; u < PD; ++u) mma_step(pa[u], pb[u]);
        st += PD;
    }
    for (; st < nst; ++st) {  // guarded tail (and short K ranges)
        const int64_t k = kfirst + (int64_t)st * kstep + h;
        V a;
        T b[G];
        if (k < kend) {
            a = load_vec_guarded<T>(A + k * lda, row, m, vec_ok);
            const T* xr = X + k * ldp;
#pragma unroll
            for (int g = 0; g < G; ++g) b[g] = xr[pcol(r, g)];
        } else {
            T* e = reinterpret_cast<T*>(&a);
#pragma unroll
            for (int t = 0; t < VW; ++t) e[t] = T(0);
#pragma unroll
            for (int g = 0; g < G; ++g) b[g] = T(0);
        }
        mma_step(a, b);
    }

    // wave partials -> LDS [w][local row][col]
    T* mine = red + (size_t)w * WR * LP;
#pragma unroll
    for (int t = 0; t < VW; ++t)
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int lr = VW * M::row(h, j) + t;
                mine[lr * LP + pcol(r, g)] = acc[t][g][j];
            }
    __syncthreads();
    T* dst = out + (int64_t)s * slab_stride;
    for (int e = threadIdx.x * VW; e < WR * LP; e += blockDim.x * VW) {
        V sum = *reinterpret_cast<const V*>(red + e);
        T* sp = reinterpret_cast<T*>(&sum);
#pragma unroll
        for (int ww = 1; ww < kWaves; ++ww) {
            const V o = *reinterpret_cast<const V*>(red + (size_t)ww * WR * LP + e);
            const T* op = reinterpret_cast<const T*>(&o);
#pragma unroll
            for (int t = 0; t < VW; ++t) sp[t] += op[t];
        }
        const int lr = e / LP;
        if (i0 + lr < m) *reinterpret_cast<V*>(dst + (i0 + lr) * ldp + (e % LP)) = sum;
    }
}

// ------------------------------------------------------------------------------------------------
template <typename T, int LP, int JT>
__global__ __launch_bounds__(kWave* kWaves) void proj_tn_kernel(
    const T* __restrict__ A, int64_t lda, int64_t m, int64_t n, const T* __restrict__ Q,
    T* __restrict__ out, int64_t slab_stride, int64_t ichunk, int ncolblk, int vec_ok, int ldp) {
    typedef Mfma<T> M;
    typedef typename M::acc_t acc_t;
    typedef typename Vec16<T>::type V;
    constexpr int VW = Vec16<T>::N;
    constexpr int G = LP / 16;
    constexpr int WJ = 16 * JT;
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    T* red = reinterpret_cast<T*>(smem_raw);  // [kWaves][WJ][LP]

    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = lane & 15, h = lane >> 4;
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int cb = bid % ncolblk, s = bid / ncolblk;
    const int64_t j0 = (int64_t)cb * WJ;
    const int64_t ibeg = (int64_t)s * ichunk;
    const int64_t iend = (ibeg + ichunk < m) ? ibeg + ichunk : m;

    acc_t acc[JT][G];
#pragma unroll
    for (int jt = 0; jt < JT; ++jt)
#pragma unroll
        for (int g = 0; g < G; ++g) acc[jt][g] = M::zero();

    constexpr int ISTEP = 4 * VW;  // rows of A consumed per MFMA group
    constexpr int PD = kPrefetchTN;
    constexpr bool PERM = sizeof(T) == 4 && G == 4;  // as in proj_nn: column 4r + g of the panel
    const int64_t istep = (int64_t)ISTEP * kWaves, ifirst = ibeg + ISTEP * w;
    const int nst = (ifirst < iend) ? (int)((iend - ifirst + istep - 1) / istep) : 0;
    auto mma_step = [&](const V* a, T (*b)[G]) {
#pragma unroll
        for (int t = 0; t < VW; ++t)
#pragma unroll
            for (int jt = 0; jt < JT; ++jt) {
                const T at = Vec16<T>::get(a[jt], t);
#pragma unroll
                for (int g = 0; g < G; ++g) acc[jt][g] = M::mma(at, b[t][g], acc[jt][g]);
            }
    };
    // full steps: all ISTEP rows below iend, all JT column tiles inside n, vector loads legal
    const bool fast_cols = vec_ok && j0 + WJ <= n;
    const int nfull = (fast_cols && ifirst + ISTEP <= iend) ? (int)((iend - ifirst - ISTEP) / istep) + 1 : 0;
    int st = 0;
    if (nfull >= PD) {
        V pa[PD][JT];
        T pb[PD][VW][G];
        const T* ap = A + (j0 + r) * lda + ifirst + VW * h;
        const T* qp = Q + (ifirst + VW * h) * ldp + (PERM ? 4 * r : r);
        const int64_t qstride = istep * ldp;
        auto load_fast = [&](V* a, T (*b)[G]) {
#pragma unroll
            for (int jt = 0; jt < JT; ++jt) a[jt] = *reinterpret_cast<const V*>(ap + (int64_t)16 * jt * lda);
#pragma unroll
            for (int t = 0; t < VW; ++t) {
                if constexpr (PERM) {
                    const float4 q4 = *reinterpret_cast<const float4*>(qp + t * ldp);
                    b[t][0] = q4.x; b[t][1] = q4.y; b[t][2] = q4.z; b[t][3] = q4.w;
                } else {
#pragma unroll
                    for (int g = 0; g < G; ++g) b[t][g] = qp[t * ldp + 16 * g];
                }
            }
            ap += istep;
            qp += qstride;
        };
#pragma unroll
        for (int u = 0; u < PD; ++u) load_fast(pa[u], pb[u]);
        for (; st + 2 * PD <= nfull; st += PD) {
#pragma unroll
            for (int u = 0; u < PD; ++u) {
#ifdef RSVD_LFTN
                V a[JT];
                T b[VW][G];
#pragma unroll
                for (int jt = 0; jt < JT; ++jt) a[jt] = pa[u][jt];
#pragma unroll
                for (int t = 0; t < VW; ++t)
#pragma unroll
                    for (int g = 0; g < G; ++g) b[t][g] = pb[u][t][g];
                load_fast(pa[u], pb[u]);
                mma_step(a, b);
#else
                mma_step(pa[u], pb[u]);
                load_fast(pa[u], pb[u]);
#endif
            }
        }
#pragma unroll
        for (int u = 0; u < PD; ++u) mma_step(pa[u], pb[u]);
        st += PD;
    }
    for (; st < nst; ++st) {  // guarded tail
        const int64_t ib = ifirst + (int64_t)st * istep + VW * h;
        V a[JT];
        T b[VW][G];
#pragma unroll
        for (int jt = 0; jt < JT; ++jt) {
            const int64_t j = j0 + 16 * jt + r;
            if (j < n) {
                a[jt] = load_vec_guarded<T>(A + j * lda, ib, iend, vec_ok);
            } else {
                T* e = reinterpret_cast<T*>(&a[jt]);
#pragma unroll
                for (int t = 0; t < VW; ++t) e[t] = T(0);
            }
        }
#pragma unroll
        for (int t = 0; t < VW; ++t) {
            const int64_t i = ib + t;
            const T* qr = Q + i * ldp;
#pragma unroll
            for (int g = 0; g < G; ++g) b[t][g] = (i < iend) ? qr[PERM ? 4 * r + g : 16 * g + r] : T(0);
        }
        mma_step(a, b);
    }

    T* mine = red + (size_t)w * WJ * LP;
#pragma unroll
    for (int jt = 0; jt < JT; ++jt)
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                mine[(16 * jt + M::row(h, j)) * LP + (PERM ? 4 * r + g : 16 * g + r)] = acc[jt][g][j];
    __syncthreads();
    T* dst = out + (int64_t)s * slab_stride;
    for (int e = threadIdx.x * VW; e < WJ * LP; e += blockDim.x * VW) {
        V sum = *reinterpret_cast<const V*>(red + e);
        T* sp = reinterpret_cast<T*>(&sum);
#pragma unroll
        for (int ww = 1; ww < kWaves; ++ww) {
            const V o = *reinterpret_cast<const V*>(red + (size_t)ww * WJ * LP + e);
            const T* op = reinterpret_cast<const T*>(&o);
#pragma unroll
            for (int t = 0; t < VW; ++t) sp[t] += op[t];
        }
        const int lr = e / LP;
        if (j0 + lr < n) *reinterpret_cast<V*>(dst + (j0 + lr) * ldp + (e % LP)) = sum;
    }
}

int64_t round_up(int64_t x, int64_t q) { return (x + q - 1) / q * q; }

// Pick the K split so the grid has ~1 workgroup per CU (256 CUs) while every wave keeps at least
// ~8 MFMA groups of work and the slab traffic stays bounded.  Measured on C2 (tools/kernel_lab,
// grid target 128 / 192 / 256 / 320 / 512 / 1024 workgroups): 256 is best -- NN 29.7 us (splits 4),
// TN 27.0 us (splits 2) against 33.4 / 31.6 us at 512; odd split counts lose more.
ProjPlan make_plan(int64_t K, int blocks, int64_t kstep_wg) {
    ProjPlan p;
    p.blocks = blocks;
    int64_t splits = (256 + blocks - 1) / blocks;
    const int64_t max_by_work = K / (kstep_wg * 8);
    if (splits > max_by_work) splits = max_by_work;
    if (splits > 32) splits = 32;
    if (splits < 1) splits = 1;
    p.chunk = round_up((K + splits - 1) / splits, kstep_wg);
    p.splits = (int)((K + p.chunk - 1) / p.chunk);
    return p;
}

// ldp = panel row stride; ldp > LP runs the kernel once per LP-wide column group (wide sketches
// on fp32 / fp64 A: A is re-read ldp / LP times) and reduces all groups' slabs in one pass.
template <typename T, int LP>
hipError_t nn_dispatch(const T* A, int64_t lda, int64_t m, int64_t n, const T* X, const ProjPlan& p,
                       T* slabs, T* Y, hipStream_t s, hipEvent_t done, int ldp) {
    constexpr int VW = Vec16<T>::N;
    constexpr int WR = 16 * VW;
    const size_t lds = (size_t)kWaves * WR * LP * sizeof(T);
    T* out = (p.splits == 1) ? Y : slabs;
    const int64_t stride = m * ldp;
    const int vec_ok = (lda % VW == 0) && ((reinterpret_cast<uintptr_t>(A) & 15) == 0);
    for (int c0 = 0; c0 < ldp; c0 += LP) {
        hipLaunchKernelGGL((proj_nn_kernel<T, LP>), dim3(p.blocks * p.splits), dim3(kWave * kWaves), lds, s, A,
                           lda, m, n, X + c0, out + c0, stride, p.chunk, p.blocks, vec_ok, ldp);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    hipError_t e = hipSuccess;
    if (done) e = hipEventRecord(done, s);
    if (e != hipSuccess || p.splits == 1) return e;
    return launch_sum_slabs<T>(slabs, stride, p.splits, m * ldp, Y, s);
}

template <typename T, int LP>
hipError_t tn_dispatch(const T* A, int64_t lda, int64_t m, int64_t n, const T* Q, const ProjPlan& p,
                       T* slabs, T* Z, hipStream_t s, hipEvent_t done, int ldp) {
    constexpr int VW = Vec16<T>::N;
    constexpr int JT = 2;
    constexpr int WJ = 16 * JT;
    const size_t lds = (size_t)kWaves * WJ * LP * sizeof(T);
    T* out = (p.splits == 1) ? Z : slabs;
    const int64_t stride = n * ldp;
    const int vec_ok = (lda % VW == 0) && ((reinterpret_cast<uintptr_t>(A) & 15) == 0);
    for (int c0 = 0; c0 < ldp; c0 += LP) {
        hipLaunchKernelGGL((proj_tn_kernel<T, LP, JT>), dim3(p.blocks * p.splits), dim3(kWave * kWaves), lds, s,
                           A, lda, m, n, Q + c0, out + c0, stride, p.chunk, p.blocks, vec_ok, ldp);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    hipError_t e = hipSuccess;
    if (done) e = hipEventRecord(done, s);
    if (e != hipSuccess || p.splits == 1) return e;
    return launch_sum_slabs<T>(slabs, stride, p.splits, n * ldp, Z, s);
}

}  // namespace

template <typename T>
ProjPlan plan_proj_nn(int64_t m, int64_t n, int LP) {
    (void)LP;
    constexpr int WR = 16 * Vec16<T>::N;
    return make_plan(n, (int)((m + WR - 1) / WR), 4 * kWaves);
}

template <typename T>
ProjPlan plan_proj_tn(int64_t m, int64_t n, int LP) {
    (void)LP;
    return make_plan(m, (int)((n + 31) / 32), 4 * Vec16<T>::N * kWaves);
}

template <typename T>
hipError_t launch_proj_nn(const T* A, int64_t lda, int64_t m, int64_t n, const T* X, int LP,
                          const ProjPlan& p, T* slabs, T* Y, hipStream_t s, hipEvent_t done) {
    switch (LP) {
        case 16: return nn_dispatch<T, 16>(A, lda, m, n, X, p, slabs, Y, s, done, 16);
        case 32: return nn_dispatch<T, 32>(A, lda, m, n, X, p, slabs, Y, s, done, 32);
        case 48: return nn_dispatch<T, 48>(A, lda, m, n, X, p, slabs, Y, s, done, 48);
        case 64: return nn_dispatch<T, 64>(A, lda, m, n, X, p, slabs, Y, s, done, 64);
        default:
            if (LP % 64 || LP > 512) return hipErrorInvalidValue;
            return nn_dispatch<T, 64>(A, lda, m, n, X, p, slabs, Y, s, done, LP);
    }
}

template <typename T>
hipError_t launch_proj_tn(const T* A, int64_t lda, int64_t m, int64_t n, const T* Q, int LP,
                          const ProjPlan& p, T* slabs, T* Z, hipStream_t s, hipEvent_t done) {
    switch (LP) {
        case 16: return tn_dispatch<T, 16>(A, lda, m, n, Q, p, slabs, Z, s, done, 16);
        case 32: return tn_dispatch<T, 32>(A, lda, m, n, Q, p, slabs, Z, s, done, 32);
        case 48: return tn_dispatch<T, 48>(A, lda, m, n, Q, p, slabs, Z, s, done, 48);
        case 64: return tn_dispatch<T, 64>(A, lda, m, n, Q, p, slabs, Z, s, done, 64);
        default:
            if (LP % 64 || LP > 512) return hipErrorInvalidValue;
            return tn_dispatch<T, 64>(A, lda, m, n, Q, p, slabs, Z, s, done, LP);
    }
}

#define RSVD_INST(T)                                                                                   \
    template ProjPlan plan_proj_nn<T>(int64_t, int64_t, int);                                          \
    template ProjPlan plan_proj_tn<T>(int64_t, int64_t, int);                                          \
    template hipError_t launch_proj_nn<T>(const T*, int64_t, int64_t, int64_t, const T*, int,          \
                                          const ProjPlan&, T*, T*, hipStream_t, hipEvent_t);           \
    template hipError_t launch_proj_tn<T>(const T*, int64_t, int64_t, int64_t, const T*, int,          \
                                          const ProjPlan&, T*, T*, hipStream_t, hipEvent_t);
RSVD_INST(float)
RSVD_INST(double)
#undef RSVD_INST

}  // namespace rsvd
