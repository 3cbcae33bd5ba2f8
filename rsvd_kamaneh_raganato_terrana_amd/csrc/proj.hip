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
constexpr int kPrefetch = 8;  // k-steps of A kept in flight per wave (NN; TN keeps half as many, wider)

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
    // steps ahead so that enough A bytes are in flight per CU to cover HBM latency.
    constexpr int PD = kPrefetch;
    const int64_t kstep = 4 * kWaves, kfirst = kbeg + 4 * w;
    const int nst = (kfirst < kend) ? (int)((kend - kfirst + kstep - 1) / kstep) : 0;
    V pa[PD];
    T pb[PD][G];
    auto load = [&](int st, V& a, T* b) {
        const int64_t k = kfirst + (int64_t)st * kstep + h;
        if (st < nst && k < kend) {
            a = load_vec_guarded<T>(A + k * lda, row, m, vec_ok);
            const T* xr = X + k * ldp + r;
#pragma unroll
            for (int g = 0; g < G; ++g) b[g] = xr[16 * g];
        } else {
            T* e = reinterpret_cast<T*>(&a);
#pragma unroll
            for (int t = 0; t < VW; ++t) e[t] = T(0);
#pragma unroll
            for (int g = 0; g < G; ++g) b[g] = T(0);
        }
    };
#pragma unroll
    for (int u = 0; u < PD; ++u) load(u, pa[u], pb[u]);
    for (int base = 0; base < nst; base += PD) {
#pragma unroll
        for (int u = 0; u < PD; ++u) {
            if (base + u >= nst) break;
            const V a = pa[u];
            T b[G];
#pragma unroll
            for (int g = 0; g < G; ++g) b[g] = pb[u][g];
            load(base + u + PD, pa[u], pb[u]);
#pragma unroll
            for (int t = 0; t < VW; ++t) {
                const T at = Vec16<T>::get(a, t);
#pragma unroll
                for (int g = 0; g < G; ++g) acc[t][g] = M::mma(at, b[g], acc[t][g]);
            }
        }
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
                mine[lr * LP + 16 * g + r] = acc[t][g][j];
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
    constexpr int PD = kPrefetch / 2;
    const int64_t istep = (int64_t)ISTEP * kWaves, ifirst = ibeg + ISTEP * w;
    const int nst = (ifirst < iend) ? (int)((iend - ifirst + istep - 1) / istep) : 0;
    V pa[PD][JT];
    T pb[PD][VW][G];
    auto load = [&](int st, V* a, T (*b)[G]) {
        const int64_t ib = ifirst + (int64_t)st * istep + VW * h;
        const bool ok = st < nst;
#pragma unroll
        for (int jt = 0; jt < JT; ++jt) {
            const int64_t j = j0 + 16 * jt + r;
            if (ok && j < n) {
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
            const T* qr = Q + i * ldp + r;
#pragma unroll
            for (int g = 0; g < G; ++g) b[t][g] = (ok && i < iend) ? qr[16 * g] : T(0);
        }
    };
#pragma unroll
    for (int u = 0; u < PD; ++u) load(u, pa[u], pb[u]);
    for (int base = 0; base < nst; base += PD) {
#pragma unroll
        for (int u = 0; u < PD; ++u) {
            if (base + u >= nst) break;
            V a[JT];
            T b[VW][G];
#pragma unroll
            for (int jt = 0; jt < JT; ++jt) a[jt] = pa[u][jt];
#pragma unroll
            for (int t = 0; t < VW; ++t)
#pragma unroll
                for (int g = 0; g < G; ++g) b[t][g] = pb[u][t][g];
            load(base + u + PD, pa[u], pb[u]);
#pragma unroll
            for (int t = 0; t < VW; ++t)
#pragma unroll
                for (int jt = 0; jt < JT; ++jt) {
                    const T at = Vec16<T>::get(a[jt], t);
#pragma unroll
                    for (int g = 0; g < G; ++g) acc[jt][g] = M::mma(at, b[t][g], acc[jt][g]);
                }
        }
    }

    T* mine = red + (size_t)w * WJ * LP;
#pragma unroll
    for (int jt = 0; jt < JT; ++jt)
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int j = 0; j < 4; ++j) mine[(16 * jt + M::row(h, j)) * LP + 16 * g + r] = acc[jt][g][j];
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

// Pick the K split so the grid has ~2 workgroups per CU (256 CUs) while every wave keeps
// at least ~8 MFMA groups of work and the slab traffic stays bounded.
ProjPlan make_plan(int64_t K, int blocks, int64_t kstep_wg) {
    ProjPlan p;
    p.blocks = blocks;
    int64_t splits = (512 + blocks - 1) / blocks;
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
