// common.hpp -- shared device helpers for the gfx950 (MI355X / CDNA4) rSVD kernels.
//
// Conventions used by every kernel in this directory:
//  * A (the big m x n operand) is column-major with leading dimension lda, exactly as the
//    reference's Eigen::MatrixXd (include/rSVD.hpp:9).
//  * "Skinny" panels (Omega, Y = A*Omega, Q, Z = A^T*Q, B^T) live in HBM ROW-major with a
//    padded width LP = 16*ceil(l/16): one panel row is one contiguous LP-vector, which is the
//    natural B-operand feed of the 16x16x4 MFMA (16 lanes read 16 consecutive columns) and the
//    row-per-thread feed of the QR kernels.  Columns l..LP-1 are kept exactly zero.
//  * Wave = 64 lanes.  lane = threadIdx.x & 63, r = lane & 15, h = lane >> 4.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>

namespace rsvd {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

// ---------------------------------------------------------------------------------------------
// MFMA 16x16x4 (f32-in exact f32, or f64).  Operand maps (cdna_hip_programming.md §3):
//   A: lane l holds A[row = l & 15][k = l >> 4];  B: lane l holds B[k = l >> 4][col = l & 15]
//   C/D f32: col = lane & 15, row = (lane >> 4) * 4 + reg
//   C/D f64: col = lane & 15, row = (lane >> 4) + 4 * reg
// ---------------------------------------------------------------------------------------------
template <typename T> struct Mfma;

template <> struct Mfma<float> {
    typedef f32x4 acc_t;
    static __device__ __forceinline__ acc_t zero() { return acc_t{0.f, 0.f, 0.f, 0.f}; }
    static __device__ __forceinline__ acc_t mma(float a, float b, acc_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    // row of register `reg` for lane half h (= lane >> 4)
    static __device__ __forceinline__ int row(int h, int reg) { return h * 4 + reg; }
};

template <> struct Mfma<double> {
    typedef f64x4 acc_t;
    static __device__ __forceinline__ acc_t zero() { return acc_t{0.0, 0.0, 0.0, 0.0}; }
    static __device__ __forceinline__ acc_t mma(double a, double b, acc_t c) {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ int row(int h, int reg) { return h + 4 * reg; }
};

// 16-byte vector of T: 4 floats or 2 doubles.
template <typename T> struct Vec16;
template <> struct Vec16<float> {
    static constexpr int N = 4;
    typedef float4 type;
    static __device__ __forceinline__ float get(const float4& v, int t) {
        return t == 0 ? v.x : (t == 1 ? v.y : (t == 2 ? v.z : v.w));
    }
};
template <> struct Vec16<double> {
    static constexpr int N = 2;
    typedef double2 type;
    static __device__ __forceinline__ double get(const double2& v, int t) { return t == 0 ? v.x : v.y; }
};

// Launch of a persistent grid whose workgroups wait on each other (grid barriers, spin hand-offs).
// Residency comes from the grid size alone (plain, cooperative and graph launches of one grid are
// equally resident, MI355X_MICROARCH.md coop-launch row): launch_coresident checks the grid against
// the occupancy query x CU count itself -- the check hipLaunchCooperativeKernel would make -- refuses
// an oversize grid, and every spin in these kernels is bounded.  Round 6: the launch is PLAIN by
// default.  The cooperative launch bought nothing beyond that check and cost wall time in the rSVD
// loop: same box, alternating (gpurun_out ab_coop_*, profiles/r06_coop_ab.txt) C4 22.73 / 22.74 ->
// 22.44 / 22.54 ms, C5 17.00 / 17.01 -> 16.72 / 16.76 ms per rSVD, with one or two persistent
// launches per rSVD (tridiagonalisation phase 1, block Jacobi).  RSVD_COOP=1 selects
// hipLaunchCooperativeKernel (under rocprofv3 7.2 --kernel-trace ANY process that made a cooperative
// launch segfaults in the HIP runtime's exit-time teardown, after the trace is written --
// reproduced without this library by tools/coop_repro.hip, profiles/r04_exit_segv/README.md).
inline bool coop_launch_enabled() {
    static const int env = [] {
        const char* v = std::getenv("RSVD_COOP");
        return v ? std::atoi(v) : 0;
    }();
    return env != 0;
}

// How many workgroups of `kernel` (block threads, lds bytes of dynamic LDS) the device holds at
// once: the occupancy calculator's per-CU count times the CU count.  A persistent grid larger
// than this cannot be co-resident -- the caller shrinks it or refuses the size.  A failing HIP
// query returns its error code negated (< 0), which launch_coresident passes through (ADVICE r05:
// it is not a size the device cannot hold).
// (Cached per device, kernel, block and LDS size: the persistent kernels launch once per rSVD.)
template <typename... P>
int64_t coresident_capacity(void (*kernel)(P...), int block, size_t lds) {
    int dev = 0, per_cu = 0, cus = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return -(int64_t)e;
    static std::mutex mu;
    static std::map<std::tuple<int, const void*, int, size_t>, int64_t> cache;
    const auto key = std::make_tuple(dev, reinterpret_cast<const void*>(kernel), block, lds);
    {
        std::lock_guard<std::mutex> g(mu);
        auto it = cache.find(key);
        if (it != cache.end()) return it->second;
    }
    e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return -(int64_t)e;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(kernel), block, lds);
    if (e != hipSuccess) return -(int64_t)e;
    const int64_t cap = (int64_t)per_cu * cus;
    std::lock_guard<std::mutex> g(mu);
    cache[key] = cap;
    return cap;
}

template <typename... P, typename... A>
hipError_t launch_coresident(void (*kernel)(P...), dim3 grid, dim3 block, size_t lds, hipStream_t s, A&&... a) {
    // refuse a grid the device cannot hold at once (a plain launch of it would deadlock in the
    // kernel's grid barriers until the bounded spins gave up)
    const int64_t cap = coresident_capacity(kernel, (int)(block.x * block.y * block.z), lds);
    if (cap < 0) return (hipError_t)(-cap);  // the occupancy query itself failed
    if ((int64_t)grid.x * grid.y * grid.z > cap) return hipErrorCooperativeLaunchTooLarge;
    if (!coop_launch_enabled()) {
        hipLaunchKernelGGL(kernel, grid, block, lds, s, static_cast<P>(a)...);
        return hipGetLastError();
    }
    std::tuple<P...> args(static_cast<P>(a)...);
    void* argv[sizeof...(P) > 0 ? sizeof...(P) : 1];
    std::apply([&](auto&... x) {
        int i = 0;
        ((argv[i++] = static_cast<void*>(&x)), ...);
    }, args);
    return hipLaunchCooperativeKernel(reinterpret_cast<const void*>(kernel), grid, block, argv, (unsigned)lds, s);
}

// XCD-aware bijective block remap (cdna_hip_programming.md §5 "XCD swizzle must be bijective"):
// blocks that the dispatcher deals to the same XCD (b % 8) get consecutive logical ids, so
// neighbouring tiles (which share A columns / panel rows) meet in one L2.
__device__ __forceinline__ int xcd_remap(int b, int nwg) {
    const int xcd = b & 7, q = nwg >> 3, r = nwg & 7;
    const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + (b >> 3);
}

__device__ __forceinline__ double warp_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Counter-based Philox4x32-10 Gaussian stream shared by every GPU and the CPU oracle
// (oracle/rsvd_oracle.c orc_philox_gaussian): element e of the stream keyed by `seed`.
__device__ __forceinline__ void philox4x32_10(uint64_t ctr, uint64_t seed, uint32_t out[4]) {
    uint32_t c0 = (uint32_t)ctr, c1 = (uint32_t)(ctr >> 32), c2 = 0x52535644u, c3 = 0u;
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

__device__ __forceinline__ double gauss_elem(uint64_t e, uint64_t seed) {
    uint32_t x[4];
    philox4x32_10(e >> 1, seed, x);
    const double two_m53 = 1.1102230246251565404e-16;
    const double u1 = ((double)(((uint64_t)(x[0] >> 5) << 26) | (x[1] >> 6)) + 0.5) * two_m53;
    const double u2 = ((double)(((uint64_t)(x[2] >> 5) << 26) | (x[3] >> 6)) + 0.5) * two_m53;
    const double rr = sqrt(-2.0 * log(u1));
    const double th = 6.283185307179586476925286766559 * u2;
    return (e & 1) ? rr * sin(th) : rr * cos(th);
}

}  // namespace rsvd
