// fetch_calib.hip -- calibration of rocprofv3 FETCH_SIZE for the access shapes of the projection
// kernels (MI355X_MICROARCH.md, HBM: "Other access widths are uncalibrated: calibrate on a known
// byte count in your own access pattern before trusting an absolute").
//
// Each variant reads an 8 GiB column-major bf16 matrix (65536 x 65536, the C4 A; far beyond the
// 256 MiB Infinity Cache) exactly once with global_load_lds_dwordx4, in the shape of
// wproj2_kernel's TN A stream: a 512-thread workgroup owns 256 columns and, per k-step, copies a
// RUN-byte run of each of them (RUN = 32: e4m3 TN, 64: bf16 TN single-step, 128: bf16 TN two-step);
// plus the contiguous 16-B/lane streaming read the guide's factor 1/2 was measured on.
// Known bytes per dispatch = 2^33.  FETCH_SIZE (KiB) * 1024 / 2^33 is the factor to undo.
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/fetch_calib tools/fetch_calib.hip
// run:   rocprofv3 --pmc FETCH_SIZE -d gpurun_out/calib -o run -- ./tools/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

constexpr long kRows = 65536, kCols = 65536;  // bf16 elements (the C4 matrix: 256 workgroups)
typedef __attribute__((address_space(3))) void* lds_ptr;

template <int RUN>
__global__ __launch_bounds__(512) void column_runs(const unsigned short* __restrict__ A, float* __restrict__ sink) {
    extern __shared__ __attribute__((aligned(1024))) char lds[];
    constexpr int CHUNKS = RUN / 16;              // 16-B chunks per column per k-step
    constexpr int PER_T = 256 * CHUNKS / 512;     // glds per thread per k-step (>= 1 for RUN >= 32)
    constexpr long STEPS = kRows * 2 / RUN;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const long col0 = (long)blockIdx.x * 256;
    for (long st = 0; st < STEPS; ++st) {
#pragma unroll
        for (int t = 0; t < PER_T; ++t) {
            const int u = (t * 8 + w) * 64 + lane;  // chunk index within the step
            const int j = u / CHUNKS, c = u % CHUNKS;
            const char* src = reinterpret_cast<const char*>(A + (col0 + j) * kRows) + st * RUN + 16 * c;
            __builtin_amdgcn_global_load_lds(src, (lds_ptr)(lds + (t * 8 + w) * 1024), 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    }
    if (tid == 0) sink[blockIdx.x] = reinterpret_cast<float*>(lds)[0];
}

// contiguous streaming read: every thread copies consecutive 16-B chunks of the flat buffer
__global__ __launch_bounds__(512) void streaming(const unsigned short* __restrict__ A, float* __restrict__ sink) {
    extern __shared__ __attribute__((aligned(1024))) char lds[];
    const long total = kRows * kCols * 2 / 16;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    for (long base = (long)blockIdx.x * 512; base < total; base += (long)gridDim.x * 512) {
        const long u = base + w * 64 + lane;
        const char* src = reinterpret_cast<const char*>(A) + 16 * (u < total ? u : total - 1);
        __builtin_amdgcn_global_load_lds(src, (lds_ptr)(lds + w * 1024), 16, 0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (tid == 0) sink[blockIdx.x] = reinterpret_cast<float*>(lds)[0];
}

int main() {
    const size_t bytes = (size_t)kRows * kCols * 2;
    unsigned short* A;
    float* sink;
    CK(hipMalloc(&A, bytes));
    CK(hipMalloc(&sink, 65536 * sizeof(float)));
    CK(hipMemset(A, 0x3c, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int grid = (int)(kCols / 256);
    for (int rep = 0; rep < 2; ++rep) {
        float ms[4];
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(column_runs<32>, dim3(grid), dim3(512), 8192, 0, A, sink);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms[0], e0, e1));
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(column_runs<64>, dim3(grid), dim3(512), 16384, 0, A, sink);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms[1], e0, e1));
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(column_runs<128>, dim3(grid), dim3(512), 32768, 0, A, sink);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms[2], e0, e1));
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(streaming, dim3(1024), dim3(512), 8192, 0, A, sink);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms[3], e0, e1));
        std::printf("rep %d: %.3f GB read per dispatch; ms: run32 %.2f run64 %.2f run128 %.2f stream %.2f\n", rep,
                    bytes / 1e9, ms[0], ms[1], ms[2], ms[3]);
    }
    CK(hipFree(A));
    CK(hipFree(sink));
    return 0;
}
