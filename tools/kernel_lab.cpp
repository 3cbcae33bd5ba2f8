// kernel_lab.cpp -- per-kernel hipEvent timings of the rSVD kernels on synthetic inputs (tuning aid).
// Build: make -C rsvd_kamaneh_raganato_terrana_amd/csrc lab ; run on the GPU box.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <random>
#include <vector>

#include "../rsvd_kamaneh_raganato_terrana_amd/csrc/kernels.hpp"

using namespace rsvd;

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e = (x);                                                           \
        if (e != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

// ---- latency microbenchmarks ------------------------------------------------------------------
__global__ void mb_barrier(double* out, int steps) {  // LDS write -> barrier -> LDS read, 256 threads
    __shared__ double buf[2][64];
    double acc = threadIdx.x;
    for (int k = 0; k < steps; ++k) {
        if (threadIdx.x < 64) buf[k & 1][threadIdx.x] = acc;
        __syncthreads();
        acc += buf[k & 1][(threadIdx.x + 1) & 63] * 1e-9;
    }
    out[threadIdx.x] = acc;
}
__global__ void mb_wave_lds(double* out, int steps) {  // single wave: dependent LDS write/read chain
    __shared__ double buf[64];
    double acc = threadIdx.x;
    for (int k = 0; k < steps; ++k) {
        buf[threadIdx.x] = acc;
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        acc += buf[(threadIdx.x + 1) & 63] * 1e-9;
    }
    out[threadIdx.x] = acc;
}
__global__ void mb_fma64(double* out, int steps) {  // dependent fp64 FMA chain
    double a = threadIdx.x, b = 1.0000001;
    for (int k = 0; k < steps; ++k) a = fma(a, b, 1e-9);
    out[threadIdx.x] = a;
}
__global__ void mb_sqrtdiv64(double* out, int steps) {  // dependent sqrt + div chain (correctly rounded)
    double a = threadIdx.x + 2.0;
    for (int k = 0; k < steps; ++k) a = 1.0 + 1.0 / sqrt(a);
    out[threadIdx.x] = a;
}
__global__ void mb_rsq64(double* out, int steps) {  // dependent v_rsq_f64 chain
    double a = threadIdx.x + 2.0;
    for (int k = 0; k < steps; ++k) a = 1.0 + __builtin_amdgcn_rsq(a);
    out[threadIdx.x] = a;
}
__global__ void mb_clock(unsigned long long* out, int steps) {  // shader clock vs real time
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    double a = threadIdx.x;
    for (int k = 0; k < steps; ++k) a = fma(a, 1.0000001, 1e-9);
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = r1 - r0; out[2] = (unsigned long long)a; }
}

static double time_us(hipStream_t s, int reps, const std::function<void()>& f) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) f();
    CK(hipEventRecord(a, s));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms * 1e3 / reps;
}

int main(int argc, char** argv) {
    const int64_t m = argc > 1 ? atoll(argv[1]) : 4096;
    const int64_t n = argc > 2 ? atoll(argv[2]) : 4096;
    const int l = argc > 3 ? atoi(argv[3]) : 64;
    const int LP = (l + 15) / 16 * 16;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    std::mt19937 gen(1);
    std::normal_distribution<float> nd;
    std::vector<float> hA(m * n), hP(std::max(m, n) * LP, 0.f);
    for (auto& x : hA) x = nd(gen);
    for (int64_t i = 0; i < std::max(m, n); ++i)
        for (int j = 0; j < l; ++j) hP[i * LP + j] = nd(gen);
    float *A, *P, *Q, *Y, *slab;
    double *gs, *R, *Rinv, *Uw, *Vw, *G;
    float* S;
    unsigned* ctr;
    int* flag;
    CK(hipMalloc(&A, sizeof(float) * m * n));
    CK(hipMalloc(&P, sizeof(float) * std::max(m, n) * LP));
    CK(hipMalloc(&Q, sizeof(float) * std::max(m, n) * LP));
    CK(hipMalloc(&Y, sizeof(float) * std::max(m, n) * LP));
    CK(hipMalloc(&slab, sizeof(float) * 64 * std::max(m, n) * LP));
    CK(hipMalloc(&gs, sizeof(double) * 33 * LP * LP));
    CK(hipMalloc(&R, sizeof(double) * LP * LP));
    CK(hipMalloc(&Rinv, sizeof(double) * LP * LP));
    CK(hipMalloc(&Uw, sizeof(double) * LP * LP));
    CK(hipMalloc(&Vw, sizeof(double) * LP * LP));
    CK(hipMalloc(&G, sizeof(double) * LP * LP));
    CK(hipMalloc(&S, sizeof(float) * LP));
    CK(hipMalloc(&ctr, 256));
    CK(hipMalloc(&flag, 256));
    CK(hipMemset(ctr, 0, 256));
    CK(hipMemset(flag, 0, 256));
    CK(hipMemcpy(A, hA.data(), sizeof(float) * m * n, hipMemcpyHostToDevice));
    CK(hipMemcpy(P, hP.data(), sizeof(float) * std::max(m, n) * LP, hipMemcpyHostToDevice));
    const int reps = 50;
    const int nb = plan_gram_blocks(m);
    printf("m=%ld n=%ld l=%d LP=%d gram_blocks=%d\n", (long)m, (long)n, l, LP, nb);

    double t;
    const unsigned NT = (unsigned)gram_tiles(LP, 0), NTX = (unsigned)gram_tiles(LP, 1);
    unsigned t0 = 0, t1 = 0;
    double* tiles = gs + 32 * LP * LP;
    t0 += nb; t1 += NT;  // produce a valid Gram G first (mode 0)
    CK(launch_gram_chol<float>(P, m, LP, nb, gs, tiles, ctr, t0, t1, 0, 1, G, l, R, Rinv, flag, flag + 8, s));
    for (int f32 = 1; f32 >= 0; --f32) {
        t = time_us(s, reps, [&] { t0 += nb; t1 += NT; CK(launch_gram_chol<float>(P, m, LP, nb, gs, tiles, ctr, t0, t1, 1, f32, nullptr, l, R, Rinv, flag, flag + 8, s)); });
        printf("gram_chol fused (factor %s)    %9.2f us\n", f32 ? "fp32" : "fp64", t);
        t = time_us(s, reps, [&] { CK(launch_chol(G, l, LP, f32, R, Rinv, flag, s)); });
        printf("chol + inverse alone (%s)      %9.2f us\n", f32 ? "fp32" : "fp64", t);
    }
    t = time_us(s, reps, [&] { t0 += nb; t1 += NT; CK(launch_gram_chol<float>(P, m, LP, nb, gs, tiles, ctr, t0, t1, 0, 1, G, l, R, Rinv, flag, flag + 8, s)); });
    printf("gram + tile reduce (mode 0)      %9.2f us\n", t);
    t = time_us(s, reps, [&] { t0 += nb; t1 += NTX; CK(launch_cross_gram<float>(P, Q, m, LP, nb, gs, tiles, ctr, t0, t1, G, l, flag + 8, s)); });
    printf("cross gram                       %9.2f us\n", t);
    t = time_us(s, reps, [&] { CK(launch_panel_small<float>(P, m, LP, Rinv, Q, 0, 0, 0, s)); });
    printf("panel_small (row-major out)      %9.2f us\n", t);
    t = time_us(s, reps, [&] { CK(launch_panel_small<float>(P, m, LP, Rinv, Y, 1, l, m, s)); });
    printf("panel_small (col-major out)      %9.2f us\n", t);
    t = time_us(s, 10, [&] { CK(launch_small_svd<float>(R, l, LP, Uw, Vw, S, flag + 4, s)); });
    int info[8];
    CK(hipMemcpy(info, flag, sizeof(info), hipMemcpyDeviceToHost));
    printf("small_svd fp32 (Jacobi)          %9.2f us   sweeps=%d chol_flags=%d timeouts=%d\n", t, info[4], info[0], info[2]);
    double* Sd;
    CK(hipMalloc(&Sd, sizeof(double) * LP));
    t = time_us(s, 10, [&] { CK(launch_small_svd<double>(R, l, LP, Uw, Vw, Sd, flag + 4, s)); });
    CK(hipMemcpy(info, flag, sizeof(info), hipMemcpyDeviceToHost));
    printf("small_svd fp64 (Jacobi)          %9.2f us   sweeps=%d\n", t, info[4]);
    ProjPlan pnn = plan_proj_nn<float>(m, n, LP), ptn = plan_proj_tn<float>(m, n, LP);
    t = time_us(s, reps, [&] { CK(launch_proj_nn<float>(A, m, m, n, P, LP, pnn, slab, Y, s)); });
    printf("proj_nn + sum (splits=%2d)        %9.2f us  %7.1f TF/s\n", pnn.splits, t, 2.0 * m * n * l / t * 1e-6);
    t = time_us(s, reps, [&] { CK(launch_proj_tn<float>(A, m, m, n, P, LP, ptn, slab, Y, s)); });
    printf("proj_tn + sum (splits=%2d)        %9.2f us  %7.1f TF/s\n", ptn.splits, t, 2.0 * m * n * l / t * 1e-6);
    t = time_us(s, reps, [&] { CK(launch_philox_omega<float>(P, n, l, LP, 7, s)); });
    printf("philox omega                     %9.2f us\n", t);
    t = time_us(s, reps, [&] { CK(hipMemsetAsync(flag, 0, 16, s)); });
    printf("memset (launch floor)            %9.2f us\n", t);
    {
        double* mb;
        unsigned long long* clk;
        CK(hipMalloc(&mb, 4096));
        CK(hipMalloc(&clk, 64));
        const int st = 10000;
        t = time_us(s, 5, [&] { hipLaunchKernelGGL(mb_barrier, dim3(1), dim3(256), 0, s, mb, st); });
        printf("barrier step (256 thr)           %9.1f ns/step\n", t * 1e3 / st);
        t = time_us(s, 5, [&] { hipLaunchKernelGGL(mb_barrier, dim3(1), dim3(64), 0, s, mb, st); });
        printf("barrier step (64 thr)            %9.1f ns/step\n", t * 1e3 / st);
        t = time_us(s, 5, [&] { hipLaunchKernelGGL(mb_wave_lds, dim3(1), dim3(64), 0, s, mb, st); });
        printf("wave LDS write->read chain       %9.1f ns/step\n", t * 1e3 / st);
        t = time_us(s, 5, [&] { hipLaunchKernelGGL(mb_fma64, dim3(1), dim3(64), 0, s, mb, st); });
        printf("dependent fp64 FMA               %9.1f ns/op\n", t * 1e3 / st);
        t = time_us(s, 5, [&] { hipLaunchKernelGGL(mb_sqrtdiv64, dim3(1), dim3(64), 0, s, mb, st); });
        printf("dependent fp64 sqrt+div          %9.1f ns/op\n", t * 1e3 / st);
        t = time_us(s, 5, [&] { hipLaunchKernelGGL(mb_rsq64, dim3(1), dim3(64), 0, s, mb, st); });
        printf("dependent v_rsq_f64 + add        %9.1f ns/op\n", t * 1e3 / st);
        hipLaunchKernelGGL(mb_clock, dim3(1), dim3(64), 0, s, clk, 1000000);
        unsigned long long hc[3];
        CK(hipMemcpy(hc, clk, sizeof(hc), hipMemcpyDeviceToHost));
        printf("shader clock during 1-wave loop  %9.1f MHz (memtime %llu ticks / realtime %llu @100MHz)\n",
               (double)hc[0] / (double)hc[1] * 100.0, hc[0], hc[1]);
    }
    return 0;
}
