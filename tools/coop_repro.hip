// Minimal reproducer for the exit-time SIGSEGV seen under `rocprofv3 --kernel-trace` after a
// cooperative launch.  No rSVD code, no torch: one hipLaunchCooperativeKernel of
// a kernel that writes one int, a synchronize, and a normal return from main.
//   hipcc --offload-arch=gfx950 -O2 tools/coop_repro.hip -o tools/coop_repro
//   rocprofv3 --kernel-trace --stats -d out -o run -- tools/coop_repro [plain]
// With "plain" the same kernel is launched with hipLaunchKernelGGL (the control).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

__global__ void touch(int* p) {
    if (threadIdx.x == 0) p[blockIdx.x] = (int)blockIdx.x;
}

int main(int argc, char** argv) {
    const bool plain = argc > 1 && std::strcmp(argv[1], "plain") == 0;
    int* d = nullptr;
    if (hipMalloc(&d, 64 * sizeof(int)) != hipSuccess) return 2;
    hipError_t e;
    if (plain) {
        hipLaunchKernelGGL(touch, dim3(8), dim3(64), 0, 0, d);
        e = hipGetLastError();
    } else {
        void* args[] = {&d};
        e = hipLaunchCooperativeKernel(reinterpret_cast<const void*>(touch), dim3(8), dim3(64), args, 0, 0);
    }
    if (e != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
        std::printf("launch failed: %s\n", hipGetErrorString(e));
        return 3;
    }
    int h[8];
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 4;
    (void)hipFree(d);
    std::printf("%s launch ok: %d %d\n", plain ? "plain" : "cooperative", h[0], h[7]);
    return 0;
}
