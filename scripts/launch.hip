// Micro-benchmark (diagnostic, not product): per-launch cost of back-to-back kernels in a HIP
// graph as a function of block size, dynamic LDS and kernel-argument bytes.
// Build: hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-kernarg-preload-count=16 scripts/launch.hip -o scripts/_launch
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                             \
    do {                                                                  \
        hipError_t e = (x);                                               \
        if (e != hipSuccess) {                                            \
            printf("%s failed: %s\n", #x, hipGetErrorString(e));          \
            return 1;                                                     \
        }                                                                 \
    } while (0)

struct Big {
    long long w[16];
};
__global__ void k_empty() {}
__global__ void k_lds() {
    extern __shared__ int sm[];
    if (threadIdx.x == 1000) sm[0] = 1;
}
__global__ void k_args(Big a, int *p) {
    if (threadIdx.x == 1000) p[0] = (int)a.w[3];
}
__global__ void k_args2(char *base, int P, int PS, int BA, int pk, const float *r, const float *v, const float *po,
                        const float *be, const void *prm, int hsx, float disc, int f, const char *pool, long long ps,
                        long long rb, char *go, int *ix, int *iy, int *ac) {
    if (threadIdx.x == 1000) ix[0] = P + PS + BA + pk + hsx + f + (int)ps + (int)rb + (int)disc;
}
__global__ void k_scratch(int n, int *out) {
    volatile int a[64];
    for (int i = 0; i < 64; ++i) a[i] = i * n;
    if (threadIdx.x == 1000) out[0] = a[n & 63];
}

template <typename F>
int timeit(const char *name, hipStream_t st, F launch) {
    hipGraph_t g;
    hipGraphExec_t ge;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int i = 0; i < 200; ++i) launch();
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    float best = 1e9;
    for (int rep = 0; rep < 5; ++rep) {
        CK(hipEventRecord(e0, st));
        CK(hipGraphLaunch(ge, st));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    printf("%-48s %.2f us per launch\n", name, best * 1000 / 200);
    return 0;
}

int main() {
    hipStream_t st;
    CK(hipStreamCreate(&st));
    int *p;
    CK(hipMalloc(&p, 4096));
    Big big{};
    CK(hipFuncSetAttribute((const void *)k_lds, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    timeit("empty, 256 x 64", st, [&] { hipLaunchKernelGGL(k_empty, dim3(256), dim3(64), 0, st); });
    timeit("empty, 256 x 128", st, [&] { hipLaunchKernelGGL(k_empty, dim3(256), dim3(128), 0, st); });
    timeit("empty, 256 x 128, 26 KB dynamic LDS", st, [&] { hipLaunchKernelGGL(k_lds, dim3(256), dim3(128), 26 * 1024, st); });
    timeit("empty, 256 x 128, 64 KB dynamic LDS", st, [&] { hipLaunchKernelGGL(k_lds, dim3(256), dim3(128), 64 * 1024, st); });
    timeit("empty, 256 x 128, 136 B by-value arg", st, [&] { hipLaunchKernelGGL(k_args, dim3(256), dim3(128), 0, st, big, p); });
    timeit("empty, 256 x 128, k_step-like 20 args", st, [&] {
        hipLaunchKernelGGL(k_args2, dim3(256), dim3(128), 0, st, (char *)p, 1, 2, 3, 4, (const float *)p, (const float *)p,
                           (const float *)p, (const float *)p, (const void *)p, 5, 0.5f, 1, (const char *)p, 7ll, 8ll,
                           (char *)p, p, p, p);
    });
    timeit("scratch-using kernel, 256 x 128", st, [&] { hipLaunchKernelGGL(k_scratch, dim3(256), dim3(128), 0, st, 3, p); });
    return 0;
}
