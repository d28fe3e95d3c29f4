// Micro-benchmark (diagnostic, not product): per-launch period of back-to-back kernels in a HIP
// graph against the grid size and the workgroup size, with each workgroup reading 16 bytes per lane
// that the previous launch wrote (one dependent round trip, then a store) -- does the launch
// boundary of the per-simulation tree kernels depend on how many workgroups a launch has?
// Build: hipcc --offload-arch=gfx950 -O3 scripts/gridsize.hip -o scripts/_gridsize
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e = (x);                                                      \
        if (e != hipSuccess) {                                                   \
            printf("%s failed: %s\n", #x, hipGetErrorString(e));                 \
            return 1;                                                            \
        }                                                                        \
    } while (0)

__global__ void k_rw(int4 *buf, int flip) {
    const int t = threadIdx.x;
    int4 *src = buf + ((size_t)blockIdx.x * 2 + flip) * 1024;
    int4 *dst = buf + ((size_t)blockIdx.x * 2 + (flip ^ 1)) * 1024;
    if (t < 64) {
        const int4 v = src[t];
        dst[t] = make_int4(v.x + 1, v.y, v.z, flip);
    }
}

__global__ void k_empty() {}

int main() {
    int4 *buf = nullptr;
    CK(hipMalloc(&buf, (size_t)4096 * 2 * 1024 * sizeof(int4)));
    CK(hipMemset(buf, 0, (size_t)4096 * 2 * 1024 * sizeof(int4)));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int L = 49;
    const int grids[] = {8, 32, 64, 128, 192, 256, 384, 512, 1024};
    const int blocks[] = {64, 192, 512};
    for (int kind = 0; kind < 2; ++kind)
        for (int b : blocks)
            for (int g : grids) {
                hipGraph_t gr;
                hipGraphExec_t ge;
                CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
                for (int i = 0; i < L; ++i) {
                    if (kind == 0) hipLaunchKernelGGL(k_empty, dim3(g), dim3(b), 0, s);
                    else hipLaunchKernelGGL(k_rw, dim3(g), dim3(b), 0, s, buf, i & 1);
                }
                CK(hipStreamEndCapture(s, &gr));
                CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
                float best = 1e9f;
                for (int rep = 0; rep < 12; ++rep) {
                    CK(hipEventRecord(e0, s));
                    CK(hipGraphLaunch(ge, s));
                    CK(hipEventRecord(e1, s));
                    CK(hipEventSynchronize(e1));
                    float ms = 0.f;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    if (rep >= 2 && ms < best) best = ms;
                }
                printf("{\"kernel\": \"%s\", \"grid\": %d, \"block\": %d, \"us_per_launch\": %.3f}\n",
                       kind ? "read16B+write" : "empty", g, b, best * 1000.f / L);
                CK(hipGraphExecDestroy(ge));
                CK(hipGraphDestroy(gr));
            }
    return 0;
}
