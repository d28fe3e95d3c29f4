// Micro-benchmarks of the latencies that bound the per-simulation kernel (diagnostic, not product):
//   clock   s_memtime ticks per s_memrealtime tick (100 MHz)
//   chase   dependent global-load chain latency (L2-resident data), per load
//   first   first load of data written by the previous kernel
//   dma     N x global_load_lds (16 B/lane) issued together, then waited for
//   empty   back-to-back empty kernels (launch + teardown), timed with events
// Build: hipcc --offload-arch=gfx950 -O3 scripts/ulat.hip -o scripts/_ulat
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e = (x);                                                             \
        if (e != hipSuccess) {                                                          \
            printf("%s failed: %s\n", #x, hipGetErrorString(e));                        \
            return 1;                                                                   \
        }                                                                               \
    } while (0)

__device__ __forceinline__ unsigned long long memtime() {
    unsigned long long t;
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
__device__ __forceinline__ unsigned long long realtime() {
    unsigned long long t;
    asm volatile("s_memrealtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

__global__ void k_clock(unsigned long long *out) {
    unsigned long long a = memtime(), ra = realtime();
    unsigned long long x = 0;
    for (int i = 0; i < 200000; ++i) x += __builtin_amdgcn_readfirstlane(i) * 3;
    unsigned long long b = memtime(), rb = realtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        out[0] = b - a;
        out[1] = rb - ra;
        out[2] = x;
    }
}

__global__ void k_write(int *buf, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) buf[i] = (i * 7 + 1) % n;
}

// per wave: `hops` dependent loads starting at wave-specific index
__global__ void k_chase(const int *buf, int hops, unsigned long long *out) {
    int idx = blockIdx.x * 977 % 4096;
    unsigned long long t0 = memtime();
    for (int h = 0; h < hops; ++h) idx = __builtin_amdgcn_readfirstlane(buf[idx]);
    unsigned long long t1 = memtime();
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0 + (idx == -1);
}

__global__ void k_dma(const int4 *src, int n16, unsigned long long *out) {
    extern __shared__ int4 lds[];
    const int l = threadIdx.x;
    unsigned long long t0 = memtime();
    const int4 *s = src + (size_t)blockIdx.x * n16 * 64;
    for (int k = 0; k < n16; ++k)
        __builtin_amdgcn_global_load_lds((const void *)(s + k * 64 + l),
                                         (__attribute__((address_space(3))) void *)(lds + k * 64), 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned long long t1 = memtime();
    if (l == 0) out[blockIdx.x] = t1 - t0 + (lds[5].x == 12345);
}

__global__ void k_empty() {}

// DPP wave shifts: out[l] = value lane l receives from (lane index + 100) under each control
__global__ void k_dpp(int *out) {
    const int l = threadIdx.x;
    const int v = l + 100;
    out[l] = __builtin_amdgcn_update_dpp(-1, v, 0x130, 0xf, 0xf, false);        // wave_shl:1
    out[64 + l] = __builtin_amdgcn_update_dpp(-1, v, 0x138, 0xf, 0xf, false);   // wave_shr:1
}

// instruction-fetch cost: 2048 straight-line VALU ops vs the same count in a 16-op loop
__global__ void k_straight(unsigned long long *out) {
    unsigned long long t0 = memtime();
    float x = threadIdx.x;
    asm volatile(".rept 2048\n v_add_f32 %0, 1.0, %0\n .endr" : "+v"(x));
    unsigned long long t1 = memtime();
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0 + (x == -1.f);
}
__global__ void k_looped(unsigned long long *out) {
    unsigned long long t0 = memtime();
    float x = threadIdx.x;
    for (int i = 0; i < 128; ++i) asm volatile(".rept 16\n v_add_f32 %0, 1.0, %0\n .endr" : "+v"(x));
    unsigned long long t1 = memtime();
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0 + (x == -1.f);
}

// one load from each of `nbuf` separately allocated buffers, issued together (wave-uniform)
struct Bufs {
    int *p[16];
};
__global__ void k_multi(Bufs bufs, int nbuf, int stride_ints, unsigned long long *out) {
    const int l = threadIdx.x;
    unsigned long long t0 = memtime();
    int acc = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k)
        if (k < nbuf) acc += bufs.p[k][(blockIdx.x * stride_ints + l) & ((1 << 20) - 1)];
    acc = __builtin_amdgcn_readfirstlane(acc);
    unsigned long long t1 = memtime();
    if (l == 0) out[blockIdx.x] = t1 - t0 + (acc == 12345);
}

int main() {
    const int B = 256;
    int *buf;
    unsigned long long *out;
    int4 *big;
    CK(hipMalloc(&buf, 4096 * 4));
    CK(hipMalloc(&out, 1024 * 8));
    CK(hipMalloc(&big, (size_t)B * 16 * 64 * 16));
    CK(hipMemset(big, 0, (size_t)B * 16 * 64 * 16));
    std::vector<unsigned long long> h(1024);
    auto med = [&](int n) {
        std::vector<unsigned long long> v(h.begin(), h.begin() + n);
        std::sort(v.begin(), v.end());
        return (double)v[n / 2];
    };

    hipLaunchKernelGGL(k_clock, dim3(1), dim3(64), 0, 0, out);
    CK(hipMemcpy(h.data(), out, 24, hipMemcpyDeviceToHost));
    const double ratio = (double)h[0] / (double)h[1];
    printf("clock: memtime/realtime = %.2f  -> memtime ~ %.0f MHz\n", ratio, ratio * 100.0);

    hipLaunchKernelGGL(k_write, dim3(16), dim3(256), 0, 0, buf, 4096);
    for (int hops : {1, 2, 8, 32}) {
        hipLaunchKernelGGL(k_chase, dim3(B), dim3(64), 0, 0, buf, hops, out);  // warm
        hipLaunchKernelGGL(k_chase, dim3(B), dim3(64), 0, 0, buf, hops, out);
        CK(hipMemcpy(h.data(), out, B * 8, hipMemcpyDeviceToHost));
        printf("chase hops=%2d: median %.0f cycles (%.0f per load)\n", hops, med(B), med(B) / hops);
    }
    // first touch of freshly written data
    hipLaunchKernelGGL(k_write, dim3(16), dim3(256), 0, 0, buf, 4096);
    hipLaunchKernelGGL(k_chase, dim3(B), dim3(64), 0, 0, buf, 1, out);
    CK(hipMemcpy(h.data(), out, B * 8, hipMemcpyDeviceToHost));
    printf("first load after a writer kernel: median %.0f cycles\n", med(B));

    for (int n16 : {1, 4, 8, 16}) {
        hipLaunchKernelGGL(k_dma, dim3(B), dim3(64), n16 * 64 * 16, 0, big, n16, out);
        hipLaunchKernelGGL(k_dma, dim3(B), dim3(64), n16 * 64 * 16, 0, big, n16, out);
        CK(hipMemcpy(h.data(), out, B * 8, hipMemcpyDeviceToHost));
        printf("global_load_lds x%2d (16 B/lane): median %.0f cycles\n", n16, med(B));
    }

    {
        // TLB / allocation spread: loads to 1, 4, 16 separately allocated 4 MiB buffers
        std::vector<int *> bl(16);
        for (auto &p : bl) {
            CK(hipMalloc(&p, 4 << 20));
            CK(hipMemset(p, 0, 4 << 20));
        }
        Bufs dbl;
        for (int k = 0; k < 16; ++k) dbl.p[k] = bl[k];
        for (int nbuf : {1, 4, 16}) {
            for (int stride : {64, 4096}) {
                hipLaunchKernelGGL(k_multi, dim3(B), dim3(64), 0, 0, dbl, nbuf, stride, out);
                hipLaunchKernelGGL(k_multi, dim3(B), dim3(64), 0, 0, dbl, nbuf, stride, out);
                CK(hipMemcpy(h.data(), out, B * 8, hipMemcpyDeviceToHost));
                printf("loads from %2d buffers (wave stride %5d B): median %.0f cycles\n", nbuf, stride * 4, med(B));
            }
        }
    }
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_straight, dim3(B), dim3(64), 0, 0, out);
        CK(hipMemcpy(h.data(), out, B * 8, hipMemcpyDeviceToHost));
        const double a = med(B);
        hipLaunchKernelGGL(k_looped, dim3(B), dim3(64), 0, 0, out);
        CK(hipMemcpy(h.data(), out, B * 8, hipMemcpyDeviceToHost));
        printf("2048 VALU ops: straight-line %.0f cycles, looped %.0f cycles\n", a, med(B));
    }
    {
        int *dd;
        CK(hipMalloc(&dd, 128 * 4));
        hipLaunchKernelGGL(k_dpp, dim3(1), dim3(64), 0, 0, dd);
        std::vector<int> hv(128);
        CK(hipMemcpy(hv.data(), dd, 128 * 4, hipMemcpyDeviceToHost));
        printf("dpp wave_shl:1 lanes 0,1,15,16,62,63 get: %d %d %d %d %d %d\n", hv[0], hv[1], hv[15], hv[16], hv[62], hv[63]);
        printf("dpp wave_shr:1 lanes 0,1,15,16,62,63 get: %d %d %d %d %d %d\n", hv[64], hv[65], hv[79], hv[80], hv[126], hv[127]);
    }
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int grid : {1, 256}) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(k_empty, dim3(grid), dim3(64), 0, st);
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, st));
        CK(hipStreamSynchronize(st));
        CK(hipEventRecord(e0, st));
        CK(hipGraphLaunch(ge, st));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("empty kernel in a graph, grid %d: %.2f us per launch\n", grid, ms * 1000 / 200);
    }
    return 0;
}
