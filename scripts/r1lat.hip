// Micro-benchmark (diagnostic, not product): round-1 latency of a kernel that reads what the
// previous launch of a HIP graph wrote, in s_memtime ticks measured by wave 0 (256 workgroups of
// 2 waves, 49 launches per graph, alternating buffers as the tree kernels do).  Each launch stores
// 3 KiB per workgroup (the next launch's input).  Variants (one load round, then the wait):
//   vgpr1 / vgpr12   1 / 12 global_load_dwordx4 into VGPRs
//   dma1 / dma12     1 / 12 global_load_lds_dwordx4
//   smem             s_load_dwordx8 of the workgroup's first 32 bytes
//   mix              12 LDS-DMA + the scalar load (k_chain's round 1)
// Build: hipcc --offload-arch=gfx950 -O3 -Wno-inline-asm scripts/r1lat.hip -o scripts/_r1lat
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e = (x);                                                      \
        if (e != hipSuccess) {                                                   \
            printf("%s failed: %s\n", #x, hipGetErrorString(e));                 \
            return 1;                                                            \
        }                                                                        \
    } while (0)

typedef __attribute__((address_space(3))) void lds_void;
__device__ __forceinline__ void dma16(const void *src, void *lds) {
    const unsigned a = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_void *)lds);
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(a) : "memory", "m0");
}

__global__ __launch_bounds__(128) void k_r1(int4 *buf, int mode, int flip, unsigned long long *out) {
    __shared__ __attribute__((aligned(16))) int4 sm[12 * 64];
    const int t = threadIdx.x, l = t & 63, w = t >> 6;
    const int4 *src = buf + (size_t)(blockIdx.x * 2 + flip) * 4096;
    int4 *dst = buf + (size_t)(blockIdx.x * 2 + (flip ^ 1)) * 4096;
    int4 acc = make_int4(0, 0, 0, 0);
    unsigned long long t0 = 0, t1 = 0;
    if (w == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        if (mode == 0 || mode == 1) {
            const int n = mode == 0 ? 1 : 12;
            int4 v[12];
#pragma unroll
            for (int k = 0; k < 12; ++k)
                if (k < n) asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v[k]) : "v"(src + k * 64 + l) : "memory");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
            for (int k = 0; k < 12; ++k)
                if (k < n) acc.x += v[k].x;
        } else if (mode == 2 || mode == 3 || mode == 5) {
            const int n = mode == 2 ? 1 : 12;
            for (int k = 0; k < n; ++k) dma16(src + k * 64 + l, sm + k * 64);
            if (mode == 5) {
                int s;
                asm volatile("s_load_dword %0, %1, 0x0" : "=s"(s) : "s"(src + 1024) : "memory");
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                acc.y += s;
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            acc.x += sm[l].x;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        } else if (mode == 4) {
            int s;
            asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(s) : "s"(src + 1024) : "memory");
            acc.x += s;
        }
        t1 = __builtin_amdgcn_s_memtime();
    }
    __syncthreads();
    for (int o = t; o < 192; o += 128) dst[o] = make_int4(o + acc.x, acc.y, 0, flip);
    if (t == 0 && flip) out[blockIdx.x] += t1 - t0;
}

int main() {
    const int B = 256, L = 49;
    int4 *buf;
    unsigned long long *out;
    CK(hipMalloc(&buf, (size_t)B * 2 * 65536));
    CK(hipMemset(buf, 0, (size_t)B * 2 * 65536));
    CK(hipMalloc(&out, sizeof(unsigned long long) * B));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    const char *names[] = {"vgpr1", "vgpr12", "dma1", "dma12", "smem", "mix"};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int mode = 0; mode < 6; ++mode) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        for (int i = 0; i < L; ++i) k_r1<<<B, 128, 0, st>>>(buf, mode, i & 1, out);
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, st));
        CK(hipStreamSynchronize(st));
        CK(hipMemset(out, 0, sizeof(unsigned long long) * B));
        const int R = 10;
        CK(hipEventRecord(e0, st));
        for (int r = 0; r < R; ++r) CK(hipGraphLaunch(ge, st));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::vector<unsigned long long> h(B);
        CK(hipMemcpy(h.data(), out, sizeof(unsigned long long) * B, hipMemcpyDeviceToHost));
        double s = 0;
        for (auto v : h) s += (double)v;
        printf("%-7s round-1 %.0f ticks, %.3f us per launch\n", names[mode], s / (B * R * (L / 2)), ms * 1000.f / (R * L));
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    return 0;
}
