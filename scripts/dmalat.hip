// Micro-benchmark (diagnostic, not product): issue and completion costs of the memory operations
// the tree kernels chain, in s_memtime ticks, measured by wave 0 of a 4-wave workgroup per CU
// (256 workgroups), cold addresses (a fresh 64 MiB window per launch):
//   memtime   back-to-back s_memtime with a wait between (the stamp's own cost)
//   dma_issue 8 global_load_lds_dword (asm, m0 per instruction) issued, no wait
//   dma_wait  ... then s_waitcnt vmcnt(0)
//   vld_issue 8 global_load_dword into VGPRs issued, no wait
//   vld_wait  ... then s_waitcnt vmcnt(0)
//   lds_idle  ds_read_b32 + s_waitcnt lgkmcnt(0), nothing else outstanding
//   lds_dma   the same right after 8 LDS-DMA loads were issued (still in flight)
//   smem      s_load_dword (cold) + s_waitcnt lgkmcnt(0)
//   lds_smem  ds_read_b32 + lgkmcnt(0) right after a cold s_load_dword was issued
// With BUSY=1 waves 1-3 issue 24 LDS-DMA dwordx4 loads each at the same time (round-1 traffic).
// Build: hipcc --offload-arch=gfx950 -O3 -Wno-inline-asm scripts/dmalat.hip -o scripts/_dmalat
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
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

__device__ __forceinline__ unsigned long long mt() { return __builtin_amdgcn_s_memtime(); }
__device__ __forceinline__ void wlgkm() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void wvm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void dma4(const void *src, void *lds) {
    const unsigned a = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_void *)lds);
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(src), "s"(a) : "memory", "m0");
}
__device__ __forceinline__ void dma16(const void *src, void *lds) {
    const unsigned a = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_void *)lds);
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(a) : "memory", "m0");
}

constexpr int kN = 9;

__global__ __launch_bounds__(256) void k_dma(const int *buf, long long win, int busy, unsigned long long *out) {
    __shared__ __attribute__((aligned(16))) int lds[8192];
    const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int *b = buf + win + (long long)blockIdx.x * 65536;  // 256 KiB per block
    unsigned long long r[kN] = {0};
    __syncthreads();
    if (wv > 0) {
        if (busy)
            for (int k = 0; k < 24; ++k) dma16(b + 32768 + wv * 8192 + k * 256 + l * 4, lds + 2048 + (wv - 1) * 2048 + (k & 7) * 256);
        wvm();
        return;
    }
    unsigned long long t0, t1, t2;
    // memtime
    t0 = mt();
    wlgkm();
    t1 = mt();
    wlgkm();
    r[0] = t1 - t0;
    // dma
    t0 = mt();
#pragma unroll
    for (int k = 0; k < 8; ++k) dma4(b + k * 1024 + l, lds + k * 64);
    t1 = mt();
    wvm();
    t2 = mt();
    wlgkm();
    r[1] = t1 - t0;
    r[2] = t2 - t0;
    // vgpr loads
    int v[8];
    t0 = mt();
#pragma unroll
    for (int k = 0; k < 8; ++k) asm volatile("global_load_dword %0, %1, off" : "=v"(v[k]) : "v"(b + 8192 + k * 1024 + l) : "memory");
    t1 = mt();
    wvm();
    t2 = mt();
    wlgkm();
    r[3] = t1 - t0;
    r[4] = t2 - t0;
    int s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += v[k];
    // lds idle
    int x;
    t0 = mt();
    wlgkm();
    t0 = mt();
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(x) : "v"(l * 4) : "memory");
    t1 = mt();
    wlgkm();
    r[5] = t1 - t0;
    s += x;
    // lds with dma in flight
#pragma unroll
    for (int k = 0; k < 8; ++k) dma4(b + 16384 + k * 1024 + l, lds + 512 + k * 64);
    t0 = mt();
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(x) : "v"(l * 4 + 4) : "memory");
    t1 = mt();
    wlgkm();
    r[6] = t1 - t0;
    s += x;
    wvm();
    // smem cold
    int sv;
    t0 = mt();
    wlgkm();
    t0 = mt();
    asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(sv) : "s"(b + 24576) : "memory");
    t1 = mt();
    wlgkm();
    r[7] = t1 - t0;
    s += sv;
    // lds right after a cold smem
    int sv2;
    t0 = mt();
    wlgkm();
    t0 = mt();
    asm volatile("s_load_dword %0, %2, 0x0\n\tds_read_b32 %1, %3\n\ts_waitcnt lgkmcnt(0)" : "=s"(sv2), "=v"(x) : "s"(b + 28672), "v"(l * 4 + 8) : "memory");
    t1 = mt();
    wlgkm();
    r[8] = t1 - t0;
    s += sv2 + x;
    if (l == 0)
        for (int k = 0; k < kN; ++k) out[(size_t)blockIdx.x * kN + k] = r[k] + (s == 0x7fffffff ? 1 : 0);
}

int main() {
    const int B = 256;
    const long long win = 64ll << 20;  // ints per launch window (256 MiB)
    const int nl = 8;
    int *buf;
    unsigned long long *out;
    CK(hipMalloc(&buf, sizeof(int) * win * (nl + 1)));
    CK(hipMemset(buf, 0, sizeof(int) * win * (nl + 1)));
    CK(hipMalloc(&out, sizeof(unsigned long long) * B * kN));
    const char *names[kN] = {"memtime", "dma_issue", "dma_wait", "vld_issue", "vld_wait", "lds_idle", "lds_dma", "smem", "lds_smem"};
    for (int busy = 0; busy < 2; ++busy) {
        std::vector<double> acc(kN, 0.0);
        for (int it = 0; it < nl; ++it) {
            k_dma<<<B, 256>>>(buf, (it + 1) * win, busy, out);
            CK(hipDeviceSynchronize());
            std::vector<unsigned long long> h(B * kN);
            CK(hipMemcpy(h.data(), out, sizeof(unsigned long long) * B * kN, hipMemcpyDeviceToHost));
            if (it == 0) continue;  // cold code
            for (int b = 0; b < B; ++b)
                for (int k = 0; k < kN; ++k) acc[k] += (double)h[(size_t)b * kN + k];
        }
        printf("busy=%d:", busy);
        for (int k = 0; k < kN; ++k) printf(" %s=%.0f", names[k], acc[k] / (B * (nl - 1)));
        printf("\n");
    }
    return 0;
}
