// Micro-benchmark (diagnostic, not product): per-launch cost of back-to-back kernels in a HIP graph
// when each launch reads what the previous one wrote (one workgroup of 256 threads per CU, 256
// workgroups, 49 launches per graph, as the fused tree kernels run):
//   empty         nothing
//   write W       each workgroup stores W bytes (16 B per lane, coalesced)
//   read R        each workgroup loads R bytes the previous launch wrote, waits, exits
//   rw R W        both (loads first, stores after they landed)
//   chain2 R      two dependent load rounds of R bytes each (the address of round 2 from round 1)
//   dma R W       the loads as LDS-DMA (global_load_lds_dwordx4), waited, read back from LDS
//   smem W        one wave's scalar load of 64 bytes the previous launch wrote, then the stores
// Build: hipcc --offload-arch=gfx950 -O3 scripts/boundary.hip -o scripts/_boundary
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

typedef __attribute__((address_space(3))) void lds_void;
__device__ __forceinline__ void dma16(const void *src, void *lds) {
    const unsigned a = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_void *)lds);
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(a) : "memory", "m0");
}

__global__ __launch_bounds__(256) void k_dma(int4 *buf, int rd, int wr, int flip) {
    __shared__ __attribute__((aligned(16))) int4 sm[1024];
    const int t = threadIdx.x;
    int4 *src = buf + (size_t)(blockIdx.x * 2 + flip) * 4096;
    int4 *dst = buf + (size_t)(blockIdx.x * 2 + (flip ^ 1)) * 4096;
    const int w = t >> 6, l = t & 63;
    for (int o = w * 64; o < rd / 16; o += 256) dma16(src + o + l, sm + o);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int4 acc = sm[t & 1023];
    for (int o = t; o < wr / 16; o += 256) dst[o] = make_int4(o + acc.x, acc.y, acc.z, flip);
}

__global__ __launch_bounds__(256) void k_smem(int4 *buf, int wr, int flip) {
    const int t = threadIdx.x;
    const int *src = (const int *)(buf + (size_t)(blockIdx.x * 2 + flip) * 4096);
    int4 *dst = buf + (size_t)(blockIdx.x * 2 + (flip ^ 1)) * 4096;
    int v;
    asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(src) : "memory");
    for (int o = t; o < wr / 16; o += 256) dst[o] = make_int4(o + v, v, 0, flip);
}

__global__ __launch_bounds__(256) void k_io(int4 *buf, int rd, int wr, int chain, int flip) {
    const int t = threadIdx.x;
    int4 *src = buf + (size_t)(blockIdx.x * 2 + flip) * 4096;      // 64 KiB per slot
    int4 *dst = buf + (size_t)(blockIdx.x * 2 + (flip ^ 1)) * 4096;
    int4 acc = make_int4(0, 0, 0, 0);
    for (int o = t; o < rd / 16; o += 256) {
        const int4 v = src[o];
        acc.x += v.x;
        acc.y += v.y;
    }
    if (chain) {
        const int j = (acc.x & 7) + t;  // round 2 depends on round 1
        for (int o = j; o < j + rd / 16; o += 256) {
            const int4 v = src[2048 + (o & 2047)];
            acc.z += v.z;
        }
    }
    for (int o = t; o < wr / 16; o += 256) dst[o] = make_int4(o + acc.x, acc.y, acc.z, flip);
}

int main() {
    const int B = 256, L = 49;
    int4 *buf;
    CK(hipMalloc(&buf, (size_t)B * 2 * 65536));
    CK(hipMemset(buf, 0, (size_t)B * 2 * 65536));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    struct Cfg {
        const char *name;
        int rd, wr, chain;
    } cfgs[] = {{"empty", 0, 0, 0},          {"write 3K", 0, 3072, 0},   {"write 16K", 0, 16384, 0},
                {"read 3K", 3072, 0, 0},     {"read 16K", 16384, 0, 0},  {"rw 3K 3K", 3072, 3072, 0},
                {"rw 16K 16K", 16384, 16384, 0}, {"chain2 3K", 3072, 0, 1}, {"chain2 3K w3K", 3072, 3072, 1},
                {"dma 3K w3K", 3072, 3072, 2}, {"dma 16K w3K", 16384, 3072, 2}, {"smem w3K", 0, 3072, 3},
                {"rw 3K 3K (again)", 3072, 3072, 0}, {"empty (again)", 0, 0, 0}};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (auto &c : cfgs) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        for (int i = 0; i < L; ++i) {
            if (c.chain == 2) k_dma<<<B, 256, 0, st>>>(buf, c.rd, c.wr, i & 1);
            else if (c.chain == 3) k_smem<<<B, 256, 0, st>>>(buf, c.wr, i & 1);
            else k_io<<<B, 256, 0, st>>>(buf, c.rd, c.wr, c.chain, i & 1);
        }
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int w = 0; w < 5; ++w) CK(hipGraphLaunch(ge, st));
        CK(hipStreamSynchronize(st));
        float best = 1e30f;
        for (int r = 0; r < 20; ++r) {
            CK(hipEventRecord(e0, st));
            CK(hipGraphLaunch(ge, st));
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        printf("%-16s %.3f us per launch\n", c.name, best * 1000.f / L);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    return 0;
}
