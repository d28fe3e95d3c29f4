// Micro-benchmark (diagnostic, not product): cost of executing code that has not run in this
// dispatch.  One wave per workgroup, 256 workgroups, kernels launched back to back in a stream.
//   straight  N distinct VALU instructions (v_add_u32 with a literal: 8 bytes each), run once
//   loop      the same N adds as a loop over a 64-instruction body
//   far/near  32 taken branches to cold 256-byte-aligned blocks / to the next instruction
// Each wave times its block with s_memtime; the host prints the mean cycles per instruction over
// the last 20 of 30 launches.  Straight-line cycles/instr far above the loop's means the code is
// fetched cold every dispatch.
// Build: hipcc --offload-arch=gfx950 -O3 scripts/icache.hip -o scripts/_icache
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

#define A1 "v_add_u32 %0, 0x12345, %0\n"
#define A8 A1 A1 A1 A1 A1 A1 A1 A1
#define A64 A8 A8 A8 A8 A8 A8 A8 A8
#define A512 A64 A64 A64 A64 A64 A64 A64 A64

__global__ void k_straight(unsigned long long *out, int *sink) {
    int v = threadIdx.x;
    unsigned long long t0, t1;
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    asm volatile(A512 A512 A512 A512 : "+v"(v));  // 2048 adds, 16 KiB of code
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
    if (v == -1) *sink = v;
}

__global__ void k_loop(unsigned long long *out, int *sink) {
    int v = threadIdx.x;
    unsigned long long t0, t1;
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    for (int i = 0; i < 32; ++i) asm volatile(A64 : "+v"(v));  // 2048 adds, 512 B of code
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
    if (v == -1) *sink = v;
}


// 32 taken branches, each to a fresh 256-byte-aligned block (cold line per jump) / to the next
// instruction (same lines)
__global__ void k_far(unsigned long long *out, int *sink) {
    unsigned long long t0, t1;
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    asm volatile(
        "s_branch 1f\n .p2align 8\n 1:\n"
        "s_branch 2f\n .p2align 8\n 2:\n"
        "s_branch 3f\n .p2align 8\n 3:\n"
        "s_branch 4f\n .p2align 8\n 4:\n"
        "s_branch 5f\n .p2align 8\n 5:\n"
        "s_branch 6f\n .p2align 8\n 6:\n"
        "s_branch 7f\n .p2align 8\n 7:\n"
        "s_branch 8f\n .p2align 8\n 8:\n"
        "s_branch 9f\n .p2align 8\n 9:\n"
        "s_branch 10f\n .p2align 8\n 10:\n"
        "s_branch 11f\n .p2align 8\n 11:\n"
        "s_branch 12f\n .p2align 8\n 12:\n"
        "s_branch 13f\n .p2align 8\n 13:\n"
        "s_branch 14f\n .p2align 8\n 14:\n"
        "s_branch 15f\n .p2align 8\n 15:\n"
        "s_branch 16f\n .p2align 8\n 16:\n"
        "s_branch 17f\n .p2align 8\n 17:\n"
        "s_branch 18f\n .p2align 8\n 18:\n"
        "s_branch 19f\n .p2align 8\n 19:\n"
        "s_branch 20f\n .p2align 8\n 20:\n"
        "s_branch 21f\n .p2align 8\n 21:\n"
        "s_branch 22f\n .p2align 8\n 22:\n"
        "s_branch 23f\n .p2align 8\n 23:\n"
        "s_branch 24f\n .p2align 8\n 24:\n"
        "s_branch 25f\n .p2align 8\n 25:\n"
        "s_branch 26f\n .p2align 8\n 26:\n"
        "s_branch 27f\n .p2align 8\n 27:\n"
        "s_branch 28f\n .p2align 8\n 28:\n"
        "s_branch 29f\n .p2align 8\n 29:\n"
        "s_branch 30f\n .p2align 8\n 30:\n"
        "s_branch 31f\n .p2align 8\n 31:\n"
        "s_branch 32f\n .p2align 8\n 32:\n"
        :::"memory");
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
}
__global__ void k_near(unsigned long long *out, int *sink) {
    unsigned long long t0, t1;
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    asm volatile(
        "s_branch 1f\n 1:\n"
        "s_branch 2f\n 2:\n"
        "s_branch 3f\n 3:\n"
        "s_branch 4f\n 4:\n"
        "s_branch 5f\n 5:\n"
        "s_branch 6f\n 6:\n"
        "s_branch 7f\n 7:\n"
        "s_branch 8f\n 8:\n"
        "s_branch 9f\n 9:\n"
        "s_branch 10f\n 10:\n"
        "s_branch 11f\n 11:\n"
        "s_branch 12f\n 12:\n"
        "s_branch 13f\n 13:\n"
        "s_branch 14f\n 14:\n"
        "s_branch 15f\n 15:\n"
        "s_branch 16f\n 16:\n"
        "s_branch 17f\n 17:\n"
        "s_branch 18f\n 18:\n"
        "s_branch 19f\n 19:\n"
        "s_branch 20f\n 20:\n"
        "s_branch 21f\n 21:\n"
        "s_branch 22f\n 22:\n"
        "s_branch 23f\n 23:\n"
        "s_branch 24f\n 24:\n"
        "s_branch 25f\n 25:\n"
        "s_branch 26f\n 26:\n"
        "s_branch 27f\n 27:\n"
        "s_branch 28f\n 28:\n"
        "s_branch 29f\n 29:\n"
        "s_branch 30f\n 30:\n"
        "s_branch 31f\n 31:\n"
        "s_branch 32f\n 32:\n"
        :::"memory");
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
}

int main() {
    const int B = 256, reps = 30;
    unsigned long long *d_out;
    int *sink;
    CK(hipMalloc(&d_out, sizeof(unsigned long long) * B * reps * 4));
    CK(hipMalloc(&sink, 4));
    for (int r = 0; r < reps; ++r) {
        hipLaunchKernelGGL(k_straight, dim3(B), dim3(64), 0, 0, d_out + (size_t)r * B, sink);
        hipLaunchKernelGGL(k_loop, dim3(B), dim3(64), 0, 0, d_out + (size_t)(reps + r) * B, sink);
        hipLaunchKernelGGL(k_far, dim3(B), dim3(64), 0, 0, d_out + (size_t)(2 * reps + r) * B, sink);
        hipLaunchKernelGGL(k_near, dim3(B), dim3(64), 0, 0, d_out + (size_t)(3 * reps + r) * B, sink);
    }
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> h((size_t)B * reps * 4);
    CK(hipMemcpy(h.data(), d_out, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost));
    const char *names[4] = {"straight", "loop", "far jumps", "near jumps"};
    const double per[4] = {2048.0, 2048.0, 32.0, 32.0};
    for (int k = 0; k < 4; ++k) {
        double s = 0;
        int n = 0;
        for (int r = 10; r < reps; ++r)
            for (int b = 0; b < B; ++b, ++n) s += (double)h[(size_t)(k * reps + r) * B + b];
        double first = 0;
        for (int b = 0; b < B; ++b) first += (double)h[(size_t)(k * reps) * B + b];
        printf("%s: %.0f cycles per wave (%.2f per unit); first launch %.0f\n", names[k], s / n, s / n / per[k],
               first / B);
    }
    return 0;
}
