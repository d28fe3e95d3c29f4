// Micro-benchmark (diagnostic, not product): dependent-chain latencies inside one wave, in
// s_memtime ticks per step (one workgroup of one wave per CU, 256 workgroups, warm launches):
//   lds       ds_read_b32 pointer chase (uniform address, then v_readfirstlane into the address)
//   ldsv      ds_read_b32 pointer chase with the address kept in a VGPR
//   fmuladd   f32 multiply then add (b = r + d * b), operands in VGPRs
//   fsgpr     the same with r from an SGPR
//   dpp       v_mul_f32_dpp wave_shl:1 + v_add_f32 (the DPP bootstrap step)
//   rfl       v_readfirstlane -> s_add -> v_mov round trip
// Build: hipcc --offload-arch=gfx950 -O3 scripts/lat.hip -o scripts/_lat
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

__device__ __forceinline__ unsigned long long memtime() {
    unsigned long long t;
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

constexpr int kSteps = 256;

__global__ void k_lat(unsigned long long *out, float *sink) {
    __shared__ int nxt[1024];
    const int l = threadIdx.x;
    for (int i = l; i < 1024; i += 64) nxt[i] = (i * 37 + 11) & 1023;
    __syncthreads();
    unsigned long long t[7];
    // lds: uniform pointer chase
    int x = 0;
    t[0] = memtime();
    for (int k = 0; k < kSteps; ++k) x = __builtin_amdgcn_readfirstlane(nxt[x]);
    t[1] = memtime();
    // ldsv: VGPR pointer chase
    int xv = l * 4;
    for (int k = 0; k < kSteps; ++k) {
        asm volatile("ds_read_b32 %0, %0\n s_waitcnt lgkmcnt(0)" : "+v"(xv)::"memory");
        xv = (xv & 1023) << 2;
    }
    t[2] = memtime();
    // fmuladd: VGPR operands
    float b = 1.0f + l, d = 0.997f, r = 0.5f;
    for (int k = 0; k < kSteps; ++k) asm volatile("v_mul_f32 %0, %1, %0\n v_add_f32 %0, %2, %0" : "+v"(b) : "v"(d), "v"(r));
    t[3] = memtime();
    // fsgpr: r from an SGPR
    float rs = __builtin_amdgcn_readfirstlane(__float_as_int(r)) * 1.0f;
    for (int k = 0; k < kSteps; ++k) asm volatile("v_mul_f32 %0, %1, %0\n v_add_f32 %0, %2, %0" : "+v"(b) : "v"(d), "s"(rs));
    t[4] = memtime();
    // dpp: the bootstrap step
    float tmp = 0.f;
    for (int k = 0; k < kSteps; ++k)
        asm volatile("s_nop 1\n v_mul_f32_dpp %1, %0, %2 wave_shl:1 row_mask:0xf bank_mask:0xf\n v_add_f32 %0, %3, %1"
                     : "+v"(b), "+v"(tmp) : "v"(d), "v"(r));
    t[5] = memtime();
    // rfl: VGPR -> SGPR -> VGPR
    int v = l;
    for (int k = 0; k < kSteps; ++k) {
        int sv = __builtin_amdgcn_readfirstlane(v);
        asm volatile("s_add_u32 %0, %0, 1" : "+s"(sv)::"scc");
        v = sv + l;
    }
    t[6] = memtime();
    if (l == 0)
        for (int k = 0; k < 6; ++k) out[blockIdx.x * 6 + k] = t[k + 1] - t[k];
    if (x == -1 || b == 12345.f || xv == -1 || v == -1) sink[0] = b + tmp;
}

int main() {
    const int B = 256, reps = 10;
    unsigned long long *d;
    float *sink;
    CK(hipMalloc(&d, sizeof(unsigned long long) * B * 6));
    CK(hipMalloc(&sink, 4));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_lat, dim3(B), dim3(64), 0, 0, d, sink);
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> h(B * 6);
    CK(hipMemcpy(h.data(), d, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost));
    const char *names[6] = {"lds (uniform chase)", "ldsv (vgpr chase)", "fmuladd", "fsgpr", "dpp", "rfl"};
    for (int k = 0; k < 6; ++k) {
        double s = 0;
        for (int b = 0; b < B; ++b) s += (double)h[b * 6 + k];
        printf("%-20s %.1f ticks per step\n", names[k], s / B / kSteps);
    }
    return 0;
}
