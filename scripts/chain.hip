// Micro-benchmark (diagnostic, not product): cycles per step of the serial f32 recurrence
// b = r_k + g * b (the back-propagation bootstrap chain) in several formulations, one wave per CU.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off scripts/chain.hip -o scripts/_chain
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>
#include <cstring>

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
constexpr int kSteps = 48;

// 0: pure VGPR chain, inline asm (mul, add), rewards in VGPRs
__global__ void k0(const float *r, float g, unsigned long long *out, float *sink) {
    const int l = threadIdx.x;
    float rr[8];
    for (int j = 0; j < 8; ++j) rr[j] = r[j];
    float b = r[9];
    const unsigned long long t0 = memtime();
#pragma unroll
    for (int k = 0; k < kSteps; ++k) {
        asm volatile("v_mul_f32 %0, %1, %0\n v_add_f32 %0, %2, %0" : "+v"(b) : "s"(g), "v"(rr[k & 7]));
    }
    const unsigned long long t1 = memtime();
    if (l == 0) out[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * 64 + l] = b;
}
// 1: rewards read with v_readlane from one VGPR (lane k), compiled
__global__ void k1(const float *r, float g, unsigned long long *out, float *sink) {
    const int l = threadIdx.x;
    const float rn = r[l];
    float b = __builtin_amdgcn_readfirstlane(__float_as_int(r[70])) * 1.0f;
    const unsigned long long t0 = memtime();
#pragma unroll
    for (int k = 0; k < kSteps; ++k) b = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(rn), k)) + g * b;
    const unsigned long long t1 = memtime();
    if (l == 0) out[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * 64 + l] = b;
}
// 2: as 1 plus per-lane capture (mine = l == k ? b : mine)
__global__ void k2(const float *r, float g, unsigned long long *out, float *sink) {
    const int l = threadIdx.x;
    const float rn = r[l];
    float b = r[70], mine = 0.f;
    const unsigned long long t0 = memtime();
#pragma unroll
    for (int k = 0; k < kSteps; ++k) {
        b = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(rn), k)) + g * b;
        mine = (l == k) ? b : mine;
    }
    const unsigned long long t1 = memtime();
    if (l == 0) out[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * 64 + l] = mine;
}
// 3: pure VGPR chain with capture through v_cndmask on an SGPR mask built by SALU
__global__ void k3(const float *r, float g, unsigned long long *out, float *sink) {
    const int l = threadIdx.x;
    float rr[8];
    for (int j = 0; j < 8; ++j) rr[j] = r[j];
    float b = r[9], mine = 0.f;
    const unsigned long long t0 = memtime();
#pragma unroll
    for (int k = 0; k < kSteps; ++k) {
        const unsigned long long m = 1ull << k;
        asm volatile("v_mul_f32 %0, %2, %0\n v_add_f32 %0, %3, %0\n v_cndmask_b32_e64 %1, %1, %0, %4"
                     : "+v"(b), "+v"(mine)
                     : "s"(g), "v"(rr[k & 7]), "s"(m));
    }
    const unsigned long long t1 = memtime();
    if (l == 0) out[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * 64 + l] = mine + b;
}
// 4: f64 add chain (pure VGPR)
__global__ void k4(const double *r, unsigned long long *out, double *sink) {
    const int l = threadIdx.x;
    double rr[8];
    for (int j = 0; j < 8; ++j) rr[j] = r[j];
    double b = r[9];
    const unsigned long long t0 = memtime();
#pragma unroll
    for (int k = 0; k < kSteps; ++k) asm volatile("v_add_f64 %0, %1, %0" : "+v"(b) : "v"(rr[k & 7]));
    const unsigned long long t1 = memtime();
    if (l == 0) out[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * 64 + l] = b;
}
// 5: independent VALU ops (issue rate): 2*kSteps v_mul_f32 on 8 independent accumulators
__global__ void k5(const float *r, float g, unsigned long long *out, float *sink) {
    const int l = threadIdx.x;
    float a[8];
    for (int j = 0; j < 8; ++j) a[j] = r[j] + l;
    const unsigned long long t0 = memtime();
#pragma unroll
    for (int k = 0; k < 2 * kSteps; ++k) asm volatile("v_mul_f32 %0, %1, %0" : "+v"(a[k & 7]) : "s"(g));
    const unsigned long long t1 = memtime();
    float s = 0;
    for (int j = 0; j < 8; ++j) s += a[j];
    if (l == 0) out[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * 64 + l] = s;
}
// 6: SGPR written by v_readfirstlane then consumed by a VALU, dependent round trip per step
__global__ void k6(const float *r, float g, unsigned long long *out, float *sink) {
    const int l = threadIdx.x;
    float b = r[9];
    const unsigned long long t0 = memtime();
#pragma unroll
    for (int k = 0; k < kSteps; ++k) {
        int sb;
        asm volatile("v_mul_f32 %1, %2, %1\n v_readfirstlane_b32 %0, %1" : "=s"(sb), "+v"(b) : "s"(g));
        asm volatile("v_add_f32 %0, %1, %0" : "+v"(b) : "s"(sb));
    }
    const unsigned long long t1 = memtime();
    if (l == 0) out[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * 64 + l] = b;
}

// 7: k3's chain in wave 0 while wave 1 of the same workgroup runs VALU work (busy = 1) or exits
__global__ void k7(const float *r, float g, int busy, unsigned long long *out, float *sink) {
    const int l = threadIdx.x & 63;
    if (threadIdx.x >= 64) {
        if (!busy) return;
        float a[8];
        for (int j = 0; j < 8; ++j) a[j] = r[j] + l;
#pragma unroll
        for (int k = 0; k < 8 * kSteps; ++k) asm volatile("v_mul_f32 %0, %1, %0" : "+v"(a[k & 7]) : "s"(g));
        float s = 0;
        for (int j = 0; j < 8; ++j) s += a[j];
        sink[blockIdx.x * 64 + l] = s;
        return;
    }
    float rr[8];
    for (int j = 0; j < 8; ++j) rr[j] = r[j];
    float b = r[9], mine = 0.f;
    const unsigned long long t0 = memtime();
#pragma unroll
    for (int k = 0; k < kSteps; ++k) {
        const unsigned long long m = 1ull << k;
        asm volatile("v_mul_f32 %0, %2, %0\n v_add_f32 %0, %3, %0\n v_cndmask_b32_e64 %1, %1, %0, %4"
                     : "+v"(b), "+v"(mine)
                     : "s"(g), "v"(rr[k & 7]), "s"(m));
    }
    const unsigned long long t1 = memtime();
    if (l == 0) out[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * 64 + l] = mine + b;
}
// 8: hardware ids of the two waves of a workgroup (HW_ID: SIMD id in bits 5:4)
__global__ void k8(unsigned *out) {
    unsigned id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(id));
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 2 + (threadIdx.x >> 6)] = id;
}

// 9: the product's bootstrap loop (grouped v_readlane + SALU-mask capture), runtime level count
__device__ __forceinline__ float rlf(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }
__device__ __forceinline__ float sel_lane(float v, float x, unsigned long long m) {
    asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(v) : "v"(x), "s"(m));
    return v;
}
__global__ void k9(const float *r, float disc, int nl, unsigned long long *out, float *sink) {
    const int l = threadIdx.x;
    const float rn = r[l];
    float carry = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(r[70])));
    unsigned long long t0;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    carry += (t0 == 0) ? 1.f : 0.f;
    float mine = (l == nl) ? carry : 0.f;
    float b = carry;
    int k = nl - 1;
    for (; k >= 7; k -= 8) {
        float r8[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) r8[j] = rlf(rn, k - j);
        asm volatile("" : "+s"(r8[0]), "+s"(r8[1]), "+s"(r8[2]), "+s"(r8[3]), "+s"(r8[4]), "+s"(r8[5]),
                     "+s"(r8[6]), "+s"(r8[7]));
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            b = r8[j] + disc * b;
            mine = sel_lane(mine, b, 1ull << (k - j));
        }
    }
    for (; k >= 0; --k) {
        b = rlf(rn, k) + disc * b;
        mine = sel_lane(mine, b, 1ull << k);
    }
    unsigned long long t1;
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1) : "v"(mine), "v"(b) : "memory");
    if (l == 0) out[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * 64 + l] = mine;
}

// 10: rewards staged in LDS and read back as broadcasts (ds_read2, all lanes one address) one
// block ahead; SALU-mask capture
__global__ void k10(const float *r, float disc, int nl, unsigned long long *out, float *sink) {
    __shared__ float st[64 + 8];
    const int l = threadIdx.x;
    const float rn = r[l];
    float carry = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(r[70])));
    unsigned long long t0;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    carry += (t0 == 0) ? 1.f : 0.f;
    st[l] = rn;  // level l's reward (the product stages it the same way)
    float mine = (l == nl) ? carry : 0.f;
    float b = carry;
    int k = nl - 1;
    // blocks of 8 levels [k-7, k] (clamped reads below level 0 are never used)
    float cur[8], nxt[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) cur[j] = st[k - j >= 0 ? k - j : 0];
    while (k >= 0) {
        const bool more = k >= 8;
        if (more) {
#pragma unroll
            for (int j = 0; j < 8; ++j) nxt[j] = st[k - 8 - j >= 0 ? k - 8 - j : 0];
        }
        if (k >= 7) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                b = cur[j] + disc * b;
                mine = sel_lane(mine, b, 1ull << (k - j));
            }
        } else {
            for (int j = 0; j <= k; ++j) {
                b = cur[j] + disc * b;
                mine = sel_lane(mine, b, 1ull << (k - j));
            }
        }
        k -= 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) cur[j] = nxt[j];
    }
    unsigned long long t1;
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1) : "v"(mine), "v"(b) : "memory");
    if (l == 0) out[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * 64 + l] = mine;
}

// 11: k3 with the lane mask advanced by s_lshr_b64 on one SGPR pair (product's boot_chain4)
__global__ void k11(const float *r, float g, int k0, unsigned long long *out, float *sink) {
    const int l = threadIdx.x;
    float rr[4];
    for (int j = 0; j < 4; ++j) rr[j] = r[j];
    float b = r[9], mine = 0.f;
    const unsigned long long t0 = memtime();
    for (int k = kSteps - 1; k >= 3; k -= 4) {
        unsigned long long m;
        asm volatile(
            "s_lshl_b64 %[m], 1, %[k]\n"
            "v_mul_f32 %[b], %[d], %[b]\n v_add_f32 %[b], %[r0], %[b]\n v_cndmask_b32_e64 %[mi], %[mi], %[b], %[m]\n s_lshr_b64 %[m], %[m], 1\n"
            "v_mul_f32 %[b], %[d], %[b]\n v_add_f32 %[b], %[r1], %[b]\n v_cndmask_b32_e64 %[mi], %[mi], %[b], %[m]\n s_lshr_b64 %[m], %[m], 1\n"
            "v_mul_f32 %[b], %[d], %[b]\n v_add_f32 %[b], %[r2], %[b]\n v_cndmask_b32_e64 %[mi], %[mi], %[b], %[m]\n s_lshr_b64 %[m], %[m], 1\n"
            "v_mul_f32 %[b], %[d], %[b]\n v_add_f32 %[b], %[r3], %[b]\n v_cndmask_b32_e64 %[mi], %[mi], %[b], %[m]\n s_lshr_b64 %[m], %[m], 1\n"
            : [b] "+v"(b), [mi] "+v"(mine), [m] "=&s"(m)
            : [d] "s"(g), [k] "s"(k + k0), [r0] "v"(rr[0]), [r1] "v"(rr[1]), [r2] "v"(rr[2]), [r3] "v"(rr[3]));
    }
    unsigned long long t1;
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1) : "v"(mine), "v"(b) : "memory");
    if (l == 0) out[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * 64 + l] = mine;
}
// 12: k11 without the capture (mul, add only, plus the SALU shift)
__global__ void k12(const float *r, float g, int k0, unsigned long long *out, float *sink) {
    const int l = threadIdx.x;
    float rr[4];
    for (int j = 0; j < 4; ++j) rr[j] = r[j];
    float b = r[9];
    const unsigned long long t0 = memtime();
    for (int k = kSteps - 1; k >= 3; k -= 4) {
        asm volatile(
            "v_mul_f32 %[b], %[d], %[b]\n v_add_f32 %[b], %[r0], %[b]\n"
            "v_mul_f32 %[b], %[d], %[b]\n v_add_f32 %[b], %[r1], %[b]\n"
            "v_mul_f32 %[b], %[d], %[b]\n v_add_f32 %[b], %[r2], %[b]\n"
            "v_mul_f32 %[b], %[d], %[b]\n v_add_f32 %[b], %[r3], %[b]\n"
            : [b] "+v"(b)
            : [d] "s"(g), [r0] "v"(rr[0]), [r1] "v"(rr[1]), [r2] "v"(rr[2]), [r3] "v"(rr[3]));
    }
    unsigned long long t1;
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1) : "v"(b) : "memory");
    if (l == 0) out[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * 64 + l] = b;
}
// 13: as 12 but the multiply reads the discount from a VGPR
__global__ void k13(const float *r, float g, int k0, unsigned long long *out, float *sink) {
    const int l = threadIdx.x;
    float rr[4];
    for (int j = 0; j < 4; ++j) rr[j] = r[j];
    float b = r[9], gv = g + r[l] * 0.f;
    const unsigned long long t0 = memtime();
    for (int k = kSteps - 1; k >= 3; k -= 4) {
        asm volatile(
            "v_mul_f32 %[b], %[d], %[b]\n v_add_f32 %[b], %[r0], %[b]\n"
            "v_mul_f32 %[b], %[d], %[b]\n v_add_f32 %[b], %[r1], %[b]\n"
            "v_mul_f32 %[b], %[d], %[b]\n v_add_f32 %[b], %[r2], %[b]\n"
            "v_mul_f32 %[b], %[d], %[b]\n v_add_f32 %[b], %[r3], %[b]\n"
            : [b] "+v"(b)
            : [d] "v"(gv), [r0] "v"(rr[0]), [r1] "v"(rr[1]), [r2] "v"(rr[2]), [r3] "v"(rr[3]));
    }
    unsigned long long t1;
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1) : "v"(b) : "memory");
    if (l == 0) out[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * 64 + l] = b;
}

// 14: the product's boot_chain4 (v_readlane with SGPR lane selects inside the asm block)
__device__ __forceinline__ void boot_chain4(float &b, float &mine, float disc, float rn, int k) {
    unsigned long long m;
    int r0, r1, r2, r3;
    const int k1 = k - 1, k2 = k - 2, k3 = k - 3;
#define MZ_BOOT_STEP(R)                                 \
    "v_mul_f32 %[b], %[d], %[b]\n"                      \
    "v_add_f32 %[b], %[" R "], %[b]\n"                  \
    "v_cndmask_b32_e64 %[mi], %[mi], %[b], %[m]\n"      \
    "s_lshr_b64 %[m], %[m], 1\n"
    asm volatile(
        "v_readlane_b32 %[r0], %[rn], %[k0]\n"
        "v_readlane_b32 %[r1], %[rn], %[k1]\n"
        "v_readlane_b32 %[r2], %[rn], %[k2]\n"
        "v_readlane_b32 %[r3], %[rn], %[k3]\n"
        "s_lshl_b64 %[m], 1, %[k0]\n" MZ_BOOT_STEP("r0") MZ_BOOT_STEP("r1") MZ_BOOT_STEP("r2") MZ_BOOT_STEP("r3")
        : [b] "+v"(b), [mi] "+v"(mine), [m] "=&s"(m), [r0] "=&s"(r0), [r1] "=&s"(r1), [r2] "=&s"(r2), [r3] "=&s"(r3)
        : [d] "s"(disc), [rn] "v"(rn), [k0] "s"(k), [k1] "s"(k1), [k2] "s"(k2), [k3] "s"(k3));
#undef MZ_BOOT_STEP
}
__global__ void k14(const float *r, float disc, int nl, unsigned long long *out, float *sink) {
    const int l = threadIdx.x;
    const float rn = r[l];
    float b = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(r[70])));
    unsigned long long t0;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    b += (t0 == 0) ? 1.f : 0.f;
    float mine = 0.f;
    int k = nl - 1;
    for (; k >= 3; k -= 4) boot_chain4(b, mine, disc, rn, k);
    unsigned long long t1;
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1) : "v"(mine), "v"(b) : "memory");
    if (l == 0) out[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * 64 + l] = mine;
}
// 15: readlane only: 48 v_readlane_b32 with SGPR lane select, results summed by SALU
__global__ void k15(const float *r, float disc, int nl, unsigned long long *out, float *sink) {
    const int l = threadIdx.x;
    const float rn = r[l];
    unsigned long long t0;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    int acc = 0;
    for (int k = nl - 1; k >= 3; k -= 4) {
        int r0, r1, r2, r3;
        asm volatile(
            "v_readlane_b32 %[r0], %[rn], %[k0]\n"
            "v_readlane_b32 %[r1], %[rn], %[k1]\n"
            "v_readlane_b32 %[r2], %[rn], %[k2]\n"
            "v_readlane_b32 %[r3], %[rn], %[k3]\n"
            : [r0] "=&s"(r0), [r1] "=&s"(r1), [r2] "=&s"(r2), [r3] "=&s"(r3)
            : [rn] "v"(rn), [k0] "s"(k), [k1] "s"(k - 1), [k2] "s"(k - 2), [k3] "s"(k - 3));
        acc ^= r0 ^ r1 ^ r2 ^ r3;
    }
    unsigned long long t1;
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1) : "s"(acc) : "memory");
    if (l == 0) out[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * 64 + l] = acc;
}

// 16: lane-parallel chain: level i at lane 63 - (top - i); each step every lane takes its upper
// neighbour's b through DPP wave_shl:1 fused into the multiply; lane 63 (the carry) is outside
// EXEC, and the lane below it has tmp pre-set to disc * carry (so either DPP semantics for an
// inactive source lane gives the right value).  out2 gets lanes' b for checking.
__global__ void k16(const float *r, float disc, int nl, unsigned long long *out, float *outb) {
    const int l = threadIdx.x;
    const float carry = r[70];
    const float rn = r[l];  // lane l's reward (any values)
    const float dv = disc + r[l] * 0.f;  // VGPR copy of the discount
    float b = (l == 63) ? carry : 0.f;
    float tmp = (l == 62) ? disc * carry : 0.f;
    unsigned long long t0;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    b += (t0 == 0) ? 1.f : 0.f;
    if (nl > 0) {
        unsigned long long saved;
        int n4 = nl >> 2, n1 = nl & 3;
#define STEP "s_nop 1\n v_mul_f32_dpp %[t], %[b], %[d] wave_shl:1 row_mask:0xf bank_mask:0xf\n v_add_f32 %[b], %[r], %[t]\n"
        asm volatile(
            "s_mov_b64 %[sv], exec\n"
            "s_bitset0_b64 exec, 63\n"
            "s_cmp_eq_u32 %[n4], 0\n"
            "s_cbranch_scc1 2f\n"
            "1:\n" STEP STEP STEP STEP
            "s_sub_u32 %[n4], %[n4], 1\n"
            "s_cmp_lg_u32 %[n4], 0\n"
            "s_cbranch_scc1 1b\n"
            "2:\n"
            "s_cmp_eq_u32 %[n1], 0\n"
            "s_cbranch_scc1 4f\n"
            "3:\n" STEP
            "s_sub_u32 %[n1], %[n1], 1\n"
            "s_cmp_lg_u32 %[n1], 0\n"
            "s_cbranch_scc1 3b\n"
            "4:\n"
            "s_mov_b64 exec, %[sv]\n"
            : [b] "+v"(b), [t] "+v"(tmp), [sv] "=&s"(saved), [n4] "+s"(n4), [n1] "+s"(n1)
            : [d] "v"(dv), [r] "v"(rn)
            : "memory", "scc");
#undef STEP
    }
    unsigned long long t1;
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1) : "v"(b) : "memory");
    if (l == 0) out[blockIdx.x] = t1 - t0;
    outb[blockIdx.x * 64 + l] = b;
}

int main() {
    const int B = 256;
    float *r, *sink;
    double *rd, *sinkd;
    unsigned long long *out;
    CK(hipMalloc(&r, 128 * 4));
    CK(hipMalloc(&rd, 128 * 8));
    CK(hipMalloc(&sink, B * 64 * 4));
    CK(hipMalloc(&sinkd, B * 64 * 8));
    CK(hipMalloc(&out, B * 8));
    std::vector<float> hr(128);
    for (int i = 0; i < 128; ++i) hr[i] = 0.01f * i;
    CK(hipMemcpy(r, hr.data(), 128 * 4, hipMemcpyHostToDevice));
    CK(hipMemset(rd, 0, 128 * 8));
    std::vector<unsigned long long> h(B);
    auto run = [&](const char *name, auto launch) {
        launch();
        launch();
        hipDeviceSynchronize();
        hipMemcpy(h.data(), out, B * 8, hipMemcpyDeviceToHost);
        std::sort(h.begin(), h.end());
        printf("%-44s median %6.0f cycles = %5.1f per step\n", name, (double)h[B / 2], (double)h[B / 2] / kSteps);
    };
    const float g = 0.997f;
    run("0 asm chain mul+add (VGPR operands)", [&] { hipLaunchKernelGGL(k0, dim3(B), dim3(64), 0, 0, r, g, out, sink); });
    run("1 readlane-fed chain", [&] { hipLaunchKernelGGL(k1, dim3(B), dim3(64), 0, 0, r, g, out, sink); });
    run("2 readlane-fed chain + cmp/cndmask capture", [&] { hipLaunchKernelGGL(k2, dim3(B), dim3(64), 0, 0, r, g, out, sink); });
    run("3 asm chain + cndmask on SALU mask", [&] { hipLaunchKernelGGL(k3, dim3(B), dim3(64), 0, 0, r, g, out, sink); });
    run("4 f64 add chain", [&] { hipLaunchKernelGGL(k4, dim3(B), dim3(64), 0, 0, rd, out, sinkd); });
    run("5 independent v_mul_f32 x2 (issue rate)", [&] { hipLaunchKernelGGL(k5, dim3(B), dim3(64), 0, 0, r, g, out, sink); });
    run("6 VALU->readfirstlane->VALU round trip", [&] { hipLaunchKernelGGL(k6, dim3(B), dim3(64), 0, 0, r, g, out, sink); });
    for (int nl : {8, 25, 48}) {
        char nm[64];
        snprintf(nm, sizeof nm, "9 product bootstrap loop, %d levels (per level)", nl);
        hipLaunchKernelGGL(k9, dim3(B), dim3(64), 0, 0, r, g, nl, out, sink);
        hipLaunchKernelGGL(k9, dim3(B), dim3(64), 0, 0, r, g, nl, out, sink);
        hipDeviceSynchronize();
        hipMemcpy(h.data(), out, B * 8, hipMemcpyDeviceToHost);
        std::sort(h.begin(), h.end());
        printf("%-52s median %6.0f cycles = %5.1f per level\n", nm, (double)h[B / 2], (double)h[B / 2] / nl);
    }
    for (int nl : {8, 25, 48}) {
        hipLaunchKernelGGL(k10, dim3(B), dim3(64), 0, 0, r, g, nl, out, sink);
        hipLaunchKernelGGL(k10, dim3(B), dim3(64), 0, 0, r, g, nl, out, sink);
        hipDeviceSynchronize();
        hipMemcpy(h.data(), out, B * 8, hipMemcpyDeviceToHost);
        std::sort(h.begin(), h.end());
        printf("10 LDS-broadcast bootstrap loop, %2d levels         median %6.0f cycles = %5.1f per level\n", nl, (double)h[B / 2], (double)h[B / 2] / nl);
    }
    run("11 k3 + s_lshr mask chain (product chain4)", [&] { hipLaunchKernelGGL(k11, dim3(B), dim3(64), 0, 0, r, g, 0, out, sink); });
    run("12 mul+add only, 4-step asm blocks", [&] { hipLaunchKernelGGL(k12, dim3(B), dim3(64), 0, 0, r, g, 0, out, sink); });
    run("13 as 12, discount in a VGPR", [&] { hipLaunchKernelGGL(k13, dim3(B), dim3(64), 0, 0, r, g, 0, out, sink); });
    run("14 product boot_chain4 (readlane in asm), 48 lv", [&] { hipLaunchKernelGGL(k14, dim3(B), dim3(64), 0, 0, r, g, 48, out, sink); });
    run("15 v_readlane x4 blocks only, 48", [&] { hipLaunchKernelGGL(k15, dim3(B), dim3(64), 0, 0, r, g, 48, out, sink); });
    for (int nl : {25, 63}) {
        for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(k16, dim3(B), dim3(64), 0, 0, r, g, nl, out, sink);
        hipDeviceSynchronize();
        hipMemcpy(h.data(), out, B * 8, hipMemcpyDeviceToHost);
        std::vector<float> hb(64);
        hipMemcpy(hb.data(), sink, 64 * 4, hipMemcpyDeviceToHost);
        std::sort(h.begin(), h.end());
        // host reference: lane 63 = carry; lane j = r[j] + g * b[j+1] for j in [63-nl, 62]
        std::vector<float> ref(64, 0.f);
        ref[63] = hr[70];
        int bad = 0;
        for (int j = 62; j >= 63 - nl; --j) {
            volatile float t = g * ref[j + 1];
            ref[j] = hr[j] + t;
        }
        for (int j = 63 - nl; j < 64; ++j) bad += (memcmp(&ref[j], &hb[j], 4) != 0);
        printf("16 DPP lane-parallel chain, %2d levels             median %6.0f cycles = %5.1f per level, mismatches %d\n", nl, (double)h[B / 2], (double)h[B / 2] / nl, bad);
    }
    run("7 k3 chain, sibling wave idle", [&] { hipLaunchKernelGGL(k7, dim3(B), dim3(128), 0, 0, r, g, 0, out, sink); });
    run("7 k3 chain, sibling wave VALU-busy", [&] { hipLaunchKernelGGL(k7, dim3(B), dim3(128), 0, 0, r, g, 1, out, sink); });
    {
        unsigned *ids;
        CK(hipMalloc(&ids, B * 2 * 4));
        hipLaunchKernelGGL(k8, dim3(B), dim3(128), 0, 0, ids);
        std::vector<unsigned> hid(B * 2);
        CK(hipMemcpy(hid.data(), ids, B * 2 * 4, hipMemcpyDeviceToHost));
        int same = 0;
        for (int i = 0; i < B; ++i) same += (((hid[2 * i] >> 4) & 3) == ((hid[2 * i + 1] >> 4) & 3));
        printf("8 workgroups whose two waves share a SIMD: %d of %d (first: simd %u / %u)\n", same, B,
               (hid[0] >> 4) & 3, (hid[1] >> 4) & 3);
    }
    return 0;
}
