// mzmcts.hip — MI355X (gfx950) batched sampled-MCTS tree: HIP kernels + the C-ABI of
// include/mzmcts.h.  Replaces the reference's CPU tree core (core/mcts/ctree/ctree_sampled/lib/
// cnode.{h,cpp}, common_lib/utils.{h,cpp}) behind the same Tree_batch surface.
//
// Execution model.  One wavefront owns one tree for the whole kernel (grid = #trees, block = 64):
// no cross-tree interaction exists in the algorithm (cnode.cpp:633-641, 663-669), so there is no
// inter-workgroup communication at all.  Each launch stages the tree's node records from HBM into
// LDS with LDS-DMA (global_load_lds), walks / updates the tree in LDS, and writes back only what
// it changed.  Per-simulation work is one launch (mz_expand_backup_select) fusing expansion +
// back-propagation of simulation s with the selection of s+1 and the leaf hidden-state gather.
//
// Data layout in HBM (tree-major structure of arrays; node n of tree t at index t*P + n, where
// P = 1 + min(K, A^N)*(S+1) is the nodes a search can create; the reference allocates K*(S+2),
// cnode.cpp:562):
//   A[t][n]  int4  {visit, prior, value, reward}           (value = ws/tw, 0 while unexpanded)
//   Bn[t][n] int4  {first_child, nc | action<<8 | (maxdepth+1)<<16, pred_value, hidden_state_index_x}
//   Q[t][n]  float q = qsa - parent.pred_value, the node's member of the min/max set (cnode.cpp:435,445)
//   PP[t][n] float parent's pred_value (fixed when the node is created)
//   C[t][n]  float4{weighted_sum, tot_weight, -, -}        SubTreeValueSet scalars (utils.h:29)
//   D[t][n]  float4{pred_prob, beta, beta_hat, -}          readback-only
//   V[t][n][E] int2 {depth, value}                         every backed-up value of the node, sorted by
//                                                          (depth, value); E = S+1 = max visits
//   R[t][W]  u32   the tree's pre-generated std::mt19937 stream (cnode.cpp:574)
// Children of a node are contiguous (the reference allocates them consecutively, cnode.cpp:290-292),
// so scoring a node's children is one 16-B-per-lane LDS read.
//
// Bit-exactness.  Built with -ffp-contract=off, correctly rounded f32 division and no fast-math;
// every float expression keeps the reference's operation order.  The pUCT coefficient
// pb_c(n, v) = (float)((double)(logf((n + c2 + 1)/c2) + c1) * (sqrt(n) / (v + 1))) (cnode.cpp:313-314)
// depends only on the parent's total child visits n and the child's visits v <= n; the host
// tabulates it with glibc logf and IEEE double arithmetic, i.e. with exactly the reference's
// operations, so no device transcendental enters a result.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "../../include/mzmcts.h"
#include "../../include/mzdriver.h"
#include "mz_internal.h"
#include "mt_seed.inc"

namespace {

#ifndef MZ_STAMPS
#define MZ_STAMPS 0  // diagnostic build: per-phase s_memtime stamps into the stats counters
#endif

constexpr int kWave = 64;
constexpr int kRngWin = 256;     // RNG words staged in LDS per launch
constexpr int kMaxActions = 64;  // one lane per action
constexpr int kMtN = 624;
constexpr int kTableLdsMax = 48 * 1024;  // the pUCT table is staged in LDS when it fits this
constexpr int kNxt = 32;  // RNG words for the next expansion carried in the tree header (2K <= kNxt)
// the kernels stage a tree's counters as 2 * MZ_S_COUNT dwords, one per lane
static_assert(2 * MZ_S_COUNT <= 64, "statistics staging: one dword per lane");

enum : int {
    kErrPool = 1,      // node pool exhausted (more expansions than simulation_num allows)
    kErrRng = 2,       // pre-generated RNG stream exhausted
    kErrValueSet = 4,  // SubTreeValueSet::update invariant (utils.cpp:130)
    kErrPath = 8,      // search path longer than the pool allows
    kErrRoot = 16,     // selection on an unexpanded root (reference: UB, cnode.cpp:410)
    kErrTable = 32,    // visit count beyond the pUCT table
};

struct TreeHdr {
    int cursor, tot, D, err;
    float mm_min, mm_max;
    int mm_cnt, leaf;
    // 1 while every reward and pred_value of the tree lies in [-1e30, 1e30] and every prior in
    // [0, 1e30]: then (with the handle's fast_ok conditions) no pUCT score can be NaN or below
    // FLOAT_MIN, so a K = 1 selection consumes one engine word per non-forced level (select_walk)
    int tame;
    unsigned nxt[kNxt];  // R[cursor .. cursor + kNxt): the next expansion's engine words
};

struct Geo {
    int B, A, K, S, P, E, W, PS;
    int TT;         // pUCT table entries (PS*(PS+1)/2, padded to 4)
    int use_table;  // pUCT table staged in LDS (else pb/sq tables + double arithmetic)
    int root_offset;
    unsigned seed;
    float one_minus_rho, delta;
    int reg_cap;  // value entries staged in LDS per back-propagation chunk
    // dynamic-LDS byte offsets of k_step
    int oA, oB, oQ, oPP, oVs, oC, oPath, oFlag, oT, oPb, oSq, oLp, oRng, oBoot, oReg, oX, oPar, oSc, lds;
    // agent_num > 1 (joint-action trees, general layout only): agents, N*A, and the LDS regions of
    // the nodes' joint actions [P][N] (bytes), the staged policy / beta / noise [N][A], the
    // per-agent CDFs [N][A] (double) and the draws [K][N]
    int N, NA, JP;  // JP: bytes of joint actions per tree (P*N rounded up to 16)
    int oJ, oJpol, oJbet, oJcp, oJdraw;
};

#ifdef __HIP_DEVICE_COMPILE__
typedef __attribute__((address_space(1))) char gchar;
#else
typedef char gchar;
#endif

struct Dev {
    // Every array lives in one device allocation (the handle's arena): a base pointer plus
    // 32-bit offsets in 256-byte units keeps the kernel arguments small (each pointer would take
    // two SGPRs for the whole kernel).
    // On the device the arena pointer is typed as global memory, so every access through it is a
    // global_* op: a flat_* op also counts against lgkmcnt, and every LDS wait after it would wait
    // for the HBM access too (outstanding write-backs included).
    gchar *base;
    unsigned o_Par, o_J, o_A, o_Bn, o_Q, o_PP, o_C, o_D, o_V, o_R, o_hdr, o_path, o_stats, o_err, o_T, o_pb, o_sq, o_lp, o_seed;
    __host__ __device__ int *Par() const { return (int *)(base + (size_t)o_Par * 256); }  // [P] parent index
    __host__ __device__ unsigned char *J() const { return (unsigned char *)(base + (size_t)o_J * 256); }  // [P][N] joint actions (agent_num > 1)
    __host__ __device__ int4 *A() const { return (int4 *)(base + (size_t)o_A * 256); }  // [P] {visit, prior, value, reward}
    __host__ __device__ int4 *Bn() const { return (int4 *)(base + (size_t)o_Bn * 256); }  // [P] {first_child, nc|act<<8|(maxdepth+1)<<16, pred_value, hsx}
    __host__ __device__ float *Q() const { return (float *)(base + (size_t)o_Q * 256); }  // [P] q - parent.pred_value
    __host__ __device__ float *PP() const { return (float *)(base + (size_t)o_PP * 256); }  // [P] parent pred_value
    __host__ __device__ float4 *C() const { return (float4 *)(base + (size_t)o_C * 256); }  // [P] {weighted_sum, tot_weight, -, -}
    __host__ __device__ float4 *D() const { return (float4 *)(base + (size_t)o_D * 256); }  // [P] {pred_prob, beta, beta_hat, -}
    __host__ __device__ int2 *V() const { return (int2 *)(base + (size_t)o_V * 256); }  // [P][E] {depth, value}
    __host__ __device__ unsigned *R() const { return (unsigned *)(base + (size_t)o_R * 256); }  // [W] mt19937 stream
    __host__ __device__ TreeHdr *hdr() const { return (TreeHdr *)(base + (size_t)o_hdr * 256); }  // [B] tree header
    __host__ __device__ int2 *path() const { return (int2 *)(base + (size_t)o_path * 256); }  // [B][PS] {node, visit-at-selection}
    __host__ __device__ long long *stats() const { return (long long *)(base + (size_t)o_stats * 256); }  // [B][MZ_S_COUNT]
    __host__ __device__ int *err() const { return (int *)(base + (size_t)o_err * 256); }  // [1]
    __host__ __device__ float *T() const { return (float *)(base + (size_t)o_T * 256); }  // [TT] pUCT coefficient table, index n*(n+1)/2 + v
    __host__ __device__ float *pb() const { return (float *)(base + (size_t)o_pb * 256); }  // [PS] logf((n + c2 + 1)/c2) + c1
    __host__ __device__ double *sq() const { return (double *)(base + (size_t)o_sq * 256); }  // [PS] sqrt(n)
    __host__ __device__ float *lp() const { return (float *)(base + (size_t)o_lp * 256); }  // [PS+1] lambda^d as a float chain
    __host__ __device__ unsigned *seed() const { return (unsigned *)(base + (size_t)o_seed * 256); }  // [1] random_seed, read by k_prepare
};

struct StepArgs {
    int hsx;
    float discount;
    int K;
    int ne, pe;  // host bounds on the node count and path length (skip waiting for the header)
    const float *reward, *value, *policy, *beta;  // expansion inputs
    int *idx_x, *idy, *act;
    const char *pool;
    long long pool_stride, row_bytes;
    char *gather_out;
};

struct PrepArgs {
    const float *reward, *value, *policy, *beta, *noise;
    float eps;
    int K;
    int *idx_x, *idy, *act;  // non-null: also the first selection (mz_prepare_select)
};

// Per-handle constants, written once to device memory at mz_create: kernels take a pointer to
// them, so the kernel-argument block is only that pointer plus the launch's own arguments (~120 B).
// Large by-value kernel arguments are expensive in HIP graphs, whose kernel nodes keep a copy of
// every launch's argument block.
struct Params {
    Geo g;
    Dev d;
    // std::mt19937 seeding checkpoints (seed_table): row v holds x_{16j}(v), j < 39, for v < cp_n;
    // null: k_prepare runs the seeding chain
    const unsigned *cp;
    unsigned cp_n;
};

// Arena offsets of every array a k_step launch reads in its first round, as a function of the
// geometry alone (B, P, PS): mz_create's ArenaPlan requests the arrays in exactly this order and
// checks the result against this function, so the kernel computes these addresses from its
// preloaded SGPR arguments and its first loads do not wait for the Params block.
__host__ __device__ __forceinline__ unsigned long long arena_span(unsigned long long bytes) {
    return (bytes + 64 + 255) / 256;  // ArenaPlan::span, in 256-byte units
}
// arena_span(c * n + k) in 32-bit arithmetic (c a power of two dividing 256): the kernels compute
// these offsets in their prologue, where 64-bit scalar pairs cost SGPRs (and spills) on every wave
template <unsigned c>
__host__ __device__ __forceinline__ unsigned span_n(unsigned n, unsigned k = 0) {
    return n / (256 / c) + (c * (n % (256 / c)) + k + 64 + 255) / 256;
}
// (mz_create: B < 2^24, B * P < 2^32 and B * PS < 2^32, so every product below fits 32 bits)
// The node arrays come first: their offsets then follow from B * P alone (k_chain3 computes them
// with a dozen scalar instructions before its first load).
__host__ __device__ __forceinline__ void arena_nodes(Dev &d, unsigned B, unsigned P) {
    const unsigned nodes = B * P;
    const unsigned s16 = span_n<16>(nodes), s4 = span_n<4>(nodes);
    d.o_A = (unsigned)arena_span(sizeof(Params));
    d.o_Par = d.o_A + s16;
    d.o_Bn = d.o_Par + s4;
    d.o_Q = d.o_Bn + s16;
    d.o_PP = d.o_Q + s4;
    d.o_C = d.o_PP + s4;
    d.o_hdr = d.o_C + s16;
}
// pUCT coefficient table entries, T[n (n + 1) / 2 + v] = pb_c(n, v) for n < PS, padded to 4.  Only
// k_step's LDS-staged table (4 TT <= kTableLdsMax: PS <= 155) and k_tree's prior scores (value
// entries E <= kBkCap: PS <= 342) read past T[0]; every other kernel computes pb_c from the
// per-n pb / sq tables with the same double arithmetic.  Past kTableFullPS the table is T[0] alone,
// O(S) instead of O(S^2) on host and device (S = 65,000 would need 8.5 GB).
constexpr unsigned kTableFullPS = 512;
__host__ __device__ __forceinline__ unsigned table_entries(unsigned PS) {
    return PS <= kTableFullPS ? ((PS * (PS + 1) / 2) + 3) & ~3u : 4u;
}
__host__ __device__ __forceinline__ void arena_hot(Dev &d, unsigned B, unsigned P, unsigned PS) {
    const unsigned TT = table_entries(PS);
    arena_nodes(d, B, P);
    unsigned o = d.o_hdr;
    o += (B * (unsigned)sizeof(TreeHdr) + 64 + 255) / 256;
    d.o_stats = o; o += span_n<8>(B * MZ_S_COUNT);
    d.o_err = o; o += span_n<4>(1);
    d.o_seed = o; o += span_n<4>(1);
    d.o_lp = o; o += span_n<4>(PS + 1 + kWave);
    d.o_T = o; o += span_n<4>(TT + 4 * kWave);
    d.o_pb = o; o += span_n<4>(PS + kWave);
    d.o_sq = o; o += span_n<8>(PS + kWave);
    d.o_path = o; o += span_n<8>(B * PS);
    d.o_V = o;  // [P][E] value entries, E = S + 1 = PS - 1
}

#ifdef MZ_ARGCHECK
// Diagnostic build (graph-replay investigation): records of inconsistent launches in a device
// buffer, read back with mz_debug_dump (device printf does not reach the host from graph replays).
constexpr int kDbgRecs = 64, kDbgWords = 32;
__device__ unsigned g_dbg[kDbgRecs][kDbgWords];
__device__ int g_dbg_n;
__device__ unsigned g_dbg_sites;
__device__ __noinline__ void argcheck_record(unsigned kind, bool EB, bool SEL, int t, char *base, int P, int PS,
                                             int BA, int pk, int K, int hsx, float discount, int pe, int ne,
                                             TreeHdr *hv, int tot, int cur, int D, int herr, const unsigned *ka,
                                             const float *reward, const float *value, const char *pool, int err) {
    const int gK = (int)((unsigned)pk >> 17), B = BA & 0xffffff;
    const int tot2 = __hip_atomic_load(&hv->tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int cur2 = __hip_atomic_load(&hv->cursor, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int D2 = __hip_atomic_load(&hv->D, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    Params *pv = (Params *)base;
    const int pP = __hip_atomic_load(&pv->g.P, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int pPS = __hip_atomic_load(&pv->g.PS, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int pB = __hip_atomic_load(&pv->g.B, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int pK = __hip_atomic_load(&pv->g.K, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long kbase = (unsigned long long)ka[0] | ((unsigned long long)ka[1] << 32);
    unsigned bad = 0;
    if (tot2 != tot || cur2 != cur || D2 != D) bad |= 1;                        // scalar cache vs L2
    if (EB && gK == 1 && !herr && tot != hsx + 1) bad |= 2;                     // K = 1 chain invariant
    if (pP != P || pPS != PS || pB != B || pK != gK) bad |= 4;                   // args vs Params
    if (kbase != (unsigned long long)base || (int)ka[2] != P || (int)ka[3] != PS || (int)ka[4] != BA ||
        (int)ka[5] != pk)
        bad |= 8;                                                                // preloaded vs memory
    if (EB && gK == 1 && pe != (hsx + 1 < PS ? hsx + 1 : PS)) bad |= 16;         // host path bound
    if (kind == 1 && !bad) return;
    const int r = atomicAdd(&g_dbg_n, 1);
    if (r >= kDbgRecs) return;
    unsigned *o = g_dbg[r];
    const unsigned long long kp = (unsigned long long)ka;
    const unsigned w[kDbgWords] = {kind, bad, (unsigned)EB | ((unsigned)SEL << 1), (unsigned)t, (unsigned)tot,
                                   (unsigned)cur, (unsigned)D, (unsigned)herr, (unsigned)tot2, (unsigned)cur2,
                                   (unsigned)D2, (unsigned)P, (unsigned)PS, (unsigned)BA, (unsigned)pk, (unsigned)K,
                                   (unsigned)hsx, __float_as_uint(discount), (unsigned)pe, (unsigned)ne,
                                   (unsigned)pP, (unsigned)pPS, (unsigned)pB, (unsigned)pK,
                                   (unsigned)kp, (unsigned)(kp >> 32), (unsigned)kbase, (unsigned)(kbase >> 32),
                                   (unsigned)(unsigned long long)base, (unsigned)((unsigned long long)base >> 32),
                                   (unsigned)err, (unsigned)(unsigned long long)reward};
    for (int k = 0; k < kDbgWords; ++k) o[k] = w[k];
    (void)value;
    (void)pool;
}
#define MZ_SITE(n) atomicOr(&g_dbg_sites, 1u << (n))
#else
#define MZ_SITE(n) ((void)0)
#endif

#ifdef __HIP_DEVICE_COMPILE__
typedef const __attribute__((address_space(4))) Params cParams;
typedef const __attribute__((address_space(4))) TreeHdr cTreeHdr;
#else
typedef const Params cParams;
typedef const TreeHdr cTreeHdr;
#endif
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }
__device__ __forceinline__ unsigned long long ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ float i2f(int x) { return __int_as_float(x); }
__device__ __forceinline__ int f2i(float x) { return __float_as_int(x); }
// Cross-lane reads.  Values read from LDS are divergent for the compiler even when every lane read
// the same address; uni() states the uniformity (v_readfirstlane), so wave-uniform state lives in
// SGPRs and uniform control flow compiles to scalar branches instead of exec-mask juggling.
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ float unif(float v) { return i2f(uni(f2i(v))); }
__device__ __forceinline__ int4 uni4(int4 v) { return make_int4(uni(v.x), uni(v.y), uni(v.z), uni(v.w)); }
__device__ __forceinline__ int rl(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
// lane l of v := x (l, x uniform)
__device__ __forceinline__ int wl(int v, int x, int l) { return (lane_id() == l) ? x : v; }
__device__ __forceinline__ float rlf(float v, int l) { return i2f(__builtin_amdgcn_readlane(f2i(v), l)); }
__device__ __forceinline__ double rld(double v, int l) {
    const long long b = __double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b & 0xffffffffll), l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)((unsigned long long)b >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Node-record field packing: Bn.y = nc | action<<8 | (maxdepth+1)<<16
__device__ __forceinline__ int nc_of(int y) { return y & 0xff; }
__device__ __forceinline__ int act_of(int y) { return (y >> 8) & 0xff; }
__device__ __forceinline__ int md_of(int y) { return (int)((unsigned)y >> 16) - 1; }
__device__ __forceinline__ int pack_y(int nc, int act, int md) { return nc | (act << 8) | ((md + 1) << 16); }

// --------------------------------------------------------------------------------------------
// Readbacks (cnode.cpp:672-781, cytree.pyx:93-247): root value, marginal visit counts / priors,
// root degree and every per-child field of the root, field-major (4-byte words):
//   [B] root value | [B*A] marginal visits | [B*A] marginal priors | [B] degree |
//   MZ_F_COUNT x [B*Wd] per-child fields padded with zeros to Wd = max degree
// Destinations: the handle's packed buffer (readback_dev) or the caller's device buffers
// (mz_get_roots_device); a null field is not written.  Per-child fields are [B][Wd(*N)] either way.
// --------------------------------------------------------------------------------------------
struct RbPtrs {
    float *values;  // [B]
    int *mv;        // [B][N*A] marginal visit counts
    float *mp;      // [B][N*A] marginal priors
    int *deg;       // [B] root degrees
    int *f[MZ_F_COUNT];
};
// A fused readback's destinations and constants, in device memory (mz_expand_backup_readback): the
// search's last expansion kernel reads it (SEL = false launches pass it in their gather_out slot)
struct RbDesc {
    RbPtrs o;
    float disc;  // the discount of the q values (cnode.cpp:165)
    int Wd;      // per-child field width
    int pad[2];
};

// Tree t's readback from its final records, one lane per root child (lane l < nc: child fc + l):
// ra = the root's {visit, prior, value, reward}; ca / cb / cd = the child's {visit, prior, value,
// reward} / {first_child, nc|act|md, pred_value, hsx} / {pred_prob, beta, beta_hat}.  jt: the
// children's joint actions [nc][N] (N > 1), else unused.
__device__ __forceinline__ void readback_emit(const RbPtrs &o, float disc, int Wd, int t, int A, int N, int nc, int4 ra,
                                              int4 ca, int4 cb, float4 cd, const unsigned char *jt) {
    const int l = threadIdx.x & 63;
    const int NA = N * A;
    if (l == 0) {
        if (o.values) o.values[t] = (nc > 0) ? i2f(ra.z) : 0.f;
        if (o.deg) o.deg[t] = nc;
    }
    const bool has = l < nc;
    const int act = act_of(cb.y);
    // marginal visit counts / priors (cnode.cpp:69-91): cell (agent j, action a) collects, in child
    // order, every child whose action for agent j is a
    if (o.mv || o.mp)
        for (int cell = l; cell < NA; cell += 64) {
            const int j = cell / A, av = cell - j * A;
            int mv = 0;
            float mp = 0.f;
            for (int c = 0; c < nc; ++c) {
                const int aj = (N == 1) ? rl(act, c) : (int)jt[c * N + j];
                const int vj = rl(ca.x, c);
                const float pj = rlf(i2f(ca.y), c);
                if (aj == av) {
                    mv += vj;
                    mp += pj;
                }
            }
            if (o.mv) o.mv[(size_t)t * NA + cell] = mv;
            if (o.mp) o.mp[(size_t)t * NA + cell] = mp;
        }
    if (l < Wd) {
        const size_t r = (size_t)t * Wd + l;
        const float val = i2f(ca.z);  // CNode::value(): 0 when not expanded (stored that way)
        const float rew = i2f(ca.w);
        if (int *fa = o.f[MZ_F_ACTIONS]) {
            if (N == 1)
                fa[r] = has ? act : 0;
            else
                for (int i = 0; i < N; ++i) fa[r * N + i] = has ? (int)jt[l * N + i] : 0;
        }
        if (o.f[MZ_F_VISIT_COUNT]) o.f[MZ_F_VISIT_COUNT][r] = has ? ca.x : 0;
        const float fv[MZ_F_COUNT] = {0.f, 0.f, cd.x, cd.y, cd.z, i2f(ca.y), cd.z / cd.y * cd.x, i2f(cb.z), val, rew,
                                      rew + disc * val};
#pragma unroll
        for (int f = MZ_F_PRED_PROBS; f < MZ_F_COUNT; ++f)
            if (o.f[f]) ((float *)o.f[f])[r] = has ? fv[f] : 0.f;
    }
}

// Wait for this wave's memory traffic (LDS-DMA included via vmcnt) / LDS traffic; compiler fence.
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void wait_lds() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// A store with the system-coherence bits (sc0 sc1): written through to memory rather than left
// dirty in L2, so the dependent-kernel boundary has less to write back.  Only for data this
// kernel does not read again (the asm is invisible to the compiler's wait counting).
__device__ __forceinline__ void st_wt16(void *p, int4 v) {
    typedef int i4v __attribute__((ext_vector_type(4)));
    const i4v x = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(x) : "memory");
}

// Workgroup barrier for data exchanged through LDS only: unlike __syncthreads() it does not wait for
// the wave's outstanding global stores (vmcnt), which take ~1,000 cycles to drain.  LDS-DMA data
// a wave hands over must be waited for (wait_vm) before it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n s_barrier" ::: "memory"); }

// LDS-DMA: lane l copies `bytes` (4 or 16) from its own src into lds_base + l*bytes (lds_base
// must be wave-uniform).
__device__ __forceinline__ void glds4(const void *src, void *lds_base) {
    __builtin_amdgcn_global_load_lds((glb_void *)src, (lds_void *)lds_base, 4, 0, 0);
}
__device__ __forceinline__ void glds16(const void *src, void *lds_base) {
    __builtin_amdgcn_global_load_lds((glb_void *)src, (lds_void *)lds_base, 16, 0, 0);
}

// The same LDS-DMA issued through inline assembly: the compiler's wait-count pass does not track it,
// so it inserts no conservative vmcnt(0) before later LDS accesses (with the builtin, any LDS access
// after a DMA on ANY control-flow path -- another wave's role branch included -- waits for every
// outstanding vector memory operation, this wave's global stores too).  The caller waits (wait_vm)
// before it reads the staged data.
__device__ __forceinline__ void glds4a(const void *src, void *lds_base) {
    const unsigned lds = (unsigned)(uintptr_t)(lds_void *)lds_base;
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(src), "s"(lds) : "memory", "m0");
}
__device__ __forceinline__ void glds16a(const void *src, void *lds_base) {
    const unsigned lds = (unsigned)(uintptr_t)(lds_void *)lds_base;
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds) : "memory", "m0");
}

// Phase stamp (diagnostic builds): the shader clock when the wave's instruction stream gets here
// (no forced wait: loads in flight stay in flight).
__device__ __forceinline__ void stamp(unsigned long long *ts, int i) {
    if constexpr (MZ_STAMPS != 0) ts[i] = __builtin_amdgcn_s_memtime();
}

// Launch spans (diagnostic builds, MZ_SPANS=1 or MZ_STAMPS=1): each fused launch's workgroups record
// their first wave's start and end on the chip-wide 100 MHz clock (s_memrealtime) with one plain
// 16-byte store per workgroup (no atomics: contended atomics would lengthen the very launch they
// time), per simulation slot (hsx) and tree.  The host takes min(start) / max(end) per launch:
// against the HIP-event period of back-to-back launches that splits a launch into its body and
// the boundary between two kernels (bench.py reads it through mz_debug_spans).
#ifndef MZ_SPANS
#define MZ_SPANS MZ_STAMPS
#endif
#if MZ_SPANS
constexpr int kSpanSlots = 256, kSpanTrees = 1024;
__device__ ulonglong2 g_span[kSpanSlots][kSpanTrees][2];  // {wave 0 start, wave 0 end}, {wave 1 end, wave 2 end}
#endif
__device__ __forceinline__ unsigned long long span_open() {
#if MZ_SPANS
    return __builtin_amdgcn_s_memrealtime();
#else
    return 0;
#endif
}
__device__ __forceinline__ void span_close(int slot, unsigned long long t0) {
#if MZ_SPANS
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    const int t = blockIdx.x;
    if (lane_id() == 0 && slot >= 0 && slot < kSpanSlots && t < kSpanTrees) g_span[slot][t][0] = make_ulonglong2(t0, t1);
#else
    (void)slot;
    (void)t0;
#endif
}
// k_tree: a tree's shape in this launch and three of wave 0's phase ends (10 ns units after its
// start, 16 bits each), beside wave 0's span (bit 63 marks both words as no time)
__device__ __forceinline__ unsigned long long span_mark() {
#if MZ_SPANS
    return __builtin_amdgcn_s_memrealtime();
#else
    return 0;
#endif
}
__device__ __forceinline__ void span_info(int slot, unsigned long long info, unsigned long long t0,
                                          unsigned long long m1, unsigned long long m2, unsigned long long m3) {
#if MZ_SPANS
    const int t = blockIdx.x;
    const unsigned long long ph = ((m1 - t0) & 0xffff) | (((m2 - t0) & 0xffff) << 16) | (((m3 - t0) & 0xffff) << 32);
    if (lane_id() == 0 && slot >= 0 && slot < kSpanSlots && t < kSpanTrees)
        g_span[slot][t][1] = make_ulonglong2((1ull << 63) | info, (1ull << 63) | ph);
#else
    (void)slot;
    (void)info;
    (void)t0;
    (void)m1;
    (void)m2;
    (void)m3;
#endif
}
// the end of another wave role (1 or 2) of the same launch
__device__ __forceinline__ void span_end(int slot, int role) {
#if MZ_SPANS
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    const int t = blockIdx.x;
    if (lane_id() == 0 && slot >= 0 && slot < kSpanSlots && t < kSpanTrees) {
        unsigned long long *e = (unsigned long long *)&g_span[slot][t][1];
        e[role - 1] = t1;
    }
#else
    (void)slot;
    (void)role;
#endif
}

// Whole-wave reductions with DPP (no LDS round trips): xor-pairs, xor-quads, half-row and row
// mirrors reduce each 16-lane row; the four row results are combined from SGPRs.  All lanes must
// be active.
template <int CTRL>
__device__ __forceinline__ int dpp(int v) {
    return __builtin_amdgcn_update_dpp(v, v, CTRL, 0xf, 0xf, false);
}
__device__ __forceinline__ float wave_min(float v) {
    v = fminf(v, i2f(dpp<0xB1>(f2i(v))));   // quad_perm [1,0,3,2]
    v = fminf(v, i2f(dpp<0x4E>(f2i(v))));   // quad_perm [2,3,0,1]
    v = fminf(v, i2f(dpp<0x141>(f2i(v))));  // row_half_mirror
    v = fminf(v, i2f(dpp<0x140>(f2i(v))));  // row_mirror
    return fminf(fminf(rlf(v, 0), rlf(v, 16)), fminf(rlf(v, 32), rlf(v, 48)));
}
__device__ __forceinline__ float wave_max(float v) {
    v = fmaxf(v, i2f(dpp<0xB1>(f2i(v))));
    v = fmaxf(v, i2f(dpp<0x4E>(f2i(v))));
    v = fmaxf(v, i2f(dpp<0x141>(f2i(v))));
    v = fmaxf(v, i2f(dpp<0x140>(f2i(v))));
    return fmaxf(fmaxf(rlf(v, 0), rlf(v, 16)), fmaxf(rlf(v, 32), rlf(v, 48)));
}
// Full-wave min / max whose result is exact in lane 63 only: the row reduction of wave_min, then
// row_bcast:15 / row_bcast:31 fold rows 0-1 and 2-3 into lane 63 (no v_readlane).
__device__ __forceinline__ float wave_min_to63(float v) {
    v = fminf(v, i2f(dpp<0xB1>(f2i(v))));
    v = fminf(v, i2f(dpp<0x4E>(f2i(v))));
    v = fminf(v, i2f(dpp<0x141>(f2i(v))));
    v = fminf(v, i2f(dpp<0x140>(f2i(v))));
    v = fminf(v, i2f(__builtin_amdgcn_update_dpp(f2i(v), f2i(v), 0x142, 0xa, 0xf, false)));  // row_bcast:15
    v = fminf(v, i2f(__builtin_amdgcn_update_dpp(f2i(v), f2i(v), 0x143, 0xc, 0xf, false)));  // row_bcast:31
    return v;
}
__device__ __forceinline__ float wave_max_to63(float v) {
    v = fmaxf(v, i2f(dpp<0xB1>(f2i(v))));
    v = fmaxf(v, i2f(dpp<0x4E>(f2i(v))));
    v = fmaxf(v, i2f(dpp<0x141>(f2i(v))));
    v = fmaxf(v, i2f(dpp<0x140>(f2i(v))));
    v = fmaxf(v, i2f(__builtin_amdgcn_update_dpp(f2i(v), f2i(v), 0x142, 0xa, 0xf, false)));
    v = fmaxf(v, i2f(__builtin_amdgcn_update_dpp(f2i(v), f2i(v), 0x143, 0xc, 0xf, false)));
    return v;
}
__device__ __forceinline__ int wave_sum(int v) {
    v += dpp<0xB1>(v);
    v += dpp<0x4E>(v);
    v += dpp<0x141>(v);
    v += dpp<0x140>(v);
    return rl(v, 0) + rl(v, 16) + rl(v, 32) + rl(v, 48);
}

// Inclusive prefix sum over the wave: row scans by DPP shifts, then the row totals by row
// broadcasts (all lanes active).
__device__ __forceinline__ int wave_incl_scan(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15 (rows 1, 3)
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31 (rows 2, 3)
    return v;
}

__device__ __forceinline__ bool tame_val(float x) { return x >= -1e30f && x <= 1e30f; }  // false for NaN
__device__ __forceinline__ bool tame_prior(float x) { return x >= 0.f && x <= 1e30f; }

// size_lim of SubTreeValueSet::update (utils.cpp:31): max(1, (int)ceil(count * (1 - rho)))
__device__ __forceinline__ int value_lim(int c, float one_minus_rho) {
    const int v = (int)ceilf((float)c * one_minus_rho);
    return v < 1 ? 1 : v;
}

// --------------------------------------------------------------------------------------------
// One tree's view of LDS
// --------------------------------------------------------------------------------------------
struct Lds {
    int4 *A, *B;
    float *Q, *PP, *Vs;
    int *Par;   // parent index per node (general walks)
    float *Sc;  // pUCT score of every node under its parent, computed before the walk
    float4 *C;
    int2 *path;
    int *flag;
    float *T, *pb;
    double *sq;
    float *lp;
    unsigned *rng;
    float *boot;
    int2 *reg;
    int *il;  // internal-node list of the precomputed walk (layout classes)
};

// LDS layout of k_step.  Capacity classes NC = 64 .. 1024 (node pool P <= NC) have a
// compile-time layout: every LDS address folds into an instruction's immediate offset and no
// offset occupies an SGPR for the kernel's lifetime.  NC = 0 is the general layout, whose offsets
// come from Geo (trees above 1024 nodes).  The compile-time classes compute pUCT coefficients from
// the pb / sq tables (no staged pUCT table).
constexpr int kRegCap = 2048;  // value entries staged per back-propagation chunk (static layouts)

template <int NC>
struct Layout {
    static constexpr int r16(int x) { return (x + 15) & ~15; }
    static constexpr int oA = 0;
    static constexpr int oB = oA + r16(16 * NC);
    static constexpr int oQ = oB + r16(16 * NC);
    static constexpr int oPP = oQ + r16(4 * NC);
    static constexpr int oVs = oPP + r16(4 * NC);
    static constexpr int oC = oVs + r16(4 * NC);
    static constexpr int oPath = oC + r16(16 * NC);
    static constexpr int oFlag = oPath + r16(8 * NC);
    static constexpr int oPb = oFlag + r16(4 * NC);
    static constexpr int oSq = oPb + r16(4 * (NC + kWave));
    static constexpr int oLp = oSq + r16(8 * (NC + kWave));
    static constexpr int oRng = oLp + r16(4 * (NC + 1 + kWave));
    static constexpr int oBoot = oRng + r16(4 * kRngWin);
    static constexpr int oReg = oBoot + r16(4 * (NC + kWave));
    static constexpr int oX = oReg + r16(8 * kRegCap);
    static constexpr int oPar = oX + r16(8 * (2 * MZ_S_COUNT + 4));
    static constexpr int oSc = oPar + r16(4 * NC);
    static constexpr int oIl = oSc + r16(4 * NC);
    static constexpr int total = oIl + r16(4 * NC);
};

template <int NC>
__device__ __forceinline__ Lds make_lds(unsigned char *m, const Geo &g) {
    Lds s;
    if constexpr (NC > 0) {
        using L = Layout<NC>;
        s.A = (int4 *)(m + L::oA);
        s.B = (int4 *)(m + L::oB);
        s.Q = (float *)(m + L::oQ);
        s.PP = (float *)(m + L::oPP);
        s.Vs = (float *)(m + L::oVs);
        s.C = (float4 *)(m + L::oC);
        s.path = (int2 *)(m + L::oPath);
        s.flag = (int *)(m + L::oFlag);
        s.T = nullptr;
        s.pb = (float *)(m + L::oPb);
        s.sq = (double *)(m + L::oSq);
        s.lp = (float *)(m + L::oLp);
        s.rng = (unsigned *)(m + L::oRng);
        s.boot = (float *)(m + L::oBoot);
        s.reg = (int2 *)(m + L::oReg);
        s.Par = (int *)(m + L::oPar);
        s.Sc = (float *)(m + L::oSc);
        s.il = (int *)(m + L::oIl);
    } else {
        s.A = (int4 *)(m + g.oA);
        s.B = (int4 *)(m + g.oB);
        s.Q = (float *)(m + g.oQ);
        s.PP = (float *)(m + g.oPP);
        s.Vs = (float *)(m + g.oVs);
        s.C = (float4 *)(m + g.oC);
        s.path = (int2 *)(m + g.oPath);
        s.flag = (int *)(m + g.oFlag);
        s.T = (float *)(m + g.oT);
        s.pb = (float *)(m + g.oPb);
        s.sq = (double *)(m + g.oSq);
        s.lp = (float *)(m + g.oLp);
        s.rng = (unsigned *)(m + g.oRng);
        s.boot = (float *)(m + g.oBoot);
        s.reg = (int2 *)(m + g.oReg);
        s.Par = (int *)(m + g.oPar);
        s.Sc = (float *)(m + g.oSc);
        s.il = nullptr;
    }
    return s;
}

template <int NC>
__device__ __forceinline__ long long *lds_xchg(unsigned char *m, const Geo &g) {
    if constexpr (NC > 0) return (long long *)(m + Layout<NC>::oX);
    return (long long *)(m + g.oX);
}

// RNG word `idx` (per lane) of tree t: LDS window [wbase, wbase+kRngWin) or HBM.
__device__ __forceinline__ unsigned rng_word_lane(const Geo &g, const Dev &d, const unsigned *win, int wbase, int t,
                                                  int idx, int &err) {
    const int o = idx - wbase;
    if (win && o >= 0 && o < kRngWin) return win[o];
    if (idx >= g.W) {
        err |= kErrRng;
        return 0u;
    }
    return d.R()[(size_t)t * g.W + idx];
}

// RNG word `idx` (per lane) from the LDS window only (0 outside it: select_word checks the range)
__device__ __forceinline__ unsigned rng_word_win(const unsigned *win, int wbase, int idx) {
    const int o = idx - wbase;
    return (o >= 0 && o < kRngWin) ? win[o] : 0u;
}

// std::discrete_distribution<int>::param_type::_M_initialize (libstdc++ random.tcc:2656-2690) for
// the distribution whose weight for action `lane` is `bd` (0 for lanes >= A): sequential double
// sum, p = w / sum, sequential prefix sums, the last forced to 1.0.  Returns this lane's cumulative
// probability.  Serial chains in blocks of 8 fully unrolled steps (readlane is convergent, so the
// compiler cannot unroll a runtime-count loop over it by itself).
// v = (bit l of m) ? x : v for this lane l, with m built by the scalar unit (one v_cndmask per
// dword, no VALU compare)
__device__ __forceinline__ float sel_lane(float v, float x, unsigned long long m) {
    asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(v) : "v"(x), "s"(m));
    return v;
}
__device__ __forceinline__ double sel_lane(double v, double x, unsigned long long m) {
    const long long vb = __double_as_longlong(v), xb = __double_as_longlong(x);
    const float lo = sel_lane(__int_as_float((int)(unsigned)(vb & 0xffffffffll)),
                              __int_as_float((int)(unsigned)(xb & 0xffffffffll)), m);
    const float hi = sel_lane(__int_as_float((int)(vb >> 32)), __int_as_float((int)(xb >> 32)), m);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)__float_as_int(hi) << 32) |
                                            (unsigned)__float_as_int(lo)));
}

__device__ __forceinline__ long long sel_lane(long long v, long long x, unsigned long long m) {
    return __double_as_longlong(sel_lane(__longlong_as_double(v), __longlong_as_double(x), m));
}

__device__ __forceinline__ double cdf_lane(double bd, int A) {
    const int l = lane_id();
    // Both chains read their operands into SGPRs 8 at a time ahead of the dependent adds (a
    // v_readlane result consumed right away by a VALU stalls the chain); lane a keeps its prefix
    // sum through v_cndmask on a SALU-built lane mask.
    double sum = 0.0;
    int a0 = 0;
    for (; a0 + 8 <= A; a0 += 8) {
        double w8[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) w8[j] = rld(bd, a0 + j);
        asm volatile("" : "+s"(w8[0]), "+s"(w8[1]), "+s"(w8[2]), "+s"(w8[3]), "+s"(w8[4]), "+s"(w8[5]),
                     "+s"(w8[6]), "+s"(w8[7]));
#pragma unroll
        for (int j = 0; j < 8; ++j) sum += w8[j];
    }
    for (; a0 < A; ++a0) sum += rld(bd, a0);
    const double p = bd / sum;
    double acc = rld(p, 0), cp = (l == 0) ? acc : 0.0;
    a0 = 1;
    for (; a0 + 8 <= A; a0 += 8) {
        double p8[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) p8[j] = rld(p, a0 + j);
        asm volatile("" : "+s"(p8[0]), "+s"(p8[1]), "+s"(p8[2]), "+s"(p8[3]), "+s"(p8[4]), "+s"(p8[5]),
                     "+s"(p8[6]), "+s"(p8[7]));
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            acc = acc + p8[j];
            cp = sel_lane(cp, acc, 1ull << (a0 + j));
        }
    }
    for (; a0 < A; ++a0) {
        acc = acc + rld(p, a0);
        cp = (l == a0) ? acc : cp;
    }
    if (l == A - 1) cp = 1.0;
    return cp;
}

// std::discrete_distribution's cumulative table (libstdc++ random.tcc:2656-2690, as cdf_lane) for
// the weights staged in sw[0 .. 64) (sw[l] = 0 for l >= A; lane l's own weight is wl): the
// sequential double sum and the sequential prefix sums run on every lane from broadcast LDS reads
// instead of v_readlane.  N terms (A <= N): trailing +0.0 terms are exact no-ops on the
// non-negative sums, so N only has to cover A -- the class (4, 8, 12, 16) is picked once per call,
// not per term.  Lane a returns cp[a] (cp[A-1] forced to 1.0).
template <int N>
__device__ __forceinline__ double cdf_terms(int A, const float *sw, double *sp, float wl) {
    const int l = lane_id();
    float w[N];
#pragma unroll
    for (int q = 0; q < N / 4; ++q) {
        const float4 v = *(const float4 *)(sw + 4 * q);
        w[4 * q] = v.x;
        w[4 * q + 1] = v.y;
        w[4 * q + 2] = v.z;
        w[4 * q + 3] = v.w;
    }
    double sum = 0.0;
#pragma unroll
    for (int j = 0; j < N; ++j) sum += (double)w[j];
    const double p = (l < A) ? (double)wl / sum : 0.0;
    sp[l] = p;
    wait_lds();
    double pj[N];
#pragma unroll
    for (int q = 0; q < N / 2; ++q) {
        const double2 v = *(const double2 *)(sp + 2 * q);
        pj[2 * q] = v.x;
        pj[2 * q + 1] = v.y;
    }
    double acc = pj[0], cp = (l == 0) ? pj[0] : 0.0;
#pragma unroll
    for (int j = 1; j < N; ++j) {
        acc = acc + pj[j];
        cp = sel_lane(cp, acc, 1ull << j);
    }
    if (l == A - 1) cp = 1.0;
    return cp;
}
// A > 16: batches of 16 terms, then the rest in steps of 4 up to A rounded up to 4 (27m: 36 terms,
// not three batches of 16); each batch's LDS reads issued together ahead of its adds
__device__ __forceinline__ double cdf_long(int A, const float *sw, double *sp, float wl) {
    const int l = lane_id();
    const int A4 = (A + 3) & ~3;
    double sum = 0.0;
    int a0 = 0;
    for (; a0 + 16 <= A4; a0 += 16) {
        float w[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float4 v = *(const float4 *)(sw + a0 + 4 * q);
            w[4 * q] = v.x;
            w[4 * q + 1] = v.y;
            w[4 * q + 2] = v.z;
            w[4 * q + 3] = v.w;
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) sum += (double)w[j];
    }
    // 0, 4, 8 or 12 terms left; the three reads are issued together, so with fewer left they run
    // past sw / sp into the caller's next LDS region (read, never used)
    const int rest = A4 - a0;
    if (rest > 0) {
        const float4 v0 = *(const float4 *)(sw + a0), v1 = *(const float4 *)(sw + a0 + 4),
                     v2 = *(const float4 *)(sw + a0 + 8);
        sum += (double)v0.x;
        sum += (double)v0.y;
        sum += (double)v0.z;
        sum += (double)v0.w;
        if (rest > 4) {
            sum += (double)v1.x;
            sum += (double)v1.y;
            sum += (double)v1.z;
            sum += (double)v1.w;
        }
        if (rest > 8) {
            sum += (double)v2.x;
            sum += (double)v2.y;
            sum += (double)v2.z;
            sum += (double)v2.w;
        }
    }
    const double p = (l < A) ? (double)wl / sum : 0.0;
    sp[l] = p;
    wait_lds();
    double acc = 0.0, cp = 0.0;
    a0 = 0;
    for (; a0 + 16 <= A4; a0 += 16) {
        double pj[16];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const double2 v = *(const double2 *)(sp + a0 + 2 * q);
            pj[2 * q] = v.x;
            pj[2 * q + 1] = v.y;
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            acc = (a0 + j == 0) ? pj[0] : acc + pj[j];
            cp = sel_lane(cp, acc, 1ull << (j & 63) << (a0 & 63));
        }
    }
    if (rest > 0) {
        double pj[12];
#pragma unroll
        for (int q = 0; q < 6; ++q) {
            const double2 v = *(const double2 *)(sp + a0 + 2 * q);
            pj[2 * q] = v.x;
            pj[2 * q + 1] = v.y;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            acc = acc + pj[j];
            cp = sel_lane(cp, acc, 1ull << (a0 + j));
        }
        if (rest > 4) {
#pragma unroll
            for (int j = 4; j < 8; ++j) {
                acc = acc + pj[j];
                cp = sel_lane(cp, acc, 1ull << (a0 + j));
            }
        }
        if (rest > 8) {
#pragma unroll
            for (int j = 8; j < 12; ++j) {
                acc = acc + pj[j];
                cp = sel_lane(cp, acc, 1ull << (a0 + j));
            }
        }
    }
    if (l == A - 1) cp = 1.0;
    return cp;
}
// cdf for weights already staged in sw[0..A) (sw[l] = 0 for l >= A)
__device__ __forceinline__ double cdf_staged(int A, const float *sw, double *sp) {
    const float wl = sw[lane_id()];
    if (A <= 4) return cdf_terms<4>(A, sw, sp, wl);
    if (A <= 8) return cdf_terms<8>(A, sw, sp, wl);
    if (A <= 12) return cdf_terms<12>(A, sw, sp, wl);
    if (A <= 16) return cdf_terms<16>(A, sw, sp, wl);
    return cdf_long(A, sw, sp, wl);
}
// the same for the weights bet held one per lane (lane a < A); `during` runs while the weights'
// LDS store is in flight (independent per-lane work of the caller)
struct NoWork {
    __device__ void operator()() const {}
};
template <class F = NoWork>
__device__ __forceinline__ double cdf_bcast(float bet, int A, float *sw, double *sp, F &&during = F()) {
    const int l = lane_id();
    sw[l] = (l < A) ? bet : 0.f;  // kMaxActions = kWave entries
    during();
    wait_lds();
    if (A <= 4) return cdf_terms<4>(A, sw, sp, bet);
    if (A <= 8) return cdf_terms<8>(A, sw, sp, bet);
    if (A <= 12) return cdf_terms<12>(A, sw, sp, bet);
    if (A <= 16) return cdf_terms<16>(A, sw, sp, bet);
    return cdf_long(A, sw, sp, bet);
}

// --------------------------------------------------------------------------------------------
// CTree::expand (cnode.cpp:224-295) for one node, agent_num = 1.  Lane a < A holds the node's
// policy / beta / noise entry for action a.  Children are created for the distinct sampled actions
// in ascending order (std::map<long> key order, cnode.cpp:243,268).  Sampling restates
// std::discrete_distribution<int> + generate_canonical<double,53> (libstdc++ random.tcc:
// 2656-2713, 3348-3378): double prefix sums of beta/sum(beta), last forced to 1.0; two engine words
// per draw; index = lower_bound.  Fewer than two actions => no draw and no engine word.
// Creates the children in HBM (and in the LDS mirrors when given), advances cursor / tot and
// returns nc.  `pv` is the expanded node's pred_value (the children's PP).
// --------------------------------------------------------------------------------------------
__device__ __forceinline__ int expand_node(const Geo &g, const Dev &d, int t, int parent, float pol, float bet, float noi, float eps,
                           int K, float pv, int &cursor, int &tot, const unsigned *win, int wbase, Lds *s, int &err,
                           long long &st_new, bool have_w, unsigned w1r, unsigned w2r, long long *stl, int &wild,
                           int *first_act = nullptr, float *cdf_w = nullptr, double *cdf_p = nullptr) {
    const int l = lane_id();
    const int A = g.A;
    int cnt = 0;  // number of draws that hit action l
    unsigned long long e0 = 0, e1 = 0, e2 = 0;
    if (MZ_STAMPS && stl) e0 = __builtin_amdgcn_s_memtime();
    if (A < 2) {
        cnt = (l == 0) ? K : 0;
    } else {
        // (with LDS scratch of 64 floats + 64 doubles: the same chains from LDS broadcasts, cdf_bcast)
        const double cp = cdf_w ? cdf_bcast((l < A) ? bet : 0.f, A, cdf_w, cdf_p) : cdf_lane((l < A) ? (double)bet : 0.0, A);
        if (MZ_STAMPS && stl) {
            asm volatile("" ::"v"(cp));
            e1 = __builtin_amdgcn_s_memtime();
        }
        // K draws, 64 at a time: lane k of a chunk forms the canonical double of draw k0+k; then,
        // draw by draw, lane a compares its cp[a] with u and lower_bound = popcount of the ballot
        for (int k0 = 0; k0 < K; k0 += kWave) {
            const int nk = (K - k0) < kWave ? (K - k0) : kWave;
            double u = 0.0;
            if (l < nk) {
                const int w = cursor + 2 * (k0 + l);
                const bool reg = have_w && k0 == 0;
                const double w1 = (double)(reg ? w1r : rng_word_lane(g, d, win, wbase, t, w, err));
                const double w2 = (double)(reg ? w2r : rng_word_lane(g, d, win, wbase, t, w + 1, err));
                u = (w1 + w2 * 4294967296.0) / 18446744073709551616.0;
                if (u >= 1.0) u = 0x1.fffffffffffffp-1;  // nextafter(1, 0)
            }
            if (cdf_w) {
                // with LDS scratch: lane k takes draw k0 + k and counts the actions whose cp is below its
                // u from the broadcast CDF (lanes >= A hold +inf: never below), the same count as the
                // ballot's popcount; the draws' counts per action by LDS atomics
                int *hits = (int *)cdf_w;
                if (k0 == 0) {
                    cdf_p[l] = (l < A) ? cp : INFINITY;
                    hits[l] = 0;
                    wait_lds();
                }
                if (l < nk) {
                    int ix = 0;
                    const int A4 = (A + 3) & ~3;
                    for (int a0 = 0; a0 < A4; a0 += 4) {
                        const double2 c01 = *(const double2 *)(cdf_p + a0), c23 = *(const double2 *)(cdf_p + a0 + 2);
                        ix += (c01.x < u ? 1 : 0) + (c01.y < u ? 1 : 0) + (c23.x < u ? 1 : 0) + (c23.y < u ? 1 : 0);
                    }
                    atomicAdd(&hits[ix], 1);
                }
                if (k0 + kWave >= K) {
                    wait_lds();
                    cnt = (l < A) ? hits[l] : 0;
                }
                continue;
            }
            int k = 0;
            for (; k + 4 <= nk; k += 4) {  // (four draws per step, as k_tree)
                const double u0 = rld(u, k), u1 = rld(u, k + 1), u2 = rld(u, k + 2), u3 = rld(u, k + 3);
                const int i0 = __popcll(ballot(l < A && cp < u0)), i1 = __popcll(ballot(l < A && cp < u1));
                const int i2 = __popcll(ballot(l < A && cp < u2)), i3 = __popcll(ballot(l < A && cp < u3));
                cnt += ((i0 == l) ? 1 : 0) + ((i1 == l) ? 1 : 0) + ((i2 == l) ? 1 : 0) + ((i3 == l) ? 1 : 0);
            }
            for (; k < nk; ++k) {
                const double uk = rld(u, k);
                const int idx = __popcll(ballot(l < A && cp < uk));
                cnt += (l == idx) ? 1 : 0;
            }
        }
        cursor += 2 * K;
    }
    if (MZ_STAMPS && stl) {
        asm volatile("" ::"v"(cnt));
        e2 = __builtin_amdgcn_s_memtime();
        if (e1 == 0) e1 = e0;
    }
    // the loads still in flight (the RNG window, the leaf's record, a prefetched row) land before
    // this expansion's stores are issued, so later waits need not drain the stores
    wait_vm();
    const bool has = (l < A) && cnt > 0;
    const unsigned long long m = ballot(has);
    const int nc = __popcll(m);
    if (first_act) *first_act = m ? (int)__builtin_ctzll(m) : 0;  // the first child's action (ascending order)
    if (tot + nc > g.P) {
        err |= kErrPool;
        return 0;
    }
    if (has) {
        const int rank = __popcll(m & ((1ull << l) - 1ull));
        const int c = tot + rank;
        const float bh = (float)cnt / (float)K;  // betahat_prob = count / sampled_times
        float prior = (eps > 0) ? (pol * (1 - eps) + noi * eps) : pol;
        prior = prior * bh / bet;  // prior * betahat_prob / beta_prob
        if (!tame_prior(prior)) wild = 1;
        const int4 a4 = make_int4(0, f2i(prior), f2i(0.0f), f2i(0.0f));
        const int4 b4 = make_int4(0, pack_y(0, l, -1), f2i(0.0f), -1);
        const size_t gi = (size_t)t * g.P + c;
        d.A()[gi] = a4;
        d.Bn()[gi] = b4;
        d.C()[gi] = make_float4(0.f, 0.f, 0.f, 0.f);
        d.D()[gi] = make_float4(pol, bet, bh, 0.f);
        d.Q()[gi] = 0.f;
        d.PP()[gi] = pv;
        d.Par()[gi] = parent;
        if (s) {
            s->A[c] = a4;
            s->B[c] = b4;
            s->Q[c] = 0.f;
            s->PP[c] = pv;
            s->Par[c] = parent;
        }
    }
    wild = (ballot(wild != 0) != 0ull) ? 1 : 0;
    st_new += nc;
    tot += nc;  // the children occupy [old tot, old tot + nc)
    if (MZ_STAMPS && stl) {
        wait_lds();
        const unsigned long long e3 = __builtin_amdgcn_s_memtime();
        stl[MZ_S_CYC_EXP_CDF] += (long long)(e1 - e0);
        stl[MZ_S_CYC_EXP_DRAW] += (long long)(e2 - e1);
        stl[MZ_S_CYC_EXP_NODES] += (long long)(e3 - e2);
    }
    return nc;
}

// --------------------------------------------------------------------------------------------
// CTree::expand (cnode.cpp:224-295), agent_num = 1, for action spaces past one lane per action
// (64 < A <= kWideActions; k_prepare and k_hbm): lane l holds actions l + 64 j, j < 4.  The same
// std::discrete_distribution restatement as expand_node -- the sequential double sum, p = w / sum,
// the sequential prefix sums with the last forced to 1.0, two engine words per draw, lower_bound --
// with the serial chains walking the chunks in action order.  pol / bet / noi: the node's A inputs
// in global memory (noi may be null when eps == 0).
// --------------------------------------------------------------------------------------------
constexpr int kWideActions = 255;  // (Bn.y packs the action and the children count in 8 bits each)
__device__ int expand_wide(const Geo &g, const Dev &d, int t, int parent, const float *pol_g, const float *bet_g,
                           const float *noi_g, float eps, int K, float pv, int &cursor, int &tot, int &err,
                           long long &st_new, int &wild, int *first_act = nullptr) {
    const int l = lane_id();
    const int A = g.A;
    float pol[4], bet[4], noi[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int a = 64 * j + l;
        pol[j] = (a < A) ? pol_g[a] : 0.f;
        bet[j] = (a < A) ? bet_g[a] : 0.f;
        noi[j] = (a < A && noi_g && eps > 0) ? noi_g[a] : 0.f;
    }
    int cnt[4] = {0, 0, 0, 0};  // draws that hit action 64 j + l
    if (A < 2) {
        cnt[0] = (l == 0) ? K : 0;
    } else {
        double sum = 0.0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const double w = (double)bet[j];
            for (int a = 0; a < kWave && 64 * j + a < A; ++a) sum += rld(w, a);
        }
        double cp[4];
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const double p = (64 * j + l < A) ? (double)bet[j] / sum : 0.0;
            double c = 0.0;
            for (int a = 0; a < kWave && 64 * j + a < A; ++a) {
                const double pa = rld(p, a);
                acc = (j == 0 && a == 0) ? pa : acc + pa;
                c = (l == a) ? acc : c;
            }
            if (64 * j + l == A - 1) c = 1.0;
            cp[j] = c;
        }
        for (int k0 = 0; k0 < K; k0 += kWave) {
            const int nk = (K - k0) < kWave ? (K - k0) : kWave;
            double u = 0.0;
            if (l < nk) {
                const int w = cursor + 2 * (k0 + l);
                const double w1 = (double)rng_word_lane(g, d, nullptr, 0, t, w, err);
                const double w2 = (double)rng_word_lane(g, d, nullptr, 0, t, w + 1, err);
                u = (w1 + w2 * 4294967296.0) / 18446744073709551616.0;
                if (u >= 1.0) u = 0x1.fffffffffffffp-1;  // nextafter(1, 0)
            }
            for (int k = 0; k < nk; ++k) {
                const double uk = rld(u, k);
                int idx = 0;
#pragma unroll
                for (int j = 0; j < 4; ++j) idx += __popcll(ballot(64 * j + l < A && cp[j] < uk));
#pragma unroll
                for (int j = 0; j < 4; ++j) cnt[j] += (idx == 64 * j + l) ? 1 : 0;
            }
        }
        cursor += 2 * K;
    }
    wait_vm();
    unsigned long long m[4];
    int below[4], nc = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        m[j] = ballot(64 * j + l < A && cnt[j] > 0);
        below[j] = nc;
        nc += __popcll(m[j]);
    }
    if (first_act) {
        int f = 0;
#pragma unroll
        for (int j = 3; j >= 0; --j)
            if (m[j]) f = 64 * j + (int)__builtin_ctzll(m[j]);
        *first_act = f;
    }
    if (tot + nc > g.P) {
        err |= kErrPool;
        return 0;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (cnt[j] > 0 && 64 * j + l < A) {
            const int c = tot + below[j] + __popcll(m[j] & ((1ull << l) - 1ull));
            const float bh = (float)cnt[j] / (float)K;  // betahat_prob = count / sampled_times
            float prior = (eps > 0) ? (pol[j] * (1 - eps) + noi[j] * eps) : pol[j];
            prior = prior * bh / bet[j];  // prior * betahat_prob / beta_prob
            if (!tame_prior(prior)) wild = 1;
            const size_t gi = (size_t)t * g.P + c;
            d.A()[gi] = make_int4(0, f2i(prior), f2i(0.0f), f2i(0.0f));
            d.Bn()[gi] = make_int4(0, pack_y(0, 64 * j + l, -1), f2i(0.0f), -1);
            d.C()[gi] = make_float4(0.f, 0.f, 0.f, 0.f);
            d.D()[gi] = make_float4(pol[j], bet[j], bh, 0.f);
            d.Q()[gi] = 0.f;
            d.PP()[gi] = pv;
            d.Par()[gi] = parent;
        }
    }
    wild = (ballot(wild != 0) != 0ull) ? 1 : 0;
    st_new += nc;
    tot += nc;
    return nc;
}

// --------------------------------------------------------------------------------------------
// CTree::expand (cnode.cpp:224-295) with agent_num = N > 1, K <= 64 (lane k = draw k).  One
// discrete distribution per agent; draw k takes agent 0..N-1 in turn, two engine words per agent
// draw (none when A < 2); key = key * 23333 + a_i in 64-bit two's complement (the reference's
// `long`, which wraps past N = 4); children = the distinct keys in ascending signed order
// (std::map<long>), beta_hat = count / K, products over agents in agent order.  pol / bet / noi are
// the node's [N][A] inputs in LDS; cp [N][A] and draw [K][N] are LDS scratch.
// --------------------------------------------------------------------------------------------
__device__ __forceinline__ long long rl64(long long v, int j) {
    const int lo = __builtin_amdgcn_readlane((int)(unsigned)(v & 0xffffffffll), j);
    const int hi = __builtin_amdgcn_readlane((int)(v >> 32), j);
    return (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

__device__ int expand_joint(const Geo &g, const Dev &d, int t, int parent, const float *pol, const float *bet,
                            const float *noi,
                            float eps, int K, float pv, int &cursor, int &tot, const unsigned *win, int wbase,
                            Lds *s, unsigned char *sJ, double *cp, int *draw, int &err, long long &st_new) {
    const int l = lane_id();
    const int N = g.N, A = g.A;
    if (A >= 2) {
        for (int i = 0; i < N; ++i) {
            const double c = cdf_lane((l < A) ? (double)bet[i * A + l] : 0.0, A);
            if (l < A) cp[i * A + l] = c;
        }
        wait_lds();
    }
    unsigned long long key = 0;
    if (l < K) {
        for (int i = 0; i < N; ++i) {
            int act = 0;
            if (A >= 2) {
                const int w = cursor + 2 * (l * N + i);
                const double w1 = (double)rng_word_lane(g, d, win, wbase, t, w, err);
                const double w2 = (double)rng_word_lane(g, d, win, wbase, t, w + 1, err);
                double u = (w1 + w2 * 4294967296.0) / 18446744073709551616.0;
                if (u >= 1.0) u = 0x1.fffffffffffffp-1;  // nextafter(1, 0)
                for (int a = 0; a < A; ++a) act += (cp[i * A + a] < u) ? 1 : 0;  // lower_bound
            }
            draw[l * N + i] = act;
            key = key * 23333ull + (unsigned long long)act;
        }
    }
    if (A >= 2) cursor += 2 * K * N;
    wait_lds();
    // distinct keys: first occurrence, multiplicity, rank among the distinct keys (signed order)
    const long long sk = (long long)key;
    bool first = l < K;
    int count = 0;
    for (int j = 0; j < K; ++j) {
        const long long kj = rl64(sk, j);
        if (l < K && kj == sk) {
            ++count;
            if (j < l) first = false;
        }
    }
    const unsigned long long fm = ballot(first);
    int rank = 0;
    for (unsigned long long m = fm; m; m &= m - 1ull) {
        const long long kj = rl64(sk, __builtin_ctzll(m));
        rank += (kj < sk) ? 1 : 0;
    }
    const int nc = __popcll(fm);
    if (tot + nc > g.P) {
        err |= kErrPool;
        return 0;
    }
    if (first) {
        const int c = tot + rank;
        const float bh = (float)count / (float)K;  // betahat_prob = count / sampled_times
        float beta_prob = 1.0f, pred_prob = 1.0f, prior = 1.0f;
        for (int i = 0; i < N; ++i) {
            const int act = draw[l * N + i];
            const float pa = pol[i * A + act];
            beta_prob *= bet[i * A + act];
            pred_prob *= pa;
            if (eps > 0) {
                const float p = pa * (1 - eps) + noi[i * A + act] * eps;
                prior *= p;
            } else {
                prior *= pa;
            }
        }
        prior = prior * bh / beta_prob;
        const int4 a4 = make_int4(0, f2i(prior), f2i(0.0f), f2i(0.0f));
        const int4 b4 = make_int4(0, pack_y(0, draw[l * N], -1), f2i(0.0f), -1);
        const size_t gi = (size_t)t * g.P + c;
        d.A()[gi] = a4;
        d.Bn()[gi] = b4;
        d.C()[gi] = make_float4(0.f, 0.f, 0.f, 0.f);
        d.D()[gi] = make_float4(pred_prob, beta_prob, bh, 0.f);
        d.Q()[gi] = 0.f;
        d.PP()[gi] = pv;
        d.Par()[gi] = parent;
        for (int i = 0; i < N; ++i) {
            d.J()[(size_t)t * g.JP + (size_t)c * N + i] = (unsigned char)draw[l * N + i];
            if (sJ) sJ[c * N + i] = (unsigned char)draw[l * N + i];
        }
        if (s) {
            s->A[c] = a4;
            s->B[c] = b4;
            s->Q[c] = 0.f;
            s->PP[c] = pv;
            s->Par[c] = parent;
        }
    }
    st_new += nc;
    tot += nc;
    return nc;
}

// --------------------------------------------------------------------------------------------
// Prepare (CTree_batch::prepare, cnode.cpp:589-614 -> CTree::prepare, cnode.cpp:205-222):
// generate the tree's mt19937 stream (seed random_seed*2333 + i, cnode.cpp:574) with all four
// waves, then expand the root with wave 0.
// --------------------------------------------------------------------------------------------
__device__ __forceinline__ unsigned mt_twist(unsigned cur, unsigned nxt) {
    const unsigned y = (cur & 0x80000000u) | (nxt & 0x7fffffffu);
    return (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}
__device__ __forceinline__ unsigned mt_temper(unsigned z) {
    z ^= (z >> 11);
    z ^= (z << 7) & 0x9d2c5680u;
    z ^= (z << 15) & 0xefc60000u;
    z ^= (z >> 18);
    return z;
}

// std::mt19937::seed(v) is the chain x_0 = v, x_i = 1812433253 (x_{i-1} ^ (x_{i-1} >> 30)) + i,
// 623 dependent steps (~5 us per tree on the scalar unit, most of k_prepare).  Its state is the
// previous word alone, so the words x_{16j} split it into 39 independent 16-step pieces: the
// per-device table (seed_table) holds them for every v below its size, and k_prepare's lanes
// replay the pieces in parallel.  Row v: x_{16j}(v) for j < 39 (word 39 unused, 160-byte rows).
constexpr int kSeedStep = 16, kSeedRow = 40;
static_assert(kMtN % kSeedStep == 0 && kMtN / kSeedStep < kSeedRow, "seeding checkpoints");

// One block builds 256 consecutive rows in LDS (thread k: row v0 + k) and writes them out as one
// contiguous 40 KB span with 16-byte stores (a thread storing its own 160-byte row directly made
// every store instruction touch 64 rows: ~6x the table in HBM writes, round 4's PMC).
__global__ __launch_bounds__(256) void k_seed_table(unsigned *cp, unsigned n) {
    __shared__ __attribute__((aligned(16))) unsigned rows[256 * kSeedRow];
    const unsigned v0 = blockIdx.x * 256u;
    const unsigned v = v0 + threadIdx.x;
    unsigned *row = rows + threadIdx.x * kSeedRow;
    unsigned x = v;
    row[0] = x;
    for (int i = 1; i < kMtN; ++i) {
        x = 1812433253u * (x ^ (x >> 30)) + (unsigned)i;
        if (i % kSeedStep == 0) row[i / kSeedStep] = x;
    }
    row[kSeedRow - 1] = 0u;
    __syncthreads();
    const unsigned nrows = (n - v0) < 256u ? (n - v0) : 256u;
    const int4 *src = (const int4 *)rows;
    int4 *dst = (int4 *)(cp + (size_t)v0 * kSeedRow);  // (160-byte rows: 16-byte aligned)
    for (unsigned i = threadIdx.x; i < nrows * (kSeedRow / 4); i += 256u) dst[i] = src[i];
}

__global__ __launch_bounds__(256) void k_prepare(const Params *__restrict__ prm, PrepArgs a) {
    const Geo g = prm->g;
    const Dev d = prm->d;
    __shared__ unsigned mt[kMtN];
    __shared__ unsigned mt2[kMtN];
    __shared__ unsigned w0[kMtN];
    const int t = blockIdx.x;
    const int tid = threadIdx.x;
    // the handle's error word starts clean (no runtime memset node in captured graphs).  A tree's
    // error also stays in its header, and every later kernel re-reports the errors of dead trees,
    // so an error raised by another block before this store is not lost.
    if (t == 0 && tid == 0) *d.err() = 0;
    const unsigned seed_v = d.seed()[0] * 2333u + (unsigned)(g.root_offset + t);
    const unsigned *cp = prm->cp;
    if (cp && seed_v < prm->cp_n) {
        // the seeding chain from the checkpoints: lane j replays words 16j .. 16j + 15
        if (tid < kMtN / kSeedStep) {
            const int i0 = kSeedStep * tid;
            unsigned x = cp[(size_t)seed_v * kSeedRow + tid];
            mt[i0] = x;
#pragma unroll
            for (int i = 1; i < kSeedStep; ++i) {
                x = 1812433253u * (x ^ (x >> 30)) + (unsigned)(i0 + i);
                mt[i0 + i] = x;
            }
        }
    } else
#if defined(MZ_ABL_NOSEED)  // ablation (timing experiments only): no seeding chain
    if (tid < kWave) {
        const unsigned x = d.seed()[0] * 2333u + (unsigned)(g.root_offset + t);
        for (int i = tid; i < kMtN; i += kWave) mt[i] = x + (unsigned)i;
    }
#elif !defined(MZ_SEED_LOOP)
    if (tid < kWave) {
        // std::mt19937::seed (sequential by definition) on the scalar unit: 4 SALU operations per
        // word, word i into lane i % 64 of VGPR i / 64 (mt_seed.inc, scripts/gen_mt_seed.py), then
        // ten LDS stores.  Replaces a compiler loop of ~6.5 instructions per word (10.4 us -> ...)
        unsigned x = (unsigned)__builtin_amdgcn_readfirstlane((int)(d.seed()[0] * 2333u + (unsigned)(g.root_offset + t)));
        unsigned tt;
        int v0 = (int)x, v1 = 0, v2 = 0, v3 = 0, v4 = 0, v5 = 0, v6 = 0, v7 = 0, v8 = 0, v9 = 0;
        asm volatile(MZ_MT_SEED_ASM
                     : [x] "+s"(x), [t] "=&s"(tt), [v0] "+v"(v0), [v1] "+v"(v1), [v2] "+v"(v2), [v3] "+v"(v3),
                       [v4] "+v"(v4), [v5] "+v"(v5), [v6] "+v"(v6), [v7] "+v"(v7), [v8] "+v"(v8), [v9] "+v"(v9)
                     :
                     : "scc");
        const int l = tid;
        mt[l] = (unsigned)v0;
        mt[64 + l] = (unsigned)v1;
        mt[128 + l] = (unsigned)v2;
        mt[192 + l] = (unsigned)v3;
        mt[256 + l] = (unsigned)v4;
        mt[320 + l] = (unsigned)v5;
        mt[384 + l] = (unsigned)v6;
        mt[448 + l] = (unsigned)v7;
        mt[512 + l] = (unsigned)v8;
        if (576 + l < kMtN) mt[576 + l] = (unsigned)v9;
    }
#else
    if (tid == 0) {  // std::mt19937::seed: sequential by definition
        unsigned x = d.seed()[0] * 2333u + (unsigned)(g.root_offset + t);
        mt[0] = x;
        for (int i = 1; i < kMtN; ++i) {
            x = 1812433253u * (x ^ (x >> 30)) + (unsigned)i;
            mt[i] = x;
        }
    }
#endif
    // (the twist exchanges LDS data only: barriers that leave the tempered words' global stores in
    // flight instead of draining them at every phase)
    lds_barrier();
    int nb = g.W / kMtN;
#ifdef MZ_ABL_NOTWIST  // ablation (timing experiments only): no twist / tempering
    nb = 0;
#endif
    // One twist per 624-word block (std::mt19937::_M_gen_rand), one barrier each: thread k < 227
    // computes the three words k, k + 227, k + 454 of the new state in registers.  Word k uses old
    // words only; word k + 227 uses new word k (its x[k + 227 - 227]); word k + 454 uses new word
    // k + 227; the last word (623, thread 169) also uses new word 0, which it recomputes.  The old
    // state is read from one LDS buffer and the new one written to the other.
    unsigned *cur = mt, *nxt = mt2;
    for (int blk = 0; blk < nb; ++blk) {
        unsigned *dst = d.R() + (size_t)t * g.W + (size_t)blk * kMtN;
        if (tid < 227) {
            const int k = tid;
            const unsigned n0 = cur[k + 397] ^ mt_twist(cur[k], cur[k + 1]);
            const unsigned n1 = n0 ^ mt_twist(cur[k + 227], cur[k + 228]);
            nxt[k] = n0;
            nxt[k + 227] = n1;
            const unsigned z0 = mt_temper(n0), z1 = mt_temper(n1);
            dst[k] = z0;
            dst[k + 227] = z1;
            if (blk == 0) {
                w0[k] = z0;
                w0[k + 227] = z1;
            }
            if (k < kMtN - 454) {
                const unsigned nx = (k + 455 < kMtN) ? cur[k + 455] : (cur[397] ^ mt_twist(cur[0], cur[1]));
                const unsigned n2 = n1 ^ mt_twist(cur[k + 454], nx);
                nxt[k + 454] = n2;
                const unsigned z2 = mt_temper(n2);
                dst[k + 454] = z2;
                if (blk == 0) w0[k + 454] = z2;
            }
        }
        lds_barrier();
        unsigned *tmp = cur;
        cur = nxt;
        nxt = tmp;
    }
    // a root expansion that reads engine words past the LDS window (more than kRngWin / 2 engine-word
    // pairs, or the wide expansion, which reads them all from HBM) reads what every wave just stored:
    // a full workgroup barrier (stores drained) first
    if (g.A > kMaxActions || 2 * a.K * g.N > kRngWin) __syncthreads();
    if (tid >= kWave) return;

    // ---- root expansion by wave 0 ----
    const int l = tid;
    const int A = g.A;
    const float r = a.reward[t];
    const float v = a.value[t];
    int err = 0;
    int cursor = 0, tot = 1;
    long long st_new = 0;
    int nc;
    int first_act = 0;
    int wild = (g.N > 1) ? 1 : 0;  // joint-action trees always take the exact selection
    if (g.N > 1) {  // joint actions: the root's [N][A] inputs staged in (dynamic) LDS
        extern __shared__ __attribute__((aligned(16))) unsigned char jsm[];
        const int NA = g.NA;
        float *jp = (float *)jsm, *jb = jp + NA, *jn = jb + NA;
        double *jcp = (double *)(jsm + ((12 * NA + 15) & ~15));
        int *jd = (int *)(jcp + NA);
        const size_t ib = (size_t)t * NA;
        for (int i = l; i < NA; i += kWave) {
            jp[i] = a.policy[ib + i];
            jb[i] = a.beta[ib + i];
            jn[i] = a.noise[ib + i];
        }
        wait_lds();
        nc = expand_joint(g, d, t, 0, jp, jb, jn, a.eps, a.K, v, cursor, tot, w0, 0, nullptr, nullptr, jcp, jd, err,
                          st_new);
    } else if (A > kMaxActions) {  // more actions than lanes (the root's inputs read from HBM)
        const size_t ib = (size_t)t * A;
        nc = expand_wide(g, d, t, 0, a.policy + ib, a.beta + ib, a.noise ? a.noise + ib : nullptr, a.eps, a.K, v,
                         cursor, tot, err, st_new, wild, &first_act);
    } else {
        const size_t ib = (size_t)t * A;
        const float pol = (l < A) ? a.policy[ib + l] : 0.f;
        const float bet = (l < A) ? a.beta[ib + l] : 0.f;
        const float noi = (l < A) ? a.noise[ib + l] : 0.f;
        nc = expand_node(g, d, t, 0, pol, bet, noi, a.eps, a.K, v, cursor, tot, w0, 0, nullptr, err, st_new, false, 0u,
                         0u, nullptr, wild, &first_act);
    }
    if (l == 0) {
        // root: CNode(1,1,1,1,true) (cnode.cpp:217), expanded, visit += 1, subtree.update(value, 0)
        const size_t gi = (size_t)t * g.P;
        // first SubTreeValueSet::update: count 1, big and small empty -> insert into big
        float ws = 0.f, tw = 0.f;
        const float lp0 = d.lp()[0];
        if (value_lim(1, g.one_minus_rho) != 1) err |= kErrValueSet;
        tw += lp0;
        ws += lp0 * v;
        const float val = (nc > 0) ? ws / tw : 0.f;
        d.A()[gi] = make_int4(1, f2i(1.0f), f2i(val), f2i(r));
        d.Bn()[gi] = make_int4(1, pack_y(nc, 0, 0), f2i(v), 0);
        d.C()[gi] = make_float4(ws, tw, 0.f, 0.f);
        d.D()[gi] = make_float4(1.f, 1.f, 1.f, 0.f);
        d.Q()[gi] = 0.f;
        d.PP()[gi] = 0.f;
        d.V()[gi * g.E] = make_int2(0, f2i(v));
        // mz_prepare_select: the first selection (select_path, cnode.cpp:381-413) right after
        // prepare: the root has one visit and nc >= 1 children, so the forced round-robin takes
        // child 0 (cnode.cpp:398-399) without scoring and without an engine word
        const bool sel = a.idx_x != nullptr;
        int D = 0, leaf = 0, sact = 0;
        if (sel && !err) {
            if (nc > 0) {
                D = 1;
                leaf = 1;  // the root's first child
                sact = first_act;
            } else {
                err |= kErrRoot;
            }
        }
        TreeHdr h;
        h.cursor = cursor;
        h.tot = tot;
        h.D = D;
        h.err = err;
        h.mm_min = 0.f;
        h.mm_max = 0.f;
        h.mm_cnt = 0;
        h.leaf = leaf;
        h.tame = (!wild && tame_val(v) && tame_val(r)) ? 1 : 0;
        for (int j = 0; j < kNxt; ++j) h.nxt[j] = (cursor + j < kMtN) ? w0[cursor + j] : 0u;
        d.hdr()[t] = h;
        d.path()[(size_t)t * g.PS] = make_int2(0, 1);
        if (D == 1) d.path()[(size_t)t * g.PS + 1] = make_int2(1, 0);
        long long *st = d.stats() + (size_t)t * MZ_S_COUNT;
        st[MZ_S_EXPANDS] += 1;
        st[MZ_S_NEW_CHILDREN] += st_new;
        if (sel) {
            a.idx_x[t] = 0;  // the root's hidden_state_index_x
            a.idy[t] = t;
            a.act[t] = err ? 0 : sact;
            if (!err) {
                st[MZ_S_SELECTS] += 1;
                st[MZ_S_PATH_EDGES] += 1;
            }
        }
        if (err) atomicOr(d.err(), err);
    }
}

// Bootstrap recurrence b = r + disc * b (cnode.cpp:448) over `n` levels, lane-parallel: level
// i sits at lane 63 - (top - i), lane 63 holds the chunk's starting value (outside EXEC for the
// whole loop), and each step every lane takes its upper neighbour's b through DPP wave_shl:1
// fused into the multiply (tmp = b[l+1] * disc), then adds its own reward: after n steps lanes
// 63-n .. 62 hold exactly the sequential recurrence's values.  The lane below the carry has tmp
// preset to disc * carry, so it is right whether DPP reads an inactive source lane or leaves
// the destination untouched.  Measured ~30 cycles per level, against ~46 for a wave-uniform
// chain fed by v_readlane (each v_readlane costs ~30 cycles on gfx950).
__device__ __forceinline__ void boot_dpp(float &b, float &tmp, float dv, float rn, int n) {
    unsigned long long saved;
    int n4 = n >> 2, n1 = n & 3;
#define MZ_BOOT_STEP                                                                   \
    "s_nop 1\n"                                                                        \
    "v_mul_f32_dpp %[t], %[b], %[d] wave_shl:1 row_mask:0xf bank_mask:0xf\n"           \
    "v_add_f32 %[b], %[r], %[t]\n"
    asm volatile(
        "s_mov_b64 %[sv], exec\n"
        "s_bitset0_b64 exec, 63\n"
        "s_cmp_eq_u32 %[n4], 0\n"
        "s_cbranch_scc1 2f\n"
        "1:\n" MZ_BOOT_STEP MZ_BOOT_STEP MZ_BOOT_STEP MZ_BOOT_STEP
        "s_sub_u32 %[n4], %[n4], 1\n"
        "s_cmp_lg_u32 %[n4], 0\n"
        "s_cbranch_scc1 1b\n"
        "2:\n"
        "s_cmp_eq_u32 %[n1], 0\n"
        "s_cbranch_scc1 4f\n"
        "3:\n" MZ_BOOT_STEP
        "s_sub_u32 %[n1], %[n1], 1\n"
        "s_cmp_lg_u32 %[n1], 0\n"
        "s_cbranch_scc1 3b\n"
        "4:\n"
        "s_mov_b64 exec, %[sv]\n"
        : [b] "+v"(b), [t] "+v"(tmp), [sv] "=&s"(saved), [n4] "+s"(n4), [n1] "+s"(n1)
        : [d] "v"(dv), [r] "v"(rn)
        : "memory", "scc");
#undef MZ_BOOT_STEP
}

// --------------------------------------------------------------------------------------------
// Back-propagation staging: the value entries of the path nodes [i0, i0+cnt) that need them ->
// LDS with LDS-DMA.  A node needs its entries only when the new value's depth is not beyond its
// deepest entry (otherwise the update is an append with an empty depth class: always so in K=1
// chains).  Chunks hold <= 64 nodes whose needed entries fit g.reg_cap.  Returns cnt (uniform);
// lane l gets its node id, entry count (= visit at selection), need flag and staging offset.
// --------------------------------------------------------------------------------------------
template <bool kAsmDma = false>
__device__ __forceinline__ int stage_regions(const Geo &g, const Dev &d, Lds &s, int t, int D, int i0, int &n, int &nv, int &need,
                             int &off, unsigned long long *sp = nullptr) {
    const int l = lane_id();
    const int i = i0 + l;
    n = 0;
    nv = 0;
    need = 0;
    off = 0;
    if (i <= D) {
        if (g.K == 1) {
            // K = 1 trees are chains: the path is node i at level i, its entry count the visit
            // count staged this launch, and every update appends with an empty depth class
            n = i;
            nv = s.A[i].x;
        } else {
            const int2 pe = s.path[i];
            n = pe.x;
            nv = pe.y;
            need = (nv > 0 && md_of(s.B[n].y) >= D - i) ? 1 : 0;
        }
    }
    if (MZ_STAMPS && sp) {
        asm volatile("" ::"v"(need));
        sp[0] = __builtin_amdgcn_s_memtime();
    }
    const int lim = (D + 1 - i0) < kWave ? (D + 1 - i0) : kWave;
    // prefix sum of the needed entry counts over the chunk: a uniform loop over the needing lanes
    // only (none in K=1 chains); the chunk ends before the first node that would overflow reg_cap
    int acc = 0, cnt = lim;
    for (unsigned long long m = ballot(l < lim && need); m; m &= m - 1ull) {
        const int j = __builtin_ctzll(m);
        const int vj = rl(nv, j);
        if (acc + vj > g.reg_cap) {
            cnt = j;
            break;
        }
        if (l == j) off = acc;
        acc += vj;
    }
    if (MZ_STAMPS && sp) {
        asm volatile("" ::"v"(off));
        sp[1] = __builtin_amdgcn_s_memtime();
    }
    const int2 *gV = d.V() + (size_t)t * g.P * g.E;
    int *regdw = (int *)s.reg;
    const unsigned long long nm = ballot(l < cnt && need);
    for (unsigned long long m = nm; m; m &= m - 1ull) {
        const int j = __builtin_ctzll(m);
        const int nj = rl(n, j), vj = rl(nv, j), oj = rl(off, j);
        const int dw = 2 * vj;
        const int *src = (const int *)(gV + (size_t)nj * g.E);
        for (int c = 0; c < dw; c += kWave)
            if (c + l < dw) {
                if constexpr (kAsmDma) glds4a(src + c + l, regdw + 2 * oj + c);
                else glds4(src + c + l, regdw + 2 * oj + c);
            }
    }
    return cnt;
}

// --------------------------------------------------------------------------------------------
// CTree::back_propagate (cnode.cpp:415-450) over the path held in LDS.  Lane i owns path node i.
// Bootstrap values are a sequential f32 recurrence b_{i-1} = reward_i + discount * b_i, computed
// once by the whole wave.  Each node's SubTreeValueSet::update (utils.cpp:20-71) reads min(big)
// / max(small) as order statistics of its sorted entries at that depth and replays the
// reference's f32 op sequence.  Afterwards the min/max normaliser (CMinMaxStats, utils.cpp:
// 79-103) is recomputed as a reduction over the q of every visited non-root node -- exactly the
// multiset's content.  Chunk 0's entries must already be in flight (stage_regions).
// --------------------------------------------------------------------------------------------
__device__ __forceinline__ void backup(const Geo &g, const Dev &d, Lds &s, int t, int D, int tot, float value, float reward, float disc,
                       TreeHdr &h, int cnt0, int n0, int nv0, int need0, int off0, int &err, long long *stl,
                       float *xmm) {
    const int l = lane_id();
    const unsigned long long b0 = (MZ_STAMPS != 0) ? __builtin_amdgcn_s_memtime() : 0ull;
    unsigned long long b1 = 0, bw = 0;
#ifdef MZ_PROBE5
    unsigned long long pre5 = 0;
#endif
    // bootstrap values (cnode.cpp:424,448): b_{i-1} = reward_i + discount * b_i from b_D = value,
    // one f32 multiply and one add per level, in the reference's order, in chunks of up to 63
    // levels (boot_dpp): lane j of a chunk topped by level hi holds level hi - 63 + j.
    {
        float carry = value;
        int hi = D;
        const float dv = disc;
        while (true) {
            const int lo = hi > 63 ? hi - 63 : 0;
            const int nl = hi - lo;  // steps of this chunk
            const int lev = hi - 63 + l;
            float rn = 0.f;  // reward of the level above this lane's
            if (lev >= lo && lev < hi) {
                const int up = (g.K == 1) ? lev + 1 : s.path[lev + 1].x;  // K = 1: path[i] = node i
                rn = (lev + 1 == D) ? reward : i2f(s.A[up].w);
            }
            float b = (l == 63) ? carry : 0.f;
            float tmp = (l == 62) ? disc * carry : 0.f;
#ifdef MZ_PROBE5  // diagnostic: everything outstanding drained before the chain itself
            {
                unsigned long long q;
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(q)::"memory");
                if (hi == D) pre5 = q;
            }
#endif
            int steps = nl;
#ifdef MZ_ABL_NOBOOT  // ablation (timing experiments only): no recurrence
            steps = 0;
#endif
            boot_dpp(b, tmp, dv, rn, steps);
            if (lev >= lo && lev <= hi) s.boot[lev] = b;
            if (lo == 0) break;
            carry = rlf(b, 63 - nl);  // level lo, the next chunk's top
            hi = lo;
        }
    }
    if (MZ_STAMPS) {
        wait_lds();
        b1 = __builtin_amdgcn_s_memtime();
    }
    int2 *gV = d.V() + (size_t)t * g.P * g.E;
    int cnt = cnt0, n = n0, nv = nv0, need = need0, off = off0;
    long long ent_r = 0, ent_w = 0;
    for (int i0 = 0; i0 <= D;) {
        if (cnt == 0) {
            err |= kErrPath;
            MZ_SITE(1);
            return;
        }
        unsigned long long w0s = 0;
        if (MZ_STAMPS) w0s = __builtin_amdgcn_s_memtime();
        wait_vm();
        wait_lds();
        if (MZ_STAMPS) bw += __builtin_amdgcn_s_memtime() - w0s;
        const int i = i0 + l;
        // position of this lane's new (depth, value) among its node's sorted entries: entries of a
        // smaller depth (lo), of the same depth (c), of the same depth and a smaller value (pv).
        // Counted by the whole wave, one needing node at a time, 64 entries per ballot.
        int lo = nv, c = 0, pv = 0;
        const float key = (l < cnt) ? s.boot[i] : 0.f;
        for (unsigned long long m = ballot(l < cnt && need); m; m &= m - 1ull) {
            const int j = __builtin_ctzll(m);
            const int nvj = rl(nv, j), offj = rl(off, j), depj = D - (i0 + j);
            const float keyj = rlf(key, j);
            int cl = 0, cc = 0, cp = 0;
            for (int e0 = 0; e0 < nvj; e0 += kWave) {
                const bool on = e0 + l < nvj;
                const int2 e = on ? s.reg[offj + e0 + l] : make_int2(0x7fffffff, 0);
                cl += __popcll(ballot(on && e.x < depj));
                cc += __popcll(ballot(on && e.x == depj));
                cp += __popcll(ballot(on && e.x == depj && i2f(e.y) < keyj));
            }
            if (l == j) {
                lo = cl;
                c = cc;
                pv = cp;
            }
            ent_r += nvj;
        }
        int pos = 0;
        if (l < cnt) {
            const int dep = D - i;
            const int2 *R = s.reg + off;
            const float4 cw = s.C[n];  // staged per node in round 1
            float ws = cw.x, tw = cw.y;
            const float lp = s.lp[dep];
            const int cur = (c == 0) ? 0 : value_lim(c, g.one_minus_rho);
            const int nl = value_lim(c + 1, g.one_minus_rho);
            if (cur == nl) {
                const float mb = i2f(R[lo + c - cur].y);  // *big.begin()
                if (!(key < mb)) {
                    ws -= lp * mb;
                    tw -= lp;
                    tw += lp;
                    ws += lp * key;
                }
            } else {
                if (cur + 1 != nl) err |= kErrValueSet;
                if (c - cur == 0) {
                    tw += lp;
                    ws += lp * key;
                } else {
                    const float ms = i2f(R[lo + c - cur - 1].y);  // *(--small.end())
                    if (key > ms) {
                        tw += lp;
                        ws += lp * key;
                    } else {
                        tw += lp;
                        ws += lp * ms;
                    }
                }
            }
            // insert (dep, key) at its sorted place (the tail moves up by one below, by the wave)
            pos = lo + pv;
            int2 *G = gV + (size_t)n * g.E;
            if (nv + 1 > g.E) {
                err |= kErrPath;
                MZ_SITE(2);
                pos = nv;  // no shift
            } else {
                G[pos] = make_int2(dep, f2i(key));
            }
            // node scalars
            // the leaf's record is being expanded by the other wave: it has children now (nc >= 1),
            // its reward is this simulation's input, and its B record belongs to the expansion
            const bool is_leaf = (i == D);
            int4 a4 = s.A[n];
            if (is_leaf) a4.w = f2i(reward);
            const int4 b4 = s.B[n];
            const int nc = is_leaf ? 1 : nc_of(b4.y);
            const float val = (nc > 0) ? ws / tw : 0.f;  // CNode::value (cnode.cpp:42-56)
            const int4 na = make_int4(a4.x + 1, a4.y, f2i(val), a4.w);
            const int md = md_of(b4.y);
            s.A[n] = na;
            const size_t gi = (size_t)t * g.P + n;
            d.A()[gi] = na;
            d.C()[gi] = make_float4(ws, tw, 0.f, 0.f);
            if (dep > md && !is_leaf) {
                const int4 nb4 = make_int4(b4.x, pack_y(nc, act_of(b4.y), dep), b4.z, b4.w);
                s.B[n] = nb4;
                d.Bn()[gi] = nb4;
            }
            if (i >= 1) {
                const float q = (i2f(a4.w) + disc * val) - s.PP[n];  // get_qsa - father->pred_value
                s.Q[n] = q;
                d.Q()[gi] = q;
            }
        }
        // the sorted entries' tails move up by one slot, node by node, 64 entries per store
        for (unsigned long long m = ballot(l < cnt && nv > pos); m; m &= m - 1ull) {
            const int j = __builtin_ctzll(m);
            const int nvj = rl(nv, j), posj = rl(pos, j), offj = rl(off, j), nj = rl(n, j);
            ent_w += nvj - posj;
            int2 *Gj = gV + (size_t)nj * g.E;
            for (int e0 = posj; e0 < nvj; e0 += kWave)
                if (e0 + l < nvj) Gj[e0 + l + 1] = s.reg[offj + e0 + l];
        }
        ent_w += cnt;  // each updated node writes its new entry (plus the tail shifts above)
        wait_lds();
        i0 += cnt;
        if (i0 <= D) cnt = stage_regions(g, d, s, t, D, i0, n, nv, need, off);
    }
    stl[MZ_S_BACKUP_NODES] += D + 1;
    stl[MZ_S_ENTRIES_READ] += ent_r;
    stl[MZ_S_ENTRIES_WRITTEN] += ent_w;
    if (MZ_STAMPS) {
        wait_lds();
        const unsigned long long b2 = __builtin_amdgcn_s_memtime();
        stl[MZ_S_CYC_BAK_BOOT] += (long long)(b1 - b0);
#ifdef MZ_PROBE5
        stl[MZ_S_CYC_MINMAX] += (long long)(pre5 - b0);  // entry -> chain start (all drained)
#endif
        stl[MZ_S_CYC_BAK_WAIT] += (long long)bw;
        stl[MZ_S_CYC_BAK_NODES] += (long long)(b2 - b1 - bw);
    }
    // min/max over the q of visited non-root nodes (`tot` = the node count before this
    // simulation's expansion: the new children are unvisited, and the other wave writes them)
    // The reductions end in lane 63 (no v_readlane, ~30 cycles each on gfx950), which hands
    // min / max to the other wave through LDS; the count is a scalar popcount of ballots.
    float mn = INFINITY, mx = -INFINITY;
    int cv = 0;
    for (int base = 1; base < tot; base += kWave) {
        const int nn = base + l;
        const bool on = nn < tot && s.A[nn].x > 0;
        if (on) {
            const float q = s.Q[nn];
            mn = fminf(mn, q);
            mx = fmaxf(mx, q);
        }
        cv += __popcll(ballot(on));
    }
    mn = wave_min_to63(mn);
    mx = wave_max_to63(mx);
    if (l == 63) {
        xmm[0] = mn;
        xmm[1] = mx;
    }
    h.mm_cnt = cv;
    stl[MZ_S_MINMAX_NODES] += tot - 1;
}

// pUCT coefficient pb_c(n, v) for this lane (cnode.cpp:313-314): the host-built table when it is
// staged, else the same double arithmetic on the pb / sq tables.
__device__ __forceinline__ float puct(const Geo &g, const Lds &s, int n, int v) {
    if (g.use_table) return s.T[n * (n + 1) / 2 + v];
    const float pbl = s.pb[n];
    const double sqn = s.sq[n];
    return (float)((double)pbl * (sqn / (double)(v + 1)));
}

// value part of ucb_score for every node (cnode.cpp:317-331): qsa - parent.pred_value (0 while
// unvisited), min/max normalised, clamped to [0, 1].  One float division per node, all nodes in
// parallel.  General trees also get the whole ucb_score under the parent (Sc), which the tie lists
// of select_walk read.
__device__ __forceinline__ void value_scores(const Geo &g, Lds &s, int tot, float disc, const TreeHdr &h) {
    const int l = lane_id();
    const bool mm_on = h.mm_cnt > 0;
    const float mmn = h.mm_min, mmx = h.mm_max;
    float den = 0.f;
    if (mm_on) {
        const float delta = mmx - mmn;
        den = (g.delta < delta) ? delta : g.delta;  // std::max(delta_lb, delta)
    }
    for (int base = 0; base < tot; base += kWave) {
        const int n = base + l;
        if (n < tot) {
            const int4 a4 = s.A[n];
            float vs = (a4.x == 0) ? 0.0f : ((i2f(a4.w) + disc * i2f(a4.z)) - s.PP[n]);
            if (mm_on) vs = (vs - mmn) / den;
            if (vs < 0) vs = 0;
            if (vs > 1) vs = 1;
            s.Vs[n] = vs;
            if (g.K > 1 && n >= 1) {
                // ucb_score under the parent (cnode.cpp:297-335); a parent outside the pUCT table
                // range is reported by its tie list (select_walk)
                const int np = s.A[s.Par[n]].x - 1;  // total_children_visit_counts
                s.Sc[n] = (np >= 0 && np < g.PS) ? puct(g, s, np, a4.x) * i2f(a4.y) + vs : 0.f;
            }
        }
    }
    wait_lds();
}

__device__ __forceinline__ unsigned select_word(const Geo &g, const Dev &d, const Lds &s, int t, int cursor, int wbase,
                                                int lds_base, unsigned rw0, unsigned rw1, int &err) {
    // rw0 / rw1 hold words wbase + [0, 128) copied from the LDS window only (rng_word_win), so
    // reading them waits for LDS, never for the expansion's outstanding stores
    const int o = cursor - wbase, ol = cursor - lds_base;
    if (ol >= 0 && ol < kRngWin) {
        if (o >= 0 && o < kWave) return (unsigned)rl((int)rw0, o);
        if (o >= kWave && o < 2 * kWave) return (unsigned)rl((int)rw1, o - kWave);
        return (unsigned)uni((int)s.rng[ol]);
    }
    if (cursor < g.W) return (unsigned)uni((int)d.R()[(size_t)t * g.W + cursor]);
    err |= kErrRng;
    return 0u;
}

// ucb score of node `child` under node `parent` (used for the single-child checks)
__device__ __forceinline__ float path_score(const Geo &g, const Lds &s, int parent, int child, int &err) {
    const int n = s.A[parent].x - 1;
    if (n < 0 || n >= g.PS) {
        err |= kErrTable;
        return 0.f;
    }
    const int4 ca = s.A[child];
    return puct(g, s, n, ca.x) * i2f(ca.y) + s.Vs[child];
}

// Layout classes up to this pool size take the precomputed walk (cheaper while the per-node
// scoring passes are few); larger classes and the general layout take the level walk.  Measured
// on one box: 3m K = 5 (260 nodes) 12.0 us precomputed against 12.7 us by levels; 3s5z K = 5 (510
// nodes) 14.5 against 13.9 us; 27m K = 5 (1010 nodes) 19.1 against 15.8 us.  A compile-time
// choice: with both walks in one kernel the compiler kept the LDS view in scratch memory.
template <int NC>
constexpr bool kWalkPrecomputed = (NC > 0 && NC <= 384);

// The internal nodes (children count > 0) among nodes [0, tot), compacted into s.il in node
// order with ballots; returns their number (wave-uniform).
__device__ __forceinline__ int compact_internal(Lds &s, int tot) {
    const int l = lane_id();
    int nint = 0;
    for (int base = 0; base < tot; base += kWave) {
        const int n = base + l;
        const bool in = n < tot && nc_of(s.B[n].y) > 0;
        const unsigned long long m = ballot(in);
        if (in) s.il[nint + __popcll(m & ((1ull << l) - 1ull))] = n;
        nint += __popcll(m);
    }
    wait_lds();
    return uni(nint);
}

// General trees, small pools: select_child resolved for every internal node first (scores per
// node by value_scores, one lane per internal node for the tie lists), then a pointer chase.
__device__ __forceinline__ void walk_precomputed(const Geo &g, const Dev &d, Lds &s, int t, int tot, TreeHdr &h, int lds_base, unsigned rw0, unsigned rw1,
                            int &err, int &out_idx, int &out_act, long long *stl, float disc, int cursor0, int wbase,
                            int nint_pre) {
    const int l = lane_id();
    long long scored = 0;
#ifdef MZ_PROBE3
    unsigned long long q0 = __builtin_amdgcn_s_memtime(), q1 = 0, q2 = 0, q3 = 0;
#endif
    // (1) internal nodes (children count > 0) in s.il: compacted by the expanding wave while it
    // waited for the back-propagation (nint_pre >= 0), else here
    constexpr int kNxtLeaf = -1, kNxtSlow = -2;
    int *ilist = s.il;
    int *nxt = s.Par;  // (the parent indices are not needed after value_scores)
    int nint = nint_pre;
    if (nint < 0) nint = compact_internal(s, tot);
    wait_lds();
#ifdef MZ_PROBE3
    q1 = __builtin_amdgcn_s_memtime();
#endif
    // (2) select_child's tie list of every internal node (cnode.cpp:355-370), one lane per node,
    // over its children's scores (value_scores): the reference's sequential arg-max with epsilon
    // ties.  A one-child list (the usual case) is stored as the next node; other lists go to the
    // record {bits lo (Vs), bits hi (flag), size | table error << 16 (Q)} for the exact path (the
    // walk reads no node's Vs / flag / Q otherwise; Q is re-staged from HBM by the next launch).
    for (int j0 = 0; j0 < nint; j0 += kWave) {
        const int j = j0 + l;
        if (j < nint) {
            const int p = ilist[j];
            const int pv = s.A[p].x;
            const int4 pbn = s.B[p];
            const int fc = pbn.x, nc = nc_of(pbn.y);
            const int np = pv - 1;  // total_children_visit_counts = node->visit_count - 1
            const bool terr = np < 0 || np >= g.PS;
            float mx = -1000000.0f;  // FLOAT_MIN (utils.h:12)
            unsigned long long lst = 0ull;
            int cnt = 0;
            for (int i0 = 0; i0 < nc; i0 += 4) {
                float sc[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) sc[u] = s.Sc[fc + ((i0 + u < nc) ? i0 + u : i0)];
#pragma unroll
                for (int u = 0; u < 4; ++u) {  // branch-free (selects): lanes diverge in nc
                    const int i = i0 + u;
                    const float v = sc[u];
                    const bool ok = i < nc;
                    const bool gt = ok && (mx < v);
                    const bool ge = ok && !gt && (v >= mx - 0.000001f);
                    const unsigned long long bit = 1ull << (i & 63);
                    lst = gt ? bit : (ge ? (lst | bit) : lst);
                    cnt = gt ? 1 : (cnt + (ge ? 1 : 0));
                    mx = gt ? v : mx;
                }
            }
            if (cnt == 1 && !terr) {
                nxt[p] = fc + __builtin_ctzll(lst);
            } else {
                nxt[p] = kNxtSlow;
                s.Vs[p] = i2f((int)(unsigned)(lst & 0xffffffffull));
                s.flag[p] = (int)(unsigned)(lst >> 32);
                s.Q[p] = i2f(cnt | (terr ? 0x10000 : 0));
            }
        }
    }
    wait_lds();
#ifdef MZ_PROBE3
    q2 = __builtin_amdgcn_s_memtime();
#endif
    // (3) the walk: one LDS read per level (the next node), one engine word per level; the
    // exact record only for ties, empty lists and table errors.  Level i's node goes to lane i of
    // px (LDS beyond 64 levels).
    int x = 0, D = 0, cursor = cursor0;
    int px = 0;
    {
        const int4 r0b = uni4(s.B[0]);
        const int rv = uni(s.A[0].x);
        const int nc0 = nc_of(r0b.y);
        int v;
        if (nc0 == 0) {
            v = kNxtLeaf;
        } else if (rv <= nc0) {
            v = r0b.x + rv - 1;  // forced root round-robin (cnode.cpp:398-399): no word
        } else {
            v = uni(nxt[0]);
            if (v >= 0) ++cursor;
        }
        // (every branch condition and loop-carried value goes through readfirstlane, so the
        // compiler keeps the loop on the scalar unit instead of an exec-masked loop)
        while (true) {
            v = uni(v);
            cursor = uni(cursor);
            if (v < 0) {
                if (v == kNxtLeaf) break;
                // exact path for this level: ties (engine word modulo the list size), an empty
                // list (child 0, no word) or a table error
                const int xfl = uni(f2i(s.Q[x]));
                if (uni(xfl >> 16)) {
                    err |= kErrTable;
                    break;
                }
                const int cnt = uni(xfl & 0xffff);
                int ci = 0;
                if (cnt > 0) {
                    unsigned long long lst = ((unsigned long long)(unsigned)uni(s.flag[x]) << 32) |
                                             (unsigned)uni(f2i(s.Vs[x]));
                    if (cnt > 1) {
                        const unsigned w = select_word(g, d, s, t, cursor, wbase, lds_base, rw0, rw1, err);
                        for (int k = uni((int)(w % (unsigned)cnt)); k > 0; --k) lst &= lst - 1ull;
                    }
                    ++cursor;
                    ci = uni(__builtin_ctzll(lst));
                }
                v = uni(uni(s.B[x].x) + ci);
            }
            if (D + 1 >= g.PS) {
                err |= kErrPath;
                MZ_SITE(3);
                break;
            }
            x = v;
            ++D;
            if (D < kWave) px = wl(px, x, D);
            else if (l == 0) s.path[D].x = x;
            const int vn = nxt[x];
            const int ncx = uni(nc_of(s.B[x].y));
            v = (ncx == 0) ? kNxtLeaf : uni(vn);  // (nxt holds records of internal nodes only)
            if (v >= 0) ++cursor;
        }
    }
#ifdef MZ_PROBE3
    wait_lds();
    const unsigned long long q2b = __builtin_amdgcn_s_memtime();
#endif
    if (cursor > g.W) err |= kErrRng;  // a consumed word beyond the stream (select_word's check)
    if (D == 0) err |= kErrRoot;
    wait_lds();
    // the path {node, visit at selection} for the next back-propagation, the statistics and the
    // outputs, by the whole wave
    int2 *gp = d.path() + (size_t)t * g.PS;
    int nsc = 0;
    int xpar = 0;
    for (int i0 = 0; i0 <= D; i0 += kWave) {
        const int i = i0 + l;
        if (i <= D) {
            const int xi = (i < kWave) ? px : s.path[i].x;
            const int2 e = make_int2(xi, s.A[xi].x);
            gp[i] = e;
            s.path[i] = e;
            const int4 bi = s.B[xi];
            if (i < D && !(i == 0 && e.y <= nc_of(bi.y))) nsc += nc_of(bi.y);  // scored levels
            if (i == D - 1) xpar = bi.w;
        }
    }
    scored = wave_sum(nsc);
    h.cursor = cursor;
    h.D = D;
    h.leaf = x;
    out_idx = uni(rl(xpar, (D - 1) & (kWave - 1)));  // parent->hidden_state_index_x
    if (D == 0) out_idx = uni(s.B[0].w);
    out_act = act_of(uni(s.B[x].y));  // children_action of the last edge
    stl[MZ_S_SELECTS] += 1;
    stl[MZ_S_PATH_EDGES] += D;
    stl[MZ_S_SCORED] += scored;
#ifdef MZ_PROBE3
    q3 = __builtin_amdgcn_s_memtime();
    stl[MZ_S_CYC_W1_ROUND1] += (long long)(q1 - q0);  // compaction
    stl[MZ_S_CYC_W1_STAGE2] += (long long)(q2 - q1);  // tie lists
    stl[MZ_S_CYC_W1_BACKUP] += (long long)(q3 - q2);  // walk + path
    stl[MZ_S_CYC_W1_SYNC] += (long long)(q2b - q2);  // walk loop only
#endif
}

// General trees, large pools: level by level, each level's children scored on the fly.
__device__ __forceinline__ void walk_levels(const Geo &g, const Dev &d, Lds &s, int t, int tot, TreeHdr &h, int lds_base, unsigned rw0, unsigned rw1,
                            int &err, int &out_idx, int &out_act, long long *stl, float disc, int cursor0, int wbase) {
    const int l = lane_id();
#ifdef MZ_PROBE3
    const unsigned long long q0 = __builtin_amdgcn_s_memtime();
#endif
    // General trees: level by level, select_child (cnode.cpp:337-379) scored on the fly, lane j
    // for child j, with ucb_score's arithmetic (cnode.cpp:297-335).  The reference's sequential
    // arg-max with epsilon ties is the closed form [r] + {i > r : s_i >= M - eps} (M the maximum,
    // r its first index; {i : s_i >= FLOAT_MIN} when M <= FLOAT_MIN): a row / wave max and two
    // ballots.  Every branch condition and loop-carried value goes through readfirstlane, so
    // the loop stays on the scalar unit.  Level i's node goes to lane i of px (LDS past 64).
    const bool mm_on = h.mm_cnt > 0;
    const float mmn = h.mm_min, mmx = h.mm_max;
    float den = 0.f;
    if (mm_on) {
        const float delta = mmx - mmn;
        den = (g.delta < delta) ? delta : g.delta;  // std::max(delta_lb, delta)
    }
    int x = 0, D = 0, cursor = cursor0;
    int px = 0;
    int xv = uni(s.A[0].x);
    int4 xb = uni4(s.B[0]);
    long long nscored = 0;
    while (true) {
        x = uni(x);
        xv = uni(xv);
        cursor = uni(cursor);
        const int nc = uni(nc_of(xb.y));
        if (nc == 0) break;
        const int fc = uni(xb.x);
        int ci = 0;
        if (x == 0 && xv <= nc) {
            ci = xv - 1;  // forced root round-robin (cnode.cpp:398-399)
        } else {
            const int np = xv - 1;  // total_children_visit_counts = node->visit_count - 1
            if (np < 0 || np >= g.PS) {
                err |= kErrTable;
                break;
            }
            nscored += nc;
            const bool has = l < nc;
            float sc = -INFINITY;
            if (has) {
                const int4 ca = s.A[fc + l];
                float vs = (ca.x == 0) ? 0.0f : ((i2f(ca.w) + disc * i2f(ca.z)) - s.PP[fc + l]);
                if (mm_on) vs = (vs - mmn) / den;
                if (vs < 0) vs = 0;
                if (vs > 1) vs = 1;
                sc = puct(g, s, np, ca.x) * i2f(ca.y) + vs;
            }
            float M;
            if (nc <= 16) {  // one DPP row holds every child
                float v = sc;
                v = fmaxf(v, i2f(dpp<0xB1>(f2i(v))));
                v = fmaxf(v, i2f(dpp<0x4E>(f2i(v))));
                v = fmaxf(v, i2f(dpp<0x141>(f2i(v))));
                v = fmaxf(v, i2f(dpp<0x140>(f2i(v))));
                M = unif(v);
            } else {
                M = unif(wave_max(sc));
            }
            unsigned long long lst;
            if (M > -1000000.0f) {  // FLOAT_MIN (utils.h:12)
                const unsigned long long first = ballot(has && sc == M);
                const int r = uni(__builtin_ctzll(first));
                lst = ballot(has && sc >= M - 0.000001f) & (~0ull << r);
            } else {
                lst = ballot(has && sc >= -1000000.0f);
            }
            const int cnt = uni(__popcll(lst));
            if (cnt > 0) {  // one engine word (gen() % size); its value matters only for ties
                if (cnt > 1) {
                    const unsigned w = select_word(g, d, s, t, cursor, wbase, lds_base, rw0, rw1, err);
                    for (int k = uni((int)(w % (unsigned)cnt)); k > 0; --k) lst &= lst - 1ull;
                } else if (cursor >= g.W) {
                    err |= kErrRng;
                }
                ++cursor;
                ci = uni(__builtin_ctzll(lst));
            }
        }
        if (D + 1 >= g.PS) {
            err |= kErrPath;
            MZ_SITE(4);
            break;
        }
        x = uni(fc + ci);
        ++D;
        if (D < kWave) px = wl(px, x, D);
        else if (l == 0) s.path[D].x = x;
        xv = uni(s.A[x].x);
        xb = uni4(s.B[x]);
    }
    if (D == 0) err |= kErrRoot;
    wait_lds();
#ifdef MZ_PROBE3
    const unsigned long long q1 = __builtin_amdgcn_s_memtime();
#endif
    // the path {node, visit at selection} for the next back-propagation and the outputs, by the
    // whole wave
    int2 *gp = d.path() + (size_t)t * g.PS;
    int xpar = 0;
    for (int i0 = 0; i0 <= D; i0 += kWave) {
        const int i = i0 + l;
        if (i <= D) {
            const int xi = (i < kWave) ? px : s.path[i].x;
            const int2 e = make_int2(xi, s.A[xi].x);
            gp[i] = e;
            s.path[i] = e;
            if (i == D - 1) xpar = s.B[xi].w;
        }
    }
    h.cursor = cursor;
    h.D = D;
    h.leaf = x;
    out_idx = (D == 0) ? uni(s.B[0].w) : uni(rl(xpar, (D - 1) & (kWave - 1)));  // parent->hidden_state_index_x
    out_act = act_of(uni(s.B[x].y));  // children_action of the last edge
    stl[MZ_S_SELECTS] += 1;
    stl[MZ_S_PATH_EDGES] += D;
    stl[MZ_S_SCORED] += nscored;
#ifdef MZ_PROBE3
    const unsigned long long q2 = __builtin_amdgcn_s_memtime();
    stl[MZ_S_CYC_W1_ROUND1] += 0;
    stl[MZ_S_CYC_W1_STAGE2] += 0;
    stl[MZ_S_CYC_W1_BACKUP] += (long long)(q2 - q0);  // walk + path
    stl[MZ_S_CYC_W1_SYNC] += (long long)(q1 - q0);    // walk loop only
#endif
}

// --------------------------------------------------------------------------------------------
// CTree::select_path (cnode.cpp:381-413) with select_child (337-379) and ucb_score (297-335).
//
// K = 1 trees are chains (one child per expansion), so the path is every node in creation order
// and the only data-dependent effect of a level is whether select_child's tie list is non-empty
// (score >= FLOAT_MIN, not NaN), which decides whether an engine word is consumed: all levels
// are scored in parallel and the words counted with one ballot.
//
// Otherwise select_child (its tie list: the sequential arg-max with epsilon ties) is evaluated for
// every internal node at once, one lane per node, before the walk; the walk then descends one LDS
// round trip per level and spends serial work only on the engine word (one per non-forced level
// with a non-empty list; the pick among several tied children takes it modulo the list size).
// --------------------------------------------------------------------------------------------
template <int NC>
__device__ __forceinline__ void select_walk(const Geo &g, const Dev &d, Lds &s, int t, int tot, TreeHdr &h, int lds_base,
                            unsigned rw0, unsigned rw1, int &err, int &out_idx, int &out_act, long long *stl,
                            bool fast, float disc, int nint_pre) {
    const int l = lane_id();
    const int cursor0 = h.cursor;
    const int wbase = cursor0;  // register window [wbase, wbase + 128)
    long long scored = 0;
    if (g.K == 1) {
        const int D = tot - 1;
        if (D < 1) err |= kErrRoot;
        if (D + 1 > g.PS) { err |= kErrPath; MZ_SITE(5); }
        int words = 0;
        if (!err) {
            const int root_visit = uni(s.A[0].x);
            if (fast) {
                // Every level's tie list is non-empty: the pUCT coefficients are finite and >= 0
                // (fast_ok), priors lie in [0, 1e30] and rewards / values in [-1e30, 1e30]
                // (TreeHdr::tame), so with |discount| <= 1, 0 <= lambda <= 1 and delta_lb > 0 every
                // q, min/max bound and normalised value is finite, the value score lies in [0, 1]
                // and the score prior_score + value_score is >= 0 (+inf at worst), never NaN.
                // Each level consumes one word except the forced root child (cnode.cpp:398-399).
                // Parent visit totals stay below the table size (root visits <= S + 1 < PS).
                if (root_visit - 1 >= g.PS) err |= kErrTable;
                words = D - ((root_visit <= 1) ? 1 : 0);
            } else {
                for (int base = 0; base <= D; base += kWave) {
                    const int i = base + l;
                    bool valid = false;
                    if (i <= D) {
                        if (i >= 1 && !(i == 1 && root_visit <= 1)) {
                            const float sc = path_score(g, s, i - 1, i, err);
                            valid = sc >= -1000000.0f;  // tie list non-empty (FLOAT_MIN, utils.h:12)
                        }
                    }
                    words += __popcll(ballot(valid));
                }
            }
            scored = D;
        }
        h.cursor = cursor0 + words;
        h.D = D;
        h.leaf = D;
        const int4 pb = uni4(s.B[D > 0 ? D - 1 : 0]);
        const int4 lb = uni4(s.B[D > 0 ? D : 0]);
        out_idx = pb.w;
        out_act = act_of(lb.y);
        stl[MZ_S_SELECTS] += 1;
        stl[MZ_S_PATH_EDGES] += D;
        stl[MZ_S_SCORED] += scored;
        // (no path record: the next back-propagation walks the chain itself, stage_regions)
        return;
    }

    if constexpr (kWalkPrecomputed<NC>)
        walk_precomputed(g, d, s, t, tot, h, lds_base, rw0, rw1, err, out_idx, out_act, stl, disc, cursor0, wbase,
                         nint_pre);
    else
        walk_levels(g, d, s, t, tot, h, lds_base, rw0, rw1, err, out_idx, out_act, stl, disc, cursor0, wbase);
}

// --------------------------------------------------------------------------------------------
// One simulation step of one tree: [expand + back-propagate (sim s)] -> [select (sim s+1)] ->
// [gather the selected leaf's parent hidden state].
// Memory round trips: (1) tree header (scalar), tables and network outputs; (2) path, node
// records, q / parent values, RNG window -- issued before one wait; (3) path-node scalars and the
// value entries the back-propagation needs, in flight while the leaf is expanded.
// --------------------------------------------------------------------------------------------
// Scalar arguments, the ones each wave needs first leading: with kernel-argument preloading
// (-mllvm -amdgpu-kernarg-preload-count) the first 16 dwords arrive in SGPRs at wave launch, so the
// round-1 addresses do not wait for a kernel-argument load.
template <bool EB, bool SEL, int NC, bool JOINT>
__global__ __launch_bounds__(128) void k_step(char *base, int P, int PS, int BA, int pk, const float *reward,
                                              const float *value, const float *policy, const float *beta, int K,
                                              int hsx, float discount,
                                              int fast_ok, const char *pool, long long pool_stride, long long row_bytes,
                                              char *gather_out, int *idx_x, int *idy, int *act) {
#ifdef MZ_PROBE2
    unsigned long long pt0;
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(pt0)::"memory");
#endif
#ifdef MZ_ABL_EMPTY  // ablation (timing experiments only): launch cost of this kernel
    if (true) return;
#endif
    // The first 14 argument dwords arrive in SGPRs (kernel-argument preloading): the arena base,
    // the geometry (B | A << 24, path bound | handle K << 17: the host passes exactly the Params
    // block's values) and the four network-output pointers, so every round-1 address is computed
    // without a memory round trip.  Compile-time layout classes read the other arguments and the
    // rest of Params in one batch after the round-1 loads are issued (kLateParams).
    constexpr bool kLateParams = (NC > 0 && !JOINT);
    const int B = BA & 0xffffff, A = (int)((unsigned)BA >> 24);
    const int pe = pk & 0x1ffff, gK = (int)((unsigned)pk >> 17);
    const int ne = (1ll + (long long)gK * (pe - 1)) < P ? 1 + gK * (pe - 1) : P;  // node bound (launch_step)
    Geo g;
    Dev d;
    const Params *prm = (const Params *)base;  // the Params block heads the arena (mz_create)
    if constexpr (!kLateParams) {
        g = prm->g;
        d = prm->d;
    }
    g.B = B;
    g.P = P;
    g.PS = PS;
    g.A = A;
    g.K = gK;
    d.base = (gchar *)base;
    arena_hot(d, B, P, PS);
    StepArgs a;
    a.reward = reward;
    a.value = value;
    a.policy = policy;
    a.beta = beta;
    a.hsx = hsx;
    a.ne = ne;
    a.pe = pe;
    a.K = K;
    a.discount = discount;
    a.pool = pool;
    a.pool_stride = pool_stride;
    a.row_bytes = row_bytes;
    a.gather_out = gather_out;
    a.idx_x = idx_x;
    a.idy = idy;
    a.act = act;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    Lds s = make_lds<NC>(smem, g);
    const int t = blockIdx.x;
    const int l = threadIdx.x & (kWave - 1);
    // Two waves per tree.  Wave 0 expands the leaf, then selects and gathers; wave 1 back-propagates
    // the path and recomputes the min/max normaliser at the same time: the expansion only creates
    // new nodes and the leaf's structure fields, the back-propagation only updates existing path
    // nodes (the leaf's visit / value / reward), so the two share no LDS or HBM word.
    const int wv = uni((int)(threadIdx.x >> 6));
    long long *xst = lds_xchg<NC>(smem, g);  // wave 1 -> wave 0: statistics, min/max, error
    unsigned long long ts[10] = {0};
    stamp(ts, 0);
    const size_t nb = (size_t)t * g.P;
    // ---- round 1: everything that does not depend on the tree header, issued with it --------
    float pol = 0.f, bet = 0.f, r_in = 0.f, v_in = 0.f;
    unsigned w1r = 0u, w2r = 0u;
    const bool have_w = !JOINT && 2 * g.K <= kNxt;  // (call K <= handle K)
    float *sJpol = JOINT ? (float *)(smem + g.oJpol) : nullptr;
    float *sJbet = JOINT ? (float *)(smem + g.oJbet) : nullptr;
    unsigned char *sJ = JOINT ? (smem + g.oJ) : nullptr;

#ifdef MZ_PROBE
    unsigned long long pr0 = __builtin_amdgcn_s_memtime(), pr1 = 0, pr2 = 0;
#endif
    if (wv == 0) {
        if (SEL) {
            if (NC == 0 && g.use_table) {
                for (int i0 = 0; i0 < g.TT; i0 += 4 * kWave)
                    if (i0 + 4 * l < g.TT) glds16(d.T() + i0 + 4 * l, s.T + i0);
            } else {
                for (int i0 = 0; i0 < g.PS; i0 += kWave)
                    if (i0 + l < g.PS) glds4(d.pb() + i0 + l, s.pb + i0);
                for (int i0 = 0; i0 < 2 * g.PS; i0 += kWave)
                    if (i0 + l < 2 * g.PS) glds4((const int *)d.sq() + i0 + l, (int *)s.sq + i0);
            }
        }
#ifdef MZ_PROBE
        pr1 = __builtin_amdgcn_s_memtime();
#endif
        if (EB && JOINT) {
            const size_t ib = (size_t)t * g.NA;
            for (int i0 = 0; i0 < g.NA; i0 += kWave)
                if (i0 + l < g.NA) {
                    glds4(a.policy + ib + i0 + l, sJpol + i0);
                    glds4(a.beta + ib + i0 + l, sJbet + i0);
                }
        } else if (EB) {
            const size_t ib = (size_t)t * g.A;
            if (l < g.A) {
                pol = a.policy[ib + l];
                bet = a.beta[ib + l];
            }
            if (have_w && l < g.K) {
                w1r = d.hdr()[t].nxt[2 * l];
                w2r = d.hdr()[t].nxt[2 * l + 1];
            }
        }
    } else {
        for (int i0 = 0; i0 < a.ne; i0 += kWave) {
            if (i0 + l < a.ne) {
                glds16(d.A() + nb + i0 + l, s.A + i0);
                glds16(d.Bn() + nb + i0 + l, s.B + i0);
                glds4(d.PP() + nb + i0 + l, s.PP + i0);
                if (SEL && kWalkPrecomputed<NC> && g.K > 1) glds4(d.Par() + nb + i0 + l, s.Par + i0);  // parents (general walk)
                if (EB) {
                    glds4(d.Q() + nb + i0 + l, s.Q + i0);
                    glds16(d.C() + nb + i0 + l, s.C + i0);  // value-set scalars, read by node
                }
            }
        }
        if (EB) {
            for (int i0 = 0; i0 < g.PS + 1; i0 += kWave)
                if (i0 + l < g.PS + 1) glds4(d.lp() + i0 + l, s.lp + i0);
            if (g.K > 1)  // (K = 1 chains need no path: stage_regions)
                for (int i0 = 0; i0 < 2 * a.pe; i0 += kWave)
                    if (i0 + l < 2 * a.pe)
                        glds4((const int *)(d.path() + (size_t)t * g.PS) + i0 + l, (int *)s.path + i0);
        }
    }
    // (the loads above take their addresses from preloaded arguments only; what needs the other
    // kernel arguments or the Params block comes after them)
    TreeHdr h;
    {
        // scalar loads straight into SGPRs (no v_readfirstlane, ~30 cycles each on gfx950): the
        // header was written by an earlier launch and the scalar cache starts every dispatch
        // invalidated; this launch writes it only after reading it
        const cTreeHdr *hp = (const cTreeHdr *)(d.hdr() + t);
        h.cursor = hp->cursor;
        h.tot = hp->tot;
        h.D = hp->D;
        h.err = hp->err;
        h.mm_cnt = hp->mm_cnt;
        h.tame = hp->tame;
        h.mm_min = hp->mm_min;
        h.mm_max = hp->mm_max;
        h.leaf = hp->leaf;
    }
    if (EB) {  // this simulation's network outputs for the leaf (both waves)
        r_in = reward[t];
        v_in = value[t];
    }
#ifdef MZ_ABL_VEC1  // ablation (timing experiments only): launch + the preloaded-address loads only
    if (true) {
        wait_vm();
        return;
    }
#endif
    if constexpr (kLateParams) {
        // Params heads the arena: scalar loads from the preloaded base (the scheduler may issue
        // them earlier; nothing above waits for them)
        const cParams *pl = (const cParams *)__builtin_assume_aligned(base, 256);
        g.K = pl->g.K;  // (equals gK)
        g.S = pl->g.S;
        g.E = pl->g.E;
        g.W = pl->g.W;
        g.TT = pl->g.TT;
        g.use_table = 0;  // compile-time layout classes compute pUCT coefficients from pb / sq
        g.root_offset = pl->g.root_offset;
        g.seed = pl->g.seed;
        g.one_minus_rho = pl->g.one_minus_rho;
        g.delta = pl->g.delta;
        g.reg_cap = pl->g.reg_cap;
        g.N = 1;
        g.NA = A;
        g.JP = 0;
        d.o_J = 0;
        d.o_D = pl->d.o_D;
        d.o_V = pl->d.o_V;
        d.o_R = pl->d.o_R;
        // every scalar the rest of the kernel reads, loaded here in one batch (one wait, while the
        // round-1 vector loads are in flight) instead of lazily behind later branches
        asm volatile("" ::"s"(g.K), "s"(g.E), "s"(g.W), "s"(g.one_minus_rho), "s"(g.delta), "s"(g.reg_cap),
                     "s"(d.o_V), "s"(d.o_R), "s"(d.o_D), "s"(K), "s"(hsx), "s"(discount), "s"(fast_ok), "s"(pool),
                     "s"(pool_stride), "s"(row_bytes), "s"(gather_out), "s"(idx_x), "s"(idy), "s"(act));
        asm volatile("" ::"s"(h.cursor), "s"(h.tot), "s"(h.D), "s"(h.err), "s"(h.mm_cnt), "s"(h.tame), "s"(h.mm_min),
                     "s"(h.mm_max), "s"(h.leaf));
    }
    // gathered row chunks (four named registers: an array here ends up in scratch memory).  A K = 1
    // tree is a chain: the next leaf is the child this simulation's expansion creates, whose
    // parent has hidden_state_index_x = a.hsx, so its row is fetched now and checked after the
    // selection.
    bool gath_pending = false;
    int4 gv0 = make_int4(0, 0, 0, 0), gv1 = gv0, gv2 = gv0, gv3 = gv0;
    char *gdst = nullptr;
    long long grb = 0;
    const bool g_fast = SEL && a.pool &&
                        (((a.row_bytes | a.pool_stride | (long long)(uintptr_t)a.pool |
                           (long long)(uintptr_t)a.gather_out) & 15) == 0) &&
                        a.row_bytes <= 4 * 16 * kWave;
    const bool g_pre = EB && g_fast && g.K == 1;
    // rows above 4 KiB (27m: 13.5 KiB) are staged through LDS with LDS-DMA (no registers held),
    // in the value-entry staging area s.reg: free in K = 1 chains for the whole launch (their
    // updates never read entries) and free in every tree once the back-propagation wave is done
    unsigned char *sbig = (unsigned char *)s.reg;
    const long long big_cap = 8ll * (NC > 0 ? kRegCap : g.reg_cap);
    const bool g_big = SEL && a.pool && !JOINT &&
                       (((a.row_bytes | a.pool_stride | (long long)(uintptr_t)a.pool |
                          (long long)(uintptr_t)a.gather_out) & 15) == 0) &&
                       a.row_bytes > 4 * 16 * kWave && a.row_bytes <= 16 * 16 * kWave && a.row_bytes <= big_cap;
    const bool g_pre_big = EB && g_big && g.K == 1;
    bool gath_lds = false;
    long long *st = d.stats() + (size_t)t * MZ_S_COUNT;
    // counters written per launch: the algorithmic ones, plus the cycle stamps in diagnostic builds
    constexpr int kStatN = (MZ_STAMPS != 0) ? MZ_S_COUNT : MZ_S_CYC_HEADER;
    const long long st_old = (wv == 0 && l < kStatN) ? st[l] : 0;
#ifdef MZ_PROBE
    pr2 = __builtin_amdgcn_s_memtime();
#endif
    if (wv == 0 && g_pre) {
        // issued last and always exactly four loads (offsets clamped into the row), so the
        // round-1 wait below can leave them in flight: the row is needed only at the very end
        const char *src = a.pool + (long long)a.hsx * a.pool_stride + (long long)t * a.row_bytes;
        const long long last = a.row_bytes - 16, o = (long long)l * 16;
        gv0 = *(const int4 *)(src + (o < last ? o : last));
        gv1 = *(const int4 *)(src + (o + 1024 < last ? o + 1024 : last));
        gv2 = *(const int4 *)(src + (o + 2048 < last ? o + 2048 : last));
        gv3 = *(const int4 *)(src + (o + 3072 < last ? o + 3072 : last));
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else if (wv == 0 && g_pre_big) {
        // the same for a big row: always sixteen 1 KiB LDS-DMA chunks (clamped), left in flight
        const char *src = a.pool + (long long)a.hsx * a.pool_stride + (long long)t * a.row_bytes;
        const long long last = a.row_bytes - 16, o = (long long)l * 16;
#pragma unroll
        for (int k = 0; k < 16; ++k) glds16(src + (o + 1024 * k < last ? o + 1024 * k : last), sbig + 1024 * k);
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    } else {
        wait_vm();
    }
    stamp(ts, 1);
#ifdef MZ_ARGCHECK
    // diagnostic build (graph-replay investigation): the scalar-cache header against an L2 read of
    // the same words, the K = 1 chain invariant tot == hsx + 1 on entry, and the preloaded
    // arguments against the Params block and the kernel-argument memory
    if (wv == 0 && l == 0)
        argcheck_record(1, EB, SEL, t, base, P, PS, BA, pk, K, hsx, discount, pe, ne, d.hdr() + t, h.tot, h.cursor,
                        h.D, h.err, (const unsigned *)__builtin_amdgcn_kernarg_segment_ptr(), reward, value, pool, 0);
#endif
#ifdef MZ_ABL_ROUND1  // ablation (timing experiments only): launch + round 1, nothing else
    if (true) {
        wait_vm();
        return;
    }
#endif
    if (h.err) {  // a dead tree stays dead (both waves see the same header) and re-reports its error
        if (wv == 0 && l == 0) atomicOr(d.err(), h.err);
        if (SEL && wv == 0) {
            if (l == 0) {
                a.idx_x[t] = 0;
                a.idy[t] = t;
            }
            if (l < (JOINT ? g.N : 1)) a.act[(size_t)t * (JOINT ? g.N : 1) + l] = 0;
        }
        wait_vm();
        return;
    }
    int err = 0;
    long long stl[MZ_S_COUNT];
#pragma unroll
    for (int k = 0; k < MZ_S_COUNT; ++k) stl[k] = 0;

    const int tot = h.tot;
    // slow path: the host bounds were too small (e.g. a graph replayed out of sequence)
    if (wv == 1 && (tot > a.ne || (EB && h.D + 1 > a.pe))) {
        for (int i0 = a.ne; i0 < tot; i0 += kWave) {
            if (i0 + l < tot) {
                glds16(d.A() + nb + i0 + l, s.A + i0);
                glds16(d.Bn() + nb + i0 + l, s.B + i0);
                glds4(d.PP() + nb + i0 + l, s.PP + i0);
                if (SEL && kWalkPrecomputed<NC> && g.K > 1) glds4(d.Par() + nb + i0 + l, s.Par + i0);
                if (EB) {
                    glds4(d.Q() + nb + i0 + l, s.Q + i0);
                    glds16(d.C() + nb + i0 + l, s.C + i0);
                }
            }
        }
        if (EB && g.K > 1)
            for (int i0 = 2 * a.pe; i0 < 2 * (h.D + 1); i0 += kWave)
                if (i0 + l < 2 * (h.D + 1))
                    glds4((const int *)(d.path() + (size_t)t * g.PS) + i0 + l, (int *)s.path + i0);
        wait_vm();
    }
    stamp(ts, 2);

    // ---- round 2: wave 0 the RNG window (and the leaf's structure record); wave 1 the path
    // nodes' value-set scalars and the value entries the back-propagation needs ------------
    int cnt0 = 0, n0 = 0, nv0 = 0, need0 = 0, off0 = 0;
    const int wbase = h.cursor;
    int4 leaf_b = make_int4(0, 0, 0, 0);
    if (wv == 0) {
        for (int i0 = 0; i0 < kRngWin; i0 += kWave)
            if (wbase + i0 + l < g.W) glds4(d.R() + (size_t)t * g.W + wbase + i0 + l, s.rng + i0);
        if (EB) leaf_b = d.Bn()[nb + h.leaf];  // used after the expansion: no wait here
        if (!EB || !have_w) wait_vm();  // the expansion reads its words from the window
    } else {
        if (JOINT) {  // the nodes' joint actions (tree block of JP bytes, 16-byte aligned)
            const int dw = (tot * g.N + 3) >> 2;
            const unsigned *src = (const unsigned *)(d.J() + (size_t)t * g.JP);
            for (int i0 = 0; i0 < dw; i0 += kWave)
                if (i0 + l < dw) glds4(src + i0 + l, (unsigned *)sJ + i0);
        }
        if (EB) {
            cnt0 = stage_regions(g, d, s, t, h.D, 0, n0, nv0, need0, off0);
        }
    }
    stamp(ts, 3);

    int cursor = h.cursor;
    int ntot = tot;
    int nint_pre = -1;  // internal nodes compacted early by wave 0 (precomputed walk)
    if (EB) {
        if (wv == 0) {
            // ---- CTree::expand (cnode.cpp:224-295) of the leaf (expand_and_backprop, :452-469) ----
            const int leaf = h.leaf;
            long long st_new = 0;
            int nc;
            if (JOINT) {
                nc = expand_joint(g, d, t, leaf, sJpol, sJbet, nullptr, 0.f, a.K, v_in, cursor, ntot, s.rng, wbase, &s, sJ,
                                  (double *)(smem + g.oJcp), (int *)(smem + g.oJdraw), err, st_new);
                h.tame = 0;
            } else {
                int wild = 0;
                nc = expand_node(g, d, t, leaf, pol, bet, 0.f, 0.f, a.K, v_in, cursor, ntot, s.rng, wbase, &s, err, st_new,
                                 have_w, w1r, w2r, stl, wild);
                if (wild || !tame_val(v_in) || !tame_val(r_in)) h.tame = 0;
            }
            stl[MZ_S_EXPANDS] += 1;
            stl[MZ_S_NEW_CHILDREN] += st_new;
            if (!err && l == 0) {
                // the leaf's structure: first child, children count, (maxdepth >= 0 after this
                // simulation's back-propagation), pred_value, hidden_state_index_x
                const int ly = uni(leaf_b.y);
                const int md = md_of(ly) < 0 ? 0 : md_of(ly);
                const int4 nbv = make_int4(tot, pack_y(nc, act_of(ly), md), f2i(v_in), a.hsx);
                s.B[leaf] = nbv;
                d.Bn()[nb + leaf] = nbv;
            }
            if constexpr (SEL && !JOINT && kWalkPrecomputed<NC>) {
                // while the other wave back-propagates: the selection's internal-node list (children
                // counts do not change in the back-propagation; this simulation's new children are
                // leaves, so nodes [0, tot) with the leaf's record just written)
                if (g.K > 1 && !err) {
                    wait_lds();
                    nint_pre = compact_internal(s, tot);
                }
            }
            stamp(ts, 4);
        } else {
            // ---- CTree::back_propagate (cnode.cpp:415-450) + the min/max normaliser ----
            stamp(ts, 4);
#ifndef MZ_ABL_W1SKIP  // ablation (timing experiments only): no back-propagation
            backup(g, d, s, t, h.D, tot, v_in, r_in, a.discount, h, cnt0, n0, nv0, need0, off0, err, stl,
                   (float *)(xst + 2 * MZ_S_COUNT));
#endif
            stamp(ts, 5);
#if defined(MZ_PROBE2) || defined(MZ_PROBE3)
            if (false) {
#else
            if (MZ_STAMPS && SEL) {
#endif
                stl[MZ_S_CYC_W1_ROUND1] += (long long)(ts[1] - ts[0]);
                stl[MZ_S_CYC_W1_STAGE2] += (long long)(ts[3] - ts[2]);
                stl[MZ_S_CYC_W1_BACKUP] += (long long)(ts[5] - ts[4]);
                stl[MZ_S_CYC_W1_SYNC] += (long long)(ts[5] - ts[0]);  // wave 1's whole span
            }
            for (unsigned long long m = ballot(err != 0); m; m &= m - 1ull) err |= rl(err, __builtin_ctzll(m));  // any lane's
            if (l == 0) {
#pragma unroll
                for (int k = 0; k < kStatN; ++k) xst[MZ_S_COUNT + k] = stl[k];  // wave 1's counters
                float *xf = (float *)(xst + 2 * MZ_S_COUNT);
                int *xi = (int *)(xst + 2 * MZ_S_COUNT);
                if (MZ_STAMPS) xst[2 * MZ_S_COUNT + 2] = (long long)ts[0];  // wave 1's start
                (void)xf;  // min / max: written by lane 63 in backup()
                xi[2] = h.mm_cnt;
                xi[3] = err;
            }
        }
        if (JOINT && wv == 1) wait_vm();  // the joint actions staged for the selection
        lds_barrier();  // the waves' global stores stay in flight
        if (wv == 1) {
            wait_vm();  // nothing of wave 1 may be in flight when the block ends
            return;
        }
        // wave 0: merge wave 1's results
        {
            const float *xf = (const float *)(xst + 2 * MZ_S_COUNT);
            const int *xi = (const int *)(xst + 2 * MZ_S_COUNT);
            // diagnostic builds: how much later than wave 0 wave 1 started (in the 'minmax' slot)
            if (MZ_STAMPS && SEL) stl[MZ_S_CYC_MINMAX] += xst[2 * MZ_S_COUNT + 2] - (long long)ts[0];
            const float omn = h.mm_min, omx = h.mm_max;
            const int ocnt = h.mm_cnt;
            h.mm_min = unif(xf[0]);
            h.mm_max = unif(xf[1]);
            h.mm_cnt = uni(xi[2]);
            err |= uni(xi[3]);
            if (h.mm_cnt > 0 && (ocnt == 0 || f2i(h.mm_min) != f2i(omn) || f2i(h.mm_max) != f2i(omx)))
                stl[MZ_S_MM_MOVED] += 1;
        }
        if (!err) {
            h.cursor = cursor;
            h.tot = ntot;
        }
    } else {
        if (wv == 1) wait_vm();
        __syncthreads();  // wave 1 staged the node records the selection reads
        if (wv == 1) return;
    }
    stamp(ts, 5);
    if (!EB || JOINT) wait_vm();  // RNG window (and anything staged) has landed (expand_node waited)
    stamp(ts, 6);
    if (SEL && !err) {
#ifdef MZ_PROBE3
        const unsigned long long v0 = __builtin_amdgcn_s_memtime();
#endif
        // K = 1 chains of a tame tree (TreeHdr::tame) under tame handle constants select without
        // scoring: no score can be NaN or below FLOAT_MIN there (select_walk)
        const bool fast = !JOINT && g.K == 1 && fast_ok && h.tame && fabsf(a.discount) <= 1.0f;
        if (!fast && (g.K == 1 || kWalkPrecomputed<NC>)) value_scores(g, s, h.tot, a.discount, h);
#ifdef MZ_PROBE3
        stl[MZ_S_CYC_EXP_CDF] = (long long)(__builtin_amdgcn_s_memtime() - v0);  // value scores
#endif
        // register RNG window: words h.cursor + [0, 128) (select's words follow the expansion's)
        const unsigned rw0 = fast ? 0u : rng_word_win(s.rng, wbase, h.cursor + l);
        const unsigned rw1 = fast ? 0u : rng_word_win(s.rng, wbase, h.cursor + kWave + l);
        int idx = 0, act = 0;
#ifdef MZ_PROBE3
        wait_vm();
        wait_lds();
        asm volatile("" ::"v"(rw0), "v"(rw1));
        stl[MZ_S_CYC_EXP_DRAW] = (long long)(__builtin_amdgcn_s_memtime() - v0);  // up to the walk
#endif
        select_walk<NC>(g, d, s, t, h.tot, h, wbase, rw0, rw1, err, idx, act, stl, fast, a.discount, nint_pre);
        if (l == 0) {
            a.idx_x[t] = idx;
            a.idy[t] = t;
        }
        if (JOINT) {
            wait_lds();
            if (l < g.N) a.act[(size_t)t * g.N + l] = err ? 0 : (int)sJ[h.leaf * g.N + l];
        } else if (l == 0) {
            a.act[t] = act;
        }
        stamp(ts, 7);
        if (a.pool) {  // mcts_sampled.py:130-134: leaf hidden state = pool[idx_x][t]
            const char *src = a.pool + (long long)idx * a.pool_stride + (long long)t * a.row_bytes;
            char *dst = a.gather_out + (long long)t * a.row_bytes;
            const long long rb = a.row_bytes;
            if (g_pre && idx == a.hsx) {  // prefetched in round 1
                gath_pending = true;
                gdst = dst;
                grb = rb;
            } else if (g_pre_big && idx == a.hsx) {  // staged in LDS in round 1
                gath_lds = true;
                gdst = dst;
                grb = rb;
            } else if (g_big) {
                const long long last = rb - 16, o = (long long)l * 16;
#pragma unroll
                for (int k = 0; k < 16; ++k)
                    glds16(src + (o + 1024 * k < last ? o + 1024 * k : last), sbig + 1024 * k);
                gath_lds = true;
                gdst = dst;
                grb = rb;
            } else if (g_fast) {
                // up to 4 KiB per row: all loads in flight at once, stores after the header write-back
                const long long o = (long long)l * 16;
                if (o < rb) gv0 = *(const int4 *)(src + o);
                if (o + 1024 < rb) gv1 = *(const int4 *)(src + o + 1024);
                if (o + 2048 < rb) gv2 = *(const int4 *)(src + o + 2048);
                if (o + 3072 < rb) gv3 = *(const int4 *)(src + o + 3072);
                gath_pending = true;
                gdst = dst;
                grb = rb;
            } else if (((rb | (long long)(uintptr_t)src | (long long)(uintptr_t)dst) & 15) == 0) {
                for (long long o2 = (long long)l * 16; o2 < rb; o2 += 16 * kWave)
                    *(int4 *)(dst + o2) = *(const int4 *)(src + o2);
            } else {
                for (long long o2 = (long long)l * 4; o2 < rb; o2 += 4 * kWave)
                    *(int *)(dst + o2) = *(const int *)(src + o2);
            }
        }
    } else if (SEL) {
        if (l == 0) {
            a.idx_x[t] = 0;
            a.idy[t] = t;
        }
        if (l < (JOINT ? g.N : 1)) a.act[(size_t)t * (JOINT ? g.N : 1) + l] = 0;
    }
    stamp(ts, 8);
    // header: scalars from lane 0, the next expansion's engine words from lanes 0..kNxt-1
    {
        int perr = 0;
        TreeHdr *hp = d.hdr() + t;
        if (l < kNxt) hp->nxt[l] = rng_word_lane(g, d, s.rng, wbase, t, h.cursor + l, perr);
        if (l == 0) {
            hp->cursor = h.cursor;
            hp->tot = h.tot;
            hp->D = h.D;
            hp->err = err;
            hp->mm_min = h.mm_min;
            hp->mm_max = h.mm_max;
            hp->mm_cnt = h.mm_cnt;
            hp->tame = h.tame;
            hp->leaf = h.leaf;
        }
    }
    if (gath_lds) {
        wait_vm();  // the LDS-DMA chunks have landed
        for (long long o = (long long)l * 16; o < grb; o += 16 * kWave)
            *(int4 *)(gdst + o) = *(const int4 *)(sbig + o);
    }
    if (gath_pending) {
        const long long o = (long long)l * 16;
        if (o < grb) *(int4 *)(gdst + o) = gv0;
        if (o + 1024 < grb) *(int4 *)(gdst + o + 1024) = gv1;
        if (o + 2048 < grb) *(int4 *)(gdst + o + 2048) = gv2;
        if (o + 3072 < grb) *(int4 *)(gdst + o + 3072) = gv3;
    }
    stamp(ts, 9);
#ifdef MZ_PROBE
    if (EB && SEL && !err) {
        stl[MZ_S_CYC_W1_ROUND1] = (long long)(pr0 - ts[0]);   // kernel start -> first loads issued
        stl[MZ_S_CYC_W1_STAGE2] = (long long)(pr1 - pr0);     // T table issue
        stl[MZ_S_CYC_W1_BACKUP] = (long long)(pr2 - pr1);     // inputs + header issue
        stl[MZ_S_CYC_W1_SYNC] = (long long)(ts[1] - pr2);     // wait for round 1
    }
#endif
#ifdef MZ_PROBE2
    if (EB && SEL && !err) {
        unsigned long long pt1;
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(pt1)::"memory");
        stl[MZ_S_CYC_W1_ROUND1] = (long long)(ts[0] - pt0);  // kernel entry -> first stamp
        stl[MZ_S_CYC_W1_STAGE2] = (long long)(pt1 - pt0);    // whole wave-0 span incl. store drain
        stl[MZ_S_CYC_W1_BACKUP] = (long long)(pt1 - ts[9]);  // store drain after the last stamp
        stl[MZ_S_CYC_W1_SYNC] = 0;
    }
#endif
    if (MZ_STAMPS && EB && SEL && !err) {
        // wave 0's timeline: header, stage1, stage2, expand, wait for the back-propagation wave,
        // value-set/RNG wait, select(+outputs), gather, epilogue
        for (int k = 0; k < 9; ++k) stl[MZ_S_CYC_HEADER + k] += (long long)(ts[k + 1] - ts[k]);
        stl[MZ_S_STAMPED] += 1;
    }
    // per-tree statistics: wave 0's counters through LDS (lane 0 writes, lane k reads counter k),
    // plus wave 1's when it back-propagated
    if (l == 0) {
#pragma unroll
        for (int k = 0; k < kStatN; ++k) xst[k] = stl[k];
    }
    wait_lds();
    if (l < kStatN) st[l] = st_old + xst[l] + (EB ? xst[MZ_S_COUNT + l] : 0ll);
    if (l == 0 && err) atomicOr(d.err(), err);
#ifdef MZ_ARGCHECK
    if (l == 0 && err)
        argcheck_record(2 + wv, EB, SEL, t, base, P, PS, BA, pk, K, hsx, discount, pe, ne, d.hdr() + t, h.tot,
                        h.cursor, h.D, 0, (const unsigned *)__builtin_amdgcn_kernarg_segment_ptr(), reward, value, pool,
                        err);
#endif
}

// ================================================================================================
// K = 1 trees: the fused simulation step as a chain kernel
// ================================================================================================
// With sampled_times = 1 every expansion creates exactly one child, so a tree is a chain: node i
// sits at depth i, the leaf is the newest node and every selection walks the whole chain down to
// the child the last expansion created (cnode.cpp:381-413 with one child per node).  Before the
// fused launch of simulation s (hsx = s + 1) the tree holds nodes 0..hsx, the leaf is node hsx and
// the back-propagation path is 0..hsx: every address a launch touches follows from its arguments,
// so both waves issue all their loads at launch and only check the header when it arrives (a
// graph replayed out of sequence falls back to the header's values).
//
// The work splits differently from k_step:
//  - wave 1 computes only the bootstrap recurrence b_{i-1} = r_i + discount * b_i (cnode.cpp:
//    424,448), the one serial chain of the step, and hands the values over through LDS;
//  - wave 0 expands the leaf meanwhile (one draw), then updates every node of the chain
//    (SubTreeValueSet::update appends to an empty depth class: utils.cpp:20-71 with count 0),
//    recomputes the min/max normaliser over the chain's q values, and selects.  On a tame tree
//    (select_walk's fast case) the selection is known without scoring: the new child, one engine
//    word per level, and its parent's hidden_state_index_x is this launch's hsx.
// One barrier per launch.  What K = 1 trees never read again is not written: value-set entries
// (every update appends to an empty depth class), q of interior nodes (every back-propagation
// recomputes all of them), maxdepth, parents, and the readback record D of non-root children.
// --------------------------------------------------------------------------------------------
template <int NC>  // node capacity class (P = S + 2 <= NC); 0: offsets from P at run time
struct ChainLayout {
    int oA, oC, oPP, oLp, oR, oBoot, oW, oP, oPol, oLb, oSt, total;
    __host__ __device__ static constexpr int r16(int x) { return (x + 15) & ~15; }
    __host__ __device__ constexpr ChainLayout(int P)
        : oA(0),
          oC(r16(16 * P)),
          oPP(oC + r16(16 * P)),
          oLp(oPP + r16(4 * P)),
          oR(oLp + r16(4 * (P + 1 + kWave))),
          oBoot(oR + r16(4 * (P + kWave))),
          oW(oBoot + r16(4 * (P + kWave))),
          oP(oW + r16(4 * kMaxActions)),
          oPol(oP + r16(8 * kMaxActions)),
          oLb(oPol + r16(4 * kMaxActions)),
          oSt(oLb + 16),
          total(oSt + r16(8 * kWave)) {}
};
template <int NC>
__device__ __forceinline__ ChainLayout<NC> chain_layout(int P) {
    if constexpr (NC > 0) {
        constexpr ChainLayout<NC> L(NC);
        return L;
    } else {
        return ChainLayout<NC>(P);
    }
}
int chain_lds_bytes(int P, int nc) { return ChainLayout<0>(nc > 0 ? nc : P).total; }

// n dwords global -> LDS by LDS-DMA (asm, uncounted by the compiler): 16-byte chunks when src and dst
// are 16-byte aligned (a quarter of the instructions; up to 3 dwords past n are read and written:
// callers' arrays are padded), else dwords
__device__ __forceinline__ void dma_dwords(const void *src, unsigned lds, int n, bool al16) {
    const int l = lane_id();
    if (al16) {
        const int n4 = (n + 3) >> 2;
        for (int c = 0; c < n4; c += kWave)
            if (c + l < n4)
                asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"((const int4 *)src + c + l),
                             "s"(lds + 16u * c)
                             : "memory", "m0");
    } else {
        for (int c = 0; c < n; c += kWave)
            if (c + l < n)
                asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"((const int *)src + c + l),
                             "s"(lds + 4u * c)
                             : "memory", "m0");
    }
}
__device__ __forceinline__ unsigned lds_addr(const void *p) { return (unsigned)(uintptr_t)(lds_void *)p; }

// A wave-uniform load through the scalar cache (s_load: counted by lgkmcnt, not vmcnt)
__device__ __forceinline__ float ldsc(const float *p) {
    return *(const __attribute__((address_space(4))) float *)p;
}
typedef float f32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ldsc4(const float4 *p) {  // (one s_load_dwordx4)
    const f32x4v v = *(const __attribute__((address_space(4))) f32x4v *)p;
    return make_float4(v.x, v.y, v.z, v.w);
}

template <int NC, bool SEL = true>  // SEL = false: the last expansion of a search (mz_expand_backup)
__global__ __launch_bounds__(128) void k_chain(char *base, const float *policy, const float *beta, int P, int PS,
                                               int BA, int pk, int hsx, int K, float discount, int fast_ok,
                                               const float *reward, const float *value, const char *pool,
                                               long long pool_stride, long long row_bytes, char *gather_out,
                                               int *idx_x, int *idy, int *act) {
    (void)pk;
    (void)K;
    const int B = BA & 0xffffff, A = (int)((unsigned)BA >> 24);
    Dev d;
    d.base = (gchar *)base;
    arena_hot(d, B, P, PS);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const ChainLayout<NC> L = chain_layout<NC>(P);
    unsigned char *sbig = smem + L.total;  // leaf rows above 4 KiB (LDS-DMA staging, 16 KiB)
    int4 *sA = (int4 *)(smem + L.oA);
    float4 *sC = (float4 *)(smem + L.oC);
    float *sPP = (float *)(smem + L.oPP);
    float *sLp = (float *)(smem + L.oLp);
    float *sR = (float *)(smem + L.oR);
    float *sBoot = (float *)(smem + L.oBoot);
    const int t = blockIdx.x;
    const int l = threadIdx.x & (kWave - 1);
    const int wv = uni((int)(threadIdx.x >> 6));
    const size_t nb = (size_t)t * P;
    unsigned long long ts[8] = {0};
    stamp(ts, 0);
    const unsigned long long rt0 = span_open();
    // ---- round 1: everything, from the arguments (the chain's length is hsx) ----
    // the header, the leaf's structure record and the handle's constants (scalar loads from the
    // preloaded arena base, issued first; the network outputs follow the LDS-DMA below)
    TreeHdr h;
    {
        const cTreeHdr *hp = (const cTreeHdr *)(d.hdr() + t);
        h.cursor = hp->cursor;
        h.tot = hp->tot;
        h.D = hp->D;
        h.err = hp->err;
        h.tame = hp->tame;
        h.leaf = hp->leaf;
        h.nxt[0] = hp->nxt[0];
        h.nxt[1] = hp->nxt[1];
    }
    // the root's visit count before this back-propagation (wave 0's selection; wave 1 owns sA)
    const int root_vis0 = *(const __attribute__((address_space(4))) int *)&d.A()[nb].x;
    const cParams *pl = (const cParams *)__builtin_assume_aligned(base, 256);
    const int gW = pl->g.W;
    const float omr = pl->g.one_minus_rho;
    const unsigned oR = pl->d.o_R;
    d.o_D = pl->d.o_D;
    int Dp = hsx;  // back-propagation path 0..Dp, leaf Dp, tot = Dp + 1
    if (Dp < 0 || Dp + 1 > P) Dp = 0;
    float pol = 0.f, bet = 0.f;
    unsigned long long st_old = 0;
    long long *st = d.stats() + (size_t)t * MZ_S_COUNT;
    int4 leaf_b = make_int4(0, 0, 0, 0);
    // the next leaf's parent is this launch's leaf (hidden_state_index_x = hsx): its row is
    // fetched now and stored at the end (four 16-byte chunks per lane up to 4 KiB, LDS-DMA above)
    bool row_al = false, g_reg = false, g_lds = false;
    int4 gv0 = make_int4(0, 0, 0, 0), gv1 = gv0, gv2 = gv0, gv3 = gv0;
    // Round 1 is LDS-DMA and scalar loads (invisible to the compiler's wait counting) plus, last,
    // the leaf row's loads: the counted wait below leaves exactly those in flight until the end.
    float *sPol = (float *)(smem + L.oPol);
    float *sW = (float *)(smem + L.oW);
    long long *sSt = (long long *)(smem + L.oSt);
    if (wv == 0) {
        const size_t ib = (size_t)t * A + (l < A ? l : 0);
        glds4a(policy + ib, sPol);
        glds4a(beta + ib, sW);  // (lanes >= A: zero weights, below)
        glds4a((const int *)st + (l < 2 * MZ_S_COUNT ? l : 0), (int *)sSt);
        if (l == 0) glds16a(d.Bn() + nb + Dp, smem + L.oLb);
        // the leaf-row arguments are not preloaded: their kernel-argument load is first waited for
        // here, after the loads above were issued (the asm keeps the compiler from computing the
        // row's class, and so waiting, any earlier)
        unsigned long long pool_u = (unsigned long long)(uintptr_t)pool, out_u = (unsigned long long)(uintptr_t)gather_out;
        asm volatile("" : "+s"(pool_u), "+s"(pool_stride), "+s"(row_bytes), "+s"(out_u));
        pool = (const char *)(const gchar *)(uintptr_t)pool_u;
        gather_out = (char *)(uintptr_t)out_u;
        row_al = SEL && pool && (((row_bytes | pool_stride | (long long)(uintptr_t)pool |
                                   (long long)(uintptr_t)gather_out) & 15) == 0);
        g_reg = row_al && row_bytes <= 4 * 16 * kWave;
        g_lds = row_al && !g_reg && row_bytes <= 16 * 16 * kWave;
        if (g_reg || g_lds) {
            const char *src = pool + (long long)hsx * pool_stride + (long long)t * row_bytes;
            const long long last = row_bytes - 16, o = (long long)l * 16;
            if (g_reg) {  // always four loads (offsets clamped into the row)
                gv0 = *(const int4 *)(src + (o < last ? o : last));
                gv1 = *(const int4 *)(src + (o + 1024 < last ? o + 1024 : last));
                gv2 = *(const int4 *)(src + (o + 2048 < last ? o + 2048 : last));
                gv3 = *(const int4 *)(src + (o + 3072 < last ? o + 3072 : last));
            } else {  // always sixteen chunks
#pragma unroll
                for (int k = 0; k < 16; ++k) glds16a(src + (o + 1024 * k < last ? o + 1024 * k : last), sbig + 1024 * k);
            }
        }
    } else {  // wave 1 back-propagates: the chain's node records
        for (int i0 = 0; i0 <= Dp; i0 += kWave)
            if (i0 + l <= Dp) {
                glds16a(d.A() + nb + i0 + l, sA + i0);
                glds16a(d.C() + nb + i0 + l, sC + i0);
                glds4a(d.PP() + nb + i0 + l, sPP + i0);
                glds4a(d.lp() + i0 + l, sLp + i0);
            }
    }
    const float r_in = ldsc(reward + t), v_in = ldsc(value + t);
    if (wv == 0 && g_reg) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");        // the row stays in flight
    else if (wv == 0 && g_lds) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // (its chunks too)
    else wait_vm();
    if (wv == 0) {
        if (l >= A) sW[l] = 0.f;
        pol = sPol[l < A ? l : 0];
        bet = sW[l < A ? l : 0];
        if (l < ((MZ_STAMPS != 0) ? MZ_S_COUNT : MZ_S_CYC_HEADER)) st_old = (unsigned long long)sSt[l];
        leaf_b = *(const int4 *)(smem + L.oLb);
    }
    stamp(ts, 1);
    if (h.err) {  // a dead tree stays dead (both waves see the same header) and re-reports its error
        if (wv == 0) {
            if (l == 0) {
                if (SEL) {
                    idx_x[t] = 0;
                    idy[t] = t;
                    act[t] = 0;
                }
                atomicOr(d.err(), h.err);
            }
        }
        wait_vm();  // (the row's loads / chunks)
        return;
    }
    // a graph replayed out of sequence: the header's chain, not the arguments' (both waves)
    const int D = h.D;
    if (D != Dp || h.tot != D + 1 || h.leaf != D) {
        if (D + 1 > P || h.tot != D + 1 || h.leaf != D) {  // not a chain: refuse (reported below)
            if (wv == 0 && l == 0) {
                if (SEL) {
                    idx_x[t] = 0;
                    idy[t] = t;
                    act[t] = 0;
                }
                TreeHdr *hp = d.hdr() + t;
                hp->err = kErrPath;
                atomicOr(d.err(), kErrPath);
            }
            wait_vm();
            return;
        }
        if (wv == 1)
            for (int i0 = 0; i0 <= D; i0 += kWave)
                if (i0 + l <= D) {
                    glds16a(d.A() + nb + i0 + l, sA + i0);
                    glds16a(d.C() + nb + i0 + l, sC + i0);
                    glds4a(d.PP() + nb + i0 + l, sPP + i0);
                    glds4a(d.lp() + i0 + l, sLp + i0);
                }
        if (wv == 0 && l == 0) glds16a(d.Bn() + nb + D, smem + L.oLb);
        wait_vm();
        if (wv == 0) leaf_b = *(const int4 *)(smem + L.oLb);
    }

    if (wv == 1) {
        // ---- the bootstrap values b_i, i = D .. 0 (cnode.cpp:424,448), in chunks of 63 levels ----
        float carry = v_in;
        int hi = D;
        const float dv = discount;
        while (true) {
            const int lo = hi > 63 ? hi - 63 : 0;
            const int nl = hi - lo;
            const int lev = hi - 63 + l;
            float rn = 0.f;  // reward of the level above this lane's
            if (lev >= lo && lev < hi) rn = (lev + 1 == D) ? r_in : i2f(sA[lev + 1].w);
            float b = (l == 63) ? carry : 0.f;
            float tmp = (l == 62) ? dv * carry : 0.f;
            boot_dpp(b, tmp, dv, rn, nl);
            if (lev >= lo && lev <= hi) sBoot[lev] = b;
            if (lo == 0) break;
            carry = rlf(b, 63 - nl);
            hi = lo;
        }
        wait_lds();
        stamp(ts, 2);
        // ---- CTree::back_propagate (cnode.cpp:415-450) over the chain, lane i = node i ----
        float mn = INFINITY, mx = -INFINITY;
        for (int i0 = 0; i0 <= D; i0 += kWave) {
            const int i = i0 + l;
            if (i <= D) {
                const int dep = D - i;
                const float key = sBoot[i];
                int4 a4 = sA[i];
                if (i == D) a4.w = f2i(r_in);  // the leaf's reward is this simulation's
                const float4 cw = sC[i];
                const float lp = sLp[dep];
                float ws = cw.x, tw = cw.y;
                tw += lp;  // an empty depth class: big gets the value (utils.cpp:36-44)
                ws += lp * key;
                const float val = ws / tw;  // CNode::value (cnode.cpp:42-56); every chain node has a child
                const int4 na = make_int4(a4.x + 1, a4.y, f2i(val), a4.w);
                sA[i] = na;
                d.A()[nb + i] = na;
                *(float2 *)&d.C()[nb + i] = make_float2(ws, tw);
                if (i >= 1) {
                    const float q = (i2f(a4.w) + discount * val) - sPP[i];  // get_qsa - father->pred_value
                    mn = fminf(mn, q);
                    mx = fmaxf(mx, q);
                }
            }
        }
        // min / max over the q of the visited non-root nodes: the whole chain 1..D
        mn = unif(rlf(wave_min_to63(mn), 63));
        mx = unif(rlf(wave_max_to63(mx), 63));
        if (l == 0) {
            sR[2] = mn;
            sR[3] = mx;
            if (MZ_STAMPS) {
                *(unsigned long long *)(smem + L.oR) = ts[2] - ts[1];  // the bootstrap chain
                *(unsigned long long *)(smem + L.oR + 16) = __builtin_amdgcn_s_memtime() - ts[2];  // node updates
            }
        }
        lds_barrier();
        wait_vm();  // nothing of this wave may be in flight when the block ends
        return;
    }

    // ---- wave 0: CTree::expand (cnode.cpp:224-295) of the leaf: one draw ----
    int err = 0;
    const int leaf = D, c = D + 1;  // the new child
    int cursor = h.cursor;
    int a = 0;
    if (A >= 2) {
        const double cp = cdf_bcast(bet, A, (float *)(smem + L.oW), (double *)(smem + L.oP));
        const double w1 = (double)h.nxt[0], w2 = (double)h.nxt[1];
        double u = (w1 + w2 * 4294967296.0) / 18446744073709551616.0;
        if (u >= 1.0) u = 0x1.fffffffffffffp-1;  // nextafter(1, 0)
        a = __popcll(ballot(l < A && cp < u));    // lower_bound
        cursor += 2;
    }
    a = uni(a);
    stamp(ts, 2);
    if (c + 1 > P) err |= kErrPool;
    const float bh = 1.0f;  // betahat_prob = count / sampled_times = 1 / 1
    const float pol_a = rlf(pol, a), bet_a = rlf(bet, a);
    float prior = pol_a * bh / bet_a;  // prior * betahat_prob / beta_prob (eps = 0 after the root)
    const bool wild = !tame_prior(prior);
    leaf_b = uni4(leaf_b);
    if (!err && l == 0) {
        const size_t gi = nb + c;
        d.A()[gi] = make_int4(0, f2i(prior), f2i(0.0f), f2i(0.0f));
        d.Bn()[gi] = make_int4(0, pack_y(0, a, -1), f2i(0.0f), -1);
        d.C()[gi] = make_float4(0.f, 0.f, 0.f, 0.f);
        d.PP()[gi] = v_in;
        if (leaf == 0) d.D()[gi] = make_float4(pol_a, bet_a, bh, 0.f);  // (readbacks: root children)
        const int md = md_of(leaf_b.y) < 0 ? 0 : md_of(leaf_b.y);
        d.Bn()[nb + leaf] = make_int4(c, pack_y(1, act_of(leaf_b.y), md), f2i(v_in), hsx);
    }
    const int tame = (h.tame && !wild && tame_val(v_in) && tame_val(r_in)) ? 1 : 0;
    const bool fast = !SEL || (fast_ok && tame && fabsf(discount) <= 1.0f);  // (no selection: no words)
    // the selection on a tame tree (select_walk): the new child; one word per level but the
    // forced first one (root visits after this back-propagation = the staged count + 1)
    const int Ds = c;
    int root_visit = 0, words = 0;
    if (SEL && fast) {
        root_visit = root_vis0 + 1;
        if (root_visit - 1 >= PS) err |= kErrTable;
        words = Ds - ((root_visit <= 1) ? 1 : 0);
    }
    if (SEL && Ds + 1 > PS) err |= kErrPath;
    // the next expansion's engine words, for the header (in flight during the back-propagation)
    unsigned nxt_w = 0;
    const unsigned *Rt = (const unsigned *)(base + (size_t)oR * 256) + (size_t)t * gW;
    if (fast && l < kNxt && cursor + words + l < gW) nxt_w = Rt[cursor + words + l];
    if (value_lim(1, omr) != 1) err |= kErrValueSet;  // (count 1: size_lim must be 1, utils.cpp:31)

    stamp(ts, 3);
    lds_barrier();  // wave 1's back-propagation (sA, sPP updated) and min / max
    stamp(ts, 4);
    float mn = unif(sR[2]), mx = unif(sR[3]);  // wave 1's min / max over the q of nodes 1..D
    stamp(ts, 5);
    const int mm_cnt = D;

    if (SEL && !fast && !err) {
        // ---- select_walk's exact case: every level's tie list must be non-empty to consume a
        // word (score >= FLOAT_MIN, not NaN); levels 1..Ds scored in parallel ----
        sA[c] = make_int4(0, f2i(prior), f2i(0.0f), f2i(0.0f));
        wait_lds();
        root_visit = uni(sA[0].x);
        const float gdelta = pl->g.delta;
        const bool mm_on = mm_cnt > 0;
        float den = 0.f;
        if (mm_on) {
            const float delta = mx - mn;
            den = (gdelta < delta) ? delta : gdelta;  // std::max(delta_lb, delta)
        }
        const float *pbt = d.pb();
        const double *sqt = d.sq();
        bool terr = false;
        for (int i0 = 0; i0 <= Ds; i0 += kWave) {
            const int i = i0 + l;
            bool valid = false;
            if (i >= 1 && i <= Ds && !(i == 1 && root_visit <= 1)) {
                const int n = sA[i - 1].x - 1;  // the parent's total_children_visit_counts
                if (n < 0 || n >= PS) {
                    terr = true;
                } else {
                    const int4 ca = sA[i];
                    const float pp = (i == Ds) ? v_in : sPP[i];
                    float vs = (ca.x == 0) ? 0.0f : ((i2f(ca.w) + discount * i2f(ca.z)) - pp);
                    if (mm_on) vs = (vs - mn) / den;
                    if (vs < 0) vs = 0;
                    if (vs > 1) vs = 1;
                    const float pbc = (float)((double)pbt[n] * (sqt[n] / (double)(ca.x + 1)));
                    const float sc = pbc * i2f(ca.y) + vs;
                    valid = sc >= -1000000.0f;  // FLOAT_MIN (utils.h:12)
                }
            }
            words += __popcll(ballot(valid));
        }
        if (ballot(terr)) err |= kErrTable;
        if (!err && l < kNxt && cursor + words + l < gW) nxt_w = Rt[cursor + words + l];
    }

    // ---- outputs (mcts_sampled.py:123-134), the header, the statistics ----
    stamp(ts, 6);
    if (SEL && l == 0) {
        idx_x[t] = err ? 0 : hsx;  // parent->hidden_state_index_x: the expanded leaf's
        idy[t] = t;
        act[t] = err ? 0 : a;
    }
    if (SEL && pool && !err) {
        const char *src = pool + (long long)hsx * pool_stride + (long long)t * row_bytes;
        char *dst = gather_out + (long long)t * row_bytes;
        const long long o = (long long)l * 16;
        if (g_reg) {
            if (o < row_bytes) *(int4 *)(dst + o) = gv0;
            if (o + 1024 < row_bytes) *(int4 *)(dst + o + 1024) = gv1;
            if (o + 2048 < row_bytes) *(int4 *)(dst + o + 2048) = gv2;
            if (o + 3072 < row_bytes) *(int4 *)(dst + o + 3072) = gv3;
        } else if (g_lds) {
            for (long long o2 = o; o2 < row_bytes; o2 += 16 * kWave) *(int4 *)(dst + o2) = *(const int4 *)(sbig + o2);
        } else if (row_al) {
            for (long long o2 = o; o2 < row_bytes; o2 += 16 * kWave) *(int4 *)(dst + o2) = *(const int4 *)(src + o2);
        } else {
            for (long long o2 = (long long)l * 4; o2 < row_bytes; o2 += 4 * kWave)
                *(int *)(dst + o2) = *(const int *)(src + o2);
        }
    }
    {
        TreeHdr *hp = d.hdr() + t;
        if (l < kNxt) hp->nxt[l] = nxt_w;
        if (l == 0) {
            hp->cursor = err ? h.cursor : cursor + words;
            hp->tot = err ? h.tot : c + 1;
            hp->D = (err || !SEL) ? h.D : Ds;
            hp->err = err;
            hp->mm_min = mn;
            hp->mm_max = mx;
            hp->mm_cnt = mm_cnt;
            hp->tame = tame;
            hp->leaf = (err || !SEL) ? h.leaf : c;
        }
    }
    stamp(ts, 7);
    constexpr int kStatN = (MZ_STAMPS != 0) ? MZ_S_COUNT : MZ_S_CYC_HEADER;
    if (l < kStatN) {
        long long add = 0;
        switch (l) {
            case MZ_S_CYC_HEADER: add = (long long)(ts[1] - ts[0]); break;   // round 1
            case MZ_S_CYC_EXP_CDF: add = (long long)(ts[2] - ts[1]); break;  // distribution + draw
            case MZ_S_CYC_EXPAND: add = (long long)(ts[3] - ts[2]); break;   // child, header words
            case MZ_S_CYC_BACKUP: add = (long long)(ts[4] - ts[3]); break;   // wait for the chain
            case MZ_S_CYC_MINMAX: add = (long long)(ts[5] - ts[4]); break;   // min / max read
            case MZ_S_CYC_BAK_NODES: add = MZ_STAMPS ? *(const long long *)(smem + L.oR + 16) : 0; break;  // wave 1
            case MZ_S_CYC_SELECT: add = (long long)(ts[6] - ts[5]); break;   // selection
            case MZ_S_CYC_EPILOGUE: add = (long long)(ts[7] - ts[6]); break; // outputs, header
            case MZ_S_CYC_BAK_BOOT: add = MZ_STAMPS ? *(const long long *)(smem + L.oR) : 0; break;
            case MZ_S_STAMPED: add = 1; break;
            case MZ_S_SELECTS: add = SEL ? 1 : 0; break;
            case MZ_S_PATH_EDGES: add = SEL ? Ds : 0; break;
            case MZ_S_SCORED: add = SEL ? Ds : 0; break;
            case MZ_S_EXPANDS: add = 1; break;
            case MZ_S_NEW_CHILDREN: add = 1; break;
            case MZ_S_BACKUP_NODES: add = D + 1; break;
            case MZ_S_MINMAX_NODES: add = D; break;
            default: break;
        }
        st[l] = (long long)st_old + add;
    }
    if (l == 0 && err) atomicOr(d.err(), err);
    span_close(hsx, rt0);
}

// ================================================================================================
// K = 1 chains, round 3: three wave roles, the bootstrap recurrence in registers
// ================================================================================================
// The same simulation step as k_chain (expansion of the leaf, back-propagation over the chain,
// min/max normaliser, selection of the new child, leaf-row gather), re-split so that nothing but
// the expansion and the back-propagation sits on a launch's critical path:
//  - wave 0 expands the leaf (distribution, draw, the child's records), writes the selection
//    outputs and, after the one barrier, the header;
//  - wave 1 back-propagates.  Its node records arrive in registers (lane i = node i).  The
//    recurrence b_{i-1} = r_i + discount * b_i (cnode.cpp:424,448) runs in registers on every lane
//    at once (all lanes hold the same b), fed by the chain's rewards read from LDS sixteen at a
//    time: one dependent multiply + add per level instead of a DPP lane shift;
//  - wave 2 does what depends only on the header: the leaf-row gather (the next leaf's parent is
//    this launch's leaf), the next expansion's engine words when the selection is known to take
//    one word per level (every prior of the leaf's distribution tame: select_walk's fast case
//    whatever the draw), and the statistics counters.
// Every error and output is decided from the same scalar inputs as k_chain: results are bit-identical.
//
// Launch arguments.  The first 14 dwords arrive preloaded in SGPRs; they hold everything round 1
// addresses (the node arrays lead the arena, so their offsets follow from B and P: arena_nodes).
// The outputs (ChainIO) are read through the kernel-argument
// pointer by the waves that need them, where they need them: the compiler would otherwise load
// every argument in the common prologue and wait there.  Round 1's scalar loads are issued by
// inline assembly (sload*) and waited for with one explicit wait (swait): the compiler would sink
// each load past the first branch after it.
// --------------------------------------------------------------------------------------------
struct ChainIO {
    const char *pool;
    long long pool_stride, row_bytes;
    char *gather_out;
    int *idx_x, *idy, *act;
};
struct Chain3Args {  // k_chain3's parameter list, for the kernel-argument offset of ChainIO
    char *base;
    const float *policy, *beta, *reward, *value;
    int ppk, bak, hsx;
    float discount;
    const char *src_slot;
    ChainIO io;
};
// (the first 16 dwords, through src_slot, arrive preloaded in SGPRs)
static_assert(offsetof(Chain3Args, src_slot) == 56 && offsetof(Chain3Args, io) == 64 && sizeof(ChainIO) == 56,
              "k_chain3 argument layout");
#ifdef __HIP_DEVICE_COMPILE__
typedef const __attribute__((address_space(4))) ChainIO cChainIO;
#else
typedef const ChainIO cChainIO;
#endif

typedef int int4v __attribute__((ext_vector_type(4)));
typedef int int8v __attribute__((ext_vector_type(8)));
typedef int int16v __attribute__((ext_vector_type(16)));
// scalar loads issued here and waited for by swait (invisible to the compiler's wait counting, which
// stays correct: its own LDS waits only ever wait longer with more loads outstanding)
__device__ __forceinline__ int sload1(const void *p) {
    int v;
    asm volatile("s_load_dword %0, %1, 0x0" : "=s"(v) : "s"(p) : "memory");
    return v;
}
typedef int int2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int2v sload2(const void *p) {
    int2v v;
    asm volatile("s_load_dwordx2 %0, %1, 0x0" : "=s"(v) : "s"(p) : "memory");
    return v;
}
__device__ __forceinline__ uintptr_t u64_of(int lo, int hi) {
    return (uintptr_t)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ int4v sload4(const void *p) {
    int4v v;
    asm volatile("s_load_dwordx4 %0, %1, 0x0" : "=s"(v) : "s"(p) : "memory");
    return v;
}
__device__ __forceinline__ int8v sload8(const void *p) {
    int8v v;
    asm volatile("s_load_dwordx8 %0, %1, 0x0" : "=s"(v) : "s"(p) : "memory");
    return v;
}
__device__ __forceinline__ int16v sload16(const void *p) {
    int16v v;
    asm volatile("s_load_dwordx16 %0, %1, 0x0" : "=s"(v) : "s"(p) : "memory");
    return v;
}

template <int NC>
struct Chain3Layout {
    int oW, oP, oRv, oBv, oA, oPP, oX, total;
    __host__ __device__ static constexpr int r16(int x) { return (x + 15) & ~15; }
    __host__ __device__ constexpr Chain3Layout(int P)
        : oW(0),                         // float[64]  the leaf's weights (distribution broadcast)
          oP(4 * kWave),                 // double[64] its probabilities
          oRv(oP + 8 * kWave),           // float[P + 32]  rewards reversed: [j] = r_{D-j}
          oBv(oRv + r16(4 * (P + 32))),  // float[P + 32]  bootstrap values: [j] = b_{D-1-j}
          oA(oBv + r16(4 * (P + 32))),   // int4[P + 1]    node records after the back-propagation
          oPP(oA + r16(16 * (P + 1))),   // float[P + 1]   parents' pred_value
          oX(oPP + r16(4 * (P + 1))),    // min, max, wave 2's flag, v_in; stamps from 64
          total(oX + 128) {}
};
int chain3_lds_bytes(int nc) { return Chain3Layout<0>(nc).total; }

// ROW: the leaf-row gather's class -- 0 any row, 1 16-byte aligned rows of <= 4 KiB (registers), 2
// aligned rows of <= 16 KiB (LDS-DMA), 3 no gather (no pool, or no selection).  For ROW 1 and 2 the
// host passes the leaf's slot (pool + hsx * pool_stride) in the preloaded argument src_slot and the
// row size in 16-byte units in ppk's top bits: wave 2 issues the row's loads at its first instruction.
template <int NC, bool SEL, int ROW>
__global__ __launch_bounds__(192) void k_chain3(char *base, const float *policy, const float *beta, const float *reward,
                                                const float *value, int ppk, int bak, int hsx, float discount,
                                                const char *src_slot, ChainIO io) {
    static_assert(NC >= kWave && NC % kWave == 0 && NC < 1024, "k_chain3 node classes are whole waves, < 1024");
    (void)io;  // (read through the kernel-argument pointer, see above)
    constexpr int NCH = NC / kWave;  // node chunks of one wave
    constexpr Chain3Layout<NC> L(NC);
    const int P = ppk & 0x3ff, PS = (ppk >> 10) & 0x3ff;
    const int A = (bak >> 24) & 0x7f, fast_ok = (int)((unsigned)bak >> 31);
    const int B = bak & 0xffffff;
    Dev d;
    d.base = (gchar *)base;
    arena_nodes(d, B, P);
    cChainIO *iop = (cChainIO *)((const char *)__builtin_amdgcn_kernarg_segment_ptr() + offsetof(Chain3Args, io));
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float *sX = (float *)(smem + L.oX);
    int *sXi = (int *)(smem + L.oX);
    long long *sXl = (long long *)(smem + L.oX + 64);
    int4 *sA = (int4 *)(smem + L.oA);
    float *sPP = (float *)(smem + L.oPP);
    float *sRv = (float *)(smem + L.oRv);
    float *sBv = (float *)(smem + L.oBv);
    const int t = blockIdx.x;
    const int l = threadIdx.x & (kWave - 1);
    const int wv = uni((int)(threadIdx.x >> 6));
    const size_t nb = (size_t)t * P;
    unsigned long long ts[8] = {0};
    stamp(ts, 0);
    const unsigned long long rt0 = span_open();
    TreeHdr *hp = d.hdr() + t;
    const cParams *pl = (const cParams *)__builtin_assume_aligned(base, 256);
    const int Dp = (hsx >= 0 && hsx + 1 <= P) ? hsx : 0;  // the chain's leaf, if the header agrees

    if (wv == 1) {
        // ======== wave 1: CTree::back_propagate (cnode.cpp:415-450) over the chain ========
        int8v hv = sload8(hp);  // cursor, tot, D, err, mm_min, mm_max, mm_cnt, leaf
        int r_i = sload1(reward + t), v_i = sload1(value + t);
        int o_lp = sload1(&pl->d.o_lp);
        int4 a4[NCH];
        float2 cw[NCH];
        float pp[NCH], lpv[NCH];
        auto load = [&](int D, const float *lp) {
#pragma unroll
            for (int c = 0; c < NCH; ++c) {
                const int i = c * kWave + l;
                a4[c] = make_int4(0, 0, 0, 0);
                cw[c] = make_float2(0.f, 0.f);
                pp[c] = 0.f;
                lpv[c] = 0.f;
                if (i <= D) {
                    a4[c] = d.A()[nb + i];
                    cw[c] = *(const float2 *)&d.C()[nb + i];
                    pp[c] = d.PP()[nb + i];
                    lpv[c] = lp[D - i];  // lambda^(D - i): this back-propagation's depth at node i
                }
            }
        };
        // (lp's offset arrives with the header: the node records go first)
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const int i = c * kWave + l;
            a4[c] = make_int4(0, 0, 0, 0);
            cw[c] = make_float2(0.f, 0.f);
            pp[c] = 0.f;
            if (i <= Dp) {
                a4[c] = d.A()[nb + i];
                cw[c] = *(const float2 *)&d.C()[nb + i];
                pp[c] = d.PP()[nb + i];
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(hv), "+s"(r_i), "+s"(v_i), "+s"(o_lp)::"memory");
        const float *lpt = (const float *)(base + (size_t)(unsigned)o_lp * 256);
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const int i = c * kWave + l;
            lpv[c] = (i <= Dp) ? lpt[Dp - i] : 0.f;
        }
        const float r_in = i2f(r_i), v_in = i2f(v_i);
        const int herr = hv[3], D = hv[2], toth = hv[1], leafh = hv[7];
        if (herr) return;  // (wave 0 reports; no wave takes the barrier on the error paths)
        if (D != Dp || toth != D + 1 || leafh != D) {
            if (D + 1 > P || toth != D + 1 || leafh != D) return;  // not a chain (wave 0 reports)
            load(D, lpt);  // a graph replayed out of sequence: the header's chain
        }
        const float g = discount;
        // the chain's rewards, reversed: sRv[j] = r_{D-j} (r_D = this simulation's reward)
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const int i = c * kWave + l;
            if (i >= 1 && i <= D) sRv[D - i] = (i == D) ? r_in : i2f(a4[c].w);
        }
        wait_lds();
        stamp(ts, 1);
        // b_{D-1-j} = r_{D-j} + discount * b_{D-j}, j = 0 .. D-1, sixteen levels per LDS round
        // (the next sixteen rewards are read while these run; levels past the root compute values
        // nobody reads: sRv / sBv are padded)
        {
            float b = v_in;
            float4 n0 = *(const float4 *)(sRv), n1 = *(const float4 *)(sRv + 4), n2 = *(const float4 *)(sRv + 8),
                   n3 = *(const float4 *)(sRv + 12);
            for (int j0 = 0; j0 < D; j0 += 16) {
                const float4 c0 = n0, c1 = n1, c2 = n2, c3 = n3;
                n0 = *(const float4 *)(sRv + j0 + 16);
                n1 = *(const float4 *)(sRv + j0 + 20);
                n2 = *(const float4 *)(sRv + j0 + 24);
                n3 = *(const float4 *)(sRv + j0 + 28);
                float4 o0, o1, o2, o3;
                b = c0.x + g * b; o0.x = b;
                b = c0.y + g * b; o0.y = b;
                b = c0.z + g * b; o0.z = b;
                b = c0.w + g * b; o0.w = b;
                b = c1.x + g * b; o1.x = b;
                b = c1.y + g * b; o1.y = b;
                b = c1.z + g * b; o1.z = b;
                b = c1.w + g * b; o1.w = b;
                b = c2.x + g * b; o2.x = b;
                b = c2.y + g * b; o2.y = b;
                b = c2.z + g * b; o2.z = b;
                b = c2.w + g * b; o2.w = b;
                b = c3.x + g * b; o3.x = b;
                b = c3.y + g * b; o3.y = b;
                b = c3.z + g * b; o3.z = b;
                b = c3.w + g * b; o3.w = b;
                *(float4 *)(sBv + j0) = o0;
                *(float4 *)(sBv + j0 + 4) = o1;
                *(float4 *)(sBv + j0 + 8) = o2;
                *(float4 *)(sBv + j0 + 12) = o3;
            }
        }
        wait_lds();
        stamp(ts, 2);
        // ---- every node of the chain, lane i = node i: visits, value set (an append to an empty
        // depth class, utils.cpp:36-44), value (cnode.cpp:42-56); min / max over the q of 1..D ----
        float mn = INFINITY, mx = -INFINITY;
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const int i = c * kWave + l;
            if (i <= D) {
                const float key = (i == D) ? v_in : sBv[D - 1 - i];
                const float rw = (i == D) ? r_in : i2f(a4[c].w);  // the leaf's reward is this simulation's
                const float tw = cw[c].y + lpv[c];
                const float ws = cw[c].x + lpv[c] * key;
                const float val = ws / tw;
                const int4 na = make_int4(a4[c].x + 1, a4[c].y, f2i(val), f2i(rw));
                d.A()[nb + i] = na;
                *(float2 *)&d.C()[nb + i] = make_float2(ws, tw);
                sA[i] = na;
                sPP[i] = pp[c];
                if (i >= 1) {
                    const float q = (rw + g * val) - pp[c];  // get_qsa - father->pred_value
                    mn = fminf(mn, q);
                    mx = fmaxf(mx, q);
                }
            }
        }
        mn = unif(rlf(wave_min_to63(mn), 63));
        mx = unif(rlf(wave_max_to63(mx), 63));
        if (l == 0) {
            sX[0] = mn;
            sX[1] = mx;
            // (the header's normaliser is this wave's: wave 0 skips the barrier in select_walk's
            // fast case and writes the rest of the header)
            hp->mm_min = mn;
            hp->mm_max = mx;
            if (MZ_STAMPS) {
                sXl[0] = (long long)(ts[2] - ts[1]);                         // the recurrence
                sXl[1] = (long long)(__builtin_amdgcn_s_memtime() - ts[2]);  // node updates
                sXl[2] = (long long)(ts[1] - ts[0]);                         // round 1
            }
        }
        // no barrier: this wave's LDS writes are done when it ends, and a wave that has ended no longer
        // counts at s_barrier, so wave 0's barrier (the exact case, the fused readback) completes once
        // this wave has ended.  (With a barrier here this wave sat in it until wave 0 ended -- in the
        // fast case wave 0 takes none -- and the MZ_SPANS build recorded it as the launch's last wave,
        // 0.17 us after wave 0; without it the spans period is 3.20 -> 2.98 us, but the product's
        // launch is unchanged, 3.10 us: wave 0 ends last either way, profiles/round6/ab)
        wait_lds();
        span_end(hsx, 1);
        return;
    }

    if (wv == 2) {
        // ======== wave 2: the leaf-row gather and the counters ========
        // Straight-line code in issue order (the row class ROW is a template argument): every wait
        // the compiler places then counts exactly the loads issued after the one it needs.
        // The row of this launch's leaf (hidden_state_index_x = hsx) is issued first, from preloaded
        // arguments only (ROW 1, 2); then one scalar round trip: the outputs' kernel arguments, the
        // header, the handle's constants.  This wave takes no barrier: nothing it does is read by
        // another wave, and s_barrier waits only for the workgroup's waves that have not ended.
        const long long o = (long long)l * 16;
        unsigned char *sbig = smem + L.total;  // (ROW 2: 16 KiB past the layout)
        int4 gv0 = make_int4(0, 0, 0, 0), gv1 = gv0, gv2 = gv0, gv3 = gv0;
        if constexpr (ROW == 1 || ROW == 2) {
            const long long rb = (long long)((unsigned)ppk >> 20) * 16, lst = rb - 16;
            const char *srow = (const char *)(const gchar *)src_slot + (long long)t * rb;
            if constexpr (ROW == 1) {  // up to 4 KiB: four 16-byte registers per lane, offsets clamped into the row
                gv0 = *(const int4 *)(srow + (o < lst ? o : lst));
                gv1 = *(const int4 *)(srow + (o + 1024 < lst ? o + 1024 : lst));
                gv2 = *(const int4 *)(srow + (o + 2048 < lst ? o + 2048 : lst));
                gv3 = *(const int4 *)(srow + (o + 3072 < lst ? o + 3072 : lst));
            } else {  // up to 16 KiB: sixteen LDS-DMA chunks of 1 KiB
#pragma unroll
                for (int k = 0; k < 16; ++k) glds16a(srow + (o + 1024 * k < lst ? o + 1024 * k : lst), sbig + 1024 * k);
            }
        }
        int8v io8 = sload8((const void *)iop);  // pool, pool_stride, row_bytes, gather_out
        int8v hv = sload8(hp);                  // cursor, tot, D, err, mm_min, mm_max, mm_cnt, leaf
        int rv0 = sload1(&d.A()[nb].x), omri = sload1(&pl->g.one_minus_rho), osti = sload1(&pl->d.o_stats);
        asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(io8), "+s"(hv), "+s"(rv0), "+s"(omri), "+s"(osti) : : "memory");
        stamp(ts, 1);
        // (typed as global memory: flat accesses would count against lgkmcnt too)
        const char *pool = (const char *)(const gchar *)u64_of(io8[0], io8[1]);
        const long long pool_stride = (long long)u64_of(io8[2], io8[3]);
        const long long row_bytes = (long long)u64_of(io8[4], io8[5]);
        char *gather_out = (char *)(gchar *)u64_of(io8[6], io8[7]);
        const int toth = hv[1], D = hv[2], herr = hv[3], leafh = hv[7];
        const int root_vis0 = rv0;
        const float omr = i2f(omri);
        const char *src = pool + (long long)hsx * pool_stride + (long long)t * row_bytes;  // (ROW 0)
        d.o_stats = (unsigned)osti;
        long long *st = d.stats() + (size_t)t * MZ_S_COUNT;
        const long long st_old = st[l < MZ_S_CYC_HEADER ? l : 0];
        // a dead or inconsistent tree: wave 0 reports; no wave takes the barrier on these paths (all
        // three read the same header)
        if (herr || D + 1 > P || toth != D + 1 || leafh != D) {
            wait_vm();  // (no LDS-DMA may land after the workgroup ends)
            return;
        }
        const int c = D + 1, Ds = c;
        int err = (c + 1 > P) ? kErrPool : 0;
        if (value_lim(1, omr) != 1) err |= kErrValueSet;
        if (SEL && Ds + 1 > PS) err |= kErrPath;
        if (SEL && !err && root_vis0 >= PS) err |= kErrTable;  // the root's child visits index the pUCT table
        stamp(ts, 2);
        stamp(ts, 3);
        stamp(ts, 4);
        if (SEL && ROW != 3 && !err) {
            char *dst = gather_out + (long long)t * row_bytes;
            if constexpr (ROW == 1) {
                // written through (sc0 sc1): the rows are most of this launch's stores, and lines
                // left dirty in L2 are written back at the kernel boundary (same-box A/B: 3m env
                // step 0.4743 -> 0.4679 ms, 2s3z 1.110 -> 1.080; k_tree's 3m row measured 0.5 %
                // slower this way)
                if (o < row_bytes) st_wt16(dst + o, gv0);
                if (o + 1024 < row_bytes) st_wt16(dst + o + 1024, gv1);
                if (o + 2048 < row_bytes) st_wt16(dst + o + 2048, gv2);
                if (o + 3072 < row_bytes) st_wt16(dst + o + 3072, gv3);
            } else if constexpr (ROW == 2) {
                wait_vm();
                // (written through as well: 27m's 13.5 KiB rows, env step 26.42 -> 24.53 ms)
                for (long long o2 = o; o2 < row_bytes; o2 += 16 * kWave) st_wt16(dst + o2, *(const int4 *)(sbig + o2));
            } else {  // any other row: 16-byte copies when aligned, else 4-byte
                if (((row_bytes | pool_stride | (long long)(uintptr_t)pool | (long long)(uintptr_t)gather_out) & 15) == 0) {
                    for (long long o2 = o; o2 < row_bytes; o2 += 16 * kWave) *(int4 *)(dst + o2) = *(const int4 *)(src + o2);
                } else {
                    for (long long o2 = (long long)l * 4; o2 < row_bytes; o2 += 4 * kWave)
                        *(int *)(dst + o2) = *(const int *)(src + o2);
                }
            }
        }
        stamp(ts, 5);
        if (MZ_STAMPS && l == 0) {  // (wave 2's phases, stamped builds: slots wave 0 leaves alone)
            st[MZ_S_CYC_STAGE1] += (long long)(ts[1] - ts[0]);  // scalar round trip
            st[MZ_S_CYC_STAGE2] += (long long)(ts[2] - ts[0]);  // header checks done
            st[MZ_S_CYC_GATHER] += (long long)(ts[4] - ts[0]);  // (the same point: no barrier)
            st[MZ_S_CYC_W1_STAGE2] += (long long)(ts[5] - ts[0]);  // row stored
        }
        if (l < MZ_S_CYC_HEADER) {
            long long add = 0;
            switch (l) {
                case MZ_S_SELECTS: add = SEL ? 1 : 0; break;
                case MZ_S_PATH_EDGES: add = SEL ? Ds : 0; break;
                case MZ_S_SCORED: add = SEL ? Ds : 0; break;
                case MZ_S_EXPANDS: add = 1; break;
                case MZ_S_NEW_CHILDREN: add = 1; break;
                case MZ_S_BACKUP_NODES: add = D + 1; break;
                case MZ_S_MINMAX_NODES: add = D; break;
                default: break;
            }
            st[l] = st_old + add;
        }
        if constexpr (ROW == 2) wait_vm();
        span_end(hsx, 2);
        return;
    }

    // ======== wave 0: CTree::expand (cnode.cpp:224-295) of the leaf: one draw ========
    int16v hv = sload16(hp);  // cursor, tot, D, err, mm_min, mm_max, mm_cnt, leaf, tame, nxt[0 .. 6]
    int root_vis0 = sload1(&d.A()[nb].x);
    int r_i = sload1(reward + t), v_i = sload1(value + t);
    int4v lb = sload4(&d.Bn()[nb + Dp]);
    int4v io_xy = sload4((const char *)iop + offsetof(ChainIO, idx_x));  // idx_x, idy
    int2v io_a = sload2((const char *)iop + offsetof(ChainIO, act));
    int omri = sload1(&pl->g.one_minus_rho), gWi = sload1(&pl->g.W), oRi = sload1(&pl->d.o_R);
    const float pol = policy[(size_t)t * A + (l < A ? l : 0)];
    const float bet = beta[(size_t)t * A + (l < A ? l : 0)];
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+s"(hv), "+s"(root_vis0), "+s"(r_i), "+s"(v_i), "+s"(lb), "+s"(io_xy), "+s"(io_a), "+s"(omri),
                   "+s"(gWi), "+s"(oRi)
                 :
                 : "memory");
    // The next expansion's engine words (the header's nxt), read now for select_walk's fast case --
    // one word per level below the root (its first level is forced while it has one visit): they
    // land while the distribution is built.  The exact case re-reads them after the barrier.
    const int gW = gWi;
    const unsigned *Rt = (const unsigned *)(base + (size_t)(unsigned)oRi * 256) + (size_t)t * gW;
    const int dA = (A >= 2) ? 2 : 0;
    const int words_fast = SEL ? (hv[2] + 1) - ((root_vis0 + 1 <= 1) ? 1 : 0) : 0;
    const int wi = hv[0] + dA + words_fast + l;
    const unsigned w_fast = Rt[(wi >= 0 && wi < gW) ? wi : 0];
    const float r_in = i2f(r_i), v_in = i2f(v_i);
    int *const idx_x = (int *)(gchar *)u64_of(io_xy[0], io_xy[1]), *const idy = (int *)(gchar *)u64_of(io_xy[2], io_xy[3]);
    int *const act = (int *)(gchar *)u64_of(io_a[0], io_a[1]);
    int4 leaf_b = make_int4(lb.x, lb.y, lb.z, lb.w);
    TreeHdr h;
    h.cursor = hv[0];
    h.tot = hv[1];
    h.D = hv[2];
    h.err = hv[3];
    h.leaf = hv[7];
    h.tame = hv[8];
    h.nxt[0] = (unsigned)hv[9];
    h.nxt[1] = (unsigned)hv[10];
    d.o_err = pl->d.o_err;
    if (h.err) {  // a dead tree stays dead and re-reports its error
        if (l == 0) {
            if (SEL) {
                idx_x[t] = 0;
                idy[t] = t;
                act[t] = 0;
            }
            atomicOr(d.err(), h.err);
        }
        return;
    }
    const int D = h.D;
    if (D != Dp || h.tot != D + 1 || h.leaf != D) {
        if (D + 1 > P || h.tot != D + 1 || h.leaf != D) {  // not a chain: refuse
            if (l == 0) {
                if (SEL) {
                    idx_x[t] = 0;
                    idy[t] = t;
                    act[t] = 0;
                }
                hp->err = kErrPath;
                atomicOr(d.err(), kErrPath);
            }
            return;
        }
        leaf_b = d.Bn()[nb + D];  // out of sequence: the header's leaf
    }
    stamp(ts, 1);
    int err = 0;
    const int leaf = D, c = D + 1;  // the new child
    int cursor = h.cursor;
    int a = 0;
    const float bh = 1.0f;  // betahat_prob = count / sampled_times = 1 / 1
    // every lane's prior * betahat_prob / beta_prob (eps = 0 after the root), computed while the
    // distribution's first LDS store is in flight; the drawn lane's is read after the draw
    float prior_l = 0.f;
    if (A >= 2) {
        const double cp = cdf_bcast(bet, A, (float *)(smem + L.oW), (double *)(smem + L.oP),
                                    [&]() { prior_l = pol * bh / bet; });
        const double w1 = (double)h.nxt[0], w2 = (double)h.nxt[1];
        double u = (w1 + w2 * 4294967296.0) / 18446744073709551616.0;
        if (u >= 1.0) u = 0x1.fffffffffffffp-1;  // nextafter(1, 0)
        a = __popcll(ballot(l < A && cp < u));    // lower_bound
        cursor += 2;
    } else {
        prior_l = pol * bh / bet;
    }
    a = uni(a);
    stamp(ts, 2);
    const float omr = i2f(omri);
    if (c + 1 > P) err |= kErrPool;
    if (value_lim(1, omr) != 1) err |= kErrValueSet;  // (count 1: size_lim must be 1, utils.cpp:31)
    const float pol_a = rlf(pol, a), bet_a = rlf(bet, a);
    const float prior = rlf(prior_l, a);
    const bool wild = !tame_prior(prior);
    leaf_b = uni4(leaf_b);
    if (!err && l == 0) {
        const size_t gi = nb + c;
        d.A()[gi] = make_int4(0, f2i(prior), f2i(0.0f), f2i(0.0f));
        d.Bn()[gi] = make_int4(0, pack_y(0, a, -1), f2i(0.0f), -1);
        d.C()[gi] = make_float4(0.f, 0.f, 0.f, 0.f);
        d.PP()[gi] = v_in;
        if (leaf == 0) {  // (readbacks: root children)
            d.o_D = pl->d.o_D;
            d.D()[gi] = make_float4(pol_a, bet_a, bh, 0.f);
        }
        const int md = md_of(leaf_b.y) < 0 ? 0 : md_of(leaf_b.y);
        d.Bn()[nb + leaf] = make_int4(c, pack_y(1, act_of(leaf_b.y), md), f2i(v_in), hsx);
    }
    const int tame = (h.tame && !wild && tame_val(v_in) && tame_val(r_in)) ? 1 : 0;
    const bool fast = !SEL || (fast_ok && tame && fabsf(discount) <= 1.0f);  // (no selection: no words)
    const int Ds = c;
    if (SEL && Ds + 1 > PS) err |= kErrPath;
    // the root's total child visits after this back-propagation index the pUCT table (select_walk
    // checks it in the fast case; in the exact case it is the largest parent count of the path)
    if (SEL && root_vis0 >= PS && (fast || !err)) err |= kErrTable;
    if (SEL && l == 0) {
        idx_x[t] = err ? 0 : hsx;  // parent->hidden_state_index_x: the expanded leaf's
        idy[t] = t;
        act[t] = err ? 0 : a;
    }
    stamp(ts, 3);
    // wave 1's back-propagation (sA, sPP) and min / max: read by the exact case and the fused
    // readback only.  In select_walk's fast case (one word per level) wave 0 takes no barrier (wave
    // 1's waits for this wave's end instead: s_barrier counts the waves that have not ended)
    const bool bar = MZ_STAMPS || !SEL || !fast;  // (stamped builds: wave 1's stamps come through LDS)
    if (bar) lds_barrier();
    stamp(ts, 4);
    const float mn = bar ? unif(sX[0]) : 0.f, mx = bar ? unif(sX[1]) : 0.f;
    const int mm_cnt = D;
    int words = 0;
    if (SEL && fast) {
        words = Ds - ((root_vis0 + 1 <= 1) ? 1 : 0);  // one per level but the forced first one
    } else if (SEL && !err) {
        // ---- select_walk's exact case: every level's tie list must be non-empty to consume a
        // word (score >= FLOAT_MIN, not NaN); levels 1..Ds scored in parallel ----
        sA[c] = make_int4(0, f2i(prior), f2i(0.0f), f2i(0.0f));
        wait_lds();
        const int root_visit = uni(sA[0].x);
        const float gdelta = pl->g.delta;
        const bool mm_on = mm_cnt > 0;
        float den = 0.f;
        if (mm_on) {
            const float delta = mx - mn;
            den = (gdelta < delta) ? delta : gdelta;  // std::max(delta_lb, delta)
        }
        d.o_pb = pl->d.o_pb;
        d.o_sq = pl->d.o_sq;
        const float *pbt = d.pb();
        const double *sqt = d.sq();
        for (int i0 = 0; i0 <= Ds; i0 += kWave) {
            const int i = i0 + l;
            bool valid = false;
            if (i >= 1 && i <= Ds && !(i == 1 && root_visit <= 1)) {
                const int n = sA[i - 1].x - 1;  // the parent's total_children_visit_counts (< PS: checked)
                const int4 ca = sA[i];
                const float pp = (i == Ds) ? v_in : sPP[i];
                float vs = (ca.x == 0) ? 0.0f : ((i2f(ca.w) + discount * i2f(ca.z)) - pp);
                if (mm_on) vs = (vs - mn) / den;
                if (vs < 0) vs = 0;
                if (vs > 1) vs = 1;
                const float pbc = (float)((double)pbt[n] * (sqt[n] / (double)(ca.x + 1)));
                const float sc = pbc * i2f(ca.y) + vs;
                valid = sc >= -1000000.0f;  // FLOAT_MIN (utils.h:12)
            }
            words += __popcll(ballot(valid));
        }
    }
    stamp(ts, 5);
    if (l < kNxt) {
        unsigned nxt_w = 0;
        if (fast) {
            nxt_w = (wi >= 0 && wi < gW) ? w_fast : 0u;  // (cursor + words + l == wi)
        } else if (SEL && !err && cursor + words + l < gW) {
            nxt_w = Rt[cursor + words + l];
        }
        hp->nxt[l] = nxt_w;
    }
    if (l == 0) {
        hp->cursor = err ? h.cursor : cursor + words;
        hp->tot = err ? h.tot : c + 1;
        hp->D = (err || !SEL) ? h.D : Ds;
        hp->err = err;
        hp->mm_cnt = mm_cnt;  // (mm_min / mm_max: wave 1)
        hp->tame = tame;
        hp->leaf = (err || !SEL) ? h.leaf : c;
    }
    if constexpr (!SEL) {
        // the fused readback (mz_expand_backup_readback, include/mzdriver.h): the search's outputs
        // from this launch's final records.  Wave 1 left every chain node's new {visit, prior, value,
        // reward} in sA (read after the barrier above); the structure records come from HBM but the
        // leaf's, rewritten above, and the root children's probabilities from HBM (written at prepare)
        // (a tree that failed writes an empty readback -- no children, value 0 -- rather than leave
        // the caller's buffers as they were; the error word reports it)
        const RbDesc *rbd = (const RbDesc *)(const void *)iop->gather_out;
        if (rbd) {
            const int4 rbn = err ? make_int4(0, 0, 0, 0) : uni4(d.Bn()[nb]);
            const int nc = nc_of(rbn.y), fc = rbn.x;
            d.o_D = pl->d.o_D;
            const int md = md_of(leaf_b.y) < 0 ? 0 : md_of(leaf_b.y);
            const int4 leaf_new = make_int4(c, pack_y(1, act_of(leaf_b.y), md), f2i(v_in), hsx);
            int4 ca = make_int4(0, 0, 0, 0), cb = ca;
            float4 cd = make_float4(0.f, 0.f, 0.f, 0.f);
            if (l < nc) {
                const int n = fc + l;
                ca = sA[n];
                cb = (n == leaf) ? leaf_new : d.Bn()[nb + n];
                cd = d.D()[nb + n];
            }
            readback_emit(rbd->o, rbd->disc, rbd->Wd, t, A, 1, nc, err ? make_int4(0, 0, 0, 0) : sA[0], ca, cb, cd,
                          nullptr);
        }
    }
    stamp(ts, 6);
    if (MZ_STAMPS && l >= MZ_S_CYC_HEADER && l < MZ_S_COUNT) {
        d.o_stats = pl->d.o_stats;
        long long *st = d.stats() + (size_t)t * MZ_S_COUNT;
        long long add = 0;
        switch (l) {
            case MZ_S_CYC_HEADER: add = (long long)(ts[1] - ts[0]); break;   // round 1
            case MZ_S_CYC_EXP_CDF: add = (long long)(ts[2] - ts[1]); break;  // distribution + draw
            case MZ_S_CYC_EXPAND: add = (long long)(ts[3] - ts[2]); break;   // child, outputs
            case MZ_S_CYC_BACKUP: add = (long long)(ts[4] - ts[3]); break;   // waiting at the barrier
            case MZ_S_CYC_SELECT: add = (long long)(ts[5] - ts[4]); break;   // selection (exact case)
            case MZ_S_CYC_EPILOGUE: add = (long long)(ts[6] - ts[5]); break; // header
            case MZ_S_CYC_BAK_BOOT: add = sXl[0]; break;                     // wave 1: recurrence
            case MZ_S_CYC_BAK_NODES: add = sXl[1]; break;                    // wave 1: node updates
            case MZ_S_CYC_W1_ROUND1: add = sXl[2]; break;                    // wave 1: round 1
            case MZ_S_STAMPED: add = 1; break;
            default: break;
        }
        const bool w2_slot = l == MZ_S_CYC_STAGE1 || l == MZ_S_CYC_STAGE2 || l == MZ_S_CYC_GATHER ||
                             l == MZ_S_CYC_W1_STAGE2;
        if (!w2_slot) st[l] += add;
    }
    if (l == 0 && err) atomicOr(d.err(), err);
    span_close(hsx, rt0);
}

// ================================================================================================
// General trees (2 <= sampled_times <= 64, agent_num = 1, pools of <= 1024 nodes): the fused
// simulation step on four waves
// ================================================================================================
// k_step's general walks score every node (or build every internal node's tie list) after the
// back-propagation, on one wave's critical path.  Here the work is split by what it depends on:
//  - the back-propagation changes only the path nodes (visits + 1, value, the leaf's reward) and
//    the min/max normaliser.  The prior part of every ucb score, pb_c(parent's child visits, child
//    visits) * prior (cnode.cpp:313-316), is therefore known before the back-propagation ends:
//    visits after it are the staged ones plus one on the path.  Waves 2 and 3 compute it for every
//    node (pb_c from the host-built table in HBM, one gather per node), and the min/max over the
//    visited nodes off the path, while wave 1 back-propagates and wave 0 expands the leaf;
//  - after the barrier that hands the results over, wave 0 joins the min/max with the path nodes'
//    new q values and walks level by level (select_child, cnode.cpp:337-379): per level only the
//    value scores of the node's children (one lane each) are computed, from records read in one
//    LDS round trip that also carries the next level's structure record.
// Two barriers: after round 1 (every staged record has landed, path nodes flagged) and after the
// expansion / back-propagation / prior scores.  The engine-word draws of the expansion need no
// staged record and run before the first.
// --------------------------------------------------------------------------------------------
// back-propagation waves of k_tree (waves 1 .. kBkN; wave 0 expands): seven (eight waves, two per
// SIMD) for pools up to 384 nodes, whose trees hold one workgroup per CU, and for the 1,024-node
// class, whose LDS (150 KB with seven) holds one workgroup per CU either way; four (five waves) for
// the 512-node class, whose LDS then still fits two workgroups per CU (3s5z: 512 trees)
#ifndef MZ_TREE_BK
#define MZ_TREE_BK 7
#endif
#ifndef MZ_TREE_BK1024
#define MZ_TREE_BK1024 MZ_TREE_BK
#endif
#ifndef MZ_TREE_BK512
#define MZ_TREE_BK512 MZ_TREE_BK
#endif
// The 1024-node class for searches with S + 1 <= 128 (round 5): 128-entry value-entry slots and
// the layout below fit ~80 KB, two workgroups per CU (3s5z at K = 10: 512 trees of 1,011 nodes in
// one round over the 256 CUs instead of two).  A class id of its own, one node above 1024.
constexpr int kTree1024S = 1025;
template <int NC>
constexpr int kBkN = (NC <= 384) ? MZ_TREE_BK : (NC >= 1024 ? MZ_TREE_BK1024 : MZ_TREE_BK512);
template <int NC>
constexpr int kTreeWavesN = kBkN<NC> + 1;
constexpr int kBkCap = 340;  // value entries per staging slot (two per wave): S + 1 <= 340
static_assert(kBkCap + 2 <= (int)kTableFullPS, "k_tree's prior scores read the full pUCT table");
// the 512-node class with seven back-propagation waves keeps two workgroups per CU (76 KB of LDS
// each) with slots of 128 entries (S + 1 <= 128; larger searches take k_step); so does kTree1024S
template <int NC>
constexpr int kBkCapN = (NC == kTree1024S || (NC == 512 && kBkN<NC> > 4)) ? 128 : kBkCap;
// a staging slot's stride in int2 entries: CAP entries plus one of lead-in for the 16-byte DMA from
// the aligned address below a node's first entry (its entries are 8-byte aligned), and one of
// tail-out, an even count so that every slot starts 16-byte aligned
template <int CAP>
constexpr int kBkSlot = CAP + 2;
// The 1024-node classes walk level by level instead (O(depth) after the barrier instead of
// O(pool) / 4 waves).  Measured on one box, k_tree fused launch: 27m K = 5 (1010 nodes) 13.8 us by
// levels against 14.1 us with tree_select_prep; 3m K = 5 (260 nodes) 10.4 against 11.6 us,
// 3s5z K = 5 (510 nodes) 12.0 against 12.6 us the other way round.
#ifndef MZ_LEVELS_FROM  // (experiment builds: the smallest class that walks by levels)
#define MZ_LEVELS_FROM 1024
#endif
template <int NC>
constexpr bool kTreeLevels = (NC >= MZ_LEVELS_FROM);
// pb_c of the prior scores from the host table in HBM (one gather per node, L2-resident) instead of
// the staged per-n factors and a double division per node: the gather's wait leaves the SIMD to the
// wave that shares it.  Same-box A/B: 3s5z K = 5 10.50 -> 10.38 us, 3m K = 5 unchanged;
// MZ_PBC_FACTORS builds the factor path for A/B runs
#ifdef MZ_PBC_FACTORS
template <int NC>
constexpr bool kTreePbTable = kTreeLevels<NC>;
#else
template <int NC>
constexpr bool kTreePbTable = true;
#endif
// The path nodes' new {value, reward} (sAz): per node where the precomputed walk's tie-list records
// share the array, per path level in the level-walk classes (their walk knows which child lies on
// the back-propagated path without a lookup: 8 B per node of LDS saved)
template <int NC>
constexpr bool kTreeAzLevel = kTreeLevels<NC>;
// the value-set scalars staged for every node (MZ_C_STAGE A/B builds) or scalar-loaded per path
// level (default, round 4; see bk_prestage)
#ifdef MZ_C_STAGE
constexpr bool kTreeCStage = true;
#else
constexpr bool kTreeCStage = false;
#endif
// per back-propagation wave, exchanged at barrier (2): its min/max partial, visited-node count,
// error word and value-entry counters
struct BkOut {
    float mn, mx;
    int cv, err;
    long long er, ew;
};

template <int NC>
struct TreeLayout {
    static constexpr int r16(int x) { return (x + 15) & ~15; }
    static constexpr int BK = kBkN<NC>;
    static constexpr int CAP = kBkCapN<NC>;
    // staging int2s: two slots per back-propagation wave, at least 16 KiB for big leaf rows except in
    // kTree1024S (its rows up to 8 * kTreeReg bytes are staged, larger ones copied directly)
    static constexpr int kTreeReg = (NC == kTree1024S || 2 * BK * kBkSlot<CAP> > kRegCap) ? 2 * BK * kBkSlot<CAP> : kRegCap;
    // path levels: PS = S + 2 <= P / K <= NC / 2, and S + 1 <= CAP (the handle takes k_tree only then)
    static constexpr int PSx = (NC / 2 + 1 < CAP + 1) ? NC / 2 + 1 : CAP + 1;
    static constexpr int oA = 0;                                   // int4 [NC] staged {visit, prior, value, reward}
    static constexpr int oB = oA + r16(16 * NC);                   // int4 [NC] staged structure records
    static constexpr int oPP = oB + r16(16 * NC);                  // f32 [NC] parent's pred_value
    static constexpr int oQ = oPP + r16(4 * NC);                   // f32 [NC] min/max members
    static constexpr int oPar = oQ + r16(4 * NC);                  // i32 [NC] parent index
    static constexpr int oPS = oPar + r16(4 * NC);                 // f32 [NC] prior score after the back-propagation
    static constexpr int oFl = oPS + r16(4 * NC);                  // i32 [NC] 1 + path level (path nodes), else 0
    static constexpr int oAz = oFl + r16(4 * NC);                  // float2 path nodes' new {value, reward}
    // (per node [NC], or per path level [PSx + 64] in the level-walk classes, kTreeAzLevel)
    static constexpr int oPath = oAz + (kTreeAzLevel<NC> ? r16(8 * (PSx + kWave)) : r16(8 * NC));  // int2 [PSx] the path
    static constexpr int oLp = oPath + r16(8 * (PSx + kWave));     // f32 lambda powers
    static constexpr int oRng = oLp + r16(4 * (PSx + 1 + kWave));  // u32 [kRngWin] engine words
    static constexpr int oBoot = oRng + r16(4 * kRngWin);          // f32 [BK][PSx + 64] bootstrap values
    static constexpr int oReg = oBoot + r16(4 * BK * (PSx + kWave));  // int2 [kTreeReg] value entries; big leaf rows
    static constexpr int oX = oReg + r16(8 * kTreeReg);            // exchange between the waves
    static constexpr int oW = oX + r16(256);                       // f32 [64] sampling weights
    static constexpr int oP = oW + r16(4 * kWave);                 // f64 [64] probabilities, then the CDF
    static constexpr int oU = oP + r16(8 * kWave);                 // f64 [64] the draws' canonical doubles
    static constexpr int oIx = oU + r16(8 * kWave);                // i32 [64] the draws' actions
    static constexpr int oPol = oIx + r16(4 * kWave);              // f32 [64] the leaf's policy
    static constexpr int oNxt = oPol + r16(4 * kWave);             // u32 [64] the header's engine words
    static constexpr int oSt = oNxt + r16(4 * kWave);              // i64 [64] the tree's statistics counters
    static constexpr int oCn = oSt + r16(8 * kWave);               // float4 [NC] staged value-set scalars (kTreeCStage)
    static constexpr int oPb = oCn + (kTreeCStage ? r16(16 * NC) : 0);  // f32 [PSx] logf((n + c2 + 1)/c2) + c1
    static constexpr int oSq = oPb + (kTreePbTable<NC> ? 0 : r16(4 * (PSx + kWave)));  // f64 [PSx] sqrt(n)
    static constexpr int oXB = oSq + (kTreePbTable<NC> ? 0 : r16(8 * (PSx + kWave)));  // BkOut [BK + 1] (index = wave)
    static constexpr int total = oXB + r16((int)sizeof(BkOut) * (BK + 1));
};
int tree_lds_bytes(int nc) {
    switch (nc) {
        case 64: return TreeLayout<64>::total;
        case 128: return TreeLayout<128>::total;
        case 256: return TreeLayout<256>::total;
        case 384: return TreeLayout<384>::total;
        case 512: return TreeLayout<512>::total;
        case kTree1024S: return TreeLayout<kTree1024S>::total;
        default: return TreeLayout<1024>::total;
    }
}
static_assert(TreeLayout<kTree1024S>::total <= 80 * 1024, "kTree1024S: two workgroups per CU");

// ------------------------------------------------------------------------------------------------
// k_tree's back-propagation on four waves: path level i belongs to wave 1 + i % 4 (kBk waves).
// A wave stages the value entries of its first two levels before barrier (1), from path records it
// reads with scalar loads (every entry of the node: stage_regions' need test reads structure records
// that land only at barrier (1)); a third or later level is staged after the previous one is done.
// After barrier (1) each wave computes the bootstrap values itself and updates its nodes: one
// lane-parallel pass over a node's entries for the order statistics (utils.cpp:20-71), the node's
// scalars on every lane, the tail shift of the sorted entries lane-parallel.
// ------------------------------------------------------------------------------------------------

// The value-set scalars (C: weighted_sum, tot_weight) are read by the back-propagation for its path
// nodes only.  Default: each back-propagation wave loads its own levels' records with scalar loads
// (the pre-staged levels' in round 1, from the path records it already holds; later levels when it
// reaches them), instead of a round-1 LDS-DMA of every node's record (16 bytes x the pool per tree
// and launch, round 3).  MZ_C_STAGE builds the staged variant for A/B runs.
// (kTreeCStage: defined with the class traits above)

// Round-1 staging of k_tree's node records through registers instead of LDS-DMA (-DMZ_STAGE_VGPR,
// round-6 experiment): every 16-byte record of two arrays loaded into VGPRs (all loads of a batch
// issued together), then written to LDS.  Bit-exact; same-box A/B: 3m K = 5 7.27 -> 7.37 us, 3m
// K = 10 7.44 -> 7.59, 3s5z K = 5 9.99 -> 9.91, 27m K = 5 11.48 -> 11.43 (profiles/round6/ab)
#ifdef MZ_STAGE_VGPR
constexpr bool kStageVgpr = true;
#else
constexpr bool kStageVgpr = false;
#endif
template <int MAXC>
__device__ __forceinline__ void stage_regs16x2(const int4 *s0, int4 *d0, const int4 *s1, int4 *d1, int n) {
    typedef int int4x __attribute__((ext_vector_type(4)));
    typedef const __attribute__((address_space(1))) int4x gi4;
    const int l = lane_id();
    for (int b0 = 0; b0 < n; b0 += MAXC * kWave) {
        int4x v0[MAXC], v1[MAXC];
#pragma unroll
        for (int c = 0; c < MAXC; ++c) {
            const int i = b0 + c * kWave + l;
            if (i < n) {
                v0[c] = *((gi4 *)(const void *)s0 + i);
                v1[c] = *((gi4 *)(const void *)s1 + i);
            }
        }
#pragma unroll
        for (int c = 0; c < MAXC; ++c) {
            const int i = b0 + c * kWave + l;
            if (i < n) {
                *((int4x *)(void *)d0 + i) = v0[c];
                *((int4x *)(void *)d1 + i) = v1[c];
            }
        }
    }
}
template <int MAXC>
__device__ __forceinline__ void stage_regs4x3(const float *s0, float *d0, const float *s1, float *d1, const int *s2,
                                              int *d2, int n) {
    typedef const __attribute__((address_space(1))) float gf;
    typedef const __attribute__((address_space(1))) int gi;
    const int l = lane_id();
    for (int b0 = 0; b0 < n; b0 += MAXC * kWave) {
        float v0[MAXC], v1[MAXC];
        int v2[MAXC];
#pragma unroll
        for (int c = 0; c < MAXC; ++c) {
            const int i = b0 + c * kWave + l;
            if (i < n) {
                v0[c] = *((gf *)(const void *)s0 + i);
                v1[c] = *((gf *)(const void *)s1 + i);
                v2[c] = *((gi *)(const void *)s2 + i);
            }
        }
#pragma unroll
        for (int c = 0; c < MAXC; ++c) {
            const int i = b0 + c * kWave + l;
            if (i < n) {
                d0[i] = v0[c];
                d1[i] = v1[c];
                d2[i] = v2[c];
            }
        }
    }
}

struct BkPre {
    int n0, nv0, n1, nv1;  // the pre-staged levels' nodes and entry counts (nv < 0: not staged)
    int ndma;              // LDS-DMA instructions issued for them (the wave's last ones before barrier (1))
    float4 c0, c1;         // their value-set scalars (scalar loads; unless kTreeCStage)
    int sh0, sh1;          // their first entry's place in the slot (int2 units: 16-byte DMA from below it)
};

// The back-propagation's arena offsets as values of this point of the wave (they depend only on
// the kernel arguments): computed while the wave waits for its round-1 loads, instead of the ~60
// scalar instructions the compiler otherwise re-derives them with after barrier (1), on the
// back-propagation's critical path
__device__ __forceinline__ void bk_pin_offsets(Dev &d) {
#ifndef MZ_NO_PIN
    asm volatile("" : "+s"(d.o_V), "+s"(d.o_A), "+s"(d.o_C), "+s"(d.o_Bn), "+s"(d.o_Q));
#else
    (void)d;
#endif
}

// s_waitcnt vmcnt(n) for a wave-uniform n: all but the wave's n most recent vector-memory operations
__device__ __forceinline__ void wait_vm_but(int n) {
    switch (n) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
        case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    }
}

__device__ __forceinline__ int2 ldsc2(const int2 *p) {
    const long long v = *(const __attribute__((address_space(4))) long long *)p;
    return make_int2((int)(v & 0xffffffffll), (int)(v >> 32));
}

// the path records of wave k's first two levels (scalar loads, issued at the wave's start: indices
// clamped into the tree's PS records, so the reads need not wait for the header's path length)
template <int BK>
__device__ __forceinline__ void bk_path_records(const Dev &d, int t, int PS, int k, int2 &p0, int2 &p1) {
    const int2 *gp = d.path() + (size_t)t * PS;
    p0 = ldsc2(gp + (k < PS ? k : PS - 1));
    p1 = ldsc2(gp + (k + BK < PS ? k + BK : PS - 1));
}

// their value entries -> the wave's two staging slots (every entry of the node)
template <int BK, int CAP>
__device__ __forceinline__ BkPre bk_prestage(const Dev &d, int t, int P, int E, int D, int k, int2 p0, int2 p1,
                                             int2 *sReg) {
    const int l = lane_id();
    BkPre r{0, -1, 0, -1, 0, make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f), 0, 0};
    const int2 *gV = d.V() + (size_t)t * P * E;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int i = k + BK * j;
        const int2 pe = j == 0 ? p0 : p1;
        if (i > D) break;
        if (pe.x < 0 || pe.x >= P || pe.y < 0 || pe.y > CAP) continue;  // (staged after barrier (1))
        // 16-byte LDS-DMA from the aligned address at or below the node's first entry (four times the
        // bytes per instruction of 4-byte chunks; the chunks past the last entry read the next node's)
        const int2 *src = gV + (size_t)pe.x * E;
        const int sh = (int)(((uintptr_t)src >> 3) & 1);  // 8 bytes past a 16-byte boundary
        const int4 *asrc = (const int4 *)(src - sh);
        int2 *dst = sReg + (2 * k + j) * kBkSlot<CAP>;
        const int n16 = (sh + pe.y + 1) >> 1;
        for (int c = 0; c < n16; c += kWave)
            if (c + l < n16) glds16a(asrc + c + l, (int4 *)dst + c);
        r.ndma += (n16 + kWave - 1) / kWave;
        if (j == 0) r.sh0 = sh;
        else r.sh1 = sh;
        // (scalar loads, counted by lgkmcnt: landed by the first LDS wait after barrier (1))
        const float4 cw = (kTreeCStage) ? make_float4(0.f, 0.f, 0.f, 0.f) : ldsc4(d.C() + (size_t)t * P + pe.x);
        if (j == 0) {
            r.n0 = pe.x;
            r.nv0 = pe.y;
            r.c0 = cw;
        } else {
            r.n1 = pe.x;
            r.nv1 = pe.y;
            r.c1 = cw;
        }
    }
    return r;
}

// the bootstrap values b_{i-1} = reward_i + discount * b_i (cnode.cpp:424,448) of levels 0..D into boot[]
__device__ __forceinline__ void bk_boot(const Lds &s, float *boot, int D, float value, float reward, float disc) {
    const int l = lane_id();
    float carry = value;
    int hi = D;
    while (true) {
        const int lo = hi > 63 ? hi - 63 : 0;
        const int nl = hi - lo;
        const int lev = hi - 63 + l;
        float rn = 0.f;
        if (lev >= lo && lev < hi) rn = (lev + 1 == D) ? reward : i2f(s.A[s.path[lev + 1].x].w);
        float b = (l == 63) ? carry : 0.f;
        float tmp = (l == 62) ? disc * carry : 0.f;
        boot_dpp(b, tmp, disc, rn, nl);
        if (lev >= lo && lev <= hi) boot[lev] = b;
        if (lo == 0) break;
        carry = rlf(b, 63 - nl);
        hi = lo;
    }
    wait_lds();
}

// wave k's path levels k, k + BK, ... (CTree::back_propagate, cnode.cpp:415-450, node by node)
template <int BK, int CAP, bool AZL>  // AZL: sAz per path level (kTreeAzLevel), else per node
__device__ __forceinline__ void bk_levels(const Geo &g, const Dev &d, const Lds &s, const float4 *sCn, float2 *sAz,
                                          const float *boot, int2 *sReg, BkPre pre, int t, int D, float reward,
                                          float disc, int k, int &err, long long &ent_r, long long &ent_w, float &pmn,
                                          float &pmx, unsigned long long *tl = nullptr) {
    const int l = lane_id();
    int2 *gV = d.V() + (size_t)t * g.P * g.E;
    pmn = INFINITY;
    pmx = -INFINITY;
    wait_vm();  // the pre-staged entries (in flight across barrier (1))
    if (MZ_STAMPS && tl) tl[0] = __builtin_amdgcn_s_memtime();
    for (int j = 0, i = k; i <= D; ++j, i += BK) {
        // the level's node: from the pre-stage's scalar path records (no LDS round trip) or the path
        int n, nv;
        if (j == 0 && pre.nv0 >= 0) {
            n = pre.n0;
            nv = pre.nv0;
        } else if (j == 1 && pre.nv1 >= 0) {
            n = pre.n1;
            nv = pre.nv1;
        } else {
            const int2 pe = s.path[i];
            n = uni(pe.x);
            nv = uni(pe.y);
        }
        if (n < 0 || n >= g.P || nv < 0 || nv > CAP) {
            err |= kErrPath;
            continue;
        }
        const int dep = D - i;
        // every record of the node in one LDS round trip
        const int4 b4 = s.B[n];
        const int4 a4r = s.A[n];
        float4 cw;
        if (kTreeCStage) cw = sCn[n];
        else if (j == 0 && pre.nv0 >= 0) cw = pre.c0;
        else if (j == 1 && pre.nv1 >= 0) cw = pre.c1;
        else cw = ldsc4(d.C() + (size_t)t * g.P + n);  // (a later level)
        const float ppn = s.PP[n];
        const float lp = s.lp[dep];
        const float key = boot[i];
        const int2 *R;
        if (j == 0 && pre.nv0 >= 0) {
            R = sReg + (2 * k) * kBkSlot<CAP> + pre.sh0;
        } else if (j == 1 && pre.nv1 >= 0) {
            R = sReg + (2 * k + 1) * kBkSlot<CAP> + pre.sh1;
        } else {  // a later level (or a pre-stage that did not match): slot 0, free once level j - 2 is done
            int2 *dst = sReg + (2 * k) * kBkSlot<CAP>;
            const int *src = (const int *)(gV + (size_t)n * g.E);
            for (int c = 0; c < 2 * nv; c += kWave)
                if (c + l < 2 * nv) glds4a(src + c + l, (int *)dst + c);
            wait_vm();
            R = dst;
        }
        const int by = uni(b4.y);
        // entries of a smaller depth / the same depth / the same depth and a smaller value; none but
        // smaller depths when the node's deepest entry is above dep (stage_regions' need test)
        int lo = nv, c = 0, pv = 0;
        // (a node of at most one wave of entries keeps them in lane e's registers: the order
        // statistic and the tail shift below then read no LDS)
        const bool reg1 = nv <= kWave;
        int2 e1 = make_int2(0x7fffffff, 0);
        if (nv > 0 && md_of(by) >= dep) {
            lo = 0;
            for (int e0 = 0; e0 < nv; e0 += kWave) {
                const bool on = e0 + l < nv;
                const int2 e = on ? R[e0 + l] : make_int2(0x7fffffff, 0);
                if (e0 == 0) e1 = e;
                lo += __popcll(ballot(on && e.x < dep));
                c += __popcll(ballot(on && e.x == dep));
                pv += __popcll(ballot(on && e.x == dep && i2f(e.y) < key));
            }
            ent_r += nv;
        }
        auto entry_y = [&](int i) {  // R[i].y, 0 <= i < nv, read only after the pass above loaded R
            return reg1 ? rl(e1.y, i) : R[i].y;
        };
        float ws = cw.x, tw = cw.y;
        const int cur = (c == 0) ? 0 : value_lim(c, g.one_minus_rho);
        const int nl = value_lim(c + 1, g.one_minus_rho);
        if (cur == nl) {  // SubTreeValueSet::update (utils.cpp:20-71)
            const float mb = i2f(entry_y(lo + c - cur));  // *big.begin()
            if (!(key < mb)) {
                ws -= lp * mb;
                tw -= lp;
                tw += lp;
                ws += lp * key;
            }
        } else {
            if (cur + 1 != nl) err |= kErrValueSet;
            if (c - cur == 0) {
                tw += lp;
                ws += lp * key;
            } else {
                const float ms = i2f(entry_y(lo + c - cur - 1));  // *(--small.end())
                if (key > ms) {
                    tw += lp;
                    ws += lp * key;
                } else {
                    tw += lp;
                    ws += lp * ms;
                }
            }
        }
        int pos = lo + pv;
        int2 *G = gV + (size_t)n * g.E;
        if (nv + 1 > g.E) {
            err |= kErrPath;
            pos = nv;
        } else if (l == 0) {
            G[pos] = make_int2(dep, f2i(key));
        }
        if (reg1) {  // the entries after the insertion point move up by one (from the registers)
            if (l >= pos && l < nv) G[l + 1] = e1;
        } else {
            for (int e0 = pos; e0 < nv; e0 += kWave)
                if (e0 + l < nv) G[e0 + l + 1] = R[e0 + l];
        }
        ent_w += nv - pos + 1;
        const bool is_leaf = (i == D);  // its structure record belongs to the expanding wave
        int4 a4 = a4r;
        if (is_leaf) a4.w = f2i(reward);
        const int nc = is_leaf ? 1 : nc_of(by);
        const float val = (nc > 0) ? ws / tw : 0.f;  // CNode::value (cnode.cpp:42-56)
        const size_t gi = (size_t)t * g.P + n;
        float q = 0.f;
        if (i >= 1) q = (i2f(a4.w) + disc * val) - ppn;  // get_qsa - father->pred_value
        if (l == 0) {
            d.A()[gi] = make_int4(a4.x + 1, a4.y, f2i(val), a4.w);
            d.C()[gi] = make_float4(ws, tw, 0.f, 0.f);
            if (!is_leaf && dep > md_of(by)) d.Bn()[gi] = make_int4(b4.x, pack_y(nc, act_of(by), dep), b4.z, b4.w);
            if (i >= 1) d.Q()[gi] = q;
            sAz[AZL ? i : n] = make_float2(val, i2f(a4.w));
        }
        if (i >= 1) {
            pmn = fminf(pmn, q);
            pmx = fmaxf(pmx, q);
        }
        if (MZ_STAMPS && tl && j < 2) tl[1 + j] = __builtin_amdgcn_s_memtime();
    }
}

// k_tree after barrier (2), run by all four waves (64-node blocks dealt round-robin):
//  (S1) every node's ucb score under its parent (cnode.cpp:297-335) -- the prior score of waves 2
//       and 3 plus the value score, min/max-normalised with the joined min/max -- in place of the
//       prior score;
//  (S2) every node's select_child outcome (cnode.cpp:337-379): the reference's sequential arg-max
//       with epsilon ties over its children's scores.  A one-child tie list (the usual case) is
//       stored as the next node (sPar, free now); leaves get kTreeLeaf; other lists (ties, an empty
//       list, a parent beyond the pUCT table) get kTreeSlow and an exact record: list bits in sAz,
//       size | table error << 16 in sQ.
// Wave 0 then chases next nodes one LDS read per level.
constexpr int kTreeLeaf = -1, kTreeSlow = -2;



// Who stages the value-set scalars in round 1: wave 0 (with the path, the flags and the leaf's
// inputs) or, for the 1024-node class, wave 4.  Same-box A/B: 3m K = 10 9.77 -> 9.64 us with wave 4;
// the smaller classes measured no gain (3m K = 5) or a loss (3s5z K = 5, 10.47 -> 10.59 us).
// Who gathers the leaf's row in the precomputed-walk classes: wave 1, after its own copy of the
// chase (the same reads of the same LDS state), while wave 0 writes the path record, the header
// and the counters; the level walk (1024-node class) gathers on wave 0.
template <int NC>
#ifdef MZ_NO_W1G
constexpr bool kTreeW1Gather = false;
#else
constexpr bool kTreeW1Gather = !kTreeLevels<NC>;
#endif

// The waves that score every node and resolve the tie lists after barrier (2) (tree_select_prep):
// four where a pass of four waves covers the pool (<= 256 nodes), every wave of the workgroup in the
// larger classes, where four waves took two passes of each phase (round 6, same-box A/B against the
// same build with four, MZ_SEL_W4: 3s5z K = 5 10.08 -> 9.98 us, 3m K = 10 unchanged at 7.60)
template <int NC>
#ifdef MZ_SEL_W4
constexpr int kSelW = 4;
#else
constexpr int kSelW = (NC > 256 && !kTreeLevels<NC>) ? kTreeWavesN<NC> : 4;
#endif

// Round-6 experiment (-DMZ_HELPER_CDF): the leaf's sampling distribution (discrete_distribution's
// probabilities and prefix sums, cnode.cpp:243-262) computed before barrier (1) by the last
// back-propagation role (hardware wave 4, on wave 0's SIMD; its path levels are the deepest and
// usually absent) while wave 0 waits for its round-1 loads, wave 0 reading the CDF after barrier (1).
// Bit-exact, but slower in every configuration (same-box A/B against the same build without it:
// 3m K = 5 7.22 -> 7.57 us, 3m K = 10 7.44 -> 7.60, 3s5z K = 5 9.92 -> 9.98, 27m K = 5
// 11.43 -> 11.58; profiles/round6/ab): the helper's beta load and distribution delay barrier (1)
// for every wave, and the expansion it shortens ends before the back-propagation anyway
#ifdef MZ_HELPER_CDF
constexpr bool kTreeHelperCdf = true;
#else
constexpr bool kTreeHelperCdf = false;
#endif

// Round-6 experiment (-DMZ_SCORE_WALK): in the precomputed classes, after barrier (2) the four waves
// score every node (S1) and each chase copy then walks from the root over those scores (score_walk:
// per level the children's scores in one LDS round trip, the sequential arg-max in closed form by a
// DPP row max and two ballots) instead of resolving every internal node's tie list (S2) and chasing
// the resolved outcomes (tree_chase).  Bit-exact (the GPU suite passes on it), but slower: wave 0's
// stamps at 3m K = 5 put S1 at ~1,400 cycles and S2 at ~1,380, and a walked level at ~950 cycles
// against ~460 per chased level (its serial chain of LDS round trip, DPP max, readfirstlane, two
// ballots and readlanes), so S1 + walk ~5,200 against S1 + S2 + chase ~4,600; fused launch
// 7.26 -> 8.47 us, 3m K = 10 7.50 -> 8.13, 3s5z K = 5 10.10 -> 10.96 (profiles/round6/ab).
template <int NC>
#ifdef MZ_SCORE_WALK
constexpr bool kTreeScoreWalk = !kTreeLevels<NC>;
#else
constexpr bool kTreeScoreWalk = false;
#endif

template <int NC>
#ifdef MZ_C_W4
constexpr bool kTreeCW4 = true;
#else
constexpr bool kTreeCW4 = kTreeLevels<NC>;
#endif


// The chase's common levels (wave 0, uniform control flow): while the current outcome v is a child
// (a one-member list inside the table, tree_select_prep's next node) and the path stays under lim
// levels, step to it -- path lane Dn := x -- and read its outcome, one engine word per outcome that
// is a child.  ~18 instructions and one LDS round trip a level; stops at a leaf, an exact record
// or the end of the path lanes, where the general step takes over.  nb: nxt's LDS byte address.
__device__ __forceinline__ void chase_next(int &v, int &cursor, int &x, int &Dn, int &xprev, int &px, int lane,
                                          unsigned nb, int lim) {
    int t0, t1, va, r0;
    asm volatile(
        ".Lcn%=_top:\n\t"
        "s_cmp_lt_i32 %[v], 0\n\t"
        "s_cbranch_scc1 .Lcn%=_out\n\t"
        "s_add_i32 %[t0], %[dn], 1\n\t"
        "s_cmp_ge_i32 %[t0], %[lim]\n\t"
        "s_cbranch_scc1 .Lcn%=_out\n\t"
        "s_lshl_b32 %[t1], %[v], 2\n\t"
        "s_add_u32 %[t1], %[t1], %[nb]\n\t"
        "v_mov_b32 %[va], %[t1]\n\t"
        "ds_read_b32 %[r0], %[va]\n\t"
        "s_mov_b32 %[xp], %[x]\n\t"
        "s_mov_b32 %[x], %[v]\n\t"
        "s_mov_b32 %[dn], %[t0]\n\t"
        "v_cmp_eq_u32_e32 vcc, %[dn], %[ln]\n\t"
        "v_mov_b32 %[va], %[x]\n\t"
        "s_nop 1\n\t"
        "v_cndmask_b32_e32 %[px], %[px], %[va], vcc\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_readfirstlane_b32 %[v], %[r0]\n\t"
        "s_cmp_gt_i32 %[v], -1\n\t"
        "s_cselect_b32 %[t1], 1, 0\n\t"
        "s_add_i32 %[cur], %[cur], %[t1]\n\t"
        "s_branch .Lcn%=_top\n"
        ".Lcn%=_out:"
        : [v] "+s"(v), [cur] "+s"(cursor), [x] "+s"(x), [dn] "+s"(Dn), [xp] "+s"(xprev), [px] "+v"(px),
          [t0] "=&s"(t0), [t1] "=&s"(t1), [va] "=&v"(va), [r0] "=&v"(r0)
        : [nb] "s"(nb), [lim] "s"(lim), [ln] "v"(lane)
        : "vcc", "scc", "memory");
}

// The level walk's common level in one straight run (round 6, the two-level passes): the tie list of
// the group of eight at lane `base` from the pass's ballots (tT / tE: the group's bits of the
// threshold and first-maximum ballots; big: its maximum beats FLOAT_MIN), as pick computes it; then,
// unless the list has two or more members (a tie: an engine word decides), the node is the root
// under forced round-robin, its visit count is outside the table, the stream has ended or the path
// lanes end here -- returned as 1 with nothing changed, pick and advance take the level --, the step
// to the chosen child: one word if the list is not empty, path lane Dn := {x, visits}, the child's
// structure record by readlane.  No branch but the exit.
__device__ __forceinline__ int walk_step8(unsigned tT, unsigned tE, unsigned big, int base, int nc, int fc, int PS,
                                          int gW, int lim, int &x, int &xv, int &xbx, int &xby, int &xbw,
                                          int &cursor, int &Dn, int &par_hsx, int &px, int &pvv, int cvis, int cbx,
                                          int cby, int cbw, int lane) {
    int slow, t0, t1, r, cnt, ci, ln, lst, a0, a1;
    asm volatile(
        "s_ff1_i32_b32 %[r], %[tE]\n\t"
        "s_lshl_b32 %[t0], -1, %[r]\n\t"
        "s_cmp_lg_u32 %[big], 0\n\t"
        "s_cselect_b32 %[t0], %[t0], -1\n\t"
        "s_and_b32 %[lst], %[tT], %[t0]\n\t"
        "s_bcnt1_i32_b32 %[cnt], %[lst]\n\t"
        "s_ff1_i32_b32 %[ci], %[lst]\n\t"
        "s_max_i32 %[ci], %[ci], 0\n\t"
        "s_cmp_gt_u32 %[cnt], 1\n\t"
        "s_cselect_b32 %[slow], 1, 0\n\t"
        "s_cmp_ge_i32 %[cur], %[gW]\n\t"
        "s_cselect_b32 %[t0], %[cnt], 0\n\t"
        "s_or_b32 %[slow], %[slow], %[t0]\n\t"
        "s_add_i32 %[t0], %[xv], -1\n\t"
        "s_cmp_ge_u32 %[t0], %[PS]\n\t"
        "s_cselect_b32 %[t0], 1, 0\n\t"
        "s_or_b32 %[slow], %[slow], %[t0]\n\t"
        "s_cmp_eq_u32 %[x], 0\n\t"
        "s_cselect_b32 %[t0], 1, 0\n\t"
        "s_cmp_le_i32 %[xv], %[nc]\n\t"
        "s_cselect_b32 %[t0], %[t0], 0\n\t"
        "s_or_b32 %[slow], %[slow], %[t0]\n\t"
        "s_add_i32 %[t1], %[dn], 1\n\t"
        "s_cmp_ge_i32 %[t1], %[lim]\n\t"
        "s_cselect_b32 %[t0], 1, 0\n\t"
        "s_or_b32 %[slow], %[slow], %[t0]\n\t"
        "s_cmp_lg_u32 %[slow], 0\n\t"
        "s_cbranch_scc1 .Lws%=_out\n\t"
        "s_add_i32 %[cur], %[cur], %[cnt]\n\t"
        "s_mov_b32 %[phs], %[xbw]\n\t"
        "s_add_i32 %[ln], %[base], %[ci]\n\t"
        "s_add_i32 %[x], %[fc], %[ci]\n\t"
        "s_mov_b32 %[dn], %[t1]\n\t"
        "s_nop 3\n\t"
        "v_readlane_b32 %[xv], %[cvis], %[ln]\n\t"
        "v_readlane_b32 %[xbx], %[cbx], %[ln]\n\t"
        "v_readlane_b32 %[xby], %[cby], %[ln]\n\t"
        "v_readlane_b32 %[xbw], %[cbw], %[ln]\n\t"
        "v_cmp_eq_u32_e32 vcc, %[dn], %[lane]\n\t"
        "v_mov_b32 %[a0], %[x]\n\t"
        "s_nop 4\n\t"
        "v_mov_b32 %[a1], %[xv]\n\t"
        "v_cndmask_b32_e32 %[px], %[px], %[a0], vcc\n\t"
        "s_nop 1\n\t"
        "v_cndmask_b32_e32 %[pvv], %[pvv], %[a1], vcc\n"
        ".Lws%=_out:\n\t"
        "s_nop 4"
        : [slow] "=&s"(slow), [t0] "=&s"(t0), [t1] "=&s"(t1), [r] "=&s"(r), [cnt] "=&s"(cnt), [ci] "=&s"(ci),
          [ln] "=&s"(ln), [lst] "=&s"(lst), [a0] "=&v"(a0), [a1] "=&v"(a1), [x] "+s"(x), [xv] "+s"(xv),
          [xbx] "+s"(xbx), [xby] "+s"(xby), [xbw] "+s"(xbw), [cur] "+s"(cursor), [dn] "+s"(Dn),
          [phs] "+s"(par_hsx), [px] "+v"(px), [pvv] "+v"(pvv)
        : [tT] "s"(tT), [tE] "s"(tE), [big] "s"(big), [base] "s"(base), [nc] "s"(nc), [fc] "s"(fc), [PS] "s"(PS),
          [gW] "s"(gW), [lim] "s"(lim), [cvis] "v"(cvis), [cbx] "v"(cbx), [cby] "v"(cby), [cbw] "v"(cbw),
          [lane] "v"(lane)
        : "vcc", "scc");
    return slow;
}

// the back-propagation waves' exchange records (after barrier (2)): joined error word, min/max and
// visited-node count (path nodes 1 .. D are visited now, cnode.cpp:431-447)
// Lane j (1 <= j <= BK <= 7) reads record j, and three DPP steps within each row's first eight lanes
// join them: min / max are exact and order-free (NaN partials lose to numbers, as in fminf), the
// counts and error bits are integers.
template <int NC>
__device__ __forceinline__ void bk_join(const unsigned char *smem, int D, int &err, float &mn, float &mx, int &cnt) {
    const BkOut *xb = (const BkOut *)(smem + TreeLayout<NC>::oXB);
    const int j = lane_id() & 7;
    const bool on = j >= 1 && j <= kBkN<NC>;
    const int jj = on ? j : 1;
    float a = xb[jj].mn, b = xb[jj].mx;
    int c = xb[jj].cv, e = xb[jj].err;
    if (!on) {
        a = INFINITY;
        b = -INFINITY;
        c = 0;
        e = 0;
    }
    a = fminf(a, i2f(dpp<0xB1>(f2i(a))));
    b = fmaxf(b, i2f(dpp<0xB1>(f2i(b))));
    c += dpp<0xB1>(c);
    e |= dpp<0xB1>(e);
    a = fminf(a, i2f(dpp<0x4E>(f2i(a))));
    b = fmaxf(b, i2f(dpp<0x4E>(f2i(b))));
    c += dpp<0x4E>(c);
    e |= dpp<0x4E>(e);
    a = fminf(a, i2f(dpp<0x141>(f2i(a))));
    b = fmaxf(b, i2f(dpp<0x141>(f2i(b))));
    c += dpp<0x141>(c);
    e |= dpp<0x141>(e);
    mn = unif(a);
    mx = unif(b);
    cnt = (D >= 1 ? D : 0) + uni(c);  // path nodes 1 .. D are visited now; record 1 counts 0
    err = uni(e);
}
template <int NC>
__device__ __forceinline__ int bk_err(const unsigned char *smem) {
    int e, c;
    float a, b;
    bk_join<NC>(smem, 0, e, a, b, c);
    return e;
}
template <int NC>
__device__ __forceinline__ void bk_minmax(const unsigned char *smem, int D, float &mn, float &mx, int &cnt) {
    int e;
    bk_join<NC>(smem, D, e, mn, mx, cnt);
}

template <int NC>
__device__ __forceinline__ void tree_select_prep(unsigned char *smem, int wv, int ntot, float disc, float gdelta, int PS,
                                                 int D, unsigned long long *tp = nullptr) {
    using L = TreeLayout<NC>;
    const int l = lane_id();
    const int4 *sA = (const int4 *)(smem + L::oA);
    const int4 *sB = (const int4 *)(smem + L::oB);
    const float *sPP = (const float *)(smem + L::oPP);
    float *sQ = (float *)(smem + L::oQ);
    int *nxt = (int *)(smem + L::oPar);
    float *sSc = (float *)(smem + L::oPS);
    const int *sFl = (const int *)(smem + L::oFl);
    float2 *sAz = (float2 *)(smem + L::oAz);
    float mmn, mmx;
    int mm_cnt;
    bk_minmax<NC>(smem, D, mmn, mmx, mm_cnt);
    const bool mm_on = mm_cnt > 0;
    float den = 0.f;
    if (mm_on) {
        const float delta = mmx - mmn;
        den = (gdelta < delta) ? delta : gdelta;  // std::max(delta_lb, delta)
    }
#ifdef MZ_S12_FUSED
    // (S) one pass (round-5 experiment, MZ_S12_FUSED builds): every internal node scores its own
    // children inline (ucb_score, cnode.cpp:297-335) and resolves select_child (cnode.cpp:337-379),
    // with no barrier between the scores and the tie lists; the exact records' list bits go to the
    // value-entry staging area.  Measured and kept out (same-box A/B, fused launch): 3m K = 5
    // 7.57 -> 8.65 us, 3m K = 10 7.87 -> 9.71, 3s5z K = 5 10.25 -> 11.57: a lane scores up to eight
    // children (~25 instructions each, every lane of the wave issuing them) where (S1) scores one
    // node per lane, which costs more than the barrier it saves.
    float2 *sRec = (float2 *)(smem + L::oReg);
    auto score = [&](int c) {
        const int4 a = sA[c];
        const int fl = sFl[c];
        const float2 az = sAz[c];
        const int vis = a.x + (fl ? 1 : 0);
        const float val = fl ? az.x : i2f(a.z);
        const float rw = fl ? az.y : i2f(a.w);
        float vs = (vis == 0) ? 0.0f : ((rw + disc * val) - sPP[c]);
        if (mm_on) vs = (vs - mmn) / den;
        if (vs < 0) vs = 0;
        if (vs > 1) vs = 1;
        return sSc[c] + vs;  // prior_score + value_score
    };
    if (MZ_STAMPS && tp) tp[0] = __builtin_amdgcn_s_memtime();
#else
    float2 *sRec = sAz;
    auto score = [&](int c) { return sSc[c]; };
    for (int n0 = wv * kWave; n0 < ntot; n0 += kSelW<NC> * kWave) {  // (S1)
        const int n = n0 + l;
        if (n >= 1 && n < ntot) {
            const int4 a = sA[n];
            const int fl = sFl[n];
            const float2 az = sAz[n];
            const int vis = a.x + (fl ? 1 : 0);
            const float val = fl ? az.x : i2f(a.z);
            const float rw = fl ? az.y : i2f(a.w);
            float vs = (vis == 0) ? 0.0f : ((rw + disc * val) - sPP[n]);
            if (mm_on) vs = (vs - mmn) / den;
            if (vs < 0) vs = 0;
            if (vs > 1) vs = 1;
            sSc[n] = sSc[n] + vs;  // prior_score + value_score
            if constexpr (kTreeScoreWalk<NC>) sQ[n] = i2f(vis);  // (score_walk: visits after the back-propagation)
        }
    }
    if (MZ_STAMPS && tp) {
        wait_lds();
        tp[0] = __builtin_amdgcn_s_memtime();
    }
    lds_barrier();  // (3)
    if constexpr (kTreeScoreWalk<NC>) return;  // (no tie lists: the walk resolves its own levels)
#endif
    for (int p0 = wv * kWave; p0 < ntot; p0 += kSelW<NC> * kWave) {  // (S2)
        const int p = p0 + l;
        if (p < ntot) {
            const int4 b = sB[p];
            const int fc = b.x, nc = nc_of(b.y);
            if (nc == 0) {
                nxt[p] = kTreeLeaf;
            } else {
                const int np = sA[p].x + (sFl[p] ? 1 : 0) - 1;  // total_children_visit_counts
                const bool terr = np < 0 || np >= PS;
                float mx = -1000000.0f;  // FLOAT_MIN (utils.h:12)
                unsigned long long lst = 0ull;
                int cnt = 0;
#ifndef MZ_S2_SEQ
                if (nc <= 8) {
                    // up to eight children: the sequential arg-max in closed form (as the level walk),
                    // the first maximum r and every later child within epsilon of it; {s >= FLOAT_MIN}
                    // when no score beats FLOAT_MIN.  NaN scores join no list either way, and == makes
                    // the sign of a zero maximum irrelevant
                    float sc[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) sc[u] = score(fc + (u < nc ? u : 0));
#pragma unroll
                    for (int u = 0; u < 8; ++u)
                        if (u >= nc) sc[u] = -INFINITY;
                    const float M = fmaxf(fmaxf(fmaxf(sc[0], sc[1]), fmaxf(sc[2], sc[3])),
                                          fmaxf(fmaxf(sc[4], sc[5]), fmaxf(sc[6], sc[7])));
                    unsigned eq = 0u, ge = 0u;
                    if (M > mx) {
                        const float thr = M - 0.000001f;
#pragma unroll
                        for (int u = 0; u < 8; ++u) {
                            eq |= (sc[u] == M) ? (1u << u) : 0u;
                            ge |= (sc[u] >= thr) ? (1u << u) : 0u;
                        }
                        ge &= ~0u << __builtin_ctz(eq);
                    } else {
#pragma unroll
                        for (int u = 0; u < 8; ++u) ge |= (sc[u] >= mx) ? (1u << u) : 0u;
                    }
                    lst = ge;
                    cnt = __builtin_popcount(ge);
                } else
#endif
                for (int i0 = 0; i0 < nc; i0 += 4) {
                    float sc[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) sc[u] = score(fc + ((i0 + u < nc) ? i0 + u : i0));
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int i = i0 + u;
                        const float v = sc[u];
                        const bool ok = i < nc;
                        const bool gt = ok && (mx < v);
                        const bool ge = ok && !gt && (v >= mx - 0.000001f);
                        const unsigned long long bit = 1ull << (i & 63);
                        lst = gt ? bit : (ge ? (lst | bit) : lst);
                        cnt = gt ? 1 : (cnt + (ge ? 1 : 0));
                        mx = gt ? v : mx;
                    }
                }
                if (cnt == 1 && !terr) {
                    nxt[p] = fc + __builtin_ctzll(lst);
                } else {
                    nxt[p] = kTreeSlow;
                    sRec[p] = make_float2(i2f((int)(unsigned)(lst & 0xffffffffull)), i2f((int)(unsigned)(lst >> 32)));
                    sQ[p] = i2f(cnt | (terr ? 0x10000 : 0));
                }
            }
        }
    }
    if (MZ_STAMPS && tp) {
        wait_lds();
        tp[1] = __builtin_amdgcn_s_memtime();
    }
    lds_barrier();  // (4)
}

// The chase after tree_select_prep (cnode.cpp:381-413 over the precomputed outcomes): from the root,
// next nodes one LDS read a level (chase_next), exact records (ties: the engine word modulo the list
// size; an empty list: child 0; table errors) in the general step.  Wave 0 records the path (REC);
// wave 1 runs the same chase on the same LDS state for the leaf's parent only, and gathers its row.
template <int NC, bool REC>
__device__ __forceinline__ void tree_chase(unsigned char *smem, const Dev &d, int t, int gW, int wbase, int wsh,
                                           int PS, int &cursor, int &err, int &Dn, int &x, int &xprev, int &px,
                                           int &nbw) {
    using L = TreeLayout<NC>;
    const int l = lane_id();
    const int4 *sA = (const int4 *)(smem + L::oA);
    const int4 *sB = (const int4 *)(smem + L::oB);
    const float *sQ = (const float *)(smem + L::oQ);
    int2 *sPath = (int2 *)(smem + L::oPath);
    const unsigned *sRng = (const unsigned *)(smem + L::oRng);
    const int *nxt = (const int *)(smem + L::oPar);
#ifdef MZ_S12_FUSED
    const float2 *rec = (const float2 *)(smem + L::oReg);  // (tree_select_prep's exact records)
#else
    const float2 *rec = (const float2 *)(smem + L::oAz);
#endif
    cursor = uni(cursor);
    int v;
    const unsigned nxb = lds_addr(smem) + L::oPar;
    const int lim = PS < kWave ? PS : kWave;
    {
        const int4 r0b = uni4(sB[0]);
        const int rv = uni(sA[0].x) + 1;  // the root is on every path
        const int nc0 = nc_of(r0b.y);
        if (nc0 == 0) {
            v = kTreeLeaf;
        } else if (rv <= nc0) {
            v = r0b.x + rv - 1;  // forced root round-robin (cnode.cpp:398-399): no word
        } else {
            v = uni(nxt[0]);
            if (v >= 0) ++cursor;
        }
    }
    while (true) {
        chase_next(v, cursor, x, Dn, xprev, px, l, nxb, lim);
        v = uni(v);
        cursor = uni(cursor);
        if (v < 0) {
            if (v == kTreeLeaf) break;
#ifndef MZ_SLOW_OLD
            // the exact record: ties (engine word modulo the list size), an empty list (child 0, no
            // word) or a table error.  Everything it reads depends only on x and the cursor, so all
            // of it is one LDS round trip; the k-th listed child is one ballot (mbcnt rank)
            const int o = cursor - wbase + wsh;
            const bool inwin = o >= wsh && o < kRngWin;
            const float qv = sQ[x];
            const float2 rb = rec[x];
            const int bx = sB[x].x;
            const unsigned wwin = sRng[inwin ? o : 0];
            const int xfl = uni(f2i(qv));
            if (uni(xfl >> 16)) {
                err |= kErrTable;
                break;
            }
            const int cnt = uni(xfl & 0xffff);
            int ci = 0;
            if (cnt > 0) {
                if (cursor >= gW) {
                    err |= kErrRng;
                    break;
                }
                const unsigned lo = (unsigned)uni(f2i(rb.x)), hi = (unsigned)uni(f2i(rb.y));
                if (cnt > 1) {
                    if (!inwin) ++nbw;  // (MZ_S_RNG_TIE_BEYOND)
                    const unsigned w = inwin ? (unsigned)uni((int)wwin) : (unsigned)uni((int)d.R()[(size_t)t * gW + cursor]);
                    const int k = uni((int)(w % (unsigned)cnt));
                    const unsigned lst_l = (l < 32) ? (lo >> l) : (hi >> (l - 32));
                    const int below = (int)__builtin_amdgcn_mbcnt_hi(hi, __builtin_amdgcn_mbcnt_lo(lo, 0u));
                    ci = uni(__builtin_ctzll(ballot((lst_l & 1u) && below == k)));
                } else {
                    ci = lo ? __builtin_ctz(lo) : 32 + __builtin_ctz(hi);
                }
                ++cursor;
            }
            v = uni(uni(bx) + ci);
#else
            // the exact record: ties (engine word modulo the list size), an empty list (child
            // 0, no word) or a table error
            const int xfl = uni(f2i(sQ[x]));
            if (uni(xfl >> 16)) {
                err |= kErrTable;
                break;
            }
            const int cnt = uni(xfl & 0xffff);
            int ci = 0;
            if (cnt > 0) {
                const float2 rb = rec[x];
                unsigned long long lst = ((unsigned long long)(unsigned)uni(f2i(rb.y)) << 32) |
                                         (unsigned)uni(f2i(rb.x));
                if (cursor >= gW) {
                    err |= kErrRng;
                    break;
                }
                if (cnt > 1) {
                    const int o = cursor - wbase + wsh;
                    const unsigned w = (o >= wsh && o < kRngWin) ? (unsigned)uni((int)sRng[o])
                                                               : (unsigned)uni((int)d.R()[(size_t)t * gW + cursor]);
                    for (int k = uni((int)(w % (unsigned)cnt)); k > 0; --k) lst &= lst - 1ull;
                }
                ++cursor;
                ci = uni(__builtin_ctzll(lst));
            }
            v = uni(uni(sB[x].x) + ci);
#endif
        }
        if (Dn + 1 >= PS) {
            err |= kErrPath;
            break;
        }
        xprev = x;
        x = v;
        ++Dn;
        if (Dn < kWave) px = wl(px, x, Dn);
        else if (REC && l == 0) sPath[Dn] = make_int2(x, 0);
        v = uni(nxt[x]);
        if (v >= 0) ++cursor;
    }
    if (cursor > gW) err |= kErrRng;  // a consumed word beyond the stream
    if (Dn == 0) err |= kErrRoot;
}

// select_path (cnode.cpp:381-413) over the scores of tree_select_prep's S1 (sSc: every node's ucb_score
// under its parent after this back-propagation; sQ: its visits).  The interface and outcomes of
// tree_chase: per level one LDS round trip for the children's scores, structure records and visits
// (lane j = child j), the first maximum by a DPP row max (a wave max past 16 children) and
// select_child's tie list (cnode.cpp:355-370) in closed form, one engine word per non-empty list
// (gen() % size, cnode.cpp:373-377), the next level's records from the chosen lane.
template <int NC, bool REC>
__device__ __forceinline__ void score_walk(unsigned char *smem, const Dev &d, int t, int gW, int wbase, int wsh,
                                           int PS, int &cursor, int &err, int &Dn, int &x, int &xprev, int &px,
                                           int &nbw) {
    using L = TreeLayout<NC>;
    const int l = lane_id();
    const int4 *sA = (const int4 *)(smem + L::oA);
    const int4 *sB = (const int4 *)(smem + L::oB);
    const float *sSc = (const float *)(smem + L::oPS);
    const int *sVis = (const int *)(smem + L::oQ);
    int2 *sPath = (int2 *)(smem + L::oPath);
    const unsigned *sRng = (const unsigned *)(smem + L::oRng);
    cursor = uni(cursor);
    int xv = uni(sA[0].x) + 1;  // the root is on every back-propagated path
    int xb_x = uni(sB[0].x), xb_y = uni(sB[0].y);
    x = 0;
    while (true) {
        const int nc = uni(nc_of(xb_y));
        if (nc == 0) break;  // a leaf
        const int fc = uni(xb_x);
        const bool has = l < nc;
        float sc = -INFINITY;
        int cbx = 0, cby = 0, cvis = 0;
        if (has) {
            sc = sSc[fc + l];
            const int2 cb = *(const int2 *)&sB[fc + l];
            cbx = cb.x;
            cby = cb.y;
            cvis = sVis[fc + l];
        }
        int ci = 0;
        if (x == 0 && xv <= nc) {
            ci = xv - 1;  // forced root round-robin (cnode.cpp:398-399): no word
        } else {
            const int np = xv - 1;  // total_children_visit_counts = node->visit_count - 1
            if (np < 0 || np >= PS) {
                err |= kErrTable;
                break;
            }
            float M;
            if (nc <= 16) {  // one DPP row holds every child
                float v = sc;
                v = fmaxf(v, i2f(dpp<0xB1>(f2i(v))));
                v = fmaxf(v, i2f(dpp<0x4E>(f2i(v))));
                v = fmaxf(v, i2f(dpp<0x141>(f2i(v))));
                v = fmaxf(v, i2f(dpp<0x140>(f2i(v))));
                M = unif(v);
            } else {
                M = unif(wave_max(sc));
            }
            unsigned long long lst;
            if (M > -1000000.0f) {  // FLOAT_MIN (utils.h:12)
                const unsigned long long first = ballot(has && sc == M);
                const int r = uni(__builtin_ctzll(first));
                lst = ballot(has && sc >= M - 0.000001f) & (~0ull << r);
            } else {
                lst = ballot(has && sc >= -1000000.0f);
            }
            const int cnt = uni(__popcll(lst));
            if (cnt > 0) {
                if (cursor >= gW) {
                    err |= kErrRng;
                    break;
                }
                if (cnt > 1) {  // ties: the engine word modulo the list size picks the listed child
                    const int o = cursor - wbase + wsh;
                    const bool inwin = o >= wsh && o < kRngWin;
                    if (!inwin) ++nbw;  // (MZ_S_RNG_TIE_BEYOND)
                    const unsigned w = inwin ? (unsigned)uni((int)sRng[o]) : (unsigned)uni((int)d.R()[(size_t)t * gW + cursor]);
                    for (int k = uni((int)(w % (unsigned)cnt)); k > 0; --k) lst &= lst - 1ull;
                }
                ++cursor;
                ci = uni(__builtin_ctzll(lst));
            }
        }
        if (Dn + 1 >= PS) {
            err |= kErrPath;
            break;
        }
        xprev = x;
        x = uni(fc + ci);
        ++Dn;
        if (Dn < kWave) px = wl(px, x, Dn);
        else if (REC && l == 0) sPath[Dn] = make_int2(x, 0);
        xv = uni(rl(cvis, ci));
        xb_x = uni(rl(cbx, ci));
        xb_y = uni(rl(cby, ci));
    }
    if (Dn == 0) err |= kErrRoot;
}

// the precomputed classes' selection from the state tree_select_prep left: score_walk or tree_chase
template <int NC, bool REC>
__device__ __forceinline__ void tree_select(unsigned char *smem, const Dev &d, int t, int gW, int wbase, int wsh, int PS,
                                            int &cursor, int &err, int &Dn, int &x, int &xprev, int &px, int &nbw) {
    if constexpr (kTreeScoreWalk<NC>)
        score_walk<NC, REC>(smem, d, t, gW, wbase, wsh, PS, cursor, err, Dn, x, xprev, px, nbw);
    else
        tree_chase<NC, REC>(smem, d, t, gW, wbase, wsh, PS, cursor, err, Dn, x, xprev, px, nbw);
}

template <int NC, bool SEL = true>  // SEL = false: the last expansion of a search (mz_expand_backup)
__global__ __launch_bounds__(kTreeWavesN<NC> * 64) void k_tree(char *base, const float *policy, const float *beta, int P, int PS,
                                              int BA, int pk, int hsx, int K, float discount, int fast_ok,
                                              const float *reward, const float *value, const char *pool,
                                              long long pool_stride, long long row_bytes, char *gather_out,
                                              int *idx_x, int *idy, int *act) {
    // Each wave role runs to its own return: no control-flow join follows the split, so the
    // compiler's wait-count state of one role (its loads, stores and LDS-DMA) never forces waits
    // into another's code.  The barriers are the same two s_barrier in every role.
    using L = TreeLayout<NC>;
    // fast_ok bit 1: one workgroup per CU (B <= the CU count), where wave 1 gathers the leaf's row;
    // with two workgroups sharing a CU its copy of the chase competes for the other's SIMDs
    // (3s5z K = 5, 512 trees: +0.5 us per launch), so wave 0 gathers there
    const bool w1g = kTreeW1Gather<NC> && (fast_ok & 2) != 0;
    // the level-walk classes with one workgroup per CU: wave 0 hands the leaf's parent over through
    // LDS (xi[56]: 0 pending, index + 1, or -1 for none) and wave 1 gathers the row, in parallel
    // with wave 0's epilogue
#ifdef MZ_NO_LVG
    constexpr bool lvg = false;
#else
    const bool lvg = SEL && kTreeLevels<NC> && pool != nullptr && (fast_ok & 2) != 0;
#endif
    const int B = BA & 0xffffff, A = (int)((unsigned)BA >> 24);
    const int pe = pk & 0x1ffff, gK = (int)((unsigned)pk >> 17);
    const int ne = (1ll + (long long)gK * (pe - 1)) < P ? 1 + gK * (pe - 1) : P;  // node bound (launch_step)
    Dev d;
    d.base = (gchar *)base;
    arena_hot(d, B, P, PS);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    int4 *sA = (int4 *)(smem + L::oA);
    int4 *sB = (int4 *)(smem + L::oB);
    float *sPP = (float *)(smem + L::oPP);
    float *sQ = (float *)(smem + L::oQ);
    int *sPar = (int *)(smem + L::oPar);
    float *sPS = (float *)(smem + L::oPS);
    int *sFl = (int *)(smem + L::oFl);
    float2 *sAz = (float2 *)(smem + L::oAz);
    int2 *sPath = (int2 *)(smem + L::oPath);
    float *spb = (float *)(smem + L::oPb);
    double *ssq = (double *)(smem + L::oSq);
    float *sLp = (float *)(smem + L::oLp);
    unsigned *sRng = (unsigned *)(smem + L::oRng);
    float *xf = (float *)(smem + L::oX);
    int *xi = (int *)(smem + L::oX);
    long long *xl = (long long *)(smem + L::oX + 64);
    const int t = blockIdx.x;
    const int l = threadIdx.x & (kWave - 1);
    // wave roles: 0 expands, 1 .. 4 back-propagate (2 and 3 also stage).  Five waves on four SIMDs:
    // one SIMD holds two, so the lightest roles, 3 and 4, get hardware waves 0 and 4 (wave w on SIMD
    // w % 4); role 4 ends at barrier (2), before the scores and tie lists of roles 0 .. 3
    // (eight waves: hardware waves w and w + 4 share SIMD w % 4; roles 0 .. 3 -- the expansion, the
    // root, path levels 1 and 2 -- get one SIMD each, paired with the roles of the deepest levels 6,
    // 5, 4, 3, which also take the prior-score blocks)
    constexpr int BK = kBkN<NC>;
    const int hw = (int)(threadIdx.x >> 6);
    const int wv = uni(BK == 4 ? (hw == 0 ? 3 : (hw == 4 ? 4 : hw - 1)) : (hw < 4 ? hw : BK + 4 - hw));
    BkOut *xbo = (BkOut *)(smem + L::oXB);
    const size_t nb = (size_t)t * P;
    unsigned long long ts[10] = {0};
#ifdef MZ_STAMPS_WALK
    unsigned long long tw[9] = {0};
#endif
    stamp(ts, 0);
    const unsigned long long rt0 = span_open();
    const cTreeHdr *hp0 = (const cTreeHdr *)(d.hdr() + t);
    const cParams *pl = (const cParams *)__builtin_assume_aligned(base, 256);

    if (wv >= 2) {
        // ======== waves 2 .. kBk: stage the node records (waves 2, 3); back-propagate their path
        // levels; then the prior scores after the back-propagation and the min/max over the visited
        // nodes off the path ========
        // (the helper role: the leaf's beta, one action per lane, first)
        const bool cdf_helper = kTreeHelperCdf && wv == BK && A >= 2;
        float hbet = 0.f;
        if (cdf_helper && l < A) hbet = beta[(size_t)t * A + l];
        int2 bp0, bp1;
        bk_path_records<BK>(d, t, PS, wv - 1, bp0, bp1);
        const float omr = pl->g.one_minus_rho, gdel = pl->g.delta;  // (issued with the header's loads)
        if constexpr (!kTreeLevels<NC>) bk_pin_offsets(d);  // (the 1024-node class: measured slower)
        const bool al = (P & 3) == 0;  // the tree's 4-byte arrays start 16-byte aligned
        if (kStageVgpr && wv == 2) {
            stage_regs16x2<(NC >= 512 ? 4 : NC / kWave)>(d.A() + nb, sA, d.Bn() + nb, sB, ne);
        } else if (kStageVgpr && wv == 3) {
            stage_regs4x3<(NC >= 512 ? 8 : NC / kWave)>(d.PP() + nb, sPP, d.Q() + nb, sQ, d.Par() + nb, sPar, ne);
        } else if (wv == 2) {
            dma_dwords(d.A() + nb, lds_addr(smem) + L::oA, 4 * ne, true);
            dma_dwords(d.Bn() + nb, lds_addr(smem) + L::oB, 4 * ne, true);
        } else if (wv == 3) {
            dma_dwords(d.PP() + nb, lds_addr(smem) + L::oPP, ne, al);
            dma_dwords(d.Q() + nb, lds_addr(smem) + L::oQ, ne, al);
            dma_dwords(d.Par() + nb, lds_addr(smem) + L::oPar, ne, al);
        } else if (kTreeCStage && kTreeCW4<NC> && wv == 4) {  // wave 4: the value-set scalars (kTreeCW4)
            for (int i0 = 0; i0 < ne; i0 += kWave)
                if (i0 + l < ne)
                    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(d.C() + nb + i0 + l), "s"(lds_addr(smem) + (unsigned)(L::oCn + 16 * i0)) : "memory", "m0");
        }
#ifdef MZ_ABL_LINES  // experiment: MZ_ABL_LINES x 16 extra cache lines in round 1 (value entries, discarded)
        if (wv == 2) {
            const int2 *gVt = (const int2 *)(d.base + (size_t)pl->d.o_V * 256) + (size_t)t * P * pl->g.E;
            for (int k = 0; k < MZ_ABL_LINES; ++k) glds16a((const char *)gVt + 1024 * k + 16 * l, smem + L::oReg + 1024 * k);
        }
#endif
        if (SEL && !kTreePbTable<NC> && wv == 3) {  // the pUCT factors per parent visit count (no gathers)
            dma_dwords(d.pb(), lds_addr(smem) + L::oPb, PS, true);
            dma_dwords(d.sq(), lds_addr(smem) + L::oSq, 2 * PS, true);
        }
        const int herr = hp0->err, tot = hp0->tot, D = hp0->D;
        if (herr) {
            wait_vm();
            return;
        }
        Geo g;
        g.B = B;
        g.A = A;
        g.K = gK;
        g.P = P;
        g.PS = PS;
        g.E = PS - 1;  // (S + 1)
        g.one_minus_rho = omr;
        if (tot > ne)  // slow path: the host bound was too small (a graph replayed out of sequence)
            for (int i0 = ne; i0 < tot; i0 += kWave)
                if (i0 + l < tot) {
                    if (wv == 2) {
                        glds16a(d.A() + nb + i0 + l, sA + i0);
                        glds16a(d.Bn() + nb + i0 + l, sB + i0);
                        if (kTreeCStage) glds16a(d.C() + nb + i0 + l, (float4 *)(smem + L::oCn) + i0);  // (wave 0 stages ne)
                    } else if (wv == 3) {
                        glds4a(d.PP() + nb + i0 + l, sPP + i0);
                        glds4a(d.Q() + nb + i0 + l, sQ + i0);
                        glds4a(d.Par() + nb + i0 + l, sPar + i0);
                    }
                }
        // this wave's path levels' value entries: issued last, in flight across barrier (1)
        const BkPre pre = bk_prestage<BK, kBkCapN<NC>>(d, t, P, g.E, D, wv - 1, bp0, bp1, (int2 *)(smem + L::oReg));
        wait_vm_but(pre.ndma);
        if (cdf_helper) {
            // the leaf's CDF for wave 0's draws: cp[a] in oU (oIx: the weights' broadcast scratch, free
            // until the epilogue)
            double *hcp = (double *)(smem + L::oU);
            const double cp = cdf_bcast(hbet, A, (float *)(smem + L::oIx), hcp);
            hcp[l] = cp;  // (after this wave's own reads of the probabilities there)
        }
        stamp(ts, 1);
        lds_barrier();  // (1)
        stamp(ts, 2);
        // this wave's path levels first (the back-propagation is the critical path)
        const float r_in = unif(xf[60]), v_in = unif(xf[61]);  // (wave 1 staged them)
        Lds s{};
        s.A = sA;
        s.B = sB;
        s.PP = sPP;
        s.path = sPath;
        s.lp = sLp;
        float *boot = (float *)(smem + L::oBoot) + (wv - 1) * (L::PSx + kWave);
        bk_boot(s, boot, D, v_in, r_in, discount);
        int berr = 0;
        long long ber = 0, bew = 0;
        float bmn, bmx;
        bk_levels<BK, kBkCapN<NC>, kTreeAzLevel<NC>>(g, d, s, (const float4 *)(smem + L::oCn), sAz, boot, (int2 *)(smem + L::oReg), pre, t, D, r_in,
                  discount, wv - 1, berr, ber, bew, bmn, bmx);
        stamp(ts, 3);
        // nodes 1 .. tot-1 in 64-node blocks dealt round-robin over waves 2 .. kBk, the deepest
        // path levels' wave first: wave kBk takes blocks 0, kBk - 1, .. (its levels, kBk - 1, ..,
        // are the shallowest work), wave 2 (levels 1, kBk + 1, ..) the last of each round
        constexpr int NPW = BK - 1;
        constexpr int NBW = (NC + NPW * kWave - 1) / (NPW * kWave);
        const float *T = d.T();
        (void)T;
        float pbc[NBW];
        float mn = INFINITY, mx = -INFINITY;
        int cv = 0;
#pragma unroll
        for (int k = 0; k < NBW; ++k) {
            const int n = (NPW * k + BK - wv) * kWave + l;
            pbc[k] = 0.f;
            if (n >= 1 && n < tot) {
                const int4 a = sA[n];
                const int p = sPar[n];
                const int np = sA[p].x + (sFl[p] ? 1 : 0) - 1;  // the parent's total child visits, after
                const int fn = sFl[n];
                int v = a.x + (fn ? 1 : 0);
                if (SEL && np >= 0 && np < PS) {
                    if (v > np) v = np;  // (not in a consistent tree; as the host table's range)
                    // pb_c (cnode.cpp:313-314): the host-built table for the 1024-node class (its many
                    // nodes make the double division cost more than the gathers), else from the
                    // staged per-n factors with the same double arithmetic
                    if constexpr (kTreePbTable<NC>) pbc[k] = T[np * (np + 1) / 2 + v];
                    else pbc[k] = (float)((double)spb[np] * (ssq[np] / (double)(v + 1)));
                }
                if (a.x > 0 && !fn) {
                    const float q = sQ[n];
                    mn = fminf(mn, q);
                    mx = fmaxf(mx, q);
                    ++cv;
                }
            }
        }
        if constexpr (SEL) {
#pragma unroll
            for (int k = 0; k < NBW; ++k) {
                const int n = (NPW * k + BK - wv) * kWave + l;
                if (n >= 1 && n < tot) sPS[n] = pbc[k] * i2f(sA[n].y);  // pb_c * prior (cnode.cpp:316)
            }
        }
        cv = wave_sum(cv);
        mn = fminf(wave_min_to63(mn), bmn);  // (with this wave's path nodes)
        mx = fmaxf(wave_max_to63(mx), bmx);
        if (l == 63) {
            xbo[wv].mn = mn;
            xbo[wv].mx = mx;
        }
        if (l == 0) {
            xbo[wv].cv = cv;
            xbo[wv].err = berr;
            xbo[wv].er = ber;
            xbo[wv].ew = bew;
        }
        if (l == 0 && wv < 4) {
            if (MZ_STAMPS) {
                xl[wv + 2] = (long long)(ts[1] - ts[0]);  // (xl[4], xl[5]) arrival at barrier (1)
                xl[wv + 4] = (long long)(ts[3] - ts[2]);  // (xl[6], xl[7]) its path levels
                xl[wv + 6] = (long long)(__builtin_amdgcn_s_memtime() - ts[2]);  // (xl[8], xl[9]) all work after (1)
            }
        }
#ifdef MZ_SPANS_B2
        if (l == 0) xl[1 + wv] = (long long)span_mark();  // (diagnostic: arrival at barrier (2))
#endif
        lds_barrier();  // (2)
        if (SEL && !kTreeLevels<NC> && wv < kSelW<NC>) {
            const int ncl = uni(xi[15]), err = bk_err<NC>(smem) | uni(xi[14]);
            tree_select_prep<NC>(smem, wv, err ? tot : tot + ncl, discount, gdel, PS, D);
            if (wv == 2 && !err) {  // (every fused launch of the precomputed classes: see wave 0's header)
                // where wave 1 gathers the row and writes the path record, this wave runs a third
                // copy of the chase and writes the header but its tame flag (wave 0's), so that wave
                // 0's epilogue is the selection outputs and the counters
                const int gW2 = pl->g.W;
                d.o_R = pl->d.o_R;
                int cur = uni(xi[58]), Dn = 0, x = 0, xprev = 0, px = 0, e = 0, nbw = 0;
                tree_select<NC, false>(smem, d, t, gW2, uni(xi[62]), uni(xi[59]), PS, cur, e, Dn, x, xprev, px, nbw);
                if (!e) {
                    TreeHdr *hp = d.hdr() + t;
                    const int wb = uni(xi[62]), ws = uni(xi[59]);
                    const int o0 = cur - wb + ws;
                    const unsigned *sRng2 = (const unsigned *)(smem + L::oRng);
                    if (uni((int)(o0 >= ws && o0 + kNxt <= kRngWin))) {
                        if (l < kNxt) hp->nxt[l] = sRng2[o0 + l];
                    } else {  // beyond the window (rare)
                        unsigned *scr = (unsigned *)(smem + L::oIx);
                        const int w = cur + l < gW2 ? cur + l : gW2 - 1;
                        glds4a(d.R() + (size_t)t * gW2 + w, scr);
                        wait_vm();
                        if (l < kNxt) hp->nxt[l] = (cur + l < gW2) ? scr[l] : 0u;
                    }
                    float mn2, mx2;
                    int cnt2;
                    bk_minmax<NC>(smem, D, mn2, mx2, cnt2);
                    if (l == 0) {
                        hp->cursor = cur;
                        hp->tot = tot + ncl;
                        hp->D = Dn;
                        hp->err = 0;
                        hp->mm_min = mn2;
                        hp->mm_max = mx2;
                        hp->mm_cnt = cnt2;
                        hp->leaf = x;
                    }
                }
            }
        }
        wait_vm();  // nothing of this wave may be in flight when the block ends
        return;
    }

    if (wv == 1) {
        // ======== wave 1: CTree::back_propagate (cnode.cpp:415-450) of its levels ========
        int2 bp0, bp1;
        bk_path_records<BK>(d, t, PS, 0, bp0, bp1);
        const float omr = pl->g.one_minus_rho, gdel = pl->g.delta;  // (issued with the header's loads)
        const int gW1 = pl->g.W;
        d.o_R = pl->d.o_R;  // (its copy of the chase reads words past the LDS window from the stream)
        if constexpr (!kTreeLevels<NC>) bk_pin_offsets(d);  // (the 1024-node class: measured slower)
        dma_dwords(d.lp(), lds_addr(smem) + L::oLp, PS + 1, true);
        unsigned long long tw1[4] = {0};
        stamp(tw1, 0);
        const int herr = hp0->err, tot = hp0->tot, D = hp0->D;
        // this simulation's reward and value for every wave, through LDS-DMA (a scalar load would
        // hold up every later LDS wait of the wave behind its two scalar round trips)
        if (l == 0) {
            glds4a(reward + t, xf + 60);
            glds4a(value + t, xf + 61);
        }
        Geo g;
        g.B = B;
        g.A = A;
        g.K = gK;
        g.P = P;
        g.PS = PS;
        g.E = PS - 1;  // (S + 1)
        g.one_minus_rho = omr;
        if (herr) {
            wait_vm();
            return;
        }
        stamp(tw1, 1);
        const BkPre pre = bk_prestage<BK, kBkCapN<NC>>(d, t, P, g.E, D, 0, bp0, bp1, (int2 *)(smem + L::oReg));
        stamp(tw1, 2);
        wait_vm_but(pre.ndma);  // the lambda powers, reward and value (the entries stay in flight)
        stamp(tw1, 3);
        stamp(ts, 2);
        lds_barrier();  // (1)
        stamp(ts, 1);
        const float r_in = unif(xf[60]), v_in = unif(xf[61]);
        Lds s{};
        s.A = sA;
        s.B = sB;
        s.PP = sPP;
        s.path = sPath;
        s.lp = sLp;
        float *boot = (float *)(smem + L::oBoot);
        bk_boot(s, boot, D, v_in, r_in, discount);
        unsigned long long tl[4] = {0};
        stamp(tl, 3);
        int err = 0;
        long long ent_r = 0, ent_w = 0;
        float pmn, pmx;
        bk_levels<BK, kBkCapN<NC>, kTreeAzLevel<NC>>(g, d, s, (const float4 *)(smem + L::oCn), sAz, boot, (int2 *)(smem + L::oReg), pre, t, D, r_in,
                  discount, 0, err, ent_r, ent_w, pmn, pmx, tl);
        if (l == 0) {
            xbo[1].mn = pmn;
            xbo[1].mx = pmx;
            xbo[1].cv = 0;
            xbo[1].err = err;
            xbo[1].er = ent_r;
            xbo[1].ew = ent_w;
            if (MZ_STAMPS) {
                xl[2] = (long long)(__builtin_amdgcn_s_memtime() - ts[1]);  // its path levels
                xl[3] = (long long)(ts[2] - ts[0]);                          // arrival at barrier (1)
                xl[15] = (long long)(tl[3] - ts[1]);                         // bootstrap values
                xl[16] = (long long)(tw1[1] - ts[0]);                        // round 1: header landed
                xl[17] = (long long)(tl[1] - tl[0]);                         // level 0 (the root)
                xl[18] = (long long)(tw1[3] - tw1[1]);                       // round 1: pre-stage, path landed
            }
        }
#ifdef MZ_SPANS_B2
        if (l == 0) xl[2] = (long long)span_mark();  // (diagnostic: arrival at barrier (2))
#endif
        lds_barrier();  // (2): its global stores stay in flight
        if constexpr (SEL && !kTreeLevels<NC>) {
            const int ncl = uni(xi[15]);
            int e = bk_err<NC>(smem) | uni(xi[14]);
            tree_select_prep<NC>(smem, 1, e ? tot : tot + ncl, discount, gdel, PS, D);
            if (w1g && pool && !e) {
                // the leaf's hidden-state row (mcts_sampled.py:130-134): pool[parent's hsx][t], after
                // this wave's copy of wave 0's chase; while the row's loads are in flight, the path
                // record {node, visits at selection} for the next back-propagation and the scored
                // children's count (wave 0's epilogue leaves both to this wave)
                int cur = uni(xi[58]), Dn = 0, x = 0, xprev = 0, px = 0, nbw = 0;
                tree_select<NC, true>(smem, d, t, gW1, uni(xi[62]), uni(xi[59]), PS, cur, e, Dn, x, xprev, px, nbw);
                auto write_path = [&]() {
                    int2 *gp = d.path() + (size_t)t * PS;
                    const int2 *sPath1 = (const int2 *)(smem + L::oPath);
                    const int *sFl1 = (const int *)(smem + L::oFl);
                    const int4 *sA1 = (const int4 *)(smem + L::oA);
                    int nsc = 0;
                    for (int i0 = 0; i0 <= Dn; i0 += kWave) {
                        const int i = i0 + l;
                        if (i <= Dn) {
                            const int xi_ = (i < kWave) ? px : sPath1[i].x;
                            const int vis = sA1[xi_].x + (sFl1[xi_] ? 1 : 0);
                            gp[i] = make_int2(xi_, vis);
                            const int nci = nc_of(sB[xi_].y);
                            if (i < Dn && !(i == 0 && vis <= nci)) nsc += nci;  // scored levels
                        }
                    }
                    const long long nscored = wave_sum(nsc);
                    const long long *sSt1 = (const long long *)(smem + L::oSt);
                    if (l == 0) d.stats()[(size_t)t * MZ_S_COUNT + MZ_S_SCORED] = sSt1[MZ_S_SCORED] + nscored;
                };
                if (!e) {
                    const int oi = uni(sB[Dn == 0 ? 0 : xprev].w);  // parent->hidden_state_index_x
                    const char *src = pool + (long long)oi * pool_stride + (long long)t * row_bytes;
                    char *gdst = gather_out + (long long)t * row_bytes;
                    const bool al = ((row_bytes | pool_stride | (long long)(uintptr_t)pool |
                                      (long long)(uintptr_t)gather_out) & 15) == 0;
                    const long long o = (long long)l * 16, last = row_bytes - 16;
                    if (al && row_bytes >= 16 && row_bytes <= 4 * 16 * kWave) {
                        // up to 4 KiB: four 16-byte loads per lane issued together (offsets clamped
                        // into the row, so no load is conditional), then the stores
                        const int4 v0 = *(const int4 *)(src + (o < last ? o : last));
                        const int4 v1 = *(const int4 *)(src + (o + 1024 < last ? o + 1024 : last));
                        const int4 v2 = *(const int4 *)(src + (o + 2048 < last ? o + 2048 : last));
                        const int4 v3 = *(const int4 *)(src + (o + 3072 < last ? o + 3072 : last));
                        write_path();
                        if (o < row_bytes) *(int4 *)(gdst + o) = v0;
                        if (o + 1024 < row_bytes) *(int4 *)(gdst + o + 1024) = v1;
                        if (o + 2048 < row_bytes) *(int4 *)(gdst + o + 2048) = v2;
                        if (o + 3072 < row_bytes) *(int4 *)(gdst + o + 3072) = v3;
                    } else if (al) {
                        for (long long o2 = o; o2 < row_bytes; o2 += 16 * kWave) *(int4 *)(gdst + o2) = *(const int4 *)(src + o2);
                        write_path();
                    } else {
                        for (long long o2 = (long long)l * 4; o2 < row_bytes; o2 += 4 * kWave)
                            *(int *)(gdst + o2) = *(const int *)(src + o2);
                        write_path();
                    }
                }
            }
        }
        if (lvg) {
            // wait for wave 0's walk (LDS-coherent within the workgroup; bounded, and wave 0 writes
            // the slot on every path after barrier (2))
            volatile int *slot = (volatile int *)(xi + 56);
            int v = 0;
            for (int it = 0; it < (1 << 22); ++it) {
                v = uni(*slot);
                if (v != 0) break;
                __builtin_amdgcn_s_sleep(1);
            }
            if (v > 0) {  // mcts_sampled.py:130-134: pool[parent's hsx][t]
                const char *src = pool + (long long)(v - 1) * pool_stride + (long long)t * row_bytes;
                char *gdst = gather_out + (long long)t * row_bytes;
                const bool al = ((row_bytes | pool_stride | (long long)(uintptr_t)pool |
                                  (long long)(uintptr_t)gather_out) & 15) == 0;
                if (al) {  // sixteen 16-byte loads per lane in flight, then their stores, written through
                    for (long long o0 = (long long)l * 16; o0 < row_bytes; o0 += 16 * 16 * kWave) {
                        int4 rv[16];
#pragma unroll
                        for (int u = 0; u < 16; ++u) {
                            const long long o = o0 + (long long)u * 16 * kWave;
                            if (o < row_bytes) rv[u] = *(const int4 *)(src + o);
                        }
#pragma unroll
                        for (int u = 0; u < 16; ++u) {
                            const long long o = o0 + (long long)u * 16 * kWave;
                            if (o < row_bytes) st_wt16(gdst + o, rv[u]);
                        }
                    }
                } else {
                    for (long long o2 = (long long)l * 4; o2 < row_bytes; o2 += 4 * kWave)
                        *(int *)(gdst + o2) = *(const int *)(src + o2);
                }
            } else if (v == 0 && l == 0) {
                atomicOr(d.err(), kErrPath);  // (never: wave 0 did not hand over)
            }
        }
        wait_vm();  // nothing of this wave may be in flight when the block ends
        return;
    }

    // ======== wave 0: expansion (cnode.cpp:224-295), selection (381-413), gather, header ========
    // Round 1 is LDS-DMA and scalar loads only, so every wait below is an explicit, counted one:
    // the four window chunks may stay in flight through the draws.
    const bool have_w = 2 * K <= kNxt;  // the expansion's words are in the header
    float *sW = (float *)(smem + L::oW);
    float *sPol = (float *)(smem + L::oPol);
    unsigned *sNxt = (unsigned *)(smem + L::oNxt);
    long long *sSt = (long long *)(smem + L::oSt);
    long long *st = d.stats() + (size_t)t * MZ_S_COUNT;
    constexpr int kStatN = (MZ_STAMPS != 0) ? MZ_S_COUNT : MZ_S_CYC_HEADER;
    {
        // the path (the flags below; the back-propagation waves read it after barrier (1)): wave 0
        // has the slack before barrier (1), wave 1's round 1 is the longest
        dma_dwords(d.path() + (size_t)t * PS, lds_addr(smem) + L::oPath, 2 * pe, (PS & 1) == 0);
        const size_t ib = (size_t)t * A + (l < A ? l : 0);
        glds4a(policy + ib, sPol);
        glds4a(beta + ib, sW);  // (lanes >= A: zero weights, below)
        glds4a(&d.hdr()[t].nxt[l < kNxt ? l : 0], sNxt);
        glds4a((const int *)st + (l < 2 * MZ_S_COUNT ? l : 0), (int *)sSt);
        // the value-set scalars of the nodes (the back-propagation waves' path nodes read them)
        if constexpr (kTreeCStage && !kTreeCW4<NC>)
        for (int i0 = 0; i0 < ne; i0 += kWave)
            if (i0 + l < ne)
                asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(d.C() + nb + i0 + l), "s"(lds_addr(smem) + (unsigned)(L::oCn + 16 * i0)) : "memory", "m0");
    }
    const float t00 = ldsc(d.T());  // pb_c(0, 0): the coefficient of the leaf's new children
    TreeHdr h;
    h.cursor = hp0->cursor;
    h.tot = hp0->tot;
    h.D = hp0->D;
    h.err = hp0->err;
    h.tame = hp0->tame;
    h.leaf = hp0->leaf;
    h.mm_min = hp0->mm_min;  // (the normaliser before this back-propagation: MZ_S_MM_MOVED)
    h.mm_max = hp0->mm_max;
    h.mm_cnt = hp0->mm_cnt;
    // (held from here in the level-walk classes: left to the compiler, these were reloaded from the
    // header by scalar loads where they are used, in the epilogue, each with a wait for its round
    // trip; same-box A/B, 27m K = 5 11.91 -> 11.78 us.  The other classes' SGPR pressure makes it a
    // loss there: 3m K = 5 7.54 -> 7.61)
    if constexpr (kTreeLevels<NC>) asm volatile("" : "+s"(h.tame), "+s"(h.mm_min), "+s"(h.mm_max), "+s"(h.mm_cnt));
    const int gW = pl->g.W;
    const float gdelta = pl->g.delta;
    d.o_D = pl->d.o_D;
    d.o_R = pl->d.o_R;
    const int wbase = h.cursor;
    // pb_c(0, 0) pinned to an SGPR here, with the header's scalar round trip: left to the compiler the
    // load sank to its use in the expansion as a vector load, whose wait (vmcnt(0)) also waited for
    // the new children's stores there and left a vmcnt(0) in the score pass behind it
    asm volatile("" ::"s"(t00));
    // the selection's engine words (the expansion's when K > kNxt / 2): word wbase + o is sRng[o + wsh].
    // One 16-byte chunk per lane from the aligned word below wbase when the window lies inside the
    // stream (the tree's stream starts 16-byte aligned: W is a multiple of 624), else four dword chunks.
    const int wsh = ((gW & 3) == 0 && (wbase & ~3) + kRngWin <= gW) ? (wbase & 3) : 0;
    {
        const unsigned *Rt = d.R() + (size_t)t * gW;
        if ((gW & 3) == 0 && (wbase & ~3) + kRngWin <= gW) {
            asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(Rt + (wbase & ~3) + 4 * l), "s"(lds_addr(smem) + (unsigned)L::oRng) : "memory", "m0");
        } else {
#pragma unroll
            for (int i0 = 0; i0 < kRngWin; i0 += kWave) {
                const int w = wbase + i0 + l;
                glds4a(Rt + (w < gW ? w : gW - 1), sRng + i0);
            }
        }
    }
    for (int i0 = 0; i0 < ne; i0 += kWave)  // path-node flags cleared while round 1 is in flight
        if (i0 + l < ne) sFl[i0 + l] = 0;
    if ((gW & 3) == 0 && (wbase & ~3) + kRngWin <= gW) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // round 1 landed (the window may not have)
    unsigned long long tq[4] = {0};
    stamp(tq, 0);
    if (h.err) {  // a dead tree stays dead (every wave reads the same header) and re-reports its error
        if (l == 0) {
            if (SEL) {
                idx_x[t] = 0;
                idy[t] = t;
                act[t] = 0;
            }
            atomicOr(d.err(), h.err);
        }
        wait_vm();
        return;
    }
    const int tot = h.tot, D = h.D;
    if (D + 1 > pe) {  // a path beyond the host bound (a graph replayed out of sequence)
        for (int i0 = 2 * pe; i0 < 2 * (D + 1); i0 += kWave)
            if (i0 + l < 2 * (D + 1)) glds4a((const int *)(d.path() + (size_t)t * PS) + i0 + l, (int *)sPath + i0);
        wait_vm();
    }
    {  // path-node flags (1 + path level, else 0): the rest cleared, then set from the staged path
        for (int i0 = ne; i0 < tot; i0 += kWave)
            if (i0 + l < tot) sFl[i0 + l] = 0;
        for (int i0 = 0; i0 <= D; i0 += kWave)
            if (i0 + l <= D) {
                const int n = sPath[i0 + l].x;
                if (n >= 0 && n < tot) sFl[n] = i0 + l + 1;
            }
    }
    if (l >= A) sW[l] = 0.f;
    const float pol = sPol[l < A ? l : 0], bet = sW[l < A ? l : 0];
    stamp(ts, 1);
    // (1) every staged record has landed and the path nodes are flagged: waves 1-3 back-propagate
    // and score from here on, while this wave expands
    lds_barrier();
    stamp(ts, 2);
#if !defined(MZ_SPANS_EPI) && !defined(MZ_SPANS_EXP) && !defined(MZ_SPANS_B2)
    const unsigned long long rm1 = span_mark();
#else
    unsigned long long rm1 = 0, rm2 = 0, rm3 = 0;  // (diagnostic marks placed below)
#endif
    const float r_in = unif(xf[60]), v_in = unif(xf[61]);  // (wave 1 staged them)
    // the sampling distribution and the K draws (std::discrete_distribution, two engine words per
    // draw, cnode.cpp:243-262)
    int cursor = h.cursor;
    int cnt = 0;  // draws that hit action l
    int err = 0;
    if (A < 2) {
        cnt = (l == 0) ? K : 0;
    } else {
        double *sp = (double *)(smem + L::oP);
        wait_lds();
        const double cp = kTreeHelperCdf ? ((const double *)(smem + L::oU))[l] : cdf_staged(A, sW, sp);
        if (MZ_STAMPS) {
            asm volatile("" ::"v"(cp));
            stamp(tq, 1);
        }
#ifdef MZ_SPANS_EXP
        asm volatile("" ::"v"(cp));
        rm1 = span_mark();
#endif
        if (!have_w) wait_vm();  // the words come from the window
        double u = 0.0;
        if (l < K) {
            const unsigned a1 = have_w ? sNxt[2 * l] : ((2 * l + wsh < kRngWin) ? sRng[2 * l + wsh] : 0u);
            const unsigned a2 = have_w ? sNxt[2 * l + 1] : ((2 * l + 1 + wsh < kRngWin) ? sRng[2 * l + 1 + wsh] : 0u);
            u = ((double)a1 + (double)a2 * 4294967296.0) / 18446744073709551616.0;
            if (u >= 1.0) u = 0x1.fffffffffffffp-1;  // nextafter(1, 0)
        }
        if (cursor + 2 * K > gW || 2 * K > kRngWin) err |= kErrRng;
        // draw k's lower_bound (the actions whose cumulative probability is below u_k) as one ballot
        // over the CDF, one action per lane; lane a counts the draws that chose action a
        // (four draws per step: their readlanes and ballots issue back to back; the compiler does
        // not unroll a runtime-count loop over convergent operations by itself)
        int k = 0;
        for (; k + 4 <= K; k += 4) {
            const double u0 = rld(u, k), u1 = rld(u, k + 1), u2 = rld(u, k + 2), u3 = rld(u, k + 3);
            const int i0 = __popcll(ballot(l < A && cp < u0)), i1 = __popcll(ballot(l < A && cp < u1));
            const int i2 = __popcll(ballot(l < A && cp < u2)), i3 = __popcll(ballot(l < A && cp < u3));
            cnt += ((i0 == l) ? 1 : 0) + ((i1 == l) ? 1 : 0) + ((i2 == l) ? 1 : 0) + ((i3 == l) ? 1 : 0);
        }
        for (; k < K; ++k) {
            const double uk = rld(u, k);
            const int ix = __popcll(ballot(l < A && cp < uk));
            cnt += (ix == l) ? 1 : 0;
        }
        cursor += 2 * K;
    }
    if (MZ_STAMPS) {
        asm volatile("" ::"v"(cnt));
        stamp(tq, 2);
    }
#ifdef MZ_SPANS_EXP
    asm volatile("" ::"v"(cnt));
    rm2 = span_mark();
#endif
    const long long st_old = (l < kStatN) ? sSt[l] : 0ll;
    // the leaf's children (cnode.cpp:264-293), in ascending action order
    wait_vm();  // the window landed: later waits need not drain this wave's stores
    const int leaf = h.leaf;
    int ncl = 0;
    {
        const bool hasc = (l < A) && cnt > 0;
        const unsigned long long m = ballot(hasc);
        ncl = __popcll(m);
        int wild = 0;
        if (tot + ncl > P) {
            err |= kErrPool;
            ncl = 0;
        } else if (hasc) {
            const int c = tot + __popcll(m & ((1ull << l) - 1ull));
            const float bh = (float)cnt / (float)K;  // betahat_prob = count / sampled_times
            const float prior = pol * bh / bet;      // prior * betahat_prob / beta_prob (no noise below the root)
            if (!tame_prior(prior)) wild = 1;
            const int4 a4 = make_int4(0, f2i(prior), f2i(0.0f), f2i(0.0f));
            const int4 b4 = make_int4(0, pack_y(0, l, -1), f2i(0.0f), -1);
            const size_t gi = nb + c;
            d.A()[gi] = a4;
            d.Bn()[gi] = b4;
            d.C()[gi] = make_float4(0.f, 0.f, 0.f, 0.f);
            d.D()[gi] = make_float4(pol, bet, bh, 0.f);
            d.Q()[gi] = 0.f;
            d.PP()[gi] = v_in;
            d.Par()[gi] = leaf;
            sA[c] = a4;
            sB[c] = b4;
            sPP[c] = v_in;
            sFl[c] = 0;
            sPS[c] = t00 * prior;  // prior score under the leaf after its first visit: pb_c(0, 0) * prior
        }
        if (ballot(wild != 0) || !tame_val(v_in) || !tame_val(r_in)) h.tame = 0;
        if (!err && l == 0) {  // the leaf's structure: first child, children count, pred_value, hidden_state_index_x
            const int ly = sB[leaf].y;
            const int md = md_of(ly) < 0 ? 0 : md_of(ly);
            const int4 nbv = make_int4(tot, pack_y(ncl, act_of(ly), md), f2i(v_in), hsx);
            sB[leaf] = nbv;
            d.Bn()[nb + leaf] = nbv;
        }
    }
#ifdef MZ_SPANS_EXP
    rm3 = span_mark();
#endif
    if (l == 0) {
        xi[56] = 0;  // (the level-walk classes' row hand-over: pending)
        xi[15] = ncl;
        xi[14] = err;
        xi[58] = cursor;  // the selection's first engine word, for wave 1's copy of the chase
        xi[59] = wsh;
        xi[62] = wbase;
    }
    stamp(ts, 3);
#ifdef MZ_SPANS_B2
    const unsigned long long b2own = span_mark();
#endif
    lds_barrier();  // (2) back-propagation, prior scores, min/max partials and the children are in LDS
    stamp(ts, 4);
#if !defined(MZ_SPANS_EPI) && !defined(MZ_SPANS_EXP) && !defined(MZ_SPANS_B2)
    const unsigned long long rm2 = span_mark();
#endif
#ifdef MZ_SPANS_B2  // wave 0's own arrival, the last of roles 1-3, the last of roles 4-7
    rm1 = b2own;
    rm2 = (unsigned long long)xl[2];
    rm3 = (unsigned long long)xl[5];
    for (int j = 3; j <= 4; ++j) rm2 = (unsigned long long)xl[j] > rm2 ? (unsigned long long)xl[j] : rm2;
    for (int j = 6; j <= BK + 1; ++j) rm3 = (unsigned long long)xl[j] > rm3 ? (unsigned long long)xl[j] : rm3;
#endif

    // ---- the selection of the next simulation (cnode.cpp:381-413) ----
    err |= bk_err<NC>(smem);  // the back-propagation waves
    float mmn, mmx;
    int mm_cnt;
    bk_minmax<NC>(smem, D, mmn, mmx, mm_cnt);
    const int moved = (mm_cnt > 0 && (h.mm_cnt == 0 || f2i(mmn) != f2i(h.mm_min) || f2i(mmx) != f2i(h.mm_max))) ? 1 : 0;
    long long ent_r = 0, ent_w = 0;
#pragma unroll
    for (int j = 1; j <= BK; ++j) {
        ent_r += xbo[j].er;
        ent_w += xbo[j].ew;
    }
    const int ntot = err ? tot : tot + ncl;
    unsigned long long tp[4] = {0};
    int Dn = 0, x = 0, out_idx = 0, out_act = 0;
    long long nscored = 0;
    int nbeyond = 0, nxbeyond = 0;  // engine words read past the LDS window: ties, header words
    int px = 0, pvv = 0;  // level i's node (and, by levels, its visits) in lane i; sPath past 64 levels
    if constexpr (!SEL) {
        stamp(ts, 5);
    } else if constexpr (kTreeLevels<NC>) {
        stamp(ts, 5);
#ifdef MZ_STAMPS_WALK
        // (diagnostic builds with -DMZ_STAMPS_WALK -DMZ_STAMPS_W0: wave 0's slots become the walk's
        // root reads, its passes 1..5 (0 past the last), and the exit)
        tw[0] = __builtin_amdgcn_s_memtime();
        int twn = 0;
#define MZ_WALK_TOP()                                                          \
    do {                                                                        \
        const unsigned long long n_ = __builtin_amdgcn_s_memtime();             \
        if (twn == 0) tw[1] = n_; else if (twn == 1) tw[2] = n_;                \
        else if (twn == 2) tw[3] = n_; else if (twn == 3) tw[4] = n_;           \
        else if (twn == 4) tw[5] = n_; else if (twn == 5) tw[6] = n_;           \
        ++twn;                                                                  \
    } while (0)
#else
#define MZ_WALK_TOP() do {} while (0)
#endif
#ifdef MZ_STAMPS_SEG
        // (diagnostic builds with -DMZ_STAMPS_SEG -DMZ_STAMPS_W0: the two-level passes' segments summed
        // over a tree's passes -- children landed, grandchildren landed, scores + ballots, level 1,
        // level 2 -- and the pass count, in wave 0's slots)
        unsigned long long sg0 = 0, sg1 = 0, sg2 = 0, sg3 = 0, sg4 = 0, sgl = 0, sgn = 0;
#define MZ_SEG(acc)                                                            \
    do {                                                                        \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                      \
        const unsigned long long n_ = __builtin_amdgcn_s_memtime();             \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                      \
        acc += n_ - sgl;                                                        \
        sgl = n_;                                                               \
    } while (0)
#else
#define MZ_SEG(acc) do {} while (0)
#endif
    if (!err) {
        cursor = uni(cursor);
        const bool mm_on = mm_cnt > 0;
        float den = 0.f;
        if (mm_on) {
            const float delta = mmx - mmn;
            den = (gdelta < delta) ? delta : gdelta;  // std::max(delta_lb, delta)
        }
        int xv = uni(sA[0].x) + 1;  // the root is on every path
        int4 xb = uni4(sB[0]);
        int par_hsx = xb.w;
        pvv = wl(pvv, xv, 0);
        const int lim8 = PS < kWave ? PS : kWave;  // (walk_step8: path lanes)
        (void)lim8;
        while (true) {
            MZ_WALK_TOP();
            x = uni(x);
            xv = uni(xv);
            cursor = uni(cursor);
            const int nc = uni(nc_of(xb.y));
            if (nc == 0) break;
            const int fc = uni(xb.x);
#ifndef MZ_NO_WALK2
            if (nc <= 7) {
#ifdef MZ_STAMPS_SEG
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                sgl = __builtin_amdgcn_s_memtime();
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                ++sgn;
#endif
                // Two levels per pass (nc <= 7 and every child's nc <= 8): lanes 0..7 hold x's children,
                // lanes 8 + 8g + i child g's child i.  Each lane scores its node as the one-level pass
                // below would at that node's level (the scores depend on the node and the launch's
                // min-max only); one segmented DPP max over eight lanes gives every group's maximum, and
                // the tie lists of all groups come from two ballots.  The first level's outcome picks
                // the group whose list resolves the second; the engine words are consumed in the same
                // order (one per scored level).  Bit-exact with two one-level passes.
                const int g = (l >> 3) - 1;  // -1: x's children
                const int sl = l & 7;
                const bool lo = l < 8;
                const bool has1 = (lo ? sl : g) < nc;
                int4 ca = make_int4(0, 0, 0, 0), cb = ca;
                float cpp = 0.f, cps = 0.f;
                float2 caz = make_float2(0.f, 0.f);
                int cfl = 0;
                const float2 az1 = kTreeAzLevel<NC> ? sAz[Dn + 1] : make_float2(0.f, 0.f);
                const float2 az2 = kTreeAzLevel<NC> ? sAz[Dn + 2] : make_float2(0.f, 0.f);  // Dn + 2 <= PS
                if (has1) {
                    const int n1 = fc + (lo ? sl : g);
                    cb = sB[n1];  // (the groups: their parent's structure record)
                    if (lo) {
                        ca = sA[n1];
                        cpp = sPP[n1];
                        cps = sPS[n1];
                        cfl = sFl[n1];
                        if constexpr (!kTreeAzLevel<NC>) caz = sAz[n1];
                    }
                }
                MZ_SEG(sg0);
                const int gnc = nc_of(cb.y);
                const bool ok2 = ballot(!lo && has1 && gnc > 8) == 0ull;
                const bool has2 = !lo && has1 && sl < gnc;
                if (has2) {
                    const int n2 = cb.x + sl;
                    ca = sA[n2];
                    cb = sB[n2];
                    cpp = sPP[n2];
                    cps = sPS[n2];
                    cfl = sFl[n2];
                    if constexpr (!kTreeAzLevel<NC>) caz = sAz[n2];
                }
                MZ_SEG(sg1);
                if constexpr (kTreeAzLevel<NC>) caz = lo ? az1 : az2;
                const bool has = lo ? has1 : has2;
                const int cvis = ca.x + (cfl ? 1 : 0);
                float sc = -INFINITY;
                if (has) {  // ucb_score (cnode.cpp:297-335), as below
                    const float val = cfl ? caz.x : i2f(ca.z);
                    const float rw = cfl ? caz.y : i2f(ca.w);
                    float vs = (cvis == 0) ? 0.0f : ((rw + discount * val) - cpp);
                    if (mm_on) vs = (vs - mmn) / den;
                    if (vs < 0) vs = 0;
                    if (vs > 1) vs = 1;
                    sc = cps + vs;
                }
                float Ms = sc;  // the maximum of the lane's group of eight
                Ms = fmaxf(Ms, i2f(dpp<0xB1>(f2i(Ms))));
                Ms = fmaxf(Ms, i2f(dpp<0x4E>(f2i(Ms))));
                Ms = fmaxf(Ms, i2f(dpp<0x141>(f2i(Ms))));
                const bool big = Ms > -1000000.0f;
                const unsigned long long bB = ballot(big);
                const unsigned long long bE = ballot(has && sc == Ms);
                const float thr = big ? Ms - 0.000001f : -1000000.0f;
                const unsigned long long bT = ballot(has && sc >= thr);
#ifdef MZ_STAMPS_SEG
                asm volatile("" ::"s"(bT), "s"(bE));
#endif
                MZ_SEG(sg2);
                // one level's select_child from group `base`'s lanes: -1 (err set) ends the walk
                auto pick = [&](int base, int ncl) -> int {
                    if (x == 0 && xv <= ncl) return xv - 1;  // forced root round-robin (cnode.cpp:398-399)
                    const int np = xv - 1;
                    if (np < 0 || np >= PS) {
                        err |= kErrTable;
                        return -1;
                    }
                    nscored += ncl;
                    unsigned long long lst = (bT >> base) & 0xffull;
                    if (i2f(rl(f2i(Ms), base)) > -1000000.0f)
                        lst &= ~0ull << uni(__builtin_ctzll((bE >> base) & 0xffull));
                    const int cntl = uni(__popcll(lst));
                    if (cntl == 0) return 0;
                    if (cursor >= gW) {
                        err |= kErrRng;
                        return -1;
                    }
                    if (cntl > 1) {
                        const int o = cursor - wbase + wsh;
                        if (!(o >= wsh && o < kRngWin)) ++nbeyond;
                        const unsigned w = (o >= wsh && o < kRngWin) ? (unsigned)uni((int)sRng[o])
                                                                   : (unsigned)uni((int)d.R()[(size_t)t * gW + cursor]);
                        for (int k = uni((int)(w % (unsigned)cntl)); k > 0; --k) lst &= lst - 1ull;
                    }
                    ++cursor;
                    return uni(__builtin_ctzll(lst));
                };
                auto advance = [&](int fcl, int ln) -> bool {  // to the child in lane ln
                    if (Dn + 1 >= PS) {
                        err |= kErrPath;
                        return false;
                    }
                    par_hsx = uni(xb.w);
                    x = uni(fcl + (ln & 7));
                    ++Dn;
                    xv = uni(rl(cvis, ln));
                    xb = make_int4(uni(rl(cb.x, ln)), uni(rl(cb.y, ln)), 0, uni(rl(cb.w, ln)));
                    if (Dn < kWave) {
                        px = wl(px, x, Dn);
                        pvv = wl(pvv, xv, Dn);
                    } else if (l == 0) {
                        sPath[Dn] = make_int2(x, xv);
                    }
                    return true;
                };
#ifndef MZ_NO_WALKASM
                // the common case in one straight run (walk_step8); pick and advance otherwise
                auto step8 = [&](int base, int ncl, int fcl) -> int {  // the chosen child (lane - base), or -1
                    const unsigned tT = (unsigned)(bT >> base) & 0xffu, tE = (unsigned)(bE >> base) & 0xffu;
                    const unsigned bg = (unsigned)(bB >> base) & 1u;
                    if (walk_step8(tT, tE, bg, base, ncl, fcl, PS, gW, lim8, x, xv, xb.x, xb.y, xb.w, cursor, Dn,
                                   par_hsx, px, pvv, cvis, cb.x, cb.y, cb.w, l))
                        return -1;
                    nscored += ncl;
                    return x - fcl;  // (x = fcl + the child)
                };
                int ci = step8(0, nc, fc);
                if (ci < 0) {
                    ci = pick(0, nc);
                    if (ci < 0 || !advance(fc, ci)) break;
                }
#else
                const int ci = pick(0, nc);
                if (ci < 0 || !advance(fc, ci)) break;
#endif
                MZ_SEG(sg3);
                if (!ok2) continue;
                const int nc2 = uni(nc_of(xb.y));
                if (nc2 == 0) break;
                const int fc2 = uni(xb.x);
                const int base = 8 + 8 * ci;  // child ci's group: its children at fc2 + i
#ifndef MZ_NO_WALKASM
                if (step8(base, nc2, fc2) < 0) {
                    const int ci2 = pick(base, nc2);
                    if (ci2 < 0 || !advance(fc2, base + ci2)) break;
                }
#else
                const int ci2 = pick(base, nc2);
                if (ci2 < 0 || !advance(fc2, base + ci2)) break;
#endif
                MZ_SEG(sg4);
                continue;
            }
#endif
            // the children's records (lane j = child j), the next level's structure record included
            const bool has = l < nc;
            int4 ca = make_int4(0, 0, 0, 0), cb = ca;
            float cpp = 0.f, cps = 0.f;
            float2 caz = make_float2(0.f, 0.f);
            int cfl = 0;
            // (per-level sAz: a child on the back-propagated path sits at level Dn + 1 of it, since the
            // walk reaches the path's nodes at their own depths; read with the children's records)
            const float2 azl = kTreeAzLevel<NC> ? sAz[Dn + 1] : make_float2(0.f, 0.f);
            if (has) {
                ca = sA[fc + l];
                cb = sB[fc + l];
                cpp = sPP[fc + l];
                cps = sPS[fc + l];
                cfl = sFl[fc + l];
                if constexpr (!kTreeAzLevel<NC>) caz = sAz[fc + l];
            }
            if constexpr (kTreeAzLevel<NC>) caz = azl;
            const int cvis = ca.x + (cfl ? 1 : 0);
            int ci = 0;
            if (x == 0 && xv <= nc) {
                ci = xv - 1;  // forced root round-robin (cnode.cpp:398-399)
            } else {
                const int np = xv - 1;  // total_children_visit_counts = node->visit_count - 1
                if (np < 0 || np >= PS) {
                    err |= kErrTable;
                    break;
                }
                nscored += nc;
                float sc = -INFINITY;
                if (has) {  // ucb_score (cnode.cpp:297-335)
                    const float val = cfl ? caz.x : i2f(ca.z);
                    const float rw = cfl ? caz.y : i2f(ca.w);
                    float vs = (cvis == 0) ? 0.0f : ((rw + discount * val) - cpp);
                    if (mm_on) vs = (vs - mmn) / den;
                    if (vs < 0) vs = 0;
                    if (vs > 1) vs = 1;
                    sc = cps + vs;
                }
                float M;
                if (nc <= 16) {  // one DPP row holds every child
                    float v = sc;
                    v = fmaxf(v, i2f(dpp<0xB1>(f2i(v))));
                    v = fmaxf(v, i2f(dpp<0x4E>(f2i(v))));
                    v = fmaxf(v, i2f(dpp<0x141>(f2i(v))));
                    v = fmaxf(v, i2f(dpp<0x140>(f2i(v))));
                    M = unif(v);
                } else {
                    M = unif(wave_max(sc));
                }
                // select_child's tie list (cnode.cpp:355-370) in closed form: the first maximum and
                // every later child within epsilon of it; {s >= FLOAT_MIN} when no score beats FLOAT_MIN
                unsigned long long lst;
                if (M > -1000000.0f) {
                    const unsigned long long first = ballot(has && sc == M);
                    const int r = uni(__builtin_ctzll(first));
                    lst = ballot(has && sc >= M - 0.000001f) & (~0ull << r);
                } else {
                    lst = ballot(has && sc >= -1000000.0f);
                }
                const int cntl = uni(__popcll(lst));
                if (cntl > 0) {  // one engine word (gen() % size); its value matters only for ties
                    if (cursor >= gW) {
                        err |= kErrRng;
                        break;
                    }
                    if (cntl > 1) {
                        const int o = cursor - wbase + wsh;
                        if (!(o >= wsh && o < kRngWin)) ++nbeyond;
                        const unsigned w = (o >= wsh && o < kRngWin) ? (unsigned)uni((int)sRng[o])
                                                                   : (unsigned)uni((int)d.R()[(size_t)t * gW + cursor]);
                        for (int k = uni((int)(w % (unsigned)cntl)); k > 0; --k) lst &= lst - 1ull;
                    }
                    ++cursor;
                    ci = uni(__builtin_ctzll(lst));
                }
            }
            if (Dn + 1 >= PS) {
                err |= kErrPath;
                break;
            }
            par_hsx = uni(xb.w);
            x = uni(fc + ci);
            ++Dn;
            xv = uni(rl(cvis, ci));
            xb = make_int4(uni(rl(cb.x, ci)), uni(rl(cb.y, ci)), 0, uni(rl(cb.w, ci)));
            if (Dn < kWave) {
                px = wl(px, x, Dn);
                pvv = wl(pvv, xv, Dn);
            } else if (l == 0) {
                sPath[Dn] = make_int2(x, xv);
            }
        }
        if (Dn == 0) err |= kErrRoot;
        out_idx = (Dn == 0) ? uni(sB[0].w) : par_hsx;  // parent->hidden_state_index_x
        out_act = act_of(uni(xb.y));                   // children_action of the last edge
    }
#ifdef MZ_STAMPS_WALK
        {
            const unsigned long long n_ = __builtin_amdgcn_s_memtime();
            if (twn < 1) tw[1] = n_;
            if (twn < 2) tw[2] = n_;
            if (twn < 3) tw[3] = n_;
            if (twn < 4) tw[4] = n_;
            if (twn < 5) tw[5] = n_;
            if (twn < 6) tw[6] = n_;
            tw[7] = n_;
            tw[8] = n_;
        }
#endif
#ifdef MZ_STAMPS_SEG
        tw[0] = 0;
        tw[1] = sg0;
        tw[2] = tw[1] + sg1;
        tw[3] = tw[2] + sg2;
        tw[4] = tw[3] + sg3;
        tw[5] = tw[4] + sg4;
        tw[6] = tw[5];
        tw[7] = tw[6] + sgn;
        tw[8] = tw[7];
#endif
#undef MZ_SEG
#undef MZ_WALK_TOP
        stamp(tp, 3);
    } else {
        // every node's select_child outcome by the four waves (tree_select_prep), then the chase
        tree_select_prep<NC>(smem, 0, ntot, discount, gdelta, PS, D, tp);
        stamp(ts, 5);
    if (!err) {
        int xprev = 0;
        tree_select<NC, true>(smem, d, t, gW, wbase, wsh, PS, cursor, err, Dn, x, xprev, px, nbeyond);
        out_idx = uni(sB[Dn == 0 ? 0 : xprev].w);  // parent->hidden_state_index_x
        out_act = act_of(uni(sB[x].y));            // children_action of the last edge
    }
    }
    stamp(ts, 6);
#if !defined(MZ_SPANS_EPI) && !defined(MZ_SPANS_EXP) && !defined(MZ_SPANS_B2)
    const unsigned long long rm3 = span_mark();
#endif
    if (SEL && l == 0) {
        idx_x[t] = err ? 0 : out_idx;
        idy[t] = t;
        act[t] = err ? 0 : out_act;
    }
    // the leaf's hidden-state row (mcts_sampled.py:130-134): pool[idx_x][t].  Rows up to 16 KiB go
    // through LDS-DMA into the value-entry area (free once wave 1 is done), so nothing waits for
    // them until the copy-out at the very end
    if (lvg && l == 0) *(volatile int *)(xi + 56) = err ? -1 : out_idx + 1;  // (wave 1 gathers)
    bool gath_lds = false;
    char *gdst = nullptr;
    unsigned char *sbig = smem + L::oReg;
    if (SEL && !w1g && !lvg && pool && !err) {
        const char *src = pool + (long long)out_idx * pool_stride + (long long)t * row_bytes;
        gdst = gather_out + (long long)t * row_bytes;
        const bool al = ((row_bytes | pool_stride | (long long)(uintptr_t)pool | (long long)(uintptr_t)gather_out) &
                         15) == 0;
        const long long o = (long long)l * 16;
        if (al && row_bytes <= 16 * 16 * kWave && row_bytes <= 8ll * L::kTreeReg) {
            const long long last = row_bytes - 16;
            for (int k = 0; 1024ll * k < row_bytes; ++k)
                glds16a(src + (o + 1024 * k < last ? o + 1024 * k : last), sbig + 1024 * k);
            gath_lds = true;
        } else if (al) {
            for (long long o2 = o; o2 < row_bytes; o2 += 16 * kWave) *(int4 *)(gdst + o2) = *(const int4 *)(src + o2);
        } else {
            for (long long o2 = (long long)l * 4; o2 < row_bytes; o2 += 4 * kWave)
                *(int *)(gdst + o2) = *(const int *)(src + o2);
        }
    }
#ifdef MZ_SPANS_EPI
    rm1 = span_mark();
#endif
    const bool w1path = SEL && w1g && pool;  // (wave 1 writes the path record and the scored count)
    if (SEL && !err && !w1path) {
        // the path {node, visits at selection} for the next back-propagation (and the scored
        // children), while the row's loads are in flight
        wait_lds();
        int2 *gp = d.path() + (size_t)t * PS;
        int nsc = 0;
        for (int i0 = 0; i0 <= Dn; i0 += kWave) {
            const int i = i0 + l;
            if (i <= Dn) {
                const int xi_ = (i < kWave) ? px : sPath[i].x;
                if constexpr (kTreeLevels<NC>) {
                    gp[i] = (i < kWave) ? make_int2(xi_, pvv) : sPath[i];
                } else {
                    const int vis = sA[xi_].x + (sFl[xi_] ? 1 : 0);
                    gp[i] = make_int2(xi_, vis);
                    const int nci = nc_of(sB[xi_].y);
                    if (i < Dn && !(i == 0 && vis <= nci)) nsc += nci;  // scored levels
                }
            }
        }
        if constexpr (!kTreeLevels<NC>) nscored = wave_sum(nsc);
    }
    stamp(ts, 7);
#ifdef MZ_SPANS_EPI
    rm2 = span_mark();
#endif
    if (SEL && !kTreeLevels<NC> && !err) {  // (wave 2 writes the rest of the header)
        if (l == 0) d.hdr()[t].tame = h.tame;
        const int o0 = cursor - wbase + wsh;  // (wave 2's fetch past the window, counted here)
        if (!(o0 >= wsh && o0 + kNxt <= kRngWin)) nxbeyond = 1;
    } else {  // the header: scalars from lane 0, the next expansion's engine words from lanes 0..kNxt-1
        const int cur = err ? h.cursor : cursor;
        const int o0 = cur - wbase + wsh;
        TreeHdr *hp = d.hdr() + t;
        if (uni((int)(o0 >= wsh && o0 + kNxt <= kRngWin))) {
            if (l < kNxt) hp->nxt[l] = sRng[o0 + l];
        } else {  // beyond the window (rare): through LDS-DMA (no compiler wait on the row's loads)
            nxbeyond = 1;
            unsigned *scr = (unsigned *)(smem + L::oIx);
            const int w = cur + l < gW ? cur + l : gW - 1;
            glds4a(d.R() + (size_t)t * gW + w, scr);
            wait_vm();
            if (l < kNxt) hp->nxt[l] = (cur + l < gW) ? scr[l] : 0u;
        }
        if (l == 0) {
            hp->cursor = cur;
            hp->tot = err ? h.tot : ntot;
            hp->D = (err || !SEL) ? h.D : Dn;
            hp->err = err;
            hp->mm_min = mmn;
            hp->mm_max = mmx;
            hp->mm_cnt = mm_cnt;
            hp->tame = h.tame;
            hp->leaf = (err || !SEL) ? h.leaf : x;
        }
    }
    if constexpr (!SEL) {
        // the fused readback (mz_expand_backup_readback, include/mzdriver.h): the search's outputs
        // from the state after barrier (2) -- the staged records (sA, sB), the path nodes' new value
        // and reward (sAz; flagged in sFl, one more visit), the leaf's new structure record (sB) --
        // and the root children's probabilities from HBM (written at prepare)
        // (a tree that failed writes an empty readback, as k_chain3)
        const RbDesc *rbd = (const RbDesc *)(const void *)gather_out;
        if (rbd) {
            auto upd = [&](int n) {
                int4 a = sA[n];
                const int fl = sFl[n];
                if (fl) {
                    const float2 az = sAz[kTreeAzLevel<NC> ? fl - 1 : n];
                    a = make_int4(a.x + 1, a.y, f2i(az.x), f2i(az.y));
                }
                return a;
            };
            const int4 rbn = err ? make_int4(0, 0, 0, 0) : uni4(sB[0]);
            const int nc = nc_of(rbn.y), fc = rbn.x;
            int4 ca = make_int4(0, 0, 0, 0), cb = ca;
            float4 cd = make_float4(0.f, 0.f, 0.f, 0.f);
            if (l < nc) {
                ca = upd(fc + l);
                cb = sB[fc + l];
                cd = d.D()[nb + fc + l];
            }
            readback_emit(rbd->o, rbd->disc, rbd->Wd, t, A, 1, nc, err ? make_int4(0, 0, 0, 0) : upd(0), ca, cb, cd,
                          nullptr);
        }
    }
    if (gath_lds) {
        wait_vm();
#ifdef MZ_SPANS_EPI
        rm3 = span_mark();
#endif
        // written through (st_wt16; same-box A/B: 3s5z K = 5 env step 8.50 -> 8.42 ms, 27m K = 5
        // 66.65 -> 66.34)
        for (long long o = (long long)l * 16; o < row_bytes; o += 16 * kWave) st_wt16(gdst + o, *(const int4 *)(sbig + o));
    }
    stamp(ts, 8);
    if (l < kStatN) {
        // lane l's counter: the uniform values placed by SALU-built lane masks (a switch on the lane
        // index compiles to a chain of exec-masked branches on this wave's critical path)
        long long add = 0;
        add = sel_lane(add, (long long)((err || !SEL) ? 0 : 1), 1ull << MZ_S_SELECTS);
        add = sel_lane(add, (long long)Dn, 1ull << MZ_S_PATH_EDGES);
        add = sel_lane(add, nscored, 1ull << MZ_S_SCORED);
        add = sel_lane(add, 1ll, 1ull << MZ_S_EXPANDS);
        add = sel_lane(add, (long long)ncl, 1ull << MZ_S_NEW_CHILDREN);
        add = sel_lane(add, (long long)(D + 1), 1ull << MZ_S_BACKUP_NODES);
        add = sel_lane(add, ent_r, 1ull << MZ_S_ENTRIES_READ);
        add = sel_lane(add, ent_w, 1ull << MZ_S_ENTRIES_WRITTEN);
        add = sel_lane(add, (long long)(tot - 1), 1ull << MZ_S_MINMAX_NODES);
        add = sel_lane(add, (long long)moved, 1ull << MZ_S_MM_MOVED);
        add = sel_lane(add, (long long)nbeyond, 1ull << MZ_S_RNG_TIE_BEYOND);
        add = sel_lane(add, (long long)nxbeyond, 1ull << MZ_S_RNG_NXT_BEYOND);
#ifdef MZ_STAMPS_W0
        // (diagnostic builds with -DMZ_STAMPS_W0: wave 0's eight phases in slots CYC_HEADER + k = ts[k+1]
        // - ts[k]: round 1, barrier (1), expansion, barrier (2), scores + tie lists (precomputed
        // classes; 0 in the level walk), chase / walk, path record, epilogue)
        if (MZ_STAMPS && l >= MZ_S_CYC_HEADER && l < MZ_S_CYC_HEADER + 8) {
            const int k = l - MZ_S_CYC_HEADER;
            unsigned long long d0 = 0, d1 = 0;
#pragma unroll
            for (int q = 0; q < 8; ++q)
                if (q == k) {
#ifdef MZ_STAMPS_WALK
                    d0 = tw[q];
                    d1 = tw[q + 1];
#else
                    d0 = ts[q];
                    d1 = ts[q + 1];
#endif
                }
            add = (long long)(d1 - d0);
        } else if (MZ_STAMPS && l == MZ_S_STAMPED) {
            add = 1;
        }
        if (false)
#endif
        if (MZ_STAMPS) switch (l) {
            case MZ_S_CYC_HEADER: add = (long long)(ts[1] - ts[0]); break;    // round 1
            case MZ_S_CYC_STAGE2: add = (long long)(ts[2] - ts[1]); break;    // barrier (1) wait
            case MZ_S_CYC_EXPAND: add = (long long)(ts[3] - ts[2]); break;    // draws + children
            case MZ_S_CYC_BACKUP: add = (long long)(ts[4] - ts[3]); break;    // barrier (2) wait
            case MZ_S_CYC_MINMAX: add = (long long)(ts[5] - ts[4]); break;    // scores + tie lists (4 waves)
            case MZ_S_CYC_STAGE1: add = MZ_STAMPS ? xl[15] : 0; break;       // wave 1: bootstrap
            case MZ_S_CYC_GATHER: add = (long long)(ts[7] - ts[6]); break;
            case MZ_S_CYC_EPILOGUE: add = MZ_STAMPS ? xl[18] : 0; break;     // wave 1: pre-stage + path wait
            case MZ_S_STAMPED: add = 1; break;
            case MZ_S_CYC_W1_BACKUP: add = MZ_STAMPS ? xl[2] : 0; break;      // wave 1: its path levels
            case MZ_S_CYC_EXP_CDF: add = MZ_STAMPS ? xl[16] : 0; break;      // wave 1: header landed
            case MZ_S_CYC_EXP_DRAW: add = (long long)(tq[1] - tq[0]); break;  // barrier (1) + distribution
            case MZ_S_CYC_EXP_NODES: add = MZ_STAMPS ? xl[17] : 0; break;    // wave 1: level 0
            case MZ_S_CYC_BAK_BOOT: add = MZ_STAMPS ? xl[3] : 0; break;       // wave 1: arrival at (1)
            case MZ_S_CYC_W1_STAGE2: add = MZ_STAMPS ? xl[4] : 0; break;      // wave 2: arrival at (1)
            case MZ_S_CYC_BAK_NODES: add = MZ_STAMPS ? xl[5] : 0; break;      // wave 3: arrival at (1)
            case MZ_S_CYC_W1_ROUND1: add = MZ_STAMPS ? xl[6] : 0; break;      // wave 2: its path levels
            case MZ_S_CYC_W1_SYNC: add = MZ_STAMPS ? xl[7] : 0; break;        // wave 3: its path levels
            case MZ_S_CYC_SELECT: add = MZ_STAMPS ? xl[8] : 0; break;         // wave 2: all after (1)
            case MZ_S_CYC_BAK_WAIT: add = MZ_STAMPS ? xl[9] : 0; break;       // wave 3: all after (1)
            default: break;
        }
        if (!(w1path && l == MZ_S_SCORED)) st[l] = st_old + add;
    }
    if (l == 0 && err) atomicOr(d.err(), err);
    span_close(hsx, rt0);
    span_info(hsx, (unsigned long long)(D & 0xffff) | ((unsigned long long)(ntot & 0xffff) << 16) |
                       ((unsigned long long)(Dn & 0xffff) << 32) | ((unsigned long long)moved << 48), rt0, rm1, rm2, rm3);
}

// mz_create's device initialisation in one launch (instead of three copies and three memsets,
// each a synchronous runtime call): the Params block, the seed word, the lambda powers (the float
// chain lp[k] = lp[k - 1] * lam of utils.cpp:25-27, on one thread, in the order the host ran it),
// zeroed tree headers, statistics and error word
__global__ __launch_bounds__(256) void k_init(Params p, unsigned seed, float lam, int nlp, int hdr_words,
                                              int stat_words) {
    const Dev &d = p.d;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i == 0) {
        *(Params *)(void *)d.base = p;
        *d.seed() = seed;
        *d.err() = 0;
        float *lp = d.lp();
        float v = 1.0f;
        lp[0] = v;
        for (int k = 1; k < p.g.PS + 1; ++k) {
            v = v * lam;
            lp[k] = v;
        }
        for (int k = p.g.PS + 1; k < nlp; ++k) lp[k] = 0.f;
    }
    for (int w = i; w < hdr_words; w += gridDim.x * 256) ((int *)d.hdr())[w] = 0;
    for (int w = i; w < stat_words; w += gridDim.x * 256) ((int *)d.stats())[w] = 0;
}

// Standalone hidden-state gather: out[i] = pool[idx_x[i]][i]   (mcts_sampled.py:130-134)
// One device word, set by a kernel.  Captured search graphs never hold a runtime memset node: under
// the HIP runtime's graph packet capture, a replayed hipMemsetAsync node can write a stale fill
// pattern once enough ordinary launches have run (scripts/memset_graph_repro.py).
__global__ void k_set_word(unsigned *w, unsigned v) { *w = v; }

// Small device-to-device copies of readback fields: one launch of this kernel is cheaper inside
// a graph than the runtime's blit kernel for a memcpy node (~4 us each in rocprof).
__global__ __launch_bounds__(256) void k_copy_words(int *__restrict__ dst, const int *__restrict__ src, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) dst[i] = src[i];
}

__global__ __launch_bounds__(64) void k_gather(const char *pool, long long stride, long long rb, const int *idx,
                                              char *out) {
    const int t = blockIdx.x;
    const int l = threadIdx.x;
    const char *src = pool + (long long)idx[t] * stride + (long long)t * rb;
    char *dst = out + (long long)t * rb;
    if (((rb | (long long)(uintptr_t)src | (long long)(uintptr_t)dst) & 15) == 0) {
        for (long long o = (long long)l * 16; o < rb; o += 16 * kWave) *(int4 *)(dst + o) = *(const int4 *)(src + o);
    } else {
        for (long long o = (long long)l * 4; o < rb; o += 4 * kWave) *(int *)(dst + o) = *(const int *)(src + o);
    }
}

// The readback of a tree whose root may have more than 64 children or whose action space is
// wider than a wave (64 < A <= kWideActions, agent_num = 1): the per-child fields 64 at a time, the
// marginals through an action -> child map in LDS (with one agent a cell collects at most one child:
// its visits, and 0 + its prior, as readback_emit's sums in child order give).
__device__ void readback_wide(const RbPtrs &o, const Dev &d, size_t nb, float disc, int Wd, int t, int A, int nc,
                              int fc, int4 ra, int *inv) {
    const int l = lane_id();
    if (l == 0) {
        if (o.values) o.values[t] = (nc > 0) ? i2f(ra.z) : 0.f;
        if (o.deg) o.deg[t] = nc;
    }
    for (int a = l; a < A; a += kWave) inv[a] = -1;
    wait_lds();
    for (int i = l; i < nc; i += kWave) inv[act_of(d.Bn()[nb + fc + i].y)] = i;
    wait_lds();
    if (o.mv || o.mp)
        for (int a = l; a < A; a += kWave) {
            const int i = inv[a];
            int mv = 0;
            float mp = 0.f;
            if (i >= 0) {
                const int4 ca = d.A()[nb + fc + i];
                mv += ca.x;
                mp += i2f(ca.y);
            }
            if (o.mv) o.mv[(size_t)t * A + a] = mv;
            if (o.mp) o.mp[(size_t)t * A + a] = mp;
        }
    for (int i = l; i < Wd; i += kWave) {
        const bool has = i < nc;
        int4 ca = make_int4(0, 0, 0, 0), cb = ca;
        float4 cd = make_float4(0.f, 0.f, 0.f, 0.f);
        if (has) {
            ca = d.A()[nb + fc + i];
            cb = d.Bn()[nb + fc + i];
            cd = d.D()[nb + fc + i];
        }
        const size_t r = (size_t)t * Wd + i;
        const float val = i2f(ca.z), rew = i2f(ca.w);
        if (int *fa = o.f[MZ_F_ACTIONS]) fa[r] = has ? act_of(cb.y) : 0;
        if (o.f[MZ_F_VISIT_COUNT]) o.f[MZ_F_VISIT_COUNT][r] = has ? ca.x : 0;
        const float fv[MZ_F_COUNT] = {0.f, 0.f, cd.x, cd.y, cd.z, i2f(ca.y), cd.z / cd.y * cd.x, i2f(cb.z), val, rew,
                                      rew + disc * val};
#pragma unroll
        for (int f = MZ_F_PRED_PROBS; f < MZ_F_COUNT; ++f)
            if (o.f[f]) ((float *)o.f[f])[r] = has ? fv[f] : 0.f;
    }
}

// Readbacks (cnode.cpp:672-781 over CNode getters 69-171), all fields in one pass (readback_emit)
__global__ __launch_bounds__(64) void k_readback(const Params *__restrict__ prm, float disc, int Wd, RbPtrs o) {
    const Geo g = prm->g;
    const Dev d = prm->d;
    const int t = blockIdx.x;
    const int l = threadIdx.x;
    const size_t nb = (size_t)t * g.P;
    const int4 ra = d.A()[nb];
    const int4 rbn = d.Bn()[nb];
    const int nc = nc_of(uni(rbn.y));
    const int fc = uni(rbn.x);
    {
        const int herr = d.hdr()[t].err;  // dead trees re-report their error (see k_prepare)
        if (l == 0 && herr) atomicOr(d.err(), herr);
    }
    if (g.N == 1 && (g.A > kMaxActions || Wd > kWave)) {
        __shared__ int inv[kWideActions + 1];
        readback_wide(o, d, nb, disc, Wd, t, g.A, nc, fc, ra, inv);
        return;
    }
    int4 ca = make_int4(0, 0, 0, 0), cb = make_int4(0, 0, 0, 0);
    float4 cd = make_float4(0.f, 0.f, 0.f, 0.f);
    if (l < nc) {
        ca = d.A()[nb + fc + l];
        cb = d.Bn()[nb + fc + l];
        cd = d.D()[nb + fc + l];
    }
    const unsigned char *jt = d.J() + (size_t)t * g.JP + (size_t)fc * g.N;  // joint actions (N > 1)
    readback_emit(o, disc, Wd, t, g.A, g.N, nc, ra, ca, cb, cd, jt);
}

// pools past the per-CU LDS image: k_hbm
#include "mzhbm.inc"

}  // namespace

// ================================================================================================
// Host side
// ================================================================================================
struct mz_batch {
    int B, N, A, K, S, P, E, W, PS, Wd;
    int NA;  // N * A: per-root policy / marginal entries
    int device;
    Geo geo;
    Dev dev;
    hipStream_t stream = nullptr;
    hipEvent_t order_ev = nullptr;  // recorded after the last eager work the handle enqueued (mz_set_stream)
    bool order_live = false;        // order_ev marks work that may still be running
    bool dirty = false;             // work enqueued by the current call (OrderMark records order_ev)
    std::vector<void *> allocs;
    size_t arena_bytes = 0;
    float *in_dev = nullptr;  // host-input staging [B*(2+3A)]
    int *sel_dev = nullptr;   // select output staging [3B]
    int *rb_dev = nullptr;    // packed readback
    // fused readbacks (mz_expand_backup_readback): descriptor slots in device memory and their host
    // copies (a slot is uploaded once and never rewritten, so a recorded launch may keep reading it)
    RbDesc *rb_desc_dev = nullptr;
    RbDesc rb_desc_host[8];
    int rb_desc_n = 0;
    bool fused_rb = true;
    size_t rb_words = 0;
    int *rb_host = nullptr;     // packed readback, host mirror (in the pinned stage)
    bool rb_valid = false;      // rb_host mirrors the current tree state
    bool rb_dev_valid = false;  // rb_dev mirrors the current tree state
    float rb_disc = 0.f;
    float tbl_c2 = NAN, tbl_c1 = NAN;
    int consts_ok = 0;  // delta_lb > 0 and 0 <= lambda <= 1 (mz_create)
    int fast_ok = 0;    // consts_ok and every pUCT coefficient finite and >= 0 (ensure_tables)
    bool prepared = false;
    long long expansions = 0;  // expansions since prepare (incl. the root's): bounds tot and depth
    int nc = 0;                // k_step layout class (0 = layout from Geo)
    int chain_nc = -1;         // k_chain node class for K = 1 trees (-1: k_step for every launch)
    int chain3_nc = 0;         // k_chain3 node class (64 .. 1024) for K = 1 trees, 0: k_chain / k_step
    int tree_nc = -1;          // k_tree node class for 2 <= K <= 64 trees (-1: k_step)
    bool hbm = false;          // the pool's LDS image exceeds a CU's LDS: every step launch is k_hbm
    bool seed_ref = false;     // holds a reference on its device's seeding table (seed_table)
    // device bytes by kind (mz_arena_info): pUCT tables, value entries, engine streams, node records
    size_t mem_tables = 0, mem_values = 0, mem_stream = 0, mem_nodes = 0;
    Params *prm = nullptr;     // device copy of {geo, dev} (in the arena)
    // Host-memory path (the cytree numpy surface): one pinned stage per handle, laid out
    // [inputs B*(2+3NA) | selection B*(2+N) | error word | packed readback rb_words] (4-byte words).
    // Inputs are packed into it on the host and go to the device in one copy; a host-memory
    // expansion is only staged (`pend`) and launched with the next call -- fused with the selection
    // when that call is batch_selection, as the reference driver's loop always does.
    char *stage = nullptr;
    size_t stage_bytes = 0;
    float *st_in = nullptr;
    int32_t *st_sel = nullptr;
    int32_t *st_err = nullptr;
    // zero-copy (default; MZ_HOST_COPY=1 at mz_create: DMA copies instead): the kernels read the
    // staged inputs and write the selection straight through the stage's device mapping
    bool zc = true;
    const float *st_in_d = nullptr;
    int32_t *st_sel_d = nullptr, *st_err_d = nullptr;
    hipEvent_t st_ev = nullptr;  // the last copy out of st_in has been read when this fires
    bool st_busy = false;
    bool pend = false;           // a staged host-memory expansion not launched yet
    int pend_hsx = 0, pend_K = 0;
    float pend_disc = 0.f;
};

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &m) {
    g_err = m;
    return code;
}

#define HIP_TRY(expr)                                                                                  \
    do {                                                                                               \
        hipError_t _e = (expr);                                                                        \
        if (_e != hipSuccess) return fail(MZ_ERR_DEVICE, std::string(#expr " failed: ") + hipGetErrorString(_e)); \
    } while (0)

int round16(int x) { return (x + 15) & ~15; }

// The per-device table of std::mt19937 seeding checkpoints (k_seed_table), shared by every handle
// of the device: rows for every seed value v = random_seed * 2333 + root index (cnode.cpp:574) below
// its size, sized for random_seed < 256 (np_random.choice(256), mcts_sampled.py:89) and at least
// 4096 roots (~97 MB).  Built once (a few ms), grown when a handle's roots need more; an outgrown
// table stays allocated while handles made before it (and graphs they recorded) may read it.  Every
// live handle holding a table counts in `live`; mz_trim_caches frees a device's tables when none
// does.  Seeds outside the table take the sequential chain.
struct SeedTable {
    unsigned *p = nullptr;
    unsigned n = 0;
    int live = 0;                // live handles that read this device's tables
    std::vector<void *> old;     // outgrown tables
    size_t bytes = 0;            // of p and old together
};
constexpr int kSeedTabDevices = 64;
std::mutex g_seed_mu;
SeedTable g_seed_tab[kSeedTabDevices];

void seed_table(int dev, unsigned long long need, const unsigned **cp, unsigned *cp_n) {
    *cp = nullptr;
    *cp_n = 0;
    if (dev < 0 || dev >= kSeedTabDevices) return;
    std::lock_guard<std::mutex> lk(g_seed_mu);
    SeedTable &st = g_seed_tab[dev];
    if (st.n < need) {
        unsigned long long n = 256ull * 2333ull + 4096ull;
        if (n < need) n = need;
        if (n > 0xffffffffull) n = 0xffffffffull;
        void *p = nullptr;
        hipStream_t s = nullptr;
        bool ok = hipMalloc(&p, (size_t)n * kSeedRow * sizeof(unsigned)) == hipSuccess;
        ok = ok && hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess;
        if (ok) {
            hipLaunchKernelGGL(k_seed_table, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (unsigned *)p,
                               (unsigned)n);
            ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(s) == hipSuccess;
        }
        if (s) (void)hipStreamDestroy(s);
        if (!ok) {  // (no table: k_prepare runs the chain)
            if (p) (void)hipFree(p);
            (void)hipGetLastError();
            return;
        }
        if (st.p) st.old.push_back(st.p);
        st.p = (unsigned *)p;
        st.n = (unsigned)n;
        st.bytes += (size_t)n * kSeedRow * sizeof(unsigned);
    }
    *cp = st.p;
    *cp_n = st.n;
    ++st.live;
}

void seed_table_release(int dev) {
    if (dev < 0 || dev >= kSeedTabDevices) return;
    std::lock_guard<std::mutex> lk(g_seed_mu);
    if (g_seed_tab[dev].live > 0) --g_seed_tab[dev].live;
}

// the tables of every device no live handle reads; returns the bytes freed
size_t seed_table_trim() {
    std::lock_guard<std::mutex> lk(g_seed_mu);
    size_t freed = 0;
    for (SeedTable &st : g_seed_tab) {
        if (st.live > 0 || !st.p) continue;
        (void)hipFree(st.p);
        for (void *q : st.old) (void)hipFree(q);
        freed += st.bytes;
        st = SeedTable{};
    }
    return freed;
}

// A non-blocking stream per device for mz_create's initialisation launch (never captured, so a
// capture running on another stream is not disturbed)
hipStream_t init_stream(int dev) {
    static hipStream_t st[kSeedTabDevices];
    if (dev < 0 || dev >= kSeedTabDevices) return nullptr;
    std::lock_guard<std::mutex> lk(g_seed_mu);
    if (!st[dev] && hipStreamCreateWithFlags(&st[dev], hipStreamNonBlocking) != hipSuccess) {
        (void)hipGetLastError();
        st[dev] = nullptr;
    }
    return st[dev];
}

bool getenv_flag(const char *name) {
    const char *v = std::getenv(name);
    return v && v[0] == '1';
}

const char *err_message(int bits) {
    if (bits & kErrValueSet) return "SubTreeValueSet::update: cur_size+1!=size_lim.";
    if (bits & kErrPool) return "node pool exhausted: more expansions than simulation_num allows";
    if (bits & kErrRng) return "random stream exhausted: more simulations than simulation_num allows";
    if (bits & kErrPath) return "search path or value-set capacity exceeded";
    if (bits & kErrRoot) return "selection on an unexpanded root";
    if (bits & kErrTable) return "visit count beyond the pUCT table (more simulations than simulation_num)";
    return "device-side search error";
}

// Process-wide caches of released device arenas and pinned stages, reused by size: the
// reference builds a new Tree_batch per search (mcts_sampled.py:89), and hipFree synchronises the
// whole device while hipHostMalloc costs tens of microseconds.  Bounded; the rest is freed.
struct BlockCache {
    struct Blk {
        int device;
        size_t bytes;
        void *p;
    };
    std::mutex mu;
    std::vector<Blk> free;
    size_t held = 0;
    // free every cached block of `device` (-1: all); returns the bytes released
    size_t drain(int device, bool host) {
        std::vector<Blk> out;
        {
            std::lock_guard<std::mutex> g(mu);
            for (size_t i = 0; i < free.size();)
                if (device < 0 || free[i].device == device) {
                    out.push_back(free[i]);
                    held -= free[i].bytes;
                    free.erase(free.begin() + (long)i);
                } else {
                    ++i;
                }
        }
        size_t n = 0;
        for (auto &b : out) {
            if (host) (void)hipHostFree(b.p);
            else (void)hipFree(b.p);
            n += b.bytes;
        }
        return n;
    }
    void *take(int device, size_t bytes) {
        std::lock_guard<std::mutex> g(mu);
        for (size_t i = 0; i < free.size(); ++i)
            if (free[i].device == device && free[i].bytes == bytes) {
                void *p = free[i].p;
                held -= bytes;
                free.erase(free.begin() + (long)i);
                return p;
            }
        return nullptr;
    }
    // true: kept (the caller must not free it)
    bool give(int device, size_t bytes, void *p, size_t cap_bytes, size_t cap_blocks) {
        std::lock_guard<std::mutex> g(mu);
        if (held + bytes > cap_bytes || free.size() >= cap_blocks) return false;
        free.push_back({device, bytes, p});
        held += bytes;
        return true;
    }
};
BlockCache &arena_cache() {
    static BlockCache *c = new BlockCache;  // never destroyed: handles may outlive static teardown
    return *c;
}
BlockCache &stage_cache() {
    static BlockCache *c = new BlockCache;
    return *c;
}
// (what stays resident: at most kArenaCacheBytes of released arenas and kStageCacheBytes of pinned
// stages per process, plus the per-device seeding table of ~97 MB; mz_trim_caches releases the
// first two, and an arena allocation that fails releases them and tries once more)
constexpr size_t kArenaCacheBytes = (size_t)2 << 30, kArenaCacheBlocks = 16;
constexpr size_t kStageCacheBytes = (size_t)256 << 20, kStageCacheBlocks = 32;

int ensure_device(mz_batch *b) {
    int cur = -1;
    HIP_TRY(hipGetDevice(&cur));
    if (cur != b->device) HIP_TRY(hipSetDevice(b->device));
    return MZ_OK;
}

// Poll the handle's error word (synchronises the stream).
int ensure_stage(mz_batch *b);
int copy_words(mz_batch *b, void *dst, const int *src, size_t n);
int check_device_errors(mz_batch *b) {
    int rc = ensure_stage(b);
    if (rc) return rc;
    if (b->zc) {  // (a one-word kernel store into the stage's device mapping: no DMA round trip)
        rc = copy_words(b, b->st_err_d, b->dev.err(), 1);
        if (rc) return rc;
    } else {
        HIP_TRY(hipMemcpyAsync(b->st_err, b->dev.err(), sizeof(int), hipMemcpyDeviceToHost, b->stream));
    }
    HIP_TRY(hipStreamSynchronize(b->stream));
    b->st_busy = false;  // (every copy out of the stage has completed)
    b->dirty = b->order_live = false;  // nothing of this handle is in flight
    const int e = *b->st_err;
    if (e) {
        char bits[32];
        std::snprintf(bits, sizeof bits, " (device error word 0x%x)", (unsigned)e);
        return fail(MZ_ERR_RUNTIME, std::string(err_message(e)) + bits);
    }
    return MZ_OK;
}

// pUCT tables for (c2, c1): pb[n] = logf(((float)n + c2 + 1) / c2) + c1 with glibc logf, exactly as
// ucb_score evaluates it (cnode.cpp:313), and sq[n] = sqrt((double)n) (cnode.cpp:314).
int ensure_tables(mz_batch *b, float c2, float c1) {
    if (b->tbl_c2 == c2 && b->tbl_c1 == c1) return MZ_OK;
    std::vector<float> pb(b->PS);
    std::vector<double> sq(b->PS);
    for (int n = 0; n < b->PS; ++n) {
        float x = (float)n + c2;
        x = x + 1.0f;
        x = x / c2;
        pb[n] = ::logf(x) + c1;
        sq[n] = ::sqrt((double)n);
    }
    // pb_c(n, v) for every parent total n and child visits v <= n, with ucb_score's operations:
    // pb_c = pb[n]; pb_c *= (sqrt(n) / (v + 1))   (float *= double); past kTableFullPS only T[0]
    // (table_entries)
    std::vector<float> T(b->geo.TT, 0.f);
    const int tn = b->PS <= (int)kTableFullPS ? b->PS : 1;
    for (int n = 0; n < tn; ++n)
        for (int v = 0; v <= n; ++v) {
            float pbc = pb[n];
            pbc = (float)((double)pbc * (sq[n] / (double)(v + 1)));
            T[(size_t)n * (n + 1) / 2 + v] = pbc;
        }
    HIP_TRY(hipMemcpyAsync(b->dev.T(), T.data(), sizeof(float) * T.size(), hipMemcpyHostToDevice, b->stream));
    HIP_TRY(hipMemcpyAsync(b->dev.pb(), pb.data(), sizeof(float) * b->PS, hipMemcpyHostToDevice, b->stream));
    HIP_TRY(hipMemcpyAsync(b->dev.sq(), sq.data(), sizeof(double) * b->PS, hipMemcpyHostToDevice, b->stream));
    HIP_TRY(hipStreamSynchronize(b->stream));
    b->tbl_c2 = c2;
    b->tbl_c1 = c1;
    bool pb_ok = true;
    for (int n = 0; n < b->PS; ++n) pb_ok = pb_ok && std::isfinite(pb[n]) && pb[n] >= 0.f;
    b->fast_ok = (b->consts_ok && pb_ok) ? 1 : 0;
    return MZ_OK;
}

// Sub-allocation of one device buffer (256-byte aligned arrays, in request order): Dev arrays get
// offsets from Dev::base, host-side staging buffers get plain pointers.
struct ArenaPlan {
    struct Req {
        unsigned *off;
        void **ptr;
        size_t at;
    };
    std::vector<Req> req;
    size_t total = 0;
    static size_t span(size_t bytes) { return (bytes + 64 + 255) & ~(size_t)255; }
    template <typename T>
    void dev(unsigned &off, size_t count) {
        req.push_back({&off, nullptr, total});
        total += span(count * sizeof(T));
    }
    template <typename T>
    void ptr(T **p, size_t count) {
        req.push_back({nullptr, (void **)p, total});
        total += span(count * sizeof(T));
    }
    int allocate(mz_batch *b, Dev &d) {
        if (total / 256 > 0xffffffffull) return fail(MZ_ERR_UNSUPPORTED, "device arena larger than 1 TiB");
        void *q = arena_cache().take(b->device, total);
        if (!q && hipMalloc(&q, total) != hipSuccess) {
            // cached arenas of other sizes may be what is missing: release them, try once more
            (void)hipGetLastError();
            q = nullptr;
            (void)arena_cache().drain(b->device, false);
            HIP_TRY(hipMalloc(&q, total));
        }
        b->allocs.push_back(q);
        b->arena_bytes = total;
        d.base = (gchar *)q;
        for (auto &r : req) {
            if (r.off) *r.off = (unsigned)(r.at / 256);
            else *r.ptr = (char *)q + r.at;
        }
        return MZ_OK;
    }
};

template <int NC, bool JOINT = false>
void launch_nc(mz_batch *b, bool eb, bool sel, const StepArgs &a) {
    const Geo &g = b->geo;
#define MZ_STEP_ARGS                                                                                       \
    (char *)b->dev.base, g.P, g.PS, g.B | (g.A << 24), a.pe | (g.K << 17), a.reward, a.value, a.policy, a.beta,  \
        a.K, a.hsx, a.discount, b->fast_ok, a.pool, a.pool_stride, a.row_bytes, a.gather_out, a.idx_x, a.idy,      \
        a.act
    if (eb && sel)
        hipLaunchKernelGGL((k_step<true, true, NC, JOINT>), dim3(g.B), dim3(2 * kWave), g.lds, b->stream, MZ_STEP_ARGS);
    else if (eb)
        hipLaunchKernelGGL((k_step<true, false, NC, JOINT>), dim3(g.B), dim3(2 * kWave), g.lds, b->stream,
                           MZ_STEP_ARGS);
    else
        hipLaunchKernelGGL((k_step<false, true, NC, JOINT>), dim3(g.B), dim3(2 * kWave), g.lds, b->stream,
                           MZ_STEP_ARGS);
#undef MZ_STEP_ARGS
}

template <int NC, bool JOINT = false>
void set_lds_limit(int lds) {
    const auto attr = hipFuncAttributeMaxDynamicSharedMemorySize;
    (void)hipFuncSetAttribute((const void *)k_step<true, true, NC, JOINT>, attr, lds);
    (void)hipFuncSetAttribute((const void *)k_step<true, false, NC, JOINT>, attr, lds);
    (void)hipFuncSetAttribute((const void *)k_step<false, true, NC, JOINT>, attr, lds);
}

template <int NC, bool SEL = true>
void launch_chain(mz_batch *b, const StepArgs &a, int lds) {
    const Geo &g = b->geo;
    // (the first 14 argument dwords, through the discount, arrive preloaded in SGPRs: round 1 needs no
    // kernel-argument load)
    hipLaunchKernelGGL((k_chain<NC, SEL>), dim3(g.B), dim3(2 * kWave), lds, b->stream, (char *)b->dev.base, a.policy,
                       a.beta, g.P, g.PS, g.B | (g.A << 24), a.pe | (g.K << 17), a.hsx, a.K, a.discount, b->fast_ok,
                       a.reward, a.value, a.pool, a.pool_stride, a.row_bytes, a.gather_out, a.idx_x, a.idy, a.act);
}

template <int NC, bool SEL, int ROW>
void launch_chain3_row(mz_batch *b, const StepArgs &a) {
    const Geo &g = b->geo;
    const Dev &dv = b->dev;
    // (the first 14 argument dwords, through the discount, arrive preloaded in SGPRs)
    const ChainIO io{a.pool, a.pool_stride, a.row_bytes, a.gather_out, a.idx_x, a.idy, a.act};
    // ROW 1, 2: the leaf's slot and the row size (16-byte units, <= 1024) ride in preloaded arguments
    const bool pre = ROW == 1 || ROW == 2;
    const char *src_slot = pre ? a.pool + (long long)a.hsx * a.pool_stride : nullptr;
    const int rb16 = pre ? (int)(a.row_bytes / 16) : 0;
    hipLaunchKernelGGL((k_chain3<NC, SEL, ROW>), dim3(g.B), dim3(3 * kWave),
                       chain3_lds_bytes(NC) + (ROW == 2 ? 16 * 16 * kWave : 0), b->stream, (char *)dv.base, a.policy,
                       a.beta, a.reward, a.value, g.P | (g.PS << 10) | (rb16 << 20),
                       (int)((unsigned)g.B | ((unsigned)g.A << 24) | ((unsigned)b->fast_ok << 31)), a.hsx, a.discount,
                       src_slot, io);
}
// the row class of a launch (k_chain3's ROW)
int chain3_row(const StepArgs &a, bool sel) {
    if (!sel || !a.pool) return 3;
    const bool al = ((a.row_bytes | a.pool_stride | (long long)(uintptr_t)a.pool | (long long)(uintptr_t)a.gather_out) &
                     15) == 0;
    if (al && a.row_bytes > 0 && a.row_bytes <= 4 * 16 * kWave) return 1;
    if (al && a.row_bytes > 0 && a.row_bytes <= 16 * 16 * kWave) return 2;
    return 0;
}
template <int NC, bool SEL = true>
void launch_chain3(mz_batch *b, const StepArgs &a) {
    switch (chain3_row(a, SEL)) {
        case 1: launch_chain3_row<NC, SEL, 1>(b, a); break;
        case 2: launch_chain3_row<NC, SEL, 2>(b, a); break;
        case 3: launch_chain3_row<NC, SEL, 3>(b, a); break;
        default: launch_chain3_row<NC, SEL, 0>(b, a); break;
    }
}

static int device_cus() {  // compute units of the current device (one MI355X: 256)
    static int n = 0;
    if (n == 0) {
        int dev = 0, c = 0;
        if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && c > 0) n = c;
        else n = 1;
    }
    return n;
}

template <int NC, bool SEL = true>
void launch_tree(mz_batch *b, const StepArgs &a) {
    const Geo &g = b->geo;
    const int flags = (b->fast_ok ? 1 : 0) | (g.B <= device_cus() ? 2 : 0);
    hipLaunchKernelGGL((k_tree<NC, SEL>), dim3(g.B), dim3(kTreeWavesN<NC> * kWave), TreeLayout<NC>::total, b->stream,
                       (char *)b->dev.base, a.policy, a.beta, g.P, g.PS, g.B | (g.A << 24), a.pe | (g.K << 17), a.hsx,
                       a.K, a.discount, flags, a.reward, a.value, a.pool, a.pool_stride, a.row_bytes,
                       a.gather_out, a.idx_x, a.idy, a.act);
}

template <bool EB, bool SEL, bool JOINT>
void launch_hbm_t(mz_batch *b, const StepArgs &a) {
    hipLaunchKernelGGL((k_hbm<EB, SEL, JOINT>), dim3(b->B), dim3(kHbmWaves * kWave), hbm_lds_bytes(b->N, b->NA),
                       b->stream, b->prm, a);
}
template <bool JOINT>
void launch_hbm(mz_batch *b, bool eb, bool sel, const StepArgs &a) {
    if (eb && sel) launch_hbm_t<true, true, JOINT>(b, a);
    else if (eb) launch_hbm_t<true, false, JOINT>(b, a);
    else launch_hbm_t<false, true, JOINT>(b, a);
}

int launch_step(mz_batch *b, bool eb, bool sel, StepArgs a) {
    const Geo &g = b->geo;
    b->dirty = true;
    if (b->hbm) {  // pools past the LDS image: every launch of the handle
        if (b->N > 1) launch_hbm<true>(b, eb, sel, a);
        else launch_hbm<false>(b, eb, sel, a);
        HIP_TRY(hipGetLastError());
        if (eb) {
            b->rb_valid = b->rb_dev_valid = false;
            ++b->expansions;
        }
        return MZ_OK;
    }
    if (eb && b->chain3_nc > 0) {  // K = 1 trees: the three-wave chain kernel
        if (sel) {
            switch (b->chain3_nc) {
                case 64: launch_chain3<64>(b, a); break;
                case 128: launch_chain3<128>(b, a); break;
                default: launch_chain3<256>(b, a); break;
            }
        } else {
            switch (b->chain3_nc) {
                case 64: launch_chain3<64, false>(b, a); break;
                case 128: launch_chain3<128, false>(b, a); break;
                default: launch_chain3<256, false>(b, a); break;
            }
        }
        HIP_TRY(hipGetLastError());
        b->rb_valid = b->rb_dev_valid = false;
        ++b->expansions;
        return MZ_OK;
    }
    if (eb && b->chain_nc >= 0) {  // K = 1 trees: the chain kernel
        const bool big = sel && a.pool && a.row_bytes > 4 * 16 * kWave && a.row_bytes <= 16 * 16 * kWave;
        const int lds = chain_lds_bytes(g.P, b->chain_nc) + (big ? 16 * 16 * kWave : 0);
        if (sel) {
            switch (b->chain_nc) {
                case 64: launch_chain<64>(b, a, lds); break;
                case 128: launch_chain<128>(b, a, lds); break;
                case 256: launch_chain<256>(b, a, lds); break;
                case 512: launch_chain<512>(b, a, lds); break;
                case 1024: launch_chain<1024>(b, a, lds); break;
                default: launch_chain<0>(b, a, lds); break;
            }
        } else {
            switch (b->chain_nc) {
                case 64: launch_chain<64, false>(b, a, lds); break;
                case 128: launch_chain<128, false>(b, a, lds); break;
                case 256: launch_chain<256, false>(b, a, lds); break;
                case 512: launch_chain<512, false>(b, a, lds); break;
                case 1024: launch_chain<1024, false>(b, a, lds); break;
                default: launch_chain<0, false>(b, a, lds); break;
            }
        }
        HIP_TRY(hipGetLastError());
        b->rb_valid = b->rb_dev_valid = false;
        ++b->expansions;
        return MZ_OK;
    }
    // tot <= 1 + K * expansions and depth <= expansions: the kernel stages that much without
    // waiting for the tree header (and falls back to the header's values if they are larger)
    {
        const long long ne = 1 + (long long)g.K * b->expansions;
        a.ne = (int)(ne < g.P ? ne : g.P);
        const long long pe = b->expansions + 1;
        a.pe = (int)(pe < g.PS ? pe : g.PS);
    }
    if (eb && b->tree_nc > 0) {  // 2 <= K <= 64 trees: the four-wave kernel
        if (sel) {
            switch (b->tree_nc) {
                case 64: launch_tree<64>(b, a); break;
                case 128: launch_tree<128>(b, a); break;
                case 256: launch_tree<256>(b, a); break;
                case 384: launch_tree<384>(b, a); break;
                case 512: launch_tree<512>(b, a); break;
                case kTree1024S: launch_tree<kTree1024S>(b, a); break;
                default: launch_tree<1024>(b, a); break;
            }
        } else {
            switch (b->tree_nc) {
                case 64: launch_tree<64, false>(b, a); break;
                case 128: launch_tree<128, false>(b, a); break;
                case 256: launch_tree<256, false>(b, a); break;
                case 384: launch_tree<384, false>(b, a); break;
                case 512: launch_tree<512, false>(b, a); break;
                case kTree1024S: launch_tree<kTree1024S, false>(b, a); break;
                default: launch_tree<1024, false>(b, a); break;
            }
        }
        HIP_TRY(hipGetLastError());
        b->rb_valid = b->rb_dev_valid = false;
        ++b->expansions;
        return MZ_OK;
    }
#ifndef MZ_NO_JOINT
    if (b->N > 1) {
        launch_nc<0, true>(b, eb, sel, a);
    } else
#endif
    switch (b->nc) {
        case 64: launch_nc<64>(b, eb, sel, a); break;
        case 128: launch_nc<128>(b, eb, sel, a); break;
        case 256: launch_nc<256>(b, eb, sel, a); break;
        case 384: launch_nc<384>(b, eb, sel, a); break;
        case 512: launch_nc<512>(b, eb, sel, a); break;
        case 1024: launch_nc<1024>(b, eb, sel, a); break;
        default: launch_nc<0>(b, eb, sel, a); break;
    }
    HIP_TRY(hipGetLastError());
#ifdef MZ_ARGCHECK
    {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        (void)hipStreamIsCapturing(b->stream, &cs);
        if (cs == hipStreamCaptureStatusActive)
            fprintf(stderr, "MZCAPTURE step eb%d sel%d b %p base %p hsx %d pe %d ne %d K %d reward %p pool %p out %p\n",
                    (int)eb, (int)sel, (void *)b, (void *)b->dev.base, a.hsx, a.pe, a.ne, a.K, (const void *)a.reward,
                    (const void *)a.pool, (void *)a.idx_x);
    }
#endif
    if (eb) {
        b->rb_valid = b->rb_dev_valid = false;
        ++b->expansions;
    }
    return MZ_OK;
}

// Packed readback layout (4-byte words): [B] root value | [B*NA] marginal visits | [B*NA] marginal
// priors | [B] degree | MZ_F_COUNT x [B*Wd*N] per-child fields (actions fill [B][Wd][N], the
// others the first B*Wd words).
size_t rb_deg_base(const mz_batch *b) { return (size_t)b->B + 2 * (size_t)b->B * b->NA; }
size_t rb_field_base(const mz_batch *b, int field) {
    return rb_deg_base(b) + (size_t)b->B + (size_t)field * b->B * b->Wd * b->N;
}
size_t rb_field_width(const mz_batch *b, int field) { return (size_t)b->Wd * (field == MZ_F_ACTIONS ? b->N : 1); }


// Every public call that enqueues work on the handle's stream ends by recording order_ev behind it
// (OrderMark), so that mz_set_stream orders a new stream after that work without ever touching the
// old stream, which the caller may have destroyed since.  Work recorded into a graph capture is
// ordered by the capture (nothing to mark); a synchronisation leaves nothing to order.
void mark_order(mz_batch *b) {
    if (!b->dirty) return;
    b->dirty = false;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(b->stream, &cs) != hipSuccess) {  // (the stream of this very call)
        (void)hipGetLastError();
        return;
    }
    if (cs != hipStreamCaptureStatusNone) return;
    if (!b->order_ev && hipEventCreateWithFlags(&b->order_ev, hipEventDisableTiming) != hipSuccess) return;
    if (hipEventRecord(b->order_ev, b->stream) == hipSuccess) b->order_live = true;
}
struct OrderMark {
    mz_batch *b;
    ~OrderMark() {
        if (b) mark_order(b);
    }
};

// --- the host-memory path's pinned stage ------------------------------------------------------
size_t stage_in_words(const mz_batch *b) { return (size_t)b->B * (2 + 3 * (size_t)b->NA); }
size_t stage_sel_words(const mz_batch *b) { return (size_t)b->B * (2 + (size_t)b->N); }

int ensure_stage(mz_batch *b) {
    if (b->stage) return MZ_OK;
    auto r64 = [](size_t w) { return (w + 15) & ~(size_t)15; };  // 64-byte aligned sections
    const size_t w_in = r64(stage_in_words(b)), w_sel = r64(stage_sel_words(b)), w_err = 16, w_rb = r64(b->rb_words);
    const size_t bytes = 4 * (w_in + w_sel + w_err + w_rb);
    void *p = stage_cache().take(-1, bytes);
    if (!p) HIP_TRY(hipHostMalloc(&p, bytes, hipHostMallocMapped | hipHostMallocPortable));
    b->stage = (char *)p;
    b->stage_bytes = bytes;
    b->st_in = (float *)p;
    b->st_sel = (int32_t *)p + w_in;
    b->st_err = (int32_t *)p + w_in + w_sel;
    b->rb_host = (int *)p + w_in + w_sel + w_err;
    if (!b->st_ev) HIP_TRY(hipEventCreateWithFlags(&b->st_ev, hipEventDisableTiming));
    void *pd = nullptr;
    HIP_TRY(hipHostGetDevicePointer(&pd, p, 0));
    b->st_in_d = (const float *)pd;
    b->st_sel_d = (int32_t *)pd + w_in;
    b->st_err_d = (int32_t *)pd + w_in + w_sel;
    return MZ_OK;
}

// where a launch reads the staged inputs: the stage itself (zero-copy) or in_dev after stage_upload
const float *stage_src(const mz_batch *b) { return b->zc ? b->st_in_d : b->in_dev; }

// a launch reading the stage was enqueued: st_in may be rewritten once it has run
int stage_consumed(mz_batch *b) {
    if (!b->zc) return MZ_OK;
    HIP_TRY(hipEventRecord(b->st_ev, b->stream));
    b->st_busy = true;
    return MZ_OK;
}

// st_in may be rewritten: the previous copy out of it has been read
int stage_wait(mz_batch *b) {
    int rc = ensure_stage(b);
    if (rc) return rc;
    if (b->st_busy) {
        HIP_TRY(hipEventSynchronize(b->st_ev));
        b->st_busy = false;
    }
    return MZ_OK;
}

// the first `words` of st_in -> in_dev, one copy on the handle's stream (none when zero-copy)
int stage_upload(mz_batch *b, size_t words) {
    if (b->zc) return MZ_OK;
    HIP_TRY(hipMemcpyAsync(b->in_dev, b->st_in, 4 * words, hipMemcpyHostToDevice, b->stream));
    HIP_TRY(hipEventRecord(b->st_ev, b->stream));
    b->st_busy = true;
    b->dirty = true;
    return MZ_OK;
}

// host arrays -> st_in in in_dev's layout [rewards B | values B | policy B*NA | beta B*NA (| noises B*NA)]
void stage_pack(mz_batch *b, const float *rewards, const float *values, const float *policy, const float *beta,
                const float *noises) {
    const size_t B = b->B, NA = (size_t)b->NA;
    float *p = b->st_in;
    std::memcpy(p, rewards, 4 * B);
    std::memcpy(p + B, values, 4 * B);
    std::memcpy(p + 2 * B, policy, 4 * B * NA);
    std::memcpy(p + 2 * B + B * NA, beta, 4 * B * NA);
    if (noises) std::memcpy(p + 2 * B + 2 * B * NA, noises, 4 * B * NA);
}

StepArgs staged_expand_args(mz_batch *b) {
    const size_t B = b->B, NA = (size_t)b->NA;
    StepArgs a{};
    const float *src = stage_src(b);
    a.hsx = b->pend_hsx;
    a.discount = b->pend_disc;
    a.K = b->pend_K;
    a.reward = src;
    a.value = src + B;
    a.policy = src + 2 * B;
    a.beta = src + 2 * B + B * NA;
    return a;
}

// Launch a staged host-memory expansion on its own (every call but batch_selection, which fuses it).
int flush_pending(mz_batch *b) {
    if (!b->pend) return MZ_OK;
    b->pend = false;
    int rc = stage_upload(b, 2 * (size_t)b->B * (1 + (size_t)b->NA));
    if (rc) return rc;
    rc = launch_step(b, true, false, staged_expand_args(b));
    if (rc) return rc;
    return stage_consumed(b);
}

// the packed readback buffer's fields
RbPtrs packed_rb(const mz_batch *b) {
    RbPtrs o;
    int *rb = b->rb_dev;
    const size_t n = (size_t)b->B * b->NA;
    o.values = (float *)rb;
    o.mv = rb + b->B;
    o.mp = (float *)(rb + b->B + n);
    o.deg = rb + rb_deg_base(b);
    for (int f = 0; f < MZ_F_COUNT; ++f) o.f[f] = rb + rb_field_base(b, f);
    return o;
}

// The device slot holding a fused readback's descriptor (destinations, discount, width), uploaded
// on first use; null when every slot is taken by other destinations, or when the first use comes
// inside a graph capture (the upload is eager work): the caller then launches k_readback itself.
const RbDesc *rb_desc_slot(mz_batch *b, const RbPtrs &o, float disc) {
    constexpr int kSlots = (int)(sizeof(b->rb_desc_host) / sizeof(RbDesc));
    RbDesc want;
    std::memset(&want, 0, sizeof want);
    want.o = o;
    want.disc = disc;
    want.Wd = b->Wd;
    for (int i = 0; i < b->rb_desc_n; ++i)
        if (!std::memcmp(&b->rb_desc_host[i], &want, sizeof want)) return b->rb_desc_dev + i;
    if (b->rb_desc_n >= kSlots) return nullptr;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(b->stream, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
        (void)hipGetLastError();
        return nullptr;
    }
    const int i = b->rb_desc_n;
    b->rb_desc_host[i] = want;
    if (hipMemcpyAsync(b->rb_desc_dev + i, &b->rb_desc_host[i], sizeof(RbDesc), hipMemcpyHostToDevice, b->stream) !=
        hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    b->rb_desc_n = i + 1;
    return b->rb_desc_dev + i;
}

// Packed readback computed on the device (stream-ordered, no synchronisation).
int readback_dev(mz_batch *b, float disc) {
    int rc = flush_pending(b);
    if (rc) return rc;
    if (b->rb_dev_valid && b->rb_disc == disc) return MZ_OK;
    const RbPtrs o = packed_rb(b);
    b->dirty = true;
    hipLaunchKernelGGL(k_readback, dim3(b->B), dim3(kWave), 0, b->stream, b->prm, disc, b->Wd, o);
    HIP_TRY(hipGetLastError());
    b->rb_dev_valid = true;
    b->rb_valid = false;
    b->rb_disc = disc;
    return MZ_OK;
}

int copy_words(mz_batch *b, void *dst, const int *src, size_t n) {
    if (n == 0) return MZ_OK;
    b->dirty = true;
    hipLaunchKernelGGL(k_copy_words, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, b->stream, (int *)dst, src, (int)n);
    HIP_TRY(hipGetLastError());
    return MZ_OK;
}

// ... and mirrored to the host (synchronises; reports deferred device errors).
int readback(mz_batch *b, float disc) {
    if (b->rb_valid && b->rb_disc == disc) return MZ_OK;
    int rc = readback_dev(b, disc);
    if (rc) return rc;
    rc = ensure_stage(b);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(b->rb_host, b->rb_dev, sizeof(int) * b->rb_words, hipMemcpyDeviceToHost, b->stream));
    rc = check_device_errors(b);
    if (rc) return rc;
    b->rb_valid = true;
    return MZ_OK;
}

}  // namespace

extern "C" {

const char *mz_last_error(void) { return g_err.c_str(); }
int mz_abi_version(void) { return MZ_ABI_VERSION; }
const char *mz_backend(void) { return "hip-gfx950"; }

int mz_create(int B, int N, int A, int K, int S, float delta_lb, uint32_t seed, float rho, float lam, int root_offset,
              mz_batch **out) {
    if (!out) return fail(MZ_ERR_ARG, "null output handle");
    *out = nullptr;
    if (B < 1 || A < 1 || K < 1 || S < 0) return fail(MZ_ERR_ARG, "bad tree-batch dimensions");
    if (B >= (1 << 24)) return fail(MZ_ERR_UNSUPPORTED, "root_num >= 2^24");  // packed with A in k_step's arguments
    if (N < 1) return fail(MZ_ERR_ARG, "agent_num must be >= 1");
    // action spaces past one lane per action (64 < A <= 255) take the wide expansion and k_hbm;
    // Bn.y packs the action and the children count in 8 bits each
    if (A > kWideActions) return fail(MZ_ERR_UNSUPPORTED, "action_space_size > 255");
    if (N > 1 && (K > kWave || N > kWave || A > kMaxActions || (long long)N * A > 4096))
        return fail(MZ_ERR_UNSUPPORTED, "joint-action trees (agent_num > 1) need sampled_times <= 64, "
                                         "agent_num <= 64, action_space_size <= 64 and "
                                         "agent_num * action_space_size <= 4096");
    if (S > 65000) return fail(MZ_ERR_UNSUPPORTED, "simulation_num > 65000");
    if (K > (1 << 20)) return fail(MZ_ERR_UNSUPPORTED, "sampled_times > 2^20");
    // max degree of any node: min(K, A^N) (children are the distinct sampled joint actions,
    // cnode.cpp:242-294)
    int Wd = 1;
    {
        long long an = 1;
        for (int i = 0; i < N && an < K; ++i) an *= A;
        Wd = (int)(K < an ? K : an);
        if (Wd < 1) Wd = 1;
    }
    // Node pool per tree: the nodes a search can create, the root and at most Wd children for each of
    // the S + 1 expansions (prepare + one per simulation).  The reference allocates K * (S + 2)
    // (cnode.cpp:562); sizing by what is reachable picks the smallest layout class (3m K = 10:
    // 460 nodes, not 1,040).  More expansions than simulation_num are refused either way (the
    // engine stream and value-entry capacity are sized for S).
    const long long P = 1 + (long long)Wd * (S + 1);
    if ((long long)B * P > 0xffffffffll)  // arena_hot's 32-bit offsets (> 256 GiB of node records)
        return fail(MZ_ERR_UNSUPPORTED, "root_num * (1 + min(K, A^N) * (simulation_num + 1)) >= 2^32 nodes");
    auto *b = new mz_batch;
    b->B = B;
    b->N = N;
    b->A = A;
    b->NA = N * A;
    b->K = K;
    b->S = S;
    b->P = (int)P;
    b->E = S + 1;
    b->PS = S + 2;
    b->Wd = Wd;
    // RNG words a search can consume: 2KN per expansion (S+1 of them, +1 slack) and at most
    // (leaf depth) words per selection, sum_{s<=S} (s+1); rounded up to whole 624-word blocks.
    {
        const long long need = 2ll * K * N * (S + 2) + (long long)(S + 1) * (S + 2) / 2 + kRngWin;
        const long long w = ((need + kMtN - 1) / kMtN) * kMtN;
        if (w > 0x7fffffffll) {
            delete b;
            return fail(MZ_ERR_UNSUPPORTED, "engine stream of a tree >= 2^31 words (sampled_times * simulation_num)");
        }
        b->W = (int)w;
    }
    if (hipGetDevice(&b->device) != hipSuccess) {
        delete b;
        return fail(MZ_ERR_DEVICE, "no HIP device");
    }
    Geo &g = b->geo;
    g.B = B;
    g.A = A;
    g.K = K;
    g.S = S;
    g.P = b->P;
    g.E = b->E;
    g.W = b->W;
    g.PS = b->PS;
    g.root_offset = root_offset;
    g.seed = seed;
    g.one_minus_rho = 1 - rho;
    g.delta = delta_lb;
    b->consts_ok = (delta_lb > 0.f && std::isfinite(delta_lb) && lam >= 0.f && lam <= 1.f) ? 1 : 0;
    {
        // worst case of sum(visits) over a path: every value entry of the tree
        const long long worst = 1ll + S + (long long)S * (S + 1) / 2;
        long long cap = worst < 4096 ? worst : 4096;  // <= 32 KiB of staged entries per chunk
        if (cap < S + 1) cap = S + 1;
        g.reg_cap = (int)cap;
    }
    g.TT = (int)table_entries((unsigned)g.PS);
    g.use_table = (g.PS <= (int)kTableFullPS && 4ll * g.TT <= kTableLdsMax) ? 1 : 0;
#ifdef MZ_NO_TABLE
    g.use_table = 0;
#endif
    auto lay = [&]() {
    int o = 0;
    g.oA = o; o += round16(16 * g.P);
    g.oB = o; o += round16(16 * g.P);
    g.oQ = o; o += round16(4 * g.P);
    g.oPP = o; o += round16(4 * g.P);
    g.oVs = o; o += round16(4 * g.P);
    g.oC = o; o += round16(16 * g.P);
    g.oPath = o; o += round16(8 * g.PS);
    g.oFlag = o; o += round16(4 * (g.P > g.PS ? g.P : g.PS));  // per node: tie-list sizes (select_walk)
    g.oT = o; o += g.use_table ? round16(4 * g.TT) : 0;
    g.oPb = o; o += round16(4 * (g.PS + kWave));
    g.oSq = o; o += round16(8 * (g.PS + kWave));
    g.oLp = o; o += round16(4 * (g.PS + 1 + kWave));
    g.oRng = o; o += round16(4 * kRngWin);
    g.oBoot = o; o += round16(4 * (g.PS + kWave));
    g.oReg = o; o += round16(8 * g.reg_cap);
    g.oX = o; o += round16(8 * (2 * MZ_S_COUNT + 4));
    g.oPar = o; o += round16(4 * g.P);
    g.oSc = o; o += round16(4 * g.P);
    g.N = N;
    g.NA = N * A;
    g.JP = (N > 1) ? round16(b->P * N) : 0;
    if (N > 1) {
        g.oJ = o; o += round16(b->P * N);
        g.oJpol = o; o += round16(4 * g.NA);
        g.oJbet = o; o += round16(4 * g.NA);
        g.oJcp = o; o += round16(8 * g.NA);
        g.oJdraw = o; o += round16(4 * kWave * N);
    } else {
        g.oJ = g.oJpol = g.oJbet = g.oJcp = g.oJdraw = 0;
    }
    g.lds = o;
    };
    lay();
    if (g.lds > 160 * 1024 && N == 1) {
        // a pool too large for the LDS image as laid out: the pUCT coefficients from the pb / sq
        // tables instead of a staged table, and smaller value-entry chunks (the back-propagation
        // stages a path node's entries chunk by chunk), before refusing the tree (k_step's general
        // layout: 3m-sized actions at K = 10 reach S = 200 this way)
        g.use_table = 0;
        if (g.reg_cap > 512) g.reg_cap = (S + 1 > 512) ? S + 1 : 512;
        lay();
    }
    // compile-time layout class (pb / sq pUCT tables, value-entry chunks of kRegCap)
    b->nc = 0;
    for (int nc : {64, 128, 256, 384, 512, 1024})
        if (b->P <= nc) {
            b->nc = nc;
            break;
        }
#ifdef MZ_DYNAMIC_LAYOUT
    b->nc = 0;
#endif
    if (N > 1) b->nc = 0;  // joint-action trees use the general layout (joint regions from Geo)
    if (b->nc) {
        g.use_table = 0;
        if (g.reg_cap > kRegCap) g.reg_cap = kRegCap;
        switch (b->nc) {
            case 64: g.lds = Layout<64>::total; break;
            case 128: g.lds = Layout<128>::total; break;
            case 256: g.lds = Layout<256>::total; break;
            case 384: g.lds = Layout<384>::total; break;
            case 512: g.lds = Layout<512>::total; break;
            default: g.lds = Layout<1024>::total; break;
        }
    }
    // a pool whose LDS image does not fit one CU (or MZ_HBM=1 at mz_create, for tests): every step
    // launch of the handle is k_hbm, which keeps the tree in the arena (the reference allocates
    // K * (S + 2) nodes for any K and S, cnode.cpp:553-577)
    b->hbm = g.lds > 160 * 1024 || A > kMaxActions || K > 4096 || getenv_flag("MZ_HBM");
    if (b->hbm) b->nc = 0;
    if (!b->hbm && K == 1 && N == 1 && !getenv_flag("MZ_NO_CHAIN")) {
        b->chain_nc = 0;
        for (int nc : {64, 128, 256, 512, 1024})
            if (b->P <= nc) {
                b->chain_nc = nc;
                break;
            }
        if (chain_lds_bytes(b->P, b->chain_nc) + 16 * 16 * kWave > 160 * 1024) b->chain_nc = -1;
    }
    // (k_tree stages one path node's value entries per slot: E <= kBkCap)
    if (!b->hbm && N == 1 && K >= 2 && K <= kWave && b->nc > 0 && g.E <= (b->nc == 512 ? kBkCapN<512> : kBkCap) && !getenv_flag("MZ_NO_TREE")) {
        b->tree_nc = b->nc;
        // searches of S + 1 <= 128 in the 1024-node class: the ~80 KB layout, two workgroups per CU
        if (b->nc == 1024 && g.E <= kBkCapN<kTree1024S> && !getenv_flag("MZ_NO_TREE_1024S")) b->tree_nc = kTree1024S;
    }
    b->zc = !getenv_flag("MZ_HOST_COPY");
    b->fused_rb = !getenv_flag("MZ_NO_FUSED_READBACK");
    Dev &d = b->dev;
    const size_t nodes = (size_t)B * b->P;
    int rc = 0;
    // One device allocation for every array of the handle, the arrays each launch touches first:
    // every distinct allocation a kernel touches costs it a serialised address-translation miss
    // (~270 cycles each, measured with scripts/ulat.hip), so the per-launch working set is packed
    // into as few 2 MiB pages as possible.
    {
        ArenaPlan plan;
        plan.ptr(&b->prm, 1);
        plan.dev<int4>(d.o_A, nodes);
        plan.dev<int>(d.o_Par, nodes);
        plan.dev<int4>(d.o_Bn, nodes);
        plan.dev<float>(d.o_Q, nodes);
        plan.dev<float>(d.o_PP, nodes);
        plan.dev<float4>(d.o_C, nodes);
        plan.dev<TreeHdr>(d.o_hdr, (size_t)B);
        plan.dev<long long>(d.o_stats, (size_t)B * MZ_S_COUNT);
        plan.dev<int>(d.o_err, 1);
        plan.dev<unsigned>(d.o_seed, 1);
        plan.dev<float>(d.o_lp, (size_t)b->PS + 1 + kWave);
        plan.dev<float>(d.o_T, (size_t)g.TT + 4 * kWave);
        plan.dev<float>(d.o_pb, (size_t)b->PS + kWave);
        plan.dev<double>(d.o_sq, (size_t)b->PS + kWave);
        plan.dev<int2>(d.o_path, (size_t)B * b->PS);
        plan.dev<int2>(d.o_V, nodes * b->E);
        plan.dev<unsigned>(d.o_R, (size_t)B * b->W);
        plan.dev<float4>(d.o_D, nodes);
        b->mem_tables = ArenaPlan::span(4 * ((size_t)g.TT + 4 * kWave)) + ArenaPlan::span(4 * ((size_t)b->PS + kWave)) +
                        ArenaPlan::span(8 * ((size_t)b->PS + kWave));
        b->mem_values = ArenaPlan::span(8 * nodes * b->E);
        b->mem_stream = ArenaPlan::span(4 * (size_t)B * b->W);
        b->mem_nodes = 4 * ArenaPlan::span(16 * nodes) + 3 * ArenaPlan::span(4 * nodes);
        plan.ptr(&b->sel_dev, (size_t)B * (2 + N));
        plan.ptr(&b->in_dev, (size_t)B * (2 + 3 * (size_t)N * A));
        b->rb_words = (size_t)2 * B + 2 * (size_t)B * N * A + (size_t)MZ_F_COUNT * B * b->Wd * N;
        if (N > 1) plan.dev<unsigned char>(d.o_J, (size_t)B * g.JP);
        plan.ptr(&b->rb_dev, b->rb_words);
        plan.ptr(&b->rb_desc_dev, sizeof(b->rb_desc_host) / sizeof(RbDesc));
        rc = plan.allocate(b, d);
        if (!rc) {
            Dev chk = d;
            arena_hot(chk, B, b->P, b->PS);
            const bool same = chk.o_hdr == d.o_hdr && chk.o_stats == d.o_stats && chk.o_err == d.o_err &&
                              chk.o_seed == d.o_seed && chk.o_lp == d.o_lp && chk.o_T == d.o_T && chk.o_pb == d.o_pb &&
                              chk.o_sq == d.o_sq && chk.o_A == d.o_A && chk.o_Par == d.o_Par && chk.o_Bn == d.o_Bn &&
                              chk.o_Q == d.o_Q && chk.o_PP == d.o_PP && chk.o_C == d.o_C && chk.o_path == d.o_path &&
                              chk.o_V == d.o_V && b->E == b->PS - 1;
            if (!same || (char *)b->prm != (char *)d.base)
                rc = fail(MZ_ERR_RUNTIME, "internal: arena layout differs from arena_hot()");
        }
    }
    if (rc) {
        std::string m = g_err;
        mz_destroy(b);
        return fail(MZ_ERR_DEVICE, m);
    }
    // k_chain3 takes P and PS in 10 bits each (its pools have <= 256 nodes)
    // (pools above 256 nodes keep k_chain: wave 1 holds the chain's records in registers, 8 per 64 nodes)
    if (b->chain_nc > 0 && b->chain_nc <= 256 && b->P < 1024 && b->PS < 1024 && !getenv_flag("MZ_CHAIN_V2"))
        b->chain3_nc = b->chain_nc;
    const unsigned *seed_cp = nullptr;
    unsigned seed_cp_n = 0;
    if (!getenv_flag("MZ_NO_SEED_TABLE"))
        seed_table(b->device, 255ull * 2333ull + (unsigned long long)(root_offset > 0 ? root_offset : 0) + (unsigned long long)B,
                   &seed_cp, &seed_cp_n);
    b->seed_ref = seed_cp != nullptr;
    const Params host_params{b->geo, b->dev, seed_cp, seed_cp_n};
    {
        // one launch on the device's init stream, waited for here (the handle's stream is bound later)
        hipStream_t is = init_stream(b->device);
        const int hw = (int)(sizeof(TreeHdr) / 4) * B, sw = 2 * MZ_S_COUNT * B;
        const int nblk = (int)std::min<long long>(1024, ((long long)(hw > sw ? hw : sw) + 255) / 256 + 1);
        hipLaunchKernelGGL(k_init, dim3(nblk), dim3(256), 0, is, host_params, seed, lam, b->PS + 1 + kWave, hw, sw);
        if (!is || hipGetLastError() != hipSuccess || hipStreamSynchronize(is) != hipSuccess) {
            (void)hipGetLastError();
            mz_destroy(b);
            return fail(MZ_ERR_DEVICE, "device initialisation failed");
        }
    }
    if (b->hbm) {
        const int hl = hbm_lds_bytes(N, b->NA);
        if (hl > 48 * 1024) {
            const auto attr = hipFuncAttributeMaxDynamicSharedMemorySize;
            (void)hipFuncSetAttribute((const void *)k_hbm<true, true, true>, attr, hl);
            (void)hipFuncSetAttribute((const void *)k_hbm<true, false, true>, attr, hl);
            (void)hipFuncSetAttribute((const void *)k_hbm<false, true, true>, attr, hl);
        }
    }
    if (N > 1) {  // k_prepare's dynamic LDS for the root's joint inputs (mz_prepare)
        const int jl = ((12 * b->NA + 15) & ~15) + 8 * b->NA + 4 * kWave * N;
        if (jl > 48 * 1024)
            (void)hipFuncSetAttribute((const void *)k_prepare, hipFuncAttributeMaxDynamicSharedMemorySize, jl);
    }
    if (!b->hbm && g.lds > 64 * 1024) {
#ifndef MZ_NO_JOINT
        if (N > 1) set_lds_limit<0, true>(g.lds);
        else
#endif
        switch (b->nc) {
            case 64: set_lds_limit<64>(g.lds); break;
            case 128: set_lds_limit<128>(g.lds); break;
            case 256: set_lds_limit<256>(g.lds); break;
            case 384: set_lds_limit<384>(g.lds); break;
            case 512: set_lds_limit<512>(g.lds); break;
            case 1024: set_lds_limit<1024>(g.lds); break;
            default: set_lds_limit<0>(g.lds); break;
        }
    }
    if (b->tree_nc > 0 && tree_lds_bytes(b->tree_nc) > 64 * 1024) {
        const auto attr = hipFuncAttributeMaxDynamicSharedMemorySize;
        const int tl = tree_lds_bytes(b->tree_nc);
        switch (b->tree_nc) {
            case 64: (void)hipFuncSetAttribute((const void *)k_tree<64, true>, attr, tl); (void)hipFuncSetAttribute((const void *)k_tree<64, false>, attr, tl); break;
            case 128: (void)hipFuncSetAttribute((const void *)k_tree<128, true>, attr, tl); (void)hipFuncSetAttribute((const void *)k_tree<128, false>, attr, tl); break;
            case 256: (void)hipFuncSetAttribute((const void *)k_tree<256, true>, attr, tl); (void)hipFuncSetAttribute((const void *)k_tree<256, false>, attr, tl); break;
            case 384: (void)hipFuncSetAttribute((const void *)k_tree<384, true>, attr, tl); (void)hipFuncSetAttribute((const void *)k_tree<384, false>, attr, tl); break;
            case 512: (void)hipFuncSetAttribute((const void *)k_tree<512, true>, attr, tl); (void)hipFuncSetAttribute((const void *)k_tree<512, false>, attr, tl); break;
            case kTree1024S: (void)hipFuncSetAttribute((const void *)k_tree<kTree1024S, true>, attr, tl); (void)hipFuncSetAttribute((const void *)k_tree<kTree1024S, false>, attr, tl); break;
            default: (void)hipFuncSetAttribute((const void *)k_tree<1024, true>, attr, tl); (void)hipFuncSetAttribute((const void *)k_tree<1024, false>, attr, tl); break;
        }
    }
    if (b->chain_nc >= 0) {
        const int cl = chain_lds_bytes(b->P, b->chain_nc) + 16 * 16 * kWave;
        if (cl > 64 * 1024) {
            const auto attr = hipFuncAttributeMaxDynamicSharedMemorySize;
            switch (b->chain_nc) {
                case 64: (void)hipFuncSetAttribute((const void *)k_chain<64, true>, attr, cl); (void)hipFuncSetAttribute((const void *)k_chain<64, false>, attr, cl); break;
                case 128: (void)hipFuncSetAttribute((const void *)k_chain<128, true>, attr, cl); (void)hipFuncSetAttribute((const void *)k_chain<128, false>, attr, cl); break;
                case 256: (void)hipFuncSetAttribute((const void *)k_chain<256, true>, attr, cl); (void)hipFuncSetAttribute((const void *)k_chain<256, false>, attr, cl); break;
                case 512: (void)hipFuncSetAttribute((const void *)k_chain<512, true>, attr, cl); (void)hipFuncSetAttribute((const void *)k_chain<512, false>, attr, cl); break;
                case 1024: (void)hipFuncSetAttribute((const void *)k_chain<1024, true>, attr, cl); (void)hipFuncSetAttribute((const void *)k_chain<1024, false>, attr, cl); break;
                default: (void)hipFuncSetAttribute((const void *)k_chain<0, true>, attr, cl); (void)hipFuncSetAttribute((const void *)k_chain<0, false>, attr, cl); break;
            }
        }
    }
    *out = b;
    return MZ_OK;
}

int mz_destroy(mz_batch *b) {
    if (!b) return MZ_OK;
    if (b->stream) (void)hipStreamSynchronize(b->stream);
    else (void)hipDeviceSynchronize();
    // (a staged host-memory expansion nobody reads any more is dropped)
    for (void *p : b->allocs)
        if (!(b->arena_bytes && arena_cache().give(b->device, b->arena_bytes, p, kArenaCacheBytes, kArenaCacheBlocks)))
            (void)hipFree(p);
    if (b->stage && !stage_cache().give(-1, b->stage_bytes, b->stage, kStageCacheBytes, kStageCacheBlocks))
        (void)hipHostFree(b->stage);
    if (b->order_ev) (void)hipEventDestroy(b->order_ev);
    if (b->st_ev) (void)hipEventDestroy(b->st_ev);
    if (b->seed_ref) seed_table_release(b->device);
    delete b;
    return MZ_OK;
}

int mz_set_stream(mz_batch *b, void *stream) {
    if (!b) return fail(MZ_ERR_ARG, "null handle");
    hipStream_t ns = (hipStream_t)stream;
    if (ns == b->stream) return MZ_OK;
    int rc = ensure_device(b);
    if (rc) return rc;
    // The new stream waits for the eager work the handle enqueued last (order_ev, recorded behind it
    // by that call): the old stream itself is never touched -- not even to launch a staged host-memory
    // expansion, which runs on the new stream after the wait -- so one the caller has destroyed
    // since is harmless.  Not across a graph-capture boundary: a capture orders nothing outside it and
    // may not wait on an event recorded outside it.
    hipStreamCaptureStatus cn = hipStreamCaptureStatusNone;
    HIP_TRY(hipStreamIsCapturing(ns, &cn));
    if (cn != hipStreamCaptureStatusNone && b->pend) {  // (eager work cannot enter a capture: as it was)
        rc = flush_pending(b);
        mark_order(b);
        if (rc) return rc;
    }
    if (b->order_live && cn == hipStreamCaptureStatusNone) HIP_TRY(hipStreamWaitEvent(ns, b->order_ev, 0));
    b->order_live = false;
    b->stream = ns;
    OrderMark om{b};
    return flush_pending(b);
}

int mz_synchronize(mz_batch *b) {
    if (!b) return fail(MZ_ERR_ARG, "null handle");
    OrderMark om{b};
    int rc = ensure_device(b);
    if (rc) return rc;
    rc = flush_pending(b);
    if (rc) return rc;
    return check_device_errors(b);
}

int mz_prepare(mz_batch *b, const float *rewards, const float *values, const float *policy, const float *beta, int K,
               float noise_eps, const float *noises, int mem) {
    if (!b) return fail(MZ_ERR_ARG, "null handle");
    OrderMark om{b};
    if (K < 1 || K > b->K) return fail(MZ_ERR_UNSUPPORTED, "sampled_times must be in [1, the constructor's value]");
    int rc = ensure_device(b);
    if (rc) return rc;
    rc = flush_pending(b);
    if (rc) return rc;
    const size_t B = b->B, NA = (size_t)b->NA;
    PrepArgs a;
    if (mem == MZ_MEM_HOST) {  // one copy out of the pinned stage
        rc = stage_wait(b);
        if (rc) return rc;
        stage_pack(b, rewards, values, policy, beta, noises);
        rc = stage_upload(b, stage_in_words(b));
        if (rc) return rc;
        const float *p = stage_src(b);
        a.reward = p;
        a.value = p + B;
        a.policy = p + 2 * B;
        a.beta = p + 2 * B + B * NA;
        a.noise = p + 2 * B + 2 * B * NA;
    } else if (mem == MZ_MEM_DEVICE) {
        a.reward = rewards;
        a.value = values;
        a.policy = policy;
        a.beta = beta;
        a.noise = noises;
    } else {
        return fail(MZ_ERR_ARG, "bad memory kind");
    }
    a.eps = noise_eps;
    a.K = K;
    a.idx_x = a.idy = a.act = nullptr;
    const size_t jl = (b->N > 1) ? (size_t)((12 * b->NA + 15) & ~15) + 8 * (size_t)b->NA + 4 * (size_t)kWave * b->N : 0;
    b->dirty = true;
    hipLaunchKernelGGL(k_prepare, dim3(b->B), dim3(256), jl, b->stream, b->prm, a);
    HIP_TRY(hipGetLastError());
    b->rb_valid = b->rb_dev_valid = false;
    b->prepared = true;
    b->expansions = 1;
    if (mem == MZ_MEM_HOST) return check_device_errors(b);
    return MZ_OK;
}

int mz_prepare_select(mz_batch *b, const float *rewards, const float *values, const float *policy, const float *beta,
                      int K, float noise_eps, const float *noises, float c2, float c1, float discount, int32_t *idx_x,
                      int32_t *idy, int32_t *actions) {
    if (!b) return fail(MZ_ERR_ARG, "null handle");
    OrderMark om{b};
    if (K < 1 || K > b->K) return fail(MZ_ERR_UNSUPPORTED, "sampled_times must be in [1, the constructor's value]");
    if (!idx_x || !idy || !actions) return fail(MZ_ERR_ARG, "null selection output");
    if (b->N > 1) {  // joint-action trees: the two calls
        int rc = mz_prepare(b, rewards, values, policy, beta, K, noise_eps, noises, MZ_MEM_DEVICE);
        if (rc) return rc;
        return mz_select(b, c2, c1, discount, idx_x, idy, actions, MZ_MEM_DEVICE);
    }
    int rc = ensure_device(b);
    if (rc) return rc;
    rc = flush_pending(b);
    if (rc) return rc;
    rc = ensure_tables(b, c2, c1);  // (for the launches that follow; the first selection needs none)
    if (rc) return rc;
    PrepArgs a;
    a.reward = rewards;
    a.value = values;
    a.policy = policy;
    a.beta = beta;
    a.noise = noises;
    a.eps = noise_eps;
    a.K = K;
    a.idx_x = idx_x;
    a.idy = idy;
    a.act = actions;
    b->dirty = true;
    hipLaunchKernelGGL(k_prepare, dim3(b->B), dim3(256), 0, b->stream, b->prm, a);
    HIP_TRY(hipGetLastError());
    b->rb_valid = b->rb_dev_valid = false;
    b->prepared = true;
    b->expansions = 1;
    return MZ_OK;
}

int mz_select(mz_batch *b, float c2, float c1, float discount, int32_t *idx_x, int32_t *idy, int32_t *actions,
              int mem) {
    if (!b) return fail(MZ_ERR_ARG, "null handle");
    OrderMark om{b};
    if (!b->prepared) return fail(MZ_ERR_RUNTIME, "batch_selection before prepare");
    int rc = ensure_device(b);
    if (rc) return rc;
    rc = ensure_tables(b, c2, c1);
    if (rc) return rc;
    if (mem != MZ_MEM_HOST && mem != MZ_MEM_DEVICE) return fail(MZ_ERR_ARG, "bad memory kind");
    const bool fuse = mem == MZ_MEM_HOST && b->pend;  // the staged expansion + this selection, one launch
    if (!fuse) {
        rc = flush_pending(b);
        if (rc) return rc;
    }
    StepArgs a{};
    if (fuse) {
        b->pend = false;
        rc = stage_upload(b, 2 * (size_t)b->B * (1 + (size_t)b->NA));
        if (rc) return rc;
        a = staged_expand_args(b);
    }
    a.discount = discount;
    if (mem == MZ_MEM_HOST) {
        rc = ensure_stage(b);
        if (rc) return rc;
        // zero-copy: the kernel writes the selection into the stage's device mapping
        int32_t *o = b->zc ? b->st_sel_d : b->sel_dev;
        a.idx_x = o;
        a.idy = o + b->B;
        a.act = o + 2 * b->B;
    } else {
        a.idx_x = idx_x;
        a.idy = idy;
        a.act = actions;
    }
    rc = launch_step(b, fuse, true, a);
    if (rc) return rc;
    if (mem == MZ_MEM_HOST) {  // selection + error word into the pinned stage, one synchronisation
        const size_t n = stage_sel_words(b);
        if (!b->zc)
            HIP_TRY(hipMemcpyAsync(b->st_sel, b->sel_dev, sizeof(int32_t) * n, hipMemcpyDeviceToHost, b->stream));
        rc = check_device_errors(b);
        if (rc) return rc;
        std::memcpy(idx_x, b->st_sel, sizeof(int32_t) * b->B);
        std::memcpy(idy, b->st_sel + b->B, sizeof(int32_t) * b->B);
        std::memcpy(actions, b->st_sel + 2 * b->B, sizeof(int32_t) * b->B * b->N);
    }
    return MZ_OK;
}

// device-memory inputs of an expansion (host-memory ones go through the pinned stage)
static int expand_inputs(mz_batch *b, const float *rewards, const float *values, const float *policy,
                         const float *beta, StepArgs &a) {
    (void)b;
    a.reward = rewards;
    a.value = values;
    a.policy = policy;
    a.beta = beta;
    return MZ_OK;
}

int mz_expand_backup(mz_batch *b, int hsx, float discount, int K, const float *rewards, const float *values,
                     const float *policy, const float *beta, int mem) {
    if (!b) return fail(MZ_ERR_ARG, "null handle");
    OrderMark om{b};
    if (!b->prepared) return fail(MZ_ERR_RUNTIME, "batch_expansion_and_backup before prepare");
    if (K < 1 || K > b->K) return fail(MZ_ERR_UNSUPPORTED, "sampled_times must be in [1, the constructor's value]");
    if (mem != MZ_MEM_HOST && mem != MZ_MEM_DEVICE) return fail(MZ_ERR_ARG, "bad memory kind");
    int rc = ensure_device(b);
    if (rc) return rc;
    rc = flush_pending(b);
    if (rc) return rc;
    if (mem == MZ_MEM_HOST) {
        // staged in pinned memory; launched by the next call (with batch_selection: one fused
        // launch).  Its device-side errors surface at that call.
        rc = stage_wait(b);
        if (rc) return rc;
        stage_pack(b, rewards, values, policy, beta, nullptr);
        b->pend = true;
        b->pend_hsx = hsx;
        b->pend_disc = discount;
        b->pend_K = K;
        b->rb_valid = b->rb_dev_valid = false;
        return MZ_OK;
    }
    StepArgs a{};
    a.hsx = hsx;
    a.discount = discount;
    a.K = K;
    rc = expand_inputs(b, rewards, values, policy, beta, a);
    if (rc) return rc;
    return launch_step(b, true, false, a);
}

int mz_expand_backup_select(mz_batch *b, int hsx, float discount, int K, const float *rewards, const float *values,
                            const float *policy, const float *beta, float c2, float c1, int32_t *idx_x, int32_t *idy,
                            int32_t *actions, const void *pool, int64_t pool_slot_stride, int64_t row_bytes,
                            void *gather_out) {
    if (!b) return fail(MZ_ERR_ARG, "null handle");
    OrderMark om{b};
    if (!b->prepared) return fail(MZ_ERR_RUNTIME, "expansion before prepare");
    if (K < 1 || K > b->K) return fail(MZ_ERR_UNSUPPORTED, "sampled_times must be in [1, the constructor's value]");
    if (pool && (!gather_out || row_bytes <= 0 || (row_bytes & 3)))
        return fail(MZ_ERR_ARG, "gather needs an output buffer and row_bytes a positive multiple of 4");
    int rc = ensure_device(b);
    if (rc) return rc;
    rc = flush_pending(b);
    if (rc) return rc;
    rc = ensure_tables(b, c2, c1);
    if (rc) return rc;
    StepArgs a{};
    a.hsx = hsx;
    a.discount = discount;
    a.K = K;
    rc = expand_inputs(b, rewards, values, policy, beta, a);
    if (rc) return rc;
    a.idx_x = idx_x;
    a.idy = idy;
    a.act = actions;
    a.pool = (const char *)pool;
    a.pool_stride = pool_slot_stride;
    a.row_bytes = row_bytes;
    a.gather_out = (char *)gather_out;
    return launch_step(b, true, true, a);
}

// include/mzdriver.h
int mz_reseed(mz_batch *b, uint32_t seed) {
    if (!b) return fail(MZ_ERR_ARG, "null handle");
    OrderMark om{b};
    int rc = ensure_device(b);
    if (rc) return rc;
    rc = flush_pending(b);
    if (rc) return rc;
    b->geo.seed = seed;
    b->prepared = false;
    b->dirty = true;
    hipLaunchKernelGGL(k_set_word, dim3(1), dim3(1), 0, b->stream, b->dev.seed(), (unsigned)seed);
    HIP_TRY(hipGetLastError());
    return MZ_OK;
}

int mz_state_changed(mz_batch *b) {
    if (!b) return fail(MZ_ERR_ARG, "null handle");
    OrderMark om{b};
    int rc = flush_pending(b);
    if (rc) return rc;
    b->rb_valid = b->rb_dev_valid = false;
    b->prepared = true;
    return MZ_OK;
}

int mz_fused_kernel(mz_batch *b, char *out, int len) {
    if (!b || !out || len < 1) return fail(MZ_ERR_ARG, "mz_fused_kernel: null argument");
    char name[48];
    if (b->hbm) std::snprintf(name, sizeof name, b->N > 1 ? "k_hbm<joint>" : "k_hbm");
    else if (b->chain3_nc > 0) std::snprintf(name, sizeof name, "k_chain3<%d>", b->chain3_nc);
    else if (b->chain_nc >= 0) std::snprintf(name, sizeof name, "k_chain<%d>", b->chain_nc);
    else if (b->tree_nc == kTree1024S) std::snprintf(name, sizeof name, "k_tree<1024,s128>");
    else if (b->tree_nc > 0) std::snprintf(name, sizeof name, "k_tree<%d>", b->tree_nc);
    else if (b->N > 1) std::snprintf(name, sizeof name, "k_step<0,joint>");
    else std::snprintf(name, sizeof name, "k_step<%d>", b->nc);
    std::snprintf(out, (size_t)len, "%s", name);
    return MZ_OK;
}

int mz_trim_caches(int64_t *released) {
    const size_t n = arena_cache().drain(-1, false) + stage_cache().drain(-1, true) + seed_table_trim();
    if (released) *released = (int64_t)n;
    return MZ_OK;
}

// Internal hooks for the driver-glue TU (csrc/mz_internal.h).
int mz_internal_fail(int code, const char *msg) { return fail(code, msg); }

int mz_internal_launch_info(mz_batch *b, int *B, int *A, hipStream_t *stream) {
    if (!b) return fail(MZ_ERR_ARG, "null handle");
    int rc = ensure_device(b);
    if (rc) return rc;
    rc = flush_pending(b);
    if (rc) return rc;
    *B = b->B;
    *A = b->A;
    *stream = b->stream;
    return MZ_OK;
}

int mz_internal_agent_num(mz_batch *b) { return b ? b->N : 0; }

void mz_internal_enqueued(mz_batch *b) {
    if (!b) return;
    b->dirty = true;
    mark_order(b);
}

int mz_gather_rows(mz_batch *b, const void *pool, int64_t stride, int64_t row_bytes, const int32_t *idx_x, void *out) {
    if (!b) return fail(MZ_ERR_ARG, "null handle");
    OrderMark om{b};
    if (row_bytes <= 0 || (row_bytes & 3)) return fail(MZ_ERR_ARG, "row_bytes must be a positive multiple of 4");
    int rc = ensure_device(b);
    if (rc) return rc;
    rc = flush_pending(b);
    if (rc) return rc;
    b->dirty = true;
    hipLaunchKernelGGL(k_gather, dim3(b->B), dim3(kWave), 0, b->stream, (const char *)pool, (long long)stride,
                       (long long)row_bytes, (const int *)idx_x, (char *)out);
    HIP_TRY(hipGetLastError());
    return MZ_OK;
}

int mz_get_roots_device(mz_batch *b, float discount, const mz_readback_out *out) {
    if (!b) return fail(MZ_ERR_ARG, "null handle");
    OrderMark om{b};
    if (!out) return fail(MZ_ERR_ARG, "null output list");
    int rc = ensure_device(b);
    if (rc) return rc;
    rc = flush_pending(b);
    if (rc) return rc;
    RbPtrs o;
    o.values = out->values;
    o.mv = out->marginal_visit_count;
    o.mp = out->marginal_priors;
    o.deg = out->degrees;
    for (int f = 0; f < MZ_F_COUNT; ++f) o.f[f] = (int *)out->sampled[f];
    b->dirty = true;
    hipLaunchKernelGGL(k_readback, dim3(b->B), dim3(kWave), 0, b->stream, b->prm, discount, b->Wd, o);
    HIP_TRY(hipGetLastError());
    return MZ_OK;
}

// include/mzdriver.h
int mz_expand_backup_readback(mz_batch *b, int hsx, float discount, int K, const float *rewards, const float *values,
                              const float *policy, const float *beta, float readback_discount,
                              const mz_readback_out *out) {
    if (!b) return fail(MZ_ERR_ARG, "null handle");
    OrderMark om{b};
    if (!b->prepared) return fail(MZ_ERR_RUNTIME, "batch_expansion_and_backup before prepare");
    if (K < 1 || K > b->K) return fail(MZ_ERR_UNSUPPORTED, "sampled_times must be in [1, the constructor's value]");
    int rc = ensure_device(b);
    if (rc) return rc;
    rc = flush_pending(b);
    if (rc) return rc;
    RbPtrs o;
    if (out) {
        o.values = out->values;
        o.mv = out->marginal_visit_count;
        o.mp = out->marginal_priors;
        o.deg = out->degrees;
        for (int f = 0; f < MZ_F_COUNT; ++f) o.f[f] = (int *)out->sampled[f];
    } else {
        o = packed_rb(b);
    }
    StepArgs a{};
    a.hsx = hsx;
    a.discount = discount;
    a.K = K;
    rc = expand_inputs(b, rewards, values, policy, beta, a);
    if (rc) return rc;
    // the chain and tree kernels write the readback themselves (their SEL = false launches take the
    // descriptor in the gather_out slot); the other kernels are followed by k_readback
    const bool fusable = b->fused_rb && (b->chain3_nc > 0 || b->tree_nc > 0);
    const RbDesc *slot = fusable ? rb_desc_slot(b, o, readback_discount) : nullptr;
    a.gather_out = (char *)slot;
    rc = launch_step(b, true, false, a);
    if (rc) return rc;
    if (!slot) {
        b->dirty = true;
        hipLaunchKernelGGL(k_readback, dim3(b->B), dim3(kWave), 0, b->stream, b->prm, readback_discount, b->Wd, o);
        HIP_TRY(hipGetLastError());
    }
    if (!out) {  // the packed buffer now mirrors the trees
        b->rb_dev_valid = true;
        b->rb_valid = false;
        b->rb_disc = readback_discount;
    }
    return MZ_OK;
}

int mz_readback_ready(mz_batch *b, float discount) {
    if (!b) return fail(MZ_ERR_ARG, "null handle");
    OrderMark om{b};
    int rc = flush_pending(b);
    if (rc) return rc;
    b->prepared = true;
    b->rb_valid = false;
    b->rb_dev_valid = true;
    b->rb_disc = discount;
    return MZ_OK;
}

int mz_get_roots_values(mz_batch *b, float *out, int mem) {
    if (!b) return fail(MZ_ERR_ARG, "null handle");
    OrderMark om{b};
    int rc = ensure_device(b);
    if (rc) return rc;
    if (mem == MZ_MEM_DEVICE) {
        rc = readback_dev(b, b->rb_dev_valid ? b->rb_disc : 0.f);
        if (rc) return rc;
        rc = copy_words(b, out, b->rb_dev, (size_t)b->B);
        if (rc) return rc;
        return MZ_OK;
    }
    rc = readback(b, (b->rb_valid || b->rb_dev_valid) ? b->rb_disc : 0.f);
    if (rc) return rc;
    std::memcpy(out, b->rb_host, 4 * (size_t)b->B);
    return MZ_OK;
}

int mz_get_roots_marginal_visit_count(mz_batch *b, int32_t *out, int mem) {
    if (!b) return fail(MZ_ERR_ARG, "null handle");
    OrderMark om{b};
    int rc = ensure_device(b);
    if (rc) return rc;
    rc = (mem == MZ_MEM_DEVICE) ? readback_dev(b, b->rb_dev_valid ? b->rb_disc : 0.f)
                                : readback(b, (b->rb_valid || b->rb_dev_valid) ? b->rb_disc : 0.f);
    if (rc) return rc;
    const size_t n = (size_t)b->B * b->NA;
    if (mem == MZ_MEM_DEVICE) {
        rc = copy_words(b, out, b->rb_dev + b->B, n);
        if (rc) return rc;
        return MZ_OK;
    }
    std::memcpy(out, b->rb_host + b->B, 4 * n);
    return MZ_OK;
}

int mz_get_roots_marginal_priors(mz_batch *b, float *out, int mem) {
    if (!b) return fail(MZ_ERR_ARG, "null handle");
    OrderMark om{b};
    int rc = ensure_device(b);
    if (rc) return rc;
    rc = (mem == MZ_MEM_DEVICE) ? readback_dev(b, b->rb_dev_valid ? b->rb_disc : 0.f)
                                : readback(b, (b->rb_valid || b->rb_dev_valid) ? b->rb_disc : 0.f);
    if (rc) return rc;
    const size_t n = (size_t)b->B * b->NA;
    if (mem == MZ_MEM_DEVICE) {
        rc = copy_words(b, out, b->rb_dev + b->B + n, n);
        if (rc) return rc;
        return MZ_OK;
    }
    std::memcpy(out, b->rb_host + b->B + n, 4 * n);
    return MZ_OK;
}

int mz_get_num_children_of_root(mz_batch *b, int tree_id, int32_t *out) {
    if (!b) return fail(MZ_ERR_ARG, "null handle");
    if (tree_id < 0 || tree_id >= b->B) return fail(MZ_ERR_ARG, "tree_id out of range");
    int rc = ensure_device(b);
    if (rc) return rc;
    rc = readback(b, (b->rb_valid || b->rb_dev_valid) ? b->rb_disc : 0.f);
    if (rc) return rc;
    *out = b->rb_host[rb_deg_base(b) + tree_id];
    return MZ_OK;
}

int mz_max_children(mz_batch *b, int32_t *out) {
    if (!b) return fail(MZ_ERR_ARG, "null handle");
    *out = b->Wd;
    return MZ_OK;
}

int mz_get_root_sampled(mz_batch *b, int field, int tree_id, float discount, void *out) {
    if (!b) return fail(MZ_ERR_ARG, "null handle");
    if (tree_id < 0 || tree_id >= b->B) return fail(MZ_ERR_ARG, "tree_id out of range");
    if (field < 0 || field >= MZ_F_COUNT) return fail(MZ_ERR_ARG, "unknown field");
    int rc = ensure_device(b);
    if (rc) return rc;
    rc = readback(b, field == MZ_F_QVALUES ? discount : ((b->rb_valid || b->rb_dev_valid) ? b->rb_disc : discount));
    if (rc) return rc;
    const int deg = b->rb_host[rb_deg_base(b) + tree_id];
    const size_t per = (field == MZ_F_ACTIONS) ? (size_t)b->N : 1;
    std::memcpy(out, b->rb_host + rb_field_base(b, field) + (size_t)tree_id * b->Wd * per, 4 * (size_t)deg * per);
    return MZ_OK;
}

int mz_get_roots_sampled_padded(mz_batch *b, int field, float discount, void *out, int32_t *degrees, int mem) {
    if (!b) return fail(MZ_ERR_ARG, "null handle");
    OrderMark om{b};
    if (field < 0 || field >= MZ_F_COUNT) return fail(MZ_ERR_ARG, "unknown field");
    int rc = ensure_device(b);
    if (rc) return rc;
    const float disc = field == MZ_F_QVALUES ? discount : ((b->rb_valid || b->rb_dev_valid) ? b->rb_disc : discount);
    rc = (mem == MZ_MEM_DEVICE) ? readback_dev(b, disc) : readback(b, disc);
    if (rc) return rc;
    const size_t n = (size_t)b->B * rb_field_width(b, field);
    const size_t dego = rb_deg_base(b);
    if (mem == MZ_MEM_DEVICE) {
        rc = copy_words(b, out, b->rb_dev + rb_field_base(b, field), n);
        if (rc) return rc;
        if (degrees) {
            rc = copy_words(b, degrees, b->rb_dev + dego, (size_t)b->B);
            if (rc) return rc;
        }
        return MZ_OK;
    }
    std::memcpy(out, b->rb_host + rb_field_base(b, field), 4 * n);
    if (degrees) std::memcpy(degrees, b->rb_host + dego, 4 * (size_t)b->B);
    return MZ_OK;
}

#if MZ_SPANS
// diagnostic builds only (not in include/mzmcts.h): reset == 1 zeroes the launch spans; else
// out[((k * trees + t) * 4 + {0, 1, 2, 3}] = slot k's tree t: wave 0 start, wave 0 end, wave 1 end,
// wave 2 end (100 MHz ticks; 0 = no such launch / wave), k < slots <= 256, t < trees <= 1024
int mz_debug_spans(unsigned long long *out, int slots, int trees, int reset) {
    static ulonglong2 host[kSpanSlots][kSpanTrees][2];
    HIP_TRY(hipDeviceSynchronize());
    if (reset) {
        std::memset(host, 0, sizeof(host));
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_span), host, sizeof(host)));
        return MZ_OK;
    }
    if (slots > kSpanSlots || trees > kSpanTrees) return fail(MZ_ERR_ARG, "mz_debug_spans: too many slots / trees");
    HIP_TRY(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_span), sizeof(host)));
    for (int k = 0; k < slots; ++k)
        for (int t = 0; t < trees; ++t) {
            unsigned long long *o = out + ((size_t)k * trees + t) * 4;
            o[0] = host[k][t][0].x;
            o[1] = host[k][t][0].y;
            o[2] = host[k][t][1].x;
            o[3] = host[k][t][1].y;
        }
    return MZ_OK;
}
#endif

#ifdef MZ_ARGCHECK
// diagnostic build only: [0] = record count, [1] = kErrPath site bits, then the records
int mz_debug_dump(unsigned *out, int max_words) {
    int n = 0;
    unsigned sites = 0;
    std::vector<unsigned> rec((size_t)kDbgRecs * kDbgWords);
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_dbg_n), sizeof(int)));
    HIP_TRY(hipMemcpyFromSymbol(&sites, HIP_SYMBOL(g_dbg_sites), sizeof(unsigned)));
    HIP_TRY(hipMemcpyFromSymbol(rec.data(), HIP_SYMBOL(g_dbg), sizeof(unsigned) * rec.size()));
    if (max_words < 2) return fail(MZ_ERR_ARG, "buffer too small");
    out[0] = (unsigned)n;
    out[1] = sites;
    for (int k = 0; k + 2 < max_words && k < (int)rec.size(); ++k) out[k + 2] = rec[k];
    return MZ_OK;
}
// diagnostic build only: n words of the arena from the error word on, and the arena's layout
int mz_debug_peek(mz_batch *b, unsigned *out, int n, unsigned long long *layout) {
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(out, b->dev.err(), sizeof(unsigned) * n, hipMemcpyDeviceToHost));
    layout[0] = (unsigned long long)b->dev.base;
    layout[1] = (unsigned long long)b->dev.err();
    layout[2] = (unsigned long long)b->dev.seed();
    layout[3] = (unsigned long long)b->dev.lp();
    layout[4] = (unsigned long long)b->dev.T();
    layout[5] = (unsigned long long)b->dev.hdr();
    layout[6] = (unsigned long long)b->dev.stats();
    return MZ_OK;
}
#endif

int mz_get_stats(mz_batch *b, int64_t *out) {
    if (!b) return fail(MZ_ERR_ARG, "null handle");
    int rc = ensure_device(b);
    if (rc) return rc;
    rc = flush_pending(b);
    if (rc) return rc;
    std::vector<long long> st((size_t)b->B * MZ_S_COUNT);
    HIP_TRY(hipMemcpyAsync(st.data(), b->dev.stats(), sizeof(long long) * st.size(), hipMemcpyDeviceToHost, b->stream));
    HIP_TRY(hipStreamSynchronize(b->stream));
    for (int k = 0; k < MZ_S_COUNT; ++k) out[k] = 0;
    for (int t = 0; t < b->B; ++t)
        for (int k = 0; k < MZ_S_COUNT; ++k) out[k] += st[(size_t)t * MZ_S_COUNT + k];
    return MZ_OK;
}

int mz_arena_info(mz_batch *b, int64_t *out, int n) {
    if (!b || !out || n < 0) return fail(MZ_ERR_ARG, "mz_arena_info: bad argument");
    const int64_t v[5] = {(int64_t)b->arena_bytes, (int64_t)b->mem_tables, (int64_t)b->mem_values,
                          (int64_t)b->mem_stream, (int64_t)b->mem_nodes};
    for (int i = 0; i < n && i < 5; ++i) out[i] = v[i];
    return MZ_OK;
}

int mz_debug_paths(mz_batch *b, int32_t *header, int32_t *path, int max_levels) {
    if (!b || !header || !path || max_levels < 1) return fail(MZ_ERR_ARG, "mz_debug_paths: bad argument");
    int rc = ensure_device(b);
    if (rc) return rc;
    rc = flush_pending(b);
    if (rc) return rc;
    std::vector<TreeHdr> h(b->B);
    std::vector<int2> pr((size_t)b->B * b->PS);
    std::vector<int4> bn((size_t)b->B * b->P);
    HIP_TRY(hipMemcpyAsync(h.data(), b->dev.hdr(), sizeof(TreeHdr) * h.size(), hipMemcpyDeviceToHost, b->stream));
    HIP_TRY(hipMemcpyAsync(pr.data(), b->dev.path(), sizeof(int2) * pr.size(), hipMemcpyDeviceToHost, b->stream));
    HIP_TRY(hipMemcpyAsync(bn.data(), b->dev.Bn(), sizeof(int4) * bn.size(), hipMemcpyDeviceToHost, b->stream));
    HIP_TRY(hipStreamSynchronize(b->stream));
    const bool chain = !b->hbm && b->chain_nc >= 0;  // (K = 1 chains: no path record)
    for (int t = 0; t < b->B; ++t) {
        const TreeHdr &ht = h[t];
        int32_t *ho = header + (size_t)t * 6;
        ho[0] = ht.cursor;
        ho[1] = ht.tot;
        ho[2] = ht.D;
        ho[3] = ht.err;
        ho[4] = ht.leaf;
        ho[5] = ht.tame;
        for (int i = 0; i < max_levels; ++i) {
            int32_t *po = path + ((size_t)t * max_levels + i) * 4;
            po[0] = po[1] = po[2] = po[3] = -1;
            if (i > ht.D || i >= b->PS || (chain && i > 0)) continue;
            const int2 e = pr[(size_t)t * b->PS + i];
            po[0] = e.x;
            po[1] = e.y;
            if (e.x >= 0 && e.x < b->P) {
                const int4 r = bn[(size_t)t * b->P + e.x];
                po[2] = r.w;
                po[3] = i == 0 ? -1 : (r.y >> 8) & 0xff;
            }
        }
    }
    return MZ_OK;
}

int mz_print(mz_batch *b) {
    if (!b) return fail(MZ_ERR_ARG, "null handle");
    int rc = ensure_device(b);
    if (rc) return rc;
    rc = flush_pending(b);
    if (rc) return rc;
    std::vector<TreeHdr> h(b->B);
    HIP_TRY(hipMemcpyAsync(h.data(), b->dev.hdr(), sizeof(TreeHdr) * b->B, hipMemcpyDeviceToHost, b->stream));
    HIP_TRY(hipStreamSynchronize(b->stream));
    for (int t = 0; t < b->B; ++t)
        fprintf(stderr, "tree %d: nodes %d, rng cursor %d, last path length %d, err %d, minmax [%f, %f] (%d)\n", t,
                h[t].tot, h[t].cursor, h[t].D, h[t].err, h[t].mm_min, h[t].mm_max, h[t].mm_cnt);
    return MZ_OK;
}

}  // extern "C"
