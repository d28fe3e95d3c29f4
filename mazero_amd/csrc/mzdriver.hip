// mzdriver.hip — device glue of the sampled-MCTS driver loop (include/mzdriver.h).
//
// The reference driver (core/mcts/tree_search/mcts_sampled.py:114-172) moves every simulation's
// network outputs to the host and prepares the next tree inputs with numpy.  These kernels do the
// same arithmetic on the device, one wavefront per root, so that the results equal the numpy
// expressions bit for bit:
//   - np.exp on float32: numpy 2.x's SIMD float32 exponential (AVX512F and AVX2/FMA3 loops; same
//     algorithm): k = rint(x * log2 e); y = x + k*(-ln2_hi) + k*(-ln2_lo) with FMAs; exp(y) = P5(y)
//     / Q2(y), Horner with FMAs; result scaled by 2^k.  Validated here against np.exp on ~2e7
//     float32 inputs including the denormal range (tests/test_driver.py checks it on every host).
//   - np.sum(axis=-1) of a contiguous row of n <= 128 elements: pairwise summation base case, 8
//     interleaved accumulators r[j] += a[i + j], combined as ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)),
//     then the n % 8 tail; n < 8 sums sequentially from 0.
//   - float16 arrays (policy logits under torch autocast): numpy's half loops evaluate each
//     operation in float32 and round the result to half; half sums accumulate in float32 and
//     round once.
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <mutex>

#include "../../include/mzdriver.h"
#include "mz_internal.h"

namespace {

constexpr int kWave = 64;

// numpy's float32 exp constants (rational minimax approximation on [-ln2/2, ln2/2]).
constexpr float kLog2e = 1.442695040888963387f;
constexpr float kLn2Hi = -6.93145752e-1f;
constexpr float kLn2Lo = -1.42860677e-6f;
constexpr float kP0 = 9.999999999980870924916e-01f;
constexpr float kP1 = 7.257664613233124478488e-01f;
constexpr float kP2 = 2.473615434895520810817e-01f;
constexpr float kP3 = 5.114512081637298353406e-02f;
constexpr float kP4 = 6.757896990527504603057e-03f;
constexpr float kP5 = 5.082762527590693718096e-04f;
constexpr float kQ0 = 1.0f;
constexpr float kQ1 = -2.742335390411667452936e-01f;
constexpr float kQ2 = 2.159509375685829852307e-02f;

__device__ float np_expf(float x) {
    if (x != x) return x + x;                 // NaN
    if (x > 88.72283935546875f) return INFINITY;
    if (x < -104.0f) return 0.0f;             // below half the smallest denormal
    const float k = rintf(x * kLog2e);        // product rounded to f32, then to nearest even
    float y = fmaf(k, kLn2Hi, x);
    y = fmaf(k, kLn2Lo, y);
    float num = fmaf(kP5, y, kP4);
    num = fmaf(num, y, kP3);
    num = fmaf(num, y, kP2);
    num = fmaf(num, y, kP1);
    num = fmaf(num, y, kP0);
    float den = fmaf(kQ2, y, kQ1);
    den = fmaf(den, y, kQ0);
    return ldexpf(num / den, (int)k);
}

__device__ __forceinline__ float to_half_and_back(float v) { return __half2float(__float2half_rn(v)); }

// np.exp of a float16 array.  numpy does not always evaluate it as float32 exp rounded to half: on
// AVX512_SKX hosts its half loop uses a vectorised float32 exponential of its own, which rounds to a
// different half for a few inputs (4 of the 63,488 finite halves on this image's numpy 2.2).  The
// host hands its numpy's answer for every half bit pattern (mz_set_half_exp_table); without that
// table the kernels round numpy's float32 SIMD exp to half.
__device__ __forceinline__ float np_exp_half(float d, const unsigned short *table) {
    if (table) return __half2float(__ushort_as_half(table[__half_as_ushort(__float2half_rn(d))]));
    return to_half_and_back(np_expf(d));
}

template <bool F16>
__device__ __forceinline__ float np_exp_as(float d, const unsigned short *table) {
    if constexpr (F16) return np_exp_half(d, table);
    return np_expf(d);
}

template <bool F16>
__device__ __forceinline__ float round_as(float v) {
    if constexpr (F16) return to_half_and_back(v);
    return v;
}

template <bool F16>
__device__ __forceinline__ float load_elem(const void *p, long long i) {
    if constexpr (F16) return __half2float(static_cast<const __half *>(p)[i]);
    return static_cast<const float *>(p)[i];
}

// numpy pairwise-sum base case over lds[0..n), n <= 128; result broadcast to every lane.
__device__ float np_row_sum(float v, int l, int n, float *lds, float *acc) {
    if (l < n) lds[l] = v;
    __syncthreads();
    if (n >= 8 && l < 8) {
        const int n8 = n - n % 8;
        float r = lds[l];
        for (int i = 8; i < n8; i += 8) r += lds[i + l];
        acc[l] = r;
    }
    __syncthreads();
    if (l == 0) {
        float res;
        if (n < 8) {
            res = 0.f;
            for (int i = 0; i < n; ++i) res += lds[i];
        } else {
            res = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
            for (int i = n - n % 8; i < n; ++i) res += lds[i];
        }
        acc[8] = res;
    }
    __syncthreads();
    const float out = acc[8];
    __syncthreads();
    return out;
}

__device__ __forceinline__ float wave_max(float v) {
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
    return v;
}

// numpy's `x ** e` for an array x >= 0 of the logits' dtype and the exponent e = 1 / sampled_tau,
// which NEP 50 casts to that dtype (the caller passes it so rounded).  numpy's exponents 2 and 0.5
// are np.square / np.sqrt, its float16 loop is libm's powf rounded to half, and libm's powf is
// correctly rounded in all but ~0.07 % of inputs: the float64 pow rounded to float is the correctly
// rounded result (up to results within a float64 ulp of a float midpoint), so all of these agree
// with it.  numpy's float32 loop on AVX-512 hosts is SVML's powf, which is not correctly rounded
// (about 1 in 5 results is one ulp off); that case is not reproducible here.
// use_pow: 0 no power (exponent 1.0: numpy returns the array), kPowSquare / kPowSqrt (numpy's
// fast_scalar_power for the Python exponents 2.0 and 0.5), kPowGeneral
constexpr int kPowGeneral = 1, kPowSquare = 2, kPowSqrt = 3;
template <bool F16>
__device__ __forceinline__ float np_pow_as(float x, float e, int mode) {
    if (mode == kPowSquare) return round_as<F16>(x * x);
    if (mode == kPowSqrt) return round_as<F16>(sqrtf(x));  // (IEEE: -fhip-fp32-correctly-rounded-divide-sqrt)
    return round_as<F16>((float)pow((double)x, (double)e));
}

int pow_mode(double inv) {
    return inv == 1.0 ? 0 : inv == 2.0 ? kPowSquare : inv == 0.5 ? kPowSqrt : kPowGeneral;
}

// mcts_sampled.py:158-161 (+ .astype(np.float32), :169-170) for root blockIdx.x.
template <bool F16>
__global__ __launch_bounds__(kWave) void k_policy_glue(const void *logits, long long row_stride, long long col_off,
                                                       int A, int use_pow, float tau_inv, float *probs,
                                                       float *beta, const unsigned short *hexp) {
    __shared__ float lds[kWave];
    __shared__ float acc[9];
    const int t = blockIdx.x;
    const int l = threadIdx.x;
    const bool on = l < A;
    const float x = on ? load_elem<F16>(logits, (long long)t * row_stride + col_off + l) : -INFINITY;
    // np.max(..., axis=-1): NaN propagates
    const bool nan_any = __ballot(on && (x != x)) != 0;
    const float m = nan_any ? NAN : wave_max(on ? x : -INFINITY);
    const float d = round_as<F16>(x - m);
    const float e = np_exp_as<F16>(d, hexp);
    const float s = round_as<F16>(np_row_sum(e, l, A, lds, acc));
    const float p = round_as<F16>(e / s);
    // `** (1 / sampled_tau)`: numpy returns the array itself for an exponent of 1.0
    const float q = use_pow ? np_pow_as<F16>(p, tau_inv, use_pow) : p;
    const float s2 = round_as<F16>(np_row_sum(q, l, A, lds, acc));
    const float b = round_as<F16>(q / s2);
    if (on) {
        probs[(long long)t * A + l] = p;
        beta[(long long)t * A + l] = b;
    }
}

// float64 -> float16 with one rounding (round to nearest, ties to even), as numpy casts a float64
// result into a float16 array (npy_double_to_half); via float32 it would round twice.
__device__ float round_d2h(double d) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(d);
    const unsigned short sign = (unsigned short)((b >> 48) & 0x8000u);
    const int ex = (int)((b >> 52) & 0x7ff);
    const unsigned long long mant = b & 0xfffffffffffffull;
    unsigned short h;
    if (ex == 0x7ff) {
        h = (unsigned short)(sign | 0x7c00u | (mant ? 0x200u : 0u));  // inf / NaN
    } else if (ex == 0) {
        h = sign;  // double zero / subnormal: far below half's range
    } else {
        int e = ex - 1023 + 15;                               // half's biased exponent
        const unsigned long long m = (1ull << 52) | mant;     // 53-bit significand
        const int shift = (e >= 1) ? 42 : 42 + (1 - e);       // bits dropped (subnormal results: more)
        if (shift >= 64) {
            h = sign;
        } else {
            unsigned long long q = m >> shift;
            const unsigned long long rem = m & ((1ull << shift) - 1ull), half = 1ull << (shift - 1);
            if (rem > half || (rem == half && (q & 1ull))) ++q;
            if (e >= 1) {
                if (q == (1ull << 11)) {  // the rounding carried into the next binade
                    q >>= 1;
                    ++e;
                }
                h = (e >= 31) ? (unsigned short)(sign | 0x7c00u) : (unsigned short)(sign | (e << 10) | (q & 0x3ffu));
            } else {
                h = (unsigned short)(sign | q);  // subnormal (q == 0x400: the smallest normal)
            }
        }
    }
    return __half2float(__ushort_as_half(h));
}

// a float64 result stored into an array of the logits' dtype
template <bool F16>
__device__ __forceinline__ float store_d(double v) {
    if constexpr (F16) return round_d2h(v);
    return (float)v;
}

// Root preprocessing of mcts_sampled.py:64-100 for root blockIdx.x (prepare's policy, beta and noise
// arguments, :102-106), with numpy 2.x's dtype rules (NEP 50):
//   probs = softmax(logits) in the logits' dtype                                       :64-65
//   legal (integer array): probs *= legal; probs += legal * 1e-4 (float64 arithmetic, stored in the
//     logits' dtype); probs /= sum(probs); noises (float32) likewise                     :73-83
//   beta = probs * (1 - eps) [logits' dtype] + noises * eps [float32] -> float32          :93
//   beta **= 1 / tau; beta *= legal (float64, stored float32); beta /= sum(beta)          :94-100
// `legal` holds the agent's row as int32 (the caller checked the integer array's values fit), or is
// null.  The Dirichlet noise is drawn by the caller (np_random order) and arrives as float32.
template <bool F16>
__global__ __launch_bounds__(kWave) void k_root_glue(const void *logits, long long row_stride, long long col_off,
                                                     int A, const int *legal, long long legal_stride,
                                                     const float *noise_in, double one_minus_eps, double eps,
                                                     int use_pow, float tau_inv, float *probs, float *beta,
                                                     float *noise_out, const unsigned short *hexp) {
    __shared__ float lds[kWave];
    __shared__ float acc[9];
    const int t = blockIdx.x;
    const int l = threadIdx.x;
    const bool on = l < A;
    const float x = on ? load_elem<F16>(logits, (long long)t * row_stride + col_off + l) : -INFINITY;
    const bool nan_any = __ballot(on && (x != x)) != 0;
    const float m = nan_any ? NAN : wave_max(on ? x : -INFINITY);
    const float d = round_as<F16>(x - m);
    const float e = np_exp_as<F16>(d, hexp);
    const float s = round_as<F16>(np_row_sum(e, l, A, lds, acc));
    float p = round_as<F16>(e / s);
    float n = on ? noise_in[(long long)t * A + l] : 0.f;
    double lg = 0.0;
    if (legal) {
        lg = on ? (double)legal[(long long)t * legal_stride + l] : 0.0;
        const double tiny = lg * 1e-4;  // `legal * 1e-4`: a float64 array
        p = store_d<F16>((double)p * lg);
        p = store_d<F16>((double)p + tiny);
        const float sp = round_as<F16>(np_row_sum(p, l, A, lds, acc));
        p = round_as<F16>(p / sp);
        n = (float)((double)n * lg);
        n = (float)((double)n + tiny);
        const float sn = np_row_sum(n, l, A, lds, acc);
        n = n / sn;
    }
    // probs * (1 - eps): the Python float becomes the array's dtype (NEP 50); noises * eps in float32;
    // the sum of a half and a float32 array is float32
    const float c1 = store_d<F16>(one_minus_eps), c2 = (float)eps;
    const float a1 = round_as<F16>(p * c1);
    float b = a1 + n * c2;
    if (use_pow) b = np_pow_as<false>(b, tau_inv, use_pow);  // a float32 array
    if (legal) b = (float)((double)b * lg);
    const float sb = np_row_sum(b, l, A, lds, acc);
    b = b / sb;
    if (on) {
        probs[(long long)t * A + l] = p;
        beta[(long long)t * A + l] = b;
        noise_out[(long long)t * A + l] = n;
    }
}

// mcts_sampled.py:116-147 for root blockIdx.x: previous agents from `factor`, the current agent
// from the selection, the following agents by numpy argmax of the leaf policy logits.
template <bool F16>
__global__ __launch_bounds__(kWave) void k_joint_action(const void *pred, int N, int A, int cur, const int *factor,
                                                        int fcols, const int *actions, long long *joint) {
    const int t = blockIdx.x;
    const int l = threadIdx.x;
    if (l < N && l <= cur) joint[(long long)t * N + l] = (l < cur) ? (long long)factor[(long long)t * fcols + l]
                                                                    : (long long)actions[t];
    for (int k = cur + 1; k < N; ++k) {
        const bool on = l < A;
        const float v = on ? load_elem<F16>(pred, ((long long)t * N + k) * A + l) : -INFINITY;
        const unsigned long long nan_mask = __ballot(on && (v != v));
        int idx;
        if (nan_mask) {
            idx = __ffsll((long long)nan_mask) - 1;
        } else {
            const float m = wave_max(v);
            idx = __ffsll((long long)__ballot(on && v == m)) - 1;
        }
        if (l == 0) joint[(long long)t * N + k] = idx;
    }
}

// the table of mz_set_half_exp_table per device (allocated once, never freed: captured graphs keep
// its address)
constexpr int kMaxDevices = 64;
unsigned short *g_half_exp[kMaxDevices];
std::mutex g_half_exp_mu;

// the current device's table (the launchers call this after making the handle's device current)
const unsigned short *half_exp_table() {
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return nullptr;
    std::lock_guard<std::mutex> lk(g_half_exp_mu);
    return g_half_exp[dev];
}

}  // namespace

extern "C" {

int mz_set_half_exp_table(const uint16_t *table) {
    if (!table) return mz_internal_fail(MZ_ERR_ARG, "mz_set_half_exp_table: null table");
    int dev = -1;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return mz_internal_fail(MZ_ERR_DEVICE, hipGetErrorString(e));
    if (dev < 0 || dev >= kMaxDevices) return mz_internal_fail(MZ_ERR_UNSUPPORTED, "mz_set_half_exp_table: device id");
    std::lock_guard<std::mutex> lk(g_half_exp_mu);
    if (!g_half_exp[dev]) {
        void *p = nullptr;
        e = hipMalloc(&p, 65536 * sizeof(uint16_t));
        if (e != hipSuccess) return mz_internal_fail(MZ_ERR_DEVICE, hipGetErrorString(e));
        g_half_exp[dev] = (unsigned short *)p;
    }
    e = hipMemcpy(g_half_exp[dev], table, 65536 * sizeof(uint16_t), hipMemcpyHostToDevice);
    if (e != hipSuccess) return mz_internal_fail(MZ_ERR_DEVICE, hipGetErrorString(e));
    return MZ_OK;
}

int mz_policy_glue(mz_batch *b, const void *logits, int dtype, int64_t row_stride, int64_t col_offset,
                   double sampled_tau, float *probs_out, float *beta_out) {
    int B = 0, A = 0;
    hipStream_t stream = nullptr;
    int rc = mz_internal_launch_info(b, &B, &A, &stream);
    if (rc) return rc;
    if (A > kWave)  // (one lane per action; the tree itself takes up to 255 actions)
        return mz_internal_fail(MZ_ERR_UNSUPPORTED, "mz_policy_glue: action_space_size > 64");
    if (!logits || !probs_out || !beta_out) return mz_internal_fail(MZ_ERR_ARG, "mz_policy_glue: null buffer");
    if (dtype != MZ_DT_F32 && dtype != MZ_DT_F16) return mz_internal_fail(MZ_ERR_ARG, "mz_policy_glue: bad dtype");
    if (row_stride < A || col_offset < 0 || col_offset + A > row_stride)
        return mz_internal_fail(MZ_ERR_ARG, "mz_policy_glue: logits row does not hold the agent's actions");
    if (!(sampled_tau > 0.0)) return mz_internal_fail(MZ_ERR_ARG, "mz_policy_glue: sampled_tau must be > 0");
    const double inv = 1.0 / sampled_tau;  // Python's `1 / sampled_tau`, cast to the array's dtype
    const float tau_inv = (dtype == MZ_DT_F16) ? (float)(_Float16)inv : (float)inv;
    const int use_pow = pow_mode(inv);
    if (dtype == MZ_DT_F16)
        hipLaunchKernelGGL(k_policy_glue<true>, dim3(B), dim3(kWave), 0, stream, logits, (long long)row_stride,
                           (long long)col_offset, A, use_pow, tau_inv, probs_out, beta_out, half_exp_table());
    else
        hipLaunchKernelGGL(k_policy_glue<false>, dim3(B), dim3(kWave), 0, stream, logits, (long long)row_stride,
                           (long long)col_offset, A, use_pow, tau_inv, probs_out, beta_out, half_exp_table());
    mz_internal_enqueued(b);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return mz_internal_fail(MZ_ERR_DEVICE, hipGetErrorString(e));
    return MZ_OK;
}

int mz_root_glue(mz_batch *b, const void *logits, int dtype, int64_t row_stride, int64_t col_offset,
                 const int32_t *legal, int64_t legal_stride, const float *noises, double noise_eps,
                 double sampled_tau, float *probs_out, float *beta_out, float *noises_out) {
    int B = 0, A = 0;
    hipStream_t stream = nullptr;
    int rc = mz_internal_launch_info(b, &B, &A, &stream);
    if (rc) return rc;
    if (A > kWave)  // (one lane per action; the tree itself takes up to 255 actions)
        return mz_internal_fail(MZ_ERR_UNSUPPORTED, "mz_root_glue: action_space_size > 64");
    if (!logits || !noises || !probs_out || !beta_out || !noises_out)
        return mz_internal_fail(MZ_ERR_ARG, "mz_root_glue: null buffer");
    if (dtype != MZ_DT_F32 && dtype != MZ_DT_F16) return mz_internal_fail(MZ_ERR_ARG, "mz_root_glue: bad dtype");
    if (row_stride < A || col_offset < 0 || col_offset + A > row_stride)
        return mz_internal_fail(MZ_ERR_ARG, "mz_root_glue: logits row does not hold the agent's actions");
    if (legal && legal_stride < A) return mz_internal_fail(MZ_ERR_ARG, "mz_root_glue: legal rows hold fewer than A");
    if (!(sampled_tau > 0.0)) return mz_internal_fail(MZ_ERR_ARG, "mz_root_glue: sampled_tau must be > 0");
    const double inv = 1.0 / sampled_tau;  // beta is a float32 array here (:93)
    const float tau_inv = (float)inv;
    const int use_pow = pow_mode(inv);
    const double ome = 1.0 - noise_eps;  // (Python float arithmetic)
    if (dtype == MZ_DT_F16)
        hipLaunchKernelGGL(k_root_glue<true>, dim3(B), dim3(kWave), 0, stream, logits, (long long)row_stride,
                           (long long)col_offset, A, (const int *)legal, (long long)legal_stride, noises, ome,
                           noise_eps, use_pow, tau_inv, probs_out, beta_out, noises_out, half_exp_table());
    else
        hipLaunchKernelGGL(k_root_glue<false>, dim3(B), dim3(kWave), 0, stream, logits, (long long)row_stride,
                           (long long)col_offset, A, (const int *)legal, (long long)legal_stride, noises, ome,
                           noise_eps, use_pow, tau_inv, probs_out, beta_out, noises_out, half_exp_table());
    mz_internal_enqueued(b);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return mz_internal_fail(MZ_ERR_DEVICE, hipGetErrorString(e));
    return MZ_OK;
}

int mz_joint_action(mz_batch *b, const void *pred_logits, int dtype, int num_agents, int current_agent,
                    const int32_t *factor, int factor_cols, const int32_t *actions, int64_t *joint_out) {
    int B = 0, A = 0;
    hipStream_t stream = nullptr;
    int rc = mz_internal_launch_info(b, &B, &A, &stream);
    if (rc) return rc;
    if (A > kWave)  // (one lane per action; the tree itself takes up to 255 actions)
        return mz_internal_fail(MZ_ERR_UNSUPPORTED, "mz_joint_action: action_space_size > 64");
    if (num_agents < 1 || num_agents > kWave || current_agent < 0 || current_agent >= num_agents)
        return mz_internal_fail(MZ_ERR_ARG, "mz_joint_action: bad agent index / count");
    if (!actions || !joint_out) return mz_internal_fail(MZ_ERR_ARG, "mz_joint_action: null buffer");
    if (current_agent > 0 && (!factor || factor_cols < current_agent))
        return mz_internal_fail(MZ_ERR_ARG, "mz_joint_action: factor must hold the previous agents' actions");
    if (current_agent + 1 < num_agents && !pred_logits)
        return mz_internal_fail(MZ_ERR_ARG, "mz_joint_action: leaf policy logits required for later agents");
    if (dtype != MZ_DT_F32 && dtype != MZ_DT_F16) return mz_internal_fail(MZ_ERR_ARG, "mz_joint_action: bad dtype");
    if (dtype == MZ_DT_F16)
        hipLaunchKernelGGL(k_joint_action<true>, dim3(B), dim3(kWave), 0, stream, pred_logits, num_agents, A,
                           current_agent, (const int *)factor, factor_cols, (const int *)actions,
                           (long long *)joint_out);
    else
        hipLaunchKernelGGL(k_joint_action<false>, dim3(B), dim3(kWave), 0, stream, pred_logits, num_agents, A,
                           current_agent, (const int *)factor, factor_cols, (const int *)actions,
                           (long long *)joint_out);
    mz_internal_enqueued(b);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return mz_internal_fail(MZ_ERR_DEVICE, hipGetErrorString(e));
    return MZ_OK;
}

// nodes and memset nodes of a graph, child graphs (hipGraphNodeTypeGraph: a nested capture, an
// embedded graph) included
static hipError_t census(hipGraph_t g, int depth, int *total, int *memsets) {
    if (depth > 16) return hipErrorInvalidValue;
    size_t n = 0;
    hipError_t e = hipGraphGetNodes(g, nullptr, &n);
    if (e != hipSuccess) return e;
    hipGraphNode_t *nodes = (hipGraphNode_t *)malloc(sizeof(hipGraphNode_t) * (n ? n : 1));
    if (!nodes) return hipErrorOutOfMemory;
    e = hipGraphGetNodes(g, nodes, &n);
    *total += (int)n;
    for (size_t k = 0; e == hipSuccess && k < n; ++k) {
        hipGraphNodeType ty;
        e = hipGraphNodeGetType(nodes[k], &ty);
        if (e != hipSuccess) break;
        if (ty == hipGraphNodeTypeMemset) {
            ++*memsets;
        } else if (ty == hipGraphNodeTypeGraph) {
            hipGraph_t child = nullptr;
            e = hipGraphChildGraphNodeGetGraph(nodes[k], &child);
            if (e == hipSuccess) e = census(child, depth + 1, total, memsets);
        }
    }
    free(nodes);
    return e;
}

int mz_graph_census(void *graph, int *total_nodes, int *memset_nodes) {
    if (!graph || !total_nodes || !memset_nodes) return mz_internal_fail(MZ_ERR_ARG, "mz_graph_census: null argument");
    int total = 0, ms = 0;
    hipError_t e = census((hipGraph_t)graph, 0, &total, &ms);
    if (e != hipSuccess) return mz_internal_fail(MZ_ERR_DEVICE, hipGetErrorString(e));
    *total_nodes = total;
    *memset_nodes = ms;
    return MZ_OK;
}

}  // extern "C"
