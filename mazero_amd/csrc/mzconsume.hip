// mzconsume.hip — on-device consumers of the search output (include/mzconsume.h).
//
// The reference workers make their per-root decisions in Python after each search:
//   select_action + eps_greedy_action (core/utils.py:289-334, called at selfplay_worker.py:228-252),
//   the stored policy probability and visit entropy (selfplay_worker.py:278-293),
//   the reanalyze action and policy product (reanalyze_worker.py:296-332).
// Here one lane handles one root and walks its row sequentially, in the reference's own order of
// floating-point operations (Python's left-to-right sum, numpy's sequential cumsum, IEEE
// division), so every probability and index is bit-identical.  The work is a few hundred bytes per
// root, far below any bandwidth bound: these kernels exist to keep the search output on the device
// (no device-to-host copy of the per-root lists between the search and the environment step).
#include <hip/hip_runtime.h>

#include <math.h>

#include "../../include/mzconsume.h"
#include "mz_internal.h"

namespace {

constexpr int kLanes = 64;

// v ** e for a visit count v (core/utils.py:302): numpy evaluates it as the double power of
// float64(v).  For an integer exponent the repeated product is exact, hence equal to libm pow,
// whenever v**e < 2**53 (visit counts up to 9000 with e <= 4).
__device__ __forceinline__ double visit_pow(int v, int ipow, double e) {
    const double x = (double)v;
    if (ipow <= 0) return pow(x, e);
    double r = x;
    for (int k = 1; k < ipow; ++k) r *= x;
    return r;
}

__global__ __launch_bounds__(kLanes) void k_select_actions(int B, int N, const int *__restrict__ deg,
                                                           const int *__restrict__ visits,
                                                           const int *__restrict__ actions, int width, int ipow,
                                                           double e, int deterministic,
                                                           const double *__restrict__ uniforms, int *pos_out,
                                                           int *act_out, double *ent_out) {
    const int i = blockIdx.x * kLanes + threadIdx.x;
    if (i >= B) return;
    const int n = deg[i];
    const int *row = visits + (long long)i * width;
    long long vsum = 0;
    for (int j = 0; j < n; ++j) vsum += row[j];
    if (n <= 0 || n > width || vsum <= 0) {  // assert sum(visit_counts) > 0 (core/utils.py:301)
        pos_out[i] = -1;
        act_out[i] = -1;
        if (ent_out) ent_out[i] = NAN;
        return;
    }
    // total_count = sum(action_probs): Python's sum, left to right from 0 (utils.py:304)
    double total = 0.0;
    for (int j = 0; j < n; ++j) total += visit_pow(row[j], ipow, e);
    int pos = 0;
    if (deterministic) {
        for (int j = 1; j < n; ++j)
            if (row[j] > row[pos]) pos = j;  // np.argmax: first maximum
    } else {
        // np_random.choice(n, p=probs): cdf = probs.cumsum(); cdf /= cdf[-1];
        // cdf.searchsorted(u, side='right')
        double last = 0.0;
        for (int j = 0; j < n; ++j) last += visit_pow(row[j], ipow, e) / total;
        const double u = uniforms[i];
        double c = 0.0;
        pos = n - 1;
        for (int j = 0; j < n; ++j) {
            c += visit_pow(row[j], ipow, e) / total;
            if (c / last > u) {
                pos = j;
                break;
            }
        }
    }
    pos_out[i] = pos;
    act_out[i] = actions[(long long)i * width * N + (long long)pos * N];  // sampled_actions[pos, 0]
    if (ent_out) {
        // scipy.stats.entropy(action_probs, base=2): pk / sum(pk), sum of -pk log pk, / log(2)
        double ps = 0.0;
        for (int j = 0; j < n; ++j) ps += visit_pow(row[j], ipow, e) / total;
        double h = 0.0;
        for (int j = 0; j < n; ++j) {
            const double pk = (visit_pow(row[j], ipow, e) / total) / ps;
            if (pk > 0.0) h -= pk * log(pk);
        }
        ent_out[i] = h / log(2.0);
    }
}

__global__ __launch_bounds__(kLanes) void k_eps_greedy(int B, int A, const int *__restrict__ legal, long long stride,
                                                       float eps, const float *__restrict__ u_eps,
                                                       const double *__restrict__ u_cat, int *action_io) {
    const int i = blockIdx.x * kLanes + threadIdx.x;
    if (i >= B) return;
    if (!(u_eps[i] < eps)) return;  // pick_random = (rand < eps) in float32 (utils.py:327-328)
    const int *w = legal + (long long)i * stride;
    long long tot = 0;
    for (int a = 0; a < A; ++a) tot += w[a];
    if (tot <= 0) return;
    // Categorical(legal_action_mask).sample() (utils.py:329): inverse cdf of the mask weights
    const double u = u_cat[i];
    long long c = 0;
    for (int a = 0; a < A; ++a) {
        c += w[a];
        if ((double)c / (double)tot > u) {
            action_io[i] = a;
            return;
        }
    }
}

__global__ __launch_bounds__(kLanes) void k_marginal_policy(int B, int A, const int *__restrict__ marginal,
                                                            long long mstride, const int *__restrict__ legal,
                                                            long long lstride, int mode, int *action_io,
                                                            double *prob_io, double *ent_out) {
    const int i = blockIdx.x * kLanes + threadIdx.x;
    if (i >= B) return;
    const int *m = marginal + (long long)i * mstride;
    long long msum = 0;
    for (int a = 0; a < A; ++a) msum += m[a];
    if (mode == MZ_MARGINAL_ARGMAX) {
        if (msum <= 0) {  // the reference draws np_random.choice(legal_indices) (reanalyze_worker.py:313-315)
            action_io[i] = -1;
            return;
        }
        // np.argmax(marginal_visits * legal_actions): first maximum of the int64 products
        const int *l = legal + (long long)i * lstride;
        int best = 0;
        long long bv = (long long)m[0] * l[0];
        for (int a = 1; a < A; ++a) {
            const long long v = (long long)m[a] * l[a];
            if (v > bv) bv = v, best = a;
        }
        action_io[i] = best;
    }
    const int act = action_io[i];
    if (msum <= 0) {  // selfplay_worker.py:287-288
        prob_io[i] *= 1.0 / (double)A;
        if (ent_out) ent_out[i] = 0.0;
        return;
    }
    const double s = (double)msum;
    // prob *= (marginal / np.sum(marginal))[action]  (selfplay_worker.py:284-286, reanalyze_worker.py:336-343)
    prob_io[i] *= (act >= 0 && act < A) ? (double)m[act] / s : NAN;
    if (ent_out) {
        double h = 0.0;  // -np.sum(p * np.log(p + 1e-9))  (selfplay_worker.py:286)
        for (int a = 0; a < A; ++a) {
            const double p = (double)m[a] / s;
            h += p * log(p + 1e-9);
        }
        ent_out[i] = -h;
    }
}

int launch_status() {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return mz_internal_fail(MZ_ERR_DEVICE, hipGetErrorString(e));
    return MZ_OK;
}

}  // namespace

extern "C" {

int mz_select_actions(mz_batch *b, const int32_t *degrees, const int32_t *visits, const int32_t *actions, int width,
                      double temperature, int deterministic, const double *uniforms, int32_t *pos_out,
                      int32_t *action_out, double *entropy_out) {
    int B = 0, A = 0;
    hipStream_t stream = nullptr;
    int rc = mz_internal_launch_info(b, &B, &A, &stream);
    if (rc) return rc;
    if (!degrees || !visits || !actions || !pos_out || !action_out || (!deterministic && !uniforms))
        return mz_internal_fail(MZ_ERR_ARG, "mz_select_actions: null buffer");
    if (width < 1) return mz_internal_fail(MZ_ERR_ARG, "mz_select_actions: width must be >= 1");
    if (!(temperature > 0.0)) return mz_internal_fail(MZ_ERR_ARG, "mz_select_actions: temperature must be > 0");
    const double e = 1.0 / temperature;  // 1 / temperature, as Python computes it
    const int ipow = (e == floor(e) && e >= 1.0 && e <= 8.0) ? (int)e : 0;
    hipLaunchKernelGGL(k_select_actions, dim3((B + kLanes - 1) / kLanes), dim3(kLanes), 0, stream, B,
                       mz_internal_agent_num(b), (const int *)degrees, (const int *)visits, (const int *)actions,
                       width, ipow, e, deterministic, uniforms, (int *)pos_out, (int *)action_out, entropy_out);
    mz_internal_enqueued(b);
    return launch_status();
}

int mz_eps_greedy(mz_batch *b, const int32_t *legal, int64_t legal_stride, float eps, const float *u_eps,
                  const double *u_cat, int32_t *action_io) {
    int B = 0, A = 0;
    hipStream_t stream = nullptr;
    int rc = mz_internal_launch_info(b, &B, &A, &stream);
    if (rc) return rc;
    if (!legal || !u_eps || !u_cat || !action_io) return mz_internal_fail(MZ_ERR_ARG, "mz_eps_greedy: null buffer");
    if (legal_stride < A) return mz_internal_fail(MZ_ERR_ARG, "mz_eps_greedy: legal rows hold fewer than A entries");
    hipLaunchKernelGGL(k_eps_greedy, dim3((B + kLanes - 1) / kLanes), dim3(kLanes), 0, stream, B, A,
                       (const int *)legal, (long long)legal_stride, eps, u_eps, u_cat, (int *)action_io);
    mz_internal_enqueued(b);
    return launch_status();
}

int mz_marginal_policy(mz_batch *b, const int32_t *marginal, int64_t marginal_stride, const int32_t *legal,
                       int64_t legal_stride, int mode, int32_t *action_io, double *prob_io, double *entropy_out) {
    int B = 0, A = 0;
    hipStream_t stream = nullptr;
    int rc = mz_internal_launch_info(b, &B, &A, &stream);
    if (rc) return rc;
    if (mode != MZ_MARGINAL_GIVEN && mode != MZ_MARGINAL_ARGMAX)
        return mz_internal_fail(MZ_ERR_ARG, "mz_marginal_policy: bad mode");
    if (!marginal || !action_io || !prob_io || (mode == MZ_MARGINAL_ARGMAX && !legal))
        return mz_internal_fail(MZ_ERR_ARG, "mz_marginal_policy: null buffer");
    if (marginal_stride < A || (mode == MZ_MARGINAL_ARGMAX && legal_stride < A))
        return mz_internal_fail(MZ_ERR_ARG, "mz_marginal_policy: rows hold fewer than A entries");
    hipLaunchKernelGGL(k_marginal_policy, dim3((B + kLanes - 1) / kLanes), dim3(kLanes), 0, stream, B, A,
                       (const int *)marginal, (long long)marginal_stride, (const int *)legal, (long long)legal_stride,
                       mode, (int *)action_io, prob_io, entropy_out);
    mz_internal_enqueued(b);
    return launch_status();
}

}  // extern "C"
