/*
 * mzconsume.h — C-ABI of the on-device consumers of the search output.
 *
 * After each agent's search the reference workers pull every root's result to the host and make
 * their decisions per root in Python:
 *   - self-play: select_action over the root children's visit counts (core/utils.py:289-316),
 *     then eps_greedy_action (core/utils.py:319-334), then the stored policy probability and the
 *     visit entropy from the marginal visit counts (core/selfplay_worker.py:228-293);
 *   - reanalyze: the action argmax(marginal visits * legal mask) and the product of the agents'
 *     marginal visit distributions at the chosen actions (core/reanalyze_worker.py:296-332).
 * These entry points make the same decisions on the device, one lane per root, reading the padded
 * device results of mz_get_roots_sampled_padded / mz_get_roots_marginal_visit_count, in the
 * stream of a tree handle (mzmcts.h).  Random draws are inputs: the caller draws them on the host
 * from the same generator, in the same order as the reference (see each function).
 *
 * Integer and index results are exact; the float64 probabilities are the reference's own
 * operation sequence (Python sum, numpy cumsum, IEEE division), so they are bit-identical too.
 * The entropies use the device log and are within 1e-12 (relative) of scipy / numpy.
 *
 * Exported only by the product library (mazero_amd/_build/libmzmcts.so); device memory only.
 */
#ifndef MZCONSUME_H
#define MZCONSUME_H

#include <stdint.h>

#include "mzmcts.h"

#ifdef __cplusplus
extern "C" {
#endif

/* select_action(sampled_visit_count[i], temperature, deterministic, np_random)
 * (core/utils.py:289-316) for every root i, as the self-play worker calls it
 * (core/selfplay_worker.py:240-247), then agent_action = sampled_actions[pos, 0].
 *   degrees   int32 [B]              children of each root (mz_get_roots_sampled_padded)
 *   visits    int32 [B, width]       per-child visit counts, row i valid up to degrees[i]
 *   actions   int32 [B, width * N]   per-child joint actions (N = agent_num of the handle)
 *   uniforms  float64 [B]            np_random.random(B): the double each root's
 *                                    np_random.choice(len, p=probs) draws, in root order
 *                                    (ignored when deterministic)
 *   pos_out   int32 [B]   chosen child; action_out int32 [B] its action for agent 0;
 *   entropy_out float64 [B] scipy.stats.entropy(action_probs, base=2) (may be NULL).
 * probs = v ** (1 / temperature) / sum(...): exact repeated products when 1/temperature is an
 * integer up to 8 (the reference's schedule uses 1, 2, 4; config.py:392-401), else the device pow.
 * A root without children or without visits gets -1 (the reference asserts / draws from the
 * legal actions instead; neither happens after num_simulations >= 1). */
int mz_select_actions(mz_batch *b, const int32_t *degrees, const int32_t *visits, const int32_t *actions,
                      int width, double temperature, int deterministic, const double *uniforms, int32_t *pos_out,
                      int32_t *action_out, double *entropy_out);

/* eps_greedy_action(greedy, legal_mask, eps) (core/utils.py:319-334) for every root:
 *   action_io = (u_eps[i] < (float)eps) ? categorical(legal[i, :]; u_cat[i]) : action_io[i]
 * legal: int32 [B, A] (row stride legal_stride elements), the agent's legal-action weights;
 * categorical(w; u) = the first a with cumsum(w)[a] / sum(w) > u (float64), i.e. a draw from
 * torch.distributions.Categorical(w).  u_eps float32 [B], u_cat float64 [B] in [0, 1): the
 * reference draws them from torch's global generator per root; the caller supplies them (the same
 * distribution, not the same stream).  A root with no legal action keeps its greedy action. */
int mz_eps_greedy(mz_batch *b, const int32_t *legal, int64_t legal_stride, float eps, const float *u_eps,
                  const double *u_cat, int32_t *action_io);

enum mz_marginal_mode {
    MZ_MARGINAL_GIVEN = 0,  /* self-play record: action given (core/selfplay_worker.py:278-290) */
    MZ_MARGINAL_ARGMAX = 1, /* reanalyze: action = argmax(marginal * legal) (reanalyze_worker.py:303-319) */
};

/* One agent's marginal visit distribution dist = marginal / sum(marginal) (float64) at each root:
 *   MZ_MARGINAL_ARGMAX: action_io[i] = first argmax_a marginal[i, a] * legal[i, a] (int64 products);
 *   prob_io[i] *= dist[action_io[i]]  (the running product over agents; start it at 1.0);
 *   entropy_out[i] = -sum_a dist[a] * log(dist[a] + 1e-9)  (may be NULL).
 * When sum(marginal) == 0 (only with num_simulations == 0): GIVEN multiplies by 1/A and reports
 * entropy 0 (as the self-play worker); ARGMAX writes action -1 and leaves prob_io and entropy_out
 * unchanged -- the reference draws that root's action from np_random -- for the caller to resolve.
 * marginal: int32 [B, A] (row stride marginal_stride); legal: int32 [B, A] (row stride
 * legal_stride), required for ARGMAX, ignored by GIVEN. */
int mz_marginal_policy(mz_batch *b, const int32_t *marginal, int64_t marginal_stride, const int32_t *legal,
                       int64_t legal_stride, int mode, int32_t *action_io, double *prob_io, double *entropy_out);

#ifdef __cplusplus
}
#endif

#endif /* MZCONSUME_H */
