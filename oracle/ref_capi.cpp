// ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called from the product.
//
// C-ABI wrapper (include/mzmcts.h) around the *reference* tree, tree::CTree_batch, compiled from
// the reference sources where they lie under /root/reference (see oracle/Makefile; nothing of the
// reference is copied into this repository).  Output: oracle/_ref/libmzref.so.
//
// Used (a) by oracle/gen_golden.py to record the golden vectors in tests/golden/, and (b) by
// bench.py's cpu_baseline leg as the "reference CPU ctree" timed on the host cores.
// Host memory only; exceptions from the reference's my_assert (common_lib/utils.cpp:8-18) are
// caught and reported through mz_last_error(), the way Cython's `except +` turns them into
// RuntimeError (ctree_sampled/ctree.pxd:14-20).
// The reference's Cython build compiles the tree as ONE translation unit: ctree.pxd pulls in
// "../common_lib/utils.cpp" and "lib/cnode.cpp" with `cdef extern from` (ctree.pxd:4-8), which is
// what instantiates the Array2D/Array3D templates defined in utils.cpp.  Do the same here, with
// the sources included in place from the reference tree (-I$(REF_TREE)/ctree_sampled).
#include "lib/cnode.cpp"
#include "../common_lib/utils.cpp"

#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../include/mzmcts.h"

struct mz_batch {
    tree::CTree_batch *t;
    int B, N, A, K;
};

static thread_local std::string g_err;

static int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define GUARD_HOST(mem)                                                                  \
    if ((mem) != MZ_MEM_HOST) return fail(MZ_ERR_UNSUPPORTED, "reference oracle: host memory only")

extern "C" {

const char *mz_last_error(void) { return g_err.c_str(); }
int mz_abi_version(void) { return MZ_ABI_VERSION; }
const char *mz_backend(void) { return "reference-ctree"; }

int mz_create(int root_num, int agent_num, int action_space_size, int sampled_times,
              int simulation_num, float delta_lb, uint32_t random_seed, float rho, float lam,
              int root_offset, mz_batch **out) {
    if (!out) return fail(MZ_ERR_ARG, "null output handle");
    if (root_offset != 0) return fail(MZ_ERR_UNSUPPORTED, "reference oracle: root_offset must be 0");
    try {
        auto *b = new mz_batch;
        b->t = new tree::CTree_batch(root_num, agent_num, action_space_size, sampled_times,
                                     simulation_num, delta_lb, random_seed, rho, lam);
        b->B = root_num;
        b->N = agent_num;
        b->A = action_space_size;
        b->K = sampled_times;
        *out = b;
        return MZ_OK;
    } catch (const std::exception &e) {
        return fail(MZ_ERR_RUNTIME, e.what());
    }
}

int mz_destroy(mz_batch *b) {
    if (b) {
        delete b->t;
        delete b;
    }
    return MZ_OK;
}

int mz_set_stream(mz_batch *, void *) { return MZ_OK; }
int mz_synchronize(mz_batch *) { return MZ_OK; }

int mz_prepare(mz_batch *b, const float *rewards, const float *values, const float *policy,
               const float *beta, int sampled_times, float noise_eps, const float *noises, int mem) {
    GUARD_HOST(mem);
    try {
        b->t->prepare(const_cast<float *>(rewards), const_cast<float *>(values),
                      const_cast<float *>(policy), const_cast<float *>(beta), sampled_times,
                      noise_eps, const_cast<float *>(noises));
        return MZ_OK;
    } catch (const std::exception &e) {
        return fail(MZ_ERR_RUNTIME, e.what());
    }
}

int mz_select(mz_batch *b, float c2, float c1, float discount, int32_t *idx_x, int32_t *idy,
              int32_t *actions, int mem) {
    GUARD_HOST(mem);
    try {
        b->t->cbatch_selection(c2, c1, discount, idx_x, idy, actions);
        return MZ_OK;
    } catch (const std::exception &e) {
        return fail(MZ_ERR_RUNTIME, e.what());
    }
}

int mz_expand_backup(mz_batch *b, int hsx, float discount, int sampled_times, const float *rewards,
                     const float *values, const float *policy, const float *beta, int mem) {
    GUARD_HOST(mem);
    try {
        b->t->cbatch_expansion_and_backup(hsx, discount, sampled_times, const_cast<float *>(rewards),
                                          const_cast<float *>(values), const_cast<float *>(policy),
                                          const_cast<float *>(beta));
        return MZ_OK;
    } catch (const std::exception &e) {
        return fail(MZ_ERR_RUNTIME, e.what());
    }
}

int mz_expand_backup_select(mz_batch *, int, float, int, const float *, const float *, const float *,
                            const float *, float, float, int32_t *, int32_t *, int32_t *,
                            const void *, int64_t, int64_t, void *) {
    return fail(MZ_ERR_UNSUPPORTED, "reference oracle: fused device path not available");
}

int mz_prepare_select(mz_batch *, const float *, const float *, const float *, const float *, int, float,
                      const float *, float, float, float, int32_t *, int32_t *, int32_t *) {
    return fail(MZ_ERR_UNSUPPORTED, "reference oracle: fused device path not available");
}
int mz_get_roots_device(mz_batch *, float, const mz_readback_out *) {
    return fail(MZ_ERR_UNSUPPORTED, "reference oracle: device readbacks not available");
}
int mz_gather_rows(mz_batch *, const void *, int64_t, int64_t, const int32_t *, void *) {
    return fail(MZ_ERR_UNSUPPORTED, "reference oracle: device gather not available");
}

int mz_get_roots_values(mz_batch *b, float *out, int mem) {
    GUARD_HOST(mem);
    b->t->get_roots_values(out);
    return MZ_OK;
}

int mz_get_roots_marginal_visit_count(mz_batch *b, int32_t *out, int mem) {
    GUARD_HOST(mem);
    b->t->get_roots_marginal_visit_count(out);
    return MZ_OK;
}

int mz_get_roots_marginal_priors(mz_batch *b, float *out, int mem) {
    GUARD_HOST(mem);
    b->t->get_roots_marginal_priors(out);
    return MZ_OK;
}

int mz_get_num_children_of_root(mz_batch *b, int tree_id, int32_t *out) {
    if (tree_id < 0 || tree_id >= b->B) return fail(MZ_ERR_ARG, "tree_id out of range");
    *out = b->t->get_num_children_of_root(tree_id);
    return MZ_OK;
}

static int sampled_one(mz_batch *b, int field, int i, float discount, void *out) {
    tree::CTree_batch *t = b->t;
    switch (field) {
    case MZ_F_ACTIONS: t->get_root_sampled_actions(i, (int *)out); break;
    case MZ_F_VISIT_COUNT: t->get_root_sampled_visit_count(i, (int *)out); break;
    case MZ_F_PRED_PROBS: t->get_root_sampled_pred_probs(i, (float *)out); break;
    case MZ_F_BETA: t->get_root_sampled_beta(i, (float *)out); break;
    case MZ_F_BETA_HAT: t->get_root_sampled_beta_hat(i, (float *)out); break;
    case MZ_F_PRIORS: t->get_root_sampled_priors(i, (float *)out); break;
    case MZ_F_IMP_RATIO: t->get_root_sampled_imp_ratio(i, (float *)out); break;
    case MZ_F_PRED_VALUES: t->get_root_sampled_pred_values(i, (float *)out); break;
    case MZ_F_MCTS_VALUES: t->get_root_sampled_mcts_values(i, (float *)out); break;
    case MZ_F_REWARDS: t->get_root_sampled_rewards(i, (float *)out); break;
    case MZ_F_QVALUES: t->get_root_sampled_qvalues(i, (float *)out, discount); break;
    default: return fail(MZ_ERR_ARG, "unknown field");
    }
    return MZ_OK;
}

int mz_get_root_sampled(mz_batch *b, int field, int tree_id, float discount, void *out) {
    if (tree_id < 0 || tree_id >= b->B) return fail(MZ_ERR_ARG, "tree_id out of range");
    try {
        return sampled_one(b, field, tree_id, discount, out);
    } catch (const std::exception &e) {
        return fail(MZ_ERR_RUNTIME, e.what());
    }
}

int mz_max_children(mz_batch *b, int32_t *out) {
    long long deg = 1;
    for (int i = 0; i < b->N; ++i) deg *= b->A;
    *out = (int32_t)(deg < b->K ? deg : b->K);
    return MZ_OK;
}

int mz_get_roots_sampled_padded(mz_batch *b, int field, float discount, void *out, int32_t *degrees,
                                int mem) {
    GUARD_HOST(mem);
    int32_t maxdeg;
    mz_max_children(b, &maxdeg);
    const int width = (field == MZ_F_ACTIONS) ? maxdeg * b->N : maxdeg;
    std::memset(out, 0, sizeof(float) * (size_t)b->B * width);
    std::vector<char> tmp(sizeof(float) * (size_t)width + 16);
    for (int i = 0; i < b->B; ++i) {
        int deg = b->t->get_num_children_of_root(i);
        if (degrees) degrees[i] = deg;
        if (deg == 0) continue;
        int rc = mz_get_root_sampled(b, field, i, discount, tmp.data());
        if (rc) return rc;
        const int n = (field == MZ_F_ACTIONS) ? deg * b->N : deg;
        std::memcpy((char *)out + sizeof(float) * (size_t)i * width, tmp.data(), sizeof(float) * n);
    }
    return MZ_OK;
}

int mz_get_stats(mz_batch *, int64_t *out) {
    for (int i = 0; i < MZ_S_COUNT; ++i) out[i] = 0;
    return MZ_OK;
}

int mz_print(mz_batch *b) {
    b->t->print();
    return MZ_OK;
}

}  // extern "C"
