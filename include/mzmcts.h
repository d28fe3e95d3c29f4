/*
 * mzmcts.h — C-ABI of the MI355X-native batched sampled-MCTS tree (MAZero hot path).
 *
 * One opaque handle = one batch of independent search trees, the drop-in replacement for
 * `tree::CTree_batch` (reference core/mcts/ctree/ctree_sampled/lib/cnode.h:107-141) as it is
 * driven through the Cython class `cytree.Tree_batch` (ctree_sampled/cytree.pyx:7-247).
 *
 * Three shared libraries export exactly this ABI:
 *   mazero_amd/_build/libmzmcts.so  the product: HIP/gfx950 kernels, tree state resident in HBM
 *   oracle/_ref/libmzref.so         test oracle: the reference C++ tree compiled from its sources
 *   oracle/_build/libmzport.so      test oracle: CPU restatement of the reference algorithm
 * The two oracle builds accept MZ_MEM_HOST buffers only.
 *
 * Conventions (mirroring cytree.pyx):
 *   - every float buffer is float32, C-contiguous, shaped as documented; shapes are not checked
 *     (the reference indexes raw pointers, common_lib/utils.h:58 "no bound check").
 *   - input buffers are borrowed for the duration of the call (stream-ordered for device
 *     pointers); outputs go to caller-provided buffers.
 *   - `mem` selects where caller buffers live: MZ_MEM_HOST (pageable host memory; the call is
 *     synchronous like the reference) or MZ_MEM_DEVICE (device pointers; the call is enqueued
 *     on the handle's stream and returns immediately).
 *   - every entry point returns MZ_OK (0) or an error code; mz_last_error() gives the message of
 *     the last failing call on the calling thread.  The reference raises RuntimeError from
 *     `my_assert` (common_lib/utils.cpp:8-18) in the ctor, prepare, cbatch_selection and
 *     cbatch_expansion_and_backup (ctree.pxd:14-20); the Python shim raises in the same places.
 *   - a handle is single-threaded: calls on one handle must not overlap (reference: the GIL).
 */
#ifndef MZMCTS_H
#define MZMCTS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2 (round 6): MZ_S_RNG_TIE_BEYOND / MZ_S_RNG_NXT_BEYOND inserted at 10 and 11, the stamp slots
 * moved up by two, MZ_S_COUNT 32 */
#define MZ_ABI_VERSION 2

typedef struct mz_batch mz_batch;

enum mz_status {
    MZ_OK = 0,
    MZ_ERR_ARG = 1,         /* bad argument (null handle, unsupported memory kind, bad field) */
    MZ_ERR_RUNTIME = 2,     /* search invariant violated (reference: std::runtime_error)       */
    MZ_ERR_DEVICE = 3,      /* HIP runtime error                                               */
    MZ_ERR_UNSUPPORTED = 4  /* configuration outside what this backend implements             */
};

enum mz_mem { MZ_MEM_HOST = 0, MZ_MEM_DEVICE = 1 };

/* Per-child fields of the root, in root-child order (cytree.pyx:111-241, cnode.cpp:69-171). */
enum mz_field {
    MZ_F_ACTIONS = 0,     /* int32 [deg, agent_num]  CTree::get_root_sampled_actions  cnode.cpp:483 */
    MZ_F_VISIT_COUNT = 1, /* int32 [deg]  CNode::get_sampled_visit_count  cnode.cpp:93   */
    MZ_F_PRED_PROBS = 2,  /* f32   [deg]  CNode::get_sampled_pred_probs   cnode.cpp:101  */
    MZ_F_BETA = 3,        /* f32   [deg]  CNode::get_sampled_beta         cnode.cpp:109  */
    MZ_F_BETA_HAT = 4,    /* f32   [deg]  CNode::get_sampled_beta_hat     cnode.cpp:117  */
    MZ_F_PRIORS = 5,      /* f32   [deg]  CNode::get_sampled_priors       cnode.cpp:125  */
    MZ_F_IMP_RATIO = 6,   /* f32   [deg]  CNode::get_sampled_imp_ratio    cnode.cpp:133  */
    MZ_F_PRED_VALUES = 7, /* f32   [deg]  CNode::get_sampled_pred_values  cnode.cpp:141  */
    MZ_F_MCTS_VALUES = 8, /* f32   [deg]  CNode::get_sampled_mcts_values  cnode.cpp:149  */
    MZ_F_REWARDS = 9,     /* f32   [deg]  CNode::get_sampled_rewards      cnode.cpp:157  */
    MZ_F_QVALUES = 10,    /* f32   [deg]  CNode::get_sampled_qvalues      cnode.cpp:165 (uses discount) */
    MZ_F_COUNT = 11
};

/* Counters the product kernels accumulate (for algorithmic-byte accounting in bench.py). */
enum mz_stat {
    MZ_S_SELECTS = 0,        /* tree-selections performed                                  */
    MZ_S_PATH_EDGES = 1,     /* sum of search_len over selections                          */
    MZ_S_SCORED = 2,         /* children whose pUCT score was evaluated                    */
    MZ_S_EXPANDS = 3,        /* leaf expansions (incl. root prepare)                       */
    MZ_S_NEW_CHILDREN = 4,   /* nodes created                                              */
    MZ_S_BACKUP_NODES = 5,   /* node updates in back-propagation                           */
    MZ_S_ENTRIES_READ = 6,   /* value-set entries scanned by back-propagation              */
    MZ_S_ENTRIES_WRITTEN = 7,/* value-set entries written by back-propagation              */
    MZ_S_MINMAX_NODES = 8,   /* node q-values scanned for the min/max normaliser           */
    MZ_S_MM_MOVED = 9,       /* back-propagations after which the min/max normaliser (its min
                              * or max, CMinMaxStats utils.cpp:79-103) differs from before:
                              * every internal node's select_child outcome may change then
                              * (counted by k_tree, k_step and k_hbm; 0 for the K = 1 chains)  */
    MZ_S_RNG_TIE_BEYOND = 10,/* tie draws (gen() % size, cnode.cpp:373-377) whose engine word
                              * lies past the launch's LDS window of the tree's stream, read
                              * from HBM by the selection's chase (k_tree only)              */
    MZ_S_RNG_NXT_BEYOND = 11,/* launches whose next expansion's engine words (the header's
                              * copy) lie past that window, read from HBM (k_tree only)      */
    /* Diagnostic builds only (compiled with MZ_STAMPS=1; zero otherwise): shader cycles of the
     * fused simulation-step kernel, summed over trees and launches, read with s_memtime where the
     * wave's instruction stream reaches each point (no forced waits).  Wave 0 (expansion,
     * selection, gather): */
    MZ_S_CYC_HEADER = 12,     /* round 1: header, tables, network outputs issued and waited   */
    MZ_S_CYC_STAGE1 = 13,    /* slow-path check (host bounds too small)                    */
    MZ_S_CYC_STAGE2 = 14,    /* round 2 issue: RNG window, the leaf's record               */
    MZ_S_CYC_EXPAND = 15,    /* leaf expansion                                             */
    MZ_S_CYC_BACKUP = 16,    /* waiting for the back-propagation wave (barrier)            */
    MZ_S_CYC_MINMAX = 17,    /* waiting for the RNG window                                 */
    MZ_S_CYC_SELECT = 18,    /* value scores + selection walk                              */
    MZ_S_CYC_GATHER = 19,    /* hidden-state gather loads                                  */
    MZ_S_CYC_EPILOGUE = 20,  /* header write-back, gather stores, statistics               */
    MZ_S_STAMPED = 21,       /* stamped launches x trees                                   */
    /* wave 1 (back-propagation): */
    MZ_S_CYC_W1_ROUND1 = 22, /* round 1: node records, path, lambda powers issued and waited */
    MZ_S_CYC_W1_STAGE2 = 23, /* round 2 issue: path-node value sets, value entries         */
    MZ_S_CYC_W1_BACKUP = 24, /* back-propagation + min/max                                 */
    MZ_S_CYC_W1_SYNC = 25,   /* wave 1's whole span, start to back-propagation done        */
    MZ_S_CYC_EXP_CDF = 26,   /* expansion: sampling distribution                           */
    MZ_S_CYC_EXP_DRAW = 27,  /* expansion: K draws                                         */
    MZ_S_CYC_EXP_NODES = 28, /* expansion: child creation                                  */
    MZ_S_CYC_BAK_BOOT = 29,  /* back-propagation: bootstrap values                         */
    MZ_S_CYC_BAK_WAIT = 30,  /* back-propagation: waiting for staged entries               */
    MZ_S_CYC_BAK_NODES = 31, /* back-propagation: node updates                             */
    MZ_S_COUNT = 32
};

/* --- library -------------------------------------------------------------------------- */
const char *mz_last_error(void);
int mz_abi_version(void);
/* Name of the backend: "hip-gfx950", "reference-ctree" or "cpu-port". */
const char *mz_backend(void);

/* --- lifetime ------------------------------------------------------------------------- */
/* Replaces CTree_batch::CTree_batch (cnode.cpp:553-577) / Tree_batch.__cinit__ (cytree.pyx:11-16).
 * Tree i of this batch is seeded with random_seed*2333 + (root_offset + i) (cnode.cpp:574);
 * root_offset lets a rank own a contiguous shard of a larger batch with bit-identical trees. */
int mz_create(int root_num, int agent_num, int action_space_size, int sampled_times,
              int simulation_num, float tree_value_stat_delta_lb, uint32_t random_seed,
              float rho, float lam, int root_offset, mz_batch **out);
/* Replaces CTree_batch::~CTree_batch (cnode.cpp:579-587). */
int mz_destroy(mz_batch *b);
/* Make subsequent device work of this handle run on `stream` (a hipStream_t; NULL = default).
 * The handle's eager work already queued is ordered before it (a wait on an event each enqueueing
 * call records behind its work), unless `stream` is capturing a graph.  The previous stream is
 * not touched: the caller may have destroyed it. */
int mz_set_stream(mz_batch *b, void *stream);
/* Wait for all work of this handle and report any deferred device-side error. */
int mz_synchronize(mz_batch *b);

/* --- search ---------------------------------------------------------------------------- */
/* Replaces CTree_batch::prepare (cnode.cpp:589-614) / Tree_batch.prepare (cytree.pyx:21-47).
 * rewards, values: [B]; policy_probs, beta, noises: [B, agent_num, A].
 * Host memory (MZ_MEM_HOST): packed into the handle's pinned stage, launched, synchronised. */
int mz_prepare(mz_batch *b, const float *rewards, const float *values, const float *policy_probs,
               const float *beta, int sampled_times, float noise_eps, const float *noises, int mem);

/* Replaces CTree_batch::cbatch_selection (cnode.cpp:616-642) / Tree_batch.batch_selection
 * (cytree.pyx:50-67).  Outputs: idx_x [B] (hidden_state_index_x of the leaf's parent),
 * idy [B] (= 0..B-1), actions [B, agent_num] (action on the edge into the leaf).
 * Host memory: an expansion staged by mz_expand_backup(MZ_MEM_HOST) just before runs fused with
 * this selection in one launch; the kernel writes the outputs through the stage's device mapping
 * (MZ_HOST_COPY=1 at mz_create: one device->host copy); one synchronisation, which reports the
 * device-side errors of both. */
int mz_select(mz_batch *b, float pb_c_base, float pb_c_init, float discount,
              int32_t *idx_x, int32_t *idy, int32_t *actions, int mem);

/* Replaces CTree_batch::cbatch_expansion_and_backup (cnode.cpp:644-670) /
 * Tree_batch.batch_expansion_and_backup (cytree.pyx:69-91).
 * rewards, values: [B]; policy_probs, beta: [B, agent_num, A].
 * Host memory: the inputs are packed into the handle's pinned stage and the launch is deferred to
 * the handle's next call (fused with it when that is mz_select with host outputs); its device-side
 * errors are reported by that call.  Device memory: enqueued on the handle's stream. */
int mz_expand_backup(mz_batch *b, int hidden_state_index_x, float discount, int sampled_times,
                     const float *rewards, const float *values, const float *policy_probs,
                     const float *beta, int mem);

/* Fused device path (no reference counterpart): the expansion+backup of simulation s followed by
 * the selection of simulation s+1 in one launch; identical results to mz_expand_backup followed
 * by mz_select.  When `pool` is non-null the leaf hidden states of the new selection are also
 * gathered: gather_out[i, :] = pool[idx_x[i]][root i][:]  (mcts_sampled.py:130-134), where pool
 * is laid out [slots, B, row_bytes] with slot stride pool_slot_stride bytes.  Device memory only. */
int mz_expand_backup_select(mz_batch *b, int hidden_state_index_x, float discount, int sampled_times,
                            const float *rewards, const float *values, const float *policy_probs,
                            const float *beta, float pb_c_base, float pb_c_init,
                            int32_t *idx_x, int32_t *idy, int32_t *actions,
                            const void *pool, int64_t pool_slot_stride, int64_t row_bytes,
                            void *gather_out);

/* Fused device path (no reference counterpart): mz_prepare followed by mz_select in one launch.
 * Right after prepare the root has one visit and at least one child, so the first selection is
 * the forced round-robin child 0 (cnode.cpp:398-399, no scoring, no engine word): identical
 * results to the two calls.  Device memory only. */
int mz_prepare_select(mz_batch *b, const float *rewards, const float *values, const float *policy_probs,
                      const float *beta, int sampled_times, float noise_eps, const float *noises,
                      float pb_c_base, float pb_c_init, float discount,
                      int32_t *idx_x, int32_t *idy, int32_t *actions);

/* Standalone hidden-state gather (mcts_sampled.py:130-134): out[i] = pool[idx_x[i]][i].
 * Device memory only; row_bytes must be a multiple of 4. */
int mz_gather_rows(mz_batch *b, const void *pool, int64_t pool_slot_stride, int64_t row_bytes,
                   const int32_t *idx_x, void *out);

/* --- readbacks ------------------------------------------------------------------------- */
/* CTree_batch::get_roots_values (cnode.cpp:672-679): out [B]. */
int mz_get_roots_values(mz_batch *b, float *out, int mem);
/* CTree_batch::get_roots_marginal_visit_count (cnode.cpp:682-690): out [B, agent_num, A]. */
int mz_get_roots_marginal_visit_count(mz_batch *b, int32_t *out, int mem);
/* CTree_batch::get_roots_marginal_priors (cnode.cpp:692-700): out [B, agent_num, A]. */
int mz_get_roots_marginal_priors(mz_batch *b, float *out, int mem);
/* CTree_batch::get_num_children_of_root (cnode.cpp:702-705). */
int mz_get_num_children_of_root(mz_batch *b, int tree_id, int32_t *out);
/* CTree_batch::get_root_sampled_* (cnode.cpp:707-781) for one tree, host memory. */
int mz_get_root_sampled(mz_batch *b, int field, int tree_id, float discount, void *out);
/* Upper bound on deg(root) for every tree of this batch (= min(K, A^agent_num)). */
int mz_max_children(mz_batch *b, int32_t *out);
/* Batched form of all get_root_sampled_* readbacks: out [B, max_children(, agent_num)] padded
 * with zeros past each root's degree; degrees [B] (may be NULL). */
int mz_get_roots_sampled_padded(mz_batch *b, int field, float discount, void *out,
                                int32_t *degrees, int mem);

/* Every readback above for all roots in one launch, written straight into device buffers
 * (mcts_sampled.py:176-191 reads them all after each search); a NULL entry is not written.
 * values [B]; marginal_* [B, agent_num, A]; degrees [B]; sampled[f] is the MZ_F_* field f as
 * mz_get_roots_sampled_padded lays it out ([B, max_children(, agent_num)], zero-padded).
 * Device memory only; stream-ordered, no synchronisation. */
typedef struct {
    float *values;
    int32_t *marginal_visit_count;
    float *marginal_priors;
    int32_t *degrees;
    void *sampled[MZ_F_COUNT];
} mz_readback_out;
int mz_get_roots_device(mz_batch *b, float discount, const mz_readback_out *out);

/* --- diagnostics ----------------------------------------------------------------------- */
/* Counters accumulated since creation (MZ_S_COUNT int64 values of this header's ABI: size the buffer
 * by the MZ_S_COUNT of the MZ_ABI_VERSION that mz_abi_version() returns); host memory. */
int mz_get_stats(mz_batch *b, int64_t *out);
/* CTree_batch::print (cnode.cpp:783-791): debug dump to stderr. */
int mz_print(mz_batch *b);

#ifdef __cplusplus
}
#endif

#endif /* MZMCTS_H */
