// ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called from the product.
//
// CPU restatement of the reference sampled-MCTS tree (RDG0818/MAZero core/mcts/ctree), written
// from the algorithm, not copied: it uses the data layout the HIP kernels use (per-node value
// entries kept sorted by (depth, value); the min/max normaliser as a reduction over the current
// q-values of visited non-root nodes) and restates the two libstdc++ (GCC 11.4) pieces the
// reference leans on -- std::mt19937 and std::discrete_distribution<int> -- explicitly.
// Every function cites the reference line it follows.  It exports the C-ABI of
// include/mzmcts.h (host memory only) as oracle/_build/libmzport.so.
//
// Parity pinning: checked bit-exactly against (i) the golden vectors in tests/golden/ recorded
// from the compiled reference (oracle/gen_golden.py) and (ii) oracle/_ref/libmzref.so when built.
//
// Floating point: build with -O2 -ffp-contract=off (no FMA contraction), like the reference's
// x86-64 -O2 build which has no FMA instructions available.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "../include/mzmcts.h"

namespace port {

static const float kFloatMin = -1000000.0f;  // FLOAT_MIN, common_lib/utils.h:11-12

// ---- std::mt19937 (libstdc++ bits/random.tcc, mersenne_twister_engine) -----------------------
struct Mt19937 {
    uint32_t x[624];
    int p;
    void seed(uint32_t s) {  // seed(result_type), [rand.eng.mers]/9
        x[0] = s;
        for (int i = 1; i < 624; ++i) x[i] = 1812433253u * (x[i - 1] ^ (x[i - 1] >> 30)) + (uint32_t)i;
        p = 624;
    }
    void twist() {  // _M_gen_rand
        const uint32_t up = 0x80000000u, lo = 0x7fffffffu, a = 0x9908b0dfu;
        for (int k = 0; k < 624 - 397; ++k) {
            uint32_t y = (x[k] & up) | (x[k + 1] & lo);
            x[k] = x[k + 397] ^ (y >> 1) ^ ((y & 1u) ? a : 0u);
        }
        for (int k = 624 - 397; k < 623; ++k) {
            uint32_t y = (x[k] & up) | (x[k + 1] & lo);
            x[k] = x[k + (397 - 624)] ^ (y >> 1) ^ ((y & 1u) ? a : 0u);
        }
        uint32_t y = (x[623] & up) | (x[0] & lo);
        x[623] = x[396] ^ (y >> 1) ^ ((y & 1u) ? a : 0u);
        p = 0;
    }
    uint32_t operator()() {
        if (p >= 624) twist();
        uint32_t z = x[p++];
        z ^= (z >> 11);
        z ^= (z << 7) & 0x9d2c5680u;
        z ^= (z << 15) & 0xefc60000u;
        z ^= (z >> 18);
        return z;
    }
};

// ---- std::discrete_distribution<int> over float weights --------------------------------------
// param_type::_M_initialize (random.tcc:2656-2678) + operator() (random.tcc:2697-2713) +
// generate_canonical<double,53> (random.tcc:3348-3378): two engine words per draw.
struct Discrete {
    std::vector<double> cp;  // empty when fewer than 2 weights: draws return 0 and consume nothing
    void init(const float *w, int n) {
        cp.clear();
        if (n < 2) return;
        double sum = 0.0;
        for (int i = 0; i < n; ++i) sum += (double)w[i];
        double acc = 0.0;
        cp.resize(n);
        for (int i = 0; i < n; ++i) {
            acc = (i == 0) ? ((double)w[0] / sum) : (acc + (double)w[i] / sum);
            cp[i] = acc;
        }
        cp[n - 1] = 1.0;
    }
    int operator()(Mt19937 &g) const {
        if (cp.empty()) return 0;
        double w1 = (double)g();
        double w2 = (double)g();
        double u = (w1 + w2 * 4294967296.0) / 18446744073709551616.0;
        if (u >= 1.0) u = std::nextafter(1.0, 0.0);
        return (int)(std::lower_bound(cp.begin(), cp.end(), u) - cp.begin());
    }
};

struct Entry {
    int depth;
    float value;
};

struct Node {  // CNode, cnode.h:11-45 / ctor cnode.cpp:14-29
    int visit = 0, nc = 0, first_child = 0, hsx = -1;
    float reward = 0.f, pred_value = 0.f, prior = 0.f, pred_prob = 0.f, beta = 0.f, beta_hat = 0.f;
    float ws = 0.f, tw = 0.f;  // SubTreeValueSet weighted_sum / tot_weight (utils.h:18-40)
    std::vector<Entry> vals;   // every backed-up value, sorted by (depth, value)
    std::vector<int> action;   // joint action on the edge into this node, [agent_num]
};

struct Tree {
    Mt19937 gen;
    std::vector<Node> nodes;  // nodes[0] is the root; children of a node are contiguous
    std::vector<int> path;
    int search_len = 0;
    int pool_cap = 0;
};

struct Batch {
    int B, N, A, K, S, root_offset;
    float delta_lb, rho, lam;
    std::vector<float> lam_pow;  // lam_pow[d] = lam_pow[d-1]*lam  (utils.cpp:25-27)
    std::vector<Tree> trees;
};

// CNode::value (cnode.cpp:42-56) with SubTreeValueSet::value_estimation (utils.cpp:73-77)
static inline float node_value(const Node &n) { return n.nc > 0 ? n.ws / n.tw : 0.0f; }
// CNode::get_qsa (cnode.cpp:58-67)
static inline float node_qsa(const Node &n, float discount) { return n.reward + discount * node_value(n); }

// SubTreeValueSet::update (utils.cpp:20-71) on the sorted-entry representation: the multiset
// `big` is always the top max(1,ceil(count*(1-rho))) values of the depth and `small` the rest,
// so min(big) / max(small) are order statistics of the depth's sorted segment.
static void value_update(Batch &bt, Node &n, float key, int depth) {
    auto first = std::lower_bound(n.vals.begin(), n.vals.end(), depth,
                                  [](const Entry &e, int d) { return e.depth < d; });
    auto last = std::upper_bound(first, n.vals.end(), depth,
                                 [](int d, const Entry &e) { return d < e.depth; });
    const int lo = (int)(first - n.vals.begin());
    const int c = (int)(last - first);
    const float lp = bt.lam_pow.at(depth);
    const int cur = (c == 0) ? 0 : std::max(1, (int)std::ceil((float)c * (1.0f - bt.rho)));
    const int lim = std::max(1, (int)std::ceil((float)(c + 1) * (1.0f - bt.rho)));
    if (cur == lim) {
        const float mb = n.vals[lo + c - cur].value;  // *big.begin()
        if (!(key < mb)) {
            n.ws -= lp * mb;
            n.tw -= lp;
            n.tw += lp;
            n.ws += lp * key;
        }
    } else {
        if (cur + 1 != lim) throw std::runtime_error("SubTreeValueSet::update: cur_size+1!=size_lim.");
        if (c - cur == 0) {
            n.tw += lp;
            n.ws += lp * key;
        } else {
            const float ms = n.vals[lo + c - cur - 1].value;  // *(--small.end())
            if (key > ms) {
                n.tw += lp;
                n.ws += lp * key;
            } else {
                n.tw += lp;
                n.ws += lp * ms;
            }
        }
    }
    auto pos = std::lower_bound(n.vals.begin() + lo, n.vals.begin() + lo + c, key,
                                [](const Entry &e, float k) { return e.value < k; });
    n.vals.insert(pos, Entry{depth, key});
}

// CTree::expand (cnode.cpp:224-295)
static void expand(Batch &bt, Tree &t, int node_id, int hsx, float reward, float value,
                   const float *policy, const float *beta, int sampled_times, float noise_eps,
                   const float *noises) {
    const int N = bt.N, A = bt.A;
    {
        Node &n = t.nodes[node_id];
        n.hsx = hsx;
        n.reward = reward;
        n.pred_value = value;
    }
    std::vector<Discrete> dists(N);
    for (int i = 0; i < N; ++i) dists[i].init(beta + (size_t)i * A, A);
    std::map<long, std::pair<float, std::vector<int>>> children;  // key order = child order
    for (int k = 0; k < sampled_times; ++k) {
        long key = 0;
        std::vector<int> act(N);
        for (int i = 0; i < N; ++i) {
            act[i] = dists[i](t.gen);
            key = (long)((unsigned long)key * 23333ul + (unsigned long)act[i]);
        }
        auto &slot = children[key];
        slot.first += 1.0f;
        slot.second = act;
    }
    if ((int)t.nodes.size() + (int)children.size() > t.pool_cap)
        throw std::runtime_error("node pool overflow");
    const int first = (int)t.nodes.size();
    for (auto &kv : children) {
        const float count = kv.second.first;
        const std::vector<int> &act = kv.second.second;
        const float betahat_prob = count / (float)sampled_times;
        float beta_prob = 1.0f, pred_prob = 1.0f, prior = 1.0f;
        for (int i = 0; i < N; ++i) {
            const float pa = policy[(size_t)i * A + act[i]];
            beta_prob *= beta[(size_t)i * A + act[i]];
            pred_prob *= pa;
            if (noise_eps > 0) {
                const float p = pa * (1 - noise_eps) + noises[(size_t)i * A + act[i]] * noise_eps;
                prior *= p;
            } else {
                prior *= pa;
            }
        }
        prior = prior * betahat_prob / beta_prob;
        Node c;
        c.prior = prior;
        c.pred_prob = pred_prob;
        c.beta = beta_prob;
        c.beta_hat = betahat_prob;
        c.action = act;
        t.nodes.push_back(std::move(c));
    }
    Node &n = t.nodes[node_id];
    n.first_child = first;
    n.nc = (int)children.size();
}

struct MinMax {  // CMinMaxStats (utils.cpp:79-103) as a reduction over current q-values
    bool empty = true;
    float mn = 0.f, mx = 0.f;
    float normalize(float v, float delta_lb) const {
        if (empty) return v;
        const float delta = mx - mn;
        return (v - mn) / std::max(delta_lb, delta);
    }
};

// The multiset {q(n) : n visited, n not root}, q = qsa(n) - pred_value(parent) (cnode.cpp:431-446)
static MinMax tree_minmax(const Tree &t, float discount) {
    MinMax m;
    for (size_t p = 0; p < t.nodes.size(); ++p) {
        const Node &par = t.nodes[p];
        for (int j = 0; j < par.nc; ++j) {
            const Node &c = t.nodes[par.first_child + j];
            if (c.visit == 0) continue;
            const float q = node_qsa(c, discount) - par.pred_value;
            if (m.empty) {
                m.mn = m.mx = q;
                m.empty = false;
            } else {
                m.mn = std::min(m.mn, q);
                m.mx = std::max(m.mx, q);
            }
        }
    }
    return m;
}

// CTree::ucb_score (cnode.cpp:297-335); logf / double sqrt as the reference's build resolves them
static float ucb_score(const Batch &bt, const MinMax &mm, const Node &child, float parent_q,
                       int total, float c2, float c1, float discount) {
    float pb_c = std::log(((float)total + c2 + 1) / c2) + c1;
    pb_c *= (std::sqrt((double)total) / (double)(child.visit + 1));
    const float prior_score = pb_c * child.prior;
    float value_score = (child.visit == 0) ? 0.0f : node_qsa(child, discount) - parent_q;
    value_score = mm.normalize(value_score, bt.delta_lb);
    if (value_score < 0) value_score = 0;
    if (value_score > 1) value_score = 1;
    return prior_score + value_score;
}

// CTree::select_child (cnode.cpp:337-379): sequential arg-max with epsilon ties, one engine word
static int select_child(const Batch &bt, Tree &t, const MinMax &mm, const Node &n, float c2, float c1,
                        float discount) {
    float max_score = kFloatMin;
    const float eps = 0.000001f;
    std::vector<int> lst;
    for (int j = 0; j < n.nc; ++j) {
        const float s = ucb_score(bt, mm, t.nodes[n.first_child + j], n.pred_value, n.visit - 1, c2, c1,
                                  discount);
        if (max_score < s) {
            max_score = s;
            lst.clear();
            lst.push_back(j);
        } else if (s >= max_score - eps) {
            lst.push_back(j);
        }
    }
    if (lst.empty()) return 0;
    return lst[t.gen() % lst.size()];
}

// CTree::select_path (cnode.cpp:381-413)
static void select_path(const Batch &bt, Tree &t, float c2, float c1, float discount, int *idx,
                        int *act) {
    const MinMax mm = tree_minmax(t, discount);
    t.path.assign(1, 0);
    int x = 0;
    const int *last_action = nullptr;
    while (t.nodes[x].nc > 0) {
        const Node &n = t.nodes[x];
        int ci;
        if (x == 0 && n.visit <= n.nc) ci = n.visit - 1;
        else ci = select_child(bt, t, mm, n, c2, c1, discount);
        x = n.first_child + ci;
        last_action = t.nodes[x].action.data();
        t.path.push_back(x);
    }
    t.search_len = (int)t.path.size() - 1;
    if (t.search_len < 1) throw std::runtime_error("select on an unexpanded root");
    *idx = t.nodes[t.path[t.search_len - 1]].hsx;
    for (int i = 0; i < bt.N; ++i) act[i] = last_action[i];
}

// CTree::back_propagate (cnode.cpp:415-450); the min/max multiset is recomputed lazily
static void back_propagate(Batch &bt, Tree &t, float value, float discount) {
    float boot = value;
    const int D = t.search_len;
    for (int i = D; i >= 0; --i) {
        Node &n = t.nodes[t.path[i]];
        n.visit += 1;
        value_update(bt, n, boot, D - i);
        boot = n.reward + discount * boot;
    }
}

static std::string g_err;
static int fail(int code, const std::string &m) {
    g_err = m;
    return code;
}

}  // namespace port

using namespace port;

struct mz_batch {
    Batch b;
};

#define GUARD_HOST(mem) \
    if ((mem) != MZ_MEM_HOST) return fail(MZ_ERR_UNSUPPORTED, "cpu port: host memory only")

extern "C" {

const char *mz_last_error(void) { return g_err.c_str(); }
int mz_abi_version(void) { return MZ_ABI_VERSION; }
const char *mz_backend(void) { return "cpu-port"; }

// CTree_batch::CTree_batch (cnode.cpp:553-577)
int mz_create(int B, int N, int A, int K, int S, float delta_lb, uint32_t seed, float rho, float lam,
              int root_offset, mz_batch **out) {
    if (!out || B < 0 || N < 1 || A < 1 || K < 0 || S < 0) return fail(MZ_ERR_ARG, "bad arguments");
    auto *h = new mz_batch;
    Batch &b = h->b;
    b.B = B; b.N = N; b.A = A; b.K = K; b.S = S; b.root_offset = root_offset;
    b.delta_lb = delta_lb; b.rho = rho; b.lam = lam;
    b.lam_pow.resize(S + 3);
    b.lam_pow[0] = 1.0f;
    for (int d = 1; d < S + 3; ++d) b.lam_pow[d] = b.lam_pow[d - 1] * lam;
    b.trees.resize(B);
    for (int i = 0; i < B; ++i) {
        b.trees[i].gen.seed(seed * 2333u + (uint32_t)(root_offset + i));
        b.trees[i].pool_cap = K * (S + 2);
        b.trees[i].nodes.reserve(b.trees[i].pool_cap);
    }
    *out = h;
    return MZ_OK;
}

int mz_destroy(mz_batch *h) {
    delete h;
    return MZ_OK;
}
int mz_set_stream(mz_batch *, void *) { return MZ_OK; }
int mz_synchronize(mz_batch *) { return MZ_OK; }

// CTree_batch::prepare (cnode.cpp:589-614) -> CTree::prepare (cnode.cpp:205-222)
int mz_prepare(mz_batch *h, const float *rewards, const float *values, const float *policy,
               const float *beta, int K, float noise_eps, const float *noises, int mem) {
    GUARD_HOST(mem);
    Batch &b = h->b;
    const size_t stride = (size_t)b.N * b.A;
    try {
        for (int i = 0; i < b.B; ++i) {
            Tree &t = b.trees[i];
            t.nodes.clear();
            Node root;
            root.prior = root.pred_prob = root.beta = root.beta_hat = 1.0f;
            t.nodes.push_back(root);
            expand(b, t, 0, 0, rewards[i], values[i], policy + i * stride, beta + i * stride, K,
                   noise_eps, noises + i * stride);
            t.nodes[0].visit += 1;
            value_update(b, t.nodes[0], values[i], 0);
        }
    } catch (const std::exception &e) {
        return fail(MZ_ERR_RUNTIME, e.what());
    }
    return MZ_OK;
}

// CTree_batch::cbatch_selection (cnode.cpp:616-642)
int mz_select(mz_batch *h, float c2, float c1, float discount, int32_t *idx_x, int32_t *idy,
              int32_t *actions, int mem) {
    GUARD_HOST(mem);
    Batch &b = h->b;
    try {
        for (int i = 0; i < b.B; ++i) {
            select_path(b, b.trees[i], c2, c1, discount, &idx_x[i], &actions[(size_t)i * b.N]);
            idy[i] = i;
        }
    } catch (const std::exception &e) {
        return fail(MZ_ERR_RUNTIME, e.what());
    }
    return MZ_OK;
}

// CTree_batch::cbatch_expansion_and_backup (cnode.cpp:644-670) -> CTree::expand_and_backprop
int mz_expand_backup(mz_batch *h, int hsx, float discount, int K, const float *rewards,
                     const float *values, const float *policy, const float *beta, int mem) {
    GUARD_HOST(mem);
    Batch &b = h->b;
    const size_t stride = (size_t)b.N * b.A;
    try {
        for (int i = 0; i < b.B; ++i) {
            Tree &t = b.trees[i];
            expand(b, t, t.path[t.search_len], hsx, rewards[i], values[i], policy + i * stride,
                   beta + i * stride, K, 0.f, nullptr);
            back_propagate(b, t, values[i], discount);
        }
    } catch (const std::exception &e) {
        return fail(MZ_ERR_RUNTIME, e.what());
    }
    return MZ_OK;
}

int mz_expand_backup_select(mz_batch *, int, float, int, const float *, const float *, const float *,
                            const float *, float, float, int32_t *, int32_t *, int32_t *,
                            const void *, int64_t, int64_t, void *) {
    return fail(MZ_ERR_UNSUPPORTED, "cpu port: fused device path not available");
}
int mz_prepare_select(mz_batch *, const float *, const float *, const float *, const float *, int, float,
                      const float *, float, float, float, int32_t *, int32_t *, int32_t *) {
    return fail(MZ_ERR_UNSUPPORTED, "cpu port: fused device path not available");
}
int mz_get_roots_device(mz_batch *, float, const mz_readback_out *) {
    return fail(MZ_ERR_UNSUPPORTED, "cpu port: device readbacks not available");
}
int mz_gather_rows(mz_batch *, const void *, int64_t, int64_t, const int32_t *, void *) {
    return fail(MZ_ERR_UNSUPPORTED, "cpu port: device gather not available");
}

int mz_get_roots_values(mz_batch *h, float *out, int mem) {
    GUARD_HOST(mem);
    for (int i = 0; i < h->b.B; ++i) out[i] = node_value(h->b.trees[i].nodes[0]);
    return MZ_OK;
}

// CNode::get_marginal_visit_count / get_marginal_priors (cnode.cpp:69-91)
int mz_get_roots_marginal_visit_count(mz_batch *h, int32_t *out, int mem) {
    GUARD_HOST(mem);
    Batch &b = h->b;
    std::memset(out, 0, sizeof(int32_t) * (size_t)b.B * b.N * b.A);
    for (int i = 0; i < b.B; ++i) {
        const Tree &t = b.trees[i];
        const Node &r = t.nodes[0];
        for (int j = 0; j < r.nc; ++j) {
            const Node &c = t.nodes[r.first_child + j];
            for (int a = 0; a < b.N; ++a) out[((size_t)i * b.N + a) * b.A + c.action[a]] += c.visit;
        }
    }
    return MZ_OK;
}

int mz_get_roots_marginal_priors(mz_batch *h, float *out, int mem) {
    GUARD_HOST(mem);
    Batch &b = h->b;
    std::memset(out, 0, sizeof(float) * (size_t)b.B * b.N * b.A);
    for (int i = 0; i < b.B; ++i) {
        const Tree &t = b.trees[i];
        const Node &r = t.nodes[0];
        for (int j = 0; j < r.nc; ++j) {
            const Node &c = t.nodes[r.first_child + j];
            for (int a = 0; a < b.N; ++a) out[((size_t)i * b.N + a) * b.A + c.action[a]] += c.prior;
        }
    }
    return MZ_OK;
}

int mz_get_num_children_of_root(mz_batch *h, int tree_id, int32_t *out) {
    if (tree_id < 0 || tree_id >= h->b.B) return fail(MZ_ERR_ARG, "tree_id out of range");
    *out = h->b.trees[tree_id].nodes.empty() ? 0 : h->b.trees[tree_id].nodes[0].nc;
    return MZ_OK;
}

// CNode::get_sampled_* (cnode.cpp:93-171)
int mz_get_root_sampled(mz_batch *h, int field, int tree_id, float discount, void *out) {
    Batch &b = h->b;
    if (tree_id < 0 || tree_id >= b.B) return fail(MZ_ERR_ARG, "tree_id out of range");
    const Tree &t = b.trees[tree_id];
    if (t.nodes.empty()) return MZ_OK;
    const Node &r = t.nodes[0];
    float *f = (float *)out;
    int32_t *iv = (int32_t *)out;
    for (int j = 0; j < r.nc; ++j) {
        const Node &c = t.nodes[r.first_child + j];
        switch (field) {
        case MZ_F_ACTIONS:
            for (int a = 0; a < b.N; ++a) iv[j * b.N + a] = c.action[a];
            break;
        case MZ_F_VISIT_COUNT: iv[j] = c.visit; break;
        case MZ_F_PRED_PROBS: f[j] = c.pred_prob; break;
        case MZ_F_BETA: f[j] = c.beta; break;
        case MZ_F_BETA_HAT: f[j] = c.beta_hat; break;
        case MZ_F_PRIORS: f[j] = c.prior; break;
        case MZ_F_IMP_RATIO: f[j] = c.beta_hat / c.beta * c.pred_prob; break;
        case MZ_F_PRED_VALUES: f[j] = c.pred_value; break;
        case MZ_F_MCTS_VALUES: f[j] = node_value(c); break;
        case MZ_F_REWARDS: f[j] = c.reward; break;
        case MZ_F_QVALUES: f[j] = node_qsa(c, discount); break;
        default: return fail(MZ_ERR_ARG, "unknown field");
        }
    }
    return MZ_OK;
}

int mz_max_children(mz_batch *h, int32_t *out) {
    long long deg = 1;
    for (int i = 0; i < h->b.N; ++i) deg *= h->b.A;
    *out = (int32_t)(deg < h->b.K ? deg : h->b.K);
    return MZ_OK;
}

int mz_get_roots_sampled_padded(mz_batch *h, int field, float discount, void *out, int32_t *degrees,
                                int mem) {
    GUARD_HOST(mem);
    Batch &b = h->b;
    int32_t maxdeg;
    mz_max_children(h, &maxdeg);
    const int width = (field == MZ_F_ACTIONS) ? maxdeg * b.N : maxdeg;
    std::memset(out, 0, sizeof(float) * (size_t)b.B * width);
    for (int i = 0; i < b.B; ++i) {
        int32_t deg;
        mz_get_num_children_of_root(h, i, &deg);
        if (degrees) degrees[i] = deg;
        int rc = mz_get_root_sampled(h, field, i, discount, (char *)out + sizeof(float) * (size_t)i * width);
        if (rc) return rc;
    }
    return MZ_OK;
}

int mz_get_stats(mz_batch *, int64_t *out) {
    for (int i = 0; i < MZ_S_COUNT; ++i) out[i] = 0;
    return MZ_OK;
}

int mz_print(mz_batch *h) {
    for (int i = 0; i < h->b.B; ++i) {
        fprintf(stderr, "---------- Tree %d info ----------\n", i);
        const Tree &t = h->b.trees[i];
        for (size_t n = 0; n < t.nodes.size(); ++n) {
            const Node &u = t.nodes[n];
            fprintf(stderr, "node %zu: visit %d idx %d reward %f prior %f value %f children %d\n", n,
                    u.visit, u.hsx, u.reward, u.prior, node_value(u), u.nc);
        }
    }
    return MZ_OK;
}

}  // extern "C"
