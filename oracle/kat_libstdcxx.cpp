// ORACLE — TEST INFRASTRUCTURE ONLY.
// Known-answer generator for the two libstdc++ (GCC 11.4) facilities the reference tree uses:
// std::mt19937 (seeded per tree with random_seed*2333+i, cnode.cpp:574) and
// std::discrete_distribution<int> over float weights (cnode.cpp:249,257).  Run by
// oracle/gen_golden.py; its output is committed as tests/golden/kat_libstdcxx.json so the
// restatements (oracle/ptree.py, oracle/cpu_port.cpp, the HIP kernels) are pinned against the real
// library without the library.
//
// Output (one JSON object on stdout):
//   mt:   [[seed, [first 1300 words]] ...]        (1300 > 2 twist blocks)
//   mt10000_5489: the 10000th output of a default-seeded mt19937 (C++ standard: 4123659995)
//   dd:   [[seed, weights[], [draws...], words_consumed] ...]
#include <cstdio>
#include <random>
#include <vector>

int main() {
    std::printf("{\"mt\": [");
    const unsigned seeds[] = {0u, 1u, 5489u, 2333u * 17u + 3u, 4294967295u, 255u * 2333u + 1023u};
    for (size_t si = 0; si < sizeof(seeds) / sizeof(seeds[0]); ++si) {
        std::mt19937 g(seeds[si]);
        std::printf("%s[%u, [", si ? ", " : "", seeds[si]);
        for (int k = 0; k < 1300; ++k) std::printf("%s%u", k ? ", " : "", (unsigned)g());
        std::printf("]]");
    }
    {
        std::mt19937 g;
        unsigned v = 0;
        for (int k = 0; k < 10000; ++k) v = (unsigned)g();
        std::printf("], \"mt10000_5489\": %u, \"dd\": [", v);
    }
    // weight vectors: uniform, skewed, zeros inside / at the ends, single entry, denormal-ish
    std::vector<std::vector<float>> W = {
        {1.f, 1.f, 1.f},
        {0.7f, 0.2f, 0.1f},
        {0.f, 0.5f, 0.f, 0.5f, 0.f},
        {1.f},
        {0.05f, 0.05f, 0.1f, 0.2f, 0.6f, 0.f, 0.f, 0.f, 0.f},
        {1e-30f, 1.f, 1e-30f},
        {0.1f, 0.1f, 0.1f, 0.1f, 0.1f, 0.1f, 0.1f, 0.1f, 0.1f, 0.1f, 0.1f, 0.1f, 0.1f, 0.1f, 0.1f},
    };
    int first = 1;
    for (unsigned seed : {7u, 2333u * 5u + 2u, 99991u}) {
        for (auto &w : W) {
            std::mt19937 g(seed), probe(seed);
            std::discrete_distribution<> d(w.begin(), w.end());
            std::printf("%s[%u, [", first ? "" : ", ", seed);
            first = 0;
            for (size_t k = 0; k < w.size(); ++k) std::printf("%s%.9g", k ? ", " : "", (double)w[k]);
            std::printf("], [");
            const int n = 200;
            for (int k = 0; k < n; ++k) std::printf("%s%d", k ? ", " : "", d(g));
            // count engine words consumed by comparing engine states
            long consumed = 0;
            while (!(probe == g) && consumed < 100000) {
                probe();
                ++consumed;
            }
            std::printf("], %ld]", consumed);
        }
    }
    std::printf("]}\n");
    return 0;
}
