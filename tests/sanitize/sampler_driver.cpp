// Sanitizer driver for the host negative sampler (ncf_amd/csrc/sampler.cpp,
// mt_jump.h): compiled together with sampler.cpp under -fsanitize=address or
// -fsanitize=thread by tests/test_sanitizers.py (CPU only, no HIP).
//
// Input file (little-endian): int64 n_pos, int32 n_users, int32 n_items,
// int32 num_ng, uint32 seed, int32 passes, int32 users[n_pos], int32 items[n_pos].
// For each thread count given on the command line it runs `passes` consecutive
// ng_sample passes (datasets.py:53-69) from np.random.seed(seed) on the parallel
// pass (threads > 1) and on the sequential pass (threads = 1), requires equal
// negatives, word counts and end states, and checks the parallel word generator
// (ncf_words_fill, the randperm words) against ncf_mt_words.  The first pass's
// negatives of the first thread count go to the output file (int32), for the test
// to compare with the oracle's C restatement (oracle/sampler_oracle.c).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/ncf_sampler.h"

static bool read_all(FILE* f, void* p, size_t n) { return fread(p, 1, n, f) == n; }

struct Run {
    std::vector<std::vector<int32_t>> neg;
    std::vector<int64_t> words;
    std::vector<uint32_t> key;
    int32_t pos = 0;
};

static Run run(void* s, int32_t threads, int32_t n_items, int32_t num_ng, uint32_t seed, int passes, int64_t n_pos) {
    Run r;
    if (ncf_sampler_set_threads(s, threads) != 0) {
        fprintf(stderr, "set_threads(%d) failed\n", threads);
        exit(2);
    }
    r.key.assign(624, 0);
    ncf_mt_seed(seed, r.key.data(), &r.pos);
    for (int p = 0; p < passes; ++p) {
        std::vector<int32_t> out((size_t)n_pos * num_ng);
        const int64_t w = ncf_sampler_sample(s, n_items, num_ng, r.key.data(), &r.pos, out.data());
        if (w < 0) {
            fprintf(stderr, "ncf_sampler_sample returned %lld\n", (long long)w);
            exit(2);
        }
        r.words.push_back(w);
        r.neg.push_back(std::move(out));
    }
    return r;
}

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s input output threads...\n", argv[0]);
        return 2;
    }
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    int64_t n_pos;
    int32_t n_users, n_items, num_ng, passes;
    uint32_t seed;
    if (!read_all(f, &n_pos, 8) || !read_all(f, &n_users, 4) || !read_all(f, &n_items, 4) ||
        !read_all(f, &num_ng, 4) || !read_all(f, &seed, 4) || !read_all(f, &passes, 4))
        return 2;
    std::vector<int32_t> users(n_pos), items(n_pos);
    if (!read_all(f, users.data(), 4 * n_pos) || !read_all(f, items.data(), 4 * n_pos)) return 2;
    fclose(f);

    void* s = ncf_sampler_create(users.data(), items.data(), n_pos, n_users, n_items);
    if (!s) return 2;
    const Run seq = run(s, 1, n_items, num_ng, seed, passes, n_pos);
    int bad = 0;
    for (int a = 3; a < argc; ++a) {
        const int32_t t = atoi(argv[a]);
        const Run par = run(s, t, n_items, num_ng, seed, passes, n_pos);
        for (int p = 0; p < passes; ++p) {
            if (par.neg[p] != seq.neg[p] || par.words[p] != seq.words[p]) {
                fprintf(stderr, "threads %d pass %d: negatives or word count differ from the sequential pass\n", t, p);
                ++bad;
            }
        }
        if (par.key != seq.key || par.pos != seq.pos) {
            fprintf(stderr, "threads %d: end state differs\n", t);
            ++bad;
        }
        if (a == 3) {
            FILE* o = fopen(argv[2], "wb");
            if (!o || fwrite(par.neg[0].data(), 4, par.neg[0].size(), o) != par.neg[0].size()) return 2;
            fclose(o);
        }
        // the parallel word generator against the sequential stream (randperm words)
        const int64_t nw = 3 * 624 * 1000 + 77;
        std::vector<uint32_t> k1(624), k2(624), w1(nw), w2(nw);
        int32_t p1, p2;
        ncf_mt_seed(seed ^ 0x5a5a5a5au, k1.data(), &p1);
        k2 = k1;
        p2 = p1;
        ncf_mt_words(k1.data(), &p1, nw, w1.data());
        void* wg = ncf_words_create(t);
        if (!wg || ncf_words_fill(wg, k2.data(), &p2, nw, w2.data()) != 0) return 2;
        ncf_words_destroy(wg);
        if (w1 != w2 || k1 != k2 || p1 != p2) {
            fprintf(stderr, "threads %d: ncf_words_fill differs from ncf_mt_words\n", t);
            ++bad;
        }
    }
    int64_t st[16] = {0};
    ncf_sampler_stats(s, st, 16);
    ncf_sampler_destroy(s);
    printf("passes parallel %lld sequential %lld redone %lld bad %d\n", (long long)st[0], (long long)st[1],
           (long long)st[3], bad);
    return bad ? 1 : 0;
}
