/*
 * TEST INFRASTRUCTURE ONLY -- CPU oracle for the negative-sampling stream.
 * Never linked or loaded by the product (ncf_amd/); only tests/, bench.py's
 * cpu_baseline leg and __graft_entry__.smoke() may use it, as the checker.
 *
 * Restates NCFData.ng_sample (reference src/data/datasets.py:53-69):
 *     for (u, i) in positives (file order):
 *         for t in range(num_ng):
 *             j = np.random.randint(num_item)
 *             while (u, j) in train_mat: j = np.random.randint(num_item)
 * with NumPy's legacy global RandomState:
 *   - np.random.seed(s) == MT19937 init_genrand(s) (Matsumoto & Nishimura 1998),
 *   - randint(n) == masked rejection on 32-bit outputs: mask = smallest 2^k-1
 *     >= n-1, draw w until (w & mask) <= n-1   (numpy legacy bounded int path).
 * Membership uses a sorted (u<<32|i) key array + binary search, i.e. the dok
 * matrix's set semantics (datasets.py:23-24, 61).
 * Pinned against tests/golden/G1_negatives.npz (reference outputs).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define MT_N 624
#define MT_M 397

typedef struct { uint32_t mt[MT_N]; int mti; } mt_state;

static void mt_seed(mt_state *s, uint32_t seed) {
    s->mt[0] = seed;
    for (int i = 1; i < MT_N; i++)
        s->mt[i] = 1812433253u * (s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) + (uint32_t)i;
    s->mti = MT_N;
}

static uint32_t mt_next(mt_state *s) {
    static const uint32_t mag01[2] = {0u, 0x9908b0dfu};
    if (s->mti >= MT_N) {
        int k;
        uint32_t y;
        for (k = 0; k < MT_N - MT_M; k++) {
            y = (s->mt[k] & 0x80000000u) | (s->mt[k + 1] & 0x7fffffffu);
            s->mt[k] = s->mt[k + MT_M] ^ (y >> 1) ^ mag01[y & 1u];
        }
        for (; k < MT_N - 1; k++) {
            y = (s->mt[k] & 0x80000000u) | (s->mt[k + 1] & 0x7fffffffu);
            s->mt[k] = s->mt[k + (MT_M - MT_N)] ^ (y >> 1) ^ mag01[y & 1u];
        }
        y = (s->mt[MT_N - 1] & 0x80000000u) | (s->mt[0] & 0x7fffffffu);
        s->mt[MT_N - 1] = s->mt[MT_M - 1] ^ (y >> 1) ^ mag01[y & 1u];
        s->mti = 0;
    }
    uint32_t y = s->mt[s->mti++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

static uint32_t randint(mt_state *s, uint32_t n) {
    uint32_t rng = n - 1u, mask = rng, v;
    if (rng == 0) return 0;   /* numpy returns `off` without consuming a word */
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    while ((v = (mt_next(s) & mask)) > rng) {}
    return v;
}

static int cmp_u64(const void *a, const void *b) {
    uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return (x > y) - (x < y);
}

static int contains(const uint64_t *keys, int64_t n, uint64_t k) {
    int64_t lo = 0, hi = n - 1;
    while (lo <= hi) {
        int64_t mid = (lo + hi) >> 1;
        if (keys[mid] == k) return 1;
        if (keys[mid] < k) lo = mid + 1; else hi = mid - 1;
    }
    return 0;
}

/* users/items: the positives in file order; out_items: n_pos*num_ng negatives.
 * Returns the number of 32-bit MT words consumed (for stream-position checks). */
int64_t oracle_ng_sample(const int64_t *users, const int64_t *items, int64_t n_pos,
                         int64_t num_item, int64_t num_ng, uint32_t seed,
                         int64_t *out_items) {
    uint64_t *keys = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)(n_pos > 0 ? n_pos : 1));
    for (int64_t p = 0; p < n_pos; p++) keys[p] = ((uint64_t)users[p] << 32) | (uint64_t)items[p];
    qsort(keys, (size_t)n_pos, sizeof(uint64_t), cmp_u64);
    mt_state s;
    mt_seed(&s, seed);
    int64_t o = 0;
    for (int64_t p = 0; p < n_pos; p++) {
        uint64_t u = (uint64_t)users[p];
        for (int64_t t = 0; t < num_ng; t++) {
            uint32_t j = randint(&s, (uint32_t)num_item);
            while (contains(keys, n_pos, (u << 32) | j)) j = randint(&s, (uint32_t)num_item);
            out_items[o++] = j;
        }
    }
    free(keys);
    return o;
}

/* Raw MT19937 words after np.random.seed(seed), for stream tests. */
void oracle_mt_words(uint32_t seed, int64_t n, uint32_t *out) {
    mt_state s;
    mt_seed(&s, seed);
    for (int64_t k = 0; k < n; k++) out[k] = mt_next(&s);
}
