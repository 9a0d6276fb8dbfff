// Host negative sampler (include/ncf_sampler.h).  Bit-exact with the reference
// NCFData.ng_sample (src/data/datasets.py:53-69) under NumPy's legacy global
// RandomState: same MT19937 word stream, same masked-rejection randint, same
// membership test.  Membership is a per-user bitset when U*I bits fit in
// 512 MiB (ml-1m: 2.8 MB, ml-20m: 463 MB), else CSR rows + binary search.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/ncf_sampler.h"

namespace {

constexpr int N = 624, M = 397;

struct Sampler {
    int32_t n_users = 0, n_items = 0;
    bool use_bits = false;
    int64_t words_per_user = 0;
    std::vector<uint64_t> bits;
    std::vector<int64_t> row_ptr;
    std::vector<int32_t> cols;
    std::vector<int32_t> pos_users;  // file order

    bool contains(int32_t u, int32_t i) const {
        if (u < 0 || u >= n_users || i < 0) return false;
        if (use_bits) {
            if (i >= n_items) return false;
            return (bits[(size_t)(u * words_per_user + (i >> 6))] >> (i & 63)) & 1ull;
        }
        const int32_t* b = cols.data() + row_ptr[u];
        const int32_t* e = cols.data() + row_ptr[u + 1];
        return std::binary_search(b, e, i);
    }
};

inline void regenerate(uint32_t* mt) {
    int k;
    uint32_t y;
    for (k = 0; k < N - M; k++) {
        y = (mt[k] & 0x80000000u) | (mt[k + 1] & 0x7fffffffu);
        mt[k] = mt[k + M] ^ (y >> 1) ^ (-(y & 1u) & 0x9908b0dfu);
    }
    for (; k < N - 1; k++) {
        y = (mt[k] & 0x80000000u) | (mt[k + 1] & 0x7fffffffu);
        mt[k] = mt[k + (M - N)] ^ (y >> 1) ^ (-(y & 1u) & 0x9908b0dfu);
    }
    y = (mt[N - 1] & 0x80000000u) | (mt[0] & 0x7fffffffu);
    mt[N - 1] = mt[M - 1] ^ (y >> 1) ^ (-(y & 1u) & 0x9908b0dfu);
}

inline uint32_t temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

}  // namespace

extern "C" {

void* ncf_sampler_create(const int32_t* users, const int32_t* items, int64_t n_pos, int32_t n_users,
                         int32_t n_items) {
    if (n_pos < 0 || n_users <= 0 || n_items <= 0 || (n_pos > 0 && (!users || !items))) return nullptr;
    Sampler* s = new Sampler();
    s->n_users = n_users;
    s->n_items = n_items;
    s->pos_users.assign(users, users + n_pos);
    const int64_t wpu = (n_items + 63) / 64;
    if ((double)n_users * (double)wpu * 8.0 <= 512.0 * 1024 * 1024) {
        s->use_bits = true;
        s->words_per_user = wpu;
        s->bits.assign((size_t)(n_users * wpu), 0ull);
        for (int64_t p = 0; p < n_pos; ++p) {
            const int32_t u = users[p], i = items[p];
            if (u >= 0 && u < n_users && i >= 0 && i < n_items)
                s->bits[(size_t)(u * wpu + (i >> 6))] |= 1ull << (i & 63);
        }
    } else {
        s->row_ptr.assign((size_t)n_users + 1, 0);
        for (int64_t p = 0; p < n_pos; ++p)
            if (users[p] >= 0 && users[p] < n_users) s->row_ptr[(size_t)users[p] + 1]++;
        for (int32_t u = 0; u < n_users; ++u) s->row_ptr[u + 1] += s->row_ptr[u];
        s->cols.resize((size_t)s->row_ptr[n_users]);
        std::vector<int64_t> fill(s->row_ptr.begin(), s->row_ptr.end() - 1);
        for (int64_t p = 0; p < n_pos; ++p)
            if (users[p] >= 0 && users[p] < n_users) s->cols[(size_t)fill[users[p]]++] = items[p];
        for (int32_t u = 0; u < n_users; ++u)
            std::sort(s->cols.begin() + s->row_ptr[u], s->cols.begin() + s->row_ptr[u + 1]);
    }
    return s;
}

void ncf_sampler_destroy(void* s) { delete static_cast<Sampler*>(s); }

int ncf_sampler_contains(const void* s, int32_t u, int32_t i) {
    return static_cast<const Sampler*>(s)->contains(u, i) ? 1 : 0;
}

void ncf_mt_seed(uint32_t seed, uint32_t* key, int32_t* pos) {
    key[0] = seed;
    for (int i = 1; i < N; i++) key[i] = 1812433253u * (key[i - 1] ^ (key[i - 1] >> 30)) + (uint32_t)i;
    *pos = N;
}

int64_t ncf_sampler_sample(const void* sp, int32_t num_item, int32_t num_ng, uint32_t* key, int32_t* pos,
                           int32_t* out_items) {
    const Sampler* s = static_cast<const Sampler*>(sp);
    if (!s || !key || !pos || num_item <= 0 || num_ng < 0 || *pos < 0 || *pos > N) return -1;
    if (num_ng > 0 && !out_items && !s->pos_users.empty()) return -1;
    uint32_t mt[N];
    std::memcpy(mt, key, sizeof(mt));
    int p = *pos;
    int64_t words = 0;
    const uint32_t rng = (uint32_t)num_item - 1u;
    uint32_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    auto next = [&]() -> uint32_t {
        if (p >= N) {
            regenerate(mt);
            p = 0;
        }
        ++words;
        return temper(mt[p++]);
    };
    auto randint = [&]() -> int32_t {
        if (rng == 0) return 0;  // numpy returns `low` without consuming a word
        uint32_t v;
        while ((v = (next() & mask)) > rng) {
        }
        return (int32_t)v;
    };
    int64_t o = 0;
    for (const int32_t u : s->pos_users) {
        for (int t = 0; t < num_ng; ++t) {
            int32_t j = randint();
            while (s->contains(u, j)) j = randint();
            out_items[o++] = j;
        }
    }
    std::memcpy(key, mt, sizeof(mt));
    *pos = p;
    return words;
}

}  // extern "C"
