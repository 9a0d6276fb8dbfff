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

// Bulk word generation for the device epoch pipeline: whole 624-word blocks
// regenerated and tempered in straight loops the compiler vectorises (an AVX2
// clone is picked at load time where the CPU has it).  Same stream as next().
__attribute__((target_clones("avx2", "default"))) void fill_words(uint32_t* mt, int* p, int64_t n,
                                                                   uint32_t* out) {
    int q = *p;
    int64_t o = 0;
    while (o < n) {
        if (q >= N) {
            // k in [0, N-M): old mt[k+1], mt[k+M]
            for (int k = 0; k < N - M; k++) {
                const uint32_t y = (mt[k] & 0x80000000u) | (mt[k + 1] & 0x7fffffffu);
                mt[k] = mt[k + M] ^ (y >> 1) ^ (-(y & 1u) & 0x9908b0dfu);
            }
            // k in [N-M, N-1): old mt[k+1], new mt[k+M-N] (227 behind: vector-safe)
            for (int k = N - M; k < N - 1; k++) {
                const uint32_t y = (mt[k] & 0x80000000u) | (mt[k + 1] & 0x7fffffffu);
                mt[k] = mt[k + (M - N)] ^ (y >> 1) ^ (-(y & 1u) & 0x9908b0dfu);
            }
            const uint32_t y = (mt[N - 1] & 0x80000000u) | (mt[0] & 0x7fffffffu);
            mt[N - 1] = mt[M - 1] ^ (y >> 1) ^ (-(y & 1u) & 0x9908b0dfu);
            q = 0;
        }
        const int64_t take = (n - o) < (N - q) ? (n - o) : (N - q);
        if (out != nullptr) {
            uint32_t* dst = out + o;
            const uint32_t* src = mt + q;
            for (int64_t k = 0; k < take; ++k) {
                uint32_t y = src[k];
                y ^= (y >> 11);
                y ^= (y << 7) & 0x9d2c5680u;
                y ^= (y << 15) & 0xefc60000u;
                y ^= (y >> 18);
                dst[k] = y;
            }
        }
        q += (int)take;
        o += take;
    }
    *p = q;
}

}  // namespace

extern "C" {

void ncf_mt_words(uint32_t* key, int32_t* pos, int64_t n, uint32_t* out) {
    if (!key || !pos || n <= 0 || *pos < 0 || *pos > N) return;
    int p = *pos;
    fill_words(key, &p, n, out);
    *pos = p;
}

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

}  // extern "C"

// Blocked pass (same draws as the reference loop): the MT19937 stream is run in
// 9,984-word blocks by fill_words (vectorised regenerate + temper), each block is
// masked and compacted branch-free into its randint candidates (v = w & mask <=
// n - 1), and the walk over the positives skips the candidates that are positives
// of the slot's user.  The state after the pass: the snapshot taken before the
// block holding the last accepted word, advanced to just past that word.
// (A generator thread feeding this walk was measured slower: the blocks' cache
// lines moving between cores cost more than the generation it overlapped.)
namespace {
constexpr int BLK_WORDS = N * 16;
}  // namespace

template <typename Cand, bool BITS>
static int64_t sample_blocked(const Sampler* s, uint32_t num_item, int32_t num_ng, uint32_t* key, int32_t* pos,
                              int32_t* out_items) {
    const uint32_t rng = num_item - 1u;
    uint32_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    uint32_t mt[N], snap[N];
    std::memcpy(mt, key, sizeof(mt));
    int q = *pos, snap_q = q;
    std::vector<uint32_t> buf(BLK_WORDS);
    std::vector<Cand> cand(BLK_WORDS);
    Cand* const cp = cand.data();
    int nc = 0, c = 0;
    int64_t blocks = 0;
    const int64_t wpu = s->words_per_user;
    const uint32_t n_items = (uint32_t)s->n_items;
    const uint64_t* const bits = BITS ? s->bits.data() : nullptr;
    const int64_t npos = (int64_t)s->pos_users.size();
    const int32_t* const pusers = s->pos_users.data();
    int64_t o = 0;
    for (int64_t p = 0; p < npos; ++p) {
        const int32_t u = pusers[p];
        const uint64_t* row = BITS ? bits + (size_t)(u >= 0 && u < s->n_users ? u : 0) * wpu : nullptr;
        const bool uok = u >= 0 && u < s->n_users;
        for (int t = 0; t < num_ng; ++t) {
            for (;;) {
                if (c >= nc) {
                    std::memcpy(snap, mt, sizeof(mt));
                    snap_q = q;
                    fill_words(mt, &q, BLK_WORDS, buf.data());
                    ++blocks;
                    nc = 0;
                    const uint32_t* bp = buf.data();
                    for (int k = 0; k < BLK_WORDS; ++k) {
                        const uint32_t v = bp[k] & mask;
                        cp[nc] = (Cand)v;
                        nc += v <= rng;
                    }
                    c = 0;
                    continue;
                }
                const uint32_t v = cp[c++];
                const bool member = BITS ? (uok && v < n_items && ((row[v >> 6] >> (v & 63)) & 1ull))
                                         : s->contains(u, (int32_t)v);
                if (member) continue;  // (u, j) in train_mat: draw again
                out_items[o++] = (int32_t)v;
                break;
            }
        }
    }
    // word offset (in the current block) of candidate c - 1, the last one taken
    int k = 0;
    for (int seen = 0; k < BLK_WORDS; ++k) {
        if ((buf[k] & mask) <= rng && ++seen == c) break;
    }
    std::memcpy(key, snap, sizeof(snap));
    int qq = snap_q;
    fill_words(key, &qq, (int64_t)k + 1, nullptr);
    *pos = qq;
    return (blocks - 1) * BLK_WORDS + k + 1;
}

extern "C" {

int64_t ncf_sampler_sample(const void* sp, int32_t num_item, int32_t num_ng, uint32_t* key, int32_t* pos,
                           int32_t* out_items) {
    const Sampler* s = static_cast<const Sampler*>(sp);
    if (!s || !key || !pos || num_item <= 0 || num_ng < 0 || *pos < 0 || *pos > N) return -1;
    if (num_ng > 0 && !out_items && !s->pos_users.empty()) return -1;
    if (num_ng == 0 || s->pos_users.empty()) return 0;
    if (num_item >= 2)
        return num_item <= 65536
                   ? (s->use_bits ? sample_blocked<uint16_t, true>(s, (uint32_t)num_item, num_ng, key, pos, out_items)
                                  : sample_blocked<uint16_t, false>(s, (uint32_t)num_item, num_ng, key, pos, out_items))
                   : (s->use_bits ? sample_blocked<uint32_t, true>(s, (uint32_t)num_item, num_ng, key, pos, out_items)
                                  : sample_blocked<uint32_t, false>(s, (uint32_t)num_item, num_ng, key, pos, out_items));
    // num_item == 1: numpy's randint(1) returns 0 without consuming a word
    int64_t o = 0;
    for (const int32_t u : s->pos_users) {
        for (int t = 0; t < num_ng; ++t) {
            while (s->contains(u, 0)) {
            }
            out_items[o++] = 0;
        }
    }
    return 0;
}

}  // extern "C"
