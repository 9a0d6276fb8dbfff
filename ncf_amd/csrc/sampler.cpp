// Host negative sampler (include/ncf_sampler.h).  Bit-exact with the reference
// NCFData.ng_sample (src/data/datasets.py:53-69) under NumPy's legacy global
// RandomState: same MT19937 word stream, same masked-rejection randint, same
// membership test.  Membership is a per-user bitset when U*I bits fit in
// 512 MiB (ml-1m: 2.8 MB, ml-20m: 463 MB), else CSR rows + binary search.
#include <immintrin.h>

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
// 9,984-word blocks by fill_words (vectorised regenerate + temper); each block is
// masked and compacted into its randint candidates (v = w & mask <= n - 1; AVX-512
// compress where the CPU has it); then each run of consecutive positives of one
// user (file order: the training file is sorted by user) takes its num_ng * run
// slots from the candidates: the non-members of the user's positives, in order
// (a member is the reference's "draw again").  With AVX-512, 16 candidates at a
// time: membership bits gathered first, non-members compressed into the slots.  The state after the pass: the snapshot taken
// before the block holding the last accepted word, advanced to just past it.
// (A generator thread feeding the walk was measured slower: the blocks' cache
// lines moving between cores cost more than the generation it overlapped.)
namespace {
constexpr int BLK_WORDS = N * 16;
constexpr int CAND_PAD = 16;  // full-vector stores past the last candidate

__attribute__((target("avx512f"))) int compact_avx512(const uint32_t* w, uint32_t mask, uint32_t rng, uint32_t* out) {
    const __m512i vm = _mm512_set1_epi32((int)mask), vr = _mm512_set1_epi32((int)rng);
    int nc = 0;
    for (int k = 0; k < BLK_WORDS; k += 16) {
        const __m512i v = _mm512_and_si512(_mm512_loadu_si512(w + k), vm);
        const __mmask16 keep = _mm512_cmple_epu32_mask(v, vr);
        _mm512_storeu_si512(out + nc, _mm512_maskz_compress_epi32(keep, v));
        nc += __builtin_popcount((unsigned)keep);
    }
    return nc;
}

int compact_scalar(const uint32_t* w, uint32_t mask, uint32_t rng, uint32_t* out) {
    int nc = 0;
    for (int k = 0; k < BLK_WORDS; ++k) {
        const uint32_t v = w[k] & mask;
        out[nc] = v;
        nc += v <= rng;
    }
    return nc;
}

const bool g_avx512 = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("bmi2");

int compact(const uint32_t* w, uint32_t mask, uint32_t rng, uint32_t* out) {
    return g_avx512 ? compact_avx512(w, mask, rng, out) : compact_scalar(w, mask, rng, out);
}

// One user's walk over candidates cp[*c .. nc) filling out[*o .. end): 16
// candidates at a time, their membership bits gathered from the user's bitset
// row first (no dependence on the slot), the non-members compressed into the
// next slots.  Returns with *o == end or the block exhausted (*c > nc - 16: the
// scalar loop finishes it).
__attribute__((target("avx512f,bmi2"))) void walk_avx512(const uint32_t* cp, int* c, int nc, const uint64_t* row,
                                                          int32_t* out, int64_t* o, int64_t end, int64_t S) {
    int cc = *c;
    int64_t oo = *o;
    const __m512i one = _mm512_set1_epi64(1);
    while (oo < end && cc + 16 <= nc) {
        const __m512i v = _mm512_loadu_si512(cp + cc);
        const __m512i wi = _mm512_srli_epi32(v, 6);
        const __m512i lo = _mm512_i32gather_epi64(_mm512_castsi512_si256(wi), (const long long*)row, 8);
        const __m512i hi = _mm512_i32gather_epi64(_mm512_extracti64x4_epi64(wi, 1), (const long long*)row, 8);
        const __m512i sh = _mm512_and_si512(v, _mm512_set1_epi32(63));
        const __m512i blo = _mm512_srlv_epi64(lo, _mm512_cvtepu32_epi64(_mm512_castsi512_si256(sh)));
        const __m512i bhi = _mm512_srlv_epi64(hi, _mm512_cvtepu32_epi64(_mm512_extracti64x4_epi64(sh, 1)));
        const __mmask8 mlo = _mm512_test_epi64_mask(blo, one), mhi = _mm512_test_epi64_mask(bhi, one);
        const unsigned keep = ~((unsigned)mlo | ((unsigned)mhi << 8)) & 0xffffu;
        const int cnt = __builtin_popcount(keep);
        const int64_t room = end - oo;
        if (cnt < room) {  // the run goes on past these 16
            if (oo + 16 <= S) _mm512_storeu_si512(out + oo, _mm512_maskz_compress_epi32((__mmask16)keep, v));
            else _mm512_mask_compressstoreu_epi32(out + oo, (__mmask16)keep, v);
            oo += cnt;
            cc += 16;
        } else {  // the run ends inside these 16: its last slot takes the room-th non-member,
                  // and the candidates after it belong to the next run
            const unsigned k2 = _pdep_u32((1u << room) - 1u, keep);
            _mm512_mask_compressstoreu_epi32(out + oo, (__mmask16)k2, v);
            oo = end;
            cc += 32 - __builtin_clz(k2);
        }
    }
    *c = cc;
    *o = oo;
}
}  // namespace

template <bool BITS>
static int64_t sample_blocked(const Sampler* s, uint32_t num_item, int32_t num_ng, uint32_t* key, int32_t* pos,
                              int32_t* out_items) {
    const uint32_t rng = num_item - 1u;
    uint32_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    uint32_t mt[N], snap[N];
    std::memcpy(mt, key, sizeof(mt));
    int q = *pos, snap_q = q;
    std::vector<uint32_t> buf(BLK_WORDS);
    std::vector<uint32_t> cand(BLK_WORDS + CAND_PAD);
    const uint32_t* const cp = cand.data();
    int nc = 0, c = 0;
    int64_t blocks = 0;
    const int64_t wpu = s->words_per_user;
    const uint32_t n_items = (uint32_t)s->n_items;
    const int64_t npos = (int64_t)s->pos_users.size();
    const int32_t* const pusers = s->pos_users.data();
    const int64_t S = npos * num_ng;
    const bool vec = g_avx512 && num_item <= n_items;  // every candidate then indexes inside the row
    int64_t o = 0;
    for (int64_t p = 0; p < npos;) {
        const int32_t u = pusers[p];
        int64_t p1 = p + 1;
        while (p1 < npos && pusers[p1] == u) ++p1;
        const int64_t end = o + (p1 - p) * num_ng;
        const bool uok = u >= 0 && u < s->n_users;
        const uint64_t* row = BITS ? s->bits.data() + (size_t)(uok ? u : 0) * wpu : nullptr;
        while (o < end) {
            if (c >= nc) {
                std::memcpy(snap, mt, sizeof(mt));
                snap_q = q;
                fill_words(mt, &q, BLK_WORDS, buf.data());
                ++blocks;
                nc = compact(buf.data(), mask, rng, cand.data());
                c = 0;
                continue;
            }
            if (BITS) {
                if (vec && uok) walk_avx512(cp, &c, nc, row, out_items, &o, end, S);
                while (c < nc && o < end) {  // scalar: the block's tail, or no AVX-512
                    const uint32_t v = cp[c++];
                    if (uok && v < n_items && ((row[v >> 6] >> (v & 63)) & 1ull)) continue;  // (u, v) in train_mat
                    out_items[o++] = (int32_t)v;
                }
            } else {
                const uint32_t v = cp[c++];
                if (!s->contains(u, (int32_t)v)) out_items[o++] = (int32_t)v;
            }
        }
        p = p1;
    }
    // word offset (in the current block) of candidate c - 1, the last one taken
    std::memcpy(mt, snap, sizeof(mt));
    int qb = snap_q;
    fill_words(mt, &qb, BLK_WORDS, buf.data());
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
        return s->use_bits ? sample_blocked<true>(s, (uint32_t)num_item, num_ng, key, pos, out_items)
                           : sample_blocked<false>(s, (uint32_t)num_item, num_ng, key, pos, out_items);
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
