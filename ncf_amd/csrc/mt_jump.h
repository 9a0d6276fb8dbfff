// MT19937 jump-ahead for the host samplers (sampler.cpp).
//
// The generator's untempered word stream x_0, x_1, ... obeys
//   x_{k+624} = x_{k+397} ^ twist(x_k, x_{k+1})
// so the 624-word window W_k = (x_k .. x_{k+623}) evolves by a GF(2)-linear map F
// (W_{k+1} = F W_k).  Its minimal polynomial is Phi(x) = x * phi(x): phi is the
// degree-19937 characteristic polynomial of MT19937 proper (irreducible), the
// factor x covers the 31 low bits of x_k, which nothing after W_k depends on.  For a
// jump of J words, g = x^J mod Phi gives F^J = g(F), i.e.
//   W_{k+J} = XOR over {i : g_i = 1} of W_{k+i}
// -- a correlation of g's coefficient bits with the next ~20K words of the stream
// (Haramoto, Matsumoto, Nishimura, Panneton, L'Ecuyer: "Efficient jump ahead for
// F2-linear random number generators", INFORMS J. Computing 2008).  phi itself is
// found once per process by Berlekamp-Massey on one bit of the stream.
//
// A jump lands on a window boundary of the caller's choosing, so the window it
// returns is exactly the key[624] array numpy's legacy RandomState / torch's CPU
// generator hold at that point (their arrays are the windows at multiples of 624
// words from the seeding point); the samplers keep that alignment.
#pragma once

#include <immintrin.h>

#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

// Function multiversioning (an AVX-512 / AVX2 clone picked at load time).
// NCF_SANITIZE (the ASan / TSan builds of tests/test_sanitizers.py): one version --
// the clones' ifunc resolver runs during relocation, before a sanitizer runtime is
// initialised, and an instrumented resolver faults there.
#ifdef NCF_SANITIZE
#define NCF_TARGET_CLONES(...)
#else
#define NCF_TARGET_CLONES(...) __attribute__((target_clones(__VA_ARGS__)))
#endif

namespace mtj {

constexpr int N = 624, M = 397;
constexpr uint32_t MATRIX_A = 0x9908b0dfu, UPPER = 0x80000000u, LOWER = 0x7fffffffu;
constexpr int PHI_DEG = 19937;
constexpr int MOD_DEG = PHI_DEG + 1;             // Phi = x * phi
constexpr int PW = (MOD_DEG + 1 + 63) / 64;      // words of a reduced polynomial (degree < MOD_DEG)

using Poly = std::vector<uint64_t>;  // bit i = coefficient of x^i

inline int degree(const Poly& p) {
    for (int w = (int)p.size() - 1; w >= 0; --w)
        if (p[w]) return w * 64 + 63 - __builtin_clzll(p[w]);
    return -1;
}
inline int bit(const Poly& p, int i) { return (int)((p[(size_t)i >> 6] >> (i & 63)) & 1u); }

// one stream step on a linear buffer: b[k + N] from b[k], b[k + 1], b[k + M]
inline uint32_t next_word(const uint32_t* b) {
    const uint32_t y = (b[0] & UPPER) | (b[1] & LOWER);
    return b[M] ^ (y >> 1) ^ ((y & 1u) ? MATRIX_A : 0u);
}

// r ^= a << s (r sized to hold it)
inline void xor_shifted(uint64_t* r, const uint64_t* a, int na, int s) {
    const int q = s >> 6, sh = s & 63;
    if (sh == 0) {
        for (int k = 0; k < na; ++k) r[q + k] ^= a[k];
    } else {
        for (int k = 0; k < na; ++k) {
            r[q + k] ^= a[k] << sh;
            r[q + k + 1] ^= a[k] >> (64 - sh);
        }
    }
}

// Berlekamp-Massey over GF(2): the connection polynomial C (C_0 = 1) of the
// shortest LFSR generating s[0..n); returns its length L.
inline int berlekamp_massey(const std::vector<uint8_t>& s, Poly& C) {
    const int n = (int)s.size();
    const int W = (n + 63) / 64 + 2;
    C.assign(W, 0);
    Poly B(W, 0), T;
    C[0] = B[0] = 1;
    // reversed sequence bits: rev bit j = s[n - 1 - j], so sum_i C_i s[k - i] is the
    // parity of C & (rev >> (n - 1 - k)) over bits 0..L
    Poly rev(W + 1, 0);
    for (int j = 0; j < n; ++j)
        if (s[n - 1 - j]) rev[(size_t)j >> 6] |= 1ull << (j & 63);
    int L = 0, m = 1;
    for (int k = 0; k < n; ++k) {
        const int off = n - 1 - k;  // bit offset of s[k] in rev
        const int nw = L / 64 + 1;
        uint64_t acc = 0;
        const int q = off >> 6, sh = off & 63;
        for (int w = 0; w < nw; ++w) {
            uint64_t v = rev[(size_t)(q + w)] >> sh;
            if (sh && q + w + 1 < (int)rev.size()) v |= rev[(size_t)(q + w + 1)] << (64 - sh);
            if (w == nw - 1 && ((L + 1) & 63)) v &= (1ull << ((L + 1) & 63)) - 1;  // bits 0..L
            acc ^= C[(size_t)w] & v;
        }
        if (!(__builtin_popcountll(acc) & 1)) {
            ++m;
        } else if (2 * L <= k) {  // C ^= B x^m (B's words past W - q - 1 are zero: deg B + m <= n)
            T = C;
            xor_shifted(C.data(), B.data(), W - (m >> 6) - 1, m);
            L = k + 1 - L;
            B = T;
            m = 1;
        } else {
            xor_shifted(C.data(), B.data(), W - (m >> 6) - 1, m);
            ++m;
        }
    }
    return L;
}

// Phi = x * phi, phi = x^L C(1/x) from Berlekamp-Massey on the top bit of a
// seeded stream (any nonzero bit sequence of the invariant part has phi as its
// minimal polynomial: phi is irreducible).
inline const Poly& modulus() {
    static Poly phi_x;
    static std::once_flag once;
    std::call_once(once, [] {
        const int n = 2 * PHI_DEG + 64;
        std::vector<uint32_t> b((size_t)n + 2 * N);
        b[0] = 5489u;
        for (int i = 1; i < N; i++) b[i] = 1812433253u * (b[i - 1] ^ (b[i - 1] >> 30)) + (uint32_t)i;
        for (size_t k = 0; k + N < b.size(); ++k) b[k + N] = next_word(&b[k]);
        std::vector<uint8_t> s((size_t)n);
        for (int k = 0; k < n; ++k) s[(size_t)k] = (uint8_t)(b[(size_t)k + N] >> 31);  // skip the seeded window
        Poly C;
        const int L = berlekamp_massey(s, C);
        Poly phi((size_t)PW + 1, 0);
        for (int i = 0; i <= L; ++i)
            if (bit(C, i)) phi[(size_t)(L - i) >> 6] |= 1ull << ((L - i) & 63);
        // Phi = x * phi
        phi_x.assign((size_t)PW + 1, 0);
        for (int w = (int)phi.size() - 1; w >= 0; --w) {
            phi_x[(size_t)w] |= phi[(size_t)w] << 1;
            if (w + 1 < (int)phi_x.size()) phi_x[(size_t)w + 1] |= phi[(size_t)w] >> 63;
        }
        if (L != PHI_DEG || degree(phi_x) != MOD_DEG) phi_x.clear();  // checked by ncf_mt_jump_selftest
    });
    return phi_x;
}

// r (any length) reduced mod Phi, result PW words
inline Poly reduce(Poly r) {
    const Poly& P = modulus();
    const int np = (int)P.size();
    for (int i = degree(r); i >= MOD_DEG; --i) {
        if (!bit(r, i)) continue;
        xor_shifted(r.data(), P.data(), std::min(np, (int)r.size() - ((i - MOD_DEG) >> 6) - 1), i - MOD_DEG);
    }
    r.resize((size_t)PW);
    return r;
}

__attribute__((target("pclmul,sse2"))) inline void clmul_acc(uint64_t* r, const uint64_t* a, int na, const uint64_t* b,
                                                               int nb) {
    for (int i = 0; i < na; ++i) {
        if (!a[i]) continue;
        const __m128i ai = _mm_cvtsi64_si128((long long)a[i]);
        for (int j = 0; j < nb; ++j) {
            const __m128i p = _mm_clmulepi64_si128(ai, _mm_cvtsi64_si128((long long)b[j]), 0);
            r[i + j] ^= (uint64_t)_mm_cvtsi128_si64(p);
            r[i + j + 1] ^= (uint64_t)_mm_cvtsi128_si64(_mm_unpackhi_epi64(p, p));
        }
    }
}

inline Poly mulmod(const Poly& a, const Poly& b) {
    Poly r(a.size() + b.size() + 1, 0);
    if (__builtin_cpu_supports("pclmul")) {
        clmul_acc(r.data(), a.data(), (int)a.size(), b.data(), (int)b.size());
    } else {
        for (int i = 0; i < (int)a.size() * 64; ++i)
            if (bit(a, i)) xor_shifted(r.data(), b.data(), (int)b.size(), i);
    }
    return reduce(std::move(r));
}

// x^J mod Phi (square and multiply, top bit first)
inline Poly pow_x_uncached(uint64_t J) {
    Poly g((size_t)PW, 0);
    g[0] = 1;
    for (int b = 63; b >= 0; --b) {
        g = mulmod(g, g);
        if ((J >> b) & 1u) {  // g *= x
            Poly h((size_t)PW + 1, 0);
            for (int w = 0; w < PW; ++w) {
                h[(size_t)w] |= g[(size_t)w] << 1;
                h[(size_t)w + 1] |= g[(size_t)w] >> 63;
            }
            g = reduce(std::move(h));
        }
    }
    return g;
}

// cached: every sampler of a process jumps by the same few distances
inline Poly pow_x(uint64_t J) {
    static std::mutex mu;
    static std::map<uint64_t, Poly> cache;
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = cache.find(J);
        if (it != cache.end()) return it->second;
    }
    Poly g = pow_x_uncached(J);
    std::lock_guard<std::mutex> lk(mu);
    cache.emplace(J, g);
    return g;
}

// acc[0..N) ^= src[0..N)
__attribute__((target("avx512f"))) inline void xor_window_avx512(uint32_t* acc, const uint32_t* src) {
    for (int j = 0; j + 16 <= N; j += 16)
        _mm512_storeu_si512(acc + j, _mm512_xor_si512(_mm512_loadu_si512(acc + j), _mm512_loadu_si512(src + j)));
    // N = 624 = 39 * 16: no tail
}
inline void xor_window_scalar(uint32_t* acc, const uint32_t* src) {
    for (int j = 0; j < N; ++j) acc[j] ^= src[j];
}

// out = the window J words after `win` (g = pow_x(J)); out may alias win.
// Direct form: XOR of the windows W_i, i in g's support (~10K windows of 624 words).
inline void jump_direct(const uint32_t* win, const Poly& g, uint32_t* out) {
    const int dg = degree(g);
    if (dg < 0) {  // cannot happen for a valid modulus
        std::memset(out, 0, sizeof(uint32_t) * N);
        return;
    }
    std::vector<uint32_t> b((size_t)dg + N + 1);
    std::memcpy(b.data(), win, sizeof(uint32_t) * N);
    for (size_t k = 0; k + N < b.size(); ++k) b[k + N] = next_word(&b[k]);
    alignas(64) uint32_t acc[N];
    std::memset(acc, 0, sizeof(acc));
    static const bool avx512 = __builtin_cpu_supports("avx512f");
    for (int w = 0; w <= dg / 64; ++w) {
        uint64_t v = g[(size_t)w];
        while (v) {
            const int i = w * 64 + __builtin_ctzll(v);
            v &= v - 1;
            if (avx512) xor_window_avx512(acc, &b[(size_t)i]);
            else xor_window_scalar(acc, &b[(size_t)i]);
        }
    }
    std::memcpy(out, acc, sizeof(acc));
}

// acc (circular, first word at s) ^= t (linear)
NCF_TARGET_CLONES("avx512f", "avx2", "default") inline void xor_rotated(uint32_t* acc, int s,
                                                                                    const uint32_t* t) {
    const int n1 = N - s;
    for (int j = 0; j < n1; ++j) acc[s + j] ^= t[j];
    for (int j = n1; j < N; ++j) acc[j - n1] ^= t[j];
}

// Horner form over 8-bit chunks of g (top first): acc = F^8(acc) ^ T[chunk], with
// T[v] = XOR_{j: v_j} W_j (256 windows built once per jump) and F applied to the
// circular window in place (8 new words).  ~4x fewer window XORs than jump_direct.
inline void jump(const uint32_t* win, const Poly& g, uint32_t* out) {
    constexpr int Q = 8;
    const int dg = degree(g);
    if (dg < 2 * Q) {
        jump_direct(win, g, out);
        return;
    }
    uint32_t b[N + Q];
    std::memcpy(b, win, sizeof(uint32_t) * N);
    for (int k = 0; k < Q; ++k) b[k + N] = next_word(&b[k]);
    std::vector<uint32_t> T((size_t)(1 << Q) * N);
    std::memset(T.data(), 0, sizeof(uint32_t) * N);
    for (int v = 1; v < (1 << Q); ++v) {
        const uint32_t* lo = &T[(size_t)(v & (v - 1)) * N];
        const uint32_t* w = &b[__builtin_ctz(v)];
        uint32_t* d = &T[(size_t)v * N];
        for (int j = 0; j < N; ++j) d[j] = lo[j] ^ w[j];
    }
    alignas(64) uint32_t acc[N];
    std::memset(acc, 0, sizeof(acc));
    int s = 0;
    for (int c = dg / Q; c >= 0; --c) {
        if (c != dg / Q) {
            for (int k = 0; k < Q; ++k) {  // acc = F(acc): the new word replaces the dropped one
                const uint32_t x0 = acc[s], x1 = acc[s + 1 < N ? s + 1 : 0];
                const uint32_t xm = acc[s + M < N ? s + M : s + M - N];
                const uint32_t y = (x0 & UPPER) | (x1 & LOWER);
                acc[s] = xm ^ (y >> 1) ^ ((y & 1u) ? MATRIX_A : 0u);
                s = s + 1 < N ? s + 1 : 0;
            }
        }
        const int i = c * Q;
        const uint32_t v = (uint32_t)((g[(size_t)i >> 6] >> (i & 63)) & ((1u << Q) - 1));  // Q | 64
        if (v) xor_rotated(acc, s, &T[(size_t)v * N]);
    }
    for (int j = 0; j < N; ++j) out[j] = acc[(s + j) % N];
}

}  // namespace mtj
