// Host sampler microbenchmark (ml-1m-sized synthetic positives): the full pass and
// its two halves -- word generation + masking, and the membership walk.
#include "../../ncf_amd/csrc/sampler.cpp"
#include <chrono>
#include <cstdio>
#include <random>
static double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}
int main() {
    const int U = 6041, I = 3707;
    std::mt19937 g(1);
    std::vector<int32_t> pu, pi;
    for (int u = 0; u < U; u++) { int c = 1 + g() % 330; for (int k = 0; k < c; k++) { pu.push_back(u); pi.push_back(g() % I); } }
    Sampler* s = (Sampler*)ncf_sampler_create(pu.data(), pi.data(), pu.size(), U, I);
    std::vector<int32_t> out(pu.size() * 4);
    uint32_t key[624]; int32_t pos; ncf_mt_seed(5, key, &pos);
    for (int r = 0; r < 5; r++) {
        auto t0 = std::chrono::steady_clock::now();
        int64_t w = ncf_sampler_sample(s, I, 4, key, &pos, out.data());
        printf("full pass: %ld words %.2f ms\n", (long)w, ms_since(t0));
    }
    std::vector<uint32_t> buf(BLK_WORDS); std::vector<uint16_t> cand(BLK_WORDS);
    for (int r = 0; r < 3; r++) {
        auto t0 = std::chrono::steady_clock::now(); int q = pos; long tot = 0;
        for (int b = 0; b < 470; b++) { fill_words(key, &q, BLK_WORDS, buf.data()); tot += buf[7]; }
        double a = ms_since(t0); t0 = std::chrono::steady_clock::now();
        for (int b = 0; b < 470; b++) { int n = 0; for (int k = 0; k < BLK_WORDS; k++) { uint32_t v = buf[k] & 4095u; cand[n] = (uint16_t)v; n += v <= 3706u; } tot += n; }
        printf("generate %.2f ms, mask+compact %.2f ms (%ld)\n", a, ms_since(t0), tot);
    }
    std::vector<uint16_t> cands(6000000); for (auto& x : cands) x = g() % I;
    for (int r = 0; r < 3; r++) {
        auto t0 = std::chrono::steady_clock::now(); size_t c = 0; int64_t o = 0;
        for (const int32_t u : s->pos_users) { const uint64_t* row = s->bits.data() + (size_t)u * s->words_per_user;
            for (int t = 0; t < 4; t++) for (;;) { uint32_t v = cands[c++]; if ((row[v >> 6] >> (v & 63)) & 1ull) continue; out[o++] = v; break; } }
        printf("walk only %.2f ms (%zu candidates)\n", ms_since(t0), c);
    }
}
