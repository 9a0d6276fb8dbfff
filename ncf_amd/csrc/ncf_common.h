// Shared definitions for the NeuMF HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ncf_hip.h"

typedef float f4 __attribute__((ext_vector_type(4)));

// v_mfma_f32_16x16x4_f32: exact f32 FMA chain, 32-cycle issue per SIMD.
//   A operand: lane l holds A[i = l&15][k = l>>4]
//   B operand: lane l holds B[k = l>>4][j = l&15]
//   C/D      : lane l, reg r holds C[i = 4*(l>>4) + r][j = l&15]
#define MFMA4(a, b, c) __builtin_amdgcn_mfma_f32_16x16x4f32((a), (b), (c), 0, 0, 0)

static constexpr int WAVE = 64;

__device__ __forceinline__ float lane_get(const f4& v, int r) {
    return r == 0 ? v.x : (r == 1 ? v.y : (r == 2 ? v.z : v.w));
}

__device__ __forceinline__ float shfl_xor(float v, int m) { return __shfl_xor(v, m, 64); }

// Exact reference-order BCE-with-logits pieces (torch binary_cross_entropy_with_logits):
//   loss = (1 - y) * x + m + log(exp(-m) + exp(-x - m)),  m = max(-x, 0)
__device__ __forceinline__ float bce_loss(float x, float y) {
    float m = fmaxf(-x, 0.0f);
    return (1.0f - y) * x + m + logf(expf(-m) + expf(-x - m));
}
__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

// Dropout keep hash (include/ncf_hip.h ncf_dropout_hash): splitmix64 finalizer of
// the mixed (seed, step, layer, row, column), upper 32 bits.
__host__ __device__ __forceinline__ uint32_t dropout_hash(uint32_t seed, uint32_t t, uint32_t layer, int64_t row,
                                                          uint32_t col) {
    uint64_t x = ((uint64_t)seed << 32) ^ ((uint64_t)t * 0x9E3779B97F4A7C15ull) ^
                 ((uint64_t)row * 0xBF58476D1CE4E5B9ull) ^ ((uint64_t)((layer << 16) | col) * 0x94D049BB133111EBull);
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return (uint32_t)(x >> 32);
}

// Distillation response term of one row (src/distillation/base.py:27-34 with T > 0,
// response.py:28-32 with T <= 0): *r = its per-row loss, returns d r / d z.
__device__ __forceinline__ float kd_response(float z, float t, float T, float* r) {
    if (T > 0.f) {
        const float ss = sigmoidf_(z / T), st = sigmoidf_(t / T);
        const float d = ss - st;
        *r = d * d * (T * T);
        return 2.f * T * d * (ss * (1.f - ss));
    }
    const float d = z - t;
    *r = d * d;
    return 2.f * d;
}
