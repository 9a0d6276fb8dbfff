// Dense Adam pieces shared by the optimizer launches (ncf_ops.hip) and the fused
// step's in-step optimizer (ncf_train.hip, NCF_LAYOUT_ADAM_IN_STEP): the float4 active
// ranges, torch.optim.Adam's per-element update, and the step-scalar cache entries.
#pragma once
#include "ncf_common.h"

namespace ncf {

struct Ranges {
    int64_t begin[8];
    int64_t prefix[9];  // prefix sums of float4 counts
    int n;
};

__device__ __forceinline__ int64_t range_locate(const Ranges& R, int64_t q, int* which) {
    int k = 0;
#pragma unroll
    for (int i = 1; i < 8; ++i)
        if (i < R.n && q >= R.prefix[i]) k = i;
    *which = k;
    return R.begin[k] + (q - R.prefix[k]) * 4;
}

__device__ __forceinline__ bool in_ranges(const Ranges& R, int64_t i) {
    for (int k = 0; k < R.n; ++k)
        if (i >= R.begin[k] && i < R.begin[k] + (R.prefix[k + 1] - R.prefix[k]) * 4) return true;
    return false;
}

__device__ __forceinline__ void adam_f4(f4& p, f4& m, f4& v, const f4& g, float w1, float b2, float omb2,
                                        float bc2s, float eps, float neg_step) {
#pragma clang fp contract(off)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float gr = lane_get(g, r);
        float mr = lane_get(m, r), vr = lane_get(v, r), pr = lane_get(p, r);
        mr = fmaf(w1, gr - mr, mr);          // exp_avg.lerp_(grad, 1 - beta1)   (fmadd form)
        vr = vr * b2 + omb2 * gr * gr;       // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, 1 - beta2)
        const float den = sqrtf(vr) / bc2s + eps;  // (exp_avg_sq.sqrt() / bias_correction2_sqrt).add_(eps)
        pr = pr + neg_step * mr / den;       // param.addcdiv_(exp_avg, denom, value=-step_size)
        if (r == 0) { m.x = mr; v.x = vr; p.x = pr; }
        else if (r == 1) { m.y = mr; v.y = vr; p.y = pr; }
        else if (r == 2) { m.z = mr; v.z = vr; p.z = pr; }
        else { m.w = mr; v.w = vr; p.w = pr; }
    }
}

// Step-t scalars in double like torch's Python scalars, by thread 0 of the block:
// sc[0] = -(lr / (1 - beta1^t)), sc[1] = sqrt(1 - beta2^t) (torch _single_tensor_adam).
// The two double pows take ~2.5 us on one lane -- longer than the launch's loads --
// so each optimizer launch also computes step t + 1's pair (one lane of block 0,
// beside its other work) into a per-control-block cache entry, and step t + 1's
// launch reads it instead: entry [t & 1] is only written by the launch of step t - 1
// (a finished kernel), never by the launch that reads it.  The entry holds its
// inputs (t, lr, beta1, beta2); any mismatch -- first step, a reloaded or
// teacher-forced state, another optimizer on the same control block -- computes
// the pair again, so the cached value is always the one pow gives.
struct ScCache {
    int64_t t;
    double lr, beta1, beta2;
    float sc0, sc1;
    int64_t pad;
};
constexpr int SC_SLOTS = 1024;

__device__ __forceinline__ void step_pair(int64_t t_step, double lr, double beta1, double beta2, float* a, float* b) {
    const double t = (double)t_step;
    *a = (float)(-(lr / (1.0 - pow(beta1, t))));
    *b = (float)sqrt(1.0 - pow(beta2, t));
}

// thread 0: the cache entry of step t, requested (issue early, resolve late)
__device__ __forceinline__ ScCache sc_peek(const ScCache* cache, int64_t t_step) {
    ScCache e;
    e.t = -1;
    if (threadIdx.x == 0 && cache != nullptr) e = cache[t_step & 1];
    return e;
}

__device__ __forceinline__ void sc_resolve(const ScCache& e, int64_t t_step, double lr, double beta1, double beta2,
                                           float* sc) {
    if (threadIdx.x == 0) {
        if (e.t == t_step && e.lr == lr && e.beta1 == beta1 && e.beta2 == beta2) {
            sc[0] = e.sc0;
            sc[1] = e.sc1;
        } else {
            step_pair(t_step, lr, beta1, beta2, &sc[0], &sc[1]);
        }
    }
}

__device__ __forceinline__ void step_scalars(const ScCache* cache, int64_t t_step, double lr, double beta1,
                                             double beta2, float* sc) {
    sc_resolve(sc_peek(cache, t_step), t_step, lr, beta1, beta2, sc);
}

// step t + 1's entry, by lane 0 of wave 1 of this block (vector stores)
__device__ __forceinline__ void step_scalars_ahead_lane(ScCache* cache, int64_t t_step, double lr, double beta1,
                                                        double beta2) {
    if (cache == nullptr || threadIdx.x != 64) return;
    ScCache e;
    e.t = t_step + 1;
    e.lr = lr;
    e.beta1 = beta1;
    e.beta2 = beta2;
    e.pad = 0;
    step_pair(t_step + 1, lr, beta1, beta2, &e.sc0, &e.sc1);
    cache[(t_step + 1) & 1] = e;
}
// ... by block 0
__device__ __forceinline__ void step_scalars_ahead(ScCache* cache, int64_t t_step, double lr, double beta1,
                                                   double beta2) {
    if (blockIdx.x == 0) step_scalars_ahead_lane(cache, t_step, lr, beta1, beta2);
}

// Scalar form of adam_f4 (the same operations per element, so the same bits).
__device__ __forceinline__ float adam_1(float p, float& m, float& v, float g, float w1, float b2, float omb2, float bc2s,
                                        float eps, float neg_step) {
#pragma clang fp contract(off)
    m = fmaf(w1, g - m, m);
    v = v * b2 + omb2 * g * g;
    const float den = sqrtf(v) / bc2s + eps;
    return p + neg_step * m / den;
}

// One float4 column j of the tower slab's total, summed by one thread in the order of
// slab_column_total (ncf_ops.hip): row group rg of 16 sums rows rg, rg + 16, ... (and
// the remainder row), then the 16 group sums in order -- the same bits.
__device__ __forceinline__ f4 slab_column_serial(const float* __restrict__ slab, int64_t j, int stride, int rows) {
    const int per = rows / 16;
    f4 t = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int rg = 0; rg < 16; ++rg) {
        f4 s = f4{0.f, 0.f, 0.f, 0.f};
        const float* q = slab + (int64_t)rg * stride + j;
        for (int r = 0; r < per; ++r) {
            const f4 x = *reinterpret_cast<const f4*>(q + (int64_t)r * 16 * stride);
            s.x += x.x; s.y += x.y; s.z += x.z; s.w += x.w;
        }
        if (rg < rows - 16 * per) {
            const f4 x = *reinterpret_cast<const f4*>(q + (int64_t)per * 16 * stride);
            s.x += x.x; s.y += x.y; s.z += x.z; s.w += x.w;
        }
        if (rg == 0) {
            t = s;
        } else {
            t.x += s.x; t.y += s.y; t.z += s.z; t.w += s.w;
        }
    }
    return t;
}

}  // namespace ncf
