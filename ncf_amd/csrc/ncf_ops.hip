// Optimizer, reduction, epoch-shuffle and evaluation kernels + the C ABI
// (include/ncf_hip.h) of libncf_hip.so.  gfx950 only.
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <unordered_map>

#include "ncf_adam.h"
#include "ncf_kernels.h"
#include "ncf_layered.h"

namespace ncf {

// ---------------------------------------------------------------------------
// Slab reduction: grads[tb + j] = sum_w slab[w][j], fixed order (bitwise
// reproducible).  Block = 256 threads = 16 float4 columns x 16 row groups, each
// thread 16 independent 16-byte loads; the 16 row-group partials are combined
// in LDS in a fixed order.  Thread 0 of block 0 also advances the step control
// block (batch, adam_t): the fused step before it has read `batch`, the
// optimizer after it reads the advanced `adam_t` (kernel boundaries order it).
// W0's columns on the factored path: the gradient is the sum of the per-block
// partials of ncf_expand_grads (fact_expand_kernel), [nblk][dm][dm], user blocks
// [0, nbu) for W0[:, :dm], item blocks [nbu, nblk) for W0[:, dm:].  cols = 0: none.
struct W0Part {
    const float* p;
    int nbu, nblk, dm, cols;
};

// This thread's share (row group rg of 16) of the W0 gradient at tower column j.
__device__ __forceinline__ f4 w0_part_sum(const W0Part& P, int j, int rg) {
    f4 s = f4{0.f, 0.f, 0.f, 0.f};
    const int row = j / (2 * P.dm), col = j - row * 2 * P.dm;
    if (row >= P.dm) return s;  // alignment padding of the W0 segment
    const bool item = col >= P.dm;
    const int64_t off = (int64_t)row * P.dm + (item ? col - P.dm : col);
    const int b1 = item ? P.nblk : P.nbu;
    const int64_t bstride = (int64_t)P.dm * P.dm;
#pragma unroll 8
    for (int b = (item ? P.nbu : 0) + rg; b < b1; b += 16) {
        const f4 v = *reinterpret_cast<const f4*>(P.p + (int64_t)b * bstride + off);
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    return s;
}

// One float4 column j of the slab reduction by the 16 row groups of a 256-thread
// block (thread = column c4 of 16, row group rg): the total, for the rg == 0 threads
// (j < stride); every thread of the block must call it (one barrier).
__device__ __forceinline__ f4 slab_column_total(const float* __restrict__ slab, int j, int stride, int rows,
                                                const W0Part& wp, int rg, int c4, f4 (*part)[16]) {
    f4 s = f4{0.f, 0.f, 0.f, 0.f};
    if (j < wp.cols) {
        s = w0_part_sum(wp, j, rg);
    } else if (j < stride) {
        const float* p = slab + (int64_t)rg * stride + j;
        const int per = rows / 16;
#pragma unroll 16
        for (int r = 0; r < per; ++r) {
            const f4 v = *reinterpret_cast<const f4*>(p + (int64_t)r * 16 * stride);
            s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        }
        if (rg < rows - 16 * per) {  // rows not a multiple of 16 (the layered path's single row)
            const f4 v = *reinterpret_cast<const f4*>(p + (int64_t)per * 16 * stride);
            s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        }
    }
    part[rg][c4] = s;
    __syncthreads();
    f4 t = part[0][c4];
    if (rg == 0 && j < stride) {
#pragma unroll
        for (int q = 1; q < 16; ++q) {
            const f4 v = part[q][c4];
            t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
        }
    }
    return t;
}

__global__ __launch_bounds__(256) void reduce_slab_kernel(const float* __restrict__ slab, float* __restrict__ out,
                                                          int lo, int stride, int rows, ncf_step_ctl* ctl, W0Part wp) {
    __shared__ f4 part[16][16];
    const int c4 = threadIdx.x & 15, rg = threadIdx.x >> 4;
    const int j = lo + (blockIdx.x * 16 + c4) * 4;
    const f4 t = slab_column_total(slab, j, stride, rows, wp, rg, c4, part);
    if (rg == 0 && j < stride) *reinterpret_cast<f4*>(out + j) = t;
    if (ctl != nullptr && blockIdx.x == 0 && threadIdx.x == 0) {
        ctl->batch = ctl->batch + 1;
        ctl->adam_t = ctl->adam_t + 1;
    }
}

// ---------------------------------------------------------------------------
// Dense Adam (torch.optim.Adam, single-tensor path) + fused grad zeroing.
// Loss bookkeeping of the step: done by one thread, no cross-block protocol.
__device__ __forceinline__ void record_loss(const ncf_step_ctl* ctl, const float* grads, int64_t loss_slot,
                                            float* loss_hist, int64_t hist_len) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && loss_hist != nullptr && loss_slot >= 0 && hist_len > 0) {
        const int64_t b = ctl->batch - 1;  // ncf_reduce_slab advanced it
        loss_hist[((b % hist_len) + hist_len) % hist_len] = grads[loss_slot];
    }
}

__device__ ScCache g_sc_cache[SC_SLOTS][2];

// The step-scalar cache entry pair of a control block (see ScCache): one slot per
// (device, ctl pointer) seen, for the life of the process; null (always recompute)
// past SC_SLOTS control blocks on a device.  g_sc_cache has one copy per device, so
// its address is looked up per device -- the device of the launch's stream -- with
// that device current for the lookup.
static ScCache* sc_cache_for(const void* ctl, void* stream) {
    struct DevSlots {
        ScCache* base = nullptr;
        bool failed = false;
        std::unordered_map<const void*, int> slots;
    };
    static std::mutex mu;
    static std::unordered_map<int, DevSlots> devs;
    int dev = -1;
    if (hipStreamGetDevice((hipStream_t)stream, &dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    DevSlots& d = devs[dev];
    if (d.failed) return nullptr;
    if (d.base == nullptr) {
        int cur = -1;
        if (hipGetDevice(&cur) != hipSuccess) return nullptr;
        if (cur != dev && hipSetDevice(dev) != hipSuccess) {
            d.failed = true;
            return nullptr;
        }
        const hipError_t e = hipGetSymbolAddress((void**)&d.base, HIP_SYMBOL(g_sc_cache));
        if (cur != dev) (void)hipSetDevice(cur);
        if (e != hipSuccess) {
            d.base = nullptr;
            d.failed = true;
            return nullptr;
        }
    }
    auto it = d.slots.find(ctl);
    if (it != d.slots.end()) return d.base + 2 * it->second;
    if ((int)d.slots.size() >= SC_SLOTS) return nullptr;
    const int k = (int)d.slots.size();
    d.slots.emplace(ctl, k);
    return d.base + 2 * k;
}

__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                                   float* __restrict__ v, Ranges R, const ncf_step_ctl* ctl, double lr,
                                                   double beta1, double beta2, float eps, int64_t loss_slot,
                                                   float* loss_hist, int64_t hist_len, ScCache* scc) {
#pragma clang fp contract(off)
    __shared__ float sc[2];
    const int64_t t_step = ctl->adam_t;  // advanced by ncf_reduce_slab
    step_scalars(scc, t_step, lr, beta1, beta2, sc);
    step_scalars_ahead(scc, t_step, lr, beta1, beta2);
    __syncthreads();
    const float neg_step = sc[0], bc2s = sc[1];
    const float w1 = (float)(1.0 - beta1);
    const float b2 = (float)beta2;
    const float omb2 = (float)(1.0 - beta2);
    const int64_t total = R.prefix[R.n];
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t q0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q0 < total; q0 += 2 * stride) {
        const int64_t q1 = q0 + stride;
        const bool has1 = q1 < total;
        int which;
        const int64_t i0 = range_locate(R, q0, &which);
        const int64_t i1 = has1 ? range_locate(R, q1, &which) : i0;
        f4 g0 = *reinterpret_cast<const f4*>(g + i0), g1 = *reinterpret_cast<const f4*>(g + i1);
        f4 m0 = *reinterpret_cast<const f4*>(m + i0), m1 = *reinterpret_cast<const f4*>(m + i1);
        f4 v0 = *reinterpret_cast<const f4*>(v + i0), v1 = *reinterpret_cast<const f4*>(v + i1);
        f4 p0 = *reinterpret_cast<const f4*>(p + i0), p1 = *reinterpret_cast<const f4*>(p + i1);
        adam_f4(p0, m0, v0, g0, w1, b2, omb2, bc2s, eps, neg_step);
        *reinterpret_cast<f4*>(m + i0) = m0;
        *reinterpret_cast<f4*>(v + i0) = v0;
        *reinterpret_cast<f4*>(p + i0) = p0;
        *reinterpret_cast<f4*>(g + i0) = f4{0.f, 0.f, 0.f, 0.f};
        if (has1) {
            adam_f4(p1, m1, v1, g1, w1, b2, omb2, bc2s, eps, neg_step);
            *reinterpret_cast<f4*>(m + i1) = m1;
            *reinterpret_cast<f4*>(v + i1) = v1;
            *reinterpret_cast<f4*>(p + i1) = p1;
            *reinterpret_cast<f4*>(g + i1) = f4{0.f, 0.f, 0.f, 0.f};
        }
    }
    record_loss(ctl, g, loss_slot, loss_hist, hist_len);
}

__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ p, float* __restrict__ g, Ranges R,
                                                  const ncf_step_ctl* ctl, float lr, int64_t loss_slot, float* loss_hist,
                                                  int64_t hist_len) {
#pragma clang fp contract(off)
    const int64_t total = R.prefix[R.n];
    const float nlr = -lr;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (int64_t)gridDim.x * blockDim.x) {
        int which;
        const int64_t i = range_locate(R, q, &which);
        f4 gg = *reinterpret_cast<const f4*>(g + i);
        f4 pp = *reinterpret_cast<const f4*>(p + i);
        pp.x = pp.x + nlr * gg.x;  // param.add_(grad, alpha=-lr)
        pp.y = pp.y + nlr * gg.y;
        pp.z = pp.z + nlr * gg.z;
        pp.w = pp.w + nlr * gg.w;
        *reinterpret_cast<f4*>(p + i) = pp;
        *reinterpret_cast<f4*>(g + i) = f4{0.f, 0.f, 0.f, 0.f};
    }
    record_loss(ctl, g, loss_slot, loss_hist, hist_len);
}

// ---------------------------------------------------------------------------
// ncf_reduce_adam_step: blocks [0, nA) each reduce 64 slab columns (the order of
// reduce_slab_kernel) and apply Adam to the active ones in place; blocks
// [nA, grid) run the plain Adam over the embedding ranges RE.  t and the batch
// come from the snapshot the train step wrote; block 0 commits them.
// Block of the tower part (blockIdx.x < nA): reduce 64 slab columns (W0's from the
// expansion's partials), apply Adam to the active ones in place; the loss column
// goes to the history.  sc[0..1] = (-step size, sqrt(bias correction 2)) of step t,
// computed by thread 0 of the block after its loads are in flight.
__device__ __forceinline__ void tower_reduce_adam_block(const float* __restrict__ slab, int lo, int stride, int rows,
                                                        int64_t tb, int64_t tower_len, float* __restrict__ p,
                                                        float* __restrict__ m, float* __restrict__ v, const Ranges& R,
                                                        int64_t t_step, int64_t b_step, double lr, double beta1,
                                                        double beta2, float eps, float* loss_hist, int64_t hist_len,
                                                        const W0Part& wp, float* sc, f4 (*part)[16],
                                                        const ScCache* scc, const float* __restrict__ pre = nullptr) {
#pragma clang fp contract(off)
    const ScCache sce = sc_peek(scc, t_step);  // arrives with the first slab loads
    const float w1 = (float)(1.0 - beta1);
    const float b2 = (float)beta2;
    const float omb2 = (float)(1.0 - beta2);
    const int c4 = threadIdx.x & 15, rg = threadIdx.x >> 4;
    const int j = lo + (blockIdx.x * 16 + c4) * 4;
    // the updating threads' optimizer state, requested ahead of the slab reads
    const int64_t i = tb + j;
    const bool upd = rg == 0 && j < tower_len && in_ranges(R, i);
    f4 pp, mm, vv;
    if (upd) {
        pp = *reinterpret_cast<const f4*>(p + i);
        mm = *reinterpret_cast<const f4*>(m + i);
        vv = *reinterpret_cast<const f4*>(v + i);
    }
    f4 s = f4{0.f, 0.f, 0.f, 0.f};
    if (pre != nullptr) {  // the summed (all-reduced) tower gradient: tail of the packed buffer
        if (rg == 0 && j < stride) s = *reinterpret_cast<const f4*>(pre + j);
    } else if (j < wp.cols) {
        s = w0_part_sum(wp, j, rg);
    } else if (j < stride) {
        const float* q = slab + (int64_t)rg * stride + j;
        const int per = rows / 16;
#pragma unroll 16
        for (int r = 0; r < per; ++r) {
            const f4 x = *reinterpret_cast<const f4*>(q + (int64_t)r * 16 * stride);
            s.x += x.x; s.y += x.y; s.z += x.z; s.w += x.w;
        }
        if (rg < rows - 16 * per) {
            const f4 x = *reinterpret_cast<const f4*>(q + (int64_t)per * 16 * stride);
            s.x += x.x; s.y += x.y; s.z += x.z; s.w += x.w;
        }
    }
    part[rg][c4] = s;
    sc_resolve(sce, t_step, lr, beta1, beta2, sc);
    __syncthreads();
    const float neg_step = sc[0], bc2s = sc[1];
    if (rg == 0 && j < stride) {
        f4 gs = part[0][c4];
        if (pre == nullptr) {
#pragma unroll
            for (int q = 1; q < 16; ++q) {
                const f4 x = part[q][c4];
                gs.x += x.x; gs.y += x.y; gs.z += x.z; gs.w += x.w;
            }
        }
        if (j == tower_len) {
            if (loss_hist != nullptr && hist_len > 0) loss_hist[((b_step % hist_len) + hist_len) % hist_len] = gs.x;
        } else if (upd) {
            adam_f4(pp, mm, vv, gs, w1, b2, omb2, bc2s, eps, neg_step);
            *reinterpret_cast<f4*>(m + i) = mm;
            *reinterpret_cast<f4*>(v + i) = vv;
            *reinterpret_cast<f4*>(p + i) = pp;
        }
    }
}

// Tower block for slabs of at most 16 rows and no dW0 partials (the layered path: 1-16
// rows; the fused small-batch steps: one row per workgroup): one float4 column per
// thread, its rows summed in order (the same additions as the 16-row-group form: rows 0,
// 1, ..., then the empty groups' zeros, folded into one + 0), then Adam -- every thread
// updates, where the 16 x 16 form reduced through LDS with one thread in 16 updating
// (a stress tower of 700K floats ran 11K such blocks).
__device__ __forceinline__ void tower_col_adam(const float* __restrict__ slab, int lo, int stride, int rows,
                                               int64_t tb, int64_t tower_len, float* __restrict__ p,
                                               float* __restrict__ m, float* __restrict__ v, const Ranges& R,
                                               int64_t t_step, int64_t b_step, double lr, double beta1,
                                               double beta2, float eps, float* loss_hist, int64_t hist_len, float* sc,
                                               const ScCache* scc) {
#pragma clang fp contract(off)
    const ScCache sce = sc_peek(scc, t_step);
    const float w1 = (float)(1.0 - beta1), b2 = (float)beta2, omb2 = (float)(1.0 - beta2);
    const int j = lo + ((int)blockIdx.x * 256 + (int)threadIdx.x) * 4;
    const int64_t i = tb + j;
    const bool upd = j < tower_len && in_ranges(R, i);
    f4 pp, mm, vv;
    if (upd) {
        pp = *reinterpret_cast<const f4*>(p + i);
        mm = *reinterpret_cast<const f4*>(m + i);
        vv = *reinterpret_cast<const f4*>(v + i);
    }
    f4 x[16];
#pragma unroll
    for (int r = 0; r < 16; ++r)
        x[r] = (r < rows && j < stride) ? *reinterpret_cast<const f4*>(slab + (int64_t)r * stride + j)
                                        : f4{0.f, 0.f, 0.f, 0.f};
    f4 gs = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 16; ++r)
        if (r < rows) { gs.x += x[r].x; gs.y += x[r].y; gs.z += x[r].z; gs.w += x[r].w; }
    if (rows < 16) { gs.x += 0.f; gs.y += 0.f; gs.z += 0.f; gs.w += 0.f; }
    sc_resolve(sce, t_step, lr, beta1, beta2, sc);
    __syncthreads();
    if (j == tower_len) {
        if (loss_hist != nullptr && hist_len > 0) loss_hist[((b_step % hist_len) + hist_len) % hist_len] = gs.x;
    } else if (upd) {
        adam_f4(pp, mm, vv, gs, w1, b2, omb2, sc[1], eps, sc[0]);
        *reinterpret_cast<f4*>(m + i) = mm;
        *reinterpret_cast<f4*>(v + i) = vv;
        *reinterpret_cast<f4*>(p + i) = pp;
    }
}

__global__ __launch_bounds__(256) void reduce_adam_kernel(const float* __restrict__ slab, int lo, int stride, int rows,
                                                          int nA, int64_t tb, int64_t tower_len, float* __restrict__ p,
                                                          float* __restrict__ g, float* __restrict__ m,
                                                          float* __restrict__ v, Ranges R, Ranges RE,
                                                          ncf_step_ctl* ctl, double lr, double beta1, double beta2,
                                                          float eps, float* loss_hist, int64_t hist_len, W0Part wp,
                                                          ScCache* scc, int colmode) {
#pragma clang fp contract(off)
    __shared__ float sc[2];
    __shared__ f4 part[16][16];
    const int64_t t_step = ctl->snap_t;
    const int64_t b_step = ctl->snap_batch;
    step_scalars_ahead(scc, t_step, lr, beta1, beta2);
    if ((int)blockIdx.x < nA && colmode) {
        tower_col_adam(slab, lo, stride, rows, tb, tower_len, p, m, v, R, t_step, b_step, lr, beta1, beta2, eps,
                       loss_hist, hist_len, sc, scc);
    } else if ((int)blockIdx.x < nA) {
        tower_reduce_adam_block(slab, lo, stride, rows, tb, tower_len, p, m, v, R, t_step, b_step, lr, beta1, beta2,
                                eps, loss_hist, hist_len, wp, sc, part, scc);
    } else {
        const float w1 = (float)(1.0 - beta1);
        const float b2 = (float)beta2;
        const float omb2 = (float)(1.0 - beta2);
        const int64_t total = RE.prefix[RE.n];
        const int64_t nthr = (int64_t)(gridDim.x - nA) * blockDim.x;
        int64_t q = (int64_t)(blockIdx.x - nA) * blockDim.x + threadIdx.x;
        int64_t i = 0;
        f4 gg, mm, vv, pp;
        auto load = [&]() {
            int which;
            i = range_locate(RE, q, &which);
            gg = *reinterpret_cast<const f4*>(g + i);
            mm = *reinterpret_cast<const f4*>(m + i);
            vv = *reinterpret_cast<const f4*>(v + i);
            pp = *reinterpret_cast<const f4*>(p + i);
        };
        const ScCache sce = sc_peek(scc, t_step);
        if (q < total) load();  // the first element's loads fly while thread 0 resolves the scalars
        sc_resolve(sce, t_step, lr, beta1, beta2, sc);
        __syncthreads();
        const float neg_step = sc[0], bc2s = sc[1];
        while (q < total) {
            adam_f4(pp, mm, vv, gg, w1, b2, omb2, bc2s, eps, neg_step);
            *reinterpret_cast<f4*>(m + i) = mm;
            *reinterpret_cast<f4*>(v + i) = vv;
            *reinterpret_cast<f4*>(p + i) = pp;
            *reinterpret_cast<f4*>(g + i) = f4{0.f, 0.f, 0.f, 0.f};
            q += nthr;
            if (q < total) load();
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // no other block of this launch reads these two
        ctl->adam_t = t_step;
        ctl->batch = b_step + 1;
    }
}

// ---------------------------------------------------------------------------
// Deferred ("catch-up") Adam over the embedding tables -- exactly the dense
// torch.optim.Adam of train_neumf.py:90,115, moving only the rows that need it.
// For a row whose gradient is exactly zero, Adam step s is a fixed per-element fp32
// sequence with step-s scalars (adam_f4 with g = 0), so the steps a row sat out
// can be replayed, in order, when it is next needed, with a bitwise-identical
// result.  last[row] (users [0, U), items [U, U + I)) is the last step applied to
// the row; ring[s % ring_n] the step-s scalars, written by step s's launch.
//
// ncf_batch_touched builds, per global batch b of the epoch stream and per side
// (users, items), three disjoint sorted lists (segments k = 2 * list + side):
//   A_b = the rows batch b touches            (their gradient is in grads)
//   B_b = the rows batch b + 1 touches, not A_b (the next forward reads them);
//         on the epoch's last batch: every row not in A_b
//   C_b = the rows of slice (b % span) of the side's ids, in neither
//         (rolling catch-up: no row falls more than `span` steps behind)
// Step t's launch brings every listed row from last + 1 through t: the replays
// with g = 0, then step t with its gradient (A rows; zero for B and C rows, whose
// gradient is not read).  A rows sat out nothing (they were in A or B the step
// before), B and C rows at most `span` steps, whose scalars are staged in LDS.
// The lists are disjoint, so no row is claimed twice: no atomics.  Each wave
// takes whole rows -- floor(64 / W) rows of W float4 side by side, or one row
// looped over 64 lanes -- so a row's lanes read last before any of them writes it.
// Flush: every row through t = ctl->adam_t (all gradients zero by then).
struct LazyArgs {
    float* p;
    float* g;
    float* m;
    float* v;
    int64_t off[4];  // Ug, Ig, Um, Im flat offsets (< 0: table inactive)
    int w4[4];       // float4s per row of each table
    int U, I;
    const int64_t* seg;  // ncf_batch_touched: [nb * 6 + 1] list offsets (segment k of batch b: 6b + k)
    const int32_t* ids;  // the lists' ids
    int64_t nb;
    int32_t* last;  // [U + I]
    float* ring;    // [ring_n][2]
    int64_t ring_n;
    // packed mode (data parallel, ncf_touched_pack): A_b's summed gradients at
    // packed[k * wrow[side] + ...] (k = position in A_b's list, users first)
    const float* packed;
    int64_t pk_items;  // float offset of the item rows
    int64_t pk_tail;   // float offset of the tower gradient
    int wrow[2];       // floats per packed user / item row
};

constexpr int LZ_WIN = 512;  // step scalars of the last LZ_WIN steps staged in LDS per block

// The block's copy of the step scalars ring[s] for s in [t - LZ_WIN, t).
__device__ __forceinline__ void stage_ring(const LazyArgs& a, int64_t t, float2* win) {
    for (int k = threadIdx.x; k < LZ_WIN; k += blockDim.x) {
        const int64_t s = t - LZ_WIN + k;
        win[k] = s >= 1 ? reinterpret_cast<const float2*>(a.ring)[s % a.ring_n] : float2{0.f, 0.f};
    }
}

__host__ __device__ __forceinline__ int lz_row_w4(const LazyArgs& a, int side) {
    return (a.off[side] >= 0 ? a.w4[side] : 0) + (a.off[side + 2] >= 0 ? a.w4[side + 2] : 0);
}

// flat index of float4 slot k of a row (g table first, then m table)
__device__ __forceinline__ int64_t lz_elem(const LazyArgs& a, int side, int id, int k) {
    const int wa = a.off[side] >= 0 ? a.w4[side] : 0;
    return k < wa ? a.off[side] + ((int64_t)id * a.w4[side] + k) * 4
                  : a.off[side + 2] + ((int64_t)id * a.w4[side + 2] + (k - wa)) * 4;
}

// Bring one float4 of a row from `old` + 1 through t (grad: step t's gradient, or
// null for zero) and store it.
__device__ __forceinline__ void lz_update(const LazyArgs& a, int64_t e, int old, int64_t t, const float* grad,
                                          bool clear_g, float neg_t, float bc2s_t, float w1, float b2, float omb2,
                                          float eps, const float2* win) {
#pragma clang fp contract(off)
    const f4 zero = f4{0.f, 0.f, 0.f, 0.f};
    f4 pp = *reinterpret_cast<const f4*>(a.p + e);
    f4 mm = *reinterpret_cast<const f4*>(a.m + e);
    f4 vv = *reinterpret_cast<const f4*>(a.v + e);
    const f4 gg = grad != nullptr ? *reinterpret_cast<const f4*>(grad) : zero;
    for (int s = old + 1; s < (int)t; ++s) {  // the steps this row sat out: g = 0
        const int64_t kw = s - (t - LZ_WIN);
        const float2 sc = kw >= 0 ? win[kw] : reinterpret_cast<const float2*>(a.ring)[s % a.ring_n];
        adam_f4(pp, mm, vv, zero, w1, b2, omb2, sc.y, eps, sc.x);
    }
    adam_f4(pp, mm, vv, gg, w1, b2, omb2, bc2s_t, eps, neg_t);
    *reinterpret_cast<f4*>(a.m + e) = mm;
    *reinterpret_cast<f4*>(a.v + e) = vv;
    *reinterpret_cast<f4*>(a.p + e) = pp;
    if (clear_g) *reinterpret_cast<f4*>(a.g + e) = zero;
}

// The embedding rows of step t, batch b (flush: every row), one wave task per
// group of rows; tasks per segment: ceil(rows / rows per wave).
__device__ __forceinline__ void lazy_rows(const LazyArgs& a, int64_t t, int64_t b, bool flush, float neg_t,
                                          float bc2s_t, float w1, float b2, float omb2, float eps,
                                          const float2* win, int64_t wave, int64_t nwaves) {
    const int lane = threadIdx.x & 63;
    int64_t n[6], first[6];  // the six segments (flush: every user, every item as segments 2, 3)
    for (int k = 0; k < 6; ++k) {
        if (flush) {
            n[k] = k == 2 ? a.U : (k == 3 ? a.I : 0);
            first[k] = 0;
        } else {
            first[k] = a.seg[6 * b + k];
            n[k] = a.seg[6 * b + k + 1] - first[k];
        }
    }
    int W[2], per[2];
    for (int sd = 0; sd < 2; ++sd) {
        W[sd] = lz_row_w4(a, sd);
        per[sd] = W[sd] == 0 ? 0 : (W[sd] <= 64 ? 64 / W[sd] : 1);
    }
    int64_t tasks[6], tsum = 0;
    for (int k = 0; k < 6; ++k) {
        const int sd = k & 1;
        tasks[k] = per[sd] == 0 ? 0 : (n[k] + per[sd] - 1) / per[sd];
        tsum += tasks[k];
    }
    for (int64_t task = wave; task < tsum; task += nwaves) {
        int k = 0;
        int64_t q = task;
        while (q >= tasks[k]) q -= tasks[k++];
        const int sd = k & 1;
        const int w = W[sd];
        const int r = w <= 64 ? lane / w : 0;  // this lane's row of the task
        const int64_t item = q * per[sd] + r;
        if (r >= per[sd] || item >= n[k]) continue;
        const int id = flush ? (int)item : a.ids[first[k] + item];
        const int64_t slot = sd ? a.U + id : id;
        const int old = a.last[slot];
        const bool is_a = k < 2;  // A rows carry step t's gradient
        if (old < (int)t) {
            const int k0 = w <= 64 ? lane - r * w : lane, kstep = w <= 64 ? w : 64;
            for (int kk = k0; kk < w; kk += kstep) {
                const int64_t e = lz_elem(a, sd, id, kk);
                const float* grad = nullptr;
                if (is_a)
                    grad = a.packed != nullptr
                               ? a.packed + (sd ? a.pk_items + item * a.wrow[1] : item * a.wrow[0]) + 4 * kk
                               : a.g + e;
                lz_update(a, e, old, t, grad, is_a && a.packed == nullptr, neg_t, bc2s_t, w1, b2, omb2, eps, win);
            }
            // every lane of the row has read `last` (one wave, in program order): publish t
            if (lane == (w <= 64 ? r * w : 0)) a.last[slot] = (int)t;
        }
    }
}

__global__ __launch_bounds__(256) void lazy_adam_kernel(const float* __restrict__ slab, int lo, int stride, int rows,
                                                        int nA, int64_t tb, int64_t tower_len, Ranges R,
                                                        ncf_step_ctl* ctl, double lr, double beta1, double beta2,
                                                        float eps, float* loss_hist, int64_t hist_len, W0Part wp,
                                                        LazyArgs a, ScCache* scc) {
#pragma clang fp contract(off)
    __shared__ float sc[2];
    __shared__ f4 part[16][16];
    __shared__ float2 win[LZ_WIN];
    const int64_t t_step = ctl->snap_t;
    const int64_t b_step = ctl->snap_batch;
    step_scalars_ahead(scc, t_step, lr, beta1, beta2);
    if ((int)blockIdx.x < nA) {
        tower_reduce_adam_block(slab, lo, stride, rows, tb, tower_len, a.p, a.m, a.v, R, t_step, b_step, lr, beta1,
                                beta2, eps, loss_hist, hist_len, wp, sc, part, scc,
                                a.packed != nullptr ? a.packed + a.pk_tail : nullptr);
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            a.ring[2 * (t_step % a.ring_n)] = sc[0];
            a.ring[2 * (t_step % a.ring_n) + 1] = sc[1];
        }
    } else {
        const ScCache sce = sc_peek(scc, t_step);
        stage_ring(a, t_step, win);
        sc_resolve(sce, t_step, lr, beta1, beta2, sc);
        __syncthreads();
        const int64_t b = ((b_step % a.nb) + a.nb) % a.nb;
        const int64_t wpb = blockDim.x >> 6;
        lazy_rows(a, t_step, b, false, sc[0], sc[1], (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), eps, win,
                  (int64_t)(blockIdx.x - nA) * wpb + (threadIdx.x >> 6), (int64_t)(gridDim.x - nA) * wpb);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        ctl->adam_t = t_step;
        ctl->batch = b_step + 1;
    }
}

__global__ __launch_bounds__(256) void lazy_flush_kernel(const ncf_step_ctl* ctl, double beta1, double beta2, float eps,
                                                         LazyArgs a) {
    const int64_t t = ctl->adam_t;
    if (t <= 0) return;
    __shared__ float2 win[LZ_WIN];
    stage_ring(a, t, win);
    __syncthreads();
    const float* sc = a.ring + 2 * (t % a.ring_n);
    const int64_t wpb = blockDim.x >> 6;
    lazy_rows(a, t, 0, true, sc[0], sc[1], (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), eps, win,
              (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6), (int64_t)gridDim.x * wpb);
}

// ---------------------------------------------------------------------------
// ncf_batch_touched: per (global batch b, side) block, LDS bitmaps of the side's ids
// in batch b and in batch b + 1; the three lists A, B, C of lazy_rows' comment.
// Pass 0 counts them into seg[6 b + k + 1]; a one-block scan turns the counts into
// offsets; pass 1 writes the ids in order (block prefix scans of popcounts).
constexpr int BT_THREADS = 1024;

__device__ __forceinline__ int bt_block_scan(int c, int* wsum, int* total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int incl = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
    }
    __syncthreads();
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    int base = 0, all = 0;
    for (int q = 0; q < BT_THREADS / 64; ++q) {
        if (q < wv) base += wsum[q];
        all += wsum[q];
    }
    *total = all;
    return base + incl - c;
}

__global__ __launch_bounds__(BT_THREADS) void batch_touched_kernel(const uint64_t* __restrict__ rows, int64_t n,
                                                                   int64_t B, int U, int I, int64_t nb, int span,
                                                                   int pass, int64_t* __restrict__ seg,
                                                                   int32_t* __restrict__ ids) {
    extern __shared__ uint32_t bits[];  // [cur | nxt], nw words each
    __shared__ int wsum[BT_THREADS / 64];
    const int64_t b = blockIdx.x >> 1;
    const int side = blockIdx.x & 1;
    const int N = side ? I : U;
    const int nw = (N + 31) / 32;
    uint32_t* cur = bits;
    uint32_t* nxt = bits + nw;
    const bool last_b = b + 1 >= nb;
    for (int k = threadIdx.x; k < 2 * nw; k += BT_THREADS) bits[k] = 0u;
    __syncthreads();
    for (int h = 0; h < (last_b ? 1 : 2); ++h) {
        uint32_t* bm = h ? nxt : cur;
        const int64_t r0 = (b + h) * B, r1 = r0 + B < n ? r0 + B : n;
        for (int64_t r = r0 + threadIdx.x; r < r1; r += BT_THREADS) {
            const uint64_t row = rows[r];
            const uint32_t u = (uint32_t)row;
            if (u == 0xffffffffu) continue;  // padding row
            const uint32_t id = side ? (uint32_t)((row >> 32) & 0x7fffffffu) : u;
            if (id < (uint32_t)N) atomicOr(&bm[id >> 5], 1u << (id & 31));
        }
    }
    __syncthreads();
    // slice (b % span) of the ids: [lo, hi)
    const int64_t sl = span > 0 ? b % span : 0;
    const int lo = span > 0 ? (int)(sl * N / span) : 0, hi = span > 0 ? (int)((sl + 1) * N / span) : 0;
    const int per = (nw + BT_THREADS - 1) / BT_THREADS;
    const int w0 = threadIdx.x * per, w1 = w0 + per < nw ? w0 + per : nw;
    auto slice_mask = [&](int w) -> uint32_t {  // bits of word w inside [lo, hi)
        const int a0 = w * 32, a1 = a0 + 32;
        if (last_b || a1 <= lo || a0 >= hi) return 0u;
        uint32_t m = 0xffffffffu;
        if (lo > a0) m &= 0xffffffffu << (lo - a0);
        if (hi < a1) m &= 0xffffffffu >> (a1 - hi);
        return m;
    };
    auto tail_mask = [&](int w) -> uint32_t {  // ids < N
        const int a1 = w * 32 + 32;
        return a1 <= N ? 0xffffffffu : (0xffffffffu >> (a1 - N));
    };
    for (int list = 0; list < 3; ++list) {
        auto word = [&](int w) -> uint32_t {
            const uint32_t c = cur[w], x = nxt[w];
            if (list == 0) return c;
            if (list == 1) return last_b ? (~c & tail_mask(w)) : (x & ~c);
            return slice_mask(w) & ~c & ~x;
        };
        int c = 0;
        for (int w = w0; w < w1; ++w) c += __popc(word(w));
        int total;
        const int pos0 = bt_block_scan(c, wsum, &total);
        const int64_t k = 6 * b + 2 * list + side;
        if (pass == 0) {
            if (threadIdx.x == 0) seg[k + 1] = total;
        } else {
            int32_t* dst = ids + seg[k];
            int pos = pos0;
            for (int w = w0; w < w1; ++w) {
                uint32_t x = word(w);
                while (x) {
                    const int q = __ffs(x) - 1;
                    x &= x - 1;
                    dst[pos++] = w * 32 + q;
                }
            }
        }
    }
}

// counts (seg[1 .. m]) -> offsets (seg[0 .. m]), one block
__global__ __launch_bounds__(BT_THREADS) void touched_scan_kernel(int64_t* __restrict__ seg, int64_t m) {
    __shared__ int64_t wsum[BT_THREADS / 64];
    const int per = (int)((m + BT_THREADS - 1) / BT_THREADS);
    const int64_t i0 = (int64_t)threadIdx.x * per, i1 = i0 + per < m ? i0 + per : m;
    int64_t c = 0;
    for (int64_t i = i0; i < i1; ++i) c += seg[i + 1];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int64_t incl = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int64_t y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    int64_t base = 0;
    for (int q = 0; q < wv; ++q) base += wsum[q];
    int64_t run = base + incl - c;
    __syncthreads();
    for (int64_t i = i0; i < i1; ++i) {
        const int64_t v = seg[i + 1];
        seg[i + 1] = run + v;  // inclusive: seg[i + 1] = offset of segment i + 1
        run += v;
    }
    if (threadIdx.x == 0) seg[0] = 0;
}

// ncf_touched_pack: this rank's gradient of batch b's A rows (users, then items;
// each row its active tables' floats, g table first) into packed slots in list
// order, those rows of grads cleared; slots past the batch's count are zeroed so
// the all-reduce adds nothing stale.  One wave task per group of rows.
__global__ __launch_bounds__(256) void touched_pack_kernel(const ncf_step_ctl* __restrict__ ctl, LazyArgs a, int64_t su,
                                                           int64_t si, float* __restrict__ packed) {
    const int lane = threadIdx.x & 63;
    const int64_t b = ((ctl->snap_batch % a.nb) + a.nb) % a.nb;
    const int64_t nu = a.seg[6 * b + 1] - a.seg[6 * b], ni = a.seg[6 * b + 2] - a.seg[6 * b + 1];
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const f4 zero = f4{0.f, 0.f, 0.f, 0.f};
    int W[2], per[2];
    for (int sd = 0; sd < 2; ++sd) {
        W[sd] = lz_row_w4(a, sd);
        per[sd] = W[sd] == 0 ? 0 : (W[sd] <= 64 ? 64 / W[sd] : 1);
    }
    const int64_t tu = per[0] ? (su + per[0] - 1) / per[0] : 0, ti = per[1] ? (si + per[1] - 1) / per[1] : 0;
    for (int64_t task = wave; task < tu + ti; task += nwaves) {
        const int sd = task < tu ? 0 : 1;
        const int64_t q = sd ? task - tu : task;
        const int w = W[sd];
        const int r = w <= 64 ? lane / w : 0;
        const int64_t item = q * per[sd] + r;
        if (r >= per[sd] || item >= (sd ? si : su)) continue;
        float* dst = packed + (sd ? a.pk_items + item * a.wrow[1] : item * a.wrow[0]);
        const int k0 = w <= 64 ? lane - r * w : lane, kstep = w <= 64 ? w : 64;
        if (item >= (sd ? ni : nu)) {
            for (int kk = k0; kk < w; kk += kstep) *reinterpret_cast<f4*>(dst + 4 * kk) = zero;
            continue;
        }
        const int id = a.ids[a.seg[6 * b + sd] + item];
        for (int kk = k0; kk < w; kk += kstep) {
            const int64_t e = lz_elem(a, sd, id, kk);
            *reinterpret_cast<f4*>(dst + 4 * kk) = *reinterpret_cast<const f4*>(a.g + e);
            *reinterpret_cast<f4*>(a.g + e) = zero;
        }
    }
}

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void zero_f32_kernel(f4* __restrict__ p, int64_t n4) {
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += (int64_t)gridDim.x * blockDim.x)
        p[q] = f4{0.f, 0.f, 0.f, 0.f};
}

// Packed rows (include/ncf_hip.h NCF_ROW_PACK): u | item << 32 | label << 63.
__device__ __forceinline__ int row_item(uint64_t r) { return (int)((r >> 32) & 0x7fffffffu); }

__global__ __launch_bounds__(256) void pack_rows_kernel(const int32_t* __restrict__ u, const int32_t* __restrict__ it,
                                                        const float* __restrict__ y, int64_t n, uint64_t* __restrict__ out) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x)
        out[k] = NCF_ROW_PACK(u[k], it[k], y ? y[k] : 0.f);
}

__global__ __launch_bounds__(256) void gather_epoch_kernel(const uint64_t* __restrict__ rows,
                                                           const int64_t* __restrict__ perm, int64_t n,
                                                           uint64_t* __restrict__ out) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x)
        out[k] = rows[perm[k]];
}

// ---------------------------------------------------------------------------
// Epoch preparation (ncf_prepare_epoch).  Global batch b is rows perm[b*B ..
// b*B+cnt) of the unshuffled stream (DataLoader shuffle=True membership); it is
// written back grouped by item.  Three launches, all HBM/L2-bound byte work:
//   1. shuffle_hist: shuf[j] = rows[perm[j]] (one random 8-byte gather per row,
//      coalesced write) and hist[b][item]++ (global atomics, no return).
//   2. scan_parts: per batch, hist -> exclusive item offsets in place, and the
//      batch is cut into P parts of ~cnt/P rows at item boundaries: part q owns
//      the items whose start offset s satisfies floor(s*P/cnt) == q, i.e. a
//      contiguous item range [I_q, I_q+1) and output region [R_q, R_q+1).
//   3. sort_part: one workgroup per (batch, part) streams the batch's shuffled
//      rows (L2-resident: the P parts of a batch run on one XCD), keeps those of
//      its items, places them by LDS atomics on the item offsets into an LDS
//      staging buffer and writes its region out contiguously.  Regions or item
//      ranges too large for LDS fall back to global offsets / direct writes.
constexpr int SH_THREADS = 256, SH_UNROLL = 8;
constexpr int SCAN_THREADS = 1024;
constexpr int SORT_THREADS = 1024, SORT_UNROLL = 8;
constexpr int STAGE_ROWS = 16384, ITEM_CAP = 6144;
constexpr int64_t SORT_LDS = (int64_t)STAGE_ROWS * 8 + (int64_t)ITEM_CAP * 4;
constexpr int PART_ROWS = 8192;  // nominal rows per part
constexpr int64_t PREP_GROUP_MIN = 4096;  // smaller global batches are shuffled, not grouped

__global__ __launch_bounds__(SH_THREADS) void shuffle_hist_kernel(const uint64_t* __restrict__ rows,
                                                                  const int64_t* __restrict__ perm, int64_t n,
                                                                  int64_t B, int item_num, uint64_t* __restrict__ shuf,
                                                                  int* __restrict__ hist) {
    const int64_t j0 = (int64_t)blockIdx.x * (SH_THREADS * SH_UNROLL) + threadIdx.x;
    int64_t src[SH_UNROLL];
    uint64_t r[SH_UNROLL];
#pragma unroll
    for (int k = 0; k < SH_UNROLL; ++k) {
        const int64_t j = j0 + k * SH_THREADS;
        const int64_t s = j < n ? perm[j] : 0;
        src[k] = s < 0 ? 0 : (s >= n ? n - 1 : s);
    }
#pragma unroll
    for (int k = 0; k < SH_UNROLL; ++k) r[k] = rows[src[k]];
#pragma unroll
    for (int k = 0; k < SH_UNROLL; ++k) {
        const int64_t j = j0 + k * SH_THREADS;
        if (j < n) {
            shuf[j] = r[k];
            atomicAdd(hist + (j / B) * item_num + min(row_item(r[k]), item_num - 1), 1);
        }
    }
}

// LDS-privatised variant for large batches: block (b, c) covers rows
// [b*B + c*SH_CHUNK, ...) of batch b only, counts its items in LDS and adds each
// non-zero bin to hist once -- no same-address atomic chains on hot items.
constexpr int SH2_THREADS = 1024, SH2_UNROLL = 8, SH_CHUNK = 16384;
constexpr int SH2_MAX_ITEMS = 32768;
__global__ __launch_bounds__(SH2_THREADS) void shuffle_hist_lds_kernel(const uint64_t* __restrict__ rows,
                                                                      const int64_t* __restrict__ perm, int64_t n,
                                                                      int64_t B, int item_num, int chunks,
                                                                      uint64_t* __restrict__ shuf,
                                                                      int* __restrict__ hist) {
    extern __shared__ int lh[];  // [item_num]
    const int tid = threadIdx.x;
    const int64_t b = blockIdx.x / chunks;
    const int c = blockIdx.x - (int)(b * chunks);
    const int64_t b0 = b * B;
    const int cnt = (int)((n - b0) < B ? (n - b0) : B);
    const int r0 = c * SH_CHUNK, r1 = min(cnt, r0 + SH_CHUNK);
    if (r0 >= r1) return;  // block-uniform
    for (int i = tid; i < item_num; i += SH2_THREADS) lh[i] = 0;
    __syncthreads();
    for (int q0 = r0; q0 < r1; q0 += SH2_UNROLL * SH2_THREADS) {
        int64_t src[SH2_UNROLL];
        uint64_t r[SH2_UNROLL];
#pragma unroll
        for (int k = 0; k < SH2_UNROLL; ++k) {
            const int q = q0 + k * SH2_THREADS + tid;
            const int64_t s = q < r1 ? perm[b0 + q] : 0;
            src[k] = s < 0 ? 0 : (s >= n ? n - 1 : s);
        }
#pragma unroll
        for (int k = 0; k < SH2_UNROLL; ++k) r[k] = rows[src[k]];
#pragma unroll
        for (int k = 0; k < SH2_UNROLL; ++k) {
            const int q = q0 + k * SH2_THREADS + tid;
            if (q < r1) {
                shuf[b0 + q] = r[k];
                atomicAdd(&lh[min(row_item(r[k]), item_num - 1)], 1);
            }
        }
    }
    __syncthreads();
    int* h = hist + b * item_num;
    for (int i = tid; i < item_num; i += SH2_THREADS) {
        const int v = lh[i];
        if (v) atomicAdd(h + i, v);
    }
}

__global__ __launch_bounds__(SCAN_THREADS) void scan_parts_kernel(int* __restrict__ hist, int64_t n, int64_t B,
                                                                  int item_num, int P, int* __restrict__ parts) {
    __shared__ int wpart[SCAN_THREADS / 64];
    const int tid = threadIdx.x;
    const int64_t b = blockIdx.x;
    const int64_t b0 = b * B;
    const int cnt = (int)((n - b0) < B ? (n - b0) : B);
    int* h = hist + b * item_num;
    int* pb = parts + b * (P + 1) * 2;
    const int per = (item_num + SCAN_THREADS - 1) / SCAN_THREADS;
    const int i0 = min(item_num, tid * per), i1 = min(item_num, i0 + per);
    int tot = 0;
    for (int i = i0; i < i1; ++i) tot += h[i];
    const int lane = tid & 63, wv = tid >> 6;
    int incl = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wpart[wv] = incl;
    __syncthreads();
    if (tid == 0) {
        int acc = 0;
        for (int q = 0; q < SCAN_THREADS / 64; ++q) {
            const int v = wpart[q];
            wpart[q] = acc;
            acc += v;
        }
        pb[0] = 0;
        pb[1] = 0;
    }
    __syncthreads();
    int s = wpart[wv] + incl - tot;
    // first part whose threshold T_q = ceil(q*cnt/P) lies above s
    int q = (int)((int64_t)s * P / cnt) + 1;
    for (int i = i0; i < i1; ++i) {
        const int c = h[i];
        h[i] = s;
        const int sn = s + c;
        while (q <= P) {
            const int T = (int)(((int64_t)q * cnt + P - 1) / P);
            if (T > sn) break;
            pb[2 * q] = i + 1;  // items [.., i] end before part q; item i + 1 starts it
            pb[2 * q + 1] = sn;
            ++q;
        }
        s = sn;
    }
}

// Canonical order of a batch's grouped rows (ncf_prepare_epoch2, NCF_PREP_CANONICAL):
// the LDS-atomic placement leaves the rows of one item in arrival order, which
// differs from run to run; data parallelism needs every rank's stream identical
// (rank r takes rows [r per, (r + 1) per) of each global batch), so with the flag
// each part is sorted by (item, user, label) -- a total order on the rows' values,
// identical duplicates being interchangeable -- which keeps the item grouping.
__device__ __forceinline__ uint64_t canon_key(uint64_t r) {
    return (((r >> 32) & 0x7fffffffull) << 33) | ((r & 0xffffffffull) << 1) | (r >> 63);
}
// Ascending sort of a[0 .. n) in place by canon_key, one workgroup (any n): the
// bitonic network in its all-ascending form (each merge stage starts with a flip
// comparison i <-> i ^ (k - 1), then half-cleaners i <-> i + j), so positions past
// n act as +infinity and are simply skipped.
template <int NT, class T>
__device__ void canon_sort(T* a, int n) {
    int n2 = 1;
    while (n2 < n) n2 <<= 1;
    for (int k = 2; k <= n2; k <<= 1) {
        for (int j = k >> 1; j >= 1; j >>= 1) {
            for (int q = threadIdx.x; q < (n2 >> 1); q += NT) {
                const int i = (q / j) * 2 * j + (q % j);
                const int p = j == (k >> 1) ? (i ^ (k - 1)) : i + j;  // flip, then half-cleaners
                if (p < n) {
                    const uint64_t x = a[i], y = a[p];
                    if (canon_key(x) > canon_key(y)) {
                        a[i] = y;
                        a[p] = x;
                    }
                }
            }
            __syncthreads();
        }
    }
}

__global__ __launch_bounds__(SORT_THREADS) void sort_part_kernel(const uint64_t* __restrict__ shuf,
                                                                 int* __restrict__ hist, const int* __restrict__ parts,
                                                                 int64_t n, int64_t B, int item_num, int P, int64_t nb,
                                                                 uint64_t* __restrict__ out, int canon) {
    extern __shared__ uint64_t stg[];                       // [STAGE_ROWS]
    int* loff = reinterpret_cast<int*>(stg + STAGE_ROWS);  // [ITEM_CAP]
    const int tid = threadIdx.x;
    const int x = blockIdx.x;
    int64_t b;
    int o;
    if (P >= 8) {  // the P parts of a batch share one XCD (blocks are dealt round-robin to the 8 XCDs)
        const int xcd = x & 7, k = x >> 3;
        b = (int64_t)(k / P) * 8 + xcd;
        o = k % P;
    } else {
        b = x / P;
        o = x % P;
    }
    if (b >= nb) return;
    const int64_t b0 = b * B;
    const int cnt = (int)((n - b0) < B ? (n - b0) : B);
    const int* pb = parts + b * (P + 1) * 2;
    const int ilo = pb[2 * o], rlo = pb[2 * o + 1], ihi = pb[2 * o + 2], rhi = pb[2 * o + 3];
    const int nrows = rhi - rlo, nit = ihi - ilo;
    if (nrows <= 0) return;  // block-uniform
    int* h = hist + b * item_num;
    const bool stage = nrows <= STAGE_ROWS, local = nit <= ITEM_CAP;
    if (local)
        for (int e = tid; e < nit; e += SORT_THREADS) loff[e] = h[ilo + e] - rlo;
    __syncthreads();
    const uint64_t* sb = shuf + b0;
    uint64_t* ob = out + b0 + rlo;
    for (int j0 = 0; j0 < cnt; j0 += SORT_UNROLL * SORT_THREADS) {
        uint64_t r[SORT_UNROLL];
#pragma unroll
        for (int k = 0; k < SORT_UNROLL; ++k) {
            const int j = j0 + k * SORT_THREADS + tid;
            r[k] = sb[j < cnt ? j : 0];
        }
#pragma unroll
        for (int k = 0; k < SORT_UNROLL; ++k) {
            const int j = j0 + k * SORT_THREADS + tid;
            const int it = min(row_item(r[k]), item_num - 1);
            if (j < cnt && it >= ilo && it < ihi) {
                const int pos = local ? atomicAdd(&loff[it - ilo], 1) : atomicAdd(&h[it], 1) - rlo;
                if (stage)
                    stg[pos] = r[k];
                else
                    ob[pos] = r[k];
            }
        }
    }
    if (stage) {
        __syncthreads();
        if (canon) canon_sort<SORT_THREADS>(stg, nrows);
        for (int e = tid; e < nrows; e += SORT_THREADS) ob[e] = stg[e];
    } else if (canon) {  // the region in place in global memory (a part beyond the LDS stage)
        __threadfence_block();
        __syncthreads();
        canon_sort<SORT_THREADS>(ob, nrows);
    }
}

// User order (ncf_user_order): one workgroup per rank slice of a batch, counting
// sort by user in LDS (histogram, exclusive scan, placement by LDS atomics).  The
// slice's rows are read twice (the second pass from L2); the entries are written
// inside the slice's own 8-byte-per-row window.
constexpr int UO_THREADS = 1024, UO_UNROLL = 16;
constexpr int UO_MAX_USERS = 32767;
__device__ __forceinline__ int uo_bin(uint64_t rw, int user_num) {
    const int u = (int)(uint32_t)rw;
    return (u < 0 || u >= user_num) ? user_num : u;  // padding rows (-1) last
}
__global__ __launch_bounds__(UO_THREADS) void user_order_kernel(const uint64_t* __restrict__ rows, int64_t n,
                                                                int64_t B, int world, int user_num,
                                                                int64_t* __restrict__ order) {
    extern __shared__ int uh[];  // [user_num + 1]
    __shared__ int wsum[UO_THREADS / 64];
    const int tid = threadIdx.x;
    const int64_t b = blockIdx.x / world;
    const int r = (int)(blockIdx.x - b * world);
    const int64_t b0 = b * B;
    if (b0 >= n) return;  // block-uniform
    const int64_t cnt = (n - b0) < B ? (n - b0) : B;
    const int64_t per = (cnt + world - 1) / world;
    const int64_t lo = (int64_t)r * per;
    if (lo >= cnt) return;
    const int len = (int)((cnt - lo) < per ? (cnt - lo) : per);
    const uint64_t* rb = rows + b0 + lo;
    int64_t* ob = order + b0 + lo;
    int32_t* ib = reinterpret_cast<int32_t*>(order + n) + b0 + lo;  // inverse: row offset -> position
    const int nbin = user_num + 1;
    for (int i = tid; i < nbin; i += UO_THREADS) uh[i] = 0;
    __syncthreads();
    // rows in batches of UO_UNROLL per thread, loads issued together ahead of the LDS
    // atomics (one dependent load -> atomic per row was latency-bound: 160 us/epoch)
    for (int k0 = 0; k0 < len; k0 += UO_THREADS * UO_UNROLL) {
        int bins[UO_UNROLL];
#pragma unroll
        for (int q = 0; q < UO_UNROLL; ++q) {
            const int k = k0 + q * UO_THREADS + tid;
            bins[q] = k < len ? uo_bin(rb[k], user_num) : -1;
        }
#pragma unroll
        for (int q = 0; q < UO_UNROLL; ++q)
            if (bins[q] >= 0) atomicAdd(&uh[bins[q]], 1);
    }
    __syncthreads();
    const int chunk = (nbin + UO_THREADS - 1) / UO_THREADS;
    const int i0 = min(nbin, tid * chunk), i1 = min(nbin, i0 + chunk);
    int tot = 0;
    for (int i = i0; i < i1; ++i) tot += uh[i];
    const int lane = tid & 63, wv = tid >> 6;
    int incl = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    if (tid == 0) {
        int acc = 0;
        for (int q = 0; q < UO_THREADS / 64; ++q) {
            const int v = wsum[q];
            wsum[q] = acc;
            acc += v;
        }
    }
    __syncthreads();
    int s = wsum[wv] + incl - tot;
    for (int i = i0; i < i1; ++i) {
        const int c = uh[i];
        uh[i] = s;
        s += c;
    }
    __syncthreads();
    for (int k0 = 0; k0 < len; k0 += UO_THREADS * UO_UNROLL) {
        int bins[UO_UNROLL];
#pragma unroll
        for (int q = 0; q < UO_UNROLL; ++q) {
            const int k = k0 + q * UO_THREADS + tid;
            bins[q] = k < len ? uo_bin(rb[k], user_num) : -1;
        }
#pragma unroll
        for (int q = 0; q < UO_UNROLL; ++q) {
            const int k = k0 + q * UO_THREADS + tid;
            if (bins[q] >= 0) {
                const int pos = atomicAdd(&uh[bins[q]], 1);
                ob[pos] = (int64_t)(((uint64_t)(uint32_t)(bins[q] < user_num ? bins[q] : -1) << 32) | (uint32_t)k);
                ib[k] = pos;
            }
        }
    }
}

// User store-and-sum (NCF_LAYOUT_USER_STORE).  Float atomics run at the memory side at
// ~1.3 TB/s of added bytes (MI355X_MICROARCH.md, Global float atomics), plain stores at
// ~6 TB/s: at C3 the user half of the step's scatter (65,536 rows x (64 + 16) floats,
// ~10.8 rows per user per batch, rows in item order so nothing merges in a tile) was
// the largest single atomic stream of the step.  The step stores each row's user-side
// gradient into ustore[row][uw] ([Um part][Ug part], row = slice offset); this launch
// walks the slice's user order (ncf_user_order: entries user << 32 | offset, users
// ascending, padding last) in pieces of US_SPAN positions, one wave per piece: the
// piece's rows are loaded together, summed per run of equal users in order, and each
// run's sum is added to its user's Um / Ug rows by one float atomic per column -- every
// wave the same work whatever the user skew, and ~US_SPAN / (runs + 1) times fewer
// atomic bytes than per row.  Lane = column (uw <= 64 * US_NCH).
constexpr int US_SPAN = 32, US_WAVES = 4, US_NCH = 4;
struct UsArgs {
    const float* ustore;
    const int64_t* order;
    float* grads;
    const ncf_step_ctl* ctl;
    int64_t batch_global, um, ug;
    int world, rank, dmu, f, uw;
};
template <int NCH>
__global__ __launch_bounds__(US_WAVES * 64) void user_sum_kernel(UsArgs A) {
    // this rank's slice of the current batch (ncf_train.hip: the step's own rows)
    const int64_t ntot = A.ctl->n_total;
    const int64_t nbatch = (ntot + A.batch_global - 1) / A.batch_global;
    const int64_t b = nbatch > 0 ? A.ctl->batch % nbatch : 0;
    const int64_t b0 = b * A.batch_global;
    int64_t gb = ntot - b0;
    if (gb > A.batch_global) gb = A.batch_global;
    if (gb < 0) gb = 0;
    const int64_t per = (gb + A.world - 1) / A.world;
    int64_t lo = (int64_t)A.rank * per, hi = lo + per;
    if (lo > gb) lo = gb;
    if (hi > gb) hi = gb;
    const int64_t base = b0 + lo, nloc = hi - lo;
    const int lane = threadIdx.x & 63;
    const int64_t p0 = ((int64_t)blockIdx.x * US_WAVES + (threadIdx.x >> 6)) * US_SPAN;
    if (p0 >= nloc) return;  // wave-uniform
    const int64_t e = lane < US_SPAN && p0 + lane < nloc ? A.order[base + p0 + lane] : -1;
    const int eu = (int)(e >> 32), eo = (int)(uint32_t)e;  // past the slice: user -1 (stop)
    float v[US_SPAN][NCH];
#pragma unroll
    for (int t = 0; t < US_SPAN; ++t) {
        const int ut = __builtin_amdgcn_readlane(eu, t), ot = __builtin_amdgcn_readlane(eo, t);
        const float* src = A.ustore + (int64_t)ot * A.uw;
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch)
            v[t][ch] = (ut >= 0 && ch * 64 + lane < A.uw) ? src[ch * 64 + lane] : 0.f;
    }
    float acc[NCH];
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) acc[ch] = 0.f;
#pragma unroll
    for (int t = 0; t < US_SPAN; ++t) {
        const int ut = __builtin_amdgcn_readlane(eu, t);
        if (ut < 0) break;  // padding rows sort last
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) acc[ch] += v[t][ch];
        const int un = t + 1 < US_SPAN ? __builtin_amdgcn_readlane(eu, t + 1) : -1;
        if (un != ut) {  // the run (or this piece of it) ends: one atomic per column
#pragma unroll
            for (int ch = 0; ch < NCH; ++ch) {
                const int col = ch * 64 + lane;
                if (col < A.dmu)
                    atomicAdd(A.grads + A.um + (int64_t)ut * A.dmu + col, acc[ch]);
                else if (col < A.uw)
                    atomicAdd(A.grads + A.ug + (int64_t)ut * A.f + (col - A.dmu), acc[ch]);
                acc[ch] = 0.f;
            }
        }
    }
}

static int prep_parts(int64_t B) {
    if (B <= PART_ROWS) return 1;
    const int64_t need = (B + PART_ROWS - 1) / PART_ROWS;
    int P = 1;
    while (P < need) P <<= 1;
    return P;
}

static int64_t al256(int64_t x) { return (x + 255) & ~(int64_t)255; }

// ---------------------------------------------------------------------------
// HR / NDCG per batch.  One wave per batch; the batch's logits staged in LDS.
// rank(e) = #{e' : x[e'] > x[e] or (x[e'] == x[e] and e' < e)}  (stable order)
constexpr int HR_MAXB = 1024;
__global__ __launch_bounds__(256) void hr_ndcg_kernel(const float* __restrict__ logits, const int32_t* __restrict__ items,
                                                      int64_t n, int bs, int k, int64_t nb, int32_t* hr, float* ndcg) {
    __shared__ float sx[4][HR_MAXB];
    __shared__ int si[4][HR_MAXB];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int64_t b = (int64_t)blockIdx.x * 4 + w;
    if (b >= nb) return;  // wave-uniform; no workgroup barrier below
    const int64_t r0 = b * bs;
    const int cnt = (int)((n - r0) < bs ? (n - r0) : bs);
    for (int e = l; e < cnt; e += 64) {
        sx[w][e] = logits[r0 + e];
        si[w][e] = items[r0 + e];
    }
    __builtin_amdgcn_wave_barrier();  // LDS is in-order per wave: the writes above are seen below
    const int gt = si[w][0];
    int best = 0x7fffffff;
    for (int e = l; e < cnt; e += 64) {
        if (si[w][e] != gt) continue;
        const float x = sx[w][e];
        int rank = 0;
        for (int e2 = 0; e2 < cnt; ++e2) {
            const float y = sx[w][e2];
            rank += (y > x) || (y == x && e2 < e);
        }
        if (rank < k && rank < best) best = rank;
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const int o = __shfl_xor(best, m, 64);
        best = o < best ? o : best;
    }
    if (l == 0) {
        const bool hit = best < k;
        hr[b] = hit ? 1 : 0;
        ndcg[b] = hit ? (float)(1.0 / log2((double)best + 2.0)) : 0.0f;
    }
}

static const KernelEntry* find_entry(int mode, int F, int L) {
    int n = 0;
    const KernelEntry* t = kernel_table(&n);
    const int Lk = (mode == NCF_MODEL_GMF) ? 1 : L;
    for (int i = 0; i < n; ++i)
        if (t[i].mode == mode && t[i].F == F && t[i].L == Lk) return &t[i];
    return nullptr;
}

static int64_t train_lds_floats(const KernelEntry* e, const ncf_layout* lay, int geo = GEO_8) {
    const int64_t img = lay->tower_len + 1;
    return e->w_total + e->misc[geo] + (e->stage[geo] > img ? e->stage[geo] : img);
}

static Ranges make_ranges(const int64_t* ranges, int nranges, int* err) {
    Ranges R;
    memset(&R, 0, sizeof(R));
    *err = 0;
    if (nranges < 1 || nranges > 8) {
        *err = 1;
        return R;
    }
    R.n = nranges;
    R.prefix[0] = 0;
    for (int i = 0; i < nranges; ++i) {
        const int64_t b = ranges[2 * i], e = ranges[2 * i + 1];
        if (b < 0 || e < b || (b & 3) || ((e - b) & 3)) *err = 1;
        R.begin[i] = b;
        R.prefix[i + 1] = R.prefix[i] + (e - b) / 4;
    }
    for (int i = nranges + 1; i < 9; ++i) R.prefix[i] = R.prefix[nranges];
    return R;
}

static int g_diag = 0;
static unsigned long long* g_stamps = nullptr;
// ncf_debug_set_geometry: 0 = ncf_layout_tune decides, 4 / NWAVES = forced (A/B, tests)
static int g_geo_waves = 0;
// ncf_debug_set_per_row: -1 = ncf_layout_tune's rule (2 rows < U + I), 0 / 1 forced (A/B)
static int g_per_row = -1;
// ncf_debug_set_user_store: 0 = off (the default: measured slower),
// -1 = ncf_layout_tune decides by the per-rank batch, 1 = wherever it applies
static int g_user_store = 0;
// ncf_layout_tune: user store-and-sum from this many rows per launch up
#ifndef NCF_US_MIN_ROWS
#define NCF_US_MIN_ROWS 16384
#endif
// ncf_layout_tune: 8-wave workgroups from this many 128-row tiles up, else 4-wave
#ifndef NCF_GEO_MIN_WGS
#define NCF_GEO_MIN_WGS 256
#endif
constexpr int64_t GEO_MIN_WGS = NCF_GEO_MIN_WGS;

static int launch_status() { return hipGetLastError() == hipSuccess ? NCF_OK : NCF_E_LAUNCH; }

// hipFuncSetAttribute once per (kernel, size): nothing but launches happen on
// the hot path, so a step can be captured into a hipGraph.
static int ensure_lds(const void* fn, int64_t bytes) {
    struct Slot { const void* fn; int64_t bytes; };
    static Slot slots[128];
    static int nslots = 0;
    for (int i = 0; i < nslots; ++i)
        if (slots[i].fn == fn && slots[i].bytes >= bytes) return NCF_OK;
    if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) != hipSuccess)
        return NCF_E_LAUNCH;
    for (int i = 0; i < nslots; ++i)
        if (slots[i].fn == fn) { slots[i].bytes = bytes; return NCF_OK; }
    if (nslots < 128) slots[nslots++] = Slot{fn, bytes};
    return NCF_OK;
}

// ---------------------------------------------------------------------------
// Feature distillation terms (reference src/distillation/feature.py:51-123): one
// wave per row of this rank's shard of the current global batch.  Per feature key:
// the student feature x goes to the wave's LDS row, phase 1 (lanes over adapter
// outputs o) forms a_o = c_o + A[o,:] x, the teacher feature and the loss, and
// stores da_o = 2 coef (a_o - t_o) / (B T); phase 2 (lanes over inputs s) forms
// dx_s = sum_o A[o,s] da_o and scatter-adds it into the student's embedding rows.
// The adapters are small (at most [2048 x 1024]) and read through L1/L2.
struct KdKey {
    const float* A;  // [T][S] nn.Linear weight, nullptr = identity
    const float* c;  // [T] bias
    float coef;      // beta / count; 0 = key not matched
    int S, T;
};
struct KdFeatArgs {
    ncf_layout sl, tl;
    const float* sp;
    float* sg;
    const float* tp;
    const uint64_t* rows;
    const ncf_step_ctl* ctl;
    int64_t batch_global;
    int world, rank;
    KdKey key[2];
    float* loss_out;
};
constexpr int KD_MAXS = 1024, KD_MAXT = 2048, KD_WAVES = 4;

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ __launch_bounds__(256) void kd_feature_kernel(KdFeatArgs a) {
    __shared__ float sx[KD_WAVES][KD_MAXS];
    __shared__ float sd[KD_WAVES][KD_MAXT];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    // rows of this rank: the selection of ncf_train_step (ncf_train.hip)
    const int64_t ntot = a.ctl->n_total;
    const int64_t nbatch = (ntot + a.batch_global - 1) / a.batch_global;
    const int64_t b = nbatch > 0 ? a.ctl->batch % nbatch : 0;
    const int64_t b0 = b * a.batch_global;
    int64_t gb = ntot - b0;
    if (gb > a.batch_global) gb = a.batch_global;
    if (gb < 0) gb = 0;
    const int64_t per = (gb + a.world - 1) / a.world;
    int64_t lo = (int64_t)a.rank * per, hi = lo + per;
    if (lo > gb) lo = gb;
    if (hi > gb) hi = gb;
    const float gbf = (float)gb;
    const ncf_layout& sl = a.sl;
    const ncf_layout& tl = a.tl;
    float lossw = 0.f;
    for (int64_t r = lo + (int64_t)blockIdx.x * KD_WAVES + w; r < hi; r += (int64_t)gridDim.x * KD_WAVES) {
        const uint64_t pr = a.rows[b0 + r];
        const int u = (int)(uint32_t)pr;
        const int it = (int)((pr >> 32) & 0x7fffffffu);
        if (u < 0) continue;  // padding row (wave-uniform)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const KdKey K = a.key[k];
            if (K.coef == 0.f) continue;
            const int S = K.S, T = K.T;
            const float scale = K.coef / (gbf * (float)T);
            float us = 0.f, is = 0.f;
            if (k == 0) {  // gmf_features = embed_user_GMF(u) * embed_item_GMF(i)  (feature.py:56-59)
                if (l < S) {
                    us = a.sp[sl.ug + (int64_t)u * S + l];
                    is = a.sp[sl.ig + (int64_t)it * S + l];
                    sx[w][l] = us * is;
                }
            } else {  // mlp_input = cat(embed_user_MLP(u), embed_item_MLP(i))  (feature.py:61-65)
                const int dms = S / 2;
                for (int s = l; s < S; s += 64)
                    sx[w][s] = s < dms ? a.sp[sl.um + (int64_t)u * dms + s] : a.sp[sl.im + (int64_t)it * dms + (s - dms)];
            }
            wave_sync_lds();
            for (int o = l; o < T; o += 64) {
                float av;
                if (K.A != nullptr) {  // adapter nn.Linear (feature.py:36-46, 97-100)
                    const float* Ar = K.A + (int64_t)o * S;
                    av = 0.f;
                    for (int s = 0; s < S; ++s) av += Ar[s] * sx[w][s];
                    av += K.c[o];
                } else {
                    av = sx[w][o];
                }
                float xt;
                if (k == 0) {
                    xt = a.tp[tl.ug + (int64_t)u * T + o] * a.tp[tl.ig + (int64_t)it * T + o];
                } else {
                    const int dmt = T / 2;
                    xt = o < dmt ? a.tp[tl.um + (int64_t)u * dmt + o] : a.tp[tl.im + (int64_t)it * dmt + (o - dmt)];
                }
                const float d = av - xt;
                lossw += scale * (d * d);     // F.mse_loss(student_feat, teacher_feat), feature.py:110
                sd[w][o] = 2.f * scale * d;
            }
            wave_sync_lds();
            for (int s = l; s < S; s += 64) {
                float dx;
                if (K.A != nullptr) {
                    dx = 0.f;
                    for (int o = 0; o < T; ++o) dx += K.A[(int64_t)o * S + s] * sd[w][o];
                } else {
                    dx = sd[w][s];
                }
                if (k == 0) {
                    atomicAdd(a.sg + sl.ug + (int64_t)u * S + s, dx * is);
                    atomicAdd(a.sg + sl.ig + (int64_t)it * S + s, dx * us);
                } else {
                    const int dms = S / 2;
                    if (s < dms)
                        atomicAdd(a.sg + sl.um + (int64_t)u * dms + s, dx);
                    else
                        atomicAdd(a.sg + sl.im + (int64_t)it * dms + (s - dms), dx);
                }
            }
            wave_sync_lds();
        }
    }
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) lossw += __shfl_xor(lossw, m, 64);
    if (l == 0 && lossw != 0.f) atomicAdd(a.loss_out, lossw);
}

// ---------------------------------------------------------------------------
// Factored layer 0 (ncf_train.hip, FACT): the step left G_u = sum of the D0 rows
// of user u in grads[um] and H_i in grads[im] (width DM = S(1)).  fact_expand_kernel
// turns them into the true gradients; one block per cpb consecutive CH-row chunks of one table X
// (X = Um with koff = 0, or Im with koff = DM), its G and X rows and the W0 half it
// needs staged in LDS once, 16 waves each owning output tiles:
//   dX = G W0[:, koff : koff + DM]   (16 x 16 tiles), written over G
//   P_b = G^T X                       the block's partial of dW0[:, koff : koff + DM]
//                                     (NT x NT tiles), plain stores to partials[b][DM][DM]
// The tower reductions (reduce_slab_kernel / reduce_adam_kernel, W0Part) sum the
// partials of each half in block order (deterministic, no atomics: every block's
// partial covers the same 16 KB of W0, so float atomics would serialise on it).  v_mfma_f32_16x16x4_f32 throughout:
// (U + I)/16 tile GEMMs per step in place of the per-row layer-0 dgrad / wgrad of B/16.
constexpr int FX_WAVES = 16;  // 16 waves: dW0 / dX output tiles dealt round-robin

// Chunk rows per LDS pass: 64 up to DM = 64, 32 at DM = 128 (W0 half + 3 chunk
// images = 118 KB).  A block walks `cpb` consecutive chunks of one table with the
// W0 half staged once and its dW0 partial held in registers across them.
#ifndef NCF_FX_CPB128
#define NCF_FX_CPB128 2
#endif
#ifndef NCF_FX_CH64  // chunk rows up to DM = 64 (experiment switch)
#define NCF_FX_CH64 64
#endif
template <int DM>
struct FxShape {
    static constexpr int CH = DM <= 64 ? NCF_FX_CH64 : 32;
    static constexpr int CPB = DM <= 64 ? 1 : NCF_FX_CPB128;  // chunks per block
    static constexpr int ST = DM + 4, NT = (DM + 15) / 16, Q4 = DM / 4;
    static constexpr int TPW = (NT * NT + FX_WAVES - 1) / FX_WAVES;  // dW0 tiles per wave
    static constexpr int64_t LDS = ((int64_t)DM * ST + 3LL * CH * ST) * 4;
};

// Expansion modes: FX_FULL (dX over G and the dW0 partials), FX_DW0 (NCF_LAYOUT_FACT_
// DEFER_DX: the dW0 partials only, the W0 the step ran with saved to the snapshot),
// FX_DX (ncf_adam_step_fact: dX only, over the Um / Im rows of one rank's reduce-
// scattered gradient shard, W0 from the snapshot).
enum { FX_FULL = 0, FX_DW0 = 1, FX_DX = 2 };
struct FxArgs {
    const float* prm;   // X rows (params; FX_FULL / FX_DW0)
    const float* w0;    // W0 [DM][2 DM] (row stride 2 DM): params' W0, or the snapshot (FX_DX)
    float* g;           // G rows: flat element q of the gradient at g[q - gofs]; dX written over them
    int64_t gofs;
    int64_t xoff[2];    // Um / Im offsets
    int64_t r0[2], r1[2];  // rows [r0, r1) of each table expanded
    float* partials;    // [nblk][DM][DM] (FX_FULL / FX_DW0)
    float* w0snap;      // FX_DW0: the snapshot written
    int nbu, mode;
};

template <int DM>
__global__ __launch_bounds__(FX_WAVES * 64) void fact_expand_kernel(FxArgs A) {
    using X_ = FxShape<DM>;
    constexpr int CH = X_::CH, ST = X_::ST, NT = X_::NT, Q4 = X_::Q4, TPW = X_::TPW, cpb = X_::CPB;
    extern __shared__ __attribute__((aligned(16))) float fsm[];
    float* sW = fsm;           // W0[:, koff : koff + DM]  [DM][ST]
    float* sG = sW + DM * ST;  // G rows  [CH][ST]
    float* sX = sG + CH * ST;  // X rows  [CH][ST]
    float* sO = sX + CH * ST;  // dX rows [CH][ST]
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, c = l & 15, g = l >> 4;
    const int t = (int)blockIdx.x < A.nbu ? 0 : 1;  // 0: Um, 1: Im
    const int64_t rend = A.r1[t];
    const int64_t xoff = A.xoff[t];
    const int koff = t * DM;
    const bool want_dw = A.mode != FX_DX, want_dx = A.mode != FX_DW0;
    const int64_t rb = A.r0[t] + (int64_t)(t == 0 ? blockIdx.x : blockIdx.x - A.nbu) * cpb * CH;  // first row
    float* gx = A.g + (xoff - A.gofs);  // row r of the table's G at gx + r DM
    // the W0 half: loads issued here, stored to LDS behind the first chunk's loads
    constexpr int NW4 = DM * Q4, PW = (NW4 + FX_WAVES * 64 - 1) / (FX_WAVES * 64);
    f4 wv[PW];
#pragma unroll
    for (int q = 0; q < PW; ++q) {
        const int e4 = tid + q * FX_WAVES * 64, j = e4 / Q4, k4 = e4 - j * Q4;
        wv[q] = e4 < NW4 ? *reinterpret_cast<const f4*>(A.w0 + (int64_t)j * 2 * DM + koff + 4 * k4)
                         : f4{0.f, 0.f, 0.f, 0.f};
    }
    // FX_DW0: the first block of each table saves its W0 half (the weights this step
    // ran with) for the sharded dX expansion of ncf_adam_step_fact
    if (A.mode == FX_DW0 && A.w0snap != nullptr && (blockIdx.x == 0 || (int)blockIdx.x == A.nbu)) {
#pragma unroll
        for (int q = 0; q < PW; ++q) {
            const int e4 = tid + q * FX_WAVES * 64, j = e4 / Q4, k4 = e4 - j * Q4;
            if (e4 < NW4) *reinterpret_cast<f4*>(A.w0snap + (int64_t)j * 2 * DM + koff + 4 * k4) = wv[q];
        }
    }
    f4 accw[TPW];
#pragma unroll
    for (int q = 0; q < TPW; ++q) accw[q] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ch = 0; ch < cpb; ++ch) {
        const int64_t r0 = rb + (int64_t)ch * CH;
        if (r0 >= rend) break;  // block-uniform
        if (ch > 0) __syncthreads();  // the previous chunk's images are consumed
        {   // the chunk's G (and X) rows -> LDS (each thread's loads issued together)
            constexpr int NR4 = CH * Q4, PR = (NR4 + FX_WAVES * 64 - 1) / (FX_WAVES * 64);
            f4 gv[PR], xv[PR];
#pragma unroll
            for (int q = 0; q < PR; ++q) {
                const int e4 = tid + q * FX_WAVES * 64, row = e4 / Q4, k4 = e4 - row * Q4;
                const bool ok = e4 < NR4 && r0 + row < rend;
                gv[q] = ok ? *reinterpret_cast<const f4*>(gx + (r0 + row) * DM + 4 * k4) : f4{0.f, 0.f, 0.f, 0.f};
                xv[q] = ok && want_dw ? *reinterpret_cast<const f4*>(A.prm + xoff + (r0 + row) * DM + 4 * k4)
                                      : f4{0.f, 0.f, 0.f, 0.f};
            }
            if (ch == 0) {
#pragma unroll
                for (int q = 0; q < PW; ++q) {
                    const int e4 = tid + q * FX_WAVES * 64, j = e4 / Q4, k4 = e4 - j * Q4;
                    if (e4 < NW4) *reinterpret_cast<f4*>(sW + j * ST + 4 * k4) = wv[q];
                }
            }
#pragma unroll
            for (int q = 0; q < PR; ++q) {
                const int e4 = tid + q * FX_WAVES * 64, row = e4 / Q4, k4 = e4 - row * Q4;
                if (e4 < NR4) {
                    *reinterpret_cast<f4*>(sG + row * ST + 4 * k4) = gv[q];
                    if (want_dw) *reinterpret_cast<f4*>(sX + row * ST + 4 * k4) = xv[q];
                }
            }
        }
        __syncthreads();
        // dW0 partial, tiles (mt, nt) dealt round-robin to the waves:
        // A[i = j][k = row] = G[row][j],  B[k = row][n = k'] = X[row][k']
        if (want_dw) {
#pragma unroll
            for (int q = 0; q < TPW; ++q) {
                const int tt = w + q * FX_WAVES;
                if (tt >= NT * NT) break;
                const int mt = tt / NT, nt = tt - mt * NT;
                const bool jok = 16 * mt + c < DM, kok = 16 * nt + c < DM;
                f4 a0 = accw[q], a1 = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
                for (int s4 = 0; s4 < CH / 4; s4 += 2) {
                    const int ra = 4 * s4 + g, rb2 = ra + 4;
                    a0 = MFMA4(jok ? sG[ra * ST + 16 * mt + c] : 0.f, kok ? sX[ra * ST + 16 * nt + c] : 0.f, a0);
                    a1 = MFMA4(jok ? sG[rb2 * ST + 16 * mt + c] : 0.f, kok ? sX[rb2 * ST + 16 * nt + c] : 0.f, a1);
                }
                a0.x += a1.x; a0.y += a1.y; a0.z += a1.z; a0.w += a1.w;
                accw[q] = a0;
            }
        }
        // FX_DW0: G stays; the owner of each row expands it after the reduce-scatter
        if (!want_dx) continue;
        // dX = G W0h, tiles (rt, nt): A[i = row][k = j] = G[row][j],  B[k = j][n = k'] = W0h[j][k']
        for (int tt = w; tt < (CH / 16) * NT; tt += FX_WAVES) {
            const int rt = tt / NT, nt = tt - rt * NT;
            const bool nok = 16 * nt + c < DM;
            f4 d = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kk = 0; kk < DM / 4; ++kk)
                d = MFMA4(sG[(16 * rt + c) * ST + 4 * kk + g], nok ? sW[(4 * kk + g) * ST + 16 * nt + c] : 0.f, d);
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (nok) sO[(16 * rt + 4 * g + q) * ST + 16 * nt + c] = lane_get(d, q);
        }
        __syncthreads();
        for (int e = tid; e < CH * Q4; e += FX_WAVES * 64) {
            const int row = e / Q4, q = e - row * Q4;
            if (r0 + row < rend)
                *reinterpret_cast<f4*>(gx + (r0 + row) * DM + 4 * q) = *reinterpret_cast<const f4*>(sO + row * ST + 4 * q);
        }
    }
    if (!want_dw) return;
    // the block's dW0 partial: plain stores (every block covers the same W0 half)
    float* pb = A.partials + (int64_t)blockIdx.x * DM * DM;
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        const int tt = w + q * FX_WAVES;
        if (tt >= NT * NT) break;
        const int mt = tt / NT, nt = tt - mt * NT;
        const bool kok = 16 * nt + c < DM;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int j = 16 * mt + 4 * g + r;
            if (j < DM && kok) pb[j * DM + 16 * nt + c] = lane_get(accw[q], r);
        }
    }
}


// ncf_adam_step_fact in one launch (dp_mode "zero1", NCF_LAYOUT_FACT_DEFER_DX, DM <= 64):
// three block roles over the rank's gradient shard --
//   [0, nbx)           one CH-row chunk of the Um / Im rows inside the shard each: G rows
//                      (gshard) and the W0 half (the step's snapshot) to LDS, dX = G W0h
//                      on MFMA tiles into LDS, then Adam on those elements straight from
//                      LDS (their p, m, v requested before the MFMAs);
//   [nbx, nbx + nba)   Adam over the shard's other active ranges (RA: the ranges minus the
//                      two table windows);
//   the rest           clear the local gradient bucket for the next step's accumulation.
// gshard is not cleared (the next reduce-scatter overwrites all of it).
struct FsArgs {
    float* p;
    const float* g;
    float* m;
    float* v;            // shard views: element i = flat shard_begin + i
    const float* w0s;    // W0 as the step ran with it, [DM][2 DM]
    int64_t xrel[2];     // Um / Im offset - shard_begin
    int64_t r0[2], r1[2];
    int nbu, nbx, nba;
    Ranges RA;
    f4* zero;            // local bucket (f4s), may be null
    int64_t zn4;
    const ncf_step_ctl* ctl;
    double lr, beta1, beta2;
    float eps;
    int64_t loss_slot;
    float* loss_hist;
    int64_t hist_len;
    ScCache* scc;
};

template <int DM>
__global__ __launch_bounds__(FX_WAVES * 64) void adam_fact_shard_kernel(FsArgs A) {
#pragma clang fp contract(off)
    using X_ = FxShape<DM>;
    constexpr int CH = X_::CH, ST = X_::ST, NT = X_::NT, Q4 = X_::Q4;
    static_assert(X_::CPB == 1, "one chunk per block");
    __shared__ float sc[2];
    const int tid = threadIdx.x, b = (int)blockIdx.x;
    const int64_t t_step = A.ctl->adam_t;  // advanced by ncf_reduce_slab
    if (b >= A.nbx + A.nba) {  // clear the local bucket
        const int64_t nthr = (int64_t)(gridDim.x - A.nbx - A.nba) * blockDim.x;
        for (int64_t q = (int64_t)(b - A.nbx - A.nba) * blockDim.x + tid; q < A.zn4; q += nthr)
            A.zero[q] = f4{0.f, 0.f, 0.f, 0.f};
        return;
    }
    step_scalars(A.scc, t_step, A.lr, A.beta1, A.beta2, sc);
    step_scalars_ahead(A.scc, t_step, A.lr, A.beta1, A.beta2);
    const float w1 = (float)(1.0 - A.beta1), b2 = (float)A.beta2, omb2 = (float)(1.0 - A.beta2);
    if (b >= A.nbx) {  // plain Adam over RA
        __syncthreads();
        const float neg_step = sc[0], bc2s = sc[1];
        const int64_t total = A.RA.prefix[A.RA.n];
        const int64_t nthr = (int64_t)A.nba * blockDim.x;
        for (int64_t q = (int64_t)(b - A.nbx) * blockDim.x + tid; q < total; q += nthr) {
            int which;
            const int64_t i = range_locate(A.RA, q, &which);
            const f4 gg = *reinterpret_cast<const f4*>(A.g + i);
            f4 mm = *reinterpret_cast<const f4*>(A.m + i);
            f4 vv = *reinterpret_cast<const f4*>(A.v + i);
            f4 pp = *reinterpret_cast<const f4*>(A.p + i);
            adam_f4(pp, mm, vv, gg, w1, b2, omb2, bc2s, A.eps, neg_step);
            *reinterpret_cast<f4*>(A.m + i) = mm;
            *reinterpret_cast<f4*>(A.v + i) = vv;
            *reinterpret_cast<f4*>(A.p + i) = pp;
        }
        if (b == A.nbx && tid == 0 && A.loss_hist != nullptr && A.loss_slot >= 0 && A.hist_len > 0) {
            const int64_t bt = A.ctl->batch - 1;  // ncf_reduce_slab advanced it (record_loss)
            A.loss_hist[((bt % A.hist_len) + A.hist_len) % A.hist_len] = A.g[A.loss_slot];
        }
        return;
    }
    // expansion + Adam of one chunk of table rows
    extern __shared__ __attribute__((aligned(16))) float fsm[];
    float* sW = fsm;           // W0[:, koff : koff + DM]  [DM][ST]
    float* sG = sW + DM * ST;  // G rows  [CH][ST]
    float* sO = sG + CH * ST;  // dX rows [CH][ST] (FxShape's X image unused)
    const int w = tid >> 6, l = tid & 63, c = l & 15, g = l >> 4;
    const int t = b < A.nbu ? 0 : 1;
    const int64_t rend = A.r1[t];
    const int64_t r0 = A.r0[t] + (int64_t)(t == 0 ? b : b - A.nbu) * CH;
    const int64_t xrel = A.xrel[t];
    constexpr int NW4 = DM * Q4, PW = (NW4 + FX_WAVES * 64 - 1) / (FX_WAVES * 64);
    constexpr int NR4 = CH * Q4, PR = (NR4 + FX_WAVES * 64 - 1) / (FX_WAVES * 64);
    f4 wv[PW], gv[PR], pp[PR], mm[PR], vv[PR];
#pragma unroll
    for (int q = 0; q < PW; ++q) {
        const int e4 = tid + q * FX_WAVES * 64, j = e4 / Q4, k4 = e4 - j * Q4;
        wv[q] = e4 < NW4 ? *reinterpret_cast<const f4*>(A.w0s + (int64_t)j * 2 * DM + t * DM + 4 * k4)
                         : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int q = 0; q < PR; ++q) {
        const int e4 = tid + q * FX_WAVES * 64, row = e4 / Q4, k4 = e4 - row * Q4;
        const bool ok = e4 < NR4 && r0 + row < rend;
        const int64_t i = xrel + (r0 + row) * DM + 4 * k4;
        const f4 z = f4{0.f, 0.f, 0.f, 0.f};
        gv[q] = ok ? *reinterpret_cast<const f4*>(A.g + i) : z;
        pp[q] = ok ? *reinterpret_cast<const f4*>(A.p + i) : z;
        mm[q] = ok ? *reinterpret_cast<const f4*>(A.m + i) : z;
        vv[q] = ok ? *reinterpret_cast<const f4*>(A.v + i) : z;
    }
#pragma unroll
    for (int q = 0; q < PW; ++q) {
        const int e4 = tid + q * FX_WAVES * 64, j = e4 / Q4, k4 = e4 - j * Q4;
        if (e4 < NW4) *reinterpret_cast<f4*>(sW + j * ST + 4 * k4) = wv[q];
    }
#pragma unroll
    for (int q = 0; q < PR; ++q) {
        const int e4 = tid + q * FX_WAVES * 64, row = e4 / Q4, k4 = e4 - row * Q4;
        if (e4 < NR4) *reinterpret_cast<f4*>(sG + row * ST + 4 * k4) = gv[q];
    }
    __syncthreads();
    // dX = G W0h, tiles (rt, nt): A[i = row][k = j] = G[row][j],  B[k = j][n = k'] = W0h[j][k']
    for (int tt = w; tt < (CH / 16) * NT; tt += FX_WAVES) {
        const int rt = tt / NT, nt = tt - rt * NT;
        const bool nok = 16 * nt + c < DM;
        f4 d = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < DM / 4; ++kk)
            d = MFMA4(sG[(16 * rt + c) * ST + 4 * kk + g], nok ? sW[(4 * kk + g) * ST + 16 * nt + c] : 0.f, d);
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (nok) sO[(16 * rt + 4 * g + q) * ST + 16 * nt + c] = lane_get(d, q);
    }
    __syncthreads();
    const float neg_step = sc[0], bc2s = sc[1];
#pragma unroll
    for (int q = 0; q < PR; ++q) {
        const int e4 = tid + q * FX_WAVES * 64, row = e4 / Q4, k4 = e4 - row * Q4;
        if (e4 < NR4 && r0 + row < rend) {
            const int64_t i = xrel + (r0 + row) * DM + 4 * k4;
            const f4 gg = *reinterpret_cast<const f4*>(sO + row * ST + 4 * k4);
            adam_f4(pp[q], mm[q], vv[q], gg, w1, b2, omb2, bc2s, A.eps, neg_step);
            *reinterpret_cast<f4*>(A.m + i) = mm[q];
            *reinterpret_cast<f4*>(A.v + i) = vv[q];
            *reinterpret_cast<f4*>(A.p + i) = pp[q];
        }
    }
}


int launch_zero_f32(float* p, int64_t n, hipStream_t st) {
    if (!p || n < 0 || (n & 3) || (reinterpret_cast<uintptr_t>(p) & 15)) return NCF_E_ARG;
    if (n == 0) return NCF_OK;
    int64_t grid = (n / 4 + 255) / 256;
    if (grid > 2048) grid = 2048;
    hipLaunchKernelGGL(zero_f32_kernel, dim3((int)grid), dim3(256), 0, st, reinterpret_cast<f4*>(p), n / 4);
    return hipGetLastError() == hipSuccess ? NCF_OK : NCF_E_LAUNCH;
}

// Factored layer 0 for this layout?  MLP shapes whose two embedding tables have
// fewer rows than FACT_MAX_ROWS (the expand pass works on U + I rows per step, the
// per-row layer-0 gradients on B rows: at ml-1m 9.7K vs 65K; at ml-20m the tables
// have 165K rows and the per-row form stays), on the fused path or, for DM up to
// 128, the layered one (there the layer-0 forward is a per-step projection of the
// tables too, ncf_layered.hip).
#ifndef NCF_FACT_MAX_ROWS
#define NCF_FACT_MAX_ROWS 32768
#endif
constexpr int64_t FACT_MAX_ROWS = NCF_FACT_MAX_ROWS;
// Fused kernel for this layout, or nullptr (then the layered path runs).
static const KernelEntry* fused_entry(const ncf_layout* lay) {
    const KernelEntry* e = find_entry(lay->model_type, lay->factor_num, lay->num_layers);
    if (!e) return nullptr;
    return train_lds_floats(e, lay) * 4 <= LDS_LIMIT_BYTES ? e : nullptr;
}
// Fused kernel of a training step: none with dropout (the layered path applies it).
static const KernelEntry* train_fused(const ncf_layout* lay) {
    if (lay->flags & NCF_LAYOUT_LAYERED) return nullptr;
    return lay->dropout > 0.f ? nullptr : fused_entry(lay);
}
static int fact_dm(const ncf_layout* lay) { return lay->factor_num << (lay->num_layers - 1); }
static bool fact_mode(const ncf_layout* lay) {
    if (lay->model_type == NCF_MODEL_GMF || (lay->flags & NCF_LAYOUT_PER_ROW_L0)) return false;
    if (lay->dropout > 0.f) return false;  // masks per row: layer 0 does not factor per entity
    if ((int64_t)lay->user_num + lay->item_num > FACT_MAX_ROWS) return false;
    const int dm = fact_dm(lay);
    const bool lds_dm = dm == 8 || dm == 16 || dm == 32 || dm == 64 || dm == 128;  // fact_expand_kernel<DM>
    const KernelEntry* e = train_fused(lay);
    if (e) return lds_dm && e->train_fact[GEO_8] != nullptr;
    // layered path: wider dm (256, 512) expanded with GEMMs (ncf_layered.hip lyr_fact_dx / dw0)
    return (lds_dm || dm == 256 || dm == FACT_MAX_DM) && lay->factor_num <= LYR_MAX_FACTOR;
}

// Launch geometry of the fused training step: 4-wave workgroups where
// ncf_layout_tune asked for them (the NCF_LAYOUT_GEO field) and the kernel exists.
static int train_geo(const KernelEntry* e, const ncf_layout* lay) {
    const int g = (lay->flags >> NCF_LAYOUT_GEO_SHIFT) & NCF_LAYOUT_GEO_MASK;
    if (g == GEO_8) return GEO_8;
    const void* fn = fact_mode(lay) ? e->train_fact[g] : e->train[g];
    return fn != nullptr ? g : GEO_8;
}

// Workgroups of the fused step = rows of the slab the reductions read.
static int slab_rows_of(const ncf_layout* lay) {
    const int w = (lay->flags >> NCF_LAYOUT_WG_SHIFT) & NCF_LAYOUT_WG_MASK;
    return (w > 0 && w < SLAB_ROWS) ? w : SLAB_ROWS;
}

// First tower column (relative to tower_begin) the reductions produce: GMF models
// have no tower.
static int slab_lo(const ncf_layout* lay) {
    if (lay->model_type == NCF_MODEL_GMF) return (int)(lay->wp - lay->tower_begin);
    return 0;
}

static int fact_ch(const ncf_layout* lay) { return fact_dm(lay) <= 64 ? NCF_FX_CH64 : 32; }  // FxShape<DM>::CH
static int fact_cpb(const ncf_layout* lay) { return fact_dm(lay) <= 64 ? 1 : NCF_FX_CPB128; }  // FxShape<DM>::CPB

static int fact_blocks(const ncf_layout* lay, int* nbu) {
    const int64_t per = (int64_t)fact_ch(lay) * fact_cpb(lay);
    const int bu = (int)((lay->user_num + per - 1) / per), bi = (int)((lay->item_num + per - 1) / per);
    *nbu = bu;
    return bu + bi;
}

// NCF_LAYOUT_USER_STORE: user-side gradient row width ([Um part][Ug part]) and
// whether the fused step can run it (user_order_kernel's user bound, the sum
// kernel's columns, vector-aligned parts).
static int us_uw(const ncf_layout* lay) {
    const bool mlp = lay->model_type != NCF_MODEL_GMF, gmf = lay->model_type != NCF_MODEL_MLP;
    return (mlp ? (lay->factor_num << (lay->num_layers - 1)) : 0) + (gmf ? lay->factor_num : 0);
}
static bool us_applies(const ncf_layout* lay) {
    return train_fused(lay) != nullptr && lay->user_num <= UO_MAX_USERS && lay->factor_num % 4 == 0 &&
           us_uw(lay) <= 64 * US_NCH;
}
static bool us_on(const ncf_layout* lay) { return (lay->flags & NCF_LAYOUT_USER_STORE) && us_applies(lay); }
static int64_t us_floats(const ncf_layout* lay, int64_t rows) {
    return us_on(lay) ? ((rows + TILE_ROWS + 63) & ~(int64_t)63) * us_uw(lay) : 0;
}

static int64_t fact_partials_floats(const ncf_layout* lay) {
    if (fact_dm(lay) > FACT_LDS_DM) return 0;  // W0 into the slab (the layered GEMM expansion)
    int nbu;
    const int64_t DM = (int64_t)lay->factor_num << (lay->num_layers - 1);
    return (int64_t)fact_blocks(lay, &nbu) * DM * DM;
}

// The dW0 partials in the train workspace: after the fused path's slab rows, or
// after the layered path's single slab row (ncf_layered.hip).
static float* fact_partials(const ncf_layout* lay, void* workspace) {
    const int64_t stride = lay->tower_len + 64;
    return static_cast<float*>(workspace) +
           (train_fused(lay) ? (int64_t)SLAB_ROWS * stride : rup64((int64_t)lyr_slab_rows(lay) * stride));
}

// Rows of the partial slab the reductions sum: the fused step's workgroups, or the
// layered path's lyr_slab_rows.
static int reduce_rows(const ncf_layout* lay) { return train_fused(lay) ? slab_rows_of(lay) : lyr_slab_rows(lay); }

// NCF_LAYOUT_FACT_DEFER_DX: the W0 the step ran with ([DM][2 DM]), saved by the
// expansion after the dW0 partials; ncf_adam_step_fact forms dX = G W0 half from it
// while the same launch updates W0 itself (fused path, dm <= FACT_LDS_DM).
static int64_t fact_w0_snap_floats(const ncf_layout* lay) {
    const int64_t DM = fact_dm(lay);
    return DM <= FACT_LDS_DM ? 2 * DM * DM : 0;
}
static float* fact_w0_snap(const ncf_layout* lay, void* workspace) {
    return fact_partials(lay, workspace) + fact_partials_floats(lay);
}

static W0Part w0_part(const ncf_layout* lay, const void* workspace) {
    W0Part wp;
    memset(&wp, 0, sizeof(wp));
    if (!fact_mode(lay) || fact_dm(lay) > FACT_LDS_DM) return wp;  // W0 from the slab
    wp.p = fact_partials(lay, const_cast<void*>(workspace));
    wp.nblk = fact_blocks(lay, &wp.nbu);
    wp.dm = lay->factor_num << (lay->num_layers - 1);
    wp.cols = (int)(lay->b[0] - lay->w[0]);
    return wp;
}

static int fact_expand_entry(int DM, const void** fe, int64_t* lds) {
    switch (DM) {
#define NCF_FX(D) case D: *fe = reinterpret_cast<const void*>(&fact_expand_kernel<D>); *lds = FxShape<D>::LDS; break;
        NCF_FX(8) NCF_FX(16) NCF_FX(32) NCF_FX(64) NCF_FX(128)
#undef NCF_FX
        default: return NCF_E_UNSUPPORTED;
    }
    return ensure_lds(*fe, *lds) == NCF_OK ? NCF_OK : NCF_E_LAUNCH;
}

static int launch_fx(const void* fe, int64_t lds, FxArgs& A, int nblk, hipStream_t st) {
    if (nblk <= 0) return NCF_OK;
    void* ae[] = {&A};
    if (hipLaunchKernel(fe, dim3((unsigned)nblk), dim3(FX_WAVES * 64), ae, (size_t)lds, st) != hipSuccess)
        return NCF_E_LAUNCH;
    return hipGetLastError() == hipSuccess ? NCF_OK : NCF_E_LAUNCH;
}

// After the train step: FX_FULL, or FX_DW0 under NCF_LAYOUT_FACT_DEFER_DX.
static int launch_fact_expand(const ncf_layout* lay, const float* params, float* grads, float* partials,
                              float* w0snap, hipStream_t st) {
    const int DM = lay->factor_num << (lay->num_layers - 1);
    if (DM > FACT_LDS_DM) return NCF_OK;  // expanded by the layered path itself (lyr_run)
    const void* fe;
    int64_t lds;
    int rc = fact_expand_entry(DM, &fe, &lds);
    if (rc != NCF_OK) return rc;
    FxArgs A;
    memset(&A, 0, sizeof(A));
    A.prm = params;
    A.w0 = params + lay->w[0];
    A.g = grads;
    A.xoff[0] = lay->um;
    A.xoff[1] = lay->im;
    A.r1[0] = lay->user_num;
    A.r1[1] = lay->item_num;
    A.partials = partials;
    A.w0snap = w0snap;
    A.mode = (lay->flags & NCF_LAYOUT_FACT_DEFER_DX) ? FX_DW0 : FX_FULL;
    const int nblk = fact_blocks(lay, &A.nbu);
    return launch_fx(fe, lds, A, nblk, st);
}

// ncf_adam_step_fact: FX_DX over the Um / Im rows inside one rank's gradient shard
// [shard_begin, shard_begin + shard_len) -- G in gshard, dX written over it.
static int launch_fact_dx(const ncf_layout* lay, const float* w0snap, float* gshard, int64_t shard_begin,
                          int64_t shard_len, hipStream_t st) {
    const int DM = fact_dm(lay);
    const void* fe;
    int64_t lds;
    int rc = fact_expand_entry(DM, &fe, &lds);
    if (rc != NCF_OK) return rc;
    FxArgs A;
    memset(&A, 0, sizeof(A));
    A.w0 = w0snap;
    A.g = gshard;
    A.gofs = shard_begin;
    A.xoff[0] = lay->um;
    A.xoff[1] = lay->im;
    A.mode = FX_DX;
    const int64_t nrows[2] = {lay->user_num, lay->item_num};
    const int64_t per = (int64_t)fact_ch(lay) * fact_cpb(lay);
    int64_t nb[2];
    for (int t = 0; t < 2; ++t) {  // the table's rows inside the shard (rows never straddle: 64-aligned)
        int64_t lo = (shard_begin - A.xoff[t] + DM - 1), hi = shard_begin + shard_len - A.xoff[t];
        lo = lo < 0 ? 0 : lo / DM;
        hi = hi < 0 ? 0 : hi / DM;
        if (hi > nrows[t]) hi = nrows[t];
        if (lo > hi) lo = hi;
        A.r0[t] = lo;
        A.r1[t] = hi;
        nb[t] = (hi - lo + per - 1) / per;
    }
    A.nbu = (int)nb[0];
    return launch_fx(fe, lds, A, (int)(nb[0] + nb[1]), st);
}

}  // namespace ncf

using namespace ncf;

extern "C" {

int ncf_abi_version(void) { return NCF_ABI_VERSION; }

int ncf_debug_set_diag(int flags) {
    g_diag = flags;
    return NCF_OK;
}

int ncf_debug_set_stamps(unsigned long long* dev_buf) {
    g_stamps = dev_buf;
    return NCF_OK;
}

int ncf_slab_rows(void) { return SLAB_ROWS; }

int ncf_fact_mode(const ncf_layout* lay) { return lay && fact_mode(lay) ? 1 : 0; }

int ncf_reduce_rows(const ncf_layout* lay) { return lay ? reduce_rows(lay) : -1; }

uint32_t ncf_dropout_hash(uint32_t seed, uint32_t t, uint32_t layer, int64_t row, uint32_t col) {
    return dropout_hash(seed, t, layer, row, col);
}

int64_t ncf_fact_partials_bytes(const ncf_layout* lay) {
    return lay && fact_mode(lay) ? fact_partials_floats(lay) * 4 : 0;
}

int ncf_layout_tune(ncf_layout* lay, int64_t rows) {
    if (!lay || rows <= 0) return NCF_E_ARG;
    int32_t f = lay->flags & ~(NCF_LAYOUT_PER_ROW_L0 | (NCF_LAYOUT_GEO_MASK << NCF_LAYOUT_GEO_SHIFT) |
                               (NCF_LAYOUT_WG_MASK << NCF_LAYOUT_WG_SHIFT) | NCF_LAYOUT_USER_STORE);
    if (g_per_row == 1 || (g_per_row < 0 && 2 * rows < (int64_t)lay->user_num + lay->item_num))
        f |= NCF_LAYOUT_PER_ROW_L0;
    lay->flags = f;
    // geometry: forced (ncf_debug_set_geometry), else 8-wave workgroups where the
    // batch has GEO_MIN_WGS 128-row tiles and 4-wave ones below (twice the workgroups,
    // one wave per SIMD).  Measured on the MI355X (profiles/r04_evidence/geometry_*):
    // C2 (1,024 rows) 22.3 / 19.1 / 19.8 / 20.8 us per step at 8 / 4 / 2 / 1 waves,
    // C5 (256) 13.3 / 12.4 / 12.8 / 13.2, the C3 step at 8,192 rows per rank 31.0 /
    // 27.5 (train launch); the 2- and 1-wave kernels stay for A/B.
    const KernelEntry* e = train_fused(lay);
    int g = GEO_8;
    if (e) {
        auto avail = [&](int gg) {
            lay->flags = f | (gg << NCF_LAYOUT_GEO_SHIFT);
            return train_geo(e, lay) == gg;
        };
        if (g_geo_waves != 0) {
            for (int gg = 0; gg < NGEO; ++gg)
                if (geo_waves(gg) == g_geo_waves && avail(gg)) g = gg;
        } else if ((rows + 127) / 128 < GEO_MIN_WGS && avail(GEO_4)) {
            g = GEO_4;
        }
    }
    f |= g << NCF_LAYOUT_GEO_SHIFT;
    // user store-and-sum (user_sum_kernel), when enabled: forced, or by the per-rank
    // batch (-1).  Off by default: at C3 the step kernel went 41.1 -> 39.2 us without
    // its user atomics but the sum launch took 11.0 us (and the user order 1.7 us per
    // step), 65.4 -> 75.6 us per step (profiles/r04_evidence/user_store_ab.json)
    lay->flags = f;
    if (us_applies(lay) && (g_user_store == 1 || (g_user_store < 0 && rows >= NCF_US_MIN_ROWS)))
        f |= NCF_LAYOUT_USER_STORE;
    const int tr = 16 * geo_waves(g);
    const int64_t tiles = (rows + tr - 1) / tr;
    if (tiles < SLAB_ROWS) f |= (int32_t)tiles << NCF_LAYOUT_WG_SHIFT;
    lay->flags = f;
    return NCF_OK;
}

int ncf_debug_set_per_row(int mode) {
    if (mode < -1 || mode > 1) return NCF_E_ARG;
    g_per_row = mode;
    return NCF_OK;
}

int ncf_debug_set_user_store(int mode) {
    if (mode < -1 || mode > 1) return NCF_E_ARG;
    g_user_store = mode;
    return NCF_OK;
}

int ncf_debug_set_geometry(int waves) {
    if (waves != 0 && waves != 1 && waves != 2 && waves != 4 && waves != NWAVES) return NCF_E_ARG;
    g_geo_waves = waves;
    return NCF_OK;
}

int ncf_layout_init(int U, int I, int F, int L, int mode, ncf_layout* o) {
    if (!o || U <= 0 || I <= 0 || F <= 0 || L < 1 || L > 4 || mode < 0 || mode > 2) return NCF_E_ARG;
    memset(o, 0, sizeof(*o));
    const int64_t DM = (int64_t)F << (L - 1);
    const int64_t P = mode == NCF_MODEL_NEUMF ? 2 * F : F;
    int64_t off = 0;
    o->ug = off; off += rup64((int64_t)U * F);
    o->ig = off; off += rup64((int64_t)I * F);
    o->um = off; off += rup64((int64_t)U * DM);
    o->im = off; off += rup64((int64_t)I * DM);
    o->tower_begin = off;
    for (int k = 0; k < 4; ++k) {
        if (k < L) {
            const int64_t si = (2 * DM) >> k, so = si / 2;
            o->w[k] = off; off += rup64(so * si);
            o->b[k] = off; off += rup64(so);
        } else {
            o->w[k] = -1;
            o->b[k] = -1;
        }
    }
    o->wp = off; off += rup64(P);
    o->bp = off; off += 64;
    o->tower_len = off - o->tower_begin;
    off += 64;  // loss slot + pad
    o->total = off;
    o->user_num = U; o->item_num = I; o->factor_num = F; o->num_layers = L; o->model_type = mode;
    return NCF_OK;
}

int ncf_supported(int mode, int F, int L) {
    ncf_layout lay;
    if (ncf_layout_init(1, 1, F, L, mode, &lay) != NCF_OK) return 0;
    if (fused_entry(&lay)) return NCF_PATH_FUSED;
    return F <= LYR_MAX_FACTOR ? NCF_PATH_LAYERED : 0;
}

// fused-path workspace: slab rows, [factored: dW0 partials, W0 snapshot], [user store]
static int64_t us_base_floats(const ncf_layout* lay) {
    return (int64_t)SLAB_ROWS * ncf_slab_stride(lay) +
           (fact_mode(lay) ? fact_partials_floats(lay) + fact_w0_snap_floats(lay) : 0);
}

int64_t ncf_workspace_bytes(const ncf_layout* lay, int64_t rows) {
    if (!lay || rows < 0) return -1;
    if (train_fused(lay))
        return (us_base_floats(lay) + us_floats(lay, rows)) * 4;
    return lyr_workspace_floats(lay, rows, true, fact_mode(lay) ? fact_partials_floats(lay) : -1) * 4;
}

int64_t ncf_forward_workspace_bytes(const ncf_layout* lay, int64_t n) {
    if (!lay || n < 0) return -1;
    if (fused_entry(lay)) return 0;
    return lyr_workspace_floats(lay, n, false, -1) * 4;
}

static int train_step_impl(const ncf_layout* lay, const float* params, float* grads, const uint64_t* rows,
                           const int64_t* user_order, const float* dlogit, ncf_step_ctl* ctl, int64_t batch_global,
                           int world, int rank,
                           int dz_mode, float kd_wt, float kd_wr, float kd_temp, void* workspace,
                           int64_t workspace_bytes,
                           float* logits_out, void* stream) {
    if (!lay || !params || !grads || !rows || !ctl || !workspace) return NCF_E_ARG;
    if (batch_global <= 0 || world < 1 || rank < 0 || rank >= world) return NCF_E_ARG;
    if (dz_mode != NCF_DZ_BCE && dz_mode != NCF_DZ_DLOGIT && dz_mode != NCF_DZ_KD) return NCF_E_ARG;
    if (dz_mode != NCF_DZ_BCE && !dlogit) return NCF_E_ARG;
    const int64_t rows_max = (batch_global + world - 1) / world;
    if (workspace_bytes < ncf_workspace_bytes(lay, rows_max)) return NCF_E_ARG;
    float* slab = static_cast<float*>(workspace);
    const KernelEntry* e = train_fused(lay);
    if (!e) {
        LyrArgs la;
        memset(&la, 0, sizeof(la));
        la.lay = *lay;
        la.params = params;
        la.grads = grads;
        la.rows = rows;
        la.uorder = ncf_uses_user_order(lay) ? user_order : nullptr;
        la.dlogit = dlogit;
        la.ctl = ctl;
        la.batch_global = batch_global;
        la.world = world;
        la.rank = rank;
        la.dz_mode = dz_mode;
        la.kd_wt = kd_wt;
        la.kd_wr = kd_wr;
        la.kd_temp = kd_temp;
        la.logits_out = logits_out;
        la.fact_part_floats = fact_mode(lay) ? fact_partials_floats(lay) : -1;
        const int rc = lyr_run(la, slab, rows_max, true, (hipStream_t)stream);
        if (rc != NCF_OK || la.fact_part_floats < 0) return rc;
        return launch_fact_expand(lay, params, grads, fact_partials(lay, workspace), nullptr, (hipStream_t)stream);
    }
    const int geo = train_geo(e, lay);
    const int64_t lds = train_lds_floats(e, lay, geo) * 4;
    if (lds > LDS_LIMIT_BYTES) return NCF_E_UNSUPPORTED;
    const void* fn = fact_mode(lay) ? e->train_fact[geo] : e->train[geo];
    if (ensure_lds(fn, lds) != NCF_OK) return NCF_E_LAUNCH;
    TrainArgs a;
    memset(&a, 0, sizeof(a));
    a.lay = *lay;
    a.params = params;
    a.grads = grads;
    a.rows = rows;
    // BCE mode: point dlogit at the rows so the per-row load stays unconditional
    a.dlogit = dz_mode != NCF_DZ_BCE ? dlogit : reinterpret_cast<const float*>(rows);
    a.ctl = ctl;
    a.batch_global = batch_global;
    a.world = world;
    a.rank = rank;
    a.dz_mode = dz_mode;
    a.kd_wt = kd_wt;
    a.kd_wr = kd_wr;
    a.kd_temp = kd_temp;
    a.diag = g_diag;
    a.stamps = g_stamps;
    a.slab = slab;
    a.logits_out = logits_out;
    const bool us = us_on(lay) && user_order != nullptr;
    if (us) {
        a.ustore = slab + us_base_floats(lay);
        a.uw = us_uw(lay);
    }
    void* args[] = {&a};
    if (hipLaunchKernel(fn, dim3(slab_rows_of(lay)), dim3(geo_waves(geo) * WAVE), args, (size_t)lds,
                        (hipStream_t)stream) != hipSuccess)
        return NCF_E_LAUNCH;
    int rc = launch_status();
    if (rc != NCF_OK) return rc;
    if (us) {  // the stored user-side rows summed per user (before the factored expansion reads G)
        UsArgs ua;
        memset(&ua, 0, sizeof(ua));
        ua.ustore = a.ustore;
        ua.order = user_order;
        ua.grads = grads;
        ua.ctl = ctl;
        ua.batch_global = batch_global;
        ua.um = lay->um;
        ua.ug = lay->ug;
        ua.world = world;
        ua.rank = rank;
        ua.uw = a.uw;
        ua.dmu = lay->model_type != NCF_MODEL_GMF ? (lay->factor_num << (lay->num_layers - 1)) : 0;
        ua.f = lay->factor_num;
        const int64_t waves = (rows_max + US_SPAN - 1) / US_SPAN;
        const dim3 grid((unsigned)((waves + US_WAVES - 1) / US_WAVES)), blk(US_WAVES * 64);
        const hipStream_t st = (hipStream_t)stream;
        switch ((a.uw + 63) / 64) {
            case 1: hipLaunchKernelGGL(user_sum_kernel<1>, grid, blk, 0, st, ua); break;
            case 2: hipLaunchKernelGGL(user_sum_kernel<2>, grid, blk, 0, st, ua); break;
            case 3: hipLaunchKernelGGL(user_sum_kernel<3>, grid, blk, 0, st, ua); break;
            default: hipLaunchKernelGGL(user_sum_kernel<US_NCH>, grid, blk, 0, st, ua); break;
        }
        rc = launch_status();
        if (rc != NCF_OK) return rc;
    }
    if (!fact_mode(lay)) return rc;
    // factored layer 0: the per-user / per-item D0 sums -> dUm, dIm, dW0 partials
    return launch_fact_expand(lay, params, grads, fact_partials(lay, workspace), fact_w0_snap(lay, workspace),
                              (hipStream_t)stream);
}

int ncf_train_step(const ncf_layout* lay, const float* params, float* grads, const uint64_t* rows,
                   const int64_t* user_order, const float* dlogit, ncf_step_ctl* ctl, int64_t batch_global,
                   int world, int rank,
                   int dz_mode, void* workspace, int64_t workspace_bytes, float* logits_out, void* stream) {
    if (dz_mode == NCF_DZ_KD) return NCF_E_ARG;  // ncf_train_step_kd carries the weights
    return train_step_impl(lay, params, grads, rows, user_order, dlogit, ctl, batch_global, world, rank, dz_mode, 0.f,
                           0.f, 0.f,
                           workspace, workspace_bytes, logits_out, stream);
}

int ncf_train_step_kd(const ncf_layout* lay, const float* params, float* grads, const uint64_t* rows,
                      const int64_t* user_order, const float* teacher_logits, ncf_step_ctl* ctl,
                      int64_t batch_global, int world, int rank,
                      float w_task, float w_resp, float temperature, void* workspace, int64_t workspace_bytes,
                      float* logits_out, void* stream) {
    if (!teacher_logits) return NCF_E_ARG;
    return train_step_impl(lay, params, grads, rows, user_order, teacher_logits, ctl, batch_global, world, rank, NCF_DZ_KD,
                           w_task, w_resp, temperature, workspace, workspace_bytes, logits_out, stream);
}

// ---- the previous step's Adam inside the training launch (ABI 18, NCF_LAYOUT_ADAM_IN_STEP)
}  // extern "C"

namespace ncf {

// The fused kernel with the in-step optimizer for this layout and its geometry, or null.
static const void* ais_kernel(const ncf_layout* lay, int* geo) {
    const KernelEntry* e = train_fused(lay);
    if (!e || fact_mode(lay) || us_on(lay)) return nullptr;
    const int g = train_geo(e, lay);
    *geo = g;
    return e->train_ais[g];
}

// ncf_ais_begin: no update pending, S_{adam_t} in buffer 0; the three gradient buffers
// cleared over the active ranges and the loss slot.
__global__ __launch_bounds__(256) void ais_begin_kernel(ncf_step_ctl* ctl, int64_t* st, float* g0, float* g1, float* g2,
                                                        Ranges R, int64_t loss_i) {
    const int64_t total = R.prefix[R.n];
    const f4 z = f4{0.f, 0.f, 0.f, 0.f};
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (int64_t)gridDim.x * blockDim.x) {
        int which;
        const int64_t i = range_locate(R, q, &which);
        *reinterpret_cast<f4*>(g0 + i) = z;
        *reinterpret_cast<f4*>(g1 + i) = z;
        *reinterpret_cast<f4*>(g2 + i) = z;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        g0[loss_i] = g1[loss_i] = g2[loss_i] = 0.f;
        st[0] = 0;
        st[1] = ctl->adam_t & 1;
    }
}

// ncf_ais_bump: a chunk of k launches done -- k batches, k - 1 + pending updates applied,
// one pending for the next launch.
__global__ void ais_bump_kernel(ncf_step_ctl* ctl, int64_t* st, int64_t k) {
    if (threadIdx.x == 0) {
        const int64_t pend0 = st[0];
        ctl->adam_t = ctl->adam_t + k - 1 + pend0;
        ctl->batch = ctl->batch + k;
        st[0] = 1;
    }
}

// ncf_ais_flush, first launch: the pending update written into buffer 0 (or, with
// none pending, S_{adam_t} copied there from buffer 1), its loss recorded, its gradient
// cleared; reads ctl / st only (the second launch advances them).
__global__ __launch_bounds__(256) void ais_flush_kernel(AisArgs x, ncf_step_ctl* ctl, int64_t loss_i) {
#pragma clang fp contract(off)
    __shared__ float sc[2];
    const int64_t pend = x.st[0], par = x.st[1];
    const int64_t n = ctl->adam_t + 1;
    const int rb = (int)((pend ? n - 1 + par : ctl->adam_t + par) & 1);
    const ScCache sce = sc_peek(x.scc, n);
    float* gr = x.g[n % 3];
    if (pend) {
        if (blockIdx.x == 0 && threadIdx.x == 0 && x.loss_hist != nullptr && x.hist_len > 0) {
            const int64_t b = ctl->batch - 1;
            x.loss_hist[((b % x.hist_len) + x.hist_len) % x.hist_len] = gr[loss_i];
        }
        sc_resolve(sce, n, x.lr, x.beta1, x.beta2, sc);
        step_scalars_ahead(x.scc, n, x.lr, x.beta1, x.beta2);
    }
    __syncthreads();
    if (!pend && rb == 0) return;  // block-uniform: already in buffer 0
    const float neg_step = sc[0], bc2s = sc[1];
    const float w1 = (float)(1.0 - x.beta1), b2 = (float)x.beta2, omb2 = (float)(1.0 - x.beta2);
    const int64_t total = x.R.prefix[x.R.n];
    const f4 z = f4{0.f, 0.f, 0.f, 0.f};
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (int64_t)gridDim.x * blockDim.x) {
        int which;
        const int64_t i = range_locate(x.R, q, &which);
        f4 pp = *reinterpret_cast<const f4*>(x.p[rb] + i), mm = *reinterpret_cast<const f4*>(x.m[rb] + i),
           vv = *reinterpret_cast<const f4*>(x.v[rb] + i);
        if (pend) {
            const f4 gg = *reinterpret_cast<const f4*>(gr + i);
            adam_f4(pp, mm, vv, gg, w1, b2, omb2, bc2s, x.eps, neg_step);
            *reinterpret_cast<f4*>(gr + i) = z;
        }
        *reinterpret_cast<f4*>(x.p[0] + i) = pp;
        *reinterpret_cast<f4*>(x.m[0] + i) = mm;
        *reinterpret_cast<f4*>(x.v[0] + i) = vv;
    }
    if (pend && blockIdx.x == 0 && threadIdx.x == 0) gr[loss_i] = 0.f;
}

__global__ void ais_flush_done_kernel(ncf_step_ctl* ctl, int64_t* st) {
    if (threadIdx.x == 0) {
        const int64_t t = ctl->adam_t + st[0];
        ctl->adam_t = t;
        st[0] = 0;
        st[1] = t & 1;
    }
}

static int ais_args(const ncf_layout* lay, float* params, float* grads, float* exp_avg, float* exp_avg_sq,
                    const ncf_ais_bufs* b, const int64_t* ranges, int nranges, AisArgs* x) {
    if (!lay || !params || !grads || !exp_avg || !exp_avg_sq || !b || !ranges) return NCF_E_ARG;
    if (!b->params_b || !b->exp_avg_b || !b->exp_avg_sq_b || !b->grads_1 || !b->grads_2 || !b->state) return NCF_E_ARG;
    memset(x, 0, sizeof(*x));
    int err = 0;
    x->R = make_ranges(ranges, nranges, &err);
    if (err) return NCF_E_ARG;
    for (int i = 0; i < nranges; ++i)  // every active float inside the flat buffers
        if (ranges[2 * i + 1] > lay->total) return NCF_E_ARG;
    x->p[0] = params;
    x->p[1] = b->params_b;
    x->m[0] = exp_avg;
    x->m[1] = b->exp_avg_b;
    x->v[0] = exp_avg_sq;
    x->v[1] = b->exp_avg_sq_b;
    x->g[0] = grads;
    x->g[1] = b->grads_1;
    x->g[2] = b->grads_2;
    x->st = b->state;
    return NCF_OK;
}

static unsigned ais_grid(const Ranges& R, int64_t cap) {
    int64_t g = (R.prefix[R.n] + 255) / 256;
    if (g > cap) g = cap;
    return (unsigned)(g < 1 ? 1 : g);
}

}  // namespace ncf

extern "C" {

int ncf_ais_supported(const ncf_layout* lay) {
    int geo = 0;
    return (lay && ais_kernel(lay, &geo) != nullptr) ? 1 : 0;
}

int ncf_ais_begin(const ncf_layout* lay, float* params, float* grads, float* exp_avg, float* exp_avg_sq,
                  const ncf_ais_bufs* b, const int64_t* ranges, int nranges, ncf_step_ctl* ctl, void* stream) {
    AisArgs x;
    const int rc = ais_args(lay, params, grads, exp_avg, exp_avg_sq, b, ranges, nranges, &x);
    if (rc != NCF_OK) return rc;
    if (!ctl) return NCF_E_ARG;
    const hipStream_t st = (hipStream_t)stream;
    const size_t bytes = (size_t)lay->total * 4;  // buffer 1 = buffer 0 (inactive floats stay equal)
    if (hipMemcpyAsync(b->params_b, params, bytes, hipMemcpyDeviceToDevice, st) != hipSuccess ||
        hipMemcpyAsync(b->exp_avg_b, exp_avg, bytes, hipMemcpyDeviceToDevice, st) != hipSuccess ||
        hipMemcpyAsync(b->exp_avg_sq_b, exp_avg_sq, bytes, hipMemcpyDeviceToDevice, st) != hipSuccess)
        return NCF_E_LAUNCH;
    hipLaunchKernelGGL(ais_begin_kernel, dim3(ais_grid(x.R, 1024)), dim3(256), 0, st, ctl, b->state, grads, b->grads_1,
                       b->grads_2, x.R, lay->tower_begin + lay->tower_len);
    return launch_status();
}

int ncf_train_step_ais(const ncf_layout* lay, float* params, float* grads, float* exp_avg, float* exp_avg_sq,
                       const ncf_ais_bufs* b, const int64_t* ranges, int nranges, const uint64_t* rows,
                       const float* dlogit, ncf_step_ctl* ctl, int64_t batch_global, int dz_mode, float kd_wt,
                       float kd_wr, float kd_temp, double lr, double beta1, double beta2, double eps,
                       float* loss_hist, int64_t hist_len, int64_t step_i, void* stream) {
    AisArgs x;
    int rc = ais_args(lay, params, grads, exp_avg, exp_avg_sq, b, ranges, nranges, &x);
    if (rc != NCF_OK) return rc;
    if (!rows || !ctl || batch_global <= 0 || step_i < 0) return NCF_E_ARG;
    if (dz_mode != NCF_DZ_BCE && dz_mode != NCF_DZ_DLOGIT && dz_mode != NCF_DZ_KD) return NCF_E_ARG;
    if (dz_mode != NCF_DZ_BCE && !dlogit) return NCF_E_ARG;
    int geo = 0;
    const void* fn = ais_kernel(lay, &geo);
    if (!fn) return NCF_E_UNSUPPORTED;
    const KernelEntry* e = train_fused(lay);
    const int64_t lds = train_lds_floats(e, lay, geo) * 4;
    if (lds > LDS_LIMIT_BYTES) return NCF_E_UNSUPPORTED;
    if (ensure_lds(fn, lds) != NCF_OK) return NCF_E_LAUNCH;
    x.lr = lr;
    x.beta1 = beta1;
    x.beta2 = beta2;
    x.eps = (float)eps;
    x.loss_hist = loss_hist;
    x.hist_len = hist_len;
    x.scc = sc_cache_for(ctl, stream);
    x.step_i = step_i;
    x.ntrain = slab_rows_of(lay);
    TrainArgs a;
    memset(&a, 0, sizeof(a));
    a.lay = *lay;
    a.params = params;
    a.grads = grads;
    a.rows = rows;
    a.dlogit = dz_mode != NCF_DZ_BCE ? dlogit : reinterpret_cast<const float*>(rows);
    a.ctl = ctl;
    a.batch_global = batch_global;
    a.world = 1;
    a.rank = 0;
    a.dz_mode = dz_mode;
    a.kd_wt = kd_wt;
    a.kd_wr = kd_wr;
    a.kd_temp = kd_temp;
    a.diag = g_diag;
    a.stamps = g_stamps;
    a.ais = x;
    // the dense update over every active float by the workgroups past the training ones:
    // a few, so their bursts of loads do not queue ahead of the training workgroups'
    // dependent round trips (NCF_AIS_EXTRA, default 192)
    static const int extra_cap = [] {
        const char* e = getenv("NCF_AIS_EXTRA");
        const int v = e ? atoi(e) : 192;
        return v < 1 ? 1 : (v > 1024 ? 1024 : v);
    }();
    const int64_t t4 = x.R.prefix[x.R.n];  // float4 of the update; two per thread
    int64_t extra = (t4 + 2 * 256 - 1) / (2 * 256);
    if (extra > extra_cap) extra = extra_cap;
    if (extra < 1) extra = 1;
    void* args[] = {&a};  // + 1: the step-scalar workgroup (ais_dense_block)
    if (hipLaunchKernel(fn, dim3((unsigned)(x.ntrain + extra + 1)), dim3(geo_waves(geo) * WAVE), args,
                        (size_t)lds, (hipStream_t)stream) != hipSuccess)
        return NCF_E_LAUNCH;
    return launch_status();
}

int ncf_ais_bump(ncf_step_ctl* ctl, const ncf_ais_bufs* b, int64_t k, void* stream) {
    if (!ctl || !b || !b->state || k < 1) return NCF_E_ARG;
    hipLaunchKernelGGL(ais_bump_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, ctl, b->state, k);
    return launch_status();
}

int ncf_ais_flush(const ncf_layout* lay, float* params, float* grads, float* exp_avg, float* exp_avg_sq,
                  const ncf_ais_bufs* b, const int64_t* ranges, int nranges, ncf_step_ctl* ctl, double lr,
                  double beta1, double beta2, double eps, float* loss_hist, int64_t hist_len, void* stream) {
    AisArgs x;
    const int rc = ais_args(lay, params, grads, exp_avg, exp_avg_sq, b, ranges, nranges, &x);
    if (rc != NCF_OK) return rc;
    if (!ctl) return NCF_E_ARG;
    x.lr = lr;
    x.beta1 = beta1;
    x.beta2 = beta2;
    x.eps = (float)eps;
    x.loss_hist = loss_hist;
    x.hist_len = hist_len;
    x.scc = sc_cache_for(ctl, stream);
    const hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(ais_flush_kernel, dim3(ais_grid(x.R, 1024)), dim3(256), 0, st, x, ctl,
                       lay->tower_begin + lay->tower_len);
    if (launch_status() != NCF_OK) return NCF_E_LAUNCH;
    hipLaunchKernelGGL(ais_flush_done_kernel, dim3(1), dim3(64), 0, st, ctl, b->state);
    return launch_status();
}

int ncf_kd_feature_step(const ncf_layout* student, const float* s_params, float* s_grads, const ncf_layout* teacher,
                        const float* t_params, const uint64_t* rows, const ncf_step_ctl* ctl, int64_t batch_global,
                        int world, int rank, const float* gmf_w, const float* gmf_b, float gmf_coef,
                        const float* mlp_w, const float* mlp_b, float mlp_coef, void* workspace, void* stream) {
    if (!student || !s_params || !s_grads || !teacher || !t_params || !rows || !ctl || !workspace) return NCF_E_ARG;
    if (batch_global <= 0 || world < 1 || rank < 0 || rank >= world) return NCF_E_ARG;
    KdFeatArgs a;
    memset(&a, 0, sizeof(a));
    a.sl = *student;
    a.tl = *teacher;
    a.sp = s_params;
    a.sg = s_grads;
    a.tp = t_params;
    a.rows = rows;
    a.ctl = ctl;
    a.batch_global = batch_global;
    a.world = world;
    a.rank = rank;
    const int fs = student->factor_num, ft = teacher->factor_num;
    const int ms = 2 * (student->factor_num << (student->num_layers - 1));
    const int mt = 2 * (teacher->factor_num << (teacher->num_layers - 1));
    a.key[0] = KdKey{gmf_w, gmf_b, gmf_coef, fs, ft};
    a.key[1] = KdKey{mlp_w, mlp_b, mlp_coef, ms, mt};
    for (int k = 0; k < 2; ++k) {
        const KdKey& K = a.key[k];
        if (K.coef == 0.f) continue;
        if (K.A == nullptr && K.S != K.T) return NCF_E_ARG;   // identity needs equal widths
        if (K.A != nullptr && K.c == nullptr) return NCF_E_ARG;
        if (K.S > (k == 0 ? 64 : KD_MAXS) || K.T > (k == 0 ? 64 : KD_MAXT)) return NCF_E_UNSUPPORTED;
    }
    a.loss_out = static_cast<float*>(workspace) + student->tower_len;  // slab row 0, loss column
    const int64_t per = (batch_global + world - 1) / world;
    int64_t grid = (per + KD_WAVES - 1) / KD_WAVES;
    if (grid > 2048) grid = 2048;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(kd_feature_kernel, dim3((unsigned)grid), dim3(64 * KD_WAVES), 0, (hipStream_t)stream, a);
    return launch_status();
}

int ncf_forward(const ncf_layout* lay, const float* params, const uint64_t* rows, int64_t n, float* logits,
                void* workspace, int64_t workspace_bytes, void* stream) {
    if (!lay || !params || !rows || !logits || n < 0) return NCF_E_ARG;
    if (n == 0) return NCF_OK;
    const KernelEntry* e = find_entry(lay->model_type, lay->factor_num, lay->num_layers);
    if (!fused_entry(lay)) {
        if (!workspace || workspace_bytes < ncf_forward_workspace_bytes(lay, n)) return NCF_E_ARG;
        LyrArgs la;
        memset(&la, 0, sizeof(la));
        la.lay = *lay;
        la.params = params;
        la.rows = rows;
        la.fwd_n = n;
        la.world = 1;
        la.logits_out = logits;
        la.fact_part_floats = -1;
        return lyr_run(la, static_cast<float*>(workspace), n, false, (hipStream_t)stream);
    }
    const int64_t lds = (int64_t)(e->w_total + e->misc[GEO_8]) * 4;
    if (lds > LDS_LIMIT_BYTES) return NCF_E_UNSUPPORTED;
    if (ensure_lds(e->fwd, lds) != NCF_OK) return NCF_E_LAUNCH;
    TrainArgs a;
    memset(&a, 0, sizeof(a));
    a.lay = *lay;
    a.params = params;
    a.rows = rows;
    a.logits_out = logits;
    a.fwd_n = n;
    a.world = 1;
    const int64_t ntiles = (n + TILE_ROWS - 1) / TILE_ROWS;
    const int grid = (int)(ntiles < 2 * SLAB_ROWS ? ntiles : 2 * SLAB_ROWS);
    void* args[] = {&a};
    if (hipLaunchKernel(e->fwd, dim3(grid), dim3(NTHREADS), args, (size_t)lds, (hipStream_t)stream) != hipSuccess)
        return NCF_E_LAUNCH;
    return launch_status();
}

int64_t ncf_slab_stride(const ncf_layout* lay) { return lay ? lay->tower_len + 64 : -1; }

int ncf_reduce_slab(const ncf_layout* lay, const void* workspace, float* grads, ncf_step_ctl* ctl, void* stream) {
    if (!lay || !workspace || !grads) return NCF_E_ARG;
    const float* slab = static_cast<const float*>(workspace);
    const int stride = (int)ncf_slab_stride(lay);
    const int lo = slab_lo(lay);
    const int blocks = (stride - lo + 63) / 64;
    const int rows = reduce_rows(lay);
    hipLaunchKernelGGL(reduce_slab_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, slab,
                       grads + lay->tower_begin, lo, stride, rows, ctl, w0_part(lay, workspace));
    return launch_status();
}

int ncf_adam_step(float* params, float* grads, float* exp_avg, float* exp_avg_sq, const int64_t* ranges,
                  int nranges, ncf_step_ctl* ctl, double lr, double beta1, double beta2, double eps,
                  int64_t loss_slot, float* loss_hist, int64_t hist_len, void* stream) {
    if (!params || !grads || !exp_avg || !exp_avg_sq || !ranges || !ctl) return NCF_E_ARG;
    int err = 0;
    Ranges R = make_ranges(ranges, nranges, &err);
    if (err) return NCF_E_ARG;
    const int64_t total = R.prefix[R.n];
    int64_t grid = (total + 511) / 512;  // two float4 per thread
    if (grid > 4096) grid = 4096;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(adam_kernel, dim3((int)grid), dim3(256), 0, (hipStream_t)stream, params, grads, exp_avg,
                       exp_avg_sq, R, ctl, lr, beta1, beta2, (float)eps, loss_slot, loss_hist, hist_len,
                       sc_cache_for(ctl, stream));
    return launch_status();
}

// Sharded Adam of the factored path (dp_mode "zero1" with NCF_LAYOUT_FACT_DEFER_DX):
// the reduce-scattered gradient shard holds, in its Um / Im rows, the summed
// per-entity D0 sums G (the train step expanded only the dW0 partials), so the rank
// that owns them forms dX = G W0half (the W0 the step ran with, from the snapshot)
// and Adam applies it -- one launch, adam_fact_shard_kernel (each window of table rows
// inside one active range, at most 8 other ranges), else fact_expand_kernel's FX_DX
// mode in place and the plain Adam launch.  The same launch clears the local gradient
// bucket (grads_local, grads_n floats) for the next step.  The shard is 64-float
// aligned and DM divides 64 (and the table offsets), so a G row never straddles two
// shards; its length is the ranges' largest end.
int ncf_adam_step_fact(const ncf_layout* lay, const void* workspace, float* params, float* gshard,
                       float* exp_avg, float* exp_avg_sq, const int64_t* ranges, int nranges, int64_t shard_begin,
                       float* grads_local, int64_t grads_n, ncf_step_ctl* ctl, double lr, double beta1, double beta2,
                       double eps, int64_t loss_slot, float* loss_hist, int64_t hist_len, void* stream) {
    if (!lay || !workspace || !params || !gshard || !exp_avg || !exp_avg_sq || !ranges || !ctl || nranges <= 0)
        return NCF_E_ARG;
    if (grads_n < 0 || (grads_n & 3) || (grads_n > 0 && !grads_local)) return NCF_E_ARG;
    const int dm = fact_dm(lay);
    if (!fact_mode(lay) || !train_fused(lay) || dm > 64 || (shard_begin & 63) || (lay->um % dm) || (lay->im % dm) ||
        !(lay->flags & NCF_LAYOUT_FACT_DEFER_DX))
        return NCF_E_UNSUPPORTED;
    int err = 0;
    (void)make_ranges(ranges, nranges, &err);
    if (err) return NCF_E_ARG;
    const hipStream_t st = (hipStream_t)stream;
    int64_t shard_len = 0;
    for (int r = 0; r < nranges; ++r) shard_len = ranges[2 * r + 1] > shard_len ? ranges[2 * r + 1] : shard_len;
    const float* w0s = fact_w0_snap(lay, const_cast<void*>(workspace));
    FsArgs A;
    memset(&A, 0, sizeof(A));
    // the Um / Im rows inside the shard (rows never straddle: 64-aligned shard, DM | 64)
    const int64_t xoff[2] = {lay->um, lay->im}, nrows[2] = {lay->user_num, lay->item_num};
    int64_t wb[2], we[2];  // shard-relative windows
    int nbt[2];
    const int CH = fact_ch(lay);
    for (int t = 0; t < 2; ++t) {
        int64_t lo = shard_begin - xoff[t] + dm - 1, hi = shard_begin + shard_len - xoff[t];
        lo = lo < 0 ? 0 : lo / dm;
        hi = hi < 0 ? 0 : hi / dm;
        if (hi > nrows[t]) hi = nrows[t];
        if (lo > hi) lo = hi;
        A.r0[t] = lo;
        A.r1[t] = hi;
        A.xrel[t] = xoff[t] - shard_begin;
        wb[t] = A.xrel[t] + lo * dm;
        we[t] = A.xrel[t] + hi * dm;
        nbt[t] = (int)((hi - lo + CH - 1) / CH);
    }
    // the active ranges minus the windows; each window wholly inside one active range
    // (else the two-launch form below)
    int64_t ra[16];
    int nra = 0;
    bool fused = fact_cpb(lay) == 1;
    for (int t = 0; t < 2 && fused; ++t) {
        if (we[t] <= wb[t]) continue;
        bool cov = false;
        for (int r = 0; r < nranges; ++r) cov |= ranges[2 * r] <= wb[t] && we[t] <= ranges[2 * r + 1];
        fused = cov;
    }
    for (int r = 0; r < nranges && fused; ++r) {
        int64_t pieces[6] = {ranges[2 * r], ranges[2 * r + 1]};
        int np = 1;
        for (int t = 0; t < 2; ++t) {
            if (we[t] <= wb[t]) continue;
            int64_t out[6];
            int no = 0;
            for (int k = 0; k < np; ++k) {
                const int64_t b = pieces[2 * k], e = pieces[2 * k + 1];
                if (we[t] <= b || e <= wb[t]) { out[2 * no] = b; out[2 * no + 1] = e; ++no; continue; }
                if (b < wb[t]) { out[2 * no] = b; out[2 * no + 1] = wb[t]; ++no; }
                if (we[t] < e) { out[2 * no] = we[t]; out[2 * no + 1] = e; ++no; }
            }
            np = no;
            for (int k = 0; k < 2 * np; ++k) pieces[k] = out[k];
        }
        for (int k = 0; k < np && fused; ++k) {
            if (pieces[2 * k + 1] <= pieces[2 * k]) continue;
            if (nra == 8) { fused = false; break; }
            ra[2 * nra] = pieces[2 * k];
            ra[2 * nra + 1] = pieces[2 * k + 1];
            ++nra;
        }
    }
    if (!fused) {  // two launches (+ the clear): the expansion in place, then the plain Adam
        if (grads_n > 0) {
            const int rc0 = launch_zero_f32(grads_local, grads_n, st);
            if (rc0 != NCF_OK) return rc0;
        }
        const int rc = launch_fact_dx(lay, w0s, gshard, shard_begin, shard_len, st);
        if (rc != NCF_OK) return rc;
        return ncf_adam_step(params, gshard, exp_avg, exp_avg_sq, ranges, nranges, ctl, lr, beta1, beta2, eps,
                             loss_slot, loss_hist, hist_len, stream);
    }
    if (nra == 0) {  // nothing outside the windows: an empty range keeps the loss bookkeeping
        ra[0] = ra[1] = 0;
        nra = 1;
    }
    A.RA = make_ranges(ra, nra, &err);
    if (err) return NCF_E_ARG;
    A.p = params;
    A.g = gshard;
    A.m = exp_avg;
    A.v = exp_avg_sq;
    A.w0s = w0s;
    A.nbu = nbt[0];
    A.nbx = nbt[0] + nbt[1];
    const int64_t na4 = A.RA.prefix[A.RA.n];
    int64_t nba = (na4 + FX_WAVES * 64 - 1) / (FX_WAVES * 64);
    A.nba = (int)(nba < 1 ? 1 : (nba > 512 ? 512 : nba));
    A.zero = reinterpret_cast<f4*>(grads_local);
    A.zn4 = grads_n / 4;
    int64_t nbz = (A.zn4 + 4 * FX_WAVES * 64 - 1) / (4 * FX_WAVES * 64);  // 4 f4 per thread
    if (nbz > 512) nbz = 512;
    A.ctl = ctl;
    A.lr = lr;
    A.beta1 = beta1;
    A.beta2 = beta2;
    A.eps = (float)eps;
    A.loss_slot = loss_slot;
    A.loss_hist = loss_hist;
    A.hist_len = hist_len;
    A.scc = sc_cache_for(ctl, stream);
    const void* fn;
    int64_t lds;
    switch (dm) {
#define NCF_FS(D) case D: fn = reinterpret_cast<const void*>(&adam_fact_shard_kernel<D>); lds = FxShape<D>::LDS; break;
        NCF_FS(8) NCF_FS(16) NCF_FS(32) NCF_FS(64)
#undef NCF_FS
        default: return NCF_E_UNSUPPORTED;
    }
    if (ensure_lds(fn, lds) != NCF_OK) return NCF_E_LAUNCH;
    void* ae[] = {&A};
    const unsigned grid = (unsigned)(A.nbx + A.nba + nbz);
    if (hipLaunchKernel(fn, dim3(grid), dim3(FX_WAVES * 64), ae, (size_t)lds, st) != hipSuccess) return NCF_E_LAUNCH;
    return launch_status();
}

int ncf_reduce_adam_step(const ncf_layout* lay, const void* workspace, float* params, float* grads, float* exp_avg,
                         float* exp_avg_sq, const int64_t* ranges, int nranges, ncf_step_ctl* ctl, double lr,
                         double beta1, double beta2, double eps, float* loss_hist, int64_t hist_len, void* stream) {
    if (!lay || !workspace || !params || !grads || !exp_avg || !exp_avg_sq || !ranges || !ctl) return NCF_E_ARG;
    if (lay->flags & NCF_LAYOUT_RETIRED_0X20) return NCF_E_UNSUPPORTED;
    int err = 0;
    Ranges R = make_ranges(ranges, nranges, &err);
    if (err) return NCF_E_ARG;
    // plain-Adam part of the active ranges: [begin, min(end, tower_begin)), the
    // embedding tables (their gradient is in grads)
    const int64_t plain_end = lay->tower_begin;
    int64_t er[16];
    int ne = 0;
    for (int i = 0; i < nranges; ++i) {
        const int64_t b = ranges[2 * i];
        const int64_t e = ranges[2 * i + 1] < plain_end ? ranges[2 * i + 1] : plain_end;
        if (e > b) {
            er[2 * ne] = b;
            er[2 * ne + 1] = e;
            ++ne;
        }
    }
    Ranges RE;
    memset(&RE, 0, sizeof(RE));
    if (ne > 0) {
        RE = make_ranges(er, ne, &err);
        if (err) return NCF_E_ARG;
    }
    const int stride = (int)ncf_slab_stride(lay);
    const int lo = slab_lo(lay);
    const int rows = reduce_rows(lay);
    const W0Part wp = w0_part(lay, workspace);
    // tower blocks: one float4 column per thread on the layered path (slab of <= 16 rows,
    // no dW0 partials): stress 857 -> 841 us/step; CLI unchanged; on the fused
    // small-batch step (C2: 16 rows, a 6K-float tower, 6 such blocks) the 16 x 16 form
    // stays, 18.6 against 19.7 us (profiles/r06_evidence/tower_col_ab/).  NCF_TOWER_COL=0:
    // the 16 x 16 form everywhere (A/B)
    static const bool col_ok = [] {
        const char* e = getenv("NCF_TOWER_COL");
        return !(e != nullptr && e[0] == '0');
    }();
    const int colmode = col_ok && rows <= 16 && wp.p == nullptr && train_fused(lay) == nullptr ? 1 : 0;
    const int nA = colmode ? ((stride - lo) / 4 + 1 + 255) / 256 : (stride - lo + 63) / 64;
    const int64_t etotal = RE.prefix[RE.n];
    int64_t nB = (etotal + 255) / 256;
    // embedding-Adam blocks at most: one float4 per thread up to 2M float4 (C4's 3.3M
    // float4: 8192 against 2048 blocks took the step 132.4 -> 129.8 us; 16384 / 65536 the
    // same as 8192; profiles/r06_evidence/adam_blocks_ab/).  NCF_ADAM_MAXB: A/B
    static const int64_t max_b = [] {
        const char* e = getenv("NCF_ADAM_MAXB");
        const long v = e ? atol(e) : 0;
        return (int64_t)(v > 0 ? v : 8192);
    }();
    if (nB > max_b) nB = max_b;
    hipLaunchKernelGGL(reduce_adam_kernel, dim3((unsigned)(nA + nB)), dim3(256), 0, (hipStream_t)stream,
                       static_cast<const float*>(workspace), lo, stride, rows, nA, lay->tower_begin, lay->tower_len,
                       params, grads, exp_avg, exp_avg_sq, R, RE, ctl, lr, beta1, beta2, (float)eps, loss_hist,
                       hist_len, wp, sc_cache_for(ctl, stream), colmode);
    return launch_status();
}

// ---- deferred Adam (ABI 14)
// C-list slice count: a row not touched by two consecutive batches falls at most
// this many steps behind (NCF_LAZY_SPAN, default 32, < LZ_WIN)
static int lazy_span() {
    static const int span = [] {
        const char* e = getenv("NCF_LAZY_SPAN");
        const int v = e ? atoi(e) : 32;
        return v < 1 ? 1 : (v > LZ_WIN - 2 ? LZ_WIN - 2 : v);
    }();
    return span;
}

constexpr int LZ_MAX_ROWS = 1 << 19;  // per side: two LDS bitmaps of the ids in ncf_batch_touched

static int lazy_args(const ncf_layout* lay, float* params, float* grads, float* m, float* v, const int64_t* ranges,
                     int nranges, int32_t* last, float* ring, int64_t ring_n, LazyArgs* a) {
    const int f = lay->factor_num, dm = f << (lay->num_layers - 1);
    if (f % 4 != 0 || lay->user_num > LZ_MAX_ROWS || lay->item_num > LZ_MAX_ROWS) return NCF_E_UNSUPPORTED;
    const int64_t offs[4] = {lay->ug, lay->ig, lay->um, lay->im};
    const int64_t widths[4] = {f, f, dm, dm};
    const int64_t nrows[4] = {lay->user_num, lay->item_num, lay->user_num, lay->item_num};
    memset(a, 0, sizeof(*a));
    for (int k = 0; k < 4; ++k) {
        const int64_t b = offs[k], e = offs[k] + nrows[k] * widths[k];
        bool act = false;
        for (int i = 0; i < nranges; ++i)
            if (ranges[2 * i] < e && ranges[2 * i + 1] > b) act = true;
        a->off[k] = act ? offs[k] : -1;
        a->w4[k] = (int)(widths[k] / 4);
    }
    a->p = params;
    a->g = grads;
    a->m = m;
    a->v = v;
    a->U = lay->user_num;
    a->I = lay->item_num;
    a->last = last;
    a->ring = ring;
    a->ring_n = ring_n;
    return NCF_OK;
}

// touched-list geometry: batches, per-batch A slots per side, id capacity
struct TouchedShape {
    int64_t nb, su, si, segs, cap;
};

static TouchedShape touched_shape(int64_t n, int64_t B, int U, int I) {
    TouchedShape t;
    t.nb = (n + B - 1) / B;
    t.su = U < B ? U : B;
    t.si = I < B ? I : B;
    t.segs = 6 * t.nb + 1;
    const int span = lazy_span();
    // per batch and side: |A| + |B| <= min(N, 2 min(N, B)), |C| <= N / span + 1; the
    // last batch lists every id once
    const int64_t ab = (U < 2 * t.su ? U : 2 * t.su) + (I < 2 * t.si ? I : 2 * t.si);
    t.cap = t.nb * (ab + U / span + I / span + 2) + U + I;
    return t;
}

int64_t ncf_touched_bytes(int64_t n, int64_t batch_global, int user_num, int item_num) {
    if (n <= 0 || batch_global <= 0 || user_num <= 0 || item_num <= 0) return -1;
    const TouchedShape t = touched_shape(n, batch_global, user_num, item_num);
    return (8 * t.segs + 4 * t.cap + 15) / 16 * 16;
}

static void touched_lists(LazyArgs* a, const int32_t* touched, const TouchedShape& t) {
    a->nb = t.nb;
    a->seg = reinterpret_cast<const int64_t*>(touched);
    a->ids = touched + 2 * t.segs;
}

int ncf_batch_touched(const uint64_t* rows, int64_t n, int64_t batch_global, int user_num, int item_num,
                      int32_t* touched, void* stream) {
    if (!rows || !touched || n <= 0 || batch_global <= 0 || user_num <= 0 || item_num <= 0) return NCF_E_ARG;
    if ((reinterpret_cast<uintptr_t>(touched) & 7) != 0) return NCF_E_ARG;
    if (user_num > LZ_MAX_ROWS || item_num > LZ_MAX_ROWS) return NCF_E_UNSUPPORTED;
    const TouchedShape t = touched_shape(n, batch_global, user_num, item_num);
    const int mx = user_num > item_num ? user_num : item_num;
    const int64_t lds = 2 * (int64_t)((mx + 31) / 32) * 4;
    if (lds > 64 * 1024 && ensure_lds((const void*)batch_touched_kernel, lds) != NCF_OK) return NCF_E_LAUNCH;
    int64_t* seg = reinterpret_cast<int64_t*>(touched);
    int32_t* ids = touched + 2 * t.segs;
    const int span = lazy_span();
    hipLaunchKernelGGL(batch_touched_kernel, dim3((unsigned)(2 * t.nb)), dim3(BT_THREADS), (size_t)lds,
                       (hipStream_t)stream, rows, n, batch_global, user_num, item_num, t.nb, span, 0, seg, ids);
    hipLaunchKernelGGL(touched_scan_kernel, dim3(1), dim3(BT_THREADS), 0, (hipStream_t)stream, seg, t.segs - 1);
    hipLaunchKernelGGL(batch_touched_kernel, dim3((unsigned)(2 * t.nb)), dim3(BT_THREADS), (size_t)lds,
                       (hipStream_t)stream, rows, n, batch_global, user_num, item_num, t.nb, span, 1, seg, ids);
    return launch_status();
}

// blocks for one step's rows: an upper bound of its wave tasks, 4 waves a block
static int64_t lazy_blocks(const LazyArgs& a, int64_t rows_u, int64_t rows_i) {
    int64_t waves = 0;
    for (int sd = 0; sd < 2; ++sd) {
        const int w = (a.off[sd] >= 0 ? a.w4[sd] : 0) + (a.off[sd + 2] >= 0 ? a.w4[sd + 2] : 0);
        if (w == 0) continue;
        const int per = w <= 64 ? 64 / w : 1;
        waves += ((sd ? rows_i : rows_u) + per - 1) / per;
    }
    int64_t nB = (waves + 3) / 4;
    if (nB > 2048) nB = 2048;
    return nB < 1 ? 1 : nB;
}

static int64_t step_blocks(const LazyArgs& a, const TouchedShape& t) {
    const int span = lazy_span();
    const int64_t ru = (a.U < 2 * t.su ? a.U : 2 * t.su) + a.U / span + 1;
    const int64_t ri = (a.I < 2 * t.si ? a.I : 2 * t.si) + a.I / span + 1;
    return lazy_blocks(a, ru, ri);
}

int ncf_lazy_adam_step(const ncf_layout* lay, const void* workspace, float* params, float* grads, float* exp_avg,
                       float* exp_avg_sq, const int64_t* ranges, int nranges, ncf_step_ctl* ctl, double lr,
                       double beta1, double beta2, double eps, float* loss_hist, int64_t hist_len,
                       const int32_t* touched, int64_t n_total, int64_t batch_global, int32_t* last_step,
                       float* step_scalars, int64_t ring, void* stream) {
    if (!lay || !workspace || !params || !grads || !exp_avg || !exp_avg_sq || !ranges || !ctl || !touched ||
        !last_step || !step_scalars || n_total <= 0 || batch_global <= 0 || ring < LZ_WIN + 2)
        return NCF_E_ARG;
    int err = 0;
    Ranges R = make_ranges(ranges, nranges, &err);
    if (err) return NCF_E_ARG;
    LazyArgs a;
    const int rc = lazy_args(lay, params, grads, exp_avg, exp_avg_sq, ranges, nranges, last_step, step_scalars, ring, &a);
    if (rc != NCF_OK) return rc;
    const TouchedShape t = touched_shape(n_total, batch_global, lay->user_num, lay->item_num);
    touched_lists(&a, touched, t);
    const int stride = (int)ncf_slab_stride(lay);
    const int lo = slab_lo(lay);
    const int nA = (stride - lo + 63) / 64;
    const int rows = reduce_rows(lay);
    const int64_t nB = step_blocks(a, t);
    hipLaunchKernelGGL(lazy_adam_kernel, dim3((unsigned)(nA + nB)), dim3(256), 0, (hipStream_t)stream,
                       static_cast<const float*>(workspace), lo, stride, rows, nA, lay->tower_begin, lay->tower_len, R,
                       ctl, lr, beta1, beta2, (float)eps, loss_hist, hist_len, w0_part(lay, workspace), a,
                       sc_cache_for(ctl, stream));
    return launch_status();
}

// packed mode geometry: floats per packed user / item row, the item rows' offset,
// the tail (tower gradient + loss, ncf_slab_stride floats) and the total
static void packed_geometry(const ncf_layout* lay, LazyArgs* a, int64_t su, int64_t si, int64_t* total) {
    a->wrow[0] = 4 * ((a->off[0] >= 0 ? a->w4[0] : 0) + (a->off[2] >= 0 ? a->w4[2] : 0));
    a->wrow[1] = 4 * ((a->off[1] >= 0 ? a->w4[1] : 0) + (a->off[3] >= 0 ? a->w4[3] : 0));
    a->pk_items = su * a->wrow[0];
    a->pk_tail = a->pk_items + si * a->wrow[1];
    *total = a->pk_tail + ncf_slab_stride(lay);
}

int64_t ncf_touched_packed_floats(const ncf_layout* lay, const int64_t* ranges, int nranges, int64_t batch_global) {
    if (!lay || !ranges || batch_global <= 0) return -1;
    LazyArgs a;
    if (lazy_args(lay, nullptr, nullptr, nullptr, nullptr, ranges, nranges, nullptr, nullptr, 1, &a) != NCF_OK)
        return -1;
    const TouchedShape t = touched_shape(1, batch_global, lay->user_num, lay->item_num);
    int64_t total;
    packed_geometry(lay, &a, t.su, t.si, &total);
    return total;
}

int ncf_touched_pack(const ncf_layout* lay, const void* workspace, float* grads, const int64_t* ranges, int nranges,
                     const int32_t* touched, int64_t n_total, int64_t batch_global, const ncf_step_ctl* ctl,
                     float* packed, void* stream) {
    if (!lay || !workspace || !grads || !ranges || !touched || !ctl || !packed || n_total <= 0 || batch_global <= 0 )
        return NCF_E_ARG;
    LazyArgs a;
    const int rc = lazy_args(lay, nullptr, grads, nullptr, nullptr, ranges, nranges, nullptr, nullptr, 1, &a);
    if (rc != NCF_OK) return rc;
    const TouchedShape t = touched_shape(n_total, batch_global, lay->user_num, lay->item_num);
    touched_lists(&a, touched, t);
    int64_t total;
    packed_geometry(lay, &a, t.su, t.si, &total);
    // tower gradient (slab rows, W0 partials; loss at tower_len) into the tail
    const int stride = (int)ncf_slab_stride(lay);
    const int lo = slab_lo(lay);
    hipLaunchKernelGGL(reduce_slab_kernel, dim3((stride - lo + 63) / 64), dim3(256), 0, (hipStream_t)stream,
                       static_cast<const float*>(workspace), packed + a.pk_tail, lo, stride, reduce_rows(lay),
                       (ncf_step_ctl*)nullptr, w0_part(lay, workspace));
    // tail[0, lo) is never written: it stays as allocated (zero), and sums to zero
    hipLaunchKernelGGL(touched_pack_kernel, dim3((unsigned)lazy_blocks(a, t.su, t.si)), dim3(256), 0,
                       (hipStream_t)stream, ctl, a, t.su, t.si, packed);
    return launch_status();
}

int ncf_lazy_adam_step_packed(const ncf_layout* lay, float* params, float* exp_avg, float* exp_avg_sq,
                              const int64_t* ranges, int nranges, ncf_step_ctl* ctl, double lr, double beta1,
                              double beta2, double eps, float* loss_hist, int64_t hist_len, const int32_t* touched,
                              int64_t n_total, int64_t batch_global, int32_t* last_step, float* step_scalars,
                              int64_t ring, const float* packed, void* stream) {
    if (!lay || !params || !exp_avg || !exp_avg_sq || !ranges || !ctl || !touched || !last_step || !step_scalars ||
        !packed || n_total <= 0 || batch_global <= 0 || ring < LZ_WIN + 2)
        return NCF_E_ARG;
    int err = 0;
    Ranges R = make_ranges(ranges, nranges, &err);
    if (err) return NCF_E_ARG;
    LazyArgs a;
    const int rc = lazy_args(lay, params, nullptr, exp_avg, exp_avg_sq, ranges, nranges, last_step, step_scalars,
                             ring, &a);
    if (rc != NCF_OK) return rc;
    const TouchedShape t = touched_shape(n_total, batch_global, lay->user_num, lay->item_num);
    touched_lists(&a, touched, t);
    a.packed = packed;
    int64_t total;
    packed_geometry(lay, &a, t.su, t.si, &total);
    const int stride = (int)ncf_slab_stride(lay);
    const int lo = slab_lo(lay);
    const int nA = (stride - lo + 63) / 64;
    const int64_t nB = step_blocks(a, t);
    hipLaunchKernelGGL(lazy_adam_kernel, dim3((unsigned)(nA + nB)), dim3(256), 0, (hipStream_t)stream,
                       (const float*)nullptr, lo, stride, 0, nA, lay->tower_begin, lay->tower_len, R, ctl, lr, beta1,
                       beta2, (float)eps, loss_hist, hist_len, W0Part{nullptr, 0, 0, 0, 0}, a, sc_cache_for(ctl, stream));
    return launch_status();
}

int ncf_lazy_adam_flush(const ncf_layout* lay, float* params, float* grads, float* exp_avg, float* exp_avg_sq,
                        const int64_t* ranges, int nranges, const ncf_step_ctl* ctl, double beta1, double beta2,
                        double eps, int32_t* last_step, const float* step_scalars, int64_t ring, void* stream) {
    if (!lay || !params || !grads || !exp_avg || !exp_avg_sq || !ranges || !ctl || !last_step || !step_scalars ||
        ring < LZ_WIN + 2)
        return NCF_E_ARG;
    LazyArgs a;
    const int rc = lazy_args(lay, params, grads, exp_avg, exp_avg_sq, ranges, nranges, last_step,
                             const_cast<float*>(step_scalars), ring, &a);
    if (rc != NCF_OK) return rc;
    a.nb = 1;
    hipLaunchKernelGGL(lazy_flush_kernel, dim3((unsigned)lazy_blocks(a, a.U, a.I)), dim3(256), 0, (hipStream_t)stream,
                       ctl, beta1, beta2, (float)eps, a);
    return launch_status();
}

int ncf_sgd_step(float* params, float* grads, const int64_t* ranges, int nranges, ncf_step_ctl* ctl, double lr,
                 int64_t loss_slot, float* loss_hist, int64_t hist_len, void* stream) {
    if (!params || !grads || !ranges || !ctl) return NCF_E_ARG;
    int err = 0;
    Ranges R = make_ranges(ranges, nranges, &err);
    if (err) return NCF_E_ARG;
    const int64_t total = R.prefix[R.n];
    int64_t grid = (total + 255) / 256;
    if (grid > 2048) grid = 2048;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(sgd_kernel, dim3((int)grid), dim3(256), 0, (hipStream_t)stream, params, grads, R, ctl, (float)lr,
                       loss_slot, loss_hist, hist_len);
    return launch_status();
}

int ncf_zero_f32(float* p, int64_t n, void* stream) { return launch_zero_f32(p, n, (hipStream_t)stream); }

int ncf_expand_grads(const ncf_layout* lay, const float* params, float* grads, void* workspace, void* stream) {
    (void)workspace;
    (void)stream;
    // ABI 8: ncf_train_step[_kd] launches the expansion itself; kept as a no-op so
    // an ABI-7 call sequence (step -> expand -> reduce) still trains correctly.
    if (!lay || !params || !grads) return NCF_E_ARG;
    return NCF_OK;
}

int ncf_pack_rows(const int32_t* users, const int32_t* items, const float* labels, int64_t n, uint64_t* rows_out,
                  void* stream) {
    if (!users || !items || !rows_out || n < 0) return NCF_E_ARG;
    if (n == 0) return NCF_OK;
    int64_t grid = (n + 255) / 256;
    if (grid > 4096) grid = 4096;
    hipLaunchKernelGGL(pack_rows_kernel, dim3((int)grid), dim3(256), 0, (hipStream_t)stream, users, items, labels, n,
                       rows_out);
    return launch_status();
}

int ncf_gather_epoch(const uint64_t* rows, const int64_t* perm, int64_t n, uint64_t* rows_out, void* stream) {
    if (!rows || !perm || !rows_out || n < 0) return NCF_E_ARG;
    if (n == 0) return NCF_OK;
    int64_t grid = (n + 255) / 256;
    if (grid > 4096) grid = 4096;
    hipLaunchKernelGGL(gather_epoch_kernel, dim3((int)grid), dim3(256), 0, (hipStream_t)stream, rows, perm, n,
                       rows_out);
    return launch_status();
}

int64_t ncf_prepare_epoch_workspace(int64_t n, int64_t batch_global, int item_num) {
    if (n < 0 || batch_global <= 0 || item_num <= 0) return -1;
    if (batch_global < PREP_GROUP_MIN) return al256(8);  // plain shuffle: no histogram, no parts
    const int64_t nb = (n + batch_global - 1) / batch_global;
    const int P = prep_parts(batch_global);
    return al256(n * 8) + al256(nb * item_num * 4) + al256(nb * (P + 1) * 2 * 4);
}

int ncf_prepare_epoch(const uint64_t* rows, const int64_t* perm, int64_t n, int64_t batch_global, int item_num,
                      uint64_t* rows_out, void* workspace, int64_t workspace_bytes, void* stream) {
    return ncf_prepare_epoch2(rows, perm, n, batch_global, item_num, 0, rows_out, workspace, workspace_bytes, stream);
}

int ncf_prepare_epoch2(const uint64_t* rows, const int64_t* perm, int64_t n, int64_t batch_global, int item_num,
                       int flags, uint64_t* rows_out, void* workspace, int64_t workspace_bytes, void* stream) {
    if (!rows || !perm || !rows_out || !workspace || n < 0 || batch_global <= 0 || item_num <= 0) return NCF_E_ARG;
    if (flags & ~NCF_PREP_CANONICAL) return NCF_E_ARG;
    if (batch_global > 0x7fffffff) return NCF_E_ARG;
    if (workspace_bytes < ncf_prepare_epoch_workspace(n, batch_global, item_num)) return NCF_E_ARG;
    if (n == 0) return NCF_OK;
    hipStream_t st = (hipStream_t)stream;
    if (batch_global < PREP_GROUP_MIN) {  // small batches: item runs ~1 row, grouping buys nothing
        int64_t grid = (n + 255) / 256;
        if (grid > 8192) grid = 8192;
        hipLaunchKernelGGL(gather_epoch_kernel, dim3((int)grid), dim3(256), 0, st, rows, perm, n, rows_out);
        return launch_status();
    }
    const int64_t nb = (n + batch_global - 1) / batch_global;
    const int P = prep_parts(batch_global);
    char* ws = static_cast<char*>(workspace);
    uint64_t* shuf = reinterpret_cast<uint64_t*>(ws);
    int* hist = reinterpret_cast<int*>(ws + al256(n * 8));
    int* parts = reinterpret_cast<int*>(ws + al256(n * 8) + al256(nb * item_num * 4));
    if (hipMemsetAsync(hist, 0, (size_t)(nb * item_num * 4), st) != hipSuccess) return NCF_E_LAUNCH;
    if (item_num <= SH2_MAX_ITEMS && !(g_diag & DIAG_PREP_DIRECT)) {
        const int chunks = (int)((batch_global + SH_CHUNK - 1) / SH_CHUNK);
        const int64_t lds = (int64_t)item_num * 4;
        if (ensure_lds(reinterpret_cast<const void*>(&shuffle_hist_lds_kernel), lds) != NCF_OK) return NCF_E_LAUNCH;
        hipLaunchKernelGGL(shuffle_hist_lds_kernel, dim3((unsigned)(nb * chunks)), dim3(SH2_THREADS), (size_t)lds, st,
                           rows, perm, n, batch_global, item_num, chunks, shuf, hist);
    } else {
        const int64_t g1 = (n + SH_THREADS * SH_UNROLL - 1) / (SH_THREADS * SH_UNROLL);
        hipLaunchKernelGGL(shuffle_hist_kernel, dim3((unsigned)g1), dim3(SH_THREADS), 0, st, rows, perm, n,
                           batch_global, item_num, shuf, hist);
    }
    hipLaunchKernelGGL(scan_parts_kernel, dim3((unsigned)nb), dim3(SCAN_THREADS), 0, st, hist, n, batch_global,
                       item_num, P, parts);
    if (ensure_lds(reinterpret_cast<const void*>(&sort_part_kernel), SORT_LDS) != NCF_OK) return NCF_E_LAUNCH;
    const int64_t g3 = P >= 8 ? ((nb + 7) / 8) * 8 * P : nb * P;
    hipLaunchKernelGGL(sort_part_kernel, dim3((unsigned)g3), dim3(SORT_THREADS), (size_t)SORT_LDS, st, shuf, hist,
                       parts, n, batch_global, item_num, P, nb, rows_out, (flags & NCF_PREP_CANONICAL) ? 1 : 0);
    return launch_status();
}

int ncf_user_order(const uint64_t* rows, int64_t n, int64_t batch_global, int world, int user_num, int64_t* order,
                   void* stream) {
    if (!rows || !order || n < 0 || batch_global <= 0 || world < 1 || user_num <= 0) return NCF_E_ARG;
    if (user_num > UO_MAX_USERS) return NCF_E_UNSUPPORTED;
    if (n == 0) return NCF_OK;
    const int64_t nb = (n + batch_global - 1) / batch_global;
    if (nb * world > 0x7fffffff) return NCF_E_ARG;
    const int64_t lds = (int64_t)(user_num + 1) * 4;
    if (ensure_lds(reinterpret_cast<const void*>(&user_order_kernel), lds) != NCF_OK) return NCF_E_LAUNCH;
    hipLaunchKernelGGL(user_order_kernel, dim3((unsigned)(nb * world)), dim3(UO_THREADS), (size_t)lds,
                       (hipStream_t)stream, rows, n, batch_global, world, user_num, order);
    return launch_status();
}

int ncf_uses_user_order(const ncf_layout* lay) {
    if (!lay) return 0;
    return ((fact_mode(lay) && !train_fused(lay) && lay->user_num <= UO_MAX_USERS) || us_on(lay)) ? 1 : 0;
}

int ncf_hr_ndcg(const float* logits, const int32_t* items, int64_t n, int batch, int top_k, int32_t* hr, float* ndcg,
                void* stream) {
    if (!logits || !items || !hr || !ndcg || n <= 0 || batch <= 0 || batch > HR_MAXB || top_k <= 0) return NCF_E_ARG;
    const int64_t nb = (n + batch - 1) / batch;
    const int64_t last = n - (nb - 1) * batch;
    if (top_k > batch || top_k > last) return NCF_E_ARG;  // torch.topk: "selected index k out of range"
    const int64_t grid = (nb + 3) / 4;
    hipLaunchKernelGGL(hr_ndcg_kernel, dim3((int)grid), dim3(256), 0, (hipStream_t)stream, logits, items, n, batch,
                       top_k, nb, hr, ndcg);
    return launch_status();
}

}  // extern "C"

// dp_mode "owner" (ABI 17): the owner-sharded sparse exchange
#include "ncf_owner.inc"

