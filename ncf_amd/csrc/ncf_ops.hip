// Optimizer, reduction, epoch-shuffle and evaluation kernels + the C ABI
// (include/ncf_hip.h) of libncf_hip.so.  gfx950 only.
#include <math.h>
#include <string.h>

#include "ncf_kernels.h"

namespace ncf {

static inline int64_t rup64(int64_t x) { return (x + 63) / 64 * 64; }

// ---------------------------------------------------------------------------
// Slab reduction: grads[tb + j] = sum_w slab[w][j], fixed order (bitwise
// reproducible).  Block = 256 threads = 16 float4 columns x 16 row groups, each
// thread 16 independent 16-byte loads; the 16 row-group partials are combined
// in LDS in a fixed order.  Thread 0 of block 0 also advances the step control
// block (batch, adam_t): the fused step before it has read `batch`, the
// optimizer after it reads the advanced `adam_t` (kernel boundaries order it).
__global__ __launch_bounds__(256) void reduce_slab_kernel(const float* __restrict__ slab, float* __restrict__ out,
                                                          int lo, int stride, int rows, ncf_step_ctl* ctl) {
    __shared__ f4 part[16][16];
    const int c4 = threadIdx.x & 15, rg = threadIdx.x >> 4;
    const int j = lo + (blockIdx.x * 16 + c4) * 4;
    f4 s = f4{0.f, 0.f, 0.f, 0.f};
    if (j < stride) {
        const float* p = slab + (int64_t)rg * stride + j;
        const int per = rows / 16;
#pragma unroll 16
        for (int r = 0; r < per; ++r) {
            const f4 v = *reinterpret_cast<const f4*>(p + (int64_t)r * 16 * stride);
            s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        }
    }
    part[rg][c4] = s;
    __syncthreads();
    if (rg == 0 && j < stride) {
        f4 t = part[0][c4];
#pragma unroll
        for (int q = 1; q < 16; ++q) {
            const f4 v = part[q][c4];
            t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
        }
        *reinterpret_cast<f4*>(out + j) = t;
    }
    if (ctl != nullptr && blockIdx.x == 0 && threadIdx.x == 0) {
        ctl->batch = ctl->batch + 1;
        ctl->adam_t = ctl->adam_t + 1;
    }
}

// ---------------------------------------------------------------------------
// Dense Adam (torch.optim.Adam, single-tensor path) + fused grad zeroing.
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

// Loss bookkeeping of the step: done by one thread, no cross-block protocol.
__device__ __forceinline__ void record_loss(const ncf_step_ctl* ctl, const float* grads, int64_t loss_slot,
                                            float* loss_hist, int64_t hist_len) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && loss_hist != nullptr && loss_slot >= 0 && hist_len > 0) {
        const int64_t b = ctl->batch - 1;  // ncf_reduce_slab advanced it
        loss_hist[((b % hist_len) + hist_len) % hist_len] = grads[loss_slot];
    }
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

__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                                   float* __restrict__ v, Ranges R, const ncf_step_ctl* ctl, double lr,
                                                   double beta1, double beta2, float eps, int64_t loss_slot,
                                                   float* loss_hist, int64_t hist_len) {
#pragma clang fp contract(off)
    __shared__ float sc[2];
    if (threadIdx.x == 0) {  // bias corrections once per block, in double like torch's Python scalars
        const double t = (double)ctl->adam_t;  // advanced by ncf_reduce_slab
        const double bc1 = 1.0 - pow(beta1, t);
        const double bc2 = 1.0 - pow(beta2, t);
        sc[0] = (float)(-(lr / bc1));
        sc[1] = (float)sqrt(bc2);
    }
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
__global__ __launch_bounds__(256) void gather_epoch_kernel(const int32_t* __restrict__ u, const int32_t* __restrict__ it,
                                                           const float* __restrict__ y, const int64_t* __restrict__ perm,
                                                           int64_t n, int32_t* uo, int32_t* io, float* yo) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = perm[k];
        uo[k] = u[s];
        io[k] = it[s];
        yo[k] = y[s];
    }
}

// ---------------------------------------------------------------------------
// Epoch preparation: one workgroup per global batch.  Rows perm[b*B .. b*B+cnt)
// of the unshuffled stream are the batch (DataLoader shuffle=True membership);
// they are written back grouped by item (counting sort in LDS).  Row order
// inside a batch does not change the batch's gradient, it only lets the fused
// step reduce item-side gradients per item segment before its atomics.
constexpr int PREP_THREADS = 1024;
__global__ __launch_bounds__(PREP_THREADS) void prepare_epoch_kernel(
    const int32_t* __restrict__ users, const int32_t* __restrict__ items, const float* __restrict__ labels,
    const int64_t* __restrict__ perm, int64_t n, int64_t B, int item_num, int32_t* __restrict__ uo,
    int32_t* __restrict__ io, float* __restrict__ yo) {
    extern __shared__ int hist[];  // [item_num] counts -> offsets, then [32] wave partials
    int* part = hist + ((item_num + 3) & ~3);
    const int tid = threadIdx.x;
    const int64_t b0 = (int64_t)blockIdx.x * B;
    const int cnt = (int)((n - b0) < B ? (n - b0) : B);
    for (int i = tid; i < item_num; i += PREP_THREADS) hist[i] = 0;
    __syncthreads();
    constexpr int U16 = 16;
    for (int j0 = 0; j0 < cnt; j0 += U16 * PREP_THREADS) {
        int64_t src[U16];
        int it[U16];
#pragma unroll
        for (int k = 0; k < U16; ++k) {
            const int j = j0 + k * PREP_THREADS + tid;
            src[k] = j < cnt ? perm[b0 + j] : -1;
        }
#pragma unroll
        for (int k = 0; k < U16; ++k) it[k] = items[src[k] < 0 ? 0 : src[k]];
#pragma unroll
        for (int k = 0; k < U16; ++k)
            if (src[k] >= 0) atomicAdd(&hist[min(max(it[k], 0), item_num - 1)], 1);
    }
    __syncthreads();
    // exclusive scan: contiguous chunk per thread, wave scan, then across waves
    const int per = (item_num + PREP_THREADS - 1) / PREP_THREADS;
    const int i0 = tid * per, i1 = min(item_num, i0 + per);
    int tot = 0;
    for (int i = i0; i < i1; ++i) tot += hist[i];
    const int lane = tid & 63, wv = tid >> 6;
    int incl = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) part[wv] = incl;
    __syncthreads();
    if (tid == 0) {
        int acc = 0;
        for (int q = 0; q < PREP_THREADS / 64; ++q) {
            const int v = part[q];
            part[q] = acc;
            acc += v;
        }
    }
    __syncthreads();
    int run = part[wv] + incl - tot;
    for (int i = i0; i < i1; ++i) {
        const int v = hist[i];
        hist[i] = run;
        run += v;
    }
    __syncthreads();
    for (int j0 = 0; j0 < cnt; j0 += U16 * PREP_THREADS) {
        int64_t src[U16];
        int it[U16], us[U16];
        float ys[U16];
#pragma unroll
        for (int k = 0; k < U16; ++k) {
            const int j = j0 + k * PREP_THREADS + tid;
            src[k] = j < cnt ? perm[b0 + j] : -1;
        }
#pragma unroll
        for (int k = 0; k < U16; ++k) {
            const int64_t sk = src[k] < 0 ? 0 : src[k];
            it[k] = items[sk];
            us[k] = users[sk];
            ys[k] = labels[sk];
        }
#pragma unroll
        for (int k = 0; k < U16; ++k) {
            if (src[k] >= 0) {
                const int pos = atomicAdd(&hist[min(max(it[k], 0), item_num - 1)], 1);
                uo[b0 + pos] = us[k];
                io[b0 + pos] = it[k];
                yo[b0 + pos] = ys[k];
            }
        }
    }
}

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

static int64_t train_lds_floats(const KernelEntry* e, const ncf_layout* lay) {
    const int64_t img = lay->tower_len + 1;
    return e->w_total + e->misc + (e->stage8 > img ? e->stage8 : img);
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
    const KernelEntry* e = find_entry(mode, F, L);
    if (!e) return 0;
    ncf_layout lay;
    if (ncf_layout_init(1, 1, F, L, mode, &lay) != NCF_OK) return 0;
    return train_lds_floats(e, &lay) * 4 <= LDS_LIMIT_BYTES ? 1 : 0;
}

int ncf_train_step(const ncf_layout* lay, const float* params, float* grads, const int32_t* users,
                   const int32_t* items, const float* labels, const ncf_step_ctl* ctl, int64_t batch_global,
                   int world, int rank, int dz_mode, float* slab, float* logits_out, void* stream) {
    if (!lay || !params || !grads || !users || !items || !labels || !ctl || !slab) return NCF_E_ARG;
    if (batch_global <= 0 || world < 1 || rank < 0 || rank >= world) return NCF_E_ARG;
    if (dz_mode != NCF_DZ_BCE && dz_mode != NCF_DZ_DLOGIT) return NCF_E_ARG;
    const KernelEntry* e = find_entry(lay->model_type, lay->factor_num, lay->num_layers);
    if (!e) return NCF_E_UNSUPPORTED;
    const int64_t lds = train_lds_floats(e, lay) * 4;
    if (lds > LDS_LIMIT_BYTES) return NCF_E_UNSUPPORTED;
    if (ensure_lds(e->train, lds) != NCF_OK) return NCF_E_LAUNCH;
    TrainArgs a;
    memset(&a, 0, sizeof(a));
    a.lay = *lay;
    a.params = params;
    a.grads = grads;
    a.users = users;
    a.items = items;
    a.labels = labels;
    a.ctl = ctl;
    a.batch_global = batch_global;
    a.world = world;
    a.rank = rank;
    a.dz_mode = dz_mode;
    a.diag = g_diag;
    a.stamps = g_stamps;
    a.slab = slab;
    a.logits_out = logits_out;
    void* args[] = {&a};
    if (hipLaunchKernel(e->train, dim3(SLAB_ROWS), dim3(NTHREADS), args, (size_t)lds, (hipStream_t)stream) !=
        hipSuccess)
        return NCF_E_LAUNCH;
    return launch_status();
}

int ncf_forward(const ncf_layout* lay, const float* params, const int32_t* users, const int32_t* items, int64_t n,
                float* logits, void* stream) {
    if (!lay || !params || !users || !items || !logits || n < 0) return NCF_E_ARG;
    if (n == 0) return NCF_OK;
    const KernelEntry* e = find_entry(lay->model_type, lay->factor_num, lay->num_layers);
    if (!e) return NCF_E_UNSUPPORTED;
    const int64_t lds = (int64_t)(e->w_total + e->misc) * 4;
    if (lds > LDS_LIMIT_BYTES) return NCF_E_UNSUPPORTED;
    if (ensure_lds(e->fwd, lds) != NCF_OK) return NCF_E_LAUNCH;
    TrainArgs a;
    memset(&a, 0, sizeof(a));
    a.lay = *lay;
    a.params = params;
    a.users = users;
    a.items = items;
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

int ncf_reduce_slab(const ncf_layout* lay, const float* slab, float* grads, ncf_step_ctl* ctl, void* stream) {
    if (!lay || !slab || !grads) return NCF_E_ARG;
    const int stride = (int)ncf_slab_stride(lay);
    const int lo = lay->model_type == NCF_MODEL_GMF ? (int)(lay->wp - lay->tower_begin) : 0;
    const int blocks = (stride - lo + 63) / 64;
    hipLaunchKernelGGL(reduce_slab_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, slab,
                       grads + lay->tower_begin, lo, stride, SLAB_ROWS, ctl);
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
                       exp_avg_sq, R, ctl, lr, beta1, beta2, (float)eps, loss_slot, loss_hist, hist_len);
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

int ncf_gather_epoch(const int32_t* users, const int32_t* items, const float* labels, const int64_t* perm, int64_t n,
                     int32_t* users_out, int32_t* items_out, float* labels_out, void* stream) {
    if (!users || !items || !labels || !perm || !users_out || !items_out || !labels_out || n < 0) return NCF_E_ARG;
    if (n == 0) return NCF_OK;
    int64_t grid = (n + 255) / 256;
    if (grid > 4096) grid = 4096;
    hipLaunchKernelGGL(gather_epoch_kernel, dim3((int)grid), dim3(256), 0, (hipStream_t)stream, users, items, labels,
                       perm, n, users_out, items_out, labels_out);
    return launch_status();
}

int ncf_prepare_epoch(const int32_t* users, const int32_t* items, const float* labels, const int64_t* perm,
                      int64_t n, int64_t batch_global, int item_num, int32_t* users_out, int32_t* items_out,
                      float* labels_out, void* stream) {
    if (!users || !items || !labels || !perm || !users_out || !items_out || !labels_out || n < 0 ||
        batch_global <= 0 || item_num <= 0)
        return NCF_E_ARG;
    if (n == 0) return NCF_OK;
    const int64_t lds = (int64_t)(((item_num + 3) & ~3) + 32) * 4;
    if (lds > LDS_LIMIT_BYTES) return NCF_E_UNSUPPORTED;
    if (ensure_lds(reinterpret_cast<const void*>(&prepare_epoch_kernel), lds) != NCF_OK) return NCF_E_LAUNCH;
    const int64_t nb = (n + batch_global - 1) / batch_global;
    hipLaunchKernelGGL(prepare_epoch_kernel, dim3((unsigned)nb), dim3(PREP_THREADS), (size_t)lds,
                       (hipStream_t)stream, users, items, labels, perm, n, batch_global, item_num, users_out,
                       items_out, labels_out);
    return launch_status();
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
