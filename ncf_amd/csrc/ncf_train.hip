// Fused NeuMF training step for MI355X (gfx950, CDNA4).
//
// One persistent launch per global batch computes, for every row of this
// rank's shard:   gather -> GMF product -> MLP tower (MFMA f32) -> predict ->
// BCE-with-logits -> dlogit -> tower dgrad/wgrad (MFMA f32) -> embedding
// scatter-add.  It replaces NCF.forward (reference src/ncf/models.py:97-118),
// nn.BCEWithLogitsLoss (scripts/train_neumf.py:86,113) and the autograd
// backward (train_neumf.py:114) of the reference.
//
// Geometry: 512-thread workgroups (8 waves, 2 per SIMD), one per CU, looping
// over 128-row tiles (16 rows per wave).  Tower weights live in LDS for the
// whole launch.  Activations stay in MFMA accumulator layout in VGPRs:
//   orientation A:  C[i = feature][j = row]: lane (c = l&15, g = l>>4) holds
//                   row c, features 16*t + 4*g + r  (r = f4 element)
// which is directly the B operand of the next layer's MFMA (K order permuted
// to match), so forward and dgrad never move activations through LDS.
// Weight gradients sum over rows: the 8 waves stage their (dpre_k, H_k) tiles
// row-major in LDS once per layer and each wave accumulates its own subset of
// the dW output tiles over all 128 rows (K = 128), in registers across tiles.
// The layer-0 dgrad runs in orientation B (C[i = row][j = feature]) so each
// atomic wave-instruction adds 4 rows x 64 contiguous bytes.
// Per-workgroup tower/predict partials go to a slab reduced by ncf_reduce_slab
// (deterministic; no atomics on tower grads).
#include <utility>

#include "ncf_common.h"
#include "ncf_kernels.h"

namespace ncf {

template <int K>
struct IC {
    static constexpr int value = K;
};
template <typename Fn, int... Is>
__device__ __forceinline__ void sf_impl(Fn&& fn, std::integer_sequence<int, Is...>) {
    (fn(IC<Is>{}), ...);
}
template <int N, typename Fn>
__device__ __forceinline__ void static_for(Fn&& fn) {
    sf_impl(fn, std::make_integer_sequence<int, N>{});
}

// Diagnostics: wave 0 / lane 0 of each workgroup records the shader clock at
// phase boundaries (one asm statement incl. its lgkmcnt wait, fenced by
// sched_barriers).  Never on in production (a.stamps == nullptr).
__device__ __forceinline__ void stamp(const TrainArgs& a, int idx) {
#ifndef NCF_STAMPS
    (void)a;
    (void)idx;
#else
    if (a.stamps != nullptr && threadIdx.x == 0 && idx < NSTAMP) {
        __builtin_amdgcn_sched_barrier(0);
        unsigned long long t;
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
        a.stamps[(size_t)blockIdx.x * NSTAMP + idx] = t;
        __builtin_amdgcn_sched_barrier(0);
    }
#endif
}

// Workgroup barrier for LDS hand-offs only.  __syncthreads() also waits for
// every outstanding global op of the wave (vmcnt(0)) -- i.e. for all in-flight
// embedding-gradient atomics -- at every barrier; nothing here needs that, so
// only the wave's LDS ops are drained.  The "memory" clobber keeps the compiler
// from moving LDS accesses across it.
// Scatter ablations exist only in the diagnostics build (results wrong while set).
#ifdef NCF_STAMPS
#define DIAG_ON(a, f) (((a).diag & (f)) != 0)
#else
#define DIAG_ON(a, f) false
#endif

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ void set_r(f4& v, int r, float x) {
    if (r == 0) v.x = x;
    else if (r == 1) v.y = x;
    else if (r == 2) v.z = x;
    else v.w = x;
}

// FACT (factored layer 0, MLP shapes): the step does not form the layer-0 weight
// and data gradients per row.  With W0 = [W0u | W0i] and X0 = [Um[u] | Im[i]],
//   dUm[u] = (sum over the batch rows r of user u of D0_r) W0u,   dW0u = sum_u G_u^T Um[u]
// (G_u = that row sum), likewise for items: the step scatter-adds D0_r (width
// S(1) = DM) into the user and item rows of the gradient buffer and
// fact_expand_kernel (ncf_ops.hip) turns those sums into dUm, dIm, dW0 with
// (U + I) / 16 tile GEMMs instead of B / 16.  Every wave then touches only its own
// rows of LDS after the weight prologue, so tiles need no workgroup barrier.
// NCF_LAYOUT_ADAM_IN_STEP, workgroups [ntrain, grid) of a training launch: update n
// (pending) written for every active float -- S_n into buffer wb from S_{n-1} in rb
// with the gradient g[n % 3], exactly the values the training workgroups compute on
// the fly for what they read -- and g[(n + 2) % 3] cleared for the next launch's
// accumulation.  Block 0 of them also records update n's loss and computes update
// n + 1's step scalars (two double pows) into the cache.
__device__ __forceinline__ void ais_dense_block(const TrainArgs& a, int64_t n, bool pending, int rb, float* sc) {
#pragma clang fp contract(off)
    const AisArgs& x = a.ais;
    // the last extra workgroup only computes update n + 1's step scalars (two double
    // pows, ~2.5 us on one lane) -- beside the others, not ahead of a barrier of theirs
    if ((int)blockIdx.x == (int)gridDim.x - 1) {
        step_scalars_ahead_lane(x.scc, n, x.lr, x.beta1, x.beta2);
        return;
    }
    const int e = (int)blockIdx.x - x.ntrain, ne = (int)gridDim.x - 1 - x.ntrain;
    const int64_t tb = a.lay.tower_begin, loss_i = tb + a.lay.tower_len;
    float* gz = x.g[(n + 2) % 3];
    const float* gr = x.g[n % 3];
    const float *pr = x.p[rb], *mr = x.m[rb], *vr = x.v[rb];
    float *pw = x.p[rb ^ 1], *mw = x.m[rb ^ 1], *vw = x.v[rb ^ 1];
    const int64_t total = x.R.prefix[x.R.n];
    const int64_t nthr = (int64_t)ne * blockDim.x;
    const ScCache sce = sc_peek(x.scc, n);
    if (e == 0 && threadIdx.x == 0) {
        gz[loss_i] = 0.f;
        if (pending && x.loss_hist != nullptr && x.hist_len > 0) {
            const int64_t b = a.ctl->batch + x.step_i - 1;  // the batch whose gradient is update n's
            x.loss_hist[((b % x.hist_len) + x.hist_len) % x.hist_len] = gr[loss_i];
        }
    }
    sc_resolve(sce, n, x.lr, x.beta1, x.beta2, sc);
    __syncthreads();
    const float neg_step = sc[0], bc2s = sc[1];
    const float w1 = (float)(1.0 - x.beta1), b2 = (float)x.beta2, omb2 = (float)(1.0 - x.beta2);
    const f4 z4 = f4{0.f, 0.f, 0.f, 0.f};
    // two float4 per thread and pass, all loads of a pass issued before its stores
    for (int64_t q0 = (int64_t)e * blockDim.x + threadIdx.x; q0 < total; q0 += 2 * nthr) {
        const int64_t q1 = q0 + nthr;
        const bool has1 = q1 < total;
        int which;
        const int64_t i0 = range_locate(x.R, q0, &which);
        const int64_t i1 = has1 ? range_locate(x.R, q1, &which) : i0;
        if (pending) {
            f4 p0 = *reinterpret_cast<const f4*>(pr + i0), m0 = *reinterpret_cast<const f4*>(mr + i0),
               v0 = *reinterpret_cast<const f4*>(vr + i0);
            const f4 g0 = *reinterpret_cast<const f4*>(gr + i0);
            f4 p1 = *reinterpret_cast<const f4*>(pr + i1), m1 = *reinterpret_cast<const f4*>(mr + i1),
               v1 = *reinterpret_cast<const f4*>(vr + i1);
            const f4 g1 = *reinterpret_cast<const f4*>(gr + i1);
            adam_f4(p0, m0, v0, g0, w1, b2, omb2, bc2s, x.eps, neg_step);
            *reinterpret_cast<f4*>(pw + i0) = p0;
            *reinterpret_cast<f4*>(mw + i0) = m0;
            *reinterpret_cast<f4*>(vw + i0) = v0;
            if (has1) {
                adam_f4(p1, m1, v1, g1, w1, b2, omb2, bc2s, x.eps, neg_step);
                *reinterpret_cast<f4*>(pw + i1) = p1;
                *reinterpret_cast<f4*>(mw + i1) = m1;
                *reinterpret_cast<f4*>(vw + i1) = v1;
            }
        }
        *reinterpret_cast<f4*>(gz + i0) = z4;
        if (has1) *reinterpret_cast<f4*>(gz + i1) = z4;
    }
}

template <int F, int L, int MODE, bool FWD_ONLY, bool FACT, int NW, bool AIS = false>
__global__ __launch_bounds__(NW * WAVE, 2) void ncf_step_kernel(TrainArgs a) {
    using S_ = Shape<F, L, MODE, NW>;
    // workgroup geometry: NW waves, 16 rows each, per tile (NW = 8, or 4 for small batches)
    constexpr int NWV = S_::NWV, NTH = S_::NTH, TRW = S_::TR;
    static_assert(!FACT || S_::MLP, "factored layer 0 needs the MLP tower");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* sW = smem;
    int* su2 = reinterpret_cast<int*>(smem + S_::W_TOTAL);  // [2][TRW] user ids (-1 = padding row)
    int* si2 = su2 + 2 * TRW;                         // [2][TRW] item ids
    float* slab2 = reinterpret_cast<float*>(si2 + 2 * TRW);  // [2][TRW] labels / dlogits
    float* szg = slab2 + 2 * TRW;  // GMF part of the logit, per tile row
    float* sdz = szg + TRW;        // dlogit, per tile row
    float* stl2 = sdz + TRW;       // [2][TRW] NCF_DZ_KD: teacher logits
    float* sB = stl2 + 2 * TRW;    // biases, layer k at boff(k), zero-padded
    float* sWP = sB + 128;               // predict weights, zero-padded
    float* sstage = sWP + 128;           // union: per-wave staging | epilogue images
    static_assert(10 * TRW + 256 == S_::MISC, "LDS carve-up must match Shape::MISC (the launch's LDS size)");

    const int tid = threadIdx.x;
    const int w = tid >> 6;
    const bool wv_hi = __builtin_amdgcn_readfirstlane(w) >= NWV / 2;  // wave-uniform (scalar branch)
    const int l0 = tid & 63;
    const int c0 = l0 & 15;
    const int g0 = l0 >> 4;
    const ncf_layout& lay = a.lay;
    const float* __restrict__ prm = a.params;
    float* __restrict__ grads = a.grads;

    // NCF_LAYOUT_ADAM_IN_STEP: the state this launch reads (S_{n-1}, with update n
    // pending, applied on the fly), the gradient it accumulates (update n + 1's)
    static_assert(!AIS || (!FACT && !FWD_ONLY), "in-step Adam: per-row layer 0, training launches");
    const float* mrd = nullptr;
    const float* vrd = nullptr;
    const float* gread = nullptr;
    bool ais_pend = false;
    float* ais_sc = smem + S_::W_TOTAL + 10 * TRW;  // = sB below, written after the scalars are read
    if constexpr (AIS) {
        if ((int)blockIdx.x < a.ais.ntrain) stamp(a, 63);  // diag: kernel entry
        // both cache entries requested with the control block (the entry of update n
        // is picked once n is known: one round trip, not two dependent ones)
        ScCache sce2[2];
        sce2[0].t = sce2[1].t = -1;
        if (threadIdx.x == 0 && a.ais.scc != nullptr) {
            sce2[0] = a.ais.scc[0];
            sce2[1] = a.ais.scc[1];
        }
        const int64_t pend0 = a.ais.st[0], par = a.ais.st[1];
        const int64_t n = a.ctl->adam_t + a.ais.step_i + pend0;
        ais_pend = a.ais.step_i > 0 || pend0 != 0;
        const int rb = (int)((ais_pend ? n - 1 + par : n + par) & 1);
        prm = a.ais.p[rb];
        mrd = a.ais.m[rb];
        vrd = a.ais.v[rb];
        gread = a.ais.g[n % 3];
        grads = a.ais.g[(n + 1) % 3];
        if ((int)blockIdx.x >= a.ais.ntrain) {
            ais_dense_block(a, n, ais_pend, rb, ais_sc);
            return;
        }
        if (ais_pend) sc_resolve((n & 1) ? sce2[1] : sce2[0], n, a.ais.lr, a.ais.beta1, a.ais.beta2, ais_sc);
    }
    float ais_w1 = 0.f, ais_b2 = 0.f, ais_omb2 = 0.f, ais_ns = 0.f, ais_bc = 1.f;
    if constexpr (AIS) {
        ais_w1 = (float)(1.0 - a.ais.beta1);
        ais_b2 = (float)a.ais.beta2;
        ais_omb2 = (float)(1.0 - a.ais.beta2);
    }
    // one parameter float as this launch sees it (the per-row layer-0 wgrad operand)
    auto pval = [&](int64_t i) -> float {
        float pp = prm[i];
        if constexpr (AIS) {
            if (ais_pend) {
                float mm = mrd[i], vv = vrd[i];
                pp = adam_1(pp, mm, vv, gread[i], ais_w1, ais_b2, ais_omb2, ais_bc, a.ais.eps, ais_ns);
            }
        }
        return pp;
    };
    // AIS: the tower after update n, built into the (idle) staging region before the
    // weights are read: in_ranges floats updated, the others as stored
    const float* tw = prm;  // tower floats: tw[i - toff]
    int64_t toff = 0;
    float* sstage_ = smem + S_::W_TOTAL + S_::MISC;  // = sstage below
    // (issued after the row indices: its loads fly with theirs)
    auto build_image = [&]() {
        // the tower's loads issued before the scalar barrier (AIS_TQ float4 per thread
        // in flight; more in a second pass)
        constexpr int AIS_TQ = 4;
        const int64_t tb = lay.tower_begin;
        const int n4 = (int)((lay.tower_len + 3) / 4);
        for (int q0 = 0; q0 < n4; q0 += AIS_TQ * NTH) {
            f4 pp[AIS_TQ], mm[AIS_TQ], vv[AIS_TQ], gg[AIS_TQ];
#pragma unroll
            for (int u = 0; u < AIS_TQ; ++u) {
                const int q = q0 + u * NTH + tid;
                const int64_t i = tb + 4 * (int64_t)(q < n4 ? q : 0);
                pp[u] = *reinterpret_cast<const f4*>(prm + i);
                if (ais_pend) {
                    mm[u] = *reinterpret_cast<const f4*>(mrd + i);
                    vv[u] = *reinterpret_cast<const f4*>(vrd + i);
                    gg[u] = *reinterpret_cast<const f4*>(gread + i);
                }
            }
            if (q0 == 0) {
                __syncthreads();  // ais_sc
                ais_ns = ais_sc[0];
                ais_bc = ais_sc[1];
            }
#pragma unroll
            for (int u = 0; u < AIS_TQ; ++u) {
                const int q = q0 + u * NTH + tid;
                if (q >= n4) continue;
                if (ais_pend && in_ranges(a.ais.R, tb + 4 * (int64_t)q))
                    adam_f4(pp[u], mm[u], vv[u], gg[u], ais_w1, ais_b2, ais_omb2, ais_bc, a.ais.eps, ais_ns);
                *reinterpret_cast<f4*>(sstage_ + 4 * q) = pp[u];
            }
        }
        if (n4 == 0) {  // (every layout has the predict weights: not reached)
            __syncthreads();
            ais_ns = ais_sc[0];
            ais_bc = ais_sc[1];
        }
        __syncthreads();
        tw = sstage_;
        toff = tb;
    };

    // Tower weight / bias loads first: they depend on nothing, so they fly while
    // the control block and the row indices make their round trips (AIS: from the
    // image, after the row indices are requested).
    constexpr int PERMAX = S_::MLP ? (16 * S_::MT(0) * (S_::S(0) / 4) + NTH - 1) / NTH : 1;
    f4 wreg[L][PERMAX];
    constexpr int BPER = (128 + NTH - 1) / NTH;  // bias entries per thread (16 * MT(k) <= 128)
    float breg[L][BPER];
    auto load_wregs = [&]() {
    if constexpr (S_::MLP) {
        static_for<L>([&](auto kk) {
            constexpr int k = decltype(kk)::value;
            constexpr int rows = 16 * S_::MT(k), cols4 = S_::S(k) / 4, outs = S_::S(k + 1);
            constexpr int PER = (rows * cols4 + NTH - 1) / NTH;
            const f4* Wg = reinterpret_cast<const f4*>(tw + (lay.w[k] - toff));
#pragma unroll
            for (int q = 0; q < PER; ++q) {
                const int e = tid + q * NTH;
                const int o = e / cols4;
                wreg[k][q] = (e < rows * cols4 && o < outs) ? Wg[e] : f4{0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll
            for (int q = 0; q < BPER; ++q) {
                const int e = tid + q * NTH;
                breg[k][q] = e < outs ? tw[lay.b[k] - toff + e] : 0.f;
            }
        });
    }
    };
    if constexpr (!AIS) load_wregs();

    // ---- rows of this rank -------------------------------------------------
    int64_t base, nloc;
    float gb_f = 1.0f;
    if constexpr (FWD_ONLY) {
        base = 0;
        nloc = a.fwd_n;
    } else {
        const int64_t ntot = a.ctl->n_total;
        const int64_t nbatch = (ntot + a.batch_global - 1) / a.batch_global;
        const int64_t b = nbatch > 0 ? (a.ctl->batch + (AIS ? a.ais.step_i : 0)) % nbatch : 0;  // epochs repeat past the end
        const int64_t b0 = b * a.batch_global;
        int64_t gb = ntot - b0;
        if (gb > a.batch_global) gb = a.batch_global;
        if (gb < 0) gb = 0;
        const int64_t per = (gb + a.world - 1) / a.world;
        int64_t lo = (int64_t)a.rank * per;
        int64_t hi = lo + per;
        if (lo > gb) lo = gb;
        if (hi > gb) hi = gb;
        base = b0 + lo;
        nloc = hi - lo;
        gb_f = (float)gb;
        if (!AIS && blockIdx.x == 0 && tid == 0) {  // step snapshot for ncf_reduce_adam_step (fields no WG reads here)
            a.ctl->snap_batch = a.ctl->batch;
            a.ctl->snap_t = a.ctl->adam_t + 1;
        }
    }
    const int64_t ntiles = (nloc + TRW - 1) / TRW;
    const int64_t gtrain = AIS ? (int64_t)a.ais.ntrain : (int64_t)gridDim.x;  // training workgroups
    stamp(a, 0);

    // Row prefetch: every thread issues the same loads (clamped row), so the
    // vector-memory stream is straight-line and hipcc can count vmcnt waits
    // exactly instead of draining everything at a branch merge.  Each wave
    // loads and publishes its own 16 rows (lanes l < 16 publish): with one
    // barrier per tile, a fast wave writing tile t+2's ids into the buffer of
    // tile t must never overwrite rows another wave still reads after tile t's
    // barrier -- and past that barrier waves read only their own rows.
    const int prow = 16 * w + (l0 & 15);
    const bool pub = l0 < 16;
    // The next tile's packed row is fetched early and decoded only where it is
    // published into LDS: nothing touches the loaded registers before then, so no
    // wait for it (and, the vmcnt counter being in order, for every scatter atomic
    // issued before it) lands at the top of a tile.
    // FACT: two tiles ahead (npr2 ...), shifted into npr ... behind the explicit
    // wait before each tile's scatter, so no wait for them follows any atomic.
    uint64_t npr = 0, npr2 = 0;
    float ndl = 0.f, ndl2 = 0.f;
    bool nok = false, nok2 = false;
    auto load_idx = [&](int64_t row0) {
        const int64_t r = row0 + prow;
        nok = r < nloc;
        const int64_t rc = base + (nok ? r : 0);
        npr = a.rows[rc];
        if constexpr (!FWD_ONLY) ndl = a.dlogit[rc];  // forward launches carry no labels
    };
    auto load_idx2 = [&](int64_t row0) {
        const int64_t r = row0 + prow;
        nok2 = r < nloc;
        const int64_t rc = base + (nok2 ? r : 0);
        npr2 = a.rows[rc];
        if constexpr (!FWD_ONLY) ndl2 = a.dlogit[rc];
    };
    auto publish = [&](int off) {
        if (pub) {
            su2[off + prow] = nok ? (int)(uint32_t)npr : -1;
            si2[off + prow] = nok ? (int)((npr >> 32) & 0x7fffffffu) : -1;
            if constexpr (!FWD_ONLY) {
                slab2[off + prow] = a.dz_mode == NCF_DZ_DLOGIT ? ndl : (float)(uint32_t)(npr >> 63);
                stl2[off + prow] = ndl;  // NCF_DZ_KD: the teacher logit (else unused)
            }
        }
    };
    if ((int64_t)blockIdx.x < ntiles) load_idx((int64_t)blockIdx.x * TRW);
    if constexpr (AIS) {
        stamp(a, 58);  // diag: AIS row indices requested
        build_image();
        stamp(a, 59);  // diag: AIS tower image built
        load_wregs();
    }
    if constexpr (FACT && !FWD_ONLY) load_idx2(((int64_t)blockIdx.x + gtrain) * TRW);

    // ---- tower weights, biases, predict weights -> LDS (zero-padded) ---------
    if constexpr (S_::MLP) {
        // (their loads were issued at the top of the kernel, ahead of the control
        // block read the row range depends on)
        static_for<L>([&](auto kk) {
            constexpr int k = decltype(kk)::value;
            constexpr int rows = 16 * S_::MT(k), cols4 = S_::S(k) / 4;
            constexpr int PER = (rows * cols4 + NTH - 1) / NTH;
            float* Ws = sW + S_::woff(k);
#pragma unroll
            for (int q = 0; q < PER; ++q) {
                const int e = tid + q * NTH;
                const int o = e / cols4, i4 = e - o * cols4;
                if (e < rows * cols4) *reinterpret_cast<f4*>(Ws + o * S_::SW(k) + 4 * i4) = wreg[k][q];
            }
#pragma unroll
            for (int q = 0; q < BPER; ++q)
                if (tid + q * NTH < 16 * S_::MT(k)) sB[S_::boff(k) + tid + q * NTH] = breg[k][q];
        });
    }
    for (int e = tid; e < 128; e += NTH) sWP[e] = e < S_::P ? tw[lay.wp - toff + e] : 0.f;

    // ---- per-lane persistent accumulators ----------------------------------
    constexpr int MT0 = S_::MLP ? S_::MT(0) : 1;
    constexpr int KT0 = S_::KT0;
    constexpr int MTL = S_::MLP ? S_::MT(L - 1) : 1;
    // per-row layer-0 wgrad: each wave owns the 16-column blocks nt = w + j * NWV of
    // dW0 (j < CB0; one block at 8 waves, several in narrow workgroups)
    constexpr int CB0 = S_::MLP && !FACT ? (KT0 + NWV - 1) / NWV : 1;
    // OWN0: layer 0's wgrad from the wave's own rows (Shape::OWN0), no staging barrier
    constexpr bool OWN0 = S_::OWN0 && !FACT && !FWD_ONLY;
    f4 accL0[OWN0 ? MT0 * KT0 : 1];
#pragma unroll
    for (int t = 0; t < (OWN0 ? MT0 * KT0 : 1); ++t) accL0[t] = f4{0.f, 0.f, 0.f, 0.f};
    f4 accW0[CB0][MT0];     // dW_0 tiles (mt, nt = w + j * NWV)
    float dbAcc[L];
    f4 dWpT[MTL];
    f4 accK[S_::NKT > 0 ? S_::NKT : 1];    // dW_k tiles of layers k >= 1, this wave's rows
    float dbK[S_::NMB > 0 ? S_::NMB : 1];  // db_k partials (output 16mt + c, rows 4g..4g+3)
    float dWpG = 0.f, dbpAcc = 0.f, lossAcc = 0.f;
#pragma unroll
    for (int t = 0; t < S_::NKT; ++t) accK[t] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < S_::NMB; ++t) dbK[t] = 0.f;
#pragma unroll
    for (int k = 0; k < L; ++k) {
        dbAcc[k] = 0.f;
    }
#pragma unroll
    for (int t = 0; t < MT0; ++t)
#pragma unroll
        for (int j = 0; j < CB0; ++j) accW0[j][t] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < MTL; ++t) dWpT[t] = f4{0.f, 0.f, 0.f, 0.f};

    constexpr int RPI = S_::GMF ? 64 / F : 1;  // GMF rows per wave-instruction
    constexpr int NI = S_::GMF ? 16 / RPI : 1;
    const float bpv = tw[lay.bp - toff];
    const float wpf = S_::GMF ? tw[lay.wp - toff + l0 % F] : 0.f;
    publish(0);
    if constexpr (FACT && !FWD_ONLY) {
        npr = npr2;
        ndl = ndl2;
        nok = nok2;
    }
    __syncthreads();

    // Embedding fragments of the current tile, loaded one tile ahead:
    //   X0[t]  : MLP input, orientation A: row c, features 16t + 4g .. +3
    //   ugv/igv: GMF rows, row-major lanes (feature l % F, rows j*RPI + l / F)
    f4 X0[KT0];
    float ugv[NI], igv[NI];
    // AIS: the optimizer state of the fragments rides with them; the pending update is
    // applied where the fragments are first used (ais_finish at the top of the tile),
    // so the early loads keep their distance from their use (and from the waits that
    // would also drain the scatter atomics issued after them)
    constexpr int AKT = AIS ? KT0 : 1, ANI = AIS ? NI : 1;
    f4 Xm[AKT], Xv[AKT], Xg[AKT];
    float um_[ANI], uv_[ANI], ug_[ANI], im_[ANI], iv_[ANI], ig_[ANI];
    auto raw4 = [&](int64_t off, f4& pp, f4& mm, f4& vv, f4& gg) {
        pp = *reinterpret_cast<const f4*>(prm + off);
#ifdef NCF_AIS_NO_EMB_STATE  // timing experiment only (wrong results): no optimizer-state loads
        return;
#endif
        if constexpr (AIS) {
            mm = *reinterpret_cast<const f4*>(mrd + off);
            vv = *reinterpret_cast<const f4*>(vrd + off);
            gg = *reinterpret_cast<const f4*>(gread + off);
        }
    };
    auto ais_finish = [&]() {
        if constexpr (AIS) {
            if (ais_pend) {
                if constexpr (S_::MLP) {
#pragma unroll
                    for (int t = 0; t < KT0; ++t)
                        adam_f4(X0[t], Xm[t], Xv[t], Xg[t], ais_w1, ais_b2, ais_omb2, ais_bc, a.ais.eps, ais_ns);
                }
                if constexpr (S_::GMF) {
#pragma unroll
                    for (int j = 0; j < NI; ++j) {
                        ugv[j] = adam_1(ugv[j], um_[j], uv_[j], ug_[j], ais_w1, ais_b2, ais_omb2, ais_bc, a.ais.eps, ais_ns);
                        igv[j] = adam_1(igv[j], im_[j], iv_[j], ig_[j], ais_w1, ais_b2, ais_omb2, ais_bc, a.ais.eps, ais_ns);
                    }
                }
            }
        }
    };
    auto load_mlp = [&](const int* su, const int* si, int c, int g) {
        const int wr = w * 16;
        if constexpr (S_::MLP) {
            constexpr int DM = S_::DM;
            const int uc = max(su[wr + c], 0);
            const int ic = max(si[wr + c], 0);
#pragma unroll
            for (int t = 0; t < KT0; ++t) {
                const int j0 = 16 * t + 4 * g;
                const bool isu = j0 < DM;
                const int64_t off = isu ? lay.um + (int64_t)uc * DM + j0 : lay.im + (int64_t)ic * DM + (j0 - DM);
                raw4(off, X0[t], Xm[AIS ? t : 0], Xv[AIS ? t : 0], Xg[AIS ? t : 0]);
            }
        }
    };
    auto load_gmf = [&](const int* su, const int* si, int l) {
        const int wr = w * 16;
        if constexpr (S_::GMF) {
            const int gf = l % F, gq0 = l / F;
#pragma unroll
            for (int j = 0; j < NI; ++j) {
                const int q = wr + j * RPI + gq0;
                const int64_t ou = lay.ug + (int64_t)max(su[q], 0) * F + gf;
                const int64_t oi = lay.ig + (int64_t)max(si[q], 0) * F + gf;
                ugv[j] = prm[ou];
                igv[j] = prm[oi];
#ifndef NCF_AIS_NO_EMB_STATE
                if constexpr (AIS) {
                    um_[j] = mrd[ou];
                    uv_[j] = vrd[ou];
                    ug_[j] = gread[ou];
                    im_[j] = mrd[oi];
                    iv_[j] = vrd[oi];
                    ig_[j] = gread[oi];
                }
#endif
            }
        }
    };
    auto load_emb = [&](const int* su, const int* si, int c, int g, int l) {
        load_mlp(su, si, c, g);
        load_gmf(su, si, l);
    };
    // FACT (not FWD_ONLY): the next tile's ids are published and its embedding
    // fragments requested early in the tile -- MLP rows right after this tile's
    // forward has consumed X0, GMF rows after the GMF backward -- so they land long
    // before the next tile needs them instead of in its first phase.
    constexpr bool EARLY = (FACT || OWN0) && !FWD_ONLY;
    // Item-side embedding gradients of a wave's 16 rows: rows of a tile are
    // grouped by item (ncf_prepare_epoch counting-sorts each batch by item), so
    // consecutive equal items are summed in LDS and each item segment issues one
    // atomic per feature -- 256 contiguous bytes per wave-instruction for the MLP
    // table -- instead of one per row.  Correct for any row order (unsorted
    // input just yields shorter segments).  scr holds the MLP item rows
    // [16][SCM] (written by the caller); the GMF item rows go to [16][SCG] after it.
    // The wave's 16 row ids (wave-uniform) into scalar registers: four 16-byte LDS
    // reads, then readfirstlane, so segment boundaries are scalar branches.
    auto wave_ids = [&](const int* ids16, int (&ids)[16]) {
        const int4* p4 = reinterpret_cast<const int4*>(ids16);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int4 v = p4[q];
            ids[4 * q + 0] = v.x;
            ids[4 * q + 1] = v.y;
            ids[4 * q + 2] = v.z;
            ids[4 * q + 3] = v.w;
        }
    };
    auto item_segments = [&](float* scr, const TrainArgs& a, const int* su, const int* si, int wr, int l,
                             const float* gIg, int gf, int gq0) {
        (void)su;
        if constexpr (S_::GMF) {
            float* sg = scr + 16 * S_::SCM;
#pragma unroll
            for (int j = 0; j < NI; ++j) sg[(j * RPI + gq0) * S_::SCG + gf] = gIg[j];
        }
        int ids[16];
        wave_ids(si + wr, ids);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // same-wave LDS hand-off
#pragma unroll
        for (int r = 0; r < 16; ++r) ids[r] = __builtin_amdgcn_readfirstlane(ids[r]);
        // All 16 rows' values are read before the walk (one LDS wait, not one per row).
        if constexpr (S_::MLP) {
            constexpr int DM = S_::DM;
#pragma unroll
            for (int f0 = 0; f0 < DM; f0 += 64) {
                const int f = f0 + l;
                const int fc = f < DM ? f : DM - 1;
                float v[16];
#pragma unroll
                for (int row = 0; row < 16; ++row) v[row] = scr[row * S_::SCM + fc];
                float sum = 0.f;
#pragma unroll
                for (int row = 0; row < 16; ++row) {
                    sum += v[row];
                    if (row == 15 || ids[row + 1] != ids[row]) {
                        if (ids[row] >= 0 && f < DM && !DIAG_ON(a, DIAG_NO_ITEM_SCATTER))
                            atomicAdd(grads + lay.im + (int64_t)ids[row] * DM + f, sum);
                        sum = 0.f;
                    }
                }
            }
        }
        if constexpr (S_::GMF) {
            const float* sg = scr + 16 * S_::SCM;
            const int lc = l < F ? l : F - 1;
            float v[16];
#pragma unroll
            for (int row = 0; row < 16; ++row) v[row] = sg[row * S_::SCG + lc];
            float sum = 0.f;
#pragma unroll
            for (int row = 0; row < 16; ++row) {
                sum += v[row];
                if (row == 15 || ids[row + 1] != ids[row]) {
                    if (ids[row] >= 0 && l < F && !DIAG_ON(a, DIAG_NO_GMF_SCATTER))
                        atomicAdd(grads + lay.ig + (int64_t)ids[row] * F + l, sum);
                    sum = 0.f;
                }
            }
        }
    };
    load_emb(su2, si2, c0, g0, l0);
    // Consume the first tile's fragments here: the loop header then sees them
    // as complete on entry, and hipcc's counted wait at their first use inside
    // the loop is set by the steady state (older than this tile's scatter
    // atomics: vmcnt(#atomics + 3)), not drained to the index loads.
    if constexpr (S_::MLP) {
#pragma unroll
        for (int t = 0; t < KT0; ++t) asm volatile("" ::"v"(X0[t]));
    }
    if constexpr (S_::GMF) {
#pragma unroll
        for (int j = 0; j < NI; ++j) asm volatile("" ::"v"(ugv[j]), "v"(igv[j]));
    }
    // EARLY: nothing in flight at the loop entry (the prologue's scalars included),
    // so the loop's only pending memory operations are its own
    if constexpr (EARLY) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    stamp(a, 1);
    int titer = 0;

    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gtrain) {
        ais_finish();  // AIS: this tile's fragments after the pending update
        const int64_t row0 = tile * TRW;
        const int buf = titer & 1;
        const int* su = su2 + buf * TRW;
        const int* si = si2 + buf * TRW;
        const float* slab_ = slab2 + buf * TRW;
        const bool has_next = tile + gtrain < ntiles;
        const int sb = 2 + 14 * titer;  // stamp base of this tile
        stamp(a, sb + 0);
        const int wr = w * 16;  // first tile row of this wave
        // Opaque per-tile copies of the lane coordinates: addresses are recomputed
        // inside the loop instead of being hoisted out of it (and spilled).
        int c = c0, g = g0, l = l0;
        asm volatile("" : "+v"(c), "+v"(g), "+v"(l));
        const int gf = l % F;
        const int gq0 = l / F;

        // (a) next tile's indices
        if constexpr (EARLY) {
            load_idx2(row0 + 2 * gtrain * TRW);
        } else {
            load_idx(row0 + gtrain * TRW);
            nok = nok && has_next;
        }

        // (b) GMF forward
        if constexpr (S_::GMF) {
#pragma unroll
            for (int j = 0; j < NI; ++j) {
                float v = wpf * (ugv[j] * igv[j]);
#pragma unroll
                for (int m = 1; m < F; m <<= 1) v += shfl_xor(v, m);
                if (gf == 0) szg[wr + j * RPI + gq0] = v;
            }
        }

        // (c) MLP forward (orientation A)
        const int myq = wr + c;
        f4 H[L + 1][KT0];
        if constexpr (S_::MLP) {
#pragma unroll
            for (int t = 0; t < KT0; ++t) H[0][t] = X0[t];
            static_for<L>([&](auto kk) {
                constexpr int k = decltype(kk)::value;
                f4 acc[S_::MT(k)];
#pragma unroll
                for (int mt = 0; mt < S_::MT(k); ++mt)
                    acc[mt] = *reinterpret_cast<const f4*>(sB + S_::boff(k) + 16 * mt + 4 * g);
                const float* Ws = sW + S_::woff(k);
#pragma unroll
                for (int t = 0; t < S_::KT(k); ++t) {
                    const f4 xv = H[k][t];
#pragma unroll
                    for (int mt = 0; mt < S_::MT(k); ++mt) {
                        const f4 wv = *reinterpret_cast<const f4*>(Ws + (16 * mt + c) * S_::SW(k) + 16 * t + 4 * g);
                        acc[mt] = MFMA4(wv.x, xv.x, acc[mt]);
                        acc[mt] = MFMA4(wv.y, xv.y, acc[mt]);
                        acc[mt] = MFMA4(wv.z, xv.z, acc[mt]);
                        acc[mt] = MFMA4(wv.w, xv.w, acc[mt]);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
#pragma unroll
                for (int mt = 0; mt < S_::MT(k); ++mt) {
                    f4 h;
                    h.x = fmaxf(acc[mt].x, 0.f);
                    h.y = fmaxf(acc[mt].y, 0.f);
                    h.z = fmaxf(acc[mt].z, 0.f);
                    h.w = fmaxf(acc[mt].w, 0.f);
                    H[k + 1][mt] = h;
                }
            });
        }
        stamp(a, sb + 1);
        if constexpr (EARLY) {
            publish((buf ^ 1) * TRW);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // same-wave LDS hand-off
            load_mlp(su2 + (buf ^ 1) * TRW, si2 + (buf ^ 1) * TRW, c, g);
        }

        // predict
        float zt = 0.f;
        if constexpr (S_::MLP) {
            // sWP is zero-padded past P and H[L] is 0 past F (zero weight rows, zero
            // bias, ReLU), so no bounds test: one 16-byte LDS read per output tile
#pragma unroll
            for (int mt = 0; mt < MTL; ++mt) {
                const f4 wp4 = *reinterpret_cast<const f4*>(sWP + S_::POFF + 16 * mt + 4 * g);
                const f4 h = H[L][mt];
                zt += wp4.x * h.x;
                zt += wp4.y * h.y;
                zt += wp4.z * h.z;
                zt += wp4.w * h.w;
            }
            zt += shfl_xor(zt, 16);
            zt += shfl_xor(zt, 32);
        }
        if constexpr (S_::GMF) zt += szg[myq];
        const float z = zt + bpv;
        const bool valid = su[myq] >= 0;

        if constexpr (FWD_ONLY) {
            if (g == 0 && valid) a.logits_out[base + row0 + myq] = z;
            publish((buf ^ 1) * TRW);
            lds_barrier();
            load_emb(su2 + (buf ^ 1) * TRW, si2 + (buf ^ 1) * TRW, c, g, l);
            ++titer;
            continue;
        } else {
            // (d) layer-0 wgrad operand: X0 rows of the whole tile, columns 16*nt + c
            constexpr int DM = S_::DM;
            float bx[CB0][S_::MLP && !FACT && !OWN0 ? NWV * 4 : 1];
            if constexpr (S_::MLP && !FACT && !OWN0) {
#pragma unroll
                for (int j = 0; j < CB0; ++j) {
                    const int ntj = w + j * NWV < KT0 ? w + j * NWV : KT0 - 1;
                    const int fj = 16 * ntj + c;
                    const bool isu = fj < DM;
                    const int64_t tab = isu ? lay.um + fj : lay.im + (fj - DM);
                    const int* ids = isu ? su : si;
#pragma unroll
                    for (int ws = 0; ws < NWV; ++ws) {
#pragma unroll
                        for (int s = 0; s < 4; ++s) {
                            const int id = max(ids[ws * 16 + 4 * g + s], 0);
                            bx[j][ws * 4 + s] = pval(tab + (int64_t)id * DM);
                        }
                    }
                }
            }

            if (titer < 2) stamp(a, 44 + 3 * titer);  // diag sub-phase: bx gather issued
            // (e) loss + dlogit
            if (a.logits_out != nullptr && g == 0 && valid) a.logits_out[row0 + myq] = z;
            float dz = 0.f;
            if (valid) {
                if (a.dz_mode == NCF_DZ_BCE) {
                    const float y = slab_[myq];
                    dz = (sigmoidf_(z) - y) / gb_f;
                    if (g == 0) lossAcc += bce_loss(z, y);
                } else if (a.dz_mode == NCF_DZ_KD) {
                    // distillation (base.py:40-50; response term: kd_response)
                    const float y = slab_[myq];
                    float rl;
                    const float rg = kd_response(z, stl2[buf * TRW + myq], a.kd_temp, &rl);
                    dz = (a.kd_wt * (sigmoidf_(z) - y) + a.kd_wr * rg) / gb_f;
                    if (g == 0) lossAcc += a.kd_wt * bce_loss(z, y) + a.kd_wr * rl;
                } else {
                    dz = slab_[myq];  // labels[] carries dL/dlogit
                }
            }
            if (g == 0) {
                sdz[myq] = dz;
                dbpAcc += dz;
            }
            if (titer < 2) stamp(a, 45 + 3 * titer);  // diag sub-phase: loss + dz
            // GMF backward.  User side: unconditional atomics (padding rows add 0
            // to row 0).  Item side: kept for the per-item segment reduction.
            float gIg[NI];
            if constexpr (S_::GMF) {
#pragma unroll
                for (int j = 0; j < NI; ++j) {
                    const int q = wr + j * RPI + gq0;
                    const float dzq = sdz[q];
                    dWpG += dzq * (ugv[j] * igv[j]);
                    const float dgm = dzq * wpf;
                    if (a.ustore != nullptr)  // NCF_LAYOUT_USER_STORE: [Um part][Ug part] of row q
                        a.ustore[(row0 + q) * a.uw + (S_::MLP ? S_::DM : 0) + gf] = dgm * igv[j];
                    else if (!DIAG_ON(a, DIAG_NO_GMF_SCATTER))
                        atomicAdd(grads + lay.ug + (int64_t)max(su[q], 0) * F + gf, dgm * igv[j]);
                    gIg[j] = dgm * ugv[j];
                }
                if constexpr (EARLY) load_gmf(su2 + (buf ^ 1) * TRW, si2 + (buf ^ 1) * TRW, l);
            }
            stamp(a, sb + 2);

            if constexpr (S_::MLP) {
                f4 D[L][KT0];  // D[k] = dpre_k (orientation A)
#pragma unroll
                for (int mt = 0; mt < MTL; ++mt) {
                    const f4 h = H[L][mt];
                    f4 d;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int o = 16 * mt + 4 * g + r;
                        const float hv = lane_get(h, r);
                        const float wv = o < F ? sWP[S_::POFF + o] : 0.f;
                        set_r(d, r, hv > 0.f ? dz * wv : 0.f);
                    }
                    D[L - 1][mt] = d;
                    dWpT[mt].x += dz * h.x;
                    dWpT[mt].y += dz * h.y;
                    dWpT[mt].z += dz * h.z;
                    dWpT[mt].w += dz * h.w;
                }
                // layer-0 dX rows (orientation B: acc[nt] = C[i = row 4g+r][j = in-feature 16*nt + c])
                // scattered into the Um / Im rows of the gradient buffer through the wave's
                // scratch `scr`: item half segment-reduced (item_segments), user half
                // transposed so each atomic wave-instruction adds whole contiguous rows
                auto scatter_dx0 = [&](const f4 (&acc)[KT0], float* scr, const int* su, const int* si, int wr,
                                       int l, int c, int g, const float (&gIg)[NI], int gf, int gq0) {
                    constexpr int DM = S_::DM;
                    if constexpr (DM >= 16) {  // the split is 16-column aligned
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
#pragma unroll
                            for (int nt = DM / 16; nt < KT0; ++nt)
                                scr[(4 * g + r) * S_::SCM + 16 * nt + c - DM] = lane_get(acc[nt], r);
                        }
                        item_segments(scr, a, su, si, wr, l, gIg, gf, gq0);
                        // user half: transpose through the (now free) scratch so each
                        // atomic wave-instruction adds whole contiguous rows
                        // (min(DM, 64) floats per row) instead of 4 rows x 64 B
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
#pragma unroll
                            for (int nt = 0; nt < DM / 16; ++nt)
                                scr[(4 * g + r) * S_::SCM + 16 * nt + c] = lane_get(acc[nt], r);
                        }
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                        constexpr int RPW = DM >= 64 ? 1 : 64 / DM;  // rows per wave-instruction
                        constexpr int FPI = DM >= 64 ? 64 : DM;
                        constexpr int NQ = 16 / RPW, NF = DM / FPI;
                        // read every value first (one LDS wait), then the atomics back to back
                        float uv[NQ][NF];
                        int uid[NQ];
#pragma unroll
                        for (int qi = 0; qi < NQ; ++qi) {
                            const int q = qi * RPW + l / FPI;
                            uid[qi] = max(su[wr + q], 0);
#pragma unroll
                            for (int fi = 0; fi < NF; ++fi) uv[qi][fi] = scr[q * S_::SCM + fi * FPI + l % FPI];
                        }
#pragma unroll
                        for (int qi = 0; qi < NQ; ++qi) {
#pragma unroll
                            for (int fi = 0; fi < NF; ++fi) {
                                const int f = fi * FPI + l % FPI;
                                if (a.ustore != nullptr)
                                    a.ustore[(row0 + wr + qi * RPW + l / FPI) * a.uw + f] = uv[qi][fi];
                                else if (!DIAG_ON(a, DIAG_NO_USER_SCATTER))
                                    atomicAdd(grads + lay.um + (int64_t)uid[qi] * DM + f, uv[qi][fi]);
                            }
                        }
                    } else {  // DM == 8: one 16-column tile, lanes c < 8 user, c >= 8 item
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            if (c >= DM) scr[(4 * g + r) * S_::SCM + c - DM] = lane_get(acc[0], r);
                        item_segments(scr, a, su, si, wr, l, gIg, gf, gq0);
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int uu = max(su[wr + 4 * g + r], 0);
                            if (c < DM && a.ustore != nullptr)
                                a.ustore[(row0 + wr + 4 * g + r) * a.uw + c] = lane_get(acc[0], r);
                            else if (c < DM)
                                atomicAdd(grads + lay.um + (int64_t)uu * DM + c, lane_get(acc[0], r));
                        }
                    }
                };
                static_for<L>([&](auto ii) {
                    constexpr int k = L - 1 - decltype(ii)::value;
                    if constexpr (k >= 1) {
                        stamp(a, sb + 3 + 3 * (L - 1 - k));
                        // wgrad of layer k from this wave's own rows, no staging and no
                        // barrier: D_k and H_k (orientation A: row on the lane) are
                        // transposed to orientation B (rows in the K slots) by four
                        // exact selector MFMAs per 16x16 tile, and each 16x16 block of
                        // dW_k accumulates four MFMAs over the 16 rows in registers
                        // (summed over the waves once, in the epilogue); db_k likewise.
                        if (!(a.diag & DIAG_NO_WGRAD)) {
                            float sel[4];
#pragma unroll
                            for (int q = 0; q < 4; ++q) sel[q] = c == 4 * g + q ? 1.f : 0.f;
                            auto tr16 = [&](const f4& x) {
                                f4 y = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                                for (int q = 0; q < 4; ++q) y = MFMA4(lane_get(x, q), sel[q], y);
                                return y;
                            };
                            f4 DB[S_::MT(k)];
#pragma unroll
                            for (int mt = 0; mt < S_::MT(k); ++mt) {
                                DB[mt] = tr16(D[k][mt]);
                                dbK[S_::mb_off(k) + mt] += (DB[mt].x + DB[mt].y) + (DB[mt].z + DB[mt].w);
                            }
#pragma unroll
                            for (int t = 0; t < S_::KT(k); ++t) {
                                const f4 HB = tr16(H[k][t]);
#pragma unroll
                                for (int mt = 0; mt < S_::MT(k); ++mt) {
                                    f4& acc = accK[S_::kt_off(k) + mt * S_::KT(k) + t];
#pragma unroll
                                    for (int q = 0; q < 4; ++q) acc = MFMA4(lane_get(DB[mt], q), lane_get(HB, q), acc);
                                }
                            }
                        }
                        stamp(a, sb + 4 + 3 * (L - 1 - k));
                        // dgrad
                        const float* Ws = sW + S_::woff(k);
                        f4 acc[S_::KT(k)];
#pragma unroll
                        for (int m2 = 0; m2 < S_::KT(k); ++m2) acc[m2] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                        for (int t = 0; t < S_::MT(k); ++t) {
                            const f4 dv = D[k][t];
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                const float bv = lane_get(dv, r);
#pragma unroll
                                for (int m2 = 0; m2 < S_::KT(k); ++m2) {
                                    const float wv = Ws[(16 * t + 4 * g + r) * S_::SW(k) + 16 * m2 + c];
                                    acc[m2] = MFMA4(wv, bv, acc[m2]);
                                }
                            }
                            __builtin_amdgcn_sched_barrier(0);
                        }
#pragma unroll
                        for (int m2 = 0; m2 < S_::KT(k); ++m2) {
                            const f4 h = H[k][m2];
                            f4 d;
                            d.x = h.x > 0.f ? acc[m2].x : 0.f;
                            d.y = h.y > 0.f ? acc[m2].y : 0.f;
                            d.z = h.z > 0.f ? acc[m2].z : 0.f;
                            d.w = h.w > 0.f ? acc[m2].w : 0.f;
                            D[k - 1][m2] = d;
                        }
                        stamp(a, sb + 5 + 3 * (L - 1 - k));
                    } else if constexpr (FACT) {
                        // layer 0, factored: stage this wave's D0 rows row-major in its
                        // scratch, publish its next-tile ids (own rows only: no barrier),
                        // db0, next tile's embedding fragments, then scatter-add the D0
                        // rows into the user and the item rows of the gradient buffer.
                        float* scr = sstage + w * S_::WAVE_STAGE;
#pragma unroll
                        for (int mt = 0; mt < S_::MT(0); ++mt)
                            if (16 * mt + 4 * g < S_::S(1))
                                *reinterpret_cast<f4*>(scr + c * S_::SCM + 16 * mt + 4 * g) = D[0][mt];
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // same-wave LDS hand-off
                        stamp(a, sb + 3 + 3 * (L - 1));
                        if (l < S_::S(1)) {
                            float s = 0.f;
#pragma unroll
                            for (int rr = 0; rr < 16; ++rr) s += scr[rr * S_::SCM + l];
                            dbAcc[0] += s;
                        }
                        // EARLY: the next tile's fragments (issued after the forward and
                        // the GMF backward) are waited for here, before the scatter, as a
                        // waitcnt the compiler sees: their first uses in the next tile
                        // then need no wait that would also drain this tile's atomics.
                        if constexpr (EARLY) {
                            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
                            npr = npr2;  // the rows of tile t + 2, published in tile t + 1
                            ndl = ndl2;
                            nok = nok2;
                        }
                        stamp(a, sb + 4 + 3 * (L - 1));
                        item_segments(scr, a, su, si, wr, l, gIg, gf, gq0);
                        constexpr int RPW = DM >= 64 ? 1 : 64 / DM;  // rows per wave-instruction
                        constexpr int FPI = DM >= 64 ? 64 : DM;
                        constexpr int NQ = 16 / RPW, NF = (DM + FPI - 1) / FPI;
                        float uv[NQ][NF];
                        int uid[NQ];
#pragma unroll
                        for (int qi = 0; qi < NQ; ++qi) {
                            const int q = qi * RPW + l / FPI;
                            uid[qi] = max(su[wr + q], 0);
#pragma unroll
                            for (int fi = 0; fi < NF; ++fi) uv[qi][fi] = scr[q * S_::SCM + fi * FPI + l % FPI];
                        }
#pragma unroll
                        for (int qi = 0; qi < NQ; ++qi) {
#pragma unroll
                            for (int fi = 0; fi < NF; ++fi) {
                                const int f = fi * FPI + l % FPI;
                                if (a.ustore != nullptr)
                                    a.ustore[(row0 + wr + qi * RPW + l / FPI) * a.uw + f] = uv[qi][fi];
                                else if (!DIAG_ON(a, DIAG_NO_USER_SCATTER))
                                    atomicAdd(grads + lay.um + (int64_t)uid[qi] * DM + f, uv[qi][fi]);
                            }
                        }
                        stamp(a, sb + 5 + 3 * (L - 1));
                    } else if constexpr (OWN0) {
                        // layer 0, per row, small tower (Shape::OWN0): the wgrad from this
                        // wave's own 16 rows like layers k >= 1 (selector-MFMA transposes,
                        // dW0 tiles in registers, summed over the waves in the epilogue),
                        // db0 from the transposed D0, the dgrad in orientation B, then the
                        // scatter -- nothing staged across waves, no workgroup barrier
                        // (the next tile's ids and fragments come EARLY, as in FACT).
                        stamp(a, sb + 3 + 3 * (L - 1));
                        if (!(a.diag & DIAG_NO_WGRAD)) {
                            float sel[4];
#pragma unroll
                            for (int q = 0; q < 4; ++q) sel[q] = c == 4 * g + q ? 1.f : 0.f;
                            auto tr16 = [&](const f4& x) {
                                f4 y = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                                for (int q = 0; q < 4; ++q) y = MFMA4(lane_get(x, q), sel[q], y);
                                return y;
                            };
                            f4 DB[MT0];
#pragma unroll
                            for (int mt = 0; mt < MT0; ++mt) {
                                DB[mt] = tr16(D[0][mt]);
                                // lane (c, g): rows 4g .. 4g+3 of feature 16mt + c; the sum over
                                // g lands on every lane, lane 16g + c keeps feature 16g + c
                                float sdb = (DB[mt].x + DB[mt].y) + (DB[mt].z + DB[mt].w);
                                sdb += shfl_xor(sdb, 16);
                                sdb += shfl_xor(sdb, 32);
                                if (g == mt) dbAcc[0] += sdb;
                            }
#pragma unroll
                            for (int t = 0; t < KT0; ++t) {
                                const f4 HB = tr16(H[0][t]);
#pragma unroll
                                for (int mt = 0; mt < MT0; ++mt) {
                                    f4& acc = accL0[mt * KT0 + t];
#pragma unroll
                                    for (int q = 0; q < 4; ++q) acc = MFMA4(lane_get(DB[mt], q), lane_get(HB, q), acc);
                                }
                            }
                        }
                        const float* Ws = sW + S_::woff(0);
                        f4 acc[KT0];
#pragma unroll
                        for (int nt = 0; nt < KT0; ++nt) acc[nt] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                        for (int t = 0; t < S_::MT(0); ++t) {
                            const f4 dv = D[0][t];
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                const float av = lane_get(dv, r);
#pragma unroll
                                for (int nt = 0; nt < KT0; ++nt) {
                                    const float wv = Ws[(16 * t + 4 * g + r) * S_::SW(0) + 16 * nt + c];
                                    acc[nt] = MFMA4(av, wv, acc[nt]);
                                }
                                __builtin_amdgcn_sched_barrier(0);
                            }
                        }
                        // the next tile's fragments and rows (requested EARLY) are waited for
                        // here, before the scatter atomics (see the FACT branch)
                        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
                        npr = npr2;
                        ndl = ndl2;
                        nok = nok2;
                        stamp(a, sb + 4 + 3 * (L - 1));
                        scatter_dx0(acc, sstage + w * S_::WAVE_STAGE, su, si, wr, l, c, g, gIg, gf, gq0);
                        stamp(a, sb + 5 + 3 * (L - 1));
                    } else {
                        // layer 0: its wgrad needs every row of the tile -> stage this
                        // wave's D_0 rows (half titer & 1 when ALT0) and publish the next
                        // tile's indices with the tile's one barrier
                        const int RK0s = S_::ALT0 ? ((titer & 1) ? S_::HALF0 : 0) : 0;
                        float* st = sstage + w * S_::WAVE_STAGE + RK0s;
#pragma unroll
                        for (int mt = 0; mt < S_::MT(0); ++mt)
                            *reinterpret_cast<f4*>(st + c * S_::SD(0) + 16 * mt + 4 * g) = D[0][mt];
                        publish((buf ^ 1) * TRW);
                        lds_barrier();
                        stamp(a, sb + 3 + 3 * (L - 1));
                        // bias grad: this wave's 16 rows, lane = output feature
                        if (l < S_::S(1)) {
                            float s = 0.f;
#pragma unroll
                            for (int rr = 0; rr < 16; ++rr) s += st[rr * S_::SD(0) + l];
                            dbAcc[0] += s;
                        }
                    auto wgrad0 = [&]() {
                        if (!(a.diag & DIAG_NO_WGRAD)) {
                            // layer-0 staging region of this tile (see RK below)
                            const int RK0 = S_::ALT0 ? ((titer & 1) ? S_::HALF0 : 0) : 0;
#pragma unroll
                            for (int j = 0; j < CB0; ++j) {
                                if (w + j * NWV >= KT0) break;  // wave-uniform
#pragma unroll
                                for (int mt = 0; mt < MT0; ++mt) {
                                    f4 acc0 = accW0[j][mt], acc1 = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                                    for (int ws = 0; ws < NWV; ++ws) {
                                        const float* sto = sstage + ws * S_::WAVE_STAGE + RK0;
#pragma unroll
                                        for (int s = 0; s < 4; ++s) {
                                            const float av = sto[(4 * g + s) * S_::SD(0) + 16 * mt + c];
                                            if (ws & 1)
                                                acc1 = MFMA4(av, bx[j][ws * 4 + s], acc1);
                                            else
                                                acc0 = MFMA4(av, bx[j][ws * 4 + s], acc0);
                                        }
                                        if (ws & 1) __builtin_amdgcn_sched_barrier(0);
                                    }
                                    acc0.x += acc1.x;
                                    acc0.y += acc1.y;
                                    acc0.z += acc1.z;
                                    acc0.w += acc1.w;
                                    accW0[j][mt] = acc0;
                                }
                            }
                        }
                    };
                        // Waves s and s + 4 share SIMD s: the upper half runs the layer-0
                        // wgrad first, so each SIMD overlaps one wave's scatter with the
                        // other's MFMAs (both orders when WGRAD0_LATE; else wgrad first).
                        if (!S_::WGRAD0_LATE || wv_hi) wgrad0();
                        // (h) next tile's embedding fragments: before this tile's
                        // scatter atomics, so the next tile waits on them only
                        load_emb(su2 + (buf ^ 1) * TRW, si2 + (buf ^ 1) * TRW, c, g, l);
                        const float* Ws = sW + S_::woff(0);
                        // orientation B: C[i = row 4g+r][j = in-feature 16*nt + c]
                        f4 acc[KT0];
#pragma unroll
                        for (int nt = 0; nt < KT0; ++nt) acc[nt] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                        for (int t = 0; t < S_::MT(0); ++t) {
                            const f4 dv = D[0][t];
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                const float av = lane_get(dv, r);
#pragma unroll
                                for (int nt = 0; nt < KT0; ++nt) {
                                    const float wv = Ws[(16 * t + 4 * g + r) * S_::SW(0) + 16 * nt + c];
                                    acc[nt] = MFMA4(av, wv, acc[nt]);
                                }
                                __builtin_amdgcn_sched_barrier(0);
                            }
                        }
                        // The layer-0 wgrad operands (bx, loaded in (d)) must be complete
                        // before the scatter: consumed here, the wait is a counted one on
                        // old loads; at their use after the branchy scatter it would
                        // drain the atomics too.
                        if (S_::WGRAD0_LATE && !wv_hi) {
#pragma unroll
                            for (int i = 0; i < NWV * 4; ++i)
#pragma unroll
                                for (int j = 0; j < CB0; ++j) asm volatile("" ::"v"(bx[j][i]));
                        }
                        stamp(a, sb + 4 + 3 * (L - 1));
                        // item half -> this wave's scratch rows (segment-reduced below);
                        // user half -> unconditional atomics (padding rows add 0 to row 0)
                        // scratch: the half / region not holding this tile's layer-0 staging
                        float* scr = sstage + w * S_::WAVE_STAGE + (S_::ALT0 ? ((titer & 1) ? 0 : S_::HALF0) : S_::ST0);
                        scatter_dx0(acc, scr, su, si, wr, l, c, g, gIg, gf, gq0);
                        stamp(a, sb + 5 + 3 * (L - 1));
                        if (S_::WGRAD0_LATE && !wv_hi) wgrad0();
                    }
                });
            } else {
                // GMF-only model: item-side GMF rows, then publish next indices
                item_segments(sstage + w * S_::WAVE_STAGE, a, su, si, wr, l, gIg, gf, gq0);
                publish((buf ^ 1) * TRW);
                lds_barrier();
                load_emb(su2 + (buf ^ 1) * TRW, si2 + (buf ^ 1) * TRW, c, g, l);
            }
            // Tile end: no barrier unless the staging layout needs one (END_BARRIER):
            // the next tile's first cross-wave staging goes to the other region and
            // its first barrier resynchronises, so a wave still scattering overlaps
            // the others' next forward.
            if constexpr (S_::END_BARRIER && !FACT && !OWN0) lds_barrier();
            stamp(a, sb + 13);
            ++titer;
        }
    }

    if constexpr (!FWD_ONLY) {
        // ---- this workgroup's tower/predict partial -> its slab row, stored straight
        // from registers (sums over the waves through per-wave LDS images).  Every
        // slab entry in [lo, len) is written exactly once, the alignment gaps with 0.
        const int64_t tb = lay.tower_begin;
        const int len = (int)lay.tower_len + 64;  // slab stride (ncf_slab_stride); loss at tower_len
        float* out = a.slab + (int64_t)blockIdx.x * len;
        // AIS: no slab -- the tower partials (and the loss at tower_len) are added into the
        // gradient buffer, which the next launch reads like the embedding rows
        auto put = [&](int64_t pos, float v) {
            if constexpr (AIS) {
#ifndef NCF_AIS_NO_TOWER_ATOMICS  // timing experiment only (wrong results)
                atomicAdd(grads + tb + pos, v);
#endif
            } else {
                out[pos] = v;
            }
        };
        const int l = l0, c = c0, g = g0;
        // layer-0 wgrad: this wave's 16-column block, already summed over the rows
        // (FACT: formed after the step by fact_expand_kernel; its slab columns unused;
        // OWN0: per-wave tiles, summed over the waves with layers k >= 1 below)
        if constexpr (S_::MLP && !FACT && !OWN0) {
#pragma unroll
            for (int j = 0; j < CB0; ++j) {
                const int ntj = w + j * NWV;
                if (ntj >= KT0) break;
#pragma unroll
                for (int mt = 0; mt < MT0; ++mt) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int o = 16 * mt + 4 * g + r;
                        if (o < S_::S(1)) put((lay.w[0] - tb) + o * S_::S(0) + 16 * ntj + c, lane_get(accW0[j][mt], r));
                    }
                }
            }
        }
        // Tail partials [db_0 | wp | bp | loss]: reduced inside the wave by shuffles
        // (before the barrier), then one per-wave LDS image like the layers k >= 1.
        constexpr int S1 = S_::MLP ? S_::S(1) : 0;
        constexpr int NT = S1 + S_::P + 2;
        // the tail rides with the last layer's round where both images fit
        constexpr bool TAIL_MERGED = S_::MLP && L >= 2 && S_::rwk(L - 1) + NT <= S_::WAVE_STAGE;
        constexpr int TOFF = TAIL_MERGED ? S_::rwk(L - 1) : 0;
        static_assert(TOFF + NT <= S_::WAVE_STAGE, "epilogue tail image");
        float tw[MTL][4];  // predict-weight partials summed over the wave's rows (lanes c == 0)
        if constexpr (S_::MLP) {
#pragma unroll
            for (int mt = 0; mt < MTL; ++mt) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float v = lane_get(dWpT[mt], r);  // row c, predict input 16mt + 4g + r
#pragma unroll
                    for (int m = 1; m < 16; m <<= 1) v += shfl_xor(v, m);
                    tw[mt][r] = v;
                }
            }
        }
        float vg = dWpG;  // GMF: feature l % F, rows l / F
        if constexpr (S_::GMF) {
#pragma unroll
            for (int m = F; m < 64; m <<= 1) vg += shfl_xor(vg, m);
        }
        float vb = dbpAcc, vl = lossAcc;  // nonzero on g == 0 lanes only
#pragma unroll
        for (int m = 1; m < 64; m <<= 1) {
            vb += shfl_xor(vb, m);
            vl += shfl_xor(vl, m);
        }
        auto write_tail = [&]() {
            float* tv = sstage + w * S_::WAVE_STAGE + TOFF;
            if constexpr (S_::MLP) {
                if (l < S1) tv[l] = dbAcc[0];
#pragma unroll
                for (int mt = 0; mt < MTL; ++mt) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int o = 16 * mt + 4 * g + r;
                        if (c == 0 && o < F) tv[S1 + S_::POFF + o] = tw[mt][r];
                    }
                }
            }
            if constexpr (S_::GMF)
                if (l < F) tv[S1 + l] = vg;
            if (l == 0) {
                tv[S1 + S_::P] = vb;
                tv[S1 + S_::P + 1] = vl / gb_f;
            }
        };
        auto sum_tail = [&]() {
            for (int e = tid; e < NT; e += NTH) {
                float ts = 0.f;
#pragma unroll
                for (int ws = 0; ws < NWV; ++ws) ts += sstage[ws * S_::WAVE_STAGE + TOFF + e];
                const int64_t pos = e < S1 ? (lay.b[0] - tb) + e
                                  : e < S1 + S_::P ? (lay.wp - tb) + (e - S1)
                                  : e == S1 + S_::P ? (lay.bp - tb) : (int64_t)lay.tower_len;
                put(pos, ts);
            }
        };
        // every wave past its last tile: the staging is free.  FACT: a wave's staging
        // slot was private to it during the tiles (no layer-0 wgrad across waves), so
        // each wave writes its images into it as soon as it is done, and the first
        // cross-wave read below waits at that round's barrier instead.
        if constexpr (!FACT && !OWN0) lds_barrier();
        stamp(a, 62);
        if constexpr (S_::MLP && (L >= 2 || OWN0)) {
            // Layers k >= 1 (and layer 0 under OWN0): each wave writes its register
            // partials to its own LDS image, then every thread sums its share of the
            // entries over the waves (plain stores and loads: LDS float atomics run ~2
            // cycles per lane).  OWN0's db0 rides in the tail (dbAcc[0]).
            static_for<L>([&](auto kk) {
                constexpr int k = decltype(kk)::value;
                if constexpr (k >= 1 || OWN0) {
                    constexpr int SK = S_::S(k), SO = S_::S(k + 1);
                    constexpr bool BIAS = k >= 1;
                    float* im = sstage + w * S_::WAVE_STAGE;
#pragma unroll
                    for (int mt = 0; mt < S_::MT(k); ++mt) {
#pragma unroll
                        for (int t = 0; t < S_::KT(k); ++t) {
                            f4 v;
                            if constexpr (k >= 1)
                                v = accK[S_::kt_off(k) + mt * S_::KT(k) + t];
                            else
                                v = accL0[mt * KT0 + t];
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                const int o = 16 * mt + 4 * g + r;
                                if (o < SO) im[o * SK + 16 * t + c] = lane_get(v, r);
                            }
                        }
                        if constexpr (BIAS) {
                            const int o = 16 * mt + c;
                            if (o < SO) im[SO * SK + g * SO + o] = dbK[S_::mb_off(k) + mt];
                        }
                    }
                    if constexpr (TAIL_MERGED && k == L - 1) write_tail();
                    lds_barrier();
                    constexpr int NE = (SO * SK + (BIAS ? SO : 0) + NTH - 1) / NTH;
#pragma unroll
                    for (int j = 0; j < NE; ++j) {
                        const int e = tid + j * NTH;
                        if (e < SO * SK) {
                            float s = 0.f;
#pragma unroll
                            for (int ws = 0; ws < NWV; ++ws) s += sstage[ws * S_::WAVE_STAGE + e];
                            put((lay.w[k] - tb) + e, s);
                        } else if (BIAS && e < SO * SK + SO) {
                            float s = 0.f;
#pragma unroll
                            for (int ws = 0; ws < NWV; ++ws)
#pragma unroll
                                for (int gg = 0; gg < 4; ++gg) s += sstage[ws * S_::WAVE_STAGE + SO * SK + gg * SO + (e - SO * SK)];
                            put((lay.b[k] - tb) + (e - SO * SK), s);
                        }
                    }
                    if constexpr (TAIL_MERGED && k == L - 1)
                        sum_tail();
                    else
                        lds_barrier();
                }
            });
        }
        if constexpr (!TAIL_MERGED) {
            write_tail();
            lds_barrier();
            sum_tail();
        }
        stamp(a, 60);
        // alignment gaps of the 64-float segments (ncf_layout_init)
        auto zero_gap = [&](int64_t seg, int n) {
            const int gap = ((n + 63) & ~63) - n;
            if (!AIS && tid < gap) out[(seg - tb) + n + tid] = 0.f;
        };
        if constexpr (S_::MLP) {
            static_for<L>([&](auto kk) {
                constexpr int k = decltype(kk)::value;
                if (!FACT || k > 0) zero_gap(lay.w[k], S_::S(k + 1) * S_::S(k));
                zero_gap(lay.b[k], S_::S(k + 1));
            });
        }
        zero_gap(lay.wp, S_::P);
        zero_gap(lay.bp, 1);
        zero_gap(tb + lay.tower_len, 1);
#ifdef NCF_STAMPS
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
        stamp(a, 61);
    }
}

// ---------------------------------------------------------------------------
// host-side dispatch table
// Narrow workgroups (4 / 2 / 1 waves) for the small shapes: each thread stages a
// 1/(64 waves) share of the tower weights through registers in the prologue (at most
// 16 16-byte pieces, WREG), and the per-row layer-0 wgrad gives each wave
// CB0 = KT(0) / waves column blocks of dW0 in registers, so that kernel is built where
// dW0 has at most 8 16x16 tiles (the factored kernel and GMF have no such term).
template <int F, int L, int MODE, int G>
static void set_geo(KernelEntry& e) {
    constexpr int NW = geo_waves(G);
    using SG = Shape<F, L, MODE, NW>;
    using S8 = Shape<F, L, MODE>;
    constexpr bool regs_ok = NW == NWAVES || SG::WREG <= 16;  // the prologue's weight registers
#ifndef NCF_FACT_WREG_MAX
#define NCF_FACT_WREG_MAX 16
#endif
    constexpr bool fregs_ok = NW == NWAVES || SG::WREG <= NCF_FACT_WREG_MAX;  // (A/B switch)
    if constexpr (regs_ok && (!S8::MLP || S8::MT(0) * S8::KT(0) <= 8 || NW == NWAVES))
        e.train[G] = reinterpret_cast<const void*>(&ncf_step_kernel<F, L, MODE, false, false, NW>);
    else
        e.train[G] = nullptr;
    if constexpr (S8::MLP && fregs_ok)
        e.train_fact[G] = reinterpret_cast<const void*>(&ncf_step_kernel<F, L, MODE, false, true, NW>);
    else
        e.train_fact[G] = nullptr;
    // in-step Adam (NCF_LAYOUT_ADAM_IN_STEP): the small-batch geometries
    if constexpr (G != GEO_8 && regs_ok && (!S8::MLP || S8::MT(0) * S8::KT(0) <= 8))
        e.train_ais[G] = reinterpret_cast<const void*>(&ncf_step_kernel<F, L, MODE, false, false, NW, true>);
    else
        e.train_ais[G] = nullptr;
    e.misc[G] = SG::MISC;
    e.stage[G] = NW * SG::WAVE_STAGE;
}

template <int F, int L, int MODE>
static KernelEntry make_entry() {
    using S_ = Shape<F, L, MODE>;
    KernelEntry e;
    e.mode = MODE;
    e.F = F;
    e.L = L;
    set_geo<F, L, MODE, GEO_8>(e);
    set_geo<F, L, MODE, GEO_4>(e);
    set_geo<F, L, MODE, GEO_2>(e);
    set_geo<F, L, MODE, GEO_1>(e);
    e.fwd = reinterpret_cast<const void*>(&ncf_step_kernel<F, L, MODE, true, false, NWAVES>);
    e.w_total = S_::W_TOTAL;
    return e;
}

const KernelEntry* kernel_table(int* n) {
    static const KernelEntry table[] = {
#ifdef NCF_DEV_ONE
        make_entry<16, 3, NCF_MODEL_NEUMF>(),
#else
        make_entry<8, 1, NCF_MODEL_GMF>(),   make_entry<16, 1, NCF_MODEL_GMF>(),
        make_entry<32, 1, NCF_MODEL_GMF>(),  make_entry<64, 1, NCF_MODEL_GMF>(),
#define NCF_TOWER(F, L) make_entry<F, L, NCF_MODEL_MLP>(), make_entry<F, L, NCF_MODEL_NEUMF>()
        NCF_TOWER(8, 1),  NCF_TOWER(8, 2),  NCF_TOWER(8, 3),  NCF_TOWER(8, 4),  NCF_TOWER(16, 1),
        NCF_TOWER(16, 2), NCF_TOWER(16, 3), NCF_TOWER(32, 1), NCF_TOWER(32, 2), NCF_TOWER(64, 1),
#undef NCF_TOWER
#endif
    };
    *n = (int)(sizeof(table) / sizeof(table[0]));
    return table;
}

}  // namespace ncf
