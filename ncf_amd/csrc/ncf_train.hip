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

__device__ __forceinline__ void set_r(f4& v, int r, float x) {
    if (r == 0) v.x = x;
    else if (r == 1) v.y = x;
    else if (r == 2) v.z = x;
    else v.w = x;
}

template <int F, int L, int MODE, bool FWD_ONLY>
__global__ __launch_bounds__(NTHREADS, 2) void ncf_step_kernel(TrainArgs a) {
    using S_ = Shape<F, L, MODE>;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* sW = smem;
    int* su = reinterpret_cast<int*>(smem + S_::W_TOTAL);
    int* si = su + TILE_ROWS;
    float* slab_ = reinterpret_cast<float*>(si + TILE_ROWS);
    float* szg = slab_ + TILE_ROWS;
    float* sdz = szg + TILE_ROWS;
    float* sstage = sdz + TILE_ROWS;  // union: per-wave staging | slab image

    const int tid = threadIdx.x;
    const int w = tid >> 6;
    const int l0 = tid & 63;
    const int c0 = l0 & 15;
    const int g0 = l0 >> 4;
    const ncf_layout& lay = a.lay;
    const float* __restrict__ prm = a.params;

    // ---- rows of this rank -------------------------------------------------
    int64_t base, nloc;
    float gb_f = 1.0f;
    if constexpr (FWD_ONLY) {
        base = 0;
        nloc = a.fwd_n;
    } else {
        const int64_t ntot = a.ctl->n_total;
        const int64_t nbatch = (ntot + a.batch_global - 1) / a.batch_global;
        const int64_t b = nbatch > 0 ? a.ctl->batch % nbatch : 0;  // epochs repeat past the end
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
    }
    const int64_t ntiles = (nloc + TILE_ROWS - 1) / TILE_ROWS;

    // ---- tower weights -> LDS (rows padded to 16*MT with zeros) -------------
    if constexpr (S_::MLP) {
        static_for<L>([&](auto kk) {
            constexpr int k = decltype(kk)::value;
            constexpr int rows = 16 * S_::MT(k), cols = S_::S(k), outs = S_::S(k + 1);
            const float* Wg = prm + lay.w[k];
            float* Ws = sW + S_::woff(k);
            for (int e = tid; e < rows * cols; e += NTHREADS) {
                const int o = e / cols, i = e - o * cols;
                Ws[o * S_::SW(k) + i] = o < outs ? Wg[e] : 0.0f;
            }
        });
    }

    // ---- per-lane persistent accumulators ----------------------------------
    constexpr int TPW0 = S_::TPW(0) > 0 ? S_::TPW(0) : 1;
    constexpr int MTL = S_::MLP ? S_::MT(L - 1) : 1;
    f4 accW[L][TPW0];
    float dbAcc[L];
    f4 dWpT[MTL];
    float dWpG = 0.f, dbpAcc = 0.f, lossAcc = 0.f;
#pragma unroll
    for (int k = 0; k < L; ++k) {
        dbAcc[k] = 0.f;
#pragma unroll
        for (int j = 0; j < TPW0; ++j) accW[k][j] = f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int t = 0; t < MTL; ++t) dWpT[t] = f4{0.f, 0.f, 0.f, 0.f};

    constexpr int RPI = S_::GMF ? 64 / F : 1;  // GMF rows per wave-instruction
    constexpr int NI = S_::GMF ? 16 / RPI : 1;
    const float bpv = prm[lay.bp];
    const float wpf = S_::GMF ? prm[lay.wp + l0 % F] : 0.f;
    __syncthreads();

    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t row0 = tile * TILE_ROWS;
        if (tid < TILE_ROWS) {
            const int64_t r = row0 + tid;
            const bool ok = r < nloc;
            su[tid] = ok ? a.users[base + r] : -1;
            si[tid] = ok ? a.items[base + r] : -1;
            if constexpr (!FWD_ONLY) slab_[tid] = ok ? a.labels[base + r] : 0.f;
        }
        __syncthreads();
        const int wr = w * 16;  // first WG-tile row of this wave
        // Opaque per-tile copies of the lane coordinates: every address below is
        // recomputed inside the tile loop instead of being hoisted out of it and
        // held in (spilled) VGPRs for the whole launch.
        int c = c0, g = g0, l = l0;
        asm volatile("" : "+v"(c), "+v"(g), "+v"(l));
        const int gf = l % F;
        const int gq0 = l / F;

        // ================= GMF forward (row-major lanes: f = l % F) ==========
        float ugv[NI], igv[NI];
        if constexpr (S_::GMF) {
#pragma unroll
            for (int j = 0; j < NI; ++j) {
                const int q = wr + j * RPI + gq0;
                const int u = su[q] < 0 ? 0 : su[q];
                const int it = si[q] < 0 ? 0 : si[q];
                ugv[j] = prm[lay.ug + (int64_t)u * F + gf];
                igv[j] = prm[lay.ig + (int64_t)it * F + gf];
            }
#pragma unroll
            for (int j = 0; j < NI; ++j) {
                float v = wpf * (ugv[j] * igv[j]);
#pragma unroll
                for (int m = 1; m < F; m <<= 1) v += shfl_xor(v, m);
                if (gf == 0) szg[wr + j * RPI + gq0] = v;
            }
        }

        // ================= MLP forward (orientation A) =======================
        const int myq = wr + c;
        f4 H[L + 1][S_::KT0];
        if constexpr (S_::MLP) {
            constexpr int DM = S_::DM;
            const int uc = su[myq] < 0 ? 0 : su[myq];
            const int ic = si[myq] < 0 ? 0 : si[myq];
#pragma unroll
            for (int t = 0; t < S_::KT(0); ++t) {
                const int j0 = 16 * t + 4 * g;
                const bool isu = j0 < DM;
                const int64_t off = isu ? lay.um + (int64_t)uc * DM + j0 : lay.im + (int64_t)ic * DM + (j0 - DM);
                H[0][t] = *reinterpret_cast<const f4*>(prm + off);
            }
            static_for<L>([&](auto kk) {
                constexpr int k = decltype(kk)::value;
                f4 acc[S_::MT(k)];
                const float* bk = prm + lay.b[k];
#pragma unroll
                for (int mt = 0; mt < S_::MT(k); ++mt) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int o = 16 * mt + 4 * g + r;
                        set_r(acc[mt], r, o < S_::S(k + 1) ? bk[o] : 0.f);
                    }
                }
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

        // ================= predict + loss + dlogit ===========================
        float zt = 0.f;
        if constexpr (S_::MLP) {
#pragma unroll
            for (int mt = 0; mt < MTL; ++mt) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int o = 16 * mt + 4 * g + r;
                    if (o < F) zt += prm[lay.wp + S_::POFF + o] * lane_get(H[L][mt], r);
                }
            }
            zt += shfl_xor(zt, 16);
            zt += shfl_xor(zt, 32);
        }
        if constexpr (S_::GMF) zt += szg[myq];
        const float z = zt + bpv;
        const bool valid = su[myq] >= 0;
        if constexpr (FWD_ONLY) {
            if (g == 0 && valid) a.logits_out[base + row0 + myq] = z;
            __syncthreads();
            continue;
        } else {
            if (a.logits_out != nullptr && g == 0 && valid) a.logits_out[row0 + myq] = z;
            float dz = 0.f;
            if (valid) {
                if (a.dz_mode == NCF_DZ_BCE) {
                    const float y = slab_[myq];
                    dz = (sigmoidf_(z) - y) / gb_f;
                    if (g == 0) lossAcc += bce_loss(z, y);
                } else {
                    dz = slab_[myq];  // labels[] carries dL/dlogit
                }
            }
            if (g == 0) {
                sdz[myq] = dz;
                dbpAcc += dz;
            }

            // ============= GMF backward (row-major lanes) =====================
            if constexpr (S_::GMF) {
#pragma unroll
                for (int j = 0; j < NI; ++j) {
                    const int q = wr + j * RPI + gq0;
                    const float dzq = sdz[q];
                    dWpG += dzq * (ugv[j] * igv[j]);
                    if (su[q] >= 0 && !(a.diag & DIAG_NO_ATOMICS)) {
                        const float dgm = dzq * wpf;
                        atomicAdd(a.grads + lay.ug + (int64_t)su[q] * F + gf, dgm * igv[j]);
                        atomicAdd(a.grads + lay.ig + (int64_t)si[q] * F + gf, dgm * ugv[j]);
                    }
                }
            }

            // ============= MLP backward =======================================
            if constexpr (S_::MLP) {
                f4 D[L][S_::KT0];  // D[k] = dpre_k (orientation A)
#pragma unroll
                for (int mt = 0; mt < MTL; ++mt) {
                    const f4 h = H[L][mt];
                    f4 d;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int o = 16 * mt + 4 * g + r;
                        const float hv = lane_get(h, r);
                        const float wv = o < F ? prm[lay.wp + S_::POFF + o] : 0.f;
                        set_r(d, r, hv > 0.f ? dz * wv : 0.f);
                    }
                    D[L - 1][mt] = d;
                    dWpT[mt].x += dz * h.x;
                    dWpT[mt].y += dz * h.y;
                    dWpT[mt].z += dz * h.z;
                    dWpT[mt].w += dz * h.w;
                }
                static_for<L>([&](auto ii) {
                    constexpr int k = L - 1 - decltype(ii)::value;
                    constexpr int RK = (k & 1) ? S_::R0 : 0;
                    // ---- stage dpre_k (and H_k) row-major for the shared wgrad
                    float* st = sstage + w * S_::WAVE_STAGE + RK;
#pragma unroll
                    for (int mt = 0; mt < S_::MT(k); ++mt)
                        *reinterpret_cast<f4*>(st + c * S_::SD(k) + 16 * mt + 4 * g) = D[k][mt];
                    if constexpr (k >= 1) {
                        float* sh = st + 16 * S_::SD(k);
#pragma unroll
                        for (int t = 0; t < S_::KT(k); ++t)
                            *reinterpret_cast<f4*>(sh + c * S_::SH(k) + 16 * t + 4 * g) = H[k][t];
                    }
                    __syncthreads();
                    // ---- bias grad: this wave's 16 rows, lane = output feature
                    if (l < S_::S(k + 1)) {
                        float s = 0.f;
#pragma unroll
                        for (int rr = 0; rr < 16; ++rr) s += st[rr * S_::SD(k) + l];
                        dbAcc[k] += s;
                    }
                    // ---- wgrad: dW_k[out][in] += sum_rows dpre_k[row][out] * H_k[row][in]
                    constexpr int T = S_::MT(k) * S_::KT(k);
                    constexpr int tpw = S_::TPW(k);
                    float bx[k == 0 ? NWAVES * 4 : 1];
                    int loaded_nt = -1;
#pragma unroll
                    for (int jl = 0; jl < tpw; ++jl) {
                        const int j = w * tpw + jl;
                        if (j < T && !(a.diag & DIAG_NO_WGRAD)) {
                            const int mt = j % S_::MT(k);
                            const int nt = j / S_::MT(k);
                            if constexpr (k == 0) {
                                if (nt != loaded_nt) {
                                    // layer-0 input rows come straight from the embedding tables
                                    constexpr int DM = S_::DM;
                                    const int fj = 16 * nt + c;
#pragma unroll
                                    for (int ws = 0; ws < NWAVES; ++ws) {
#pragma unroll
                                        for (int s = 0; s < 4; ++s) {
                                            const int q = ws * 16 + 4 * g + s;
                                            const bool isu = fj < DM;
                                            const int id = max(isu ? su[q] : si[q], 0);
                                            const int64_t off = (isu ? lay.um : lay.im - DM) + (int64_t)id * DM + fj;
                                            bx[ws * 4 + s] = prm[off];
                                        }
                                    }
                                    loaded_nt = nt;
                                }
                            }
                            f4 acc = accW[k][jl];
#pragma unroll
                            for (int ws = 0; ws < NWAVES; ++ws) {
                                const float* sto = sstage + ws * S_::WAVE_STAGE + RK;
#pragma unroll
                                for (int s = 0; s < 4; ++s) {
                                    const int row = 4 * g + s;
                                    const float av = sto[row * S_::SD(k) + 16 * mt + c];
                                    float bv;
                                    if constexpr (k >= 1)
                                        bv = sto[16 * S_::SD(k) + row * S_::SH(k) + 16 * nt + c];
                                    else
                                        bv = bx[ws * 4 + s];
                                    acc = MFMA4(av, bv, acc);
                                }
                                __builtin_amdgcn_sched_barrier(0);
                            }
                            accW[k][jl] = acc;
                        }
                    }
                    // ---- dgrad
                    const float* Ws = sW + S_::woff(k);
                    if constexpr (k >= 1) {
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
                    } else {
                        // orientation B: C[i = row 4g+r][j = in-feature 16*nt + c]
                        constexpr int DM = S_::DM;
                        f4 acc[S_::KT(0)];
#pragma unroll
                        for (int nt = 0; nt < S_::KT(0); ++nt) acc[nt] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                        for (int t = 0; t < S_::MT(0); ++t) {
                            const f4 dv = D[0][t];
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                const float av = lane_get(dv, r);
#pragma unroll
                                for (int nt = 0; nt < S_::KT(0); ++nt) {
                                    const float wv = Ws[(16 * t + 4 * g + r) * S_::SW(0) + 16 * nt + c];
                                    acc[nt] = MFMA4(av, wv, acc[nt]);
                                }
                                __builtin_amdgcn_sched_barrier(0);
                            }
                        }
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int q = wr + 4 * g + r;
                            const int uu = su[q];
                            const int iq = si[q];
                            if (uu >= 0 && !(a.diag & DIAG_NO_ATOMICS)) {
#pragma unroll
                                for (int nt = 0; nt < S_::KT(0); ++nt) {
                                    const int fj = 16 * nt + c;
                                    const bool isu = fj < DM;
                                    const int64_t off = (isu ? lay.um : lay.im - DM) + (int64_t)(isu ? uu : iq) * DM + fj;
                                    atomicAdd(a.grads + off, lane_get(acc[nt], r));
                                }
                            }
                        }
                    }
                });
            }
            __syncthreads();
        }
    }

    if constexpr (!FWD_ONLY) {
        // ---- this workgroup's tower/predict partial: assemble in LDS, store once
        const int64_t tb = lay.tower_begin;
        const int lo = S_::MLP ? 0 : (int)(lay.wp - tb);
        const int len = (int)lay.tower_len + 64;  // slab stride (ncf_slab_stride); loss at tower_len
        float* img = sstage;
        const int l = l0, c = c0, g = g0, gf = l0 % F;
        __syncthreads();
        for (int e = lo + tid; e < len; e += NTHREADS) img[e] = 0.f;
        __syncthreads();
        if constexpr (S_::MLP) {
            static_for<L>([&](auto kk) {
                constexpr int k = decltype(kk)::value;
                constexpr int T = S_::MT(k) * S_::KT(k);
                constexpr int tpw = S_::TPW(k);
                float* dW = img + (lay.w[k] - tb);
#pragma unroll
                for (int jl = 0; jl < tpw; ++jl) {
                    const int j = w * tpw + jl;
                    if (j < T) {
                        const int mt = j % S_::MT(k);
                        const int nt = j / S_::MT(k);
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int o = 16 * mt + 4 * g + r;
                            if (o < S_::S(k + 1)) dW[o * S_::S(k) + 16 * nt + c] = lane_get(accW[k][jl], r);
                        }
                    }
                }
                if (l < S_::S(k + 1)) atomicAdd(img + (lay.b[k] - tb) + l, dbAcc[k]);
            });
#pragma unroll
            for (int mt = 0; mt < MTL; ++mt) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int o = 16 * mt + 4 * g + r;
                    if (o < F) atomicAdd(img + (lay.wp - tb) + S_::POFF + o, lane_get(dWpT[mt], r));
                }
            }
        }
        if constexpr (S_::GMF) atomicAdd(img + (lay.wp - tb) + gf, dWpG);
        if (g == 0) {
            atomicAdd(img + (lay.bp - tb), dbpAcc);
            atomicAdd(img + lay.tower_len, lossAcc / gb_f);
        }
        __syncthreads();
        float* out = a.slab + (int64_t)blockIdx.x * len;
        for (int e = lo + tid; e < len; e += NTHREADS) out[e] = img[e];
    }
}

// ---------------------------------------------------------------------------
// host-side dispatch table
template <int F, int L, int MODE>
static KernelEntry make_entry() {
    using S_ = Shape<F, L, MODE>;
    KernelEntry e;
    e.mode = MODE;
    e.F = F;
    e.L = L;
    e.train = reinterpret_cast<const void*>(&ncf_step_kernel<F, L, MODE, false>);
    e.fwd = reinterpret_cast<const void*>(&ncf_step_kernel<F, L, MODE, true>);
    e.w_total = S_::W_TOTAL;
    e.misc = S_::MISC;
    e.stage8 = NWAVES * S_::WAVE_STAGE;
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
