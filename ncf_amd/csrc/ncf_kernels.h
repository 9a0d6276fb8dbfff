// Internal (C++) declarations shared by the kernel translation units and the C ABI.
#pragma once
#include "ncf_adam.h"
#include "ncf_common.h"

namespace ncf {

constexpr int NWAVES = 8;
constexpr int NTHREADS = NWAVES * WAVE;
constexpr int TILE_ROWS = NWAVES * 16;
constexpr int SLAB_ROWS = 256;  // one workgroup per CU on MI355X
constexpr int LDS_LIMIT_BYTES = 160 * 1024;

// NW_: waves per workgroup of the fused step (16 rows each per tile): NWAVES, or 4
// for small per-rank batches (twice the workgroups, one wave per SIMD).
template <int F_, int L_, int MODE_, int NW_ = NWAVES>
struct Shape {
    static constexpr int F = F_, L = L_, MODE = MODE_;
    static constexpr int NWV = NW_, NTH = NW_ * WAVE, TR = NW_ * 16;
    static constexpr bool GMF = MODE != NCF_MODEL_MLP;
    static constexpr bool MLP = MODE != NCF_MODEL_GMF;
    static constexpr int DM = F << (L - 1);
    static constexpr int P = (MODE == NCF_MODEL_NEUMF) ? 2 * F : F;
    static constexpr int POFF = (MODE == NCF_MODEL_NEUMF) ? F : 0;  // tower output offset in predict input
    __host__ __device__ static constexpr int S(int k) { return (2 * DM) >> k; }
    __host__ __device__ static constexpr int MT(int k) { return (S(k + 1) + 15) / 16; }  // output 16-tiles
    __host__ __device__ static constexpr int KT(int k) { return S(k) / 16; }             // input 16-tiles
    __host__ __device__ static constexpr int SW(int k) { return S(k) + 4; }              // LDS stride of W_k
    __host__ __device__ static constexpr int SD(int k) { return 16 * MT(k) + 4; }        // staged dpre_k
    __host__ __device__ static constexpr int SH(int k) { return S(k) + 4; }              // staged H_k
    __host__ __device__ static constexpr int wsize(int k) { return MLP ? 16 * MT(k) * SW(k) : 0; }
    __host__ __device__ static constexpr int woff(int k) { return k == 0 ? 0 : woff(k - 1) + wsize(k - 1); }
    static constexpr int W_TOTAL = woff(L);
    // Per-wave LDS: only layer 0 is staged across waves (its wgrad needs every row
    // of the tile); layers k >= 1 accumulate their wgrad per wave in registers
    // (see ncf_train.hip), summed over the waves once, in the epilogue.  The
    // per-wave scratch of the layer-0 phase (item-side rows before the segment
    // walk): [16][DM + 4] MLP part, [16][F + 4] GMF part.
    static constexpr int ST0 = MLP ? 16 * SD(0) : 0;
    static constexpr int SCM = MLP ? DM + 4 : 0;
    static constexpr int SCG = GMF ? F + 4 : 0;
    static constexpr int SCR = 16 * (SCM + SCG);
    // Register accumulators of layers k >= 1: MT(k) x KT(k) 16x16 dW_k tiles and
    // MT(k) bias partials per lane; kt_off / mb_off index layer k's first one.
    __host__ __device__ static constexpr int nkt(int k) { return (MLP && k >= 1) ? MT(k) * KT(k) : 0; }
    __host__ __device__ static constexpr int kt_off(int k) { return k <= 1 ? 0 : kt_off(k - 1) + nkt(k - 1); }
    __host__ __device__ static constexpr int mb_off(int k) { return k <= 1 ? 0 : mb_off(k - 1) + MT(k - 1); }
    static constexpr int NKT = MLP ? kt_off(L) : 0;
    static constexpr int NMB = (MLP && L > 1) ? mb_off(L) : 0;
    // Epilogue: per-wave LDS image of layer k's partials ([S(k+1)][S(k)] + 4 bias
    // partials per output) and the entries of their sum over the waves per thread.
    __host__ __device__ static constexpr int rwk(int k) { return S(k + 1) * S(k) + 4 * S(k + 1); }
    __host__ __device__ static constexpr int nek(int k) {
        return (MLP && k >= 1) ? (S(k + 1) * S(k) + S(k + 1) + NTH - 1) / NTH : 0;
    }
    // su[2], si[2], labels[2] (double-buffered tile indices), zgmf, dz, teacher
    // logits[2] (10 floats per tile row), then 128 floats of biases (each layer's
    // padded to 16*MT) and 128 of predict weights
    static constexpr int MISC = 10 * TR + 256;
    // Two halves per wave whose roles (layer-0 staging / scatter scratch) alternate
    // with tile parity: the next tile's staging never overwrites rows a slow wave
    // still reads, so there is no tile-end barrier (if the LDS budget allows).
    static constexpr int HALF0 = ST0 > SCR ? ST0 : SCR;
    static constexpr bool ALT0_FITS = (W_TOTAL + MISC + NWV * 2 * HALF0) * 4 <= LDS_LIMIT_BYTES;
#ifdef NCF_KEEP_END_BARRIER  // experiment switch: one region + tile-end barrier
    static constexpr bool ALT0 = false;
#else
    static constexpr bool ALT0 = MLP && ALT0_FITS;
#endif
    static constexpr bool END_BARRIER = !ALT0;
    // OWN0 (small towers, dW0 at most 8 16x16 tiles): the per-row layer-0 wgrad from
    // each wave's own rows in registers, like layers k >= 1 (ncf_train.hip) -- no
    // cross-wave staging or barrier in the tile; its epilogue image needs rwk(0)
    static constexpr bool OWN0 = MLP && MT(0) * KT(0) <= 8;
    static constexpr int WAVE_STAGE_BASE = ALT0 ? 2 * HALF0 : ST0 + SCR;
    static constexpr int WAVE_STAGE = (OWN0 && rwk(0) > WAVE_STAGE_BASE) ? rwk(0) : WAVE_STAGE_BASE;
    static_assert(!MLP || L < 2 || rwk(1) <= WAVE_STAGE, "epilogue wgrad image exceeds the staging region");
    __host__ __device__ static constexpr int boff(int k) { return k == 0 ? 0 : boff(k - 1) + 16 * MT(k - 1); }
    static_assert(!MLP || boff(L) <= 128, "bias LDS region");
    static_assert(P <= 128, "predict LDS region");
    static constexpr int KT0 = MLP ? KT(0) : 1;
    // tower weights staged through registers by each thread in the prologue (16-byte
    // pieces): the narrow workgroup geometries are built where this stays <= 16
    __host__ __device__ static constexpr int wper(int k) { return MLP ? (16 * MT(k) * (S(k) / 4) + NTH - 1) / NTH : 0; }
    __host__ __device__ static constexpr int wreg_total(int k) { return k < 0 ? 0 : wper(k) + wreg_total(k - 1); }
    static constexpr int WREG = wreg_total(L - 1);
    // Layer-0 wgrad after the embedding scatter (its atomics drain under the wgrad
    // MFMAs) keeps the wgrad operands live through the dgrad: off where that
    // exceeds the register file (NeuMF f=64).
    static constexpr bool WGRAD0_LATE = !(MLP && GMF && F >= 64);
    static_assert(F >= 8 && F <= 64 && (F & (F - 1)) == 0, "factor_num must be 8..64, a power of 2");
    static_assert(L >= 1 && L <= 4, "num_layers must be 1..4");
};

// NCF_LAYOUT_ADAM_IN_STEP (ncf_train_step_ais): the previous step's dense Adam runs
// inside this launch -- its training workgroups apply it on the fly to every tower
// float and embedding row they read, its extra workgroups write it for every float --
// so a small-batch step is one launch.  State S_n (after update n) lives in buffer
// (n + st[1]) & 1; update n's gradient in g[n % 3], its tower partials in slab[n & 1].
struct AisArgs {
    float* p[2];
    float* m[2];
    float* v[2];
    float* g[3];
    float* slab[2];
    int64_t* st;  // device: [0] an update is pending at the chunk's first launch, [1] parity
    Ranges R, RE;  // active float4 ranges; their embedding part (below the tower)
    double lr, beta1, beta2;
    float eps;
    float* loss_hist;
    int64_t hist_len;
    ScCache* scc;
    int64_t step_i;  // this launch's index in its chunk (ncf_ais_bump closes the chunk)
    int ntrain;      // training workgroups; workgroups [ntrain, grid) run the dense update
    int lo, stride, rows;  // tower slab: first column, row stride, rows (the ntrain workgroups)
};

struct TrainArgs {
    ncf_layout lay;
    const float* params;
    float* grads;
    const uint64_t* rows;  // packed rows (NCF_ROW_PACK)
    const float* dlogit;   // NCF_DZ_DLOGIT: dL/dlogit per row (BCE: aliases rows, unused)
    ncf_step_ctl* ctl;
    int64_t batch_global;
    int world, rank, dz_mode;
    float kd_wt, kd_wr, kd_temp;  // NCF_DZ_KD: task / response weights, temperature (<= 0: logit MSE)
    float* slab;
    float* logits_out;
    int64_t fwd_n;  // FWD_ONLY: number of rows
    int diag;       // DIAG_* ablation switches (0 in production)
    unsigned long long* stamps;  // diagnostics: per-workgroup s_memtime stamps (nullptr in production)
    // NCF_LAYOUT_USER_STORE: the user-side embedding gradients of row k of the slice go
    // with plain stores to ustore[k * uw ...] ([Um part DM][Ug part F]) instead of float
    // atomics into grads; user_sum_kernel (ncf_ops.hip) sums them per user afterwards.
    float* ustore;
    int uw;
    AisArgs ais;  // ncf_step_kernel<..., AIS = true> only
};

constexpr int NSTAMP = 64;  // stamps per workgroup

// Ablation switches for performance diagnosis (ncf_debug_set_diag); results are
// wrong when any is set.
constexpr int DIAG_NO_WGRAD = 2;  // skip the weight-gradient MFMAs
constexpr int DIAG_NO_USER_SCATTER = 8;   // diag build only: skip the Um atomics
constexpr int DIAG_NO_ITEM_SCATTER = 16;  // diag build only: skip the Im segment atomics
constexpr int DIAG_NO_GMF_SCATTER = 32;   // diag build only: skip the Ug / Ig atomics
constexpr int DIAG_PREP_DIRECT = 4;  // ncf_prepare_epoch: global-atomic histogram variant (still correct)

// Launch geometries of the fused step (the NCF_LAYOUT_GEO field): GEO_8 = NWAVES-wave
// workgroups on 128-row tiles, GEO_4 / GEO_2 / GEO_1 = 4 / 2 / 1 waves on 64 / 32 /
// 16-row tiles for small per-rank batches.
enum { GEO_8 = 0, GEO_4 = 1, GEO_2 = 2, GEO_1 = 3, NGEO = 4 };
__host__ __device__ constexpr int geo_waves(int g) { return g == GEO_8 ? NWAVES : (8 >> g); }

struct KernelEntry {
    int mode, F, L;
    const void* train[NGEO];       // per geometry; nullptr where it has no instantiation
    const void* fwd;               // GEO_8
    const void* train_fact[NGEO];  // factored layer 0 (MLP shapes; see ncf_train.hip), else nullptr
    const void* train_ais[NGEO];   // the previous step's Adam inside the launch (per-row layer 0), else nullptr
    int w_total;                   // LDS floats
    int misc[NGEO], stage[NGEO];   // LDS floats per geometry
};

const KernelEntry* kernel_table(int* n);

}  // namespace ncf
