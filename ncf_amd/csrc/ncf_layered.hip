// Layered NeuMF step for every shape the fused kernel does not cover: tower
// weights too large for LDS (e.g. NCF(32,3): 172 KB; NCF(64,4): 2.8 MB) or a
// factor_num without an instantiation (the reference's factor sweeps use any f).
//
// Same arithmetic as NCF.forward / BCEWithLogitsLoss / loss.backward()
// (reference src/ncf/models.py:97-118, scripts/train_neumf.py:112-114), one
// layer at a time, activations staged in a caller-provided HBM workspace:
//
//   lyr_fwd<FIRST>        H_{k+1} = ReLU(A_k W_k^T + b_k)       A_0 gathered from Um/Im rows
//   lyr_predict<TRAIN>    logit = wp.[Ug*Ig || H_L] + bp; BCE; dz; GMF scatter;
//                         dY_{L-1} = dz * wp_mlp * [H_L > 0]; dwp, dbp, loss -> slab
//   lyr_bwd_w<FIRST>      dW_k += dY_k^T A_k,  db_k += colsum(dY_k)   (split over rows)
//   lyr_bwd_data<FIRST>   dY_{k-1} = (dY_k W_k) * [H_k > 0], or for k = 0 the
//                         Um/Im embedding scatter-add
//
// Factored layer 0 (train, tables of at most FACT_MAX_ROWS rows, ncf_ops.hip
// fact_mode): with W0 = [W0u | W0i] the layer-0 pre-activation of a row is
// Um[u] W0u^T + Im[i] W0i^T, so
//   lyr_proj              P = [Um W0u^T ; Im W0i^T]     (U + I rows, once per step)
//   lyr_fwd0_fact         H_1 = ReLU(P[u] + P[U + i] + b_0)   (a gather per row)
//   lyr_scatter0          dY_0 rows scatter-added into the user / item rows of the
//                         gradient buffer (item runs summed first), db_0
// and fact_expand_kernel (ncf_ops.hip) turns those per-row-sum rows into dUm, dIm
// and the dW0 partials -- three (U + I)-row GEMMs in place of three B-row ones.
//
// All three GEMM shapes run on one MFMA core: v_mfma_f32_16x16x4f32 (exact
// fp32), 256 threads = 4 waves, 64x64 block tile, each wave a 32x32 sub-tile
// (2x2 MFMA tiles), K in steps of 16 through double-buffered LDS.  Operand
// loaders map lanes along the operand's contiguous memory dimension.  Rows at
// or past the batch's end are padding: they gather id 0 and their dz is 0, so
// every gradient contribution from them is zero.
#include <cstring>

#include "ncf_common.h"
#include "ncf_layered.h"

namespace ncf {
namespace {

constexpr int GBM = 64, GBN = 64, GBK = 16, GNT = 256, GPAD = 4;

struct Sel {
    int64_t base, nloc;
    float gb;
};

// Rows of this launch: the fused kernel's selection (ncf_train.hip), i.e. global
// batch ctl->batch of the epoch stream, this rank's contiguous shard of it.
__device__ __forceinline__ Sel select_rows(const LyrArgs& a) {
    if (a.ctl == nullptr) return Sel{0, a.fwd_n, 1.f};
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
    return Sel{b0 + lo, hi - lo, (float)gb};
}

// Dropout of the input of tower layer k (training steps with lay.dropout > 0):
// element (epoch-stream row r, column c) is multiplied by 1 / (1 - p) when kept,
// else 0 (ncf_hip.h ncf_dropout_hash).  Off for forward-only launches (ctl null).
struct Drop {
    bool on;
    uint32_t seed, t, thr;
    float scale;
};
__device__ __forceinline__ Drop drop_of(const LyrArgs& a) {
    Drop d{false, 0, 0, 0, 1.f};
    if (a.ctl == nullptr || !(a.lay.dropout > 0.f)) return d;
    const float p = a.lay.dropout;
    d.on = true;
    d.seed = a.lay.dropout_seed;
    d.t = (uint32_t)a.ctl->adam_t;
    d.thr = p >= 1.f ? 0xffffffffu : (uint32_t)((double)p * 4294967296.0);
    d.scale = p >= 1.f ? 0.f : 1.0f / (1.0f - p);
    return d;
}
__device__ __forceinline__ float drop_mul(const Drop& d, int k, int64_t row, int c) {
    return dropout_hash(d.seed, d.t, (uint32_t)k, row, (uint32_t)c) >= d.thr ? d.scale : 0.f;
}

// This thread's grid-stride share of zeroing n4 16-byte units at p (the step's slab,
// cleared by its first kernel instead of a launch of its own).
__device__ __forceinline__ void zero_share(float* p, int64_t n4) {
    const int64_t nt = (int64_t)gridDim.x * gridDim.y * blockDim.x;
    const int64_t id = ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x;
    for (int64_t i = id; i < n4; i += nt) reinterpret_cast<f4*>(p)[i] = f4{0.f, 0.f, 0.f, 0.f};
}

// XCD-aware tile order for the 2-D GEMM grids (MI355X dispatches consecutive
// workgroups round-robin over its 8 XCDs, each with its own L2): the launch's
// workgroups, in dispatch order, are relabelled so that each group of workgroups
// sharing an XCD walks a contiguous run of (row tile, column tile) pairs, column tile
// fastest -- the column tiles of one row tile read the same A rows back to back from
// one L2 instead of from HBM once per tile.  A bijection (the guide's T1 form for
// grids not a multiple of 8), so a speed choice only.
__device__ __forceinline__ void xcd_tile(int& tm, int& tn) {
    const int64_t nwg = (int64_t)gridDim.x * gridDim.y;
    const int64_t orig = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
    const int64_t q = nwg / 8, r = nwg % 8, x = orig % 8;
    const int64_t w = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + orig / 8;
    tm = (int)(w / gridDim.y);
    tn = (int)(w % gridDim.y);
}

__device__ __forceinline__ void row_ids(const LyrArgs& a, const Sel& s, int64_t m, int& u, int& it) {
    if (m < s.nloc) {
        const uint64_t r = a.rows[s.base + m];
        u = (int)(uint32_t)r;
        it = (int)((r >> 32) & 0x7fffffffu);
        if (u < 0) it = -1;
    } else {
        u = it = -1;
    }
}

// Lane -> tile-element maps.  KC: the operand is contiguous along K (16 lanes
// per row, 4 passes of 16 rows); otherwise contiguous along M/N (64 lanes per
// k, 4 passes of 4 k).
template <bool KC>
__device__ __forceinline__ int map_mn(int t, int p) { return KC ? (t >> 4) + 16 * p : (t & 63); }
template <bool KC>
__device__ __forceinline__ int map_k(int t, int p) { return KC ? (t & 15) : (t >> 6) + 4 * p; }

// Store-time hook on the A operand (sa(value) once per loaded element, when it is
// written to LDS -- the load has landed by then, so no extra wait): the weight
// gradient sums dY's columns through it for db_k.
struct NoHook {
    template <class T>
    __device__ __forceinline__ void operator()(const T&) const {}
};

// C[mb..mb+32) x [nb..nb+32) for this wave: acc[ti][tj] reg r at
// row 16*ti + 4*(l>>4) + r, col 16*tj + (l&15).
template <bool AKC, bool BKC, class GA, class GB, class EP, class SA = NoHook>
__device__ __forceinline__ void gemm_block(int64_t m0, int64_t n0, int64_t kbeg, int64_t kend, GA ga, GB gb,
                                           EP ep, SA sa = SA{}) {
    __shared__ float As[2][GBK][GBM + GPAD];
    __shared__ float Bs[2][GBK][GBN + GPAD];
    const int t = threadIdx.x, l = t & 63, w = t >> 6;
    const int wm = (w >> 1) * 32, wn = (w & 1) * 32;
    float ra[4], rb[4];
    auto load = [&](int64_t k0) {
#pragma unroll
        for (int p = 0; p < 4; ++p) ra[p] = ga(map_mn<AKC>(t, p), k0 + map_k<AKC>(t, p));
#pragma unroll
        for (int p = 0; p < 4; ++p) rb[p] = gb(k0 + map_k<BKC>(t, p), map_mn<BKC>(t, p));
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int p = 0; p < 4; ++p) sa(ra[p]);
#pragma unroll
        for (int p = 0; p < 4; ++p) As[buf][map_k<AKC>(t, p)][map_mn<AKC>(t, p)] = ra[p];
#pragma unroll
        for (int p = 0; p < 4; ++p) Bs[buf][map_k<BKC>(t, p)][map_mn<BKC>(t, p)] = rb[p];
    };
    f4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    load(kbeg);
    store(0);
    __syncthreads();
    int buf = 0;
    for (int64_t k0 = kbeg; k0 < kend; k0 += GBK) {
        const bool more = k0 + GBK < kend;
        if (more) load(k0 + GBK);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int kk = 4 * s + (l >> 4);
            const float a0 = As[buf][kk][wm + (l & 15)], a1 = As[buf][kk][wm + 16 + (l & 15)];
            const float b0 = Bs[buf][kk][wn + (l & 15)], b1 = Bs[buf][kk][wn + 16 + (l & 15)];
            acc[0][0] = MFMA4(a0, b0, acc[0][0]);
            acc[0][1] = MFMA4(a0, b1, acc[0][1]);
            acc[1][0] = MFMA4(a1, b0, acc[1][0]);
            acc[1][1] = MFMA4(a1, b1, acc[1][1]);
        }
        if (more) store(buf ^ 1);
        __syncthreads();
        buf ^= 1;
    }
    (void)m0;
    (void)n0;
    ep(acc, wm, wn, l);
}

// Same tile and MFMA schedule with one 16-byte operand load per thread per K step:
// ga4 / gb4 return four elements along the operand's contiguous dimension (KC: K,
// else M/N), which must be a multiple of 4 with 16-byte aligned rows (factor_num
// % 4 == 0).  KC tile [64][16]: thread t loads row t / 4, k 4 (t % 4) .. + 3;
// otherwise [16][64]: k t / 16, columns 4 (t % 16) .. + 3 (one LDS f4 store).
template <bool AKC, bool BKC, class GA, class GB, class EP, class SA = NoHook>
__device__ __forceinline__ void gemm_block_v(int64_t kbeg, int64_t kend, GA ga4, GB gb4, EP ep, SA sa = SA{}) {
    __shared__ __attribute__((aligned(16))) float As[2][GBK][GBM + GPAD];
    __shared__ __attribute__((aligned(16))) float Bs[2][GBK][GBN + GPAD];
    const int t = threadIdx.x, l = t & 63, w = t >> 6;
    const int wm = (w >> 1) * 32, wn = (w & 1) * 32;
    const int a_mn = AKC ? (t >> 2) : 4 * (t & 15), a_k = AKC ? 4 * (t & 3) : (t >> 4);
    const int b_mn = BKC ? (t >> 2) : 4 * (t & 15), b_k = BKC ? 4 * (t & 3) : (t >> 4);
    f4 ra, rb;
    auto load = [&](int64_t k0) {
        ra = ga4(a_mn, k0 + a_k);
        rb = gb4(k0 + b_k, b_mn);
    };
    auto store = [&](int buf) {
        sa(ra);
        if constexpr (AKC) {
#pragma unroll
            for (int i = 0; i < 4; ++i) As[buf][a_k + i][a_mn] = lane_get(ra, i);
        } else {
            *reinterpret_cast<f4*>(&As[buf][a_k][a_mn]) = ra;
        }
        if constexpr (BKC) {
#pragma unroll
            for (int i = 0; i < 4; ++i) Bs[buf][b_k + i][b_mn] = lane_get(rb, i);
        } else {
            *reinterpret_cast<f4*>(&Bs[buf][b_k][b_mn]) = rb;
        }
    };
    f4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    load(kbeg);
    store(0);
    __syncthreads();
    int buf = 0;
    for (int64_t k0 = kbeg; k0 < kend; k0 += GBK) {
        const bool more = k0 + GBK < kend;
        if (more) load(k0 + GBK);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int kk = 4 * s + (l >> 4);
            const float a0 = As[buf][kk][wm + (l & 15)], a1 = As[buf][kk][wm + 16 + (l & 15)];
            const float b0 = Bs[buf][kk][wn + (l & 15)], b1 = Bs[buf][kk][wn + 16 + (l & 15)];
            acc[0][0] = MFMA4(a0, b0, acc[0][0]);
            acc[0][1] = MFMA4(a0, b1, acc[0][1]);
            acc[1][0] = MFMA4(a1, b0, acc[1][0]);
            acc[1][1] = MFMA4(a1, b1, acc[1][1]);
        }
        if (more) store(buf ^ 1);
        __syncthreads();
        buf ^= 1;
    }
    ep(acc, wm, wn, l);
}

// ---------------------------------------------------------------------------
// fp32 GEMM on the bf16 matrix cores (three-plane split, six products).
//
// gfx950 runs v_mfma_f32_16x16x4_f32 at 1/16 of the bf16 rate and has no xf32.
// Every fp32 operand element is split exactly into three bf16 planes by
// round-to-nearest, x = h + m + l (h = bf16(x), m = bf16(x - h), l = x - h - m; each
// remainder is exact in fp32 and the last fits bf16, so the sum is exact), and
//   x * y ~= h h' + (h m' + m h') + (h l' + m m' + l h')
// drops only m l', l m', l l': |m| <= 2^-8 |x|, |l| <= 2^-16 |x|, so each is
// <= 2^-24 |x y| and, the residuals being signed, unbiased -- about one fp32
// rounding per product (a truncating split leaves 8x larger, same-sign terms:
// max 4.7e-7 against 5.9e-8 relative over 2M random pairs).
// Accumulated in fp32 by v_mfma_f32_16x16x32_bf16 (exact bf16 x bf16 products).
// Per K = 32: 6 bf16 MFMAs of 16 cycles against 8 f32 MFMAs of 32.
//
// gemm_block_x6s keeps gemm_block_v's contract (64 x 64 block tile, 4 waves of 32 x 32,
// the same loaders, store hook and accumulator layout -- C/D of the bf16 16x16x32
// MFMA is the f32 16x16x4 map), with K in steps of 32 through double-buffered LDS.
typedef short bf16x8 __attribute__((ext_vector_type(8)));
constexpr int XBK = 32;

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float bitsf(uint32_t u) { return __builtin_bit_cast(float, u); }
// (a, b) -> packed bf16 pair, round to nearest even (v_cvt_pk_bf16_f32), a in the low half
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
    const f2_t v = {a, b};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}
// (x0, x1) -> three packed bf16 pairs (x0 in the low half): h, m, l with x = h + m + l
__device__ __forceinline__ void split3(float x0, float x1, uint32_t& h, uint32_t& m, uint32_t& l) {
    h = pk_bf16(x0, x1);
    const float r0 = x0 - bitsf(h << 16), r1 = x1 - bitsf(h & 0xffff0000u);
    m = pk_bf16(r0, r1);
    const float s0 = r0 - bitsf(m << 16), s1 = r1 - bitsf(m & 0xffff0000u);
    l = pk_bf16(s0, s1);
}

// B-operand loaders take (k, mn): adapt to the (mn, k) form above
template <class G>
struct X6Swap {
    G g;
    __device__ __forceinline__ f4 operator()(int mn, int64_t k) const { return g(k, mn); }
};

// The split happens in registers: the LDS holds the fp32 tiles ([mn][k], 32 k per row,
// 4-float chunks XOR-swizzled by (r ^ r >> 3) & 7: conflict-free ds_read_b128 operand
// reads and 16-byte stores, 2-way dword stores), 32 KB per block; each wave reads its
// fragments (two ds_read_b128 per 16-row tile) and splits them before its MFMAs.
__device__ __forceinline__ int x6s_addr(int r, int k) { return r * XBK + 4 * ((k >> 2) ^ ((r ^ (r >> 3)) & 7)) + (k & 3); }

template <bool KC, class G>
__device__ __forceinline__ void x6s_load(G g, int64_t k0, int t, f4 (&v)[2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int q = t + 256 * h;
        v[h] = KC ? g(q >> 3, k0 + 4 * (q & 7)) : g(4 * (q & 15), k0 + (q >> 4));
    }
}
template <bool KC>
__device__ __forceinline__ void x6s_store(float* S, int t, const f4 (&v)[2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int q = t + 256 * h;
        if constexpr (KC) {
            *reinterpret_cast<f4*>(S + x6s_addr(q >> 3, 4 * (q & 7))) = v[h];
        } else {
            const int k = q >> 4, mn = 4 * (q & 15);
#pragma unroll
            for (int i = 0; i < 4; ++i) S[x6s_addr(mn + i, k)] = lane_get(v[h], i);
        }
    }
}
// lane l's 8 k of row r (k 8 (l >> 4) .. + 7) -> the three bf16 planes of its fragment
__device__ __forceinline__ void x6s_frag(const float* S, int r, int l, bf16x8 (&f)[3]) {
    const int k = 8 * (l >> 4);
    const f4 x = *reinterpret_cast<const f4*>(S + x6s_addr(r, k));
    const f4 y = *reinterpret_cast<const f4*>(S + x6s_addr(r, k + 4));
    uint4 h, m, lo;
    split3(x.x, x.y, h.x, m.x, lo.x);
    split3(x.z, x.w, h.y, m.y, lo.y);
    split3(y.x, y.y, h.z, m.z, lo.z);
    split3(y.z, y.w, h.w, m.w, lo.w);
    f[0] = __builtin_bit_cast(bf16x8, h);
    f[1] = __builtin_bit_cast(bf16x8, m);
    f[2] = __builtin_bit_cast(bf16x8, lo);
}

template <bool AKC, bool BKC, class GA, class GB, class EP, class SA = NoHook>
__device__ __forceinline__ void gemm_block_x6s(int64_t kbeg, int64_t kend, GA ga4, GB gb4, EP ep, SA sa = SA{}) {
    __shared__ __attribute__((aligned(16))) float As[2][64 * XBK];
    __shared__ __attribute__((aligned(16))) float Bs[2][64 * XBK];
    const int t = threadIdx.x, l = t & 63, w = t >> 6;
    const int wm = (w >> 1) * 32, wn = (w & 1) * 32;
    const X6Swap<GB> gbs{gb4};
    f4 ra[2], rb[2];
    auto load = [&](int64_t k0) {
        x6s_load<AKC>(ga4, k0, t, ra);
        x6s_load<BKC>(gbs, k0, t, rb);
    };
    auto store = [&](int buf) {
        sa(ra[0]);
        sa(ra[1]);
        x6s_store<AKC>(As[buf], t, ra);
        x6s_store<BKC>(Bs[buf], t, rb);
    };
    f4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    load(kbeg);
    store(0);
    __syncthreads();
    int buf = 0;
    for (int64_t k0 = kbeg; k0 < kend; k0 += XBK) {
        const bool more = k0 + XBK < kend;
        if (more) load(k0 + XBK);
        bf16x8 fa[2][3], fb[2][3];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            x6s_frag(As[buf], wm + 16 * i + (l & 15), l, fa[i]);
            x6s_frag(Bs[buf], wn + 16 * i + (l & 15), l, fb[i]);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                f4 c = acc[i][j];
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][2], fb[j][0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], fb[j][1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[j][2], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], fb[j][0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[j][1], c, 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[j][0], c, 0, 0, 0);
            }
        if (more) store(buf ^ 1);
        __syncthreads();
        buf ^= 1;
    }
    ep(acc, wm, wn, l);
}

// gemm_block_x6w: the split core on a 128 x 128 block tile, each of the 4 waves a 64 x 64
// quadrant (4 x 4 MFMA tiles).  The x6s core's waves own 32 x 32 quadrants: per K step a
// wave splits 4 fragments (three bf16 planes each, ~40 VALU per fragment) for 24 MFMAs,
// and a wave64 VALU instruction occupies the SIMD 4 cycles -- ~960 VALU cycles against
// 384 MFMA cycles, so the split sets the time (SQ: 10 VALU per MFMA instruction in the
// weight-gradient launch, MFMA busy 0.21).  Here a wave splits 8 fragments for 96 MFMAs.
// Same planes, products, product order and K order per output element as x6s (the
// outputs are bitwise the same for the same K range).  LDS: 2 x (128 + 128) x 32 fp32
// = 64 KB, dynamic (X6W_LDS bytes; launchers set the attribute).  The epilogue gets
// acc[4][4] and the wave's quadrant origin (wm, wn) in {0, 64}.
constexpr int X6W_TB = 128;
constexpr int X6W_LDS = 2 * 2 * X6W_TB * XBK * 4;

template <bool KC, int TB, class G>
__device__ __forceinline__ void x6w_load(G g, int64_t k0, int t, f4 (&v)[TB / 32]) {
#pragma unroll
    for (int h = 0; h < TB / 32; ++h) {
        const int q = t + 256 * h;
        v[h] = KC ? g(q >> 3, k0 + 4 * (q & 7)) : g(4 * (q % (TB / 4)), k0 + q / (TB / 4));
    }
}
// (A register-transposed form for !KC -- four consecutive k rows per thread stored as f4
// along k -- removed the weight-gradient launch's 17M LDS bank-conflict cycles but ran
// 164.5 -> 194.8 us: profiles/r06_evidence/gemm_tile_ab/.)
template <bool KC, int TB>
__device__ __forceinline__ void x6w_store(float* S, int t, const f4 (&v)[TB / 32]) {
#pragma unroll
    for (int h = 0; h < TB / 32; ++h) {
        const int q = t + 256 * h;
        if constexpr (KC) {
            *reinterpret_cast<f4*>(S + x6s_addr(q >> 3, 4 * (q & 7))) = v[h];
        } else {
            const int k = q / (TB / 4), mn = 4 * (q % (TB / 4));
#pragma unroll
            for (int i = 0; i < 4; ++i) S[x6s_addr(mn + i, k)] = lane_get(v[h], i);
        }
    }
}

template <bool AKC, bool BKC, class GA, class GB, class EP, class SA = NoHook>
__device__ __forceinline__ void gemm_block_x6w(int64_t kbeg, int64_t kend, GA ga4, GB gb4, EP ep, SA sa = SA{}) {
    constexpr int TB = X6W_TB, NH = TB / 32;
    extern __shared__ __attribute__((aligned(16))) float x6w_sm[];
    float* As = x6w_sm;                  // [2][TB * XBK]
    float* Bs = x6w_sm + 2 * TB * XBK;   // [2][TB * XBK]
    const int t = threadIdx.x, l = t & 63, w = t >> 6;
    const int wm = (w >> 1) * 64, wn = (w & 1) * 64;
    const X6Swap<GB> gbs{gb4};
    f4 ra[NH], rb[NH];
    auto load = [&](int64_t k0) {
        x6w_load<AKC, TB>(ga4, k0, t, ra);
        x6w_load<BKC, TB>(gbs, k0, t, rb);
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int h = 0; h < NH; ++h) sa(ra[h]);
        x6w_store<AKC, TB>(As + buf * TB * XBK, t, ra);
        x6w_store<BKC, TB>(Bs + buf * TB * XBK, t, rb);
    };
    f4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    load(kbeg);
    store(0);
    __syncthreads();
    int buf = 0;
    for (int64_t k0 = kbeg; k0 < kend; k0 += XBK) {
        const bool more = k0 + XBK < kend;
        if (more) load(k0 + XBK);
        const float* Ab = As + buf * TB * XBK;
        const float* Bb = Bs + buf * TB * XBK;
        bf16x8 fa[4][3];
#pragma unroll
        for (int i = 0; i < 4; ++i) x6s_frag(Ab, wm + 16 * i + (l & 15), l, fa[i]);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            bf16x8 fb[3];
            x6s_frag(Bb, wn + 16 * j + (l & 15), l, fb);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                f4 c = acc[i][j];
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][2], fb[0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], fb[1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[2], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], fb[0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[1], c, 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[0], c, 0, 0, 0);
            }
        }
        if (more) store(buf ^ 1);
        __syncthreads();
        buf ^= 1;
    }
    ep(acc, wm, wn, l);
}

// gemm_block_x6b: the x6s core (64 x 64 block tile, 4 waves of 32 x 32) with the B
// operand already split: bimg is the block's first 16-column group of a fragment-major
// image (lyr_wc_prep_kernel's W0 images: per 16-column group ngs bytes, per K step of 32
// three planes x 64 lanes x 16 B), read straight from memory (L2-resident, 1.5 MB per
// image) one K step ahead.  Only A passes through LDS and the split, so a wave splits 2
// fragments per 24 MFMAs instead of 4 (the weight operand is split once per step instead
// of once per block).  Same planes, products and K order per element as x6s.
template <bool AKC, class GA, class EP>
__device__ __forceinline__ void gemm_block_x6b(int64_t kbeg, int64_t kend, GA ga4, const char* __restrict__ bimg,
                                               int64_t ngs, EP ep) {
    __shared__ __attribute__((aligned(16))) float As[2][64 * XBK];
    const int t = threadIdx.x, l = t & 63, w = t >> 6;
    const int wm = (w >> 1) * 32, wn = (w & 1) * 32;
    f4 ra[2];
    bf16x8 fb[2][3], fn[2][3];
    auto load_b = [&](int64_t k0, bf16x8 (&f)[2][3]) {
        const char* p = bimg + (k0 / XBK) * 3072 + l * 16;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 3; ++q)
                f[j][q] = *reinterpret_cast<const bf16x8*>(p + (int64_t)(wn / 16 + j) * ngs + q * 1024);
    };
    f4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    x6s_load<AKC>(ga4, kbeg, t, ra);
    load_b(kbeg, fb);
    x6s_store<AKC>(As[0], t, ra);
    __syncthreads();
    int buf = 0;
    for (int64_t k0 = kbeg; k0 < kend; k0 += XBK) {
        const bool more = k0 + XBK < kend;
        if (more) {
            x6s_load<AKC>(ga4, k0 + XBK, t, ra);
            load_b(k0 + XBK, fn);
        }
        bf16x8 fa[2][3];
#pragma unroll
        for (int i = 0; i < 2; ++i) x6s_frag(As[buf], wm + 16 * i + (l & 15), l, fa[i]);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                f4 c = acc[i][j];
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][2], fb[j][0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], fb[j][1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[j][2], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], fb[j][0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[j][1], c, 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[j][0], c, 0, 0, 0);
            }
        if (more) {
            x6s_store<AKC>(As[buf ^ 1], t, ra);
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int q = 0; q < 3; ++q) fb[j][q] = fn[j][q];
        }
        __syncthreads();
        buf ^= 1;
    }
    ep(acc, wm, wn, l);
}

// The GEMM core of the layered kernels' 16-byte loader path: the bf16 split core, or
// (-DNCF_GEMM_F32, the A/B library variant) the f32-MFMA core.  (A variant that split
// once per block into three bf16 plane images in LDS -- 48 KB per block, 3 blocks per
// CU -- measured slower: stress 1304 against 1093 us per step.)
template <bool AKC, bool BKC, class GA, class GB, class EP, class SA = NoHook>
__device__ __forceinline__ void gemm_block_vx(int64_t kbeg, int64_t kend, GA ga4, GB gb4, EP ep, SA sa = SA{}) {
#if defined(NCF_GEMM_F32)
    gemm_block_v<AKC, BKC>(kbeg, kend, ga4, gb4, ep, sa);
#else
    gemm_block_x6s<AKC, BKC>(kbeg, kend, ga4, gb4, ep, sa);
#endif
}

// TB = 64: gemm_block_vx; TB = X6W_TB: the 128 x 128 split core (dynamic LDS X6W_LDS)
template <int TB, bool AKC, bool BKC, class GA, class GB, class EP, class SA = NoHook>
__device__ __forceinline__ void gemm_tile(int64_t kbeg, int64_t kend, GA ga4, GB gb4, EP ep, SA sa = SA{}) {
    static_assert(TB == 64 || TB == X6W_TB, "block tile");
    if constexpr (TB == X6W_TB)
        gemm_block_x6w<AKC, BKC>(kbeg, kend, ga4, gb4, ep, sa);
    else
        gemm_block_vx<AKC, BKC>(kbeg, kend, ga4, gb4, ep, sa);
}

__device__ __forceinline__ f4 ld4(const float* p) { return *reinterpret_cast<const f4*>(p); }
__device__ __forceinline__ f4 zero4() { return f4{0.f, 0.f, 0.f, 0.f}; }

// ---------------------------------------------------------------------------
// Forward layer k: H_{k+1}[m][n] = ReLU(sum_c A[m][c] W_k[n][c] + b_k[n]).
// grid (ceil(R/64), ceil(N/64)).
template <bool FIRST, bool DROP, bool VEC>
__global__ __launch_bounds__(GNT) void lyr_fwd_kernel(LyrArgs a, int k, const float* __restrict__ Ain,
                                                      float* __restrict__ Hout, int64_t R) {
    __shared__ int su[GBM], si[GBM];
    const Sel s = select_rows(a);
    const ncf_layout& lay = a.lay;
    const int DM = lay.factor_num << (lay.num_layers - 1);
    const int K = (2 * DM) >> k, N = K / 2;
    int tm, tn;
    xcd_tile(tm, tn);
    const int64_t m0 = (int64_t)tm * GBM;
    const int n0 = tn * GBN;
    const float* prm = a.params;
    const float* W = prm + lay.w[k];
    const float* bias = prm + lay.b[k];
    if (FIRST && a.zero_p != nullptr) zero_share(a.zero_p, a.zero_n4);  // the step's first kernel
    if (FIRST && threadIdx.x < GBM) {
        int u, it;
        row_ids(a, s, m0 + threadIdx.x, u, it);
        su[threadIdx.x] = u < 0 ? 0 : u;
        si[threadIdx.x] = it < 0 ? 0 : it;
    }
    if (FIRST) __syncthreads();
    const Drop dr = DROP ? drop_of(a) : Drop{false, 0, 0, 0, 1.f};
    auto ga = [&](int r, int64_t c) -> float {
        const int64_t m = m0 + r;
        if (m >= R || c >= K) return 0.f;
        float v;
        if constexpr (FIRST) {
            v = c < DM ? prm[lay.um + (int64_t)su[r] * DM + c] : prm[lay.im + (int64_t)si[r] * DM + (c - DM)];
        } else {
            v = Ain[m * K + c];
        }
        if constexpr (DROP) v *= drop_mul(dr, k, s.base + m, (int)c);
        return v;
    };
    auto gb = [&](int64_t c, int n) -> float {
        const int nn = n0 + n;
        return (nn < N && c < K) ? W[(int64_t)nn * K + c] : 0.f;
    };
    auto ep = [&](f4 (&acc)[2][2], int wm, int wn, int l) {
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
            for (int tj = 0; tj < 2; ++tj) {
                const int n = n0 + wn + 16 * tj + (l & 15);
                if (n >= N) continue;
                const float bn = bias[n];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int64_t m = m0 + wm + 16 * ti + 4 * (l >> 4) + r;
                    if (m < R) Hout[m * N + n] = fmaxf(lane_get(acc[ti][tj], r) + bn, 0.f);
                }
            }
    };
    if constexpr (VEC) {
        auto ga4 = [&](int r, int64_t c) -> f4 {
            const int64_t m = m0 + r;
            if (m >= R || c >= K) return zero4();
            f4 v;
            if constexpr (FIRST) {
                v = c < DM ? ld4(prm + lay.um + (int64_t)su[r] * DM + c) : ld4(prm + lay.im + (int64_t)si[r] * DM + (c - DM));
            } else {
                v = ld4(Ain + m * K + c);
            }
            if constexpr (DROP) {
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] *= drop_mul(dr, k, s.base + m, (int)c + i);
            }
            return v;
        };
        auto gb4 = [&](int64_t c, int n) -> f4 {
            const int nn = n0 + n;
            return (nn < N && c < K) ? ld4(W + (int64_t)nn * K + c) : zero4();
        };
        gemm_block_vx<true, true>(0, K, ga4, gb4, ep);
    } else {
        gemm_block<true, true>(m0, n0, 0, K, ga, gb, ep);
    }
}

// ---------------------------------------------------------------------------
// Backward data of layer k: C[m][n] = sum_j dY_k[m][j] W_k[j][n]   (n < s_k).
//   k > 0: dY_{k-1}[m][n] = C * [H_k[m][n] > 0]
//   k = 0: scatter-add C into grad Um[u_m] (n < dm) / Im[i_m] (n >= dm)
// grid (ceil(R/64), ceil(s_k/64)).
template <bool FIRST, bool DROP, bool VEC>
__global__ __launch_bounds__(GNT) void lyr_bwd_data_kernel(LyrArgs a, int k, const float* __restrict__ D,
                                                           const float* __restrict__ Hk, float* __restrict__ Dout,
                                                           int64_t R) {
    __shared__ int su[GBM], si[GBM];
    const Sel s = select_rows(a);
    const ncf_layout& lay = a.lay;
    const int DM = lay.factor_num << (lay.num_layers - 1);
    const int N = (2 * DM) >> k, J = N / 2;  // this layer: in = N, out = J
    int tm, tn;
    xcd_tile(tm, tn);
    const int64_t m0 = (int64_t)tm * GBM;
    const int n0 = tn * GBN;
    const float* W = a.params + lay.w[k];
    if (FIRST && threadIdx.x < GBM) {
        int u, it;
        row_ids(a, s, m0 + threadIdx.x, u, it);
        su[threadIdx.x] = u;
        si[threadIdx.x] = it;
    }
    if (FIRST) __syncthreads();
    const Drop dr = DROP ? drop_of(a) : Drop{false, 0, 0, 0, 1.f};
    auto ga = [&](int r, int64_t j) -> float {
        const int64_t m = m0 + r;
        return (m < R && j < J) ? D[m * J + j] : 0.f;
    };
    auto gb = [&](int64_t j, int n) -> float {
        const int nn = n0 + n;
        return (j < J && nn < N) ? W[j * N + nn] : 0.f;
    };
    auto ep = [&](f4 (&acc)[2][2], int wm, int wn, int l) {
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
            for (int tj = 0; tj < 2; ++tj) {
                const int n = n0 + wn + 16 * tj + (l & 15);
                if (n >= N) continue;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int rr = wm + 16 * ti + 4 * (l >> 4) + r;
                    const int64_t m = m0 + rr;
                    if (m >= R) continue;
                    float v = lane_get(acc[ti][tj], r);
                    if constexpr (DROP) v *= drop_mul(dr, k, s.base + m, n);  // through layer k's input dropout
                    if constexpr (FIRST) {
                        const int id = n < DM ? su[rr] : si[rr];
                        if (id >= 0)
                            atomicAdd(a.grads + (n < DM ? lay.um + (int64_t)id * DM + n
                                                        : lay.im + (int64_t)id * DM + (n - DM)),
                                      v);
                    } else {
                        Dout[m * N + n] = Hk[m * N + n] > 0.f ? v : 0.f;
                    }
                }
            }
    };
    if constexpr (VEC) {
        auto ga4 = [&](int r, int64_t j) -> f4 {
            const int64_t m = m0 + r;
            return (m < R && j < J) ? ld4(D + m * J + j) : zero4();
        };
        auto gb4 = [&](int64_t j, int n) -> f4 {
            const int nn = n0 + n;
            return (j < J && nn < N) ? ld4(W + j * N + nn) : zero4();
        };
        // K = J <= 256 here (2-8 K steps of 32): the masked epilogue dominates and the
        // f32 core's occupancy (8 waves / SIMD against 3) wins -- stress 88.8 against
        // 95.4 us per launch with the split core (profiles/r03x6/stress_kernel_stats_*.csv)
        gemm_block_v<true, false>(0, J, ga4, gb4, ep);
    } else {
        gemm_block<true, false>(m0, n0, 0, J, ga, gb, ep);
    }
}

// ---------------------------------------------------------------------------
// Backward weight of layer k over the row chunk of blockIdx.z:
//   dW_k[j][c] += sum_m dY_k[m][j] A_k[m][c]   (c < s_k)
//   db_k[j]    += sum_m dY_k[m][j]             (the extra column c = s_k of ones)
// into the slab (tower partials, reduced by ncf_reduce_slab).
// grid (ceil(J/64), ceil((s_k+1)/64), splits).
template <bool FIRST, bool DROP, bool VEC, int TB = 64>
__device__ __forceinline__ void bwd_w_body(const LyrArgs& a, int k, const float* __restrict__ D,
                                           const float* __restrict__ Ain, int64_t R, int64_t chunk, int bx, int by,
                                           int bz) {
    static_assert(TB == 64 || (VEC && !FIRST), "the 128-tile core: 16-byte loaders, layers k >= 1");
    constexpr int NT = TB / 32;
    __shared__ int su[FIRST ? GBK * 64 : 1], si[FIRST ? GBK * 64 : 1];  // ids of up to 1024 rows of the chunk (FIRST)
    const Sel s = select_rows(a);
    const ncf_layout& lay = a.lay;
    const int DM = lay.factor_num << (lay.num_layers - 1);
    const int K = (2 * DM) >> k, J = K / 2;
    const int j0 = bx * TB;
    const int c0 = by * TB;
    const int64_t r0 = (int64_t)bz * chunk;
    int64_t r1 = r0 + chunk;
    if (r1 > R) r1 = R;
    if (r1 > s.nloc) r1 = s.nloc;  // padding rows carry dY = 0
    if (r0 >= r1) return;          // block-uniform
    const float* prm = a.params;
    float* slab = a.slab + (int64_t)(bz % lyr_slab_rows(&lay)) * (lay.tower_len + 64);
    const int64_t tb = lay.tower_begin;
    const Drop dr = DROP ? drop_of(a) : Drop{false, 0, 0, 0, 1.f};
    // db_k = column sums of dY_k: summed by the blocks of column tile 0 from the dY
    // values they stage anyway (store-time hook of the GEMM core), instead of a ones
    // column appended to A, which costs a whole extra 64-wide tile when K % 64 == 0
    const bool dbt = by == 0;  // block-uniform
    f4 db4 = zero4();
    float db1 = 0.f;
    auto sa4 = [&](const f4& v) {
        if (dbt) {
            db4.x += v.x;
            db4.y += v.y;
            db4.z += v.z;
            db4.w += v.w;
        }
    };
    auto sa1 = [&](const float& v) {
        if (dbt) db1 += v;
    };
    auto ep = [&](f4 (&acc)[NT][NT], int wm, int wn, int l) {
#pragma unroll
        for (int ti = 0; ti < NT; ++ti)
#pragma unroll
            for (int tj = 0; tj < NT; ++tj) {
                const int c = c0 + wn + 16 * tj + (l & 15);
                if (c >= K) continue;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int j = j0 + wm + 16 * ti + 4 * (l >> 4) + r;
                    if (j >= J) continue;
                    atomicAdd(slab + (lay.w[k] - tb) + (int64_t)j * K + c, lane_get(acc[ti][tj], r));
                }
            }
    };
    auto ga = [&](int jr, int64_t m) -> float {
        const int j = j0 + jr;
        return (m < r1 && j < J) ? D[m * J + j] : 0.f;
    };
    if constexpr (FIRST) {
        // rows processed in sub-chunks of 1024 with their ids staged in LDS
        for (int64_t q0 = r0; q0 < r1; q0 += GBK * 64) {
            const int64_t q1 = q0 + GBK * 64 < r1 ? q0 + GBK * 64 : r1;
            __syncthreads();
            for (int e = threadIdx.x; e < GBK * 64; e += GNT) {
                int u, it;
                row_ids(a, s, q0 + e, u, it);
                su[e] = u < 0 ? 0 : u;
                si[e] = it < 0 ? 0 : it;
            }
            __syncthreads();
            auto gb = [&](int64_t m, int cr) -> float {
                const int c = c0 + cr;
                if (m >= q1 || c >= K) return 0.f;
                const int e = (int)(m - q0);
                float v = c < DM ? prm[lay.um + (int64_t)su[e] * DM + c] : prm[lay.im + (int64_t)si[e] * DM + (c - DM)];
                if constexpr (DROP) v *= drop_mul(dr, k, s.base + m, c);
                return v;
            };
            auto ga2 = [&](int jr, int64_t m) -> float {
                const int j = j0 + jr;
                return (m < q1 && j < J) ? D[m * J + j] : 0.f;
            };
            if constexpr (VEC) {
                auto ga4 = [&](int jr, int64_t m) -> f4 {
                    const int j = j0 + jr;
                    return (m < q1 && j < J) ? ld4(D + m * J + j) : zero4();
                };
                auto gb4 = [&](int64_t m, int cr) -> f4 {
                    const int c = c0 + cr;
                    if (m >= q1 || c >= K) return zero4();
                    const int e = (int)(m - q0);
                    f4 v = c < DM ? ld4(prm + lay.um + (int64_t)su[e] * DM + c)
                                  : ld4(prm + lay.im + (int64_t)si[e] * DM + (c - DM));
                    if constexpr (DROP) {
#pragma unroll
                        for (int i = 0; i < 4; ++i) v[i] *= drop_mul(dr, k, s.base + m, c + i);
                    }
                    return v;
                };
                gemm_block_vx<false, false>(q0, q1, ga4, gb4, ep, sa4);
            } else {
                gemm_block<false, false>(j0, c0, q0, q1, ga2, gb, ep, sa1);
            }
        }
    } else {
        auto gb = [&](int64_t m, int cr) -> float {
            const int c = c0 + cr;
            if (m >= r1 || c >= K) return 0.f;
            float v = Ain[m * K + c];
            if constexpr (DROP) v *= drop_mul(dr, k, s.base + m, c);
            return v;
        };
        if constexpr (VEC) {
            auto ga4 = [&](int jr, int64_t m) -> f4 {
                const int j = j0 + jr;
                return (m < r1 && j < J) ? ld4(D + m * J + j) : zero4();
            };
            auto gb4 = [&](int64_t m, int cr) -> f4 {
                const int c = c0 + cr;
                if (m >= r1 || c >= K) return zero4();
                f4 v = ld4(Ain + m * K + c);
                if constexpr (DROP) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) v[i] *= drop_mul(dr, k, s.base + m, c + i);
                }
                return v;
            };
            gemm_tile<TB, false, false>(r0, r1, ga4, gb4, ep, sa4);
        } else {
            if constexpr (TB == 64) gemm_block<false, false>(j0, c0, r0, r1, ga, gb, ep, sa1);
        }
    }
    if (dbt) {  // db_k: per-thread column sums -> LDS -> one atomic per column per block
        // A operand [TB / 4 rows of m][TB j] per load: VEC thread t holds j 4 (t % (TB / 4))
        // .. + 3 (TB = 64: 16 slots, 128: 8); scalar thread t holds j t % 64 of rows t / 64
        constexpr int NS = VEC ? 256 / (TB / 4) : 4;
        __shared__ float dred[NS][TB];
        const int t = threadIdx.x;
        if constexpr (VEC) {
#pragma unroll
            for (int i = 0; i < 4; ++i) dred[t / (TB / 4)][4 * (t % (TB / 4)) + i] = lane_get(db4, i);
        } else {
            dred[t >> 6][t & 63] = db1;
        }
        __syncthreads();
        if (t < TB) {
            float sum = 0.f;
#pragma unroll
            for (int q = 0; q < NS; ++q) sum += dred[q][t];
            const int j = j0 + t;
            if (j < J && sum != 0.f) atomicAdd(slab + (lay.b[k] - tb) + j, sum);
        }
    }
}

template <bool FIRST, bool DROP, bool VEC>
__global__ __launch_bounds__(GNT) void lyr_bwd_w_kernel(LyrArgs a, int k, const float* __restrict__ D,
                                                        const float* __restrict__ Ain, int64_t R, int64_t chunk) {
    // XCD-aware order (xcd_tile): the (j, column) tiles of one row chunk share an XCD,
    // so its D and A rows are read from one L2
    const int64_t per = (int64_t)gridDim.x * gridDim.y, nwg = per * gridDim.z;
    const int64_t orig = ((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    const int64_t q = nwg / 8, r = nwg % 8, x = orig % 8;
    const int64_t w = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + orig / 8;
    const int bz = (int)(w / per), rem = (int)(w % per);
    bwd_w_body<FIRST, DROP, VEC>(a, k, D, Ain, R, chunk, rem % gridDim.x, rem / gridDim.x, bz);
}

// The weight gradients of several layers k >= 1 in one launch (the step chain leaves
// every D_k and H_k in the workspace at once): a 1-D grid, layer i owning blocks
// [start[i], start[i + 1]), each decoded to the (j tile, column tile, row chunk) of
// lyr_bwd_w_kernel's 3-D grid.  The layers' GEMMs are small (NCF(32,3): 64 x 128 and
// 32 x 64 outputs over 65,536 rows): two launches paid the launch ramp and the drain
// of the split atomics twice.
// With the user order, blocks past the layers' run the user-order walk of D_0
// (user_walk_body with 256-thread blocks), which is independent of them.
struct BwMulti {
    int n;
    int k[3], gx[3], gy[3];
    const float* D[3];
    const float* A[3];
    int64_t chunk[3];
    int start[4];
    const float* D0u;  // user-order D_0 (nullptr: no walk blocks)
    int walk_dm;
};
__device__ __forceinline__ void user_walk_body(const LyrArgs& a, const float* __restrict__ D0u, int64_t blk,
                                               int nt, int dm);
template <int TB>
__global__ __launch_bounds__(GNT) void lyr_bwd_w_multi_kernel(LyrArgs a, BwMulti m, int64_t R) {
    const int b = blockIdx.x;
    if (b >= m.start[m.n]) {  // block-uniform
        user_walk_body(a, m.D0u, b - m.start[m.n], GNT, m.walk_dm);
        return;
    }
    int i = 0;
#pragma unroll
    for (int q = 1; q < 3; ++q)
        if (q < m.n && b >= m.start[q]) i = q;
    const int loc = b - m.start[i], per = m.gx[i] * m.gy[i];
    const int bz = loc / per, rem = loc - bz * per;
    bwd_w_body<false, false, true, TB>(a, m.k[i], m.D[i], m.A[i], R, m.chunk[i], rem % m.gx[i], rem / m.gx[i], bz);
}

// ---------------------------------------------------------------------------
// Factored layer 0.  Projection: P[r][n] = sum_c X[r][c] W0[n][koff + c] over the
// user rows (blocks [0, nbu), X = Um, koff = 0) then the item rows (X = Im,
// koff = DM); grid (nbu + nbi, ceil(DM / 64)).  The GEMM core shares each W0 tile
// through LDS over 64 rows (an LDS-free wave-per-16-rows variant re-read the 64 KB
// W0 half per wave at dm 128: 15.5 against 9.4 us).  It is the step's first kernel
// and also clears the slab (zp, zn4).
// BPRE: W0 comes pre-split (bimg: the users' image, the items' one W0 image later;
// lyr_wc_prep_kernel) through gemm_block_x6b
template <int TB, bool BPRE = false>
__global__ __launch_bounds__(GNT) void lyr_proj_kernel(ncf_layout lay, const float* __restrict__ prm,
                                                       float* __restrict__ P, int nbu, float* __restrict__ zp,
                                                       int64_t zn4, const char* __restrict__ bimg = nullptr) {
    if (zp != nullptr) zero_share(zp, zn4);
    constexpr int NT = TB / 32;  // 16 x 16 tiles per wave side
    const int DM = lay.factor_num << (lay.num_layers - 1);
    const bool user = (int)blockIdx.x < nbu;
    const int64_t nrows = user ? lay.user_num : lay.item_num;
    const int64_t m0 = (int64_t)(user ? blockIdx.x : blockIdx.x - nbu) * TB;
    const int n0 = blockIdx.y * TB;
    const float* X = prm + (user ? lay.um : lay.im);
    const float* W = prm + lay.w[0] + (user ? 0 : DM);  // row stride 2 DM
    float* Pout = P + (user ? 0 : (int64_t)lay.user_num * DM);
    auto ep = [&](f4 (&acc)[NT][NT], int wm, int wn, int l) {
#pragma unroll
        for (int ti = 0; ti < NT; ++ti)
#pragma unroll
            for (int tj = 0; tj < NT; ++tj) {
                const int n = n0 + wn + 16 * tj + (l & 15);
                if (n >= DM) continue;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int64_t m = m0 + wm + 16 * ti + 4 * (l >> 4) + r;
                    if (m < nrows) Pout[m * DM + n] = lane_get(acc[ti][tj], r);
                }
            }
    };
    auto ga4 = [&](int r, int64_t c) -> f4 {
        const int64_t m = m0 + r;
        return (m < nrows && c < DM) ? ld4(X + m * DM + c) : zero4();
    };
    auto gb4 = [&](int64_t c, int n) -> f4 {
        const int nn = n0 + n;
        return (nn < DM && c < DM) ? ld4(W + (int64_t)nn * 2 * DM + c) : zero4();
    };
    if constexpr (BPRE) {
        static_assert(TB == 64, "pre-split B: the 64 x 64 core");
        const int64_t ngs = (int64_t)(DM / 32) * 3072, img = (int64_t)(DM / 16) * ngs;
        gemm_block_x6b<true>(0, DM, ga4, bimg + (user ? 0 : img) + (int64_t)(n0 / 16) * ngs, ngs, ep);
    } else {
        gemm_tile<TB, true, true>(0, DM, ga4, gb4, ep);  // factored path: dm in {8, ..., 512}
    }
}

// H_1[m][n] = ReLU(P[u_m][n] + P[U + i_m][n] + b_0[n]), four outputs per thread
// (padding rows gather id 0, as lyr_fwd_kernel<true>).
// Factored layer 0 with dm > 128 (NCF(64,4): dm 512), too wide for
// fact_expand_kernel's LDS-staged W0 half (1 MB): the expansion as GEMMs on the core.
// G = the D_0 row sums the scatter left in a table's gradient rows.
//   lyr_fact_dx_kernel   dX = G W0[:, koff : koff + DM] per table into the projection
//                        buffer (dead after the forward; copied over G afterwards);
//                        grid (nbu + nbi, ceil(DM / 64)) like lyr_proj_kernel
//   lyr_fact_dw0_kernel  dW0[:, koff + c] += G^T X over row chunks of each table
//                        (z < zu: users), into the slab's W0 columns (no partials at
//                        dm > 128: the reductions read W0 from the slab)
template <int TB, bool BPRE = false>
__global__ __launch_bounds__(GNT) void lyr_fact_dx_kernel(ncf_layout lay, const float* __restrict__ prm,
                                                          const float* __restrict__ grads, float* __restrict__ out,
                                                          int nbu, const char* __restrict__ bimg = nullptr) {
    constexpr int NT = TB / 32;
    const int DM = lay.factor_num << (lay.num_layers - 1);
    const bool user = (int)blockIdx.x < nbu;
    const int64_t nrows = user ? lay.user_num : lay.item_num;
    const int64_t m0 = (int64_t)(user ? blockIdx.x : blockIdx.x - nbu) * TB;
    const int n0 = blockIdx.y * TB;
    const float* G = grads + (user ? lay.um : lay.im);
    const float* W = prm + lay.w[0] + (user ? 0 : DM);  // W0[o][koff + i], row stride 2 DM
    float* O = out + (user ? 0 : (int64_t)lay.user_num * DM);
    auto ep = [&](f4 (&acc)[NT][NT], int wm, int wn, int l) {
#pragma unroll
        for (int ti = 0; ti < NT; ++ti)
#pragma unroll
            for (int tj = 0; tj < NT; ++tj) {
                const int n = n0 + wn + 16 * tj + (l & 15);
                if (n >= DM) continue;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int64_t m = m0 + wm + 16 * ti + 4 * (l >> 4) + r;
                    if (m < nrows) O[m * DM + n] = lane_get(acc[ti][tj], r);
                }
            }
    };
    auto ga4 = [&](int r, int64_t k) -> f4 {  // G[m][o..o+3]
        const int64_t m = m0 + r;
        return (m < nrows && k < DM) ? ld4(G + m * DM + k) : zero4();
    };
    auto gb4 = [&](int64_t k, int n) -> f4 {  // W0[o][koff + i .. + 3]
        const int nn = n0 + n;
        return (k < DM && nn < DM) ? ld4(W + k * 2 * DM + nn) : zero4();
    };
    if constexpr (BPRE) {
        static_assert(TB == 64, "pre-split B: the 64 x 64 core");
        const int64_t ngs = (int64_t)(DM / 32) * 3072, img = (int64_t)(DM / 16) * ngs;
        gemm_block_x6b<true>(0, DM, ga4, bimg + (user ? 0 : img) + (int64_t)(n0 / 16) * ngs, ngs, ep);
    } else {
        gemm_tile<TB, true, false>(0, DM, ga4, gb4, ep);
    }
}

template <int TB>
__global__ __launch_bounds__(GNT) void lyr_fact_dw0_kernel(LyrArgs a, int zu, int64_t chunk) {
    constexpr int NT = TB / 32;
    const ncf_layout& lay = a.lay;
    const int DM = lay.factor_num << (lay.num_layers - 1);
    const bool user = (int)blockIdx.z < zu;
    const int64_t nrows = user ? lay.user_num : lay.item_num;
    const int64_t r0 = (int64_t)(user ? blockIdx.z : blockIdx.z - zu) * chunk;
    const int64_t r1 = r0 + chunk < nrows ? r0 + chunk : nrows;
    if (r0 >= r1) return;  // block-uniform
    const int o0 = blockIdx.x * TB, c0 = blockIdx.y * TB;
    const float* G = a.grads + (user ? lay.um : lay.im);
    const float* X = a.params + (user ? lay.um : lay.im);
    const int koff = user ? 0 : DM;
    float* slab = a.slab + (int64_t)(blockIdx.z % lyr_slab_rows(&lay)) * (lay.tower_len + 64) +
                  (lay.w[0] - lay.tower_begin);
    auto ep = [&](f4 (&acc)[NT][NT], int wm, int wn, int l) {
#pragma unroll
        for (int ti = 0; ti < NT; ++ti)
#pragma unroll
            for (int tj = 0; tj < NT; ++tj) {
                const int c = c0 + wn + 16 * tj + (l & 15);
                if (c >= DM) continue;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int o = o0 + wm + 16 * ti + 4 * (l >> 4) + r;
                    if (o < DM) atomicAdd(slab + (int64_t)o * 2 * DM + koff + c, lane_get(acc[ti][tj], r));
                }
            }
    };
    auto ga4 = [&](int jr, int64_t m) -> f4 {  // G[m][o .. o + 3]
        const int o = o0 + jr;
        return (m < r1 && o < DM) ? ld4(G + m * DM + o) : zero4();
    };
    auto gb4 = [&](int64_t m, int cr) -> f4 {  // X[m][c .. c + 3]
        const int c = c0 + cr;
        return (m < r1 && c < DM) ? ld4(X + m * DM + c) : zero4();
    };
    gemm_tile<TB, false, false>(r0, r1, ga4, gb4, ep);
}

__global__ __launch_bounds__(GNT) void lyr_fwd0_fact_kernel(LyrArgs a, const float* __restrict__ P,
                                                            float* __restrict__ H1, int64_t R) {
    const Sel s = select_rows(a);
    const ncf_layout& lay = a.lay;
    const int DM = lay.factor_num << (lay.num_layers - 1);
    const int q4 = DM / 4;
    const float* b0 = a.params + lay.b[0];
    const float* Pi = P + (int64_t)lay.user_num * DM;
    for (int64_t e = (int64_t)blockIdx.x * GNT + threadIdx.x; e < R * q4; e += (int64_t)gridDim.x * GNT) {
        const int64_t m = e / q4;
        const int n = 4 * (int)(e - m * q4);
        int u, it;
        row_ids(a, s, m, u, it);
        u = u < 0 ? 0 : u;
        it = it < 0 ? 0 : it;
        const f4 pu = *reinterpret_cast<const f4*>(P + (int64_t)u * DM + n);
        const f4 pi = *reinterpret_cast<const f4*>(Pi + (int64_t)it * DM + n);
        const f4 bb = *reinterpret_cast<const f4*>(b0 + n);
        f4 h;
        h.x = fmaxf(pu.x + pi.x + bb.x, 0.f);
        h.y = fmaxf(pu.y + pi.y + bb.y, 0.f);
        h.z = fmaxf(pu.z + pi.z + bb.z, 0.f);
        h.w = fmaxf(pu.w + pi.w + bb.w, 0.f);
        *reinterpret_cast<f4*>(H1 + m * DM + n) = h;
    }
}

// Factored step chain (training, every tower width a multiple of 4): a tile's rows
// are independent through the whole forward and data-gradient chain, so one launch
// does, for 64-row tiles (4 waves x 16 rows), everything but the weight gradients:
//   H_1 = ReLU(P[u] + P[U + i] + b_0), H_{k+1} = ReLU(W_k H_k + b_k)   (k = 1 .. L-1)
//   logit, BCE / KD / given dL/dlogit, the GMF backward (user rows per row, item runs
//   summed first: batches are grouped by item), dwp / dbp / loss
//   D_{L-1} = dz wp_mlp [H_L > 0],  D_{k-1} = (D_k W_k) [H_k > 0]   (k = L-1 .. 1)
// with the tower weights in LDS and activations in the fused kernel's register
// orientation (lane (c, g): row c, features 16t + 4g .. +3; a layer's output is the
// next MFMA's B operand, the forward values stay in registers as the dgrad masks).
// H_k and D_k are written for lyr_bwd_w_kernel / lyr_scatter0_kernel, none is read
// back.  Replaces lyr_fwd0_fact_kernel, L - 1 lyr_fwd_kernel, lyr_predict_kernel and
// L - 1 lyr_bwd_data_kernel launches.
template <int DM, int L>
struct ChainShape {
    __host__ __device__ static constexpr int S(int k) { return (2 * DM) >> k; }  // S(1) = DM, S(L) = F
    __host__ __device__ static constexpr int T16(int n) { return (n + 15) / 16; }
    __host__ __device__ static constexpr int SW(int k) { return 16 * T16(S(k)) + 4; }   // LDS row stride of W_k
    __host__ __device__ static constexpr int WR(int k) { return 16 * T16(S(k + 1)); }   // W_k rows, padded
    __host__ __device__ static constexpr int woff(int k) { return k <= 1 ? 0 : woff(k - 1) + WR(k - 1) * SW(k - 1); }
    __host__ __device__ static constexpr int boff(int k) { return k == 0 ? 0 : boff(k - 1) + 16 * T16(S(k)); }
    static constexpr int F = DM >> (L - 1);
    static constexpr int W_TOTAL = woff(L);  // layers 1 .. L-1
    static constexpr int B_TOTAL = boff(L);  // b_0 .. b_{L-1}, each padded to 16
    static constexpr int KT1 = T16(DM), MT1 = T16(DM / 2), TF = T16(F);
};
struct ChainBufs {
    float* H[5];  // H[1 .. L]
    float* D[4];  // D[0 .. L-1]: dL/d pre-activation of layer k, row stride S(k + 1)
};
#ifndef NCF_CHAIN_NT
#define NCF_CHAIN_NT 256
#endif
constexpr int CNT = NCF_CHAIN_NT, CROWS = CNT / 4;  // threads per block, rows per tile (16 per wave)
// UORD (the step was given the epoch's user order): the chain also sums item runs of
// D_0 (rows are item-grouped) and db_0 from an LDS image of the tile, and writes each
// D_0 row at its position in the user order, so the user-side walk
// (the walk blocks of lyr_bwd_w_multi_kernel) reads D_0 sequentially.  Without it,
// D_0 in row order and lyr_scatter0_kernel does all three.
template <int DM, int L, bool UORD>
__global__ __launch_bounds__(CNT, 2) void lyr_step_chain_kernel(LyrArgs a, const float* __restrict__ P, ChainBufs o,
                                                                int64_t R) {
    using C_ = ChainShape<DM, L>;
    constexpr int F = C_::F, TF = C_::TF, NW = CNT / 64;
    constexpr int SROW = (UORD && DM > 16 * TF ? DM : 16 * TF) + 1;  // staging row: GMF item grads, then D_0
    __shared__ __attribute__((aligned(16))) float sW[C_::W_TOTAL > 0 ? C_::W_TOTAL : 4];
    __shared__ __attribute__((aligned(16))) float sB[C_::B_TOTAL];
    __shared__ __attribute__((aligned(16))) float sWP[2][16 * TF];  // wp: [0] GMF part, [1] tower part (zero-padded)
    __shared__ float sIg[NW][16][SROW];                           // per wave: GMF item-gradient rows, then D_0 rows
    __shared__ int sIt[NW][16];                                    // per wave: item id per row (-1: none)
    __shared__ float sred[2 * 16 * TF + 2];                        // block sums: dwp GMF | dwp tower | dbp | loss
    const Sel s = select_rows(a);
    const ncf_layout& lay = a.lay;
    const float* prm = a.params;
    const bool gmf = lay.model_type != NCF_MODEL_MLP;
    const int Pg = gmf ? F : 0;
    const int t = threadIdx.x, l = t & 63, w = t >> 6, c = l & 15, g = l >> 4;
    if (blockIdx.x == 0 && t == 0) {  // step snapshot for ncf_reduce_adam_step
        a.ctl->snap_batch = a.ctl->batch;
        a.ctl->snap_t = a.ctl->adam_t + 1;
    }
    // weights: every thread's 16-byte loads issued together, then the LDS stores
#pragma unroll
    for (int k = 1; k < L; ++k) {
        constexpr int PERMAX = (C_::WR(1) * (C_::SW(1) / 4) + CNT - 1) / CNT;
        const int sw4 = C_::SW(k) / 4, in4 = C_::S(k) / 4, out = C_::S(k + 1), n4 = C_::WR(k) * sw4;
        const f4* Wg = reinterpret_cast<const f4*>(prm + lay.w[k]);  // [out][in], in % 4 == 0
        f4* Ws = reinterpret_cast<f4*>(sW + C_::woff(k));
        f4 v[PERMAX];
#pragma unroll
        for (int q = 0; q < PERMAX; ++q) {
            const int e = t + q * CNT, r = e / sw4, i4 = e - r * sw4;
            v[q] = (e < n4 && r < out && i4 < in4) ? Wg[(int64_t)r * in4 + i4] : zero4();
        }
#pragma unroll
        for (int q = 0; q < PERMAX; ++q) {
            const int e = t + q * CNT;
            if (e < n4) Ws[e] = v[q];
        }
    }
#pragma unroll
    for (int k = 0; k < L; ++k) {
        const int out = C_::S(k + 1);
        for (int e = t; e < 16 * C_::T16(out); e += CNT) sB[C_::boff(k) + e] = e < out ? prm[lay.b[k] + e] : 0.f;
    }
    for (int e = t; e < 16 * TF; e += CNT) {
        sWP[0][e] = (gmf && e < F) ? prm[lay.wp + e] : 0.f;
        sWP[1][e] = e < F ? prm[lay.wp + Pg + e] : 0.f;
    }
    for (int e = t; e < 2 * 16 * TF + 2; e += CNT) sred[e] = 0.f;
    __shared__ float sdb0[UORD ? DM : 1];  // UORD: db_0 block sums
    if (UORD)
        for (int e = t; e < DM; e += CNT) sdb0[e] = 0.f;
    const int32_t* inv = nullptr;  // UORD: row offset -> position in the user order (ncf_user_order)
    if constexpr (UORD) inv = reinterpret_cast<const int32_t*>(a.uorder + a.ctl->n_total) + s.base;
    float db0[(DM + 63) / 64];
#pragma unroll
    for (int i = 0; i < (DM + 63) / 64; ++i) db0[i] = 0.f;
    __syncthreads();
    const float bp = prm[lay.bp];
    // per-lane partials over the block's rows: dwp (features 16q + 4g .. +3), dbp, loss
    f4 aWg[TF], aWm[TF];
#pragma unroll
    for (int q = 0; q < TF; ++q) aWg[q] = aWm[q] = zero4();
    float aB = 0.f, aL = 0.f;
    const int64_t ntile = (R + CROWS - 1) / CROWS;
    auto fetch = [&](int64_t tile) -> uint64_t {  // the next tile's packed row, requested early
        const int64_t m = tile * CROWS + 16 * w + c;
        return (tile < ntile && m < s.nloc) ? a.rows[s.base + m] : ~0ull;  // ~0: padding (user -1)
    };
    uint64_t nrow = fetch(blockIdx.x);
    for (int64_t tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
        const int64_t m = tile * CROWS + 16 * w + c;  // this lane's row
        const uint64_t rw = nrow;
        nrow = fetch(tile + gridDim.x);
        int u = (int)(uint32_t)rw, it = (int)((rw >> 32) & 0x7fffffffu);
        const bool valid = u >= 0 && m < R;  // padding rows gather id 0 and get dz = 0
        if (u < 0) u = it = 0;
        // ---- forward
        f4 h[L + 1][C_::KT1];  // h[k]: H_k, orientation A
        {
            const float* pu = P + (int64_t)u * DM;
            const float* pi = P + ((int64_t)lay.user_num + it) * DM;
#pragma unroll
            for (int q = 0; q < C_::KT1; ++q) {
                const int j0 = 16 * q + 4 * g;
                h[1][q] = zero4();
                if (j0 < DM) {
                    const f4 vu = ld4(pu + j0), vi = ld4(pi + j0), bb = ld4(sB + j0);
                    h[1][q].x = fmaxf(vu.x + vi.x + bb.x, 0.f);
                    h[1][q].y = fmaxf(vu.y + vi.y + bb.y, 0.f);
                    h[1][q].z = fmaxf(vu.z + vi.z + bb.z, 0.f);
                    h[1][q].w = fmaxf(vu.w + vi.w + bb.w, 0.f);
                    if (L > 1 && m < R) *reinterpret_cast<f4*>(o.H[1] + m * DM + j0) = h[1][q];  // H_L: not stored
                }
            }
        }
        f4 ug[TF], ig[TF];
        if (gmf) {  // GMF rows, same orientation (requested before the tower MFMAs)
#pragma unroll
            for (int q = 0; q < TF; ++q) {
                const int j0 = 16 * q + 4 * g;
                ug[q] = j0 < F ? ld4(prm + lay.ug + (int64_t)u * F + j0) : zero4();
                ig[q] = j0 < F ? ld4(prm + lay.ig + (int64_t)it * F + j0) : zero4();
            }
        }
#pragma unroll
        for (int k = 1; k < L; ++k) {
            const int KT = C_::T16(C_::S(k)), MT = C_::T16(C_::S(k + 1)), out = C_::S(k + 1), sw = C_::SW(k);
            const float* Ws = sW + C_::woff(k);
#pragma unroll
            for (int mt = 0; mt < C_::MT1; ++mt) {
                if (mt >= MT) continue;
                f4 acc = ld4(sB + C_::boff(k) + 16 * mt + 4 * g);
                f4 wv[C_::KT1];
#pragma unroll
                for (int q = 0; q < C_::KT1; ++q)
                    if (q < KT) wv[q] = ld4(Ws + (16 * mt + c) * sw + 16 * q + 4 * g);
#pragma unroll
                for (int q = 0; q < C_::KT1; ++q) {
                    if (q >= KT) continue;
                    acc = MFMA4(wv[q].x, h[k][q].x, acc);
                    acc = MFMA4(wv[q].y, h[k][q].y, acc);
                    acc = MFMA4(wv[q].z, h[k][q].z, acc);
                    acc = MFMA4(wv[q].w, h[k][q].w, acc);
                }
                f4 hh;
                hh.x = fmaxf(acc.x, 0.f);
                hh.y = fmaxf(acc.y, 0.f);
                hh.z = fmaxf(acc.z, 0.f);
                hh.w = fmaxf(acc.w, 0.f);
                const int j0 = 16 * mt + 4 * g;
                if (k + 1 < L && m < R && j0 < out) *reinterpret_cast<f4*>(o.H[k + 1] + m * out + j0) = hh;
                h[k + 1][mt] = hh;  // padded outputs are 0: zero weight rows and bias
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        // ---- predict, loss, dz
        float zp = 0.f;
#pragma unroll
        for (int q = 0; q < TF; ++q) {
            const f4 wm = ld4(&sWP[1][16 * q + 4 * g]);
            zp += wm.x * h[L][q].x + wm.y * h[L][q].y + wm.z * h[L][q].z + wm.w * h[L][q].w;
            if (gmf) {
                const f4 wg = ld4(&sWP[0][16 * q + 4 * g]);
                zp += wg.x * (ug[q].x * ig[q].x) + wg.y * (ug[q].y * ig[q].y) + wg.z * (ug[q].z * ig[q].z) +
                      wg.w * (ug[q].w * ig[q].w);
            }
        }
        zp += __shfl_xor(zp, 16, 64);
        zp += __shfl_xor(zp, 32, 64);
        const float z = zp + bp;
        if (valid && g == 0 && a.logits_out != nullptr) a.logits_out[m] = z;
        float dz = 0.f;
        if (valid) {
            if (a.dz_mode == NCF_DZ_BCE) {
                const float y = (float)(uint32_t)(rw >> 63);
                dz = (sigmoidf_(z) - y) / s.gb;
                if (g == 0) aL += bce_loss(z, y) / s.gb;
            } else if (a.dz_mode == NCF_DZ_KD) {
                const float y = (float)(uint32_t)(rw >> 63);
                float rl;
                const float rg = kd_response(z, a.dlogit[s.base + m], a.kd_temp, &rl);
                dz = (a.kd_wt * (sigmoidf_(z) - y) + a.kd_wr * rg) / s.gb;
                if (g == 0) aL += (a.kd_wt * bce_loss(z, y) + a.kd_wr * rl) / s.gb;
            } else {
                dz = a.dlogit[s.base + m];
            }
        }
        if (g == 0) aB += dz;
        // ---- GMF backward: user rows per row, item rows staged for the run walk
        if (g == 0) sIt[w][c] = valid ? it : -1;
        if (gmf) {
#pragma unroll
            for (int q = 0; q < TF; ++q) {
                const int j0 = 16 * q + 4 * g;
                const f4 wg = ld4(&sWP[0][16 * q + 4 * g]);
                aWg[q].x += dz * (ug[q].x * ig[q].x);
                aWg[q].y += dz * (ug[q].y * ig[q].y);
                aWg[q].z += dz * (ug[q].z * ig[q].z);
                aWg[q].w += dz * (ug[q].w * ig[q].w);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float dg = dz * lane_get(wg, r);
                    if (valid && j0 + r < F) atomicAdd(a.grads + lay.ug + (int64_t)u * F + j0 + r, dg * lane_get(ig[q], r));
                    if (j0 + r < 16 * TF) sIg[w][c][j0 + r] = dg * lane_get(ug[q], r);
                }
            }
        }
        // ---- GMF item rows: runs of equal items summed (lane = feature) before the atomics
        if (gmf) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // same-wave LDS hand-off
            int ids[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) ids[r] = __builtin_amdgcn_readfirstlane(sIt[w][r]);
            for (int f0 = 0; f0 < F; f0 += 64) {
                const int f = f0 + l;
                const int fc = f < F ? f : F - 1;
                float v[16];
#pragma unroll
                for (int r = 0; r < 16; ++r) v[r] = sIg[w][r][fc];
                float run = 0.f;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    run += v[r];
                    if (r == 15 || ids[r + 1] != ids[r]) {
                        if (ids[r] >= 0 && f < F) atomicAdd(a.grads + lay.ig + (int64_t)ids[r] * F + f, run);
                        run = 0.f;
                    }
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next tile's writes
        }
        // ---- tower backward: D_{L-1} = dz wp [H_L > 0], then D_{k-1} = (D_k W_k) [H_k > 0]
        f4 d[C_::KT1];
#pragma unroll
        for (int q = 0; q < TF; ++q) {
            const f4 wm = ld4(&sWP[1][16 * q + 4 * g]);
            aWm[q].x += dz * h[L][q].x;
            aWm[q].y += dz * h[L][q].y;
            aWm[q].z += dz * h[L][q].z;
            aWm[q].w += dz * h[L][q].w;
            d[q].x = h[L][q].x > 0.f ? dz * wm.x : 0.f;
            d[q].y = h[L][q].y > 0.f ? dz * wm.y : 0.f;
            d[q].z = h[L][q].z > 0.f ? dz * wm.z : 0.f;
            d[q].w = h[L][q].w > 0.f ? dz * wm.w : 0.f;
            const int j0 = 16 * q + 4 * g;
            if (UORD && L == 1) {  // D_0 at the row's position in the user order
                if (m < s.nloc && j0 < F) *reinterpret_cast<f4*>(o.D[0] + (int64_t)inv[m] * F + j0) = d[q];
            } else if (m < R && j0 < F) {
                *reinterpret_cast<f4*>(o.D[L - 1] + m * F + j0) = d[q];
            }
        }
#pragma unroll
        for (int k = L - 1; k >= 1; --k) {
            const int MT = C_::T16(C_::S(k + 1)), KT = C_::T16(C_::S(k)), in = C_::S(k), sw = C_::SW(k);
            const float* Ws = sW + C_::woff(k);
            f4 acc[C_::KT1];
#pragma unroll
            for (int m2 = 0; m2 < C_::KT1; ++m2) acc[m2] = zero4();
#pragma unroll
            for (int q = 0; q < C_::MT1; ++q) {
                if (q >= MT) continue;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float bv = lane_get(d[q], r);
#pragma unroll
                    for (int m2 = 0; m2 < C_::KT1; ++m2) {
                        if (m2 >= KT) continue;
                        acc[m2] = MFMA4(Ws[(16 * q + 4 * g + r) * sw + 16 * m2 + c], bv, acc[m2]);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int m2 = 0; m2 < C_::KT1; ++m2) {
                if (m2 >= KT) continue;
                const f4 hv = h[k][m2];
                f4 dd;
                dd.x = hv.x > 0.f ? acc[m2].x : 0.f;
                dd.y = hv.y > 0.f ? acc[m2].y : 0.f;
                dd.z = hv.z > 0.f ? acc[m2].z : 0.f;
                dd.w = hv.w > 0.f ? acc[m2].w : 0.f;
                const int j0 = 16 * m2 + 4 * g;
                if (UORD && k == 1) {  // D_0 at the row's position in the user order
                    if (m < s.nloc && j0 < in) *reinterpret_cast<f4*>(o.D[0] + (int64_t)inv[m] * in + j0) = dd;
                } else if (m < R && j0 < in) {
                    *reinterpret_cast<f4*>(o.D[k - 1] + m * in + j0) = dd;
                }
                d[m2] = dd;
            }
        }
        // ---- D_0 (UORD): item runs and db_0 from the tile's LDS image, rows to user-order positions
        if constexpr (UORD) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the GMF walk's reads are done
#pragma unroll
            for (int m2 = 0; m2 < C_::KT1; ++m2) {
                const int j0 = 16 * m2 + 4 * g;
                if (j0 < DM) {
                    sIg[w][c][j0] = d[m2].x;
                    sIg[w][c][j0 + 1] = d[m2].y;
                    sIg[w][c][j0 + 2] = d[m2].z;
                    sIg[w][c][j0 + 3] = d[m2].w;
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // same-wave LDS hand-off
            int ids[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) ids[r] = __builtin_amdgcn_readfirstlane(sIt[w][r]);
#pragma unroll
            for (int i = 0; i < (DM + 63) / 64; ++i) {
                const int f = 64 * i + l;
                const int fc = f < DM ? f : DM - 1;
                float v[16];
#pragma unroll
                for (int r = 0; r < 16; ++r) v[r] = sIg[w][r][fc];
                float run = 0.f;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    db0[i] += v[r];  // padding rows carry 0
                    run += v[r];
                    if (r == 15 || ids[r + 1] != ids[r]) {
                        if (ids[r] >= 0 && f < DM) atomicAdd(a.grads + lay.im + (int64_t)ids[r] * DM + f, run);
                        run = 0.f;
                    }
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next tile's writes
        }
    }
    // ---- block tail: dwp (sum over the 16 rows of a lane group), dbp, loss -> LDS -> slab
#pragma unroll
    for (int q = 0; q < TF; ++q) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float vg = lane_get(aWg[q], r), vm = lane_get(aWm[q], r);
#pragma unroll
            for (int o2 = 1; o2 < 16; o2 <<= 1) {
                vg += __shfl_xor(vg, o2, 64);
                vm += __shfl_xor(vm, o2, 64);
            }
            const int f = 16 * q + 4 * g + r;
            if (c == 0 && f < F) {
                if (gmf) atomicAdd(&sred[f], vg);
                atomicAdd(&sred[16 * TF + f], vm);
            }
        }
    }
#pragma unroll
    for (int o2 = 1; o2 < 64; o2 <<= 1) {
        aB += __shfl_xor(aB, o2, 64);
        aL += __shfl_xor(aL, o2, 64);
    }
    if (l == 0) {
        atomicAdd(&sred[2 * 16 * TF], aB);
        atomicAdd(&sred[2 * 16 * TF + 1], aL);
    }
    if constexpr (UORD) {
#pragma unroll
        for (int i = 0; i < (DM + 63) / 64; ++i)
            if (64 * i + l < DM) atomicAdd(&sdb0[64 * i + l], db0[i]);
    }
    __syncthreads();
    const int64_t tb = lay.tower_begin;
    float* slab = a.slab + (int64_t)(blockIdx.x % lyr_slab_rows(&lay)) * (lay.tower_len + 64);
    if constexpr (UORD) {
        for (int e = t; e < DM; e += CNT)
            if (sdb0[e] != 0.f) atomicAdd(slab + (lay.b[0] - tb) + e, sdb0[e]);
    }
    for (int e = t; e < 2 * F + 2; e += CNT) {
        int src;
        int64_t off;
        if (e < F) {
            if (!gmf) continue;
            src = e;
            off = (lay.wp - tb) + e;
        } else if (e < 2 * F) {
            src = 16 * TF + (e - F);
            off = (lay.wp - tb) + Pg + (e - F);
        } else {
            src = 2 * 16 * TF + (e - 2 * F);
            off = e == 2 * F ? (lay.bp - tb) : lay.tower_len;
        }
        const float v = sred[src];
        if (v != 0.f) atomicAdd(slab + off, v);
    }
}

#ifndef NCF_CHAIN_GRID
#define NCF_CHAIN_GRID 512
#endif
// Launch the step chain for (DM, L) with factor_num = DM >> (L - 1) a multiple of 4;
// false if there is no instantiation (the caller runs the per-layer kernels).
static bool launch_step_chain(const LyrArgs& a, const float* P, const ChainBufs& o, int64_t R, hipStream_t st) {
    const ncf_layout& lay = a.lay;
    const int L = lay.num_layers, DM = lay.factor_num << (L - 1);
    int64_t grid = (R + CROWS - 1) / CROWS;
    if (grid > NCF_CHAIN_GRID) grid = NCF_CHAIN_GRID;  // weights staged once per block, several tiles each
    if (grid < 1) grid = 1;
#define NCF_CHAIN(D, LL)                                                                                   \
    if (DM == D && L == LL) {                                                                              \
        if (a.uorder)                                                                                      \
            hipLaunchKernelGGL((lyr_step_chain_kernel<D, LL, true>), dim3((unsigned)grid), dim3(CNT), 0, st, a, \
                               P, o, R);                                                                   \
        else                                                                                               \
            hipLaunchKernelGGL((lyr_step_chain_kernel<D, LL, false>), dim3((unsigned)grid), dim3(CNT), 0, st, a, \
                               P, o, R);                                                                   \
        return true;                                                                                       \
    }
    NCF_CHAIN(8, 1) NCF_CHAIN(8, 2)
    NCF_CHAIN(16, 1) NCF_CHAIN(16, 2) NCF_CHAIN(16, 3)
    NCF_CHAIN(32, 1) NCF_CHAIN(32, 2) NCF_CHAIN(32, 3) NCF_CHAIN(32, 4)
    NCF_CHAIN(64, 1) NCF_CHAIN(64, 2) NCF_CHAIN(64, 3) NCF_CHAIN(64, 4)
    NCF_CHAIN(128, 1) NCF_CHAIN(128, 2) NCF_CHAIN(128, 3) NCF_CHAIN(128, 4)
#undef NCF_CHAIN
    return false;
}

// dY_0 rows -> grads[um][u] and grads[im][i] (width DM), db_0 -> slab.  A walker of
// DM lanes (one feature each; 256 / DM walkers per block, a walker may span two
// waves: nothing crosses lanes) takes SC_ROWS consecutive rows: its rows' values are
// loaded first, then the walk sums runs of equal items (each batch is grouped by
// item, ncf_prepare_epoch) before their atomics.  Users: with the epoch's user
// order (UORD, ncf_user_order) the walker takes the same number of consecutive
// positions of that order and sums runs of equal users likewise (a second, gathered
// pass over D0: ~10 rows per user in a 65,536-row batch of ML-1M, so ~5x fewer user
// atomics); without it, one atomic per row and feature.  One feature per lane keeps
// the grid at 4 x 65,536 / SC_ROWS waves for a dm-128 batch of 65,536: the dependent
// loads (order entry -> D0 row) are latency-bound and need the waves.
// db_0: walker sums -> LDS -> one atomic per feature per block; 1,024-thread blocks
// (8 walkers at dm 128) keep those slab atomics 4x fewer than 256-thread ones.
constexpr int SC_ROWS = 16, SC_NT = 1024;
template <int DM, bool UORD>
__global__ __launch_bounds__(SC_NT) void lyr_scatter0_kernel(LyrArgs a, const float* __restrict__ D0) {
    constexpr int NW = SC_NT / DM;  // walkers per block
    __shared__ float sdb[NW][DM];
    const Sel s = select_rows(a);
    const ncf_layout& lay = a.lay;
    const int n = threadIdx.x % DM, wk = threadIdx.x / DM;
    const int64_t r0 = ((int64_t)blockIdx.x * NW + wk) * SC_ROWS;
    float db = 0.f;
    if (r0 < s.nloc) {
        const int nr = (int)(s.nloc - r0 < SC_ROWS ? s.nloc - r0 : SC_ROWS);
        int us[SC_ROWS], is[SC_ROWS];
        float v[SC_ROWS];
#pragma unroll
        for (int k = 0; k < SC_ROWS; ++k) {
            const int64_t m = r0 + (k < nr ? k : 0);
            const uint64_t rw = a.rows[s.base + m];
            us[k] = (int)(uint32_t)rw;
            is[k] = us[k] < 0 ? -1 : (int)((rw >> 32) & 0x7fffffffu);  // row_ids: padding rows add nothing
            v[k] = D0[m * DM + n];
        }
        float run = 0.f;
#pragma unroll
        for (int k = 0; k < SC_ROWS; ++k) {
            if (k < nr) {
                const bool end = k + 1 >= nr || is[k + 1 < SC_ROWS ? k + 1 : k] != is[k];  // item run ends here
                db += v[k];
                if (!UORD && us[k] >= 0) atomicAdd(a.grads + lay.um + (int64_t)us[k] * DM + n, v[k]);
                run += v[k];
                if (end) {
                    if (is[k] >= 0) atomicAdd(a.grads + lay.im + (int64_t)is[k] * DM + n, run);
                    run = 0.f;
                }
            }
        }
        if constexpr (UORD) {
            int64_t ms[SC_ROWS];
#pragma unroll
            for (int k = 0; k < SC_ROWS; ++k) {
                const int64_t e = a.uorder[s.base + r0 + (k < nr ? k : 0)];  // user << 32 | offset
                const int64_t m = (int64_t)(uint32_t)e;
                const bool ok = m < s.nloc;
                ms[k] = ok ? m : 0;
                us[k] = ok ? (int)(e >> 32) : -1;
            }
#pragma unroll
            for (int k = 0; k < SC_ROWS; ++k) v[k] = D0[ms[k] * DM + n];
            run = 0.f;
#pragma unroll
            for (int k = 0; k < SC_ROWS; ++k) {
                if (k < nr) {
                    const bool end = k + 1 >= nr || us[k + 1 < SC_ROWS ? k + 1 : k] != us[k];  // user run ends here
                    run += v[k];
                    if (end) {
                        if (us[k] >= 0) atomicAdd(a.grads + lay.um + (int64_t)us[k] * DM + n, run);
                        run = 0.f;
                    }
                }
            }
        }
    }
    sdb[wk][n] = db;
    __syncthreads();
    if (threadIdx.x < DM) {  // DM <= 128 < SC_NT
        float t = 0.f;
#pragma unroll
        for (int k = 0; k < NW; ++k) t += sdb[k][threadIdx.x];
        if (t != 0.f)
            atomicAdd(a.slab + (int64_t)(blockIdx.x % lyr_slab_rows(&lay)) * (lay.tower_len + 64) +
                          (lay.b[0] - lay.tower_begin) + threadIdx.x,
                      t);
    }
}

template <int DM>
static void launch_scatter0(const LyrArgs& a, const float* D0, int64_t R, hipStream_t st) {
    const int64_t per_block = (int64_t)(SC_NT / DM) * SC_ROWS;
    const dim3 grid((unsigned)((R + per_block - 1) / per_block));
    if (a.uorder)
        hipLaunchKernelGGL((lyr_scatter0_kernel<DM, true>), grid, dim3(SC_NT), 0, st, a, D0);
    else
        hipLaunchKernelGGL((lyr_scatter0_kernel<DM, false>), grid, dim3(SC_NT), 0, st, a, D0);
}

// User side of the factored layer 0 after the step chain (UORD): D_0 rows already
// sit in user order (position p of the rank slice at D0u + p * DM), so a walker of
// DM lanes reads SC_ROWS consecutive positions sequentially, takes each position's
// user from its order entry (user << 32 | offset) and sums runs of equal users
// before the atomics into grads[um].  Items and db_0 were done in the chain.
// Walker share of the user-order walk: block `blk` of `nt` threads, feature n = t % dm,
// walker t / dm over SC_ROWS consecutive positions of the user order.
__device__ __forceinline__ void user_walk_body(const LyrArgs& a, const float* __restrict__ D0u, int64_t blk,
                                               int nt, int dm) {
    const Sel s = select_rows(a);
    const ncf_layout& lay = a.lay;
    const int n = threadIdx.x % dm, wk = threadIdx.x / dm;
    const int64_t r0 = (blk * (nt / dm) + wk) * SC_ROWS;
    if (r0 >= s.nloc) return;
    const int nr = (int)(s.nloc - r0 < SC_ROWS ? s.nloc - r0 : SC_ROWS);
    int us[SC_ROWS];
    float v[SC_ROWS];
#pragma unroll
    for (int k = 0; k < SC_ROWS; ++k) {
        const int64_t p = r0 + (k < nr ? k : 0);
        us[k] = (int)(a.uorder[s.base + p] >> 32);
        v[k] = D0u[p * dm + n];
    }
    float run = 0.f;
#pragma unroll
    for (int k = 0; k < SC_ROWS; ++k) {
        if (k < nr) {
            const bool end = k + 1 >= nr || us[k + 1 < SC_ROWS ? k + 1 : k] != us[k];
            run += v[k];
            if (end) {
                if (us[k] >= 0) atomicAdd(a.grads + lay.um + (int64_t)us[k] * dm + n, run);
                run = 0.f;
            }
        }
    }
}



// ---------------------------------------------------------------------------
// Predict + loss + GMF backward.  A walker of G lanes (G = min(64, pow2 >= F);
// feature f on lane f % G, slot f / G < NS) takes PR_ROWS consecutive rows: their
// operands are loaded first, the G-lane logit reductions of all of them run
// interleaved, and runs of equal items (each batch is grouped by item,
// ncf_prepare_epoch) are summed before the GMF item-gradient atomics.  dwp / dbp /
// loss: registers -> LDS -> one atomic per value per block, into slab row
// blockIdx % lyr_slab_rows.
constexpr int PR_ROWS = 8;  // NS <= 4: F <= 256 (LYR_MAX_FACTOR)
template <bool TRAIN, int NS>
__global__ __launch_bounds__(GNT) void lyr_predict_kernel(LyrArgs a, const float* __restrict__ HL,
                                                          float* __restrict__ Dout, int64_t R, int G) {
    extern __shared__ float red[];  // [P + 2]: dwp[P], dbp, loss
    const Sel s = select_rows(a);
    const ncf_layout& lay = a.lay;
    const int F = lay.factor_num;
    const bool gmf = lay.model_type != NCF_MODEL_MLP, mlp = lay.model_type != NCF_MODEL_GMF;
    const int Pg = gmf ? F : 0, P = Pg + (mlp ? F : 0);
    const float* prm = a.params;
    const float* wp = prm + lay.wp;
    const int t = threadIdx.x;
    if (TRAIN) {
        for (int e = t; e < P + 2; e += GNT) red[e] = 0.f;
        if (blockIdx.x == 0 && t == 0) {  // step snapshot for ncf_reduce_adam_step
            a.ctl->snap_batch = a.ctl->batch;
            a.ctl->snap_t = a.ctl->adam_t + 1;
        }
    }
    const int gl = t % G;
    const int64_t r0 = ((int64_t)blockIdx.x * (GNT / G) + t / G) * PR_ROWS;
    float wpg[NS], wpm[NS];
#pragma unroll
    for (int q = 0; q < NS; ++q) {
        const int f = gl + q * G;
        wpg[q] = (gmf && f < F) ? wp[f] : 0.f;
        wpm[q] = (mlp && f < F) ? wp[Pg + f] : 0.f;
    }
    // the walker's rows and operands (row_ids: padding rows have user -1)
    uint64_t rw[PR_ROWS];
    int us[PR_ROWS], is_[PR_ROWS];
    bool val[PR_ROWS];
    float ug[PR_ROWS][NS], ig[PR_ROWS][NS], hv[PR_ROWS][NS];
#pragma unroll
    for (int k = 0; k < PR_ROWS; ++k) {
        const int64_t m = r0 + k;
        const bool in = m < s.nloc;
        rw[k] = in ? a.rows[s.base + m] : 0;
        const int u = in ? (int)(uint32_t)rw[k] : -1;
        val[k] = m < R && u >= 0;
        us[k] = u < 0 ? 0 : u;
        is_[k] = val[k] ? (int)((rw[k] >> 32) & 0x7fffffffu) : -1;
        const int ii = is_[k] < 0 ? 0 : is_[k];
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            const int f = gl + q * G;
            const bool ok = val[k] && f < F;
            ug[k][q] = (gmf && ok) ? prm[lay.ug + (int64_t)us[k] * F + f] : 0.f;
            ig[k][q] = (gmf && ok) ? prm[lay.ig + (int64_t)ii * F + f] : 0.f;
            hv[k][q] = (mlp && ok) ? HL[m * F + f] : 0.f;
        }
    }
    float z[PR_ROWS];
#pragma unroll
    for (int k = 0; k < PR_ROWS; ++k) {
        float part = 0.f;
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            if (gmf) part += wpg[q] * (ug[k][q] * ig[k][q]);
            if (mlp) part += wpm[q] * hv[k][q];
        }
        z[k] = part;
    }
    for (int o = G >> 1; o >= 1; o >>= 1) {
#pragma unroll
        for (int k = 0; k < PR_ROWS; ++k) z[k] += __shfl_xor(z[k], o, 64);
    }
    const float bp = prm[lay.bp];
#pragma unroll
    for (int k = 0; k < PR_ROWS; ++k) {
        z[k] += bp;
        if (val[k] && gl == 0 && a.logits_out != nullptr) a.logits_out[r0 + k] = z[k];
    }
    if constexpr (TRAIN) {
        float accG[NS], accM[NS], run[NS];
#pragma unroll
        for (int q = 0; q < NS; ++q) accG[q] = accM[q] = run[q] = 0.f;
        float accB = 0.f, accL = 0.f;
#pragma unroll
        for (int k = 0; k < PR_ROWS; ++k) {
            const int64_t m = r0 + k;
            if (!val[k]) {
                if (mlp && m < R)
#pragma unroll
                    for (int q = 0; q < NS; ++q) {
                        const int f = gl + q * G;
                        if (f < F) Dout[m * F + f] = 0.f;
                    }
                continue;
            }
            float dz;
            if (a.dz_mode == NCF_DZ_BCE) {
                const float y = (float)(uint32_t)(rw[k] >> 63);
                dz = (sigmoidf_(z[k]) - y) / s.gb;
                if (gl == 0) accL += bce_loss(z[k], y) / s.gb;
            } else if (a.dz_mode == NCF_DZ_KD) {
                const float y = (float)(uint32_t)(rw[k] >> 63);
                float rl;
                const float rg = kd_response(z[k], a.dlogit[s.base + m], a.kd_temp, &rl);
                dz = (a.kd_wt * (sigmoidf_(z[k]) - y) + a.kd_wr * rg) / s.gb;
                if (gl == 0) accL += (a.kd_wt * bce_loss(z[k], y) + a.kd_wr * rl) / s.gb;
            } else {
                dz = a.dlogit[s.base + m];
            }
            if (gl == 0) accB += dz;
            const bool end = k + 1 >= PR_ROWS || is_[k + 1 < PR_ROWS ? k + 1 : k] != is_[k];  // item run ends
#pragma unroll
            for (int q = 0; q < NS; ++q) {
                const int f = gl + q * G;
                if (f >= F) continue;
                if (gmf) {
                    accG[q] += dz * (ug[k][q] * ig[k][q]);
                    const float dg = dz * wpg[q];
                    atomicAdd(a.grads + lay.ug + (int64_t)us[k] * F + f, dg * ig[k][q]);
                    run[q] += dg * ug[k][q];
                    if (end) {
                        atomicAdd(a.grads + lay.ig + (int64_t)is_[k] * F + f, run[q]);
                        run[q] = 0.f;
                    }
                }
                if (mlp) {
                    accM[q] += dz * hv[k][q];
                    Dout[m * F + f] = hv[k][q] > 0.f ? dz * wpm[q] : 0.f;
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            const int f = gl + q * G;
            if (f >= F) continue;
            if (gmf) atomicAdd(&red[f], accG[q]);
            if (mlp) atomicAdd(&red[Pg + f], accM[q]);
        }
        if (gl == 0) {
            atomicAdd(&red[P], accB);
            atomicAdd(&red[P + 1], accL);
        }
        __syncthreads();
        const int64_t tb = lay.tower_begin;
        float* slab = a.slab + (int64_t)(blockIdx.x % lyr_slab_rows(&lay)) * (lay.tower_len + 64);
        for (int e = t; e < P + 2; e += GNT) {
            const float v = red[e];
            if (v == 0.f) continue;
            const int64_t off = e < P ? (lay.wp - tb) + e : (e == P ? (lay.bp - tb) : lay.tower_len);
            atomicAdd(slab + off, v);
        }
    }
}

#include "ncf_chain_wide.inc"

// Block tile of the chained path's weight-gradient GEMMs (dm >= 256): X6W_TB, the 128 x
// 128 core (stress: lyr_bwd_w_multi 230 -> 165 us per step), or 64 with NCF_GEMM_TILE=64
// (A/B).  The projection and the factored expansion (K = dm = 512: 16 K steps) keep the
// 64 x 64 core: with 128-tiles they ran at a quarter of the blocks and slower (proj 55 ->
// 58, dX 56 -> 60, dW0 61 -> 68 us, profiles/r06_evidence/gemm_tile_ab/); NCF_PROJ_TILE=128
// selects the 128 x 128 core for them (A/B).
int lyr_gemm_tile() {
    static int tb = -1;
    if (tb < 0) {
        const char* e = getenv("NCF_GEMM_TILE");
        tb = (e != nullptr && atoi(e) == 64) ? 64 : X6W_TB;
    }
    return tb;
}
// NCF_W0PRE=0: the wide chain's projection and dX split W0 per block (A/B)
bool w0_pre_enabled() {
    static int on = -1;
    if (on < 0) {
        const char* e = getenv("NCF_W0PRE");
        on = (e != nullptr && e[0] == '0') ? 0 : 1;
    }
    return on == 1;
}
int lyr_proj_tile() {
    static int tb = -1;
    if (tb < 0) {
        const char* e = getenv("NCF_PROJ_TILE");
        tb = (e != nullptr && atoi(e) == X6W_TB) ? X6W_TB : 64;
    }
    return tb;
}
// dynamic LDS of a 128-tile kernel (set once per kernel)
bool x6w_ready(const void* fn) {
    static const void* done[8] = {};
    for (const void* d : done)
        if (d == fn) return true;
    if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, X6W_LDS) != hipSuccess) return false;
    for (auto& d : done)
        if (d == nullptr) {
            d = fn;
            break;
        }
    return true;
}
int64_t env_int(const char* name, int64_t dflt) {
    const char* e = getenv(name);
    const long long v = e ? atoll(e) : 0;
    return v > 0 ? (int64_t)v : dflt;
}

}  // namespace

// ---------------------------------------------------------------------------
int lyr_launch_proj(const ncf_layout* lay, const float* params, float* P, float* zero, int64_t zero_floats,
                    hipStream_t st) {
    const int DM = lay->factor_num << (lay->num_layers - 1);
    const int TB = DM >= 256 ? lyr_proj_tile() : 64;
    const int nbu = (int)((lay->user_num + TB - 1) / TB), nbi = (int)((lay->item_num + TB - 1) / TB);
    const dim3 grid((unsigned)(nbu + nbi), (unsigned)((DM + TB - 1) / TB));
    if (TB == X6W_TB) {
        if (!x6w_ready(reinterpret_cast<const void*>(&lyr_proj_kernel<X6W_TB>))) return NCF_E_LAUNCH;
        hipLaunchKernelGGL(lyr_proj_kernel<X6W_TB>, grid, dim3(GNT), X6W_LDS, st, *lay, params, P, nbu, zero,
                           zero_floats / 4);
    } else {
        hipLaunchKernelGGL(lyr_proj_kernel<64>, grid, dim3(GNT), 0, st, *lay, params, P, nbu, zero, zero_floats / 4);
    }
    return hipGetLastError() == hipSuccess ? NCF_OK : NCF_E_LAUNCH;
}

int64_t lyr_workspace_floats(const ncf_layout* lay, int64_t rows, bool train, int64_t fact_part_floats) {
    int64_t fl = rup64((int64_t)lyr_slab_rows(lay) * (lay->tower_len + 64));
    if (lay->model_type == NCF_MODEL_GMF) return fl;
    const int DM = lay->factor_num << (lay->num_layers - 1);
    if (train && fact_part_floats >= 0)  // dW0 partials, table projections
        fl += rup64(fact_part_floats) + rup64(((int64_t)lay->user_num + lay->item_num) * DM);
    for (int k = 1; k <= lay->num_layers; ++k) fl += rup64(rows * ((2 * DM) >> k));
    if (train) fl += 2 * rup64(rows * DM);
    if (train && fact_part_floats >= 0 && DM == wc::DM && lay->num_layers == wc::L)
        fl += rup64((int64_t)wc::NCH * wc::CHUNK / 4 + 4 * wc::W0_IMG_BYTES / 4);  // the wide chain's weight images
    return fl;
}

// The factored expansion as GEMMs (dm > FACT_LDS_DM, after the layer-0 scatter): dX
// into the dead projection buffer, dW0 into the slab's W0 columns (both read G), then
// dX copied over G.
static int launch_gemm_expand(const LyrArgs& a, float* Pj, hipStream_t st, const char* w0img = nullptr) {
    const ncf_layout& lay = a.lay;
    const int DM = lay.factor_num << (lay.num_layers - 1);
    const int U = lay.user_num, I = lay.item_num;
    const int TB = lyr_proj_tile();
    const int nbu = (U + TB - 1) / TB, nbi = (I + TB - 1) / TB;
    const dim3 gx((unsigned)(nbu + nbi), (unsigned)((DM + TB - 1) / TB));
    // dW0 row chunks: each chunk adds its whole tile with float atomics; 512 rows (16 K
    // steps per block) against 256 took the stress step 846 -> 832 us (NCF_DW0_CHUNK:
    // A/B, profiles/r06_evidence/dw0_chunk_ab/)
    const int64_t chunk = env_int("NCF_DW0_CHUNK", 512);
    const int zu = (int)((U + chunk - 1) / chunk), zi = (int)((I + chunk - 1) / chunk);
    const dim3 gw((unsigned)((DM + TB - 1) / TB), (unsigned)((DM + TB - 1) / TB), (unsigned)(zu + zi));
    if (w0img != nullptr && TB == 64) {  // dX with W0 pre-split (images 2, 3 of lyr_wc_prep_kernel)
        hipLaunchKernelGGL((lyr_fact_dx_kernel<64, true>), gx, dim3(GNT), 0, st, lay, a.params, a.grads, Pj, nbu,
                           w0img + 2 * wc::W0_IMG_BYTES);
        hipLaunchKernelGGL(lyr_fact_dw0_kernel<64>, gw, dim3(GNT), 0, st, a, zu, chunk);
    } else if (TB == X6W_TB) {
        if (!x6w_ready(reinterpret_cast<const void*>(&lyr_fact_dx_kernel<X6W_TB>)) ||
            !x6w_ready(reinterpret_cast<const void*>(&lyr_fact_dw0_kernel<X6W_TB>)))
            return NCF_E_LAUNCH;
        hipLaunchKernelGGL(lyr_fact_dx_kernel<X6W_TB>, gx, dim3(GNT), X6W_LDS, st, lay, a.params, a.grads, Pj, nbu);
        hipLaunchKernelGGL(lyr_fact_dw0_kernel<X6W_TB>, gw, dim3(GNT), X6W_LDS, st, a, zu, chunk);
    } else {
        hipLaunchKernelGGL(lyr_fact_dx_kernel<64>, gx, dim3(GNT), 0, st, lay, a.params, a.grads, Pj, nbu);
        hipLaunchKernelGGL(lyr_fact_dw0_kernel<64>, gw, dim3(GNT), 0, st, a, zu, chunk);
    }
    if (hipMemcpyAsync(a.grads + lay.um, Pj, (size_t)U * DM * 4, hipMemcpyDeviceToDevice, st) != hipSuccess ||
        hipMemcpyAsync(a.grads + lay.im, Pj + (int64_t)U * DM, (size_t)I * DM * 4, hipMemcpyDeviceToDevice, st) !=
            hipSuccess)
        return NCF_E_LAUNCH;
    return hipGetLastError() == hipSuccess ? NCF_OK : NCF_E_LAUNCH;
}

int lyr_run(const LyrArgs& a0, float* ws, int64_t R, bool train, hipStream_t st) {
    LyrArgs a = a0;
    const ncf_layout& lay = a.lay;
    const int L = lay.num_layers, F = lay.factor_num;
    const int DM = F << (L - 1);
    const bool mlp = lay.model_type != NCF_MODEL_GMF;
    if (F > LYR_MAX_FACTOR) return NCF_E_UNSUPPORTED;
    float* slab = ws;
    a.slab = slab;
    float* H[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    float* Da = nullptr;
    float* Db = nullptr;
    const int64_t slab_floats = (int64_t)lyr_slab_rows(&lay) * (lay.tower_len + 64);
    int64_t off = rup64(slab_floats);
    const bool fact = train && mlp && a.fact_part_floats >= 0;
    const bool drop = train && mlp && lay.dropout > 0.f;  // dropout-masked kernel instantiations
    const bool vec = (F % 4) == 0;  // every tower width a multiple of 4: 16-byte operand loads
    float* Pj = nullptr;  // factored layer 0: table projections
    if (fact) {
        off += rup64(a.fact_part_floats);  // dW0 partials (ncf_ops.hip fact_partials)
        Pj = ws + off;
        off += rup64(((int64_t)lay.user_num + lay.item_num) * DM);
    }
    if (mlp) {
        for (int k = 1; k <= L; ++k) {
            H[k] = ws + off;
            off += rup64(R * ((2 * DM) >> k));
        }
        if (train) {
            Da = ws + off;
            off += rup64(R * DM);
            Db = ws + off;
            off += rup64(R * DM);
        }
    }
    // the slab is cleared by the step's first kernel (the projection or the first
    // forward layer) -- every slab add comes later in the stream; GMF-only: a launch
    if (train && mlp) {
        a.zero_p = slab;
        a.zero_n4 = slab_floats / 4;
    } else if (train && launch_zero_f32(slab, slab_floats, st) != NCF_OK) {
        return NCF_E_LAUNCH;
    }
    const unsigned mt = (unsigned)((R + GBM - 1) / GBM);
    char* w0img = nullptr;  // the pre-split W0 images of the wide chain's step (W0PRE)
    // factored training with f % 4 == 0: the step chain (forward, predict, data
    // gradients in one launch); D_0 in Da, D_1 .. D_{L-1} packed into Db
    ChainBufs cb;
    bool chained = false;
    bool wide = false;  // the wide chain (dm 512): D_0 in row order, scatter0 does items / users / db_0
    if (fact && vec && !drop) {
        // H_L feeds nothing after the chain (the predict layer is in it): not stored
        for (int k = 0; k < 5; ++k) cb.H[k] = (k >= 1 && k < L) ? H[k] : nullptr;
        float* q = Db;
        for (int k = 0; k < 4; ++k) {
            cb.D[k] = k == 0 ? Da : (k < L ? q : nullptr);
            if (k >= 1 && k < L) q += R * (DM >> k);  // row stride S(k + 1) = DM >> k, a multiple of 4
        }
    }
    if (mlp) {
        for (int k = 0; k < L; ++k) {
            const int N = (2 * DM) >> (k + 1);
            const dim3 grid(mt, (unsigned)((N + GBN - 1) / GBN));
            if (k == 0 && fact) {
                // the wide chain: its weight images (and W0's for the projection and the
                // expansion, W0PRE) prepared first, in one launch
                const bool wide_ok = vec && !drop && wide_chain_applies(lay);
                char* wimg = reinterpret_cast<char*>(ws + off);
                if (wide_ok && w0_pre_enabled()) {
                    w0img = wimg + (int64_t)wc::NCH * wc::CHUNK;
                    launch_wc_prep(a, wimg, w0img, st);
                    const int nbu = (lay.user_num + 63) / 64, nbi = (lay.item_num + 63) / 64;
                    hipLaunchKernelGGL((lyr_proj_kernel<64, true>), dim3((unsigned)(nbu + nbi), (unsigned)(DM / 64)),
                                       dim3(GNT), 0, st, lay, a.params, Pj, nbu, a.zero_p, a.zero_n4, w0img);
                } else if (lyr_launch_proj(&lay, a.params, Pj, a.zero_p, 4 * a.zero_n4, st) != NCF_OK) {
                    return NCF_E_LAUNCH;
                }
                if (vec && !drop && launch_step_chain(a, Pj, cb, R, st)) {
                    chained = true;
                    break;
                }
                if (wide_ok && launch_wide_chain(a, Pj, cb, wimg, R, st, w0img != nullptr)) {
                    chained = wide = true;
                    break;
                }
                int64_t g0 = (R * (DM / 4) + GNT - 1) / GNT;
                if (g0 > 8192) g0 = 8192;
                hipLaunchKernelGGL(lyr_fwd0_fact_kernel, dim3((unsigned)g0), dim3(GNT), 0, st, a, Pj, H[1], R);
            } else if (k == 0)
                {
                if (drop) hipLaunchKernelGGL((lyr_fwd_kernel<true, true, false>), grid, dim3(GNT), 0, st, a, k, nullptr, H[1], R);
                else if (vec) hipLaunchKernelGGL((lyr_fwd_kernel<true, false, true>), grid, dim3(GNT), 0, st, a, k, nullptr, H[1], R);
                else hipLaunchKernelGGL((lyr_fwd_kernel<true, false, false>), grid, dim3(GNT), 0, st, a, k, nullptr, H[1], R);
            }
            else
                {
                if (drop) hipLaunchKernelGGL((lyr_fwd_kernel<false, true, false>), grid, dim3(GNT), 0, st, a, k, H[k], H[k + 1], R);
                else if (vec) hipLaunchKernelGGL((lyr_fwd_kernel<false, false, true>), grid, dim3(GNT), 0, st, a, k, H[k], H[k + 1], R);
                else hipLaunchKernelGGL((lyr_fwd_kernel<false, false, false>), grid, dim3(GNT), 0, st, a, k, H[k], H[k + 1], R);
            }
        }
    }
    if (chained) {  // weight gradients of layers L-1 .. 1 (one launch), then the layer-0 scatter
        BwMulti bm;
        memset(&bm, 0, sizeof(bm));
        // blocks per layer (row splits x tiles): 1,024 64 x 64 blocks, or 256 of the 128
        // x 128 core (4x the work per row each; the float atomics of the split partials
        // stay at one dW per 2,048 rows of layer 1); layer 1 (the largest) first
        const int TB = DM >= 256 ? lyr_gemm_tile() : 64;  // narrower towers: 64-row tiles fit
        const int64_t bw_blocks = env_int("NCF_BW_BLOCKS", TB == X6W_TB ? 256 : 1024);
        for (int kk = 1; kk <= L - 1; ++kk) {
            const int k = TB == X6W_TB ? kk : L - kk;
            const int K = (2 * DM) >> k, J = K / 2;
            const int64_t tiles = (int64_t)((J + TB - 1) / TB) * ((K + TB - 1) / TB);
            int64_t splits = bw_blocks / tiles;
            const int64_t max_splits = (R + 255) / 256;
            if (splits > max_splits) splits = max_splits;
            if (splits < 1) splits = 1;
            int64_t chunk = (R + splits - 1) / splits;
            chunk = (chunk + GBK - 1) / GBK * GBK;
            splits = (R + chunk - 1) / chunk;
            const int i = bm.n++;
            bm.k[i] = k;
            bm.gx[i] = (J + TB - 1) / TB;
            bm.gy[i] = (K + TB - 1) / TB;
            bm.D[i] = cb.D[k];
            bm.A[i] = H[k];
            bm.chunk[i] = chunk;
            bm.start[i + 1] = bm.start[i] + (int)(bm.gx[i] * bm.gy[i] * splits);
        }
        int walk = 0;
        if (a.uorder && !wide) {  // the user-order walk of D_0 rides in the same launch
            const int64_t per_block = (int64_t)(GNT / DM) * SC_ROWS;
            walk = (int)((R + per_block - 1) / per_block);
            bm.D0u = cb.D[0];
            bm.walk_dm = DM;
        }
        if (bm.start[bm.n] + walk > 0) {
            const dim3 grid((unsigned)(bm.start[bm.n] + walk));
            if (TB == X6W_TB) {
                if (!x6w_ready(reinterpret_cast<const void*>(&lyr_bwd_w_multi_kernel<X6W_TB>))) return NCF_E_LAUNCH;
                hipLaunchKernelGGL(lyr_bwd_w_multi_kernel<X6W_TB>, grid, dim3(GNT), X6W_LDS, st, a, bm, R);
            } else {
                hipLaunchKernelGGL(lyr_bwd_w_multi_kernel<64>, grid, dim3(GNT), 0, st, a, bm, R);
            }
        }
        // with the user order the chain did the item runs and db_0 and left D_0 in user
        // order (the walk blocks of the launch above read it sequentially); without,
        // the full scatter
#define NCF_L0(DD)                           \
    case DD:                                 \
        if (!a.uorder || wide)               \
            launch_scatter0<DD>(a, cb.D[0], R, st);  \
        break;
        switch (DM) {
            NCF_L0(8) NCF_L0(16) NCF_L0(32) NCF_L0(64) NCF_L0(128) NCF_L0(256) NCF_L0(512)
            default: return NCF_E_UNSUPPORTED;
        }
#undef NCF_L0
        if (DM > FACT_LDS_DM && launch_gemm_expand(a, Pj, st, w0img) != NCF_OK) return NCF_E_LAUNCH;
        return hipGetLastError() == hipSuccess ? NCF_OK : NCF_E_LAUNCH;
    }
    int G = 1;
    while (G < F && G < 64) G <<= 1;
    const int P = (lay.model_type == NCF_MODEL_NEUMF ? 2 : 1) * F;
    const int NS = (F + G - 1) / G;  // <= 4 (F <= 256)
    const int64_t rows_per_block = (int64_t)(GNT / G) * PR_ROWS;
    const unsigned pg = (unsigned)((R + rows_per_block - 1) / rows_per_block);
    const size_t lds = (size_t)(P + 2) * 4;
    float* Dtop = Da;
    float* HLp = mlp ? H[L] : nullptr;
#define NCF_PRED(T, N) hipLaunchKernelGGL((lyr_predict_kernel<T, N>), dim3(pg), dim3(GNT), lds, st, a, HLp, \
                                          T ? Dtop : nullptr, R, G)
    switch (NS * 2 + (train ? 1 : 0)) {
        case 2: NCF_PRED(false, 1); break;
        case 3: NCF_PRED(true, 1); break;
        case 4: NCF_PRED(false, 2); break;
        case 5: NCF_PRED(true, 2); break;
        case 6: NCF_PRED(false, 3); break;
        case 7: NCF_PRED(true, 3); break;
        case 8: NCF_PRED(false, 4); break;
        case 9: NCF_PRED(true, 4); break;
        default: return NCF_E_UNSUPPORTED;
    }
#undef NCF_PRED
    if (!train || !mlp) return hipGetLastError() == hipSuccess ? NCF_OK : NCF_E_LAUNCH;
    float* Dcur = Da;
    float* Dnext = Db;
    for (int k = L - 1; k >= 0; --k) {
        const int K = (2 * DM) >> k, J = K / 2;
        if (k == 0 && fact) {  // dY_0 into the table rows; dW0 / dUm / dIm by fact_expand_kernel
            switch (DM) {  // factored path: dm in {8, ..., 512} (fact_mode)
                case 8: launch_scatter0<8>(a, Dcur, R, st); break;
                case 16: launch_scatter0<16>(a, Dcur, R, st); break;
                case 32: launch_scatter0<32>(a, Dcur, R, st); break;
                case 64: launch_scatter0<64>(a, Dcur, R, st); break;
                case 128: launch_scatter0<128>(a, Dcur, R, st); break;
                case 256: launch_scatter0<256>(a, Dcur, R, st); break;
                case 512: launch_scatter0<512>(a, Dcur, R, st); break;
                default: return NCF_E_UNSUPPORTED;
            }
            if (DM > FACT_LDS_DM && launch_gemm_expand(a, Pj, st) != NCF_OK) return NCF_E_LAUNCH;
            break;
        }
        // weight gradient: split the rows so the launch has ~512 blocks
        const int64_t tiles = (int64_t)((J + GBM - 1) / GBM) * ((K + GBN - 1) / GBN);
        int64_t splits = 1024 / tiles;
        const int64_t max_splits = (R + 255) / 256;
        if (splits > max_splits) splits = max_splits;
        if (splits < 1) splits = 1;
        int64_t chunk = (R + splits - 1) / splits;
        chunk = (chunk + GBK - 1) / GBK * GBK;
        splits = (R + chunk - 1) / chunk;
        const dim3 gw((unsigned)((J + GBM - 1) / GBM), (unsigned)((K + GBN - 1) / GBN), (unsigned)splits);
        if (k == 0)
            {
                if (drop) hipLaunchKernelGGL((lyr_bwd_w_kernel<true, true, false>), gw, dim3(GNT), 0, st, a, k, Dcur, nullptr, R, chunk);
                else if (vec) hipLaunchKernelGGL((lyr_bwd_w_kernel<true, false, true>), gw, dim3(GNT), 0, st, a, k, Dcur, nullptr, R, chunk);
                else hipLaunchKernelGGL((lyr_bwd_w_kernel<true, false, false>), gw, dim3(GNT), 0, st, a, k, Dcur, nullptr, R, chunk);
            }
        else
            {
                if (drop) hipLaunchKernelGGL((lyr_bwd_w_kernel<false, true, false>), gw, dim3(GNT), 0, st, a, k, Dcur, H[k], R, chunk);
                else if (vec) hipLaunchKernelGGL((lyr_bwd_w_kernel<false, false, true>), gw, dim3(GNT), 0, st, a, k, Dcur, H[k], R, chunk);
                else hipLaunchKernelGGL((lyr_bwd_w_kernel<false, false, false>), gw, dim3(GNT), 0, st, a, k, Dcur, H[k], R, chunk);
            }
        const dim3 gd(mt, (unsigned)((K + GBN - 1) / GBN));
        if (k == 0) {
            {
                if (drop) hipLaunchKernelGGL((lyr_bwd_data_kernel<true, true, false>), gd, dim3(GNT), 0, st, a, k, Dcur, nullptr, nullptr, R);
                else if (vec) hipLaunchKernelGGL((lyr_bwd_data_kernel<true, false, true>), gd, dim3(GNT), 0, st, a, k, Dcur, nullptr, nullptr, R);
                else hipLaunchKernelGGL((lyr_bwd_data_kernel<true, false, false>), gd, dim3(GNT), 0, st, a, k, Dcur, nullptr, nullptr, R);
            }
        } else {
            {
                if (drop) hipLaunchKernelGGL((lyr_bwd_data_kernel<false, true, false>), gd, dim3(GNT), 0, st, a, k, Dcur, H[k], Dnext, R);
                else if (vec) hipLaunchKernelGGL((lyr_bwd_data_kernel<false, false, true>), gd, dim3(GNT), 0, st, a, k, Dcur, H[k], Dnext, R);
                else hipLaunchKernelGGL((lyr_bwd_data_kernel<false, false, false>), gd, dim3(GNT), 0, st, a, k, Dcur, H[k], Dnext, R);
            }
            float* tmp = Dcur;
            Dcur = Dnext;
            Dnext = tmp;
        }
    }
    return hipGetLastError() == hipSuccess ? NCF_OK : NCF_E_LAUNCH;
}

}  // namespace ncf
