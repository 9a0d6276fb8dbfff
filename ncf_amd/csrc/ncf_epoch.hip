// Device epoch pipeline (gfx950): the DataLoader(shuffle=True) permutation of the
// reference's training loop and the epoch's packed rows, built on the GPU.
//
//   DataLoader(shuffle=True)       scripts/train_neumf.py:55 -> RandomSampler ->
//     torch.randperm(n, generator=g), g.manual_seed(seed): Fisher-Yates,
//     for i < n - 1: swap(r[i], r[i + w_i % (n - i)]) over the MT19937 words w_i
//     (the words come from the host: ncf_mt_words in libncf_sampler.so).
//
// The negatives (NCFData.ng_sample, datasets.py:53-69) stay on the host sampler:
// each draw's acceptance depends on the user of the slot it lands in, which
// depends on every earlier rejection.  A chunked fixed-point formulation of that
// scan (start = scan(count(start))) was tried on the device and does not contract:
// a shifted start changes counts at every user boundary again, so the corrected
// prefix grew by ~10 users per iteration (hundreds of iterations at ml-1m).
//
// * ncf_randperm -- Fisher-Yates as parallel rounds (Shun et al., "Sequential
//   random permutation, list contraction and tree contraction are highly
//   parallel", SODA 2015): every pending swap i reserves positions i and
//   H[i] = i + w_i % (n - i) with a priority-min of (round tag, i); a swap that
//   holds both reservations has no pending earlier swap touching its positions,
//   so it commits now.  Same permutation as the sequential loop; ~2.3 log2(n)
//   rounds, the pending set shrinking ~0.7x per round.
// * ncf_build_rows -- features_fill / labels_fill (datasets.py:65-69) packed
//   (NCF_ROW_PACK): positives in file order, then positive p's num_ng negatives.
#include <string.h>

#include "ncf_common.h"

namespace ncf {

constexpr int EP_THREADS = 256;

static int64_t al256e(int64_t x) { return (x + 255) & ~(int64_t)255; }
static int ep_status() { return hipGetLastError() == hipSuccess ? NCF_OK : NCF_E_LAUNCH; }
static unsigned ep_grid(int64_t n, int64_t cap) {
    int64_t g = (n + EP_THREADS - 1) / EP_THREADS;
    if (g > cap) g = cap;
    if (g < 1) g = 1;
    return (unsigned)g;
}

__global__ __launch_bounds__(EP_THREADS) void fill_u64_kernel(unsigned long long* p, int64_t n, unsigned long long v) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) p[k] = v;
}

// ---------------------------------------------------------------------------
// Fisher-Yates rounds.  The first FY_FLAG_ROUNDS rounds walk every index with a
// pending flag (most swaps are pending: an appended list would put one
// same-address atomic per wave on the critical path -- 0.9 ms in round 1 at
// n = 5M); then the ~1% still pending are compacted once (one atomic per block)
// and the remaining rounds walk that list.
constexpr int FY_FLAG_ROUNDS = 13;  // 0.7^13 ~ 1% pending
__global__ __launch_bounds__(EP_THREADS) void fy_init_kernel(const uint32_t* __restrict__ words, int64_t n, int32_t* H,
                                                             int64_t* A, uint8_t* done) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        A[i] = i;
        if (i < n - 1) H[i] = (int32_t)(i + (int64_t)(words[i] % (uint32_t)(n - i)));  // generator->random() % (n - i)
        else H[i] = (int32_t)i;
        done[i] = i >= n - 1;
    }
}

__global__ __launch_bounds__(EP_THREADS) void fy_reserve_flags_kernel(const uint8_t* __restrict__ done, int64_t n,
                                                                      const int32_t* __restrict__ H,
                                                                      unsigned long long* R, uint32_t tag) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        if (done[i]) continue;
        const unsigned long long key = ((unsigned long long)tag << 32) | (uint32_t)i;
        atomicMin(R + i, key);
        const int h = H[i];
        if (h != i) atomicMin(R + h, key);
    }
}

__global__ __launch_bounds__(EP_THREADS) void fy_commit_flags_kernel(uint8_t* done, int64_t n,
                                                                     const int32_t* __restrict__ H,
                                                                     const unsigned long long* R, uint32_t tag,
                                                                     int64_t* A) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        if (done[i]) continue;
        const unsigned long long key = ((unsigned long long)tag << 32) | (uint32_t)i;
        const int h = H[i];
        if (R[i] == key && R[h] == key) {
            const int64_t x = A[i];
            A[i] = A[h];
            A[h] = x;
            done[i] = 1;
        }
    }
}

// Pending indices -> list (order irrelevant), one atomic per block.
constexpr int FY_CPT = 16;  // indices per thread
__global__ __launch_bounds__(EP_THREADS) void fy_compact_kernel(const uint8_t* __restrict__ done, int64_t n,
                                                                int32_t* list, int* count) {
    __shared__ int wsum[EP_THREADS / 64];
    __shared__ int base;
    const int64_t i0 = ((int64_t)blockIdx.x * EP_THREADS + threadIdx.x) * FY_CPT;
    int c = 0;
#pragma unroll
    for (int k = 0; k < FY_CPT; ++k) c += (i0 + k < n && !done[i0 + k]);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int q = 0; q < EP_THREADS / 64; ++q) t += wsum[q];
        base = t ? atomicAdd(count, t) : 0;
    }
    __syncthreads();
    int off = base + incl - c;
    for (int q = 0; q < wv; ++q) off += wsum[q];
#pragma unroll
    for (int k = 0; k < FY_CPT; ++k)
        if (i0 + k < n && !done[i0 + k]) list[off++] = (int32_t)(i0 + k);
}

__global__ __launch_bounds__(EP_THREADS) void fy_reserve_kernel(const int32_t* __restrict__ list, const int* count,
                                                                const int32_t* __restrict__ H, unsigned long long* R,
                                                                uint32_t tag, int* next_count) {
    const int n = *count;
    if (blockIdx.x == 0 && threadIdx.x == 0) *next_count = 0;  // the next round's list (read by nobody now)
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
        const int i = list[j];
        const unsigned long long key = ((unsigned long long)tag << 32) | (uint32_t)i;
        atomicMin(R + i, key);
        const int h = H[i];
        if (h != i) atomicMin(R + h, key);
    }
}

__global__ __launch_bounds__(EP_THREADS) void fy_commit_kernel(const int32_t* __restrict__ list, const int* count,
                                                               const int32_t* __restrict__ H,
                                                               const unsigned long long* R, uint32_t tag, int64_t* A,
                                                               int32_t* next_list, int* next_count) {
    const int n = *count;
    const int lane = threadIdx.x & 63;
    // grid-stride with a wave-uniform trip count: every lane reaches the ballot
    const int stride = gridDim.x * blockDim.x;
    for (int j0 = blockIdx.x * blockDim.x + (threadIdx.x & ~63); j0 < n; j0 += stride) {
        const int j = j0 + lane;
        bool pend = false;
        int i = 0;
        if (j < n) {
            i = list[j];
            const unsigned long long key = ((unsigned long long)tag << 32) | (uint32_t)i;
            const int h = H[i];
            if (R[i] == key && R[h] == key) {
                const int64_t x = A[i];
                A[i] = A[h];
                A[h] = x;
            } else {
                pend = true;
            }
        }
        // wave-aggregated append of the swaps still pending (few by now)
        const unsigned long long bal = __ballot(pend);
        if (bal == 0) continue;
        int base = 0;
        if (lane == __ffsll((long long)bal) - 1) base = atomicAdd(next_count, __popcll(bal));
        base = __shfl(base, __ffsll((long long)bal) - 1, 64);
        if (pend) next_list[base + __popcll(bal & ((1ull << lane) - 1))] = i;
    }
}

// After the parallel rounds: the swaps still pending (none in practice: the
// rounds launched cover ~1.3x the depth observed at n = 1e5 .. 1e8) are applied
// in index order by one thread, so the call always completes; more than
// FY_TAIL of them is reported through *remaining instead.
constexpr int FY_TAIL = 4096;
__global__ __launch_bounds__(1024) void fy_finish_kernel(const int32_t* __restrict__ list, const int* count,
                                                         const int32_t* __restrict__ H, int64_t* A, int32_t* remaining) {
    __shared__ int32_t srt[FY_TAIL];
    const int n = *count;
    if (n > FY_TAIL) {
        if (threadIdx.x == 0) *remaining = n;
        return;
    }
    for (int j = threadIdx.x; j < n; j += blockDim.x) {  // rank by counting (indices are distinct)
        const int i = list[j];
        int r = 0;
        for (int k = 0; k < n; ++k) r += list[k] < i;
        srt[r] = i;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 0; k < n; ++k) {
            const int i = srt[k], h = H[i];
            const int64_t x = A[i];
            A[i] = A[h];
            A[h] = x;
        }
        *remaining = 0;
    }
}

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(EP_THREADS) void build_rows_kernel(const int32_t* __restrict__ pu, const int32_t* __restrict__ pi,
                                                                int64_t P, const int32_t* __restrict__ neg, int ng,
                                                                uint64_t* __restrict__ rows) {
    const int64_t n = P * (1 + ng);
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        if (k < P) {
            rows[k] = NCF_ROW_PACK(pu[k], pi[k], 1);
        } else {
            const int64_t j = k - P;
            rows[k] = NCF_ROW_PACK(pu[j / ng], neg[j], 0);
        }
    }
}

struct FyLayout {
    int32_t* H;
    unsigned long long* R;
    int32_t* list[2];
    int* count;  // [2]
    uint8_t* done;
};

static FyLayout fy_layout(void* ws, int64_t n) {
    char* p = static_cast<char*>(ws);
    FyLayout f;
    f.count = reinterpret_cast<int*>(p);
    p += 256;
    f.R = reinterpret_cast<unsigned long long*>(p);
    p += al256e(n * 8);
    f.H = reinterpret_cast<int32_t*>(p);
    p += al256e(n * 4);
    f.list[0] = reinterpret_cast<int32_t*>(p);
    p += al256e(n * 4);
    f.list[1] = reinterpret_cast<int32_t*>(p);
    p += al256e(n * 4);
    f.done = reinterpret_cast<uint8_t*>(p);
    return f;
}

}  // namespace ncf

using namespace ncf;

extern "C" {

int64_t ncf_randperm_workspace(int64_t n) {
    if (n <= 0 || n > 0x7fffffff) return -1;
    return 256 + al256e(n * 8) + 3 * al256e(n * 4) + al256e(n);
}

int ncf_randperm(const uint32_t* words, int64_t n, int64_t* perm, int rounds, void* workspace, int64_t workspace_bytes,
                 int32_t* remaining, void* stream) {
    if (!perm || !workspace || !remaining || n <= 0 || n > 0x7fffffff || rounds < 1 || rounds > 0xfff0) return NCF_E_ARG;
    if (n > 1 && !words) return NCF_E_ARG;
    if (workspace_bytes < ncf_randperm_workspace(n)) return NCF_E_ARG;
    FyLayout F = fy_layout(workspace, n);
    hipStream_t st = (hipStream_t)stream;
    const unsigned g = ep_grid(n, 8192);
    hipLaunchKernelGGL(fill_u64_kernel, dim3(g), dim3(EP_THREADS), 0, st, F.R, n, ~0ull);
    hipLaunchKernelGGL(fy_init_kernel, dim3(g), dim3(EP_THREADS), 0, st, words, n, F.H, perm, F.done);
    const int fr = rounds < FY_FLAG_ROUNDS ? rounds : FY_FLAG_ROUNDS;
    for (int r = 0; r < fr; ++r) {
        const uint32_t tag = 0xffffu - (uint32_t)r;  // later rounds win over stale reservations
        hipLaunchKernelGGL(fy_reserve_flags_kernel, dim3(g), dim3(EP_THREADS), 0, st, F.done, n, F.H, F.R, tag);
        hipLaunchKernelGGL(fy_commit_flags_kernel, dim3(g), dim3(EP_THREADS), 0, st, F.done, n, F.H, F.R, tag, perm);
    }
    if (hipMemsetAsync(F.count, 0, 8, st) != hipSuccess) return NCF_E_LAUNCH;
    const int64_t per_block = (int64_t)EP_THREADS * FY_CPT;
    hipLaunchKernelGGL(fy_compact_kernel, dim3((unsigned)((n + per_block - 1) / per_block)), dim3(EP_THREADS), 0, st,
                       F.done, n, F.list[0], F.count);
    // list rounds: grids sized for ~2% of n pending (grid-stride covers any count)
    const unsigned gl = ep_grid(n / 48 + 1024, 4096);
    for (int r = fr; r < rounds; ++r) {
        const uint32_t tag = 0xffffu - (uint32_t)r;
        const int cur = (r - fr) & 1;
        hipLaunchKernelGGL(fy_reserve_kernel, dim3(gl), dim3(EP_THREADS), 0, st, F.list[cur], F.count + cur, F.H, F.R,
                           tag, F.count + (cur ^ 1));
        hipLaunchKernelGGL(fy_commit_kernel, dim3(gl), dim3(EP_THREADS), 0, st, F.list[cur], F.count + cur, F.H, F.R,
                           tag, perm, F.list[cur ^ 1], F.count + (cur ^ 1));
    }
    const int last = (rounds - fr) & 1;
    hipLaunchKernelGGL(fy_finish_kernel, dim3(1), dim3(1024), 0, st, F.list[last], F.count + last, F.H, perm,
                       remaining);
    return ep_status();
}

int ncf_build_rows(const int32_t* pos_users, const int32_t* pos_items, int64_t n_pos, const int32_t* neg, int num_ng,
                   uint64_t* rows_out, void* stream) {
    if (!pos_users || !pos_items || !rows_out || n_pos < 0 || num_ng < 0 || (num_ng > 0 && !neg)) return NCF_E_ARG;
    const int64_t n = n_pos * (1 + num_ng);
    if (n == 0) return NCF_OK;
    hipLaunchKernelGGL(build_rows_kernel, dim3(ep_grid(n, 8192)), dim3(EP_THREADS), 0, (hipStream_t)stream, pos_users,
                       pos_items, n_pos, neg, num_ng, rows_out);
    return ep_status();
}

}  // extern "C"
