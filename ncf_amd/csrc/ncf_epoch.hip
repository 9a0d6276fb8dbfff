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
// * ncf_randperm -- Fisher-Yates in closed form.  With H[i] = i + w_i % (n - i)
//   (H[n-1] = n-1), step i swaps positions i and H[i] >= i, so position p is
//   final after step p and only steps j < p with H[j] = p touch it before then.
//   Let S_q = {j : H[j] = q, j < q} ("the steps that target q") and
//   P(q) = max S_q (q itself when S_q is empty).  The value at position p when
//   step p starts is D(p) = D(P(p)) -- what step P(p) carried into p is what sat
//   at P(p) when that step started -- i.e. the root of the chain p -> P(p) -> ...
//   Step i then leaves at position i:
//       D(i)                    when H[i] = i,
//       D(k), k = max{j in S_{H[i]} : j < i}   (the previous step into H[i]),
//       H[i]                    when no earlier step targeted H[i].
//   The groups S_q come from one stable radix sort of (H[j], j) (rocPRIM
//   onesweep; LDS-local digit histograms, no per-element global atomics): in
//   sorted order each step's predecessor is its left neighbour, and the last of
//   each run is P(q).  Then one gather pass follows each chain to its root
//   (a few hops: chains are ~log n long for MT19937 words; any input is correct).
// * ncf_build_rows -- features_fill / labels_fill (datasets.py:65-69) packed
//   (NCF_ROW_PACK): positives in file order, then positive p's num_ng negatives.
#include <string.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

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

__device__ __forceinline__ int fy_target(const uint32_t* __restrict__ words, int64_t n, int i) {
    // generator->random() % (n - i), as torch.randperm's CPU loop
    return i < n - 1 ? (int)(i + (int64_t)(words[i] % (uint32_t)(n - i))) : i;
}

// Sort keys: H[j] for the steps that move something, n (past every target) for
// H[j] = j; P starts as the identity (empty S_q).
__global__ __launch_bounds__(EP_THREADS) void fy_keys_kernel(const uint32_t* __restrict__ words, int64_t n,
                                                             uint32_t* __restrict__ keys, int32_t* __restrict__ P) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int h = fy_target(words, n, i);
        keys[i] = h == i ? (uint32_t)n : (uint32_t)h;
        P[i] = i;
    }
}

// Sorted by (H, j): K[j] = left neighbour in the same run (-1 for the first),
// P(q) = the run's last step.
__global__ __launch_bounds__(EP_THREADS) void fy_runs_kernel(const uint32_t* __restrict__ ks,
                                                             const int32_t* __restrict__ vs, int64_t n,
                                                             int32_t* __restrict__ P, int32_t* __restrict__ K) {
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x) {
        const uint32_t q = ks[t];
        if (q == (uint32_t)n) continue;
        const int j = vs[t];
        K[j] = (t > 0 && ks[t - 1] == q) ? vs[t - 1] : -1;
        if (t + 1 == n || ks[t + 1] != q) P[q] = j;
    }
}

__device__ __forceinline__ int fy_root(const int32_t* __restrict__ P, int x) {
    for (int p = P[x]; p != x; p = P[x]) x = p;  // P(x) < x off the roots
    return x;
}

__global__ __launch_bounds__(EP_THREADS) void fy_final_kernel(const uint32_t* __restrict__ words, int64_t n,
                                                              const int32_t* __restrict__ P,
                                                              const int32_t* __restrict__ K, int64_t* __restrict__ A) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int h = fy_target(words, n, i);
        const int x = h == i ? i : K[i];
        A[i] = x < 0 ? h : fy_root(P, x);
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
    uint32_t *keys, *keys_sorted;
    int32_t *steps_sorted, *P, *K;
    void* sort_tmp;
    size_t sort_bytes;
};

static unsigned fy_key_bits(int64_t n) { return 64 - __builtin_clzll((unsigned long long)n); }  // keys <= n

// Sort temporary bytes for n keys (rocPRIM's own query; host-side arithmetic).
static bool fy_sort_bytes(int64_t n, size_t* bytes) {
    *bytes = 0;
    return rocprim::radix_sort_pairs(nullptr, *bytes, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                     rocprim::counting_iterator<int32_t>(0), (int32_t*)nullptr, (size_t)n, 0,
                                     fy_key_bits(n)) == hipSuccess;
}

static bool fy_layout(void* ws, int64_t n, FyLayout* f) {
    if (!fy_sort_bytes(n, &f->sort_bytes)) return false;
    char* p = static_cast<char*>(ws);
    void** parts[5] = {(void**)&f->keys, (void**)&f->keys_sorted, (void**)&f->steps_sorted, (void**)&f->P,
                       (void**)&f->K};
    for (auto* q : parts) {
        *q = p;
        p += al256e(n * 4);
    }
    f->sort_tmp = p;
    return true;
}

}  // namespace ncf

using namespace ncf;

extern "C" {

int64_t ncf_randperm_workspace(int64_t n) {
    if (n <= 0 || n > 0x7fffffff) return -1;
    size_t sb = 0;
    if (!fy_sort_bytes(n, &sb)) return -1;
    return 5 * al256e(n * 4) + al256e((int64_t)sb);
}

int ncf_randperm(const uint32_t* words, int64_t n, int64_t* perm, void* workspace, int64_t workspace_bytes,
                 void* stream) {
    if (!perm || !workspace || n <= 0 || n > 0x7fffffff) return NCF_E_ARG;
    if (n > 1 && !words) return NCF_E_ARG;
    const int64_t need = ncf_randperm_workspace(n);
    if (need < 0 || workspace_bytes < need) return NCF_E_ARG;
    FyLayout F;
    if (!fy_layout(workspace, n, &F)) return NCF_E_ARG;
    hipStream_t st = (hipStream_t)stream;
    const unsigned g = ep_grid(n, 8192);
    hipLaunchKernelGGL(fy_keys_kernel, dim3(g), dim3(EP_THREADS), 0, st, words, n, F.keys, F.P);
    size_t sb = F.sort_bytes;
    if (rocprim::radix_sort_pairs(F.sort_tmp, sb, F.keys, F.keys_sorted, rocprim::counting_iterator<int32_t>(0),
                                  F.steps_sorted, (size_t)n, 0, fy_key_bits(n), st) != hipSuccess)
        return NCF_E_LAUNCH;
    hipLaunchKernelGGL(fy_runs_kernel, dim3(g), dim3(EP_THREADS), 0, st, F.keys_sorted, F.steps_sorted, n, F.P, F.K);
    hipLaunchKernelGGL(fy_final_kernel, dim3(g), dim3(EP_THREADS), 0, st, words, n, F.P, F.K, perm);
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
