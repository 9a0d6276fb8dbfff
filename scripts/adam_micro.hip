// Microbenchmark (not product code): the latency floor of the dense embedding Adam
// pass at the C3 / C2 / C4 table sizes on MI355X.  Variants:
//   copy   : read g, m, v, p (one float4 each per thread), write m, v, p, g  (no math)
//   adam   : the same with adam arithmetic, scalars passed in (no pow)
//   adampow: adam + thread 0 computes the double pow scalars, block barrier
//   adam2  : adam, 2 float4 per thread (half the blocks)
// Each timed as 200 back-to-back launches between two events, and as a 200-node graph.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/adam_micro scripts/adam_micro.hip
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

typedef float4 f4;

__device__ __forceinline__ void adam1(float& p, float& m, float& v, float g, float w1, float b2, float omb2,
                                      float bc2s, float eps, float ns) {
#pragma clang fp contract(off)
    m = fmaf(w1, g - m, m);
    v = v * b2 + omb2 * g * g;
    const float den = sqrtf(v) / bc2s + eps;
    p = p + ns * m / den;
}

template <int MODE, int PER>
__global__ __launch_bounds__(256) void k_adam(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                               float* __restrict__ v, long n4, long t, float ns_in, float bc_in) {
    __shared__ float sc[2];
    if (MODE == 3) return;
    const long base = ((long)blockIdx.x * blockDim.x * PER) + threadIdx.x;
    f4 pp[PER], gg[PER], mm[PER], vv[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const long q = base + (long)k * blockDim.x;
        if (q < n4) {
            pp[k] = reinterpret_cast<f4*>(p)[q];
            gg[k] = reinterpret_cast<f4*>(g)[q];
            mm[k] = reinterpret_cast<f4*>(m)[q];
            vv[k] = reinterpret_cast<f4*>(v)[q];
        }
    }
    float ns = ns_in, bc = bc_in;
    if (MODE == 2) {
        if (threadIdx.x == 0) {
            sc[0] = (float)(-(1e-3 / (1.0 - pow(0.9, (double)t))));
            sc[1] = (float)sqrt(1.0 - pow(0.999, (double)t));
        }
        __syncthreads();
        ns = sc[0];
        bc = sc[1];
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const long q = base + (long)k * blockDim.x;
        if (q >= n4) continue;
        if (MODE != 0) {
            adam1(pp[k].x, mm[k].x, vv[k].x, gg[k].x, 0.1f, 0.999f, 0.001f, bc, 1e-8f, ns);
            adam1(pp[k].y, mm[k].y, vv[k].y, gg[k].y, 0.1f, 0.999f, 0.001f, bc, 1e-8f, ns);
            adam1(pp[k].z, mm[k].z, vv[k].z, gg[k].z, 0.1f, 0.999f, 0.001f, bc, 1e-8f, ns);
            adam1(pp[k].w, mm[k].w, vv[k].w, gg[k].w, 0.1f, 0.999f, 0.001f, bc, 1e-8f, ns);
        } else {
            pp[k].x += gg[k].x; mm[k].y += gg[k].y; vv[k].z += gg[k].z;
        }
        reinterpret_cast<f4*>(p)[q] = pp[k];
        reinterpret_cast<f4*>(m)[q] = mm[k];
        reinterpret_cast<f4*>(v)[q] = vv[k];
        reinterpret_cast<f4*>(g)[q] = f4{0.f, 0.f, 0.f, 0.f};
    }
}

template <int MODE, int PER>
static void run(const char* name, float* p, float* g, float* m, float* v, long n4, hipStream_t st) {
    const long per_block = 256L * PER;
    const unsigned grid = (unsigned)((n4 + per_block - 1) / per_block);
    const int R = 200;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 20; ++i) k_adam<MODE, PER><<<grid, 256, 0, st>>>(p, g, m, v, n4, i + 1, -1e-3f, 0.5f);
    CK(hipEventRecord(e0, st));
    for (int i = 0; i < R; ++i) k_adam<MODE, PER><<<grid, 256, 0, st>>>(p, g, m, v, n4, i + 1, -1e-3f, 0.5f);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms_eager;
    CK(hipEventElapsedTime(&ms_eager, e0, e1));
    hipGraph_t gr;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int i = 0; i < R; ++i) k_adam<MODE, PER><<<grid, 256, 0, st>>>(p, g, m, v, n4, i + 1, -1e-3f, 0.5f);
    CK(hipStreamEndCapture(st, &gr));
    CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    CK(hipEventRecord(e0, st));
    CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms_graph;
    CK(hipEventElapsedTime(&ms_graph, e0, e1));
    const double bytes = (double)n4 * 16 * 8;
    printf("{\"variant\": \"%s\", \"n_floats\": %ld, \"grid\": %u, \"us_eager\": %.2f, \"us_graph\": %.2f, "
           "\"GBps_graph\": %.0f}\n",
           name, n4 * 4, grid, ms_eager * 1e3 / R, ms_graph * 1e3 / R, bytes / (ms_graph * 1e-3 / R) / 1e9);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(gr));
}

int main() {
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const long sizes[] = {390000, 780000, 3120000, 13200000};  // C2, C3, 4x C3, C4 embedding floats
    for (long nf : sizes) {
        const long n4 = nf / 4;
        float *p, *g, *m, *v;
        CK(hipMalloc(&p, n4 * 16));
        CK(hipMalloc(&g, n4 * 16));
        CK(hipMalloc(&m, n4 * 16));
        CK(hipMalloc(&v, n4 * 16));
        CK(hipMemset(p, 0, n4 * 16));
        CK(hipMemset(g, 0, n4 * 16));
        CK(hipMemset(m, 0, n4 * 16));
        CK(hipMemset(v, 0, n4 * 16));
        run<3, 1>("empty", p, g, m, v, n4, st);
        run<0, 1>("copy", p, g, m, v, n4, st);
        run<1, 1>("adam", p, g, m, v, n4, st);
        run<2, 1>("adampow", p, g, m, v, n4, st);
        run<1, 2>("adam2", p, g, m, v, n4, st);
        run<1, 4>("adam4", p, g, m, v, n4, st);
        CK(hipFree(p));
        CK(hipFree(g));
        CK(hipFree(m));
        CK(hipFree(v));
    }
    return 0;
}
