// Ceiling probe of the embedding access pattern (bench.py `roofline_cache`).
//
// The fused step's memory side is a gather of the four embedding rows of every
// batch row (Ug[u], Ig[i], Um[u], Im[i]: models.py:108-112) and the float-atomic
// scatter-add of their gradients into the same rows (embedding_dense_backward,
// train_neumf.py:114).  At ml-1m the tables (3.1 MB) sit in L2 / the MALL, so the
// HBM roofline says little about them; this probe measures what the chip does with
// exactly that pattern and nothing else -- the same packed rows, the same tables,
// 16-byte row loads and per-float atomics, no arithmetic -- so a step's gather +
// scatter rate can be put against a measured cache ceiling.  Modes: 1 gather only,
// 2 scatter only, 3 both (each row's values gathered, then added back).
#include "ncf_common.h"
#include "ncf_kernels.h"

namespace ncf {

struct ProbeArgs {
    const float* prm;
    float* grads;
    float* sink;  // one float per thread (keeps the gathers live)
    const uint64_t* rows;
    int64_t n;
    int64_t ug, ig, um, im;
    int f, dm, mode;
};

// One thread per 16-byte piece of a row's four embedding rows: the pieces of a batch
// row are consecutive threads (E4 = (2f + 2dm) / 4 of them), so each table row is one
// contiguous run of lanes -- the step kernel's coalescing.
__global__ __launch_bounds__(256) void probe_gs_kernel(ProbeArgs a) {
    const int e4n = (2 * a.f + 2 * a.dm) / 4;
    const int64_t total = a.n * e4n;
    f4 acc = f4{0.f, 0.f, 0.f, 0.f};
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = q / e4n;
        const int e = (int)(q - r * e4n) * 4;
        const uint64_t pr = a.rows[r];
        const int64_t u = (int64_t)(uint32_t)pr, it = (int64_t)((pr >> 32) & 0x7fffffffu);
        int64_t off;
        if (e < a.f) off = a.ug + u * a.f + e;
        else if (e < 2 * a.f) off = a.ig + it * a.f + (e - a.f);
        else if (e < 2 * a.f + a.dm) off = a.um + u * a.dm + (e - 2 * a.f);
        else off = a.im + it * a.dm + (e - 2 * a.f - a.dm);
        f4 v = f4{1e-30f, 1e-30f, 1e-30f, 1e-30f};
        if (a.mode & 1) {
            v = *reinterpret_cast<const f4*>(a.prm + off);
            acc.x += v.x;
            acc.y += v.y;
            acc.z += v.z;
            acc.w += v.w;
        }
        if (a.mode & 2) {
            atomicAdd(a.grads + off, v.x);
            atomicAdd(a.grads + off + 1, v.y);
            atomicAdd(a.grads + off + 2, v.z);
            atomicAdd(a.grads + off + 3, v.w);
        }
    }
    if (a.mode & 1) a.sink[(int64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
}

}  // namespace ncf

using namespace ncf;

extern "C" int ncf_probe_gather_scatter(const ncf_layout* lay, const float* params, float* grads, float* sink,
                                        const uint64_t* rows, int64_t n, int mode, void* stream) {
    if (!lay || !params || !grads || !rows || n <= 0 || mode < 1 || mode > 3) return NCF_E_ARG;
    if ((mode & 1) && !sink) return NCF_E_ARG;
    const int f = lay->factor_num, dm = f << (lay->num_layers - 1);
    if (f % 4 || lay->model_type != NCF_MODEL_NEUMF) return NCF_E_UNSUPPORTED;
    ProbeArgs a;
    a.prm = params;
    a.grads = grads;
    a.sink = sink;
    a.rows = rows;
    a.n = n;
    a.ug = lay->ug;
    a.ig = lay->ig;
    a.um = lay->um;
    a.im = lay->im;
    a.f = f;
    a.dm = dm;
    a.mode = mode;
    hipLaunchKernelGGL(probe_gs_kernel, dim3(NCF_PROBE_BLOCKS), dim3(256), 0, (hipStream_t)stream, a);
    return hipGetLastError() == hipSuccess ? NCF_OK : NCF_E_LAUNCH;
}
