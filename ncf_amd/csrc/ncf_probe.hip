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

// Gather: one thread per 16-byte piece of a row's four embedding rows (E4 = (2f +
// 2dm) / 4 consecutive threads per batch row: each table row one contiguous run of
// lanes, the step kernel's coalescing).  Scatter: one thread per float, so one atomic
// wave-instruction adds 64 consecutive floats of a row (the step's row-contiguous
// atomics; it also sums runs of equal items first, which this probe does not).
__global__ __launch_bounds__(256) void probe_gs_kernel(ProbeArgs a) {
    const int en = 2 * a.f + 2 * a.dm;
    const int e4n = en / 4;
    const int64_t nt = (int64_t)gridDim.x * blockDim.x;
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    auto offset = [&](int64_t r, int e) {
        const uint64_t pr = a.rows[r];
        const int64_t u = (int64_t)(uint32_t)pr, it = (int64_t)((pr >> 32) & 0x7fffffffu);
        if (e < a.f) return a.ug + u * a.f + e;
        if (e < 2 * a.f) return a.ig + it * a.f + (e - a.f);
        if (e < 2 * a.f + a.dm) return a.um + u * a.dm + (e - 2 * a.f);
        return a.im + it * a.dm + (e - 2 * a.f - a.dm);
    };
    if (a.mode & 1) {
        f4 acc = f4{0.f, 0.f, 0.f, 0.f};
        for (int64_t q = t0; q < a.n * e4n; q += nt) {
            const int64_t r = q / e4n;
            const f4 v = *reinterpret_cast<const f4*>(a.prm + offset(r, (int)(q - r * e4n) * 4));
            acc.x += v.x;
            acc.y += v.y;
            acc.z += v.z;
            acc.w += v.w;
        }
        a.sink[t0] = acc.x + acc.y + acc.z + acc.w;
    }
    if (a.mode & 2) {
        for (int64_t q = t0; q < a.n * en; q += nt) {
            const int64_t r = q / en;
            atomicAdd(a.grads + offset(r, (int)(q - r * en)), 1e-30f);
        }
    }
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
