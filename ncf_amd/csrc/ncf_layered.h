// Layered (unfused) NeuMF step: the path for shapes without a fused kernel.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ncf_hip.h"

namespace ncf {

constexpr int LYR_MAX_FACTOR = 256;  // predict kernel: <= 4 features per lane
// Factored layer 0: fact_expand_kernel (LDS-staged W0 half) up to this dm; wider
// (256, 512) the layered path expands with GEMMs (lyr_fact_dx / lyr_fact_dw0).
#ifndef NCF_FACT_LDS_DM  // experiment switch: a smaller value takes the GEMM expansion from there up
#define NCF_FACT_LDS_DM 128
#endif
constexpr int FACT_LDS_DM = NCF_FACT_LDS_DM;
constexpr int FACT_MAX_DM = 512;

static inline int64_t rup64(int64_t x) { return (x + 63) / 64 * 64; }

// Rows of the layered path's partial slab [rows][tower_len + 64]: blocks that add
// the same tower partials (weight-gradient row splits, predict blocks) spread their
// float atomics over the rows (block index mod rows) instead of queueing on one
// address; the reductions sum the rows in a fixed order.  As many rows as fit
// 4M floats, at most 16.
__host__ __device__ static inline int lyr_slab_rows(const ncf_layout* lay) {
    const int64_t stride = lay->tower_len + 64;
    int64_t r = ((int64_t)4 << 20) / stride;
    return (int)(r < 1 ? 1 : (r > 16 ? 16 : r));
}

struct LyrArgs {
    ncf_layout lay;
    const float* params;
    float* grads;            // train: dense gradient buffer (embedding scatter targets)
    const uint64_t* rows;    // packed rows (NCF_ROW_PACK)
    const int64_t* uorder;   // train, factored layer 0: ncf_user_order of rows (nullptr: per-row user atomics)
    const float* dlogit;     // NCF_DZ_DLOGIT: dL/dlogit per row
    ncf_step_ctl* ctl;       // train: batch selection; nullptr = forward over fwd_n rows
    int64_t batch_global, fwd_n;
    int world, rank, dz_mode;
    float kd_wt, kd_wr, kd_temp;  // NCF_DZ_KD: task / response weights, temperature; dlogit = teacher logits
    float* slab;             // lyr_slab_rows() rows [tower_len + 64] of tower/predict partials (+ loss)
    float* logits_out;       // optional per-row logits
    int64_t fact_part_floats;  // train: >= 0 factored layer 0 (that many floats of dW0 partials
                               // follow the slab row, filled by fact_expand_kernel); -1 per-row
    float* zero_p;             // train: the slab, zeroed by the step's first kernel (zero_n4 16-byte units)
    int64_t zero_n4;
};

// p[0 .. n) = 0 (n % 4 == 0, p 16-byte aligned) on stream st.
int launch_zero_f32(float* p, int64_t n, hipStream_t st);

// Workspace floats for `rows` rows per launch: slab row [+ dW0 partials + table
// projections (factored layer 0, fact_part_floats >= 0)] + activations [+ dY buffers].
int64_t lyr_workspace_floats(const ncf_layout* lay, int64_t rows, bool train, int64_t fact_part_floats);

// Factored layer 0: P = [Um W0[:, :DM]^T ; Im W0[:, DM:]^T] ((U + I) x DM floats at P),
// the per-step table projection the layered step's layer-0 forward gathers from; the
// launch also zeroes zero[0 .. zero_floats) (the step's slab; 16-byte aligned, % 4 == 0).
int lyr_launch_proj(const ncf_layout* lay, const float* params, float* P, float* zero, int64_t zero_floats,
                    hipStream_t st);

// Launch the layered forward (train = false) or forward + BCE + backward (train = true)
// over at most R rows; ws = lyr_workspace_floats(lay, R, train) floats.
int lyr_run(const LyrArgs& a, float* ws, int64_t R, bool train, hipStream_t st);

}  // namespace ncf
