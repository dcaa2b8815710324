// mrnnt_internal.h -- device problem descriptor and kernel launchers shared by the host code
// (mrnnt_capi.cpp) and the kernels (mrnnt_kernels.hip). Not installed; not part of the ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mrnnt {

// Everything a kernel needs, passed by value as a kernel argument.
// Row r = (b, t, s) lives at row_off[b] + t*(S_b+1) + s; column (b, t) at col_off[b] + t.
struct DevProblem {
    const float *acts;          // [N, V]
    const int *labels;          // [B, label_stride]
    int64_t label_stride;
    const int *T;               // [B]
    const int *S;               // [B]
    const int64_t *row_off;     // [B+1] (workspace, built by the setup kernel)
    const int64_t *col_off;     // [B+1]
    const int *min_s;           // [cols] alignment band (nullptr = unrestricted)
    const int *max_s;           // [cols]
    int B, V, blank;
    int64_t num_cols;           // sum_b T_b
    float *den;                 // [N]  log-softmax denominator  -max - log sum exp(z - max)
    double *lpb;                // [N]  z[r, blank] + den[r]
    double *lpe;                // [N]  z[r, label(s)] + den[r]   (s < S)
    double *alpha;              // [N]  alpha(t, s), masked cells = -inf
    double *beta;               // [N]  beta(t, s)
    double *ll;                 // [B]  alpha(T-1, S)
    double *llb;                // [B]  beta(0, 0)
};

// Launch-shape knobs (experiment hook: mrnnt_tune in mrnnt_capi.cpp). Defaults are the tuned values.
struct Tuning {
    int softmax_variant = 2;  // 0 = row-at-a-time, 1 = software-pipelined, 2 = two rows per wave (V >= 768)
    int grad_variant = 0;     // 0 = row-at-a-time, 1 = software-pipelined, 2 = two rows per wave (V >= 768)
    int softmax_grid_per_cu = 0;  // workgroups (of 4 waves) per CU; 0 = one workgroup per lattice column
    int grad_grid_per_cu = 32;    // same for the gradient kernel
    int nt_store = 1;         // nontemporal stores of grads
    int nt_load = 1;          // nontemporal loads of acts (both streaming kernels)
    int dp_variant = 1;       // 0 = one wave/direction (shuffles), 1 = four waves (DPP + LDS), 2 = one wave (DPP)
};
Tuning &tuning();

// Kernel-family ids for the profiling counters (mrnnt_profile_read order).
enum KernelId { K_BAND = 0, K_SOFTMAX = 1, K_DP = 2, K_GRAD = 3, K_SETUP = 4, K_COUNT = 5 };

hipError_t launch_setup(const int *T, const int *S, int B, int64_t *row_off, int64_t *col_off, hipStream_t stream);
hipError_t launch_align(const DevProblem &p, const int *alignment, int64_t align_stride, int align_blank,
                        int max_shift, int *mtmp, int *min_s, int *max_s, hipStream_t stream);
hipError_t launch_softmax(const DevProblem &p, int grid, hipStream_t stream);
hipError_t launch_dp(const DevProblem &p, int S_max, int with_beta, float *costs, hipStream_t stream);
hipError_t launch_grad(const DevProblem &p, const float *scale, float *grads, int grid, hipStream_t stream);
hipError_t launch_synth(float *out, int64_t begin, int64_t count, uint64_t seed, int normal, hipStream_t stream);

// Largest S+1 the DP kernel instantiations cover (64 lanes x 32 cells per lane).
constexpr int kMaxLabelsPlusOne = 64 * 32;
// Padding (elements) around the lp arrays so the DP's whole-wave row loads never leave the allocation.
constexpr int64_t kLpPad = 64 * 32 + 64;

}  // namespace mrnnt
