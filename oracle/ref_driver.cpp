// ref_driver.cpp -- a thin C-ABI driver around the REFERENCE's own CPU computer, compiled from the
// reference sources where they lie (/root/reference/include, never copied) into oracle/_ref/.
//
// TEST INFRASTRUCTURE ONLY: used to (1) generate the golden vectors in tests/golden/ and pin the
// restatement in rnnt_oracle.c, and (2) as the "reference" CPU baseline timed by bench.py.
//
// It drives CpuRNNTWorkspaceManager<dtype> + CpuRNNTComputer<dtype> exactly the way the reference's
// pytorch_binding/monotonic_rnnt.cu:16-77 does (create_workspace -> [restrict_to_alignment] ->
// cost_and_grad / cost -> free_workspace).  Inspection outputs (denominators, alpha, beta) are read
// back through the manager's public getters.
//
// The reference uses 32-bit act offsets (cpu_workspace_manager.h:48,125): callers must keep
// sum_b T_b (S_b+1) V < 2^31 per call; this driver refuses larger calls with status 2.
#include <cstdint>
#include <cstring>
#include <vector>

#include "cpu_rnnt.h"
#include "cpu_workspace_manager.h"

template <typename dtype>
static int run(const float *acts_f, const int *labels, int B, const int *T, const int *S, int V, int blank,
               const int *alignment, int max_shift, int align_blank, dtype *costs, dtype *grads, dtype *denom_out,
               dtype *alpha_out, dtype *beta_out, int num_threads) {
    int64_t rows = 0;
    for (int b = 0; b < B; ++b) rows += (int64_t)T[b] * (S[b] + 1);
    if (rows * (int64_t)V >= (int64_t)1 << 31) return 2;

    std::vector<dtype> acts_conv;
    const dtype *acts;
    if (sizeof(dtype) == sizeof(float)) {
        acts = reinterpret_cast<const dtype *>(acts_f);
    } else {
        acts_conv.assign(acts_f, acts_f + rows * V);
        acts = acts_conv.data();
    }

    CpuRNNTWorkspaceManager<dtype> wm(acts, labels, B, T, S, V);
    RNNTStatus st = wm.create_workspace();
    if (st != RNNT_STATUS_SUCCESS) return (int)st;
    if (alignment) wm.restrict_to_alignment(alignment, max_shift, align_blank);
    {
        CpuRNNTComputer<dtype> computer(wm, blank, num_threads);
        st = grads ? computer.cost_and_grad(costs, grads) : computer.cost(costs);
    }
    if (st == RNNT_STATUS_SUCCESS) {
        int64_t r = 0;
        for (int b = 0; b < B; ++b)
            for (int t = 0; t < T[b]; ++t)
                for (int s = 0; s <= S[b]; ++s, ++r) {
                    if (denom_out) denom_out[r] = wm.get_denom(b, t, s);
                    if (alpha_out) alpha_out[r] = wm.get_alpha(b, t, s);
                    if (beta_out) beta_out[r] = grads ? wm.get_beta(b, t, s) : -INFINITY;
                }
    }
    wm.free_workspace();
    return (int)st;
}

extern "C" {

int ref_rnnt_f32(const float *acts, const int *labels, int B, const int *T, const int *S, int V, int blank,
                 const int *alignment, int max_shift, int align_blank, float *costs, float *grads, float *denom_out,
                 float *alpha_out, float *beta_out, int num_threads) {
    return run<float>(acts, labels, B, T, S, V, blank, alignment, max_shift, align_blank, costs, grads, denom_out,
                      alpha_out, beta_out, num_threads);
}

int ref_rnnt_f64(const float *acts, const int *labels, int B, const int *T, const int *S, int V, int blank,
                 const int *alignment, int max_shift, int align_blank, double *costs, double *grads,
                 double *denom_out, double *alpha_out, double *beta_out, int num_threads) {
    return run<double>(acts, labels, B, T, S, V, blank, alignment, max_shift, align_blank, costs, grads, denom_out,
                       alpha_out, beta_out, num_threads);
}
}
