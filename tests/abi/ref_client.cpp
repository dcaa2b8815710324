// ref_client.cpp -- reference-API client code compiled against THIS repository's headers (include/) and linked
// against libmonotonic_rnnt_amd.so: the body of oracle/ref_driver.cpp (which drives the reference's own
// CpuRNNTComputer exactly as the reference's pytorch_binding/monotonic_rnnt.cu:16-77 does: create_workspace ->
// [restrict_to_alignment] -> cost_and_grad / cost -> get_denom / get_alpha / get_beta -> free_workspace), unchanged
// except that only the float instantiation exists here (the reference's entry point accepts only float,
// src/rnnt_entrypoint.cpp:23). It proves a reference C++ user compiles and runs against this library as-is;
// tests/test_ref_client.py checks its outputs against the golden vectors of the reference itself.
#include <cmath>
#include <cstdio>
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

// The rest of the reference's public manager interface (cpu_workspace_manager.h:63-205), exercised on the state
// the run above leaves: returns 0 when every accessor agrees with what the computation used.
static int accessors(const float *acts, const int *labels, int B, const int *T, const int *S, int V, int blank,
                     const int *alignment, int max_shift) {
    CpuRNNTWorkspaceManager<float> wm(acts, labels, B, T, S, V);
    if (wm.create_workspace() != RNNT_STATUS_SUCCESS) return 1;
    if (alignment) wm.restrict_to_alignment(alignment, max_shift, blank);
    std::vector<float> costs(B);
    CpuRNNTComputer<float> computer(wm, blank, 0);
    if (computer.cost(costs.data()) != RNNT_STATUS_SUCCESS) return 2;
    int bad = 0, S_max = 0;
#define CHECK(cond)                                                                   \
    do {                                                                              \
        if (!(cond)) {                                                                \
            ++bad;                                                                    \
            std::fprintf(stderr, "accessor check failed (b=%d): %s\n", b, #cond);    \
        }                                                                             \
    } while (0)
    for (int b = 0; b < B; ++b) S_max = S[b] > S_max ? S[b] : S_max;
    int64_t row = 0;
    for (int b = 0; b < B; ++b) {
        CHECK(wm.T(b) == T[b] && wm.S(b) == S[b]);
        for (int s = 0; s < S[b]; ++s) CHECK(wm.label(b, s) == labels[b * S_max + s]);
        for (int t = 0; t < T[b]; ++t) {
            for (int s = 0; s <= S[b]; ++s, ++row)
                for (int v = 0; v < V; v += (V > 3 ? V / 3 : 1)) {
                    CHECK(wm.act_index(b, t, s, v) == row * V + v);
                    CHECK(wm.act(b, t, s, v) == acts[row * V + v]);
                }
            // alpha outside [alpha_s_min, alpha_s_max] is -inf, inside finite (a feasible band)
            for (int s = 0; s <= S[b]; ++s) {
                const bool in = s >= wm.alpha_s_min(b, t) && s <= wm.alpha_s_max(b, t);
                CHECK(in || std::isinf(wm.get_alpha(b, t, s)));
            }
            CHECK(wm.beta_s_min(b, t) >= 0 && wm.beta_s_max(b, t) <= t);
        }
        // virtual boundaries (cpu_workspace_manager.h:161-205)
        CHECK(wm.get_alpha(b, -1, 0) == 0.0f);
        CHECK(std::isinf(wm.get_alpha(b, -1, 1)) && wm.get_alpha(b, -1, 1) < 0);
        CHECK(std::isinf(wm.get_alpha(b, 0, -1)) && wm.get_alpha(b, 0, -1) < 0);
        CHECK(wm.get_beta(b, T[b], S[b]) == 0.0f);
        CHECK(std::isinf(wm.get_beta(b, 0, S[b] + 1)) && wm.get_beta(b, 0, S[b] + 1) < 0);
        // -log p = -alpha(T-1, S) (cpu_rnnt.h:180, :82)
        if (std::isfinite(costs[b]))
            CHECK(std::fabs(-wm.get_alpha(b, T[b] - 1, S[b]) - costs[b]) <= 1e-4f * std::fmax(1.0f, std::fabs(costs[b])));
        else
            CHECK(!std::isfinite(wm.get_alpha(b, T[b] - 1, S[b])));
        // set_* / get_* round trips
        const float d0 = wm.get_denom(b, 0, 0);
        wm.set_denom(b, 0, 0, 1.25f);
        CHECK(wm.get_denom(b, 0, 0) == 1.25f);
        wm.set_denom(b, 0, 0, d0);
        wm.set_alpha(b, 0, 0, -2.5f);  // (a cell outside the alignment band reads -inf whatever is stored)
        CHECK(wm.get_alpha(b, 0, 0) == (wm.alpha_s_min(b, 0) <= 0 ? -2.5f : -INFINITY));
        wm.set_beta(b, 0, 0, -3.5f);
        CHECK(wm.get_beta(b, 0, 0) == -3.5f);
    }
    if (wm.B() != B || wm.V() != V) ++bad;
#undef CHECK
    wm.free_workspace();
    return bad;
}

extern "C" {

int client_rnnt_f32(const float *acts, const int *labels, int B, const int *T, const int *S, int V, int blank,
                    const int *alignment, int max_shift, int align_blank, float *costs, float *grads, float *denom_out,
                    float *alpha_out, float *beta_out, int num_threads) {
    return run<float>(acts, labels, B, T, S, V, blank, alignment, max_shift, align_blank, costs, grads, denom_out,
                      alpha_out, beta_out, num_threads);
}

int client_accessors(const float *acts, const int *labels, int B, const int *T, const int *S, int V, int blank,
                     const int *alignment, int max_shift) {
    return accessors(acts, labels, B, T, S, V, blank, alignment, max_shift);
}
}
