// gpu_ref_client.cpp -- reference-API GPU client compiled against THIS repository's headers (include/) and linked
// against libmonotonic_rnnt_amd.so: it drives GpuRNNTWorkspaceManager<float> + GpuRNNTComputer<float> the way the
// reference's pytorch_binding/monotonic_rnnt.cu:81-152 does, then reads the workspace back through every public
// host getter of the reference's manager (gpu_workspace_manager.h:87-190), as the reference's own computer and debug
// paths call them (gpu_rnnt.h:28-35,53-54,118-119,133,166,180), and reads the manager's public data members (:58-85)
// the way the reference's own computer reads wm.ll_forward / wm.denom on the device (gpu_rnnt.h:105-229), checking
// them against the getters. tests/test_ref_client.py compares the read-backs with the golden denom_f64 / alpha_f64 /
// beta_f64 of the reference itself.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "gpu_rnnt.h"
#include "gpu_workspace_manager.h"

template <typename T>
static T *to_gpu(const T *h, size_t n) {
    T *p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(1, n) * sizeof(T)) != hipSuccess) return nullptr;
    if (n && hipMemcpy(p, h, n * sizeof(T), hipMemcpyHostToDevice) != hipSuccess) return nullptr;
    return p;
}

template <typename T>
static int put(const std::vector<T> &v, T *out, size_t expect) {
    if (!out) return 0;
    if (v.size() != expect) return 1;
    std::copy(v.begin(), v.end(), out);
    return 0;
}

template <typename T>
static std::vector<T> from_gpu(const T *d, size_t n) {
    std::vector<T> h(n);
    if (!d || (n && hipMemcpy(h.data(), d, n * sizeof(T), hipMemcpyDeviceToHost) != hipSuccess)) return {};
    return h;
}

template <typename T>
static int same(const std::vector<T> &a, const std::vector<T> &b) {
    return a.size() != b.size() || std::memcmp(a.data(), b.data(), a.size() * sizeof(T)) != 0;
}

static int check_members(GpuRNNTWorkspaceManager<float> &wm, int B, int V, size_t N, int T_max, bool grads) {
    int bad = 0;
    bad += wm.workspace_ == nullptr || wm.B_h != B || wm.V_h != V || wm.acts == nullptr || wm.labels == nullptr;
    bad += same(from_gpu(wm.denom, N), wm.denom_host());
    bad += same(from_gpu(wm.alphas, N), wm.alphas_host());
    bad += same(from_gpu(wm.ll_forward, (size_t)B), wm.ll_forward_host());
    if (grads) {
        bad += same(from_gpu(wm.betas, N), wm.betas_host());
        bad += same(from_gpu(wm.ll_backward, (size_t)B), wm.ll_backward_host());
    }
    bad += same(from_gpu(wm.min_allowed_s, (size_t)B * T_max), wm.min_allowed_s_host());
    bad += same(from_gpu(wm.max_allowed_s, (size_t)B * T_max), wm.max_allowed_s_host());
    bad += same(from_gpu(wm.var_start_offsets, (size_t)B), wm.var_start_offsets_host());
    bad += same(from_gpu(wm.denom_start_indices, (size_t)B), wm.var_start_offsets_host());
    const std::vector<int> c = {B, V, wm.S_max_host(), T_max};
    auto one = [](const int *d) {
        const std::vector<int> h = from_gpu(d, 1);
        return h.empty() ? -1 : h[0];
    };
    const std::vector<int> got = {one(wm.B), one(wm.V), one(wm.S_max), one(wm.T_max)};
    bad += c != got;
    bad += same(from_gpu(wm.T, (size_t)B), wm.T_host()) + same(from_gpu(wm.S, (size_t)B), wm.S_host());
    return bad;
}

extern "C" {

// sizes: N = sum_b T_b (S_b+1) rows; labels [B, max S] (the reference's stride), alignment [B, max T] or NULL.
// Outputs (host, any may be NULL): costs [B], grads [N, V] (NULL: cost() only), denom / alphas / betas [N],
// ll_fwd / ll_bwd [B], min_s / max_s [B * max T], var_off [B], sizes[4] = {num_denoms, num_fwd_bwd_var_positions,
// S_max, T_max}, acts_back [N * V]. Returns the number of failed calls / size mismatches (0 = all good).
int client_gpu_getters(const float *acts, const int *labels, int B, const int *T, const int *S, int V, int blank,
                       const int *alignment, int max_shift, float *costs, float *grads, float *denom, float *alphas,
                       float *betas, float *ll_fwd, float *ll_bwd, int *min_s, int *max_s, int *var_off, int *sizes,
                       float *acts_back) {
    int64_t N = 0;
    int S_max = 0, T_max = 0;
    for (int b = 0; b < B; ++b) {
        N += (int64_t)T[b] * (S[b] + 1);
        S_max = std::max(S_max, S[b]);
        T_max = std::max(T_max, T[b]);
    }
    float *d_acts = to_gpu(acts, (size_t)N * V);
    int *d_labels = to_gpu(labels, (size_t)B * S_max);
    int *d_T = to_gpu(T, (size_t)B), *d_S = to_gpu(S, (size_t)B);
    int *d_align = alignment ? to_gpu(alignment, (size_t)B * T_max) : nullptr;
    float *d_grads = nullptr;
    if (grads) (void)hipMalloc(&d_grads, (size_t)N * V * sizeof(float));
    int bad = 0;
    hipStream_t stream;
    (void)hipStreamCreateWithFlags(&stream, hipStreamNonBlocking);
    {
        GpuRNNTWorkspaceManager<float> wm(d_acts, d_labels, B, d_T, d_S, V);
        bad += wm.create_workspace() != RNNT_STATUS_SUCCESS;
        if (d_align) wm.restrict_to_alignment(d_align, max_shift, blank);
        GpuRNNTComputer<float> computer(wm, blank, stream);
        std::vector<float> c(B);
        bad += (grads ? computer.cost_and_grad(c.data(), d_grads) : computer.cost(c.data())) != RNNT_STATUS_SUCCESS;
        if (costs) std::copy(c.begin(), c.end(), costs);
        if (grads) bad += hipMemcpy(grads, d_grads, (size_t)N * V * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess;
        const size_t n = (size_t)N;
        bad += put(wm.denom_host(), denom, n);
        bad += put(wm.alphas_host(), alphas, n);
        if (grads) bad += put(wm.betas_host(), betas, n);
        bad += put(wm.ll_forward_host(), ll_fwd, (size_t)B);
        if (grads) bad += put(wm.ll_backward_host(), ll_bwd, (size_t)B);
        bad += put(wm.min_allowed_s_host(), min_s, (size_t)B * T_max);
        bad += put(wm.max_allowed_s_host(), max_s, (size_t)B * T_max);
        bad += put(wm.var_start_offsets_host(), var_off, (size_t)B);
        bad += put(wm.acts_host(), acts_back, n * V);
        if (sizes) {
            sizes[0] = wm.num_denoms();
            sizes[1] = wm.num_fwd_bwd_var_positions();
            sizes[2] = wm.S_max_host();
            sizes[3] = wm.T_max_host();
        }
        bad += wm.B_host() != B || wm.V_host() != V;
        // the reference's public data members (gpu_workspace_manager.h:58-85): device pointers a client kernel
        // reads after the call -- the same values as the getters, in the same layout
        bad += check_members(wm, B, V, (size_t)N, T_max, grads != nullptr);
        const std::vector<int> Th = wm.T_host(), Sh = wm.S_host();
        bad += !std::equal(Th.begin(), Th.end(), T) || !std::equal(Sh.begin(), Sh.end(), S);
        wm.free_workspace();
    }
    (void)hipStreamDestroy(stream);
    for (void *p : {(void *)d_acts, (void *)d_labels, (void *)d_T, (void *)d_S, (void *)d_align, (void *)d_grads})
        if (p) (void)hipFree(p);
    return bad;
}

// The band members are OUTPUT-only here (include/gpu_workspace_manager.h): a client that writes
// its own band into wm.min_allowed_s / wm.max_allowed_s before cost() gets the unrestricted result (restrict_to_
// alignment is the way to restrict), and after the call the members hold the band of that computation ([0, S_b]).
// Returns the number of mismatches (0 = the pinned behaviour).
int client_band_members_output_only(const float *acts, const int *labels, int B, const int *T, const int *S, int V,
                                    int blank) {
    int64_t N = 0;
    int S_max = 0, T_max = 0;
    for (int b = 0; b < B; ++b) {
        N += (int64_t)T[b] * (S[b] + 1);
        S_max = std::max(S_max, S[b]);
        T_max = std::max(T_max, T[b]);
    }
    float *d_acts = to_gpu(acts, (size_t)N * V);
    int *d_labels = to_gpu(labels, (size_t)B * S_max);
    int *d_T = to_gpu(T, (size_t)B), *d_S = to_gpu(S, (size_t)B);
    int bad = 0;
    hipStream_t stream;
    (void)hipStreamCreateWithFlags(&stream, hipStreamNonBlocking);
    std::vector<float> plain(B), written(B);
    {
        GpuRNNTWorkspaceManager<float> wm(d_acts, d_labels, B, d_T, d_S, V);
        bad += wm.create_workspace() != RNNT_STATUS_SUCCESS;
        GpuRNNTComputer<float> computer(wm, blank, stream);
        bad += computer.cost(plain.data()) != RNNT_STATUS_SUCCESS;
        wm.free_workspace();
    }
    {
        GpuRNNTWorkspaceManager<float> wm(d_acts, d_labels, B, d_T, d_S, V);
        bad += wm.create_workspace() != RNNT_STATUS_SUCCESS;
        // a band of one label position per frame (min = max = 0): under the reference's computer this would leave
        // only the path that emits nothing, and an infinite cost wherever S_b > 0
        const std::vector<int> zero((size_t)B * T_max, 0);
        bad += hipMemcpy(wm.min_allowed_s, zero.data(), zero.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess;
        bad += hipMemcpy(wm.max_allowed_s, zero.data(), zero.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess;
        GpuRNNTComputer<float> computer(wm, blank, stream);
        bad += computer.cost(written.data()) != RNNT_STATUS_SUCCESS;
        bad += same(plain, written);  // the write was not an input
        std::vector<int> emx((size_t)B * T_max);
        for (int b = 0; b < B; ++b) std::fill_n(emx.begin() + (size_t)b * T_max, T_max, S[b]);
        bad += same(from_gpu(wm.min_allowed_s, zero.size()), zero);  // overwritten with this computation's band
        bad += same(from_gpu(wm.max_allowed_s, emx.size()), emx);
        wm.free_workspace();
    }
    (void)hipStreamDestroy(stream);
    for (void *p : {(void *)d_acts, (void *)d_labels, (void *)d_T, (void *)d_S})
        if (p) (void)hipFree(p);
    return bad;
}
}
