// test_gpu_abi.cpp -- the reference's own GPU test program shape (tests/test_gpu.cu: 7 tests), written
// against this repository's headers and linked against libmonotonic_rnnt_amd.so. It exercises the C++
// surface a reference user links to: GpuRNNTWorkspaceManager<float> + GpuRNNTComputer<float> and the
// extern "C" compute_rnnt_loss entry point (src/rnnt_entrypoint.cpp). Returns 0 when every test passes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

#include "gpu_rnnt.h"
#include "gpu_workspace_manager.h"
#include "rnnt_entrypoint.h"

static const float kProbs[36] = {0.6, 0.3, 0.1, 0.7, 0.1, 0.2, 0.5, 0.1, 0.4, 0.5, 0.4, 0.1,
                                 0.5, 0.1, 0.4, 0.8, 0.1, 0.1, 0.4, 0.3, 0.3, 0.5, 0.1, 0.4,
                                 0.7, 0.2, 0.1, 0.8, 0.1, 0.1, 0.3, 0.1, 0.6, 0.8, 0.1, 0.1};
static const float kGrads[36] = {0.04, -0.14, 0.1, 0,    0,    0,     0,    0,     0,     0.13,  -0.19, 0.06,
                                 -0.04, 0.04, -0.01, 0,   0,    0,     0.06, -0.1,  0.04,  0.01,  0.07,  -0.08,
                                 -0.06, 0.04, 0.02,  0,   0,    0,     0.14, 0.05,  -0.19, -0.11, 0.05,  0.05};

template <typename T>
static T *to_gpu(const std::vector<T> &v) {
    T *p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(1, v.size()) * sizeof(T)) != hipSuccess) return nullptr;
    if (!v.empty() && hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice) != hipSuccess) return nullptr;
    return p;
}

static bool close(float a, float b, float tol = 1e-4f) { return std::fabs(a - b) < tol; }

static std::vector<float> toy_logits(int copies) {
    std::vector<float> l;
    for (int c = 0; c < copies; ++c)
        for (float p : kProbs) l.push_back(std::log(p));
    return l;
}

struct Buffers {
    float *acts;
    int *labels, *T, *S;
};

static Buffers upload(const std::vector<float> &acts, const std::vector<int> &labels, const std::vector<int> &T,
                      const std::vector<int> &S) {
    return Buffers{to_gpu(acts), to_gpu(labels), to_gpu(T), to_gpu(S)};
}

static void release(Buffers &b) {
    (void)hipFree(b.acts);
    (void)hipFree(b.labels);
    (void)hipFree(b.T);
    (void)hipFree(b.S);
}

// test_gpu.cu fwd_test / bwd_test / grads_test through GpuRNNTComputer
static bool toy_tests() {
    Buffers g = upload(toy_logits(1), {1, 2}, {4}, {2});
    GpuRNNTWorkspaceManager<float> wm(g.acts, g.labels, 1, g.T, g.S, 3);
    if (wm.create_workspace() != RNNT_STATUS_SUCCESS) return false;
    hipStream_t stream;
    (void)hipStreamCreate(&stream);
    GpuRNNTComputer<float> computer(wm, 0, stream);
    float cost_fwd = 0, cost_bwd = 0;
    bool ok = computer.cost(&cost_fwd) == RNNT_STATUS_SUCCESS;
    ok = ok && close(cost_fwd, -std::log(0.363f));
    float *grads;
    (void)hipMalloc(&grads, 36 * sizeof(float));
    ok = ok && computer.cost_and_grad(&cost_bwd, grads) == RNNT_STATUS_SUCCESS;
    ok = ok && close(cost_fwd, cost_bwd);
    std::vector<float> gh(36);
    (void)hipMemcpy(gh.data(), grads, 36 * sizeof(float), hipMemcpyDeviceToHost);
    for (int i = 0; i < 36; ++i) ok = ok && std::fabs(gh[i] - kGrads[i]) < 1e-2f;
    (void)hipFree(grads);
    wm.free_workspace();
    (void)hipStreamDestroy(stream);
    release(g);
    std::printf("toy fwd/bwd/grads: %s (cost %.6f)\n", ok ? "ok" : "FAIL", cost_fwd);
    return ok;
}

// test_gpu.cu multibatch_test through compute_rnnt_loss (the C entry point)
static bool multibatch_test() {
    std::vector<float> probs;
    const int rows0[4] = {0, 1, 3, 4};
    for (int r : rows0)
        for (int v = 0; v < 3; ++v) probs.push_back(kProbs[r * 3 + v]);
    for (float p : kProbs) probs.push_back(p);
    std::vector<float> logits(probs.size());
    std::transform(probs.begin(), probs.end(), logits.begin(), [](float p) { return std::log(p); });
    Buffers g = upload(logits, {1, 0, 1, 2}, {2, 4}, {1, 2});
    GpuRNNTWorkspaceManager<float> wm(g.acts, g.labels, 2, g.T, g.S, 3);
    size_t bytes = 0;
    bool ok = wm.get_workspace_size(&bytes) == RNNT_STATUS_SUCCESS && bytes > 0;
    void *ws = nullptr;
    (void)hipMalloc(&ws, bytes);
    wm.set_workspace(ws);
    RNNTOptions opt;
    opt.num_threads = 0;
    opt.stream = nullptr;
    opt.blank_label = 0;
    opt.loc = RNNT_GPU;
    float costs[2] = {0, 0};
    ok = ok && compute_rnnt_loss(wm, opt, costs, nullptr) == RNNT_STATUS_SUCCESS;
    ok = ok && close(costs[0], -std::log(0.39f)) && close(costs[1], -std::log(0.363f));
    float *grads;
    (void)hipMalloc(&grads, logits.size() * sizeof(float));
    float costs2[2] = {0, 0};
    ok = ok && compute_rnnt_loss(wm, opt, costs2, grads) == RNNT_STATUS_SUCCESS;
    ok = ok && close(costs[0], costs2[0]) && close(costs[1], costs2[1]);
    std::vector<float> gh(logits.size());
    (void)hipMemcpy(gh.data(), grads, gh.size() * sizeof(float), hipMemcpyDeviceToHost);
    const float exp0[12] = {-0.02, -0.08, 0.1, 0.0, 0.0, 0.0, 0.31, -0.37, 0.06, -0.19, 0.04, 0.15};
    for (int i = 0; i < 12; ++i) ok = ok && std::fabs(gh[i] - exp0[i]) < 1e-2f;
    for (int i = 0; i < 36; ++i) ok = ok && std::fabs(gh[12 + i] - kGrads[i]) < 1e-2f;
    // entry-point argument checks (src/rnnt_entrypoint.cpp:18-20, :41-46)
    ok = ok && compute_rnnt_loss(wm, opt, nullptr, nullptr) == RNNT_STATUS_INVALID_VALUE;
    RNNTOptions cpu = opt;
    cpu.loc = RNNT_CPU;
    ok = ok && compute_rnnt_loss(wm, cpu, costs, nullptr) == RNNT_STATUS_INVALID_VALUE;  // not a CPU manager
    (void)hipFree(grads);
    (void)hipFree(ws);
    release(g);
    std::printf("multibatch (compute_rnnt_loss): %s (%.6f %.6f)\n", ok ? "ok" : "FAIL", costs[0], costs[1]);
    return ok;
}

// test_gpu.cu infnan_test shape: T=50, S=10, V=15
static bool infnan_test() {
    const int T = 50, S = 10, V = 15;
    std::vector<float> acts(T * (S + 1) * V);
    unsigned x = 12345u;
    for (auto &a : acts) {
        x = x * 1664525u + 1013904223u;
        a = (x >> 8) * (1.0f / 16777216.0f);
    }
    std::vector<int> labels(S);
    for (int i = 0; i < S; ++i) labels[i] = 1 + (i * 7) % (V - 1);
    labels[S / 2] = labels[S / 2 + 1];
    labels[S / 2 - 1] = labels[S / 2];
    Buffers g = upload(acts, labels, {T}, {S});
    GpuRNNTWorkspaceManager<float> wm(g.acts, g.labels, 1, g.T, g.S, V);
    bool ok = wm.create_workspace() == RNNT_STATUS_SUCCESS;
    GpuRNNTComputer<float> computer(wm, 0, nullptr);
    float cost = 0;
    float *grads;
    (void)hipMalloc(&grads, acts.size() * sizeof(float));
    ok = ok && computer.cost_and_grad(&cost, grads) == RNNT_STATUS_SUCCESS;
    std::vector<float> gh(acts.size());
    (void)hipMemcpy(gh.data(), grads, gh.size() * sizeof(float), hipMemcpyDeviceToHost);
    ok = ok && std::isfinite(cost);
    for (float v : gh) ok = ok && std::isfinite(v);
    (void)hipFree(grads);
    wm.free_workspace();
    release(g);
    std::printf("infnan: %s (cost %.6f)\n", ok ? "ok" : "FAIL", cost);
    return ok;
}

// test_gpu.cu align_restrict_test / align_restrict_multibatch_test
static bool align_tests() {
    bool ok = true;
    {
        Buffers g = upload(toy_logits(1), {1, 2}, {4}, {2});
        int *al = to_gpu(std::vector<int>{0, 1, 0, 2});
        GpuRNNTWorkspaceManager<float> wm(g.acts, g.labels, 1, g.T, g.S, 3);
        ok = ok && wm.create_workspace() == RNNT_STATUS_SUCCESS;
        GpuRNNTComputer<float> computer(wm, 0, nullptr);
        float c = 0;
        ok = ok && computer.cost(&c) == RNNT_STATUS_SUCCESS && close(c, -std::log(0.363f));
        const int shifts[3] = {2, 0, 1};
        const float expect[3] = {0.363f, 0.072f, 0.2958f};
        for (int i = 0; i < 3; ++i) {
            wm.restrict_to_alignment(al, shifts[i], 0);
            ok = ok && computer.cost(&c) == RNNT_STATUS_SUCCESS && close(c, -std::log(expect[i]));
        }
        wm.free_workspace();
        (void)hipFree(al);
        release(g);
    }
    {
        Buffers g = upload(toy_logits(2), {1, 2, 1, 2}, {4, 4}, {2, 2});
        int *al = to_gpu(std::vector<int>{0, 1, 0, 2, 1, 2, 0, 0});
        GpuRNNTWorkspaceManager<float> wm(g.acts, g.labels, 2, g.T, g.S, 3);
        ok = ok && wm.create_workspace() == RNNT_STATUS_SUCCESS;
        GpuRNNTComputer<float> computer(wm, 0, nullptr);
        float c[2];
        const int shifts[3] = {3, 0, 1};
        const float e0[3] = {0.363f, 0.072f, 0.2958f}, e1[3] = {0.363f, 0.0672f, 0.192f};
        for (int i = 0; i < 3; ++i) {
            wm.restrict_to_alignment(al, shifts[i], 0);
            ok = ok && computer.cost(c) == RNNT_STATUS_SUCCESS && close(c[0], -std::log(e0[i])) &&
                 close(c[1], -std::log(e1[i]));
        }
        wm.free_workspace();
        (void)hipFree(al);
        release(g);
    }
    std::printf("align_restrict (+multibatch): %s\n", ok ? "ok" : "FAIL");
    return ok;
}

int main() {
    bool ok = true;
    ok &= toy_tests();
    ok &= multibatch_test();
    ok &= infnan_test();
    ok &= align_tests();
    std::printf(ok ? "Tests pass\n" : "Some or all tests fail\n");
    return ok ? 0 : 1;
}
