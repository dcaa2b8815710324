// test_cpu_abi.cpp -- the reference's own CPU test program shape (tests/test_cpu.cpp: fwd, bwd, grads,
// multibatch, infnan, align_restrict, align_restrict_multibatch), written against this repository's headers
// and linked against libmonotonic_rnnt_amd.so. Host code only (g++): it drives the library's CPU
// implementation through CpuRNNTWorkspaceManager<float> + CpuRNNTComputer<float> and through the extern "C"
// compute_rnnt_loss entry point with loc = RNNT_CPU (src/rnnt_entrypoint.cpp:22-31). Known answers from the
// reference's test (README.md:117-174). Returns 0 when every test passes.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

#include "cpu_rnnt.h"
#include "cpu_workspace_manager.h"
#include "rnnt_entrypoint.h"

static const float kProbs[36] = {0.6, 0.3, 0.1, 0.7, 0.1, 0.2, 0.5, 0.1, 0.4, 0.5, 0.4, 0.1,
                                 0.5, 0.1, 0.4, 0.8, 0.1, 0.1, 0.4, 0.3, 0.3, 0.5, 0.1, 0.4,
                                 0.7, 0.2, 0.1, 0.8, 0.1, 0.1, 0.3, 0.1, 0.6, 0.8, 0.1, 0.1};
static const float kGrads[36] = {0.04, -0.14, 0.1, 0,    0,    0,     0,    0,     0,     0.13,  -0.19, 0.06,
                                 -0.04, 0.04, -0.01, 0,   0,    0,     0.06, -0.1,  0.04,  0.01,  0.07,  -0.08,
                                 -0.06, 0.04, 0.02,  0,   0,    0,     0.14, 0.05,  -0.19, -0.11, 0.05,  0.05};

static bool close(float a, float b, float tol = 1e-4f) { return std::fabs(a - b) < tol; }

static std::vector<float> toy_logits(int copies) {
    std::vector<float> l;
    for (int c = 0; c < copies; ++c)
        for (float p : kProbs) l.push_back(std::log(p));
    return l;
}

// fwd_test / bwd_test / grads_test through CpuRNNTComputer (test_cpu.cpp:10-192)
static bool toy_tests() {
    std::vector<float> logits = toy_logits(1);
    std::vector<int> labels = {1, 2}, T = {4}, S = {2};
    CpuRNNTWorkspaceManager<float> wm(logits.data(), labels.data(), 1, T.data(), S.data(), 3);
    if (wm.create_workspace() != RNNT_STATUS_SUCCESS) return false;
    CpuRNNTComputer<float> computer(wm, 0, 1);
    float cost_fwd = 0, cost_bwd = 0;
    bool ok = computer.cost(&cost_fwd) == RNNT_STATUS_SUCCESS;
    ok = ok && close(cost_fwd, -std::log(0.363f));
    std::vector<float> grads(36, 7.0f);
    ok = ok && computer.cost_and_grad(&cost_bwd, grads.data()) == RNNT_STATUS_SUCCESS;
    ok = ok && close(cost_fwd, cost_bwd);
    for (int i = 0; i < 36; ++i) ok = ok && std::fabs(grads[i] - kGrads[i]) < 1e-2f;
    wm.free_workspace();
    std::printf("toy fwd/bwd/grads: %s (cost %.6f)\n", ok ? "ok" : "FAIL", cost_fwd);
    return ok;
}

// multibatch_test (test_cpu.cpp:194-295) through compute_rnnt_loss with loc = RNNT_CPU
static bool multibatch_test() {
    std::vector<float> probs;
    const int rows0[4] = {0, 1, 3, 4};
    for (int r : rows0)
        for (int v = 0; v < 3; ++v) probs.push_back(kProbs[r * 3 + v]);
    for (float p : kProbs) probs.push_back(p);
    std::vector<float> logits(probs.size());
    std::transform(probs.begin(), probs.end(), logits.begin(), [](float p) { return std::log(p); });
    std::vector<int> labels = {1, 0, 1, 2}, T = {2, 4}, S = {1, 2};
    CpuRNNTWorkspaceManager<float> wm(logits.data(), labels.data(), 2, T.data(), S.data(), 3);
    size_t bytes = 0;
    bool ok = wm.get_workspace_size(&bytes) == RNNT_STATUS_SUCCESS && bytes > 0;
    std::vector<char> ws(bytes);
    wm.set_workspace(ws.data());
    RNNTOptions opt;
    opt.num_threads = 2;
    opt.stream = nullptr;
    opt.blank_label = 0;
    opt.loc = RNNT_CPU;
    float costs[2] = {0, 0};
    ok = ok && compute_rnnt_loss(wm, opt, costs, nullptr) == RNNT_STATUS_SUCCESS;
    ok = ok && close(costs[0], -std::log(0.39f)) && close(costs[1], -std::log(0.363f));
    std::vector<float> grads(logits.size());
    float costs2[2] = {0, 0};
    ok = ok && compute_rnnt_loss(wm, opt, costs2, grads.data()) == RNNT_STATUS_SUCCESS;
    ok = ok && close(costs[0], costs2[0]) && close(costs[1], costs2[1]);
    const float exp0[12] = {-0.02, -0.08, 0.1, 0.0, 0.0, 0.0, 0.31, -0.37, 0.06, -0.19, 0.04, 0.15};
    for (int i = 0; i < 12; ++i) ok = ok && std::fabs(grads[i] - exp0[i]) < 1e-2f;
    for (int i = 0; i < 36; ++i) ok = ok && std::fabs(grads[12 + i] - kGrads[i]) < 1e-2f;
    // entry-point argument checks (src/rnnt_entrypoint.cpp:18-20, :44-46)
    ok = ok && compute_rnnt_loss(wm, opt, nullptr, nullptr) == RNNT_STATUS_INVALID_VALUE;
    RNNTOptions bad = opt;
    bad.loc = static_cast<rnntComputeLocation>(7);
    ok = ok && compute_rnnt_loss(wm, bad, costs, nullptr) == RNNT_STATUS_INVALID_VALUE;
    std::printf("multibatch (compute_rnnt_loss, RNNT_CPU): %s (%.6f %.6f)\n", ok ? "ok" : "FAIL", costs[0], costs[1]);
    return ok;
}

// infnan_test shape (test_cpu.cpp:297-333): T=50, S=10, V=15, uniform [0, 1) logits, repeated labels
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
    std::vector<int> Tv = {T}, Sv = {S};
    CpuRNNTWorkspaceManager<float> wm(acts.data(), labels.data(), 1, Tv.data(), Sv.data(), V);
    bool ok = wm.create_workspace() == RNNT_STATUS_SUCCESS;
    CpuRNNTComputer<float> computer(wm, 0, 1);
    float cost = 0;
    std::vector<float> grads(acts.size());
    ok = ok && computer.cost_and_grad(&cost, grads.data()) == RNNT_STATUS_SUCCESS;
    ok = ok && std::isfinite(cost);
    for (float v : grads) ok = ok && std::isfinite(v);
    wm.free_workspace();
    std::printf("infnan: %s (cost %.6f)\n", ok ? "ok" : "FAIL", cost);
    return ok;
}

// align_restrict_test / align_restrict_multibatch_test (test_cpu.cpp:335-552)
static bool align_tests() {
    bool ok = true;
    {
        std::vector<float> logits = toy_logits(1);
        std::vector<int> labels = {1, 2}, T = {4}, S = {2}, al = {0, 1, 0, 2};
        CpuRNNTWorkspaceManager<float> wm(logits.data(), labels.data(), 1, T.data(), S.data(), 3);
        ok = ok && wm.create_workspace() == RNNT_STATUS_SUCCESS;
        CpuRNNTComputer<float> computer(wm, 0, 1);
        float c = 0;
        ok = ok && computer.cost(&c) == RNNT_STATUS_SUCCESS && close(c, -std::log(0.363f));
        const int shifts[3] = {2, 0, 1};
        const float expect[3] = {0.363f, 0.072f, 0.2958f};
        for (int i = 0; i < 3; ++i) {
            wm.restrict_to_alignment(al.data(), shifts[i], 0);
            ok = ok && computer.cost(&c) == RNNT_STATUS_SUCCESS && close(c, -std::log(expect[i]));
        }
        wm.free_workspace();
    }
    {
        std::vector<float> logits = toy_logits(2);
        std::vector<int> labels = {1, 2, 1, 2}, T = {4, 4}, S = {2, 2}, al = {0, 1, 0, 2, 1, 2, 0, 0};
        CpuRNNTWorkspaceManager<float> wm(logits.data(), labels.data(), 2, T.data(), S.data(), 3);
        ok = ok && wm.create_workspace() == RNNT_STATUS_SUCCESS;
        CpuRNNTComputer<float> computer(wm, 0, 1);
        float c[2];
        const int shifts[3] = {3, 0, 1};
        const float e0[3] = {0.363f, 0.072f, 0.2958f}, e1[3] = {0.363f, 0.0672f, 0.192f};
        for (int i = 0; i < 3; ++i) {
            wm.restrict_to_alignment(al.data(), shifts[i], 0);
            ok = ok && computer.cost(c) == RNNT_STATUS_SUCCESS && close(c[0], -std::log(e0[i])) &&
                 close(c[1], -std::log(e1[i]));
        }
        wm.free_workspace();
    }
    std::printf("align_restrict (+multibatch): %s\n", ok ? "ok" : "FAIL");
    return ok;
}

// invalid lengths (cpu_workspace_manager.h:99-107): T < S is RNNT_STATUS_INVALID_VALUE
static bool invalid_test() {
    std::vector<float> logits = toy_logits(1);
    std::vector<int> labels = {1, 2, 1}, T = {2}, S = {3};
    CpuRNNTWorkspaceManager<float> wm(logits.data(), labels.data(), 1, T.data(), S.data(), 3);
    const bool ok = wm.create_workspace() == RNNT_STATUS_INVALID_VALUE;
    std::printf("invalid lengths: %s\n", ok ? "ok" : "FAIL");
    return ok;
}

int main() {
    bool ok = true;
    ok &= toy_tests();
    ok &= multibatch_test();
    ok &= infnan_test();
    ok &= align_tests();
    ok &= invalid_test();
    std::printf(ok ? "Tests pass\n" : "Some or all tests fail\n");
    return ok ? 0 : 1;
}
