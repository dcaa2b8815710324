// cpu_workspace_manager.h -- CpuRNNTWorkspaceManager<float>, the host-side workspace object of the
// reference's C entry point with loc = RNNT_CPU (reference include/cpu_workspace_manager.h:12-355,
// installed by the reference's CMakeLists.txt:144). The reference's constructor and public methods, including the
// per-element accessors its computer uses (:63-205); the implementation lives in libmonotonic_rnnt_amd.so
// (csrc/mrnnt_cpu.cpp) and is this library's own multithreaded host implementation (not the reference's, and not
// the test oracle).
//
// Pointer conventions follow the reference: acts, labels, T, S and alignments are HOST pointers; labels
// use row stride max(S) and the alignment row stride max(T) (cpu_workspace_manager.h:121,192).
//
// Differences: the workspace layout is private (dense fp64 alpha / beta per lattice row instead
// of the reference's packed fp32 band, :286-354); get_alpha / get_beta read the state of the last computation
// (returned in float, with the reference's virtual boundaries and -inf outside the band); get_denom covers every
// row (a row outside the band or alignment window, which the computation never reads, is reduced on first access,
// as the reference's denominator pass covers all rows); restrict_to_alignment() copies the alignment (the band is
// rebuilt at compute time); act_index is 64-bit (the reference's int overflows beyond 2^31 elements, :125-135).
// Only the accessors are not thread-safe against a concurrent computation on the same manager, as in the reference.
#ifndef MONOTONIC_RNNT_CPU_WORKSPACE_MANAGER_H
#define MONOTONIC_RNNT_CPU_WORKSPACE_MANAGER_H

#include <cstddef>
#include <vector>

#include "status.h"
#include "workspace_manager.h"

struct mrnnt_cpu_ws_state;

template <typename dtype>
class CpuRNNTWorkspaceManager;  // only <float> is provided

template <>
class CpuRNNTWorkspaceManager<float> : public RNNTWorkspaceManager {
   public:
    CpuRNNTWorkspaceManager(const float *const acts, const int *const labels, const int B, const int *T, const int *S,
                            const int V);

    CpuRNNTWorkspaceManager(const CpuRNNTWorkspaceManager &) = delete;

    ~CpuRNNTWorkspaceManager() override;

    // Required bytes of the caller-provided host workspace (reference :95-114). Validates lengths:
    // B > 0, T_b > 0, S_b >= 0, T_b >= S_b, else RNNT_STATUS_INVALID_VALUE.
    RNNTStatus get_workspace_size(size_t *size_bytes) const;

    // Use caller-owned host memory of at least get_workspace_size() bytes (reference :221-234).
    void set_workspace(void *workspace);

    // malloc a workspace of the required size and use it (reference :236-245).
    RNNTStatus create_workspace();

    // Free a workspace made by create_workspace() (reference :247).
    void free_workspace();

    // Restrict paths to within max_shift frames of a reference alignment [B, max(T)] (host), blank_idx
    // marks blank frames in it (reference :191-219). The alignment is copied; it applies to later calls.
    void restrict_to_alignment(const int *const alignments, int max_shift, int blank_idx);

    [[nodiscard]] int B() const;
    [[nodiscard]] int V() const;
    [[nodiscard]] int T(int b) const;
    [[nodiscard]] int S(int b) const;

    // Lattice band of alpha(t, .) / beta(t, .) including the alignment restriction (reference :67-86)
    [[nodiscard]] int alpha_s_min(int b, int t) const;
    [[nodiscard]] int alpha_s_max(int b, int t) const;
    [[nodiscard]] int beta_s_min(int b, int t) const;
    [[nodiscard]] int beta_s_max(int b, int t) const;

    // Inputs (reference :117-137): label s of utterance b (row stride max(S)), element index and value of acts
    int label(int b, int s) const;
    [[nodiscard]] long long act_index(int b, int t, int s, int v) const;
    [[nodiscard]] float act(int b, int t, int s, int v) const;

    // Per-row state of the workspace (reference :139-205): log-softmax denominator, alpha(t, s) with the virtual
    // starts alpha(-1, 0) = 0, alpha(., -1) = alpha(-1, s > 0) = -inf, beta(t, s) with beta(T, S) = 0,
    // beta(T, s != S) = beta(., S+1) = -inf; -inf outside the (alignment) band
    void set_denom(int b, int t, int s, float value);
    float &get_denom(int b, int t, int s);
    void set_alpha(int b, int t, int s, float value);
    float get_alpha(int b, int t, int s) const;
    void set_beta(int b, int t, int s, float value);
    float get_beta(int b, int t, int s);

    mrnnt_cpu_ws_state *state() const { return st_; }

   private:
    mrnnt_cpu_ws_state *st_;
};

#endif  // MONOTONIC_RNNT_CPU_WORKSPACE_MANAGER_H
