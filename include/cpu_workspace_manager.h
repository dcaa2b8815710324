// cpu_workspace_manager.h -- CpuRNNTWorkspaceManager<float>, the host-side workspace object of the
// reference's C entry point with loc = RNNT_CPU (reference include/cpu_workspace_manager.h:12-355,
// installed by the reference's CMakeLists.txt:144). Same constructor and public lifecycle methods; the
// implementation lives in libmonotonic_rnnt_amd.so (csrc/mrnnt_cpu.cpp) and is this library's own
// multithreaded host implementation (not the reference's, and not the test oracle).
//
// Pointer conventions follow the reference: acts, labels, T, S and alignments are HOST pointers; labels
// use row stride max(S) and the alignment row stride max(T) (cpu_workspace_manager.h:121,192).
//
// Differences: the workspace layout is private (the reference's per-element accessors
// act()/get_alpha()/set_denom()... are not part of this header), restrict_to_alignment() copies the
// alignment and the band is built at compute time, and offsets are 64-bit (the reference indexes acts
// with int, cpu_workspace_manager.h:125-135, which overflows beyond 2^31 elements).
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

    mrnnt_cpu_ws_state *state() const { return st_; }

   private:
    mrnnt_cpu_ws_state *st_;
};

#endif  // MONOTONIC_RNNT_CPU_WORKSPACE_MANAGER_H
