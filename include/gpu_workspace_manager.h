// gpu_workspace_manager.h -- GpuRNNTWorkspaceManager<float>, the workspace object the reference's C
// entry point takes (reference include/gpu_workspace_manager.h:15-346). Same constructor and public
// methods; the implementation lives in libmonotonic_rnnt_amd.so (only the float instantiation exists,
// which is the only one the reference's entry point accepts: src/rnnt_entrypoint.cpp:34).
//
// Pointer conventions follow the reference: acts, labels, T, S and alignments are DEVICE pointers.
// Like the reference, the manager copies T and S to the host to size the workspace
// (gpu_workspace_manager.h:87-96); unlike it, labels use row stride max(S) and the alignment row
// stride max(T) exactly as the reference does (gpu_rnnt_kernel.h:133, gpu_workspace_manager.h:200).
//
// Differences: the workspace layout is private (no public data members), and
// restrict_to_alignment() records the alignment and builds the band on the device at compute time
// instead of a host loop with blocking copies (gpu_workspace_manager.h:191-219).
#ifndef MONOTONIC_RNNT_GPU_WORKSPACE_MANAGER_H
#define MONOTONIC_RNNT_GPU_WORKSPACE_MANAGER_H

#include <cstddef>
#include <vector>

#include "status.h"
#include "workspace_manager.h"

struct mrnnt_gpu_ws_state;

template <typename dtype>
class GpuRNNTWorkspaceManager;  // only <float> is provided

template <>
class GpuRNNTWorkspaceManager<float> : public RNNTWorkspaceManager {
   public:
    GpuRNNTWorkspaceManager(const float *const acts, const int *const labels, const int B, const int *T, const int *S,
                            const int V);

    GpuRNNTWorkspaceManager(const GpuRNNTWorkspaceManager &) = delete;

    ~GpuRNNTWorkspaceManager() override;

    // Required bytes for the caller-provided workspace (reference :228-254). Validates lengths:
    // B > 0, T_b > 0, S_b >= 0, T_b >= S_b, else RNNT_STATUS_INVALID_VALUE.
    RNNTStatus get_workspace_size(size_t *size_bytes) const;

    // Use caller-owned device memory of at least get_workspace_size() bytes (reference :256-329).
    void set_workspace(void *workspace);

    // hipMalloc a workspace of the required size and use it (reference :331-340).
    RNNTStatus create_workspace();

    // Free a workspace made by create_workspace() (reference :342).
    void free_workspace();

    // Restrict paths to within max_shift frames of a reference alignment [B, max(T)] (device),
    // blank_idx marks blank frames in it (reference :191-219). Takes effect on the next computation.
    void restrict_to_alignment(const int *const alignments, int max_shift, int blank_idx);

    // Host-side getters (reference :87-190 subset)
    [[nodiscard]] int B_host() const;
    [[nodiscard]] int V_host() const;
    [[nodiscard]] std::vector<int> T_host() const;
    [[nodiscard]] std::vector<int> S_host() const;
    [[nodiscard]] int num_denoms() const;

    mrnnt_gpu_ws_state *state() const { return st_; }

   private:
    mrnnt_gpu_ws_state *st_;
};

#endif  // MONOTONIC_RNNT_GPU_WORKSPACE_MANAGER_H
