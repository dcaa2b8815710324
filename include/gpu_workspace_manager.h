// gpu_workspace_manager.h -- GpuRNNTWorkspaceManager<float>, the workspace object the reference's C
// entry point takes (reference include/gpu_workspace_manager.h:15-346). The reference's constructor and public
// methods, including its host-side inspection getters (:87-190); the implementation lives in
// libmonotonic_rnnt_amd.so (only the float instantiation exists, which is the only one the reference's entry point
// accepts: src/rnnt_entrypoint.cpp:34).
//
// Pointer conventions follow the reference: acts, labels, T, S and alignments are DEVICE pointers. Like the
// reference, the manager copies T and S to the host to size the workspace (gpu_workspace_manager.h:87-96); labels
// use row stride max(S) and the alignment row stride max(T), as the reference does (gpu_rnnt_kernel.h:133,
// gpu_workspace_manager.h:200).
//
// The reference's public data members (:58-85) are here with the same names, types and meaning: device pointers into
// the workspace, laid out in the reference's order (:228-254), holding the reference's view of the last computation
// -- denom of every row, fp32 alpha / beta in the dense T*(S+1) per-utterance order with -inf outside the band,
// ll_forward / ll_backward, the [B, T_max] band, var_start_offsets / denom_start_indices, B, V, S_max, T_max. The
// library computes in its own layout (fp64 state) and writes this view after each cost() / cost_and_grad(), so a
// client kernel that reads wm.ll_forward or wm.alphas after the call sees what the reference's would.
//
// Differences:
//  * restrict_to_alignment() records the alignment, and the band is built on the device at compute time instead of
//    a host loop with blocking copies (:191-219);
//  * every data member is an OUTPUT: min_allowed_s / max_allowed_s show the band of the last computation; the
//    reference's computer reads the band from them (gpu_rnnt.h:103,149,196), this library does not -- a band written
//    into them is ignored (the call is unrestricted unless restrict_to_alignment() was called) and overwritten;
//  * the getters read the state of the last cost() / cost_and_grad() on this workspace (betas / ll_backward only
//    after cost_and_grad, as in the reference, whose cost() skips the beta pass). Cells outside the lattice band
//    read -inf (the reference leaves them unwritten), and denom_host() covers every row as the reference's reduce
//    does. Host copies are ordered on the computer's stream and synchronous, like the reference's cudaMemcpy.
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

    // Host-side getters (reference :87-190)
    [[nodiscard]] int B_host() const;
    [[nodiscard]] int V_host() const;
    [[nodiscard]] std::vector<int> T_host() const;
    [[nodiscard]] std::vector<int> S_host() const;
    [[nodiscard]] int num_denoms() const;                 // sum_b T_b (S_b+1)
    [[nodiscard]] int num_fwd_bwd_var_positions() const;  // the same count (dense alpha / beta storage)
    [[nodiscard]] std::vector<int> var_start_offsets_host() const;  // [B] first row of each utterance
    [[nodiscard]] std::vector<float> acts_host() const;   // [num_denoms() * V]
    [[nodiscard]] std::vector<float> denom_host() const;  // [num_denoms()] -max - log sum exp of every row
    [[nodiscard]] std::vector<float> alphas_host() const; // [num_denoms()] alpha(t, s) at var_start_offsets[b] + t(S_b+1) + s
    [[nodiscard]] std::vector<float> betas_host() const;  // [num_denoms()] beta(t, s), same order
    [[nodiscard]] int S_max_host() const;
    [[nodiscard]] int T_max_host() const;
    [[nodiscard]] std::vector<int> min_allowed_s_host() const;  // [B * T_max] alignment band (0 unrestricted)
    [[nodiscard]] std::vector<int> max_allowed_s_host() const;  // [B * T_max] (S_b unrestricted)
    [[nodiscard]] std::vector<float> ll_forward_host() const;   // [B] alpha(T_b-1, S_b)
    [[nodiscard]] std::vector<float> ll_backward_host() const;  // [B] beta(0, 0)

    mrnnt_gpu_ws_state *state() const { return st_; }

   private:
    mrnnt_gpu_ws_state *st_;

   public:
    // the reference's public data members (gpu_workspace_manager.h:58-85); set by set_workspace()
    void *workspace_;  // device

    const int B_h;  // host
    const int V_h;  // host

    const int *T;  // device
    const int *S;  // device
    int *B;        // device
    int *V;        // device

    const float *const acts;  // device
    const int *const labels;  // device

    float *denom;   // workspace
    float *alphas;  // workspace
    float *betas;   // workspace

    int *min_allowed_s;  // workspace
    int *max_allowed_s;  // workspace

    int *denom_start_indices;  // workspace
    int *var_start_offsets;    // workspace

    int *S_max;  // workspace
    int *T_max;  // workspace

    float *ll_forward;   // workspace
    float *ll_backward;  // workspace
};

#endif  // MONOTONIC_RNNT_GPU_WORKSPACE_MANAGER_H
