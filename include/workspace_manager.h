/* workspace_manager.h -- polymorphic base of the workspace managers; identical contract to the
 * reference (include/workspace_manager.h:4-11): compute_rnnt_loss takes it by reference and
 * downcasts to the GPU manager. */
#ifndef MONOTONIC_RNNT_WORKSPACE_MANAGER_H
#define MONOTONIC_RNNT_WORKSPACE_MANAGER_H

class RNNTWorkspaceManager {
   public:
    RNNTWorkspaceManager() = default;

    RNNTWorkspaceManager(const RNNTWorkspaceManager &) = delete;

    virtual ~RNNTWorkspaceManager() = default;
};

#endif  // MONOTONIC_RNNT_WORKSPACE_MANAGER_H
