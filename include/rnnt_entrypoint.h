/* rnnt_entrypoint.h -- the reference's C entry point, same symbol and signature
 * (reference include/rnnt_entrypoint.h:13-27, src/rnnt_entrypoint.cpp:16-48), served by
 * libmonotonic_rnnt_amd.so.
 *
 *   workspace_manager : a GpuRNNTWorkspaceManager<float> (gpu_workspace_manager.h) whose workspace was
 *                       set with set_workspace() or create_workspace()
 *   options           : RNNTOptions; loc must be RNNT_GPU, kernels go to options.stream
 *   costs             : HOST pointer [B], required (NULL -> RNNT_STATUS_INVALID_VALUE); the call returns
 *                       after the costs have been copied to the host (as the reference does)
 *   gradients         : DEVICE pointer [sum_b T_b (S_b+1), V] or NULL for cost only
 */
#ifndef MONOTONIC_RNNT_ENTRYPOINT_H
#define MONOTONIC_RNNT_ENTRYPOINT_H

#include "options.h"
#include "status.h"
#include "workspace_manager.h"

extern "C" {

RNNTStatus compute_rnnt_loss(RNNTWorkspaceManager &workspace_manager, RNNTOptions options, float *costs,
                             float *gradients);

}  // extern "C"

#endif  // MONOTONIC_RNNT_ENTRYPOINT_H
