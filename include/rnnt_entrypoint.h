/* rnnt_entrypoint.h -- the reference's C entry point, same symbol and signature
 * (reference include/rnnt_entrypoint.h:13-27, src/rnnt_entrypoint.cpp:16-48), served by
 * libmonotonic_rnnt_amd.so.
 *
 *   workspace_manager : loc = RNNT_GPU: a GpuRNNTWorkspaceManager<float> (gpu_workspace_manager.h);
 *                       loc = RNNT_CPU: a CpuRNNTWorkspaceManager<float> (cpu_workspace_manager.h);
 *                       its workspace set with set_workspace() or create_workspace(). A manager of the other
 *                       kind is RNNT_STATUS_INVALID_VALUE.
 *   options           : RNNTOptions; GPU kernels go to options.stream, CPU work uses options.num_threads
 *   costs             : HOST pointer [B], required (NULL -> RNNT_STATUS_INVALID_VALUE); the call returns
 *                       after the costs are on the host (as the reference does)
 *   gradients         : [sum_b T_b (S_b+1), V], DEVICE pointer (GPU) or HOST pointer (CPU), or NULL for cost
 *                       only
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
