// gpu_rnnt.h -- GpuRNNTComputer<float>, the GPU computer the reference's bindings and tests drive
// directly (reference include/gpu_rnnt.h:16-249). Same constructor and methods:
//   cost_and_grad(costs_host, grads_device)  -- costs[B] on the host, grads [N, V] on the device
//   cost(costs_host)                         -- forward only (log-softmax + alpha recursion)
// Implemented in libmonotonic_rnnt_amd.so on top of the flat C API in mrnnt.h: three HIP kernels on
// `stream`, one D2H copy of the costs at the end (the reference's only required sync, gpu_rnnt.h:229).
#ifndef MONOTONIC_RNNT_GPU_RNNT_H
#define MONOTONIC_RNNT_GPU_RNNT_H

#include "gpu_workspace_manager.h"
#include "options.h"
#include "status.h"

template <typename ProbT>
class GpuRNNTComputer;  // only <float> is provided

template <>
class GpuRNNTComputer<float> {
   public:
    GpuRNNTComputer(GpuRNNTWorkspaceManager<float> &workspace_manager, int blank, hipStream_t stream);

    GpuRNNTComputer(const GpuRNNTComputer &) = delete;

    GpuRNNTComputer &operator=(const GpuRNNTComputer &) = delete;

    RNNTStatus cost_and_grad(float *costs, float *grads);

    RNNTStatus cost(float *costs);

   private:
    GpuRNNTWorkspaceManager<float> &workspace_manager_;
    int blank_;
    hipStream_t stream_;
};

#endif  // MONOTONIC_RNNT_GPU_RNNT_H
