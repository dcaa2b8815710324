// cpu_rnnt.h -- CpuRNNTComputer<float>, the host computer the reference's tests and bindings drive
// directly (reference include/cpu_rnnt.h:23-264). Same constructor and methods:
//   cost_and_grad(costs, grads)  -- costs[B] and grads [N, V], both host
//   cost(costs)                  -- forward only (log-softmax + alpha recursion)
// Implemented in libmonotonic_rnnt_amd.so (csrc/mrnnt_cpu.cpp): OpenMP over lattice rows for the two
// streaming passes (the reference parallelises over utterances only, cpu_rnnt.h:54-57, so at most B
// threads work), SIMD exp, fp64 recursion state. num_threads > 0 sets the thread count of this
// computer's parallel regions (the reference sets the process-global OpenMP default, cpu_rnnt.h:30-34).
#ifndef MONOTONIC_RNNT_CPU_RNNT_H
#define MONOTONIC_RNNT_CPU_RNNT_H

#include "cpu_workspace_manager.h"
#include "status.h"

template <typename ProbT>
class CpuRNNTComputer;  // only <float> is provided

template <>
class CpuRNNTComputer<float> {
   public:
    CpuRNNTComputer(CpuRNNTWorkspaceManager<float> &workspace_manager, int blank, int num_threads);

    CpuRNNTComputer(const CpuRNNTComputer &) = delete;

    CpuRNNTComputer &operator=(const CpuRNNTComputer &) = delete;

    RNNTStatus cost_and_grad(float *costs, float *grads);

    RNNTStatus cost(float *costs);

   private:
    CpuRNNTWorkspaceManager<float> &workspace_manager_;
    int blank_;
    int num_threads_;
};

#endif  // MONOTONIC_RNNT_CPU_RNNT_H
