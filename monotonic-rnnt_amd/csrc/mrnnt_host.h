// mrnnt_host.h -- declarations shared by the host translation units of libmonotonic_rnnt_amd.so: the HIP
// side (mrnnt_capi.cpp, hipcc), the host-only C ABI (mrnnt_entry.cpp, g++) and the CPU implementation (mrnnt_cpu.cpp,
// g++). Plain C++, no HIP types.
// Not installed; not part of the ABI.
#pragma once

#include <string>

#include "options.h"
#include "status.h"
#include "workspace_manager.h"

namespace mrnnt {

// Record `msg` as this thread's mrnnt_last_error() and return `st` (defined in mrnnt_entry.cpp).
RNNTStatus set_error(RNNTStatus st, const std::string &msg);

// compute_rnnt_loss for loc = RNNT_GPU (mrnnt_capi.cpp; a weak stub in mrnnt_entry.cpp serves host-only builds).
RNNTStatus gpu_compute_rnnt_loss(RNNTWorkspaceManager &workspace_manager, RNNTOptions options, float *costs,
                                 float *gradients);

// A lattice row (t, s) with alpha(t-1, s) + beta(t, s) - ll < kDeadLogOcc has occupancy below e^-110 =
// 2^-158.7: every element of its fp32 gradient, p_v * occupancy minus the blank / label corrections (each
// bounded by the occupancy), is below half the smallest fp32 denormal (2^-150) and rounds to exactly 0 --
// in these kernels and in the reference's fp32 arithmetic alike. Such rows are stored as 0 * grad_scale
// without reading acts. (NaN state compares false and takes the full path.)
constexpr double kDeadLogOcc = -110.0;

}  // namespace mrnnt
