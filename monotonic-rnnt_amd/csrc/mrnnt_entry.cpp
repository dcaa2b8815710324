// mrnnt_entry.cpp -- the host-only part of the library's C ABI, plain C++ (g++, no HIP): this thread's error state
// (mrnnt_last_error, mrnnt::set_error), mrnnt_version, the host lattice builder (mrnnt_lattice_bytes / _host) and the
// reference's entry point compute_rnnt_loss (reference src/rnnt_entrypoint.cpp:16-48), which dispatches on
// options.loc: RNNT_CPU to the CPU computer (mrnnt_cpu.cpp) here, RNNT_GPU to mrnnt::gpu_compute_rnnt_loss in
// mrnnt_capi.cpp. Kept free of HIP so that the sanitizer build (`make -C monotonic-rnnt_amd asan`) runs this file
// with the CPU implementation under AddressSanitizer / UBSan on a host without a GPU.
#include <cstdint>
#include <cstring>
#include <string>

// only the declarations of the public headers are exported (the library is built with -fvisibility=hidden)
#pragma GCC visibility push(default)
#include "cpu_rnnt.h"
#include "cpu_workspace_manager.h"
#include "mrnnt.h"
#include "rnnt_entrypoint.h"
#pragma GCC visibility pop
#include "mrnnt_host.h"

namespace {

thread_local std::string g_last_error = "no error";

}  // namespace

RNNTStatus mrnnt::set_error(RNNTStatus st, const std::string &msg) {
    g_last_error = msg;
    return st;
}

// The product library links mrnnt_capi.cpp's definition; this weak one is what a host-only build (the sanitizer
// targets) links instead, and it says so rather than pretending to compute.
__attribute__((weak)) RNNTStatus mrnnt::gpu_compute_rnnt_loss(RNNTWorkspaceManager &, RNNTOptions, float *, float *) {
    return set_error(RNNT_STATUS_EXECUTION_FAILED, "this is a host-only build of the library: no RNNT_GPU path");
}

extern "C" {

int mrnnt_version(void) { return MRNNT_VERSION; }

const char *mrnnt_last_error(void) { return g_last_error.c_str(); }

RNNTStatus mrnnt_lattice_bytes(const mrnnt_problem *p, size_t *bytes) {
    // needs only B, T_host and S_host
    if (!bytes || !p) return mrnnt::set_error(RNNT_STATUS_INVALID_VALUE, "null argument");
    if (p->B <= 0 || !p->T_host || !p->S_host)
        return mrnnt::set_error(RNNT_STATUS_INVALID_VALUE, "B > 0 and host lengths required");
    int64_t cols = 0;
    for (int b = 0; b < p->B; ++b) {
        if (p->T_host[b] <= 0 || p->S_host[b] < 0 || p->T_host[b] < p->S_host[b])
            return mrnnt::set_error(RNNT_STATUS_INVALID_VALUE, "invalid lengths at utterance " + std::to_string(b));
        cols += p->T_host[b];
    }
    *bytes = sizeof(int64_t) * 2 * ((size_t)p->B + 1) + sizeof(int) * (size_t)cols;
    return RNNT_STATUS_SUCCESS;
}

RNNTStatus mrnnt_lattice_host(const mrnnt_problem *p, void *host, size_t bytes) {
    size_t need = 0;
    const RNNTStatus st = mrnnt_lattice_bytes(p, &need);
    if (st != RNNT_STATUS_SUCCESS) return st;
    if (!host || bytes < need)
        return mrnnt::set_error(RNNT_STATUS_INVALID_VALUE, "lattice buffer too small: need " + std::to_string(need));
    int64_t *row = static_cast<int64_t *>(host), *col = row + p->B + 1;
    int *col_b = reinterpret_cast<int *>(col + p->B + 1);
    row[0] = col[0] = 0;
    for (int b = 0; b < p->B; ++b) {
        row[b + 1] = row[b] + (int64_t)p->T_host[b] * (p->S_host[b] + 1);
        col[b + 1] = col[b] + p->T_host[b];
        for (int64_t c = col[b]; c < col[b + 1]; ++c) col_b[c] = b;
    }
    return RNNT_STATUS_SUCCESS;
}

RNNTStatus compute_rnnt_loss(RNNTWorkspaceManager &workspace_manager, RNNTOptions options, float *costs,
                             float *gradients) {
    // src/rnnt_entrypoint.cpp:16-48 (a manager of the wrong kind is RNNT_STATUS_INVALID_VALUE here; the
    // reference's reference-typed dynamic_cast throws std::bad_cast across the C boundary)
    if (costs == nullptr) return mrnnt::set_error(RNNT_STATUS_INVALID_VALUE, "costs is null");
    // the location as the caller stored it: a C or FFI caller may put any int there, and loading an out-of-range
    // value through the enum type is undefined behaviour in C++ (found by the UBSan build, `make asan`)
    int loc = 0;
    static_assert(sizeof(loc) == sizeof(options.loc), "rnntComputeLocation is int-sized");
    std::memcpy(&loc, &options.loc, sizeof(loc));
    if (loc == RNNT_CPU) {
        auto *cm = dynamic_cast<CpuRNNTWorkspaceManager<float> *>(&workspace_manager);
        if (!cm)
            return mrnnt::set_error(RNNT_STATUS_INVALID_VALUE,
                                    "workspace manager is not a CpuRNNTWorkspaceManager<float>");
        CpuRNNTComputer<float> computer(*cm, options.blank_label, options.num_threads);
        return gradients != nullptr ? computer.cost_and_grad(costs, gradients) : computer.cost(costs);
    }
    if (loc != RNNT_GPU) return mrnnt::set_error(RNNT_STATUS_INVALID_VALUE, "unknown compute location");
    return mrnnt::gpu_compute_rnnt_loss(workspace_manager, options, costs, gradients);
}

}  // extern "C"
