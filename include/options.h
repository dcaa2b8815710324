/* options.h -- RNNTOptions, field-for-field the reference's struct (include/options.h:12-24).
 * The only change: `stream` is a HIP stream (the reference forward-declares CUstream). The typedef
 * below is the same one hip_runtime_api.h makes, so this header needs no HIP include. */
#ifndef MONOTONIC_RNNT_OPTIONS_H
#define MONOTONIC_RNNT_OPTIONS_H

typedef struct ihipStream_t *hipStream_t;

typedef enum { RNNT_CPU = 0, RNNT_GPU = 1 } rnntComputeLocation;

struct RNNTOptions {
    /* The maximum number of threads that can be used (RNNT_CPU only; <= 0 = the OpenMP default) */
    int num_threads;

    /* HIP stream the kernels are launched on (0 = legacy default stream) */
    hipStream_t stream;

    /* the label value/index that the RNNT calculation should use as the blank label */
    int blank_label;

    /* where the calculation should take place: RNNT_GPU (HIP kernels, GpuRNNTWorkspaceManager<float>) or
     * RNNT_CPU (the library's host implementation, CpuRNNTWorkspaceManager<float>) */
    rnntComputeLocation loc;
};

#endif /* MONOTONIC_RNNT_OPTIONS_H */
