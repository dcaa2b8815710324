/* mrnnt.h -- flat, pure-C ABI of libmonotonic_rnnt_amd.so (plain pointers and sizes only).
 *
 * This is the boundary every binding calls (the Python autograd op via ctypes, the C++ classes in
 * gpu_rnnt.h / rnnt_entrypoint.h, and any cgo/JNI/N-API stub: INTEGRATION.md). It replaces the
 * reference's pybind entry points (reference pytorch_binding/monotonic_rnnt.cu:81-152) and the
 * GpuRNNTComputer they construct (reference include/gpu_rnnt.h:27-235), split so an autograd
 * Function can run the loss in forward and the logit gradient (with dL/dcost fused) in backward.
 *
 * Data layout (same contract as the reference, monotonic_rnnt_op.py:133-140):
 *   acts    [N, V] fp32, N = sum_b T_b (S_b+1); utterance b contiguous, then t-major, then s
 *   labels  [B, label_stride] int32, label of (b, s) at labels[b*label_stride + s]
 *   T, S    [B] int32 input / label lengths (device copies for the kernels, host copies to plan)
 *   alignment (optional) [B, align_stride] int32, frames equal to align_blank are blanks
 * All device pointers are HIP device memory; nothing is allocated inside the calls.
 */
#ifndef MONOTONIC_RNNT_MRNNT_H
#define MONOTONIC_RNNT_MRNNT_H

#include <stddef.h>
#include <stdint.h>

#include "options.h"
#include "status.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MRNNT_VERSION 1

typedef struct mrnnt_problem {
    int B;                   /* utterances */
    int V;                   /* alphabet size including blank */
    int blank;               /* blank label index */
    int max_shift;           /* alignment restriction k (ignored when alignment == NULL) */
    const int *T_host;       /* host [B] */
    const int *S_host;       /* host [B] */
    const int *T_dev;        /* device [B] (same values) */
    const int *S_dev;        /* device [B] */
    const float *acts;       /* device [N, V] */
    const int *labels;       /* device [B, label_stride] */
    int64_t label_stride;
    const int *alignment;    /* device [B, align_stride] or NULL */
    int64_t align_stride;
    int align_blank;         /* value marking blank frames in `alignment` */
    int64_t num_rows;        /* N as the caller sized acts; must equal sum_b T_b (S_b+1) (checked) */
} mrnnt_problem;

/* Validate lengths (reference semantics: B > 0, V > 0, T_b > 0, S_b >= 0, T_b >= S_b) and return the
 * device workspace bytes needed by mrnnt_forward / mrnnt_backward for this problem. Host-only. */
RNNTStatus mrnnt_workspace_size(const mrnnt_problem *p, size_t *bytes);

/* Forward: log-softmax row reduce + alpha (and, if with_beta, beta) recursion.
 * Writes costs_dev[b] = -log p(labels_b | acts_b) (device fp32, may be NULL) and keeps the per-row
 * state needed by mrnnt_backward in `workspace`. Asynchronous on `stream`. */
RNNTStatus mrnnt_forward(const mrnnt_problem *p, void *workspace, size_t workspace_bytes, float *costs_dev,
                         int with_beta, hipStream_t stream);

/* Backward: grads[r, v] = grad_scale[b(r)] * dcost_b / dacts[r, v] for every row (out-of-band rows
 * are written with zeros; no pre-zeroing needed). grad_scale (device [B]) may be NULL (= 1).
 * Requires a preceding mrnnt_forward(with_beta=1) on the same workspace and inputs. */
RNNTStatus mrnnt_backward(const mrnnt_problem *p, const void *workspace, const float *grad_scale, float *grads,
                          hipStream_t stream);

/* forward(with_beta = grads != NULL) followed by backward. */
RNNTStatus mrnnt_cost_and_grad(const mrnnt_problem *p, void *workspace, size_t workspace_bytes, float *costs_dev,
                               float *grads, const float *grad_scale, hipStream_t stream);

/* Forward log-likelihoods from the workspace (device double [B]), for debugging/inspection:
 * ll_fwd = alpha(T-1, S), ll_bwd = beta(0, 0). Either may be NULL. Asynchronous on `stream`. */
RNNTStatus mrnnt_read_loglik(const mrnnt_problem *p, const void *workspace, double *ll_fwd_dev, double *ll_bwd_dev,
                             hipStream_t stream);

/* Message describing the last non-success status returned on this thread. */
const char *mrnnt_last_error(void);

int mrnnt_version(void);

/* Kernel-time accounting over HIP events recorded around each launch on its stream.
 * enable=1 starts recording (clearing previous records). mrnnt_profile_read synchronises the
 * recorded events and returns per-kernel totals in ms and launch counts for
 *   [0] band, [1] log-softmax row reduce, [2] alpha/beta DP, [3] logit gradient, [4] setup. */
void mrnnt_profile_enable(int enable);
int mrnnt_profile_read(double *total_ms, int64_t *launches, int n);

/* Launch-shape knobs for experiments (defaults are the tuned values): "softmax_variant" (0 row-at-a-time,
 * 1 pipelined), "grad_variant" (0/1), "softmax_grid_per_cu" / "grad_grid_per_cu" (persistent workgroups per
 * CU, 0 = one workgroup per lattice column; "grid_per_cu" sets both), "nt_store" (0/1), "dp_variant"
 * (0 one wave per utterance and direction, 1 four waves).
 * Sets `key` to `value` (value < 0: query only) and returns the previous value, or -1 for an unknown key.
 * Process-global; not thread-safe against concurrent launches. */
int mrnnt_tune(const char *key, int value);

/* Bench helper: fill out[0..count) with the counter-based synthetic generator (bit-identical to the
 * host twin in oracle/rnnt_oracle.c): element i gets hash(seed, begin + i) as N(0,1)-like
 * (normal=1) or U[0,1) (normal=0). */
RNNTStatus mrnnt_synth_acts(float *out, int64_t begin, int64_t count, uint64_t seed, int normal, hipStream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* MONOTONIC_RNNT_MRNNT_H */
