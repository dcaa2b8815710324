/* mrnnt.h -- flat, pure-C ABI of libmonotonic_rnnt_amd.so (plain pointers and sizes only).
 *
 * This is the boundary every binding calls (the Python autograd op via ctypes, the C++ classes in
 * gpu_rnnt.h / rnnt_entrypoint.h, and any cgo/JNI/N-API stub: INTEGRATION.md). It replaces the
 * reference's pybind entry points (reference pytorch_binding/monotonic_rnnt.cu:81-152) and the
 * GpuRNNTComputer they construct (reference include/gpu_rnnt.h:27-235), split so an autograd
 * Function can run the loss in forward and the logit gradient (with dL/dcost fused) in backward.
 *
 * Data layout (same contract as the reference, monotonic_rnnt_op.py:133-140):
 *   acts    [N, V], N = sum_b T_b (S_b+1); utterance b contiguous, then t-major, then s ("packed").
 *           Extension (acts_layout): padded [B, pad_T, pad_S1, V] with (b, t, s) at row
 *           (b*pad_T + t)*pad_S1 + s -- the joint network's natural output, no packing copy.
 *           Element type fp32 (reference), or bf16 / fp16 (acts_dtype); grads use the same type and
 *           layout. The arithmetic is fp32/fp64 in registers whatever the element type.
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

#define MRNNT_VERSION 12

/* acts / grads element types */
#define MRNNT_F32 0
#define MRNNT_BF16 1
#define MRNNT_F16 2

typedef struct mrnnt_problem {
    int B;                   /* utterances */
    int V;                   /* alphabet size including blank */
    int blank;               /* blank label index */
    int max_shift;           /* alignment restriction k (ignored when alignment == NULL) */
    const int *T_host;       /* host [B] */
    const int *S_host;       /* host [B] */
    const int *T_dev;        /* device [B] (same values) */
    const int *S_dev;        /* device [B] */
    const void *acts;        /* device [N, V] packed, or [B, pad_T, pad_S1, V] padded; acts_dtype elements */
    const int *labels;       /* device [B, label_stride] */
    int64_t label_stride;
    const int *alignment;    /* device [B, align_stride] or NULL */
    int64_t align_stride;
    int align_blank;         /* value marking blank frames in `alignment` */
    int64_t num_rows;        /* rows of acts as the caller sized it (checked; < 0 skips the check): packed
                                sum_b T_b (S_b+1), padded B*pad_T*pad_S1 */
    /* --- version 2 --- (zero-initialised = the reference contract: packed fp32) */
    int acts_dtype;          /* MRNNT_F32 / MRNNT_BF16 / MRNNT_F16 */
    int64_t pad_T;           /* padded layout: frames per utterance slot (>= max T_b) */
    int64_t pad_S1;          /* padded layout: label positions per frame (>= max S_b + 1); 0 = packed */
    /* --- version 4 --- */
    const void *lattice;     /* optional: device copy of mrnnt_lattice_host's output for these lengths. The lattice
                                offsets then come from it and mrnnt_forward launches no setup kernel (a caller that
                                repeats shapes uploads it once); NULL = built on the device in every forward. The
                                workspace then holds no offsets of its own: pass the same lattice to every later
                                call on that workspace (mrnnt_backward, mrnnt_read_*, mrnnt_grad_live_rows), and
                                only a lattice built from these lengths (it is not checked against them) */
    /* --- version 6 --- */
    int grad_scale_broadcast; /* 1: grad_scale[0] scales every utterance (a stride-0 upstream gradient, e.g. the
                                backward of costs.sum(): no copy into a [B] vector); 0: grad_scale[b] */
    /* --- version 7 --- */
    int lengths_on_device;   /* 1: the lengths exist only on the device (T_dev / S_dev; T_host / S_host may be NULL),
                                as the reference's GPU binding requires (monotonic_rnnt.cu:85-88). The launch is then
                                planned from bounds the host knows without reading them back -- num_rows (required:
                                the packed rows, or B*pad_T*pad_S1 padded) and label_stride (>= every S_b) -- and the
                                lattice offsets are built and the lengths validated on the device (T_b > 0, S_b >= 0,
                                T_b >= S_b, S_b <= label_stride, packed rows == num_rows, padded / alignment strides).
                                No host synchronisation; capturable in a HIP graph. lattice must be NULL. A length set
                                that fails validation makes every cost and gradient of the call NaN (nothing outside
                                the caller's buffers is touched) and raises *status_host. */
    int *status_host;        /* optional, with lengths_on_device: a host word from mrnnt_status_word(); the device
                                stores RNNT_STATUS_INVALID_VALUE into it when validation fails (never clears it) */
} mrnnt_problem;

/* A process-wide host-mapped int (initially 0) the device can store into without a copy: pass it as
 * mrnnt_problem.status_host and poll it from the host at leisure (reset it to 0 yourself). */
int *mrnnt_status_word(void);

/* Validate lengths (reference semantics: B > 0, V > 0, T_b > 0, S_b >= 0, T_b >= S_b) and return the
 * device workspace bytes needed by mrnnt_forward / mrnnt_backward for this problem. Host-only. */
RNNTStatus mrnnt_workspace_size(const mrnnt_problem *p, size_t *bytes);

/* Lattice offsets of the problem's lengths, computed on the host from T_host / S_host: int64 row_off[B+1]
 * (first lattice row of each utterance), int64 col_off[B+1] (first column), int32 col_b[sum_b T_b] (utterance
 * of each column). mrnnt_lattice_bytes gives the size; mrnnt_lattice_host fills `host` (>= that many bytes).
 * Upload it to device memory and pass it as mrnnt_problem.lattice. Host-only. */
RNNTStatus mrnnt_lattice_bytes(const mrnnt_problem *p, size_t *bytes);
RNNTStatus mrnnt_lattice_host(const mrnnt_problem *p, void *host, size_t bytes);

/* Forward: log-softmax row reduce + alpha (and, if with_beta, beta) recursion.
 * Writes costs_dev[b] = -log p(labels_b | acts_b) (device fp32, may be NULL) and keeps the per-row
 * state needed by mrnnt_backward in `workspace`. Asynchronous on `stream`. */
RNNTStatus mrnnt_forward(const mrnnt_problem *p, void *workspace, size_t workspace_bytes, float *costs_dev,
                         int with_beta, hipStream_t stream);

/* Backward: grads[r, v] = grad_scale[b(r)] * dcost_b / dacts[r, v] for every row (out-of-band rows
 * are written with 0 * grad_scale, padding rows of the padded layout with 0; no pre-zeroing needed).
 * grads has the layout and element type of acts. grad_scale (device fp32 [B], or [1] with
 * grad_scale_broadcast) may be NULL (= 1).
 * Requires a preceding mrnnt_forward(with_beta=1) on the same workspace and inputs. */
RNNTStatus mrnnt_backward(const mrnnt_problem *p, const void *workspace, const float *grad_scale, void *grads,
                          hipStream_t stream);

/* forward(with_beta = grads != NULL) followed by backward. */
RNNTStatus mrnnt_cost_and_grad(const mrnnt_problem *p, void *workspace, size_t workspace_bytes, float *costs_dev,
                               void *grads, const float *grad_scale, hipStream_t stream);

/* Forward log-likelihoods from the workspace (device double [B]), for debugging/inspection:
 * ll_fwd = alpha(T-1, S), ll_bwd = beta(0, 0). Either may be NULL. Asynchronous on `stream`. */
RNNTStatus mrnnt_read_loglik(const mrnnt_problem *p, const void *workspace, double *ll_fwd_dev, double *ll_bwd_dev,
                             hipStream_t stream);

/* Per-row state of the last mrnnt_forward on this workspace, for inspection / parity tests: den[r] (fp32
 * log-softmax denominator -max - log sum exp(z - max) of the rows the forward reduced: the in-band or
 * alignment-window rows, 0 elsewhere), alpha[r] = alpha(t, s) and beta[r] = beta(t, s) (fp64, -inf outside the
 * band; beta only after with_beta = 1), all in the packed lattice row order r = sum_{b'<b} T_b'(S_b'+1) +
 * t (S_b+1) + s. Device buffers of N elements; any may be NULL. Asynchronous on `stream`. */
RNNTStatus mrnnt_read_state(const mrnnt_problem *p, const void *workspace, float *den_dev, double *alpha_dev,
                            double *beta_dev, hipStream_t stream);

/* Log-softmax denominator of EVERY lattice row, den[r] = -max_v z - log sum_v exp(z - max) in the packed row
 * order of mrnnt_read_state (the reference's denom_host(), gpu_workspace_manager.h:137-141, whose reduce covers
 * all rows): the rows the last mrnnt_forward reduced are copied from the workspace, the others (outside the band or
 * the alignment window, which the forward never reads) are reduced from acts here. den_dev: device fp32 [N].
 * Asynchronous on `stream`. */
RNNTStatus mrnnt_read_denoms(const mrnnt_problem *p, const void *workspace, float *den_dev, hipStream_t stream);

/* The alignment band of the problem in the reference's [B, ld] layout (gpu_workspace_manager.h:167-177,191-219):
 * min_dev[b*ld + t] / max_dev[b*ld + t] = the lowest / highest label position alpha(t, .) may take, for t < T_b;
 * 0 / S_b for t >= T_b and for every t without an alignment (the reference's initial values, :317-328). Builds the
 * band in `workspace` from p->alignment (device kernels, as mrnnt_forward does), so it needs no preceding
 * forward. ld >= max T_b; either output may be NULL. Asynchronous on `stream`. */
RNNTStatus mrnnt_read_band(const mrnnt_problem *p, void *workspace, int *min_dev, int *max_dev, int64_t ld,
                           hipStream_t stream);

/* Message describing the last non-success status returned on this thread. */
const char *mrnnt_last_error(void);

/* Number of in-band lattice rows whose acts the gradient kernel reads ("live" rows) for the problem of the
 * last mrnnt_forward(with_beta=1) on this workspace, written to *count_dev (device uint64). A row whose
 * occupancy exp(alpha(t-1,s) + beta(t,s) - ll) is below e^-110 has an exactly-zero fp32 gradient and is
 * stored without reading acts ("occ_skip" knob, on by default). Inspection/bench only; asynchronous. */
RNNTStatus mrnnt_grad_live_rows(const mrnnt_problem *p, const void *workspace, unsigned long long *count_dev,
                                hipStream_t stream);

/* ---- host implementation (RNNT_CPU; reference cpu_rnnt.h / pytorch_binding cpu_monotonic_rnnt) --------
 * The same problem description with every pointer on the HOST: acts (fp32 only), labels, alignment,
 * T_host / S_host (T_dev / S_dev are ignored), workspace, costs, grads, grad_scale. Lengths, strides and
 * labels are validated (a label outside [0, V) is RNNT_STATUS_INVALID_VALUE). num_threads <= 0 uses the
 * OpenMP default. Results follow the GPU path's semantics (fp64 recursion, occupancy-exact zero rows). */
RNNTStatus mrnnt_cpu_workspace_size(const mrnnt_problem *p, size_t *bytes);

/* Log-softmax row reduce + alpha (and, if with_beta, beta) recursion; costs[b] = -log p (may be NULL). */
RNNTStatus mrnnt_cpu_forward(const mrnnt_problem *p, void *workspace, size_t workspace_bytes, float *costs,
                             int with_beta, int num_threads);

/* grads[r, v] = grad_scale[b(r)] * dcost_b / dacts[r, v] for every row (grad_scale may be NULL = 1), after
 * mrnnt_cpu_forward(with_beta=1) on the same workspace and inputs. grads may be acts itself (in place). */
RNNTStatus mrnnt_cpu_backward(const mrnnt_problem *p, const void *workspace, const float *grad_scale, float *grads,
                              int num_threads);

/* mrnnt_read_state for the host implementation (host buffers). */
RNNTStatus mrnnt_cpu_read_state(const mrnnt_problem *p, const void *workspace, float *den, double *alpha,
                                double *beta);

/* ---- fused joint network + loss (extension) -------------------------------------
 * The logits are not an input: z(b,t,s,:) = weight * tanh(enc[b,t,:] + pred[b,s,:]) + bias is formed on the
 * matrix cores inside the log-softmax and gradient passes and never stored (bf16 operands, fp32 accumulate).
 * Labels, lengths, blank and costs have the meaning of mrnnt_problem. H must be 128, 256, 384, 512 or 640. */
typedef struct mrnnt_joint_problem {
    int B;
    int V;
    int H;
    int blank;
    const int *T_host;       /* host [B] */
    const int *S_host;       /* host [B] */
    const int *T_dev;        /* device [B] */
    const int *S_dev;        /* device [B] */
    const int *labels;       /* device [B, label_stride] */
    int64_t label_stride;
    const void *enc;         /* device bf16, row (b, t) at enc + b*enc_stride + t*H (elements) */
    int64_t enc_stride;      /* multiple of 8, >= max_b T_b * H */
    const void *pred;        /* device bf16, row (b, s) at pred + b*pred_stride + s*H */
    int64_t pred_stride;     /* multiple of 8, >= (max_b S_b + 1) * H */
    const void *weight;      /* device bf16 [V, H] */
    const float *bias;       /* device fp32 [V] or NULL */
    const int *alignment;    /* device [B, align_stride] or NULL: restriction as in mrnnt_problem */
    int64_t align_stride;
    int align_blank;
    int max_shift;
    int64_t hact_ld;         /* (version 3) Hact row stride in elements, 0 = H; a multiple of 8 > H makes
                                mrnnt_joint_backward write columns H .. hact_ld-1 of every row as [1, 0, ...],
                                so that the dweight GEMM G^T Hact also yields dbias = sum_i G[i] in column H */
    float *dbias;            /* (version 8) device fp32 [V] or NULL: mrnnt_joint_backward ADDS sum_i G[i] (the fp32
                                values before their bf16 rounding) into it -- zero it first; H <= 512 only, and V small
                                enough for its per-wave LDS column sums (mrnnt_joint_backward reports otherwise). Summed
                                in a fixed order: bitwise reproducible (version 9; version 8 used float atomics) */
    void *reduce_scratch;    /* (version 9) device memory for mrnnt_joint_reduce, >= mrnnt_joint_reduce_scratch_bytes,
                                or NULL (a slower one-block-per-utterance form runs); e.g. G once dH = G weight exists */
    size_t reduce_scratch_bytes;
    const unsigned long long *live_count_dev; /* (version 12) device uint64 or NULL: the count mrnnt_joint_live_rows
                                wrote. When set, the n_live argument of mrnnt_joint_backward (and of mrnnt_joint_dpre /
                                mrnnt_joint_reduce / mrnnt_joint_reduce_pre) is a host-known UPPER BOUND on the count
                                (mrnnt_joint_row_bound) and the kernels take the count from this word: no device-to-host
                                read between the forward and the backward, so a training step can be captured in a HIP
                                graph. mrnnt_joint_backward then also writes rows [count, n_live) of G and Hact as zeros,
                                so library GEMMs over all n_live rows (dweight, dH) see zero rows there. */
} mrnnt_joint_problem;

RNNTStatus mrnnt_joint_workspace_size(const mrnnt_joint_problem *p, size_t *bytes);

/* (version 12) A host-known upper bound on the live-row count of mrnnt_joint_live_rows: the lattice rows inside the
 * monotonic band, from the host lengths (no device read). Size G / Hact with it under p->live_count_dev. */
RNNTStatus mrnnt_joint_row_bound(const mrnnt_joint_problem *p, int64_t *rows);

/* Forward: costs_dev[b] = -log P(labels_b | enc_b, pred_b); with_beta as in mrnnt_forward. */
RNNTStatus mrnnt_joint_forward(const mrnnt_joint_problem *p, void *workspace, size_t workspace_bytes,
                               float *costs_dev, int with_beta, hipStream_t stream);

/* After mrnnt_joint_forward(with_beta=1): list the live lattice rows (those with a non-zero fp32 logit
 * gradient) in the workspace and write their number to *count_dev (device uint64). */
RNNTStatus mrnnt_joint_live_rows(const mrnnt_joint_problem *p, void *workspace, unsigned long long *count_dev,
                                 hipStream_t stream);

/* After mrnnt_joint_live_rows: for live row i (n_live = the count it produced, read back by the caller),
 * G[i, :] = grad_scale[b] * dcost_b/dz (bf16 [n_live, V]), Hact[i, :] = tanh(enc + pred) (bf16 [n_live, H]),
 * bt_idx[i] = b*(enc_stride/H) + t and bs_idx[i] = b*(pred_stride/H) + s (int64; either may be NULL). Then
 * dweight = G^T Hact, dbias = sum_i G[i] (= column H of G^T Hact when hact_ld > H), and with
 * dpre = (G weight) * (1 - Hact^2):
 * denc[bt_idx[i]] += dpre[i], dpred[bs_idx[i]] += dpre[i]. grad_scale may be NULL (= 1). */
RNNTStatus mrnnt_joint_backward(const mrnnt_joint_problem *p, void *workspace, int64_t n_live,
                                const float *grad_scale, void *G, void *Hact, int64_t *bt_idx, int64_t *bs_idx,
                                hipStream_t stream);

/* (version 10) After mrnnt_joint_backward: dpre = (G weight) * (1 - Hact^2), bf16 [n_live, H], on hand-written MFMA
 * tiles (mrnnt_joint_gemm.hip): the dH GEMM with the tanh derivative in its epilogue. weight_t is the weight
 * transposed, bf16 [H, V] row-major; Hact as mrnnt_joint_backward wrote it (row stride p->hact_ld, 0 = H). Needs
 * H = 256 or 512 and V a multiple of 8 (RNNT_STATUS_INVALID_VALUE otherwise: use a library GEMM for dH and
 * mrnnt_joint_reduce with Hact). Sum dpre with mrnnt_joint_reduce_pre. */
RNNTStatus mrnnt_joint_dpre(const mrnnt_joint_problem *p, int64_t n_live, const void *G, const void *weight_t,
                            const void *Hact, void *dpre, hipStream_t stream);

/* After mrnnt_joint_backward, with dH = G weight (bf16 [n_live, H], e.g. a library GEMM): accumulate
 * dpre = dH * (1 - Hact^2) into d_enc (fp32, enc's [B, enc_stride/H, H] shape; rows (b, t < T_b) are
 * overwritten) and d_pred (fp32, pred's shape; added to: zero it first). Zero d_enc's padding rows yourself.
 * Hact is required (RNNT_STATUS_INVALID_VALUE when NULL with n_live > 0). Every sum has a fixed order (bitwise reproducible). p->reduce_scratch (version 9) lets it run on blocks of frames
 * whose d_pred sums are then added in block order; see mrnnt_joint_reduce_scratch_bytes. */
RNNTStatus mrnnt_joint_reduce(const mrnnt_joint_problem *p, void *workspace, int64_t n_live, const void *dH,
                              const void *Hact, float *d_enc, float *d_pred, hipStream_t stream);

/* (version 11) mrnnt_joint_reduce for a dH that already holds dpre = dH * (1 - Hact^2) (mrnnt_joint_dpre's output,
 * bf16 [n_live, H]): the same sums of dpre into d_enc / d_pred, in the same fixed order. (Version 10 signalled this
 * with Hact = NULL on mrnnt_joint_reduce, which made a forgotten Hact a silent wrong gradient.) */
RNNTStatus mrnnt_joint_reduce_pre(const mrnnt_joint_problem *p, void *workspace, int64_t n_live, const void *dpre,
                                  float *d_enc, float *d_pred, hipStream_t stream);

/* (version 9) Bytes of p->reduce_scratch for the blocked form of mrnnt_joint_reduce. */
RNNTStatus mrnnt_joint_reduce_scratch_bytes(const mrnnt_joint_problem *p, size_t *bytes);

/* Nontemporal zero fill of `bytes` (a multiple of 16) at `dst` (16-byte aligned device memory), in the gradient
 * pass's store pattern. The Python surface times it once over a newly allocated large grads buffer to pick a
 * fast-writing physical placement; also usable as a plain fill. Asynchronous on `stream`. */
RNNTStatus mrnnt_fill_zero(void *dst, size_t bytes, hipStream_t stream);

int mrnnt_version(void);

/* Kernel-time accounting over HIP events recorded around each launch on its stream.
 * enable=1 starts recording (clearing previous records). mrnnt_profile_read synchronises the
 * recorded events and returns per-kernel totals in ms and launch counts for
 *   [0] band, [1] log-softmax row reduce, [2] alpha/beta DP, [3] logit gradient, [4] setup,
 *   [5] joint forward, [6] joint backward, [7] joint reduce, [8] chase launch (log-softmax + alpha/beta),
 *   [9] joint dpre GEMM (version 10). */
void mrnnt_profile_enable(int enable);
int mrnnt_profile_read(double *total_ms, int64_t *launches, int n);

#ifdef __cplusplus
}
#endif

#endif /* MONOTONIC_RNNT_MRNNT_H */
