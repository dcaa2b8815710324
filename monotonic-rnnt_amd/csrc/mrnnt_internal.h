// mrnnt_internal.h -- device problem descriptor, launch knobs and kernel launchers shared by the host
// code (mrnnt_capi.cpp) and the kernels (mrnnt_*.hip). Not installed; not part of the ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mrnnt_host.h"

namespace mrnnt {

// Element type of acts and grads (the math is fp32/fp64 inside the kernels).
enum ElemType { ELEM_F32 = 0, ELEM_BF16 = 1, ELEM_F16 = 2 };

// Device-resident lengths (mrnnt_problem.lengths_on_device): the setup kernel of the call validates the lengths
// and publishes what the host could not plan, for the later kernels of the same call (one 64-byte line).
// The two log-probabilities of a lattice row the recursion reads, side by side: one 16-byte access per row (the
// alpha step takes lpe(t, s - 1) as the shifted sum alpha(t - 1, s - 1) + lpe(t, s - 1) formed in lane s - 1).
struct alignas(16) Lp {
    double b;  // lpb = z[r, blank] + den[r]
    double e;  // lpe = z[r, label(s)] + den[r] (s < S; s == S: den[r])
};

struct DynWords {
    int status;                // 0, or RNNT_STATUS_INVALID_VALUE: the lengths failed validation (nothing runs)
    int pad_;
    int64_t num_cols;          // sum_b T_b
    int64_t num_rows;          // sum_b T_b (S_b + 1)
    int64_t col_mul;           // scattered column order: a multiplier coprime with num_cols (0: in order)
    unsigned long long steal;  // work counter of the log-softmax's column walk (zeroed by the setup kernel)
    int64_t spare_[3];
};

// Everything a kernel needs, passed by value as a kernel argument.
// Internal per-row arrays use the packed lattice row r = row_off[b] + t*(S_b+1) + s (column (b, t) at
// col_off[b] + t). acts/grads rows use the caller's layout: packed (the same r) or padded
// [B, pad_T, pad_S1, V] with row (b*pad_T + t)*pad_S1 + s.
struct DevProblem {
    const void *acts;           // [rows, V] of elem type
    const int *labels;          // [B, label_stride]
    int64_t label_stride;
    const int *T;               // [B]
    const int *S;               // [B]
    const int64_t *row_off;     // [B+1] (workspace, built by the setup kernel)
    const int64_t *col_off;     // [B+1]
    const int *col_b;           // [cols] utterance of each lattice column (setup kernel)
    const int *min_s;           // [cols] alignment band (nullptr = unrestricted)
    const int *max_s;           // [cols]
    int B, V, blank;
    int occ_skip;               // skip the acts read of rows whose gradient is exactly zero (mrnnt_grad.hip)
    int64_t num_cols;           // sum_b T_b
    int64_t num_rows;           // N = sum_b T_b (S_b + 1)
    int64_t pad_T, pad_S1;      // padded acts layout (pad_S1 == 0: packed)
    int64_t scale_stride;       // upstream-gradient stride: grad_scale[b * scale_stride] (0 = one value for all)
    int64_t col_mul;            // column visiting order of the streaming kernels (visit_col): 0 in order, > 0 the
                                // i-th column visited is (i * col_mul) % num_cols (coprime), < 0 XCD-chunked
    float *den;                 // [N]  log-softmax denominator  -max - log sum exp(z - max)
    Lp *lp;                     // [N]  {z[r, blank] + den[r], z[r, label(s)] + den[r] (s < S)}; 64 pads either side
    double *alpha;              // [N]  alpha(t, s), masked cells = -inf
    double *beta;               // [N]  beta(t, s)
    double *ll;                 // [B]  alpha(T-1, S)
    double *llb;                // [B]  beta(0, 0)
    DynWords *dyn;              // device-resident lengths: num_cols / num_rows / col_mul above are host bounds and
                                // the kernels take the real values from here (resolve_dyn); nullptr otherwise
    int steal;                  // log-softmax: columns past the grid handed out by dyn->steal (work stealing)
    // device-resident lengths planned inside the log-softmax launch itself (dyn_fused; B <= 64, no alignment):
    // every wave validates the lengths and locates its columns from registers, and the launch publishes the
    // lattice offsets, the column map and the DynWords for the later kernels -- no separate setup kernel
    int dyn_fused;
    int64_t s_cap, t_cap, s1_cap;  // validation limits (S_b <= s_cap; T_b <= t_cap, S_b + 1 <= s1_cap when > 0)
    int64_t scatter_above;         // publish a scattered-order multiplier when there are more columns than this
    int *status_host;              // device address of the caller's host-mapped status word, or nullptr
};

// Fused joint network (mrnnt_joint.hip): logits z(b,t,s,:) = W * tanh(enc[b,t,:] + pred[b,s,:]) + bias are
// formed on MFMA inside the log-softmax and gradient passes and never stored. Operands are bf16 bit patterns.
struct JointArgs {
    const unsigned short *enc;   // [B, *, H]: row (b, t) at enc + b*enc_sb + t*H
    int64_t enc_sb;
    const unsigned short *pred;  // [B, *, H]: row (b, s) at pred + b*pred_sb + s*H
    int64_t pred_sb;
    const unsigned short *W;     // [V, H] (torch Linear weight layout)
    const float *bias;           // [V] or nullptr
    int H;
    const int *lcol;             // row list: lattice column and label position of entry i
    const int *ls;
    int64_t n;                   // entries in the list (an upper bound when n_dev is set)
    const unsigned long long *n_dev;  // entries in the list, on the device (alignment windows), or nullptr
    // backward outputs, one row per list entry
    unsigned short *G;           // [n, V] bf16 dL/dz
    unsigned short *Hact;        // [n, hact_ld] bf16 tanh(enc + pred) (columns >= H: [1, 0, ...])
    int64_t hact_ld;             // Hact row stride (elements), >= H
    int64_t *bt_idx;             // [n] b * enc_sb / H + t   (row of enc viewed as [B * T_slots, H])
    int64_t *bs_idx;             // [n] b * pred_sb / H + s  (row of pred viewed as [B * S_slots, H])
    const float *scale;          // [B] upstream dL/dcost or nullptr
    float *dbias;                // [V] fp32: the backward adds sum_i G[i] into it (16x16x32 backward only), or nullptr
    float *dbias_part;           // with dbias: the backward's per-workgroup column sums, then the segment sums
                                 // (joint_dbias_part_bytes), summed in order by launch_joint_dbias_sum
    const int *wplain;           // forward only: device flag, 1 when no logit can leave [-64, 64] (the weight bound of
                                 // joint_wbound_kernel) -- the epilogue then sums exp(z) without a running max
    int opt = 3;                 // forward / backward loop forms (development A/B of round 6): bit 0 the weight-chunk DMA
                                 // from loop-invariant per-lane offsets, bit 1 log2 e folded into a prescaled bias row
    int probe;                   // development build, timing probes (results wrong): forward bit 0 every row's
                                 // activation reads pred row s = 0, bit 1 enc row t = 0, bit 3 the running-max
                                 // epilogue whatever the weight bound; reduce bit 2 no frame barriers / d_enc sum, bit 4 its
                                 // timeline stamps (g_reduce_trace)
};

// Row lists over the lattice: mode 0 = every in-band row, mode 1 = live rows (needs alpha/beta/ll).
hipError_t launch_row_list(const DevProblem &p, int mode, int64_t *col_cnt, int *lcol, int *ls,
                           unsigned long long *total, hipStream_t stream);
hipError_t launch_joint_forward(const DevProblem &p, const JointArgs &j, hipStream_t stream);
// flag = 1 when max_v (sum_h |W[v, h]| + |bias[v]|) <= 64 (then |z| <= 64 for every logit: |tanh| <= 1), else 0
hipError_t launch_joint_wbound(const unsigned short *W, const float *bias, int V, int H, int *flag, hipStream_t stream);
hipError_t launch_joint_backward(const DevProblem &p, const JointArgs &j, hipStream_t stream);
hipError_t launch_joint_reduce(const DevProblem &p, const JointArgs &j, const int64_t *off, int T_max, int S_max,
                               const unsigned short *dH, float *d_enc, float *d_pred, void *scratch,
                               size_t scratch_bytes, hipStream_t stream);
// scratch of the blocked d_enc / d_pred reduce (per-block d_pred sums and label ranges)
size_t joint_reduce_scratch_bytes(int B, int T_max, int S_max, int H);
// dpre = (G W) * (1 - Hact^2) on MFMA (mrnnt_joint_gemm.hip); H in {256, 512}, V % 8 == 0
hipError_t launch_joint_dpre(const unsigned short *G, const unsigned short *Wt, const unsigned short *Hact,
                             int64_t hact_ld, unsigned short *dpre, int64_t n, int V, int H, hipStream_t stream);
hipError_t launch_zero(void *ptr, size_t bytes, hipStream_t stream);
// dbias: the fixed-order sum of the backward's per-workgroup column sums (scratch: joint_dbias_part_bytes)
size_t joint_dbias_part_bytes(int64_t n_max, int V);
hipError_t launch_joint_dbias_sum(const JointArgs &j, int V, hipStream_t stream);
// rows [*count_dev, n) of G ([n, V]) and Hact ([n, hact_ld]) as zeros (the live count on the device, n a host bound)
hipError_t launch_joint_tail_zero(unsigned short *G, int V, unsigned short *Hact, int64_t hact_ld, int64_t n,
                                  const unsigned long long *count_dev, hipStream_t stream);
// LDS the fused joint kernels need at least (two weight-tile buffers + the bias row); at most 160 KiB per CU
size_t joint_min_lds_bytes(int H, int V);
// ... and the 16x16x32 backward when it sums dbias (one column-sum row per wave more)
size_t joint_dbias_lds_bytes(int H, int V);

// Launch-shape knobs (experiment hook: mrnnt_tune in mrnnt_capi.cpp). Defaults are the tuned values.
struct Tuning {
    int softmax_variant = 13;     // log-softmax kernel: 13 -> rows of <= 64 vectors on 16-lane groups (4 rows per
                                  // wave), longer single-chunk rows per wave with the wave max first, longer rows with
                                  // a running max, 2 rows per wave; 21 -> no 16-lane groups; 16 -> running max for
                                  // every row; 14 / 15 -> running max, 1 / 4 rows; 0/2 -> first kernel, 1/2 rows
    int grad_variant = 5;         // gradient kernel: 5 -> staged coefficients (1 / 2 / 4 rows per wave for rows of
                                  // >= 192 / >= 96 / fewer vectors; short rows loaded nontemporally: per-row
                                  // kernel, 2 rows), 6 -> staged, 2 rows;
                                  // 0 / 2 -> per-row coefficients, default / 2 rows; 3 -> row-stride sweep (packed)
    int softmax_grid_per_cu = 0;  // workgroups (of 4 waves) per CU; 0 = one workgroup per lattice column
    int grad_grid_per_cu = 32;    // same for the gradient kernel
    int nt_store = 1;             // nontemporal stores of grads
    int nt_load = 2;              // loads of acts in both streaming kernels: 1 nontemporal, 0 default policy,
                                  // 2 by size (nt_acts_loads)
    int occ_skip = 1;             // gradient: no acts read for rows with log-occupancy < kDeadLogOcc
    int joint_bwd_mfma = 16;      // fused joint backward MFMA tile for H <= 512: 16 (v_mfma_f32_16x16x32_bf16) or 32
                                  // (32x32x16, development build); H = 640 always 32
    int joint_reduce_sparse = 0;  // joint d_enc/d_pred reduce: 0 / 1 frame by frame, one workgroup per utterance and
                                  // hidden slice (fixed order, bitwise reproducible); 2 (development build) the
                                  // row-parallel kernel with float atomics
    int dp_halo = 2;              // alpha/beta: halo recursion (one barrier per 8 steps, 8 / 16-step prefetch
                                  // blocks: 1 / 2) for S+1 <= 448; 0: one barrier per step
    int dp_lean = 1;              // halo recursion without an alignment: 1 -> the lean step (row pointers advanced
                                  // per frame + lane offsets, bound-ctrl DPP shifts, no band mask); 0 -> masked step
    int col_scatter = 2;          // visit columns in a scattered order (DevProblem::col_mul): bit 0 log-softmax,
                                  // bit 1 gradient
    int dyn_fused = 1;            // device-resident lengths, B <= 64, no alignment: plan inside the log-softmax launch
                                  // (0: a separate setup kernel)
    int chase = 1;                // forward as one launch, the recursion chasing the log-softmax (mrnnt_chase.hip) where
                                  // it applies (no alignment, f32 rows of <= 256 vectors, S + 1 <= 224; device lengths:
                                  // B <= 64) and pays (chase_pays)
    int chase_grid_per_cu = 0;    // log-softmax workgroups of the chase launch per CU (0: one per slot)
    int chase_wait_us = 100;      // a chase recursion wave computes a column itself after waiting this long for it
    int chase_stage = 1;          // one-wave chase recursion: lp frames staged in LDS by a loader wave (0: direct
                                  // gated loads; development build)
    int chase_delay_us = 0;       // development probe: every chase producer workgroup starts this late
    int chase_probe = 0;          // development probe: ChaseArgs::probe (the staged walk's step cost; results wrong)
    int joint_opt = 3;            // JointArgs::opt (development A/B of the round-6 forward loop forms)
    int chase_pair = 1;           // staged chase walk: 1 one log-sum-exp per frame (the product); development A/B of
                                  // round 6: 2 frame pairs on the walk, 3 frame pairs with the side values on wave 2
    int chase_early_free = 1;     // staged chase walk: ring slots freed when read into registers (0: after their use)
    int chase_ring = 64;          // staged chase walk: cap on the LDS ring's frames (16: round 5's depth)
    int joint_reduce_hact = 1;    // joint reduce: 1 reads Hact; 0 (development build) recomputes the activation from
                                  // enc / pred (the gradient pass's bits; measured slower, mrnnt_joint.hip)
    int joint_reduce_pad = 1;     // joint reduce: accumulator LDS pitch HS + 1 (0: HS, development A/B; bit-identical)
    int joint_trace = 0;          // development build: the joint forward with its timeline stamps (tools/joint_trace.py)
    int joint_probe = 0;          // development probe: JointArgs::probe of the joint forward (results wrong)
    int joint_dpre_nw = 0;        // joint dpre GEMM (mrnnt_joint_gemm.hip): 0 -> the 16x16x32 form (8 waves, 256 rows x
                                  // 256 h per workgroup, both operands through LDS, fragments a chunk ahead, DMA issue
                                  // interleaved with the MFMA groups, LDS-staged epilogue); development build: 1 / 2
                                  // the 32x32x16 direct / persistent forms (G straight to registers, round 5), 4 / 8 /
                                  // 42 / 81 / 421 / ... staged 32x32x16 tile shapes (tens digit: waves, then row tiles,
                                  // stages; trailing 1: LDS epilogue, 2: plain dH), 160-167 the 16x16x32 form's
                                  // stage / priority / interleave / Hact-prefetch A/Bs
    int joint_dpre_abl = 0;       // development ablations of the staged dpre forms: bit 0 no epilogue, bit 1 G rows
                                  // from one L2-resident row tile per XCD (results wrong)
    int col_xcd = 0;              // XCD-chunked column order (visit_col, col_mul < 0; overrides col_scatter): bit 0
                                  // log-softmax, bit 1 gradient
};
Tuning &tuning();

// The launch variants the knobs above select besides the tuned defaults are compiled into the development build
// only (libmonotonic_rnnt_amd_dev.so, -DMRNNT_DEVTOOLS, where mrnnt_tune can reach them); the product library,
// whose knobs never change, carries the default kernels alone.
#ifdef MRNNT_DEVTOOLS
constexpr bool kVariants = true;
#else
constexpr bool kVariants = false;
#endif

// Acts tensors up to this size stay in the 256 MiB Infinity Cache between the log-softmax pass and the gradient
// pass's re-read when both load them with the default policy (MI355X_MICROARCH.md, Infinity Cache residency:
// table + every byte streamed in between <= ~256 MiB); larger ones stream with nontemporal loads.
constexpr int64_t kCachedActsBytes = 160ll << 20;

inline bool nt_acts_loads(const DevProblem &p, int elem_bytes) {
    const int k = tuning().nt_load;
    if (k != 2) return k != 0;
    const int64_t rows = p.pad_S1 ? (int64_t)p.B * p.pad_T * p.pad_S1 : p.num_rows;
    return rows * (int64_t)p.V * elem_bytes > kCachedActsBytes;
}

// Kernel-family ids for the profiling counters (mrnnt_profile_read order).
enum KernelId { K_BAND = 0, K_SOFTMAX = 1, K_DP = 2, K_GRAD = 3, K_SETUP = 4, K_JOINT_FWD = 5, K_JOINT_BWD = 6,
                K_JOINT_RED = 7, K_CHASE = 8, K_JOINT_DPRE = 9, K_COUNT = 10 };

// lp (may be null): zero its 64 pad entries either side of [0, n)
hipError_t launch_setup(const int *T, const int *S, int B, int64_t *row_off, int64_t *col_off, int *col_b,
                        Lp *lp, int64_t n, hipStream_t stream);
// Device-resident lengths: lattice offsets, column map, validation and the DynWords in one launch (B workgroups).
struct DynSetupArgs {
    const int *T;
    const int *S;
    int B;
    int packed;         // 1: sum_b T_b (S_b+1) must equal rows; 0 (padded layout): rows is an upper bound
    int64_t rows;
    int64_t cols_cap;   // capacity of col_b (and of the alignment band arrays)
    int64_t S_cap;      // S_b <= S_cap (the label row stride)
    int64_t T_cap;      // T_b <= T_cap (alignment row stride / pad_T), 0 = unbounded
    int64_t S1_cap;     // S_b + 1 <= S1_cap (pad_S1), 0 = unbounded
    int64_t scatter_above;  // publish a scattered column-order multiplier when there are more columns than this
                            // (the gradient's grid); INT64_MAX: never
    int64_t *row_off;
    int64_t *col_off;
    int *col_b;
    Lp *lp;             // lp array: its 64 entries either side of [0, rows) are zeroed
    DynWords *dyn;
    int *status_host;   // device address of the caller's host-mapped status word, or nullptr
};
hipError_t launch_setup_dyn(const DynSetupArgs &a, hipStream_t stream);
// mrnnt_read_denoms: den of every row (copied where the forward reduced it, reduced from acts elsewhere)
hipError_t launch_den_all(const DevProblem &p, int elem, float *den_out, hipStream_t stream);
// mrnnt_read_band: min / max allowed s in the [B, ld] layout
hipError_t launch_band_read(const DevProblem &p, int *min_out, int *max_out, int64_t ld, hipStream_t stream);
hipError_t launch_align(const DevProblem &p, const int *alignment, int64_t align_stride, int align_blank,
                        int max_shift, int *mtmp, int *min_s, int *max_s, hipStream_t stream);
hipError_t launch_softmax(const DevProblem &p, int elem, int grid, hipStream_t stream);
// mrnnt_read_state: alpha / beta cells outside the compute band set to -inf (either may be null)
hipError_t launch_mask_state(const DevProblem &p, double *alpha, double *beta, hipStream_t stream);
// the reference manager's view: fp32 alpha / beta (band-masked) and log-likelihoods (any may be null)
hipError_t launch_state_f32(const DevProblem &p, float *alpha, float *beta, float *ll, float *llb, hipStream_t stream);
hipError_t launch_dp(const DevProblem &p, int S_max, int with_beta, float *costs, hipStream_t stream);

// The chase launch (mrnnt_chase.hip): log-softmax and alpha / beta recursion in one launch, the recursion consuming
// columns as they are published. Ready flags: one 64-bit word per lattice column, holding the tag of the launch that
// published it (never cleared: every launch derives a tag of its own from its dispatch id).
struct ChaseArgs {
    unsigned long long *flags;
    int64_t slots;             // of the production order (host lengths: chase_slots; device lengths: 0, planned on the
                               // device from the lengths)
    unsigned long long epoch;  // fresh per call (never 0), mixed with the dispatch id into the launch's tag
    uint32_t budget;           // ticks of the 100 MHz constant clock a recursion wave waits for a column before it
                               // computes the column itself
    uint32_t delay;            // development probe (ticks): producer workgroups start this late
    int stage;                 // one-wave recursion: LDS-staged frames (the product's only form) or direct loads
    int probe;                 // development probe of the staged walk's step (results wrong): bit 0 no alpha/beta
                               // stores, bit 1 a max in place of the log-sum-exp, bit 2 no ring reads after the first P
    int pair;                  // staged walk: frames per dependent log-sum-exp (1, or 2: a three-term step)
    int early_free;            // staged walk: ring slots are freed once read into registers (else after their use)
    int ring;                  // staged walk: at most this many frames in the LDS ring (development A/B)
};
// The log-softmax body the chase launch carries for f32 rows of V elements: 0 rows on 16-lane groups (<= 64
// vectors), 2 / 3 single-chunk rows of <= 128 vectors (full / partial chunk), 4 / 5 of <= 256; -1 none.
inline int chase_body_shape(int V) {
    if (V <= 0 || V % 4) return -1;
    const int VL = V / 4;
    if (VL <= 64) return 0;
    if (VL >= 96 && VL <= 128) return VL == 128 ? 2 : 3;
    if (VL >= 192 && VL <= 256) return VL == 256 ? 4 : 5;
    return -1;
}
// the body for this problem (f32 acts, 16-byte aligned), -1 for none
int chase_body(const DevProblem &p, int elem);
inline int64_t chase_slots(int B, int T_max, int with_beta) {
    return (with_beta ? (int64_t)(T_max + 1) / 2 : (int64_t)T_max) * (with_beta ? 2 * (int64_t)B : (int64_t)B);
}
// development build: columns chase recursion waves computed themselves (since the last reset)
unsigned long long chase_helped(bool reset);
int chase_trace(unsigned long long *out, int n);  // development build: the chase launch timeline
int chase_walk_trace(unsigned long long *out, int n);  // development build: walk / loader progress (probe bit 8)
int joint_trace(unsigned long long *out, int n);  // development build: the fused joint forward's wave timeline
int joint_reduce_trace(unsigned long long *out, int n);  // development build: the joint reduce's timeline
hipError_t launch_chase(const DevProblem &p, const ChaseArgs &c, int elem, int S_max, int with_beta, int producers,
                        float *costs, hipStream_t stream);
hipError_t launch_grad(const DevProblem &p, int elem, const float *scale, void *grads, int grid, hipStream_t stream);
hipError_t launch_count_live(const DevProblem &p, unsigned long long *count, hipStream_t stream);
hipError_t launch_pad_zero(const DevProblem &p, int elem, void *grads, hipStream_t stream);
hipError_t launch_fill_zero(void *dst, size_t bytes, int grid_max, hipStream_t stream);

// kDeadLogOcc (the exact-zero gradient-row threshold) is in mrnnt_host.h, shared with the CPU implementation.

// Largest S+1 the recursion instantiations cover (8 waves x 64 lanes x 4 cells per lane).
constexpr int kMaxLabelsPlusOne = 2048;
// Padding (elements) around the lp arrays so the recursion's whole-workgroup row loads never leave the
// allocation (>= the largest lanes x cells block).
constexpr int64_t kLpPad = 2048 + 64;

}  // namespace mrnnt
