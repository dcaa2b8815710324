// mrnnt_kernels.hip -- the monotonic RNN-T hot path for CDNA4 (gfx950, wave64).
//
// Three kernels carry the work (plus two tiny metadata kernels):
//   softmax_*_kernel : one pass over the in-band rows of acts. Per row: online (max, sum-exp) per lane,
//                      one wave64 butterfly reduce, den = -max - log(sum); the blank and label logits
//                      are captured from registers on the way, so it also emits lpb/lpe (the only
//                      two log-probs the lattice recursion needs).  Replaces reduce.h:79-154 (two
//                      full passes over acts + host syncs) and the strided acts gathers of
//                      gpu_rnnt_kernel.h:80-84.
//   dp_kernel        : alpha and beta recursions concurrently, one wave per (utterance, direction);
//                      the s axis lives in registers (K cells per lane), the s-1 / s+1 neighbour
//                      crosses lanes with one shuffle per step, lp rows stream through a D-deep
//                      register prefetch ring. fp64 state, fp32 hardware transcendentals for the
//                      bounded log1p(exp(-d)) term. Replaces gpu_rnnt_kernel.h:121-237.
//   grad_*_kernel    : the bandwidth-bound pass: reads the in-band rows of acts once, writes every
//                      row of grads once (zeros outside the band, as gpu_rnnt_kernel.h:266-271),
//                      per-row coefficients precomputed in fp64 from alpha/beta/den/lpb/lpe, one
//                      exp2 + fma per element, dL/dcost scale fused. Replaces gpu_rnnt_kernel.h:239-288
//                      plus the Torch glue's extra scale pass (monotonic_rnnt_op.py:96-118).
//
// Work decomposition of the streaming kernels: a persistent grid walks the lattice columns (b, t)
// (grid-stride, a monotone per-workgroup utterance cursor, no per-block b search); inside a column
// the four waves of a workgroup take rows s. All offsets are 64-bit.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mrnnt_internal.h"

namespace mrnnt {

#define NEG_INF_F (-__builtin_huge_valf())
#define NEG_INF_D (-__builtin_huge_val())
constexpr float kLog2e = 1.4426950408889634f;
constexpr double kLog2eD = 1.4426950408889634073599;
constexpr float kLn2 = 0.69314718055994531f;

// native 16-byte vector (the nontemporal builtins and dwordx4 codegen want ext_vector_type)
typedef float f4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------------------------------------
// small helpers

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float fast_log2(float x) { return __builtin_amdgcn_logf(x); }

// log(exp(x) + exp(y)) with the reference's -inf short-circuits (rnnt_helper.h:16-30).
// State is fp64; the bounded correction log1p(exp(-|x-y|)) in [0, ln 2] is evaluated with the fp32
// hardware exp2/log2 plus the classic log1p rounding correction (abs error ~1e-7 per step).
__device__ __forceinline__ double lse(double x, double y) {
    const bool gt = x > y;
    const double hi = gt ? x : y;
    const double lo = gt ? y : x;
    const float d = (float)(lo - hi);
    const float e = fast_exp2(d * kLog2e);
    const float u = 1.0f + e;
    const float corr = ((u - 1.0f) - e) * __builtin_amdgcn_rcpf(u);
    const float c = fast_log2(u) * kLn2 - corr;
    const double r = hi + (double)c;
    return (lo == NEG_INF_D) ? hi : r;
}

template <bool NTL>
__device__ __forceinline__ f4 ld4(const f4 *ptr) {
    if constexpr (NTL)
        return __builtin_nontemporal_load(ptr);
    else
        return *ptr;
}

__device__ __forceinline__ float pick4(const f4 &x, int c) {
    return c == 0 ? x.x : (c == 1 ? x.y : (c == 2 ? x.z : x.w));
}

__device__ __forceinline__ float max4(const f4 &x) { return fmaxf(fmaxf(x.x, x.y), fmaxf(x.z, x.w)); }

// Utterance cursor for a workgroup walking columns in increasing order.
struct Cursor {
    int b;
    __device__ __forceinline__ void init(const int64_t *col_off, int B, int64_t c) {
        int lo = 0, hi = B - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (col_off[mid] <= c) lo = mid; else hi = mid - 1;
        }
        b = lo;
    }
    __device__ __forceinline__ void advance(const int64_t *col_off, int64_t c) {
        while (col_off[b + 1] <= c) ++b;
    }
};

// wave64 butterfly reduction of an online-softmax (max, sum) pair.
__device__ __forceinline__ void wave_reduce_max_sum(float &m, float &s) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const float m2 = __shfl_xor(m, off);
        const float s2 = __shfl_xor(s, off);
        const float mn = fmaxf(m, m2);
        const float mr = (mn == NEG_INF_F) ? 0.0f : mn;
        s = s * fast_exp2((m - mr) * kLog2e) + s2 * fast_exp2((m2 - mr) * kLog2e);
        m = mn;
    }
}

// ------------------------------------------------------------------------------------------------
// metadata: row/column offsets from the device length arrays (one wave, any B)

__global__ __launch_bounds__(64) void setup_kernel(const int *__restrict__ T, const int *__restrict__ S, int B,
                                                   int64_t *__restrict__ row_off, int64_t *__restrict__ col_off) {
    const int lane = threadIdx.x;
    int64_t carry_r = 0, carry_c = 0;
    if (lane == 0) {
        row_off[0] = 0;
        col_off[0] = 0;
    }
    for (int base = 0; base < B; base += 64) {
        const int b = base + lane;
        int64_t r = 0, c = 0;
        if (b < B) {
            const int t = T[b];
            r = (int64_t)t * (S[b] + 1);
            c = t;
        }
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int64_t rr = __shfl_up(r, off);
            const int64_t cc = __shfl_up(c, off);
            if (lane >= off) {
                r += rr;
                c += cc;
            }
        }
        if (b < B) {
            row_off[b + 1] = carry_r + r;
            col_off[b + 1] = carry_c + c;
        }
        carry_r += __shfl(r, 63);
        carry_c += __shfl(c, 63);
    }
}

// Alignment band, reference semantics (gpu_workspace_manager.h:191-219): m[t+1] = #non-blank frames
// in alignment[0..t]; min_s[t] = m[max(0, t+1-k)], max_s[t] = m[min(T, t+1+k)].
// Built on the device: a ballot/popcount prefix per utterance, then one thread per frame.
__global__ __launch_bounds__(64) void align_prefix_kernel(DevProblem p, const int *__restrict__ alignment,
                                                          int64_t astride, int ablank, int *__restrict__ m) {
    const int b = blockIdx.x;
    const int lane = threadIdx.x;
    const int T = p.T[b];
    const int64_t mb = p.col_off[b] + b;  // utterance b owns T_b + 1 prefix entries
    if (lane == 0) m[mb] = 0;
    int carry = 0;
    for (int t0 = 0; t0 < T; t0 += 64) {
        const int t = t0 + lane;
        const bool nb = (t < T) && alignment[(int64_t)b * astride + t] != ablank;
        const unsigned long long mask = __ballot(nb);
        const unsigned long long upto = (lane == 63) ? ~0ull : ((2ull << lane) - 1ull);
        const int incl = __popcll(mask & upto);
        if (t < T) m[mb + t + 1] = carry + incl;
        carry += __popcll(mask);
    }
}

__global__ __launch_bounds__(256) void align_band_kernel(DevProblem p, int k, const int *__restrict__ m,
                                                         int *__restrict__ min_s, int *__restrict__ max_s) {
    const int b = blockIdx.y;
    const int T = p.T[b];
    const int64_t mb = p.col_off[b] + b;
    const int64_t cb = p.col_off[b];
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < T; t += gridDim.x * blockDim.x) {
        const int i0 = min(max(0, t + 1 - k), T);
        const int i1 = max(0, min(T, t + 1 + k));
        min_s[cb + t] = m[mb + i0];
        max_s[cb + t] = m[mb + i1];
    }
}

// Rows of the column outside the log-softmax band get lpb = lpe = 0 (finite), so the recursion can add
// them to a -inf predecessor without a guard (a never-written row could hold NaN).
__device__ __forceinline__ void zero_fill_outside_band(const DevProblem &p, int64_t rowc, int S, int lo, int hi) {
    for (int s = threadIdx.x; s <= S; s += blockDim.x)
        if (s < lo || s > hi) {
            p.lpb[rowc + s] = 0.0;
            p.lpe[rowc + s] = 0.0;
        }
}

// ------------------------------------------------------------------------------------------------
// log-softmax row reduce (vector path: V % 4 == 0 and 16-B aligned rows)
//
// U = float4 per lane per chunk (chunk = 256*U floats), R = rows a wave works on at once (R*U <= 4
// keeps 4 float4 loads per lane in flight for both V = 1024 and V = 256).

template <int U, int R, bool NTL>
__global__ __launch_bounds__(256) void softmax_vec_kernel(DevProblem p) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int V4 = p.V >> 2;
    const f4 *__restrict__ acts4 = reinterpret_cast<const f4 *>(p.acts);
    const int blank = p.blank;
    const int blank4 = blank >> 2;
    const int blank_c = blank & 3;
    const int blank_lane = blank4 & 63;

    Cursor cur;
    cur.init(p.col_off, p.B, blockIdx.x);
    for (int64_t c = blockIdx.x; c < p.num_cols; c += gridDim.x) {
        cur.advance(p.col_off, c);
        const int b = cur.b;
        const int T = p.T[b], S = p.S[b];
        const int t = (int)(c - p.col_off[b]);
        const int64_t rowc = p.row_off[b] + (int64_t)t * (S + 1);
        const int lo = max(0, t - (T - S));
        const int hi = min(t, S);
        const int *__restrict__ lab_b = p.labels + (int64_t)b * p.label_stride;
        zero_fill_outside_band(p, rowc, S, lo, hi);

        for (int s = lo + wave * R; s <= hi; s += 4 * R) {
            float m[R], sum[R], zb[R], ze[R];
            int lab[R];
            bool ok[R];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int sr = s + r;
                ok[r] = sr <= hi;
                lab[r] = (ok[r] && sr < S) ? lab_b[sr] : -1;
                m[r] = NEG_INF_F;
                sum[r] = 0.0f;
                zb[r] = 0.0f;
                ze[r] = 0.0f;
            }
            for (int base = 0; base < V4; base += 64 * U) {
                f4 x[R][U];
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const int j4 = base + lane + 64 * u;
                        if (ok[r] && j4 < V4)
                            x[r][u] = ld4<NTL>(&acts4[(rowc + s + r) * (int64_t)V4 + j4]);
                        else
                            x[r][u] = (f4){NEG_INF_F, NEG_INF_F, NEG_INF_F, NEG_INF_F};
                    }
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    float cm = NEG_INF_F;
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const int j4 = base + lane + 64 * u;
                        if (j4 == blank4) zb[r] = pick4(x[r][u], blank_c);
                        if (lab[r] >= 0 && j4 == (lab[r] >> 2)) ze[r] = pick4(x[r][u], lab[r] & 3);
                        cm = fmaxf(cm, max4(x[r][u]));
                    }
                    const float mn = fmaxf(m[r], cm);
                    const float mr = (mn == NEG_INF_F) ? 0.0f : mn;
                    float acc = sum[r] * fast_exp2((m[r] - mr) * kLog2e);
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        acc += fast_exp2((x[r][u].x - mr) * kLog2e);
                        acc += fast_exp2((x[r][u].y - mr) * kLog2e);
                        acc += fast_exp2((x[r][u].z - mr) * kLog2e);
                        acc += fast_exp2((x[r][u].w - mr) * kLog2e);
                    }
                    sum[r] = acc;
                    m[r] = mn;
                }
            }
#pragma unroll
            for (int r = 0; r < R; ++r) wave_reduce_max_sum(m[r], sum[r]);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if (!ok[r]) continue;
                const float zbv = __shfl(zb[r], blank_lane);
                const float zev = lab[r] >= 0 ? __shfl(ze[r], (lab[r] >> 2) & 63) : 0.0f;
                const double den = -(double)m[r] - log((double)sum[r]);
                if (lane == 0) {
                    const int64_t row = rowc + s + r;
                    p.den[row] = (float)den;
                    p.lpb[row] = (double)zbv + den;
                    p.lpe[row] = (double)zev + den;
                }
            }
        }
    }
}


// Software-pipelined variant: a wave walks its (row, chunk) sequence with the NEXT chunk's loads (and
// the next row's label) already in flight while it reduces the current one, so every wave keeps
// U * 1 KiB of loads outstanding through its reduce/epilogue instead of draining between rows.
template <int U>
__device__ __forceinline__ void load_chunk(const f4 *__restrict__ acts4, int64_t row, int V4, int ch, int lane,
                                           f4 (&x)[U]) {
    const int base = ch * 64 * U;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int j4 = base + lane + 64 * u;
        if (j4 < V4)
            x[u] = acts4[row * (int64_t)V4 + j4];
        else
            x[u] = (f4){NEG_INF_F, NEG_INF_F, NEG_INF_F, NEG_INF_F};
    }
}

template <int U>
__global__ __launch_bounds__(256) void softmax_pipe_kernel(DevProblem p) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int V4 = p.V >> 2;
    const int nch = (V4 + 64 * U - 1) / (64 * U);
    const f4 *__restrict__ acts4 = reinterpret_cast<const f4 *>(p.acts);
    const int blank = p.blank;
    const int blank4 = blank >> 2;
    const int blank_c = blank & 3;
    const int blank_lane = blank4 & 63;

    Cursor cur;
    cur.init(p.col_off, p.B, blockIdx.x);
    for (int64_t c = blockIdx.x; c < p.num_cols; c += gridDim.x) {
        cur.advance(p.col_off, c);
        const int b = cur.b;
        const int T = p.T[b], S = p.S[b];
        const int t = (int)(c - p.col_off[b]);
        const int64_t rowc = p.row_off[b] + (int64_t)t * (S + 1);
        const int lo = max(0, t - (T - S));
        const int hi = min(t, S);
        const int *__restrict__ lab_b = p.labels + (int64_t)b * p.label_stride;
        zero_fill_outside_band(p, rowc, S, lo, hi);

        int s = lo + wave;
        if (s > hi) continue;
        int ch = 0;
        int lab = s < S ? lab_b[s] : -1;
        f4 xa[U];
        load_chunk<U>(acts4, rowc + s, V4, 0, lane, xa);
        float m = NEG_INF_F, sum = 0.0f, zb = 0.0f, ze = 0.0f;
        for (;;) {
            int ns = s, nc = ch + 1;
            if (nc == nch) {
                nc = 0;
                ns = s + 4;
            }
            const bool more = ns <= hi;
            f4 xb[U];
            int nlab = lab;
            if (more) {
                load_chunk<U>(acts4, rowc + ns, V4, nc, lane, xb);
                if (nc == 0) nlab = ns < S ? lab_b[ns] : -1;
            }
            {
                const int base = ch * 64 * U;
                float cm = NEG_INF_F;
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int j4 = base + lane + 64 * u;
                    if (j4 == blank4) zb = pick4(xa[u], blank_c);
                    if (lab >= 0 && j4 == (lab >> 2)) ze = pick4(xa[u], lab & 3);
                    cm = fmaxf(cm, max4(xa[u]));
                }
                const float mn = fmaxf(m, cm);
                const float mr = (mn == NEG_INF_F) ? 0.0f : mn;
                float acc = sum * fast_exp2((m - mr) * kLog2e);
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    acc += fast_exp2((xa[u].x - mr) * kLog2e);
                    acc += fast_exp2((xa[u].y - mr) * kLog2e);
                    acc += fast_exp2((xa[u].z - mr) * kLog2e);
                    acc += fast_exp2((xa[u].w - mr) * kLog2e);
                }
                sum = acc;
                m = mn;
            }
            if (ch == nch - 1) {
                wave_reduce_max_sum(m, sum);
                const float zbv = __shfl(zb, blank_lane);
                const float zev = lab >= 0 ? __shfl(ze, (lab >> 2) & 63) : 0.0f;
                const double den = -(double)m - log((double)sum);
                if (lane == 0) {
                    const int64_t row = rowc + s;
                    p.den[row] = (float)den;
                    p.lpb[row] = (double)zbv + den;
                    p.lpe[row] = (double)zev + den;
                }
                m = NEG_INF_F;
                sum = 0.0f;
                zb = 0.0f;
                ze = 0.0f;
            }
            if (!more) break;
#pragma unroll
            for (int u = 0; u < U; ++u) xa[u] = xb[u];
            s = ns;
            ch = nc;
            lab = nlab;
        }
    }
}

// scalar path (any V, any alignment): one row per wave, lanes stride over v
__global__ __launch_bounds__(256) void softmax_scalar_kernel(DevProblem p) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int V = p.V;
    const int blank = p.blank;
    Cursor cur;
    cur.init(p.col_off, p.B, blockIdx.x);
    for (int64_t c = blockIdx.x; c < p.num_cols; c += gridDim.x) {
        cur.advance(p.col_off, c);
        const int b = cur.b;
        const int T = p.T[b], S = p.S[b];
        const int t = (int)(c - p.col_off[b]);
        const int64_t rowc = p.row_off[b] + (int64_t)t * (S + 1);
        const int lo = max(0, t - (T - S));
        const int hi = min(t, S);
        const int *__restrict__ lab_b = p.labels + (int64_t)b * p.label_stride;
        zero_fill_outside_band(p, rowc, S, lo, hi);
        for (int s = lo + wave; s <= hi; s += 4) {
            const int lab = s < S ? lab_b[s] : -1;
            const float *__restrict__ z = p.acts + (rowc + s) * (int64_t)V;
            float m = NEG_INF_F, sum = 0.0f, zb = 0.0f, ze = 0.0f;
            for (int v0 = 0; v0 < V; v0 += 256) {
                float x[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int v = v0 + lane + 64 * u;
                    x[u] = v < V ? z[v] : NEG_INF_F;
                    if (v == blank) zb = x[u];
                    if (v == lab) ze = x[u];
                }
                const float mn = fmaxf(m, fmaxf(fmaxf(x[0], x[1]), fmaxf(x[2], x[3])));
                const float mr = (mn == NEG_INF_F) ? 0.0f : mn;
                float acc = sum * fast_exp2((m - mr) * kLog2e);
#pragma unroll
                for (int u = 0; u < 4; ++u) acc += fast_exp2((x[u] - mr) * kLog2e);
                sum = acc;
                m = mn;
            }
            wave_reduce_max_sum(m, sum);
            const float zbv = __shfl(zb, blank & 63);
            const float zev = lab >= 0 ? __shfl(ze, lab & 63) : 0.0f;
            const double den = -(double)m - log((double)sum);
            if (lane == 0) {
                const int64_t row = rowc + s;
                p.den[row] = (float)den;
                p.lpb[row] = (double)zbv + den;
                p.lpe[row] = (double)zev + den;
            }
        }
    }
}

// ------------------------------------------------------------------------------------------------
// alpha / beta recursion: one wave per (utterance, direction), K lattice cells per lane, a D-deep
// register ring prefetching lp rows t+1..t+D while step t computes.
//
// Masking follows the reference getters exactly (cpu_workspace_manager.h:161-205 /
// gpu_rnnt_kernel.h:10-72): every cell outside the compute band is stored as -inf, so the stored
// arrays equal get_alpha()/get_beta() on [0,T) x [0,S]. A predecessor at -inf yields -inf without
// touching its lp (rows outside the log-softmax band are never written).

template <int K, int D>
__device__ __forceinline__ void alpha_pass(const DevProblem &p, int b, float *__restrict__ costs) {
    const int lane = threadIdx.x;
    const int T = p.T[b], S = p.S[b], W = S + 1;
    const int64_t r0 = p.row_off[b], c0 = p.col_off[b];
    const int s0 = lane * K;
    const bool band = p.min_s != nullptr;

    double a[K];
#pragma unroll
    for (int k = 0; k < K; ++k) a[k] = (s0 + k == 0) ? 0.0 : NEG_INF_D;  // alpha(-1, s)

    double pb[D][K], pe[D][K];
    int mn[D], mx[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const int tt = min(d, T - 1);
        const double *rb = p.lpb + r0 + (int64_t)tt * W + s0;
        const double *re = p.lpe + r0 + (int64_t)tt * W + s0 - 1;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            pb[d][k] = rb[k];
            pe[d][k] = re[k];
        }
        mn[d] = band ? p.min_s[c0 + tt] : 0;
        mx[d] = band ? p.max_s[c0 + tt] : S;
    }

    for (int t0 = 0; t0 < T; t0 += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int t = t0 + d;
            if (t >= T) break;
            const int lo = max(max(t - (T - 1 - S), mn[d]), 0);
            const int hi = min(min(t + 1, S), mx[d]);
            double carry = __shfl_up(a[K - 1], 1);
            if (lane == 0) carry = NEG_INF_D;
            double na[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int s = s0 + k;
                const double ne = (a[k] == NEG_INF_D) ? NEG_INF_D : a[k] + pb[d][k];
                const double am1 = (k == 0) ? carry : a[k - 1];
                const double em = (am1 == NEG_INF_D) ? NEG_INF_D : am1 + pe[d][k];
                const double v = lse(em, ne);
                na[k] = (s >= lo && s <= hi) ? v : NEG_INF_D;
            }
            double *out = p.alpha + r0 + (int64_t)t * W + s0;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                a[k] = na[k];
                if (s0 + k < W) out[k] = na[k];
            }
            // refill this ring slot with row t + D
            const int tn = min(t + D, T - 1);
            const double *rb = p.lpb + r0 + (int64_t)tn * W + s0;
            const double *re = p.lpe + r0 + (int64_t)tn * W + s0 - 1;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                pb[d][k] = rb[k];
                pe[d][k] = re[k];
            }
            mn[d] = band ? p.min_s[c0 + tn] : 0;
            mx[d] = band ? p.max_s[c0 + tn] : S;
        }
    }
#pragma unroll
    for (int k = 0; k < K; ++k)
        if (s0 + k == S) {
            p.ll[b] = a[k];
            if (costs) costs[b] = (float)(-a[k]);
        }
}

template <int K, int D>
__device__ __forceinline__ void beta_pass(const DevProblem &p, int b) {
    const int lane = threadIdx.x;
    const int T = p.T[b], S = p.S[b], W = S + 1;
    const int64_t r0 = p.row_off[b], c0 = p.col_off[b];
    const int s0 = lane * K;
    const bool band = p.min_s != nullptr;

    double bn[K];
#pragma unroll
    for (int k = 0; k < K; ++k) bn[k] = (s0 + k == S) ? 0.0 : NEG_INF_D;  // beta(T, s)

    double pb[D][K], pe[D][K];
    int mn[D], mx[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const int tt = max(T - 1 - d, 0);
        const double *rb = p.lpb + r0 + (int64_t)tt * W + s0;
        const double *re = p.lpe + r0 + (int64_t)tt * W + s0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            pb[d][k] = rb[k];
            pe[d][k] = re[k];
        }
        mn[d] = (band && tt > 0) ? p.min_s[c0 + tt - 1] : 0;
        mx[d] = (band && tt > 0) ? p.max_s[c0 + tt - 1] : S;
    }

    for (int t0 = T - 1; t0 >= 0; t0 -= D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int t = t0 - d;
            if (t < 0) break;
            int lo, hi;
            if (t == 0) {
                lo = 0;
                hi = 0;
            } else {
                lo = max(max(t - (T - S), mn[d]), 0);
                hi = min(min(t, S), mx[d]);
            }
            double carry = __shfl_down(bn[0], 1);
            if (lane == 63) carry = NEG_INF_D;
            double nb[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int s = s0 + k;
                const double ne = (bn[k] == NEG_INF_D) ? NEG_INF_D : bn[k] + pb[d][k];
                const double bp1 = (k == K - 1) ? carry : bn[k + 1];
                const double em = (s >= S || bp1 == NEG_INF_D) ? NEG_INF_D : bp1 + pe[d][k];
                const double v = lse(em, ne);
                nb[k] = (s >= lo && s <= hi) ? v : NEG_INF_D;
            }
            double *out = p.beta + r0 + (int64_t)t * W + s0;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                bn[k] = nb[k];
                if (s0 + k < W) out[k] = nb[k];
            }
            const int tn = max(t - D, 0);
            const double *rb = p.lpb + r0 + (int64_t)tn * W + s0;
            const double *re = p.lpe + r0 + (int64_t)tn * W + s0;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                pb[d][k] = rb[k];
                pe[d][k] = re[k];
            }
            mn[d] = (band && tn > 0) ? p.min_s[c0 + tn - 1] : 0;
            mx[d] = (band && tn > 0) ? p.max_s[c0 + tn - 1] : S;
        }
    }
    if (lane == 0) p.llb[b] = bn[0];
}

template <int K, int D>
__global__ __launch_bounds__(64) void dp_kernel(DevProblem p, int with_beta, float *__restrict__ costs) {
    const int b = with_beta ? (int)(blockIdx.x >> 1) : (int)blockIdx.x;
    const bool bwd = with_beta && (blockIdx.x & 1);
    if (bwd)
        beta_pass<K, D>(p, b);
    else
        alpha_pass<K, D>(p, b, costs);
}


// ------------------------------------------------------------------------------------------------
// Four-wave recursion: 256 lanes per (utterance, direction), K cells per lane (s = 256-lane blocks).
// The s-1 (alpha) / s+1 (beta) neighbour crosses lanes with a DPP wave shift (v_mov_b32_dpp
// wave_shr:1 / wave_shl:1, no LDS round trip) and crosses waves through a double-buffered LDS slot,
// one s_barrier per step. The lp arrays are finite on every row of [0, S] (the log-softmax kernels
// zero-fill out-of-band rows), so a predecessor at -inf stays -inf without guards; the only
// non-finite case left in the LSE is both inputs at -inf.

__device__ __forceinline__ double dpp_shr1(double v) {  // lane i <- lane i-1 (lane 0 <- 0)
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x138, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x138, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double dpp_shl1(double v) {  // lane i <- lane i+1 (lane 63 <- 0)
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x130, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x130, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}

// log(e^x + e^y) for x, y in [-inf, +inf): m + log1p(exp(-|x - y|)); one -inf input gives d = -inf,
// e = 0, r = m exactly; both -inf is the only NaN case and is patched to -inf.
__device__ __forceinline__ double lse2(double x, double y) {
    const double m = fmax(x, y);
    const float d = (float)(-fabs(x - y));
    const float e = fast_exp2(d * kLog2e);
    const float u = 1.0f + e;
    const float corr = ((u - 1.0f) - e) * __builtin_amdgcn_rcpf(u);
    const float c = fast_log2(u) * kLn2 - corr;
    const double r = m + (double)c;
    return (m == NEG_INF_D) ? NEG_INF_D : r;
}

template <int K, int D, int NW, bool BAND>
__device__ __forceinline__ void alpha_pass4(const DevProblem &p, int b, float *__restrict__ costs, double (*xb)[8]) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int T = p.T[b], S = p.S[b], W = S + 1;
    const int64_t r0 = p.row_off[b], c0 = p.col_off[b];
    const int s0 = (wave * 64 + lane) * K;
    constexpr bool band = BAND;
    static_assert(NW == 1 || NW == 2 || NW == 4 || NW == 8, "cross-wave slots sized for <= 8 waves");

    double a[K];
#pragma unroll
    for (int k = 0; k < K; ++k) a[k] = (s0 + k == 0) ? 0.0 : NEG_INF_D;
    if (NW > 1 && lane == 0) xb[1][wave] = NEG_INF_D;  // alpha(-1, s) for the cross-wave neighbour of step 0

    double pb[D][K], pe[D][K];
    int mn[D], mx[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const int tt = min(d, T - 1);
        const double *rb = p.lpb + r0 + (int64_t)tt * W + s0;
        const double *re = p.lpe + r0 + (int64_t)tt * W + s0 - 1;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            pb[d][k] = rb[k];
            pe[d][k] = re[k];
        }
        mn[d] = band ? p.min_s[c0 + tt] : 0;
        mx[d] = band ? p.max_s[c0 + tt] : S;
    }
    __syncthreads();

    for (int t0 = 0; t0 < T; t0 += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int t = t0 + d;
            if (t >= T) break;
            const int lo = max(max(t - (T - 1 - S), mn[d]), 0);
            const int hi = min(min(t + 1, S), mx[d]);
            double carry = dpp_shr1(a[K - 1]);
            if (lane == 0) carry = (NW == 1 || wave == 0) ? NEG_INF_D : xb[(t + 1) & 1][wave - 1];
            double na[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int s = s0 + k;
                const double am1 = (k == 0) ? carry : a[k - 1];
                const double v = lse2(a[k] + pb[d][k], am1 + pe[d][k]);
                na[k] = (s >= lo && s <= hi) ? v : NEG_INF_D;
            }
            double *out = p.alpha + r0 + (int64_t)t * W + s0;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                a[k] = na[k];
                if (s0 + k < W) out[k] = na[k];
            }
            if (NW > 1 && lane == 63) xb[t & 1][wave] = na[K - 1];
            const int tn = min(t + D, T - 1);
            const double *rb = p.lpb + r0 + (int64_t)tn * W + s0;
            const double *re = p.lpe + r0 + (int64_t)tn * W + s0 - 1;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                pb[d][k] = rb[k];
                pe[d][k] = re[k];
            }
            mn[d] = band ? p.min_s[c0 + tn] : 0;
            mx[d] = band ? p.max_s[c0 + tn] : S;
            if (NW > 1) __syncthreads();
        }
    }
#pragma unroll
    for (int k = 0; k < K; ++k)
        if (s0 + k == S) {
            p.ll[b] = a[k];
            if (costs) costs[b] = (float)(-a[k]);
        }
}

template <int K, int D, int NW, bool BAND>
__device__ __forceinline__ void beta_pass4(const DevProblem &p, int b, double (*xb)[8]) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int T = p.T[b], S = p.S[b], W = S + 1;
    const int64_t r0 = p.row_off[b], c0 = p.col_off[b];
    const int s0 = (wave * 64 + lane) * K;
    constexpr bool band = BAND;

    double bn[K];
#pragma unroll
    for (int k = 0; k < K; ++k) bn[k] = (s0 + k == S) ? 0.0 : NEG_INF_D;  // beta(T, s)
    // beta(T, s) of the first cell of every wave, read by the previous wave's lane 63 at step T-1
    if (NW > 1 && lane == 0) xb[(T - 1 + 1) & 1][wave] = bn[0];

    double pb[D][K], pe[D][K];
    int mn[D], mx[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const int tt = max(T - 1 - d, 0);
        const double *rb = p.lpb + r0 + (int64_t)tt * W + s0;
        const double *re = p.lpe + r0 + (int64_t)tt * W + s0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            pb[d][k] = rb[k];
            pe[d][k] = re[k];
        }
        mn[d] = (band && tt > 0) ? p.min_s[c0 + tt - 1] : 0;
        mx[d] = (band && tt > 0) ? p.max_s[c0 + tt - 1] : S;
    }
    __syncthreads();

    for (int t0 = T - 1; t0 >= 0; t0 -= D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int t = t0 - d;
            if (t < 0) break;
            int lo, hi;
            if (t == 0) {
                lo = 0;
                hi = 0;
            } else {
                lo = max(max(t - (T - S), mn[d]), 0);
                hi = min(min(t, S), mx[d]);
            }
            double carry = dpp_shl1(bn[0]);
            if (lane == 63) carry = (NW == 1 || wave == NW - 1) ? NEG_INF_D : xb[(t + 1) & 1][wave + 1];
            double nb[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int s = s0 + k;
                const double bp1 = (k == K - 1) ? carry : bn[k + 1];
                const double v = lse2(bn[k] + pb[d][k], bp1 + pe[d][k]);
                nb[k] = (s >= lo && s <= hi) ? v : NEG_INF_D;
            }
            double *out = p.beta + r0 + (int64_t)t * W + s0;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                bn[k] = nb[k];
                if (s0 + k < W) out[k] = nb[k];
            }
            if (NW > 1 && lane == 0) xb[t & 1][wave] = nb[0];
            const int tn = max(t - D, 0);
            const double *rb = p.lpb + r0 + (int64_t)tn * W + s0;
            const double *re = p.lpe + r0 + (int64_t)tn * W + s0;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                pb[d][k] = rb[k];
                pe[d][k] = re[k];
            }
            mn[d] = (band && tn > 0) ? p.min_s[c0 + tn - 1] : 0;
            mx[d] = (band && tn > 0) ? p.max_s[c0 + tn - 1] : S;
            if (NW > 1) __syncthreads();
        }
    }
    if (threadIdx.x == 0) p.llb[b] = bn[0];
}

template <int K, int D, int NW, bool BAND>
__global__ __launch_bounds__(64 * NW) void dp4_kernel(DevProblem p, int with_beta, float *__restrict__ costs) {
    __shared__ double xb[2][8];
    const int b = with_beta ? (int)(blockIdx.x >> 1) : (int)blockIdx.x;
    const bool bwd = with_beta && (blockIdx.x & 1);
    if (bwd)
        beta_pass4<K, D, NW, BAND>(p, b, xb);
    else
        alpha_pass4<K, D, NW, BAND>(p, b, costs, xb);
}

// ------------------------------------------------------------------------------------------------
// logit gradient (cpu_rnnt.h:216-236 / gpu_rnnt_kernel.h:239-288):
//   g[v] = exp(z[v] + den + alpha(t-1,s) + beta(t,s) - ll)
//        - [v == blank]                     exp(lpb + alpha(t-1,s) + beta(t+1,s)   - ll)
//        - [v != blank, s < S, v == label]  exp(lpe + alpha(t-1,s) + beta(t+1,s+1) - ll)
// times grad_scale[b]. Per row the three coefficients are formed in fp64 from the recursion state;
// per element it is one fma + one exp2 (+ a select for the <= 2 special columns).

struct RowCoef {
    float c2;   // (den + alpha(t-1,s) + beta(t,s) - ll) * log2(e)
    float cb;   // blank correction
    float ce;   // label correction
    int lab;    // label(s) or -1
};

__device__ __forceinline__ RowCoef row_coef(const DevProblem &p, int b, int t, int T, int S, int s, int64_t row,
                                            double ll, const int *__restrict__ lab_b) {
    const int W = S + 1;
    const double am = (t == 0) ? (s == 0 ? 0.0 : NEG_INF_D) : p.alpha[row - W];
    const double b0 = p.beta[row];
    const double b1 = (t == T - 1) ? (s == S ? 0.0 : NEG_INF_D) : p.beta[row + W];
    const double b2 = (s == S) ? NEG_INF_D : ((t == T - 1) ? (s + 1 == S ? 0.0 : NEG_INF_D) : p.beta[row + W + 1]);
    const double base = am - ll;
    RowCoef rc;
    rc.c2 = (float)(((double)p.den[row] + base + b0) * kLog2eD);
    rc.cb = (float)exp(p.lpb[row] + base + b1);
    rc.ce = (s < S) ? (float)exp(p.lpe[row] + base + b2) : 0.0f;
    rc.lab = (s < S) ? lab_b[s] : -1;
    return rc;
}

template <int U, int R, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void grad_vec_kernel(DevProblem p, const float *__restrict__ scale,
                                                       float *__restrict__ grads) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int V4 = p.V >> 2;
    const int blank = p.blank;
    const f4 *__restrict__ acts4 = reinterpret_cast<const f4 *>(p.acts);
    f4 *__restrict__ g4 = reinterpret_cast<f4 *>(grads);

    Cursor cur;
    cur.init(p.col_off, p.B, blockIdx.x);
    for (int64_t c = blockIdx.x; c < p.num_cols; c += gridDim.x) {
        cur.advance(p.col_off, c);
        const int b = cur.b;
        const int T = p.T[b], S = p.S[b];
        const int t = (int)(c - p.col_off[b]);
        const int64_t rowc = p.row_off[b] + (int64_t)t * (S + 1);
        const int lo = max(0, t - (T - S));
        const int hi = min(t, S);
        const double ll = p.ll[b];
        const float sc = scale ? scale[b] : 1.0f;
        const float zf = 0.0f * sc;  // out-of-band rows: 0 * scale, as the reference's backward
        const int *__restrict__ lab_b = p.labels + (int64_t)b * p.label_stride;

        for (int s = wave * R; s <= S; s += 4 * R) {
            RowCoef rc[R];
            bool ok[R], inb[R];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int sr = s + r;
                ok[r] = sr <= S;
                inb[r] = ok[r] && sr >= lo && sr <= hi;
                if (inb[r]) rc[r] = row_coef(p, b, t, T, S, sr, rowc + sr, ll, lab_b);
                else rc[r] = RowCoef{0.0f, 0.0f, 0.0f, -1};
            }
            for (int base = 0; base < V4; base += 64 * U) {
                f4 x[R][U];
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const int j4 = base + lane + 64 * u;
                        if (inb[r] && j4 < V4) x[r][u] = ld4<NTL>(&acts4[(rowc + s + r) * (int64_t)V4 + j4]);
                    }
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const int j4 = base + lane + 64 * u;
                        if (!ok[r] || j4 >= V4) continue;
                        f4 g;
                        if (inb[r]) {
                            const float c2 = rc[r].c2;
                            g.x = fast_exp2(fmaf(x[r][u].x, kLog2e, c2));
                            g.y = fast_exp2(fmaf(x[r][u].y, kLog2e, c2));
                            g.z = fast_exp2(fmaf(x[r][u].z, kLog2e, c2));
                            g.w = fast_exp2(fmaf(x[r][u].w, kLog2e, c2));
                            const int v0 = j4 * 4;
                            const int db = blank - v0;
                            const int lab = rc[r].lab;
                            const int de = (lab >= 0 && lab != blank) ? lab - v0 : -1;
                            const float cb = rc[r].cb, ce = rc[r].ce;
                            g.x -= (db == 0 ? cb : 0.0f) + (de == 0 ? ce : 0.0f);
                            g.y -= (db == 1 ? cb : 0.0f) + (de == 1 ? ce : 0.0f);
                            g.z -= (db == 2 ? cb : 0.0f) + (de == 2 ? ce : 0.0f);
                            g.w -= (db == 3 ? cb : 0.0f) + (de == 3 ? ce : 0.0f);
                            g.x *= sc;
                            g.y *= sc;
                            g.z *= sc;
                            g.w *= sc;
                        } else {
                            g = (f4){zf, zf, zf, zf};
                        }
                        if constexpr (NTS)
                            __builtin_nontemporal_store(g, &g4[(rowc + s + r) * (int64_t)V4 + j4]);
                        else
                            g4[(rowc + s + r) * (int64_t)V4 + j4] = g;
                    }
            }
        }
    }
}


// Software-pipelined gradient: the next (row, chunk)'s acts loads and the next row's recursion state
// (scalar loads) are issued before the current chunk is computed and stored; the fp64 coefficient math
// of the next row runs after the current chunk's stores are queued.
struct RowRaw {
    double am, b0, b1, b2, lpb, lpe;
    float den;
    int lab;
};

__device__ __forceinline__ RowRaw row_raw(const DevProblem &p, int t, int T, int S, int s, int64_t row,
                                          const int *__restrict__ lab_b) {
    const int W = S + 1;
    RowRaw r;
    r.am = (t == 0) ? (s == 0 ? 0.0 : NEG_INF_D) : p.alpha[row - W];
    r.b0 = p.beta[row];
    r.b1 = (t == T - 1) ? (s == S ? 0.0 : NEG_INF_D) : p.beta[row + W];
    r.b2 = (s == S) ? NEG_INF_D : ((t == T - 1) ? (s + 1 == S ? 0.0 : NEG_INF_D) : p.beta[row + W + 1]);
    r.lpb = p.lpb[row];
    r.lpe = p.lpe[row];
    r.den = p.den[row];
    r.lab = (s < S) ? lab_b[s] : -1;
    return r;
}

__device__ __forceinline__ RowCoef row_finish(const RowRaw &r, double ll, int S, int s) {
    const double base = r.am - ll;
    RowCoef rc;
    rc.c2 = (float)(((double)r.den + base + r.b0) * kLog2eD);
    rc.cb = (float)exp(r.lpb + base + r.b1);
    rc.ce = (s < S) ? (float)exp(r.lpe + base + r.b2) : 0.0f;
    rc.lab = r.lab;
    return rc;
}

__device__ __forceinline__ f4 grad_chunk(const f4 &x, const RowCoef &rc, int j4, int blank, float sc) {
    f4 g;
    const float c2 = rc.c2;
    g.x = fast_exp2(fmaf(x.x, kLog2e, c2));
    g.y = fast_exp2(fmaf(x.y, kLog2e, c2));
    g.z = fast_exp2(fmaf(x.z, kLog2e, c2));
    g.w = fast_exp2(fmaf(x.w, kLog2e, c2));
    const int v0 = j4 * 4;
    const int db = blank - v0;
    const int de = (rc.lab >= 0 && rc.lab != blank) ? rc.lab - v0 : -1;
    g.x -= (db == 0 ? rc.cb : 0.0f) + (de == 0 ? rc.ce : 0.0f);
    g.y -= (db == 1 ? rc.cb : 0.0f) + (de == 1 ? rc.ce : 0.0f);
    g.z -= (db == 2 ? rc.cb : 0.0f) + (de == 2 ? rc.ce : 0.0f);
    g.w -= (db == 3 ? rc.cb : 0.0f) + (de == 3 ? rc.ce : 0.0f);
    g.x *= sc;
    g.y *= sc;
    g.z *= sc;
    g.w *= sc;
    return g;
}

template <bool NT>
__device__ __forceinline__ void store4(f4 *ptr, const f4 &v) {
    if constexpr (NT)
        __builtin_nontemporal_store(v, ptr);
    else
        *ptr = v;
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void grad_pipe_kernel(DevProblem p, const float *__restrict__ scale,
                                                        float *__restrict__ grads) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int V4 = p.V >> 2;
    const int nch = (V4 + 64 * U - 1) / (64 * U);
    const int blank = p.blank;
    const f4 *__restrict__ acts4 = reinterpret_cast<const f4 *>(p.acts);
    f4 *__restrict__ g4 = reinterpret_cast<f4 *>(grads);

    Cursor cur;
    cur.init(p.col_off, p.B, blockIdx.x);
    for (int64_t c = blockIdx.x; c < p.num_cols; c += gridDim.x) {
        cur.advance(p.col_off, c);
        const int b = cur.b;
        const int T = p.T[b], S = p.S[b];
        const int t = (int)(c - p.col_off[b]);
        const int64_t rowc = p.row_off[b] + (int64_t)t * (S + 1);
        const int lo = max(0, t - (T - S));
        const int hi = min(t, S);
        const double ll = p.ll[b];
        const float sc = scale ? scale[b] : 1.0f;
        const float zf = 0.0f * sc;
        const f4 z4 = (f4){zf, zf, zf, zf};
        const int *__restrict__ lab_b = p.labels + (int64_t)b * p.label_stride;

        int s = wave;
        if (s > S) continue;
        int ch = 0;
        bool inb = s >= lo && s <= hi;
        RowCoef rc = RowCoef{0.0f, 0.0f, 0.0f, -1};
        f4 xa[U];
        if (inb) {
            rc = row_finish(row_raw(p, t, T, S, s, rowc + s, lab_b), ll, S, s);
            load_chunk<U>(acts4, rowc + s, V4, 0, lane, xa);
        }
        for (;;) {
            int ns = s, nc = ch + 1;
            if (nc == nch) {
                nc = 0;
                ns = s + 4;
            }
            const bool more = ns <= S;
            const bool ninb = more && ns >= lo && ns <= hi;
            f4 xb[U];
            RowRaw nraw;
            if (ninb) {
                load_chunk<U>(acts4, rowc + ns, V4, nc, lane, xb);
                if (nc == 0) nraw = row_raw(p, t, T, S, ns, rowc + ns, lab_b);
            }
            const int base = ch * 64 * U;
            f4 *__restrict__ out = g4 + (rowc + s) * (int64_t)V4;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int j4 = base + lane + 64 * u;
                if (j4 < V4) store4<NT>(out + j4, inb ? grad_chunk(xa[u], rc, j4, blank, sc) : z4);
            }
            if (!more) break;
            if (nc == 0) rc = ninb ? row_finish(nraw, ll, S, ns) : RowCoef{0.0f, 0.0f, 0.0f, -1};
#pragma unroll
            for (int u = 0; u < U; ++u) xa[u] = xb[u];
            s = ns;
            ch = nc;
            inb = ninb;
        }
    }
}

__global__ __launch_bounds__(256) void grad_scalar_kernel(DevProblem p, const float *__restrict__ scale,
                                                          float *__restrict__ grads) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int V = p.V;
    const int blank = p.blank;
    Cursor cur;
    cur.init(p.col_off, p.B, blockIdx.x);
    for (int64_t c = blockIdx.x; c < p.num_cols; c += gridDim.x) {
        cur.advance(p.col_off, c);
        const int b = cur.b;
        const int T = p.T[b], S = p.S[b];
        const int t = (int)(c - p.col_off[b]);
        const int64_t rowc = p.row_off[b] + (int64_t)t * (S + 1);
        const int lo = max(0, t - (T - S));
        const int hi = min(t, S);
        const double ll = p.ll[b];
        const float sc = scale ? scale[b] : 1.0f;
        const float zf = 0.0f * sc;
        const int *__restrict__ lab_b = p.labels + (int64_t)b * p.label_stride;
        for (int s = wave; s <= S; s += 4) {
            const int64_t row = rowc + s;
            float *__restrict__ g = grads + row * (int64_t)V;
            if (s < lo || s > hi) {
                for (int v = lane; v < V; v += 64) g[v] = zf;
                continue;
            }
            const RowCoef rc = row_coef(p, b, t, T, S, s, row, ll, lab_b);
            const float *__restrict__ z = p.acts + row * (int64_t)V;
            for (int v = lane; v < V; v += 64) {
                float gv = fast_exp2(fmaf(z[v], kLog2e, rc.c2));
                if (v == blank) gv -= rc.cb;
                else if (v == rc.lab) gv -= rc.ce;
                g[v] = gv * sc;
            }
        }
    }
}

// ------------------------------------------------------------------------------------------------
// synthetic generator (bench / tests), bit-identical to mrnnt_oracle_synth_acts (oracle/rnnt_oracle.c)

__device__ __forceinline__ uint64_t splitmix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ __launch_bounds__(256) void synth_kernel(float *__restrict__ out, int64_t begin, int64_t count,
                                                    uint64_t seed, int normal) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += stride) {
        const uint64_t h = splitmix(seed * 0xD1B54A32D192ED03ull + (uint64_t)(begin + i));
        float v;
        if (!normal) {
            v = (float)(uint32_t)(h >> 40) * (1.0f / 16777216.0f);
        } else {
            const int32_t s4 = (int32_t)(h & 0xFFFF) + (int32_t)((h >> 16) & 0xFFFF) +
                               (int32_t)((h >> 32) & 0xFFFF) + (int32_t)(h >> 48);
            v = (float)(s4 - 131070) * (1.0f / 37837.23f);
        }
        out[i] = v;
    }
}

// ------------------------------------------------------------------------------------------------
// launchers

hipError_t launch_setup(const int *T, const int *S, int B, int64_t *row_off, int64_t *col_off, hipStream_t stream) {
    setup_kernel<<<1, 64, 0, stream>>>(T, S, B, row_off, col_off);
    return hipGetLastError();
}

hipError_t launch_align(const DevProblem &p, const int *alignment, int64_t align_stride, int align_blank,
                        int max_shift, int *mtmp, int *min_s, int *max_s, hipStream_t stream) {
    align_prefix_kernel<<<p.B, 64, 0, stream>>>(p, alignment, align_stride, align_blank, mtmp);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    dim3 grid(8, p.B);
    align_band_kernel<<<grid, 256, 0, stream>>>(p, max_shift, mtmp, min_s, max_s);
    return hipGetLastError();
}

static bool vec_ok(const DevProblem &p, const void *extra) {
    return (p.V % 4) == 0 && (reinterpret_cast<uintptr_t>(p.acts) % 16) == 0 &&
           (extra == nullptr || reinterpret_cast<uintptr_t>(extra) % 16 == 0);
}

Tuning &tuning() {
    static Tuning t;
    return t;
}

template <bool NTL>
static void softmax_vec_launch(const DevProblem &p, int grid, hipStream_t stream) {
    const int V4 = p.V / 4;
    if (V4 >= 192 && tuning().softmax_variant == 2)
        softmax_vec_kernel<4, 2, NTL><<<grid, 256, 0, stream>>>(p);
    else if (V4 >= 192)
        softmax_vec_kernel<4, 1, NTL><<<grid, 256, 0, stream>>>(p);
    else if (V4 >= 96)
        softmax_vec_kernel<2, 2, NTL><<<grid, 256, 0, stream>>>(p);
    else
        softmax_vec_kernel<1, 4, NTL><<<grid, 256, 0, stream>>>(p);
}

hipError_t launch_softmax(const DevProblem &p, int grid, hipStream_t stream) {
    if (vec_ok(p, nullptr) && tuning().softmax_variant == 1) {
        const int V4 = p.V / 4;
        if (V4 >= 192)
            softmax_pipe_kernel<4><<<grid, 256, 0, stream>>>(p);
        else if (V4 >= 96)
            softmax_pipe_kernel<2><<<grid, 256, 0, stream>>>(p);
        else
            softmax_pipe_kernel<1><<<grid, 256, 0, stream>>>(p);
    } else if (vec_ok(p, nullptr)) {
        if (tuning().nt_load)
            softmax_vec_launch<true>(p, grid, stream);
        else
            softmax_vec_launch<false>(p, grid, stream);
    } else {
        softmax_scalar_kernel<<<grid, 256, 0, stream>>>(p);
    }
    return hipGetLastError();
}

template <int K>
static void dp_launch_k(const DevProblem &p, int with_beta, float *costs, hipStream_t stream) {
    // prefetch depth: deep ring for the common small K, shallower where registers run out
    constexpr int D = K <= 4 ? 8 : (K <= 8 ? 4 : (K <= 12 ? 2 : 1));
    const int blocks = with_beta ? 2 * p.B : p.B;
    dp_kernel<K, D><<<blocks, 64, 0, stream>>>(p, with_beta, costs);
}

template <int K, int NW>
static void dp4_launch_k(const DevProblem &p, int with_beta, float *costs, hipStream_t stream) {
    constexpr int D = K <= 2 ? 8 : (K <= 4 ? 4 : (K <= 8 ? 2 : 1));
    const int blocks = with_beta ? 2 * p.B : p.B;
    if (p.min_s)
        dp4_kernel<K, D, NW, true><<<blocks, 64 * NW, 0, stream>>>(p, with_beta, costs);
    else
        dp4_kernel<K, D, NW, false><<<blocks, 64 * NW, 0, stream>>>(p, with_beta, costs);
}

hipError_t launch_dp(const DevProblem &p, int S_max, int with_beta, float *costs, hipStream_t stream) {
    const int W = S_max + 1;
    if (tuning().dp_variant == 1) {  // NW waves x K cells per lane, sized to S+1
        if (W <= 64) dp4_launch_k<1, 1>(p, with_beta, costs, stream);
        else if (W <= 128) dp4_launch_k<1, 2>(p, with_beta, costs, stream);
        else if (W <= 256) dp4_launch_k<1, 4>(p, with_beta, costs, stream);
        else if (W <= 512) dp4_launch_k<1, 8>(p, with_beta, costs, stream);
        else if (W <= 1024) dp4_launch_k<2, 8>(p, with_beta, costs, stream);
        else if (W <= 1536) dp4_launch_k<3, 8>(p, with_beta, costs, stream);
        else if (W <= kMaxLabelsPlusOne) dp4_launch_k<4, 8>(p, with_beta, costs, stream);
        else return hipErrorInvalidValue;
        return hipGetLastError();
    }
    if (tuning().dp_variant == 3) {  // always four waves (round-1 shape), for A/B
        if (W <= 256) dp4_launch_k<1, 4>(p, with_beta, costs, stream);
        else if (W <= 512) dp4_launch_k<2, 4>(p, with_beta, costs, stream);
        else if (W <= 1024) dp4_launch_k<4, 4>(p, with_beta, costs, stream);
        else if (W <= kMaxLabelsPlusOne) dp4_launch_k<8, 4>(p, with_beta, costs, stream);
        else return hipErrorInvalidValue;
        return hipGetLastError();
    }
    if (tuning().dp_variant == 2) {  // one wave, K cells per lane, DPP neighbours, no barrier
        if (W <= 64) dp4_launch_k<1, 1>(p, with_beta, costs, stream);
        else if (W <= 128) dp4_launch_k<2, 1>(p, with_beta, costs, stream);
        else if (W <= 192) dp4_launch_k<3, 1>(p, with_beta, costs, stream);
        else if (W <= 256) dp4_launch_k<4, 1>(p, with_beta, costs, stream);
        else if (W <= 320) dp4_launch_k<5, 1>(p, with_beta, costs, stream);
        else if (W <= 384) dp4_launch_k<6, 1>(p, with_beta, costs, stream);
        else if (W <= 512) dp4_launch_k<8, 1>(p, with_beta, costs, stream);
        else if (W <= 1024) dp4_launch_k<16, 1>(p, with_beta, costs, stream);
        else if (W <= kMaxLabelsPlusOne) dp4_launch_k<32, 1>(p, with_beta, costs, stream);
        else return hipErrorInvalidValue;
        return hipGetLastError();
    }
    if (W <= 64) dp_launch_k<1>(p, with_beta, costs, stream);
    else if (W <= 128) dp_launch_k<2>(p, with_beta, costs, stream);
    else if (W <= 192) dp_launch_k<3>(p, with_beta, costs, stream);
    else if (W <= 256) dp_launch_k<4>(p, with_beta, costs, stream);
    else if (W <= 320) dp_launch_k<5>(p, with_beta, costs, stream);
    else if (W <= 384) dp_launch_k<6>(p, with_beta, costs, stream);
    else if (W <= 512) dp_launch_k<8>(p, with_beta, costs, stream);
    else if (W <= 768) dp_launch_k<12>(p, with_beta, costs, stream);
    else if (W <= 1024) dp_launch_k<16>(p, with_beta, costs, stream);
    else if (W <= 1536) dp_launch_k<24>(p, with_beta, costs, stream);
    else if (W <= kMaxLabelsPlusOne) dp_launch_k<32>(p, with_beta, costs, stream);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

template <bool NT>
static void grad_pipe_launch(const DevProblem &p, const float *scale, float *grads, int grid, hipStream_t stream) {
    const int V4 = p.V / 4;
    if (V4 >= 192)
        grad_pipe_kernel<4, NT><<<grid, 256, 0, stream>>>(p, scale, grads);
    else if (V4 >= 96)
        grad_pipe_kernel<2, NT><<<grid, 256, 0, stream>>>(p, scale, grads);
    else
        grad_pipe_kernel<1, NT><<<grid, 256, 0, stream>>>(p, scale, grads);
}

template <bool NTL, bool NTS>
static void grad_vec_launch(const DevProblem &p, const float *scale, float *grads, int grid, hipStream_t stream) {
    const int V4 = p.V / 4;
    if (V4 >= 192 && tuning().grad_variant == 2)
        grad_vec_kernel<4, 2, NTL, NTS><<<grid, 256, 0, stream>>>(p, scale, grads);
    else if (V4 >= 192)
        grad_vec_kernel<4, 1, NTL, NTS><<<grid, 256, 0, stream>>>(p, scale, grads);
    else if (V4 >= 96)
        grad_vec_kernel<2, 2, NTL, NTS><<<grid, 256, 0, stream>>>(p, scale, grads);
    else
        grad_vec_kernel<1, 4, NTL, NTS><<<grid, 256, 0, stream>>>(p, scale, grads);
}

hipError_t launch_grad(const DevProblem &p, const float *scale, float *grads, int grid, hipStream_t stream) {
    if (vec_ok(p, grads) && tuning().grad_variant == 1) {
        if (tuning().nt_store)
            grad_pipe_launch<true>(p, scale, grads, grid, stream);
        else
            grad_pipe_launch<false>(p, scale, grads, grid, stream);
    } else if (vec_ok(p, grads)) {
        const bool ntl = tuning().nt_load != 0, nts = tuning().nt_store != 0;
        if (ntl && nts)
            grad_vec_launch<true, true>(p, scale, grads, grid, stream);
        else if (ntl)
            grad_vec_launch<true, false>(p, scale, grads, grid, stream);
        else if (nts)
            grad_vec_launch<false, true>(p, scale, grads, grid, stream);
        else
            grad_vec_launch<false, false>(p, scale, grads, grid, stream);
    } else {
        grad_scalar_kernel<<<grid, 256, 0, stream>>>(p, scale, grads);
    }
    return hipGetLastError();
}

hipError_t launch_synth(float *out, int64_t begin, int64_t count, uint64_t seed, int normal, hipStream_t stream) {
    if (count <= 0) return hipSuccess;
    int64_t blocks = (count + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    synth_kernel<<<(int)blocks, 256, 0, stream>>>(out, begin, count, seed, normal);
    return hipGetLastError();
}

}  // namespace mrnnt
