// mrnnt_device.h -- device-side helpers shared by the kernels of libmonotonic_rnnt_amd.so
// (gfx950 / CDNA4, wave64): constants, fast transcendentals, the fp64 log-sum-exp, wave reductions,
// utterance cursors, the element-type traits of the acts/grads I/O, and acts-layout addressing.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mrnnt_internal.h"

namespace mrnnt {

#define NEG_INF_F (-__builtin_huge_valf())
#define NEG_INF_D (-__builtin_huge_val())
constexpr float kLog2e = 1.4426950408889634f;
constexpr double kLog2eD = 1.4426950408889634073599;
constexpr float kLn2 = 0.69314718055994531f;

// native 16-byte vectors (dwordx4 loads/stores; the nontemporal builtins want ext_vector_type)
typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned int u4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }  // v_exp_f32
__device__ __forceinline__ float fast_log2(float x) { return __builtin_amdgcn_logf(x); }   // v_log_f32

// log(e^x + e^y) with fp64 state (rnnt_helper.h:16-30 semantics): m + log1p(exp(-|x - y|)). The bounded
// correction (in [0, ln 2]) is log2(1 + e) * ln 2 on the fp32 hardware exp2/log2: <= ~1e-7 absolute per step (the
// rounding of 1 + e to fp32, 6e-8, plus v_log_f32's). The classic log1p rounding fix (((u - 1) - e) / u) halved that
// but put three more dependent operations on the one-wave recursion's chain. One -inf input gives
// d = -inf, e = 0, r = m exactly; both -inf is the only NaN case and is patched to -inf.
__device__ __forceinline__ double max_f64(double x, double y) {
    // v_max_f64 without the canonicalising max fmax() emits for an operand the compiler cannot prove canonical (a DPP
    // result): the same value for every non-NaN input, one instruction fewer per recursion step
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
    return r;
}

__device__ __forceinline__ double lse2(double x, double y) {
    const double m = max_f64(x, y);
    const float d = (float)(-fabs(x - y));
    const float e = fast_exp2(d * kLog2e);
    const float c = fast_log2(1.0f + e) * kLn2;
    const double r = m + (double)c;
    return (m == NEG_INF_D) ? NEG_INF_D : r;
}

// log(e^x + e^y + e^z), the same form with three terms: m + log(sum e^(x_i - m)), the sum in [1, 3] in fp32 (one
// term is exactly 1), log2 on v_log_f32 -- <= ~2e-7 absolute, the error of two lse2 steps, for a step that replaces
// two of them on a dependent chain (the staged walk's frame pairs, mrnnt_chase.hip). All -inf gives -inf.
__device__ __forceinline__ double lse3(double x, double y, double z) {
    const double m = max_f64(max_f64(x, y), z);
    const float ex = fast_exp2((float)(x - m) * kLog2e);
    const float ey = fast_exp2((float)(y - m) * kLog2e);
    const float ez = fast_exp2((float)(z - m) * kLog2e);
    const float c = fast_log2(ex + ey + ez) * kLn2;
    const double r = m + (double)c;
    return (m == NEG_INF_D) ? NEG_INF_D : r;
}

// wave64 butterfly reduction of an online-softmax (max, sum-exp) pair
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

// DPP wave64 reductions with a wave-uniform result (read from lane 63 into an SGPR): quad xor 1, xor 2,
// half-row mirror, row mirror (every row of 16 holds its total), then row_bcast:15 / row_bcast:31 carry the
// row totals up to lane 63. Six DPP-fed VALU ops and one v_readlane, no LDS (cf. ds_bpermute butterflies).
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ float dpp_f(float old, float src) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(src), CTRL, ROW_MASK, 0xf,
                                                      false));
}

__device__ __forceinline__ float wave_max_uniform(float v) {
    v = fmaxf(v, dpp_f<0xB1>(v, v));        // quad_perm [1,0,3,2]
    v = fmaxf(v, dpp_f<0x4E>(v, v));        // quad_perm [2,3,0,1]
    v = fmaxf(v, dpp_f<0x141>(v, v));       // row_half_mirror
    v = fmaxf(v, dpp_f<0x140>(v, v));       // row_mirror
    v = fmaxf(v, dpp_f<0x142, 0xa>(v, v));  // row_bcast:15 into rows 1, 3
    v = fmaxf(v, dpp_f<0x143, 0xc>(v, v));  // row_bcast:31 into rows 2, 3
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

__device__ __forceinline__ float wave_sum_uniform(float v) {
    v += dpp_f<0xB1>(0.0f, v);
    v += dpp_f<0x4E>(0.0f, v);
    v += dpp_f<0x141>(0.0f, v);
    v += dpp_f<0x140>(0.0f, v);
    v += dpp_f<0x142, 0xa>(0.0f, v);  // rows 0, 2 add the old value 0
    v += dpp_f<0x143, 0xc>(0.0f, v);
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// Monotone utterance cursor over a prefix-offset array (col_off or row_off), for a workgroup/wave that
// walks indices in increasing order: one binary search at start, then amortised O(1) advances.
struct Cursor {
    int b;
    __device__ __forceinline__ void init(const int64_t *off, int B, int64_t i) {
        int lo = 0, hi = B - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (off[mid] <= i) lo = mid; else hi = mid - 1;
        }
        b = lo;
    }
    __device__ __forceinline__ void advance(const int64_t *off, int64_t i) {
        while (off[b + 1] <= i) ++b;
    }
};

// Column taken at visit ci of a streaming kernel's column walk. col_mul == 0: in order; > 0: scattered,
// (ci * col_mul) % num_cols; < 0: XCD-chunked -- workgroups are dispatched round-robin over the 8 XCDs, so visit
// ci runs on XCD ci % 8 (every grid is a multiple of 8 or one workgroup per column), and XCD x walks its own
// contiguous eighth of the columns in order, x * q + min(x, r) + ci / 8 (q, r = num_cols / 8, % 8): the window of
// acts an XCD's L2 and address-translation caches see at once is one region, not all eight XCDs' interleaved.
__device__ __forceinline__ int64_t visit_col(const DevProblem &p, int64_t ci) {
    if (p.col_mul == 0) return ci;
    if (p.col_mul > 0) return (ci * p.col_mul) % p.num_cols;
    const int64_t n = p.num_cols, q = n >> 3, r = n & 7, x = ci & 7;
    return x * q + (x < r ? x : r) + (ci >> 3);
}

// Device-resident lengths: the real column / row counts and the column-order multiplier published by the call's
// setup kernel replace the host bounds in the kernel's copy of the problem. Returns false when the lengths failed
// validation (then num_cols = 0: column walks do nothing). Without device lengths, and in the log-softmax launch
// that plans them itself (dyn_fused, before the words exist): a no-op returning true.
__device__ __forceinline__ bool resolve_dyn(DevProblem &p) {
    if (!p.dyn || p.dyn_fused) return true;
    const int st = __builtin_amdgcn_readfirstlane(p.dyn->status);
    if (st) {
        p.num_cols = 0;
        return false;
    }
    p.num_cols = p.dyn->num_cols;
    p.num_rows = p.dyn->num_rows;
    if (p.col_mul > 0) p.col_mul = p.dyn->col_mul;  // scattered order requested: the device's coprime multiplier
    return true;
}

__device__ __forceinline__ int64_t uniform64(int64_t v) {
    const int lo = __builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const int hi = __builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

__device__ __forceinline__ int64_t readlane64(int64_t v, int lane) {
    const int lo = __builtin_amdgcn_readlane((int)(uint32_t)v, lane);
    const int hi = __builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), lane);
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// One lattice column as a streaming kernel walks it: column c = (utterance b, frame t), lattice row of (t, 0).
struct ColRef {
    int64_t c;
    int b, T, S, t;
    int64_t rowc;
};

__device__ __forceinline__ ColRef col_ref(const DevProblem &p, int64_t c) {
    ColRef k;
    k.c = c;
    k.b = p.col_b[c];
    k.T = p.T[k.b];
    k.S = p.S[k.b];
    k.t = (int)(c - p.col_off[k.b]);
    k.rowc = p.row_off[k.b] + (int64_t)k.t * (k.S + 1);
    return k;
}

// dyn_fused: the lengths of a batch of <= 64 utterances in the registers of every wave -- lane b holds T_b, S_b and
// the inclusive prefix sums of the columns and rows -- so a column's utterance is one ballot away.
struct WaveLengths {
    int T, S;
    int64_t cols, rows;  // inclusive prefix sums at lane b (lanes >= B: the totals)
    int64_t C, R;        // totals (uniform)
    bool ok;             // every length valid and the totals inside the host's plan (uniform)
};

__device__ __forceinline__ int64_t wave_incl_scan64(int64_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int64_t u = __shfl_up(v, off);
        if (lane >= off) v += u;
    }
    return v;
}

__device__ __forceinline__ WaveLengths wave_lengths(const DevProblem &p) {
    const int lane = threadIdx.x & 63;
    const bool in = lane < p.B;
    WaveLengths w;
    w.T = in ? p.T[lane] : 0;
    w.S = in ? p.S[lane] : 0;
    const bool good = !in || (w.T > 0 && w.S >= 0 && w.T >= w.S && w.S <= p.s_cap && (p.t_cap == 0 || w.T <= p.t_cap) &&
                              (p.s1_cap == 0 || (int64_t)w.S + 1 <= p.s1_cap));
    w.cols = wave_incl_scan64((in && good) ? w.T : 0);
    w.rows = wave_incl_scan64((in && good) ? (int64_t)w.T * (w.S + 1) : 0);
    w.C = readlane64(w.cols, 63);
    w.R = readlane64(w.rows, 63);
    w.ok = __ballot(!good) == 0 && (p.pad_S1 ? w.R <= p.num_rows : w.R == p.num_rows) && w.C <= p.num_cols;
    return w;
}

__device__ __forceinline__ ColRef wave_locate(const WaveLengths &w, int64_t c) {
    ColRef k;
    k.c = c;
    k.b = __popcll(__ballot(w.cols <= c));  // utterances whose columns all lie before c
    k.T = __builtin_amdgcn_readlane(w.T, k.b);
    k.S = __builtin_amdgcn_readlane(w.S, k.b);
    const int64_t c0 = k.b ? readlane64(w.cols, k.b - 1) : 0;
    const int64_t r0 = k.b ? readlane64(w.rows, k.b - 1) : 0;
    k.t = (int)(c - c0);
    k.rowc = r0 + (int64_t)k.t * (k.S + 1);
    return k;
}

// dyn_fused, workgroup 0 (wave 0): what the setup kernel would have written -- lattice offsets, DynWords, status
// report, the lp pads around [0, R) -- for the recursion and gradient kernels that follow in the stream.
__device__ __forceinline__ void publish_lengths(const DevProblem &p, const WaveLengths &w) {
    const int lane = threadIdx.x & 63;
    if (threadIdx.x >= 64) return;
    int64_t *row_off = const_cast<int64_t *>(p.row_off);
    int64_t *col_off = const_cast<int64_t *>(p.col_off);
    if (lane < p.B) {
        row_off[lane + 1] = w.ok ? w.rows : 0;
        col_off[lane + 1] = w.ok ? w.cols : 0;
    }
    int64_t mul = 0;
    if (w.ok && w.C > p.scatter_above && w.C >= 3 && w.C < (1ll << 31)) {  // as setup_dyn_kernel
        for (uint32_t base = max(2u, (uint32_t)(0.6180339887 * (double)w.C));; base += 64) {
            uint32_t x = base + lane, y = (uint32_t)w.C;
            while (y) {
                const uint32_t rem = x % y;
                x = y;
                y = rem;
            }
            const unsigned long long hit = __ballot(x == 1);
            if (hit) {
                mul = (int64_t)base + __ffsll((long long)hit) - 1;
                break;
            }
        }
    }
    if (lane == 0) {
        row_off[0] = 0;
        col_off[0] = 0;
        DynWords *d = p.dyn;
        d->status = w.ok ? 0 : (int)RNNT_STATUS_INVALID_VALUE;
        d->num_cols = w.ok ? w.C : 0;
        d->num_rows = w.ok ? w.R : 0;
        d->col_mul = mul;
        d->steal = 0;
        if (!w.ok && p.status_host)  // a plain system-scope store into the caller's host-mapped word
            __hip_atomic_store(p.status_host, (int)RNNT_STATUS_INVALID_VALUE, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
    const int64_t end = w.ok ? w.R : 0;
    p.lp[lane - 64] = Lp{0.0, 0.0};
    p.lp[end + lane] = Lp{0.0, 0.0};
}

// Column walk of a workgroup of a streaming kernel: visits ci = blockIdx.x, blockIdx.x + gridDim.x, ... < num_cols,
// calling body(ColRef) for column visit_col(ci) (the whole workgroup, uniform). With p.steal (device-resident lengths
// with a separate setup kernel, whose column count the host does not know: the grid is sized to the CUs) the first
// gridDim.x columns go to the workgroups in order and every later one to the workgroup that finishes first -- a
// shared counter the setup kernel zeroed, the next index requested at the start of a column and handed over through
// LDS at its end (one barrier per column), so a persistent grid balances like the hardware-scheduled
// one-workgroup-per-column launch. With p.dyn_fused the walk locates its columns from the lengths in registers (no
// column map yet: it writes one for the later kernels) over a grid the host sized to the lower bound of the column
// count (rows / (label stride + 1)): exactly one column per workgroup when every S_b equals the bound.
template <class F>
__device__ __forceinline__ void walk_columns(const DevProblem &p, F &&body) {
    if (p.dyn_fused) {
        const WaveLengths w = wave_lengths(p);
        if (blockIdx.x == 0) publish_lengths(p, w);
        if (!w.ok) return;
        int *col_b = const_cast<int *>(p.col_b);
        for (int64_t c = blockIdx.x; c < w.C; c += gridDim.x) {
            const ColRef k = wave_locate(w, c);
            if (threadIdx.x == 0) col_b[c] = k.b;  // the column map of the recursion / gradient kernels
            body(k);
        }
        return;
    }
    // (a grid that covers every column -- known here, after resolve_dyn -- needs no counter: one atomic per workgroup
    // on one address would serialise thousands of workgroups for nothing)
    if (!p.steal || (int64_t)gridDim.x >= p.num_cols) {
        for (int64_t ci = blockIdx.x; ci < p.num_cols; ci += gridDim.x) body(col_ref(p, visit_col(p, ci)));
        return;
    }
    __shared__ int64_t next_col[2];
    int par = 0;
    int64_t ci = blockIdx.x;
    while (ci < p.num_cols) {
        unsigned long long mine = 0;
        if (threadIdx.x == 0) mine = atomicAdd(&p.dyn->steal, 1ull);
        body(col_ref(p, visit_col(p, ci)));
        if (threadIdx.x == 0) next_col[par] = (int64_t)gridDim.x + (int64_t)mine;
        __syncthreads();
        ci = uniform64(next_col[par]);
        par ^= 1;
    }
}

// First acts/grads row of lattice column (b, t): packed layout (reference contract) = the internal
// row rowc; padded [B, pad_T, pad_S1, V] layout = (b * pad_T + t) * pad_S1.
__device__ __forceinline__ int64_t acts_col_base(const DevProblem &p, int b, int t, int64_t rowc) {
    return p.pad_S1 ? ((int64_t)b * p.pad_T + t) * p.pad_S1 : rowc;
}

// Alignment-restricted calls (restrict_to_alignment, gpu_workspace_manager.h:191-219): only the rows the recursion
// can use inside the alignment band need the log-softmax. alpha(t, s), s in [min_s(t), max_s(t)], reads rows s and
// s-1 of column t; beta(t, s), s in [min_s(t-1), max_s(t-1)] (t > 0; beta(0, .) only s = 0), reads row s; every
// other cell is -inf, so the other rows' lp only meet -inf and no gradient row outside the window is live. The
// row reads of the pass drop from the whole band to a few rows per column.
__device__ __forceinline__ void align_window(const DevProblem &p, int64_t c, int t, int &lo, int &hi) {
    if (!p.min_s) return;
    int wlo = p.min_s[c] - 1, whi = p.max_s[c];
    if (t > 0) {
        wlo = min(wlo, p.min_s[c - 1]);
        whi = max(whi, p.max_s[c - 1]);
    } else {
        wlo = min(wlo, 0);
        whi = max(whi, 0);
    }
    lo = max(lo, wlo);
    hi = min(hi, whi);
}

// Label of row s as the log-softmax kernels use it (has = s < S). Device labels are not range-checked on the
// host (that would need a sync), so a label outside [0, V) reads no logit: it is returned as -1 (no capture)
// and the row's label logit `ze` starts as NaN: the transitions through that label carry NaN, which the
// recursion turns into NaN or no probability, so the utterance's cost is not finite (NaN / +inf) and its
// gradient non-finite.
// A row without a label (s == S) returns -1 with ze = 0.
__device__ __forceinline__ int checked_label(bool has, int l, int V, float &ze) {
    const bool bad = has && (unsigned)l >= (unsigned)V;
    ze = bad ? __builtin_nanf("") : 0.0f;
    return (has && !bad) ? l : -1;
}

// ln(s) of a row's fp32 exp-sum (s in [1, V] for a finite row) without the fp64 log routine: s = m * 2^e with the
// exponent exact in fp64 and m in [sqrt(1/2), sqrt(2)), whose |log2 m| <= 1/2 the fp32 v_log_f32 resolves to ~3e-8
// absolute -- below the fp32 rounding of s itself. 0 -> -inf, inf / NaN propagate as in log().
__device__ __forceinline__ double log_row_sum(float s) {
    int e = __builtin_amdgcn_frexp_expf(s);
    float m = __builtin_amdgcn_frexp_mantf(s);  // [0.5, 1)
    if (m < 0.70710678f) {
        m *= 2.0f;
        e -= 1;
    }
    return ((double)e + (double)fast_log2(m)) * 0.69314718055994530942;
}

__device__ __forceinline__ void write_row(const DevProblem &p, int64_t row, float m, float sum, float zb, float ze) {
    const double den = -(double)m - log_row_sum(sum);
    p.den[row] = (float)den;
    p.lp[row] = Lp{(double)zb + den, (double)ze + den};
}

// ---- element-type traits of the acts / grads I/O (math is fp32 in registers) ----------------------

struct IoF32 {
    typedef float S;
    static constexpr int E = 4;  // elements per 16-byte vector
    typedef f4 V;
    __device__ static __forceinline__ void unpack(const V &v, float (&x)[E]) {
        x[0] = v.x;
        x[1] = v.y;
        x[2] = v.z;
        x[3] = v.w;
    }
    __device__ static __forceinline__ V pack(const float (&x)[E]) { return (V){x[0], x[1], x[2], x[3]}; }
    __device__ static __forceinline__ float to_f(S s) { return s; }
    __device__ static __forceinline__ S from_f(float f) { return f; }
};

struct IoBF16 {
    typedef unsigned short S;  // bf16 bits
    static constexpr int E = 8;
    typedef u4 V;
    __device__ static __forceinline__ void unpack(const V &v, float (&x)[E]) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            x[2 * i] = __uint_as_float(v[i] << 16);
            x[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
        }
    }
    __device__ static __forceinline__ unsigned pack2(float a, float b) {  // v_cvt_pk_bf16_f32, RNE
        const unsigned short lo = __builtin_bit_cast(unsigned short, (__bf16)a);
        const unsigned short hi = __builtin_bit_cast(unsigned short, (__bf16)b);
        return (unsigned)lo | ((unsigned)hi << 16);
    }
    __device__ static __forceinline__ V pack(const float (&x)[E]) {
        return (V){pack2(x[0], x[1]), pack2(x[2], x[3]), pack2(x[4], x[5]), pack2(x[6], x[7])};
    }
    __device__ static __forceinline__ float to_f(S s) { return __uint_as_float((unsigned)s << 16); }
    __device__ static __forceinline__ S from_f(float f) { return __builtin_bit_cast(unsigned short, (__bf16)f); }
};

struct IoF16 {
    typedef unsigned short S;  // binary16 bits
    static constexpr int E = 8;
    typedef u4 V;
    __device__ static __forceinline__ float h2f(unsigned short h) { return (float)__builtin_bit_cast(_Float16, h); }
    __device__ static __forceinline__ void unpack(const V &v, float (&x)[E]) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            x[2 * i] = h2f((unsigned short)(v[i] & 0xffffu));
            x[2 * i + 1] = h2f((unsigned short)(v[i] >> 16));
        }
    }
    __device__ static __forceinline__ unsigned pack2(float a, float b) {
        const unsigned short lo = __builtin_bit_cast(unsigned short, (_Float16)a);
        const unsigned short hi = __builtin_bit_cast(unsigned short, (_Float16)b);
        return (unsigned)lo | ((unsigned)hi << 16);
    }
    __device__ static __forceinline__ V pack(const float (&x)[E]) {
        return (V){pack2(x[0], x[1]), pack2(x[2], x[3]), pack2(x[4], x[5]), pack2(x[6], x[7])};
    }
    __device__ static __forceinline__ float to_f(S s) { return h2f(s); }
    __device__ static __forceinline__ S from_f(float f) { return __builtin_bit_cast(unsigned short, (_Float16)f); }
};

// ---- per-row gradient coefficients (shared by the gradient kernels of mrnnt_grad.hip and mrnnt_joint.hip) ----
// g[v] = exp(z[v] + den + alpha(t-1,s) + beta(t,s) - ll) - [v == blank] cb - [v == label(s)] ce

struct RowCoef {
    float c2;   // (den + alpha(t-1,s) + beta(t,s) - ll) * log2(e)
    float cb;   // blank correction
    float ce;   // label correction
    int lab;    // label(s) (-1 for s == S or label == blank)
    bool live;  // false: the row's gradient is exactly 0 (kDeadLogOcc) and acts need not be read
};

// alpha(t-1, s) of an in-band row (alpha(-1, s) = [s == 0])
__device__ __forceinline__ double alpha_prev(const DevProblem &p, int t, int s, int64_t row, int W) {
    return (t == 0) ? (s == 0 ? 0.0 : NEG_INF_D) : p.alpha[row - W];
}

// Value of a row whose gradient is not computed (out of band, or dead), times the upstream gradient: the CPU
// reference -- the parity oracle -- forms every row as exp(... - ll) (cpu_rnnt.h:221-231), i.e. 0 for a finite
// log-likelihood and NaN for ll = -inf (no path survives, e.g. an alignment band that excludes them all) or NaN.
// The reference's GPU kernel writes a literal 0 to out-of-band rows instead (gpu_rnnt_kernel.h:266-271), so for
// ll = -inf the two reference paths disagree on those rows; this build follows cpu_rnnt.h.
__device__ __forceinline__ float zero_row_value(double ll, float sc) {
    return (ll > NEG_INF_D ? 0.0f : __builtin_nanf("")) * sc;
}

// The dead-row predicate (mrnnt_host.h kDeadLogOcc); NaN state is live.
__device__ __forceinline__ bool row_live(double log_occ) { return !(log_occ < kDeadLogOcc); }

__device__ __forceinline__ RowCoef row_coef(const DevProblem &p, int t, int T, int S, int s, int64_t row, double ll,
                                            const int *__restrict__ lab_b) {
    const int W = S + 1;
    const double am = alpha_prev(p, t, s, row, W);
    const double b0 = p.beta[row];
    const double b1 = (t == T - 1) ? (s == S ? 0.0 : NEG_INF_D) : p.beta[row + W];
    const double b2 = (s == S) ? NEG_INF_D : ((t == T - 1) ? (s + 1 == S ? 0.0 : NEG_INF_D) : p.beta[row + W + 1]);
    const double base = am - ll;
    RowCoef rc;
    rc.live = !p.occ_skip || row_live(base + b0);
    rc.c2 = (float)(((double)p.den[row] + base + b0) * kLog2eD);
    // the exponents are O(10) after the fp64 cancellation of alpha + beta - ll: fp32 v_exp_f32 on the
    // rounded exponent (relative error ~1e-6 of a coefficient <= 1)
    const Lp l = p.lp[row];
    rc.cb = fast_exp2((float)((l.b + base + b1) * kLog2eD));
    rc.ce = (s < S) ? fast_exp2((float)((l.e + base + b2) * kLog2eD)) : 0.0f;
    const int lab = (s < S) ? lab_b[s] : -1;
    rc.lab = (lab == p.blank || (unsigned)lab >= (unsigned)p.V) ? -1 : lab;  // out of range: never matched / written
    return rc;
}

// Device-resident lengths that failed validation: every gradient element is NaN (the costs are NaN too), written
// over the caller's whole grads buffer (rows as the host sized it) by the workgroups of the gradient launch.
template <class IO>
__device__ __forceinline__ void fill_failed_grads(const DevProblem &p, void *grads) {
    typename IO::S *g = static_cast<typename IO::S *>(grads);
    const int64_t rows = p.pad_S1 ? (int64_t)p.B * p.pad_T * p.pad_S1 : p.num_rows;
    const int64_t n = rows * (int64_t)p.V;
    const typename IO::S nan = IO::from_f(__builtin_nanf(""));
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        g[i] = nan;
}

template <bool NT, class V>
__device__ __forceinline__ V vload(const V *ptr) {
    if constexpr (NT)
        return __builtin_nontemporal_load(ptr);
    else
        return *ptr;
}

template <bool NT, class V>
__device__ __forceinline__ void vstore(V *ptr, const V &v) {
    if constexpr (NT)
        __builtin_nontemporal_store(v, ptr);
    else
        *ptr = v;
}

// ---- in-launch hand-off words (the chase launch, mrnnt_chase.hip; cdna_hip_programming.md Guideline 16, R1) ----
// 4- / 8-byte accesses through the GLOBAL address space at agent scope: relaxed atomic stores are write-through
// (`sc1`) and relaxed atomic loads read past this CU's L1 and this XCD's L2 (`sc1`), so a payload stored this way,
// drained (s_waitcnt vmcnt(0)) before a flag store of the same kind, is seen by a consumer on any XCD that loads it
// this way after seeing the flag -- no release / acquire fence.
template <int N> struct WordOf;
template <> struct WordOf<4> { typedef unsigned T; };
template <> struct WordOf<8> { typedef unsigned long long T; };

template <class T>
__device__ __forceinline__ void store_wt(T *ptr, T v) {
    typedef typename WordOf<sizeof(T)>::T W;
    __hip_atomic_store((__attribute__((address_space(1))) W *)ptr, __builtin_bit_cast(W, v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

template <class T>
__device__ __forceinline__ T load_wt(const T *ptr) {
    typedef typename WordOf<sizeof(T)>::T W;
    return __builtin_bit_cast(
        T, __hip_atomic_load((__attribute__((address_space(1))) W *)ptr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// The lp array as a buffer resource: 16-byte write-through stores and L1-bypassing loads of whole Lp rows (an
// agent-scope atomic covers 8 bytes at most; 8-byte sc1 loads run at about half the 16-byte rate). Rows [0, N) only
// (the chase launch checks N * 16 < 2^31 on the host); the descriptor is built from kernel-argument values only.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t lp_rsrc(const DevProblem &p) {
    return __builtin_amdgcn_make_buffer_rsrc(static_cast<void *>(p.lp), (short)0, (int)(p.num_rows * (int64_t)sizeof(Lp)),
                                             0x00020000);
}
constexpr int kAuxSc1 = 16;  // buffer instruction cache-policy bits: sc1
__device__ __forceinline__ Lp load_lp_wt(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff) {
    return __builtin_bit_cast(Lp, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, kAuxSc1));
}
__device__ __forceinline__ void store_lp_wt(__amdgpu_buffer_rsrc_t r, unsigned voff, Lp v) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v), r, voff, 0, kAuxSc1);
}

// every store this wave issued has completed (the drain before a hand-off flag)
// s_waitcnt vmcnt(0) through the builtin, which the compiler's wait-count pass sees: an inline-asm wait is opaque to
// it, so it would go on counting the operations before it as outstanding -- an LDS-DMA among them makes it wait for
// vmcnt(0) again before later LDS accesses, e.g. once per recursion step on the walk's global stores. (The empty asm
// statements keep memory operations from moving across it.)
__device__ __forceinline__ void wait_vmcnt0() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt = 0; expcnt, lgkmcnt unconstrained
    asm volatile("" ::: "memory");
}
__device__ __forceinline__ void drain_stores() { wait_vmcnt0(); }

template <class IO>
__device__ __forceinline__ typename IO::V splat(float f) {
    float x[IO::E];
#pragma unroll
    for (int i = 0; i < IO::E; ++i) x[i] = f;
    return IO::pack(x);
}

template <int E>
__device__ __forceinline__ float pick(const float (&x)[E], int c) {
    float r = x[0];
#pragma unroll
    for (int i = 1; i < E; ++i) r = (c == i) ? x[i] : r;
    return r;
}

}  // namespace mrnnt
