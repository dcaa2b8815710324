// mrnnt_cpu.cpp -- the host (RNNT_CPU) implementation of libmonotonic_rnnt_amd.so: the flat C entry points
// mrnnt_cpu_* (include/mrnnt.h), CpuRNNTWorkspaceManager<float> (include/cpu_workspace_manager.h) and
// CpuRNNTComputer<float> (include/cpu_rnnt.h). It serves the reference's CPU surface
// (src/rnnt_entrypoint.cpp:22-31, pytorch_binding/monotonic_rnnt.cu:16-77) with the GPU path's semantics.
//
// Same three passes as the HIP path, laid out for a multicore host instead of a port of cpu_rnnt.h:
//   1. log-softmax row reduce over the in-band (or alignment-window) rows, OpenMP over lattice columns,
//      SIMD max / exp-sum (fp32 lanes, fp64 block totals) -> den, lpb = z[blank] + den, lpe = z[label] + den
//      (the reference: OpenMP over utterances only and a serial log_sum_exp per element, cpu_rnnt.h:96-111)
//   2. alpha / beta recursion per utterance in fp64 (cpu_rnnt.h:140-214 semantics, rnnt_helper.h:16-30 LSE),
//      OpenMP over utterances x direction
//   3. logit gradient, OpenMP over lattice columns, SIMD exp, dL/dcost fused, rows whose occupancy is below
//      e^-110 written as exact zeros without reading acts (cpu_rnnt.h:216-249 formula)
// Offsets are 64-bit throughout (the reference's int act_index overflows past 2^31 elements).
// The hot row loops are compiled three times (AVX-512 / AVX2+FMA / baseline x86-64) and picked at load
// time by the CPU's features (GCC function multiversioning).
#include <omp.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <string>
#include <vector>

#pragma GCC visibility push(default)
#include "cpu_rnnt.h"
#include "cpu_workspace_manager.h"
#include "mrnnt.h"
#pragma GCC visibility pop
#include "mrnnt_host.h"

using mrnnt::set_error;

namespace {

constexpr double kNegInf = -std::numeric_limits<double>::infinity();

// ---- SIMD row kernels ---------------------------------------------------------------------------------

// e^x in fp32 from plain arithmetic (so the loops vectorise): Cody-Waite reduction by ln 2, degree-6
// polynomial on |r| <= ln2/2 (relative error ~2e-7), exponent assembled in the bits. Results below
// e^-87 (< 1.7e-38, the fp32 normal range) flush to 0; x > 88.7 gives +inf; NaN propagates.
static inline __attribute__((always_inline)) float vexp(float x) {
    constexpr float kMagic = 12582912.0f;  // 1.5 * 2^23: adding it rounds to an integer in the low bits
    const float xc = std::min(std::max(x, -87.0f), 88.7f);
    const float tq = xc * 1.44269504088896341f + kMagic;
    // the integer part in unsigned arithmetic: NaN input makes tq NaN and n garbage (the result is replaced below),
    // which in signed arithmetic was an overflow / negative left shift (UBSan, `make asan`)
    const unsigned n = __builtin_bit_cast(unsigned, tq) - __builtin_bit_cast(unsigned, kMagic);
    const float fn = tq - kMagic;
    float r = xc - fn * 0.693145751953125f;
    r = r - fn * 1.428606765330187045e-06f;
    const float p =
        1.0f + r * (1.0f + r * (0.5f + r * (0.166666672f + r * (0.0416666418f + r * (0.00833345205f +
                                                                                     r * 0.00138888808f)))));
    float res = p * __builtin_bit_cast(float, (n + 127u) << 23);
    res = (x < -87.0f) ? 0.0f : res;
    res = (x > 88.7f) ? std::numeric_limits<float>::infinity() : res;
    return (x != x) ? x : res;
}

constexpr int kBlock = 512;  // elements per fp32 partial-sum block (then accumulated in fp64)

// max and sum_v e^(z_v - max) of one row; NaN elements are skipped by the max and poison the sum
static inline __attribute__((always_inline)) void row_max_sum_body(const float *__restrict__ z, int V, float &m_out,
                                                                   double &sum_out) {
    float m = -std::numeric_limits<float>::infinity();
#pragma omp simd reduction(max : m)
    for (int v = 0; v < V; ++v) m = z[v] > m ? z[v] : m;
    double sum = 0.0;
    for (int v0 = 0; v0 < V; v0 += kBlock) {
        const int v1 = std::min(V, v0 + kBlock);
        float s = 0.0f;
#pragma omp simd reduction(+ : s)
        for (int v = v0; v < v1; ++v) s += vexp(z[v] - m);
        sum += (double)s;
    }
    m_out = m;
    sum_out = sum;
}

// g_v = e^(z_v + c) * sc (g may be z itself: element-wise, each element read before it is written)
static inline __attribute__((always_inline)) void grad_row_body(const float *z, float *g, int V, float c, float sc) {
#pragma omp simd
    for (int v = 0; v < V; ++v) g[v] = vexp(z[v] + c) * sc;
}

__attribute__((target("default"))) void row_max_sum(const float *z, int V, float &m, double &s) {
    row_max_sum_body(z, V, m, s);
}
__attribute__((target("avx2,fma"))) void row_max_sum(const float *z, int V, float &m, double &s) {
    row_max_sum_body(z, V, m, s);
}
__attribute__((target("avx512f,avx512dq,avx512bw,avx512vl,fma"))) void row_max_sum(const float *z, int V, float &m,
                                                                                    double &s) {
    row_max_sum_body(z, V, m, s);
}

__attribute__((target("default"))) void grad_row(const float *z, float *g, int V, float c, float sc) {
    grad_row_body(z, g, V, c, sc);
}
__attribute__((target("avx2,fma"))) void grad_row(const float *z, float *g, int V, float c, float sc) {
    grad_row_body(z, g, V, c, sc);
}
__attribute__((target("avx512f,avx512dq,avx512bw,avx512vl,fma"))) void grad_row(const float *z, float *g, int V,
                                                                                 float c, float sc) {
    grad_row_body(z, g, V, c, sc);
}

// log(e^x + e^y) with fp64 state (rnnt_helper.h:16-30): one -inf input returns the other exactly, both
// -inf is -inf, NaN propagates (the HIP path's lse2 in mrnnt_device.h has the same cases).
inline double lse(double x, double y) {
    const double m = std::fmax(x, y);
    if (m == kNegInf) return kNegInf;
    return m + std::log1p(std::exp(-std::fabs(x - y)));
}

// ---- plan --------------------------------------------------------------------------------------------

struct CpuPlan {
    int B = 0, V = 0, S_max = 0, T_max = 0;
    int64_t N = 0, cols = 0, pad_T = 0, pad_S1 = 0;
    bool align = false;
    std::vector<int64_t> row_off, col_off;
    size_t off_den = 0, off_lpb = 0, off_lpe = 0, off_alpha = 0, off_beta = 0, off_ll = 0, off_llb = 0, off_min = 0,
           off_max = 0, total = 0;
};

constexpr size_t kAlign = 64;
size_t align_up(size_t x) { return (x + kAlign - 1) / kAlign * kAlign; }

RNNTStatus make_cpu_plan(const mrnnt_problem *p, CpuPlan *pl) {
    if (!p) return set_error(RNNT_STATUS_INVALID_VALUE, "null problem");
    if (p->B <= 0) return set_error(RNNT_STATUS_INVALID_VALUE, "B must be > 0");
    if (p->V <= 0) return set_error(RNNT_STATUS_INVALID_VALUE, "V must be > 0");
    if (!p->T_host || !p->S_host) return set_error(RNNT_STATUS_INVALID_VALUE, "host lengths are required");
    if (p->blank < 0 || p->blank >= p->V) return set_error(RNNT_STATUS_INVALID_VALUE, "blank label out of range [0, V)");
    if (p->acts_dtype != MRNNT_F32)
        return set_error(RNNT_STATUS_INVALID_VALUE, "the CPU implementation takes float32 acts only");
    CpuPlan q;
    q.B = p->B;
    q.V = p->V;
    q.row_off.assign(q.B + 1, 0);
    q.col_off.assign(q.B + 1, 0);
    for (int b = 0; b < q.B; ++b) {
        const int T = p->T_host[b], S = p->S_host[b];
        // reference validation: cpu_workspace_manager.h:99-107
        if (T <= 0 || S < 0 || T < S)
            return set_error(RNNT_STATUS_INVALID_VALUE, "invalid lengths at utterance " + std::to_string(b) + ": T=" +
                                                            std::to_string(T) + " S=" + std::to_string(S) +
                                                            " (need T > 0, S >= 0, T >= S)");
        q.row_off[b + 1] = q.row_off[b] + (int64_t)T * (S + 1);
        q.col_off[b + 1] = q.col_off[b] + T;
        q.S_max = std::max(q.S_max, S);
        q.T_max = std::max(q.T_max, T);
    }
    q.N = q.row_off[q.B];
    q.cols = q.col_off[q.B];
    if (q.S_max > 0 && p->label_stride < q.S_max)
        return set_error(RNNT_STATUS_INVALID_VALUE, "label row stride " + std::to_string(p->label_stride) +
                                                        " < max label length " + std::to_string(q.S_max));
    q.align = p->alignment != nullptr;
    if (q.align && p->align_stride < q.T_max)
        return set_error(RNNT_STATUS_INVALID_VALUE, "alignment row stride " + std::to_string(p->align_stride) +
                                                        " < max input length " + std::to_string(q.T_max));
    q.pad_T = p->pad_T;
    q.pad_S1 = p->pad_S1;
    int64_t acts_rows = q.N;
    if (q.pad_S1 != 0) {
        if (q.pad_S1 < (int64_t)q.S_max + 1 || q.pad_T < q.T_max)
            return set_error(RNNT_STATUS_INVALID_VALUE, "padded layout too small for max T " + std::to_string(q.T_max) +
                                                            ", max S " + std::to_string(q.S_max));
        acts_rows = (int64_t)q.B * q.pad_T * q.pad_S1;
    }
    if (p->num_rows >= 0 && p->num_rows != acts_rows)
        return set_error(RNNT_STATUS_INVALID_VALUE, "acts has " + std::to_string(p->num_rows) + " rows but the " +
                                                        (q.pad_S1 ? "padded layout needs " : "lattice needs sum_b T_b(S_b+1) = ") +
                                                        std::to_string(acts_rows));
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t at = o;
        o = align_up(o + bytes);
        return at;
    };
    q.off_den = take(sizeof(float) * q.N);
    q.off_lpb = take(sizeof(double) * q.N);
    q.off_lpe = take(sizeof(double) * q.N);
    q.off_alpha = take(sizeof(double) * q.N);
    q.off_beta = take(sizeof(double) * q.N);
    q.off_ll = take(sizeof(double) * q.B);
    q.off_llb = take(sizeof(double) * q.B);
    q.off_min = q.align ? take(sizeof(int) * q.cols) : 0;
    q.off_max = q.align ? take(sizeof(int) * q.cols) : 0;
    q.total = o;
    *pl = std::move(q);
    return RNNT_STATUS_SUCCESS;
}

RNNTStatus check_inputs(const mrnnt_problem *p, const CpuPlan &pl) {
    if (!p->acts) return set_error(RNNT_STATUS_INVALID_VALUE, "acts is null");
    if (pl.S_max > 0 && !p->labels) return set_error(RNNT_STATUS_INVALID_VALUE, "labels is null");
    for (int b = 0; b < pl.B; ++b) {
        const int *lab = p->labels + (int64_t)b * p->label_stride;
        for (int s = 0; s < p->S_host[b]; ++s)
            if (lab[s] < 0 || lab[s] >= pl.V)
                return set_error(RNNT_STATUS_INVALID_VALUE, "label " + std::to_string(lab[s]) + " at (" +
                                                                std::to_string(b) + ", " + std::to_string(s) +
                                                                ") outside [0, V = " + std::to_string(pl.V) + ")");
    }
    return RNNT_STATUS_SUCCESS;
}

// Workspace views.
struct Views {
    float *den;
    double *lpb, *lpe, *alpha, *beta, *ll, *llb;
    int *min_s, *max_s;
};

Views views(const CpuPlan &pl, void *ws) {
    char *w = static_cast<char *>(ws);
    Views v;
    v.den = reinterpret_cast<float *>(w + pl.off_den);
    v.lpb = reinterpret_cast<double *>(w + pl.off_lpb);
    v.lpe = reinterpret_cast<double *>(w + pl.off_lpe);
    v.alpha = reinterpret_cast<double *>(w + pl.off_alpha);
    v.beta = reinterpret_cast<double *>(w + pl.off_beta);
    v.ll = reinterpret_cast<double *>(w + pl.off_ll);
    v.llb = reinterpret_cast<double *>(w + pl.off_llb);
    v.min_s = pl.align ? reinterpret_cast<int *>(w + pl.off_min) : nullptr;
    v.max_s = pl.align ? reinterpret_cast<int *>(w + pl.off_max) : nullptr;
    return v;
}

// utterance of lattice column c (col_off is increasing)
inline int col_utt(const CpuPlan &pl, int64_t c) {
    return (int)(std::upper_bound(pl.col_off.begin(), pl.col_off.end(), c) - pl.col_off.begin()) - 1;
}

// first acts / grads row of column (b, t) (W = S_b + 1): packed = the lattice row, padded = (b * pad_T + t) * pad_S1
inline int64_t acts_row(const CpuPlan &pl, int b, int t, int W) {
    return pl.pad_S1 ? ((int64_t)b * pl.pad_T + t) * pl.pad_S1 : pl.row_off[b] + (int64_t)t * W;
}

int threads_of(int num_threads) { return num_threads > 0 ? num_threads : omp_get_max_threads(); }

// Alignment band (restrict_to_alignment, cpu_workspace_manager.h:207-224): with m(t) = aligned labels among
// the first t frames, alpha(t, .) lives in [m(t+1-k), m(t+1+k)] (indices clamped to [0, T]).
void band_utt(const int *al, int T, int k, int align_blank, int *min_s, int *max_s) {
    std::vector<int> m(T + 1, 0);
    for (int t = 0; t < T; ++t) m[t + 1] = m[t] + (al[t] != align_blank ? 1 : 0);
    for (int t = 0; t < T; ++t) {
        min_s[t] = m[std::min(std::max(0, t + 1 - k), T)];
        max_s[t] = m[std::max(0, std::min(T, t + 1 + k))];
    }
}

void build_band(const mrnnt_problem *p, const CpuPlan &pl, const Views &w, int nt) {
#pragma omp parallel for schedule(dynamic, 1) num_threads(nt)
    for (int b = 0; b < pl.B; ++b) {
        const int64_t c0 = pl.col_off[b];
        band_utt(p->alignment + (int64_t)b * p->align_stride, p->T_host[b], p->max_shift, p->align_blank,
                 w.min_s + c0, w.max_s + c0);
    }
}

// Rows of column (b, t) the recursion can touch: the band max(0, t-(T-S)) <= s <= min(t, S), narrowed under an
// alignment to the rows alpha(t, [min_s(t), max_s(t)]) and beta(t, [min_s(t-1), max_s(t-1)]) read (the HIP
// path's align_window, mrnnt_device.h). Every other row only meets -inf state.
inline void row_window(const CpuPlan &pl, const Views &w, int64_t c, int t, int T, int S, int &lo, int &hi) {
    lo = std::max(0, t - (T - S));
    hi = std::min(t, S);
    if (!w.min_s) return;
    int wlo = w.min_s[c] - 1, whi = w.max_s[c];
    if (t > 0) {
        wlo = std::min(wlo, w.min_s[c - 1]);
        whi = std::max(whi, w.max_s[c - 1]);
    } else {
        wlo = std::min(wlo, 0);
        whi = std::max(whi, 0);
    }
    lo = std::max(lo, wlo);
    hi = std::min(hi, whi);
}

void softmax_pass(const mrnnt_problem *p, const CpuPlan &pl, const Views &w, int nt) {
    const float *acts = static_cast<const float *>(p->acts);
    const int V = pl.V;
#pragma omp parallel for schedule(dynamic, 4) num_threads(nt)
    for (int64_t c = 0; c < pl.cols; ++c) {
        const int b = col_utt(pl, c);
        const int t = (int)(c - pl.col_off[b]);
        const int T = p->T_host[b], S = p->S_host[b], W = S + 1;
        const int *lab = p->labels ? p->labels + (int64_t)b * p->label_stride : nullptr;
        const int64_t r0 = pl.row_off[b] + (int64_t)t * W;  // lattice row of (t, 0)
        const int64_t a0 = acts_row(pl, b, t, W);           // acts row of (t, 0)
        int lo, hi;
        row_window(pl, w, c, t, T, S, lo, hi);
        for (int s = 0; s < W; ++s) {
            const int64_t r = r0 + s;
            if (s < lo || s > hi) {  // finite filler: the recursion only adds it to -inf state
                w.den[r] = 0.0f;
                w.lpb[r] = 0.0;
                w.lpe[r] = 0.0;
                continue;
            }
            const float *z = acts + (a0 + s) * V;
            float m;
            double sum;
            row_max_sum(z, V, m, sum);
            const double den = -(double)m - std::log(sum);
            w.den[r] = (float)den;
            w.lpb[r] = (double)z[p->blank] + den;
            w.lpe[r] = (s < S) ? (double)z[lab[s]] + den : 0.0;
        }
    }
}

// alpha(t, s) = lse(alpha(t-1, s) + lpb(t, s), alpha(t-1, s-1) + lpe(t, s-1)) on
// max(min_s(t), t-(T-1-S)) <= s <= min(max_s(t), t+1), -inf elsewhere (cpu_rnnt.h:140-161,
// cpu_workspace_manager.h:62-64,160-181); returns alpha(T-1, S).
double alpha_utt(const CpuPlan &pl, const Views &w, int b, int T, int S) {
    const int W = S + 1;
    const int64_t r0 = pl.row_off[b], c0 = pl.col_off[b];
    double *A = w.alpha + r0;
    for (int t = 0; t < T; ++t) {
        int lo = std::max(0, t - (T - 1 - S)), hi = std::min(S, t + 1);
        if (w.min_s) {
            lo = std::max(lo, w.min_s[c0 + t]);
            hi = std::min(hi, w.max_s[c0 + t]);
        }
        double *a = A + (int64_t)t * W;
        const double *ap = A + (int64_t)(t - 1) * W;
        const double *pb = w.lpb + r0 + (int64_t)t * W;
        const double *pe = w.lpe + r0 + (int64_t)t * W;
        for (int s = 0; s < W; ++s) {
            if (s < lo || s > hi) {
                a[s] = kNegInf;
                continue;
            }
            const double stay = (t == 0) ? (s == 0 ? 0.0 : kNegInf) : ap[s];
            const double move = (s == 0) ? kNegInf : ((t == 0) ? (s == 1 ? 0.0 : kNegInf) : ap[s - 1]);
            a[s] = lse(stay + pb[s], (s == 0) ? kNegInf : move + pe[s - 1]);
        }
    }
    return A[(int64_t)(T - 1) * W + S];
}

// beta(t, s) = lse(beta(t+1, s) + lpb(t, s), beta(t+1, s+1) + lpe(t, s)) on
// max(min_s(t-1), t-(T-S)) <= s <= min(max_s(t-1), t) (t > 0; beta(0, .) is s = 0 only), -inf elsewhere,
// beta(T, s) = [s == S] (cpu_rnnt.h:163-214, cpu_workspace_manager.h:66-85,183-205); returns beta(0, 0).
double beta_utt(const CpuPlan &pl, const Views &w, int b, int T, int S) {
    const int W = S + 1;
    const int64_t r0 = pl.row_off[b], c0 = pl.col_off[b];
    double *Bt = w.beta + r0;
    for (int t = T - 1; t >= 0; --t) {
        int lo = 0, hi = 0;
        if (t > 0) {
            lo = std::max(0, t - (T - S));
            hi = std::min(S, t);
            if (w.min_s) {
                lo = std::max(lo, w.min_s[c0 + t - 1]);
                hi = std::min(hi, w.max_s[c0 + t - 1]);
            }
        }
        double *bt = Bt + (int64_t)t * W;
        const double *bn = Bt + (int64_t)(t + 1) * W;
        const double *pb = w.lpb + r0 + (int64_t)t * W;
        const double *pe = w.lpe + r0 + (int64_t)t * W;
        for (int s = 0; s < W; ++s) {
            if (s < lo || s > hi) {
                bt[s] = kNegInf;
                continue;
            }
            const double stay = (t == T - 1) ? (s == S ? 0.0 : kNegInf) : bn[s];
            double move = kNegInf;
            if (s < S) move = ((t == T - 1) ? (s + 1 == S ? 0.0 : kNegInf) : bn[s + 1]) + pe[s];
            bt[s] = lse(stay + pb[s], move);
        }
    }
    return Bt[0];
}

// Gradient of one lattice column (b, t), every row s in [0, S] (cpu_rnnt.h:216-249):
//   g[v] = e^(z[v] + den + alpha(t-1,s) + beta(t,s) - ll) - [v == blank] e^(lpb + alpha(t-1,s) + beta(t+1,s) - ll)
//          - [v == label(s), label != blank] e^(lpe + alpha(t-1,s) + beta(t+1,s+1) - ll),
// times grad_scale[b]. Out-of-band rows are 0 * scale (NaN * scale for ll = -inf: the reference's exp(... - ll)),
// in-band rows below the occupancy threshold (kDeadLogOcc) are exact zeros written without reading acts.
void grad_column(const mrnnt_problem *p, const CpuPlan &pl, const Views &w, const float *scale, float *grads, int b,
                 int t) {
    const int T = p->T_host[b], S = p->S_host[b], W = S + 1, V = pl.V, blank = p->blank;
    const int *lab = p->labels ? p->labels + (int64_t)b * p->label_stride : nullptr;
    const float *acts = static_cast<const float *>(p->acts);
    const float sc = scale ? scale[p->grad_scale_broadcast ? 0 : b] : 1.0f;
    const double ll = w.ll[b];
    const float zero = (ll > kNegInf ? 0.0f : std::numeric_limits<float>::quiet_NaN()) * sc;
    const int64_t r0 = pl.row_off[b] + (int64_t)t * W, a0 = acts_row(pl, b, t, W);
    const double *A = w.alpha + pl.row_off[b], *Bt = w.beta + pl.row_off[b];
    const int lo = std::max(0, t - (T - S)), hi = std::min(t, S);
    for (int s = 0; s < W; ++s) {
        float *g = grads + (a0 + s) * V;
        if (s < lo || s > hi) {
            std::fill(g, g + V, zero);
            continue;
        }
        const double am = (t == 0) ? (s == 0 ? 0.0 : kNegInf) : A[(int64_t)(t - 1) * W + s];
        const double b0 = Bt[(int64_t)t * W + s];
        const double b1 = (t == T - 1) ? (s == S ? 0.0 : kNegInf) : Bt[(int64_t)(t + 1) * W + s];
        const double b2 = (s == S) ? kNegInf : ((t == T - 1) ? (s + 1 == S ? 0.0 : kNegInf) : Bt[(int64_t)(t + 1) * W + s + 1]);
        const double base = am - ll;
        if (base + b0 < mrnnt::kDeadLogOcc) {
            std::fill(g, g + V, 0.0f * sc);
            continue;
        }
        const int64_t r = r0 + s;
        const float c = (float)((double)w.den[r] + base + b0);
        const float *z = acts + (a0 + s) * V;
        const int l = (s < S && (unsigned)lab[s] < (unsigned)V && lab[s] != blank) ? lab[s] : -1;
        const float zb = z[blank], zl = l >= 0 ? z[l] : 0.0f;  // read first: grads may alias acts
        grad_row(z, g, V, c, sc);
        const float cb = (float)std::exp(w.lpb[r] + base + b1);
        g[blank] = (vexp(zb + c) - cb) * sc;
        if (l >= 0) {
            const float ce = (float)std::exp(w.lpe[r] + base + b2);
            g[l] = (vexp(zl + c) - ce) * sc;
        }
    }
}

}  // namespace

// =================================================================================================
// flat C entry points

extern "C" {

RNNTStatus mrnnt_cpu_workspace_size(const mrnnt_problem *p, size_t *bytes) {
    if (!bytes) return set_error(RNNT_STATUS_INVALID_VALUE, "null size pointer");
    CpuPlan pl;
    const RNNTStatus st = make_cpu_plan(p, &pl);
    if (st != RNNT_STATUS_SUCCESS) return st;
    *bytes = pl.total;
    return RNNT_STATUS_SUCCESS;
}

RNNTStatus mrnnt_cpu_forward(const mrnnt_problem *p, void *ws, size_t ws_bytes, float *costs, int with_beta,
                             int num_threads) {
    CpuPlan pl;
    RNNTStatus st = make_cpu_plan(p, &pl);
    if (st != RNNT_STATUS_SUCCESS) return st;
    if ((st = check_inputs(p, pl)) != RNNT_STATUS_SUCCESS) return st;
    if (!ws || ws_bytes < pl.total)
        return set_error(RNNT_STATUS_INVALID_VALUE, "workspace too small: need " + std::to_string(pl.total) + " bytes");
    const Views w = views(pl, ws);
    const int nt = threads_of(num_threads);
    if (pl.align) build_band(p, pl, w, nt);
    softmax_pass(p, pl, w, nt);
    const int dirs = with_beta ? 2 : 1;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nt)
    for (int i = 0; i < pl.B * dirs; ++i) {
        const int b = i / dirs;
        const int T = p->T_host[b], S = p->S_host[b];
        if (i % dirs == 0) {
            const double ll = alpha_utt(pl, w, b, T, S);
            w.ll[b] = ll;
            if (costs) costs[b] = (float)(-ll);
        } else {
            w.llb[b] = beta_utt(pl, w, b, T, S);
        }
    }
    return RNNT_STATUS_SUCCESS;
}

RNNTStatus mrnnt_cpu_backward(const mrnnt_problem *p, const void *ws, const float *grad_scale, float *grads,
                              int num_threads) {
    CpuPlan pl;
    RNNTStatus st = make_cpu_plan(p, &pl);
    if (st != RNNT_STATUS_SUCCESS) return st;
    if (!p->acts) return set_error(RNNT_STATUS_INVALID_VALUE, "acts is null");
    if (!ws) return set_error(RNNT_STATUS_INVALID_VALUE, "workspace is null");
    if (!grads) return set_error(RNNT_STATUS_INVALID_VALUE, "grads is null");
    const Views w = views(pl, const_cast<void *>(ws));
    const int nt = threads_of(num_threads);
#pragma omp parallel for schedule(dynamic, 4) num_threads(nt)
    for (int64_t c = 0; c < pl.cols; ++c) {
        const int b = col_utt(pl, c);
        grad_column(p, pl, w, grad_scale, grads, b, (int)(c - pl.col_off[b]));
    }
    if (pl.pad_S1) {  // padding rows of the padded layout: 0 (the HIP path's pad-zero kernel)
        const int V = pl.V;
#pragma omp parallel for schedule(static) num_threads(nt)
        for (int64_t pc = 0; pc < (int64_t)pl.B * pl.pad_T; ++pc) {
            const int b = (int)(pc / pl.pad_T), t = (int)(pc % pl.pad_T);
            const int T = p->T_host[b], S = p->S_host[b];
            const int s0 = t < T ? S + 1 : 0;
            float *g = grads + (pc * pl.pad_S1 + s0) * V;
            std::fill(g, g + (pl.pad_S1 - s0) * V, 0.0f);
        }
    }
    return RNNT_STATUS_SUCCESS;
}

RNNTStatus mrnnt_cpu_read_state(const mrnnt_problem *p, const void *ws, float *den, double *alpha, double *beta) {
    CpuPlan pl;
    RNNTStatus st = make_cpu_plan(p, &pl);
    if (st != RNNT_STATUS_SUCCESS) return st;
    if (!ws) return set_error(RNNT_STATUS_INVALID_VALUE, "workspace is null");
    const Views w = views(pl, const_cast<void *>(ws));
    if (den) std::memcpy(den, w.den, sizeof(float) * pl.N);
    if (alpha) std::memcpy(alpha, w.alpha, sizeof(double) * pl.N);
    if (beta) std::memcpy(beta, w.beta, sizeof(double) * pl.N);
    return RNNT_STATUS_SUCCESS;
}

}  // extern "C"

// =================================================================================================
// reference-shaped C++ surface (reference include/cpu_workspace_manager.h, include/cpu_rnnt.h)

struct mrnnt_cpu_ws_state {
    const float *acts;
    const int *labels;
    int B, V;
    std::vector<int> T, S;
    std::vector<int64_t> row_off, col_off;  // lattice row / column offsets (row_off[b] + t (S_b+1) + s)
    int S_max = 0, T_max = 0;
    void *workspace = nullptr;
    bool owned = false;
    std::vector<int> alignment;  // copied by restrict_to_alignment, row stride max(T)
    bool restricted = false;
    int max_shift = 0;
    int align_blank = 0;
    std::vector<int> min_s, max_s;  // band per lattice column: the reference's min/max_allowed_s_ (:51-56, :207-224)
    // views of the workspace's per-row state (set_workspace), and the band of the last computation
    float *den = nullptr;
    double *alpha = nullptr, *beta = nullptr;
    bool computed_restricted = false;
    std::vector<int> cmin_s, cmax_s;
};

namespace {

mrnnt_problem cpu_problem_of(const mrnnt_cpu_ws_state *s, int blank) {
    mrnnt_problem p;
    std::memset(&p, 0, sizeof(p));
    p.B = s->B;
    p.V = s->V;
    p.blank = blank;
    p.T_host = s->T.data();
    p.S_host = s->S.data();
    p.acts = s->acts;
    p.labels = s->labels;
    // the reference's strides: labels max(S) (cpu_workspace_manager.h:121), alignment max(T) (:208)
    p.label_stride = s->S_max;
    p.alignment = s->restricted ? s->alignment.data() : nullptr;
    p.align_stride = s->T_max;
    p.align_blank = s->align_blank;
    p.max_shift = s->max_shift;
    p.num_rows = -1;
    return p;
}

RNNTStatus cpu_compute(mrnnt_cpu_ws_state *s, int blank, int num_threads, float *costs, float *grads) {
    if (!costs) return set_error(RNNT_STATUS_INVALID_VALUE, "costs is null");
    if (!s->workspace) return set_error(RNNT_STATUS_INVALID_VALUE, "workspace not set (set_workspace/create_workspace)");
    const mrnnt_problem p = cpu_problem_of(s, blank);
    size_t bytes = 0;
    RNNTStatus st = mrnnt_cpu_workspace_size(&p, &bytes);
    if (st != RNNT_STATUS_SUCCESS) return st;
    st = mrnnt_cpu_forward(&p, s->workspace, bytes, costs, grads != nullptr, num_threads);
    if (st != RNNT_STATUS_SUCCESS) return st;
    s->computed_restricted = s->restricted;
    s->cmin_s = s->min_s;
    s->cmax_s = s->max_s;
    if (!grads) return st;
    return mrnnt_cpu_backward(&p, s->workspace, nullptr, grads, num_threads);
}

constexpr float kNegInfF = -std::numeric_limits<float>::infinity();
constexpr float kNaNF = std::numeric_limits<float>::quiet_NaN();

}  // namespace

CpuRNNTWorkspaceManager<float>::CpuRNNTWorkspaceManager(const float *const acts, const int *const labels, const int B,
                                                        const int *T, const int *S, const int V)
    : st_(new mrnnt_cpu_ws_state) {
    st_->acts = acts;
    st_->labels = labels;
    st_->B = B;
    st_->V = V;
    if (B > 0 && T && S) {
        st_->T.assign(T, T + B);
        st_->S.assign(S, S + B);
        st_->S_max = *std::max_element(S, S + B);
        st_->T_max = *std::max_element(T, T + B);
        st_->row_off.assign(B + 1, 0);
        st_->col_off.assign(B + 1, 0);
        for (int b = 0; b < B; ++b) {  // (invalid lengths are rejected by get_workspace_size; keep offsets sane)
            st_->row_off[b + 1] = st_->row_off[b] + (int64_t)std::max(0, T[b]) * (std::max(0, S[b]) + 1);
            st_->col_off[b + 1] = st_->col_off[b] + std::max(0, T[b]);
        }
        st_->min_s.assign(st_->col_off[B], 0);
        st_->max_s.resize(st_->col_off[B]);
        for (int b = 0; b < B; ++b)
            std::fill(st_->max_s.begin() + st_->col_off[b], st_->max_s.begin() + st_->col_off[b + 1], S[b]);
    }
}

CpuRNNTWorkspaceManager<float>::~CpuRNNTWorkspaceManager() {
    if (st_->owned) std::free(st_->workspace);
    delete st_;
}

RNNTStatus CpuRNNTWorkspaceManager<float>::get_workspace_size(size_t *size_bytes) const {
    if (st_->B <= 0 || (int)st_->T.size() != st_->B) return set_error(RNNT_STATUS_INVALID_VALUE, "B must be > 0");
    // an alignment may be registered later: size for the restricted layout so either works
    mrnnt_problem p = cpu_problem_of(st_, 0);
    int dummy = 0;
    p.alignment = &dummy;
    return mrnnt_cpu_workspace_size(&p, size_bytes);
}

void CpuRNNTWorkspaceManager<float>::set_workspace(void *workspace) {
    if (st_->owned && st_->workspace && st_->workspace != workspace) std::free(st_->workspace);
    st_->workspace = workspace;
    st_->owned = false;
    st_->den = nullptr;
    st_->alpha = st_->beta = nullptr;
    CpuPlan pl;  // the per-row state's offsets do not depend on the alignment (the band comes last)
    const mrnnt_problem p = cpu_problem_of(st_, 0);
    if (workspace && st_->B > 0 && make_cpu_plan(&p, &pl) == RNNT_STATUS_SUCCESS) {
        const Views w = views(pl, workspace);
        st_->den = w.den;
        st_->alpha = w.alpha;
        st_->beta = w.beta;
    }
}

RNNTStatus CpuRNNTWorkspaceManager<float>::create_workspace() {
    size_t bytes = 0;
    const RNNTStatus st = get_workspace_size(&bytes);
    if (st != RNNT_STATUS_SUCCESS) return st;
    void *w = std::malloc(std::max<size_t>(1, bytes));
    if (!w) return set_error(RNNT_STATUS_MEMOPS_FAILED, "malloc workspace");
    set_workspace(w);
    st_->owned = true;
    return RNNT_STATUS_SUCCESS;
}

void CpuRNNTWorkspaceManager<float>::free_workspace() {
    if (st_->owned) std::free(st_->workspace);
    st_->workspace = nullptr;
    st_->owned = false;
    st_->den = nullptr;
    st_->alpha = st_->beta = nullptr;
}

void CpuRNNTWorkspaceManager<float>::restrict_to_alignment(const int *const alignments, int max_shift, int blank_idx) {
    st_->alignment.assign(alignments, alignments + (size_t)st_->B * st_->T_max);
    st_->restricted = true;
    st_->max_shift = max_shift;
    st_->align_blank = blank_idx;
    for (int b = 0; b < st_->B && !st_->col_off.empty(); ++b)
        band_utt(st_->alignment.data() + (size_t)b * st_->T_max, st_->T[b], max_shift, blank_idx,
                 st_->min_s.data() + st_->col_off[b], st_->max_s.data() + st_->col_off[b]);
}

int CpuRNNTWorkspaceManager<float>::B() const { return st_->B; }
int CpuRNNTWorkspaceManager<float>::V() const { return st_->V; }
int CpuRNNTWorkspaceManager<float>::T(int b) const { return st_->T[b]; }
int CpuRNNTWorkspaceManager<float>::S(int b) const { return st_->S[b]; }

int CpuRNNTWorkspaceManager<float>::alpha_s_min(int b, int t) const {
    return std::max(st_->min_s[st_->col_off[b] + t], t - (st_->T[b] - 1 - st_->S[b]));
}
int CpuRNNTWorkspaceManager<float>::alpha_s_max(int b, int t) const {
    return std::min(st_->max_s[st_->col_off[b] + t], t + 1);
}
int CpuRNNTWorkspaceManager<float>::beta_s_min(int b, int t) const {
    return t == 0 ? 0 : std::max(st_->min_s[st_->col_off[b] + t - 1], t - (st_->T[b] - st_->S[b]));
}
int CpuRNNTWorkspaceManager<float>::beta_s_max(int b, int t) const {
    return t == 0 ? 0 : std::min(st_->max_s[st_->col_off[b] + t - 1], t);
}

int CpuRNNTWorkspaceManager<float>::label(int b, int s) const {
    return st_->labels[(int64_t)b * st_->S_max + s];
}

long long CpuRNNTWorkspaceManager<float>::act_index(int b, int t, int s, int v) const {
    return (st_->row_off[b] + (int64_t)t * (st_->S[b] + 1) + s) * (int64_t)st_->V + v;
}

float CpuRNNTWorkspaceManager<float>::act(int b, int t, int s, int v) const { return st_->acts[act_index(b, t, s, v)]; }

void CpuRNNTWorkspaceManager<float>::set_denom(int b, int t, int s, float value) { get_denom(b, t, s) = value; }

float &CpuRNNTWorkspaceManager<float>::get_denom(int b, int t, int s) {
    static thread_local float none;
    if (!st_->den) return none = kNaNF;
    const int T = st_->T[b], S = st_->S[b];
    const int64_t c = st_->col_off[b] + t, r = st_->row_off[b] + (int64_t)t * (S + 1) + s;
    // rows the last computation reduced: the band (and alignment window), as in softmax_pass / row_window
    int lo = std::max(0, t - (T - S)), hi = std::min(t, S);
    if (st_->computed_restricted && !st_->cmin_s.empty()) {
        int wlo = st_->cmin_s[c] - 1, whi = st_->cmax_s[c];
        wlo = std::min(wlo, t > 0 ? st_->cmin_s[c - 1] : 0);
        whi = std::max(whi, t > 0 ? st_->cmax_s[c - 1] : 0);
        lo = std::max(lo, wlo);
        hi = std::min(hi, whi);
    }
    if (s < lo || s > hi) {  // never read by the computation: reduce it now (the reference's pass covers every row)
        float m;
        double sum;
        row_max_sum(st_->acts + r * st_->V, st_->V, m, sum);
        st_->den[r] = (float)(-(double)m - std::log(sum));
    }
    return st_->den[r];
}

void CpuRNNTWorkspaceManager<float>::set_alpha(int b, int t, int s, float value) {
    if (st_->alpha) st_->alpha[st_->row_off[b] + (int64_t)t * (st_->S[b] + 1) + s] = value;
}

float CpuRNNTWorkspaceManager<float>::get_alpha(int b, int t, int s) const {
    // reference cpu_workspace_manager.h:161-181: virtual starts, alignment band, lattice band
    const int T = st_->T[b], S = st_->S[b];
    if (s == -1) return kNegInfF;
    if (t == -1) return s == 0 ? 0.0f : kNegInfF;
    const int64_t c = st_->col_off[b] + t;
    if (s < st_->min_s[c] || s > st_->max_s[c]) return kNegInfF;
    if (s > t + 1 || S - s > T - 1 - t) return kNegInfF;
    if (!st_->alpha) return kNaNF;
    return (float)st_->alpha[st_->row_off[b] + (int64_t)t * (S + 1) + s];
}

void CpuRNNTWorkspaceManager<float>::set_beta(int b, int t, int s, float value) {
    if (st_->beta) st_->beta[st_->row_off[b] + (int64_t)t * (st_->S[b] + 1) + s] = value;
}

float CpuRNNTWorkspaceManager<float>::get_beta(int b, int t, int s) {
    // reference cpu_workspace_manager.h:185-205
    const int T = st_->T[b], S = st_->S[b];
    if (s == S + 1) return kNegInfF;
    if (t == T) return s == S ? 0.0f : kNegInfF;
    const int64_t c = st_->col_off[b] + t;
    if (t > 0 && (s < st_->min_s[c - 1] || s > st_->max_s[c - 1])) return kNegInfF;
    if (s > t || S - s - 1 > T - 1 - t) return kNegInfF;
    if (!st_->beta) return kNaNF;
    return (float)st_->beta[st_->row_off[b] + (int64_t)t * (S + 1) + s];
}

CpuRNNTComputer<float>::CpuRNNTComputer(CpuRNNTWorkspaceManager<float> &workspace_manager, int blank, int num_threads)
    : workspace_manager_(workspace_manager), blank_(blank), num_threads_(num_threads) {}

RNNTStatus CpuRNNTComputer<float>::cost_and_grad(float *costs, float *grads) {
    if (!grads) return set_error(RNNT_STATUS_INVALID_VALUE, "grads is null");
    return cpu_compute(workspace_manager_.state(), blank_, num_threads_, costs, grads);
}

RNNTStatus CpuRNNTComputer<float>::cost(float *costs) {
    return cpu_compute(workspace_manager_.state(), blank_, num_threads_, costs, nullptr);
}
