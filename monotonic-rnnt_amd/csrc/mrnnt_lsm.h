// mrnnt_lsm.h -- the log-softmax column bodies (reference reduce.h:79-154 and the acts gathers of
// gpu_rnnt_kernel.h:80-84): one lattice column's in-band rows reduced by one workgroup of 4 waves, emitting den, lpb
// and lpe per row. Shared by the streaming log-softmax kernels (mrnnt_softmax.hip) and the chase launch, where the
// same bodies publish their rows write-through to the recursion workgroups of the launch (mrnnt_chase.hip).
#pragma once

#include "mrnnt_device.h"

namespace mrnnt {

// Per-row lp output of the pass. WT (the chase launch, mrnnt_chase.hip): a 16-byte write-through store (`sc1`), the
// producer half of a hand-off to workgroups of the same launch on other XCDs (cdna_hip_programming.md Guideline 16,
// R1); otherwise a plain store, read by later launches. (den is read by later launches only: plain either way.)
template <bool WT>
__device__ __forceinline__ void st_lp(const DevProblem &p, int64_t row, Lp v) {
    if constexpr (WT)
        store_lp_wt(lp_rsrc(p), (unsigned)(row * (int64_t)sizeof(Lp)), v);
    else
        p.lp[row] = v;
}

// rows of the column that are not reduced: finite lp (the recursion reads them, masked) and den (the gradient's
// per-row coefficient of such a row meets alpha or beta = -inf and comes out exactly 0)
// NWV: the waves sharing the column (4: the whole workgroup; 1: one wave alone, the chase launch's self-help), rows
// [rlo, rhi] of the column only
template <bool WT, int NWV = 4>
__device__ __forceinline__ void zero_fill_outside_band(const DevProblem &p, int64_t rowc, int S, int lo, int hi,
                                                       int rlo = 0, int rhi = 1 << 30) {
    const int first = NWV == 1 ? (int)(threadIdx.x & 63) : (int)threadIdx.x;
    const int stride = NWV == 1 ? 64 : (int)blockDim.x;
    const int end = min(S, rhi);
    for (int s = rlo + first; s <= end; s += stride)
        if (s < lo || s > hi) {
            st_lp<WT>(p, rowc + s, Lp{0.0, 0.0});
            p.den[rowc + s] = 0.0f;
        }
}

// The 64 lp entries either side of [0, N): the recursion's in-band cell s = 0 of utterance 0 adds lpe[-1] to its
// -inf predecessor, and a NaN / +inf left in the (reused) workspace there would turn alpha(0, 0) into NaN (then
// -inf through fmax in the next LSE: an infinite cost). Zeroed by the first workgroup of every log-softmax launch.
__device__ __forceinline__ void zero_lp_pads(const DevProblem &p) {
    if (blockIdx.x == 0 && threadIdx.x < 64) {
        const int i = threadIdx.x;
        p.lp[i - 64] = Lp{0.0, 0.0};
        p.lp[p.num_rows + i] = Lp{0.0, 0.0};
    }
}

// Element v of a lane's slice of the row (x[u][i], vector j = v / E in lane j % 64, u = j / 64 % U) into
// every lane (wave-uniform u, i: one indexed register move), then v_readlane from the owning lane.
template <int N>
__device__ __forceinline__ float lane_pick(const float (&x)[N], int k) {
    typedef float VN __attribute__((ext_vector_type(N)));
    VN v;
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = x[i];
    return v[k];
}

// Lean kernel (softmax_variant 13, the default; 14 / 15 select R = 1 / 4 rows per wave): the same
// column walk and online per-lane (max, sum) as softmax_kernel, with the per-row overhead taken off the
// vector pipe -- (max, sum) merged by DPP reductions into wave-uniform scalars (no ds_bpermute butterfly, one
// exp per lane instead of two per step), blank / label logits read with a uniform indexed move + v_readlane
// (no LDS spill of the row slice), and den / lpb / lpe of the R rows formed in parallel by lanes 0..R-1
// (one fp64 log per R rows). FULL: V is a multiple of 64*U*E (no per-load bounds checks).
// ONE: the row is a single chunk (VL <= 64 U, every configuration up to V = 1024): the wave max is reduced first and
// every lane's exps are taken against it, so there is no per-lane running max, no rescale of lane partial sums
// before the wave sum (one exp and its bookkeeping per row fewer), and the R rows' DPP chains interleave.
// NWV / wv / [rlo, rhi]: the waves sharing the column, this wave's index among them and the rows to produce (the
// producers: 4 waves, every row; the chase launch's self-help: one wave, the rows its recursion lanes read). A row's
// value does not depend on which rows share its pass, so every split produces the same bits.
template <class IO, int U, int R, bool NTL, bool FULL, bool ONE, bool WT, int NWV = 4>
__device__ __forceinline__ void lean_column(const DevProblem &p, const ColRef &k, int wv = -1, int rlo = 0,
                                            int rhi = 1 << 30) {
    constexpr int E = IO::E;
    constexpr int CH = 64 * U;  // vectors per chunk
    typedef typename IO::V Vec;
    const int lane = threadIdx.x & 63;
    const int wave = wv >= 0 ? wv : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int VL = p.V / E;
    const Vec *__restrict__ av = reinterpret_cast<const Vec *>(p.acts);
    const int blank = p.blank;
    const Vec ninf = splat<IO>(NEG_INF_F);
    const int64_t c = k.c;
    const int b = k.b, T = k.T, S = k.S, t = k.t;
    const int64_t rowc = k.rowc;
    const int64_t arow = acts_col_base(p, b, t, rowc);
    int lo = max(0, t - (T - S)), hi = min(t, S);
    align_window(p, c, t, lo, hi);
    const int *__restrict__ lab_b = p.labels + (int64_t)b * p.label_stride;
    zero_fill_outside_band<WT, NWV>(p, rowc, S, lo, hi, rlo, rhi);
    lo = max(lo, rlo);
    hi = min(hi, rhi);

    if constexpr (ONE) {
        for (int s = lo + wave * R; s <= hi; s += NWV * R) {
            const int nrow = __builtin_amdgcn_readfirstlane(min(R, hi - s + 1));
            Vec x[R][U];
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int j = lane + 64 * u;
                    x[r][u] = (r < nrow && (FULL || j < VL)) ? vload<NTL>(&av[(arow + s + r) * (int64_t)VL + j])
                                                             : ninf;
                }
            float xf[R][U * E], M[R], zb[R], ze[R];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const bool has = r < nrow && s + r < S;
                const int lab = checked_label(has, has ? __builtin_amdgcn_readfirstlane(lab_b[s + r]) : 0, p.V,
                                              ze[r]);
                float cm = NEG_INF_F;
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    float t4[E];
                    IO::unpack(x[r][u], t4);
#pragma unroll
                    for (int i = 0; i < E; ++i) {
                        xf[r][u * E + i] = t4[i];
                        cm = fmaxf(cm, t4[i]);
                    }
                }
                const int jb = blank / E;
                zb[r] = __int_as_float(__builtin_amdgcn_readlane(
                    __float_as_int(lane_pick<U * E>(xf[r], (jb >> 6) * E + blank % E)), jb & 63));
                if (lab >= 0) {
                    const int je = lab / E;
                    ze[r] = __int_as_float(__builtin_amdgcn_readlane(
                        __float_as_int(lane_pick<U * E>(xf[r], (je >> 6) * E + lab % E)), je & 63));
                }
                M[r] = wave_max_uniform(cm);
            }
            float em = 0.0f, es = 1.0f, ezb = 0.0f, eze = 0.0f;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if (r >= nrow) break;
                const float off = -((M[r] == NEG_INF_F) ? 0.0f : M[r]) * kLog2e;
                float acc = 0.0f;
#pragma unroll
                for (int k = 0; k < U * E; ++k) acc += fast_exp2(fmaf(xf[r][k], kLog2e, off));
                const float Ssum = wave_sum_uniform(acc);
                if (lane == r) {
                    em = M[r];
                    es = Ssum;
                    ezb = zb[r];
                    eze = ze[r];
                }
            }
            if (lane < nrow) {
                const int64_t row = rowc + s + lane;
                const double den = -(double)em - log_row_sum(es);
                p.den[row] = (float)den;
                st_lp<WT>(p, row, Lp{(double)ezb + den, (double)eze + den});
            }
        }
        return;  // next column
    }
    for (int s = lo + wave * R; s <= hi; s += NWV * R) {
        const int nrow = __builtin_amdgcn_readfirstlane(min(R, hi - s + 1));
        float m[R], sum[R], zb[R], ze[R];
        int lab[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const bool has = r < nrow && s + r < S;
            lab[r] = checked_label(has, has ? __builtin_amdgcn_readfirstlane(lab_b[s + r]) : 0, p.V, ze[r]);
            m[r] = NEG_INF_F;
            sum[r] = 0.0f;
            zb[r] = 0.0f;
        }
        for (int base = 0; base < VL; base += CH) {
            Vec x[R][U];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if (r < nrow) {
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const int j = base + lane + 64 * u;
                        x[r][u] = (FULL || j < VL) ? vload<NTL>(&av[(arow + s + r) * (int64_t)VL + j]) : ninf;
                    }
                } else {
#pragma unroll
                    for (int u = 0; u < U; ++u) x[r][u] = ninf;
                }
            }
#pragma unroll
            for (int r = 0; r < R; ++r) {
                float xf[U * E];
                float cm = NEG_INF_F;
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    float t4[E];
                    IO::unpack(x[r][u], t4);
#pragma unroll
                    for (int i = 0; i < E; ++i) {
                        xf[u * E + i] = t4[i];
                        cm = fmaxf(cm, t4[i]);
                    }
                }
                // blank / label logits: uniform position inside this chunk -> indexed move + readlane
                const int jb = blank / E - base;
                if (jb >= 0 && jb < CH) {
                    const float v = lane_pick<U * E>(xf, (jb >> 6) * E + blank % E);
                    zb[r] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), jb & 63));
                }
                const int je = lab[r] >= 0 ? lab[r] / E - base : -1;
                if (je >= 0 && je < CH) {
                    const float v = lane_pick<U * E>(xf, (je >> 6) * E + lab[r] % E);
                    ze[r] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), je & 63));
                }
                const float mn = fmaxf(m[r], cm);
                const float mr = (mn == NEG_INF_F) ? 0.0f : mn;
                const float off = -mr * kLog2e;
                float acc = 0.0f;  // the first chunk has no running sum to rescale
                if (base > 0) acc = sum[r] * fast_exp2(fmaf(m[r], kLog2e, off));
#pragma unroll
                for (int k = 0; k < U * E; ++k) acc += fast_exp2(fmaf(xf[k], kLog2e, off));
                sum[r] = acc;
                m[r] = mn;
            }
        }
        // merge the lanes: wave max, rescale each lane's sum to it, wave sum (uniform results)
        float em = 0.0f, es = 1.0f, ezb = 0.0f, eze = 0.0f;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (r >= nrow) break;
            const float M = wave_max_uniform(m[r]);
            const float Mr = (M == NEG_INF_F) ? 0.0f : M;
            const float part = sum[r] * fast_exp2((m[r] - Mr) * kLog2e);
            const float Ssum = wave_sum_uniform(part);
            if (lane == r) {
                em = M;
                es = Ssum;
                ezb = zb[r];
                eze = ze[r];
            }
        }
        if (lane < nrow) {
            const int64_t row = rowc + s + lane;
            const double den = -(double)em - log_row_sum(es);
            p.den[row] = (float)den;
            st_lp<WT>(p, row, Lp{(double)ezb + den, (double)eze + den});
        }
    }
}

// 16-lane rows (the default for rows of <= 64 vectors: f32 V <= 256, bf16 / fp16 V <= 512; softmax_variant 13 /
// 22, 23 = two rows per group per pass; configs[1]: 23.7 -> 19.4 us against one wave per row, wave max first). A wave reduces
// four rows at once, one per 16-lane DPP row, so the max and sum reductions are four DPP steps inside the
// hardware row (quad_perm x2, half-row mirror, row mirror) serving all four rows per instruction -- against six
// DPP steps + a readlane per row and reduction when a whole wave holds one row. The blank / label logits (4-byte
// loads issued with the row) and den / lpb / lpe stay per row in lane 0 of each 16-lane group. NR: rows per lane
// group per pass (NR * 4 rows per wave in flight).
template <int CTRL>
__device__ __forceinline__ float dpp16(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), CTRL, 0xf, 0xf, false));
}

template <class IO, int NR, bool NTL, bool WT, int NWV = 4>
__device__ __forceinline__ void row16_column(const DevProblem &p, const ColRef &k, int wv = -1, int rlo = 0,
                                             int rhi = 1 << 30) {
    constexpr int E = IO::E;
    typedef typename IO::V Vec;
    typedef typename IO::S Sc;
    const int lane = threadIdx.x & 63;
    const int g = lane >> 4, l16 = lane & 15;
    const int wave = wv >= 0 ? wv : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int VL = p.V / E;  // <= 64: up to 4 vectors per lane of a group
    const Vec *__restrict__ av = reinterpret_cast<const Vec *>(p.acts);
    const Sc *__restrict__ as = reinterpret_cast<const Sc *>(p.acts);
    const int blank = p.blank;
    const Vec ninf = splat<IO>(NEG_INF_F);
    const int64_t c = k.c;
    const int b = k.b, T = k.T, S = k.S, t = k.t;
    const int64_t rowc = k.rowc;
    const int64_t arow = acts_col_base(p, b, t, rowc);
    int lo = max(0, t - (T - S)), hi = min(t, S);
    align_window(p, c, t, lo, hi);
    const int *__restrict__ lab_b = p.labels + (int64_t)b * p.label_stride;
    zero_fill_outside_band<WT, NWV>(p, rowc, S, lo, hi, rlo, rhi);
    lo = max(lo, rlo);
    hi = min(hi, rhi);

    // wave w, pass k: rows lo + 4 NWV NR k + 4 NR w + 4 r + g (r < NR) -- a row per 16-lane group
    for (int s0 = lo + wave * 4 * NR; s0 <= hi; s0 += NWV * 4 * NR) {
        Vec x[NR][4];
        float zb[NR], ze[NR];
        bool ok[NR];
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const int s = s0 + 4 * r + g;
            ok[r] = s <= hi;
            const int64_t ar = (arow + s) * (int64_t)VL;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int j = l16 + 16 * u;
                x[r][u] = (ok[r] && j < VL) ? vload<NTL>(&av[ar + j]) : ninf;
            }
            zb[r] = 0.0f;
            ze[r] = 0.0f;
            if (ok[r] && l16 == 0) {  // the two logits the recursion needs, loaded with the row
                const int64_t ae = (arow + s) * (int64_t)p.V;
                zb[r] = IO::to_f(as[ae + blank]);
                const bool has = s < S;
                const int lab = checked_label(has, has ? lab_b[s] : 0, p.V, ze[r]);
                if (lab >= 0) ze[r] = IO::to_f(as[ae + lab]);
            }
        }
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            float xf[4 * E];
            float m = NEG_INF_F;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                float t4[E];
                IO::unpack(x[r][u], t4);
#pragma unroll
                for (int i = 0; i < E; ++i) {
                    xf[u * E + i] = t4[i];
                    m = fmaxf(m, t4[i]);
                }
            }
            m = fmaxf(m, dpp16<0xB1>(m));   // quad_perm [1,0,3,2]
            m = fmaxf(m, dpp16<0x4E>(m));   // quad_perm [2,3,0,1]
            m = fmaxf(m, dpp16<0x141>(m));  // row_half_mirror
            m = fmaxf(m, dpp16<0x140>(m));  // row_mirror: every lane of the 16-lane row holds its max
            const float off = -((m == NEG_INF_F) ? 0.0f : m) * kLog2e;
            float acc = 0.0f;
#pragma unroll
            for (int k = 0; k < 4 * E; ++k) acc += fast_exp2(fmaf(xf[k], kLog2e, off));
            acc += dpp16<0xB1>(acc);
            acc += dpp16<0x4E>(acc);
            acc += dpp16<0x141>(acc);
            acc += dpp16<0x140>(acc);
            if (ok[r] && l16 == 0) {
                const int64_t row = rowc + s0 + 4 * r + g;
                const double den = -(double)m - log_row_sum(acc);
                p.den[row] = (float)den;
                st_lp<WT>(p, row, Lp{(double)zb[r] + den, (double)ze[r] + den});
            }
        }
    }
}

}  // namespace mrnnt
