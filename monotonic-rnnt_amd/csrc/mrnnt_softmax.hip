// mrnnt_softmax.hip -- log-softmax row reduce (replaces reference reduce.h:79-154 and the
// strided acts gathers of gpu_rnnt_kernel.h:80-84).
//
// One pass over the in-band rows of acts. Work decomposition: workgroups walk lattice columns (b, t)
// (one workgroup per column by default, or a persistent grid with a monotone utterance cursor); inside a
// column the four waves take rows s. Per row each lane keeps an online (max, sum-exp) over its 16-byte
// vector loads, the lanes are merged (DPP reductions in softmax_lean_kernel, the default for rows of >= 96
// vectors; a shuffle butterfly in softmax_kernel), den = -max - log(sum) is formed in fp64, and the
// blank / label logits are captured from registers on the way, so the kernel also emits
//   lpb[r] = z[r, blank] + den[r],   lpe[r] = z[r, label(s)] + den[r]
// -- the only two log-probs the recursion reads. Rows outside the band are never read; their lp entries
// are zero-filled (finite) so the recursion needs no guards.
#include "mrnnt_lsm.h"

namespace mrnnt {

// Vector path: V % E == 0, 16-byte aligned rows. U = vector loads per lane per chunk (a chunk covers
// 64*U*E elements), R = rows a wave reduces at once (U*R vector loads in flight per lane).
template <class IO, int U, int R, bool NTL>
__global__ __launch_bounds__(256) void softmax_kernel(DevProblem p) {
    resolve_dyn(p);
    zero_lp_pads(p);
    constexpr int NW = 4;
    constexpr int E = IO::E;
    typedef typename IO::V Vec;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int VL = p.V / E;  // vector loads per row
    const Vec *__restrict__ av = reinterpret_cast<const Vec *>(p.acts);
    const int blank = p.blank;
    const int bj = blank / E, bc = blank % E, blane = bj & 63;
    const Vec ninf = splat<IO>(NEG_INF_F);

    walk_columns(p, [&](const ColRef &k) {
    const int64_t c = k.c;
        const int b = k.b, T = k.T, S = k.S, t = k.t;
        const int64_t rowc = k.rowc;
        const int64_t arow = acts_col_base(p, b, t, rowc);
        int lo = max(0, t - (T - S)), hi = min(t, S);
        align_window(p, c, t, lo, hi);
        const int *__restrict__ lab_b = p.labels + (int64_t)b * p.label_stride;
        zero_fill_outside_band<false>(p, rowc, S, lo, hi);

        for (int s = lo + wave * R; s <= hi; s += NW * R) {
            float m[R], sum[R], zb[R], ze[R];
            int lab[R];
            bool ok[R];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int sr = s + r;
                ok[r] = sr <= hi;
                lab[r] = checked_label(ok[r] && sr < S, (ok[r] && sr < S) ? lab_b[sr] : 0, p.V, ze[r]);
                m[r] = NEG_INF_F;
                sum[r] = 0.0f;
                zb[r] = 0.0f;
            }
            for (int base = 0; base < VL; base += 64 * U) {
                Vec x[R][U];
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const int j = base + lane + 64 * u;
                        if (ok[r] && j < VL)
                            x[r][u] = vload<NTL>(&av[(arow + s + r) * (int64_t)VL + j]);
                        else
                            x[r][u] = ninf;
                    }
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    float xf[U][E];
                    float cm = NEG_INF_F;
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const int j = base + lane + 64 * u;
                        IO::unpack(x[r][u], xf[u]);
#pragma unroll
                        for (int i = 0; i < E; ++i) cm = fmaxf(cm, xf[u][i]);
                        if (j == bj) zb[r] = pick<E>(xf[u], bc);
                        if (lab[r] >= 0 && j == lab[r] / E) ze[r] = pick<E>(xf[u], lab[r] % E);
                    }
                    const float mn = fmaxf(m[r], cm);
                    const float mr = (mn == NEG_INF_F) ? 0.0f : mn;
                    float acc = sum[r] * fast_exp2((m[r] - mr) * kLog2e);
#pragma unroll
                    for (int u = 0; u < U; ++u)
#pragma unroll
                        for (int i = 0; i < E; ++i) acc += fast_exp2((xf[u][i] - mr) * kLog2e);
                    sum[r] = acc;
                    m[r] = mn;
                }
            }
#pragma unroll
            for (int r = 0; r < R; ++r) wave_reduce_max_sum(m[r], sum[r]);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if (!ok[r]) continue;
                const float zbv = __shfl(zb[r], blane);
                const float zev = lab[r] >= 0 ? __shfl(ze[r], (lab[r] / E) & 63) : ze[r];  // ze: 0, or NaN (bad label)
                if (lane == 0) write_row(p, rowc + s + r, m[r], sum[r], zbv, zev);
            }
        }
    });
}

template <class IO, int U, int R, bool NTL, bool FULL, bool ONE = false>
__global__ __launch_bounds__(256) void softmax_lean_kernel(DevProblem p) {
    resolve_dyn(p);
    zero_lp_pads(p);
    walk_columns(p, [&](const ColRef &k) { lean_column<IO, U, R, NTL, FULL, ONE, false>(p, k); });
}

template <class IO, int NR, bool NTL>
__global__ __launch_bounds__(256) void softmax_row16_kernel(DevProblem p) {
    resolve_dyn(p);
    zero_lp_pads(p);
    walk_columns(p, [&](const ColRef &k) { row16_column<IO, NR, NTL, false>(p, k); });
}

// Scalar path (any V, any alignment, any element type): one row per wave, lanes stride over v.
template <class IO>
__global__ __launch_bounds__(256) void softmax_scalar_kernel(DevProblem p) {
    resolve_dyn(p);
    zero_lp_pads(p);
    typedef typename IO::S Sc;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int V = p.V;
    const int blank = p.blank;
    const Sc *__restrict__ acts = reinterpret_cast<const Sc *>(p.acts);
    walk_columns(p, [&](const ColRef &k) {
    const int64_t c = k.c;
        const int b = k.b, T = k.T, S = k.S, t = k.t;
        const int64_t rowc = k.rowc;
        const int64_t arow = acts_col_base(p, b, t, rowc);
        int lo = max(0, t - (T - S)), hi = min(t, S);
        align_window(p, c, t, lo, hi);
        const int *__restrict__ lab_b = p.labels + (int64_t)b * p.label_stride;
        zero_fill_outside_band<false>(p, rowc, S, lo, hi);
        for (int s = lo + wave; s <= hi; s += 4) {
            float ze;
            const int lab = checked_label(s < S, s < S ? lab_b[s] : 0, V, ze);
            const Sc *__restrict__ z = acts + (arow + s) * (int64_t)V;
            float m = NEG_INF_F, sum = 0.0f, zb = 0.0f;
            for (int v0 = 0; v0 < V; v0 += 256) {
                float x[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int v = v0 + lane + 64 * u;
                    x[u] = v < V ? IO::to_f(z[v]) : NEG_INF_F;
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
            const float zev = lab >= 0 ? __shfl(ze, lab & 63) : ze;  // ze: 0, or NaN (bad label)
            if (lane == 0) write_row(p, rowc + s, m, sum, zbv, zev);
        }
    });
}

template <class IO, bool NTL, int U>
static void launch_u(const DevProblem &p, int grid, hipStream_t stream) {
    const int VL = p.V / IO::E;
    const bool full = VL % (64 * U) == 0;
    constexpr int RD = U == 1 ? 4 : 2;  // rows per wave of the default (softmax_variant 13)
    if constexpr (!kVariants) {  // the product library: the tuned default only
        if (VL <= 64)
            softmax_row16_kernel<IO, 1, NTL><<<grid, 256, 0, stream>>>(p);
        else if (VL <= 64 * U && full)
            softmax_lean_kernel<IO, U, RD, NTL, true, true><<<grid, 256, 0, stream>>>(p);
        else if (VL <= 64 * U)
            softmax_lean_kernel<IO, U, RD, NTL, false, true><<<grid, 256, 0, stream>>>(p);
        else if (full)
            softmax_lean_kernel<IO, U, RD, NTL, true><<<grid, 256, 0, stream>>>(p);
        else
            softmax_lean_kernel<IO, U, RD, NTL, false><<<grid, 256, 0, stream>>>(p);
    } else {
        const int v = tuning().softmax_variant;
        if (v == 0 || v == 2) {  // first kernel (shuffle butterflies), 1 or 2 rows per wave
            if (v == 0) softmax_kernel<IO, U, 1, NTL><<<grid, 256, 0, stream>>>(p);
            else softmax_kernel<IO, U, 2, NTL><<<grid, 256, 0, stream>>>(p);
            return;
        }
        if ((v == 13 || v == 22 || v == 23) && VL <= 64) {  // 16-lane rows (the default), 1 / 2 rows per group per pass
            if (v != 23) softmax_row16_kernel<IO, 1, NTL><<<grid, 256, 0, stream>>>(p);
            else softmax_row16_kernel<IO, 2, NTL><<<grid, 256, 0, stream>>>(p);
            return;
        }
        if ((v == 13 || v == 21) && VL <= 64 * U) {  // single-chunk rows (the default): wave max first, 4 / 2 rows per wave
            constexpr int RO = U == 1 ? 4 : 2;
            if (full) softmax_lean_kernel<IO, U, RO, NTL, true, true><<<grid, 256, 0, stream>>>(p);
            else softmax_lean_kernel<IO, U, RO, NTL, false, true><<<grid, 256, 0, stream>>>(p);
            return;
        }
        // running-max lean kernel: 13 (rows of several chunks) / 16 (any row) -> 2 rows per wave (4 for rows of < 96
        // vectors), 14 -> 1, 15 -> 4
        const int R = v == 14 ? 1 : (v == 15 || ((v == 13 || v == 16) && U == 1)) ? 4 : 2;
    #define MRNNT_LEAN(RR)                                                                              \
        (full ? softmax_lean_kernel<IO, U, RR, NTL, true><<<grid, 256, 0, stream>>>(p)                 \
              : softmax_lean_kernel<IO, U, RR, NTL, false><<<grid, 256, 0, stream>>>(p))
        if (R == 1) MRNNT_LEAN(1);
        else if (R == 4) MRNNT_LEAN(4);
        else MRNNT_LEAN(2);
    #undef MRNNT_LEAN
    }
}

// U = 16-byte loads per lane per chunk: a 4 KiB chunk for rows of >= 192 vectors, 2 KiB for >= 96, else 1 KiB
template <class IO, bool NTL>
static void launch_vec(const DevProblem &p, int grid, hipStream_t stream) {
    const int VL = p.V / IO::E;
    if (VL >= 192) launch_u<IO, NTL, 4>(p, grid, stream);
    else if (VL >= 96) launch_u<IO, NTL, 2>(p, grid, stream);
    else launch_u<IO, NTL, 1>(p, grid, stream);
}

template <class IO>
static void launch_io(const DevProblem &p, int grid, hipStream_t stream) {
    const bool vec = (p.V % IO::E) == 0 && (reinterpret_cast<uintptr_t>(p.acts) % 16) == 0;
    if (!vec)
        softmax_scalar_kernel<IO><<<grid, 256, 0, stream>>>(p);
    else if (nt_acts_loads(p, sizeof(typename IO::S)))
        launch_vec<IO, true>(p, grid, stream);
    else
        launch_vec<IO, false>(p, grid, stream);
}

hipError_t launch_softmax(const DevProblem &p, int elem, int grid, hipStream_t stream) {
    switch (elem) {
        case ELEM_F32: launch_io<IoF32>(p, grid, stream); break;
        case ELEM_BF16: launch_io<IoBF16>(p, grid, stream); break;
        case ELEM_F16: launch_io<IoF16>(p, grid, stream); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace mrnnt
