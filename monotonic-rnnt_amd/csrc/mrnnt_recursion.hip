// mrnnt_recursion.hip -- alpha / beta recursion over the monotonic lattice (replaces the
// reference's compute_alphas_kernel / compute_betas_kernel, gpu_rnnt_kernel.h:88-232, and the CPU
// recursion cpu_rnnt.h:140-214). One workgroup per (utterance, direction); the two directions of an
// utterance run concurrently (with_beta), so the whole batch is one launch of 2B workgroups.
//
// Monotonic transitions (one label or blank per frame):
//   alpha(t, s) = lse(alpha(t-1, s) + lpb(t, s), alpha(t-1, s-1) + lpe(t, s-1))
//   beta(t, s)  = lse(beta(t+1, s) + lpb(t, s), beta(t+1, s+1) + lpe(t, s))
// restricted to the band s <= t+1, S-s <= T-1-t (and the alignment band min_s/max_s when given).
// State and LSE are fp64 (the reference's accumulation type, rnnt_helper.h:16-30).
#include "mrnnt_dp.h"

namespace mrnnt {

// NW-wave recursion: 64*NW lanes per (utterance, direction), K consecutive cells s per lane.
// The s-1 (alpha) / s+1 (beta) neighbour crosses lanes with a DPP wave shift (v_mov_b32_dpp
// wave_shr:1 / wave_shl:1, no LDS round trip) and crosses waves through a double-buffered LDS slot,
// one s_barrier per step. The lp arrays are finite on every row of [0, S] (the log-softmax kernels
// zero-fill out-of-band rows), so a predecessor at -inf stays -inf without guards; the only
// non-finite case left in the LSE is both inputs at -inf.

template <int K, int D, int NW, bool BAND>
__device__ __forceinline__ void alpha_pass(const DevProblem &p, int b, float *__restrict__ costs, double (*xb)[8]) {
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
        const Lp *rl = p.lp + r0 + (int64_t)tt * W + s0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            pb[d][k] = rl[k].b;
            pe[d][k] = rl[k - 1].e;
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
            const Lp *rl = p.lp + r0 + (int64_t)tn * W + s0;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                pb[d][k] = rl[k].b;
                pe[d][k] = rl[k - 1].e;
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
__device__ __forceinline__ void beta_pass(const DevProblem &p, int b, double (*xb)[8]) {
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
        const Lp *rl = p.lp + r0 + (int64_t)tt * W + s0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            pb[d][k] = rl[k].b;
            pe[d][k] = rl[k].e;
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
            const Lp *rl = p.lp + r0 + (int64_t)tn * W + s0;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                pb[d][k] = rl[k].b;
                pe[d][k] = rl[k].e;
            }
            mn[d] = (band && tn > 0) ? p.min_s[c0 + tn - 1] : 0;
            mx[d] = (band && tn > 0) ? p.max_s[c0 + tn - 1] : S;
            if (NW > 1) __syncthreads();
        }
    }
    if (threadIdx.x == 0) p.llb[b] = bn[0];
}

// Device-resident lengths that failed validation (mrnnt_setup.hip, setup_dyn_kernel): the workgroup's lengths may be
// anything, so it touches no lattice array -- its cost and log-likelihoods are NaN.
__device__ __forceinline__ bool dyn_failed(const DevProblem &p, int b, bool bwd, float *costs) {
    if (!p.dyn || !__builtin_amdgcn_readfirstlane(p.dyn->status)) return false;
    if (threadIdx.x == 0) {
        if (bwd) {
            p.llb[b] = __builtin_nan("");
        } else {
            p.ll[b] = __builtin_nan("");
            if (costs) costs[b] = __builtin_nanf("");
        }
    }
    return true;
}

template <int K, int D, int NW, bool BAND>
__global__ __launch_bounds__(64 * NW) void recursion_kernel(DevProblem p, int with_beta, float *__restrict__ costs) {
    __shared__ double xb[2][8];
    const int b = with_beta ? (int)(blockIdx.x >> 1) : (int)blockIdx.x;
    const bool bwd = with_beta && (blockIdx.x & 1);
    if (dyn_failed(p, b, bwd, costs)) return;
    if (bwd)
        beta_pass<K, D, NW, BAND>(p, b, xb);
    else
        alpha_pass<K, D, NW, BAND>(p, b, costs, xb);
}


template <int D, int NW, int HL, bool BAND, int LEAN = 0>
__global__ __launch_bounds__(64 * NW) void recursion_halo_kernel(DevProblem p, int with_beta,
                                                                 float *__restrict__ costs) {
    __shared__ double xh[2][8][HL > 0 ? HL : 1];
    const int b = with_beta ? (int)(blockIdx.x >> 1) : (int)blockIdx.x;
    const bool bwd = with_beta && (blockIdx.x & 1);
    if (dyn_failed(p, b, bwd, costs)) return;
    const Utt u = utt_of(p, b);
    if (bwd)
        beta_pass_halo<D, NW, HL, BAND, LEAN>(p, u, b, xh);
    else
        alpha_pass_halo<D, NW, HL, BAND, LEAN>(p, u, b, costs, xh);
}

template <int NW, int HL = 8>
static void launch_halo(const DevProblem &p, int with_beta, float *costs, hipStream_t stream) {
    const int blocks = with_beta ? 2 * p.B : p.B;
    if constexpr (!kVariants) {  // the product library: 16-step prefetch blocks, the lean step when unrestricted
        if (p.min_s)
            recursion_halo_kernel<16, NW, HL, true><<<blocks, 64 * NW, 0, stream>>>(p, with_beta, costs);
        else
            recursion_halo_kernel<16, NW, HL, false, 1><<<blocks, 64 * NW, 0, stream>>>(p, with_beta, costs);
    } else {
        if (tuning().dp_lean && tuning().dp_halo == 2 && !p.min_s) {  // unrestricted: the lean step
            recursion_halo_kernel<16, NW, HL, false, 1><<<blocks, 64 * NW, 0, stream>>>(p, with_beta, costs);
            return;
        }
        if (tuning().dp_halo == 2) {  // 16-step prefetch blocks
            if (p.min_s)
                recursion_halo_kernel<16, NW, HL, true><<<blocks, 64 * NW, 0, stream>>>(p, with_beta, costs);
            else
                recursion_halo_kernel<16, NW, HL, false><<<blocks, 64 * NW, 0, stream>>>(p, with_beta, costs);
            return;
        }
        if (p.min_s)
            recursion_halo_kernel<8, NW, HL, true><<<blocks, 64 * NW, 0, stream>>>(p, with_beta, costs);
        else
            recursion_halo_kernel<8, NW, HL, false><<<blocks, 64 * NW, 0, stream>>>(p, with_beta, costs);
    }
}

template <int K, int NW>
static void launch_k(const DevProblem &p, int with_beta, float *costs, hipStream_t stream) {
    // D = rows of lp prefetched ahead (register ring), shallower where K cells per lane use the registers
    constexpr int D = K <= 2 ? 8 : (K <= 4 ? 4 : (K <= 8 ? 2 : 1));
    const int blocks = with_beta ? 2 * p.B : p.B;
    if (p.min_s)
        recursion_kernel<K, D, NW, true><<<blocks, 64 * NW, 0, stream>>>(p, with_beta, costs);
    else
        recursion_kernel<K, D, NW, false><<<blocks, 64 * NW, 0, stream>>>(p, with_beta, costs);
}

// NW waves x K cells per lane, sized to the longest S+1 of the batch: the per-step latency is one fp64
// LSE chain of K cells plus (NW > 1) one barrier, so small S runs on one wave with no barrier at all.
hipError_t launch_dp(const DevProblem &p, int S_max, int with_beta, float *costs, hipStream_t stream) {
    const int W = S_max + 1;
    if (tuning().dp_halo && W <= 64) {  // one wave, one cell per lane, no halo
        launch_halo<1, 0>(p, with_beta, costs, stream);
        return hipGetLastError();
    }
    if (tuning().dp_halo && W <= 8 * 56) {  // halo recursion: 56 own cells per wave
        switch ((W + 55) / 56) {
            case 2: launch_halo<2>(p, with_beta, costs, stream); break;
            case 3: launch_halo<3>(p, with_beta, costs, stream); break;
            case 4: launch_halo<4>(p, with_beta, costs, stream); break;
            case 5: launch_halo<5>(p, with_beta, costs, stream); break;
            case 6: launch_halo<6>(p, with_beta, costs, stream); break;
            case 7: launch_halo<7>(p, with_beta, costs, stream); break;
            default: launch_halo<8>(p, with_beta, costs, stream); break;
        }
        return hipGetLastError();
    }
    if constexpr (kVariants) {  // dp_halo = 0 (development build): the per-step-barrier kernel for short rows too
        if (W <= 64) launch_k<1, 1>(p, with_beta, costs, stream);
        else if (W <= 128) launch_k<1, 2>(p, with_beta, costs, stream);
        else if (W <= 256) launch_k<1, 4>(p, with_beta, costs, stream);
        if (W <= 256) return hipGetLastError();
    }
    if (W <= 512) launch_k<1, 8>(p, with_beta, costs, stream);
    else if (W <= 1024) launch_k<2, 8>(p, with_beta, costs, stream);
    else if (W <= 1536) launch_k<3, 8>(p, with_beta, costs, stream);
    else if (W <= kMaxLabelsPlusOne) launch_k<4, 8>(p, with_beta, costs, stream);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace mrnnt
