// mrnnt_dp.h -- the alpha / beta halo recursion passes (the reference's compute_alphas_kernel /
// compute_betas_kernel, gpu_rnnt_kernel.h:88-232, and cpu_rnnt.h:140-214), shared by the recursion kernels of
// mrnnt_recursion.hip and the chase launch of mrnnt_chase.hip, whose recursion workgroups consume the log-softmax
// columns of the same launch as they are published (CH: every lp row read is gated on its column's ready flag).
#pragma once

#include "mrnnt_device.h"

namespace mrnnt {

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

// Shifts with bound_ctrl: the lane without a source reads 0 (no "old" operand to initialise).
__device__ __forceinline__ double dpp_shr1_bc(double v) {
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x138, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x138, 0xf, 0xf, true);
    return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double dpp_shl1_bc(double v) {
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x130, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x130, 0xf, 0xf, true);
    return __hiloint2double(hi, lo);
}

// Shifts that bring -inf into the lane without a source (alpha: lane 0, beta: lane 63): the low word of -inf is 0
// (bound_ctrl), its high word is the DPP move's old value -- one move per half and no select after it on the chain.
__device__ __forceinline__ double dpp_shr1_ninf(double v) {
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x138, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp((int)0xFFF00000u, __double2hiint(v), 0x138, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double dpp_shl1_ninf(double v) {
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x130, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp((int)0xFFF00000u, __double2hiint(v), 0x130, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}

// One utterance's lattice as a recursion pass walks it: lengths and the offsets of its first row and column. The
// recursion kernels read them from the lattice arrays; the chase launch under device-resident lengths takes them from
// the lengths every wave holds in registers (wave_lengths), before the arrays are published.
struct Utt {
    int T, S;
    int64_t r0, c0;
};

__device__ __forceinline__ Utt utt_of(const DevProblem &p, int b) { return Utt{p.T[b], p.S[b], p.row_off[b], p.col_off[b]}; }

// The passes without a chase (mrnnt_recursion.hip): nothing gates the lp loads.
struct NoChase {
    static constexpr bool kOn = false;
    __device__ __forceinline__ void refresh() {}
    __device__ __forceinline__ void gate(int) {}
};

// Halo recursion (64 < S+1 <= 8 * (64 - HL)): NW waves, one cell per lane, and no per-step barrier. Wave w
// owns C = 64 - HL consecutive cells and its remaining HL lanes recompute the HL cells next to them that the
// neighbouring wave owns (alpha: the cells below, beta: the cells above). Those halo lanes lose one valid lane
// per step (their outer neighbour is not in the wave), so the own cells stay exact for HL steps; then the
// neighbour's HL boundary cells are copied in through LDS (one barrier per HL steps instead of one per step).
// Ch: NoChase, or the chase launch's gate (mrnnt_chase.hip: every lp row is read only after its column's ready flag,
// with sc1 loads).
template <int D, int NW, int HL, bool BAND, int LEAN, class Ch = NoChase>
__device__ __forceinline__ void alpha_pass_halo(const DevProblem &p, const Utt &u, int b, float *__restrict__ costs,
                                                double (*xh)[8][HL > 0 ? HL : 1], Ch *ch = nullptr) {
    constexpr bool CH = Ch::kOn;
    static_assert(!CH || (LEAN && !BAND), "the chase launch runs the lean, unrestricted step");
    static_assert((HL == 0 ? NW == 1 : D % HL == 0) && NW <= 8,
                  "halo refreshes at prefetch-block positions (HL = 0: one wave, no halo); xh sized for <= 8 waves");
    constexpr int C = 64 - HL;
    constexpr int HLD = HL > 0 ? HL : 1;  // divisor for the (compiled-out when HL == 0) refresh logic
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int T = u.T, S = u.S, W = S + 1;
    const int64_t r0 = u.r0, c0 = u.c0;
    const int s0 = wave * C - HL + lane;  // negative for the halo lanes of wave 0 (always out of band)
    const bool own = lane >= HL && s0 < W;
    // LEAN: every row access is a uniform row pointer (SGPRs) + an unsigned lane offset; the halo lanes of wave 0
    // (s0 < 0, never in band) read cell 0
    const unsigned sl = (unsigned)max(s0, 0);
    // Every lane reads the lp of its own row (t, s): lpb for its own transition and lpe for its upper neighbour's,
    // which gets alpha(t-1, s) + lpe(t, s) shifted up one lane -- one 16-byte load per lane and frame.
    // CH: lp rows are read only inside this utterance's column: rows of other columns may not be published yet. The
    // lanes above S (which feed only cells above S) read row S instead (clamped offset, unconditional load -- a load
    // under an exec branch would cost the prefetch its overlap); the halo lanes of wave 0 read row 0 as before.
    const unsigned slc = CH ? min(sl, (unsigned)S) : sl;
    auto ld = [&](const Lp *row) -> Lp {
        if constexpr (CH)
            return load_lp_wt(lp_rsrc(p), slc * (unsigned)sizeof(Lp), (unsigned)((row - p.lp) * (int64_t)sizeof(Lp)));
        else
            return row[slc];
    };

    double a = (s0 == 0) ? 0.0 : NEG_INF_D;
    double pb[D], pe[D];
    int mn[D], mx[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const int tt = min(d, T - 1);
        if constexpr (CH) ch->gate(tt);
        const Lp l = LEAN ? ld(p.lp + (r0 + (int64_t)tt * W)) : p.lp[r0 + (int64_t)tt * W + s0];
        pb[d] = l.b;
        pe[d] = l.e;
        mn[d] = BAND ? p.min_s[c0 + tt] : 0;
        mx[d] = BAND ? p.max_s[c0 + tt] : S;
    }
    double *ap = p.alpha + r0;                                           // alpha row of the next frame
    const Lp *lpp = p.lp + r0 + (int64_t)min(D, T - 1) * W;              // lp row of the next prefetch
    auto step_lean = [&](int t, int d) {
        // unrestricted: no band mask -- a cell above the band only ever sees -inf predecessors (so it is -inf), a
        // cell below it only feeds cells below it and is never read (mrnnt_read_state masks it for inspection);
        // halo lanes are garbage between refreshes exactly as in the masked step (they only feed halo lanes)
        double y = dpp_shr1_bc(a + pe[d]);  // alpha(t-1, s-1) + lpe(t, s-1), from lane s-1
        if (HL == 0 && lane == 0) y = NEG_INF_D;
        const double v = lse2(a + pb[d], y);
        if (BAND) {
            const int lo = max(max(t - (T - 1 - S), mn[d]), 0);
            const int hi = min(min(t + 1, S), mx[d]);
            a = (s0 >= lo && s0 <= hi) ? v : NEG_INF_D;
        } else {
            // the halo lanes of wave 0 stand for cells s < 0 and feed cell 0: they stay -inf
            a = (HL > 0 && s0 < 0) ? NEG_INF_D : v;
        }
        // row pointers advance by W per frame (no per-frame 64-bit multiply on the scalar unit)
        if (own) ap[sl] = a;
        ap += W;
        if constexpr (CH) ch->gate(min(t + D, T - 1));
        const Lp l = ld(lpp);
        pb[d] = l.b;
        pe[d] = l.e;
        if (t + D < T - 1) lpp += W;
        if (BAND) {
            const int tn = min(t + D, T - 1);
            mn[d] = p.min_s[c0 + tn];
            mx[d] = p.max_s[c0 + tn];
        }
    };
    auto step = [&](int t, int d) {
        if (LEAN) {
            step_lean(t, d);
            return;
        }
        const int lo = max(max(t - (T - 1 - S), mn[d]), 0);
        const int hi = min(min(t + 1, S), mx[d]);
        double y = dpp_shr1(a + pe[d]);  // lane 0: garbage that only ever feeds halo lanes ...
        if (HL == 0 && lane == 0) y = NEG_INF_D;  // ... or, with no halo, alpha(t-1, -1) + lpe
        const double v = lse2(a + pb[d], y);
        a = (s0 >= lo && s0 <= hi) ? v : NEG_INF_D;
        if (own) p.alpha[r0 + (int64_t)t * W + s0] = a;
        const int tn = min(t + D, T - 1);
        const Lp l = p.lp[r0 + (int64_t)tn * W + s0];
        pb[d] = l.b;
        pe[d] = l.e;
        mn[d] = BAND ? p.min_s[c0 + tn] : 0;
        mx[d] = BAND ? p.max_s[c0 + tn] : S;
    };
    // whole blocks of D == HL steps (no early exit inside: the vmcnt waits stay D steps deep), a halo refresh from
    // the wave below (its top HL own cells) after each, then the tail
    int t0 = 0;
    for (; t0 + D <= T; t0 += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            if constexpr (CH) if (d == 0) ch->refresh();
            step(t0 + d, d);
            if (HL > 0 && (d + 1) % HLD == 0 && (d + 1 < D || t0 + D < T)) {
                const int par = ((t0 + d) / HLD) & 1;
                if (lane >= C) xh[par][wave][lane - C] = a;
                __syncthreads();
                if (wave > 0 && lane < HL) a = xh[par][wave - 1][lane];
            }
        }
    }
#pragma unroll
    for (int d = 0; d < D; ++d) {
        if (t0 + d >= T) break;
        step(t0 + d, d);
        if (HL > 0 && (d + 1) % HLD == 0 && t0 + d + 1 < T) {
            const int par = ((t0 + d) / HLD) & 1;
            if (lane >= C) xh[par][wave][lane - C] = a;
            __syncthreads();
            if (wave > 0 && lane < HL) a = xh[par][wave - 1][lane];
        }
    }
    if (own && s0 == S) {
        p.ll[b] = a;
        if (costs) costs[b] = (float)(-a);
    }
}

template <int D, int NW, int HL, bool BAND, int LEAN, class Ch = NoChase>
__device__ __forceinline__ void beta_pass_halo(const DevProblem &p, const Utt &u, int b,
                                               double (*xh)[8][HL > 0 ? HL : 1], Ch *ch = nullptr) {
    constexpr bool CH = Ch::kOn;
    static_assert(!CH || (LEAN && !BAND), "the chase launch runs the lean, unrestricted step");
    static_assert((HL == 0 ? NW == 1 : D % HL == 0) && NW <= 8,
                  "halo refreshes at prefetch-block positions (HL = 0: one wave, no halo); xh sized for <= 8 waves");
    constexpr int C = 64 - HL;
    constexpr int HLD = HL > 0 ? HL : 1;  // divisor for the (compiled-out when HL == 0) refresh logic
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int T = u.T, S = u.S, W = S + 1;
    const int64_t r0 = u.r0, c0 = u.c0;
    const int s0 = wave * C + lane;  // lanes >= C: halo, the first HL cells of the wave above
    const bool own = lane < C && s0 < W;
    const unsigned sl = (unsigned)s0;
    // CH: lp rows read only inside this utterance's column: the cells above S (which stay -inf) read row S instead
    // (clamped offset, unconditional load; as alpha_pass_halo)
    const unsigned slc = CH ? min(sl, (unsigned)S) : sl;
    auto ld = [&](const Lp *row) -> Lp {
        if constexpr (CH)
            return load_lp_wt(lp_rsrc(p), slc * (unsigned)sizeof(Lp), (unsigned)((row - p.lp) * (int64_t)sizeof(Lp)));
        else
            return row[slc];
    };

    double bn = (s0 == S) ? 0.0 : NEG_INF_D;  // beta(T, s)
    double pb[D], pe[D];
    int mn[D], mx[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const int tt = max(T - 1 - d, 0);
        if constexpr (CH) ch->gate(tt);
        const Lp l = ld(p.lp + (r0 + (int64_t)tt * W));
        pb[d] = l.b;
        pe[d] = l.e;
        mn[d] = (BAND && tt > 0) ? p.min_s[c0 + tt - 1] : 0;
        mx[d] = (BAND && tt > 0) ? p.max_s[c0 + tt - 1] : S;
    }
    double *bp_ = p.beta + r0 + (int64_t)(T - 1) * W;                   // beta row of the next frame (downwards)
    const Lp *lpp = p.lp + r0 + (int64_t)max(T - 1 - D, 0) * W;          // lp row of the next prefetch
    auto step_lean = [&](int t, int d) {
        // unrestricted: no band mask -- a cell below the band only sees -inf successors, one above it (s > t) only
        // feeds cells above it and is never read (mrnnt_read_state masks it for inspection)
        double carry = dpp_shl1_bc(bn);
        if (HL == 0 && lane == 63) carry = NEG_INF_D;
        const double v = lse2(bn + pb[d], carry + pe[d]);
        if (BAND) {
            int lo = 0, hi = 0;
            if (t > 0) {
                lo = max(max(t - (T - S), mn[d]), 0);
                hi = min(min(t, S), mx[d]);
            }
            bn = (s0 >= lo && s0 <= hi) ? v : NEG_INF_D;
        } else {
            // lanes past S (halo lanes of the top wave) feed cell S from above: they stay -inf (with one wave, lane
            // 63's successor is -inf and so are they)
            bn = (HL > 0 && s0 > S) ? NEG_INF_D : v;
        }
        if (own) bp_[sl] = bn;
        bp_ -= W;
        if constexpr (CH) ch->gate(max(t - D, 0));
        const Lp l = ld(lpp);
        pb[d] = l.b;
        pe[d] = l.e;
        if (t - D > 0) lpp -= W;
        if (BAND) {
            const int tn = max(t - D, 0);
            mn[d] = tn > 0 ? p.min_s[c0 + tn - 1] : 0;
            mx[d] = tn > 0 ? p.max_s[c0 + tn - 1] : S;
        }
    };
    auto step = [&](int t, int d) {
        if (LEAN) {
            step_lean(t, d);
            return;
        }
        int lo, hi;
        if (t == 0) {
            lo = 0;
            hi = 0;
        } else {
            lo = max(max(t - (T - S), mn[d]), 0);
            hi = min(min(t, S), mx[d]);
        }
        double carry = dpp_shl1(bn);  // lane 63: garbage that only ever feeds halo lanes ...
        if (HL == 0 && lane == 63) carry = NEG_INF_D;  // ... or, with no halo, beta(t+1, 64) (S + 1 <= 64)
        const double v = lse2(bn + pb[d], carry + pe[d]);
        bn = (s0 >= lo && s0 <= hi) ? v : NEG_INF_D;
        if (own) p.beta[r0 + (int64_t)t * W + s0] = bn;
        const int tn = max(t - D, 0);
        const Lp l = p.lp[r0 + (int64_t)tn * W + s0];
        pb[d] = l.b;
        pe[d] = l.e;
        mn[d] = (BAND && tn > 0) ? p.min_s[c0 + tn - 1] : 0;
        mx[d] = (BAND && tn > 0) ? p.max_s[c0 + tn - 1] : S;
    };
    int t0 = T - 1;
    for (; t0 - D + 1 >= 0; t0 -= D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            if constexpr (CH) if (d == 0) ch->refresh();
            step(t0 - d, d);
            if (HL > 0 && (d + 1) % HLD == 0 && (d + 1 < D || t0 - D >= 0)) {  // refresh from the wave above
                const int par = ((T - 1 - t0 + d) / HLD) & 1;
                if (lane < HL) xh[par][wave][lane] = bn;
                __syncthreads();
                if (wave < NW - 1 && lane >= C) bn = xh[par][wave + 1][lane - C];
            }
        }
    }
#pragma unroll
    for (int d = 0; d < D; ++d) {
        if (t0 - d < 0) break;
        step(t0 - d, d);
        if (HL > 0 && (d + 1) % HLD == 0 && t0 - d - 1 >= 0) {
            const int par = ((T - 1 - t0 + d) / HLD) & 1;
            if (lane < HL) xh[par][wave][lane] = bn;
            __syncthreads();
            if (wave < NW - 1 && lane >= C) bn = xh[par][wave + 1][lane - C];
        }
    }
    if (threadIdx.x == 0) p.llb[b] = bn;
}

}  // namespace mrnnt
