// mrnnt_chase.hip -- the forward pass as one launch: the log-softmax and the alpha / beta recursion
// (§8 a2) overlapped. The reference runs them back to back (gpu_rnnt.h:99-191: the reduce kernels, a device sync,
// then compute_alphas_kernel / compute_betas_kernel); here the recursion is latency-bound (one fp64 LSE chain per
// frame, ~0.1 us) while the log-softmax is HBM-bound, so the recursion workgroups run beside the log-softmax
// workgroups and consume each lattice column as soon as it is published.
//
// Grid: first the recursion workgroups (one per utterance and direction, B or 2B), then G log-softmax workgroups
// that take the slots of the production order round-robin (slot si, si + G, ...). The order feeds both walks from
// their ends: round k publishes frames k and T_b - 1 - k of every utterance (alpha walks up from frame 0, beta down
// from T - 1), so neither walk waits for the whole pass; alpha alone (no beta): round k publishes frame k. G is a
// few workgroups per CU, not one per slot: with every slot's workgroup resident at once the columns would share the
// bandwidth and all land near the end; G at a time, they land in order, batch after batch.
//
// Hand-off (cdna_hip_programming.md Guideline 16, R1): a log-softmax workgroup stores its den / lpb / lpe rows
// write-through (sc1), every wave drains its stores, a barrier, then one lane stores the column's ready flag (one per
// direction). A recursion wave reads a column's lp rows only after seeing its flag and only with sc1 loads
// (mrnnt_dp.h, Chase), never from a stale L1 / L2 line. Nothing else crosses workgroups inside the launch.
//
// Flag words: 64-bit, in the workspace, tagged with the launch's epoch (a fresh host value per call: a producer stores
// it, a consumer waits for exactly it), and cleared by each recursion workgroup when its walk is done -- so a graph
// replay, whose epoch is frozen at capture, starts from cleared flags, and an eager call never needs a memset node
// (4 us of a 90 us configs[1] step). A workspace's words that were never cleared are older epochs (distinct) or
// unrelated bytes, which equal a fresh 64-bit epoch with probability 2^-64 per word. A wait is bounded: a recursion
// workgroup that gives up returns NaN for its utterance.
//
// Every lp value, every LSE and every store is the one the two-kernel path computes (the log-softmax bodies are
// mrnnt_lsm.h's, the recursion passes mrnnt_dp.h's), so results are bit-identical to it.
#include "mrnnt_dp.h"
#include "mrnnt_lsm.h"

namespace mrnnt {

template <int SM, class IO, bool NTL>
__device__ __forceinline__ void chase_column(const DevProblem &p, const ColRef &k) {
    constexpr int U = SM <= 1 ? 1 : (SM <= 3 ? 2 : 4);
    constexpr bool FULL = (SM & 1) == 0;
    if constexpr (SM == 0)
        row16_column<IO, 1, NTL, true>(p, k);
    else
        lean_column<IO, U, 2, NTL, FULL, true, true>(p, k);
}

// SM: the log-softmax body -- 0 rows on 16-lane groups (rows of <= 64 vectors), 2 / 3 single-chunk rows of <= 128
// vectors (U = 2), 4 / 5 of <= 256 (U = 4), even = every chunk full (the product launch_u's choices for these rows).
// NW: recursion waves (1: S + 1 <= 64, one cell per lane; 4: the halo recursion with 56 own cells per wave, S + 1 <=
// 224). D: lp rows prefetched per lane (8: 16-byte rows, 0.8 us ahead; 16 in the development build).
template <class IO, int SM, bool NTL, int NW, int D>
__global__ __launch_bounds__(256) void chase_kernel(DevProblem p, ChaseArgs c, int with_beta, float *__restrict__ costs) {
    constexpr int HL = NW > 1 ? 8 : 0;
    __shared__ double xh[2][8][HL > 0 ? HL : 1];
    __shared__ int fail;
    const int nrec = with_beta ? 2 * p.B : p.B;
    if ((int)blockIdx.x < nrec) {
        // ---- recursion workgroup ----
        if (threadIdx.x >= 64 * NW) return;  // one-wave recursion: the other waves of the workgroup have no work
        if constexpr (kVariants) {
            if (c.probe == 1 || c.probe == 2) return;  // (development probes: the log-softmax side alone; no costs)
        }
        const int b = with_beta ? (int)(blockIdx.x >> 1) : (int)blockIdx.x;
        const bool bwd = with_beta && (blockIdx.x & 1);
        if (threadIdx.x == 0) fail = 0;
        if (NW > 1) __syncthreads();
        Chase ch;
        unsigned long long *mine = c.flags + (bwd ? c.cols : 0) + p.col_off[b];
        ch.init(mine, c.epoch, p.T[b], !bwd, &fail);
        if constexpr (kVariants) {
            ch.nowait = c.probe >= 3;  // (development probes: the recursion without waiting)
            if (c.probe == 5) {        // (development probe: the two-kernel recursion pass inside this launch)
                if (bwd)
                    beta_pass_halo<D, NW, HL, false, 1>(p, b, xh);
                else
                    alpha_pass_halo<D, NW, HL, false, 1>(p, b, costs, xh);
                return;
            }
            if (c.probe == 6) {  // (development probe: the chase pass with plain lp loads, not waiting)
                if (bwd)
                    beta_pass_halo<D, NW, HL, false, 1, true, false>(p, b, xh, &ch);
                else
                    alpha_pass_halo<D, NW, HL, false, 1, true, false>(p, b, costs, xh, &ch);
                return;
            }
        }
        if (bwd)
            beta_pass_halo<D, NW, HL, false, 1, true>(p, b, xh, &ch);
        else
            alpha_pass_halo<D, NW, HL, false, 1, true>(p, b, costs, xh, &ch);
        drain_stores();  // this wave's ll / cost store lands before the NaN below (same address, other wave)
        if (NW > 1) __syncthreads();  // (every wave is past its last poll)
        if (threadIdx.x == 0 && fail) {  // a wave gave up waiting: its cells may have read unpublished rows
            if (bwd) {
                p.llb[b] = __builtin_nan("");
            } else {
                p.ll[b] = __builtin_nan("");
                if (costs) costs[b] = __builtin_nanf("");
            }
        }
        for (int i = threadIdx.x; i < p.T[b]; i += 64 * NW) mine[i] = 0ull;  // cleared for the next launch
        return;
    }
    // ---- log-softmax workgroups: slots si, si + G, ... of the production order (G = the producer grid) ----
    if constexpr (kVariants) {
        if (c.probe >= 4) return;  // (development probes: the recursion side alone)
    }
    const int64_t per = with_beta ? 2 * (int64_t)p.B : (int64_t)p.B;
    const int64_t G = (int64_t)gridDim.x - nrec;
    if (blockIdx.x == (unsigned)nrec && threadIdx.x < 64) {  // the lp pads around [0, N)
        const int i = threadIdx.x;
        p.lp[i - 64] = Lp{0.0, 0.0};
        p.lp[p.num_rows + i] = Lp{0.0, 0.0};
    }
    for (int64_t si = (int64_t)blockIdx.x - nrec; si < c.slots; si += G) {
        const int kr = (int)(si / per);
        const int r = (int)(si - (int64_t)kr * per);
        const int b = with_beta ? (r >> 1) : r;
        const int T = p.T[b];
        int t;
        if (!with_beta) {
            if (kr >= T) continue;
            t = kr;
        } else if (r & 1) {
            t = T - 1 - kr;
            if (t <= kr) continue;  // (the middle frame of an odd T is published by side 0)
        } else {
            if (2 * kr > T - 1) continue;
            t = kr;
        }
        ColRef k;
        k.b = b;
        k.T = T;
        k.S = p.S[b];
        k.t = t;
        k.c = p.col_off[b] + t;
        k.rowc = p.row_off[b] + (int64_t)t * (k.S + 1);
        if constexpr (kVariants) {
            if (c.probe == 2) {  // (development probe: the production order alone -- plain stores, no hand-off)
                if constexpr (SM == 0)
                    row16_column<IO, 1, NTL, false>(p, k);
                else
                    lean_column<IO, SM <= 3 ? 2 : 4, 2, NTL, (SM & 1) == 0, true, false>(p, k);
                continue;
            }
        }
        chase_column<SM, IO, NTL>(p, k);
        drain_stores();  // every wave: its write-through rows have landed
        __syncthreads();
        if (threadIdx.x == 0) {
            store_wt(&c.flags[k.c], c.epoch);
            if (with_beta) store_wt(&c.flags[c.cols + k.c], c.epoch);
        }
    }
}

// The log-softmax body the chase launch carries for this problem (-1: none -- the two-kernel path runs). f32 acts,
// 16-byte aligned rows of <= 256 vectors (V <= 1024), the same shapes launch_u picks for them.
int chase_body(const DevProblem &p, int elem) {
    if (elem != ELEM_F32 || p.V % 4 || (reinterpret_cast<uintptr_t>(p.acts) & 15)) return -1;
    const int VL = p.V / 4;
    if (VL <= 64) return 0;
    if (VL >= 96 && VL <= 128) return VL == 128 ? 2 : 3;
    if (VL >= 192 && VL <= 256) return VL == 256 ? 4 : 5;
    return -1;
}

template <int SM, bool NTL, int D>
static void launch_d(const DevProblem &p, const ChaseArgs &c, int nw, int with_beta, float *costs, int64_t grid,
                     hipStream_t stream) {
    if (nw == 1)
        chase_kernel<IoF32, SM, NTL, 1, D><<<(unsigned)grid, 256, 0, stream>>>(p, c, with_beta, costs);
    else
        chase_kernel<IoF32, SM, NTL, 4, D><<<(unsigned)grid, 256, 0, stream>>>(p, c, with_beta, costs);
}

template <int SM, bool NTL>
static void launch_sm(const DevProblem &p, const ChaseArgs &c, int nw, int with_beta, float *costs, int64_t grid,
                      hipStream_t stream) {
    if constexpr (kVariants) {
        if (tuning().chase_depth == 16) {
            launch_d<SM, NTL, 16>(p, c, nw, with_beta, costs, grid, stream);
            return;
        }
    }
    launch_d<SM, NTL, 8>(p, c, nw, with_beta, costs, grid, stream);
}

template <bool NTL>
static void launch_ntl(const DevProblem &p, const ChaseArgs &c, int sm, int nw, int with_beta, float *costs,
                       int64_t grid, hipStream_t stream) {
    switch (sm) {
        case 0: launch_sm<0, NTL>(p, c, nw, with_beta, costs, grid, stream); break;
        case 2: launch_sm<2, NTL>(p, c, nw, with_beta, costs, grid, stream); break;
        case 3: launch_sm<3, NTL>(p, c, nw, with_beta, costs, grid, stream); break;
        case 4: launch_sm<4, NTL>(p, c, nw, with_beta, costs, grid, stream); break;
        default: launch_sm<5, NTL>(p, c, nw, with_beta, costs, grid, stream); break;
    }
}

int64_t chase_slots(const DevProblem &p, int T_max, int with_beta) {
    const int64_t rounds = with_beta ? (T_max + 1) / 2 : T_max;
    const int64_t per = with_beta ? 2 * (int64_t)p.B : (int64_t)p.B;
    return rounds * per;
}

hipError_t launch_chase(const DevProblem &p, const ChaseArgs &c, int elem, int S_max, int with_beta, int producers,
                        float *costs, hipStream_t stream) {
    const int sm = chase_body(p, elem);
    const int W = S_max + 1;
    if (sm < 0 || W > 4 * 56 || p.min_s || p.dyn || producers < 1) return hipErrorInvalidValue;
    const int64_t grid = (with_beta ? 2 * (int64_t)p.B : (int64_t)p.B) + producers;
    if (grid > (int64_t)1 << 22) return hipErrorInvalidValue;
    const int nw = W <= 64 ? 1 : 4;
    if (nt_acts_loads(p, sizeof(float)))
        launch_ntl<true>(p, c, sm, nw, with_beta, costs, grid, stream);
    else
        launch_ntl<false>(p, c, sm, nw, with_beta, costs, grid, stream);
    return hipGetLastError();
}

}  // namespace mrnnt
