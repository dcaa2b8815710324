// mrnnt_setup.hip -- per-call metadata on the device (no host copies): lattice row/column offsets from the
// length arrays, the alignment band, and the launch knobs.
#include <algorithm>

#include "mrnnt_device.h"

namespace mrnnt {

Tuning &tuning() {
    static Tuning t;
    return t;
}

// row_off[b] = sum_{b'<b} T_b'(S_b'+1), col_off[b] = sum_{b'<b} T_b' -- one wave, any B (reference
// gpu_workspace_manager.h:256-329 computes these on the host and copies them with blocking memcpys).
// It also zeroes the 64 lp entries either side of the lp array: rows just outside [0, N) that recursion lanes
// outside an utterance's column read, and a NaN / +inf left in the (reused) workspace there must not reach a kept
// cell (it would turn alpha(0, 0) into NaN, then -inf through fmax in the next LSE: an infinite cost).
__global__ __launch_bounds__(64) void setup_kernel(const int *__restrict__ T, const int *__restrict__ S, int B,
                                                   int64_t *__restrict__ row_off, int64_t *__restrict__ col_off,
                                                   Lp *__restrict__ lp, int64_t n) {
    const int lane = threadIdx.x;
    int64_t carry_r = 0, carry_c = 0;
    if (lane == 0) {
        row_off[0] = 0;
        col_off[0] = 0;
    }
    if (lp) {
        lp[lane - 64] = Lp{0.0, 0.0};
        lp[n + lane] = Lp{0.0, 0.0};
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

// Alignment band, reference semantics (gpu_workspace_manager.h:191-219): m[t+1] = #non-blank frames in
// alignment[0..t]; min_s[t] = m[max(0, t+1-k)], max_s[t] = m[min(T, t+1+k)]. A ballot/popcount prefix per
// utterance, then one thread per frame.
__global__ __launch_bounds__(64) void align_prefix_kernel(DevProblem p, const int *__restrict__ alignment,
                                                          int64_t astride, int ablank, int *__restrict__ m) {
    if (!resolve_dyn(p)) return;  // device-resident lengths failed validation: offsets are not trustworthy
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
    if (!resolve_dyn(p)) return;
    for (int b = blockIdx.y; b < p.B; b += gridDim.y) {  // grid y is capped at 65535 utterances per pass
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
}

// col_b[c] = utterance of lattice column c: one load instead of a binary search over col_off per workgroup
__global__ __launch_bounds__(256) void col_map_kernel(const int *__restrict__ T, const int64_t *__restrict__ col_off,
                                                      int *__restrict__ col_b) {
    const int b = blockIdx.x;
    const int64_t c0 = col_off[b];
    for (int t = threadIdx.x; t < T[b]; t += blockDim.x) col_b[c0 + t] = b;
}

hipError_t launch_setup(const int *T, const int *S, int B, int64_t *row_off, int64_t *col_off, int *col_b,
                        Lp *lp, int64_t n, hipStream_t stream) {
    setup_kernel<<<1, 64, 0, stream>>>(T, S, B, row_off, col_off, lp, n);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    col_map_kernel<<<B, 256, 0, stream>>>(T, col_off, col_b);
    return hipGetLastError();
}

hipError_t launch_align(const DevProblem &p, const int *alignment, int64_t align_stride, int align_blank,
                        int max_shift, int *mtmp, int *min_s, int *max_s, hipStream_t stream) {
    align_prefix_kernel<<<p.B, 64, 0, stream>>>(p, alignment, align_stride, align_blank, mtmp);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    align_band_kernel<<<dim3(8, std::min(p.B, 65535)), 256, 0, stream>>>(p, max_shift, mtmp, min_s, max_s);
    return hipGetLastError();
}

// mrnnt_read_state: cells outside the compute band as -inf (the reference getters' values). Without an alignment
// the lean recursion step (mrnnt_recursion.hip) leaves finite values in cells that no in-band cell and no gradient
// row reads.
__global__ __launch_bounds__(64) void mask_state_kernel(DevProblem p, double *__restrict__ alpha,
                                                        double *__restrict__ beta) {
    resolve_dyn(p);
    for (int64_t c = blockIdx.x; c < p.num_cols; c += gridDim.x) {
        const int b = p.col_b[c];
        const int T = p.T[b], S = p.S[b];
        const int t = (int)(c - p.col_off[b]);
        const int64_t rowc = p.row_off[b] + (int64_t)t * (S + 1);
        for (int s = threadIdx.x; s <= S; s += 64) {
            if (alpha && (s > min(t + 1, S) || s < t - (T - 1 - S))) alpha[rowc + s] = -__builtin_huge_val();
            const bool bin = t == 0 ? s == 0 : (s <= t && s >= t - (T - S));
            if (beta && !bin) beta[rowc + s] = -__builtin_huge_val();
        }
    }
}

// The reference manager's view (GpuRNNTWorkspaceManager public members): fp32 alpha / beta, -inf outside the band as
// mask_state_kernel, and the log-likelihoods (any output may be null)
__global__ __launch_bounds__(64) void state_f32_kernel(DevProblem p, float *__restrict__ alpha, float *__restrict__ beta,
                                                       float *__restrict__ ll, float *__restrict__ llb) {
    resolve_dyn(p);
    if (blockIdx.x == 0)
        for (int b = threadIdx.x; b < p.B; b += 64) {
            if (ll) ll[b] = (float)p.ll[b];
            if (llb) llb[b] = (float)p.llb[b];
        }
    for (int64_t c = blockIdx.x; c < p.num_cols; c += gridDim.x) {
        const int b = p.col_b[c];
        const int T = p.T[b], S = p.S[b];
        const int t = (int)(c - p.col_off[b]);
        const int64_t rowc = p.row_off[b] + (int64_t)t * (S + 1);
        for (int s = threadIdx.x; s <= S; s += 64) {
            if (alpha) {
                const bool ain = !(s > min(t + 1, S) || s < t - (T - 1 - S));
                alpha[rowc + s] = ain ? (float)p.alpha[rowc + s] : -__builtin_huge_valf();
            }
            if (beta) {
                const bool bin = t == 0 ? s == 0 : (s <= t && s >= t - (T - S));
                beta[rowc + s] = bin ? (float)p.beta[rowc + s] : -__builtin_huge_valf();
            }
        }
    }
}

hipError_t launch_state_f32(const DevProblem &p, float *alpha, float *beta, float *ll, float *llb, hipStream_t stream) {
    const int grid = (int)(p.num_cols < (1 << 16) ? p.num_cols : (1 << 16));
    state_f32_kernel<<<grid > 0 ? grid : 1, 64, 0, stream>>>(p, alpha, beta, ll, llb);
    return hipGetLastError();
}

hipError_t launch_mask_state(const DevProblem &p, double *alpha, double *beta, hipStream_t stream) {
    const int grid = (int)(p.num_cols < (1 << 16) ? p.num_cols : (1 << 16));
    mask_state_kernel<<<grid > 0 ? grid : 1, 64, 0, stream>>>(p, alpha, beta);
    return hipGetLastError();
}

// ---- device-resident lengths (mrnnt_problem.lengths_on_device) -------------------------------------------------
// One workgroup per utterance: the prefix of the valid lengths before it gives its lattice row / column offsets, it
// writes its own column map entries, and the last workgroup, which reads every length, validates the batch and
// publishes the DynWords (status, real column / row counts, scattered-order multiplier, zeroed work counter) for the
// later kernels of the call. Invalid lengths count as empty utterances, so no offset leaves the capacities the host
// sized; the call then fails closed (DynWords.status: the later kernels write NaN costs and gradients only).
// O(B^2 / 256) length reads in all -- one launch instead of a scan kernel + a map kernel.
__device__ __forceinline__ bool dyn_len_ok(const DynSetupArgs &a, int T, int S) {
    return T > 0 && S >= 0 && T >= S && S <= a.S_cap && (a.T_cap == 0 || T <= a.T_cap) &&
           (a.S1_cap == 0 || (int64_t)S + 1 <= a.S1_cap);
}

// Block sums of (rows, columns, invalid count) in one LDS round (256 threads; every thread gets the sums)
__device__ __forceinline__ void block_sum3(int64_t &r, int64_t &c, int64_t &bad, int64_t (*red)[4]) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        r += __shfl_xor(r, off);
        c += __shfl_xor(c, off);
        bad += __shfl_xor(bad, off);
    }
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = r;
        red[1][threadIdx.x >> 6] = c;
        red[2][threadIdx.x >> 6] = bad;
    }
    __syncthreads();
    r = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    c = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    bad = red[2][0] + red[2][1] + red[2][2] + red[2][3];
}

__global__ __launch_bounds__(256) void setup_dyn_kernel(DynSetupArgs a) {
    __shared__ int64_t red[3][4];
    const int b = blockIdx.x;
    const bool last = b == a.B - 1;
    int64_t r = 0, c = 0, bad = 0;
    const int n = last ? a.B : b;
    for (int i = threadIdx.x; i < n; i += 256) {
        const int T = a.T[i], S = a.S[i];
        const bool ok = dyn_len_ok(a, T, S);
        bad += ok ? 0 : 1;
        if (ok && i < b) {
            r += (int64_t)T * (S + 1);
            c += T;
        }
    }
    block_sum3(r, c, bad, red);
    const int T = a.T[b], S = a.S[b];
    const bool ok = dyn_len_ok(a, T, S);
    const int64_t rb = ok ? (int64_t)T * (S + 1) : 0, cb = ok ? T : 0;
    if (threadIdx.x == 0) {
        if (b == 0) {
            a.row_off[0] = 0;
            a.col_off[0] = 0;
        }
        a.row_off[b + 1] = r + rb;
        a.col_off[b + 1] = c + cb;
    }
    if (ok && c + cb <= a.cols_cap)
        for (int t = threadIdx.x; t < T; t += 256) a.col_b[c + t] = b;
    if (!last) return;
    const int64_t R = r + rb, C = c + cb;
    const bool fail = bad != 0 || (a.packed ? R != a.rows : R > a.rows) || C > a.cols_cap;
    // scattered column order (visit_col), only where a streaming grid walks more than one column per workgroup: the
    // first multiplier >= 0.618 C coprime with C, 64 candidates per pass with lane-parallel Euclid (any coprime
    // multiplier makes i -> i * m mod C a permutation)
    int64_t mul = 0;
    if (!fail && C > a.scatter_above && C >= 3 && C < (1ll << 31) && threadIdx.x < 64) {
        for (uint32_t base = max(2u, (uint32_t)(0.6180339887 * (double)C));; base += 64) {
            uint32_t x = base + threadIdx.x, y = (uint32_t)C;
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
    if (threadIdx.x == 0) {
        DynWords *d = a.dyn;
        d->status = fail ? (int)RNNT_STATUS_INVALID_VALUE : 0;
        d->num_cols = fail ? 0 : C;
        d->num_rows = fail ? 0 : R;
        d->col_mul = mul;
        d->steal = 0;
        if (fail && a.status_host)  // a plain system-scope store into the caller's host-mapped word
            __hip_atomic_store(a.status_host, (int)RNNT_STATUS_INVALID_VALUE, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (threadIdx.x < 64 && a.lp) {  // the recursion's reads just outside [0, N) (see setup_kernel)
        const int i = threadIdx.x;
        const int64_t end = fail ? 0 : R;
        a.lp[i - 64] = Lp{0.0, 0.0};
        a.lp[end + i] = Lp{0.0, 0.0};
    }
}

hipError_t launch_setup_dyn(const DynSetupArgs &a, hipStream_t stream) {
    setup_dyn_kernel<<<a.B, 256, 0, stream>>>(a);
    return hipGetLastError();
}

// ---- inspection (not on the hot path) ---------------------------------------------------------------------------
// mrnnt_read_denoms: den of every lattice row. Rows the forward reduced (in band, inside the alignment window) are
// copied; the others are reduced here from acts, one wave per row (the reference's reduce covers every row,
// reduce.h:79-139, and its getter returns them all).
template <class IO>
__global__ __launch_bounds__(256) void den_all_kernel(DevProblem p, float *__restrict__ out) {
    resolve_dyn(p);
    typedef typename IO::S Sc;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const Sc *__restrict__ acts = reinterpret_cast<const Sc *>(p.acts);
    for (int64_t c = blockIdx.x; c < p.num_cols; c += gridDim.x) {
        const int b = p.col_b[c];
        const int T = p.T[b], S = p.S[b];
        const int t = (int)(c - p.col_off[b]);
        const int64_t rowc = p.row_off[b] + (int64_t)t * (S + 1);
        const int64_t arow = acts_col_base(p, b, t, rowc);
        int lo = max(0, t - (T - S)), hi = min(t, S);
        align_window(p, c, t, lo, hi);
        for (int s = wave; s <= S; s += 4) {
            if (s >= lo && s <= hi) {
                if (lane == 0) out[rowc + s] = p.den[rowc + s];
                continue;
            }
            const Sc *__restrict__ z = acts + (arow + s) * (int64_t)p.V;
            float m = NEG_INF_F, sum = 0.0f;
            for (int v = lane; v < p.V; v += 64) {
                const float x = IO::to_f(z[v]);
                const float mn = fmaxf(m, x);
                const float mr = (mn == NEG_INF_F) ? 0.0f : mn;
                sum = sum * fast_exp2((m - mr) * kLog2e) + fast_exp2((x - mr) * kLog2e);
                m = mn;
            }
            wave_reduce_max_sum(m, sum);
            if (lane == 0) out[rowc + s] = (float)(-(double)m - log_row_sum(sum));
        }
    }
}

hipError_t launch_den_all(const DevProblem &p, int elem, float *den_out, hipStream_t stream) {
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(p.num_cols, 1 << 16));
    switch (elem) {
        case ELEM_F32: den_all_kernel<IoF32><<<grid, 256, 0, stream>>>(p, den_out); break;
        case ELEM_BF16: den_all_kernel<IoBF16><<<grid, 256, 0, stream>>>(p, den_out); break;
        case ELEM_F16: den_all_kernel<IoF16><<<grid, 256, 0, stream>>>(p, den_out); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// mrnnt_read_band: the band in the reference's [B, ld] layout; t >= T_b and unrestricted calls give (0, S_b)
__global__ __launch_bounds__(256) void band_read_kernel(DevProblem p, int *__restrict__ min_out,
                                                        int *__restrict__ max_out, int64_t ld) {
    if (!resolve_dyn(p)) return;
    for (int b = blockIdx.x; b < p.B; b += gridDim.x) {
        const int T = p.T[b], S = p.S[b];
        const int64_t c0 = p.col_off[b];
        for (int64_t t = threadIdx.x; t < ld; t += blockDim.x) {
            const bool in = p.min_s && t < T;
            if (min_out) min_out[(int64_t)b * ld + t] = in ? p.min_s[c0 + t] : 0;
            if (max_out) max_out[(int64_t)b * ld + t] = in ? p.max_s[c0 + t] : S;
        }
    }
}

hipError_t launch_band_read(const DevProblem &p, int *min_out, int *max_out, int64_t ld, hipStream_t stream) {
    band_read_kernel<<<std::max(1, std::min(p.B, 65535)), 256, 0, stream>>>(p, min_out, max_out, ld);
    return hipGetLastError();
}

}  // namespace mrnnt
