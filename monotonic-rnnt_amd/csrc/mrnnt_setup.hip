// mrnnt_setup.hip -- per-call metadata on the device (no host copies): lattice row/column offsets from the
// length arrays, the alignment band, and the launch knobs.
#include "mrnnt_device.h"

namespace mrnnt {

Tuning &tuning() {
    static Tuning t;
    return t;
}

// row_off[b] = sum_{b'<b} T_b'(S_b'+1), col_off[b] = sum_{b'<b} T_b' -- one wave, any B (reference
// gpu_workspace_manager.h:256-329 computes these on the host and copies them with blocking memcpys).
// It also zeroes the 64 lp entries either side of the lp arrays: the recursion's in-band cell s = 0 of
// utterance 0 adds lpe[-1] to its -inf predecessor, and a NaN / +inf left in the (reused) workspace there
// would turn alpha(0, 0) into NaN (then -inf through fmax in the next LSE: an infinite cost).
__global__ __launch_bounds__(64) void setup_kernel(const int *__restrict__ T, const int *__restrict__ S, int B,
                                                   int64_t *__restrict__ row_off, int64_t *__restrict__ col_off,
                                                   double *__restrict__ lpb, double *__restrict__ lpe, int64_t n) {
    const int lane = threadIdx.x;
    int64_t carry_r = 0, carry_c = 0;
    if (lane == 0) {
        row_off[0] = 0;
        col_off[0] = 0;
    }
    if (lpb) {
        lpb[lane - 64] = 0.0;
        lpe[lane - 64] = 0.0;
        lpb[n + lane] = 0.0;
        lpe[n + lane] = 0.0;
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
                        double *lpb, double *lpe, int64_t n, hipStream_t stream) {
    setup_kernel<<<1, 64, 0, stream>>>(T, S, B, row_off, col_off, lpb, lpe, n);
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

hipError_t launch_mask_state(const DevProblem &p, double *alpha, double *beta, hipStream_t stream) {
    const int grid = (int)(p.num_cols < (1 << 16) ? p.num_cols : (1 << 16));
    mask_state_kernel<<<grid > 0 ? grid : 1, 64, 0, stream>>>(p, alpha, beta);
    return hipGetLastError();
}

}  // namespace mrnnt
