// mrnnt_setup.hip -- per-call metadata on the device (no host copies): lattice row/column offsets from the
// length arrays, the alignment band, plus the bench/test synthetic generator and the launch knobs.
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

// synthetic generator (bench / tests), bit-identical to mrnnt_oracle_synth_acts (oracle/rnnt_oracle.c):
// integer hashing + one exact int->float conversion and one multiply, nothing that rounds differently
// on the host.
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

// bandwidth probe: a device copy in the gradient pass's access pattern -- each workgroup streams its own
// contiguous slab of 16-byte elements, 4 loads in flight per lane, nontemporal loads and stores
__global__ __launch_bounds__(256) void copy_probe_kernel(const u4 *__restrict__ a, u4 *__restrict__ b, int64_t n,
                                                         int64_t slab) {
    for (int64_t c0 = (int64_t)blockIdx.x * slab; c0 < n; c0 += (int64_t)gridDim.x * slab) {
        const int64_t end = min(c0 + slab, n);
        for (int64_t i = c0 + threadIdx.x; i < end; i += 256 * 4) {
            u4 x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + 256 * u < end) x[u] = __builtin_nontemporal_load(&a[i + 256 * u]);
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + 256 * u < end) __builtin_nontemporal_store(x[u], &b[i + 256 * u]);
        }
    }
}

hipError_t launch_copy_probe(void *dst, const void *src, size_t bytes, hipStream_t stream) {
    const int64_t n = (int64_t)(bytes / 16);
    if (n <= 0) return hipSuccess;
    int dev = 0, cus = 256;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return e;
    // 32 workgroups per CU, each streaming >= 8 slabs in turn (a single pass of one slab per workgroup
    // measures the launch tail, not the memory); slabs of 16 KiB .. 800 KiB, whole 4 KiB workgroup steps
    const int64_t blocks_max = (int64_t)32 * cus;
    const int64_t slab = std::min<int64_t>(50 * 1024, std::max<int64_t>(1024, n / (blocks_max * 8) / 1024 * 1024));
    const int64_t blocks = std::min<int64_t>((n + slab - 1) / slab, blocks_max);
    copy_probe_kernel<<<(int)blocks, 256, 0, stream>>>(static_cast<const u4 *>(src), static_cast<u4 *>(dst), n, slab);
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
