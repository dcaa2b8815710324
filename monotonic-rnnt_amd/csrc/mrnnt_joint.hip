// mrnnt_joint.hip -- the joint network fused into the loss ("fusing the joint network's
// final projection with the softmax pass so the N x V tensor is never materialised").
//
//   z(b,t,s,:) = W * tanh(enc[b,t,:] + pred[b,s,:]) + bias          (W: [V, H] bf16, fp32 accumulate)
//
// The packed logits the reference's loss takes as `acts` (monotonic_rnnt_op.py:133-140) are formed on MFMA
// (v_mfma_f32_32x32x16_bf16) tile by tile inside two passes and never written to HBM:
//   forward  : per in-band lattice row the log-softmax denominator and the blank / label log-probs (what
//              mrnnt_softmax.hip computes from stored acts), then the unchanged alpha/beta recursion;
//   backward : per LIVE row (the occupancy-skip predicate of mrnnt_grad.hip) the logit gradient
//              g = dL/dz (bf16) and the joint activation tanh(enc + pred) (bf16), so that dW = G^T Hact,
//              dH = G W and dbias = sum G are plain GEMMs / reductions over live rows only.
//
// Tiling: a workgroup of 8 waves (two per SIMD) owns 256 consecutive rows of a row list; a wave owns 32 rows and
// keeps their activations as the MFMA B operand in registers (lane l: row l&31, k = 16 ks + 8 (l>>5) + [0,8)),
// built once from enc/pred with a fast tanh. W streams through LDS in 32-vocabulary chunks (LDS-DMA, double-
// buffered, XOR-swizzled against bank conflicts) shared by the 8 waves; each chunk is one 32x32 output tile per wave,
// D[vocab][row] = sum_k W[vocab][k] h[row][k]: the accumulator holds 16 vocabulary entries of ONE row per
// lane (vocab = (i&3) + 8 (i>>2) + 4 (l>>5)), so the per-row online softmax is register-local and the two
// lane halves merge once at the end.
#include <algorithm>
#include <type_traits>
#include <utility>

#include "mrnnt_device.h"

namespace mrnnt {

#ifdef MRNNT_DEVTOOLS
// development build: the forward's per-wave timeline (s_memrealtime ticks) for every wave (8) of the first
// kJointTraceWgs workgroups, 8 marks each: start, bias staged, activations built, first chunk done, end, and inside
// chunk 0: after the DMA wait, after the barrier, after the MFMAs
constexpr int kJointTraceWgs = 4096;
__device__ unsigned long long g_joint_trace[kJointTraceWgs * 64];
// development build, joint_probe bit 4: the reduce's timeline -- thread 0 of the first kRedTraceWgs workgroups stamps
// [0] start, [1] setup done, [2 + 2f] frame f's rows summed, [3 + 2f] frame f's barriers passed (f < 6), [14] frame
// loop done, [15] flush done (s_memrealtime, 10 ns)
constexpr int kRedTraceWgs = 8192;
__device__ unsigned long long g_reduce_trace[kRedTraceWgs * 16];
#define JOINT_MARK(i)                                                                                         \
    do {                                                                                                      \
        if ((threadIdx.x & 63) == 0 && blockIdx.x < (unsigned)kJointTraceWgs && threadIdx.x < 512)            \
            g_joint_trace[blockIdx.x * 64 + (threadIdx.x >> 6) * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define JOINT_MARK(i) ((void)0)
#endif
#define FWD_MARK(i)                 \
    do {                            \
        if constexpr (TR) JOINT_MARK(i); \
    } while (0)

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f2 __attribute__((ext_vector_type(2)));

// scalar f32 in the MFMA loop's epilogue: a packed v_pk_fma/add_f32 beside MFMAs costs more issue time than the
// two scalar ops it replaces (MI355X_MICROARCH.md, per-instruction constants; the joint file is built with
// -fno-slp-vectorize so these stay scalar -- measured 2 % faster forward and backward than packed)
__device__ __forceinline__ f2 add2(f2 a, f2 b) { return (f2){a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ f2 mul2(f2 a, f2 b) { return (f2){a.x * b.x, a.y * b.y}; }
__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return (f2){fmaf(a.x, b.x, c.x), fmaf(a.y, b.y, c.y)}; }

__device__ __forceinline__ float bf16_lo(unsigned u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf16_hi(unsigned u) { return __uint_as_float(u & 0xffff0000u); }


// tanh(x) = sign(x) (1 - e) / (1 + e), e = exp(-2|x|) (v_exp_f32 + v_rcp_f32, |error| ~ 1e-7), two at a time on
// packed f32 (v_pk_*): the build runs before the MFMA loop, where packing halves its VALU. (The form
// 1 - 2 / (1 + e^{2x}) has 39 % fewer non-transcendental VALU and measured 0.1-0.2 ms slower at H = 512:
// profiles/r02/joint/joint_tanh_rcp_ab.json.)
__device__ __forceinline__ f2 fast_tanh2(f2 x) {
    const f2 ax = {fabsf(x.x), fabsf(x.y)};
    const f2 t = ax * (f2){-2.0f * kLog2e, -2.0f * kLog2e};
    const f2 e = {fast_exp2(t.x), fast_exp2(t.y)};
    const f2 num = (f2){1.0f, 1.0f} - e, den = (f2){1.0f, 1.0f} + e;
    const f2 y = num * (f2){__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
    return (f2){copysignf(y.x, x.x), copysignf(y.y, x.y)};
}

// ---------------------------------------------------------------------------------------------------------
// row lists: entries (column, s) in column order, s ascending; mode 0 = in-band rows, 1 = live rows

__device__ __forceinline__ bool list_pred(const DevProblem &p, int mode, int t, int s, int64_t row, int W,
                                          double ll) {
    if (mode == 0 || !p.occ_skip) return true;
    return row_live(alpha_prev(p, t, s, row, W) - ll + p.beta[row]);
}

template <bool WRITE>
__device__ __forceinline__ void row_list_column(const DevProblem &p, int mode, int64_t *__restrict__ cnt,
                                                int *__restrict__ lcol, int *__restrict__ ls, int64_t col, int lane) {
    const int b = p.col_b[col];
    const int T = p.T[b], S = p.S[b], W = S + 1;
    const int t = (int)(col - p.col_off[b]);
    const int64_t rowc = p.row_off[b] + (int64_t)t * W;
    int lo = max(0, t - (T - S)), hi = min(t, S);
    if (mode == 0) align_window(p, col, t, lo, hi);  // alignment-restricted: only the rows the recursion uses
    const double ll = mode ? p.ll[b] : 0.0;
    int64_t base = WRITE ? cnt[col] : 0;
    int n = 0;
    for (int s0 = lo; s0 <= hi; s0 += 64) {
        const int s = s0 + lane;
        const bool ok = s <= hi && list_pred(p, mode, t, s, rowc + s, W, ll);
        const unsigned long long mask = __ballot(ok);
        if (WRITE && ok) {
            const int rank = __popcll(mask & ((1ull << lane) - 1ull));
            lcol[base + rank] = (int)col;
            ls[base + rank] = s;
        }
        base += __popcll(mask);
        n += __popcll(mask);
    }
    if (!WRITE && lane == 0) cnt[col] = n;
}

template <bool WRITE>
__global__ __launch_bounds__(256) void row_list_kernel(DevProblem p, int mode, int64_t *__restrict__ cnt,
                                                       int *__restrict__ lcol, int *__restrict__ ls) {
    const int lane = threadIdx.x & 63;
    // grid-stride over lattice columns (one per wave): the grid is capped, any number of columns works
    for (int64_t col = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); col < p.num_cols; col += (int64_t)gridDim.x * 4)
        row_list_column<WRITE>(p, mode, cnt, lcol, ls, col, lane);
}

// exclusive scan of a[0..n) in place, a[n] = total (n = lattice columns), in two launches over tiles of 1024: the
// tile sums (one workgroup per tile), then every workgroup adds the sums of the tiles before its own (<= a few
// hundred, one wave) and scans its tile through LDS. (A single workgroup walking all columns took ~130 us per list
// at the headline's 64,000 columns.)
constexpr int kScanTile = 1024;

__device__ __forceinline__ int64_t block_incl_scan1024(int64_t v, int64_t *wsum) {  // 1024 threads
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    v = wave_incl_scan64(v);
    if (lane == 63) wsum[wave] = v;
    __syncthreads();
    if (wave == 0) {
        int64_t w = lane < 16 ? wsum[lane] : 0;
        w = wave_incl_scan64(w);
        if (lane < 16) wsum[lane] = w;
    }
    __syncthreads();
    return v + (wave > 0 ? wsum[wave - 1] : 0);
}

__global__ __launch_bounds__(1024) void scan_tiles_kernel(const int64_t *__restrict__ a, int64_t n,
                                                          int64_t *__restrict__ tile_sum) {
    __shared__ int64_t wsum[16];
    const int64_t i = (int64_t)blockIdx.x * kScanTile + threadIdx.x;
    const int64_t v = block_incl_scan1024(i < n ? a[i] : 0, wsum);
    if (threadIdx.x == kScanTile - 1) tile_sum[blockIdx.x] = v;
}

__global__ __launch_bounds__(1024) void scan_apply_kernel(int64_t *__restrict__ a, int64_t n,
                                                          const int64_t *__restrict__ tile_sum,
                                                          unsigned long long *__restrict__ total) {
    __shared__ int64_t wsum[16];
    __shared__ int64_t base;
    if (threadIdx.x < 64) {  // the tiles before this one, in order
        int64_t s = 0;
        for (int k = threadIdx.x; k < (int)blockIdx.x; k += 64) s += tile_sum[k];
        s = wave_incl_scan64(s);
        if (threadIdx.x == 63) base = s;
    }
    const int64_t i = (int64_t)blockIdx.x * kScanTile + threadIdx.x;
    const int64_t x = i < n ? a[i] : 0;
    const int64_t incl = block_incl_scan1024(x, wsum);  // (its barriers also publish `base`)
    if (i < n) a[i] = base + incl - x;
    if (i == n - 1 || (n == 0 && i == 0)) {
        a[n] = base + incl;
        if (total) *total = (unsigned long long)(base + incl);
    }
}

hipError_t launch_row_list(const DevProblem &p, int mode, int64_t *col_cnt, int *lcol, int *ls,
                           unsigned long long *total, hipStream_t stream) {
    const int64_t blocks = std::min<int64_t>((p.num_cols + 3) / 4, 1 << 20);
    row_list_kernel<false><<<(int)blocks, 256, 0, stream>>>(p, mode, col_cnt, lcol, ls);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    // the tile sums live past the counts (the workspace sizes col_cnt for it: joint_scan_scratch)
    const int64_t tiles = std::max<int64_t>(1, (p.num_cols + kScanTile - 1) / kScanTile);
    if (tiles > (1 << 20)) return hipErrorInvalidValue;
    int64_t *tile_sum = col_cnt + p.num_cols + 1;
    scan_tiles_kernel<<<(unsigned)tiles, 1024, 0, stream>>>(col_cnt, p.num_cols, tile_sum);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    scan_apply_kernel<<<(unsigned)tiles, 1024, 0, stream>>>(col_cnt, p.num_cols, tile_sum, total);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    row_list_kernel<true><<<(int)blocks, 256, 0, stream>>>(p, mode, col_cnt, lcol, ls);
    return hipGetLastError();
}

hipError_t launch_zero(void *ptr, size_t bytes, hipStream_t stream) { return hipMemsetAsync(ptr, 0, bytes, stream); }

// ---------------------------------------------------------------------------------------------------------
// the fused tile

struct RowPos {
    bool valid;
    int b, t, s, T, S, lab;
    int64_t row;  // packed lattice row
};

__device__ __forceinline__ int64_t list_len(const JointArgs &j) {
    return j.n_dev ? (int64_t)*j.n_dev : j.n;
}

__device__ __forceinline__ RowPos row_pos(const DevProblem &p, const JointArgs &j, int64_t i) {
    RowPos q{false, 0, 0, 0, 1, 0, -1, 0};
    if (i >= list_len(j)) return q;
    const int col = j.lcol[i];
    q.s = j.ls[i];
    q.b = p.col_b[col];
    q.t = (int)(col - p.col_off[q.b]);
    q.T = p.T[q.b];
    q.S = p.S[q.b];
    q.row = p.row_off[q.b] + (int64_t)q.t * (q.S + 1) + q.s;
    // -2: a label outside [0, V) (device labels are not range-checked on the host): no capture, lpe = NaN
    const int l = q.s < q.S ? p.labels[(int64_t)q.b * p.label_stride + q.s] : -1;
    q.lab = (q.s < q.S && (unsigned)l >= (unsigned)p.V) ? -2 : l;
    q.valid = true;
    return q;
}

// B operand of one row: h = bf16(tanh(enc[b,t] + pred[b,s])) for k = k0 + KSTEP ks + [0, 8), ks < NK; optionally
// stored to Hact. Invalid lanes (past the end of the list) read row 0 and zero the result: no branch around the loads
// (a branch per load makes hipcc wait vmcnt(0) after each one).
template <int NK, int KSTEP, bool STORE>
__device__ __forceinline__ void build_row(const JointArgs &j, const RowPos &q, int k0, int64_t i, bf16x8 *bfr) {
    constexpr int H = NK * KSTEP;
    const bool v = q.valid;
    const int t_ld = (kVariants && (j.probe & 2)) ? 0 : q.t, s_ld = (kVariants && (j.probe & 1)) ? 0 : q.s;
    const unsigned short *er = j.enc + (v ? (int64_t)q.b * j.enc_sb + (int64_t)t_ld * H : 0) + k0;
    const unsigned short *pr = j.pred + (v ? (int64_t)q.b * j.pred_sb + (int64_t)s_ld * H : 0) + k0;
    const float keep = v ? 1.0f : 0.0f;
#pragma unroll
    for (int ks = 0; ks < NK; ++ks) {
        const u4 ev = *reinterpret_cast<const u4 *>(er + KSTEP * ks);
        const u4 pv = *reinterpret_cast<const u4 *>(pr + KSTEP * ks);
        bf16x8 h;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const f2 y = fast_tanh2((f2){bf16_lo(ev[w]), bf16_hi(ev[w])} + (f2){bf16_lo(pv[w]), bf16_hi(pv[w])}) *
                         (f2){keep, keep};
            h[2 * w] = (__bf16)y.x;
            h[2 * w + 1] = (__bf16)y.y;
        }
        if (STORE && v) *reinterpret_cast<bf16x8 *>(j.Hact + i * j.hact_ld + KSTEP * ks + k0) = h;
        bfr[ks] = h;
    }
    if (STORE && v) {  // columns past H: a ones column (dbias from the dweight GEMM), then zeros
        for (int64_t c = H + k0; c < j.hact_ld; c += KSTEP) {
            bf16x8 e = {};
            if (c == H) e[0] = (__bf16)1.0f;
            *reinterpret_cast<bf16x8 *>(j.Hact + i * j.hact_ld + c) = e;
        }
    }
}

// 32x32x16 tile: lane l holds k = 16 ks + 8 (l >> 5) + [0, 8) of row l & 31
template <int KS, bool STORE>
__device__ __forceinline__ void build_act(const JointArgs &j, const RowPos &q, int half, int64_t i,
                                          bf16x8 (&bfr)[KS]) {
    build_row<KS, 16, STORE>(j, q, 8 * half, i, bfr);
}

// W chunk (32 vocabulary rows x H bf16) in LDS: unpadded, the 16-byte piece p of row r stored at piece
// p ^ (r & 15) (T2 XOR swizzle: the 16 lanes of a ds_read_b128 group read 16 distinct rows at one column and
// land on 16 distinct bank quads). Filled by LDS-DMA (global_load_lds_dwordx4: 1 KiB per wave-instruction,
// lane-linear destination, so the swizzle goes on the per-lane SOURCE address) -- no staging registers.
template <int KS>
struct WTile {
    static constexpr int H = 16 * KS;
    static constexpr int CPR = H / 8;    // 16-byte pieces per row (a multiple of 16 for H % 128 == 0)
    static constexpr int NI = CPR / 2;   // wave-instructions per tile: 32 * CPR / 64
    static constexpr int ELEMS = 32 * H; // bf16 elements per tile

    // issue the DMA of vocabulary chunk c into wbuf (rows >= V read row V-1; the epilogue masks them); the NW
    // waves of the workgroup split the NI wave-instructions
    template <int NW>
    __device__ static __forceinline__ void stage(const JointArgs &j, int V, int c, unsigned short *wbuf) {
        static_assert(NI % NW == 0, "DMA instructions must split evenly over the waves");
        const int lane = threadIdx.x & 63;
        const int wave = (!kVariants || (j.opt & 1)) ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : threadIdx.x >> 6;
        if ((!kVariants || (j.opt & 1)) && 32 * c + 32 <= V) {
            // a whole chunk: a wave-uniform chunk base plus loop-invariant 32-bit lane offsets (no per-chunk 64-bit
            // address arithmetic or row clamp on the vector pipe; the last partial chunk takes the clamped form)
            const char *base = reinterpret_cast<const char *>(j.W + (int64_t)32 * c * H);
#pragma unroll
            for (int ii = 0; ii < NI / NW; ++ii) {
                const int i = NW * ii + wave;
                const int L = 64 * i + lane;
                const int r = L / CPR, pc = L % CPR;
                const unsigned off = (unsigned)(r * H + 8 * (pc ^ (r & 15))) * 2u;
                __builtin_amdgcn_global_load_lds(base + off, (__attribute__((address_space(3))) void *)(wbuf + 512 * i),
                                                 16, 0, 0);
            }
            return;
        }
#pragma unroll
        for (int ii = 0; ii < NI / NW; ++ii) {
            const int i = NW * ii + wave;
            const int L = 64 * i + lane;
            const int r = L / CPR, pc = L % CPR;
            const int v = min(32 * c + r, V - 1);
            const unsigned short *g = j.W + (int64_t)v * H + 8 * (pc ^ (r & 15));
            __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void *)(wbuf + 512 * i), 16, 0, 0);
        }
    }

    // one 32x32 output tile: D[vocab][row] = sum_k W[vocab][k] h[row][k]; A fragments stream from LDS
    // through a 4-deep register ring so no MFMA waits on a ds_read it has just issued. The swizzled piece of
    // k-step ks = 8m + k' is 16m + ((2k' + half) ^ (r & 15)): 8 base addresses, m in the immediate offset.
    template <int RING = 4>
    __device__ static __forceinline__ f32x16 mma(const unsigned short *wbuf, const bf16x8 (&bfr)[KS], int lane) {
        const int r = lane & 31, half = lane >> 5;
        const unsigned short *row = wbuf + r * H;
        const unsigned short *base[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) base[k] = row + 8 * ((2 * k + half) ^ (r & 15));
        auto rd = [&](int ks) { return *reinterpret_cast<const bf16x8 *>(base[ks & 7] + 128 * (ks >> 3)); };
        constexpr int D = KS < RING ? KS : RING;
        bf16x8 a[D];
#pragma unroll
        for (int d = 0; d < D; ++d) a[d] = rd(d);
        f32x16 acc;
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ks % D], bfr[ks], acc, 0, 0, 0);
            if (ks + D < KS) a[ks % D] = rd(ks + D);
        }
        return acc;
    }
};

// The same W chunk as four 16x16 output tiles per wave (v_mfma_f32_16x16x32_bf16: at equal cycles per FLOP the
// 16x16 shape holds a higher clock than 32x32 on random operands, MI355X_MICROARCH.md 'DVFS give-back' item 7).
// A wave's 32 rows are two row tiles rt (rows 16 rt + (l & 15)); lane l holds k = 32 kk + 8 (l >> 4) + [0, 8) of
// both rows (B), and of W row 16 vt + (l & 15) (A: one ds_read_b128 feeds the MFMAs of both row tiles). Output
// d[vt][rt][r] = z(row 16 rt + (l & 15), vocab 32 c + 16 vt + 4 (l >> 4) + r).
template <int KS>
struct WTile16 {
    static constexpr int H = 16 * KS;
    static constexpr int K32 = KS / 2;  // MFMA k-steps
    struct Acc {
        f4 d[2][2];
    };

    // piece 4 kk + g of row 16 vt + c16 sits at (4 kk + g) ^ c16 (the WTile swizzle, c16 = row & 15): with
    // kk = 4 m + kk', that is 16 m + ((4 kk' + g) ^ c16): four base addresses, m and vt in the immediate offset
    template <int RING = 4>
    __device__ static __forceinline__ Acc mma(const unsigned short *wbuf, const bf16x8 (&bfr)[2][K32], int lane) {
        const int c16 = lane & 15, g = lane >> 4;
        const unsigned short *row = wbuf + c16 * H;
        const unsigned short *base[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) base[k] = row + 8 * ((4 * k + g) ^ c16);
        constexpr int NR = 2 * K32;  // A fragments per chunk, in (kk, vt) order
        auto rd = [&](int n) {
            const int kk = n >> 1, vt = n & 1;
            return *reinterpret_cast<const bf16x8 *>(base[kk & 3] + 128 * (kk >> 2) + 16 * H * vt);
        };
        constexpr int D = NR < RING ? NR : RING;
        bf16x8 a[D];
#pragma unroll
        for (int d = 0; d < D; ++d) a[d] = rd(d);
        Acc acc;
#pragma unroll
        for (int vt = 0; vt < 2; ++vt)
#pragma unroll
            for (int rt = 0; rt < 2; ++rt) acc.d[vt][rt] = (f4){0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int n = 0; n < NR; ++n) {
            const int kk = n >> 1, vt = n & 1;
            acc.d[vt][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[n % D], bfr[0][kk], acc.d[vt][0], 0, 0, 0);
            acc.d[vt][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[n % D], bfr[1][kk], acc.d[vt][1], 0, 0, 0);
            if (n + D < NR) a[n % D] = rd(n + D);
        }
        return acc;
    }
};

__device__ __forceinline__ void wait_dma() { wait_vmcnt0(); }

// wait until at most N vector-memory operations of this wave are outstanding (in-order completion): the
// DMA of the chunk after next stays in flight across the barrier
template <int N>
__device__ __forceinline__ void wait_dma_leave() {
    static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// index of the accumulator register holding vocabulary offset jj (0..31) of a chunk, or -1 if the other lane
// half holds it
__device__ __forceinline__ int acc_reg_of(int jj, int half) {
    return (((jj >> 2) & 1) == half) ? ((jj & 3) + 4 * (jj >> 3)) : -1;
}

// x[i] for a per-lane runtime i in [0, 16): a 4-level tree of bit selects (v_bfi_b32 on the bit masks of i;
// plain ternaries over arrays get rewritten into a scratch-indexed load)
__device__ __forceinline__ unsigned bsel(unsigned m, float a, float b) {  // m ? b : a, m all-ones or zero
    return (__float_as_uint(a) & ~m) | (__float_as_uint(b) & m);
}
__device__ __forceinline__ float tree_pick(const f2 (&x)[8], int i) {
    const unsigned m0 = 0u - (unsigned)(i & 1), m1 = 0u - (unsigned)((i >> 1) & 1);
    const unsigned m2 = 0u - (unsigned)((i >> 2) & 1), m3 = 0u - (unsigned)((i >> 3) & 1);
    const float a0 = __uint_as_float(bsel(m0, x[0].x, x[0].y)), a1 = __uint_as_float(bsel(m0, x[1].x, x[1].y));
    const float a2 = __uint_as_float(bsel(m0, x[2].x, x[2].y)), a3 = __uint_as_float(bsel(m0, x[3].x, x[3].y));
    const float a4 = __uint_as_float(bsel(m0, x[4].x, x[4].y)), a5 = __uint_as_float(bsel(m0, x[5].x, x[5].y));
    const float a6 = __uint_as_float(bsel(m0, x[6].x, x[6].y)), a7 = __uint_as_float(bsel(m0, x[7].x, x[7].y));
    const float b0 = __uint_as_float(bsel(m1, a0, a1)), b1 = __uint_as_float(bsel(m1, a2, a3));
    const float b2 = __uint_as_float(bsel(m1, a4, a5)), b3 = __uint_as_float(bsel(m1, a6, a7));
    const float c0 = __uint_as_float(bsel(m2, b0, b1)), c1 = __uint_as_float(bsel(m2, b2, b3));
    return __uint_as_float(bsel(m3, c0, c1));
}

// z = acc + bias as 8 packed pairs (pair k = registers 2k, 2k+1: vocabulary 32c + (2k&3) + 8(k>>1) + 4 half + {0,1});
// entries past V come out -inf through the padded bias
__device__ __forceinline__ void logits2(const f32x16 &acc, const float *bias_lds, int c, int half, f2 (&z)[8]) {
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
        const f4 bv = *reinterpret_cast<const f4 *>(bias_lds + 32 * c + 8 * q4 + 4 * half);
        z[2 * q4] = add2((f2){acc[4 * q4], acc[4 * q4 + 1]}, (f2){bv.x, bv.y});
        z[2 * q4 + 1] = add2((f2){acc[4 * q4 + 2], acc[4 * q4 + 3]}, (f2){bv.z, bv.w});
    }
}

__device__ __forceinline__ float max3(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// Chunk loop: a workgroup of NW waves (NW = 8: two waves per SIMD, 256 rows) shares each W chunk; NB LDS buffers
// keep NB - 1 chunk DMAs in flight; one raw s_barrier per chunk. `S` = vector stores the epilogue issues per chunk
// on every wave (0 forward, 4 backward; -1 = unknown): the wait before chunk c leaves the later DMAs and the
// stores of the epilogues issued after chunk c's DMA in flight (vector memory completes in issue order).
// (Staggering the two waves of a SIMD by one epilogue, and three buffers, both measured slower: registers.)
// TRACE: stamp chunk 0 into the development build's forward timeline (the forward only: the backward kernels share
// this loop and would overwrite the same slots).
template <int KS, int NB, int NW, bool TRACE = false, class Mma, class Epi>
__device__ __forceinline__ void chunk_loop_with(const JointArgs &j, int V, unsigned short *wsh, int S, Mma &&mma,
                                                Epi &&epi) {
    using WT = WTile<KS>;
    constexpr int NPW = WT::NI / NW;  // DMA instructions per wave per chunk
    const int nch = (V + 31) / 32;
#pragma unroll
    for (int c = 0; c < NB - 1; ++c)
        if (c < nch) WT::template stage<NW>(j, V, c, wsh + c * WT::ELEMS);
    for (int c = 0; c < nch; ++c) {
        // chunk c in LDS for every wave
        if (c + NB - 2 < nch && S >= 0) {
            const int older = min(c, NB - 1);  // epilogues issued after chunk c's DMA
            if (S == 0 || older == 0) wait_dma_leave<(NB - 2) * NPW>();
            else if (older == 1) wait_dma_leave<(NB - 2) * NPW + 4>();
            else wait_dma_leave<(NB - 2) * NPW + 8>();  // NB == 3
        } else {
            wait_dma();
        }
        if (TRACE && c == 0) JOINT_MARK(5);
        __builtin_amdgcn_s_barrier();
        if (TRACE && c == 0) JOINT_MARK(6);
        if (c + NB - 1 < nch) WT::template stage<NW>(j, V, c + NB - 1, wsh + ((c + NB - 1) % NB) * WT::ELEMS);
        const auto acc = mma(wsh + (c % NB) * WT::ELEMS);
        if (TRACE && c == 0) JOINT_MARK(7);
        epi(acc, c);
    }
}

template <int KS, int NB, int NW, int RG, bool TRACE = false, class Epi>
__device__ __forceinline__ void chunk_loop(const JointArgs &j, int V, unsigned short *wsh, const bf16x8 (&bfr)[KS],
                                           int lane, int S, Epi &&epi) {
    chunk_loop_with<KS, NB, NW, TRACE>(j, V, wsh, S,
                                [&](const unsigned short *wb) { return WTile<KS>::template mma<RG>(wb, bfr, lane); },
                                epi);
}

// LDS: NB W tiles, then the bias padded to whole chunks
template <int KS, int NB>
__device__ __forceinline__ float *load_bias(const JointArgs &j, int V, unsigned short *wsh, bool scaled = false) {
    float *bl = reinterpret_cast<float *>(wsh + NB * WTile<KS>::ELEMS);
    const int nb = (V + 31) / 32 * 32;
    // past V: -inf, so z = acc + bias masks the tail chunk without a compare (the clamped W rows are finite);
    // scaled (the forward): a second row, bias * log2 e, right after it
    for (int v = threadIdx.x; v < nb; v += blockDim.x) {
        const float b = v < V ? (j.bias ? j.bias[v] : 0.0f) : NEG_INF_F;
        bl[v] = b;
        if (scaled) bl[nb + v] = b * kLog2e;
    }
    return bl;
}

// two waves per SIMD: the compiler keeps each kernel within 256 registers per lane
// TR: the development build's timeline stamps (JOINT_MARK), instantiated only when the joint_trace knob asks for them:
// the stamps (a scalar clock read and a store per mark, one inside the chunk loop) cost that build's forward ~15 %
template <int KS, int NB, int NW, int RG, bool TR = false>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(2, 2))) void joint_fwd_kernel(DevProblem p,
                                                                                             JointArgs j) {
    extern __shared__ __attribute__((aligned(16))) unsigned short wsh[];
    if ((int64_t)blockIdx.x * (32 * NW) >= list_len(j)) return;  // whole workgroup past a shorter list
    FWD_MARK(0);
    const int lane = threadIdx.x & 63, half = lane >> 5;
    const int64_t i = (int64_t)blockIdx.x * (32 * NW) + (threadIdx.x >> 6) * 32 + (lane & 31);
    const RowPos q = row_pos(p, j, i);
    const int V = p.V, blank = p.blank;
    const float *bias = load_bias<KS, NB>(j, V, wsh, (j.opt & 2) != 0);
    __syncthreads();
    FWD_MARK(1);
    bf16x8 bfr[KS];
    build_act<KS, false>(j, q, half, i, bfr);
    FWD_MARK(2);

    const f2 l2e = {kLog2e, kLog2e};
    float m = NEG_INF_F, sum = 0.0f, zb = 0.0f, ze = 0.0f;
    bool fb = false, fe = false;
    // the blank / label logits of this lane's half of chunk c (the same selects in both epilogues)
    auto capture = [&](const f2 (&z)[8], int c) {
        const int jb = blank - 32 * c;  // wave-uniform: one chunk holds the blank
        if (jb >= 0 && jb < 32) {
            const int rb = acc_reg_of(jb, half);
            if (rb >= 0) {
                zb = tree_pick(z, rb);
                fb = true;
            }
        }
        const int jl = q.lab - 32 * c;
        const int rl = acc_reg_of(jl & 31, half);
        const bool mine = q.lab >= 0 && jl >= 0 && jl < 32 && rl >= 0;
        if (__ballot(mine)) {  // most chunks hold some lane's label; skip the select when none does
            const float x = tree_pick(z, rl);
            if (mine) {
                ze = x;
                fe = true;
            }
        }
    };
    // Bounded weights (j.wplain: |z| <= 64 for every logit, joint_wbound_kernel): a plain exp-sum -- 1024 terms of
    // at most e^64 cannot overflow fp32 and the largest cannot underflow -- without the running max, whose
    // per-chunk max / rescale chain cost 15 % of the forward. Otherwise the online log-sum-exp.
    const bool plain = j.wplain != nullptr && *j.wplain != 0;
    if (plain && (j.opt & 2)) {
        // exp2(fma(acc, log2 e, bias log2 e)) from a prescaled bias row (bias2, after the bias row in LDS): one fma per
        // logit where the bias add and the log2 e multiply were two; the captured blank / label logits are still
        // acc + bias (picked from the accumulator, the bias added to the picked value: the same fp32 add)
        const float *bias2 = bias + (V + 31) / 32 * 32;
        chunk_loop<KS, NB, NW, RG, TR>(j, V, wsh, bfr, lane, 0, [&](const f32x16 &acc, int c) {
            f2 s2 = {0.0f, 0.0f};
            f2 a2[8];
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
                const f4 bv = *reinterpret_cast<const f4 *>(bias2 + 32 * c + 8 * q4 + 4 * half);
                a2[2 * q4] = (f2){acc[4 * q4], acc[4 * q4 + 1]};
                a2[2 * q4 + 1] = (f2){acc[4 * q4 + 2], acc[4 * q4 + 3]};
                const f2 t0 = fma2(a2[2 * q4], l2e, (f2){bv.x, bv.y});
                const f2 t1 = fma2(a2[2 * q4 + 1], l2e, (f2){bv.z, bv.w});
                s2 = add2(s2, (f2){fast_exp2(t0.x), fast_exp2(t0.y)});
                s2 = add2(s2, (f2){fast_exp2(t1.x), fast_exp2(t1.y)});
            }
            sum += s2.x + s2.y;
            const int jb = blank - 32 * c;
            if (jb >= 0 && jb < 32) {
                const int rb = acc_reg_of(jb, half);
                if (rb >= 0) {
                    zb = tree_pick(a2, rb) + bias[32 * c + jb];
                    fb = true;
                }
            }
            const int jl = q.lab - 32 * c;
            const int rl = acc_reg_of(jl & 31, half);
            const bool mine = q.lab >= 0 && jl >= 0 && jl < 32 && rl >= 0;
            if (__ballot(mine)) {
                const float x = tree_pick(a2, rl) + bias[32 * c + (jl & 31)];
                if (mine) {
                    ze = x;
                    fe = true;
                }
            }
            if (c == 0) FWD_MARK(3);
        });
    } else if (plain) {
        chunk_loop<KS, NB, NW, RG, TR>(j, V, wsh, bfr, lane, 0, [&](const f32x16 &acc, int c) {
            f2 z[8];
            logits2(acc, bias, c, half, z);
            f2 s2 = {0.0f, 0.0f};
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const f2 t = mul2(z[k], l2e);
                s2 = add2(s2, (f2){fast_exp2(t.x), fast_exp2(t.y)});
            }
            sum += s2.x + s2.y;
            capture(z, c);
            if (c == 0) FWD_MARK(3);
        });
    }
    if (plain) {
        sum += __shfl_xor(sum, 32);
        const float zb2 = __shfl_xor(zb, 32), ze2 = __shfl_xor(ze, 32);
        const int fb2 = __shfl_xor((int)fb, 32), fe2 = __shfl_xor((int)fe, 32);
        if (!fb && fb2) zb = zb2;
        if (!fe && fe2) ze = ze2;
        if (q.valid && half == 0) {
            const double den = -log_row_sum(sum);
            p.den[q.row] = (float)den;
            p.lp[q.row] = Lp{(double)zb + den, (q.lab >= 0 ? (double)ze : (q.lab == -2 ? __builtin_nan("") : 0.0)) + den};
        }
        FWD_MARK(4);
        return;
    }
    chunk_loop<KS, NB, NW, RG, TR>(j, V, wsh, bfr, lane, 0, [&](const f32x16 &acc, int c) {
        f2 z[8];
        logits2(acc, bias, c, half, z);
        float cm = fmaxf(z[0].x, z[0].y);
#pragma unroll
        for (int k = 1; k < 8; ++k) cm = max3(cm, z[k].x, z[k].y);
        const float mn = fmaxf(m, cm);
        const float mr = (mn == NEG_INF_F) ? 0.0f : mn;
        const f2 nb = {-mr * kLog2e, -mr * kLog2e};
        f2 s2 = {0.0f, 0.0f};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const f2 t = fma2(z[k], l2e, nb);
            s2 = add2(s2, (f2){fast_exp2(t.x), fast_exp2(t.y)});
        }
        sum = sum * fast_exp2((m - mr) * kLog2e) + (s2.x + s2.y);
        m = mn;
        capture(z, c);
        if (c == 0) FWD_MARK(3);
    });
    // merge the two lane halves (same row, disjoint vocabulary)
    const float m2 = __shfl_xor(m, 32), s2 = __shfl_xor(sum, 32);
    const float zb2 = __shfl_xor(zb, 32), ze2 = __shfl_xor(ze, 32);
    const int fb2 = __shfl_xor((int)fb, 32), fe2 = __shfl_xor((int)fe, 32);
    const float mn = fmaxf(m, m2);
    const float mr = (mn == NEG_INF_F) ? 0.0f : mn;
    sum = sum * fast_exp2((m - mr) * kLog2e) + s2 * fast_exp2((m2 - mr) * kLog2e);
    if (!fb && fb2) zb = zb2;
    if (!fe && fe2) ze = ze2;
    if (q.valid && half == 0) {
        const double den = -(double)mn - log_row_sum(sum);
        p.den[q.row] = (float)den;
        p.lp[q.row] = Lp{(double)zb + den, (q.lab >= 0 ? (double)ze : (q.lab == -2 ? __builtin_nan("") : 0.0)) + den};
    }
    FWD_MARK(4);
}

#ifdef MRNNT_DEVTOOLS
int joint_reduce_trace(unsigned long long *out, int n) {
    n = std::min(n, kRedTraceWgs * 16);
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_reduce_trace), sizeof(unsigned long long) * n) != hipSuccess) return -1;
    return n;
}

int joint_trace(unsigned long long *out, int n) {
    n = std::min(n, kJointTraceWgs * 64);
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_joint_trace), sizeof(unsigned long long) * n) != hipSuccess) return -1;
    return n;
}
#endif

template <int KS, int NB, int NW, int RG>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(2, 2))) void joint_bwd_kernel(DevProblem p,
                                                                                             JointArgs j) {
    extern __shared__ __attribute__((aligned(16))) unsigned short wsh[];
    if (j.n_dev && (int64_t)blockIdx.x * (32 * NW) >= list_len(j)) return;  // past the device count (tail zeroed)
    const int lane = threadIdx.x & 63, half = lane >> 5;
    const int64_t i = (int64_t)blockIdx.x * (32 * NW) + (threadIdx.x >> 6) * 32 + (lane & 31);
    const RowPos q = row_pos(p, j, i);
    RowCoef rc{0.0f, 0.0f, 0.0f, -1, false};
    float sc = 0.0f;
    if (q.valid) {
        rc = row_coef(p, q.t, q.T, q.S, q.s, q.row, p.ll[q.b], p.labels + (int64_t)q.b * p.label_stride);
        sc = j.scale ? j.scale[q.b] : 1.0f;
        if (half == 0 && j.bt_idx) j.bt_idx[i] = (int64_t)q.b * (j.enc_sb / j.H) + q.t;
        if (half == 0 && j.bs_idx) j.bs_idx[i] = (int64_t)q.b * (j.pred_sb / j.H) + q.s;
    }
    const int V = p.V, blank = p.blank;
    const float *bias = load_bias<KS, NB>(j, V, wsh);
    __syncthreads();
    bf16x8 bfr[KS];
    build_act<KS, true>(j, q, half, i, bfr);

    // exactly 4 vector stores per chunk on every wave with a valid lane: leave them in flight at the barrier
    const bool vec_out = (V & 3) == 0;
    const bool leave = vec_out && __ballot(!q.valid) == 0;
    unsigned short *grow = j.G + (q.valid ? i : 0) * V;
    const f2 l2e = {kLog2e, kLog2e}, c2 = {rc.c2, rc.c2}, sc2 = {sc, sc};
    chunk_loop<KS, NB, NW, RG>(j, V, wsh, bfr, lane, leave ? 4 : -1, [&](const f32x16 &acc, int c) {
        f2 g[8];
        logits2(acc, bias, c, half, g);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const f2 t = fma2(g[k], l2e, c2);
            g[k] = (f2){fast_exp2(t.x), fast_exp2(t.y)};
        }
        // the <= 2 corrected entries of the row are rewritten by a second (2-byte) store after the vector store
        const int jb = blank - 32 * c;
        const int rb = (jb >= 0 && jb < 32) ? acc_reg_of(jb, half) : -1;
        const int jl = rc.lab - 32 * c;
        const int rl = acc_reg_of(jl & 31, half);
        const bool mine = rc.lab >= 0 && jl >= 0 && jl < 32 && rl >= 0;
        float gb = 0.0f, gl = 0.0f;
        if (rb >= 0) gb = tree_pick(g, rb);
        if (__ballot(mine)) gl = tree_pick(g, rl);
#pragma unroll
        for (int k = 0; k < 8; ++k) g[k] = mul2(g[k], sc2);
        if (q.valid) {
#pragma unroll
            for (int qd = 0; qd < 4; ++qd) {
                const int v0 = 32 * c + 8 * qd + 4 * half;
                if (vec_out && v0 + 3 < V) {
                    const unsigned lo = IoBF16::pack2(g[2 * qd].x, g[2 * qd].y);
                    const unsigned hi = IoBF16::pack2(g[2 * qd + 1].x, g[2 * qd + 1].y);
                    *reinterpret_cast<uint2 *>(grow + v0) = make_uint2(lo, hi);
                } else {
                    const float e4[4] = {g[2 * qd].x, g[2 * qd].y, g[2 * qd + 1].x, g[2 * qd + 1].y};
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (v0 + e < V) grow[v0 + e] = IoBF16::from_f(e4[e]);
                }
            }
            if (rb >= 0) grow[blank] = IoBF16::from_f((gb - rc.cb) * sc);
            if (mine) grow[rc.lab] = IoBF16::from_f((gl - rc.ce) * sc);
        }
    });
}

// ---------------------------------------------------------------------------------------------------------
// the same passes on the 16x16x32 tile (WTile16): each lane carries two rows (row tiles rt = 0, 1) and 8 of the
// chunk's 32 vocabulary entries of each; the four lane groups g = l >> 4 hold disjoint vocabulary and merge once.

// x[i] for a per-lane i in [0, 8): a 3-level select tree (v_cndmask; never an indexed register array)
__device__ __forceinline__ float pick8(const float (&x)[8], int i) {
    const bool b0 = i & 1, b1 = i & 2, b2 = i & 4;
    const float a0 = b0 ? x[1] : x[0], a1 = b0 ? x[3] : x[2], a2 = b0 ? x[5] : x[4], a3 = b0 ? x[7] : x[6];
    const float c0 = b1 ? a1 : a0, c1 = b1 ? a3 : a2;
    return b2 ? c1 : c0;
}

// vocabulary offset jj (0..31) of a chunk: held by lane group (jj >> 2) & 3 at index 4 (jj >> 4) + (jj & 3)
__device__ __forceinline__ int pick8_index(int jj) { return 4 * (jj >> 4) + (jj & 3); }

// z = acc + bias for row tile rt: x[4 vt + r] = vocabulary 32 c + 16 vt + 4 g + r (past V: -inf through the bias)
template <int KS>
__device__ __forceinline__ void logits8(const typename WTile16<KS>::Acc &acc, const f4 (&bv)[2], int rt,
                                        float (&x)[8]) {
#pragma unroll
    for (int vt = 0; vt < 2; ++vt)
#pragma unroll
        for (int r = 0; r < 4; ++r) x[4 * vt + r] = acc.d[vt][rt][r] + bv[vt][r];
}

template <int KS, int NB, int NW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(2, 2))) void joint_bwd16_kernel(
    DevProblem p, JointArgs j) {
    extern __shared__ __attribute__((aligned(16))) unsigned short wsh[];
    constexpr int K32 = KS / 2;
    if (j.n_dev && (int64_t)blockIdx.x * (32 * NW) >= list_len(j)) {  // past the device count: only its dbias row
        if (j.dbias)
            for (int v = threadIdx.x; v < (p.V + 31) / 32 * 32; v += blockDim.x)
                j.dbias_part[(int64_t)blockIdx.x * ((p.V + 31) / 32 * 32) + v] = 0.0f;
        return;
    }
    const int lane = threadIdx.x & 63, c16 = lane & 15, g = lane >> 4;
    const int64_t i0 = (int64_t)blockIdx.x * (32 * NW) + (threadIdx.x >> 6) * 32 + c16;
    const RowPos q[2] = {row_pos(p, j, i0), row_pos(p, j, i0 + 16)};
    RowCoef rc[2];
    float sc[2];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
        const RowPos &qr = q[rt];
        const int64_t i = i0 + 16 * rt;
        rc[rt] = RowCoef{0.0f, 0.0f, 0.0f, -1, false};
        sc[rt] = 0.0f;
        if (qr.valid) {
            rc[rt] = row_coef(p, qr.t, qr.T, qr.S, qr.s, qr.row, p.ll[qr.b], p.labels + (int64_t)qr.b * p.label_stride);
            sc[rt] = j.scale ? j.scale[qr.b] : 1.0f;
            if (g == 0 && j.bt_idx) j.bt_idx[i] = (int64_t)qr.b * (j.enc_sb / j.H) + qr.t;
            if (g == 0 && j.bs_idx) j.bs_idx[i] = (int64_t)qr.b * (j.pred_sb / j.H) + qr.s;
        }
    }
    const int V = p.V, blank = p.blank;
    const float *bias = load_bias<KS, NB>(j, V, wsh);
    // dbias: this workgroup's column sums of G, in a fixed order (bitwise reproducible): per chunk, each wave's 32
    // column sums (a DPP row reduction over each lane group's 16 rows) go to that wave's own LDS row (every entry
    // written once), and after the loop the NW rows are added in wave order; the workgroup's row of sums then goes to
    // dbias_part[blockIdx.x] for the ordered sum over workgroups (launch_joint_dbias_sum). launch_kt sizes the LDS.
    const int vpad = (V + 31) / 32 * 32;
    const int wave = threadIdx.x >> 6;
    float *dbw = const_cast<float *>(bias) + vpad;  // [NW][vpad]
    __syncthreads();  // the bias row in LDS
    bf16x8 bfr[2][K32];
    build_row<K32, 32, true>(j, q[0], 8 * g, i0, bfr[0]);
    build_row<K32, 32, true>(j, q[1], 8 * g, i0 + 16, bfr[1]);

    // exactly 4 vector stores per chunk (2 row tiles x 2 vocabulary tiles) on every wave whose lanes are all valid:
    // leave them in flight at the barrier
    const bool vec_out = (V & 3) == 0;
    const bool leave = vec_out && __ballot(!(q[0].valid && q[1].valid)) == 0;
    unsigned short *grow[2] = {j.G + (q[0].valid ? i0 : 0) * V, j.G + (q[1].valid ? i0 + 16 : 0) * V};
    chunk_loop_with<KS, NB, NW>(
        j, V, wsh, leave ? 4 : -1, [&](const unsigned short *wb) { return WTile16<KS>::template mma<4>(wb, bfr, lane); },
        [&](const typename WTile16<KS>::Acc &acc, int c) {
            const f4 bv[2] = {*reinterpret_cast<const f4 *>(bias + 32 * c + 4 * g),
                              *reinterpret_cast<const f4 *>(bias + 32 * c + 16 + 4 * g)};
            const int jb = blank - 32 * c;
            const bool hb = jb >= 0 && jb < 32 && ((jb >> 2) & 3) == g;
            float cs[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};  // dbias: this lane's two rows
#pragma unroll
            for (int rt = 0; rt < 2; ++rt) {
                float x[8];
                logits8<KS>(acc, bv, rt, x);
#pragma unroll
                for (int k = 0; k < 8; ++k) x[k] = fast_exp2(fmaf(x[k], kLog2e, rc[rt].c2));
                // the <= 2 corrected entries of the row are rewritten by a second (2-byte) store after the vector store
                const int jl = rc[rt].lab - 32 * c;
                const bool mine = rc[rt].lab >= 0 && jl >= 0 && jl < 32 && ((jl >> 2) & 3) == g;
                float gb = 0.0f, gl = 0.0f;
                if (jb >= 0 && jb < 32) gb = pick8(x, pick8_index(jb));
                if (__ballot(mine)) gl = pick8(x, pick8_index(jl & 31));
                if (q[rt].valid) {
                    const float s = sc[rt];
#pragma unroll
                    for (int vt = 0; vt < 2; ++vt) {
                        const int v0 = 32 * c + 16 * vt + 4 * g;
                        const float e4[4] = {x[4 * vt] * s, x[4 * vt + 1] * s, x[4 * vt + 2] * s, x[4 * vt + 3] * s};
#pragma unroll
                        for (int e = 0; e < 4; ++e) cs[4 * vt + e] += e4[e];
                        if (vec_out && v0 + 3 < V) {
                            *reinterpret_cast<uint2 *>(grow[rt] + v0) =
                                make_uint2(IoBF16::pack2(e4[0], e4[1]), IoBF16::pack2(e4[2], e4[3]));
                        } else {
#pragma unroll
                            for (int e = 0; e < 4; ++e)
                                if (v0 + e < V) grow[rt][v0 + e] = IoBF16::from_f(e4[e]);
                        }
                    }
                    if (hb) grow[rt][blank] = IoBF16::from_f((gb - rc[rt].cb) * s);
                    if (mine) grow[rt][rc[rt].lab] = IoBF16::from_f((gl - rc[rt].ce) * s);
                    if (j.dbias) {  // the two corrected entries: the column sums above hold them uncorrected
                        const int kb = hb ? pick8_index(jb) : -1, kl = mine ? pick8_index(jl & 31) : -1;
                        const float db = rc[rt].cb * s, dl = rc[rt].ce * s;
#pragma unroll
                        for (int k = 0; k < 8; ++k) {
                            if (k == kb) cs[k] -= db;
                            if (k == kl) cs[k] -= dl;
                        }
                    }
                }
            }
            if (j.dbias) {  // sum the 16 lanes of each lane group (one DPP row: rows of the tile), lane 15 adds to LDS
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    float v = cs[k];
                    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x111, 0xf, 0xf, true));
                    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x112, 0xf, 0xf, true));
                    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x114, 0xf, 0xf, true));
                    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x118, 0xf, 0xf, true));
                    cs[k] = v;
                }
                if (c16 == 15) {
                    float *row = dbw + wave * vpad + 32 * c;
#pragma unroll
                    for (int k = 0; k < 8; ++k) row[16 * (k >> 2) + 4 * g + (k & 3)] = cs[k];
                }
            }
        });
    if (j.dbias) {
        __syncthreads();
        float *row = j.dbias_part + (int64_t)blockIdx.x * vpad;
        for (int v = threadIdx.x; v < vpad; v += blockDim.x) {
            float t = 0.0f;
#pragma unroll
            for (int w = 0; w < NW; ++w) t += dbw[w * vpad + v];
            row[v] = t;
        }
    }
}

// dbias += the column sums of the backward's per-workgroup rows, in a fixed order: stage 1 sums segments of
// kDbiasSeg rows (64 columns x 4 row lanes per workgroup, each lane its rows in order, the 4 lanes in order),
// stage 2 the segments in order. Bitwise reproducible, unlike float atomics (cdna_hip_programming.md Guideline 12).
constexpr int kDbiasSeg = 256;

__global__ __launch_bounds__(256) void dbias_seg_kernel(const float *__restrict__ part, int64_t nrows, int vpad,
                                                        float *__restrict__ seg_out) {
    __shared__ float red[4][64];
    const int col = blockIdx.x * 64 + (threadIdx.x & 63), rl = threadIdx.x >> 6;
    const int64_t r0 = (int64_t)blockIdx.y * kDbiasSeg, r1 = min(r0 + kDbiasSeg, nrows);
    float t = 0.0f;
    if (col < vpad)
        for (int64_t r = r0 + rl; r < r1; r += 4) t += part[r * vpad + col];
    red[rl][threadIdx.x & 63] = t;
    __syncthreads();
    if (rl == 0 && col < vpad)
        seg_out[(int64_t)blockIdx.y * vpad + col] = ((red[0][col & 63] + red[1][col & 63]) + red[2][col & 63]) +
                                                    red[3][col & 63];
}

__global__ __launch_bounds__(256) void dbias_total_kernel(const float *__restrict__ seg, int nseg, int vpad, int V,
                                                          float *__restrict__ dbias) {
    const int v = blockIdx.x * 256 + threadIdx.x;
    if (v >= V) return;
    float t = 0.0f;
    for (int k = 0; k < nseg; ++k) t += seg[(int64_t)k * vpad + v];
    dbias[v] += t;
}

int64_t joint_bwd_blocks(int64_t n) { return (n + 255) / 256; }  // the backward's workgroups (8 waves x 32 rows)

// Rows [count, n) of G ([n, V] bf16) and Hact ([n, ld] bf16) as zeros, count = *count_dev (a device-counted live-row
// list sized by a host bound, JointArgs::n_dev): library GEMMs over all n rows then see zero rows there. Grid-stride
// 16-byte stores over the tail's byte range (rows are contiguous), 2-byte stores for its unaligned ends.
__global__ __launch_bounds__(256) void joint_tail_zero_kernel(unsigned short *__restrict__ G, int64_t gld,
                                                              unsigned short *__restrict__ Hact, int64_t hld, int64_t n,
                                                              const unsigned long long *__restrict__ count_dev) {
    const int64_t c = min((int64_t)*count_dev, n);
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (int64_t)gridDim.x * blockDim.x;
    for (int which = 0; which < 2; ++which) {
        unsigned short *base = which ? Hact : G;
        const int64_t ld = which ? hld : gld;
        const int64_t e0 = c * ld, e1 = n * ld;  // elements
        const int64_t a0 = min(e1, (e0 + 7) / 8 * 8), a1 = max(a0, e1 / 8 * 8);
        if (tid < a0 - e0) base[e0 + tid] = 0;
        if (tid < e1 - a1) base[a1 + tid] = 0;
        for (int64_t o = a0 + tid * 8; o < a1; o += nth * 8) *reinterpret_cast<u4 *>(base + o) = u4{0u, 0u, 0u, 0u};
    }
}

hipError_t launch_joint_tail_zero(unsigned short *G, int V, unsigned short *Hact, int64_t hact_ld, int64_t n,
                                  const unsigned long long *count_dev, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    joint_tail_zero_kernel<<<2048, 256, 0, stream>>>(G, V, Hact, hact_ld, n, count_dev);
    return hipGetLastError();
}

size_t joint_dbias_part_bytes(int64_t n_max, int V) {
    const int64_t vpad = (V + 31) / 32 * 32, nb = joint_bwd_blocks(n_max);
    return sizeof(float) * (size_t)vpad * (size_t)(nb + (nb + kDbiasSeg - 1) / kDbiasSeg);
}

hipError_t launch_joint_dbias_sum(const JointArgs &j, int V, hipStream_t stream) {
    const int vpad = (V + 31) / 32 * 32;
    const int64_t nb = joint_bwd_blocks(j.n);
    if (nb <= 0) return hipSuccess;
    const int64_t nseg = (nb + kDbiasSeg - 1) / kDbiasSeg;
    if (nseg > 65535) return hipErrorInvalidValue;
    float *seg = j.dbias_part + nb * vpad;
    dbias_seg_kernel<<<dim3((vpad + 63) / 64, (unsigned)nseg), 256, 0, stream>>>(j.dbias_part, nb, vpad, seg);
    dbias_total_kernel<<<(V + 255) / 256, 256, 0, stream>>>(seg, (int)nseg, vpad, V, j.dbias);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------------------
// backward tail: dpre = dH * (1 - Hact^2) over the live rows, summed into denc[b, t] (over s; written once per
// column) and dpred[b, s] (over t, accumulated in LDS frame by frame). One workgroup per (utterance, block of TT frames,
// slice of HS hidden units); 4 hidden units per thread (8-byte loads), 256/(HS/4) rows in flight. Bitwise
// reproducible: every sum has one fixed order and one writer -- a block's d_pred sums go to its own rows of a scratch
// buffer (part, with the label range it touched in rng) and pred_sum_kernel adds the blocks in block order; without
// scratch one block covers the whole utterance (TT = T_max) and flushes d_pred itself (fewer, longer workgroups).

constexpr int kReduceTT = 64;  // frames per workgroup (blocked form, and the sparse variant)

// SRC: where the tanh derivative's activation comes from.
//   kRedHact (default): read from Hact;
//   kRedTanh (development build, joint_reduce_hact = 0): recomputed, h = bf16(fast_tanh2(enc + pred)) exactly as the
//     gradient pass built it (same function and operands: the stored Hact's bits, test_joint_reduce_recomputed_
//     activation_is_bit_identical) -- enc[b, t] once per frame, the pred slice staged in LDS, so the reduce streams dH
//     alone (4 GB at H = 512 instead of 8). Measured slower, 2.71 -> 4.26 ms: the frame loop is latency-bound, and the
//     staged slice costs occupancy (three workgroups per CU instead of five) -- the bytes were not its limit;
//   kRedPre: dH already holds dpre = dH * (1 - Hact^2) (mrnnt_joint_dpre's epilogue).
constexpr int kRedTanh = 0, kRedHact = 1, kRedPre = 2;

// AP: LDS row pitch of the accumulators (HS + 1: a column's consecutive rows start on successive banks, so the four
// 4-byte accesses per thread -- 8 threads per row, 4 rows per 32-lane bank group -- are conflict-free; a pitch of HS
// put rows s and s + 2 on the same banks, SQ_LDS_BANK_CONFLICT 0.67 of the LDS cycles in round 4).
template <int HS, int SRC, int AP>
__global__ __launch_bounds__(256) void joint_reduce_kernel(DevProblem p, JointArgs j, const int64_t *__restrict__ off,
                                                           const unsigned short *__restrict__ dH,
                                                           float *__restrict__ d_enc, float *__restrict__ d_pred,
                                                           int tt, int ntb, int wstride, float *__restrict__ part,
                                                           int *__restrict__ rng) {
    constexpr int TPR = HS / 4;     // threads per row slice
    constexpr int RP = 256 / TPR;   // rows in parallel
    extern __shared__ float lds[];  // acc[(S_b+1) * AP], red[RP][AP], then (kRedTanh) pred slice [S_b+1][HS] bf16
    const int H = j.H;
    const int nh = H / HS;
    // the h-slices of one block of frames are consecutive workgroups: they read the same rows (L2 reuse)
    const int bx = blockIdx.x / nh;
    const int h0 = (blockIdx.x % nh) * HS;
    const int b = bx / ntb, blk = bx % ntb;
    const int t0 = blk * tt;
    const int T = p.T[b], S = p.S[b];
    const int tid = threadIdx.x;
    if (t0 >= T) {  // (past this utterance's frames: an empty label range for the block sum)
        if (part && h0 == 0 && tid == 0) {
            rng[2 * bx] = 1;
            rng[2 * bx + 1] = 0;
        }
        return;
    }
    const int hl = (tid % TPR) * 4, rsub = tid / TPR;
#ifdef MRNNT_DEVTOOLS
    const bool trace = (j.probe & 16) && blockIdx.x < (unsigned)kRedTraceWgs;
#define RED_MARK(i) \
    do { if (trace && tid == 0) g_reduce_trace[blockIdx.x * 16 + (i)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define RED_MARK(i) ((void)0)
#endif
    RED_MARK(0);
    float *acc = lds;
    float *red = lds + (S + 1) * AP;
    const int64_t tslots = j.enc_sb / H, sslots = j.pred_sb / H;
    const int t1 = min(t0 + tt, T);
    // label positions this block of frames touches: rows of a column are listed by ascending s, so the first and
    // last row of each column bound them (a few labels under an alignment restriction, the band otherwise); only
    // that slice of the d_pred accumulator is cleared and flushed (min / max: order-independent)
    __shared__ int srange[2];
    // the block's list offsets, read once here (kReduceTT frames): the frame loop then starts each frame's row loads
    // without first waiting for a global load of its offsets
    __shared__ int64_t soff[kReduceTT + 1];
    const bool staged_off = t1 - t0 <= kReduceTT && !(kVariants && (j.probe & 64));  // (probe bit 6: A/B)
    if (tid == 0) {
        srange[0] = S + 1;
        srange[1] = -1;
    }
    __syncthreads();
    for (int t = t0 + tid; t < t1; t += 256) {
        const int64_t col = p.col_off[b] + t;
        const int64_t r0 = off[col], r1 = off[col + 1];
        if (staged_off) {
            soff[t - t0] = r0;
            if (t == t1 - 1) soff[t1 - t0] = r1;
        }
        if (r1 > r0) {
            atomicMin(&srange[0], j.ls[r0]);
            atomicMax(&srange[1], j.ls[r1 - 1]);
        }
    }
    __syncthreads();
    const int s_lo = srange[0], s_hi = srange[1];
    for (int i = s_lo * HS + tid; i < (s_hi + 1) * HS; i += 256) acc[i / HS * AP + i % HS] = 0.0f;
    // kRedTanh: pred[b, s, h0 .. h0 + HS) for the touched s, 8 bytes per thread and row
    unsigned short *pl = reinterpret_cast<unsigned short *>(red + RP * AP);
    if constexpr (SRC == kRedTanh) {
        for (int i = s_lo * TPR + tid; i < (s_hi + 1) * TPR; i += 256) {
            const int ss = i / TPR, hq = (i % TPR) * 4;
            *reinterpret_cast<uint2 *>(pl + ss * HS + hq) =
                *reinterpret_cast<const uint2 *>(j.pred + (int64_t)b * j.pred_sb + (int64_t)ss * H + h0 + hq);
        }
    }
    __syncthreads();
    RED_MARK(1);
    for (int t = t0; t < t1; ++t) {
        const int64_t col = p.col_off[b] + t;
        const int64_t r0 = staged_off ? soff[t - t0] : off[col], r1 = staged_off ? soff[t - t0 + 1] : off[col + 1];
        float e0 = 0.0f, e1 = 0.0f, e2 = 0.0f, e3 = 0.0f;
        uint2 ev = make_uint2(0u, 0u);
        if constexpr (SRC == kRedTanh)
            if (r1 > r0) ev = *reinterpret_cast<const uint2 *>(j.enc + (int64_t)b * j.enc_sb + (int64_t)t * H + h0 + hl);
        for (int64_t r = r0 + rsub; r < r1; r += RP) {
            const int s = j.ls[r];
            const uint2 dv = *reinterpret_cast<const uint2 *>(dH + r * H + h0 + hl);
            float v0 = bf16_lo(dv.x), v1 = bf16_hi(dv.x), v2 = bf16_lo(dv.y), v3 = bf16_hi(dv.y);
            if constexpr (SRC != kRedPre) {
                float h_0, h_1, h_2, h_3;
                if constexpr (SRC == kRedHact) {
                    const uint2 hv = *reinterpret_cast<const uint2 *>(j.Hact + r * j.hact_ld + h0 + hl);
                    h_0 = bf16_lo(hv.x), h_1 = bf16_hi(hv.x), h_2 = bf16_lo(hv.y), h_3 = bf16_hi(hv.y);
                } else {  // build_row's activation, bit for bit
                    const uint2 pv = *reinterpret_cast<const uint2 *>(pl + s * HS + hl);
                    const f2 ya = fast_tanh2((f2){bf16_lo(ev.x), bf16_hi(ev.x)} + (f2){bf16_lo(pv.x), bf16_hi(pv.x)});
                    const f2 yb = fast_tanh2((f2){bf16_lo(ev.y), bf16_hi(ev.y)} + (f2){bf16_lo(pv.y), bf16_hi(pv.y)});
                    h_0 = (float)(__bf16)ya.x, h_1 = (float)(__bf16)ya.y, h_2 = (float)(__bf16)yb.x;
                    h_3 = (float)(__bf16)yb.y;
                }
                v0 *= 1.0f - h_0 * h_0;
                v1 *= 1.0f - h_1 * h_1;
                v2 *= 1.0f - h_2 * h_2;
                v3 *= 1.0f - h_3 * h_3;
            }
            e0 += v0;
            e1 += v1;
            e2 += v2;
            e3 += v3;
            float *a = acc + s * AP + hl;  // distinct s within a column: one writer per element
            a[0] += v0;
            a[1] += v1;
            a[2] += v2;
            a[3] += v3;
        }
        if (kVariants && (j.probe & 4)) {  // development timing probe: no frame barriers / d_enc sum (wrong results)
            if (rsub == 0) {
                float *de = d_enc + ((int64_t)b * tslots + t) * H + h0 + hl;
                de[0] = e0;
                de[1] = e1;
                de[2] = e2;
                de[3] = e3;
            }
            continue;
        }
        if (t - t0 < 6) RED_MARK(2 + 2 * (t - t0));
        float *rr = red + rsub * AP + hl;
        rr[0] = e0;
        rr[1] = e1;
        rr[2] = e2;
        rr[3] = e3;
        __syncthreads();
        if (tid < HS) {
            float sum = 0.0f;
#pragma unroll 4
            for (int g = 0; g < RP; ++g) sum += red[g * AP + tid];
            d_enc[((int64_t)b * tslots + t) * H + h0 + tid] = sum;
        }
        __syncthreads();
        if (t - t0 < 6) RED_MARK(3 + 2 * (t - t0));
    }
    RED_MARK(14);
    if (!part) {  // one block per utterance: this workgroup is the one writer
        for (int i = s_lo * HS + tid; i < (s_hi + 1) * HS; i += 256)
            d_pred[((int64_t)b * sslots + i / HS) * H + h0 + i % HS] += acc[i / HS * AP + i % HS];
        return;
    }
    float *pb = part + (int64_t)bx * wstride * H;
    for (int i = s_lo * HS + tid; i < (s_hi + 1) * HS; i += 256)
        pb[(int64_t)(i / HS) * H + h0 + i % HS] = acc[i / HS * AP + i % HS];
    if (h0 == 0 && tid == 0) {
        rng[2 * bx] = s_lo;
        rng[2 * bx + 1] = s_hi;
    }
    RED_MARK(15);
#undef RED_MARK
}

// d_pred[b, s, :] += the blocks' sums of label position s, in block order (the blocks whose range holds s)
__global__ __launch_bounds__(256) void pred_sum_kernel(DevProblem p, const float *__restrict__ part,
                                                       const int *__restrict__ rng, int ntb, int wstride, int H,
                                                       int64_t sslots, float *__restrict__ d_pred) {
    const int b = blockIdx.y;
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int s = (int)(e / H), h = (int)(e % H);
    if (s > p.S[b]) return;
    float t = 0.0f;
    for (int k = 0; k < ntb; ++k) {
        const int bx = b * ntb + k;
        if (s >= rng[2 * bx] && s <= rng[2 * bx + 1]) t += part[((int64_t)bx * wstride + s) * H + h];
    }
    d_pred[((int64_t)b * sslots + s) * H + h] += t;
}

size_t joint_reduce_scratch_bytes(int B, int T_max, int S_max, int H) {
    const int64_t ntb = (T_max + kReduceTT - 1) / kReduceTT;
    return sizeof(float) * (size_t)B * ntb * (S_max + 1) * H + sizeof(int) * 2 * (size_t)B * ntb + 256;
}


// Sparse variant (development build, joint_reduce_sparse = 2; float atomics: not bitwise reproducible) (few live rows per frame, e.g. alignment-restricted training): the rows of a block of frames are
// processed all at once (TPR threads per row) instead of frame by frame, so a workgroup does not wait one
// dependent load chain per frame; d_enc and d_pred partials meet in LDS through ds_add_f32.
template <int HS>
__global__ __launch_bounds__(256) void joint_reduce_sparse_kernel(DevProblem p, JointArgs j,
                                                                  const int64_t *__restrict__ off,
                                                                  const unsigned short *__restrict__ dH,
                                                                  float *__restrict__ d_enc, float *__restrict__ d_pred,
                                                                  int ntb) {
    constexpr int TPR = HS / 4;
    constexpr int RP = 256 / TPR;
    extern __shared__ float lds[];  // acc_pred[(S_b+1) * HS] then acc_enc[kReduceTT * HS]
    const int H = j.H;
    const int nh = H / HS;
    const int bx = blockIdx.x / nh;
    const int h0 = (blockIdx.x % nh) * HS;
    const int b = bx / ntb;
    const int t0 = (bx % ntb) * kReduceTT;
    const int T = p.T[b], S = p.S[b];
    if (t0 >= T) return;
    const int tid = threadIdx.x;
    const int hl = (tid % TPR) * 4, rsub = tid / TPR;
    const int t1 = min(t0 + kReduceTT, T);
    float *accp = lds;
    float *acce = lds + (S + 1) * HS;
    const int64_t c0 = p.col_off[b];
    const int64_t rb = off[c0 + t0], re = off[c0 + t1];
    // the label range the rows touch: only that slice of the d_pred accumulator is cleared and flushed
    __shared__ int srange[2];
    if (tid == 0) {
        srange[0] = S + 1;
        srange[1] = -1;
    }
    for (int i = tid; i < kReduceTT * HS; i += 256) acce[i] = 0.0f;
    __syncthreads();
    for (int64_t r = rb + tid; r < re; r += 256) {
        const int s = j.ls[r];
        atomicMin(&srange[0], s);
        atomicMax(&srange[1], s);
    }
    __syncthreads();
    const int s_lo = srange[0], s_hi = srange[1];
    for (int i = s_lo * HS + tid; i < (s_hi + 1) * HS; i += 256) accp[i] = 0.0f;
    __syncthreads();
    for (int64_t r = rb + rsub; r < re; r += RP) {
        const int s = j.ls[r];
        const int tt = (int)(j.lcol[r] - c0 - t0);
        const uint2 dv = *reinterpret_cast<const uint2 *>(dH + r * H + h0 + hl);
        const uint2 hv = *reinterpret_cast<const uint2 *>(j.Hact + r * j.hact_ld + h0 + hl);
        const float h_0 = bf16_lo(hv.x), h_1 = bf16_hi(hv.x), h_2 = bf16_lo(hv.y), h_3 = bf16_hi(hv.y);
        const float v[4] = {bf16_lo(dv.x) * (1.0f - h_0 * h_0), bf16_hi(dv.x) * (1.0f - h_1 * h_1),
                            bf16_lo(dv.y) * (1.0f - h_2 * h_2), bf16_hi(dv.y) * (1.0f - h_3 * h_3)};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            atomicAdd(&acce[tt * HS + hl + q], v[q]);
            atomicAdd(&accp[s * HS + hl + q], v[q]);
        }
    }
    __syncthreads();
    const int64_t tslots = j.enc_sb / H, sslots = j.pred_sb / H;
    for (int i = tid; i < (t1 - t0) * HS; i += 256)  // rows (b, t < T_b) of d_enc are overwritten (ABI)
        d_enc[((int64_t)b * tslots + t0 + i / HS) * H + h0 + i % HS] = acce[i];
    for (int i = s_lo * HS + tid; i < (s_hi + 1) * HS; i += 256) {
        const float v = accp[i];
        if (v != 0.0f) atomicAdd(&d_pred[((int64_t)b * sslots + i / HS) * H + h0 + i % HS], v);
    }
}

hipError_t launch_joint_reduce(const DevProblem &p, const JointArgs &j_in, const int64_t *off, int T_max, int S_max,
                               const unsigned short *dH, float *d_enc, float *d_pred, void *scratch,
                               size_t scratch_bytes, hipStream_t stream) {
    JointArgs j = j_in;
    if (kVariants) j.probe = tuning().joint_probe;
    const int ntb = (T_max + kReduceTT - 1) / kReduceTT;
    const int W = S_max + 1;
    // the row-parallel sparse kernel with float atomics: development A/B only (joint_reduce_sparse = 2; dH + Hact)
    const bool pre = j.Hact == nullptr;  // dH holds dpre (mrnnt_joint_dpre)
    const bool sparse = kVariants && tuning().joint_reduce_sparse == 2 && !pre;
    const bool tanh_src = kVariants && tuning().joint_reduce_hact == 0 && !pre;
    auto go = [&](auto hs_tag) -> hipError_t {
        constexpr int HS = decltype(hs_tag)::value;
        // (accumulator pitch HS + 1; the development build's joint_reduce_pad = 0 runs pitch HS, bit-identical)
        constexpr int AP = HS + 1;
        const bool nopad = kVariants && tuning().joint_reduce_pad == 0;
        auto kern = pre ? (nopad ? joint_reduce_kernel<HS, kRedPre, HS> : joint_reduce_kernel<HS, kRedPre, AP>)
                        : (tanh_src ? joint_reduce_kernel<HS, kRedTanh, AP>
                                    : (nopad ? joint_reduce_kernel<HS, kRedHact, HS>
                                             : joint_reduce_kernel<HS, kRedHact, AP>));
        const int apitch = nopad ? HS : AP;
        if (sparse) {
            const size_t lds = sizeof(float) * ((size_t)W * HS + (size_t)kReduceTT * HS);
            joint_reduce_sparse_kernel<HS><<<p.B * ntb * (j.H / HS), 256, lds, stream>>>(p, j, off, dH, d_enc,
                                                                                          d_pred, ntb);
            return hipSuccess;
        }
        // (+ the staged pred slice, bf16 [W][HS], of the recomputing form: up to 88 KiB)
        const size_t lds = sizeof(float) * ((size_t)W * apitch + 256 / (HS / 4) * apitch) +
                           (tanh_src ? sizeof(unsigned short) * W * HS : 0);
        if (lds > 65536) {  // (no launch with too little LDS: the attribute's failure is the call's error)
            const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
        }
        if (scratch && scratch_bytes >= joint_reduce_scratch_bytes(p.B, T_max, S_max, j.H)) {
            // blocks of kReduceTT frames, their d_pred sums added in block order by pred_sum_kernel
            float *part = static_cast<float *>(scratch);
            int *rng = reinterpret_cast<int *>(part + (size_t)p.B * ntb * W * j.H);
            kern<<<p.B * ntb * (j.H / HS), 256, lds, stream>>>(p, j, off, dH, d_enc, d_pred, kReduceTT, ntb, W, part,
                                                                rng);
            pred_sum_kernel<<<dim3((unsigned)(((int64_t)W * j.H + 255) / 256), (unsigned)p.B), 256, 0, stream>>>(
                p, part, rng, ntb, W, j.H, j.pred_sb / j.H, d_pred);
        } else {  // one block per utterance (no scratch)
            kern<<<p.B * (j.H / HS), 256, lds, stream>>>(p, j, off, dH, d_enc, d_pred, T_max, 1, W, nullptr, nullptr);
        }
        return hipSuccess;
    };
    if ((int64_t)p.B * ntb * (j.H / 4) > (1ll << 24)) return hipErrorInvalidValue;  // 32-bit dispatch size
    // LDS = W * HS fp32 + 4 KiB + W * HS bf16: about 43 KiB at the headline (three workgroups per CU), <= 88 KiB
    const hipError_t e = W <= 448    ? go(std::integral_constant<int, 32>())
                         : W <= 896  ? go(std::integral_constant<int, 16>())
                         : W <= 1792 ? go(std::integral_constant<int, 8>())
                                     : go(std::integral_constant<int, 4>());
    return e != hipSuccess ? e : hipGetLastError();
}

// kernel of a launch shape: MF = the backward's MFMA tile (32: 32x32x16, 16: 16x16x32); the forward runs 32x32x16
template <int KS, int NB, int NW, int MF, bool BWD, int RG>
static hipError_t launch_knw(const DevProblem &p, const JointArgs &j, size_t lds, hipStream_t stream) {
    const int64_t blocks = (j.n + 32 * NW - 1) / (32 * NW);
    if (blocks * 64 * NW > 0xffffffffll) return hipErrorInvalidValue;  // 32-bit dispatch size in work-items
    void (*kern)(DevProblem, JointArgs);
    if constexpr (MF == 16 && BWD) kern = joint_bwd16_kernel<KS, NB, NW>;
    else if constexpr (BWD) kern = joint_bwd_kernel<KS, NB, NW, RG>;
    else {
        kern = joint_fwd_kernel<KS, NB, NW, RG>;
        if constexpr (kVariants)
            if (tuning().joint_trace) kern = joint_fwd_kernel<KS, NB, NW, RG, true>;
    }
    if (lds > 65536) {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    kern<<<(int)blocks, 64 * NW, lds, stream>>>(p, j);
    return hipGetLastError();
}

// One workgroup of 8 waves per CU (two per SIMD, 256 rows sharing each W chunk), two DMA buffers. (Measured and
// removed, DESIGN.md §4a: three buffers, two 4-wave workgroups per CU, deeper A-fragment rings, the forward on the
// 16x16x32 tile, a persistent forward, the pipelined one-wave-per-SIMD forward, the bias as the initial accumulator
// and the label logit as a dot product.)
template <int KS, int MF, bool BWD>
static hipError_t launch_kt(const DevProblem &p, const JointArgs &j, hipStream_t stream) {
    // the 16x16x32 backward with dbias keeps one row of column sums per wave (8) behind the bias; the forward a
    // bias * log2 e row (JointArgs::opt bit 1) where both rows fit, the unscaled epilogue otherwise
    const size_t row = sizeof(float) * ((p.V + 31) / 32 * 32);
    const size_t tile = sizeof(unsigned short) * WTile<KS>::ELEMS;
    JointArgs jj = j;
    if (!BWD && 2 * tile + 2 * row > 160 * 1024) jj.opt &= ~2;
    const size_t bias = row * ((MF == 16 && BWD && j.dbias) ? 9 : (!BWD && (jj.opt & 2)) ? 2 : 1);
    if (j.dbias && !(MF == 16 && BWD)) return hipErrorInvalidValue;
    if (2 * tile + bias <= 160 * 1024) return launch_knw<KS, 2, 8, MF, BWD, 2>(p, jj, 2 * tile + bias, stream);
    return hipErrorInvalidValue;
}

// The backward's MFMA tile: 16x16x32 for H <= 512 (its epilogue carries no per-row running state, and there the
// 16x16 tile's higher clock pays), 32x32x16 at H = 640 (the 16x16 one spills there: two rows' state per lane beside
// 160 B-operand registers); the development build can force 32x32x16 (joint_bwd_mfma = 32).
template <int KS, bool BWD>
static hipError_t launch_kb(const DevProblem &p, const JointArgs &j, hipStream_t stream) {
    constexpr int kDefault = KS > 32 ? 32 : BWD ? Tuning{}.joint_bwd_mfma : 32;
    if constexpr (kVariants && KS <= 32 && BWD) {
        if (tuning().joint_bwd_mfma == 32) return launch_kt<KS, 32, BWD>(p, j, stream);
    }
    return launch_kt<KS, kDefault, BWD>(p, j, stream);
}

template <int KS>
static hipError_t launch_kh(const DevProblem &p, const JointArgs &j, bool bwd, hipStream_t stream) {
    return bwd ? launch_kb<KS, true>(p, j, stream) : launch_kb<KS, false>(p, j, stream);
}

size_t joint_min_lds_bytes(int H, int V) {  // two weight tiles + the bias row
    return 2 * sizeof(unsigned short) * 32 * (size_t)H + sizeof(float) * (((size_t)V + 31) / 32 * 32);
}

size_t joint_dbias_lds_bytes(int H, int V) {  // the 16x16x32 backward with dbias: + one column-sum row per wave
    return joint_min_lds_bytes(H, V) + 8 * sizeof(float) * (((size_t)V + 31) / 32 * 32);
}

static hipError_t launch_joint(const DevProblem &p, const JointArgs &j, bool bwd, hipStream_t stream) {
    if (j.n <= 0) return hipSuccess;
    switch (j.H) {
        case 128: return launch_kh<8>(p, j, bwd, stream);
        case 256: return launch_kh<16>(p, j, bwd, stream);
        case 384: return launch_kh<24>(p, j, bwd, stream);
        case 512: return launch_kh<32>(p, j, bwd, stream);
        case 640: return launch_kh<40>(p, j, bwd, stream);
        default: return hipErrorInvalidValue;
    }
}

// flag = 1 when max_v (sum_h |W[v, h]| + |bias[v]|) <= 64: every logit z = W_v . h + b_v with |h| <= 1 (tanh,
// rounded to bf16) then lies in [-64, 64]. One workgroup (no cross-workgroup combine, no flag reset launch), a wave per
// weight row at a time, 16-byte loads (a 1 KiB row of H = 512 in one load per lane group): the V x H bf16 weights
// (1 MiB at the headline joint size) are read once, a few microseconds. NaN / inf weights compare false: flag 0, the
// running-max epilogue.
__global__ __launch_bounds__(1024) void joint_wbound_kernel(const unsigned short *__restrict__ W,
                                                            const float *__restrict__ bias, int V, int H,
                                                            int *__restrict__ flag) {
    __shared__ int bad;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x == 0) bad = 0;
    __syncthreads();
    int mine = 0;
    for (int v0 = wave; v0 < V; v0 += 64) {  // four rows per wave per pass: eight loads in flight per lane
        float s[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int v = v0 + 16 * r;
            s[r] = 0.0f;
#pragma unroll
            for (int k = 0; k < 2; ++k) {  // H <= 640 < 1024 (the joint plan's shapes), a multiple of 8
                const int h = 8 * lane + 512 * k;
                if (v < V && h < H) {
                    const uint4 u = *reinterpret_cast<const uint4 *>(W + (int64_t)v * H + h);
                    s[r] += (fabsf(bf16_lo(u.x)) + fabsf(bf16_hi(u.x))) + (fabsf(bf16_lo(u.y)) + fabsf(bf16_hi(u.y))) +
                            (fabsf(bf16_lo(u.z)) + fabsf(bf16_hi(u.z))) + (fabsf(bf16_lo(u.w)) + fabsf(bf16_hi(u.w)));
                }
            }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int v = v0 + 16 * r;
            float t = s[r];
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) t += __shfl_xor(t, o);
            if (v < V) {
                if (bias) t += fabsf(bias[v]);
                if (!(t <= 64.0f)) mine = 1;
            }
        }
    }
    if (mine && lane == 0) atomicOr(&bad, 1);
    __syncthreads();
    if (threadIdx.x == 0) *flag = bad ? 0 : 1;
}

hipError_t launch_joint_wbound(const unsigned short *W, const float *bias, int V, int H, int *flag,
                               hipStream_t stream) {
    if (V <= 0 || H <= 0 || H > 1024 || (H & 7)) return hipErrorInvalidValue;
    joint_wbound_kernel<<<1, 1024, 0, stream>>>(W, bias, V, H, flag);
    return hipGetLastError();
}

hipError_t launch_joint_forward(const DevProblem &p, const JointArgs &j, hipStream_t stream) {
    if (kVariants && tuning().joint_probe) {
        JointArgs jp = j;
        jp.probe = tuning().joint_probe;
        if (jp.probe & 8) jp.wplain = nullptr;  // (A/B: the running-max epilogue whatever the bound)
        return launch_joint(p, jp, false, stream);
    }
    return launch_joint(p, j, false, stream);
}

hipError_t launch_joint_backward(const DevProblem &p, const JointArgs &j, hipStream_t stream) {
    return launch_joint(p, j, true, stream);
}

}  // namespace mrnnt
