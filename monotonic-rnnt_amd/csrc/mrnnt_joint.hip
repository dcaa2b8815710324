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
// Tiling: a workgroup of 4 waves owns 128 consecutive rows of a row list; a wave owns 32 rows and keeps their
// activations as the MFMA B operand in registers (lane l: row l&31, k = 16 ks + 8 (l>>5) + [0,8)), built
// once from enc/pred with a fast tanh. W streams through LDS in 32-vocabulary chunks (double-buffered,
// padded rows against bank conflicts) shared by the 4 waves; each chunk is one 32x32 output tile per wave,
// D[vocab][row] = sum_k W[vocab][k] h[row][k]: the accumulator holds 16 vocabulary entries of ONE row per
// lane (vocab = (i&3) + 8 (i>>2) + 4 (l>>5)), so the per-row online softmax is register-local and the two
// lane halves merge once at the end.
#include <type_traits>

#include "mrnnt_device.h"

namespace mrnnt {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float bf16_lo(unsigned u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf16_hi(unsigned u) { return __uint_as_float(u & 0xffff0000u); }

// tanh(x) = sign(x) (1 - e) / (1 + e), e = exp(-2|x|): v_exp_f32 + v_rcp_f32, |error| ~ 1e-7
__device__ __forceinline__ float fast_tanh(float x) {
    const float e = fast_exp2(-2.0f * kLog2e * fabsf(x));
    return copysignf((1.0f - e) * __builtin_amdgcn_rcpf(1.0f + e), x);
}

// x[c] for a runtime c, as a sum of selects (a select chain gets rewritten into a scratch-indexed load)
template <int N>
__device__ __forceinline__ float pick_n(const float (&x)[N], int c) {
    float r = 0.0f;
#pragma unroll
    for (int i = 0; i < N; ++i) r += (c == i) ? x[i] : 0.0f;
    return r;
}

// ---------------------------------------------------------------------------------------------------------
// row lists: entries (column, s) in column order, s ascending; mode 0 = in-band rows, 1 = live rows

__device__ __forceinline__ bool list_pred(const DevProblem &p, int mode, int t, int s, int64_t row, int W,
                                          double ll) {
    if (mode == 0 || !p.occ_skip) return true;
    return row_live(alpha_prev(p, t, s, row, W) - ll + p.beta[row]);
}

template <bool WRITE>
__global__ __launch_bounds__(256) void row_list_kernel(DevProblem p, int mode, int64_t *__restrict__ cnt,
                                                       int *__restrict__ lcol, int *__restrict__ ls) {
    const int lane = threadIdx.x & 63;
    const int64_t col = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (col >= p.num_cols) return;
    Cursor cur;
    cur.init(p.col_off, p.B, col);
    const int b = cur.b;
    const int T = p.T[b], S = p.S[b], W = S + 1;
    const int t = (int)(col - p.col_off[b]);
    const int64_t rowc = p.row_off[b] + (int64_t)t * W;
    const int lo = max(0, t - (T - S));
    const int hi = min(t, S);
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

// exclusive scan of a[0..n) in place, a[n] = total (one workgroup; n = lattice columns)
__global__ __launch_bounds__(1024) void scan_kernel(int64_t *__restrict__ a, int64_t n,
                                                    unsigned long long *__restrict__ total) {
    __shared__ int64_t part[1024];
    const int tid = threadIdx.x;
    const int64_t seg = (n + 1023) / 1024;
    const int64_t lo = min(n, tid * seg), hi = min(n, lo + seg);
    int64_t loc = 0;
    for (int64_t i = lo; i < hi; ++i) loc += a[i];
    part[tid] = loc;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan
        const int64_t v = tid >= off ? part[tid - off] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    int64_t run = part[tid] - loc;
    for (int64_t i = lo; i < hi; ++i) {
        const int64_t v = a[i];
        a[i] = run;
        run += v;
    }
    if (tid == 1023) {
        a[n] = part[1023];
        if (total) *total = (unsigned long long)part[1023];
    }
}

hipError_t launch_row_list(const DevProblem &p, int mode, int64_t *col_cnt, int *lcol, int *ls,
                           unsigned long long *total, hipStream_t stream) {
    const int64_t blocks = (p.num_cols + 3) / 4;
    row_list_kernel<false><<<(int)blocks, 256, 0, stream>>>(p, mode, col_cnt, lcol, ls);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    scan_kernel<<<1, 1024, 0, stream>>>(col_cnt, p.num_cols, total);
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

__device__ __forceinline__ RowPos row_pos(const DevProblem &p, const JointArgs &j, int64_t i) {
    RowPos q{false, 0, 0, 0, 1, 0, -1, 0};
    if (i >= j.n) return q;
    const int col = j.lcol[i];
    q.s = j.ls[i];
    Cursor c;
    c.init(p.col_off, p.B, col);
    q.b = c.b;
    q.t = (int)(col - p.col_off[q.b]);
    q.T = p.T[q.b];
    q.S = p.S[q.b];
    q.row = p.row_off[q.b] + (int64_t)q.t * (q.S + 1) + q.s;
    q.lab = q.s < q.S ? p.labels[(int64_t)q.b * p.label_stride + q.s] : -1;
    q.valid = true;
    return q;
}

// B operand: h = bf16(tanh(enc[b,t] + pred[b,s])) for k = 16 ks + 8 half + [0, 8); optionally stored to Hact.
// Invalid lanes (past the end of the list) read row 0 and zero the result: no branch around the loads (a
// branch per load makes hipcc wait vmcnt(0) after each one).
template <int KS, bool STORE>
__device__ __forceinline__ void build_act(const JointArgs &j, const RowPos &q, int half, int64_t i,
                                          bf16x8 (&bfr)[KS]) {
    constexpr int H = 16 * KS;
    const bool v = q.valid;
    const unsigned short *er = j.enc + (v ? (int64_t)q.b * j.enc_sb + (int64_t)q.t * H : 0) + 8 * half;
    const unsigned short *pr = j.pred + (v ? (int64_t)q.b * j.pred_sb + (int64_t)q.s * H : 0) + 8 * half;
    const float keep = v ? 1.0f : 0.0f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        const u4 ev = *reinterpret_cast<const u4 *>(er + 16 * ks);
        const u4 pv = *reinterpret_cast<const u4 *>(pr + 16 * ks);
        bf16x8 h;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            h[2 * w] = (__bf16)(keep * fast_tanh(bf16_lo(ev[w]) + bf16_lo(pv[w])));
            h[2 * w + 1] = (__bf16)(keep * fast_tanh(bf16_hi(ev[w]) + bf16_hi(pv[w])));
        }
        if (STORE && v) *reinterpret_cast<bf16x8 *>(j.Hact + i * H + 16 * ks + 8 * half) = h;
        bfr[ks] = h;
    }
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

    // issue the DMA of vocabulary chunk c into wbuf (rows >= V read row V-1; the epilogue masks them)
    __device__ static __forceinline__ void stage(const JointArgs &j, int V, int c, unsigned short *wbuf) {
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
        for (int ii = 0; ii < NI / 4; ++ii) {
            const int i = 4 * ii + wave;
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

__device__ __forceinline__ void wait_dma() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// wait until at most N vector-memory operations of this wave are outstanding (in-order completion): the
// DMA of the chunk after next stays in flight across the barrier
template <int N>
__device__ __forceinline__ void wait_dma_leave() {
    static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// z for the 16 accumulator entries of a lane: + bias, -inf past V. bias_lds holds the whole (padded) bias.
__device__ __forceinline__ void logits(const f32x16 &acc, const float *bias_lds, int c, int half, int V,
                                       float (&z)[16]) {
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
        const int v0 = 32 * c + 8 * q4 + 4 * half;
        const f4 bv = *reinterpret_cast<const f4 *>(bias_lds + v0);
#pragma unroll
        for (int e = 0; e < 4; ++e) z[4 * q4 + e] = acc[4 * q4 + e] + bv[e];
    }
    if (32 * c + 32 > V) {  // only the last chunk can reach past the vocabulary
#pragma unroll
        for (int r = 0; r < 16; ++r)
            if (32 * c + (r & 3) + 8 * (r >> 2) + 4 * half >= V) z[r] = NEG_INF_F;
    }
}

// index of the accumulator register holding vocabulary offset jj (0..31) of a chunk, or -1 if the other lane
// half holds it
__device__ __forceinline__ int acc_reg_of(int jj, int half) {
    return (((jj >> 2) & 1) == half) ? ((jj & 3) + 4 * (jj >> 3)) : -1;
}

// Chunk pipeline shared by both passes: NB LDS buffers; chunk c's MFMAs run beside the epilogue of chunk c-1
// (registers only) while the DMAs of chunks c+1 .. c+NB-1 are in flight; one raw s_barrier per chunk (a
// __syncthreads would drain every DMA with vmcnt(0)).
template <int KS, int NB, class Epi>
__device__ __forceinline__ void chunk_loop(const JointArgs &j, int V, unsigned short *wsh, const bf16x8 (&bfr)[KS],
                                           int lane, Epi &&epi) {
    using WT = WTile<KS>;
    constexpr int NPW = WT::NI / 4;  // DMA instructions per wave per chunk
    const int nch = (V + 31) / 32;
#pragma unroll
    for (int c = 0; c < NB - 1; ++c)
        if (c < nch) WT::stage(j, V, c, wsh + c * WT::ELEMS);
    auto ready = [&](int c) {  // chunk c landed in LDS for every wave
        if (c + NB - 2 < nch) wait_dma_leave<(NB - 2) * NPW>();
        else wait_dma();
        __builtin_amdgcn_s_barrier();
    };
    auto buf = [&](int c) { return wsh + (c % NB) * WT::ELEMS; };
    ready(0);
    if (NB - 1 < nch) WT::stage(j, V, NB - 1, buf(NB - 1));
    f32x16 acc0 = WT::mma(buf(0), bfr, lane), acc1;
    if (nch > 1) ready(1);
    // two chunks per trip so the ping-pong accumulators keep fixed registers
    for (int c = 1;; c += 2) {
        if (c >= nch) {
            epi(acc0, c - 1);
            break;
        }
        if (c + NB - 1 < nch) WT::stage(j, V, c + NB - 1, buf(c + NB - 1));
        acc1 = WT::mma(buf(c), bfr, lane);
        epi(acc0, c - 1);
        if (c + 1 >= nch) {
            epi(acc1, c);
            break;
        }
        ready(c + 1);
        if (c + NB < nch) WT::stage(j, V, c + NB, buf(c + NB));
        acc0 = WT::mma(buf(c + 1), bfr, lane);
        epi(acc1, c);
        if (c + 2 < nch) ready(c + 2);
    }
}

// Simple chunk loop for two workgroups per CU (two waves per SIMD): double-buffered DMA, one accumulator; the
// partner workgroup's MFMAs cover this one's epilogue and activation build.
template <int KS, class Epi>
__device__ __forceinline__ void chunk_loop_simple(const JointArgs &j, int V, unsigned short *wsh,
                                                  const bf16x8 (&bfr)[KS], int lane, Epi &&epi) {
    using WT = WTile<KS>;
    const int nch = (V + 31) / 32;
    WT::stage(j, V, 0, wsh);
    wait_dma();
    __builtin_amdgcn_s_barrier();
    for (int c = 0; c < nch; ++c) {
        if (c + 1 < nch) WT::stage(j, V, c + 1, wsh + ((c + 1) & 1) * WT::ELEMS);
        const f32x16 acc = WT::template mma<2>(wsh + (c & 1) * WT::ELEMS, bfr, lane);
        epi(acc, c);
        wait_dma();
        __builtin_amdgcn_s_barrier();
    }
}

template <int KS, int NB, int OCC, class Epi>
__device__ __forceinline__ void run_chunks(const JointArgs &j, int V, unsigned short *wsh, const bf16x8 (&bfr)[KS],
                                           int lane, Epi &&epi) {
    if constexpr (OCC == 1)
        chunk_loop<KS, NB>(j, V, wsh, bfr, lane, epi);
    else
        chunk_loop_simple<KS>(j, V, wsh, bfr, lane, epi);
}

// LDS: NB W tiles, then the bias padded to whole chunks
template <int KS, int NB>
__device__ __forceinline__ float *load_bias(const JointArgs &j, int V, unsigned short *wsh) {
    float *bl = reinterpret_cast<float *>(wsh + NB * WTile<KS>::ELEMS);
    const int nb = (V + 31) / 32 * 32;
    for (int v = threadIdx.x; v < nb; v += blockDim.x) bl[v] = (v < V && j.bias) ? j.bias[v] : 0.0f;
    return bl;
}

template <int KS, int NB, int OCC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC, OCC))) void joint_fwd_kernel(DevProblem p,
                                                                                          JointArgs j) {
    extern __shared__ __attribute__((aligned(16))) unsigned short wsh[];
    const int lane = threadIdx.x & 63, half = lane >> 5;
    const int64_t i = (int64_t)blockIdx.x * 128 + (threadIdx.x >> 6) * 32 + (lane & 31);
    const RowPos q = row_pos(p, j, i);
    const int V = p.V, blank = p.blank;
    const float *bias = load_bias<KS, NB>(j, V, wsh);
    __syncthreads();
    bf16x8 bfr[KS];
    build_act<KS, false>(j, q, half, i, bfr);

    float m = NEG_INF_F, sum = 0.0f, zb = 0.0f, ze = 0.0f;
    bool fb = false, fe = false;
    run_chunks<KS, NB, OCC>(j, V, wsh, bfr, lane, [&](const f32x16 &acc, int c) {
        float z[16];
        logits(acc, bias, c, half, V, z);
        float cm = z[0];
#pragma unroll
        for (int r = 1; r < 16; ++r) cm = fmaxf(cm, z[r]);
        const float mn = fmaxf(m, cm);
        const float mr = (mn == NEG_INF_F) ? 0.0f : mn;
        float a = sum * fast_exp2((m - mr) * kLog2e);
#pragma unroll
        for (int r = 0; r < 16; ++r) a += fast_exp2((z[r] - mr) * kLog2e);
        sum = a;
        m = mn;
        const int jb = blank - 32 * c;
        if (jb >= 0 && jb < 32) {
            const int rb = acc_reg_of(jb, half);
            if (rb >= 0) {
                zb = pick_n<16>(z, rb);
                fb = true;
            }
        }
        const int jl = q.lab - 32 * c;
        const int rl = acc_reg_of(jl & 31, half);
        if (q.lab >= 0 && jl >= 0 && jl < 32 && rl >= 0) {
            ze = pick_n<16>(z, rl);
            fe = true;
        }
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
        const double den = -(double)mn - log((double)sum);
        p.den[q.row] = (float)den;
        p.lpb[q.row] = (double)zb + den;
        p.lpe[q.row] = (q.lab >= 0 ? (double)ze : 0.0) + den;
    }
}

template <int KS, int NB, int OCC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC, OCC))) void joint_bwd_kernel(DevProblem p,
                                                                                          JointArgs j) {
    extern __shared__ __attribute__((aligned(16))) unsigned short wsh[];
    const int lane = threadIdx.x & 63, half = lane >> 5;
    const int64_t i = (int64_t)blockIdx.x * 128 + (threadIdx.x >> 6) * 32 + (lane & 31);
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

    const bool vec_out = (V & 3) == 0;
    unsigned short *grow = j.G + (q.valid ? i : 0) * V;
    run_chunks<KS, NB, OCC>(j, V, wsh, bfr, lane, [&](const f32x16 &acc, int c) {
        float z[16];
        logits(acc, bias, c, half, V, z);
        float g[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int v = 32 * c + (r & 3) + 8 * (r >> 2) + 4 * half;
            float x = fast_exp2(fmaf(z[r], kLog2e, rc.c2));
            x -= (v == blank ? rc.cb : 0.0f) + (v == rc.lab ? rc.ce : 0.0f);
            g[r] = x * sc;
        }
        if (q.valid) {
#pragma unroll
            for (int qd = 0; qd < 4; ++qd) {
                const int v0 = 32 * c + 8 * qd + 4 * half;
                if (vec_out && v0 + 3 < V) {
                    const unsigned lo = IoBF16::pack2(g[4 * qd], g[4 * qd + 1]);
                    const unsigned hi = IoBF16::pack2(g[4 * qd + 2], g[4 * qd + 3]);
                    *reinterpret_cast<uint2 *>(grow + v0) = make_uint2(lo, hi);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (v0 + e < V) grow[v0 + e] = IoBF16::from_f(g[4 * qd + e]);
                }
            }
        }
    });
}

// ---------------------------------------------------------------------------------------------------------
// backward tail: dpre = dH * (1 - Hact^2) over the live rows, summed into denc[b, t] (over s; written once per
// column) and dpred[b, s] (over t; accumulated in LDS over a block of TT columns, then one fp32 atomic per
// (s, h) per block). One workgroup per (utterance, block of TT frames, slice of HS hidden units); 4 hidden
// units per thread (8-byte loads), 256/(HS/4) rows in flight.

constexpr int kReduceTT = 64;

template <int HS>
__global__ __launch_bounds__(256) void joint_reduce_kernel(DevProblem p, JointArgs j, const int64_t *__restrict__ off,
                                                           const unsigned short *__restrict__ dH,
                                                           float *__restrict__ d_enc, float *__restrict__ d_pred,
                                                           int ntb) {
    constexpr int TPR = HS / 4;     // threads per row slice
    constexpr int RP = 256 / TPR;   // rows in parallel
    extern __shared__ float lds[];  // acc[(S_b+1) * HS] then red[RP][HS]
    const int H = j.H;
    const int nh = H / HS;
    // the h-slices of one block of frames are consecutive workgroups: they read the same rows (L2 reuse)
    const int bx = blockIdx.x / nh;
    const int h0 = (blockIdx.x % nh) * HS;
    const int b = bx / ntb;
    const int t0 = (bx % ntb) * kReduceTT;
    const int T = p.T[b], S = p.S[b];
    if (t0 >= T) return;
    const int tid = threadIdx.x;
    const int hl = (tid % TPR) * 4, rsub = tid / TPR;
    float *acc = lds;
    float *red = lds + (S + 1) * HS;
    for (int i = tid; i < (S + 1) * HS; i += 256) acc[i] = 0.0f;
    __syncthreads();
    const int64_t tslots = j.enc_sb / H, sslots = j.pred_sb / H;
    const int t1 = min(t0 + kReduceTT, T);
    for (int t = t0; t < t1; ++t) {
        const int64_t col = p.col_off[b] + t;
        const int64_t r0 = off[col], r1 = off[col + 1];
        float e0 = 0.0f, e1 = 0.0f, e2 = 0.0f, e3 = 0.0f;
        for (int64_t r = r0 + rsub; r < r1; r += RP) {
            const int s = j.ls[r];
            const uint2 dv = *reinterpret_cast<const uint2 *>(dH + r * H + h0 + hl);
            const uint2 hv = *reinterpret_cast<const uint2 *>(j.Hact + r * H + h0 + hl);
            const float h_0 = bf16_lo(hv.x), h_1 = bf16_hi(hv.x), h_2 = bf16_lo(hv.y), h_3 = bf16_hi(hv.y);
            const float v0 = bf16_lo(dv.x) * (1.0f - h_0 * h_0), v1 = bf16_hi(dv.x) * (1.0f - h_1 * h_1);
            const float v2 = bf16_lo(dv.y) * (1.0f - h_2 * h_2), v3 = bf16_hi(dv.y) * (1.0f - h_3 * h_3);
            e0 += v0;
            e1 += v1;
            e2 += v2;
            e3 += v3;
            float *a = acc + s * HS + hl;  // distinct s within a column: one writer per element
            a[0] += v0;
            a[1] += v1;
            a[2] += v2;
            a[3] += v3;
        }
        float *rr = red + rsub * HS + hl;
        rr[0] = e0;
        rr[1] = e1;
        rr[2] = e2;
        rr[3] = e3;
        __syncthreads();
        if (tid < HS) {
            float sum = 0.0f;
#pragma unroll 4
            for (int g = 0; g < RP; ++g) sum += red[g * HS + tid];
            d_enc[((int64_t)b * tslots + t) * H + h0 + tid] = sum;
        }
        __syncthreads();
    }
    for (int i = tid; i < (S + 1) * HS; i += 256) {
        const float v = acc[i];
        if (v != 0.0f) atomicAdd(&d_pred[((int64_t)b * sslots + i / HS) * H + h0 + i % HS], v);
    }
}

hipError_t launch_joint_reduce(const DevProblem &p, const JointArgs &j, const int64_t *off, int T_max, int S_max,
                               const unsigned short *dH, float *d_enc, float *d_pred, hipStream_t stream) {
    const int ntb = (T_max + kReduceTT - 1) / kReduceTT;
    const int W = S_max + 1;
    auto go = [&](auto hs_tag) {
        constexpr int HS = decltype(hs_tag)::value;
        const size_t lds = sizeof(float) * ((size_t)W * HS + 256 / (HS / 4) * HS);
        joint_reduce_kernel<HS><<<p.B * ntb * (j.H / HS), 256, lds, stream>>>(p, j, off, dH, d_enc, d_pred, ntb);
    };
    // LDS = W * HS + 4 KiB of fp32: about 30 KiB at the headline (several workgroups per CU), <= 64 KiB always
    if (W <= 448) go(std::integral_constant<int, 32>());
    else if (W <= 896) go(std::integral_constant<int, 16>());
    else if (W <= 1792) go(std::integral_constant<int, 8>());
    else go(std::integral_constant<int, 4>());
    return hipGetLastError();
}

template <int KS, int NB, int OCC>
static hipError_t launch_knb(const DevProblem &p, const JointArgs &j, bool bwd, size_t lds, hipStream_t stream) {
    const int64_t blocks = (j.n + 127) / 128;
    auto kern = bwd ? joint_bwd_kernel<KS, NB, OCC> : joint_fwd_kernel<KS, NB, OCC>;
    if (lds > 65536) {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    kern<<<(int)blocks, 256, lds, stream>>>(p, j);
    return hipGetLastError();
}

// joint_variant 0: one workgroup per CU, ping-pong accumulators, three LDS buffers when they fit (else two);
// joint_variant 1: two workgroups per CU (256 registers per lane), double-buffered simple loop
template <int KS>
static hipError_t launch_kh(const DevProblem &p, const JointArgs &j, bool bwd, hipStream_t stream) {
    const size_t bias = sizeof(float) * ((p.V + 31) / 32 * 32);
    const size_t tile = sizeof(unsigned short) * WTile<KS>::ELEMS;
    if (tuning().joint_variant == 1 && 2 * (2 * tile + bias) <= 160 * 1024)
        return launch_knb<KS, 2, 2>(p, j, bwd, 2 * tile + bias, stream);
    if (3 * tile + bias <= 160 * 1024) return launch_knb<KS, 3, 1>(p, j, bwd, 3 * tile + bias, stream);
    if (2 * tile + bias <= 160 * 1024) return launch_knb<KS, 2, 1>(p, j, bwd, 2 * tile + bias, stream);
    return hipErrorInvalidValue;
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

hipError_t launch_joint_forward(const DevProblem &p, const JointArgs &j, hipStream_t stream) {
    return launch_joint(p, j, false, stream);
}

hipError_t launch_joint_backward(const DevProblem &p, const JointArgs &j, hipStream_t stream) {
    return launch_joint(p, j, true, stream);
}

}  // namespace mrnnt
