// mrnnt_joint_gemm.hip -- the fused joint network's backward GEMMs on hand-written MFMA tiles:
//
//   dpre[r, h] = (sum_v G[r, v] W[v, h]) * (1 - Hact[r, h]^2)      r < n_live, h < H          (joint_dpre_kernel)
//
// i.e. dH = G W (the gradient of the joint activations) with the tanh derivative applied in the epilogue, so the
// d_enc / d_pred reduce reads one [n, H] tensor instead of dH and Hact (mrnnt_joint_reduce with Hact = NULL). G is
// the bf16 logit gradient of the live rows (mrnnt_joint_backward), W the [V, H] weight, given transposed ([H, V],
// k = v contiguous in both operands).
//
// Tile: a workgroup of 4 waves (one per SIMD, 512 registers each) owns 256 rows x 256 hidden units; wave w computes
// 128 h x 128 r as 4 x 4 v_mfma_f32_32x32x16_bf16 tiles (256 accumulator registers): A = W^T rows (h), B = G rows (r),
// so the accumulator of a lane holds 16 hidden units of ONE row -- four runs of 4 consecutive h, one 8-byte Hact
// load and one 8-byte dpre store each. K (= V) streams through LDS in chunks of 32 by LDS-DMA (buffer_load ... lds:
// no staging registers), 4 stages deep, each stage one [256][32] image of G and one of W^T with the 16-byte piece p of
// row r stored at piece p ^ ((r >> 2) & 3): the 16 lanes of each ds_read_b128 group land on 16 distinct bank quads.
// The two h-halves of a row tile (H = 512) run as blocks b and b + 8 -- on the same XCD, dispatched together -- so
// the second reads G from that XCD's L2.
#include <algorithm>

#include "mrnnt_device.h"

namespace mrnnt {

typedef __bf16 gbf16x8 __attribute__((ext_vector_type(8)));
typedef float gf32x16 __attribute__((ext_vector_type(16)));
typedef float gf32x4 __attribute__((ext_vector_type(4)));

constexpr int kGT = 256;          // rows and hidden units per workgroup tile
constexpr int kGKC = 32;          // k per LDS stage
constexpr int kGImage = kGT * kGKC * 2;              // bytes of one [256][32] bf16 image (16 KiB)

__device__ __forceinline__ float bf16_lo_f(unsigned u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf16_hi_f(unsigned u) { return __uint_as_float(u & 0xffff0000u); }

__device__ __forceinline__ int gimg_off(int r, int p) { return r * 64 + ((p ^ ((r >> 2) & 3)) << 4); }

// one LDS-DMA piece: 16 bytes per lane from the buffer into LDS at dst + 16 lane (a plain __device__ function: the
// address-space cast in a kernel template's body makes clang drop the template's host-side instantiation)
__device__ __forceinline__ void gemm_dma(__amdgpu_buffer_rsrc_t rs, unsigned char *dst, unsigned voff, unsigned soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void *)dst, 16, voff, soff, 0, 0);
}

// The workgroup barrier of the chunk loops: LDS reads of this wave retired (the stage refilled after the barrier is
// the one every wave read in the previous chunk), then a raw s_barrier. __syncthreads() would also wait vmcnt(0) --
// its fence covers the LDS-DMA still in flight -- and drain the stages staged ahead at every chunk.
__device__ __forceinline__ void gemm_barrier() {
    __builtin_amdgcn_s_waitcnt(15 | (7 << 4) | (0 << 8) | (3 << 14));  // lgkmcnt(0), vmcnt / expcnt untouched
    __builtin_amdgcn_s_barrier();
}

// wait until at most N vector-memory operations of this wave are outstanding (issue order = completion order)
template <int N>
__device__ __forceinline__ void gemm_wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// Both operands through LDS (LDS-DMA), NS stages of 32 k. NW waves; wave w computes 128 h (w & 1) x 32 RT rows
// (w >> 1), so a workgroup tile is TR = 16 NW RT rows x 256 h. NW = 8, RT = 2: two waves per SIMD, 256 rows;
// NW = 4, RT = 4: one wave per SIMD, 256 rows; NW = 4, RT = 2, NS = 3: 128 rows in 72 KiB of LDS and 256 registers,
// so two workgroups share a CU and one's epilogue runs beside the other's MFMAs (WPE = waves per SIMD the register
// budget allows). The fragments, their k order and every accumulation are the same in all: bit-identical results.
template <int NW, int RT, int NS, int WPE, int EPI>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void joint_dpre_kernel(
    const unsigned short *__restrict__ G, const unsigned short *__restrict__ Wt, const unsigned short *__restrict__ Hact,
    int64_t hact_ld, unsigned short *__restrict__ dpre, int64_t n, int V, int H, int abl) {
    constexpr int TR = 16 * NW * RT;           // rows per tile
    constexpr int GI = TR * kGKC * 2;          // G image bytes per stage
    constexpr int WI = kGImage;                // W^T image bytes per stage (256 h)
    constexpr int SB = GI + WI;
    constexpr int DG = GI / 1024 / NW;         // LDS-DMA wave-instructions per stage per wave: G, W^T
    constexpr int DW = WI / 1024 / NW;
    static_assert(DG >= 1 && DW >= 1 && NS >= 2, "tile shape");
    extern __shared__ __attribute__((aligned(16))) unsigned char glds[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // XCD-aware tile order: blocks are dispatched round-robin over the 8 XCDs, so b and b + 8 share an XCD
    const int nh = H / kGT;
    const int64_t b = blockIdx.x;
    const int64_t xcd = b & 7, j = b >> 3;
    const int hh = (int)(j % nh);
    const int64_t rt = (j / nh) * 8 + xcd;
    const int64_t r0 = rt * TR;
    if (r0 >= n) return;
    const int h0 = hh * kGT;
    const int rows = (int)min<int64_t>(TR, n - r0);
    if ((abl & 4) && b >= 256 && b < 512) {  // development: the second workgroup of each CU starts ~half a tile late
        for (int i = 0; i < 2; ++i) __builtin_amdgcn_s_sleep(127);
    }
    // buffer resources over this tile's rows of G (rows past n read as zero) and of W^T
    // development ablation (joint_dpre_abl bit 1): every tile reads the G rows of row tile xcd (L2-resident)
    const int64_t rg0 = (abl & 2) ? (int64_t)xcd * TR : r0;
    const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<unsigned short *>(G) + rg0 * V, (short)0, rows * V * 2, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<unsigned short *>(Wt) + (int64_t)h0 * V, (short)0, kGT * V * 2, 0x00020000);
    auto src_off = [&](int piece16) {  // 16-row piece of an image -> this lane's source offset (swizzle on the source)
        const int row = 16 * piece16 + (lane >> 2);
        const int p = (lane & 3) ^ ((row >> 2) & 3);
        return (unsigned)(row * V + 8 * p) * 2u;
    };
    unsigned goff[DG], woff[DW];
#pragma unroll
    for (int i = 0; i < DG; ++i) goff[i] = src_off(DG * wave + i);
#pragma unroll
    for (int i = 0; i < DW; ++i) woff[i] = src_off(DW * wave + i);
    const int nch = (V + kGKC - 1) / kGKC;
    auto stage = [&](int c) {
        unsigned char *s = glds + (c % NS) * SB;
#pragma unroll
        for (int i = 0; i < DG; ++i) gemm_dma(rg, s + 1024 * (DG * wave + i), goff[i] + (unsigned)(c * kGKC * 2), 0u);
#pragma unroll
        for (int i = 0; i < DW; ++i) gemm_dma(rw, s + GI + 1024 * (DW * wave + i), woff[i] + (unsigned)(c * kGKC * 2), 0u);
    };
#pragma unroll
    for (int c = 0; c < NS - 1; ++c)
        if (c < nch) stage(c);

    const int wh = wave & 1, wr = wave >> 1;  // this wave: h 128 wh .. +128, rows 32 RT wr .. +32 RT of the tile
    const int l32 = lane & 31, half = lane >> 5;
    gf32x16 acc[4][RT];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int q = 0; q < RT; ++q)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[a][q][e] = 0.0f;

    for (int c = 0; c < nch; ++c) {
        // chunk c landed for this wave (the chunks staged after it stay in flight), then for every wave
        constexpr int kPer = DG + DW;
        const int later = min(NS - 2, nch - 1 - c);
        if (later >= 3) gemm_wait_vm<(NS - 2 >= 3 ? 3 : 0) * kPer>();
        else if (later == 2) gemm_wait_vm<2 * kPer>();
        else if (later == 1) gemm_wait_vm<kPer>();
        else gemm_wait_vm<0>();
        gemm_barrier();
        if (c + NS - 1 < nch) stage(c + NS - 1);  // into the stage every wave finished with at c - 1
        const unsigned char *s = glds + (c % NS) * SB;
        const unsigned char *gi = s, *wi = s + GI;
        const bool tail = (c + 1) * kGKC > V;  // k past V in this chunk: those fragments are zeroed (both operands)
#pragma unroll
        for (int ks = 0; ks < kGKC / 16; ++ks) {
            const int p = 2 * ks + half;
            gbf16x8 fa[4], fb[RT];
#pragma unroll
            for (int t = 0; t < 4; ++t)
                fa[t] = *reinterpret_cast<const gbf16x8 *>(wi + gimg_off(128 * wh + 32 * t + l32, p));
#pragma unroll
            for (int t = 0; t < RT; ++t)
                fb[t] = *reinterpret_cast<const gbf16x8 *>(gi + gimg_off(32 * RT * wr + 32 * t + l32, p));
            if (tail && c * kGKC + 8 * p >= V) {
#pragma unroll
                for (int t = 0; t < 4; ++t) fa[t] = (gbf16x8){};
#pragma unroll
                for (int t = 0; t < RT; ++t) fb[t] = (gbf16x8){};
            }
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int q = 0; q < RT; ++q)
                    acc[a][q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[a], fb[q], acc[a][q], 0, 0, 0);
        }
    }

    if constexpr (EPI == 2) {
        // development: plain dH (no tanh derivative, no Hact read) through the LDS-staged copy-out
        constexpr int EI = TR / 2 / NW;
        gemm_barrier();
#pragma unroll
        for (int q = 0; q < RT; ++q) {
            const int row = 32 * RT * wr + 32 * q + l32;
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int U = 16 * wh + 4 * a + g;
                    *reinterpret_cast<uint2 *>(glds + row * 512 + ((U ^ (row & 15)) << 4) + half * 8) =
                        make_uint2(IoBF16::pack2(acc[a][q][4 * g], acc[a][q][4 * g + 1]),
                                   IoBF16::pack2(acc[a][q][4 * g + 2], acc[a][q][4 * g + 3]));
                }
        }
        gemm_barrier();
#pragma unroll
        for (int i = 0; i < EI; ++i) {
            const int row = 2 * (EI * wave + i) + (lane >> 5);
            const uint4 v = *reinterpret_cast<const uint4 *>(glds + 1024 * (EI * wave + i) + 16 * lane);
            if (row < rows)
                *reinterpret_cast<uint4 *>(dpre + (r0 + row) * H + h0 + 8 * ((lane & 31) ^ (row & 15))) = v;
        }
        return;
    }
    if constexpr (EPI == 1) {
        // The epilogue through LDS (the stages are free once every wave is past its last chunk): the tile's Hact rows
        // land by LDS-DMA, 2 rows of 256 h per wave-instruction, the 16-byte unit u of row r stored at slot
        // u ^ (r & 15); each lane turns its own 8-byte Hact pieces into dpre in place (a lane reads and writes only
        // its pieces); then every wave copies 2 whole rows per 16-byte-per-lane store.
        static_assert(TR * kGT * 2 <= NS * SB, "the Hact tile fits the stages");
        constexpr int EI = TR / 2 / NW;  // 1 KiB pieces per wave
        gemm_barrier();
        const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<unsigned short *>(Hact) + r0 * hact_ld, (short)0, (int)(rows * hact_ld * 2), 0x00020000);
#pragma unroll
        for (int i = 0; i < EI; ++i) {
            const int row = 2 * (EI * wave + i) + (lane >> 5);
            const int u = (lane & 31) ^ (row & 15);
            gemm_dma(rh, glds + 1024 * (EI * wave + i), (unsigned)(row * hact_ld + h0 + 8 * u) * 2u, 0u);
        }
        gemm_wait_vm<0>();
        gemm_barrier();
#pragma unroll
        for (int q = 0; q < RT; ++q) {
            const int row = 32 * RT * wr + 32 * q + l32;
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int U = 16 * wh + 4 * a + g;
                    uint2 *pp = reinterpret_cast<uint2 *>(glds + row * 512 + ((U ^ (row & 15)) << 4) + half * 8);
                    const uint2 hv = *pp;
                    const float h0v = bf16_lo_f(hv.x), h1v = bf16_hi_f(hv.x);
                    const float h2v = bf16_lo_f(hv.y), h3v = bf16_hi_f(hv.y);
                    const float d0 = acc[a][q][4 * g] * (1.0f - h0v * h0v), d1 = acc[a][q][4 * g + 1] * (1.0f - h1v * h1v);
                    const float d2 = acc[a][q][4 * g + 2] * (1.0f - h2v * h2v);
                    const float d3 = acc[a][q][4 * g + 3] * (1.0f - h3v * h3v);
                    *pp = make_uint2(IoBF16::pack2(d0, d1), IoBF16::pack2(d2, d3));
                }
        }
        gemm_barrier();
#pragma unroll
        for (int i = 0; i < EI; ++i) {
            const int row = 2 * (EI * wave + i) + (lane >> 5);
            const uint4 v = *reinterpret_cast<const uint4 *>(glds + 1024 * (EI * wave + i) + 16 * lane);
            if (row < rows)
                *reinterpret_cast<uint4 *>(dpre + (r0 + row) * H + h0 + 8 * ((lane & 31) ^ (row & 15))) = v;
        }
        return;
    }
    if (abl & 1) {  // development ablation (joint_dpre_abl bit 0): no epilogue, the accumulators kept live
        float sum = 0.0f;
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int q = 0; q < RT; ++q)
#pragma unroll
                for (int e = 0; e < 16; ++e) sum += acc[a][q][e];
        if (sum == 1.25e30f) dpre[r0 * H] = 1;
        return;
    }
    // epilogue: lane (l32, half) holds row r = r0 + 32 RT wr + 32 q + l32 and, in register 4 g + e of tile (a, q),
    // hidden unit h = h0 + 128 wh + 32 a + 8 g + 4 half + e
#pragma unroll
    for (int q = 0; q < RT; ++q) {
        const int rr = 32 * RT * wr + 32 * q + l32;
        if (rr >= rows) continue;
        const int64_t r = r0 + rr;
        const unsigned short *hrow = Hact + r * hact_ld;
        unsigned short *orow = dpre + r * H;
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int h = h0 + 128 * wh + 32 * a + 8 * g + 4 * half;
                const uint2 hv = *reinterpret_cast<const uint2 *>(hrow + h);
                const float h0v = bf16_lo_f(hv.x), h1v = bf16_hi_f(hv.x), h2v = bf16_lo_f(hv.y), h3v = bf16_hi_f(hv.y);
                const float d0 = acc[a][q][4 * g] * (1.0f - h0v * h0v), d1 = acc[a][q][4 * g + 1] * (1.0f - h1v * h1v);
                const float d2 = acc[a][q][4 * g + 2] * (1.0f - h2v * h2v), d3 = acc[a][q][4 * g + 3] * (1.0f - h3v * h3v);
                *reinterpret_cast<uint2 *>(orow + h) = make_uint2(IoBF16::pack2(d0, d1), IoBF16::pack2(d2, d3));
            }
    }
}

// The 16x16x32 form (joint_dpre_nw = 16x): v_mfma_f32_16x16x32_bf16 (the shape that holds the clock better on random
// operands), both operands through LDS by LDS-DMA in NS stages of 32 k, tile 256 rows x 256 h, 8 waves (two per SIMD)
// of 64 rows x 128 h: per chunk a wave issues 12 ds_read_b128 (8 W^T + 4 G fragments) and 32 MFMAs. A chunk's
// fragments are read one chunk ahead: the wait and barrier of chunk c retire chunk c + 1's DMA, so the reads of c + 1
// go out beside the MFMAs of c and the MFMA stream does not stop at the barrier for an LDS round trip. The image of
// a 32-k chunk holds row r's 16-byte piece p at slot p ^ (3 ((r >> 3) & 1)): the 16 lanes of every ds_read_b128 group
// (rows l & 15, pieces l >> 4) land on 16 distinct bank quads. PRIO: s_setprio 1 around each MFMA cluster.
__device__ __forceinline__ int k16_swz(int row) { return 3 * ((row >> 3) & 1); }

template <int NS, bool PRIO, bool IL, bool HP>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void joint_dpre_k16_kernel(
    const unsigned short *__restrict__ G, const unsigned short *__restrict__ Wt, const unsigned short *__restrict__ Hact,
    int64_t hact_ld, unsigned short *__restrict__ dpre, int64_t n, int V, int H) {
    constexpr int NW = 8, TR = kGT;
    constexpr int GI = TR * kGKC * 2, WI = kGT * kGKC * 2, SB = GI + WI;  // 16 + 16 KiB per stage
    constexpr int DG = GI / 1024 / NW, DW = WI / 1024 / NW;              // 2 + 2 DMA wave-instructions per stage
    static_assert(NS >= 4 && TR * kGT * 2 <= NS * SB, "the Hact tile of the epilogue fits the stages");
    static_assert(!HP || NS == 4, "the Hact prefetch maps its four quarters onto the four stage slots");
    extern __shared__ __attribute__((aligned(16))) unsigned char glds[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nh = H / kGT;
    const int64_t b = blockIdx.x;
    const int64_t xcd = b & 7, j = b >> 3;
    const int hh = (int)(j % nh);
    const int64_t r0 = ((j / nh) * 8 + xcd) * TR;
    if (r0 >= n) return;
    const int h0 = hh * kGT;
    const int rows = (int)min<int64_t>(TR, n - r0);
    const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<unsigned short *>(G) + r0 * V, (short)0, rows * V * 2, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<unsigned short *>(Wt) + (int64_t)h0 * V, (short)0, kGT * V * 2, 0x00020000);
    auto src_off = [&](int piece16) {
        const int row = 16 * piece16 + (lane >> 2);
        return (unsigned)(row * V + 8 * ((lane & 3) ^ k16_swz(row))) * 2u;
    };
    unsigned goff[DG], woff[DW];
#pragma unroll
    for (int i = 0; i < DG; ++i) goff[i] = src_off(DG * wave + i);
#pragma unroll
    for (int i = 0; i < DW; ++i) woff[i] = src_off(DW * wave + i);
    const int nch = (V + kGKC - 1) / kGKC;
    auto stage = [&](int c) {
        unsigned char *st = glds + (c % NS) * SB;
#pragma unroll
        for (int i = 0; i < DG; ++i) gemm_dma(rg, st + 1024 * (DG * wave + i), goff[i] + (unsigned)(c * kGKC * 2), 0u);
#pragma unroll
        for (int i = 0; i < DW; ++i) gemm_dma(rw, st + GI + 1024 * (DW * wave + i), woff[i] + (unsigned)(c * kGKC * 2), 0u);
    };
    constexpr int kPer = DG + DW;
    // wait until chunk `want` of this wave landed, given chunks up to `issued` were staged (in order)
    auto wait_chunk = [&](int want, int issued) {
        const int later = min(issued, nch - 1) - want;
        if (later >= 3) gemm_wait_vm<3 * kPer>();
        else if (later == 2) gemm_wait_vm<2 * kPer>();
        else if (later == 1) gemm_wait_vm<kPer>();
        else gemm_wait_vm<0>();
    };
    const int wh = wave & 1, wr = wave >> 1;  // this wave: h 128 wh .. +128, rows 64 wr .. +64 of the tile
    const int l16 = lane & 15, pc = lane >> 4;
    // fragment offsets inside an image: row 16 t + l16 (t = tile), piece pc; the swizzle depends on l16 alone
    const int foff = l16 * 64 + ((pc ^ k16_swz(l16)) << 4);
    const int aoff = GI + (128 * wh) * 64 + foff;  // W^T rows 128 wh + 16 a + l16: + 1024 a
    const int boff = (64 * wr) * 64 + foff;        // G rows 64 wr + 16 q + l16: + 1024 q
    const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<unsigned short *>(Hact) + r0 * hact_ld, (short)0, (int)(rows * hact_ld * 2), 0x00020000);
    // one 1 KiB piece (2 rows of 256 h) of the epilogue's Hact image: the 16-byte unit u of row r at slot u ^ (r & 15)
    auto hact_piece = [&](int P) {
        const int row = 2 * P + (lane >> 5);
        const int u = (lane & 31) ^ (row & 15);
        gemm_dma(rh, glds + 1024 * P, (unsigned)(row * hact_ld + h0 + 8 * u) * 2u, 0u);
    };
    // HP: the Hact image is staged during the last three chunks, quarter Q (64 rows, 32 KiB) into stage slot Q as
    // soon as that slot's chunk is in registers: two quarters at chunk nch - 3, one at each of the last two
    const bool hp = HP && nch >= NS;
    gf32x4 acc[8][4];
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[a][q] = (gf32x4){0.0f, 0.0f, 0.0f, 0.0f};
    auto read_frags = [&](int c, gbf16x8 (&fa)[8], gbf16x8 (&fb)[4]) {
        const unsigned char *st = glds + (c % NS) * SB;
#pragma unroll
        for (int q = 0; q < 4; ++q) fb[q] = *reinterpret_cast<const gbf16x8 *>(st + boff + 1024 * q);
#pragma unroll
        for (int a = 0; a < 8; ++a) fa[a] = *reinterpret_cast<const gbf16x8 *>(st + aoff + 1024 * a);
    };
    auto mma = [&](int c, gbf16x8 (&fa)[8], gbf16x8 (&fb)[4]) {
        if ((c + 1) * kGKC > V && c * kGKC + 8 * pc >= V) {  // k past V: zero both operands
#pragma unroll
            for (int a = 0; a < 8; ++a) fa[a] = (gbf16x8){};
#pragma unroll
            for (int q = 0; q < 4; ++q) fb[q] = (gbf16x8){};
        }
        if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int a = 0; a < 8; ++a)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[a][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[a], fb[q], acc[a][q], 0, 0, 0);
        if (PRIO) __builtin_amdgcn_s_setprio(0);
    };
#pragma unroll
    for (int c = 0; c < NS - 1; ++c)
        if (c < nch) stage(c);
    wait_chunk(0, NS - 2);
    gemm_barrier();
    gbf16x8 fa0[8], fb0[4], fa1[8], fb1[4];
    read_frags(0, fa0, fb0);
    // iteration c: chunk c + 1 retired and visible (wait + barrier), chunk c + NS - 1 staged into the slot read last
    // at c - 1, chunk c + 1's fragments read, chunk c's MFMAs
    // IL: the chunk's 4 DMA pieces and 12 fragment reads issued between its 4 groups of 8 MFMAs (an LDS-DMA issue
    // costs ~60-185 cycles of the issuing wave; issued together after the barrier, both waves of a SIMD stall there)
    auto step = [&](int c, gbf16x8 (&fa)[8], gbf16x8 (&fb)[4], gbf16x8 (&na)[8], gbf16x8 (&nb)[4]) {
        if (c + 1 < nch) {
            if (hp && c == nch - 2) gemm_wait_vm<8>();  // chunk nch - 1; the two Hact quarters issued after it fly on
            else wait_chunk(c + 1, c + NS - 2);
        }
        gemm_barrier();
        if constexpr (!IL) {
            if (c + NS - 1 < nch) stage(c + NS - 1);
            if (c + 1 < nch) read_frags(c + 1, na, nb);
            mma(c, fa, fb);
        } else {
            const bool st = c + NS - 1 < nch, rd = c + 1 < nch;
            unsigned char *sd = glds + ((c + NS - 1) % NS) * SB;
            const unsigned char *sr = glds + ((c + 1) % NS) * SB;
            const unsigned ko = (unsigned)((c + NS - 1) * kGKC * 2);
            if ((c + 1) * kGKC > V && c * kGKC + 8 * pc >= V) {  // k past V: zero both operands
#pragma unroll
                for (int a = 0; a < 8; ++a) fa[a] = (gbf16x8){};
#pragma unroll
                for (int q = 0; q < 4; ++q) fb[q] = (gbf16x8){};
            }
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
                for (int a = 2 * g; a < 2 * g + 2; ++a)
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        acc[a][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[a], fb[q], acc[a][q], 0, 0, 0);
                if (PRIO) __builtin_amdgcn_s_setprio(0);
                __builtin_amdgcn_sched_barrier(0);
                if (st) {
                    if (g < 2) gemm_dma(rg, sd + 1024 * (DG * wave + g), goff[g] + ko, 0u);
                    else gemm_dma(rw, sd + GI + 1024 * (DW * wave + g - 2), woff[g - 2] + ko, 0u);
                } else if (hp && c >= nch - 3) {
                    // quarter Q = slot: pieces 32 Q + 4 wave + i of the image
                    if (c == nch - 3) {
                        hact_piece(32 * ((c - 1) % NS) + 4 * wave + g);
                        hact_piece(32 * (c % NS) + 4 * wave + g);
                    } else {
                        hact_piece(32 * (c % NS) + 4 * wave + g);
                    }
                }
                if (rd) {
                    if (g == 0) {
#pragma unroll
                        for (int q = 0; q < 3; ++q) nb[q] = *reinterpret_cast<const gbf16x8 *>(sr + boff + 1024 * q);
                    } else if (g == 1) {
                        nb[3] = *reinterpret_cast<const gbf16x8 *>(sr + boff + 3072);
                        na[0] = *reinterpret_cast<const gbf16x8 *>(sr + aoff);
                        na[1] = *reinterpret_cast<const gbf16x8 *>(sr + aoff + 1024);
                    } else {
#pragma unroll
                        for (int a = 3 * g - 4; a < 3 * g - 1; ++a)
                            na[a] = *reinterpret_cast<const gbf16x8 *>(sr + aoff + 1024 * a);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    };
    int c = 0;
    for (; c + 1 < nch; c += 2) {
        step(c, fa0, fb0, fa1, fb1);
        step(c + 1, fa1, fb1, fa0, fb0);
    }
    if (c < nch) step(c, fa0, fb0, fa1, fb1);

    // epilogue through LDS, as joint_dpre_kernel's EPI = 1: lane (l16, pc) holds row 64 wr + 16 q + l16 and, in
    // register e of tile (a, q), hidden unit 128 wh + 16 a + 4 pc + e
    constexpr int EI = TR / 2 / NW;
    gemm_barrier();
    if (!hp) {
#pragma unroll
        for (int i = 0; i < EI; ++i) hact_piece(EI * wave + i);
    }
    gemm_wait_vm<0>();
    gemm_barrier();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int row = 64 * wr + 16 * q + l16;
#pragma unroll
        for (int a = 0; a < 8; ++a) {
            const int U = 16 * wh + 2 * a + (pc >> 1);
            uint2 *pp = reinterpret_cast<uint2 *>(glds + row * 512 + ((U ^ (row & 15)) << 4) + (pc & 1) * 8);
            const uint2 hv = *pp;
            const float h0v = bf16_lo_f(hv.x), h1v = bf16_hi_f(hv.x), h2v = bf16_lo_f(hv.y), h3v = bf16_hi_f(hv.y);
            const float d0 = acc[a][q][0] * (1.0f - h0v * h0v), d1 = acc[a][q][1] * (1.0f - h1v * h1v);
            const float d2 = acc[a][q][2] * (1.0f - h2v * h2v), d3 = acc[a][q][3] * (1.0f - h3v * h3v);
            *pp = make_uint2(IoBF16::pack2(d0, d1), IoBF16::pack2(d2, d3));
        }
    }
    gemm_barrier();
#pragma unroll
    for (int i = 0; i < EI; ++i) {
        const int row = 2 * (EI * wave + i) + (lane >> 5);
        const uint4 v = *reinterpret_cast<const uint4 *>(glds + 1024 * (EI * wave + i) + 16 * lane);
        if (row < rows) *reinterpret_cast<uint4 *>(dpre + (r0 + row) * H + h0 + 8 * ((lane & 31) ^ (row & 15))) = v;
    }
}

template <int NS, bool PRIO, bool IL, bool HP = false>
static hipError_t launch_dpre_k16(const unsigned short *G, const unsigned short *Wt, const unsigned short *Hact,
                                  int64_t hact_ld, unsigned short *dpre, int64_t n, int V, int H, hipStream_t stream) {
    const size_t lds = (size_t)NS * 2 * kGT * kGKC * 2;
    const int64_t rtiles = (n + kGT - 1) / kGT;
    const int64_t blocks = ((rtiles + 7) / 8) * 8 * (H / kGT);
    if (blocks > 0x7fffffff / 512) return hipErrorInvalidValue;
    auto kern = joint_dpre_k16_kernel<NS, PRIO, IL, HP>;
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    kern<<<(unsigned)blocks, 512, lds, stream>>>(G, Wt, Hact, hact_ld, dpre, n, V, H);
    return hipGetLastError();
}

// Every buffer access below puts the whole offset (row, piece and k chunk) in voffset, none in soffset: a raw buffer's
// range check covers voffset (+ the instruction offset) only, so a tail chunk's k offset in soffset would let the
// last row of a resource read past its end.
//
// The default form (joint_dpre_nw = 0): only W^T goes through LDS; each wave owns 32 rows x all 256 hidden units of
// the tile (8 x 1 tiles, 128 accumulator registers) and loads its rows of G straight into the B operand with 16-byte
// global loads -- every G element reaches the CU once, and the LDS-DMA per MFMA is half the staged forms' (the DMA
// issue, not the MFMA, set their pace). K runs in chunks of 64 with the k order permuted inside a chunk (step ks,
// lane half hf, element e <-> k = 32 hf + 8 ks + e; A and B agree, so the products summed are the same): a lane's four
// G fragments of a chunk are 64 contiguous bytes, a whole 128-byte line per row between the two lane halves.
constexpr int kDKC = 64;                      // k per chunk
constexpr int kDStages = 4;                   // W^T stages of [256][64] bf16 (32 KiB each)
constexpr int kDImage = kGT * kDKC * 2;

__device__ __forceinline__ int dimg_off(int r, int p) { return r * 128 + ((p ^ ((r >> 1) & 7)) << 4); }

// One chunk of 64 k of the direct / persistent forms: 4 k-steps x 8 MFMAs. The A fragments of k-step ks + 1 are read
// from LDS before the MFMAs of ks are issued (two fragment sets, sched_barrier-fenced): left to itself the compiler
// reuses two fragment registers and waits out an LDS round trip every second MFMA.
template <bool TAILV>
__device__ __forceinline__ void dchunk_mma(const unsigned char *wi, const int (&aoff)[4], const gbf16x8 (&gc)[4],
                                           gf32x16 (&acc)[8], int k0, int hf, int V) {
    gbf16x8 fa[2][8];
#pragma unroll
    for (int a = 0; a < 8; ++a) fa[0][a] = *reinterpret_cast<const gbf16x8 *>(wi + aoff[0] + 4096 * a);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
        if (ks + 1 < 4) {
#pragma unroll
            for (int a = 0; a < 8; ++a)
                fa[(ks + 1) & 1][a] = *reinterpret_cast<const gbf16x8 *>(wi + aoff[ks + 1] + 4096 * a);
        }
        __builtin_amdgcn_sched_barrier(0);
        gbf16x8 fb = gc[ks];
        if constexpr (TAILV) {
            if (k0 + 32 * hf + 8 * ks >= V) {  // k = k0 + 32 hf + 8 ks + [0, 8)
                fb = (gbf16x8){};
#pragma unroll
                for (int a = 0; a < 8; ++a) fa[ks & 1][a] = (gbf16x8){};
            }
        }
#pragma unroll
        for (int a = 0; a < 8; ++a) acc[a] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[ks & 1][a], fb, acc[a], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// TAILV: V is not a multiple of 64 -- fragments of k >= V are zeroed in both operands (a per-lane select in every
// chunk); V % 64 == 0 compiles without it. The chunk loop runs in pairs so the two G register sets alternate without
// copies, and every A-fragment read is one base address per k-step plus the tile's immediate offset (the swizzle of
// row 32 a + l32 depends on l32 alone).
template <bool TAILV>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void joint_dpre_direct_kernel(
    const unsigned short *__restrict__ G, const unsigned short *__restrict__ Wt, const unsigned short *__restrict__ Hact,
    int64_t hact_ld, unsigned short *__restrict__ dpre, int64_t n, int V, int H) {
    constexpr int NW = 8;
    constexpr int DPI = kDImage / 1024 / NW;  // LDS-DMA wave-instructions per W^T chunk per wave (4)
    extern __shared__ __attribute__((aligned(16))) unsigned char glds[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nh = H / kGT;
    const int64_t b = blockIdx.x;
    const int64_t xcd = b & 7, j = b >> 3;
    const int hh = (int)(j % nh);
    const int64_t rt = (j / nh) * 8 + xcd;
    const int64_t r0 = rt * kGT;
    if (r0 >= n) return;
    const int h0 = hh * kGT;
    const int l32 = lane & 31, hf = lane >> 5;
    // this lane's row of G: rows past n read as zero (buffer bounds); 32-bit offsets within the resource
    const int rr = 32 * wave + l32;
    const int rows = (int)min<int64_t>(kGT, n - r0);
    const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<unsigned short *>(G) + r0 * V, (short)0, rows * V * 2, 0x00020000);
    const unsigned gvoff = (unsigned)(rr * V + 32 * hf) * 2u;
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<unsigned short *>(Wt) + (int64_t)h0 * V, (short)0, kGT * V * 2, 0x00020000);
    unsigned wvoff[DPI];
#pragma unroll
    for (int i = 0; i < DPI; ++i) {
        const int row = 8 * (DPI * wave + i) + (lane >> 3);
        const int p = (lane & 7) ^ ((row >> 1) & 7);
        wvoff[i] = (unsigned)(row * V + 8 * p) * 2u;
    }
    // A fragment of tile a, k-step ks: image row 32 a + l32, piece 4 hf + ks -> aoff[ks] + 4096 a
    int aoff[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) aoff[ks] = l32 * 128 + (((4 * hf + ks) ^ ((l32 >> 1) & 7)) << 4);
    const int nch = (V + kDKC - 1) / kDKC;
    auto stage = [&](int c) {
        unsigned char *s = glds + (c % kDStages) * kDImage;
#pragma unroll
        for (int i = 0; i < DPI; ++i) gemm_dma(rw, s + 1024 * (DPI * wave + i), wvoff[i] + (unsigned)(c * kDKC * 2), 0u);
    };
    auto gload = [&](int c, gbf16x8 (&f)[4]) {
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
            f[ks] = __builtin_bit_cast(gbf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                                    rg, gvoff + 16u * ks + (unsigned)(c * kDKC * 2), 0u, 0));
    };
#pragma unroll
    for (int c = 0; c < kDStages - 1; ++c)
        if (c < nch) stage(c);
    gbf16x8 g0[4], g1[4];
    gload(0, g0);
    if (1 < nch) gload(1, g1);
    gf32x16 acc[8];
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[a][e] = 0.0f;

    // one chunk: wait for its W^T and G (in-order completion: iteration i issues W^T chunk i + 3, then G chunk i + 2,
    // so after G chunk c come W^T chunk c + 2 and G chunk c + 1, 4 ops each), barrier, refill, 32 MFMAs
    auto chunk = [&](int c, gbf16x8 (&gc)[4]) {
        static_assert(DPI == 4 && kDStages == 4, "the wait counts assume 4 DMA ops per chunk and 4 stages");
        if (c == 0) {
            if (nch > 1) gemm_wait_vm<4>();
            else gemm_wait_vm<0>();
        } else if (c + 2 < nch) {
            gemm_wait_vm<8>();
        } else if (c + 1 < nch) {
            gemm_wait_vm<4>();
        } else {
            gemm_wait_vm<0>();
        }
        gemm_barrier();
        if (c + kDStages - 1 < nch) stage(c + kDStages - 1);
        dchunk_mma<TAILV>(glds + (c % kDStages) * kDImage, aoff, gc, acc, c * kDKC, hf, V);
    };
    int c = 0;
    for (; c + 1 < nch; c += 2) {
        chunk(c, g0);
        if (c + 2 < nch) gload(c + 2, g0);
        chunk(c + 1, g1);
        if (c + 3 < nch) gload(c + 3, g1);
    }
    if (c < nch) chunk(c, g0);

    // epilogue: lane (l32, hf) holds row r0 + 32 wave + l32 and, in register 4 g + e of tile a, hidden unit
    // h = h0 + 32 a + 8 g + 4 hf + e
    if (rr >= rows) return;
    const int64_t r = r0 + rr;
    const unsigned short *hrow = Hact + r * hact_ld;
    unsigned short *orow = dpre + r * H;
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int h = h0 + 32 * a + 8 * g + 4 * hf;
            const uint2 hv = *reinterpret_cast<const uint2 *>(hrow + h);
            const float h0v = bf16_lo_f(hv.x), h1v = bf16_hi_f(hv.x), h2v = bf16_lo_f(hv.y), h3v = bf16_hi_f(hv.y);
            const float d0 = acc[a][4 * g] * (1.0f - h0v * h0v), d1 = acc[a][4 * g + 1] * (1.0f - h1v * h1v);
            const float d2 = acc[a][4 * g + 2] * (1.0f - h2v * h2v), d3 = acc[a][4 * g + 3] * (1.0f - h3v * h3v);
            *reinterpret_cast<uint2 *>(orow + h) = make_uint2(IoBF16::pack2(d0, d1), IoBF16::pack2(d2, d3));
        }
}

template <int NW, int RT, int NS, int WPE, int EPI>
static hipError_t launch_dpre_nw(const unsigned short *G, const unsigned short *Wt, const unsigned short *Hact,
                                 int64_t hact_ld, unsigned short *dpre, int64_t n, int V, int H, hipStream_t stream) {
    constexpr int TR = 16 * NW * RT;
    const size_t lds = (size_t)NS * (TR + kGT) * kGKC * 2;
    const int64_t rtiles = (n + TR - 1) / TR;
    const int64_t blocks = ((rtiles + 7) / 8) * 8 * (H / kGT);  // (row tile, h-half) pairs in XCD order; extras exit
    if (blocks > 0x7fffffff / 512) return hipErrorInvalidValue;
    auto kern = joint_dpre_kernel<NW, RT, NS, WPE, EPI>;
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    kern<<<(unsigned)blocks, 64 * NW, lds, stream>>>(G, Wt, Hact, hact_ld, dpre, n, V, H, tuning().joint_dpre_abl);
    return hipGetLastError();
}

// The persistent form (default, joint_dpre_nw = 0): the direct form's tile, one workgroup per CU walking tiles
// b, b + G, ... (G = grid size, a multiple of 8, so the XCD pairing holds), with the W^T DMA and the G loads running
// on across tile boundaries -- the next tile's first chunks are in flight while this one's epilogue runs, and no
// workgroup start, prologue or drained pipeline separates the tiles.
template <bool TAILV>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void joint_dpre_persist_kernel(
    const unsigned short *__restrict__ G, const unsigned short *__restrict__ Wt, const unsigned short *__restrict__ Hact,
    int64_t hact_ld, unsigned short *__restrict__ dpre, int64_t n, int V, int H, int64_t slots) {
    constexpr int NW = 8;
    constexpr int DPI = kDImage / 1024 / NW;  // LDS-DMA wave-instructions per W^T chunk per wave (4)
    constexpr int kEpi = 64;                  // vector-memory ops of one epilogue per wave (32 Hact loads, 32 stores)
    extern __shared__ __attribute__((aligned(16))) unsigned char glds[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int l32 = lane & 31, hf = lane >> 5;
    const int nh = H / kGT;
    const int64_t rtiles = (n + kGT - 1) / kGT;
    const int64_t gsz = gridDim.x;
    // slot t -> (row tile, h-half): rt = 8 (t / (8 nh)) + t % 8, hh = (t / 8) % nh; only the last group of 8 row tiles
    // can hold invalid slots, so this workgroup's valid slots are a prefix of b, b + G, ...
    auto tile_rt = [&](int64_t t) { return ((t >> 3) / nh) * 8 + (t & 7); };
    int ntile = 0;
    for (int64_t t = blockIdx.x; t < slots && tile_rt(t) < rtiles; t += gsz) ++ntile;
    if (ntile == 0) return;
    const int nch = (V + kDKC - 1) / kDKC;
    const int nq = ntile * nch;  // < 2^31: ntile <= slots / G, nch <= V / 64
    struct Tile {
        int64_t r0;
        int h0, rows;
    };
    auto tile = [&](int k) {
        const int64_t t = blockIdx.x + (int64_t)k * gsz;
        Tile x;
        x.r0 = tile_rt(t) * kGT;
        x.h0 = (int)((t >> 3) % nh) * kGT;
        x.rows = (int)min<int64_t>(kGT, n - x.r0);
        return x;
    };
    const int rr = 32 * wave + l32;  // this lane's row of a tile
    const unsigned gvoff = (unsigned)(rr * V + 32 * hf) * 2u;
    unsigned wvoff[DPI];
#pragma unroll
    for (int i = 0; i < DPI; ++i) {
        const int row = 8 * (DPI * wave + i) + (lane >> 3);
        const int p = (lane & 7) ^ ((row >> 1) & 7);
        wvoff[i] = (unsigned)(row * V + 8 * p) * 2u;
    }
    int aoff[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) aoff[ks] = l32 * 128 + (((4 * hf + ks) ^ ((l32 >> 1) & 7)) << 4);
    // stream positions q = k nch + c (tile k of this workgroup, chunk c)
    auto stage = [&](int q) {
        if (q >= nq) return;
        const int k = q / nch, c = q - k * nch;
        const Tile x = tile(k);
        const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<unsigned short *>(Wt) + (int64_t)x.h0 * V, (short)0, kGT * V * 2, 0x00020000);
        unsigned char *s = glds + (q % kDStages) * kDImage;
#pragma unroll
        for (int i = 0; i < DPI; ++i) gemm_dma(rw, s + 1024 * (DPI * wave + i), wvoff[i] + (unsigned)(c * kDKC * 2), 0u);
    };
    auto gload = [&](int q, gbf16x8 (&f)[4]) {
        if (q >= nq) return;
        const int k = q / nch, c = q - k * nch;
        const Tile x = tile(k);
        const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<unsigned short *>(G) + x.r0 * V, (short)0, x.rows * V * 2, 0x00020000);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
            f[ks] = __builtin_bit_cast(gbf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                                    rg, gvoff + 16u * ks + (unsigned)(c * kDKC * 2), 0u, 0));
    };
    auto is_last_full = [&](int q) {  // q ends a tile whose 256 rows are all valid (its epilogue issued kEpi ops)
        if (q < 0) return false;
        const int k = q / nch;
        return q - k * nch == nch - 1 && tile(k).rows == kGT;
    };
#pragma unroll
    for (int q = 0; q < kDStages - 1; ++q) stage(q);
    gbf16x8 g0[4], g1[4];
    gload(0, g0);
    gload(1, g1);
    gf32x16 acc[8];
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[a][e] = 0.0f;

    // position q: wait for its W^T and G (in-order completion; after G(q), issued at the end of position q - 2, come
    // position q - 1's W^T(q + 2), epilogue and G(q + 1): wait for the largest supported count not above that),
    // barrier, W^T(q + 3), 32 MFMAs, the epilogue at a tile's last chunk; the caller then loads G(q + 2)
    auto step = [&](int q, gbf16x8 (&gc)[4]) {
        int after = 0;
        if (q >= 1) after += (q + 2 < nq ? DPI : 0) + (q + 1 < nq ? 4 : 0) + (is_last_full(q - 1) ? kEpi : 0);
        else after += (1 < nq ? 4 : 0);  // the prologue: G(1) after G(0)
        if (after >= 63) gemm_wait_vm<63>();
        else if (after >= 8) gemm_wait_vm<8>();
        else if (after >= 4) gemm_wait_vm<4>();
        else gemm_wait_vm<0>();
        gemm_barrier();
        stage(q + kDStages - 1);
        const int k = q / nch, c = q - k * nch;
        dchunk_mma<TAILV>(glds + (q % kDStages) * kDImage, aoff, gc, acc, c * kDKC, hf, V);
        if (c == nch - 1) {
            const Tile x = tile(k);
            if (rr < x.rows) {
                const int64_t r = x.r0 + rr;
                const unsigned short *hrow = Hact + r * hact_ld;
                unsigned short *orow = dpre + r * H;
#pragma unroll
                for (int a = 0; a < 8; ++a)
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const int h = x.h0 + 32 * a + 8 * g + 4 * hf;
                        const uint2 hv = *reinterpret_cast<const uint2 *>(hrow + h);
                        const float h0v = bf16_lo_f(hv.x), h1v = bf16_hi_f(hv.x);
                        const float h2v = bf16_lo_f(hv.y), h3v = bf16_hi_f(hv.y);
                        const float d0 = acc[a][4 * g] * (1.0f - h0v * h0v), d1 = acc[a][4 * g + 1] * (1.0f - h1v * h1v);
                        const float d2 = acc[a][4 * g + 2] * (1.0f - h2v * h2v);
                        const float d3 = acc[a][4 * g + 3] * (1.0f - h3v * h3v);
                        *reinterpret_cast<uint2 *>(orow + h) = make_uint2(IoBF16::pack2(d0, d1), IoBF16::pack2(d2, d3));
                    }
            }
#pragma unroll
            for (int a = 0; a < 8; ++a)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[a][e] = 0.0f;
        }
    };
    int q = 0;
    for (; q + 1 < nq; q += 2) {
        step(q, g0);
        gload(q + 2, g0);
        step(q + 1, g1);
        gload(q + 3, g1);
    }
    if (q < nq) step(q, g0);
}

template <bool TAILV>
static hipError_t launch_dpre_persist(const unsigned short *G, const unsigned short *Wt, const unsigned short *Hact,
                                      int64_t hact_ld, unsigned short *dpre, int64_t n, int V, int H, int64_t slots,
                                      hipStream_t stream) {
    const size_t lds = (size_t)kDStages * kDImage;
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(joint_dpre_persist_kernel<TAILV>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || cus <= 0)
        cus = 256;
    const int64_t grid = std::min<int64_t>(slots, (int64_t)(cus + 7) / 8 * 8);  // a multiple of 8: the XCD pairing
    joint_dpre_persist_kernel<TAILV><<<(unsigned)grid, 512, lds, stream>>>(G, Wt, Hact, hact_ld, dpre, n, V, H, slots);
    return hipGetLastError();
}

template <bool TAILV>
static hipError_t launch_dpre_direct(const unsigned short *G, const unsigned short *Wt, const unsigned short *Hact,
                                     int64_t hact_ld, unsigned short *dpre, int64_t n, int V, int H, int64_t blocks,
                                     hipStream_t stream) {
    const size_t lds = (size_t)kDStages * kDImage;
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(joint_dpre_direct_kernel<TAILV>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    joint_dpre_direct_kernel<TAILV><<<(unsigned)blocks, 512, lds, stream>>>(G, Wt, Hact, hact_ld, dpre, n, V, H);
    return hipGetLastError();
}

// dpre over the live rows; H in {256, 512}, V a multiple of 8 (16-byte rows), n_live < 2^31 / (2 V) per tile of 256
hipError_t launch_joint_dpre(const unsigned short *G, const unsigned short *Wt, const unsigned short *Hact,
                             int64_t hact_ld, unsigned short *dpre, int64_t n, int V, int H, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    if ((H != 256 && H != 512) || V % 8 || (int64_t)kGT * V * 2 >= ((int64_t)1 << 31) || hact_ld < H)
        return hipErrorInvalidValue;
    const int nh = H / kGT;
    const int64_t rtiles = (n + kGT - 1) / kGT;
    const int64_t blocks = ((rtiles + 7) / 8) * 8 * nh;  // (row tile, h-half) pairs in XCD order; extras exit
    if (blocks > 0x7fffffff / 512) return hipErrorInvalidValue;
    if constexpr (kVariants) {
        switch (tuning().joint_dpre_nw) {
        case 4: return launch_dpre_nw<4, 4, 4, 1, 0>(G, Wt, Hact, hact_ld, dpre, n, V, H, stream);
        case 8: return launch_dpre_nw<8, 2, 4, 2, 0>(G, Wt, Hact, hact_ld, dpre, n, V, H, stream);
        case 81: return launch_dpre_nw<8, 2, 4, 2, 1>(G, Wt, Hact, hact_ld, dpre, n, V, H, stream);
        case 42: return launch_dpre_nw<4, 2, 3, 2, 0>(G, Wt, Hact, hact_ld, dpre, n, V, H, stream);
        case 421: return launch_dpre_nw<4, 2, 3, 2, 1>(G, Wt, Hact, hact_ld, dpre, n, V, H, stream);
        case 431: return launch_dpre_nw<4, 2, 4, 2, 1>(G, Wt, Hact, hact_ld, dpre, n, V, H, stream);
        case 851: return launch_dpre_nw<8, 2, 5, 2, 1>(G, Wt, Hact, hact_ld, dpre, n, V, H, stream);
        case 812: return launch_dpre_nw<8, 2, 4, 2, 2>(G, Wt, Hact, hact_ld, dpre, n, V, H, stream);
        case 4212: return launch_dpre_nw<4, 2, 3, 2, 2>(G, Wt, Hact, hact_ld, dpre, n, V, H, stream);
        case 160: return launch_dpre_k16<4, false, false>(G, Wt, Hact, hact_ld, dpre, n, V, H, stream);
        case 161: return launch_dpre_k16<4, true, false>(G, Wt, Hact, hact_ld, dpre, n, V, H, stream);
        case 162: return launch_dpre_k16<5, false, false>(G, Wt, Hact, hact_ld, dpre, n, V, H, stream);
        case 163: return launch_dpre_k16<5, true, false>(G, Wt, Hact, hact_ld, dpre, n, V, H, stream);
        case 164: return launch_dpre_k16<4, false, true>(G, Wt, Hact, hact_ld, dpre, n, V, H, stream);
        case 165: return launch_dpre_k16<4, true, true>(G, Wt, Hact, hact_ld, dpre, n, V, H, stream);
        case 166: return launch_dpre_k16<5, false, true>(G, Wt, Hact, hact_ld, dpre, n, V, H, stream);
        case 167: return launch_dpre_k16<4, true, true, true>(G, Wt, Hact, hact_ld, dpre, n, V, H, stream);
        default: break;
        }
    }
    if constexpr (kVariants) {
        if (tuning().joint_dpre_nw == 1)
            return V % kDKC ? launch_dpre_direct<true>(G, Wt, Hact, hact_ld, dpre, n, V, H, blocks, stream)
                            : launch_dpre_direct<false>(G, Wt, Hact, hact_ld, dpre, n, V, H, blocks, stream);
        if (tuning().joint_dpre_nw == 2)  // round 5's default
            return V % kDKC ? launch_dpre_persist<true>(G, Wt, Hact, hact_ld, dpre, n, V, H, blocks, stream)
                            : launch_dpre_persist<false>(G, Wt, Hact, hact_ld, dpre, n, V, H, blocks, stream);
    }
    // the default (round 6): 16x16x32 tiles, fragments read a chunk ahead, DMA and reads interleaved with the MFMA
    // groups at s_setprio 1, the LDS-staged epilogue (profiles/r06/dpre/: 6.3 -> 4.85 ms at the headline size)
    return launch_dpre_k16<4, true, true>(G, Wt, Hact, hact_ld, dpre, n, V, H, stream);
}

}  // namespace mrnnt
