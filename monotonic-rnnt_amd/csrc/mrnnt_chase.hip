// mrnnt_chase.hip -- the forward pass as one launch: the log-softmax and the alpha / beta recursion
// (§8 a2) overlapped. The reference runs them back to back (gpu_rnnt.h:99-191: the reduce kernels, a device sync,
// then compute_alphas_kernel / compute_betas_kernel); here the recursion is latency-bound (one fp64 LSE chain per
// frame, ~0.1 us) while the log-softmax is HBM-bound, so the recursion workgroups run beside the log-softmax
// workgroups and consume each lattice column as soon as it is published.
//
// Grid: first the recursion workgroups (one per utterance and direction, B or 2B), then the log-softmax (producer)
// workgroups, which take the slots of the production order grid-stride. The order feeds both walks from their ends:
// round k publishes frames k and T_b - 1 - k of every utterance (alpha walks up from frame 0, beta down from T - 1),
// so neither walk waits for the whole pass; alpha alone (no beta): round k publishes frame k.
//
// Hand-off (cdna_hip_programming.md Guideline 16, R1): a producer workgroup stores its lp rows write-through (sc1),
// every wave drains its stores, a barrier, then one lane stores the column's ready flag. A recursion workgroup reads
// a column's lp rows only after seeing its flag and only with sc1 loads (L1 bypassed), never from a stale line.
//
// Ready tags: one 64-bit flag word per lattice column in the workspace, holding the tag of the launch that published
// it. The tag is a bijective mix of the host's per-call epoch with the launch's dispatch id (the AQL packet index of
// its queue) and queue address, so every launch -- a HIP-graph replay included, whose kernel arguments are frozen at
// capture -- waits for a tag no earlier launch stored: flags are never cleared, and a producer that publishes late
// cannot mislead a later launch. (Workspace bytes that were never a flag match with probability 2^-64.)
//
// Progress does not depend on scheduling. A recursion wave that has waited `budget` ticks of the 100 MHz constant
// clock for a column computes the rows it needs itself, with the producers' own column body (one wave, its rows):
// the same bits, so the result is unchanged whoever computes them. A kernel that holds the CUs on another stream, or
// recursion workgroups that fill the chip, make the launch slower, never wrong.
//
// One-wave recursion (S + 1 <= 64; configs[1]): wave 1 of the recursion workgroup is a loader. It polls the flags,
// copies each ready frame's lp rows into an LDS ring with one LDS-DMA instruction per frame (sc1, no registers), and
// counts them in LDS; wave 0 runs the dependent LSE chain from LDS, so no lp load on the chain waits for L2.
//
// Device-resident lengths (the reference's calling convention, monotonic_rnnt.cu:85-88; B <= 64): every wave holds
// the lengths in registers (wave_lengths) and locates its utterance or its slot's column from them, the first
// producer workgroup publishes the lattice offsets and the validation status (publish_lengths) for the gradient pass,
// each producer writes its column's entry of the column map, and lengths that fail validation make every workgroup
// stop: NaN costs, the status word set -- as the two-kernel path.
//
// Every lp value, every LSE and every store is the one the two-kernel path computes (the log-softmax bodies are
// mrnnt_lsm.h's, the recursion steps mrnnt_dp.h's), so results are bit-identical to it.
#include <algorithm>
#include <type_traits>

#include "mrnnt_dp.h"
#include "mrnnt_lsm.h"

namespace mrnnt {

extern "C" __device__ uint64_t mrnnt_llvm_dispatch_id() __asm("llvm.amdgcn.dispatch.id");

#ifdef MRNNT_DEVTOOLS
__device__ unsigned long long g_chase_helped;  // development build: columns a recursion wave computed itself
// development build: per-workgroup timeline (s_memrealtime ticks) of the first kTraceWgs workgroups, 4 marks each --
// recursion: start, lengths resolved, first frame in hand, walk done; producer: start, first slot, first flag, done
constexpr int kTraceWgs = 4096;
__device__ unsigned long long g_chase_trace[kTraceWgs * 4];
#define CHASE_MARK(i)                                                                          \
    do {                                                                                       \
        if (threadIdx.x == 0 && blockIdx.x < (unsigned)kTraceWgs)                              \
            g_chase_trace[blockIdx.x * 4 + (i)] = __builtin_amdgcn_s_memrealtime();            \
    } while (0)
// development build: walk progress of the first kWalkWgs recursion workgroups, 64 stamps each -- [0, 32): the walk
// wave finished walk positions [0, 8 (i + 1)); [32, 64): the loader published `loaded` >= 8 (i - 31)
constexpr int kWalkWgs = 128;
__device__ unsigned long long g_walk_trace[kWalkWgs * 64];
#define WALK_MARK(i)                                                                                         \
    do {                                                                                                     \
        if ((threadIdx.x & 63) == 0 && blockIdx.x < (unsigned)kWalkWgs && (unsigned)(i) < 64u)               \
            g_walk_trace[blockIdx.x * 64 + (i)] = __builtin_amdgcn_s_memrealtime();                          \
    } while (0)
#else
#define CHASE_MARK(i) ((void)0)
#define WALK_MARK(i) ((void)0)
#endif

// this launch's ready tag (scalar unit): a bijection of the dispatch id for a given epoch and queue
__device__ __forceinline__ unsigned long long launch_tag(unsigned long long epoch) {
    uint64_t x = epoch ^ ((mrnnt_llvm_dispatch_id() + 0x9E3779B97F4A7C15ull) * 0xBF58476D1CE4E5B9ull);
    x ^= (uint64_t)(uintptr_t)__builtin_amdgcn_queue_ptr() * 0x94D049BB133111EBull;
    x ^= x >> 31;
    x *= 0xD6E8FEB86659FD93ull;
    x ^= x >> 32;
    return x ? x : 1;
}

__device__ __forceinline__ uint32_t clock100() { return (uint32_t)__builtin_amdgcn_s_memrealtime(); }

// The log-softmax body of the chase launch. SM: 0 rows on 16-lane groups (rows of <= 64 vectors), 2 / 3
// single-chunk rows of <= 128 vectors (U = 2), 4 / 5 of <= 256 (U = 4), even = every chunk full (the product
// launch_u's choices for these rows). NWV / wv / [rlo, rhi]: the producers (4 waves, every row) or one wave's
// self-help (its rows; R = 1: the same per-row arithmetic with fewer registers live beside the recursion).
template <int SM, class IO, bool NTL, int NWV>
__device__ __forceinline__ void chase_column(const DevProblem &p, const ColRef &k, int wv = -1, int rlo = 0,
                                             int rhi = 1 << 30) {
    constexpr int U = SM <= 1 ? 1 : (SM <= 3 ? 2 : 4);
    constexpr bool FULL = (SM & 1) == 0;
    constexpr int R = NWV == 1 ? 1 : 2;
    if constexpr (SM == 0)
        row16_column<IO, 1, NTL, true, NWV>(p, k, wv, rlo, rhi);
    else
        lean_column<IO, U, R, NTL, FULL, true, true, NWV>(p, k, wv, rlo, rhi);
}

// A recursion wave's self-help: column t of its utterance, rows [rlo, rhi], computed by this wave and stored
// write-through like a producer's, then drained (the wave reads them back with sc1 loads). (Inlined: as a call, the
// ABI's saves around it cost more registers in the whole kernel than the body does inline.)
template <int SM, class IO, bool NTL>
struct SelfHelp {
    const DevProblem *p;
    Utt u;
    int b, rlo, rhi;
    __device__ __forceinline__ void operator()(int t) const {
        ColRef k;
        k.b = b;
        k.T = u.T;
        k.S = u.S;
        k.t = t;
        k.c = u.c0 + t;
        k.rowc = u.r0 + (int64_t)t * (u.S + 1);
        chase_column<SM, IO, NTL, 1>(*p, k, 0, rlo, rhi);
        drain_stores();
#ifdef MRNNT_DEVTOOLS
        if ((threadIdx.x & 63) == 0) atomicAdd(&g_chase_helped, 1ull);
#endif
    }
};

// The gate of the direct form (mrnnt_dp.h passes, Ch = Chase): a wave keeps the run of walk positions known ready
// (rdy). At the start of every prefetch block it reads the poll it issued one block earlier -- the flags of the 64
// positions from rdy, one vector load -- and issues the next: unconditional, so the compiler's wait for it counts the
// lp loads issued since and does not drain them, and a wave that runs behind the producers never stalls on a poll
// round trip. A frame beyond rdy waits in a blocking poll, for at most `budget` ticks, then is self-helped.
template <class Help>
struct Chase {
    static constexpr bool kOn = true;
    const unsigned long long *flags;  // ready flag of frame 0 of this utterance
    unsigned long long want;          // this launch's tag
    int T;
    bool fwd;       // alpha walks t = 0, 1, ...; beta t = T - 1, T - 2, ...
    int rdy;        // walk positions [0, rdy) known ready (wave-uniform)
    int ahead_at;   // `ahead`: this lane's flag of walk position ahead_at + lane (a poll issued earlier)
    unsigned long long ahead;
    uint32_t budget;
    const Help *help;

    __device__ __forceinline__ Chase(const unsigned long long *f, unsigned long long w, int T_, bool forward,
                                     uint32_t bud, const Help *h)
        : flags(f), want(w), T(T_), fwd(forward), rdy(0), ahead_at(0), ahead(0), budget(bud), help(h) {}
    // this lane's flag of walk position u + lane (positions past the walk read as ready)
    __device__ __forceinline__ unsigned long long poll(int u) const {
        const int i = u + (int)(threadIdx.x & 63);
        return i < T ? load_wt(&flags[fwd ? i : T - 1 - i]) : want;
    }
    __device__ __forceinline__ int run_of(unsigned long long v) const {
        const unsigned long long miss = ~__ballot(v == want);
        return miss ? __builtin_ctzll(miss) : 64;
    }
    __device__ __forceinline__ void refresh() {
        const int run = run_of(ahead);
        if (ahead_at <= rdy) rdy = max(rdy, ahead_at + run);
        ahead_at = min(rdy, T);
        ahead = poll(ahead_at);
    }
    __device__ __forceinline__ void gate(int f) {
        const int u = fwd ? f : T - 1 - f;
        if (u < rdy) return;
        uint32_t t0 = 0;
        bool timing = false;  // (the clock is read only once a poll has failed: a frame found ready costs none)
        for (;;) {
            const int run = run_of(poll(u));
            if (run > 0) {
                rdy = u + run;
                return;
            }
            const uint32_t now = clock100();
            if (!timing) {
                t0 = now;
                timing = true;
            } else if (now - t0 >= budget) {
                (*help)(f);
                rdy = u + 1;
                return;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
};

// ---- one-wave recursion with LDS-staged frames -----------------------------------------------------------------

// The LDS ring of lp frames, packed at the frame's width (W = S + 1 rows of 16 bytes; the loader's LDS-DMA writes
// lanes < W only): 16 KiB, the largest power-of-two count of frames that fits (16 at configs[1]'s W = 41, 32 for W <=
// 32, 64 for W <= 16). Round 6 measured the product launch (rocprofv3, one box, alternating builds: DESIGN.md 6):
// this ring with ring slots freed as soon as the walk has read them into registers (early_free) 34.2 us against the
// round-5 ring's 35.8; a 21 KiB ring of 32 frames costs the co-resident producers a workgroup per CU (7 instead of 9)
// and the launch 37.8 us with frame pairs; the frame-pair walks (PAIR 2 / 3 below) 37.0-41.0 us -- the walk's chain
// is not what bounds the product launch, the producers' occupancy is.
#ifndef MRNNT_CHASE_RING_LP  // (product A/B builds of round 6 override these three)
#define MRNNT_CHASE_RING_LP 1024
#endif
#ifndef MRNNT_CHASE_PAIR
#define MRNNT_CHASE_PAIR 1
#endif
#ifndef MRNNT_CHASE_EARLY
#define MRNNT_CHASE_EARLY 1
#endif
constexpr int kRingLp = MRNNT_CHASE_RING_LP;
__device__ __forceinline__ int ring_frames(int W, int cap) {
    int r = 64;
    while (r > 1 && r * W > kRingLp) r >>= 1;  // the largest power of two that fits
    return min(r, cap);
}

struct StageLds {
    Lp ring[kRingLp];
    int loaded;        // walk positions [0, loaded) are in the ring (the loader wave)
    int consumed[64];  // [0]: walk positions [0, consumed) have been read by the recursion wave (every lane of it
                       // stores its own word, so the store needs no lane-0 branch); PAIR = 3: by the side wave
    int chained[64];   // PAIR = 3, [0]: walk positions [0, chained) walked, their chain values handed to the side wave
    double sink[64];   // PAIR = 3: where the hand-off stores of lanes past S go
};
struct NoStage {};

__device__ __forceinline__ int lds_get(const int *w) {
    return __builtin_amdgcn_readfirstlane(__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
}
__device__ __forceinline__ void lds_put(int *w, int v) {
    __hip_atomic_store(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Wave 1: walk position u (frame fwd ? u : T - 1 - u) into ring slot u % R (R = ring_frames), lane l < W <- lp row l
// frame. One iteration = one poll round trip: the explicit vmcnt(0) before publishing `loaded` covers every DMA
// issued before the poll, then the DMAs of the frames the poll found ready (as far as the ring has room) are issued.
template <class Help>
__device__ __forceinline__ void stage_loader(const DevProblem &p, const Utt &u, bool fwd, const unsigned long long *flags,
                                             unsigned long long want, uint32_t budget, const Help &help,
                                             StageLds &st, int R, int probe = 0) {
    const int lane = threadIdx.x & 63;
    const int T = u.T, W = u.S + 1;
    const unsigned col = (unsigned)min(lane, u.S);
    const __amdgpu_buffer_rsrc_t rs = lp_rsrc(p);
    int issued = 0;
    uint32_t t_wait = 0;
    bool waiting = false;
#ifdef MRNNT_DEVTOOLS
    int marked = 0;
#endif
    for (;;) {
        const int i = issued + lane;
        const unsigned long long v = i < T ? load_wt(&flags[fwd ? i : T - 1 - i]) : want;
        wait_vmcnt0();  // the poll and every earlier DMA have landed
        lds_put(&st.loaded, issued);
#ifdef MRNNT_DEVTOOLS
        if (probe & 8) {
            for (int m = marked + 1; m <= issued / 8; ++m) WALK_MARK(31 + m);
            marked = max(marked, issued / 8);
        }
#endif
        if (issued >= T) return;
        const unsigned long long miss = ~__ballot(v == want);
        int ready = issued + (miss ? __builtin_ctzll(miss) : 64);
        if (ready == issued) {
            const uint32_t now = clock100();
            if (!waiting) {
                waiting = true;
                t_wait = now;
            }
            if (now - t_wait >= budget) {
                help(fwd ? issued : T - 1 - issued);
                ready = issued + 1;
            } else {
                __builtin_amdgcn_s_sleep(2);
            }
        }
        if (ready > issued) waiting = false;
        const int room = lds_get(&st.consumed[0]) + R;
        const int end = min(min(ready, room), T);
        for (; issued < end; ++issued) {
            const int t = fwd ? issued : T - 1 - issued;
            const unsigned off = (unsigned)((u.r0 + (int64_t)t * W) * (int64_t)sizeof(Lp)) + col * (unsigned)sizeof(Lp);
            if (lane < W)  // (the frame's rows only: the next slot starts right after them)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rs, (__attribute__((address_space(3))) void *)&st.ring[(issued & (R - 1)) * W], 16, off, 0, 0,
                    kAuxSc1);
        }
        if (end < ready && ready > issued) __builtin_amdgcn_s_sleep(1);  // ring full: the recursion wave catches up
    }
}

// Wave 0: walk position u's lp row from the ring (its own row; the same value the direct pass loads), P frames ahead.
// The walk starts with an explicit vmcnt(0): the compiler's wait-count pass joins the other roles' paths into this
// one (the kernel's control flow is structurised), takes the loader's LDS-DMAs for outstanding here, and would
// otherwise put a vmcnt(0) -- a wait for the walk's own alpha / beta stores -- before every LDS access of the walk.
template <int P>
struct RingReader {
    StageLds &st;
    int avail = 0;
    const int R, W, col;  // ring frames, frame width, this lane's row in a frame (lanes past S read row S)
    __device__ __forceinline__ RingReader(StageLds &s, int R_, int S) : st(s), R(R_), W(S + 1), col(min((int)(threadIdx.x & 63), S)) {}
    __device__ __forceinline__ Lp read(int u) {
        while (avail <= u) {
            avail = lds_get(&st.loaded);
            if (avail <= u) __builtin_amdgcn_s_sleep(1);
        }
        asm volatile("" ::: "memory");
        return st.ring[(u & (R - 1)) * W + col];
    }
    __device__ __forceinline__ void done(int u) {  // walk positions [0, u] may be refilled (once per block of P)
        lds_put(&st.consumed[threadIdx.x & 63], u + 1);
    }
};

// The walk's alpha / beta stores through a buffer resource over the utterance's rows: lanes past S get an offset
// outside the resource and the hardware drops their store -- no exec-mask branch around every step's store.
struct RowStore {
    __amdgpu_buffer_rsrc_t rs;
    unsigned voff;
    __device__ __forceinline__ RowStore(double *rows, int64_t n, int lane, int W)
        : rs(__builtin_amdgcn_make_buffer_rsrc(static_cast<void *>(rows), (short)0, (int)(n * (int64_t)sizeof(double)),
                                               0x00020000)),
          voff(lane < W ? (unsigned)lane * 8u : 0x80000000u) {}
    __device__ __forceinline__ void put(double v, unsigned soff) const {
        typedef unsigned u2 __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, v), rs, voff, soff, 0);
    }
};

// The steps of alpha_pass_halo / beta_pass_halo at NW = 1, HL = 0, lean (the same operations, so the same bits),
// laid out for a one-wave chain: blocks of P steps with no branch inside (the ring read of each step clamps its frame
// instead of testing it, the stores are buffer stores, consumption is published once per block: the positions read
// into registers so far with early_free, else the positions used).
//
// PAIR = 2: the chain advances two frames per dependent log-sum-exp. Over frames t, t + 1 a cell s is reached from
// s (two blanks), s - 1 (an emission at t or at t + 1) or s - 2 (two emissions), so
//   alpha(t+1, s) = lse3(alpha(t-1, s)   + lpb(t, s) + lpb(t+1, s),
//                        alpha(t-1, s-1) + lse2(lpe(t, s-1) + lpb(t+1, s), lpb(t, s-1) + lpe(t+1, s-1)),
//                        alpha(t-1, s-2) + lpe(t, s-2) + lpe(t+1, s-1))
// whose coefficients do not depend on alpha: the chain carries one three-term step (two DPP shifts deep) where it
// carried two two-term steps, and alpha(t, .) -- the single step, exactly as PAIR = 1 forms it from alpha(t-1, .) -- is
// formed beside it for the store. Results agree with the single-step chain to fp64 rounding of the LSE corrections
// (~1e-7), not bit for bit.
template <int P, int PAIR>
__device__ __forceinline__ void alpha_staged(const DevProblem &p, const Utt &u, int b, float *__restrict__ costs,
                                             StageLds &st, int R, int probe = 0, int early_free = 1) {
    static_assert(P % 2 == 0, "frame pairs inside a block");
    const int lane = threadIdx.x & 63;
    const int T = u.T, S = u.S, W = S + 1;
    RingReader<P> rr(st, R, S);
    wait_vmcnt0();  // (see RingReader)
    const RowStore out(p.alpha + u.r0, (int64_t)T * W, lane, W);
    double a = (lane == 0) ? 0.0 : NEG_INF_D;
    Lp q[P];
#pragma unroll
    for (int d = 0; d < P; ++d) q[d] = rr.read(min(d, T - 1));
    CHASE_MARK(2);
    unsigned soff = 0;
    const unsigned row = (unsigned)W * 8u;
    auto step = [&](int t, int d) {
        const double y = dpp_shr1_ninf(a + q[d].e);  // alpha(t-1, s-1) + lpe(t, s-1), from lane s-1 (lane 0: -inf)
        if (kVariants && (probe & 2))
            a = max_f64(a + q[d].b, y);
        else
            a = lse2(a + q[d].b, y);
        if (!kVariants || !(probe & 1)) out.put(a, soff);
        soff += row;
        if (!kVariants || !(probe & 4)) q[d] = rr.read(min(t + P, T - 1));
    };
    auto pair = [&](int t, int d) {  // frames t, t + 1 from q[d], q[d + 1]
        const Lp q0 = q[d], q1 = q[d + 1];
        const double y = dpp_shr1_ninf(a + q0.e);                       // alpha(t-1, s-1) + lpe(t, s-1)
        const double a1 = lse2(a + q0.b, y);                            // alpha(t, s), off the chain
        const double k1 = lse2(q0.e + dpp_shl1_ninf(q1.b), q0.b + q1.e);  // s -> s+1 over t, t+1 (lane s)
        const double x0 = a + (q0.b + q1.b);
        const double x1 = dpp_shr1_ninf(a + k1);
        const double x2 = dpp_shr1_ninf(y + q1.e);
        a = lse3(x0, x1, x2);
        out.put(a1, soff);
        out.put(a, soff + row);
        soff += 2 * row;
        if (!kVariants || !(probe & 4)) {
            q[d] = rr.read(min(t + P, T - 1));
            q[d + 1] = rr.read(min(t + 1 + P, T - 1));
        }
    };
    // PAIR = 3: the chain only -- alpha(t, .) is left to the side wave (alpha_side), which takes the chain value
    // alpha(t-1, .) from the ring slot of frame t - 1, where this wave writes it (lpb of that frame, read already)
    double *const hand = lane < W ? &st.ring[lane].b : &st.sink[lane];
    auto pair3 = [&](int t, int d) {
        const Lp q0 = q[d], q1 = q[d + 1];
        const double y = dpp_shr1_ninf(a + q0.e);
        const double k1 = lse2(q0.e + dpp_shl1_ninf(q1.b), q0.b + q1.e);
        const double x0 = a + (q0.b + q1.b);
        const double x1 = dpp_shr1_ninf(a + k1);
        const double x2 = dpp_shr1_ninf(y + q1.e);
        a = lse3(x0, x1, x2);
        out.put(a, soff + row);
        hand[lane < W ? ((t + 1) & (R - 1)) * W * 2 : 0] = a;  // (Lp = two doubles: slot stride 2 W doubles)
        asm volatile("" ::: "memory");
        lds_put(&st.chained[lane], t + 2);
        soff += 2 * row;
        q[d] = rr.read(min(t + P, T - 1));
        q[d + 1] = rr.read(min(t + 1 + P, T - 1));
    };
    int t0 = 0;
    for (; t0 + P <= T; t0 += P) {
        if constexpr (PAIR == 3) {
#pragma unroll
            for (int d = 0; d < P; d += 2) pair3(t0 + d, d);
        } else if constexpr (PAIR == 2) {
#pragma unroll
            for (int d = 0; d < P; d += 2) pair(t0 + d, d);
        } else {
#pragma unroll
            for (int d = 0; d < P; ++d) step(t0 + d, d);
        }
        if constexpr (PAIR != 3) rr.done(early_free ? t0 + 2 * P - 1 : t0 + P - 1);
#ifdef MRNNT_DEVTOOLS
        if ((probe & 8) && ((t0 + P) & 7) == 0) WALK_MARK((t0 + P) / 8 - 1);
#endif
    }
    if constexpr (PAIR == 3) {
#pragma unroll
        for (int d = 0; d < P; d += 2) {
            if (t0 + d + 1 < T)
                pair3(t0 + d, d);
            else if (t0 + d < T)
                step(t0 + d, d);
        }
        asm volatile("" ::: "memory");
        lds_put(&st.chained[lane], T);
    } else if constexpr (PAIR == 2) {
#pragma unroll
        for (int d = 0; d < P; d += 2) {
            if (t0 + d + 1 < T)
                pair(t0 + d, d);
            else if (t0 + d < T)
                step(t0 + d, d);
        }
    } else {
#pragma unroll
        for (int d = 0; d < P; ++d) {
            if (t0 + d >= T) break;
            step(t0 + d, d);
        }
    }
    if (lane == S) {
        p.ll[b] = a;
        if (costs) costs[b] = (float)(-a);
    }
}

// PAIR = 2 (as alpha_staged), walk positions w, w + 1 = frames t = T - 1 - w and t - 1:
//   beta(t-1, s) = lse3(beta(t+1, s)   + lpb(t-1, s) + lpb(t, s),
//                       beta(t+1, s+1) + lse2(lpb(t-1, s) + lpe(t, s), lpe(t-1, s) + lpb(t, s+1)),
//                       beta(t+1, s+2) + lpe(t-1, s) + lpe(t, s+1))
template <int P, int PAIR>
__device__ __forceinline__ void beta_staged(const DevProblem &p, const Utt &u, int b, StageLds &st, int R,
                                            int probe = 0, int early_free = 1) {
    static_assert(P % 2 == 0, "frame pairs inside a block");
    const int lane = threadIdx.x & 63;
    const int T = u.T, S = u.S, W = S + 1;
    RingReader<P> rr(st, R, S);
    wait_vmcnt0();  // (see RingReader)
    const RowStore out(p.beta + u.r0, (int64_t)T * W, lane, W);
    double bn = (lane == S) ? 0.0 : NEG_INF_D;  // beta(T, s)
    Lp q[P];
#pragma unroll
    for (int d = 0; d < P; ++d) q[d] = rr.read(min(d, T - 1));
    CHASE_MARK(2);
    const unsigned row = (unsigned)W * 8u;
    unsigned soff = (unsigned)(T - 1) * row;
    auto step = [&](int w, int d) {  // walk position w = frame T - 1 - w
        const double carry = dpp_shl1_ninf(bn);  // beta(t+1, s+1), from lane s+1 (lane 63: -inf)
        if (kVariants && (probe & 2))
            bn = max_f64(bn + q[d].b, carry + q[d].e);
        else
            bn = lse2(bn + q[d].b, carry + q[d].e);
        if (!kVariants || !(probe & 1)) out.put(bn, soff);
        soff -= row;
        if (!kVariants || !(probe & 4)) q[d] = rr.read(min(w + P, T - 1));
    };
    auto pair = [&](int w, int d) {  // frames t = T - 1 - w (q[d]) and t - 1 (q[d + 1])
        const Lp q0 = q[d], q1 = q[d + 1];
        const double carry = dpp_shl1_ninf(bn);                         // beta(t+1, s+1)
        const double g = carry + q0.e;
        const double b1 = lse2(bn + q0.b, g);                           // beta(t, s), off the chain
        const double d1 = lse2(q1.b + q0.e, q1.e + dpp_shl1_ninf(q0.b));  // s -> s+1 over t-1, t (lane s)
        const double x0 = bn + (q1.b + q0.b);
        const double x1 = carry + d1;
        const double x2 = dpp_shl1_ninf(g) + q1.e;
        bn = lse3(x0, x1, x2);
        out.put(b1, soff);
        out.put(bn, soff - row);
        soff -= 2 * row;
        if (!kVariants || !(probe & 4)) {
            q[d] = rr.read(min(w + P, T - 1));
            q[d + 1] = rr.read(min(w + 1 + P, T - 1));
        }
    };
    double *const hand = lane < W ? &st.ring[lane].b : &st.sink[lane];
    auto pair3 = [&](int w, int d) {  // PAIR = 3: the chain only (beta_side forms beta(t, .))
        const Lp q0 = q[d], q1 = q[d + 1];
        const double carry = dpp_shl1_ninf(bn);
        const double g = carry + q0.e;
        const double d1 = lse2(q1.b + q0.e, q1.e + dpp_shl1_ninf(q0.b));
        const double x0 = bn + (q1.b + q0.b);
        const double x1 = carry + d1;
        const double x2 = dpp_shl1_ninf(g) + q1.e;
        bn = lse3(x0, x1, x2);
        out.put(bn, soff - row);
        hand[lane < W ? ((w + 1) & (R - 1)) * W * 2 : 0] = bn;
        asm volatile("" ::: "memory");
        lds_put(&st.chained[lane], w + 2);
        soff -= 2 * row;
        q[d] = rr.read(min(w + P, T - 1));
        q[d + 1] = rr.read(min(w + 1 + P, T - 1));
    };
    int w0 = 0;
    for (; w0 + P <= T; w0 += P) {
        if constexpr (PAIR == 3) {
#pragma unroll
            for (int d = 0; d < P; d += 2) pair3(w0 + d, d);
        } else if constexpr (PAIR == 2) {
#pragma unroll
            for (int d = 0; d < P; d += 2) pair(w0 + d, d);
        } else {
#pragma unroll
            for (int d = 0; d < P; ++d) step(w0 + d, d);
        }
        if constexpr (PAIR != 3) rr.done(early_free ? w0 + 2 * P - 1 : w0 + P - 1);
#ifdef MRNNT_DEVTOOLS
        if ((probe & 8) && ((w0 + P) & 7) == 0) WALK_MARK((w0 + P) / 8 - 1);
#endif
    }
    if constexpr (PAIR == 3) {
#pragma unroll
        for (int d = 0; d < P; d += 2) {
            if (w0 + d + 1 < T)
                pair3(w0 + d, d);
            else if (w0 + d < T)
                step(w0 + d, d);
        }
        asm volatile("" ::: "memory");
        lds_put(&st.chained[lane], T);
    } else if constexpr (PAIR == 2) {
#pragma unroll
        for (int d = 0; d < P; d += 2) {
            if (w0 + d + 1 < T)
                pair(w0 + d, d);
            else if (w0 + d < T)
                step(w0 + d, d);
        }
    } else {
#pragma unroll
        for (int d = 0; d < P; ++d) {
            if (w0 + d >= T) break;
            step(w0 + d, d);
        }
    }
    if (lane == 0) p.llb[b] = bn;
}

// PAIR = 3, wave 2: alpha(t, .) for the first frame t of every pair, from the chain value alpha(t-1, .) the walk
// handed over in the ring slot of frame t - 1 (t = 0: alpha(-1, .) = [0, -inf, ...]) and frame t's lp rows, still
// in the ring: the walk's side step, exactly as PAIR = 2 forms it (the same bits). It frees ring slots for the loader.
// (Polls only when the counts it last read do not cover the pair: one LDS round trip per pair besides the data.)
__device__ __forceinline__ int side_wait(const int *w, int have, int need) {
    while (have < need) {
        have = lds_get(w);
        if (have < need) __builtin_amdgcn_s_sleep(1);
    }
    return have;
}

__device__ __forceinline__ void alpha_side(const DevProblem &p, const Utt &u, StageLds &st, int R) {
    const int lane = threadIdx.x & 63;
    const int T = u.T, S = u.S, W = S + 1, col = min(lane, S);
    const RowStore out(p.alpha + u.r0, (int64_t)T * W, lane, W);
    const unsigned row = (unsigned)W * 8u;
    double prev = (lane == 0) ? 0.0 : NEG_INF_D;
    int chained = 0, loaded = 0;
    for (int k = 0; 2 * k + 1 < T; ++k) {
        chained = side_wait(&st.chained[0], chained, 2 * k);  // the chain value of frame 2k - 1
        loaded = side_wait(&st.loaded, loaded, 2 * k + 1);     // frame 2k in the ring
        asm volatile("" ::: "memory");
        const Lp q0 = st.ring[((2 * k) & (R - 1)) * W + col];
        if (k) prev = lane <= S ? st.ring[((2 * k - 1) & (R - 1)) * W + col].b : NEG_INF_D;
        const double y = dpp_shr1_ninf(prev + q0.e);
        out.put(lse2(prev + q0.b, y), (unsigned)(2 * k) * row);
        asm volatile("" ::: "memory");
        lds_put(&st.consumed[lane], 2 * k + 1);
    }
    lds_put(&st.consumed[lane], T);
}

__device__ __forceinline__ void beta_side(const DevProblem &p, const Utt &u, StageLds &st, int R) {
    const int lane = threadIdx.x & 63;
    const int T = u.T, S = u.S, W = S + 1, col = min(lane, S);
    const RowStore out(p.beta + u.r0, (int64_t)T * W, lane, W);
    const unsigned row = (unsigned)W * 8u;
    double prev = (lane == S) ? 0.0 : NEG_INF_D;  // beta(T, .)
    int chained = 0, loaded = 0;
    for (int k = 0; 2 * k + 1 < T; ++k) {  // walk position 2k = frame T - 1 - 2k
        chained = side_wait(&st.chained[0], chained, 2 * k);
        loaded = side_wait(&st.loaded, loaded, 2 * k + 1);
        asm volatile("" ::: "memory");
        const Lp q0 = st.ring[((2 * k) & (R - 1)) * W + col];
        if (k) prev = lane <= S ? st.ring[((2 * k - 1) & (R - 1)) * W + col].b : NEG_INF_D;
        const double carry = dpp_shl1_ninf(prev);
        out.put(lse2(prev + q0.b, carry + q0.e), (unsigned)(T - 1 - 2 * k) * row);
        asm volatile("" ::: "memory");
        lds_put(&st.consumed[lane], 2 * k + 1);
    }
    lds_put(&st.consumed[lane], T);
}

// ---- the launch ------------------------------------------------------------------------------------------------

// NW: recursion waves (1: S + 1 <= 64, one cell per lane; 4: the halo recursion with 56 own cells per wave, S + 1 <=
// 224). STG (NW = 1): frames staged in LDS by a loader wave (else the direct gated loads, development A/B). D: lp rows
// the direct form prefetches per lane. DYN: device-resident lengths.
template <class IO, int SM, bool NTL, int NW, bool STG, bool DYN>
__global__ __launch_bounds__(256) void chase_kernel(DevProblem p, ChaseArgs c, int with_beta, float *__restrict__ costs) {
    constexpr int HL = NW > 1 ? 8 : 0;
    constexpr int D = 8;
    __shared__ double xh[2][8][HL > 0 ? HL : 1];
    __shared__ typename std::conditional<STG && NW == 1, StageLds, NoStage>::type st;
    const int nrec = with_beta ? 2 * p.B : p.B;
    CHASE_MARK(0);
    const unsigned long long tag = launch_tag(c.epoch);
    WaveLengths wl;
    if constexpr (DYN) wl = wave_lengths(p);
    if ((int)blockIdx.x < nrec) {
        // ---- recursion workgroup ----
        const int b = with_beta ? (int)(blockIdx.x >> 1) : (int)blockIdx.x;
        const bool bwd = with_beta && (blockIdx.x & 1);
        Utt u;
        if constexpr (DYN) {
            if (!wl.ok) {  // lengths failed validation: touch no lattice array (publish_lengths reports it)
                if (threadIdx.x == 0) {
                    if (bwd) {
                        p.llb[b] = __builtin_nan("");
                    } else {
                        p.ll[b] = __builtin_nan("");
                        if (costs) costs[b] = __builtin_nanf("");
                    }
                }
                return;
            }
            u.T = __builtin_amdgcn_readlane(wl.T, b);
            u.S = __builtin_amdgcn_readlane(wl.S, b);
            u.c0 = b ? readlane64(wl.cols, b - 1) : 0;
            u.r0 = b ? readlane64(wl.rows, b - 1) : 0;
        } else {
            u = utt_of(p, b);
        }
        const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        const unsigned long long *flags = c.flags + u.c0;
        CHASE_MARK(1);
        if constexpr (STG && NW == 1) {
            const int R = ring_frames(u.S + 1, kVariants ? c.ring : 64);
            if (threadIdx.x == 0) {  // (LDS holds whatever the CU's previous workgroup left)
                st.loaded = 0;
                st.consumed[0] = 0;
                st.chained[0] = 0;
            }
            __syncthreads();
            const int pair = kVariants ? c.pair : MRNNT_CHASE_PAIR;
            if (wave == 2 && pair == 3) {  // the side wave of the chain-only walk
                if (bwd)
                    beta_side(p, u, st, R);
                else
                    alpha_side(p, u, st, R);
                return;
            }
            if (wave >= 2) return;
            if (wave == 1) {
                const SelfHelp<SM, IO, NTL> help{&p, u, b, 0, u.S};
                stage_loader(p, u, !bwd, flags, tag, c.budget, help, st, R, kVariants ? c.probe : 0);
                return;
            }
            const int probe = kVariants ? c.probe : 0, early = kVariants ? c.early_free : MRNNT_CHASE_EARLY;
            if (pair == 1) {  // (development A/B: one log-sum-exp per frame)
                if (bwd)
                    beta_staged<4, 1>(p, u, b, st, R, probe, early);
                else
                    alpha_staged<4, 1>(p, u, b, costs, st, R, probe, early);
            } else if (pair == 2) {  // (development A/B: the side step on the walk itself)
                if (bwd)
                    beta_staged<4, 2>(p, u, b, st, R, probe, early);
                else
                    alpha_staged<4, 2>(p, u, b, costs, st, R, probe, early);
            } else {
                if (bwd)
                    beta_staged<4, 3>(p, u, b, st, R, probe, early);
                else
                    alpha_staged<4, 3>(p, u, b, costs, st, R, probe, early);
            }
            CHASE_MARK(3);
            return;
        }
        if (wave >= NW) return;  // one-wave direct recursion: the other waves of the workgroup have no work
        // the rows this wave's lanes read (alpha: cells wave * 56 - HL + lane, beta: wave * 56 + lane; clamped to S)
        const int first = bwd ? wave * (64 - HL) : wave * (64 - HL) - HL;
        const SelfHelp<SM, IO, NTL> help{&p, u, b, max(first, 0), min(first + 63, u.S)};
        Chase<SelfHelp<SM, IO, NTL>> ch(flags, tag, u.T, !bwd, c.budget, &help);
        if (bwd)
            beta_pass_halo<D, NW, HL, false, 1>(p, u, b, xh, &ch);
        else
            alpha_pass_halo<D, NW, HL, false, 1>(p, u, b, costs, xh, &ch);
        return;
    }
    // ---- log-softmax workgroups: slots si, si + G, ... of the production order (G = the producer grid) ----
    if constexpr (DYN) {
        if (blockIdx.x == (unsigned)nrec) publish_lengths(p, wl);  // offsets, status, lp pads (wave 0)
        if (!wl.ok) return;
    } else if (blockIdx.x == (unsigned)nrec && threadIdx.x < 64) {  // the lp pads around [0, N)
        const int i = threadIdx.x;
        p.lp[i - 64] = Lp{0.0, 0.0};
        p.lp[p.num_rows + i] = Lp{0.0, 0.0};
    }
    if constexpr (kVariants) {
        if (c.delay) {  // (development probe: producers held back, so the recursion has to help itself)
            const uint32_t t0 = clock100();
            while (clock100() - t0 < c.delay) __builtin_amdgcn_s_sleep(64);
        }
    }
    const int64_t per = with_beta ? 2 * (int64_t)p.B : (int64_t)p.B;
    const int64_t G = (int64_t)gridDim.x - nrec;
    int64_t slots = c.slots;
    if constexpr (DYN) {
        int tmax = wl.T;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) tmax = max(tmax, __shfl_xor(tmax, off));
        tmax = __builtin_amdgcn_readfirstlane(tmax);
        slots = (with_beta ? (int64_t)(tmax + 1) / 2 : (int64_t)tmax) * per;
    }
    CHASE_MARK(1);
    bool first = true;
    for (int64_t si = (int64_t)blockIdx.x - nrec; si < slots; si += G) {
        const int kr = (int)(si / per);
        const int r = (int)(si - (int64_t)kr * per);
        const int b = with_beta ? (r >> 1) : r;
        ColRef k;
        k.b = b;
        if constexpr (DYN) {
            k.T = __builtin_amdgcn_readlane(wl.T, b);
            k.S = __builtin_amdgcn_readlane(wl.S, b);
        } else {
            k.T = p.T[b];
            k.S = p.S[b];
        }
        const int T = k.T;
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
        k.t = t;
        if constexpr (DYN) {
            k.c = (b ? readlane64(wl.cols, b - 1) : 0) + t;
            k.rowc = (b ? readlane64(wl.rows, b - 1) : 0) + (int64_t)t * (k.S + 1);
            if (threadIdx.x == 0) const_cast<int *>(p.col_b)[k.c] = b;  // the gradient pass's column map
        } else {
            k.c = p.col_off[b] + t;
            k.rowc = p.row_off[b] + (int64_t)t * (k.S + 1);
        }
        chase_column<SM, IO, NTL, 4>(p, k);
        drain_stores();  // every wave: its write-through rows have landed
        __syncthreads();
        if (threadIdx.x == 0) store_wt(&c.flags[k.c], tag);
        if (first) CHASE_MARK(2);
        first = false;
    }
    CHASE_MARK(3);
}

// The log-softmax body the chase launch carries for this problem (-1: none -- the two-kernel path runs). f32 acts,
// 16-byte aligned rows of <= 256 vectors (V <= 1024), the same shapes launch_u picks for them.
int chase_body(const DevProblem &p, int elem) {
    if (elem != ELEM_F32 || p.V % 4 || (reinterpret_cast<uintptr_t>(p.acts) & 15)) return -1;
    return chase_body_shape(p.V);
}

template <int SM, bool NTL, bool DYN>
static void launch_sm(const DevProblem &p, const ChaseArgs &c, int nw, int with_beta, float *costs, int64_t grid,
                      hipStream_t stream) {
    if (nw == 1) {
        if constexpr (kVariants) {
            if (!c.stage) {
                chase_kernel<IoF32, SM, NTL, 1, false, DYN><<<(unsigned)grid, 256, 0, stream>>>(p, c, with_beta, costs);
                return;
            }
        }
        chase_kernel<IoF32, SM, NTL, 1, true, DYN><<<(unsigned)grid, 256, 0, stream>>>(p, c, with_beta, costs);
    } else {
        chase_kernel<IoF32, SM, NTL, 4, false, DYN><<<(unsigned)grid, 256, 0, stream>>>(p, c, with_beta, costs);
    }
}

template <bool NTL, bool DYN>
static void launch_ntl(const DevProblem &p, const ChaseArgs &c, int sm, int nw, int with_beta, float *costs,
                       int64_t grid, hipStream_t stream) {
    switch (sm) {
        case 0: launch_sm<0, NTL, DYN>(p, c, nw, with_beta, costs, grid, stream); break;
        case 2: launch_sm<2, NTL, DYN>(p, c, nw, with_beta, costs, grid, stream); break;
        case 3: launch_sm<3, NTL, DYN>(p, c, nw, with_beta, costs, grid, stream); break;
        case 4: launch_sm<4, NTL, DYN>(p, c, nw, with_beta, costs, grid, stream); break;
        default: launch_sm<5, NTL, DYN>(p, c, nw, with_beta, costs, grid, stream); break;
    }
}

hipError_t launch_chase(const DevProblem &p, const ChaseArgs &c, int elem, int S_max, int with_beta, int producers,
                        float *costs, hipStream_t stream) {
    const int sm = chase_body(p, elem);
    const int W = S_max + 1;
    if (sm < 0 || W > 4 * 56 || p.min_s || producers < 1) return hipErrorInvalidValue;
    if (p.dyn && p.B > 64) return hipErrorInvalidValue;  // wave_lengths: one utterance per lane
    const int64_t grid = (with_beta ? 2 * (int64_t)p.B : (int64_t)p.B) + producers;
    if (grid > (int64_t)1 << 22) return hipErrorInvalidValue;
    const int nw = W <= 64 ? 1 : 4;
    const bool nt = nt_acts_loads(p, sizeof(float));
    if (p.dyn) {
        if (nt) launch_ntl<true, true>(p, c, sm, nw, with_beta, costs, grid, stream);
        else launch_ntl<false, true>(p, c, sm, nw, with_beta, costs, grid, stream);
    } else {
        if (nt) launch_ntl<true, false>(p, c, sm, nw, with_beta, costs, grid, stream);
        else launch_ntl<false, false>(p, c, sm, nw, with_beta, costs, grid, stream);
    }
    return hipGetLastError();
}

#ifdef MRNNT_DEVTOOLS
int chase_walk_trace(unsigned long long *out, int n) {
    n = std::min(n, kWalkWgs * 64);
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_walk_trace), sizeof(unsigned long long) * n) != hipSuccess) return -1;
    return n;
}

int chase_trace(unsigned long long *out, int n) {
    n = std::min(n, kTraceWgs * 4);
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_chase_trace), sizeof(unsigned long long) * n) != hipSuccess) return -1;
    return n;
}

unsigned long long chase_helped(bool reset) {
    unsigned long long v = 0;
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_chase_helped), sizeof(v)) != hipSuccess) return ~0ull;
    if (reset) {
        const unsigned long long z = 0;
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_chase_helped), &z, sizeof(z)) != hipSuccess) return ~0ull;
    }
    return v;
}
#endif

}  // namespace mrnnt
