// mrnnt_grad.hip -- logit gradient (replaces compute_grad_kernel, gpu_rnnt_kernel.h:239-288,
// and the CPU loop cpu_rnnt.h:216-236), with the upstream gradient (grad_scale[b]) fused:
//   g[v] = exp(z[v] + den + alpha(t-1,s) + beta(t,s) - ll)
//        - [v == blank]                     exp(lpb + alpha(t-1,s) + beta(t+1,s)   - ll)
//        - [v != blank, s < S, v == label]  exp(lpe + alpha(t-1,s) + beta(t+1,s+1) - ll)
// times grad_scale[b]. Per row the three coefficients are formed in fp64 from the recursion state; per
// element it is one fma + one v_exp_f32 (+ a select for the <= 2 special columns) in fp32 registers,
// then one conversion to the output element type. Out-of-band lattice rows store 0 * grad_scale (the
// reference's backward multiplies its zero rows by grad_output; NaN when ll = -inf, zero_row_value); padding
// rows of the padded layout store 0 (launch_pad_zero).
#include <algorithm>

#include "mrnnt_device.h"

namespace mrnnt {

template <class IO>
__device__ __forceinline__ typename IO::V grad_vec(const typename IO::V &xv, const RowCoef &rc, int j, int blank,
                                                   float sc) {
    constexpr int E = IO::E;
    float x[E];
    IO::unpack(xv, x);
    const int v0 = j * E;
    const int db = blank - v0;
    const int de = rc.lab >= 0 ? rc.lab - v0 : -1;
#pragma unroll
    for (int i = 0; i < E; ++i) {
        float g = fast_exp2(fmaf(x[i], kLog2e, rc.c2));
        g -= (db == i ? rc.cb : 0.0f) + (de == i ? rc.ce : 0.0f);
        x[i] = g * sc;
    }
    return IO::pack(x);
}

// Column-walking kernel with per-row coefficients (grad_variant 0 / 2): workgroups walk lattice columns, the
// four waves take rows s (R at a time), lanes take 16-byte vectors of the row, U per lane per chunk.
template <class IO, int U, int R, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void grad_kernel(DevProblem p, const float *__restrict__ scale,
                                                       void *__restrict__ grads) {
    if (!resolve_dyn(p)) {  // device-resident lengths failed validation: NaN gradients
        fill_failed_grads<IO>(p, grads);
        return;
    }
    typedef typename IO::V Vec;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int VL = p.V / IO::E;
    const int blank = p.blank;
    const Vec *__restrict__ av = reinterpret_cast<const Vec *>(p.acts);
    Vec *__restrict__ gv = reinterpret_cast<Vec *>(grads);

    Cursor cur;
    cur.b = blockIdx.x < p.num_cols ? p.col_b[blockIdx.x] : 0;
    for (int64_t c = blockIdx.x; c < p.num_cols; c += gridDim.x) {
        cur.advance(p.col_off, c);
        const int b = cur.b;
        const int T = p.T[b], S = p.S[b];
        const int t = (int)(c - p.col_off[b]);
        const int64_t rowc = p.row_off[b] + (int64_t)t * (S + 1);
        const int64_t arow = acts_col_base(p, b, t, rowc);
        const int lo = max(0, t - (T - S));
        const int hi = min(t, S);
        const double ll = p.ll[b];
        const float sc = scale ? scale[b * p.scale_stride] : 1.0f;
        const Vec zv = splat<IO>(zero_row_value(ll, sc));
        const int *__restrict__ lab_b = p.labels + (int64_t)b * p.label_stride;

        for (int s = wave * R; s <= S; s += 4 * R) {
            RowCoef rc[R];
            bool ok[R], inb[R];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int sr = s + r;
                ok[r] = sr <= S;
                inb[r] = ok[r] && sr >= lo && sr <= hi;
                if (inb[r]) {
                    rc[r] = row_coef(p, t, T, S, sr, rowc + sr, ll, lab_b);
                    inb[r] = rc[r].live;  // dead rows are stored like out-of-band rows
                } else {
                    rc[r] = RowCoef{0.0f, 0.0f, 0.0f, -1, false};
                }
            }
            for (int base = 0; base < VL; base += 64 * U) {
                Vec x[R][U];
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const int j = base + lane + 64 * u;
                        if (inb[r] && j < VL) x[r][u] = vload<NTL>(&av[(arow + s + r) * (int64_t)VL + j]);
                    }
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const int j = base + lane + 64 * u;
                        if (!ok[r] || j >= VL) continue;
                        const Vec g = inb[r] ? grad_vec<IO>(x[r][u], rc[r], j, blank, sc) : zv;
                        vstore<NTS>(&gv[(arow + s + r) * (int64_t)VL + j], g);
                    }
            }
        }
    }
}

// Staged-coefficient kernel (grad_variant 5, the default, and 6: 2 rows per wave). Work unit = a segment of up to 256
// rows of one lattice column. Phase A: one row per thread, the row's coefficients (row_coef: alpha/beta/den/lp
// read as coalesced vectors along s, the two fp64 exps lane-parallel) go to an LDS slot {c2, cb, ce, label|dead}.
// Phase B: the waves stream the segment's rows; a row's acts loads wait only for one broadcast LDS read, not for
// a chain of dependent scalar loads and fp64 math, so every wave keeps its row(s) of acts in flight. Two LDS
// buffers alternate between work units: one barrier per unit.
template <class IO, int U, int R, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void grad_staged_kernel(DevProblem p, const float *__restrict__ scale,
                                                          void *__restrict__ grads) {
    if (!resolve_dyn(p)) {  // device-resident lengths failed validation: NaN gradients
        fill_failed_grads<IO>(p, grads);
        return;
    }
    typedef typename IO::V Vec;
    constexpr int SEG = 256;
    constexpr int DEAD = -2;  // label slot of a row whose gradient is exactly zero (out of band or dead)
    __shared__ float4 coef[2][SEG];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int VL = p.V / IO::E;
    const int blank = p.blank;
    const Vec *__restrict__ av = reinterpret_cast<const Vec *>(p.acts);
    Vec *__restrict__ gv = reinterpret_cast<Vec *>(grads);

    Cursor cur;
    cur.b = blockIdx.x < p.num_cols ? p.col_b[blockIdx.x] : 0;
    int buf = 0;
    for (int64_t ci = blockIdx.x; ci < p.num_cols; ci += gridDim.x) {
        const int64_t c = visit_col(p, ci);
        if (p.col_mul) cur.b = p.col_b[c];
        else cur.advance(p.col_off, c);
        const int b = cur.b;
        const int T = p.T[b], S = p.S[b];
        const int t = (int)(c - p.col_off[b]);
        const int64_t rowc = p.row_off[b] + (int64_t)t * (S + 1);
        const int64_t arow = acts_col_base(p, b, t, rowc);
        const int lo = max(0, t - (T - S));
        const int hi = min(t, S);
        const double ll = p.ll[b];
        const float sc = scale ? scale[b * p.scale_stride] : 1.0f;
        const Vec zv = splat<IO>(zero_row_value(ll, sc));
        const int *__restrict__ lab_b = p.labels + (int64_t)b * p.label_stride;

        for (int seg = 0; seg <= S; seg += SEG, buf ^= 1) {
            {  // phase A
                const int s = seg + tid;
                float4 cf = make_float4(0.0f, 0.0f, 0.0f, __int_as_float(DEAD));
                if (s >= lo && s <= hi) {
                    const RowCoef rc = row_coef(p, t, T, S, s, rowc + s, ll, lab_b);
                    if (rc.live) cf = make_float4(rc.c2, rc.cb, rc.ce, __int_as_float(rc.lab));
                }
                if (s <= S) coef[buf][tid] = cf;
            }
            __syncthreads();
            const int n = min(SEG, S + 1 - seg);
            for (int i = wave * R; i < n; i += 4 * R) {
                float4 cf[R];
                bool live[R], ok[R];
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    ok[r] = i + r < n;
                    cf[r] = coef[buf][ok[r] ? i + r : i];
                    live[r] = ok[r] && __float_as_int(cf[r].w) != DEAD;
                }
                for (int base = 0; base < VL; base += 64 * U) {
                    Vec x[R][U];
#pragma unroll
                    for (int r = 0; r < R; ++r)
#pragma unroll
                        for (int u = 0; u < U; ++u) {
                            const int j = base + lane + 64 * u;
                            if (live[r] && j < VL)
                                x[r][u] = vload<NTL>(&av[(arow + seg + i + r) * (int64_t)VL + j]);
                        }
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        if (!ok[r]) continue;
                        const RowCoef rc{cf[r].x, cf[r].y, cf[r].z, __float_as_int(cf[r].w), true};
#pragma unroll
                        for (int u = 0; u < U; ++u) {
                            const int j = base + lane + 64 * u;
                            if (j >= VL) continue;
                            const Vec g = live[r] ? grad_vec<IO>(x[r][u], rc, j, blank, sc) : zv;
                            vstore<NTS>(&gv[(arow + seg + i + r) * (int64_t)VL + j], g);
                        }
                    }
                }
            }
        }
    }
}

// Row-stride kernel (grad_variant 3, packed layout only): every wave of the grid sweeps lattice rows in
// memory order (wave w takes rows w, w + nwaves, ...), so the grid streams one contiguous window of acts
// and grads like a grid-stride copy; (b, t, s) of a row come from a per-wave monotone cursor over row_off
// and one 32-bit division.
template <class IO, int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void grad_rows_kernel(DevProblem p, const float *__restrict__ scale,
                                                            void *__restrict__ grads) {
    if (!resolve_dyn(p)) {  // device-resident lengths failed validation: NaN gradients
        fill_failed_grads<IO>(p, grads);
        return;
    }
    typedef typename IO::V Vec;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t gw = (int64_t)blockIdx.x * 4 + wave;
    const int64_t nw = (int64_t)gridDim.x * 4;
    const int VL = p.V / IO::E;
    const int blank = p.blank;
    const Vec *__restrict__ av = reinterpret_cast<const Vec *>(p.acts);
    Vec *__restrict__ gv = reinterpret_cast<Vec *>(grads);

    Cursor cur;
    cur.init(p.row_off, p.B, gw);
    for (int64_t row = gw; row < p.num_rows; row += nw) {
        cur.advance(p.row_off, row);
        const int b = cur.b;
        const int T = p.T[b], S = p.S[b];
        const unsigned loc = (unsigned)(row - p.row_off[b]);
        const int t = (int)(loc / (unsigned)(S + 1));
        const int s = (int)(loc - (unsigned)t * (unsigned)(S + 1));
        const bool inb = s <= t && (S - s) <= (T - t);
        const float sc = scale ? scale[b * p.scale_stride] : 1.0f;
        Vec *__restrict__ out = gv + row * (int64_t)VL;
        RowCoef rc;
        if (inb) rc = row_coef(p, t, T, S, s, row, p.ll[b], p.labels + (int64_t)b * p.label_stride);
        if (!inb || !rc.live) {
            const Vec zv = splat<IO>(zero_row_value(p.ll[b], sc));
            for (int j = lane; j < VL; j += 64) vstore<NTS>(out + j, zv);
            continue;
        }
        for (int base = 0; base < VL; base += 64 * U) {
            Vec x[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int j = base + lane + 64 * u;
                if (j < VL) x[u] = vload<NTL>(&av[row * (int64_t)VL + j]);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int j = base + lane + 64 * u;
                if (j < VL) vstore<NTS>(out + j, grad_vec<IO>(x[u], rc, j, blank, sc));
            }
        }
    }
}

// Scalar path (any V, any alignment): one row per wave, lanes stride over v.
template <class IO>
__global__ __launch_bounds__(256) void grad_scalar_kernel(DevProblem p, const float *__restrict__ scale,
                                                          void *__restrict__ grads) {
    if (!resolve_dyn(p)) {  // device-resident lengths failed validation: NaN gradients
        fill_failed_grads<IO>(p, grads);
        return;
    }
    typedef typename IO::S Sc;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int V = p.V;
    const int blank = p.blank;
    const Sc *__restrict__ acts = reinterpret_cast<const Sc *>(p.acts);
    Sc *__restrict__ gs = reinterpret_cast<Sc *>(grads);
    Cursor cur;
    cur.b = blockIdx.x < p.num_cols ? p.col_b[blockIdx.x] : 0;
    for (int64_t c = blockIdx.x; c < p.num_cols; c += gridDim.x) {
        cur.advance(p.col_off, c);
        const int b = cur.b;
        const int T = p.T[b], S = p.S[b];
        const int t = (int)(c - p.col_off[b]);
        const int64_t rowc = p.row_off[b] + (int64_t)t * (S + 1);
        const int64_t arow = acts_col_base(p, b, t, rowc);
        const int lo = max(0, t - (T - S));
        const int hi = min(t, S);
        const double ll = p.ll[b];
        const float sc = scale ? scale[b * p.scale_stride] : 1.0f;
        const Sc zs = IO::from_f(zero_row_value(ll, sc));
        const int *__restrict__ lab_b = p.labels + (int64_t)b * p.label_stride;
        for (int s = wave; s <= S; s += 4) {
            Sc *__restrict__ g = gs + (arow + s) * (int64_t)V;
            RowCoef rc;
            const bool inb = s >= lo && s <= hi;
            if (inb) rc = row_coef(p, t, T, S, s, rowc + s, ll, lab_b);
            if (!inb || !rc.live) {
                for (int v = lane; v < V; v += 64) g[v] = zs;
                continue;
            }
            const Sc *__restrict__ z = acts + (arow + s) * (int64_t)V;
            for (int v = lane; v < V; v += 64) {
                float gv = fast_exp2(fmaf(IO::to_f(z[v]), kLog2e, rc.c2));
                if (v == blank) gv -= rc.cb;
                else if (v == rc.lab) gv -= rc.ce;
                g[v] = IO::from_f(gv * sc);
            }
        }
    }
}

// Number of in-band rows whose acts the gradient kernels read (live rows; all in-band rows with
// occ_skip = 0). Not on the hot path: bench/inspection only (mrnnt_grad_live_rows).
__global__ __launch_bounds__(256) void count_live_kernel(DevProblem p, unsigned long long *__restrict__ count) {
    resolve_dyn(p);
    __shared__ unsigned long long part[4];
    unsigned long long n = 0;
    Cursor cur;
    cur.b = blockIdx.x < p.num_cols ? p.col_b[blockIdx.x] : 0;
    for (int64_t c = blockIdx.x; c < p.num_cols; c += gridDim.x) {
        cur.advance(p.col_off, c);
        const int b = cur.b;
        const int T = p.T[b], S = p.S[b], W = S + 1;
        const int t = (int)(c - p.col_off[b]);
        const int64_t rowc = p.row_off[b] + (int64_t)t * W;
        const int lo = max(0, t - (T - S));
        const int hi = min(t, S);
        const double ll = p.ll[b];
        for (int s = lo + threadIdx.x; s <= hi; s += blockDim.x) {
            const int64_t row = rowc + s;
            n += (!p.occ_skip || row_live(alpha_prev(p, t, s, row, W) - ll + p.beta[row])) ? 1 : 0;
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) n += __shfl_xor(n, off);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = n;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(count, part[0] + part[1] + part[2] + part[3]);
}

hipError_t launch_count_live(const DevProblem &p, unsigned long long *count, hipStream_t stream) {
    const hipError_t e = hipMemsetAsync(count, 0, sizeof(*count), stream);
    if (e != hipSuccess) return e;
    const int64_t blocks = std::min<int64_t>(std::max<int64_t>(p.num_cols, 1), 2048);
    count_live_kernel<<<(int)blocks, 256, 0, stream>>>(p, count);
    return hipGetLastError();
}

// Padded layout: rows (b, t, s) with t >= T_b or s > S_b are not lattice rows; their gradient is 0.
// One wave per padded row, grid-stride; lattice rows are skipped (written by the gradient kernel).
template <class IO>
__global__ __launch_bounds__(256) void pad_zero_kernel(DevProblem p, void *__restrict__ grads, int vec) {
    if (!resolve_dyn(p)) return;  // the gradient kernel filled the whole buffer with NaN
    typedef typename IO::S Sc;
    typedef typename IO::V Vec;
    const int lane = threadIdx.x & 63;
    const int64_t gw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t nw = (int64_t)gridDim.x * 4;
    const int64_t rows = (int64_t)p.B * p.pad_T * p.pad_S1;
    const int V = p.V;
    for (int64_t row = gw; row < rows; row += nw) {
        const int64_t bt = row / p.pad_S1;
        const int s = (int)(row - bt * p.pad_S1);
        const int b = (int)(bt / p.pad_T);
        const int t = (int)(bt - (int64_t)b * p.pad_T);
        if (t < p.T[b] && s <= p.S[b]) continue;
        if (vec) {
            const int VL = V / IO::E;
            Vec *__restrict__ g = reinterpret_cast<Vec *>(grads) + row * (int64_t)VL;
            const Vec zv = splat<IO>(0.0f);
            for (int j = lane; j < VL; j += 64) vstore<true>(g + j, zv);
        } else {
            Sc *__restrict__ g = reinterpret_cast<Sc *>(grads) + row * (int64_t)V;
            const Sc zs = IO::from_f(0.0f);
            for (int v = lane; v < V; v += 64) g[v] = zs;
        }
    }
}

template <class IO>
static bool vec_ok(const DevProblem &p, const void *grads) {
    return (p.V % IO::E) == 0 && (reinterpret_cast<uintptr_t>(p.acts) % 16) == 0 &&
           (reinterpret_cast<uintptr_t>(grads) % 16) == 0;
}

template <class IO, bool NTL, bool NTS, int U>
static void launch_u(const DevProblem &p, const float *scale, void *grads, int grid, hipStream_t stream) {
    constexpr int RD = U == 4 ? 1 : (U == 2 ? 2 : 4);  // rows per wave: >= 4 KiB of acts in flight per wave
    if constexpr (!kVariants) {  // the product library: the tuned default (grad_variant 5) only
        if constexpr (U == 1 && NTL)
            grad_kernel<IO, U, 2, NTL, NTS><<<grid, 256, 0, stream>>>(p, scale, grads);
        else
            grad_staged_kernel<IO, U, RD, NTL, NTS><<<grid, 256, 0, stream>>>(p, scale, grads);
    } else {
        const int variant = tuning().grad_variant;
        if (variant == 3 && p.pad_S1 == 0)
            grad_rows_kernel<IO, U, NTL, NTS><<<grid, 256, 0, stream>>>(p, scale, grads);
        else if (variant == 0)
            grad_kernel<IO, U, RD, NTL, NTS><<<grid, 256, 0, stream>>>(p, scale, grads);
        else if (variant == 2 || (variant == 5 && U == 1 && NTL))
            // 1 KiB rows streamed from HBM: per-row coefficients, 2 rows per wave (configs[1] shape with nontemporal
            // loads: 50.0 us against 56.3 for 4 rows and 60.2 staged, profiles/r02/kbench/grad_short_rows_c2*.json)
            grad_kernel<IO, U, 2, NTL, NTS><<<grid, 256, 0, stream>>>(p, scale, grads);
        else if (variant == 6)
            grad_staged_kernel<IO, U, 2, NTL, NTS><<<grid, 256, 0, stream>>>(p, scale, grads);
        else  // (1 KiB rows resident in the Infinity Cache, configs[1]: staged, 4 rows per wave, 40.2 against 47.6 us)
            grad_staged_kernel<IO, U, RD, NTL, NTS><<<grid, 256, 0, stream>>>(p, scale, grads);
    }
}

// U = 16-byte vectors per lane per chunk: 4 KiB chunks for rows of >= 192 vectors, 2 KiB for >= 96, else 1 KiB
template <class IO, bool NTL, bool NTS>
static void launch_vec(const DevProblem &p, const float *scale, void *grads, int grid, hipStream_t stream) {
    const int VL = p.V / IO::E;
    if (VL >= 192) launch_u<IO, NTL, NTS, 4>(p, scale, grads, grid, stream);
    else if (VL >= 96) launch_u<IO, NTL, NTS, 2>(p, scale, grads, grid, stream);
    else launch_u<IO, NTL, NTS, 1>(p, scale, grads, grid, stream);
}

template <class IO>
static void launch_io(const DevProblem &p, const float *scale, void *grads, int grid, hipStream_t stream) {
    if (!vec_ok<IO>(p, grads)) {
        grad_scalar_kernel<IO><<<grid, 256, 0, stream>>>(p, scale, grads);
        return;
    }
    const bool ntl = nt_acts_loads(p, sizeof(typename IO::S)), nts = tuning().nt_store != 0;
    if (ntl && nts) launch_vec<IO, true, true>(p, scale, grads, grid, stream);
    else if (ntl) launch_vec<IO, true, false>(p, scale, grads, grid, stream);
    else if (nts) launch_vec<IO, false, true>(p, scale, grads, grid, stream);
    else launch_vec<IO, false, false>(p, scale, grads, grid, stream);
}

hipError_t launch_grad(const DevProblem &p, int elem, const float *scale, void *grads, int grid, hipStream_t stream) {
    switch (elem) {
        case ELEM_F32: launch_io<IoF32>(p, scale, grads, grid, stream); break;
        case ELEM_BF16: launch_io<IoBF16>(p, scale, grads, grid, stream); break;
        case ELEM_F16: launch_io<IoF16>(p, scale, grads, grid, stream); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_pad_zero(const DevProblem &p, int elem, void *grads, hipStream_t stream) {
    if (p.pad_S1 == 0) return hipSuccess;
    const int64_t rows = (int64_t)p.B * p.pad_T * p.pad_S1;
    if (rows == 0) return hipSuccess;
    int64_t blocks = (rows + 3) / 4;
    if (blocks > 8192) blocks = 8192;
    switch (elem) {
        case ELEM_F32:
            pad_zero_kernel<IoF32><<<(int)blocks, 256, 0, stream>>>(p, grads, (int)vec_ok<IoF32>(p, grads));
            break;
        case ELEM_BF16:
            pad_zero_kernel<IoBF16><<<(int)blocks, 256, 0, stream>>>(p, grads, (int)vec_ok<IoBF16>(p, grads));
            break;
        case ELEM_F16:
            pad_zero_kernel<IoF16><<<(int)blocks, 256, 0, stream>>>(p, grads, (int)vec_ok<IoF16>(p, grads));
            break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// Nontemporal zero fill, each workgroup streaming contiguous slabs in turn: the gradient pass's store stream
// without its loads. The Python surface times it once over a new large grads buffer (placement probe).
typedef unsigned int fill_u4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void fill_zero_kernel(fill_u4 *__restrict__ dst, int64_t n, int64_t slab) {
    const fill_u4 z = {0u, 0u, 0u, 0u};
    for (int64_t c0 = (int64_t)blockIdx.x * slab; c0 < n; c0 += (int64_t)gridDim.x * slab) {
        const int64_t end = min(c0 + slab, n);
        for (int64_t i = c0 + threadIdx.x; i < end; i += 256) __builtin_nontemporal_store(z, &dst[i]);
    }
}

hipError_t launch_fill_zero(void *dst, size_t bytes, int grid_max, hipStream_t stream) {
    const int64_t n = (int64_t)(bytes / 16);
    if (n <= 0) return hipSuccess;
    // >= 8 slabs per workgroup (one slab each would time the launch tail); 16 KiB .. 800 KiB slabs
    const int64_t slab = std::min<int64_t>(50 * 1024, std::max<int64_t>(1024, n / ((int64_t)grid_max * 8) / 1024 * 1024));
    const int64_t blocks = std::min<int64_t>((n + slab - 1) / slab, grid_max);
    fill_zero_kernel<<<(int)blocks, 256, 0, stream>>>(static_cast<fill_u4 *>(dst), n, slab);
    return hipGetLastError();
}

}  // namespace mrnnt
