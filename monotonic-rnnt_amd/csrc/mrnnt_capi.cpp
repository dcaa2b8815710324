// mrnnt_capi.cpp -- host side of libmonotonic_rnnt_amd.so: validation, workspace plan, kernel
// orchestration on the caller's stream, the flat C ABI (include/mrnnt.h), and the reference-shaped
// C++ surface (include/rnnt_entrypoint.h, gpu_workspace_manager.h, gpu_rnnt.h).
//
// No host synchronisation happens inside mrnnt_forward / mrnnt_backward (the reference synchronises
// after each reduce and copies T/S/band arrays to the host every call: reduce.h:162,
// gpu_rnnt.h:28-35). The only sync is in the reference-compatible compute_rnnt_loss /
// GpuRNNTComputer path, whose contract returns host costs (gpu_rnnt.h:229).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <random>
#include <string>
#include <vector>

// The library is built with -fvisibility=hidden: only the declarations of the public headers below are
// exported (the kernels and launchers in mrnnt_internal.h stay internal).
#pragma GCC visibility push(default)
#include "cpu_rnnt.h"
#include "cpu_workspace_manager.h"
#include "gpu_rnnt.h"
#include "gpu_workspace_manager.h"
#include "mrnnt.h"
#include "rnnt_entrypoint.h"
#pragma GCC visibility pop
#include "mrnnt_internal.h"

using namespace mrnnt;

namespace {

// this thread's mrnnt_last_error() (the error state lives in mrnnt_entry.cpp)
RNNTStatus fail(RNNTStatus st, const std::string &msg) { return mrnnt::set_error(st, msg); }

RNNTStatus fail_hip(hipError_t e, const char *where) {
    return fail(RNNT_STATUS_EXECUTION_FAILED, std::string(where) + ": " + hipGetErrorString(e));
}

constexpr size_t kAlign = 256;
size_t align_up(size_t x) { return (x + kAlign - 1) / kAlign * kAlign; }

// Launch plan of one problem. With host lengths every size is exact. With device-resident lengths
// (lengths_on_device) the host plans from bounds it knows without a read-back: N = the rows of acts (packed: exact,
// checked on the device; padded: B*pad_T*pad_S1), cols <= N (packed; every column holds >= 1 row) or B*pad_T
// (padded), S_max <= label_stride; the setup kernel publishes the real values (DynWords) for the kernels.
struct Plan {
    int B = 0, V = 0, S_max = 0, T_max = 0;
    int64_t N = 0, cols = 0;
    int elem = ELEM_F32;
    int64_t pad_T = 0, pad_S1 = 0;
    bool align = false;
    bool dyn = false;
    size_t off_flags = 0, flags_bytes = 0;  // the chase launch's ready flags (8 bytes per column), where it can run
    size_t off_row, off_col, off_colb, off_mtmp, off_min, off_max, off_den, off_lp, off_alpha, off_beta, off_ll,
        off_llb, off_dyn, total;
};

int cu_count_of_device() {
    static int cu_count[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    if (cu_count[dev] == 0) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cu_count[dev] = n;
    }
    return cu_count[dev];
}

// Mean frames per utterance: exact with host lengths; with device lengths the plan's lower bound on the column count
// over B (exact when every S_b equals the label row stride), or pad_T for the padded layout.
double mean_frames(const Plan &pl) {
    if (!pl.dyn) return (double)pl.cols / pl.B;
    if (pl.pad_S1) return (double)pl.pad_T;
    return (double)((pl.N + pl.S_max) / (pl.S_max + 1)) / pl.B;
}

// The chase launch (mrnnt_chase.hip) where its shape allows it and it pays:
// * f32 rows it has a body for, no alignment band, the halo recursion in one 4-wave workgroup (S + 1 <= 4 * 56), the
//   lp array one buffer descriptor (N * 16 bytes < 2^31), device lengths for B <= 64 (one utterance per lane);
// * its recursion workgroups spin while they wait, so together they should leave the chip to the producers: at most
//   one per CU (B or 2B <= CUs). (Progress does not rely on it -- a starved recursion wave computes its columns
//   itself -- but a launch that has to is slow.)
// * it saves the recursion's time (~T steps of ~0.1 us) at the price of a slightly slower log-softmax pass (+5-10 %,
//   the hand-off and the production order): taken when the recursion is at least a quarter of the pass's streaming
//   time (configs[1]: 20 vs 22 us; the headline: 0.16 vs 6.5 ms, not taken).
bool chase_shape_ok(const Plan &pl) {
    if (pl.align || pl.elem != ELEM_F32 || chase_body_shape(pl.V) < 0) return false;
    if (pl.S_max + 1 > 4 * 56 || pl.N * (int64_t)sizeof(Lp) >= ((int64_t)1 << 31)) return false;
    if (pl.dyn && pl.B > 64) return false;
    // one recursion workgroup per utterance and direction: the cost-only forward needs B of them, the gradient call 2B
    // (chase_pays decides per call). The flags are sized here, so the workspace size depends on the CU count of the
    // device current when the plan is made (a problem of B > CUs utterances never takes the chase).
    if (pl.B > cu_count_of_device()) return false;
    const double pass_s = (double)pl.N * pl.V * 4.0 / 6.0e12, recursion_s = mean_frames(pl) * 1.0e-7;
    return recursion_s >= 0.25 * pass_s;
}

bool chase_pays(const Plan &pl, bool with_beta) {
    return pl.flags_bytes && (with_beta ? 2 * pl.B : pl.B) <= cu_count_of_device();
}

RNNTStatus plan_device_lengths(const mrnnt_problem *p, Plan &q) {
    if (!p->T_dev || !p->S_dev) return fail(RNNT_STATUS_INVALID_VALUE, "device lengths are required");
    if (p->lattice)
        return fail(RNNT_STATUS_INVALID_VALUE, "lattice must be NULL with lengths_on_device (built on the device)");
    if (p->num_rows < 0) return fail(RNNT_STATUS_INVALID_VALUE, "num_rows is required with lengths_on_device");
    if (p->label_stride < 0) return fail(RNNT_STATUS_INVALID_VALUE, "negative label row stride");
    if (p->pad_S1 != 0) {
        if (p->pad_S1 < 1 || p->pad_T < 1) return fail(RNNT_STATUS_INVALID_VALUE, "padded layout needs pad_T, pad_S1 >= 1");
        q.N = (int64_t)p->B * p->pad_T * p->pad_S1;
        q.cols = (int64_t)p->B * p->pad_T;
        q.T_max = (int)std::min<int64_t>(p->pad_T, 1 << 30);
        q.S_max = (int)std::min<int64_t>(p->label_stride, p->pad_S1 - 1);
    } else {
        q.N = p->num_rows;
        q.cols = q.N;
        q.T_max = (int)std::min<int64_t>(q.N, 1 << 30);
        q.S_max = (int)std::min<int64_t>(p->label_stride, 1 << 30);
    }
    if (q.S_max + 1 > kMaxLabelsPlusOne)
        return fail(RNNT_STATUS_INVALID_VALUE, "with device lengths the label row stride (" +
                                                   std::to_string(p->label_stride) + ") bounds S_b and must be <= " +
                                                   std::to_string(kMaxLabelsPlusOne - 1) +
                                                   ": pass labels no wider than the longest label sequence");
    if (p->num_rows != q.N)
        return fail(RNNT_STATUS_INVALID_VALUE, "acts has " + std::to_string(p->num_rows) + " rows but the padded layout needs " +
                                                   std::to_string(q.N));
    return RNNT_STATUS_SUCCESS;
}

RNNTStatus make_plan(const mrnnt_problem *p, Plan *pl) {
    if (!p) return fail(RNNT_STATUS_INVALID_VALUE, "null problem");
    if (p->B <= 0) return fail(RNNT_STATUS_INVALID_VALUE, "B must be > 0");
    if (p->V <= 0) return fail(RNNT_STATUS_INVALID_VALUE, "V must be > 0");
    const bool dyn = p->lengths_on_device != 0;
    if (!dyn && (!p->T_host || !p->S_host)) return fail(RNNT_STATUS_INVALID_VALUE, "host lengths are required");
    if (p->blank < 0 || p->blank >= p->V) return fail(RNNT_STATUS_INVALID_VALUE, "blank label out of range [0, V)");
    Plan q;
    q.B = p->B;
    q.V = p->V;
    q.dyn = dyn;
    if (dyn) {
        const RNNTStatus st = plan_device_lengths(p, q);
        if (st != RNNT_STATUS_SUCCESS) return st;
    }
    for (int b = 0; !dyn && b < p->B; ++b) {
        const int T = p->T_host[b], S = p->S_host[b];
        // reference validation: cpu_workspace_manager.h:103-107 / gpu_workspace_manager.h:235-239
        if (T <= 0 || S < 0 || T < S)
            return fail(RNNT_STATUS_INVALID_VALUE, "invalid lengths at utterance " + std::to_string(b) + ": T=" +
                                                       std::to_string(T) + " S=" + std::to_string(S) +
                                                       " (need T > 0, S >= 0, T >= S)");
        q.N += (int64_t)T * (S + 1);
        q.cols += T;
        q.S_max = std::max(q.S_max, S);
        q.T_max = std::max(q.T_max, T);
    }
    if (q.S_max + 1 > kMaxLabelsPlusOne)
        return fail(RNNT_STATUS_INVALID_VALUE, "max label length " + std::to_string(q.S_max) + " exceeds " +
                                                   std::to_string(kMaxLabelsPlusOne - 1));
    // the kernels read labels[b * label_stride + s] for s < S_b and alignment[b * align_stride + t] for t < T_b
    // (with device lengths the setup kernel checks S_b <= label_stride and T_b <= align_stride)
    if (q.S_max > 0 && p->label_stride < q.S_max)
        return fail(RNNT_STATUS_INVALID_VALUE, "label row stride " + std::to_string(p->label_stride) +
                                                   " < max label length " + std::to_string(q.S_max));
    if (!dyn && p->alignment && p->align_stride < q.T_max)
        return fail(RNNT_STATUS_INVALID_VALUE, "alignment row stride " + std::to_string(p->align_stride) +
                                                   " < max input length " + std::to_string(q.T_max));
    if (dyn && p->alignment && p->align_stride < 1)
        return fail(RNNT_STATUS_INVALID_VALUE, "alignment row stride must be >= 1");
    if (p->acts_dtype != ELEM_F32 && p->acts_dtype != ELEM_BF16 && p->acts_dtype != ELEM_F16)
        return fail(RNNT_STATUS_INVALID_VALUE, "unknown acts_dtype " + std::to_string(p->acts_dtype));
    q.elem = p->acts_dtype;
    q.pad_T = p->pad_T;
    q.pad_S1 = p->pad_S1;
    int64_t acts_rows = q.N;
    if (dyn) {
        // sizes are bounds (plan_device_lengths); nothing more to check on the host
    } else if (q.pad_S1 != 0) {
        if (q.pad_S1 < (int64_t)q.S_max + 1 || q.pad_T < q.T_max)
            return fail(RNNT_STATUS_INVALID_VALUE, "padded layout [B, " + std::to_string(q.pad_T) + ", " +
                                                       std::to_string(q.pad_S1) + ", V] too small for max T " +
                                                       std::to_string(q.T_max) + ", max S " + std::to_string(q.S_max));
        acts_rows = (int64_t)q.B * q.pad_T * q.pad_S1;
    }
    if (p->num_rows >= 0 && p->num_rows != acts_rows)
        return fail(RNNT_STATUS_INVALID_VALUE, "acts has " + std::to_string(p->num_rows) + " rows but the " +
                                                   (q.pad_S1 ? "padded layout needs " : "lattice needs sum_b T_b(S_b+1) = ") +
                                                   std::to_string(acts_rows));
    q.align = p->alignment != nullptr;
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t at = o;
        o = align_up(o + bytes);
        return at;
    };
    q.off_row = take(sizeof(int64_t) * (q.B + 1));
    q.off_col = take(sizeof(int64_t) * (q.B + 1));
    q.off_colb = take(sizeof(int) * q.cols);
    q.off_den = take(sizeof(float) * q.N);
    q.off_lp = take(sizeof(Lp) * (q.N + 2 * kLpPad));
    q.off_alpha = take(sizeof(double) * q.N);
    q.off_beta = take(sizeof(double) * q.N);
    q.off_ll = take(sizeof(double) * q.B);
    q.off_llb = take(sizeof(double) * q.B);
    // the alignment band after the per-row state, so the state's offsets do not depend on the alignment flag (the
    // C++ manager's band getter rebuilds the band in a workspace that holds the state of an earlier computation)
    q.off_mtmp = q.align ? take(sizeof(int) * (q.cols + q.B)) : 0;
    q.off_min = q.align ? take(sizeof(int) * q.cols) : 0;
    q.off_max = q.align ? take(sizeof(int) * q.cols) : 0;
    q.off_dyn = q.dyn ? take(sizeof(DynWords)) : 0;
    // the chase launch's ready flags (mrnnt_chase.hip), one word per column (device lengths: per column of the bound),
    // for problems whose shape can take it -- last, so no other offset depends on it
    if (chase_shape_ok(q)) {
        q.flags_bytes = sizeof(unsigned long long) * (size_t)q.cols;
        q.off_flags = take(q.flags_bytes);
    }
    q.total = o;
    *pl = q;
    return RNNT_STATUS_SUCCESS;
}

// mrnnt_status_word(): one host-mapped word per process, and its device address
std::mutex g_status_mu;
int *g_status_host = nullptr;
int *g_status_dev = nullptr;

// Device address of a caller's status word (host-mapped memory), nullptr for none.
RNNTStatus status_device_ptr(const mrnnt_problem *p, int **dev) {
    *dev = nullptr;
    if (!p->status_host) return RNNT_STATUS_SUCCESS;
    {
        std::lock_guard<std::mutex> lk(g_status_mu);
        if (p->status_host == g_status_host) {
            *dev = g_status_dev;
            return RNNT_STATUS_SUCCESS;
        }
    }
    void *d = nullptr;
    if (hipHostGetDevicePointer(&d, p->status_host, 0) != hipSuccess || !d)
        return fail(RNNT_STATUS_INVALID_VALUE, "status_host is not host-mapped memory (use mrnnt_status_word())");
    *dev = static_cast<int *>(d);
    return RNNT_STATUS_SUCCESS;
}

// A multiplier spreading consecutive column indices over the whole lattice: the first prime >= 0.618 cols
// that does not divide cols (so i -> i * m mod cols is a permutation).
int64_t scatter_mul(int64_t cols) {
    if (cols < 3) return 0;
    for (int64_t m = std::max<int64_t>(2, (int64_t)(0.6180339887 * (double)cols));; ++m) {
        bool prime = true;
        for (int64_t f = 2; f * f <= m && prime; ++f) prime = (m % f) != 0;
        if (prime && cols % m != 0) return m;
    }
}

// A fresh 64-bit tag per chase launch (mrnnt_chase.hip): a bijective mix of a process-wide counter whose start is
// random per process, so no two calls of a process share one and a stale word matches with probability 2^-64.
uint64_t chase_epoch() {
    static std::atomic<uint64_t> ctr{((uint64_t)std::random_device{}() << 32) ^ (uint64_t)std::random_device{}() ^
                                     (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count()};
    uint64_t x = ctr.fetch_add(1, std::memory_order_relaxed) * 0x9E3779B97F4A7C15ull;
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x ? x : 1;
}

DevProblem make_dev(const mrnnt_problem *p, const Plan &pl, const void *ws) {
    char *w = static_cast<char *>(const_cast<void *>(ws));
    DevProblem d;
    d.acts = p->acts;
    d.labels = p->labels;
    d.label_stride = p->label_stride;
    d.T = p->T_dev;
    d.S = p->S_dev;
    if (p->lattice) {  // caller-provided lattice offsets (mrnnt_lattice_host layout)
        const int64_t *lat = static_cast<const int64_t *>(p->lattice);
        d.row_off = lat;
        d.col_off = lat + pl.B + 1;
        d.col_b = reinterpret_cast<const int *>(lat + 2 * (pl.B + 1));
    } else {
        d.row_off = reinterpret_cast<const int64_t *>(w + pl.off_row);
        d.col_off = reinterpret_cast<const int64_t *>(w + pl.off_col);
        d.col_b = reinterpret_cast<const int *>(w + pl.off_colb);
    }
    d.min_s = pl.align ? reinterpret_cast<const int *>(w + pl.off_min) : nullptr;
    d.max_s = pl.align ? reinterpret_cast<const int *>(w + pl.off_max) : nullptr;
    d.B = pl.B;
    d.V = pl.V;
    d.blank = p->blank;
    d.occ_skip = tuning().occ_skip;
    d.num_cols = pl.cols;
    d.num_rows = pl.N;
    d.pad_T = pl.pad_T;
    d.pad_S1 = pl.pad_S1;
    d.scale_stride = p->grad_scale_broadcast ? 0 : 1;
    d.col_mul = 0;  // set per pass by mrnnt_forward / mrnnt_backward (tuning().col_scatter)
    d.den = reinterpret_cast<float *>(w + pl.off_den);
    d.lp = reinterpret_cast<Lp *>(w + pl.off_lp) + kLpPad;
    d.alpha = reinterpret_cast<double *>(w + pl.off_alpha);
    d.beta = reinterpret_cast<double *>(w + pl.off_beta);
    d.ll = reinterpret_cast<double *>(w + pl.off_ll);
    d.llb = reinterpret_cast<double *>(w + pl.off_llb);
    d.dyn = pl.dyn ? reinterpret_cast<DynWords *>(w + pl.off_dyn) : nullptr;
    d.steal = 0;
    d.dyn_fused = 0;
    d.s_cap = d.t_cap = d.s1_cap = 0;
    d.scatter_above = INT64_MAX;
    d.status_host = nullptr;
    return d;
}

// Column order of a streaming pass (DevProblem::col_mul): XCD-chunked (< 0), scattered (> 0: with device lengths a
// marker the kernels replace by the device's multiplier, resolve_dyn) or in order (0). bit: 1 log-softmax, 2 gradient.
int64_t column_order(const Plan &pl, int bit) {
    if (tuning().col_xcd & bit) return -1;
    if (!(tuning().col_scatter & bit)) return 0;
    return pl.dyn ? 1 : scatter_mul(pl.cols);
}

// Workgroups of 4 waves per CU of the log-softmax's persistent, work-stealing grid (device-resident lengths: the
// host does not know the column count to launch one workgroup per column)
constexpr int kStealGridPerCU = 16;

RNNTStatus check_pointers(const mrnnt_problem *p) {
    if (!p->acts) return fail(RNNT_STATUS_INVALID_VALUE, "acts is null");
    if (!p->T_dev || !p->S_dev) return fail(RNNT_STATUS_INVALID_VALUE, "device lengths are required");
    if (!p->labels) return fail(RNNT_STATUS_INVALID_VALUE, "labels is null");
    return RNNT_STATUS_SUCCESS;
}

// ---- device properties -------------------------------------------------------------------------

int streaming_grid(int64_t cols, int per_cu) {
    static int cu_count[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    if (cu_count[dev] == 0) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cu_count[dev] = n;
    }
    // per_cu workgroups of 4 waves per CU walking the columns grid-stride, never more than the columns;
    // per_cu == 0: one workgroup per column (hardware-scheduled)
    // (the hardware-scheduled grid is capped at 2^22 workgroups: the dispatch size in work-items is 32-bit, and
    // every streaming kernel walks its columns grid-stride, so larger problems just take more than one turn)
    const int64_t g = per_cu <= 0 ? std::min<int64_t>(cols, 1 << 22) : (int64_t)cu_count[dev] * per_cu;
    return (int)std::max<int64_t>(1, std::min<int64_t>(g, cols));
}

// ---- profiling ---------------------------------------------------------------------------------

struct ProfRec {
    int id;
    hipEvent_t a, b;
};
std::mutex g_prof_mu;
bool g_prof_on = false;
std::vector<ProfRec> g_prof;
// events are created ahead (mrnnt_profile_enable) and recycled, so a timed launch adds two event records and
// no hipEventCreate to the host path it measures (that matters for 0.1 ms steps)
std::vector<hipEvent_t> g_event_pool;
constexpr size_t kEventPrealloc = 2048;

// timing-only events: no system-scope fence at record (a cache writeback + invalidate between the timed kernels
// would slow the launches being measured)
hipError_t make_timing_event(hipEvent_t *e) { return hipEventCreateWithFlags(e, hipEventDisableSystemFence); }

hipEvent_t pooled_event() {  // g_prof_mu held
    if (!g_event_pool.empty()) {
        const hipEvent_t e = g_event_pool.back();
        g_event_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    return make_timing_event(&e) == hipSuccess ? e : nullptr;
}

template <class F>
hipError_t timed(int id, hipStream_t s, F &&launch) {
    ProfRec r{id, nullptr, nullptr};
    {
        std::lock_guard<std::mutex> lk(g_prof_mu);
        if (!g_prof_on) return launch();
        r.a = pooled_event();
        r.b = pooled_event();
        if (!r.a || !r.b) {
            if (r.a) g_event_pool.push_back(r.a);
            if (r.b) g_event_pool.push_back(r.b);
            r.a = r.b = nullptr;
        }
    }
    if (!r.a) return launch();
    (void)hipEventRecord(r.a, s);
    const hipError_t e = launch();
    (void)hipEventRecord(r.b, s);
    std::lock_guard<std::mutex> lk(g_prof_mu);
    g_prof.push_back(r);
    return e;
}

}  // namespace

// =================================================================================================
// flat C ABI

extern "C" {

// mrnnt_version, mrnnt_last_error, mrnnt_lattice_bytes / mrnnt_lattice_host: mrnnt_entry.cpp (host-only)

RNNTStatus mrnnt_workspace_size(const mrnnt_problem *p, size_t *bytes) {
    if (!bytes) return fail(RNNT_STATUS_INVALID_VALUE, "null size pointer");
    Plan pl;
    const RNNTStatus st = make_plan(p, &pl);
    if (st != RNNT_STATUS_SUCCESS) return st;
    *bytes = pl.total;
    return RNNT_STATUS_SUCCESS;
}

RNNTStatus mrnnt_forward(const mrnnt_problem *p, void *ws, size_t ws_bytes, float *costs_dev, int with_beta,
                         hipStream_t stream) {
    Plan pl;
    RNNTStatus st = make_plan(p, &pl);
    if (st != RNNT_STATUS_SUCCESS) return st;
    if ((st = check_pointers(p)) != RNNT_STATUS_SUCCESS) return st;
    if (!ws || ws_bytes < pl.total)
        return fail(RNNT_STATUS_INVALID_VALUE, "workspace too small: need " + std::to_string(pl.total) + " bytes");
    DevProblem d = make_dev(p, pl, ws);
    char *w = static_cast<char *>(ws);
    hipError_t e = hipSuccess;
    // device-resident lengths of a small batch without an alignment: planned inside the log-softmax launch itself
    // (every wave holds the lengths in registers, walk_columns in mrnnt_device.h) -- no separate setup kernel, whose
    // ~4.7 us launch would be 5 % of a configs[1] step; otherwise one setup kernel before the passes
    const bool fused = pl.dyn && pl.B <= 64 && !pl.align && tuning().softmax_grid_per_cu <= 0 && tuning().dyn_fused;
    const int64_t scatter_above = ((tuning().col_scatter & 3) != 0 && !(tuning().col_xcd & 3))
                                      ? (int64_t)streaming_grid(pl.cols, tuning().grad_grid_per_cu)
                                      : INT64_MAX;
    if (pl.dyn && !fused) {  // device-resident lengths: offsets, column map and validation in one launch, no read-back
        DynSetupArgs a;
        std::memset(&a, 0, sizeof(a));
        if ((st = status_device_ptr(p, &a.status_host)) != RNNT_STATUS_SUCCESS) return st;
        a.T = p->T_dev;
        a.S = p->S_dev;
        a.B = pl.B;
        a.packed = pl.pad_S1 == 0;
        a.rows = pl.N;
        a.cols_cap = pl.cols;
        a.S_cap = pl.S_max;
        a.T_cap = pl.pad_S1 ? pl.pad_T : 0;
        if (p->alignment) a.T_cap = a.T_cap ? std::min<int64_t>(a.T_cap, p->align_stride) : p->align_stride;
        a.S1_cap = pl.pad_S1;
        // the scattered order only matters where a workgroup walks several columns: the gradient's persistent grid
        // (the log-softmax's default is in order)
        a.scatter_above = scatter_above;
        a.row_off = reinterpret_cast<int64_t *>(w + pl.off_row);
        a.col_off = reinterpret_cast<int64_t *>(w + pl.off_col);
        a.col_b = reinterpret_cast<int *>(w + pl.off_colb);
        a.lp = d.lp;
        a.dyn = d.dyn;
        e = timed(K_SETUP, stream, [&] { return launch_setup_dyn(a, stream); });
        if (e != hipSuccess) return fail_hip(e, "device-lengths setup kernel");
    } else if (!pl.dyn && !p->lattice) {  // lattice offsets on the device (the log-softmax kernel zeroes the lp pads)
        e = timed(K_SETUP, stream, [&] {
            return launch_setup(p->T_dev, p->S_dev, pl.B, reinterpret_cast<int64_t *>(w + pl.off_row),
                                reinterpret_cast<int64_t *>(w + pl.off_col),
                                reinterpret_cast<int *>(w + pl.off_colb), nullptr, 0, stream);
        });
        if (e != hipSuccess) return fail_hip(e, "setup kernel");
    }
    if (pl.align) {
        e = timed(K_BAND, stream, [&] {
            return launch_align(d, p->alignment, p->align_stride, p->align_blank, p->max_shift,
                                reinterpret_cast<int *>(w + pl.off_mtmp), reinterpret_cast<int *>(w + pl.off_min),
                                reinterpret_cast<int *>(w + pl.off_max), stream);
        });
        if (e != hipSuccess) return fail_hip(e, "alignment band kernels");
    }
    // no alignment: the forward as one launch, the recursion chasing the log-softmax (mrnnt_chase.hip), where it has a
    // body for these rows and pays (chase_pays); with device lengths the launch also plans and validates them
    if (tuning().chase && chase_body(d, pl.elem) >= 0 && chase_pays(pl, with_beta) && (!pl.dyn || fused)) {
        ChaseArgs ca;
        ca.flags = reinterpret_cast<unsigned long long *>(w + pl.off_flags);
        // device lengths: the slots come from the lengths on the device; the grid from the plan's column bound
        // (rows / (label stride + 1), exact when every S_b equals the stride; + B for the middle frames of odd T)
        const int64_t slot_bound = pl.dyn ? (pl.pad_S1 ? pl.cols : (pl.N + pl.S_max) / (pl.S_max + 1)) + pl.B
                                          : chase_slots(pl.B, pl.T_max, with_beta ? 1 : 0);
        ca.slots = pl.dyn ? 0 : slot_bound;
        ca.epoch = chase_epoch();
        ca.budget = (uint32_t)std::min<int64_t>((int64_t)std::max(0, tuning().chase_wait_us) * 100, UINT32_MAX / 2);
        ca.delay = kVariants ? (uint32_t)std::max(0, tuning().chase_delay_us) * 100u : 0u;
        ca.stage = kVariants ? tuning().chase_stage : 1;
        ca.probe = kVariants ? tuning().chase_probe : 0;
        ca.pair = kVariants ? tuning().chase_pair : 1;
        ca.early_free = kVariants ? tuning().chase_early_free : 1;
        ca.ring = kVariants ? tuning().chase_ring : 64;
        const int nrec = with_beta ? 2 * pl.B : pl.B;
        const int producers = (int)std::min<int64_t>(streaming_grid(slot_bound, tuning().chase_grid_per_cu),
                                                     ((int64_t)1 << 22) - nrec);
        DevProblem dc = d;
        if (pl.dyn) {  // validation limits and the status report, as the fused log-softmax launch (walk_columns)
            dc.s_cap = pl.S_max;
            dc.t_cap = pl.pad_S1 ? pl.pad_T : 0;
            dc.s1_cap = pl.pad_S1;
            dc.scatter_above = scatter_above;
            if ((st = status_device_ptr(p, &dc.status_host)) != RNNT_STATUS_SUCCESS) return st;
        }
        e = timed(K_CHASE, stream, [&] {
            return launch_chase(dc, ca, pl.elem, pl.S_max, with_beta ? 1 : 0, producers, costs_dev, stream);
        });
        if (e != hipSuccess) return fail_hip(e, "chase kernel");
        return RNNT_STATUS_SUCCESS;
    }
    int grid = streaming_grid(pl.cols, tuning().softmax_grid_per_cu);
    DevProblem ds = d;  // the log-softmax launch's view
    ds.col_mul = column_order(pl, 1);
    if (fused) {
        // one workgroup per column at the lower bound of the column count, rows / (label stride + 1) (exact when every
        // S_b equals the stride; more columns are walked grid-stride), or B * pad_T for the padded layout
        const int64_t lower = pl.pad_S1 ? pl.cols : (pl.N + pl.S_max) / (pl.S_max + 1);
        grid = (int)std::max<int64_t>(1, std::min<int64_t>(lower, 1 << 22));
        ds.dyn_fused = 1;
        ds.s_cap = pl.S_max;
        ds.t_cap = pl.pad_S1 ? pl.pad_T : 0;
        ds.s1_cap = pl.pad_S1;
        ds.scatter_above = scatter_above;
        ds.col_mul = 0;
        if ((st = status_device_ptr(p, &ds.status_host)) != RNNT_STATUS_SUCCESS) return st;
    } else if (pl.dyn && tuning().softmax_grid_per_cu <= 0) {  // one workgroup per column needs the column count
        grid = streaming_grid(pl.cols, kStealGridPerCU);
        ds.steal = grid < pl.cols;
    }
    e = timed(K_SOFTMAX, stream, [&] { return launch_softmax(ds, pl.elem, grid, stream); });
    if (e != hipSuccess) return fail_hip(e, "log-softmax kernel");
    e = timed(K_DP, stream, [&] { return launch_dp(d, pl.S_max, with_beta ? 1 : 0, costs_dev, stream); });
    if (e != hipSuccess) return fail_hip(e, "alpha/beta kernel");
    return RNNT_STATUS_SUCCESS;
}

RNNTStatus mrnnt_backward(const mrnnt_problem *p, const void *ws, const float *grad_scale, void *grads,
                          hipStream_t stream) {
    Plan pl;
    RNNTStatus st = make_plan(p, &pl);
    if (st != RNNT_STATUS_SUCCESS) return st;
    if ((st = check_pointers(p)) != RNNT_STATUS_SUCCESS) return st;
    if (!ws) return fail(RNNT_STATUS_INVALID_VALUE, "workspace is null");
    if (!grads) return fail(RNNT_STATUS_INVALID_VALUE, "grads is null");
    DevProblem d = make_dev(p, pl, ws);
    d.col_mul = column_order(pl, 2);
    // grad_variant 3 sweeps rows (packed layout only), the others walk lattice columns
    const int grid = (tuning().grad_variant == 3 && pl.pad_S1 == 0)
                         ? streaming_grid(pl.N, std::max(1, tuning().grad_grid_per_cu))
                         : streaming_grid(pl.cols, tuning().grad_grid_per_cu);
    hipError_t e = timed(K_GRAD, stream, [&] { return launch_grad(d, pl.elem, grad_scale, grads, grid, stream); });
    if (e != hipSuccess) return fail_hip(e, "gradient kernel");
    if (pl.pad_S1 != 0) {
        e = launch_pad_zero(d, pl.elem, grads, stream);
        if (e != hipSuccess) return fail_hip(e, "padding-rows zero kernel");
    }
    return RNNT_STATUS_SUCCESS;
}

RNNTStatus mrnnt_cost_and_grad(const mrnnt_problem *p, void *ws, size_t ws_bytes, float *costs_dev, void *grads,
                               const float *grad_scale, hipStream_t stream) {
    RNNTStatus st = mrnnt_forward(p, ws, ws_bytes, costs_dev, grads != nullptr, stream);
    if (st != RNNT_STATUS_SUCCESS || grads == nullptr) return st;
    return mrnnt_backward(p, ws, grad_scale, grads, stream);
}

RNNTStatus mrnnt_read_loglik(const mrnnt_problem *p, const void *ws, double *ll_fwd_dev, double *ll_bwd_dev,
                             hipStream_t stream) {
    Plan pl;
    RNNTStatus st = make_plan(p, &pl);
    if (st != RNNT_STATUS_SUCCESS) return st;
    const char *w = static_cast<const char *>(ws);
    if (ll_fwd_dev && hipMemcpyAsync(ll_fwd_dev, w + pl.off_ll, sizeof(double) * pl.B, hipMemcpyDeviceToDevice,
                                     stream) != hipSuccess)
        return fail(RNNT_STATUS_MEMOPS_FAILED, "copy ll_fwd");
    if (ll_bwd_dev && hipMemcpyAsync(ll_bwd_dev, w + pl.off_llb, sizeof(double) * pl.B, hipMemcpyDeviceToDevice,
                                     stream) != hipSuccess)
        return fail(RNNT_STATUS_MEMOPS_FAILED, "copy ll_bwd");
    return RNNT_STATUS_SUCCESS;
}

RNNTStatus mrnnt_read_state(const mrnnt_problem *p, const void *ws, float *den_dev, double *alpha_dev,
                            double *beta_dev, hipStream_t stream) {
    Plan pl;
    RNNTStatus st = make_plan(p, &pl);
    if (st != RNNT_STATUS_SUCCESS) return st;
    if (!ws) return fail(RNNT_STATUS_INVALID_VALUE, "workspace is null");
    const DevProblem d = make_dev(p, pl, ws);
    if (den_dev && hipMemcpyAsync(den_dev, d.den, sizeof(float) * pl.N, hipMemcpyDeviceToDevice, stream) != hipSuccess)
        return fail(RNNT_STATUS_MEMOPS_FAILED, "copy den");
    if (alpha_dev &&
        hipMemcpyAsync(alpha_dev, d.alpha, sizeof(double) * pl.N, hipMemcpyDeviceToDevice, stream) != hipSuccess)
        return fail(RNNT_STATUS_MEMOPS_FAILED, "copy alpha");
    if (beta_dev && hipMemcpyAsync(beta_dev, d.beta, sizeof(double) * pl.N, hipMemcpyDeviceToDevice, stream) != hipSuccess)
        return fail(RNNT_STATUS_MEMOPS_FAILED, "copy beta");
    if ((alpha_dev || beta_dev) && launch_mask_state(d, alpha_dev, beta_dev, stream) != hipSuccess)
        return fail(RNNT_STATUS_EXECUTION_FAILED, "mask state");
    return RNNT_STATUS_SUCCESS;
}

RNNTStatus mrnnt_read_denoms(const mrnnt_problem *p, const void *ws, float *den_dev, hipStream_t stream) {
    Plan pl;
    RNNTStatus st = make_plan(p, &pl);
    if (st != RNNT_STATUS_SUCCESS) return st;
    if ((st = check_pointers(p)) != RNNT_STATUS_SUCCESS) return st;
    if (!ws || !den_dev) return fail(RNNT_STATUS_INVALID_VALUE, "workspace / den is null");
    const hipError_t e = launch_den_all(make_dev(p, pl, ws), pl.elem, den_dev, stream);
    if (e != hipSuccess) return fail_hip(e, "denominator read-out kernel");
    return RNNT_STATUS_SUCCESS;
}

RNNTStatus mrnnt_read_band(const mrnnt_problem *p, void *ws, int *min_dev, int *max_dev, int64_t ld,
                           hipStream_t stream) {
    Plan pl;
    RNNTStatus st = make_plan(p, &pl);
    if (st != RNNT_STATUS_SUCCESS) return st;
    if (!ws) return fail(RNNT_STATUS_INVALID_VALUE, "workspace is null");
    if (!p->T_dev || !p->S_dev) return fail(RNNT_STATUS_INVALID_VALUE, "device lengths are required");
    if (ld < 1 || (!pl.dyn && ld < pl.T_max))
        return fail(RNNT_STATUS_INVALID_VALUE, "band row stride " + std::to_string(ld) + " < max input length");
    DevProblem d = make_dev(p, pl, ws);
    char *w = static_cast<char *>(ws);
    hipError_t e = hipSuccess;
    if (pl.dyn) {  // offsets + validation exactly as mrnnt_forward builds them
        DynSetupArgs a;
        std::memset(&a, 0, sizeof(a));
        a.T = p->T_dev;
        a.S = p->S_dev;
        a.B = pl.B;
        a.packed = pl.pad_S1 == 0;
        a.rows = pl.N;
        a.cols_cap = pl.cols;
        a.S_cap = pl.S_max;
        a.T_cap = pl.pad_S1 ? pl.pad_T : 0;
        if (p->alignment) a.T_cap = a.T_cap ? std::min<int64_t>(a.T_cap, p->align_stride) : p->align_stride;
        a.S1_cap = pl.pad_S1;
        a.scatter_above = INT64_MAX;
        a.row_off = reinterpret_cast<int64_t *>(w + pl.off_row);
        a.col_off = reinterpret_cast<int64_t *>(w + pl.off_col);
        a.col_b = reinterpret_cast<int *>(w + pl.off_colb);
        a.dyn = d.dyn;
        e = launch_setup_dyn(a, stream);
    } else if (!p->lattice) {
        e = launch_setup(p->T_dev, p->S_dev, pl.B, reinterpret_cast<int64_t *>(w + pl.off_row),
                         reinterpret_cast<int64_t *>(w + pl.off_col), reinterpret_cast<int *>(w + pl.off_colb), nullptr, 0,
                         stream);
    }
    if (e != hipSuccess) return fail_hip(e, "setup kernel");
    if (pl.align) {
        e = launch_align(d, p->alignment, p->align_stride, p->align_blank, p->max_shift,
                         reinterpret_cast<int *>(w + pl.off_mtmp), reinterpret_cast<int *>(w + pl.off_min),
                         reinterpret_cast<int *>(w + pl.off_max), stream);
        if (e != hipSuccess) return fail_hip(e, "alignment band kernels");
    }
    if ((e = launch_band_read(d, min_dev, max_dev, ld, stream)) != hipSuccess) return fail_hip(e, "band read-out kernel");
    return RNNT_STATUS_SUCCESS;
}

int *mrnnt_status_word(void) {
    std::lock_guard<std::mutex> lk(g_status_mu);
    if (!g_status_host) {
        void *h = nullptr, *d = nullptr;
        if (hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent) != hipSuccess)
            return nullptr;
        if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
            (void)hipHostFree(h);
            return nullptr;
        }
        std::memset(h, 0, 64);
        g_status_host = static_cast<int *>(h);
        g_status_dev = static_cast<int *>(d);
    }
    return g_status_host;
}

RNNTStatus mrnnt_grad_live_rows(const mrnnt_problem *p, const void *ws, unsigned long long *count_dev,
                                hipStream_t stream) {
    Plan pl;
    RNNTStatus st = make_plan(p, &pl);
    if (st != RNNT_STATUS_SUCCESS) return st;
    if ((st = check_pointers(p)) != RNNT_STATUS_SUCCESS) return st;
    if (!ws || !count_dev) return fail(RNNT_STATUS_INVALID_VALUE, "workspace / count is null");
    const hipError_t e = launch_count_live(make_dev(p, pl, ws), count_dev, stream);
    if (e != hipSuccess) return fail_hip(e, "live-row count kernel");
    return RNNT_STATUS_SUCCESS;
}

// ---- fused joint network + loss ------------------------------------------------------------------

}  // extern "C"

namespace {

struct JointPlan {
    Plan base;
    int64_t n_inband = 0;
    size_t off_cnt = 0, off_lcol = 0, off_ls = 0, off_total = 0, off_wplain = 0, off_dbias = 0, total = 0;
};

mrnnt_problem base_problem(const mrnnt_joint_problem *jp) {
    mrnnt_problem p;
    std::memset(&p, 0, sizeof(p));
    p.B = jp->B;
    p.V = jp->V;
    p.blank = jp->blank;
    p.T_host = jp->T_host;
    p.S_host = jp->S_host;
    p.T_dev = jp->T_dev;
    p.S_dev = jp->S_dev;
    p.acts = jp->enc;  // the lattice kernels never read acts on this path
    p.labels = jp->labels;
    p.label_stride = jp->label_stride;
    p.alignment = jp->alignment;
    p.align_stride = jp->align_stride;
    p.align_blank = jp->align_blank;
    p.max_shift = jp->max_shift;
    p.num_rows = -1;
    return p;
}

bool aligned16(const void *ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15) == 0; }

RNNTStatus make_joint_plan(const mrnnt_joint_problem *jp, JointPlan *jl) {
    if (!jp) return fail(RNNT_STATUS_INVALID_VALUE, "null joint problem");
    const mrnnt_problem p = base_problem(jp);
    JointPlan q;
    RNNTStatus st = make_plan(&p, &q.base);
    if (st != RNNT_STATUS_SUCCESS) return st;
    const int H = jp->H;
    if (H != 128 && H != 256 && H != 384 && H != 512 && H != 640)
        return fail(RNNT_STATUS_INVALID_VALUE, "joint H must be 128, 256, 384, 512 or 640 (got " + std::to_string(H) + ")");
    if (joint_min_lds_bytes(H, jp->V) > 160 * 1024)
        return fail(RNNT_STATUS_INVALID_VALUE, "V = " + std::to_string(jp->V) + " is too large for the fused joint kernels at H = " +
                                                   std::to_string(H) + " (weight tiles + bias need " +
                                                   std::to_string(joint_min_lds_bytes(H, jp->V) / 1024) +
                                                   " KiB of LDS, 160 KiB per CU); use the unfused loss");
    if (jp->enc_stride % 8 || jp->pred_stride % 8)
        return fail(RNNT_STATUS_INVALID_VALUE, "enc/pred utterance strides must be multiples of 8 elements");
    if (jp->hact_ld != 0 && (jp->hact_ld < H || jp->hact_ld % 8))
        return fail(RNNT_STATUS_INVALID_VALUE, "hact_ld must be 0 or a multiple of 8 that is >= H");
    if (jp->enc_stride < (int64_t)q.base.T_max * H || jp->pred_stride < (int64_t)(q.base.S_max + 1) * H)
        return fail(RNNT_STATUS_INVALID_VALUE, "enc/pred utterance strides smaller than max T * H / (max S + 1) * H");
    for (int b = 0; b < jp->B; ++b) {
        const int T = jp->T_host[b], S = jp->S_host[b];
        for (int t = 0; t < T; ++t) q.n_inband += std::min(t, S) - std::max(0, t - (T - S)) + 1;
    }
    size_t o = q.base.total;
    auto take = [&](size_t bytes) {
        const size_t at = o;
        o = align_up(o + bytes);
        return at;
    };
    // per-column counts + their exclusive scan, and the scan's tile sums (launch_row_list)
    q.off_cnt = take(sizeof(int64_t) * (q.base.cols + 2 + (q.base.cols + 1023) / 1024));
    q.off_lcol = take(sizeof(int) * std::max<int64_t>(1, q.n_inband));
    q.off_ls = take(sizeof(int) * std::max<int64_t>(1, q.n_inband));
    q.off_total = take(sizeof(unsigned long long));
    q.off_wplain = take(sizeof(int));  // the forward's weight-bound flag (launch_joint_wbound)
    // the gradient pass's per-workgroup dbias column sums (fixed-order reduction), when there is a bias
    q.off_dbias = (jp->bias && H <= 512) ? take(joint_dbias_part_bytes(std::max<int64_t>(1, q.n_inband), jp->V)) : 0;
    q.total = o;
    *jl = q;
    return RNNT_STATUS_SUCCESS;
}

RNNTStatus check_joint_pointers(const mrnnt_joint_problem *jp) {
    if (!jp->enc || !jp->pred || !jp->weight) return fail(RNNT_STATUS_INVALID_VALUE, "enc / pred / weight is null");
    if (!aligned16(jp->enc) || !aligned16(jp->pred) || !aligned16(jp->weight))
        return fail(RNNT_STATUS_INVALID_VALUE, "enc / pred / weight must be 16-byte aligned");
    if (!jp->T_dev || !jp->S_dev) return fail(RNNT_STATUS_INVALID_VALUE, "device lengths are required");
    if (!jp->labels) return fail(RNNT_STATUS_INVALID_VALUE, "labels is null");
    return RNNT_STATUS_SUCCESS;
}

JointArgs joint_args(const mrnnt_joint_problem *jp, const JointPlan &jl, void *ws, int64_t n) {
    char *w = static_cast<char *>(ws);
    JointArgs j;
    std::memset(&j, 0, sizeof(j));
    j.enc = static_cast<const unsigned short *>(jp->enc);
    j.enc_sb = jp->enc_stride;
    j.pred = static_cast<const unsigned short *>(jp->pred);
    j.pred_sb = jp->pred_stride;
    j.W = static_cast<const unsigned short *>(jp->weight);
    j.bias = jp->bias;
    j.H = jp->H;
    j.hact_ld = jp->hact_ld ? jp->hact_ld : jp->H;
    j.lcol = reinterpret_cast<const int *>(w + jl.off_lcol);
    j.ls = reinterpret_cast<const int *>(w + jl.off_ls);
    j.n = n;
    j.opt = kVariants ? tuning().joint_opt : 3;
    return j;
}

}  // namespace

extern "C" {

RNNTStatus mrnnt_joint_workspace_size(const mrnnt_joint_problem *jp, size_t *bytes) {
    if (!bytes) return fail(RNNT_STATUS_INVALID_VALUE, "null size pointer");
    JointPlan jl;
    const RNNTStatus st = make_joint_plan(jp, &jl);
    if (st != RNNT_STATUS_SUCCESS) return st;
    *bytes = jl.total;
    return RNNT_STATUS_SUCCESS;
}

RNNTStatus mrnnt_joint_row_bound(const mrnnt_joint_problem *jp, int64_t *rows) {
    if (!rows) return fail(RNNT_STATUS_INVALID_VALUE, "null rows pointer");
    JointPlan jl;
    const RNNTStatus st = make_joint_plan(jp, &jl);
    if (st != RNNT_STATUS_SUCCESS) return st;
    *rows = jl.n_inband;
    return RNNT_STATUS_SUCCESS;
}

RNNTStatus mrnnt_joint_forward(const mrnnt_joint_problem *jp, void *ws, size_t ws_bytes, float *costs_dev,
                               int with_beta, hipStream_t stream) {
    JointPlan jl;
    RNNTStatus st = make_joint_plan(jp, &jl);
    if (st != RNNT_STATUS_SUCCESS) return st;
    if ((st = check_joint_pointers(jp)) != RNNT_STATUS_SUCCESS) return st;
    if (!ws || ws_bytes < jl.total)
        return fail(RNNT_STATUS_INVALID_VALUE, "workspace too small: need " + std::to_string(jl.total) + " bytes");
    const Plan &pl = jl.base;
    const mrnnt_problem p = base_problem(jp);
    DevProblem d = make_dev(&p, pl, ws);
    char *w = static_cast<char *>(ws);
    hipError_t e = timed(K_SETUP, stream, [&] {
        return launch_setup(jp->T_dev, jp->S_dev, pl.B, reinterpret_cast<int64_t *>(w + pl.off_row),
                            reinterpret_cast<int64_t *>(w + pl.off_col),
                            reinterpret_cast<int *>(w + pl.off_colb), nullptr, 0, stream);
    });
    if (e != hipSuccess) return fail_hip(e, "setup kernel");
    if (pl.align) {
        e = timed(K_BAND, stream, [&] {
            return launch_align(d, p.alignment, p.align_stride, p.align_blank, p.max_shift,
                                reinterpret_cast<int *>(w + pl.off_mtmp), reinterpret_cast<int *>(w + pl.off_min),
                                reinterpret_cast<int *>(w + pl.off_max), stream);
        });
        if (e != hipSuccess) return fail_hip(e, "alignment band kernels");
    }
    // out-of-band lp entries must be finite for the recursion (the acts path zero-fills them in its pass)
    if ((e = launch_zero(w + pl.off_lp, pl.off_alpha - pl.off_lp, stream)) != hipSuccess)
        return fail_hip(e, "lp zero fill");
    e = launch_row_list(d, 0, reinterpret_cast<int64_t *>(w + jl.off_cnt), reinterpret_cast<int *>(w + jl.off_lcol),
                        reinterpret_cast<int *>(w + jl.off_ls), reinterpret_cast<unsigned long long *>(w + jl.off_total),
                        stream);
    if (e != hipSuccess) return fail_hip(e, "row list kernels");
    JointArgs j = joint_args(jp, jl, ws, jl.n_inband);
    if (pl.align) j.n_dev = reinterpret_cast<const unsigned long long *>(w + jl.off_total);  // alignment windows
    // the weight bound decides the forward's epilogue on the device (no host sync): counted in the forward's time
    int *wplain = reinterpret_cast<int *>(w + jl.off_wplain);
    j.wplain = wplain;
    e = timed(K_JOINT_FWD, stream, [&] {
        const hipError_t eb = launch_joint_wbound(j.W, j.bias, jp->V, jp->H, wplain, stream);
        return eb != hipSuccess ? eb : launch_joint_forward(d, j, stream);
    });
    if (e != hipSuccess) return fail_hip(e, "joint log-softmax kernel");
    e = timed(K_DP, stream, [&] { return launch_dp(d, pl.S_max, with_beta ? 1 : 0, costs_dev, stream); });
    if (e != hipSuccess) return fail_hip(e, "alpha/beta kernel");
    return RNNT_STATUS_SUCCESS;
}

RNNTStatus mrnnt_joint_live_rows(const mrnnt_joint_problem *jp, void *ws, unsigned long long *count_dev,
                                 hipStream_t stream) {
    JointPlan jl;
    RNNTStatus st = make_joint_plan(jp, &jl);
    if (st != RNNT_STATUS_SUCCESS) return st;
    if (!ws || !count_dev) return fail(RNNT_STATUS_INVALID_VALUE, "workspace / count is null");
    const mrnnt_problem p = base_problem(jp);
    DevProblem d = make_dev(&p, jl.base, ws);
    char *w = static_cast<char *>(ws);
    hipError_t e = launch_row_list(d, 1, reinterpret_cast<int64_t *>(w + jl.off_cnt),
                                   reinterpret_cast<int *>(w + jl.off_lcol), reinterpret_cast<int *>(w + jl.off_ls),
                                   count_dev, stream);
    if (e != hipSuccess) return fail_hip(e, "live row list kernels");
    return RNNT_STATUS_SUCCESS;
}

RNNTStatus mrnnt_joint_backward(const mrnnt_joint_problem *jp, void *ws, int64_t n_live, const float *grad_scale,
                                void *G, void *Hact, int64_t *bt_idx, int64_t *bs_idx, hipStream_t stream) {
    JointPlan jl;
    RNNTStatus st = make_joint_plan(jp, &jl);
    if (st != RNNT_STATUS_SUCCESS) return st;
    if ((st = check_joint_pointers(jp)) != RNNT_STATUS_SUCCESS) return st;
    if (!ws) return fail(RNNT_STATUS_INVALID_VALUE, "workspace is null");
    if (n_live < 0 || n_live > jl.n_inband)
        return fail(RNNT_STATUS_INVALID_VALUE, "n_live outside [0, in-band rows]");
    if (n_live > 0 && (!G || !Hact)) return fail(RNNT_STATUS_INVALID_VALUE, "G / Hact is null");
    if (n_live > 0 && (!aligned16(G) || !aligned16(Hact)))
        return fail(RNNT_STATUS_INVALID_VALUE, "G / Hact must be 16-byte aligned");
    const mrnnt_problem p = base_problem(jp);
    DevProblem d = make_dev(&p, jl.base, ws);
    JointArgs j = joint_args(jp, jl, ws, n_live);
    j.n_dev = jp->live_count_dev;  // n_live a host bound: workgroups past the device count exit (their rows zeroed below)
    j.G = static_cast<unsigned short *>(G);
    j.Hact = static_cast<unsigned short *>(Hact);
    j.bt_idx = bt_idx;
    j.bs_idx = bs_idx;
    j.scale = grad_scale;
    j.dbias = jp->dbias;
    if (jp->dbias && jp->H > 512) return fail(RNNT_STATUS_INVALID_VALUE, "dbias in the gradient pass needs H <= 512");
    if (jp->dbias && joint_dbias_lds_bytes(jp->H, jp->V) > 160 * 1024)
        return fail(RNNT_STATUS_INVALID_VALUE, "dbias in the gradient pass: V too large for its LDS column sums at this H "
                                               "(sum G's columns outside: dbias = NULL)");
    if (jp->dbias && !jl.off_dbias)
        return fail(RNNT_STATUS_INVALID_VALUE, "dbias needs a bias (the workspace holds its partial sums only then)");
    if (jp->dbias) j.dbias_part = reinterpret_cast<float *>(static_cast<char *>(ws) + jl.off_dbias);
    hipError_t e = timed(K_JOINT_BWD, stream, [&] {
        const hipError_t eb = launch_joint_backward(d, j, stream);
        if (eb != hipSuccess || !jp->live_count_dev) return eb;
        return launch_joint_tail_zero(j.G, jp->V, j.Hact, j.hact_ld, n_live, jp->live_count_dev, stream);
    });
    if (e != hipSuccess) return fail_hip(e, "joint gradient kernel");
    if (jp->dbias && n_live > 0) {
        e = launch_joint_dbias_sum(j, jp->V, stream);
        if (e != hipSuccess) return fail_hip(e, "joint dbias sum kernels");
    }
    return RNNT_STATUS_SUCCESS;
}

// pre: dH already holds dpre (Hact unused; the kRedPre kernel form)
static RNNTStatus joint_reduce(const mrnnt_joint_problem *jp, void *ws, int64_t n_live, const void *dH,
                               const void *Hact, bool pre, float *d_enc, float *d_pred, hipStream_t stream) {
    JointPlan jl;
    RNNTStatus st = make_joint_plan(jp, &jl);
    if (st != RNNT_STATUS_SUCCESS) return st;
    if ((st = check_joint_pointers(jp)) != RNNT_STATUS_SUCCESS) return st;
    if (!ws || !d_enc || !d_pred) return fail(RNNT_STATUS_INVALID_VALUE, "workspace / d_enc / d_pred is null");
    if (n_live < 0 || n_live > jl.n_inband) return fail(RNNT_STATUS_INVALID_VALUE, "n_live outside [0, in-band rows]");
    if (n_live > 0 && (!dH || (reinterpret_cast<uintptr_t>(dH) & 7)))
        return fail(RNNT_STATUS_INVALID_VALUE, pre ? "dpre null or not 8-byte aligned" : "dH null or not 8-byte aligned");
    if (!pre && n_live > 0 && (!Hact || (reinterpret_cast<uintptr_t>(Hact) & 7)))
        return fail(RNNT_STATUS_INVALID_VALUE, "Hact null or not 8-byte aligned (a dH that already holds dpre: "
                                               "mrnnt_joint_reduce_pre)");
    const mrnnt_problem p = base_problem(jp);
    DevProblem d = make_dev(&p, jl.base, ws);
    JointArgs j = joint_args(jp, jl, ws, n_live);
    j.Hact = pre ? nullptr : static_cast<unsigned short *>(const_cast<void *>(Hact));
    const int64_t *off = reinterpret_cast<const int64_t *>(static_cast<char *>(ws) + jl.off_cnt);
    const hipError_t e = timed(K_JOINT_RED, stream, [&] {
        return launch_joint_reduce(d, j, off, jl.base.T_max, jl.base.S_max, static_cast<const unsigned short *>(dH),
                                   d_enc, d_pred, jp->reduce_scratch, jp->reduce_scratch_bytes, stream);
    });
    if (e != hipSuccess) return fail_hip(e, "joint reduce kernel");
    return RNNT_STATUS_SUCCESS;
}

RNNTStatus mrnnt_joint_reduce(const mrnnt_joint_problem *jp, void *ws, int64_t n_live, const void *dH,
                              const void *Hact, float *d_enc, float *d_pred, hipStream_t stream) {
    return joint_reduce(jp, ws, n_live, dH, Hact, false, d_enc, d_pred, stream);
}

RNNTStatus mrnnt_joint_reduce_pre(const mrnnt_joint_problem *jp, void *ws, int64_t n_live, const void *dpre,
                                  float *d_enc, float *d_pred, hipStream_t stream) {
    return joint_reduce(jp, ws, n_live, dpre, nullptr, true, d_enc, d_pred, stream);
}

RNNTStatus mrnnt_joint_dpre(const mrnnt_joint_problem *jp, int64_t n_live, const void *G, const void *weight_t,
                            const void *Hact, void *dpre, hipStream_t stream) {
    JointPlan jl;
    RNNTStatus st = make_joint_plan(jp, &jl);
    if (st != RNNT_STATUS_SUCCESS) return st;
    if (jp->H != 256 && jp->H != 512)
        return fail(RNNT_STATUS_INVALID_VALUE, "mrnnt_joint_dpre: H must be 256 or 512 (use a library GEMM)");
    if (jp->V % 8) return fail(RNNT_STATUS_INVALID_VALUE, "mrnnt_joint_dpre: V must be a multiple of 8");
    if (n_live < 0 || n_live > jl.n_inband) return fail(RNNT_STATUS_INVALID_VALUE, "n_live outside [0, in-band rows]");
    const int64_t ld = jp->hact_ld ? jp->hact_ld : jp->H;
    if (ld < jp->H || ld % 4) return fail(RNNT_STATUS_INVALID_VALUE, "hact_ld must be >= H and a multiple of 4");
    if (n_live == 0) return RNNT_STATUS_SUCCESS;
    for (const void *q : {G, weight_t, Hact, static_cast<const void *>(dpre)})
        if (!q || (reinterpret_cast<uintptr_t>(q) & 15))
            return fail(RNNT_STATUS_INVALID_VALUE, "mrnnt_joint_dpre: G / weight_t / Hact / dpre null or not 16-byte aligned");
    const hipError_t e = timed(K_JOINT_DPRE, stream, [&] {
        return launch_joint_dpre(static_cast<const unsigned short *>(G), static_cast<const unsigned short *>(weight_t),
                                 static_cast<const unsigned short *>(Hact), ld, static_cast<unsigned short *>(dpre),
                                 n_live, jp->V, jp->H, stream);
    });
    if (e != hipSuccess) return fail_hip(e, "joint dpre kernel");
    return RNNT_STATUS_SUCCESS;
}

RNNTStatus mrnnt_joint_reduce_scratch_bytes(const mrnnt_joint_problem *jp, size_t *bytes) {
    if (!bytes) return fail(RNNT_STATUS_INVALID_VALUE, "null size pointer");
    JointPlan jl;
    const RNNTStatus st = make_joint_plan(jp, &jl);
    if (st != RNNT_STATUS_SUCCESS) return st;
    *bytes = joint_reduce_scratch_bytes(jl.base.B, jl.base.T_max, jl.base.S_max, jp->H);
    return RNNT_STATUS_SUCCESS;
}

RNNTStatus mrnnt_fill_zero(void *dst, size_t bytes, hipStream_t stream) {
    if (bytes == 0) return RNNT_STATUS_SUCCESS;
    if (!dst || (reinterpret_cast<uintptr_t>(dst) & 15) || (bytes & 15))
        return fail(RNNT_STATUS_INVALID_VALUE, "fill_zero: null or not 16-byte aligned pointer / size");
    const hipError_t e = launch_fill_zero(dst, bytes, streaming_grid((int64_t)1 << 40, 32), stream);
    if (e != hipSuccess) return fail_hip(e, "zero fill kernel");
    return RNNT_STATUS_SUCCESS;
}

void mrnnt_profile_enable(int enable) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    for (auto &r : g_prof) {  // recycled: a record still pending is complete before the event is recorded again
        g_event_pool.push_back(r.a);
        g_event_pool.push_back(r.b);
    }
    g_prof.clear();
    g_prof_on = enable != 0;
    while (g_prof_on && g_event_pool.size() < kEventPrealloc) {
        hipEvent_t e = nullptr;
        if (make_timing_event(&e) != hipSuccess) break;
        g_event_pool.push_back(e);
    }
}

int mrnnt_profile_read(double *total_ms, int64_t *launches, int n) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    for (int i = 0; i < n; ++i) {
        if (total_ms) total_ms[i] = 0.0;
        if (launches) launches[i] = 0;
    }
    int bad = 0;
    for (auto &r : g_prof) {
        if (hipEventSynchronize(r.b) != hipSuccess) {
            ++bad;
            continue;
        }
        float ms = 0.0f;
        if (hipEventElapsedTime(&ms, r.a, r.b) != hipSuccess) {
            ++bad;
            continue;
        }
        if (r.id < n) {
            if (total_ms) total_ms[r.id] += ms;
            if (launches) launches[r.id] += 1;
        }
    }
    return bad;
}

#ifdef MRNNT_DEVTOOLS
// development build: columns chase recursion waves computed themselves since the last reset (mrnnt_chase.hip)
__attribute__((visibility("default"))) unsigned long long mrnnt_chase_helped(int reset) { return chase_helped(reset != 0); }
__attribute__((visibility("default"))) int mrnnt_chase_trace(unsigned long long *out, int n) { return chase_trace(out, n); }
__attribute__((visibility("default"))) int mrnnt_chase_walk_trace(unsigned long long *out, int n) {
    return chase_walk_trace(out, n);
}
__attribute__((visibility("default"))) int mrnnt_joint_trace(unsigned long long *out, int n) { return joint_trace(out, n); }
__attribute__((visibility("default"))) int mrnnt_joint_reduce_trace(unsigned long long *out, int n) {
    return joint_reduce_trace(out, n);
}

// launch knobs: exported by the development build only (libmonotonic_rnnt_amd_dev.so, `make dev`)
__attribute__((visibility("default"))) int mrnnt_tune(const char *key, int value) {
    if (!key) return -1;
    int *slot = nullptr;
    Tuning &t = tuning();
    if (!std::strcmp(key, "softmax_variant")) slot = &t.softmax_variant;
    else if (!std::strcmp(key, "grad_variant")) slot = &t.grad_variant;
    else if (!std::strcmp(key, "col_scatter")) slot = &t.col_scatter;
    else if (!std::strcmp(key, "col_xcd")) slot = &t.col_xcd;
    else if (!std::strcmp(key, "dp_halo")) slot = &t.dp_halo;
    else if (!std::strcmp(key, "dp_lean")) slot = &t.dp_lean;
    else if (!std::strcmp(key, "joint_reduce_sparse")) slot = &t.joint_reduce_sparse;
    else if (!std::strcmp(key, "joint_dpre_nw")) slot = &t.joint_dpre_nw;
    else if (!std::strcmp(key, "joint_dpre_abl")) slot = &t.joint_dpre_abl;
    else if (!std::strcmp(key, "joint_reduce_hact")) slot = &t.joint_reduce_hact;
    else if (!std::strcmp(key, "joint_probe")) slot = &t.joint_probe;
    else if (!std::strcmp(key, "joint_opt")) slot = &t.joint_opt;
    else if (!std::strcmp(key, "joint_trace")) slot = &t.joint_trace;
    else if (!std::strcmp(key, "joint_reduce_pad")) slot = &t.joint_reduce_pad;
    else if (!std::strcmp(key, "softmax_grid_per_cu")) slot = &t.softmax_grid_per_cu;
    else if (!std::strcmp(key, "grad_grid_per_cu")) slot = &t.grad_grid_per_cu;
    else if (!std::strcmp(key, "grid_per_cu")) {  // both streaming kernels
        const int prev = t.grad_grid_per_cu;
        if (value >= 0) t.softmax_grid_per_cu = t.grad_grid_per_cu = value;
        return prev;
    }
    else if (!std::strcmp(key, "nt_store")) slot = &t.nt_store;
    else if (!std::strcmp(key, "dyn_fused")) slot = &t.dyn_fused;
    else if (!std::strcmp(key, "chase")) slot = &t.chase;
    else if (!std::strcmp(key, "chase_wait_us")) slot = &t.chase_wait_us;
    else if (!std::strcmp(key, "chase_stage")) slot = &t.chase_stage;
    else if (!std::strcmp(key, "chase_delay_us")) slot = &t.chase_delay_us;
    else if (!std::strcmp(key, "chase_probe")) slot = &t.chase_probe;
    else if (!std::strcmp(key, "chase_pair")) slot = &t.chase_pair;
    else if (!std::strcmp(key, "chase_early_free")) slot = &t.chase_early_free;
    else if (!std::strcmp(key, "chase_ring")) slot = &t.chase_ring;
    else if (!std::strcmp(key, "chase_grid_per_cu")) slot = &t.chase_grid_per_cu;
    else if (!std::strcmp(key, "nt_load")) slot = &t.nt_load;
    else if (!std::strcmp(key, "occ_skip")) slot = &t.occ_skip;
    else if (!std::strcmp(key, "joint_bwd_mfma")) slot = &t.joint_bwd_mfma;
    if (!slot) return -1;
    const int prev = *slot;
    if (value >= 0) *slot = value;
    return prev;
}
#endif  // MRNNT_DEVTOOLS

}  // extern "C"

// =================================================================================================
// reference-shaped C++ surface: GpuRNNTWorkspaceManager<float>, GpuRNNTComputer<float>,
// compute_rnnt_loss (reference gpu_workspace_manager.h, gpu_rnnt.h, src/rnnt_entrypoint.cpp)

struct mrnnt_gpu_ws_state {
    const float *acts;
    const int *labels;
    int B, V;
    const int *T_dev;
    const int *S_dev;
    void *workspace = nullptr;
    bool owned = false;
    const int *alignment = nullptr;
    int max_shift = 0;
    int align_blank = 0;
    // the last computation on the workspace (what the inspection getters read back)
    bool computed = false;
    bool with_beta = false;
    int blank = 0;
    hipStream_t stream = nullptr;
};

namespace {

// Host copies of T/S (the reference makes the same D2H copies, gpu_workspace_manager.h:87-96), ordered on `stream`.
bool host_lengths(const mrnnt_gpu_ws_state *s, std::vector<int> &T, std::vector<int> &S, hipStream_t stream = nullptr) {
    T.assign(s->B, 0);
    S.assign(s->B, 0);
    if (s->B <= 0) return true;
    if (hipMemcpyAsync(T.data(), s->T_dev, sizeof(int) * s->B, hipMemcpyDeviceToHost, stream) != hipSuccess) return false;
    if (hipMemcpyAsync(S.data(), s->S_dev, sizeof(int) * s->B, hipMemcpyDeviceToHost, stream) != hipSuccess) return false;
    return hipStreamSynchronize(stream) == hipSuccess;
}

mrnnt_problem problem_of(const mrnnt_gpu_ws_state *s, const std::vector<int> &T, const std::vector<int> &S,
                         int blank) {
    mrnnt_problem p;
    std::memset(&p, 0, sizeof(p));
    p.B = s->B;
    p.V = s->V;
    p.blank = blank;
    p.T_host = T.data();
    p.S_host = S.data();
    p.T_dev = s->T_dev;
    p.S_dev = s->S_dev;
    p.acts = s->acts;
    p.labels = s->labels;
    // reference quirks kept on this surface: label row stride = max(S) (gpu_rnnt_kernel.h:133),
    // alignment row stride = max(T) (gpu_workspace_manager.h:200)
    p.label_stride = S.empty() ? 0 : *std::max_element(S.begin(), S.end());
    p.alignment = s->alignment;
    p.align_stride = T.empty() ? 0 : *std::max_element(T.begin(), T.end());
    p.align_blank = s->align_blank;
    p.max_shift = s->max_shift;
    p.num_rows = -1;
    return p;
}

// The reference manager's public view (gpu_workspace_manager.h:58-85, laid out in its order, :228-254, 301-346).
struct RefView {
    size_t denom, alphas, betas, dsi, vso, llf, llb, B, V, Smax, Tmax, mn, mx, total;
};

RefView ref_view_layout(int B, int64_t N, int T_max) {
    RefView v;
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t at = o;
        o += bytes;
        return at;
    };
    v.denom = take(sizeof(float) * N);
    v.alphas = take(sizeof(float) * N);
    v.betas = take(sizeof(float) * N);
    v.dsi = take(sizeof(int) * B);
    v.vso = take(sizeof(int) * B);
    v.llf = take(sizeof(float) * B);
    v.llb = take(sizeof(float) * B);
    v.B = take(sizeof(int));
    v.V = take(sizeof(int));
    v.Smax = take(sizeof(int));
    v.Tmax = take(sizeof(int));
    v.mn = take(sizeof(int) * (size_t)B * T_max);
    v.mx = take(sizeof(int) * (size_t)B * T_max);
    v.total = o;
    return v;
}

// The manager's workspace = the flat plan + B device floats for the costs + the reference's view. The view's offset
// is fixed by the larger of the plans with and without an alignment (restrict_to_alignment may come after
// set_workspace); the costs follow the plan of the current call.
RNNTStatus manager_size(const mrnnt_gpu_ws_state *s, const std::vector<int> &T, const std::vector<int> &S,
                        size_t *bytes, size_t *costs_off, size_t *view_off = nullptr) {
    mrnnt_problem p = problem_of(s, T, S, 0);
    // size only depends on lengths and the alignment flag; blank range is checked at compute time
    size_t b = 0, b_max = 0;
    RNNTStatus st = mrnnt_workspace_size(&p, &b);
    if (st != RNNT_STATUS_SUCCESS) return st;
    int dummy = 0;
    p.alignment = p.alignment ? p.alignment : &dummy;
    p.align_stride = T.empty() ? 0 : *std::max_element(T.begin(), T.end());
    if ((st = mrnnt_workspace_size(&p, &b_max)) != RNNT_STATUS_SUCCESS) return st;
    p.alignment = nullptr;
    size_t b_plain = 0;
    if ((st = mrnnt_workspace_size(&p, &b_plain)) != RNNT_STATUS_SUCCESS) return st;
    b_max = std::max(b_max, b_plain);
    *costs_off = align_up(b);
    const size_t voff = align_up(align_up(b_max) + sizeof(float) * std::max(1, s->B));
    int64_t N = 0;
    for (size_t i = 0; i < T.size(); ++i) N += (int64_t)T[i] * (S[i] + 1);
    const int T_max = T.empty() ? 0 : *std::max_element(T.begin(), T.end());
    *bytes = voff + ref_view_layout(s->B, N, T_max).total;
    if (view_off) *view_off = voff;
    return RNNT_STATUS_SUCCESS;
}

RNNTStatus manager_compute(GpuRNNTWorkspaceManager<float> &wm, int blank, hipStream_t stream, float *costs,
                           float *grads) {
    mrnnt_gpu_ws_state *s = wm.state();
    if (!costs) return fail(RNNT_STATUS_INVALID_VALUE, "costs is null");
    if (!s->workspace) return fail(RNNT_STATUS_INVALID_VALUE, "workspace not set (set_workspace/create_workspace)");
    std::vector<int> T, S;
    if (!host_lengths(s, T, S, stream)) return fail(RNNT_STATUS_MEMOPS_FAILED, "copying lengths to host");
    size_t bytes = 0, coff = 0;
    RNNTStatus st = manager_size(s, T, S, &bytes, &coff);
    if (st != RNNT_STATUS_SUCCESS) return st;
    mrnnt_problem p = problem_of(s, T, S, blank);
    // this surface synchronises anyway (host costs): read the labels back and range-check them, as the flat
    // entry points cannot without a sync (there an out-of-range device label gives a non-finite cost). The copy
    // is ordered on the caller's stream, after whatever produced the labels there.
    if (p.label_stride > 0) {
        std::vector<int> lab((size_t)s->B * p.label_stride);
        if (hipMemcpyAsync(lab.data(), s->labels, sizeof(int) * lab.size(), hipMemcpyDeviceToHost, stream) !=
                hipSuccess ||
            hipStreamSynchronize(stream) != hipSuccess)
            return fail(RNNT_STATUS_MEMOPS_FAILED, "copying labels to host");
        for (int b = 0; b < s->B; ++b)
            for (int i = 0; i < S[b]; ++i) {
                const int l = lab[(size_t)b * p.label_stride + i];
                if (l < 0 || l >= s->V)
                    return fail(RNNT_STATUS_INVALID_VALUE, "label " + std::to_string(l) + " at (" + std::to_string(b) +
                                                               ", " + std::to_string(i) + ") outside [0, V)");
            }
    }
    float *costs_dev = reinterpret_cast<float *>(static_cast<char *>(s->workspace) + coff);
    st = mrnnt_cost_and_grad(&p, s->workspace, coff, costs_dev, grads, nullptr, stream);
    if (st != RNNT_STATUS_SUCCESS) return st;
    s->computed = true;
    s->with_beta = grads != nullptr;
    s->blank = blank;
    s->stream = stream;
    // the reference's public members: the view of this computation (betas / ll_backward only with the gradient, as
    // the reference's cost() skips the beta pass)
    if (wm.denom) {
        Plan pl;
        if ((st = make_plan(&p, &pl)) != RNNT_STATUS_SUCCESS) return st;
        const DevProblem d = make_dev(&p, pl, s->workspace);
        if ((st = mrnnt_read_denoms(&p, s->workspace, wm.denom, stream)) != RNNT_STATUS_SUCCESS) return st;
        hipError_t ev = launch_state_f32(d, wm.alphas, grads ? wm.betas : nullptr, wm.ll_forward,
                                         grads ? wm.ll_backward : nullptr, stream);
        if (ev != hipSuccess) return fail_hip(ev, "reference view kernel");
        const int T_max = *std::max_element(T.begin(), T.end());
        if ((st = mrnnt_read_band(&p, s->workspace, wm.min_allowed_s, wm.max_allowed_s, T_max, stream)) !=
            RNNT_STATUS_SUCCESS)
            return st;
    }
    hipError_t e = hipMemcpyAsync(costs, costs_dev, sizeof(float) * s->B, hipMemcpyDeviceToHost, stream);
    if (e != hipSuccess) return fail(RNNT_STATUS_MEMOPS_FAILED, std::string("costs D2H: ") + hipGetErrorString(e));
    e = hipStreamSynchronize(stream);
    if (e != hipSuccess) return fail_hip(e, "stream synchronize");
    return RNNT_STATUS_SUCCESS;
}

// A device scratch buffer for the inspection getters (they are synchronous, as the reference's are).
struct DevBuf {
    void *p = nullptr;
    explicit DevBuf(size_t bytes) {
        if (hipMalloc(&p, std::max<size_t>(bytes, 16)) != hipSuccess) p = nullptr;
    }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
};

// Reads back n elements of type Out (converted from In) through `read`, which fills a device buffer of n In on
// `stream`; empty on failure or when there is no workspace.
template <class In, class Out, class F>
std::vector<Out> read_back(const mrnnt_gpu_ws_state *s, size_t n, hipStream_t stream, F &&read) {
    if (!s->workspace) return {};
    DevBuf buf(sizeof(In) * n);
    if (!buf.p || read(static_cast<In *>(buf.p)) != RNNT_STATUS_SUCCESS) return {};
    std::vector<In> h(n);
    if (n && (hipMemcpyAsync(h.data(), buf.p, sizeof(In) * n, hipMemcpyDeviceToHost, stream) != hipSuccess ||
              hipStreamSynchronize(stream) != hipSuccess))
        return {};
    return std::vector<Out>(h.begin(), h.end());
}

}  // namespace

GpuRNNTWorkspaceManager<float>::GpuRNNTWorkspaceManager(const float *const acts_, const int *const labels_,
                                                        const int B_, const int *T_, const int *S_, const int V_)
    : st_(new mrnnt_gpu_ws_state),
      workspace_(nullptr),
      B_h(B_),
      V_h(V_),
      T(T_),
      S(S_),
      B(nullptr),
      V(nullptr),
      acts(acts_),
      labels(labels_),
      denom(nullptr),
      alphas(nullptr),
      betas(nullptr),
      min_allowed_s(nullptr),
      max_allowed_s(nullptr),
      denom_start_indices(nullptr),
      var_start_offsets(nullptr),
      S_max(nullptr),
      T_max(nullptr),
      ll_forward(nullptr),
      ll_backward(nullptr) {
    st_->acts = acts_;
    st_->labels = labels_;
    st_->B = B_;
    st_->V = V_;
    st_->T_dev = T_;
    st_->S_dev = S_;
}

GpuRNNTWorkspaceManager<float>::~GpuRNNTWorkspaceManager() { delete st_; }

RNNTStatus GpuRNNTWorkspaceManager<float>::get_workspace_size(size_t *size_bytes) const {
    if (st_->B <= 0) return fail(RNNT_STATUS_INVALID_VALUE, "B must be > 0");
    std::vector<int> Th, Sh;
    if (!host_lengths(st_, Th, Sh)) return fail(RNNT_STATUS_MEMOPS_FAILED, "copying lengths to host");
    size_t coff = 0;
    // alignment may be registered later: manager_size sizes the view for either layout
    return manager_size(st_, Th, Sh, size_bytes, &coff);
}

// (reference :256-329) the public members point into the workspace's view region; the constants and the default band
// are uploaded with blocking copies, as the reference's cudaMemcpy calls do
void GpuRNNTWorkspaceManager<float>::set_workspace(void *workspace) {
    if (st_->owned && st_->workspace && st_->workspace != workspace) (void)hipFree(st_->workspace);
    st_->workspace = workspace;
    st_->owned = false;
    st_->computed = false;
    workspace_ = workspace;
    denom = alphas = betas = ll_forward = ll_backward = nullptr;
    B = V = S_max = T_max = min_allowed_s = max_allowed_s = denom_start_indices = var_start_offsets = nullptr;
    std::vector<int> Th, Sh;
    size_t bytes = 0, coff = 0, voff = 0;
    if (!workspace || st_->B <= 0 || !host_lengths(st_, Th, Sh) ||
        manager_size(st_, Th, Sh, &bytes, &coff, &voff) != RNNT_STATUS_SUCCESS)
        return;
    std::vector<int> off(st_->B);
    int64_t N = 0;
    for (int b = 0; b < st_->B; ++b) {
        off[b] = (int)N;
        N += (int64_t)Th[b] * (Sh[b] + 1);
    }
    const int Tm = *std::max_element(Th.begin(), Th.end()), Sm = *std::max_element(Sh.begin(), Sh.end());
    const RefView v = ref_view_layout(st_->B, N, Tm);
    char *base = static_cast<char *>(workspace) + voff;
    denom = reinterpret_cast<float *>(base + v.denom);
    alphas = reinterpret_cast<float *>(base + v.alphas);
    betas = reinterpret_cast<float *>(base + v.betas);
    denom_start_indices = reinterpret_cast<int *>(base + v.dsi);
    var_start_offsets = reinterpret_cast<int *>(base + v.vso);
    ll_forward = reinterpret_cast<float *>(base + v.llf);
    ll_backward = reinterpret_cast<float *>(base + v.llb);
    B = reinterpret_cast<int *>(base + v.B);
    V = reinterpret_cast<int *>(base + v.V);
    S_max = reinterpret_cast<int *>(base + v.Smax);
    T_max = reinterpret_cast<int *>(base + v.Tmax);
    min_allowed_s = reinterpret_cast<int *>(base + v.mn);
    max_allowed_s = reinterpret_cast<int *>(base + v.mx);
    std::vector<int> mn((size_t)st_->B * Tm, 0), mx((size_t)st_->B * Tm);
    for (int b = 0; b < st_->B; ++b) std::fill_n(mx.begin() + (size_t)b * Tm, Tm, Sh[b]);
    const int consts[4] = {st_->B, st_->V, Sm, Tm};
    bool ok = hipMemcpy(denom_start_indices, off.data(), sizeof(int) * off.size(), hipMemcpyHostToDevice) == hipSuccess;
    ok = ok && hipMemcpy(var_start_offsets, off.data(), sizeof(int) * off.size(), hipMemcpyHostToDevice) == hipSuccess;
    ok = ok && hipMemcpy(B, consts, sizeof(consts), hipMemcpyHostToDevice) == hipSuccess;  // B, V, S_max, T_max
    ok = ok && hipMemcpy(min_allowed_s, mn.data(), sizeof(int) * mn.size(), hipMemcpyHostToDevice) == hipSuccess;
    ok = ok && hipMemcpy(max_allowed_s, mx.data(), sizeof(int) * mx.size(), hipMemcpyHostToDevice) == hipSuccess;
    if (!ok) (void)fail(RNNT_STATUS_MEMOPS_FAILED, "set_workspace: uploading the reference view's constants");
}

RNNTStatus GpuRNNTWorkspaceManager<float>::create_workspace() {
    size_t bytes = 0;
    const RNNTStatus st = get_workspace_size(&bytes);
    if (st != RNNT_STATUS_SUCCESS) return st;
    void *w = nullptr;
    if (hipMalloc(&w, bytes) != hipSuccess) return fail(RNNT_STATUS_MEMOPS_FAILED, "hipMalloc workspace");
    set_workspace(w);
    st_->owned = true;
    return RNNT_STATUS_SUCCESS;
}

void GpuRNNTWorkspaceManager<float>::free_workspace() {
    if (st_->workspace) (void)hipFree(st_->workspace);
    st_->workspace = nullptr;
    st_->owned = false;
    st_->computed = false;
    workspace_ = nullptr;
    denom = alphas = betas = ll_forward = ll_backward = nullptr;
    B = V = S_max = T_max = min_allowed_s = max_allowed_s = denom_start_indices = var_start_offsets = nullptr;
}

void GpuRNNTWorkspaceManager<float>::restrict_to_alignment(const int *const alignments, int max_shift, int blank_idx) {
    st_->alignment = alignments;
    st_->max_shift = max_shift;
    st_->align_blank = blank_idx;
}

int GpuRNNTWorkspaceManager<float>::B_host() const { return st_->B; }
int GpuRNNTWorkspaceManager<float>::V_host() const { return st_->V; }

std::vector<int> GpuRNNTWorkspaceManager<float>::T_host() const {
    std::vector<int> T, S;
    host_lengths(st_, T, S, st_->stream);
    return T;
}

std::vector<int> GpuRNNTWorkspaceManager<float>::S_host() const {
    std::vector<int> T, S;
    host_lengths(st_, T, S, st_->stream);
    return S;
}

int GpuRNNTWorkspaceManager<float>::num_denoms() const {
    std::vector<int> T, S;
    host_lengths(st_, T, S, st_->stream);
    int64_t n = 0;
    for (size_t b = 0; b < T.size(); ++b) n += (int64_t)T[b] * (S[b] + 1);
    return (int)n;
}

int GpuRNNTWorkspaceManager<float>::num_fwd_bwd_var_positions() const { return num_denoms(); }

std::vector<int> GpuRNNTWorkspaceManager<float>::var_start_offsets_host() const {
    std::vector<int> T, S;
    host_lengths(st_, T, S, st_->stream);
    std::vector<int> off(T.size(), 0);
    int64_t r = 0;
    for (size_t b = 0; b < T.size(); ++b) {
        off[b] = (int)r;
        r += (int64_t)T[b] * (S[b] + 1);
    }
    return off;
}

int GpuRNNTWorkspaceManager<float>::S_max_host() const {
    const std::vector<int> S = S_host();
    return S.empty() ? 0 : *std::max_element(S.begin(), S.end());
}

int GpuRNNTWorkspaceManager<float>::T_max_host() const {
    const std::vector<int> T = T_host();
    return T.empty() ? 0 : *std::max_element(T.begin(), T.end());
}

std::vector<float> GpuRNNTWorkspaceManager<float>::acts_host() const {
    const size_t n = (size_t)num_denoms() * (size_t)std::max(0, st_->V);
    std::vector<float> h(n);
    if (n && (hipMemcpyAsync(h.data(), st_->acts, sizeof(float) * n, hipMemcpyDeviceToHost, st_->stream) != hipSuccess ||
              hipStreamSynchronize(st_->stream) != hipSuccess))
        return {};
    return h;
}

// The getters below read the state of the last cost / cost_and_grad on this workspace through the flat
// inspection entry points (mrnnt_read_denoms / _state / _loglik / _band), in the reference's dense T*(S+1)
// per-utterance order (var_start_offsets[b] + t*(S_b+1) + s).
std::vector<float> GpuRNNTWorkspaceManager<float>::denom_host() const {
    std::vector<int> T, S;
    if (!host_lengths(st_, T, S, st_->stream)) return {};
    const mrnnt_problem p = problem_of(st_, T, S, st_->blank);
    return read_back<float, float>(st_, (size_t)num_denoms(), st_->stream,
                                   [&](float *d) { return mrnnt_read_denoms(&p, st_->workspace, d, st_->stream); });
}

std::vector<float> GpuRNNTWorkspaceManager<float>::alphas_host() const {
    std::vector<int> T, S;
    if (!host_lengths(st_, T, S, st_->stream)) return {};
    const mrnnt_problem p = problem_of(st_, T, S, st_->blank);
    return read_back<double, float>(st_, (size_t)num_denoms(), st_->stream, [&](double *d) {
        return mrnnt_read_state(&p, st_->workspace, nullptr, d, nullptr, st_->stream);
    });
}

std::vector<float> GpuRNNTWorkspaceManager<float>::betas_host() const {
    std::vector<int> T, S;
    if (!host_lengths(st_, T, S, st_->stream)) return {};
    const mrnnt_problem p = problem_of(st_, T, S, st_->blank);
    return read_back<double, float>(st_, (size_t)num_denoms(), st_->stream, [&](double *d) {
        return mrnnt_read_state(&p, st_->workspace, nullptr, nullptr, d, st_->stream);
    });
}

std::vector<float> GpuRNNTWorkspaceManager<float>::ll_forward_host() const {
    std::vector<int> T, S;
    if (!host_lengths(st_, T, S, st_->stream)) return {};
    const mrnnt_problem p = problem_of(st_, T, S, st_->blank);
    return read_back<double, float>(st_, (size_t)st_->B, st_->stream, [&](double *d) {
        return mrnnt_read_loglik(&p, st_->workspace, d, nullptr, st_->stream);
    });
}

std::vector<float> GpuRNNTWorkspaceManager<float>::ll_backward_host() const {
    std::vector<int> T, S;
    if (!host_lengths(st_, T, S, st_->stream)) return {};
    const mrnnt_problem p = problem_of(st_, T, S, st_->blank);
    return read_back<double, float>(st_, (size_t)st_->B, st_->stream, [&](double *d) {
        return mrnnt_read_loglik(&p, st_->workspace, nullptr, d, st_->stream);
    });
}

std::vector<int> GpuRNNTWorkspaceManager<float>::min_allowed_s_host() const {
    std::vector<int> T, S;
    if (!host_lengths(st_, T, S, st_->stream)) return {};
    const mrnnt_problem p = problem_of(st_, T, S, st_->blank);
    const int64_t ld = std::max<int64_t>(1, p.align_stride);
    return read_back<int, int>(st_, (size_t)st_->B * ld, st_->stream, [&](int *d) {
        return mrnnt_read_band(&p, st_->workspace, d, nullptr, ld, st_->stream);
    });
}

std::vector<int> GpuRNNTWorkspaceManager<float>::max_allowed_s_host() const {
    std::vector<int> T, S;
    if (!host_lengths(st_, T, S, st_->stream)) return {};
    const mrnnt_problem p = problem_of(st_, T, S, st_->blank);
    const int64_t ld = std::max<int64_t>(1, p.align_stride);
    return read_back<int, int>(st_, (size_t)st_->B * ld, st_->stream, [&](int *d) {
        return mrnnt_read_band(&p, st_->workspace, nullptr, d, ld, st_->stream);
    });
}

GpuRNNTComputer<float>::GpuRNNTComputer(GpuRNNTWorkspaceManager<float> &workspace_manager, int blank,
                                        hipStream_t stream)
    : workspace_manager_(workspace_manager), blank_(blank), stream_(stream) {}

RNNTStatus GpuRNNTComputer<float>::cost_and_grad(float *costs, float *grads) {
    return manager_compute(workspace_manager_, blank_, stream_, costs, grads);
}

RNNTStatus GpuRNNTComputer<float>::cost(float *costs) {
    return manager_compute(workspace_manager_, blank_, stream_, costs, nullptr);
}

// compute_rnnt_loss (mrnnt_entry.cpp) for loc = RNNT_GPU
RNNTStatus mrnnt::gpu_compute_rnnt_loss(RNNTWorkspaceManager &workspace_manager, RNNTOptions options, float *costs,
                                        float *gradients) {
    auto *gm = dynamic_cast<GpuRNNTWorkspaceManager<float> *>(&workspace_manager);
    if (!gm) return fail(RNNT_STATUS_INVALID_VALUE, "workspace manager is not a GpuRNNTWorkspaceManager<float>");
    GpuRNNTComputer<float> computer(*gm, options.blank_label, options.stream);
    return gradients != nullptr ? computer.cost_and_grad(costs, gradients) : computer.cost(costs);
}
