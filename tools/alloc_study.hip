// alloc_study.hip -- does the allocation method decide how fast a large buffer streams?
//
//   hipcc --offload-arch=gfx950 -O3 tools/alloc_study.hip -o tools/alloc_study
//   ./tools/alloc_study METHOD [K] [GIB]     (one method per process: the study runs several fresh processes)
//
// METHOD: malloc (hipMalloc), contig (hipExtMallocWithFlags hipDeviceMallocContiguous), vmm (hipMemCreate of the
// whole buffer at the recommended granularity, hipMemMap, hipMemSetAccess), vmm2m (the same from 2 MiB physical
// chunks mapped back to back), pool (hipMallocAsync from the default pool after one priming allocation).
// K buffers of GIB GiB each (default 4 x 48). Per buffer: nontemporal / plain streaming write, nontemporal read
// and the gradient pass's 1:1 nontemporal copy into it from the next buffer, GB/s of algorithmic bytes (median of
// 5). Prints one JSON object. The gradient kernel's run-to-run spread (round 1: 12.4 - 15.9 ms for the same
// launch) follows its grads buffer; this isolates whether the backing of that buffer is the cause.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                         \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                \
        }                                                                                \
    } while (0)

__global__ __launch_bounds__(256) void k_write_nt(f4 *__restrict__ b, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const f4 z = (f4){0.f, 1.f, 2.f, 3.f};
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        __builtin_nontemporal_store(z, &b[i]);
}

__global__ __launch_bounds__(256) void k_write(f4 *__restrict__ b, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const f4 z = (f4){0.f, 1.f, 2.f, 3.f};
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) b[i] = z;
}

__global__ __launch_bounds__(256) void k_read_nt(const f4 *__restrict__ a, int64_t n, float *__restrict__ out) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    float acc = 0.f;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 7 * stride < n; i += 8 * stride) {
        f4 x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = __builtin_nontemporal_load(&a[i + u * stride]);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += x[u].x + x[u].w;
    }
    for (; i < n; i += stride) acc += a[i].x;
    if (acc == 1234.5f) out[0] = acc;
}

// contiguous slab per workgroup, 4 loads in flight per lane (the gradient pass's shape)
__global__ __launch_bounds__(256) void k_copy_nt(const f4 *__restrict__ a, f4 *__restrict__ b, int64_t n, int64_t slab) {
    for (int64_t c0 = (int64_t)blockIdx.x * slab; c0 < n; c0 += (int64_t)gridDim.x * slab) {
        const int64_t end = c0 + slab < n ? c0 + slab : n;
        for (int64_t i = c0 + threadIdx.x; i < end; i += 1024) {
            f4 x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + 256 * u < end) x[u] = __builtin_nontemporal_load(&a[i + 256 * u]);
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + 256 * u < end) __builtin_nontemporal_store(x[u], &b[i + 256 * u]);
        }
    }
}

template <class F>
static float median_ms(F f, int reps = 5) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    f();
    CHECK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int r = 0; r < reps; ++r) {
        CHECK(hipEventRecord(e0));
        f();
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
    return ts[ts.size() / 2];
}

static void *vmm_alloc(size_t bytes, size_t chunk) {
    int dev = 0;
    CHECK(hipGetDevice(&dev));
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = dev;
    size_t gran = 0;
    CHECK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
    if (chunk == 0) chunk = bytes;
    chunk = (chunk + gran - 1) / gran * gran;
    bytes = (bytes + chunk - 1) / chunk * chunk;
    hipDeviceptr_t base = nullptr;
    CHECK(hipMemAddressReserve(&base, bytes, 0, nullptr, 0));
    for (size_t o = 0; o < bytes; o += chunk) {
        hipMemGenericAllocationHandle_t h;
        CHECK(hipMemCreate(&h, chunk, &prop, 0));
        CHECK(hipMemMap(reinterpret_cast<char *>(base) + o, chunk, 0, h, 0));
        CHECK(hipMemRelease(h));
    }
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    CHECK(hipMemSetAccess(base, bytes, &acc, 1));
    return base;
}

int main(int argc, char **argv) {
    const std::string method = argc > 1 ? argv[1] : "malloc";
    const int K = argc > 2 ? std::atoi(argv[2]) : 4;
    const double gib = argc > 3 ? std::atof(argv[3]) : 48.0;
    const size_t bytes = (size_t)(gib * (1ull << 30));
    const int64_t n = (int64_t)(bytes / 16);
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int grid = cus * 32;
    float *out;
    CHECK(hipMalloc(&out, 16));
    std::vector<f4 *> buf(K);
    hipStream_t s0 = nullptr;
    if (method == "pool") {  // prime the pool so it holds the memory, then carve the buffers from it
        void *p;
        CHECK(hipMallocAsync(&p, bytes * K, s0));
        CHECK(hipFreeAsync(p, s0));
        CHECK(hipStreamSynchronize(s0));
    }
    for (int k = 0; k < K; ++k) {
        void *p = nullptr;
        if (method == "malloc") CHECK(hipMalloc(&p, bytes));
        else if (method == "contig") CHECK(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocContiguous));
        else if (method == "vmm") p = vmm_alloc(bytes, 0);
        else if (method == "vmm2m") p = vmm_alloc(bytes, 2u << 20);
        else if (method == "pool") CHECK(hipMallocAsync(&p, bytes, s0));
        else {
            std::fprintf(stderr, "unknown method %s\n", method.c_str());
            return 2;
        }
        buf[k] = static_cast<f4 *>(p);
        k_write<<<grid, 256>>>(buf[k], n);
    }
    CHECK(hipDeviceSynchronize());
    const int64_t slab = std::min<int64_t>(50 * 1024, std::max<int64_t>(1024, n / ((int64_t)grid * 8) / 1024 * 1024));
    const double B = (double)n * 16;
    std::printf("{\"method\": \"%s\", \"gib\": %.1f, \"buffers\": [", method.c_str(), gib);
    for (int k = 0; k < K; ++k) {
        f4 *a = buf[k], *src = buf[(k + 1) % K];
        const float w_nt = median_ms([&] { k_write_nt<<<grid, 256>>>(a, n); });
        const float w = median_ms([&] { k_write<<<grid, 256>>>(a, n); });
        const float r_nt = median_ms([&] { k_read_nt<<<grid, 256>>>(a, n, out); });
        const float c_nt = median_ms([&] { k_copy_nt<<<grid, 256>>>(src, a, n, slab); });
        std::printf("%s{\"k\": %d, \"ptr\": \"%p\", \"write_nt\": %.0f, \"write\": %.0f, \"read_nt\": %.0f, \"copy_in_nt\": %.0f}",
                    k ? ", " : "", k, (void *)a, B / (w_nt * 1e-3) / 1e9, B / (w * 1e-3) / 1e9, B / (r_nt * 1e-3) / 1e9,
                    2 * B / (c_nt * 1e-3) / 1e9);
        std::fflush(stdout);
    }
    std::printf("]}\n");
    return 0;
}
