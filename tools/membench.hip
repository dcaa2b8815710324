// membench.hip -- HBM ceilings on this MI355X for the access shapes of the hot path:
//   read    : float4 loads, reduce to a register (the log-softmax pass)
//   write   : float4 stores (the zero rows of the gradient)
//   copy    : float4 load -> store (the gradient pass, 1 read : 1 write)
//   copy_nt : copy with nontemporal stores
// Grid-stride over 16-B elements with UNROLL loads in flight per lane; reports GB/s of algorithmic
// bytes. Build: hipcc --offload-arch=gfx950 -O3 tools/membench.hip -o membench ; run: ./membench [GiB]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <string>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                        \
    do {                                                                                \
        hipError_t e = (x);                                                             \
        if (e != hipSuccess) {                                                          \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

template <int UNROLL>
__global__ __launch_bounds__(256) void k_read(const f4 *__restrict__ a, int64_t n, float *__restrict__ out) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    float acc = 0.f;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (UNROLL - 1) * stride < n; i += UNROLL * stride) {
        f4 x[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) x[u] = a[i + u * stride];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc += x[u].x + x[u].y + x[u].z + x[u].w;
    }
    for (; i < n; i += stride) acc += a[i].x;
    if (acc == 1234.5f) out[0] = acc;
}

template <int UNROLL>
__global__ __launch_bounds__(256) void k_read_nt(const f4 *__restrict__ a, int64_t n, float *__restrict__ out) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    float acc = 0.f;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (UNROLL - 1) * stride < n; i += UNROLL * stride) {
        f4 x[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) x[u] = __builtin_nontemporal_load(&a[i + u * stride]);
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc += x[u].x + x[u].y + x[u].z + x[u].w;
    }
    for (; i < n; i += stride) acc += a[i].x;
    if (acc == 1234.5f) out[0] = acc;
}

// each workgroup streams a contiguous slab of `chunk` float4s (like one lattice column per workgroup)
template <int UNROLL>
__global__ __launch_bounds__(256) void k_read_chunk(const f4 *__restrict__ a, int64_t n, int64_t chunk,
                                                    float *__restrict__ out) {
    float acc = 0.f;
    for (int64_t c0 = (int64_t)blockIdx.x * chunk; c0 < n; c0 += (int64_t)gridDim.x * chunk) {
        const int64_t end = c0 + chunk < n ? c0 + chunk : n;
        for (int64_t i = c0 + threadIdx.x; i < end; i += 256 * UNROLL) {
            f4 x[UNROLL];
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) x[u] = (i + u * 256 < end) ? a[i + u * 256] : (f4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) acc += x[u].x + x[u].y + x[u].z + x[u].w;
        }
    }
    if (acc == 1234.5f) out[0] = acc;
}

template <int UNROLL>
__global__ __launch_bounds__(256) void k_write_plain(f4 *__restrict__ b, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const f4 z = (f4){0.f, 0.f, 0.f, 0.f};
    for (; i < n; i += stride) b[i] = z;
}

template <int UNROLL>
__global__ __launch_bounds__(256) void k_write(f4 *__restrict__ b, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const f4 z = (f4){0.f, 0.f, 0.f, 0.f};
    for (; i < n; i += stride) __builtin_nontemporal_store(z, &b[i]);
}

template <int UNROLL, bool NT>
__global__ __launch_bounds__(256) void k_copy(const f4 *__restrict__ a, f4 *__restrict__ b, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (UNROLL - 1) * stride < n; i += UNROLL * stride) {
        f4 x[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) x[u] = a[i + u * stride];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            if constexpr (NT)
                __builtin_nontemporal_store(x[u], &b[i + u * stride]);
            else
                b[i + u * stride] = x[u];
        }
    }
    for (; i < n; i += stride) b[i] = a[i];
}

// contiguous-chunk variant: each workgroup streams its own contiguous slab (like one lattice column
// per workgroup), 4 KiB per wave-iteration
template <bool NT>
__global__ __launch_bounds__(256) void k_copy_chunk(const f4 *__restrict__ a, f4 *__restrict__ b, int64_t n,
                                                    int64_t chunk) {
    for (int64_t c0 = (int64_t)blockIdx.x * chunk; c0 < n; c0 += (int64_t)gridDim.x * chunk) {
        const int64_t end = c0 + chunk < n ? c0 + chunk : n;
        for (int64_t i = c0 + threadIdx.x; i < end; i += 256 * 4) {
            f4 x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + u * 256 < end) x[u] = a[i + u * 256];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + u * 256 < end) {
                    if constexpr (NT)
                        __builtin_nontemporal_store(x[u], &b[i + u * 256]);
                    else
                        b[i + u * 256] = x[u];
                }
        }
    }
}

__global__ void k_fill(f4 *a, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        a[i] = (f4){(float)(i & 7), 1.f, 2.f, 3.f};
}

template <class F>
static float time_ms(F f, int reps) {
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
    return ts[ts.size() / 2];
}

// write patterns for the buffer study: each wave writes whole 4 KiB rows (the gradient kernel's store shape);
// rows visited in order (grid-stride over rows) or with the row index multiplied by an odd constant mod rows
// (scattered); and 2 MiB pages visited in a scattered order, each page written by one workgroup
__global__ __launch_bounds__(256) void k_write_rows(f4 *__restrict__ b, int64_t rows, int64_t mul) {
    const int lane = threadIdx.x & 63;
    const int64_t gw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (int64_t)gridDim.x * 4;
    const f4 z = (f4){0.f, 0.f, 0.f, 0.f};
    for (int64_t r = gw; r < rows; r += nw) {
        const int64_t row = mul ? (r * mul) % rows : r;
        f4 *o = b + row * 256;
#pragma unroll
        for (int u = 0; u < 4; ++u) __builtin_nontemporal_store(z, o + lane + 64 * u);
    }
}

__global__ __launch_bounds__(256) void k_write_pages(f4 *__restrict__ b, int64_t pages, int64_t mul) {
    const f4 z = (f4){0.f, 0.f, 0.f, 0.f};
    for (int64_t pg = blockIdx.x; pg < pages; pg += gridDim.x) {
        f4 *o = b + ((pg * mul) % pages) * (int64_t)(2 << 20) / 16;
        for (int i = threadIdx.x; i < (2 << 20) / 16; i += 256) __builtin_nontemporal_store(z, o + i);
    }
}

// --buffers K GIB SUB [FRAG]: K buffers of GIB GiB each; per buffer the streaming read / write rates of the whole buffer
// and the nontemporal write rate of every SUB-GiB sub-range (does a buffer's speed depend on where it sits, and
// is a slow buffer slow everywhere?)
static int buffers_mode(int K, double gib, double sub, double frag_gib) {
    // optional: map frag_gib GiB as 2 MiB pieces and free every other one first, so the buffers are built from
    // scattered 2 MiB physical pieces
    std::vector<void *> keep;
    if (frag_gib > 0) {
        std::vector<void *> pieces((size_t)(frag_gib * 512));
        for (auto &q : pieces) CHECK(hipMalloc(&q, 2 << 20));
        for (size_t i = 0; i < pieces.size(); ++i) {
            if (i & 1) CHECK(hipFree(pieces[i]));
            else keep.push_back(pieces[i]);
        }
    }
    const int64_t n = (int64_t)(gib * (1 << 30)) / 16;
    const int64_t ns = (int64_t)(sub * (1 << 30)) / 16;
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int grid = cus * 32;
    std::vector<f4 *> buf(K);
    float *out;
    CHECK(hipMalloc(&out, 16));
    for (int k = 0; k < K; ++k) {
        CHECK(hipMalloc(&buf[k], n * 16));
        k_fill<<<4096, 256>>>(buf[k], n);
    }
    CHECK(hipDeviceSynchronize());
    const double bytes = (double)n * 16;
    std::printf("{\"gib\": %.1f, \"sub_gib\": %.1f, \"buffers\": [\n", gib, sub);
    for (int k = 0; k < K; ++k) {
        f4 *a = buf[k];
        const float r_nt = time_ms([&] { k_read_nt<8><<<grid, 256>>>(a, n, out); }, 3);
        const float r_pl = time_ms([&] { k_read<8><<<grid, 256>>>(a, n, out); }, 3);
        const float w_nt = time_ms([&] { k_write<1><<<grid, 256>>>(a, n); }, 3);
        const float w_pl = time_ms([&] { k_write_plain<1><<<grid, 256>>>(a, n); }, 3);
        const float c_nt = time_ms([&] { k_copy<4, true><<<grid, 256>>>(buf[(k + 1) % K], a, n); }, 3);
        const int64_t rows = n / 256, pages = n * 16 / (2 << 20);
        const float w_rows = time_ms([&] { k_write_rows<<<grid, 256>>>(a, rows, 0); }, 3);
        const float w_rows_sc = time_ms([&] { k_write_rows<<<grid, 256>>>(a, rows, 7919); }, 3);
        const float w_pages_sc = time_ms([&] { k_write_pages<<<cus * 8, 256>>>(a, pages, 4093); }, 3);
        std::printf("%s {\"ptr\": \"%p\", \"read_nt\": %.1f, \"read\": %.1f, \"write_nt\": %.1f, \"write\": %.1f, "
                    "\"copy_in_nt\": %.1f, \"write_rows\": %.1f, \"write_rows_scattered\": %.1f, "
                    "\"write_pages_scattered\": %.1f, \"sub_write_nt\": [",
                    k ? ",\n" : "", (void *)a, bytes / (r_nt * 1e-3) / 1e9, bytes / (r_pl * 1e-3) / 1e9,
                    bytes / (w_nt * 1e-3) / 1e9, bytes / (w_pl * 1e-3) / 1e9, 2 * bytes / (c_nt * 1e-3) / 1e9,
                    bytes / (w_rows * 1e-3) / 1e9, bytes / (w_rows_sc * 1e-3) / 1e9, bytes / (w_pages_sc * 1e-3) / 1e9);
        for (int64_t o = 0; o + ns <= n; o += ns) {
            const float ms = time_ms([&] { k_write<1><<<grid, 256>>>(a + o, ns); }, 3);
            std::printf("%s%.0f", o ? ", " : "", (double)ns * 16 / (ms * 1e-3) / 1e9);
        }
        std::printf("]}");
    }
    std::printf("\n]}\n");
    return 0;
}

int main(int argc, char **argv) {
    if (argc > 1 && std::string(argv[1]) == "--buffers")
        return buffers_mode(argc > 2 ? std::atoi(argv[2]) : 4, argc > 3 ? std::atof(argv[3]) : 48.0,
                            argc > 4 ? std::atof(argv[4]) : 4.0, argc > 5 ? std::atof(argv[5]) : 0.0);
    const double gib = argc > 1 ? std::atof(argv[1]) : 16.0;
    const int64_t n = (int64_t)(gib * (1 << 30)) / 16;
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    f4 *a, *b;
    float *out;
    CHECK(hipMalloc(&a, n * 16));
    CHECK(hipMalloc(&b, n * 16));
    CHECK(hipMalloc(&out, 16));
    k_fill<<<4096, 256>>>(a, n);
    k_fill<<<4096, 256>>>(b, n);
    CHECK(hipDeviceSynchronize());
    const double bytes = (double)n * 16;
    std::printf("{\"gib\": %.1f, \"cus\": %d, \"results\": [\n", gib, cus);
    bool first = true;
    auto rep = [&](const char *name, int wg_per_cu, double mult, float ms) {
        std::printf("%s {\"kernel\": \"%s\", \"wg_per_cu\": %d, \"ms\": %.3f, \"gbps\": %.1f}", first ? "" : ",\n", name,
                    wg_per_cu, ms, mult * bytes / (ms * 1e-3) / 1e9);
        first = false;
    };
    for (int w : {8, 16, 32}) {
        const int grid = cus * w;
        rep("read_u8", w, 1.0, time_ms([&] { k_read<8><<<grid, 256>>>(a, n, out); }, 5));
        rep("read_u16", w, 1.0, time_ms([&] { k_read<16><<<grid, 256>>>(a, n, out); }, 5));
        rep("read_nt_u8", w, 1.0, time_ms([&] { k_read_nt<8><<<grid, 256>>>(a, n, out); }, 5));
        rep("read_chunk64k_u4", w, 1.0, time_ms([&] { k_read_chunk<4><<<grid, 256>>>(a, n, 65536 / 16, out); }, 5));
        rep("read_chunk800k_u4", w, 1.0, time_ms([&] { k_read_chunk<4><<<grid, 256>>>(a, n, 823296 / 16, out); }, 5));
        rep("read_chunk800k_u8", w, 1.0, time_ms([&] { k_read_chunk<8><<<grid, 256>>>(a, n, 823296 / 16, out); }, 5));
        rep("write_nt", w, 1.0, time_ms([&] { k_write<1><<<grid, 256>>>(b, n); }, 5));
        rep("write_plain", w, 1.0, time_ms([&] { k_write_plain<1><<<grid, 256>>>(b, n); }, 5));
        rep("copy_u4", w, 2.0, time_ms([&] { k_copy<4, false><<<grid, 256>>>(a, b, n); }, 5));
        rep("copy_u4_nt", w, 2.0, time_ms([&] { k_copy<4, true><<<grid, 256>>>(a, b, n); }, 5));
        rep("copy_chunk800k_nt", w, 2.0,
            time_ms([&] { k_copy_chunk<true><<<grid, 256>>>(a, b, n, 823296 / 16); }, 5));
    }
    {
        const int64_t chunks = (n + 823296 / 16 - 1) / (823296 / 16);
        rep("read_chunk800k_onewgper", 0, 1.0,
            time_ms([&] { k_read_chunk<4><<<(int)chunks, 256>>>(a, n, 823296 / 16, out); }, 5));
        rep("copy_chunk800k_onewgper_nt", 0, 2.0,
            time_ms([&] { k_copy_chunk<true><<<(int)chunks, 256>>>(a, b, n, 823296 / 16); }, 5));
    }
    std::printf("\n]}\n");
    return 0;
}
