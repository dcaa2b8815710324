// mrnnt_devtools.hip -- libmrnnt_devtools.so: bench / test helpers kept OUT of the product library.
//
//   mrnnt_synth_acts  : counter-based synthetic logits on the device, bit-identical to the host twin
//                       mrnnt_oracle_synth_acts (oracle/rnnt_oracle.c), so a test can regenerate any
//                       utterance's acts on the host without copying 50+ GB back
//   mrnnt_copy_probe  : a device copy in the gradient pass's access pattern, so a bench can report this
//                       card's copy rate between the same two buffers the gradient kernel streams
//
// Nothing here is called by libmonotonic_rnnt_amd.so, and the product never loads this library.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdio>

#pragma GCC visibility push(default)
#include "mrnnt_devtools.h"
#pragma GCC visibility pop

namespace {

typedef unsigned int u4 __attribute__((ext_vector_type(4)));

// integer hashing + one exact int->float conversion and one multiply: nothing that rounds differently on
// the host
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

// each workgroup streams its own contiguous slab of 16-byte elements, 4 loads in flight per lane,
// nontemporal loads and stores
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

// nontemporal stores only, same slab walk as the copy probe
__global__ __launch_bounds__(256) void write_probe_kernel(u4 *__restrict__ b, int64_t n, int64_t slab) {
    const u4 z = {0u, 0u, 0u, 0u};
    for (int64_t c0 = (int64_t)blockIdx.x * slab; c0 < n; c0 += (int64_t)gridDim.x * slab) {
        const int64_t end = min(c0 + slab, n);
        for (int64_t i = c0 + threadIdx.x; i < end; i += 256) __builtin_nontemporal_store(z, &b[i]);
    }
}

// nontemporal loads only (the log-softmax pass's stream), same slab walk; the xor keeps the loads live
__global__ __launch_bounds__(256) void read_probe_kernel(const u4 *__restrict__ a, int64_t n, int64_t slab,
                                                         unsigned *__restrict__ sink) {
    unsigned acc = 0;
    for (int64_t c0 = (int64_t)blockIdx.x * slab; c0 < n; c0 += (int64_t)gridDim.x * slab) {
        const int64_t end = min(c0 + slab, n);
        for (int64_t i = c0 + threadIdx.x; i < end; i += 256 * 4) {
            u4 x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                x[u] = (i + 256 * u < end) ? __builtin_nontemporal_load(&a[i + 256 * u]) : (u4){0u, 0u, 0u, 0u};
#pragma unroll
            for (int u = 0; u < 4; ++u) acc ^= x[u].x ^ x[u].y ^ x[u].z ^ x[u].w;
        }
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;  // practically never: the loads cannot be dropped
}

extern "C" __device__ uint64_t mrnnt_dev_dispatch_id() __asm("llvm.amdgcn.dispatch.id");

__global__ void dispatch_probe_kernel(uint64_t *out, int slot) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        out[2 * slot] = mrnnt_dev_dispatch_id();
        out[2 * slot + 1] = (uint64_t)(uintptr_t)__builtin_amdgcn_queue_ptr();
    }
}

// every wave sleeps until `ticks` of the 100 MHz constant clock have passed since its workgroup started
__global__ __launch_bounds__(256) void occupy_kernel(uint64_t ticks) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(32);
}

// slab size and grid of the probes: 32 workgroups per CU, each streaming >= 8 slabs in turn (a single pass
// of one slab per workgroup measures the launch tail, not the memory); slabs of 16 KiB .. 800 KiB
int probe_grid(int64_t n, int64_t *slab, int64_t *blocks) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return 3;
    const int64_t blocks_max = (int64_t)32 * cus;
    *slab = std::min<int64_t>(50 * 1024, std::max<int64_t>(1024, n / (blocks_max * 8) / 1024 * 1024));
    *blocks = std::min<int64_t>((n + *slab - 1) / *slab, blocks_max);
    return 0;
}

// a launch's status: an error left by an earlier call on this thread is reported (not blamed on this launch)
int launch_status(const char *what, hipError_t stale) {
    if (stale != hipSuccess)
        std::fprintf(stderr, "mrnnt_devtools: error pending before %s: %s\n", what, hipGetErrorString(stale));
    const hipError_t e = hipGetLastError();
    if (e == hipSuccess) return 0;
    std::fprintf(stderr, "mrnnt_devtools: %s launch failed: %s\n", what, hipGetErrorString(e));
    return 3;
}

}  // namespace

extern "C" {

int mrnnt_synth_acts(float *out, int64_t begin, int64_t count, uint64_t seed, int normal, hipStream_t stream) {
    if (count <= 0) return 0;
    if (!out) return 2;
    const int64_t blocks = std::min<int64_t>((count + 255) / 256, 65536);
    const hipError_t stale = hipGetLastError();
    synth_kernel<<<(int)blocks, 256, 0, stream>>>(out, begin, count, seed, normal);
    return launch_status("synth", stale);
}

int mrnnt_copy_probe(void *dst, const void *src, size_t bytes, hipStream_t stream) {
    if ((bytes & 15) || (reinterpret_cast<uintptr_t>(dst) & 15) || (reinterpret_cast<uintptr_t>(src) & 15)) return 2;
    const int64_t n = (int64_t)(bytes / 16);
    if (n <= 0) return 0;
    int64_t slab = 0, blocks = 0;
    if (probe_grid(n, &slab, &blocks)) return 3;
    const hipError_t stale = hipGetLastError();
    copy_probe_kernel<<<(int)blocks, 256, 0, stream>>>(static_cast<const u4 *>(src), static_cast<u4 *>(dst), n, slab);
    return launch_status("copy probe", stale);
}

int mrnnt_read_probe(const void *src, size_t bytes, void *sink, hipStream_t stream) {
    if ((bytes & 15) || (reinterpret_cast<uintptr_t>(src) & 15) || !sink) return 2;
    const int64_t n = (int64_t)(bytes / 16);
    if (n <= 0) return 0;
    int64_t slab = 0, blocks = 0;
    if (probe_grid(n, &slab, &blocks)) return 3;
    const hipError_t stale = hipGetLastError();
    read_probe_kernel<<<(int)blocks, 256, 0, stream>>>(static_cast<const u4 *>(src), n, slab,
                                                       static_cast<unsigned *>(sink));
    return launch_status("read probe", stale);
}

int mrnnt_write_probe(void *dst, size_t bytes, hipStream_t stream) {
    if ((bytes & 15) || (reinterpret_cast<uintptr_t>(dst) & 15)) return 2;
    const int64_t n = (int64_t)(bytes / 16);
    if (n <= 0) return 0;
    int64_t slab = 0, blocks = 0;
    if (probe_grid(n, &slab, &blocks)) return 3;
    const hipError_t stale = hipGetLastError();
    write_probe_kernel<<<(int)blocks, 256, 0, stream>>>(static_cast<u4 *>(dst), n, slab);
    return launch_status("write probe", stale);
}

int mrnnt_dispatch_probe(uint64_t *out, int slot, hipStream_t stream) {
    if (!out || slot < 0) return 2;
    const hipError_t stale = hipGetLastError();
    dispatch_probe_kernel<<<1, 64, 0, stream>>>(out, slot);
    return launch_status("dispatch probe", stale);
}

int mrnnt_occupy(int us, int blocks_per_cu, hipStream_t stream) {
    if (us < 0 || us > 10000000 || blocks_per_cu < 1 || blocks_per_cu > 8) return 2;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return 3;
    const hipError_t stale = hipGetLastError();
    occupy_kernel<<<cus * blocks_per_cu, 256, 0, stream>>>((uint64_t)us * 100);
    return launch_status("occupy", stale);
}

}  // extern "C"
