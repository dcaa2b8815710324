// probe: v_dot2c_f32_bf16 semantics (development check)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
__global__ void k(float *o, const unsigned *a, const unsigned *b) {
    const int i = threadIdx.x;
    bf16x2 x = __builtin_bit_cast(bf16x2, a[i]), y = __builtin_bit_cast(bf16x2, b[i]);
    o[i] = __builtin_amdgcn_fdot2_f32_bf16(x, y, 0.5f, false);
}
static unsigned short bf(float f) { unsigned u; memcpy(&u, &f, 4); return (unsigned short)(u >> 16); }
int main() {
    unsigned ha[4], hb[4];
    float va[8] = {1.0f, 2.0f, -3.0f, 0.5f, 1.5f, 4.0f, 0.25f, -1.0f}, vb[8] = {3.0f, 5.0f, 2.0f, 2.0f, -1.0f, 0.5f, 8.0f, 1.0f};
    for (int i = 0; i < 4; ++i) {
        ha[i] = bf(va[2 * i]) | ((unsigned)bf(va[2 * i + 1]) << 16);
        hb[i] = bf(vb[2 * i]) | ((unsigned)bf(vb[2 * i + 1]) << 16);
    }
    float *o; unsigned *a, *b;
    hipMalloc(&o, 16); hipMalloc(&a, 16); hipMalloc(&b, 16);
    hipMemcpy(a, ha, 16, hipMemcpyHostToDevice); hipMemcpy(b, hb, 16, hipMemcpyHostToDevice);
    k<<<1, 4>>>(o, a, b);
    float r[4]; hipMemcpy(r, o, 16, hipMemcpyDeviceToHost);
    for (int i = 0; i < 4; ++i) printf("dot2 %d: got %g expect %g\n", i, r[i], va[2*i]*vb[2*i] + va[2*i+1]*vb[2*i+1] + 0.5f);
    return 0;
}
