/*
 * rnnt_oracle.c -- CPU restatement of the reference's monotonic RNN-T CPU path
 * (include/cpu_rnnt.h + include/cpu_workspace_manager.h + include/rnnt_helper.h).
 *
 * TEST INFRASTRUCTURE ONLY. This library is the *checker*: only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it. The product (monotonic-rnnt_amd/) never links,
 * loads or calls it, and fails loudly if its HIP library is missing.
 *
 * Pinned by: the reference's own known answers (tests/test_cpu.cpp, pytorch_binding/test.py,
 * README.md:117-174) and by golden vectors produced by the reference itself compiled here
 * (oracle/_ref, see oracle/Makefile and tests/golden/make_golden.py).
 *
 * Differences from the reference, all deliberate and documented in DESIGN.md:
 *   - 64-bit row/element offsets (the reference's int offsets overflow at N*V >= 2^31,
 *     cpu_workspace_manager.h:48,125);
 *   - dense [T][S+1] alpha/beta storage instead of the packed band (getter values identical);
 *   - label and alignment row strides are explicit arguments (the reference hard-wires
 *     max(S) and max(T): cpu_workspace_manager.h:122 and :208-213);
 *   - the alpha compute range is clamped to s <= S (the reference writes out of range when an
 *     alignment holds more non-blanks than S -- undefined behaviour there).
 *
 * Exports:
 *   mrnnt_oracle_f64(...)   REAL = double: the parity golden (cpu_rnnt.h<double> on fp32 inputs)
 *   mrnnt_oracle_f32(...)   REAL = float : mirrors cpu_rnnt.h<float>, for distance reporting
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define REAL double
#define SFX(x) x##_f64
#include "oracle_impl.h"
#undef REAL
#undef SFX

#define REAL float
#define SFX(x) x##_f32
#include "oracle_impl.h"
#undef REAL
#undef SFX

/* Counter-based synthetic generator, bit-identical to the device generator in
 * monotonic-rnnt_amd/devtools/mrnnt_devtools.hip (integer hashing + one exact int->float conversion and one
 * multiply, so no transcendental rounding can differ between host and device):
 *   h = SplitMix64(seed * K + index)
 *   uniform : U[0,1)   = (h >> 40) * 2^-24
 *   normal  : N(0,1)-like Irwin-Hall(4) = (sum of four 16-bit fields - 131070) / 37837.23 */
static inline uint64_t mrnnt_splitmix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

void mrnnt_oracle_synth_acts(float *out, int64_t begin, int64_t count, uint64_t seed, int normal) {
#pragma omp parallel for schedule(static) if (count > (1 << 22))
    for (int64_t i = 0; i < count; ++i) {
        uint64_t h = mrnnt_splitmix(seed * 0xD1B54A32D192ED03ull + (uint64_t)(begin + i));
        if (!normal) {
            out[i] = (float)(uint32_t)(h >> 40) * (1.0f / 16777216.0f);
        } else {
            int32_t s4 = (int32_t)(h & 0xFFFF) + (int32_t)((h >> 16) & 0xFFFF) + (int32_t)((h >> 32) & 0xFFFF) +
                         (int32_t)(h >> 48);
            out[i] = (float)(s4 - 131070) * (1.0f / 37837.23f);
        }
    }
}
