// exactdiv_check.hip -- device check of csrc/exactdiv.h against HIP's own
// correctly rounded f32 divide, on gfx950.
//   1. xdiv_rcp(b) == 1.0f / b for EVERY float b in [2^-40, 2^40] (671M values).
//   2. xdiv(a, b) == a / b for every 23-bit numerator significand against
//      NDEN denominators (specials + random significands, random exponents in
//      the guarded range, random numerator exponents and signs).
//   3. Numerator edge values (+-0, +-2^-60, +-(2^60 - ulp)) against every
//      denominator of (2); the guard predicates on boundary values.
//   4. xsqrt(a) == sqrtf(a) for all 2^32 inputs.
// Prints the mismatch counts and exits 1 on any mismatch.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I../rust-swift-raytracer_amd/csrc
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "exactdiv.h"

#pragma clang fp contract(off)

using namespace rtamd;

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(2);                                                                  \
        }                                                                             \
    } while (0)

struct Bad {
    unsigned long long count;
    uint32_t first_a, first_b;
};

__device__ void record(Bad *bad, uint32_t a, uint32_t b) {
    if (atomicAdd(&bad->count, 1ull) == 0) {
        bad->first_a = a;
        bad->first_b = b;
    }
}

__global__ void rcp_kernel(uint32_t lo, uint32_t n, Bad *bad) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t bits = lo + i;
        const float b = __uint_as_float(bits);
        const float ref = 1.0f / b;
        const float y = xdiv_rcp(b);
        if (__float_as_uint(y) != __float_as_uint(ref) || !xdiv_den_ok(b)) record(bad, 0, bits);
    }
}

// numerator word: sign | exponent | every significand; den[blockIdx.y]
__global__ void div_kernel(const uint32_t *den, const uint32_t *numhi, Bad *bad) {
    const float b = __uint_as_float(den[blockIdx.y]);
    const float y = xdiv_rcp(b);
    const uint32_t hi = numhi[blockIdx.y];
    for (uint32_t m = blockIdx.x * blockDim.x + threadIdx.x; m < (1u << 23); m += gridDim.x * blockDim.x) {
        const uint32_t abits = hi | m;
        const float a = __uint_as_float(abits);
        const float q = xdiv(a, b, y);
        const float ref = a / b;
        if (__float_as_uint(q) != __float_as_uint(ref) || !xdiv_num3_ok(a, 0.0f, 0.0f))
            record(bad, abits, __float_as_uint(b));
    }
}

__global__ void edge_kernel(const uint32_t *den, uint32_t nden, Bad *bad, Bad *guard) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nden) return;
    const float b = __uint_as_float(den[i]);
    const float y = xdiv_rcp(b);
    const float nums[8] = {0.0f, -0.0f, 0x1p-60f, -0x1p-60f, 0x1.fffffep59f, -0x1.fffffep59f, 1.0f, -3.0f};
    for (int k = 0; k < 8; ++k) {
        const float a = nums[k];
        if (__float_as_uint(xdiv(a, b, y)) != __float_as_uint(a / b)) record(bad, __float_as_uint(a), den[i]);
        if (!xdiv_num3_ok(a, 1.0f, -1.0f)) record(guard, __float_as_uint(a), 1);
    }
    if (i == 0) {
        // values the guards must reject
        const float rej_num[7] = {0x1.fffffep-61f, 0x1p60f, __builtin_inff(), __builtin_nanf(""), 1e-40f,
                                  -0x1p60f, -__builtin_inff()};
        for (int k = 0; k < 7; ++k) {
            if (xdiv_num3_ok(1.0f, rej_num[k], 0.0f)) record(guard, __float_as_uint(rej_num[k]), 2);
            if (xdiv_num3_ok(rej_num[k], 1.0f, 0.0f)) record(guard, __float_as_uint(rej_num[k]), 5);
            if (xdiv_num3_ok(0.0f, 1.0f, rej_num[k])) record(guard, __float_as_uint(rej_num[k]), 6);
        }
        const float rej_den[7] = {0.0f, -1.0f, 0x1.fffffep-41f, 0x1.000002p40f, __builtin_inff(), __builtin_nanf(""), -0.0f};
        for (int k = 0; k < 7; ++k)
            if (xdiv_den_ok(rej_den[k])) record(guard, __float_as_uint(rej_den[k]), 3);
        if (!xdiv_den_ok(0x1p-40f) || !xdiv_den_ok(0x1p40f)) record(guard, 0, 4);
    }
}

// xsqrt(a) == sqrtf(a), bit for bit, for every 32-bit input (NaNs included)
__global__ void sqrt_kernel(Bad *bad) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < (1ull << 32);
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t bits = (uint32_t)i;
        const float a = __uint_as_float(bits);
        if (__float_as_uint(xsqrt(a)) != __float_as_uint(__builtin_sqrtf(a))) record(bad, bits, 0);
    }
}

static uint32_t xs32(uint32_t &s) {
    s ^= s << 13;
    s ^= s >> 17;
    s ^= s << 5;
    return s;
}

int main(int argc, char **argv) {
    const uint32_t nden = argc > 1 ? (uint32_t)atoi(argv[1]) : 4096u;
    Bad *bad;
    CHECK(hipMallocManaged(&bad, 3 * sizeof(Bad)));
    for (int k = 0; k < 3; ++k) bad[k] = Bad{0, 0, 0};

    // 1. every reciprocal in range
    const uint32_t lo = 0x2B800000u, hi = 0x53800000u;
    hipLaunchKernelGGL(rcp_kernel, dim3(8192), dim3(256), 0, 0, lo, hi - lo + 1u, bad);
    CHECK(hipDeviceSynchronize());
    printf("rcp: %u values in [2^-40, 2^40], %llu mismatches", hi - lo + 1u, bad[0].count);
    if (bad[0].count) printf(" (first b=0x%08x)", bad[0].first_b);
    printf("\n");

    // 2. every numerator significand against nden denominators
    std::vector<uint32_t> den(nden), numhi(nden);
    const uint32_t specials[] = {0x3F800000u, 0x3F800001u, 0x3FFFFFFFu, 0x3FC00000u, 0x3F7FFFFFu,
                                 0x3FAAAAABu, 0x40400000u, 0x2B800000u, 0x53800000u, 0x2B800001u,
                                 0x537FFFFFu, 0x44EFE000u /* 1919 */, 0x44868000u /* 1076 */};
    uint32_t s = 2547549u;
    for (uint32_t i = 0; i < nden; ++i) {
        uint32_t d;
        if (i < sizeof(specials) / 4) {
            d = specials[i];
        } else {
            const uint32_t e = 87u + xs32(s) % 81u;  // 2^-40 .. 2^40
            d = (e << 23) | (xs32(s) & 0x7FFFFFu);
            if (i % 7 == 0) d |= 0x7FFF00u;  // long runs of ones
        }
        den[i] = d;
        const uint32_t ea = 67u + xs32(s) % 120u;  // numerator 2^-60 .. 2^59
        numhi[i] = ((xs32(s) & 1u) << 31) | (ea << 23);
    }
    uint32_t *dden, *dnum;
    CHECK(hipMalloc(&dden, nden * 4));
    CHECK(hipMalloc(&dnum, nden * 4));
    CHECK(hipMemcpy(dden, den.data(), nden * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dnum, numhi.data(), nden * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(div_kernel, dim3(1024, nden), dim3(256), 0, 0, dden, dnum, bad + 1);
    CHECK(hipDeviceSynchronize());
    printf("div: %u denominators x 2^23 numerator significands, %llu mismatches", nden, bad[1].count);
    if (bad[1].count) printf(" (first a=0x%08x b=0x%08x)", bad[1].first_a, bad[1].first_b);
    printf("\n");

    // 3. edge numerators and guard predicates
    hipLaunchKernelGGL(edge_kernel, dim3((nden + 255) / 256), dim3(256), 0, 0, dden, nden, bad + 1, bad + 2);
    CHECK(hipDeviceSynchronize());
    printf("edges: %llu division mismatches, %llu guard errors", bad[1].count, bad[2].count);
    if (bad[2].count) printf(" (first value 0x%08x, case %u)", bad[2].first_a, bad[2].first_b);
    printf("\n");
    // 4. every square root
    Bad *sq;
    CHECK(hipMallocManaged(&sq, sizeof(Bad)));
    *sq = Bad{0, 0, 0};
    hipLaunchKernelGGL(sqrt_kernel, dim3(16384), dim3(256), 0, 0, sq);
    CHECK(hipDeviceSynchronize());
    printf("sqrt: all 2^32 inputs, %llu mismatches", sq->count);
    if (sq->count) printf(" (first a=0x%08x)", sq->first_a);
    printf("\n");
    const bool ok = bad[0].count == 0 && bad[1].count == 0 && bad[2].count == 0 && sq->count == 0;
    printf("%s\n", ok ? "exactdiv OK" : "exactdiv FAILED");
    return ok ? 0 : 1;
}
