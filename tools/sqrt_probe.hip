// sqrt_probe.hip -- how far is gfx950's v_sqrt_f32 from the correctly rounded
// square root?  For every positive normal float a, compares
// __builtin_amdgcn_sqrtf(a) (one v_sqrt_f32) with HIP's IEEE sqrtf (LLVM's
// correction sequence) and counts results 1 ulp low / 1 ulp high / further
// off, per input-exponent band.  Diagnostic for a cheaper exact sqrt.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#pragma clang fp contract(off)

__global__ void probe(uint32_t lo, uint32_t n, unsigned long long *cnt) {
    unsigned long long lowc = 0, highc = 0, far = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const float a = __uint_as_float(lo + i);
        const uint32_t hw = __float_as_uint(__builtin_amdgcn_sqrtf(a));
        const uint32_t ref = __float_as_uint(__builtin_sqrtf(a));
        if (hw == ref) continue;
        if (hw + 1 == ref) ++lowc;
        else if (hw == ref + 1) ++highc;
        else ++far;
    }
    if (lowc) atomicAdd(&cnt[0], lowc);
    if (highc) atomicAdd(&cnt[1], highc);
    if (far) atomicAdd(&cnt[2], far);
}

int main() {
    unsigned long long *cnt;
    hipMallocManaged(&cnt, 3 * 8);
    // bands of 16 binades from 2^-126 up to 2^128
    unsigned long long tot[3] = {0, 0, 0};
    for (int e = 1; e < 255; e += 16) {
        const int e1 = e + 16 < 255 ? e + 16 : 255;
        cnt[0] = cnt[1] = cnt[2] = 0;
        const uint32_t lo = (uint32_t)e << 23, n = (uint32_t)(e1 - e) << 23;
        hipLaunchKernelGGL(probe, dim3(4096), dim3(256), 0, 0, lo, n, cnt);
        hipDeviceSynchronize();
        printf("exp [%4d, %4d): low %llu high %llu far %llu\n", e - 127, e1 - 127, cnt[0], cnt[1], cnt[2]);
        for (int k = 0; k < 3; ++k) tot[k] += cnt[k];
    }
    printf("total: low %llu high %llu far %llu\n", tot[0], tot[1], tot[2]);
    return 0;
}
