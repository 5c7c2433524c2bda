// Issue rate of VALU encodings on gfx950: 32-bit VOP2 forms against 64-bit
// VOP3 forms of the same operation (probe, not product).
#include <hip/hip_runtime.h>
#include <cstdio>
#define CHAINS 8
template <int KIND>
__global__ __launch_bounds__(256) void kern(float *out, int iters) {
    float a[CHAINS];
    float b = 1.0000001f + threadIdx.x * 1e-9f, c = 0.5f;
#pragma unroll
    for (int i = 0; i < CHAINS; ++i) a[i] = threadIdx.x + i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < CHAINS; ++i) {
            if (KIND == 0) asm volatile("v_add_f32_e32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            if (KIND == 1) asm volatile("v_add_f32_e64 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            if (KIND == 2) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
            if (KIND == 3) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
            if (KIND == 4) asm volatile("v_fmac_f32_e32 %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
            if (KIND == 5) asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            if (KIND == 6) asm volatile("v_add_f32_e32 %0, %0, %1\n v_add_f32_e32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            if (KIND == 7) asm volatile("v_add_f32_e32 %0, %0, %1\n s_nop 0" : "+v"(a[i]) : "v"(b));
        }
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < CHAINS; ++i) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int KIND>
double run(float *out, int blocks, int iters, int per) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(kern<KIND>, dim3(blocks), dim3(256), 0, 0, out, iters);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(kern<KIND>, dim3(blocks), dim3(256), 0, 0, out, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return (double)blocks * 256 * iters * CHAINS * per / (ms * 1e-3) / 1e12;
}
int main() {
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    float *out;
    (void)hipMalloc(&out, (size_t)prop.multiProcessorCount * 8 * 256 * sizeof(float));
    const char *names[] = {"v_add_f32_e32", "v_add_f32_e64", "v_fma_f32", "v_max3_f32", "v_fmac_f32_e32",
                           "v_add_u32_e32", "2x v_add_f32_e32", "v_add_f32_e32 + s_nop"};
    for (int wpc : {1, 2, 4, 8}) {
        const int blocks = prop.multiProcessorCount * wpc;
        const int iters = 20000;
        double r[8] = {run<0>(out, blocks, iters, 1), run<1>(out, blocks, iters, 1), run<2>(out, blocks, iters, 1),
                       run<3>(out, blocks, iters, 1), run<4>(out, blocks, iters, 1), run<5>(out, blocks, iters, 1),
                       run<6>(out, blocks, iters, 2), run<7>(out, blocks, iters, 1)};
        for (int k = 0; k < 8; ++k)
            std::printf("{\"waves_per_simd\": %d, \"op\": \"%s\", \"tera_lane_insts_per_s\": %.2f}\n", wpc, names[k], r[k]);
    }
    return 0;
}
