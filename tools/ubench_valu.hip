// ubench_valu.hip -- issue-rate microbenchmark for the f32 VALU forms the
// sphere test can use on gfx950: v_add_f32 / v_mul_f32 (one f32 op per lane)
// against v_pk_add_f32 / v_pk_mul_f32 (two f32 ops per lane).  Decides
// whether packing two spheres per instruction pays.
// Build: hipcc --offload-arch=gfx950 -O3 -o ubench_valu ubench_valu.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float float2_t __attribute__((ext_vector_type(2)));

#define CHAINS 8

template <int KIND>
__global__ __launch_bounds__(256) void kern(float *out, int iters) {
    float a[CHAINS];
    float2_t p[CHAINS];
    float b = 1.0000001f + threadIdx.x * 1e-9f;
    float2_t pb = {b, b};
#pragma unroll
    for (int i = 0; i < CHAINS; ++i) { a[i] = threadIdx.x + i; p[i] = float2_t{a[i], a[i] + 1.0f}; }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < CHAINS; ++i) {
            if (KIND == 0) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            if (KIND == 1) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            if (KIND == 2) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p[i]) : "v"(pb));
            if (KIND == 3) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p[i]) : "v"(pb));
            if (KIND == 4) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(b));
        }
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < CHAINS; ++i) s += a[i] + p[i].x + p[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int KIND>
double run(float *out, int blocks, int iters) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(kern<KIND>, dim3(blocks), dim3(256), 0, 0, out, iters);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern<KIND>, dim3(blocks), dim3(256), 0, 0, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double lane_ops = (double)blocks * 256 * iters * CHAINS * ((KIND == 2 || KIND == 3) ? 2 : 1);
    return lane_ops / (ms * 1e-3) / 1e12;  // T lane-ops/s
}

int main() {
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int blocks = prop.multiProcessorCount * 8;
    float *out;
    hipMalloc(&out, (size_t)blocks * 256 * sizeof(float));
    const int iters = 20000;
    const char *names[] = {"v_add_f32", "v_mul_f32", "v_pk_add_f32", "v_pk_mul_f32", "v_fma_f32"};
    double r[5] = {run<0>(out, blocks, iters), run<1>(out, blocks, iters),
                   run<2>(out, blocks, iters), run<3>(out, blocks, iters),
                   run<4>(out, blocks, iters)};
    for (int k = 0; k < 5; ++k)
        std::printf("{\"op\": \"%s\", \"tera_lane_f32_ops_per_s\": %.2f}\n", names[k], r[k]);
    hipFree(out);
    return 0;
}
