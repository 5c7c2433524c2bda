// ubench_exec.hip -- does a wave64 VALU instruction cost less when one 32-lane
// half of the exec mask is empty?  Each wave runs a long chain of independent
// v_fma_f32 with exec = all 64 lanes, the low 32 lanes, every other lane (32
// lanes spread over both halves), or 16 low lanes; prints ns per wave per
// instruction for each.  Diagnostic.
//   hipcc -O3 --offload-arch=gfx950 ubench_exec.hip -o ubench_exec
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 4096;

__global__ __launch_bounds__(256) void chain(float *out, int mode) {
    const int lane = threadIdx.x % 64;
    bool on = true;
    if (mode == 1) on = lane < 32;
    if (mode == 2) on = (lane & 1) == 0;
    if (mode == 3) on = lane < 16;
    float a = threadIdx.x * 1e-3f, b = a + 1, c = a + 2, d = a + 3, e = a + 4, f = a + 5, g = a + 6, h = a + 7;
    if (on) {
        for (int i = 0; i < kIters; ++i) {
            a = __builtin_fmaf(a, 1.0001f, 0.5f);
            b = __builtin_fmaf(b, 1.0001f, 0.5f);
            c = __builtin_fmaf(c, 1.0001f, 0.5f);
            d = __builtin_fmaf(d, 1.0001f, 0.5f);
            e = __builtin_fmaf(e, 1.0001f, 0.5f);
            f = __builtin_fmaf(f, 1.0001f, 0.5f);
            g = __builtin_fmaf(g, 1.0001f, 0.5f);
            h = __builtin_fmaf(h, 1.0001f, 0.5f);
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = ((a + b) + (c + d)) + ((e + f) + (g + h));
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 8;  // 8 waves per SIMD (4 waves per block)
    float *out;
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipEvent_t t0, t1;
    hipEventCreate(&t0);
    hipEventCreate(&t1);
    const char *names[] = {"all 64 lanes", "low 32 lanes", "even lanes (32)", "low 16 lanes"};
    for (int rep = 0; rep < 2; ++rep)
        for (int mode = 0; mode < 4; ++mode) {
            hipLaunchKernelGGL(chain, dim3(blocks), dim3(256), 0, 0, out, mode);
            hipEventRecord(t0);
            hipLaunchKernelGGL(chain, dim3(blocks), dim3(256), 0, 0, out, mode);
            hipEventRecord(t1);
            hipEventSynchronize(t1);
            float ms = 0;
            hipEventElapsedTime(&ms, t0, t1);
            // per SIMD: waves * iterations * 8 instructions, in sequence
            const double waves_per_simd = (double)blocks * 4 / (cus * 4);
            const double cyc = ms * 1e-3 * 2.4e9 / (waves_per_simd * kIters * 8);
            if (rep) std::printf("%-16s %.3f ms  %.2f cycles per wave-instruction (at 2.4 GHz)\n", names[mode], ms, cyc);
        }
    hipFree(out);
    return 0;
}
