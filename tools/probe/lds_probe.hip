// LDS limits of the device: per-block dynamic LDS above 64 KB (probe, not product)
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void __launch_bounds__(1024) touch(int n, int *out) {
    extern __shared__ int s[];
    for (int i = threadIdx.x; i < n; i += blockDim.x) s[i] = i;
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = s[n - 1];
}
int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    printf("sharedMemPerBlock %zu maxSharedMemoryPerMultiProcessor %zu sharedMemPerBlockOptin %zu\n",
           p.sharedMemPerBlock, p.maxSharedMemoryPerMultiProcessor, p.sharedMemPerBlockOptin);
    int *d;
    hipMalloc(&d, 4096);
    for (size_t kb : {60, 64, 70, 80, 100, 160}) {
        int nb = -1;
        hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, touch, 1024, kb * 1024);
        hipGetLastError();
        hipLaunchKernelGGL(touch, dim3(4), dim3(1024), kb * 1024, 0, (int)(kb * 256), d);
        hipError_t e2 = hipGetLastError();
        hipError_t e3 = hipDeviceSynchronize();
        printf("%zu KB: occupancy %d (%s) launch %s sync %s\n", kb, nb, hipGetErrorString(e), hipGetErrorString(e2),
               hipGetErrorString(e3));
    }
    hipFuncSetAttribute((const void *)touch, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    for (size_t kb : {70, 80}) {
        int nb = -1;
        hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, touch, 1024, kb * 1024);
        hipLaunchKernelGGL(touch, dim3(4), dim3(1024), kb * 1024, 0, (int)(kb * 256), d);
        hipError_t e2 = hipGetLastError();
        printf("after attr %zu KB: occupancy %d (%s) launch %s sync %s\n", kb, nb, hipGetErrorString(e),
               hipGetErrorString(e2), hipGetErrorString(hipDeviceSynchronize()));
    }
    return 0;
}
