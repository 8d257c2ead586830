// Latency of a dependent record lookup from a 32-VGPR block (uniform dynamic
// VGPR index + readlane) vs the same chase through LDS (traceback design).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <stdint.h>

__global__ void k_vgpr(const uint32_t *in, uint32_t *out, unsigned long long *cyc, int n)
{
    uint32_t blk[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) blk[i] = in[i * 64 + threadIdx.x];
    uint32_t r = __builtin_amdgcn_readfirstlane(in[2047]), acc = 0;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int s = 0; s < n; ++s) {
        const uint32_t v = blk[__builtin_amdgcn_readfirstlane(r & 31)];
        const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)v, (int)(r >> 5) & 63);
        r = c;
        acc += c;
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_lds(const uint32_t *in, uint32_t *out, unsigned long long *cyc, int n)
{
    __shared__ uint32_t lds[2048];
    for (int i = threadIdx.x; i < 2048; i += 64) lds[i] = in[i];
    __syncthreads();
    uint32_t r = __builtin_amdgcn_readfirstlane(in[2047]), acc = 0;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int s = 0; s < n; ++s) {
        const uint32_t c = __builtin_amdgcn_readfirstlane(lds[r & 2047]);
        r = c;
        acc += c;
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main()
{
    uint32_t *in, *out;
    unsigned long long *cyc, h;
    hipMalloc(&in, 2048 * 4);
    hipMalloc(&out, 4096);
    hipMalloc(&cyc, 64);
    uint32_t hin[2048];
    for (int i = 0; i < 2048; ++i) hin[i] = (i * 1103515245u + 12345u) >> 5;
    hipMemcpy(in, hin, sizeof(hin), hipMemcpyHostToDevice);
    const int n = 4096;
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_vgpr, dim3(1), dim3(64), 0, 0, in, out, cyc, n);
        hipDeviceSynchronize();
    }
    hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
    printf("vgpr-indexed record chase  %8.2f cycles/step\n", (double)h / n);
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_lds, dim3(1), dim3(64), 0, 0, in, out, cyc, n);
        hipDeviceSynchronize();
    }
    hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
    printf("lds record chase           %8.2f cycles/step\n", (double)h / n);
    return 0;
}
