// s_barrier round trip for a 2-wave workgroup, waves idle or doing equal work
#include <hip/hip_runtime.h>
#include <cstdio>
#define N 256
__global__ void __launch_bounds__(128) k_bar(unsigned long long *cyc, int work)
{
    int a = threadIdx.x;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) {
        for (int k = 0; k < work; ++k) asm volatile("v_add_u32 %0, %0, %0" : "+v"(a));
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[threadIdx.x >> 6] = t1 - t0 + (a == 12345);
}
int main()
{
    unsigned long long *cyc, h[2];
    (void)hipMalloc(&cyc, 16);
    for (int grid : {1, 1000, 2000}) {
        for (int work : {0, 16, 64}) {
            for (int rep = 0; rep < 3; ++rep) {
                hipLaunchKernelGGL(k_bar, dim3(grid), dim3(128), 0, 0, cyc, work);
                (void)hipDeviceSynchronize();
            }
            (void)hipMemcpy(h, cyc, 16, hipMemcpyDeviceToHost);
            printf("grid %4d, %2d VALU per wave between barriers: %.1f ticks per iteration\n", grid, work,
                   (double)h[0] / N);
        }
    }
    return 0;
}
