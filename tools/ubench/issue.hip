// Issue-rate calibration for one wave per SIMD vs two (DESIGN.md cost model):
// straight-line streams of independent VALU, mixed VALU+SALU, DPP, readlane.
#include <hip/hip_runtime.h>
#include <cstdio>
#define N 256
#define REP8(x) x x x x x x x x

__global__ void k_valu(int *out, unsigned long long *cyc, int seed)
{
    int a = threadIdx.x + seed, b = a + 1, c = a + 2, d = a + 3, e = a + 4, f = a + 5, g = a + 6, h = a + 7;
    __builtin_amdgcn_s_barrier();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < N / 8; ++i)
        asm volatile(REP8("v_add_u32 %0, %1, %0\n\t") : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h));
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + threadIdx.x] = a + b + c + d + e + f + g + h;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void k_mix(int *out, unsigned long long *cyc, int seed)
{
    int a = threadIdx.x + seed, b = a + 1, c = a + 2, d = a + 3;
    int s0 = seed, s1 = seed + 1, s2 = seed + 2, s3 = seed + 3;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < N / 8; ++i)
        asm volatile("v_add_u32 %0, %0, %4\n\ts_add_u32 %4, %4, %5\n\tv_add_u32 %1, %1, %5\n\ts_add_u32 %5, %5, %6\n\t"
                     "v_add_u32 %2, %2, %6\n\ts_add_u32 %6, %6, %7\n\tv_add_u32 %3, %3, %7\n\ts_add_u32 %7, %7, %4"
                     : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3));
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + threadIdx.x] = a + b + c + d + s0 + s1 + s2 + s3;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void k_salu(int *out, unsigned long long *cyc, int seed)
{
    int s0 = seed, s1 = seed + 1, s2 = seed + 2, s3 = seed + 3;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < N / 4; ++i)
        asm volatile("s_add_u32 %0, %0, %1\n\ts_add_u32 %1, %1, %2\n\ts_add_u32 %2, %2, %3\n\ts_add_u32 %3, %3, %0"
                     : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3));
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + threadIdx.x] = s0 + s1 + s2 + s3;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void k_dpp4(int *out, unsigned long long *cyc, int seed)
{
    int a = threadIdx.x + seed, b = a + 1, c = a + 2, d = a + 3;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < N / 4; ++i)
        asm volatile("v_max_i32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
                     "v_max_i32_dpp %1, %1, %1 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
                     "v_max_i32_dpp %2, %2, %2 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
                     "v_max_i32_dpp %3, %3, %3 row_shr:1 row_mask:0xf bank_mask:0xf"
                     : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + threadIdx.x] = a + b + c + d;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void k_wall(unsigned long long *cyc)
{
    // memtime vs a fixed-rate clock: 100 MHz s_memrealtime
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    int a = threadIdx.x;
    for (int i = 0; i < 200000; ++i) asm volatile("v_add_u32 %0, %0, %0" : "+v"(a));
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) cyc[0] = t1 - t0, cyc[1] = r1 - r0, cyc[2] = a;
}

int main()
{
    int *out;
    unsigned long long *cyc, h[4096];
    hipMalloc(&out, 4096 * 64 * 4);
    hipMalloc(&cyc, 4096 * 8);
    struct {
        const char *name;
        void (*k)(int *, unsigned long long *, int);
        int ops;
    } ks[] = {{"valu 8 indep chains", k_valu, N}, {"valu+salu alternating", k_mix, N},
              {"salu 4 chains", k_salu, N}, {"dpp max 4 chains", k_dpp4, N}};
    for (int grid : {1, 1024, 2048, 4096}) {
        for (auto &k : ks) {
            for (int rep = 0; rep < 3; ++rep) {
                hipLaunchKernelGGL(k.k, dim3(grid), dim3(64), 0, 0, out, cyc, rep);
                hipDeviceSynchronize();
            }
            hipMemcpy(h, cyc, grid * 8, hipMemcpyDeviceToHost);
            double s = 0;
            for (int i = 0; i < grid; ++i) s += h[i];
            printf("grid %4d (%.0f waves/SIMD)  %-24s %6.2f ticks/op per wave\n", grid, grid / 1024.0, k.name,
                   s / grid / k.ops);
        }
    }
    hipLaunchKernelGGL(k_wall, dim3(1), dim3(64), 0, 0, cyc);
    hipDeviceSynchronize();
    hipMemcpy(h, cyc, 24, hipMemcpyDeviceToHost);
    printf("memtime/memrealtime = %.3f (memrealtime = 100 MHz -> memtime %.2f GHz)\n", (double)h[0] / h[1],
           (double)h[0] / h[1] * 0.1);
    return 0;
}
