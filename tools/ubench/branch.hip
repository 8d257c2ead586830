// Cost of control flow for a lone wave: taken scalar branches, exec-masked
// (divergent) if-blocks, v_readlane -> SALU -> branch chains.
#include <hip/hip_runtime.h>
#include <cstdio>
#define N 256

__global__ void k_straight(int *out, unsigned long long *cyc, int seed)
{
    int a = threadIdx.x + seed, b = a + 1;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < N / 2; ++i) asm volatile("v_add_u32 %0, %0, %1\n\tv_add_u32 %1, %1, %0" : "+v"(a), "+v"(b));
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a + b;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_taken(int *out, unsigned long long *cyc, int seed)
{
    int a = threadIdx.x + seed, b = a + 1;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < N / 2; ++i)
        asm volatile("v_add_u32 %0, %0, %1\n\ts_branch 1f\n\tv_add_u32 %1, %1, %1\n1:\n\tv_add_u32 %1, %1, %0" : "+v"(a), "+v"(b));
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a + b;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_scc(int *out, unsigned long long *cyc, int seed)
{
    int a = threadIdx.x + seed, b = a + 1, s = seed;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < N / 2; ++i)
        asm volatile("v_add_u32 %0, %0, %1\n\ts_cmp_eq_u32 %2, 77\n\ts_cbranch_scc1 1f\n\tv_add_u32 %1, %1, %0\n1:" : "+v"(a), "+v"(b), "+s"(s));
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a + b + s;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_exec(int *out, unsigned long long *cyc, int seed)
{
    int a = threadIdx.x + seed, b = a + 1;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < N / 2; ++i)
        asm volatile("v_add_u32 %0, %0, %1\n\tv_cmp_eq_u32 vcc, 63, %0\n\ts_and_saveexec_b64 s[40:41], vcc\n\ts_cbranch_execz 1f\n"
                     "\tv_add_u32 %1, %1, %0\n1:\n\ts_or_b64 exec, exec, s[40:41]" : "+v"(a), "+v"(b) :: "vcc", "s40", "s41");
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a + b;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_rl_chain(int *out, unsigned long long *cyc, int seed)
{
    int a = threadIdx.x + seed, s = seed;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < N / 4; ++i)
        asm volatile("v_readlane_b32 %1, %0, 5\n\ts_add_u32 %1, %1, 1\n\ts_and_b32 %1, %1, 63\n\tv_add_u32 %0, %1, %0" : "+v"(a), "+s"(s));
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a + s;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_lds_rt(int *out, unsigned long long *cyc, int seed)
{
    __shared__ int lds[64];
    lds[threadIdx.x] = threadIdx.x;
    int a = threadIdx.x + seed;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < N / 4; ++i)
        asm volatile("ds_write_b32 %1, %0\n\tds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)\n\tv_add_u32 %0, %0, 1" : "+v"(a) : "v"(threadIdx.x * 4));
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main()
{
    int *out;
    unsigned long long *cyc, h;
    hipMalloc(&out, 4096 * 4);
    hipMalloc(&cyc, 64);
    struct {
        const char *name;
        void (*k)(int *, unsigned long long *, int);
        int units;
    } ks[] = {{"2 dep VALU (per pair)", k_straight, N / 2}, {"2 VALU + taken s_branch", k_taken, N / 2},
              {"VALU + s_cmp + not-taken cbranch + VALU", k_scc, N / 2},
              {"VALU + exec-masked 1-op if", k_exec, N / 2}, {"readlane->2 SALU->VALU chain", k_rl_chain, N / 4},
              {"ds_write+ds_read+wait round trip", k_lds_rt, N / 4}};
    for (auto &k : ks) {
        for (int rep = 0; rep < 3; ++rep) {
            hipLaunchKernelGGL(k.k, dim3(1), dim3(64), 0, 0, out, cyc, rep);
            (void)hipDeviceSynchronize();
        }
        (void)hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
        printf("%-42s %7.2f ticks per unit\n", k.name, (double)h / k.units);
    }
    return 0;
}
