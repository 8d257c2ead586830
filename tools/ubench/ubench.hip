// Micro-benchmarks of instruction latency for a single wave on MI355X
// (calibrates the DP row-loop cost model in DESIGN.md).
#include <hip/hip_runtime.h>
#include <cstdio>

#define N 512

__global__ void k_valu_dep(int *out, unsigned long long *cyc, int seed)
{
    int v = threadIdx.x + seed;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("v_add_u32 %0, %0, %0" : "+v"(v));
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = v;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_valu_ind(int *out, unsigned long long *cyc, int seed)
{
    int a = threadIdx.x + seed, b = a + 1, c = a + 2, d = a + 3;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < N / 4; ++i)
        asm volatile("v_add_u32 %0, %0, %0\n\tv_add_u32 %1, %1, %1\n\tv_add_u32 %2, %2, %2\n\tv_add_u32 %3, %3, %3"
                     : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a + b + c + d;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_dpp_dep(int *out, unsigned long long *cyc, int seed)
{
    int v = threadIdx.x + seed;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < N / 2; ++i)
        asm volatile("s_nop 1\n\tv_max_i32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(v));
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = v;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_readlane(int *out, unsigned long long *cyc, int seed)
{
    int v = threadIdx.x + seed;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N / 4; ++i) {
        int s = __builtin_amdgcn_readlane(v, 63);
        v = v + s;
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = v;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_lds_chase(int *out, unsigned long long *cyc, int seed)
{
    __shared__ int lds[256];
    lds[threadIdx.x] = (threadIdx.x * 7 + seed) & 63;
    lds[threadIdx.x + 64] = (threadIdx.x * 5 + 1) & 63;
    __syncthreads();
    int p = threadIdx.x;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N / 8; ++i) p = lds[p];
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = p;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_ballot(int *out, unsigned long long *cyc, int seed)
{
    int v = threadIdx.x + seed;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N / 4; ++i) {
        unsigned long long b = __ballot(v > 40);
        v += (int)__builtin_ctzll(b | (1ull << 63));
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = v;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main()
{
    int *out;
    unsigned long long *cyc, h;
    hipMalloc(&out, 4096);
    hipMalloc(&cyc, 64);
    struct {
        const char *name;
        void (*k)(int *, unsigned long long *, int);
        int ops;
    } ks[] = {{"valu dependent add", k_valu_dep, N}, {"valu 4 independent chains", k_valu_ind, N},
              {"dpp max dependent (+s_nop 1)", k_dpp_dep, N / 2}, {"readlane->valu loop", k_readlane, N / 4},
              {"lds pointer chase", k_lds_chase, N / 8}, {"ballot+ctz loop", k_ballot, N / 4}};
    for (auto &k : ks) {
        for (int rep = 0; rep < 3; ++rep) {
            hipLaunchKernelGGL(k.k, dim3(1), dim3(64), 0, 0, out, cyc, rep);
            hipDeviceSynchronize();
        }
        hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
        printf("%-32s %8.2f cycles/op\n", k.name, (double)h / k.ops);
    }
    return 0;
}
