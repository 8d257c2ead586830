// Isolated cost of wave 0's DP row (dpA_row) and wave 1's (dpB_row): one
// workgroup, synthetic graph = one chain whose bases equal the read (every row
// takes the "band moved by one" path after the first W/2 rows).
#include "../../ccsx_amd/csrc/ccsx_kernel.hip"
#include <cstdio>

using namespace ccsx;

__global__ void __launch_bounds__(128) k_rows(unsigned long long *cyc, int *out, uint32_t nrow, uint32_t m, int with_b)
{
    extern __shared__ int32_t smem[];
    const int lane = lane_id();
    Z z;
    z.lds = smem;
    z.rd = reinterpret_cast<uint8_t *>(smem + kLdsFixed);
    z.R = nrow;
    z.status = 0;
    // read: code(j) = (j * 7 + j / 5) & 3, nibble pairs
    for (uint32_t b = threadIdx.x; b < m / 2 + 64; b += 128) {
        auto cd = [](uint32_t j) { return (j * 7u + j / 5u) & 3u; };
        const uint32_t j = 2 * b;
        z.rd[b] = (uint8_t)((cd(j) | cd(j + 1) << 2) | (cd(j + 1) | cd(j + 2) << 2) << 4);
    }
    for (int i = threadIdx.x; i < kRingA * 16; i += 128) {
        const int k = i & 15;
        const int w = k < 4 ? k : k < 8 ? kHc + kW + (k - 4) : k < 12 ? kDc - 4 + (k - 8) : kDc + kW + (k - 12);
        smem[kLdsRing + (i >> 4) * kRowW + w] = k < 8 ? kNegH : kNeg;
    }
    __syncthreads();
    if (threadIdx.x >= 64) return;
    AState S;
    S.H0 = S.H1 = kNegH, S.D0 = S.D1 = kNeg;
    S.pOff = 0, S.pArg = 0, S.vOff = 0, S.vKey = 0;
    S.qn = z.rd[lane];
    const int32_t lim = (int32_t)m - kW;
    const LaneK c = lane_consts(lane);
    unsigned long long t0 = 0, fast = 0, tb = 0;
    BState B;
    B.bE = INT32_MIN, B.bKey = 0, B.vMi = kNone, B.nmulti = 0, B.mg0 = 0;
    for (uint32_t r = 0; r < nrow; ++r) {
        if ((r & 63u) == 0) {
            const uint32_t rr = r + lane;
            const uint32_t bse = (rr * 7u + rr / 5u) & 3u;
            S.W.cur.info = bse | (rr ? (kInfoChain | (1u << 8)) : 0u);
            S.W.cur.p0 = rr ? rr - 1 : 0u;
            S.W.cur.p1 = S.W.cur.p2 = S.W.cur.p3 = 0;
        }
        if (r == 256) t0 = __builtin_amdgcn_s_memtime();
        const int32_t coff = min(max(S.pArg + 1 - kW / 2, 0), lim);
        fast += (coff - S.pOff == 1);
        dpA_row(z, S, r, lim, c);
        if (with_b) {
            B.W.cur = S.W.cur;
            z.lds[kLdsOffRing + lane] = S.vOff;
            const int32_t vOff = S.vOff;
            unsigned long long u0;
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(u0)::"memory");
            dpB_row(z, B, r, m, lim, vOff, c);
            unsigned long long u1;
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(u1)::"memory");
            if (r >= 256) tb += u1 - u0;
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[lane] = S.H0 + S.H1;
    out[64 + lane] = B.bE;
    if (lane == 0) cyc[0] = t1 - t0, cyc[1] = fast, cyc[2] = tb;
}

int main()
{
    unsigned long long *cyc, h[3];
    int *out;
    (void)hipMalloc(&cyc, 24);
    (void)hipMalloc(&out, 1024);
    const uint32_t nrow = 4096 + 256, m = 8192;
    const uint32_t lds = (kLdsFixedWords + m / 8 + 64) * 4;
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_rows), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    for (int wb = 0; wb < 2; ++wb) {
        for (int rep = 0; rep < 3; ++rep) {
            hipLaunchKernelGGL(k_rows, dim3(1), dim3(128), lds, 0, cyc, out, nrow, m, wb);
            (void)hipDeviceSynchronize();
        }
        (void)hipMemcpy(h, cyc, 24, hipMemcpyDeviceToHost);
        if (!wb)
            printf("dpA_row: %.1f ticks/row over %u rows (%llu of %u rows on the fast path)\n",
                   (double)h[0] / (nrow - 256), nrow - 256, h[1], nrow);
        else
            printf("dpB_row: %.1f ticks/row (stamped, incl. ~30 ticks of stamp overhead)\n", (double)h[2] / (nrow - 256));
    }
    return 0;
}
