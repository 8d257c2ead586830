// exit_cost.cpp -- what a process exit costs after holding device memory and
// pinned host memory (the CLI's timed region ends at its exit).
//
//   exit_cost DEV_GB HOST_GB MODE   (MODE: 0 hipHostMalloc, 1 THP mapping +
//                                    hipHostRegister; DEV_GB of hipMalloc,
//                                    touched by hipMemset)
// Prints the epoch right before _Exit; tools/ubench/exit_cost.py times the
// rest from the parent.
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static double epoch()
{
    return std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv)
{
    if (argc < 4) return 2;
    const double dev_gb = atof(argv[1]), host_gb = atof(argv[2]);
    const int mode = atoi(argv[3]);
    std::vector<void *> dev;
    const size_t piece = 8ull << 30;
    for (size_t left = (size_t)(dev_gb * (1ull << 30)); left;) {
        const size_t n = left < piece ? left : piece;
        void *p = nullptr;
        if (hipMalloc(&p, n) != hipSuccess) return 3;
        if (hipMemset(p, 0, n) != hipSuccess) return 4;
        dev.push_back(p);
        left -= n;
    }
    const size_t hb = (size_t)(host_gb * (1ull << 30)) & ~size_t((2u << 20) - 1);
    if (hb) {
        void *h = nullptr;
        if (mode == 0) {
            if (hipHostMalloc(&h, hb, hipHostMallocDefault) != hipSuccess) return 5;
            memset(h, 1, hb);
        } else {
            h = mmap(nullptr, hb, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
            if (h == MAP_FAILED) return 6;
            madvise(h, hb, MADV_HUGEPAGE);
            memset(h, 1, hb);
            if (hipHostRegister(h, hb, hipHostRegisterDefault) != hipSuccess) return 7;
        }
    }
    if (hipDeviceSynchronize() != hipSuccess) return 8;
    printf("%.6f\n", epoch());
    fflush(stdout);
    std::_Exit(0);
}
