// bspoa_gpu.cpp -- the bspoa-compatible API (include/ccsx_bspoa.h) on the GPU.
//
// beg/push collect reads on the host; end_bspoa stages them as one "ZMW" and
// runs the kSinglePoa kernel mode (SPEC.md §2-§6 on the device), which also
// writes the tidy MSA, so tidy_msa_bspoa only exposes it.
#include "ccsx_bspoa.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ccsx_gpu.h"

extern "C" int ccsx_gpu_single_poa(ccsx_ctx *c, const ccsx_zmw_in *z, const uint8_t **cns, uint32_t *ncns,
                                   const uint8_t **msa, uint32_t *ncols);

namespace {

struct Impl {
    ccsx_ctx *ctx = nullptr;
    std::string seqs;
    std::vector<uint32_t> off, len;
    ccsx_u1v cns{}, msacols{};
    ccsx_u4v msaidxs{};
};

[[noreturn]] void die(const char *what, const char *msg)
{
    fprintf(stderr, "[ccsx_bspoa] %s: %s\n", what, msg);
    abort();
}

template <class V, class T>
void put(V &v, const T *src, uint64_t n)
{
    if (n + 1 > v.cap) {
        v.cap = (n + 1) * 2;
        v.buffer = static_cast<decltype(v.buffer)>(realloc(v.buffer, v.cap * sizeof(T)));
        if (!v.buffer) die("alloc", "out of memory");
    }
    if (n) memcpy(v.buffer, src, n * sizeof(T));
    v.size = n;
}

}  // namespace

extern "C" {

BSPOA *init_bspoa(BSPOAPar par)
{
    if (par.M != 2 || par.X != -6 || par.O != -3 || par.E != -2 || par.Q != 0 || par.P != 0 || par.bandwidth != 128)
        die("init_bspoa", "only main.c's parameters (M=2 X=-6 O=-3 E=-2 Q=P=0 bandwidth=128) are supported");
    auto *im = new Impl();
    const char *dev = getenv("CCSX_DEVICE");
    if (ccsx_gpu_open(dev ? atoi(dev) : 0, &im->ctx)) die("init_bspoa", "cannot open the GPU");
    auto *g = static_cast<BSPOA *>(calloc(1, sizeof(BSPOA)));
    g->par = par;
    g->impl = im;
    g->cns = &im->cns;
    g->msaidxs = &im->msaidxs;
    g->msacols = &im->msacols;
    return g;
}

void beg_bspoa(BSPOA *g)
{
    auto *im = static_cast<Impl *>(g->impl);
    im->seqs.clear();
    im->off.clear();
    im->len.clear();
    im->cns.size = im->msaidxs.size = im->msacols.size = 0;
    g->nseq = 0;
}

void push_bspoa(BSPOA *g, char *seq, uint32_t len)
{
    auto *im = static_cast<Impl *>(g->impl);
    im->off.push_back((uint32_t)im->seqs.size());
    im->len.push_back(len);
    im->seqs.append(seq, len);
    g->nseq++;
}

void end_bspoa(BSPOA *g)
{
    auto *im = static_cast<Impl *>(g->impl);
    ccsx_zmw_in z{im->seqs.data(), im->off.data(), im->len.data(), (uint32_t)im->len.size()};
    const uint8_t *cns = nullptr, *msa = nullptr;
    uint32_t ncns = 0, ncols = 0;
    if (ccsx_gpu_single_poa(im->ctx, &z, &cns, &ncns, &msa, &ncols)) die("end_bspoa", ccsx_gpu_error(im->ctx));
    std::vector<uint8_t> codes(ncns);
    for (uint32_t i = 0; i < ncns; ++i) {
        const char c = (char)cns[i];
        codes[i] = c == 'A' ? 0 : c == 'C' ? 1 : c == 'G' ? 2 : 3;
    }
    put(im->cns, codes.data(), ncns);
    put(im->msacols, msa, (uint64_t)ncols * (g->nseq + 4));
    std::vector<uint32_t> idx(ncols);
    for (uint32_t j = 0; j < ncols; ++j) idx[j] = j;
    put(im->msaidxs, idx.data(), ncols);
}

void tidy_msa_bspoa(BSPOA *g) { (void)g; }

void free_bspoa(BSPOA *g)
{
    if (!g) return;
    auto *im = static_cast<Impl *>(g->impl);
    ccsx_gpu_close(im->ctx);
    free(im->cns.buffer);
    free(im->msacols.buffer);
    free(im->msaidxs.buffer);
    delete im;
    free(g);
}

}  // extern "C"
