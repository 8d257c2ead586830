// host_sanitize.cpp -- drives the host C++ of the product (ingest, seqio C-ABI,
// ccs_prepare, the pairwise aligner, the synthetic source, the dispatch
// partitioner) under AddressSanitizer + UndefinedBehaviorSanitizer on the CPU.
// tests/test_sanitize.py compiles it together with those sources
// (-fsanitize=address,undefined; no HIP code is involved) and runs it on the
// golden ingest fixtures and synthetic ZMWs.
//   host_sanitize FIXTURE:is_bam ...   prints one line per ZMW read
#include <zlib.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "ccsx_host.h"
#include "ccsx_seqio.h"

static uint32_t crc(const char *p, size_t n) { return (uint32_t)crc32(0, reinterpret_cast<const unsigned char *>(p), (uInt)n); }

int main(int argc, char **argv)
{
    // 1. ingest: every fixture at several block sizes (records crossing blocks)
    for (int a = 1; a < argc; ++a) {
        std::string arg(argv[a]);
        const size_t c = arg.rfind(':');
        const std::string path = arg.substr(0, c);
        const int bam = atoi(arg.c_str() + c + 1);
        for (const char *blk : {"1", "5", "64", ""}) {
            if (*blk) setenv("CCSX_INGEST_BLOCK", blk, 1);
            else unsetenv("CCSX_INGEST_BLOCK");
            ccsx_reader *r = ccsx_reader_open(path.c_str(), bam);
            if (!r) return 3;
            const char *movie, *hole, *seqs;
            const uint32_t *lens;
            // main.c step 0: a chunk ends at -1, the next one reads on, and
            // the input ends at the first chunk without a ZMW
            int l, got = 1;
            while (got) {
                got = 0;
                while ((l = ccsx_reader_next(r, &movie, &hole, &seqs, &lens)) >= 0) {
                    ++got;
                    size_t tot = 0;
                    for (int k = 0; k < l; ++k) tot += lens[k];
                    if (*blk == 0) printf("%s %s/%s %d %zu %08x\n", path.c_str(), movie, hole, l, tot, crc(seqs, tot));
                    // prepare + strand flip on what was read
                    std::string s(seqs, tot);
                    std::vector<uint32_t> off(l), len(l);
                    const uint32_t ns = ccsx_prepare_apply(&s[0], lens, (uint32_t)l, off.data(), len.data());
                    for (uint32_t k = 0; k < ns; ++k)
                        if (off[k] + (uint64_t)len[k] > tot) return 4;
                }
                if (*blk == 0) printf("%s -1\n", path.c_str());
            }
            ccsx_reader_close(r);
        }
    }
    // 2. ccs_prepare on synthetic ZMWs with abnormal subreads (random
    // truncations, adapters read through, short and empty subreads)
    std::mt19937_64 rng(7);
    for (int z = 0; z < 60; ++z) {
        const uint32_t L = 300 + (uint32_t)(rng() % 3000), passes = 3 + (uint32_t)(rng() % 9);
        std::string out((size_t)passes * (2 * L + 16) + 16, '\0');
        std::vector<uint32_t> lens(passes);
        ccsx_synth_zmw(20201104, (uint64_t)z, L, passes, &out[0], lens.data(), nullptr);
        std::string seqs;
        size_t o = 0;
        std::vector<uint32_t> l2;
        for (uint32_t k = 0; k < passes; ++k) {
            std::string sub = out.substr(o, lens[k]);
            o += lens[k];
            switch (rng() % 6) {
            case 0: sub = sub.substr(0, sub.size() / 3); break;                         // truncated
            case 1: { std::string rc = sub; ccsx_revcomp(&rc[0], (uint32_t)rc.size()); sub += rc; break; }  // palindrome
            case 2: sub.clear(); break;                                                   // empty
            default: break;
            }
            seqs += sub;
            l2.push_back((uint32_t)sub.size());
        }
        std::vector<uint32_t> off(passes), len(passes);
        std::vector<uint8_t> rev(passes);
        const uint32_t ns = ccsx_prepare(seqs.data(), l2.data(), passes, off.data(), len.data(), rev.data());
        for (uint32_t k = 0; k < ns; ++k)
            if (off[k] + (uint64_t)len[k] > seqs.size()) return 5;
        printf("prepare %d %u\n", z, ns);
    }
    // 3. the pairwise aligner on random 2-bit sequences (codes >= 4 included)
    for (int t = 0; t < 40; ++t) {
        std::vector<uint8_t> q(rng() % 3000), s(rng() % 3000);
        for (auto &x : q) x = (uint8_t)(rng() % 5);
        for (auto &x : s) x = (uint8_t)(rng() % 5);
        const ccsx_pairaln r = ccsx_pairwise(q.data(), (uint32_t)q.size(), s.data(), (uint32_t)s.size());
        if (r.qe < r.qb || r.te < r.tb) return 6;
    }
    // 4. the dispatch partitioner
    for (int t = 0; t < 50; ++t) {
        const uint32_t n = (uint32_t)(rng() % 5000);
        std::vector<uint64_t> cost(n);
        for (auto &x : cost) x = rng() % 1000000;
        std::vector<uint32_t> order(n ? n : 1), bounds(n + 1);
        const uint32_t nb = ccsx_partition(cost.data(), n, 1 + (uint32_t)(rng() % 40), 1 + (uint32_t)(rng() % 300),
                                           order.data(), bounds.data());
        if (nb > n || bounds[nb] != n) return 7;
    }
    printf("ok\n");
    return 0;
}
