// ingest_bench.cpp -- CPU-only timing of the host program's step 0 + the CPU
// half of step 1 (no GPU): read and group ZMWs into chunks as ccsx does
// (host/ingest.cpp), then assemble the bases and run ccs_prepare + strand flip
// on T threads.  Prints one JSON line; with --dump, one line per ZMW
// (movie, hole, lens, crc of the prepared bases) for parity checks.
//   g++ -O2 -std=c++17 -I include -I ccsx_amd/csrc/host tools/ingest_bench.cpp \
//       -L ccsx_amd -lccsx_amd -Wl,-rpath,$PWD/ccsx_amd -o build/ingest_bench
//   build/ingest_bench IN [is_bam] [threads] [chunk] [--dump]
#include <zlib.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "ccsx_host.h"
#include "ingest.h"

int main(int argc, char **argv)
{
    if (argc < 2) return 2;
    const bool bam = argc > 2 && atoi(argv[2]);
    const int nt = argc > 3 ? atoi(argv[3]) : 16;
    const size_t chunk = argc > 4 ? (size_t)atol(argv[4]) : 16384;
    const bool dump = argc > 5 && !strcmp(argv[5], "--dump");
    using clk = std::chrono::steady_clock;
    auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    const auto t0 = clk::now();
    auto src = ccsx_ingest::ZmwSource::open(argv[1], bam, nt);
    if (!src) return 1;
    double t_read = 0, t_prep = 0;
    uint64_t nzmw = 0, bases = 0;
    for (;;) {
        const auto a = clk::now();
        std::vector<ccsx_ingest::ZmwRef> zs;
        ccsx_ingest::ZmwRef z;
        while (src->next(z) >= 0) {
            zs.push_back(std::move(z));
            if (zs.size() >= chunk) break;
        }
        const auto b = clk::now();
        t_read += ms(a, b);
        if (zs.empty()) break;
        std::vector<uint32_t> crc(zs.size());
        std::atomic<size_t> nx(0);
        auto work = [&]() {
            std::string seqs;
            std::vector<uint32_t> lens, so, sl;
            std::vector<uint8_t> rv;
            for (size_t i; (i = nx.fetch_add(1)) < zs.size();) {
                const auto &r = zs[i];
                seqs.resize(r.total());
                lens.clear();
                size_t o = 0;
                for (const auto &x : r.recs) {
                    ccsx_ingest::write_bases(x, &seqs[o]);
                    lens.push_back(x.len);
                    o += x.len;
                }
                const uint32_t n = (uint32_t)lens.size();
                so.resize(n), sl.resize(n), rv.resize(n);
                const uint32_t ns = ccsx_prepare(seqs.data(), lens.data(), n, so.data(), sl.data(), rv.data());
                uint32_t c = 0;
                for (uint32_t k = 0; k < ns; ++k) {
                    if (rv[k]) ccsx_revcomp(&seqs[so[k]], sl[k]);
                    c = (uint32_t)crc32(c, reinterpret_cast<const unsigned char *>(&seqs[so[k]]), sl[k]);
                }
                crc[i] = c;
            }
        };
        std::vector<std::thread> th;
        for (int t = 1; t < nt; ++t) th.emplace_back(work);
        work();
        for (auto &t : th) t.join();
        t_prep += ms(b, clk::now());
        for (size_t i = 0; i < zs.size(); ++i) {
            bases += zs[i].total();
            if (dump) {
                printf("%s\t%s\t", zs[i].movie.c_str(), zs[i].hole.c_str());
                for (size_t k = 0; k < zs[i].recs.size(); ++k) printf(k ? ",%u" : "%u", zs[i].recs[k].len);
                printf("\t%08x\n", crc[i]);
            }
        }
        nzmw += zs.size();
    }
    const double tot = ms(t0, clk::now());
    if (!dump)
        printf("{\"zmws\": %llu, \"bases\": %llu, \"threads\": %d, \"read_ms\": %.1f, \"prepare_ms\": %.1f, "
               "\"total_ms\": %.1f, \"zmws_per_s\": %.0f, \"gbases_per_s\": %.3f}\n",
               (unsigned long long)nzmw, (unsigned long long)bases, nt, t_read, t_prep, tot, nzmw / (tot / 1e3),
               bases / (tot / 1e3) / 1e9);
    return 0;
}
