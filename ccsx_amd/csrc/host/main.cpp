// main.cpp -- the C host program: ccsx's CLI and 3-stage pipeline on top of the
// MI355X engine.
//
// Restates main.c:723-870 (options, I/O, chunked pipeline) and step 0 / step 2
// of worker_pipeline (main.c:649-720).  Step 1 -- kt_for(ccs_for2/ccs_for) --
// becomes: ccs_prepare + strand flip on -j CPU threads, then one batched
// device call per GPU (include/ccsx_gpu.h), the chunk's ZMWs split across the
// visible GPUs in contiguous ranges and gathered back in input order.
#include <getopt.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <future>
#include <string>
#include <thread>
#include <unordered_set>
#include <vector>

#include "ccsx_gpu.h"
#include "ccsx_host.h"
#include "ccsx_seqio.h"

namespace {

struct Zmw {
    std::string movie, hole, seqs;
    std::vector<uint32_t> lens;
    std::vector<uint32_t> seg_off, seg_len;
    std::string ccs;
};

int usage()
{
    fprintf(stdout,
            "Program: ccsx\n"
            "Version: 1.0.0 (MI355X engine)\n"
            "Usage  : ccsx  [options] <INPUT> <OUTPUT>\n"
            "Generate circular consensus sequences (ccs) from subreads.\n"
            "\n"
            "Options:\n"
            "-h             Output this help \n"
            "-v             debug \n"
            "-m     <int>   Minimum total length of subreads in a hole to use for generating CCS. [5000] \n"
            "-M     <int>   Maximum total length of subreads in a hole to use for generating CCS. [500000] \n"
            "-c     <int>   Minimum number of subreads required to generate CCS. [3] \n"
            "-A             For fasta/fastq input,gzip allowed  \n"
            "-P             primitive bsalign,subread shred by default \n"
            "-X\t\t<str>   Exclude ZMWs from output file,a comma-separated list of ID \n"
            "-j     <int>   Number of CPU threads for subread preparation. [1] \n"
            "\n"
            "Environment:\n"
            "CCSX_NGPU      Number of GPUs to use [all visible]\n"
            "\n"
            "Arguments:\n"
            "input          Input file.\n"
            "output         Output file.\n"
            "\n");
    return 1;
}

// ccs_prepare + strand flip for every ZMW of the chunk on nthreads threads
// (the CPU half of step 1, main.c:520-536)
void prepare_chunk(std::vector<Zmw> &zs, int nthreads, int verbose)
{
    std::atomic<size_t> next(0);
    auto work = [&]() {
        for (size_t i; (i = next.fetch_add(1)) < zs.size();) {
            Zmw &z = zs[i];
            const uint32_t n = (uint32_t)z.lens.size();
            z.seg_off.resize(n);
            z.seg_len.resize(n);
            const uint32_t ns = ccsx_prepare_apply(&z.seqs[0], z.lens.data(), n, z.seg_off.data(), z.seg_len.data());
            z.seg_off.resize(ns);
            z.seg_len.resize(ns);
            if (verbose)
                for (uint32_t l = 0; l < ns; ++l)
                    fprintf(stderr, ">%s_%u/%u len=%u \n%.*s\n", z.hole.c_str(), l, ns, z.seg_len[l], (int)z.seg_len[l],
                            z.seqs.data() + z.seg_off[l]);
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; ++t) th.emplace_back(work);
    work();
    for (auto &t : th) t.join();
}

// the GPU half of step 1: contiguous ranges of the chunk per device
bool run_chunk(std::vector<Zmw> &zs, std::vector<ccsx_ctx *> &ctx, int mode)
{
    const size_t ng = ctx.size(), nz = zs.size();
    std::vector<std::thread> th;
    std::atomic<bool> ok(true);
    for (size_t g = 0; g < ng; ++g) {
        const size_t b = nz * g / ng, e = nz * (g + 1) / ng;
        th.emplace_back([&, g, b, e]() {
            if (b == e) return;
            std::vector<ccsx_zmw_in> in(e - b);
            std::vector<ccsx_zmw_out> out(e - b);
            for (size_t i = b; i < e; ++i)
                in[i - b] = ccsx_zmw_in{zs[i].seqs.data(), zs[i].seg_off.data(), zs[i].seg_len.data(),
                                        (uint32_t)zs[i].seg_len.size()};
            if (ccsx_gpu_run(ctx[g], mode, in.data(), in.size(), out.data()) != 0) {
                fprintf(stderr, "[ccsx] GPU %zu: %s\n", g, ccsx_gpu_error(ctx[g]));
                ok = false;
                return;
            }
            for (size_t i = b; i < e; ++i) zs[i].ccs.assign(out[i - b].ccs, out[i - b].len);
        });
    }
    for (auto &t : th) t.join();
    return ok;
}

}  // namespace

int main(int argc, char **argv)
{
    int c, verbose = 0, min_subread_len = 5000, max_subread_len = 500000, min_fulllen_count = 3, nthreads = 1;
    int isbam = 1, split_subread = 1;
    std::unordered_set<std::string> hole_set;
    bool have_holes = false;
    while ((c = getopt(argc, argv, "hm:M:c:j:X:PAv")) != -1) {
        switch (c) {
        case 'm': min_subread_len = atoi(optarg); break;
        case 'M': max_subread_len = atoi(optarg); break;
        case 'P': split_subread = 0; break;
        case 'A': isbam = 0; break;
        case 'X': {  // main.c:772-782 (ksplit on ',': empty fields skipped)
            have_holes = true;
            std::string s(optarg), f;
            for (size_t i = 0; i <= s.size(); ++i) {
                if (i == s.size() || s[i] == ',') {
                    if (!f.empty()) hole_set.insert(f);
                    f.clear();
                } else {
                    f.push_back(s[i]);
                }
            }
            break;
        }
        case 'c':
            min_fulllen_count = atoi(optarg);
            if (min_fulllen_count < 3) {
                fprintf(stderr, "Error! min fulllen count=[%d] (>=3) !\n", min_fulllen_count);
                return -1;
            }
            break;
        case 'v': verbose++; break;
        case 'j': nthreads = atoi(optarg); break;
        default: return usage();
        }
    }
    // main.c:802-826
    const char *in_path = "-";
    FILE *fp_out = nullptr;
    if (argc - optind == 0) {
        fp_out = stdout;
    } else if (argc - optind == 1) {
        in_path = argv[optind];
        fp_out = stdout;
    } else if (argc - optind == 2) {
        in_path = argv[optind];
        fp_out = strcmp(argv[optind + 1], "-") == 0 ? stdout : fopen(argv[optind + 1], "w+");
    } else {
        return usage();
    }
    ccsx_reader *rd = ccsx_reader_open(in_path, isbam);
    if (!rd) {
        fprintf(stderr, "Error: Failed to open infile!\n");
        return 1;
    }
    if (!fp_out) {
        fprintf(stderr, "Cannot open file for write!\n");
        return 1;
    }
    int ndev = ccsx_gpu_device_count();
    if (ndev <= 0) {
        fprintf(stderr, "[ccsx] no HIP device: the MI355X engine needs a GPU\n");
        return 1;
    }
    if (const char *e = getenv("CCSX_NGPU")) ndev = std::max(1, std::min(ndev, atoi(e)));
    // CCSX_SLOTS=2: two chunk slots per GPU, each with its own context and
    // stream, chunk k + 1 launched on the other slot while chunk k drains (so
    // the CUs its finished workgroups free could take chunk k + 1's work).
    // Measured slower on MI355X (the concurrent chunk's
    // staging stalls the running one), so one chunk in flight is the default;
    // with one slot, chunk k + 1 is launched before chunk k is written out.
    int nslot = 1;
    if (const char *e = getenv("CCSX_SLOTS")) nslot = std::max(1, std::min(2, atoi(e)));
    std::vector<std::vector<ccsx_ctx *>> ctx(nslot, std::vector<ccsx_ctx *>(ndev, nullptr));
    for (int s = 0; s < nslot; ++s)
        for (int g = 0; g < ndev; ++g) {
            if (ccsx_gpu_open(g, &ctx[s][g]) != 0) return 1;
            ccsx_gpu_set_mem_share(ctx[s][g], (uint32_t)nslot);
            ccsx_gpu_set_prealloc(ctx[s][g], 1);
        }
    if (nthreads < 1) nthreads = 1;

    // main.c:652-697 (step 0), 698-706 (step 1), 707-717 (step 2).  As the
    // reference's kt_pipeline overlaps step 0 of the next chunk with step 1,
    // chunk k + 1 is read and prepared on the CPU while the GPUs run chunk k;
    // chunks are written in input order.
    size_t chunk_size = 1024;
    // CCSX_TIMING=1: per-chunk wall-clock phases on stderr (ms since start)
    const bool timing = getenv("CCSX_TIMING") && atoi(getenv("CCSX_TIMING"));
    const auto tstart = std::chrono::steady_clock::now();
    auto now_ms = [tstart]() {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tstart).count();
    };
    auto read_chunk = [&](std::vector<Zmw> &zs) -> bool {
        const double t0 = now_ms();
        const char *movie, *hole, *seqs;
        const uint32_t *lens;
        int l;
        while ((l = ccsx_reader_next(rd, &movie, &hole, &seqs, &lens)) >= 0) {
            if (l < min_fulllen_count + 2) continue;
            size_t total = 0;
            for (int i = 0; i < l; ++i) total += lens[i];
            if (total > (size_t)max_subread_len || total < (size_t)min_subread_len) continue;
            if (have_holes && hole_set.count(hole)) continue;
            Zmw z;
            z.movie = movie, z.hole = hole;
            z.seqs.assign(seqs, total);
            z.lens.assign(lens, lens + l);
            zs.push_back(std::move(z));
            if (zs.size() >= chunk_size) {
                if (chunk_size < 16384) chunk_size *= 4;
                break;
            }
        }
        // kt_pipeline stops on an empty chunk (main.c:694-697); a chunk cut
        // short by -1 (end of input or an invalid name) is processed and the
        // next call reads on, as the reference's next step 0 does
        if (zs.empty()) return false;
        const double t1 = now_ms();
        prepare_chunk(zs, nthreads, verbose);
        if (timing)
            fprintf(stderr, "[ccsx] chunk %zu ZMWs: read %.0f-%.0f ms, prepare until %.0f ms\n", zs.size(), t0, t1,
                    now_ms());
        return true;
    };
    int rc = 0;
    const int mode = split_subread ? CCSX_MODE_SHRED : CCSX_MODE_PRIMITIVE;
    std::vector<Zmw> buf[2];
    std::future<bool> run[2];
    auto start = [&](int s) {
        if (verbose > 1)
            for (auto &z : buf[s]) fprintf(stderr, "poa begin %s\n", z.hole.c_str());
        run[s] = std::async(std::launch::async, [&, s]() {
            const double t0 = now_ms();
            const bool ok = run_chunk(buf[s], ctx[s % nslot], mode);
            if (timing) fprintf(stderr, "[ccsx] chunk %zu ZMWs: GPU %.0f-%.0f ms\n", buf[s].size(), t0, now_ms());
            return ok;
        });
    };
    bool have = read_chunk(buf[0]);
    if (have) start(0);
    for (int s = 0; have; s ^= 1) {
        // step 0 of chunk k + 1 overlaps chunk k on the GPUs; with two slots
        // its launch does too
        const int o = s ^ 1;
        std::vector<Zmw>().swap(buf[o]);
        bool next = false;
        if (nslot == 2) {
            next = read_chunk(buf[o]);
            if (next) start(o);
        } else {
            std::future<bool> ahead = std::async(std::launch::async, [&]() { return read_chunk(buf[o]); });
            const bool ok = run[s].get();
            next = ahead.get();
            if (next && ok) start(o);
            run[s] = std::async(std::launch::deferred, [ok]() { return ok; });
        }
        const bool ok = run[s].get();
        if (ok) {
            for (auto &z : buf[s]) {
                if (verbose > 1) fprintf(stderr, "poa end %s\n", z.hole.c_str());
                if (!z.ccs.empty()) fprintf(fp_out, ">%s/%s/ccs\n%s\n", z.movie.c_str(), z.hole.c_str(), z.ccs.c_str());
            }
        }
        if (!ok) {
            if (next && run[o].valid()) run[o].get();
            rc = 1;
            break;
        }
        have = next;
    }
    for (auto &v : ctx)
        for (auto *x : v) ccsx_gpu_close(x);
    ccsx_reader_close(rd);
    if (fp_out != stdout) fclose(fp_out);
    else fflush(stdout);
    return rc;
}
