// seqio.cpp -- C-ABI subread reader (include/ccsx_seqio.h) on the block-based
// ingest of host/ingest.cpp: kseq_zmw_read (seqio.h:152-201) over FASTA/FASTQ
// records (kseq.h:178-218) or BAM records (bamlite.c:78-165, seqio.h:92-118),
// with the ZMW's bases assembled into one string per call.
#include "ccsx_seqio.h"

#include <cstdlib>
#include <string>
#include <vector>

#include "ingest.h"

struct ccsx_reader {
    std::unique_ptr<ccsx_ingest::ZmwSource> src;
    ccsx_ingest::ZmwRef z;
    std::string seqs;
    std::vector<uint32_t> lens;
};

extern "C" {

ccsx_reader *ccsx_reader_open(const char *path, int is_bam)
{
    int nt = 4;
    if (const char *e = getenv("CCSX_INGEST_THREADS")) nt = atoi(e) > 0 ? atoi(e) : 1;
    auto src = ccsx_ingest::ZmwSource::open(path, is_bam != 0, nt);
    if (!src) return nullptr;
    auto *r = new ccsx_reader();
    r->src = std::move(src);
    return r;
}

int ccsx_reader_next(ccsx_reader *r, const char **movie, const char **hole, const char **seqs, const uint32_t **lens)
{
    const int l = r->src->next(r->z);
    r->seqs.clear();
    r->lens.clear();
    if (l > 0) {
        for (const auto &x : r->z.recs) {
            ccsx_ingest::append_bases(x, r->seqs);
            r->lens.push_back(x.len);
        }
    }
    *movie = r->z.movie.c_str(), *hole = r->z.hole.c_str(), *seqs = r->seqs.data(), *lens = r->lens.data();
    return l;
}

void ccsx_reader_close(ccsx_reader *r) { delete r; }

}  // extern "C"
