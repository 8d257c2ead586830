// ingest.h -- block-based subread ingest of the C host program (internal C++
// API; the C-ABI wrapper is include/ccsx_seqio.h, seqio.cpp).
//
// Step 0 of the reference's pipeline (main.c:652-697) reads one character at a
// time through kseq's 16 KB buffer (kseq.h:178-218) or gzread per BAM record
// (bamlite.c:135-165) on one thread, serialised across chunks
// (kthread.c:199-213).  Here:
//  * a producer thread fills large blocks of decompressed input: read() for
//    plain files, parallel raw inflate of BGZF members (BAM / bgzip FASTA),
//    gzread for other gzip streams and stdin;
//  * the consumer parses records with memchr-driven scans that keep kseq's
//    exact semantics (header search, name token, comment, per-line '\r'
//    rule, '+' quality lines) and bamlite's BAM layout, without copying any
//    sequence: a record is a span of its block;
//  * ZMW grouping (kseq_zmw_read, seqio.h:152-201) runs on the spans;
//  * the bases are assembled (line joins, nt16 decode) by whoever consumes
//    the ZMW, in parallel (the CLI's prepare threads).
#pragma once
#include <stdint.h>

#include <memory>
#include <string>
#include <vector>

namespace ccsx_ingest {

struct Block;  // one decompressed input block, shared by the records in it

// one subread as a span of its block
struct Rec {
    const char *seq = nullptr;  // first byte of the sequence region
    uint64_t span = 0;          // bytes of the region
    uint32_t len = 0;           // bases (after kseq's line rules / BAM l_qseq)
    uint8_t kind = 0;           // kAscii1, kAsciiLines or kNt16
};
enum : uint8_t { kAscii1 = 0, kAsciiLines = 1, kNt16 = 2 };

// the bases of r appended to out (exactly what kseq / bamlite would hold)
void append_bases(const Rec &r, std::string &out);
// ... written to dst (r.len bytes)
void write_bases(const Rec &r, char *dst);

struct ZmwRef {
    std::string movie, hole;
    std::vector<Rec> recs;
    std::vector<std::shared_ptr<Block>> keep;  // blocks the records point into
    uint64_t total() const
    {
        uint64_t t = 0;
        for (const Rec &r : recs) t += r.len;
        return t;
    }
};

class ZmwSource {
public:
    // path "-" = stdin; nthreads: inflate workers for BGZF input
    static std::unique_ptr<ZmwSource> open(const char *path, bool is_bam, int nthreads);
    virtual ~ZmwSource() = default;
    // kseq_zmw_read (seqio.h:152-201): the next ZMW's subreads (returns their
    // count), or -1 at the end of input or after an invalid record name
    // ("invalid zmw name :<name>" on stderr; the next call reads on)
    virtual int next(ZmwRef &z) = 0;
    // the caller reads no record byte below `upto` any more (records of
    // earlier ZMWs): a mapped input may unmap those pages
    virtual void release(const char *upto) { (void)upto; }
};

}  // namespace ccsx_ingest
