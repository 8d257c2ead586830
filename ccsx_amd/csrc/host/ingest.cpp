// ingest.cpp -- block-based subread ingest (host/ingest.h).
//
// Record semantics follow the reference exactly:
//  * FASTA/FASTQ: kseq_read, kseq.h:178-218 (header search anywhere, name =
//    token up to whitespace, comment line, sequence lines until a line
//    starting with '>', '+' or '@', one trailing '\r' stripped per appended
//    line when the string is longer than 1, quality lines until at least as
//    long as the sequence -- at least one line is read);
//  * BAM: bam_header_read / bam_read1, bamlite.c:78-165, decoded with
//    seq_nt16_str as kseq_extend_read does (seqio.h:92-118);
//  * grouping: kseq_zmw_read, seqio.h:152-201.
// tests/golden/host pins all three against the reference's own seqio.h.
#include "ingest.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>

namespace ccsx_ingest {

struct Block {
    std::unique_ptr<char[]> mem;
    size_t cap = 0;
    char *data = nullptr;  // first valid byte (mem + headroom - carried tail)
    size_t len = 0;        // valid bytes
    bool eof = false;      // nothing follows this block
    void *map = nullptr;   // a whole-file mapping instead of mem (MmapSource)
    size_t map_len = 0;
    ~Block()
    {
        if (map) munmap(map, map_len);
    }
    // `head` bytes of headroom in front of the payload for the carried tail
    // of the previous block
    static std::shared_ptr<Block> make(size_t payload, size_t head)
    {
        auto b = std::make_shared<Block>();
        b->cap = head + payload;
        b->mem.reset(new char[b->cap]);
        b->data = b->mem.get() + head;
        return b;
    }
};

namespace {

// ---------------------------------------------------------------- byte sources
struct ByteSource {
    // decompressed bytes per block (CCSX_INGEST_BLOCK overrides it per
    // source: the tests use a few bytes so every record crosses blocks)
    size_t block = 32u << 20;
    size_t head() const { return std::min<size_t>(2u << 20, 4 * block); }
    virtual ~ByteSource() = default;
    // next block of decompressed bytes (len may be 0 only with eof)
    virtual std::shared_ptr<Block> next() = 0;
};

// plain file or pipe: read(2) straight into the block
struct FdSource : ByteSource {
    int fd;
    bool done = false;
    explicit FdSource(int f) : fd(f) {}
    ~FdSource() override
    {
        if (fd > 2) close(fd);
    }
    std::shared_ptr<Block> next() override
    {
        auto b = Block::make(block, head());
        while (!done && b->len < block) {
            const ssize_t r = read(fd, b->data + b->len, block - b->len);
            if (r <= 0) done = true;
            else b->len += (size_t)r;
        }
        b->eof = done;
        return b;
    }
};

// a regular uncompressed file: one block that maps the whole file (no copy,
// no carried tails); a toucher thread faults the pages in ahead of the parser
struct MmapSource : ByteSource {
    std::shared_ptr<Block> b;
    std::thread toucher;
    std::atomic<bool> stop{false};
    std::atomic<size_t> touched{0};  // the toucher is past this offset
    std::mutex rel_m;
    size_t released = 0;  // [0, released) unmapped
    // the caller reads no byte below `upto` any more: unmap those pages (the
    // teardown of a 65 GB mapping otherwise falls on the process exit), never
    // above what the toucher has passed
    void release(const char *upto)
    {
        std::lock_guard<std::mutex> g(rel_m);
        if (!b->map || !upto) return;
        const char *base = static_cast<const char *>(b->map);
        if (upto <= base) return;
        size_t hi = std::min<size_t>((size_t)(upto - base), touched.load());
        hi &= ~size_t(4095);
        if (hi > released) {
            munmap(const_cast<char *>(base) + released, hi - released);
            released = hi;
        }
    }
    MmapSource(int fd, size_t size)
    {
        b = std::make_shared<Block>();
        void *m = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
        close(fd);
        if (m == MAP_FAILED) {
            b->eof = true;  // read as empty
            return;
        }
        madvise(m, size, MADV_WILLNEED);
        b->map = m, b->map_len = size;
        b->data = static_cast<char *>(m), b->len = size, b->eof = true;
        toucher = std::thread([this, m, size] {
            volatile const char *p = static_cast<const char *>(m);
            char sink = 0;
            for (size_t o = 0; o < size && !stop; o += 4096) {
                sink ^= p[o];
                if ((o & ((2u << 20) - 1)) == 0) touched.store(o);
            }
            touched.store(size);
            (void)sink;
        });
    }
    ~MmapSource() override
    {
        stop = true;
        if (toucher.joinable()) toucher.join();
        // the block may outlive the source (a parser still holds it): leave
        // it only the part still mapped, so its destructor never unmaps the
        // released prefix, where unrelated mappings may live by now
        std::lock_guard<std::mutex> g(rel_m);
        if (b->map && released) {
            if (released >= b->map_len) {
                b->map = nullptr, b->map_len = 0;
            } else {
                b->map = static_cast<char *>(b->map) + released;
                b->map_len -= released;
            }
        }
    }
    std::shared_ptr<Block> next() override { return b; }
};

// gzip (non-BGZF) or stdin: zlib's gzread (transparent for plain data)
struct GzSource : ByteSource {
    gzFile fp;
    bool done = false;
    explicit GzSource(gzFile f) : fp(f) { gzbuffer(fp, 1u << 20); }
    ~GzSource() override { gzclose(fp); }
    std::shared_ptr<Block> next() override
    {
        auto b = Block::make(block, head());
        while (!done && b->len < block) {
            const int r = gzread(fp, b->data + b->len, (unsigned)std::min<size_t>(block - b->len, 1u << 30));
            if (r <= 0) done = true;
            else b->len += (size_t)r;
        }
        b->eof = done;
        return b;
    }
};

// BGZF (SAM spec 4.1): gzip members of <= 64 KiB, each with its compressed
// size in the BC extra field and its inflated size in the trailer, so a run
// of members inflates in parallel straight to known offsets of the block
struct BgzfSource : ByteSource {
    int fd;
    int nthreads;
    std::vector<unsigned char> in;  // compressed bytes not yet consumed
    size_t ipos = 0;
    bool in_eof = false, done = false, bad = false;
    BgzfSource(int f, int nt) : fd(f), nthreads(std::max(1, nt)) {}
    ~BgzfSource() override
    {
        if (fd > 2) close(fd);
    }
    // at least `need` bytes from ipos on (appends only: the members of the
    // block being built keep their offsets)
    bool fill(size_t need)
    {
        if (in.size() - ipos >= need) return true;
        need += ipos;
        while (!in_eof && in.size() < need) {
            const size_t old = in.size(), want = std::max<size_t>(need - old, 16u << 20);
            in.resize(old + want);
            const ssize_t r = read(fd, in.data() + old, want);
            in.resize(old + (r > 0 ? (size_t)r : 0));
            if (r <= 0) in_eof = true;
        }
        return in.size() >= need;
    }
    // size of the member at ipos (0 = end, not BGZF, or a header that does
    // not describe a whole member: every subfield inside XLEN, BSIZE + 1 at
    // least the header and the 8-byte trailer)
    size_t member_size()
    {
        if (!fill(18)) return 0;
        const unsigned char *h = in.data() + ipos;
        if (h[0] != 31 || h[1] != 139 || h[2] != 8 || !(h[3] & 4)) return 0;
        const size_t xlen = h[10] | (size_t)h[11] << 8;
        if (!fill(12 + xlen)) return 0;
        h = in.data() + ipos;
        for (size_t x = 12; x + 4 <= 12 + xlen;) {
            const size_t sl = h[x + 2] | (size_t)h[x + 3] << 8;
            if (x + 4 + sl > 12 + xlen) return 0;
            if (h[x] == 66 && h[x + 1] == 67 && sl == 2) {
                const size_t sz = (h[x + 4] | (size_t)h[x + 5] << 8) + 1;
                return sz >= 12 + xlen + 8 ? sz : 0;
            }
            x += 4 + sl;
        }
        return 0;
    }
    std::shared_ptr<Block> next() override
    {
        struct M {
            size_t off, size, out, isize;
        };
        std::vector<M> ms;
        size_t total = 0;
        if (ipos) {  // drop the members of the previous block
            in.erase(in.begin(), in.begin() + (ptrdiff_t)ipos);
            ipos = 0;
        }
        while (!done && total < block) {
            const size_t sz = member_size();
            if (!sz || !fill(sz)) {
                // end of input (a partial or foreign member ends it, as a
                // truncated stream ends gzread)
                if (!(in_eof && in.size() == ipos)) bad = true;
                done = true;
                break;
            }
            const unsigned char *t = in.data() + ipos + sz - 4;
            const size_t isize = t[0] | (size_t)t[1] << 8 | (size_t)t[2] << 16 | (size_t)t[3] << 24;
            if (isize > 65536) {  // a BGZF member inflates to at most 64 KiB
                bad = done = true;
                break;
            }
            ms.push_back({ipos, sz, total, isize});
            total += isize;
            ipos += sz;
            if (ipos > (64u << 20)) break;  // keep the compressed window bounded
        }
        auto b = Block::make(std::max<size_t>(total, 1), head());
        b->len = total;
        std::atomic<size_t> nx(0);
        std::atomic<bool> err(false);
        auto work = [&]() {
            z_stream s;
            memset(&s, 0, sizeof s);
            if (inflateInit2(&s, -15) != Z_OK) {
                err = true;
                return;
            }
            for (size_t i; (i = nx.fetch_add(1)) < ms.size();) {
                const M &m = ms[i];
                const unsigned char *h = in.data() + m.off;
                const size_t xlen = h[10] | (size_t)h[11] << 8;
                inflateReset(&s);
                s.next_in = const_cast<unsigned char *>(h + 12 + xlen);
                s.avail_in = (unsigned)(m.size - 12 - xlen - 8);
                s.next_out = reinterpret_cast<unsigned char *>(b->data + m.out);
                s.avail_out = (unsigned)m.isize;
                const int rc = inflate(&s, Z_FINISH);
                const unsigned char *t = h + m.size - 8;
                const uint32_t crc = t[0] | (uint32_t)t[1] << 8 | (uint32_t)t[2] << 16 | (uint32_t)t[3] << 24;
                if (rc != Z_STREAM_END || s.avail_out ||
                    crc32(0, reinterpret_cast<const unsigned char *>(b->data + m.out), (unsigned)m.isize) != crc)
                    err = true;
            }
            inflateEnd(&s);
        };
        const int nt = (int)std::min<size_t>((size_t)nthreads, ms.size());
        std::vector<std::thread> th;
        for (int t = 1; t < nt; ++t) th.emplace_back(work);
        work();
        for (auto &t : th) t.join();
        if (err) {
            // a corrupt member: gzread would stop with an error; keep the
            // bytes before this block and end the input
            b->len = 0;
            bad = done = true;
        }
        if (bad) fprintf(stderr, "[ccsx] BGZF input truncated or corrupt; reading stops here\n");
        b->eof = done;
        return b;
    }
};

// the producer thread: keeps up to two blocks decompressed ahead
class Prefetch {
public:
    explicit Prefetch(std::unique_ptr<ByteSource> s) : src_(std::move(s))
    {
        th_ = std::thread([this] {
            for (;;) {
                {
                    std::unique_lock<std::mutex> g(m_);
                    cv_.wait(g, [this] { return stop_ || q_.size() < 2; });
                    if (stop_) return;
                }
                auto b = src_->next();
                const bool eof = b->eof;
                {
                    std::lock_guard<std::mutex> g(m_);
                    q_.push_back(std::move(b));
                }
                cv_.notify_all();
                if (eof) return;
            }
        });
    }
    ~Prefetch()
    {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        th_.join();
    }
    std::shared_ptr<Block> pop()
    {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [this] { return !q_.empty(); });
        auto b = std::move(q_.front());
        q_.pop_front();
        cv_.notify_all();
        return b;
    }

private:
    std::unique_ptr<ByteSource> src_;
    std::thread th_;
    std::mutex m_;
    std::condition_variable cv_;
    std::deque<std::shared_ptr<Block>> q_;
    bool stop_ = false;
};

// ---------------------------------------------------------------- byte cursor
// The consumer's view: the current block from `pos`; more() appends the next
// block behind the unconsumed bytes from `keep_from` on (copied into the next
// block's headroom when it fits)
class Cursor {
public:
    explicit Cursor(std::unique_ptr<ByteSource> s) : pf_(std::move(s)) { cur_ = pf_.pop(); }
    const char *data() const { return cur_->data; }
    size_t size() const { return cur_->len; }
    bool eof() const { return cur_->eof; }
    const std::shared_ptr<Block> &block() const { return cur_; }
    size_t pos = 0;
    // bring more input behind data()[keep_from ..]; positions are rebased so
    // keep_from becomes 0.  Returns false at the end of input.
    bool more(size_t keep_from)
    {
        if (cur_->eof) return false;
        auto nb = pf_.pop();
        const size_t tail = cur_->len - keep_from;
        if (tail <= (size_t)(nb->data - nb->mem.get())) {
            nb->data -= tail;
            memcpy(nb->data, cur_->data + keep_from, tail);
            nb->len += tail;
        } else {
            auto big = Block::make(tail + nb->len, nb->mem ? (size_t)(nb->data - nb->mem.get()) : 0);
            memcpy(big->data, cur_->data + keep_from, tail);
            memcpy(big->data + tail, nb->data, nb->len);
            big->len = tail + nb->len;
            big->eof = nb->eof;
            nb = std::move(big);
        }
        pos -= keep_from;
        cur_ = std::move(nb);
        return true;
    }

private:
    Prefetch pf_;
    std::shared_ptr<Block> cur_;
};

constexpr int kNeed = -100;

// kseq's sequence lines over [b, b + n) as one region ends them (a line
// starting with '>', '+' or '@', or the end): appends the bases to out when
// STORE, returns their number
template <bool STORE>
uint32_t seq_lines(const char *b, size_t n, std::string *out)
{
    uint64_t len = 0;
    char last = 0;
    size_t q = 0;
    while (q < n) {
        const char ch = b[q];
        if (ch == '>' || ch == '+' || ch == '@') break;
        ++q;
        if (ch == '\n') continue;
        const char *nl = static_cast<const char *>(memchr(b + q, '\n', n - q));
        const size_t le = nl ? (size_t)(nl - b) : n;
        const size_t L = le - (q - 1);
        const char prev = last;
        if (STORE) out->append(b + q - 1, L);
        len += L;
        last = b[le - 1];
        // (kseq strips a line's '\r' in ks_getuntil2, which returns before
        // the strip when the line's first char was the input's last byte)
        if (len > 1 && last == '\r' && (L > 1 || nl)) {
            --len;
            last = L >= 2 ? b[le - 2] : prev;
            if (STORE) out->pop_back();
        }
        q = nl ? le + 1 : n;
    }
    return (uint32_t)len;
}

}  // namespace

void append_bases(const Rec &r, std::string &out)
{
    if (r.kind == kAscii1) {
        out.append(r.seq, r.len);
    } else if (r.kind == kAsciiLines) {
        seq_lines<true>(r.seq, r.span, &out);
    } else {
        const size_t o = out.size();
        out.resize(o + r.len);
        write_bases(r, &out[o]);
    }
}

void write_bases(const Rec &r, char *dst)
{
    static const char nt16[] = "=ACMGRSVTWYHKDBN";
    if (r.kind == kAscii1) {
        memcpy(dst, r.seq, r.len);
    } else if (r.kind == kAsciiLines) {
        std::string s;
        s.reserve(r.len);
        seq_lines<true>(r.seq, r.span, &s);
        memcpy(dst, s.data(), r.len);
    } else {
        const unsigned char *s = reinterpret_cast<const unsigned char *>(r.seq);
        for (uint32_t i = 0; i + 1 < r.len; i += 2) {
            dst[i] = nt16[s[i >> 1] >> 4];
            dst[i + 1] = nt16[s[i >> 1] & 15];
        }
        if (r.len & 1) dst[r.len - 1] = nt16[s[r.len >> 1] >> 4];
    }
}

namespace {

// ---------------------------------------------------------------- records
class RecordReader {
public:
    virtual ~RecordReader() = default;
    // >= 0: a record (name, r, its block in keep); < 0: end (kseq / bam_read1
    // error values; every negative value ends the input, seqio.h:170)
    virtual int next(std::string &name, Rec &r, std::shared_ptr<Block> &keep) = 0;
};

// kseq_read (kseq.h:178-218) on the cursor
class FxReader : public RecordReader {
public:
    explicit FxReader(std::unique_ptr<ByteSource> s) : c_(std::move(s)) {}
    int next(std::string &name, Rec &r, std::shared_ptr<Block> &keep) override
    {
        for (;;) {
            const int l = parse(name, r);
            if (l != kNeed) {
                if (l >= 0) keep = c_.block();
                return l;
            }
            // the record continues beyond the block: keep it from its last
            // committed position (its header char) and retry on more input
            if (!c_.more(c_.pos)) eof_ = true;  // (not reached: the last block is parsed as eof)
        }
    }

private:
    Cursor c_;
    bool at_header_ = false;  // c_.pos is at a header char kseq holds as last_char
    bool eof_ = false;
    std::string qual_;

    int parse(std::string &name, Rec &r)
    {
        const char *b = c_.data();
        const size_t n = c_.size();
        const bool eof = c_.eof() || eof_;
        size_t q = c_.pos;
        if (!at_header_) {
            // jump to the next '>' or '@' anywhere
            while (q < n && b[q] != '>' && b[q] != '@') {
                const void *g = memchr(b + q, '>', n - q), *a = memchr(b + q, '@', n - q);
                const char *h = !g ? static_cast<const char *>(a)
                              : !a ? static_cast<const char *>(g)
                                   : std::min(static_cast<const char *>(g), static_cast<const char *>(a));
                q = h ? (size_t)(h - b) : n;
            }
            if (q >= n) {
                c_.pos = n;  // skipped bytes are dropped, as kseq drops them
                return eof ? -1 : kNeed;
            }
            c_.pos = q;
            at_header_ = true;
        }
        const size_t s = q + 1;
        size_t e = s;
        while (e < n && !isspace((unsigned char)b[e])) ++e;
        if (e >= n) {
            if (!eof) return kNeed;
            if (e == s) return -1;  // EOF right after the header char
            // name up to EOF: no comment, no sequence (kseq returns 0)
            name.assign(b + s, e - s);
            r = Rec{b + n, 0, 0, kAscii1};
            c_.pos = n;
            at_header_ = false;
            return 0;
        }
        name.assign(b + s, e - s);
        q = e + 1;
        if (b[e] != '\n') {
            const char *nl = static_cast<const char *>(memchr(b + q, '\n', n - q));
            if (!nl && !eof) return kNeed;
            q = nl ? (size_t)(nl - b) + 1 : n;
        }
        // sequence lines
        const size_t s0 = q;
        uint64_t len = 0;
        char last = 0;
        int nlines = 0;
        size_t ls = 0, ll = 0;  // the single content line
        int term = -1;
        for (;;) {
            if (q >= n) {
                if (!eof) return kNeed;
                break;
            }
            const char ch = b[q];
            if (ch == '>' || ch == '+' || ch == '@') {
                term = ch;
                break;
            }
            ++q;
            if (ch == '\n') continue;
            const char *nl = static_cast<const char *>(memchr(b + q, '\n', n - q));
            if (!nl && !eof) return kNeed;
            const size_t le = nl ? (size_t)(nl - b) : n;
            const size_t L = le - (q - 1);
            const char prev = last;
            len += L;
            last = b[le - 1];
            if (len > 1 && last == '\r' && (L > 1 || nl)) --len, last = L >= 2 ? b[le - 2] : prev;
            if (++nlines == 1) ls = q - 1, ll = L;
            q = nl ? le + 1 : n;
        }
        if (nlines == 1 && (len == ll || len + 1 == ll)) r = Rec{b + ls, ll, (uint32_t)len, kAscii1};
        else r = Rec{b + s0, q - s0, (uint32_t)len, kAsciiLines};
        if (term == '>' || term == '@') {
            c_.pos = q;  // the next header char (kseq's last_char)
            return (int)len;
        }
        if (term != '+') {
            c_.pos = n;
            at_header_ = false;
            return (int)len;
        }
        // FASTQ: skip the '+' line, then quality lines
        ++q;
        const char *nl = static_cast<const char *>(memchr(b + q, '\n', n - q));
        if (!nl) {
            if (!eof) return kNeed;
            c_.pos = n;
            at_header_ = false;
            return -2;
        }
        q = (size_t)(nl - b) + 1;
        qual_.clear();
        for (;;) {
            // ks_getuntil2(LINE, append): -1 only with no byte left
            if (q >= n) {
                if (!eof) return kNeed;
                break;
            }
            const char *ql = static_cast<const char *>(memchr(b + q, '\n', n - q));
            if (!ql && !eof) return kNeed;
            const size_t le = ql ? (size_t)(ql - b) : n;
            qual_.append(b + q, le - q);
            if (qual_.size() > 1 && qual_.back() == '\r') qual_.pop_back();
            q = ql ? le + 1 : n;
            if (qual_.size() >= len) break;
        }
        c_.pos = q;
        at_header_ = false;
        return qual_.size() == len ? (int)len : -2;
    }
};

// bam_header_read + bam_read1 (bamlite.c:78-165) on the cursor
class BamReader : public RecordReader {
public:
    explicit BamReader(std::unique_ptr<ByteSource> s) : c_(std::move(s)) {}
    int next(std::string &name, Rec &r, std::shared_ptr<Block> &keep) override
    {
        if (!header_done_) {
            header_done_ = true;
            if (!header()) {
                fprintf(stderr, "[bam_header_read] invalid BAM header.\n");
                dead_ = true;  // seqio.h:27-31 prints and carries on; nothing can be read
            }
        }
        if (dead_) return -1;
        uint32_t x[8];
        int32_t block_len;
        if (!get(&block_len, 4)) return -1;
        if (block_len < 32) return -3;
        if (!avail((size_t)block_len)) return -4;
        const char *p = c_.data() + c_.pos;
        memcpy(x, p, 32);
        const uint32_t l_qname = x[2] & 0xff, n_cigar = x[3] & 0xffff;
        const int32_t l_qseq = (int32_t)x[4];
        const char *data = p + 32;
        const size_t data_len = (size_t)block_len - 32;
        if (l_qseq < 0 || (size_t)l_qname + n_cigar * 4 + (size_t)(l_qseq + 1) / 2 > data_len) return -4;
        name.assign(data, strnlen(data, l_qname));
        r = Rec{data + l_qname + n_cigar * 4, (uint64_t)(l_qseq + 1) / 2, (uint32_t)l_qseq, kNt16};
        keep = c_.block();
        c_.pos += (size_t)block_len;
        return l_qseq;
    }

private:
    Cursor c_;
    bool header_done_ = false, dead_ = false;
    // n bytes available at pos (fetching more input as needed)
    bool avail(size_t n)
    {
        while (c_.size() - c_.pos < n)
            if (!c_.more(c_.pos)) return false;
        return true;
    }
    bool get(void *dst, size_t n)
    {
        if (!avail(n)) return false;
        memcpy(dst, c_.data() + c_.pos, n);
        c_.pos += n;
        return true;
    }
    bool header()
    {
        char magic[4];
        int32_t l_text, n_ref, l_name, l_ref;
        if (!get(magic, 4) || memcmp(magic, "BAM\1", 4) != 0) return false;
        if (!get(&l_text, 4) || l_text < 0 || !avail((size_t)l_text)) return false;
        c_.pos += (size_t)l_text;
        if (!get(&n_ref, 4)) return false;
        for (int32_t i = 0; i < n_ref; ++i) {
            if (!get(&l_name, 4) || l_name < 0 || !avail((size_t)l_name)) return false;
            c_.pos += (size_t)l_name;
            if (!get(&l_ref, 4)) return false;
        }
        return true;
    }
};

// ksplit(name, '/') (kstring.c:65-107): the non-empty fields; `shown` is what
// the reference prints for an invalid name (ksplit NUL-terminates the first
// field in place)
int split3(const std::string &name, std::string f[3], std::string &shown)
{
    int n = 0;
    size_t i = 0;
    const size_t L = name.size();
    bool first_end = false;
    shown.clear();
    while (i < L) {
        while (i < L && name[i] == '/') ++i;
        if (i >= L) break;
        size_t j = i;
        while (j < L && name[j] != '/') ++j;
        if (n < 3) f[n] = name.substr(i, j - i);
        if (!first_end) {
            shown = name.substr(0, j);
            first_end = true;
        }
        ++n;
        i = j;
    }
    if (!first_end) shown = name;
    return n;
}

// ---------------------------------------------------------------- grouping
class Grouper : public ZmwSource {
public:
    Grouper(std::unique_ptr<RecordReader> rr, MmapSource *mm) : rr_(std::move(rr)), mm_(mm) {}
    void release(const char *upto) override
    {
        if (mm_) mm_->release(upto);
    }
    // (a negative record value ends this call only: the reference's next
    // step 0 calls kseq_zmw_read again and reads on, e.g. after a bad FASTQ
    // record)
    int next(ZmwRef &z) override
    {
        z.recs.clear();
        z.keep.clear();
        z.movie.clear();
        z.hole.clear();
        if (have_last_) {
            z.hole = last_hole_;
            z.movie = last_movie_;
            z.recs.push_back(last_rec_);
            z.keep.push_back(last_keep_);
        }
        std::string name, f[3], shown;
        Rec r;
        std::shared_ptr<Block> keep;
        for (;;) {
            const int l = rr_->next(name, r, keep);
            if (l < 0) break;
            if (split3(name, f, shown) != 3) {
                fprintf(stderr, "invalid zmw name :%s\n", shown.c_str());
                return -1;
            }
            if (!have_last_) {
                z.movie = f[0], z.hole = f[1];
                add(z, r, keep);
                last_hole_ = z.hole, last_movie_ = z.movie, last_rec_ = r, last_keep_ = keep;
                have_last_ = true;
            } else if (last_hole_ != f[1] || z.movie != f[0]) {
                last_movie_ = f[0], last_hole_ = f[1], last_rec_ = r, last_keep_ = keep;
                return (int)z.recs.size();
            } else {
                add(z, r, keep);
            }
        }
        have_last_ = false;
        last_keep_.reset();
        return z.recs.empty() ? -1 : (int)z.recs.size();
    }

private:
    std::unique_ptr<RecordReader> rr_;
    MmapSource *mm_;  // the whole-file mapping the records point into (owned by rr_), or null
    bool have_last_ = false;
    std::string last_movie_, last_hole_;
    Rec last_rec_;
    std::shared_ptr<Block> last_keep_;
    static void add(ZmwRef &z, const Rec &r, const std::shared_ptr<Block> &k)
    {
        z.recs.push_back(r);
        if (z.keep.empty() || z.keep.back() != k) z.keep.push_back(k);
    }
};

}  // namespace

std::unique_ptr<ZmwSource> ZmwSource::open(const char *path, bool is_bam, int nthreads)
{
    const char *e = getenv("CCSX_INGEST_BLOCK");
    const size_t block = e ? (size_t)std::max<long>(1, atol(e)) : (32u << 20);
    std::unique_ptr<ByteSource> src;
    MmapSource *mm = nullptr;
    // stdin redirected from a regular file, not read yet: the file's own
    // path below (mmap, parallel BGZF, gzread), else a gzread stream
    bool stdin_stream = false;
    if (strcmp(path, "-") == 0) {
        struct stat st;
        stdin_stream = !(fstat(0, &st) == 0 && S_ISREG(st.st_mode) && lseek(0, 0, SEEK_CUR) == 0);
    }
    if (stdin_stream) {
        gzFile g = gzdopen(dup(0), "rb");
        if (!g) return nullptr;
        src.reset(new GzSource(g));
    } else {
        const int fd = strcmp(path, "-") == 0 ? dup(0) : ::open(path, O_RDONLY);
        if (fd < 0) return nullptr;
        unsigned char h[18];
        const ssize_t k = pread(fd, h, sizeof h, 0);
        const bool gz = k >= 2 && h[0] == 31 && h[1] == 139;
        bool bgzf = false;
        if (k == 18 && gz && h[2] == 8 && (h[3] & 4)) {
            const size_t xlen = h[10] | (size_t)h[11] << 8;
            bgzf = xlen >= 6 && h[12] == 66 && h[13] == 67 && h[14] == 2 && h[15] == 0;
        }
        if (bgzf) {
            src.reset(new BgzfSource(fd, nthreads));
        } else if (gz) {
            gzFile g = gzdopen(fd, "rb");
            if (!g) {
                close(fd);
                return nullptr;
            }
            src.reset(new GzSource(g));
        } else {
            struct stat st;
            if (fstat(fd, &st) == 0 && S_ISREG(st.st_mode) && st.st_size > 0 && !getenv("CCSX_INGEST_BLOCK"))
                src.reset(mm = new MmapSource(fd, (size_t)st.st_size));
            else
                src.reset(new FdSource(fd));
        }
    }
    src->block = block;
    std::unique_ptr<RecordReader> rr;
    if (is_bam) rr.reset(new BamReader(std::move(src)));
    else rr.reset(new FxReader(std::move(src)));
    return std::unique_ptr<ZmwSource>(new Grouper(std::move(rr), mm));
}

}  // namespace ccsx_ingest
