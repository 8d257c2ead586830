// seqio.cpp -- subread ingest (include/ccsx_seqio.h).
//
// FASTA/FASTQ records follow kseq.h:178-218; BAM records bamlite.c:78-165 and
// seqio.h:92-118; grouping into ZMWs follows kseq_zmw_read, seqio.h:152-201,
// including its quirks: an invalid record name returns -1 without touching
// the "last record" state, so the caller's next call resumes after it.
#include "ccsx_seqio.h"

#include <zlib.h>

#include <cctype>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

struct ccsx_reader {
    gzFile fp = nullptr;
    bool bam = false;
    std::vector<unsigned char> buf;
    size_t bpos = 0, bend = 0;
    bool eof = false;
    int last_char = 0;
    std::string name, seq, qual;
    // ZMW grouping state (seqio.h:14-19)
    std::string movie, hole, seqs, last_movie, last_hole, last_seq;
    std::vector<uint32_t> lens;
    std::vector<uint8_t> bamrec;
};

namespace {

int getc_(ccsx_reader *r)
{
    if (r->bpos >= r->bend) {
        if (r->eof) return -1;
        int n = gzread(r->fp, r->buf.data(), (unsigned)r->buf.size());
        if (n <= 0) {
            r->eof = true;
            return -1;
        }
        r->bpos = 0;
        r->bend = (size_t)n;
    }
    return r->buf[r->bpos++];
}

// rest of the line into s (append); strips one trailing '\r' (kseq.h:141)
int getline_(ccsx_reader *r, std::string &s)
{
    int c;
    while ((c = getc_(r)) >= 0 && c != '\n') s.push_back((char)c);
    if (s.size() > 1 && s.back() == '\r') s.pop_back();
    return c;
}

// kseq.h:178-218
int kseq_read(ccsx_reader *r)
{
    int c;
    if (r->last_char == 0) {
        while ((c = getc_(r)) >= 0 && c != '>' && c != '@') {
        }
        if (c < 0) return -1;
        r->last_char = c;
    }
    r->name.clear(), r->seq.clear(), r->qual.clear();
    while ((c = getc_(r)) >= 0 && !isspace(c)) r->name.push_back((char)c);
    if (c < 0 && r->name.empty()) return -1;
    if (c >= 0 && c != '\n') {
        std::string comment;
        getline_(r, comment);
    }
    while ((c = getc_(r)) >= 0 && c != '>' && c != '+' && c != '@') {
        if (c == '\n') continue;
        r->seq.push_back((char)c);
        getline_(r, r->seq);
    }
    if (c == '>' || c == '@') r->last_char = c;
    if (c != '+') return (int)r->seq.size();
    while ((c = getc_(r)) >= 0 && c != '\n') {
    }
    if (c == -1) return -2;
    while (r->qual.size() < r->seq.size()) {
        size_t before = r->qual.size();
        c = getline_(r, r->qual);
        if (c < 0 && r->qual.size() == before) break;
        if (c < 0) break;
    }
    r->last_char = 0;
    if (r->seq.size() != r->qual.size()) return -2;
    return (int)r->seq.size();
}

bool gz_exact(gzFile fp, void *p, unsigned n) { return gzread(fp, p, n) == (int)n; }

// bamlite.c:78-115 (header) -- returns false on an invalid header
bool bam_header(ccsx_reader *r)
{
    char magic[4];
    int32_t l_text, n_ref, l_name, l_ref;
    if (!gz_exact(r->fp, magic, 4) || memcmp(magic, "BAM\1", 4) != 0) return false;
    if (!gz_exact(r->fp, &l_text, 4) || l_text < 0) return false;
    std::vector<char> text((size_t)l_text + 1);
    if (l_text && !gz_exact(r->fp, text.data(), (unsigned)l_text)) return false;
    if (!gz_exact(r->fp, &n_ref, 4)) return false;
    for (int32_t i = 0; i < n_ref; ++i) {
        if (!gz_exact(r->fp, &l_name, 4) || l_name < 0) return false;
        std::vector<char> nm((size_t)l_name);
        if (l_name && !gz_exact(r->fp, nm.data(), (unsigned)l_name)) return false;
        if (!gz_exact(r->fp, &l_ref, 4)) return false;
    }
    return true;
}

// bamlite.c:135-165 + seqio.h:93-118
int bam_read(ccsx_reader *r)
{
    static const char nt16[] = "=ACMGRSVTWYHKDBN";
    int32_t block_len;
    int n = gzread(r->fp, &block_len, 4);
    if (n != 4) return -1;
    if (block_len < 32) return -3;
    r->bamrec.resize((size_t)block_len);
    if (!gz_exact(r->fp, r->bamrec.data(), (unsigned)block_len)) return -4;
    uint32_t x[8];
    memcpy(x, r->bamrec.data(), 32);
    const uint32_t l_qname = x[2] & 0xff, n_cigar = x[3] & 0xffff;
    const int32_t l_qseq = (int32_t)x[4];
    const uint8_t *data = r->bamrec.data() + 32;
    const size_t data_len = (size_t)block_len - 32;
    if (l_qseq < 0 || (size_t)l_qname + n_cigar * 4 + (size_t)(l_qseq + 1) / 2 > data_len) return -4;
    r->name.assign(reinterpret_cast<const char *>(data), strnlen(reinterpret_cast<const char *>(data), l_qname));
    const uint8_t *s = data + l_qname + n_cigar * 4;
    r->seq.resize((size_t)l_qseq);
    for (int32_t i = 0; i < l_qseq; ++i) r->seq[(size_t)i] = nt16[(s[i / 2] >> (4 * (1 - i % 2))) & 0xf];
    return l_qseq;
}

int read_record(ccsx_reader *r) { return r->bam ? bam_read(r) : kseq_read(r); }

// ksplit(name, '/'): non-empty fields; returns the field count
int split3(const std::string &name, std::string f[3], std::string &shown)
{
    int n = 0;
    size_t i = 0, L = name.size();
    shown.clear();
    bool first_end = false;
    while (i < L) {
        while (i < L && name[i] == '/') ++i;
        if (i >= L) break;
        size_t j = i;
        while (j < L && name[j] != '/') ++j;
        if (n < 3) f[n] = name.substr(i, j - i);
        if (!first_end) {
            shown = name.substr(0, j);  // ksplit NUL-terminates the first field in place
            first_end = true;
        }
        ++n;
        i = j;
    }
    if (!first_end) shown = name;
    return n;
}

}  // namespace

extern "C" {

ccsx_reader *ccsx_reader_open(const char *path, int is_bam)
{
    gzFile fp = (strcmp(path, "-") == 0) ? gzdopen(fileno(stdin), "rb") : gzopen(path, "rb");
    if (!fp) return nullptr;
    auto *r = new ccsx_reader();
    r->fp = fp;
    r->bam = is_bam != 0;
    r->buf.resize(1 << 16);
    if (r->bam && !bam_header(r)) {
        fprintf(stderr, "[bam_header_read] invalid BAM header.\n");
        r->eof = true;  // seqio.h:27-31 prints and carries on; nothing can be read
        gzclose(r->fp);
        r->fp = nullptr;
    }
    return r;
}

int ccsx_reader_next(ccsx_reader *r, const char **movie, const char **hole, const char **seqs, const uint32_t **lens)
{
    r->lens.clear();
    r->movie.clear(), r->hole.clear(), r->seqs.clear();
    if (!r->last_movie.empty()) {
        r->hole = r->last_hole;
        r->movie = r->last_movie;
        r->seqs = r->last_seq;
        r->lens.push_back((uint32_t)r->last_seq.size());
    }
    int l;
    while (r->fp && (l = read_record(r)) >= 0) {
        std::string f[3], shown;
        if (split3(r->name, f, shown) != 3) {
            fprintf(stderr, "invalid zmw name :%s\n", shown.c_str());
            return -1;
        }
        if (r->last_movie.empty()) {
            r->movie = f[0], r->hole = f[1];
            r->seqs += r->seq;
            r->lens.push_back((uint32_t)r->seq.size());
            r->last_hole = r->hole, r->last_movie = r->movie, r->last_seq = r->seq;
        } else if (r->last_hole != f[1] || r->movie != f[0]) {
            r->last_movie = f[0], r->last_hole = f[1], r->last_seq = r->seq;
            *movie = r->movie.c_str(), *hole = r->hole.c_str(), *seqs = r->seqs.data(), *lens = r->lens.data();
            return (int)r->lens.size();
        } else {
            r->seqs += r->seq;
            r->lens.push_back((uint32_t)r->seq.size());
        }
    }
    r->last_movie.clear(), r->last_hole.clear(), r->last_seq.clear();
    *movie = r->movie.c_str(), *hole = r->hole.c_str(), *seqs = r->seqs.data(), *lens = r->lens.data();
    return r->lens.empty() ? -1 : (int)r->lens.size();
}

void ccsx_reader_close(ccsx_reader *r)
{
    if (!r) return;
    if (r->fp) gzclose(r->fp);
    delete r;
}

}  // extern "C"
