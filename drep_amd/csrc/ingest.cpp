// ingest.cpp -- host FASTA ingest for libdrephip: what `mash sketch <fasta>`
// reads (drep/d_cluster.py:543-544), turned into the packed layout the sketch
// kernel streams (2-bit codes + validity bitmap, include/drephip.h).
//
// Parsing follows kseq.h as Mash uses it: a record starts at a line beginning
// with '>' (or '@'); its sequence is every following line, line breaks (and a
// line-final '\r') dropped, until the next header; a line starting with '+'
// ends the sequence (FASTQ quality follows).  Bytes are upper-cased a-z; only
// A/C/G/T are valid bases, anything else breaks k-mers.  Plain or gzip input.
#include "ctx.h"

#include <zlib.h>
#include <cstring>

namespace drephip {

int read_fasta(const char *path, Genome &g) {
    gzFile f = gzopen(path, "rb");
    if (!f) { set_error(std::string("cannot open ") + path); return -1; }
    gzbuffer(f, 1 << 20);
    g.seq.clear(); g.rec_len.clear(); g.length = 0;
    std::vector<unsigned char> buf(1 << 20);
    bool line_start = true, in_header = false, in_seq = false, pending_cr = false;
    for (;;) {
        const int got = gzread(f, buf.data(), (unsigned)buf.size());
        if (got < 0) { gzclose(f); set_error(std::string("read error in ") + path); return -1; }
        if (got == 0) break;
        for (int i = 0; i < got; i++) {
            unsigned char ch = buf[i];
            if (in_header) {
                if (ch == '\n') { in_header = false; line_start = true; }
                continue;
            }
            if (pending_cr) {
                pending_cr = false;
                if (ch != '\n' && in_seq) { g.seq.push_back('\r'); g.rec_len.back()++; }
            }
            if (ch == '\n') { line_start = true; continue; }
            if (line_start) {
                line_start = false;
                if (ch == '>' || ch == '@') {
                    in_header = true; in_seq = true;
                    g.rec_len.push_back(0);
                    continue;
                }
                if (ch == '+') { in_seq = false; in_header = true; continue; }
            }
            if (ch == '\r') { pending_cr = true; continue; }
            if (!in_seq) continue;
            g.seq.push_back(ch);
            g.rec_len.back()++;
        }
    }
    gzclose(f);
    for (uint64_t l : g.rec_len) g.length += l;
    return 0;
}

uint64_t genome_span(const uint64_t *rec_len, uint32_t n_rec) {
    uint64_t span = 0;
    for (uint32_t r = 0; r < n_rec; r++) span += rec_len[r];
    return span + (n_rec ? n_rec - 1 : 0);   // one invalid separator between records
}

// base code per byte: 0..3 for A/C/G/T (either case), 4 = invalid
static const uint8_t *code_lut() {
    static uint8_t lut[256];
    static bool init = [] {
        memset(lut, 4, sizeof(lut));
        lut['A'] = lut['a'] = 0; lut['C'] = lut['c'] = 1;
        lut['G'] = lut['g'] = 2; lut['T'] = lut['t'] = 3;
        return true;
    }();
    (void)init;
    return lut;
}

uint64_t pack_records(const uint8_t *seq, const uint64_t *rec_len, uint32_t n_rec, int k,
                      uint32_t *codes, uint32_t *valid, uint64_t base_off) {
    const uint8_t *lut = code_lut();
    uint64_t p = base_off, nk = 0;
    const uint8_t *s = seq;
    for (uint32_t r = 0; r < n_rec; r++) {
        uint64_t run = 0;
        for (uint64_t i = 0; i < rec_len[r]; i++) {
            const uint8_t c = lut[s[i]];
            if (c < 4) {
                codes[p >> 4] |= (uint32_t)c << (2 * (p & 15));
                valid[p >> 5] |= 1u << (p & 31);
                run++;
                nk += run >= (uint64_t)k;
            } else {
                run = 0;
            }
            p++;
        }
        s += rec_len[r];
        p++;   // separator (invalid)
    }
    return nk;
}

}  // namespace drephip
