// ingest.cpp -- host FASTA ingest for libdrephip: what `mash sketch <fasta>`
// reads (drep/d_cluster.py:543-544), turned into the packed layout the sketch
// kernel streams (2-bit codes + validity bitmap, include/drephip.h).
//
// Parsing follows kseq.h as Mash uses it: a record starts at a line beginning
// with '>' (or '@'); its sequence is every following line, line breaks (and a
// line-final '\r') dropped, until the next header; a line starting with '+'
// ends the sequence (FASTQ quality follows).  Bytes are upper-cased a-z; only
// A/C/G/T are valid bases, anything else breaks k-mers.  Plain or gzip input.
//
// Speed: the file is read in 4 MiB blocks, lines are found with memchr and
// sequence lines appended with memcpy; packing builds each 32-base group
// (two code words + one validity word) in registers from a byte LUT and
// stores it once.
#include "ctx.h"

#include <zlib.h>
#include <algorithm>
#include <cstdio>
#include <cstring>

namespace drephip {

int read_fasta(const char *path, Genome &g) {
    gzFile f = gzopen(path, "rb");
    if (!f) { set_error(std::string("cannot open ") + path); return -1; }
    gzbuffer(f, 1 << 20);
    g.seq.clear(); g.rec_len.clear(); g.length = 0;
    if (FILE *fp = fopen(path, "rb")) {          // capacity hint: file size (x4 if gzip)
        fseek(fp, 0, SEEK_END);
        const long sz = ftell(fp);
        fclose(fp);
        if (sz > 0) g.seq.reserve((size_t)sz * (gzdirect(f) ? 1 : 4));
    }
    const size_t kBlock = 4u << 20;
    std::vector<char> buf(kBlock + 1);
    std::string carry;                    // partial line spanning blocks
    bool in_seq = false;                  // inside a record's sequence lines

    auto line = [&](const char *p, size_t n) {
        if (n && p[n - 1] == '\r') n--;
        if (n == 0) return;
        const char c0 = p[0];
        if (c0 == '>' || c0 == '@') { g.rec_len.push_back(0); in_seq = true; return; }
        if (c0 == '+') { in_seq = false; return; }
        if (!in_seq) return;
        const size_t old = g.seq.size();
        g.seq.resize(old + n);
        memcpy(g.seq.data() + old, p, n);
        g.rec_len.back() += n;
    };
    for (;;) {
        const int got = gzread(f, buf.data(), (unsigned)kBlock);
        if (got < 0) { gzclose(f); set_error(std::string("read error in ") + path); return -1; }
        if (got == 0) break;
        const char *p = buf.data(), *end = p + got;
        if (!carry.empty()) {
            const char *nl = (const char *)memchr(p, '\n', end - p);
            if (!nl) { carry.append(p, end - p); continue; }
            carry.append(p, nl - p);
            line(carry.data(), carry.size());
            carry.clear();
            p = nl + 1;
        }
        while (p < end) {
            const char *nl = (const char *)memchr(p, '\n', end - p);
            if (!nl) { carry.assign(p, end - p); break; }
            line(p, nl - p);
            p = nl + 1;
        }
    }
    if (!carry.empty()) line(carry.data(), carry.size());
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

// Mask of positions (bits) ending a run of >= k set bits in `v` (k <= 32),
// by doubling: a1 = v, a2 = a1 & a1<<1, a4, a8, a16, then the binary digits of
// k combined at growing offsets.
static inline uint64_t run_k_mask(uint64_t v, int k) {
    uint64_t a[6];
    a[0] = v;
    for (int i = 1; i < 6; i++) a[i] = a[i - 1] & (a[i - 1] << (1 << (i - 1)));
    uint64_t m = ~0ull;
    int off = 0;
    for (int i = 5; i >= 0; i--)
        if (k & (1 << i)) { m &= a[i] << off; off += 1 << i; }
    return m;
}

// Pack n bytes of one record starting at base position pos (any alignment).
// Whole 32-base groups are built in registers; partial groups at either end
// are OR-ed into the (zeroed) arrays.  Returns the valid k-mers ending in it.
static uint64_t pack_span(const uint8_t *s, uint64_t n, uint64_t pos, int k, const uint8_t *lut,
                          uint32_t *codes, uint32_t *valid) {
    uint64_t hist = 0;                  // validity of the previous group (bits 0..31)
    uint64_t nk = 0;
    uint64_t i = 0;
    while (i < n) {
        const uint64_t q = (pos + i) >> 5;
        const uint32_t o = (uint32_t)((pos + i) & 31);
        const uint32_t take = (uint32_t)std::min<uint64_t>(32 - o, n - i);
        uint64_t clo = 0;
        uint32_t vw = 0;
        if (take == 32) {
#pragma GCC unroll 32
            for (uint32_t t = 0; t < 32; t++) {
                const uint32_t c = lut[s[i + t]];
                clo |= (uint64_t)(c & 3u) << (2 * t);
                vw |= ((c >> 2) ^ 1u) << t;
            }
        } else {
            for (uint32_t t = 0; t < take; t++) {
                const uint32_t c = lut[s[i + t]];
                clo |= (uint64_t)(c & 3u) << (2 * (o + t));
                vw |= ((c >> 2) ^ 1u) << (o + t);
            }
        }
        codes[2 * q] |= (uint32_t)clo;
        codes[2 * q + 1] |= (uint32_t)(clo >> 32);
        valid[q] |= vw;
        // k-mers ending in this group: runs over (previous group, this group);
        // bits before the record start are 0 in hist/vw
        const uint64_t h = (hist >> 32) | ((uint64_t)vw << 32);
        nk += (uint64_t)__builtin_popcountll(run_k_mask(h, k) >> 32);
        hist = h;
        i += take;
    }
    return nk;
}

uint64_t pack_records(const uint8_t *seq, const uint64_t *rec_len, uint32_t n_rec, int k,
                      uint32_t *codes, uint32_t *valid, uint64_t base_off) {
    const uint8_t *lut = code_lut();
    uint64_t pos = base_off, nk = 0;
    const uint8_t *s = seq;
    for (uint32_t r = 0; r < n_rec; r++) {
        nk += pack_span(s, rec_len[r], pos, k, lut, codes, valid);
        s += rec_len[r];
        pos += rec_len[r] + 1;          // one invalid separator between records
    }
    return nk;
}

}  // namespace drephip
