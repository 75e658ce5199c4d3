// ingest.cpp -- host FASTA ingest for libdrephip: what `mash sketch <fasta>`
// reads (drep/d_cluster.py:543-544), turned into the packed layout the sketch
// kernel streams (2-bit codes + validity bitmap, include/drephip.h).
//
// Parsing follows kseq.h's kseq_read as Mash loops over it (oracle/
// mash_oracle.c restates it byte by byte): with no header pending, any bytes
// up to the next '>' or '@' are skipped; the header is the rest of that line;
// the sequence is every following line (line breaks and a line-final '\r'
// dropped) until a line starting with '>', '@' or '+'; after '+' (FASTQ) the
// rest of that line is skipped and whole quality lines are read until the
// quality is at least as long as the sequence -- a quality of a different
// length (or none) ends the file there, that record not kept, as kseq_read's
// -2 ends Mash's loop.  Bytes are upper-cased a-z; only A/C/G/T are valid
// bases, anything else breaks k-mers.  Plain or gzip input (gzip inflated
// whole by libdeflate when it is present, else streamed through zlib).
//
// Speed: the file is read in 4 MiB blocks, lines are found with memchr and
// sequence lines appended with memcpy; packing builds each 32-base group
// (two code words + one validity word) with SSE2 compares and BMI2 pext (a
// byte LUT for the partial groups at record ends) and stores it once.
#include "ctx.h"

#include <zlib.h>
#include <dlfcn.h>
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <immintrin.h>

namespace drephip {

// 64-bit mask of the '\n' bytes among p[0..63] (SSE2)
__attribute__((target("sse2"))) static inline uint64_t newline_mask64(const char *p) {
    const __m128i nl = _mm_set1_epi8('\n');
    uint64_t m = 0;
#pragma GCC unroll 4
    for (int h = 0; h < 4; h++)
        m |= (uint64_t)(uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128((const __m128i *)(p + 16 * h)), nl))
             << (16 * h);
    return m;
}

// first '>' or '@' in [p, end), or end
static inline const char *find_header_char(const char *p, const char *end) {
    while (p < end && *p != '>' && *p != '@') p++;
    return p;
}

// libdeflate (Ubuntu's libdeflate0 1.10; its header is not installed, so the
// four entry points used are declared here and bound at run time): a gzip file
// is read whole and inflated in one call, 2-3x zlib's streaming inflate.  Any
// file it does not take (no library, DREPHIP_NO_LIBDEFLATE, not gzip, a
// member it rejects) goes through zlib's gzread, which defines the semantics
// (concatenated members, trailing garbage ignored).
namespace {
struct Libdeflate {
    typedef void *(*alloc_t)();
    typedef int (*gunzip_t)(void *, const void *, size_t, void *, size_t, size_t *, size_t *);
    typedef void (*free_t)(void *);
    alloc_t alloc = nullptr;
    gunzip_t gunzip = nullptr;
    free_t release = nullptr;
    Libdeflate() {
        if (std::getenv("DREPHIP_NO_LIBDEFLATE")) return;
        void *h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        alloc = (alloc_t)dlsym(h, "libdeflate_alloc_decompressor");
        gunzip = (gunzip_t)dlsym(h, "libdeflate_gzip_decompress_ex");
        release = (free_t)dlsym(h, "libdeflate_free_decompressor");
        if (!alloc || !gunzip || !release) alloc = nullptr;
    }
};
const Libdeflate &libdeflate() {
    static const Libdeflate d;
    return d;
}
struct Decompressor {                      // one per worker thread
    void *d = nullptr;
    ~Decompressor() { if (d) libdeflate().release(d); }
};
constexpr int kLdSuccess = 0, kLdInsufficientSpace = 3;

// the whole gzip file at `path` inflated into out[0..*n); false: not taken
bool gunzip_whole(const char *path, std::vector<char> &in, std::vector<char> &out, size_t *n) {
    const Libdeflate &L = libdeflate();
    if (!L.alloc) return false;
    FILE *fp = fopen(path, "rb");
    if (!fp) return false;
    unsigned char magic[2] = {0, 0};
    if (fread(magic, 1, 2, fp) != 2 || magic[0] != 0x1f || magic[1] != 0x8b) { fclose(fp); return false; }   // plain: zlib path
    fseek(fp, 0, SEEK_END);
    const long sz = ftell(fp);
    fseek(fp, 0, SEEK_SET);
    if (sz < 18) { fclose(fp); return false; }
    if (in.size() < (size_t)sz) in.resize((size_t)sz);
    const size_t got = fread(in.data(), 1, (size_t)sz, fp);
    fclose(fp);
    if (got != (size_t)sz) return false;
    static thread_local Decompressor dec;
    if (!dec.d && !(dec.d = L.alloc())) return false;
    // the last member's ISIZE (exact for the usual single-member file)
    uint32_t isize;
    memcpy(&isize, in.data() + sz - 4, 4);
    size_t pos = 0, o = 0;
    if (out.size() < (size_t)isize + 64) out.resize((size_t)isize + 64);
    while (pos < (size_t)sz) {
        if (sz - pos < 18 || (uint8_t)in[pos] != 0x1f || (uint8_t)in[pos + 1] != 0x8b) break;   // trailing bytes
        size_t used_in = 0, produced = 0;
        const int r = L.gunzip(dec.d, in.data() + pos, (size_t)sz - pos, out.data() + o, out.size() - o, &used_in, &produced);
        if (r == kLdInsufficientSpace) { out.resize(2 * out.size() + (1u << 20)); continue; }
        if (r != kLdSuccess) return false;
        pos += used_in;
        o += produced;
    }
    *n = o;
    return true;
}
}  // namespace

int read_fasta(const char *path, Genome &g) {
    static thread_local std::vector<char> zin, zout;              // libdeflate buffers, reused across files
    size_t zn = 0;
    const bool whole = gunzip_whole(path, zin, zout, &zn);
    gzFile f = nullptr;
    if (!whole) {
        f = gzopen(path, "rb");
        if (!f) { set_error(std::string("cannot open ") + path); return -1; }
        gzbuffer(f, 1 << 20);
    }
    g.seq.clear(); g.rec_len.clear(); g.length = 0;
    // the sequence buffer is sized once (file size; x4 if gzip; the inflated
    // size) and written through a cursor, then trimmed at the end
    size_t used = 0;
    if (whole) {
        g.seq.resize(zn);
    } else if (FILE *fp = fopen(path, "rb")) {
        fseek(fp, 0, SEEK_END);
        const long sz = ftell(fp);
        fclose(fp);
        if (sz > 0) g.seq.resize((size_t)sz * (gzdirect(f) ? 1 : 4));
    }
    auto append = [&](const char *p, size_t n) {
        if (used + n > g.seq.size()) g.seq.resize(std::max(used + n, 2 * g.seq.size() + 64));
        memcpy(g.seq.data() + used, p, n);
        used += n;
        g.rec_len.back() += n;
    };
    auto end_seq_line = [&] {                      // a line-final '\r' is dropped
        if (used && g.seq[used - 1] == '\r' && g.rec_len.back()) { used--; g.rec_len.back()--; }
    };
    auto drop_last_record = [&] { used -= g.rec_len.back(); g.rec_len.pop_back(); };
    // Byte state machine, carried across blocks:
    //   HUNT   no header pending: skip to the next '>' or '@' (anywhere)
    //   HDR0   just after '>'/'@': the record exists once one more byte does
    //   HDR    rest of the header line
    //   START  first byte of a line inside a record
    //   SEQ    inside a sequence line (copied in 64-byte chunks up to '\n')
    //   PLUS   rest of a FASTQ '+' line
    //   QUAL   FASTQ quality lines, counted until >= the sequence length
    enum { HUNT, HDR0, HDR, START, SEQ, PLUS, QUAL } st = HUNT;
    uint64_t qlen = 0, qline = 0;                  // quality so far; current quality line's length
    char qlast = 0;                                // its last byte (a final '\r' is not counted)
    bool stop = false;
    // one block of the file through the state machine
    auto feed = [&](const char *p, const char *end) {
        while (p < end && !stop) {
            switch (st) {
            case HUNT:
                p = find_header_char(p, end);
                if (p < end) { p++; st = HDR0; }
                continue;
            case HDR0:
                g.rec_len.push_back(0);
                st = HDR;
                continue;
            case HDR: {
                const char *nl = (const char *)memchr(p, '\n', end - p);
                if (!nl) { p = end; continue; }
                p = nl + 1;
                st = START;
                continue;
            }
            case PLUS: {
                const char *nl = (const char *)memchr(p, '\n', end - p);
                if (!nl) { p = end; continue; }
                p = nl + 1;
                st = QUAL; qlen = 0; qline = 0; qlast = 0;
                continue;
            }
            case QUAL: {
                const char *nl = (const char *)memchr(p, '\n', end - p);
                const char *le = nl ? nl : end;
                if (le > p) { qline += (uint64_t)(le - p); qlast = le[-1]; }
                if (!nl) { p = end; continue; }
                p = nl + 1;
                qlen += qline - (qline && qlast == '\r');
                qline = 0; qlast = 0;
                if (qlen >= g.rec_len.back()) {
                    if (qlen != g.rec_len.back()) { drop_last_record(); stop = true; }     // kseq_read: -2
                    st = HUNT;
                }
                continue;
            }
            case START: {
                const char c = *p;
                if (c == '\n') { p++; continue; }                                     // empty line
                if (c == '>' || c == '@') { p++; st = HDR0; continue; }
                if (c == '+') { p++; st = PLUS; continue; }
                st = SEQ;
                continue;
            }
            case SEQ:
                break;
            }
            // SEQ: 64-byte chunks; every sequence line inside a chunk is
            // compacted with a fixed 64-byte copy (the output cursor advances by
            // the line's length, later copies overwrite the excess); a line that
            // starts with '>', '@' or '+' hands over to START
            while (end - p >= 64) {
                uint64_t m = newline_mask64(p);
                if (used + 128 > g.seq.size()) g.seq.resize(std::max(used + 128, 2 * g.seq.size()));
                uint8_t *out = g.seq.data();
                int pos = 0;
                bool handover = false;
                while (m) {
                    const int j = __builtin_ctzll(m);
                    memcpy(out + used, p + pos, 64);
                    used += (size_t)(j - pos);
                    g.rec_len.back() += (uint64_t)(j - pos);
                    // line-final '\r': inside this segment, or (newline first in
                    // a chunk that continues a line) at the end of the previous one
                    const bool cr = j > pos ? p[j - 1] == '\r' : (j == 0 && used && out[used - 1] == '\r');
                    if (cr && g.rec_len.back()) { used--; g.rec_len.back()--; }
                    pos = j + 1;
                    m &= m - 1;
                    if (pos < 64) {
                        const char c = p[pos];
                        if (c == '>' || c == '@' || c == '+') { handover = true; break; }
                    } else {
                        break;
                    }
                }
                if (handover || pos == 64) {                // next byte starts a line
                    p += pos;
                    st = START;
                    goto next_state;
                }
                memcpy(out + used, p + pos, 64);            // rest of the chunk: inside a sequence line
                used += (size_t)(64 - pos);
                g.rec_len.back() += (uint64_t)(64 - pos);
                p += 64;
            }
            {
                const char *nl = (const char *)memchr(p, '\n', end - p);
                if (!nl) { append(p, end - p); p = end; break; }
                append(p, nl - p);
                p = nl + 1;
            }
            end_seq_line();
            st = START;
        next_state:;
        }
    };
    if (whole) {
        feed(zout.data(), zout.data() + zn);
    } else {
        const size_t kBlock = 4u << 20;
        static thread_local std::vector<char> buf(kBlock + 64);   // reused across files (no 4 MiB memset each)
        while (!stop) {
            const int got = gzread(f, buf.data(), (unsigned)kBlock);
            if (got < 0) { gzclose(f); set_error(std::string("read error in ") + path); return -1; }
            if (got == 0) break;
            feed(buf.data(), buf.data() + got);
        }
        gzclose(f);
    }
    // end of file
    if (st == SEQ) end_seq_line();
    else if (st == HDR0) { /* '>' as the last byte: kseq_read returns -1, no record */ }
    else if (st == PLUS) drop_last_record();                       // no quality string: -2
    else if (st == QUAL && !stop) {
        if (qline) qlen += qline - (qlast == '\r');                  // last line, no '\n'
        if (qlen != g.rec_len.back()) drop_last_record();            // short quality: -2
    }
    g.seq.resize(used);
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

// 32 bases -> 64 code bits + 32 validity bits with SSE2 (+ BMI2 pext when the
// host has it).  Codes: ((c >> 1) ^ (c >> 2)) & 3 maps A/C/G/T and a/c/g/t to
// 0/1/2/3 (bits 1..3 of each byte; 16-bit shifts leak nothing into bits 0..1
// of a byte); valid: (c & 0xDF) is one of 'A','C','G','T'; invalid bytes get
// code 0, as in the scalar path.
static inline uint64_t gather2_swar(uint64_t c) {      // 8 bytes of 2-bit values -> 16 bits
    uint64_t t = (c | (c >> 6)) & 0x000F000F000F000Full;
    t = (t | (t >> 12)) & 0x000000FF000000FFull;
    return (t | (t >> 24)) & 0xFFFFull;
}
__attribute__((target("bmi2"))) static inline uint64_t gather2_pext(uint64_t c) {
    return _pext_u64(c, 0x0303030303030303ull);
}
template <bool PEXT>
__attribute__((target("sse2,bmi2"))) static inline void pack32(const uint8_t *s, uint64_t &codes, uint32_t &valid) {
    const __m128i m3 = _mm_set1_epi8(3), mDF = _mm_set1_epi8((char)0xDF);
    const __m128i A = _mm_set1_epi8('A'), Cc = _mm_set1_epi8('C'), G = _mm_set1_epi8('G'), T = _mm_set1_epi8('T');
    uint64_t out = 0;
    uint32_t vm = 0;
#pragma GCC unroll 2
    for (int h = 0; h < 2; h++) {
        const __m128i v = _mm_loadu_si128((const __m128i *)(s + 16 * h));
        const __m128i u = _mm_and_si128(v, mDF);
        const __m128i ok = _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(u, A), _mm_cmpeq_epi8(u, Cc)),
                                        _mm_or_si128(_mm_cmpeq_epi8(u, G), _mm_cmpeq_epi8(u, T)));
        vm |= (uint32_t)_mm_movemask_epi8(ok) << (16 * h);
        const __m128i c = _mm_and_si128(_mm_and_si128(_mm_xor_si128(_mm_srli_epi16(v, 1), _mm_srli_epi16(v, 2)), m3),
                                        ok);                            // invalid bases: code 0 (layout contract)
        const uint64_t lo = (uint64_t)_mm_cvtsi128_si64(c), hi = (uint64_t)_mm_cvtsi128_si64(_mm_unpackhi_epi64(c, c));
        const uint64_t g = PEXT ? (gather2_pext(lo) | gather2_pext(hi) << 16) : (gather2_swar(lo) | gather2_swar(hi) << 16);
        out |= g << (32 * h);
    }
    codes = out;
    valid = vm;
}
static bool host_has_bmi2() {
    static const bool b = __builtin_cpu_supports("bmi2");
    return b;
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
template <bool PEXT>
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
            pack32<PEXT>(s + i, clo, vw);
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
    const bool pext = host_has_bmi2();
    for (uint32_t r = 0; r < n_rec; r++) {
        nk += pext ? pack_span<true>(s, rec_len[r], pos, k, lut, codes, valid)
                   : pack_span<false>(s, rec_len[r], pos, k, lut, codes, valid);
        s += rec_len[r];
        pos += rec_len[r] + 1;          // one invalid separator between records
    }
    return nk;
}

}  // namespace drephip
