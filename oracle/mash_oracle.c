/*
 * mash_oracle.c -- CPU restatement of the Mash sketch / dist arithmetic that
 * dRep's primary clustering shells out to.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP path
 * in drep_amd/csrc/ and the "port" CPU baseline of bench.py.  Nothing in the
 * product (drep_amd/, libdrephip.so) links, loads or calls it; only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may.
 *
 * Where the algorithm lives: the external Mash binary (marbl/Mash, C++).  It is
 * NOT vendored under /root/reference and not installed, so this is a
 * restatement of its published algorithm; the only version statement in the
 * reference is docs/installation.rst:34 ("v1.1.1 confirmed works").  Call sites
 * it stands in for:
 *   mash sketch <fa> -s S -o out      drep/d_cluster.py:543-544
 *   mash dist -p P ALL.msh ALL.msh    drep/d_cluster.py:570-572
 * Parity pin: tests/golden/ holds the reference's own fixtures
 * (tests/test_solutions/ecoli_wd/data/MASH_files/: the five sketches/<genome>.msh,
 * ALL.msh and MASH_table.tsv); tests/test_oracle.py checks this file against every one of
 * them (4 FASTA -> .msh sketches bit-exact, 25/25 TSV rows).
 *
 * Spec (SURVEY.md section 8 "Mash spec"):
 *   sketch: every record of a FASTA (kseq semantics) is upper-cased; a k-mer is
 *   valid iff all k bytes are in {A,C,G,T}; k-mers never span records;
 *   canon = memcmp(fwd, revcomp) <= 0 ? fwd : revcomp;
 *   h = MurmurHash3_x64_128(canon, k, seed).h1; sketch = s smallest DISTINCT h,
 *   ascending; length = sum of record lengths (N included).
 *   dist: merge of the two sorted sketches until denom == s (Mash
 *   Sketch::compare / CommandDistance::compare).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#include <math.h>
#include <zlib.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ---------------------------------------------------------------- Murmur3 */
/* MurmurHash3_x64_128 (public-domain algorithm by A. Appleby), first 64 bits.
 * Mash: getHash() -> MurmurHash3_x64_128(seq, k, seed, data); hash64=data[0]. */
static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t fmix64(uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33; return k;
}

uint64_t oracle_murmur3_h1(const uint8_t *data, int len, uint32_t seed) {
    const uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
    uint64_t h1 = seed, h2 = seed;
    int nblocks = len / 16;
    for (int i = 0; i < nblocks; i++) {
        uint64_t k1, k2;
        memcpy(&k1, data + 16 * i, 8);
        memcpy(&k2, data + 16 * i + 8, 8);
        k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
        h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
        k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
        h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
    }
    const uint8_t *tail = data + 16 * nblocks;
    uint64_t k1 = 0, k2 = 0;
    int rem = len & 15;
    if (rem > 8) {
        for (int i = rem - 1; i >= 8; i--) k2 ^= (uint64_t)tail[i] << (8 * (i - 8));
        k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
    }
    if (rem > 0) {
        int top = rem > 8 ? 8 : rem;
        for (int i = top - 1; i >= 0; i--) k1 ^= (uint64_t)tail[i] << (8 * i);
        k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
    }
    h1 ^= (uint64_t)len; h2 ^= (uint64_t)len;
    h1 += h2; h2 += h1;
    h1 = fmix64(h1); h2 = fmix64(h2);
    h1 += h2;
    return h1;
}

/* ------------------------------------------------------- bottom-s "heap" */
/* Restatement of Mash's MinHashHeap::tryInsert (no multiplicity filter,
 * the dRep call never passes -m): a max-heap of the current s smallest
 * distinct hashes plus a set for the distinctness test. */
typedef struct {
    uint64_t *heap; uint32_t n, cap;
    uint64_t *set; uint32_t set_mask;   /* open addressing, tombstones */
    uint32_t tombs;                     /* rebuilt when tombstones pile up */
} bottom_s;

#define SET_EMPTY 0xFFFFFFFFFFFFFFFFULL
#define SET_TOMB  0xFFFFFFFFFFFFFFFEULL

static uint32_t set_slot(uint64_t h, uint32_t mask) { return (uint32_t)(fmix64(h) & mask); }

static int set_has(const bottom_s *b, uint64_t h) {
    uint32_t i = set_slot(h, b->set_mask);
    for (;;) {
        uint64_t v = b->set[i];
        if (v == h) return 1;
        if (v == SET_EMPTY) return 0;
        i = (i + 1) & b->set_mask;
    }
}
static void set_add(bottom_s *b, uint64_t h) {
    uint32_t i = set_slot(h, b->set_mask);
    while (b->set[i] != SET_EMPTY && b->set[i] != SET_TOMB) i = (i + 1) & b->set_mask;
    b->set[i] = h;
}
static void set_del(bottom_s *b, uint64_t h) {
    uint32_t i = set_slot(h, b->set_mask);
    for (;;) {
        if (b->set[i] == h) { b->set[i] = SET_TOMB; b->tombs++; return; }
        if (b->set[i] == SET_EMPTY) return;
        i = (i + 1) & b->set_mask;
    }
}
static void set_rebuild(bottom_s *b) {
    b->tombs = 0;
    memset(b->set, 0xFF, sizeof(uint64_t) * (b->set_mask + 1));
    for (uint32_t i = 0; i < b->n; i++) set_add(b, b->heap[i]);
}

static int bs_init(bottom_s *b, uint32_t s) {
    b->cap = s; b->n = 0; b->tombs = 0;
    uint32_t sz = 16; while (sz < 4 * s + 16) sz <<= 1;
    b->set_mask = sz - 1;
    b->heap = (uint64_t *)malloc(sizeof(uint64_t) * (s + 1));
    b->set = (uint64_t *)malloc(sizeof(uint64_t) * sz);
    if (!b->heap || !b->set) return -1;
    memset(b->set, 0xFF, sizeof(uint64_t) * sz);
    return 0;
}
static void bs_free(bottom_s *b) { free(b->heap); free(b->set); }

static void heap_up(uint64_t *h, uint32_t i) {
    while (i > 0) { uint32_t p = (i - 1) / 2; if (h[p] >= h[i]) break;
        uint64_t t = h[p]; h[p] = h[i]; h[i] = t; i = p; }
}
static void heap_down(uint64_t *h, uint32_t n, uint32_t i) {
    for (;;) { uint32_t l = 2 * i + 1, r = l + 1, m = i;
        if (l < n && h[l] > h[m]) m = l;
        if (r < n && h[r] > h[m]) m = r;
        if (m == i) break;
        uint64_t t = h[m]; h[m] = h[i]; h[i] = t; i = m; }
}

static inline void bs_try_insert(bottom_s *b, uint64_t h) {
    if (b->n == b->cap && h >= b->heap[0]) return;      /* the common case */
    if (set_has(b, h)) return;
    if (b->n < b->cap) {
        b->heap[b->n++] = h; heap_up(b->heap, b->n - 1); set_add(b, h);
    } else {
        set_del(b, b->heap[0]);
        b->heap[0] = h; heap_down(b->heap, b->n, 0);
        if (b->tombs > b->cap) set_rebuild(b); else set_add(b, h);
    }
}

static int cmp_u64(const void *a, const void *b) {
    uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : (x > y);
}

/* ------------------------------------------------------------ k-mer scan */
static inline uint8_t comp_base(uint8_t c) {   /* only called on A/C/G/T */
    return c == 'A' ? 'T' : c == 'C' ? 'G' : c == 'G' ? 'C' : 'A';
}
static inline int is_acgt(uint8_t c) { return c == 'A' || c == 'C' || c == 'G' || c == 'T'; }

/* Visit every valid canonical k-mer hash of one record (already upper-cased).
 * Mash Sketch.cpp addMinHashes(): skip past any byte not in the alphabet,
 * canonical = memcmp(fwd, rev, k) <= 0 ? fwd : rev. */
typedef void (*hash_sink)(void *ctx, uint64_t h);
static void scan_record(const uint8_t *seq, uint64_t len, int k, uint32_t seed,
                        hash_sink sink, void *ctx) {
    if (len < (uint64_t)k) return;
    uint8_t rc[64];
    uint64_t run = 0;                 /* valid bases ending at i */
    for (uint64_t i = 0; i < len; i++) {
        run = is_acgt(seq[i]) ? run + 1 : 0;
        if (run < (uint64_t)k) continue;
        const uint8_t *fwd = seq + i + 1 - k;
        for (int j = 0; j < k; j++) rc[j] = comp_base(fwd[k - 1 - j]);
        const uint8_t *canon = memcmp(fwd, rc, k) <= 0 ? fwd : rc;
        sink(ctx, oracle_murmur3_h1(canon, k, seed));
    }
}

/* ------------------------------------------------------------ FASTA input */
/* kseq.h's kseq_read as Mash loops over it (`while ((l = kseq_read(seq)) >=
 * 0)`), restated character by character (klib kseq.h, public domain):
 *   - with no header character pending, skip ANY bytes up to the next '>' or
 *     '@' (text before the first header; the bytes after a FASTQ record);
 *   - the header line is the rest of that line;
 *   - sequence: lines whose first byte is not '>', '+' or '@' (empty lines
 *     skipped), each without its '\n' (and, as Mash's parse of CRLF files
 *     behaves, without a line-final '\r'); a '>'/'@' line start ends the record
 *     with the next header's first byte already read;
 *   - '+' (FASTQ): the rest of that line is skipped, then whole quality lines
 *     are read until the quality is at least as long as the sequence; a
 *     quality of a different length, or none (EOF), makes kseq_read return -2:
 *     that record is not kept and reading stops.
 * Returns a malloc'd buffer of the concatenated, upper-cased record sequences
 * and a malloc'd record-offset array (n_rec + 1 entries). gz or plain. */
typedef struct { gzFile f; unsigned char buf[1 << 16]; int n, i; } kbuf;
static int kgetc(kbuf *k) {
    if (k->i == k->n) { k->n = gzread(k->f, k->buf, sizeof(k->buf)); k->i = 0; if (k->n <= 0) { k->n = 0; return -1; } }
    return k->buf[k->i++];
}
/* one line (after its first byte c0, if c0 >= 0) up to '\n' or EOF: length
 * without the '\n' and a final '\r'; *end = '\n' or -1 */
static size_t kline_len(kbuf *k, int c0, int *end) {
    size_t ll = 0; int c, lastc = -1;
    if (c0 >= 0) { ll = 1; lastc = c0; }
    while ((c = kgetc(k)) >= 0 && c != '\n') { ll++; lastc = c; }
    if (lastc == '\r') ll--;
    *end = c;
    return ll;
}
int oracle_read_fasta(const char *path, uint8_t **seq_out, uint64_t **off_out,
                      uint32_t *nrec_out, uint64_t *len_out) {
    kbuf *k = (kbuf *)malloc(sizeof(kbuf));
    k->f = gzopen(path, "rb");
    if (!k->f) { free(k); return -1; }
    k->n = k->i = 0;
    size_t cap = 1 << 20, n = 0; uint8_t *seq = (uint8_t *)malloc(cap);
    size_t ocap = 64; uint32_t nrec = 0; uint64_t *off = (uint64_t *)malloc(ocap * 8);
    int last = 0, c = 0;
    for (;;) {
        if (!last) {                                   /* hunt for the next header */
            while ((c = kgetc(k)) >= 0 && c != '>' && c != '@') {}
            if (c < 0) break;
        }
        last = 0;
        c = kgetc(k);                                  /* header line */
        if (c < 0) break;                              /* '>' as the last byte: kseq_read returns -1 */
        while (c >= 0 && c != '\n') c = kgetc(k);
        const size_t start = n;
        if (c >= 0) {
            while ((c = kgetc(k)) >= 0 && c != '>' && c != '+' && c != '@') {
                if (c == '\n') continue;
                const size_t line0 = n;
                do {
                    if (n + 1 > cap) { cap *= 2; seq = (uint8_t *)realloc(seq, cap); }
                    seq[n++] = (uint8_t)((c > 96 && c < 123) ? c - 32 : c);
                } while ((c = kgetc(k)) >= 0 && c != '\n');
                if (n > line0 && seq[n - 1] == '\r') n--;
                if (c < 0) break;
            }
        }
        if (c == '>' || c == '@') last = c;            /* the next header's first byte is read */
        if (c == '+') {                                  /* FASTQ: skip the '+' line, then quality lines */
            int e;
            (void)kline_len(k, -1, &e);
            int bad = e < 0;                             /* no quality string */
            size_t q = 0;
            if (!bad) {
                for (;;) {
                    const int c0 = kgetc(k);
                    if (c0 < 0) break;                   /* EOF: no further line */
                    q += c0 == '\n' ? 0 : kline_len(k, c0, &e);
                    if (q >= n - start || (c0 != '\n' && e < 0)) break;
                }
                bad = q != n - start;                    /* quality of a different length */
            }
            if (bad) { n = start; break; }               /* kseq_read returns -2: record dropped, reading stops */
        }
        if (nrec + 2 > ocap) { ocap *= 2; off = (uint64_t *)realloc(off, ocap * 8); }
        off[nrec++] = start;
        if (c < 0 && !last) break;
    }
    gzclose(k->f); free(k);
    off[nrec] = n;
    *seq_out = seq; *off_out = off; *nrec_out = nrec; *len_out = n;
    return 0;
}

/* --------------------------------------------------------------- sketches */
static void sink_bottom(void *ctx, uint64_t h) { bs_try_insert((bottom_s *)ctx, h); }

/* Sketch of one genome given as records (upper-case ASCII).  out: up to s
 * ascending hashes; returns count. */
int oracle_sketch_records(const uint8_t *seq, const uint64_t *rec_off, uint32_t n_rec,
                          int k, uint32_t s, uint32_t seed, uint64_t *out, uint32_t *nout) {
    bottom_s b;
    if (bs_init(&b, s)) return -1;
    for (uint32_t r = 0; r < n_rec; r++)
        scan_record(seq + rec_off[r], rec_off[r + 1] - rec_off[r], k, seed, sink_bottom, &b);
    memcpy(out, b.heap, sizeof(uint64_t) * b.n);
    qsort(out, b.n, sizeof(uint64_t), cmp_u64);
    *nout = b.n;
    bs_free(&b);
    return 0;
}

/* Spec-literal variant used only to cross-check the heap: every hash, sort,
 * unique, first s. */
typedef struct { uint64_t *v; size_t n, cap; } vec64;
static void sink_all(void *ctx, uint64_t h) {
    vec64 *v = (vec64 *)ctx;
    if (v->n == v->cap) { v->cap = v->cap ? 2 * v->cap : 1024; v->v = (uint64_t *)realloc(v->v, 8 * v->cap); }
    v->v[v->n++] = h;
}
int oracle_sketch_records_sortuniq(const uint8_t *seq, const uint64_t *rec_off, uint32_t n_rec,
                                   int k, uint32_t s, uint32_t seed, uint64_t *out, uint32_t *nout) {
    vec64 v = {0, 0, 0};
    for (uint32_t r = 0; r < n_rec; r++)
        scan_record(seq + rec_off[r], rec_off[r + 1] - rec_off[r], k, seed, sink_all, &v);
    qsort(v.v, v.n, 8, cmp_u64);
    uint32_t m = 0;
    for (size_t i = 0; i < v.n && m < s; i++)
        if (m == 0 || out[m - 1] != v.v[i]) out[m++] = v.v[i];
    *nout = m; free(v.v);
    return 0;
}

int oracle_sketch_fasta(const char *path, int k, uint32_t s, uint32_t seed,
                        uint64_t *out, uint32_t *nout, uint64_t *length) {
    uint8_t *seq; uint64_t *off; uint32_t nrec; uint64_t len;
    if (oracle_read_fasta(path, &seq, &off, &nrec, &len)) return -1;
    int rc = oracle_sketch_records(seq, off, nrec, k, s, seed, out, nout);
    *length = len;
    free(seq); free(off);
    return rc;
}

/* Many files, one OpenMP thread per file (Mash: one `mash sketch` process per
 * genome on a p-thread pool, d_cluster.py:547-549).  out: n*s row-major. */
int oracle_sketch_fasta_many(const char **paths, uint32_t n, int k, uint32_t s, uint32_t seed,
                             uint64_t *out, uint32_t *nout, uint64_t *length, int threads) {
    int err = 0;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 1) reduction(| : err)
#endif
    for (uint32_t g = 0; g < n; g++)
        err |= oracle_sketch_fasta(paths[g], k, s, seed, out + (size_t)g * s, nout + g, length + g) != 0;
    return err ? -1 : 0;
}

/* ----------------------------------------------- synthetic genome family */
/* The bench's synthetic input: genome g of length L, one
 * record, ACGT only.  Family f = g / family_size shares an ancestor drawn
 * from a counter-based PRNG; genome g substitutes each base independently at
 * a per-genome rate from {0.1,0.5,1,2,5,10,20}%.  drep_amd/csrc generates the
 * identical sequence on device, 2-bit packed. */
static inline uint64_t splitmix64(uint64_t x) {
    x += 0x9e3779b97f4a7c15ULL;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
    return x ^ (x >> 31);
}
#define SYN_SEED_A 0xD2E9A5C31F00AB01ULL
#define SYN_SEED_M 0x5BD1E9955A11CE07ULL
#define SYN_SEED_R 0x27D4EB2F165667C5ULL
static const uint32_t syn_rate_thr[7] = {   /* rate * 2^32 */
    4294967u, 21474836u, 42949673u, 85899346u, 214748365u, 429496730u, 858993459u };

uint32_t oracle_synth_base(uint64_t seed, uint32_t g, uint32_t family_size, uint64_t p) {
    uint32_t f = g / family_size;
    uint64_t w = splitmix64((SYN_SEED_A ^ seed) ^ ((uint64_t)f << 32) ^ (p >> 5));
    uint32_t c = (uint32_t)(w >> (2 * (p & 31))) & 3u;
    uint32_t ri = (uint32_t)(splitmix64((SYN_SEED_R ^ seed) ^ g) % 7);
    uint64_t u = splitmix64((SYN_SEED_M ^ seed) ^ ((uint64_t)g << 32) ^ p);
    if ((uint32_t)(u >> 32) < syn_rate_thr[ri]) c = (c + 1 + (uint32_t)(u & 0xffffffffu) % 3u) & 3u;
    return c;
}

void oracle_synth_ascii(uint64_t seed, uint32_t g, uint32_t family_size, uint64_t L, uint8_t *out) {
    static const uint8_t asc[4] = {'A', 'C', 'G', 'T'};
    for (uint64_t p = 0; p < L; p++) out[p] = asc[oracle_synth_base(seed, g, family_size, p)];
}

/* Sketch genomes [g0, g0+n) of the synthetic family, one thread per genome. */
int oracle_sketch_synth(uint64_t seed, uint32_t g0, uint32_t n, uint32_t family_size, uint64_t L,
                        int k, uint32_t s, uint32_t hseed, uint64_t *out, uint32_t *nout, int threads) {
    int err = 0;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 1) reduction(| : err)
#endif
    for (uint32_t i = 0; i < n; i++) {
        uint8_t *buf = (uint8_t *)malloc(L ? L : 1);
        if (!buf) { err |= 1; continue; }
        oracle_synth_ascii(seed, g0 + i, family_size, L, buf);
        uint64_t off[2] = {0, L};
        err |= oracle_sketch_records(buf, off, 1, k, s, hseed, out + (size_t)i * s, nout + i) != 0;
        free(buf);
    }
    return err ? -1 : 0;
}

/* ------------------------------------------------------------------- dist */
/* Mash CommandDistance::compare / Sketch merge, per (reference, query). */
void oracle_dist_pair(const uint64_t *a, uint32_t na, const uint64_t *b, uint32_t nb,
                      uint32_t s, uint32_t *common_out, uint32_t *denom_out) {
    uint32_t i = 0, j = 0, common = 0, denom = 0;
    while (denom < s && i < na && j < nb) {
        if (a[i] < b[j]) i++;
        else if (b[j] < a[i]) j++;
        else { i++; j++; common++; }
        denom++;
    }
    if (denom < s) {
        if (i < na) { uint32_t r = na - i; denom += (s - denom < r) ? s - denom : r; }
        if (j < nb) { uint32_t r = nb - j; denom += (s - denom < r) ? s - denom : r; }
    }
    *common_out = common; *denom_out = denom;
}

/* Mash distance (double): J = common/denom; d = -ln(2J/(1+J))/k, clamped. */
double oracle_mash_distance(uint32_t common, uint32_t denom, int k) {
    if (common == denom) return 0.0;
    if (common == 0) return 1.0;
    double j = (double)common / (double)denom;
    double d = -log(2.0 * j / (1.0 + j)) / (double)k;
    return d > 1.0 ? 1.0 : d;
}

/* Condensed upper triangle, row-major over i<j (scipy squareform order).
 * Pairs for rows [r0, r1) only; out has room for exactly those pairs. */
void oracle_allpairs_rows(const uint64_t *hashes, const uint32_t *nhash, uint32_t N, uint32_t s,
                          uint32_t r0, uint32_t r1, uint16_t *common_out, uint16_t *denom_out,
                          int threads) {
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int64_t ii = r0; ii < (int64_t)r1; ii++) {
        uint64_t i = (uint64_t)ii;
        uint64_t base = i * N - i * (i + 1) / 2 - ((uint64_t)r0 * N - (uint64_t)r0 * (r0 + 1) / 2);
        for (uint64_t j = i + 1; j < N; j++) {
            uint32_t c, d;
            oracle_dist_pair(hashes + i * s, nhash[i], hashes + j * s, nhash[j], s, &c, &d);
            common_out[base + (j - i - 1)] = (uint16_t)c;
            if (denom_out) denom_out[base + (j - i - 1)] = (uint16_t)d;
        }
    }
}

/* Pairs given explicitly (used by bench.py's bounded CPU sample). */
void oracle_dist_pairs_list(const uint64_t *hashes, const uint32_t *nhash, uint32_t s,
                            const uint32_t *pi, const uint32_t *pj, uint64_t npairs,
                            uint16_t *common_out, int threads) {
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(static, 1024)
#endif
    for (int64_t t = 0; t < (int64_t)npairs; t++) {
        uint32_t c, d;
        oracle_dist_pair(hashes + (uint64_t)pi[t] * s, nhash[pi[t]],
                         hashes + (uint64_t)pj[t] * s, nhash[pj[t]], s, &c, &d);
        common_out[t] = (uint16_t)c;
    }
}

int oracle_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
