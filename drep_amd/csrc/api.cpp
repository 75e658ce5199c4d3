// api.cpp -- the extern "C" surface of libdrephip.so (include/drephip.h).
// Host glue only: argument checks, device scratch, host<->device staging,
// threads for FASTA ingest.  All sketch/dist arithmetic runs in the HIP
// kernels of sketch.hip and allpairs.hip.
#include "ctx.h"
#include "../../include/drephip.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <mutex>
#include <cstdlib>
#include <cstring>
#include <new>
#include <thread>
#include <vector>

#define DREPHIP_EXPORT extern "C" __attribute__((visibility("default")))

namespace drephip {

static thread_local std::string g_err;
void set_error(const std::string &msg) { g_err = msg; }

int scratch(drephip_ctx *ctx, const char *name, size_t bytes, void **out) {
    DevBuf &b = ctx->bufs[name];
    if (bytes == 0) bytes = 8;
    if (b.bytes < bytes) {
        const size_t want = std::max(bytes, b.bytes + b.bytes / 4);
        if (b.ptr) {
            HIPC(hipStreamSynchronize(ctx->stream));
            HIPC(hipDeviceSynchronize());
            HIPC(hipFree(b.ptr));
            b.ptr = nullptr; b.bytes = 0;
        }
        ctx->alloc_gen++;                      // invalidates contents cached in scratch
        hipError_t e = hipMalloc(&b.ptr, want);
        if (e != hipSuccess) {
            set_error(std::string("hipMalloc(") + std::to_string(want) + ") for " + name + ": " +
                      hipGetErrorString(e));
            b.ptr = nullptr;
            return DREPHIP_ERR_NOMEM;
        }
        b.bytes = want;
    }
    *out = b.ptr;
    return DREPHIP_OK;
}

int pinned_host(drephip_ctx *ctx, const char *name, size_t bytes, void **out) {
    DevBuf &b = ctx->pinned[name];
    if (bytes == 0) bytes = 8;
    if (b.bytes < bytes) {
        if (b.ptr) {
            HIPC(hipStreamSynchronize(ctx->stream));
            HIPC(hipHostFree(b.ptr));
            b.ptr = nullptr; b.bytes = 0;
        }
        const size_t want = std::max(bytes, (size_t)4096);
        hipError_t e = hipHostMalloc(&b.ptr, want, hipHostMallocDefault);
        if (e != hipSuccess) {
            set_error(std::string("hipHostMalloc for ") + name + ": " + hipGetErrorString(e));
            b.ptr = nullptr;
            return DREPHIP_ERR_NOMEM;
        }
        b.bytes = want;
    }
    *out = b.ptr;
    return DREPHIP_OK;
}

void timing_begin(drephip_ctx *ctx) {
    for (int i = 0; i < 5; i++) { ctx->kms[i] = 0; ctx->kn[i] = 0; }
    ctx->spans.clear();
    ctx->ev_used = 0;
}

static hipEvent_t next_event(drephip_ctx *ctx) {
    if (ctx->ev_used == ctx->ev_pool.size()) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        ctx->ev_pool.push_back(e);
    }
    return ctx->ev_pool[ctx->ev_used++];
}

void timing_mark(drephip_ctx *ctx, int which, hipStream_t st, bool start) {
    if (!((ctx->timing >> which) & 1u)) return;
    hipEvent_t e = next_event(ctx);
    if (!e) return;
    (void)hipEventRecord(e, st);
    if (start) ctx->spans.push_back({which, e, nullptr});
    else if (!ctx->spans.empty()) ctx->spans.back().b = e;
}

void timing_collect(drephip_ctx *ctx) {
    if (!ctx->timing) return;
    for (auto &sp : ctx->spans) {
        if (!sp.a || !sp.b) continue;
        float ms = 0;
        if (hipEventSynchronize(sp.b) == hipSuccess && hipEventElapsedTime(&ms, sp.a, sp.b) == hipSuccess) {
            ctx->kms[sp.which] += ms;
            ctx->kn[sp.which] += 1;
        }
    }
    ctx->spans.clear();
    ctx->ev_used = 0;
}

}  // namespace drephip

using namespace drephip;

#define GUARD_CTX(ctx)                                              \
    do {                                                            \
        if (!(ctx)) { set_error("null context"); return DREPHIP_ERR_ARG; } \
        HIPC(hipSetDevice((ctx)->device));                          \
    } while (0)

// Device-pointer entry points run on the caller's stream.  0 is the HIP null
// stream (also torch's default stream handle), exactly as in the HIP API, so
// work is ordered after whatever the caller queued there.
static hipStream_t pick_stream(drephip_ctx *, void *stream) { return (hipStream_t)stream; }
static void pend_release(drephip_ctx *ctx);

// A deferred sketch (drephip_sketch_device_async) owns the sketch scratch and
// its status check until drephip_sketch_wait: any other sketch call is refused
// rather than dropping that check or reusing scratch its kernels still read.
static int refuse_if_pending(drephip_ctx *ctx) {
    if (!ctx->pend.active) return DREPHIP_OK;
    set_error("a deferred sketch (drephip_sketch_device_async) is pending: call drephip_sketch_wait first");
    return DREPHIP_ERR_ARG;
}

DREPHIP_EXPORT int drephip_version(void) { return 100; }

#ifndef DREPHIP_SRC_DIGEST
#define DREPHIP_SRC_DIGEST "unknown"
#endif
#ifndef DREPHIP_BUILD_FLAGS
#define DREPHIP_BUILD_FLAGS ""
#endif
DREPHIP_EXPORT const char *drephip_build_id(void) {
    return "src=" DREPHIP_SRC_DIGEST ";arch=gfx950;extra=" DREPHIP_BUILD_FLAGS;
}

DREPHIP_EXPORT const char *drephip_last_error(void) { return g_err.c_str(); }

DREPHIP_EXPORT int drephip_device_count(int *n) {
    if (!n) { set_error("null pointer"); return DREPHIP_ERR_ARG; }
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) { *n = 0; set_error(hipGetErrorString(e)); return DREPHIP_ERR_HIP; }
    *n = c;
    return DREPHIP_OK;
}

DREPHIP_EXPORT uint32_t drephip_max_sketch(void) { return kMaxSketch; }
DREPHIP_EXPORT uint64_t drephip_tile_bases(void) { return kTile; }

DREPHIP_EXPORT uint64_t drephip_padded_bases(const uint64_t *rec_len, uint32_t n_rec) {
    return padded_span(genome_span(rec_len, n_rec));
}

DREPHIP_EXPORT int drephip_create(int device, int k, uint32_t s, uint32_t seed, drephip_ctx **out) {
    if (!out) { set_error("null out"); return DREPHIP_ERR_ARG; }
    *out = nullptr;
    if (k < 1 || k > 32) { set_error("k must be in 1..32"); return DREPHIP_ERR_ARG; }
    if (s < 1 || s > kMaxSketch) {
        set_error("sketch size must be in 1.." + std::to_string(kMaxSketch));
        return DREPHIP_ERR_UNSUPPORTED;
    }
    int n = 0;
    HIPC(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) { set_error("no such HIP device"); return DREPHIP_ERR_ARG; }
    HIPC(hipSetDevice(device));
    drephip_ctx *c = new (std::nothrow) drephip_ctx();
    if (!c) { set_error("out of host memory"); return DREPHIP_ERR_NOMEM; }
    c->device = device; c->k = k; c->s = s; c->seed = seed;
    if (const char *lp = std::getenv("DREPHIP_LINK_PATH"))      // default linkage path (tests, A/B runs)
        c->link_path = !strcmp(lp, "dense") ? DREPHIP_LINK_PATH_DENSE : !strcmp(lp, "sparse") ? DREPHIP_LINK_PATH_SPARSE
                                                                                                : DREPHIP_LINK_PATH_AUTO;
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) { delete c; set_error(hipGetErrorString(e)); return DREPHIP_ERR_HIP; }
    *out = c;
    return DREPHIP_OK;
}

DREPHIP_EXPORT int drephip_destroy(drephip_ctx *ctx) {
    if (!ctx) return DREPHIP_OK;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    // deferred calls may still be writing the pinned readback buffers
    if (ctx->pend.active && ctx->pend.done) (void)hipEventSynchronize(ctx->pend.done);
    if (ctx->apend.active && ctx->apend.ev) (void)hipEventSynchronize(ctx->apend.ev);
    for (auto &kv : ctx->bufs) if (kv.second.ptr) (void)hipFree(kv.second.ptr);
    for (auto &kv : ctx->pinned) if (kv.second.ptr) (void)hipHostFree(kv.second.ptr);
    pend_release(ctx);
    for (auto e : ctx->ev_pool) (void)hipEventDestroy(e);
    if (ctx->pend.done) (void)hipEventDestroy(ctx->pend.done);
    if (ctx->apend.ev) (void)hipEventDestroy(ctx->apend.ev);
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return DREPHIP_OK;
}

DREPHIP_EXPORT int drephip_set_timing(drephip_ctx *ctx, int kernels) {
    if (!ctx) { set_error("null context"); return DREPHIP_ERR_ARG; }
    ctx->timing = (uint32_t)kernels & 0x1Fu;
    return DREPHIP_OK;
}

DREPHIP_EXPORT int drephip_set_allpairs_path(drephip_ctx *ctx, int path, uint32_t band_cap) {
    if (!ctx) { set_error("null context"); return DREPHIP_ERR_ARG; }
    if (path < DREPHIP_AP_AUTO || path > DREPHIP_AP_MERGE) { set_error("unknown all-pairs path"); return DREPHIP_ERR_ARG; }
    if (band_cap < 1 || band_cap > 1024) { set_error("band_cap must be in 1..1024"); return DREPHIP_ERR_ARG; }
    ctx->ap_path = path;
    ctx->band_cap = band_cap;
    return DREPHIP_OK;
}

DREPHIP_EXPORT int drephip_set_allpairs_screen(drephip_ctx *ctx, int mode) {
    if (!ctx) { set_error("null context"); return DREPHIP_ERR_ARG; }
    if (mode < DREPHIP_SCREEN_AUTO || mode > DREPHIP_SCREEN_OFF) { set_error("unknown screen mode"); return DREPHIP_ERR_ARG; }
    ctx->screen = mode;
    return DREPHIP_OK;
}

DREPHIP_EXPORT int drephip_last_screen_stats(drephip_ctx *ctx, int *used, uint64_t *entries, uint64_t *runs,
                                             uint64_t *checks, uint64_t *marked, uint64_t *simple) {
    if (!ctx) { set_error("null context"); return DREPHIP_ERR_ARG; }
    const ScreenResult &r = ctx->last_screen;
    if (used) *used = r.use ? 1 : 0;
    if (entries) *entries = r.entries;
    if (runs) *runs = r.runs;
    if (checks) *checks = r.checks;
    if (marked) *marked = r.marked;
    if (simple) *simple = r.simple;
    return DREPHIP_OK;
}

DREPHIP_EXPORT int drephip_last_kernel_ms(drephip_ctx *ctx, int which, double *ms, int *launches) {
    if (!ctx || which < 0 || which > 4 || !ms) { set_error("bad argument"); return DREPHIP_ERR_ARG; }
    *ms = ctx->kms[which];
    if (launches) *launches = ctx->kn[which];
    return DREPHIP_OK;
}

DREPHIP_EXPORT int drephip_fasta_info(const char *path, int k, uint64_t *length, uint64_t *padded,
                                      uint32_t *n_records, uint64_t *n_kmers) {
    if (!path) { set_error("null path"); return DREPHIP_ERR_ARG; }
    Genome g;
    if (read_fasta(path, g)) return DREPHIP_ERR_IO;
    const uint32_t nr = (uint32_t)g.rec_len.size();
    if (length) *length = g.length;
    if (padded) *padded = padded_span(genome_span(g.rec_len.data(), nr));
    if (n_records) *n_records = nr;
    if (n_kmers) {
        uint64_t nk = 0, off = 0;
        for (uint32_t r = 0; r < nr; r++) {
            uint64_t run = 0;
            for (uint64_t i = 0; i < g.rec_len[r]; i++) {
                const uint8_t c = g.seq[off + i] & 0xDF;
                const bool ok = c == 'A' || c == 'C' || c == 'G' || c == 'T';
                run = ok ? run + 1 : 0;
                nk += run >= (uint64_t)k;
            }
            off += g.rec_len[r];
        }
        *n_kmers = nk;
    }
    return DREPHIP_OK;
}

DREPHIP_EXPORT int drephip_fasta_pack(const char *path, int k, uint32_t *codes, uint32_t *valid,
                                      uint64_t base_off, uint64_t cap_bases, uint64_t *length,
                                      uint64_t *n_kmers) {
    if (!path || !codes || !valid) { set_error("null argument"); return DREPHIP_ERR_ARG; }
    if (base_off % kTile) { set_error("base_off must be a tile multiple"); return DREPHIP_ERR_ARG; }
    Genome g;
    if (read_fasta(path, g)) return DREPHIP_ERR_IO;
    const uint32_t nr = (uint32_t)g.rec_len.size();
    const uint64_t P = padded_span(genome_span(g.rec_len.data(), nr));
    if (base_off + P > cap_bases) { set_error("packed buffer too small"); return DREPHIP_ERR_ARG; }
    const uint64_t nk = pack_records(g.seq.data(), g.rec_len.data(), nr, k, codes, valid, base_off);
    if (length) *length = g.length;
    if (n_kmers) *n_kmers = nk;
    return DREPHIP_OK;
}

// Stage a packed genome set (already laid out on the host) and sketch it.
static int sketch_packed_host(drephip_ctx *ctx, const uint32_t *codes, uint64_t n_codes, const uint32_t *valid,
                              uint64_t n_valid, const std::vector<uint64_t> &off, const std::vector<uint64_t> &pad,
                              const std::vector<uint64_t> &nk, uint64_t *hashes_out, uint32_t *nhash_out) {
    const uint32_t n = (uint32_t)off.size();
    hipStream_t st = ctx->stream;
    uint32_t *d_codes, *d_valid, *d_nhash;
    uint64_t *d_hashes;
    int rc;
    if ((rc = refuse_if_pending(ctx))) return rc;
    if ((rc = scratch(ctx, "in_codes", n_codes * 4, (void **)&d_codes))) return rc;
    if ((rc = scratch(ctx, "in_valid", n_valid * 4, (void **)&d_valid))) return rc;
    if ((rc = scratch(ctx, "out_hashes", (uint64_t)n * ctx->s * 8, (void **)&d_hashes))) return rc;
    if ((rc = scratch(ctx, "out_nhash", n * 4ull, (void **)&d_nhash))) return rc;
    HIPC(hipMemcpyAsync(d_codes, codes, n_codes * 4, hipMemcpyHostToDevice, st));
    HIPC(hipMemcpyAsync(d_valid, valid, n_valid * 4, hipMemcpyHostToDevice, st));
    timing_begin(ctx);
    rc = sketch_device_impl(ctx, d_codes, d_valid, off.data(), pad.data(), nk.data(), n, d_hashes, d_nhash, st);
    if (rc) return rc;
    timing_collect(ctx);
    HIPC(hipMemcpyAsync(hashes_out, d_hashes, (uint64_t)n * ctx->s * 8, hipMemcpyDeviceToHost, st));
    HIPC(hipMemcpyAsync(nhash_out, d_nhash, n * 4ull, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    return DREPHIP_OK;
}

template <class F>
static void parallel_for(uint32_t n, int threads, F fn) {
    int nt = threads > 0 ? threads : (int)std::thread::hardware_concurrency();
    nt = std::max(1, std::min<int>(nt, (int)n));
    std::atomic<uint32_t> next(0);
    std::vector<std::thread> pool;
    for (int t = 0; t < nt; t++)
        pool.emplace_back([&] {
            for (uint32_t i = next++; i < n; i = next++) fn(i);
        });
    for (auto &th : pool) th.join();
}

DREPHIP_EXPORT int drephip_sketch(drephip_ctx *ctx, const uint8_t *seq, const uint64_t *rec_off,
                                  uint32_t n_rec, const uint64_t *genome_rec_off, uint32_t n_genomes,
                                  uint64_t *hashes_out, uint32_t *nhash_out, uint64_t *length_out) {
    GUARD_CTX(ctx);
    if (n_genomes == 0) return DREPHIP_OK;
    if (!rec_off || !genome_rec_off || !hashes_out || !nhash_out || (!seq && n_rec && rec_off[n_rec] > 0)) {
        set_error("null argument"); return DREPHIP_ERR_ARG;
    }
    if (genome_rec_off[0] != 0 || genome_rec_off[n_genomes] != n_rec) {
        set_error("genome_rec_off must start at 0 and end at n_rec"); return DREPHIP_ERR_ARG;
    }
    std::vector<uint64_t> off(n_genomes), pad(n_genomes), nk(n_genomes), reclen(n_rec);
    for (uint32_t r = 0; r < n_rec; r++) {
        if (rec_off[r + 1] < rec_off[r]) { set_error("rec_off must be non-decreasing"); return DREPHIP_ERR_ARG; }
        reclen[r] = rec_off[r + 1] - rec_off[r];
    }
    uint64_t cur = kTile;
    for (uint32_t g = 0; g < n_genomes; g++) {
        const uint64_t r0 = genome_rec_off[g], r1 = genome_rec_off[g + 1];
        if (r1 < r0) { set_error("genome_rec_off must be non-decreasing"); return DREPHIP_ERR_ARG; }
        off[g] = cur;
        pad[g] = padded_span(genome_span(reclen.data() + r0, (uint32_t)(r1 - r0)));
        cur += pad[g];
        uint64_t L = 0;
        for (uint64_t r = r0; r < r1; r++) L += reclen[r];
        if (length_out) length_out[g] = L;
    }
    std::vector<uint32_t> codes(cur / 16, 0), valid(cur / 32, 0);
    parallel_for(n_genomes, 0, [&](uint32_t g) {
        const uint64_t r0 = genome_rec_off[g], r1 = genome_rec_off[g + 1];
        nk[g] = pack_records(seq + (r1 > r0 ? rec_off[r0] : 0), reclen.data() + r0, (uint32_t)(r1 - r0),
                             ctx->k, codes.data(), valid.data(), off[g]);
    });
    return sketch_packed_host(ctx, codes.data(), codes.size(), valid.data(), valid.size(), off, pad, nk, hashes_out,
                              nhash_out);
}

// One batch of FASTA files read and packed into pinned host memory.
struct IngestBatch {
    uint32_t g0 = 0, n = 0;
    std::vector<uint64_t> off, pad, nk, length;
    uint64_t bases = 0;                 // padded positions of the batch (codes/valid span)
    int err = 0;
    std::string msg;
    double seconds = 0;
    double read_thread_s = 0, pack_thread_s = 0;
    uint32_t overflow = 0;
};
static uint64_t ingest_batch_bases() {
    if (const char *e = getenv("DREPHIP_INGEST_BATCH_BASES")) {     // tests: force many batches
        const uint64_t v = strtoull(e, nullptr, 10);
        if (v) return v;
    }
    return 1ull << 30;                  // ~1 Gbase of sequence per batch
}

// Upper bound on a file's bases (every base is one byte of the uncompressed
// text): the size of a plain file; for a gzip file its trailer's ISIZE (the
// uncompressed size mod 2^32 of the LAST member -- exact for the usual
// single-member file; a multi-member (bgzf) file shows an ISIZE below its
// compressed size and gets the generic guess of 4x).  A wrong guess costs an
// overflow repack, never a wrong result.
static uint64_t estimate_bases(const char *path) {
    FILE *fp = fopen(path, "rb");
    if (!fp) return 0;
    uint8_t magic[2] = {0, 0};
    const size_t got = fread(magic, 1, 2, fp);
    fseek(fp, 0, SEEK_END);
    const long sz = ftell(fp);
    uint64_t est = sz > 0 ? (uint64_t)sz : 0;
    if (got == 2 && magic[0] == 0x1f && magic[1] == 0x8b && sz >= 18) {
        uint8_t t[4];
        fseek(fp, -4, SEEK_END);
        if (fread(t, 1, 4, fp) == 4) {
            const uint64_t isize = (uint64_t)t[0] | (uint64_t)t[1] << 8 | (uint64_t)t[2] << 16 | (uint64_t)t[3] << 24;
            est = isize >= (uint64_t)sz ? isize : 4 * (uint64_t)sz;
        }
    }
    fclose(fp);
    return est;
}

// Grow a pinned slot keeping its first `keep_c` / `keep_v` words.
static int grow_pinned(PinnedSlot &slot, size_t cb, size_t vb, size_t keep_c, size_t keep_v) {
    PinnedSlot n;
    if (n.reserve(cb, vb)) return -1;
    memcpy(n.codes, slot.codes, keep_c * 4);
    memcpy(n.valid, slot.valid, keep_v * 4);
    std::swap(slot.codes, n.codes); std::swap(slot.codes_bytes, n.codes_bytes);
    std::swap(slot.valid, n.valid); std::swap(slot.valid_bytes, n.valid_bytes);
    return 0;                          // n frees the old buffers
}

// One batch: files [g0, ...) chosen by their estimated bases until the batch
// holds >= target, each given a tile-aligned region of its estimated padded
// span; then ONE pass over the batch's files on `threads` workers (dynamic
// scheduling): a worker reads + parses a file into its own reused buffer and
// packs it straight into the pinned batch while the sequence is cache-hot (a
// genome whose real span outgrew its estimate is kept and packed after the
// pass, at the end of the batch).  Regions are zeroed by their worker; the
// slack between a genome's padded span and its region stays zero and no tile
// covers it.
static void produce_batch(const char *const *paths, uint32_t g0, uint32_t n_genomes, int threads, int k,
                          uint64_t target, PinnedSlot &slot, IngestBatch &B, int device) {
    const auto t0 = std::chrono::steady_clock::now();
    (void)hipSetDevice(device);         // the pinned batch belongs with the context's device
    B = IngestBatch();
    B.g0 = g0;
    std::vector<uint64_t> reserved;
    uint64_t est_total = 0;
    uint32_t g1 = g0;
    while (g1 < n_genomes && (g1 == g0 || est_total < target)) {
        const uint64_t e = estimate_bases(paths[g1]);
        reserved.push_back(padded_span(e));
        est_total += e;
        g1++;
    }
    const uint32_t n = g1 - g0;
    B.n = n;
    B.off.resize(n); B.pad.resize(n); B.nk.resize(n); B.length.resize(n);
    uint64_t cur = kTile;
    for (uint32_t i = 0; i < n; i++) { B.off[i] = cur; cur += reserved[i]; }
    if (slot.reserve(cur / 16 * 4, cur / 32 * 4)) {
        B.err = DREPHIP_ERR_NOMEM; B.msg = "hipHostMalloc of the pinned ingest batch failed"; return;
    }
    memset(slot.codes, 0, kTile / 16 * 4);
    memset(slot.valid, 0, kTile / 32 * 4);
    std::vector<int> err(n, 0);
    std::vector<std::string> msg(n);
    std::vector<Genome> overflow(n);                 // genomes whose span outgrew the estimate (rare)
    std::vector<char> over(n, 0);
    std::vector<Genome> work(std::max(1, threads > 0 ? threads : (int)std::thread::hardware_concurrency()));
    std::atomic<uint32_t> next(0);
    std::vector<double> t_read(work.size(), 0.0), t_pack(work.size(), 0.0);
    auto worker = [&](uint32_t w) {
        Genome &g = work[w];                         // reused: no fresh pages per file
        for (uint32_t i = next++; i < n; i = next++) {
            const auto r0 = std::chrono::steady_clock::now();
            const int rr = read_fasta(paths[g0 + i], g);
            const auto r1 = std::chrono::steady_clock::now();
            t_read[w] += std::chrono::duration<double>(r1 - r0).count();
            if (rr) { err[i] = DREPHIP_ERR_IO; msg[i] = drephip_last_error(); continue; }
            const uint64_t P = padded_span(genome_span(g.rec_len.data(), (uint32_t)g.rec_len.size()));
            B.length[i] = g.length;
            B.pad[i] = P;
            if (P > reserved[i]) { std::swap(overflow[i], g); over[i] = 1; continue; }
            memset(slot.codes + B.off[i] / 16, 0, reserved[i] / 16 * 4);
            memset(slot.valid + B.off[i] / 32, 0, reserved[i] / 32 * 4);
            B.nk[i] = pack_records(g.seq.data(), g.rec_len.data(), (uint32_t)g.rec_len.size(), k, slot.codes,
                                   slot.valid, B.off[i]);
            t_pack[w] += std::chrono::duration<double>(std::chrono::steady_clock::now() - r1).count();
        }
    };
    const uint32_t nt = (uint32_t)std::min<size_t>(work.size(), n);
    std::vector<std::thread> pool;
    for (uint32_t w = 1; w < nt; w++) pool.emplace_back(worker, w);
    worker(0);
    for (auto &th : pool) th.join();
    for (uint32_t i = 0; i < n; i++)
        if (err[i]) { B.err = err[i]; B.msg = msg[i]; return; }
    for (size_t w = 0; w < work.size(); w++) { B.read_thread_s += t_read[w]; B.pack_thread_s += t_pack[w]; }
    uint64_t end = cur;
    for (uint32_t i = 0; i < n; i++) if (over[i]) { end += B.pad[i]; B.overflow++; }
    if (end > cur) {
        if (grow_pinned(slot, end / 16 * 4, end / 32 * 4, cur / 16, cur / 32)) {
            B.err = DREPHIP_ERR_NOMEM; B.msg = "hipHostMalloc of the pinned ingest batch failed"; return;
        }
        uint64_t at = cur;
        for (uint32_t i = 0; i < n; i++) {
            if (!over[i]) continue;
            const Genome &g = overflow[i];
            B.off[i] = at;
            memset(slot.codes + at / 16, 0, B.pad[i] / 16 * 4);
            memset(slot.valid + at / 32, 0, B.pad[i] / 32 * 4);
            B.nk[i] = pack_records(g.seq.data(), g.rec_len.data(), (uint32_t)g.rec_len.size(), k, slot.codes,
                                   slot.valid, at);
            at += B.pad[i];
        }
    }
    B.bases = end;
    B.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// Ingest pipeline: one producer thread reads + packs batch i+1 (on `threads`
// workers, into the other of two pinned buffers) while this thread copies
// batch i to the GPU and sketches it -- the GPU work hides behind the host
// ingest, which is the slower side by an order of magnitude.  The producer
// lives for the whole call (a thread per batch paid the HIP runtime's
// per-thread setup and teardown, ~30 ms, on every batch).
DREPHIP_EXPORT int drephip_sketch_files(drephip_ctx *ctx, const char *const *paths, uint32_t n_genomes,
                                        int threads, uint64_t *hashes_out, uint32_t *nhash_out,
                                        uint64_t *length_out) {
    GUARD_CTX(ctx);
    ctx->ingest = IngestStats();
    if (n_genomes == 0) return DREPHIP_OK;
    if (!paths || !hashes_out || !nhash_out) { set_error("null argument"); return DREPHIP_ERR_ARG; }
    int rc;
    if ((rc = refuse_if_pending(ctx))) return rc;
    const auto t0 = std::chrono::steady_clock::now();
    const uint64_t target = ingest_batch_bases();
    PinnedSlot *slots = ctx->ingest_slots;          // kept across calls: pinned allocation is slow
    IngestBatch B[2];
    const int k = ctx->k;
    std::mutex mu;
    std::condition_variable cv;
    uint32_t produced = 0, consumed = 0;            // batches handed over / released
    bool stop = false;
    std::thread producer([&] {
        uint32_t g = 0;
        for (uint32_t i = 0; g < n_genomes; i++) {
            {   // slot i & 1 is free once batch i - 2 has been consumed
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop || consumed + 2 > i; });
                if (stop) return;
            }
            produce_batch(paths, g, n_genomes, threads, k, target, slots[i & 1], B[i & 1], ctx->device);
            const bool last = B[i & 1].err || g + B[i & 1].n >= n_genomes;
            g += B[i & 1].n;
            {
                std::lock_guard<std::mutex> lk(mu);
                produced = i + 1;
            }
            cv.notify_all();
            if (last) return;
        }
    });
    rc = DREPHIP_OK;
    for (uint32_t b = 0;; b++) {
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return produced > b; });
        }
        IngestBatch &cur = B[b & 1];
        if (cur.err) { set_error(cur.msg); rc = cur.err; break; }
        const bool more = cur.g0 + cur.n < n_genomes;
        const auto g0 = std::chrono::steady_clock::now();
        if (length_out) std::copy(cur.length.begin(), cur.length.end(), length_out + cur.g0);
        rc = sketch_packed_host(ctx, slots[b & 1].codes, cur.bases / 16, slots[b & 1].valid, cur.bases / 32, cur.off,
                                cur.pad, cur.nk, hashes_out + (uint64_t)cur.g0 * ctx->s, nhash_out + cur.g0);
        ctx->ingest.gpu_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - g0).count();
        ctx->ingest.produce_s += cur.seconds;
        ctx->ingest.read_thread_s += cur.read_thread_s;
        ctx->ingest.pack_thread_s += cur.pack_thread_s;
        ctx->ingest.overflow += cur.overflow;
        ctx->ingest.batches++;
        {
            std::lock_guard<std::mutex> lk(mu);
            consumed = b + 1;
        }
        cv.notify_all();
        if (rc || !more) break;
    }
    {
        std::lock_guard<std::mutex> lk(mu);
        stop = true;                                // a producer waiting for a slot ends
    }
    cv.notify_all();
    producer.join();
    ctx->ingest.wall_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

DREPHIP_EXPORT int drephip_last_ingest_stats(drephip_ctx *ctx, double *produce_s, double *gpu_s, double *wall_s,
                                             uint32_t *batches) {
    if (!ctx) { set_error("null context"); return DREPHIP_ERR_ARG; }
    if (produce_s) *produce_s = ctx->ingest.produce_s;
    if (gpu_s) *gpu_s = ctx->ingest.gpu_s;
    if (wall_s) *wall_s = ctx->ingest.wall_s;
    if (batches) *batches = ctx->ingest.batches;
    return DREPHIP_OK;
}

DREPHIP_EXPORT int drephip_last_ingest_phases(drephip_ctx *ctx, double *read_thread_s, double *pack_thread_s,
                                              uint32_t *overflow) {
    if (!ctx) { set_error("null context"); return DREPHIP_ERR_ARG; }
    if (read_thread_s) *read_thread_s = ctx->ingest.read_thread_s;
    if (pack_thread_s) *pack_thread_s = ctx->ingest.pack_thread_s;
    if (overflow) *overflow = ctx->ingest.overflow;
    return DREPHIP_OK;
}

DREPHIP_EXPORT int drephip_sketch_device(drephip_ctx *ctx, const uint32_t *d_codes, const uint32_t *d_valid,
                                         const uint64_t *h_base_off, const uint64_t *h_padded,
                                         const uint64_t *h_nkmers, uint32_t n_genomes, uint64_t *d_hashes,
                                         uint32_t *d_nhash, void *stream) {
    GUARD_CTX(ctx);
    if (n_genomes == 0) return DREPHIP_OK;
    if (!d_codes || !d_valid || !h_base_off || !h_padded || !h_nkmers || !d_hashes || !d_nhash) {
        set_error("null argument"); return DREPHIP_ERR_ARG;
    }
    int rc;
    if ((rc = refuse_if_pending(ctx))) return rc;
    hipStream_t st = pick_stream(ctx, stream);
    timing_begin(ctx);
    rc = sketch_device_impl(ctx, d_codes, d_valid, h_base_off, h_padded, h_nkmers, n_genomes, d_hashes,
                            d_nhash, st);
    if (rc) return rc;
    timing_collect(ctx);
    return DREPHIP_OK;
}

// Drop a deferred sketch's bookkeeping: its timing events go back to the pool.
static void pend_release(drephip_ctx *ctx) {
    auto &p = ctx->pend;
    for (hipEvent_t e : p.events) ctx->ev_pool.push_back(e);
    p.events.clear();
    p.spans.clear();
    p.active = false;
}

DREPHIP_EXPORT int drephip_sketch_device_async(drephip_ctx *ctx, const uint32_t *d_codes, const uint32_t *d_valid,
                                               const uint64_t *h_base_off, const uint64_t *h_padded,
                                               const uint64_t *h_nkmers, uint32_t n_genomes, uint64_t *d_hashes,
                                               uint32_t *d_nhash, void *stream) {
    GUARD_CTX(ctx);
    int rc;
    if ((rc = refuse_if_pending(ctx))) return rc;
    if (n_genomes == 0) return DREPHIP_OK;
    if (!d_codes || !d_valid || !h_base_off || !h_padded || !h_nkmers || !d_hashes || !d_nhash) {
        set_error("null argument"); return DREPHIP_ERR_ARG;
    }
    hipStream_t st = pick_stream(ctx, stream);
    timing_begin(ctx);
    rc = sketch_device_impl(ctx, d_codes, d_valid, h_base_off, h_padded, h_nkmers, n_genomes, d_hashes,
                            d_nhash, st, true);
    if (rc) { ctx->pend.active = false; return rc; }
    // the queued kernels' events leave the pool until drephip_sketch_wait reads them
    auto &p = ctx->pend;
    p.spans.swap(ctx->spans);
    p.events.assign(ctx->ev_pool.begin(), ctx->ev_pool.begin() + ctx->ev_used);
    ctx->ev_pool.erase(ctx->ev_pool.begin(), ctx->ev_pool.begin() + ctx->ev_used);
    ctx->ev_used = 0;
    return DREPHIP_OK;
}

DREPHIP_EXPORT int drephip_sketch_wait(drephip_ctx *ctx, int *redone) {
    GUARD_CTX(ctx);
    if (redone) *redone = 0;
    auto &p = ctx->pend;
    if (!p.active) return DREPHIP_OK;
    HIPC(hipEventSynchronize(p.done));                 // the status copy (not what was queued after it)
    double kms[2] = {0, 0};
    int kn[2] = {0, 0};
    for (auto &sp : p.spans) {
        float ms = 0;
        if (sp.a && sp.b && sp.which < 2 && hipEventElapsedTime(&ms, sp.a, sp.b) == hipSuccess) {
            kms[sp.which] += ms;
            kn[sp.which] += 1;
        }
    }
    bool ok = true;
    for (uint32_t g = 0; g < p.n; g++) ok &= p.h_status[g] == 0;   // ST_OK
    pend_release(ctx);
    if (ok) {
        for (int w = 0; w < 2; w++) { ctx->kms[w] = kms[w]; ctx->kn[w] = kn[w]; }
        return DREPHIP_OK;
    }
    // a genome needs another threshold round: rerun the whole call synchronously
    // (finalize left every set empty, so this starts from a clean state)
    const auto off = p.off, pad = p.pad, nk = p.nk;
    timing_begin(ctx);
    int rc = sketch_device_impl(ctx, p.d_codes, p.d_valid, off.data(), pad.data(), nk.data(), p.n, p.d_hashes,
                                p.d_nhash, p.st);
    if (rc) return rc;
    timing_collect(ctx);
    if (redone) *redone = 1;
    return DREPHIP_OK;
}

DREPHIP_EXPORT int drephip_synth_device(drephip_ctx *ctx, uint64_t seed, uint32_t g0, uint32_t n,
                                        uint32_t family_size, uint64_t L, uint32_t *d_codes, uint32_t *d_valid,
                                        void *stream) {
    GUARD_CTX(ctx);
    if (!d_codes || !d_valid) { set_error("null argument"); return DREPHIP_ERR_ARG; }
    return synth_device_impl(ctx, seed, g0, n, family_size, L, d_codes, d_valid, pick_stream(ctx, stream));
}

DREPHIP_EXPORT int drephip_allpairs_device(drephip_ctx *ctx, const uint64_t *d_hashes, const uint32_t *d_nhash,
                                           uint32_t N, uint32_t row0, uint32_t row1, uint16_t *d_common,
                                           uint16_t *d_denom, void *stream) {
    GUARD_CTX(ctx);
    if (!d_hashes || !d_nhash || !d_common) { set_error("null argument"); return DREPHIP_ERR_ARG; }
    timing_begin(ctx);
    int rc = allpairs_device_impl(ctx, d_hashes, d_nhash, N, row0, row1, d_common, d_denom,
                                  pick_stream(ctx, stream), false);
    if (rc) return rc;
    timing_collect(ctx);
    return DREPHIP_OK;
}

DREPHIP_EXPORT int drephip_allpairs_device_async(drephip_ctx *ctx, const uint64_t *d_hashes,
                                                 const uint32_t *d_nhash, uint32_t N, uint32_t row0,
                                                 uint32_t row1, uint16_t *d_common, uint16_t *d_denom,
                                                 void *stream) {
    GUARD_CTX(ctx);
    if (!d_hashes || !d_nhash || !d_common) { set_error("null argument"); return DREPHIP_ERR_ARG; }
    int rc = allpairs_wait_impl(ctx);                  // an earlier call's check comes first
    if (rc) return rc;
    timing_begin(ctx);
    rc = allpairs_device_impl(ctx, d_hashes, d_nhash, N, row0, row1, d_common, d_denom,
                              pick_stream(ctx, stream), false, true);
    if (rc) { ctx->apend.active = false; return rc; }
    if (!ctx->apend.active) timing_collect(ctx);      // the call completed synchronously
    return DREPHIP_OK;
}

DREPHIP_EXPORT int drephip_allpairs_wait(drephip_ctx *ctx) {
    GUARD_CTX(ctx);
    return allpairs_wait_impl(ctx);
}

// ------------------------------------------------------------ sharded screen
DREPHIP_EXPORT int drephip_screen_geometry(drephip_ctx *ctx, uint32_t *rows_per_tile) {
    if (!ctx || !rows_per_tile) { set_error("null argument"); return DREPHIP_ERR_ARG; }
    uint32_t R;
    int path;
    int rc = allpairs_geometry(ctx, &R, &path);
    if (rc) return rc;
    *rows_per_tile = R;
    return DREPHIP_OK;
}

DREPHIP_EXPORT int drephip_screen_part(drephip_ctx *ctx, const uint64_t *d_hashes, const uint32_t *d_nhash,
                                       uint32_t N, uint32_t part, uint32_t nparts, uint64_t *checks,
                                       uint32_t *n_cells, uint32_t *n_records, void *stream) {
    GUARD_CTX(ctx);
    if (!d_hashes || !d_nhash || !checks || !n_cells || !n_records) { set_error("null argument"); return DREPHIP_ERR_ARG; }
    if (nparts == 0 || part >= nparts) { set_error("part must be below nparts"); return DREPHIP_ERR_ARG; }
    if (N < 2) { set_error("the screen needs N >= 2"); return DREPHIP_ERR_ARG; }
    if (ctx->apend.active) {
        int rc = allpairs_wait_impl(ctx);
        if (rc) return rc;
    }
    uint32_t R;
    int path;
    int rc = allpairs_geometry(ctx, &R, &path);
    if (rc) return rc;
    timing_begin(ctx);
    rc = screen_part_impl(ctx, d_hashes, d_nhash, N, R, part, nparts, pick_stream(ctx, stream), checks, n_cells,
                          n_records);
    if (rc) return rc;
    timing_collect(ctx);
    return DREPHIP_OK;
}

DREPHIP_EXPORT int drephip_screen_part_copy(drephip_ctx *ctx, uint32_t *d_cells, uint32_t *d_records, void *stream) {
    GUARD_CTX(ctx);
    const PartResult &p = ctx->part;
    if (!p.valid) { set_error("no screen part to copy (drephip_screen_part first)"); return DREPHIP_ERR_ARG; }
    if ((p.ncells && !d_cells) || (p.nrec && !d_records)) { set_error("null argument"); return DREPHIP_ERR_ARG; }
    hipStream_t st = pick_stream(ctx, stream);
    if (p.ncells) HIPC(hipMemcpyAsync(d_cells, p.cells, (uint64_t)p.ncells * 16, hipMemcpyDeviceToDevice, st));
    if (p.nrec) HIPC(hipMemcpyAsync(d_records, p.rec, (uint64_t)p.nrec * 16, hipMemcpyDeviceToDevice, st));
    HIPC(hipStreamSynchronize(st));
    return DREPHIP_OK;
}

DREPHIP_EXPORT int drephip_screen_worth(drephip_ctx *ctx, uint32_t N, uint64_t checks, int *applies, int *use) {
    if (!ctx || !use) { set_error("null argument"); return DREPHIP_ERR_ARG; }
    const bool ap = screen_applies(ctx, N);
    if (applies) *applies = ap ? 1 : 0;
    *use = ap && (screen_mode(ctx) == DREPHIP_SCREEN_ON || screen_worth(N, ctx->s, checks)) ? 1 : 0;
    return DREPHIP_OK;
}

DREPHIP_EXPORT int drephip_allpairs_device_marked(drephip_ctx *ctx, const uint64_t *d_hashes, const uint32_t *d_nhash,
                                                  uint32_t N, uint32_t row0, uint32_t row1, uint16_t *d_common,
                                                  uint16_t *d_denom, const uint32_t *d_cells, uint64_t n_cells,
                                                  const uint32_t *d_records, uint64_t n_records, void *stream) {
    GUARD_CTX(ctx);
    if (!d_hashes || !d_nhash || !d_common || (n_cells && !d_cells) || (n_records && !d_records)) {
        set_error("null argument");
        return DREPHIP_ERR_ARG;
    }
    if ((uint64_t)N * ctx->s >= (1ull << 32)) { set_error("the screen needs N x s < 2^32"); return DREPHIP_ERR_UNSUPPORTED; }
    if (ctx->ap_path == DREPHIP_AP_MERGE) { set_error("marks need the table or band path"); return DREPHIP_ERR_ARG; }
    timing_begin(ctx);
    ctx->ext = ExtMarks{true, (const uint4 *)d_cells, n_cells, (const uint4 *)d_records, n_records};
    int rc = allpairs_device_impl(ctx, d_hashes, d_nhash, N, row0, row1, d_common, d_denom, pick_stream(ctx, stream),
                                  false);
    ctx->ext = ExtMarks{};
    if (rc) return rc;
    timing_collect(ctx);
    return DREPHIP_OK;
}

DREPHIP_EXPORT int drephip_allpairs_merge_device(drephip_ctx *ctx, const uint64_t *d_hashes,
                                                 const uint32_t *d_nhash, uint32_t N, uint32_t row0,
                                                 uint32_t row1, uint16_t *d_common, uint16_t *d_denom,
                                                 void *stream) {
    GUARD_CTX(ctx);
    if (!d_hashes || !d_nhash || !d_common) { set_error("null argument"); return DREPHIP_ERR_ARG; }
    timing_begin(ctx);
    int rc = allpairs_device_impl(ctx, d_hashes, d_nhash, N, row0, row1, d_common, d_denom,
                                  pick_stream(ctx, stream), true);
    if (rc) return rc;
    timing_collect(ctx);
    return DREPHIP_OK;
}

// Host-buffer all-pairs over rows [row0, row1): stage the sketch matrix, run
// the kernels on the context's stream, copy the condensed segment back.
static int allpairs_host_rows(drephip_ctx *ctx, const uint64_t *hashes, const uint32_t *nhash, uint32_t N,
                              uint32_t row0, uint32_t row1, uint16_t *common_out, uint16_t *denom_out) {
    if (!hashes || !nhash || !common_out) { set_error("null argument"); return DREPHIP_ERR_ARG; }
    if (row1 > N) row1 = N;
    if (N < 2 || row0 >= row1 || row0 >= N - 1) return DREPHIP_OK;
    for (uint32_t i = 0; i < N; i++) {                    // the kernels read rows past nhash: must be padding
        if (nhash[i] > ctx->s) { set_error("nhash[i] > s"); return DREPHIP_ERR_ARG; }
        const uint64_t *row = hashes + (uint64_t)i * ctx->s;
        for (uint32_t j = nhash[i]; j < ctx->s; j++)
            if (row[j] != ~0ull) { set_error("sketch rows must be UINT64_MAX past nhash[i]"); return DREPHIP_ERR_ARG; }
    }
    auto start = [&](uint64_t i) { return i * N - i * (i + 1) / 2; };
    const uint64_t npairs = start(std::min(row1, N - 1)) - start(row0);
    hipStream_t st = ctx->stream;
    uint64_t *d_h;
    uint32_t *d_n;
    uint16_t *d_c, *d_d = nullptr;
    int rc;
    if ((rc = scratch(ctx, "ap_in_h", (uint64_t)N * ctx->s * 8, (void **)&d_h))) return rc;
    if ((rc = scratch(ctx, "ap_in_n", N * 4ull, (void **)&d_n))) return rc;
    if ((rc = scratch(ctx, "ap_out_c", npairs * 2, (void **)&d_c))) return rc;
    if (denom_out && (rc = scratch(ctx, "ap_out_d", npairs * 2, (void **)&d_d))) return rc;
    HIPC(hipMemcpyAsync(d_h, hashes, (uint64_t)N * ctx->s * 8, hipMemcpyHostToDevice, st));
    HIPC(hipMemcpyAsync(d_n, nhash, N * 4ull, hipMemcpyHostToDevice, st));
    timing_begin(ctx);
    rc = allpairs_device_impl(ctx, d_h, d_n, N, row0, row1, d_c, d_d, st, false);
    if (rc) return rc;
    timing_collect(ctx);
    HIPC(hipMemcpyAsync(common_out, d_c, npairs * 2, hipMemcpyDeviceToHost, st));
    if (denom_out) HIPC(hipMemcpyAsync(denom_out, d_d, npairs * 2, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    return DREPHIP_OK;
}

DREPHIP_EXPORT int drephip_allpairs(drephip_ctx *ctx, const uint64_t *hashes, const uint32_t *nhash, uint32_t N,
                                    uint16_t *common_out, uint16_t *denom_out) {
    GUARD_CTX(ctx);
    return allpairs_host_rows(ctx, hashes, nhash, N, 0, N, common_out, denom_out);
}

DREPHIP_EXPORT int drephip_allpairs_rows(drephip_ctx *ctx, const uint64_t *hashes, const uint32_t *nhash, uint32_t N,
                                         uint32_t row0, uint32_t row1, uint16_t *common_out, uint16_t *denom_out) {
    GUARD_CTX(ctx);
    return allpairs_host_rows(ctx, hashes, nhash, N, row0, row1, common_out, denom_out);
}

DREPHIP_EXPORT int drephip_distance_lut(int k, uint32_t denom, double *lut) {
    if (!lut || k < 1 || denom == 0) { set_error("bad argument"); return DREPHIP_ERR_ARG; }
    for (uint32_t c = 0; c <= denom; c++) {
        double d;
        if (c == denom) d = 0.0;
        else if (c == 0) d = 1.0;
        else {
            const double j = (double)c / (double)denom;
            d = -std::log(2.0 * j / (1.0 + j)) / (double)k;
            if (d > 1.0) d = 1.0;
        }
        lut[c] = d;
    }
    return DREPHIP_OK;
}

// Sparse linkage limits.  The automatic choice takes the sparse path only
// where it beats the dense GPU chain: a step there scans one row of the top's
// component on the host (~1 us per 1000 members) against ~6 us per GPU step,
// so the largest component may hold 4096 members (DREPHIP_LINK_SPARSE_MAXCOMP)
// and the matrices 2^28 cells (2 GB; DREPHIP_LINK_SPARSE_CELLS); the pair list
// is first counted on the device and not read back beyond 32 pairs per genome
// (+2^20).  Mash data at s = 1000 has a few random shared hashes per 1000
// unrelated pairs (two 5 Mbp genomes share ~6 random 21-mers), so beyond a few
// thousand genomes everything is one component and the dense path runs.  An
// explicit sparse request (drephip_set_linkage_path / drephip_linkage_sparse)
// allows 2^31 cells and any component size.
constexpr uint64_t kSparseMaxCells = 1ull << 31;      // 16 GB
constexpr uint64_t kSparseMaxPairs = 1ull << 26;      // device pair list: 768 MB

static uint64_t env_u64(const char *name, uint64_t dflt) {
    if (const char *e = std::getenv(name)) return std::strtoull(e, nullptr, 10);
    return dflt;
}
static uint64_t sparse_cells(const drephip_ctx *ctx) {
    return ctx->link_path == DREPHIP_LINK_PATH_SPARSE ? kSparseMaxCells : env_u64("DREPHIP_LINK_SPARSE_CELLS", 1ull << 28);
}
static uint32_t sparse_maxcomp(const drephip_ctx *ctx) {
    return ctx->link_path == DREPHIP_LINK_PATH_SPARSE ? 0xFFFFFFFFu
                                                      : (uint32_t)env_u64("DREPHIP_LINK_SPARSE_MAXCOMP", 4096);
}
static uint64_t sparse_pair_cap(const drephip_ctx *ctx, uint32_t n) {
    const uint64_t all = (uint64_t)n * (n - 1) / 2;
    const uint64_t cap = ctx->link_path == DREPHIP_LINK_PATH_SPARSE ? kSparseMaxPairs
                                                                    : std::min<uint64_t>(kSparseMaxPairs, 32ull * n + (1ull << 20));
    return std::min(all, cap);
}

DREPHIP_EXPORT int drephip_set_linkage_path(drephip_ctx *ctx, int path) {
    GUARD_CTX(ctx);
    if (path < DREPHIP_LINK_PATH_AUTO || path > DREPHIP_LINK_PATH_SPARSE) { set_error("bad linkage path"); return DREPHIP_ERR_ARG; }
    ctx->link_path = path;
    return DREPHIP_OK;
}

DREPHIP_EXPORT int drephip_linkage_sparse(uint32_t n, uint64_t npairs, const uint32_t *i, const uint32_t *j,
                                          const double *v, int method, double *Z) {
    if (n < 2) return DREPHIP_OK;
    if (!Z || (npairs && (!i || !j || !v))) { set_error("null argument"); return DREPHIP_ERR_ARG; }
    // components too large for their matrices: the sparse-row chain
    return linkage_sparse_impl(n, npairs, i, j, v, method, kSparseMaxCells, 0xFFFFFFFFu, Z, nullptr, 1);
}

// the sparse path from a host condensed vector: the pairs below 1.0 when no
// value exceeds 1.0; returns 1 when it produced Z, 0 when the dense path must run
static int linkage_condensed_sparse(drephip_ctx *ctx, const double *y, uint32_t n, int method, double *Z, int *rc) {
    *rc = DREPHIP_OK;
    if (ctx->link_path == DREPHIP_LINK_PATH_DENSE) return 0;
    const double t0 = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
    // the pairs below 1.0, scanned by host threads over row ranges of equal
    // pair counts; any value above 1.0 (or NaN) means no sparse form, more
    // pairs than the cap means the dense path
    const uint64_t np_all = (uint64_t)n * (n - 1) / 2, cap = sparse_pair_cap(ctx, n);
    const unsigned T = host_threads();
    std::vector<uint32_t> rb(T + 1, n - 1);
    rb[0] = 0;
    for (unsigned k = 1; k < T; k++) {             // first row whose pairs start at or after k/T of all
        const uint64_t target = np_all * k / T;
        uint32_t lo = rb[k - 1], hi = n - 1;
        while (lo < hi) {
            const uint32_t mid = lo + (hi - lo) / 2;
            if ((uint64_t)mid * n - (uint64_t)mid * (mid + 1) / 2 < target) lo = mid + 1; else hi = mid;
        }
        rb[k] = lo;
    }
    std::vector<std::vector<uint32_t>> qi(T), qj(T);
    std::vector<std::vector<double>> qv(T);
    std::atomic<int> above(0);
    std::atomic<uint64_t> found(0);
    {
        std::vector<std::thread> pool;
        for (unsigned k = 0; k < T; k++)
            pool.emplace_back([&, k] {
                uint64_t t = (uint64_t)rb[k] * n - (uint64_t)rb[k] * (rb[k] + 1) / 2;
                for (uint32_t a = rb[k]; a < rb[k + 1] && !above.load(std::memory_order_relaxed); a++) {
                    uint64_t local = 0;
                    for (uint32_t b = a + 1; b < n; b++, t++) {
                        const double d = y[t];
                        // above 1.0, NaN or negative: no sparse form (scipy takes negative
                        // values; the dense path does too)
                        if (!(d <= 1.0) || d < 0.0) { above = 1; return; }
                        if (d < 1.0) { qi[k].push_back(a); qj[k].push_back(b); qv[k].push_back(d); local++; }
                    }
                    if (found.fetch_add(local) + local > cap) return;     // dense path; stop early
                }
            });
        for (auto &th : pool) th.join();
    }
    if (above) {
        if (ctx->link_path == DREPHIP_LINK_PATH_SPARSE) { set_error("sparse linkage: a distance above 1.0, below 0 or NaN"); *rc = DREPHIP_ERR_ARG; }
        return 0;
    }
    if (found.load() > cap) {
        if (ctx->link_path == DREPHIP_LINK_PATH_SPARSE) { set_error("sparse linkage: more pairs below 1.0 than the pair list holds"); *rc = DREPHIP_ERR_UNSUPPORTED; }
        return 0;
    }
    std::vector<uint32_t> pi, pj;
    std::vector<double> pv;
    pi.reserve(found.load()); pj.reserve(found.load()); pv.reserve(found.load());
    for (unsigned k = 0; k < T; k++) {
        pi.insert(pi.end(), qi[k].begin(), qi[k].end());
        pj.insert(pj.end(), qj[k].begin(), qj[k].end());
        pv.insert(pv.end(), qv[k].begin(), qv[k].end());
    }
    const double t1 = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
    const int r = linkage_sparse_impl(n, pi.size(), pi.data(), pj.data(), pv.data(), method, sparse_cells(ctx),
                                      sparse_maxcomp(ctx), Z, &ctx->link.sp,
                                      ctx->link_path == DREPHIP_LINK_PATH_SPARSE ? 1 : 0);
    if (r == DREPHIP_ERR_UNSUPPORTED && ctx->link_path != DREPHIP_LINK_PATH_SPARSE) return 0;
    if (r) { *rc = r; return 0; }
    ctx->link.sparse = 1;
    ctx->link.matrix_s = t1 - t0;
    ctx->link.chain_s = ctx->link.sp.setup_s + ctx->link.sp.chain_s;
    ctx->link.finish_s = ctx->link.sp.finish_s;
    return 1;
}

DREPHIP_EXPORT int drephip_linkage(drephip_ctx *ctx, const double *y, uint32_t n, int method, double *Z) {
    GUARD_CTX(ctx);
    if (n < 2) return DREPHIP_OK;
    if (!y || !Z) { set_error("null argument"); return DREPHIP_ERR_ARG; }
    if (n > 200000) { set_error("linkage supports n <= 200000 (n x n f64 matrix in HBM)"); return DREPHIP_ERR_UNSUPPORTED; }
    timing_begin(ctx);
    ctx->link = LinkStats{};
    const auto t0 = std::chrono::steady_clock::now();
    int rc;
    if (!linkage_condensed_sparse(ctx, y, n, method, Z, &rc)) {
        if (rc) return rc;
        double *d_D;
        rc = dist_from_condensed_impl(ctx, y, n, &d_D, ctx->stream);
        if (rc) return rc;
        rc = linkage_device_impl(ctx, d_D, n, method, Z, ctx->stream);
        if (rc) return rc;
    }
    timing_collect(ctx);
    ctx->link.wall_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return DREPHIP_OK;
}

DREPHIP_EXPORT int drephip_linkage_square(drephip_ctx *ctx, const float *M, uint32_t n, int method, double *Z) {
    GUARD_CTX(ctx);
    if (n < 2) return DREPHIP_OK;
    if (!M || !Z) { set_error("null argument"); return DREPHIP_ERR_ARG; }
    if (n > 200000) { set_error("linkage supports n <= 200000 (n x n f64 matrix in HBM)"); return DREPHIP_ERR_UNSUPPORTED; }
    if (method != DREPHIP_LINK_SINGLE && method != DREPHIP_LINK_COMPLETE && method != DREPHIP_LINK_AVERAGE &&
        method != DREPHIP_LINK_WEIGHTED) {
        set_error("linkage method must be single, complete, average or weighted");
        return DREPHIP_ERR_UNSUPPORTED;
    }
    timing_begin(ctx);
    ctx->link = LinkStats{};
    const auto t0 = std::chrono::steady_clock::now();
    double *d_D;
    uint32_t flags = 0;
    int rc = dist_from_square_impl(ctx, M, n, &d_D, &flags, ctx->stream);
    if (rc) return rc;
    // scipy's order: squareform's symmetry check, its diagonal check, then linkage's finiteness check
    if (flags & 1) { set_error("Distance matrix 'X' must be symmetric."); return DREPHIP_ERR_ARG; }
    if (flags & 2) { set_error("Distance matrix 'X' diagonal must be zero."); return DREPHIP_ERR_ARG; }
    if (flags & 4) { set_error("The condensed distance matrix must contain only finite values."); return DREPHIP_ERR_ARG; }
    rc = linkage_device_impl(ctx, d_D, n, method, Z, ctx->stream);
    if (rc) return rc;
    timing_collect(ctx);
    ctx->link.wall_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return DREPHIP_OK;
}

DREPHIP_EXPORT int drephip_linkage_counts_device(drephip_ctx *ctx, const uint16_t *d_common, const uint16_t *d_denom,
                                                 uint32_t n, const uint32_t *perm, const double *lut,
                                                 uint32_t lut_len, const int32_t *lut_off, int method, double *Z,
                                                 void *stream) {
    GUARD_CTX(ctx);
    if (n < 2) return DREPHIP_OK;
    if (!d_common || !perm || !lut || !lut_off || !Z) { set_error("null argument"); return DREPHIP_ERR_ARG; }
    if (n > 200000) { set_error("linkage supports n <= 200000 (n x n f64 matrix in HBM)"); return DREPHIP_ERR_UNSUPPORTED; }
    for (uint32_t d = 0; d <= ctx->s; d++)
        if (lut_off[d] >= 0 && (uint64_t)lut_off[d] + d + 1 > lut_len) { set_error("lut_off/lut_len mismatch"); return DREPHIP_ERR_ARG; }
    if (!d_denom && lut_off[ctx->s] < 0) {
        set_error("d_denom is NULL (every denominator is s) but lut_off[s] < 0");
        return DREPHIP_ERR_ARG;
    }
    std::vector<char> seen(n, 0);
    for (uint32_t i = 0; i < n; i++) {
        if (perm[i] >= n || seen[perm[i]]) { set_error("perm is not a permutation of 0..n-1"); return DREPHIP_ERR_ARG; }
        seen[perm[i]] = 1;
    }
    // the counts are read after everything the caller queued on `stream`
    // (e.g. the all-pairs call that wrote them, deferred or not)
    int rc = allpairs_wait_impl(ctx);
    if (rc) return rc;
    HIPC(hipStreamSynchronize(pick_stream(ctx, stream)));
    timing_begin(ctx);
    ctx->link = LinkStats{};
    const auto t0 = std::chrono::steady_clock::now();
    bool done = false;
    if (ctx->link_path != DREPHIP_LINK_PATH_DENSE) {
        // sparse path: the pairs below 1.0 (nonzero counts) extracted on the GPU,
        // scipy's algorithm replayed on them on the host (linkage_sparse.cpp)
        const bool forced = ctx->link_path == DREPHIP_LINK_PATH_SPARSE;
        const uint64_t cap = sparse_pair_cap(ctx, n);
        uint32_t *ij = nullptr, *lidx = nullptr, flags = 0;
        uint64_t np = 0;
        rc = sparse_pairs_impl(ctx, d_common, d_denom, n, perm, lut, lut_len, lut_off, cap, &ij, &lidx, &np, &flags,
                               ctx->stream);
        if (rc) return rc;
        ctx->link.sp.pairs = np;
        if (flags & 1) {
            set_error("a pair's denominator has no distance table (lut_off < 0) or its count exceeds it");
            return DREPHIP_ERR_ARG;
        }
        const double t1 = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (!(flags & 2) && np <= cap) {
            std::vector<uint32_t> pi(np), pj(np);
            std::vector<double> pv(np);
            for (uint64_t t = 0; t < np; t++) { pi[t] = ij[2 * t]; pj[t] = ij[2 * t + 1]; pv[t] = lut[lidx[t]]; }
            rc = linkage_sparse_impl(n, np, pi.data(), pj.data(), pv.data(), method, sparse_cells(ctx),
                                     sparse_maxcomp(ctx), Z, &ctx->link.sp, forced ? 1 : 0);
            if (rc == DREPHIP_OK) {
                done = true;
                ctx->link.sparse = 1;
                ctx->link.matrix_s = t1;
                ctx->link.chain_s = ctx->link.sp.setup_s + ctx->link.sp.chain_s;
                ctx->link.finish_s = ctx->link.sp.finish_s;
            } else if (rc != DREPHIP_ERR_UNSUPPORTED || forced) {
                return rc;
            }
        } else if (forced) {
            set_error(flags & 2 ? "sparse linkage: the distance table holds a value above 1.0 (or 0 shared hashes is not 1.0)"
                                : "sparse linkage: more pairs below 1.0 than the pair list holds");
            return DREPHIP_ERR_UNSUPPORTED;
        }
    }
    if (!done) {
        double *d_D;
        rc = dist_matrix_impl(ctx, d_common, d_denom, n, perm, lut, lut_len, lut_off, &d_D, ctx->stream);
        if (rc) return rc;
        rc = linkage_device_impl(ctx, d_D, n, method, Z, ctx->stream);
        if (rc) return rc;
    }
    timing_collect(ctx);
    ctx->link.wall_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return DREPHIP_OK;
}

DREPHIP_EXPORT int drephip_linkage_reserve(drephip_ctx *ctx, uint32_t n) {
    GUARD_CTX(ctx);
    if (n > 200000) { set_error("linkage supports n <= 200000 (n x n f64 matrix in HBM)"); return DREPHIP_ERR_UNSUPPORTED; }
    if (n < 2) return DREPHIP_OK;
    void *p;
    return scratch(ctx, "lk_D", (uint64_t)n * n * 8, &p);
}

DREPHIP_EXPORT int drephip_last_linkage_info(drephip_ctx *ctx, int *sparse, uint64_t *pairs, uint32_t *components,
                                             uint32_t *largest) {
    if (!ctx) { set_error("null context"); return DREPHIP_ERR_ARG; }
    if (!sparse || !pairs || !components || !largest) { set_error("null argument"); return DREPHIP_ERR_ARG; }
    *sparse = ctx->link.sparse;
    *pairs = ctx->link.sp.pairs;
    *components = ctx->link.sp.components;
    *largest = ctx->link.sp.largest;
    return DREPHIP_OK;
}

DREPHIP_EXPORT int drephip_last_linkage_launches(drephip_ctx *ctx, uint64_t *launches) {
    if (!ctx || !launches) { set_error("null argument"); return DREPHIP_ERR_ARG; }
    *launches = ctx->link.launches;
    return DREPHIP_OK;
}

DREPHIP_EXPORT int drephip_last_linkage_stats(drephip_ctx *ctx, double *alloc_s, double *matrix_s, double *chain_s,
                                              double *finish_s, double *wall_s) {
    if (!ctx) { set_error("null context"); return DREPHIP_ERR_ARG; }
    if (!alloc_s || !matrix_s || !chain_s || !finish_s || !wall_s) { set_error("null argument"); return DREPHIP_ERR_ARG; }
    *alloc_s = ctx->link.alloc_s;
    *matrix_s = ctx->link.matrix_s;
    *chain_s = ctx->link.chain_s;
    *finish_s = ctx->link.finish_s;
    *wall_s = ctx->link.wall_s;
    return DREPHIP_OK;
}
