// ctx.h -- the drephip_ctx object behind the C ABI (host side).
#pragma once

#include "common.h"

#include <hip/hip_runtime.h>
#include <map>
#include <memory>
#include <utility>
#include <string>
#include <vector>

struct DevBuf {
    void *ptr = nullptr;
    size_t bytes = 0;
};

// A pinned host buffer pair of the ingest pipeline (drephip_sketch_files).
struct PinnedSlot {
    uint32_t *codes = nullptr, *valid = nullptr;
    size_t codes_bytes = 0, valid_bytes = 0;
    PinnedSlot() = default;
    PinnedSlot(const PinnedSlot &) = delete;
    PinnedSlot &operator=(const PinnedSlot &) = delete;
    ~PinnedSlot() {
        if (codes) (void)hipHostFree(codes);
        if (valid) (void)hipHostFree(valid);
    }
    int reserve(size_t cb, size_t vb) {
        if (cb > codes_bytes) {
            if (codes) (void)hipHostFree(codes);
            codes = nullptr; codes_bytes = 0;
            if (hipHostMalloc((void **)&codes, cb, hipHostMallocPortable) != hipSuccess) { codes = nullptr; return -1; }
            codes_bytes = cb;
        }
        if (vb > valid_bytes) {
            if (valid) (void)hipHostFree(valid);
            valid = nullptr; valid_bytes = 0;
            if (hipHostMalloc((void **)&valid, vb, hipHostMallocPortable) != hipSuccess) { valid = nullptr; return -1; }
            valid_bytes = vb;
        }
        return 0;
    }
};

struct IngestStats {          // last drephip_sketch_files call
    double produce_s = 0;     // host read + pack, summed over batches (producer thread)
    double gpu_s = 0;         // H2D + sketch kernels + D2H, summed over batches (calling thread)
    double wall_s = 0;        // the whole call
    uint32_t batches = 0;
    double read_thread_s = 0; // read + parse (incl. gzip inflate), summed over worker threads
    double pack_thread_s = 0; // 2-bit pack into the pinned batch, summed over worker threads
    uint32_t overflow = 0;    // genomes repacked because their span outgrew the file-size estimate
};

struct SparseLinkInfo {       // the sparse linkage path (linkage_sparse.cpp)
    uint64_t pairs = 0;       // listed pairs (distance below 1.0)
    uint32_t components = 0;  // connected components with >= 2 members (0 for single linkage)
    uint32_t largest = 0;     // members of the largest one
    uint64_t cells = 0;       // per-component matrix cells (sum of m^2)
    int rows = 0;             // 1: the sparse-row chain ran (no per-component matrices)
    uint64_t scanned = 0;     // sparse-row chain: row entries read by the searches and merges
    double setup_s = 0;       // components + matrices
    double chain_s = 0;       // nn-chain / Prim steps
    double finish_s = 0;      // stable sort + relabel
};

struct LinkStats {            // last drephip_linkage* call, host wall clock (seconds)
    double alloc_s = 0;       // device scratch for the n x n matrix (hipMalloc; 0 when reused)
    double matrix_s = 0;      // matrix build from the counts / condensed input (incl. its H2D copies);
                              // sparse path: the pair extraction (kernel + readback)
    double chain_s = 0;       // nn-chain / MST steps (graph replays; sparse path: host setup + steps)
    uint64_t launches = 0;    // dense chain: step launches that did work (0: sparse path / none)
    uint64_t compactions = 0; // dense chain: matrix compactions (linkage.hip, k_lk_cmp_rank)
    double finish_s = 0;      // Z readback + stable sort + relabel on the host
    double wall_s = 0;        // the whole call
    int sparse = 0;           // 1: the sparse path produced Z
    SparseLinkInfo sp;        // its figures (pairs also when the dense path was chosen)
};

// The shared-hash screen of the last all-pairs call (screen.hip).
struct ScreenResult {
    bool use = false;             // the screened lists below replace the dense item plan
    const uint32_t *clist = nullptr;   // marked columns, per row tile, ascending (device)
    const uint4 *items = nullptr;      // {i0, list offset, count, 0} (device)
    uint32_t nitems = 0;
    uint64_t entries = 0;         // sketch entries sorted
    uint64_t runs = 0;            // runs of >= 2 equal 32-bit keys
    uint64_t checks = 0;          // pair checks of the marking (sum of m(m-1)/2)
    uint64_t marked = 0;          // marked (row tile, column) cells
    uint64_t simple = 0;          // pairs sharing exactly one hash, written by the screen itself
    // use == false after a dense verdict: per genome, the 64-element chunks
    // whose hits need the high-word check (k_cmask_*; device, or null)
    const uint32_t *cmask = nullptr;
};

// The last hash part a sharded screen grouped (screen_part_impl): its marked
// cells as the nonzero words of its (row tile from row 0, column) bitmap and
// its records of runs of two, in the context's scratch until the next screen
// call.
struct PartResult {
    bool valid = false;
    uint32_t N = 0, R = 0;
    const uint4 *cells = nullptr;       // {row tile, word, bits, 0}
    uint32_t ncells = 0;
    const uint4 *rec = nullptr;         // {a, b, (i << 16) | j, 0}
    uint32_t nrec = 0;
    uint64_t entries = 0, runs = 0, checks = 0;
};
// Marks handed to the next all-pairs call (drephip_allpairs_device_marked):
// the parts' cell words and records; the call screens its rows from them.
struct ExtMarks {
    bool active = false;
    const uint4 *cells = nullptr;
    uint64_t ncells = 0;
    const uint4 *rec = nullptr;
    uint64_t nrec = 0;
};

// A run of all-pairs work items (allpairs.hip, plan_items): `size` row tiles
// from i0 (step R) against column tile c0, at offset `off` of its XCD's list.
struct ApItemGroup { uint32_t i0, c0, off, size; };

struct drephip_ctx {
    int device = 0;
    int k = 21;
    uint32_t s = 1000;
    uint32_t seed = 42;
    hipStream_t stream = nullptr;
    uint32_t timing = 0;      // bitmask of timed kernels (bit w = `which` w of drephip_last_kernel_ms)
    int ap_path = 0;          // DREPHIP_AP_*: 0 auto (table for s <= 2048, else band)
    int screen = 0;           // DREPHIP_SCREEN_*: 0 auto, 1 on, 2 off
    ScreenResult last_screen; // the last all-pairs call's screen (stats; pointers into scratch)
    PartResult part;          // the last sharded-screen part (drephip_screen_part)
    ExtMarks ext;             // marks for the current drephip_allpairs_device_marked call
    int link_path = 0;        // DREPHIP_LINK_PATH_*: 0 auto (sparse when it applies, else dense)
    uint32_t band_cap = 1024; // elements per row per band of the banded all-pairs kernel (clamped to its LDS budget)
    uint32_t band_round = 0;  // elements per row per value round of the band kernel (0: no rounds; A/B)
    // named grow-only device scratch buffers
    std::map<std::string, DevBuf> bufs;
    // per-kernel timing of the last call: {sum ms, launches}
    double kms[5] = {0, 0, 0, 0, 0};
    int kn[5] = {0, 0, 0, 0, 0};
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;
    struct Span { int which; hipEvent_t a, b; };
    std::vector<Span> spans;
    uint64_t alloc_gen = 1;   // bumped by every scratch (re)allocation
    // sketch tile table of the last call (reused while the genome layout is the
    // same and no scratch buffer has been reallocated since: sk_gen == alloc_gen)
    std::vector<uint64_t> sk_off, sk_pad, sk_nk;
    // candidate sets / counts known to be empty / zero: the first sk_clean_n
    // genomes' slots of these buffers (every finalize resets what it read)
    unsigned long long *sk_clean_sets = nullptr;
    uint32_t *sk_clean_cnt = nullptr;
    uint32_t sk_clean_n = 0;
    uint64_t sk_clean_gen = 0;   // alloc_gen when they were last left clean
    uint64_t sk_gen = 0;
    uint64_t sk_tab_gen = 0;     // alloc_gen when the Murmur table image was built
    // pinned host staging for the small per-call readbacks (status, failure count)
    std::map<std::string, DevBuf> pinned;
    // all-pairs work-item list of the last call, reused on the same shape (its
    // group table kept on the host: a deferred call's H2D copy may still be queued)
    uint64_t ap_items_key[5] = {0, 0, 0, 0, 0};
    uint64_t ap_items_gen = 0;
    uint64_t ap_items_n = 0;
    std::vector<ApItemGroup> ap_groups_host;
    // deferred sketch (drephip_sketch_device_async): the first round is queued
    // without reading its status back; drephip_sketch_wait checks it (and
    // reruns the call synchronously if a genome needs another threshold round).
    // While it is pending, every other sketch call on the context is refused.
    struct PendingSketch {
        bool active = false;
        const uint32_t *d_codes = nullptr, *d_valid = nullptr;
        std::vector<uint64_t> off, pad, nk;
        uint32_t n = 0;
        uint64_t *d_hashes = nullptr;
        uint32_t *d_nhash = nullptr;
        hipStream_t st = nullptr;
        const uint8_t *h_status = nullptr;     // pinned, written by the queued copy
        std::vector<Span> spans;               // timing spans of the queued kernels
        std::vector<hipEvent_t> events;        // their events, out of ev_pool until collected
        hipEvent_t done = nullptr;             // after the status copy
    } pend;
    // deferred all-pairs call (drephip_allpairs_device_async, table path):
    // an event after its kernels
    struct PendingAllpairs {
        bool active = false;
        hipEvent_t ev = nullptr;
    } apend;
    IngestStats ingest;
    LinkStats link;
    PinnedSlot ingest_slots[2];   // the two pinned batch buffers, kept across calls
};

namespace drephip {

// hip error -> set_error + return code
#define HIPC(expr)                                                                     \
    do {                                                                               \
        hipError_t _e = (expr);                                                        \
        if (_e != hipSuccess) {                                                        \
            ::drephip::set_error(std::string(#expr) + ": " + hipGetErrorString(_e)); \
            return DREPHIP_ERR_HIP;                                                    \
        }                                                                              \
    } while (0)

// Grow-only named scratch buffer on the context's device.
int scratch(drephip_ctx *ctx, const char *name, size_t bytes, void **out);
// Grow-only named pinned host buffer (hipHostMalloc) for async readbacks.
int pinned_host(drephip_ctx *ctx, const char *name, size_t bytes, void **out);

// Bracket kernel launches with events when their bit of ctx->timing is set; resolved by
// timing_collect() after the stream is synchronised.
void timing_begin(drephip_ctx *ctx);
void timing_mark(drephip_ctx *ctx, int which, hipStream_t st, bool start);
void timing_collect(drephip_ctx *ctx);

// Kernel drivers (sketch.hip / allpairs.hip).
int sketch_device_impl(drephip_ctx *ctx, const uint32_t *d_codes, const uint32_t *d_valid,
                       const uint64_t *base_off, const uint64_t *padded, const uint64_t *nkmers,
                       uint32_t n, uint64_t *d_hashes, uint32_t *d_nhash, hipStream_t st,
                       bool defer = false);
int synth_device_impl(drephip_ctx *ctx, uint64_t seed, uint32_t g0, uint32_t n, uint32_t family_size,
                      uint64_t L, uint32_t *d_codes, uint32_t *d_valid, hipStream_t st);
int allpairs_device_impl(drephip_ctx *ctx, const uint64_t *d_hashes, const uint32_t *d_nhash,
                         uint32_t N, uint32_t row0, uint32_t row1, uint16_t *d_common,
                         uint16_t *d_denom, hipStream_t st, bool force_merge, bool defer = false);
int allpairs_wait_impl(drephip_ctx *ctx);
// The shared-hash screen (screen.hip): the (row tile of R rows, column) cells
// of rows [row0, row1) whose row and column share a hash, as per-tile column
// lists and LIST work items of at most C columns.  When it applies it also
// writes the segment: every pair as no-shared-hash, then the pairs that share
// exactly one hash (outside the listed cells); the LIST kernels complete it.
// res->use = false when the set is too dense for it to pay (unless force) or
// too large for its 32-bit indices; the dense path runs then (and rewrites
// every pair).  `band`: the LIST kernel is the band kernel (s > 2048), the
// only one the light cells pay for.  Synchronises the stream.
int screen_impl(drephip_ctx *ctx, const uint64_t *d_hashes, const uint32_t *d_nhash, uint32_t N, uint32_t row0,
                uint32_t row1, uint32_t R, uint32_t C, uint64_t seg0, uint64_t npairs, uint16_t *d_common,
                uint16_t *d_denom, bool force, bool band, hipStream_t st, ScreenResult *res);
// The sharded screen (screen.hip): one hash part's marks for every row
// (ctx->part), and a rank's rows screened from every part's marks.
int screen_part_impl(drephip_ctx *ctx, const uint64_t *d_hashes, const uint32_t *d_nhash, uint32_t N, uint32_t R,
                     uint32_t part, uint32_t nparts, hipStream_t st, uint64_t *checks, uint32_t *ncells,
                     uint32_t *nrec);
int screen_marked_impl(drephip_ctx *ctx, const uint32_t *d_nhash, uint32_t N, uint32_t row0, uint32_t row1,
                       uint32_t R, uint32_t C, uint64_t seg0, uint64_t npairs, uint16_t *d_common, uint16_t *d_denom,
                       const uint4 *d_cells, uint64_t ncells, const uint4 *d_rec, uint64_t nrec, hipStream_t st,
                       ScreenResult *res);
// the dense-set rule on the whole triangle's pair checks E
bool screen_worth(uint32_t N, uint32_t s, uint64_t E);
// rows per row tile and the all-pairs path (table / band) the all-pairs call
// takes for this context's s (the sharded screen's parts and ranks share it)
int allpairs_geometry(drephip_ctx *ctx, uint32_t *R, int *path);
int screen_mode(drephip_ctx *ctx);
bool screen_applies(drephip_ctx *ctx, uint32_t N);
// Every pair of the segment as an unscreened one: common 0, denominator
// min(s, |A| + |B|); the LIST kernels then overwrite the screened pairs.
int screen_fill_impl(drephip_ctx *ctx, const uint32_t *d_nhash, uint32_t N, uint32_t row0, uint32_t row1,
                     uint64_t seg0, uint64_t npairs, uint16_t *d_common, uint16_t *d_denom, hipStream_t st);

// Primary clustering (linkage.hip).
int linkage_device_impl(drephip_ctx *ctx, double *d_D, uint32_t n, int method, double *Z_out, hipStream_t st);
int dist_matrix_impl(drephip_ctx *ctx, const uint16_t *d_common, const uint16_t *d_denom, uint32_t n,
                     const uint32_t *perm, const double *lut, uint32_t lut_len, const int32_t *lut_off,
                     double **d_D_out, hipStream_t st);
int dist_from_condensed_impl(drephip_ctx *ctx, const double *y, uint32_t n, double **d_D_out, hipStream_t st);
// from a host n x n float32 matrix (the pivot's values); *flags: bit 0 not
// symmetric, bit 1 a nonzero diagonal entry, bit 2 a non-finite value
int dist_from_square_impl(drephip_ctx *ctx, const float *M, uint32_t n, double **d_D_out, uint32_t *flags,
                          hipStream_t st);
// pairs below 1.0 of the device counts (rows/columns through perm), as (perm i, perm j, lut index) in
// pinned context buffers (*h_ij, *h_lidx; valid until the next call);
// *np = their count (> cap: not written); *flags bit 0: a pair's denominator has no table or its count
// exceeds it, bit 1: the table holds a value above 1.0 or NaN (no sparse form).  Blocking.
int sparse_pairs_impl(drephip_ctx *ctx, const uint16_t *d_common, const uint16_t *d_denom, uint32_t n,
                      const uint32_t *perm, const double *lut, uint32_t lut_len, const int32_t *lut_off,
                      uint64_t cap, uint32_t **h_ij, uint32_t **h_lidx, uint64_t *np, uint32_t *flags,
                      hipStream_t st);
// Host (linkage_sparse.cpp): scipy's linkage from the pairs below 1.0 (every other pair at 1.0).
// DREPHIP_ERR_UNSUPPORTED when the per-component matrices would exceed max_cells or a component
// max_comp members.
int linkage_sparse_impl(uint32_t n, uint64_t np, const uint32_t *pi, const uint32_t *pj, const double *pv,
                        int method, uint64_t max_cells, uint32_t max_comp, double *Z_out, SparseLinkInfo *info,
                        int rows = 0);
// rows: 0 never the sparse-row chain, 1 where the components exceed the
// matrix limits, 2 always (DREPHIP_LINK_ROWS overrides: 0 / 1 / 2)
void sort_and_label(std::vector<double> &Z, uint32_t n);
// host worker threads of the linkage paths: OMP_NUM_THREADS if set, else the
// hardware threads, at most 16
unsigned host_threads();

// Host ingest (ingest.cpp).
// std::allocator that leaves new elements uninitialised (resize() without the
// memset: the FASTA reader writes every byte it keeps)
template <class T>
struct NoInitAlloc : std::allocator<T> {
    template <class U> struct rebind { using other = NoInitAlloc<U>; };
    NoInitAlloc() = default;
    template <class U> NoInitAlloc(const NoInitAlloc<U> &) {}
    template <class U> void construct(U *) noexcept {}
    template <class U, class... A> void construct(U *p, A &&...a) { ::new ((void *)p) U(std::forward<A>(a)...); }
};

struct Genome {
    std::vector<uint8_t, NoInitAlloc<uint8_t>> seq;   // concatenated record bytes (raw case)
    std::vector<uint64_t> rec_len;   // record lengths
    uint64_t length = 0;             // sum of record lengths
};
int read_fasta(const char *path, Genome &g);
uint64_t genome_span(const uint64_t *rec_len, uint32_t n_rec);
// pack records into codes/valid at base offset; returns valid k-mer count
uint64_t pack_records(const uint8_t *seq, const uint64_t *rec_len, uint32_t n_rec, int k,
                      uint32_t *codes, uint32_t *valid, uint64_t base_off);

}  // namespace drephip
