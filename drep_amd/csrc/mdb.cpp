// mdb.cpp -- the Mdb table and its pivot on the host (no GPU).
//
// dRep materialises the Mash result as an N^2-row DataFrame (Mdb,
// drep/d_cluster.py:575-596) and primary clustering turns it back into an
// N x N matrix with DataFrame.pivot (cluster_mash_database, 619-621).  Both
// are pure layout work on N^2 cells -- 10^8 at 10^4 genomes, where pandas
// needs ~4 s to build the table and ~50 s to pivot it.  Here:
//
//  * drephip_mdb_square: the table's columns straight from the condensed
//    all-pairs counts: each row q of the square is the condensed row q (the
//    pairs r > q, contiguous) plus, below the diagonal, a blocked transpose of
//    the rows already written (the matrix is symmetric: Mash's distance is);
//  * drephip_pivot_scan / drephip_pivot_fill: the pivot on category codes --
//    for the table all_vs_all_MASH returns (genome1 cycling fastest) a
//    permuted, blocked transpose; for any other row order a scatter that
//    detects duplicate cells and leaves missing ones NaN, as pandas does.
//
// Memory-bound: every cell is written once (dist, similarity, two codes:
// 12 B with int16 codes) and read at most twice; rows are split over host
// threads by equal cell counts.
#include "ctx.h"
#include "../../include/drephip.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <limits>
#include <thread>
#include <vector>

#define DREPHIP_EXPORT extern "C" __attribute__((visibility("default")))

namespace drephip {

static unsigned pick_threads(int threads) {
    unsigned T = threads > 0 ? (unsigned)threads : std::thread::hardware_concurrency();
    return std::max(1u, std::min(T, 64u));
}

template <class F>
static void parallel_for(unsigned T, uint64_t n, F &&f) {       // f(t, lo, hi) over T equal slices
    T = (unsigned)std::min<uint64_t>(T, std::max<uint64_t>(n, 1));
    if (T <= 1) { f(0u, (uint64_t)0, n); return; }
    std::vector<std::thread> pool;
    for (unsigned t = 1; t < T; t++) pool.emplace_back([&, t] { f(t, n * t / T, n * (t + 1) / T); });
    f(0u, (uint64_t)0, n / T);
    for (auto &th : pool) th.join();
}

template <class F>
static void parallel_strided(unsigned T, uint64_t n, F &&f) {   // f(i) for i = t, t + T, ... on thread t
    T = (unsigned)std::min<uint64_t>(T, std::max<uint64_t>(n, 1));
    auto run = [&](unsigned t) { for (uint64_t i = t; i < n; i += T) f(i); };
    std::vector<std::thread> pool;
    for (unsigned t = 1; t < T; t++) pool.emplace_back(run, t);
    run(0);
    for (auto &th : pool) th.join();
}

static inline uint64_t cidx(uint64_t i, uint64_t j, uint64_t N) {      // i < j
    return i * N - i * (i + 1) / 2 + (j - i - 1);
}

template <class C>
static inline int64_t code_at(const void *p, uint64_t k) { return (int64_t)((const C *)p)[k]; }

static int64_t load_code(const void *p, int bytes, uint64_t k) {
    return bytes == 1 ? code_at<int8_t>(p, k) : bytes == 2 ? code_at<int16_t>(p, k) : code_at<int32_t>(p, k);
}

template <class C>
static void fill_codes(void *g1, void *g2, const int32_t *codes, uint32_t N, uint32_t q) {
    C *a = (C *)g1 + (uint64_t)q * N, *b = (C *)g2 + (uint64_t)q * N;
    if (g1) for (uint32_t r = 0; r < N; r++) a[r] = (C)codes[r];
    if (g2) std::fill(b, b + N, (C)codes[q]);
}

constexpr uint32_t kT = 64;          // transpose tile

}  // namespace drephip

using namespace drephip;

DREPHIP_EXPORT int drephip_mdb_square(uint32_t N, const uint16_t *common, const uint16_t *denom, uint32_t s,
                                      const float *lut32, uint32_t lut_len, const int32_t *lut_off,
                                      const int32_t *codes, int code_bytes, void *g1, void *g2, float *dist,
                                      float *sim, int threads) {
    if (!dist || !lut32 || !lut_off || (N > 1 && !common) || ((g1 || g2) && !codes)) {
        set_error("null argument");
        return DREPHIP_ERR_ARG;
    }
    if (code_bytes != 1 && code_bytes != 2 && code_bytes != 4) { set_error("code_bytes must be 1, 2 or 4"); return DREPHIP_ERR_ARG; }
    if (s > 32767) { set_error("s must be <= 32767"); return DREPHIP_ERR_ARG; }
    for (uint32_t d = 0; d <= s; d++)
        if (lut_off[d] >= 0 && (uint64_t)lut_off[d] + d + 1 > lut_len) { set_error("lut_off/lut_len mismatch"); return DREPHIP_ERR_ARG; }
    const unsigned T = pick_threads(threads);
    std::atomic<int> bad(0);
    // 1. rows q: the diagonal, the pairs r > q from the condensed row, the codes.
    //    Rows by equal cell counts of their upper parts (row q has N-1-q pairs).
    const uint64_t np = (uint64_t)N * (N - (N ? 1 : 0)) / 2;
    std::vector<uint32_t> rb(T + 1, N);
    rb[0] = 0;
    for (unsigned k = 1; k < T; k++) {
        const uint64_t target = np * k / T;
        uint32_t lo = rb[k - 1], hi = N;
        while (lo < hi) {
            const uint32_t mid = lo + (hi - lo) / 2;
            if ((uint64_t)mid * N - (uint64_t)mid * (mid + 1) / 2 < target) lo = mid + 1; else hi = mid;   // pairs of rows < mid
        }
        rb[k] = lo;
    }
    auto rows = [&](unsigned k) {
        for (uint32_t q = rb[k]; q < rb[k + 1]; q++) {
            float *row = dist + (uint64_t)q * N;
            row[q] = 0.0f;
            const uint64_t t0 = q + 1 < N ? cidx(q, q + 1, N) : 0;
            int b = 0;
            if (denom) {
                for (uint32_t r = q + 1; r < N; r++) {
                    const uint32_t d = denom[t0 + (r - q - 1)], c = common[t0 + (r - q - 1)];
                    const int32_t o = d <= s ? lut_off[d] : -1;
                    const bool good = o >= 0 && c <= d;
                    b |= !good;
                    row[r] = good ? lut32[o + c] : 0.0f;
                }
            } else {
                const int32_t o = lut_off[s];
                if (o < 0) { b = 1; }
                else {
                    const float *L = lut32 + o;
                    const uint16_t *cr = common + t0 - (q + 1);
                    for (uint32_t r = q + 1; r < N; r++) {
                        const uint32_t c = cr[r];
                        b |= c > s;
                        row[r] = L[c <= s ? c : 0];
                    }
                }
            }
            if (b) bad = 1;
            if (sim) {
                float *srow = sim + (uint64_t)q * N;
                for (uint32_t r = q; r < N; r++) srow[r] = 1.0f - row[r];
            }
            if (g1 || g2) {
                if (code_bytes == 1) fill_codes<int8_t>(g1, g2, codes, N, q);
                else if (code_bytes == 2) fill_codes<int16_t>(g1, g2, codes, N, q);
                else fill_codes<int32_t>(g1, g2, codes, N, q);
            }
        }
    };
    {
        std::vector<std::thread> pool;
        for (unsigned k = 1; k < T; k++) pool.emplace_back(rows, k);
        rows(0);
        for (auto &th : pool) th.join();
    }
    if (bad) {
        set_error("a pair's denominator has no distance table (lut_off < 0) or its count exceeds it");
        return DREPHIP_ERR_ARG;
    }
    // 2. below the diagonal: the transpose of the upper part, tile by tile
    //    (tiles (bq, br) with br <= bq; row bq of tiles has bq + 1 of them, so
    //    the rows are dealt round robin), with the similarity of those cells
    const uint32_t nb = (N + kT - 1) / kT;
    parallel_strided(T, nb, [&](uint64_t bq) {
        {
            const uint32_t q0 = (uint32_t)bq * kT, q1 = std::min(N, q0 + kT);
            for (uint32_t br = 0; br <= bq; br++) {
                const uint32_t r0 = br * kT, r1 = std::min(N, r0 + kT);
                for (uint32_t q = q0; q < q1; q++) {
                    float *row = dist + (uint64_t)q * N;
                    float *srow = sim ? sim + (uint64_t)q * N : nullptr;
                    const uint32_t re = std::min(r1, q);          // r < q
                    for (uint32_t r = r0; r < re; r++) {
                        const float v = dist[(uint64_t)r * N + q];
                        row[r] = v;
                        if (srow) srow[r] = 1.0f - v;
                    }
                }
            }
        }
    });
    return DREPHIP_OK;
}

DREPHIP_EXPORT int drephip_pivot_scan(uint64_t nrows, const void *codes1, const void *codes2, int code_bytes,
                                      uint32_t ncat, uint8_t *present1, uint8_t *present2, uint64_t *period,
                                      int threads) {
    if (!present1 || !present2 || !period || (nrows && (!codes1 || !codes2))) { set_error("null argument"); return DREPHIP_ERR_ARG; }
    if (code_bytes != 1 && code_bytes != 2 && code_bytes != 4) { set_error("code_bytes must be 1, 2 or 4"); return DREPHIP_ERR_ARG; }
    const unsigned T = pick_threads(threads);
    std::memset(present1, 0, ncat);
    std::memset(present2, 0, ncat);
    *period = 0;
    if (!nrows) return DREPHIP_OK;
    // the candidate period: the first row where genome2 changes
    uint64_t n = 1;
    const int64_t head = load_code(codes2, code_bytes, 0);
    while (n < nrows && load_code(codes2, code_bytes, n) == head) n++;
    const bool may = nrows % n == 0;
    std::vector<std::vector<uint8_t>> p1(T, std::vector<uint8_t>(ncat, 0)), p2(T, std::vector<uint8_t>(ncat, 0));
    std::atomic<int> neg(0), broken(may ? 0 : 1);
    parallel_for(T, nrows, [&](unsigned t, uint64_t lo, uint64_t hi) {
        uint8_t *a = p1[t].data(), *b = p2[t].data();
        bool per = may;
        for (uint64_t k = lo; k < hi; k++) {
            const int64_t x = load_code(codes1, code_bytes, k), y = load_code(codes2, code_bytes, k);
            if (x < 0 || y < 0 || x >= (int64_t)ncat || y >= (int64_t)ncat) { neg = 1; return; }
            a[x] = 1;
            b[y] = 1;
            if (per) {
                const uint64_t m = k % n;
                per = x == load_code(codes1, code_bytes, m) && y == load_code(codes2, code_bytes, k - m);
            }
        }
        if (!per) broken = 1;
    });
    if (neg) { set_error("a row's genome is missing (negative or out-of-range category code)"); return DREPHIP_ERR_UNSUPPORTED; }
    for (unsigned t = 0; t < T; t++)
        for (uint32_t c = 0; c < ncat; c++) { present1[c] |= p1[t][c]; present2[c] |= p2[t][c]; }
    *period = broken ? 0 : n;
    return DREPHIP_OK;
}

DREPHIP_EXPORT int drephip_pivot_fill(uint64_t nrows, const void *codes1, const void *codes2, int code_bytes,
                                      const int32_t *pos1, const int32_t *pos2, uint32_t ncat, const float *vals,
                                      uint32_t n1, uint32_t n2, uint64_t period, float *out, int threads) {
    if (!pos1 || !pos2 || !out || (nrows && (!codes1 || !codes2 || !vals))) { set_error("null argument"); return DREPHIP_ERR_ARG; }
    if (code_bytes != 1 && code_bytes != 2 && code_bytes != 4) { set_error("code_bytes must be 1, 2 or 4"); return DREPHIP_ERR_ARG; }
    for (uint32_t c = 0; c < ncat; c++)
        if (pos1[c] >= (int64_t)n1 || pos2[c] >= (int64_t)n2) { set_error("pivot position out of range"); return DREPHIP_ERR_ARG; }
    const unsigned T = pick_threads(threads);
    const uint64_t cells = (uint64_t)n1 * n2;
    std::atomic<int> bad(0);
    if (period && period == n1 && nrows == cells && n1 && n2) {
        // all_vs_all_MASH's layout: row b*n + a = (genome1 codes1[a], genome2 codes2[b*n]),
        // each of the n1 genome1 values once per block (n == n1 present values) and
        // each block a different genome2 (nrows / n == n2): out[P1[a]][J[b]] = vals[b n + a]
        const uint64_t n = period, m = nrows / n;
        std::vector<int32_t> P1(n), J(m);
        for (uint64_t a = 0; a < n; a++) P1[a] = pos1[load_code(codes1, code_bytes, a)];
        for (uint64_t b = 0; b < m; b++) J[b] = pos2[load_code(codes2, code_bytes, b * n)];
        std::vector<uint8_t> seen1(n1, 0), seen2(n2, 0);
        for (uint64_t a = 0; a < n; a++) { if (P1[a] < 0 || seen1[P1[a]]) bad = 1; else seen1[P1[a]] = 1; }
        for (uint64_t b = 0; b < m; b++) { if (J[b] < 0 || seen2[J[b]]) bad = 1; else seen2[J[b]] = 1; }
        if (!bad) {
            // threads own output rows (kT values of a each: every page of `out`
            // is first touched by one thread), tiles of kT x kT through L1
            const uint64_t nat = (n + kT - 1) / kT;
            parallel_for(T, nat, [&](unsigned, uint64_t lo, uint64_t hi) {
                for (uint64_t ta = lo; ta < hi; ta++) {
                    const uint64_t a0 = ta * kT, a1 = std::min(n, a0 + kT);
                    for (uint64_t b0 = 0; b0 < m; b0 += kT) {
                        const uint64_t b1 = std::min(m, b0 + kT);
                        for (uint64_t a = a0; a < a1; a++) {
                            float *orow = out + (uint64_t)P1[a] * n2;
                            const float *v = vals + a;
                            for (uint64_t b = b0; b < b1; b++) orow[J[b]] = v[b * n];
                        }
                    }
                }
            });
            return DREPHIP_OK;
        }
        bad = 0;                                                     // not that layout after all: scatter
    }
    // any row order: missing cells NaN, a cell named twice fails
    const float nanv = std::numeric_limits<float>::quiet_NaN();
    parallel_for(T, cells, [&](unsigned, uint64_t lo, uint64_t hi) { std::fill(out + lo, out + hi, nanv); });
    std::vector<std::atomic<uint64_t>> seen((cells + 63) / 64);
    parallel_for(T, seen.size(), [&](unsigned, uint64_t lo, uint64_t hi) {
        for (uint64_t w = lo; w < hi; w++) seen[w].store(0, std::memory_order_relaxed);
    });
    parallel_for(T, nrows, [&](unsigned, uint64_t lo, uint64_t hi) {
        for (uint64_t k = lo; k < hi && !bad.load(std::memory_order_relaxed); k++) {
            const int64_t x = load_code(codes1, code_bytes, k), y = load_code(codes2, code_bytes, k);
            if (x < 0 || y < 0 || x >= (int64_t)ncat || y >= (int64_t)ncat || pos1[x] < 0 || pos2[y] < 0) { bad = 2; return; }
            const uint64_t cell = (uint64_t)pos1[x] * n2 + (uint64_t)pos2[y];
            const uint64_t bit = 1ull << (cell & 63);
            if (seen[cell >> 6].fetch_or(bit, std::memory_order_relaxed) & bit) { bad = 1; return; }
            out[cell] = vals[k];
        }
    });
    if (bad == 2) { set_error("a row's genome has no pivot position"); return DREPHIP_ERR_ARG; }
    if (bad) { set_error("Index contains duplicate entries, cannot reshape"); return DREPHIP_ERR_ARG; }
    return DREPHIP_OK;
}
