// common.h -- shared definitions of libdrephip (HIP, gfx950 only).
//
// Layout, constants and the two integer mixers (MurmurHash3_x64_128 as Mash
// uses it, and the splitmix64 synthetic-genome generator) shared by the
// device kernels and the host ingest.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdlib>
#include <string>

namespace drephip {

// ------------------------------------------------------------------ layout
// One sketch workgroup (256 lanes) owns a tile of 256 * 128 window-end
// positions; every genome starts on a tile boundary (see include/drephip.h).
constexpr uint32_t kLaneBases = 128;          // window ends per lane
constexpr uint32_t kSketchWG = 256;           // lanes per sketch workgroup
constexpr uint64_t kTile = (uint64_t)kLaneBases * kSketchWG;   // 32768 bases
constexpr uint32_t kWarm = 32;                // bases rolled before the first window end
constexpr uint64_t kEmpty = ~0ull;            // empty slot / "no hash" sentinel
constexpr uint64_t kMaxThr = ~0ull - 1;       // inclusive threshold that admits every hash but kEmpty
constexpr uint32_t kLdsSortSketch = 12000;    // up to here finalize sorts <= 16384 candidates in LDS
constexpr uint32_t kMaxSketch = 32767;        // above: a global sort buffer; counts are uint16 (<= s), and
                                              // 0xFFFF stays an impossible count

inline uint64_t round_up(uint64_t x, uint64_t m) { return (x + m - 1) / m * m; }

// One dispatch covers fewer than 2^32 work-items (the AQL grid size is a
// 32-bit work-item count; a larger grid is silently truncated), so every
// launch whose grid scales with N is issued in pieces of at most
// kMaxLaunchItems work-items.  A multiple of 8 workgroups per piece keeps the
// XCD-interleaved item order of the all-pairs kernels intact.
// DREPHIP_MAX_LAUNCH_ITEMS (tests only) lowers the cap so the split runs at
// small sizes too.
constexpr uint64_t kMaxLaunchItems = 1ull << 31;
inline uint64_t max_blocks(uint32_t wg) {
    uint64_t cap = kMaxLaunchItems;
    if (const char *e = std::getenv("DREPHIP_MAX_LAUNCH_ITEMS")) {
        const uint64_t v = std::strtoull(e, nullptr, 10);
        if (v) cap = v < 8ull * wg ? 8ull * wg : v > kMaxLaunchItems ? kMaxLaunchItems : v;
    }
    return cap / wg / 8 * 8;
}

// padded footprint of a genome whose records (incl. the 1-base separators)
// span `span` bases: at least one invalid base after it, rounded to a tile.
inline uint64_t padded_span(uint64_t span) { return round_up(span + 1, kTile); }

// ----------------------------------------------------------------- Murmur3
__host__ __device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) {
    return (x << r) | (x >> (64 - r));
}
__host__ __device__ __forceinline__ uint64_t fmix64(uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33; return k;
}

// MurmurHash3_x64_128(key, K, seed) word 0, where the K key bytes are given
// as little-endian 64-bit words w[0..(K+7)/8) (bytes past K are zero).
template <int K>
__host__ __device__ __forceinline__ uint64_t murmur3_h1_words(const uint64_t *w, uint32_t seed) {
    constexpr uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
    constexpr int nblocks = K / 16;
    constexpr int rem = K & 15;
    uint64_t h1 = seed, h2 = seed;
#pragma unroll
    for (int i = 0; i < nblocks; i++) {
        uint64_t k1 = w[2 * i], k2 = w[2 * i + 1];
        k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
        h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
        k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
        h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
    }
    if constexpr (rem > 8) {
        uint64_t k2 = w[2 * nblocks + 1];
        k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
    }
    if constexpr (rem > 0) {
        uint64_t k1 = w[2 * nblocks];
        k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
    }
    h1 ^= (uint64_t)K; h2 ^= (uint64_t)K;
    h1 += h2; h2 += h1;
    h1 = fmix64(h1); h2 = fmix64(h2);
    return h1 + h2;
}

// --------------------------------------------------- synthetic genome family
// Bench input; identical to oracle_synth_base() in
// oracle/mash_oracle.c, which the parity tests hold it against.
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9e3779b97f4a7c15ULL;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
    return x ^ (x >> 31);
}
constexpr uint64_t kSynA = 0xD2E9A5C31F00AB01ULL;
constexpr uint64_t kSynM = 0x5BD1E9955A11CE07ULL;
constexpr uint64_t kSynR = 0x27D4EB2F165667C5ULL;
__host__ __device__ __forceinline__ uint32_t synth_rate_thr(uint32_t i) {
    // {0.1, 0.5, 1, 2, 5, 10, 20} % as fractions of 2^32
    const uint32_t t[7] = {4294967u, 21474836u, 42949673u, 85899346u,
                           214748365u, 429496730u, 858993459u};
    return t[i];
}

// ------------------------------------------------------------------ errors
void set_error(const std::string &msg);

}  // namespace drephip
