// screen.hip -- the shared-hash screen in front of the all-pairs kernels
// (replaces nothing in dRep: an exact shortcut inside `mash dist`,
// drep/d_cluster.py:569-573).
//
// Mash's merge of two sketches that share no hash gives common = 0 and
// denominator min(s, |A| + |B|) (merge_pair, oracle_dist_pair), whatever the
// hash values are.  In a large genome set almost every pair is such a pair:
// at configs[3] (10^5 genomes) 0.2 % of the 5x10^9 pairs share a hash (the
// families, plus ~0.1 % of unrelated pairs that share one by chance).  So the
// all-pairs stage first finds the pairs that share any hash, by grouping the
// N x s sketch entries by value, and runs the merge-equivalent kernels
// (k_allpairs_q / k_allpairs_band in LIST mode) only on those; every other
// pair is written as (0, min(s, |A| + |B|)).  Exact by construction: the
// screen keeps a superset of the pairs with a nonzero count.
//
//   keys    entry (g, k), k < nhash[g]: key lo32(H[g][k]), value g * s + k
//   sort    radix sort of the (key, value) pairs on the 32-bit key (rocPRIM
//           through hipCUB): equal hashes become adjacent
//   runs    runs of >= 2 equal keys, counted and written per block in two
//           passes; sum of m(m-1)/2 = the pair checks the marking will make;
//           two-entry runs kept apart
//   mark    runs of >= 3 in first-genome order, a workgroup per 256 runs:
//           every pair of a run's entries with equal 64-bit hashes marks cell
//           (row tile of the smaller genome, larger genome) in a bitmap
//           [row tiles][N bits] through an LDS window of it; two-entry runs
//           go to a pair map (k_screen_mark2), and a pair sharing exactly one
//           hash, both sketches full, is written by the screen itself
//           (common = rank sum < s, k_screen_simple) instead of marked
//   lists   per row tile: its marked columns in ascending order and its work
//           items {i0, list offset, count <= C, 0} for the LIST kernels
//
// When the run sum says the set is dense (many related genomes: marking
// would cost more than the kernels save) the caller runs the dense path.
// Roofline: the sort (HBM/LDS-bound, ~16 B per entry per pass) and the
// marking (L2 loads, one per pair check); both O(N s + shared pairs) against
// the dense kernels' O(N^2 s).

#include "ctx.h"
#include "../../include/drephip.h"

#include <hipcub/device/device_radix_sort.hpp>
#include <hipcub/device/device_scan.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace drephip {

constexpr int kScWG = 256;
constexpr uint32_t kItemBlock = 32;          // row tiles per XCD block of the LIST items

// Entry values: g s + k in the low vbits bits (vbits = the bits N s needs),
// and in the bits above them, when there are any, the low bits of the hash's
// high word -- a fingerprint: two entries of one run (equal low words) whose
// fingerprints differ hold different hashes, with no read of the hashes
// (k_screen_mark).  Every reader masks the index with vmask.
__device__ __forceinline__ uint32_t entry_val(uint32_t idx, uint64_t h, uint32_t vbits) {
    return vbits >= 32 ? idx : idx | ((uint32_t)(h >> 32) << vbits);
}
// every entry (g, k < nhash[g]) at eoff[g] + k; one workgroup per genome
__global__ __launch_bounds__(kScWG) void k_screen_keys(const uint64_t *__restrict__ H, const uint32_t *__restrict__ nh,
                                                       const uint64_t *__restrict__ eoff, uint32_t s, uint32_t vbits,
                                                       uint32_t *__restrict__ keys, uint32_t *__restrict__ vals) {
    const uint32_t g = blockIdx.x;
    const uint32_t n = nh[g];
    const uint64_t o = eoff[g];
    const uint64_t *A = H + (uint64_t)g * s;
    for (uint32_t k = threadIdx.x; k < n; k += kScWG) {
        const uint64_t h = A[k];
        keys[o + k] = (uint32_t)h;
        vals[o + k] = entry_val(g * s + k, h, vbits);
    }
}

// total entry count after the exclusive scan of nhash (eoff[N] = eoff[N-1] + nh[N-1])
__global__ void k_screen_total(const uint32_t *__restrict__ nh, uint64_t *__restrict__ eoff, uint32_t N) {
    if (threadIdx.x == 0) eoff[N] = eoff[N - 1] + nh[N - 1];
}

// one counter bump per workgroup: the waves' sums through LDS (a bump per wave
// from thousands of workgroups serialised on the counter: ~0.2 ms)
__device__ __forceinline__ void block_count_add(uint32_t mine, unsigned long long *counter) {
    __shared__ uint32_t red[kScWG / 64];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mine += __shfl_xor(mine, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mine;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < kScWG / 64; w++) t += red[w];
        if (t) atomicAdd(counter, (unsigned long long)t);
    }
}

// Hash parts (the sharded screen, screen_part_impl): part p of P holds the
// hashes in the value range [bnd[p - 1], bnd[p]) (bnd[-1] = 0, bnd[P - 1] =
// infinity).  Equal hashes share a part, and as a sketch is ascending, a
// genome's entries of one part are one contiguous range of its row, found by
// two binary searches: a part's entries are read from 1/P of the matrix.
// (The first sharded screen cut the parts by low word, which left every run
// of equal keys whole but read all N s entries twice per part: 0.36 of its
// 1.48 ms at configs[4], W = 8.)  A run of equal low words in one part holds
// only that part's hashes, so low-word collisions across parts fall apart --
// fewer pairwise checks, the same marks.
//
// A bottom-s sketch holds the s smallest hashes of its genome, ~uniform on
// [0, T_g] with T_g set by the genome's k-mer count, so fixed cuts of the
// 64-bit range would put every entry in part 0.  bnd[p - 1] is the median
// over (up to 1024 evenly spaced) genomes of the genome's own p/P quantile
// A_g[n_g p / P]: every rank computes the same cuts from the same gathered
// sketches, and a part holds ~1/P of a typical genome's entries.  (Medians of
// nondecreasing sequences are nondecreasing: the cuts are ordered.)
constexpr uint32_t kBndSample = 1024;
__global__ __launch_bounds__(kBndSample) void k_part_bounds(const uint64_t *__restrict__ H,
                                                            const uint32_t *__restrict__ nh, uint32_t N, uint32_t s,
                                                            uint32_t nparts, uint64_t *__restrict__ bnd) {
    __shared__ uint64_t v[kBndSample];
    const uint32_t p = blockIdx.x + 1, t = threadIdx.x;
    const uint32_t ns = N < kBndSample ? N : kBndSample;
    uint64_t x = ~0ull;                                                // no sample: sorts last
    if (t < ns) {
        const uint32_t g = (uint32_t)((uint64_t)t * N / ns), n = nh[g];
        if (n) x = H[(uint64_t)g * s + (uint64_t)n * p / nparts];
    }
    const uint32_t valid = __syncthreads_count(x != ~0ull);
    v[t] = x;
    for (uint32_t k = 2; k <= kBndSample; k <<= 1)                     // bitonic sort, ascending
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            __syncthreads();
            const uint32_t o = t ^ j;
            if (o > t) {
                const uint64_t a = v[t], b = v[o];
                if ((a > b) == ((t & k) == 0)) {
                    v[t] = b;
                    v[o] = a;
                }
            }
        }
    __syncthreads();
    if (t == 0) bnd[p - 1] = valid ? v[valid / 2] : ~0ull;
}
// first k in [0, n) with A[k] >= x (A ascending)
__device__ __forceinline__ uint32_t lower_bound_u64(const uint64_t *__restrict__ A, uint32_t n, uint64_t x) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (A[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
// the part's range [beg[g], beg[g] + cnt[g]) of every genome's row
__global__ __launch_bounds__(kScWG) void k_part_range(const uint64_t *__restrict__ H, const uint32_t *__restrict__ nh,
                                                      const uint64_t *__restrict__ bnd, uint32_t N, uint32_t s,
                                                      uint32_t part, uint32_t nparts, uint32_t *__restrict__ beg,
                                                      uint32_t *__restrict__ cnt) {
    const uint32_t g = blockIdx.x * kScWG + threadIdx.x;
    if (g >= N) return;
    const uint32_t n = nh[g];
    const uint64_t *A = H + (uint64_t)g * s;
    const uint32_t b = part == 0 ? 0 : lower_bound_u64(A, n, bnd[part - 1]);
    const uint32_t e = part + 1 >= nparts ? n : b + lower_bound_u64(A + b, n - b, bnd[part]);
    beg[g] = b;
    cnt[g] = e - b;
}
// the part's entries in genome order (the sorted runs list their genomes in
// ascending order, as k_screen_keys' full set does): one wave per genome
// copies its range
constexpr uint32_t kPartWaves = kScWG / 64;
__global__ __launch_bounds__(kScWG) void k_part_keys(const uint64_t *__restrict__ H, const uint32_t *__restrict__ beg,
                                                     const uint32_t *__restrict__ cnt, const uint64_t *__restrict__ eoff,
                                                     uint32_t N, uint32_t s, uint32_t vbits, uint32_t *__restrict__ keys,
                                                     uint32_t *__restrict__ vals) {
    const uint32_t g = blockIdx.x * kPartWaves + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (g >= N) return;                                                // wave-uniform
    const uint32_t b = beg[g], n = cnt[g];
    const uint64_t o = eoff[g];
    const uint64_t *A = H + (uint64_t)g * s + b;
#pragma unroll 4
    for (uint32_t k = lane; k < n; k += 64) {
        const uint64_t h = A[k];
        keys[o + k] = (uint32_t)h;
        vals[o + k] = entry_val(g * s + b + k, h, vbits);
    }
}

// Runs of equal keys in the sorted keys, without a serial walk: the heads
// (position 0 and every key change) counted per chunk of the sorted keys
// (k_head_count), the counts scanned, and each chunk writing its heads' run
// bounds at its offset in order (k_head_write): run r = [rstart[r], rend[r]).
// Two read passes over the keys (round 5 wrote a head flag per position,
// scanned all M of them and read them back: 1.1 ms at 10^8 entries).  (A head
// thread walking its run measured 35.6 ms at 10^8 entries, the walks'
// dependent loads holding every wave with a head.)
__global__ __launch_bounds__(kScWG) void k_head_count(const uint32_t *__restrict__ keys, uint32_t M, uint32_t chunk,
                                                      uint32_t *__restrict__ bcount) {
    __shared__ uint32_t red[kScWG / 64];
    const uint32_t i0 = blockIdx.x * chunk, i1 = min(i0 + chunk, M);
    uint32_t c = 0;
    for (uint32_t i = i0 + threadIdx.x; i < i1; i += kScWG) c += i == 0 || keys[i - 1] != keys[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < kScWG / 64; w++) t += red[w];
        bcount[blockIdx.x] = t;
    }
}
__device__ __forceinline__ uint32_t block_exclusive_count(bool f, uint32_t *wsum, uint32_t *total);
__global__ __launch_bounds__(kScWG) void k_head_write(const uint32_t *__restrict__ keys, uint32_t M, uint32_t chunk,
                                                      const uint32_t *__restrict__ boff, uint32_t nb,
                                                      uint32_t *__restrict__ rstart, uint32_t *__restrict__ rend) {
    __shared__ uint32_t wsum[kScWG / 64];
    const uint32_t i0 = blockIdx.x * chunk, i1 = min(i0 + chunk, M);
    uint32_t r0 = boff[blockIdx.x];
    for (uint32_t ib = i0; ib < i1; ib += kScWG) {                    // uniform trip count
        const uint32_t i = ib + threadIdx.x;
        const bool head = i < i1 && (i == 0 || keys[i - 1] != keys[i]);
        uint32_t tot;
        const uint32_t r = r0 + block_exclusive_count(head, wsum, &tot);
        if (head) {
            rstart[r] = i;
            if (r > 0) rend[r - 1] = i;                                // the previous run ends here
        }
        r0 += tot;
    }
    if (blockIdx.x == nb - 1 && threadIdx.x == 0) rend[boff[nb] - 1] = M;
}

// runs of >= 2 entries: (start, length) and their first (smallest) genome --
// a run lists its entries in ascending genome order (the radix sort is
// stable and the keys were written genome by genome).  Two passes over the
// same contiguous blocks of runs, no contended atomics: k_run_count counts
// each block's runs of >= 2 (cnt[b]) and their pair checks (chk[b]); after a
// scan of the counts k_run_write writes each block's runs at its offset, in
// order.  (One atomic counter for all ~5x10^6 runs serialised the pass:
// 16 ms at 10^8 entries.)
constexpr uint32_t kRunBlocks = 4096;
__device__ __forceinline__ uint32_t block_exclusive_count(bool f, uint32_t *wsum, uint32_t *total) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t mask = __ballot(f);
    const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
    if (lane == 0) wsum[wave] = (uint32_t)__popcll(mask);
    __syncthreads();
    uint32_t base = 0, tot = 0;
    for (uint32_t w = 0; w < kScWG / 64; w++) {
        if (w < wave) base += wsum[w];
        tot += wsum[w];
    }
    __syncthreads();
    *total = tot;
    return base + below;
}

__global__ __launch_bounds__(kScWG) void k_run_count(const uint32_t *__restrict__ rstart,
                                                     const uint32_t *__restrict__ rend, uint32_t nr, uint32_t per,
                                                     uint32_t *__restrict__ cnt2, uint32_t *__restrict__ cnt3,
                                                     unsigned long long *__restrict__ chk) {
    __shared__ uint32_t wsum[2][kScWG / 64];
    __shared__ unsigned long long esum[kScWG / 64];
    const uint32_t r0 = blockIdx.x * per, r1 = min(r0 + per, nr);
    uint32_t c2 = 0, c3 = 0;
    unsigned long long e = 0;
    for (uint32_t r = r0 + threadIdx.x; r < r1; r += kScWG) {
        const uint32_t m = rend[r] - rstart[r];
        c2 += m == 2;
        c3 += m >= 3;
        if (m >= 2) e += (unsigned long long)m * (m - 1) / 2;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        c2 += __shfl_xor(c2, o, 64);
        c3 += __shfl_xor(c3, o, 64);
        e += __shfl_xor(e, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        wsum[0][threadIdx.x >> 6] = c2;
        wsum[1][threadIdx.x >> 6] = c3;
        esum[threadIdx.x >> 6] = e;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t2 = 0, t3 = 0;
        unsigned long long te = 0;
        for (int w = 0; w < kScWG / 64; w++) { t2 += wsum[0][w]; t3 += wsum[1][w]; te += esum[w]; }
        cnt2[blockIdx.x] = t2;
        cnt3[blockIdx.x] = t3;
        chk[blockIdx.x] = te;
    }
}

// the runs of two entries (chance sharing, mostly) as their start positions
// (pairs), the longer ones with their first genome (runs, rfirst, ridx)
__global__ __launch_bounds__(kScWG) void k_run_write(const uint32_t *__restrict__ rstart,
                                                     const uint32_t *__restrict__ rend, uint32_t nr, uint32_t per,
                                                     const uint32_t *__restrict__ off2, const uint32_t *__restrict__ off3,
                                                     const uint32_t *__restrict__ vals, uint32_t s, uint32_t vmask,
                                                     uint32_t *__restrict__ pairs, uint2 *__restrict__ runs,
                                                     uint32_t *__restrict__ rfirst, uint32_t *__restrict__ ridx) {
    __shared__ uint32_t wsum[kScWG / 64];
    const uint32_t r0 = blockIdx.x * per, r1 = min(r0 + per, nr);
    uint32_t b2 = off2[blockIdx.x], b3 = off3[blockIdx.x];
    for (uint32_t rb = r0; rb < r1; rb += kScWG) {                  // uniform trip count
        const uint32_t r = rb + threadIdx.x;
        uint32_t st = 0, m = 0;
        if (r < r1) { st = rstart[r]; m = rend[r] - st; }
        uint32_t t2, t3;
        const uint32_t q2 = b2 + block_exclusive_count(m == 2, wsum, &t2);
        const uint32_t q3 = b3 + block_exclusive_count(m >= 3, wsum, &t3);
        if (m == 2) pairs[q2] = st;
        if (m >= 3) {
            runs[q3] = make_uint2(st, m);
            rfirst[q3] = (vals[st] & vmask) / s;
            ridx[q3] = q3;
        }
        b2 += t2;
        b3 += t3;
    }
}

// Runs of two entries (chance sharing, mostly): one lane each.  Two genomes
// holding one 64-bit hash go into a pair map (key (a, b), a < b; how many
// such runs hold the pair; the hash's positions i in a and j in b) instead of
// the bitmap: a pair that shares exactly one hash has count (i + j < s) --
// the hash's rank in A u B is i + j -- and needs no kernel (k_screen_simple).
// Chunk masks for the dense all-pairs kernel (the screen's verdict "dense"):
// bit k of cmask[g] is set when 64-element chunk k of sketch g holds a
// position the whole-row kernel must confirm by the hash's high word -- a
// position at or past nhash[g] (padding, or past s: those lanes read 0), or an
// entry whose low word (the sort key) another, different 64-bit hash of the
// matrix shares.  A probe hit on a clear chunk then needs no high-word read:
// the row key it found has the column element's low word, and no other hash
// has that low word (k_allpairs_q, probe_rows_v).  Exact: a run of equal keys
// is clean only when every entry's 64-bit hash equals the first's.
//
// Positions past nhash read UINT64_MAX (padding) or 0 (past s, through the
// buffer bounds): harmless unless some entry of the matrix has the low word
// 0xFFFFFFFF or 0 -- the sorted keys' last and first -- and only then are
// their chunks flagged.
__global__ __launch_bounds__(kScWG) void k_cmask_init(const uint32_t *__restrict__ nh, uint32_t N,
                                                      const uint32_t *__restrict__ keys, uint32_t M,
                                                      uint32_t *__restrict__ cmask) {
    const uint32_t g = blockIdx.x * kScWG + threadIdx.x;
    if (g >= N) return;
    const bool edge = keys[0] == 0u || keys[M - 1] == 0xFFFFFFFFu;
    const uint32_t first = nh[g] / 64;                             // the first chunk holding a position >= nhash
    cmask[g] = (!edge || first >= 32) ? 0u : ~0u << first;
}
// runs of two: one lane each
__global__ __launch_bounds__(kScWG) void k_cmask_pairs(const uint32_t *__restrict__ vals, const uint64_t *__restrict__ H,
                                                       uint32_t s, uint32_t vmask, const uint32_t *__restrict__ pairs,
                                                       uint32_t n2, uint32_t *__restrict__ cmask) {
    for (uint32_t i = blockIdx.x * kScWG + threadIdx.x; i < n2; i += gridDim.x * kScWG) {
        const uint32_t st = pairs[i];
        const uint32_t a = vals[st] & vmask, b = vals[st + 1] & vmask;    // g s + k
        if (H[a] != H[b]) {
            atomicOr(&cmask[a / s], 1u << ((a % s) / 64));
            atomicOr(&cmask[b / s], 1u << ((b % s) / 64));
        }
    }
}
// runs of three or more: one wave each (grid-stride over the runs)
__global__ __launch_bounds__(kScWG) void k_cmask_runs(const uint32_t *__restrict__ vals, const uint64_t *__restrict__ H,
                                                      uint32_t s, uint32_t vmask, const uint2 *__restrict__ runs,
                                                      uint32_t nruns, uint32_t *__restrict__ cmask) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nw = gridDim.x * (kScWG / 64);
    for (uint32_t r = blockIdx.x * (kScWG / 64) + (threadIdx.x >> 6); r < nruns; r += nw) {     // wave-uniform
        const uint2 run = runs[r];
        const uint64_t h0 = H[vals[run.x] & vmask];
        bool mixed = false;
        for (uint32_t e = lane; e < run.y; e += 64) mixed |= H[vals[run.x + e] & vmask] != h0;
        if (__ballot(mixed) == 0) continue;
        for (uint32_t e = lane; e < run.y; e += 64) {
            const uint32_t v = vals[run.x + e] & vmask;
            atomicOr(&cmask[v / s], 1u << ((v % s) / 64));
        }
    }
}

constexpr uint64_t kPairEmpty = ~0ull;
constexpr uint64_t kMaxPairMap = 1ull << 30;   // pair-map slots (16 B each); above it the screen gives way
constexpr uint64_t kLightBudget = 1ull << 30;  // bytes of the light screen's per-cell run ids (sc_crun)
__device__ __forceinline__ uint32_t pair_slot(uint64_t key, uint32_t mask) {
    uint64_t h = key * 0x9E3779B97F4A7C15ull;
    return (uint32_t)(h >> 32) & mask;
}
__global__ __launch_bounds__(kScWG) void k_screen_mark2(const uint32_t *__restrict__ vals, const uint64_t *__restrict__ H,
                                                        uint32_t s, uint32_t vmask, const uint32_t *__restrict__ pairs, uint32_t n2,
                                                        uint32_t row0, uint32_t row1,
                                                        unsigned long long *__restrict__ pkey, uint32_t *__restrict__ pcnt,
                                                        uint32_t *__restrict__ ppos, uint32_t pmask) {
    for (uint32_t q = blockIdx.x * kScWG + threadIdx.x; q < n2; q += gridDim.x * kScWG) {
        const uint32_t st = pairs[q];
        const uint32_t ix = vals[st] & vmask, iy = vals[st + 1] & vmask;
        const uint32_t gx = ix / s, gy = iy / s;          // gx <= gy (a run is in genome order)
        if (gx == gy || gx < row0 || gx >= row1 || H[ix] != H[iy]) continue;
        const unsigned long long key = ((unsigned long long)gx << 32) | gy;
        for (uint32_t slot = pair_slot(key, pmask);; slot = (slot + 1) & pmask) {
            const unsigned long long k = atomicCAS(&pkey[slot], kPairEmpty, key);
            if (k == kPairEmpty) {                        // first run of this pair: its positions
                ppos[slot] = ((ix - gx * s) << 16) | (iy - gy * s);
                atomicAdd(&pcnt[slot], 1u);
                break;
            }
            if (k == key) { atomicAdd(&pcnt[slot], 1u); break; }
        }
    }
}

// The sharded screen's runs of two: instead of this part's own pair map, one
// record {a, b, (i << 16) | j, 0} per run whose two entries hold one 64-bit hash
// in two genomes (a < b; i, j their positions), for every row: the rank owning
// row a builds the pair map from every part's records (k_screen_map2).  One
// device counter, bumped once per wave.
__global__ __launch_bounds__(kScWG) void k_screen_emit2(const uint32_t *__restrict__ vals, const uint64_t *__restrict__ H,
                                                        uint32_t s, uint32_t vmask, const uint32_t *__restrict__ pairs, uint32_t n2,
                                                        uint4 *__restrict__ rec, uint32_t *__restrict__ nrec) {
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t q0 = blockIdx.x * kScWG; q0 < n2; q0 += gridDim.x * kScWG) {   // wave-uniform trip count
        const uint32_t q = q0 + threadIdx.x;
        bool ok = false;
        uint32_t ix = 0, iy = 0, gx = 0, gy = 0;
        if (q < n2) {
            const uint32_t st = pairs[q];
            ix = vals[st] & vmask;
            iy = vals[st + 1] & vmask;
            gx = ix / s;
            gy = iy / s;
            ok = gx != gy && H[ix] == H[iy];
        }
        const uint64_t m = __ballot(ok);
        if (m == 0) continue;
        uint32_t base = 0;
        if (lane == (uint32_t)(__ffsll((long long)m) - 1)) base = atomicAdd(nrec, (uint32_t)__popcll(m));
        base = __shfl(base, __ffsll((long long)m) - 1, 64);
        if (ok) {
            const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
            rec[base + below] = make_uint4(gx, gy, ((ix - gx * s) << 16) | (iy - gy * s), 0u);
        }
    }
}

// the records of rows [row0, row1) (the pair map's size); one counter bump per wave
__global__ __launch_bounds__(kScWG) void k_rec_count(const uint4 *__restrict__ rec, uint64_t nrec, uint32_t row0,
                                                     uint32_t row1, unsigned long long *__restrict__ cnt) {
    uint32_t mine = 0;
    for (uint64_t q = (uint64_t)blockIdx.x * kScWG + threadIdx.x; q < nrec; q += (uint64_t)gridDim.x * kScWG) {
        const uint32_t a = rec[q].x;
        mine += a >= row0 && a < row1;
    }
    block_count_add(mine, cnt);
}

// the pair map of rows [row0, row1) from every part's records (k_screen_emit2):
// the insert of k_screen_mark2
__global__ __launch_bounds__(kScWG) void k_screen_map2(const uint4 *__restrict__ rec, uint64_t nrec, uint32_t row0,
                                                       uint32_t row1, unsigned long long *__restrict__ pkey,
                                                       uint32_t *__restrict__ pcnt, uint32_t *__restrict__ ppos,
                                                       uint32_t pmask) {
    for (uint64_t q = (uint64_t)blockIdx.x * kScWG + threadIdx.x; q < nrec; q += (uint64_t)gridDim.x * kScWG) {
        const uint4 r = rec[q];
        if (r.x < row0 || r.x >= row1) continue;
        const unsigned long long key = ((unsigned long long)r.x << 32) | r.y;
        for (uint32_t slot = pair_slot(key, pmask);; slot = (slot + 1) & pmask) {
            const unsigned long long k = atomicCAS(&pkey[slot], kPairEmpty, key);
            if (k == kPairEmpty) {
                ppos[slot] = r.z;
                atomicAdd(&pcnt[slot], 1u);
                break;
            }
            if (k == key) { atomicAdd(&pcnt[slot], 1u); break; }
        }
    }
}

// A part's marks leave as cell words: every nonzero word of its bitmap as
// {row tile T (rows [T R, (T + 1) R) from row 0), word w (columns 32 w ..
// 32 w + 31), bits, 0} -- ~1 record per marked cell word, against N^2 / (32 R)
// words of the whole bitmap (312 MB per part at 10^5 genomes).  Counted per
// chunk, scanned, written in order.
__global__ __launch_bounds__(kScWG) void k_cells_count(const uint32_t *__restrict__ bm, uint64_t nwords, uint32_t chunk,
                                                       uint32_t *__restrict__ bcount) {
    __shared__ uint32_t red[kScWG / 64];
    const uint64_t i0 = (uint64_t)blockIdx.x * chunk, i1 = min(i0 + chunk, nwords);
    uint32_t c = 0;
    for (uint64_t i = i0 + threadIdx.x; i < i1; i += kScWG) c += bm[i] != 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < kScWG / 64; w++) t += red[w];
        bcount[blockIdx.x] = t;
    }
}
__global__ __launch_bounds__(kScWG) void k_cells_write(const uint32_t *__restrict__ bm, uint64_t nwords, uint32_t chunk,
                                                       const uint32_t *__restrict__ boff, uint32_t NW,
                                                       uint4 *__restrict__ cells) {
    __shared__ uint32_t wsum[kScWG / 64];
    const uint64_t i0 = (uint64_t)blockIdx.x * chunk, i1 = min(i0 + chunk, nwords);
    uint32_t o = boff[blockIdx.x];
    for (uint64_t ib = i0; ib < i1; ib += kScWG) {                    // uniform trip count
        const uint64_t i = ib + threadIdx.x;
        const uint32_t v = i < i1 ? bm[i] : 0u;
        uint32_t tot;
        const uint32_t q = o + block_exclusive_count(v != 0, wsum, &tot);
        if (v) cells[q] = make_uint4((uint32_t)(i / NW), (uint32_t)(i % NW), v, 0u);
        o += tot;
    }
}
// A rank's bitmap from every part's cell words: the cell's rows clipped to
// [row0, row1) and OR-ed into the rank's tiles (rows from row0).  With tile-
// aligned rank boundaries (parallel.row_partition) a part's tile is one of
// the rank's; otherwise it covers two, each getting the whole word -- a
// superset (an extra cell costs kernel work, never exactness: the kernels
// rewrite every pair of a marked cell).
__global__ __launch_bounds__(kScWG) void k_cells_scatter(const uint4 *__restrict__ cells, uint64_t ncells, uint32_t row0,
                                                         uint32_t row1, uint32_t rshift, uint32_t NW,
                                                         uint32_t *__restrict__ bm) {
    for (uint64_t q = (uint64_t)blockIdx.x * kScWG + threadIdx.x; q < ncells; q += (uint64_t)gridDim.x * kScWG) {
        const uint4 c = cells[q];
        const uint64_t ra = max((uint64_t)c.x << rshift, (uint64_t)row0);
        const uint64_t rb = min(((uint64_t)c.x + 1) << rshift, (uint64_t)row1);
        if (ra >= rb) continue;                                        // not this rank's rows
        const uint32_t ta = (uint32_t)((ra - row0) >> rshift), tb = (uint32_t)((rb - 1 - row0) >> rshift);
        for (uint32_t t = ta; t <= tb; t++) atomicOr(bm + (uint64_t)t * NW + c.y, c.z);
    }
}

// The pair map: a pair held by one run of two with both sketches full shares
// exactly one hash unless a longer run holds it too -- and then that run has
// marked its cell -- so when its cell is unmarked its count is written here,
// (i + j < s), over the no-shared-hash fill (the denominator, s, is already
// right).  Pairs held by several runs, or with a partial sketch (whose
// denominator depends on the merge), mark their cell for the LIST kernel,
// which runs after this and rewrites every pair of a marked cell exactly.
__global__ __launch_bounds__(kScWG) void k_screen_simple(const unsigned long long *__restrict__ pkey,
                                                         const uint32_t *__restrict__ pcnt,
                                                         const uint32_t *__restrict__ ppos, uint32_t pcap,
                                                         const uint32_t *__restrict__ nh, uint32_t s, uint32_t N,
                                                         uint32_t row0, uint32_t rshift, uint32_t NW,
                                                         uint64_t seg0, uint32_t *__restrict__ bm,
                                                         uint32_t *__restrict__ bmH,
                                                         uint16_t *__restrict__ common, unsigned long long *__restrict__ nsimple) {
    uint32_t mine = 0;
    for (uint32_t q = blockIdx.x * kScWG + threadIdx.x; q < pcap; q += gridDim.x * kScWG) {
        const unsigned long long key = pkey[q];
        if (key == kPairEmpty) continue;
        const uint32_t a = (uint32_t)(key >> 32), b = (uint32_t)key;
        const uint64_t wo = (uint64_t)((a - row0) >> rshift) * NW + (b >> 5);
        uint32_t *w = bm + wo;
        const uint32_t bit = 1u << (b & 31);
        // (bmH, the light screen's heavy cells: the cell needs the LIST kernel)
        if (pcnt[q] >= 2 || nh[a] != s || nh[b] != s) {
            atomicOr(w, bit);
            if (bmH) atomicOr(bmH + wo, bit);
            continue;
        }
        if (*w & bit) {                                               // a longer run holds the pair too
            if (bmH) atomicOr(bmH + wo, bit);
            continue;
        }
        const uint32_t pos = ppos[q];
        const uint64_t o = (uint64_t)a * N - (uint64_t)a * (a + 1) / 2 + (b - a - 1) - seg0;
        common[o] = (uint16_t)(((pos >> 16) + (pos & 0xFFFFu)) < s ? 1 : 0);
        mine++;
    }
    block_count_add(mine, nsimple);
}

// Marking, one workgroup per chunk of kMarkChunk runs taken in order of their
// first genome (runs sorted by it): a family's runs -- each of its ~10^3
// shared hashes is one -- land in the same few chunks, so their pairs are
// OR-ed into an LDS window of the bitmap (kMarkTiles row tiles from the
// chunk's first genome x kMarkCols columns; rows padded to 65 words so the
// tiles of one column sit in different banks) and each window word reaches
// HBM once, by one atomicOr.  Pairs outside the window (chance sharing across
// families) go to the bitmap directly.  Inside a run a wave compares every
// entry pair: lane = x entry, the y entries broadcast by readlane; a pair of
// equal 64-bit hashes of two genomes marks (row tile of gx, gy), gx < gy.
// The x entries are in ascending genome order, so lanes of one row tile are
// adjacent: only the first ok lane of each tile marks (one LDS atomic per
// tile and y, none on a shared word).
// (Marking a collision run whole, without any same-hash test and with the
// light screen checking each pair's hashes, left 4.8x the cells to the
// kernels at configs[4] -- 770k vs 159k, band LIST kernel 9.2 vs 4.0 ms: such
// runs are not rare among 10^8 entries and span two families' genomes.  The
// fingerprint test below keeps them apart without the hash reads.)
#ifndef DREPHIP_SC_ABL
#define DREPHIP_SC_ABL 0    // timing ablations (never the product): 1 no marking by same-hash runs, 2 no same-hash check
#endif
constexpr uint32_t kMarkWG = 1024;
constexpr uint32_t kFpBits = 4;      // fingerprint bits from which the same-hash test reads no hashes
constexpr uint32_t kMarkChunk = 256;
constexpr uint32_t kMarkTiles = 128;
constexpr uint32_t kMarkCols = 2048;
constexpr uint32_t kMarkWords = kMarkCols / 32;
constexpr uint32_t kMarkStride = kMarkWords + 1;
template <bool LIGHT>
__global__ __launch_bounds__(kMarkWG) void k_screen_mark(const uint32_t *__restrict__ vals, const uint64_t *__restrict__ H,
                                                       uint32_t s, uint32_t vbits, const uint2 *__restrict__ runs,
                                                       const uint32_t *__restrict__ order,
                                                       const uint32_t *__restrict__ rfirst_sorted, uint32_t nruns,
                                                       uint32_t row0, uint32_t row1, uint32_t rshift, uint32_t NW,
                                                       uint32_t *__restrict__ bm, uint32_t *__restrict__ bmH,
                                                       uint32_t *__restrict__ crun, uint32_t N) {
    __shared__ uint32_t win[kMarkTiles * kMarkStride];
    __shared__ uint32_t winH[LIGHT ? kMarkTiles * kMarkStride : 1];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t q0 = blockIdx.x * kMarkChunk;
    const uint32_t q1 = min(q0 + kMarkChunk, nruns);
    for (uint32_t i = threadIdx.x; i < kMarkTiles * kMarkStride; i += kMarkWG) {
        win[i] = 0;
        if (LIGHT) winH[i] = 0;
    }
    // window: row tiles [t_lo, t_lo + kMarkTiles), columns [c_lo, c_lo + kMarkCols)
    const uint32_t g_lo = rfirst_sorted[q0];
    const uint32_t t_lo = g_lo > row0 ? (g_lo - row0) >> rshift : 0;
    const uint32_t c_lo = g_lo & ~31u;
    __syncthreads();
    // one cell mark: the LDS window when (tile, column) falls in it, else the
    // bitmap.  LIGHT: a cell marked before (by another run) goes to the heavy
    // bitmap (winH / bmH); a cell marked for the first time records the run
    // (crun), and a run whose entries do not all hold one hash (`heavy`) marks
    // its cells heavy at once
    auto mark = [&](uint32_t t, uint32_t col, uint32_t bits, uint32_t run_id, bool heavy) {
        uint32_t old;
        if (t - t_lo < kMarkTiles && col - c_lo < kMarkCols) {
            const uint32_t wi = (t - t_lo) * kMarkStride + ((col - c_lo) >> 5);
            old = atomicOr(&win[wi], bits);
            if (LIGHT && ((old & bits) || heavy)) atomicOr(&winH[wi], heavy ? bits : old & bits);
        } else {
            old = atomicOr(bm + (uint64_t)t * NW + (col >> 5), bits);
            if (LIGHT && ((old & bits) || heavy)) atomicOr(bmH + (uint64_t)t * NW + (col >> 5), heavy ? bits : old & bits);
        }
        if (LIGHT && !heavy) {
            uint32_t nb = bits & ~old;
            while (nb) {
                const uint32_t b = __ffs(nb) - 1;
                nb &= nb - 1;
                crun[(uint64_t)t * N + (col & ~31u) + b] = run_id;
            }
        }
    };
    for (uint32_t q = q0 + wave; q < q1; q += kMarkWG / 64) {
        const uint32_t run_id = order[q];
        const uint2 run = runs[run_id];
        const uint32_t start = run.x, m = run.y;
        // a run whose entries all hold one 64-bit hash (a hash shared by m
        // genomes; only a low-word collision breaks this) takes the fast path.
        // With >= kFpBits fingerprint bits in the entry values the test reads
        // only the values: different fingerprints, different hashes (the slow
        // path); equal ones are taken as one hash -- a collision run whose
        // fingerprints agree (1 in 2^fbits) then marks a superset, which the
        // kernels and the light screen's hash check (k_screen_light) resolve.
        // Without them, every entry's hash is read (~1.3 of the marking's 3.5 ms
        // at configs[4] when it was the only test)
        bool same = true;
        const uint32_t vmask = vbits >= 32 ? 0xFFFFFFFFu : (1u << vbits) - 1;
#if DREPHIP_SC_ABL != 2
        if (32 - vbits >= kFpBits) {
            const uint32_t f0 = vals[start] >> vbits;
            for (uint32_t b = 0; b < m && same; b += 64) {
                const uint32_t x = b + lane;
                const uint32_t f = x < m ? vals[start + x] >> vbits : f0;
                same = __ballot(f != f0) == 0;
            }
        } else {
            const uint64_t v0 = H[vals[start] & vmask];
            for (uint32_t b = 0; b < m && same; b += 64) {
                const uint32_t x = b + lane;
                const uint64_t v = x < m ? H[vals[start + x] & vmask] : v0;
                same = __ballot(v != v0) == 0;
            }
        }
#endif
#if DREPHIP_SC_ABL == 1
        if (same) continue;
#endif
        uint32_t tcarry = 0xFFFFFFFFu;                       // the previous x block's last row tile
        for (uint32_t xb = 0; xb + 1 < m; xb += 64) {
            const uint32_t x = xb + lane;
            const uint32_t ix = vals[start + (x < m ? x : m - 1)] & vmask;
            const uint32_t gx = ix / s;
            const bool x_ok = x < m && gx >= row0 && gx < row1;
            const uint32_t tx = x_ok ? (gx - row0) >> rshift : 0xFFFFFFFFu;
            // first lane of its row tile among the x entries (lanes are in
            // genome order; a tile continued from the previous x block has its
            // head there, which marked every y after it: one mark per run and cell)
            const uint32_t tprev = __shfl_up(tx, 1, 64);
            const bool tile_head = lane == 0 ? tx != tcarry || tx == 0xFFFFFFFFu : tprev != tx;
            tcarry = __builtin_amdgcn_readlane(tx, 63);
            // an x block with no genome among this call's rows marks nothing: a
            // rank of a sharded job walks only its own part of each long run
            // (the run's entries are in genome order, so that part is contiguous)
            if (__ballot(x_ok) == 0) continue;
            for (uint32_t yb = xb; yb < m; yb += 64) {
                const uint32_t yl = yb + lane;
                const bool y_ok = yl < m;
                const uint32_t iyl = vals[start + (y_ok ? yl : m - 1)] & vmask;
                const uint32_t gyl = iyl / s;
                if (same) {
                    // every x before y pairs with y: for each row tile T among the
                    // x entries (its first position p), every y after p marks
                    // (T, gy).  The y lanes' columns, in genome order, form runs
                    // of one bitmap word; each lane holds the OR of its own and the
                    // later bits of its word (a segmented suffix scan), so a tile
                    // costs one atomic per word: the word's first lane after p.
                    const uint32_t word = gyl >> 5;
                    uint32_t suf = y_ok ? 1u << (gyl & 31) : 0u;
#pragma unroll
                    for (int d = 1; d < 64; d <<= 1) {
                        const uint32_t o = __shfl_down(suf, d, 64);
                        const uint32_t ow = __shfl_down(word, d, 64);
                        if (lane + d < 64 && ow == word) suf |= o;
                    }
                    const uint32_t wprev = __shfl_up(word, 1, 64);
                    const bool seg_head = lane == 0 || wprev != word;
                    uint64_t heads = __ballot(x_ok && tile_head);
                    while (heads) {
                        const uint32_t p = (uint32_t)__ffsll((long long)heads) - 1;
                        heads &= heads - 1;
                        const uint32_t T = __builtin_amdgcn_readlane(tx, p);
                        const int32_t qd = (int32_t)(xb + p) - (int32_t)yb;      // y lanes after the tile's first x
                        if (y_ok && (int32_t)lane > qd && (seg_head || (int32_t)lane == qd + 1)) mark(T, gyl, suf, run_id, false);
                    }
                    continue;
                }
                const uint64_t vx = H[ix];
                const uint64_t vyl = H[iyl];
                const uint32_t ny = min(64u, m - yb);
                for (uint32_t yi = 0; yi < ny; yi++) {
                    const uint32_t vlo = __builtin_amdgcn_readlane((uint32_t)vyl, yi);
                    const uint32_t vhi = __builtin_amdgcn_readlane((uint32_t)(vyl >> 32), yi);
                    const uint32_t gy = __builtin_amdgcn_readlane(gyl, yi);
                    // x before y in the run: gx <= gy (gx == gy: two hashes of one
                    // genome with equal low words, never equal hashes)
                    const bool ok = x_ok && x < yb + yi && (uint32_t)vx == vlo && (uint32_t)(vx >> 32) == vhi && gx != gy;
                    const uint64_t okm = __ballot(ok);
                    if (okm == 0) continue;
                    // the first ok lane of each row tile marks (lane - 1 not ok, or another tile)
                    const bool prev_ok = lane > 0 && ((okm >> (lane - 1)) & 1ull);
                    if (!ok || (prev_ok && !tile_head)) continue;
                    mark(tx, gy, 1u << (gy & 31), run_id, true);
                }
            }
        }
    }
    __syncthreads();
    const uint32_t tmax = ((row1 - row0) + (1u << rshift) - 1) >> rshift;
    for (uint32_t i = threadIdx.x; i < kMarkTiles * kMarkStride; i += kMarkWG) {
        const uint32_t v = win[i];
        if (!v) continue;
        const uint32_t t = t_lo + i / kMarkStride, w = (c_lo >> 5) + i % kMarkStride;
        if (t < tmax && w < NW) {
            const uint32_t old = atomicOr(bm + (uint64_t)t * NW + w, v);
            if (LIGHT) {
                const uint32_t hv = winH[i] | (old & v);          // marked here twice, or by another chunk too
                if (hv) atomicOr(bmH + (uint64_t)t * NW + w, hv);
            }
        }
    }
}

// The light cells (round 5): a (row tile, column) cell marked by exactly one
// run of >= 3 entries that all hold one 64-bit hash h, and by no run of two
// (k_screen_simple marks those heavy).  Each of the tile's rows r < c that
// holds h shares exactly h with column c -- a second shared hash would be a
// second run marking the cell -- so its count is (i + j < s), i and j the
// positions of h in r and in c (h's rank in A u B), and its denominator is s
// when both sketches are full: the screen writes it here, over the
// no-shared-hash fill, and the LIST kernel never streams the column.  At
// configs[4] these are most cells: unrelated families sharing one hash by
// chance (each such hash marks family x family cells).  A cell with a partial
// sketch goes heavy.  One thread per bitmap word.
__global__ __launch_bounds__(kScWG) void k_screen_light(const uint32_t *__restrict__ bm, uint32_t *__restrict__ bmH,
                                                        const uint32_t *__restrict__ crun, const uint2 *__restrict__ runs,
                                                        const uint32_t *__restrict__ vals, const uint64_t *__restrict__ H,
                                                        const uint32_t *__restrict__ nh, uint32_t s, uint32_t vmask,
                                                        uint32_t N, uint32_t row0, uint32_t row1, uint32_t R,
                                                        uint32_t NW, uint64_t nwords, uint64_t seg0,
                                                        uint16_t *__restrict__ common,
                                                        unsigned long long *__restrict__ nlight) {
    uint32_t mine = 0;
    for (uint64_t wi = (uint64_t)blockIdx.x * kScWG + threadIdx.x; wi < nwords; wi += (uint64_t)gridDim.x * kScWG) {
        uint32_t L = bm[wi] & ~bmH[wi];
        if (!L) continue;
        const uint32_t t = (uint32_t)(wi / NW), w = (uint32_t)(wi % NW);
        const uint32_t r0 = row0 + t * R;
        uint32_t heavy = 0;
        while (L) {
            const uint32_t b = __ffs(L) - 1;
            L &= L - 1;
            const uint32_t c = w * 32 + b;
            const uint2 run = runs[crun[(uint64_t)t * N + c]];
            // position of genome g's entry in the run (entries in genome order),
            // or -1; dup: g holds a second entry of the run (two hashes of g
            // agreeing in their low word)
            auto find = [&](uint32_t g, bool &dup) -> int32_t {
                uint32_t lo = 0, hi = run.y;
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if ((vals[run.x + mid] & vmask) / s < g) lo = mid + 1; else hi = mid;
                }
                dup = false;
                if (lo < run.y && (vals[run.x + lo] & vmask) / s == g) {
                    dup = lo + 1 < run.y && (vals[run.x + lo + 1] & vmask) / s == g;
                    return (int32_t)((vals[run.x + lo] & vmask) - g * s);
                }
                return -1;
            };
            bool part = nh[c] != s;
            for (uint32_t j = 0; j < R; j++) {
                const uint32_t r = r0 + j;
                if (r >= row1 || r >= c) break;
                part |= nh[r] != s;
            }
            bool dup;
            const int32_t pc = find(c, dup);
            if (part || pc < 0 || dup) { heavy |= 1u << b; continue; }
            // the run may mix hashes that agree in their low word (marked as one
            // by the fingerprint test, k_screen_mark): a row holding another hash
            // of the run than c shares none with c -- a second shared hash would
            // be a second run marking the cell -- unless it holds two of them
            const uint64_t hc = H[(uint64_t)c * s + pc];
            uint32_t wrote = 0;
            for (uint32_t j = 0; j < R; j++) {
                const uint32_t r = r0 + j;
                if (r >= row1 || r >= c) break;
                const int32_t pr = find(r, dup);
                if (pr < 0) continue;                                  // r shares no hash with c
                if (dup) { heavy |= 1u << b; break; }                  // the kernel decides
                if (H[(uint64_t)r * s + pr] != hc) continue;           // another hash of the run: none shared
                const uint64_t o = (uint64_t)r * N - (uint64_t)r * (r + 1) / 2 + (c - r - 1) - seg0;
                common[o] = (uint16_t)((uint32_t)(pr + pc) < s ? 1 : 0);
                wrote++;
            }
            if (!((heavy >> b) & 1u)) mine += wrote;
        }
        if (heavy) atomicOr(bmH + wi, heavy);
    }
    block_count_add(mine, nlight);
}

// per row tile (one workgroup): marked columns -> cnt[t], items -> itc[t]
__global__ __launch_bounds__(kScWG) void k_screen_count(const uint32_t *__restrict__ bm, uint32_t NW, uint32_t C,
                                                        uint32_t *__restrict__ cnt, uint64_t *__restrict__ cnt64,
                                                        uint32_t *__restrict__ itc) {
    __shared__ uint32_t red[kScWG / 64];
    const uint32_t t = blockIdx.x;
    const uint32_t *row = bm + (uint64_t)t * NW;
    uint32_t c = 0;
    for (uint32_t w = threadIdx.x; w < NW; w += kScWG) c += __popc(row[w]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (int k = 0; k < kScWG / 64; k++) tot += red[k];
        cnt[t] = tot;
        cnt64[t] = tot;
        itc[t] = (tot + C - 1) / C;
    }
}

// per row tile (one workgroup): its marked columns in ascending order at
// coff[t] (thread u takes words [u*per, (u+1)*per)).  Item j of tile t goes
// to launch slot ibase[t] + 8 j: slot w runs on XCD w % 8, and the host deals
// blocks of kItemBlock consecutive row tiles to the XCDs, so the tiles of one
// block (a genome family's rows, whose marked columns largely coincide) stream
// their column sketches through one L2 (measured neutral).
__global__ __launch_bounds__(kScWG) void k_screen_lists(const uint32_t *__restrict__ bm, uint32_t NW, uint32_t C,
                                                        uint32_t row0, uint32_t R, const uint32_t *__restrict__ cnt,
                                                        const uint64_t *__restrict__ coff,
                                                        const uint32_t *__restrict__ ibase, uint32_t *__restrict__ clist,
                                                        uint4 *__restrict__ items, int desc) {
    __shared__ uint32_t wsum[kScWG / 64];
    const uint32_t t = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const uint32_t *row = bm + (uint64_t)t * NW;
    const uint32_t per = (NW + kScWG - 1) / kScWG;
    const uint32_t w0 = min(tid * per, NW), w1 = min(w0 + per, NW);
    uint32_t mine = 0;
    for (uint32_t w = w0; w < w1; w++) mine += __popc(row[w]);
    uint32_t inc = mine;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if (lane >= (uint32_t)d) inc += y;
    }
    if (lane == 63) wsum[tid >> 6] = inc;
    __syncthreads();
    uint32_t pos = inc - mine;
    for (uint32_t k = 0; k < (tid >> 6); k++) pos += wsum[k];
    uint32_t *out = clist + coff[t];
    const uint32_t n = cnt[t];
    for (uint32_t w = w0; w < w1; w++) {
        uint32_t bits = row[w];
        while (bits) {
            const uint32_t b = __ffs(bits) - 1;
            bits &= bits - 1;
            // (desc, A/B: descending, so that the row tiles of a family, whose lists
            // end at different columns but share the family's last ones, start together)
            out[desc ? n - 1 - pos : pos] = w * 32 + b;
            pos++;
        }
    }
    const uint32_t ni = (n + C - 1) / C;
    for (uint32_t j = tid; j < ni; j += kScWG)
        items[(uint64_t)ibase[t] + 8ull * j] = make_uint4(row0 + t * R, (uint32_t)(coff[t] + (uint64_t)j * C),
                                                          min(C, n - j * C), 0);
}

// denominators of the unscreened pairs: min(s, |A| + |B|) (no shared hash);
// one workgroup per row of the segment
__global__ __launch_bounds__(kScWG) void k_screen_denoms(const uint32_t *__restrict__ nh, uint32_t s, uint32_t N,
                                                         uint32_t row0, uint64_t seg0, uint16_t *__restrict__ denom) {
    const uint32_t i = row0 + blockIdx.x;
    const uint32_t ni = nh[i];
    const uint64_t o = (uint64_t)i * N - (uint64_t)i * (i + 1) / 2 - seg0;       // cond_index(i, i + 1) - seg0
    for (uint32_t j = i + 1 + threadIdx.x; j < N; j += kScWG) {
        const uint32_t u = ni + nh[j];
        denom[o + (j - i - 1)] = (uint16_t)(u < s ? u : s);
    }
}

// DREPHIP_SCREEN_PROF=1: HIP events between the phases, printed to stderr
struct ScreenProf {
    bool on = getenv("DREPHIP_SCREEN_PROF") != nullptr;
    std::vector<std::pair<const char *, hipEvent_t>> ev;
    void mark(const char *name, hipStream_t st) {
        if (!on) return;
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return;
        (void)hipEventRecord(e, st);
        ev.push_back({name, e});
    }
    ~ScreenProf() {
        if (!on || ev.empty()) return;
        (void)hipEventSynchronize(ev.back().second);
        fprintf(stderr, "[drephip] screen phases (ms):");
        for (size_t i = 1; i < ev.size(); i++) {
            float ms = 0;
            (void)hipEventElapsedTime(&ms, ev[i - 1].second, ev[i].second);
            fprintf(stderr, " %s %.3f", ev[i].first, ms);
        }
        fprintf(stderr, "\n");
        for (auto &p : ev) (void)hipEventDestroy(p.second);
    }
};

template <class I, class T>
static int hip_scan(drephip_ctx *ctx, const char *name, const I *in, T *out, uint32_t n, hipStream_t st) {
    size_t tb = 0;
    HIPC(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, in, out, n, st));
    void *tmp;
    int rc;
    if ((rc = scratch(ctx, name, std::max<size_t>(tb, 16), &tmp))) return rc;
    HIPC(hipcub::DeviceScan::ExclusiveSum(tmp, tb, in, out, n, st));
    return DREPHIP_OK;
}

// ---------------------------------------------------------------- host phases
// front: the entries (all, or one hash part's) grouped by key, and their runs
struct ScreenFront {
    uint32_t vbits = 32, vmask = 0xFFFFFFFFu;   // entry index bits (the rest: hash fingerprint, entry_val)
    uint32_t M = 0;                 // entries grouped
    uint32_t nr = 0;                // distinct keys
    uint32_t n2 = 0, nruns = 0;     // runs of two; of three or more
    uint64_t E = 0;                 // pair checks of the runs: sum of m (m - 1) / 2
    uint32_t *k_out = nullptr;      // the sorted keys
    uint32_t *v_out = nullptr;      // entry values g s + k in key order
    uint2 *runs = nullptr;          // {start, length} of the runs of >= 3
    uint32_t *rfirst = nullptr, *ridx = nullptr;      // their first genome, index (unsorted)
    uint32_t *pairs = nullptr;      // start of each run of two
};

static int screen_front(drephip_ctx *ctx, const uint64_t *d_hashes, const uint32_t *d_nhash, uint32_t N,
                        uint32_t part, uint32_t nparts, hipStream_t st, ScreenProf &prof, ScreenFront *F) {
    const uint32_t s = ctx->s;
    int rc;
    uint64_t *d_eoff, *h_tot;
    uint32_t *d_pcnt = nullptr, *d_pbeg = nullptr;
    F->vbits = 1;
    while (F->vbits < 32 && (1ull << F->vbits) < (uint64_t)N * s) F->vbits++;
    F->vmask = F->vbits >= 32 ? 0xFFFFFFFFu : (1u << F->vbits) - 1;
    if ((rc = scratch(ctx, "sc_eoff", (N + 1) * 8ull, (void **)&d_eoff))) return rc;
    if ((rc = pinned_host(ctx, "sc_tot", 64, (void **)&h_tot))) return rc;
    if (nparts > 1) {
        // the part's entries per genome, then their offsets
        if ((rc = scratch(ctx, "sc_part_cnt", (N + 1) * 4ull, (void **)&d_pcnt))) return rc;
        if ((rc = scratch(ctx, "sc_part_beg", (N + 1) * 4ull, (void **)&d_pbeg))) return rc;
        uint64_t *d_bnd;
        if ((rc = scratch(ctx, "sc_part_bnd", nparts * 8ull, (void **)&d_bnd))) return rc;
        hipLaunchKernelGGL(k_part_bounds, dim3(nparts - 1), dim3(kBndSample), 0, st, d_hashes, d_nhash, N, s, nparts,
                           d_bnd);
        hipLaunchKernelGGL(k_part_range, dim3((N + kScWG - 1) / kScWG), dim3(kScWG), 0, st, d_hashes, d_nhash, d_bnd,
                           N, s, part, nparts, d_pbeg, d_pcnt);
        if ((rc = hip_scan(ctx, "sc_scan_tmp0", (const uint32_t *)d_pcnt, d_eoff, N, st))) return rc;
        hipLaunchKernelGGL(k_screen_total, dim3(1), dim3(64), 0, st, d_pcnt, d_eoff, N);
    } else {
        if ((rc = hip_scan(ctx, "sc_scan_tmp0", d_nhash, d_eoff, N, st))) return rc;
        hipLaunchKernelGGL(k_screen_total, dim3(1), dim3(64), 0, st, d_nhash, d_eoff, N);
    }
    HIPC(hipMemcpyAsync(h_tot, d_eoff + N, 8, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    const uint32_t M = (uint32_t)h_tot[0];
    F->M = M;
    if (M < 2) return DREPHIP_OK;
    uint32_t *k_in, *k_out, *v_in, *v_out;
    if ((rc = scratch(ctx, "sc_kin", M * 4ull + 16, (void **)&k_in))) return rc;
    if ((rc = scratch(ctx, "sc_kout", M * 4ull + 16, (void **)&k_out))) return rc;
    if ((rc = scratch(ctx, "sc_vin", M * 4ull + 16, (void **)&v_in))) return rc;
    if ((rc = scratch(ctx, "sc_vout", M * 4ull + 16, (void **)&v_out))) return rc;
    if ((rc = scratch(ctx, "sc_runs", (M / 2 + 1) * 8ull, (void **)&F->runs))) return rc;
    prof.mark("offsets+alloc", st);
    if (nparts > 1)
        hipLaunchKernelGGL(k_part_keys, dim3((N + kPartWaves - 1) / kPartWaves), dim3(kScWG), 0, st, d_hashes, d_pbeg,
                           d_pcnt, d_eoff, N, s, F->vbits, k_in, v_in);
    else
        hipLaunchKernelGGL(k_screen_keys, dim3(N), dim3(kScWG), 0, st, d_hashes, d_nhash, d_eoff, s, F->vbits, k_in, v_in);
    prof.mark("keys", st);
    {
        size_t tb = 0;
        HIPC(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k_in, k_out, v_in, v_out, M, 0, 32, st));
        void *tmp;
        if ((rc = scratch(ctx, "sc_sort_tmp", std::max<size_t>(tb, 16), &tmp))) return rc;
        HIPC(hipcub::DeviceRadixSort::SortPairs(tmp, tb, k_in, k_out, v_in, v_out, M, 0, 32, st));
    }
    prof.mark("sort", st);
    // runs: heads counted per chunk -> offsets -> run bounds
    uint32_t *rstart, *rend, *hcnt, *hoff;
    if ((rc = scratch(ctx, "sc_rstart", M * 4ull + 16, (void **)&rstart))) return rc;
    if ((rc = scratch(ctx, "sc_rend", M * 4ull + 16, (void **)&rend))) return rc;
    const uint32_t hchunk = std::max<uint32_t>(4096, (M + 8191) / 8192);
    const uint32_t nhb = (M + hchunk - 1) / hchunk;
    if ((rc = scratch(ctx, "sc_hcnt", (nhb + 1) * 4ull, (void **)&hcnt))) return rc;
    if ((rc = scratch(ctx, "sc_hoff", (nhb + 1) * 4ull, (void **)&hoff))) return rc;
    HIPC(hipMemsetAsync(hcnt + nhb, 0, 4, st));
    hipLaunchKernelGGL(k_head_count, dim3(nhb), dim3(kScWG), 0, st, k_out, M, hchunk, hcnt);
    if ((rc = hip_scan(ctx, "sc_scan_tmp3", hcnt, hoff, nhb + 1, st))) return rc;
    hipLaunchKernelGGL(k_head_write, dim3(nhb), dim3(kScWG), 0, st, k_out, M, hchunk, hoff, nhb, rstart, rend);
    HIPC(hipMemcpyAsync(h_tot, hoff + nhb, 4, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    uint32_t *flag = k_in, *rid = v_in;                           // free after the sort
    const uint32_t nr = ((const uint32_t *)h_tot)[0];             // distinct keys
    F->nr = nr;
    // the run lists (at most M / 2 runs of >= 2); rfirst / ridx reuse the key
    // and value inputs of the sort, which are free now
    F->rfirst = flag;
    F->ridx = rid;
    const uint32_t per = (nr + kRunBlocks - 1) / kRunBlocks;
    uint32_t *bcnt2, *bcnt3, *boff2, *boff3;
    unsigned long long *bchk;
    if ((rc = scratch(ctx, "sc_bcnt2", (kRunBlocks + 1) * 4ull, (void **)&bcnt2))) return rc;
    if ((rc = scratch(ctx, "sc_bcnt3", (kRunBlocks + 1) * 4ull, (void **)&bcnt3))) return rc;
    if ((rc = scratch(ctx, "sc_boff2", (kRunBlocks + 1) * 4ull, (void **)&boff2))) return rc;
    if ((rc = scratch(ctx, "sc_boff3", (kRunBlocks + 1) * 4ull, (void **)&boff3))) return rc;
    if ((rc = scratch(ctx, "sc_bchk", kRunBlocks * 8ull, (void **)&bchk))) return rc;
    if ((rc = scratch(ctx, "sc_pairs", (M / 2 + 1) * 4ull, (void **)&F->pairs))) return rc;
    HIPC(hipMemsetAsync(bcnt2 + kRunBlocks, 0, 4, st));
    HIPC(hipMemsetAsync(bcnt3 + kRunBlocks, 0, 4, st));
    hipLaunchKernelGGL(k_run_count, dim3(kRunBlocks), dim3(kScWG), 0, st, rstart, rend, nr, per, bcnt2, bcnt3, bchk);
    if ((rc = hip_scan(ctx, "sc_scan_tmp4", bcnt2, boff2, kRunBlocks + 1, st))) return rc;
    if ((rc = hip_scan(ctx, "sc_scan_tmp5", bcnt3, boff3, kRunBlocks + 1, st))) return rc;
    hipLaunchKernelGGL(k_run_write, dim3(kRunBlocks), dim3(kScWG), 0, st, rstart, rend, nr, per, boff2, boff3, v_out, s,
                       F->vmask, F->pairs, F->runs, F->rfirst, F->ridx);
    HIPC(hipGetLastError());
    unsigned long long *h_chk;
    if ((rc = pinned_host(ctx, "sc_chk", kRunBlocks * 8ull, (void **)&h_chk))) return rc;
    HIPC(hipMemcpyAsync(h_chk, bchk, kRunBlocks * 8ull, hipMemcpyDeviceToHost, st));
    HIPC(hipMemcpyAsync(h_tot, boff2 + kRunBlocks, 4, hipMemcpyDeviceToHost, st));
    HIPC(hipMemcpyAsync((uint32_t *)h_tot + 1, boff3 + kRunBlocks, 4, hipMemcpyDeviceToHost, st));
    prof.mark("runs", st);
    HIPC(hipStreamSynchronize(st));
    F->n2 = ((const uint32_t *)h_tot)[0];                         // runs of two entries
    F->nruns = ((const uint32_t *)h_tot)[1];                      // runs of three or more
    uint64_t E = 0;
    for (uint32_t b = 0; b < kRunBlocks; b++) E += h_chk[b];
    F->E = E;
    F->k_out = k_out;
    F->v_out = v_out;
    return DREPHIP_OK;
}

// the runs of >= 3 in first-genome order, marked into bm (row tiles from row0)
static int screen_mark_runs(drephip_ctx *ctx, const ScreenFront &F, const uint64_t *d_hashes, uint32_t N,
                            uint32_t row0, uint32_t row1, uint32_t rshift, uint32_t NW, uint32_t *d_bm,
                            uint32_t *d_bmH, uint32_t *d_crun, hipStream_t st, ScreenProf &prof) {
    if (!F.nruns) return DREPHIP_OK;
    const uint32_t s = ctx->s, M = F.M;
    int rc;
    uint32_t *rfirst_s, *ridx_s;
    if ((rc = scratch(ctx, "sc_rfirst_s", (M / 2 + 1) * 4ull, (void **)&rfirst_s))) return rc;
    if ((rc = scratch(ctx, "sc_ridx_s", (M / 2 + 1) * 4ull, (void **)&ridx_s))) return rc;
    // first genomes are < N: only their low bits are sorted (2 passes instead
    // of 4 below 2^16 genomes)
    int gbits = 1;
    while (gbits < 32 && (1ull << gbits) < N) gbits++;
    size_t tb = 0;
    HIPC(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, F.rfirst, rfirst_s, F.ridx, ridx_s, F.nruns, 0, gbits, st));
    void *tmp;
    if ((rc = scratch(ctx, "sc_sort_tmp2", std::max<size_t>(tb, 16), &tmp))) return rc;
    HIPC(hipcub::DeviceRadixSort::SortPairs(tmp, tb, F.rfirst, rfirst_s, F.ridx, ridx_s, F.nruns, 0, gbits, st));
    prof.mark("run-sort", st);
    const dim3 grid((F.nruns + kMarkChunk - 1) / kMarkChunk);
    if (d_bmH)
        hipLaunchKernelGGL(k_screen_mark<true>, grid, dim3(kMarkWG), 0, st, F.v_out, d_hashes, s, F.vbits, F.runs, ridx_s,
                           rfirst_s, F.nruns, row0, row1, rshift, NW, d_bm, d_bmH, d_crun, N);
    else
        hipLaunchKernelGGL(k_screen_mark<false>, grid, dim3(kMarkWG), 0, st, F.v_out, d_hashes, s, F.vbits, F.runs, ridx_s,
                           rfirst_s, F.nruns, row0, row1, rshift, NW, d_bm, nullptr, nullptr, N);
    HIPC(hipGetLastError());
    return DREPHIP_OK;
}

// the pair map (pcap slots, a power of two) cleared
static int screen_pair_map(drephip_ctx *ctx, uint64_t n, hipStream_t st, uint64_t *pcap_out,
                           unsigned long long **pkey, uint32_t **pcnt, uint32_t **ppos) {
    uint64_t pcap = 1024;
    while (pcap < 2ull * n) pcap <<= 1;
    *pcap_out = pcap;
    if (pcap > kMaxPairMap) return DREPHIP_OK;                       // too large: the caller gives way
    int rc;
    if ((rc = scratch(ctx, "sc_pkey", pcap * 8ull, (void **)pkey))) return rc;
    if ((rc = scratch(ctx, "sc_pcnt", pcap * 4ull, (void **)pcnt))) return rc;
    if ((rc = scratch(ctx, "sc_ppos", pcap * 4ull, (void **)ppos))) return rc;
    HIPC(hipMemsetAsync(*pkey, 0xFF, pcap * 8ull, st));
    HIPC(hipMemsetAsync(*pcnt, 0, pcap * 4ull, st));
    return DREPHIP_OK;
}

// marked cells (d_bl) -> each row tile's column list and the LIST items
static int screen_lists(drephip_ctx *ctx, const uint32_t *d_bl, uint32_t ntiles, uint32_t NW, uint32_t C,
                        uint32_t row0, uint32_t R, const unsigned long long *d_nsimple, hipStream_t st,
                        ScreenProf &prof, ScreenResult *res) {
    int rc;
    uint32_t *d_cnt, *d_itc;
    uint64_t *d_coff, *d_cnt64, *h_tot;
    if ((rc = pinned_host(ctx, "sc_tot", 64, (void **)&h_tot))) return rc;
    if ((rc = scratch(ctx, "sc_tcnt", (ntiles + 1) * 4ull, (void **)&d_cnt))) return rc;
    if ((rc = scratch(ctx, "sc_tcnt64", (ntiles + 1) * 8ull, (void **)&d_cnt64))) return rc;
    if ((rc = scratch(ctx, "sc_titc", (ntiles + 1) * 4ull, (void **)&d_itc))) return rc;
    if ((rc = scratch(ctx, "sc_coff", (ntiles + 1) * 8ull, (void **)&d_coff))) return rc;
    hipLaunchKernelGGL(k_screen_count, dim3(ntiles), dim3(kScWG), 0, st, d_bl, NW, C, d_cnt, d_cnt64, d_itc);
    // the last entry of each scan holds the totals: count entries ntiles + 1, the last one zero.
    // The column offsets are summed in 64 bits (the marked cells may pass 2^32;
    // a 32-bit scan would wrap and the fallback below would never fire)
    HIPC(hipMemsetAsync(d_cnt64 + ntiles, 0, 8, st));
    if ((rc = hip_scan(ctx, "sc_scan_tmp1", d_cnt64, d_coff, ntiles + 1, st))) return rc;
    prof.mark("count+scans", st);
    uint32_t *h_itc, *ibase;
    if ((rc = pinned_host(ctx, "sc_itc", ntiles * 4ull, (void **)&h_itc))) return rc;
    if ((rc = pinned_host(ctx, "sc_ibase_h", ntiles * 4ull, (void **)&ibase))) return rc;
    HIPC(hipMemcpyAsync(h_tot, d_coff + ntiles, 8, hipMemcpyDeviceToHost, st));
    HIPC(hipMemcpyAsync(h_tot + 2, d_nsimple, 8, hipMemcpyDeviceToHost, st));
    HIPC(hipMemcpyAsync(h_itc, d_itc, ntiles * 4ull, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    const uint64_t marked = h_tot[0];
    res->marked = marked;
    res->simple = h_tot[2];
    // XCD placement: blocks of kItemBlock row tiles dealt in order to the
    // least-loaded XCD; a tile's items sit at slots xcd + 8 (offset in that
    // XCD's list + j); the lists are padded to one length with idle items
    {
        uint64_t load[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (uint32_t b0 = 0; b0 < ntiles; b0 += kItemBlock) {
            uint32_t x = 0;
            for (uint32_t k = 1; k < 8; k++) if (load[k] < load[x]) x = k;
            for (uint32_t t = b0; t < std::min(ntiles, b0 + kItemBlock); t++) {
                ibase[t] = (uint32_t)std::min<uint64_t>(x + 8 * load[x], 0xFFFFFFFFull);
                load[x] += h_itc[t];
            }
        }
        uint64_t lmax = 0;
        for (uint32_t k = 0; k < 8; k++) lmax = std::max(lmax, load[k]);
        h_tot[1] = 8 * lmax;
    }
    const uint64_t nitems = h_tot[1];
    if (marked >= (1ull << 32) || nitems >= (1ull << 31)) return DREPHIP_OK;     // res->use stays false
    uint32_t *d_list, *d_ibase;
    uint4 *d_items;
    if ((rc = scratch(ctx, "sc_list", std::max<uint64_t>(marked, 1) * 4, (void **)&d_list))) return rc;
    if ((rc = scratch(ctx, "sc_items", std::max<uint64_t>(nitems, 1) * 16, (void **)&d_items))) return rc;
    if ((rc = scratch(ctx, "sc_ibase", ntiles * 4ull, (void **)&d_ibase))) return rc;
    HIPC(hipMemcpyAsync(d_ibase, ibase, ntiles * 4ull, hipMemcpyHostToDevice, st));
    HIPC(hipMemsetAsync(d_items, 0xFF, std::max<uint64_t>(nitems, 1) * 16, st));       // idle items: i0 = ~0
    prof.mark("readback+alloc", st);
    const char *de = getenv("DREPHIP_SCREEN_DESC");
    hipLaunchKernelGGL(k_screen_lists, dim3(ntiles), dim3(kScWG), 0, st, d_bl, NW, C, row0, R, d_cnt, d_coff, d_ibase,
                       d_list, d_items, de ? atoi(de) : 0);
    prof.mark("lists", st);
    HIPC(hipGetLastError());
    res->use = true;
    res->clist = d_list;
    res->items = d_items;
    res->nitems = (uint32_t)nitems;
    return DREPHIP_OK;
}

static uint32_t tile_shift(uint32_t R) {
    uint32_t rshift = 0;
    while ((1u << rshift) < R) rshift++;
    return rshift;
}

// the dense-set rule: a pair check costs about as much as a few probes of the
// dense kernels, which make ~s/2 probes per pair (DREPHIP_SCREEN_RATIO scales
// the bound).  E counts the checks of the whole triangle (every entry is
// grouped), weighed against the whole triangle's pairs: every rank of a
// sharded job, and the one-GPU call, take the same path
bool screen_worth(uint32_t N, uint32_t s, uint64_t E) {
    const char *re = getenv("DREPHIP_SCREEN_RATIO");
    const double ratio = re ? atof(re) : 16.0;
    const double all_pairs = (double)N * (double)(N - 1) / 2.0;
    return (double)E * ratio <= all_pairs * s;
}

int screen_impl(drephip_ctx *ctx, const uint64_t *d_hashes, const uint32_t *d_nhash, uint32_t N, uint32_t row0,
                uint32_t row1, uint32_t R, uint32_t C, uint64_t seg0, uint64_t npairs, uint16_t *d_common,
                uint16_t *d_denom, bool force, bool band, hipStream_t st, ScreenResult *res) {
    *res = ScreenResult{};
    const uint32_t s = ctx->s;
    if ((uint64_t)N * s >= (1ull << 32)) return DREPHIP_OK;          // entry values g * s + k are 32-bit
    int rc;
    timing_mark(ctx, 4, st, true);
    ScreenProf prof;
    prof.mark("start", st);
    ScreenFront F;
    if ((rc = screen_front(ctx, d_hashes, d_nhash, N, 0, 1, st, prof, &F))) return rc;
    if (F.M < 2) {
        // fewer than two sketch entries: no pair shares a hash; every pair
        // gets the no-shared-hash fill, no LIST work
        if ((rc = screen_fill_impl(ctx, d_nhash, N, row0, row1, seg0, npairs, d_common, d_denom, st))) return rc;
        timing_mark(ctx, 4, st, false);
        res->entries = F.M;
        res->use = true;
        return DREPHIP_OK;
    }
    res->entries = F.M;
    res->runs = (uint64_t)F.n2 + F.nruns;
    res->checks = F.E;
    if (!force && !screen_worth(N, s, F.E)) {
        // the dense path runs: its chunk masks from the runs just grouped
        // (k_cmask_*; whole-row tables only, s <= 2048: <= 32 chunks; and
        // s >= 64, which the unchecked probe's rank test relies on).
        // DREPHIP_AP_CMASK=0 leaves every chunk to the high-word check (A/B)
        const char *ce = getenv("DREPHIP_AP_CMASK");
        if (s >= 64 && s <= 2048 && (!ce || atoi(ce) != 0)) {
            uint32_t *d_cm;
            if ((rc = scratch(ctx, "sc_cmask", N * 4ull, (void **)&d_cm))) return rc;
            hipLaunchKernelGGL(k_cmask_init, dim3((N + kScWG - 1) / kScWG), dim3(kScWG), 0, st, d_nhash, N, F.k_out, F.M,
                               d_cm);
            if (F.n2)
                hipLaunchKernelGGL(k_cmask_pairs, dim3(std::min(4096u, (F.n2 + kScWG - 1) / kScWG)), dim3(kScWG), 0, st,
                                   F.v_out, d_hashes, s, F.vmask, F.pairs, F.n2, d_cm);
            if (F.nruns)
                hipLaunchKernelGGL(k_cmask_runs, dim3(std::min(4096u, (F.nruns + 3) / 4)), dim3(kScWG), 0, st, F.v_out,
                                   d_hashes, s, F.vmask, F.runs, F.nruns, d_cm);
            HIPC(hipGetLastError());
            // timing A/B only: 2 = every chunk checked, 3 = none (wrong counts)
            if (ce && atoi(ce) >= 2) HIPC(hipMemsetAsync(d_cm, atoi(ce) == 2 ? 0xFF : 0, N * 4ull, st));
            res->cmask = d_cm;
        }
        timing_mark(ctx, 4, st, false);
        return DREPHIP_OK;
    }

    const uint32_t rows = row1 - row0;
    const uint32_t ntiles = (rows + R - 1) / R;
    const uint32_t NW = (N + 31) / 32;
    const uint32_t rshift = tile_shift(R);
    uint32_t *d_bm;
    if ((rc = scratch(ctx, "sc_bitmap", (uint64_t)ntiles * NW * 4, (void **)&d_bm))) return rc;
    // Light cells (k_screen_light): a heavy-cell bitmap and each cell's first
    // marking run, (ntiles x N) words -- taken when that fits kLightBudget
    // (N = 10^4 with R = 4: 100 MB), for the band kernel only: at configs[4]
    // its LIST time 9.0 -> 4.0 ms for +0.9 ms of screen; at configs[2] (the q
    // kernel, s = 1000) 0.39 -> 0.35 ms of LIST for +0.33 ms of screen
    // (profiles/r05_screen_light_c2_ab.txt).  DREPHIP_SCREEN_LIGHT=0/1 forces it (A/B)
    const char *le = getenv("DREPHIP_SCREEN_LIGHT");
    const bool light = (le ? atoi(le) != 0 : band) && (uint64_t)ntiles * N * 4 <= kLightBudget;
    uint32_t *d_bmH = nullptr, *d_crun = nullptr;
    if (light) {
        if ((rc = scratch(ctx, "sc_bitmap_heavy", (uint64_t)ntiles * NW * 4, (void **)&d_bmH))) return rc;
        if ((rc = scratch(ctx, "sc_crun", (uint64_t)ntiles * N * 4, (void **)&d_crun))) return rc;
    }
    // the pair map of the runs of two (k_screen_mark2), twice their count; a
    // map beyond kMaxPairMap slots (16 B each) is not built: the dense path runs
    uint64_t pcap;
    unsigned long long *pkey = nullptr, *d_nsimple;
    uint32_t *pcnt = nullptr, *ppos = nullptr;
    if ((rc = screen_pair_map(ctx, F.n2, st, &pcap, &pkey, &pcnt, &ppos))) return rc;
    if (pcap > kMaxPairMap) { timing_mark(ctx, 4, st, false); return DREPHIP_OK; }
    if ((rc = scratch(ctx, "sc_nsimple", 8, (void **)&d_nsimple))) return rc;
    prof.mark("readback+alloc", st);
    // every pair as no-shared-hash first: the simple pairs are written over it
    // below, the LIST kernel over both
    if ((rc = screen_fill_impl(ctx, d_nhash, N, row0, row1, seg0, npairs, d_common, d_denom, st))) return rc;
    prof.mark("fill", st);
    HIPC(hipMemsetAsync(d_bm, 0, (uint64_t)ntiles * NW * 4, st));
    if (light) HIPC(hipMemsetAsync(d_bmH, 0, (uint64_t)ntiles * NW * 4, st));
    HIPC(hipMemsetAsync(d_nsimple, 0, 8, st));
    prof.mark("bitmap-clear", st);
    if ((rc = screen_mark_runs(ctx, F, d_hashes, N, row0, row1, rshift, NW, d_bm, d_bmH, d_crun, st, prof))) return rc;
    if (F.n2) {
        const uint32_t g2 = std::max(1u, std::min(8192u, (F.n2 + kScWG - 1) / kScWG));
        hipLaunchKernelGGL(k_screen_mark2, dim3(g2), dim3(kScWG), 0, st, F.v_out, d_hashes, s, F.vmask, F.pairs, F.n2, row0, row1,
                           pkey, pcnt, ppos, (uint32_t)(pcap - 1));
        const uint32_t gs = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(2048, (pcap + kScWG - 1) / kScWG));
        hipLaunchKernelGGL(k_screen_simple, dim3(gs), dim3(kScWG), 0, st, pkey, pcnt, ppos, (uint32_t)pcap, d_nhash, s, N, row0,
                           rshift, NW, seg0, d_bm, d_bmH, d_common, d_nsimple);
    }
    prof.mark("mark", st);
    if (light && F.nruns) {
        const uint64_t nwords = (uint64_t)ntiles * NW;
        const uint32_t gl = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(4096, (nwords + kScWG - 1) / kScWG));
        hipLaunchKernelGGL(k_screen_light, dim3(gl), dim3(kScWG), 0, st, d_bm, d_bmH, d_crun, F.runs, F.v_out, d_hashes,
                           d_nhash, s, F.vmask, N, row0, row1, R, NW, nwords, seg0, d_common, d_nsimple);
        prof.mark("light", st);
    }
    // the LIST kernels take the heavy cells (every marked cell without the light screen)
    rc = screen_lists(ctx, light ? d_bmH : d_bm, ntiles, NW, C, row0, R, d_nsimple, st, prof, res);
    timing_mark(ctx, 4, st, false);
    return rc;
}

// ------------------------------------------------------- the sharded screen
// Part `part` of `nparts` hash ranges (one per rank of a sharded job): its
// entries grouped, its runs of >= 3 marked into a bitmap of row tiles of R
// rows counted from row 0 -- every row, not only this rank's -- sent out as
// its nonzero words (cell records), and its runs of two listed as records.
// The caller routes every part's cells and records to the ranks owning their
// rows (drephip_screen_part_copy), and each rank finishes its rows from them
// (screen_marked_impl).  Results stay in the context's scratch until the next
// screen call.
int screen_part_impl(drephip_ctx *ctx, const uint64_t *d_hashes, const uint32_t *d_nhash, uint32_t N, uint32_t R,
                     uint32_t part, uint32_t nparts, hipStream_t st, uint64_t *checks, uint32_t *ncells_out,
                     uint32_t *nrec) {
    const uint32_t s = ctx->s;
    *checks = 0;
    *ncells_out = 0;
    *nrec = 0;
    ctx->part = PartResult{};
    if ((uint64_t)N * s >= (1ull << 32)) { set_error("the screen needs N x s < 2^32"); return DREPHIP_ERR_UNSUPPORTED; }
    int rc;
    timing_mark(ctx, 4, st, true);
    ScreenProf prof;
    prof.mark("start", st);
    ScreenFront F;
    if ((rc = screen_front(ctx, d_hashes, d_nhash, N, part, nparts, st, prof, &F))) return rc;
    const uint32_t NW = (N + 31) / 32, ntg = (N + R - 1) / R, rshift = tile_shift(R);
    uint32_t *d_gbm, *d_nrec;
    uint4 *d_rec;
    const uint64_t gwords = (uint64_t)ntg * NW;
    if ((rc = scratch(ctx, "sc_part_bitmap", gwords * 4, (void **)&d_gbm))) return rc;
    if ((rc = scratch(ctx, "sc_part_nrec", 8, (void **)&d_nrec))) return rc;
    if ((rc = scratch(ctx, "sc_part_rec", (uint64_t)std::max<uint32_t>(F.n2, 1) * 16, (void **)&d_rec))) return rc;
    HIPC(hipMemsetAsync(d_gbm, 0, gwords * 4, st));
    HIPC(hipMemsetAsync(d_nrec, 0, 4, st));
    if (F.M >= 2) {
        if ((rc = screen_mark_runs(ctx, F, d_hashes, N, 0, N, rshift, NW, d_gbm, nullptr, nullptr, st, prof))) return rc;
        if (F.n2) {
            const uint32_t g2 = std::max(1u, std::min(8192u, (F.n2 + kScWG - 1) / kScWG));
            hipLaunchKernelGGL(k_screen_emit2, dim3(g2), dim3(kScWG), 0, st, F.v_out, d_hashes, s, F.vmask, F.pairs, F.n2,
                               d_rec, d_nrec);
        }
        prof.mark("mark", st);
    }
    // the marks as cell words (nonzero words of the bitmap)
    const uint32_t cchunk = (uint32_t)std::max<uint64_t>(8192, (gwords + 8191) / 8192);
    const uint32_t ncb = (uint32_t)((gwords + cchunk - 1) / cchunk);
    uint32_t *ccnt, *coff;
    if ((rc = scratch(ctx, "sc_cells_cnt", (ncb + 1) * 4ull, (void **)&ccnt))) return rc;
    if ((rc = scratch(ctx, "sc_cells_off", (ncb + 1) * 4ull, (void **)&coff))) return rc;
    HIPC(hipMemsetAsync(ccnt + ncb, 0, 4, st));
    hipLaunchKernelGGL(k_cells_count, dim3(ncb), dim3(kScWG), 0, st, d_gbm, gwords, cchunk, ccnt);
    if ((rc = hip_scan(ctx, "sc_scan_tmp6", ccnt, coff, ncb + 1, st))) return rc;
    uint64_t *h_tot;
    if ((rc = pinned_host(ctx, "sc_tot", 64, (void **)&h_tot))) return rc;
    HIPC(hipMemcpyAsync(h_tot, d_nrec, 4, hipMemcpyDeviceToHost, st));
    HIPC(hipMemcpyAsync((uint32_t *)h_tot + 1, coff + ncb, 4, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    const uint32_t ncells = ((const uint32_t *)h_tot)[1];
    uint4 *d_cells;
    if ((rc = scratch(ctx, "sc_part_cells", (uint64_t)std::max<uint32_t>(ncells, 1) * 16, (void **)&d_cells))) return rc;
    hipLaunchKernelGGL(k_cells_write, dim3(ncb), dim3(kScWG), 0, st, d_gbm, gwords, cchunk, coff, NW, d_cells);
    HIPC(hipGetLastError());
    HIPC(hipStreamSynchronize(st));
    prof.mark("cells", st);
    timing_mark(ctx, 4, st, false);
    ctx->part.valid = true;
    ctx->part.N = N;
    ctx->part.R = R;
    ctx->part.cells = d_cells;
    ctx->part.ncells = ncells;
    ctx->part.rec = d_rec;
    ctx->part.nrec = ((const uint32_t *)h_tot)[0];
    ctx->part.entries = F.M;
    ctx->part.runs = (uint64_t)F.n2 + F.nruns;
    ctx->part.checks = F.E;
    *checks = F.E;
    *ncells_out = ncells;
    *nrec = ctx->part.nrec;
    return DREPHIP_OK;
}

// Rows [row0, row1) from every part's marks: the cell words OR-ed into this
// rank's row tiles, the pair map from every part's records of these rows, the
// pairs sharing exactly one hash written here (k_screen_simple), the lists.
// No light cells (their single marking run may live in another part).
int screen_marked_impl(drephip_ctx *ctx, const uint32_t *d_nhash, uint32_t N, uint32_t row0, uint32_t row1,
                       uint32_t R, uint32_t C, uint64_t seg0, uint64_t npairs, uint16_t *d_common, uint16_t *d_denom,
                       const uint4 *d_cells, uint64_t ncells, const uint4 *d_rec, uint64_t nrec, hipStream_t st,
                       ScreenResult *res) {
    *res = ScreenResult{};
    const uint32_t s = ctx->s;
    int rc;
    timing_mark(ctx, 4, st, true);
    ScreenProf prof;
    prof.mark("start", st);
    const uint32_t rows = row1 - row0, ntiles = (rows + R - 1) / R, NW = (N + 31) / 32;
    const uint32_t rshift = tile_shift(R);
    uint32_t *d_bm;
    unsigned long long *pkey = nullptr, *d_nsimple;
    uint32_t *pcnt = nullptr, *ppos = nullptr;
    uint64_t pcap;
    if ((rc = scratch(ctx, "sc_bitmap", (uint64_t)ntiles * NW * 4, (void **)&d_bm))) return rc;
    if ((rc = scratch(ctx, "sc_nsimple", 8, (void **)&d_nsimple))) return rc;
    // the pair map holds this rank's records only (every part's records of its rows)
    uint64_t nown = 0;
    if (nrec) {
        uint64_t *h_tot;
        if ((rc = pinned_host(ctx, "sc_tot", 64, (void **)&h_tot))) return rc;
        HIPC(hipMemsetAsync(d_nsimple, 0, 8, st));
        const uint32_t gc = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(1024, (nrec + kScWG - 1) / kScWG));
        hipLaunchKernelGGL(k_rec_count, dim3(gc), dim3(kScWG), 0, st, d_rec, nrec, row0, row1, d_nsimple);
        HIPC(hipMemcpyAsync(h_tot, d_nsimple, 8, hipMemcpyDeviceToHost, st));
        HIPC(hipStreamSynchronize(st));
        nown = h_tot[0];
    }
    if ((rc = screen_pair_map(ctx, nown, st, &pcap, &pkey, &pcnt, &ppos))) return rc;
    if (pcap > kMaxPairMap) { timing_mark(ctx, 4, st, false); return DREPHIP_OK; }
    if ((rc = screen_fill_impl(ctx, d_nhash, N, row0, row1, seg0, npairs, d_common, d_denom, st))) return rc;
    HIPC(hipMemsetAsync(d_nsimple, 0, 8, st));
    HIPC(hipMemsetAsync(d_bm, 0, (uint64_t)ntiles * NW * 4, st));
    if (ncells) {
        const uint32_t gc = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(4096, (ncells + kScWG - 1) / kScWG));
        hipLaunchKernelGGL(k_cells_scatter, dim3(gc), dim3(kScWG), 0, st, d_cells, ncells, row0, row1, rshift, NW, d_bm);
    }
    prof.mark("cells", st);
    if (nown) {
        const uint32_t g2 = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(8192, (nrec + kScWG - 1) / kScWG));
        hipLaunchKernelGGL(k_screen_map2, dim3(g2), dim3(kScWG), 0, st, d_rec, nrec, row0, row1, pkey, pcnt, ppos,
                           (uint32_t)(pcap - 1));
        const uint32_t gs = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(2048, (pcap + kScWG - 1) / kScWG));
        hipLaunchKernelGGL(k_screen_simple, dim3(gs), dim3(kScWG), 0, st, pkey, pcnt, ppos, (uint32_t)pcap, d_nhash, s, N,
                           row0, rshift, NW, seg0, d_bm, nullptr, d_common, d_nsimple);
    }
    prof.mark("pairs", st);
    HIPC(hipGetLastError());
    rc = screen_lists(ctx, d_bm, ntiles, NW, C, row0, R, d_nsimple, st, prof, res);
    timing_mark(ctx, 4, st, false);
    if (ctx->part.valid && ctx->part.N == N) {
        // this rank's own part (the entries it grouped), for the stats
        res->entries = ctx->part.entries;
        res->runs = ctx->part.runs;
        res->checks = ctx->part.checks;
    }
    return rc;
}

int screen_fill_impl(drephip_ctx *ctx, const uint32_t *d_nhash, uint32_t N, uint32_t row0, uint32_t row1,
                     uint64_t seg0, uint64_t npairs, uint16_t *d_common, uint16_t *d_denom, hipStream_t st) {
    HIPC(hipMemsetAsync(d_common, 0, npairs * 2, st));
    if (d_denom)
        hipLaunchKernelGGL(k_screen_denoms, dim3(row1 - row0), dim3(kScWG), 0, st, d_nhash, ctx->s, N, row0, seg0,
                           d_denom);
    HIPC(hipGetLastError());
    return DREPHIP_OK;
}

}  // namespace drephip
