// sketch.hip -- MI355X sketch path: replaces `mash sketch <fa> -s S` per
// genome (drep/d_cluster.py:531-549) and `mash paste` (551-567).
//
// Three kernels, one pass over the packed genome set per round:
//   k_sketch_hash21   one workgroup per 32768-base tile; each lane covers 64
//                     window ends (2-bit codes + validity from HBM, one load
//                     per 16 bases), cuts the forward and reverse-complement
//                     k-mers out of the code stream, hashes the canonical one
//                     with MurmurHash3_x64_128 (seed 42, h1) using per-workgroup
//                     LDS tables for the base-local parts, and admits it only if
//                     h <= T[g] (per-genome candidate threshold).  Admitted
//                     hashes are staged in LDS and, after the tile, inserted
//                     into a per-genome open-addressing set in HBM (64-bit CAS),
//                     so duplicates drop out at insert.
//   k_sketch_finalize_bucket one workgroup per genome: bucket-sorts the set in
//                     LDS and writes the s smallest.
//   k_synth           bench input generator (not on the product path).
// The threshold is seeded from the k-mer count so ~F*s distinct candidates
// survive; a genome whose set ends with fewer than s distinct hashes (T too
// low) or more than the LDS sort holds (T too high) is re-run with a bisected
// T -- exact for every input, normally a single round.
//
// Roofline: integer VALU issue and LDS table reads (see k_sketch_hash21);
// HBM traffic is 3 bits/base (0.375 B/base) plus the candidate sets.

#include "ctx.h"
#include "../../include/drephip.h"

#include <algorithm>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace drephip {

__device__ __forceinline__ void set_insert(unsigned long long *S, uint32_t mask, uint32_t *cnt,
                                           uint32_t limit, uint64_t h) {
    if (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= limit) return;
    uint32_t slot = (uint32_t)h & mask;
    for (uint32_t probe = 0; probe <= mask; probe++) {
        unsigned long long old = atomicCAS(&S[slot], (unsigned long long)kEmpty, (unsigned long long)h);
        if (old == kEmpty) { atomicAdd(cnt, 1u); return; }
        if (old == h) return;
        slot = (slot + 1) & mask;
    }
}

// ------------------------------------------------------------- Murmur parts
// K = 21 (Mash/dRep default): 3 Murmur words = one 16-byte block + 5-byte tail.
// Rotations are two v_alignbit_b32 and h*5+c is one v_lshl_add_u64.
__device__ __forceinline__ uint64_t rotl64_ab(uint64_t x, int r) {
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    uint32_t nlo, nhi;
    if (r < 32) {
        nhi = __builtin_amdgcn_alignbit(hi, lo, 32 - r);
        nlo = __builtin_amdgcn_alignbit(lo, hi, 32 - r);
    } else {
        nhi = __builtin_amdgcn_alignbit(lo, hi, 64 - r);
        nlo = __builtin_amdgcn_alignbit(hi, lo, 64 - r);
    }
    return ((uint64_t)nhi << 32) | nlo;
}
__device__ __forceinline__ uint64_t x5_plus(uint64_t x, uint64_t c) {
    uint64_t y;
    asm("v_lshl_add_u64 %0, %1, 2, %1" : "=v"(y) : "v"(x));
    return y + c;
}
__device__ __forceinline__ uint64_t add64(uint64_t a, uint64_t b) {   // one v_lshl_add_u64
    uint64_t y;
    asm("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(y) : "v"(a), "v"(b));
    return y;
}
// fmix64 up to its last multiply: q = ((k ^ k >> 33) C1) ^ (... >> 33); the
// state before fmix64's final xorshift is then q C2 (fmix_mul)
constexpr uint64_t kFmixC2 = 0xc4ceb9fe1a85ec53ULL;
__device__ __forceinline__ uint64_t fmix64_q(uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33;
    return k;
}
__device__ __forceinline__ uint64_t fmix_mul(uint64_t q) { return q * kFmixC2; }
// hi(q1 C2) + hi(q2 C2) + 1 (mod 2^32) with the multiplies shared:
// hi(q C2) = hi(lo q lo C2) + lo q hi C2 + hi q lo C2
__device__ __forceinline__ uint32_t prefilter_hi(uint64_t q1, uint64_t q2) {
    const uint32_t a1 = (uint32_t)q1, b1 = (uint32_t)(q1 >> 32), a2 = (uint32_t)q2, b2 = (uint32_t)(q2 >> 32);
    return __umulhi(a1, (uint32_t)kFmixC2) + __umulhi(a2, (uint32_t)kFmixC2) + (a1 + a2) * (uint32_t)(kFmixC2 >> 32) +
           (b1 + b2) * (uint32_t)kFmixC2 + 1u;
}
// Candidates are staged in an LDS buffer (wave-aggregated LDS atomic) and only
// flushed to the per-genome set after the tile, so the hot loop issues no
// global memory operation with a wait; a full buffer spills to the set
// directly.
#ifndef DREPHIP_SK_STAGE
#define DREPHIP_SK_STAGE 128       // ~13 admitted hashes per tile expected; overflow goes straight to the set
#endif
constexpr uint32_t kStage = DREPHIP_SK_STAGE;

// ------------------------------------------------------------- hash kernel
// One workgroup of kTile / LANE lanes per 32768-base tile; lane l owns the
// LANE window ends [tile + LANE l, tile + LANE (l + 1)).  No per-base rolling state: the
// forward and reverse-complement k-mers are cut out of the 2-bit code stream
// with two v_alignbit_b32 each, the canonical one is chosen on the codes, and
// the parts of MurmurHash3_x64_128 (seed 42, h1) that depend only on a few
// bases come from per-workgroup LDS tables.
//
// Streams (code word j holds bases 16j..16j+15, base i at bits 2i):
//   NF[j] = ~F[j]: a 64-bit little-endian cut holding bases q-31..q has base q
//     in the top bits, i.e. it is the reverse complement read MSB-first --
//     top-aligned (bases of the k-mer in bits 22..63, junk below);
//   R[j] = F[j] with its 16 fields reversed: a big-endian cut of R starting at
//     base q-20 is the forward k-mer MSB-first, top-aligned the same way.
// memcmp order of the ASCII k-mers = unsigned order of those top-aligned values
// (A<C<G<T = 0<1<2<3; junk bits never decide: k is odd, so no k-mer equals its
// reverse complement).
//
// Murmur's block words are k1 = ASCII of bases 0-7 and k2 = bases 8-15; the
// tail k3 = bases 16-20.  A 64-bit product k * c splits as
//     k * c = A03 * c + (A47 * lo(c)) << 32       (A03, A47: ASCII of 4 bases)
// so X = k1 * c1 has lo(X) = lo(A03 c1) and hi(X) = hi(A03 c1) + A47 lo(c1).
// Then rotl(X, 31) = (hi(X) >> 1) + (lo(X) << 31) + ((hi(X) & 1) << 63) is a
// disjoint bit sum and, c2 being odd,
//     rotl(X, 31) * c2 = (hi(X) >> 1) * c2 + TT1 + ((hi(X) & 1) << 63),
//     TT1 = (lo(X) << 31) * c2,
// one v_mad_u64_u32 plus a high-word fix.  Likewise for k2:
//     rotl(X, 33) * c1 = hi(X) * (2 c1) + TT2,
//     TT2 = ((lo(X) & 0x7fffffff) << 33) * c1 + (lo(X) >> 31) * c1.
// The tail is one table entry, rotl31(k3 c1) c2 ^ 21 (Murmur's h1 ^= len).
//
// Cost model (measured, profiles/r02_sketch_ab.json): the loop is VALU-issue
// bound -- its time follows the VALU instruction count (a layout with 17 %
// more VALU instructions and half the LDS cycles ran 16 % slower), so the
// tables exist to take VALU work off the loop.  Every lookup index is data
// dependent: a wave's 64 reads of one instruction hit the LDS banks at
// random, ~3.2x the conflict-free cycles for 4- and 8-byte reads and ~3x for
// 16-byte reads (profiles/r02_lds_microbench.json).  Per dword fetched a
// 16-byte read therefore costs half a 4-byte one, so what a block word needs
// from its 4-base index is one 16-byte entry {lo(TT), hi(TT), hi(A03 c), 0}
// (ds_read_b128; TT in the first two words lands in the register pair the
// v_mad_u64_u32 adds), the A47 lo(c) terms are an 8- and a 4-byte read and
// the tail one 8-byte read: five reads per k-mer.
// The k1 word's high-word fix (X << 31) is folded into the tables: mod 2^32
// it is (hi(A03 c1) << 31) + (A47 lo(c1) << 31), the first added to hi(TT1)
// (a carry out of the 64-bit addend is discarded, as in the product), the
// second stored next to A47 lo(c1): one v_add3_u32 instead of a move, a
// v_mad_u64_u32 and a v_lshl_add_u32.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));   // one LDS vector load (a struct is split)
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
struct SketchTablesQ {
    u32x4 e1[256];        // {lo(TT1), hi(TT1) + (hi(A03 c1) << 31), hi(A03 c1), 0}  by bases 0-3
    u32x4 e2[256];        // {lo(TT2), hi(TT2), hi(A03 c2), hi(A03 c2) hi(2 c1)}     by bases 8-11
    u32x2 b1[256];        // {A47 lo(c1), A47 lo(c1) << 31}                         by bases 4-7
    u32x2 b2[256];        // {A47 lo(c2), A47 lo(c2) hi(2 c1)}                      by bases 12-15
    uint64_t t3[1024];    // tail, by bases 16-20
};

__device__ __forceinline__ uint32_t ascii4(uint32_t x) {      // 4 bases, base 0 in bits 6-7
    const uint32_t sel = ((x >> 6) & 3u) | (((x >> 4) & 3u) << 8) | (((x >> 2) & 3u) << 16) | ((x & 3u) << 24);
    return __builtin_amdgcn_perm(0u, 0x54474341u, sel);
}

__device__ void build_tables(SketchTablesQ &tb, uint32_t tid, uint32_t nthreads) {
    constexpr uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
    for (uint32_t x = tid; x < 256; x += nthreads) {
        const uint32_t a = ascii4(x);
        const uint64_t A1 = (uint64_t)a * c1, A2 = (uint64_t)a * c2;
        const uint32_t x1 = (uint32_t)A1, x2 = (uint32_t)A2;
        const uint32_t ta1 = (uint32_t)(A1 >> 32), ta2 = (uint32_t)(A2 >> 32);
        const uint64_t t1 = ((uint64_t)x1 << 31) * c2 + ((uint64_t)(ta1 << 31) << 32);
        const uint64_t t2 = ((uint64_t)(x2 & 0x7fffffffu) << 33) * c1 + (uint64_t)(x2 >> 31) * c1;
        tb.e1[x] = u32x4{(uint32_t)t1, (uint32_t)(t1 >> 32), ta1, 0u};
        constexpr uint32_t d1hi = (uint32_t)((c1 * 2) >> 32);
        tb.e2[x] = u32x4{(uint32_t)t2, (uint32_t)(t2 >> 32), ta2, ta2 * d1hi};
        const uint32_t m1 = a * (uint32_t)c1;
        tb.b1[x] = u32x2{m1, m1 << 31};
        const uint32_t m2 = a * (uint32_t)c2;
        tb.b2[x] = u32x2{m2, m2 * d1hi};
    }
    for (uint32_t y = tid; y < 1024; y += nthreads) {
        // bases 16..19 = bits 9..2, base 20 = bits 1..0
        const uint64_t k3 = (uint64_t)ascii4(y >> 2) | ((uint64_t)ascii4((y & 3u) << 6) & 0xffu) << 32;
        tb.t3[y] = (rotl64_ab(k3 * c1, 31) * c2) ^ 21u;
    }
}

// The tables depend on nothing but the Murmur constants: built once per
// context into a device image (k_sketch_tables), which every hash workgroup
// copies into LDS with 16-byte loads (~5 per lane, L2-resident) instead of
// recomputing ~1,300 entries (the build cost ~1.2 VALU instructions per k-mer).
constexpr uint32_t kTabVec = sizeof(SketchTablesQ) / 16;
constexpr uint32_t kSketchTabShifts = 4u | (3u << 8);     // log2 of the 16- and 8-byte entry sizes (fetch_ent)
static_assert(sizeof(SketchTablesQ) % 16 == 0, "table image is copied in 16-byte pieces");
__global__ __launch_bounds__(256) void k_sketch_tables(SketchTablesQ *__restrict__ img) {
    __shared__ SketchTablesQ tb;
    build_tables(tb, threadIdx.x, 256);
    __syncthreads();
    const u32x4 *src = (const u32x4 *)&tb;
    u32x4 *dst = (u32x4 *)img;
    for (uint32_t i = threadIdx.x; i < kTabVec; i += 256) dst[i] = src[i];
}

__device__ __forceinline__ uint32_t rev_fields16(uint32_t x) {     // reverse the 16 2-bit fields
    const uint32_t y = __builtin_bitreverse32(x);
    return ((y >> 1) & 0x55555555u) | ((y & 0x55555555u) << 1);
}

__device__ __forceinline__ uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) {   // one v_mad_u64_u32
    return (uint64_t)a * b + c;
}

// Murmur h1 of the canonical k-mer (top-aligned codes hi:lo), returned as the
// two fmix64 states q1, q2 before their last multiply: with p = q C2,
// h1 = fin(p1) + fin(p2), fin(k) = k ^ (k >> 33).  fin leaves the high word
// unchanged, so
//     h1 <= T  implies  hi(p1) + hi(p2) + 1  <=  hi(T) + 1   (mod 2^32)
// (the low-word sum carries at most 1 into the high word; both sides are
// taken one past so a wrapping 0xFFFFFFFF + carry = 0 is kept): the prefilter
// (prefilter_hi, the two high words with shared multiplies, and a compare);
// the exact test runs in the rare admit branch.
// the five table entries of one k-mer
struct MEnt { u32x4 e1; u32x2 f1; u32x4 e2; u32x2 f2; uint64_t k3; };
// Table addresses are byte index << entry size.  The shift amounts come in
// as kernel arguments (sh = 4 | 3 << 8, held in SGPRs): with literal shifts the
// compiler rematerialised 4 and 3 into VGPRs for the byte-select shifts of
// every k-mer (two v_mov_b32 each)
#ifndef DREPHIP_SK_ABLATE
#define DREPHIP_SK_ABLATE 0
#endif
__device__ __forceinline__ MEnt fetch_ent(const SketchTablesQ &tb, uint32_t hi, uint32_t lo, uint32_t sh) {
    const char *base = (const char *)&tb;
#if DREPHIP_SK_ABLATE
    // A/B build for the binding-resource measurement (tools/sketch_ablate.py;
    // never the product): every table index is ANDed with a mask from the
    // kernel argument -- all ones (real lookups, +5 VALU per k-mer) or zero
    // (every lane reads entry 0: broadcast, no bank conflicts) -- so the two
    // runs issue the same instructions and differ only in the LDS bank traffic
    const uint32_t s16 = sh & 0xfu, s8 = (sh >> 8) & 0xfu, km = (sh >> 16) & 0x3ffu;
#if DREPHIP_SK_ABLATE == 2
    // no tables at all: the entries are the k-mer's own words (no LDS read, no
    // address arithmetic; the hash is garbage) -- the VALU-only time of the rest
    (void)base; (void)s16; (void)s8; (void)km;
    return MEnt{u32x4{hi, lo, hi, lo}, u32x2{lo, hi}, u32x4{lo, hi, lo, hi}, u32x2{hi, lo},
                ((uint64_t)hi << 32) | lo};
#endif
    return MEnt{*(const u32x4 *)(base + (((hi >> 24) & km) << s16)),
                *(const u32x2 *)(base + offsetof(SketchTablesQ, b1) + (((hi >> 16) & km & 0xffu) << s8)),
                *(const u32x4 *)(base + offsetof(SketchTablesQ, e2) + (((hi >> 8) & km & 0xffu) << s16)),
                *(const u32x2 *)(base + offsetof(SketchTablesQ, b2) + ((hi & km & 0xffu) << s8)),
                tb.t3[(lo >> 22) & km]};
#else
    const uint32_t s16 = sh & 0xffu, s8 = sh >> 8;
    return MEnt{*(const u32x4 *)(base + ((hi >> 24) << s16)),
                *(const u32x2 *)(base + offsetof(SketchTablesQ, b1) + (((hi >> 16) & 0xffu) << s8)),
                *(const u32x4 *)(base + offsetof(SketchTablesQ, e2) + (((hi >> 8) & 0xffu) << s16)),
                *(const u32x2 *)(base + offsetof(SketchTablesQ, b2) + ((hi & 0xffu) << s8)),
                tb.t3[lo >> 22]};
#endif
}
__device__ __forceinline__ void murmur21_ent(const MEnt &E, uint32_t seed, uint64_t &q1, uint64_t &q2) {
    constexpr uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
    constexpr uint64_t d1 = c1 * 2;                                  // 2 c1 mod 2^64
    const u32x4 e1 = E.e1;
    const u32x2 f1 = E.f1;
    const u32x4 e2 = E.e2;
    const u32x2 f2 = E.f2;
    const uint64_t k3 = E.k3;
    const uint32_t X1 = e1.z + f1.x;                                 // hi(k1 * c1)
    const uint32_t X2 = e2.z + f2.x;                                 // hi(k2 * c2)
    const uint64_t tt1 = ((uint64_t)e1.y << 32) | e1.x;
    const uint64_t tt2 = ((uint64_t)e2.y << 32) | e2.x;
    // rotl(k1 c1, 31) c2 ^ seed  (its (X1 << 31) term: in e1.y and f1.y)
    const uint32_t h = X1 >> 1;
    const uint64_t P1 = mad64(h, (uint32_t)c2, tt1);
    const uint32_t g1hi = (uint32_t)(P1 >> 32) + h * (uint32_t)(c2 >> 32) + f1.y;
    uint64_t h1 = ((uint64_t)g1hi << 32) | ((uint32_t)P1 ^ seed);
    h1 = x5_plus(rotl64_ab(h1, 27), 5ull * seed + 0x52dce729);   // (rotl + seed) * 5 + c
    // rotl(k2 c2, 33) c1 ^ seed
    const uint64_t P2 = mad64(X2, (uint32_t)d1, tt2);
    // X2 hi(d1) = e2.z hi(d1) + f2.x hi(d1) (mod 2^32): both products are table
    // entries, one add instead of a move and a multiply
    const uint32_t g2hi = (uint32_t)(P2 >> 32) + e2.w + f2.y;
    uint64_t h2 = ((uint64_t)g2hi << 32) | ((uint32_t)P2 ^ seed);
    h2 = x5_plus(add64(rotl64_ab(h2, 31), h1), 0x38495ab5);
    h1 ^= k3;
    h2 ^= 21u;
    h1 = add64(h1, h2);
    h2 = add64(h2, h1);
    q1 = fmix64_q(h1);
    q2 = fmix64_q(h2);
}
__device__ __forceinline__ void murmur21_q(const SketchTablesQ &tb, uint32_t hi, uint32_t lo, uint32_t seed,
                                           uint32_t sh, uint64_t &q1, uint64_t &q2) {
    murmur21_ent(fetch_ent(tb, hi, lo, sh), seed, q1, q2);
}
__device__ __forceinline__ uint64_t murmur_fin(uint64_t q1, uint64_t q2) {
    const uint64_t p1 = fmix_mul(q1), p2 = fmix_mul(q2);
    return add64(p1 ^ (p1 >> 33), p2 ^ (p2 >> 33));
}

#ifndef DREPHIP_SK_BATCH
#define DREPHIP_SK_BATCH 2          // k-mers per admit test: 52 VGPRs (4: 58, 0.8 % slower; 8: 73, 7 waves, 2 % slower;
                                    // all 16 of a chunk as one block, keeping only the prefilter bits and recomputing
                                    // the rare hits: 56 VGPRs, 4 % slower -- profiles/r03_sketch_ab_block16.txt).
                                    // Issuing a batch's table reads before its hash (64 VGPRs), or the next
                                    // k-mer's reads before this one's (65; capped at 64: 8 B of spill) measured
                                    // 0.3-0.7 % slower (profiles/r03_sketch_ab_sched.txt): the LDS latency is
                                    // already covered by the other waves
#endif
#ifndef DREPHIP_SK_MINW
#define DREPHIP_SK_MINW 1
#endif
// window ends per lane: 64, i.e. 512-lane workgroups per 32768-base tile.  The
// tables (23.5 KiB of LDS per workgroup) then serve 8 waves instead of 4, so
// LDS allows 8 waves per SIMD instead of 6: 1.3 % faster than 128 (8.24 vs
// 8.35 ms, same box; 32 window ends per lane: 8.37 ms)
constexpr uint32_t kHashLane = 64;
template <int LANE, int BATCH>
__global__ __launch_bounds__(kTile / LANE, DREPHIP_SK_MINW) void k_sketch_hash21(
    const SketchTablesQ *__restrict__ img, const uint32_t *__restrict__ codes, const uint32_t *__restrict__ valid,
    const uint64_t *__restrict__ tile_base, const uint32_t *__restrict__ tile_genome,
    const uint64_t *__restrict__ thr, unsigned long long *__restrict__ sets,
    uint32_t *__restrict__ cnt, uint32_t set_log2, uint32_t limit, uint32_t seed, uint64_t wlast, uint32_t sh) {
    constexpr uint32_t WG = kTile / LANE;
    constexpr int NCH = LANE / 16;
    __shared__ SketchTablesQ tb;
    __shared__ uint64_t stage[kStage];
    __shared__ uint32_t nstage;
    const uint32_t t = blockIdx.x;
    const uint32_t g = tile_genome[t];
    const uint64_t T = thr[g];
    const uint32_t Thi = (uint32_t)(T >> 32);
    const uint32_t Tp = Thi == 0xFFFFFFFFu ? Thi : Thi + 1;     // prefilter bound (see murmur21_q)
    const uint64_t start = tile_base[t] + (uint64_t)threadIdx.x * LANE;
    const uint32_t mask = (1u << set_log2) - 1;
    unsigned long long *S = sets + ((uint64_t)g << set_log2);
    uint32_t *C = cnt + g;
    if (threadIdx.x == 0) nstage = 0;
    {
        const u32x4 *src = (const u32x4 *)img;
        u32x4 *dst = (u32x4 *)&tb;
        for (uint32_t i = threadIdx.x; i < kTabVec; i += WG) dst[i] = src[i];
    }

    // code words through a per-workgroup buffer resource based two words before
    // the tile: the lane's word offset is a fixed VGPR, the word index an
    // immediate or SGPR, and words past wlast read 0 (buffer bounds) -- junk
    // either way, every k-mer touching them is invalid
    const uint64_t w0 = tile_base[t] / 16 - 2;       // >= 0: genomes start at tile 1
    const uint64_t nrec = (wlast + 1 - w0) * 4;
    const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(codes + w0), (short)0, (int)(nrec < 0xFFFFFFF0ull ? nrec : 0xFFFFFFF0ull), 0x00020000);
    const uint32_t lane_off = threadIdx.x * (LANE / 16) * 4;
    auto ld = [&](int j) -> uint32_t {               // word m0 + j, m0 = the lane's first window end / 16
        return __builtin_amdgcn_raw_buffer_load_b32(crs, lane_off, (uint32_t)__builtin_amdgcn_readfirstlane(j + 2) * 4u, 0);
    };
    // registers: F words m-2..m (complemented), R words m-2..m+1
    uint32_t nf0 = ~ld(-2), nf1 = ~ld(-1), nf2 = ~ld(0);
    uint32_t r0 = rev_fields16(~nf0), r1 = rev_fields16(~nf1), r2 = rev_fields16(~nf2);
    uint32_t f3 = ld(1);                             // raw F[m+1]
    uint32_t r3 = rev_fields16(f3);
    uint32_t fnext = ld(2);
    const uint32_t *vw = valid + (start - kWarm) / 32;
    uint64_t vhist = (uint64_t)vw[0] << 32;          // bit 63 = newest base
    uint32_t vcur = vw[1];
    __syncthreads();

    // fully unrolled (NCH = 4 chunks of 16 window ends): the code-word
    // registers rotate by renaming and every load is issued up front.  Rolled,
    // the compiler copied the rotating words at the back edge behind a wait
    // for the chunk's own load (7.84 vs 8.00 ms).  The count is explicit: a
    // bare `#pragma unroll` produced different, slower code (8.09 ms)
    static_assert(NCH == 4, "unroll count");
#pragma unroll 4
    for (int wi = 0; wi < NCH; wi++) {
        const uint32_t vbits = (vcur >> ((wi & 1) * 16)) & 0xffffu;
        if (wi + 1 < NCH && (wi & 1)) vcur = vw[2 + (wi >> 1)];
        vhist = (vhist >> 16) | ((uint64_t)vbits << 48);
        // canonical k-mer (top-aligned codes) of window end q = 16m + r
        auto canon = [&](int r) -> uint64_t {
            uint32_t chi, clo, fhi, flo;
            if (r == 15) { chi = nf2; clo = nf1; }
            else {
                chi = __builtin_amdgcn_alignbit(nf2, nf1, 2 * (r + 1));
                clo = __builtin_amdgcn_alignbit(nf1, nf0, 2 * (r + 1));
            }
            if (r < 4) {                             // k-mer starts in word m-2 at field r+12
                fhi = __builtin_amdgcn_alignbit(r0, r1, 32 - 2 * (r + 12));
                flo = __builtin_amdgcn_alignbit(r1, r2, 32 - 2 * (r + 12));
            } else if (r == 4) {
                fhi = r1; flo = r2;
            } else {                                 // starts in word m-1 at field r-4
                fhi = __builtin_amdgcn_alignbit(r1, r2, 32 - 2 * (r - 4));
                flo = __builtin_amdgcn_alignbit(r2, r3, 32 - 2 * (r - 4));
            }
            const uint64_t fw = ((uint64_t)fhi << 32) | flo;
            const uint64_t rc = ((uint64_t)chi << 32) | clo;
            return fw <= rc ? fw : rc;
        };
#pragma unroll
        for (int b0 = 0; b0 < 16; b0 += BATCH) {
            uint64_t p1[BATCH], p2[BATCH];
            bool hit = false;
#pragma unroll
            for (int b = 0; b < BATCH; b++) {
                const uint64_t cc = canon(b0 + b);
                murmur21_q(tb, (uint32_t)(cc >> 32), (uint32_t)cc, seed, sh, p1[b], p2[b]);
                hit |= prefilter_hi(p1[b], p2[b]) <= Tp;
            }
            if (__builtin_expect(hit, 0)) {
#pragma unroll
                for (int b = 0; b < BATCH; b++) {
                    const uint64_t h = murmur_fin(p1[b], p2[b]);
                    // the 21 bases ending at history bit 48 + r are all valid
                    // (per k-mer, here: a shared run mask over the whole chunk
                    // was hoisted out of this rare branch into every chunk)
                    const bool ok = (~(uint32_t)(vhist >> (28 + b0 + b)) & 0x1FFFFFu) == 0;
                    if (h <= T && ok) {
                        const uint32_t slot = atomicAdd(&nstage, 1u);
                        if (slot < kStage) stage[slot] = h;
                        else set_insert(S, mask, C, limit, h);
                    }
                }
            }
        }
        // slide one code word
        nf0 = nf1; nf1 = nf2; nf2 = ~f3;
        r0 = r1; r1 = r2; r2 = r3;
        f3 = fnext;
        r3 = rev_fields16(f3);
        fnext = ld(wi + 3);
    }
    __syncthreads();
    const uint32_t n = min(nstage, kStage);
    for (uint32_t i = threadIdx.x; i < n; i += WG) set_insert(S, mask, C, limit, stage[i]);
}

// ----------------------------------------------------------------- finalize
enum : uint8_t { ST_OK = 0, ST_UP = 1, ST_DOWN = 2 };

// Every finalize leaves the genome's candidate set empty and its count zero
// (the slots it reads are reset as it goes; a genome sent back for another
// round is reset whole), so the next call needs no memset of the sets.
__device__ __forceinline__ void finalize_reset(unsigned long long *S, uint32_t slots, uint32_t *cnt_g) {
    for (uint32_t i = threadIdx.x; i < slots; i += blockDim.x) S[i] = kEmpty;
    __syncthreads();                                   // every thread has read *cnt_g
    if (threadIdx.x == 0) *cnt_g = 0;
}

// Bucket-sort finalize.  The candidates of one genome are distinct
// hashes <= T spread evenly over [0, T], so a counting sort on their top bits
// (NB buckets, bucket = h >> shift with T >> shift < NB; monotone in h) leaves
// ~1-4 hashes per bucket, which one thread then insertion-sorts in LDS.  Exact
// for any input (only the speed depends on the spread).  Replaces the
// P log^2 P bitonic network: at s = 10^4 the sort of 16384 candidates took
// 105 barrier-separated stages.
template <int MAXC, int NB>
__global__ __launch_bounds__(1024) void k_sketch_finalize_bucket(
    unsigned long long *__restrict__ sets, uint32_t *__restrict__ cnt,
    const uint64_t *__restrict__ thr, const uint32_t *__restrict__ glist, uint32_t set_log2,
    uint32_t maxc, uint32_t s, uint64_t *__restrict__ out, uint32_t *__restrict__ nhash,
    uint8_t *__restrict__ status) {
    constexpr uint32_t WG = 1024, PER = NB / WG, LOGNB = __builtin_ctz(NB);
    static_assert(NB % WG == 0 && (NB & (NB - 1)) == 0, "NB: power of two, multiple of the workgroup");
    __shared__ uint64_t buf[MAXC];
    __shared__ uint32_t bk[NB];            // counts, then running end offsets
    __shared__ uint32_t wsum[WG / 64];
    const uint32_t g = glist[blockIdx.x];
    const uint32_t n = cnt[g];
    const uint32_t tid = threadIdx.x;
    const uint64_t T = thr[g];
    unsigned long long *S = sets + ((uint64_t)g << set_log2);
    const uint32_t slots = 1u << set_log2;
    if (n > maxc || (n < s && T < kMaxThr)) {
        if (tid == 0) status[g] = n > maxc ? ST_DOWN : ST_UP;
        finalize_reset(S, slots, cnt + g);
        return;
    }
    const uint32_t tbits = 64 - __builtin_clzll(T | 1);
    const uint32_t shift = tbits > LOGNB ? tbits - LOGNB : 0;
    for (uint32_t i = tid; i < NB; i += WG) bk[i] = 0;
    __syncthreads();
    if (tid == 0) cnt[g] = 0;                          // every thread has read it
    for (uint32_t i = tid; i < slots; i += WG) {
        const uint64_t v = S[i];
        if (v != kEmpty) atomicAdd(&bk[min((uint32_t)(v >> shift), (uint32_t)NB - 1u)], 1u);
    }
    __syncthreads();
    // exclusive scan of the counts: PER consecutive buckets per thread, a
    // wave scan of the thread sums, then the 16 wave totals
    uint32_t loc[PER], sum = 0;
#pragma unroll
    for (int j = 0; j < PER; j++) { loc[j] = sum; sum += bk[tid * PER + j]; }
    uint32_t inc = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if ((tid & 63) >= d) inc += y;
    }
    if ((tid & 63) == 63) wsum[tid >> 6] = inc;
    __syncthreads();
    uint32_t base = inc - sum;
    for (uint32_t w = 0; w < (tid >> 6); w++) base += wsum[w];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PER; j++) bk[tid * PER + j] = base + loc[j];
    __syncthreads();
    for (uint32_t i = tid; i < slots; i += WG) {
        const uint64_t v = S[i];
        if (v != kEmpty) {
            buf[atomicAdd(&bk[min((uint32_t)(v >> shift), (uint32_t)NB - 1u)], 1u)] = v;
            S[i] = kEmpty;
        }
    }
    __syncthreads();
    // bk[b] is now the end of bucket b (= the start of bucket b + 1)
    for (uint32_t b = tid; b < NB; b += WG) {
        const uint32_t lo = b ? bk[b - 1] : 0, hi = bk[b];
        for (uint32_t i = lo + 1; i < hi; i++) {
            const uint64_t v = buf[i];
            uint32_t j = i;
            while (j > lo && buf[j - 1] > v) { buf[j] = buf[j - 1]; j--; }
            buf[j] = v;
        }
    }
    __syncthreads();
    const uint32_t m = n < s ? n : s;
    uint64_t *o = out + (uint64_t)g * s;
    for (uint32_t i = tid; i < s; i += WG) o[i] = i < m ? buf[i] : kEmpty;
    if (tid == 0) { nhash[g] = m; status[g] = ST_OK; }
}

// The same bucket sort for sketches above kLdsSortSketch (more candidates than
// the LDS holds): the bucket counts stay in LDS, the candidates go to a
// per-workgroup slice of a global buffer (gbuf + blockIdx.x * maxc, L2-resident
// at these sizes) and each bucket (~2-3 hashes) is insertion-sorted there.
// The grid is at most kFinGlobalSlices workgroups, each looping over the
// genome list, so the buffer stays bounded (kFinGlobalSlices * maxc * 8 B,
// 2 GiB at s = 32767) however many genomes one call sketches.
constexpr uint32_t kFinGlobalSlices = 2048;
template <int NB>
__global__ __launch_bounds__(1024) void k_sketch_finalize_global(
    unsigned long long *__restrict__ sets, uint32_t *__restrict__ cnt,
    const uint64_t *__restrict__ thr, const uint32_t *__restrict__ glist, uint32_t ng, uint32_t set_log2,
    uint32_t maxc, uint32_t s, uint64_t *__restrict__ out, uint32_t *__restrict__ nhash,
    uint8_t *__restrict__ status, uint64_t *__restrict__ gbuf) {
    constexpr uint32_t WG = 1024, PER = NB / WG, LOGNB = __builtin_ctz(NB);
    static_assert(NB % WG == 0 && (NB & (NB - 1)) == 0, "NB: power of two, multiple of the workgroup");
    __shared__ uint32_t bk[NB];            // counts, then running end offsets
    __shared__ uint32_t wsum[WG / 64];
    const uint32_t tid = threadIdx.x;
    uint64_t *buf = gbuf + (uint64_t)blockIdx.x * maxc;
    const uint32_t slots = 1u << set_log2;
    for (uint32_t gi = blockIdx.x; gi < ng; gi += gridDim.x) {
        const uint32_t g = glist[gi];
        const uint32_t n = cnt[g];
        const uint64_t T = thr[g];
        unsigned long long *S = sets + ((uint64_t)g << set_log2);
        if (n > maxc || (n < s && T < kMaxThr)) {         // (uniform over the workgroup)
            if (tid == 0) status[g] = n > maxc ? ST_DOWN : ST_UP;
            finalize_reset(S, slots, cnt + g);
            __syncthreads();
            continue;
        }
        const uint32_t tbits = 64 - __builtin_clzll(T | 1);
        const uint32_t shift = tbits > LOGNB ? tbits - LOGNB : 0;
        for (uint32_t i = tid; i < NB; i += WG) bk[i] = 0;
        __syncthreads();
        if (tid == 0) cnt[g] = 0;                          // every thread has read it
        for (uint32_t i = tid; i < slots; i += WG) {
            const uint64_t v = S[i];
            if (v != kEmpty) atomicAdd(&bk[min((uint32_t)(v >> shift), (uint32_t)NB - 1u)], 1u);
        }
        __syncthreads();
        uint32_t loc[PER], sum = 0;
#pragma unroll
        for (int j = 0; j < PER; j++) { loc[j] = sum; sum += bk[tid * PER + j]; }
        uint32_t inc = sum;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(inc, d, 64);
            if ((tid & 63) >= d) inc += y;
        }
        if ((tid & 63) == 63) wsum[tid >> 6] = inc;
        __syncthreads();
        uint32_t base = inc - sum;
        for (uint32_t w = 0; w < (tid >> 6); w++) base += wsum[w];
        __syncthreads();
#pragma unroll
        for (int j = 0; j < PER; j++) bk[tid * PER + j] = base + loc[j];
        __syncthreads();
        for (uint32_t i = tid; i < slots; i += WG) {
            const uint64_t v = S[i];
            if (v != kEmpty) {
                buf[atomicAdd(&bk[min((uint32_t)(v >> shift), (uint32_t)NB - 1u)], 1u)] = v;
                S[i] = kEmpty;
            }
        }
        // the scatter's global stores are visible to the sorting threads of this
        // workgroup after the barrier (same CU, device-coherent L2 path)
        __threadfence_block();
        __syncthreads();
        for (uint32_t b = tid; b < NB; b += WG) {
            const uint32_t lo = b ? bk[b - 1] : 0, hi = bk[b];
            for (uint32_t i = lo + 1; i < hi; i++) {
                const uint64_t v = buf[i];
                uint32_t j = i;
                while (j > lo && buf[j - 1] > v) { buf[j] = buf[j - 1]; j--; }
                buf[j] = v;
            }
        }
        __threadfence_block();
        __syncthreads();
        const uint32_t m = n < s ? n : s;
        uint64_t *o = out + (uint64_t)g * s;
        for (uint32_t i = tid; i < s; i += WG) o[i] = i < m ? buf[i] : kEmpty;
        if (tid == 0) { nhash[g] = m; status[g] = ST_OK; }
        __syncthreads();                                   // buf and bk are reused by the next genome
    }
}

__global__ void k_reset_sets(unsigned long long *__restrict__ sets, uint32_t *__restrict__ cnt,
                             const uint32_t *__restrict__ glist, uint32_t set_log2) {
    const uint32_t g = glist[blockIdx.x];
    unsigned long long *S = sets + ((uint64_t)g << set_log2);
    const uint32_t slots = 1u << set_log2;
    for (uint32_t i = threadIdx.x; i < slots; i += blockDim.x) S[i] = kEmpty;
    if (threadIdx.x == 0) cnt[g] = 0;
}

// ----------------------------------------------------------------- synth
// One thread per 32-base word pair (two code words + one validity word).
__global__ void k_synth(uint64_t seed, uint32_t g0, uint32_t n, uint32_t fam, uint64_t L,
                        uint64_t P, uint32_t *__restrict__ codes, uint32_t *__restrict__ valid,
                        uint64_t nwords32, uint64_t w0) {
    const uint64_t w = w0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= nwords32) return;
    const uint64_t p0 = w * 32;
    uint32_t c_lo = 0, c_hi = 0, v = 0;
    if (p0 >= kTile) {
        const uint64_t rel = p0 - kTile;
        const uint32_t i = (uint32_t)(rel / P);
        const uint64_t q0 = rel - (uint64_t)i * P;   // 32-aligned (P is a tile multiple)
        if (i < n && q0 < L) {
            const uint32_t g = g0 + i;
            const uint32_t f = g / fam;
            const uint64_t anc = splitmix64((kSynA ^ seed) ^ ((uint64_t)f << 32) ^ (q0 >> 5));
            const uint32_t thr = synth_rate_thr((uint32_t)(splitmix64((kSynR ^ seed) ^ g) % 7));
            for (int b = 0; b < 32; b++) {
                const uint64_t q = q0 + b;
                if (q >= L) break;
                uint32_t c = (uint32_t)(anc >> (2 * b)) & 3u;
                const uint64_t u = splitmix64((kSynM ^ seed) ^ ((uint64_t)g << 32) ^ q);
                if ((uint32_t)(u >> 32) < thr) c = (c + 1 + (uint32_t)(u & 0xffffffffu) % 3u) & 3u;
                if (b < 16) c_lo |= c << (2 * b); else c_hi |= c << (2 * (b - 16));
                v |= 1u << b;
            }
        }
    }
    codes[2 * w] = c_lo;
    codes[2 * w + 1] = c_hi;
    valid[w] = v;
}

// ------------------------------------------------------------- host driver
static uint64_t initial_threshold(uint64_t nk, uint32_t s, double F) {
    const double E = F * (double)s;
    if ((double)nk <= E) return kMaxThr;
    const long double t = (long double)18446744073709551616.0L * (long double)E / (long double)nk;
    if (t >= (long double)kMaxThr) return kMaxThr;
    return (uint64_t)t < 1 ? 1 : (uint64_t)t;
}

struct SketchPlan {
    uint32_t maxc, set_log2;
    double F;
};
static SketchPlan plan_for(uint32_t s) {
    SketchPlan p;
    p.F = s <= 4096 ? 2.0 : 1.3;
    const double E = p.F * s;
    uint32_t mc = 1024;
    // LDS sort up to 16384 candidates (s <= kLdsSortSketch), else the global one
    const uint32_t mcmax = s <= kLdsSortSketch ? 16384u : (1u << 17);
    while (mc < 2 * E && mc < mcmax) mc <<= 1;
    p.maxc = mc;
    p.set_log2 = 1;
    while ((1u << p.set_log2) < 2 * mc) p.set_log2++;
    return p;
}

// the hash kernel's `sh` argument: the table entry shifts; in the ablation
// build also the index mask (DREPHIP_SK_KMASK, default all ones)
static uint32_t sk_shifts() {
#if DREPHIP_SK_ABLATE
    const char *m = getenv("DREPHIP_SK_KMASK");
    return kSketchTabShifts | ((m ? (uint32_t)strtoul(m, nullptr, 0) : 0x3FFu) & 0xFFFFu) << 16;
#else
    return kSketchTabShifts;
#endif
}

int sketch_device_impl(drephip_ctx *ctx, const uint32_t *d_codes, const uint32_t *d_valid,
                       const uint64_t *base_off, const uint64_t *padded, const uint64_t *nkmers,
                       uint32_t n, uint64_t *d_hashes, uint32_t *d_nhash, hipStream_t st,
                       bool defer) {
    if (n == 0) return DREPHIP_OK;
    if (ctx->k != 21) { set_error("sketch kernel is instantiated for k=21 (Mash/dRep default) only"); return DREPHIP_ERR_UNSUPPORTED; }
    const uint32_t s = ctx->s;
    const SketchPlan plan = plan_for(s);
    const uint64_t slots = 1ull << plan.set_log2;
    const uint32_t limit = (uint32_t)(slots * 3 / 4);

    // tile table (tile -> base, genome), reused across calls on the same layout
    std::vector<uint64_t> tfirst(n + 1, 0);           // first tile of each genome
    uint64_t wlast = 0;                                // last code word any tile may touch
    for (uint32_t g = 0; g < n; g++) {
        if (base_off[g] % kTile || padded[g] % kTile || base_off[g] < kTile) {
            set_error("genome base_off/padded must be tile multiples and base_off >= tile");
            return DREPHIP_ERR_ARG;
        }
        tfirst[g + 1] = tfirst[g] + padded[g] / kTile;
        wlast = std::max(wlast, (base_off[g] + padded[g]) / 16 - 1);
    }
    if (tfirst[n] >= (1ull << 31)) { set_error("too many tiles in one sketch call"); return DREPHIP_ERR_ARG; }
    const uint32_t ntiles = (uint32_t)tfirst[n];
    std::vector<uint64_t> T(n), lo(n, 0), hi(n, 0);   // hi == 0: unknown
    for (uint32_t g = 0; g < n; g++) T[g] = initial_threshold(nkmers[g], s, plan.F);

    uint64_t *d_tb, *d_thr, *d_tbsub;
    uint32_t *d_tg, *d_cnt, *d_gl, *d_tgsub;
    unsigned long long *d_sets;
    uint8_t *d_st;
    int rc;
    if ((rc = scratch(ctx, "sk_tb", ntiles * 8ull, (void **)&d_tb))) return rc;
    if ((rc = scratch(ctx, "sk_tg", ntiles * 4ull, (void **)&d_tg))) return rc;
    if ((rc = scratch(ctx, "sk_tbsub", ntiles * 8ull, (void **)&d_tbsub))) return rc;
    if ((rc = scratch(ctx, "sk_tgsub", ntiles * 4ull, (void **)&d_tgsub))) return rc;
    if ((rc = scratch(ctx, "sk_thr", n * 8ull, (void **)&d_thr))) return rc;
    if ((rc = scratch(ctx, "sk_cnt", n * 4ull, (void **)&d_cnt))) return rc;
    if ((rc = scratch(ctx, "sk_gl", n * 4ull, (void **)&d_gl))) return rc;
    if ((rc = scratch(ctx, "sk_st", n * 1ull, (void **)&d_st))) return rc;
    if ((rc = scratch(ctx, "sk_sets", (uint64_t)n * slots * 8ull, (void **)&d_sets))) return rc;
    // Murmur table image (once per context; rebuilt after any reallocation)
    SketchTablesQ *d_img;
    if ((rc = scratch(ctx, "sk_tables", sizeof(SketchTablesQ), (void **)&d_img))) return rc;
    if (ctx->sk_tab_gen != ctx->alloc_gen) {
        hipLaunchKernelGGL(k_sketch_tables, dim3(1), dim3(256), 0, st, d_img);
        HIPC(hipGetLastError());
        ctx->sk_tab_gen = ctx->alloc_gen;
    }
    // first-round thresholds and genome list: device copies cached with the tile table
    uint64_t *d_thr0;
    uint32_t *d_gl0;
    uint8_t *h_st;                                     // pinned: the per-round status readback
    if ((rc = scratch(ctx, "sk_thr0", n * 8ull, (void **)&d_thr0))) return rc;
    if ((rc = scratch(ctx, "sk_gl0", n * 4ull, (void **)&d_gl0))) return rc;
    if ((rc = pinned_host(ctx, "sk_status", n, (void **)&h_st))) return rc;

    const bool cached = ctx->sk_gen == ctx->alloc_gen && ctx->sk_off.size() == n &&
                        !memcmp(ctx->sk_off.data(), base_off, n * 8ull) &&
                        !memcmp(ctx->sk_pad.data(), padded, n * 8ull) &&
                        !memcmp(ctx->sk_nk.data(), nkmers, n * 8ull);
    if (!cached) {
        std::vector<uint64_t> tbase(ntiles);
        std::vector<uint32_t> tgen(ntiles);
        for (uint32_t g = 0; g < n; g++)
            for (uint64_t t = tfirst[g]; t < tfirst[g + 1]; t++) {
                tbase[t] = base_off[g] + (t - tfirst[g]) * kTile;
                tgen[t] = g;
            }
        std::vector<uint32_t> glist(n);
        for (uint32_t g = 0; g < n; g++) glist[g] = g;
        ctx->sk_gen = 0;
        HIPC(hipMemcpyAsync(d_tb, tbase.data(), ntiles * 8ull, hipMemcpyHostToDevice, st));
        HIPC(hipMemcpyAsync(d_tg, tgen.data(), ntiles * 4ull, hipMemcpyHostToDevice, st));
        HIPC(hipMemcpyAsync(d_thr0, T.data(), n * 8ull, hipMemcpyHostToDevice, st));
        HIPC(hipMemcpyAsync(d_gl0, glist.data(), n * 4ull, hipMemcpyHostToDevice, st));
        HIPC(hipStreamSynchronize(st));                // host vectors die here
        ctx->sk_off.assign(base_off, base_off + n);
        ctx->sk_pad.assign(padded, padded + n);
        ctx->sk_nk.assign(nkmers, nkmers + n);
        ctx->sk_gen = ctx->alloc_gen;
    }
    // sets and counts: finalize leaves them empty, so only the part not known
    // to be clean (new buffers, more genomes than before, a failed call) is reset
    const uint32_t clean = (ctx->sk_clean_gen == ctx->alloc_gen && ctx->sk_clean_sets == d_sets &&
                            ctx->sk_clean_cnt == d_cnt) ? ctx->sk_clean_n : 0;
    ctx->sk_clean_n = 0;                               // dirty until this call completes
    if (n > clean) {
        HIPC(hipMemsetAsync(d_sets + (uint64_t)clean * slots, 0xFF, (uint64_t)(n - clean) * slots * 8ull, st));
        HIPC(hipMemsetAsync(d_cnt + clean, 0, (n - clean) * 4ull, st));
    }

    uint8_t *status = h_st;
    std::vector<uint32_t> todo(n);
    for (uint32_t g = 0; g < n; g++) todo[g] = g;
    bool first = true;
    for (int round = 0; round < 130 && !todo.empty(); round++) {
        const uint32_t *tb_tiles_g = d_tg;
        const uint64_t *tb_tiles_b = d_tb;
        const uint64_t *thr_p = first ? d_thr0 : d_thr;   // round 0 reads the cached first-round values
        const uint32_t *gl_p = first ? d_gl0 : d_gl;
        uint32_t nt = ntiles;
        if (!first) {
            // subset: reset sets of the retried genomes, gather their tiles
            std::vector<uint64_t> sb;
            std::vector<uint32_t> sg;
            for (uint32_t g : todo)
                for (uint64_t t = tfirst[g]; t < tfirst[g + 1]; t++) {
                    sb.push_back(base_off[g] + (t - tfirst[g]) * kTile);
                    sg.push_back(g);
                }
            nt = (uint32_t)sb.size();
            HIPC(hipMemcpyAsync(d_tbsub, sb.data(), nt * 8ull, hipMemcpyHostToDevice, st));
            HIPC(hipMemcpyAsync(d_tgsub, sg.data(), nt * 4ull, hipMemcpyHostToDevice, st));
            HIPC(hipMemcpyAsync(d_gl, todo.data(), todo.size() * 4ull, hipMemcpyHostToDevice, st));
            HIPC(hipMemcpyAsync(d_thr, T.data(), n * 8ull, hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL(k_reset_sets, dim3((uint32_t)todo.size()), dim3(256), 0, st, d_sets,
                               d_cnt, d_gl, plan.set_log2);
            tb_tiles_g = d_tgsub;
            tb_tiles_b = d_tbsub;
        }
        if (nt > 0) {
            timing_mark(ctx, 0, st, true);
            for (uint32_t t0 = 0; t0 < nt; t0 += (uint32_t)max_blocks(kTile / kHashLane)) {
                const uint32_t ntc = std::min<uint32_t>(nt - t0, (uint32_t)max_blocks(kTile / kHashLane));
                const uint64_t *tbb = tb_tiles_b + t0;
                const uint32_t *tbg = tb_tiles_g + t0;
                hipLaunchKernelGGL((k_sketch_hash21<kHashLane, DREPHIP_SK_BATCH>), dim3(ntc), dim3(kTile / kHashLane), 0, st,
                                   d_img, d_codes, d_valid, tbb, tbg, thr_p, d_sets, d_cnt, plan.set_log2, limit,
                                   ctx->seed, wlast, sk_shifts());
            }
            timing_mark(ctx, 0, st, false);
        }
        uint64_t *d_gbuf = nullptr;                       // the global finalize's sort buffers (bounded)
        const uint32_t gslices = std::min<uint32_t>((uint32_t)todo.size(), kFinGlobalSlices);
        if (s > kLdsSortSketch &&
            (rc = scratch(ctx, "sk_gbuf", (uint64_t)gslices * plan.maxc * 8ull, (void **)&d_gbuf)))
            return rc;
        timing_mark(ctx, 1, st, true);
        if (s > kLdsSortSketch)
            hipLaunchKernelGGL((k_sketch_finalize_global<16384>), dim3(gslices), dim3(1024), 0, st,
                               d_sets, d_cnt, thr_p, gl_p, (uint32_t)todo.size(), plan.set_log2, plan.maxc, s,
                               d_hashes, d_nhash, d_st, d_gbuf);
        else if (plan.maxc <= 4096)
            hipLaunchKernelGGL((k_sketch_finalize_bucket<4096, 4096>), dim3((uint32_t)todo.size()), dim3(1024), 0, st,
                               d_sets, d_cnt, thr_p, gl_p, plan.set_log2, plan.maxc, s, d_hashes, d_nhash, d_st);
        else
            hipLaunchKernelGGL((k_sketch_finalize_bucket<16384, 4096>), dim3((uint32_t)todo.size()), dim3(1024), 0,
                               st, d_sets, d_cnt, thr_p, gl_p, plan.set_log2, plan.maxc, s, d_hashes, d_nhash, d_st);
        timing_mark(ctx, 1, st, false);
        HIPC(hipGetLastError());
        HIPC(hipMemcpyAsync(status, d_st, n, hipMemcpyDeviceToHost, st));
        if (defer) {
            // deferred: the sets are left empty by finalize whatever the status
            // (finalize_reset), so a rerun from scratch is always valid
            auto &p = ctx->pend;
            p.active = true;
            p.d_codes = d_codes; p.d_valid = d_valid;
            p.off.assign(base_off, base_off + n);
            p.pad.assign(padded, padded + n);
            p.nk.assign(nkmers, nkmers + n);
            p.n = n; p.d_hashes = d_hashes; p.d_nhash = d_nhash; p.st = st;
            p.h_status = status;
            if (!p.done) HIPC(hipEventCreateWithFlags(&p.done, hipEventDisableTiming));
            HIPC(hipEventRecord(p.done, st));
            ctx->sk_clean_gen = ctx->alloc_gen;
            ctx->sk_clean_sets = d_sets;
            ctx->sk_clean_cnt = d_cnt;
            ctx->sk_clean_n = std::max(clean, n);
            return DREPHIP_OK;
        }
        HIPC(hipStreamSynchronize(st));
        first = false;
#if DREPHIP_SK_ABLATE
        if (getenv("DREPHIP_SK_ONE_ROUND")) { todo.clear(); break; }   // timing only: the first round's kernels
#endif
        if (getenv("DREPHIP_DEBUG")) {
            uint32_t nu = 0, nd = 0;
            for (uint32_t g : todo) { nu += status[g] == ST_UP; nd += status[g] == ST_DOWN; }
            fprintf(stderr, "[drephip] sketch round %d: %zu genomes, %u up, %u down\n", round, todo.size(), nu, nd);
            for (uint32_t g : todo) if (status[g] != ST_OK && nu + nd <= 8)
                fprintf(stderr, "[drephip]   genome %u status %d T=%llu\n", g, status[g], (unsigned long long)T[g]);
        }
        std::vector<uint32_t> next;
        for (uint32_t g : todo) {
            if (status[g] == ST_OK) continue;
            if (status[g] == ST_UP) {
                lo[g] = T[g];
                if (hi[g]) T[g] = (uint64_t)(((unsigned __int128)lo[g] + hi[g]) / 2);
                else T[g] = T[g] > kMaxThr / 8 ? kMaxThr : T[g] * 8;
            } else if (status[g] == ST_DOWN) {
                hi[g] = T[g];
                T[g] = (uint64_t)(((unsigned __int128)lo[g] + hi[g]) / 2);
            } else {
                set_error("sketch finalize left an unknown status");
                return DREPHIP_ERR_INTERNAL;
            }
            if (T[g] <= lo[g] || (hi[g] && T[g] >= hi[g])) {
                set_error("sketch threshold bisection did not converge");
                return DREPHIP_ERR_INTERNAL;
            }
            next.push_back(g);
        }
        todo.swap(next);
    }
    if (!todo.empty()) { set_error("sketch did not converge"); return DREPHIP_ERR_INTERNAL; }
    ctx->sk_clean_gen = ctx->alloc_gen;
    ctx->sk_clean_sets = d_sets;
    ctx->sk_clean_cnt = d_cnt;
    ctx->sk_clean_n = std::max(clean, n);
    return DREPHIP_OK;
}

int synth_device_impl(drephip_ctx *ctx, uint64_t seed, uint32_t g0, uint32_t n, uint32_t family_size,
                      uint64_t L, uint32_t *d_codes, uint32_t *d_valid, hipStream_t st) {
    if (family_size == 0) { set_error("family_size must be > 0"); return DREPHIP_ERR_ARG; }
    const uint64_t P = padded_span(L);
    const uint64_t total = kTile + (uint64_t)n * P;
    const uint64_t nw32 = total / 32;
    const uint64_t blocks = (nw32 + 255) / 256;
    for (uint64_t b0 = 0; b0 < blocks; b0 += max_blocks(256))
        hipLaunchKernelGGL(k_synth, dim3((uint32_t)std::min<uint64_t>(blocks - b0, max_blocks(256))), dim3(256), 0, st,
                           seed, g0, n, family_size, L, P, d_codes, d_valid, nw32, b0 * 256);
    HIPC(hipGetLastError());
    HIPC(hipStreamSynchronize(st));
    return DREPHIP_OK;
}

}  // namespace drephip
