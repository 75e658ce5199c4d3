// allpairs.hip -- MI355X all-pairs Mash dist: replaces
// `mash dist -p P ALL.msh ALL.msh` (drep/d_cluster.py:569-573).
//
// Mash's merge (oracle_dist_pair) walks the union of the two sorted sketches
// and stops after s union elements, so a shared hash v counts iff it is one
// of the s smallest elements of A u B.  For v = A[i] = B[j] its union rank is
// i + j - m, m = shared hashes below v, hence
//     common(A,B) = #{ j : B[j] = A[i]  and  i + j - m_j < s },
// m_j = number of matches among B[0..j).  A wave holds a whole column sketch B
// in registers (64-element chunks, one element per lane, coalesced 512-B loads,
// the next column prefetched while this one is processed); membership and i
// come from a quotiented two-choice cuckoo table of A's low words (2H 32-bit
// slots, H >= 2s, load <= 1/4; the slot position implies B bits of the low
// word, which the stored word reuses for i), plus A's high words by position
// (V[i]) to confirm a hit; m_j is the running match count plus a
// ballot/popcount prefix within the chunk.  Elements past A's largest hash
// (A full) cannot match, which ends the scan.  A membership test is two
// independent 4-byte LDS reads (for four interleaved rows: two ds_read_b128)
// and two 32-bit compares; only a row with a hit in the chunk reads V.  The
// next chunk's slot words are read before the current chunk is tested.  R row
// tables live in LDS per workgroup; results are staged in LDS and written as
// contiguous runs of the condensed triangle.
// Roofline: LDS random-read throughput + VALU (integer compare/select); no
// MFMA (set intersection is not a dense contraction).
//
// k_allpairs_band (value bands, s > 2048) and k_allpairs_merge (the literal
// Mash merge, one lane per pair; cross-check and fallback) are further down.

#include "ctx.h"
#include "../../include/drephip.h"

#include <algorithm>
#include <cstring>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <vector>

namespace drephip {

#ifndef DREPHIP_AP_MID
#define DREPHIP_AP_MID 1          // first union-rank test one chunk into its group (ap_columns); 0: at the group start
#endif
constexpr int kApWG = 1024;                     // 16 waves per workgroup
// columns per work item (fewer when the grid would not fill the chip): 512
// amortises the row image's prologue over 4x the columns of round 5's 128 --
// dense 10^4 set 14.9 -> 14.0 ms, configs[2] unscreened 7.1 -> 6.5 ms, 1024
// slower again (profiles/r06_ap_cols_ab.txt); -DDREPHIP_AP_COLS=... for A/Bs
#ifndef DREPHIP_AP_COLS
#define DREPHIP_AP_COLS 512
#endif
constexpr uint32_t kApCols = DREPHIP_AP_COLS;
constexpr uint32_t kApMinCols = 16;             // one column per wave
constexpr uint32_t kApSlots = 2 * 256;          // workgroup slots of the chip (two per CU)
constexpr uint32_t kMaxFam = 6;                 // cuckoo field families tried per table
constexpr uint32_t kFamTwins = 0x40;            // k_build_q32 family byte: the row has two keys with one low word
constexpr uint32_t kFamFailed = 0xFF;           // ... no family worked (the row's pairs are merged literally)
constexpr uint32_t kLdsBudget = 156 * 1024;     // dynamic LDS per workgroup
constexpr uint32_t kScreenMinN = 4096;          // genomes from which the shared-hash screen runs (auto)
constexpr uint32_t kListCols = 512;             // screened columns per whole-row LIST item

__host__ __device__ __forceinline__ uint64_t cond_index(uint64_t i, uint64_t j, uint64_t N) {
    return i * N - i * (i + 1) / 2 + (j - i - 1);
}
__device__ __forceinline__ uint32_t rfl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane(v); }

// ------------------------------------------------------- row tables
// Quotiented two-choice cuckoo table over the keys' low words x = lo32(key):
// choice 1 sits at T[f1(x)], choice 2 at T[H + f2(x)], where f1/f2 are
// disjoint B-bit fields of x at offsets o1/o2 (family f picks them).  Because
// a slot's position p fixes those B bits, the stored word replaces them with
// the key's position i xor p, and is kept rotated right by the field offset:
//     e = rotr32((x & ~F) | ((i ^ p) << o), o)       (field at bits [0, B))
// A probe of slot p = f(b) computes d = e ^ rotr32(b, o): its quotient bits are
// zero iff the slot holds low word lo32(b), and then its field bits are
// (i ^ p) ^ f(b) = i, so d <= 2^B - 1 is the test AND d is the position -- for
// two choices, min(d1, d2) is both.  The key's high word is then compared with
// V[i] = hi32(A[i]).  An empty slot p holds empty_word(p): all-ones quotient,
// field hm ^ p, so a probe that "matches" it (a low word whose quotient is all
// ones) decodes to i = hm, past every real position (H >= 2s), and loses
// every min against a real hit.  Two keys of one row with equal low words
// (twins) occupy the two slots they share; the generic probe retries the
// other choice when the high word does not match, and k_build_q32 keeps rows
// with twins off the fast probe.  Exact for every key.
struct QFields { uint32_t o1, o2; };
__host__ __device__ __forceinline__ uint32_t rotr32(uint32_t x, uint32_t r) {
    return r ? (x >> r) | (x << (32 - r)) : x;
}
__host__ __device__ __forceinline__ QFields qfields(uint32_t fam) {
    // disjoint fields inside the low word for B <= 12 (o + B <= 32).  Family 0
    // (used for nearly every row) takes bits [4, 4+B) and [20, 20+B): with R =
    // 4 interleaved rows a slot is 16 bytes, so the field AS IT STANDS in the
    // key is already the slot's byte address (blo & (hm << 4)) -- one VALU op
    // per choice instead of extract + scale
    const uint32_t o1[6] = {4, 20, 0, 16, 2, 18};
    const uint32_t o2[6] = {20, 4, 16, 0, 18, 2};
    return {o1[fam], o2[fam]};
}

// The empty word of slot `slot` (either region): all-ones quotient, field
// hm ^ p, so that a probe decodes it to position hm
__host__ __device__ __forceinline__ uint32_t empty_word(uint32_t slot, uint32_t hm) {
    return ~hm | ((slot & hm) ^ hm);
}
// Insert (x, ix) into an LDS table whose slot p lives at T[p * stride + col]
// (stride R, col r: the interleaved band tables; stride 1: one row).
__device__ __forceinline__ bool cuckoo_insert32(uint32_t *T, uint32_t stride, uint32_t col, uint32_t H,
                                                uint32_t hm, QFields q, uint32_t x, uint32_t ix) {
    const uint32_t F1 = hm << q.o1, F2 = hm << q.o2;
    uint32_t pos = (x >> q.o1) & hm;
    for (int kick = 0; kick < 96; kick++) {
        const bool second = pos >= H;
        const uint32_t o = second ? q.o2 : q.o1, F = second ? F2 : F1;
        const uint32_t lp = pos & hm;                            // position within the region
        const uint32_t old_r = atomicExch(&T[pos * stride + col], rotr32((x & ~F) | ((ix ^ lp) << o), o));
        if (old_r == empty_word(pos, hm)) return true;
        const uint32_t old = rotr32(old_r, (32 - o) & 31);      // decode the evicted entry
        ix = ((old >> o) & hm) ^ lp;
        x = (old & ~F) | (lp << o);
        pos = second ? ((x >> q.o1) & hm) : (H + ((x >> q.o2) & hm));
    }
    return false;
}
// (x, ix) is stored in one of its two slots
__device__ __forceinline__ bool cuckoo_has32(const uint32_t *T, uint32_t stride, uint32_t col, uint32_t H,
                                             uint32_t hm, QFields q, uint32_t x, uint32_t ix) {
    const uint32_t e1 = T[((x >> q.o1) & hm) * stride + col];
    const uint32_t e2 = T[(H + ((x >> q.o2) & hm)) * stride + col];
    return (e1 ^ rotr32(x, q.o1)) == ix || (e2 ^ rotr32(x, q.o2)) == ix;
}
// Both of x's slots hold a key with x's low word (x and a twin; an empty
// word's false match decodes to hm and does not count)
__device__ __forceinline__ bool cuckoo_twin32(const uint32_t *T, uint32_t stride, uint32_t col, uint32_t H,
                                              uint32_t hm, QFields q, uint32_t x) {
    const uint32_t e1 = T[((x >> q.o1) & hm) * stride + col];
    const uint32_t e2 = T[(H + ((x >> q.o2) & hm)) * stride + col];
    return (e1 ^ rotr32(x, q.o1)) < hm && (e2 ^ rotr32(x, q.o2)) < hm;
}

// One table per row g = row0 + blockIdx.x, written straight into the LDS
// image of its row group (R consecutive rows, `stride` words per group): the
// 2H slot words interleaved with the group's other rows (slot k of row r at
// k*R + r), then the row's s high words at R*2H + r*s.  The main kernel copies
// a group's image into LDS with 16-byte loads.  Rows past row1 (padding of the
// last group) get empty slots.
__global__ __launch_bounds__(1024) void k_build_q32(const uint64_t *__restrict__ hashes,
                                                   const uint32_t *__restrict__ nhash, uint32_t s,
                                                   uint32_t row0, uint32_t row1, uint32_t B, uint32_t R,
                                                   uint32_t *__restrict__ blk, uint32_t stride,
                                                   uint8_t *__restrict__ fam_out) {
    extern __shared__ uint32_t Tb[];
    __shared__ int fail, twins;
    const uint32_t H = 1u << B, hm = H - 1;
    const uint32_t r = blockIdx.x;
    const uint32_t g = row0 + r;
    uint32_t *img = blk + (uint64_t)(r / R) * stride;
    const uint32_t rr = r % R;
    if (g >= row1) {
        for (uint32_t i = threadIdx.x; i < 2 * H; i += blockDim.x) img[i * R + rr] = empty_word(i, hm);
        for (uint32_t i = threadIdx.x; i < s; i += blockDim.x) img[2 * H * R + i * R + rr] = 0;
        if (threadIdx.x == 0) fam_out[r] = 0;
        return;
    }
    const uint32_t n = nhash[g];
    const uint64_t *A = hashes + (uint64_t)g * s;
    for (uint32_t i = threadIdx.x; i < s; i += blockDim.x) img[2 * H * R + i * R + rr] = (uint32_t)(A[i] >> 32);
    for (uint32_t fam = 0; fam < kMaxFam; fam++) {
        const QFields q = qfields(fam);
        for (uint32_t i = threadIdx.x; i < 2 * H; i += blockDim.x) Tb[i] = empty_word(i, hm);
        if (threadIdx.x == 0) { fail = 0; twins = 0; }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < n; i += blockDim.x)
            if (!cuckoo_insert32(Tb, 1, 0, H, hm, q, (uint32_t)A[i], i)) fail = 1;
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < n; i += blockDim.x)
            if (!cuckoo_has32(Tb, 1, 0, H, hm, q, (uint32_t)A[i], i)) fail = 1;
        __syncthreads();
        if (!fail) {
            // twins: two keys with one low word occupy both of their shared
            // slots, so a lookup matches both (two real positions < hm) and
            // min(d1, d2) may name the wrong one -- only the generic probe
            // retries (kFamTwins keeps this row off FAST).  An empty word's
            // false match decodes to hm and never wins the min.
            for (uint32_t i = threadIdx.x; i < n; i += blockDim.x)
                if (cuckoo_twin32(Tb, 1, 0, H, hm, q, (uint32_t)A[i])) twins = 1;
            __syncthreads();
            for (uint32_t i = threadIdx.x; i < 2 * H; i += blockDim.x) img[i * R + rr] = Tb[i];
            if (threadIdx.x == 0) fam_out[r] = (uint8_t)(fam | (twins ? kFamTwins : 0u));
            return;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) fam_out[r] = kFamFailed;    // k_allpairs_q merges this row's pairs literally
}

// ------------------------------------------------------- literal merge
// Mash's merge loop for one pair (oracle_dist_pair): walk the union of the two
// sorted sketches for at most s elements; common = shared hashes seen, denom =
// union elements seen (topped up from the unwalked tails when < s).
__device__ __forceinline__ void merge_pair(const uint64_t *__restrict__ a, uint32_t na,
                                           const uint64_t *__restrict__ b, uint32_t nb, uint32_t s,
                                           uint32_t &common, uint32_t &denom) {
    uint32_t x = 0, y = 0, c = 0, d = 0;
    while (d < s && x < na && y < nb) {
        const uint64_t u = a[x], v = b[y];
        if (u < v) x++;
        else if (v < u) y++;
        else { x++; y++; c++; }
        d++;
    }
    if (d < s) {
        if (x < na) { const uint32_t r = na - x; d += (s - d < r) ? s - d : r; }
        if (y < nb) { const uint32_t r = nb - y; d += (s - d < r) ? s - d : r; }
    }
    common = c;
    denom = d;
}

// ------------------------------------------------------- probe
// Slot words of one chunk element (this lane) for R interleaved row tables
// (slot k of row r at T[k * R + r]): in the FAST layout (family 0 for every
// row) one slot address serves all R rows -- R = 4: one ds_read_b128 per
// choice.
template <int R>
struct Slots { uint32_t e1[R], e2[R]; };

template <int R, bool FAST, int KB, bool ABS = false>
__device__ __forceinline__ Slots<R> read_slots(uint32_t blo, const uint32_t *T, uint32_t H, uint32_t hm,
                                               const uint32_t (&o1)[R], const uint32_t (&o2)[R]) {
    Slots<R> sl;
    if (FAST) {
        // family 0: fields at bits 4 and 20; a slot of R rows is 4R bytes, so
        // its byte offset is the field (x 16) scaled by R/4.  KB = log2 H when
        // known at compile time puts the second region's start in the
        // instruction's offset field.
        const uint32_t f1 = blo & (hm << 4), f2 = (blo >> 16) & (hm << 4);
        const uint32_t a1 = R >= 4 ? f1 * (R / 4) : f1 / (4 / R);
        const uint32_t a2 = R >= 4 ? f2 * (R / 4) : f2 / (4 / R);
        const char *Tb = (const char *)T;
        const char *T2 = KB ? Tb + (4u << KB) * R : Tb + H * 4 * R;
        const uint32_t *p1 = (const uint32_t *)(Tb + a1);
        const uint32_t *p2 = (const uint32_t *)(T2 + a2);
        if constexpr (ABS && R == 4 && KB > 0) {
            // the tables start the kernel's LDS (k_allpairs_q declares no
            // static LDS: T == lds == LDS address 0): address the slots
            // absolutely, without an add of the (link-time) base per read
            typedef uint32_t v4u __attribute__((ext_vector_type(4)));
            typedef __attribute__((address_space(3))) const v4u lds_v4u;
            const v4u v1 = *(lds_v4u *)(size_t)a1;
            const v4u v2 = *(lds_v4u *)(size_t)(a2 + (4u << KB) * R);
            sl.e1[0] = v1[0]; sl.e1[1] = v1[1]; sl.e1[2] = v1[2]; sl.e1[3] = v1[3];
            sl.e2[0] = v2[0]; sl.e2[1] = v2[1]; sl.e2[2] = v2[2]; sl.e2[3] = v2[3];
        } else if constexpr (R >= 4) {
#pragma unroll
            for (int r = 0; r < R; r += 4) {
                const uint4 v1 = *(const uint4 *)(p1 + r);
                const uint4 v2 = *(const uint4 *)(p2 + r);
                sl.e1[r] = v1.x; sl.e1[r + 1] = v1.y; sl.e1[r + 2] = v1.z; sl.e1[r + 3] = v1.w;
                sl.e2[r] = v2.x; sl.e2[r + 1] = v2.y; sl.e2[r + 2] = v2.z; sl.e2[r + 3] = v2.w;
            }
        } else if constexpr (R == 2) {
            const uint2 v1 = *(const uint2 *)p1, v2 = *(const uint2 *)p2;
            sl.e1[0] = v1.x; sl.e1[1] = v1.y; sl.e2[0] = v2.x; sl.e2[1] = v2.y;
        } else {
            sl.e1[0] = p1[0]; sl.e2[0] = p2[0];
        }
    } else {
#pragma unroll
        for (int r = 0; r < R; r++) {                                // inactive rows read empty words
            sl.e1[r] = T[((blo >> o1[r]) & hm) * R + r];
            sl.e2[r] = T[(H + ((blo >> o2[r]) & hm)) * R + r];
        }
    }
    return sl;
}

// One 64-element chunk of column elements (one per lane; position j) against
// R row tables, with wave-level lane masks kept in SGPRs: per row the two
// slot words are compared and their ballots OR-ed; only a row with a hit in
// the chunk (uniform branch) selects i, confirms the high word against
// V[r * vs + i] (VIL: the whole-row image's row-interleaved V[i * R + r], one
// base for every row) and applies the union-rank rule
//     i + j < s + mrun + (matches in lower lanes)
// with scalar popcounts -- counts stay in SGPRs, no per-lane reduction.
// i = ibase[r] + field, valid below ilim[r].  lanemask drops lanes (band
// kernel: outside the band).
template <int R, bool FAST, bool RETRY = true, bool VIL = false>
__device__ __forceinline__ void probe_rows(const Slots<R> &sl, uint64_t b, uint32_t j, const uint32_t *V,
                                           uint32_t vs, uint32_t hm, const uint32_t (&o1)[R],
                                           const uint32_t (&o2)[R], uint32_t actmask, uint64_t lanemask,
                                           const uint32_t (&ibase)[R], const uint32_t (&ilim)[R], uint32_t s,
                                           uint32_t (&mrun)[R], uint32_t (&cnt)[R]) {
    const uint32_t blo = (uint32_t)b, bhi = (uint32_t)(b >> 32);
    const uint32_t b4 = rotr32(blo, 4), b20 = rotr32(blo, 20);      // family 0's fields, rotated to bit 0
    uint32_t xs1[R], xs2[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        xs1[r] = sl.e1[r] ^ (FAST ? b4 : rotr32(blo, o1[r]));
        xs2[r] = sl.e2[r] ^ (FAST ? b20 : rotr32(blo, o2[r]));
    }
    {
        // one test for all rows first (a min3 chain, one compare, one ballot,
        // one branch): most chunks hit no row.  Inactive rows take part; they
        // can only send a chunk to the per-row tests, which skip them.
        // (R = 4: a v_min3 tree over the eight words, 4 VALU; the per-row
        // minima are formed only on the rare hit path)
        uint32_t mn;
        if constexpr (R == 4) {
            const uint32_t m1 = min(min(xs1[0], xs1[1]), xs1[2]);
            const uint32_t m2 = min(min(xs1[3], xs2[0]), xs2[1]);
            mn = min(min(m1, m2), min(xs2[2], xs2[3]));
        } else {
            mn = min(xs1[0], xs2[0]);
#pragma unroll
            for (int r = 1; r < R; r++) mn = min(mn, min(xs1[r], xs2[r]));
        }
        if ((__builtin_amdgcn_ballot_w64(mn <= hm) & lanemask) == 0) return;
    }
#pragma unroll
    for (int r = 0; r < R; r++) {
        if (!((actmask >> r) & 1u)) continue;                        // wave-uniform
        const uint32_t x1 = xs1[r], x2 = xs2[r];
        // one compare, one mask: a hit in either slot <=> min(x1, x2) <= hm
        uint64_t m = __builtin_amdgcn_ballot_w64(min(x1, x2) <= hm) & lanemask;
        if (m == 0) continue;                                        // wave-uniform: no hit in this row
        // the probe value of a hit is its position (row tables above): the
        // smaller of the two is the hit, an empty word's false match (hm) loses
        uint32_t f = min(x1, x2);
        // the high-word read runs on every lane (index clamped) and both tests
        // become lane masks: no exec branch, no bool-to-mask conversions.
        // f >= ilim only for the empty word's false match (f = hm)
        const uint32_t vlast = (VIL ? s : vs) - 1;                   // a valid index of the row's V
        const uint32_t fc = min(f, vlast);
        const uint32_t vhi = VIL ? V[fc * R + r] : V[r * vs + fc];
        if constexpr (!RETRY) {
            // masks straight from the compares (a ballot of a combined bool
            // costs a select and a compare to rebuild the mask)
            m &= __builtin_amdgcn_ballot_w64(vhi == bhi) & __builtin_amdgcn_ballot_w64(f < ilim[r]);
        } else {
            bool ok = vhi == bhi && f < ilim[r];
            // both slots match when two of the row's keys share this low word
            // (RETRY = false: k_build_q32 found no such pair in any row), or
            // when the first is an empty word's false match (see k_build_q32)
            const bool retry = max(x1, x2) <= hm && !ok;
            if (__builtin_amdgcn_ballot_w64(retry) != 0) {
                const uint32_t f2 = max(x1, x2);
                const uint32_t f2c = min(f2, vlast);
                const bool ok2 = retry && f2 < ilim[r] && (VIL ? V[f2c * R + r] : V[r * vs + f2c]) == bhi;
                f = ok2 ? f2 : f;
                ok = ok || ok2;
            }
            m &= __builtin_amdgcn_ballot_w64(ok);
        }
        const uint32_t lim = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                             __builtin_amdgcn_mbcnt_lo((uint32_t)m, s + mrun[r]));
        cnt[r] += (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(ibase[r] + f + j < lim) & m);
        mrun[r] += (uint32_t)__popcll(m);
    }
}

// The whole-row kernel's probe for chunks where many lanes hit (genomes of one
// species share ~20-30 % of their sketches: c ~ 180-280 of 1000, a hit in
// most rows of most chunks).  probe_rows tests each row behind a uniform
// branch -- row active, any hit -- and its high-word read waits right there,
// so a chunk's rows cost four dependent LDS round trips, ~11 scalar
// instructions and three branches each.  Here, once the all-rows test finds
// a hit: every row's position f and high word V[f] are read first (R LDS
// reads in flight together), then each row is straight-line mask arithmetic
// with no branch -- a row with no hit adds 0, an inactive row's counts are
// never written:
//   m    = ballot(V[f] == hi(b)) & ballot(f < nA)        shared hashes
//   rank = ballot(f + j - (s + mrun) < mbcnt(m))          union rank < s
//          (signed: f + j < s + mrun + shared hashes in lower lanes)
//   cnt += popc(rank & m);  mrun += popc(m)
// nb[r] = -(s + mrun) is kept instead of mrun, so the rank operand is one
// three-input add with a scalar (v_add3) and mbcnt needs no scalar base.
//
// EXACT = false (a chunk the dense verdict's chunk mask leaves clear,
// screen.hip k_cmask_*): no other 64-bit hash of the matrix shares a low word
// with this chunk's elements, so a slot holding b's low word holds b itself --
// the high-word reads and compares are skipped, m = ballot(f < nA).
template <int R, bool EXACT = true>
__device__ __forceinline__ void probe_rows_v(const Slots<R> &sl, uint64_t b, uint32_t jl, const uint32_t *V,
                                             uint32_t hm, uint32_t s, const uint32_t (&nA)[R], int32_t (&nb)[R],
                                             uint32_t (&cnt)[R]) {
    const uint32_t blo = (uint32_t)b, bhi = (uint32_t)(b >> 32);
    const uint32_t b4 = rotr32(blo, 4), b20 = rotr32(blo, 20);
    uint32_t xs1[R], xs2[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        xs1[r] = sl.e1[r] ^ b4;
        xs2[r] = sl.e2[r] ^ b20;
    }
    {
        uint32_t mn;
        if constexpr (R == 4) {
            const uint32_t m1 = min(min(xs1[0], xs1[1]), xs1[2]);
            const uint32_t m2 = min(min(xs1[3], xs2[0]), xs2[1]);
            mn = min(min(m1, m2), min(xs2[2], xs2[3]));
        } else {
            mn = min(xs1[0], xs2[0]);
#pragma unroll
            for (int r = 1; r < R; r++) mn = min(mn, min(xs1[r], xs2[r]));
        }
        if (__builtin_amdgcn_ballot_w64(mn <= hm) == 0) return;
    }
    uint32_t f[R], vh[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        // !EXACT: clamped to hm (v_min3, no extra instruction), so a lane
        // without a hit has f + j - (s + mrun) >= hm - s >= s - 1 >= 63 >= its
        // lower-lane count (mrun <= j; the masks are built for s >= 64 only):
        // the rank test below needs no AND with the match mask
        f[r] = EXACT ? min(xs1[r], xs2[r]) : min(min(xs1[r], xs2[r]), hm);
        if constexpr (EXACT) vh[r] = V[min(f[r], s - 1) * R + r];    // row-interleaved high words
    }
    if constexpr (EXACT) {
#pragma unroll
        for (int r = 0; r < R; r++) asm volatile("" : "+v"(vh[r]));  // all R reads issued before the first use
    }
#pragma unroll
    for (int r = 0; r < R; r++) {
        const uint64_t m = EXACT ? __builtin_amdgcn_ballot_w64(vh[r] == bhi) & __builtin_amdgcn_ballot_w64(f[r] < nA[r])
                                 : __builtin_amdgcn_ballot_w64(f[r] < nA[r]);
        const int32_t pre = (int32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        const int32_t key = (int32_t)(f[r] + jl) + nb[r];
        const uint64_t rank = __builtin_amdgcn_ballot_w64(key < pre);
        cnt[r] += (uint32_t)__popcll(EXACT ? rank & m : rank);
        nb[r] -= (int32_t)__popcll(m);
    }
}

// ------------------------------------------------------- whole-row tables
// The columns of one work item, processed by one wave.  The column elements
// stream through a ring of kRing chunks in registers, loaded kRing chunks
// ahead of use (the next column's first kRing chunks are loaded when a column
// starts), so a wave holds ~16 VGPRs of sketch instead of whole columns and
// two workgroups fit a CU.  Slot words are read one chunk ahead of the tests.
// Counts go straight to the condensed output (lane 0).
constexpr int kRing = 4;
// chunks between a slot read and its use: 1 (2 and 3 measured 1-2 % and 8 %
// slower -- a slot read that far ahead waits on a ring load only 2-1 chunks old)
constexpr int kSlotAhead = 1;
static_assert(kSlotAhead >= 1 && kSlotAhead < kRing, "slot prefetch distance");

// Column element loads are raw buffer loads against a per-column resource
// (base = the column's sketch, num_records = s * 8): the lane's byte offset is
// a fixed VGPR, the chunk's offset an SGPR, so a ring refill costs no VALU
// instruction, and lanes past s read 0 without a clamp (they are masked by
// the tail mask where the chunk is used).
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
constexpr int kBufferRsrcWord3 = 0x00020000;      // gfx9 raw-buffer descriptor dword 3 (CK's value for gfx9)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t column_rsrc(const uint64_t *col, uint32_t s) {
    return __builtin_amdgcn_make_buffer_rsrc((void *)col, (short)0, (int)(s * 8u), kBufferRsrcWord3);
}
__device__ __forceinline__ uint64_t ld_chunk(__amdgpu_buffer_rsrc_t rs, uint32_t lane_off, uint32_t chunk) {
    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, lane_off, rfl(chunk) * 512u, 0);
    return ((uint64_t)v[1] << 32) | v[0];
}
// the same with the chunk's byte offset split into a per-group SGPR (soff) and
// a constant (CB, the instruction's immediate offset field)
template <uint32_t CB>
__device__ __forceinline__ uint64_t ld_chunk_at(__amdgpu_buffer_rsrc_t rs, uint32_t lane_off, uint32_t soff) {
    static_assert(CB < 4096, "MUBUF immediate offset");
    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, lane_off + CB, soff, 0);
    return ((uint64_t)v[1] << 32) | v[0];
}

// MASKED = false (the common case): no per-chunk tail work at all.  Lanes and
// chunks past s read 0 through the buffer bounds, and an element 0 can only
// hit a row holding the key 0 itself (the probe needs the low word 0 in a slot
// and V == 0), so when no active row's smallest key is 0 the chunks are
// probed unmasked and unclamped: no tail mask, no chunk-in-range test, no
// refill clamp -- only the group loop and the early-end tests are scalar
// work.  MASKED = true keeps them (rows holding the key 0, the generic probe).
//
// LIST (the screened path, screen.hip): the item's columns are clist[0..cend)
// -- ascending, each sharing a hash with a row of the tile -- and c_first /
// c_step walk that list instead of the column range.
template <int R, int NCH, bool FAST, int KB, bool MASKED, bool LIST = false, bool HITQ = false, bool HITV = false,
          bool COLL = false>
__device__ __forceinline__ void ap_columns(const uint64_t *__restrict__ hashes, const uint32_t *__restrict__ nhash,
                                           const uint32_t *T, const uint32_t *V, uint32_t H, uint32_t hm, uint32_t s,
                                           uint32_t N, uint32_t i0, uint32_t nrows, uint32_t cend, uint32_t c_first,
                                           uint32_t c_step, const uint32_t *__restrict__ clist,
                                           const uint32_t (&nA)[R], const uint32_t (&o1)[R],
                                           const uint32_t (&o2)[R], const uint64_t (&alast)[R],
                                           const uint64_t (&thr1)[R], const uint64_t (&thr2)[R], uint32_t okmask,
                                           bool any_partial_row, uint16_t *__restrict__ common,
                                           uint16_t *__restrict__ denom, uint64_t seg0,
                                           const uint32_t *__restrict__ cmask = nullptr) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t lane_off = lane * 8u;
    const uint32_t nch = (s + 63) / 64;
    const uint32_t tail = s - (nch - 1) * 64;                        // valid lanes of the last chunk
    const uint64_t tailmask = tail >= 64 ? ~0ull : (1ull << tail) - 1;
    uint64_t rg[kRing], nx[kRing];
    uint32_t zero[R];
#pragma unroll
    for (int r = 0; r < R; r++) zero[r] = 0;
    uint32_t kc = rfl(c_first);                                      // wave-uniform: scalar column loop
    auto column_of = [&](uint32_t k) -> uint32_t { return LIST ? rfl(clist[k]) : k; };
    uint32_t c = kc < cend ? column_of(kc) : 0;
    // COLL: the next column's chunk mask, by a vector (buffer) load issued with
    // its first chunks -- a scalar load in flight across the chunk loop would
    // hold every LDS wait there at lgkmcnt(0)
    uint32_t cmn = ~0u;
    const __amdgpu_buffer_rsrc_t rcm =
        __builtin_amdgcn_make_buffer_rsrc((void *)cmask, (short)0, COLL ? (int)(N * 4u) : 0, kBufferRsrcWord3);
    auto next_cmask = [&](uint32_t cn) {
        if constexpr (COLL) cmn = __builtin_amdgcn_raw_buffer_load_b32(rcm, 0u, cn * 4u, 0);
    };
    auto first_chunks = [&](__amdgpu_buffer_rsrc_t rn) {
        if constexpr (MASKED) {
#pragma unroll
            for (int k = 0; k < kRing; k++) nx[k] = ld_chunk(rn, lane_off, min((uint32_t)k, nch - 1));
        } else {
            nx[0] = ld_chunk_at<0>(rn, lane_off, 0);
            nx[1] = ld_chunk_at<512>(rn, lane_off, 0);
            nx[2] = ld_chunk_at<1024>(rn, lane_off, 0);
            nx[3] = ld_chunk_at<1536>(rn, lane_off, 0);
        }
    };
    static_assert(kRing == 4, "first_chunks / refill offsets");
    if (kc < cend) {
        next_cmask(c);
        first_chunks(column_rsrc(hashes + (uint64_t)c * s, s));
    }
    // per item, not per column: the active rows and their largest hash once
    // every row of the tile is left of the column (c >= i0 + R: all columns
    // but the diagonal tile's), and row 0's output offset (row r + 1's is row
    // r's plus N - (i0 + r) - 2)
    uint32_t act_full = 0;
    uint64_t amax_full = 0;
#pragma unroll
    for (int r = 0; r < R; r++) {
        const bool act = (uint32_t)r < nrows && ((okmask >> r) & 1u);
        act_full |= (uint32_t)act << r;
        if (act) amax_full = alast[r] > amax_full ? alast[r] : amax_full;
    }
    const uint64_t obase = cond_index(i0, 0, N) - seg0;            // + c: row i0's pair (i0, c)
    for (uint32_t cnext = 0; kc < cend; kc += c_step, c = cnext) {
        const __amdgpu_buffer_rsrc_t rc = column_rsrc(hashes + (uint64_t)c * s, s);
#pragma unroll
        for (int k = 0; k < kRing; k++) rg[k] = nx[k];
        const uint32_t cmc = cmn;                                      // this column's chunk mask (COLL)
        const uint32_t kn = kc + c_step;
        cnext = kn < cend ? column_of(kn) : 0;
        if (kn < cend) {
            next_cmask(cnext);
            first_chunks(column_rsrc(hashes + (uint64_t)cnext * s, s));
        }
        const uint32_t cm = COLL ? rfl(cmc) : ~0u;                    // bit k: chunk k needs the high-word check
        uint32_t cnt[R], mrun[R], actmask = act_full;
        int32_t nb[R];                                                // HITV: -(s + matches so far), probe_rows_v
        // elements past every active row's largest hash cannot match: the
        // scan ends at the first chunk whose smallest element is past them
        uint64_t amax = amax_full;
#pragma unroll
        for (int r = 0; r < R; r++) { cnt[r] = 0; mrun[r] = 0; nb[r] = -(int32_t)s; }
        auto mrun_of = [&](int r) -> uint32_t { return HITV ? (uint32_t)(-nb[r] - (int32_t)s) : mrun[r]; };
        if (c < i0 + R) {                                             // the diagonal tile: rows right of c drop out
            actmask = 0;
            amax = 0;
#pragma unroll
            for (int r = 0; r < R; r++) {
                const bool act = ((act_full >> r) & 1u) && i0 + r < c;
                actmask |= (uint32_t)act << r;
                if (act) amax = alast[r] > amax ? alast[r] : amax;
            }
        }
        if (!actmask) continue;                                       // column at or left of the tile's rows
        // slot words of chunk k live in sb[k % kRing]: read kSlotAhead chunks
        // ahead (the LDS reads are bank-conflicted random 16-byte reads, ~3x
        // their conflict-free cycles; one chunk of work did not cover them)
        Slots<R> sb[kRing];
#pragma unroll
        for (int u = 0; u < kSlotAhead; u++)
            sb[u] = read_slots<R, FAST, KB, true>((uint32_t)rg[u], T, H, hm, o1, o2);
        // runtime loop over groups of kRing chunks; ring slots are static.  The
        // scan-end test runs once per group, on the group's first chunk (a
        // chunk past every row's largest hash cannot hit, so finishing the
        // group is only wasted work, never a wrong count), and the union-rank
        // end: b0 at column position j0 has rank u(b0) = j0 + #{A < b0} -
        // #{matches below b0} in A u B and every later column element ranks
        // higher, so once u(b0) >= s for every active row no later element is
        // among the s smallest of A_r u B -- the rank rule (probe_rows) counts
        // nothing more, and |A u B| > s makes a partial pair's denominator s
        // whatever mrun the rest would add.  Tested for rows with no match so
        // far, one chunk into the group starting at chunk kb1 (j0 = 64 (kb1 + 1),
        // just past half the column, where unrelated sketches get there) and
        // at every later group start: b0 > A_r[s - j0 - 1] (thr1, thr2:
        // scalar, loaded with the row's largest hash) gives #{A_r < b0} >=
        // s - j0, and thr2 stays a sufficient bound at every later j0.  Scalar
        // compares only (a sampled high-word read per row measured slower than
        // the chunks it skipped).  At the group start itself (j0 = 64 kb1) the
        // test ended only ~40 % of unrelated columns with 4 rows (B[512] >
        // A_r[487] holds for ~79 % of rows at s = 1000); one chunk later it ends
        // nearly all: N = 6000 2.67 -> 2.54 ms, 20000 29.1 -> 26.5 ms, same
        // registers (profiles/r03_allpairs_ab_midtest.txt).  Keeping the
        // group-start test as well (same 52 VGPRs) is 5-8 % slower
        // (profiles/r03_allpairs_ab_twotests.txt).
        const uint32_t kb1 = 4u * ((s / 2 + 255) / 256);
        auto past = [&](uint64_t bv, const uint64_t (&thr)[R]) {          // wave-uniform
            const uint64_t b0 = ((uint64_t)rfl((uint32_t)(bv >> 32)) << 32) | rfl((uint32_t)bv);
            bool all_past = true;
#pragma unroll
            for (int r = 0; r < R; r++)
                if (((actmask >> r) & 1u) && (mrun_of(r) != 0 || !(b0 > thr[r]))) all_past = false;
            return all_past;
        };
        // HITQ: the union-rank end for rows WITH shared hashes too.  b at
        // column position jb ranks u(b) = jb + #{A_r < b} - mrun_r in A_r u B
        // (mrun_r: the shared hashes before it), so u(b) >= s once A_r holds
        // s - jb + mrun_r elements below b, i.e. once b > A_r[p], p = s - jb +
        // mrun_r - 1 -- tested on the high words in LDS (V: hi(b) > V_r[p]
        // implies b > A_r[p]; an equal high word just continues the scan).  A
        // row of one species shares a few hashes with most columns, so the
        // thresholds above (rows without matches) never end its scan, which
        // then ran to A's last element: ~2x the chunks of the cutoff near
        // s (1 + J) / 2.  p >= nA (a partial row) cannot end it.
        auto past_v = [&](uint64_t bv, uint32_t jb) {                       // wave-uniform
            const uint32_t hb = rfl((uint32_t)(bv >> 32));
            uint32_t vr[R], pr[R];
#pragma unroll
            for (int r = 0; r < R; r++) {
                pr[r] = s + mrun_of(r) - jb - 1;                              // >= 0: jb < s
                vr[r] = V[min(pr[r], s - 1) * R + r];
            }
            bool all_past = true;
#pragma unroll
            for (int r = 0; r < R; r++)
                if (((actmask >> r) & 1u) && !(pr[r] < nA[r] && hb > rfl(vr[r]))) all_past = false;
            return all_past;
        };
        // one group of kRing chunks; false: the column's scan ends here.
        // EXACT: every hit confirmed by its high word (COLL: only the groups
        // from the first chunk the column's mask flags on; the groups before it
        // run the unchecked probe, with no per-chunk branch)
        auto group = [&](uint32_t kb, auto exact_tag) -> bool {
            {
                const uint64_t b = rg[0];
                // smallest element of the group (lane 0; readfirstlane returns
                // int: through uint32_t so the low word is not sign-extended)
                const uint64_t b0 = ((uint64_t)rfl((uint32_t)(b >> 32)) << 32) | rfl((uint32_t)b);
                if (b0 == kEmpty || b0 > amax) return false;
#if DREPHIP_AP_MID
                if (!HITQ && kb > kb1 && past(b, thr2)) return false;      // wave-uniform
#else
                if (kb >= kb1 && past(b, kb == kb1 ? thr1 : thr2)) return false;    // wave-uniform
#endif
            }
            const uint32_t gofs = rfl(kb) * 512u;                        // the group's byte offset (SGPR)
#pragma unroll
            for (int u = 0; u < kRing; u++) {
                const uint32_t k = kb + u;
                const uint64_t b = rg[u];
                // lanes past s in the last chunk read 0 (buffer bounds): masked
                // out (MASKED), or harmless (see above)
                const uint64_t lm = MASKED ? (k == nch - 1 ? tailmask : ~0ull) : ~0ull;
                // chunk k + kSlotAhead: in rg[(u + kSlotAhead) % kRing] (refilled
                // earlier in this group when that index is below u)
                sb[(u + kSlotAhead) % kRing] =
                    read_slots<R, FAST, KB, true>((uint32_t)rg[(u + kSlotAhead) % kRing], T, H, hm, o1, o2);
                // a chunk past the last one (the group's tail) only skips the
                // probe: the ring and slot updates above stay unconditional, or
                // the compiler merges the ring registers through a copy that
                // waits for the refill load issued in the same chunk
                if constexpr (HITV) {
                    static_assert(FAST && !MASKED, "probe_rows_v: the FAST unmasked path");
                    probe_rows_v<R, decltype(exact_tag)::value>(sb[u], b, k * 64 + lane, V, hm, s, nA, nb, cnt);
                } else if (!MASKED || k < nch) {                          // wave-uniform
                    probe_rows<R, FAST, !FAST, true>(sb[u], b, k * 64 + lane, V, s, hm, o1, o2, actmask, lm, zero, nA, s,
                                               mrun, cnt);
                }
                // refill the ring unconditionally and after the chunk's last use,
                // so the load reuses the chunk's registers: a conditional update,
                // or one while the old value is live, makes the compiler copy the
                // ring at the loop back edge behind a wait for the loads just
                // issued.  MASKED: past the end, the last chunk again; else the
                // chunk itself (zeros past s), its offset in the immediate field
                if constexpr (MASKED) {
                    rg[u] = ld_chunk(rc, lane_off, min(k + kRing, nch - 1));
                } else {
                    if (u == 0) rg[u] = ld_chunk_at<(0 + kRing) * 512>(rc, lane_off, gofs);
                    if (u == 1) rg[u] = ld_chunk_at<(1 + kRing) * 512>(rc, lane_off, gofs);
                    if (u == 2) rg[u] = ld_chunk_at<(2 + kRing) * 512>(rc, lane_off, gofs);
                    if (u == 3) rg[u] = ld_chunk_at<(3 + kRing) * 512>(rc, lane_off, gofs);
                }
#if DREPHIP_AP_MID
                // the first union-rank test one chunk into group kb1: B[64 (kb1 + 1)]
                // against A_r[s - 64 (kb1 + 1) - 1] (thr1) after chunk kb1's probe
                if constexpr (HITQ) {
                    // every group from kb1 on, one chunk in: B[64 (kb + 1)] with the
                    // matches of every chunk before it
                    // (tested twice per group, chunks 0 and 2: 2 % slower on the dense
                    // 10^4 set, equal elsewhere -- profiles/r06_allpairs_hit_ab.txt)
                    if (u == 0 && kb >= kb1 && kb + 1 < nch && past_v(rg[1], 64 * (kb + 1))) return false;
                } else {
                    if (u == 0 && kb == kb1 && kb1 + 1 < nch && past(rg[1], thr1)) return false;
                }
#endif
            }
            return true;
        };
        {
            uint32_t kb = 0;
            if constexpr (COLL) {
                const uint32_t kf = cm ? ((uint32_t)__builtin_ctz(cm) & ~(uint32_t)(kRing - 1)) : 32u;
                for (; kb < kf && kb < nch; kb += kRing)
                    if (!group(kb, std::false_type{})) goto column_done;
            }
            for (; kb < nch; kb += kRing)
                if (!group(kb, std::true_type{})) goto column_done;
        }
    column_done:
        if (lane == 0) {
            // the column's count is read only here: a scalar load left in flight
            // across the chunk loop would force every LDS wait there to lgkmcnt(0)
            const uint32_t nB = nhash[c];
            const bool partial = any_partial_row || nB < s;
            uint64_t o = obase + c;
#pragma unroll
            for (int r = 0; r < R; r++) {
                if (r > 0) o += N - (i0 + r - 1) - 2;                   // cond_index(i0 + r, c) - seg0
                if (!((actmask >> r) & 1u)) continue;
                common[o] = (uint16_t)cnt[r];
                if (denom) {
                    uint32_t dd = s;
                    if (partial) {
                        const uint32_t u = nA[r] + nB - mrun_of(r);  // |A u B|; mrun = |A n B| when partial
                        dd = u < s ? u : s;
                    }
                    denom[o] = (uint16_t)dd;
                }
            }
        }
    }
}

__host__ __device__ constexpr size_t q_lds_bytes(uint32_t R, uint32_t TS, uint32_t s) {
    return (size_t)R * TS * 4 + (size_t)R * s * 4;
}

// R rows (tables in LDS) x kApCols columns per workgroup of kApWG lanes; each
// wave walks every 16th column of the item.  MINW = 8: two workgroups per CU
// (LDS <= 80 KiB, <= 64 VGPRs).
// LIST: items are {i0, list offset, count, 0} over the screened column list
// (screen.hip); otherwise {i0, c0, cend, 0} over the column range.
template <int R, int NCH, int MINW, bool LIST = false>
__global__ __launch_bounds__(kApWG, MINW) void k_allpairs_q(
    const uint64_t *__restrict__ hashes, const uint32_t *__restrict__ nhash,
    const uint32_t *__restrict__ blk, uint32_t stride, const uint8_t *__restrict__ fam, uint32_t s, uint32_t N,
    uint32_t row0, uint32_t row1, uint32_t B, const uint4 *__restrict__ items,
    uint16_t *__restrict__ common, uint16_t *__restrict__ denom, uint64_t seg0, const uint32_t *__restrict__ clist,
    int hitq, const uint32_t *__restrict__ cmask) {
    constexpr int WG = kApWG;
    extern __shared__ __align__(16) uint32_t lds[];    // 16-B aligned: slot words are read with ds_read_b128
    const uint32_t H = 1u << B, hm = H - 1, TS = 2 * H;
    uint32_t *T = lds;                                  // [TS][R] interleaved slot words
    uint32_t *V = T + R * TS;                           // [s][R] high words by position (row-interleaved)
    const uint32_t i0 = items[blockIdx.x].x;
    const uint32_t c0 = items[blockIdx.x].y;
    if (i0 == 0xFFFFFFFFu) return;                      // idle padding item (make_items)
    const uint32_t nrows = min((uint32_t)R, row1 - i0);
    // LIST: c0 = the item's list offset, cend = its column count
    const uint32_t cend = LIST ? items[blockIdx.x].z : min(items[blockIdx.x].z, N);
    const uint32_t *ilist = LIST ? clist + c0 : nullptr;
    const uint32_t cfirst = LIST ? 0 : c0;
    const uint32_t tid = threadIdx.x, wave = tid >> 6;
    {   // the row group's LDS image (k_build_q32) by LDS-DMA: wave w copies the
        // 1 KiB pieces w, w + 16, ... (global_load_lds_dwordx4 writes a piece
        // lane-linearly); every load is in flight at once, no VGPR round trip,
        // and the per-row loads below overlap it.  Drained by the barrier.
        const uint4 *src = (const uint4 *)(blk + (uint64_t)((i0 - row0) / R) * stride);
        const uint32_t n16 = stride / 4, lane = tid & 63;
        for (uint32_t p = wave * 64; p < n16; p += WG) {
            if (p + lane < n16)
                __builtin_amdgcn_global_load_lds((const void *)(src + p + lane),
                                                 (__attribute__((address_space(3))) void *)(
                                                     (__attribute__((address_space(3))) uint4 *)lds + p),
                                                 16, 0, 0);
        }
    }
    uint32_t nA[R], o1[R], o2[R];
    uint64_t alast[R], thr1[R], thr2[R];
    uint32_t failmask = 0;
    bool any_partial_row = false, fast = true, zero_key = false;
    {   // per-row scalars: uniform loads with clamped rows, no branches, so none
        // of them waits on the image's DMA above (the family bytes as one
        // aligned 8-byte word; the fam buffer is padded to 8 bytes)
        const uint32_t fi = i0 - row0;
        const uint64_t fw = *(const uint64_t *)(fam + (fi & ~7u));
        uint32_t nraw[R];
        uint64_t lraw[R], t1raw[R], t2raw[R], fraw[R];
        // union-rank thresholds (ap_columns): A_r[s - j0 - 1] for the two test
        // groups, j0 = 64 kb1 and 64 (kb1 + 4); positions below 0 clamp to 0
        // (never used then: such a group does not exist or the test is moot)
        const uint32_t kb1 = 4u * ((s / 2 + 255) / 256);
        const uint32_t j1 = 64 * (kb1 + (DREPHIP_AP_MID ? 1 : 0));         // column position of the first test
        const uint32_t p1 = s > j1 ? s - j1 - 1 : 0, p2 = s > 64 * (kb1 + 4) ? s - 64 * (kb1 + 4) - 1 : 0;
#pragma unroll
        for (int r = 0; r < R; r++) {
            const uint32_t i = min(i0 + (uint32_t)r, row1 - 1);
            nraw[r] = nhash[i];
            lraw[r] = hashes[(uint64_t)i * s + s - 1];
            t1raw[r] = hashes[(uint64_t)i * s + p1];
            t2raw[r] = hashes[(uint64_t)i * s + p2];
            fraw[r] = hashes[(uint64_t)i * s];
        }
#pragma unroll
        for (int r = 0; r < R; r++) {
            const bool ok = (uint32_t)r < nrows;
            nA[r] = ok ? nraw[r] : s;
            uint32_t f = ok ? (uint32_t)(fw >> (((fi & 7u) + (uint32_t)r) * 8)) & 0xFFu : 0;
            failmask |= (uint32_t)(f == kFamFailed) << r;   // no field family worked: merged literally below
            f = f == kFamFailed ? 0 : f;
            fast &= f == 0;                                  // family 0 and no twins (kFamTwins)
            const QFields q = qfields(f & ~kFamTwins);
            o1[r] = q.o1; o2[r] = q.o2;
            alast[r] = (ok && nA[r] >= s) ? lraw[r] : kEmpty;
            // a threshold past the row's last element (partial row) or of a
            // group with j0 >= s never ends the scan (kEmpty: b0 > it is false)
            thr1[r] = (ok && s > j1 && p1 < nA[r]) ? t1raw[r] : kEmpty;
            thr2[r] = (ok && s > 64 * (kb1 + 4) && p2 < nA[r]) ? t2raw[r] : kEmpty;
            any_partial_row |= nA[r] < s;
            zero_key |= ok && fraw[r] == 0;                  // the row holds the hash value 0 (MASKED probe)
        }
    }
    __syncthreads();
    // NCH = 16 means 512 < s <= 1024, i.e. H = 2048 (B = 11) for every such s.
    // The kernel declares no static LDS (.group_segment_fixed_size 0, checked
    // by tests/test_host.py), so `lds` is LDS address 0 (read_slots).
    constexpr int KB = NCH == 16 ? 11 : 0;
    if (fast && !zero_key && hitq && !LIST && cmask)
        // the dense path after the screen's verdict: chunk masks (probe_rows_v)
        ap_columns<R, NCH, true, KB, false, LIST, true, true, !LIST>(hashes, nhash, T, V, H, hm, s, N, i0, nrows, cend,
                                                                    cfirst + wave, WG / 64, ilist, nA, o1, o2, alast, thr1,
                                                                    thr2, ~failmask, any_partial_row, common, denom, seg0,
                                                                    cmask);
    else if (fast && !zero_key && hitq)
        ap_columns<R, NCH, true, KB, false, LIST, true, true>(hashes, nhash, T, V, H, hm, s, N, i0, nrows, cend,
                                                        cfirst + wave, WG / 64, ilist, nA, o1, o2, alast, thr1, thr2,
                                                        ~failmask, any_partial_row, common, denom, seg0);
    else if (fast && !zero_key)
        ap_columns<R, NCH, true, KB, false, LIST>(hashes, nhash, T, V, H, hm, s, N, i0, nrows, cend, cfirst + wave, WG / 64, ilist,
                                            nA, o1, o2, alast, thr1, thr2, ~failmask, any_partial_row, common, denom,
                                            seg0);
    else if (fast)
        ap_columns<R, NCH, true, KB, true, LIST>(hashes, nhash, T, V, H, hm, s, N, i0, nrows, cend, cfirst + wave, WG / 64, ilist,
                                           nA, o1, o2, alast, thr1, thr2, ~failmask, any_partial_row, common, denom,
                                           seg0);
    else
        ap_columns<R, NCH, false, KB, true, LIST>(hashes, nhash, T, V, H, hm, s, N, i0, nrows, cend, cfirst + wave, WG / 64, ilist,
                                            nA, o1, o2, alast, thr1, thr2, ~failmask, any_partial_row, common, denom,
                                            seg0);
    if (failmask) {
        // a row whose table could not be built (three of its keys share a low
        // word under every field family; never observed on real sketches):
        // its pairs of this item by Mash's literal merge, one lane per pair
        const uint32_t ncol = cend - cfirst;
        for (uint32_t t = tid; t < (uint32_t)R * ncol; t += WG) {
            const uint32_t r = t / ncol, c = LIST ? ilist[t % ncol] : c0 + t % ncol, i = i0 + r;
            if (!((failmask >> r) & 1u) || c <= i) continue;
            uint32_t cm, dd;
            merge_pair(hashes + (uint64_t)i * s, nhash[i], hashes + (uint64_t)c * s, nhash[c], s, cm, dd);
            const uint64_t o = cond_index(i, c, N) - seg0;
            common[o] = (uint16_t)cm;
            if (denom) denom[o] = (uint16_t)dd;
        }
    }
}

// ------------------------------------------------------- literal merge
// Literal Mash merge, one lane per pair of the condensed segment.
__global__ __launch_bounds__(256) void k_allpairs_merge(const uint64_t *__restrict__ hashes,
                                                        const uint32_t *__restrict__ nhash, uint32_t s,
                                                        uint32_t N, uint64_t seg0, uint64_t npairs,
                                                        uint16_t *__restrict__ common,
                                                        uint16_t *__restrict__ denom) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= npairs) return;
    const uint64_t idx = seg0 + t;
    const double M = 2.0 * N - 1.0;
    int64_t i = (int64_t)floor((M - sqrt(fmax(M * M - 8.0 * (double)idx, 0.0))) / 2.0);
    if (i < 0) i = 0;
    while (i > 0 && cond_index(i, i + 1, N) > idx) i--;
    while (i + 1 < (int64_t)N - 1 && cond_index(i + 1, i + 2, N) <= idx) i++;
    const uint64_t j = idx - cond_index(i, i + 1, N) + i + 1;
    uint32_t c, d;
    merge_pair(hashes + (uint64_t)i * s, nhash[i], hashes + j * s, nhash[j], s, c, d);
    common[t] = (uint16_t)c;
    if (denom) denom[t] = (uint16_t)d;
}

// ------------------------------------------------------- banded all-pairs
// Large sketches (s > 2048, up to kMaxSketch = 32767): a whole-row table no longer fits
// LDS, so the hash range is cut into value bands per row tile.  Band k of a
// tile of R rows is [lo_k, hi_k) with hi_k = min over rows of A_r[p_r + cap]
// (p_r = the row's first element >= lo_k), so every row has <= cap elements in
// the band; those get an LDS cuckoo table (same quotiented format as above,
// storing the element's position *within the band*, at most cap - 1 < H - 1,
// so the empty word still decodes to "absent") and their high words V.  Every
// column of the tile keeps a cursor into its sketch (first element >= lo_k, in
// LDS); a wave streams the column's elements in [lo_k, hi_k) in 64-element
// chunks and counts, per row, shared elements whose union rank
//     i + j - m_j < s          (i = p_r + band position, j = column position)
// is below s -- the same rule as k_allpairs_q, with the running match count
// m and the partial counts carried across bands in LDS.  Bands run until
// every row is exhausted; column elements past the rows' largest element end
// the last band.  Tables are rebuilt per band by the whole workgroup (every
// key verified; up to kMaxFam field families, then the host falls back to the
// literal merge); a band's build is amortised over kBandCols columns.
// Roofline: as k_allpairs_q (LDS random reads + VALU); column chunks are read
// once per band per tile, i.e. s * 8 / R bytes per pair from L2.
//
// Geometry (template): R rows per tile, 2^BB slots per choice, CAP elements
// per row per band (launch_band: R = 4, 2^11, 768).
// Round 4: the columns a band visits come from a live list built by the band
// before it -- a column whose union-rank end has passed for every row is
// dropped once instead of being re-tested (and its first chunks re-loaded)
// in every later band.
constexpr uint32_t kBandCols = 128;

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t w = __shfl_xor(v, o, 64);
        v = w < v ? w : v;
    }
    return v;
}
// 64 column elements from position `first` (wave-uniform) on, one per lane,
// through the column's buffer resource: lanes past s read 0 (buffer bounds)
// and are dropped by tail_mask where the chunk is used.  Elements past nB are
// kEmpty in the sketch matrix and fail every band test (b < hi <= the rows'
// largest element + 1).
__device__ __forceinline__ uint64_t ld_elems(__amdgpu_buffer_rsrc_t rs, uint32_t lane_off, uint32_t first) {
    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, lane_off, rfl(first) * 8u, 0);
    return ((uint64_t)v[1] << 32) | v[0];
}
__device__ __forceinline__ uint64_t tail_mask(uint32_t j0, uint32_t s) {     // lanes with j0 + lane < s
    return j0 + 64 <= s ? ~0ull : j0 >= s ? 0ull : (1ull << (s - j0)) - 1;
}

// The column phase of one band: wave w takes the live columns w, w+NW, ... of
// the band's list (live[0..nlive)).  A column's band segment streams through a
// ring of kRing chunks in registers, loaded kRing chunks ahead (the next
// column's first kRing chunks when a column starts) by raw buffer loads; slot
// words are read one chunk ahead of the tests.  After the band a column goes
// on the next band's list (next, *nnext) unless its union-rank end has passed
// for every row with the next band's row positions pn.
template <int R, uint32_t NW, int BB, int CAP, bool FAST, bool RETRY, bool LIST>
__device__ __forceinline__ void band_columns(const uint64_t *__restrict__ hashes, uint32_t s, const uint32_t *T,
                                             const uint32_t *V, uint32_t *cur, uint16_t *pcnt, uint16_t *pm,
                                             const uint8_t *live, uint32_t nlive, uint8_t *next, uint32_t *nnext,
                                             uint32_t c0, const uint32_t *__restrict__ cl, uint32_t i0, uint32_t nrows,
                                             uint32_t wave, uint64_t hi, uint32_t fam, const uint32_t (&pr)[R],
                                             const uint32_t (&pn)[R]) {
    // column of item column ci: c0 + ci, or (LIST) the screened list's entry
    auto col = [&](uint32_t ci) -> uint32_t { return LIST ? rfl(cl[ci]) : c0 + ci; };
    constexpr uint32_t H = 1u << BB, hm = H - 1;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t lane_off = lane * 8u;
    uint32_t li = wave;
    uint64_t nx[kRing];
    uint32_t nq = 0;
    auto load_first = [&](uint32_t cc) {
        nq = rfl(cur[cc]);
        const __amdgpu_buffer_rsrc_t rn = column_rsrc(hashes + (uint64_t)col(cc) * s, s);
#pragma unroll
        for (int k = 0; k < kRing; k++) nx[k] = ld_elems(rn, lane_off, nq + 64 * k);
    };
    uint32_t cnx = li < nlive ? rfl(live[li]) : 0;
    if (li < nlive) load_first(cnx);
    uint32_t o1[R], o2[R], cap_r[R];
    const QFields qf = qfields(fam);
#pragma unroll
    for (int r = 0; r < R; r++) { o1[r] = qf.o1; o2[r] = qf.o2; cap_r[r] = CAP; }
    for (; li < nlive; li += NW) {
        const uint32_t ci = cnx;
        const uint32_t c = col(ci);
        const uint32_t q0 = nq;
        uint64_t rg[kRing];
#pragma unroll
        for (int k = 0; k < kRing; k++) rg[k] = nx[k];
        if (li + NW < nlive) { cnx = rfl(live[li + NW]); load_first(cnx); }
        uint32_t actmask = 0;
#pragma unroll
        for (int r = 0; r < R; r++) actmask |= (uint32_t)((uint32_t)r < nrows && i0 + r < c) << r;
        uint32_t mrun[R], cnt[R];
#pragma unroll
        for (int r = 0; r < R; r++) { mrun[r] = rfl(pm[r * kBandCols + ci]); cnt[r] = 0; }   // scalar counters
        const __amdgpu_buffer_rsrc_t rc = column_rsrc(hashes + (uint64_t)c * s, s);
        uint32_t q = q0;
        bool more = true;
        // as ap_columns: ring refill and slot reads unconditional, the refill
        // after the chunk's last use; a finished column only skips the probe
        Slots<R> sb[kRing];
#pragma unroll
        for (int u = 0; u < kSlotAhead; u++) sb[u] = read_slots<R, FAST, BB>((uint32_t)rg[u], T, H, hm, o1, o2);
        for (uint32_t kb = 0; more; kb += kRing) {
#pragma unroll
            for (int u = 0; u < kRing; u++) {
                const uint64_t b = rg[u];
                const uint32_t j0 = q0 + 64 * (kb + u);
                sb[(u + kSlotAhead) % kRing] =
                    read_slots<R, FAST, BB>((uint32_t)rg[(u + kSlotAhead) % kRing], T, H, hm, o1, o2);
                if (more) {                                           // wave-uniform
                    const uint64_t inb = __builtin_amdgcn_ballot_w64(b < hi) & tail_mask(j0, s);
                    probe_rows<R, FAST, RETRY>(sb[u], b, q + lane, V, CAP, hm, o1, o2, actmask, inb, pr, cap_r,
                                               s, mrun, cnt);
                    const uint32_t nin = (uint32_t)__popcll(inb);
                    q += nin;
                    more = nin == 64;
                }
                rg[u] = ld_elems(rc, lane_off, j0 + 64 * kRing);    // refill the ring
            }
        }
        // union-rank end for the next band: the column's next element b
        // (position q, at or above the next band's low bound, below which A_r
        // has pn[r] elements) has rank u(b) = q + #{A_r < b} - #{matches below
        // b} >= q + pn[r] - mrun in A_r u B, and every later column element
        // ranks higher.  Once that is >= s for every active row, the rank rule
        // counts nothing more in any later band (cursor, counts and
        // shared-so-far stay; |A u B| > s then makes a partial pair's
        // denominator s whatever mrun misses).  Mash's merge stops at the s-th
        // union element the same way; unrelated sketches get there about half
        // way down the column.
        bool all_past = true;
#pragma unroll
        for (int r = 0; r < R; r++)
            if (((actmask >> r) & 1u) && q + pn[r] < s + mrun[r]) all_past = false;
        if (lane == 0) {
#pragma unroll
            for (int r = 0; r < R; r++) { pcnt[r * kBandCols + ci] += cnt[r]; pm[r * kBandCols + ci] = mrun[r]; }
            cur[ci] = q;
            if (!all_past) next[atomicAdd(nnext, 1u)] = (uint8_t)ci;
        }
    }
}

template <int R, int BB, int CAP>
__host__ __device__ constexpr size_t band_lds_bytes() {
    // slot words, high words, cursors, counts + shared-so-far, two live lists
    return (size_t)R * (2u << BB) * 4 + (size_t)R * CAP * 4 + kBandCols * 4 + 2ull * R * kBandCols * 2 +
           2ull * kBandCols;
}
static_assert(kBandCols <= 256, "live lists hold column indices in bytes");
static_assert(band_lds_bytes<4, 11, 768>() <= 80 * 1024 - 128, "R = 4: two workgroups per CU");

// Value rounds (round 5).  Each launch of the ROUNDS kernel takes every item
// of a chunk through one global value range [ends[k-1], ends[k]): its bands
// stop at ends[k], and the item's per-column state (cursors, counts,
// shared-so-far, live lists) and row positions go to global memory until the
// next launch.  The items running together on one XCD -- the row tiles of one
// family, placed there by the screen -- then read the same short segment of
// each family column (s / rounds elements) within one launch, so the column
// stream is fetched from HBM about once per family and re-read from that
// XCD's L2, instead of once per (row tile, column) cell: without rounds the
// tiles of a family drift apart by whole bands, and an L2 line lives a few
// microseconds under the stream (profiles/r04_allpairs_N10000_s10000.json: L2
// hit 0.17, HBM 48x the algorithmic bytes).  Bands and counts are the same
// arithmetic as one launch; only the band cuts fall at the round ends too.
// State blob: the LDS words from cur to the end of the lists, then a header.
template <int R>
__host__ __device__ constexpr uint32_t band_blob_words() {
    return (kBandCols * 4 + 2 * R * kBandCols * 2 + 2 * kBandCols) / 4;
}
template <int R>
__host__ __device__ constexpr uint32_t band_state_words() {     // blob + header, in 64-B lines
    return (band_blob_words<R>() + R + 8 + 15) / 16 * 16;
}
enum : uint32_t { kBsDone = 1u };

// LIST (the screened path, screen.hip): items are {i0, list offset, count, 0}
// (litems) over the column list clist; otherwise {i0, c0} over kBandCols
// consecutive columns.  ROUNDS: one value round per launch (above); bstate
// holds this launch's items' states, ends the rounds' upper bounds.
template <int R, int BB, int CAP, int WG, int MINW, bool LIST = false, bool ROUNDS = false>
__global__ __launch_bounds__(WG, MINW) void k_allpairs_band(
    const uint64_t *__restrict__ hashes, const uint32_t *__restrict__ nhash, uint32_t s, uint32_t N,
    uint32_t row1, uint32_t cap, const uint2 *__restrict__ items, uint16_t *__restrict__ common,
    uint16_t *__restrict__ denom, uint64_t seg0, uint32_t *__restrict__ nfail, uint64_t *__restrict__ prof,
    const uint4 *__restrict__ litems, const uint32_t *__restrict__ clist, uint32_t *__restrict__ bstate,
    const uint64_t *__restrict__ ends, uint32_t round) {
    constexpr uint32_t H = 1u << BB, hm = H - 1, TS = 2 * H;
    constexpr uint32_t NW = WG / 64;
    static_assert(CAP < H, "band positions stay below the empty word's position hm");
    extern __shared__ __align__(16) uint32_t lds[];    // 16-B aligned: slot words are read with ds_read_b128
    uint32_t *T = lds;                                               // [TS][R] interleaved slot words
    uint32_t *V = T + R * TS;                                        // [R][CAP] high words
    uint32_t *cur = V + R * CAP;                                     // [kBandCols] column cursors
    uint16_t *pcnt = (uint16_t *)(cur + kBandCols);                  // [R][kBandCols] counts (<= s)
    uint16_t *pm = pcnt + R * kBandCols;                             // [R][kBandCols] shared so far (<= s)
    uint8_t *lists = (uint8_t *)(pm + R * kBandCols);                // [2][kBandCols] live columns per band
    __shared__ uint32_t s_p[R], s_q[R], s_nlive[2];
    __shared__ uint64_t s_hi, s_lo;
    __shared__ int s_done, s_fail, s_abort, s_twin;

    const uint32_t i0 = LIST ? litems[blockIdx.x].x : items[blockIdx.x].x;
    const uint32_t c0 = LIST ? 0 : items[blockIdx.x].y;
    if (i0 == 0xFFFFFFFFu) return;                      // idle padding item (make_items)
    constexpr uint32_t BW = band_blob_words<R>();
    uint32_t *gst = ROUNDS ? bstate + (size_t)blockIdx.x * band_state_words<R>() : nullptr;
    const uint64_t rend = ROUNDS ? ends[round] : kEmpty;
    if (ROUNDS && round > 0 && (gst[BW + R + 3] & kBsDone)) return;          // finished in an earlier round
    const uint32_t nrows = min((uint32_t)R, row1 - i0);
    const uint32_t *cl = LIST ? clist + litems[blockIdx.x].y : nullptr;
    const uint32_t ncols = LIST ? litems[blockIdx.x].z : min(c0 + kBandCols, N) - c0;
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t wave = rfl(tid >> 6);          // wave-uniform for the compiler: scalar column loop

    uint32_t nA[R];
    bool any_partial_row = false;
#pragma unroll
    for (int r = 0; r < R; r++) {
        nA[r] = (uint32_t)r < nrows ? nhash[i0 + r] : 0;
        any_partial_row |= (uint32_t)r < nrows && nA[r] < s;
    }
    // largest element over the tile's rows: column elements past it cannot match
    uint64_t maxlast = 0;
#pragma unroll
    for (int r = 0; r < R; r++)
        if (nA[r]) { const uint64_t v = hashes[(uint64_t)(i0 + r) * s + nA[r] - 1]; maxlast = v > maxlast ? v : maxlast; }
    uint32_t band0 = 0;
    if (ROUNDS && round > 0) {
        // the state the previous round left (the blob is the LDS image from cur on)
        for (uint32_t k = tid; k < BW; k += WG) cur[k] = gst[k];
        if (tid < (uint32_t)R) s_p[tid] = gst[BW + tid];
        if (tid == 0) {
            s_nlive[0] = gst[BW + R];
            s_nlive[1] = gst[BW + R + 1];
            s_lo = (uint64_t)gst[BW + R + 4] | ((uint64_t)gst[BW + R + 5] << 32);
            s_abort = 0;
        }
        band0 = gst[BW + R + 2];
    } else {
        for (uint32_t k = tid; k < kBandCols; k += WG) cur[k] = 0;
        for (uint32_t k = tid; k < R * kBandCols; k += WG) { pcnt[k] = 0; pm[k] = 0; }
        if (tid < (uint32_t)R) s_p[tid] = 0;
        if (tid == 0) { s_abort = 0; s_nlive[0] = 0; s_nlive[1] = 0; s_lo = 0; }
        __syncthreads();
        // the first band's list: every column right of the tile's first row
        // (columns left of every row have no pair in the item)
        for (uint32_t k = tid; k < ncols; k += WG)
            if (i0 < (LIST ? cl[k] : c0 + k)) lists[atomicAdd(&s_nlive[0], 1u)] = (uint8_t)k;
    }

    for (uint32_t band = band0;; band++) {
        const uint32_t lb = band & 1u;                   // this band's list; the next band's is lb ^ 1
        __syncthreads();
        if (ROUNDS && rend != kEmpty && s_lo >= rend) {
            // this round's values are done: park the state for the next launch
            for (uint32_t k = tid; k < BW; k += WG) gst[k] = cur[k];
            if (tid < (uint32_t)R) gst[BW + tid] = s_p[tid];
            if (tid == 0) {
                gst[BW + R] = s_nlive[0];
                gst[BW + R + 1] = s_nlive[1];
                gst[BW + R + 2] = band;
                gst[BW + R + 3] = 0;
                gst[BW + R + 4] = (uint32_t)s_lo;
                gst[BW + R + 5] = (uint32_t)(s_lo >> 32);
            }
            return;
        }
        if (wave == 0) {
            // band bound: the (cap+1)-th remaining element of the tightest row
            uint64_t v = kEmpty;
            bool left = false;
            if (lane < (uint32_t)R && lane < nrows) {
                uint32_t nl = 0;
#pragma unroll
                for (int r = 0; r < R; r++) if ((uint32_t)r == lane) nl = nA[r];
                const uint32_t p = s_p[lane];
                left = p < nl;
                if (p + cap < nl) v = hashes[(uint64_t)(i0 + lane) * s + p + cap];
            }
            v = wave_min_u64(v);
            const bool any_left = __ballot(left) != 0;
            if (lane == 0) {
                v = v < maxlast + 1 ? v : maxlast + 1;
                s_hi = v < rend ? v : rend;                  // (a round's end cuts the band too)
                s_done = !any_left || s_nlive[lb] == 0;
                s_fail = 0;
                s_nlive[lb ^ 1u] = 0;
            }
            if (lane < (uint32_t)R) s_q[lane] = 0;
        }
        __syncthreads();
        if (s_done) break;
        const uint64_t hi = s_hi;
        uint32_t pr[R];
#pragma unroll
        for (int r = 0; r < R; r++) pr[r] = s_p[r];

        uint64_t t_b0 = prof ? wall_clock64() : 0;
        // ---- build the R band tables (quotiented cuckoo, band positions) and V
        uint32_t fam = 0;
        for (; fam < kMaxFam; fam++) {
            const QFields qf = qfields(fam);
            for (uint32_t k = tid; k < R * TS; k += WG) T[k] = empty_word(k / R, hm);
            if (tid == 0) { s_fail = 0; s_twin = 0; }
            __syncthreads();
            for (uint32_t idx = tid; idx < R * cap; idx += WG) {
                const uint32_t r = idx / cap, t = idx - r * cap;
                uint32_t p = 0, nl = 0;
#pragma unroll
                for (int rr = 0; rr < R; rr++) if ((uint32_t)rr == r) { p = pr[rr]; nl = nA[rr]; }
                if (p + t >= nl) continue;
                const uint64_t x = hashes[(uint64_t)(i0 + r) * s + p + t];
                if (x >= hi) continue;
                if (fam == 0) V[r * CAP + t] = (uint32_t)(x >> 32);
                if (!cuckoo_insert32(T, R, r, H, hm, qf, (uint32_t)x, t)) s_fail = 1;
            }
            __syncthreads();
            // verify every key of the band; count the band's elements per row
            for (uint32_t idx = tid; idx < R * cap; idx += WG) {
                const uint32_t r = idx / cap, t = idx - r * cap;
                uint32_t p = 0, nl = 0;
#pragma unroll
                for (int rr = 0; rr < R; rr++) if ((uint32_t)rr == r) { p = pr[rr]; nl = nA[rr]; }
                if (p + t >= nl) continue;
                const uint64_t x = hashes[(uint64_t)(i0 + r) * s + p + t];
                if (x >= hi) continue;
                if (!cuckoo_has32(T, R, r, H, hm, qf, (uint32_t)x, t)) s_fail = 1;
                if (cuckoo_twin32(T, R, r, H, hm, qf, (uint32_t)x)) s_twin = 1;
                if (fam == 0) atomicAdd(&s_q[r], 1u);
            }
            __syncthreads();
            if (!s_fail) break;
        }
        if (fam == kMaxFam) {                       // no field family worked: host reruns with the merge kernel
            if (tid == 0) { s_abort = 1; atomicAdd(nfail, 1u); }
            break;
        }
        // the next band's row positions (s_q is final after the build)
        uint32_t pn[R];
#pragma unroll
        for (int r = 0; r < R; r++) pn[r] = pr[r] + s_q[r];

        uint64_t t_c0 = prof ? wall_clock64() : 0;
        // ---- columns: wave w takes the live columns w, w+NW, ...
        // the fast probe without the second-slot retry unless a band table has twins
        const uint8_t *live = lists + lb * kBandCols;
        uint8_t *next = lists + (lb ^ 1u) * kBandCols;
        const uint32_t nlive = s_nlive[lb];
        if (fam == 0 && !s_twin)
            band_columns<R, NW, BB, CAP, true, false, LIST>(hashes, s, T, V, cur, pcnt, pm, live, nlive, next, &s_nlive[lb ^ 1u],
                                                      c0, cl, i0, nrows, wave, hi, fam, pr, pn);
        else if (fam == 0)
            band_columns<R, NW, BB, CAP, true, true, LIST>(hashes, s, T, V, cur, pcnt, pm, live, nlive, next, &s_nlive[lb ^ 1u],
                                                     c0, cl, i0, nrows, wave, hi, fam, pr, pn);
        else
            band_columns<R, NW, BB, CAP, false, true, LIST>(hashes, s, T, V, cur, pcnt, pm, live, nlive, next, &s_nlive[lb ^ 1u],
                                                      c0, cl, i0, nrows, wave, hi, fam, pr, pn);
        __syncthreads();
        if (tid < (uint32_t)R) s_p[tid] += s_q[tid];
        if (tid == 0) s_lo = hi;
        if (prof && tid == 0) {
            const uint64_t t_e = wall_clock64();
            atomicAdd((unsigned long long *)&prof[0], (unsigned long long)(t_c0 - t_b0));
            atomicAdd((unsigned long long *)&prof[1], (unsigned long long)(t_e - t_c0));
            atomicAdd((unsigned long long *)&prof[2], 1ull);
        }
    }
    __syncthreads();
    if (ROUNDS && tid == 0) gst[BW + R + 3] = kBsDone;     // later rounds skip the item
    if (s_abort) return;
    if (LIST) {
        // the screened columns: one pair per (row, list entry) right of the row
        for (uint32_t t = tid; t < nrows * ncols; t += WG) {
            const uint32_t r = t / ncols, ci = t - r * ncols, i = i0 + r, c = cl[ci];
            if (c <= i) continue;
            uint32_t nl = 0;
#pragma unroll
            for (int rr = 0; rr < R; rr++) if ((uint32_t)rr == r) nl = nA[rr];
            const uint64_t o = cond_index(i, c, N) - seg0;
            common[o] = (uint16_t)pcnt[r * kBandCols + ci];
            if (denom) {
                const uint32_t nB = nhash[c];
                uint32_t dd = s;
                if (any_partial_row || nB < s) {
                    const uint32_t u = nl + nB - pm[r * kBandCols + ci];
                    dd = u < s ? u : s;
                }
                denom[o] = (uint16_t)dd;
            }
        }
        return;
    }
    const uint32_t cend = c0 + ncols;
    for (uint32_t r = 0; r < nrows; r++) {
        const uint32_t i = i0 + r;
        const uint32_t cs = max(c0, i + 1);
        if (cs >= cend) continue;
        uint32_t nl = 0;
#pragma unroll
        for (int rr = 0; rr < R; rr++) if ((uint32_t)rr == r) nl = nA[rr];
        const uint64_t base = cond_index(i, cs, N) - seg0;
        for (uint32_t t = tid; t < cend - cs; t += WG) {
            const uint32_t ci = cs - c0 + t;
            common[base + t] = (uint16_t)pcnt[r * kBandCols + ci];
            if (denom) {
                const uint32_t nB = nhash[cs + t];
                uint32_t dd = s;
                if (any_partial_row || nB < s) {
                    const uint32_t u = nl + nB - pm[r * kBandCols + ci];
                    dd = u < s ? u : s;
                }
                denom[base + t] = (uint16_t)dd;
            }
        }
    }
}

// ------------------------------------------------------------- host driver
// Work items (row tile i0, column tile c0) of the upper triangle in an
// XCD-aware order.  Column tiles are aligned (c0 = ct * C) so every row tile
// shares them; tiles are dealt to the 8 XCDs (largest first, least-loaded
// XCD) and the per-XCD lists are interleaved so that workgroup b -- which the
// dispatcher places on XCD b % 8 -- comes from XCD (b % 8)'s list: the
// workgroups running on one XCD then stream the same ~C column sketches,
// which stay in that XCD's L2 (the mapping is a speed hint only; any
// placement gives the same result).  Lists are padded with idle items
// (i0 = kIdleItem).
//
// The items of column tile ct are the row tiles i0 = row0, row0 + R, ... up to
// (ct + 1) C - 2: an arithmetic run.  The host therefore plans only groups --
// runs of one tile's items, {first i0, c0, offset in its XCD's list, count} --
// and k_expand_items writes the item array on the device (at N = 10^5 the
// list holds ~10^7 items: built item by item on the host and copied, it cost
// ~0.1 s per call shape).
constexpr uint32_t kXcds = 8;
constexpr uint32_t kIdleItem = 0xFFFFFFFFu;

using ItemGroup = ApItemGroup;
struct XcdStarts { uint32_t v[kXcds + 1]; };      // list x = groups [v[x], v[x + 1]), ascending off
struct ItemPlan {
    std::vector<ItemGroup> groups;
    XcdStarts xs{};
    uint64_t slots = 0;                          // kXcds x the longest list
};

static ItemPlan plan_items(uint32_t row0, uint32_t row1, uint32_t N, uint32_t R, uint32_t C) {
    const uint32_t nct = (N + C - 1) / C;
    auto count = [&](uint32_t ct) -> uint64_t {   // row tiles i0 in [row0, row1) with (i0 + 1) / C <= ct
        const uint64_t lim = std::min<uint64_t>(row1 - 1, (uint64_t)(ct + 1) * C - 2);
        return (uint64_t)row0 + 1 > (uint64_t)(ct + 1) * C - 1 ? 0 : (lim - row0) / R + 1;
    };
    uint64_t total = 0;
    for (uint32_t ct = 0; ct < nct; ct++) total += count(ct);
    // groups of at most ~1/16 of an XCD's share, so that dealing them
    // largest-first balances the XCDs
    const uint64_t gmax = std::max<uint64_t>(1, total / (kXcds * 16));
    struct G { uint32_t ct; uint64_t first, size; };
    std::vector<G> gs;
    for (uint32_t ct = 0; ct < nct; ct++) {
        const uint64_t n = count(ct);
        for (uint64_t i = 0; i < n; i += gmax) gs.push_back({ct, i, std::min(gmax, n - i)});
    }
    std::stable_sort(gs.begin(), gs.end(), [](const G &a, const G &b) { return a.size > b.size; });
    std::vector<std::vector<ItemGroup>> lists(kXcds);
    uint64_t len[kXcds] = {};
    for (const G &g : gs) {
        uint32_t best = 0;
        for (uint32_t x = 1; x < kXcds; x++) if (len[x] < len[best]) best = x;
        lists[best].push_back({(uint32_t)(row0 + g.first * R), g.ct * C, (uint32_t)len[best], (uint32_t)g.size});
        len[best] += g.size;
    }
    ItemPlan p;
    uint64_t lmax = 0;
    for (uint32_t x = 0; x < kXcds; x++) {
        p.xs.v[x] = (uint32_t)p.groups.size();
        p.groups.insert(p.groups.end(), lists[x].begin(), lists[x].end());
        lmax = std::max(lmax, len[x]);
    }
    p.xs.v[kXcds] = (uint32_t)p.groups.size();
    p.slots = lmax * kXcds;
    return p;
}

// slot t = the (t / 8)-th item of XCD (t % 8)'s list, or idle past its end;
// whole-row-table items are {i0, c0, c0 + C, 0}, band items {i0, c0}
template <bool WIDE>
__global__ __launch_bounds__(256) void k_expand_items(const ItemGroup *__restrict__ g, XcdStarts xs, uint64_t slots,
                                                     uint32_t R, uint32_t C, void *__restrict__ out) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= slots) return;
    const uint32_t x = (uint32_t)(t % kXcds), i = (uint32_t)(t / kXcds);
    uint32_t lo = xs.v[x], hi = xs.v[x + 1];
    uint32_t i0 = kIdleItem, c0 = 0;
    if (lo < hi) {                                   // the last group with off <= i (the first has off 0)
        while (hi - lo > 1) {
            const uint32_t m = (lo + hi) / 2;
            if (g[m].off <= i) lo = m; else hi = m;
        }
        const ItemGroup G = g[lo];
        if (i - G.off < G.size) { i0 = G.i0 + (i - G.off) * R; c0 = G.c0; }
    }
    if (WIDE) ((uint4 *)out)[t] = make_uint4(i0, c0, c0 + C, 0);
    else ((uint2 *)out)[t] = make_uint2(i0, c0);
}

// Upload a plan's groups (host copy kept in *host until the next plan: the
// copy is queued) and expand them into the item array *d_items (grow-only
// scratch `name`).  Returns the item count in *nitems.
template <bool WIDE>
static int expand_items(drephip_ctx *ctx, ItemPlan &&plan, std::vector<ItemGroup> &host, const char *name,
                        uint32_t R, uint32_t C, hipStream_t st, void **d_items, uint64_t *nitems) {
    int rc;
    *nitems = plan.slots;
    host = std::move(plan.groups);
    if (plan.slots == 0) return DREPHIP_OK;
    const std::string gname = std::string(name) + "_groups";
    ItemGroup *d_groups;
    if ((rc = scratch(ctx, gname.c_str(), host.size() * sizeof(ItemGroup), (void **)&d_groups))) return rc;
    if ((rc = scratch(ctx, name, plan.slots * (WIDE ? sizeof(uint4) : sizeof(uint2)), d_items))) return rc;
    HIPC(hipMemcpyAsync(d_groups, host.data(), host.size() * sizeof(ItemGroup), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_expand_items<WIDE>, dim3((uint32_t)((plan.slots + 255) / 256)), dim3(256), 0, st, d_groups,
                       plan.xs, plan.slots, R, C, *d_items);
    HIPC(hipGetLastError());
    return DREPHIP_OK;
}

static int launch_merge(drephip_ctx *ctx, const uint64_t *d_hashes, const uint32_t *d_nhash, uint32_t N,
                        uint64_t seg0, uint64_t npairs, uint16_t *d_common, uint16_t *d_denom,
                        hipStream_t st) {
    const uint64_t per = max_blocks(256) * 256;      // pairs per dispatch
    timing_mark(ctx, 2, st, true);
    for (uint64_t p0 = 0; p0 < npairs; p0 += per) {
        const uint64_t np = std::min(per, npairs - p0);
        hipLaunchKernelGGL(k_allpairs_merge, dim3((uint32_t)((np + 255) / 256)), dim3(256), 0, st, d_hashes, d_nhash,
                           ctx->s, N, seg0 + p0, np, d_common + p0, d_denom ? d_denom + p0 : nullptr);
    }
    timing_mark(ctx, 2, st, false);
    HIPC(hipGetLastError());
    HIPC(hipStreamSynchronize(st));
    return DREPHIP_OK;
}

// The value rounds' upper bounds: block k < nr - 1 takes, over up to 1024
// genomes spread evenly over the set, the element at quantile (k + 1) / nr of
// each sketch and writes their median; the last round ends at kEmpty (no
// bound).  Medians of per-sketch quantiles rise with k, so the rounds tile the
// value line in order.  Any bounds give the same counts; these only aim each
// round at ~s / nr elements per row.
__global__ __launch_bounds__(1024) void k_band_ends(const uint64_t *__restrict__ hashes,
                                                    const uint32_t *__restrict__ nhash, uint32_t s, uint32_t N,
                                                    uint32_t nr, uint64_t *__restrict__ ends) {
    __shared__ uint64_t v[1024];
    const uint32_t k = blockIdx.x, t = threadIdx.x;
    if (k == nr - 1) {
        if (t == 0) ends[k] = kEmpty;
        return;
    }
    const uint32_t m = min(N, 1024u);
    uint64_t x = kEmpty;
    if (t < m) {
        const uint32_t g = (uint32_t)((uint64_t)t * N / m);
        const uint32_t nh = min(nhash[g], s);
        const uint32_t idx = (uint32_t)((uint64_t)(k + 1) * nh / nr);
        if (idx < nh) x = hashes[(uint64_t)g * s + idx];
    }
    v[t] = x;
    for (uint32_t kk = 2; kk <= 1024; kk <<= 1)          // bitonic sort, ascending
        for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
            __syncthreads();
            const uint32_t p = t ^ j;
            if (p > t) {
                const uint64_t a = v[t], b = v[p];
                if ((a > b) == ((t & kk) == 0)) { v[t] = b; v[p] = a; }
            }
        }
    __syncthreads();
    if (t == 0) ends[k] = v[m / 2];
}

// Items per round chunk: every round of a chunk runs before the next chunk
// starts, so the state buffer stays bounded (kBandChunk x ~3 KB) at any N.
constexpr uint64_t kBandChunk = 16384;
static_assert(kBandChunk % 8 == 0, "chunks keep the XCD-interleaved item order");

// One band-kernel geometry: R rows per tile, 2^BB slots per choice, CAP
// elements per row per band, MINW = 8 (two workgroups per CU) or 4 (one).
// scr: the screened lists (LIST kernel over them, every other pair filled as
// no-shared-hash), or null for the dense item plan.  Value rounds: ~`per`
// elements per row per round (ctx->band_round, DREPHIP_BAND_ROUND; 0 = one
// launch per item as before round 5).
template <int R, int BB, int CAP, int MINW>
static int launch_band_cfg(drephip_ctx *ctx, const uint64_t *d_hashes, const uint32_t *d_nhash, uint32_t N,
                           uint32_t row0, uint32_t row1, uint64_t seg0, uint64_t npairs, uint16_t *d_common,
                           uint16_t *d_denom, hipStream_t st, const ScreenResult *scr) {
    const uint32_t cap = std::min(std::max(ctx->band_cap, 1u), (uint32_t)CAP);
    uint32_t per = ctx->band_round;
    if (const char *e = getenv("DREPHIP_BAND_ROUND")) per = (uint32_t)atoi(e);
    const uint32_t nr = per ? (ctx->s + per - 1) / per : 1;
    uint2 *d_items = nullptr;
    uint64_t nitems;
    uint32_t *d_nfail;
    int rc;
    std::vector<ItemGroup> groups;                   // lives until the stream sync below
    if (scr) {
        nitems = scr->nitems;
    } else if ((rc = expand_items<false>(ctx, plan_items(row0, row1, N, R, kBandCols), groups, "apb_items", R,
                                         kBandCols, st, (void **)&d_items, &nitems))) {
        return rc;
    }
    if (nitems == 0) {                              // (screened: the screen wrote the whole segment)
        if (scr) HIPC(hipStreamSynchronize(st));
        return DREPHIP_OK;
    }
    if ((rc = scratch(ctx, "ap_nfail_band", 4, (void **)&d_nfail))) return rc;
    HIPC(hipMemsetAsync(d_nfail, 0, 4, st));
    uint64_t *d_prof = nullptr;                      // DREPHIP_BAND_PROF=1: per-phase wall-clock sums
    const bool prof = getenv("DREPHIP_BAND_PROF") != nullptr;
    if (prof) {
        if ((rc = scratch(ctx, "apb_prof", 64, (void **)&d_prof))) return rc;
        HIPC(hipMemsetAsync(d_prof, 0, 64, st));
    }
    constexpr size_t lds = band_lds_bytes<R, BB, CAP>();
    const bool rounds = nr > 1;
    auto kern = scr ? (rounds ? k_allpairs_band<R, BB, CAP, 1024, MINW, true, true>
                              : k_allpairs_band<R, BB, CAP, 1024, MINW, true, false>)
                    : (rounds ? k_allpairs_band<R, BB, CAP, 1024, MINW, false, true>
                              : k_allpairs_band<R, BB, CAP, 1024, MINW, false, false>);
    HIPC(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    uint32_t *d_state = nullptr;
    uint64_t *d_ends = nullptr;
    if (rounds) {
        if ((rc = scratch(ctx, "apb_state", std::min(nitems, kBandChunk) * band_state_words<R>() * 4ull,
                          (void **)&d_state)))
            return rc;
        if ((rc = scratch(ctx, "apb_ends", nr * 8ull, (void **)&d_ends))) return rc;
    }
    timing_mark(ctx, 2, st, true);
    if (rounds)
        hipLaunchKernelGGL(k_band_ends, dim3(nr), dim3(1024), 0, st, d_hashes, d_nhash, ctx->s, N, nr, d_ends);
    uint64_t chunk = rounds ? kBandChunk : nitems;
    if (const char *e = getenv("DREPHIP_BAND_CHUNK"))          // tests only: several chunks at small sizes
        if (rounds && atoll(e) > 0) chunk = std::min<uint64_t>(kBandChunk, std::max<uint64_t>(8, atoll(e) / 8 * 8));
    for (uint64_t b0 = 0; b0 < nitems; b0 += chunk) {
        const uint64_t b1 = std::min(nitems, b0 + chunk);
        for (uint32_t k = 0; k < nr; k++)
            for (uint64_t i0 = b0; i0 < b1; i0 += max_blocks(1024))
                hipLaunchKernelGGL(kern, dim3((uint32_t)std::min<uint64_t>(b1 - i0, max_blocks(1024))), dim3(1024), lds,
                                   st, d_hashes, d_nhash, ctx->s, N, row1, cap, scr ? nullptr : d_items + i0, d_common,
                                   d_denom, seg0, d_nfail, d_prof, scr ? scr->items + i0 : nullptr,
                                   scr ? scr->clist : nullptr, rounds ? d_state + (i0 - b0) * band_state_words<R>() : nullptr,
                                   d_ends, k);
    }
    timing_mark(ctx, 2, st, false);
    HIPC(hipGetLastError());
    uint32_t nfail = 0;
    HIPC(hipMemcpyAsync(&nfail, d_nfail, 4, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    if (prof) {
        uint64_t h[3];
        HIPC(hipMemcpy(h, d_prof, 24, hipMemcpyDeviceToHost));
        fprintf(stderr, "[drephip] band kernel R=%d 2^%d slots cap %u: %llu bands over %zu items; per band: build %.2f us, columns %.2f us (100 MHz wall clock)\n",
                R, BB, cap, (unsigned long long)h[2], (size_t)nitems, h[2] ? h[0] / 100.0 / h[2] : 0.0,
                h[2] ? h[1] / 100.0 / h[2] : 0.0);
    }
    if (nfail)   // a band table could not be built with any field pair: exact merge kernel instead
        return launch_merge(ctx, d_hashes, d_nhash, N, seg0, npairs, d_common, d_denom, st);
    return DREPHIP_OK;
}

// Band geometry: R = 4 rows, 2^11 slots per choice, cap 768, two workgroups
// per CU.  Round 4 measured R = 8 (configs[4], N = 10^4, s = 10^4, whole
// triangle exact): 113 ms with 2^11 slots / cap 768 / one workgroup per CU and
// 147 ms with 2^10 slots / cap 352 / two per CU, against 84 ms here
// (profiles/r04_band_geometry_ab.json): the band bound is the tightest of R
// rows, so more rows mean narrower bands, more table builds and more
// per-column band overhead, which outweighs the halved column stream.  Two
// workgroups per CU cap the kernel at 64 VGPRs (15 spilled, 64 B/lane of
// scratch); one per CU (82 VGPRs, no spills) measured slower: 19.2 vs 16.1 ms
// screened at configs[4], 5.1 vs 4.3 ms dense at N = 2000, s = 10^4.  R = 8 in
// the screened (LIST) mode, where the kernel streams column sketches at
// ~5 TB/s: 21.8 vs 16.0 ms at configs[4], 11.4 vs 8.9 ms at N = 6000 -- the
// union of eight rows' marked columns outgrows the halved stream.
constexpr uint32_t kBandR = 4;
static int launch_band(drephip_ctx *ctx, const uint64_t *d_hashes, const uint32_t *d_nhash, uint32_t N,
                       uint32_t row0, uint32_t row1, uint64_t seg0, uint64_t npairs, uint16_t *d_common,
                       uint16_t *d_denom, hipStream_t st, const ScreenResult *scr) {
    return launch_band_cfg<kBandR, 11, 768, 8>(ctx, d_hashes, d_nhash, N, row0, row1, seg0, npairs, d_common, d_denom,
                                               st, scr);
}

// LIST: the screened items / column list (clist)
template <int R, int NCH, int MINW, bool LIST>
static int launch_q(drephip_ctx *ctx, uint32_t nitems, size_t lds, hipStream_t st, const uint64_t *h,
                    const uint32_t *nh, const uint32_t *blk, uint32_t stride, const uint8_t *fam, uint32_t N, uint32_t row0,
                    uint32_t row1, uint32_t B, const uint4 *items, uint16_t *cm, uint16_t *dn,
                    uint64_t seg0, const uint32_t *clist, const uint32_t *cmask) {
    HIPC(hipFuncSetAttribute((const void *)k_allpairs_q<R, NCH, MINW, LIST>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)lds));
    // the branch-free hit probe and the union-rank end for rows with matches
    // (probe_rows_v, ap_columns HITQ/HITV); DREPHIP_AP_HIT=0 runs the round-5
    // probe and ends (A/B)
    const char *he = getenv("DREPHIP_AP_HIT");
    const int hitq = he ? atoi(he) : 1;
    timing_mark(ctx, 2, st, true);
    for (uint32_t i0 = 0; i0 < nitems; i0 += (uint32_t)max_blocks(kApWG))
        hipLaunchKernelGGL((k_allpairs_q<R, NCH, MINW, LIST>),
                           dim3(std::min<uint32_t>(nitems - i0, (uint32_t)max_blocks(kApWG))), dim3(kApWG), lds, st, h,
                           nh, blk, stride, fam, ctx->s, N, row0, row1, B, items + i0, cm, dn, seg0, clist, hitq,
                           LIST ? nullptr : cmask);
    timing_mark(ctx, 2, st, false);
    HIPC(hipGetLastError());
    return DREPHIP_OK;
}

// the screen mode (DREPHIP_SCREEN_*; DREPHIP_AP_SCREEN overrides) and whether
// it screens an all-pairs call over N genomes
int screen_mode(drephip_ctx *ctx) {
    int smode = ctx->screen;
    if (const char *e = getenv("DREPHIP_AP_SCREEN")) smode = atoi(e);
    return smode;
}
bool screen_applies(drephip_ctx *ctx, uint32_t N) {
    const int smode = screen_mode(ctx);
    const char *mn = getenv("DREPHIP_SCREEN_MIN_N");
    const uint32_t min_n = mn ? (uint32_t)atoi(mn) : kScreenMinN;
    return (smode == DREPHIP_SCREEN_ON || (smode == DREPHIP_SCREEN_AUTO && N >= min_n)) &&
           (uint64_t)N * ctx->s < (1ull << 32) && ctx->ap_path != DREPHIP_AP_MERGE;
}

// Rows per work item / row tile and the kernel path for this context's s:
// whole-row LDS tables (B-bit fields, 2H slots, H = 2^B >= 2s) when they fit,
// else value bands.  The sharded screen's parts tile rows by the same R.
int allpairs_geometry(drephip_ctx *ctx, uint32_t *R_out, int *path_out) {
    const uint32_t s = ctx->s;
    // table: 2H slots, H = 2^B >= 2s (load <= 1/4, and every position and the
    // empty word's 2^B - 1 fit the field); 32-bit families need B <= 12
    uint32_t B = 4;
    while ((1u << B) < 2 * s) B++;
    const uint32_t TS = 2u << B;
    const bool fits = B <= 12 && q_lds_bytes(1, TS, s) <= kLdsBudget;
    int path = ctx->ap_path;
    if (path == DREPHIP_AP_AUTO) path = fits ? DREPHIP_AP_TABLE : DREPHIP_AP_BAND;
    if (path == DREPHIP_AP_TABLE && !fits) {
        set_error("whole-row table all-pairs kernel needs s <= 2048");
        return DREPHIP_ERR_UNSUPPORTED;
    }
    // rows per workgroup: the most (8, 4, 2, 1) whose tables + high words fit
    static const uint32_t kR[] = {8, 4, 2, 1};
    uint32_t R = 1;
    for (uint32_t r : kR) if (q_lds_bytes(r, TS, s) + 16 <= kLdsBudget) { R = r; break; }
    if (const char *e = getenv("DREPHIP_AP_R")) {
        // A/B override: R rows per workgroup if their tables fit the whole
        // 160 KiB of a CU (one workgroup per CU above 80 KiB)
        const uint32_t r = (uint32_t)atoi(e);
        if ((r == 1 || r == 2 || r == 4 || r == 8) && q_lds_bytes(r, TS, s) <= 160 * 1024) R = r;
    }
    if (path == DREPHIP_AP_BAND) R = kBandR;
    *R_out = R;
    *path_out = path;
    return DREPHIP_OK;
}

int allpairs_device_impl(drephip_ctx *ctx, const uint64_t *d_hashes, const uint32_t *d_nhash, uint32_t N,
                         uint32_t row0, uint32_t row1, uint16_t *d_common, uint16_t *d_denom,
                         hipStream_t st, bool force_merge, bool defer) {
    // an earlier deferred call completes first (its queued item-list copy
    // reads host memory this call may replace)
    if (ctx->apend.active) {
        int rc = allpairs_wait_impl(ctx);
        if (rc) return rc;
    }
    if (row1 > N) row1 = N;
    if (N < 2 || row0 >= row1 || row0 >= N - 1) return DREPHIP_OK;
    if (row1 > N - 1) row1 = N - 1;
    const uint32_t s = ctx->s;
    const uint64_t seg0 = cond_index(row0, row0 + 1, N);
    const uint64_t seg1 = row1 < N - 1 ? cond_index(row1, row1 + 1, N) : (uint64_t)N * (N - 1) / 2;
    const uint64_t npairs = seg1 - seg0;
    uint32_t R = 1;
    int path = DREPHIP_AP_MERGE;
    const int rc0 = allpairs_geometry(ctx, &R, &path);
    if (force_merge) path = DREPHIP_AP_MERGE;         // (the literal merge needs no table)
    else if (rc0) return rc0;
    uint32_t B = 4;
    while ((1u << B) < 2 * s) B++;
    const uint32_t TS = 2u << B;
    ctx->last_screen = ScreenResult{};
    if (path == DREPHIP_AP_MERGE)
        return launch_merge(ctx, d_hashes, d_nhash, N, seg0, npairs, d_common, d_denom, st);

    // the shared-hash screen (screen.hip): auto from kScreenMinN genomes on
    const int smode = screen_mode(ctx);
    const char *mn = getenv("DREPHIP_SCREEN_MIN_N");
    const uint32_t min_n = mn ? (uint32_t)atoi(mn) : kScreenMinN;
    ScreenResult scr;
    if (ctx->ext.active) {
        // the sharded screen: this call's rows from the parts' marks
        // (drephip_allpairs_device_marked); no light cells
        int rc = screen_marked_impl(ctx, d_nhash, N, row0, row1, R, path == DREPHIP_AP_BAND ? kBandCols : kListCols,
                                    seg0, npairs, d_common, d_denom, ctx->ext.cells, ctx->ext.ncells, ctx->ext.rec,
                                    ctx->ext.nrec, st, &scr);
        if (rc) return rc;
        ctx->last_screen = scr;
    } else if (smode == DREPHIP_SCREEN_ON || (smode == DREPHIP_SCREEN_AUTO && N >= min_n)) {
        // LIST items: the band kernel's per-column LDS state holds kBandCols
        // columns; the whole-row kernel takes up to kListCols per item, so a
        // row tile's image is loaded once for most tiles
        int rc = screen_impl(ctx, d_hashes, d_nhash, N, row0, row1, R, path == DREPHIP_AP_BAND ? kBandCols : kListCols,
                             seg0, npairs, d_common, d_denom, smode == DREPHIP_SCREEN_ON, path == DREPHIP_AP_BAND, st,
                             &scr);
        if (rc) return rc;
        ctx->last_screen = scr;
    }
    if (path == DREPHIP_AP_BAND)
        return launch_band(ctx, d_hashes, d_nhash, N, row0, row1, seg0, npairs, d_common, d_denom, st,
                           scr.use ? &scr : nullptr);

    // row-group LDS images (tables + high words), built once per call
    const uint32_t nrows = row1 - row0;
    const uint32_t ngroups = (nrows + R - 1) / R;
    const uint32_t stride = (uint32_t)((q_lds_bytes(R, TS, s) / 4 + 3) & ~3ull);   // words, 16-B multiple
    uint32_t *d_blk;
    uint8_t *d_fam;
    uint4 *d_items;
    int rc;
    if ((rc = scratch(ctx, "ap_blk", (uint64_t)ngroups * stride * 4, (void **)&d_blk))) return rc;
    if ((rc = scratch(ctx, "ap_fam", ((uint64_t)ngroups * R + 7) & ~7ull, (void **)&d_fam))) return rc;
    const size_t blds = (size_t)TS * 4;
    HIPC(hipFuncSetAttribute((const void *)k_build_q32, hipFuncAttributeMaxDynamicSharedMemorySize, (int)blds));
    timing_mark(ctx, 3, st, true);
    hipLaunchKernelGGL(k_build_q32, dim3(ngroups * R), dim3(1024), blds, st, d_hashes, d_nhash, s, row0, row1, B, R,
                       d_blk, stride, d_fam);
    timing_mark(ctx, 3, st, false);
    HIPC(hipGetLastError());
    // column tile: the widest (<= kApCols) whose item count still gives every
    // workgroup slot of the chip (256 CUs x 2) about four items; small
    // problems (a rank's shard on 8 GPUs, N ~ 10^3) get narrower items.  (Items
    // of equal pair count cut from each row group's whole column range -- one
    // row image per workgroup slot -- measured 5-25 % slower at N = 1000.)
    uint32_t C = kApCols;
    auto nitems_for = [&](uint32_t c) {
        uint64_t n = 0;
        const uint32_t nct = (N + c - 1) / c;
        for (uint32_t i0 = row0; i0 < row1; i0 += R) n += nct - (i0 + 1) / c;
        return n;
    };
    if (!scr.use) while (C > kApMinCols && nitems_for(C) < 4ull * kApSlots) C /= 2;
    // the item list depends only on (N, rows, R, C): reused while the shape and
    // the scratch allocation are unchanged (repeated calls: bench steps, shards).
    // Its group table lives in the context until the next plan replaces it (the
    // queued H2D copy may still be reading it when a deferred call returns).
    const uint64_t key[5] = {N, row0, row1, R, C};
    if (scr.use) {
        // the screened items (the screen has written every other pair)
        d_items = (uint4 *)scr.items;
    } else if (ctx->ap_items_gen == ctx->alloc_gen && !memcmp(ctx->ap_items_key, key, sizeof(key))) {
        if ((rc = scratch(ctx, "ap_items", ctx->ap_items_n * sizeof(uint4), (void **)&d_items))) return rc;
    } else {
        uint64_t n;
        ctx->ap_items_gen = 0;
        if ((rc = expand_items<true>(ctx, plan_items(row0, row1, N, R, C), ctx->ap_groups_host, "ap_items", R, C, st,
                                     (void **)&d_items, &n)))
            return rc;
        ctx->ap_items_n = n;
        memcpy(ctx->ap_items_key, key, sizeof(key));
        ctx->ap_items_gen = ctx->alloc_gen;
    }
    const uint32_t ni = scr.use ? scr.nitems : (uint32_t)ctx->ap_items_n;
    const bool lst = scr.use;
    // a row whose table cannot be built is merged literally inside the main
    // kernel (k_allpairs_q): no host round trip, nothing to check afterwards
    const size_t lds = (size_t)stride * 4;
    const uint32_t nch = (s + 63) / 64;
    // two workgroups per CU when the LDS allows
    const bool two = lds <= 80 * 1024;
#define DREPHIP_Q1(RR, NC, MW, LS) launch_q<RR, NC, MW, LS>(ctx, ni, lds, st, d_hashes, d_nhash, d_blk, stride, d_fam, N, row0, row1, B, \
                                                          d_items, d_common, d_denom, seg0, scr.clist, scr.use ? nullptr : scr.cmask)
#define DREPHIP_Q(RR, NC) (two ? (lst ? DREPHIP_Q1(RR, NC, 8, true) : DREPHIP_Q1(RR, NC, 8, false)) \
                               : (lst ? DREPHIP_Q1(RR, NC, 4, true) : DREPHIP_Q1(RR, NC, 4, false)))
    if (nch <= 8) {
        switch (R) {
            case 8: rc = DREPHIP_Q(8, 8); break;
            case 4: rc = DREPHIP_Q(4, 8); break;
            case 2: rc = DREPHIP_Q(2, 8); break;
            default: rc = DREPHIP_Q(1, 8); break;
        }
    } else if (nch <= 16) {
        switch (R) {
            case 8: rc = DREPHIP_Q(8, 16); break;
            case 4: rc = DREPHIP_Q(4, 16); break;
            case 2: rc = DREPHIP_Q(2, 16); break;
            default: rc = DREPHIP_Q(1, 16); break;
        }
    } else {
        switch (R) {
            case 4: rc = DREPHIP_Q(4, 32); break;
            case 2: rc = DREPHIP_Q(2, 32); break;
            default: rc = DREPHIP_Q(1, 32); break;
        }
    }
#undef DREPHIP_Q
#undef DREPHIP_Q1
    if (rc) return rc;
    if (defer) {
        // drephip_allpairs_wait (or the next all-pairs call) waits for this event
        auto &p = ctx->apend;
        if (!p.ev) HIPC(hipEventCreateWithFlags(&p.ev, hipEventDisableTiming));
        HIPC(hipEventRecord(p.ev, st));
        p.active = true;
        return DREPHIP_OK;
    }
    HIPC(hipStreamSynchronize(st));
    return DREPHIP_OK;
}

// Completes a deferred table-path call (drephip_allpairs_device_async): waits
// for its kernels.  Nothing is recomputed here -- the kernels themselves
// handle every row, including rows whose table could not be built.
int allpairs_wait_impl(drephip_ctx *ctx) {
    auto &p = ctx->apend;
    if (!p.active) return DREPHIP_OK;
    p.active = false;
    HIPC(hipEventSynchronize(p.ev));
    return DREPHIP_OK;
}

}  // namespace drephip
