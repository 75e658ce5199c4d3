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
// come from a quotiented two-choice cuckoo table of A (2H slots, H >= 2s, load
// <= 1/4; the slot position implies B key bits, which the stored word reuses
// for i) built once per row (k_build_qcuckoo); m_j is the running match count
// plus a ballot/popcount prefix within the chunk.  Elements past A's largest
// hash (A full) cannot match, which ends the scan.  A membership test is two
// independent ds_read_b64 and two 64-bit compares: no probe loop, no
// divergence.  R row tables live in LDS per workgroup; results are staged in
// LDS and written as contiguous runs of the condensed triangle.
// Roofline: LDS random-read throughput + VALU (integer compare/select); no
// MFMA (set intersection is not a dense contraction).
//
// k_allpairs_merge is the literal Mash merge, one lane per pair: any s, used
// for s > 2048 and as an in-library cross-check.

#include "ctx.h"
#include "../../include/drephip.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace drephip {

constexpr int kApWG = 1024;                     // 16 waves: 4 per SIMD at 1 workgroup/CU
// 32 chunks (s > 1024) double-buffered take 128 VGPRs of sketch alone: half the
// waves, twice the registers
__host__ __device__ constexpr int ap_wg(int nch) { return nch > 16 ? kApWG / 2 : kApWG; }
constexpr uint32_t kApCols = 128;               // columns per work item
constexpr uint32_t kMaxFam = 6;                 // cuckoo hash families tried per row
constexpr uint32_t kLdsTables = 128 * 1024;     // LDS bytes for row tables per workgroup

__host__ __device__ __forceinline__ uint64_t cond_index(uint64_t i, uint64_t j, uint64_t N) {
    return i * N - i * (i + 1) / 2 + (j - i - 1);
}


// ------------------------------------------------------- row tables
// Quotiented two-choice cuckoo table: choice 1 sits at T[f1(x)], choice 2 at
// T[H + f2(x)], where f1/f2 are disjoint B-bit fields of the key at offsets
// o1/o2 (family f picks them).  Because a slot's position fixes those B bits,
// the stored word replaces them with the key's sketch position i, and is kept
// rotated right by the field offset:  e = rotr((x & ~F) | (i << o), o), so the
// field sits at bits [0, B); one 8-byte read returns membership AND i:
// match iff (e ^ rotr(x, o)) < 2^B, i = e & (2^B - 1) (the all-ones empty
// word decodes to i = 2^B-1 >= nA).  Exact for every key.
struct QFields { uint32_t o1, o2; };
__host__ __device__ __forceinline__ uint64_t rotr64(uint64_t x, uint32_t r) {
    return r ? (x >> r) | (x << (64 - r)) : x;
}
__host__ __device__ __forceinline__ QFields qfields(uint32_t fam) {
    // disjoint field offsets inside the low 36 key bits (bottom-s hashes of
    // any genome below ~2^28 bases have uniformly random low 36 bits).
    // Family 0 keeps both fields in the low 32 bits (kernel fast path).
    const uint32_t o1[6] = {0, 16, 3, 19, 6, 22};
    const uint32_t o2[6] = {16, 0, 19, 3, 22, 6};
    return {o1[fam], o2[fam]};
}

__global__ __launch_bounds__(256) void k_build_qcuckoo(const uint64_t *__restrict__ hashes,
                                                       const uint32_t *__restrict__ nhash, uint32_t s,
                                                       uint32_t row0, uint32_t B,
                                                       uint64_t *__restrict__ tabs,
                                                       uint8_t *__restrict__ fam_out,
                                                       uint32_t *__restrict__ nfail) {
    extern __shared__ unsigned long long T[];
    __shared__ int fail;
    const uint32_t H = 1u << B, hm = H - 1;
    const uint32_t r = blockIdx.x;
    const uint32_t g = row0 + r;
    const uint32_t n = nhash[g];
    const uint64_t *A = hashes + (uint64_t)g * s;
    for (uint32_t fam = 0; fam < kMaxFam; fam++) {
        const QFields q = qfields(fam);
        const uint64_t F1 = (uint64_t)hm << q.o1, F2 = (uint64_t)hm << q.o2;
        for (uint32_t i = threadIdx.x; i < 2 * H; i += blockDim.x) T[i] = kEmpty;
        if (threadIdx.x == 0) fail = 0;
        __syncthreads();
        // insert (key, position) pairs; an entry travels as (x, i)
        for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
            uint64_t x = A[i];
            uint32_t ix = i;
            uint32_t pos = (uint32_t)(x >> q.o1) & hm;
            bool placed = false;
            for (int kick = 0; kick < 96; kick++) {
                const bool second = pos >= H;
                const uint64_t e = second ? ((x & ~F2) | ((uint64_t)ix << q.o2))
                                          : ((x & ~F1) | ((uint64_t)ix << q.o1));
                // stored rotated right by the field offset: field at bits [0, B)
                const unsigned long long oldr = atomicExch(&T[pos], rotr64(e, second ? q.o2 : q.o1));
                if (oldr == kEmpty) { placed = true; break; }
                // decode the evicted entry back to (key, position)
                const uint64_t old = rotr64(oldr, 64 - (second ? q.o2 : q.o1));
                const uint32_t lp = second ? pos - H : pos;
                if (second) { ix = (uint32_t)(old >> q.o2) & hm; x = (old & ~F2) | ((uint64_t)lp << q.o2); }
                else        { ix = (uint32_t)(old >> q.o1) & hm; x = (old & ~F1) | ((uint64_t)lp << q.o1); }
                pos = second ? ((uint32_t)(x >> q.o1) & hm) : (H + ((uint32_t)(x >> q.o2) & hm));
            }
            if (!placed) fail = 1;
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
            const uint64_t x = A[i];
            const uint64_t e1 = rotr64(T[(uint32_t)(x >> q.o1) & hm], 64 - q.o1);
            const uint64_t e2 = rotr64(T[H + ((uint32_t)(x >> q.o2) & hm)], 64 - q.o2);
            const bool ok1 = (e1 & ~F1) == (x & ~F1) && ((uint32_t)(e1 >> q.o1) & hm) == i;
            const bool ok2 = (e2 & ~F2) == (x & ~F2) && ((uint32_t)(e2 >> q.o2) & hm) == i;
            if (!(ok1 || ok2)) fail = 1;
        }
        __syncthreads();
        if (!fail) {
            uint64_t *o = tabs + (uint64_t)r * 2 * H;
            for (uint32_t i = threadIdx.x; i < 2 * H; i += blockDim.x) o[i] = T[i];
            if (threadIdx.x == 0) fam_out[r] = (uint8_t)fam;
            return;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) { fam_out[r] = 0xFF; atomicAdd(nfail, 1u); }
}

// Slot words are stored rotated right by their field offset (field at bits
// [0, B)), so slot k holds b iff (e_k ^ rotr(b, o_k)) <= 2^B - 1, and the
// field -- b's sketch position i in A -- is e_k & hm.  The empty word (all
// ones) matches only the all-ones padding key and decodes to 2^B - 1, past
// every real position, so the ilim test below keeps `found` exact.
// One 64-element chunk of column elements (one per lane; position j) against
// R row tables, with wave-level lane masks kept in SGPRs: per row the two
// slot words are compared and their ballots OR-ed; only a row with a match in
// the chunk (uniform branch) selects i, checks it against ilim (the empty
// word decodes past it) and applies the union-rank rule
//     i + j < s + mrun + (matches in lower lanes)
// with scalar popcounts -- counts stay in SGPRs, no per-lane reduction.
// i = ibase[r] + field.  lanemask drops lanes (band kernel: outside the band).
// Row tables are interleaved in LDS (slot k of row r at k*R + r), so in the
// FAST layout (family 0 for every row) one slot address serves all R rows:
// R/2 ds_read_b128 per choice.
template <int R, bool FAST>
__device__ __forceinline__ void probe_chunk(uint64_t b, uint32_t j, const uint64_t *T, uint32_t H, uint32_t hm,
                                            const uint32_t (&o1)[R], const uint32_t (&o2)[R], uint32_t actmask,
                                            uint64_t lanemask, const uint32_t (&ibase)[R],
                                            const uint32_t (&ilim)[R], uint32_t s, uint32_t (&mrun)[R],
                                            uint32_t (&cnt)[R]) {
    const uint32_t blo = (uint32_t)b;
    uint64_t e1[R], e2[R];
    if (FAST) {
        const uint64_t *p1 = T + (uint64_t)(blo & hm) * R;
        const uint64_t *p2 = T + (uint64_t)(H + ((blo >> 16) & hm)) * R;
        if constexpr (R == 1) {
            e1[0] = p1[0]; e2[0] = p2[0];
        } else {
#pragma unroll
            for (int r = 0; r < R; r += 2) {
                const ulonglong2 v1 = *(const ulonglong2 *)(p1 + r);
                const ulonglong2 v2 = *(const ulonglong2 *)(p2 + r);
                e1[r] = v1.x; e1[r + 1] = v1.y; e2[r] = v2.x; e2[r + 1] = v2.y;
            }
        }
    } else {
#pragma unroll
        for (int r = 0; r < R; r++) {                                // inactive rows read empty words
            e1[r] = T[(uint64_t)((uint32_t)(b >> o1[r]) & hm) * R + r];
            e2[r] = T[(uint64_t)(H + ((uint32_t)(b >> o2[r]) & hm)) * R + r];
        }
    }
    const uint64_t b16 = rotr64(b, 16);                              // family 0's second field
#pragma unroll
    for (int r = 0; r < R; r++) {
        if (!((actmask >> r) & 1u)) continue;                        // wave-uniform
        const bool c1 = (e1[r] ^ (FAST ? b : rotr64(b, o1[r]))) <= (uint64_t)hm;
        const bool c2 = (e2[r] ^ (FAST ? b16 : rotr64(b, o2[r]))) <= (uint64_t)hm;
        uint64_t m = (__builtin_amdgcn_ballot_w64(c1) | __builtin_amdgcn_ballot_w64(c2)) & lanemask;
        if (m == 0) continue;                                        // wave-uniform: no shared hash here
        const uint32_t f = (c1 ? (uint32_t)e1[r] : (uint32_t)e2[r]) & hm;
        m &= __builtin_amdgcn_ballot_w64(f < ilim[r]);
        const uint32_t lim = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                             __builtin_amdgcn_mbcnt_lo((uint32_t)m, s + mrun[r]));
        cnt[r] += (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(ibase[r] + f + j < lim) & m);
        mrun[r] += (uint32_t)__popcll(m);
    }
}

// The columns of one work item, processed by one wave (double-buffered column
// sketches in registers; see the header comment for the counting rule).
template <int R, int NCH, bool FAST>
__device__ __forceinline__ void ap_columns(const uint64_t *__restrict__ hashes, const uint32_t *__restrict__ nhash,
                                           const uint64_t *T, uint32_t TS, uint32_t H, uint32_t hm, uint32_t s,
                                           uint32_t i0, uint32_t nrows, uint32_t c0, uint32_t cend, uint32_t c_first,
                                           uint32_t c_step, const uint32_t (&nA)[R], const uint32_t (&o1)[R],
                                           const uint32_t (&o2)[R], const uint64_t (&alast)[R],
                                           bool any_partial_row, uint16_t *res_c, uint16_t *res_d) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nch = (s + 63) / 64;
    uint64_t cur[NCH], nxt[NCH];
    uint32_t c = __builtin_amdgcn_readfirstlane(c_first);        // wave-uniform: scalar column loop
    if (c < cend) {
        const uint64_t *Bc = hashes + (uint64_t)c * s;
#pragma unroll
        for (int k = 0; k < NCH; k++) { const uint32_t j = k * 64 + lane; nxt[k] = (k < (int)nch && j < s) ? Bc[j] : kEmpty; }
    }
    for (; c < cend; c += c_step) {
#pragma unroll
        for (int k = 0; k < NCH; k++) cur[k] = nxt[k];
        const uint32_t cn = c + c_step;
        if (cn < cend) {
            const uint64_t *Bn = hashes + (uint64_t)cn * s;
#pragma unroll
            for (int k = 0; k < NCH; k++) { const uint32_t j = k * 64 + lane; nxt[k] = (k < (int)nch && j < s) ? Bn[j] : kEmpty; }
        }
        const uint32_t nB = nhash[c];
        const bool partial = any_partial_row || nB < s;
        uint32_t cnt[R], mrun[R], actmask = 0;
        // elements past every active row's largest hash cannot match: the
        // scan ends at the first chunk whose smallest element is past them
        uint64_t amax = 0;
#pragma unroll
        for (int r = 0; r < R; r++) {
            cnt[r] = 0; mrun[r] = 0;
            const bool act = (uint32_t)r < nrows && i0 + r < c;
            actmask |= (uint32_t)act << r;
            if (act) amax = alast[r] > amax ? alast[r] : amax;
        }
        uint32_t zero[R];
#pragma unroll
        for (int r = 0; r < R; r++) zero[r] = 0;
        bool alive = true;
#pragma unroll
        for (int k = 0; k < NCH; k++) {
            if (!alive || k >= (int)nch) continue;                        // wave-uniform
            const uint64_t b = cur[k];
            // smallest element of the chunk (lane 0; readfirstlane returns
            // int: through uint32_t so the low word is not sign-extended)
            const uint64_t b0 = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
                                (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
            if (b0 == kEmpty || b0 > amax) { alive = false; continue; }
            probe_chunk<R, FAST>(b, k * 64 + lane, T, H, hm, o1, o2, actmask, ~0ull, zero, nA, s, mrun, cnt);
        }
#pragma unroll
        for (int r = 0; r < R; r++) {
            if ((uint32_t)r >= nrows || i0 + r >= c) continue;
            const uint32_t cc = cnt[r];
            uint32_t dd = s;
            if (partial) {
                const uint32_t u = nA[r] + nB - mrun[r];      // |A u B|; mrun = |A n B| when partial
                dd = u < s ? u : s;
            }
            if (lane == 0) { res_c[r * kApCols + (c - c0)] = (uint16_t)cc; res_d[r * kApCols + (c - c0)] = (uint16_t)dd; }
        }
    }
}

// R rows (tables in LDS) x kApCols columns per workgroup of ap_wg(NCH) lanes; each
// wave walks every (WG/64)-th column of the item.
template <int R, int NCH>
__global__ __launch_bounds__(ap_wg(NCH)) void k_allpairs_q(
    const uint64_t *__restrict__ hashes, const uint32_t *__restrict__ nhash,
    const uint64_t *__restrict__ tabs, const uint8_t *__restrict__ fam, uint32_t s, uint32_t N,
    uint32_t row0, uint32_t row1, uint32_t B, const uint2 *__restrict__ items,
    uint16_t *__restrict__ common, uint16_t *__restrict__ denom, uint64_t seg0) {
    constexpr int WG = ap_wg(NCH);
    extern __shared__ __align__(16) uint64_t lds[];    // 16-B aligned: the tables are read with ds_read_b128
    const uint32_t H = 1u << B, hm = H - 1, TS = 2 * H;
    uint64_t *T = lds;
    uint16_t *res_c = (uint16_t *)(lds + (uint64_t)R * TS);
    uint16_t *res_d = res_c + R * kApCols;
    const uint32_t i0 = items[blockIdx.x].x;
    const uint32_t c0 = items[blockIdx.x].y;
    const uint32_t nrows = min((uint32_t)R, row1 - i0);
    const uint32_t cend = min(c0 + kApCols, N);
    const uint32_t tid = threadIdx.x, wave = tid >> 6;
    // interleave the R row tables: slot k of row r at k*R + r (rows past nrows empty)
    for (uint32_t k = tid; k < TS; k += WG) {
#pragma unroll
        for (int r = 0; r < R; r++)
            T[(uint64_t)k * R + r] = (uint32_t)r < nrows ? tabs[(uint64_t)(i0 - row0 + r) * TS + k] : kEmpty;
    }
    uint32_t nA[R], o1[R], o2[R];
    uint64_t alast[R];
    bool any_partial_row = false, fast = true;
#pragma unroll
    for (int r = 0; r < R; r++) {
        const bool ok = (uint32_t)r < nrows;
        nA[r] = ok ? nhash[i0 + r] : s;
        const uint32_t f = ok ? fam[i0 - row0 + r] : 0;
        const QFields q = qfields(f);
        o1[r] = q.o1; o2[r] = q.o2;
        fast &= f == 0;
        alast[r] = (ok && nA[r] >= s) ? hashes[(uint64_t)(i0 + r) * s + s - 1] : kEmpty;
        any_partial_row |= nA[r] < s;
    }
    __syncthreads();
    if (fast)
        ap_columns<R, NCH, true>(hashes, nhash, T, TS, H, hm, s, i0, nrows, c0, cend, c0 + wave, WG / 64,
                                 nA, o1, o2, alast, any_partial_row, res_c, res_d);
    else
        ap_columns<R, NCH, false>(hashes, nhash, T, TS, H, hm, s, i0, nrows, c0, cend, c0 + wave, WG / 64,
                                  nA, o1, o2, alast, any_partial_row, res_c, res_d);
    __syncthreads();
    for (uint32_t r = 0; r < nrows; r++) {
        const uint32_t i = i0 + r;
        const uint32_t cs = max(c0, i + 1);
        if (cs >= cend) continue;
        const uint64_t base = cond_index(i, cs, N) - seg0;
        for (uint32_t t = tid; t < cend - cs; t += WG) {
            common[base + t] = res_c[r * kApCols + (cs - c0) + t];
            if (denom) denom[base + t] = res_d[r * kApCols + (cs - c0) + t];
        }
    }
}

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
    const uint64_t *a = hashes + (uint64_t)i * s;
    const uint64_t *b = hashes + j * s;
    const uint32_t na = nhash[i], nb = nhash[j];
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
    common[t] = (uint16_t)c;
    if (denom) denom[t] = (uint16_t)d;
}

// ------------------------------------------------------- banded all-pairs
// Large sketches (s > 2048, up to kMaxSketch): a whole-row table no longer fits
// LDS, so the hash range is cut into value bands per row tile.  Band k of a
// tile of R rows is [lo_k, hi_k) with hi_k = min over rows of A_r[p_r + cap]
// (p_r = the row's first element >= lo_k), so every row has <= cap elements in
// the band; those get an LDS cuckoo table (same quotiented format as above,
// storing the element's position *within the band*, at most cap - 1 < H - 1,
// so the empty word still decodes to "absent").  Every column of the tile
// keeps a cursor into its sketch (first element >= lo_k, in LDS); a wave
// streams the column's elements in [lo_k, hi_k) in 64-element chunks and
// counts, per row, shared elements whose union rank
//     i + j - m_j < s          (i = p_r + band position, j = column position)
// is below s -- the same rule as k_allpairs_q, with the running match count
// m and the partial counts carried across bands in LDS.  Bands run until
// every row is exhausted; column elements past the rows' largest element end
// the last band.  Tables are rebuilt per band by the whole workgroup (every
// key verified; up to kMaxFam field families, then the host falls back to the
// literal merge); a band's build is amortised over kBandCols columns.
// Roofline: as k_allpairs_q (LDS random reads + VALU); column chunks are read
// once per band per tile, i.e. s * 8 / R bytes per pair from L2.
constexpr uint32_t kBandCols = 256;
constexpr uint32_t kBandB = 11;                       // H = 2048 slots per choice
constexpr uint32_t kBandCapMax = (1u << kBandB) / 2;  // <= 1024 elements per row per band

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t w = __shfl_xor(v, o, 64);
        v = w < v ? w : v;
    }
    return v;
}
// Column element j (kEmpty past nB): an unconditional load clamped to the
// row (no branch around it), then a select.
__device__ __forceinline__ uint64_t ld_col(const uint64_t *__restrict__ Bc, uint32_t j, uint32_t nB, uint32_t s) {
    const uint64_t v = Bc[j < s ? j : s - 1];
    return j < nB ? v : kEmpty;
}
__device__ __forceinline__ uint32_t rfl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t rfl64(uint64_t v) {
    return ((uint64_t)rfl((uint32_t)(v >> 32)) << 32) | rfl((uint32_t)v);
}

// One 64-element chunk of a column inside the current band.  Returns the
// number of chunk elements inside the band (< 64: the column's band segment
// ends in this chunk).
template <int R, bool FAST>
__device__ __forceinline__ uint32_t band_chunk(uint64_t b, uint32_t j, uint64_t hi, const uint64_t *T,
                                               const uint32_t (&o1)[R], const uint32_t (&o2)[R], uint32_t s,
                                               const uint32_t (&pr)[R], uint32_t actmask, uint32_t (&mrun)[R],
                                               uint32_t (&cnt)[R]) {
    constexpr uint32_t H = 1u << kBandB, hm = H - 1;
    uint32_t cap[R];
#pragma unroll
    for (int r = 0; r < R; r++) cap[r] = kBandCapMax;
    const uint64_t inb = __builtin_amdgcn_ballot_w64(b < hi);
    probe_chunk<R, FAST>(b, j, T, H, hm, o1, o2, actmask, inb, pr, cap, s, mrun, cnt);
    return (uint32_t)__popcll(inb);
}

// A column's band segment: the first NCH chunks from registers (loaded while
// the previous column was processed); a segment longer than NCH chunks
// continues from memory one chunk at a time.  Returns the new cursor.
template <int R, int NCH, bool FAST>
__device__ __forceinline__ uint32_t band_column(const uint64_t *__restrict__ Bc, uint32_t nB, uint32_t q,
                                                const uint64_t (&seg)[NCH], uint64_t hi, const uint64_t *T,
                                                const uint32_t (&o1)[R], const uint32_t (&o2)[R], uint32_t s,
                                                const uint32_t (&pr)[R],
                                                uint32_t actmask, uint32_t (&mrun)[R], uint32_t (&cntl)[R]) {
    const uint32_t lane = threadIdx.x & 63;
    bool more = true;
#pragma unroll
    for (int k = 0; k < NCH; k++) {
        if (!more) continue;                                       // wave-uniform
        const uint32_t nin = band_chunk<R, FAST>(seg[k], q + lane, hi, T, o1, o2, s, pr, actmask, mrun, cntl);
        q += nin;
        more = nin == 64;
    }
    if (!more) return q;
    uint64_t b = ld_col(Bc, q + lane, nB, s);
    for (;;) {
        const uint32_t jn = q + 64 + lane;
        const uint64_t bn = ld_col(Bc, jn, nB, s);
        const uint32_t nin = band_chunk<R, FAST>(b, q + lane, hi, T, o1, o2, s, pr, actmask, mrun, cntl);
        q += nin;
        if (nin < 64) break;
        b = bn;
    }
    return q;
}

template <int R, int NCH, int WG>
__global__ __launch_bounds__(WG) void k_allpairs_band(
    const uint64_t *__restrict__ hashes, const uint32_t *__restrict__ nhash, uint32_t s, uint32_t N,
    uint32_t row1, uint32_t cap, const uint2 *__restrict__ items, uint16_t *__restrict__ common,
    uint16_t *__restrict__ denom, uint64_t seg0, uint32_t *__restrict__ nfail, uint64_t *__restrict__ prof) {
    constexpr uint32_t H = 1u << kBandB, hm = H - 1, TS = 2 * H;
    constexpr uint32_t NW = WG / 64;
    extern __shared__ __align__(16) uint64_t lds[];    // 16-B aligned: the tables are read with ds_read_b128
    uint64_t *T = lds;                                               // R*TS, interleaved
    uint32_t *cur = (uint32_t *)(T + (uint64_t)R * TS);              // [kBandCols] column cursors
    uint32_t *pcnt = cur + kBandCols;                                // [R][kBandCols] counts
    uint32_t *pm = pcnt + R * kBandCols;                             // [R][kBandCols] shared so far
    __shared__ uint32_t s_p[R], s_q[R];
    __shared__ uint64_t s_hi;
    __shared__ int s_done, s_fail, s_abort;

    const uint32_t i0 = items[blockIdx.x].x;
    const uint32_t c0 = items[blockIdx.x].y;
    const uint32_t nrows = min((uint32_t)R, row1 - i0);
    const uint32_t cend = min(c0 + kBandCols, N);
    const uint32_t ncols = cend - c0;
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
    for (uint32_t k = tid; k < kBandCols; k += WG) cur[k] = 0;
    for (uint32_t k = tid; k < R * kBandCols; k += WG) { pcnt[k] = 0; pm[k] = 0; }
    if (tid < (uint32_t)R) s_p[tid] = 0;
    if (tid == 0) s_abort = 0;

    for (;;) {
        __syncthreads();
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
                s_hi = v < maxlast + 1 ? v : maxlast + 1;
                s_done = !any_left;
                s_fail = 0;
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
        // ---- build the R band tables (quotiented cuckoo, band positions)
        uint32_t fam = 0;
        for (; fam < kMaxFam; fam++) {
            const QFields qf = qfields(fam);
            const uint64_t F1 = (uint64_t)hm << qf.o1, F2 = (uint64_t)hm << qf.o2;
            for (uint32_t k = tid; k < R * TS; k += WG) T[k] = kEmpty;
            if (tid == 0) s_fail = 0;
            __syncthreads();
            for (uint32_t idx = tid; idx < R * cap; idx += WG) {
                const uint32_t r = idx / cap, t = idx - r * cap;
                uint32_t p = 0, nl = 0;
#pragma unroll
                for (int rr = 0; rr < R; rr++) if ((uint32_t)rr == r) { p = pr[rr]; nl = nA[rr]; }
                if (p + t >= nl) continue;
                uint64_t x = hashes[(uint64_t)(i0 + r) * s + p + t];
                if (x >= hi) continue;
                uint32_t ix = t;
                uint32_t pos = (uint32_t)(x >> qf.o1) & hm;
                bool placed = false;
                for (int kick = 0; kick < 96; kick++) {
                    const bool second = pos >= H;
                    const uint64_t e = second ? ((x & ~F2) | ((uint64_t)ix << qf.o2))
                                              : ((x & ~F1) | ((uint64_t)ix << qf.o1));
                    const unsigned long long oldr = atomicExch((unsigned long long *)&T[(uint64_t)pos * R + r],
                                                               (unsigned long long)rotr64(e, second ? qf.o2 : qf.o1));
                    if (oldr == kEmpty) { placed = true; break; }
                    const uint64_t old = rotr64(oldr, 64 - (second ? qf.o2 : qf.o1));
                    const uint32_t lp = second ? pos - H : pos;
                    if (second) { ix = (uint32_t)(old >> qf.o2) & hm; x = (old & ~F2) | ((uint64_t)lp << qf.o2); }
                    else        { ix = (uint32_t)(old >> qf.o1) & hm; x = (old & ~F1) | ((uint64_t)lp << qf.o1); }
                    pos = second ? ((uint32_t)(x >> qf.o1) & hm) : (H + ((uint32_t)(x >> qf.o2) & hm));
                }
                if (!placed) s_fail = 1;
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
                const uint64_t e1 = rotr64(T[(uint64_t)((uint32_t)(x >> qf.o1) & hm) * R + r], 64 - qf.o1);
                const uint64_t e2 = rotr64(T[(uint64_t)(H + ((uint32_t)(x >> qf.o2) & hm)) * R + r], 64 - qf.o2);
                const bool ok1 = (e1 & ~F1) == (x & ~F1) && ((uint32_t)(e1 >> qf.o1) & hm) == t;
                const bool ok2 = (e2 & ~F2) == (x & ~F2) && ((uint32_t)(e2 >> qf.o2) & hm) == t;
                if (!(ok1 || ok2)) s_fail = 1;
                if (fam == 0) atomicAdd(&s_q[r], 1u);
            }
            __syncthreads();
            if (!s_fail) break;
        }
        if (fam == kMaxFam) {                       // no field family worked: host reruns with the merge kernel
            if (tid == 0) { s_abort = 1; atomicAdd(nfail, 1u); }
            break;
        }

        uint64_t t_c0 = prof ? wall_clock64() : 0;
        // ---- columns: wave w takes columns w, w+NW, ...; next column's first chunk prefetched
        uint32_t ci = wave;
        uint64_t nseg[NCH];
        uint32_t nq = 0, nnB = 0;
        auto load_seg = [&](uint32_t cc) {
            nq = rfl(cur[cc]);
            nnB = nhash[c0 + cc];
            const uint64_t *Bn = hashes + (uint64_t)(c0 + cc) * s;
#pragma unroll
            for (int k = 0; k < NCH; k++) {
                const uint32_t j = nq + 64 * k + lane;
                nseg[k] = ld_col(Bn, j, nnB, s);
            }
        };
        if (ci < ncols) load_seg(ci);
        for (; ci < ncols; ci += NW) {
            const uint32_t c = c0 + ci;
            const uint32_t q0 = nq, nB = nnB;
            uint64_t seg[NCH];
#pragma unroll
            for (int k = 0; k < NCH; k++) seg[k] = nseg[k];
            if (ci + NW < ncols) load_seg(ci + NW);
            uint32_t actmask = 0;
#pragma unroll
            for (int r = 0; r < R; r++) actmask |= (uint32_t)((uint32_t)r < nrows && i0 + r < c) << r;
            if (!actmask) continue;
            uint32_t mrun[R], cntl[R];
#pragma unroll
            for (int r = 0; r < R; r++) { mrun[r] = rfl(pm[r * kBandCols + ci]); cntl[r] = 0; }   // scalar counters
            const uint64_t *Bc = hashes + (uint64_t)c * s;
            uint32_t o1[R], o2[R];
            const QFields qf = qfields(fam);
#pragma unroll
            for (int r = 0; r < R; r++) { o1[r] = qf.o1; o2[r] = qf.o2; }
            const uint32_t q = fam == 0
                ? band_column<R, NCH, true>(Bc, nB, q0, seg, hi, T, o1, o2, s, pr, actmask, mrun, cntl)
                : band_column<R, NCH, false>(Bc, nB, q0, seg, hi, T, o1, o2, s, pr, actmask, mrun, cntl);
#pragma unroll
            for (int r = 0; r < R; r++)
                if (lane == 0) { pcnt[r * kBandCols + ci] += cntl[r]; pm[r * kBandCols + ci] = mrun[r]; }
            if (lane == 0) cur[ci] = q;
        }
        __syncthreads();
        if (tid < (uint32_t)R) s_p[tid] += s_q[tid];
        if (prof && tid == 0) {
            const uint64_t t_e = wall_clock64();
            atomicAdd((unsigned long long *)&prof[0], (unsigned long long)(t_c0 - t_b0));
            atomicAdd((unsigned long long *)&prof[1], (unsigned long long)(t_e - t_c0));
            atomicAdd((unsigned long long *)&prof[2], 1ull);
        }
    }
    __syncthreads();
    if (s_abort) return;
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
static int launch_merge(drephip_ctx *ctx, const uint64_t *d_hashes, const uint32_t *d_nhash, uint32_t N,
                        uint64_t seg0, uint64_t npairs, uint16_t *d_common, uint16_t *d_denom,
                        hipStream_t st) {
    const uint64_t blocks = (npairs + 255) / 256;
    timing_mark(ctx, 2, st, true);
    hipLaunchKernelGGL(k_allpairs_merge, dim3((uint32_t)blocks), dim3(256), 0, st, d_hashes, d_nhash,
                       ctx->s, N, seg0, npairs, d_common, d_denom);
    timing_mark(ctx, 2, st, false);
    HIPC(hipGetLastError());
    HIPC(hipStreamSynchronize(st));
    return DREPHIP_OK;
}

static int launch_band(drephip_ctx *ctx, const uint64_t *d_hashes, const uint32_t *d_nhash, uint32_t N,
                       uint32_t row0, uint32_t row1, uint64_t seg0, uint64_t npairs, uint16_t *d_common,
                       uint16_t *d_denom, hipStream_t st) {
    constexpr int R = 4;
    const uint32_t cap = std::min(std::max(ctx->band_cap, 1u), kBandCapMax);
    std::vector<uint2> items;
    for (uint32_t i0 = row0; i0 < row1; i0 += R)
        for (uint32_t c0 = i0 + 1; c0 < N; c0 += kBandCols) items.push_back(make_uint2(i0, c0));
    if (items.empty()) return DREPHIP_OK;
    uint2 *d_items;
    uint32_t *d_nfail;
    int rc;
    if ((rc = scratch(ctx, "apb_items", items.size() * sizeof(uint2), (void **)&d_items))) return rc;
    if ((rc = scratch(ctx, "ap_nfail", 4, (void **)&d_nfail))) return rc;
    HIPC(hipMemsetAsync(d_nfail, 0, 4, st));
    HIPC(hipMemcpyAsync(d_items, items.data(), items.size() * sizeof(uint2), hipMemcpyHostToDevice, st));
    uint64_t *d_prof = nullptr;                      // DREPHIP_BAND_PROF=1: per-phase wall-clock sums
    const bool prof = getenv("DREPHIP_BAND_PROF") != nullptr;
    if (prof) {
        if ((rc = scratch(ctx, "apb_prof", 64, (void **)&d_prof))) return rc;
        HIPC(hipMemsetAsync(d_prof, 0, 64, st));
    }
    const size_t lds = (size_t)R * (2u << kBandB) * 8 + kBandCols * 4 + 2ull * R * kBandCols * 4;
    // 16 waves x 8 register chunks per band segment (8 waves x 16 chunks,
    // 512-lane workgroups, measured 1.35x slower at s = 10^4)
    HIPC(hipFuncSetAttribute((const void *)k_allpairs_band<R, 8, 1024>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    timing_mark(ctx, 2, st, true);
    hipLaunchKernelGGL((k_allpairs_band<R, 8, 1024>), dim3((uint32_t)items.size()), dim3(1024), lds, st, d_hashes,
                       d_nhash, ctx->s, N, row1, cap, d_items, d_common, d_denom, seg0, d_nfail, d_prof);
    timing_mark(ctx, 2, st, false);
    HIPC(hipGetLastError());
    uint32_t nfail = 0;
    HIPC(hipMemcpyAsync(&nfail, d_nfail, 4, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    if (prof) {
        uint64_t h[3];
        HIPC(hipMemcpy(h, d_prof, 24, hipMemcpyDeviceToHost));
        fprintf(stderr, "[drephip] band kernel: %llu bands over %zu items; per band: build %.2f us, columns %.2f us (100 MHz wall clock)\n",
                (unsigned long long)h[2], items.size(), h[2] ? h[0] / 100.0 / h[2] : 0.0, h[2] ? h[1] / 100.0 / h[2] : 0.0);
    }
    if (nfail)   // a band table could not be built with any field pair: exact merge kernel instead
        return launch_merge(ctx, d_hashes, d_nhash, N, seg0, npairs, d_common, d_denom, st);
    return DREPHIP_OK;
}

template <int R, int NCH>
static int launch_q(drephip_ctx *ctx, uint32_t nitems, size_t lds, hipStream_t st, const uint64_t *h,
                    const uint32_t *nh, const uint64_t *tabs, const uint8_t *fam, uint32_t N, uint32_t row0,
                    uint32_t row1, uint32_t B, const uint2 *items, uint16_t *cm, uint16_t *dn, uint64_t seg0) {
    HIPC(hipFuncSetAttribute((const void *)k_allpairs_q<R, NCH>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)lds));
    timing_mark(ctx, 2, st, true);
    hipLaunchKernelGGL((k_allpairs_q<R, NCH>), dim3(nitems), dim3(ap_wg(NCH)), lds, st, h, nh, tabs, fam, ctx->s, N,
                       row0, row1, B, items, cm, dn, seg0);
    timing_mark(ctx, 2, st, false);
    HIPC(hipGetLastError());
    return DREPHIP_OK;
}

int allpairs_device_impl(drephip_ctx *ctx, const uint64_t *d_hashes, const uint32_t *d_nhash, uint32_t N,
                         uint32_t row0, uint32_t row1, uint16_t *d_common, uint16_t *d_denom,
                         hipStream_t st, bool force_merge) {
    if (row1 > N) row1 = N;
    if (N < 2 || row0 >= row1 || row0 >= N - 1) return DREPHIP_OK;
    if (row1 > N - 1) row1 = N - 1;
    const uint32_t s = ctx->s;
    const uint64_t seg0 = cond_index(row0, row0 + 1, N);
    const uint64_t seg1 = row1 < N - 1 ? cond_index(row1, row1 + 1, N) : (uint64_t)N * (N - 1) / 2;
    const uint64_t npairs = seg1 - seg0;
    // table: 2H slots, H = 2^B >= 2s (load <= 1/4) and 2^B > s (positions fit the field)
    uint32_t B = 4;
    while ((1u << B) < 2 * s) B++;
    const uint64_t TS = 2ull << B;
    const bool fits = s <= 2048 && TS * 8 <= kLdsTables;
    int path = force_merge ? DREPHIP_AP_MERGE : ctx->ap_path;
    if (path == DREPHIP_AP_AUTO) path = fits ? DREPHIP_AP_TABLE : DREPHIP_AP_BAND;
    if (path == DREPHIP_AP_TABLE && !fits) {
        set_error("whole-row table all-pairs kernel needs s <= 2048");
        return DREPHIP_ERR_UNSUPPORTED;
    }
    if (path == DREPHIP_AP_MERGE)
        return launch_merge(ctx, d_hashes, d_nhash, N, seg0, npairs, d_common, d_denom, st);
    if (path == DREPHIP_AP_BAND)
        return launch_band(ctx, d_hashes, d_nhash, N, row0, row1, seg0, npairs, d_common, d_denom, st);

    const uint32_t nrows = row1 - row0;
    uint64_t *d_tabs;
    uint8_t *d_fam;
    uint32_t *d_nfail;
    uint2 *d_items;
    int rc;
    if ((rc = scratch(ctx, "ap_tabs", (uint64_t)nrows * TS * 8, (void **)&d_tabs))) return rc;
    if ((rc = scratch(ctx, "ap_fam", nrows, (void **)&d_fam))) return rc;
    if ((rc = scratch(ctx, "ap_nfail", 4, (void **)&d_nfail))) return rc;
    HIPC(hipMemsetAsync(d_nfail, 0, 4, st));
    const size_t blds = TS * 8;
    HIPC(hipFuncSetAttribute((const void *)k_build_qcuckoo, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)blds));
    timing_mark(ctx, 3, st, true);
    hipLaunchKernelGGL(k_build_qcuckoo, dim3(nrows), dim3(256), blds, st, d_hashes, d_nhash, s, row0, B,
                       d_tabs, d_fam, d_nfail);
    timing_mark(ctx, 3, st, false);
    HIPC(hipGetLastError());

    static const uint32_t kR[] = {8, 4, 2, 1};
    uint32_t R = 1;
    for (uint32_t r : kR) if ((uint64_t)r * TS * 8 <= kLdsTables) { R = r; break; }
    std::vector<uint2> items;
    for (uint32_t i0 = row0; i0 < row1; i0 += R)
        for (uint32_t c0 = i0 + 1; c0 < N; c0 += kApCols) items.push_back(make_uint2(i0, c0));
    if ((rc = scratch(ctx, "ap_items", items.size() * sizeof(uint2), (void **)&d_items))) return rc;
    HIPC(hipMemcpyAsync(d_items, items.data(), items.size() * sizeof(uint2), hipMemcpyHostToDevice, st));
    uint32_t nfail = 0;
    HIPC(hipMemcpyAsync(&nfail, d_nfail, 4, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    if (nfail)   // a row table could not be built with any field pair: exact merge kernel instead
        return launch_merge(ctx, d_hashes, d_nhash, N, seg0, npairs, d_common, d_denom, st);

    const size_t lds = (size_t)R * TS * 8 + (size_t)R * kApCols * 4;
    const uint32_t ni = (uint32_t)items.size();
    const bool big = s > 1024;
#define DREPHIP_Q(RR, NC) launch_q<RR, NC>(ctx, ni, lds, st, d_hashes, d_nhash, d_tabs, d_fam, N, row0, row1, B, d_items, d_common, d_denom, seg0)
    if (!big) {
        switch (R) {
            case 8: rc = DREPHIP_Q(8, 8); break;       // R = 8 only when H <= 1024, i.e. s <= 512
            case 4: rc = DREPHIP_Q(4, 16); break;
            case 2: rc = DREPHIP_Q(2, 16); break;
            default: rc = DREPHIP_Q(1, 16); break;
        }
    } else {
        switch (R) {
            case 2: rc = DREPHIP_Q(2, 32); break;
            default: rc = DREPHIP_Q(1, 32); break;
        }
    }
#undef DREPHIP_Q
    if (rc) return rc;
    HIPC(hipStreamSynchronize(st));
    return DREPHIP_OK;
}

}  // namespace drephip
