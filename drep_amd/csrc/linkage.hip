// linkage.hip -- primary clustering at scale: scipy.cluster.hierarchy.linkage
// (the call dRep's cluster_hierarchical makes, drep/d_cluster.py:453, on the
// distances built at 447) restated on the GPU, bit-identical to scipy:
//   complete / average / weighted : scipy's nn_chain (nearest-neighbour chain
//                                   with the previous chain element preferred
//                                   on ties, Lance-Williams updates in f64);
//   single                        : scipy's mst_single_linkage (Prim).
// Then, on the host as scipy does: stable sort of the merges by distance and
// the union-find relabel (scipy's `label`).
//
// The distance matrix lives in HBM as a full symmetric n x n f64 matrix (80 GB
// at n = 10^5 -- one MI355X holds it), built on the device straight from the
// all-pairs shared-hash counts through a per-(denominator, common) table of
// the exact float64 values dRep feeds scipy; nothing n^2 crosses PCIe.  Each
// step of the (inherently sequential) chain is one launch: the previous
// step's chain decision (made by every workgroup from the previous launch's
// partials), the pending merge's row + column update and the grid-wide argmin
// over the chain top's row.  Steps are launched in batches captured in a
// hipGraph; kernels after the last merge exit at once.
// Roofline: latency -- a step reads one 8n-byte row (and after a merge two
// more rows, writing a row and a strided column; a speculating step reads two
// more); at n = 10^5 (0.8 MB rows) the kernel boundary (~2 us) and the two
// dependent round trips of a step (state + partials, then the rows) dominate,
// ~5.5-7 us per launch, ~1.3 launches per merge with the speculation below
// (DESIGN.md 4.4).

#include "ctx.h"
#include "../../include/drephip.h"

#include <algorithm>
#include <cstddef>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <vector>

namespace drephip {

// step workgroups: 256 lanes, or 128 for n <= kLkSmallN (more workgroups
// per row at small n: 136 vs 143 ms of chain at n = 10^4; 256 is faster at
// 10^5 -- profiles/r03_linkage_wg_ab.txt)
constexpr int kLkWG = 256;
// Column-y stores of a merge step: 3 write-through (sc1, default), 1 plain, 2
// nontemporal, 0 none (A/B timing only).  A merge leaves one dirty line per
// row of column y (10^5 lines = 6.4 MB at n = 10^5) that a plain store leaves
// in L2 until the kernel boundary's write-back (~1 us at ~6 TB/s on the chain's
// critical path); written through, the lines leave during the step: chain at
// 10^5 967 -> 917 ms (nontemporal 945 ms; profiles/r05_linkage_protocol_colstore_ab.txt)
#ifndef DREPHIP_LK_COLSTORE
#define DREPHIP_LK_COLSTORE 3
#endif
// Row-y stores (contiguous, 8n bytes per merge): 3 write-through (default since round 5:
// the row leaves L2 during the step instead of at the kernel boundary; chain at
// 10^5 -0.8 %, profiles/r05_linkage_ab_stores.txt), 1 plain
#ifndef DREPHIP_LK_ROWSTORE
#define DREPHIP_LK_ROWSTORE 3
#endif
constexpr uint32_t kLkSmallN = 30000;
// Per-wave partials (round 5, A/B): each wave of a step workgroup stores its
// own argmin partials (no LDS exchange, no barrier at the end of the step); the
// next decision reduces WG / 64 times as many.  Measured slower at 10^5 (chain
// 898-908 vs 854-856 ms with one partial per workgroup, profiles/r05_linkage_ab_waveparts.txt):
// the decision's pass over 4x the partials (16 per lane, 234 VGPRs) costs more
// than the block reduction it saves.  0 (default): one partial per workgroup
#ifndef DREPHIP_LK_WAVEPARTS
#define DREPHIP_LK_WAVEPARTS 0
#endif
constexpr uint32_t kLkPartStride = 4096;        // partials per parity: up to 1024 workgroups x 4 waves

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct MinIdx { double v; int32_t i; };
// a step workgroup's three partial minima (P1 the top's row, P2 the merged or
// speculated merged row, P3 the speculated row below), one 48-byte record: one
// base address for the three sets (their loads and stores take immediate offsets)
struct PartRec { MinIdx p1, p2, p3; };
static_assert(sizeof(PartRec) == 48, "PartRec layout");

// Phase timestamps of the chain step (an A/B build only: make EXTRA=-DDREPHIP_LK_PHASES=1):
// s_memrealtime (100 MHz) at fixed points of workgroup 0, the last step
// workgroup and the forwarding workgroup, per launch; the host prints medians.
#ifndef DREPHIP_LK_PHASES
#define DREPHIP_LK_PHASES 0
#endif
#if DREPHIP_LK_PHASES
constexpr int kPhCap = 65536;
__device__ uint64_t *g_lk_ph;
#define LK_T(v) v = __builtin_amdgcn_s_memrealtime()
#else
#define LK_T(v) (void)0
#endif

// Adverse workgroup order (a test build only: make EXTRA=-DDREPHIP_LK_ADVERSE=1
// or 2): the step and compaction kernels' even (1) or odd (2) workgroups sleep
// ~14 us before their main loads, so the other workgroups of the same launch
// have finished their stores by the time those loads run.  Every value a
// kernel reads must then still be the one of the launch before it -- the
// rule "no workgroup reads what another workgroup of the same launch writes"
// (the producer/consumer table) -- or Z departs from scipy's
// (tests/test_gpu.py::test_linkage_adverse_workgroup_order).
#ifndef DREPHIP_LK_ADVERSE
#define DREPHIP_LK_ADVERSE 0
#endif
__device__ __forceinline__ void adverse_delay() {
#if DREPHIP_LK_ADVERSE
    if ((blockIdx.x & 1u) == (DREPHIP_LK_ADVERSE == 1 ? 0u : 1u))
        for (int k = 0; k < 4; k++) __builtin_amdgcn_s_sleep(127);
#endif
}

__device__ __forceinline__ bool better(double v, int32_t i, double bv, int32_t bi) {
    return v < bv || (v == bv && i < bi);
}

// Lance-Williams updates exactly as scipy's _hierarchy_distance_update.pxi:
// every operation rounded on its own, as in scipy's x86-64 build (this file is
// compiled with -ffp-contract=off; see the Makefile)
__device__ __forceinline__ double lw_update(int method, double dxi, double dyi, int32_t nx, int32_t ny) {
    // (method is a template argument of the step kernels: the switch folds away;
    // as a runtime argument every update in the row pass branched three ways)
    if (method == DREPHIP_LINK_COMPLETE) return fmax(dxi, dyi);
    if (method == DREPHIP_LINK_WEIGHTED) return __dmul_rn(0.5, __dadd_rn(dxi, dyi));
    // average: (size_x * d_xi + size_y * d_yi) / (size_x + size_y)
    return __ddiv_rn(__dadd_rn(__dmul_rn((double)nx, dxi), __dmul_rn((double)ny, dyi)), (double)(nx + ny));
}

// The same update with the average's division by the step-uniform n = nx + ny
// done as Markstein's correction step: with r = RN(1/n) (one IEEE division per
// launch) and q = RN(a r), within an ulp of a/n, e = a - q n is exact (one
// FMA) and RN(q + e r) = RN(a/n) -- the correctly rounded quotient, i.e. the
// same bits as the division, for every a and n without overflow or underflow
// (here a in [0, 2 x 10^5], n an integer <= 10^5; tools/div_check.c checks 4 x
// 10^8 cases of this exact expression on the host).  Three dependent f64
// operations instead of the division's ~12 on the row pass's critical path.
struct LwDiv { double n, r; };
__device__ __forceinline__ LwDiv lw_div(int32_t nx, int32_t ny) {
    const double n = (double)(nx + ny);
    return LwDiv{n, __ddiv_rn(1.0, n)};
}
__device__ __forceinline__ double lw_update(int method, double dxi, double dyi, int32_t nx, int32_t ny, LwDiv dv) {
    if (method != DREPHIP_LINK_AVERAGE) return lw_update(method, dxi, dyi, nx, ny);
    const double a = __dadd_rn(__dmul_rn((double)nx, dxi), __dmul_rn((double)ny, dyi));
    const double q = __dmul_rn(a, dv.r);
    const double e = __fma_rn(-q, dv.n, a);
    return __fma_rn(e, dv.r, q);
}

// Wave argmin by DPP (row_shr 1/2/4/8 within each 16-lane row, then
// row_bcast 15/31 across rows: lane 63 ends with the wave's minimum, which
// readlane broadcasts), in two passes: the minimum value (v_min_f64 of the
// lane and its DPP-shifted neighbour), then the smallest index among the
// lanes holding it (v_min_i32).  One pass over (value, index) pairs with the
// lexicographic compare took ~12 instructions a step -- a wave reduction is
// on a chain step's critical path several times, so it pays to keep it short.
// Lanes a shift leaves without a source keep the identity (inf, INT_MAX).
// Values are never NaN.  Needs every lane of the wave active.
template <int CTRL, int RM>
__device__ __forceinline__ double dpp_f64(double v) {
    const long long b = __double_as_longlong(v);
    const long long ib = __double_as_longlong((double)INFINITY);
    const int lo = __builtin_amdgcn_update_dpp((int)ib, (int)b, CTRL, RM, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(ib >> 32), (int)(b >> 32), CTRL, RM, 0xf, false);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
template <int CTRL, int RM>
__device__ __forceinline__ int32_t dpp_i32(int32_t i) {
    return __builtin_amdgcn_update_dpp(0x7fffffff, i, CTRL, RM, 0xf, false);
}
__device__ __forceinline__ double min_f64(double a, double b) { return fmin(a, b); }
// N independent sets at once: their steps interleave, hiding each other's
// DPP hazards and latencies
template <int N>
__device__ __forceinline__ void wave_argmin_n(double (&v)[N], int32_t (&i)[N]) {
    double m[N];
#pragma unroll
    for (int s = 0; s < N; s++) m[s] = v[s];
#define DREPHIP_DPP_MIN(C, R) _Pragma("unroll") for (int s = 0; s < N; s++) m[s] = min_f64(m[s], dpp_f64<C, R>(m[s]))
    DREPHIP_DPP_MIN(0x111, 0xf);
    DREPHIP_DPP_MIN(0x112, 0xf);
    DREPHIP_DPP_MIN(0x114, 0xf);
    DREPHIP_DPP_MIN(0x118, 0xf);
    DREPHIP_DPP_MIN(0x142, 0xa);
    DREPHIP_DPP_MIN(0x143, 0xc);
#undef DREPHIP_DPP_MIN
    int32_t c[N];
#pragma unroll
    for (int s = 0; s < N; s++) {
        const long long b = __double_as_longlong(m[s]);
        const int lo = __builtin_amdgcn_readlane((int)b, 63), hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
        m[s] = __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
        c[s] = v[s] == m[s] ? i[s] : 0x7fffffff;
    }
#define DREPHIP_DPP_MINI(C, R) _Pragma("unroll") for (int s = 0; s < N; s++) c[s] = min(c[s], dpp_i32<C, R>(c[s]))
    DREPHIP_DPP_MINI(0x111, 0xf);
    DREPHIP_DPP_MINI(0x112, 0xf);
    DREPHIP_DPP_MINI(0x114, 0xf);
    DREPHIP_DPP_MINI(0x118, 0xf);
    DREPHIP_DPP_MINI(0x142, 0xa);
    DREPHIP_DPP_MINI(0x143, 0xc);
#undef DREPHIP_DPP_MINI
#pragma unroll
    for (int s = 0; s < N; s++) { v[s] = m[s]; i[s] = __builtin_amdgcn_readlane(c[s], 63); }
}
__device__ __forceinline__ void wave_argmin(double &v, int32_t &i) {
    double vv[1] = {v};
    int32_t ii[1] = {i};
    wave_argmin_n<1>(vv, ii);
    v = vv[0]; i = ii[0];
}
// one, two or three sets (block-uniform counts), interleaved
__device__ __forceinline__ void wave_argmin_upto3(MinIdx &a, MinIdx &b, MinIdx &c, bool with_b, bool with_c) {
    if (with_c) {
        double v[3] = {a.v, b.v, c.v};
        int32_t i[3] = {a.i, b.i, c.i};
        wave_argmin_n<3>(v, i);
        a = MinIdx{v[0], i[0]}; b = MinIdx{v[1], i[1]}; c = MinIdx{v[2], i[2]};
    } else if (with_b) {
        double v[2] = {a.v, b.v};
        int32_t i[2] = {a.i, b.i};
        wave_argmin_n<2>(v, i);
        a = MinIdx{v[0], i[0]}; b = MinIdx{v[1], i[1]};
    } else {
        wave_argmin(a.v, a.i);
    }
}

// Block argmin (smallest index among equal minima); result valid in thread 0.
template <int WG>
__device__ MinIdx block_argmin(double v, int32_t i) {
    __shared__ double sv[WG / 64];
    __shared__ int32_t si[WG / 64];
    wave_argmin(v, i);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { sv[w] = v; si[w] = i; }
    __syncthreads();
    MinIdx r{INFINITY, 0x7fffffff};
    if (threadIdx.x == 0)
        for (int k = 0; k < WG / 64; k++)
            if (better(sv[k], si[k], r.v, r.i)) { r.v = sv[k]; r.i = si[k]; }
    return r;
}

// A lane's share of the previous launch's partial sets: partials lane,
// lane + 64, ... U at a time, every load in flight before the first wait
template <int U>
__device__ __forceinline__ void partial_pass(const PartRec *P, uint32_t G, MinIdx &g, MinIdx &g2, MinIdx &g3) {
    for (uint32_t b0 = threadIdx.x; b0 < G; b0 += 64 * U) {
        MinIdx m1[U], m2[U], m3[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t b = min(b0 + 64u * u, G - 1);             // (a repeated partial changes no minimum)
            m1[u] = P[b].p1; m2[u] = P[b].p2; m3[u] = P[b].p3;
        }
#pragma unroll
        for (int u = 0; u < U; u++)
            asm volatile("" : "+v"(m1[u].v), "+v"(m1[u].i), "+v"(m2[u].v), "+v"(m2[u].i), "+v"(m3[u].v), "+v"(m3[u].i));
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (better(m1[u].v, m1[u].i, g.v, g.i)) g = m1[u];
            if (better(m2[u].v, m2[u].i, g2.v, g2.i)) g2 = m2[u];
            if (better(m3[u].v, m3[u].i, g3.v, g3.i)) g3 = m3[u];
        }
    }
}

// Up to three block argmins at once, one barrier (results in thread 0): a
// chain step reduces one to three sets per launch and per decision.  b and c
// are reduced only when the (block-uniform) flags ask for them: an unneeded
// wave reduction measured as costly as the barrier it saves.
template <int WG>
__device__ void block_argmin3(MinIdx &a, MinIdx &b, MinIdx &c, bool with_b, bool with_c) {
    __shared__ double sv[3][WG / 64];
    __shared__ int32_t si[3][WG / 64];
    wave_argmin_upto3(a, b, c, with_b, with_c);
    if constexpr (WG == 64) return;                            // one wave: every lane holds the result
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        sv[0][w] = a.v; si[0][w] = a.i;
        sv[1][w] = b.v; si[1][w] = b.i;
        sv[2][w] = c.v; si[2][w] = c.i;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        a = b = c = MinIdx{INFINITY, 0x7fffffff};
        for (int k = 0; k < WG / 64; k++) {
            if (better(sv[0][k], si[0][k], a.v, a.i)) { a.v = sv[0][k]; a.i = si[0][k]; }
            if (better(sv[1][k], si[1][k], b.v, b.i)) { b.v = sv[1][k]; b.i = si[1][k]; }
            if (better(sv[2][k], si[2][k], c.v, c.i)) { c.v = sv[2][k]; c.i = si[2][k]; }
        }
    }
}

// ---------------------------------------------------------------- the steps
// One chain step per launch: the pending merge's Lance-Williams update (row and
// column y) fused with the search of the chain top's row.  The search of row
// t = chain top reads D[t][i]; the update rewrites only row/column y, so every
// D[t][i] with i != y is untouched, and the one changed entry D[t][y] is
// produced by the lane of i = y from two uniform loads (D[x][t], D[y][t]) --
// no cross-workgroup dependence within the step.  After a chain restart t may
// be y itself: then the search value of i is the freshly computed D[y][i].
//
// A step's chain decision is made at the START of the next launch: kernel s
// publishes its workgroup partials (plain stores -- the kernel boundary orders
// them) and every workgroup of kernel s + 1 reads all of them and makes step
// s's scipy decision itself (replicated: same partials, same state, same
// bits) before doing step s + 1's work.  An earlier version reduced the
// partials in the last workgroup of kernel s (a drained partial store, an
// agent-scope ticket, the last workgroup's partial loads) and measured
// 2.09 s at n = 10^5 against 1.92 s for this one (profiles/r03_linkage_*).
// Workgroup 0 alone writes the decision's side effects (Z row, chain push)
// and the state the next kernel reads; the two sizes a merge changes are
// written by workgroup 0 of the launch AFTER the deciding one, and every
// reader of that launch overrides them (it knows the decision), so no
// workgroup reads a value another workgroup of the same launch may be
// writing.  State and partials are double buffered by step parity q (kernel q
// reads buffer q ^ 1 and writes q); the chain entries a launch reads after a
// merge (the new top and below, chain[len-3] and chain[len-4]) are below the
// position a push writes.
//
// A step is a chain of dependent memory round trips, so the loads are issued
// together: each pass takes kLkPer (1, 2 or 4) entries per lane (grid-stride) and loads
// their sizes and D[t][i] (plus D[x][i], D[y][i] after a merge) before any of
// them is used or any store is made (written as one loop, the compiler kept
// each entry's loads behind the previous entry's stores: D aliases itself).
// The decision's operands -- D[t][below] and the two sizes -- are loaded with
// the partials: the chain's elements below the top are never x or y, so no
// update touches them.
//
// The state is one 64-byte line (the sizes and the row a merge changes are
// functions of pend, x, y, nx, ny); per-step diagnostic counters exist only in
// a DREPHIP_LK_DIAG=1 build.
struct alignas(64) LinkState {
    int32_t k, len, top, below, first_active;
    int32_t pend, x, y, nx, ny;   // the merge this state's launch applies: x < y, row/column y rewritten, x retired
    int32_t c3;                   // chain[len - 3]
    int32_t spec;                 // rows this launch reduces besides or instead of the top's (k_nn_step): 0-3
    int32_t known;                // 1: the next launch's first decision is the merge of top and below
    int32_t flags;                // 1: the reader first decides the previous step from its partials; 2: bad
    int32_t mx;                   // MST: current vertex
    int32_t launches;             // working launches (reported: launches per merge)
};
static_assert(sizeof(LinkState) == 64, "the step state is one 64-byte line");
constexpr int32_t kLkDecide = 1, kLkBad = 2;
#ifndef DREPHIP_LK_DIAG
#define DREPHIP_LK_DIAG 0
#endif
#if DREPHIP_LK_DIAG
// diagnostic build: counters kept by lane 0 of workgroup 0 (a dependent
// load + store per launch; never in the product build)
struct LinkDiag { int32_t twice, scans, specwin, known, m0, wmerge, recip; };
__device__ LinkDiag *g_lk_diag;
#define LK_DIAG(field) do { if (w0l) g_lk_diag->field++; } while (0)   // (a divergent store: diagnostic builds only)
#else
#define LK_DIAG(field) (void)0
#endif

// The decision's operands -- D[top][below], the two sizes and the chain
// entries a merge exposes -- are loaded by one extra workgroup of the kernel
// that makes the PREVIOUS decision (it replicates that decision and writes
// them to fwd[q] while the others run the step), so a step's critical path is
// two dependent round trips (state + partials, issued together; then the row)
// instead of three.  They are stable while that kernel runs: D[top][below]
// after a merge is between chain elements below the merged pair (never x or
// y), after a push no update is pending; the chain entries are older than the
// kernel's own push; the sizes go through the same overrides as everywhere.
struct alignas(64) LinkFwd {
    double dp;
    int32_t szt, szb, c3, c4;
    double dp2;                   // D[w][c4], w = c3 (the speculation's decision operand)
    int32_t spec;                 // 1: the P2 partials hold a speculated merged row's minimum, P3 the row below's
    int32_t c5, c6;               // chain[len - 5], chain[len - 6]: chain[len - 3], chain[len - 4] after a merge
                                  // (a known merge's row W and its decision operand D[W][below W])
};
static_assert(offsetof(LinkFwd, dp2) == 24 && offsetof(LinkFwd, spec) == 32 && offsetof(LinkFwd, c6) == 40,
              "LinkFwd word layout (fwd_from_words)");

// the chain's control block: both parities of the state and of the forwarded
// operands, and the merge count the host polls -- one base address (immediate
// offsets) for the step kernel instead of three pointers in SGPRs
struct alignas(64) LinkCtl {
    LinkState st[2];
    LinkFwd fwd[2];
    int32_t done;
};

// a uniform 32-bit word held in a VGPR -> SGPR
__device__ __forceinline__ int32_t rfl(uint32_t v) { return __builtin_amdgcn_readfirstlane((int32_t)v); }
__device__ __forceinline__ MinIdx uni(MinIdx m) {       // a wave-uniform (value, index) into SGPRs
    const uint64_t b = (uint64_t)__double_as_longlong(m.v);
    const uint32_t lo = (uint32_t)rfl((uint32_t)b), hi = (uint32_t)rfl((uint32_t)(b >> 32));
    return MinIdx{__longlong_as_double((long long)(((uint64_t)hi << 32) | lo)), rfl((uint32_t)m.i)};
}
__device__ __forceinline__ LinkState state_from_words(uint4 a, uint4 b, uint4 c, uint4 d) {
    LinkState S;
    S.k = rfl(a.x); S.len = rfl(a.y); S.top = rfl(a.z); S.below = rfl(a.w);
    S.first_active = rfl(b.x); S.pend = rfl(b.y); S.x = rfl(b.z); S.y = rfl(b.w);
    S.nx = rfl(c.x); S.ny = rfl(c.y); S.c3 = rfl(c.z); S.spec = rfl(c.w);
    S.known = rfl(d.x); S.flags = rfl(d.y); S.mx = rfl(d.z); S.launches = rfl(d.w);
    return S;
}
__device__ __forceinline__ LinkFwd fwd_from_words(uint4 a, uint4 b, uint4 c) {
    LinkFwd F;
    F.dp = __longlong_as_double((long long)(((uint64_t)(uint32_t)rfl(a.y) << 32) | (uint32_t)rfl(a.x)));
    F.szt = rfl(a.z); F.szb = rfl(a.w); F.c3 = rfl(b.x); F.c4 = rfl(b.y);
    F.dp2 = __longlong_as_double((long long)(((uint64_t)(uint32_t)rfl(b.w) << 32) | (uint32_t)rfl(b.z)));
    F.spec = rfl(c.x); F.c5 = rfl(c.y); F.c6 = rfl(c.z);
    return F;
}

// all partials of the previous kernel -> their minimum (thread 0)
template <int WG>
__device__ __forceinline__ MinIdx read_partials(const MinIdx *parts, uint32_t G) {
    double bv = INFINITY;
    int32_t bi = 0x7fffffff;
    for (uint32_t b = threadIdx.x; b < G; b += WG) {             // (WG: see k_nn_step)
        const MinIdx m = parts[b];
        if (better(m.v, m.i, bv, bi)) { bv = m.v; bi = m.i; }
    }
    return block_argmin<WG>(bv, bi);
}

// Round 4: a merge step also reduces the merged row y to its minimum (the
// "P2" partials; the new values are computed there anyway).  When the next
// step pushes y -- the new top's nearest neighbour is often the cluster just
// formed -- y's own step is decided at once from P2 instead of by a launch
// that searches y's row: up to two chain steps per launch.
//
// Speculation on a merge of the top A with the element below it, B: the launch
// reduces the row U that merge would form (index max(A, B); P2) and the row of
// the element below B, W, as it would be after it (P3: W's row without A and
// B, plus (U[W], max(A, B))).  When the next launch's decision is that merge,
// it decides W's step from P3 -- and, when W pushes the merged row, that row's
// step from P2 -- in the same launch.  The rows are taken as they are after
// this launch's own merge (x, y): row y is the update u this launch computes,
// and entry y of any other row R is U1[R] = LW(D[x][R], D[y][R]).
//   spec 1: a search launch (no merge): A, B, W as stored;
//   spec 2: a merge launch whose merged row is B (just pushed back below the top);
//   spec 3 (round 5): the next decision is KNOWN to be the merge of A and B
//           -- W's decision from P3 was a merge with the element below it, or
//           W pushed the merged row b and b's own minimum (P2) ties with W, so b
//           merges back -- and the launch speculates on that merge INSTEAD of
//           searching the top's row (which would only confirm it): the next
//           launch applies it and decides the step after it at once.  In the
//           round-4 protocol the launch searched the top again, the next one
//           merged without speculation, and a third searched the new top:
//           launches per merge 1.318 -> 1.225 at 10^4 (tools/chain_sim.py,
//           the host model of this protocol, Z identical to scipy's).
// One merge per launch stays the rule.
template <int WG, int kLkPer, int method>
__global__ __launch_bounds__(WG) void k_nn_step(double *__restrict__ D, uint32_t n,
                                                   int32_t *__restrict__ size, int32_t *__restrict__ chain,
                                                   LinkCtl *__restrict__ ctl, PartRec *__restrict__ parts,
                                                   double *__restrict__ Z, uint32_t q, int spec_on) {
    __shared__ LinkState sx;
    LinkState *const st = ctl->st;
    LinkFwd *const fwd = ctl->fwd;
    int32_t *const done = &ctl->done;
    const uint32_t G = gridDim.x - 1;                          // step workgroups; workgroup G forwards operands
    // The partial sets are reduced by wave 0 alone (the decision is wave 0's:
    // no barrier), read whether or not they are needed (valid memory either
    // way).  Their loads are issued before the state's: a state load landing
    // in a scalar register the compiler reuses waited for the state before
    // the partial loads went out (one round trip more per step).  A lane
    // takes partials lane, lane + 64, ... four at a time, all loads in flight
    // before the first wait.  (The loop steps by a constant: a blockDim.x
    // stride's kernarg load held the partial loads behind the state's.)
    // wave 0, as a wave-uniform condition (readfirstlane): the decision below
    // runs on every lane of wave 0 as scalar code, its values in SGPRs (as
    // one lane's divergent code it took ~0.8 us a launch)
    const bool wave0 = __builtin_amdgcn_readfirstlane(threadIdx.x) < 64, lane0 = threadIdx.x == 0;
    MinIdx g{INFINITY, 0x7fffffff}, g2{INFINITY, 0x7fffffff}, g3{INFINITY, 0x7fffffff};
    // state and forwarded operands: vector loads through an opaque zero lane
    // offset, issued first, so the partial loads go out behind them and one
    // wait covers both (as scalar loads, a state field landing in a scalar
    // register the compiler reused made it wait for the state before issuing
    // the partial loads: one more round trip per step); then read into SGPRs
    int32_t lz0;
    asm volatile("v_mov_b32 %0, 0" : "=v"(lz0));
    const uint4 *sv = (const uint4 *)(st + (q ^ 1)) + lz0;
    const uint4 *fv = (const uint4 *)(fwd + (q ^ 1)) + lz0;
    uint4 sw0 = sv[0], sw1 = sv[1], sw2 = sv[2], sw3 = sv[3], fw0 = fv[0], fw1 = fv[1], fw2 = fv[2];
    if (wave0) {
        const PartRec *P = parts + (uint64_t)(q ^ 1) * kLkPartStride;
        // partials: one per step wave (DREPHIP_LK_WAVEPARTS) or per step workgroup
        const uint32_t NP = DREPHIP_LK_WAVEPARTS ? G * (WG / 64) : G;
        if (NP <= 256) partial_pass<4>(P, NP, g, g2, g3);
        else if (!DREPHIP_LK_WAVEPARTS || NP <= 512) partial_pass<8>(P, NP, g, g2, g3);   // (512 a pass)
        else partial_pass<16>(P, NP, g, g2, g3);                    // (up to 1024 in one pass)
    }
    asm volatile("" : "+v"(sw0.x), "+v"(sw0.y), "+v"(sw0.z), "+v"(sw0.w), "+v"(sw1.x), "+v"(sw1.y), "+v"(sw1.z),
                 "+v"(sw1.w), "+v"(sw2.x), "+v"(sw2.y), "+v"(sw2.z), "+v"(sw2.w), "+v"(sw3.x), "+v"(sw3.y),
                 "+v"(sw3.z), "+v"(sw3.w));
    asm volatile("" : "+v"(fw0.x), "+v"(fw0.y), "+v"(fw0.z), "+v"(fw0.w), "+v"(fw1.x), "+v"(fw1.y), "+v"(fw1.z),
                 "+v"(fw1.w), "+v"(fw2.x), "+v"(fw2.y), "+v"(fw2.z));
    const LinkState S = state_from_words(sw0, sw1, sw2, sw3);
    const LinkFwd F = fwd_from_words(fw0, fw1, fw2);
#if DREPHIP_LK_PHASES
    uint64_t ph0 = 0, ph1 = 0, ph2 = 0, ph3 = 0, ph4 = 0, ph5 = 0, ph6 = 0;
#endif
    LK_T(ph0);
    if (wave0) wave_argmin_upto3(g, g2, g3, S.pend || F.spec, F.spec != 0);
    LK_T(ph1);
    if (S.k >= (int32_t)n - 1) return;                         // all merged
    const bool w0 = blockIdx.x == 0;
    // size of cluster i as of the previous decision: workgroup 0 writes that
    // decision's two sizes during this kernel, so every reader overrides them
    const int32_t spsa = S.pend ? S.x : -1, spsb = S.pend ? S.y : -1, spsbsz = S.nx + S.ny;
    auto size_prev = [=](int32_t i, int32_t stored) { return i == spsa ? 0 : i == spsb ? spsbsz : stored; };
    if (w0 && threadIdx.x == 0 && S.pend) { size[S.x] = 0; size[S.y] = spsbsz; }
    // ---- the previous step's decision, and y's when it pushes y (replicated
    // in every workgroup; its stores by lane 0 of workgroup 0)
    const bool w0l = w0 && lane0;
    if (wave0) {
        // The partial minima as scalars: g .. g3 are per-lane values in the
        // other waves, so after the `if (wave0)` above the compiler held them
        // (and everything the decision derives from them) in VGPRs under exec
        // masks -- ~1,000 cycles of one wave's vector code per launch
        g = uni(g); g2 = uni(g2); g3 = uni(g3);
        // (plain scalars, the state struct written once at the end: a struct
        // updated across the branches was kept in private memory)
        int32_t k = S.k, len = S.len, top = S.top, below = S.below, first_active = S.first_active;
        int32_t pend = 0, px = S.x, py = S.y, pnx = S.nx, pny = S.ny, bad = S.flags & kLkBad, known = 0;
        const int32_t mrow = S.pend ? S.y : -1;                // the row the previous launch's merge formed
        // c3..c6: chain[len - 3] .. chain[len - 6]; the first ck of them are
        // known exactly (a merge exposes two entries only the chain in memory
        // holds; a push shifts known ones down)
        int32_t c3 = F.c3, c4 = F.c4, c5 = F.c5, c6 = F.c6, ck = 4, dpo = 0;
        double dpov = 0.0;
        // the decision's stores (Z row, chain pushes, a restart) are recorded
        // here and made by lane 0 of workgroup 0 after it: a lane-divergent
        // store inside the decision made the compiler keep the whole decision
        // in VGPRs under exec masks instead of scalar code
        int32_t zmerge = 0, za = 0, zb = 0, zn = 0, npush = 0, pp0 = 0, pv0 = 0, pp1 = 0, pv1 = 0, restart = -1;
        double zd = 0.0;
        auto push_rec = [&](int32_t pos, int32_t v) {
            if (npush == 0) { pp0 = pos; pv0 = v; } else { pp1 = pos; pv1 = v; }
            npush++;
        };
        if (S.flags & kLkDecide) {
            int32_t szt = F.szt, szb = F.szb;
            double dp = F.dp;
            MinIdx r = g;
            for (int d = 0; d < 2; d++) {
                // a known merge (spec 3) needs no search result: the previous
                // launch decided it and speculated on it
                const bool kn = d == 0 && S.known;
                if (!kn && (uint32_t)r.i >= n) { bad = kLkBad; k = (int32_t)n - 1; break; }   // no valid partial: stop
                if (kn || (len > 1 && !(r.v < dp))) {              // merge top with below at dp
                    int32_t a = top, b = below, na = szt, nb = szb;
                    if (a > b) { a = below; b = top; na = szb; nb = szt; }
                    zmerge = 1; za = a; zb = b; zd = dp; zn = na + nb;
                    pend = 1; px = a; py = b; pnx = na; pny = nb;
                    k = S.k + 1;
                    len -= 2;
                    top = c3;
                    below = len >= 2 ? c4 : -1;
                    c3 = c5; c4 = c6;                               // (ck is 4 at either merge: at d = 0,
                    ck = ck - 2;                                    // or after one push)
                    if (len == 0 && k < (int32_t)n - 1) {           // restart at the first active cluster
                        int32_t f = S.first_active;
                        // (the loaded size read into an SGPR: a VGPR load result in this loop
                        // made the compiler treat the whole decision as divergent)
                        while (f < (int32_t)n && !(f == b || (f != a && size_prev(f, rfl((uint32_t)size[f])) > 0))) f++;
                        if (f >= (int32_t)n) { bad = kLkBad; k = (int32_t)n - 1; }
                        else {
                            restart = f;
                            first_active = f; top = f; below = -1; len = 1;
                        }
                    } else if (d == 0 && F.spec && len >= 1 && k < (int32_t)n - 1) {
                        // the previous launch searched, speculatively, the new
                        // top w's row as it is after this merge (P3) and the
                        // merged row b (P2): decide w's step, and b's when w
                        // pushes b, now.  A push makes this launch search the
                        // pushed row instead of w.  A merge is left to the next
                        // launch (one merge per launch), which then knows it:
                        // this launch speculates on it (spec 3) instead of
                        // searching.  (b is pushed only together with b's own
                        // push, or as a known merge back with w: D[top][below]
                        // must not involve b, whose row this launch rewrites,
                        // except through dpo)
                        const MinIdx r3 = g3;
                        const bool r3ok = (uint32_t)r3.i < n;
                        const bool wmerge = r3ok && len > 1 && !(r3.v < F.dp2);
                        const bool wpush = r3ok && !wmerge && len + 1 < (int32_t)n;
                        const bool bpush = r3.i == b && (uint32_t)g2.i < n && g2.v < r3.v;
                        if (wpush && (r3.i != b || bpush)) {
                            push_rec(len, r3.i);                        // w pushes r3.i
                            c6 = c5; c5 = c4; c4 = c3; c3 = below; below = top; top = r3.i;
                            ck = ck >= 4 ? 4 : ck + 1;
                            len++;
                            LK_DIAG(specwin);
                            if (bpush) {
                                push_rec(len, g2.i);                    // b pushes g2.i
                                c6 = c5; c5 = c4; c4 = c3; c3 = below; below = top; top = g2.i;
                                ck = ck >= 4 ? 4 : ck + 1;
                                len++;
                                dpo = 1; dpov = g2.v;                   // D[g2.i][b] as this launch writes it
                            }
                        } else if (wmerge && spec_on > 1) {
                            known = 1;                                  // w merges with the element below it
                            LK_DIAG(wmerge);
                        } else if (wpush && r3.i == b && spec_on > 1) {
                            push_rec(len, b);                           // w pushes b, b merges back with w
                            c6 = c5; c5 = c4; c4 = c3; c3 = below; below = top; top = b;
                            ck = ck >= 4 ? 4 : ck + 1;
                            len++;
                            dpo = 1; dpov = r3.v;                       // D[b][w] as this launch writes it
                            known = 1;
                            LK_DIAG(recip);
                        }
                    }
                    break;
                }
                // push (scipy: the previous element wins ties)
                if (len >= (int32_t)n) { bad = kLkBad; k = (int32_t)n - 1; break; }
                push_rec(len, r.i);
                c6 = c5; c5 = c4; c4 = c3; c3 = below; below = top; top = r.i;
                ck = ck >= 4 ? 4 : ck + 1;
                dp = r.v;
                szb = szt;
                len++;
                if (r.i != mrow || mrow < 0 || d == 1) break;      // the pushed row is searched by this launch
                szt = spsbsz;                                       // y: just formed, its size is the override
                r = g2;                                             // y's minimum, from the merge step
                LK_DIAG(twice);
            }
        }
        LinkState X;
        X.mx = S.mx;
        X.k = k; X.len = len; X.top = top; X.below = below; X.first_active = first_active;
        X.pend = pend; X.x = px; X.y = py; X.nx = pnx; X.ny = pny;
        X.flags = kLkDecide | bad;
        X.launches = S.launches + 1;
        X.c3 = c3;
        X.known = known;
        X.spec = 0;
        if (known) {
            X.spec = 3;                                         // speculate on the known merge, no search
            LK_DIAG(known);
        } else if (spec_on && len >= 3 && k < (int32_t)n - 1) {
            if (!pend) X.spec = 1;                              // a search launch
            else if (below == py && top != py) X.spec = 2;      // a merge launch, its row y below the top
        }
#if DREPHIP_LK_DIAG
        if (!pend) LK_DIAG(scans);
        else if (!X.spec) LK_DIAG(m0);
#endif
        if (lane0) sx = X;
        LK_T(ph2);
        if (w0l) {
            if (zmerge) {
                double *z = Z + 4ull * S.k;
                z[0] = za; z[1] = zb; z[2] = zd; z[3] = zn;
            }
            if (restart >= 0) chain[0] = restart;
            if (npush > 0) chain[pp0] = pv0;
            if (npush > 1) chain[pp1] = pv1;
            st[q] = X;
            if (X.k >= (int32_t)n - 1) st[q ^ 1] = X;           // the finished state in both buffers
            *done = X.k;
        }
        if (blockIdx.x == G && X.k < (int32_t)n - 1) {
            // the next decision's operands, sizes as of this decision.  Every
            // load is issued before any is waited for (one round trip): the
            // chain entries read are below this launch's pushes, and a spec
            // launch (no merge) knows c3 and c4 (ck = 2), so D[c3][c4] needs none
            const bool two = len > 1, l3 = len >= 3 && ck < 1, l4 = len >= 4 && ck < 2, l5 = len >= 5 && ck < 3,
                       l6 = len >= 6 && ck < 4;
            // D[c3][c4], the speculation's decision operand: c3 and c4 are
            // known in every spec launch (ck >= 2: pushes, or a merge with
            // c5 and c6 forwarded)
            const bool sp = X.spec && len >= 4 && ck >= 2;
            int32_t rzt = size[top], rzb = size[two ? below : top];
            double rdp = D[(uint64_t)top * n + (two ? below : top)];
            int32_t r3 = chain[l3 ? len - 3 : 0], r4 = chain[l4 ? len - 4 : 0], r5 = chain[l5 ? len - 5 : 0],
                    r6 = chain[l6 ? len - 6 : 0];
            double rdp2 = D[sp ? (uint64_t)c3 * n + c4 : 0];
            asm volatile("" : "+v"(rzt), "+v"(rzb), "+v"(rdp), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(rdp2));
            LK_T(ph3);
            auto size_now = [&](int32_t i, int32_t stored) {
                return pend && i == px ? 0 : pend && i == py ? pnx + pny : size_prev(i, stored);
            };
            LinkFwd f{};
            f.szt = size_now(top, rzt);                         // (also at len 1: a push and a merge may follow)
            if (two) {
                f.dp = dpo ? dpov : rdp;
                f.szb = size_now(below, rzb);
            }
            if (len >= 3) f.c3 = ck >= 1 ? c3 : r3;
            if (len >= 4) f.c4 = ck >= 2 ? c4 : r4;
            if (len >= 5) f.c5 = ck >= 3 ? c5 : r5;
            if (len >= 6) f.c6 = ck >= 4 ? c6 : r6;
            if (X.spec) {
                f.dp2 = sp ? rdp2 : 0.0;                        // D[w][c4], w = c3
                f.spec = 1;
            }
            if (lane0) fwd[q] = f;
#if DREPHIP_LK_PHASES
            if (lane0) {
                uint64_t *ph = g_lk_ph + (uint64_t)(S.launches % kPhCap) * 16;
                ph[12] = ph0; ph[13] = ph1; ph[14] = ph2; ph[15] = ph3;
            }
#endif
        }
    }
    if (blockIdx.x == G) return;                               // the forwarding workgroup has no step work
    __syncthreads();
    // the decision as wave-uniform scalars (an LDS read lands in VGPRs, which
    // the compiler then treats as per-lane values: the pass's conditions became
    // exec-mask branches and its row addresses per-lane 64-bit arithmetic)
    LinkState X;
    {
        const uint4 *xv = (const uint4 *)&sx;
        const uint4 a = xv[0], b = xv[1], c = xv[2], d = xv[3];
        X = state_from_words(a, b, c, d);
    }
    LK_T(ph3);
    if (X.k >= (int32_t)n - 1) return;
    // ---- this step: the pending update of row y fused with the search of row
    // t (P1), and either y's new row (P2) or the speculation's rows (P2, P3)
    const bool pend = X.pend != 0;
    const int32_t x = X.x, y = X.y, nx = X.nx, ny = X.ny, t = X.top;
    const int spec = X.spec;
    const bool search = spec != 3, sp = spec != 0;
    // speculation rows: A = t, B = below, W = chain[len - 3] (spec 3 at len 2: no W)
    const int32_t A = t, B = X.below, W = X.c3;
    const bool hasW = sp && X.len >= 3;
    const bool yA = pend && A == y, yB = pend && B == y, yW = pend && W == y;
    const int32_t ys = A < B ? B : A;                          // the speculated merge's row index, max(A, B)
    const double *Dx = D + (uint64_t)x * n;
    double *Dy = D + (uint64_t)y * n;
    const double *Da = D + (uint64_t)(yA ? 0 : A) * n;
    const double *Db = D + (uint64_t)(sp && !yB ? B : 0) * n;
    const double *Dw = D + (uint64_t)(hasW && !yW ? W : 0) * n;
    // entry y of the rows read (as after this launch's merge): U1[R] =
    // LW(D[x][R], D[y][R]), from uniform loads, used by the lane of i = y.
    // (Through a lane register offset: a uniform address made them scalar
    // loads, which the compiler waited for before the pass.)
    int32_t lz;
    asm volatile("v_mov_b32 %0, 0" : "=v"(lz));
    adverse_delay();
    const bool fa = pend && !yA, fb = pend && sp && !yB, fw = pend && hasW && !yW;
    // (entry (y, R) from its column copy D[R][y], which only the lane of i = y
    // writes in this launch, after this load: the row copy D[y][R] is the lane
    // of i = R's to rewrite -- reading it here raced with that store)
#if DREPHIP_LK_RACE_REPRO
    // (test build only: the round-5 race reintroduced -- entry (y, R) from the
    // row copy D[y][R], which the lane of i = R rewrites in this launch; the
    // adverse-order test must catch it)
    auto colY = [&](int32_t r) { return D[(uint64_t)y * n + r + lz]; };
#else
    auto colY = [&](int32_t r) { return D[(uint64_t)r * n + y + lz]; };
#endif
    double xa = fa ? Dx[A + lz] : 0.0, ya_ = fa ? colY(A) : 0.0;
    double xb = fb ? Dx[B + lz] : 0.0, yb = fb ? colY(B) : 0.0;
    double xw = fw ? Dx[W + lz] : 0.0, yw = fw ? colY(W) : 0.0;
    // the sizes of A and B as of this step's decision (for the speculated merge)
    int32_t rsa = sp ? size[A + lz] : 0, rsb = sp ? size[B + lz] : 0;
    // (as selects: the nested conditional form compiled to exec-mask branches)
    auto size_x = [&](int32_t i, int32_t stored) {
        int32_t s = i == spsb ? spsbsz : stored;               // size_prev
        s = i == spsa ? 0 : s;
        if (pend) {
            s = i == y ? nx + ny : s;
            s = i == x ? 0 : s;
        }
        return s;
    };
    double cay = 0.0, cby = 0.0, cwy = 0.0;                     // the y lane's entries U1[A], U1[B], U1[W]
    double bv = INFINITY, yv = INFINITY, wv = INFINITY;
    int32_t bi = 0x7fffffff, yi = 0x7fffffff, wi = 0x7fffffff;
    int32_t sxs = 0, sys = 0;                                   // the speculated merge's sizes
    LwDiv dvxy = lw_div(nx, ny);                                // (average: this step's divisor)
    LwDiv dvs{1.0, 1.0};
    const uint32_t stride = G * WG;
    bool first = true;
    for (uint32_t i0 = blockIdx.x * WG + threadIdx.x; i0 < n; i0 += kLkPer * stride) {
        int32_t sz[kLkPer];
        double da[kLkPer], dx[kLkPer], dy[kLkPer], dw[kLkPer], db[kLkPer];
#pragma unroll
        for (int k = 0; k < kLkPer; k++) {
            const uint32_t i = i0 + k * stride;
            const uint32_t ic = i < n ? i : n - 1;
            sz[k] = size[ic];
            if (!yA) da[k] = Da[ic];
            if (pend) { dx[k] = Dx[ic]; dy[k] = Dy[ic]; }
            if (sp && !yB) db[k] = Db[ic];
            if (hasW && !yW) dw[k] = Dw[ic];
        }
        // the divisor's reciprocal while the loads are in flight (the compiler
        // had sunk its IEEE division below the wait for them)
        if (method == DREPHIP_LINK_AVERAGE && pend) asm volatile("" : "+v"(dvxy.n), "+v"(dvxy.r));
        // every load of the pass in flight before any is waited for: left to
        // itself the compiler sank the row loads below the size test that
        // uses size[i] (a second round trip per step), and waited for the
        // uniform loads before the pass
#pragma unroll
        for (int k = 0; k < kLkPer; k++) {
            asm volatile("" : "+v"(sz[k]));
            if (!yA) asm volatile("" : "+v"(da[k]));
            if (pend) asm volatile("" : "+v"(dx[k]), "+v"(dy[k]));
            if (sp && !yB) asm volatile("" : "+v"(db[k]));
            if (hasW && !yW) asm volatile("" : "+v"(dw[k]));
        }
        LK_T(ph4);
        if (first) {
            first = false;
            asm volatile("" : "+v"(xa), "+v"(ya_), "+v"(xb), "+v"(yb), "+v"(xw), "+v"(yw), "+v"(rsa), "+v"(rsb));
            if (sp) {
                const int32_t sa = size_x(A, rsa), sb_ = size_x(B, rsb);
                sxs = A < B ? sa : sb_;
                sys = A < B ? sb_ : sa;
                dvs = lw_div(sxs, sys);
            }
            // (the same bits as those lanes' u: the same operands and update)
            if (fa) cay = lw_update(method, xa, ya_, nx, ny, dvxy);
            if (fb) cby = lw_update(method, xb, yb, nx, ny, dvxy);
            if (fw) cwy = lw_update(method, xw, yw, nx, ny, dvxy);
        }
#pragma unroll
        for (int k = 0; k < kLkPer; k++) {
            const int32_t i = (int32_t)(i0 + k * stride);
            // the sizes as of this step's decision: the previous decision's
            // (being written by workgroup 0) and this one's (not yet written).
            // Written as selects on `live` rather than `continue`s and nested
            // ifs: the branchy form compiled to a cascade of exec-mask branches
            // (~half the pass's instructions at one wave per SIMD)
            const bool live = i < (int32_t)n && size_x(i, sz[k]) != 0;   // (retires x)
            const bool isy = pend && i == y;
            // this launch's merge: row y's new value at i, stored to row and column y
            // (one entry's two copies, D[y][i] and D[i][y])
            auto store_row = [&](int32_t c, double v) {
#if DREPHIP_LK_ROWSTORE == 3
                __hip_atomic_store(&Dy[c], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
                Dy[c] = v;
#endif
            };
            auto store_col = [&](int32_t c, double v) {
#if DREPHIP_LK_COLSTORE == 0
                // timing-only A/B build: no column-y stores (Z is wrong)
#elif DREPHIP_LK_COLSTORE == 2
                __builtin_nontemporal_store(v, &D[(uint64_t)c * n + y]);
#elif DREPHIP_LK_COLSTORE == 3
                // write-through (sc1): the line leaves L2 now instead of at the kernel boundary
                __hip_atomic_store(&D[(uint64_t)c * n + y], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
                D[(uint64_t)c * n + y] = v;
#endif
            };
            double u = 0.0;
            if (pend) {
                u = lw_update(method, dx[k], dy[k], nx, ny, dvxy);
                if (live && !isy) {
                    store_row(i, u);
                    // the column copy D[R][y] of the rows R = A, B, W whose entry y the
                    // lane of i = y recomputes (U1[R], from D[x][R] and D[R][y]) is that
                    // lane's to store, after its load of it
                    if (!((fa && i == A) || (fb && i == B) || (fw && i == W))) store_col(i, u);
                }
                if (isy) {
                    if (fa) store_col(A, cay);
                    if (fb) store_col(B, cby);
                    if (fw) store_col(W, cwy);
                }
            }
            // the rows as they are after that merge: row y is u; entry y of a
            // row R is U1[R]
            double ca = yA ? u : da[k];
            double cb = sp ? (yB ? u : db[k]) : 0.0;
            double cw = hasW ? (yW ? u : dw[k]) : 0.0;
            if (pend) {
                ca = isy ? cay : ca;
                cb = isy ? cby : cb;
                cw = isy ? cwy : cw;
            }
            // (a lane visits its entries in increasing i, so a candidate at i
            // beats an earlier one only when strictly smaller -- except P3's
            // entry for W, which carries index ys: there the full rule)
            if (search) {                                                // P1: the top's row
                const bool lt = live & (i != t) & (ca < bv);
                bv = lt ? ca : bv;
                bi = lt ? i : bi;
            }
            if (sp) {
                // P2: the speculated merged row; P3: W's row after that merge
                const bool ok = live & (i != A) & (i != B);
                const double U = lw_update(method, A < B ? ca : cb, A < B ? cb : ca, sxs, sys, dvs);
                const bool y_lt = ok & (U < yv);
                yv = y_lt ? U : yv;
                yi = y_lt ? i : yi;
                if (hasW) {
                    const bool isW = i == W;
                    const double cv = isW ? U : cw;
                    const int32_t ci = isW ? ys : i;
                    const bool w_lt = ok & ((cv < wv) | ((cv == wv) & (ci < wi)));
                    wv = w_lt ? cv : wv;
                    wi = w_lt ? ci : wi;
                }
            } else if (pend) {                                           // P2: y's new row
                const bool lt = live & !isy & (u < yv);
                yv = lt ? u : yv;
                yi = lt ? i : yi;
            }
        }
    }
    LK_T(ph5);
    MinIdx p1{bv, bi}, p2{yv, yi}, p3{wv, wi};
#if DREPHIP_LK_WAVEPARTS
    wave_argmin_upto3(p1, p2, p3, pend || sp, hasW);
    const uint32_t pslot = blockIdx.x * (WG / 64) + (threadIdx.x >> 6);
    const bool pwrite = (threadIdx.x & 63) == 0;
#else
    block_argmin3<WG>(p1, p2, p3, pend || sp, hasW);
    const uint32_t pslot = blockIdx.x;
    const bool pwrite = threadIdx.x == 0;
#endif
    LK_T(ph6);
#if DREPHIP_LK_PHASES
    if (threadIdx.x == 0 && (blockIdx.x == 0 || blockIdx.x == G - 1)) {
        uint64_t *ph = g_lk_ph + (uint64_t)(S.launches % kPhCap) * 16;
        if (blockIdx.x == 0) { ph[0] = ph0; ph[1] = ph1; ph[2] = ph2; ph[3] = ph3; ph[4] = ph4; ph[5] = ph5; ph[6] = ph6; }
        else { ph[8] = ph0; ph[9] = ph3; ph[10] = ph6; }
    }
#endif
    if (pwrite) {
        PartRec *pr = parts + (uint64_t)q * kLkPartStride + pslot;
        if (search) pr->p1 = p1;
        if (pend || sp) pr->p2 = p2;
        if (hasW) pr->p3 = p3;
    }
}

template <int WG, int kLkPer>
__global__ __launch_bounds__(WG) void k_mst_step(const double *__restrict__ D, uint32_t n,
                                                    int32_t *__restrict__ merged, double *__restrict__ Dmin,
                                                    LinkState *__restrict__ st, MinIdx *__restrict__ parts,
                                                    int32_t *__restrict__ done, double *__restrict__ Z, uint32_t q) {
    // (the state as scalars: a LinkState copied and edited in branches was
    // kept in private memory promoted to LDS, see k_nn_step)
    __shared__ int32_t s_k, s_mx, s_ov;
    const uint32_t G = gridDim.x;
    const MinIdx g = read_partials<WG>(parts + (uint64_t)(q ^ 1) * kLkPartStride, G);     // unconditional: not held behind S
    const int32_t sk = st[q ^ 1].k, smx = st[q ^ 1].mx, sflags = st[q ^ 1].flags;
    if (sk >= (int32_t)n - 1) return;
    if (threadIdx.x == 0) {
        int32_t k = sk, mx = smx, bad = sflags & kLkBad, ov = -1;
        const bool w0 = blockIdx.x == 0;
        if (sflags & kLkDecide) {
            if ((uint32_t)g.i >= n) { bad = kLkBad; k = (int32_t)n - 1; }
            else {
                if (w0) {
                    double *z = Z + 4ull * sk;
                    z[0] = smx; z[1] = g.i; z[2] = g.v; z[3] = 0;
                    merged[g.i] = 1;
                }
                ov = g.i;
                mx = g.i;
                k = sk + 1;
            }
        }
        s_k = k; s_mx = mx; s_ov = ov;
        if (w0) {
            st[q].k = k; st[q].mx = mx; st[q].flags = kLkDecide | bad;
            if (k >= (int32_t)n - 1) { st[q ^ 1].k = k; st[q ^ 1].mx = mx; st[q ^ 1].flags = kLkDecide | bad; }
            *done = k;
        }
    }
    __syncthreads();
    if (s_k >= (int32_t)n - 1) return;
    adverse_delay();
    const int32_t ov = s_ov, x = s_mx;
    const double *Dx = D + (uint64_t)x * n;
    double bv = INFINITY;
    int32_t bi = 0x7fffffff;
    const uint32_t stride = G * WG;
    for (uint32_t i0 = blockIdx.x * WG + threadIdx.x; i0 < n; i0 += kLkPer * stride) {
        int32_t mg[kLkPer];
        double dx[kLkPer], dm[kLkPer];
#pragma unroll
        for (int k = 0; k < kLkPer; k++) {
            const uint32_t i = i0 + k * stride;
            const uint32_t ic = i < n ? i : n - 1;
            mg[k] = merged[ic];
            dx[k] = Dx[ic];
            dm[k] = Dmin[ic];
        }
#pragma unroll
        for (int k = 0; k < kLkPer; k++) {
            const uint32_t i = i0 + k * stride;
            if (i >= n || mg[k] || (int32_t)i == ov) continue;
            double m = dm[k];
            if (m > dx[k]) { m = dx[k]; Dmin[i] = m; }
            if (m < bv) { bv = m; bi = (int32_t)i; }
        }
    }
    const MinIdx part = block_argmin<WG>(bv, bi);
    if (threadIdx.x == 0) parts[(uint64_t)q * kLkPartStride + blockIdx.x] = part;
}

// ------------------------------------------------------------ compaction
// Round 5: the matrix follows the active clusters.  A merge retires a row and
// column for good, but the step kernels keep reading full n-long rows (and
// size[] entries) of the original n x n matrix, so at 10^5 the second half of
// the chain pays 10^5-entry rows for <= 5 x 10^4 clusters.  Between graph
// replays, once at most half of the matrix's rows are active, the active rows
// and columns are moved to the front as an m x m matrix (stride m) in the same
// allocation, in index order, and the chain's state is renumbered: scipy's
// decisions depend only on the distances and on the ORDER of indices (ties:
// the previous chain element, then the lowest index), which an order-keeping
// renumbering preserves, so Z in local numbers maps back to the same rows.
// The step grid is then chosen for m (fewer entries per lane, narrower
// workgroups: 7.0 us per launch at 10^5, 6.3 at 5 x 10^4, 5.9 at 2.5 x 10^4).
//
// At a replay boundary the last launch has decided and applied a merge (x, y)
// whose two sizes are still to be written by the next launch (state buffer 1,
// pend): x counts as retired and y as merged here; x's number becomes m (a
// dummy slot of the new size array, which the next launch writes 0 to).
constexpr uint32_t kCmpWG = 1024;
__device__ __forceinline__ int32_t cmp_size(const LinkState &S, const int32_t *size, uint32_t i) {
    return S.pend && (int32_t)i == S.x ? 0 : S.pend && (int32_t)i == S.y ? S.nx + S.ny : size[i];
}
// one workgroup: rank[i] = active clusters below i (rank[m] = their count),
// the new sizes and the new -> old map
__global__ __launch_bounds__(kCmpWG) void k_lk_cmp_rank(const int32_t *__restrict__ size, const LinkState *__restrict__ st,
                                                        uint32_t m, uint32_t *__restrict__ rank,
                                                        int32_t *__restrict__ size2, int32_t *__restrict__ orig) {
    __shared__ uint32_t sc[kCmpWG];
    const LinkState S = st[1];
    const uint32_t per = (m + kCmpWG - 1) / kCmpWG, b0 = min(m, threadIdx.x * per), b1 = min(m, b0 + per);
    uint32_t c = 0;
    for (uint32_t i = b0; i < b1; i++) c += cmp_size(S, size, i) > 0;
    sc[threadIdx.x] = c;
    __syncthreads();
    for (uint32_t o = 1; o < kCmpWG; o <<= 1) {                 // inclusive scan of the counts
        const uint32_t v = threadIdx.x >= o ? sc[threadIdx.x - o] : 0;
        __syncthreads();
        sc[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t r = sc[threadIdx.x] - c;
    for (uint32_t i = b0; i < b1; i++) {
        rank[i] = r;
        const int32_t e = cmp_size(S, size, i);
        if (e > 0) { size2[r] = e; orig[r] = (int32_t)i; r++; }
    }
    if (threadIdx.x == kCmpWG - 1) rank[m] = sc[kCmpWG - 1];
}
// one workgroup of 256: the state, the forwarded operands, the chain and the
// last launch's partial sets renumbered; each partial set reduced to its
// minimum in slot 0 (the next launch's grid reads np_new slots), the rest
// empty.  Indices outside [0, m) (-1, INT_MAX) are kept.
__global__ __launch_bounds__(256) void k_lk_cmp_state(LinkState *__restrict__ st, LinkFwd *__restrict__ fwd,
                                                      PartRec *__restrict__ parts, int32_t *__restrict__ chain,
                                                      const uint32_t *__restrict__ rank, uint32_t m, uint32_t np_old,
                                                      uint32_t np_new, int32_t *__restrict__ size2,
                                                      int32_t *__restrict__ done) {
    const LinkState S = st[1];
    const uint32_t mn = rank[m];
    auto tr = [&](int32_t v) { return v >= 0 && (uint32_t)v < m ? (int32_t)rank[v] : v; };
    PartRec *P = parts + kLkPartStride;
    MinIdx a{INFINITY, 0x7fffffff}, b = a, c = a;
    for (uint32_t s = threadIdx.x; s < np_old; s += 256) {
        const PartRec r = P[s];
        if (better(r.p1.v, r.p1.i, a.v, a.i)) a = r.p1;
        if (better(r.p2.v, r.p2.i, b.v, b.i)) b = r.p2;
        if (better(r.p3.v, r.p3.i, c.v, c.i)) c = r.p3;
    }
    block_argmin3<256>(a, b, c, true, true);                   // (every slot read before the barrier in it)
    const MinIdx none{INFINITY, 0x7fffffff};
    for (uint32_t s = threadIdx.x; s < np_new; s += 256)
        if (s) P[s] = PartRec{none, none, none};
    for (int32_t p = threadIdx.x; p < S.len; p += 256) chain[p] = tr(chain[p]);
    __syncthreads();                                            // (every read of st[1] before its rewrite)
    if (threadIdx.x == 0) {
        P[0] = PartRec{MinIdx{a.v, tr(a.i)}, MinIdx{b.v, tr(b.i)}, MinIdx{c.v, tr(c.i)}};
        LinkState X = S;
        X.k = S.k - (int32_t)(m - mn);                          // 0: the new epoch's merges count from here
        X.top = tr(S.top); X.below = tr(S.below); X.first_active = tr(S.first_active); X.c3 = tr(S.c3);
        if (S.pend) { X.x = (int32_t)mn; X.y = tr(S.y); }
        st[1] = X;
        LinkFwd F = fwd[1];
        F.c3 = tr(F.c3); F.c4 = tr(F.c4); F.c5 = tr(F.c5); F.c6 = tr(F.c6);
        fwd[1] = F;
        size2[mn] = 0;                                          // the retired x's dummy slot
        *done = X.k;
    }
}
// new rows [r0, r1) (stride sn) of the active rows and columns of the old
// matrix (stride so), written at dst row r - d0.  In place (src == dst) for a
// chunk with r1 <= 2 r0 when sn <= so / 2: its writes end below r1 sn <= r0 so,
// i.e. they only cover old rows below r0, which only new rows below r0 read
// (orig[r] >= r) -- earlier chunks, finished (stream order).  The first rows
// go through a scratch buffer (row 0 overlaps itself).
__global__ __launch_bounds__(256) void k_lk_cmp_rows(const double *src, uint32_t so, double *dst, uint32_t sn,
                                                     const int32_t *__restrict__ orig, uint32_t r0, uint32_t r1,
                                                     uint32_t d0) {
    adverse_delay();
    const uint32_t nb = (sn + 1023) / 1024;
    const uint64_t items = (uint64_t)(r1 - r0) * nb;
    for (uint64_t it = blockIdx.x; it < items; it += gridDim.x) {
        const uint32_t r = r0 + (uint32_t)(it / nb), c0 = (uint32_t)(it % nb) * 1024 + threadIdx.x;
        const double *s = src + (uint64_t)orig[r] * so;
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t c = c0 + 256u * u;
            v[u] = c < sn ? s[orig[c]] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t c = c0 + 256u * u;
            if (c < sn) dst[(uint64_t)(r - d0) * sn + c] = v[u];
        }
    }
}

// ------------------------------------------------------------ matrix build
// D (n x n f64, rows in perm order) from the condensed upper triangle, by
// 64 x 64 tiles of (row block bi <= column block bj): a wave reads one row's
// 64 condensed values (contiguous in j) and writes D[p(i)][p(j)] -- a
// contiguous 512-byte row piece when perm is the identity (file order =
// sorted-name order, the usual case) -- and stages them in LDS; after the
// barrier the tile is written transposed, D[p(j)][p(i)], again a row piece per
// wave.  One workgroup per row would write the transposed half one 8-byte
// element per row (~8x the HBM write traffic: 145 ms for the 80 GB matrix at
// n = 10^5).  Tiles are numbered row-major over the upper triangle, diagonal
// tiles included; the diagonal entries are 0.
constexpr uint32_t kDmT = 64;

// value of condensed pair t: the reference's float64 distance from the
// all-pairs counts (lut[off[denom] + common], denom = s when null); a pair
// whose denominator has no table (off < 0) or whose count exceeds it sets
// *bad and gets NaN (the host then refuses the result)
struct DmFromCounts {
    const uint16_t *common, *denom;
    uint32_t s;
    const double *lut;
    const int32_t *off;
    uint32_t *bad;
    // R values at once (t[q] a valid index even where ok[q] is false): each
    // of the three dependent lookups -- counts, the denominator's table
    // offset, the table -- issued for all R before the next
    template <int R>
    __device__ __forceinline__ void batch(const uint64_t (&t)[R], const bool (&ok)[R], double (&out)[R]) const {
        uint32_t dn[R], cm[R];
        int32_t o[R];
#pragma unroll
        for (int q = 0; q < R; q++) {
            dn[q] = denom ? denom[t[q]] : s;
            cm[q] = common[t[q]];
        }
#pragma unroll
        for (int q = 0; q < R; q++) o[q] = off[dn[q] <= s ? dn[q] : 0];
        bool anybad = false;
#pragma unroll
        for (int q = 0; q < R; q++) {
            const bool good = (dn[q] <= s) & (o[q] >= 0) & (cm[q] <= dn[q]);
            const double x = lut[good ? o[q] + cm[q] : 0];
            out[q] = good ? x : __builtin_nan("");
            anybad |= ok[q] & !good;
        }
        if (anybad) atomicOr(bad, 1u);
    }
};
struct DmFromCondensed {
    const double *y;
    template <int R>
    __device__ __forceinline__ void batch(const uint64_t (&t)[R], const bool (&)[R], double (&out)[R]) const {
#pragma unroll
        for (int q = 0; q < R; q++) out[q] = y[t[q]];
    }
};

// (row block, column block) of upper-triangle tile L (row-major, diagonal included)
__device__ __forceinline__ void dm_tile(uint64_t L, uint32_t nb, uint32_t &bi, uint32_t &bj) {
    // first tile of row block b: S(b) = b nb - b (b - 1) / 2
    const double B = 2.0 * nb + 1.0;
    int64_t b = (int64_t)((B - sqrt(B * B - 8.0 * (double)L)) * 0.5);
    if (b < 0) b = 0;
    if (b > (int64_t)nb - 1) b = nb - 1;
    auto S = [&](int64_t r) { return (uint64_t)(r * (int64_t)nb - r * (r - 1) / 2); };
    while (b > 0 && S(b) > L) b--;
    while (b + 1 < (int64_t)nb && S(b + 1) <= L) b++;
    bi = (uint32_t)b;
    bj = (uint32_t)(bi + (L - S(b)));
}

template <class V>
__global__ __launch_bounds__(256) void k_dist_tiles(V val, uint32_t n, uint32_t nb, const uint32_t *__restrict__ perm,
                                                    double *__restrict__ D) {
    __shared__ double tile[kDmT][kDmT + 1];          // +1: the transposed read walks banks 2 apart
    uint32_t bi, bj;
    dm_tile(blockIdx.x, nb, bi, bj);
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t i0 = bi * kDmT, j0 = bj * kDmT;
    // a wave's R rows: every value looked up before any store (a store between
    // two rows held each row's three dependent lookups behind the previous
    // row's: 42 ms for the 80 GB matrix at n = 10^5 as a row-at-a-time loop)
    constexpr int R = kDmT / 4;
    const uint32_t j = j0 + lane;
    uint64_t ti[R];
    bool ok[R];
    uint32_t pi[R];
#pragma unroll
    for (int q = 0; q < R; q++) {
        const uint32_t i = i0 + w + 4 * q;
        ok[q] = i < n && j < n && j > i;
        ti[q] = ok[q] ? (uint64_t)i * n - (uint64_t)i * (i + 1) / 2 + (j - i - 1) : 0;
        pi[q] = perm ? perm[i < n ? i : 0] : i;
    }
    const uint32_t pj = perm ? perm[j < n ? j : 0] : j;
    double v[R];
    val.template batch<R>(ti, ok, v);
#pragma unroll
    for (int q = 0; q < R; q++) {
        const uint32_t r = w + 4 * q, i = i0 + r;
        if (ok[q]) {
            tile[r][lane] = v[q];
            D[(uint64_t)pi[q] * n + pj] = v[q];
        } else if (j == i && i < n) {
            D[(uint64_t)pi[q] * n + pi[q]] = 0.0;
        }
    }
    __syncthreads();
    for (uint32_t c = w; c < kDmT; c += 4) {
        const uint32_t jj = j0 + c, i = i0 + lane;
        if (jj >= n) break;
        if (jj > i) D[(uint64_t)(perm ? perm[jj] : jj) * n + (perm ? perm[i] : i)] = tile[lane][c];
    }
}

// The linkage input from the pivot's n x n float32 matrix M (host copy in
// HBM), with squareform's and linkage's checks (d_cluster.py:445-453): tile
// (bi <= bj) holds M's upper tile U = M[i0..][j0..] and its mirror
// W = M[j0..][i0..]; U[r][c] must equal W[c][r] (==: NaN never does, +0 and
// -0 do), the diagonal must be 0 and the upper triangle finite.  Both halves
// of D take the upper value, as squareform keeps only X[i][j], i < j.
// bad: bit 0 asymmetric, 1 diagonal, 2 non-finite.  HBM-bound: 4 B read and
// 8 B written per cell.
__global__ __launch_bounds__(256) void k_square_tiles(const float *__restrict__ M, uint32_t n, uint32_t nb,
                                                      double *__restrict__ D, uint32_t *__restrict__ bad) {
    __shared__ float U[kDmT][kDmT + 1], W[kDmT][kDmT + 1];
    uint32_t bi, bj;
    dm_tile(blockIdx.x, nb, bi, bj);
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t i0 = bi * kDmT, j0 = bj * kDmT;
    for (uint32_t r = w; r < kDmT; r += 4) {
        const uint32_t i = i0 + r, j = j0 + r, c = lane;
        U[r][c] = i < n && j0 + c < n ? M[(uint64_t)i * n + j0 + c] : 0.0f;
        W[r][c] = j < n && i0 + c < n ? M[(uint64_t)j * n + i0 + c] : 0.0f;
    }
    __syncthreads();
    uint32_t flags = 0;
    for (uint32_t r = w; r < kDmT; r += 4) {              // row i of the upper tile, column j = lane
        const uint32_t i = i0 + r, j = j0 + lane;
        if (i >= n || j >= n || j < i) continue;
        const float a = U[r][lane], b = W[lane][r];       // M[i][j], M[j][i]
        if (!(a == b)) flags |= 1;
        if (j == i) {
            if (!(a == 0.0f)) flags |= 2;
            D[(uint64_t)i * n + i] = 0.0;
        } else {
            if (!isfinite(a)) flags |= 4;
            D[(uint64_t)i * n + j] = (double)a;
        }
    }
    for (uint32_t c = w; c < kDmT; c += 4) {              // the lower half: row j = j0 + c, column i = i0 + lane
        const uint32_t j = j0 + c, i = i0 + lane;
        if (j >= n || i >= n || j <= i) continue;
        D[(uint64_t)j * n + i] = (double)U[lane][c];
    }
    if (flags) atomicOr(bad, flags);
}

static void launch_dist_tiles_counts(const DmFromCounts &v, uint32_t n, const uint32_t *perm, double *D, hipStream_t st) {
    const uint32_t nb = (n + kDmT - 1) / kDmT;
    hipLaunchKernelGGL((k_dist_tiles<DmFromCounts>), dim3((uint32_t)((uint64_t)nb * (nb + 1) / 2)), dim3(256), 0, st,
                       v, n, nb, perm, D);
}
static void launch_dist_tiles_condensed(const DmFromCondensed &v, uint32_t n, double *D, hipStream_t st) {
    const uint32_t nb = (n + kDmT - 1) / kDmT;
    hipLaunchKernelGGL((k_dist_tiles<DmFromCondensed>), dim3((uint32_t)((uint64_t)nb * (nb + 1) / 2)), dim3(256), 0,
                       st, v, n, nb, (const uint32_t *)nullptr, D);
}

// ------------------------------------------------------------- host driver
// (sort_and_label: linkage_sparse.cpp, shared with the sparse path)
struct NnArgs {
    double *D; uint32_t n; int32_t *size, *chain; LinkCtl *ctl;
    PartRec *parts; double *Z; uint32_t q; int spec_on;
};
template <int W, int P>
static void launch_nn(int method, dim3 grid, dim3 blk, hipStream_t st, const NnArgs &a) {
#define DREPHIP_LK_NN(M) hipLaunchKernelGGL((k_nn_step<W, P, M>), grid, blk, 0, st, a.D, a.n, a.size, a.chain, a.ctl, \
                                            a.parts, a.Z, a.q, a.spec_on)
    if (method == DREPHIP_LINK_COMPLETE) DREPHIP_LK_NN(DREPHIP_LINK_COMPLETE);
    else if (method == DREPHIP_LINK_WEIGHTED) DREPHIP_LK_NN(DREPHIP_LINK_WEIGHTED);
    else DREPHIP_LK_NN(DREPHIP_LINK_AVERAGE);
#undef DREPHIP_LK_NN
}
int linkage_device_impl(drephip_ctx *ctx, double *d_D, uint32_t n, int method, double *Z_out, hipStream_t st) {
    if (n < 2) return DREPHIP_OK;
    const double t_chain = now_s();           // chain_s: scratch, graph capture and the steps
    if (method != DREPHIP_LINK_SINGLE && method != DREPHIP_LINK_COMPLETE && method != DREPHIP_LINK_AVERAGE &&
        method != DREPHIP_LINK_WEIGHTED) {
        set_error("linkage method must be single, complete, average or weighted");
        return DREPHIP_ERR_UNSUPPORTED;
    }
    // entries per lane of a step, i.e. the grid density: ~200 workgroups at
    // most (n = 10^5: 2 per lane, 1.76 s of chain against 1.91 s at 4 and
    // 1.89 s at 1; n = 10^4: 1 per lane, 40 workgroups, 158 ms against 176 ms
    // at 4 -- profiles/r03_linkage_grid_density.txt).  DREPHIP_LINK_PER_LANE
    // overrides it (the tests cover 1, 4 and 16: several passes)
    const char *pl = getenv("DREPHIP_LINK_PER_LANE");
    const char *tg = getenv("DREPHIP_LINK_TARGET_WG");                 // A/B runs only
    const uint32_t kLkTarget = tg ? std::max(1, atoi(tg)) : 200;
    // One-wave step workgroups (no LDS broadcast, no block reduction) with one
    // entry per lane up to n = kLkWaveN (<= 256 workgroups: the decision's wave
    // reduces <= 4 partials a lane): 70.9 vs 75.2 ms of chain at 10^4.  With
    // more entries per lane they lose (10^5: 1.21-1.41 s against 1.00 s for
    // 256-lane workgroups at 2 per lane; profiles/r04_linkage_wg64_ab.txt).
    // DREPHIP_LINK_WG = 64 / 128 / 256 forces the choice (A/B); a per-lane
    // override keeps the 128/256-lane kernels unless 64 is asked for.  Not for
    // single linkage (k_mst_step).
    constexpr uint32_t kLkWaveN = 16384;
    const char *wge = getenv("DREPHIP_LINK_WG");
    const int wreq = wge ? atoi(wge) : 0;
    struct StepCfg { uint32_t wg, grid; int tpl; };
    // (a function of the matrix's current size m: the compaction below shrinks it)
    auto cfg_for = [&](uint32_t m) {
        const bool wave_wg = method != DREPHIP_LINK_SINGLE && (wreq == 64 || (wreq == 0 && !pl && m <= kLkWaveN));
        const uint32_t wsz = wave_wg ? 64 : wreq == 512 && method != DREPHIP_LINK_SINGLE ? 512 : kLkWG;
        const uint32_t per = pl ? std::max(1, std::min(64, atoi(pl)))
                                : std::max(1u, (m + wsz * kLkTarget - 1) / (wsz * kLkTarget));
        StepCfg c;
        c.wg = wave_wg ? 64 : wreq == 128 || wreq == 256 || (wreq == 512 && method != DREPHIP_LINK_SINGLE)
                                  ? (uint32_t)wreq : m <= kLkSmallN && !pl ? 128 : kLkWG;
        c.grid = std::max(1u, std::min(1024u, (m + c.wg * per - 1) / (c.wg * per)));
        c.tpl = per <= 1 ? 1 : per <= 2 ? 2 : per <= 4 || !wave_wg ? 4 : 8;     // entries per lane per pass
        return c;
    };
    StepCfg cfg = cfg_for(n);
    int32_t *d_size, *d_chain, *d_done;
    double *d_Z, *d_Dmin;
    LinkState *d_st;
    MinIdx *d_parts;
    int rc;
    if ((rc = scratch(ctx, "lk_size", n * 4ull, (void **)&d_size))) return rc;
    if ((rc = scratch(ctx, "lk_chain", n * 4ull, (void **)&d_chain))) return rc;
    if ((rc = scratch(ctx, "lk_Z", (n - 1) * 32ull, (void **)&d_Z))) return rc;
    if ((rc = scratch(ctx, "lk_parts", 2 * kLkPartStride * sizeof(MinIdx), (void **)&d_parts))) return rc;
    PartRec *d_prec;                                 // the chain steps' partial records (d_parts: MST's)
    if ((rc = scratch(ctx, "lk_prec", 2 * kLkPartStride * sizeof(PartRec), (void **)&d_prec))) return rc;
    // the speculation (A/B): 0 off; 1 the round-4 protocol (no known-merge
    // launches); 2 (default) with the known-merge speculation (spec 3)
    const char *spe = getenv("DREPHIP_LINK_SPEC");
    const int spec_on = spe ? std::max(0, std::min(2, atoi(spe))) : 2;
    LinkCtl *d_ctl;
    if ((rc = scratch(ctx, "lk_ctl", sizeof(LinkCtl), (void **)&d_ctl))) return rc;
    d_st = d_ctl->st;                               // (device addresses inside the block)
    LinkFwd *d_fwd = d_ctl->fwd;
    d_done = &d_ctl->done;
    HIPC(hipMemsetAsync(d_fwd, 0, 2 * sizeof(LinkFwd), st));
    const bool mst = method == DREPHIP_LINK_SINGLE;
    if (mst && (rc = scratch(ctx, "lk_dmin", n * 8ull, (void **)&d_Dmin))) return rc;
    if (mst) {
        std::vector<double> inf(n, INFINITY);
        std::vector<int32_t> mg(n, 0);
        mg[0] = 1;                                            // scipy: x = 0, merged[x] = 1
        HIPC(hipMemcpyAsync(d_size, mg.data(), n * 4ull, hipMemcpyHostToDevice, st));
        HIPC(hipMemcpyAsync(d_Dmin, inf.data(), n * 8ull, hipMemcpyHostToDevice, st));
    } else {
        std::vector<int32_t> init(n, 1);
        HIPC(hipMemcpyAsync(d_size, init.data(), n * 4ull, hipMemcpyHostToDevice, st));
        int32_t zero = 0;
        HIPC(hipMemcpyAsync(d_chain, &zero, 4, hipMemcpyHostToDevice, st));
    }
    {   // the chain starts at the first active cluster, 0 (MST: at vertex 0); the
        // first kernel (parity 0) reads buffer 1, with no decision pending
        LinkState h[2] = {};
        h[1].len = 1; h[1].top = 0; h[1].below = -1; h[1].first_active = 0; h[1].mx = 0;
        h[1].c3 = -1;
        h[0] = h[1];
        HIPC(hipMemcpyAsync(d_st, h, sizeof(h), hipMemcpyHostToDevice, st));
        int32_t zero = 0;
        HIPC(hipMemcpyAsync(d_done, &zero, 4, hipMemcpyHostToDevice, st));
    }
#if DREPHIP_LK_DIAG
    LinkDiag *d_diag = nullptr;
    HIPC(hipMalloc((void **)&d_diag, sizeof(LinkDiag)));
    HIPC(hipMemset(d_diag, 0, sizeof(LinkDiag)));
    HIPC(hipMemcpyToSymbol(HIP_SYMBOL(g_lk_diag), &d_diag, sizeof(d_diag)));
#endif
#if DREPHIP_LK_PHASES
    uint64_t *d_ph = nullptr;
    if (!mst) {
        HIPC(hipMalloc((void **)&d_ph, (size_t)kPhCap * 16 * 8));
        HIPC(hipMemset(d_ph, 0, (size_t)kPhCap * 16 * 8));
        HIPC(hipMemcpyToSymbol(HIP_SYMBOL(g_lk_ph), &d_ph, sizeof(d_ph)));
    }
#endif
    // batches of steps captured in a graph, replayed until every merge is done
    // (DREPHIP_LINK_BATCH: an even batch length, and DREPHIP_LINK_POLL: the
    // replays between reads of the merge count -- small values for the tests,
    // which put compactions at many different chain states)
    const char *be = getenv("DREPHIP_LINK_BATCH"), *pe = getenv("DREPHIP_LINK_POLL");
    const int kBatch = be ? std::max(2, std::min(4096, atoi(be) & ~1)) : 256;
    const uint64_t poll = pe ? (uint64_t)std::max(1, atoi(pe)) : 4;
    // the compaction (above k_lk_cmp_rank): on for the chain methods unless
    // DREPHIP_LINK_COMPACT=0; while at least DREPHIP_LINK_COMPACT_MIN (2048)
    // clusters are active
    const char *ce = getenv("DREPHIP_LINK_COMPACT"), *cme = getenv("DREPHIP_LINK_COMPACT_MIN");
    const bool compact_on = !mst && (!ce || atoi(ce) != 0);
    const uint32_t compact_min = cme ? (uint32_t)std::max(2, atoi(cme)) : 2048;
    uint32_t m = n;                                 // the matrix's current size (stride)
    int32_t *d_sz = d_size, *d_sz2 = nullptr;       // sizes; the other buffer of a compaction
    uint32_t *d_rank = nullptr;
    int32_t *d_orig = nullptr;
    double *d_ctmp = nullptr;
    uint64_t kbase = 0;                              // merges before the current epoch
    std::vector<std::pair<uint64_t, std::vector<int32_t>>> epochs;   // (first Z row, local -> original index)
    auto capture = [&](hipGraphExec_t *exec) -> int {
        hipGraph_t graph = nullptr;
        HIPC(hipStreamSynchronize(st));
        HIPC(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        double *Zc = d_Z + 4 * kbase;
        const uint32_t wg = cfg.wg, grid = cfg.grid;
        const int tpl = cfg.tpl;
        for (int b = 0; b < kBatch; b++) {          // (even: step parity restarts at 0 with every replay)
            const uint32_t q = (uint32_t)(b & 1);
            const dim3 gm(grid), gn(grid + 1), blk(wg);
            const NnArgs a{d_D, m, d_sz, d_chain, d_ctl, d_prec, Zc, q, spec_on};
#define DREPHIP_LK_LAUNCH(W, P)                                                                                      \
    do {                                                                                                         \
        if (mst) hipLaunchKernelGGL((k_mst_step<W, P>), gm, blk, 0, st, d_D, m, d_sz, d_Dmin, d_st, d_parts, d_done, \
                                    Zc, q);                                                                      \
        else launch_nn<W, P>(method, gn, blk, st, a);                                                            \
    } while (0)
            if (wg == 64) {
                if (tpl == 1) launch_nn<64, 1>(method, gn, blk, st, a);
                else if (tpl == 2) launch_nn<64, 2>(method, gn, blk, st, a);
                else if (tpl == 4) launch_nn<64, 4>(method, gn, blk, st, a);
                else launch_nn<64, 8>(method, gn, blk, st, a);
            } else if (wg == 128) {
                if (tpl == 1) DREPHIP_LK_LAUNCH(128, 1);
                else if (tpl == 2) DREPHIP_LK_LAUNCH(128, 2);
                else DREPHIP_LK_LAUNCH(128, 4);
            } else if (wg == 512 && !mst) {
                if (tpl == 1) launch_nn<512, 1>(method, gn, blk, st, a);
                else launch_nn<512, 2>(method, gn, blk, st, a);
            } else {
                if (tpl == 1) DREPHIP_LK_LAUNCH(256, 1);
                else if (tpl == 2) DREPHIP_LK_LAUNCH(256, 2);
                else DREPHIP_LK_LAUNCH(256, 4);
            }
#undef DREPHIP_LK_LAUNCH
        }
        HIPC(hipStreamEndCapture(st, &graph));
        const hipError_t e = hipGraphInstantiate(exec, graph, nullptr, nullptr, 0);
        (void)hipGraphDestroy(graph);
        HIPC(e);
        return DREPHIP_OK;
    };
    // done = the merges of the current epoch; at most half of the m rows
    // active: the compaction, then the steps for the new m
    double compact_s = 0;                           // (host wall of the compactions, DREPHIP_DEBUG)
    auto compact = [&](int32_t done) -> int {
        const double t0 = now_s();
        int rc;
        if (!d_sz2) {
            if ((rc = scratch(ctx, "lk_size2", (n + 1) * 4ull, (void **)&d_sz2))) return rc;
            if ((rc = scratch(ctx, "lk_rank", (n + 1) * 4ull, (void **)&d_rank))) return rc;
            if ((rc = scratch(ctx, "lk_orig", n * 4ull, (void **)&d_orig))) return rc;
            if ((rc = scratch(ctx, "lk_ctmp", 64ull * (n / 2 + 1) * 8, (void **)&d_ctmp))) return rc;
        }
        const uint32_t np_old = DREPHIP_LK_WAVEPARTS ? cfg.grid * (cfg.wg / 64) : cfg.grid;
        hipLaunchKernelGGL(k_lk_cmp_rank, dim3(1), dim3(kCmpWG), 0, st, d_sz, d_st, m, d_rank, d_sz2, d_orig);
        uint32_t mn = 0;
        HIPC(hipMemcpyAsync(&mn, d_rank + m, 4, hipMemcpyDeviceToHost, st));
        HIPC(hipStreamSynchronize(st));
        if (mn != m - (uint32_t)done || mn > m / 2 || mn < 2) {
            set_error("linkage compaction: active clusters do not match the merge count");
            return DREPHIP_ERR_INTERNAL;
        }
        const StepCfg nc = cfg_for(mn);
        const uint32_t np_new = DREPHIP_LK_WAVEPARTS ? nc.grid * (nc.wg / 64) : nc.grid;
        hipLaunchKernelGGL(k_lk_cmp_state, dim3(1), dim3(256), 0, st, d_st, d_fwd, d_prec, d_chain,
                           d_rank, m, np_old, np_new, d_sz2, d_done);
        auto rows = [&](const double *src, double *dst, uint32_t r0, uint32_t r1, uint32_t d0) {
            const uint64_t items = (uint64_t)(r1 - r0) * ((mn + 1023) / 1024);
            const uint32_t g = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(8192, items));
            hipLaunchKernelGGL(k_lk_cmp_rows, dim3(g), dim3(256), 0, st, src, m, dst, mn, d_orig, r0, r1, d0);
        };
        const uint32_t R0 = std::min(64u, mn);
        rows(d_D, d_ctmp, 0, R0, 0);
        HIPC(hipMemcpyAsync(d_D, d_ctmp, (uint64_t)R0 * mn * 8, hipMemcpyDeviceToDevice, st));
        for (uint32_t r0 = R0, r1; r0 < mn; r0 = r1) {
            r1 = std::min(2 * r0, mn);
            rows(d_D, d_D, r0, r1, 0);
        }
        HIPC(hipGetLastError());
        std::vector<int32_t> loc(mn);
        HIPC(hipMemcpyAsync(loc.data(), d_orig, mn * 4ull, hipMemcpyDeviceToHost, st));
        HIPC(hipStreamSynchronize(st));
        if (!epochs.empty())
            for (auto &v : loc) v = epochs.back().second[v];
        kbase += (uint64_t)done;
        epochs.emplace_back(kbase, std::move(loc));
        std::swap(d_sz, d_sz2);
        m = mn;
        cfg = nc;
        compact_s += now_s() - t0;
        return DREPHIP_OK;
    };
    hipGraphExec_t exec = nullptr;
    if ((rc = capture(&exec))) return rc;
    // every search step either extends the chain or merges; the chain is at
    // most n long, so 3n steps always suffice (the bound only guards a hang)
    const uint64_t max_batches = (3ull * n) / kBatch + 2;
    int32_t done = 0;
    hipError_t e = hipSuccess;
    int crc = DREPHIP_OK;
    timing_mark(ctx, 2, st, true);
    for (uint64_t it = 0; it < max_batches; it++) {
        e = hipGraphLaunch(exec, st);
        if (e != hipSuccess) break;
        if (it % poll == poll - 1 || it + 1 == max_batches) {
            e = hipMemcpyAsync(&done, d_done, 4, hipMemcpyDeviceToHost, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            if (e != hipSuccess || done >= (int32_t)m - 1) break;
            if (compact_on && m - (uint32_t)done <= m / 2 && m - (uint32_t)done >= compact_min) {
                (void)hipGraphExecDestroy(exec);
                exec = nullptr;
                if ((crc = compact(done)) || (crc = capture(&exec))) break;
            }
        }
    }
    timing_mark(ctx, 2, st, false);
    if (exec) (void)hipGraphExecDestroy(exec);
    if (crc) return crc;
    HIPC(e);
    HIPC(hipMemcpyAsync(&done, d_done, 4, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    if (done != (int32_t)m - 1) { set_error("linkage did not finish"); return DREPHIP_ERR_INTERNAL; }
    ctx->link.compactions = epochs.size();
    LinkState hs[2];
    HIPC(hipMemcpy(hs, d_st, sizeof(hs), hipMemcpyDeviceToHost));
    const int32_t bad = (hs[0].flags | hs[1].flags) & kLkBad;
    ctx->link.launches = (uint64_t)std::max(hs[0].launches, hs[1].launches);
    if (getenv("DREPHIP_DEBUG"))
        fprintf(stderr, "[drephip] chain: n=%u launches %llu (%.4f per merge), speculation %d, compactions %zu (%.2f ms)\n",
                n, (unsigned long long)ctx->link.launches, (double)ctx->link.launches / (double)(n - 1), spec_on,
                epochs.size(), compact_s * 1e3);
#if DREPHIP_LK_DIAG
    {
        LinkDiag hd;
        HIPC(hipMemcpy(&hd, d_diag, sizeof(hd), hipMemcpyDeviceToHost));
        (void)hipFree(d_diag);
        fprintf(stderr, "[drephip] chain diag: twice %d scans %d specwin %d known %d (wmerge %d, recip %d) "
                        "merge launches without speculation %d\n", hd.twice, hd.scans, hd.specwin, hd.known,
                hd.wmerge, hd.recip, hd.m0);
    }
#endif
#if DREPHIP_LK_PHASES
    if (d_ph) {
        std::vector<uint64_t> h((size_t)kPhCap * 16);
        HIPC(hipMemcpy(h.data(), d_ph, h.size() * 8, hipMemcpyDeviceToHost));
        (void)hipFree(d_ph);
        const LinkState &hl = hs[0].launches > hs[1].launches ? hs[0] : hs[1];
        const int L = std::min(hl.launches, kPhCap) - 1;
        const char *names[] = {"wg0 partials reduced", "wg0 decided", "wg0 after barrier", "wg0 row loads in",
                               "wg0 row done", "wg0 reduced", "last wg start", "last wg after barrier", "last wg reduced",
                               "fwd start", "fwd partials reduced", "fwd decided", "fwd loads in", "next launch start"};
        const int col[] = {1, 2, 3, 4, 5, 6, 8, 9, 10, 12, 13, 14, 15, -1};
        for (int c = 0; c < 14; c++) {
            std::vector<double> v;
            for (int l = 100; l < L; l++) {
                const uint64_t *r = &h[(size_t)l * 16];
                if (!r[0] || !r[6]) continue;
                const uint64_t b = col[c] < 0 ? h[(size_t)(l + 1) * 16] : r[col[c]];
                if (!b) continue;
                v.push_back(((double)(int64_t)(b - r[0])) * 0.01);
            }
            if (v.empty()) continue;
            std::sort(v.begin(), v.end());
            fprintf(stderr, "[drephip] phase %-24s med %6.2f us  p90 %6.2f us (%zu launches)\n", names[c], v[v.size() / 2],
                    v[v.size() * 9 / 10], v.size());
        }
    }
#endif
    if (bad) { set_error("linkage: a chain step found no valid partial"); return DREPHIP_ERR_INTERNAL; }
    const double t_fin = now_s();
    ctx->link.chain_s = t_fin - t_chain;
    std::vector<double> Z(4ull * (n - 1));
    HIPC(hipMemcpy(Z.data(), d_Z, Z.size() * 8, hipMemcpyDeviceToHost));
    // rows merged after a compaction hold that epoch's numbers: the original ones
    for (size_t e = 0; e < epochs.size(); e++) {
        const uint64_t k1 = e + 1 < epochs.size() ? epochs[e + 1].first : n - 1;
        const std::vector<int32_t> &g = epochs[e].second;
        for (uint64_t k = epochs[e].first; k < k1; k++)
            for (int c = 0; c < 2; c++) Z[4 * k + c] = (double)g[(size_t)Z[4 * k + c]];
    }
    sort_and_label(Z, n);
    std::copy(Z.begin(), Z.end(), Z_out);
    ctx->link.finish_s = now_s() - t_fin;
    return DREPHIP_OK;
}

int dist_matrix_impl(drephip_ctx *ctx, const uint16_t *d_common, const uint16_t *d_denom, uint32_t n,
                     const uint32_t *perm, const double *lut, uint32_t lut_len, const int32_t *lut_off,
                     double **d_D_out, hipStream_t st) {
    const uint32_t s = ctx->s;
    double *d_D, *d_lut;
    uint32_t *d_perm, *d_bad, *h_bad;
    int32_t *d_off;
    int rc;
    const double t0 = now_s();
    if ((rc = scratch(ctx, "lk_D", (uint64_t)n * n * 8, (void **)&d_D))) return rc;
    const double t1 = now_s();
    ctx->link.alloc_s = t1 - t0;
    if ((rc = scratch(ctx, "lk_perm", n * 4ull, (void **)&d_perm))) return rc;
    if ((rc = scratch(ctx, "lk_bad", 4, (void **)&d_bad))) return rc;
    if ((rc = pinned_host(ctx, "lk_bad", 4, (void **)&h_bad))) return rc;
    HIPC(hipMemsetAsync(d_bad, 0, 4, st));
    if ((rc = scratch(ctx, "lk_lut", lut_len * 8ull, (void **)&d_lut))) return rc;
    if ((rc = scratch(ctx, "lk_off", (s + 1) * 4ull, (void **)&d_off))) return rc;
    HIPC(hipMemcpyAsync(d_perm, perm, n * 4ull, hipMemcpyHostToDevice, st));
    HIPC(hipMemcpyAsync(d_lut, lut, lut_len * 8ull, hipMemcpyHostToDevice, st));
    HIPC(hipMemcpyAsync(d_off, lut_off, (s + 1) * 4ull, hipMemcpyHostToDevice, st));
    timing_mark(ctx, 3, st, true);
    launch_dist_tiles_counts(DmFromCounts{d_common, d_denom, s, d_lut, d_off, d_bad}, n, d_perm, d_D, st);
    timing_mark(ctx, 3, st, false);
    HIPC(hipGetLastError());
    HIPC(hipMemcpyAsync(h_bad, d_bad, 4, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    if (*h_bad) {
        set_error("a pair's denominator has no distance table (lut_off < 0) or its count exceeds it");
        return DREPHIP_ERR_ARG;
    }
    ctx->link.matrix_s = now_s() - t1;
    *d_D_out = d_D;
    return DREPHIP_OK;
}

int dist_from_condensed_impl(drephip_ctx *ctx, const double *y, uint32_t n, double **d_D_out, hipStream_t st) {
    double *d_D, *d_y;
    int rc;
    const uint64_t np = (uint64_t)n * (n - 1) / 2;
    const double t0 = now_s();
    if ((rc = scratch(ctx, "lk_D", (uint64_t)n * n * 8, (void **)&d_D))) return rc;
    const double t1 = now_s();
    ctx->link.alloc_s = t1 - t0;
    if ((rc = scratch(ctx, "lk_y", np * 8, (void **)&d_y))) return rc;
    HIPC(hipMemcpyAsync(d_y, y, np * 8, hipMemcpyHostToDevice, st));
    timing_mark(ctx, 3, st, true);
    launch_dist_tiles_condensed(DmFromCondensed{d_y}, n, d_D, st);
    timing_mark(ctx, 3, st, false);
    HIPC(hipGetLastError());
    HIPC(hipStreamSynchronize(st));
    ctx->link.matrix_s = now_s() - t1;
    *d_D_out = d_D;
    return DREPHIP_OK;
}

int dist_from_square_impl(drephip_ctx *ctx, const float *M, uint32_t n, double **d_D_out, uint32_t *flags,
                          hipStream_t st) {
    double *d_D;
    float *d_M;
    uint32_t *d_bad, *h_bad;
    int rc;
    const double t0 = now_s();
    if ((rc = scratch(ctx, "lk_D", (uint64_t)n * n * 8, (void **)&d_D))) return rc;
    const double t1 = now_s();
    ctx->link.alloc_s = t1 - t0;
    if ((rc = scratch(ctx, "lk_sq", (uint64_t)n * n * 4, (void **)&d_M))) return rc;
    if ((rc = scratch(ctx, "lk_bad", 4, (void **)&d_bad))) return rc;
    if ((rc = pinned_host(ctx, "lk_bad", 4, (void **)&h_bad))) return rc;
    HIPC(hipMemsetAsync(d_bad, 0, 4, st));
    HIPC(hipMemcpyAsync(d_M, M, (uint64_t)n * n * 4, hipMemcpyHostToDevice, st));
    timing_mark(ctx, 3, st, true);
    const uint32_t nb = (n + kDmT - 1) / kDmT;
    hipLaunchKernelGGL(k_square_tiles, dim3((uint32_t)((uint64_t)nb * (nb + 1) / 2)), dim3(256), 0, st, d_M, n, nb,
                       d_D, d_bad);
    timing_mark(ctx, 3, st, false);
    HIPC(hipGetLastError());
    HIPC(hipMemcpyAsync(h_bad, d_bad, 4, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    *flags = *h_bad;
    ctx->link.matrix_s = now_s() - t1;
    *d_D_out = d_D;
    return DREPHIP_OK;
}


// ------------------------------------------------------- sparse pair list
// The pairs below 1.0 of the all-pairs counts, for the sparse linkage path
// (linkage_sparse.cpp): a pair with no shared hash is exactly 1.0, so only a
// nonzero count can be below it.  The condensed counts are streamed 8 per
// lane (16-byte loads, plus the denominators when some sketch is partial).
// Two passes over the same grid-stride ranges: the first counts each
// workgroup's finds, the host turns the counts into offsets (and stops there
// when the list would exceed its cap), the second writes (perm i, perm j) and
// the table index off[denom] + common at the workgroup's offset -- no global
// atomic (one counter for ~10^7 finds at 10^5 genomes serialised the pass:
// 28 ms instead of ~3).  HBM-bound: 2 B per pair (4 with denominators), 10 GB
// at n = 10^5.
constexpr int kSpWG = 256;
constexpr uint32_t kSpGrid = 4096;
__device__ __forceinline__ void cond_ij(uint64_t t, uint32_t n, uint32_t &i, uint32_t &j) {
    const double Mf = 2.0 * n - 1.0;
    int64_t r = (int64_t)((Mf - sqrt(fmax(Mf * Mf - 8.0 * (double)t, 0.0))) * 0.5);
    if (r < 0) r = 0;
    if (r > (int64_t)n - 2) r = (int64_t)n - 2;
    auto S = [&](int64_t a) { return (uint64_t)(a * (int64_t)n - a * (a + 1) / 2); };
    while (r > 0 && S(r) > t) r--;
    while (r + 1 <= (int64_t)n - 2 && S(r + 1) <= t) r++;
    i = (uint32_t)r;
    j = (uint32_t)(t - S(r) + r + 1);
}

template <bool WRITE>
__global__ __launch_bounds__(kSpWG) void k_sparse_pairs(const uint16_t *__restrict__ common,
                                                         const uint16_t *__restrict__ denom, uint64_t np,
                                                         uint32_t n, uint32_t s, const double *__restrict__ lut,
                                                         const int32_t *__restrict__ off,
                                                         const uint32_t *__restrict__ perm,
                                                         uint32_t *__restrict__ wg_count,
                                                         const uint64_t *__restrict__ wg_off,
                                                         uint32_t *__restrict__ out_ij, uint32_t *__restrict__ out_l,
                                                         uint32_t *__restrict__ flags) {
    __shared__ uint32_t s_n;
    const uint64_t nchunk = (np + 7) / 8;
    const uint64_t stride = (uint64_t)gridDim.x * kSpWG;
    const int32_t off_s = off[s];
    const uint32_t lane = threadIdx.x & 63;
    if (threadIdx.x == 0) s_n = 0;
    __syncthreads();
    const uint64_t base = WRITE ? wg_off[blockIdx.x] : 0;
    uint32_t bad = 0, mine = 0;
    for (uint64_t c0 = (uint64_t)blockIdx.x * kSpWG; c0 < nchunk; c0 += stride) {
        const uint64_t c = c0 + threadIdx.x;
        const uint64_t t0 = c * 8;
        uint16_t cm[8], dn[8];
        if (t0 + 8 <= np) {
            const uint4 w = *(const uint4 *)(common + t0);
            const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
            for (int e = 0; e < 8; e++) cm[e] = (uint16_t)(ww[e >> 1] >> (16 * (e & 1)));
            if (denom) {
                const uint4 d = *(const uint4 *)(denom + t0);
                const uint32_t dd[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
                for (int e = 0; e < 8; e++) dn[e] = (uint16_t)(dd[e >> 1] >> (16 * (e & 1)));
            }
        } else {
#pragma unroll
            for (int e = 0; e < 8; e++) {
                cm[e] = t0 + e < np ? common[t0 + e] : 0;
                dn[e] = denom && t0 + e < np ? denom[t0 + e] : (uint16_t)s;
            }
        }
        uint32_t hit = 0, lidx[8];
#pragma unroll
        for (int e = 0; e < 8; e++) {
            lidx[e] = 0;
            if (t0 + e >= np) continue;
            const uint32_t d = denom ? dn[e] : s;
            if (denom || cm[e]) {
                const int32_t o = !denom ? off_s : d <= s ? off[d] : -1;
                if (o < 0 || cm[e] > d) { bad = 1; continue; }
                lidx[e] = (uint32_t)o + cm[e];
                if (cm[e] && lut[lidx[e]] < 1.0) hit |= 1u << e;
            }
        }
        if (!WRITE) { mine += __builtin_popcount(hit); continue; }
        // the wave's finds: lane offsets by a wave scan, one LDS atomic per wave
        const uint32_t h = __builtin_popcount(hit);
        if (__ballot(h != 0)) {
            uint32_t inc = h;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(inc, d, 64);
                if (lane >= (uint32_t)d) inc += y;
            }
            uint32_t wbase = 0;
            if (lane == 63) wbase = atomicAdd(&s_n, inc);
            wbase = __shfl(wbase, 63, 64);
            uint64_t slot = base + wbase + inc - h;
            for (int e = 0; e < 8; e++) {
                if (!(hit >> e & 1)) continue;
                uint32_t i, j;
                cond_ij(t0 + e, n, i, j);
                out_ij[2 * slot] = perm[i];
                out_ij[2 * slot + 1] = perm[j];
                out_l[slot] = lidx[e];
                slot++;
            }
        }
    }
    if (bad) atomicOr(flags, 1u);
    if (!WRITE) {
        atomicAdd(&s_n, mine);
        __syncthreads();
        if (threadIdx.x == 0) wg_count[blockIdx.x] = s_n;
    }
}

int sparse_pairs_impl(drephip_ctx *ctx, const uint16_t *d_common, const uint16_t *d_denom, uint32_t n,
                      const uint32_t *perm, const double *lut, uint32_t lut_len, const int32_t *lut_off,
                      uint64_t cap, uint32_t **h_ij, uint32_t **h_lidx, uint64_t *np_out, uint32_t *flags_out,
                      hipStream_t st) {
    const uint32_t s = ctx->s;
    *np_out = 0;
    *flags_out = 0;
    // no sparse form unless a count of 0 means exactly 1.0 and nothing exceeds it
    for (uint32_t k = 0; k < lut_len; k++)
        if (!(lut[k] <= 1.0)) { *flags_out = 2; return DREPHIP_OK; }
    for (uint32_t d = 0; d <= s; d++)
        if (lut_off[d] >= 0 && lut[lut_off[d]] != 1.0) { *flags_out = 2; return DREPHIP_OK; }
    const uint64_t np = (uint64_t)n * (n - 1) / 2;
    double *d_lut;
    int32_t *d_off;
    uint32_t *d_perm, *d_ij, *d_l, *d_flags, *d_cnt, *h_cnt, *h_flags;
    uint64_t *d_wgoff, *h_wgoff;
    int rc;
    const uint64_t nchunk = (np + 7) / 8;
    const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(kSpGrid, (nchunk + kSpWG - 1) / kSpWG));
    if ((rc = scratch(ctx, "lk_lut", lut_len * 8ull, (void **)&d_lut))) return rc;
    if ((rc = scratch(ctx, "lk_off", (s + 1) * 4ull, (void **)&d_off))) return rc;
    if ((rc = scratch(ctx, "lk_perm", n * 4ull, (void **)&d_perm))) return rc;
    if ((rc = scratch(ctx, "lk_sp_cnt", (kSpGrid + 1) * 4ull, (void **)&d_cnt))) return rc;
    if ((rc = scratch(ctx, "lk_sp_off", kSpGrid * 8ull, (void **)&d_wgoff))) return rc;
    if ((rc = pinned_host(ctx, "lk_sp_cnt", (kSpGrid + 1) * 4ull, (void **)&h_cnt))) return rc;
    if ((rc = pinned_host(ctx, "lk_sp_off", kSpGrid * 8ull, (void **)&h_wgoff))) return rc;
    d_flags = d_cnt + kSpGrid;
    h_flags = h_cnt + kSpGrid;
    HIPC(hipMemcpyAsync(d_lut, lut, lut_len * 8ull, hipMemcpyHostToDevice, st));
    HIPC(hipMemcpyAsync(d_off, lut_off, (s + 1) * 4ull, hipMemcpyHostToDevice, st));
    HIPC(hipMemcpyAsync(d_perm, perm, n * 4ull, hipMemcpyHostToDevice, st));
    HIPC(hipMemsetAsync(d_flags, 0, 4, st));
    timing_mark(ctx, 3, st, true);
    hipLaunchKernelGGL(k_sparse_pairs<false>, dim3(grid), dim3(kSpWG), 0, st, d_common, d_denom, np, n, s, d_lut,
                       d_off, d_perm, d_cnt, (const uint64_t *)nullptr, (uint32_t *)nullptr, (uint32_t *)nullptr,
                       d_flags);
    timing_mark(ctx, 3, st, false);
    HIPC(hipGetLastError());
    HIPC(hipMemcpyAsync(h_cnt, d_cnt, (kSpGrid + 1) * 4ull, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    uint64_t total = 0;
    for (uint32_t b = 0; b < grid; b++) { h_wgoff[b] = total; total += h_cnt[b]; }
    *np_out = total;
    *flags_out = *h_flags;
    if (*h_flags || total > cap || total == 0) return DREPHIP_OK;
    if ((rc = scratch(ctx, "lk_sp_ij", total * 8, (void **)&d_ij))) return rc;
    if ((rc = scratch(ctx, "lk_sp_l", total * 4, (void **)&d_l))) return rc;
    HIPC(hipMemcpyAsync(d_wgoff, h_wgoff, grid * 8ull, hipMemcpyHostToDevice, st));
    timing_mark(ctx, 3, st, true);
    hipLaunchKernelGGL(k_sparse_pairs<true>, dim3(grid), dim3(kSpWG), 0, st, d_common, d_denom, np, n, s, d_lut,
                       d_off, d_perm, (uint32_t *)nullptr, d_wgoff, d_ij, d_l, d_flags);
    timing_mark(ctx, 3, st, false);
    HIPC(hipGetLastError());
    // pinned, grow-only: 60 MB at 5x10^6 pairs, kept for the next call
    if ((rc = pinned_host(ctx, "lk_sp_ij", total * 8, (void **)h_ij))) return rc;
    if ((rc = pinned_host(ctx, "lk_sp_l", total * 4, (void **)h_lidx))) return rc;
    HIPC(hipMemcpyAsync(*h_ij, d_ij, total * 8, hipMemcpyDeviceToHost, st));
    HIPC(hipMemcpyAsync(*h_lidx, d_l, total * 4, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    return DREPHIP_OK;
}

}  // namespace drephip
