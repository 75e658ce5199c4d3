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
// merge's row + column update fused with the grid-wide argmin over the chain
// top's row, whose last workgroup makes the chain decision.  Steps are
// launched in batches captured in a hipGraph; kernels after the last merge
// exit at once.
// Roofline: HBM -- a step reads one 8n-byte row (and after a merge two more
// rows, writing a row and a strided column); at n = 10^5 (0.8 MB rows) the
// ~5 us launch floor and the grid-wide reduction dominate.

#include "ctx.h"
#include "../../include/drephip.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <numeric>
#include <vector>

namespace drephip {

constexpr int kLkWG = 256;

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct LinkState {
    int32_t chain_len;
    int32_t first_active;    // smallest index with size > 0 (non-decreasing)
    int32_t top, below;      // chain[len-1], chain[len-2] (below: -1 if len < 2): a step's row without a dependent load
    int32_t k;               // merges done
    int32_t pend;            // 1: the update kernel applies merge (px <- py)
    int32_t px, py, pnx, pny;
    double pd;
    uint32_t ticket;         // last-workgroup detection of the search kernel
    int32_t x;               // MST: current vertex
    int32_t bad;             // a step found no valid partial (the host reports an internal error)
};

struct MinIdx { double v; int32_t i; };

__device__ __forceinline__ bool better(double v, int32_t i, double bv, int32_t bi) {
    return v < bv || (v == bv && i < bi);
}

// Lance-Williams updates exactly as scipy's _hierarchy_distance_update.pxi:
// every operation rounded on its own, as in scipy's x86-64 build (this file is
// compiled with -ffp-contract=off; see the Makefile)
__device__ __forceinline__ double lw_update(int method, double dxi, double dyi, int32_t nx, int32_t ny) {
    if (method == DREPHIP_LINK_COMPLETE) return fmax(dxi, dyi);
    if (method == DREPHIP_LINK_WEIGHTED) return __dmul_rn(0.5, __dadd_rn(dxi, dyi));
    // average: (size_x * d_xi + size_y * d_yi) / (size_x + size_y)
    return __ddiv_rn(__dadd_rn(__dmul_rn((double)nx, dxi), __dmul_rn((double)ny, dyi)), (double)(nx + ny));
}

// Block argmin (smallest index among equal minima); result valid in thread 0.
__device__ MinIdx block_argmin(double v, int32_t i) {
    __shared__ double sv[kLkWG / 64];
    __shared__ int32_t si[kLkWG / 64];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double ov = __shfl_xor(v, o, 64);
        const int32_t oi = __shfl_xor(i, o, 64);
        if (better(ov, oi, v, i)) { v = ov; i = oi; }
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { sv[w] = v; si[w] = i; }
    __syncthreads();
    MinIdx r{INFINITY, 0x7fffffff};
    if (threadIdx.x == 0)
        for (int k = 0; k < kLkWG / 64; k++)
            if (better(sv[k], si[k], r.v, r.i)) { r.v = sv[k]; r.i = si[k]; }
    return r;
}

// Last workgroup of a grid: every workgroup publishes its partial, then one
// agent-scope ticket; the workgroup that draws the last ticket reads all
// partials (agent-scope loads, spread over its threads) and reduces them.
// Every thread of the block must call it; the result is valid in thread 0.
//
// Visibility follows the "Valid forms" hand-off of MI355X_MICROARCH.md
// (inter-workgroup visibility, first row of its sc1 table), condition by
// condition:
//   (1) every load of a partial is an agent-scope atomic load (global_load
//       ... sc1, to registers, never flat);
//   (2) every store of a partial is an agent-scope atomic store (sc1, 8 and 4
//       bytes);
//   (3) the storing lane -- the only one -- waits s_waitcnt vmcnt(0) after its
//       stores and only then adds to the ONE unsharded ticket;
//   (4) the consumer is the workgroup whose add came last, told by the value
//       its add returned; its thread 0 reads after the add returned and the
//       other waves after the __syncthreads that thread 0 joins; hipMalloc
//       memory; at most one such workgroup per CU (grids of <= 1024
//       256-thread workgroups over 256 CUs are dealt round-robin).
// Under those four conditions the guide measured the sc1 loads as a valid
// replacement for an agent-scope acquire, so no fence is issued: the acquire
// (buffer_inv sc1 + its vmcnt wait, in the last workgroup only) measured +13 %
// chain time at n = 10^4 and +4 % at 10^5 (profiles/r03_scale_*.json), and the
// release/acquire ticket (buffer_wbl2 sc1 per workgroup per step) +21 %.  The
// argument is about the gfx942/gfx950 sc1 path, not the HIP/LLVM memory
// model, so the file refuses other targets.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__) && !defined(__gfx942__)
#error "linkage.hip's ticket reduction relies on the gfx942/gfx950 sc1 hand-off (MI355X_MICROARCH.md, Valid forms)"
#endif
__device__ bool last_block(MinIdx part, MinIdx *parts, LinkState *st, MinIdx &out) {
    __shared__ int is_last;
    if (threadIdx.x == 0) {
        __hip_atomic_store(&parts[blockIdx.x].v, part.v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&parts[blockIdx.x].i, part.i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t t = __hip_atomic_fetch_add(&st->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        is_last = t == gridDim.x - 1;
        if (is_last) st->ticket = 0;
    }
    __syncthreads();
    if (!is_last) return false;
    double bv = INFINITY;
    int32_t bi = 0x7fffffff;
    for (uint32_t b = threadIdx.x; b < gridDim.x; b += blockDim.x) {
        const double v = __hip_atomic_load(&parts[b].v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int32_t i = __hip_atomic_load(&parts[b].i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (better(v, i, bv, bi)) { bv = v; bi = i; }
    }
    out = block_argmin(bv, bi);
    return true;
}

// ---------------------------------------------------------------- nn_chain
// Merge chain top x (size sx) with y (size sy) at distance cur (scipy: the
// smaller index is dropped, the larger becomes the new cluster), pop both,
// restart an empty chain at the first active cluster.  k: merges so far.
__device__ void chain_merge(int32_t x, int32_t y, int32_t sx, int32_t sy, double cur, int32_t len, int32_t k,
                            uint32_t n, int32_t *size, int32_t *chain, LinkState *st, double *Z, int32_t c3, int32_t c4) {
    int32_t a = x, b = y, na = sx, nb = sy;
    if (a > b) { a = y; b = x; na = sy; nb = sx; }
    Z[4 * k + 0] = a; Z[4 * k + 1] = b; Z[4 * k + 2] = cur; Z[4 * k + 3] = na + nb;
    size[a] = 0;
    size[b] = na + nb;
    st->pend = 1; st->px = a; st->py = b; st->pnx = na; st->pny = nb; st->pd = cur;
    st->k = k + 1;
    st->chain_len = len - 2;
    st->top = c3;                                // chain[len-3], chain[len-4] (loaded at the step's start)
    st->below = len >= 4 ? c4 : -1;
    if (st->chain_len == 0 && k + 1 < (int32_t)n - 1) {
        int32_t f = st->first_active;
        while (size[f] == 0) f++;
        st->first_active = f;
        chain[0] = f;
        st->chain_len = 1;
        st->top = f;
        st->below = -1;
    }
}

// One chain step per launch: the pending merge's Lance-Williams update (row and
// column y) fused with the search of the chain top's row.  The search of row
// t = chain top reads D[t][i]; the update rewrites only row/column y, so every
// D[t][i] with i != y is untouched, and the one changed entry D[t][y] is
// produced by the thread of i = y (the thread of i = t skips it), which also
// uses it as its search value -- no cross-workgroup dependence.  After a chain
// restart t may be y itself: then the search value of i is the freshly
// computed D[y][i].  The last workgroup makes scipy's chain decision.
//
// A step is a chain of dependent memory round trips, so the loads are issued
// together: each pass takes kLkPer entries per lane (grid-stride) and loads
// their sizes and D[t][i] (plus D[x][i], D[y][i] after a merge) before any of
// them is used or any store is made (written as one loop, the compiler kept
// each entry's loads behind the previous entry's stores: D aliases itself).
// D[t][i] may be loaded before the update's stores because the update writes
// D[t][i] only for i = y, whose search value is the freshly computed entry.
// Likewise the chain decision's D[t][chain[len-2]] and the two sizes are
// loaded at the start by every workgroup's thread 0: the chain's elements
// below the top are never x or y, so no update of this step touches them.
// The chain's top and the element below it are kept in LinkState (the step's
// row needs no load of chain[]), and chain[len-3], chain[len-4] -- the top
// and below after a merge -- are loaded at the start too.
constexpr int kLkPer = 4;
__global__ __launch_bounds__(kLkWG) void k_nn_step(double *__restrict__ D, uint32_t n, int method,
                                                  int32_t *__restrict__ size, int32_t *__restrict__ chain,
                                                  LinkState *__restrict__ st, MinIdx *__restrict__ parts,
                                                  double *__restrict__ Z) {
    const int32_t k0 = st->k;
    if (k0 >= (int32_t)n - 1) return;                          // all merged: the rest of the batch idles
    const bool pend = st->pend != 0;
    const int32_t x = st->px, y = st->py, nx = st->pnx, ny = st->pny;
    const int32_t len = st->chain_len;
    const int32_t t = st->top;
    const double *Dt = D + (uint64_t)t * n;
    const double *Dx = D + (uint64_t)x * n;
    double *Dy = D + (uint64_t)y * n;
    // a merge is always of t with yp = chain[len-2]: thread 0 loads the
    // decision's operands (D[t][yp] and both sizes) now, off the last
    // workgroup's critical path
    int32_t yp = -1, szt = 0, szyp = 0, c3 = 0, c4 = 0;
    double dp = 0.0;
    if (threadIdx.x == 0 && len > 1) {
        yp = st->below; dp = Dt[yp]; szt = size[t]; szyp = size[yp];
        if (len >= 3) c3 = chain[len - 3];                   // the chain's new top and below after a merge
        if (len >= 4) c4 = chain[len - 4];
    }
    // the old D[x][t], D[y][t] for the lane of i = y (loaded before any store)
    const double dxt = pend ? Dx[t] : 0.0, dyt = pend ? Dy[t] : 0.0;
    double bv = INFINITY;
    int32_t bi = 0x7fffffff;
    const uint32_t stride = gridDim.x * kLkWG;
    for (uint32_t i0 = blockIdx.x * kLkWG + threadIdx.x; i0 < n; i0 += kLkPer * stride) {
        int32_t sz[kLkPer];
        double dt[kLkPer], dx[kLkPer], dy[kLkPer];
#pragma unroll
        for (int k = 0; k < kLkPer; k++) {
            const uint32_t i = i0 + k * stride;
            const uint32_t ic = i < n ? i : n - 1;              // in bounds; i >= n is skipped below
            sz[k] = size[ic];
            dt[k] = Dt[ic];
            if (pend) { dx[k] = Dx[ic]; dy[k] = Dy[ic]; }
        }
#pragma unroll
        for (int k = 0; k < kLkPer; k++) {
            const uint32_t i = i0 + k * stride;
            if (i >= n || sz[k] == 0) continue;
            double v;
            if (pend && (int32_t)i != y && (int32_t)i != t) {
                const double u = lw_update(method, dx[k], dy[k], nx, ny);
                Dy[i] = u;
                D[(uint64_t)i * n + y] = u;
                v = t == y ? u : dt[k];
            } else if (pend && (int32_t)i == y && t != y) {
                const double u = lw_update(method, dxt, dyt, nx, ny);      // entry (y, t): old values, unshared
                Dy[t] = u;
                D[(uint64_t)t * n + y] = u;
                v = u;
            } else {
                if ((int32_t)i == t) continue;
                v = dt[k];
            }
            if (v < bv) { bv = v; bi = (int32_t)i; }            // ascending i per thread: first minimum kept
        }
    }
    const MinIdx part = block_argmin(bv, bi);
    MinIdx g;
    if (!last_block(part, parts, st, g)) return;
    if (threadIdx.x != 0) return;
    if ((uint32_t)g.i >= n) {                    // no valid partial: stop every later step, the host reports it
        st->bad = 1;
        st->k = (int32_t)n - 1;
        return;
    }
    // chain decision (scipy nn_chain): the previous chain element wins ties
    st->pend = 0;
    int32_t yy = g.i;
    double cur = g.v;
    bool merge = false;
    if (len > 1 && !(g.v < dp)) { yy = yp; cur = dp; merge = true; }
    if (!merge) {
        if (len >= (int32_t)n) {                 // cannot happen on a consistent matrix: stop, no out-of-range store
            st->bad = 1;
            st->k = (int32_t)n - 1;
            return;
        }
        chain[len] = yy;
        st->chain_len = len + 1;
        st->below = t;
        st->top = yy;
        return;
    }
    chain_merge(t, yy, szt, szyp, cur, len, k0, n, size, chain, st, Z, c3, c4);
}

// ------------------------------------------------------------ MST (single)
__global__ __launch_bounds__(kLkWG) void k_mst_step(const double *__restrict__ D, uint32_t n,
                                                   int32_t *__restrict__ merged, double *__restrict__ Dmin,
                                                   LinkState *__restrict__ st, MinIdx *__restrict__ parts,
                                                   double *__restrict__ Z) {
    if (st->k >= (int32_t)n - 1) return;
    const int32_t x = st->x;
    const double *Dx = D + (uint64_t)x * n;
    double bv = INFINITY;
    int32_t bi = 0x7fffffff;
    const uint32_t stride = gridDim.x * kLkWG;
    for (uint32_t i0 = blockIdx.x * kLkWG + threadIdx.x; i0 < n; i0 += kLkPer * stride) {
        int32_t mg[kLkPer];
        double dx[kLkPer], dm[kLkPer];
#pragma unroll
        for (int k = 0; k < kLkPer; k++) {                      // loads first (as k_nn_step)
            const uint32_t i = i0 + k * stride;
            const uint32_t ic = i < n ? i : n - 1;
            mg[k] = merged[ic];
            dx[k] = Dx[ic];
            dm[k] = Dmin[ic];
        }
#pragma unroll
        for (int k = 0; k < kLkPer; k++) {
            const uint32_t i = i0 + k * stride;
            if (i >= n || mg[k]) continue;
            double m = dm[k];
            if (m > dx[k]) { m = dx[k]; Dmin[i] = m; }
            if (m < bv) { bv = m; bi = (int32_t)i; }
        }
    }
    const MinIdx part = block_argmin(bv, bi);
    MinIdx g;
    if (!last_block(part, parts, st, g)) return;
    if (threadIdx.x != 0) return;
    if ((uint32_t)g.i >= n) {
        st->bad = 1;
        st->k = (int32_t)n - 1;
        return;
    }
    const int32_t k = st->k;
    Z[4 * k + 0] = x; Z[4 * k + 1] = g.i; Z[4 * k + 2] = g.v; Z[4 * k + 3] = 0;
    merged[g.i] = 1;
    st->x = g.i;
    st->k = k + 1;
}

// --------------------------------------------------- persistent chain / MST
// The whole chain (or Prim's MST) in ONE launch: P participant workgroups of
// kPW threads (one per CU; P <= 64 << 256 CUs, so all are resident), each
// owning a contiguous slice of the n columns with its clusters' sizes (and,
// for MST, the merged flags and running minima) in LDS.  A step is the
// k_nn_step / k_mst_step work on the participant's slice, then an exchange:
// every participant publishes its slice's candidate (value, index, that
// cluster's size, and the slice's first active cluster other than the one a
// merge of this step would retire, with its size) and a step tag; every
// participant reads all P candidates and makes the SAME scipy decision from
// them (replicated, deterministic), so no state is shared between
// participants except the matrix itself and the published candidates.  The
// chain (indices + sizes) lives in each participant's LDS.
//
// Visibility (MI355X_MICROARCH.md, Valid forms, first row of the sc1 table):
// every load and store of the matrix and of the candidates is an agent-scope
// (sc1) access; every wave drains its stores (s_waitcnt vmcnt(0)) before the
// workgroup barrier behind which ONE lane stores the step tag (sc1); the
// consumer lanes poll the tags with sc1 loads and read the candidates after
// their tag matched; the other waves read after the workgroup barrier.  The
// only matrix entries one participant reads after another wrote them are the
// Lance-Williams column entries D[i][y], read as D[t][y] in a later step --
// always after the writer's tag of the step that wrote them.
//
// Every spin is bounded (2 s of s_memrealtime per step): a participant that
// never arrives makes the others stop with an error flag instead of hanging,
// and the host then runs the per-step graph path.  Every index taken from a
// candidate is range-checked before use.
constexpr bool kLinkPersistDefault = false; // auto: the per-step graph path until the persistent one is the default
constexpr int kPW = 1024;                 // threads per participant
constexpr uint32_t kPMaxSlice = 4096;     // columns per participant (LDS: sizes 16 KB, MST minima 32 KB)
constexpr uint32_t kPMaxP = 64;           // participants (one wave polls them)
constexpr uint32_t kPChainCap = 4096;     // chain entries in LDS (longer: error flag, graph path)
constexpr uint64_t kPTimeout = 200000000; // s_memrealtime ticks (100 MHz): 2 s per step

struct PCand { double v; int32_t i, sz, fa, szfa; int32_t pad[2]; };   // 32 B per participant
struct PStat { int32_t err; int32_t steps; int32_t pad[14]; };

__device__ __forceinline__ double ld1(const double *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st1(double *p, double v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ int32_t ld1i(const int32_t *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st1i(int32_t *p, int32_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// (v, i) lexicographic minimum of a workgroup plus a second minimum (f, with
// its payload fs); results in thread 0.  Payload sz rides with (v, i).
struct PRed { double v; int32_t i, sz, f, fs; };
__device__ PRed block_reduce_p(PRed r) {
    __shared__ PRed sr[kPW / 64];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        PRed q;
        q.v = __shfl_xor(r.v, o, 64); q.i = __shfl_xor(r.i, o, 64); q.sz = __shfl_xor(r.sz, o, 64);
        q.f = __shfl_xor(r.f, o, 64); q.fs = __shfl_xor(r.fs, o, 64);
        if (better(q.v, q.i, r.v, r.i)) { r.v = q.v; r.i = q.i; r.sz = q.sz; }
        if (q.f < r.f) { r.f = q.f; r.fs = q.fs; }
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) sr[w] = r;
    __syncthreads();
    if (threadIdx.x == 0)
        for (int k = 1; k < kPW / 64; k++) {
            const PRed q = sr[k];
            if (better(q.v, q.i, r.v, r.i)) { r.v = q.v; r.i = q.i; r.sz = q.sz; }
            if (q.f < r.f) { r.f = q.f; r.fs = q.fs; }
        }
    return r;
}

// Publish this participant's candidate for step `step` and collect everyone's:
// returns the global reduction in thread 0; false (all threads) on a timeout.
__device__ bool p_exchange(PRed mine, uint32_t step, uint32_t P, PCand *cand, int32_t *tags, PRed &out,
                           PStat *stat) {
    __shared__ int s_ok;
    PCand *slot = cand + (uint64_t)(step & 1) * kPMaxP;
    // every wave's matrix stores are complete before the tag (condition 3)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        PCand *c = slot + blockIdx.x;
        st1(&c->v, mine.v);
        st1i(&c->i, mine.i); st1i(&c->sz, mine.sz); st1i(&c->fa, mine.f); st1i(&c->szfa, mine.fs);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        st1i(&tags[blockIdx.x * 16], (int32_t)step);
    }
    if (threadIdx.x < 64) {
        const uint32_t lane = threadIdx.x;
        PRed r{INFINITY, 0x7fffffff, 0, 0x7fffffff, 0};
        bool ok = true;
        if (lane < P) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (ld1i(&tags[lane * 16]) != (int32_t)step) {
                __builtin_amdgcn_s_sleep(1);
                if (__builtin_amdgcn_s_memrealtime() - t0 > kPTimeout) { ok = false; break; }
            }
            if (ok) {
                const PCand *c = slot + lane;
                r.v = ld1(&c->v); r.i = ld1i(&c->i); r.sz = ld1i(&c->sz); r.f = ld1i(&c->fa); r.fs = ld1i(&c->szfa);
            }
        }
        const bool all_ok = __builtin_amdgcn_ballot_w64(!ok) == 0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            PRed q;
            q.v = __shfl_xor(r.v, o, 64); q.i = __shfl_xor(r.i, o, 64); q.sz = __shfl_xor(r.sz, o, 64);
            q.f = __shfl_xor(r.f, o, 64); q.fs = __shfl_xor(r.fs, o, 64);
            if (better(q.v, q.i, r.v, r.i)) { r.v = q.v; r.i = q.i; r.sz = q.sz; }
            if (q.f < r.f) { r.f = q.f; r.fs = q.fs; }
        }
        if (lane == 0) {
            out = r;
            s_ok = all_ok;
            if (!all_ok) st1i(&stat->err, 1);
        }
    }
    __syncthreads();
    return s_ok != 0;
}

// Replicated nn-chain state (identical in every participant; thread 0 writes
// it, everyone reads it after a barrier)
struct PChain {
    int32_t k, len, top, below, pend, x, y, nx, ny, stop;
};

template <int PER>
__global__ __launch_bounds__(kPW) void k_chain_persist(double *__restrict__ D, uint32_t n, int method, uint32_t S,
                                                       PCand *__restrict__ cand, int32_t *__restrict__ tags,
                                                       PStat *__restrict__ stat, double *__restrict__ Z) {
    __shared__ int32_t size_s[kPMaxSlice];
    __shared__ int32_t ch_i[kPChainCap], ch_s[kPChainCap];
    __shared__ PChain cs;
    __shared__ double s_dp;
    const uint32_t P = gridDim.x, p = blockIdx.x;
    const uint32_t lo = p * S, hi = min(n, lo + S);
    for (uint32_t j = threadIdx.x; j < S; j += kPW) size_s[j] = lo + j < hi ? 1 : 0;
    if (threadIdx.x == 0) {
        cs = PChain{0, 1, 0, -1, 0, 0, 0, 0, 0, 0};
        ch_i[0] = 0; ch_s[0] = 1;
    }
    __syncthreads();
    for (uint32_t step = 0;; step++) {
        const PChain c = cs;
        if (c.k >= (int32_t)n - 1 || c.stop) break;
        const int32_t t = c.top;
        const bool pend = c.pend != 0;
        const int32_t x = c.x, y = c.y;
        const int32_t a_m = c.len > 1 ? min(t, c.below) : -1;          // retired if this step merges
        const double *Dt = D + (uint64_t)t * n;
        const double *Dx = D + (uint64_t)x * n;
        double *Dy = D + (uint64_t)y * n;
        if (threadIdx.x == 0 && c.len > 1) s_dp = ld1(Dt + c.below);
        const bool own_y = pend && (uint32_t)y >= lo && (uint32_t)y < hi;
        const double dxt = own_y ? ld1(Dx + t) : 0.0, dyt = own_y ? ld1(Dy + t) : 0.0;
        PRed r{INFINITY, 0x7fffffff, 0, 0x7fffffff, 0};
        for (uint32_t j0 = threadIdx.x; j0 < hi - lo; j0 += PER * kPW) {
            int32_t sz[PER];
            double dt[PER], dx[PER], dy[PER];
#pragma unroll
            for (int q = 0; q < PER; q++) {
                const uint32_t j = j0 + q * kPW;
                const uint32_t jc = j < hi - lo ? j : hi - lo - 1;
                const uint32_t i = lo + jc;
                sz[q] = size_s[jc];
                dt[q] = ld1(Dt + i);
                if (pend) { dx[q] = ld1(Dx + i); dy[q] = ld1(Dy + i); }
            }
#pragma unroll
            for (int q = 0; q < PER; q++) {
                const uint32_t j = j0 + q * kPW;
                if (j >= hi - lo || sz[q] == 0) continue;
                const int32_t i = (int32_t)(lo + j);
                if (i != a_m && i < r.f) { r.f = i; r.fs = sz[q]; }
                double v;
                if (pend && i != y && i != t) {
                    const double u = lw_update(method, dx[q], dy[q], c.nx, c.ny);
                    st1(Dy + i, u);
                    st1(D + (uint64_t)i * n + y, u);
                    v = t == y ? u : dt[q];
                } else if (pend && i == y && t != y) {
                    const double u = lw_update(method, dxt, dyt, c.nx, c.ny);
                    st1(Dy + t, u);
                    st1(D + (uint64_t)t * n + y, u);
                    v = u;
                } else {
                    if (i == t) continue;
                    v = dt[q];
                }
                if (v < r.v) { r.v = v; r.i = i; r.sz = sz[q]; }
            }
        }
        r = block_reduce_p(r);
        PRed g;
        if (!p_exchange(r, step, P, cand, tags, g, stat)) return;
        if (threadIdx.x == 0) {
            PChain d = c;
            d.pend = 0;
            if ((uint32_t)g.i >= n) { st1i(&stat->err, 2); d.stop = 1; }
            else {
                const double dp = s_dp;
                const bool merge = c.len > 1 && !(g.v < dp);
                if (!merge) {
                    if (c.len >= (int32_t)kPChainCap || c.len >= (int32_t)n) { st1i(&stat->err, 3); d.stop = 1; }
                    else {
                        ch_i[c.len] = g.i; ch_s[c.len] = g.sz;
                        d.len = c.len + 1; d.below = t; d.top = g.i;
                    }
                } else {
                    const int32_t yb = c.below;
                    const int32_t st_ = ch_s[c.len - 1], sb = ch_s[c.len - 2];
                    int32_t a = t, b = yb, na = st_, nb = sb;
                    if (a > b) { a = yb; b = t; na = sb; nb = st_; }
                    if (p == 0) {
                        double *z = Z + 4ull * c.k;
                        z[0] = a; z[1] = b; z[2] = dp; z[3] = na + nb;
                    }
                    if ((uint32_t)a >= lo && (uint32_t)a < hi) size_s[a - lo] = 0;
                    if ((uint32_t)b >= lo && (uint32_t)b < hi) size_s[b - lo] = na + nb;
                    d.pend = 1; d.x = a; d.y = b; d.nx = na; d.ny = nb;
                    d.k = c.k + 1;
                    d.len = c.len - 2;
                    d.top = d.len > 0 ? ch_i[d.len - 1] : -1;
                    d.below = d.len > 1 ? ch_i[d.len - 2] : -1;
                    if (d.len == 0 && d.k < (int32_t)n - 1) {
                        if ((uint32_t)g.f >= n) { st1i(&stat->err, 4); d.stop = 1; }
                        else { ch_i[0] = g.f; ch_s[0] = g.fs; d.len = 1; d.top = g.f; d.below = -1; }
                    }
                }
            }
            cs = d;
            if (p == 0) stat->steps = (int32_t)step + 1;
        }
        __syncthreads();
    }
}

template <int PER>
__global__ __launch_bounds__(kPW) void k_mst_persist(const double *__restrict__ D, uint32_t n, uint32_t S,
                                                     PCand *__restrict__ cand, int32_t *__restrict__ tags,
                                                     PStat *__restrict__ stat, double *__restrict__ Z) {
    __shared__ double dmin_s[kPMaxSlice];
    __shared__ uint8_t merged_s[kPMaxSlice];
    __shared__ int32_t s_x, s_k, s_stop;
    const uint32_t P = gridDim.x, p = blockIdx.x;
    const uint32_t lo = p * S, hi = min(n, lo + S);
    for (uint32_t j = threadIdx.x; j < S; j += kPW) { dmin_s[j] = INFINITY; merged_s[j] = lo + j >= hi || lo + j == 0; }
    if (threadIdx.x == 0) { s_x = 0; s_k = 0; s_stop = 0; }           // scipy: x = 0, merged[0] = 1
    __syncthreads();
    for (uint32_t step = 0;; step++) {
        const int32_t x = s_x, k = s_k;
        if (k >= (int32_t)n - 1 || s_stop) break;
        const double *Dx = D + (uint64_t)x * n;
        PRed r{INFINITY, 0x7fffffff, 0, 0x7fffffff, 0};
        for (uint32_t j0 = threadIdx.x; j0 < hi - lo; j0 += PER * kPW) {
            double dx[PER];
#pragma unroll
            for (int q = 0; q < PER; q++) {
                const uint32_t j = j0 + q * kPW;
                dx[q] = ld1(Dx + lo + (j < hi - lo ? j : hi - lo - 1));
            }
#pragma unroll
            for (int q = 0; q < PER; q++) {
                const uint32_t j = j0 + q * kPW;
                if (j >= hi - lo || merged_s[j]) continue;
                double m = dmin_s[j];
                if (m > dx[q]) { m = dx[q]; dmin_s[j] = m; }
                if (m < r.v) { r.v = m; r.i = (int32_t)(lo + j); }
            }
        }
        r = block_reduce_p(r);
        PRed g;
        if (!p_exchange(r, step, P, cand, tags, g, stat)) return;
        if (threadIdx.x == 0) {
            if ((uint32_t)g.i >= n) { st1i(&stat->err, 2); s_stop = 1; }
            else {
                if (p == 0) {
                    double *z = Z + 4ull * k;
                    z[0] = x; z[1] = g.i; z[2] = g.v; z[3] = 0;
                }
                if ((uint32_t)g.i >= lo && (uint32_t)g.i < hi) merged_s[g.i - lo] = 1;
                s_x = g.i;
                s_k = k + 1;
            }
            if (p == 0) stat->steps = (int32_t)step + 1;
        }
        __syncthreads();
    }
}

// Persistent path: returns DREPHIP_OK with d_Z filled, or DREPHIP_ERR_INTERNAL
// (with the reason in the error text) when a participant timed out or the
// chain outgrew its LDS -- the caller then runs the per-step graph path.
static int linkage_persist(drephip_ctx *ctx, double *d_D, uint32_t n, int method, double *d_Z, hipStream_t st) {
    uint32_t P = std::max(1u, std::min(kPMaxP, (n + 2047) / 2048));
    uint32_t S = (n + P - 1) / P;
    if (S > kPMaxSlice) { set_error("persistent linkage: n too large"); return DREPHIP_ERR_UNSUPPORTED; }
    PCand *d_cand;
    int32_t *d_tags;
    PStat *d_stat, *h_stat;
    int rc;
    if ((rc = scratch(ctx, "lkp_cand", 2 * kPMaxP * sizeof(PCand), (void **)&d_cand))) return rc;
    if ((rc = scratch(ctx, "lkp_tags", kPMaxP * 16 * 4, (void **)&d_tags))) return rc;
    if ((rc = scratch(ctx, "lkp_stat", sizeof(PStat), (void **)&d_stat))) return rc;
    if ((rc = pinned_host(ctx, "lkp_stat", sizeof(PStat), (void **)&h_stat))) return rc;
    HIPC(hipMemsetAsync(d_tags, 0xFF, kPMaxP * 16 * 4, st));         // tag -1: no step published
    HIPC(hipMemsetAsync(d_stat, 0, sizeof(PStat), st));
    timing_mark(ctx, 2, st, true);
    if (method == DREPHIP_LINK_SINGLE)
        hipLaunchKernelGGL(k_mst_persist<4>, dim3(P), dim3(kPW), 0, st, d_D, n, S, d_cand, d_tags, d_stat, d_Z);
    else
        hipLaunchKernelGGL(k_chain_persist<4>, dim3(P), dim3(kPW), 0, st, d_D, n, method, S, d_cand, d_tags, d_stat, d_Z);
    timing_mark(ctx, 2, st, false);
    HIPC(hipGetLastError());
    HIPC(hipMemcpyAsync(h_stat, d_stat, sizeof(PStat), hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    ctx->link.persist_steps = h_stat->steps;
    ctx->link.persist_participants = P;
    if (h_stat->err) {
        static const char *why[] = {"", "a participant timed out", "no valid candidate", "chain longer than its LDS",
                                    "no cluster to restart the chain"};
        set_error(std::string("persistent linkage stopped: ") + why[std::min(h_stat->err, 4)]);
        return DREPHIP_ERR_INTERNAL;
    }
    return DREPHIP_OK;
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
    __device__ __forceinline__ double operator()(uint64_t t) const {
        const uint32_t dn = denom ? denom[t] : s;
        const uint32_t cm = common[t];
        const int32_t o = dn <= s ? off[dn] : -1;
        if (o >= 0 && cm <= dn) return lut[o + cm];
        atomicOr(bad, 1u);
        return __builtin_nan("");
    }
};
struct DmFromCondensed {
    const double *y;
    __device__ __forceinline__ double operator()(uint64_t t) const { return y[t]; }
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
    for (uint32_t r = w; r < kDmT; r += 4) {
        const uint32_t i = i0 + r, j = j0 + lane;
        if (i >= n) break;
        const uint32_t pi = perm ? perm[i] : i;
        if (j < n && j > i) {
            const double v = val((uint64_t)i * n - (uint64_t)i * (i + 1) / 2 + (j - i - 1));
            tile[r][lane] = v;
            D[(uint64_t)pi * n + (perm ? perm[j] : j)] = v;
        } else if (j == i) {
            D[(uint64_t)pi * n + pi] = 0.0;
        }
    }
    __syncthreads();
    for (uint32_t c = w; c < kDmT; c += 4) {
        const uint32_t j = j0 + c, i = i0 + lane;
        if (j >= n) break;
        if (j > i) D[(uint64_t)(perm ? perm[j] : j) * n + (perm ? perm[i] : i)] = tile[lane][c];
    }
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
// scipy: Z sorted by distance (np.argsort kind='mergesort': stable), then
// `label` (union-find over 2n-1 nodes; the smaller root first; sizes).
static void sort_and_label(std::vector<double> &Z, uint32_t n) {
    const uint32_t m = n - 1;
    std::vector<uint32_t> order(m);
    std::iota(order.begin(), order.end(), 0u);
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return Z[4 * a + 2] < Z[4 * b + 2]; });
    std::vector<double> S(4ull * m);
    for (uint32_t r = 0; r < m; r++)
        for (int c = 0; c < 4; c++) S[4ull * r + c] = Z[4ull * order[r] + c];
    std::vector<int64_t> parent(2ull * n - 1);
    std::iota(parent.begin(), parent.end(), 0);
    std::vector<int64_t> sz(2ull * n - 1, 1);
    auto find = [&](int64_t x) {
        int64_t p = x;
        while (parent[p] != p) p = parent[p];
        while (parent[x] != p) { const int64_t nx = parent[x]; parent[x] = p; x = nx; }
        return p;
    };
    int64_t next = n;
    for (uint32_t r = 0; r < m; r++) {
        const int64_t xr = find((int64_t)S[4ull * r]), yr = find((int64_t)S[4ull * r + 1]);
        S[4ull * r] = (double)std::min(xr, yr);
        S[4ull * r + 1] = (double)std::max(xr, yr);
        parent[xr] = next; parent[yr] = next;
        sz[next] = sz[xr] + sz[yr];
        S[4ull * r + 3] = (double)sz[next];
        next++;
    }
    Z.swap(S);
}

// Which chain implementation runs: DREPHIP_LINK_PATH=persist (one persistent
// launch), graph (per-step kernels replayed from a hipGraph), or auto.
static bool use_persistent(uint32_t n) {
    const char *e = getenv("DREPHIP_LINK_PATH");
    if (e && !strcmp(e, "graph")) return false;
    if (e && !strcmp(e, "persist")) return true;
    return kLinkPersistDefault && n <= kPMaxP * kPMaxSlice;
}

int linkage_device_impl(drephip_ctx *ctx, double *d_D, uint32_t n, int method, double *Z_out, hipStream_t st,
                        const std::function<int()> &rebuild) {
    if (n < 2) return DREPHIP_OK;
    const double t_chain = now_s();           // chain_s: scratch, graph capture and the steps
    if (method != DREPHIP_LINK_SINGLE && method != DREPHIP_LINK_COMPLETE && method != DREPHIP_LINK_AVERAGE &&
        method != DREPHIP_LINK_WEIGHTED) {
        set_error("linkage method must be single, complete, average or weighted");
        return DREPHIP_ERR_UNSUPPORTED;
    }
    ctx->link.path = 0;
    if (use_persistent(n) && n <= kPMaxP * kPMaxSlice) {
        double *d_Zp;
        int rc;
        if ((rc = scratch(ctx, "lk_Z", (n - 1) * 32ull, (void **)&d_Zp))) return rc;
        rc = linkage_persist(ctx, d_D, n, method, d_Zp, st);
        if (rc == DREPHIP_OK) {
            ctx->link.path = 1;
            const double t_fin = now_s();
            ctx->link.chain_s = t_fin - t_chain;
            std::vector<double> Z(4ull * (n - 1));
            HIPC(hipMemcpy(Z.data(), d_Zp, Z.size() * 8, hipMemcpyDeviceToHost));
            sort_and_label(Z, n);
            std::copy(Z.begin(), Z.end(), Z_out);
            ctx->link.finish_s = now_s() - t_fin;
            return DREPHIP_OK;
        }
        if (rc != DREPHIP_ERR_INTERNAL) return rc;
        // a participant timed out or the chain outgrew its LDS: the matrix may
        // hold partial Lance-Williams updates -- rebuilt, then the graph path
        fprintf(stderr, "[drephip] %s; running the per-step linkage path\n", drephip_last_error());
        if ((rc = rebuild())) return rc;
    }
    // entries per lane of a step, i.e. the grid density (default kLkPer: one pass;
    // DREPHIP_LINK_PER_LANE exists for the tests, which cover 1, 4 and 16)
    const char *pl = getenv("DREPHIP_LINK_PER_LANE");
    const uint32_t per = pl ? std::max(1, std::min(64, atoi(pl))) : 4;
    const uint32_t grid = std::max(1u, std::min(1024u, (n + kLkWG * per - 1) / (kLkWG * per)));
    int32_t *d_size, *d_chain;
    double *d_Z, *d_Dmin;
    LinkState *d_st;
    MinIdx *d_parts;
    int rc;
    if ((rc = scratch(ctx, "lk_size", n * 4ull, (void **)&d_size))) return rc;
    if ((rc = scratch(ctx, "lk_chain", n * 4ull, (void **)&d_chain))) return rc;
    if ((rc = scratch(ctx, "lk_Z", (n - 1) * 32ull, (void **)&d_Z))) return rc;
    if ((rc = scratch(ctx, "lk_st", sizeof(LinkState), (void **)&d_st))) return rc;
    if ((rc = scratch(ctx, "lk_parts", 1024 * sizeof(MinIdx), (void **)&d_parts))) return rc;
    const bool mst = method == DREPHIP_LINK_SINGLE;
    if (mst && (rc = scratch(ctx, "lk_dmin", n * 8ull, (void **)&d_Dmin))) return rc;
    LinkState h{};
    std::vector<int32_t> init(n, 1);
    if (mst) {
        std::vector<double> inf(n, INFINITY);
        std::vector<int32_t> mg(n, 0);
        mg[0] = 1;                                            // scipy: x = 0, merged[x] = 1
        HIPC(hipMemcpyAsync(d_size, mg.data(), n * 4ull, hipMemcpyHostToDevice, st));
        HIPC(hipMemcpyAsync(d_Dmin, inf.data(), n * 8ull, hipMemcpyHostToDevice, st));
        h.x = 0;
    } else {
        HIPC(hipMemcpyAsync(d_size, init.data(), n * 4ull, hipMemcpyHostToDevice, st));
        int32_t zero = 0;
        HIPC(hipMemcpyAsync(d_chain, &zero, 4, hipMemcpyHostToDevice, st));
        h.chain_len = 1;                                      // chain starts at the first active cluster, 0
        h.top = 0;
        h.below = -1;
    }
    HIPC(hipMemcpyAsync(d_st, &h, sizeof(h), hipMemcpyHostToDevice, st));
    // batches of steps captured once in a graph, replayed until every merge is done
    constexpr int kBatch = 256;
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    HIPC(hipStreamSynchronize(st));
    HIPC(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int b = 0; b < kBatch; b++) {
        if (mst) {
            hipLaunchKernelGGL(k_mst_step, dim3(grid), dim3(kLkWG), 0, st, d_D, n, d_size, d_Dmin, d_st, d_parts, d_Z);
        } else {
            hipLaunchKernelGGL(k_nn_step, dim3(grid), dim3(kLkWG), 0, st, d_D, n, method, d_size, d_chain, d_st,
                               d_parts, d_Z);
        }
    }
    HIPC(hipStreamEndCapture(st, &graph));
    hipError_t e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    if (e != hipSuccess) { (void)hipGraphDestroy(graph); HIPC(e); }
    // every search step either extends the chain or merges; the chain is at
    // most n long, so 3n steps always suffice (the bound only guards a hang)
    const uint64_t max_batches = (3ull * n) / kBatch + 2;
    int32_t done = 0;
    timing_mark(ctx, 2, st, true);
    for (uint64_t it = 0; it < max_batches; it++) {
        e = hipGraphLaunch(exec, st);
        if (e != hipSuccess) break;
        if ((it & 3) == 3 || it + 1 == max_batches) {
            e = hipMemcpyAsync(&done, &d_st->k, 4, hipMemcpyDeviceToHost, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            if (e != hipSuccess || done >= (int32_t)n - 1) break;
        }
    }
    timing_mark(ctx, 2, st, false);
    (void)hipGraphExecDestroy(exec);
    (void)hipGraphDestroy(graph);
    HIPC(e);
    HIPC(hipMemcpyAsync(&done, &d_st->k, 4, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    if (done != (int32_t)n - 1) { set_error("linkage did not finish"); return DREPHIP_ERR_INTERNAL; }
    int32_t bad = 0;
    HIPC(hipMemcpy(&bad, &d_st->bad, 4, hipMemcpyDeviceToHost));
    if (bad) { set_error("linkage: a chain step found no valid partial"); return DREPHIP_ERR_INTERNAL; }
    const double t_fin = now_s();
    ctx->link.chain_s = t_fin - t_chain;
    std::vector<double> Z(4ull * (n - 1));
    HIPC(hipMemcpy(Z.data(), d_Z, Z.size() * 8, hipMemcpyDeviceToHost));
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

}  // namespace drephip
