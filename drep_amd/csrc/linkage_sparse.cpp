// linkage_sparse.cpp -- primary clustering when most pairs sit at the largest
// distance: scipy.cluster.hierarchy.linkage (the call dRep's
// cluster_hierarchical makes, drep/d_cluster.py:453) replayed on the pairs
// below 1.0 only, bit-identical to scipy's dense algorithms.
//
// Mash's distance of two genomes that share no sketch hash is exactly 1.0, the
// top of its range (Mash clamps there; every pair sharing a hash is below
// 0.42 at s <= 12000).  In a set of many species almost every pair is such a
// pair: configs[3]'s 10^5 genomes (families of 100) have 0.1 % of their pairs
// below 1.0.  Listing only those pairs, scipy's two algorithms run without the
// n x n matrix and without its ~3n-step latency chain on the GPU:
//
//  * complete / average / weighted -- scipy's nn_chain (_hierarchy.pyx).
//    Lance-Williams of two 1.0 entries is exactly 1.0 (max(1,1); (nx*1 +
//    ny*1)/(nx+ny) with integer sizes; 0.5*(1+1)), and an update involving an
//    entry below 1.0 is at most 1.0 (rounding is monotone).  So an entry below
//    1.0 only ever appears between clusters of one connected component of the
//    listed pairs, and a component keeps its own dense m x m matrix.  A merge
//    below 1.0 joins two clusters of one component.  A merge at 1.0 joins two
//    clusters whose rows are all 1.0: the top's row minimum is 1.0, and the
//    element below it pushed the top at 1.0 -- its row minimum then -- while
//    the merges above it in the chain since then only wrote 1.0 into its row.
//    A row search that finds nothing below 1.0 resolves scipy's ties without
//    reading the other n entries: the previous chain element if there is one
//    (scipy prefers it), else the lowest active index (a linked list).
//  * single -- scipy's mst_single_linkage (Prim from vertex 0).  After the
//    first step every unmerged key is <= 1.0; keys below 1.0 sit in a heap
//    ordered by (key, index), and the lowest unmerged index stands for all
//    keys at 1.0 (scipy's scan keeps the first index of a minimum).
// Then scipy's stable sort of the merges by height and its relabel
// (sort_and_label, shared with the dense GPU path).
//
// The per-component matrices are bounded (max_cells): a set whose components
// are too large for them -- one species of 10^5 genomes -- takes the dense
// path (linkage.hip).  Compiled with -ffp-contract=off, like linkage.hip:
// scipy's x86-64 build rounds every operation on its own.

#include "ctx.h"
#include "../../include/drephip.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <queue>
#include <thread>
#include <vector>
#include <sys/mman.h>

namespace drephip {

static double host_now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// scipy's _hierarchy_distance_update.pxi, each operation rounded on its own
static inline double lw_host(int method, double dxi, double dyi, int32_t nx, int32_t ny) {
    if (method == DREPHIP_LINK_COMPLETE) return dxi > dyi ? dxi : (dyi > dxi ? dyi : dxi);
    if (method == DREPHIP_LINK_WEIGHTED) return 0.5 * (dxi + dyi);
    return ((double)nx * dxi + (double)ny * dyi) / (double)(nx + ny);
}

// scipy: Z sorted by distance (np.argsort kind='mergesort': stable), then
// `label` (union-find over 2n-1 nodes; the smaller root first; sizes).
void sort_and_label(std::vector<double> &Z, uint32_t n) {
    const uint32_t m = n - 1;
    std::vector<uint32_t> order(m);
    std::iota(order.begin(), order.end(), 0u);
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return Z[4ull * a + 2] < Z[4ull * b + 2]; });
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

namespace {

constexpr uint32_t kNone = 0xFFFFFFFFu;

// active clusters in index order: a doubly linked list (sentinel n)
struct ActiveList {
    std::vector<uint32_t> nx, pv;
    uint32_t n;
    explicit ActiveList(uint32_t n_) : nx(n_ + 1), pv(n_ + 1), n(n_) {   // 0 .. n-1 linked, n the sentinel
        for (uint32_t i = 0; i <= n; i++) {
            nx[i] = i == n ? 0 : i + 1;
            pv[i] = i == 0 ? n : i - 1;
        }
    }
    uint32_t first() const { return nx[n]; }
    uint32_t after(uint32_t i) const { return nx[i]; }
    void remove(uint32_t i) { nx[pv[i]] = nx[i]; pv[nx[i]] = pv[i]; }
};

struct Comp {
    uint64_t off;      // first cell of the m x m matrix
    uint32_t m;        // members
    uint32_t first;    // first member slot (members / alive)
};

// The matrices hold +inf on the diagonal and in the columns of merged-away
// clusters (and 1.0 in columns of clusters merged away at 1.0, which no search
// can pick either), so a row search is a plain scan for the first minimum
// below 1.0 and a merge update runs over the whole row: an update touching an
// inf entry yields inf again (max, (nx inf + ny d)/(nx + ny), 0.5 (inf + d)).
int chain_sparse(uint32_t n, const std::vector<uint32_t> &cid, const std::vector<uint32_t> &loc,
                 const std::vector<Comp> &comps, const std::vector<uint32_t> &members, double *mat,
                 int method, std::vector<double> &Z) {
    std::vector<int32_t> size(n, 1);
    ActiveList act(n);
    std::vector<uint32_t> chain(n);
    uint32_t len = 0;
    // each component's active members (local indices, ascending): the rows a
    // merge's column writes must reach
    std::vector<uint32_t> alist(members.size()), nal(comps.size());
    for (size_t c = 0; c < comps.size(); c++) {
        nal[c] = comps[c].m;
        std::iota(alist.begin() + comps[c].first, alist.begin() + comps[c].first + comps[c].m, 0u);
    }
    auto dist = [&](uint32_t a, uint32_t b) -> double {       // entry of two active clusters
        const uint32_t c = cid[a];
        if (c == kNone || c != cid[b]) return 1.0;
        return mat[comps[c].off + (uint64_t)loc[a] * comps[c].m + loc[b]];
    };
    for (uint32_t k = 0; k + 1 < n; k++) {
        if (len == 0) { chain[0] = act.first(); len = 1; }
        uint32_t x, y;
        double cur;
        for (;;) {
            x = chain[len - 1];
            // row minimum below 1.0 within x's component, lowest index on ties
            double best = 1.0;
            uint32_t by = kNone;
            const uint32_t c = cid[x];
            if (c != kNone) {
                const Comp &C = comps[c];
                const double *row = &mat[C.off + (uint64_t)loc[x] * C.m];
                for (uint32_t l = 0; l < C.m; l++) best = row[l] < best ? row[l] : best;
                if (best < 1.0) {
                    uint32_t l = 0;
                    while (row[l] != best) l++;
                    by = members[C.first + l];
                }
            }
            if (len > 1) {
                // scipy: current_min = D[x, prev], y = prev; only a strictly
                // smaller entry replaces it
                const uint32_t pvx = chain[len - 2];
                const double dp = dist(x, pvx);
                if (by != kNone && best < dp) { y = by; cur = best; }
                else { y = pvx; cur = dp; break; }
            } else if (by != kNone) {
                y = by; cur = best;
            } else {                                              // every entry is 1.0
                y = act.first() == x ? act.after(x) : act.first();
                cur = 1.0;
            }
            if (len >= n) return DREPHIP_ERR_INTERNAL;
            chain[len++] = y;
        }
        len -= 2;
        if (x > y) std::swap(x, y);
        const int32_t nx = size[x], ny = size[y];
        Z[4ull * k] = x; Z[4ull * k + 1] = y; Z[4ull * k + 2] = cur; Z[4ull * k + 3] = nx + ny;
        size[x] = 0;
        size[y] = nx + ny;
        act.remove(x);
        const uint32_t cx = cid[x], cy = cid[y];
        if (cx != kNone && cx == cy) {
            const Comp &C = comps[cx];
            double *M = &mat[C.off];
            const uint32_t m = C.m, lx = loc[x], ly = loc[y];
            double *rx = M + (uint64_t)lx * m, *ry = M + (uint64_t)ly * m;
            uint32_t *al = &alist[C.first];
            const uint32_t na = nal[cx];
            uint32_t w = 0;
            for (uint32_t e = 0; e < na; e++) {
                const uint32_t l = al[e];
                if (l == lx) continue;
                al[w++] = l;
                const double u = lw_host(method, rx[l], ry[l], nx, ny);
                ry[l] = u;
                M[(uint64_t)l * m + ly] = u;
                M[(uint64_t)l * m + lx] = INFINITY;
            }
            nal[cx] = w;
            ry[lx] = INFINITY;
        } else {
            // two clusters of different components meet only at 1.0, with
            // rows of 1.0 (see the header); anything else is a broken input
            if (cur != 1.0) return DREPHIP_ERR_INTERNAL;
            if (cx != kNone) {                                    // x leaves its component's active rows
                uint32_t *al = &alist[comps[cx].first];
                const uint32_t na = nal[cx];
                uint32_t w = 0;
                for (uint32_t e = 0; e < na; e++) if (al[e] != loc[x]) al[w++] = al[e];
                nal[cx] = w;
            }
            for (uint32_t v : {x, y}) {
                const uint32_t c = cid[v];
                if (c == kNone) continue;
                const Comp &C = comps[c];
                const double *row = &mat[C.off + (uint64_t)loc[v] * C.m];
                for (uint32_t l = 0; l < C.m; l++)
                    if (row[l] < 1.0) return DREPHIP_ERR_INTERNAL;
            }
        }
    }
    return DREPHIP_OK;
}

// scipy's Prim (mst_single_linkage) restricted to one component: its members
// in index order, its matrix with 1.0 off the listed pairs.  Prim from the
// component's lowest member reaches every member through keys below 1.0
// before any key at 1.0 can win, so the global run is the components' runs in
// the order of their lowest members, joined by steps at 1.0 (stitch_mst).
// Writes the component's m - 1 steps (x, y, key) into out.
void prim_component(const Comp &C, const uint32_t *members, const double *mat, double *out) {
    const uint32_t m = C.m;
    std::vector<double> key(m, INFINITY);
    std::vector<uint8_t> done(m, 0);
    uint32_t x = 0;
    for (uint32_t k = 0; k + 1 < m; k++) {
        done[x] = 1;
        const double *row = mat + (uint64_t)x * m;
        double cur = INFINITY;
        uint32_t y = kNone;
        for (uint32_t i = 0; i < m; i++) {
            if (done[i]) continue;
            if (key[i] > row[i]) key[i] = row[i];
            if (key[i] < cur) { cur = key[i]; y = i; }
        }
        out[3ull * k] = members[x];
        out[3ull * k + 1] = members[y];
        out[3ull * k + 2] = cur;
        x = y;
    }
}

// ---------------------------------------------------------------------------
// The sparse-row chain: scipy's nn_chain without any matrix, for a set whose
// pairs below 1.0 join (almost) everything into one component -- Mash data at
// scale, where chance shared hashes link unrelated genomes.  Every cluster
// keeps the entries of its row below 1.0; an entry not stored is 1.0.
//
// Rows are never searched or edited in place.  Cluster c's row has two parts:
//   own[c]   the row written when c was formed (stamp[c]; the input pairs for
//            a genome, stamp 0): its entry for j is current while j has not
//            been re-formed since (stamp[j] <= stamp[c]), and
//   newer[c] entries (j, t, v) appended when a merge formed j at time t with
//            an entry for c: current while stamp[j] == t.
// Clusters merged away (size 0) are skipped everywhere.  So a merge of x into
// y writes y's new row once (Lance-Williams over the union of the two rows,
// 1.0 where a row has no entry) and appends one entry to each neighbour's
// newer list -- no lookups in other rows.  A search of row x reads x's two
// lists only (and drops the stale entries it meets); the ties follow scipy's
// scan as in chain_sparse: the previous chain element when nothing is
// strictly smaller, else the lowest index of the row minimum; with nothing
// below 1.0 and no previous element, the lowest active index.
struct REnt {
    uint32_t j, t;
    double v;
};

struct RList {                 // malloc'd entry list; cap == 0: a slice of the input arrays (not owned)
    REnt *p = nullptr;
    uint32_t len = 0, cap = 0;
    void release() {
        if (cap) free(p);
        p = nullptr; len = cap = 0;
    }
};

struct RowsChain {
    uint32_t n;
    int method;
    std::vector<uint64_t> meta;    // size (low 32 bits, 0 = merged away) | stamp << 32
    std::vector<RList> own, nw;
    std::vector<REnt> base;        // the input pairs, both directions, grouped by row
    std::vector<uint32_t> ep;      // merge scratch, per cluster
    std::vector<double> vx, vy;
    std::vector<uint32_t> touched;
    std::vector<REnt> row;
    bool dup = false;              // a pair listed twice (the caller refuses the list)
    uint64_t scanned = 0, appended = 0, scans = 0;
    double t_scan = 0, t_gather = 0, t_row = 0, t_append = 0;
    bool oom = false;

    static uint32_t size_of(uint64_t m) { return (uint32_t)m; }
    static uint32_t stamp_of(uint64_t m) { return (uint32_t)(m >> 32); }

    RowsChain(uint32_t n_, uint64_t np, const uint32_t *pi, const uint32_t *pj, const double *pv, int method_)
        : n(n_), method(method_), meta(n_, 1), own(n_), nw(n_), ep(n_, 0), vx(n_), vy(n_) {
        std::vector<uint64_t> off(n + 1, 0);
        for (uint64_t t = 0; t < np; t++) { off[pi[t] + 1]++; off[pj[t] + 1]++; }
        for (uint32_t v = 0; v < n; v++) off[v + 1] += off[v];
        base.resize(2 * np);
        std::vector<uint64_t> w(off.begin(), off.end() - 1);
        for (uint64_t t = 0; t < np; t++) {
            base[w[pi[t]]++] = REnt{pj[t], 0, pv[t]};
            base[w[pj[t]]++] = REnt{pi[t], 0, pv[t]};
        }
        for (uint32_t v = 0; v < n; v++) { own[v].p = base.data() + off[v]; own[v].len = (uint32_t)(off[v + 1] - off[v]); }
        // a pair listed twice shows as a repeated index in a row (host threads over row ranges)
        const unsigned T = std::max(1u, std::min(host_threads(), n / 1024 + 1));
        std::atomic<bool> d(false);
        std::vector<std::thread> pool;
        for (unsigned k = 0; k < T; k++)
            pool.emplace_back([&, k] {
                std::vector<uint32_t> mark(n, 0);
                for (uint32_t v = (uint32_t)((uint64_t)n * k / T); v < (uint32_t)((uint64_t)n * (k + 1) / T); v++)
                    for (uint64_t e = off[v]; e < off[v + 1]; e++) {
                        if (mark[base[e].j] == v + 1) { d = true; return; }
                        mark[base[e].j] = v + 1;
                    }
            });
        for (auto &th : pool) th.join();
        dup = d.load();
    }
    ~RowsChain() {
        for (auto &l : own) l.release();
        for (auto &l : nw) l.release();
    }

    bool append(RList &l, const REnt &e) {
        if (l.len == l.cap) {
            // first drop the stale entries; grow only if at least half remain
            uint32_t w = 0;
            for (uint32_t a = 0; a < l.len; a++) {
                const uint64_t m = meta[l.p[a].j];
                if (size_of(m) && stamp_of(m) == l.p[a].t) l.p[w++] = l.p[a];
            }
            l.len = w;
            if (w + 1 > l.cap / 2) {
                const uint32_t nc = std::max<uint32_t>(16, l.cap * 2);
                REnt *q = (REnt *)realloc(l.p, (size_t)nc * sizeof(REnt));
                if (!q) { oom = true; return false; }
                l.p = q; l.cap = nc;
            }
        }
        l.p[l.len++] = e;
        return true;
    }

    // calls f(j, v) for every current entry of x's row, compacting both lists
    template <class F> void visit(uint32_t x, F f) {
        const uint32_t sx = stamp_of(meta[x]);
        RList &o = own[x];
        uint32_t w = 0;
        for (uint32_t a = 0; a < o.len; a++) {
            const REnt e = o.p[a];
            const uint64_t m = meta[e.j];
            if (!size_of(m) || stamp_of(m) > sx) continue;
            o.p[w++] = e;
            f(e.j, e.v);
        }
        scanned += o.len;
        o.len = w;
        RList &q = nw[x];
        w = 0;
        for (uint32_t a = 0; a < q.len; a++) {
            const REnt e = q.p[a];
            const uint64_t m = meta[e.j];
            if (!size_of(m) || stamp_of(m) != e.t) continue;
            q.p[w++] = e;
            f(e.j, e.v);
        }
        scanned += q.len;
        q.len = w;
    }

    int run(std::vector<double> &Z) {
        ActiveList act(n);
        std::vector<uint32_t> chain(n);
        uint32_t len = 0, clock = 0, epoch = 0;
        for (uint32_t k = 0; k + 1 < n; k++) {
            if (len == 0) { chain[0] = act.first(); len = 1; }
            uint32_t x, y;
            double cur;
            double ta = host_now_s();
            for (;;) {
                x = chain[len - 1];
                scans++;
                const uint32_t pvx = len > 1 ? chain[len - 2] : kNone;
                double best = INFINITY, dp = 1.0;
                uint32_t by = kNone;
                visit(x, [&](uint32_t j, double v) {
                    if (v < best || (v == best && j < by)) { best = v; by = j; }
                    if (j == pvx) dp = v;
                });
                if (len > 1) {
                    if (best < dp) { y = by; cur = best; }
                    else { y = pvx; cur = dp; break; }
                } else if (best < 1.0) {
                    y = by; cur = best;
                } else {                                          // every entry is 1.0
                    y = act.first() == x ? act.after(x) : act.first();
                    cur = 1.0;
                }
                if (len >= n) return DREPHIP_ERR_INTERNAL;
                chain[len++] = y;
            }
            len -= 2;
            double tb = host_now_s();
            t_scan += tb - ta;
            if (x > y) std::swap(x, y);
            const uint32_t nx = size_of(meta[x]), ny = size_of(meta[y]);
            Z[4ull * k] = x; Z[4ull * k + 1] = y; Z[4ull * k + 2] = cur; Z[4ull * k + 3] = nx + ny;
            // y's new row: Lance-Williams over the union of the two rows
            epoch++;
            touched.clear();
            visit(x, [&](uint32_t j, double v) {
                if (j == y) return;
                ep[j] = epoch; vx[j] = v; vy[j] = 1.0;
                touched.push_back(j);
            });
            visit(y, [&](uint32_t j, double v) {
                if (j == x) return;
                if (ep[j] == epoch) { vy[j] = v; return; }
                ep[j] = epoch; vx[j] = 1.0; vy[j] = v;
                touched.push_back(j);
            });
            const uint32_t T = ++clock;
            double tc = host_now_s();
            t_gather += tc - tb;
            row.clear();
            for (uint32_t j : touched) {
                const double u = lw_host(method, vx[j], vy[j], (int32_t)nx, (int32_t)ny);
                if (u < 1.0) row.push_back(REnt{j, T, u});
            }
            scanned += touched.size();
            meta[x] = 0;
            meta[y] = (uint64_t)(nx + ny) | (uint64_t)T << 32;
            act.remove(x);
            own[x].release(); nw[x].release(); own[y].release(); nw[y].len = 0;
            double td = host_now_s();
            t_row += td - tc;
            appended += row.size();
            if (!row.empty()) {
                RList &o = own[y];
                o.p = (REnt *)malloc(row.size() * sizeof(REnt));
                if (!o.p) return DREPHIP_ERR_NOMEM;
                o.cap = o.len = (uint32_t)row.size();
                std::copy(row.begin(), row.end(), o.p);
                for (const REnt &e : row)
                    if (!append(nw[e.j], REnt{y, T, e.v})) return DREPHIP_ERR_NOMEM;
            }
            t_append += host_now_s() - td;
        }
        if (std::getenv("DREPHIP_DEBUG"))
            fprintf(stderr, "[drephip] rows chain: scans %llu appended %llu; scan %.3f gather %.3f row %.3f append %.3f s\n",
                    (unsigned long long)scans, (unsigned long long)appended, t_scan, t_gather, t_row, t_append);
        return oom ? DREPHIP_ERR_NOMEM : DREPHIP_OK;
    }
};

// scipy's Prim (mst_single_linkage) over the sparse rows: keys below 1.0 in a
// heap ordered by (key, index) (stale heap entries skipped), the lowest
// unmerged index for a minimum at 1.0 -- after the first step every unmerged
// key is <= 1.0, and scipy's scan keeps the first index of a minimum.
int prim_rows(uint32_t n, uint64_t np, const uint32_t *pi, const uint32_t *pj, const double *pv,
              std::vector<double> &Z, uint64_t *scanned) {
    std::vector<uint64_t> off(n + 1, 0);
    for (uint64_t t = 0; t < np; t++) { off[pi[t] + 1]++; off[pj[t] + 1]++; }
    for (uint32_t v = 0; v < n; v++) off[v + 1] += off[v];
    std::vector<uint32_t> adj(2 * np);
    std::vector<double> av(2 * np);
    {
        std::vector<uint64_t> w(off.begin(), off.end() - 1);
        for (uint64_t t = 0; t < np; t++) {
            adj[w[pi[t]]] = pj[t]; av[w[pi[t]]++] = pv[t];
            adj[w[pj[t]]] = pi[t]; av[w[pj[t]]++] = pv[t];
        }
    }
    {
        std::vector<uint32_t> mark(n, 0);
        for (uint32_t v = 0; v < n; v++)
            for (uint64_t e = off[v]; e < off[v + 1]; e++) {
                if (mark[adj[e]] == v + 1) return DREPHIP_ERR_ARG;
                mark[adj[e]] = v + 1;
            }
    }
    std::vector<double> key(n, 1.0);
    std::vector<uint8_t> merged(n, 0);
    ActiveList act(n);
    using HE = std::pair<double, uint32_t>;
    std::priority_queue<HE, std::vector<HE>, std::greater<HE>> heap;
    uint32_t x = 0;
    for (uint32_t k = 0; k + 1 < n; k++) {
        merged[x] = 1;
        act.remove(x);
        for (uint64_t e = off[x]; e < off[x + 1]; e++) {
            const uint32_t i = adj[e];
            if (!merged[i] && av[e] < key[i]) { key[i] = av[e]; heap.push(HE(av[e], i)); }
        }
        *scanned += off[x + 1] - off[x];
        while (!heap.empty() && (merged[heap.top().second] || heap.top().first != key[heap.top().second])) heap.pop();
        uint32_t y;
        double cur;
        if (!heap.empty()) { y = heap.top().second; cur = heap.top().first; heap.pop(); }
        else { y = act.first(); cur = 1.0; }
        if (y >= n) return DREPHIP_ERR_INTERNAL;
        Z[4ull * k] = x; Z[4ull * k + 1] = y; Z[4ull * k + 2] = cur; Z[4ull * k + 3] = 0;
        x = y;
    }
    return DREPHIP_OK;
}

}  // namespace

unsigned host_threads() {
    unsigned t = std::thread::hardware_concurrency();
    if (const char *e = std::getenv("OMP_NUM_THREADS")) t = (unsigned)std::max(1, atoi(e));
    return std::max(1u, std::min(t, 16u));
}

// fn(c) for every component, on host_threads() threads (dynamic)
template <class F> static void for_components(size_t nc, F fn) {
    const unsigned T = (unsigned)std::min<size_t>(host_threads(), nc);
    if (T <= 1) { for (size_t c = 0; c < nc; c++) fn(c); return; }
    std::atomic<size_t> next(0);
    std::vector<std::thread> pool;
    for (unsigned t = 0; t < T; t++)
        pool.emplace_back([&] { for (size_t c; (c = next.fetch_add(1)) < nc;) fn(c); });
    for (auto &th : pool) th.join();
}

int linkage_sparse_impl(uint32_t n, uint64_t np, const uint32_t *pi, const uint32_t *pj, const double *pv,
                        int method, uint64_t max_cells, uint32_t max_comp, double *Z_out, SparseLinkInfo *info,
                        int rows) {
    SparseLinkInfo loc_info;
    SparseLinkInfo &I = info ? *info : loc_info;
    I = SparseLinkInfo{};
    I.pairs = np;
    if (n < 2) return DREPHIP_OK;
    if (method != DREPHIP_LINK_SINGLE && method != DREPHIP_LINK_COMPLETE && method != DREPHIP_LINK_AVERAGE &&
        method != DREPHIP_LINK_WEIGHTED) {
        set_error("linkage method must be single, complete, average or weighted");
        return DREPHIP_ERR_UNSUPPORTED;
    }
    const double t0 = host_now_s();
    const double tv = t0;
    // connected components of the listed pairs (union-find, path halving)
    std::vector<uint32_t> cid(n);
    std::iota(cid.begin(), cid.end(), 0u);
    auto find = [&](uint32_t a) {
        while (cid[a] != a) { cid[a] = cid[cid[a]]; a = cid[a]; }
        return a;
    };
    for (uint64_t t = 0; t < np; t++) {
        if (pi[t] >= n || pj[t] >= n || pi[t] == pj[t]) { set_error("sparse linkage: pair index out of range or i == j"); return DREPHIP_ERR_ARG; }
        if (!(pv[t] < 1.0) || !(pv[t] >= 0.0)) {
            set_error("sparse linkage: every listed distance must be in [0, 1) (unlisted pairs are 1.0)");
            return DREPHIP_ERR_ARG;
        }
        uint32_t a = find(pi[t]), b = find(pj[t]);
        if (a != b) { if (a < b) std::swap(a, b); cid[a] = b; }     // root = the smallest member
    }
    const double tu = host_now_s();
    // components with >= 2 members, numbered by their smallest member (the root)
    std::vector<Comp> comps;
    std::vector<uint32_t> loc(n, 0);
    uint32_t slots = 0;
    {
        std::vector<uint32_t> root(n), rid(n), cnt;
        for (uint32_t v = 0; v < n; v++) {
            const uint32_t r = find(v);                          // r <= v: seen first
            root[v] = r;
            if (r == v) { rid[v] = (uint32_t)cnt.size(); cnt.push_back(1); }
            else cnt[rid[r]]++;
        }
        std::vector<uint32_t> remap(cnt.size(), kNone);
        uint64_t cells = 0;
        for (size_t c = 0; c < cnt.size(); c++) {
            if (cnt[c] < 2) continue;
            remap[c] = (uint32_t)comps.size();
            comps.push_back(Comp{cells, cnt[c], slots});
            cells += (uint64_t)cnt[c] * cnt[c];
            slots += cnt[c];
            I.largest = std::max(I.largest, cnt[c]);
        }
        I.components = (uint32_t)comps.size();
        I.cells = cells;
        if (const char *e = std::getenv("DREPHIP_LINK_ROWS")) rows = atoi(e);
        if (rows == 2 || (rows == 1 && (cells > max_cells || I.largest > max_comp))) {
            I.rows = 1;
            I.setup_s = host_now_s() - t0;
            std::vector<double> Z(4ull * (n - 1));
            int rc;
            if (method == DREPHIP_LINK_SINGLE) {
                rc = prim_rows(n, np, pi, pj, pv, Z, &I.scanned);
            } else {
                RowsChain rc_chain(n, np, pi, pj, pv, method);
                rc = rc_chain.dup ? DREPHIP_ERR_ARG : rc_chain.run(Z);
                I.scanned = rc_chain.scanned;
            }
            if (rc == DREPHIP_ERR_ARG) { set_error("sparse linkage: a pair is listed twice"); return rc; }
            if (rc) {
                set_error(rc == DREPHIP_ERR_NOMEM ? "sparse linkage: host allocation failed"
                                                  : "sparse linkage: inconsistent chain state");
                return rc;
            }
            const double t1 = host_now_s();
            I.chain_s = t1 - t0 - I.setup_s;
            sort_and_label(Z, n);
            std::copy(Z.begin(), Z.end(), Z_out);
            I.finish_s = host_now_s() - t1;
            if (std::getenv("DREPHIP_DEBUG"))
                fprintf(stderr, "[drephip] sparse-row linkage: n=%u pairs=%llu largest=%u setup %.4f s chain %.4f s "
                        "(%.3g entries read) finish %.4f s\n", n, (unsigned long long)np, I.largest, I.setup_s,
                        I.chain_s, (double)I.scanned, I.finish_s);
            return DREPHIP_OK;
        }
        if (cells > max_cells || I.largest > max_comp) {
            set_error("sparse linkage: the components need " + std::to_string(cells) + " matrix cells (limit " +
                      std::to_string(max_cells) + "), the largest has " + std::to_string(I.largest) +
                      " members (limit " + std::to_string(max_comp) + ")");
            return DREPHIP_ERR_UNSUPPORTED;
        }
        // v -> component (kNone: a singleton) and its index among the members
        std::vector<uint32_t> fill(comps.size(), 0);
        for (uint32_t v = 0; v < n; v++) {
            const uint32_t c = remap[rid[root[v]]];
            cid[v] = c;
            loc[v] = c == kNone ? 0 : fill[c]++;
        }
    }
    std::vector<uint32_t> members(n);
    for (uint32_t v = 0; v < n; v++) if (cid[v] != kNone) members[comps[cid[v]].first + loc[v]] = v;
    const double tc = host_now_s(), tb = tc;
    // per-component matrices on host threads: 2.0 (= not listed) everywhere,
    // the pairs written from equal slices of the list, then 2.0 -> 1.0; a pair
    // listed twice leaves fewer written cells than 2 per pair
    // one arena, 2 MB pages where the kernel grants them (80 MB at 10^5
    // genomes in families of 100: 40 page faults instead of 20,000)
    struct Arena {
        double *p = nullptr;
        ~Arena() { free(p); }
        double *data() const { return p; }
    } mat;
    {
        const size_t bytes = std::max<uint64_t>(I.cells, 1) * sizeof(double);
        void *p = nullptr;
        if (posix_memalign(&p, 1u << 21, (bytes + (1u << 21) - 1) & ~(size_t)((1u << 21) - 1))) {
            set_error("sparse linkage: host allocation failed");
            return DREPHIP_ERR_NOMEM;
        }
        madvise(p, bytes, MADV_HUGEPAGE);
        mat.p = (double *)p;
    }
    for_components(comps.size(), [&](size_t c) {
        const Comp &C = comps[c];
        std::fill(mat.data() + C.off, mat.data() + C.off + (uint64_t)C.m * C.m, 2.0);
    });
    const double tf = host_now_s();
    const unsigned T = host_threads();
    for_components(T, [&](size_t part) {
        const uint64_t a0 = np * part / T, a1 = np * (part + 1) / T;
        for (uint64_t t = a0; t < a1; t++) {
            const Comp &C = comps[cid[pi[t]]];
            double *M = mat.data() + C.off;
            M[(uint64_t)loc[pi[t]] * C.m + loc[pj[t]]] = pv[t];
            M[(uint64_t)loc[pj[t]] * C.m + loc[pi[t]]] = pv[t];
        }
    });
    const double tw = host_now_s();
    std::atomic<uint64_t> written(0);
    for_components(comps.size(), [&](size_t c) {
        const Comp &C = comps[c];
        double *M = mat.data() + C.off;
        uint64_t w = 0;
        for (uint64_t e = 0; e < (uint64_t)C.m * C.m; e++) {
            if (M[e] == 2.0) M[e] = 1.0;
            else w++;
        }
        for (uint32_t l = 0; l < C.m; l++) M[(uint64_t)l * C.m + l] = INFINITY;     // (2.0 there: not counted)
        written += w;
    });
    if (std::getenv("DREPHIP_DEBUG")) fprintf(stderr, "[drephip] matrices: init %.4f write %.4f final %.4f\n", tf - tb, tw - tf, host_now_s() - tw);
    if (written.load() != 2 * np) { set_error("sparse linkage: a pair is listed twice"); return DREPHIP_ERR_ARG; }
    I.setup_s = host_now_s() - t0;
    std::vector<double> Z(4ull * (n - 1));
    int rc = DREPHIP_OK;
    if (method == DREPHIP_LINK_SINGLE) {
        // every component's Prim run (in parallel), then scipy's order: from
        // vertex 0, each component from its lowest member, a step at 1.0 to
        // the lowest unmerged vertex between them
        std::vector<double> runs(3ull * (slots - comps.size()));   // m - 1 steps per component
        for_components(comps.size(), [&](size_t c) {
            const Comp &C = comps[c];
            prim_component(C, members.data() + C.first, mat.data() + C.off, runs.data() + 3ull * (C.first - c));
        });
        uint64_t k = 0;
        uint32_t x = kNone;
        for (uint32_t v = 0; v < n; v++) {           // v: lowest member of the next component (or a singleton)
            if (cid[v] != kNone && loc[v] != 0) continue;
            if (x != kNone) {
                Z[4 * k] = x; Z[4 * k + 1] = v; Z[4 * k + 2] = 1.0; Z[4 * k + 3] = 0; k++;
            }
            x = v;
            if (cid[v] != kNone) {
                const Comp &C = comps[cid[v]];
                const double *r = runs.data() + 3ull * (C.first - cid[v]);
                for (uint32_t e = 0; e + 1 < C.m; e++, k++) {
                    Z[4 * k] = r[3 * e]; Z[4 * k + 1] = r[3 * e + 1]; Z[4 * k + 2] = r[3 * e + 2]; Z[4 * k + 3] = 0;
                }
                x = (uint32_t)r[3ull * (C.m - 2) + 1];
            }
        }
        if (k != n - 1) rc = DREPHIP_ERR_INTERNAL;
    } else {
        rc = chain_sparse(n, cid, loc, comps, members, mat.data(), method, Z);
    }
    if (rc) {
        if (rc == DREPHIP_ERR_INTERNAL) set_error("sparse linkage: inconsistent chain state");
        return rc;
    }
    const double t1 = host_now_s();
    I.chain_s = t1 - t0 - I.setup_s;
    sort_and_label(Z, n);
    std::copy(Z.begin(), Z.end(), Z_out);
    I.finish_s = host_now_s() - t1;
    if (std::getenv("DREPHIP_DEBUG"))
        fprintf(stderr, "[drephip] sparse linkage setup: check %.4f union %.4f comps %.4f bucket %.4f matrices %.4f\n",
                tv - t0, tu - tv, tc - tu, tb - tc, t0 + I.setup_s - tb),
        fprintf(stderr, "[drephip] sparse linkage: n=%u pairs=%llu components=%u largest=%u cells=%llu setup %.4f s chain %.4f s finish %.4f s\n",
                n, (unsigned long long)np, I.components, I.largest, (unsigned long long)I.cells, I.setup_s, I.chain_s, I.finish_s);
    return DREPHIP_OK;
}

}  // namespace drephip
