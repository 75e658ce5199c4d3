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
//   runs    runs of >= 2 equal keys, appended by wave-aggregated atomics;
//           sum of m(m-1)/2 = the pair checks the marking will make
//   mark    one wave per run: every pair of the run's entries with equal
//           64-bit hashes marks cell (row tile of the smaller genome, larger
//           genome) in a bitmap [row tiles][N bits] (load first, atomicOr
//           only when the bit is clear: a family's ~400 shared hashes mark
//           the same cells)
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
#include <cstdlib>
#include <cstring>

namespace drephip {

constexpr int kScWG = 256;

// every entry (g, k < nhash[g]) at eoff[g] + k; one workgroup per genome
__global__ __launch_bounds__(kScWG) void k_screen_keys(const uint64_t *__restrict__ H, const uint32_t *__restrict__ nh,
                                                       const uint64_t *__restrict__ eoff, uint32_t s,
                                                       uint32_t *__restrict__ keys, uint32_t *__restrict__ vals) {
    const uint32_t g = blockIdx.x;
    const uint32_t n = nh[g];
    const uint64_t o = eoff[g];
    const uint64_t *A = H + (uint64_t)g * s;
    for (uint32_t k = threadIdx.x; k < n; k += kScWG) {
        keys[o + k] = (uint32_t)A[k];
        vals[o + k] = g * s + k;
    }
}

// total entry count after the exclusive scan of nhash (eoff[N] = eoff[N-1] + nh[N-1])
__global__ void k_screen_total(const uint32_t *__restrict__ nh, uint64_t *__restrict__ eoff, uint32_t N) {
    if (threadIdx.x == 0) eoff[N] = eoff[N - 1] + nh[N - 1];
}

// runs of >= 2 equal keys in the sorted keys: (start, length) appended to
// runs (wave-aggregated atomics), the sum of length (length - 1) / 2 to *E
__global__ __launch_bounds__(kScWG) void k_screen_runs(const uint32_t *__restrict__ keys, uint32_t M,
                                                       uint2 *__restrict__ runs, uint32_t *__restrict__ nruns,
                                                       unsigned long long *__restrict__ E) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t stride = gridDim.x * kScWG;
    // every lane of a wave runs the same number of iterations (ballots below)
    for (uint32_t i0 = blockIdx.x * kScWG; i0 < M; i0 += stride) {
        const uint32_t i = i0 + threadIdx.x;
        bool emit = false;
        uint32_t m = 0;
        if (i < M) {
            const uint32_t k = keys[i];
            const bool head = i == 0 || keys[i - 1] != k;
            if (head && i + 1 < M && keys[i + 1] == k) {
                uint32_t j = i + 2;
                while (j < M && keys[j] == k) j++;
                m = j - i;
                emit = true;
            }
        }
        const uint64_t mask = __ballot(emit);
        if (mask == 0) continue;
        uint32_t base = 0;
        unsigned long long e = emit ? (unsigned long long)m * (m - 1) / 2 : 0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) e += __shfl_xor(e, o, 64);
        const uint32_t first = (uint32_t)__ffsll((long long)mask) - 1;
        if (lane == first) {
            base = atomicAdd(nruns, (uint32_t)__popcll(mask));
            atomicAdd(E, e);
        }
        base = __shfl(base, first, 64);
        if (emit) {
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
            runs[base + rank] = make_uint2(i, m);
        }
    }
}

// One wave per run: the run's entries in 64-entry tiles (x tile <= y tile);
// lane l holds y entry yb + l, the x tile's entries are broadcast by readlane.
// Pairs with equal 64-bit hashes mark (tile of min g, max g) when the smaller
// genome is a row of this call.
__global__ __launch_bounds__(kScWG) void k_screen_mark(const uint32_t *__restrict__ vals, const uint64_t *__restrict__ H,
                                                       uint32_t s, const uint2 *__restrict__ runs,
                                                       const uint32_t *__restrict__ nruns_p, uint32_t row0,
                                                       uint32_t row1, uint32_t rshift, uint32_t NW,
                                                       uint32_t *__restrict__ bm) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nruns = *nruns_p;
    const uint32_t nwaves = gridDim.x * (kScWG / 64);
    for (uint32_t r = __builtin_amdgcn_readfirstlane(blockIdx.x * (kScWG / 64) + (threadIdx.x >> 6)); r < nruns;
         r += nwaves) {
        const uint2 run = runs[r];
        const uint32_t start = run.x, m = run.y;
        for (uint32_t yb = 0; yb < m; yb += 64) {
            const uint32_t y = yb + lane;
            const bool vy_ok = y < m;
            const uint32_t iy = vals[start + (vy_ok ? y : m - 1)];
            const uint32_t gy = iy / s;
            const uint64_t vy = H[iy];
            for (uint32_t xb = 0; xb <= yb; xb += 64) {
                const uint32_t xl = xb + lane;
                const uint32_t ix = vals[start + (xl < m ? xl : m - 1)];
                const uint32_t gxl = ix / s;
                const uint64_t vxl = H[ix];
                const uint32_t nx = min(64u, m - xb);
                for (uint32_t xi = 0; xi < nx; xi++) {
                    const uint32_t vlo = __builtin_amdgcn_readlane((uint32_t)vxl, xi);
                    const uint32_t vhi = __builtin_amdgcn_readlane((uint32_t)(vxl >> 32), xi);
                    const uint32_t gx = __builtin_amdgcn_readlane(gxl, xi);
                    const bool ok = vy_ok && xb + xi < y && (uint32_t)vy == vlo && (uint32_t)(vy >> 32) == vhi;
                    if (__ballot(ok) == 0) continue;
                    if (ok) {
                        const uint32_t a = min(gx, gy), b = max(gx, gy);
                        if (a >= row0 && a < row1) {
                            uint32_t *w = bm + (uint64_t)((a - row0) >> rshift) * NW + (b >> 5);
                            const uint32_t bit = 1u << (b & 31);
                            if (!(*w & bit)) atomicOr(w, bit);
                        }
                    }
                }
            }
        }
    }
}

// per row tile (one workgroup): marked columns -> cnt[t], items -> itc[t]
__global__ __launch_bounds__(kScWG) void k_screen_count(const uint32_t *__restrict__ bm, uint32_t NW, uint32_t C,
                                                        uint32_t *__restrict__ cnt, uint32_t *__restrict__ itc) {
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
        itc[t] = (tot + C - 1) / C;
    }
}

// per row tile (one workgroup): its marked columns in ascending order at
// coff[t], its items at ioff[t] (thread u takes words [u*per, (u+1)*per))
__global__ __launch_bounds__(kScWG) void k_screen_lists(const uint32_t *__restrict__ bm, uint32_t NW, uint32_t C,
                                                        uint32_t row0, uint32_t R, const uint32_t *__restrict__ cnt,
                                                        const uint64_t *__restrict__ coff,
                                                        const uint64_t *__restrict__ ioff, uint32_t *__restrict__ clist,
                                                        uint4 *__restrict__ items) {
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
    for (uint32_t w = w0; w < w1; w++) {
        uint32_t bits = row[w];
        while (bits) {
            const uint32_t b = __ffs(bits) - 1;
            bits &= bits - 1;
            out[pos++] = w * 32 + b;
        }
    }
    const uint32_t n = cnt[t];
    const uint32_t ni = (n + C - 1) / C;
    for (uint32_t j = tid; j < ni; j += kScWG)
        items[ioff[t] + j] = make_uint4(row0 + t * R, (uint32_t)(coff[t] + (uint64_t)j * C), min(C, n - j * C), 0);
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

template <class T>
static int hip_scan(drephip_ctx *ctx, const char *name, const uint32_t *in, T *out, uint32_t n, hipStream_t st) {
    size_t tb = 0;
    HIPC(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, in, out, n, st));
    void *tmp;
    int rc;
    if ((rc = scratch(ctx, name, std::max<size_t>(tb, 16), &tmp))) return rc;
    HIPC(hipcub::DeviceScan::ExclusiveSum(tmp, tb, in, out, n, st));
    return DREPHIP_OK;
}

int screen_impl(drephip_ctx *ctx, const uint64_t *d_hashes, const uint32_t *d_nhash, uint32_t N, uint32_t row0,
                uint32_t row1, uint32_t R, uint32_t C, uint64_t npairs, bool force, hipStream_t st, ScreenResult *res) {
    *res = ScreenResult{};
    const uint32_t s = ctx->s;
    if ((uint64_t)N * s >= (1ull << 32)) return DREPHIP_OK;          // entry values g * s + k are 32-bit
    int rc;
    uint64_t *d_eoff, *h_tot;
    if ((rc = scratch(ctx, "sc_eoff", (N + 1) * 8ull, (void **)&d_eoff))) return rc;
    if ((rc = pinned_host(ctx, "sc_tot", 32, (void **)&h_tot))) return rc;
    timing_mark(ctx, 4, st, true);
    if ((rc = hip_scan(ctx, "sc_scan_tmp0", d_nhash, d_eoff, N, st))) return rc;
    hipLaunchKernelGGL(k_screen_total, dim3(1), dim3(64), 0, st, d_nhash, d_eoff, N);
    HIPC(hipMemcpyAsync(h_tot, d_eoff + N, 8, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    const uint32_t M = (uint32_t)h_tot[0];
    uint32_t *k_in, *k_out, *v_in, *v_out, *d_nruns;
    uint2 *d_runs;
    unsigned long long *d_E;
    if ((rc = scratch(ctx, "sc_kin", M * 4ull + 16, (void **)&k_in))) return rc;
    if ((rc = scratch(ctx, "sc_kout", M * 4ull + 16, (void **)&k_out))) return rc;
    if ((rc = scratch(ctx, "sc_vin", M * 4ull + 16, (void **)&v_in))) return rc;
    if ((rc = scratch(ctx, "sc_vout", M * 4ull + 16, (void **)&v_out))) return rc;
    if ((rc = scratch(ctx, "sc_runs", (M / 2 + 1) * 8ull, (void **)&d_runs))) return rc;
    if ((rc = scratch(ctx, "sc_cnt", 16, (void **)&d_nruns))) return rc;
    d_E = (unsigned long long *)(d_nruns + 2);
    HIPC(hipMemsetAsync(d_nruns, 0, 16, st));
    hipLaunchKernelGGL(k_screen_keys, dim3(N), dim3(kScWG), 0, st, d_hashes, d_nhash, d_eoff, s, k_in, v_in);
    {
        size_t tb = 0;
        HIPC(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k_in, k_out, v_in, v_out, M, 0, 32, st));
        void *tmp;
        if ((rc = scratch(ctx, "sc_sort_tmp", std::max<size_t>(tb, 16), &tmp))) return rc;
        HIPC(hipcub::DeviceRadixSort::SortPairs(tmp, tb, k_in, k_out, v_in, v_out, M, 0, 32, st));
    }
    const uint32_t rgrid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(8192, (M + kScWG - 1) / kScWG));
    hipLaunchKernelGGL(k_screen_runs, dim3(rgrid), dim3(kScWG), 0, st, k_out, M, d_runs, d_nruns, d_E);
    HIPC(hipGetLastError());
    HIPC(hipMemcpyAsync(h_tot, d_nruns, 16, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    const uint32_t nruns = ((const uint32_t *)h_tot)[0];
    const uint64_t E = ((const unsigned long long *)h_tot)[1];
    res->entries = M;
    res->runs = nruns;
    res->checks = E;
    // dense set: a pair check costs about as much as a few probes of the
    // dense kernels, which make ~s/2 probes per pair (DREPHIP_SCREEN_RATIO
    // scales the bound; `force` skips it)
    const char *re = getenv("DREPHIP_SCREEN_RATIO");
    const double ratio = re ? atof(re) : 16.0;
    if (!force && (double)E * ratio > (double)npairs * s) { timing_mark(ctx, 4, st, false); return DREPHIP_OK; }

    const uint32_t rows = row1 - row0;
    const uint32_t ntiles = (rows + R - 1) / R;
    const uint32_t NW = (N + 31) / 32;
    uint32_t rshift = 0;
    while ((1u << rshift) < R) rshift++;
    uint32_t *d_bm, *d_cnt, *d_itc;
    uint64_t *d_coff, *d_ioff;
    if ((rc = scratch(ctx, "sc_bitmap", (uint64_t)ntiles * NW * 4, (void **)&d_bm))) return rc;
    if ((rc = scratch(ctx, "sc_tcnt", (ntiles + 1) * 4ull, (void **)&d_cnt))) return rc;
    if ((rc = scratch(ctx, "sc_titc", (ntiles + 1) * 4ull, (void **)&d_itc))) return rc;
    if ((rc = scratch(ctx, "sc_coff", (ntiles + 1) * 8ull, (void **)&d_coff))) return rc;
    if ((rc = scratch(ctx, "sc_ioff", (ntiles + 1) * 8ull, (void **)&d_ioff))) return rc;
    HIPC(hipMemsetAsync(d_bm, 0, (uint64_t)ntiles * NW * 4, st));
    if (nruns) {
        const uint32_t mgrid = std::max(1u, std::min(8192u, (nruns + 3) / 4));
        hipLaunchKernelGGL(k_screen_mark, dim3(mgrid), dim3(kScWG), 0, st, v_out, d_hashes, s, d_runs, d_nruns, row0,
                           row1, rshift, NW, d_bm);
    }
    hipLaunchKernelGGL(k_screen_count, dim3(ntiles), dim3(kScWG), 0, st, d_bm, NW, C, d_cnt, d_itc);
    // the last entry of each scan holds the totals: count entries ntiles + 1, the last one zero
    HIPC(hipMemsetAsync(d_cnt + ntiles, 0, 4, st));
    HIPC(hipMemsetAsync(d_itc + ntiles, 0, 4, st));
    if ((rc = hip_scan(ctx, "sc_scan_tmp1", d_cnt, d_coff, ntiles + 1, st))) return rc;
    if ((rc = hip_scan(ctx, "sc_scan_tmp2", d_itc, d_ioff, ntiles + 1, st))) return rc;
    HIPC(hipMemcpyAsync(h_tot, d_coff + ntiles, 8, hipMemcpyDeviceToHost, st));
    HIPC(hipMemcpyAsync(h_tot + 1, d_ioff + ntiles, 8, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    const uint64_t marked = h_tot[0], nitems = h_tot[1];
    res->marked = marked;
    if (marked >= (1ull << 32) || nitems >= (1ull << 31)) { timing_mark(ctx, 4, st, false); return DREPHIP_OK; }
    uint32_t *d_list;
    uint4 *d_items;
    if ((rc = scratch(ctx, "sc_list", std::max<uint64_t>(marked, 1) * 4, (void **)&d_list))) return rc;
    if ((rc = scratch(ctx, "sc_items", std::max<uint64_t>(nitems, 1) * 16, (void **)&d_items))) return rc;
    hipLaunchKernelGGL(k_screen_lists, dim3(ntiles), dim3(kScWG), 0, st, d_bm, NW, C, row0, R, d_cnt, d_coff, d_ioff,
                       d_list, d_items);
    timing_mark(ctx, 4, st, false);
    HIPC(hipGetLastError());
    res->use = true;
    res->clist = d_list;
    res->items = d_items;
    res->nitems = (uint32_t)nitems;
    return DREPHIP_OK;
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
