// table.cpp -- MASH_table.tsv text writer (host only).
//
// Replaces the text `mash dist -p P ALL.msh ALL.msh > MASH_table.tsv` prints
// (drep/d_cluster.py:569-573): one line per ordered pair, the query as the
// outer loop, "reference\tquery\t%g dist\t%g p-value\tcommon/denom".  Mash
// prints doubles with C++ ostream defaults, which is printf's %g (6
// significant digits).  The numbers come from the caller (the condensed
// all-pairs result, its distances and p-values); this file only formats, on
// several threads, rows written in order.  N^2 lines: 10^8 at 10^4 genomes.
#include "ctx.h"
#include "../../include/drephip.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#define DREPHIP_EXPORT extern "C" __attribute__((visibility("default")))

namespace drephip {

static inline uint64_t cidx(uint64_t i, uint64_t j, uint64_t N) {      // i < j
    return i * N - i * (i + 1) / 2 + (j - i - 1);
}

// Row q of the table (every reference r against query q) appended to out.
static void format_row(std::string &out, uint32_t q, uint32_t N, const char *const *names,
                       const uint16_t *common, const uint16_t *denom, uint16_t s_denom, const double *dist,
                       const double *pval, const uint16_t *self_count, const double *self_pval) {
    char buf[96];
    const std::string qn = names[q];
    for (uint32_t r = 0; r < N; r++) {
        double d, p;
        unsigned c, dn;
        if (r == q) {
            d = 0.0;
            p = self_pval[q];
            c = dn = self_count[q];
        } else {
            const uint64_t t = r < q ? cidx(r, q, N) : cidx(q, r, N);
            d = dist[t];
            p = pval[t];
            c = common[t];
            dn = denom ? denom[t] : s_denom;
        }
        out += names[r];
        out += '\t';
        out += qn;
        const int n = snprintf(buf, sizeof(buf), "\t%g\t%g\t%u/%u\n", d, p, c, dn);
        out.append(buf, (size_t)n);
    }
}

}  // namespace drephip

using namespace drephip;

DREPHIP_EXPORT int drephip_write_mash_table(const char *path, const char *const *names, uint32_t N,
                                            const uint16_t *common, const uint16_t *denom, uint32_t s,
                                            const double *dist, const double *pval, const uint16_t *self_count,
                                            const double *self_pval, int threads) {
    if (!path || (N && (!names || !self_count || !self_pval))) { set_error("null argument"); return DREPHIP_ERR_ARG; }
    if (N > 1 && (!common || !dist || !pval)) { set_error("null argument"); return DREPHIP_ERR_ARG; }
    for (uint32_t i = 0; i < N; i++)
        if (!names[i]) { set_error("null genome name"); return DREPHIP_ERR_ARG; }
    FILE *fh = fopen(path, "wb");
    if (!fh) { set_error(std::string("cannot open ") + path); return DREPHIP_ERR_IO; }
    unsigned T = threads > 0 ? (unsigned)threads : std::thread::hardware_concurrency();
    T = std::max(1u, std::min(T, 64u));
    // blocks of rows formatted in parallel (row q by thread q % T), written in order
    const uint32_t block = std::max<uint32_t>(T, 4 * T);
    std::vector<std::string> rows(block);
    int rc = DREPHIP_OK;
    for (uint32_t q0 = 0; q0 < N && rc == DREPHIP_OK; q0 += block) {
        const uint32_t nb = std::min(block, N - q0);
        const unsigned Tb = std::min<unsigned>(T, nb);
        auto work = [&](unsigned t) {
            for (uint32_t i = t; i < nb; i += Tb) {
                rows[i].clear();
                format_row(rows[i], q0 + i, N, names, common, denom, (uint16_t)s, dist, pval, self_count, self_pval);
            }
        };
        std::vector<std::thread> pool;
        for (unsigned t = 1; t < Tb; t++) pool.emplace_back(work, t);
        work(0);
        for (auto &th : pool) th.join();
        for (uint32_t i = 0; i < nb; i++)
            if (fwrite(rows[i].data(), 1, rows[i].size(), fh) != rows[i].size()) {
                set_error(std::string("write failed: ") + path);
                rc = DREPHIP_ERR_IO;
                break;
            }
    }
    if (fclose(fh) != 0 && rc == DREPHIP_OK) { set_error(std::string("close failed: ") + path); rc = DREPHIP_ERR_IO; }
    return rc;
}
