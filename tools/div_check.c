/* Host check of linkage.hip lw_update(..., LwDiv): Markstein's correction step
 * RN(q + fma(-q, n, a) r), r = RN(1/n), q = RN(a r), against the IEEE division
 * a / n for the average update's operands (a = RN(RN(nx dx) + RN(ny dy)), dx, dy
 * in [0, 1], n = nx + ny <= 2 x 10^5).  Not product code.
 * gcc -O2 -ffp-contract=off -o /tmp/div_check tools/div_check.c -lm && /tmp/div_check */
#include <math.h>
#include <stdio.h>
#include <stdint.h>
static uint64_t s = 88172645463325252ull;
static inline uint64_t xr(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
int main(void) {
    uint64_t bad = 0, n = 0;
    for (uint64_t it = 0; it < 400000000ull; it++) {
        uint32_t nx = 1 + xr() % 100000, ny = 1 + xr() % 100000;
        if (it & 1) { nx = 1 + xr() % 8; ny = 1 + xr() % 8; }
        double dx = (double)(xr() >> 11) * 0x1p-53, dy = (double)(xr() >> 11) * 0x1p-53;
        if ((it & 7) == 2) dx = 1.0;
        if ((it & 15) == 3) dy = 0.0;
        if ((it & 31) == 5) dx = (double)(xr() % 10001) / 10000.0;
        volatile double a1 = (double)nx * dx, a2 = (double)ny * dy;
        volatile double a = a1 + a2;
        double d = (double)(nx + ny);
        double ref = a / d;
        double y = 1.0 / d;
        double q = a * y;
        double e = fma(-q, d, a);
        double q2 = fma(e, y, q);
        n++;
        if (q2 != ref) { if (bad < 5) printf("mismatch a=%a d=%a ref=%a got=%a\n", a, d, ref, q2); bad++; }
    }
    printf("%llu cases, %llu mismatches\n", (unsigned long long)n, (unsigned long long)bad);
    return 0;
}
