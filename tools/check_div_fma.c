/* check_div_fma.c — CPU check of the walker's division shortcut (rt_kernels.hip, RT_DIV_FMA):
 * fma(fma(-y, d, q), r, y) with r = RN(1/d), y = RN(q r) equals RN(q/d) inside the guard
 * (|q| >= 2^-900, 2^-960 <= |y| <= 2^960).  Random operands with random exponents and mantissas,
 * plus mantissas near 1 and near 2 (all-zero / all-one bit patterns), N pairs (argv[1], default 1e8).
 *   gcc -O2 -o /tmp/check_div_fma tools/check_div_fma.c -lm && /tmp/check_div_fma 100000000 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t s = 0x9e3779b97f4a7c15ull;
static uint64_t next(void)
{
    uint64_t z = (s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
static double mk(int emin, int emax)
{
    uint64_t r = next(), m;
    switch (r & 7) {
    case 0: m = 0; break;                                   /* 1.0 */
    case 1: m = (1ull << 52) - 1; break;                    /* 2 - ulp */
    case 2: m = (next() & 0xff); break;                     /* near 1 */
    case 3: m = ((1ull << 52) - 1) ^ (next() & 0xff); break; /* near 2 */
    default: m = next() & ((1ull << 52) - 1);
    }
    const int e = emin + (int)(next() % (uint64_t)(emax - emin + 1));
    uint64_t bits = ((uint64_t)(e + 1023) << 52) | m;
    if (r & 8) bits |= 1ull << 63;
    double x;
    memcpy(&x, &bits, 8);
    return x;
}
int main(int argc, char **argv)
{
    const long long N = argc > 1 ? atoll(argv[1]) : 100000000ll;
    long long used = 0, bad = 0;
    for (long long i = 0; i < N; i++) {
        const double q = mk(-900, 1000), d = fabs(mk(-1000, 996));
        const double r = 1.0 / d, y = q * r;
        if (!(fabs(q) >= 0x1p-900 && fabs(y) >= 0x1p-960 && fabs(y) <= 0x1p+960)) continue;
        used++;
        const double u = fma(fma(-y, d, q), r, y), want = q / d;
        if (memcmp(&u, &want, 8) != 0) {
            if (bad++ < 10) printf("MISMATCH q=%a d=%a got %a want %a\n", q, d, u, want);
        }
    }
    printf("%lld pairs in the guard, %lld mismatches\n", used, bad);
    return bad != 0;
}
