/* Exhaustive check: pt_sincosf.h against the host libm's sinf / cosf over
 * every float in (-120, 120).  Build: gcc -O2 -ffp-contract=off -mfma
 * tools/check_sincosf.c -lm (run by tests/test_sincosf.py on a sample). */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#define PT_SC_FMA fma
#include "../pathtracing_amd/csrc/pt_sincosf.h"
static const double T[2][14] = PT_SC_TABLE;

int main(int argc, char** argv) {
    /* argv[1]: stride over the float bit patterns (1 = exhaustive) */
    unsigned stride = argc > 1 ? (unsigned)atoi(argv[1]) : 1;
    unsigned long bad = 0, tot = 0;
    union { float f; unsigned u; } v;
    for (unsigned long u = 0; u < 0x42F00000ul; u += stride) { /* [0, 120) */
        v.u = (unsigned)u;
        for (int sgn = 0; sgn < 2; sgn++) {
            float x = sgn ? -v.f : v.f;
            float a = sinf(x), b = pt_sinf_t(x, T), c = cosf(x), d = pt_cosf_t(x, T);
            bad += memcmp(&a, &b, 4) != 0;
            bad += memcmp(&c, &d, 4) != 0;
            tot += 2;
        }
    }
    printf("%lu %lu\n", tot, bad);
    return bad != 0;
}
