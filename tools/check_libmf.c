/* Check pathtracing_amd/csrc/pt_libmf.h against the host libm: expf, acosf
 * and atanf and powf(x, 5) over every float (stride argv[1]), atan2f and
 * powf(|x|, y) over argv[2] random pairs plus structured cases.  Also confirms the expf table and polynomial
 * are the host libm's own data (found byte for byte in libm.so.6).
 * Build: gcc -O2 -ffp-contract=off -mfma tools/check_libmf.c -lm
 * (run by tests/test_libmf.py on a sample). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#define PT_SC_FMA fma
#include "../pathtracing_amd/csrc/pt_libmf.h"
static const uint64_t T[32] = PT_EXPF_TABLE;
static const double PL[32] = PT_POWF_LOG2_TABLE;
static const double LT[256] = PT_LOG_TABLE;

static int same(float a, float b) { return memcmp(&a, &b, 4) == 0 || (a != a && b != b); }
static uint64_t rng_state = 0x9e3779b97f4a7c15ull;
static uint32_t rnd(void) {
    rng_state = rng_state * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)(rng_state >> 32);
}

int main(int argc, char** argv) {
    unsigned stride = argc > 1 ? (unsigned)atoi(argv[1]) : 1;
    unsigned long npair = argc > 2 ? strtoul(argv[2], 0, 10) : 100000000ul;
    unsigned long bad[5] = {0, 0, 0, 0, 0}, tot[5] = {0, 0, 0, 0, 0};
    union { float f; uint32_t u; } v;
    for (uint64_t u = 0; u < 0x100000000ull; u += stride) {
        v.u = (uint32_t)u;
        float x = v.f;
        bad[0] += !same(expf(x), pt_expf_t(x, T)), tot[0]++;
        bad[2] += !same(atanf(x), pt_atanf(x)), tot[2]++;
        if (fabsf(x) <= 1.0f) bad[1] += !same(acosf(x), pt_acosf(x)), tot[1]++;
        bad[4] += !same(powf(x, 5.0f), pt_powf_t(x, 5.0f, PL, T)), tot[4]++;
    }
    /* atan2f: random bit patterns, random unit-sphere-like pairs, specials */
    const float sp[] = {0.0f, -0.0f, 1.0f, -1.0f, INFINITY, -INFINITY, NAN, 1e-30f, -1e-30f, 1e30f, 0x1p-149f, 3.0f};
    for (int a = 0; a < 12; a++)
        for (int b = 0; b < 12; b++) bad[3] += !same(atan2f(sp[a], sp[b]), pt_atan2f(sp[a], sp[b])), tot[3]++;
    for (unsigned long k = 0; k < npair; k++) {
        float y, x;
        if (k & 1) {
            v.u = rnd();
            y = v.f;
            v.u = rnd();
            x = v.f;
        } else {
            y = (float)((int32_t)rnd()) * 0x1p-31f;
            x = (float)((int32_t)rnd()) * 0x1p-31f;
        }
        bad[3] += !same(atan2f(y, x), pt_atan2f(y, x)), tot[3]++;
        if (y != 0.0f) bad[4] += !same(powf(fabsf(x), y), pt_powf_t(fabsf(x), y, PL, T)), tot[4]++;
    }
    /* log(1 - u) for every u = k * 2^-24 the medium sampling can draw, and
     * random positive normal doubles */
    unsigned long lbad = 0, ltot = 0;
    for (uint32_t k2 = 0; k2 < (1u << 24); k2 += (stride < 64 ? 1u : stride / 64u)) {
        const double x = 1.0 - (double)k2 * 0x1p-24;
        const double a = log(x), b = pt_log_t(x, LT);
        lbad += memcmp(&a, &b, 8) != 0, ltot++;
    }
    for (unsigned long k2 = 0; k2 < npair; k2++) {
        uint64_t u = ((uint64_t)rnd() << 32) | rnd();
        u = (u & 0x000fffffffffffffull) | ((uint64_t)(1 + rnd() % 2046) << 52);
        double x;
        memcpy(&x, &u, 8);
        if (k2 & 1) x = 1.0 + (x - floor(x)) * 0x1p-3 - 0x1p-4;  /* near 1 */
        const double a = log(x), b = pt_log_t(x, LT);
        lbad += memcmp(&a, &b, 8) != 0, ltot++;
    }
    printf("expf %lu/%lu acosf %lu/%lu atanf %lu/%lu atan2f %lu/%lu powf %lu/%lu log %lu/%lu\n", bad[0], tot[0], bad[1],
           tot[1], bad[2], tot[2], bad[3], tot[3], bad[4], tot[4], lbad, ltot);
    /* the table is libm's own */
    FILE* f = fopen("/usr/lib/x86_64-linux-gnu/libm.so.6", "rb");
    int found = 0;
    if (f) {
        static unsigned char buf[4 << 20];
        size_t n = fread(buf, 1, sizeof buf, f);
        fclose(f);
        for (size_t o = 0; o + 256 <= n && !found; o += 8) found = memcmp(buf + o, T, 256) == 0;
    }
    printf("expf table in libm: %d\n", found);
    return (bad[0] | bad[1] | bad[2] | bad[3] | bad[4] | lbad) != 0;
}
