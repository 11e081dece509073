// sinf / cosf bit-identical to the host libm the reference calls
// (Material.hpp:225-229 cosine sampling, Material.hpp:131-132 GGX VNDF,
// Light.cpp sky/sphere sampling, Random.hpp inUnitDisk).
//
// glibc's float sine/cosine (the ARM optimized-routines design adopted in
// glibc 2.28; its x86-64 FMA build is what the ifunc selects on AVX2 hosts):
// reduce x to r = x - n*pi/2 in double (|x| < 120), then a degree-7 sine or
// degree-8 cosine polynomial in double with fused multiply-adds, rounded once
// to float.  The coefficients below were read from the system libm's
// __sincosf_table; the whole function was checked bit-exact against libm's
// sinf/cosf over every float in (-120, 120) (tools/check_sincosf.c).
// Shared by the device code and its host-side test; PT_SC_FN qualifies the
// functions, PT_SC_FMA is the double fma.
#pragma once
#include <stdint.h>

#ifndef PT_SC_FN
#define PT_SC_FN static inline
#endif

// sign[4], 2/pi * 2^24, pi/2, c0, c1, s1, c2, s2, c3, s3, c4 (two tables: the
// second negates the cosine polynomial, used in quadrants 2 and 3)
#define PT_SC_TABLE                                                                                            \
    {{1.0, -1.0, -1.0, 1.0, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0, 0x1.0000000000000p+0,                 \
      -0x1.ffffffd0c621cp-2, -0x1.555545995a603p-3, 0x1.55553e1068f19p-5, 0x1.1107605230bc4p-7,                \
      -0x1.6c087e89a359dp-10, -0x1.994eb3774cf24p-13, 0x1.99343027bf8c3p-16},                                   \
     {1.0, -1.0, -1.0, 1.0, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0, -0x1.0000000000000p+0,                \
      0x1.ffffffd0c621cp-2, -0x1.555545995a603p-3, -0x1.55553e1068f19p-5, 0x1.1107605230bc4p-7,                \
      0x1.6c087e89a359dp-10, -0x1.994eb3774cf24p-13, -0x1.99343027bf8c3p-16}}
enum { PT_SC_HPI_INV = 4, PT_SC_HPI = 5, PT_SC_C0 = 6, PT_SC_C1, PT_SC_S1, PT_SC_C2, PT_SC_S2, PT_SC_C3, PT_SC_S3,
       PT_SC_C4 };

PT_SC_FN uint32_t pt_sc_top12(float x) {
    union { float f; uint32_t u; } v;
    v.f = x;
    return (v.u >> 20) & 0x7ffu;
}

PT_SC_FN double pt_sc_poly(double x, double x2, const double* p, int n) {
    if ((n & 1) == 0) {
        double x3 = x * x2;
        double s1 = PT_SC_FMA(x2, p[PT_SC_S3], p[PT_SC_S2]);
        double x7 = x3 * x2;
        double s = PT_SC_FMA(x3, p[PT_SC_S1], x);
        return PT_SC_FMA(x7, s1, s);
    }
    double x4 = x2 * x2;
    double c2 = PT_SC_FMA(x2, p[PT_SC_C4], p[PT_SC_C3]);
    double c1 = PT_SC_FMA(x2, p[PT_SC_C1], p[PT_SC_C0]);
    double x6 = x4 * x2;
    double c = PT_SC_FMA(x4, p[PT_SC_C2], c1);
    return PT_SC_FMA(x6, c2, c);
}

// n = round-half-up(x * 2/pi) via the 2^24-scaled reciprocal; r = x - n*pi/2
PT_SC_FN double pt_sc_reduce(double x, const double* p, int* np) {
    double r = x * p[PT_SC_HPI_INV];
    int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
    return PT_SC_FMA(-(double)n, p[PT_SC_HPI], x);
}

// |y| < 120 (all callers pass angles in [0, 2pi]); larger arguments use the
// double-precision fallback `big`.
PT_SC_FN float pt_sinf_t(float y, const double (*T)[14]) {
    double x = y;
    const double* p = T[0];
    int n;
    if (pt_sc_top12(y) < pt_sc_top12(0x1.921FB6p-1f)) {
        if (pt_sc_top12(y) < pt_sc_top12(0x1p-12f)) return y;
        return (float)pt_sc_poly(x, x * x, p, 0);
    }
    x = pt_sc_reduce(x, p, &n);
    double s = p[n & 3];
    if (n & 2) p = T[1];
    return (float)pt_sc_poly(x * s, x * x, p, n);
}

PT_SC_FN float pt_cosf_t(float y, const double (*T)[14]) {
    double x = y;
    const double* p = T[0];
    int n;
    if (pt_sc_top12(y) < pt_sc_top12(0x1.921FB6p-1f)) {
        if (pt_sc_top12(y) < pt_sc_top12(0x1p-12f)) return 1.0f;
        return (float)pt_sc_poly(x, x * x, p, 1);
    }
    x = pt_sc_reduce(x, p, &n);
    double s = p[n & 3];
    if (n & 2) p = T[1];
    return (float)pt_sc_poly(x * s, x * x, p, n ^ 1);
}
