// expf / acosf / atan2f bit-identical to the host libm the reference calls
// (glibc 2.35, x86-64):
//   expf   HomogeneusMedium::Tr (Medium.hpp:21-24) — the optimized-routines
//          design (glibc >= 2.27): k = round(x * 32/ln2), a 32-entry table of
//          2^(i/32) and a cubic in double, rounded once to float.  Its x86-64
//          FMA build (the ifunc choice on AVX2 hosts) fuses the polynomial's
//          multiply-adds.  Table and coefficients: glibc's __exp2f_data, read
//          back from the system libm (tools/check_libmf.c finds them there).
//   acosf  Sphere uv (Shape.cpp getSphereUV), fdlibm's __ieee754_acosf in
//          float arithmetic (no multiarch variant, no contraction).
//   atan2f Sphere uv and the envmap lookups, fdlibm's __ieee754_atan2f over
//          fdlibm's atanf.
// tools/check_libmf.c checks expf, acosf and atanf over every float and
// atan2f over a large random + structured sample against the host libm.
// Shared by the device code and its host-side test; PT_SC_FN qualifies the
// functions, PT_SC_FMA is the double fma.
#pragma once
#include <stdint.h>

#ifndef PT_SC_FN
#define PT_SC_FN static inline
#endif

// tab[i] = bits(2^(i/32)) - (i << 47)
#define PT_EXPF_TABLE                                                                                          \
    {0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,               \
     0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,               \
     0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,               \
     0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,               \
     0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,               \
     0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,               \
     0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,               \
     0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull}

PT_SC_FN uint32_t pt_lm_fbits(float x) {
    union { float f; uint32_t u; } v;
    v.f = x;
    return v.u;
}
PT_SC_FN float pt_lm_bitsf(uint32_t u) {
    union { float f; uint32_t u; } v;
    v.u = u;
    return v.f;
}
PT_SC_FN double pt_lm_bitsd(uint64_t u) {
    union { double f; uint64_t u; } v;
    v.u = u;
    return v.f;
}
PT_SC_FN uint64_t pt_lm_dbits(double x) {
    union { double f; uint64_t u; } v;
    v.f = x;
    return v.u;
}

// glibc e_expf.c.  The special cases (|x| >= 88, NaN) follow its
// specialcase branch: overflow to +inf above 0x1.62e42ep6, underflow to 0
// below -0x1.9fe368p6; callers pass x <= 0 (exp(-sigma_t * t)).
PT_SC_FN float pt_expf_t(float x, const uint64_t* T) {
    const uint32_t abstop = (pt_lm_fbits(x) >> 20) & 0x7ff;
    if (abstop >= 0x42b) {  // |x| >= 88 or NaN
        if (pt_lm_fbits(x) == 0xff800000u) return 0.0f;
        if (abstop >= 0x7f8) return x + x;
        if (x > 0x1.62e42ep6f) return pt_lm_bitsf(0x7f800000u);
        if (x < -0x1.9fe368p6f) return 0.0f;
    }
    const double xd = (double)x;
    // k = round(x * 32/ln2) by the 1.5*2^52 shift; both uses of x * 32/ln2
    // fused (vfmadd / vfmsub in the FMA build)
    double kd = PT_SC_FMA(0x1.71547652b82fep+5, xd, 0x1.8p+52);
    const uint64_t ki = pt_lm_dbits(kd);
    kd -= 0x1.8p+52;
    const double r = PT_SC_FMA(0x1.71547652b82fep+5, xd, -kd);
    uint64_t t = T[ki % 32];
    t += ki << 47;
    const double s = pt_lm_bitsd(t);
    const double zc = PT_SC_FMA(0x1.c6af84b912394p-20, r, 0x1.ebfce50fac4f3p-13);
    const double r2 = r * r;
    double y = PT_SC_FMA(0x1.62e42ff0c52d6p-6, r, 1.0);
    y = PT_SC_FMA(zc, r2, y);
    y = y * s;
    return (float)y;
}

// fdlibm's rational approximation of asin(sqrt(z))/sqrt(z) - 1 around 0
PT_SC_FN float pt_acosf_rz(float z) {
    const float p = z * (0x1.555556p-3f +
                         z * (-0x1.4d6120p-2f +
                              z * (0x1.9c1550p-3f + z * (-0x1.48228cp-5f + z * (0x1.9efe08p-11f + z * 0x1.23de10p-15f)))));
    const float q = 1.0f + z * (-0x1.33a272p+1f + z * (0x1.02ae5ap+1f + z * (-0x1.6066c2p-1f + z * 0x1.3b8c5cp-4f)));
    return p / q;
}

PT_SC_FN float pt_acosf(float x) {
    const float pi = 0x1.921fb4p+1f, pio2_hi = 0x1.921fb4p+0f, pio2_lo = 0x1.4442d0p-24f;
    const uint32_t hx = pt_lm_fbits(x), ix = hx & 0x7fffffffu;
    if (ix == 0x3f800000u) return (hx >> 31) == 0 ? 0.0f : pi + 2.0f * pio2_lo;
    if (ix > 0x3f800000u) return (x - x) / (x - x);
    if (ix < 0x3f000000u) {  // |x| < 0.5
        if (ix <= 0x32800000u) return pio2_hi + pio2_lo;
        const float r = pt_acosf_rz(x * x);
        return pio2_hi - (x - (pio2_lo - x * r));
    }
    if (hx >> 31) {  // x < -0.5
        const float z = (1.0f + x) * 0.5f;
        const float s = __builtin_sqrtf(z);
        const float r = pt_acosf_rz(z);
        const float w = r * s - pio2_lo;
        return pi - 2.0f * (s + w);
    }
    const float z = (1.0f - x) * 0.5f;  // x > 0.5
    const float s = __builtin_sqrtf(z);
    const float df = pt_lm_bitsf(pt_lm_fbits(s) & 0xfffff000u);
    const float c = (z - df * df) / (s + df);
    const float r = pt_acosf_rz(z);
    const float w = r * s + c;
    return 2.0f * (df + w);
}

PT_SC_FN float pt_atanf(float x) {
    const float atanhi[4] = {0x1.dac670p-2f, 0x1.921fb4p-1f, 0x1.f730bcp-1f, 0x1.921fb4p+0f};
    const float atanlo[4] = {0x1.586ed2p-28f, 0x1.4442d0p-25f, 0x1.281f68p-25f, 0x1.4442d0p-24f};
    const uint32_t hx = pt_lm_fbits(x), ix = hx & 0x7fffffffu;
    int id;
    if (ix >= 0x4c000000u) {  // |x| >= 2^25
        if (ix > 0x7f800000u) return x + x;
        return (hx >> 31) == 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
    }
    if (ix < 0x3ee00000u) {  // |x| < 0.4375
        if (ix < 0x31000000u) return x;
        id = -1;
    } else {
        x = pt_lm_bitsf(ix);
        if (ix < 0x3f980000u) {    // |x| < 1.1875
            if (ix < 0x3f300000u) {  // 7/16 <= |x| < 11/16
                id = 0;
                x = (2.0f * x - 1.0f) / (2.0f + x);
            } else {
                id = 1;
                x = (x - 1.0f) / (x + 1.0f);
            }
        } else if (ix < 0x401c0000u) {  // |x| < 2.4375
            id = 2;
            x = (x - 1.5f) / (1.0f + 1.5f * x);
        } else {
            id = 3;
            x = -1.0f / x;
        }
    }
    const float z = x * x, w = z * z;
    const float s1 = z * (0x1.555556p-2f +
                          w * (0x1.24924ap-3f + w * (0x1.745cdcp-4f + w * (0x1.10d66ap-4f + w * (0x1.97b4b2p-5f +
                                                                                                  w * 0x1.0ad3aep-6f)))));
    const float s2 = w * (-0x1.99999ap-3f +
                          w * (-0x1.c71c70p-4f + w * (-0x1.3b0f2ap-4f + w * (-0x1.dde2d6p-5f + w * -0x1.2b4442p-5f))));
    if (id < 0) return x - x * (s1 + s2);
    const float zz = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return (hx >> 31) ? -zz : zz;
}

PT_SC_FN float pt_atan2f(float y, float x) {
    const float pi_o_4 = 0x1.921fb6p-1f, pi_o_2 = 0x1.921fb6p+0f, pi = 0x1.921fb6p+1f, pi_lo = -0x1.777a5cp-24f;
    const float tiny = 1.0e-30f;
    const uint32_t hx = pt_lm_fbits(x), ix = hx & 0x7fffffffu, hy = pt_lm_fbits(y), iy = hy & 0x7fffffffu;
    if (ix > 0x7f800000u || iy > 0x7f800000u) return x + y;
    if (hx == 0x3f800000u) return pt_atanf(y);
    const int m = (int)((hy >> 31) & 1) | (int)((hx >> 30) & 2);
    if (iy == 0) {
        switch (m) {
            case 0:
            case 1: return y;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if (ix == 0) return (hy >> 31) ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000u) {
        if (iy == 0x7f800000u) {
            switch (m) {
                case 0: return pi_o_4 + tiny;
                case 1: return -pi_o_4 - tiny;
                case 2: return 3.0f * pi_o_4 + tiny;
                default: return -3.0f * pi_o_4 - tiny;
            }
        }
        switch (m) {
            case 0: return 0.0f;
            case 1: return -0.0f;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if (iy == 0x7f800000u) return (hy >> 31) ? -pi_o_2 - tiny : pi_o_2 + tiny;
    const int k = ((int)iy - (int)ix) >> 23;
    float z;
    if (k > 60) z = pi_o_2 + 0.5f * pi_lo;
    else if ((hx >> 31) && k < -60) z = 0.0f;
    else z = pt_atanf(__builtin_fabsf(y / x));
    switch (m) {
        case 0: return z;
        case 1: return pt_lm_bitsf(pt_lm_fbits(z) ^ 0x80000000u);
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

// powf: glibc e_powf.c (optimized routines), FMA build — log2(x) from a
// 16-entry (1/c, log2 c) table and a degree-5 polynomial in double, y*log2(x),
// then 2^t through the expf table above.  Used by the Schlick term
// (Material.hpp: glm::pow(1 - cos, 5)).  Finite x and y; y != 0.
#define PT_POWF_LOG2_TABLE                                                                                     \
    {0x1.661ec79f8f3bep+0, -0x1.efec65b963019p-2, 0x1.571ed4aaf883dp+0, -0x1.b0b6832d4fca4p-2,                  \
     0x1.49539f0f010b0p+0, -0x1.7418b0a1fb77bp-2, 0x1.3c995b0b80385p+0, -0x1.39de91a6dcf7bp-2,                  \
     0x1.30d190c8864a5p+0, -0x1.01d9bf3f2b631p-2, 0x1.25e227b0b8ea0p+0, -0x1.97c1d1b3b7af0p-3,                  \
     0x1.1bb4a4a1a343fp+0, -0x1.2f9e393af3c9fp-3, 0x1.12358f08ae5bap+0, -0x1.960cbbf788d5cp-4,                  \
     0x1.0953f419900a7p+0, -0x1.a6f9db6475fcep-5, 0x1.0000000000000p+0, 0x0.0p+0,                               \
     0x1.e608cfd9a47acp-1, 0x1.338ca9f24f53dp-4, 0x1.ca4b31f026aa0p-1, 0x1.476a9543891bap-3,                    \
     0x1.b2036576afce6p-1, 0x1.e840b4ac4e4d2p-3, 0x1.9c2d163a1aa2dp-1, 0x1.40645f0c6651cp-2,                    \
     0x1.886e6037841edp-1, 0x1.88e9c2c1b9ff8p-2, 0x1.767dcf5534862p-1, 0x1.ce0a44eb17bccp-2}

// 0: not an integer, 1: odd integer, 2: even integer
PT_SC_FN int pt_powf_checkint(uint32_t iy) {
    const int e = (int)(iy >> 23 & 0xff);
    if (e < 0x7f) return 0;
    if (e > 0x7f + 23) return 2;
    if (iy & ((1u << (0x7f + 23 - e)) - 1)) return 0;
    if (iy & (1u << (0x7f + 23 - e))) return 1;
    return 2;
}

PT_SC_FN float pt_powf_t(float x, float y, const double* L, const uint64_t* T) {
    uint32_t ix = pt_lm_fbits(x);
    const uint32_t iy = pt_lm_fbits(y);
    uint64_t sign_bias = 0;
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {  // x < 0x1p-126, negative, inf or nan
        if (2 * ix - 1 >= 2u * 0x7f800000u - 1) {          // x is 0, inf or nan
            float x2 = x * x;
            if ((ix & 0x80000000u) && pt_powf_checkint(iy) == 1) x2 = -x2;
            return (iy & 0x80000000u) ? 1.0f / x2 : x2;
        }
        if (ix & 0x80000000u) {  // finite x < 0
            const int yint = pt_powf_checkint(iy);
            if (yint == 0) return (x - x) / (x - x);
            if (yint == 1) sign_bias = 1u << 16;  // SIGN_BIAS: 1 << (5 + 11)
            ix &= 0x7fffffffu;
        }
        if (ix < 0x00800000u) {  // subnormal: normalise
            ix = pt_lm_fbits(pt_lm_bitsf(ix) * 0x1p23f) & 0x7fffffffu;
            ix -= 23u << 23;
        }
    }
    // log2_inline
    const uint32_t tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> 19) % 16);
    const uint32_t top = tmp & 0xff800000u;
    const uint32_t iz = ix - top;
    const int k = (int32_t)top >> 23;
    const double invc = L[2 * i], logc = L[2 * i + 1];
    const double z = (double)pt_lm_bitsf(iz);
    const double r = PT_SC_FMA(z, invc, -1.0);
    const double y0 = logc + (double)k;
    const double r2 = r * r;
    double yy = PT_SC_FMA(r, 0x1.27616c9496e0bp-2, -0x1.71969a075c67ap-2);
    const double p = PT_SC_FMA(r, 0x1.ec70a6ca7baddp-2, -0x1.7154748bef6c8p-1);
    const double r4 = r2 * r2;
    double q = PT_SC_FMA(r, 0x1.71547652ab82bp+0, y0);
    q = PT_SC_FMA(r2, p, q);
    yy = PT_SC_FMA(yy, r4, q);
    const double ylogx = (double)y * yy;
    if (((pt_lm_dbits(ylogx) >> 47) & 0xffff) >= (0x405f800000000000ull >> 47)) {  // |y log2 x| >= 126
        if (ylogx > 0x1.fffffffd1d571p+6) return sign_bias ? -pt_lm_bitsf(0x7f800000u) : pt_lm_bitsf(0x7f800000u);
        if (ylogx <= -150.0) return sign_bias ? -0.0f : 0.0f;
    }
    // exp2_inline
    double kd = ylogx + 0x1.8p+47;
    const uint64_t ki = pt_lm_dbits(kd);
    kd -= 0x1.8p+47;
    const double rr = ylogx - kd;
    uint64_t t = T[ki % 32];
    t += (ki + sign_bias) << 47;
    const double s = pt_lm_bitsd(t);
    const double zc = PT_SC_FMA(rr, 0x1.c6af84b912394p-5, 0x1.ebfce50fac4f3p-3);
    const double rr2 = rr * rr;
    double e = PT_SC_FMA(rr, 0x1.62e42ff0c52d6p-1, 1.0);
    e = PT_SC_FMA(zc, rr2, e);
    return (float)(e * s);
}
