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

// log (double): glibc e_log.c (optimized routines, glibc >= 2.28), FMA build:
// the medium's free-flight distance -log(1 - u) / sigma_t
// (HomogeneusMedium::Sample, Medium.hpp:26-45).  x = z * 2^k: log(x) =
// log1p(z / c - 1) + log(c) + k ln2 over a 128-entry (1/c, log c) table;
// inputs in [1 - 2^-4, 1 + 0x1.09p-4) use a degree-11 polynomial with a split
// product.  Table and coefficients: glibc's __log_data, read back from the
// system libm; contraction as its FMA build compiles it.  Normal positive
// inputs only (callers pass 1 - u, u in [0, 1)); others give NaN.
#define PT_LOG_TABLE \
    {0x1.734f0c3e0de9fp+0, -0x1.7cc7f79e69000p-2, \
     0x1.713786a2ce91fp+0, -0x1.76feec20d0000p-2, \
     0x1.6f26008fab5a0p+0, -0x1.713e31351e000p-2, \
     0x1.6d1a61f138c7dp+0, -0x1.6b85b38287800p-2, \
     0x1.6b1490bc5b4d1p+0, -0x1.65d5590807800p-2, \
     0x1.69147332f0cbap+0, -0x1.602d076180000p-2, \
     0x1.6719f18224223p+0, -0x1.5a8ca86909000p-2, \
     0x1.6524f99a51ed9p+0, -0x1.54f4356035000p-2, \
     0x1.63356aa8f24c4p+0, -0x1.4f637c36b4000p-2, \
     0x1.614b36b9ddc14p+0, -0x1.49da7fda85000p-2, \
     0x1.5f66452c65c4cp+0, -0x1.445923989a800p-2, \
     0x1.5d867b5912c4fp+0, -0x1.3edf439b0b800p-2, \
     0x1.5babccb5b90dep+0, -0x1.396ce448f7000p-2, \
     0x1.59d61f2d91a78p+0, -0x1.3401e17bda000p-2, \
     0x1.5805612465687p+0, -0x1.2e9e2ef468000p-2, \
     0x1.56397cee76bd3p+0, -0x1.2941b3830e000p-2, \
     0x1.54725e2a77f93p+0, -0x1.23ec58cda8800p-2, \
     0x1.52aff42064583p+0, -0x1.1e9e129279000p-2, \
     0x1.50f22dbb2bddfp+0, -0x1.1956d2b48f800p-2, \
     0x1.4f38f4734ded7p+0, -0x1.141679ab9f800p-2, \
     0x1.4d843cfde2840p+0, -0x1.0edd094ef9800p-2, \
     0x1.4bd3ec078a3c8p+0, -0x1.09aa518db1000p-2, \
     0x1.4a27fc3e0258ap+0, -0x1.047e65263b800p-2, \
     0x1.4880524d48434p+0, -0x1.feb224586f000p-3, \
     0x1.46dce1b192d0bp+0, -0x1.f474a7517b000p-3, \
     0x1.453d9d3391854p+0, -0x1.ea4443d103000p-3, \
     0x1.43a2744b4845ap+0, -0x1.e020d44e9b000p-3, \
     0x1.420b54115f8fbp+0, -0x1.d60a22977f000p-3, \
     0x1.40782da3ef4b1p+0, -0x1.cc00104959000p-3, \
     0x1.3ee8f5d57fe8fp+0, -0x1.c202956891000p-3, \
     0x1.3d5d9a00b4ce9p+0, -0x1.b81178d811000p-3, \
     0x1.3bd60c010c12bp+0, -0x1.ae2c9ccd3d000p-3, \
     0x1.3a5242b75dab8p+0, -0x1.a45402e129000p-3, \
     0x1.38d22cd9fd002p+0, -0x1.9a877681df000p-3, \
     0x1.3755bc5847a1cp+0, -0x1.90c6d69483000p-3, \
     0x1.35dce49ad36e2p+0, -0x1.87120a645c000p-3, \
     0x1.34679984dd440p+0, -0x1.7d68fb4143000p-3, \
     0x1.32f5cceffcb24p+0, -0x1.73cb83c627000p-3, \
     0x1.3187775a10d49p+0, -0x1.6a39a9b376000p-3, \
     0x1.301c8373e3990p+0, -0x1.60b3154b7a000p-3, \
     0x1.2eb4ebb95f841p+0, -0x1.5737d76243000p-3, \
     0x1.2d50a0219a9d1p+0, -0x1.4dc7b8fc23000p-3, \
     0x1.2bef9a8b7fd2ap+0, -0x1.4462c51d20000p-3, \
     0x1.2a91c7a0c1babp+0, -0x1.3b08abc830000p-3, \
     0x1.293726014b530p+0, -0x1.31b996b490000p-3, \
     0x1.27dfa5757a1f5p+0, -0x1.2875490a44000p-3, \
     0x1.268b39b1d3bbfp+0, -0x1.1f3b9f879a000p-3, \
     0x1.2539d838ff5bdp+0, -0x1.160c8252ca000p-3, \
     0x1.23eb7aac9083bp+0, -0x1.0ce7f57f72000p-3, \
     0x1.22a012ba940b6p+0, -0x1.03cdc49fea000p-3, \
     0x1.2157996cc4132p+0, -0x1.f57bdbc4b8000p-4, \
     0x1.201201dd2fc9bp+0, -0x1.e370896404000p-4, \
     0x1.1ecf4494d480bp+0, -0x1.d17983ef94000p-4, \
     0x1.1d8f5528f6569p+0, -0x1.bf9674ed8a000p-4, \
     0x1.1c52311577e7cp+0, -0x1.adc79202f6000p-4, \
     0x1.1b17c74cb26e9p+0, -0x1.9c0c3e7288000p-4, \
     0x1.19e010c2c1ab6p+0, -0x1.8a646b372c000p-4, \
     0x1.18ab07bb670bdp+0, -0x1.78d01b3ac0000p-4, \
     0x1.1778a25efbcb6p+0, -0x1.674f145380000p-4, \
     0x1.1648d354c31dap+0, -0x1.55e0e6d878000p-4, \
     0x1.151b990275fddp+0, -0x1.4485cdea1e000p-4, \
     0x1.13f0ea432d24cp+0, -0x1.333d94d6aa000p-4, \
     0x1.12c8b7210f9dap+0, -0x1.22079f8c56000p-4, \
     0x1.11a3028ecb531p+0, -0x1.10e4698622000p-4, \
     0x1.107fbda8434afp+0, -0x1.ffa6c6ad20000p-5, \
     0x1.0f5ee0f4e6bb3p+0, -0x1.dda8d4a774000p-5, \
     0x1.0e4065d2a9fcep+0, -0x1.bbcece4850000p-5, \
     0x1.0d244632ca521p+0, -0x1.9a1894012c000p-5, \
     0x1.0c0a77ce2981ap+0, -0x1.788583302c000p-5, \
     0x1.0af2f83c636d1p+0, -0x1.5715e67d68000p-5, \
     0x1.09ddb98a01339p+0, -0x1.35c8a49658000p-5, \
     0x1.08cabaf52e7dfp+0, -0x1.149e364154000p-5, \
     0x1.07b9f2f4e28fbp+0, -0x1.e72c082eb8000p-6, \
     0x1.06ab58c358f19p+0, -0x1.a55f152528000p-6, \
     0x1.059eea5ecf92cp+0, -0x1.63d62cf818000p-6, \
     0x1.04949cdd12c90p+0, -0x1.228fb8caa0000p-6, \
     0x1.038c6c6f0ada9p+0, -0x1.c317b20f90000p-7, \
     0x1.02865137932a9p+0, -0x1.419355daa0000p-7, \
     0x1.0182427ea7348p+0, -0x1.81203c2ec0000p-8, \
     0x1.008040614b195p+0, -0x1.0040979240000p-9, \
     0x1.fe01ff726fa1ap-1, 0x1.feff384900000p-9, \
     0x1.fa11cc261ea74p-1, 0x1.7dc41353d0000p-7, \
     0x1.f6310b081992ep-1, 0x1.3cea3c4c28000p-6, \
     0x1.f25f63ceeadcdp-1, 0x1.b9fc114890000p-6, \
     0x1.ee9c8039113e7p-1, 0x1.1b0d8ce110000p-5, \
     0x1.eae8078cbb1abp-1, 0x1.58a5bd001c000p-5, \
     0x1.e741aa29d0c9bp-1, 0x1.95c8340d88000p-5, \
     0x1.e3a91830a99b5p-1, 0x1.d276aef578000p-5, \
     0x1.e01e009609a56p-1, 0x1.07598e598c000p-4, \
     0x1.dca01e577bb98p-1, 0x1.253f5e30d2000p-4, \
     0x1.d92f20b7c9103p-1, 0x1.42edd8b380000p-4, \
     0x1.d5cac66fb5ccep-1, 0x1.606598757c000p-4, \
     0x1.d272caa5ede9dp-1, 0x1.7da76356a0000p-4, \
     0x1.cf26e3e6b2ccdp-1, 0x1.9ab434e1c6000p-4, \
     0x1.cbe6da2a77902p-1, 0x1.b78c7bb0d6000p-4, \
     0x1.c8b266d37086dp-1, 0x1.d431332e72000p-4, \
     0x1.c5894bd5d5804p-1, 0x1.f0a3171de6000p-4, \
     0x1.c26b533bb9f8cp-1, 0x1.067152b914000p-3, \
     0x1.bf583eeece73fp-1, 0x1.147858292b000p-3, \
     0x1.bc4fd75db96c1p-1, 0x1.2266ecdca3000p-3, \
     0x1.b951e0c864a28p-1, 0x1.303d7a6c55000p-3, \
     0x1.b65e2c5ef3e2cp-1, 0x1.3dfc33c331000p-3, \
     0x1.b374867c9888bp-1, 0x1.4ba366b7a8000p-3, \
     0x1.b094b211d304ap-1, 0x1.5933928d1f000p-3, \
     0x1.adbe885f2ef7ep-1, 0x1.66acd2418f000p-3, \
     0x1.aaf1d31603da2p-1, 0x1.740f8ec669000p-3, \
     0x1.a82e63fd358a7p-1, 0x1.815c0f51af000p-3, \
     0x1.a5740ef09738bp-1, 0x1.8e92954f68000p-3, \
     0x1.a2c2a90ab4b27p-1, 0x1.9bb3602f84000p-3, \
     0x1.a01a01393f2d1p-1, 0x1.a8bed1c2c0000p-3, \
     0x1.9d79f24db3c1bp-1, 0x1.b5b515c01d000p-3, \
     0x1.9ae2505c7b190p-1, 0x1.c2967ccbcc000p-3, \
     0x1.9852ef297ce2fp-1, 0x1.cf635d5486000p-3, \
     0x1.95cbaeea44b75p-1, 0x1.dc1bd3446c000p-3, \
     0x1.934c69de74838p-1, 0x1.e8c01b8cfe000p-3, \
     0x1.90d4f2f6752e6p-1, 0x1.f5509c0179000p-3, \
     0x1.8e6528effd79dp-1, 0x1.00e6c121fb800p-2, \
     0x1.8bfce9fcc007cp-1, 0x1.071b80e93d000p-2, \
     0x1.899c0dabec30ep-1, 0x1.0d46b9e867000p-2, \
     0x1.87427aa2317fbp-1, 0x1.13687334bd000p-2, \
     0x1.84f00acb39a08p-1, 0x1.1980d67234800p-2, \
     0x1.82a49e8653e55p-1, 0x1.1f8ffe0cc8000p-2, \
     0x1.8060195f40260p-1, 0x1.2595fd7636800p-2, \
     0x1.7e22563e0a329p-1, 0x1.2b9300914a800p-2, \
     0x1.7beb377dcb5adp-1, 0x1.3187210436000p-2, \
     0x1.79baa679725c2p-1, 0x1.377266dec1800p-2, \
     0x1.77907f2170657p-1, 0x1.3d54ffbaf3000p-2, \
     0x1.756cadbd6130cp-1, 0x1.432eee32fe000p-2}

PT_SC_FN double pt_log_t(double x, const double* T) {
    const uint64_t ix = pt_lm_dbits(x);
    if (ix - 0x3fee000000000000ull < 0x3090000000000ull) {  // x in [1 - 2^-4, 1 + 0x1.09p-4)
        if (ix == 0x3ff0000000000000ull) return 0.0;
        const double B0 = -0.5;
        const double r = x - 1.0;
        const double r2 = r * r, r3 = r * r2;
        const double p1 = PT_SC_FMA(r2, 0x1.999999995dd0cp-3, PT_SC_FMA(r, -0x1.ffffffffffdcbp-3, 0x1.5555555555577p-2));
        const double p2 = PT_SC_FMA(r2, -0x1.fffffa4423d65p-4, PT_SC_FMA(r, 0x1.24924a344de30p-3, -0x1.55555556745a7p-3));
        double p3 = PT_SC_FMA(r, -0x1.999eb43b068ffp-4, 0x1.c7184282ad6cap-4);
        p3 = PT_SC_FMA(r2, 0x1.78182f7afd085p-4, p3);
        p3 = PT_SC_FMA(r3, -0x1.5521375d145cdp-4, p3);
        const double q = PT_SC_FMA(PT_SC_FMA(p3, r3, p2), r3, p1);
        // r split into rhi + rlo (rhi with 26 bits): w = r * 2^27, rhi = r + w - w
        const double rhi = PT_SC_FMA(-0x1p27, r, PT_SC_FMA(r, 0x1p27, r));
        const double rlo = r - rhi;
        const double rhi2 = rhi * rhi;
        const double hi = PT_SC_FMA(rhi2, B0, r);
        double lo = PT_SC_FMA(rhi2, B0, r - hi);
        lo = PT_SC_FMA(B0 * rlo, r + rhi, lo);
        return hi + PT_SC_FMA(q, r3, lo);
    }
    const uint32_t top = (uint32_t)(ix >> 48);
    if (top - 0x0010u >= 0x7ff0u - 0x0010u) return pt_lm_bitsd(0x7ff8000000000000ull);
    const uint64_t tmp = ix - 0x3fe6000000000000ull;
    const int i = (int)((tmp >> 45) & 127u);
    const int k = (int)((int64_t)tmp >> 52);
    const double z = pt_lm_bitsd(ix - (tmp & 0xfff0000000000000ull));
    const double invc = T[2 * i], logc = T[2 * i + 1];
    const double r = PT_SC_FMA(z, invc, -1.0);
    const double kd = (double)k;
    const double w = PT_SC_FMA(kd, 0x1.62e42fefa3800p-1, logc);
    const double hi = r + w;
    const double lo = PT_SC_FMA(kd, 0x1.ef35793c76730p-45, (w - hi) + r);
    const double r2 = r * r, r3 = r * r2;
    const double t = PT_SC_FMA(PT_SC_FMA(r, -0x1.55575e506c89fp-3, 0x1.999b324f10111p-3), r2,
                               PT_SC_FMA(r, -0x1.fffffffeb4590p-3, 0x1.555555551305bp-2));
    return PT_SC_FMA(r3, t, PT_SC_FMA(r2, -0x1.0000000000001p-1, lo)) + hi;
}
