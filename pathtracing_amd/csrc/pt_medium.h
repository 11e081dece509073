// Participating media for VolPathIntegrator (Integrators.cpp:296-479):
// HomogeneusMedium (Medium.hpp:14-61) and HenyeyGreenstein (PhaseFunction.*).
// The medium's two hidden random_float() draws (Medium.hpp:28-30) come from
// the sample stream; everything else follows the reference's
// float arithmetic.
#pragma once
#include "pt_shading.h"

// ray medium in the path flags (d.w): bits 25..31, 0x7F = none
#define PF_MED_SHIFT 25
#define PF_MED_NONE 0x7Fu
#define PT_MAX_MEDIA 127
__device__ __forceinline__ int flags_medium(uint32_t f) {
    const uint32_t m = f >> PF_MED_SHIFT;
    return m == PF_MED_NONE ? -1 : (int)m;
}
__device__ __forceinline__ uint32_t medium_bits(int m) {
    return (m < 0 ? PF_MED_NONE : (uint32_t)m) << PF_MED_SHIFT;
}

// phaseHG (PhaseFunction.hpp:4-8) as built: 1 + g*g, + 2g*cos and 1 - g*g fused
__device__ __forceinline__ float phase_hg(float cosT, float g) {
    const float denom = fma_(cosT, 2.0f * g, fma_(g, g, 1.0f));
    return fma_(-g, g, 1.0f) * (0.25f * (1.0f / PT_PI)) / (denom * csqrt(denom));
}

// HenyeyGreenstein::Sample (PhaseFunction.cpp:8-25): the scattered direction
__device__ f3 phase_sample(float g, f3 in, float u0, float u1) {
    float cosT;
    if (fabs((double)g) < 1e-3) {
        cosT = 1 - 2 * u0;
    } else {
        const float sqr = fma_(-g, g, 1.0f) / fma_(2.0f * g, u0, 1 - g);
        cosT = fma_(-sqr, sqr, fma_(g, g, 1.0f)) / (2 * g);
    }
    const float q = fma_(-cosT, cosT, 1.0f);
    const float sinT = q > 0 ? csqrt(q) : 0.0f;
    const float phi = 2 * PT_PI * u1;
    const float x = cos_cr(phi) * sinT, y = sin_cr(phi) * sinT, z = cosT;
    // onb(in).toWorld as built here: a0 = cross(a1, a2) with the x, y lanes
    // rounded-first; x, y lanes (x*a0 fused onto y*a1) + z*a2 unfused, z lane
    // the usual chain
    Onb b;
    b.a2 = in;
    const f3 up = (fabsf(in.x) > 0.9999) ? F3(0, 1, 0) : F3(1, 0, 0);
    b.a1 = normalize(cross(b.a2, up));
    b.a0 = cross_v(b.a1, b.a2);
    const f3 w = F3(fma_(b.a0.x, x, y * b.a1.x) + z * b.a2.x, fma_(b.a0.y, x, y * b.a1.y) + z * b.a2.y,
                    fma_(z, b.a2.z, fma_(y, b.a1.z, x * b.a0.z)));
    return normalize(w);
}

// HomogeneusMedium::Tr (Medium.hpp:21-24): exp(-sigma_t * min(t, FLT_MAX))
__device__ __forceinline__ f3 medium_tr(const pt_medium& m, float t) {
    const float tt = fminf(t, 3.402823466e38f);
    return F3(exp_cr(-m.sigma_t[0] * tt), exp_cr(-m.sigma_t[1] * tt), exp_cr(-m.sigma_t[2] * tt));
}

// HomogeneusMedium::Sample (Medium.hpp:26-45): returns the attenuation
// factor; `sampled` and the scatter point p = fma(t, d, o) when it scattered
__device__ f3 medium_sample(const pt_medium& m, f3 o, f3 d, float t, float u0, float u1, bool& sampled, f3& p) {
    const int ch = (int)(0.0f + 3.0f * u0);
    const float st = ch == 0 ? m.sigma_t[0] : (ch == 1 ? m.sigma_t[1] : m.sigma_t[2]);
    float sd = (float)(-log_cr(1.0 - (double)u1) / (double)st);  // glibc's log, restated (pt_libmf.h)
    if (!(sd < t)) sd = t;
    sampled = sd < t;
    if (sampled) p = F3(fma_(sd, d.x, o.x), fma_(sd, d.y, o.y), fma_(sd, d.z, o.z));
    const f3 tr = medium_tr(m, sd);
    float pdf;
    if (sampled)  // the sum of sigma_t*tr with the products fused
        pdf = fma_(m.sigma_t[2], tr.z, fma_(m.sigma_t[1], tr.y, tr.x * m.sigma_t[0]));
    else
        pdf = ((0.0f + tr.x) + tr.y) + tr.z;
    pdf = (float)((double)pdf / 3.0);
    return sampled ? (tr * ld3(m.sigma_s)) / pdf : tr / pdf;
}
