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

// phaseHG (PhaseFunction.hpp:4-8)
__device__ __forceinline__ float phase_hg(float cosT, float g) {
    const float denom = 1 + g * g + 2 * g * cosT;
    return 0.25f * (1.0f / PT_PI) * (1.0f - g * g) / (denom * csqrt(denom));
}

// HenyeyGreenstein::Sample (PhaseFunction.cpp:8-25): the scattered direction
__device__ f3 phase_sample(float g, f3 in, float u0, float u1) {
    float cosT;
    if (fabsf(g) < 1e-3f) {
        cosT = 1 - 2 * u0;
    } else {
        const float sqr = (1 - g * g) / (1 - g + 2 * g * u0);
        cosT = (1 + g * g - sqr * sqr) / (2 * g);
    }
    const float sinT = csqrt(fmaxf(0.0f, 1 - cosT * cosT));
    const float phi = 2 * PT_PI * u1;
    const Onb b = onb_n(in);
    return normalize(to_world(b, F3(sinT * cos_cr(phi), sinT * sin_cr(phi), cosT)));
}

// HomogeneusMedium::Tr (Medium.hpp:21-24): exp(-sigma_t * min(t, FLT_MAX))
__device__ __forceinline__ f3 medium_tr(const pt_medium& m, float t) {
    const float tt = fminf(t, 3.402823466e38f);
    return F3(expf(-m.sigma_t[0] * tt), expf(-m.sigma_t[1] * tt), expf(-m.sigma_t[2] * tt));
}

// HomogeneusMedium::Sample (Medium.hpp:26-45): returns the attenuation
// factor; `sampled` and the scatter point p = fma(t, d, o) when it scattered
__device__ f3 medium_sample(const pt_medium& m, f3 o, f3 d, float t, float u0, float u1, bool& sampled, f3& p) {
    const int ch = (int)(0.0f + 3.0f * u0);
    const float st = ch == 0 ? m.sigma_t[0] : (ch == 1 ? m.sigma_t[1] : m.sigma_t[2]);
    float sd = (float)(-log(1.0 - (double)u1) / (double)st);
    if (!(sd < t)) sd = t;
    sampled = sd < t;
    if (sampled) p = F3(fma_(sd, d.x, o.x), fma_(sd, d.y, o.y), fma_(sd, d.z, o.z));
    const f3 tr = medium_tr(m, sd);
    const f3 den = sampled ? ld3(m.sigma_t) * tr : tr;
    float pdf = 0;
    pdf += den.x;
    pdf += den.y;
    pdf += den.z;
    pdf = (float)((double)pdf / 3.0);
    return sampled ? (tr * ld3(m.sigma_s)) / pdf : tr / pdf;
}
