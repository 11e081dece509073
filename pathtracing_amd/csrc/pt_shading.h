// Device restatement of the reference's surface shading: textures
// (Texture.hpp/.cpp), materials (Material.hpp), shapes' interaction
// reconstruction (Shape.cpp), lights and light samplers (Light.cpp,
// LightSampler.cpp).  Each function cites the reference file:line.
#pragma once
#include "pt_device.h"

struct SurfInt {  // SurfaceInteraction (Interaction.hpp:36-51)
    f3 p, n, ns, tangent;
    float u, v;  // uv
    float t;
    int32_t mat, light;
};

// ------------------------------------------------------------------ table reads
// (LDS copies of the material / texture / image / light-sampler tables were
// measured slower: the reads are L1/L2 hits and each block waits for its
// staging behind a barrier, profiles/r03_ab_lds_tables.txt)
__device__ __forceinline__ pt_material mat_rec(int mid) { return S.materials[mid]; }
__device__ __forceinline__ pt_texture tex_rec(int id) { return S.textures[id]; }
__device__ __forceinline__ pt_image img_rec(int id) { return S.images[id]; }

// ------------------------------------------------------------------ textures
// The non-negative remainder by the float reciprocal: for
// |i| < 2^20 the product i * rcp(n) (rcp within 1 ulp) is within 1/4 of i / n,
// so floor() is off by at most one and one correction each way gives the
// exact remainder; other lanes take the integer division.
__device__ __forceinline__ int wrap_rcp(int i, int n) {
    const float q = floorf((float)i * __builtin_amdgcn_rcpf((float)n));
    int m = i - (int)q * n;
    m += m < 0 ? n : 0;
    m -= m >= n ? n : 0;
    return m;
}
// the traversal's alpha test: the reciprocal form where it is exact
__device__ __forceinline__ int wrap_index(int i, int n);
__device__ __forceinline__ int wrap_index_t(int i, int n) {
    if ((uint32_t)i + (1u << 20) < (2u << 20)) return wrap_rcp(i, n);
    return wrap_index(i, n);
}
__device__ __forceinline__ int wrap_index(int i, int n) {
    int m = i % n;
    if (m < 0) m += n;
    return m;
}
// byte / 255.0f exactly as the IEEE division rounds it: the product with the
// rounded reciprocal and one fma correction give the correctly rounded
// quotient for every byte 0..255 (tools/check_u8unit.c, run by
// tests/test_libmf.py) in 3 VALU instead of a division's ~11
__device__ __forceinline__ float u8_unit(uint32_t b) {
    const float x = (float)b, r = 1.0f / 255.0f;
    const float q = x * r;
    return fma_(fma_(-q, 255.0f, x), r, q);
}
// Image::GetChannelAt (Texture.hpp:43-48): byte ch-1 of the pixel, any channel count.
// wrap_index(x + 1, n) from w = wrap_index(x, n): a bilinear footprint wraps
// each axis once (one integer remainder per axis instead of one per texel)
__device__ __forceinline__ int wrap_next(int w, int n) { return w + 1 == n ? 0 : w + 1; }
// (xi, yi: wrapped coordinates)
// (an image's element index fits 32 bits: pt_scene_upload checks its size)
__device__ __forceinline__ float channel_w(const pt_image& im, int xi, int yi, int ch) {
    const uint32_t local = ((uint32_t)yi * (uint32_t)im.width + (uint32_t)xi) * (uint32_t)im.channels + (uint32_t)(ch - 1);
    const uint64_t idx = im.offset + local;
    if (im.format == PT_IMAGE_F32) {  // FloatImage::GetChannelAt (Texture.hpp:78-83): floats, no /255
        const uint64_t fi = im.offset + 4ull * local;
        if (fi + 4 > S.n_texel_bytes) return 0.0f;
        return *reinterpret_cast<const float*>(S.texels + fi);
    }
    if (idx >= S.n_texel_bytes) return 0.0f;
    return u8_unit(S.texels[idx]);
}
__device__ __forceinline__ float channel_at(const pt_image& im, int x, int y, int ch) {
    return channel_w(im, wrap_index(x, im.width), wrap_index(y, im.height), ch);
}
__device__ __forceinline__ f3 texel3_w(const pt_image& im, int xi, int yi) {
    return F3(channel_w(im, xi, yi, 1), channel_w(im, xi, yi, 2), channel_w(im, xi, yi, 3));
}

// The two texels (x, y), (x + 1, y) of a bilinear row of a u8 RGB / RGBA image
// with three aligned word loads instead of six byte loads: the 2C bytes from
// the first texel's byte on, realigned with v_alignbyte.  Same values as
// texel3 (byte / 255); false (caller falls back to texel3) when x + 1 wraps,
// for other formats, or near the end of the texel buffer (the upload pads it
// by 16 bytes, so the word loads stay inside the allocation).
__device__ __forceinline__ bool texel_pair_u8(const pt_image& im, int xi, int yi, f3& a, f3& b) {
    // (xi, yi: wrapped coordinates)
    const int C = im.channels;
    if (im.format != PT_IMAGE_U8 || (C != 3 && C != 4)) return false;
    if (xi + 1 >= im.width) return false;
    const uint64_t idx = im.offset + ((uint64_t)yi * (uint64_t)im.width + (uint64_t)xi) * (uint64_t)C;
    if (idx + 2u * (uint64_t)C > S.n_texel_bytes) return false;
    const uint32_t* w = reinterpret_cast<const uint32_t*>(S.texels + (idx & ~3ull));
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
    const uint32_t sh = (uint32_t)(idx & 3u);
    const uint32_t q0 = __builtin_amdgcn_alignbyte(w1, w0, sh), q1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
    const uint32_t qb = C == 4 ? q1 : __builtin_amdgcn_alignbyte(q1, q0, 3u);  // second texel's bytes
    auto ch = [](uint32_t q, int k) { return u8_unit((q >> (8 * k)) & 0xFFu); };
    a = F3(ch(q0, 0), ch(q0, 1), ch(q0, 2));
    b = F3(ch(qb, 0), ch(qb, 1), ch(qb, 2));
    return true;
}

// Both rows of a bilinear footprint of a u8 RGB / RGBA image (texel_pair_u8
// per row): the checks of both rows first, then the six word loads together,
// then the decode -- one memory round trip per lookup instead of one per row.
// false: the caller falls back to the texels one by one.
__device__ __forceinline__ bool texel_quad_u8(const pt_image& im, int x0, int y0, int y1, f3& a, f3& b, f3& c,
                                              f3& d) {
    const int C = im.channels;
    if (im.format != PT_IMAGE_U8 || (C != 3 && C != 4)) return false;
    if (x0 + 1 >= im.width) return false;
    const uint64_t i0 = im.offset + ((uint64_t)y0 * (uint64_t)im.width + (uint64_t)x0) * (uint64_t)C;
    const uint64_t i1 = im.offset + ((uint64_t)y1 * (uint64_t)im.width + (uint64_t)x0) * (uint64_t)C;
    if (i0 + 2u * (uint64_t)C > S.n_texel_bytes || i1 + 2u * (uint64_t)C > S.n_texel_bytes) return false;
    const uint32_t* w = reinterpret_cast<const uint32_t*>(S.texels + (i0 & ~3ull));
    const uint32_t* v = reinterpret_cast<const uint32_t*>(S.texels + (i1 & ~3ull));
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], v0 = v[0], v1 = v[1], v2 = v[2];
    auto row = [C](uint32_t r0, uint32_t r1, uint32_t r2, uint32_t sh, f3& p, f3& q) {
        const uint32_t q0 = __builtin_amdgcn_alignbyte(r1, r0, sh), q1 = __builtin_amdgcn_alignbyte(r2, r1, sh);
        const uint32_t qb = C == 4 ? q1 : __builtin_amdgcn_alignbyte(q1, q0, 3u);  // second texel's bytes
        auto ch = [](uint32_t x, int k) { return u8_unit((x >> (8 * k)) & 0xFFu); };
        p = F3(ch(q0, 0), ch(q0, 1), ch(q0, 2));
        q = F3(ch(qb, 0), ch(qb, 1), ch(qb, 2));
    };
    row(w0, w1, w2, (uint32_t)(i0 & 3u), a, b);
    row(v0, v1, v2, (uint32_t)(i1 & 3u), c, d);
    return true;
}

// Texture::Evaluate for SolidColor / CheckerTexture / ImageTexture (Texture.hpp:128-207).
// PAIR: texel_pair_u8 row loads (shading); the alpha test inside the traversal
// kernels keeps the byte loads (its callee registers count toward theirs).
template <bool PAIR>
__device__ f3 tex_eval_t(int id, float u, float v) {
    f3 scale = F3(1, 1, 1);
    bool scaled = false;
    for (int guard = 0; guard < 16; guard++) {
        // PAIR: the shading kernels (staged tables); else the traversal's alpha test
        const pt_texture t = PAIR ? tex_rec(id) : S.textures[id];
        if (t.kind == PT_TEX_SOLID) {
            f3 c = ld3(t.value);
            return scaled ? scale * c : c;
        }
        if (t.kind == PT_TEX_CHECKER) {
            int ux = (int)floorf(u * t.inv_scale[0]);
            int uy = (int)floorf(v * t.inv_scale[1]);
            // colorScale * child (Texture.hpp:205-206); nested scales multiply outward-in
            scale = scaled ? scale * ld3(t.scale) : ld3(t.scale);
            scaled = true;
            id = ((ux + uy) % 2 == 0) ? t.a : t.b;
            continue;
        }
        const pt_image im = PAIR ? img_rec(t.image) : S.images[t.image];
        float x = u * im.width - 0.5f;
        float y = v * im.height - 0.5f;
        int xi = (int)floorf(x), yi = (int)floorf(y);
        float dx = x - xi, dy = y - yi;
        const int x0 = wrap_index(xi, im.width), x1 = wrap_next(x0, im.width);
        const int y0 = wrap_index(yi, im.height), y1 = wrap_next(y0, im.height);
        f3 a, b, c, d;
        if (!PAIR || !texel_quad_u8(im, x0, y0, y1, a, b, c, d)) {
            a = texel3_w(im, x0, y0);
            b = texel3_w(im, x1, y0);
            c = texel3_w(im, x0, y1);
            d = texel3_w(im, x1, y1);
        }
        // contraction of the reference build: w_a*a rounded, then fma(w_b, b), fma(w_c, c), fma(w_d, d)
        float wa = (1 - dx) * (1 - dy), wb = dx * (1 - dy), wc = (1 - dx) * dy, wd = dx * dy;
        f3 r = F3(fma_(wd, d.x, fma_(wc, c.x, fma_(wb, b.x, rmul(wa, a.x)))),
                  fma_(wd, d.y, fma_(wc, c.y, fma_(wb, b.y, rmul(wa, a.y)))),
                  fma_(wd, d.z, fma_(wc, c.z, fma_(wb, b.z, rmul(wa, a.z)))));
        r = ld3(t.scale) * r;
        return scaled ? scale * r : r;
    }
    return F3(0, 0, 0);
}

__device__ __forceinline__ f3 tex_eval(int id, float u, float v) { return tex_eval_t<true>(id, u, v); }

// Texture::alpha (Texture.hpp:112-114, Texture.cpp:47-62, 41-45)
__device__ float tex_alpha(int id, float u, float v) {
    for (int guard = 0; guard < 16; guard++) {
        const pt_texture& t = S.textures[id];
        if (t.kind == PT_TEX_SOLID) return 1.0f;
        if (t.kind == PT_TEX_CHECKER) {
            int ux = (int)floorf(u * t.inv_scale[0]);
            int uy = (int)floorf(v * t.inv_scale[1]);
            id = ((ux + uy) % 2 == 0) ? t.a : t.b;
            continue;
        }
        const pt_image& im = S.images[t.image];
        if (im.channels != 4) return 1.0f;
        float x = u * im.width - 0.5f;
        float y = v * im.height - 0.5f;
        int xi = (int)floorf(x), yi = (int)floorf(y);
        float dx = x - xi, dy = y - yi;
        const int x0 = wrap_index(xi, im.width), x1 = wrap_next(x0, im.width);
        const int y0 = wrap_index(yi, im.height), y1 = wrap_next(y0, im.height);
        float a = channel_w(im, x0, y0, 4), b = channel_w(im, x1, y0, 4);
        float c = channel_w(im, x0, y1, 4), d = channel_w(im, x1, y1, 4);
        // ImageTexture::alpha as compiled in the reference: w_b*b rounded, then fma(w_a, a), fma(w_c, c), fma(w_d, d)
        float wa = (1 - dx) * (1 - dy), wb = dx * (1 - dy), wc = (1 - dx) * dy, wd = dx * dy;
        return fma_(wd, d, fma_(wc, c, fma_(wa, a, rmul(wb, b))));
    }
    return 1.0f;
}

__device__ __forceinline__ uint32_t fbits(float f) { return __float_as_uint(f); }
// AlphaTester Blend draws random_float() (Material.hpp:189) from an unseeded
// thread-local generator; no frame of the reference reproduces it, so the
// draw is a hash of the whole ray (its origin and direction come from the
// sample's stream, so every ray and bounce of every sample gets its own
// value) and the primitive; the accept rate is checked statistically against
// the reference's own Render (tests: blend_box).
__device__ __forceinline__ float blend_random(f3 o, f3 d, int prim) {
    uint32_t h = pcg_hash((uint32_t)prim);
    h = pcg_hash(h ^ fbits(o.x));
    h = pcg_hash(h ^ fbits(o.y));
    h = pcg_hash(h ^ fbits(o.z));
    h = pcg_hash(h ^ fbits(d.x));
    h = pcg_hash(h ^ fbits(d.y));
    h = pcg_hash(h ^ fbits(d.z));
    return (float)(h >> 8) * (1.0f / 16777216.0f);
}

// Material::Alpha (Material.hpp:336-342, 572-578)
__device__ bool mat_alpha(int mid, float u, float v, f3 ro, f3 rd, int prim) {
    if (mid < 0) return true;
    const pt_material& m = S.materials[mid];
    if (m.kind != PT_MAT_DIFFUSE && m.kind != PT_MAT_DIELECTRIC) return true;
    float a = m.alpha >= 0 ? tex_eval_t<false>(m.alpha, u, v).x : tex_alpha(m.tex, u, v);
    if (m.alpha_mode == PT_ALPHA_OPAQUE) return true;
    if (m.alpha_mode == PT_ALPHA_MASK) return a > m.alpha_cutoff;
    return a >= 1.0f ? true : (blend_random(ro, rd, prim) < a);
}

// ------------------------------------------------------------------ onb (Onb.hpp:3-30)
struct Onb {
    f3 a0, a1, a2;
};
__device__ __forceinline__ Onb onb_n(f3 n) {
    Onb b;
    b.a2 = n;
    f3 up = (fabsf(n.x) > 0.9999) ? F3(0, 1, 0) : F3(1, 0, 0);
    b.a1 = normalize(cross(b.a2, up));
    b.a0 = cross(b.a1, b.a2);
    return b;
}
__device__ __forceinline__ Onb onb_si(const SurfInt& si) {
    Onb b;
    b.a2 = si.ns;
    b.a0 = si.tangent;
    b.a1 = cross_v(b.a2, b.a0);
    return b;
}
// onb::toWorld as the reference build compiles it: the out-of-line copy the
// scatter functions call is fma(v.z, a2, fma(v.y, a1, v.x*a0)) in every lane;
// inlined into sample_normalMap the x, y lanes become fma(v.z, a2, fma(v.x, a0, v.y*a1))
__device__ __forceinline__ f3 to_world(const Onb& b, f3 v) {
    return F3(fma_(v.z, b.a2.x, fma_(v.y, b.a1.x, rmul(v.x, b.a0.x))),
              fma_(v.z, b.a2.y, fma_(v.y, b.a1.y, rmul(v.x, b.a0.y))),
              fma_(v.z, b.a2.z, fma_(v.y, b.a1.z, rmul(v.x, b.a0.z))));
}
__device__ __forceinline__ f3 to_world_nm(const Onb& b, f3 v) {
    return F3(fma_(v.z, b.a2.x, fma_(v.x, b.a0.x, rmul(v.y, b.a1.x))),
              fma_(v.z, b.a2.y, fma_(v.x, b.a0.y, rmul(v.y, b.a1.y))),
              fma_(v.z, b.a2.z, fma_(v.y, b.a1.z, rmul(v.x, b.a0.z))));
}
__device__ __forceinline__ f3 to_local(const Onb& b, f3 v) { return F3(dot(v, b.a0), dot(v, b.a1), dot(v, b.a2)); }

// sample_normalMap (Material.hpp:344-348, 580-584)
__device__ f3 normal_map(int mid, const SurfInt& si) {
    if (mid < 0) return si.ns;
    const pt_material m = mat_rec(mid);
    if ((m.kind != PT_MAT_DIFFUSE && m.kind != PT_MAT_DIELECTRIC) || m.norm < 0) return si.ns;
    f3 t = tex_eval(m.norm, si.u, si.v);
    f3 nn = normalize(2.0f * t - F3(1, 1, 1));
    return to_world_nm(onb_si(si), nn);
}

// SphereShape::GetSphereUV (Shape.hpp:35-43) after its normalisation
__device__ __forceinline__ void sphere_uv_n(f3 p, float& u, float& v) {
    float theta = pt_acosf(clampf(p.y, -1.0f, 1.0f));
    float phi = pt_atan2f(p.z, p.x);
    if (phi < 0) phi += 2.0f * PT_PI;
    u = PT_INV_PI * phi * 0.5f;
    v = PT_INV_PI * theta;
}
__device__ __forceinline__ void sphere_uv(f3 p, float& u, float& v) { sphere_uv_n(normalize(p), u, v); }

// ------------------------------------------------------------------ interaction reconstruction
// TriangleShape::Intersect shading part (Shape.cpp:206-242) from the hit's
// barycentrics; identical to computing it at the candidate (the reference does
// it per candidate, only the last accepted survives).
__device__ void tri_interaction(const DevGeom& g, const DevTriShade& R, int mid, f3 o, f3 d, float t,
                                float bu, float bv, SurfInt& si, bool nm = true) {
    // one shading record (DevTriShade, the slot's) instead of S.tri + the
    // indexed normals / uvs / tangents: the same values, the same arithmetic
    const float4 ra = R.a, rb = R.b, rc = R.c, rd = R.d;
    float u = bu, v = bv, w = 1.0f - u - v;
    si.u = lerp3f(u, rc.w, v, rd.y, w, rc.y);
    si.v = lerp3f(u, rd.x, v, rd.z, w, rc.z);
    // n0 = (a.x a.y a.z), n1 = (a.w b.x b.y), n2 = (b.z b.w c.x)
    f3 nn = normalize(F3(lerp3f(u, ra.w, v, rb.z, w, ra.x), lerp3f(u, rb.x, v, rb.w, w, ra.y),
                         lerp3f(u, rb.y, v, rc.x, w, ra.z)));
    f3 N = normalize(cross_v(xyz(g.b), xyz(g.c)));
    si.n = N;
    if (dot(N, nn) < 0) nn = -nn;
    si.t = t;
    si.ns = nn;
    // ray.at(t) + eps*N*sign as the reference build contracts it: x, y lanes
    // o + round(t*d), z lane fma(t, d, o); then one rounding for +-eps*N
    float sg = dot(d, N) > 0.0f ? -1.0f : 1.0f;
    si.p = F3(fma_(rmul(PT_EPS, N.x), sg, o.x + rmul(t, d.x)), fma_(rmul(PT_EPS, N.y), sg, o.y + rmul(t, d.y)),
              fma_(rmul(PT_EPS, N.z), sg, fma_(t, d.z, o.z)));
    if (__float_as_uint(rd.w) & 1u) {
        const float4 re = R.e, rf = R.f, rg = R.g;
        // t0 = (e.x e.y e.z), t1 = (e.w f.x f.y), t2 = (f.z f.w g.x)
        f3 tv = F3(lerp3f(u, re.w, v, rf.z, w, re.x), lerp3f(u, rf.x, v, rf.w, w, re.y),
                   lerp3f(u, rf.y, v, rg.x, w, re.z));
        float k = dot(si.ns, tv);  // tangent - ns*k fused (fixture search)
        si.tangent = normalize(F3(fma_(-si.ns.x, k, tv.x), fma_(-si.ns.y, k, tv.y), fma_(-si.ns.z, k, tv.z)));
    } else {
        f3 up = (fabsf(si.ns.x) > 0.9999f) ? F3(0, 1, 0) : F3(1, 0, 0);
        si.tangent = normalize(cross(up, si.ns));
    }
    if (nm) si.ns = normal_map(mid, si);
}

// QuadShape::Intersect (Shape.cpp:320-343) interaction part.
__device__ void quad_interaction(const pt_quad& q, f3 o, f3 d, float t, float a, float b, SurfInt& si) {
    f3 normal = ld3(q.normal);
    f3 nn = dot(d, normal) > 0 ? -normal : normal;
    si.u = a;
    si.v = b;
    si.t = t;
    si.ns = nn;
    si.n = normal;
    f3 up = (fabsf(si.ns.x) > 0.9999f) ? F3(0, 1, 0) : F3(1, 0, 0);
    si.tangent = normalize(cross(up, si.ns));
    const f3 at = at_f(o, d, t);  // as built: x, y lanes + eps*nn unfused, z lane fused
    si.p = F3(at.x + PT_EPS * nn.x, at.y + PT_EPS * nn.y, fma_(nn.z, PT_EPS, at.z));
}

// SphereShape::Intersect (Shape.cpp:3-37) interaction part.
__device__ void sphere_interaction(const pt_sphere& sp, f3 o, f3 d, float t, SurfInt& si) {
    si.t = t;
    const f3 at = at_f(o, d, t);
    si.ns = normalize(at - ld3(sp.center));
    si.n = si.ns;
    f3 up = (fabsf(si.ns.x) > 0.9999f) ? F3(0, 1, 0) : F3(1, 0, 0);
    si.tangent = normalize(cross(up, si.ns));
    si.p = F3(fma_(si.n.x, PT_EPS, at.x), fma_(si.n.y, PT_EPS, at.y), fma_(si.n.z, PT_EPS, at.z));  // fused (as built)
    sphere_uv(si.n, si.u, si.v);
}

// ------------------------------------------------------------------ microfacet (Material.hpp:55-142)
struct Dist {
    float ax, ay;
};
__device__ __forceinline__ Dist mkdist(float r) { return Dist{r * r, r * r}; }
__device__ float lambda_(const Dist& D, f3 w) {
    float cos2 = w.z * w.z;
    if (cos2 == 0) return 0;
    float sin2 = smax(0, 1 - cos2);
    float sinT = csqrt(sin2);
    float cosPhi = sinT == 0 ? 1 : clampf(w.x / sinT, -1.0f, 1.0f);
    float sinPhi = sinT == 0 ? 0 : clampf(w.y / sinT, -1.0f, 1.0f);
    // Material.hpp:66 as built: fma(cosPhi*ax, cosPhi*ax, (sinPhi*ay)^2)
    const float ca = cosPhi * D.ax, sa = sinPhi * D.ay;
    float alpha2 = fma_(ca, ca, sa * sa);
    return (csqrt(1.f + alpha2 * sin2 / cos2) - 1.0f) / 2.0f;
}
__device__ float D_(const Dist& D, f3 wh) {
    float cos2 = wh.z * wh.z;
    if (cos2 == 0) return 0;
    float cos4 = cos2 * cos2;
    float sin2 = smax(0, 1 - cos2);
    float sinT = csqrt(sin2);
    float cosPhi = sinT == 0 ? 1 : clampf(wh.x / sinT, -1.0f, 1.0f);
    float sinPhi = sinT == 0 ? 0 : clampf(wh.y / sinT, -1.0f, 1.0f);
    // Material.hpp:78-79 as built: the sum of squares fused and 1 + e fused
    // into one fma(sin2/cos2, sum, 1)
    const float cx = cosPhi / D.ax, sy = sinPhi / D.ay;
    const float e1 = fma_(sin2 / cos2, fma_(cx, cx, sy * sy), 1.0f);
    float denom = PT_PI * D.ax * D.ay * cos4 * e1 * e1;
    if (denom <= 0) return __int_as_float(0x7f800000);
    return 1 / denom;
}
__device__ __forceinline__ float G1_(const Dist& D, f3 w) { return 1 / (1 + lambda_(D, w)); }
__device__ __forceinline__ float G_(const Dist& D, f3 wo, f3 wi) { return 1 / (1 + lambda_(D, wo) + lambda_(D, wi)); }
__device__ __forceinline__ bool smooth_(const Dist& D) { return smax(D.ax, D.ay) < 1e-6; }
// MicrofacetDistribution::PDF with the caller's dot(wo, wh) (its order differs by call site)
__device__ __forceinline__ float mpdf_(const Dist& D, f3 wo, f3 wh, float dwh) {
    return D_(D, wh) * G1_(D, wo) * fabsf(dwh / wo.z);
}
// sampleGGXVNDF (Material.hpp:119-139) with the reference build's
// contractions; NE_INLINE: MicrofacetDielectric::scatter's inlined final
// normalisation (z^2 added unfused) instead of the out-of-line one
template <bool NE_INLINE>
__device__ f3 vndf_(float ax, float ay, f3 Ve, float U1, float U2) {
    f3 Vh = normalize(F3(ax * Ve.x, ay * Ve.y, Ve.z));
    float lensq = fma_(Vh.x, Vh.x, Vh.y * Vh.y);
    f3 T1 = lensq > 0 ? F3(-Vh.y, Vh.x, 0) * (1.0f / csqrt(lensq)) : F3(1, 0, 0);
    f3 T2 = cross_v(Vh, T1);
    float r = csqrt(U1);
    float phi = 2.0f * PT_PI * U2;
    float t1 = r * cos_cr(phi);
    float t2 = r * sin_cr(phi);
    float s = 0.5f * (1.0f + Vh.z);
    const float q1 = fma_(-t1, t1, 1.0f);  // 1 - t1*t1
    t2 = fma_(1.0f - s, csqrt(q1), s * t2);
    const float sq = csqrt(smax(0.0f, fma_(-t2, t2, q1)));
    // x, y lanes: t2*T2 rounded, t1*T1 fused; z lane: t1*T1 rounded, t2*T2 fused
    f3 Nh = F3(fma_(sq, Vh.x, fma_(t1, T1.x, t2 * T2.x)), fma_(sq, Vh.y, fma_(t1, T1.y, t2 * T2.y)),
               fma_(sq, Vh.z, fma_(t2, T2.z, t1 * T1.z)));
    const f3 ne = F3(ax * Nh.x, ay * Nh.y, smax(0.0f, Nh.z));
    if (!NE_INLINE) return normalize(ne);
    const float zz = Nh.z > 0 ? ne.z * ne.z : 0.0f;
    return ne * (1.0f / csqrt(fma_(ne.y, ne.y, ne.x * ne.x) + zz));
}
template <bool NE_INLINE>
__device__ __forceinline__ f3 sample_wh(const Dist& D, f3 wo, float u0, float u1) {
    bool flip = wo.z < 0;
    f3 wh = vndf_<NE_INLINE>(D.ax, D.ay, flip ? -wo : wo, u0, u1);
    return flip ? -wh : wh;
}
__device__ float fresnel_dielectric(float cosi, float eta) {  // Material.hpp:11-28
    cosi = clampf(cosi, -1.0f, 1.0f);
    if (cosi < 0) {
        eta = 1 / eta;
        cosi = -cosi;
    }
    // as built: 1 - cos^2, eta*cos -+ cost, cos -+ eta*cost and the sum of squares fused
    float sin2i = fma_(-cosi, cosi, 1.0f);
    float sin2t = sin2i / (eta * eta);
    if (sin2t >= 1) return 1.f;
    float cost = csqrt(1 - sin2t);
    float rpa = fma_(cosi, eta, -cost) / fma_(cosi, eta, cost);
    float rpe = fma_(-eta, cost, cosi) / fma_(eta, cost, cosi);
    return fma_(rpa, rpa, rpe * rpe) * 0.5f;
}
__device__ __forceinline__ f3 schlick(float c, f3 F0) {  // Material.hpp:30-32, F0 + (1 - F0)*p fused
    float p = pow_cr(1.0f - c, 5.0f);
    return F3(fma_(p, 1.0f - F0.x, F0.x), fma_(p, 1.0f - F0.y, F0.y), fma_(p, 1.0f - F0.z, F0.z));
}

// ------------------------------------------------------------------ materials
#define FL_TRANS 1u
#define FL_SPEC 2u
struct Bxdf {
    f3 f, o, d;
    float pdf;
    uint32_t flags;
    bool ok;
};

// A hit's material record and texture values, read once per hit: the
// reference evaluates the same textures again in scatter, calc_attenuation
// and PDF (Material.hpp:206-348, 392-564); the values are the same, so one
// evaluation serves all three and its texel loads are issued together.
struct MatTex {
    uint32_t kind;
    f3 col;       // tex (DIFFUSE / DIELECTRIC / THIN) or albedo (CONDUCTOR)
    float rough;  // DIFFUSE: max(rough.y, 0.0001) (GetRoughness); DIELECTRIC: rough.y
    float metal;  // DIFFUSE: metal.z
    float ri;
};
__device__ __forceinline__ MatTex mat_tex(int mid, SurfInt& si) {
    const pt_material m = mat_rec(mid);
    MatTex t;
    t.kind = m.kind;
    t.ri = m.ri;
    t.rough = 0.0f;
    t.metal = 0.0f;
    switch (m.kind) {
        case PT_MAT_DIFFUSE: {
            t.rough = smax(tex_eval(m.rough, si.u, si.v).y, 0.0001f);
            t.metal = tex_eval(m.metal, si.u, si.v).z;
            t.col = tex_eval(m.tex, si.u, si.v);
            break;
        }
        case PT_MAT_DIELECTRIC: {
            t.rough = tex_eval(m.rough, si.u, si.v).y;
            t.col = tex_eval(m.tex, si.u, si.v);
            break;
        }
        case PT_MAT_THIN: t.col = tex_eval(m.tex, si.u, si.v); break;
        default: t.col = ld3(m.albedo);
    }
    return t;
}
// onb TBN(dot(d, ns) > 0 ? -ns : ns) and wo = TBN.toLocal(-d) as
// MicrofacetDiffuse's three entry points are built: the sign test is the
// unfused dot and wo.z reuses it (+-dot(d, ns))
__device__ __forceinline__ f3 diffuse_frame(f3 d, f3 ns, Onb& tbn) {
    const float pd = dot_p(d, ns);
    tbn = onb_n(pd > 0 ? -ns : ns);
    const f3 md = -d;
    return F3(dot(md, tbn.a0), dot(md, tbn.a1), pd > 0 ? pd : -pd);
}

// MicrofacetDiffuse::scatter (Material.hpp:206-266)
__device__ Bxdf diffuse_scatter(const MatTex& m, f3 ind, const SurfInt& si, float u,
                                float uv0, float uv1) {
    Bxdf b;
    b.ok = false;
    float rough = m.rough;
    Dist D = mkdist(rough);
    float prob = rough >= 0.7 ? 1.0f : 0.5f;
    Onb tbn;
    f3 wo = diffuse_frame(ind, si.ns, tbn);
    f3 wi, wh;
    if (u >= prob) {
        wh = sample_wh<false>(D, wo, uv0, uv1);
        wi = reflect(-wo, wh);
    } else {
        float z = csqrt(1.0f - uv1);
        float phi = 2.0f * PT_PI * uv0;
        float s2 = csqrt(uv1);
        wi = F3(cos_cr(phi) * s2, sin_cr(phi) * s2, z);
        wh = normalize(wo + wi);
    }
    if (wi.z <= 0) return b;
    // as built: dot(wo, wh) in y, x, z order; prob*wi.z*inv_pi + spdf fused
    const float dwh = dot_yxz(wo, wh);
    float spdf = (1.0f - prob) * mpdf_(D, wo, wh, dwh) / (4 * fabsf(dwh));
    float pdf = fma_(prob * wi.z, PT_INV_PI, spdf);
    const f3 col = m.col;
    const float metal = m.metal;
    // glm::mix(0.04, col, metal) as built here: col*metal rounded, the other fused
    const float om = 1.0f - metal;
    f3 F0 = F3(fma_(om, 0.04f, col.x * metal), fma_(om, 0.04f, col.y * metal), fma_(om, 0.04f, col.z * metal));
    f3 F = schlick(dot_yxz(wi, wh), F0);
    f3 num = (D_(D, wh) * G_(D, wo, wi)) * F;
    float den = fabsf(4.0f * wo.z * wi.z);
    if (den == 0) return b;
    f3 spec = num / den;
    f3 kc = ((F3(1, 1, 1) - F) * om) * col;
    b.f = fma3s(PT_INV_PI, kc, spec);
    b.pdf = pdf;
    b.flags = 0;
    b.o = si.p;
    b.d = to_world(tbn, wi);
    b.ok = true;
    return b;
}
// MicrofacetDiffuse::calc_attenuation (Material.hpp:299-326)
__device__ f3 diffuse_f(const MatTex& m, f3 ind, const SurfInt& si, f3 dir) {
    Onb tbn;
    f3 wo = diffuse_frame(ind, si.ns, tbn);
    f3 wi = to_local(tbn, dir);
    f3 wh = normalize(wo + wi);
    const float rough = m.rough;
    const float metal = m.metal;
    Dist D = mkdist(rough);
    const f3 col = m.col;
    // glm::mix as built here: (1-metal)*0.04 rounded, col*metal fused
    const float om = 1.0f - metal, c4 = om * 0.04f;
    f3 F0 = F3(fma_(col.x, metal, c4), fma_(col.y, metal, c4), fma_(col.z, metal, c4));
    f3 F = schlick(dot_yxz(wi, wh), F0);
    f3 num = (D_(D, wh) * G_(D, wo, wi)) * F;
    float den = fabsf(4.0f * wo.z * wi.z);
    if (den == 0) return F3(0, 0, 0);
    const f3 kc = ((F3(1, 1, 1) - F) * om) * col;
    return fma3s(PT_INV_PI, kc, num / den);
}
// MicrofacetDiffuse::PDF (Material.hpp:281-296): no (1-prob) on the specular term (A.7)
__device__ float diffuse_pdf(const MatTex& m, f3 ind, const SurfInt& si, f3 dir) {
    const float rough = m.rough;
    Dist D = mkdist(rough);
    Onb tbn;
    f3 wo = diffuse_frame(ind, si.ns, tbn);
    f3 wh = to_local(tbn, normalize(dir - ind));
    float prob = rough >= 0.7 ? 1.0f : 0.5f;
    float diff = prob * fabsf(dot(si.ns, dir)) * PT_INV_PI;
    const float dwh = dot(wo, wh);
    float spec = mpdf_(D, wo, wh, dwh) / (4 * fabsf(dwh));
    return diff + spec;
}

// the out-of-line onb::toLocal (the dielectric's calls): x, y lanes in y, x, z order
__device__ __forceinline__ f3 to_local_ool(const Onb& b, f3 v) { return F3(dot_yxz(v, b.a0), dot_yxz(v, b.a1), dot(v, b.a2)); }

// MicrofacetDielectric::scatter (Material.hpp:392-477), contractions as built
__device__ Bxdf dielectric_scatter(const MatTex& m, f3 ino, f3 ind, const SurfInt& si,
                                   float u, float uv0, float uv1) {
    Bxdf b;
    b.ok = false;
    const float rough = m.rough;
    Dist D = mkdist(rough);
    Onb tbn = onb_si(si);
    const f3 md = -ind;
    f3 wo = to_local_ool(tbn, md);
    float ri = m.ri;
    float eta = dot_p(md, si.ns) > 0 ? 1 / ri : ri;
    const f3 hitp = at_f(ino, ind, si.t);
    if (ri == 1 || smooth_(D)) {
        f3 N = dot_p(ind, si.ns) > 0 ? -si.ns : si.ns;
        f3 Ng = dot(ind, si.n) > 0 ? -si.n : si.n;
        float F = fresnel_dielectric(wo.z, ri);
        float R = F, T = 1.0f - R;
        f3 dir;
        if (u < (R / (R + T))) {
            dir = to_world(tbn, F3(-wo.x, -wo.y, wo.z));
            b.o = F3(hitp.x + PT_EPS * Ng.x, hitp.y + PT_EPS * Ng.y, fma_(Ng.z, PT_EPS, hitp.z));
            b.f = (m.col * R) / fabsf(dot(si.ns, dir));
            b.pdf = R / (R + T);
        } else {
            dir = refract_f(ind, N, eta, dot(ind, N));
            if (is_zero(dir)) return b;
            b.o = F3(hitp.x - PT_EPS * Ng.x, hitp.y - PT_EPS * Ng.y, fma_(-Ng.z, PT_EPS, hitp.z));
            b.f = (m.col * T) / fabsf(dot(si.ns, dir));
            b.pdf = T / (R + T);
        }
        b.d = dir;
        b.flags = FL_TRANS | FL_SPEC;
        b.ok = true;
        return b;
    }
    f3 wh = sample_wh<true>(D, wo, uv0, uv1);
    f3 Ng = dot(ind, si.n) > 0 ? -si.n : si.n;
    const float dow = dot_p(wo, wh);  // dot(wo, wh), unfused, shared by every use below
    float F = fresnel_dielectric(dow, 1 / eta);
    float R = F, T = 1 - R;
    uint32_t fl = FL_TRANS | (rough < 0.001f ? FL_SPEC : 0u);
    if (u < (R / (R + T))) {
        f3 wi = -wo - (wh * (-dow)) * 2.0f;
        if (wo.z * wi.z < 0) return b;
        b.o = F3(hitp.x + PT_EPS * Ng.x, hitp.y + PT_EPS * Ng.y, fma_(Ng.z, PT_EPS, hitp.z));
        b.d = to_world(tbn, wi);
        b.pdf = mpdf_(D, wo, wh, dot(wo, wh)) / (fabsf(dow) * 4) * R / (R + T);
        b.f = (((m.col * D_(D, wh)) * G_(D, wo, wi)) * R) / fabsf(4 * wi.z * wo.z);
    } else {
        f3 wi = refract_f(-wo, wh, eta, -dow);
        if (wo.z * wi.z > 0 || wi.z == 0) return b;
        b.o = F3(hitp.x - PT_EPS * Ng.x, hitp.y - PT_EPS * Ng.y, fma_(-Ng.z, PT_EPS, hitp.z));
        b.d = to_world(tbn, wi);
        const float diw = dot(wi, wh);
        const float dn = fma_(eta, dow, diw);
        float denom = dn * dn;
        float dwh = fabsf(diw) / denom;
        b.pdf = mpdf_(D, wo, wh, dot(wo, wh)) * dwh * T / (R + T);
        float ft = T * D_(D, wh) * G_(D, wo, wi) * fabsf(diw * dow / (denom * wi.z * wo.z));
        b.f = m.col * ft;
    }
    b.flags = fl;
    b.ok = true;
    return b;
}
// MicrofacetDielectric::PDF / calc_attenuation (Material.hpp:484-564): each
// builds its own half vector, wi*etap + wo unfused in PDF and with the x, y
// lanes fused in calc_attenuation
template <bool FOR_F>
__device__ __forceinline__ bool dielectric_frame(const MatTex& m, f3 ind, const SurfInt& si, f3 dir, Dist& D,
                                                 f3& wo, f3& wi, f3& wh, float& etap, bool& refl) {
    const float rough = m.rough;
    D = mkdist(rough);
    float ri = m.ri;
    if (ri == 1 || smooth_(D)) return false;
    Onb tbn = onb_si(si);
    wo = to_local_ool(tbn, -ind);
    wi = to_local_ool(tbn, dir);
    float co = wo.z, ci = wi.z;
    refl = ci * co > 0;
    etap = 1;
    if (!refl) etap = co > 0 ? ri : (1 / ri);
    f3 h = (FOR_F && !refl) ? F3(fma_(wi.x, etap, wo.x), fma_(wi.y, etap, wo.y), co + ci * etap) : wi * etap + wo;
    if (dot(h, h) == 0) return false;
    h = normalize(h);
    if (h.z < 0) h = -h;
    wh = h;
    if (dot(h, wi) * ci <= 0.0 || dot(h, wo) * co <= 0.0) return false;
    return true;
}
__device__ void dielectric_eval(const MatTex& m, f3 ind, const SurfInt& si, f3 dir,
                                f3& f_out, float& pdf_out) {
    f_out = F3(0, 0, 0);
    pdf_out = 0;
    Dist D;
    f3 wo, wi, wh;
    float etap;
    bool refl;
    if (dielectric_frame<false>(m, ind, si, dir, D, wo, wi, wh, etap, refl)) {
        const float dow = dot(wh, wo), diw = dot(wh, wi);
        float F = fresnel_dielectric(dow, m.ri);
        float R = F, T = 1 - R;
        float pdf = mpdf_(D, wo, wh, dow);
        if (refl) {
            pdf_out = pdf / (fabsf(dow) * 4) * R / (R + T);
        } else {
            const float dn = dow / etap + diw;
            float dwh = fabsf(diw) / (dn * dn);
            pdf_out = dwh * pdf * T / (R + T);
        }
    }
    if (dielectric_frame<true>(m, ind, si, dir, D, wo, wi, wh, etap, refl)) {
        const float dow = dot(wh, wo), diw = dot(wh, wi);
        float F = fresnel_dielectric(dow, m.ri);
        const f3 col = m.col;
        if (refl) {
            f_out = (((col * D_(D, wh)) * G_(D, wo, wi)) * F) / fabsf(4 * wi.z * wo.z);
        } else {
            const float dn = dow / etap + diw;
            float den2 = dn * dn * wi.z * wo.z;
            float ft = (1 - F) * D_(D, wh) * G_(D, wo, wi) * fabsf(diw * dow / den2);
            f_out = col * ft;
        }
    }
}
// ThinDielectric::scatter (Material.hpp:605-644)
__device__ Bxdf thin_scatter(const MatTex& m, f3 ino, f3 ind, const SurfInt& si, float u) {
    Bxdf b;
    // as built: onb(si)'s cross rounded-first in every lane, wo.x and wo.y in
    // y, x, z order, 1 - R*R fused, hit point fused, +-eps*Ng unfused
    Onb tbn;
    tbn.a2 = si.ns;
    tbn.a0 = si.tangent;
    tbn.a1 = cross_r(tbn.a2, tbn.a0);
    const f3 md = -ind;
    f3 wo = F3(dot_yxz(md, tbn.a0), dot_yxz(md, tbn.a1), dot(md, tbn.a2));
    f3 Ng = dot(ind, si.n) > 0 ? -si.n : si.n;
    float F = fresnel_dielectric(wo.z, m.ri);
    float R = F, T = 1.0f - R;
    if (R < 1.0f) {
        R += T * T * R / fma_(-R, R, 1.0f);
        T = 1.0f - R;
    }
    const f3 hitp = at_f(ino, ind, si.t);
    f3 dir, f;
    if (u < (R / (R + T))) {
        dir = to_world(tbn, F3(-wo.x, -wo.y, wo.z));
        b.o = PT_EPS * Ng + hitp;
        f = (F3(1, 1, 1) * R) / fabsf(dot(si.ns, dir));
        b.pdf = R / (R + T);
    } else {
        dir = ind;
        b.o = hitp - PT_EPS * Ng;
        f = (F3(1, 1, 1) * T) / fabsf(dot(si.ns, dir));
        b.pdf = T / (R + T);
    }
    b.f = f * m.col;
    b.d = dir;
    b.flags = FL_TRANS | FL_SPEC;
    b.ok = true;
    return b;
}
// SpecularConductor::scatter (Material.hpp:664-669)
__device__ Bxdf conductor_scatter(const MatTex& m, f3 ind, const SurfInt& si) {
    Bxdf b;
    b.ok = false;
    f3 d = reflect(ind, si.ns);
    float dt = dot(d, si.ns);
    if (dt <= 0) return b;
    b.f = schlick(dot(si.ns, -ind), m.col) / dt;
    b.pdf = 1;
    b.flags = FL_SPEC;
    b.o = si.p;
    b.d = d;
    b.ok = true;
    return b;
}

// The material and light entry points are inlined into k_shade: taken out of
// line, their `const SurfInt&` argument kept the interaction in scratch memory
// on every path (k_shade<PATH>: 160 -> 16 B of scratch per lane).
__device__ __forceinline__ Bxdf mat_scatter(const MatTex& m, f3 ino, f3 ind, const SurfInt& si, float u, float uv0,
                            float uv1) {
    switch (m.kind) {
        case PT_MAT_DIFFUSE: return diffuse_scatter(m, ind, si, u, uv0, uv1);
        case PT_MAT_DIELECTRIC: return dielectric_scatter(m, ino, ind, si, u, uv0, uv1);
        case PT_MAT_THIN: return thin_scatter(m, ino, ind, si, u);
        default: return conductor_scatter(m, ind, si);
    }
}
__device__ __forceinline__ f3 mat_f(const MatTex& m, f3 ind, const SurfInt& si, f3 dir) {
    f3 f;
    float p;
    switch (m.kind) {
        case PT_MAT_DIFFUSE: return diffuse_f(m, ind, si, dir);
        case PT_MAT_DIELECTRIC: dielectric_eval(m, ind, si, dir, f, p); return f;
        case PT_MAT_THIN: return F3(0, 0, 0);
        default: return F3(1, 1, 1);  // base Material::calc_attenuation
    }
}
__device__ __forceinline__ float mat_pdf(const MatTex& m, f3 ind, const SurfInt& si, f3 dir) {
    f3 f;
    float p;
    switch (m.kind) {
        case PT_MAT_DIFFUSE: return diffuse_pdf(m, ind, si, dir);
        case PT_MAT_DIELECTRIC: dielectric_eval(m, ind, si, dir, f, p); return p;
        default: return 0;
    }
}

// ------------------------------------------------------------------ lights (Light.cpp)
// ---- instance transforms (TransformedPrimitive::Intersect / IntersectPred,
// Primitive.cpp:42-72; TransformedLight, Light.cpp:300-336): glm mat4 * vec4 as the reference build contracts it
// (fixture search): fma(m0, x, m1*y) + fma(m2, z, m3*w)
__device__ __forceinline__ f3 m4_point(const float* m, f3 p) {
    return F3(fma_(m[0], p.x, rmul(m[4], p.y)) + fma_(m[8], p.z, m[12]),
              fma_(m[1], p.x, rmul(m[5], p.y)) + fma_(m[9], p.z, m[13]),
              fma_(m[2], p.x, rmul(m[6], p.y)) + fma_(m[10], p.z, m[14]));
}
__device__ __forceinline__ f3 m4_dir(const float* m, f3 v) {
    return F3(fma_(m[0], v.x, rmul(m[4], v.y)) + fma_(m[8], v.z, rmul(m[12], 0.0f)),
              fma_(m[1], v.x, rmul(m[5], v.y)) + fma_(m[9], v.z, rmul(m[13], 0.0f)),
              fma_(m[2], v.x, rmul(m[6], v.y)) + fma_(m[10], v.z, rmul(m[14], 0.0f)));
}
// transpose(inverse(mat3(T))) (glm compute_inverse<3,3>) with the reference
// build's contraction (fixture search), NM[c*3+r]
__device__ __forceinline__ float df_(float a, float b, float c, float d) { return fma_(a, b, -rmul(c, d)); }
__device__ __forceinline__ float dfn_(float a, float b, float c, float d) { return fma_(-a, b, rmul(c, d)); }
__device__ void normal_matrix(const float* T, float* NM) {
#define M(c, r) T[(c) * 4 + (r)]
    const float D0 = df_(M(1, 1), M(2, 2), M(2, 1), M(1, 2)), D1 = df_(M(0, 1), M(2, 2), M(2, 1), M(0, 2));
    const float D2 = df_(M(0, 1), M(1, 2), M(1, 1), M(0, 2));
    const float od = 1.0f / fma_(M(2, 0), D2, fma_(M(0, 0), D0, -rmul(M(1, 0), D1)));
    // NM[c*3 + r] = Inverse[r][c]; the negated cofactors -(a*b - c*d) as the
    // build folds them, -(a*b) + c*d (FNMA: +0 where a*b == c*d, not -0)
    NM[0] = D0 * od;
    NM[1] = dfn_(M(1, 0), M(2, 2), M(2, 0), M(1, 2)) * od;
    NM[2] = df_(M(1, 0), M(2, 1), M(2, 0), M(1, 1)) * od;
    NM[3] = dfn_(M(0, 1), M(2, 2), M(2, 1), M(0, 2)) * od;
    NM[4] = df_(M(0, 0), M(2, 2), M(2, 0), M(0, 2)) * od;
    NM[5] = dfn_(M(0, 0), M(2, 1), M(2, 0), M(0, 1)) * od;
    NM[6] = D2 * od;
    NM[7] = dfn_(M(0, 0), M(1, 2), M(1, 0), M(0, 2)) * od;
    NM[8] = df_(M(0, 0), M(1, 1), M(1, 0), M(0, 1)) * od;
#undef M
}
// glm mat3 * vec3: fma(m2, z, fma(m0, x, m1*y)) per row (fixture search)
__device__ __forceinline__ f3 m3_mul(const float* M, f3 v) {
    return F3(fma_(M[6], v.z, fma_(M[0], v.x, rmul(M[3], v.y))), fma_(M[7], v.z, fma_(M[1], v.x, rmul(M[4], v.y))),
              fma_(M[8], v.z, fma_(M[2], v.x, rmul(M[5], v.y))));
}
// glm::normalize of a vec4 with w = 0: dot = fma(y, y, x*x) + z*z (fixture search)
__device__ __forceinline__ f3 normalize4(f3 v) {
    const float d = fma_(v.y, v.y, rmul(v.x, v.x)) + rmul(v.z, v.z);
    return v * (1.0f / csqrt(d));
}

// ---- AnimatedPrimitive / AnimatedLight (Primitive.cpp:76-96, Light.cpp:338-364):
// a TransformedPrimitive / TransformedLight over glm::translate(mat4(1),
// dir * t), t = glm::clamp(time - t0, t0, t1) / (t1 - t0), rebuilt per ray at
// the ray's time (the reference builds the temporary per call); its
// glm::inverse in closed form (anim_inverse below).
__device__ __forceinline__ void anim_transform(const DevInstance& I, float time, float* T) {
    const float t0 = I.t0, t1 = I.t1;
    float x = time - t0;
    x = t0 > x ? t0 : x;  // glm::max (func_common.inl:29)
    x = t1 < x ? t1 : x;  // glm::min (func_common.inl:20)
    const float t = x / (t1 - t0);
#pragma unroll
    for (int k = 0; k < 16; k++) T[k] = (k % 5 == 0) ? 1.0f : 0.0f;
    // column 3 = m[0]*v.x + m[1]*v.y + m[2]*v.z + m[3] over the identity: the
    // products are exact, so v itself, a zero made +0 by the final add
#pragma unroll
    for (int k = 0; k < 3; k++) T[12 + k] = rmul(I.mdir[k], t) + 0.0f;
}
// glm::inverse of anim_transform's matrix as the reference build computes it
// (AnimatedPrimitive::Intersect builds a TransformedPrimitive, whose ctor
// calls glm::inverse, Primitive.hpp:37), in closed form: compute_inverse<4,4>
// with g++'s contractions (pt_bvh.cpp pt_mat4_inverse; the oracle's
// mat4_inverse_) on identity + translation t (finite, never -0) gives 1 on the
// diagonal, -t in column 3 and zeros whose signs follow t's signs through the
// fused cofactors.  The rules below were read off that formula and checked
// against it on 60 000 translations from 1e-40 to 1e38 of every sign pattern;
// the motion parity scenes pin them against the reference harness.  As a
// closed form it needs no cofactor registers in the traversal's instance step.
__device__ __forceinline__ void anim_inverse(const float* T, float* out) {
    const float tx = T[12], ty = T[13], tz = T[14];
    constexpr float z = 0.0f, nz = -0.0f;
    out[0] = 1.0f, out[2] = z, out[3] = nz;
    out[5] = 1.0f, out[7] = z;
    out[8] = z, out[10] = 1.0f, out[11] = nz;
    out[1] = (ty > 0.0f || (ty == 0.0f && tz < 0.0f)) ? z : nz;
    out[4] = (tx > 0.0f || (tx == 0.0f && tz < 0.0f)) ? z : nz;
    out[6] = (tz < 0.0f && tx >= 0.0f) ? z : nz;
    out[9] = (ty < 0.0f && tx >= 0.0f) ? z : nz;
    out[12] = tx != 0.0f ? -tx : ((ty < 0.0f || (ty > 0.0f && tz >= 0.0f)) ? z : nz);
    out[13] = 0.0f - ty;
    out[14] = tz != 0.0f ? -tz : ((tx > 0.0f || (tx == 0.0f && ty < 0.0f)) ? z : nz);
    out[15] = 1.0f;
}
// An instance's transform and inverse at a ray's time: the uploaded pair, or
// an AnimatedPrimitive's rebuilt at `time` (S.motion: the scene has one)
__device__ __forceinline__ void inst_matrices(const DevInstance& I, float time, float* T, float* inv) {
    if (S.motion && I.anim) {
        anim_transform(I, time, T);
        anim_inverse(T, inv);
    } else {
#pragma unroll
        for (int k = 0; k < 16; k++) {
            T[k] = I.T[k];
            inv[k] = I.inv[k];
        }
    }
}

struct LSample {
    f3 L, p, n, dir;
    float u, v;
};
__device__ __forceinline__ uint4 tri_idx(uint32_t tri) { return S.tri[tri]; }

// the triangle parts of Shape::Area / Sample (Shape.cpp:277-315) over the
// vertices and uvs themselves (shape_area / shape_sample, or a light's
// DevLightTri: the same values, the same arithmetic)
__device__ __forceinline__ float tri_area(f3 v0, f3 v1, f3 v2) { return length(cross(v0 - v2, v1 - v2)) * 0.5f; }
__device__ __forceinline__ void tri_sample(f3 v0, f3 v1, f3 v2, float a0, float a1, float a2, float b0, float b1,
                                           float b2, float u0, float u1, LSample& ls) {
    float w = 1.0f - u0 - u1;  // not folded
    f3 n = normalize(cross(v1 - v0, v2 - v0));
    if (n.x != n.x) n = F3(0, 0, 0);
    ls.p = F3(lerp3f(u0, v1.x, u1, v2.x, w, v0.x), lerp3f(u0, v1.y, u1, v2.y, w, v0.y),
              lerp3f(u0, v1.z, u1, v2.z, w, v0.z));
    ls.u = lerp3f(u0, a1, u1, a2, w, a0);
    ls.v = lerp3f(u0, b1, u1, b2, w, b0);
    ls.n = n;
}
__device__ float shape_area(uint32_t kind, uint32_t index) {
    if (kind == PT_PRIM_QUAD) {
        const pt_quad& q = S.quads[index];
        return length(cross(ld3(q.u), ld3(q.v)));
    }
    if (kind == PT_PRIM_SPHERE) {
        float r = S.spheres[index].radius;
        return 4.0f * PT_PI * r * r;
    }
    uint4 T = tri_idx(index);
    f3 v0 = ld3(S.positions + 3 * T.x), v1 = ld3(S.positions + 3 * T.y), v2 = ld3(S.positions + 3 * T.z);
    return tri_area(v0, v1, v2);
}
// Shape::Sample (Shape.cpp:74-81, 277-297; Shape.hpp:139-141)
__device__ void shape_sample(uint32_t kind, uint32_t index, float u0, float u1, LSample& ls) {
    ls.u = 0;
    ls.v = 0;
    if (kind == PT_PRIM_QUAD) {
        const pt_quad& q = S.quads[index];
        const f3 Q = ld3(q.Q), qu = ld3(q.u), qv = ld3(q.v);  // Q + u0*u + u1*v, both fused
        ls.p = F3(fma_(qv.x, u1, fma_(qu.x, u0, Q.x)), fma_(qv.y, u1, fma_(qu.y, u0, Q.y)),
                  fma_(qv.z, u1, fma_(qu.z, u0, Q.z)));
        ls.n = ld3(q.normal);
    } else if (kind == PT_PRIM_SPHERE) {
        const pt_sphere& sp = S.spheres[index];
        float z = 1.0f - 2.0f * u0;
        float r = csqrt(fma_(-z, z, 1.0f));
        float phi = 2.0f * PT_PI * u1;
        f3 d = F3(r * cos_cr(phi), r * sin_cr(phi), z);
        f3 c = ld3(sp.center);
        ls.p = F3(fma_(sp.radius, d.x, c.x), fma_(sp.radius, d.y, c.y), fma_(sp.radius, d.z, c.z));
        ls.n = normalize(ls.p - c);
        sphere_uv(ls.p, ls.u, ls.v);
    } else {
        uint4 T = tri_idx(index);
        f3 v0 = ld3(S.positions + 3 * T.x), v1 = ld3(S.positions + 3 * T.y), v2 = ld3(S.positions + 3 * T.z);
        const float* uvs = S.uvs;
        tri_sample(v0, v1, v2, uvs[2 * T.x], uvs[2 * T.y], uvs[2 * T.z], uvs[2 * T.x + 1], uvs[2 * T.y + 1],
                   uvs[2 * T.z + 1], u0, u1, ls);
    }
}
// Shape::PDF(interaction, ray) (Shape.cpp:61-67, 303-315; Shape.hpp:151-158)
// as built: dot(to, to) in y, x, z order; the quad's (inlined into
// AreaLight::PDF) light cosine also in y, x, z order except behind the
// one-sided test, whose dot(-d, n) it reuses
__device__ float shape_pdf_a(uint32_t kind, float area, f3 p, f3 n, f3 ro, f3 rd, bool one_sided) {
    f3 to = p - ro;
    float d2 = dot_yxz(to, to);
    float lc = fabsf(kind == PT_PRIM_QUAD && !one_sided ? dot_yxz(-rd, n) : dot(-rd, n));
    if (kind == PT_PRIM_QUAD) {
        if (area == 0) return 0;
    } else if (kind == PT_PRIM_SPHERE) {
        if (area * lc == 0) return 0;
    } else {
        if (area == 0 || lc == 0 || n.x != n.x) return 0;
    }
    return d2 / (lc * area);
}
__device__ __forceinline__ float shape_pdf(uint32_t kind, uint32_t index, f3 p, f3 n, f3 ro, f3 rd, bool one_sided) {
    return shape_pdf_a(kind, shape_area(kind, index), p, n, ro, rd, one_sided);
}
// TextureInfiniteLight::Le (Light.cpp:110-112): LeScale * tex(GetSphereUV(dir))
__device__ __noinline__ f3 texinf_le(const pt_light& l, f3 d) {
    float u, v;
    sphere_uv(d, u, v);
    return l.scale * tex_eval(l.tex, u, v);
}
__device__ __forceinline__ f3 inf_le(const pt_light& l, f3 d) {
    if (l.kind == PT_LIGHT_TEX_INF) return texinf_le(l, d);
    if (l.kind == PT_LIGHT_SKY_INF) {  // main.cpp:292-295 gradient
        // (1-a)*c0 rounded, a*c1 fused (fixture search)
        float a = 0.5f * (d.y + 1.0f), b = 1.0f - a;
        return l.scale * F3(fma_(a, l.vec[0], rmul(b, l.color[0])), fma_(a, l.vec[1], rmul(b, l.color[1])),
                            fma_(a, l.vec[2], rmul(b, l.color[2])));
    }
    return ld3(l.color);
}
// TransformedLight / AnimatedLight (Light.cpp:300-364): an emitter inside an
// instance; its AreaLight's shape stays in object space (l.prim is the BLAS
// slot).  Out of line: the rare path keeps k_shade's registers.  Values in and
// out (returned in registers): a reference argument would keep the caller's
// variables in scratch memory on every path.  Nested wrappers (a
// TransformedLight of a TransformedLight, what GetLights of a nested
// TransformedPrimitive returns, Primitive.cpp:66-73) apply their levels in the
// reference's call order: sample() transforms the inner light's sample, so
// the innermost level first; PDF() and L() transform the query before the
// inner light sees it, so the outermost first.
struct PN {
    f3 p, n;
};
// the levels of a chain from its outermost record, the outermost first; returns the count
__device__ __forceinline__ int inst_chain(const DevInstance* c, const DevInstance** lv) {
    int k = 0;
    for (;; c = &S.instances[c->inner]) {
        lv[k++] = c;
        if (c->inner < 0 || k == PT_MAX_INSTANCE_DEPTH) return k;
    }
}
// The time moves an AnimatedLight (its instance's translation at the ray's time).
__device__ __noinline__ PN tlight_to_world(int inst, f3 p, f3 n, float time) {  // TransformedLight::sample
    const DevInstance* lv[PT_MAX_INSTANCE_DEPTH];
    const int k = inst_chain(&S.instances[inst], lv);
    for (int j = k - 1; j >= 0; j--) {
        float T[16], inv[16], NM[9];
        inst_matrices(*lv[j], time, T, inv);
        normal_matrix(T, NM);
        p = m4_point(T, p);
        n = m3_mul(NM, n);
    }
    return PN{p, n};
}
struct TLObj {
    f3 p, n, ro, rd;
};
__device__ __noinline__ TLObj tlight_to_object(int inst, f3 p, f3 n, f3 ro, f3 rd, float time) {  // TransformedLight::PDF
    const DevInstance* lv[PT_MAX_INSTANCE_DEPTH];
    const int k = inst_chain(&S.instances[inst], lv);
    for (int j = 0; j < k; j++) {
        float T[16], inv[16];
        inst_matrices(*lv[j], time, T, inv);
        p = m4_point(inv, p);
        n = normalize(m4_dir(inv, n));
        ro = m4_point(inv, ro);
        rd = normalize(m4_dir(inv, rd));
    }
    return TLObj{p, n, ro, rd};
}
__device__ __noinline__ f3 tlight_normal(int inst, f3 n, float time) {  // TransformedLight::L's temp.n
    const DevInstance* lv[PT_MAX_INSTANCE_DEPTH];
    const int k = inst_chain(&S.instances[inst], lv);
    for (int j = 0; j < k; j++) {
        float T[16], inv[16], NM[9];
        inst_matrices(*lv[j], time, T, inv);
        normal_matrix(T, NM);
        n = m3_mul(NM, n);
    }
    return n;
}

// TextureInfiniteLight::sample (Light.cpp:118-144): the cell whose running
// sum first exceeds fl(uc * totalWeight) (std::upper_bound over the float
// sums), then the point (u0, u1) of that cell mapped to the
// sphere.  uc is the reference's hidden random_float() (Light.cpp:120),
// drawn from the sample stream by the caller.
struct DirUV {
    f3 dir;
    float u, v;
};
__device__ __noinline__ DirUV texinf_sample(const pt_light& l, float uc, float u0, float u1) {
    const float* acc = S.light_dist + l.prim;
    constexpr uint32_t N = (uint32_t)PT_TEXINF_X * PT_TEXINF_Y;
    // float weight = random_float() * totalWeight: the double product rounded
    // to float, then std::upper_bound compares float with float
    const float weight = (float)((double)uc * (double)acc[N - 1]);
    uint32_t lo = 0, hi = N;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (acc[mid] > weight) hi = mid;
        else lo = mid + 1;
    }
    const int cx = (int)(lo % PT_TEXINF_Y), cy = (int)(lo / PT_TEXINF_Y);
    const float cu = ((float)cx + u0) / (float)PT_TEXINF_X, cv = ((float)cy + u1) / (float)PT_TEXINF_Y;
    const float z = 2.0f * cu - 1.0f;
    const float th = 2.0f * PT_PI * cv;
    const float r = csqrt(1.0f - rmul(z, z));
    DirUV o;
    o.dir = F3(r * cos_cr(th), r * sin_cr(th), z);
    sphere_uv(o.dir, o.u, o.v);
    return o;
}
// TextureInfiniteLight::PDF (Light.cpp:146-150): luminance(Le) / totalWeight
// / cellOmega, luminance in double (Util.hpp:4-6)
__device__ __noinline__ float texinf_pdf(const pt_light& l, f3 rd) {
    const f3 le = texinf_le(l, rd);
    const double lum = fma((double)le.z, 0.0722, fma((double)le.y, 0.7152, (double)le.x * 0.2126));
    const double tot = (double)S.light_dist[l.prim + (uint32_t)PT_TEXINF_X * PT_TEXINF_Y - 1u];
    constexpr float cell_omega = 4.0f * PT_PI / (float)(PT_TEXINF_X * PT_TEXINF_Y);
    return (float)((lum / tot) * (double)(1.0f / cell_omega));
}
// TextureInfiniteLight::sample's hidden random_float() (Light.cpp:120) as a
// draw of the sample's stream outside its numbered dimensions: keyed by the
// stream key and the bounce's next dimension, so every bounce gets its own
__device__ __forceinline__ float texinf_uc(uint32_t key, uint32_t dim) { return draw(key ^ 0xC3115EEDu, dim); }
// Light::PDF({}, ray) of an infinite light (the escape MIS weight)
__device__ __forceinline__ float inf_pdf(const pt_light& l, f3 rd) {
    return l.kind == PT_LIGHT_TEX_INF ? texinf_pdf(l, rd) : 1.0f / (4.0f * PT_PI);
}

// time: the ray's (Light::sample(uv, time), Light.hpp:21) -- an AnimatedLight's
// (li: the light's index in S.lights; its DevLightTri is S.ltri[li])
__device__ __forceinline__ LSample light_sample(int li, float u0, float u1, float uc = 0.0f, float time = 0.0f) {
    const pt_light& l = S.lights[li];
    LSample ls;
    ls.L = F3(0, 0, 0);
    ls.p = F3(0, 0, 0);
    ls.n = F3(0, 0, 0);
    ls.dir = F3(0, 0, 0);
    ls.u = ls.v = 0;
    if (l.kind == PT_LIGHT_AREA) {  // AreaLight::sample (Light.cpp:261-263)
        const DevLightTri* R = S.ltri + li;
        float4 ra = make_float4(0, 0, 0, 0), rb = ra, rc = ra, rd = ra;
        if (PT_LIGHT_TRI) ra = R->a, rb = R->b, rc = R->c, rd = R->d;
        if (PT_LIGHT_TRI && __float_as_uint(rd.w)) {  // a triangle: its vertices and uvs gathered at upload
            tri_sample(xyz(ra), xyz(rb), xyz(rc), ra.w, rb.w, rc.w, rd.x, rd.y, rd.z, u0, u1, ls);
        } else {
            const DevPrimInfo& pi = S.info[l.prim];
            uint32_t kind = __float_as_uint(S.geom[l.prim].a.w) & GF_KIND;
            shape_sample(kind, pi.index, u0, u1, ls);
        }
        if (l.instance >= 0) {
            const PN w = tlight_to_world(l.instance, ls.p, ls.n, time);
            ls.p = w.p;
            ls.n = w.n;
        }
        return ls;
    }
    if (l.kind == PT_LIGHT_POINT) {  // Light.cpp:236-238
        ls.L = ld3(l.color);
        ls.p = ld3(l.vec);
        ls.n = F3(1, 1, 1);
        ls.u = u0;
        ls.v = u1;
        return ls;
    }
    if (l.kind == PT_LIGHT_TEX_INF) {
        const DirUV o = texinf_sample(l, uc, u0, u1);
        ls.dir = o.dir;
        ls.u = o.u;
        ls.v = o.v;
        return ls;
    }
    // Distant / Uniform / Function light sample (Light.cpp:36-41, 62-67, 209-214):
    // 1 - z*z fused except in FunctionInfiniteLight::sample, which also adds
    // z*z unfused in its GetSphereUV normalisation
    const bool sky = l.kind == PT_LIGHT_SKY_INF;
    float z = 2.0f * u0 - 1.0f;
    float th = 2.0f * PT_PI * u1;
    float r = sky ? csqrt(1.0f - z * z) : csqrt(fma_(-z, z, 1.0f));
    const float x = cos_cr(th) * r, y = sin_cr(th) * r;
    f3 d = F3(x, y, z);
    if (l.kind == PT_LIGHT_DISTANT) {  // Light.cpp:208-215
        ls.L = ld3(l.color);
        ls.u = u0;
        ls.v = u1;
        const f3 vv = ld3(l.vec);
        ls.dir = normalize(F3(fma_(d.x, 0.02f, vv.x), fma_(d.y, 0.02f, vv.y), fma_(d.z, 0.02f, vv.z)));
        return ls;
    }
    ls.L = inf_le(l, d);  // Light.cpp:35-42, 61-68
    if (sky)
        sphere_uv_n(d * (1.0f / csqrt(fma_(y, y, x * x) + z * z)), ls.u, ls.v);
    else
        sphere_uv(d, ls.u, ls.v);
    ls.dir = d;
    return ls;
}
__device__ __forceinline__ bool light_is_delta(const pt_light& l) {
    return l.kind == PT_LIGHT_DISTANT || l.kind == PT_LIGHT_POINT;
}
// Light::PDF(interaction, ray)
__device__ __forceinline__ float light_pdf(int li, f3 p, f3 n, f3 ro, f3 rd, float time = 0.0f) {
    const pt_light& l = S.lights[li];
    if (l.kind == PT_LIGHT_AREA) {  // Light.cpp:267-272
        const DevLightTri* R = S.ltri + li;
        float4 ra = make_float4(0, 0, 0, 0), rb = ra, rc = ra;
        bool tri = false;
        if (PT_LIGHT_TRI) ra = R->a, rb = R->b, rc = R->c, tri = __float_as_uint(R->d.w) != 0u;
        if (l.instance >= 0) {
            const TLObj o = tlight_to_object(l.instance, p, n, ro, rd, time);
            p = o.p;
            n = o.n;
            ro = o.ro;
            rd = o.rd;
        }
        uint32_t kind = PT_PRIM_TRIANGLE;
        float area;
        if (tri) {
            area = tri_area(xyz(ra), xyz(rb), xyz(rc));
        } else {
            kind = __float_as_uint(S.geom[l.prim].a.w) & GF_KIND;
            area = shape_area(kind, S.info[l.prim].index);
        }
        if (l.one_sided) return dot(-rd, n) > 0 ? shape_pdf_a(kind, area, p, n, ro, rd, true) : 0;
        return shape_pdf_a(kind, area, p, n, ro, rd, false);
    }
    if (l.kind == PT_LIGHT_UNIFORM_INF || l.kind == PT_LIGHT_SKY_INF) return 1.0f / (4.0f * PT_PI);
    if (l.kind == PT_LIGHT_TEX_INF) return texinf_pdf(l, rd);
    return 0;
}
// Light::L(interaction, ray)
__device__ __forceinline__ f3 light_L(const pt_light& l, f3 n, float u, float v, f3 rd, float time = 0.0f) {
    if (l.kind == PT_LIGHT_AREA) {  // Light.cpp:257-260
        if (l.instance >= 0) {  // TransformedLight::L: fresh interaction, uv (0, 0)
            n = tlight_normal(l.instance, n, time);
            u = v = 0;
        }
        if (l.one_sided && dot(rd, n) > 0) return F3(0, 0, 0);
        return tex_eval(l.tex, u, v);
    }
    if (l.kind == PT_LIGHT_UNIFORM_INF || l.kind == PT_LIGHT_SKY_INF || l.kind == PT_LIGHT_TEX_INF) return inf_le(l, rd);
    return F3(0, 0, 0);
}
// LightSampler::Sample (LightSampler.cpp:7-11, 34-46); the power sampler's
// linear scan becomes a binary search for the first running sum >= u*total
// over the same float running sums (identical pick for every u).
__device__ int ls_sample(float u) {
    uint32_t n = S.n_sampler_lights;
    if (n == 0) return -1;
    if (S.light_sampler == PT_LS_UNIFORM) {
        int idx = (int)(u * n);
        if (idx > (int)n - 1) idx = (int)n - 1;
        return (int)S.sampler_lights[idx];
    }
    float target = u * S.sampler_total;
    // first i with cdf[i] >= target; the guide table narrows [0, n) to
    // [guide[b], guide[b + 1]): target >= fl(b / K * total) because u >= b / K
    // and rounding is monotone, and target <= fl((b + 1) / K * total)
    const uint32_t b = min((uint32_t)(u * (float)PT_LS_GUIDE), PT_LS_GUIDE - 1u);
    uint32_t lo = S.sampler_guide[b], hi = S.sampler_guide[b + 1];
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (S.sampler_cdf[mid] >= target) hi = mid;
        else lo = mid + 1;
    }
    if (lo >= n) lo = n - 1;
    return (int)S.sampler_lights[lo];
}
