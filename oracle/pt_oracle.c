/*
 * pt_oracle.c — TEST INFRASTRUCTURE ONLY (see pt_oracle.h).
 *
 * A scalar C restatement of marko176/PathTracing's per-sample hot path over
 * the flat scene of include/pt_api.h.  Each function cites the reference
 * file:line it follows.  Float expressions keep the reference's operand order;
 * the build uses -ffp-contract=fast like the reference's GCC gnu++20 build.
 */
#define _GNU_SOURCE
#include "pt_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#define EPS_SHADOW 0.00001f /* shadowEpsilon (AABB.hpp:6) */
#define FLT_EPS 1.19209290e-07f
#define PI_F 3.14159265358979323846f
#define INV_PI_F 0.318309886183790671538f

int oracle_version(void) { return 1; }

/* ------------------------------------------------------------------ vec3 */
typedef struct { float x, y, z; } v3;
static inline v3 V(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 vl(const float* p) { return V(p[0], p[1], p[2]); }
static inline v3 add(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mul(v3 a, v3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 muls(v3 a, float s) { return V(a.x * s, a.y * s, a.z * s); }
static inline v3 smul(float s, v3 a) { return V(s * a.x, s * a.y, s * a.z); }
static inline v3 divs(v3 a, float s) { return V(a.x / s, a.y / s, a.z / s); }
static inline v3 neg(v3 a) { return V(-a.x, -a.y, -a.z); }
/* a*b rounded even where -ffp-contract=fast would fuse it into an add */
static inline float rmul(float a, float b) {
    float m = a * b;
    __asm__("" : "+x"(m));
    return m;
}
/* glm::dot: tmp = a*b; tmp.x + tmp.y + tmp.z (func_geometric.inl) */
/* contracted as the reference's GCC build emits it: x product rounded, then
 * fma(y) and fma(z) (SphereShape::Intersect disassembly) */
static inline float dot(v3 a, v3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
/* other orders the build emits for glm::dot (tools/refgimple.py): y product
 * rounded then fma(x), fma(z); and the unfused sum (x + y) + z */
static inline float dot_yxz(v3 a, v3 b) { return fmaf(a.z, b.z, fmaf(a.x, b.x, a.y * b.y)); }
static inline float dot_p(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
/* glm::cross as the reference build contracts it (x, y lanes vectorised:
 * first product rounded, second fused; z scalar: first fused) */
/* glm::cross in scalar code: first product fused, second rounded
 * (glm::intersectRayTriangle's cross(dir, e2) in the reference build) */
static inline v3 cross(v3 a, v3 b) {
    return V(fmaf(a.y, b.z, -rmul(b.y, a.z)), fmaf(a.z, b.x, -rmul(b.z, a.x)), fmaf(a.x, b.y, -rmul(b.x, a.y)));
}
static inline v3 cross_r(v3 a, v3 b) { /* every lane: first product rounded, second fused */
    return V(fmaf(-b.y, a.z, rmul(a.y, b.z)), fmaf(-b.z, a.x, rmul(a.z, b.x)), fmaf(-b.x, a.y, rmul(a.x, b.y)));
}
static inline v3 cross_v(v3 a, v3 b) {
    return V(fmaf(-b.y, a.z, a.y * b.z), fmaf(-b.z, a.x, a.z * b.x), fmaf(a.x, b.y, -(b.x * a.y)));
}
static inline float length3(v3 a) { return sqrtf(dot(a, a)); }
/* glm::normalize = v * inversesqrt(dot(v,v)), inversesqrt = 1/sqrt */
static inline v3 normalize(v3 a) { return muls(a, 1.0f / sqrtf(dot(a, a))); }
static inline int is_zero(v3 a) { return a.x == 0.0f && a.y == 0.0f && a.z == 0.0f; }
static inline v3 reflect(v3 I, v3 N) { return sub(I, muls(muls(N, dot(N, I)), 2.0f)); }
static inline v3 refract(v3 I, v3 N, float eta) {
    float d = dot(N, I);
    float k = 1.0f - eta * eta * (1.0f - d * d);
    if (k >= 0.0f) return sub(smul(eta, I), smul(eta * d + sqrtf(k), N));
    return V(0, 0, 0);
}
/* u*a + v*b + w*c as glm's vector expressions compile in the reference
 * build: first product rounded, the others fused in order */
static inline float lerp3f(float u, float a, float v, float b, float w, float c) {
    return fmaf(w, c, fmaf(v, b, rmul(u, a)));
}
static inline float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }
/* a*b + c per lane, fused (glm's `c += a * b` as the reference build contracts it) */
static inline v3 fma3(v3 a, v3 b, v3 c) { return V(fmaf(a.x, b.x, c.x), fmaf(a.y, b.y, c.y), fmaf(a.z, b.z, c.z)); }
static inline v3 fma3s(float s, v3 b, v3 c) { return V(fmaf(s, b.x, c.x), fmaf(s, b.y, c.y), fmaf(s, b.z, c.z)); }
static inline float fmaxf_(float a, float b) { return a < b ? b : a; } /* std::max */

/* ------------------------------------------------------------------ RNG */
/* The sample stream (DESIGN.md "Sample stream"): PCG-RXS-M-XS hash. */
static inline uint32_t pcg_hash(uint32_t v) {
    uint32_t state = v * 747796405u + 2891336453u;
    uint32_t word = ((state >> ((state >> 28u) + 4u)) ^ state) * 277803737u;
    return (word >> 22u) ^ word;
}
static inline uint32_t stream_key(uint32_t seed, uint32_t pixel, uint32_t sample) {
    return pcg_hash(pcg_hash(seed ^ pcg_hash(pixel)) + sample);
}
typedef struct { uint32_t key, dim; } rng_t;
static inline float next1(rng_t* r) {
    return (float)(pcg_hash(r->key + 0x9E3779B9u * r->dim++) >> 8) * (1.0f / 16777216.0f);
}
/* Alpha Blend draws random_float() (Material.hpp:189) from a nondeterministic
 * thread-local generator; parity is waived there: we draw a hash of the ray. */
static inline uint32_t fbits(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}
static inline float blend_random(v3 o, v3 d, int prim) { /* the device's draw (pt_shading.h) */
    uint32_t h = pcg_hash((uint32_t)prim);
    h = pcg_hash(h ^ fbits(o.x));
    h = pcg_hash(h ^ fbits(o.y));
    h = pcg_hash(h ^ fbits(o.z));
    h = pcg_hash(h ^ fbits(d.x));
    h = pcg_hash(h ^ fbits(d.y));
    h = pcg_hash(h ^ fbits(d.z));
    return (float)(h >> 8) * (1.0f / 16777216.0f);
}

/* ------------------------------------------------------------------ ray / interaction */
/* Ray (Ray.hpp:14-41): time is what AnimatedPrimitive / AnimatedLight read */
typedef struct { v3 o, inv, d; float time; } ray_t;
static inline ray_t mkray_t(v3 o, v3 d, float time) {
    /* Ray ctor (Ray.hpp:32-35) */
    ray_t r;
    r.o = o;
    r.d = d;
    r.inv.x = fabsf(d.x) < 1e-32f ? 1e32f : 1.0f / d.x;
    r.inv.y = fabsf(d.y) < 1e-32f ? 1e32f : 1.0f / d.y;
    r.inv.z = fabsf(d.z) < 1e-32f ? 1e32f : 1.0f / d.z;
    r.time = time;
    return r;
}
static inline ray_t mkray(v3 o, v3 d) { return mkray_t(o, d, 0.0f); }
static inline v3 at(const ray_t* r, float t) { return add(r->o, smul(t, r->d)); }

typedef struct {
    v3 p, n, ns, tangent;
    float uv[2], t;
    int prim, mat, light, medium;
} si_t;

/* ------------------------------------------------------------------ scene view */
typedef struct {
    const pt_scene_desc* s;
    uint8_t lut[8][135];
} scene_t;

/* BVH4::LUT (BVH.hpp:562-718) composed with PermToIndexLUT (10-17): the
 * permutation byte P(a,b,c,d), a = child visited first. */
static int is_perm(unsigned p) {
    unsigned seen = 0;
    for (int s = 0; s < 4; s++) seen |= 1u << ((p >> (2 * s)) & 3);
    return p < 256 && seen == 0xF;
}
static void build_lut(uint8_t lut[8][135]) {
    for (unsigned rs = 0; rs < 8; rs++) {
        unsigned sg[3] = {rs & 1u, (rs >> 1) & 1u, rs >> 2};
        for (unsigned code = 0; code < 135; code++) {
            unsigned topo = code / 27, rem = code % 27;
            unsigned s0 = rem % 3, s1 = (rem / 3) % 3, s2 = rem / 9;
            unsigned p = 0, l, r, sub;
            switch (topo) {
                case 0:
                    l = sg[s1] ? 4u : 1u;
                    r = sg[s2] ? 14u : 11u;
                    p = sg[s0] ? (r << 4) + l : (l << 4) + r;
                    break;
                case 1:
                    r = sg[s2] ? 14u : 11u;
                    sub = sg[s1] ? (r << 2) | 1u : (1u << 4) | r;
                    p = sg[s0] ? (sub << 2) : sub;
                    break;
                case 2:
                    l = sg[s2] ? 9u : 6u;
                    sub = sg[s1] ? (3u << 4) | l : (l << 2) | 3u;
                    p = sg[s0] ? (sub << 2) : sub;
                    break;
                case 3:
                    l = sg[s2] ? 4u : 1u;
                    sub = sg[s1] ? (2u << 4) | l : (l << 2) | 2u;
                    p = sg[s0] ? (3u << 6) | sub : (sub << 2) | 3u;
                    break;
                default:
                    l = sg[s2] ? 9u : 6u;
                    sub = sg[s1] ? (l << 2) : l;
                    p = sg[s0] ? (3u << 6) | sub : (sub << 2) | 3u;
                    break;
            }
            lut[rs][code] = is_perm(p) ? (uint8_t)p : 27u; /* 27 = P(0,1,2,3) */
        }
    }
}

/* ------------------------------------------------------------------ textures (Texture.hpp) */
static inline int wrap_index(int i, int n) {
    int m = i % n;
    if (m < 0) m += n;
    return m;
}
static inline float channel_at(const scene_t* S, const pt_image* im, int x, int y, int ch) {
    /* Image::GetChannelAt (Texture.hpp:43-48): reads byte ch-1 of the pixel
     * whatever the channel count. */
    int xi = wrap_index(x, im->width), yi = wrap_index(y, im->height);
    uint64_t idx = im->offset + ((uint64_t)yi * (uint64_t)im->width + (uint64_t)xi) * (uint64_t)im->channels +
                   (uint64_t)(ch - 1);
    if (im->format == PT_IMAGE_F32) { /* FloatImage::GetChannelAt (Texture.hpp:78-83) */
        uint64_t fi = im->offset + 4ull * (idx - im->offset);
        if (fi + 4 > S->s->n_texel_bytes) return 0.0f;
        float f;
        memcpy(&f, S->s->texels + fi, 4);
        return f;
    }
    if (idx >= S->s->n_texel_bytes) return 0.0f;
    return S->s->texels[idx] / 255.0f;
}
/* SURVEY 8(d) shading bytes: 4 texels x C channels x texel size per bilinear
 * ImageTexture::Evaluate fetch (shading only; the alpha test's fetches are
 * traversal work).  Per thread, folded into the counters by li_one. */
static __thread uint64_t tl_tex_bytes;
static v3 tex_eval(const scene_t* S, int id, const float uv[2]) {
    const pt_texture* t = &S->s->textures[id];
    if (t->kind == PT_TEX_SOLID) return vl(t->value); /* colorScale*albedo, precomputed */
    if (t->kind == PT_TEX_CHECKER) {
        /* Texture.hpp:203-207 */
        int ux = (int)floorf(uv[0] * t->inv_scale[0]);
        int uy = (int)floorf(uv[1] * t->inv_scale[1]);
        v3 c = ((ux + uy) % 2 == 0) ? tex_eval(S, t->a, uv) : tex_eval(S, t->b, uv);
        return mul(vl(t->scale), c);
    }
    /* ImageTexture::Evaluate (Texture.hpp:143-158) */
    const pt_image* im = &S->s->images[t->image];
    tl_tex_bytes += 4ull * (uint64_t)im->channels * (im->format == PT_IMAGE_F32 ? 4u : 1u);
    float x = uv[0] * im->width - 0.5f;
    float y = uv[1] * im->height - 0.5f;
    int xi = (int)floorf(x), yi = (int)floorf(y);
    float dx = x - xi, dy = y - yi;
    v3 a = V(channel_at(S, im, xi, yi, 1), channel_at(S, im, xi, yi, 2), channel_at(S, im, xi, yi, 3));
    v3 b = V(channel_at(S, im, xi + 1, yi, 1), channel_at(S, im, xi + 1, yi, 2), channel_at(S, im, xi + 1, yi, 3));
    v3 c = V(channel_at(S, im, xi, yi + 1, 1), channel_at(S, im, xi, yi + 1, 2), channel_at(S, im, xi, yi + 1, 3));
    v3 d = V(channel_at(S, im, xi + 1, yi + 1, 1), channel_at(S, im, xi + 1, yi + 1, 2),
             channel_at(S, im, xi + 1, yi + 1, 3));
    /* contraction of the reference build: w_a*a rounded, then fma(w_b, b),
     * fma(w_c, c), fma(w_d, d) in every channel */
    float wa = (1 - dx) * (1 - dy), wb = dx * (1 - dy), wc = (1 - dx) * dy, wd = dx * dy;
    v3 r = V(fmaf(wd, d.x, fmaf(wc, c.x, fmaf(wb, b.x, wa * a.x))),
             fmaf(wd, d.y, fmaf(wc, c.y, fmaf(wb, b.y, wa * a.y))),
             fmaf(wd, d.z, fmaf(wc, c.z, fmaf(wb, b.z, wa * a.z))));
    return mul(vl(t->scale), r);
}
static float tex_alpha(const scene_t* S, int id, const float uv[2]) {
    const pt_texture* t = &S->s->textures[id];
    if (t->kind == PT_TEX_SOLID) return 1.0f;
    if (t->kind == PT_TEX_CHECKER) {
        /* Texture.cpp:41-45 */
        int ux = (int)floorf(uv[0] * t->inv_scale[0]);
        int uy = (int)floorf(uv[1] * t->inv_scale[1]);
        return ((ux + uy) % 2 == 0) ? tex_alpha(S, t->a, uv) : tex_alpha(S, t->b, uv);
    }
    /* ImageTexture::alpha (Texture.cpp:47-62) */
    const pt_image* im = &S->s->images[t->image];
    if (im->channels != 4) return 1.0f;
    float x = uv[0] * im->width - 0.5f;
    float y = uv[1] * im->height - 0.5f;
    int xi = (int)floorf(x), yi = (int)floorf(y);
    float dx = x - xi, dy = y - yi;
    float a = channel_at(S, im, xi, yi, 4), b = channel_at(S, im, xi + 1, yi, 4);
    float c = channel_at(S, im, xi, yi + 1, 4), d = channel_at(S, im, xi + 1, yi + 1, 4);
    /* contraction of the reference build (ImageTexture::alpha, scalar):
     * w_b*b rounded, then fma(w_a, a), fma(w_c, c), fma(w_d, d) */
    float wa = (1 - dx) * (1 - dy), wb = dx * (1 - dy), wc = (1 - dx) * dy, wd = dx * dy;
    return fmaf(wd, d, fmaf(wc, c, fmaf(wa, a, wb * b)));
}

/* Material::Alpha (Material.hpp:336-342, 572-578); base Material: true. */
static int mat_alpha(const scene_t* S, int mid, const float uv[2], v3 ro, v3 rd, int prim) {
    if (mid < 0) return 1;
    const pt_material* m = &S->s->materials[mid];
    if (m->kind != PT_MAT_DIFFUSE && m->kind != PT_MAT_DIELECTRIC) return 1;
    float a;
    if (m->alpha >= 0) a = tex_eval(S, m->alpha, uv).x;
    else a = tex_alpha(S, m->tex, uv);
    switch (m->alpha_mode) {
        case PT_ALPHA_OPAQUE: return 1;
        case PT_ALPHA_MASK: return a > m->alpha_cutoff;
        default: return a >= 1.0f ? 1 : (blend_random(ro, rd, prim) < a);
    }
}
static inline int mat_has_alpha(const scene_t* S, int mid) {
    if (mid < 0) return 0;
    const pt_material* m = &S->s->materials[mid];
    if (m->kind != PT_MAT_DIFFUSE && m->kind != PT_MAT_DIELECTRIC) return 0;
    return m->alpha_mode != PT_ALPHA_OPAQUE;
}

/* ------------------------------------------------------------------ onb (Onb.hpp) */
typedef struct { v3 a0, a1, a2; } onb_t;
static inline onb_t onb_n(v3 n) {
    onb_t b;
    b.a2 = n;
    v3 up = (fabsf(n.x) > 0.9999) ? V(0, 1, 0) : V(1, 0, 0);
    b.a1 = normalize(cross(b.a2, up));
    b.a0 = cross(b.a1, b.a2);
    return b;
}
static inline onb_t onb_si(const si_t* si) {
    onb_t b;
    b.a2 = si->ns;
    b.a0 = si->tangent;
    b.a1 = cross_v(b.a2, b.a0);
    return b;
}
/* onb::toWorld (Onb.hpp:18-20) as the reference build compiles it: the
 * out-of-line copy the scatter functions call is fma(v.z, a2, fma(v.y, a1,
 * v.x*a0)) in every lane; inlined into sample_normalMap the x, y lanes become
 * fma(v.z, a2, fma(v.x, a0, v.y*a1)) */
static inline v3 to_world(const onb_t* b, v3 v) {
    return V(fmaf(v.z, b->a2.x, fmaf(v.y, b->a1.x, rmul(v.x, b->a0.x))),
             fmaf(v.z, b->a2.y, fmaf(v.y, b->a1.y, rmul(v.x, b->a0.y))),
             fmaf(v.z, b->a2.z, fmaf(v.y, b->a1.z, rmul(v.x, b->a0.z))));
}
static inline v3 to_world_nm(const onb_t* b, v3 v) {
    return V(fmaf(v.z, b->a2.x, fmaf(v.x, b->a0.x, v.y * b->a1.x)),
             fmaf(v.z, b->a2.y, fmaf(v.x, b->a0.y, v.y * b->a1.y)),
             fmaf(v.z, b->a2.z, fmaf(v.y, b->a1.z, v.x * b->a0.z)));
}
static inline v3 to_local(const onb_t* b, v3 v) { return V(dot(v, b->a0), dot(v, b->a1), dot(v, b->a2)); }
/* the out-of-line onb::toLocal (the dielectric's calls): x, y lanes in y, x, z order */
static inline v3 to_local_ool(const onb_t* b, v3 v) { return V(dot_yxz(v, b->a0), dot_yxz(v, b->a1), dot(v, b->a2)); }
/* ray.at(t) fused in every lane */
static inline v3 at_f(const ray_t* r, float t) {
    return V(fmaf(t, r->d.x, r->o.x), fmaf(t, r->d.y, r->o.y), fmaf(t, r->d.z, r->o.z));
}
/* glm::refract with the build's contractions, given d = dot(N, I) */
static inline v3 refract_f(v3 I, v3 N, float eta, float d) {
    float k = fmaf(-(eta * eta), fmaf(-d, d, 1.0f), 1.0f);
    if (k >= 0.0f) {
        float c = fmaf(eta, d, sqrtf(k));
        return V(fmaf(-c, N.x, eta * I.x), fmaf(-c, N.y, eta * I.y), fmaf(-c, N.z, eta * I.z));
    }
    return V(0, 0, 0);
}

/* sample_normalMap (Material.hpp:344-348, 580-584) */
static v3 normal_map(const scene_t* S, int mid, const si_t* si) {
    if (mid < 0) return si->ns;
    const pt_material* m = &S->s->materials[mid];
    if ((m->kind != PT_MAT_DIFFUSE && m->kind != PT_MAT_DIELECTRIC) || m->norm < 0) return si->ns;
    v3 t = tex_eval(S, m->norm, si->uv);
    v3 nn = normalize(sub(smul(2.0f, t), V(1, 1, 1)));
    onb_t b = onb_si(si);
    return to_world_nm(&b, nn);
}

/* ------------------------------------------------------------------ shapes (Shape.cpp) */
static void sphere_uv_n(v3 p, float uv[2]);
static void sphere_uv(v3 p, float uv[2]) { sphere_uv_n(normalize(p), uv); }
static void sphere_uv_n(v3 p, float uv[2]) {
    /* SphereShape::GetSphereUV (Shape.hpp:35-43) after its normalisation */
    float theta = acosf(clampf(p.y, -1.0f, 1.0f));
    float phi = atan2f(p.z, p.x);
    if (phi < 0) phi += 2.0f * PI_F;
    uv[0] = INV_PI_F * phi * 0.5f;
    uv[1] = INV_PI_F * theta;
}

/* glm::intersectRayTriangle (glm/gtx/intersect.inl:29-94) */
static int tri_glm(v3 o, v3 d, v3 v0, v3 e1, v3 e2, float* bx, float* by, float* t) {
    v3 p = cross(d, e2);
    float det = dot(e1, p);
    v3 perp;
    if (det > 0.0f) {
        v3 dist = sub(o, v0);
        *bx = dot(dist, p);
        if (*bx < 0.0f || *bx > det) return 0;
        perp = cross(dist, e1);
        *by = dot(d, perp);
        if (*by < 0.0f || *bx + *by > det) return 0;
    } else if (det < 0.0f) {
        v3 dist = sub(o, v0);
        *bx = dot(dist, p);
        if (*bx > 0.0f || *bx < det) return 0;
        perp = cross(dist, e1);
        *by = dot(d, perp);
        if (*by > 0.0f || *bx + *by < det) return 0;
    } else {
        return 0;
    }
    float inv = 1.0f / det;
    *t = dot(e2, perp) * inv;
    *bx *= inv;
    *by *= inv;
    return 1;
}

typedef struct { v3 v0, v1, v2; uint32_t i0, i1, i2; } tri_t;
static inline tri_t tri_get(const scene_t* S, uint32_t tri) {
    tri_t T;
    T.i0 = S->s->tri_vidx[3 * tri + 0];
    T.i1 = S->s->tri_vidx[3 * tri + 1];
    T.i2 = S->s->tri_vidx[3 * tri + 2];
    T.v0 = vl(S->s->positions + 3 * T.i0);
    T.v1 = vl(S->s->positions + 3 * T.i1);
    T.v2 = vl(S->s->positions + 3 * T.i2);
    return T;
}

/* TriangleShape::Intersect (Shape.cpp:185-245). Returns hit; fills si. */
static int tri_intersect(const scene_t* S, uint32_t tri, int mid, const ray_t* r, float max, si_t* si) {
    tri_t T = tri_get(S, tri);
    float bx, by, t = INFINITY;
    int hit = tri_glm(r->o, r->d, T.v0, sub(T.v1, T.v0), sub(T.v2, T.v0), &bx, &by, &t);
    if (!hit || t > max || t < EPS_SHADOW) return 0;
    float u = bx, v = by, w = 1.0f - u - v;
    const float* uvs = S->s->uvs;
    const float* nr = S->s->normals;
    si->uv[0] = lerp3f(u, uvs[2 * T.i1], v, uvs[2 * T.i2], w, uvs[2 * T.i0]);
    si->uv[1] = lerp3f(u, uvs[2 * T.i1 + 1], v, uvs[2 * T.i2 + 1], w, uvs[2 * T.i0 + 1]);
    const float *n1 = nr + 3 * T.i1, *n2 = nr + 3 * T.i2, *n0 = nr + 3 * T.i0;
    v3 nn = normalize(V(lerp3f(u, n1[0], v, n2[0], w, n0[0]), lerp3f(u, n1[1], v, n2[1], w, n0[1]),
                        lerp3f(u, n1[2], v, n2[2], w, n0[2])));
    v3 e1 = sub(T.v1, T.v0), e2 = sub(T.v2, T.v0);
    v3 N = normalize(cross_v(e1, e2));
    si->n = N;
    if (dot(N, nn) < 0) nn = neg(nn);
    si->t = t;
    si->ns = nn;
    /* ray.at(t) + eps*N*sign as the reference build contracts it: x, y lanes
     * o + round(t*d), z lane fma(t, d, o); then one rounding for +-eps*N */
    float sg = dot(r->d, N) > 0.0f ? -1.0f : 1.0f;
    v3 pa = V(r->o.x + rmul(t, r->d.x), r->o.y + rmul(t, r->d.y), fmaf(t, r->d.z, r->o.z));
    si->p = V(fmaf(rmul(EPS_SHADOW, N.x), sg, pa.x), fmaf(rmul(EPS_SHADOW, N.y), sg, pa.y),
              fmaf(rmul(EPS_SHADOW, N.z), sg, pa.z));
    if (S->s->tri_flags[tri] & 1u) {
        const float* tg = S->s->tangents;
        const float *t1 = tg + 3 * T.i1, *t2 = tg + 3 * T.i2, *t0 = tg + 3 * T.i0;
        v3 tv = V(lerp3f(u, t1[0], v, t2[0], w, t0[0]), lerp3f(u, t1[1], v, t2[1], w, t0[1]),
                  lerp3f(u, t1[2], v, t2[2], w, t0[2]));
        float k = dot(si->ns, tv); /* tangent - ns*k fused (fixture search) */
        si->tangent = normalize(V(fmaf(-si->ns.x, k, tv.x), fmaf(-si->ns.y, k, tv.y), fmaf(-si->ns.z, k, tv.z)));
    } else {
        v3 up = (fabsf(si->ns.x) > 0.9999f) ? V(0, 1, 0) : V(1, 0, 0);
        si->tangent = normalize(cross(up, si->ns));
    }
    si->ns = normal_map(S, mid, si);
    return 1;
}

/* TriangleShape::IntersectPred (Shape.cpp:246-268) */
static int tri_pred(const scene_t* S, uint32_t tri, const ray_t* r, float max) {
    tri_t T = tri_get(S, tri);
    v3 edge1 = sub(T.v1, T.v0), edge2 = sub(T.v2, T.v0);
    v3 h = cross(r->d, edge2);
    float det = dot(edge1, h);
    if (det > -FLT_EPS && det < FLT_EPS) return 0;
    float inv = 1.0f / det;
    v3 s = sub(r->o, T.v0);
    float u = dot(s, h) * inv;
    if (u < 0 || u > 1) return 0;
    v3 q = cross(s, edge1);
    float v = dot(r->d, q) * inv;
    if (v < 0 || u + v > 1) return 0;
    float t = dot(edge2, q) * inv;
    return t <= max && t >= EPS_SHADOW;
}

/* QuadShape::Intersect / IntersectPred (Shape.cpp:320-359) */
/* as built: Intersect tests and divides by dot(d, nn) fused, IntersectPred
 * by the unfused dot; alpha = dot(w, cross(ph, v)), beta = dot(w, cross(u, ph))
 * with the second cross rounded-first and its dot in y, x, z order */
static int quad_hit_(const pt_quad* q, const ray_t* r, float max, float* t_out, float* a_out, float* b_out,
                     v3* nn_out, int pred) {
    v3 normal = vl(q->normal);
    v3 nn = normal;
    float DD = q->D;
    float dn = pred ? dot_p(normal, r->d) : dot(r->d, normal);
    if (dn > 0) {
        nn = neg(normal);
        DD = -q->D;
    }
    float denom = pred ? (dn > 0 ? -dn : dn) : dot(r->d, nn);
    if (fabsf(denom) < 1e-8f) return 0;
    float t = (DD - dot(nn, r->o)) / denom;
    if (t < EPS_SHADOW || t > max) return 0;
    v3 ph = sub(at_f(r, t), vl(q->Q));
    v3 w = vl(q->w);
    float alpha = dot(w, cross(ph, vl(q->v)));
    float beta = dot_yxz(cross_r(vl(q->u), ph), w);
    if (!(alpha >= 0 && alpha <= 1 && beta >= 0 && beta <= 1)) return 0;
    *t_out = t;
    *a_out = alpha;
    *b_out = beta;
    *nn_out = nn;
    return 1;
}
static int quad_hit(const pt_quad* q, const ray_t* r, float max, float* t_out, float* a_out, float* b_out,
                    v3* nn_out) {
    return quad_hit_(q, r, max, t_out, a_out, b_out, nn_out, 1);
}
static int quad_intersect(const pt_quad* q, const ray_t* r, float max, si_t* si) {
    float t, a, b;
    v3 nn;
    if (!quad_hit_(q, r, max, &t, &a, &b, &nn, 0)) return 0;
    si->uv[0] = a;
    si->uv[1] = b;
    si->t = t;
    si->ns = nn;
    si->n = vl(q->normal);
    v3 up = (fabsf(si->ns.x) > 0.9999f) ? V(0, 1, 0) : V(1, 0, 0);
    si->tangent = normalize(cross(up, si->ns));
    v3 pa = at_f(r, t);
    si->p = V(pa.x + EPS_SHADOW * nn.x, pa.y + EPS_SHADOW * nn.y, fmaf(nn.z, EPS_SHADOW, pa.z));
    return 1;
}

/* SphereShape::Intersect / IntersectPred (Shape.cpp:3-56) */
static int sphere_root(const pt_sphere* sp, const ray_t* r, float max, float* t_out) {
    v3 oc = sub(r->o, vl(sp->center));
    float a = dot(r->d, r->d);
    float b = dot(oc, r->d);
    /* the reference build's contraction (Shape.cpp:6-8 under GCC -O3 FMA):
     * c = fma(-r, r, oc.oc), disc = fma(b, b, -(a*c)).  The cancellation in
     * disc makes the root sensitive to it at ~10^2 x radius distances. */
    float c = fmaf(-sp->radius, sp->radius, dot(oc, oc));
    float disc = fmaf(b, b, -(a * c));
    if (disc > 0) {
        float temp = (-b - sqrtf(disc)) / a;
        if (temp < max && temp > EPS_SHADOW) { *t_out = temp; return 1; }
        temp = (-b + sqrtf(disc)) / a;
        if (temp < max && temp > EPS_SHADOW) { *t_out = temp; return 1; }
    }
    return 0;
}
static int sphere_intersect(const pt_sphere* sp, const ray_t* r, float max, si_t* si) {
    float t;
    if (!sphere_root(sp, r, max, &t)) return 0;
    si->t = t;
    v3 pa = at_f(r, t);
    si->ns = normalize(sub(pa, vl(sp->center)));
    si->n = si->ns;
    v3 up = (fabsf(si->ns.x) > 0.9999f) ? V(0, 1, 0) : V(1, 0, 0);
    si->tangent = normalize(cross(up, si->ns));
    si->p = V(fmaf(si->n.x, EPS_SHADOW, pa.x), fmaf(si->n.y, EPS_SHADOW, pa.y), fmaf(si->n.z, EPS_SHADOW, pa.z));
    sphere_uv(si->n, si->uv);
    return 1;
}

/* ------------------------------------------------------------------ traversal (BVH.hpp:1019-1211) */
typedef struct { uint32_t nodes, tris; } work_t;

static int prim_intersect(const scene_t* S, uint32_t slot, const ray_t* r, float max, si_t* si, work_t* wk);
static int prim_pred(const scene_t* S, uint32_t slot, const ray_t* r, float max, work_t* wk);

#ifdef ORACLE_WIDE_STATS
/* Diagnostics build only (tools/wide_stats.py): how many BVH4 node visits a
 * wide node that absorbs its children's children (greedily by surface area,
 * up to 8 slots) would save.  A visit of a node its parent absorbed counts in
 * g_wide[0] (closest) / g_wide[1] (any). */
static unsigned long long g_wide[2];
static float child_area(const pt_ref_bvh4_cluster* c, int i) {
    float dx = c->xmax[i] - c->xmin[i], dy = c->ymax[i] - c->ymin[i], dz = c->zmax[i] - c->zmin[i];
    return dx * dy + dy * dz + dz * dx;
}
static int n_valid(const pt_bvh_desc* B, pt_ref_bvh4_node nd) {
    const pt_ref_bvh4_cluster* c = &B->clusters[nd.cluster_idx];
    int v = 0;
    for (int i = 0; i < 4; i++) v += !(c->children[i].active == 0 && c->children[i].count == 0);
    return v;
}
/* bit i set: child i of the cluster is absorbed */
static unsigned absorbed(const pt_bvh_desc* B, const pt_ref_bvh4_cluster* c) {
    int slots = 0, order[4] = {0, 1, 2, 3};
    for (int i = 0; i < 4; i++) slots += !(c->children[i].active == 0 && c->children[i].count == 0);
    for (int a = 0; a < 4; a++)
        for (int b = a + 1; b < 4; b++)
            if (child_area(c, order[b]) > child_area(c, order[a])) { int t = order[a]; order[a] = order[b]; order[b] = t; }
    unsigned m = 0;
    for (int k = 0; k < 4; k++) {
        int i = order[k];
        if (c->children[i].active == 0) continue;
        int v = n_valid(B, c->children[i]);
        if (slots - 1 + v <= 8) { slots += v - 1; m |= 1u << i; }
    }
    return m;
}
void oracle_wide_stats(unsigned long long* out) { out[0] = g_wide[0]; out[1] = g_wide[1]; g_wide[0] = g_wide[1] = 0; }
#endif

/* BVH4::Intersect: ordered closest hit with entry-distance pruning. */
static int bvh_intersect(const scene_t* S, const pt_bvh_desc* B, const ray_t* r, float* max, si_t* si, work_t* wk) {
    const unsigned signs = ((r->d.z < 0) << 2) | ((r->d.y < 0) << 1) | (r->d.x < 0);
    pt_ref_bvh4_node stack[64];
    float entry[64];
#ifdef ORACLE_WIDE_STATS
    unsigned char wflag[64];
    wflag[0] = 0;
#endif
    int sp = 0;
    entry[sp] = 0;
    stack[sp++] = B->root;
    int hit = 0;
    while (sp) {
        if (entry[--sp] > *max) continue;
        pt_ref_bvh4_node nd = stack[sp];
        if (nd.active != 0) {
            const pt_ref_bvh4_cluster* c = &B->clusters[nd.cluster_idx];
            wk->nodes++;
#ifdef ORACLE_WIDE_STATS
            g_wide[0] += wflag[sp];
            const unsigned ab = absorbed(B, c);
#endif
            float te[4];
            unsigned mask = 0;
            for (int i = 0; i < 4; i++) {
                float tx1 = (c->xmin[i] - r->o.x) * r->inv.x, tx2 = (c->xmax[i] - r->o.x) * r->inv.x;
                float ty1 = (c->ymin[i] - r->o.y) * r->inv.y, ty2 = (c->ymax[i] - r->o.y) * r->inv.y;
                float tz1 = (c->zmin[i] - r->o.z) * r->inv.z, tz2 = (c->zmax[i] - r->o.z) * r->inv.z;
                /* _mm_min_ps/_mm_max_ps(a,b): a<b?a:b / a>b?a:b */
                float tminx = tx1 < tx2 ? tx1 : tx2, tmaxx = tx1 > tx2 ? tx1 : tx2;
                float tminy = ty1 < ty2 ? ty1 : ty2, tmaxy = ty1 > ty2 ? ty1 : ty2;
                float tminz = tz1 < tz2 ? tz1 : tz2, tmaxz = tz1 > tz2 ? tz1 : tz2;
                float tminxy = tminx > tminy ? tminx : tminy;
                float tEntry = tminxy > tminz ? tminxy : tminz;
                float tmaxxy = tmaxx < tmaxy ? tmaxx : tmaxy;
                float tExit = tmaxxy < tmaxz ? tmaxxy : tmaxz;
                te[i] = tEntry;
                if (tExit >= EPS_SHADOW && tEntry < *max && tEntry <= tExit) mask |= 1u << i;
            }
            unsigned perm = S->lut[signs][nd.perm];
            /* maskLUT (BVH.hpp:719-738): push far -> near so the nearest pops first */
            for (int nsh = 0; nsh <= 6; nsh += 2) {
                unsigned idx = (perm >> nsh) & 3u;
                if (mask & (1u << idx)) {
                    if (sp >= 64) return hit;
                    entry[sp] = te[idx];
#ifdef ORACLE_WIDE_STATS
                    wflag[sp] = (ab >> idx) & 1u;
#endif
                    stack[sp++] = c->children[idx];
                }
            }
        } else {
            /* intersectPrimitives (BVH.hpp:107-124) */
            uint32_t first = B->prim_base + nd.cluster_idx;
            for (uint32_t i = first; i < first + nd.count; i++) {
                if (prim_intersect(S, i, r, *max, si, wk)) {
                    hit = 1;
                    *max = si->t;
                }
            }
        }
    }
    return hit;
}

static int bvh_pred(const scene_t* S, const pt_bvh_desc* B, const ray_t* r, float max, work_t* wk) {
    pt_ref_bvh4_node stack[64];
#ifdef ORACLE_WIDE_STATS
    unsigned char wflag[64];
    wflag[0] = 0;
#endif
    int sp = 0;
    stack[sp++] = B->root;
    while (sp) {
        pt_ref_bvh4_node nd = stack[--sp];
        if (nd.active != 0) {
            const pt_ref_bvh4_cluster* c = &B->clusters[nd.cluster_idx];
            wk->nodes++;
#ifdef ORACLE_WIDE_STATS
            g_wide[1] += wflag[sp];
            const unsigned ab = absorbed(B, c);
#endif
            for (int i = 0; i < 4; i++) {
                float tx1 = (c->xmin[i] - r->o.x) * r->inv.x, tx2 = (c->xmax[i] - r->o.x) * r->inv.x;
                float ty1 = (c->ymin[i] - r->o.y) * r->inv.y, ty2 = (c->ymax[i] - r->o.y) * r->inv.y;
                float tz1 = (c->zmin[i] - r->o.z) * r->inv.z, tz2 = (c->zmax[i] - r->o.z) * r->inv.z;
                float tminx = tx1 < tx2 ? tx1 : tx2, tmaxx = tx1 > tx2 ? tx1 : tx2;
                float tminy = ty1 < ty2 ? ty1 : ty2, tmaxy = ty1 > ty2 ? ty1 : ty2;
                float tminz = tz1 < tz2 ? tz1 : tz2, tmaxz = tz1 > tz2 ? tz1 : tz2;
                float tminxy = tminx > tminy ? tminx : tminy;
                float tEntry = tminxy > tminz ? tminxy : tminz;
                float tmaxxy = tmaxx < tmaxy ? tmaxx : tmaxy;
                float tExit = tmaxxy < tmaxz ? tmaxxy : tmaxz;
                if (tExit >= EPS_SHADOW && tEntry < max && tEntry <= tExit) {
                    if (sp >= 64) return 0;
#ifdef ORACLE_WIDE_STATS
                    wflag[sp] = (ab >> i) & 1u;
#endif
                    stack[sp++] = c->children[i];
                }
            }
        } else {
            uint32_t first = B->prim_base + nd.cluster_idx;
            for (uint32_t i = first; i < first + nd.count; i++)
                if (prim_pred(S, i, r, max, wk)) return 1;
        }
    }
    return 0;
}

/* ---- TransformedPrimitive (Primitive.cpp:42-72): glm mat4 (column-major
 * m[c*4+r]) times vec4: (m0*x + m1*y) + (m2*z + m3*w), each product rounded
 * (glm/detail/type_mat4x4.inl:561-572; the TLAS fixture confirms the form) */
/* the reference build's contraction (fixture search on the instance traces):
 * a0 = fma(m0, x, m1*y), a1 = fma(m2, z, m3*w), then a0 + a1 */
static inline float m4_a0(float m0, float x, float m1, float y) { return fmaf(m0, x, rmul(m1, y)); }
static inline float m4_a1(float m2, float z, float m3, float w) { return fmaf(m2, z, rmul(m3, w)); }
static v3 m4_point(const float* m, v3 p) {
    float o[3];
    for (int r = 0; r < 3; r++) o[r] = m4_a0(m[r], p.x, m[4 + r], p.y) + m4_a1(m[8 + r], p.z, m[12 + r], 1.0f);
    return V(o[0], o[1], o[2]);
}
static v3 m4_dir(const float* m, v3 v) {
    float o[3];
    for (int r = 0; r < 3; r++) o[r] = m4_a0(m[r], v.x, m[4 + r], v.y) + m4_a1(m[8 + r], v.z, m[12 + r], 0.0f);
    return V(o[0], o[1], o[2]);
}
/* transpose(inverse(mat3(transform))) (glm compute_inverse<3,3>), NM[c*3+r] */
static void normal_matrix(const float* T, float* NM) {
#define M(c, r) T[(c) * 4 + (r)]
#define DF(a, b, c, d) fmaf(a, b, -rmul(c, d)) /* the reference build's contraction */
#define DFN(a, b, c, d) fmaf(-(a), b, rmul(c, d))
    const float D0 = DF(M(1, 1), M(2, 2), M(2, 1), M(1, 2)), D1 = DF(M(0, 1), M(2, 2), M(2, 1), M(0, 2));
    const float D2 = DF(M(0, 1), M(1, 2), M(1, 1), M(0, 2));
    /* as GCC contracts glm's determinant: fma(m20, D2, fma(m00, D0, -(m10*D1))) */
    float od = 1.0f / fmaf(M(2, 0), D2, fmaf(M(0, 0), D0, -rmul(M(1, 0), D1)));
    float inv[3][3];
    inv[0][0] = +DF(M(1, 1), M(2, 2), M(2, 1), M(1, 2)) * od;
    /* the negated cofactors -(a*b - c*d) as the build folds them (.FNMA):
     * -(a*b) + c*d, which is +0, not -0, where a*b == c*d */
    inv[1][0] = DFN(M(1, 0), M(2, 2), M(2, 0), M(1, 2)) * od;
    inv[2][0] = +DF(M(1, 0), M(2, 1), M(2, 0), M(1, 1)) * od;
    inv[0][1] = DFN(M(0, 1), M(2, 2), M(2, 1), M(0, 2)) * od;
    inv[1][1] = +DF(M(0, 0), M(2, 2), M(2, 0), M(0, 2)) * od;
    inv[2][1] = DFN(M(0, 0), M(2, 1), M(2, 0), M(0, 1)) * od;
    inv[0][2] = +DF(M(0, 1), M(1, 2), M(1, 1), M(0, 2)) * od;
    inv[1][2] = DFN(M(0, 0), M(1, 2), M(1, 0), M(0, 2)) * od;
    inv[2][2] = +DF(M(0, 0), M(1, 1), M(1, 0), M(0, 1)) * od;
#undef M
#undef DF
#undef DFN
    for (int c = 0; c < 3; c++)
        for (int r = 0; r < 3; r++) NM[c * 3 + r] = inv[r][c];
}
static inline float m3_row(float a, float x, float b, float y, float c, float z) {
    return fmaf(c, z, fmaf(a, x, rmul(b, y))); /* as the reference build contracts it */
}
static v3 m3_mul(const float* M, v3 v) { /* glm mat3 * vec3 (type_mat3x3.inl:468-474) */
    return V(m3_row(M[0], v.x, M[3], v.y, M[6], v.z), m3_row(M[1], v.x, M[4], v.y, M[7], v.z),
             m3_row(M[2], v.x, M[5], v.y, M[8], v.z));
}
/* glm::normalize(vec4 with w = 0): v * (1 / sqrt((x*x + y*y) + (z*z + w*w))) */
static v3 normalize4(v3 v) {
    const float d = fmaf(v.y, v.y, rmul(v.x, v.x)) + rmul(v.z, v.z); /* fixture search */
    return muls(v, 1.0f / sqrtf(d));
}
/* glm::inverse(mat4) (glm/detail/func_matrix.inl compute_inverse<4,4>) as
 * the reference build (g++ -O3 -march=native) contracts it: the cofactors a
 * fused first product minus a rounded second, each lane a rounded first
 * product with the other two fused in turn, the negated lanes negated after,
 * the determinant's pairs fused once (GCC's GIMPLE of that function; the
 * host's pt_mat4_inverse is the same).  Exported as oracle_mat4_inverse for
 * tests/test_mat4_inverse.py, which checks it against the reference build's
 * own glm. */
static inline float fms_(float a, float b, float c) { return fmaf(a, b, -c); }
static inline float inv_lane(float va, float fa, float vb, float fb, float vc, float fc) {
    return fmaf(vc, fc, fmaf(-vb, fb, rmul(va, fa)));
}
static void mat4_inverse_(const float* mm, float* out) {
    const float m00 = mm[0], m01 = mm[1], m02 = mm[2], m03 = mm[3];
    const float m10 = mm[4], m11 = mm[5], m12 = mm[6], m13 = mm[7];
    const float m20 = mm[8], m21 = mm[9], m22 = mm[10], m23 = mm[11];
    const float m30 = mm[12], m31 = mm[13], m32 = mm[14], m33 = mm[15];
    const float C00 = fms_(m22, m33, rmul(m32, m23)), C02 = fms_(m33, m12, rmul(m32, m13));
    const float C03 = fms_(m23, m12, rmul(m22, m13)), C04 = fms_(m33, m21, rmul(m23, m31));
    const float C06 = fms_(m33, m11, rmul(m13, m31)), C07 = fms_(m23, m11, rmul(m13, m21));
    const float C08 = fms_(m32, m21, rmul(m22, m31)), C10 = fms_(m32, m11, rmul(m12, m31));
    const float C11 = fms_(m22, m11, rmul(m12, m21)), C12 = fms_(m33, m20, rmul(m23, m30));
    const float C14 = fms_(m33, m10, rmul(m13, m30)), C15 = fms_(m23, m10, rmul(m13, m20));
    const float C16 = fms_(m32, m20, rmul(m22, m30)), C18 = fms_(m32, m10, rmul(m12, m30));
    const float C19 = fms_(m22, m10, rmul(m12, m20)), C20 = fms_(m31, m20, rmul(m21, m30));
    const float C22 = fms_(m31, m10, rmul(m11, m30)), C23 = fms_(m21, m10, rmul(m11, m20));
    float I[16];
    I[0] = inv_lane(m11, C00, m12, C04, m13, C08);
    I[1] = -inv_lane(m01, C00, m02, C04, m03, C08);
    I[2] = inv_lane(m01, C02, m02, C06, m03, C10);
    I[3] = -inv_lane(m01, C03, m02, C07, m03, C11);
    I[4] = -inv_lane(m10, C00, m12, C12, m13, C16);
    I[5] = inv_lane(m00, C00, m02, C12, m03, C16);
    I[6] = -inv_lane(m00, C02, m02, C14, m03, C18);
    I[7] = inv_lane(m00, C03, m02, C15, m03, C19);
    I[8] = inv_lane(m10, C04, m11, C12, m13, C20);
    I[9] = -inv_lane(m00, C04, m01, C12, m03, C20);
    I[10] = inv_lane(m00, C06, m01, C14, m03, C22);
    I[11] = -inv_lane(m00, C07, m01, C15, m03, C23);
    I[12] = -inv_lane(m10, C08, m11, C16, m12, C20);
    I[13] = inv_lane(m00, C08, m01, C16, m02, C20);
    I[14] = -inv_lane(m00, C10, m01, C18, m02, C22);
    I[15] = inv_lane(m00, C11, m01, C19, m02, C23);
    const float od = 1.0f / (fmaf(m01, I[4], rmul(m00, I[0])) + fmaf(m03, I[12], rmul(m02, I[8])));
    for (int k = 0; k < 16; k++) out[k] = rmul(I[k], od);
}
void oracle_mat4_inverse(const float* m, float* out) { mat4_inverse_(m, out); }

/* AnimatedPrimitive / AnimatedLight at a ray's time (Primitive.cpp:82-89,
 * Light.cpp:341-356): TransformedPrimitive / TransformedLight over
 * glm::translate(mat4(1), dir * t), t = glm::clamp(time - t0, t0, t1) /
 * (t1 - t0); tmp receives the instance with that transform and its inverse.
 * A static instance is returned as is. */
static const pt_instance* inst_at(const pt_instance* I, float time, pt_instance* tmp) {
    if (!I || !I->animated) return I;
    *tmp = *I;
    const float t0 = I->time_bounds[0], t1 = I->time_bounds[1];
    float x = time - t0;
    x = t0 > x ? t0 : x; /* glm::max (func_common.inl:29) */
    x = t1 < x ? t1 : x; /* glm::min (func_common.inl:20) */
    const float t = x / (t1 - t0);
    float* T = tmp->transform;
    for (int k = 0; k < 16; k++) T[k] = (k % 5 == 0) ? 1.0f : 0.0f;
    /* column 3 = m[0]*v.x + m[1]*v.y + m[2]*v.z + m[3] over the identity:
     * the products are exact, so v, with a zero made +0 by the final add */
    for (int k = 0; k < 3; k++) T[12 + k] = rmul(I->motion[k], t) + 0.0f;
    mat4_inverse_(T, tmp->inv);
    return tmp;
}

static ray_t instance_ray(const pt_instance* I, const ray_t* r, float* len) {
    v3 dir = m4_dir(I->inv, r->d);
    *len = length3(dir);
    return mkray_t(m4_point(I->inv, r->o), divs(dir, *len), r->time);
}

/* TransformedPrimitive::Intersect (Primitive.cpp:48-64) of instance record k:
 * its primitive is the next level down (pt_instance.inner, a nested wrapper)
 * or the BLAS; tmp.prim stays the BLAS slot */
static int inst_intersect(const scene_t* S, int32_t k, const ray_t* r, float max, si_t* si, work_t* wk) {
    pt_instance at_time;
    const pt_instance* I = inst_at(&S->s->instances[k], r->time, &at_time);
    float len;
    ray_t tr = instance_ray(I, r, &len);
    float m = max * len;
    si_t tmp;
    memset(&tmp, 0, sizeof(tmp));
    if (I->inner >= 0) {
        if (!inst_intersect(S, I->inner, &tr, m, &tmp, wk)) return 0;
    } else if (!bvh_intersect(S, &S->s->bvhs[I->bvh], &tr, &m, &tmp, wk)) {
        return 0;
    }
    float NM[9];
    normal_matrix(I->transform, NM);
    *si = tmp;
    si->p = m4_point(I->transform, tmp.p);
    si->n = normalize(m3_mul(NM, tmp.n));
    si->ns = normalize(m3_mul(NM, tmp.ns));
    si->t = tmp.t / len;
    si->tangent = normalize4(m4_dir(I->transform, tmp.tangent));
    return 1;
}
static int inst_pred(const scene_t* S, int32_t k, const ray_t* r, float max, work_t* wk) {
    pt_instance at_time;
    const pt_instance* I = inst_at(&S->s->instances[k], r->time, &at_time);
    float len;
    ray_t tr = instance_ray(I, r, &len);
    if (I->inner >= 0) return inst_pred(S, I->inner, &tr, max * len, wk);
    return bvh_pred(S, &S->s->bvhs[I->bvh], &tr, max * len, wk);
}

/* GeometricPrimitive::Intersect (Primitive.cpp:15-26) / Model::Intersect (Model.hpp:25-27) */
static int prim_intersect(const scene_t* S, uint32_t slot, const ray_t* r, float max, si_t* si, work_t* wk) {
    const pt_prim* p = &S->s->prims[slot];
    if (p->kind == PT_PRIM_BLAS) return bvh_intersect(S, &S->s->bvhs[p->index], r, &max, si, wk);
    if (p->kind == PT_PRIM_INSTANCE) {
        const pt_instance* I = &S->s->instances[p->index];
        if (!inst_intersect(S, (int32_t)p->index, r, max, si, wk)) return 0;
        si->prim = (int)(I->virt_base + ((uint32_t)si->prim - S->s->bvhs[I->bvh].prim_base));
        return 1;
    }
    si_t tmp;
    memset(&tmp, 0, sizeof(tmp));
    int hit;
    wk->tris++;
    if (p->kind == PT_PRIM_TRIANGLE) hit = tri_intersect(S, p->index, p->material, r, max, &tmp);
    else if (p->kind == PT_PRIM_QUAD) hit = quad_intersect(&S->s->quads[p->index], r, max, &tmp);
    else hit = sphere_intersect(&S->s->spheres[p->index], r, max, &tmp);
    if (!hit || (p->material >= 0 && !mat_alpha(S, p->material, tmp.uv, r->o, r->d, (int)slot))) return 0;
    *si = tmp;
    si->light = p->light;
    si->mat = p->material;
    si->medium = p->medium;
    si->prim = (int)slot;
    return 1;
}

/* GeometricPrimitive::IntersectPred (Primitive.cpp:6-14) */
static int prim_pred(const scene_t* S, uint32_t slot, const ray_t* r, float max, work_t* wk) {
    const pt_prim* p = &S->s->prims[slot];
    if (p->kind == PT_PRIM_BLAS) return bvh_pred(S, &S->s->bvhs[p->index], r, max, wk);
    if (p->kind == PT_PRIM_INSTANCE) /* TransformedPrimitive::IntersectPred (Primitive.cpp:42-47) */
        return inst_pred(S, (int32_t)p->index, r, max, wk);
    wk->tris++;
    if (mat_has_alpha(S, p->material)) {
        si_t tmp;
        memset(&tmp, 0, sizeof(tmp));
        int hit;
        if (p->kind == PT_PRIM_TRIANGLE) hit = tri_intersect(S, p->index, p->material, r, max, &tmp);
        else if (p->kind == PT_PRIM_QUAD) hit = quad_intersect(&S->s->quads[p->index], r, max, &tmp);
        else hit = sphere_intersect(&S->s->spheres[p->index], r, max, &tmp);
        return hit && mat_alpha(S, p->material, tmp.uv, r->o, r->d, (int)slot);
    }
    if (p->kind == PT_PRIM_TRIANGLE) return tri_pred(S, p->index, r, max);
    if (p->kind == PT_PRIM_QUAD) {
        float t, a, b;
        v3 nn;
        return quad_hit(&S->s->quads[p->index], r, max, &t, &a, &b, &nn);
    }
    float t;
    return sphere_root(&S->s->spheres[p->index], r, max, &t);
}

static int scene_intersect(const scene_t* S, const ray_t* r, si_t* si, work_t* wk) {
    float max = INFINITY;
    return bvh_intersect(S, &S->s->bvhs[0], r, &max, si, wk);
}
static int scene_pred(const scene_t* S, const ray_t* r, float max, work_t* wk) {
    return bvh_pred(S, &S->s->bvhs[0], r, max, wk);
}

/* ------------------------------------------------------------------ microfacet (Material.hpp:55-142) */
typedef struct { float ax, ay; } dist_t;
static inline dist_t mkdist(float rough) { dist_t d = {rough * rough, rough * rough}; return d; }
static float lambda_(const dist_t* D, v3 w) {
    float cos2 = w.z * w.z;
    if (cos2 == 0) return 0;
    float sin2 = fmaxf_(0, 1 - cos2);
    float sinT = sqrtf(sin2);
    float cosPhi = sinT == 0 ? 1 : clampf(w.x / sinT, -1.0f, 1.0f);
    float sinPhi = sinT == 0 ? 0 : clampf(w.y / sinT, -1.0f, 1.0f);
    /* Material.hpp:66 as built: fma(cosPhi*ax, cosPhi*ax, (sinPhi*ay)^2) */
    float ca = cosPhi * D->ax, sa = sinPhi * D->ay;
    float alpha2 = fmaf(ca, ca, sa * sa);
    return (sqrtf(1.f + alpha2 * sin2 / cos2) - 1.0f) / 2.0f;
}
static float D_(const dist_t* D, v3 wh) {
    float cos2 = wh.z * wh.z;
    if (cos2 == 0) return 0;
    float cos4 = cos2 * cos2;
    float sin2 = fmaxf_(0, 1 - cos2);
    float sinT = sqrtf(sin2);
    float cosPhi = sinT == 0 ? 1 : clampf(wh.x / sinT, -1.0f, 1.0f);
    float sinPhi = sinT == 0 ? 0 : clampf(wh.y / sinT, -1.0f, 1.0f);
    /* Material.hpp:78-79 as built: the sum of squares fused, and 1 + e fused
     * into one fma(sin2/cos2, sum, 1) (e itself is never rounded) */
    float cx = cosPhi / D->ax, sy = sinPhi / D->ay;
    float e1 = fmaf(sin2 / cos2, fmaf(cx, cx, sy * sy), 1.0f);
    float denom = PI_F * D->ax * D->ay * cos4 * e1 * e1;
    if (denom <= 0) return INFINITY;
    return 1 / denom;
}
static inline float G1_(const dist_t* D, v3 w) { return 1 / (1 + lambda_(D, w)); }
static inline float G_(const dist_t* D, v3 wo, v3 wi) { return 1 / (1 + lambda_(D, wo) + lambda_(D, wi)); }
static inline int smooth_(const dist_t* D) { return fmaxf_(D->ax, D->ay) < 1e-6; }
/* MicrofacetDistribution::PDF with the caller's dot(wo, wh) (its order differs by call site) */
static inline float mpdf_(const dist_t* D, v3 wo, v3 wh, float dwh) { return D_(D, wh) * G1_(D, wo) * fabsf(dwh / wo.z); }
/* sampleGGXVNDF (Material.hpp:119-139) with the contractions of the
 * reference build (MicrofacetDiffuse::scatter's inlined copy) */
static v3 vndf_(float ax, float ay, v3 Ve, float U1, float U2, int ne_inline) {
    v3 Vh = normalize(V(ax * Ve.x, ay * Ve.y, Ve.z));
    float lensq = fmaf(Vh.x, Vh.x, Vh.y * Vh.y);
    v3 T1 = lensq > 0 ? muls(V(-Vh.y, Vh.x, 0), 1.0f / sqrtf(lensq)) : V(1, 0, 0);
    v3 T2 = cross_v(Vh, T1);
    float r = sqrtf(U1);
    float phi = 2.0f * PI_F * U2;
    float t1 = r * cosf(phi);
    float t2 = r * sinf(phi);
    float s = 0.5f * (1.0f + Vh.z);
    float q1 = fmaf(-t1, t1, 1.0f); /* 1 - t1*t1 */
    t2 = fmaf(1.0f - s, sqrtf(q1), s * t2);
    float q = fmaf(-t2, t2, q1);
    float sq = sqrtf(fmaxf_(0.0f, q));
    /* x, y lanes: t2*T2 rounded, t1*T1 fused; z lane: t1*T1 rounded, t2*T2 fused */
    v3 Nh = V(fmaf(sq, Vh.x, fmaf(t1, T1.x, t2 * T2.x)), fmaf(sq, Vh.y, fmaf(t1, T1.y, t2 * T2.y)),
              fmaf(sq, Vh.z, fmaf(t2, T2.z, t1 * T1.z)));
    v3 ne = V(ax * Nh.x, ay * Nh.y, fmaxf_(0.0f, Nh.z));
    if (!ne_inline) return normalize(ne);
    /* MicrofacetDielectric::scatter's inlined copy: z^2 added unfused */
    float zz = Nh.z > 0 ? ne.z * ne.z : 0.0f;
    return muls(ne, 1.0f / sqrtf(fmaf(ne.y, ne.y, ne.x * ne.x) + zz));
}
static v3 sample_wh(const dist_t* D, v3 wo, float u0, float u1, int ne_inline) {
    int flip = wo.z < 0;
    v3 wh = vndf_(D->ax, D->ay, flip ? neg(wo) : wo, u0, u1, ne_inline);
    if (flip) wh = neg(wh);
    return wh;
}
static float fresnel_dielectric(float cosi, float eta) {
    /* Material.hpp:11-28 (T = float) */
    cosi = clampf(cosi, -1.0f, 1.0f);
    if (cosi < 0) {
        eta = 1 / eta;
        cosi = -cosi;
    }
    /* as built: 1 - cos^2, eta*cos -+ cost, cos -+ eta*cost and the sum of squares fused */
    float sin2i = fmaf(-cosi, cosi, 1.0f);
    float sin2t = sin2i / (eta * eta);
    if (sin2t >= 1) return 1.f;
    float cost = sqrtf(1 - sin2t);
    float rpa = fmaf(cosi, eta, -cost) / fmaf(cosi, eta, cost);
    float rpe = fmaf(-eta, cost, cosi) / fmaf(eta, cost, cosi);
    return fmaf(rpa, rpa, rpe * rpe) * 0.5f;
}
static inline v3 schlick(float c, v3 F0) {
#ifdef ORACLE_POW_CR
    float p = (float)pow((double)(1.0f - c), 5.0);
#else
    float p = powf(1.0f - c, 5.0f);
#endif
    /* F0 + (1 - F0) * p, fused */
    return V(fmaf(p, 1.0f - F0.x, F0.x), fmaf(p, 1.0f - F0.y, F0.y), fmaf(p, 1.0f - F0.z, F0.z));
}

/* ------------------------------------------------------------------ materials */
typedef struct { v3 f; float pdf; uint32_t flags; v3 o, d; int ok; } bxdf_t;
#define FL_TRANS 1u
#define FL_SPEC 2u

/* onb TBN(dot(d, ns) > 0 ? -ns : ns) and wo = TBN.toLocal(-d) as MicrofacetDiffuse's
 * three entry points are built: the sign test is the unfused dot, and wo.z reuses it
 * (+-dot(d, ns)) instead of dot(-d, n) */
static inline v3 diffuse_frame(v3 d, v3 ns, onb_t* tbn) {
    float pd = dot_p(d, ns);
    *tbn = onb_n(pd > 0 ? neg(ns) : ns);
    v3 md = neg(d);
    return V(dot(md, tbn->a0), dot(md, tbn->a1), pd > 0 ? pd : -pd);
}
static float diffuse_rough(const scene_t* S, const pt_material* m, const si_t* si) {
    return fmaxf_(tex_eval(S, m->rough, si->uv).y, 0.0001f);
}

/* MicrofacetDiffuse::scatter (Material.hpp:206-266) */
static bxdf_t diffuse_scatter(const scene_t* S, const pt_material* m, const ray_t* in, const si_t* si, float u,
                              float uv0, float uv1) {
    bxdf_t b;
    memset(&b, 0, sizeof(b));
    float rough = diffuse_rough(S, m, si);
    float prob = rough >= 0.7 ? 1.0f : 0.5f;
    dist_t D = mkdist(rough);
    onb_t tbn;
    v3 wo = diffuse_frame(in->d, si->ns, &tbn);
    v3 wi, wh;
    if (u >= prob) {
        wh = sample_wh(&D, wo, uv0, uv1, 0);
        wi = reflect(neg(wo), wh);
    } else {
        float z = sqrtf(1.0f - uv1);
        float phi = 2.0f * PI_F * uv0;
        float s2 = sqrtf(uv1);
        float x = cosf(phi) * s2;
        float y = sinf(phi) * s2;
        wi = V(x, y, z);
        wh = normalize(add(wo, wi));
    }
    if (wi.z <= 0) return b;
    /* as built: dot(wo, wh) in y, x, z order; prob*wi.z*inv_pi + spdf fused */
    float spdf = (1.0f - prob) * mpdf_(&D, wo, wh, dot_yxz(wo, wh)) / (4 * fabsf(dot_yxz(wo, wh)));
    float pdf = fmaf(prob * wi.z, INV_PI_F, spdf);
    v3 col = tex_eval(S, m->tex, si->uv);
    float metal = tex_eval(S, m->metal, si->uv).z;
    /* glm::mix(0.04, col, metal) as built here: col*metal rounded, the other fused */
    float om = 1.0f - metal;
    v3 F0 = V(fmaf(om, 0.04f, col.x * metal), fmaf(om, 0.04f, col.y * metal), fmaf(om, 0.04f, col.z * metal));
    v3 F = schlick(dot_yxz(wi, wh), F0);
    v3 num = muls(F, D_(&D, wh) * G_(&D, wo, wi));
    float den = fabsf(4.0f * wo.z * wi.z);
    if (den == 0) return b;
    v3 spec = divs(num, den);
    v3 kD = muls(sub(V(1, 1, 1), F), om);
    v3 kc = mul(kD, col);
    b.f = V(fmaf(kc.x, INV_PI_F, spec.x), fmaf(kc.y, INV_PI_F, spec.y), fmaf(kc.z, INV_PI_F, spec.z));
    b.pdf = pdf;
    b.flags = 0;
    b.o = si->p;
    b.d = to_world(&tbn, wi);
    b.ok = 1;
    return b;
}
static v3 diffuse_f(const scene_t* S, const pt_material* m, const ray_t* in, const si_t* si, v3 dir) {
    /* calc_attenuation (Material.hpp:299-326) */
    onb_t tbn;
    v3 wo = diffuse_frame(in->d, si->ns, &tbn);
    v3 wi = to_local(&tbn, dir);
    v3 wh = normalize(add(wo, wi));
    float rough = diffuse_rough(S, m, si);
    float metal = tex_eval(S, m->metal, si->uv).z;
    dist_t D = mkdist(rough);
    v3 col = tex_eval(S, m->tex, si->uv);
    /* glm::mix as built here: (1-metal)*0.04 rounded, col*metal fused */
    float om = 1.0f - metal, c4 = om * 0.04f;
    v3 F0 = V(fmaf(col.x, metal, c4), fmaf(col.y, metal, c4), fmaf(col.z, metal, c4));
    v3 F = schlick(dot_yxz(wi, wh), F0);
    v3 num = muls(F, D_(&D, wh) * G_(&D, wo, wi));
    float den = fabsf(4.0f * wo.z * wi.z);
    if (den == 0) return V(0, 0, 0);
    v3 spec = divs(num, den);
    v3 kc = mul(muls(sub(V(1, 1, 1), F), om), col);
    return V(fmaf(kc.x, INV_PI_F, spec.x), fmaf(kc.y, INV_PI_F, spec.y), fmaf(kc.z, INV_PI_F, spec.z));
}
static float diffuse_pdf(const scene_t* S, const pt_material* m, const ray_t* in, const si_t* si, v3 dir) {
    /* MicrofacetDiffuse::PDF (Material.hpp:281-296): no (1-prob) factor (A.7) */
    float rough = diffuse_rough(S, m, si);
    dist_t D = mkdist(rough);
    onb_t tbn;
    v3 wo = diffuse_frame(in->d, si->ns, &tbn);
    v3 wh = to_local(&tbn, normalize(sub(dir, in->d)));
    float prob = rough >= 0.7 ? 1.0f : 0.5f;
    float diff = prob * fabsf(dot(si->ns, dir)) * INV_PI_F;
    float spec = mpdf_(&D, wo, wh, dot(wo, wh)) / (4 * fabsf(dot(wo, wh)));
    return diff + spec;
}

/* MicrofacetDielectric::scatter (Material.hpp:392-477), contractions as built */
static bxdf_t dielectric_scatter(const scene_t* S, const pt_material* m, const ray_t* in, const si_t* si, float u,
                                 float uv0, float uv1) {
    bxdf_t b;
    memset(&b, 0, sizeof(b));
    float rough = tex_eval(S, m->rough, si->uv).y;
    dist_t D = mkdist(rough);
    onb_t tbn = onb_si(si);
    v3 md = neg(in->d);
    v3 wo = to_local_ool(&tbn, md);
    float ri = m->ri;
    float eta = dot_p(md, si->ns) > 0 ? 1 / ri : ri;
    v3 eps_n;
    if (ri == 1 || smooth_(&D)) {
        v3 N = dot_p(in->d, si->ns) > 0 ? neg(si->ns) : si->ns;
        v3 Ng = dot(in->d, si->n) > 0 ? neg(si->n) : si->n;
        float F = fresnel_dielectric(wo.z, ri);
        float R = F, T = 1.0f - R;
        v3 dir, p = at_f(in, si->t);
        eps_n = V(EPS_SHADOW * Ng.x, EPS_SHADOW * Ng.y, 0);
        if (u < (R / (R + T))) {
            dir = to_world(&tbn, V(-wo.x, -wo.y, wo.z));
            b.o = V(p.x + eps_n.x, p.y + eps_n.y, fmaf(Ng.z, EPS_SHADOW, p.z));
            b.f = divs(muls(tex_eval(S, m->tex, si->uv), R), fabsf(dot(si->ns, dir)));
            b.pdf = R / (R + T);
        } else {
            dir = refract_f(in->d, N, eta, dot(in->d, N));
            if (is_zero(dir)) return b;
            b.o = V(p.x - eps_n.x, p.y - eps_n.y, fmaf(-Ng.z, EPS_SHADOW, p.z));
            b.f = divs(muls(tex_eval(S, m->tex, si->uv), T), fabsf(dot(si->ns, dir)));
            b.pdf = T / (R + T);
        }
        b.d = dir;
        b.flags = FL_TRANS | FL_SPEC;
        b.ok = 1;
        return b;
    }
    v3 wh = sample_wh(&D, wo, uv0, uv1, 1);
    v3 Ng = dot(in->d, si->n) > 0 ? neg(si->n) : si->n;
    float dow = dot_p(wo, wh); /* dot(wo, wh), unfused, shared by every use below */
    float F = fresnel_dielectric(dow, 1 / eta);
    float R = F, T = 1 - R;
    v3 wi, p = at_f(in, si->t);
    eps_n = V(EPS_SHADOW * Ng.x, EPS_SHADOW * Ng.y, 0);
    uint32_t fl = FL_TRANS | (rough < 0.001f ? FL_SPEC : 0u);
    if (u < (R / (R + T))) {
        float d = -dow;
        wi = sub(neg(wo), muls(muls(wh, d), 2.0f));
        if (wo.z * wi.z < 0) return b;
        b.o = V(p.x + eps_n.x, p.y + eps_n.y, fmaf(Ng.z, EPS_SHADOW, p.z));
        b.d = to_world(&tbn, wi);
        b.pdf = mpdf_(&D, wo, wh, dot(wo, wh)) / (fabsf(dow) * 4) * R / (R + T);
        b.f = divs(muls(muls(muls(tex_eval(S, m->tex, si->uv), D_(&D, wh)), G_(&D, wo, wi)), R), fabsf(4 * wi.z * wo.z));
    } else {
        wi = refract_f(neg(wo), wh, eta, -dow);
        if (wo.z * wi.z > 0 || wi.z == 0) return b;
        b.o = V(p.x - eps_n.x, p.y - eps_n.y, fmaf(-Ng.z, EPS_SHADOW, p.z));
        b.d = to_world(&tbn, wi);
        float diw = dot(wi, wh);
        float dn = fmaf(eta, dow, diw);
        float denom = dn * dn;
        float dwh = fabsf(diw) / denom;
        b.pdf = mpdf_(&D, wo, wh, dot(wo, wh)) * dwh * T / (R + T);
        float ft = T * D_(&D, wh) * G_(&D, wo, wi) * fabsf(diw * dow / (denom * wi.z * wo.z));
        b.f = muls(tex_eval(S, m->tex, si->uv), ft);
    }
    b.flags = fl;
    b.ok = 1;
    return b;
}
/* MicrofacetDielectric::PDF / calc_attenuation (Material.hpp:484-564); each
 * builds its own half vector: wi*etap + wo unfused in PDF, x and y lanes fused
 * in calc_attenuation (and normalised out of line there) */
static int dielectric_frame(const scene_t* S, const pt_material* m, const ray_t* in, const si_t* si, v3 dir,
                            int for_f, dist_t* D, v3* wo, v3* wi, v3* wh, float* etap, int* refl) {
    float rough = tex_eval(S, m->rough, si->uv).y;
    *D = mkdist(rough);
    float ri = m->ri;
    if (ri == 1 || smooth_(D)) return 0;
    onb_t tbn = onb_si(si);
    *wo = to_local_ool(&tbn, neg(in->d));
    *wi = to_local_ool(&tbn, dir);
    float co = wo->z, ci = wi->z;
    *refl = ci * co > 0;
    *etap = 1;
    if (!*refl) *etap = co > 0 ? ri : (1 / ri);
    v3 h;
    if (for_f && !*refl)
        h = V(fmaf(wi->x, *etap, wo->x), fmaf(wi->y, *etap, wo->y), co + ci * *etap);
    else
        h = add(muls(*wi, *etap), *wo);
    if (dot(h, h) == 0) return 0;
    h = normalize(h);
    if (h.z < 0) h = neg(h);
    *wh = h;
    if (dot(h, *wi) * ci <= 0.0 || dot(h, *wo) * co <= 0.0) return 0;
    return 1;
}
static void dielectric_eval(const scene_t* S, const pt_material* m, const ray_t* in, const si_t* si, v3 dir,
                            v3* f_out, float* pdf_out) {
    *f_out = V(0, 0, 0);
    *pdf_out = 0;
    dist_t D;
    v3 wo, wi, wh;
    float etap;
    int refl;
    if (dielectric_frame(S, m, in, si, dir, 0, &D, &wo, &wi, &wh, &etap, &refl)) {
        float dow = dot(wh, wo), diw = dot(wh, wi);
        float F = fresnel_dielectric(dow, m->ri);
        float R = F, T = 1 - R;
        float pdf = mpdf_(&D, wo, wh, dow);
        if (refl) {
            *pdf_out = pdf / (fabsf(dow) * 4) * R / (R + T);
        } else {
            float dn = dow / etap + diw;
            float dwh = fabsf(diw) / (dn * dn);
            *pdf_out = dwh * pdf * T / (R + T);
        }
    }
    if (dielectric_frame(S, m, in, si, dir, 1, &D, &wo, &wi, &wh, &etap, &refl)) {
        float dow = dot(wh, wo), diw = dot(wh, wi);
        float F = fresnel_dielectric(dow, m->ri);
        v3 col = tex_eval(S, m->tex, si->uv);
        if (refl) {
            *f_out = divs(muls(muls(muls(col, D_(&D, wh)), G_(&D, wo, wi)), F), fabsf(4 * wi.z * wo.z));
        } else {
            float dn = dow / etap + diw;
            float den2 = dn * dn * wi.z * wo.z;
            float ft = (1 - F) * D_(&D, wh) * G_(&D, wo, wi) * fabsf(diw * dow / den2);
            *f_out = muls(col, ft);
        }
    }
}

/* ThinDielectric::scatter (Material.hpp:605-644) */
static bxdf_t thin_scatter(const scene_t* S, const pt_material* m, const ray_t* in, const si_t* si, float u) {
    bxdf_t b;
    memset(&b, 0, sizeof(b));
    /* as built: onb(si)'s cross with the first product rounded in every lane,
     * wo.x and wo.y in y, x, z order */
    onb_t tbn;
    tbn.a2 = si->ns;
    tbn.a0 = si->tangent;
    tbn.a1 = cross_r(tbn.a2, tbn.a0);
    v3 md = neg(in->d);
    v3 wo = V(dot_yxz(md, tbn.a0), dot_yxz(md, tbn.a1), dot(md, tbn.a2));
    v3 Ng = dot(in->d, si->n) > 0 ? neg(si->n) : si->n;
    float F = fresnel_dielectric(wo.z, m->ri);
    float R = F, T = 1.0f - R;
    if (R < 1.0f) {
        R += T * T * R / fmaf(-R, R, 1.0f);
        T = 1.0f - R;
    }
    v3 dir, f;
    if (u < (R / (R + T))) {
        dir = to_world(&tbn, V(-wo.x, -wo.y, wo.z));
        b.o = add(smul(EPS_SHADOW, Ng), at_f(in, si->t));
        f = divs(muls(V(1, 1, 1), R), fabsf(dot(si->ns, dir)));
        b.pdf = R / (R + T);
    } else {
        dir = in->d;
        b.o = sub(at_f(in, si->t), smul(EPS_SHADOW, Ng));
        f = divs(muls(V(1, 1, 1), T), fabsf(dot(si->ns, dir)));
        b.pdf = T / (R + T);
    }
    b.f = mul(f, tex_eval(S, m->tex, si->uv));
    b.d = dir;
    b.flags = FL_TRANS | FL_SPEC;
    b.ok = 1;
    return b;
}

/* SpecularConductor::scatter (Material.hpp:664-669) */
static bxdf_t conductor_scatter(const pt_material* m, const ray_t* in, const si_t* si) {
    bxdf_t b;
    memset(&b, 0, sizeof(b));
    v3 d = reflect(in->d, si->ns);
    float dt = dot(d, si->ns);
    if (dt <= 0) return b;
    b.f = divs(schlick(dot(si->ns, neg(in->d)), vl(m->albedo)), dt);
    b.pdf = 1;
    b.flags = FL_SPEC;
    b.o = si->p;
    b.d = d;
    b.ok = 1;
    return b;
}

static bxdf_t mat_scatter(const scene_t* S, int mid, const ray_t* in, const si_t* si, float u, float uv0, float uv1) {
    const pt_material* m = &S->s->materials[mid];
    switch (m->kind) {
        case PT_MAT_DIFFUSE: return diffuse_scatter(S, m, in, si, u, uv0, uv1);
        case PT_MAT_DIELECTRIC: return dielectric_scatter(S, m, in, si, u, uv0, uv1);
        case PT_MAT_THIN: return thin_scatter(S, m, in, si, u);
        default: return conductor_scatter(m, in, si);
    }
}
static v3 mat_f(const scene_t* S, int mid, const ray_t* in, const si_t* si, v3 dir) {
    const pt_material* m = &S->s->materials[mid];
    v3 f;
    float p;
    switch (m->kind) {
        case PT_MAT_DIFFUSE: return diffuse_f(S, m, in, si, dir);
        case PT_MAT_DIELECTRIC: dielectric_eval(S, m, in, si, dir, &f, &p); return f;
        case PT_MAT_THIN: return V(0, 0, 0);
        default: return V(1, 1, 1); /* base Material::calc_attenuation */
    }
}
static float mat_pdf(const scene_t* S, int mid, const ray_t* in, const si_t* si, v3 dir) {
    const pt_material* m = &S->s->materials[mid];
    v3 f;
    float p;
    switch (m->kind) {
        case PT_MAT_DIFFUSE: return diffuse_pdf(S, m, in, si, dir);
        case PT_MAT_DIELECTRIC: dielectric_eval(S, m, in, si, dir, &f, &p); return p;
        default: return 0;
    }
}

/* ------------------------------------------------------------------ lights (Light.cpp) */
typedef struct { v3 L; si_t si; v3 dir; } lsample_t;

static float shape_area(const scene_t* S, const pt_prim* p) {
    if (p->kind == PT_PRIM_QUAD) {
        const pt_quad* q = &S->s->quads[p->index];
        return length3(cross(vl(q->u), vl(q->v)));
    }
    if (p->kind == PT_PRIM_SPHERE) {
        float r = S->s->spheres[p->index].radius;
        return 4.0f * PI_F * r * r;
    }
    tri_t T = tri_get(S, p->index);
    return length3(cross(sub(T.v0, T.v2), sub(T.v1, T.v2))) * 0.5f;
}

static si_t shape_sample(const scene_t* S, const pt_prim* p, float u0, float u1) {
    si_t si;
    memset(&si, 0, sizeof(si));
    if (p->kind == PT_PRIM_QUAD) {
        const pt_quad* q = &S->s->quads[p->index];
        v3 Q = vl(q->Q), qu = vl(q->u), qv = vl(q->v); /* Q + u0*u + u1*v, both fused */
        si.p = V(fmaf(qv.x, u1, fmaf(qu.x, u0, Q.x)), fmaf(qv.y, u1, fmaf(qu.y, u0, Q.y)),
                 fmaf(qv.z, u1, fmaf(qu.z, u0, Q.z)));
        si.n = vl(q->normal);
    } else if (p->kind == PT_PRIM_SPHERE) {
        const pt_sphere* sp = &S->s->spheres[p->index];
        float z = 1.0f - 2.0f * u0;
        float r = sqrtf(fmaf(-z, z, 1.0f));
        float phi = 2.0f * PI_F * u1;
        v3 d = V(r * cosf(phi), r * sinf(phi), z);
        v3 c = vl(sp->center);
        si.p = V(fmaf(sp->radius, d.x, c.x), fmaf(sp->radius, d.y, c.y), fmaf(sp->radius, d.z, c.z));
        si.n = normalize(sub(si.p, c));
        sphere_uv(si.p, si.uv);
    } else {
        /* TriangleShape::Sample (Shape.cpp:277-297): not folded (A.6) */
        float w = 1.0f - u0 - u1;
        tri_t T = tri_get(S, p->index);
        v3 n = normalize(cross(sub(T.v1, T.v0), sub(T.v2, T.v0)));
        if (n.x != n.x) n = V(0, 0, 0);
        si.p = V(lerp3f(u0, T.v1.x, u1, T.v2.x, w, T.v0.x), lerp3f(u0, T.v1.y, u1, T.v2.y, w, T.v0.y),
                 lerp3f(u0, T.v1.z, u1, T.v2.z, w, T.v0.z));
        const float* uvs = S->s->uvs;
        si.uv[0] = lerp3f(u0, uvs[2 * T.i1], u1, uvs[2 * T.i2], w, uvs[2 * T.i0]);
        si.uv[1] = lerp3f(u0, uvs[2 * T.i1 + 1], u1, uvs[2 * T.i2 + 1], w, uvs[2 * T.i0 + 1]);
        si.n = n;
    }
    return si;
}
/* Shape::PDF(interaction, ray) as built: dot(to, to) in y, x, z order; the
 * quad's (inlined into AreaLight::PDF) light cosine also in y, x, z order,
 * except behind the one-sided test, whose dot(-d, n) it reuses */
static float shape_pdf(const scene_t* S, const pt_prim* p, const si_t* si, const ray_t* r, int one_sided) {
    v3 to = sub(si->p, r->o);
    float d2 = dot_yxz(to, to);
    float lc = fabsf(p->kind == PT_PRIM_QUAD && !one_sided ? dot_yxz(neg(r->d), si->n) : dot(neg(r->d), si->n));
    float area = shape_area(S, p);
    if (p->kind == PT_PRIM_QUAD) {
        if (area == 0) return 0;
    } else if (p->kind == PT_PRIM_SPHERE) {
        if (area * lc == 0) return 0;
    } else {
        if (area == 0 || lc == 0 || si->n.x != si->n.x) return 0;
    }
    return d2 / (lc * area);
}
static v3 sky_le(const pt_light* l, v3 d) {
    /* (1-a)*c0 rounded, a*c1 fused (fixture search) */
    float a = 0.5f * (d.y + 1.0f), b = 1.0f - a;
    return smul(l->scale, V(fmaf(a, l->vec[0], rmul(b, l->color[0])), fmaf(a, l->vec[1], rmul(b, l->color[1])),
                            fmaf(a, l->vec[2], rmul(b, l->color[2]))));
}
/* TextureInfiniteLight (Light.cpp:110-150): Le = LeScale * tex(GetSphereUV(dir)) */
static v3 texinf_le(const scene_t* S, const pt_light* l, v3 d) {
    float uv[2];
    sphere_uv(d, uv);
    return smul(l->scale, tex_eval(S, l->tex, uv));
}
static v3 inf_le_s(const scene_t* S, const pt_light* l, v3 d) {
    if (l->kind == PT_LIGHT_TEX_INF) return texinf_le(S, l, d);
    return l->kind == PT_LIGHT_SKY_INF ? sky_le(l, d) : vl(l->color);
}
#define inf_le(l, d) inf_le_s(S, l, d)
static float texinf_pdf(const scene_t* S, const pt_light* l, v3 rd) {
    v3 le = texinf_le(S, l, rd);
    double lum = fma((double)le.z, 0.0722, fma((double)le.y, 0.7152, (double)le.x * 0.2126));
    double tot = (double)S->s->light_dist[(size_t)l->prim + (size_t)PT_TEXINF_X * PT_TEXINF_Y - 1];
    const float cell_omega = 4.0f * PI_F / (float)(PT_TEXINF_X * PT_TEXINF_Y);
    return (float)((lum / tot) * (double)(1.0f / cell_omega));
}
/* Light::PDF({}, ray) of an infinite light */
static float inf_pdf(const scene_t* S, const pt_light* l, v3 rd) {
    return l->kind == PT_LIGHT_TEX_INF ? texinf_pdf(S, l, rd) : 1.0f / (4.0f * PI_F);
}
/* the hidden random_float() of TextureInfiniteLight::sample (Light.cpp:120),
 * drawn outside the stream's numbered dimensions (pt_shading.h texinf_uc) */
static float texinf_uc(const rng_t* r) {
    return (float)(pcg_hash((r->key ^ 0xC3115EEDu) + 0x9E3779B9u * r->dim) >> 8) * (1.0f / 16777216.0f);
}

/* TransformedLight / AnimatedLight (Light.cpp:300-364): the inner
 * AreaLight's shape in the instance's object space.  A nested wrapper's
 * light is a TransformedLight of a TransformedLight: lv receives the levels
 * at the time, the outermost first (tmp holds their storage); returns the
 * count, 0 for a light outside any instance */
static int light_levels(const scene_t* S, const pt_light* l, float time, pt_instance* tmp, const pt_instance** lv) {
    if (l->kind != PT_LIGHT_AREA || l->instance < 0) return 0;
    int k = 0;
    for (int32_t i = l->instance; i >= 0 && k < PT_MAX_INSTANCE_DEPTH; i = S->s->instances[i].inner, k++)
        lv[k] = inst_at(&S->s->instances[i], time, &tmp[k]);
    return k;
}
/* Light::sample(uv, time) (Light.hpp:21): the time moves an AnimatedLight */
static lsample_t light_sample(const scene_t* S, const pt_light* l, float u0, float u1, float uc, float time) {
    lsample_t ls;
    memset(&ls, 0, sizeof(ls));
    if (l->kind == PT_LIGHT_TEX_INF) { /* TextureInfiniteLight::sample (Light.cpp:118-144) */
        const float* acc = S->s->light_dist + l->prim;
        const uint32_t N = (uint32_t)PT_TEXINF_X * PT_TEXINF_Y;
        /* float weight = random_float() * totalWeight (double product, rounded) */
        float weight = (float)((double)uc * (double)acc[N - 1]);
        uint32_t i = 0, hi = N; /* std::upper_bound: first running sum > weight */
        while (i < hi) {
            uint32_t mid = (i + hi) >> 1;
            if (acc[mid] > weight) hi = mid;
            else i = mid + 1;
        }
        int cx = (int)(i % PT_TEXINF_Y), cy = (int)(i / PT_TEXINF_Y);
        float cu = ((float)cx + u0) / (float)PT_TEXINF_X, cv = ((float)cy + u1) / (float)PT_TEXINF_Y;
        float z = 2.0f * cu - 1.0f;
        float th = 2.0f * PI_F * cv;
        float r = sqrtf(1.0f - rmul(z, z));
        ls.dir = V(r * cosf(th), r * sinf(th), z);
        sphere_uv(ls.dir, ls.si.uv);
        return ls;
    }
    if (l->kind == PT_LIGHT_AREA) {
        ls.si = shape_sample(S, &S->s->prims[l->prim], u0, u1);
        pt_instance tmp[PT_MAX_INSTANCE_DEPTH];
        const pt_instance* lv[PT_MAX_INSTANCE_DEPTH];
        /* TransformedLight::sample: p by the transform, n by the normal
         * matrix, of the inner light's sample (the innermost level first) */
        for (int k = light_levels(S, l, time, tmp, lv) - 1; k >= 0; k--) {
            float NM[9];
            normal_matrix(lv[k]->transform, NM);
            ls.si.p = m4_point(lv[k]->transform, ls.si.p);
            ls.si.n = m3_mul(NM, ls.si.n);
        }
        return ls;
    }
    if (l->kind == PT_LIGHT_POINT) {
        ls.L = vl(l->color);
        ls.si.p = vl(l->vec);
        ls.si.n = V(1, 1, 1);
        ls.si.uv[0] = u0;
        ls.si.uv[1] = u1;
        return ls;
    }
    /* Distant / Uniform / Function light sample (Light.cpp:36-41, 62-67, 209-214):
     * 1 - z*z fused except in FunctionInfiniteLight::sample, which also adds
     * z*z unfused in its GetSphereUV normalisation */
    const int sky = l->kind == PT_LIGHT_SKY_INF;
    float z = 2.0f * u0 - 1.0f;
    float th = 2.0f * PI_F * u1;
    float r = sky ? sqrtf(1.0f - z * z) : sqrtf(fmaf(-z, z, 1.0f));
    float x = cosf(th) * r, y = sinf(th) * r;
    v3 d = V(x, y, z);
    if (l->kind == PT_LIGHT_DISTANT) {
        ls.L = vl(l->color);
        ls.si.uv[0] = u0;
        ls.si.uv[1] = u1;
        v3 vv = vl(l->vec);
        ls.dir = normalize(V(fmaf(d.x, 0.02f, vv.x), fmaf(d.y, 0.02f, vv.y), fmaf(d.z, 0.02f, vv.z)));
        return ls;
    }
    ls.L = inf_le(l, d);
    if (sky)
        sphere_uv_n(muls(d, 1.0f / sqrtf(fmaf(y, y, x * x) + z * z)), ls.si.uv);
    else
        sphere_uv(d, ls.si.uv);
    ls.dir = d;
    return ls;
}
static inline int light_is_delta(const pt_light* l) { return l->kind == PT_LIGHT_DISTANT || l->kind == PT_LIGHT_POINT; }
static float light_pdf(const scene_t* S, const pt_light* l, const si_t* si, const ray_t* r) {
    if (l->kind == PT_LIGHT_AREA) {
        const pt_prim* p = &S->s->prims[l->prim];
        pt_instance tmp[PT_MAX_INSTANCE_DEPTH];
        const pt_instance* lv[PT_MAX_INSTANCE_DEPTH];
        const int nl = light_levels(S, l, r->time, tmp, lv);
        if (nl) { /* TransformedLight::PDF: point, normal and ray to object space, the outermost level first */
            si_t lo = *si;
            ray_t lr = *r;
            for (int k = 0; k < nl; k++) {
                const float* inv = lv[k]->inv;
                lo.p = m4_point(inv, lo.p);
                lo.n = normalize(m4_dir(inv, lo.n));
                lr.o = m4_point(inv, lr.o);
                lr.d = normalize(m4_dir(inv, lr.d));
            }
            if (l->one_sided) return dot(neg(lr.d), lo.n) > 0 ? shape_pdf(S, p, &lo, &lr, 1) : 0;
            return shape_pdf(S, p, &lo, &lr, 0);
        }
        if (l->one_sided) return dot(neg(r->d), si->n) > 0 ? shape_pdf(S, p, si, r, 1) : 0;
        return shape_pdf(S, p, si, r, 0);
    }
    if (l->kind == PT_LIGHT_UNIFORM_INF || l->kind == PT_LIGHT_SKY_INF) return 1.0f / (4.0f * PI_F);
    if (l->kind == PT_LIGHT_TEX_INF) return texinf_pdf(S, l, r->d);
    return 0;
}
static v3 light_L(const scene_t* S, const pt_light* l, const si_t* si, const ray_t* r) {
    if (l->kind == PT_LIGHT_AREA) {
        pt_instance tmp[PT_MAX_INSTANCE_DEPTH];
        const pt_instance* lv[PT_MAX_INSTANCE_DEPTH];
        const int nl = light_levels(S, l, r->time, tmp, lv);
        if (nl) { /* TransformedLight::L: a fresh interaction, n by the normal matrix
                   * (the outermost level first), uv (0, 0) */
            v3 n = si->n;
            for (int k = 0; k < nl; k++) {
                float NM[9];
                normal_matrix(lv[k]->transform, NM);
                n = m3_mul(NM, n);
            }
            const float uv0[2] = {0, 0};
            if (l->one_sided && dot(r->d, n) > 0) return V(0, 0, 0);
            return tex_eval(S, l->tex, uv0);
        }
        if (l->one_sided && dot(r->d, si->n) > 0) return V(0, 0, 0);
        return tex_eval(S, l->tex, si->uv);
    }
    if (l->kind == PT_LIGHT_UNIFORM_INF || l->kind == PT_LIGHT_SKY_INF || l->kind == PT_LIGHT_TEX_INF)
        return inf_le(l, r->d);
    return V(0, 0, 0);
}

/* LightSampler::Sample (LightSampler.cpp:7-11, 34-46) */
static int ls_sample(const scene_t* S, float u) {
    uint32_t n = S->s->n_sampler_lights;
    if (n == 0) return -1;
    if (S->s->light_sampler == PT_LS_UNIFORM) {
        int idx = (int)(u * n);
        if (idx > (int)n - 1) idx = (int)n - 1;
        return (int)S->s->sampler_lights[idx];
    }
    float total = 0;
    for (uint32_t i = 0; i < n; i++) total += S->s->lights[S->s->sampler_lights[i]].power;
    float cur = 0, target = u * total;
    for (uint32_t i = 0; i < n; i++) {
        cur += S->s->lights[S->s->sampler_lights[i]].power;
        if (cur >= target) return (int)S->s->sampler_lights[i];
    }
    return (int)S->s->sampler_lights[n - 1];
}

/* ------------------------------------------------------------------ integrators (Integrators.cpp) */
typedef struct {
    const scene_t* S;
    uint32_t max_depth;
    int simple;
    oracle_counters* cnt;
    uint32_t kind; /* PT_INTEGRATOR_* */
    uint32_t strata_x, strata_y; /* a StratifiedSampler host's camera strata (0: none) */
} integ_t;

/* PathIntegrator::SampleLd (Integrators.cpp:260-294) */
static v3 sample_ld(const integ_t* I, const ray_t* ray, const si_t* si, float u, float uv0, float uv1, float uc) {
    const scene_t* S = I->S;
    int li = ls_sample(S, u);
    if (li < 0) return V(0, 0, 0);
    const pt_light* l = &S->s->lights[li];
    lsample_t ls = light_sample(S, l, uv0, uv1, uc, ray->time);
    v3 ldir;
    float t;
    if (is_zero(ls.si.n)) {
        ldir = ls.dir;
        t = INFINITY;
    } else {
        ldir = sub(ls.si.p, si->p);
        t = length3(ldir) - EPS_SHADOW;
    }
    ray_t sh = mkray_t(si->p, normalize(ldir), ray->time);
    float lpdf = l->pmf;
    float dt = dot_yxz(si->ns, sh.d); /* as built: y, x, z order */
    if (lpdf <= 0 || dt * dot(ray->d, si->ns) >= 0) return V(0, 0, 0);
    work_t wk = {0, 0};
    I->cnt->any++;
    int occ = scene_pred(S, &sh, t, &wk);
    I->cnt->nodes_any += wk.nodes;
    I->cnt->tris_any += wk.tris;
    if (occ) return V(0, 0, 0);
    v3 f = muls(mat_f(S, si->mat, ray, si, sh.d), fabsf(dt));
    if (light_is_delta(l)) return divs(mul(ls.L, f), lpdf);
    lpdf *= light_pdf(S, l, &ls.si, &sh);
    if (lpdf <= 0) return V(0, 0, 0);
    float w2 = lpdf * lpdf;
    float w1 = mat_pdf(S, si->mat, ray, si, sh.d);
    float wl = w2 / fmaf(w1, w1, w2); /* w1*w1 + w2 fused */
    return divs(muls(mul(light_L(S, l, &ls.si, &sh), f), wl), lpdf);
}

static int intersect_counted(const integ_t* I, const ray_t* r, si_t* si) {
    work_t wk = {0, 0};
    I->cnt->closest++;
    int h = scene_intersect(I->S, r, si, &wk);
    I->cnt->nodes_closest += wk.nodes;
    I->cnt->tris_closest += wk.tris;
    if (h) I->cnt->hits++;
    return h;
}

/* debugging aid: ORACLE_DEBUG_KEY=<stream key> prints that path's bounces */
static uint32_t dbg_key(void) {
    static int init = 0;
    static uint32_t k = 0;
    if (!init) {
        const char* e = getenv("ORACLE_DEBUG_KEY");
        k = e ? (uint32_t)strtoul(e, NULL, 0) : 0;
        init = 1;
    }
    return k;
}
#define DBG(...) do { if (dbgon) fprintf(stderr, __VA_ARGS__); } while (0)

/* PathIntegrator::Li (Integrators.cpp:182-257) */
static v3 li_path(const integ_t* I, ray_t ray, rng_t* rng) {
    const int dbgon = dbg_key() != 0 && rng->key == dbg_key();
    const scene_t* S = I->S;
    v3 att = V(1, 1, 1), out = V(0, 0, 0);
    uint32_t depth = 0, rr = 0;
    float prev = 1;
    int spec = 1;
    while (depth++ < I->max_depth && (att.x + att.y + att.z) > 0.0f) {
        si_t si;
        memset(&si, 0, sizeof(si));
        if (!intersect_counted(I, &ray, &si)) {
            DBG("O d%u miss\n", depth);
            for (uint32_t k = 0; k < S->s->n_infinite_lights; k++) {
                const pt_light* l = &S->s->lights[S->s->infinite_lights[k]];
                /* as built: out += att*Le fused; the MIS weight's lp*lp + p*p
                 * and out += (att*Le)*w fused */
                if (spec) {
                    out = fma3(inf_le(l, ray.d), att, out);
                } else if (prev > 0) {
                    float lp = l->pmf * inf_pdf(S, l, ray.d);
                    float p2 = prev * prev;
                    float w = p2 / fmaf(lp, lp, p2);
                    out = fma3s(w, mul(inf_le(l, ray.d), att), out);
                }
            }
            return out;
        }
        float r[8];
        for (int k = 0; k < 8; k++) r[k] = next1(rng);
        DBG("O d%u prim %d t %a p %a %a %a ns %a %a %a uv %a %a mat %d light %d out %a %a %a att %a %a %a\n", depth,
            si.prim, si.t, si.p.x, si.p.y, si.p.z, si.ns.x, si.ns.y, si.ns.z, si.uv[0], si.uv[1], si.mat, si.light,
            out.x, out.y, out.z, att.x, att.y, att.z);
        if (si.light >= 0) {
            const pt_light* al = &S->s->lights[si.light];
            v3 L = light_L(S, al, &si, &ray);
            if (!is_zero(L)) {
                if (spec) {
                    out = fma3(L, att, out);
                } else if (prev > 0) {
                    float lp = al->pmf * light_pdf(S, al, &si, &ray);
                    float p2 = prev * prev;
                    float w = p2 / fmaf(lp, lp, p2);
                    out = fma3s(w, mul(L, att), out);
                }
            }
        }
        if (si.mat < 0) {
            spec = 1;
            ray.o = at_f(&ray, si.t);
            continue;
        }
        bxdf_t b = mat_scatter(S, si.mat, &ray, &si, r[4], r[0], r[1]);
        if (!b.ok) return out;
        ray_t nr = mkray_t(b.o, b.d, ray.time); /* scatter: Ray(..., incoming.time) */
        spec = (b.flags & FL_SPEC) != 0;
        if (!spec) {
            v3 ld = sample_ld(I, &ray, &si, r[5], r[2], r[3], texinf_uc(rng));
            DBG("O  ld %a %a %a (light %d)\n", ld.x, ld.y, ld.z, ls_sample(S, r[5]));
            out = fma3(ld, att, out);
            prev = mat_pdf(S, si.mat, &ray, &si, nr.d);
        }
        DBG("O  scatter d %a %a %a f %a %a %a pdf %a prev %a\n", b.d.x, b.d.y, b.d.z, b.f.x, b.f.y, b.f.z, b.pdf, prev);
        att = mul(att, divs(muls(b.f, fabsf(dot(si.ns, nr.d))), b.pdf));
        if (rr++ > 3) {
            float q = fminf(0.95f, fmaxf(fmaxf(att.x, att.y), att.z));
            if (r[6] >= q) break;
            att = divs(att, q);
        }
        ray = nr;
    }
    return out;
}

/* SimplePathIntegrator::Li (Integrators.cpp:131-180) */
static v3 li_simple(const integ_t* I, ray_t ray, rng_t* rng) {
    const scene_t* S = I->S;
    v3 att = V(1, 1, 1), out = V(0, 0, 0);
    uint32_t depth = 0, rr = 0;
    while (depth++ < I->max_depth && (att.x + att.y + att.z) > 0.0f) {
        si_t si;
        memset(&si, 0, sizeof(si));
        if (!intersect_counted(I, &ray, &si)) {
            for (uint32_t k = 0; k < S->s->n_infinite_lights; k++) {
                const pt_light* l = &S->s->lights[S->s->infinite_lights[k]];
                out = fma3(inf_le(l, ray.d), att, out);
            }
            return out;
        }
        float u0 = next1(rng), u1 = next1(rng);
        float us = next1(rng);
        float ur = next1(rng);
        if (si.light >= 0) {
            v3 L = light_L(S, &S->s->lights[si.light], &si, &ray);
            if (!is_zero(L)) out = fma3(L, att, out);
        }
        if (si.mat < 0) {
            ray.o = at_f(&ray, si.t);
            continue;
        }
        bxdf_t b = mat_scatter(S, si.mat, &ray, &si, us, u0, u1);
        if (!b.ok) return out;
        ray_t nr = mkray_t(b.o, b.d, ray.time); /* scatter: Ray(..., incoming.time) */
        att = mul(att, divs(muls(b.f, fabsf(dot(si.ns, nr.d))), b.pdf));
        if (rr++ > 3) {
            float q = fminf(0.95f, fmaxf(fmaxf(att.x, att.y), att.z));
            if (ur >= q) break;
            att = divs(att, q);
        }
        ray = nr;
    }
    return out;
}

/* ------------------------------------------------------------------ media (Medium.hpp, PhaseFunction.*) */
/* phaseHG (PhaseFunction.hpp:4-8) */
static float phase_hg(float cosT, float g) {
    /* phaseHG (PhaseFunction.hpp:5-8) as built: 1 + g*g, + 2g*cos and 1 - g*g fused */
    float denom = fmaf(cosT, 2.0f * g, fmaf(g, g, 1.0f));
    return fmaf(-g, g, 1.0f) * (0.25f * (1.0f / PI_F)) / (denom * sqrtf(denom));
}
/* HenyeyGreenstein::Sample (PhaseFunction.cpp:8-25): direction, returns pdf */
static v3 phase_sample(float g, v3 in, float u0, float u1) {
    float cosT;
    if (fabs(g) < 1e-3) {
        cosT = 1 - 2 * u0;
    } else {
        float sqr = fmaf(-g, g, 1.0f) / fmaf(2.0f * g, u0, 1 - g);
        cosT = fmaf(-sqr, sqr, fmaf(g, g, 1.0f)) / (2 * g);
    }
    float q = fmaf(-cosT, cosT, 1.0f);
    float sinT = q > 0 ? sqrtf(q) : 0.0f;
    float phi = 2 * PI_F * u1;
    float x = cosf(phi) * sinT, y = sinf(phi) * sinT, z = cosT;
    /* onb(in).toWorld as built here: a0 = cross(a1, a2) with the x, y lanes
     * rounded-first; x, y lanes (x*a0 fused onto y*a1) + z*a2 unfused, z lane
     * the usual chain */
    onb_t b;
    b.a2 = in;
    v3 up = (fabsf(in.x) > 0.9999) ? V(0, 1, 0) : V(1, 0, 0);
    b.a1 = normalize(cross(b.a2, up));
    b.a0 = cross_v(b.a1, b.a2);
    v3 w = V(fmaf(b.a0.x, x, y * b.a1.x) + z * b.a2.x, fmaf(b.a0.y, x, y * b.a1.y) + z * b.a2.y,
             fmaf(z, b.a2.z, fmaf(y, b.a1.z, x * b.a0.z)));
    return normalize(w);
}
/* HomogeneusMedium::Tr (Medium.hpp:21-24) */
static v3 medium_tr(const pt_medium* m, float t) {
    float tt = t < 3.402823466e38f ? t : 3.402823466e38f;
    return V(expf(-m->sigma_t[0] * tt), expf(-m->sigma_t[1] * tt), expf(-m->sigma_t[2] * tt));
}
/* HomogeneusMedium::Sample (Medium.hpp:26-45) with its two draws from the
 * stream (channel, then distance); *scat receives the scatter point. */
static v3 medium_sample(const pt_medium* m, const ray_t* r, float t, float u0, float u1, int* sampled, v3* scat) {
    int ch = (int)(0.0f + 3.0f * u0);
    float sd = (float)(-log(1.0 - (double)u1) / (double)m->sigma_t[ch]);
    if (!(sd < t)) sd = t; /* std::min<float>(sd, t) */
    *sampled = sd < t;
    if (*sampled) *scat = V(fmaf(sd, r->d.x, r->o.x), fmaf(sd, r->d.y, r->o.y), fmaf(sd, r->d.z, r->o.z));
    v3 tr = medium_tr(m, sd);
    float pdf;
    if (*sampled) /* the sum of sigma_t*tr with the products fused */
        pdf = fmaf(m->sigma_t[2], tr.z, fmaf(m->sigma_t[1], tr.y, tr.x * m->sigma_t[0]));
    else
        pdf = ((0.0f + tr.x) + tr.y) + tr.z;
    pdf = (float)((double)pdf / 3.0);
    return *sampled ? divs(mul(tr, vl(m->sigma_s)), pdf) : divs(tr, pdf);
}
/* GeometricInteraction::getMedium (Interaction.hpp:26-29) */
static inline int get_medium(const si_t* si, v3 dir) { return dot(dir, si->n) < 0 ? si->medium : -1; }

/* Scene::IntersectTr (Scene.cpp:8-29): returns 1 if a surface with a material
 * blocks the segment; *Tr = transmittance through the media crossed. */
static int intersect_tr(const integ_t* I, ray_t ray, int med, float max, v3* Tr) {
    const scene_t* S = I->S;
    *Tr = V(1, 1, 1);
    while (max > 0) {
        si_t si;
        memset(&si, 0, sizeof(si));
        work_t wk = {0, 0};
        I->cnt->any++;
        float m = max;
        int hit = bvh_intersect(S, &S->s->bvhs[0], &ray, &m, &si, &wk);
        I->cnt->nodes_any += wk.nodes;
        I->cnt->tris_any += wk.tris;
        if (!hit) {
            if (med >= 0) *Tr = mul(*Tr, medium_tr(&S->s->media[med], max));
            return 0;
        }
        if (med >= 0) *Tr = mul(*Tr, medium_tr(&S->s->media[med], si.t));
        if (si.mat >= 0) return 1;
        ray = mkray_t(at_f(&ray, si.t), ray.d, ray.time); /* Scene.cpp:25 */
        med = get_medium(&si, ray.d);
        max -= si.t;
    }
    return 0;
}

/* VolPathIntegrator::SampleLd (Integrators.cpp:416-479); phase_g >= -1 marks a
 * medium interaction (p = si->p, f = phase pdf) */
static v3 sample_ld_vol(const integ_t* I, const ray_t* ray, int ray_med, const si_t* si, int medium_it, float g,
                        float u, float uv0, float uv1, float uc) {
    const scene_t* S = I->S;
    int li = ls_sample(S, u);
    if (li < 0) return V(0, 0, 0);
    const pt_light* l = &S->s->lights[li];
    lsample_t ls = light_sample(S, l, uv0, uv1, uc, ray->time);
    v3 ldir;
    float t;
    if (is_zero(ls.si.n)) {
        ldir = ls.dir;
        t = INFINITY;
    } else {
        ldir = sub(ls.si.p, si->p);
        t = length3(ldir) - EPS_SHADOW;
        t -= EPS_SHADOW;
    }
    ray_t sh = mkray_t(si->p, normalize(ldir), ray->time);
    float lpdf = l->pmf;
    if (lpdf <= 0) return V(0, 0, 0);
    v3 f;
    float spdf;
    if (medium_it) {
        spdf = phase_hg(dot(ray->d, sh.d), g);
        f = V(spdf, spdf, spdf);
    } else {
        float dt = dot(si->ns, sh.d);
        if (dt * dot(ray->d, si->ns) >= 0) return V(0, 0, 0);
        spdf = mat_pdf(S, si->mat, ray, si, sh.d);
        f = muls(mat_f(S, si->mat, ray, si, sh.d), fabsf(dt));
    }
    v3 Tr;
    if (is_zero(f) || intersect_tr(I, sh, ray_med, t, &Tr)) return V(0, 0, 0);
    if (light_is_delta(l)) return divs(mul(mul(Tr, ls.L), f), lpdf);
    lpdf *= light_pdf(S, l, &ls.si, &sh);
    if (lpdf <= 0) return V(0, 0, 0);
    float w2 = lpdf * lpdf;
    float wl = w2 / fmaf(spdf, spdf, w2);
    return divs(muls(mul(mul(Tr, light_L(S, l, &ls.si, &sh)), f), wl), lpdf);
}

/* VolPathIntegrator::Li (Integrators.cpp:296-413) */
static v3 li_volpath(const integ_t* I, ray_t ray, int med, rng_t* rng) {
    const scene_t* S = I->S;
    v3 att = V(1, 1, 1), out = V(0, 0, 0);
    uint32_t depth = 0, rr = 0;
    float prev = 1;
    int spec = 1;
    while (depth++ < I->max_depth && (att.x + att.y + att.z) > 0.0f) {
        si_t si;
        memset(&si, 0, sizeof(si));
        if (!intersect_counted(I, &ray, &si)) {
            for (uint32_t k = 0; k < S->s->n_infinite_lights; k++) {
                const pt_light* l = &S->s->lights[S->s->infinite_lights[k]];
                if (spec) {
                    out = fma3(inf_le(l, ray.d), att, out);
                } else if (prev > 0) {
                    float lp = l->pmf * inf_pdf(S, l, ray.d);
                    float p2 = prev * prev;
                    float w = p2 / fmaf(lp, lp, p2);
                    out = fma3s(w, mul(inf_le(l, ray.d), att), out);
                }
            }
            return out;
        }
        if (med < 0) med = S->s->scene_medium;
        int mvalid = 0;
        v3 mp = V(0, 0, 0);
        if (med >= 0) {
            float u0 = next1(rng), u1 = next1(rng);
            att = mul(att, medium_sample(&S->s->media[med], &ray, si.t, u0, u1, &mvalid, &mp));
        }
        float r[9];
        for (int k = 0; k < 9; k++) r[k] = next1(rng);
        if (mvalid) {
            const pt_medium* M = &S->s->media[med];
            si_t mi;
            memset(&mi, 0, sizeof(mi));
            mi.p = mp;
            out = fma3(att, sample_ld_vol(I, &ray, med, &mi, 1, M->g, r[5], r[2], r[3], texinf_uc(rng)), out);
            out = fma3(att, vl(M->Le), out);
            v3 sc = phase_sample(M->g, ray.d, r[6], r[7]);
            int nm = get_medium(&si, sc);
            ray = mkray_t(mp, sc, ray.time); /* Integrators.cpp:314, 361 */
            med = nm;
            spec = 0;
        } else {
            if (si.light >= 0) {
                const pt_light* al = &S->s->lights[si.light];
                v3 L = light_L(S, al, &si, &ray);
                if (!is_zero(L)) {
                    if (spec) {
                        out = fma3(att, L, out);
                    } else if (prev > 0) {
                        float lp = al->pmf * light_pdf(S, al, &si, &ray);
                        float p2 = prev * prev;
                        float w = p2 / fmaf(lp, lp, p2);
                        out = fma3s(w, mul(att, L), out);
                    }
                }
            }
            spec = 0;
            if (si.mat < 0) {
                ray.o = at_f(&ray, si.t);
                med = get_medium(&si, ray.d);
                continue;
            }
            bxdf_t b = mat_scatter(S, si.mat, &ray, &si, r[4], r[0], r[1]);
            if (!b.ok) return out;
            ray_t nr = mkray_t(b.o, b.d, ray.time); /* scatter: Ray(..., incoming.time) */
            int nm = get_medium(&si, nr.d);
            if (!(b.flags & FL_TRANS) && dot(ray.d, si.ns) <= 0) nm = med;
            spec = (b.flags & FL_SPEC) != 0;
            if (!spec) {
                out = fma3(att, sample_ld_vol(I, &ray, med, &si, 0, 0.0f, r[5], r[2], r[3], texinf_uc(rng)), out);
                prev = mat_pdf(S, si.mat, &ray, &si, nr.d);
            }
            att = mul(att, divs(muls(b.f, fabsf(dot(si.ns, nr.d))), b.pdf));
            ray = nr;
            med = nm;
        }
        if (rr++ > 3) {
            float q = fminf(0.95f, fmaxf(fmaxf(att.x, att.y), att.z));
            if (r[8] >= q) break;
            att = divs(att, q);
        }
    }
    return out;
}

/* StratifiedSampler's camera draws (Sampler.hpp:73-151) on Render's
 * per-thread clone (Integrators.cpp:39, 61-64): the stratum of sample index i
 * of the pixel in dimension d is PermutationElement(i, spp, Hash(px, py, d))
 * (Util.hpp:45-73) with Hash = MurmurHash64A over the 16 bytes {px, py, d}
 * (Util.hpp:75-168), jittered by the stream's draw of that dimension (the
 * reference's random_float()). */
static uint64_t murmur_pxd(uint32_t px, uint32_t py, uint64_t d) {
    const uint64_t m = 0xc6a4a7935bd1e995ull;
    uint64_t h = 0 ^ (16ull * m);
    const uint64_t ks[2] = {(uint64_t)px | ((uint64_t)py << 32), d};
    for (int j = 0; j < 2; j++) {
        uint64_t k = ks[j];
        k *= m;
        k ^= k >> 47;
        k *= m;
        h ^= k;
        h *= m;
    }
    h ^= h >> 47;
    h *= m;
    h ^= h >> 47;
    return h;
}
static uint32_t permutation_element(uint32_t i, uint32_t l, uint32_t p) {
    uint32_t w = l - 1;
    w |= w >> 1;
    w |= w >> 2;
    w |= w >> 4;
    w |= w >> 8;
    w |= w >> 16;
    do {
        i ^= p;
        i *= 0xe170893du;
        i ^= p >> 16;
        i ^= (i & w) >> 4;
        i ^= p >> 8;
        i *= 0x0929eb3fu;
        i ^= p >> 23;
        i ^= (i & w) >> 1;
        i *= 1u | p >> 27;
        i *= 0x6935fa69u;
        i ^= (i & w) >> 11;
        i *= 0x74dcb303u;
        i ^= (i & w) >> 2;
        i *= 0x9e501cc3u;
        i ^= (i & w) >> 2;
        i *= 0xc860a3dfu;
        i &= w;
        i ^= i >> 5;
    } while (i >= l);
    return (i + p) % l;
}
static uint32_t stratum_of(uint32_t x, uint32_t y, uint32_t d, uint32_t idx, uint32_t spp) {
    return permutation_element(idx, spp, (uint32_t)murmur_pxd(x, y, d));
}

/* Camera::GenerateRay (Camera.hpp:21-35) + camera draws (Integrators.cpp:61-64);
 * strata_x > 0: a StratifiedSampler(strata_x, strata_y) host, sample index idx
 * of the pixel's round */
static ray_t camera_ray(const pt_camera_desc* c, uint32_t x, uint32_t y, rng_t* rng, double* px, double* py,
                        uint32_t strata_x, uint32_t strata_y, uint32_t idx) {
    float ja = next1(rng), jb = next1(rng);
    float tu = next1(rng); /* time */
    float l0 = next1(rng), l1 = next1(rng);
    if (strata_x) {
        const uint32_t spp = strata_x * strata_y;
        /* getPixel2D = get2D at dimension 0: (sx + dx) / double(xSamples), in double */
        uint32_t st = stratum_of(x, y, 0, idx, spp);
        const double fx = ((int)(st % strata_x) + (double)ja) / (double)strata_x;
        const double fy = ((int)(st / strata_x) + (double)jb) / (double)strata_y;
        /* get1D at dimension 2: (stratum + random_float()) / spp, in float */
        st = stratum_of(x, y, 2, idx, spp);
        tu = ((float)st + tu) / (float)spp;
        /* get2D at dimension 3, handed to GenerateRay as a glm::vec2 */
        st = stratum_of(x, y, 3, idx, spp);
        l0 = (float)(((int)(st % strata_x) + (double)l0) / (double)strata_x);
        l1 = (float)(((int)(st / strata_x) + (double)l1) / (double)strata_y);
        *px = (double)x + fx;
        *py = (double)y + fy;
    } else {
        *px = (double)x + (double)ja;
        *py = (double)y + (double)jb;
    }
    /* t = glm::mix(shutterStart, shutterEnd, time) (Camera.hpp:25) as the
     * reference build contracts it: fma(start, 1 - time, time * end); 0 for
     * the cameras without a shutter (their bounds are uninitialised, A.14) */
    const float tm = c->has_shutter ? fmaf(c->shutter[0], 1.0f - tu, rmul(tu, c->shutter[1])) : 0.0f;
    float pxf = (float)*px, pyf = (float)*py;
    float uc = pxf / (float)c->width;
    float vc = pyf / (float)c->height;
    /* fma(b, v, fma(a, u, -w)) as the reference build contracts it (fixture search) */
    float a = (2.0f * uc - 1.0f) * c->half_width, b = (2.0f * vc - 1.0f) * c->half_height;
    v3 dir = normalize(V(fmaf(b, c->v[0], fmaf(a, c->u[0], -c->w[0])), fmaf(b, c->v[1], fmaf(a, c->u[1], -c->w[1])),
                         fmaf(b, c->v[2], fmaf(a, c->u[2], -c->w[2]))));
    if (c->focus_distance == 0 || c->focus_angle == 0) return mkray_t(vl(c->origin), dir, tm);
    float r = sqrtf(l0);
    float th = 2 * PI_F * l1;
    float lx = r * cosf(th), ly = r * sinf(th);
    v3 du = smul(c->defocus_radius, vl(c->u));
    v3 dv = smul(c->defocus_radius, vl(c->v));
    dir = muls(dir, c->focus_distance);
    /* offset = pLens.x*du + pLens.y*dv with the second product fused (as built) */
    v3 off = V(fmaf(dv.x, ly, du.x * lx), fmaf(dv.y, ly, du.y * lx), fmaf(dv.z, ly, du.z * lx));
    return mkray_t(add(off, vl(c->origin)), normalize(sub(dir, off)), tm);
}

static void scene_init(scene_t* S, const pt_scene_desc* s) {
    S->s = s;
    build_lut(S->lut);
}

static v3 li_one(const integ_t* I, const pt_camera_desc* cam, uint32_t seed, uint32_t x, uint32_t y, uint32_t s,
                 double* px, double* py) {
    rng_t rng;
    rng.key = stream_key(seed, y * (uint32_t)cam->width + x, s);
    rng.dim = 0;
    ray_t r = camera_ray(cam, x, y, &rng, px, py, I->strata_x, I->strata_y,
                         I->strata_x ? s % (I->strata_x * I->strata_y) : 0u);
    I->cnt->paths++;
    tl_tex_bytes = 0;
    v3 L;
    if (I->kind == PT_INTEGRATOR_VOLPATH) L = li_volpath(I, r, cam->medium, &rng);
    else L = I->simple ? li_simple(I, r, &rng) : li_path(I, r, &rng);
    I->cnt->tex_bytes += tl_tex_bytes;
    return L;
}

int oracle_li(const pt_scene_desc* s, const pt_camera_desc* cam, const pt_render_desc* rd, uint32_t pb, uint32_t pe,
              float* out_L, double* out_p, oracle_counters* cnt) {
    if (!s || !cam || !rd || !out_L) return -1;
    scene_t S;
    scene_init(&S, s);
    oracle_counters local;
    memset(&local, 0, sizeof(local));
    integ_t I = {&S, rd->max_depth, rd->integrator == PT_INTEGRATOR_SIMPLE, cnt ? cnt : &local, rd->integrator,
                 rd->strata[0], rd->strata[1]};
    size_t k = 0;
    for (uint32_t pix = pb; pix < pe; pix++) {
        uint32_t x = pix % (uint32_t)cam->width, y = pix / (uint32_t)cam->width;
        for (uint32_t smp = 0; smp < rd->spp; smp++, k++) {
            double px, py;
            v3 L = li_one(&I, cam, rd->seed, x, y, smp, &px, &py);
            out_L[3 * k] = L.x;
            out_L[3 * k + 1] = L.y;
            out_L[3 * k + 2] = L.z;
            if (out_p) {
                out_p[2 * k] = px;
                out_p[2 * k + 1] = py;
            }
        }
    }
    return 0;
}

/* Li of n (pixel, sample) pairs, sample = the frame's global sample index
 * (the same li_one as oracle_li; Integrators.cpp:131-257 per sample).  The
 * checker of pt_frame_samples: the exact frame bench.py times. */
int oracle_li_pairs(const pt_scene_desc* s, const pt_camera_desc* cam, const pt_render_desc* rd,
                    const uint32_t* pix, const uint32_t* smp, uint32_t n, float* out_L, oracle_counters* cnt) {
    if (!s || !cam || !rd || (n && (!pix || !smp || !out_L))) return -1;
    scene_t S;
    scene_init(&S, s);
    oracle_counters local;
    memset(&local, 0, sizeof(local));
    integ_t I = {&S, rd->max_depth, rd->integrator == PT_INTEGRATOR_SIMPLE, cnt ? cnt : &local, rd->integrator,
                 rd->strata[0], rd->strata[1]};
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t x = pix[i] % (uint32_t)cam->width, y = pix[i] / (uint32_t)cam->width;
        double px, py;
        v3 L = li_one(&I, cam, rd->seed, x, y, smp[i], &px, &py);
        out_L[3 * i] = L.x;
        out_L[3 * i + 1] = L.y;
        out_L[3 * i + 2] = L.z;
    }
    return 0;
}

int oracle_trace(const pt_scene_desc* s, const pt_ray* rays, uint32_t n, int any_hit, oracle_hit* out) {
    scene_t S;
    scene_init(&S, s);
    for (uint32_t i = 0; i < n; i++) {
        ray_t r = mkray_t(vl(rays[i].o), vl(rays[i].d), rays[i].time);
        oracle_hit* h = &out[i];
        memset(h, 0, sizeof(*h));
        h->prim = h->material = h->light = -1;
        work_t wk = {0, 0};
        if (any_hit) {
            h->hit = scene_pred(&S, &r, rays[i].tmax, &wk);
        } else {
            si_t si;
            memset(&si, 0, sizeof(si));
            si.prim = si.mat = si.light = -1;
            float max = rays[i].tmax;
            h->hit = bvh_intersect(&S, &s->bvhs[0], &r, &max, &si, &wk);
            if (h->hit) {
                h->t = si.t;
                memcpy(h->p, &si.p, 12);
                memcpy(h->n, &si.n, 12);
                memcpy(h->ns, &si.ns, 12);
                memcpy(h->tangent, &si.tangent, 12);
                h->uv[0] = si.uv[0];
                h->uv[1] = si.uv[1];
                h->prim = si.prim;
                h->material = si.mat;
                h->light = si.light;
                h->medium = si.medium;
            }
        }
        h->nodes = wk.nodes;
        h->tris = wk.tris;
    }
    return 0;
}

/* ------------------------------------------------------------------ film (Film.hpp:65-82, Filter.hpp) */
static double mitchell1(double x, double b, double c) {
    double ax = fabs(x);
    if (ax <= 1.0) return 1.0 / 6.0 * ((12 - 9 * b - 6 * c) * ax * ax * ax + (-18 + 12 * b + 6 * c) * ax * ax + (6 - 2 * b));
    if (ax <= 2) return 1.0 / 6.0 * ((-b - 6 * c) * ax * ax * ax + (6 * b + 30 * c) * ax * ax + (-12 * b - 48 * c) * ax + (8 * b + 24 * c));
    return 0;
}
static double gauss1(double x, double sigma) {
    return 0.56418958354775628695 / (sigma * 1.41421356237309504880) * exp(-(x * x) / (2 * sigma * sigma));
}
/* Sinc / WindowedSinc (Filter.hpp:17-27): LanczosFilter::Evaluate (Filter.hpp:124-126) */
static double sinc1(double x) {
    if (1.0 - x * x == 1.0) return 1.0;
    return sin(3.14159265358979323846 * x) / (3.14159265358979323846 * x);
}
static double wsinc1(double x, double radius, double tau) {
    if (fabs(x) > radius) return 0.0;
    return sinc1(x) * sinc1(x / tau);
}
static double filter_eval(const pt_render_desc* rd, float px, float py) {
    if (rd->filter == PT_FILTER_BOX) return fabsf(px) <= rd->filter_radius[0] && fabsf(py) <= rd->filter_radius[1];
    if (rd->filter == PT_FILTER_LANCZOS)
        return wsinc1(px, rd->filter_radius[0], rd->filter_params[0]) *
               wsinc1(py, rd->filter_radius[1], rd->filter_params[0]);
    if (rd->filter == PT_FILTER_GAUSSIAN) {
        double sg = rd->filter_params[0];
        double X = gauss1(rd->filter_radius[0], sg), Y = gauss1(rd->filter_radius[1], sg);
        double gx = gauss1(px, sg) - X, gy = gauss1(py, sg) - Y;
        return (gx > 0 ? gx : 0) * (gy > 0 ? gy : 0);
    }
    float ax = 2 * px / rd->filter_radius[0];
    float ay = 2 * py / rd->filter_radius[1];
    return mitchell1(ax, rd->filter_params[0], rd->filter_params[1]) *
           mitchell1(ay, rd->filter_params[0], rd->filter_params[1]);
}
static double filter_integral(const pt_render_desc* rd) {
    float rx = rd->filter_radius[0], ry = rd->filter_radius[1];
    if (rd->filter == PT_FILTER_BOX) return 4 * rx * ry;
    if (rd->filter == PT_FILTER_LANCZOS) return rd->filter_params[1]; /* the host object's Integral() */
    if (rd->filter == PT_FILTER_GAUSSIAN) {
        double sg = rd->filter_params[0];
        double X = gauss1(rx, sg), Y = gauss1(ry, sg);
        double s2 = sg * 1.41421356237309504880;
        double ix = 0.5 * (erf(rx / s2) - erf(-rx / s2));
        double iy = 0.5 * (erf(ry / s2) - erf(-ry / s2));
        return (ix - 2 * rx * X) * (iy - 2 * ry * Y);
    }
    return rx * ry / 4.0;
}

int oracle_filter_table(const pt_render_desc* rd, double* out) {
    int k = 0;
    for (int j = 0; j <= 32; j++)
        for (int i = 0; i <= 32; i++) {
            float px = -2.0f + 4.0f * i / 32.0f, py = -2.0f + 4.0f * j / 32.0f;
            out[k++] = filter_eval(rd, px, py);
        }
    out[k] = filter_integral(rd);
    return 0;
}

static void film_add(const pt_render_desc* rd, double inv_int, int W, int H, double* film, double px, double py, v3 L) {
    int rx = (int)ceilf(rd->filter_radius[0] - 0.5f), ry = (int)ceilf(rd->filter_radius[1] - 0.5f);
    double fx = px - floor(px), fy = py - floor(py);
    int ix = (int)floor(px), iy = (int)floor(py);
    for (int y = -ry; y <= ry; y++)
        for (int x = -rx; x <= rx; x++) {
            double sx = (double)x + 0.5 - fx, sy = (double)y + 0.5 - fy;
            double w = filter_eval(rd, (float)sx, (float)sy) * inv_int;
            int qx = x + ix, qy = y + iy;
            if (w <= 0 || qx < 0 || qy < 0 || qx >= W || qy >= H) continue;
            double* o = film + 4 * ((size_t)qy * W + qx);
            o[0] += (double)L.x * w;
            o[1] += (double)L.y * w;
            o[2] += (double)L.z * w;
            o[3] += w;
        }
}

typedef struct {
    const pt_scene_desc* s;
    const pt_camera_desc* cam;
    const pt_render_desc* rd;
    double* film;
    uint32_t* counts; /* adaptive: per-pixel sample counts, else NULL */
    int tiles_x, tiles;
    volatile int next;
    pthread_mutex_t mu;
    oracle_counters total;
} job_t;

/* TileIntegrator::Render's adaptive rounds for one pixel (Integrators.cpp:
 * 55-86; VarianceEstimator, Util.hpp:8-43): rounds of spp samples, round r
 * drawing stream samples r*spp .. r*spp+spp-1, until all three relative
 * variances of color * dvec3(0.2126f, 0.7152f, 0.0722f) are <= 1.5, at most
 * 128*spp samples.  Welford with the reference build's contraction: the
 * luminance product fused into both differences and into S's update.
 * Returns the pixel's sample count. */
static double rel_variance(double mean, double S, uint64_t n) {
    if (mean == 0) return 0;
    double var = n > 1 ? S / (double)(n - 1) : 0.0;
    return 1.96 * sqrt(var / (double)n) / mean;
}
static uint32_t adaptive_pixel(const integ_t* I, const job_t* J, double inv_int, int bx0, int by0, int bw, int bh,
                               double* tilebuf, int x, int y) {
    const double wl[3] = {(double)0.2126f, (double)0.7152f, (double)0.0722f};
    const uint32_t spp = J->rd->spp;
    double mean[3] = {0, 0, 0}, S[3] = {0, 0, 0};
    uint64_t n = 0;
    for (uint32_t round = 0; n < 128ull * spp; round++) {
        for (uint32_t k = 0; k < spp; k++) {
            double px, py;
            v3 L = li_one(I, J->cam, J->rd->seed, (uint32_t)x, (uint32_t)y, round * spp + k, &px, &py);
            film_add(J->rd, inv_int, bw, bh, tilebuf, px - bx0, py - by0, L);
            const double v[3] = {(double)L.x, (double)L.y, (double)L.z};
            const double dn = (double)(++n);
            for (int c = 0; c < 3; c++) {
                const double delta = fma(v[c], wl[c], -mean[c]);
                mean[c] = delta / dn + mean[c];
                const double delta2 = fma(v[c], wl[c], -mean[c]);
                S[c] = fma(delta, delta2, S[c]);
            }
        }
        if (rel_variance(mean[0], S[0], n) <= 1.5 && rel_variance(mean[1], S[1], n) <= 1.5 &&
            rel_variance(mean[2], S[2], n) <= 1.5)
            break;
    }
    return (uint32_t)n;
}

static void* render_worker(void* arg) {
    job_t* J = (job_t*)arg;
    scene_t S;
    scene_init(&S, J->s);
    oracle_counters c;
    memset(&c, 0, sizeof(c));
    integ_t I = {&S, J->rd->max_depth, J->rd->integrator == PT_INTEGRATOR_SIMPLE, &c, J->rd->integrator,
                 J->rd->strata[0], J->rd->strata[1]};
    int W = J->cam->width, H = J->cam->height;
    double inv_int = 1.0 / filter_integral(J->rd);
    int rx = (int)ceilf(J->rd->filter_radius[0] - 0.5f), ry = (int)ceilf(J->rd->filter_radius[1] - 0.5f);
    uint32_t sc = J->rd->shard_count ? J->rd->shard_count : 1;
    for (;;) {
        int tile = __sync_fetch_and_add(&J->next, 1);
        if (tile >= J->tiles) break;
        int tx = tile % J->tiles_x, ty = tile / J->tiles_x;
        int x0 = tx * 32, y0 = ty * 32, x1 = x0 + 32 < W ? x0 + 32 : W, y1 = y0 + 32 < H ? y0 + 32 : H;
        /* FilmTile over the tile + filter margin (Film.hpp:118-123), merged under a lock */
        int bx0 = x0 - rx < 0 ? 0 : x0 - rx, by0 = y0 - ry < 0 ? 0 : y0 - ry;
        int bx1 = x1 + rx > W ? W : x1 + rx, by1 = y1 + ry > H ? H : y1 + ry;
        int bw = bx1 - bx0, bh = by1 - by0;
        double* tilebuf = (double*)calloc((size_t)bw * bh * 4, sizeof(double));
        if (J->counts && (uint32_t)tile % sc != J->rd->shard_index) { /* adaptive shards own whole tiles */
            free(tilebuf);
            continue;
        }
        for (int y = y0; y < y1; y++)
            for (int x = x0; x < x1; x++) {
                if (J->counts) {
                    J->counts[(size_t)y * W + x] = adaptive_pixel(&I, J, inv_int, bx0, by0, bw, bh, tilebuf, x, y);
                    continue;
                }
                for (uint32_t smp = J->rd->shard_index; smp < J->rd->spp; smp += sc) {
                    double px, py;
                    v3 L = li_one(&I, J->cam, J->rd->seed, (uint32_t)x, (uint32_t)y, smp, &px, &py);
                    film_add(J->rd, inv_int, bw, bh, tilebuf, px - bx0, py - by0, L);
                }
            }
        pthread_mutex_lock(&J->mu);
        for (int y = 0; y < bh; y++)
            for (int x = 0; x < bw; x++)
                for (int k = 0; k < 4; k++)
                    J->film[4 * ((size_t)(y + by0) * W + (x + bx0)) + k] += tilebuf[4 * ((size_t)y * bw + x) + k];
        pthread_mutex_unlock(&J->mu);
        free(tilebuf);
    }
    pthread_mutex_lock(&J->mu);
    J->total.closest += c.closest;
    J->total.any += c.any;
    J->total.nodes_closest += c.nodes_closest;
    J->total.tris_closest += c.tris_closest;
    J->total.nodes_any += c.nodes_any;
    J->total.tris_any += c.tris_any;
    J->total.paths += c.paths;
    J->total.hits += c.hits;
    J->total.tex_bytes += c.tex_bytes;
    pthread_mutex_unlock(&J->mu);
    return NULL;
}

static int render_job(const pt_scene_desc* s, const pt_camera_desc* cam, const pt_render_desc* rd, double* film,
                      uint32_t* counts, int threads, oracle_counters* cnt);
int oracle_render(const pt_scene_desc* s, const pt_camera_desc* cam, const pt_render_desc* rd, double* film,
                  int threads, oracle_counters* cnt) {
    return render_job(s, cam, rd, film, NULL, threads, cnt);
}
int oracle_render_adaptive(const pt_scene_desc* s, const pt_camera_desc* cam, const pt_render_desc* rd,
                           double* film, uint32_t* counts, int threads, oracle_counters* cnt) {
    if (!counts) return -1;
    memset(counts, 0, sizeof(uint32_t) * (size_t)cam->width * cam->height);
    return render_job(s, cam, rd, film, counts, threads, cnt);
}
static int render_job(const pt_scene_desc* s, const pt_camera_desc* cam, const pt_render_desc* rd, double* film,
                      uint32_t* counts, int threads, oracle_counters* cnt) {
    if (!s || !cam || !rd || !film) return -1;
    if (threads < 1) threads = 1;
    job_t J;
    memset(&J, 0, sizeof(J));
    J.s = s;
    J.cam = cam;
    J.rd = rd;
    J.film = film;
    J.counts = counts;
    J.tiles_x = (cam->width + 31) / 32;
    J.tiles = J.tiles_x * ((cam->height + 31) / 32);
    pthread_mutex_init(&J.mu, NULL);
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
    for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, render_worker, &J);
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    free(th);
    pthread_mutex_destroy(&J.mu);
    if (cnt) *cnt = J.total;
    return 0;
}

/* Note: the film splat above works in tile-local coordinates; the filter
 * weights only depend on the fractional position, so this equals
 * FilmTile::Add at the absolute position. */

/* ------------------------------------------------------------------ unit cases */
/* Film::WritePNG's pixel body (Film.hpp:183-196): reinhard_jodie / ACESFilm
 * (Film.hpp:34-47) through std::function<vec3(vec3)> (float in and out),
 * linear_to_sRGB (Texture.hpp:13-17), 255.999 * clamp truncated to u8. */
static double glm_clamp01(double x) {
    double m = x < 0.0 ? 0.0 : x;
    return 1.0 < m ? 1.0 : m;
}
static double linear_to_srgb(double v) {
    v = glm_clamp01(v);
    return v < 0.0031308 ? 12.92 * v : 1.055 * pow(v, 1.0 / 2.4) - 0.055;
}
int oracle_resolve(const double* film, int W, int H, int tonemap, uint8_t* out) {
    for (size_t i = 0; i < (size_t)W * H; i++) {
        const double* a = film + 4 * i;
        double c[3], m[3];
        for (int k = 0; k < 3; k++) c[k] = (double)(float)(a[k] / a[3]);
        if (tonemap == 1) {
            const double A = 2.51f, B = 0.03f, C = 2.43f, D = 0.59f, E = 0.14f;
            for (int k = 0; k < 3; k++) m[k] = glm_clamp01((c[k] * (A * c[k] + B)) / (c[k] * (C * c[k] + D) + E));
        } else {
            double l = c[0] * 0.2126 + c[1] * 0.7152 + c[2] * 0.0722;
            for (int k = 0; k < 3; k++) {
                double t = c[k] / (1.0 + c[k]);
                m[k] = (c[k] / (1.0 + l)) * (1.0 - t) + t * t;
            }
        }
        for (int k = 0; k < 3; k++) {
            double s = linear_to_srgb((double)(float)m[k]);
            double lo = (s < 1.0) ? s : 1.0;  /* std::min(1.0, s) */
            double v = (0.0 < lo) ? lo : 0.0; /* std::max(0.0, .) */
            out[3 * i + k] = (uint8_t)(255.999 * v);
        }
    }
    return 0;
}

int oracle_bsdf(const pt_scene_desc* s, int mid, const float* in, uint32_t n, float* out) {
    scene_t S;
    scene_init(&S, s);
    for (uint32_t i = 0; i < n; i++) {
        const float* c = in + 27 * (size_t)i;
        float* o = out + 20 * (size_t)i;
        memset(o, 0, 20 * sizeof(float));
        ray_t r = mkray(V(c[0], c[1], c[2]), V(c[3], c[4], c[5]));
        si_t si;
        memset(&si, 0, sizeof(si));
        si.p = V(c[6], c[7], c[8]);
        si.n = V(c[9], c[10], c[11]);
        si.ns = V(c[12], c[13], c[14]);
        si.tangent = V(c[15], c[16], c[17]);
        si.uv[0] = c[18];
        si.uv[1] = c[19];
        si.t = c[20];
        si.mat = mid;
        bxdf_t b = mat_scatter(&S, mid, &r, &si, c[21], c[22], c[23]);
        if (b.ok) {
            o[0] = 1;
            o[1] = b.f.x; o[2] = b.f.y; o[3] = b.f.z;
            o[4] = b.pdf;
            o[5] = (float)b.flags;
            o[6] = b.o.x; o[7] = b.o.y; o[8] = b.o.z;
            o[9] = b.d.x; o[10] = b.d.y; o[11] = b.d.z;
            ray_t sc = mkray(b.o, b.d);
            v3 a = mat_f(&S, mid, &r, &si, sc.d);
            o[12] = a.x; o[13] = a.y; o[14] = a.z;
            o[15] = mat_pdf(&S, mid, &r, &si, sc.d);
        }
        v3 other = V(c[24], c[25], c[26]);
        v3 a2 = mat_f(&S, mid, &r, &si, other);
        o[16] = a2.x; o[17] = a2.y; o[18] = a2.z;
        o[19] = mat_pdf(&S, mid, &r, &si, other);
    }
    return 0;
}

int oracle_lights(const pt_scene_desc* s, const float* in, uint32_t n, float* out) {
    scene_t S;
    scene_init(&S, s);
    size_t k = 0;
    for (uint32_t li = 0; li < s->n_lights; li++) {
        const pt_light* l = &s->lights[li];
        for (uint32_t i = 0; i < n; i++, k++) {
            const float* c = in + 5 * (size_t)i;
            float* o = out + 18 * k;
            memset(o, 0, 18 * sizeof(float));
            /* a TextureInfiniteLight's hidden cell draw: a hash of the case (k_light_cases) */
            uint32_t h0, h1;
            memcpy(&h0, &c[0], 4);
            memcpy(&h1, &c[1], 4);
            const float uc = (float)(pcg_hash(pcg_hash(h0 ^ pcg_hash(h1))) >> 8) * (1.0f / 16777216.0f);
            lsample_t ls = light_sample(&S, l, c[0], c[1], uc, 0.0f);
            o[0] = ls.L.x; o[1] = ls.L.y; o[2] = ls.L.z;
            o[3] = ls.si.p.x; o[4] = ls.si.p.y; o[5] = ls.si.p.z;
            o[6] = ls.si.n.x; o[7] = ls.si.n.y; o[8] = ls.si.n.z;
            o[9] = ls.si.uv[0]; o[10] = ls.si.uv[1];
            o[11] = ls.dir.x; o[12] = ls.dir.y; o[13] = ls.dir.z;
            if (!is_zero(ls.si.n)) {
                v3 ref = V(c[2], c[3], c[4]);
                ray_t sh = mkray(ref, normalize(sub(ls.si.p, ref)));
                o[14] = light_pdf(&S, l, &ls.si, &sh);
                v3 L = light_L(&S, l, &ls.si, &sh);
                o[15] = L.x; o[16] = L.y; o[17] = L.z;
            }
        }
    }
    return 0;
}

/* ------------------------------------------------------------------ TextureInfiniteLight checks */
/* Le(dir) and PDF({}, dir) of light `li` for n directions -> out[4n] */
int oracle_inf_le(const pt_scene_desc* s, int li, const float* dirs, uint32_t n, float* out) {
    scene_t Sc;
    scene_init(&Sc, s);
    const scene_t* S = &Sc;
    const pt_light* l = &s->lights[li];
    for (uint32_t i = 0; i < n; i++) {
        v3 d = V(dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2]);
        v3 le = inf_le(l, d);
        out[4 * i] = le.x;
        out[4 * i + 1] = le.y;
        out[4 * i + 2] = le.z;
        out[4 * i + 3] = inf_pdf(S, l, d);
    }
    return 0;
}

/* TextureInfiniteLight::PreProcess's weight of cells k (Light.cpp:163-186),
 * restated independently of pt_envmap.cpp: a FloatImageTexture sky, the
 * jitter of the fixed hash (seed 0x7E1F5EED) */
static float envtex(const float* tx, int w, int h, int c, int x, int y, int ch) {
    int xi = x % w, yi = y % h;
    if (xi < 0) xi += w;
    if (yi < 0) yi += h;
    return tx[((size_t)yi * w + xi) * c + ch];
}
int oracle_texinf_weights(const float* tx, int w, int h, int c, const float cs[3], float scale, const uint32_t* cells,
                          uint32_t n, float* out) {
    for (uint32_t i = 0; i < n; i++) {
        uint32_t k = cells[i];
        int x = (int)(k % PT_TEXINF_Y), y = (int)(k / PT_TEXINF_Y);
        uint32_t key = pcg_hash(pcg_hash(0x7E1F5EEDu ^ pcg_hash(k)) + 0u);
        double temp = 0;
        for (int sp = 0; sp < 64; sp++) {
            int sx = sp % 8, sy = sp / 8;
            double jx = (double)((float)(pcg_hash(key + 0x9E3779B9u * (uint32_t)(2 * sp)) >> 8) * (1.0f / 16777216.0f));
            double jy = (double)((float)(pcg_hash(key + 0x9E3779B9u * (uint32_t)(2 * sp + 1)) >> 8) * (1.0f / 16777216.0f));
            float UVx = (float)((sx + jx) / 8.0), UVy = (float)((sy + jy) / 8.0);
            float u = ((float)x + UVx) / (float)PT_TEXINF_X, v = ((float)y + UVy) / (float)PT_TEXINF_Y;
            float z = 2.0f * u - 1.0f;
            float th = 2.0f * PI_F * v;
            float r = sqrtf(1.0f - rmul(z, z));
            v3 d = V(r * cosf(th), r * sinf(th), z);
            float uv[2];
            sphere_uv(d, uv);
            float fx = uv[0] * w - 0.5f, fy = uv[1] * h - 0.5f;
            int xi = (int)floorf(fx), yi = (int)floorf(fy);
            float dx = fx - xi, dy = fy - yi;
            float wa = (1 - dx) * (1 - dy), wb = dx * (1 - dy), wc = (1 - dx) * dy, wd = dx * dy;
            float L[3];
            for (int ch = 0; ch < 3; ch++) {
                float rr = fmaf(wd, envtex(tx, w, h, c, xi + 1, yi + 1, ch),
                                fmaf(wc, envtex(tx, w, h, c, xi, yi + 1, ch),
                                     fmaf(wb, envtex(tx, w, h, c, xi + 1, yi, ch), rmul(wa, envtex(tx, w, h, c, xi, yi, ch)))));
                L[ch] = scale * rmul(cs[ch], rr);
            }
            temp += fma((double)L[2], 0.0722, fma((double)L[1], 0.7152, (double)L[0] * 0.2126));
        }
        out[i] = (float)(temp / 64);
    }
    return 0;
}
