// BVH4 traversal for CDNA4 wave64: one ray per lane, per-lane stack of
// 32-bit node references (+ entry distances for closest hit) in LDS,
// interleaved [entry][lane] so every push/pop is bank-conflict free.
//
// Semantics follow BVH4::Intersect / IntersectPred (BVH.hpp:1019-1211):
//   slab test t = (bound - o) * inv_dir, hit iff tExit >= 1e-5 && tEntry < tmax
//   && tEntry <= tExit; closest hit visits children in the octant order of
//   BVH4::LUT (nearest first) and skips popped nodes with entry > tmax; leaf
//   primitives run the reference's exact triangle/quad/sphere tests
//   (glm::intersectRayTriangle for Intersect, the FLT_EPSILON-culled
//   Möller-Trumbore for IntersectPred, Shape.cpp:185-359) and the material
//   alpha test (Primitive.cpp:6-26).  A Model's BLAS root met in a TLAS leaf
//   is pushed and traversed with the same ray (Model.hpp:25-31).
#pragma once
#include "pt_shading.h"

#define PT_STACK 32
#ifndef PT_TRACE_BLOCK
#define PT_TRACE_BLOCK 128
#endif

struct TraceWork {
    uint32_t nodes, tris;
};

// glm::intersectRayTriangle (glm/gtx/intersect.inl:29-94), edges precomputed.
__device__ __forceinline__ bool tri_glm(f3 o, f3 d, f3 v0, f3 e1, f3 e2, float& bx, float& by, float& t) {
    f3 p = cross(d, e2);
    float det = dot(e1, p);
    f3 dist = o - v0;
    bx = dot(dist, p);
    f3 perp = cross(dist, e1);
    by = dot(d, perp);
    bool ok;
    if (det > 0.0f) ok = !(bx < 0.0f || bx > det) && !(by < 0.0f || bx + by > det);
    else if (det < 0.0f) ok = !(bx > 0.0f || bx < det) && !(by > 0.0f || bx + by < det);
    else ok = false;
    if (!ok) return false;
    float inv = 1.0f / det;
    t = dot(e2, perp) * inv;
    bx *= inv;
    by *= inv;
    return true;
}

// TriangleShape::IntersectPred (Shape.cpp:246-268)
__device__ __forceinline__ bool tri_pred(f3 o, f3 d, f3 v0, f3 e1, f3 e2, float tmax) {
    f3 h = cross(d, e2);
    float det = dot(e1, h);
    if (det > -PT_FLT_EPS && det < PT_FLT_EPS) return false;
    float inv = 1.0f / det;
    f3 s = o - v0;
    float u = dot(s, h) * inv;
    if (u < 0 || u > 1) return false;
    f3 q = cross(s, e1);
    float v = dot(d, q) * inv;
    if (v < 0 || u + v > 1) return false;
    float t = dot(e2, q) * inv;
    return t <= tmax && t >= PT_EPS;
}

// QuadShape hit test (Shape.cpp:320-359) as built: Intersect tests and
// divides by dot(d, nn) fused, IntersectPred (PRED) by the unfused dot; beta's
// cross(u, ph) rounded-first with its dot in y, x, z order
template <bool PRED>
__device__ __forceinline__ bool quad_hit(const pt_quad& q, f3 o, f3 d, float tmax, float& t, float& a, float& b) {
    f3 normal = ld3(q.normal);
    f3 nn = normal;
    float DD = q.D;
    const float dn = PRED ? dot_p(normal, d) : dot(d, normal);
    if (dn > 0) {
        nn = -normal;
        DD = -q.D;
    }
    const float denom = PRED ? (dn > 0 ? -dn : dn) : dot(d, nn);
    if (fabsf(denom) < 1e-8f) return false;
    t = (DD - dot(nn, o)) / denom;
    if (t < PT_EPS || t > tmax) return false;
    f3 ph = at_f(o, d, t) - ld3(q.Q);
    f3 w = ld3(q.w);
    a = dot(w, cross(ph, ld3(q.v)));
    b = dot_yxz(cross_r(ld3(q.u), ph), w);
    return a >= 0 && a <= 1 && b >= 0 && b <= 1;
}

// SphereShape root (Shape.cpp:3-56): first root in (1e-5, tmax)
__device__ __forceinline__ bool sphere_root(const pt_sphere& sp, f3 o, f3 d, float tmax, float& t) {
    f3 oc = o - ld3(sp.center);
    float a = dot(d, d);
    float b = dot(oc, d);
    // contraction of the reference build (DESIGN.md "Numerics"): the
    // cancellation in disc makes far-away sphere roots sensitive to it
    float c = fma_(-sp.radius, sp.radius, dot(oc, oc));
    float disc = fma_(b, b, -rmul(a, c));
    if (disc > 0) {
        float temp = (-b - csqrt(disc)) / a;
        if (temp < tmax && temp > PT_EPS) {
            t = temp;
            return true;
        }
        temp = (-b + csqrt(disc)) / a;
        if (temp < tmax && temp > PT_EPS) {
            t = temp;
            return true;
        }
    }
    return false;
}

__device__ __forceinline__ f3 inv_dir(f3 d) {  // Ray ctor (Ray.hpp:32-35)
    return F3(fabsf(d.x) < 1e-32f ? 1e32f : 1.0f / d.x, fabsf(d.y) < 1e-32f ? 1e32f : 1.0f / d.y,
              fabsf(d.z) < 1e-32f ? 1e32f : 1.0f / d.z);
}

// A u8 texel channel as channel_at reads it (wrapped coordinates, 0 past
// the texel buffer)
// (xi, yi: wrapped coordinates)
// (an image's element index fits 32 bits: pt_scene_upload checks its size;
// lim = the texel bytes from the image's offset on).  Branch-free: a texel
// past the buffer reads the buffer's first byte instead (an image texel
// exists, so the buffer does) and is replaced by 0, so the four loads of a
// footprint issue back to back instead of one branch (and one memory round
// trip) each.
__device__ __forceinline__ uint32_t alpha_texel_byte(const uint8_t* base, uint64_t lim, uint32_t local) {
    const bool in = (uint64_t)local < lim;
    const uint32_t b = *(in ? base + local : S.texels);
    return in ? b : 0u;
}
// The material alpha test of an alpha-tested triangle at its candidate hit
// (GeometricPrimitive::Intersect -> Material::Alpha, Primitive.cpp:6-26,
// Material.hpp:181-198).  ai: the slot's alpha record (DevAlpha, slot b.w):
// the record, then the four texels; ALPHA_IDX_NONE: prim info -> shading record
// -> material -> texture -> image.  Same values either way.
__device__ __forceinline__ bool tri_alpha_general(uint32_t slot, float bu, float bv, f3 o, f3 d);
__device__ __noinline__ bool tri_alpha_slow(uint32_t slot, float bu, float bv, f3 o, f3 d) {
    return tri_alpha_general(slot, bu, bv, o, d);
}
// the alpha-record path inline in the traversal loop (the general one stays a
// call): C4 1615 -> 1633 Mrays/s (closest-hit 20.58 -> 20.29 ms per launch,
// profiles/r04_ab_traversal.txt)
__device__ __forceinline__ bool tri_alpha_rec(const DevAlpha& r, uint32_t slot, float bu, float bv, f3 o, f3 d);
// ai: the alpha record index, set: its coverage mask set (pt_device.h)
__device__ __forceinline__
bool tri_alpha(uint32_t ai, uint32_t set, uint32_t slot, float bu, float bv, f3 o, f3 d) {
    if (ai != ALPHA_IDX_NONE) {
        // the whole record in three 16-B loads issued together (a reference
        // into S.alpha would let the compiler read its fields where they are
        // used, in branches, one round trip each)
        const float4* ap = reinterpret_cast<const float4*>(S.alpha + ai);
#ifndef PT_ALPHA_LAZY  // the record read only when the masks leave the cell undecided (+0.3 %, r06)
#define PT_ALPHA_LAZY 1
#endif
        float4 a0, a1, a2;
        if (!PT_ALPHA_LAZY) a0 = ap[0], a1 = ap[1], a2 = ap[2];
        if (PT_ALPHA_COV && set != PT_ALPHA_SET_NONE) {
            // the hit's cell in the two masks, read beside the record: a
            // decided cell answers without the texel reads
            const int n = 4 << (set >> 29);
            const uint32_t c = alpha_cell(bu, bv, n);
            uint32_t acc, rej;
            if (PT_ALPHA_IL) {  // the cell's accept and reject words side by side: one 8-B read
                const uint2 w = *reinterpret_cast<const uint2*>(S.amask + (set & 0x1FFFFFFFu) + 2u * (c >> 5));
                acc = w.x, rej = w.y;
            } else {
                const uint32_t* m = S.amask + (set & 0x1FFFFFFFu) + (c >> 5);
                acc = m[0], rej = m[max(1, (n * n) >> 5)];
            }
            if ((acc >> (c & 31)) & 1u) return true;
            if ((rej >> (c & 31)) & 1u) return false;
        }
        if (PT_ALPHA_LAZY) a0 = ap[0], a1 = ap[1], a2 = ap[2];
        const DevAlpha r = __builtin_bit_cast(DevAlpha, (DevGeom{a0, a1, a2}));
        return tri_alpha_rec(r, slot, bu, bv, o, d);
    }
    return tri_alpha_slow(slot, bu, bv, o, d);
}
// the test from a slot's words w0 = a.w, w1 = b.w (record index and mask set)
__device__ __forceinline__
bool tri_alpha_cov(uint32_t w0, uint32_t w1, uint32_t slot, float bu, float bv, f3 o, f3 d) {
    return tri_alpha(alpha_index(w0, w1), (w0 >> 16) | (w1 & 0xFFFF0000u), slot, bu, bv, o, d);
}
// the test over an alpha record already read
__device__ __forceinline__ bool tri_alpha_rec(const DevAlpha& r, uint32_t slot, float bu, float bv, f3 o, f3 d) {
    {
        const float u = bu, v = bv, w = 1.0f - u - v;
        const float tu = lerp3f(u, r.su[0], v, r.su[1], w, r.su[2]);
        const float tv = lerp3f(u, r.sv[0], v, r.sv[1], w, r.sv[2]);
        const uint32_t src = (r.mode >> 2) & 3u;
        float a;
        if (src == ALPHA_SRC_CONST) {
            a = __uint_as_float(r.off_lo);
        } else {
            const int W = (int)(r.wh & 0xFFFFu), H = (int)(r.wh >> 16), C = (int)((r.mode >> 8) & 0xFFu);
            const uint64_t off = (uint64_t)r.off_lo | (uint64_t)r.off_hi << 32;
            const float x = tu * W - 0.5f, y = tv * H - 0.5f;
            const int xi = (int)floorf(x), yi = (int)floorf(y);
            const float dx = x - xi, dy = y - yi;
            const int ch0 = src == ALPHA_SRC_CH4 ? 3 : 0;
            // a footprint inside the image needs no wrap; when every active
            // lane's is (a leaf card's uvs in [0, 1]: all but its edge texels),
            // the wave skips the remainders (a uniform branch)
            int x0, x1, y0, y1;
            const bool inb = (uint32_t)xi < (uint32_t)(W - 1) && (uint32_t)yi < (uint32_t)(H - 1);
            if (__ballot(!inb) == 0) {
                x0 = xi, x1 = xi + 1, y0 = yi, y1 = yi + 1;
            } else {
                x0 = wrap_index_t(xi, W), x1 = wrap_next(x0, W), y0 = wrap_index_t(yi, H), y1 = wrap_next(y0, H);
            }
            const uint8_t* base = S.texels + off;
            const uint64_t lim = S.n_texel_bytes > off ? S.n_texel_bytes - off : 0ull;
            const uint32_t r0 = (uint32_t)y0 * (uint32_t)W, r1 = (uint32_t)y1 * (uint32_t)W;
            auto at = [&](uint32_t r, int x) { return (r + (uint32_t)x) * (uint32_t)C + (uint32_t)ch0; };
            const uint32_t ba = alpha_texel_byte(base, lim, at(r0, x0)), bb = alpha_texel_byte(base, lim, at(r0, x1));
            const uint32_t bc = alpha_texel_byte(base, lim, at(r1, x0)), bd = alpha_texel_byte(base, lim, at(r1, x1));
            const float ta = u8_unit(ba), tb = u8_unit(bb), tc = u8_unit(bc), td = u8_unit(bd);
            const float wa = (1 - dx) * (1 - dy), wb = dx * (1 - dy), wc = (1 - dx) * dy, wd = dx * dy;
            // the two contractions as built: ImageTexture::alpha (tex_alpha) and
            // Evaluate(uv).x * colorScale.x (tex_eval_t)
            a = src == ALPHA_SRC_CH4 ? fma_(wd, td, fma_(wc, tc, fma_(wa, ta, rmul(wb, tb))))
                                     : r.scale * fma_(wd, td, fma_(wc, tc, fma_(wb, tb, rmul(wa, ta))));
        }
        const uint32_t mode = r.mode & 3u;
        if (mode == PT_ALPHA_OPAQUE) return true;
        if (mode == PT_ALPHA_MASK) return a > r.cut;
        return a >= 1.0f ? true : (blend_random(o, d, (int)slot) < a);
    }
}
// the general path: prim info -> shading record -> material -> texture -> image
__device__ __forceinline__ bool tri_alpha_general(uint32_t slot, float bu, float bv, f3 o, f3 d) {
    const DevPrimInfo pi = S.info[slot];
    const DevTriShade* R = S.tshade + slot;
    const float4 rc = R->c, rd = R->d;
    float u = bu, v = bv, w = 1.0f - u - v;
    // the uv TriangleShape::Intersect computes (same contraction as tri_interaction)
    float tu = lerp3f(u, rc.w, v, rd.y, w, rc.y);
    float tv = lerp3f(u, rd.x, v, rd.z, w, rc.z);
    return mat_alpha(pi.material, tu, tv, o, d, (int)slot);
}

// Rare primitive kinds (quad / sphere), closest hit.  Returns accepted hit.
__device__ __noinline__ bool other_closest(uint32_t slot, uint32_t w0, f3 o, f3 d, float tmax,
                                           float& t, float& b1, float& b2) {
    const DevPrimInfo pi = S.info[slot];
    float a = 0, b = 0;
    bool hit;
    if ((w0 & GF_KIND) == PT_PRIM_QUAD) hit = quad_hit<false>(S.quads[pi.index], o, d, tmax, t, a, b);
    else {
        hit = sphere_root(S.spheres[pi.index], o, d, tmax, t);
        if (hit && (w0 & GF_ALPHA)) {
            SurfInt si;
            sphere_interaction(S.spheres[pi.index], o, d, t, si);
            a = si.u;
            b = si.v;
        }
    }
    if (!hit) return false;
    if ((w0 & GF_ALPHA) && !mat_alpha(pi.material, a, b, o, d, (int)slot)) return false;
    b1 = a;
    b2 = b;
    return true;
}
__device__ __noinline__ bool other_pred(uint32_t slot, uint32_t w0, f3 o, f3 d, float tmax) {
    const DevPrimInfo pi = S.info[slot];
    float t, a = 0, b = 0;
    bool hit;
    // GeometricPrimitive::IntersectPred: a material with alpha runs the full
    // Intersect (GF_PRED_GLM), the others the shape's IntersectPred
    if ((w0 & GF_KIND) == PT_PRIM_QUAD)
        hit = (w0 & GF_PRED_GLM) ? quad_hit<false>(S.quads[pi.index], o, d, tmax, t, a, b)
                                 : quad_hit<true>(S.quads[pi.index], o, d, tmax, t, a, b);
    else {
        hit = sphere_root(S.spheres[pi.index], o, d, tmax, t);
        if (hit && (w0 & GF_ALPHA)) {
            SurfInt si;
            sphere_interaction(S.spheres[pi.index], o, d, t, si);
            a = si.u;
            b = si.v;
        }
    }
    if (!hit) return false;
    if ((w0 & GF_PRED_GLM) && (w0 & GF_ALPHA)) return mat_alpha(pi.material, a, b, o, d, (int)slot);
    return true;
}

// 4-wide slab test (BVH.hpp:1049-1092 / 1140-1183), children in pairs on the
// packed-FP32 ALU (v_pk_add_f32 / v_pk_mul_f32: two lanes per instruction,
// each lane the same rounded (bound - o) * inv as the scalar form)
typedef float v2f __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void slab4pe(float4 xmn, float4 xmx, float4 ymn, float4 ymx, float4 zmn, float4 zmx, f3 o,
                                        f3 inv, float tmax, uint32_t& mask, float (&te)[4]) {
    const v2f ox = {o.x, o.x}, oy = {o.y, o.y}, oz = {o.z, o.z};
    const v2f ix = {inv.x, inv.x}, iy = {inv.y, inv.y}, iz = {inv.z, inv.z};
    v2f t[2][6];
    t[0][0] = (v2f{xmn.x, xmn.y} - ox) * ix;
    t[1][0] = (v2f{xmn.z, xmn.w} - ox) * ix;
    t[0][1] = (v2f{xmx.x, xmx.y} - ox) * ix;
    t[1][1] = (v2f{xmx.z, xmx.w} - ox) * ix;
    t[0][2] = (v2f{ymn.x, ymn.y} - oy) * iy;
    t[1][2] = (v2f{ymn.z, ymn.w} - oy) * iy;
    t[0][3] = (v2f{ymx.x, ymx.y} - oy) * iy;
    t[1][3] = (v2f{ymx.z, ymx.w} - oy) * iy;
    t[0][4] = (v2f{zmn.x, zmn.y} - oz) * iz;
    t[1][4] = (v2f{zmn.z, zmn.w} - oz) * iz;
    t[0][5] = (v2f{zmx.x, zmx.y} - oz) * iz;
    t[1][5] = (v2f{zmx.z, zmx.w} - oz) * iz;
    mask = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int h = i >> 1, l = i & 1;
        const float tx1 = t[h][0][l], tx2 = t[h][1][l], ty1 = t[h][2][l], ty2 = t[h][3][l];
        const float tz1 = t[h][4][l], tz2 = t[h][5][l];
        const float tEntry = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fminf(tz1, tz2));
        const float tExit = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fmaxf(tz1, tz2));
        if (tExit >= PT_EPS && tEntry < tmax && tEntry <= tExit) mask |= 1u << i;
        te[i] = tEntry;
    }
}
__device__ __forceinline__ void slab4p(float4 xmn, float4 xmx, float4 ymn, float4 ymx, float4 zmn, float4 zmx, f3 o,
                                       f3 inv, float tmax, uint32_t& mask) {
    float te[4];
    slab4pe(xmn, xmx, ymn, ymx, zmn, zmx, o, inv, tmax, mask, te);
}

// bound = fma(byte, 2^(e-127), origin) per axis of a quantized record
__device__ __forceinline__ float qdec(uint32_t w, int k, float sc, float org) {
    return fma_((float)((w >> (8 * k)) & 0xFFu), sc, org);
}
__device__ __forceinline__ float4 qdec4(uint32_t w, float sc, float org) {
    return make_float4(qdec(w, 0, sc, org), qdec(w, 1, sc, org), qdec(w, 2, sc, org), qdec(w, 3, sc, org));
}
// The slab test on a quantized node with each axis's bounds pre-ordered by
// the sign of inv (near bound first): then min(t1, t2) is the near plane's t
// and max(t1, t2) the far plane's exactly (rounding is monotone, lo' <= hi'),
// so tEntry / tExit are one max3 / min3 per child instead of six min/max, and
// the result is bit-identical to slab4pe.  The bound words are swapped before
// decoding (one select per axis and side instead of one per child).
__device__ __forceinline__ void qslab4pe(float4 a, float4 b, float4 c, f3 o, f3 inv, float tmax, uint32_t& mask,
                                         float (&te)[4]) {
    const uint32_t ex = __float_as_uint(a.w);
    const float sx = __uint_as_float((ex & 0xFFu) << 23), sy = __uint_as_float(((ex >> 8) & 0xFFu) << 23),
                sz = __uint_as_float(((ex >> 16) & 0xFFu) << 23);
    const bool nx = inv.x < 0.0f, ny = inv.y < 0.0f, nz = inv.z < 0.0f;
    const uint32_t xl = __float_as_uint(b.x), xh = __float_as_uint(b.y), yl = __float_as_uint(b.z),
                   yh = __float_as_uint(b.w), zl = __float_as_uint(c.x), zh = __float_as_uint(c.y);
    const float4 xn = qdec4(nx ? xh : xl, sx, a.x), xf = qdec4(nx ? xl : xh, sx, a.x);
    const float4 yn = qdec4(ny ? yh : yl, sy, a.y), yf = qdec4(ny ? yl : yh, sy, a.y);
    const float4 zn = qdec4(nz ? zh : zl, sz, a.z), zf = qdec4(nz ? zl : zh, sz, a.z);
    const v2f ox = {o.x, o.x}, oy = {o.y, o.y}, oz = {o.z, o.z};
    const v2f ix = {inv.x, inv.x}, iy = {inv.y, inv.y}, iz = {inv.z, inv.z};
    v2f t[2][6];
    t[0][0] = (v2f{xn.x, xn.y} - ox) * ix;
    t[1][0] = (v2f{xn.z, xn.w} - ox) * ix;
    t[0][1] = (v2f{xf.x, xf.y} - ox) * ix;
    t[1][1] = (v2f{xf.z, xf.w} - ox) * ix;
    t[0][2] = (v2f{yn.x, yn.y} - oy) * iy;
    t[1][2] = (v2f{yn.z, yn.w} - oy) * iy;
    t[0][3] = (v2f{yf.x, yf.y} - oy) * iy;
    t[1][3] = (v2f{yf.z, yf.w} - oy) * iy;
    t[0][4] = (v2f{zn.x, zn.y} - oz) * iz;
    t[1][4] = (v2f{zn.z, zn.w} - oz) * iz;
    t[0][5] = (v2f{zf.x, zf.y} - oz) * iz;
    t[1][5] = (v2f{zf.z, zf.w} - oz) * iz;
    mask = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int h = i >> 1, l = i & 1;
        const float tEntry = fmaxf(fmaxf(t[h][0][l], t[h][2][l]), t[h][4][l]);
        const float tExit = fminf(fminf(t[h][1][l], t[h][3][l]), t[h][5][l]);
        if (tExit >= PT_EPS && tEntry < tmax && tEntry <= tExit) mask |= 1u << i;
        te[i] = tEntry;
    }
}

// Quantized node record (pt_device.h): child refs from the block base and the
// per-child descriptor bytes (offset | Q48_LEAF -> REF_LEAF | Q48_HOP ->
// REF_BLOCK), and the octant order byte BVH4::LUT[octant][perm] from the
// block's LDS copy of the table (s_lut, staged by stage_q48_lut).
__device__ __forceinline__ uint4 q48_children(float cz, float cw) {
    const uint32_t base = __float_as_uint(cz), desc = __float_as_uint(cw);
    uint32_t r[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t d = (desc >> (8 * k)) & 0xFFu;
        const uint32_t ref = (base + (d & 63u)) | ((d & Q48_LEAF) << 25) | ((d & Q48_HOP) << 22);
        r[k] = d == Q48_EMPTY ? REF_EMPTY : ref;
    }
    return make_uint4(r[0], r[1], r[2], r[3]);
}
// order_children over a quantized record's base + descriptors: the ref of a
// child is formed only when it is pushed or kept (fewer live registers than
// four decoded refs)
template <class Push>
__device__ __forceinline__ uint32_t order_children_q48(uint32_t mask, float cz, float cw, uint32_t perm, Push&& push) {
    const uint32_t base = __float_as_uint(cz), desc = __float_as_uint(cw);
    uint32_t vm = mask;
#pragma unroll
    for (int k = 0; k < 4; k++)
        if (((desc >> (8 * k)) & 0xFFu) == Q48_EMPTY) vm &= ~(1u << k);
    uint32_t cand = REF_EMPTY;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t ci = (perm >> (2 * k)) & 3u;
        const uint32_t d = (desc >> (8 * ci)) & 0xFFu;
        const uint32_t c = (base + (d & 63u)) | ((d & Q48_LEAF) << 25) | ((d & Q48_HOP) << 22);
        const bool v = (vm >> ci) & 1u;
        if (v && cand != REF_EMPTY) push(cand);
        cand = v ? c : cand;
    }
    return cand;
}
__device__ __forceinline__ uint32_t q48_perm(const uint8_t* s_lut, uint32_t oct, float aw) {
    return s_lut[(oct & OCT_MASK) * Q48_LUT_STRIDE + (__float_as_uint(aw) >> 24)];
}
#define Q48_LUT_BYTES (8 * Q48_LUT_STRIDE)  // a multiple of 16
// every thread of the block takes part (one barrier)
__device__ __forceinline__ void stage_q48_lut(uint8_t* s_lut) {
    uint32_t* w = reinterpret_cast<uint32_t*>(s_lut);
    for (uint32_t i = threadIdx.x; i < 8 * Q48_LUT_STRIDE / 4; i += blockDim.x) w[i] = S.qlut[i];
    __syncthreads();
}

// Children of a cluster in visit order: every valid child (passes the slab
// test, exists) but the last is pushed, the last becomes the next ref.  perm
// holds the visit order as 2-bit slot indices from the low end (0xE4 = slot
// order, any hit; the octant byte of BVH4::LUT, closest hit).  Selects only:
// the one conditional is the stack store, done by `push`.
template <class Push>
__device__ __forceinline__ uint32_t order_children(uint32_t mask, uint4 ch, uint32_t perm, Push&& push) {
    const uint32_t vm = mask & ((uint32_t)(ch.x != REF_EMPTY) | (uint32_t)(ch.y != REF_EMPTY) << 1 |
                                (uint32_t)(ch.z != REF_EMPTY) << 2 | (uint32_t)(ch.w != REF_EMPTY) << 3);
    uint32_t cand = REF_EMPTY;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t ci = (perm >> (2 * k)) & 3u;
        const uint32_t lo = (ci & 1u) ? ch.y : ch.x, hi = (ci & 1u) ? ch.w : ch.z;
        const uint32_t c = (ci & 2u) ? hi : lo;
        const bool v = (vm >> ci) & 1u;
        if (v && cand != REF_EMPTY) push(cand);
        cand = v ? c : cand;
    }
    return cand;
}

// ---- instances: the glm matrix helpers (m4_point, m4_dir, normal_matrix,
// m3_mul, normalize4) live in pt_shading.h (TransformedLight uses them too)

__device__ __forceinline__ uint32_t octant(f3 d) { return ((d.z < 0) << 2) | ((d.y < 0) << 1) | (d.x < 0); }

// Pops of REF_INST_ENTER, and the instance exit (ref = REF_INST_EXIT, not a
// stack entry).  Enter: save the world ray, take it to object space level by
// level, the outermost first (TransformedPrimitive::Intersect / IntersectPred,
// Primitive.cpp:42-64, once per nested wrapper: dir = inv*d, length, origin =
// inv*o, d = dir/length, max*length); the caller records its stack depth and
// continues at the BLAS root.  Exit: restore; a hit accepted inside becomes
// t/length per level, the innermost first, and its virtual slot.  Out of line
// and by value, so the traversal loop's registers are untouched by this rare
// path.
struct InstState {
    f3 o, d, inv;
    float tmax;
    uint32_t oct;
    int best;
    uint32_t ref;
    float time;  // the ray's (an AnimatedPrimitive is entered at its translation then)
};
// scratch word of level k's length: the outermost at 7, inner levels past the instance id
__device__ __forceinline__ uint32_t scr_len_word(int k) { return k == 0 ? 7u : 8u + (uint32_t)k; }
template <bool ANY, bool QN = false>
__device__ __forceinline__ InstState instance_step_inl(InstState s) {
    const uint32_t L = S.scratch_lanes;
    uint32_t* sc = S.scratch + blockIdx.x * blockDim.x + threadIdx.x;
    if (s.ref == REF_INST_EXIT) {
        const uint32_t inst = sc[8 * L];
        if (!ANY && (s.oct & OCT_HIT)) {
            const DevInstance& I = S.instances[inst];
            int levels = 1;
            for (int32_t in = I.inner; in >= 0 && levels < PT_MAX_INSTANCE_DEPTH; in = S.instances[in].inner) levels++;
            float t = s.tmax;
            for (int k = levels - 1; k >= 0; k--) t = t / __uint_as_float(sc[scr_len_word(k) * L]);
            s.tmax = t;
            s.best = (int)(I.virt_base + ((uint32_t)s.best - I.prim_base));
        } else {
            s.tmax = __uint_as_float(sc[6 * L]);
        }
        s.o = F3(__uint_as_float(sc[0]), __uint_as_float(sc[L]), __uint_as_float(sc[2 * L]));
        s.d = F3(__uint_as_float(sc[3 * L]), __uint_as_float(sc[4 * L]), __uint_as_float(sc[5 * L]));
        s.inv = inv_dir(s.d);
        // the per-ray flags survive the exit: a ray already listed for the
        // exact-tie re-trace (OCT_TIE) must not be listed again
        s.oct = octant(s.d) | (s.oct & (OCT_TIE | OCT_FOUND));
        s.ref = REF_EMPTY;
        return s;
    }
    const uint32_t slot = s.ref & REF_SLOT_MASK;
    const uint32_t inst = __float_as_uint(S.geom[slot].b.y);
    const float w[7] = {s.o.x, s.o.y, s.o.z, s.d.x, s.d.y, s.d.z, s.tmax};
    for (int k = 0; k < 7; k++) sc[k * L] = __float_as_uint(w[k]);
    sc[8 * L] = inst;
    const DevInstance* I = &S.instances[inst];
    for (int k = 0;; k++) {
        f3 dir, org;
        if (S.motion && I->anim) {  // AnimatedPrimitive::Intersect(Pred) at the ray's time (Primitive.cpp:82-89)
            float T[16], inv[16];
            anim_transform(*I, s.time, T);
            anim_inverse(T, inv);
            dir = m4_dir(inv, s.d);
            org = m4_point(inv, s.o);
        } else {
            dir = m4_dir(I->inv, s.d);
            org = m4_point(I->inv, s.o);
        }
        const float len = length(dir);
        sc[scr_len_word(k) * L] = __float_as_uint(len);
        s.o = org;
        s.d = dir / len;
        s.tmax = s.tmax * len;
        if (I->inner < 0 || k + 1 == PT_MAX_INSTANCE_DEPTH) break;  // (the upload bounds the depth)
        I = &S.instances[I->inner];
    }
    s.inv = inv_dir(s.d);
    s.oct = octant(s.d) | OCT_INST | (s.oct & (OCT_TIE | OCT_FOUND));
    s.ref = QN ? I->qroot : I->root;  // the BLAS root in the traversal's node form
    return s;
}
// The pool kernels (7 waves per SIMD, 72 VGPRs) call it out of line; the
// one-ray-per-lane kernels (5 waves) inline it (+4 % on the instanced scene).
template <bool ANY, bool QN>
__device__ __noinline__ InstState instance_step(InstState s) {
    return instance_step_inl<ANY, QN>(s);
}
// Entering records the stack depth in oct (OCT_SP_SHIFT); the instance is
// left when the traversal is back at that depth with nothing to visit
// (PT_INSTANCE_LEAVE), so no marker takes a stack entry that a full stack
// could drop.
#define PT_INSTANCE_STEP_FN(ANY_, FN_, TIME_)                                                   \
    do {                                                                                \
        const bool enter_ = ref != REF_INST_EXIT;                                       \
        const InstState st_ = FN_(InstState{o, d, inv, tmax, oct, best, ref, (TIME_)});      \
        o = st_.o;                                                                      \
        d = st_.d;                                                                      \
        inv = st_.inv;                                                                  \
        tmax = st_.tmax;                                                                \
        oct = st_.oct | (enter_ ? (uint32_t)sp << OCT_SP_SHIFT : 0u);                   \
        best = st_.best;                                                                \
        ref = st_.ref;                                                                  \
    } while (0)
// true when the lane's ray is inside an instance whose BLAS is exhausted
#define PT_INSTANCE_DONE() ((oct & OCT_INST) && (uint32_t)sp == (oct >> OCT_SP_SHIFT))
// (PT_INSTANCE_STEP: inside trace_pool, whose QN names the node form)
// TIME_: the lane's ray time (0 unless the scene has an AnimatedPrimitive)
#define PT_INSTANCE_STEP(ANY_, TIME_) PT_INSTANCE_STEP_FN(ANY_, (instance_step<ANY_, QN>), TIME_)
#define PT_INSTANCE_STEP_INL(ANY_) PT_INSTANCE_STEP_FN(ANY_, instance_step_inl<ANY_>, time)

// Closest hit.  Returns prim slot or -1; t, b1, b2 of the accepted hit.
// LN: stack entries kept in LDS; entries [LN, PT_STACK) go to ovf
// ([entry][grid lane], sized by the runtime for the one-ray-per-lane grid).
template <bool COUNT, bool INST = true, int LN = PT_STACK>
__device__ int trace_closest(f3 o, f3 d, float tmax, float& t_out, float& b1_out, float& b2_out,
                             uint32_t* s_ref, TraceWork& wk, uint32_t* __restrict__ ovf = nullptr, float time = 0.0f) {
    const uint32_t lane = threadIdx.x;
    f3 inv = inv_dir(d);
    uint32_t oct = octant(d);
    int sp = 0;
    uint32_t ref = S.root;
    int best = -1;
    float bb1 = 0, bb2 = 0;
    const uint32_t gl = blockIdx.x * PT_TRACE_BLOCK + lane, G = gridDim.x * PT_TRACE_BLOCK;
    auto push = [&](uint32_t v) {
        if (sp < PT_STACK) {
            if (LN >= PT_STACK || sp < LN) s_ref[sp * PT_TRACE_BLOCK + lane] = v;
            else ovf[(size_t)(sp - LN) * G + gl] = v;
            ++sp;
        } else {
            atomicAdd(S.stack_drops, 1u);  // counted: pt_stats::stack_overflows
        }
    };
    for (;;) {
        if (ref == REF_EMPTY) {
            if (INST && PT_INSTANCE_DONE()) {  // leave the instance
                ref = REF_INST_EXIT;
                PT_INSTANCE_STEP_INL(false);
                continue;
            }
            // pop.  Entry distances are not kept (4-byte entries double the
            // occupancy); a node the reference would skip (entry > tmax,
            // BVH.hpp:1135) is fetched and all its children fail the slab test.
            if (sp == 0) break;
            --sp;
            ref = (LN >= PT_STACK || sp < LN) ? s_ref[sp * PT_TRACE_BLOCK + lane] : ovf[(size_t)(sp - LN) * G + gl];
        }
        if (INST && ref >= REF_SPECIAL) {
            PT_INSTANCE_STEP_INL(false);
            continue;
        }
        if (!(ref & REF_LEAF)) {
            const float4* __restrict__ q = reinterpret_cast<const float4*>(S.nodes + ref);
            if (COUNT) wk.nodes++;
            const float4 q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3], q4 = q[4], q5 = q[5], q6 = q[6];
            const uint2 q7 = *reinterpret_cast<const uint2*>(q + 7);
            uint32_t mask;
            slab4p(q0, q1, q2, q3, q4, q5, o, inv, tmax, mask);
            const uint32_t ow = ((oct >> 2) & 1u) ? q7.y : q7.x;
            const uint32_t perm = (ow >> (8 * (oct & 3))) & 0xFFu;  // far -> near (BVH.hpp:1195-1204)
            ref = order_children(mask, make_uint4(__float_as_uint(q6.x), __float_as_uint(q6.y),
                                                  __float_as_uint(q6.z), __float_as_uint(q6.w)),
                                 perm, push);
            continue;
        }
        // leaf: primitives from slot until the one flagged LAST
        uint32_t slot = ref & ~REF_LEAF;
        ref = REF_EMPTY;
        for (;;) {
            const DevGeom g = S.geom[slot];
            const uint32_t w0 = __float_as_uint(g.a.w);
            const uint32_t kind = w0 & GF_KIND;
            if (COUNT) wk.tris++;
            if (kind == PT_PRIM_TRIANGLE) {
                float bx, by, t;
                if (tri_glm(o, d, xyz(g.a), xyz(g.b), xyz(g.c), bx, by, t) && !(t > tmax || t < PT_EPS)) {
                    if (!(w0 & GF_ALPHA) || tri_alpha_cov(w0, __float_as_uint(g.b.w), slot, bx, by, o, d)) {
                        tmax = t;
                        best = (int)slot;
                        bb1 = bx;
                        bb2 = by;
                        oct |= (oct & OCT_INST) << 1;  // OCT_HIT inside an instance
                    }
                }
            } else if (kind == PT_PRIM_BLAS) {  // a Model's BLAS root, or REF_INST_ENTER | slot
                // the BLAS first, the rest of the leaf after it: the
                // reference recurses inside its leaf loop (BVH.hpp:1206)
                if (COUNT) wk.tris--;
                if (!(w0 & GF_LAST)) push(REF_LEAF | (slot + 1));
                push(__float_as_uint(g.b.x));
                break;
            } else {
                float t, a, b;
                if (other_closest(slot, w0, o, d, tmax, t, a, b)) {
                    tmax = t;
                    best = (int)slot;
                    bb1 = a;
                    bb2 = b;
                    oct |= (oct & OCT_INST) << 1;
                }
            }
            if (w0 & GF_LAST) break;
            ++slot;
        }
    }
    t_out = tmax;
    b1_out = bb1;
    b2_out = bb2;
    return best;
}

// Any hit (Scene::IntersectPred).  Children pushed in slot order like the
// reference (BVH.hpp:1099-1102); the last one is visited next without a push.
template <bool COUNT, bool INST = true, int LN = PT_STACK>
__device__ bool trace_any(f3 o, f3 d, float tmax, uint32_t* s_ref, TraceWork& wk,
                          uint32_t* __restrict__ ovf = nullptr, float time = 0.0f) {
    const uint32_t lane = threadIdx.x;
    f3 inv = inv_dir(d);
    uint32_t oct = 0;
    int best = -1;
    int sp = 0;
    uint32_t ref = S.root;
    const uint32_t gl = blockIdx.x * PT_TRACE_BLOCK + lane, G = gridDim.x * PT_TRACE_BLOCK;
    auto push = [&](uint32_t v) {
        if (sp < PT_STACK) {
            if (LN >= PT_STACK || sp < LN) s_ref[sp * PT_TRACE_BLOCK + lane] = v;
            else ovf[(size_t)(sp - LN) * G + gl] = v;
            ++sp;
        } else {
            atomicAdd(S.stack_drops, 1u);  // counted: pt_stats::stack_overflows
        }
    };
    for (;;) {
        if (ref == REF_EMPTY) {
            if (INST && PT_INSTANCE_DONE()) {  // leave the instance
                ref = REF_INST_EXIT;
                PT_INSTANCE_STEP_INL(true);
                continue;
            }
            if (sp == 0) return false;
            --sp;
            ref = (LN >= PT_STACK || sp < LN) ? s_ref[sp * PT_TRACE_BLOCK + lane] : ovf[(size_t)(sp - LN) * G + gl];
        }
        if (INST && ref >= REF_SPECIAL) {
            PT_INSTANCE_STEP_INL(true);
            continue;
        }
        if (!(ref & REF_LEAF)) {
            const float4* __restrict__ q = reinterpret_cast<const float4*>(S.nodes + ref);
            if (COUNT) wk.nodes++;
            const float4 q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3], q4 = q[4], q5 = q[5], q6 = q[6];
            uint32_t mask;
            slab4p(q0, q1, q2, q3, q4, q5, o, inv, tmax, mask);
            // slot order, the last visited next (BVH.hpp:1099-1102)
            ref = order_children(mask, make_uint4(__float_as_uint(q6.x), __float_as_uint(q6.y),
                                                  __float_as_uint(q6.z), __float_as_uint(q6.w)),
                                 0xE4u, push);
            continue;
        }
        uint32_t slot = ref & ~REF_LEAF;
        ref = REF_EMPTY;
        for (;;) {
            const DevGeom g = S.geom[slot];
            const uint32_t w0 = __float_as_uint(g.a.w);
            const uint32_t kind = w0 & GF_KIND;
            if (COUNT) wk.tris++;
            if (kind == PT_PRIM_TRIANGLE) {
                if (w0 & GF_PRED_GLM) {
                    // material HasAlpha(): full Intersect + Alpha (Primitive.cpp:7-10)
                    float bx, by, t;
                    if (tri_glm(o, d, xyz(g.a), xyz(g.b), xyz(g.c), bx, by, t) && !(t > tmax || t < PT_EPS)) {
                        if (!(w0 & GF_ALPHA) || tri_alpha_cov(w0, __float_as_uint(g.b.w), slot, bx, by, o, d)) return true;
                    }
                } else if (tri_pred(o, d, xyz(g.a), xyz(g.b), xyz(g.c), tmax)) {
                    return true;
                }
            } else if (kind == PT_PRIM_BLAS) {  // a Model's BLAS root, or REF_INST_ENTER | slot
                if (COUNT) wk.tris--;
                push(__float_as_uint(g.b.x));
            } else if (other_pred(slot, w0, o, d, tmax)) {
                return true;
            }
            if (w0 & GF_LAST) break;
            ++slot;
        }
    }
}
