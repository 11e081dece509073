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
#define PT_TRACE_BLOCK 128

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

// QuadShape hit test (Shape.cpp:320-359)
__device__ __forceinline__ bool quad_hit(const pt_quad& q, f3 o, f3 d, float tmax, float& t, float& a, float& b) {
    f3 normal = ld3(q.normal);
    f3 nn = normal;
    float DD = q.D;
    if (dot(d, normal) > 0) {
        nn = -normal;
        DD = -q.D;
    }
    float denom = dot(nn, d);
    if (fabsf(denom) < 1e-8f) return false;
    t = (DD - dot(nn, o)) / denom;
    if (t < PT_EPS || t > tmax) return false;
    f3 ph = (o + t * d) - ld3(q.Q);
    f3 w = ld3(q.w);
    a = dot(w, cross(ph, ld3(q.v)));
    b = dot(w, cross(ld3(q.u), ph));
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

// Candidate uv for the alpha test on an alpha-tested triangle (rare path).
__device__ __noinline__ bool tri_alpha(uint32_t slot, float bu, float bv, f3 o, f3 d) {
    const DevPrimInfo pi = S.info[slot];
    uint4 T = S.tri[pi.index];
    float u = bu, v = bv, w = 1.0f - u - v;
    // the uv TriangleShape::Intersect computes (same contraction as tri_interaction)
    float tu = lerp3f(u, S.uvs[2 * T.y], v, S.uvs[2 * T.z], w, S.uvs[2 * T.x]);
    float tv = lerp3f(u, S.uvs[2 * T.y + 1], v, S.uvs[2 * T.z + 1], w, S.uvs[2 * T.x + 1]);
    return mat_alpha(pi.material, tu, tv, o, d, (int)slot);
}

// Rare primitive kinds (quad / sphere), closest hit.  Returns accepted hit.
__device__ __noinline__ bool other_closest(uint32_t slot, uint32_t w0, f3 o, f3 d, float tmax,
                                           float& t, float& b1, float& b2) {
    const DevPrimInfo pi = S.info[slot];
    float a = 0, b = 0;
    bool hit;
    if ((w0 & GF_KIND) == PT_PRIM_QUAD) hit = quad_hit(S.quads[pi.index], o, d, tmax, t, a, b);
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
    if ((w0 & GF_KIND) == PT_PRIM_QUAD) hit = quad_hit(S.quads[pi.index], o, d, tmax, t, a, b);
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

__device__ __forceinline__ uint32_t sel4u(uint32_t i, uint4 v) {
    return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
}
__device__ __forceinline__ float sel4f(uint32_t i, float a, float b, float c, float d) {
    return i == 0 ? a : (i == 1 ? b : (i == 2 ? c : d));
}

// 4-wide slab test (BVH.hpp:1049-1092 / 1140-1183) on a cluster's boxes
// xmin..zmax (one float4 per component, the 4 children in its lanes)
__device__ __forceinline__ void slab4q(float4 xmn, float4 xmx, float4 ymn, float4 ymx, float4 zmn, float4 zmx, f3 o,
                                       f3 inv, float tmax, uint32_t& mask, float te[4]) {
    float xa[4] = {xmn.x, xmn.y, xmn.z, xmn.w}, xb[4] = {xmx.x, xmx.y, xmx.z, xmx.w};
    float ya[4] = {ymn.x, ymn.y, ymn.z, ymn.w}, yb[4] = {ymx.x, ymx.y, ymx.z, ymx.w};
    float za[4] = {zmn.x, zmn.y, zmn.z, zmn.w}, zb[4] = {zmx.x, zmx.y, zmx.z, zmx.w};
    mask = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        float tx1 = (xa[i] - o.x) * inv.x, tx2 = (xb[i] - o.x) * inv.x;
        float ty1 = (ya[i] - o.y) * inv.y, ty2 = (yb[i] - o.y) * inv.y;
        float tz1 = (za[i] - o.z) * inv.z, tz2 = (zb[i] - o.z) * inv.z;
        float tEntry = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fminf(tz1, tz2));
        float tExit = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fmaxf(tz1, tz2));
        te[i] = tEntry;
        if (tExit >= PT_EPS && tEntry < tmax && tEntry <= tExit) mask |= 1u << i;
    }
}

template <bool COUNT>
__device__ __forceinline__ void slab4(const DevCluster* __restrict__ node, f3 o, f3 inv, float tmax, uint32_t& mask,
                                      float te[4]) {
    const float4* c4 = reinterpret_cast<const float4*>(node);
    slab4q(c4[0], c4[1], c4[2], c4[3], c4[4], c4[5], o, inv, tmax, mask, te);
}

// Closest hit.  Returns prim slot or -1; t, b1, b2 of the accepted hit.
template <bool COUNT>
__device__ int trace_closest(f3 o, f3 d, float tmax, float& t_out, float& b1_out, float& b2_out,
                             uint32_t* s_ref, TraceWork& wk) {
    const uint32_t lane = threadIdx.x;
    const f3 inv = inv_dir(d);
    const uint32_t oct = ((d.z < 0) << 2) | ((d.y < 0) << 1) | (d.x < 0);
    int sp = 0;
    uint32_t ref = S.root;
    int best = -1;
    float bb1 = 0, bb2 = 0;
    for (;;) {
        if (ref == REF_EMPTY) {
            // pop.  Entry distances are not kept (4-byte entries double the
            // occupancy); a node the reference would skip (entry > tmax,
            // BVH.hpp:1135) is fetched and all its children fail the slab test.
            if (sp == 0) break;
            --sp;
            ref = s_ref[sp * PT_TRACE_BLOCK + lane];
        }
        if (!(ref & REF_LEAF)) {
            const DevCluster* node = S.nodes + ref;
            if (COUNT) wk.nodes++;
            uint32_t mask;
            float te[4];
            slab4<COUNT>(node, o, inv, tmax, mask, te);
            const uint4 ch = *reinterpret_cast<const uint4*>(&node->child[0]);
            const uint32_t ow = node->order[oct >> 2];
            const uint32_t perm = (ow >> (8 * (oct & 3))) & 0xFFu;
            uint32_t cand = REF_EMPTY;
#pragma unroll
            for (int k = 0; k < 4; k++) {  // far -> near: 2-bit fields from the low end
                const uint32_t idx = (perm >> (2 * k)) & 3u;
                if ((mask >> idx) & 1u) {
                    const uint32_t c = sel4u(idx, ch);
                    if (c != REF_EMPTY) {
                        if (cand != REF_EMPTY && sp < PT_STACK) {
                            s_ref[sp * PT_TRACE_BLOCK + lane] = cand;
                            ++sp;
                        }
                        cand = c;
                    }
                }
            }
            ref = cand;
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
                    if (!(w0 & GF_ALPHA) || tri_alpha(slot, bx, by, o, d)) {
                        tmax = t;
                        best = (int)slot;
                        bb1 = bx;
                        bb2 = by;
                    }
                }
            } else if (kind == PT_PRIM_BLAS) {
                if (COUNT) wk.tris--;
                if (sp < PT_STACK) {
                    s_ref[sp * PT_TRACE_BLOCK + lane] = __float_as_uint(g.b.x);
                    ++sp;
                }
            } else {
                float t, a, b;
                if (other_closest(slot, w0, o, d, tmax, t, a, b)) {
                    tmax = t;
                    best = (int)slot;
                    bb1 = a;
                    bb2 = b;
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
template <bool COUNT>
__device__ bool trace_any(f3 o, f3 d, float tmax, uint32_t* s_ref, TraceWork& wk) {
    const uint32_t lane = threadIdx.x;
    const f3 inv = inv_dir(d);
    int sp = 0;
    uint32_t ref = S.root;
    for (;;) {
        if (ref == REF_EMPTY) {
            if (sp == 0) return false;
            --sp;
            ref = s_ref[sp * PT_TRACE_BLOCK + lane];
        }
        if (!(ref & REF_LEAF)) {
            const DevCluster* node = S.nodes + ref;
            if (COUNT) wk.nodes++;
            uint32_t mask;
            float te[4];
            slab4<COUNT>(node, o, inv, tmax, mask, te);
            const uint4 ch = *reinterpret_cast<const uint4*>(&node->child[0]);
            uint32_t cand = REF_EMPTY;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                if ((mask >> i) & 1u) {
                    const uint32_t c = sel4u((uint32_t)i, ch);
                    if (c != REF_EMPTY) {
                        if (cand != REF_EMPTY && sp < PT_STACK) {
                            s_ref[sp * PT_TRACE_BLOCK + lane] = cand;
                            ++sp;
                        }
                        cand = c;
                    }
                }
            }
            ref = cand;
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
                        if (!(w0 & GF_ALPHA) || tri_alpha(slot, bx, by, o, d)) return true;
                    }
                } else if (tri_pred(o, d, xyz(g.a), xyz(g.b), xyz(g.c), tmax)) {
                    return true;
                }
            } else if (kind == PT_PRIM_BLAS) {
                if (COUNT) wk.tris--;
                if (sp < PT_STACK) {
                    s_ref[sp * PT_TRACE_BLOCK + lane] = __float_as_uint(g.b.x);
                    ++sp;
                }
            } else if (other_pred(slot, w0, o, d, tmax)) {
                return true;
            }
            if (w0 & GF_LAST) break;
            ++slot;
        }
    }
}
