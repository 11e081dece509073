// Device-side scene layout and shared math for the CDNA4 wavefront tracer.
// All arithmetic follows the reference's float semantics (see DESIGN.md
// "Numerics"): correctly rounded division and sqrt (__builtin_sqrtf lowers to
// the corrected v_sqrt sequence on gfx950), glm operand order.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pt_api.h"

#define PT_EPS 0.00001f  // shadowEpsilon (AABB.hpp:6)
#define PT_FLT_EPS 1.19209290e-07f
#define PT_PI 3.14159265358979323846f
#define PT_INV_PI 0.318309886183790671538f

// ---- device BVH4 node: the reference cluster's boxes (BVH.hpp:45-60) with
// child references re-encoded for a stack of 32-bit entries, and the octant
// child order (BVH.hpp:562-738) precomputed per node.  128 bytes, 128-aligned.
#define REF_EMPTY 0xFFFFFFFFu
#define REF_LEAF 0x80000000u
// Quantized-record leaf refs only: the leaf holds a BLAS hop, whose test
// pushes a traversal, so the overlapped traversal (pt_pool.h trace_spec)
// pauses its node side until the leaf is done.  Slots < 2^29.
#define REF_BLOCK 0x20000000u
struct alignas(128) DevCluster {
    float4 xmin, xmax, ymin, ymax, zmin, zmax;  // 4 children per component
    uint32_t child[4];                          // REF_EMPTY | REF_LEAF|slot | cluster
    uint32_t order[2];                          // 8 octants x permutation byte
    uint32_t pad[2];
};
static_assert(sizeof(DevCluster) == 128, "cluster layout");

// ---- quantized BVH4 node (the upload's intermediate form of a 48-B node
// record below): the same cluster with its four
// child boxes stored as 8-bit offsets from a per-node origin in power-of-two
// steps per axis (scale 2^(e-127)).  Encoded on the host so that every
// decoded bound fma(q, scale, origin) lies outside the reference's float
// bound (lo' <= lo, hi' >= hi): the slab test on the decoded box accepts
// every child the reference accepts, so the traversal visits a superset of
// the reference's nodes in the same order and finds the same closest hit.
//   a = origin.xyz, exponents (x | y << 8 | z << 16)
//   b = x lo[4], x hi[4], y lo[4], y hi[4]   (one byte per child)
//   c = z lo[4], z hi[4], order[0], order[1]  (octant order bytes as DevCluster)
//   d = child[4]
struct alignas(64) DevQNode {
    float4 a;
    uint32_t b[4];
    uint32_t c[4];
    uint32_t child[4];
};
static_assert(sizeof(DevQNode) == 64, "qnode layout");

// ---- unified 48-B records (the quantized node form): node records
// and the primitive slots of their leaf children in ONE array, each cluster's
// children in one contiguous block (inner children 1 record, a leaf child its
// primitives' slots), so a node names its children with one base and four
// byte offsets and a node step is three 16-B loads instead of four.
//   node:  a = origin.xyz, w = ex | ey << 8 | ez << 16 | perm << 24
//              (perm: the reference's topology code, BVH4_NODE::perm; the
//              octant order byte is BVH4::LUT[octant][perm], an LDS table)
//          b = x lo[4], x hi[4], y lo[4], y hi[4]  (as DevQNode)
//          c = z lo[4], z hi[4], base, desc
//              desc = 4 x u8 per child slot: 0xFF empty, else offset (0..62)
//              from base | 0x40 leaf | 0x80 leaf holding a BLAS hop
//   primitive: the slot's DevGeom with c.w = the slot (hits and the shading
//              tables stay indexed by slot)
#define Q48_EMPTY 0xFFu
#define Q48_LEAF 0x40u
#define Q48_HOP 0x80u
#define Q48_MAX_OFFSET 62u
// escape links (DevScene::qesc, one per record): a node record's parent record
// and its child slot there, parent << 2 | k (records < 2^29); ESC_EXIT at each
// BVH's root record; ESC_BLAS marks a copy of a BLAS root in a TLAS block
#define ESC_EXIT 0xFFFFFFFFu
#define ESC_BLAS 0x80000000u
#define Q48_LUT_STRIDE 136  // bytes per octant row of the LDS order table (135 perms)

// ---- primitive slot geometry (48 B): what a leaf test reads.
// a = v0|Q|center + flags, b = e1|u|radius + index, c = e2|v
#define GF_KIND 3u
#define GF_LAST 4u        // last primitive of its leaf
#define GF_ALPHA 8u       // closest hit: run the material alpha test
#define GF_PRED_GLM 16u   // any hit: material HasAlpha() -> full Intersect + Alpha
struct alignas(16) DevGeom {
    float4 a, b, c;
};

// ---- alpha records: what tri_alpha reads for an alpha-tested triangle, in
// one 48-B record (its slot names the record index, alpha_index below;
// ALPHA_IDX_NONE: the general path).  tri_alpha otherwise walks prim info -> shading record ->
// material -> texture -> image -> texels, six dependent reads inside the
// traversal loop; here it is the record, then the texels.
//   su / sv   the triangle's uv components in lerp3f order (uv1, uv2, uv0)
//   off       the image's byte offset in the texel buffer (ALPHA_SRC_CONST:
//             word 0 = the constant alpha)
//   wh        width | height << 16;  mode = alpha mode | source << 2 |
//             channels << 8;  cut = MASK cutoff;  scale = the alpha
//             texture's colorScale.x (ALPHA_SRC_CH1)
#define ALPHA_IDX_NONE 0x7FFFFFFu
#define ALPHA_SRC_CH4 0u    // Texture::alpha of the material's texture: channel 4 (Texture.cpp:47-62)
#define ALPHA_SRC_CH1 1u    // the material's alpha texture: Evaluate(uv).x (Material.hpp:181-198)
#define ALPHA_SRC_CONST 2u  // a constant alpha (solid texture, or an image without a 4th channel)
struct alignas(16) DevAlpha {
    float su[3], sv[3];
    uint32_t off_lo, off_hi;
    uint32_t wh, mode;
    float cut, scale;
};
static_assert(sizeof(DevAlpha) == 48, "alpha record layout");
// ---- alpha coverage (pt_alpha_cov.h): an alpha-tested triangle's slot holds
// the handle of its coverage mask set (DevScene::amask word offset | log2(n /
// 4) << 29, PT_ALPHA_SET_NONE: none) in a.w bits 16-31 (low half) and b.w
// bits 16-31 (high half); the alpha record index (27 bits) is split over a.w
// bits 5-15 (high) and b.w bits 0-15 (low).  The cell of a hit's barycentrics
// (u, v) (weights of vertices 1 and 2) in the n x n subdivision: row j =
// floor(n v) has n - j lower and n-1-j upper sub-triangles; cell j (2n - j) +
// 2 i + upper.  n u and n v are exact (n a power of two); a point past the
// hypotenuse (by rounding only) goes to the diagonal's lower cell, whose
// footprint margin covers it.
// PT_ALPHA_COV: 0 no masks (the exact test always), 1 the mask sets
#ifndef PT_ALPHA_COV
#define PT_ALPHA_COV 1
#endif
#define PT_ALPHA_SET_NONE 0xFFFFFFFFu
#ifndef PT_ALPHA_IL  // mask words interleaved (accept, reject) per 32 cells (pt_alpha_cov.h): +0.5 %, r06
#define PT_ALPHA_IL 1
#endif
__device__ __forceinline__ uint32_t alpha_index(uint32_t w0, uint32_t w1) {
    return ((w0 >> 5) & 0x7FFu) << 16 | (w1 & 0xFFFFu);
}
__device__ __forceinline__ uint32_t alpha_cell(float u, float v, int n) {
    const float fn = (float)n, a = fn * u, b = fn * v;
    const float fi = __builtin_amdgcn_fmed3f(floorf(a), 0.0f, fn - 1.0f);
    const float fj = __builtin_amdgcn_fmed3f(floorf(b), 0.0f, fn - 1.0f);
    const int i = (int)fi, j = (int)fj, im = n - 1 - j;
    const bool up = (a - fi) + (b - fj) > 1.0f && i < im;
    return (uint32_t)(j * (2 * n - j) + 2 * min(i, im) + (up ? 1 : 0));
}
// Instances (TransformedPrimitive, Primitive.cpp:32-72).  A TLAS leaf slot of
// an instance is encoded like a BLAS hop whose pushed ref is
// REF_INST_ENTER | slot; popping it takes the lane's ray to object space
// (state saved in a per-lane scratch row) and records the stack depth; the
// world ray is restored (REF_INST_EXIT step) when the instance's BLAS is done.  Node refs stay
// below REF_LEAF and leaf slots below 2^30, so refs >= REF_SPECIAL are free.
#define REF_SPECIAL 0xC0000000u
#define REF_INST_ENTER 0xC0000000u
#define REF_INST_EXIT 0xFFFFFFFEu
#define REF_SLOT_MASK 0x3FFFFFFFu
#define OCT_MASK 7u
#define OCT_INST 8u   // the lane's ray is in an instance's object space
#define OCT_HIT 16u   // ... and accepted a hit there
#define OCT_FOUND 32u // overlapped traversal (pt_pool.h trace_spec): a hit was stored
#define OCT_FRESH 128u // overlapped traversal: the ray was claimed this iteration (set up after the loads)
#define OCT_TIE 64u   // pool traversal: this ray met a hit at exactly t == max (listed once for the exact re-trace)
#define OCT_SP_SHIFT 8  // ... entered at this stack depth (bits 8-13)
// scratch row: world o, d, tmax, the outermost level's length, instance, the
// inner levels' lengths (nested wrappers, pt_api.h PT_MAX_INSTANCE_DEPTH)
#define SCR_WORDS (9 + PT_MAX_INSTANCE_DEPTH - 1)
struct DevInstance {
    float T[16], inv[16];  // glm column-major transform and inverse
    uint32_t root;         // BLAS root ref
    uint32_t qroot;        // ... in the quantized records
    uint32_t prim_base;    // first slot of the BLAS
    uint32_t n_prims;
    uint32_t virt_base;    // virtual slot of the BLAS's first primitive
    // AnimatedPrimitive (Primitive.cpp:76-96): anim != 0 translates by mdir * t
    // at each ray's time (pt_shading.h anim_transform); T / inv: time 0
    float mdir[3];
    float t0, t1;
    uint32_t anim;
    int32_t inner;         // the next level down (nested wrappers), or -1
};

// ---- per-triangle shading record (128 B, one cache line): the three
// vertices' normals and uvs and the flags in the first 64 B, the tangents in
// the second (read only for meshes that carry them).  The same values as the
// indexed mesh arrays, gathered once at upload: the shading of a hit reads one
// line instead of the index and up to nine scattered vertex attributes.
//   a = n0.xyz n1.x, b = n1.yz n2.xy, c = n2.z uv0 uv1.u, d = uv1.v uv2 flags
//   e = t0.xyz t1.x, f = t1.yz t2.xy, g = t2.z
struct alignas(128) DevTriShade {
    float4 a, b, c, d, e, f, g, pad;
};
static_assert(sizeof(DevTriShade) == 128, "shading record layout");

// An area light's triangle, gathered per light at upload (what AreaLight::
// sample / PDF read through its shape: the vertices and uvs), so NEE reads it
// beside the light instead of prim info -> triangle -> vertices:
//   a = v0.xyz, uv0.x   b = v1.xyz, uv1.x   c = v2.xyz, uv2.x
//   d = uv0.y, uv1.y, uv2.y, valid (bits: 1 = a triangle area light)
struct alignas(16) DevLightTri {
    float4 a, b, c, d;
};
#ifndef PT_LIGHT_TRI  // 0: AreaLight::sample / PDF read the triangle through prim info -> S.tri -> vertices
#define PT_LIGHT_TRI 1
#endif

struct DevPrimInfo {
    int32_t material, light, medium;
    uint32_t index;  // triangle / quad / sphere id, BLAS root ref
};

// Guide table of the power light sampler: entry b = the first light whose
// running sum reaches fl(b / PT_LS_GUIDE * total) (PT_LS_GUIDE: the count of
// n lights when none does).  A draw u in bucket floor(u * PT_LS_GUIDE) has its
// pick between entries b and b + 1, so the search covers a few lights.
#define PT_LS_GUIDE 4096u

struct DevScene {
    float bb_lo[3], bb_scale[3];  // scene box: lo and 16 / extent per axis (spatial hit sort)
    const uint16_t* prim_cell;    // each primitive slot's centroid cell (spatial hit sort), else null
    const uint32_t* ray_order;    // closest-hit claim order (PT_RENDER_SORT_RAYS), else null
    const DevCluster* nodes;
    const DevGeom* geom;
    const DevPrimInfo* info;
    const DevGeom* qrec;       // the quantized records (null: the scene could not be encoded)
    const uint32_t* qlut;      // BVH4::LUT as 8 rows of Q48_LUT_STRIDE bytes (staged into LDS)
    const uint32_t* qesc;      // per record: escape link of the stackless any-hit traversal (ESC_*)
    uint32_t qrec_bytes;       // bytes of qrec (< 2^32 - 256: the traversal's buffer loads address it with 32-bit offsets)
    uint32_t qroot;            // TLAS root in the records
    uint32_t root;
    uint32_t n_prims;
    uint32_t n_nodes;
    const uint4* tri;          // i0, i1, i2, flags
    const float* positions;    // 3 per vertex
    const float* normals;
    const float* uvs;          // 2 per vertex
    const float* tangents;
    const DevTriShade* tshade;  // shading records per primitive slot (a triangle slot: its vertices x, y, z)
    const DevAlpha* alpha;      // alpha records of the alpha-tested triangles (alpha_index)
    const uint32_t* amask;      // their coverage mask sets (pt_alpha_cov.h)
    const pt_quad* quads;
    const pt_sphere* spheres;
    const pt_material* materials;
    const pt_texture* textures;
    const pt_image* images;
    const uint8_t* texels;
    uint64_t n_texel_bytes;
    const pt_light* lights;
    const DevLightTri* ltri;    // per light: its triangle (DevLightTri), valid for triangle area lights
    uint32_t n_lights;
    uint32_t light_sampler;
    const uint32_t* sampler_lights;
    const float* sampler_cdf;  // running float sums (PowerLightSampler::Sample order)
    const uint32_t* sampler_guide;  // PT_LS_GUIDE + 1 search starts over sampler_cdf (ls_sample)
    uint32_t n_sampler_lights;
    float sampler_total;
    const uint32_t* infinite_lights;
    uint32_t n_infinite_lights;
    const float* light_dist;  // TEX_INF cell running sums
    const pt_medium* media;
    uint32_t n_media;
    int32_t scene_medium;
    const DevInstance* instances;
    uint32_t n_instances;
    // motion blur (a shutter camera's frame over a scene with an
    // AnimatedPrimitive): rays carry a time (PathSoA::time, sq_time[shadow
    // record]) and animated instances are rebuilt at it; else 0 / null
    uint32_t motion;
    float* sq_time;
    uint32_t* scratch;       // SCR_WORDS x scratch_lanes (instance traversal state)
    uint32_t scratch_lanes;
    uint32_t* stack_drops;   // traversal pushes past the stack capacity (counted, rare)
    uint32_t* tie_drops;     // exact-tie list entries past its capacity (counted; none expected)
    uint32_t n_materials, n_textures, n_images;
};

// The uploaded scene of the current context, in constant memory: every
// device function reads it directly (no per-lane copy of the struct, and the
// array pointers come from scalar loads).  The runtime re-sends it before a
// launch whenever another context last used the device (pt_runtime.hip).
__constant__ DevScene S;

// ------------------------------------------------------------------ float3 helpers
struct f3 {
    float x, y, z;
};
__device__ __forceinline__ f3 F3(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 ld3(const float* p) { return f3{p[0], p[1], p[2]}; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return F3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return F3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 operator*(f3 a, f3 b) { return F3(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ f3 operator*(f3 a, float s) { return F3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ f3 operator*(float s, f3 a) { return F3(s * a.x, s * a.y, s * a.z); }
__device__ __forceinline__ f3 operator/(f3 a, float s) { return F3(a.x / s, a.y / s, a.z / s); }
__device__ __forceinline__ f3 operator-(f3 a) { return F3(-a.x, -a.y, -a.z); }
// Float semantics: the device is compiled with -ffp-contract=off and every
// fused multiply-add the reference's GCC build emits is spelled out with fma_
// at the same site (read from the reference's optimized GIMPLE,
// tools/refgimple.py; DESIGN.md "Numerics"); everything else rounds each
// operation.  The oracle (oracle/pt_oracle.c, also contract-off) writes the
// same expressions, so device and oracle agree bit for bit, and both with the
// reference.  rmul() marks a product that must stay rounded.
__device__ __forceinline__ float fma_(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
__device__ __forceinline__ float rmul(float a, float b) {
    float m = a * b;
    __asm__ volatile("" : "+v"(m));  // opaque to contraction: stays a rounded product
    return m;
}
// glm::dot: x product rounded, then fma(y), fma(z)
__device__ __forceinline__ float dot(f3 a, f3 b) { return fma_(a.z, b.z, fma_(a.y, b.y, rmul(a.x, b.x))); }
// the other orders the build emits: y product rounded, then fma(x), fma(z);
// and the unfused (x + y) + z
__device__ __forceinline__ float dot_yxz(f3 a, f3 b) { return fma_(a.z, b.z, fma_(a.x, b.x, rmul(a.y, b.y))); }
__device__ __forceinline__ float dot_p(f3 a, f3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
// glm::cross in scalar code: first product fused, second rounded
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
    return F3(fma_(a.y, b.z, -rmul(b.y, a.z)), fma_(a.z, b.x, -rmul(b.z, a.x)), fma_(a.x, b.y, -rmul(b.x, a.y)));
}
// every lane first product rounded, second fused (QuadShape::Area)
__device__ __forceinline__ f3 cross_r(f3 a, f3 b) {
    return F3(fma_(-b.y, a.z, rmul(a.y, b.z)), fma_(-b.z, a.x, rmul(a.z, b.x)), fma_(-b.x, a.y, rmul(a.x, b.y)));
}
// glm::cross where the reference build vectorises x, y (first product rounded,
// second fused) and keeps z scalar (first fused): triangle normals, onb(si)
__device__ __forceinline__ f3 cross_v(f3 a, f3 b) {
    return F3(fma_(-b.y, a.z, rmul(a.y, b.z)), fma_(-b.z, a.x, rmul(a.z, b.x)), fma_(a.x, b.y, -rmul(b.x, a.y)));
}
// u*a + v*b + w*c of glm vectors: first product rounded, the others fused
__device__ __forceinline__ float lerp3f(float u, float a, float v, float b, float w, float c) {
    return fma_(w, c, fma_(v, b, rmul(u, a)));
}
// a*b + c per lane, fused (glm's `c += a * b` as the reference build contracts it)
__device__ __forceinline__ f3 fma3(f3 a, f3 b, f3 c) { return F3(fma_(a.x, b.x, c.x), fma_(a.y, b.y, c.y), fma_(a.z, b.z, c.z)); }
__device__ __forceinline__ f3 fma3s(float s, f3 b, f3 c) { return F3(fma_(s, b.x, c.x), fma_(s, b.y, c.y), fma_(s, b.z, c.z)); }
// ray.at(t) fused in every lane
__device__ __forceinline__ f3 at_f(f3 o, f3 d, float t) { return F3(fma_(t, d.x, o.x), fma_(t, d.y, o.y), fma_(t, d.z, o.z)); }
__device__ __forceinline__ float csqrt(float x) { return __builtin_sqrtf(x); }
// sinf / cosf: the host libm's algorithm, bit-identical (pt_sincosf.h)
#define PT_SC_FN __device__ __forceinline__ static
#define PT_SC_FMA __builtin_fma
#include "pt_sincosf.h"
__constant__ const double pt_sc_table[2][14] = PT_SC_TABLE;
__device__ __forceinline__ float cos_cr(float x) { return pt_cosf_t(x, pt_sc_table); }
__device__ __forceinline__ float sin_cr(float x) { return pt_sinf_t(x, pt_sc_table); }
// expf / powf / acosf / atan2f: the host libm's algorithms, bit-identical (pt_libmf.h)
#include "pt_libmf.h"
__constant__ const uint64_t pt_expf_table[32] = PT_EXPF_TABLE;
__constant__ const double pt_powf_log2_table[32] = PT_POWF_LOG2_TABLE;
__device__ __forceinline__ float pow_cr(float x, float y) { return pt_powf_t(x, y, pt_powf_log2_table, pt_expf_table); }
__device__ __forceinline__ float exp_cr(float x) { return pt_expf_t(x, pt_expf_table); }
__constant__ const double pt_log_table[256] = PT_LOG_TABLE;
__device__ __forceinline__ double log_cr(double x) { return pt_log_t(x, pt_log_table); }
__device__ __forceinline__ float length(f3 a) { return csqrt(dot(a, a)); }
__device__ __forceinline__ f3 normalize(f3 a) { return a * (1.0f / csqrt(dot(a, a))); }
__device__ __forceinline__ bool is_zero(f3 a) { return a.x == 0.0f && a.y == 0.0f && a.z == 0.0f; }
__device__ __forceinline__ f3 reflect(f3 I, f3 N) { return I - (N * dot(N, I)) * 2.0f; }
// glm::refract with the build's contractions, given d = dot(N, I)
__device__ __forceinline__ f3 refract_f(f3 I, f3 N, float eta, float d) {
    const float k = fma_(-(eta * eta), fma_(-d, d, 1.0f), 1.0f);
    if (k >= 0.0f) {
        const float c = fma_(eta, d, csqrt(k));
        return F3(fma_(-c, N.x, eta * I.x), fma_(-c, N.y, eta * I.y), fma_(-c, N.z, eta * I.z));
    }
    return F3(0, 0, 0);
}
__device__ __forceinline__ float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }
__device__ __forceinline__ float smax(float a, float b) { return a < b ? b : a; }  // std::max
__device__ __forceinline__ f3 xyz(float4 v) { return F3(v.x, v.y, v.z); }

// ------------------------------------------------------------------ sample stream
__device__ __forceinline__ uint32_t pcg_hash(uint32_t v) {
    uint32_t state = v * 747796405u + 2891336453u;
    uint32_t word = ((state >> ((state >> 28u) + 4u)) ^ state) * 277803737u;
    return (word >> 22u) ^ word;
}
__device__ __forceinline__ uint32_t stream_key(uint32_t seed, uint32_t pixel, uint32_t sample) {
    return pcg_hash(pcg_hash(seed ^ pcg_hash(pixel)) + sample);
}
__device__ __forceinline__ float draw(uint32_t key, uint32_t dim) {
    return (float)(pcg_hash(key + 0x9E3779B9u * dim) >> 8) * (1.0f / 16777216.0f);
}
