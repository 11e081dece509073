/*
 * pt_api.h — C ABI of the MI355X wavefront path tracer (libpt_hip.so).
 *
 * This is the drop-in boundary for the reference's per-sample loop
 * (marko176/PathTracing).  The reference's `Integrator` interface
 * (Integrators.hpp:10-23: Render(threadCount), Li(Ray)) sits on top of it: a
 * host-side `HipPathIntegrator` flattens the already-built Scene (TLAS4/BLAS4
 * cluster arrays BVH.hpp:1214-1216, primitives, materials, lights, light
 * sampler, camera, film filter) into a pt_scene_desc once, then every
 * Render() becomes one pt_render().  Scene build, model loading and image
 * output stay on the host.  See INTEGRATION.md.
 *
 * Plain pointers and sizes only; no C++ or torch types.  Every call returns a
 * pt_status (0 = OK, < 0 = error, message via pt_last_error); nothing aborts.
 * All host arrays are read during the call and copied to device memory; no
 * pointer is retained after return.
 */
#ifndef PT_API_H
#define PT_API_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* v8: pt_stats.tie_overflows (was padding), pt_anim_inverse_cases
 * v9: pt_alpha_coverage */
#define PT_API_VERSION 9

typedef int32_t pt_status;
#define PT_OK 0
#define PT_ERR_ARG (-1)     /* invalid argument / inconsistent scene       */
#define PT_ERR_HIP (-2)     /* HIP runtime error                            */
#define PT_ERR_OOM (-3)     /* device allocation failed                     */
#define PT_ERR_STATE (-4)   /* call order (e.g. render before upload)       */
#define PT_ERR_NODEV (-5)   /* no HIP device                                */
#define PT_ERR_COMM (-6)    /* RCCL communicator error                      */

/* ------------------------------------------------------------------------ */
/* Reference-form BVH4 (BVH.hpp:38-60), byte-identical to BVH4_NODE /        */
/* BVH4_CLUSTER.  pt_bvh4_build reproduces BVHBase::BuildBaseThreaded        */
/* (BVH.hpp:290-390) + BVH4::buildBVH4 (788-1017).                            */
/* ------------------------------------------------------------------------ */
typedef struct pt_ref_bvh4_node {
    uint8_t count;        /* leaf: primitive count (u8, as the reference)     */
    uint8_t active;       /* 0 => leaf                                        */
    uint8_t perm;         /* topology/axis code, index into the octant LUT    */
    uint8_t pad;
    uint32_t cluster_idx; /* leaf: first primitive, else cluster index        */
} pt_ref_bvh4_node;

typedef struct pt_ref_bvh4_cluster {
    float xmin[4], xmax[4];
    float ymin[4], ymax[4];
    float zmin[4], zmax[4];
    pt_ref_bvh4_node children[4];
} pt_ref_bvh4_cluster; /* 128 bytes */

/* boxes: n x {minx,miny,minz,maxx,maxy,maxz}.  clusters must hold >= max(n,1)
 * entries.  prim_order[i] = input index of the i-th primitive in leaf order.
 * bbox (optional, 6 floats) receives the root box. */
pt_status pt_bvh4_build(const float* boxes, uint32_t n, pt_ref_bvh4_cluster* clusters, uint32_t* n_clusters,
                        pt_ref_bvh4_node* root, uint32_t* prim_order, float* bbox);

/* glm::inverse(mat4) as the reference build computes TransformedPrimitive's
 * invTransform (Primitive.hpp:37), host-side; column-major m[c*4+r]. */
pt_status pt_mat4_inverse(const float* m, float* out);

/* The octant traversal order byte for (ray-sign octant, perm) exactly as
 * BVH4::LUT / PermToIndexLUT (BVH.hpp:10-24, 562-718): 2-bit child slots,
 * most significant = nearest.  out: 8*135 bytes. */
pt_status pt_bvh4_order_table(uint8_t* out);

/* ------------------------------------------------------------------------ */
/* Flat scene                                                                */
/* ------------------------------------------------------------------------ */
enum { PT_PRIM_TRIANGLE = 0, PT_PRIM_QUAD = 1, PT_PRIM_SPHERE = 2, PT_PRIM_BLAS = 3, PT_PRIM_INSTANCE = 4 };

/* One GeometricPrimitive (Primitive.hpp:17-31) or a nested BLAS (a Model,
 * Model.hpp:25-31), indexed by its global leaf-order slot. */
typedef struct pt_prim {
    uint32_t kind;     /* PT_PRIM_*                                              */
    uint32_t index;    /* TRIANGLE: triangle id; QUAD: quad id; SPHERE: sphere id;
                          BLAS: index into pt_scene_desc.bvhs;
                          INSTANCE: index into pt_scene_desc.instances (TLAS only) */
    int32_t material;  /* -1 = none: medium boundary, rays pass through         */
    int32_t light;     /* area light id or -1                                    */
    int32_t medium;    /* inside medium of the boundary (MediumInterface), or -1:
                          GeometricInteraction::getMedium (Interaction.hpp:26-29),
                          used by VolPath only                                     */
} pt_prim;

/* TransformedPrimitive / AnimatedPrimitive (Primitive.hpp:34-66): a BLAS
 * (bvhs[bvh], a Model or a one-primitive BVH) under a glm::mat4 transform,
 * column-major m[col][row], and its glm::inverse.  A hit inside the instance
 * is reported as the virtual slot virt_base + (BLAS slot - prim_base); virtual
 * slots start at n_prims and the instances' ranges are ascending.
 *
 * Nested wrappers (a TransformedPrimitive / AnimatedPrimitive whose primitive
 * is itself one, Primitive.cpp:48-64, 86-89): `inner` chains the levels, the
 * outermost first.  inner = -1 ends the chain at bvhs[bvh]; otherwise it names
 * the next level down, an instance record with a larger index that no TLAS
 * slot references (a level record), at most PT_MAX_INSTANCE_DEPTH levels in
 * all.  Every record of a chain names the same bvh; a level record's
 * virt_base is unused.  Rays enter the levels outermost first (each level's
 * inverse, length and max * length in turn); hits leave innermost first
 * (t / length per level). */
#define PT_MAX_INSTANCE_DEPTH 4
typedef struct pt_instance {
    float transform[16];
    float inv[16];
    uint32_t bvh;
    uint32_t virt_base;
    /* AnimatedPrimitive (Primitive.hpp:52-66, Primitive.cpp:76-96): animated
     * != 0 translates by motion * t, t = clamp(time - t0, t0, t1) / (t1 - t0),
     * per ray at the ray's time; transform / inv hold the time-0 translation
     * (what a camera without a shutter sees) */
    float motion[3];
    float time_bounds[2];
    uint32_t animated;
    int32_t inner;       /* the next level down, or -1 (API v7)             */
} pt_instance;

typedef struct pt_bvh_desc {
    const pt_ref_bvh4_cluster* clusters;
    uint32_t n_clusters;
    pt_ref_bvh4_node root;
    uint32_t prim_base;  /* global slot of this BVH's primitive 0 (leaf order) */
    uint32_t n_prims;
} pt_bvh_desc;

/* QuadShape (Shape.hpp:118-171) with its ctor-derived fields. */
typedef struct pt_quad {
    float Q[3], u[3], v[3], normal[3], D, w[3];
} pt_quad;

typedef struct pt_sphere {
    float center[3], radius;
} pt_sphere;

enum { PT_TEX_SOLID = 0, PT_TEX_IMAGE = 1, PT_TEX_CHECKER = 2 };
/* SolidColor / ImageTexture / CheckerTexture (Texture.hpp:122-213). */
typedef struct pt_texture {
    uint32_t kind;
    float scale[3];      /* colorScale                                     */
    float value[3];      /* SOLID: albedo                                  */
    int32_t a, b;        /* CHECKER: children                              */
    float inv_scale[2];  /* CHECKER: 1/uvscale                             */
    int32_t image;       /* IMAGE: image id                                */
} pt_texture;

enum { PT_IMAGE_U8 = 0, PT_IMAGE_F32 = 1 };
typedef struct pt_image {
    uint64_t offset;     /* byte offset into pt_scene_desc.texels          */
    int32_t width, height, channels;
    int32_t format;      /* PT_IMAGE_U8 (Image: byte / 255) or PT_IMAGE_F32
                          * (FloatImage, Texture.hpp:70-103: float texels,
                          * offset 4-byte aligned)                          */
} pt_image;

enum { PT_MAT_DIFFUSE = 0, PT_MAT_DIELECTRIC = 1, PT_MAT_THIN = 2, PT_MAT_CONDUCTOR = 3 };
enum { PT_ALPHA_OPAQUE = 0, PT_ALPHA_BLEND = 1, PT_ALPHA_MASK = 2 };
/* MicrofacetDiffuse / MicrofacetDielectric / ThinDielectric / SpecularConductor
 * (Material.hpp:200-673).  Texture ids -1 = absent. */
typedef struct pt_material {
    uint32_t kind;
    int32_t tex, norm, rough, metal, alpha;
    uint32_t alpha_mode; /* effective AlphaTester mode (Material.hpp:176-198) */
    float alpha_cutoff;
    float ri;            /* DIELECTRIC / THIN                               */
    float albedo[3];     /* CONDUCTOR                                       */
} pt_material;

enum { PT_LIGHT_AREA = 0, PT_LIGHT_UNIFORM_INF = 1, PT_LIGHT_SKY_INF = 2, PT_LIGHT_DISTANT = 3, PT_LIGHT_POINT = 4,
       PT_LIGHT_TEX_INF = 5 };
/* TextureInfiniteLight's cell grid (Light.hpp:120-122): xSamples x ySamples */
#define PT_TEXINF_X 1920
#define PT_TEXINF_Y 1080
/* AreaLight / UniformInfiniteLight / FunctionInfiniteLight (sky gradient of
 * main.cpp:292-295, parameterised) / DistantLight / PointLight (Light.cpp). */
typedef struct pt_light {
    uint32_t kind;
    int32_t prim;        /* AREA: global prim slot of its shape             */
    int32_t tex;         /* AREA: emissive texture                          */
    uint32_t one_sided;
    float power;         /* Light::Power() after PreProcess                 */
    float pmf;           /* LightSampler::PMF(light)                        */
    float color[3];      /* UNIFORM/DISTANT/POINT colour; SKY: horizon c0   */
    float vec[3];        /* DISTANT dir; POINT position; SKY: zenith c1     */
    float scale;         /* SKY scale                                       */
    int32_t instance;    /* AREA: -1, or the instance whose transform moves
                          * the shape (TransformedLight / AnimatedLight,
                          * Light.cpp:300-364; prim is then the BLAS slot)  */
} pt_light;
/* TEX_INF (TextureInfiniteLight, Light.cpp:110-200): tex = its texture,
 * scale = LeScale, prim = offset of its PT_TEXINF_X*PT_TEXINF_Y running sums
 * (accWeights, float, std::partial_sum order) in pt_scene_desc.light_dist. */

enum { PT_LS_UNIFORM = 0, PT_LS_POWER = 1 };

/* HomogeneusMedium (Medium.hpp:14-61) after its ctor (density applied:
 * sigma_a = d*sa, sigma_s = d*ss, sigma_t = d*(sa+ss), Le = Le*LeDensity) with
 * its HenyeyGreenstein phase function (PhaseFunction.hpp:17-27, g clamped to
 * [-0.99, 0.99]). */
typedef struct pt_medium {
    float sigma_a[3], sigma_s[3], sigma_t[3];
    float Le[3];
    float g;
} pt_medium;

typedef struct pt_scene_desc {
    /* triangle meshes, global arrays */
    const float* positions;      /* 3 * n_vertices */
    const float* normals;        /* 3 * n_vertices */
    const float* uvs;            /* 2 * n_vertices */
    const float* tangents;       /* 3 * n_vertices (zeros where a mesh has none) */
    uint32_t n_vertices;
    const uint32_t* tri_vidx;    /* 3 * n_triangles */
    const uint32_t* tri_flags;   /* n_triangles: bit0 = mesh has tangents */
    uint32_t n_triangles;
    const pt_quad* quads;
    uint32_t n_quads;
    const pt_sphere* spheres;
    uint32_t n_spheres;
    /* primitives in global leaf-order slots; bvhs[0] is the TLAS */
    const pt_prim* prims;
    uint32_t n_prims;
    const pt_bvh_desc* bvhs;
    uint32_t n_bvhs;
    /* appearance */
    const pt_material* materials;
    uint32_t n_materials;
    const pt_texture* textures;
    uint32_t n_textures;
    const pt_image* images;
    uint32_t n_images;
    const uint8_t* texels;
    uint64_t n_texel_bytes;
    /* lights */
    const pt_light* lights;
    uint32_t n_lights;
    uint32_t light_sampler;          /* PT_LS_*                                 */
    const uint32_t* sampler_lights;  /* lights the sampler draws from, in order */
    uint32_t n_sampler_lights;
    const uint32_t* infinite_lights; /* Scene::infiniteLights, in order         */
    uint32_t n_infinite_lights;
    const float* light_dist;         /* TEX_INF lights' cell running sums       */
    uint64_t n_light_dist;
    /* participating media (VolPath): pt_prim.medium and the ids below index it */
    const pt_medium* media;
    uint32_t n_media;
    int32_t scene_medium;            /* Scene::GetMedium() (Scene.hpp:26), or -1 */
    /* instances (TLAS slots of kind PT_PRIM_INSTANCE index it) */
    const pt_instance* instances;
    uint32_t n_instances;
} pt_scene_desc;

/* Camera (Camera.hpp:7-35) after its ctor. */
typedef struct pt_camera_desc {
    float origin[3];
    float u[3], v[3], w[3];
    float half_width, half_height;
    float defocus_radius, focus_distance, focus_angle;
    int32_t width, height;
    int32_t medium;      /* Camera::GetMedium() (Camera.hpp:41-47), or -1   */
    /* Camera(..., glm::vec2 shutterBounds) (Camera.hpp:16-19): rays carry
     * time = mix(shutter[0], shutter[1], u) with the sample's time draw
     * (Camera.hpp:25); has_shutter 0: time 0 (the other ctors leave the
     * bounds uninitialised) */
    float shutter[2];
    int32_t has_shutter;
} pt_camera_desc;

/* PathIntegrator / SimplePathIntegrator / VolPathIntegrator (Integrators.hpp:33-67) */
enum { PT_INTEGRATOR_PATH = 0, PT_INTEGRATOR_SIMPLE = 1, PT_INTEGRATOR_VOLPATH = 2 };
enum { PT_FILTER_MITCHELL = 0, PT_FILTER_BOX = 1, PT_FILTER_GAUSSIAN = 2, PT_FILTER_LANCZOS = 3 };
#define PT_RENDER_COUNT_NODES 0x1u  /* instrumented traversal: node/tri counts */
#define PT_RENDER_TIMING 0x2u       /* per-kernel HIP-event timing into stats   */
#define PT_RENDER_TRAVERSAL_POOL 0x4u   /* force the persistent refilling traversal */
#define PT_RENDER_TRAVERSAL_SIMPLE 0x8u /* force one ray per lane (default: by BVH size) */
#define PT_RENDER_NODES_FULL 0x10u      /* pool traversal over the 128-B reference clusters */
#define PT_RENDER_NODES_QUANTIZED 0x20u /* ... over the 64-B quantized nodes (the default)  */
#define PT_RENDER_ADAPTIVE 0x40u        /* pt_render: TileIntegrator::Render's adaptive rounds */
#define PT_RENDER_SORT_MATERIAL 0x80u   /* shade each bounce's paths binned by hit material */
#define PT_RENDER_SORT_SPATIAL 0x100u   /* ... binned by the hit point's cell (16^3 Morton grid);
                                         * the default for large scenes (pool traversal) */
#define PT_RENDER_NO_SORT 0x200u        /* no hit sort (shade in path order) */
#define PT_RENDER_SORT_RAYS 0x400u      /* trace closest-hit rays in origin-cell + octant order */
#define PT_RENDER_SERIAL_SHADOW 0x800u  /* any-hit rays of a bounce after it, on one stream     */
#define PT_RENDER_OVERLAP_SHADOW 0x1000u /* ... beside the next bounce's closest-hit rays, on a
                                         * second stream (pool traversal, no instances)    */
#define PT_RENDER_NO_TAIL 0x2000u       /* no tail kernel: every bounce a wavefront iteration
                                          (default: the last bounces of a fixed-SPP Path /
                                          SimplePath chunk finish in one launch, k_tail) */
#define PT_RENDER_ANY_STACKLESS 0x4000u /* NEE any-hit rays through the stackless traversal
                                          (escape links, no stack; quantized records
                                          without instances, else ignored) */

typedef struct pt_render_desc {
    uint32_t integrator;       /* PT_INTEGRATOR_*                               */
    uint32_t spp;              /* samples per pixel of the whole frame          */
    uint32_t max_depth;
    uint32_t seed;             /* sample-stream base seed                       */
    uint32_t filter;           /* PT_FILTER_*                                   */
    float filter_radius[2];
    double filter_params[2];   /* Mitchell b,c | Gaussian sigma | Lanczos tau and
                                  the host filter object's Integral() (the
                                  reference estimates it with unseeded jitter,
                                  Filter.hpp:130-143, so the caller passes it) */
    uint32_t shard_index;      /* this call renders samples s with             */
    uint32_t shard_count;      /*   s % shard_count == shard_index              */
    uint32_t flags;            /* PT_RENDER_*                                   */
    uint32_t paths_in_flight;  /* wavefront size; 0 = library default           */
    uint32_t pixel_begin;      /* render pixels [pixel_begin, pixel_end) only;  */
    uint32_t pixel_end;        /*   0,0 = whole film                            */
    /* A StratifiedSampler(xSamples, ySamples) host (Sampler.hpp:73-151):
     * strata[0] * strata[1] == spp stratifies the camera draws of Render's
     * per-thread clone (pixel, time, lens; Integrators.cpp:39, 61-64) --
     * stratum PermutationElement(i, spp, Hash(px, py, dimension)) of sample
     * index i within the pixel's round (Util.hpp:45-73, 160-168), jittered
     * by the stream's draw; 0,0 = the plain stream */
    uint32_t strata[2];
} pt_render_desc;

typedef struct pt_stats {
    uint64_t paths;            /* camera samples traced                         */
    uint64_t rays_closest;     /* Scene::Intersect calls                        */
    uint64_t rays_any;         /* Scene::IntersectPred calls                    */
    uint64_t nodes_closest, tris_closest, nodes_any, tris_any; /* COUNT_NODES   */
    uint64_t shade_hits;       /* closest hits shaded                           */
    double ms_total;           /* host wall time of pt_render                   */
    double ms_closest;         /* TIMING: summed closest-hit kernel time        */
    double ms_any;             /* TIMING: summed any-hit kernel time            */
    double ms_shade;           /* TIMING: summed shade kernel time              */
    uint64_t launches_closest;
    uint64_t launches_any;
    uint64_t stack_overflows;  /* traversal stack pushes beyond the stack's
                                  capacity (dropped; the test suite asserts 0) */
    uint32_t n_devices;        /* devices that rendered                         */
    uint32_t tie_overflows;    /* exact-t tie re-trace list entries dropped past
                                  its capacity (a dropped tie could change which
                                  primitive wins, Shape.cpp:204; the test suite
                                  and bench's frame check assert 0)            */
} pt_stats;

/* Rays for the pt_trace test hook (Scene::Intersect / IntersectPred). */
typedef struct pt_ray {
    float o[3], d[3], tmax;
    float time;          /* Ray::time (Ray.hpp:30): AnimatedPrimitive's      */
} pt_ray;

typedef struct pt_hit {
    float t, b1, b2;           /* t; barycentrics (tri) or quad alpha/beta     */
    int32_t prim;              /* global slot or -1 (any-hit: 1/0 in prim)     */
} pt_hit;

typedef struct pt_ctx pt_ctx;

int pt_version(void);
/* A context over n_devices GPUs (device_ids: n_devices HIP device indices,
 * NULL = 0 .. n_devices-1).  It owns per device the scene replica, wavefront
 * buffers and streams, and for n_devices > 1 one RCCL communicator per device
 * (ncclCommInitAll).  pt_render / pt_render_adaptive then shard the frame over
 * the devices (one host thread per device: interleaved samples at fixed SPP,
 * 32x32 tiles when adaptive) and reduce the per-device films with
 * ncclReduce(ncclSum) onto the first device before the result reaches
 * film_accum -- the reference's Film::Merge of atomic<double> adds
 * (Film.hpp:125-132, 244-253) called from TileIntegrator::Render
 * (Integrators.cpp:112).  Test hooks run on the first device. */
pt_status pt_create(pt_ctx** ctx, int n_devices, const int* device_ids);
int pt_device_count(const pt_ctx* ctx);
/* Multi-process form of the film reduce (one process per GPU, e.g. under
 * torch.distributed): rank 0 draws an id (PT_COMM_ID_BYTES bytes), the host
 * broadcasts it, every rank joins with its rank; pt_film_reduce then sums
 * n doubles of device memory film (on the context's first device) over the
 * ranks onto `root` (ncclReduce, in place, on the context's stream; blocks).
 * A 1-rank communicator is valid (the reduce is then the identity). */
#define PT_COMM_ID_BYTES 128
pt_status pt_comm_unique_id(uint8_t* id_out);
pt_status pt_comm_init_rank(pt_ctx* ctx, int n_ranks, int rank, const uint8_t* id);
pt_status pt_film_reduce(pt_ctx* ctx, double* film, uint64_t n, int root);
/* pt_comm_init_rank joins without blocking past PT_COMM_TIMEOUT_S seconds
 * (env, default 120): if the other ranks never join it aborts and returns
 * PT_ERR_COMM.  pt_comm_destroy drops the per-process communicator
 * (ncclCommAbort), e.g. when the ranks disagree on the reduce path, so that
 * pt_comm_init_rank can run again.  Not for multi-device contexts. */
pt_status pt_comm_destroy(pt_ctx* ctx);
void pt_destroy(pt_ctx* ctx);
const char* pt_last_error(const pt_ctx* ctx);   /* ctx may be NULL          */
pt_status pt_set_stream(pt_ctx* ctx, void* hip_stream); /* NULL = ctx stream */
/* Node format of the persistent (pool) traversal: the reference's 128-B
 * clusters, or a 64-B copy with 8-bit child boxes quantized outward (every
 * child the reference's slab test accepts is accepted, so the closest hit
 * is the same).  AUTO = quantized where the scene can be encoded.  Applies
 * to pt_trace and is the default of pt_render (overridden by its flags). */
enum { PT_NODES_AUTO = 0, PT_NODES_FULL = 1, PT_NODES_QUANTIZED = 2 };
pt_status pt_set_node_format(pt_ctx* ctx, int format);
pt_status pt_scene_upload(pt_ctx* ctx, const pt_scene_desc* scene);
/* Accumulates W*H*4 doubles {sum R*w, sum G*w, sum B*w, sum w} (Film.hpp:227-253)
 * into film_accum, a host or a device pointer (detected). */
pt_status pt_render(pt_ctx* ctx, const pt_camera_desc* cam, const pt_render_desc* rd, double* film_accum,
                    pt_stats* stats);
/* TileIntegrator::Render's adaptive sampling (Integrators.cpp:55-86,
 * Util.hpp:8-43): each pixel renders rounds of spp samples (round r = stream
 * samples r*spp .. r*spp+spp-1) until the relative variance of all three
 * luminance-weighted channels is <= 1.5 or it has 128*spp samples; every
 * sample is splatted into film_accum as in pt_render.  sample_counts (NULL,
 * or W*H u32, host or device) receives each pixel's sample count (0 for
 * pixels outside this call's work).  pixel_begin/end select the work pixels;
 * shard_count > 1 splits the frame by 32x32 tiles (tile % shard_count ==
 * shard_index; Integrators.cpp:33), so each pixel's rounds run on one shard.
 * pt_render with PT_RENDER_ADAPTIVE is this call with sample_counts NULL. */
pt_status pt_render_adaptive(pt_ctx* ctx, const pt_camera_desc* cam, const pt_render_desc* rd, double* film_accum,
                             uint32_t* sample_counts, pt_stats* stats);
/* Per-sample radiance of pixels [pixel_begin, pixel_end) (0,0 = all), samples
 * [0, spp): out_L[((pix - pixel_begin) * spp + s) * 3] (host pointer).  The
 * unfiltered Integrator::Li values behind pt_render; for parity tests. */
pt_status pt_render_samples(pt_ctx* ctx, const pt_camera_desc* cam, const pt_render_desc* rd, float* out_L,
                            pt_stats* stats);
/* Check hook of the last fixed-SPP pt_render on this context (first device):
 * the per-sample radiance that frame splatted into the film, for n (pixel,
 * sample) pairs -- pixel = y*width + x, sample = the frame's sample index s
 * (this shard's: s % shard_count == shard_index) -- into out_L[3*i]
 * (host pointers).  The frame's last sample chunk is kept on the device until
 * the next render of any kind; PT_ERR_STATE when there is none, PT_ERR_ARG for
 * a sample outside it.  The unfiltered Integrator::Li values (Integrators.cpp:
 * 131-257) of the exact frame bench.py times. */
pt_status pt_frame_samples(pt_ctx* ctx, const uint32_t* pixels, const uint32_t* samples, uint32_t n, float* out_L);
/* The frame sample indices pt_frame_samples can serve: this shard's samples
 * s with first <= s <= last (s % shard_count == shard_index), the frame's last
 * sample chunk; PT_ERR_STATE when there is no fixed-SPP frame. */
pt_status pt_frame_sample_range(const pt_ctx* ctx, uint32_t* first, uint32_t* last);
/* Test hook: rays and hits are host or device pointers (detected).  any_hit:
 * 0 closest hit, 1 any hit, 2 any hit through the stackless traversal
 * (PT_RENDER_ANY_STACKLESS; PT_ERR_ARG on a scene without quantized records
 * or with instances). */
pt_status pt_trace(pt_ctx* ctx, const pt_ray* rays, uint32_t n, int any_hit, pt_hit* hits, pt_stats* stats);
/* Test hook: closest hit + the SurfaceInteraction the renderer reconstructs
 * (TriangleShape/QuadShape/SphereShape::Intersect incl. sample_normalMap,
 * Shape.cpp:3-359): out[16*i] = {hit, t, p[3], n[3], ns[3], uv[2], tangent[3]}
 * (zeros on a miss).  Host pointers. */
pt_status pt_interact(pt_ctx* ctx, const pt_ray* rays, uint32_t n, float* out);
/* Test hook: Material::scatter + calc_attenuation + PDF (Material.hpp) of
 * material `material` on n cases of 27 floats {ray o[3], d[3], p[3], n[3],
 * ns[3], tangent[3], uv[2], t, u, uv_sample[2], other_dir[3]} ->
 * 20 floats {ok, f[3], pdf, flags, o[3], d[3], f(d)[3], pdf(d), f(other)[3],
 * pdf(other)}.  Host pointers. */
pt_status pt_bsdf_cases(pt_ctx* ctx, int32_t material, const float* cases, uint32_t n, float* out);
/* Test hook: Light::sample(uv) + PDF + L (Light.cpp) for every light and
 * n cases of 5 floats {uv[2], reference point[3]} -> n_lights*n records of
 * 18 floats {L[3], p[3], n[3], uv[2], dir[3], pdf, L(p)[3]}.  Host pointers. */
pt_status pt_light_cases(pt_ctx* ctx, const float* cases, uint32_t n, float* out);
/* Test hook: LightSampler::Sample(u) (LightSampler.cpp:7-11, 34-46; replaces
 * the reference's in-Li call at Integrators.cpp:262) for n draws u ->
 * the picked light's index into pt_scene_desc.lights, -1 when the sampler
 * is empty.  Host pointers. */
pt_status pt_light_picks(pt_ctx* ctx, const float* u, uint32_t n, int32_t* out);
/* Test hook: the device's inverse of an AnimatedPrimitive's matrix at a ray's
 * time (AnimatedPrimitive::Intersect -> TransformedPrimitive's ctor ->
 * glm::inverse, Primitive.cpp:82-89, Primitive.hpp:37), for n translations
 * (3 floats each; the matrix is identity + that translation, as the device
 * builds it: components never -0) -> n glm column-major 4x4 matrices (16
 * floats).  Host pointers.  Needs a context, not a scene. */
pt_status pt_anim_inverse_cases(pt_ctx* ctx, const float* translations, uint32_t n, float* out);
/* Check hook, host code (no device): the conservative alpha coverage masks
 * pt_scene_upload stores with each alpha-tested triangle, replacing no
 * reference interface (the reference runs Material::Alpha, Material.hpp:
 * 181-198, on every candidate hit).  A cell of the triangle's n x n
 * barycentric subdivision (n = 4 ... 128 from its texel extent) is "accept"
 * when every hit in it passes the alpha test and "reject" when every hit
 * fails.  Per primitive slot, 1025 words: the set handle (word offset |
 * log2(n / 4) << 29; 0xFFFFFFFF: no set -- no alpha test, or nothing
 * decided), 512 words of accept mask, 512 of reject mask (cell c: bit c % 32
 * of word c / 32; max(1, n n / 32) words used).  out: 1025 * n_prims words. */
pt_status pt_alpha_coverage(const pt_scene_desc* scene, uint32_t* out);
/* Film resolve (Film::WritePNG / WritePPM, Film.hpp:154-217): per pixel
 * color = sum RGB*w / sum w, the tone mapper (through the writers'
 * std::function<vec3(vec3)>, i.e. in float around a double body),
 * linear_to_sRGB (Texture.hpp:13-17) and 255.999*clamp(., 0, 1) truncated to
 * u8.  rgb_out: width*height*3 bytes, row y = film row y (the PNG writer's
 * buffer; the files are written bottom row first).  film_accum / rgb_out are
 * host or device pointers (detected).  Needs a context, not a scene. */
enum { PT_TONEMAP_REINHARD_JODIE = 0, PT_TONEMAP_ACES = 1 };
pt_status pt_film_resolve(pt_ctx* ctx, const double* film_accum, int32_t width, int32_t height, uint32_t tonemap,
                          uint8_t* rgb_out);
/* TextureInfiniteLight::PreProcess's cell weights (Light.cpp:150-196) for a
 * FloatImageTexture environment (float texels, w x h x channels, row 0
 * first, colorScale), LeScale le_scale: per cell k of the 1920 x 1080 grid
 * (the reference's indexing: x = k % 1080, y = k / 1080) the mean luminance
 * of Le over 8 x 8 jittered strata, jitter from a fixed counter-based hash
 * (the reference's StratifiedSampler jitter is unseeded).  Host code, up to
 * `threads` threads; weights: PT_TEXINF_X*PT_TEXINF_Y floats. */
pt_status pt_texinf_weights(const float* texels, int32_t width, int32_t height, int32_t channels,
                            const float color_scale[3], float le_scale, float* weights, int32_t threads);
/* Device bytes held by the uploaded scene. */
uint64_t pt_scene_device_bytes(const pt_ctx* ctx);

/* Device BVH build on the context's GPU: the same
 * BVHBase::BuildBaseThreaded binned SAH (BVH.hpp:290-390) as pt_bvh4_build,
 * level-synchronous on the device (binning, SAH decision, std::partition's
 * exact permutation), small subtrees one per lane, then the BVH4 collapse
 * (BVH.hpp:788-1017) level by level.  Same arguments and byte-identical outputs
 * as pt_bvh4_build; boxes are host memory.  stats may be NULL. */
typedef struct pt_bvh_build_stats {
    double ms_total;     /* host wall time of the call                     */
    double ms_device;    /* upload + device build + download (HIP events) */
    double ms_collapse;  /* BVH4 collapse + cluster download (HIP events)  */
    uint32_t levels;     /* level-synchronous passes                       */
    uint32_t small_tasks;/* subtrees finished one per lane                 */
    uint32_t nodes;      /* binary nodes                                   */
    uint32_t pad;
} pt_bvh_build_stats;
pt_status pt_bvh4_build_device(pt_ctx* ctx, const float* boxes, uint32_t n, pt_ref_bvh4_cluster* clusters,
                               uint32_t* n_clusters, pt_ref_bvh4_node* root, uint32_t* prim_order, float* bbox,
                               pt_bvh_build_stats* stats);

#ifdef __cplusplus
}
#endif
#endif /* PT_API_H */
