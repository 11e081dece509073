// Shared declarations between the wavefront kernels and the host runtime.
#pragma once
#include "pt_pool.h"
#include "pt_medium.h"

// path flags (b.w): depth | rr_depth << 12 | spec
#define PF_DEPTH_MASK 0xFFFu
#define PF_RR_SHIFT 12
#define PF_SPEC (1u << 24)

// queue counters, each on its own 128-byte line (one word saturates at
// ~88 atomics/us: MI355X_MICROARCH.md "dequeue"); appends are aggregated per
// block so a launch issues one atomic per block per counter
#define Q_STRIDE 32
#define Q_NEXT 0                 // continuing paths, appended from the front
#define Q_SHADOW (1 * Q_STRIDE)  // shadow rays
#define Q_NEW (2 * Q_STRIDE)     // new camera paths, appended from the back
#define Q_WORDS (3 * Q_STRIDE)
// one counter set: the queue counts an iteration produces, then the pools its
// two traversals claim rays from.  The runtime rotates three sets: iteration i
// reads its input count from set i % 3 (written by iteration i - 1), appends
// into set (i + 1) % 3 and zeroes set (i + 2) % 3 for iteration i + 1.
#define Q_TIES (Q_WORDS + 2 * PT_POOL_WORDS)  // closest-hit rays met an exact-t tie (k_closest_ties)
#define Q_NEE (Q_TIES + Q_STRIDE)  // NEE jobs of a split bounce (PT_SHADE_SPLIT: k_shade -> k_shade_nee)
#define SET_WORDS (Q_NEE + Q_STRIDE)
// host snapshot slot (pinned, written by the iteration prologue)
#define SNAP_PATHS 0        // paths entering the iteration
#define SNAP_SHADOW_PREV 1  // shadow rays of the previous iteration
#define SNAP_NEW 2          // camera paths the previous iteration started
#define SNAP_WORDS 16

// 64-bit work counters
#define CNT_NODES_CLOSEST 0
#define CNT_TRIS_CLOSEST 1
#define CNT_NODES_ANY 2
#define CNT_TRIS_ANY 3
#define CNT_NEXT_SAMPLE 4
#define CNT_EXTRA_ANY 5  // VolPath: shadow-ray continuations past medium boundaries
#define CNT_TAIL_CLOSEST 6  // k_tail: closest-hit queries (Scene::Intersect) it traced
#define CNT_TAIL_ANY 7      // k_tail: NEE queries (Scene::IntersectPred) it traced
#define CNT_COUNT 8
#define CNT_SHARDS 64  // work counters are sharded by block to avoid a hot line

// Compacted path state: the live paths of one bounce occupy entries
// [0, n) of these arrays, so every kernel reads and writes them coalesced
// (lane i <-> entry i; appends are contiguous per wave).  64 B per path.
// Continuing paths fill entries [0, c) from the front and new camera paths
// [cap - r, cap) from the back, so camera rays stay in coherent waves of their
// own; path i of an iteration (i < c + r) lives at path_slot(i).
// {o, d} and {beta, L} are two 32-B records per path: the ray's readers (the
// traversal's claim) read their 32 B, the shading two sectors per path
// (random 16-B reads fetch 64 B each: profiles/r03_fetch_calib.json).  One
// 64-B record or one array per field measured slower
// (profiles/r05_ab_path_aos.txt); so did 1/d carried with the ray (C4 -0.4 %,
// profiles/r05_ab_path_inv.txt).
#define PT_PATH_STRIDE 2u
struct PField {  // one float4 field of the path state, indexed by entry
    float4* p;
    __device__ __forceinline__ float4& operator[](uint32_t e) const { return p[(size_t)e * PT_PATH_STRIDE]; }
};
struct PathSoA {
    PField o;     // origin.xyz, stream key (bits)
    PField d;     // direction.xyz, flags (bits): depth | rr << 12 | spec
    PField beta;  // attenuation.xyz, prevPDF
    PField L;     // radiance so far .xyz, next draw dimension (bits)
    uint32_t* sid;// sample id within the chunk
    uint32_t cap; // entries
    float* time;  // the path's ray time (Ray::time, constant along a path: every
                  // scatter copies it, Material.hpp:264 ...); only with S.motion
};
__device__ __forceinline__ uint32_t path_count(const uint32_t* set) { return set[Q_NEXT] + set[Q_NEW]; }
__device__ __forceinline__ uint32_t path_slot(uint32_t i, uint32_t c, uint32_t cap) {
    return i < c ? i : cap - 1u - (i - c);
}

// A deferred NEE ray.  The unoccluded contribution is added as
// out = fma(c, att, out), the reference's `output += att * SampleLd(...)` as
// its build contracts it (Integrators.cpp:239), so c and att travel apart.
struct ShadowRec {
    float4 o;  // origin, tmax
    float4 d;  // direction, target (bits): entry in next state, or DONE_BIT|entry in done list
    float4 c;  // SampleLd's value if unoccluded
    float4 a;  // the path's attenuation
};
// VolPath's: SampleLd's value is ((Tr * L) * f * w) / pdf (Integrators.cpp:
// 466-478), so its factors travel apart for Tr to multiply in first.
struct ShadowRecV {
    float4 o;  // origin, tmax
    float4 d;  // direction, target | SHADOW_MLE_BIT
    float4 L;  // light radiance, .w: the ray's medium (bits)
    float4 f;  // scattering value, .w: MIS weight (1 for delta lights)
    float4 a;  // the path's attenuation, .w: light pdf
};
#define SHADOW_DONE_BIT 0x80000000u
// medium interaction: the medium's Le is added after SampleLd's value
// (Integrators.cpp:356-357), occluded or not
#define SHADOW_MLE_BIT 0x40000000u

struct RenderParams {
    pt_camera_desc cam;
    uint32_t seed, max_depth;
    uint32_t shard_index, shard_count;
    uint32_t s_lo, s_hi;            // local sample range of this chunk
    uint32_t npix_work;             // pixels per sample index
    uint32_t tiled, tiles_x;
    uint32_t pixel_begin;
    const uint32_t* pix_list;       // adaptive rounds: work pixel i = pix_list[i] (linear id), else null
    const uint32_t* order;          // material sort: k_shade thread t shades path order[t], else t
    unsigned long long chunk_total; // npix_work * (s_hi - s_lo)
    uint32_t filter;
    int rad_x, rad_y;
    float frad[2];
    double fparam[2];
    double inv_integral;
    double gauss_x, gauss_y;
    uint32_t strata_x, strata_y;    // a StratifiedSampler host's camera strata (pt_render_desc::strata)
    uint2* nee_jobs;                // split bounce (PT_SHADE_SPLIT): {path index, shadow target} per NEE job
};
// PT_SHADE_SPLIT 1: PathIntegrator's bounce in two kernels, k_shade
// (interaction, emission, scatter, RR -> path state, + a NEE job) and
// k_shade_nee (the interaction again, SampleLd -> shadow record)
#ifndef PT_SHADE_SPLIT
#define PT_SHADE_SPLIT 0
#endif

template <bool COUNT, bool INST>
__global__ void k_closest(PathSoA P, const uint32_t* in, float4* hit, uint32_t* pool, uint32_t* ovf, uint32_t* spare,
                          uint32_t* snap, unsigned long long* counters, uint32_t* ties);
template <bool COUNT, bool INST, bool QN>
__global__ void k_closest_pool(PathSoA P, const uint32_t* in, float4* hit, uint32_t* pool, uint32_t* ovf,
                               uint32_t* spare, uint32_t* snap, unsigned long long* counters, uint32_t* ties);
// exact re-trace of the rays a pool kernel listed for exact-t ties (pt_pool.h)
template <bool INST>
__global__ void k_closest_ties(PathSoA P, const uint32_t* in, float4* hit, const uint32_t* pool, const uint32_t* ties);
template <bool COUNT, bool INST>
__global__ void k_shadow(PathSoA next, float* sample_L, ShadowRec* sq, const uint32_t* nptr, uint32_t* pool,
                         uint32_t* ovf, unsigned long long* counters);
template <bool COUNT, bool INST, bool QN>
__global__ void k_shadow_pool(PathSoA next, float* sample_L, ShadowRec* sq, const uint32_t* nptr,
                              uint32_t* pool, uint32_t* ovf, unsigned long long* counters);
template <bool COUNT>
__global__ void k_shadow_sl(PathSoA next, float* sample_L, ShadowRec* sq, const uint32_t* nptr, uint32_t* pool,
                            uint32_t* ovf, unsigned long long* counters);
__global__ void k_trace_rays_sl(const pt_ray* rays, uint32_t n, pt_hit* out, uint32_t* pool,
                                unsigned long long* counters);
template <int INTEGRATOR, bool INST, bool COUNT>
__global__ void k_tail(RenderParams R, PathSoA cur, const uint32_t* nptr, float* sample_L,
                       unsigned long long* counters);
template <int INTEGRATOR>
__global__ void k_shade(RenderParams R, PathSoA cur, const uint32_t* nptr, const float4* hit, PathSoA next,
                        float* sample_L, unsigned long long* next_sample, ShadowRec* sq, uint32_t* cnt);
__global__ void k_shade_nee(RenderParams R, PathSoA cur, const uint32_t* nptr, const float4* hit, ShadowRec* sq,
                            uint32_t* cnt);
__global__ void k_shade_vol(RenderParams R, PathSoA cur, const uint32_t* nptr, const float4* hit, PathSoA next,
                            float* sample_L, unsigned long long* next_sample, ShadowRecV* sq, uint32_t* cnt);
template <bool COUNT>
__global__ void k_shadow_tr(PathSoA next, float* sample_L, const ShadowRecV* sq, const uint32_t* nptr,
                            unsigned long long* counters);
__global__ void k_fill(RenderParams R, uint32_t n, PathSoA next, uint32_t* cnt, unsigned long long* next_sample);
__global__ void k_resolve(const double* film, uint32_t npx, uint32_t tonemap, uint8_t* rgb);
__global__ void k_frame_gather(const float* sample_L, const unsigned long long* idx, uint32_t n, float* out);
__global__ void k_tri_shade(const DevGeom* geom, const DevPrimInfo* info, const uint4* tri, const float* normals,
                            const float* uvs, const float* tangents,
                            uint32_t n, DevTriShade* out);
__global__ void k_gather(RenderParams R, const float* sample_L, double* film);

// Adaptive sampling (TileIntegrator::Render's per-pixel rounds,
// Integrators.cpp:59-86): three VarianceEstimators per pixel (Util.hpp:8-43)
struct AdaptEst {
    double mean[3], S[3];
};
#define PT_ADAPT_MAX_ROUNDS 128   // while (Samples() < 128 * samplesPerPixel)
#define PT_ADAPT_REL_VAR 1.5      // minRelativeVariance
// Hit-state binning of a bounce's paths before shading
// (PT_RENDER_SORT_MATERIAL / PT_RENDER_SORT_SPATIAL): counting sort into
// RenderParams::order.  Material: bin 0 = miss, 1 + material % 254, 255 for
// hits inside instances.  Spatial: the hit point's 16^3 Morton cell.
enum { PT_SORT_MATERIAL = 0, PT_SORT_SPATIAL = 1, PT_SORT_RAYS = 2 };
#define PT_SORT_BINS_MATERIAL 256
#ifndef PT_SORT_CELL_BITS
#define PT_SORT_CELL_BITS 4  // spatial sort: 2^bits cells per axis of the scene box
#endif
#define PT_SORT_BINS_SPATIAL (1 << (3 * PT_SORT_CELL_BITS))
// The spatial key is the hit primitive's centroid cell (a 2-B table built at
// upload, so k_sort_count reads the hit record alone, 16 B per path instead of
// the hit and the ray's 48: C4 +0.4 %, profiles/r05_ab_prim_cell.txt).  The
// hit point's cell (the key of scenes without the table), the hit slot's leaf
// range (-1.5 %, profiles/r04_ab_traversal.txt) and bins written by the
// traversal (-6.5 %, profiles/r05_ab_hitbins.txt) measured slower.
// blocks of the exact-tie re-trace (k_closest_ties, grid-stride over the
// listed rays): with 64 (a quarter of the CUs) it took 0.66 ms per C4 launch
#ifndef PT_TIE_BLOCKS
#define PT_TIE_BLOCKS 1024u
#endif
#ifndef PT_SHADE_BLOCK
// k_shade threads per block (its appends aggregate per block): C4 64 / 128 /
// 256 / 512 / 1024 -> 1206 / 1236 / 1270 / 1205 / 1278 Mrays/s
// (profiles/r02_ab_shade.txt).  r04, k_shade ms per frame on one box
// (gpurun_out/r4h): 1024 x 4 waves per SIMD 1372, 256 x 3 waves 1374,
// 512 x 3 waves 1713 (one block per CU: 2 waves per SIMD).  r05, every size
// at 4 waves per SIMD (128 VGPRs): 64 / 128 / 256 / 512 / 1024 -> 1846 /
// 1982 / 2015 / 2004 / 1970 Mrays/s (profiles/r05_ab_shade_block.txt): a
// 1024-thread block fills its CU alone, so each of its barriers (the sample
// claim, the queue appends) idles the whole CU
#define PT_SHADE_BLOCK 256
#endif
#ifndef PT_SORT_PER
#define PT_SORT_PER 64u  // paths per thread of k_sort_count / k_sort_scatter (16: -0.07 %, 32: -0.3 %; profiles/r05_ab_ties_sort.txt)
#endif
template <int KEY, int NB>
__global__ void k_sort_count(PathSoA cur, const uint32_t* nptr, const float4* hit, uint32_t* counts, uint16_t* bins);
template <int NB>
__global__ void k_sort_scan(uint32_t* counts);
template <int KEY, int NB>
__global__ void k_sort_scatter(PathSoA cur, const uint32_t* nptr, const float4* hit, uint32_t* offsets, uint32_t* order,
                               const uint16_t* bins);
// (k_sort_count keeps each path's bin for k_sort_scatter: 2 B read instead of
// the 48 B of path and hit records the bin is computed from)
__global__ void k_adapt_init(RenderParams R, uint32_t shard_index, uint32_t shard_count, uint32_t* list,
                             uint32_t* cnt, AdaptEst* est, uint32_t* counts);
__global__ void k_adapt_map(const uint32_t* list, const uint32_t* n, int32_t* map);
__global__ void k_adapt_accum(RenderParams R, const float* sample_L, AdaptEst* est, uint32_t* counts);
__global__ void k_adapt_gather(RenderParams R, const int32_t* map, const float* sample_L, double* film);
__global__ void k_adapt_decide(const uint32_t* list, const uint32_t* n, const AdaptEst* est, const uint32_t* counts,
                               uint32_t max_samples, int32_t* map, uint32_t* out_list, uint32_t* out_cnt);
__global__ void k_interact(const pt_ray* rays, uint32_t n, float* out);
__global__ void k_bsdf_cases(int mid, const float* in, uint32_t n, float* out);
__global__ void k_light_cases(const float* in, uint32_t n, float* out);
__global__ void k_light_picks(const float* u, uint32_t n, int32_t* out);
__global__ void k_anim_inverse(const float* t, uint32_t n, float* out);
template <bool QN>
__global__ void k_trace_rays(const pt_ray* rays, uint32_t n, int any, pt_hit* out, uint32_t* pool, uint32_t* ovf,
                             unsigned long long* counters, uint32_t* ties, uint32_t* n_ties);
__global__ void k_trace_rays_ties(const pt_ray* rays, pt_hit* out, const uint32_t* ties, const uint32_t* n_ties,
                                  uint32_t n_rays);
