// Shared declarations between the wavefront kernels and the host runtime.
#pragma once
#include "pt_trace.h"

// path flags (meta.z): depth | rr_depth << 12 | spec
#define PF_DEPTH_MASK 0xFFFu
#define PF_RR_SHIFT 12
#define PF_SPEC (1u << 24)

// queue counters
#define Q_NEXT 0
#define Q_DONE 1
#define Q_SHADOW 2
#define Q_COUNT 4

// 64-bit work counters
#define CNT_NODES_CLOSEST 0
#define CNT_TRIS_CLOSEST 1
#define CNT_NODES_ANY 2
#define CNT_TRIS_ANY 3
#define CNT_NEXT_SAMPLE 4
#define CNT_COUNT 8

// Path state, structure of float4/uint4 arrays indexed by slot (16-B lanes,
// dwordx4 loads and stores).
struct PathSoA {
    float4* ray_o;  // origin
    float4* ray_d;  // direction
    float4* beta;   // attenuation.xyz, prevPDF
    float4* L;      // radiance so far
    uint4* meta;    // stream key, next draw dimension, flags, sample id in chunk
    float4* hit;    // t, b1, b2, prim slot (int bits; -1 = miss)
};

struct ShadowRec {
    float4 o;  // origin, tmax
    float4 d;  // direction, path slot (bits)
    float4 c;  // contribution if unoccluded
};

struct RenderParams {
    pt_camera_desc cam;
    uint32_t seed, max_depth;
    uint32_t shard_index, shard_count;
    uint32_t s_lo, s_hi;            // local sample range of this chunk
    uint32_t npix_work;             // pixels per sample index
    uint32_t tiled, tiles_x;
    uint32_t pixel_begin;
    unsigned long long chunk_total; // npix_work * (s_hi - s_lo)
    uint32_t filter;
    int rad_x, rad_y;
    float frad[2];
    double fparam[2];
    double inv_integral;
    double gauss_x, gauss_y;
};

template <bool COUNT>
__global__ void k_closest(DevScene S, PathSoA P, const uint32_t* q, uint32_t n, unsigned long long* counters);
template <bool COUNT>
__global__ void k_shadow(DevScene S, PathSoA P, const ShadowRec* sq, const uint32_t* nptr,
                         unsigned long long* counters);
template <int INTEGRATOR>
__global__ void k_shade(DevScene S, RenderParams R, PathSoA P, const uint32_t* q, uint32_t n, uint32_t* q_next,
                        uint32_t* q_done, ShadowRec* sq, uint32_t* cnt);
__global__ void k_finish(RenderParams R, PathSoA P, const uint32_t* q, const uint32_t* nptr, uint32_t n_direct,
                         int store, uint32_t* q_next, uint32_t* cnt, unsigned long long* next_sample,
                         float* sample_L);
__global__ void k_gather(RenderParams R, const float* sample_L, double* film);
__global__ void k_trace_rays(DevScene S, const pt_ray* rays, uint32_t n, int any, pt_hit* out,
                             unsigned long long* counters);
