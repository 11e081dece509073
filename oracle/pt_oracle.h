/*
 * pt_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C) of the reference's per-sample hot path, used only
 * by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
 * checker.  The product (libpt_hip.so) never links or calls it.
 *
 * Parity of this restatement is pinned against golden vectors produced by the
 * reference itself (oracle/ref_harness.cpp compiled from /root/reference),
 * committed under tests/golden/.
 */
#ifndef PT_ORACLE_H
#define PT_ORACLE_H
#include "../include/pt_api.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Full SurfaceInteraction of a closest hit (Interaction.hpp:36-51). */
typedef struct oracle_hit {
    int32_t hit;
    float t, p[3], n[3], ns[3], uv[2], tangent[3];
    int32_t prim, material, light, medium;
    uint32_t nodes, tris; /* traversal work for this query (BVH4 clusters visited, leaf tests) */
} oracle_hit;

typedef struct oracle_counters {
    uint64_t closest, any, nodes_closest, tris_closest, nodes_any, tris_any, paths;
    uint64_t hits;      /* closest-hit queries that hit (shaded: SURVEY 8(d) +96 B +32 B) */
    uint64_t tex_bytes; /* shading texel bytes: 4 texels x C channels per bilinear fetch */
} oracle_counters;

int oracle_version(void);

/* Scene::Intersect (any_hit = 0) or Scene::IntersectPred (any_hit = 1). */
int oracle_trace(const pt_scene_desc* s, const pt_ray* rays, uint32_t n, int any_hit, oracle_hit* out);

/* Per-sample Li for pixels [pixel_begin, pixel_end) x samples [0, rd->spp):
 * out_L[(pix*spp + s)*3], out_p[(pix*spp + s)*2] (film position, double). */
int oracle_li(const pt_scene_desc* s, const pt_camera_desc* cam, const pt_render_desc* rd, uint32_t pixel_begin,
              uint32_t pixel_end, float* out_L, double* out_p, oracle_counters* cnt);
/* Li of n (pixel, sample) pairs: sample = the frame's global sample index. */
int oracle_li_pairs(const pt_scene_desc* s, const pt_camera_desc* cam, const pt_render_desc* rd, const uint32_t* pix,
                    const uint32_t* smp, uint32_t n, float* out_L, oracle_counters* cnt);

/* Whole-frame render into film_accum (W*H*4 doubles), `threads` pthreads over
 * 32x32 tiles, samples s with s % shard_count == shard_index. */
int oracle_render(const pt_scene_desc* s, const pt_camera_desc* cam, const pt_render_desc* rd, double* film_accum,
                  int threads, oracle_counters* cnt);
/* TileIntegrator::Render's adaptive sampling (Integrators.cpp:55-86): the
 * film plus each pixel's sample count (W*H u32).  Shards own 32x32 tiles. */
/* TextureInfiniteLight: Le / PDF of light li for directions (out[4n]); the
 * cell weights of pt_texinf_weights for a list of cells */
int oracle_inf_le(const pt_scene_desc* s, int li, const float* dirs, uint32_t n, float* out);
int oracle_texinf_weights(const float* tx, int w, int h, int c, const float cs[3], float scale, const uint32_t* cells,
                          uint32_t n, float* out);
int oracle_render_adaptive(const pt_scene_desc* s, const pt_camera_desc* cam, const pt_render_desc* rd,
                           double* film_accum, uint32_t* counts, int threads, oracle_counters* cnt);

/* Material cases, layout as oracle/ref_harness.cpp cmd_bsdf (27 floats in, 20 out). */
int oracle_bsdf(const pt_scene_desc* s, int material, const float* in, uint32_t n, float* out);

/* Light cases, layout as ref_harness cmd_lights (5 floats in, 18 out per light per case). */
int oracle_lights(const pt_scene_desc* s, const float* in, uint32_t n, float* out);

/* Film::WritePNG tone map + sRGB + u8 of a W*H*4 accumulation (0 = reinhard_jodie, 1 = ACES). */
int oracle_resolve(const double* film, int W, int H, int tonemap, uint8_t* out);

/* Filter weight table (33x33 grid on [-2,2]^2 + integral), as ref_harness cmd_film. */
int oracle_filter_table(const pt_render_desc* rd, double* out);

/* glm::inverse(mat4) as the reference build contracts it (tests/test_mat4_inverse.py) */
void oracle_mat4_inverse(const float* m, float* out);

#ifdef __cplusplus
}
#endif
#endif
