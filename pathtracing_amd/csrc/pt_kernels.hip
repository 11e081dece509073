// Wavefront path tracer kernels for gfx950 (CDNA4).
//
// One iteration of the persistent wavefront (host loop in pt_runtime.hip):
//   k_closest  closest-hit traversal of every active path's ray (its block 0
//              also zeroes the next counter set and publishes the input count
//              to the host's pinned snapshot)
//   k_shade    one body of PathIntegrator::Li / SimplePathIntegrator::Li
//              (Integrators.cpp:131-294): miss -> infinite lights, emission
//              with MIS, scatter, NEE light sample -> shadow queue, RR;
//              continuing paths -> next state; finished paths store their
//              sample's radiance and their entry takes the next camera sample
//              (Camera::GenerateRay)
//   k_shadow   any-hit of the NEE rays; unoccluded -> contribution added to
//              the path (or to the finished sample's radiance)
//   k_fill     the initial camera samples of a chunk
//   k_gather   after a sample chunk: every pixel gathers the Mitchell/box/
//              Gaussian-weighted samples of its neighbourhood (FilmTile::Add,
//              Film.hpp:65-82) in float64 -- deterministic, no atomics.
// Queue appends are block-aggregated: one atomic per block (__ballot/__popcll).
#include "pt_kernels.h"

// ------------------------------------------------------------------ append helpers
__device__ __forceinline__ uint32_t lanemask_lt_count(uint64_t m) {
    return (uint32_t)__popcll(m & ((1ull << __lane_id()) - 1ull));
}

// Block-aggregated append to up to three queues: per wave a ballot, per block
// one prefix over the waves in LDS and one global atomic per queue.  Every
// thread of the block must call it (it contains barriers).
template <int NQ, int BLOCK>
__device__ __forceinline__ void block_append(uint32_t* qcnt, const int (&qoff)[NQ], const bool (&pred)[NQ],
                                             uint32_t (&slot)[NQ]) {
    constexpr int NW = BLOCK / 64;
    __shared__ uint32_t s_cnt[NQ][NW + 1];
    const uint32_t wave = threadIdx.x >> 6, lane = __lane_id();
    uint64_t m[NQ];
#pragma unroll
    for (int q = 0; q < NQ; q++) {
        m[q] = __ballot(pred[q]);
        if (lane == 0) s_cnt[q][wave] = (uint32_t)__popcll(m[q]);
    }
    __syncthreads();
    if (threadIdx.x < NQ) {
        const int q = threadIdx.x;
        uint32_t tot = 0;
        for (int w = 0; w < NW; w++) {
            uint32_t c = s_cnt[q][w];
            s_cnt[q][w] = tot;
            tot += c;
        }
        s_cnt[q][NW] = tot ? atomicAdd(&qcnt[qoff[q]], tot) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NQ; q++) slot[q] = s_cnt[q][NW] + s_cnt[q][wave] + lanemask_lt_count(m[q]);
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}
__device__ __forceinline__ void count_add(unsigned long long* counters, int which, uint64_t v) {
    uint64_t s = wave_sum64(v);
    if (__lane_id() == 0 && s) atomicAdd(&counters[(blockIdx.x % CNT_SHARDS) * CNT_COUNT + which], (unsigned long long)s);
}

// Wavefront iteration prologue, run by block 0 of the iteration's first kernel
// (the closest-hit traversal): zero the spare counter set (the next
// iteration's output) and publish this iteration's input counts to the host's
// pinned snapshot slot, so the host learns them without a copy or a sync.
__device__ __forceinline__ void iteration_prologue(const uint32_t* __restrict__ in, uint32_t* __restrict__ spare,
                                                   uint32_t* __restrict__ snap) {
    if (blockIdx.x != 0 || !spare) return;
    for (uint32_t k = threadIdx.x; k < SET_WORDS; k += blockDim.x) spare[k] = 0;
    if (threadIdx.x == 0) {
        snap[SNAP_PATHS] = path_count(in);
        snap[SNAP_SHADOW_PREV] = in[Q_SHADOW];
        snap[SNAP_NEW] = in[Q_NEW];
    }
}

// SurfaceInteraction of a closest hit (Shape.cpp:58-244 via
// GeometricPrimitive::Intersect, Primitive.cpp:15-26): prim slot (or virtual
// slot of an instance), t and barycentrics / quad coordinates from the
// traversal.  Instance hits (TransformedPrimitive::Intersect,
// Primitive.cpp:48-64): the object-space ray is rebuilt, the primitive test
// re-run for t (the traversal kept the world t) and the object-space
// interaction carried back with the transform and its normal matrix.
// AnimatedPrimitive hits (S.motion) and nested wrappers (pt_instance.inner)
// go out of line (the rare path keeps k_shade's registers), values in and
// out: the object-space ray through every level at the ray's time, the
// outermost first; the interaction back through them, the innermost first
// (TransformedPrimitive::Intersect called by the wrapper around it).  Their
// world t is the traversal's, which divided the object-space t by each
// level's length in that same order.
struct ChainRay {
    f3 o, d;
};
__device__ __noinline__ ChainRay chain_object_ray(const DevInstance* I, float time, f3 ro, f3 rd) {
    const DevInstance* lv[PT_MAX_INSTANCE_DEPTH];
    const int k = inst_chain(I, lv);
    for (int j = 0; j < k; j++) {
        float T[16], inv[16];
        inst_matrices(*lv[j], time, T, inv);
        const f3 dir = m4_dir(inv, rd);
        const float len = length(dir);
        ro = m4_point(inv, ro);
        rd = dir / len;
    }
    return ChainRay{ro, rd};
}
struct SurfXf {
    f3 p, n, ns, tangent;
};
__device__ __noinline__ SurfXf chain_world_surface(const DevInstance* I, float time, f3 p, f3 n, f3 ns, f3 tangent) {
    const DevInstance* lv[PT_MAX_INSTANCE_DEPTH];
    const int k = inst_chain(I, lv);
    for (int j = k - 1; j >= 0; j--) {
        float T[16], inv[16], NM[9];
        inst_matrices(*lv[j], time, T, inv);
        normal_matrix(T, NM);
        p = m4_point(T, p);
        n = normalize(m3_mul(NM, n));
        ns = normalize(m3_mul(NM, ns));
        tangent = normalize4(m4_dir(T, tangent));
    }
    return SurfXf{p, n, ns, tangent};
}
// The slot of a hit's primitive: a virtual slot (a primitive inside an
// instance, past S.n_prims) maps to its slot in the instance's BLAS
__device__ __forceinline__ uint32_t hit_slot(int prim) {
    uint32_t slot = (uint32_t)prim;
    if (slot >= S.n_prims) {
        for (uint32_t k = 0; k < S.n_instances; k++) {
            const DevInstance& c = S.instances[k];
            if ((uint32_t)prim >= c.virt_base && (uint32_t)prim < c.virt_base + c.n_prims)
                slot = c.prim_base + ((uint32_t)prim - c.virt_base);
        }
    }
    return slot;
}
// mt (PT_MT_EARLY): the hit material's textures (mat_tex), evaluated next to
// the normal map's texture -- both need only the hit's uv -- so their reads
// overlap; the same values as mat_tex after hit_surface (C4 shade -2.3 %,
// +0.4 %; profiles/r06_ab_shade_chain.txt)
#ifndef PT_MT_EARLY
#define PT_MT_EARLY 1
#endif
__device__ __forceinline__ void hit_surface(int prim, f3 ro, f3 rd, float t, float b1, float b2, SurfInt& si,
                                         int& medium, float time = 0.0f, MatTex* mt = nullptr) {
    float len = 1.0f;
    const DevInstance* I = nullptr;
    bool xf = false;  // the hit's levels go out of line (an AnimatedPrimitive, nested wrappers)
    if ((uint32_t)prim >= S.n_prims) {
        for (uint32_t k = 0; k < S.n_instances; k++) {
            const DevInstance& c = S.instances[k];
            if ((uint32_t)prim >= c.virt_base && (uint32_t)prim < c.virt_base + c.n_prims) I = &c;
        }
        prim = (int)(I->prim_base + ((uint32_t)prim - I->virt_base));
        xf = (S.motion && I->anim) || I->inner >= 0;
        if (xf) {  // AnimatedPrimitive::Intersect at the ray's time (Primitive.cpp:86-89), level by level
            const ChainRay r = chain_object_ray(I, time, ro, rd);
            ro = r.o;
            rd = r.d;
            len = t;  // (the world t, kept for si.t)
        } else {
            const f3 dir = m4_dir(I->inv, rd);
            len = length(dir);
            ro = m4_point(I->inv, ro);
            rd = dir / len;
        }
    }
    const DevGeom g = S.geom[prim];
    const DevPrimInfo pi = S.info[prim];
    // the slot's shading record (one 128-B line) with its geometry and info:
    // three independent reads instead of info -> record
    const DevTriShade R = S.tshade[prim];
    const uint32_t kind = __float_as_uint(g.a.w) & GF_KIND;
    if (I) {  // the object-space t of the accepted hit
        if (kind == PT_PRIM_TRIANGLE) {
            float bx, by;
            tri_glm(ro, rd, xyz(g.a), xyz(g.b), xyz(g.c), bx, by, t);
        } else if (kind == PT_PRIM_QUAD) {
            float a, b;
            quad_hit<false>(S.quads[pi.index], ro, rd, __int_as_float(0x7f800000), t, a, b);
        } else {
            sphere_root(S.spheres[pi.index], ro, rd, __int_as_float(0x7f800000), t);
        }
    }
    if (kind == PT_PRIM_TRIANGLE) {
        tri_interaction(g, R, pi.material, ro, rd, t, b1, b2, si, !mt);
        if (mt) {  // the textures and the normal map's texture side by side
            if (pi.material >= 0) *mt = mat_tex(pi.material, si);
            si.ns = normal_map(pi.material, si);
        }
    } else {
        if (kind == PT_PRIM_QUAD) quad_interaction(S.quads[pi.index], ro, rd, t, b1, b2, si);
        else sphere_interaction(S.spheres[pi.index], ro, rd, t, si);
        if (mt && pi.material >= 0) *mt = mat_tex(pi.material, si);
    }
    si.mat = pi.material;
    si.light = pi.light;
    medium = pi.medium;
    if (xf) {
        const SurfXf w = chain_world_surface(I, time, si.p, si.n, si.ns, si.tangent);
        si.p = w.p;
        si.n = w.n;
        si.ns = w.ns;
        si.t = len;
        si.tangent = w.tangent;
    } else if (I) {
        float NM[9];
        normal_matrix(I->T, NM);
        si.p = m4_point(I->T, si.p);
        si.n = normalize(m3_mul(NM, si.n));
        si.ns = normalize(m3_mul(NM, si.ns));
        si.t = si.t / len;
        si.tangent = normalize4(m4_dir(I->T, si.tangent));
    }
}

// ------------------------------------------------------------------ traversal kernels
// Register budget of the pool kernels: waves per SIMD.  Step-per-iteration
// traversal (trace_pool): 7 (72 VGPRs, no hot-path spills) measured +4.5 %
// on C4 over the unconstrained 76; 8 (64 VGPRs) spills inside the step loop
// and loses 30 %.  Overlapped traversal (trace_spec, quantized nodes without
// instances): 7 (72 VGPRs, 1 spilled) since round 5's cheaper pushes and
// alpha path, closest-hit -2.1 % over 6 (profiles/r05_ab_traversal.txt; in
// round 3 it spilled and lost 3 %, profiles/r03_ab_spec.txt).
#ifndef PT_POOL_WPE
#define PT_POOL_WPE 7
#endif
#ifndef PT_SPEC_WPE
#define PT_SPEC_WPE 7
#endif
#define PT_POOL_WAVES_FOR(SPEC_) __attribute__((amdgpu_waves_per_eu((SPEC_) ? PT_SPEC_WPE : PT_POOL_WPE, \
                                                                    (SPEC_) ? PT_SPEC_WPE : PT_POOL_WPE)))
// the any-hit pool kernel's own budget (it needs fewer registers: no hit
// record): 8 waves per SIMD, C4 k_shadow_pool 10.72 -> 10.34 ms per launch
// over 7 (6: 11.50; profiles/r02_ab_shade.txt); overlapped: 7 (8 spills,
// k_shadow_pool +17 %)
#ifndef PT_SHADOW_WPE
#define PT_SHADOW_WPE 8
#endif
#ifndef PT_SPEC_SHADOW_WPE
#define PT_SPEC_SHADOW_WPE 7
#endif
#define PT_SHADOW_WAVES_FOR(SPEC_) \
    __attribute__((amdgpu_waves_per_eu((SPEC_) ? PT_SPEC_SHADOW_WPE : PT_SHADOW_WPE, \
                                       (SPEC_) ? PT_SPEC_SHADOW_WPE : PT_SHADOW_WPE)))
// which pool kernels take trace_spec (pt_pool.h trace_pool's dispatch)
#define PT_USES_SPEC(INST_, QN_) ((QN_) && !(INST_))
// The spatial hit sort's bin of a hit at o + t d: the Morton code of its
// cell in a 2^PT_SORT_CELL_BITS grid over the scene box (0 for a miss too)
__device__ __forceinline__ uint32_t hit_cell(f3 o, f3 d, float t) {
    uint32_t code = 0;
    const float p[3] = {fmaf(t, d.x, o.x), fmaf(t, d.y, o.y), fmaf(t, d.z, o.z)};
#pragma unroll
    for (int a = 0; a < 3; a++) {
        const float q = (p[a] - S.bb_lo[a]) * S.bb_scale[a];  // [0, 2^bits)
        const uint32_t c = (uint32_t)fminf(fmaxf(q, 0.0f), (float)((1 << PT_SORT_CELL_BITS) - 1));
#pragma unroll
        for (int b = 0; b < PT_SORT_CELL_BITS; b++) code |= ((c >> b) & 1u) << (3 * b + a);
    }
    return code;
}
// Persistent, refilling traversal (pt_pool.h): grid = resident blocks, rays
// claimed from the pool counters (zeroed with the queue counters).
struct ClosestSrc {
    PathSoA P;
    float4* hit;
    uint32_t front;  // continuing paths at the front of P
    uint32_t* ties;      // rays to re-trace exactly (k_closest_ties), and their count
    uint32_t* n_ties;
    // S.ray_order (PT_RENDER_SORT_RAYS): claim i traces path ray_order[i]
    __device__ __forceinline__ bool load(uint32_t i, f3& o, f3& d, float& tmax) {
        const uint32_t j = S.ray_order ? S.ray_order[i] : i;
        const uint32_t e = path_slot(j, front, P.cap);
        o = xyz(P.o[e]);
        d = xyz(P.d[e]);
        tmax = __int_as_float(0x7f800000);
        return true;
    }
    __device__ __forceinline__ void closest(uint32_t i, float t, float b1, float b2, int prim) {
        hit[S.ray_order ? S.ray_order[i] : i] = make_float4(t, b1, b2, __int_as_float(prim));
    }
    __device__ __forceinline__ float time(uint32_t i) const {
        return P.time[path_slot(S.ray_order ? S.ray_order[i] : i, front, P.cap)];
    }
    __device__ __forceinline__ void any(uint32_t, bool) {}
    // the list holds P.cap entries (a ray is listed at most once per launch:
    // OCT_TIE survives instance enter / exit, so it cannot fill); an entry
    // past it would be a dropped tie, which could change a hit
    // (Shape.cpp:204): counted as pt_stats::tie_overflows, asserted 0
    __device__ __forceinline__ void tie(uint32_t i) {
        const uint32_t k = atomicAdd(n_ties, 1u);
        if (k < P.cap) ties[k] = i;
        else atomicAdd(S.tie_drops, 1u);
    }
};

template <bool COUNT, bool INST, bool QN>
__global__ __launch_bounds__(PT_TRACE_BLOCK) PT_POOL_WAVES_FOR(PT_USES_SPEC(INST, QN)) void k_closest_pool(PathSoA P, const uint32_t* __restrict__ nptr,
                                                                float4* __restrict__ hit, uint32_t* __restrict__ pool,
                                                                uint32_t* __restrict__ ovf, uint32_t* __restrict__ spare,
                                                                uint32_t* __restrict__ snap,
                                                                unsigned long long* counters, uint32_t* __restrict__ ties) {
    __shared__ uint32_t s_ref[PT_POOL_LDS * PT_TRACE_BLOCK];
    __shared__ __attribute__((aligned(16))) uint8_t s_lut[QN ? Q48_LUT_BYTES : 4];
    iteration_prologue(nptr, spare, snap);
    const uint32_t n = path_count(nptr);
    if (n == 0) return;
    if constexpr (QN) stage_q48_lut(s_lut);
    TraceWork wk{0, 0};
    ClosestSrc src{P, hit, nptr[Q_NEXT], ties, pool + (Q_TIES - Q_WORDS)};
    trace_pool<false, COUNT, ClosestSrc, INST, PT_POOL_LDS, QN>(n, pool, src, s_ref, ovf, wk, s_lut);
    if (COUNT) {
        count_add(counters, CNT_NODES_CLOSEST, wk.nodes);
        count_add(counters, CNT_TRIS_CLOSEST, wk.tris);
    }
}

// Exact re-trace of the rays the pool kernel listed for an exact-t tie
// (pt_pool.h "Exact-t ties"): trace_closest over the reference's clusters
// in the reference's order; the listed count sits in the pool's counter set.
template <bool INST>
__global__ __launch_bounds__(PT_TRACE_BLOCK) void k_closest_ties(PathSoA P, const uint32_t* __restrict__ nptr,
                                                                float4* __restrict__ hit,
                                                                const uint32_t* __restrict__ pool,
                                                                const uint32_t* __restrict__ ties) {
    __shared__ uint32_t s_ref[PT_STACK * PT_TRACE_BLOCK];
    const uint32_t n = min(pool[Q_TIES - Q_WORDS], P.cap);
    if (n == 0) return;
    ClosestSrc src{P, hit, nptr[Q_NEXT], nullptr, nullptr};
    TraceWork wk{0, 0};
    for (uint32_t k = blockIdx.x * PT_TRACE_BLOCK + threadIdx.x; k < n; k += gridDim.x * PT_TRACE_BLOCK) {
        const uint32_t i = ties[k];
        f3 o, d;
        float tmax, t, b1, b2;
        src.load(i, o, d, tmax);
        const int prim = trace_closest<false, INST, PT_STACK>(o, d, tmax, t, b1, b2, s_ref, wk, nullptr,
                                                              (INST && S.motion) ? src.time(i) : 0.0f);
        src.closest(i, t, b1, b2, prim);
    }
}

// The unoccluded shadow ray's contribution: fma(c, att, L) into its path's
// radiance, or into its sample's when the path ended this bounce; one shadow
// ray per path per bounce, so a plain read-modify-write
__device__ __forceinline__ void shadow_add(PathSoA& next, float* __restrict__ sample_L, uint32_t tgt, float4 c,
                                           float4 a) {
    if (tgt & SHADOW_DONE_BIT) {  // the path ended this bounce: its sample's radiance
        float* L = sample_L + 3ull * (tgt & ~SHADOW_DONE_BIT);
        L[0] = fma_(c.x, a.x, L[0]);
        L[1] = fma_(c.y, a.y, L[1]);
        L[2] = fma_(c.z, a.z, L[2]);
        return;
    }
    float4* L = &next.L[tgt];
    float4 v = *L;
    v.x = fma_(c.x, a.x, v.x);
    v.y = fma_(c.y, a.y, v.y);
    v.z = fma_(c.z, a.z, v.z);
    *L = v;
}
// Shadow-ray source of the any-hit kernels: an unoccluded ray adds its
// contribution in place (deferring the add to a kernel after the traversal
// measured slower: C4 any-hit 1178 -> 1192 ms per frame,
// profiles/r04_ab_traversal.txt)
struct ShadowSrc {
    ShadowRec* sq;
    PathSoA next;
    float* sample_L;
    __device__ __forceinline__ bool load(uint32_t i, f3& o, f3& d, float& tmax) {
        const float4 ro = sq[i].o, rd = sq[i].d;
        o = xyz(ro);
        d = xyz(rd);
        tmax = ro.w;
        return true;
    }
    __device__ __forceinline__ void closest(uint32_t, float, float, float, int) {}
    __device__ __forceinline__ void tie(uint32_t) {}
    __device__ __forceinline__ float time(uint32_t i) const { return S.sq_time[i]; }
    __device__ __forceinline__ void any(uint32_t i, bool hit) {
        if (hit) return;
        shadow_add(next, sample_L, __float_as_uint(sq[i].d.w), sq[i].c, sq[i].a);
    }
};

template <bool COUNT, bool INST, bool QN>
__global__ __launch_bounds__(PT_TRACE_BLOCK) PT_SHADOW_WAVES_FOR(PT_USES_SPEC(INST, QN)) void k_shadow_pool(PathSoA next, float* __restrict__ sample_L,
                                                               ShadowRec* __restrict__ sq,
                                                               const uint32_t* __restrict__ nptr,
                                                               uint32_t* __restrict__ pool, uint32_t* __restrict__ ovf,
                                                               unsigned long long* counters) {
    __shared__ uint32_t s_ref[PT_POOL_LDS * PT_TRACE_BLOCK];
    __shared__ __attribute__((aligned(16))) uint8_t s_lut[QN ? Q48_LUT_BYTES : 4];
    TraceWork wk{0, 0};
    ShadowSrc src{sq, next, sample_L};
    const uint32_t n = *nptr;
    if (n == 0) return;
    if constexpr (QN) stage_q48_lut(s_lut);
    trace_pool<true, COUNT, ShadowSrc, INST, PT_POOL_LDS, QN>(n, pool, src, s_ref, ovf, wk, s_lut);
    if (COUNT) {
        count_add(counters, CNT_NODES_ANY, wk.nodes);
        count_add(counters, CNT_TRIS_ANY, wk.tris);
    }
}

// The stackless any-hit traversal (pt_pool.h trace_any_stackless,
// PT_RENDER_ANY_STACKLESS): quantized records without instances.  Its LDS
// holds only the octant table, so registers alone set its occupancy
#ifndef PT_SL_WPE
#define PT_SL_WPE 8
#endif
template <bool COUNT>
__global__ __launch_bounds__(PT_TRACE_BLOCK) __attribute__((amdgpu_waves_per_eu(PT_SL_WPE, PT_SL_WPE)))
void k_shadow_sl(PathSoA next, float* __restrict__ sample_L, ShadowRec* __restrict__ sq,
                 const uint32_t* __restrict__ nptr, uint32_t* __restrict__ pool, uint32_t* __restrict__,
                 unsigned long long* counters) {
    __shared__ __attribute__((aligned(16))) uint8_t s_lut[Q48_LUT_BYTES];
    TraceWork wk{0, 0};
    ShadowSrc src{sq, next, sample_L};
    const uint32_t n = *nptr;
    if (n == 0) return;
    stage_q48_lut(s_lut);
    trace_any_stackless<COUNT, ShadowSrc>(n, pool, src, wk, s_lut);
    if (COUNT) {
        count_add(counters, CNT_NODES_ANY, wk.nodes);
        count_add(counters, CNT_TRIS_ANY, wk.tris);
    }
}

// One ray per lane (grid covers all rays): lower overhead where traversal
// lengths are uniform (small scenes); the runtime picks per scene.  The
// whole-leaf inner loop of trace_closest / trace_any measures faster here than
// the one-primitive-per-step loop of pt_pool.h (C2: 171 vs 191 us per launch).
// PT_SIMPLE_LN: stack entries these kernels keep in LDS (the rest in the
// global overflow array).
#ifndef PT_SIMPLE_LN
#define PT_SIMPLE_LN PT_STACK
#endif
#define PT_SIMPLE_WAVES
template <bool COUNT, bool INST>
__global__ __launch_bounds__(PT_TRACE_BLOCK) PT_SIMPLE_WAVES void k_closest(PathSoA P, const uint32_t* __restrict__ nptr,
                                                           float4* __restrict__ hit, uint32_t* __restrict__,
                                                           uint32_t* __restrict__ ovf, uint32_t* __restrict__ spare,
                                                           uint32_t* __restrict__ snap, unsigned long long* counters,
                                                           uint32_t* __restrict__) {
    __shared__ uint32_t s_ref[PT_SIMPLE_LN * PT_TRACE_BLOCK];
    iteration_prologue(nptr, spare, snap);
    const uint32_t n = path_count(nptr);  // the grid covers the wavefront's capacity
    if (blockIdx.x * PT_TRACE_BLOCK >= n) return;
    TraceWork wk{0, 0};
    const uint32_t i = blockIdx.x * PT_TRACE_BLOCK + threadIdx.x;
    if (i < n) {
        const uint32_t e = path_slot(i, nptr[Q_NEXT], P.cap);
        const float4 o = P.o[e], d = P.d[e];
        float t, b1, b2;
        int prim = trace_closest<COUNT, INST, PT_SIMPLE_LN>(xyz(o), xyz(d), __int_as_float(0x7f800000), t, b1, b2,
                                                            s_ref, wk, ovf, (INST && S.motion) ? P.time[e] : 0.0f);
        hit[i] = make_float4(t, b1, b2, __int_as_float(prim));
    }
    if (COUNT) {
        count_add(counters, CNT_NODES_CLOSEST, wk.nodes);
        count_add(counters, CNT_TRIS_CLOSEST, wk.tris);
    }
}

template <bool COUNT, bool INST>
__global__ __launch_bounds__(PT_TRACE_BLOCK) PT_SIMPLE_WAVES void k_shadow(PathSoA next, float* __restrict__ sample_L,
                                                          ShadowRec* __restrict__ sq,
                                                          const uint32_t* __restrict__ nptr, uint32_t* __restrict__,
                                                          uint32_t* __restrict__ ovf, unsigned long long* counters) {
    __shared__ uint32_t s_ref[PT_SIMPLE_LN * PT_TRACE_BLOCK];
    const uint32_t n = *nptr;
    if (blockIdx.x * PT_TRACE_BLOCK >= n) return;
    TraceWork wk{0, 0};
    ShadowSrc src{sq, next, sample_L};
    const uint32_t i = blockIdx.x * PT_TRACE_BLOCK + threadIdx.x;
    if (i < n) {
        const ShadowRec r = sq[i];
        src.any(i, trace_any<COUNT, INST, PT_SIMPLE_LN>(xyz(r.o), xyz(r.d), r.o.w, s_ref, wk, ovf,
                                                        (INST && S.motion) ? S.sq_time[i] : 0.0f));
    }
    if (COUNT) {
        count_add(counters, CNT_NODES_ANY, wk.nodes);
        count_add(counters, CNT_TRIS_ANY, wk.tris);
    }
}

// Test hook: trace arbitrary rays (pt_trace), through the product traversal.
struct RaysSrc {
    const pt_ray* rays;
    pt_hit* out;
    uint32_t* ties;  // exact-t ties (pt_pool.h), re-traced by k_trace_rays_ties
    uint32_t* n_ties;
    uint32_t n;      // rays, and entries of the tie list
    __device__ __forceinline__ bool load(uint32_t i, f3& o, f3& d, float& tmax) {
        const pt_ray r = rays[i];
        o = F3(r.o[0], r.o[1], r.o[2]);
        d = F3(r.d[0], r.d[1], r.d[2]);
        tmax = r.tmax;
        return true;
    }
    __device__ __forceinline__ void closest(uint32_t i, float t, float b1, float b2, int prim) {
        out[i] = pt_hit{t, b1, b2, prim};
    }
    __device__ __forceinline__ void any(uint32_t i, bool hit) { out[i] = pt_hit{0, 0, 0, hit ? 1 : 0}; }
    __device__ __forceinline__ float time(uint32_t i) const { return rays[i].time; }
    __device__ __forceinline__ void tie(uint32_t i) {
        const uint32_t k = atomicAdd(n_ties, 1u);
        if (k < n) ties[k] = i;
        else atomicAdd(S.tie_drops, 1u);  // (as ClosestSrc::tie)
    }
};

template <bool QN>
__global__ __launch_bounds__(PT_TRACE_BLOCK) void k_trace_rays(const pt_ray* __restrict__ rays, uint32_t n, int any,
                                                              pt_hit* __restrict__ out, uint32_t* __restrict__ pool,
                                                              uint32_t* __restrict__ ovf, unsigned long long* counters,
                                                              uint32_t* __restrict__ ties, uint32_t* __restrict__ n_ties) {
    __shared__ uint32_t s_ref[PT_POOL_LDS * PT_TRACE_BLOCK];
    __shared__ __attribute__((aligned(16))) uint8_t s_lut[QN ? Q48_LUT_BYTES : 4];
    if constexpr (QN) stage_q48_lut(s_lut);
    TraceWork wk{0, 0};
    RaysSrc src{rays, out, ties, n_ties, n};
    if (any) trace_pool<true, true, RaysSrc, true, PT_POOL_LDS, QN>(n, pool, src, s_ref, ovf, wk, s_lut);
    else trace_pool<false, true, RaysSrc, true, PT_POOL_LDS, QN>(n, pool, src, s_ref, ovf, wk, s_lut);
    count_add(counters, any ? CNT_NODES_ANY : CNT_NODES_CLOSEST, wk.nodes);
    count_add(counters, any ? CNT_TRIS_ANY : CNT_TRIS_CLOSEST, wk.tris);
}

// pt_trace with any_hit 2: the stackless any-hit traversal on arbitrary rays
__global__ __launch_bounds__(PT_TRACE_BLOCK) __attribute__((amdgpu_waves_per_eu(PT_SL_WPE, PT_SL_WPE)))
void k_trace_rays_sl(const pt_ray* __restrict__ rays, uint32_t n, pt_hit* __restrict__ out,
                     uint32_t* __restrict__ pool, unsigned long long* counters) {
    __shared__ __attribute__((aligned(16))) uint8_t s_lut[Q48_LUT_BYTES];
    stage_q48_lut(s_lut);
    TraceWork wk{0, 0};
    RaysSrc src{rays, out, nullptr, nullptr, n};
    trace_any_stackless<true, RaysSrc>(n, pool, src, wk, s_lut);
    count_add(counters, CNT_NODES_ANY, wk.nodes);
    count_add(counters, CNT_TRIS_ANY, wk.tris);
}

// pt_trace's exact re-trace of the rays k_trace_rays listed for an exact-t tie
__global__ __launch_bounds__(PT_TRACE_BLOCK) void k_trace_rays_ties(const pt_ray* __restrict__ rays,
                                                                   pt_hit* __restrict__ out,
                                                                   const uint32_t* __restrict__ ties,
                                                                   const uint32_t* __restrict__ n_ties,
                                                                   uint32_t n_rays) {
    __shared__ uint32_t s_ref[PT_STACK * PT_TRACE_BLOCK];
    const uint32_t n = min(*n_ties, n_rays);
    TraceWork wk{0, 0};
    for (uint32_t k = blockIdx.x * PT_TRACE_BLOCK + threadIdx.x; k < n; k += gridDim.x * PT_TRACE_BLOCK) {
        const pt_ray r = rays[ties[k]];
        float t, b1, b2;
        const int prim = trace_closest<false, true, PT_STACK>(F3(r.o[0], r.o[1], r.o[2]), F3(r.d[0], r.d[1], r.d[2]),
                                                             r.tmax, t, b1, b2, s_ref, wk, nullptr, r.time);
        out[ties[k]] = pt_hit{t, b1, b2, prim};
    }
}

// Test hook: closest hit + the full SurfaceInteraction the shade kernel
// reconstructs (pt_interact): {hit, t, p, n, ns, uv, tangent} per ray, the
// layout of the reference harness's trace records.
__global__ __launch_bounds__(PT_TRACE_BLOCK) void k_interact(const pt_ray* __restrict__ rays, uint32_t n,
                                                            float* __restrict__ out) {
    __shared__ uint32_t s_ref[PT_STACK * PT_TRACE_BLOCK];
    const uint32_t i = blockIdx.x * PT_TRACE_BLOCK + threadIdx.x;
    TraceWork wk{0, 0};
    if (i >= n) return;
    const pt_ray r = rays[i];
    f3 o = F3(r.o[0], r.o[1], r.o[2]), d = F3(r.d[0], r.d[1], r.d[2]);
    float t, b1, b2;
    const int prim = trace_closest<false>(o, d, r.tmax, t, b1, b2, s_ref, wk, nullptr, r.time);
    float* w = out + 16ull * i;
    for (int k = 0; k < 16; k++) w[k] = 0.0f;
    if (prim < 0) return;
    SurfInt si;
    int medium;
    hit_surface(prim, o, d, t, b1, b2, si, medium, r.time);
    const float rec[16] = {1.0f, si.t, si.p.x, si.p.y, si.p.z, si.n.x, si.n.y, si.n.z, si.ns.x, si.ns.y, si.ns.z,
                           si.u, si.v, si.tangent.x, si.tangent.y, si.tangent.z};
    for (int k = 0; k < 16; k++) w[k] = rec[k];
}

// Test hook: Material::scatter / calc_attenuation / PDF on given
// interactions (pt_bsdf_cases); case and record layout of oracle_bsdf.
__global__ void k_bsdf_cases(int mid, const float* __restrict__ in, uint32_t n, float* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* c = in + 27ull * i;
    float* o = out + 20ull * i;
    for (int k = 0; k < 20; k++) o[k] = 0.0f;
    const f3 ro = F3(c[0], c[1], c[2]), rd = F3(c[3], c[4], c[5]);
    SurfInt si;
    si.p = F3(c[6], c[7], c[8]);
    si.n = F3(c[9], c[10], c[11]);
    si.ns = F3(c[12], c[13], c[14]);
    si.tangent = F3(c[15], c[16], c[17]);
    si.u = c[18];
    si.v = c[19];
    si.t = c[20];
    si.mat = mid;
    si.light = -1;
    const MatTex mt = mat_tex(mid, si);
    const Bxdf b = mat_scatter(mt, ro, rd, si, c[21], c[22], c[23]);
    if (b.ok) {
        o[0] = 1.0f;
        o[1] = b.f.x; o[2] = b.f.y; o[3] = b.f.z;
        o[4] = b.pdf;
        o[5] = (float)b.flags;
        o[6] = b.o.x; o[7] = b.o.y; o[8] = b.o.z;
        o[9] = b.d.x; o[10] = b.d.y; o[11] = b.d.z;
        const f3 a = mat_f(mt, rd, si, b.d);
        o[12] = a.x; o[13] = a.y; o[14] = a.z;
        o[15] = mat_pdf(mt, rd, si, b.d);
    }
    const f3 other = F3(c[24], c[25], c[26]);
    const f3 a2 = mat_f(mt, rd, si, other);
    o[16] = a2.x; o[17] = a2.y; o[18] = a2.z;
    o[19] = mat_pdf(mt, rd, si, other);
}

// Test hook: anim_inverse (pt_shading.h) on the matrix identity + t
// (pt_anim_inverse_cases), as inst_matrices forms it for an AnimatedPrimitive
__global__ void k_anim_inverse(const float* __restrict__ t, uint32_t n, float* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float T[16], inv[16];
#pragma unroll
    for (int k = 0; k < 16; k++) T[k] = (k % 5 == 0) ? 1.0f : 0.0f;
    T[12] = t[3 * i];
    T[13] = t[3 * i + 1];
    T[14] = t[3 * i + 2];
    anim_inverse(T, inv);
#pragma unroll
    for (int k = 0; k < 16; k++) out[16ull * i + k] = inv[k];
}

// Test hook: LightSampler::Sample(u) picks (pt_light_picks): the light index
// ls_sample returns (-1: no light), one per u.
__global__ void k_light_picks(const float* __restrict__ u, uint32_t n, int32_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = ls_sample(u[i]);
}

// Test hook: Light::sample / PDF / L per light x case (pt_light_cases);
// case {uv[2], ref point[3]}, record layout of oracle_lights.
__global__ void k_light_cases(const float* __restrict__ in, uint32_t n, float* __restrict__ out) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n * S.n_lights) return;
    const uint32_t li = k / n, i = k % n;
    const pt_light& l = S.lights[li];
    const float* c = in + 5ull * i;
    float* o = out + 18ull * k;
    for (int j = 0; j < 18; j++) o[j] = 0.0f;
    // a TextureInfiniteLight's hidden cell draw: a hash of the case
    const float uc = draw(pcg_hash(__float_as_uint(c[0]) ^ pcg_hash(__float_as_uint(c[1]))), 0);
    const LSample ls = light_sample(li, c[0], c[1], uc);
    o[0] = ls.L.x; o[1] = ls.L.y; o[2] = ls.L.z;
    o[3] = ls.p.x; o[4] = ls.p.y; o[5] = ls.p.z;
    o[6] = ls.n.x; o[7] = ls.n.y; o[8] = ls.n.z;
    o[9] = ls.u; o[10] = ls.v;
    o[11] = ls.dir.x; o[12] = ls.dir.y; o[13] = ls.dir.z;
    if (!is_zero(ls.n)) {
        const f3 ref = F3(c[2], c[3], c[4]);
        const f3 rd = normalize(ls.p - ref);
        o[14] = light_pdf(li, ls.p, ls.n, ref, rd);
        const f3 L = light_L(l, ls.n, ls.u, ls.v, rd);
        o[15] = L.x; o[16] = L.y; o[17] = L.z;
    }
}

// ------------------------------------------------------------------ camera / regeneration
__device__ __forceinline__ void work_pixel(const RenderParams& R, uint32_t pix_i, uint32_t& x, uint32_t& y) {
    if (R.pix_list) {  // adaptive round: the still-active pixels
        const uint32_t p = R.pix_list[pix_i];
        x = p % (uint32_t)R.cam.width;
        y = p / (uint32_t)R.cam.width;
    } else if (R.tiled) {  // 8x8 pixel tiles, tile-major: neighbouring lanes -> neighbouring pixels
        uint32_t tile = pix_i >> 6, within = pix_i & 63u;
        uint32_t tx = tile % R.tiles_x, ty = tile / R.tiles_x;
        x = tx * 8 + (within & 7u);
        y = ty * 8 + (within >> 3);
    } else {
        uint32_t p = R.pixel_begin + pix_i;
        x = p % (uint32_t)R.cam.width;
        y = p / (uint32_t)R.cam.width;
    }
}

// StratifiedSampler's camera draws (Sampler.hpp:73-151) on Render's
// per-thread clone (Integrators.cpp:39, 61-64): the stratum of the pixel's
// sample index i in dimension d is PermutationElement(i, spp, Hash(px, py, d))
// (Util.hpp:45-73; Hash = MurmurHash64A over the 16 bytes {px, py, d},
// Util.hpp:75-168), jittered by the stream's draw (the reference's
// random_float()).  Three per camera sample; the integer work is negligible
// beside the traversal.
__device__ __forceinline__ uint64_t murmur_pxd(uint32_t px, uint32_t py, uint64_t d) {
    const uint64_t m = 0xc6a4a7935bd1e995ull;
    uint64_t h = 16ull * m;
    const uint64_t ks[2] = {(uint64_t)px | ((uint64_t)py << 32), d};
#pragma unroll
    for (int j = 0; j < 2; j++) {
        uint64_t k = ks[j] * m;
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
__device__ __forceinline__ uint32_t permutation_element(uint32_t i, uint32_t l, uint32_t p) {
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
__device__ __forceinline__ uint32_t stratum_of(uint32_t x, uint32_t y, uint32_t d, uint32_t idx, uint32_t spp) {
    return permutation_element(idx, spp, (uint32_t)murmur_pxd(x, y, d));
}

// Camera::GenerateRay (Camera.hpp:21-35) with the camera draws of
// TileIntegrator::Render (Integrators.cpp:61-64): pixel2D, time, lens2D;
// sx > 0: a StratifiedSampler(sx, sy) host, idx the sample's index in its
// pixel's round.
__device__ __forceinline__ void camera_ray(const pt_camera_desc& c, uint32_t key, uint32_t x, uint32_t y, f3& o, f3& d,
                                           float& time, uint32_t sx = 0, uint32_t sy = 0, uint32_t idx = 0) {
    float a = draw(key, 0), b = draw(key, 1);
    float pxf, pyf;
    float tu = 0.0f, l0 = 0.0f, l1 = 0.0f;
    const bool lens = !(c.focus_distance == 0 || c.focus_angle == 0);
    if (sx) {
        const uint32_t spp = sx * sy;
        // getPixel2D at dimension 0: x + (stratum x + dx) / xSamples, in double
        uint32_t st = stratum_of(x, y, 0, idx, spp);
        pxf = (float)((double)x + ((double)(int)(st % sx) + (double)a) / (double)sx);
        pyf = (float)((double)y + ((double)(int)(st / sx) + (double)b) / (double)sy);
        if (c.has_shutter) {  // get1D at dimension 2: (stratum + u) / spp, in float
            st = stratum_of(x, y, 2, idx, spp);
            tu = ((float)st + draw(key, 2)) / (float)spp;
        }
        if (lens) {  // get2D at dimension 3, handed over as a glm::vec2
            st = stratum_of(x, y, 3, idx, spp);
            l0 = (float)(((double)(int)(st % sx) + (double)draw(key, 3)) / (double)sx);
            l1 = (float)(((double)(int)(st / sx) + (double)draw(key, 4)) / (double)sy);
        }
    } else {
        pxf = (float)x + a;  // == float(double(x) + a): both round the exact sum
        pyf = (float)y + b;
        if (c.has_shutter) tu = draw(key, 2);
        if (lens) {
            l0 = draw(key, 3);
            l1 = draw(key, 4);
        }
    }
    // t = glm::mix(shutterStart, shutterEnd, time) (Camera.hpp:25) as
    // TileIntegrator::Render's copy rounds it, fma(start, 1 - u, u * end); a
    // camera without a shutter: 0
    time = c.has_shutter ? fma_(c.shutter[0], 1.0f - tu, rmul(tu, c.shutter[1])) : 0.0f;
    float uc = pxf / (float)c.width;
    float vc = pyf / (float)c.height;
    f3 U = F3(c.u[0], c.u[1], c.u[2]), Vv = F3(c.v[0], c.v[1], c.v[2]), W = F3(c.w[0], c.w[1], c.w[2]);
    // fma(b, v, fma(a, u, -w)) as the reference build contracts it (fixture search)
    const float ca = (2.0f * uc - 1.0f) * c.half_width, cb = (2.0f * vc - 1.0f) * c.half_height;
    f3 dir = normalize(F3(fma_(cb, Vv.x, fma_(ca, U.x, -W.x)), fma_(cb, Vv.y, fma_(ca, U.y, -W.y)),
                          fma_(cb, Vv.z, fma_(ca, U.z, -W.z))));
    f3 org = F3(c.origin[0], c.origin[1], c.origin[2]);
    if (!lens) {
        o = org;
        d = dir;
        return;
    }
    float r = csqrt(l0);
    float th = 2 * PT_PI * l1;
    float lx = r * cos_cr(th), ly = r * sin_cr(th);
    f3 du = c.defocus_radius * U, dv = c.defocus_radius * Vv;
    dir = dir * c.focus_distance;
    // pLens.x * du + pLens.y * dv with the second product fused (as built)
    f3 off = F3(fma_(dv.x, ly, du.x * lx), fma_(dv.y, ly, du.y * lx), fma_(dv.z, ly, du.z * lx));
    o = org + off;
    d = normalize(dir - off);
}

// FilmTile::Add's pixelSample = glm::fract(p) of a camera sample (Film.hpp:
// 65-67), recomputed by the film gathers from the sample's stream: the jitter
// itself (x + a is exact in double), or a StratifiedSampler's stratum +
// jitter, p = x + (sx + a) / xSamples rounded in double as camera_ray forms it
__device__ __forceinline__ void sample_fract(const RenderParams& R, uint32_t key, uint32_t x, uint32_t y, uint32_t s,
                                             double& fx, double& fy) {
    const float a = draw(key, 0), b = draw(key, 1);
    if (R.strata_x) {
        const uint32_t spp = R.strata_x * R.strata_y;
        const uint32_t st = stratum_of(x, y, 0, s % spp, spp);
        const double px = (double)x + ((double)(int)(st % R.strata_x) + (double)a) / (double)R.strata_x;
        const double py = (double)y + ((double)(int)(st / R.strata_x) + (double)b) / (double)R.strata_y;
        fx = px - floor(px);
        fy = py - floor(py);
    } else {
        fx = (double)a;  // fract(x + a) = a, a in [0,1)
        fy = (double)b;
    }
}

struct NewSample {
    bool enq;
    uint32_t sid, key;
    f3 o, d;
    float time;
};
// Camera::GenerateRay for chunk sample ns.sid (its pixel in the chunk's work
// order, its stream key)
__device__ __forceinline__ void camera_sample(const RenderParams& R, NewSample& ns) {
    const unsigned long long g = ns.sid;
    const uint32_t s_rel = (uint32_t)(g / R.npix_work), pix_i = (uint32_t)(g % R.npix_work);
    uint32_t x, y;
    work_pixel(R, pix_i, x, y);
    const uint32_t s = R.shard_index + (R.s_lo + s_rel) * R.shard_count;
    ns.key = stream_key(R.seed, y * (uint32_t)R.cam.width + x, s);
    camera_ray(R.cam, ns.key, x, y, ns.o, ns.d, ns.time, R.strata_x, R.strata_y,
               R.strata_x ? s % (R.strata_x * R.strata_y) : 0u);
}
// One new camera sample per `want` lane: a block-aggregated claim of
// consecutive sample ids (one returning atomic per block: coherent primary
// rays), then Camera::GenerateRay for the claimed ids below the chunk's end.
// Every thread of the block calls it (barriers).
__device__ __forceinline__ NewSample claim_camera_sample(const RenderParams& R, bool want,
                                                         unsigned long long* __restrict__ next_sample) {
    __shared__ uint32_t s_w[17];  // up to 1024 threads per block
    __shared__ unsigned long long s_base;
    const uint64_t m = __ballot(want);
    const uint32_t wave = threadIdx.x >> 6;
    if (__lane_id() == 0) s_w[wave] = (uint32_t)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); w++) {
            uint32_t c = s_w[w];
            s_w[w] = tot;
            tot += c;
        }
        s_base = tot ? atomicAdd(next_sample, (unsigned long long)tot) : 0ull;
    }
    __syncthreads();
    const unsigned long long g = s_base + s_w[wave] + lanemask_lt_count(m);
    NewSample ns{want && g < R.chunk_total, (uint32_t)g, 0u, F3(0, 0, 0), F3(0, 0, 0), 0.0f};
    if (ns.enq) camera_sample(R, ns);
    return ns;
}
__device__ __forceinline__ float4 f4_of(f3 v) { return make_float4(v.x, v.y, v.z, 0.0f); }
__device__ __forceinline__ void store_camera_path(PathSoA& next, uint32_t at, const NewSample& ns, int cam_medium) {
    next.o[at] = make_float4(ns.o.x, ns.o.y, ns.o.z, __uint_as_float(ns.key));
    // depth 1 (first loop test passed), spec = true, the camera's medium (Camera.hpp:27, 34)
    next.d[at] = make_float4(ns.d.x, ns.d.y, ns.d.z, __uint_as_float(1u | PF_SPEC | medium_bits(cam_medium)));
    next.beta[at] = make_float4(1.0f, 1.0f, 1.0f, 1.0f);  // attenuation, prevPDF = 1
    next.L[at] = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(5u));  // camera used dims 0..4
    next.sid[at] = ns.sid;
    if (S.motion) next.time[at] = ns.time;
}

// Initial fill of a chunk's wavefront: one camera sample per entry.  Later
// refills happen in k_shade, where paths finish.  maxDepth 0 never gets here:
// the runtime zero-fills.
// The chunk's initial fill.  Both counters start at zero (the runtime clears
// them), so path slot i takes chunk sample i directly and one thread books
// the whole fill: the block-aggregated claims and appends the refills use
// would be two returning atomics per block on one address each (4 M for
// 512 M paths, which was the launch's whole cost: C4 k_fill 25 ms).
__global__ __launch_bounds__(256) void k_fill(RenderParams R, uint32_t n, PathSoA next, uint32_t* __restrict__ cnt,
                                             unsigned long long* __restrict__ next_sample) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const uint32_t m = (uint32_t)min((unsigned long long)n, R.chunk_total);
    if (i == 0) {
        atomicAdd(next_sample, (unsigned long long)m);
        atomicAdd(&cnt[Q_NEXT], m);
    }
    if (i >= m) return;
    NewSample ns{true, i, 0u, F3(0, 0, 0), F3(0, 0, 0), 0.0f};
    camera_sample(R, ns);
    store_camera_path(next, i, ns, R.cam.medium);
}

// ------------------------------------------------------------------ shading
// PathIntegrator::SampleLd (Integrators.cpp:260-294) at the interaction si
// with the hit's textures mt: the light pick (r5), its sample (r2, r3), the
// BSDF value and MIS weight -> the shadow record (occlusion deferred).  False
// when it contributes nothing.  dim: the bounce's dimension after its 8 draws.
// li: the light LightSampler::Sample(r5) picked (ls_sample)
__device__ __forceinline__ bool sample_ld(const MatTex& mt, const SurfInt& si, f3 rd, f3 att, float r2, float r3,
                                          int li, uint32_t key, uint32_t dim, float tm, ShadowRec& srec) {
    if (li < 0) return false;
    const pt_light& l = S.lights[li];
    const LSample ls = light_sample(li, r2, r3, texinf_uc(key, dim), tm);
    f3 ldir;
    float tmax;
    if (is_zero(ls.n)) {
        ldir = ls.dir;
        tmax = __int_as_float(0x7f800000);
    } else {
        ldir = ls.p - si.p;
        tmax = length(ldir) - PT_EPS;
    }
    const f3 sd = normalize(ldir);
    float lpdf = l.pmf;
    const float dt = dot_yxz(si.ns, sd);  // as built: y, x, z order
    if (lpdf <= 0 || dt * dot(rd, si.ns) >= 0) return false;
    const f3 f = mat_f(mt, rd, si, sd) * fabsf(dt);
    f3 c;
    if (light_is_delta(l)) {
        c = (ls.L * f) / lpdf;
    } else {
        lpdf *= light_pdf(li, ls.p, ls.n, si.p, sd, tm);
        if (lpdf <= 0) return false;
        const float w2 = lpdf * lpdf;
        const float w1 = mat_pdf(mt, rd, si, sd);
        const float wl = w2 / fma_(w1, w1, w2);  // w1*w1 + w2 fused
        c = ((light_L(l, ls.n, ls.u, ls.v, sd, tm) * f) * wl) / lpdf;
    }
    if (is_zero(c)) return false;
    srec.o = make_float4(si.p.x, si.p.y, si.p.z, tmax);
    srec.d = make_float4(sd.x, sd.y, sd.z, 0.0f);
    srec.c = make_float4(c.x, c.y, c.z, 0.0f);
    srec.a = make_float4(att.x, att.y, att.z, 0.0f);
    return true;
}

// One bounce of PathIntegrator::Li / SimplePathIntegrator::Li for one path
// (Integrators.cpp:131-294): the closest hit h = (t, b1, b2, prim) of the ray
// (ro, rd) is shaded, emission and the NEE sample drawn, the next ray sampled.
// In: the path's state (f0 = depth | rr | spec flags); out: the next state,
// cont / done, and the NEE shadow record when `shadow`.  k_shade runs it over
// the wavefront, k_tail per lane in a loop.  NEE false (PT_SHADE_SPLIT): no
// SampleLd here, `shadow` marks the bounces k_shade_nee samples it for.
template <int INTEGRATOR, bool NEE = true>
__device__ __forceinline__ void shade_bounce(const RenderParams& R, float4 h, uint32_t f0, f3& ro, f3& rd, f3& att,
                                             f3& out, float& prev, uint32_t key, uint32_t& dim, uint32_t& flags,
                                             bool& cont, bool& done, bool& shadow, ShadowRec& srec, float tm) {
    uint32_t depth = f0 & PF_DEPTH_MASK, rr = (f0 >> PF_RR_SHIFT) & PF_DEPTH_MASK;
    bool spec = (f0 & PF_SPEC) != 0;
    const int prim = __float_as_int(h.w);
    bool alive = true;
    if (prim < 0) {
        // miss: infinite lights (Integrators.cpp:140-145, 196-208)
        for (uint32_t k = 0; k < S.n_infinite_lights; k++) {
            const pt_light& l = S.lights[S.infinite_lights[k]];
            // as built: out += att * Le fused; lp*lp + p*p and out += (Le*att)*w fused
            if (INTEGRATOR == PT_INTEGRATOR_SIMPLE || spec) {
                out = fma3(inf_le(l, rd), att, out);
            } else if (prev > 0) {
                const float lp = l.pmf * inf_pdf(l, rd), p2 = prev * prev;
                const float w = p2 / fma_(lp, lp, p2);
                out = fma3s(w, inf_le(l, rd) * att, out);
            }
        }
        alive = false;
    } else {
        float r[8];
        if (INTEGRATOR == PT_INTEGRATOR_PATH) {
#pragma unroll
            for (int k = 0; k < 8; k++) r[k] = draw(key, dim + k);
            dim += 8;
        } else {
#pragma unroll
            for (int k = 0; k < 4; k++) r[k] = draw(key, dim + k);
            dim += 4;
        }
        SurfInt si;
        int smed;
        MatTex mte;
        hit_surface(prim, ro, rd, h.x, h.y, h.z, si, smed, tm, PT_MT_EARLY ? &mte : nullptr);
        // emission (Integrators.cpp:151-154, 217-226)
        if (si.light >= 0) {
            const pt_light& al = S.lights[si.light];
            f3 Le = light_L(al, si.n, si.u, si.v, rd, tm);
            if (!is_zero(Le)) {
                if (INTEGRATOR == PT_INTEGRATOR_SIMPLE || spec) {
                    out = fma3(Le, att, out);
                } else if (prev > 0) {
                    const float lp = al.pmf * light_pdf(si.light, si.p, si.n, ro, rd, tm), p2 = prev * prev;
                    const float w = p2 / fma_(lp, lp, p2);
                    out = fma3s(w, Le * att, out);
                }
            }
        }
        if (si.mat < 0) {
            // medium boundary: pass through (Integrators.cpp:156-159, 228-232)
            if (INTEGRATOR == PT_INTEGRATOR_PATH) spec = true;
            ro = at_f(ro, rd, si.t);
        } else {
            const float us = INTEGRATOR == PT_INTEGRATOR_PATH ? r[4] : r[2];
            const MatTex mt = PT_MT_EARLY ? mte : mat_tex(si.mat, si);  // the hit's textures, read once
            const Bxdf b = mat_scatter(mt, ro, rd, si, us, r[0], r[1]);
            if (!b.ok) {
                alive = false;  // absorbed
            } else {
                if (INTEGRATOR == PT_INTEGRATOR_PATH) {
                    spec = (b.flags & FL_SPEC) != 0;
                    if (!spec) {
                        // PathIntegrator::SampleLd (Integrators.cpp:260-294); occlusion
                        // deferred.  A split bounce (NEE false) leaves it to
                        // k_shade_nee: `shadow` then marks a NEE job.
                        // (the light pick drawn at the start of the bounce instead, so
                        // its reads overlap the interaction's: -1.4 %, 12 spilled
                        // VGPRs; profiles/r06_ab_shade_chain.txt)
                        if (NEE) shadow = sample_ld(mt, si, rd, att, r[2], r[3], ls_sample(r[5]), key, dim, tm, srec);
                        else shadow = true;
                        prev = mat_pdf(mt, rd, si, b.d);
                    }
                }
                att = att * ((b.f * fabsf(dot(si.ns, b.d))) / b.pdf);
                const float urr = INTEGRATOR == PT_INTEGRATOR_PATH ? r[6] : r[3];
                if (rr++ > 3) {
                    float qq = fminf(0.95f, fmaxf(fmaxf(att.x, att.y), att.z));
                    if (urr >= qq) alive = false;
                    else att = att / qq;
                }
                ro = b.o;
                rd = b.d;
            }
        }
    }
    // loop test `depth++ < maxDepth && sum(att) > 0` (Integrators.cpp:138, 193)
    // (both flags assigned: a store to one of the two through a selected
    // pointer would keep them in scratch memory)
    const bool go = alive && depth < R.max_depth && (att.x + att.y + att.z) > 0.0f;
    depth += go ? 1u : 0u;
    cont = go;
    done = !go;
    flags = depth | (rr << PF_RR_SHIFT) | (spec ? PF_SPEC : 0u);
}

template <int INTEGRATOR>
#ifndef PT_SHADE_WPE  // waves-per-SIMD budget for k_shade (pt_kernels.h PT_SHADE_BLOCK)
#define PT_SHADE_WPE 4
#endif
#define PT_SHADE_WAVES __attribute__((amdgpu_waves_per_eu(PT_SHADE_WPE, PT_SHADE_WPE)))
__global__ __launch_bounds__(PT_SHADE_BLOCK) PT_SHADE_WAVES void k_shade(RenderParams R, PathSoA cur, const uint32_t* __restrict__ nptr,
                                              const float4* __restrict__ hit, PathSoA next,
                                              float* __restrict__ sample_L,
                                              unsigned long long* __restrict__ next_sample,
                                              ShadowRec* __restrict__ sq, uint32_t* __restrict__ cnt) {
    const uint32_t n = path_count(nptr), front = nptr[Q_NEXT];
    if (blockIdx.x * PT_SHADE_BLOCK >= n) return;  // block-uniform: the grid covers the capacity
    const uint32_t t = blockIdx.x * PT_SHADE_BLOCK + threadIdx.x;
    const uint32_t i = (R.order && t < n) ? R.order[t] : t;  // material-sorted order, or the path order
    bool cont = false, done = false, shadow = false;
    ShadowRec srec;
    f3 ro = F3(0, 0, 0), rd = F3(0, 0, 0), att = F3(0, 0, 0), out = F3(0, 0, 0);
    float prev = 0, tm = 0;
    uint32_t key = 0, dim = 0, flags = 0, sid = 0;
    if (i < n) {
        const uint32_t e = path_slot(i, front, cur.cap);
        const float4 o4 = cur.o[e], d4 = cur.d[e], b4 = cur.beta[e], L4 = cur.L[e];
        const float4 h = hit[i];
        sid = cur.sid[e];
        if (S.motion) tm = cur.time[e];
        ro = xyz(o4);
        rd = xyz(d4);
        att = xyz(b4);
        out = xyz(L4);
        prev = b4.w;
        key = __float_as_uint(o4.w);
        dim = __float_as_uint(L4.w);
        shade_bounce<INTEGRATOR, !(PT_SHADE_SPLIT && INTEGRATOR == PT_INTEGRATOR_PATH)>(
            R, h, __float_as_uint(d4.w), ro, rd, att, out, prev, key, dim, flags, cont, done, shadow, srec, tm);
    }
    constexpr bool split = PT_SHADE_SPLIT && INTEGRATOR == PT_INTEGRATOR_PATH;
    // a finished path stores its sample's radiance (the pending NEE ray, if
    // any, adds to it later) and its entry takes the next camera sample
    if (done) {
        float* o = sample_L + 3ull * sid;
        o[0] = out.x;
        o[1] = out.y;
        o[2] = out.z;
    }
    // (the claim and the appends in one barrier round measured equal,
    // profiles/r05_ab_shade_block.txt)
    uint32_t at[3];
    const NewSample ns = claim_camera_sample(R, done, next_sample);
    const int qoff[3] = {Q_NEXT, split ? Q_NEE : Q_SHADOW, Q_NEW};
    const bool pred[3] = {cont, shadow, ns.enq};
    block_append<3, PT_SHADE_BLOCK>(cnt, qoff, pred, at);
    const uint32_t a = cont ? at[0] : next.cap - 1u - at[2], c = at[1];
    if (cont) {
        next.o[a] = make_float4(ro.x, ro.y, ro.z, __uint_as_float(key));
        next.d[a] = make_float4(rd.x, rd.y, rd.z, __uint_as_float(flags));
        next.beta[a] = make_float4(att.x, att.y, att.z, prev);
        next.L[a] = make_float4(out.x, out.y, out.z, __uint_as_float(dim));
        next.sid[a] = sid;
        if (S.motion) next.time[a] = tm;
    } else if (ns.enq) {
        store_camera_path(next, a, ns, R.cam.medium);
    }
    if (shadow && split) {
        R.nee_jobs[c] = make_uint2(i, cont ? a : (SHADOW_DONE_BIT | sid));
    } else if (shadow) {
        srec.d.w = __uint_as_float(cont ? a : (SHADOW_DONE_BIT | sid));
        sq[c] = srec;
        if (S.motion) S.sq_time[c] = tm;  // the shadow ray's time (Integrators.cpp:274)
    }
}

// The NEE half of a split PathIntegrator bounce (PT_SHADE_SPLIT): per job
// {path index in cur, shadow target} that k_shade appended, the hit's
// interaction and textures again (hit_surface, mat_tex: the same values) and
// SampleLd (sample_ld) with the bounce's draws 2, 3, 5 -> the shadow record.
// cur, hit and the path's attenuation are those k_shade read (it writes the
// next state elsewhere).
#ifndef PT_NEE_WPE
#define PT_NEE_WPE 4
#endif
__global__ __launch_bounds__(PT_SHADE_BLOCK) __attribute__((amdgpu_waves_per_eu(PT_NEE_WPE, PT_NEE_WPE)))
void k_shade_nee(RenderParams R, PathSoA cur, const uint32_t* __restrict__ nptr, const float4* __restrict__ hit,
                 ShadowRec* __restrict__ sq, uint32_t* __restrict__ cnt) {
    const uint32_t n = cnt[Q_NEE], front = nptr[Q_NEXT];
    if (blockIdx.x * PT_SHADE_BLOCK >= n) return;  // block-uniform: the grid covers the capacity
    const uint32_t t = blockIdx.x * PT_SHADE_BLOCK + threadIdx.x;
    bool shadow = false;
    ShadowRec srec;
    float tm = 0;
    if (t < n) {
        const uint2 job = R.nee_jobs[t];
        const uint32_t i = job.x, e = path_slot(i, front, cur.cap);
        const float4 o4 = cur.o[e], d4 = cur.d[e], b4 = cur.beta[e], L4 = cur.L[e];
        const float4 h = hit[i];
        if (S.motion) tm = cur.time[e];
        const f3 ro = xyz(o4), rd = xyz(d4);
        const uint32_t key = __float_as_uint(o4.w), dim0 = __float_as_uint(L4.w);
        SurfInt si;
        int smed;
        hit_surface(__float_as_int(h.w), ro, rd, h.x, h.y, h.z, si, smed, tm);
        const MatTex mt = mat_tex(si.mat, si);
        shadow = sample_ld(mt, si, rd, xyz(b4), draw(key, dim0 + 2), draw(key, dim0 + 3), ls_sample(draw(key, dim0 + 5)),
                           key, dim0 + 8, tm, srec);
        srec.d.w = __uint_as_float(job.y);
    }
    uint32_t c[1];
    const int qoff[1] = {Q_SHADOW};
    const bool pred[1] = {shadow};
    block_append<1, PT_SHADE_BLOCK>(cnt, qoff, pred, c);
    if (shadow) {
        sq[c[0]] = srec;
        if (S.motion) S.sq_time[c[0]] = tm;
    }
}

// The wavefront's tail (Path / SimplePath, fixed SPP): once every camera
// sample of the chunk has started and few paths remain, one launch finishes
// them, each lane looping over its own path's bounces -- the closest hit
// (trace_closest over the reference's clusters, its own order and ties), the
// bounce (shade_bounce, as k_shade), the NEE ray (trace_any) and its
// contribution fma(c, att, out) right after the bounce that drew it, as
// k_shadow_pool adds it.  A wavefront iteration per bounce would cost a
// handful of launches and a bounce-wide wait for the slowest ray each (C4:
// the last ~127 bounces took ~97 ms of a 6.2 s frame).
template <int INTEGRATOR, bool INST, bool COUNT>
__global__ __launch_bounds__(PT_TRACE_BLOCK) void k_tail(RenderParams R, PathSoA cur,
                                                         const uint32_t* __restrict__ nptr,
                                                         float* __restrict__ sample_L,
                                                         unsigned long long* counters) {
    __shared__ uint32_t s_ref[PT_STACK * PT_TRACE_BLOCK];
    const uint32_t n = path_count(nptr), front = nptr[Q_NEXT];
    TraceWork wc{0, 0}, wa{0, 0};
    uint64_t n_cl = 0, n_any = 0;
    for (uint32_t i = blockIdx.x * PT_TRACE_BLOCK + threadIdx.x; i < n; i += gridDim.x * PT_TRACE_BLOCK) {
        const uint32_t e = path_slot(i, front, cur.cap);
        const float4 o4 = cur.o[e], d4 = cur.d[e], b4 = cur.beta[e], L4 = cur.L[e];
        const uint32_t sid = cur.sid[e];
        f3 ro = xyz(o4), rd = xyz(d4), att = xyz(b4), out = xyz(L4);
        float prev = b4.w;
        const uint32_t key = __float_as_uint(o4.w);
        uint32_t dim = __float_as_uint(L4.w), flags = __float_as_uint(d4.w);
        const float tm = S.motion ? cur.time[e] : 0.0f;
        for (;;) {
            float t = 0, b1 = 0, b2 = 0;
            const int prim = trace_closest<COUNT, INST>(ro, rd, __int_as_float(0x7f800000), t, b1, b2, s_ref, wc,
                                                        nullptr, tm);
            ++n_cl;
            bool cont = false, done = false, shadow = false;
            ShadowRec srec;
            shade_bounce<INTEGRATOR>(R, make_float4(t, b1, b2, __int_as_float(prim)), flags, ro, rd, att, out, prev,
                                     key, dim, flags, cont, done, shadow, srec, tm);
            if (shadow) {
                ++n_any;
                if (!trace_any<COUNT, INST>(xyz(srec.o), xyz(srec.d), srec.o.w, s_ref, wa, nullptr, tm))
                    out = F3(fma_(srec.c.x, srec.a.x, out.x), fma_(srec.c.y, srec.a.y, out.y),
                             fma_(srec.c.z, srec.a.z, out.z));
            }
            if (!cont) break;
        }
        float* o = sample_L + 3ull * sid;
        o[0] = out.x;
        o[1] = out.y;
        o[2] = out.z;
    }
    count_add(counters, CNT_TAIL_CLOSEST, n_cl);
    count_add(counters, CNT_TAIL_ANY, n_any);
    // the previous bounce's NEE rays: its any-hit kernel traced them, and the
    // next iteration's snapshot (which the tail replaces) would have counted them
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&counters[CNT_TAIL_ANY], (unsigned long long)nptr[Q_SHADOW]);
    if (COUNT) {
        count_add(counters, CNT_NODES_CLOSEST, wc.nodes);
        count_add(counters, CNT_TRIS_CLOSEST, wc.tris);
        count_add(counters, CNT_NODES_ANY, wa.nodes);
        count_add(counters, CNT_TRIS_ANY, wa.tris);
    }
}

// ------------------------------------------------------------------ VolPathIntegrator
// GeometricInteraction::getMedium (Interaction.hpp:26-29)
__device__ __forceinline__ int get_medium(const SurfInt& si, int medium, f3 dir) {
    return dot(dir, si.n) < 0 ? medium : -1;
}

// One body of VolPathIntegrator::Li (Integrators.cpp:296-413).  Draw order per
// bounce: the medium's (channel, distance) when the ray is in a medium, then
// get2Dx4f() + get1D().  NEE (VolPathIntegrator::SampleLd, 416-479) becomes a
// shadow record whose transmittance k_shadow_tr accumulates (Scene::IntersectTr).
__global__ __launch_bounds__(256) void k_shade_vol(RenderParams R, PathSoA cur, const uint32_t* __restrict__ nptr,
                                                  const float4* __restrict__ hit, PathSoA next,
                                                  float* __restrict__ sample_L,
                                                  unsigned long long* __restrict__ next_sample,
                                                  ShadowRecV* __restrict__ sq, uint32_t* __restrict__ cnt) {
    const uint32_t n = path_count(nptr), front = nptr[Q_NEXT];
    if (blockIdx.x * 256 >= n) return;  // block-uniform: the grid covers the capacity
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    const uint32_t i = (R.order && t < n) ? R.order[t] : t;  // material-sorted order, or the path order
    bool cont = false, done = false, shadow = false;
    ShadowRecV srec;
    f3 ro = F3(0, 0, 0), rd = F3(0, 0, 0), att = F3(0, 0, 0), out = F3(0, 0, 0);
    float prev = 0, tm = 0;
    uint32_t key = 0, dim = 0, flags = 0, sid = 0;
    if (i < n) {
        const uint32_t e = path_slot(i, front, cur.cap);
        const float4 o4 = cur.o[e], d4 = cur.d[e], b4 = cur.beta[e], L4 = cur.L[e];
        const float4 h = hit[i];
        sid = cur.sid[e];
        if (S.motion) tm = cur.time[e];
        ro = xyz(o4);
        rd = xyz(d4);
        att = xyz(b4);
        out = xyz(L4);
        prev = b4.w;
        key = __float_as_uint(o4.w);
        dim = __float_as_uint(L4.w);
        const uint32_t f0 = __float_as_uint(d4.w);
        uint32_t depth = f0 & PF_DEPTH_MASK, rr = (f0 >> PF_RR_SHIFT) & PF_DEPTH_MASK;
        bool spec = (f0 & PF_SPEC) != 0;
        int med = flags_medium(f0);
        const int prim = __float_as_int(h.w);
        bool alive = true, do_rr = true;
        if (prim < 0) {
            // miss: infinite lights, no medium attenuation (Integrators.cpp:308-329)
            for (uint32_t k = 0; k < S.n_infinite_lights; k++) {
                const pt_light& l = S.lights[S.infinite_lights[k]];
                if (spec) {
                    out = fma3(inf_le(l, rd), att, out);
                } else if (prev > 0) {
                    const float lp = l.pmf * inf_pdf(l, rd), p2 = prev * prev;
                    const float w = p2 / fma_(lp, lp, p2);
                    out = fma3s(w, inf_le(l, rd) * att, out);
                }
            }
            alive = false;
        } else {
            SurfInt si;
            int smed;
            hit_surface(prim, ro, rd, h.x, h.y, h.z, si, smed, tm);
            if (med < 0) med = S.scene_medium;
            bool mvalid = false;
            f3 mp = F3(0, 0, 0);
            if (med >= 0) {
                const float u0 = draw(key, dim), u1 = draw(key, dim + 1);
                dim += 2;
                att = att * medium_sample(S.media[med], ro, rd, si.t, u0, u1, mvalid, mp);
            }
            float r[9];
#pragma unroll
            for (int k = 0; k < 9; k++) r[k] = draw(key, dim + k);
            dim += 9;
            // NEE (SampleLd): from the medium point with the phase function, or
            // from the surface with the BSDF; shadow ray in the current medium
            bool nee = false, nee_medium = false;
            if (mvalid) {
                const pt_medium& M = S.media[med];
                nee = true;
                nee_medium = true;
                // output += att * Le (Integrators.cpp:357) comes after SampleLd's
                // term: the shadow record carries it (SHADOW_MLE_BIT), else below
                (void)M;
                si.p = mp;
            } else {
                if (si.light >= 0) {
                    const pt_light& al = S.lights[si.light];
                    f3 Le = light_L(al, si.n, si.u, si.v, rd, tm);
                    if (!is_zero(Le)) {
                        if (spec) {
                            out = fma3(att, Le, out);
                        } else if (prev > 0) {
                            const float lp = al.pmf * light_pdf(si.light, si.p, si.n, ro, rd, tm), p2 = prev * prev;
                            const float w = p2 / fma_(lp, lp, p2);
                            out = fma3s(w, att * Le, out);
                        }
                    }
                }
            }
            Bxdf b;
            b.ok = false;
            MatTex mt{};
            if (!mvalid && si.mat >= 0) {
                mt = mat_tex(si.mat, si);  // the hit's textures, read once
                b = mat_scatter(mt, ro, rd, si, r[4], r[0], r[1]);
                if (b.ok && !(b.flags & FL_SPEC)) nee = true;
            }
            if (nee) {
                const int li = ls_sample(r[5]);
                if (li >= 0 && S.lights[li].pmf > 0) {
                    const pt_light& l = S.lights[li];
                    LSample ls = light_sample(li, r[2], r[3], texinf_uc(key, dim), tm);
                    f3 ldir;
                    float tmax;
                    if (is_zero(ls.n)) {
                        ldir = ls.dir;
                        tmax = __int_as_float(0x7f800000);
                    } else {
                        ldir = ls.p - si.p;
                        tmax = length(ldir) - PT_EPS;
                        tmax -= PT_EPS;
                    }
                    const f3 sd = normalize(ldir);
                    float lpdf = l.pmf;
                    f3 f;
                    float spdf;
                    bool ok = true;
                    if (nee_medium) {
                        spdf = phase_hg(dot(rd, sd), S.media[med].g);
                        f = F3(spdf, spdf, spdf);
                    } else {
                        const float dt = dot(si.ns, sd);
                        ok = !(dt * dot(rd, si.ns) >= 0);
                        spdf = ok ? mat_pdf(mt, rd, si, sd) : 0.0f;
                        f = ok ? mat_f(mt, rd, si, sd) * fabsf(dt) : F3(0, 0, 0);
                    }
                    if (ok && !is_zero(f)) {
                        // the shadow kernel forms ((Tr * L) * f * w) / pdf
                        f3 Ll;
                        float wl = 1.0f;
                        if (light_is_delta(l)) {
                            Ll = ls.L;
                        } else {
                            lpdf *= light_pdf(li, ls.p, ls.n, si.p, sd, tm);
                            if (lpdf <= 0) {
                                ok = false;
                            } else {
                                const float w2 = lpdf * lpdf;
                                wl = w2 / fma_(spdf, spdf, w2);  // spdf*spdf + w2 fused
                                Ll = light_L(l, ls.n, ls.u, ls.v, sd, tm);
                            }
                        }
                        if (ok) {
                            shadow = true;
                            srec.o = make_float4(si.p.x, si.p.y, si.p.z, tmax);
                            srec.d = make_float4(sd.x, sd.y, sd.z, __uint_as_float(nee_medium ? SHADOW_MLE_BIT : 0u));
                            srec.L = make_float4(Ll.x, Ll.y, Ll.z, __int_as_float(med));
                            srec.f = make_float4(f.x, f.y, f.z, wl);
                            srec.a = make_float4(att.x, att.y, att.z, lpdf);
                        }
                    }
                }
            }
            if (mvalid && !shadow) out = fma3(att, ld3(S.media[med].Le), out);
            if (mvalid) {
                // phase scattering (Integrators.cpp:358-361)
                const f3 sc = phase_sample(S.media[med].g, rd, r[6], r[7]);
                const int nm = get_medium(si, smed, sc);
                ro = mp;
                rd = sc;
                med = nm;
                spec = false;
            } else {
                spec = false;
                if (si.mat < 0) {
                    // medium boundary: pass through, no RR (Integrators.cpp:378-382)
                    ro = at_f(ro, rd, si.t);
                    med = get_medium(si, smed, rd);
                    do_rr = false;
                } else if (!b.ok) {
                    alive = false;  // absorbed
                } else {
                    int nm = get_medium(si, smed, b.d);
                    if (!(b.flags & FL_TRANS) && dot(rd, si.ns) <= 0) nm = med;
                    spec = (b.flags & FL_SPEC) != 0;
                    if (!spec) prev = mat_pdf(mt, rd, si, b.d);
                    att = att * ((b.f * fabsf(dot(si.ns, b.d))) / b.pdf);
                    ro = b.o;
                    rd = b.d;
                    med = nm;
                }
            }
            if (alive && do_rr && rr++ > 3) {
                float qq = fminf(0.95f, fmaxf(fmaxf(att.x, att.y), att.z));
                if (r[8] >= qq) alive = false;
                else att = att / qq;
            }
        }
        if (alive && depth < R.max_depth && (att.x + att.y + att.z) > 0.0f) {
            depth++;
            cont = true;
        } else {
            done = true;
        }
        flags = depth | (rr << PF_RR_SHIFT) | (spec ? PF_SPEC : 0u) | medium_bits(med);
    }
    if (done) {
        float* o = sample_L + 3ull * sid;
        o[0] = out.x;
        o[1] = out.y;
        o[2] = out.z;
    }
    const NewSample ns = claim_camera_sample(R, done, next_sample);
    const int qoff[3] = {Q_NEXT, Q_SHADOW, Q_NEW};
    const bool pred[3] = {cont, shadow, ns.enq};
    uint32_t at[3];
    block_append<3, 256>(cnt, qoff, pred, at);
    const uint32_t a = cont ? at[0] : next.cap - 1u - at[2], c = at[1];
    if (cont) {
        next.o[a] = make_float4(ro.x, ro.y, ro.z, __uint_as_float(key));
        next.d[a] = make_float4(rd.x, rd.y, rd.z, __uint_as_float(flags));
        next.beta[a] = make_float4(att.x, att.y, att.z, prev);
        next.L[a] = make_float4(out.x, out.y, out.z, __uint_as_float(dim));
        next.sid[a] = sid;
        if (S.motion) next.time[a] = tm;
    } else if (ns.enq) {
        store_camera_path(next, a, ns, R.cam.medium);
    }
    if (shadow) {
        srec.d.w = __uint_as_float((cont ? a : (SHADOW_DONE_BIT | sid)) | (__float_as_uint(srec.d.w) & SHADOW_MLE_BIT));
        sq[c] = srec;
        if (S.motion) S.sq_time[c] = tm;  // the shadow ray's time (Integrators.cpp:447)
    }
}

// NEE shadow rays of VolPath: Scene::IntersectTr (Scene.cpp:8-29) — closest
// hits along the segment, passing medium boundaries (no material) and
// multiplying the transmittance of the media crossed; a surface with a
// material occludes.  One ray per lane (media scenes are small).
template <bool COUNT>
__global__ __launch_bounds__(PT_TRACE_BLOCK) void k_shadow_tr(PathSoA next, float* __restrict__ sample_L,
                                                             const ShadowRecV* __restrict__ sq,
                                                             const uint32_t* __restrict__ nptr,
                                                             unsigned long long* counters) {
    __shared__ uint32_t s_ref[PT_STACK * PT_TRACE_BLOCK];
    const uint32_t n = *nptr;
    if (blockIdx.x * PT_TRACE_BLOCK >= n) return;
    const uint32_t i = blockIdx.x * PT_TRACE_BLOCK + threadIdx.x;
    TraceWork wk{0, 0};
    uint32_t extra = 0;
    if (i < n) {
        const ShadowRecV r = sq[i];
        f3 o = xyz(r.o), d = xyz(r.d);
        float max = r.o.w;
        const float tm = S.motion ? S.sq_time[i] : 0.0f;
        const int med0 = __float_as_int(r.L.w);
        int med = med0;
        f3 Tr = F3(1, 1, 1);
        bool occluded = false;
        bool first = true;
        while (max > 0) {
            if (!first) extra++;
            first = false;
            float t, b1, b2;
            const int prim = trace_closest<COUNT>(o, d, max, t, b1, b2, s_ref, wk, nullptr, tm);
            if (prim < 0) {
                if (med >= 0) Tr = Tr * medium_tr(S.media[med], max);
                break;
            }
            if (med >= 0) Tr = Tr * medium_tr(S.media[med], t);
            if (S.info[hit_slot(prim)].material >= 0) {  // (an instance's hit: a virtual slot)
                occluded = true;
                break;
            }
            SurfInt si;
            int smed;
            hit_surface(prim, o, d, t, b1, b2, si, smed, tm);
            o = at_f(o, d, t);
            med = get_medium(si, smed, d);
            max -= t;
        }
        const uint32_t tgt = __float_as_uint(r.d.w);
        const bool mle = (tgt & SHADOW_MLE_BIT) != 0;
        if (!occluded || mle) {
            // out = fma(att, ((Tr * L) * f * w) / pdf, out), then the medium's
            // Le (Integrators.cpp:356-357) — SampleLd's term is 0 when occluded
            const f3 att = xyz(r.a);
            f3 v[2];
            int nv = 0;
            if (!occluded) v[nv++] = (((Tr * xyz(r.L)) * xyz(r.f)) * r.f.w) / r.a.w;
            if (mle) v[nv++] = ld3(S.media[med0].Le);
            float* L3;
            float4* L4 = nullptr;
            f3 out;
            if (tgt & SHADOW_DONE_BIT) {
                L3 = sample_L + 3ull * (tgt & ~(SHADOW_DONE_BIT | SHADOW_MLE_BIT));
                out = F3(L3[0], L3[1], L3[2]);
            } else {
                L4 = &next.L[tgt & ~SHADOW_MLE_BIT];
                out = xyz(*L4);
            }
            for (int k = 0; k < nv; k++) out = fma3(att, v[k], out);
            if (L4) {
                const float4 w = *L4;
                *L4 = make_float4(out.x, out.y, out.z, w.w);
            } else {
                L3[0] = out.x;
                L3[1] = out.y;
                L3[2] = out.z;
            }
        }
    }
    if (COUNT) {
        count_add(counters, CNT_NODES_ANY, wk.nodes);
        count_add(counters, CNT_TRIS_ANY, wk.tris);
    }
    count_add(counters, CNT_EXTRA_ANY, extra);
}

// ------------------------------------------------------------------ film gather
// Filter::Evaluate (Filter.hpp:47-53, 69-75, 93-108) at a float position.
__device__ __forceinline__ double mitchell1(double x, double b, double c) {
    double ax = fabs(x);
    if (ax <= 1.0)
        return 1.0 / 6.0 * ((12 - 9 * b - 6 * c) * ax * ax * ax + (-18 + 12 * b + 6 * c) * ax * ax + (6 - 2 * b));
    if (ax <= 2)
        return 1.0 / 6.0 *
               ((-b - 6 * c) * ax * ax * ax + (6 * b + 30 * c) * ax * ax + (-12 * b - 48 * c) * ax + (8 * b + 24 * c));
    return 0;
}
__device__ __forceinline__ double gauss1(double x, double sigma) {
    return 0.56418958354775628695 / (sigma * 1.41421356237309504880) * exp(-(x * x) / (2 * sigma * sigma));
}
// Sinc / WindowedSinc (Filter.hpp:17-27) in double, as LanczosFilter::Evaluate
// calls them (Filter.hpp:124-126): x promoted from the float position.
__device__ __forceinline__ double sinc1(double x) {
    if (1.0 - x * x == 1.0) return 1.0;
    return sin(3.14159265358979323846 * x) / (3.14159265358979323846 * x);
}
__device__ __forceinline__ double wsinc1(double x, double radius, double tau) {
    if (fabs(x) > radius) return 0.0;
    return sinc1(x) * sinc1(x / tau);
}
__device__ __forceinline__ double filter_eval(const RenderParams& R, float px, float py) {
    if (R.filter == PT_FILTER_BOX) return (fabsf(px) <= R.frad[0] && fabsf(py) <= R.frad[1]) ? 1.0 : 0.0;
    if (R.filter == PT_FILTER_LANCZOS)
        return wsinc1(px, R.frad[0], R.fparam[0]) * wsinc1(py, R.frad[1], R.fparam[0]);
    if (R.filter == PT_FILTER_GAUSSIAN) {
        double gx = gauss1(px, R.fparam[0]) - R.gauss_x, gy = gauss1(py, R.fparam[0]) - R.gauss_y;
        return (gx > 0 ? gx : 0) * (gy > 0 ? gy : 0);
    }
    float ax = 2 * px / R.frad[0];
    float ay = 2 * py / R.frad[1];
    return mitchell1(ax, R.fparam[0], R.fparam[1]) * mitchell1(ay, R.fparam[0], R.fparam[1]);
}

__global__ __launch_bounds__(256) void k_gather(RenderParams R, const float* __restrict__ sample_L,
                                               double* __restrict__ film) {
    const uint32_t tid = blockIdx.x * 256 + threadIdx.x;
    const uint32_t W = (uint32_t)R.cam.width, H = (uint32_t)R.cam.height;
    if (tid >= W * H) return;
    const int x = (int)(tid % W), y = (int)(tid / W);
    double acc[4] = {0, 0, 0, 0};
    const uint32_t ns = R.s_hi - R.s_lo;
    for (int oy = -R.rad_y; oy <= R.rad_y; oy++) {
        for (int ox = -R.rad_x; ox <= R.rad_x; ox++) {
            // source pixel whose samples reach (x, y) with offset (ox, oy)
            const int sx = x - ox, sy = y - oy;
            if (sx < 0 || sy < 0 || sx >= (int)W || sy >= (int)H) continue;
            uint32_t pix_i;
            if (R.tiled) {
                uint32_t tile = (uint32_t)(sy >> 3) * R.tiles_x + (uint32_t)(sx >> 3);
                pix_i = tile * 64u + (uint32_t)((sy & 7) * 8 + (sx & 7));
            } else {
                pix_i = (uint32_t)(sy * (int)W + sx);
            }
            const uint32_t spix = (uint32_t)sy * W + (uint32_t)sx;
            for (uint32_t k = 0; k < ns; k++) {
                const uint32_t s = R.shard_index + (R.s_lo + k) * R.shard_count;
                const uint32_t key = stream_key(R.seed, spix, s);
                // FilmTile::Add: pixelSample = fract(p), sample_pos = (o + 0.5) - fract
                double fx, fy;
                sample_fract(R, key, (uint32_t)sx, (uint32_t)sy, s, fx, fy);
                const double spx = (double)ox + 0.5 - fx, spy = (double)oy + 0.5 - fy;
                const double w = filter_eval(R, (float)spx, (float)spy) * R.inv_integral;
                if (w <= 0) continue;
                const uint64_t g = (uint64_t)k * R.npix_work + pix_i;
                const float* L = sample_L + 3ull * g;
                acc[0] += (double)L[0] * w;
                acc[1] += (double)L[1] * w;
                acc[2] += (double)L[2] * w;
                acc[3] += w;
            }
        }
    }
    double* o = film + 4ull * tid;
    o[0] += acc[0];
    o[1] += acc[1];
    o[2] += acc[2];
    o[3] += acc[3];
}

// The same gather for a whole frame, 16x16 pixels per workgroup: every filter
// above is separable (w = f(px) * f(py) * 1/integral, the product formed as in
// filter_eval), so per sample index the workgroup draws each source pixel's
// jitter once, evaluates its 2*RAD+1 x- and y-weights once into LDS, and every
// target pixel combines them for its (2*RAD+1)^2 neighbours -- instead of
// re-hashing and re-evaluating the filter per (source, target).  Weights are
// bit-identical to k_gather's; the f64 sums run sample-major instead of
// neighbour-major.
// FILT: the filter the tile kernel is built for (-1: any, chosen per call),
// so a launch carries only its own filter's code and registers
template <int FILT = -1>
__device__ __forceinline__ double filter_1d(const RenderParams& R, float p, int axis) {
    const uint32_t f = FILT < 0 ? R.filter : (uint32_t)FILT;
    if (f == PT_FILTER_BOX) return fabsf(p) <= R.frad[axis] ? 1.0 : 0.0;
    if (f == PT_FILTER_LANCZOS) return wsinc1(p, R.frad[axis], R.fparam[0]);
    if (f == PT_FILTER_GAUSSIAN) {
        const double g = gauss1(p, R.fparam[0]) - (axis ? R.gauss_y : R.gauss_x);
        return g > 0 ? g : 0;
    }
    return mitchell1(2 * p / R.frad[axis], R.fparam[0], R.fparam[1]);
}

template <int RAD, int FILT>
__global__ __launch_bounds__(256) void k_gather_tile(RenderParams R, const float* __restrict__ sample_L,
                                                     double* __restrict__ film) {
    constexpr int T = 16, SW = T + 2 * RAD, NS = SW * SW, NW = 2 * RAD + 1;
    __shared__ float s_L[NS][3];
    __shared__ double s_wx[NS][NW], s_wy[NS][NW];
    const int W = R.cam.width, H = R.cam.height;
    const int tx0 = blockIdx.x * T, ty0 = blockIdx.y * T;
    const int lx = threadIdx.x % T, ly = threadIdx.x / T;
    const int x = tx0 + lx, y = ty0 + ly;
    const bool inside = x < W && y < H;
    const int rx = R.rad_x, ry = R.rad_y;
    const uint32_t ns = R.s_hi - R.s_lo;
    double acc[4] = {0, 0, 0, 0};
    for (uint32_t k = 0; k < ns; k++) {
        for (int q = threadIdx.x; q < NS; q += 256) {
            const int sx = tx0 - RAD + q % SW, sy = ty0 - RAD + q / SW;
            float L0 = 0, L1 = 0, L2 = 0;
            double wx[NW], wy[NW];
#pragma unroll
            for (int o = 0; o < NW; o++) wx[o] = wy[o] = 0;
            if (sx >= 0 && sy >= 0 && sx < W && sy < H) {
                uint32_t pix_i;
                if (R.tiled) {
                    const uint32_t tile = (uint32_t)(sy >> 3) * R.tiles_x + (uint32_t)(sx >> 3);
                    pix_i = tile * 64u + (uint32_t)((sy & 7) * 8 + (sx & 7));
                } else {
                    pix_i = (uint32_t)(sy * W + sx);
                }
                const uint32_t spix = (uint32_t)sy * (uint32_t)W + (uint32_t)sx;
                const uint32_t s = R.shard_index + (R.s_lo + k) * R.shard_count;
                const uint32_t key = stream_key(R.seed, spix, s);
                double fx, fy;
                sample_fract(R, key, (uint32_t)sx, (uint32_t)sy, s, fx, fy);
#pragma unroll
                for (int o = -RAD; o <= RAD; o++) {
                    if (o >= -rx && o <= rx) wx[o + RAD] = filter_1d<FILT>(R, (float)((double)o + 0.5 - fx), 0);
                    if (o >= -ry && o <= ry) wy[o + RAD] = filter_1d<FILT>(R, (float)((double)o + 0.5 - fy), 1);
                }
                const float* L = sample_L + 3ull * ((uint64_t)k * R.npix_work + pix_i);
                L0 = L[0], L1 = L[1], L2 = L[2];
            }
            s_L[q][0] = L0, s_L[q][1] = L1, s_L[q][2] = L2;
#pragma unroll
            for (int o = 0; o < NW; o++) s_wx[q][o] = wx[o], s_wy[q][o] = wy[o];
        }
        __syncthreads();
        if (inside) {
            for (int oy = -ry; oy <= ry; oy++) {
                for (int ox = -rx; ox <= rx; ox++) {
                    const int q = (ly - oy + RAD) * SW + (lx - ox + RAD);  // source (x - ox, y - oy)
                    const double w = (s_wx[q][ox + RAD] * s_wy[q][oy + RAD]) * R.inv_integral;
                    if (w <= 0) continue;
                    acc[0] += (double)s_L[q][0] * w;
                    acc[1] += (double)s_L[q][1] * w;
                    acc[2] += (double)s_L[q][2] * w;
                    acc[3] += w;
                }
            }
        }
        __syncthreads();
    }
    if (!inside) return;
    double* o = film + 4ull * ((uint64_t)y * W + x);
    o[0] += acc[0];
    o[1] += acc[1];
    o[2] += acc[2];
    o[3] += acc[3];
}

// ------------------------------------------------------------------ film resolve
// Film::WritePNG's per-pixel body (Film.hpp:183-196) with reinhard_jodie /
// ACESFilm (Film.hpp:34-47) and linear_to_sRGB (Texture.hpp:13-17).  The
// writers take the tone mapper as std::function<glm::vec3(glm::vec3)>, so the
// color is rounded to float on the way in and on the way out.
__device__ __forceinline__ double dmin_(double a, double b) { return b < a ? b : a; }  // std::min
__device__ __forceinline__ double dmax_(double a, double b) { return a < b ? b : a; }  // std::max
__device__ __forceinline__ double glm_clamp01(double x) {  // glm::clamp = min(max(x, 0), 1), NaN-propagating
    const double m = x < 0.0 ? 0.0 : x;                     // glm::max(x, 0): (x < 0) ? 0 : x
    return 1.0 < m ? 1.0 : m;                               // glm::min(m, 1): (1 < m) ? 1 : m
}
__device__ __forceinline__ double linear_to_srgb(double v) {
    v = glm_clamp01(v);
    return v < 0.0031308 ? 12.92 * v : 1.055 * pow(v, 1.0 / 2.4) - 0.055;
}
// Per-triangle shading records (DevTriShade) from the indexed mesh arrays,
// once per scene upload.
// one shading record per primitive SLOT (triangle slots; the others zero), so
// the shading reads it beside the slot's geometry and info, not after them
__global__ __launch_bounds__(256) void k_tri_shade(const DevGeom* __restrict__ geom,
                                                   const DevPrimInfo* __restrict__ info,
                                                   const uint4* __restrict__ tri, const float* __restrict__ normals,
                                                   const float* __restrict__ uvs,
                                                   const float* __restrict__ tangents, uint32_t n,
                                                   DevTriShade* __restrict__ out) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    if ((__float_as_uint(geom[s].a.w) & GF_KIND) != PT_PRIM_TRIANGLE) {
        const float4 z = make_float4(0, 0, 0, 0);
        out[s] = DevTriShade{z, z, z, z, z, z, z, z};
        return;
    }
    const uint4 T = tri[info[s].index];
    const float* n0 = normals + 3 * (size_t)T.x;
    const float* n1 = normals + 3 * (size_t)T.y;
    const float* n2 = normals + 3 * (size_t)T.z;
    const float* u0 = uvs + 2 * (size_t)T.x;
    const float* u1 = uvs + 2 * (size_t)T.y;
    const float* u2 = uvs + 2 * (size_t)T.z;
    DevTriShade r;
    r.a = make_float4(n0[0], n0[1], n0[2], n1[0]);
    r.b = make_float4(n1[1], n1[2], n2[0], n2[1]);
    r.c = make_float4(n2[2], u0[0], u0[1], u1[0]);
    r.d = make_float4(u1[1], u2[0], u2[1], __uint_as_float(T.w));
    r.e = r.f = r.g = r.pad = make_float4(0, 0, 0, 0);
    if ((T.w & 1u) && tangents) {
        const float* t0 = tangents + 3 * (size_t)T.x;
        const float* t1 = tangents + 3 * (size_t)T.y;
        const float* t2 = tangents + 3 * (size_t)T.z;
        r.e = make_float4(t0[0], t0[1], t0[2], t1[0]);
        r.f = make_float4(t1[1], t1[2], t2[0], t2[1]);
        r.g = make_float4(t2[2], 0, 0, 0);
    }
    out[s] = r;
}

// pt_frame_samples: per-sample radiance of the last fixed-SPP frame at the
// given sample-buffer indices (a check of the frame bench.py timed)
__global__ __launch_bounds__(256) void k_frame_gather(const float* __restrict__ sample_L,
                                                     const unsigned long long* __restrict__ idx, uint32_t n,
                                                     float* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float* L = sample_L + 3ull * idx[i];
    out[3 * i] = L[0];
    out[3 * i + 1] = L[1];
    out[3 * i + 2] = L[2];
}

__global__ __launch_bounds__(256) void k_resolve(const double* __restrict__ film, uint32_t npx, uint32_t tonemap,
                                                uint8_t* __restrict__ rgb) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= npx) return;
    const double4 a = reinterpret_cast<const double4*>(film)[i];
    // dvec3 / weight, then the std::function<vec3(vec3)> boundary
    double c[3] = {(double)(float)(a.x / a.w), (double)(float)(a.y / a.w), (double)(float)(a.z / a.w)};
    double m[3];
    if (tonemap == PT_TONEMAP_ACES) {
        const double A = 2.51f, B = 0.03f, C = 2.43f, D = 0.59f, E = 0.14f;
        for (int k = 0; k < 3; k++) m[k] = glm_clamp01((c[k] * (A * c[k] + B)) / (c[k] * (C * c[k] + D) + E));
    } else {
        const double l = c[0] * 0.2126 + c[1] * 0.7152 + c[2] * 0.0722;  // luminance (Util.hpp:4-6)
        for (int k = 0; k < 3; k++) {
            const double t = c[k] / (1.0 + c[k]);
            m[k] = (c[k] / (1.0 + l)) * (1.0 - t) + t * t;  // glm::mix(color/(1+l), t, t)
        }
    }
    for (int k = 0; k < 3; k++) {
        const double s = linear_to_srgb((double)(float)m[k]);
        rgb[3ull * i + k] = (uint8_t)(255.999 * dmax_(0.0, dmin_(1.0, s)));
    }
}

// ------------------------------------------------------------------ hit sort
// north_star "sort of active rays by material and hit state": the paths of a
// bounce are binned by what they hit and k_shade walks them bin by bin.
// KEY = PT_SORT_MATERIAL: miss / the hit primitive's material (one branch of
// the material code, one texture per wave); KEY = PT_SORT_SPATIAL: miss /
// the hit point's cell in a 16x16x16 Morton grid over the scene box (the
// shading gathers of nearby triangles, and the next bounce's and the shadow
// rays' origins -- appended in shading order -- stay together).  A counting
// sort: per-block LDS histograms folded into global counters, one scan, then
// a scatter that reserves each block's range of every bin with one atomic.
// Per-path results do not depend on the order, only the schedule does.
template <int KEY>
__device__ __forceinline__ uint32_t sort_bin(const PathSoA& cur, uint32_t front, const float4* __restrict__ hit,
                                             uint32_t i) {
    if (KEY == PT_SORT_RAYS) {  // the ray's origin cell (8^3 Morton) and direction octant
        const uint32_t e = path_slot(i, front, cur.cap);
        const f3 o = xyz(cur.o[e]), d = xyz(cur.d[e]);
        const float p[3] = {o.x, o.y, o.z};
        uint32_t code = ((d.z < 0) << 2) | ((d.y < 0) << 1) | (d.x < 0);
#pragma unroll
        for (int a = 0; a < 3; a++) {
            const float q = (p[a] - S.bb_lo[a]) * S.bb_scale[a] * 0.5f;  // [0, 2^(bits-1))
            const uint32_t c = (uint32_t)fminf(fmaxf(q, 0.0f), (float)((1 << (PT_SORT_CELL_BITS - 1)) - 1));
#pragma unroll
            for (int b = 0; b < PT_SORT_CELL_BITS - 1; b++) code |= ((c >> b) & 1u) << (3 + 3 * b + a);
        }
        return code;
    }
    const float4 h = hit[i];
    const int prim = __float_as_int(h.w);
    if (prim < 0) return 0u;
    if (KEY == PT_SORT_SPATIAL && S.prim_cell) {
        if ((uint32_t)prim >= S.n_prims) return PT_SORT_BINS_SPATIAL - 1u;  // a virtual slot inside an instance
        return S.prim_cell[prim];
    }
    if (KEY == PT_SORT_MATERIAL) {
        if ((uint32_t)prim >= S.n_prims) return PT_SORT_BINS_MATERIAL - 1u;  // a virtual slot inside an instance
        const int mat = S.info[prim].material;
        return mat < 0 ? 0u : 1u + (uint32_t)mat % (PT_SORT_BINS_MATERIAL - 2u);
    }
    const uint32_t e = path_slot(i, front, cur.cap);
    return hit_cell(xyz(cur.o[e]), xyz(cur.d[e]), h.x);
}
// Each block bins PT_SORT_PER paths per thread (PT_SORT_PER x 256
// consecutive paths), so clearing and folding the block's 4096-bin LDS
// histogram is paid once per 4096 paths rather than once per 256.
// bins (or null): each path's bin, for k_sort_scatter to read (2 B) instead
// of recomputing it from the path and hit records (48 B)
template <int KEY, int NB>
__global__ __launch_bounds__(256) void k_sort_count(PathSoA cur, const uint32_t* __restrict__ nptr,
                                                   const float4* __restrict__ hit, uint32_t* __restrict__ counts,
                                                   uint16_t* __restrict__ bins) {
    __shared__ uint32_t h[NB];
    const uint32_t n = path_count(nptr), front = nptr[Q_NEXT];
    const uint32_t t0 = blockIdx.x * (256u * PT_SORT_PER);
    if (t0 >= n) return;
    for (int b = threadIdx.x; b < NB; b += 256) h[b] = 0;
    __syncthreads();
#pragma unroll 4
    for (uint32_t k = 0; k < PT_SORT_PER; k++) {
        const uint32_t t = t0 + k * 256u + threadIdx.x;
        if (t < n) {
            const uint32_t b = sort_bin<KEY>(cur, front, hit, t);
            if (bins) bins[t] = (uint16_t)b;
            atomicAdd(&h[b], 1u);
        }
    }
    __syncthreads();
    for (int b = threadIdx.x; b < NB; b += 256)
        if (h[b]) atomicAdd(&counts[b], h[b]);
}
template <int NB>
__global__ __launch_bounds__(256) void k_sort_scan(uint32_t* __restrict__ counts) {  // one block
    constexpr int PER = NB / 256;
    __shared__ uint32_t part[256];
    uint32_t v[PER], acc = 0;
#pragma unroll
    for (int k = 0; k < PER; k++) {
        v[k] = counts[threadIdx.x * PER + k];
        acc += v[k];
    }
    part[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (int b = 0; b < 256; b++) {
            const uint32_t c = part[b];
            part[b] = run;
            run += c;
        }
    }
    __syncthreads();
    uint32_t run = part[threadIdx.x];
#pragma unroll
    for (int k = 0; k < PER; k++) {
        counts[threadIdx.x * PER + k] = run;
        run += v[k];
    }
}
// The block's paths keep their bins in registers between the two passes; a
// path's position inside its bin's block range comes from an LDS atomic, so
// the order within a bin is arbitrary (results do not depend on it).
template <int KEY, int NB>
__global__ __launch_bounds__(256) void k_sort_scatter(PathSoA cur, const uint32_t* __restrict__ nptr,
                                                     const float4* __restrict__ hit, uint32_t* __restrict__ offsets,
                                                     uint32_t* __restrict__ order, const uint16_t* __restrict__ bins) {
    __shared__ uint32_t h[NB];
    const uint32_t n = path_count(nptr), front = nptr[Q_NEXT];
    const uint32_t t0 = blockIdx.x * (256u * PT_SORT_PER);
    if (t0 >= n) return;
    for (int b = threadIdx.x; b < NB; b += 256) h[b] = 0;
    __syncthreads();
    uint32_t bin[PT_SORT_PER];
#pragma unroll
    for (uint32_t k = 0; k < PT_SORT_PER; k++) {
        const uint32_t t = t0 + k * 256u + threadIdx.x;
        bin[k] = t < n ? (bins ? (uint32_t)bins[t] : sort_bin<KEY>(cur, front, hit, t)) : 0u;
        if (t < n) atomicAdd(&h[bin[k]], 1u);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < NB; b += 256)
        if (h[b]) h[b] = atomicAdd(&offsets[b], h[b]);  // the block's range of bin b
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < PT_SORT_PER; k++) {
        const uint32_t t = t0 + k * 256u + threadIdx.x;
        if (t < n) order[atomicAdd(&h[bin[k]], 1u)] = t;
    }
}
template __global__ void k_sort_count<PT_SORT_MATERIAL, PT_SORT_BINS_MATERIAL>(PathSoA, const uint32_t*, const float4*,
                                                                             uint32_t*, uint16_t*);
template __global__ void k_sort_count<PT_SORT_SPATIAL, PT_SORT_BINS_SPATIAL>(PathSoA, const uint32_t*, const float4*,
                                                                           uint32_t*, uint16_t*);
template __global__ void k_sort_count<PT_SORT_RAYS, PT_SORT_BINS_SPATIAL>(PathSoA, const uint32_t*, const float4*,
                                                                        uint32_t*, uint16_t*);
template __global__ void k_sort_scatter<PT_SORT_RAYS, PT_SORT_BINS_SPATIAL>(PathSoA, const uint32_t*, const float4*,
                                                                          uint32_t*, uint32_t*, const uint16_t*);
template __global__ void k_sort_scan<PT_SORT_BINS_MATERIAL>(uint32_t*);
template __global__ void k_sort_scan<PT_SORT_BINS_SPATIAL>(uint32_t*);
template __global__ void k_sort_scatter<PT_SORT_MATERIAL, PT_SORT_BINS_MATERIAL>(PathSoA, const uint32_t*,
                                                                               const float4*, uint32_t*, uint32_t*,
                                                                               const uint16_t*);
template __global__ void k_sort_scatter<PT_SORT_SPATIAL, PT_SORT_BINS_SPATIAL>(PathSoA, const uint32_t*, const float4*,
                                                                             uint32_t*, uint32_t*, const uint16_t*);

// ------------------------------------------------------------------ adaptive sampling
// TileIntegrator::Render (Integrators.cpp:55-86): each pixel takes rounds of
// samplesPerPixel samples; after a round its three luminance-weighted
// VarianceEstimators (Util.hpp:8-43) stop it when every RelativeVariance is
// <= 1.5, else it goes on while it has fewer than 128 * spp samples.  Round r
// of a pixel draws stream samples r*spp .. r*spp + spp - 1 (the reference's
// samplers restart the sample index each round with fresh random state).
// The device runs one round for all still-active pixels at once: the active
// list is the wavefront's pixel set (RenderParams::pix_list), sample g of a
// round chunk is (pix_list[g % n], s_lo + g / n) as in the fixed-SPP chunks.

// The frame's work pixels (tile-major 8x8 order when the frame tiles, as the
// fixed-SPP path) restricted to this shard's 32x32 tiles (Integrators.cpp:33):
// a pixel's rounds stay on one rank.  Zeroes their estimators and counts.
__global__ __launch_bounds__(256) void k_adapt_init(RenderParams R, uint32_t shard_index, uint32_t shard_count,
                                                   uint32_t* __restrict__ list, uint32_t* __restrict__ cnt,
                                                   AdaptEst* __restrict__ est, uint32_t* __restrict__ counts) {
    if (blockIdx.x * 256 >= R.npix_work) return;
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    bool take = false;
    uint32_t p = 0;
    if (i < R.npix_work) {
        uint32_t x, y;
        work_pixel(R, i, x, y);
        p = y * (uint32_t)R.cam.width + x;
        const uint32_t tiles_x32 = ((uint32_t)R.cam.width + 31u) / 32u;
        take = ((y >> 5) * tiles_x32 + (x >> 5)) % shard_count == shard_index;
        if (take) {
            est[p] = AdaptEst{{0, 0, 0}, {0, 0, 0}};
            counts[p] = 0;
        }
    }
    const int qoff[1] = {0};
    const bool pred[1] = {take};
    uint32_t at[1];
    block_append<1, 256>(cnt, qoff, pred, at);
    if (take) list[at[0]] = p;
}

// pixel -> its entry in this round's active list (-1 elsewhere)
__global__ __launch_bounds__(256) void k_adapt_map(const uint32_t* __restrict__ list, const uint32_t* __restrict__ n,
                                                  int32_t* __restrict__ map) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < *n) map[list[i]] = (int32_t)i;
}

// VarianceEstimator::Add of the chunk's samples, per pixel in sample order, on
// color * dvec3(0.2126f, 0.7152f, 0.0722f).  GCC's contraction of the
// reference build (TileIntegrator::Render disassembly): the luminance product
// is fused into both differences and S's update,
//   delta = fma(c, w, -mean); mean = delta / n + mean;
//   delta2 = fma(c, w, -mean); S = fma(delta, delta2, S).
__global__ __launch_bounds__(256) void k_adapt_accum(RenderParams R, const float* __restrict__ sample_L,
                                                    AdaptEst* __restrict__ est, uint32_t* __restrict__ counts) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= R.npix_work) return;
    const uint32_t p = R.pix_list[i];
    const double wl[3] = {(double)0.2126f, (double)0.7152f, (double)0.0722f};
    AdaptEst e = est[p];
    uint32_t n = counts[p];
    const uint32_t ns = R.s_hi - R.s_lo;
    for (uint32_t k = 0; k < ns; k++) {
        const float* L = sample_L + 3ull * ((uint64_t)k * R.npix_work + i);
        const double dn = (double)(++n);
#pragma unroll
        for (int c = 0; c < 3; c++) {
            const double v = (double)L[c];
            const double delta = fma(v, wl[c], -e.mean[c]);
            e.mean[c] = delta / dn + e.mean[c];
            const double delta2 = fma(v, wl[c], -e.mean[c]);
            e.S[c] = fma(delta, delta2, e.S[c]);
        }
    }
    est[p] = e;
    counts[p] = n;
}

// FilmTile::Add of a round chunk's samples: every pixel of the frame gathers
// the samples of its active neighbours (k_gather with the source pixel's
// entry looked up in `map`), in a fixed order -- deterministic, no atomics.
__global__ __launch_bounds__(256) void k_adapt_gather(RenderParams R, const int32_t* __restrict__ map,
                                                     const float* __restrict__ sample_L, double* __restrict__ film) {
    const uint32_t tid = blockIdx.x * 256 + threadIdx.x;
    const uint32_t W = (uint32_t)R.cam.width, H = (uint32_t)R.cam.height;
    if (tid >= W * H) return;
    const int x = (int)(tid % W), y = (int)(tid / W);
    double acc[4] = {0, 0, 0, 0};
    bool any = false;
    const uint32_t ns = R.s_hi - R.s_lo;
    for (int oy = -R.rad_y; oy <= R.rad_y; oy++) {
        for (int ox = -R.rad_x; ox <= R.rad_x; ox++) {
            const int sx = x - ox, sy = y - oy;
            if (sx < 0 || sy < 0 || sx >= (int)W || sy >= (int)H) continue;
            const uint32_t spix = (uint32_t)sy * W + (uint32_t)sx;
            const int32_t j = map[spix];
            if (j < 0) continue;
            any = true;
            for (uint32_t k = 0; k < ns; k++) {
                const uint32_t key = stream_key(R.seed, spix, R.s_lo + k);
                double fx, fy;
                sample_fract(R, key, (uint32_t)sx, (uint32_t)sy, R.s_lo + k, fx, fy);
                const double spx = (double)ox + 0.5 - fx, spy = (double)oy + 0.5 - fy;
                const double w = filter_eval(R, (float)spx, (float)spy) * R.inv_integral;
                if (w <= 0) continue;
                const float* L = sample_L + 3ull * ((uint64_t)k * R.npix_work + (uint32_t)j);
                acc[0] += (double)L[0] * w;
                acc[1] += (double)L[1] * w;
                acc[2] += (double)L[2] * w;
                acc[3] += w;
            }
        }
    }
    if (!any) return;
    double* o = film + 4ull * tid;
    o[0] += acc[0];
    o[1] += acc[1];
    o[2] += acc[2];
    o[3] += acc[3];
}

// VarianceEstimator::RelativeVariance (Util.hpp:36-38)
__device__ __forceinline__ double rel_variance(double mean, double S, uint32_t n) {
    if (mean == 0) return 0;
    const double var = n > 1 ? S / (double)(n - 1) : 0.0;
    return 1.96 * sqrt(var / (double)n) / mean;
}

// End of a round: a pixel goes on unless all three relative variances are
// <= 1.5, and only while it has fewer than 128 * spp samples (the loop test).
// Clears its map entry; survivors are appended to the next round's list.
__global__ __launch_bounds__(256) void k_adapt_decide(const uint32_t* __restrict__ list, const uint32_t* __restrict__ n,
                                                     const AdaptEst* __restrict__ est,
                                                     const uint32_t* __restrict__ counts, uint32_t max_samples,
                                                     int32_t* __restrict__ map, uint32_t* __restrict__ out_list,
                                                     uint32_t* __restrict__ out_cnt) {
    const uint32_t nn = *n;
    if (blockIdx.x * 256 >= nn) return;
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    bool go = false;
    uint32_t p = 0;
    if (i < nn) {
        p = list[i];
        map[p] = -1;
        const AdaptEst e = est[p];
        const uint32_t c = counts[p];
        bool done = true;
#pragma unroll
        for (int k = 0; k < 3; k++) done = done && rel_variance(e.mean[k], e.S[k], c) <= PT_ADAPT_REL_VAR;
        go = !done && c < max_samples;
    }
    const int qoff[1] = {0};
    const bool pred[1] = {go};
    uint32_t at[1];
    block_append<1, 256>(out_cnt, qoff, pred, at);
    if (go) out_list[at[0]] = p;
}

// explicit instantiations used by the runtime
// INST: the instance enter/exit step is compiled in only for scenes that have
// instances (it costs the pool kernels registers: see DESIGN.md).
#define PT_INST_TRACE(B, I)                                                                                         \
    template __global__ void k_closest<B, I>(PathSoA, const uint32_t*, float4*, uint32_t*, uint32_t*, uint32_t*,     \
                                             uint32_t*, unsigned long long*, uint32_t*);                             \
    template __global__ void k_shadow<B, I>(PathSoA, float*, ShadowRec*, const uint32_t*, uint32_t*,           \
                                            uint32_t*, unsigned long long*);
#define PT_INST_POOL(B, I, Q)                                                                                       \
    template __global__ void k_closest_pool<B, I, Q>(PathSoA, const uint32_t*, float4*, uint32_t*, uint32_t*,        \
                                                     uint32_t*, uint32_t*, unsigned long long*, uint32_t*);          \
    template __global__ void k_shadow_pool<B, I, Q>(PathSoA, float*, ShadowRec*, const uint32_t*, uint32_t*,   \
                                                    uint32_t*, unsigned long long*);
#define PT_INST_TAIL(G, I, C)                                                                              \
    template __global__ void k_tail<G, I, C>(RenderParams, PathSoA, const uint32_t*, float*, unsigned long long*);
PT_INST_TAIL(PT_INTEGRATOR_PATH, false, false)
PT_INST_TAIL(PT_INTEGRATOR_PATH, false, true)
PT_INST_TAIL(PT_INTEGRATOR_SIMPLE, false, false)
PT_INST_TAIL(PT_INTEGRATOR_SIMPLE, false, true)
#undef PT_INST_TAIL
template __global__ void k_closest_ties<false>(PathSoA, const uint32_t*, float4*, const uint32_t*, const uint32_t*);
template __global__ void k_closest_ties<true>(PathSoA, const uint32_t*, float4*, const uint32_t*, const uint32_t*);
PT_INST_TRACE(false, false)
PT_INST_TRACE(true, false)
PT_INST_TRACE(false, true)
PT_INST_TRACE(true, true)
PT_INST_POOL(false, false, false)
PT_INST_POOL(true, false, false)
PT_INST_POOL(false, true, false)
PT_INST_POOL(true, true, false)
PT_INST_POOL(false, false, true)
PT_INST_POOL(true, false, true)
PT_INST_POOL(false, true, true)
PT_INST_POOL(true, true, true)
template __global__ void k_shadow_sl<false>(PathSoA, float*, ShadowRec*, const uint32_t*, uint32_t*, uint32_t*,
                                           unsigned long long*);
template __global__ void k_shadow_sl<true>(PathSoA, float*, ShadowRec*, const uint32_t*, uint32_t*, uint32_t*,
                                          unsigned long long*);
template __global__ void k_shadow_tr<false>(PathSoA, float*, const ShadowRecV*, const uint32_t*, unsigned long long*);
template __global__ void k_shadow_tr<true>(PathSoA, float*, const ShadowRecV*, const uint32_t*, unsigned long long*);
template __global__ void k_shade<PT_INTEGRATOR_PATH>(RenderParams, PathSoA, const uint32_t*, const float4*, PathSoA,
                                                     float*, unsigned long long*, ShadowRec*, uint32_t*);
template __global__ void k_shade<PT_INTEGRATOR_SIMPLE>(RenderParams, PathSoA, const uint32_t*, const float4*,
                                                       PathSoA, float*, unsigned long long*, ShadowRec*, uint32_t*);
