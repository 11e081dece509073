// Persistent BVH4 traversal with per-lane ray refill.
//
// Incoherent secondary rays make per-lane traversal lengths vary by an order
// of magnitude, so a wave that traces exactly its 64 rays runs as long as its
// longest one.  Here a resident wave keeps pulling rays: whenever at least
// PT_REFILL of its lanes are idle, it claims that many rays with one atomic
// on a pool counter and the idle lanes start them, so lanes stay busy until
// the pool drains.  The ray range is split into
// PT_POOL_CHUNKS chunks with one counter each (own 128-byte line); a block starts on chunk
// blockIdx % 8 (its XCD under round-robin dispatch) and moves to the next
// non-empty chunk when its own runs dry, so no single counter line takes every
// claim (MI355X_MICROARCH.md "dequeue": one word saturates near 88 claims/us).
//
// Each step advances a lane by one pop, one interior cluster or one leaf, with
// the exact semantics of trace_closest / trace_any (pt_trace.h): same octant
// child order, same leaf tests, so results are identical to the one-ray-per-
// lane kernels; only the assignment of rays to lanes changes.
#pragma once
#include "pt_trace.h"

#define PT_POOL_CHUNKS 8
#define PT_POOL_STRIDE 32  // uint32 words between chunk counters (128 B)
#define PT_POOL_WORDS (PT_POOL_CHUNKS * PT_POOL_STRIDE)
// Stack entries the pool kernels keep in LDS; entries [PT_POOL_LDS, PT_POOL_STACK)
// live in a global overflow array ([entry][grid lane], written and read back by
// the same lane only).  Deep stacks are rare, and a 20-entry LDS stack (10 KB
// per block) lets 32 waves per CU fit instead of 20 with all 32 in LDS.
// C4 r04: 16 / 20 / 24 (closest-hit kernel) -> 1596 / 1613 / 1577 Mrays/s
// (profiles/r04_ab_traversal.txt)
#ifndef PT_POOL_LDS
#define PT_POOL_LDS 20
#endif
// Idle lanes that trigger a refill: fewer claims (one atomic and one
// divergent ray start per refill) against lanes left idle meanwhile.  C4:
// 4 -> 1081, 8 -> 1198, 16 -> 1235, 24 -> 1224, 32 -> 1188 Mrays/s
// (profiles/r02_ab_shade.txt).
#ifndef PT_REFILL
#define PT_REFILL 16
#endif
// Stack capacity of the pool kernels.  The reference's stack[32] is undefined
// behaviour past 32 entries (BVH.hpp:1128); here the entries past the LDS part
// live in HBM, so a deeper stack costs only that array.  A push past the
// capacity is dropped and counted (DevScene::stack_drops -> pt_stats::
// stack_overflows; the full-size C4 test asserts none).
#ifndef PT_POOL_STACK
#define PT_POOL_STACK 48
#endif
// The record array is read through a buffer resource: a lane without a node
// (primitive) step addresses past the buffer's end, which returns zeros
// without a fetch (the runtime keeps the array below this offset).
#define Q48_OOB_OFFSET 0xFFFFFF00u  // + 32 stays below 2^32: never wraps into range
__device__ __forceinline__ float4 q48_buf_load(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
}

// Measured and removed (the commits and profiles/r0*_ab_*.txt keep them):
// entry distances kept on the stack (r02_ab_c4.txt), two primitives per leaf
// step (r02, r04_ab_traversal.txt), slot-order any hit (r02_ab_shade.txt),
// exec-masked loads, pre-claimed refills, paired pops (r04_ab_traversal.txt),
// the triangle test before the node side, an alpha record read ahead of its
// test, packed-ALU triangle tests, 128-B wide nodes (r05_ab_traversal.txt),
// the BVH top in LDS (r05_ab_treelet.txt).

// ---- Overlapped traversal (trace_spec: quantized records, no instances).
// The pool kernels wait on their loads (C4 k_closest_pool: SQ_WAIT_ANY 64 %
// of wave cycles, VALU issue 42 % busy at 2 cycles per wave64 instruction,
// profiles/r03_valu.txt): a ray costs about one dependent memory round trip
// per iteration, and a lane makes one node step or one primitive step per
// iteration.  Almost every iteration of a wave has both node lanes and
// primitive lanes (C4: 99.9 % / 97 %), so both paths are issued anyway.
// Here a lane keeps two cursors into its own depth-first order: `leaf`, the
// leaf whose primitives it is testing, and `ref`, the next node after that
// leaf, and advances both in one iteration (C4: 15 % fewer iterations).
// Primitives are still tested one at a time in the reference's order
// (BVH4::Intersect, BVH.hpp:1111-1211); what changes is that a node after the
// leaf can be tested before the leaf's primitives are all done, against a max
// not yet shortened by them, so it may visit a node the reference culls (as
// the quantized boxes already may; a hit there is accepted only if it is at
// least as near, so the closest hit is the reference's unless two primitives
// give the very same t).  A leaf holding a BLAS hop (REF_BLOCK) pauses the
// node side until it is done, so the BLAS root it pushes is visited where the
// reference visits it.  Any hit: the answer does not depend on the order.
// In an iteration the node side runs before the primitive side, so no node
// data is live across the primitive side's out-of-line calls (primitive side
// first: 13 % slower, spills); a second queued leaf saved 4 % of the
// iterations and cost 17 % (profiles/r03_ab_spec.txt).
template <bool ANY, bool COUNT, class Src, int LN>
__device__ void trace_spec(uint32_t n, uint32_t* __restrict__ pool, Src& src, uint32_t* s_ref,
                           uint32_t* __restrict__ ovf, TraceWork& wk, const uint8_t* s_lut) {
    const uint32_t lane = threadIdx.x;
    const uint32_t gl = blockIdx.x * PT_TRACE_BLOCK + lane, G = gridDim.x * PT_TRACE_BLOCK;
    const uint32_t wl = __lane_id();
    const uint32_t cs = (n + PT_POOL_CHUNKS - 1) / PT_POOL_CHUNKS;
    const uint32_t home = blockIdx.x % PT_POOL_CHUNKS;
    uint32_t dead = 0;  // wave-uniform: chunks found empty
    const uint32_t all_dead = (1u << PT_POOL_CHUNKS) - 1u;

    int ri = -1;
    f3 o = F3(0, 0, 0), d = F3(0, 0, 0), inv = F3(0, 0, 0);
    uint32_t oct = 0, ref = REF_EMPTY, leaf = REF_EMPTY;
    const __amdgpu_buffer_rsrc_t qrs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<DevGeom*>(S.qrec), (short)0, (int)S.qrec_bytes, 0x00020000);
    // closest hit: an accepted hit is stored at once (Src::closest), so the
    // barycentrics and slot need no registers; OCT_FOUND marks that one was
    float tmax = 0;
    int sp = 0;
    // the overflow entries through a buffer resource and the LDS ones through
    // ds ops, in separate branches: a pointer select of the two becomes a flat
    // access, and a flat pop waits for every outstanding vector memory op of
    // the wave (the previous iteration's hit stores, a fresh ray's loads)
    const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(ovf, (short)0, 0x7FFFFFFF, 0x00020000);
    auto push = [&](uint32_t v) {
        if (sp < PT_POOL_STACK) {
            if (LN >= PT_POOL_STACK || sp < LN) {
                s_ref[sp * PT_TRACE_BLOCK + lane] = v;
            } else {
                __builtin_amdgcn_raw_buffer_store_b32(v, ors, (uint32_t)((sp - LN) * G + gl) * 4u, 0, 0);
            }
            ++sp;
        } else {
            atomicAdd(S.stack_drops, 1u);
        }
    };
    auto pop = [&]() -> uint32_t {
        --sp;
        uint32_t v;
        if (LN >= PT_POOL_STACK || sp < LN) {
            v = s_ref[sp * PT_TRACE_BLOCK + lane];
        } else {
            v = __builtin_amdgcn_raw_buffer_load_b32(ors, (uint32_t)((sp - LN) * G + gl) * 4u, 0, 0);
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) here, on the rare overflow path only
        }
        return v;
    };
    auto is_leaf = [](uint32_t r) { return r != REF_EMPTY && (r & REF_LEAF); };
    for (;;) {
        const uint64_t idle = __ballot(ri < 0);
        const uint32_t nidle = (uint32_t)__popcll(idle);
        if (nidle >= PT_REFILL || idle == __ballot(true)) {
            // claim exactly as many rays as lanes are idle (one atomic) from the
            // home chunk or the next non-empty one; no reserve is held, so no
            // wave sits on unstarted rays while others run dry
            uint32_t base = 0, got = 0;
            if (dead != all_dead) {
                if (wl == 0) {
                    #pragma unroll 1
                    for (uint32_t k = 0; k < PT_POOL_CHUNKS; k++) {
                        const uint32_t c = (home + k) % PT_POOL_CHUNKS;
                        if ((dead >> c) & 1u) continue;
                        const uint32_t lo = c * cs, hi = min(n, lo + cs);
                        const uint32_t old = lo < hi ? atomicAdd(&pool[c * PT_POOL_STRIDE], nidle) : hi;
                        if (lo + old < hi) {
                            base = lo + old;
                            got = min(nidle, hi - base);
                            break;
                        }
                        dead |= 1u << c;
                    }
                }
                base = __builtin_amdgcn_readfirstlane(base);
                got = __builtin_amdgcn_readfirstlane(got);
                dead = __builtin_amdgcn_readfirstlane(dead);
            }
            if (ri < 0) {
                const uint32_t k = (uint32_t)__popcll(idle & ((1ull << wl) - 1ull));
                if (k < got) {
                    ri = (int)(base + k);
                    // only the loads here: the ray is set up (1/d, octant) once
                    // this iteration's node loads are in flight too, so the two
                    // round trips overlap (C4 1636.7 -> 1641.9 Mrays/s,
                    // profiles/r04_ab_traversal.txt; trace_spec's sources never
                    // skip a ray)
                    src.load((uint32_t)ri, o, d, tmax);
                    oct = OCT_FRESH;
                    ref = S.qroot;
                    leaf = REF_EMPTY;
                    sp = 0;
                }
            }
            if (got == 0 && dead == all_dead && __ballot(ri >= 0) == 0) break;
        }
        if (ri < 0) continue;

        // ---- feed the two cursors from the lane's depth-first order: the
        // leaf cursor takes the next leaf once free, the node side pops unless
        // a BLAS-hop leaf is pending (at most two pops: a leaf popped into the
        // free leaf cursor lets the node side pop once more)
        if (leaf == REF_EMPTY && is_leaf(ref)) {
            leaf = ref;
            ref = REF_EMPTY;
        }
        #pragma unroll
        for (int k = 0; k < 2; k++) {
            if (ref == REF_EMPTY && sp > 0 && !(leaf != REF_EMPTY && (leaf & REF_BLOCK))) {
                const uint32_t r = pop();
                if (leaf == REF_EMPTY && is_leaf(r)) leaf = r;
                else ref = r;
            }
        }
        if (ref == REF_EMPTY && leaf == REF_EMPTY) {  // sp == 0: no hit (any) / closest result
            if (ANY) {
                src.any((uint32_t)ri, false);
            } else {
                if (!(oct & OCT_FOUND)) src.closest((uint32_t)ri, tmax, 0.0f, 0.0f, -1);
            }
            ri = -1;
            continue;
        }
        const bool node_step = ref != REF_EMPTY && !(ref & REF_LEAF);
        const bool prim_step = leaf != REF_EMPTY;
        // both cursors' loads issue before either is used: the node record and
        // the primitive slot (48 B each), three 16-B buffer loads each; a lane
        // without the step reads past the buffer's end (zeros, no fetch)
        const uint32_t slot = prim_step ? (leaf & ~(REF_LEAF | REF_BLOCK)) : 0u;
        const uint32_t noff = node_step ? ref * 48u : Q48_OOB_OFFSET;
        const uint32_t poff = prim_step ? slot * 48u : Q48_OOB_OFFSET;
        const float4 q0 = q48_buf_load(qrs, noff), q1 = q48_buf_load(qrs, noff + 16u), q2 = q48_buf_load(qrs, noff + 32u);
        const float4 g0 = q48_buf_load(qrs, poff), g1 = q48_buf_load(qrs, poff + 16u), g2 = q48_buf_load(qrs, poff + 32u);
        __builtin_amdgcn_sched_barrier(0);  // (the scheduler would sink the slot loads past the node side)
        if (oct & OCT_FRESH) {  // a ray claimed this iteration: its origin and direction are in
            inv = inv_dir(d);
            oct = ((d.z < 0) << 2) | ((d.y < 0) << 1) | (d.x < 0);
        }

        // ---- node side
        {
            uint32_t mask;
            float te[4];
            qslab4pe(q0, q1, q2, o, inv, tmax, mask, te);
            if (!node_step) mask = 0;
            // octant order for any hit too: the occlusion answer does not
            // depend on the order, and near-first finds an occluder sooner (C4
            // k_shadow_pool 10.72 -> 9.44 ms per launch, profiles/r02_ab_shade.txt)
            const uint32_t perm = q48_perm(s_lut, oct, q0.w);
            // a lane with room for three more LDS entries pushes without the
            // capacity / overflow branches of push(): one masked LDS store per
            // pushed child (the other lanes take the general path)
            uint32_t cand;
            if ((LN >= PT_POOL_STACK ? PT_POOL_STACK : LN) - sp >= 3) {
                const uint32_t base = __float_as_uint(q2.z), desc = __float_as_uint(q2.w);
                uint32_t vm = mask;
#pragma unroll
                for (int k = 0; k < 4; k++)
                    if (((desc >> (8 * k)) & 0xFFu) == Q48_EMPTY) vm &= ~(1u << k);
                cand = REF_EMPTY;
                int np = 0;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint32_t ci = (perm >> (2 * k)) & 3u;
                    const uint32_t dd = (desc >> (8 * ci)) & 0xFFu;
                    const uint32_t c = (base + (dd & 63u)) | ((dd & Q48_LEAF) << 25) | ((dd & Q48_HOP) << 22);
                    const bool v = (vm >> ci) & 1u;
                    if (v && cand != REF_EMPTY) s_ref[(sp + np++) * PT_TRACE_BLOCK + lane] = cand;
                    cand = v ? c : cand;
                }
                sp += np;
            } else {
                cand = order_children_q48(mask, q2.z, q2.w, perm, [&](uint32_t v) { push(v); });
            }
            if (node_step) {
                if (COUNT) wk.nodes++;
                ref = cand;
            }
        }
        // ---- primitive side.  The triangle test runs on every lane (its
        // result kept only on primitive lanes), so the slot loads are used
        // outside the branches.
        {
            const uint32_t w0 = __float_as_uint(g0.w);
            const bool pred = ANY && !(w0 & GF_PRED_GLM);
            float bx = 0, by = 0, t = 0;
            bool tri_hit;
            if (pred) tri_hit = tri_pred(o, d, xyz(g0), xyz(g1), xyz(g2), tmax);
            else tri_hit = tri_glm(o, d, xyz(g0), xyz(g1), xyz(g2), bx, by, t) && !(t > tmax || t < PT_EPS);
            // BLAS hop: its root ref (b.x); triangle: its alpha record (b.w)
            const uint32_t g1v = (w0 & GF_KIND) == PT_PRIM_BLAS ? __float_as_uint(g1.x) : __float_as_uint(g1.w);
            const uint32_t g2w = __float_as_uint(g2.w);
            const uint32_t kind = w0 & GF_KIND;
            if (prim_step) {
                bool anyhit = false;
                uint32_t next = (w0 & GF_LAST) ? REF_EMPTY : (REF_LEAF | (leaf & REF_BLOCK) | (slot + 1));
                // the primitive's slot (the record keeps it in c.w)
                const uint32_t ps = g2w;
                if (kind == PT_PRIM_TRIANGLE) {
                    if (COUNT) wk.tris++;
                    if (tri_hit && (pred || !(w0 & GF_ALPHA) || tri_alpha_cov(w0, g1v, ps, bx, by, o, d))) {
                        if (ANY) {
                            anyhit = true;
                        } else {
                            if ((oct & (OCT_FOUND | OCT_TIE)) == OCT_FOUND && t == tmax) {
                                oct |= OCT_TIE;  // an exact tie: the reference's culling decides (below)
                                src.tie((uint32_t)ri);
                            }
                            tmax = t;
                            oct |= OCT_FOUND;
                            src.closest((uint32_t)ri, t, bx, by, (int)ps);
                        }
                    }
                } else if (kind == PT_PRIM_BLAS) {
                    // the reference recurses into the BLAS inside the leaf loop
                    // (Model::Intersect, BVH.hpp:1206): the rest of the leaf
                    // waits on the stack under the BLAS root, which the
                    // (paused) node side visits next
                    if (next != REF_EMPTY) push(next);
                    push(g1v);  // the BLAS root
                    next = REF_EMPTY;
                } else {
                    if (COUNT) wk.tris++;
                    // a sphere without an alpha test inline: its slot holds the
                    // center (a.xyz) and radius (b.x), so no record read and no
                    // call (other_closest / other_pred: the same root, uv 0)
                    const bool sph = kind == PT_PRIM_SPHERE && !(w0 & GF_ALPHA);
                    float t2, a2 = 0.0f, b2 = 0.0f;
                    bool oh;
                    if (sph) {
                        const pt_sphere sp{{g0.x, g0.y, g0.z}, g1.x};
                        oh = sphere_root(sp, o, d, tmax, t2);
                    } else if (ANY) {
                        oh = other_pred(ps, w0, o, d, tmax);
                    } else {
                        oh = other_closest(ps, w0, o, d, tmax, t2, a2, b2);
                    }
                    if (ANY) {
                        if (oh) anyhit = true;
                    } else {
                        if (oh) {
                            if ((oct & (OCT_FOUND | OCT_TIE)) == OCT_FOUND && t2 == tmax) {
                                oct |= OCT_TIE;
                                src.tie((uint32_t)ri);
                            }
                            tmax = t2;
                            oct |= OCT_FOUND;
                            src.closest((uint32_t)ri, t2, a2, b2, (int)ps);
                        }
                    }
                }
                leaf = next;
                if (ANY && anyhit) {  // early exit (BVH.hpp:1104-1105)
                    src.any((uint32_t)ri, true);
                    ri = -1;
                }
            }
        }
    }
}

// Src interface:
//   bool load(uint32_t ri, f3& o, f3& d, float& tmax)   (false: skip this ray)
//   float time(uint32_t ri)   the ray's time (instanced scenes with S.motion)
//   void closest(uint32_t ri, float t, float b1, float b2, int prim)
//   void any(uint32_t ri, bool hit)
//   void tie(uint32_t ri)   (closest hit: the ray met an exact-t tie, see below)
//
// Exact-t ties.  A hit at t == max replaces the current one, in the
// reference as here (Shape.cpp:204 rejects only t > max).  The pool
// traversals visit a superset of the reference's nodes (quantized boxes
// enclose the float boxes; the overlapped form tests nodes ahead of the
// pending leaf, against a max that leaf may still shorten), and the only
// primitive such an extra visit can change the result with is one at exactly
// t == max in a node the reference culled (its float box entry == max).  So
// a ray that meets t == max once a hit exists is listed (Src::tie), and
// k_closest_ties re-traces the listed rays with trace_closest over the
// reference's own clusters in the reference's order, which decides ties as
// the reference does (tests/golden tie_models: three coincident Models).
// QN: the 48-B quantized records (S.qrec), else the reference's 128-B clusters
// (S.nodes) and slots (S.geom); LN: stack entries in LDS (s_ref), the rest in
// ovf ([entry][grid lane]).  Quantized records without instances take the
// overlapped form above.
template <bool ANY, bool COUNT, class Src, bool INST = true, int LN = PT_POOL_LDS, bool QN = false>
__device__ void trace_pool(uint32_t n, uint32_t* __restrict__ pool, Src& src, uint32_t* s_ref,
                           uint32_t* __restrict__ ovf, TraceWork& wk, const uint8_t* s_lut = nullptr) {
    if constexpr (QN && !INST) {
        trace_spec<ANY, COUNT, Src, LN>(n, pool, src, s_ref, ovf, wk, s_lut);
        return;
    }
    const uint32_t lane = threadIdx.x;
    const uint32_t gl = blockIdx.x * PT_TRACE_BLOCK + lane, G = gridDim.x * PT_TRACE_BLOCK;
    const uint32_t wl = __lane_id();
    const uint32_t cs = (n + PT_POOL_CHUNKS - 1) / PT_POOL_CHUNKS;
    const uint32_t home = blockIdx.x % PT_POOL_CHUNKS;
    uint32_t dead = 0;  // wave-uniform: chunks found empty

    int ri = -1;
    f3 o = F3(0, 0, 0), d = F3(0, 0, 0), inv = F3(0, 0, 0);
    uint32_t oct = 0, ref = REF_EMPTY;
    float tmax = 0, bb1 = 0, bb2 = 0;
    int sp = 0, best = -1;

    const uint32_t all_dead = (1u << PT_POOL_CHUNKS) - 1u;
    // pushes beyond PT_POOL_STACK are dropped and counted
    auto push = [&](uint32_t v) {
        if (sp < PT_POOL_STACK) {
            if (LN >= PT_POOL_STACK || sp < LN) s_ref[sp * PT_TRACE_BLOCK + lane] = v;
            else ovf[(size_t)(sp - LN) * G + gl] = v;
            ++sp;
        } else {
            atomicAdd(S.stack_drops, 1u);
        }
    };
    auto start = [&]() {
        inv = inv_dir(d);
        oct = ((d.z < 0) << 2) | ((d.y < 0) << 1) | (d.x < 0);
        ref = QN ? S.qroot : S.root;
        sp = 0;
        best = -1;
        bb1 = bb2 = 0;
    };
    for (;;) {
        const uint64_t idle = __ballot(ri < 0);
        const uint32_t nidle = (uint32_t)__popcll(idle);
        if (nidle >= PT_REFILL || idle == __ballot(true)) {
            // claims as in trace_spec
            uint32_t base = 0, got = 0;
            if (dead != all_dead) {
                if (wl == 0) {
                    #pragma unroll 1
                    for (uint32_t k = 0; k < PT_POOL_CHUNKS; k++) {
                        const uint32_t c = (home + k) % PT_POOL_CHUNKS;
                        if ((dead >> c) & 1u) continue;
                        const uint32_t lo = c * cs, hi = min(n, lo + cs);
                        const uint32_t old = lo < hi ? atomicAdd(&pool[c * PT_POOL_STRIDE], nidle) : hi;
                        if (lo + old < hi) {
                            base = lo + old;
                            got = min(nidle, hi - base);
                            break;
                        }
                        dead |= 1u << c;
                    }
                }
                base = __builtin_amdgcn_readfirstlane(base);
                got = __builtin_amdgcn_readfirstlane(got);
                dead = __builtin_amdgcn_readfirstlane(dead);
                if (ri < 0) {
                    const uint32_t k = (uint32_t)__popcll(idle & ((1ull << wl) - 1ull));
                    if (k < got) {
                        ri = (int)(base + k);
                        if (src.load((uint32_t)ri, o, d, tmax)) start();
                        else ri = -1;
                    }
                }
            }
            if (got == 0 && dead == all_dead && __ballot(ri >= 0) == 0) break;
        }
        if (ri < 0) continue;

        // ---- one step of this lane's traversal: one cluster or one leaf
        // primitive.  Node lanes and primitive lanes issue their loads in the
        // same pass (one memory round trip per step for the whole wave); a leaf
        // continues at ref = REF_LEAF | next slot.
        if (ref == REF_EMPTY) {
            bool finished = false;
            for (;;) {
                if (INST && PT_INSTANCE_DONE()) {  // back at the depth the instance was entered at
                    ref = REF_INST_EXIT;
                    break;
                }
                if (sp == 0) {
                    finished = true;
                    break;
                }
                --sp;
                ref = (LN >= PT_POOL_STACK || sp < LN) ? s_ref[sp * PT_TRACE_BLOCK + lane]
                                                       : ovf[(size_t)(sp - LN) * G + gl];
                break;
            }
            if (finished) {  // no hit (any) / closest result
                if (ANY) src.any((uint32_t)ri, false);
                else src.closest((uint32_t)ri, tmax, bb1, bb2, best);
                ri = -1;
                continue;
            }
        }
        if constexpr (INST) {
            if (ref >= REF_SPECIAL) {  // instance enter / exit (pt_trace.h instance_step)
                PT_INSTANCE_STEP(ANY, S.motion ? src.time((uint32_t)ri) : 0.0f);
                continue;
            }
        }
        const bool node_step = !(ref & REF_LEAF);
        const uint32_t idx = ref & ~(QN ? REF_LEAF | REF_BLOCK : REF_LEAF);
        // all loads issue before any use: a primitive lane reads its 48-byte
        // slot and repeats its first 16 bytes for the node-only words (same
        // line, no extra traffic), and the cluster test below runs
        // unconditionally (its result masked off on primitive lanes) so the
        // compiler cannot sink the node loads behind the primitive branch.
        float4 q0, q1, q2;
        uint32_t mask, perm;
        float te[4];
        uint4 ch;
        if constexpr (QN) {
            // node records and leaf slots share the array: three loads either way
            const float4* __restrict__ q = reinterpret_cast<const float4*>(S.qrec + idx);
            q0 = q[0];
            q1 = q[1];
            q2 = q[2];
            qslab4pe(q0, q1, q2, o, inv, tmax, mask, te);
            ch = q48_children(q2.z, q2.w);
            perm = q48_perm(s_lut, oct, q0.w);
        } else {
            const uint32_t nk = node_step ? 1u : 0u;
            const float4* __restrict__ q = node_step ? reinterpret_cast<const float4*>(S.nodes + idx)
                                                     : reinterpret_cast<const float4*>(S.geom + idx);
            const uint32_t k3 = 3u * nk;
            q0 = q[0];
            q1 = q[1];
            q2 = q[2];
            const float4 q3 = q[k3], q4 = q[k3 ? 4u : 0u], q5 = q[k3 ? 5u : 0u];
            const float4 q6 = q[6 * nk], q7 = q[7 * nk];
            slab4pe(q0, q1, q2, q3, q4, q5, o, inv, tmax, mask, te);
            ch = make_uint4(__float_as_uint(q6.x), __float_as_uint(q6.y), __float_as_uint(q6.z),
                            __float_as_uint(q6.w));
            const uint32_t ow = ((oct >> 2) & 1u) ? __float_as_uint(q7.y) : __float_as_uint(q7.x);
            perm = (ow >> (8 * (oct & 3))) & 0xFFu;
        }
        {
            if (!node_step) mask = 0;  // no children on primitive lanes
            // visit order: octant order far -> near (BVH4::LUT, BVH.hpp:1195-1204),
            // for any hit too (see trace_spec)
            const uint32_t cand = order_children(mask, ch, perm, [&](uint32_t v) { push(v); });
            if (node_step) {
                if (COUNT) wk.nodes++;
                ref = cand;
                continue;
            }
        }
        // leaf primitive at slot idx (QN: record idx, whose c.w is the slot)
        {
            const uint32_t slot = QN ? __float_as_uint(q2.w) : idx;
            const uint32_t w0 = __float_as_uint(q0.w);
            const uint32_t kind = w0 & GF_KIND;
            bool anyhit = false;
            uint32_t next = (w0 & GF_LAST) ? REF_EMPTY : (REF_LEAF | (idx + 1));
            if (kind == PT_PRIM_TRIANGLE) {
                // Intersect (glm) or IntersectPred semantics + the material alpha
                // test (Primitive.cpp:6-26)
                if (COUNT) wk.tris++;
                if (ANY && !(w0 & GF_PRED_GLM)) {
                    if (tri_pred(o, d, xyz(q0), xyz(q1), xyz(q2), tmax)) anyhit = true;
                } else {
                    float bx, by, t;
                    if (tri_glm(o, d, xyz(q0), xyz(q1), xyz(q2), bx, by, t) && !(t > tmax || t < PT_EPS)) {
                        if (!(w0 & GF_ALPHA) || tri_alpha_cov(w0, __float_as_uint(q1.w), slot, bx, by, o, d)) {
                            if (ANY) {
                                anyhit = true;
                            } else {
                                if (best >= 0 && t == tmax && !(oct & OCT_TIE)) {
                                    oct |= OCT_TIE;
                                    src.tie((uint32_t)ri);
                                }
                                tmax = t;
                                best = (int)slot;
                                bb1 = bx;
                                bb2 = by;
                                oct |= (oct & OCT_INST) << 1;  // OCT_HIT inside an instance
                            }
                        }
                    }
                }
            } else if (kind == PT_PRIM_BLAS) {
                // BLAS (or instance) first, the rest of the leaf after it, as
                // the reference's recursion inside the leaf loop (BVH.hpp:1206)
                if (next != REF_EMPTY) push(next);
                push(__float_as_uint(q1.x));
                next = REF_EMPTY;
            } else {
                if (COUNT) wk.tris++;
                if (ANY) {
                    if (other_pred(slot, w0, o, d, tmax)) anyhit = true;
                } else {
                    float t, a, b;
                    if (other_closest(slot, w0, o, d, tmax, t, a, b)) {
                        if (best >= 0 && t == tmax && !(oct & OCT_TIE)) {
                            oct |= OCT_TIE;
                            src.tie((uint32_t)ri);
                        }
                        tmax = t;
                        best = (int)slot;
                        bb1 = a;
                        bb2 = b;
                        oct |= (oct & OCT_INST) << 1;
                    }
                }
            }
            ref = next;
            if (ANY && anyhit) {  // early exit (BVH.hpp:1104-1105)
                src.any((uint32_t)ri, true);
                ri = -1;
            }
        }
    }
}

// ---- Stackless any hit (north_star "stackless BVH4 traversal"; the runtime
// option PT_RENDER_ANY_STACKLESS).  No traversal stack: a lane keeps the node
// it is at in registers -- the record's child block (base, descriptors), the
// octant order and the visit positions still to take among the children its
// slab test hit -- and, when they run out, follows escape links
// (DevScene::qesc, built with the 48-B records) up the tree: the parent
// record is fetched again and its slab test rerun, resuming after the child
// the lane came from.  A descent into a node's last remaining child hands that
// node's own continuation down instead (a tail call), so only nodes with
// hits left are fetched again.  An occlusion answer does not depend on the
// visit order (BVH4::IntersectPred, BVH.hpp:1019-1109), so children go in
// the octant order nearest first, as the stack kernels visit them.  BLAS
// hops and BLAS root copies enter the BLAS with one saved continuation
// (the rest of the TLAS leaf, then the TLAS node), restored at the BLAS
// root's ESC_EXIT.  One node record or one primitive slot per lane per
// iteration; LDS holds only the octant table, so occupancy is set by
// registers alone.
//   continuation words: (record << 2 | k) resume `record` after its child
//   slot k; CONT_FRESH | record << 2: enter `record` (its escape applies);
//   ESC_EXIT: leave the BLAS (or finish, at the TLAS root); SL_DONE: finish
#define CONT_FRESH 0x80000000u
#define SL_DONE 0xFFFFFFFEu
#define SL_NORET 0xFFFFFFFDu  // ret_cont: no BLAS entered (ESC_EXIT is a continuation too)
#ifndef PT_SL_MAX_STEPS
#define PT_SL_MAX_STEPS (1u << 26)  // > 5 x the C4 records: a node is fetched at most once per child, a slot once
#endif
template <bool COUNT, class Src>
__device__ void trace_any_stackless(uint32_t n, uint32_t* __restrict__ pool, Src& src, TraceWork& wk,
                                    const uint8_t* s_lut) {
    const uint32_t wl = __lane_id();
    const uint32_t cs = (n + PT_POOL_CHUNKS - 1) / PT_POOL_CHUNKS;
    const uint32_t home = blockIdx.x % PT_POOL_CHUNKS;
    uint32_t dead = 0;  // wave-uniform: chunks found empty
    const uint32_t all_dead = (1u << PT_POOL_CHUNKS) - 1u;
    const __amdgpu_buffer_rsrc_t qrs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<DevGeom*>(S.qrec), (short)0, (int)S.qrec_bytes, 0x00020000);
    // the escape links through a buffer resource too: a record index out of
    // range reads 0 instead of faulting
    const __amdgpu_buffer_rsrc_t ers = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint32_t*>(S.qesc), (short)0, (int)(S.qrec_bytes / 48u * 4u), 0x00020000);

    int ri = -1;
    f3 o = F3(0, 0, 0), d = F3(0, 0, 0), inv = F3(0, 0, 0);
    uint32_t oct = 0;
    float tmax = 0;
    // steps of the lane's ray: a ray past PT_SL_MAX_STEPS is abandoned and
    // counted with the stack overflows (a traversal must end whatever the links)
    uint32_t steps = 0;
    // the node context: record nrec (REF_EMPTY: none), its child block and
    // descriptors, npk = octant order byte | positions left << 8 (position p
    // = the p-th nearest, perm index 3 - p), nup = its continuation
    uint32_t nrec = REF_EMPTY, nbase = 0, ndesc = 0, npk = 0, nup = SL_DONE;
    uint32_t leaf = REF_EMPTY, lk = 0;  // the primitive slot being tested; its child slot k in nrec
    uint32_t cont = SL_DONE;            // what follows when there is neither a leaf nor a context
    uint32_t ret_leaf = REF_EMPTY, ret_cont = SL_NORET;  // the TLAS continuation of an entered BLAS
    for (;;) {
        const uint64_t idle = __ballot(ri < 0);
        const uint32_t nidle = (uint32_t)__popcll(idle);
        if (nidle >= PT_REFILL || idle == __ballot(true)) {
            uint32_t base = 0, got = 0;
            if (dead != all_dead) {
                if (wl == 0) {
                    #pragma unroll 1
                    for (uint32_t k = 0; k < PT_POOL_CHUNKS; k++) {
                        const uint32_t c = (home + k) % PT_POOL_CHUNKS;
                        if ((dead >> c) & 1u) continue;
                        const uint32_t lo = c * cs, hi = min(n, lo + cs);
                        const uint32_t old = lo < hi ? atomicAdd(&pool[c * PT_POOL_STRIDE], nidle) : hi;
                        if (lo + old < hi) {
                            base = lo + old;
                            got = min(nidle, hi - base);
                            break;
                        }
                        dead |= 1u << c;
                    }
                }
                base = __builtin_amdgcn_readfirstlane(base);
                got = __builtin_amdgcn_readfirstlane(got);
                dead = __builtin_amdgcn_readfirstlane(dead);
            }
            if (ri < 0) {
                const uint32_t k = (uint32_t)__popcll(idle & ((1ull << wl) - 1ull));
                if (k < got) {
                    ri = (int)(base + k);
                    src.load((uint32_t)ri, o, d, tmax);
                    oct = OCT_FRESH;
                    steps = 0;
                    nrec = REF_EMPTY;
                    ret_leaf = REF_EMPTY;
                    ret_cont = SL_NORET;
                    const uint32_t r = S.qroot;
                    if (r & REF_LEAF) {  // a one-leaf TLAS
                        leaf = r & ~(REF_LEAF | REF_BLOCK);
                        cont = SL_DONE;
                    } else {
                        leaf = REF_EMPTY;
                        cont = CONT_FRESH | (r << 2);
                    }
                }
            }
            if (got == 0 && dead == all_dead && __ballot(ri >= 0) == 0) break;
        }
        if (ri < 0) continue;

        // ---- what this iteration loads: the leaf's next slot, the context's
        // next child, or the record a continuation names (registers only)
        uint32_t lrec = REF_EMPTY;  // node record to load
        bool resume = false;        // ... resuming it after child slot rk (else a descent with up = lup)
        uint32_t rk = 0, lup = SL_DONE;
        bool finished = false;
#pragma unroll 1
        for (int guard = 0; guard < 4; guard++) {
            if (leaf != REF_EMPTY || lrec != REF_EMPTY || finished) break;
            if (nrec != REF_EMPTY) {
                const uint32_t rem = npk >> 8;
                if (rem == 0) {  // the context is exhausted
                    cont = nup;
                    nrec = REF_EMPTY;
                    continue;
                }
                const uint32_t p = (uint32_t)__builtin_ctz(rem);  // the nearest child left
                const uint32_t ci = (npk >> (2 * (3 - p))) & 3u;
                const uint32_t dd = (ndesc >> (8 * ci)) & 0xFFu;
                const uint32_t c = nbase + (dd & 63u);
                const uint32_t rem2 = rem & ~(1u << p);
                npk = (npk & 0xFFu) | rem2 << 8;
                if (dd & Q48_LEAF) {  // a leaf: its slots in turn, the context kept
                    leaf = c;
                    lk = ci;
                } else {  // descend; come back here only if children are left
                    lrec = c;
                    lup = rem2 ? ((nrec << 2) | ci) : nup;
                    nrec = REF_EMPTY;
                }
            } else if (cont == SL_DONE) {
                finished = true;
            } else if (cont == ESC_EXIT) {  // out of a BLAS, or out of the TLAS root
                if (ret_cont == SL_NORET) {
                    finished = true;
                } else {
                    leaf = ret_leaf;
                    cont = ret_cont;
                    ret_leaf = REF_EMPTY;
                    ret_cont = SL_NORET;
                }
            } else {  // a record to (re-)enter
                lrec = (cont >> 2) & (REF_BLOCK - 1u);
                resume = true;
                rk = (cont & CONT_FRESH) ? 4u : (cont & 3u);
                cont = SL_DONE;
            }
        }
        if (++steps > PT_SL_MAX_STEPS) {
            atomicAdd(S.stack_drops, 1u);
            finished = true;
        }
        if (finished) {  // no occluder (BVH.hpp:1108)
            src.any((uint32_t)ri, false);
            ri = -1;
            continue;
        }
        const bool node_step = lrec != REF_EMPTY;
        // one 48-B record either way (three 16-B buffer loads), and a node's
        // escape link beside it
        const uint32_t off = (node_step ? lrec : leaf) * 48u;
        const float4 q0 = q48_buf_load(qrs, off), q1 = q48_buf_load(qrs, off + 16u), q2 = q48_buf_load(qrs, off + 32u);
        const uint32_t e = __builtin_amdgcn_raw_buffer_load_b32(ers, node_step ? lrec * 4u : Q48_OOB_OFFSET, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (oct & OCT_FRESH) {  // a ray claimed this iteration: its origin and direction are in
            inv = inv_dir(d);
            oct = ((d.z < 0) << 2) | ((d.y < 0) << 1) | (d.x < 0);
        }
        if (node_step) {
            if (COUNT) wk.nodes++;
            uint32_t mask;
            float te[4];
            qslab4pe(q0, q1, q2, o, inv, tmax, mask, te);
            const uint32_t perm = q48_perm(s_lut, oct, q0.w);
            const uint32_t desc = __float_as_uint(q2.w);
            uint32_t rem = 0, rpos = 0;
#pragma unroll
            for (int p = 0; p < 4; p++) {
                const uint32_t ci = (perm >> (2 * (3 - p))) & 3u;
                if (((mask >> ci) & 1u) && ((desc >> (8 * ci)) & 0xFFu) != Q48_EMPTY) rem |= 1u << p;
                if (ci == rk) rpos = (uint32_t)p;
            }
            uint32_t up;
            if (resume) {
                // after child slot rk: the positions up to it are done (rk 4:
                // entering afresh); a root's escape (ESC_EXIT) or a BLAS copy's
                // (its TLAS continuation is in ret_cont) leaves the BLAS
                if (rk < 4u) rem &= ~((2u << rpos) - 1u);
                up = (e & ESC_BLAS) ? ESC_EXIT : e;
            } else {
                up = lup;
                if (e != ESC_EXIT && (e & ESC_BLAS)) {  // a copy of a BLAS root: entering the BLAS
                    ret_leaf = REF_EMPTY;
                    ret_cont = lup;
                    up = ESC_EXIT;
                }
            }
            nrec = lrec;
            nbase = __float_as_uint(q2.z);
            ndesc = desc;
            npk = perm | rem << 8;
            nup = up;
        } else {
            // ---- one primitive of the leaf: GeometricPrimitive::IntersectPred
            // (Primitive.cpp:6-26), as trace_spec's primitive side
            const uint32_t w0 = __float_as_uint(q0.w);
            const uint32_t kind = w0 & GF_KIND;
            const uint32_t ps = __float_as_uint(q2.w);  // the primitive's slot
            const uint32_t next = (w0 & GF_LAST) ? REF_EMPTY : leaf + 1u;
            bool anyhit = false;
            if (kind == PT_PRIM_TRIANGLE) {
                if (COUNT) wk.tris++;
                if (!(w0 & GF_PRED_GLM)) {
                    anyhit = tri_pred(o, d, xyz(q0), xyz(q1), xyz(q2), tmax);
                } else {
                    float bx, by, t;
                    anyhit = tri_glm(o, d, xyz(q0), xyz(q1), xyz(q2), bx, by, t) && !(t > tmax || t < PT_EPS) &&
                             (!(w0 & GF_ALPHA) || tri_alpha_cov(w0, __float_as_uint(q1.w), ps, bx, by, o, d));
                }
                leaf = next;
            } else if (kind == PT_PRIM_BLAS) {
                // into the BLAS (Model::IntersectPred, Model.hpp:29-31): the rest
                // of this leaf and of its node wait in ret_leaf / ret_cont
                ret_leaf = next;
                ret_cont = nrec != REF_EMPTY ? ((npk >> 8) ? ((nrec << 2) | lk) : nup) : cont;
                nrec = REF_EMPTY;
                const uint32_t r = __float_as_uint(q1.x);  // the BLAS root (record, or a leaf ref)
                if (r & REF_LEAF) {
                    leaf = r & ~(REF_LEAF | REF_BLOCK);
                    cont = ESC_EXIT;
                } else {
                    leaf = REF_EMPTY;
                    cont = CONT_FRESH | (r << 2);
                }
            } else {
                if (COUNT) wk.tris++;
                if (kind == PT_PRIM_SPHERE && !(w0 & GF_ALPHA)) {
                    const pt_sphere sp{{q0.x, q0.y, q0.z}, q1.x};
                    float t2;
                    anyhit = sphere_root(sp, o, d, tmax, t2);
                } else {
                    anyhit = other_pred(ps, w0, o, d, tmax);
                }
                leaf = next;
            }
            if (anyhit) {  // early exit (BVH.hpp:1104-1105)
                src.any((uint32_t)ri, true);
                ri = -1;
            }
        }
    }
}
