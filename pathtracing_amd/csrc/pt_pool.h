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
#ifndef PT_POOL_CHECK
#define PT_POOL_CHECK 0
#endif
#ifndef PT_ITER_STATS
#define PT_ITER_STATS 0
#endif
#if PT_ITER_STATS
// diagnostics builds: per-iteration wave statistics of the pool kernels,
// [0] iterations [1] refill iterations [2] iterations reaching a step
// [3] with a node lane [4] with a primitive lane [5] node lane-steps
// [6] primitive lane-steps [7] lanes popping [8] with node lanes all on one
// record [9] with primitive lanes all on one slot [10] with a fresh ray's
// setup [11] with an alpha test [12] alpha-testing lanes [13] with a
// non-triangle primitive [14] alpha-testing lanes on their leaf's first slot;
// the runtime prints them
__device__ unsigned long long pt_iter[2][15];
#endif
#if PT_POOL_CHECK
// debugging builds: [0] bad refs (popped instead), [1] shade prim out of range,
// [2] shade saw an unwritten hit, [3] dropped stack pushes; the runtime prints
// them after every render
__device__ unsigned int pt_diag[4];
#endif
// Idle lanes that trigger a refill: fewer claims (one atomic and one
// divergent ray start per refill) against lanes left idle meanwhile.  C4:
// 4 -> 1081, 8 -> 1198, 16 -> 1235, 24 -> 1224, 32 -> 1188 Mrays/s
// (profiles/r02_ab_shade.txt).
#ifndef PT_REFILL
#define PT_REFILL 16
#endif

// Closest-hit pool kernels keep each stack entry's entry distance (BVH4::
// Intersect's entryDist[], BVH.hpp:1128-1135) and drop a popped node or leaf
// whose entry exceeds the current max without fetching it.  In LDS the
// distance is the float's upper 16 bits (truncated toward zero, so never
// above the true entry: a node is dropped only when the reference drops it);
// entries past the LDS part keep the full float in the overflow array.
// PT_POOL_LDS_C: stack entries in LDS for those kernels (4 + 2 B each, so
// 14 entries per lane keep 14 blocks = 28 waves per CU within 160 KiB).
// Off by default: on C4 it drops only 5 % of the node fetches (32.9 -> 31.3
// per ray) and the shorter LDS stack and extra registers (spills at 72
// VGPRs) cost more: 844 -> 676 Mrays/s (gpurun_out/r2b, profiles/r02_ab_c4.txt).
#ifndef PT_ENTRY
#define PT_ENTRY 0
#endif
#ifndef PT_POOL_LDS_C
#define PT_POOL_LDS_C (PT_ENTRY ? 14 : PT_POOL_LDS)
#endif
// Leaf steps test up to two primitives of the leaf (consecutive 48-B slots,
// one 96-B read), so a two-triangle leaf costs one memory round trip.
// Off by default: at 72 VGPRs the second test spills inside the step loop,
// 844 -> 711 Mrays/s on C4 (same A/B).
#ifndef PT_LEAF2
#define PT_LEAF2 0
#endif
// Any-hit visit order: 0 = slot order (BVH4::IntersectPred, BVH.hpp:1099-1102),
// 1 = the closest-hit octant order.  The occlusion result does not depend on
// the order (every primitive's test, alpha included, is a function of the ray
// and the primitive); only the node visit count does.  Octant order finds an
// occluder sooner: C4 k_shadow_pool 10.72 -> 9.44 ms per launch
// (profiles/r02_ab_shade.txt).
#ifndef PT_ANY_OCT
#define PT_ANY_OCT 1
#endif
// Quantized-node slab test with the bounds pre-ordered by the ray's
// direction signs (qslab4pe, bit-identical to slab4pe)
#ifndef PT_QSLAB_ORDERED
#define PT_QSLAB_ORDERED 1
#endif
// Overlapped traversal (trace_spec below) for the quantized-node kernels
// without instances: C4 1280 -> 1302 Mrays/s at 6 waves per SIMD
// (profiles/r03_ab_spec.txt)
#ifndef PT_SPEC
#define PT_SPEC 1
#endif
// PT_Q48 records in the overlapped traversal: child refs formed per pushed
// child (order_children_q48) instead of all four up front
#ifndef PT_Q48_LAZY
#define PT_Q48_LAZY 1
#endif
// overlapped traversal: node and slot loads only on the lanes that take that
// step (exec-masked) instead of every lane reading record / slot 0
#ifndef PT_MASKED_LOADS
#define PT_MASKED_LOADS 0
#endif
// ... or through a buffer resource, lanes without the step out of its range
#ifndef PT_BUFFER_LOADS
#define PT_BUFFER_LOADS 1
#endif
// overlapped traversal: each refill claims the next refill's rays (the claim's
// atomic returns while the wave traverses), and a claimed ray's origin and
// direction load beside its first node load instead of before it.  Off: C4
// closest-hit 3641 -> 3699 ms per frame (a refill then starts PT_REFILL rays,
// not every idle lane; profiles/r04_ab_traversal.txt)
#ifndef PT_PRECLAIM
#define PT_PRECLAIM 0
#endif
// overlapped traversal: a claimed ray's origin / direction load beside its
// first node load and the ray is set up (1/d, octant) after both arrive:
// C4 1636.7 -> 1641.9 Mrays/s (profiles/r04_ab_traversal.txt)
#ifndef PT_DEFER_SETUP
#define PT_DEFER_SETUP 1
#endif
// overlapped traversal: the two pops of an iteration (a leaf into the free leaf
// cursor, then a node) read the top two stack entries together
#ifndef PT_POP2
#define PT_POP2 0  // C4: +0.07 %, noise (profiles/r04_ab_traversal.txt)
#endif
// overlapped traversal: the stack's LDS and overflow parts through separate
// ds / buffer ops (no flat pops waiting on all vector memory; C4: neutral,
// 3640 vs 3641 ms per frame)
#ifndef PT_STACK_SPLIT
#define PT_STACK_SPLIT 1
#endif
// overlapped traversal: the primitive side's triangle test before the node
// side (only its result live across the node side), its hit handling after
// overlapped traversal: a leaf step tests the leaf's next primitive too when
// both are triangles (three more 16-B loads on primitive lanes).  Off: C4
// 1613 -> 1100 Mrays/s at 6 waves (spills), 1346 at 5 waves without spills
// (profiles/r04_ab_traversal.txt)
#ifndef PT_SPEC_LEAF2
#define PT_SPEC_LEAF2 0
#endif
#if PT_SPEC_LEAF2 && !(PT_Q48 && PT_BUFFER_LOADS)
#error "PT_SPEC_LEAF2 needs the buffer-load PT_Q48 form"
#endif
#ifndef PT_TRI_FIRST
#define PT_TRI_FIRST 0
#endif
#ifndef PT_ALPHA_PREFETCH  // A/B option: an alpha record read before its triangle's test
#define PT_ALPHA_PREFETCH 0
#endif
#ifndef PT_PUSH_FAST  // A/B option: branch-light child pushes while the LDS stack has room
#define PT_PUSH_FAST 1
#endif
#ifndef PT_SPHERE_INLINE  // spheres without an alpha test tested inline from their slot
#define PT_SPHERE_INLINE 1
#endif
#define Q48_OOB_OFFSET 0xFFFFFF00u  // + 32 stays below 2^32: never wraps into range
__device__ __forceinline__ float4 q48_buf_load(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
}
// overflow words per stack entry per lane (ref + entry distance)
#define PT_OVF_WORDS 2
// Stack capacity of the pool kernels.  The reference's stack[32] is undefined
// behaviour past 32 entries (BVH.hpp:1128); here the entries past the LDS part
// live in HBM, so a deeper stack costs only that array.  A push past the
// capacity is dropped and counted (DevScene::stack_drops -> pt_stats::
// stack_overflows; the full-size C4 test asserts none).
#ifndef PT_POOL_STACK
#define PT_POOL_STACK 48
#endif

// ---- Overlapped traversal (PT_SPEC).  The pool kernels wait on their loads
// (C4 k_closest_pool: SQ_WAIT_ANY 64 % of wave cycles, VALU issue 42 % busy
// at 2 cycles per wave64 instruction, profiles/r03_valu.txt): a ray costs
// about one dependent memory round trip per iteration, and a lane makes one
// node step or one primitive step per iteration.  Almost every iteration of
// a wave has both node lanes and primitive lanes (C4: 99.9 % / 97 %), so both
// paths are issued anyway.
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
template <bool ANY, bool COUNT, class Src, int LN, int TREE = (ANY ? PT_TREELET_ANY : PT_TREELET)>
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
#if PT_Q48 && PT_BUFFER_LOADS
    const __amdgpu_buffer_rsrc_t qrs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<DevGeom*>(S.qrec), (short)0, (int)S.qrec_bytes, 0x00020000);
#endif
    // closest hit: an accepted hit is stored at once (Src::closest), so the
    // barycentrics and slot need no registers; OCT_FOUND marks that one was
    float tmax = 0;
    int sp = 0;
#if PT_ITER_STATS
    unsigned long long its[15] = {};
    uint32_t lfirst = 0;  // the leaf cursor is on its leaf's first slot
    auto lead = [&]() { return wl == (uint32_t)(__ffsll((unsigned long long)__ballot(true)) - 1); };
#define PT_IT(k, v) do { const unsigned long long v_ = (v); if (lead()) its[k] += v_; } while (0)
#define PT_LF(v) (lfirst = (v))
#else
#define PT_IT(k, v) do { } while (0)
#define PT_LF(v) ((void)0)
#endif
#if PT_STACK_SPLIT
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
#else
    auto push = [&](uint32_t v) {
        if (sp < PT_POOL_STACK) {
            if (LN >= PT_POOL_STACK || sp < LN) s_ref[sp * PT_TRACE_BLOCK + lane] = v;
            else ovf[(size_t)(sp - LN) * G + gl] = v;
            ++sp;
        } else {
            atomicAdd(S.stack_drops, 1u);
        }
    };
    auto pop = [&]() -> uint32_t {
        --sp;
        return (LN >= PT_POOL_STACK || sp < LN) ? s_ref[sp * PT_TRACE_BLOCK + lane] : ovf[(size_t)(sp - LN) * G + gl];
    };
#endif
    auto is_leaf = [](uint32_t r) { return r != REF_EMPTY && (r & REF_LEAF); };
#if PT_PRECLAIM
    // the next refill's rays, claimed at this refill (PT_REFILL of them from
    // chunk pc_chunk; lane 0 holds the atomic's return until then)
    bool pc_valid = false;
    uint32_t pc_chunk = home, pc_old = 0;
#endif
    for (;;) {
        PT_IT(0, 1);
        const uint64_t idle = __ballot(ri < 0);
        const uint32_t nidle = (uint32_t)__popcll(idle);
        if (nidle >= PT_REFILL || idle == __ballot(true)) {
            // claims as in trace_pool
            uint32_t base = 0, got = 0;
            PT_IT(1, 1);
#if PT_PRECLAIM
            if (pc_valid) {  // the batch claimed at the previous refill
                const uint32_t old = __builtin_amdgcn_readfirstlane(pc_old);
                const uint32_t lo = pc_chunk * cs, hi = min(n, lo + cs);
                if (lo + old < hi) {
                    base = lo + old;
                    got = min((uint32_t)PT_REFILL, hi - base);
                } else {
                    dead |= 1u << pc_chunk;
                }
                pc_valid = false;
            }
            if (got == 0 && dead != all_dead) {
#else
            if (dead != all_dead) {
#endif
                uint32_t cc = 0;
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
                            cc = c;
                            break;
                        }
                        dead |= 1u << c;
                    }
                }
                base = __builtin_amdgcn_readfirstlane(base);
                got = __builtin_amdgcn_readfirstlane(got);
                dead = __builtin_amdgcn_readfirstlane(dead);
#if PT_PRECLAIM
                pc_chunk = __builtin_amdgcn_readfirstlane(cc);
#else
                (void)cc;
#endif
            }
            if (ri < 0) {
                const uint32_t k = (uint32_t)__popcll(idle & ((1ull << wl) - 1ull));
                if (k < got) {
                    ri = (int)(base + k);
#if PT_DEFER_SETUP
                    // only the loads here: the ray is set up (1/d, octant) once
                    // this iteration's node loads are in flight too, so the
                    // two round trips overlap (trace_spec's sources never skip
                    // a ray: ClosestSrc / ShadowSrcT::load return true)
                    if constexpr (Src::kInv) src.load_inv((uint32_t)ri, o, d, inv, tmax);
                    else src.load((uint32_t)ri, o, d, tmax);
                    oct = OCT_FRESH;
#else
                    if (!src.load((uint32_t)ri, o, d, tmax)) __builtin_trap();
                    inv = inv_dir(d);
                    oct = ((d.z < 0) << 2) | ((d.y < 0) << 1) | (d.x < 0);
#endif
                    ref = PT_Q48 ? S.qroot : S.root;
                    leaf = REF_EMPTY;
                    sp = 0;
                }
            }
#if PT_PRECLAIM
            // claim the next refill's rays now: the atomic returns while the
            // wave traverses instead of on the refill's critical path
            if (dead != all_dead) {
                #pragma unroll 1
                for (uint32_t k = 0; k < PT_POOL_CHUNKS; k++) {
                    if (!((dead >> pc_chunk) & 1u)) break;
                    pc_chunk = (pc_chunk + 1) % PT_POOL_CHUNKS;
                }
                if (wl == 0) pc_old = atomicAdd(&pool[pc_chunk * PT_POOL_STRIDE], (uint32_t)PT_REFILL);
                pc_valid = true;
            }
            if (got == 0 && dead == all_dead && !pc_valid && __ballot(ri >= 0) == 0) break;
#else
            if (got == 0 && dead == all_dead && __ballot(ri >= 0) == 0) break;
#endif
        }
        if (ri < 0) continue;

        // ---- feed the two cursors from the lane's depth-first order: the
        // leaf cursor takes the next leaf once free, the node side pops unless
        // a BLAS-hop leaf is pending (at most two pops: a leaf popped into the
        // free leaf cursor lets the node side pop once more)
        if (leaf == REF_EMPTY && is_leaf(ref)) {
            leaf = ref;
            PT_LF(1u);
            ref = REF_EMPTY;
        }
        PT_IT(7, __popcll(__ballot(ref == REF_EMPTY && sp > 0)));
#if PT_POP2
        // the top two entries read together (one LDS round trip where the
        // second pop follows a leaf taken by the free leaf cursor)
        if (ref == REF_EMPTY && sp > 0 && !(leaf != REF_EMPTY && (leaf & REF_BLOCK))) {
            uint32_t v1, v2 = REF_EMPTY;
            const bool lds2 = LN >= PT_POOL_STACK || sp <= LN;  // entries sp - 1 and sp - 2 in LDS
            if (lds2) {
                v1 = s_ref[(sp - 1) * PT_TRACE_BLOCK + lane];
                v2 = s_ref[max(sp - 2, 0) * PT_TRACE_BLOCK + lane];  // (unused when sp == 1)
                --sp;
            } else {
                v1 = pop();
            }
            if (leaf == REF_EMPTY && is_leaf(v1)) {
                leaf = v1;
                PT_LF(1u);
                if (sp > 0 && !(leaf & REF_BLOCK)) {
                    if (lds2) {
                        ref = v2;
                        --sp;
                    } else {
                        ref = pop();
                    }
                }
            } else {
                ref = v1;
            }
        }
#else
        #pragma unroll
        for (int k = 0; k < 2; k++) {
            if (ref == REF_EMPTY && sp > 0 && !(leaf != REF_EMPTY && (leaf & REF_BLOCK))) {
                const uint32_t r = pop();
                if (leaf == REF_EMPTY && is_leaf(r)) {
                    leaf = r;
                    PT_LF(1u);
                }
                else ref = r;
            }
        }
#endif
        if (ref == REF_EMPTY && leaf == REF_EMPTY) {  // sp == 0: no hit (any) / closest result
            if (ANY) {
                src.any((uint32_t)ri, false);
            } else {
                if (!(oct & OCT_FOUND)) src.closest((uint32_t)ri, tmax, 0.0f, 0.0f, -1);
                src.done((uint32_t)ri, o, d, tmax, (oct & OCT_FOUND) != 0);
            }
            ri = -1;
            continue;
        }
        const bool node_step = ref != REF_EMPTY && !(ref & REF_LEAF);
        const bool prim_step = leaf != REF_EMPTY;
#if PT_ITER_STATS
        {
            const uint32_t nn = (uint32_t)__popcll(__ballot(node_step)), np = (uint32_t)__popcll(__ballot(prim_step));
            PT_IT(2, 1);
            PT_IT(3, nn > 0);
            PT_IT(4, np > 0);
            PT_IT(5, nn);
            PT_IT(6, np);
            const uint64_t nb = __ballot(node_step), pb = __ballot(prim_step);
            const uint32_t r0 = __builtin_amdgcn_readlane(ref, nb ? __ffsll((unsigned long long)nb) - 1 : 0);
            const uint32_t l0 = __builtin_amdgcn_readlane(leaf, pb ? __ffsll((unsigned long long)pb) - 1 : 0);
            PT_IT(8, nb && __ballot(node_step && ref != r0) == 0);
            PT_IT(9, pb && __ballot(prim_step && leaf != l0) == 0);
        }
#endif
        // both cursors' loads issue before either is used: the node (48 B
        // record, PT_Q48; 64 B DevQNode otherwise) and the primitive slot
        // (48 B); a lane without one reads record / slot 0 (shared lines, no
        // extra traffic)
        const uint32_t slot = prim_step ? (leaf & ~(REF_LEAF | REF_BLOCK)) : 0u;
#if PT_Q48 && PT_BUFFER_LOADS
        // raw buffer loads over the record array: a lane without the step
        // reads past the buffer's end, which returns zeros without a fetch
        // (the runtime keeps the array below 4 GiB in this build)
        // (PT_TREELET: a node in the block's LDS copy of the top records is
        // read there, its buffer load out of range)
        const bool tnode = TREE > 0 && node_step && ref < (uint32_t)TREE;
        const uint32_t noff = (node_step && !tnode) ? ref * 48u : Q48_OOB_OFFSET;
        const uint32_t poff = prim_step ? slot * 48u : Q48_OOB_OFFSET;
        float4 q0 = q48_buf_load(qrs, noff), q1 = q48_buf_load(qrs, noff + 16u), q2 = q48_buf_load(qrs, noff + 32u);
        const float4 g0 = q48_buf_load(qrs, poff), g1 = q48_buf_load(qrs, poff + 16u), g2 = q48_buf_load(qrs, poff + 32u);
        if constexpr (TREE > 0) {
            if (tnode) {
                const float4* tr = reinterpret_cast<const float4*>(s_lut + Q48_LUT_BYTES) + 3u * ref;
                q0 = tr[0];
                q1 = tr[1];
                q2 = tr[2];
            }
        }
#if PT_SPEC_LEAF2
        const uint32_t poff2 = prim_step ? poff + 48u : Q48_OOB_OFFSET;
        const float4 h0 = q48_buf_load(qrs, poff2), h1 = q48_buf_load(qrs, poff2 + 16u),
                     h2 = q48_buf_load(qrs, poff2 + 32u);
#endif
#elif PT_Q48 && PT_MASKED_LOADS
        // each side's loads under its own exec mask: a lane without a node
        // (primitive) step issues no node (slot) loads, so the vector memory
        // pipe processes only the lanes that step (its rate is per lane)
        float4 q0, q1, q2, g0, g1, g2;  // (lanes without the step: unused values)
        if (node_step) {
            const float4* __restrict__ qn = reinterpret_cast<const float4*>(S.qrec + ref);
            q0 = qn[0];
            q1 = qn[1];
            q2 = qn[2];
        }
        if (prim_step) {
            const float4* __restrict__ qg = reinterpret_cast<const float4*>(S.qrec + slot);
            g0 = qg[0];
            g1 = qg[1];
            g2 = qg[2];
        }
#elif PT_Q48
        const float4* __restrict__ qn = reinterpret_cast<const float4*>(S.qrec + (node_step ? ref : 0u));
        const float4* __restrict__ qg = reinterpret_cast<const float4*>(S.qrec + slot);
        const float4 q0 = qn[0], q1 = qn[1], q2 = qn[2];
#else
        const float4* __restrict__ qn = reinterpret_cast<const float4*>(S.qnodes + (node_step ? ref : 0u));
        const float4* __restrict__ qg = reinterpret_cast<const float4*>(S.geom + slot);
        const float4 q0 = qn[0], q1 = qn[1], q2 = qn[2], qc = qn[3];
#endif
#if !(PT_Q48 && (PT_MASKED_LOADS || PT_BUFFER_LOADS))
        const float4 g0 = qg[0], g1 = qg[1], g2 = qg[2];
#endif
        __builtin_amdgcn_sched_barrier(0);  // (the scheduler would sink the slot loads past the node side)
#if PT_DEFER_SETUP
        PT_IT(10, __ballot(oct & OCT_FRESH) != 0);
        if (oct & OCT_FRESH) {  // a ray claimed this iteration: its origin and direction are in
            if constexpr (!Src::kInv) inv = inv_dir(d);
            oct = ((d.z < 0) << 2) | ((d.y < 0) << 1) | (d.x < 0);
        }
#endif
#if PT_TRI_FIRST
        // the triangle test first: its 12 slot words die before the node side,
        // and only its result (t, barycentrics, flags) stays live across it
        const uint32_t w0 = __float_as_uint(g0.w);
        const bool pred = ANY && !(w0 & GF_PRED_GLM);
        float bx = 0, by = 0, t = 0;
        bool tri_hit;
        if (pred) tri_hit = PT_TRI_PK ? tri_pred_pk(o, d, xyz(g0), xyz(g1), xyz(g2), tmax)
                                      : tri_pred(o, d, xyz(g0), xyz(g1), xyz(g2), tmax);
        else tri_hit = (PT_TRI_PK ? tri_glm_pk(o, d, xyz(g0), xyz(g1), xyz(g2), bx, by, t)
                                  : tri_glm(o, d, xyz(g0), xyz(g1), xyz(g2), bx, by, t)) &&
                       !(t > tmax || t < PT_EPS);
        // BLAS hop: its root ref (b.x); triangle: its alpha record (b.w)
        const uint32_t g1v = (w0 & GF_KIND) == PT_PRIM_BLAS ? __float_as_uint(g1.x) : __float_as_uint(g1.w);
        const uint32_t g2w = __float_as_uint(g2.w);
        __builtin_amdgcn_sched_barrier(0);
#endif

        // ---- node side
        {
            uint32_t mask;
            float te[4];
            qslab4pe(q0, q1, q2, o, inv, tmax, mask, te);
            if (!node_step) mask = 0;
            uint32_t perm = 0xE4u;
#if PT_Q48
            if (!ANY || PT_ANY_OCT) perm = q48_perm(s_lut, oct, q0.w);
#if PT_Q48_LAZY
#if PT_PUSH_FAST
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
#else
            const uint32_t cand = order_children_q48(mask, q2.z, q2.w, perm, [&](uint32_t v) { push(v); });
#endif
#else
            const uint4 ch = q48_children(q2.z, q2.w);
#endif
#else
            if (!ANY || PT_ANY_OCT) {
                const uint32_t ow = ((oct >> 2) & 1u) ? __float_as_uint(q2.w) : __float_as_uint(q2.z);
                perm = (ow >> (8 * (oct & 3))) & 0xFFu;
            }
            const uint4 ch = make_uint4(__float_as_uint(qc.x), __float_as_uint(qc.y), __float_as_uint(qc.z),
                                        __float_as_uint(qc.w));
#endif
#if !(PT_Q48 && PT_Q48_LAZY)
            const uint32_t cand = order_children(mask, ch, perm, [&](uint32_t v) { push(v); });
#endif
            if (node_step) {
                if (COUNT) wk.nodes++;
                ref = cand;
            }
        }
        // ---- primitive side.  The triangle test runs on every lane (its
        // result kept only on primitive lanes), so the slot loads are used
        // outside the branches.
        {
#if !PT_TRI_FIRST
            const uint32_t w0 = __float_as_uint(g0.w);
            const bool pred = ANY && !(w0 & GF_PRED_GLM);
#if PT_ALPHA_PREFETCH
            // an alpha-tested triangle's record (slot b.w), read before its
            // test so the load's latency overlaps the test
            const uint32_t ai = __float_as_uint(g1.w);
            const bool alane = prim_step && (w0 & GF_KIND) == PT_PRIM_TRIANGLE && (w0 & GF_ALPHA) && !pred &&
                               ai != ALPHA_NONE;
            DevAlpha arec;
            if (__ballot(alane)) {
                const float4* ap = reinterpret_cast<const float4*>(S.alpha + (alane ? ai : 0u));
                const float4 a0 = ap[0], a1 = ap[1], a2 = ap[2];
                arec = __builtin_bit_cast(DevAlpha, (DevGeom{a0, a1, a2}));
            }
#endif
            float bx = 0, by = 0, t = 0;
            bool tri_hit;
            if (pred) tri_hit = PT_TRI_PK ? tri_pred_pk(o, d, xyz(g0), xyz(g1), xyz(g2), tmax)
                                          : tri_pred(o, d, xyz(g0), xyz(g1), xyz(g2), tmax);
            else tri_hit = (PT_TRI_PK ? tri_glm_pk(o, d, xyz(g0), xyz(g1), xyz(g2), bx, by, t)
                                      : tri_glm(o, d, xyz(g0), xyz(g1), xyz(g2), bx, by, t)) &&
                           !(t > tmax || t < PT_EPS);
            const uint32_t g1v = (w0 & GF_KIND) == PT_PRIM_BLAS ? __float_as_uint(g1.x) : __float_as_uint(g1.w);
            const uint32_t g2w = __float_as_uint(g2.w);
#endif
            const uint32_t kind = w0 & GF_KIND;
#if PT_ITER_STATS
            {
                const uint64_t ab = __ballot(prim_step && kind == PT_PRIM_TRIANGLE && tri_hit && !pred &&
                                             (w0 & GF_ALPHA));
                PT_IT(11, ab != 0);
                PT_IT(12, __popcll(ab));
                PT_IT(13, __ballot(prim_step && kind != PT_PRIM_TRIANGLE && kind != PT_PRIM_BLAS) != 0);
                PT_IT(14, __popcll(ab & __ballot(lfirst != 0)));
            }
#endif
#if PT_SPEC_LEAF2
            const uint32_t w1 = __float_as_uint(h0.w);
            const bool pred2 = ANY && !(w1 & GF_PRED_GLM);
            float bx2 = 0, by2 = 0, t2r = 0;
            bool tri_hit2;
            if (pred2) tri_hit2 = tri_pred(o, d, xyz(h0), xyz(h1), xyz(h2), tmax);
            else tri_hit2 = tri_glm(o, d, xyz(h0), xyz(h1), xyz(h2), bx2, by2, t2r);
            const uint32_t ps2 = __float_as_uint(h2.w);
#endif
            if (prim_step) {
                bool anyhit = false;
                uint32_t next = (w0 & GF_LAST) ? REF_EMPTY : (REF_LEAF | (leaf & REF_BLOCK) | (slot + 1));
                // the primitive's slot (PT_Q48: the record keeps it in c.w)
                const uint32_t ps = PT_Q48 ? g2w : slot;
                if (kind == PT_PRIM_TRIANGLE) {
                    if (COUNT) wk.tris++;
#if PT_ALPHA_PREFETCH
                    if (tri_hit && (pred || !(w0 & GF_ALPHA) ||
                                    (alane ? tri_alpha_rec(arec, ps, bx, by, o, d) : tri_alpha(g1v, ps, bx, by, o, d)))) {
#else
                    if (tri_hit && (pred || !(w0 & GF_ALPHA) || tri_alpha(g1v, ps, bx, by, o, d))) {
#endif
                        if (ANY) {
                            anyhit = true;
                        } else {
                            if ((oct & (OCT_FOUND | OCT_TIE)) == OCT_FOUND && t == tmax) {
                                oct |= OCT_TIE;  // an exact tie: the reference's culling decides (pt_pool.h top)
                                src.tie((uint32_t)ri);
                            }
                            tmax = t;
                            oct |= OCT_FOUND;
                            src.closest((uint32_t)ri, t, bx, by, (int)ps);
                        }
                    }
#if PT_SPEC_LEAF2
                    // the leaf's next primitive in the same step when it is a
                    // triangle too (tested after the first, against its max)
                    if (!(w0 & GF_LAST) && !(ANY && anyhit) && (w1 & GF_KIND) == PT_PRIM_TRIANGLE) {
                        if (COUNT) wk.tris++;
                        if (!pred2) tri_hit2 = tri_hit2 && !(t2r > tmax || t2r < PT_EPS);
                        if (tri_hit2 && (pred2 || !(w1 & GF_ALPHA) || tri_alpha(__float_as_uint(h1.w), ps2, bx2, by2, o, d))) {
                            if (ANY) {
                                anyhit = true;
                            } else {
                                if ((oct & (OCT_FOUND | OCT_TIE)) == OCT_FOUND && t2r == tmax) {
                                    oct |= OCT_TIE;
                                    src.tie((uint32_t)ri);
                                }
                                tmax = t2r;
                                oct |= OCT_FOUND;
                                src.closest((uint32_t)ri, t2r, bx2, by2, (int)ps2);
                            }
                        }
                        next = (w1 & GF_LAST) ? REF_EMPTY : (REF_LEAF | (leaf & REF_BLOCK) | (slot + 2));
                    }
#endif
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
                    const bool sph = PT_SPHERE_INLINE && kind == PT_PRIM_SPHERE && !(w0 & GF_ALPHA);
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
                PT_LF(0u);
                if (ANY && anyhit) {  // early exit (BVH.hpp:1104-1105)
                    src.any((uint32_t)ri, true);
                    ri = -1;
                }
            }
        }
    }
#if PT_ITER_STATS
    for (int k = 0; k < 15; k++)
        if (its[k]) atomicAdd(&pt_iter[ANY ? 1 : 0][k], its[k]);
#endif
#undef PT_IT
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
// POOL = false: no refill, lane i of the grid traces ray i (small scenes,
// where traversal lengths are uniform and the claims would only cost).
// LN: stack entries in LDS (s_ref, and s_ent for closest hit with PT_ENTRY);
// the rest in ovf ([entry][grid lane] refs, then as many entry distances).
template <bool ANY, bool COUNT, class Src, bool POOL = true, bool INST = true,
          int LN = (ANY ? PT_POOL_LDS : PT_POOL_LDS_C), bool QN = false>
__device__ void trace_pool(uint32_t n, uint32_t* __restrict__ pool, Src& src, uint32_t* s_ref, uint16_t* s_ent,
                           uint32_t* __restrict__ ovf, TraceWork& wk, const uint8_t* s_lut = nullptr) {
    constexpr bool ENT = PT_ENTRY && !ANY;
    static_assert(!(PT_Q48 && (PT_WIDE || PT_ENTRY)), "PT_WIDE / PT_ENTRY read the 64-B DevQNode form (PT_Q48=0)");
    constexpr bool Q48 = QN && PT_Q48;  // nodes and leaf slots in the 48-B records
    if constexpr (PT_SPEC && QN && POOL && !INST && !ENT && !PT_WIDE) {
        trace_spec<ANY, COUNT, Src, LN>(n, pool, src, s_ref, ovf, wk, s_lut);
        return;
    }
    const uint32_t lane = threadIdx.x;
    const uint32_t gl = blockIdx.x * PT_TRACE_BLOCK + lane, G = gridDim.x * PT_TRACE_BLOCK;
    uint32_t* __restrict__ ovf_e = ovf + (size_t)(PT_POOL_STACK - LN) * G;
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
#if PT_ITER_STATS
    unsigned long long its[15] = {};
    // counted once per wave: by the first active lane of the counting point
    auto lead = [&]() { return wl == (uint32_t)(__ffsll((unsigned long long)__ballot(true)) - 1); };
#define PT_IT(k, v) do { const unsigned long long v_ = (v); if (lead()) its[k] += v_; } while (0)
#else
#define PT_IT(k, v) do { } while (0)
#endif
    // pushes beyond PT_POOL_STACK are dropped and counted;
    // e < 0: never dropped at pop (BLAS roots: a fresh traversal, entry 0)
    auto push = [&](uint32_t v, float e = -1.0f) {
        if (sp < PT_POOL_STACK) {
            if (LN >= PT_POOL_STACK || sp < LN) {
                s_ref[sp * PT_TRACE_BLOCK + lane] = v;
                if (ENT) s_ent[sp * PT_TRACE_BLOCK + lane] = (uint16_t)(__float_as_uint(e) >> 16);
            } else {
                ovf[(size_t)(sp - LN) * G + gl] = v;
                if (ENT) ovf_e[(size_t)(sp - LN) * G + gl] = __float_as_uint(e);
            }
            ++sp;
        } else {
            atomicAdd(S.stack_drops, 1u);
        }
    };
    // pop; false: the popped entry lies beyond the current max (ENT only)
    auto pop = [&](uint32_t& r) -> bool {
        --sp;
        float e = -1.0f;
        if (LN >= PT_POOL_STACK || sp < LN) {
            r = s_ref[sp * PT_TRACE_BLOCK + lane];
            if (ENT) e = __uint_as_float((uint32_t)s_ent[sp * PT_TRACE_BLOCK + lane] << 16);
        } else {
            r = ovf[(size_t)(sp - LN) * G + gl];
            if (ENT) e = __uint_as_float(ovf_e[(size_t)(sp - LN) * G + gl]);
        }
        return !(ENT && e > tmax);
    };
    auto start = [&]() {
        inv = inv_dir(d);
        oct = ((d.z < 0) << 2) | ((d.y < 0) << 1) | (d.x < 0);
        ref = Q48 ? S.qroot : S.root;
        sp = 0;
        best = -1;
        bb1 = bb2 = 0;
    };
    if (!POOL) {
        const uint32_t gi = blockIdx.x * PT_TRACE_BLOCK + lane;
        if (gi < n && src.load(gi, o, d, tmax)) {
            ri = (int)gi;
            start();
        }
    }
    for (;;) {
        if (!POOL) {
            if (__ballot(ri >= 0) == 0) break;
            if (ri < 0) continue;
        }
        PT_IT(0, 1);
        const uint64_t idle = __ballot(ri < 0);
        const uint32_t nidle = (uint32_t)__popcll(idle);
        if (POOL && (nidle >= PT_REFILL || idle == __ballot(true))) {
            // claim exactly as many rays as lanes are idle (one atomic) from the
            // home chunk or the next non-empty one; no reserve is held, so no
            // wave sits on unstarted rays while others run dry
            uint32_t base = 0, got = 0;
            PT_IT(1, 1);
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

        // ---- one step of this lane's traversal: one cluster or one leaf step
        // (one or two primitives).  Node lanes and primitive lanes issue their
        // loads in the same pass (one memory round trip per step for the whole
        // wave); a leaf continues at ref = REF_LEAF | next slot.
        PT_IT(7, __popcll(__ballot(ref == REF_EMPTY)));
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
                uint32_t r;
                if (pop(r)) {
                    ref = r;
                    break;
                }
            }
            if (finished) {  // no hit (any) / closest result
                if (ANY) {
                    src.any((uint32_t)ri, false);
                } else {
                    src.closest((uint32_t)ri, tmax, bb1, bb2, best);
                    src.done((uint32_t)ri, o, d, tmax, best >= 0);
                }
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
#if PT_ITER_STATS
        {
            const uint32_t nn = (uint32_t)__popcll(__ballot(node_step)), np = (uint32_t)__popcll(__ballot(!node_step));
            PT_IT(2, 1);
            PT_IT(3, nn > 0);
            PT_IT(4, np > 0);
            PT_IT(5, nn);
            PT_IT(6, np);
        }
#endif
        const uint32_t idx = ref & ~(QN ? REF_LEAF | REF_BLOCK : REF_LEAF);
#if PT_POOL_CHECK
        if (!Q48 && (node_step ? idx >= S.n_nodes : idx >= S.n_prims)) {  // debugging builds only
            atomicAdd(&pt_diag[0], 1u);
            ref = REF_EMPTY;
            continue;
        }
#endif
        // all loads issue before any use: a primitive lane reads its 48-byte
        // slot (and the next one with PT_LEAF2; the slot array has a pad slot
        // at its end) and repeats its first 16 bytes for the node-only words
        // (same line, no extra traffic), and the cluster test below runs
        // unconditionally (its result masked off on primitive lanes) so the
        // compiler cannot sink the node loads behind the primitive branch.
        // QN: 64-byte quantized nodes (DevQNode), four loads per step.
        const uint32_t nk = node_step ? 1u : 0u;
        float4 q0, q1, q2, q3, q4, q5;
        uint32_t mask;
        float te[4];
        uint4 ch;
        uint32_t ow0, ow1;
        uint4 ch1 = make_uint4(REF_EMPTY, REF_EMPTY, REF_EMPTY, REF_EMPTY);
        uint32_t wperm = 0;
        if constexpr (QN && PT_WIDE) {
            static_assert(!PT_ENTRY, "wide nodes keep no entry distances");
            // DevWNode: 8 loads; primitive lanes re-read their slot's first 16 B
            const float4* __restrict__ q = node_step
                                               ? reinterpret_cast<const float4*>(
                                                     reinterpret_cast<const DevWNode*>(S.qnodes) + idx)
                                               : reinterpret_cast<const float4*>(S.geom + idx);
            q0 = q[0];
            q1 = q[1];
            q2 = q[2];
            const float4 qz = q[3 * nk], qc0 = q[4 * nk], qc1 = q[5 * nk], qo0 = q[6 * nk], qo1 = q[7 * nk];
            q3 = q4 = q5 = q0;
            uint32_t m0, m1;
            qslab4pe(q0, q1, make_float4(qz.x, qz.y, 0.0f, 0.0f), o, inv, tmax, m0, te);
            qslab4pe(q0, q2, make_float4(qz.z, qz.w, 0.0f, 0.0f), o, inv, tmax, m1, te);
            mask = m0 | (m1 << 4);
            ch = make_uint4(__float_as_uint(qc0.x), __float_as_uint(qc0.y), __float_as_uint(qc0.z),
                            __float_as_uint(qc0.w));
            ch1 = make_uint4(__float_as_uint(qc1.x), __float_as_uint(qc1.y), __float_as_uint(qc1.z),
                             __float_as_uint(qc1.w));
            const float4 qo = (oct & 4u) ? qo1 : qo0;
            const float plo = (oct & 1u) ? qo.y : qo.x, phi = (oct & 1u) ? qo.w : qo.z;
            wperm = __float_as_uint((oct & 2u) ? phi : plo);
            ow0 = ow1 = 0;
        } else if constexpr (Q48) {
            // node records and leaf slots share the array: three loads either way
            const float4* __restrict__ q = reinterpret_cast<const float4*>(S.qrec + idx);
            q0 = q[0];
            q1 = q[1];
            q2 = q[2];
            q3 = q4 = q5 = q0;
            qslab4pe(q0, q1, q2, o, inv, tmax, mask, te);
            ch = q48_children(q2.z, q2.w);
            ow0 = ow1 = 0;  // the order byte comes from s_lut below
        } else if constexpr (QN) {
            const float4* __restrict__ q = node_step ? reinterpret_cast<const float4*>(S.qnodes + idx)
                                                     : reinterpret_cast<const float4*>(S.geom + idx);
            q0 = q[0];
            q1 = q[1];
            q2 = q[2];
            const float4 qc = q[3 * nk];
            q3 = q4 = q5 = q0;  // no second leaf primitive in this form
#if PT_QSLAB_ORDERED
            qslab4pe(q0, q1, q2, o, inv, tmax, mask, te);
#else
            float4 xmn, xmx, ymn, ymx, zmn, zmx;
            qnode_boxes(q0, q1, q2, xmn, xmx, ymn, ymx, zmn, zmx);
            slab4pe(xmn, xmx, ymn, ymx, zmn, zmx, o, inv, tmax, mask, te);
#endif
            ch = make_uint4(__float_as_uint(qc.x), __float_as_uint(qc.y), __float_as_uint(qc.z),
                            __float_as_uint(qc.w));
            ow0 = __float_as_uint(q2.z);
            ow1 = __float_as_uint(q2.w);
        } else {
            const float4* __restrict__ q = node_step ? reinterpret_cast<const float4*>(S.nodes + idx)
                                                     : reinterpret_cast<const float4*>(S.geom + idx);
            constexpr uint32_t pk = PT_LEAF2 ? 1u : 0u;
            const uint32_t k3 = 3u * (nk | pk);
            q0 = q[0];
            q1 = q[1];
            q2 = q[2];
            q3 = q[k3];
            q4 = q[k3 ? 4u : 0u];
            q5 = q[k3 ? 5u : 0u];
            const float4 q6 = q[6 * nk], q7 = q[7 * nk];
            slab4pe(q0, q1, q2, q3, q4, q5, o, inv, tmax, mask, te);
            ch = make_uint4(__float_as_uint(q6.x), __float_as_uint(q6.y), __float_as_uint(q6.z),
                            __float_as_uint(q6.w));
            ow0 = __float_as_uint(q7.x);
            ow1 = __float_as_uint(q7.y);
        }
        {
            if (!node_step) mask = 0;  // no children on primitive lanes
            // visit order: slot order for any hit (BVH.hpp:1099-1102), octant
            // order far -> near for closest hit (BVH4::LUT, BVH.hpp:1195-1204)
            uint32_t perm = 0xE4u;
            if (!ANY || PT_ANY_OCT) {
                if constexpr (Q48) {
                    perm = q48_perm(s_lut, oct, q0.w);
                } else {
                    const uint32_t ow = ((oct >> 2) & 1u) ? ow1 : ow0;
                    perm = (ow >> (8 * (oct & 3))) & 0xFFu;
                }
            }
            uint32_t cand;
            if constexpr (QN && PT_WIDE) {
                // any hit in slot order unless PT_ANY_OCT (identity: slot k at bits 3k)
                const uint32_t wp = (!ANY || PT_ANY_OCT) ? wperm : 0xFAC688u;
                cand = order_children8(mask, ch, ch1, wp, [&](uint32_t v) { push(v); });
            } else if (ENT) {
                cand = order_children_e(mask, ch, perm, te, push);
            } else {
                cand = order_children(mask, ch, perm, [&](uint32_t v) { push(v); });
            }
            if (node_step) {
                if (COUNT) wk.nodes++;
                ref = cand;
                continue;
            }
        }
        // leaf primitives at slot idx (and idx + 1); PT_Q48: record idx,
        // whose c.w is the slot
        {
            const uint32_t slot = Q48 ? __float_as_uint(q2.w) : idx;
            const uint32_t w0 = __float_as_uint(q0.w);
            const uint32_t kind = w0 & GF_KIND;
            bool anyhit = false;
            // one triangle of the leaf: Intersect (glm) or IntersectPred
            // semantics + the material alpha test (Primitive.cpp:6-26)
            auto tri = [&](uint32_t sl, uint32_t w, float4 a, float4 b, float4 c) {
                if (COUNT) wk.tris++;
                if (ANY && !(w & GF_PRED_GLM)) {
                    if (tri_pred(o, d, xyz(a), xyz(b), xyz(c), tmax)) anyhit = true;
                } else {
                    float bx, by, t;
                    if (tri_glm(o, d, xyz(a), xyz(b), xyz(c), bx, by, t) && !(t > tmax || t < PT_EPS)) {
                        if (!(w & GF_ALPHA) || tri_alpha(__float_as_uint(b.w), sl, bx, by, o, d)) {
                            if (ANY) {
                                anyhit = true;
                            } else {
                                if (POOL && best >= 0 && t == tmax && !(oct & OCT_TIE)) {
                                    oct |= OCT_TIE;
                                    src.tie((uint32_t)ri);
                                }
                                tmax = t;
                                best = (int)sl;
                                bb1 = bx;
                                bb2 = by;
                                oct |= (oct & OCT_INST) << 1;  // OCT_HIT inside an instance
                            }
                        }
                    }
                }
            };
            uint32_t next = (w0 & GF_LAST) ? REF_EMPTY : (REF_LEAF | (idx + 1));
            if (kind == PT_PRIM_TRIANGLE) {
                tri(slot, w0, q0, q1, q2);
                const uint32_t w1 = __float_as_uint(q3.w);
                if (PT_LEAF2 && !QN && next != REF_EMPTY && (w1 & GF_KIND) == PT_PRIM_TRIANGLE && !(ANY && anyhit)) {
                    tri(slot + 1, w1, q3, q4, q5);
                    next = (w1 & GF_LAST) ? REF_EMPTY : (REF_LEAF | (slot + 2));
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
                        if (POOL && best >= 0 && t == tmax && !(oct & OCT_TIE)) {
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
#if PT_ITER_STATS
    for (int k = 0; k < 15; k++)
        if (its[k]) atomicAdd(&pt_iter[ANY ? 1 : 0][k], its[k]);
#endif
#undef PT_IT
}
