// Device BVH build, part of pt_runtime.hip's
// translation unit (included at its end; uses pt_ctx / fail / HIPCHK).
//
// Builds the binary SAH tree of BVHBase::BuildBaseThreaded (BVH.hpp:290-390)
// on the GPU, decision for decision as pt_bvh.cpp's build2 does on the host,
// and collapses it into BVH4 clusters (BVH.hpp:788-1017) on the GPU.  The
// output is byte-identical to pt_bvh4_build because every quantity the
// reference's decisions depend on is order-independent or computed in the
// reference's own order:
//   * node boxes, centroid bounds and bin boxes are min/max reductions
//     (order-free; done with ordered-integer atomics) and bin counts are sums;
//   * the SAH sweep over a node's bins runs in one lane, in the reference's
//     operand order with GCC's FMA contraction choices written out (fmaf);
//   * std::partition (libstdc++ two-pointer, stl_algo.h __partition for
//     bidirectional iterators) swaps the k-th misplaced "false" from the left
//     with the k-th misplaced "true" from the right: with two exclusive counts
//     from one device scan every pair is found and swapped in parallel;
//   * binary node numbering (an atomic counter in the reference too) does not
//     reach the output: the collapse numbers clusters in pre-order.
// Level-synchronous passes handle every node wider than kSmall primitives
// (binning with a workgroup-local histogram when a workgroup lies inside one
// node); narrower subtrees are finished one per lane by a sequential restatement
// of build2.  Caveat: a min/max tie between -0.0f and +0.0f keeps the sign of
// the first element in the reference and the smaller key here.
#include <limits>

#include <rocprim/device/device_scan.hpp>

#include "pt_bvh_internal.h"  // PtBvh2Node

#pragma clang fp contract(off)

namespace bvhg {

constexpr uint32_t kLeaf = 2;    // BVH.hpp:95 leafSize
constexpr uint32_t kSmall = 48;  // subtrees up to this many primitives finish in one lane (tuned on C4)
constexpr uint32_t kInv = 0xFFFFFFFFu;
constexpr int kBlock = 256;
static_assert(kSmall < 1024, "one-lane subtrees use at most 16 bins");

struct Item {
    float mn[3], mx[3], c[3];
    uint32_t idx;
};  // 40 B
struct Task {
    uint32_t first, last, node, pad;
};
// Ordered-integer keys: [0,3) box min, [3,6) box max, [6,9) centroid min,
// [9,12) centroid max; ntrue = primitives with centroid <= split position.
struct Acc {
    uint32_t k[12];
    uint32_t ntrue, pad[3];
};
struct Dec {
    float lo[3], scale[3];
    uint32_t nbins, valid, split, axis;
    float pos;
    uint32_t mid, lt, rt;
};
struct Ctr {
    uint32_t next_tasks, n_small, nodes, pad;
};

__device__ __forceinline__ uint32_t fkey(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float kval(uint32_t k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}
__device__ __forceinline__ bool key_is_min(int j) { return j < 3 || (j >= 6 && j < 9); }

// Box::area of pt_bvh.cpp as GCC contracts ex*ey + ey*ez + ez*ex on x86-64-v3
__device__ __forceinline__ float area(const float* mn, const float* mx) {
    const float ex = mx[0] - mn[0], ey = mx[1] - mn[1], ez = mx[2] - mn[2];
    return __builtin_fmaf(ex, ez, __builtin_fmaf(ey, ex, ey * ez));
}
// Box::grow: std::min(mn, o) / std::max(mx, o) keep the first operand on ties
__device__ __forceinline__ void grow(float* mn, float* mx, const float* omn, const float* omx) {
    for (int a = 0; a < 3; a++) {
        mn[a] = omn[a] < mn[a] ? omn[a] : mn[a];
        mx[a] = mx[a] < omx[a] ? omx[a] : mx[a];
    }
}
__device__ __forceinline__ uint32_t nbins_for(uint32_t span) { return span >= 1024 ? 32 : span >= 64 ? 16 : 8; }

__device__ __forceinline__ void acc_empty(Acc& a) {
    for (int j = 0; j < 3; j++) {
        a.k[j] = fkey(__builtin_inff());
        a.k[3 + j] = fkey(-__builtin_inff());
        a.k[6 + j] = fkey(3.40282347e38f);   // build2's centroid bounds start at
        a.k[9 + j] = fkey(-3.40282347e38f);  // +-numeric_limits<float>::max()
    }
    a.ntrue = 0;
}

__device__ __forceinline__ void item_keys(const Item& it, uint32_t v[12]) {
    for (int a = 0; a < 3; a++) {
        v[a] = fkey(it.mn[a]);
        v[3 + a] = fkey(it.mx[a]);
        v[6 + a] = fkey(it.c[a]);
        v[9 + a] = fkey(it.c[a]);
    }
}

// Lanes grouped by `key` (a task); each group reduces in registers and its
// first lane issues one atomic per accumulator word.
__device__ void wave_acc(Acc* acc, uint32_t key, bool active, const uint32_t v[12]) {
    const int lane = __lane_id();
    unsigned long long pending = __ballot(active);
    while (pending) {
        const int leader = __ffsll(pending) - 1;
        const uint32_t k = __shfl(key, leader);
        const bool mine = active && ((pending >> lane) & 1ull) && key == k;
        const unsigned long long m = __ballot(mine);
#pragma unroll
        for (int j = 0; j < 12; j++) {
            const bool mn = key_is_min(j);
            uint32_t x = mine ? v[j] : (mn ? 0xFFFFFFFFu : 0u);
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) {
                const uint32_t y = __shfl_xor(x, off);
                x = mn ? min(x, y) : max(x, y);
            }
            if (lane == leader) {
                if (mn)
                    atomicMin(&acc[k].k[j], x);
                else
                    atomicMax(&acc[k].k[j], x);
            }
        }
        pending &= ~m;
    }
}

__device__ void wave_count(Acc* acc, uint32_t key, bool active, uint32_t v) {
    const int lane = __lane_id();
    unsigned long long pending = __ballot(active);
    while (pending) {
        const int leader = __ffsll(pending) - 1;
        const uint32_t k = __shfl(key, leader);
        const bool mine = active && ((pending >> lane) & 1ull) && key == k;
        const unsigned long long m = __ballot(mine);
        uint32_t x = mine ? v : 0u;
        for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off);
        if (lane == leader && x) atomicAdd(&acc[k].ntrue, x);
        pending &= ~m;
    }
}

// Item passes cover kSpan = kBlock * kIPT consecutive items per workgroup
// (round r touches items b0 + r*kBlock + tid, coalesced).  When a workgroup
// lies inside one node, accumulators stay in registers across the rounds and
// are reduced once per workgroup: a few global atomics per 4096 items instead
// of per wave (the top levels otherwise serialise on a dozen addresses).
constexpr int kIPT = 16;
constexpr uint32_t kSpan = kBlock * kIPT;

__device__ __forceinline__ void acc_ident(uint32_t a[12]) {
#pragma unroll
    for (int j = 0; j < 12; j++) a[j] = key_is_min(j) ? 0xFFFFFFFFu : 0u;
}
__device__ __forceinline__ void acc_merge(uint32_t a[12], const uint32_t v[12]) {
#pragma unroll
    for (int j = 0; j < 12; j++) a[j] = key_is_min(j) ? min(a[j], v[j]) : max(a[j], v[j]);
}
// wave reduction of a[12] into the workgroup's LDS accumulator s[12]
__device__ __forceinline__ void wave_to_lds(uint32_t* s, const uint32_t a[12]) {
#pragma unroll
    for (int j = 0; j < 12; j++) {
        const bool mn = key_is_min(j);
        uint32_t x = a[j];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const uint32_t y = __shfl_xor(x, off);
            x = mn ? min(x, y) : max(x, y);
        }
        if (__lane_id() == 0) {
            if (mn)
                atomicMin(&s[j], x);
            else
                atomicMax(&s[j], x);
        }
    }
}
__device__ __forceinline__ void lds_to_global(Acc* acc, uint32_t key, const uint32_t* s, int j) {
    const bool mn = key_is_min(j);
    if (s[j] == (mn ? 0xFFFFFFFFu : 0u)) return;
    if (mn)
        atomicMin(&acc[key].k[j], s[j]);
    else
        atomicMax(&acc[key].k[j], s[j]);
}

// PrimitiveInfo (BVH.hpp:84-93): box + centroid 0.5*(max+min); the root task
// accumulates every box.
__global__ __launch_bounds__(kBlock) void k_init(const float* __restrict__ boxes, uint32_t n,
                                                 Item* __restrict__ items, uint32_t* __restrict__ seg, Acc* acc) {
    __shared__ uint32_t s_acc[12];
    if (threadIdx.x < 12) s_acc[threadIdx.x] = key_is_min(threadIdx.x) ? 0xFFFFFFFFu : 0u;
    __syncthreads();
    uint32_t a[12];
    acc_ident(a);
    const uint32_t b0 = blockIdx.x * kSpan;
    for (int r = 0; r < kIPT; r++) {
        const uint32_t i = b0 + r * kBlock + threadIdx.x;
        if (i >= n) break;
        Item it;
        for (int q = 0; q < 3; q++) {
            it.mn[q] = boxes[6ull * i + q];
            it.mx[q] = boxes[6ull * i + 3 + q];
            it.c[q] = 0.5f * (it.mx[q] + it.mn[q]);
        }
        it.idx = i;
        items[i] = it;
        seg[i] = 0;
        uint32_t v[12];
        item_keys(it, v);
        acc_merge(a, v);
    }
    wave_to_lds(s_acc, a);
    __syncthreads();
    if (threadIdx.x < 12) lds_to_global(acc, 0, s_acc, threadIdx.x);
}

// Per task: node box, default leaf record, bin layout (BVH.hpp:300-330).
__global__ void k_prep(uint32_t T, const Task* __restrict__ tasks, const Acc* __restrict__ acc, Dec* __restrict__ dec,
                       PtBvh2Node* __restrict__ nodes) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    const Task tk = tasks[t];
    const Acc a = acc[t];
    PtBvh2Node& nd = nodes[tk.node];
    for (int j = 0; j < 3; j++) {
        nd.mn[j] = kval(a.k[j]);
        nd.mx[j] = kval(a.k[3 + j]);
    }
    const uint32_t span = tk.last - tk.first;
    nd.left = 0;
    nd.right = tk.first;
    nd.count = span;
    nd.axis = 0;
    Dec d{};
    d.nbins = nbins_for(span);
    for (int ax = 0; ax < 3; ax++) {
        const float hi = kval(a.k[9 + ax]), lo = kval(a.k[6 + ax]);
        d.lo[ax] = lo;
        if (fabsf(hi - lo) <= 1.1920929e-7f) continue;  // numeric_limits<float>::epsilon()
        d.scale[ax] = (float)d.nbins / (hi - lo);
        d.valid |= 1u << ax;
    }
    d.split = 0;
    d.mid = d.lt = d.rt = kInv;
    dec[t] = d;
}

// Bin counts and bin boxes per (task, axis, bin) (BVH.hpp:320-327).
// bcnt [T][3][32]; bmin / bmax [T][3][32][3] ordered keys.
// Each wave bins a contiguous 1024-item range, 64 items per round.  A round
// inside one node bins into the wave's own LDS histogram (flushed to the
// global one when the node changes); a round that straddles nodes bins
// straight into the global histograms.
__global__ __launch_bounds__(kBlock) void k_bin(const Item* __restrict__ items, const uint32_t* __restrict__ seg,
                                                uint32_t n, const Dec* __restrict__ dec, uint32_t* bcnt,
                                                uint32_t* bmin, uint32_t* bmax) {
    constexpr int NWV = kBlock / 64;
    __shared__ uint32_t s_cnt[NWV][96], s_min[NWV][288], s_max[NWV][288];
    const int wv = threadIdx.x >> 6, lane = __lane_id();
    uint32_t* hc = s_cnt[wv];
    uint32_t* hmn = s_min[wv];
    uint32_t* hmx = s_max[wv];
    const uint32_t w0 = blockIdx.x * kSpan + (uint32_t)wv * (kSpan / NWV);
    uint32_t cur = kInv;  // node of this wave's LDS histogram (wave-uniform)
    // the histogram is private to the wave, but its lanes hand entries to
    // each other between phases (init -> atomics -> flush): an LDS fence at
    // wave scope + a wave barrier orders them under the memory model, not
    // just by gfx9's in-order LDS issue
    auto wave_sync = []() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    auto flush = [&]() {
        wave_sync();
        for (int j = lane; j < 96; j += 64) {
            if (!hc[j]) continue;
            const uint64_t g = (uint64_t)cur * 96 + j;
            atomicAdd(&bcnt[g], hc[j]);
            for (int a = 0; a < 3; a++) {
                atomicMin(&bmin[g * 3 + a], hmn[j * 3 + a]);
                atomicMax(&bmax[g * 3 + a], hmx[j * 3 + a]);
            }
        }
        wave_sync();
    };
    for (int r = 0; r < (int)(kSpan / NWV / 64); r++) {
        const uint32_t c0 = w0 + r * 64;
        if (c0 >= n) break;
        const uint32_t ta = seg[c0], tb = seg[min(n, c0 + 64) - 1];
        const bool uniform = ta != kInv && ta == tb;
        if (uniform && ta != cur) {
            if (cur != kInv) flush();
            for (int j = lane; j < 288; j += 64) {
                hmn[j] = 0xFFFFFFFFu;
                hmx[j] = 0;
                if (j < 96) hc[j] = 0;
            }
            wave_sync();
            cur = ta;
        }
        const uint32_t i = c0 + lane;
        const uint32_t t = i < n ? seg[i] : kInv;
        if (t == kInv) continue;
        const Dec d = dec[t];
        const Item it = items[i];
        uint32_t v[6];
        for (int a = 0; a < 3; a++) {
            v[a] = fkey(it.mn[a]);
            v[3 + a] = fkey(it.mx[a]);
        }
        for (int ax = 0; ax < 3; ax++) {
            if (!((d.valid >> ax) & 1u)) continue;
            const int b = min((int)d.nbins - 1, (int)((it.c[ax] - d.lo[ax]) * d.scale[ax]));
            const uint32_t slot = ax * 32 + b;
            if (uniform) {
                atomicAdd(&hc[slot], 1u);
                for (int a = 0; a < 3; a++) {
                    atomicMin(&hmn[slot * 3 + a], v[a]);
                    atomicMax(&hmx[slot * 3 + a], v[3 + a]);
                }
            } else {
                const uint64_t g = (uint64_t)t * 96 + slot;
                atomicAdd(&bcnt[g], 1u);
                for (int a = 0; a < 3; a++) {
                    atomicMin(&bmin[g * 3 + a], v[a]);
                    atomicMax(&bmax[g * 3 + a], v[3 + a]);
                }
            }
        }
    }
    if (cur != kInv) flush();
}

// The SAH sweep of one node (BVH.hpp:329-360), one lane per task.
__global__ void k_sah(uint32_t T, const Task* __restrict__ tasks, const Acc* __restrict__ acc, Dec* __restrict__ dec,
                      const uint32_t* __restrict__ bcnt, const uint32_t* __restrict__ bmin,
                      const uint32_t* __restrict__ bmax) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    const Task tk = tasks[t];
    const uint32_t span = tk.last - tk.first;
    Dec d = dec[t];
    const float inf = __builtin_inff();
    uint32_t bestAxis = 0;
    float bestPos = 0, bestCost = inf;
    const uint32_t nb = d.nbins;
    for (int ax = 0; ax < 3; ax++) {
        if (!((d.valid >> ax) & 1u)) continue;
        const float lo = d.lo[ax], hi = kval(acc[t].k[9 + ax]);
        float rightArea[32];
        float rmn[3] = {inf, inf, inf}, rmx[3] = {-inf, -inf, -inf};
        const uint64_t g0 = (uint64_t)t * 96 + ax * 32;
        for (uint32_t b = nb - 1; b >= 1; b--) {
            if (bcnt[g0 + b]) {
                float omn[3], omx[3];
                for (int a = 0; a < 3; a++) {
                    omn[a] = kval(bmin[(g0 + b) * 3 + a]);
                    omx[a] = kval(bmax[(g0 + b) * 3 + a]);
                }
                grow(rmn, rmx, omn, omx);
            }
            rightArea[b - 1] = area(rmn, rmx);
        }
        const float scale = (hi - lo) / (float)nb;
        float lmn[3] = {inf, inf, inf}, lmx[3] = {-inf, -inf, -inf};
        uint32_t lsum = 0;
        for (uint32_t b = 0; b < nb - 1; b++) {
            const uint32_t c = bcnt[g0 + b];
            lsum += c;
            if (c) {
                float omn[3], omx[3];
                for (int a = 0; a < 3; a++) {
                    omn[a] = kval(bmin[(g0 + b) * 3 + a]);
                    omx[a] = kval(bmax[(g0 + b) * 3 + a]);
                }
                grow(lmn, lmx, omn, omx);
            }
            const float cost = __builtin_fmaf((float)lsum, area(lmn, lmx), (float)(span - lsum) * rightArea[b]);
            if (cost < bestCost) {
                bestAxis = ax;
                bestPos = __builtin_fmaf((float)(b + 1), scale, lo);
                bestCost = cost;
            }
        }
    }
    float pmn[3], pmx[3];
    for (int a = 0; a < 3; a++) {
        pmn[a] = kval(acc[t].k[a]);
        pmx[a] = kval(acc[t].k[3 + a]);
    }
    const float parentCost = area(pmn, pmx) * (float)span;
    if (bestCost >= parentCost) return;  // leaf (k_prep's record stands)
    d.split = 1;
    d.axis = bestAxis;
    d.pos = bestPos;
    dec[t] = d;
}

// std::partition's predicate (BVH.hpp:362-365) and the per-task true count.
__global__ void k_flag(const Item* __restrict__ items, const uint32_t* __restrict__ seg, uint32_t n,
                       const Dec* __restrict__ dec, uint8_t* __restrict__ pred, Acc* acc) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t t = i < n ? seg[i] : kInv;
    bool act = false;
    uint32_t p = 0;
    if (t != kInv) {
        const Dec d = dec[t];
        if (d.split) {
            act = true;
            p = items[i].c[d.axis] <= d.pos ? 1u : 0u;
            pred[i] = (uint8_t)p;
        }
    }
    wave_count(acc, t, act, p);
}

// Split or leaf (BVH.hpp:367-385); children wider than kSmall become next-level
// tasks, the rest one-lane subtrees.
__global__ void k_mid(uint32_t T, const Task* __restrict__ tasks, const Acc* __restrict__ acc, Dec* __restrict__ dec,
                      PtBvh2Node* __restrict__ nodes, Ctr* ctr, Task* __restrict__ next, Acc* __restrict__ next_acc,
                      Task* __restrict__ small) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    Dec d = dec[t];
    if (!d.split) return;
    const Task tk = tasks[t];
    const uint32_t mid = tk.first + acc[t].ntrue;
    if (mid == tk.first || mid == tk.last) {
        dec[t].split = 0;
        return;
    }
    const uint32_t l = atomicAdd(&ctr->nodes, 2u);
    PtBvh2Node& nd = nodes[tk.node];
    nd.left = l;
    nd.right = l + 1;
    nd.count = 0;
    nd.axis = d.axis;
    const uint32_t cf[2] = {tk.first, mid}, cl[2] = {mid, tk.last};
    uint32_t ct[2];
    for (int s = 0; s < 2; s++) {
        const Task c{cf[s], cl[s], l + s, 0};
        if (cl[s] - cf[s] > kSmall) {
            ct[s] = atomicAdd(&ctr->next_tasks, 1u);
            next[ct[s]] = c;
            Acc e;
            acc_empty(e);
            next_acc[ct[s]] = e;
        } else {
            small[atomicAdd(&ctr->n_small, 1u)] = c;
            ct[s] = kInv;
        }
    }
    d.mid = mid;
    d.lt = ct[0];
    d.rt = ct[1];
    dec[t] = d;
}

// Misplaced elements: low word "false left of mid", high word "true right of mid".
__global__ void k_mark(const uint32_t* __restrict__ seg, uint32_t n, const Dec* __restrict__ dec,
                       const uint8_t* __restrict__ pred, unsigned long long* __restrict__ vals) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    unsigned long long v = 0;
    const uint32_t t = i < n ? seg[i] : kInv;
    if (t != kInv) {
        const Dec d = dec[t];
        if (d.split) {
            if (i < d.mid && !pred[i]) v = 1ull;
            if (i >= d.mid && pred[i]) v = 1ull << 32;
        }
    }
    vals[i] = v;
}

// The k-th misplaced true from the right of its task -> pos[first + k].
__global__ void k_rank(const uint32_t* __restrict__ seg, uint32_t n, const Task* __restrict__ tasks,
                       const Dec* __restrict__ dec, const unsigned long long* __restrict__ vals,
                       const unsigned long long* __restrict__ ex, uint32_t* __restrict__ pos) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !(vals[i] >> 32)) return;
    const uint32_t t = seg[i];
    const Task tk = tasks[t];
    const uint32_t r = (uint32_t)(ex[tk.last] >> 32) - (uint32_t)(ex[i] >> 32) - 1u;
    pos[tk.first + r] = i;
}

// The k-th misplaced false from the left swaps with it (std::iter_swap).
__global__ void k_swap(const uint32_t* __restrict__ seg, uint32_t n, const Task* __restrict__ tasks,
                       const unsigned long long* __restrict__ vals, const unsigned long long* __restrict__ ex,
                       const uint32_t* __restrict__ pos, Item* __restrict__ items) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !(vals[i] & 0xFFFFFFFFull)) return;
    const uint32_t t = seg[i];
    const Task tk = tasks[t];
    const uint32_t r = (uint32_t)ex[i] - (uint32_t)ex[tk.first];
    const uint32_t j = pos[tk.first + r];
    const Item a = items[i], b = items[j];
    items[i] = b;
    items[j] = a;
}

// Items follow their node into the child task; child bounds accumulate.
__global__ __launch_bounds__(kBlock) void k_advance(const Item* __restrict__ items, uint32_t* __restrict__ seg,
                                                    uint32_t n, const Dec* __restrict__ dec, Acc* next_acc) {
    __shared__ uint32_t s_acc[2][12];
    const uint32_t b0 = blockIdx.x * kSpan;
    const uint32_t last = min(n, b0 + kSpan) - 1;
    const uint32_t t0 = seg[b0], tl = seg[last];
    if (t0 != kInv && t0 == tl) {  // one parent: two children at most, kept in registers
        const Dec d = dec[t0];
        if (threadIdx.x < 24) s_acc[threadIdx.x / 12][threadIdx.x % 12] = key_is_min(threadIdx.x % 12) ? 0xFFFFFFFFu : 0u;
        __syncthreads();
        uint32_t a0[12], a1[12];
        acc_ident(a0);
        acc_ident(a1);
        for (int r = 0; r < kIPT; r++) {
            const uint32_t i = b0 + r * kBlock + threadIdx.x;
            if (i > last) break;
            const uint32_t child = d.split ? (i < d.mid ? d.lt : d.rt) : kInv;
            seg[i] = child;
            if (child == kInv) continue;
            uint32_t v[12];
            item_keys(items[i], v);
            if (i < d.mid)
                acc_merge(a0, v);
            else
                acc_merge(a1, v);
        }
        wave_to_lds(s_acc[0], a0);
        wave_to_lds(s_acc[1], a1);
        __syncthreads();
        if (threadIdx.x < 24) {
            const int side = threadIdx.x / 12;
            const uint32_t key = side ? d.rt : d.lt;
            if (d.split && key != kInv) lds_to_global(next_acc, key, s_acc[side], threadIdx.x % 12);
        }
        return;
    }
    for (int r = 0; r < kIPT; r++) {
        const uint32_t i = b0 + r * kBlock + threadIdx.x;
        const uint32_t t = i < n ? seg[i] : kInv;
        uint32_t child = kInv;
        uint32_t v[12] = {};
        if (t != kInv) {
            const Dec d = dec[t];
            if (d.split) child = i < d.mid ? d.lt : d.rt;
            seg[i] = child;
            if (child != kInv) item_keys(items[i], v);
        }
        wave_acc(next_acc, child, child != kInv, v);
    }
}

// A subtree of at most kSmall primitives, sequentially in one lane: build2 of
// pt_bvh.cpp (BuildBaseThreaded, BVH.hpp:290-390) with an explicit stack.
__global__ void k_small(uint32_t S, const Task* __restrict__ small, Item* __restrict__ items,
                        PtBvh2Node* __restrict__ nodes, Ctr* ctr) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    const float inf = __builtin_inff();
    uint32_t sf[kSmall], sl[kSmall], sn[kSmall];
    int sp = 0;
    sf[0] = small[s].first;
    sl[0] = small[s].last;
    sn[0] = small[s].node;
    sp = 1;
    while (sp > 0) {
        sp--;
        const uint32_t first = sf[sp], last = sl[sp], ni = sn[sp];
        const uint32_t span = last - first;
        float bmn[3] = {inf, inf, inf}, bmx[3] = {-inf, -inf, -inf};
        float cmax[3] = {-3.40282347e38f, -3.40282347e38f, -3.40282347e38f};
        float cmin[3] = {3.40282347e38f, 3.40282347e38f, 3.40282347e38f};
        for (uint32_t i = first; i < last; i++) {
            const Item& it = items[i];
            grow(bmn, bmx, it.mn, it.mx);
            for (int a = 0; a < 3; a++) {
                cmax[a] = cmax[a] < it.c[a] ? it.c[a] : cmax[a];
                cmin[a] = it.c[a] < cmin[a] ? it.c[a] : cmin[a];
            }
        }
        PtBvh2Node nd;
        for (int a = 0; a < 3; a++) {
            nd.mn[a] = bmn[a];
            nd.mx[a] = bmx[a];
        }
        nd.left = 0;
        nd.right = first;
        nd.count = span;
        nd.axis = 0;
        if (span > kLeaf) {
            uint32_t bestAxis = 0;
            float bestPos = 0, bestCost = inf;
            const uint32_t nb = nbins_for(span);
            for (int ax = 0; ax < 3; ax++) {
                const float hi = cmax[ax], lo = cmin[ax];
                if (fabsf(hi - lo) <= 1.1920929e-7f) continue;
                uint32_t cnt[16];
                float qmn[16][3], qmx[16][3], rightArea[16];
                for (uint32_t b = 0; b < nb; b++) {
                    cnt[b] = 0;
                    for (int a = 0; a < 3; a++) {
                        qmn[b][a] = inf;
                        qmx[b][a] = -inf;
                    }
                }
                float scale = (float)nb / (hi - lo);
                for (uint32_t i = first; i < last; i++) {
                    const Item& it = items[i];
                    const int b = min((int)nb - 1, (int)((it.c[ax] - lo) * scale));
                    cnt[b]++;
                    grow(qmn[b], qmx[b], it.mn, it.mx);
                }
                float rmn[3] = {inf, inf, inf}, rmx[3] = {-inf, -inf, -inf};
                for (uint32_t b = nb - 1; b >= 1; b--) {
                    grow(rmn, rmx, qmn[b], qmx[b]);
                    rightArea[b - 1] = area(rmn, rmx);
                }
                scale = (hi - lo) / (float)nb;
                float lmn[3] = {inf, inf, inf}, lmx[3] = {-inf, -inf, -inf};
                uint32_t lsum = 0;
                for (uint32_t b = 0; b < nb - 1; b++) {
                    lsum += cnt[b];
                    grow(lmn, lmx, qmn[b], qmx[b]);
                    const float cost =
                        __builtin_fmaf((float)lsum, area(lmn, lmx), (float)(span - lsum) * rightArea[b]);
                    if (cost < bestCost) {
                        bestAxis = ax;
                        bestPos = __builtin_fmaf((float)(b + 1), scale, lo);
                        bestCost = cost;
                    }
                }
            }
            const float parentCost = area(bmn, bmx) * (float)span;
            if (bestCost < parentCost) {
                // libstdc++ std::partition, bidirectional form
                uint32_t f = first, l = last, mid;
                for (;;) {
                    while (f != l && items[f].c[bestAxis] <= bestPos) f++;
                    if (f == l) break;
                    l--;
                    while (f != l && !(items[l].c[bestAxis] <= bestPos)) l--;
                    if (f == l) break;
                    const Item a = items[f];
                    items[f] = items[l];
                    items[l] = a;
                    f++;
                }
                mid = f;
                if (mid != first && mid != last) {
                    const uint32_t c0 = atomicAdd(&ctr->nodes, 2u);
                    nd.left = c0;
                    nd.right = c0 + 1;
                    nd.count = 0;
                    nd.axis = bestAxis;
                    sf[sp] = mid, sl[sp] = last, sn[sp] = c0 + 1, sp++;
                    sf[sp] = first, sl[sp] = mid, sn[sp] = c0, sp++;
                }
            }
        }
        nodes[ni] = nd;
    }
}

__global__ void k_order(const Item* __restrict__ items, uint32_t n, uint32_t* __restrict__ order) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) order[i] = items[i].idx;
}

// ---------------------------------------------------------------------------
// BVH4 collapse on the device (BVH4::buildBVH4, BVH.hpp:788-1017; pt_bvh.cpp
// Collapser).  A cluster is made for every internal binary node the recursion
// visits; its up-to-four children are picked by the five topologies below.
// Clusters are numbered in pre-order with children in slot order, so:
//   A (top-down, per level)  build the cluster tree: records with the binary
//                            node, child nodes per slot, active mask, perm;
//   B (bottom-up)            subtree sizes;
//   C (top-down)             pre-order index = parent's + 1 + sizes of the
//                            earlier internal siblings; write the 128-byte
//                            clusters.
struct CRec {
    uint32_t node, kid[4], kid_rec[4];
    uint32_t active, perm, size, idx, pad;
};  // 56 B

__device__ __forceinline__ bool bleaf(const PtBvh2Node& n) { return (uint16_t)n.count != 0; }

__global__ void k_cl_topo(uint32_t r0, uint32_t r1, CRec* __restrict__ rec, const PtBvh2Node* __restrict__ nodes,
                          uint32_t* rec_count) {
    const uint32_t r = r0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= r1) return;
    CRec c = rec[r];
    const PtBvh2Node& n = nodes[c.node];
    const PtBvh2Node &L = nodes[n.left], &R = nodes[n.right];
    uint32_t k[4] = {kInv, kInv, kInv, kInv};
    uint32_t active, perm;
    if (bleaf(L) && bleaf(R)) {
        k[0] = n.left, k[2] = n.right;
        active = 0b0101;
        perm = n.axis;
    } else if (bleaf(L)) {
        const PtBvh2Node &RL = nodes[R.left], &RR = nodes[R.right];
        if (bleaf(RL) && bleaf(RR)) {
            k[0] = n.left, k[2] = R.left, k[3] = R.right;
            active = 0b1101;
            perm = n.axis + R.axis * 9;
        } else if (bleaf(RL)) {
            k[0] = n.left, k[1] = R.left, k[2] = RR.left, k[3] = RR.right;
            active = 0b1111;
            perm = n.axis + R.axis * 3 + RR.axis * 9 + 1 * 27;
        } else {
            k[0] = n.left, k[1] = RL.left, k[2] = RL.right, k[3] = R.right;
            active = 0b1111;
            perm = n.axis + R.axis * 3 + RL.axis * 9 + 2 * 27;
        }
    } else if (bleaf(R)) {
        const PtBvh2Node &LL = nodes[L.left], &LR = nodes[L.right];
        if (bleaf(LL) && bleaf(LR)) {
            k[0] = L.left, k[1] = L.right, k[2] = n.right;
            active = 0b0111;
            perm = n.axis + L.axis * 3;
        } else if (bleaf(LL)) {
            k[0] = L.left, k[1] = LR.left, k[2] = LR.right, k[3] = n.right;
            active = 0b1111;
            perm = n.axis + L.axis * 3 + LR.axis * 9 + 4 * 27;
        } else {
            k[0] = LL.left, k[1] = LL.right, k[2] = L.right, k[3] = n.right;
            active = 0b1111;
            perm = n.axis + L.axis * 3 + LL.axis * 9 + 3 * 27;
        }
    } else {
        k[0] = L.left, k[1] = L.right, k[2] = R.left, k[3] = R.right;
        active = 0b1111;
        perm = n.axis + L.axis * 3 + R.axis * 9;
    }
    for (int s = 0; s < 4; s++) {
        c.kid[s] = k[s];
        c.kid_rec[s] = kInv;
        if (k[s] != kInv && !bleaf(nodes[k[s]])) {
            const uint32_t q = atomicAdd(rec_count, 1u);
            CRec e{};
            e.node = k[s];
            e.size = 1;
            rec[q] = e;
            c.kid_rec[s] = q;
        }
    }
    c.active = active;
    c.perm = perm;
    rec[r] = c;
}

__global__ void k_cl_size(uint32_t r0, uint32_t r1, CRec* rec) {
    const uint32_t r = r0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= r1) return;
    uint32_t s = 1;
    for (int q = 0; q < 4; q++)
        if (rec[r].kid_rec[q] != kInv) s += rec[rec[r].kid_rec[q]].size;
    rec[r].size = s;
}

__global__ void k_cl_emit(uint32_t r0, uint32_t r1, CRec* __restrict__ rec, const PtBvh2Node* __restrict__ nodes,
                          pt_ref_bvh4_cluster* __restrict__ out) {
    const uint32_t r = r0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= r1) return;
    const CRec c = rec[r];
    uint32_t next = c.idx + 1;
    pt_ref_bvh4_cluster o;
    uint32_t* w = reinterpret_cast<uint32_t*>(&o);
    for (int j = 0; j < 32; j++) w[j] = 0;
    for (int s = 0; s < 4; s++) {
        if (c.kid[s] == kInv) continue;
        const PtBvh2Node& kn = nodes[c.kid[s]];
        o.xmin[s] = kn.mn[0], o.ymin[s] = kn.mn[1], o.zmin[s] = kn.mn[2];
        o.xmax[s] = kn.mx[0], o.ymax[s] = kn.mx[1], o.zmax[s] = kn.mx[2];
        pt_ref_bvh4_node d{};
        d.count = (uint8_t)(uint16_t)kn.count;
        if (c.kid_rec[s] == kInv) {
            d.cluster_idx = kn.right;
        } else {
            CRec& kc = rec[c.kid_rec[s]];
            kc.idx = next;
            d.active = (uint8_t)kc.active;
            d.perm = (uint8_t)kc.perm;
            d.cluster_idx = next;
            next += kc.size;
        }
        o.children[s] = d;
    }
    out[c.idx] = o;
}

inline uint32_t blocks(uint64_t n, int b = kBlock) { return (uint32_t)((n + b - 1) / b); }

}  // namespace bvhg

#pragma clang fp contract(fast)

extern "C" pt_status pt_bvh4_build_device(pt_ctx* c, const float* boxes, uint32_t n, pt_ref_bvh4_cluster* clusters,
                                          uint32_t* n_clusters, pt_ref_bvh4_node* root, uint32_t* prim_order,
                                          float* bbox, pt_bvh_build_stats* stats) {
    using namespace bvhg;
    if (!c || !root || !n_clusters || (n > 0 && (!boxes || !clusters || !prim_order))) return PT_ERR_ARG;
    if (n > 0x7FFFFFFFu) return fail(c, PT_ERR_ARG, "device BVH build: too many primitives (%u)", n);
    const auto t_start = std::chrono::steady_clock::now();
    pt_bvh_build_stats st{};
    if (n == 0) {
        pt_status s = pt_bvh4_build(boxes, n, clusters, n_clusters, root, prim_order, bbox);
        if (stats) *stats = st;
        return s;
    }
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t sm = c->stream;
    const uint64_t Tmax = n / (kSmall + 1) + 1;
    const uint64_t NN = 2ull * n;  // binary nodes <= 2n - 1
    std::vector<void*> bufs;
    auto dalloc = [&](void** p, uint64_t bytes) -> bool {
        if (hipMalloc(p, std::max<uint64_t>(bytes, 16)) != hipSuccess) return false;
        bufs.push_back(*p);
        return true;
    };
    auto release = [&]() {
        for (void* p : bufs) hipFree(p);
        bufs.clear();
    };
    float* d_boxes;
    Item* items;
    uint32_t *seg, *pos, *bcnt, *bmin, *bmax, *order;
    uint8_t* pred;
    unsigned long long *vals, *ex;
    PtBvh2Node* nodes;
    Task *tasks[2], *small;
    Acc* acc[2];
    Dec* dec;
    Ctr* ctr;
    CRec* crec;
    uint32_t* rec_count;
    pt_ref_bvh4_cluster* dclusters;
    size_t scan_bytes = 0;
    if (rocprim::exclusive_scan(nullptr, scan_bytes, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                0ull, (size_t)n + 1, rocprim::plus<unsigned long long>(), sm) != hipSuccess)
        return fail(c, PT_ERR_HIP, "device BVH build: scan size query failed");
    void* scan_tmp;
    bool ok = dalloc((void**)&d_boxes, 24ull * n) && dalloc((void**)&items, sizeof(Item) * (uint64_t)n) &&
              dalloc((void**)&seg, 4ull * n) && dalloc((void**)&pos, 4ull * n) && dalloc((void**)&order, 4ull * n) &&
              dalloc((void**)&pred, (uint64_t)n) && dalloc((void**)&vals, 8ull * (n + 1)) &&
              dalloc((void**)&ex, 8ull * (n + 1)) && dalloc((void**)&nodes, sizeof(PtBvh2Node) * NN) &&
              dalloc((void**)&tasks[0], sizeof(Task) * Tmax) && dalloc((void**)&tasks[1], sizeof(Task) * Tmax) &&
              dalloc((void**)&acc[0], sizeof(Acc) * Tmax) && dalloc((void**)&acc[1], sizeof(Acc) * Tmax) &&
              dalloc((void**)&dec, sizeof(Dec) * Tmax) && dalloc((void**)&small, sizeof(Task) * (uint64_t)n) &&
              dalloc((void**)&bcnt, 4ull * 96 * Tmax) && dalloc((void**)&bmin, 4ull * 288 * Tmax) &&
              dalloc((void**)&bmax, 4ull * 288 * Tmax) && dalloc((void**)&ctr, sizeof(Ctr)) &&
              dalloc(&scan_tmp, scan_bytes) && dalloc((void**)&crec, sizeof(CRec) * (uint64_t)n) &&
              dalloc((void**)&rec_count, 4) && dalloc((void**)&dclusters, sizeof(pt_ref_bvh4_cluster) * (uint64_t)n);
    if (!ok) {
        release();
        return fail(c, PT_ERR_OOM, "device BVH build: allocation failed (n = %u)", n);
    }
#define BVHCHK(x)                                                                                             \
    do {                                                                                                      \
        hipError_t e_ = (x);                                                                                  \
        if (e_ != hipSuccess) {                                                                               \
            release();                                                                                        \
            return fail(c, PT_ERR_HIP, "device BVH build: %s: %s (line %d)", #x, hipGetErrorString(e_), __LINE__); \
        }                                                                                                     \
    } while (0)
    hipEvent_t e0, e1;
    BVHCHK(hipEventCreate(&e0));
    BVHCHK(hipEventCreate(&e1));
    BVHCHK(hipEventRecord(e0, sm));
    BVHCHK(hipMemcpyAsync(d_boxes, boxes, 24ull * n, hipMemcpyHostToDevice, sm));
    // root task
    {
        Task root_task{0, n, 0, 0};
        BVHCHK(hipMemcpyAsync(tasks[0], &root_task, sizeof(Task), hipMemcpyHostToDevice, sm));
        Acc e;
        for (int j = 0; j < 3; j++) {  // acc_empty on the host (same keys)
            auto key = [](float f) {
                uint32_t u;
                std::memcpy(&u, &f, 4);
                return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
            };
            e.k[j] = key(std::numeric_limits<float>::infinity());
            e.k[3 + j] = key(-std::numeric_limits<float>::infinity());
            e.k[6 + j] = key(std::numeric_limits<float>::max());
            e.k[9 + j] = key(-std::numeric_limits<float>::max());
        }
        e.ntrue = 0;
        e.pad[0] = e.pad[1] = e.pad[2] = 0;
        BVHCHK(hipMemcpyAsync(acc[0], &e, sizeof(Acc), hipMemcpyHostToDevice, sm));
        Ctr c0{0, 0, 1, 0};
        if (n <= kSmall) {
            c0.n_small = 1;
            BVHCHK(hipMemcpyAsync(small, &root_task, sizeof(Task), hipMemcpyHostToDevice, sm));
        }
        BVHCHK(hipMemcpyAsync(ctr, &c0, sizeof(Ctr), hipMemcpyHostToDevice, sm));
    }
    hipLaunchKernelGGL(k_init, dim3(blocks(n, kSpan)), dim3(kBlock), 0, sm, d_boxes, n, items, seg, acc[0]);
    uint32_t T = n > kSmall ? 1 : 0;
    int cur = 0;
    Ctr h{};
    while (T > 0) {
        st.levels++;
        if (st.levels > 100000) {
            release();
            return fail(c, PT_ERR_STATE, "device BVH build: no progress");
        }
        Task* tk = tasks[cur];
        Acc* ac = acc[cur];
        BVHCHK(hipMemsetAsync(&ctr->next_tasks, 0, 4, sm));
        BVHCHK(hipMemsetAsync(bcnt, 0, 4ull * 96 * T, sm));
        BVHCHK(hipMemsetAsync(bmin, 0xFF, 4ull * 288 * T, sm));
        BVHCHK(hipMemsetAsync(bmax, 0x00, 4ull * 288 * T, sm));
        hipLaunchKernelGGL(k_prep, dim3(blocks(T, 64)), dim3(64), 0, sm, T, tk, ac, dec, nodes);
        hipLaunchKernelGGL(k_bin, dim3(blocks(n, kSpan)), dim3(kBlock), 0, sm, items, seg, n, dec, bcnt, bmin, bmax);
        hipLaunchKernelGGL(k_sah, dim3(blocks(T, 64)), dim3(64), 0, sm, T, tk, ac, dec, bcnt, bmin, bmax);
        hipLaunchKernelGGL(k_flag, dim3(blocks(n)), dim3(kBlock), 0, sm, items, seg, n, dec, pred, ac);
        hipLaunchKernelGGL(k_mid, dim3(blocks(T, 64)), dim3(64), 0, sm, T, tk, ac, dec, nodes, ctr, tasks[cur ^ 1],
                           acc[cur ^ 1], small);
        hipLaunchKernelGGL(k_mark, dim3(blocks((uint64_t)n + 1)), dim3(kBlock), 0, sm, seg, n, dec, pred, vals);
        BVHCHK(rocprim::exclusive_scan(scan_tmp, scan_bytes, vals, ex, 0ull, (size_t)n + 1,
                                       rocprim::plus<unsigned long long>(), sm));
        hipLaunchKernelGGL(k_rank, dim3(blocks(n)), dim3(kBlock), 0, sm, seg, n, tk, dec, vals, ex, pos);
        hipLaunchKernelGGL(k_swap, dim3(blocks(n)), dim3(kBlock), 0, sm, seg, n, tk, vals, ex, pos, items);
        hipLaunchKernelGGL(k_advance, dim3(blocks(n, kSpan)), dim3(kBlock), 0, sm, items, seg, n, dec, acc[cur ^ 1]);
        BVHCHK(hipGetLastError());
        BVHCHK(hipMemcpyAsync(&h, ctr, sizeof(Ctr), hipMemcpyDeviceToHost, sm));
        BVHCHK(hipStreamSynchronize(sm));
        T = h.next_tasks;
        if (T > Tmax) {
            release();
            return fail(c, PT_ERR_STATE, "device BVH build: task overflow (%u > %llu)", T, (unsigned long long)Tmax);
        }
        cur ^= 1;
    }
    BVHCHK(hipMemcpyAsync(&h, ctr, sizeof(Ctr), hipMemcpyDeviceToHost, sm));
    BVHCHK(hipStreamSynchronize(sm));
    if (h.n_small) hipLaunchKernelGGL(k_small, dim3(blocks(h.n_small, 64)), dim3(64), 0, sm, h.n_small, small, items,
                                      nodes, ctr);
    hipLaunchKernelGGL(k_order, dim3(blocks(n)), dim3(kBlock), 0, sm, items, n, order);
    BVHCHK(hipGetLastError());
    BVHCHK(hipMemcpyAsync(&h, ctr, sizeof(Ctr), hipMemcpyDeviceToHost, sm));
    BVHCHK(hipStreamSynchronize(sm));
    if (h.nodes > NN) {
        release();
        return fail(c, PT_ERR_STATE, "device BVH build: node overflow");
    }
    PtBvh2Node root_node;
    BVHCHK(hipMemcpyAsync(&root_node, nodes, sizeof(PtBvh2Node), hipMemcpyDeviceToHost, sm));
    BVHCHK(hipStreamSynchronize(sm));
    hipEvent_t ec0, ec1;
    BVHCHK(hipEventCreate(&ec0));
    BVHCHK(hipEventCreate(&ec1));
    BVHCHK(hipEventRecord(ec0, sm));
    uint32_t n_cl = 0;
    *root = pt_ref_bvh4_node{};
    if ((uint16_t)root_node.count != 0) {  // the root is a leaf: no clusters
        root->count = (uint8_t)(uint16_t)root_node.count;
        root->cluster_idx = root_node.right;
    } else {
        CRec r0{};
        r0.node = 0;
        r0.size = 1;
        uint32_t one = 1;
        BVHCHK(hipMemcpyAsync(crec, &r0, sizeof(CRec), hipMemcpyHostToDevice, sm));
        BVHCHK(hipMemcpyAsync(rec_count, &one, 4, hipMemcpyHostToDevice, sm));
        std::vector<uint32_t> lv{0, 1};  // record ranges per cluster-tree level
        while (lv.back() > lv[lv.size() - 2]) {
            const uint32_t a = lv[lv.size() - 2], b = lv.back();
            hipLaunchKernelGGL(k_cl_topo, dim3(blocks(b - a)), dim3(kBlock), 0, sm, a, b, crec, nodes, rec_count);
            uint32_t cnt = 0;
            BVHCHK(hipMemcpyAsync(&cnt, rec_count, 4, hipMemcpyDeviceToHost, sm));
            BVHCHK(hipStreamSynchronize(sm));
            if (cnt > n) {
                release();
                return fail(c, PT_ERR_STATE, "device BVH build: cluster overflow");
            }
            lv.push_back(cnt);
        }
        n_cl = lv.back();
        for (size_t l = lv.size() - 1; l-- > 0;)
            if (lv[l + 1] > lv[l])
                hipLaunchKernelGGL(k_cl_size, dim3(blocks(lv[l + 1] - lv[l])), dim3(kBlock), 0, sm, lv[l], lv[l + 1],
                                   crec);
        for (size_t l = 0; l + 1 < lv.size(); l++)
            if (lv[l + 1] > lv[l])
                hipLaunchKernelGGL(k_cl_emit, dim3(blocks(lv[l + 1] - lv[l])), dim3(kBlock), 0, sm, lv[l], lv[l + 1],
                                   crec, nodes, dclusters);
        BVHCHK(hipGetLastError());
        root->active = 0;
        CRec rr;
        BVHCHK(hipMemcpyAsync(&rr, crec, sizeof(CRec), hipMemcpyDeviceToHost, sm));
        BVHCHK(hipStreamSynchronize(sm));
        root->active = (uint8_t)rr.active;
        root->perm = (uint8_t)rr.perm;
        root->cluster_idx = 0;
        BVHCHK(hipMemcpyAsync(clusters, dclusters, sizeof(pt_ref_bvh4_cluster) * n_cl, hipMemcpyDeviceToHost, sm));
    }
    BVHCHK(hipEventRecord(ec1, sm));
    BVHCHK(hipMemcpyAsync(prim_order, order, 4ull * n, hipMemcpyDeviceToHost, sm));
    BVHCHK(hipEventRecord(e1, sm));
    BVHCHK(hipStreamSynchronize(sm));
    float ms = 0, ms_c = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipEventElapsedTime(&ms_c, ec0, ec1);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    hipEventDestroy(ec0);
    hipEventDestroy(ec1);
    release();
#undef BVHCHK
    *n_clusters = n_cl;
    st.ms_device = ms;
    st.ms_collapse = ms_c;
    st.small_tasks = h.n_small;
    st.nodes = h.nodes;
    if (bbox) {
        for (int a = 0; a < 3; a++) {
            bbox[a] = root_node.mn[a];
            bbox[3 + a] = root_node.mx[a];
        }
    }
    const auto t_end = std::chrono::steady_clock::now();
    st.ms_total = std::chrono::duration<double, std::milli>(t_end - t_start).count();
    if (stats) *stats = st;
    return PT_OK;
}
