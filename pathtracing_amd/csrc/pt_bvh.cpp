// Host-side BVH4 builder of libpt_hip.so.
//
// Scene build stays on the host (BASELINE.json north_star); what the GPU reads
// is this builder's output, converted to the device layout in pt_scene.cpp.
// To keep traversal statistics and primitive order identical to the reference,
// the build restates, decision for decision:
//   * BVHBase::BuildBaseThreaded (BVH.hpp:290-390): binned SAH over centroids,
//     32/16/8 bins by span (312-313), no traversal constant (341-353), stop if
//     bestCost >= parent cost (356-360), std::partition on centroid <= bestPos
//     (362-365), leaf size 2 (95); spans > 256K recurse on two threads (374-380).
//   * BVH4::buildBVH4 (BVH.hpp:788-1017): BVH2 -> 128-byte 4-wide clusters with
//     the five collapse topologies and their perm codes, clusters numbered in
//     the same pre-order, u8 leaf counts (BVH.hpp:39, 793).
//   * BVH4::LUT / PermToIndexLUT (BVH.hpp:10-24, 562-718): octant child order.
// Float expressions are written in the reference's operand order so the
// compiler's FMA contraction makes the same choices (build flags: DESIGN.md).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <thread>
#include <vector>

#include "pt_api.h"

namespace {

struct Box {
    float mn[3] = {std::numeric_limits<float>::infinity(), std::numeric_limits<float>::infinity(),
                   std::numeric_limits<float>::infinity()};
    float mx[3] = {-std::numeric_limits<float>::infinity(), -std::numeric_limits<float>::infinity(),
                   -std::numeric_limits<float>::infinity()};
    void grow(const Box& o) {
        for (int a = 0; a < 3; a++) {
            mn[a] = std::min(mn[a], o.mn[a]);  // glm::min/max operand order (AABB.hpp:62-65)
            mx[a] = std::max(mx[a], o.mx[a]);
        }
    }
    float area() const {
        float ex = mx[0] - mn[0], ey = mx[1] - mn[1], ez = mx[2] - mn[2];
        return ex * ey + ey * ez + ez * ex;
    }
};

struct Item {
    uint32_t index;
    Box box;
    float c[3];
};

struct Node2 {
    Box box;
    uint32_t left = 0, right = 0;
    uint16_t count = 0, axis = 0;
    bool leaf() const { return count != 0; }
};

struct Bin {
    Box box;
    uint32_t n = 0;
};

constexpr uint32_t kLeafSize = 2;
constexpr uint32_t kThreadSpan = 256 * 1024;

uint32_t build2(uint32_t first, uint32_t last, std::vector<Item>& items, std::vector<Node2>& nodes,
                std::atomic<uint32_t>& next) {
    const uint32_t index = next.fetch_add(1, std::memory_order_relaxed);
    Node2& node = nodes[index];
    const uint32_t span = last - first;

    float cmax[3] = {-std::numeric_limits<float>::max(), -std::numeric_limits<float>::max(),
                     -std::numeric_limits<float>::max()};
    float cmin[3] = {std::numeric_limits<float>::max(), std::numeric_limits<float>::max(),
                     std::numeric_limits<float>::max()};
    for (uint32_t i = first; i < last; i++) {
        node.box.grow(items[i].box);
        for (int a = 0; a < 3; a++) {
            cmax[a] = std::max(cmax[a], items[i].c[a]);
            cmin[a] = std::min(cmin[a], items[i].c[a]);
        }
    }
    node.right = first;
    node.count = (uint16_t)span;
    if (span <= kLeafSize) return index;

    unsigned bestAxis = 0;
    float bestPos = 0;
    float bestCost = std::numeric_limits<float>::infinity();
    const uint32_t nbins = span >= 1024 ? 32 : span >= 64 ? 16 : 8;
    Bin bins[32];
    float rightArea[32];
    for (unsigned axis = 0; axis < 3; axis++) {
        const float hi = cmax[axis], lo = cmin[axis];
        if (std::abs(hi - lo) <= std::numeric_limits<float>::epsilon()) continue;
        for (uint32_t b = 0; b < nbins; b++) bins[b] = Bin{};
        float scale = nbins / (hi - lo);
        for (uint32_t i = first; i < last; i++) {
            int b = std::min<int>(nbins - 1, (items[i].c[axis] - lo) * scale);
            ++bins[b].n;
            bins[b].box.grow(items[i].box);
        }
        Box lbox, rbox;
        for (uint32_t b = nbins - 1; b >= 1; b--) {
            rbox.grow(bins[b].box);
            rightArea[b - 1] = rbox.area();
        }
        scale = (hi - lo) / nbins;
        uint32_t lsum = 0;
        for (uint32_t b = 0; b < nbins - 1; b++) {
            lsum += bins[b].n;
            lbox.grow(bins[b].box);
            float cost = lsum * lbox.area() + (span - lsum) * rightArea[b];
            if (cost < bestCost) {
                bestAxis = axis;
                bestPos = lo + (b + 1) * scale;
                bestCost = cost;
            }
        }
    }
    float parentCost = node.box.area() * span;
    if (bestCost >= parentCost) return index;

    const uint32_t mid = (uint32_t)(std::partition(items.begin() + first, items.begin() + last,
                                                   [&](const Item& it) { return it.c[bestAxis] <= bestPos; }) -
                                    items.begin());
    if (mid == first || mid == last) return index;

    uint32_t l = 0, r = 0;
    if (span > kThreadSpan) {
        std::thread tl([&]() { l = build2(first, mid, items, nodes, next); });
        std::thread tr([&]() { r = build2(mid, last, items, nodes, next); });
        tl.join();
        tr.join();
    } else {
        l = build2(first, mid, items, nodes, next);
        r = build2(mid, last, items, nodes, next);
    }
    Node2& n2 = nodes[index];
    n2.left = l;
    n2.right = r;
    n2.count = 0;
    n2.axis = (uint16_t)bestAxis;
    return index;
}

struct Collapser {
    const std::vector<Node2>& n2;
    pt_ref_bvh4_cluster* out;
    uint32_t used = 0;

    void set_box(pt_ref_bvh4_cluster& c, const Box& b, int slot) {
        c.xmin[slot] = b.mn[0];
        c.ymin[slot] = b.mn[1];
        c.zmin[slot] = b.mn[2];
        c.xmax[slot] = b.mx[0];
        c.ymax[slot] = b.mx[1];
        c.zmax[slot] = b.mx[2];
    }

    pt_ref_bvh4_node leaf(const Node2& n) {
        pt_ref_bvh4_node d{};
        d.count = (uint8_t)n.count;
        d.cluster_idx = n.right;
        return d;
    }

    // One BVH2 subtree rooted at `id` -> a child descriptor (BVH.hpp:788-1017).
    pt_ref_bvh4_node collapse(uint32_t id) {
        const Node2& n = n2[id];
        if (n.leaf()) return leaf(n);
        const uint32_t ci = used++;
        std::memset(&out[ci], 0, sizeof(pt_ref_bvh4_cluster));
        const Node2& L = n2[n.left];
        const Node2& R = n2[n.right];
        uint8_t active = 0;
        unsigned perm = 0;
        pt_ref_bvh4_node k[4] = {};
        if (L.leaf() && R.leaf()) {
            k[0] = collapse(n.left);
            k[2] = collapse(n.right);
            set_box(out[ci], L.box, 0);
            set_box(out[ci], R.box, 2);
            active = 0b0101;
            perm = n.axis;
        } else if (L.leaf()) {
            const Node2& RL = n2[R.left];
            const Node2& RR = n2[R.right];
            if (RL.leaf() && RR.leaf()) {
                k[0] = collapse(n.left);
                k[2] = collapse(R.left);
                k[3] = collapse(R.right);
                set_box(out[ci], L.box, 0);
                set_box(out[ci], RL.box, 2);
                set_box(out[ci], RR.box, 3);
                active = 0b1101;
                perm = n.axis + R.axis * 9;
            } else if (RL.leaf()) {
                k[0] = collapse(n.left);
                k[1] = collapse(R.left);
                k[2] = collapse(RR.left);
                k[3] = collapse(RR.right);
                set_box(out[ci], L.box, 0);
                set_box(out[ci], RL.box, 1);
                set_box(out[ci], n2[RR.left].box, 2);
                set_box(out[ci], n2[RR.right].box, 3);
                active = 0b1111;
                perm = n.axis + R.axis * 3 + RR.axis * 9 + 1 * 27;
            } else {
                k[0] = collapse(n.left);
                k[1] = collapse(RL.left);
                k[2] = collapse(RL.right);
                k[3] = collapse(R.right);
                set_box(out[ci], L.box, 0);
                set_box(out[ci], n2[RL.left].box, 1);
                set_box(out[ci], n2[RL.right].box, 2);
                set_box(out[ci], RR.box, 3);
                active = 0b1111;
                perm = n.axis + R.axis * 3 + RL.axis * 9 + 2 * 27;
            }
        } else if (R.leaf()) {
            const Node2& LL = n2[L.left];
            const Node2& LR = n2[L.right];
            if (LL.leaf() && LR.leaf()) {
                k[0] = collapse(L.left);
                k[1] = collapse(L.right);
                k[2] = collapse(n.right);
                set_box(out[ci], LL.box, 0);
                set_box(out[ci], LR.box, 1);
                set_box(out[ci], R.box, 2);
                active = 0b0111;
                perm = n.axis + L.axis * 3;
            } else if (LL.leaf()) {
                k[0] = collapse(L.left);
                k[1] = collapse(LR.left);
                k[2] = collapse(LR.right);
                k[3] = collapse(n.right);
                set_box(out[ci], LL.box, 0);
                set_box(out[ci], n2[LR.left].box, 1);
                set_box(out[ci], n2[LR.right].box, 2);
                set_box(out[ci], R.box, 3);
                active = 0b1111;
                perm = n.axis + L.axis * 3 + LR.axis * 9 + 4 * 27;
            } else {
                k[0] = collapse(LL.left);
                k[1] = collapse(LL.right);
                k[2] = collapse(L.right);
                k[3] = collapse(n.right);
                set_box(out[ci], n2[LL.left].box, 0);
                set_box(out[ci], n2[LL.right].box, 1);
                set_box(out[ci], LR.box, 2);
                set_box(out[ci], R.box, 3);
                active = 0b1111;
                perm = n.axis + L.axis * 3 + LL.axis * 9 + 3 * 27;
            }
        } else {
            k[0] = collapse(L.left);
            k[1] = collapse(L.right);
            k[2] = collapse(R.left);
            k[3] = collapse(R.right);
            set_box(out[ci], n2[L.left].box, 0);
            set_box(out[ci], n2[L.right].box, 1);
            set_box(out[ci], n2[R.left].box, 2);
            set_box(out[ci], n2[R.right].box, 3);
            active = 0b1111;
            perm = n.axis + L.axis * 3 + R.axis * 9;
        }
        for (int s = 0; s < 4; s++) out[ci].children[s] = k[s];
        pt_ref_bvh4_node d{};
        d.count = (uint8_t)n.count;
        d.active = active;
        d.perm = (uint8_t)perm;
        d.cluster_idx = ci;
        return d;
    }
};

constexpr uint8_t P4(int a, int b, int c, int d) { return (uint8_t)((a << 6) | (b << 4) | (c << 2) | d); }

bool is_perm(unsigned p) {
    unsigned seen = 0;
    for (int s = 0; s < 4; s++) seen |= 1u << ((p >> (2 * s)) & 3);
    return p < 256 && seen == 0xF;
}

// Child visiting order for ray octant `rs` and topology/axis code `code`
// (BVH.hpp:562-718): 2-bit slots, most significant = visited first.
uint8_t order_byte(unsigned rs, unsigned code) {
    const unsigned sg[3] = {rs & 1u, (rs >> 1) & 1u, (rs >> 2) & 1u};
    const unsigned topo = code / 27, rem = code % 27;
    const unsigned s0 = rem % 3, s1 = (rem / 3) % 3, s2 = rem / 9;
    unsigned p = 0;
    switch (topo) {
        case 0: {  // (0,1) | (2,3)
            unsigned l = sg[s1] ? 0b0100u : 0b0001u;
            unsigned r = sg[s2] ? 0b1110u : 0b1011u;
            p = sg[s0] ? (r << 4) + l : (l << 4) + r;
            break;
        }
        case 1: {  // 0 | (1 | (2,3))
            unsigned r = sg[s2] ? 0b1110u : 0b1011u;
            unsigned sub = sg[s1] ? (r << 2) | 0b01u : (0b01u << 4) | r;
            p = sg[s0] ? (sub << 2) : sub;
            break;
        }
        case 2: {  // 0 | ((1,2) | 3)
            unsigned l = sg[s2] ? 0b1001u : 0b0110u;
            unsigned sub = sg[s1] ? (0b11u << 4) | l : (l << 2) | 0b11u;
            p = sg[s0] ? (sub << 2) : sub;
            break;
        }
        case 3: {  // ((0,1) | 2) | 3
            unsigned l = sg[s2] ? 0b0100u : 0b0001u;
            unsigned sub = sg[s1] ? (0b10u << 4) | l : (l << 2) | 0b10u;
            p = sg[s0] ? (0b11u << 6) | sub : (sub << 2) | 0b11u;
            break;
        }
        default: {  // (0 | (1,2)) | 3
            unsigned l = sg[s2] ? 0b1001u : 0b0110u;
            unsigned sub = sg[s1] ? (l << 2) : l;
            p = sg[s0] ? (0b11u << 6) | sub : (sub << 2) | 0b11u;
            break;
        }
    }
    // PermToIndex returns 0 (= P(0,1,2,3)) for codes that are not a permutation
    return is_perm(p) ? (uint8_t)p : P4(0, 1, 2, 3);
}

}  // namespace

extern "C" pt_status pt_bvh4_order_table(uint8_t* out) {
    if (!out) return PT_ERR_ARG;
    for (unsigned rs = 0; rs < 8; rs++)
        for (unsigned c = 0; c < 135; c++) out[rs * 135 + c] = order_byte(rs, c);
    return PT_OK;
}

extern "C" pt_status pt_bvh4_build(const float* boxes, uint32_t n, pt_ref_bvh4_cluster* clusters,
                                   uint32_t* n_clusters, pt_ref_bvh4_node* root, uint32_t* prim_order,
                                   float* bbox) {
    if (!root || !n_clusters || (n > 0 && (!boxes || !clusters || !prim_order))) return PT_ERR_ARG;
    *n_clusters = 0;
    *root = pt_ref_bvh4_node{};
    Box all;
    if (n == 0) {
        if (bbox) {
            for (int a = 0; a < 3; a++) {
                bbox[a] = all.mn[a];
                bbox[3 + a] = all.mx[a];
            }
        }
        return PT_OK;
    }
    std::vector<Item> items(n);
    for (uint32_t i = 0; i < n; i++) {
        Item& it = items[i];
        it.index = i;
        for (int a = 0; a < 3; a++) {
            it.box.mn[a] = boxes[6 * (size_t)i + a];
            it.box.mx[a] = boxes[6 * (size_t)i + 3 + a];
            it.c[a] = 0.5f * (it.box.mx[a] + it.box.mn[a]);  // PrimitiveInfo (BVH.hpp:89)
        }
    }
    std::vector<Node2> nodes((size_t)n * 2 - 1);
    std::atomic<uint32_t> next{0};
    build2(0, n, items, nodes, next);
    nodes.resize(next.load());
    Collapser c{nodes, clusters};
    *root = c.collapse(0);
    *n_clusters = c.used;
    for (uint32_t i = 0; i < n; i++) prim_order[i] = items[i].index;
    if (bbox) {
        for (int a = 0; a < 3; a++) {
            bbox[a] = nodes[0].box.mn[a];
            bbox[3 + a] = nodes[0].box.mx[a];
        }
    }
    return PT_OK;
}

// ---------------------------------------------------------------------------
// Instance matrices (host).  glm::inverse(mat4) (glm/detail/func_matrix.inl,
// compute_inverse<4,4>) with every fused multiply-add the reference build
// (g++ -O3 -march=native) forms in it spelled out, so that
// TransformedPrimitive's invTransform (Primitive.hpp:37) comes out bit for
// bit: the cofactors as fused a*b minus a rounded c*d, each lane of Inv0..3
// as a rounded first product with the second and third fused in turn, the
// determinant's pairs fused once (read from GCC's GIMPLE of that function;
// oracle/glm_inverse_probe.cpp computes the reference the two over random affine and
// general matrices).  Explicit, so this file's own contraction cannot change
// it.  m, out: column-major m[c*4+r].
extern "C" pt_status pt_mat4_inverse(const float* mm, float* out) {
    if (!mm || !out) return PT_ERR_ARG;
    // m[c][r]
    const float m00 = mm[0], m01 = mm[1], m02 = mm[2], m03 = mm[3];
    const float m10 = mm[4], m11 = mm[5], m12 = mm[6], m13 = mm[7];
    const float m20 = mm[8], m21 = mm[9], m22 = mm[10], m23 = mm[11];
    const float m30 = mm[12], m31 = mm[13], m32 = mm[14], m33 = mm[15];
    // Coef = a*b - c*d: the first product fused, the second rounded (FMS)
    auto fms = [](float a, float b, float c) { return std::fma(a, b, -c); };
    const float C00 = fms(m22, m33, m32 * m23), C02 = fms(m33, m12, m32 * m13), C03 = fms(m23, m12, m22 * m13);
    const float C04 = fms(m33, m21, m23 * m31), C06 = fms(m33, m11, m13 * m31), C07 = fms(m23, m11, m13 * m21);
    const float C08 = fms(m32, m21, m22 * m31), C10 = fms(m32, m11, m12 * m31), C11 = fms(m22, m11, m12 * m21);
    const float C12 = fms(m33, m20, m23 * m30), C14 = fms(m33, m10, m13 * m30), C15 = fms(m23, m10, m13 * m20);
    const float C16 = fms(m32, m20, m22 * m30), C18 = fms(m32, m10, m12 * m30), C19 = fms(m22, m10, m12 * m20);
    const float C20 = fms(m31, m20, m21 * m30), C22 = fms(m31, m10, m11 * m30), C23 = fms(m21, m10, m11 * m20);
    // Inv_i lane = (Va*Fa - Vb*Fb) + Vc*Fc: Va*Fa rounded, the other two fused in turn
    auto lane = [](float va, float fa, float vb, float fb, float vc, float fc) {
        return std::fma(vc, fc, std::fma(-vb, fb, va * fa));
    };
    float I[16];
    I[0] = lane(m11, C00, m12, C04, m13, C08);
    I[1] = -lane(m01, C00, m02, C04, m03, C08);
    I[2] = lane(m01, C02, m02, C06, m03, C10);
    I[3] = -lane(m01, C03, m02, C07, m03, C11);
    I[4] = -lane(m10, C00, m12, C12, m13, C16);
    I[5] = lane(m00, C00, m02, C12, m03, C16);
    I[6] = -lane(m00, C02, m02, C14, m03, C18);
    I[7] = lane(m00, C03, m02, C15, m03, C19);
    I[8] = lane(m10, C04, m11, C12, m13, C20);
    I[9] = -lane(m00, C04, m01, C12, m03, C20);
    I[10] = lane(m00, C06, m01, C14, m03, C22);
    I[11] = -lane(m00, C07, m01, C15, m03, C23);
    I[12] = -lane(m10, C08, m11, C16, m12, C20);
    I[13] = lane(m00, C08, m01, C16, m02, C20);
    I[14] = -lane(m00, C10, m01, C18, m02, C22);
    I[15] = lane(m00, C11, m01, C19, m02, C23);
    // Dot1 = (m00*Row0.x + m01*Row0.y) + (m02*Row0.z + m03*Row0.w), each pair fused once
    const float dot = std::fma(m01, I[4], m00 * I[0]) + std::fma(m03, I[12], m02 * I[8]);
    const float od = 1.0f / dot;
    for (int k = 0; k < 16; k++) out[k] = I[k] * od;
    return PT_OK;
}
