// Conservative per-triangle alpha coverage masks (host code, built at upload).
//
// The traversal's alpha test (GeometricPrimitive::Intersect -> Material::Alpha,
// Primitive.cpp:6-26, Material.hpp:181-198, ImageTexture::alpha
// Texture.cpp:46-62) costs a dependent read of the triangle's alpha record and
// then of four texels.  A triangle's barycentric domain is cut into the 16
// cells of its 4 x 4 subdivision (pt_device.h alpha_cell: row j = floor(4 v)
// holds 4 - j lower and 3 - j upper sub-triangles, cell j (8 - j) + 2 i +
// upper); a cell is decided ACCEPT when every hit the device can compute in
// it passes the reference's test, REJECT when every one fails, and is left to
// the exact test otherwise.  "Every hit": the cell's uv footprint (its
// corners' lerp, widened by a margin far above the float rounding of the
// barycentrics, the lerp and x = u W - 0.5), plus the bilinear neighbour, so
// every texel a hit there can read; and every value the bilinear weights can
// make of those texels (within [min, max] up to 1e-6 of the weights' rounding).
// Only records the fast path reads (u8 images, constants) get masks.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <tuple>
#include <unordered_map>
#include <string>
#include <vector>

// one alpha record's inputs (DevAlpha's fields, pt_device.h)
struct PtAlphaRecord {
    float su[3], sv[3];   // uv components in lerp3f order (uv1, uv2, uv0)
    uint64_t off;         // image byte offset (src != CONST)
    uint32_t W, H, C;     // image size and channel count
    uint32_t src;         // ALPHA_SRC_CH4 / CH1 / CONST
    uint32_t mode;        // PT_ALPHA_OPAQUE / BLEND / MASK
    float cut, scale, constant;
};
static_assert(sizeof(PtAlphaRecord) == 64, "no padding: the coverage memo keys on the bytes");

// A mask set (the upload's word array words()): an accept and a reject mask
// over the n x n cells (cell c: bit c & 31 of word c >> 5), each max(1, n n /
// 32) words, stored either one after the other or interleaved (accept word k,
// reject word k, ...; 8-B aligned: one 64-bit read gives a cell's two bits).
// Its handle = word offset | log2(n / 4) << 29;
// PT_ALPHA_SET_NONE: no cell decided (or no set computed).
#define PT_ALPHA_SET_NONE 0xFFFFFFFFu
// square-table lookups the masks of one upload may spend (host time); the
// records past it get no set
#define PT_ALPHA_LOOKUP_BUDGET (1ull << 31)

class PtAlphaCoverage {
public:
    // max_n: the finest subdivision (a power of two, 4 .. 256)
    PtAlphaCoverage(const uint8_t* texels, uint64_t n_texel_bytes, int max_n = 128, bool interleave = false)
        : texels_(texels), n_(n_texel_bytes), max_n_(max_n), il_(interleave) {}
    // the mask set of a record (n from the triangle's texel extent: cells of
    // ~8 texels, 4 .. max_n per side); identical records share one set
    uint32_t set(const PtAlphaRecord& r);
    const std::vector<uint32_t>& words() const { return words_; }

private:
    // min / max of one channel over every 2^k x 2^k square (k <= 6): any
    // rectangle is a union of (overlapping) squares, so its min / max is exact
    struct Pyramid {
        int W, H;
        std::vector<std::vector<uint8_t>> mn, mx;  // [k][y W + x]: square at (x, y)
        uint64_t query(int x0, int x1, int y0, int y1, uint8_t& lo, uint8_t& hi) const;  // -> squares read
    };
    bool footprint(const Pyramid& P, const double px[3], const double py[3], double mx, double my, uint8_t& blo,
                   uint8_t& bhi);
    const Pyramid* pyramid(uint64_t off, uint32_t W, uint32_t H, uint32_t C, uint32_t ch);
    const uint8_t* texels_;
    uint64_t n_;
    int max_n_;
    bool il_;
    std::map<std::tuple<uint64_t, uint32_t, uint32_t, uint32_t, uint32_t>, std::unique_ptr<Pyramid>> pyr_;
    std::unordered_map<std::string, uint32_t> memo_;  // identical records (leaf cards share uvs)
    std::vector<uint32_t> words_;
    uint64_t lookups_ = 0;
};
