// TextureInfiniteLight::PreProcess (Light.cpp:150-196) on the host: the
// 1920 x 1080 cell weights an environment map's light sampling draws from.
//
// Compiled with -ffp-contract=off: every fused multiply-add the reference
// build (GCC, -O3 -march=native) forms is written out with std::fma, every
// other product is rounded, as in the device and oracle restatements.
//
// Per cell k (the reference's indexing, x = k % ySamples, y = k / ySamples,
// Light.cpp:171-172) the mean over the 8 x 8 strata of a StratifiedSampler
// (Sampler.hpp:73-147) of luminance(Le(dir(uv))), uv = ((x + UV.x) / 1920,
// (y + UV.y) / 1080).  The reference's stratum permutation only reorders the
// 64 terms (of a double sum); its jitter is unseeded random_float(), here a
// fixed counter-based hash (the stream of DESIGN.md, seed PT_TEXINF_SEED),
// so the weights are a deterministic restatement of the reference's.
#include <cmath>
#include <cstdint>
#include <thread>
#include <vector>

#include "pt_api.h"
#define PT_SC_FMA(a, b, c) std::fma(a, b, c)
#include "pt_sincosf.h"

#define PT_TEXINF_SEED 0x7E1F5EEDu

namespace {

const double kSinCos[2][14] = PT_SC_TABLE;

inline uint32_t pcg_hash(uint32_t v) {  // PCG-RXS-M-XS (pt_device.h)
    uint32_t s = v * 747796405u + 2891336453u;
    uint32_t w = ((s >> ((s >> 28u) + 4u)) ^ s) * 277803737u;
    return (w >> 22u) ^ w;
}
inline uint32_t stream_key(uint32_t seed, uint32_t pixel, uint32_t sample) {
    return pcg_hash(pcg_hash(seed ^ pcg_hash(pixel)) + sample);
}
inline float draw(uint32_t key, uint32_t dim) {
    return (float)(pcg_hash(key + 0x9E3779B9u * dim) >> 8) * (1.0f / 16777216.0f);
}
inline int wrap_index(int i, int n) {
    int m = i % n;
    if (m < 0) m += n;
    return m;
}

struct Env {
    const float* tx;
    int w, h, c;
    float cs[3];
    float scale;
    float texel(int x, int y, int ch) const {  // FloatImage::GetChannelAt (Texture.hpp:78-83)
        return tx[((size_t)wrap_index(y, h) * w + wrap_index(x, w)) * c + ch];
    }
    // LeScale * FloatImageTexture::Evaluate(GetSphereUV(dir)) (Light.cpp:110-112,
    // Texture.hpp:174-189, Shape.hpp:35-43)
    void le(float dx_, float dy_, float dz, float out[3]) const {
        // glm::normalize: dot = x*x rounded, fma(y), fma(z); v * (1 / sqrt)
        const float d2 = std::fma(dz, dz, std::fma(dy_, dy_, dx_ * dx_));
        const float inv = 1.0f / std::sqrt(d2);
        const float px = dx_ * inv, py = dy_ * inv, pz = dz * inv;
        const float theta = std::acos(std::fmin(std::fmax(py, -1.0f), 1.0f));
        float phi = std::atan2(pz, px);
        if (phi < 0) phi += 2.0f * 3.14159265358979323846f;
        const float u = 0.318309886183790671538f * phi * 0.5f;
        const float v = 0.318309886183790671538f * theta;
        const float x = u * w - 0.5f, y = v * h - 0.5f;
        const int xi = (int)std::floor(x), yi = (int)std::floor(y);
        const float fx = x - xi, fy = y - yi;
        const float wa = (1 - fx) * (1 - fy), wb = fx * (1 - fy), wc = (1 - fx) * fy, wd = fx * fy;
        for (int k = 0; k < 3; k++) {
            // w_a*a rounded, then fma(w_b, b), fma(w_c, c), fma(w_d, d) (the device's image blend)
            const float r = std::fma(wd, texel(xi + 1, yi + 1, k),
                                     std::fma(wc, texel(xi, yi + 1, k),
                                              std::fma(wb, texel(xi + 1, yi, k), wa * texel(xi, yi, k))));
            out[k] = scale * (cs[k] * r);
        }
    }
};

// luminance(dvec3) (Util.hpp:4-6): dot with the double constants, GCC's
// contraction (x product rounded, fma(y), fma(z))
inline double luminance(const float l[3]) {
    return std::fma((double)l[2], 0.0722, std::fma((double)l[1], 0.7152, (double)l[0] * 0.2126));
}

float cell_weight(const Env& e, uint32_t k) {
    const int x = (int)(k % PT_TEXINF_Y), y = (int)(k / PT_TEXINF_Y);
    const uint32_t key = stream_key(PT_TEXINF_SEED, k, 0);
    double temp = 0;
    for (int sp = 0; sp < 64; sp++) {
        // StratifiedSampler::get2D: ((sx + dx) / 8, (sy + dy) / 8) in double,
        // stored into the glm::vec2 UV
        const int sx = sp % 8, sy = sp / 8;
        const double jx = (double)draw(key, 2 * sp), jy = (double)draw(key, 2 * sp + 1);
        const float UVx = (float)((sx + jx) / 8.0), UVy = (float)((sy + jy) / 8.0);
        const float u = ((float)x + UVx) / (float)PT_TEXINF_X;
        const float v = ((float)y + UVy) / (float)PT_TEXINF_Y;
        const float z = 2.0f * u - 1.0f;
        const float theta = 2.0f * 3.14159265358979323846f * v;
        const float r = std::sqrt(1.0f - z * z);
        const float cx = r * pt_cosf_t(theta, kSinCos), cy = r * pt_sinf_t(theta, kSinCos);
        float l[3];
        e.le(cx, cy, z, l);
        temp += luminance(l);
    }
    return (float)(temp / 64);
}

}  // namespace

extern "C" pt_status pt_texinf_weights(const float* texels, int32_t width, int32_t height, int32_t channels,
                                       const float color_scale[3], float le_scale, float* weights, int32_t threads) {
    if (!texels || !color_scale || !weights || width <= 0 || height <= 0 || channels < 3) return PT_ERR_ARG;
    const Env e{texels, width, height, channels, {color_scale[0], color_scale[1], color_scale[2]}, le_scale};
    const uint32_t n = (uint32_t)PT_TEXINF_X * PT_TEXINF_Y;
    const int nt = threads > 0 ? threads : 1;
    std::vector<std::thread> pool;
    for (int t = 0; t < nt; t++)
        pool.emplace_back([&, t] {
            for (uint32_t k = (uint32_t)t; k < n; k += (uint32_t)nt) weights[k] = cell_weight(e, k);
        });
    for (auto& th : pool) th.join();
    return PT_OK;
}
