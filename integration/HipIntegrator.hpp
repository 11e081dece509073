// Drop-in GPU integrators for marko176/PathTracing's C++ host.
//
// HipPathIntegrator / HipSimplePathIntegrator keep the reference's
// constructors (Integrators.hpp:36, 46) and its Render(n) call pattern
// (main.cpp:347-350): the application builds Scene / Camera / Film / Sampler
// / LightSampler exactly as before and swaps the integrator type.  Render(n)
// flattens the built scene once (the reference's own BVH4 cluster arrays,
// byte for byte), uploads it through the C ABI of libpt_hip.so
// (include/pt_api.h) to min(n, #GPUs) devices, renders the interleaved sample
// shards with the HIP wavefront tracer and merges {sum RGB*w, sum w} into the
// camera's Film through FilmTile / Film::Merge (Film.hpp:118-132).  Li(Ray)
// is inherited unchanged: the CPU integrator stays available for tests.
//
// Render(n) is adaptive like the reference's TileIntegrator::Render
// (Integrators.cpp:55-86: per-pixel rounds of spp samples until the
// luminance-weighted relative variance is <= 1.5, at most 128*spp) -- on the
// GPUs, with the devices splitting the frame by 32x32 tiles.
// SetAdaptive(false) renders exactly spp samples per pixel (interleaved
// sample shards), the fixed-SPP frame of the benchmark.
//
// The sample stream is the counter-based PCG stream of DESIGN.md; use
// pt::PCGSampler to choose its seed (any other Sampler supplies only its
// SamplesPerPixel(); the reference's own samplers are unseeded).  A
// StratifiedSampler(xSamples, ySamples) -- or a PCGSampler given strata --
// stratifies the camera draws as Render's per-thread clone of it does
// (Sampler.hpp:73-151), the stream supplying the jitter.
// FunctionInfiniteLight is supported when its function is a pt::SkyGradient
// (the gradient of main.cpp:292-295).  See INTEGRATION.md.
#pragma once
#include <array>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "Integrators.hpp"
#include "Ray.hpp"
#include "Sampler.hpp"

namespace pt {

// main.cpp:292-295's sky: scale * ((1-a)*horizon + a*zenith), a = (dir.y+1)/2
struct SkyGradient {
    glm::vec3 horizon{1.0f, 0.85f, 0.55f};
    glm::vec3 zenith{0.45f, 0.65f, 1.0f};
    float scale = 1.5f;
    glm::vec3 operator()(const Ray& ray) const {
        float a = 0.5f * (ray.dir.y + 1.0f);
        return scale * ((1.0f - a) * horizon + a * zenith);
    }
};

// The deterministic per-(pixel, sample) PCG stream shared with the GPU path:
// key = h(h(seed ^ h(pixel)) + sample), draw = (h(key + 0x9E3779B9*dim) >> 8) * 2^-24
class PCGSampler : public Sampler {
public:
    PCGSampler(unsigned spp, uint32_t seed, int width, unsigned strata_x = 0, unsigned strata_y = 0)
        : spp_(spp), seed_(seed), width_(width), strata_x_(strata_x), strata_y_(strata_y) {}
    unsigned int SamplesPerPixel() const override { return spp_; }
    void StartPixelSample(const glm::ivec2& p, int index) override;
    double get1D() override { return next(); }
    glm::dvec2 get2D() override;
    glm::dvec2 getPixel2D() override { return get2D(); }
    std::array<glm::vec2, 4> get2Dx4f() override;
    std::shared_ptr<Sampler> Clone() const override {
        return std::make_shared<PCGSampler>(spp_, seed_, width_, strata_x_, strata_y_);
    }
    uint32_t Seed() const { return seed_; }
    unsigned StrataX() const { return strata_x_; }
    unsigned StrataY() const { return strata_y_; }

private:
    float next();
    unsigned spp_;
    uint32_t seed_;
    int width_;
    unsigned strata_x_, strata_y_;  // camera strata (0: the plain stream)
    uint32_t key_ = 0, dim_ = 0;
};

struct RenderStats {
    uint64_t paths = 0, rays_closest = 0, rays_any = 0;
    uint32_t devices = 0;  // GPUs that rendered (films reduced over RCCL)
    double ms = 0;
};

class HipBackend;  // flattened scene + one multi-GPU pt_ctx

class HipPathIntegrator : public PathIntegrator {
public:
    HipPathIntegrator(const std::shared_ptr<Scene>& scene, const std::shared_ptr<Camera>& camera,
                      const std::shared_ptr<Sampler>& sampler, const std::shared_ptr<LightSampler>& lightSampler,
                      uint32_t maxDepth);
    ~HipPathIntegrator() override;
    // n = GPUs to use (capped at the devices present); blocks until the frame
    // is merged into camera->GetFilm().  Throws std::runtime_error on failure.
    void Render(unsigned int n = 1) const override;
    RenderStats LastStats() const;
    // W*H*4 {sum R*w, sum G*w, sum B*w, sum w} the last Render merged into the Film
    const std::vector<double>& LastAccumulation() const;
    // adaptive sampling on (default, as the reference's Render) or fixed SPP
    void SetAdaptive(bool on) { adaptive_ = on; }
    // W*H samples per pixel of the last Render
    const std::vector<uint32_t>& LastSampleCounts() const;

private:
    std::shared_ptr<LightSampler> ls_;
    uint32_t depth_;
    bool adaptive_ = true;
    mutable std::unique_ptr<HipBackend> be_;
    mutable std::mutex mu_;
};

class HipSimplePathIntegrator : public SimplePathIntegrator {
public:
    HipSimplePathIntegrator(const std::shared_ptr<Scene>& scene, const std::shared_ptr<Camera>& camera,
                            const std::shared_ptr<Sampler>& sampler, uint32_t maxDepth);
    ~HipSimplePathIntegrator() override;
    void Render(unsigned int n = 1) const override;
    RenderStats LastStats() const;
    const std::vector<double>& LastAccumulation() const;
    // adaptive sampling on (default, as the reference's Render) or fixed SPP
    void SetAdaptive(bool on) { adaptive_ = on; }
    // W*H samples per pixel of the last Render
    const std::vector<uint32_t>& LastSampleCounts() const;

private:
    uint32_t depth_;
    bool adaptive_ = true;
    mutable std::unique_ptr<HipBackend> be_;
    mutable std::mutex mu_;
};

// VolPathIntegrator (Integrators.hpp:56-67) on the GPU: HomogeneusMedium with a
// HenyeyGreenstein phase function (scene, camera and primitive media).  The
// medium's two hidden random_float() draws (Medium.hpp:28-30) come from the
// PCG stream on the GPU.
class HipVolPathIntegrator : public VolPathIntegrator {
public:
    HipVolPathIntegrator(const std::shared_ptr<Scene>& scene, const std::shared_ptr<Camera>& camera,
                         const std::shared_ptr<Sampler>& sampler, const std::shared_ptr<LightSampler>& lightSampler,
                         uint32_t maxDepth);
    ~HipVolPathIntegrator() override;
    void Render(unsigned int n = 1) const override;
    RenderStats LastStats() const;
    const std::vector<double>& LastAccumulation() const;
    // adaptive sampling on (default, as the reference's Render) or fixed SPP
    void SetAdaptive(bool on) { adaptive_ = on; }
    // W*H samples per pixel of the last Render
    const std::vector<uint32_t>& LastSampleCounts() const;

private:
    std::shared_ptr<LightSampler> ls_;
    uint32_t depth_;
    bool adaptive_ = true;
    mutable std::unique_ptr<HipBackend> be_;
    mutable std::mutex mu_;
};

}  // namespace pt
