// HipPathIntegrator / HipSimplePathIntegrator: see HipIntegrator.hpp.
//
// Scene export.  The reference keeps most of the state the device needs in
// private or protected members (BVH4::nodes BVH.hpp:1214-1216, the
// primitive / material / texture / light fields).  Rather than editing the
// reference, the exporter reads them through member pointers formed by
// explicit template instantiation (which the language exempts from access
// checking); a maintainer merging this into the tree would replace the
// PT_MEMBER lines with `friend class pt::SceneExport;` declarations.
#include "HipIntegrator.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <functional>
#include <map>
#include <stdexcept>
#include <thread>
#include <unordered_map>

#include "BVH.hpp"
#include "Camera.hpp"
#include "Film.hpp"
#include "Filter.hpp"
#include "Light.hpp"
#include "LightSampler.hpp"
#include "Material.hpp"
#include "Medium.hpp"
#include "Mesh.hpp"
#include "PhaseFunction.hpp"
#include "Primitive.hpp"
#include "Scene.hpp"
#include "Shape.hpp"
#include "Texture.hpp"
#ifdef PT_WITH_MODEL
#include "Model.hpp"
#endif
#include "pt_api.h"

namespace {

template <class Tag, typename Tag::type M>
struct Member {
    friend typename Tag::type get(Tag) { return M; }
};
#define PT_MEMBER(NAME, CLASS, TYPE, FIELD)      \
    struct NAME {                                \
        using type = TYPE CLASS::*;              \
        friend type get(NAME);                   \
    };                                           \
    template struct Member<NAME, &CLASS::FIELD>
#define PT_GET(OBJ, NAME) ((OBJ).*get(NAME{}))

using PrimPtr = std::shared_ptr<Primitive>;
using TexPtr = std::shared_ptr<Texture>;
using TLASBase = BVHBase<PrimPtr>;
using BLASBase = BVHBase<GeometricPrimitive>;

PT_MEMBER(SceneBvh, Scene, std::shared_ptr<TLASBase>, scene_bvh);
PT_MEMBER(TlasNodes, TLAS4, std::vector<BVH4_CLUSTER>, nodes);
PT_MEMBER(TlasRoot, TLAS4, BVH4_NODE, rootNode);
PT_MEMBER(TlasPrims, TLASBase, std::vector<PrimPtr>, primitives);
PT_MEMBER(BlasNodes, BLAS4, std::vector<BVH4_CLUSTER>, nodes);
PT_MEMBER(BlasRoot, BLAS4, BVH4_NODE, rootNode);
PT_MEMBER(BlasPrims, BLASBase, std::vector<GeometricPrimitive>, primitives);
PT_MEMBER(GpShape, GeometricPrimitive, std::shared_ptr<Shape>, shape);
PT_MEMBER(GpMaterial, GeometricPrimitive, std::shared_ptr<Material>, material);
PT_MEMBER(GpArea, GeometricPrimitive, std::shared_ptr<AreaLight>, areaLight);
PT_MEMBER(GpMedium, GeometricPrimitive, std::shared_ptr<Medium>, medium);
PT_MEMBER(MedSigmaA, HomogeneusMedium, glm::vec3, sigma_a);
PT_MEMBER(MedSigmaS, HomogeneusMedium, glm::vec3, sigma_s);
PT_MEMBER(MedSigmaT, HomogeneusMedium, glm::vec3, sigma_t);
PT_MEMBER(MedLe, HomogeneusMedium, glm::vec3, emmision);
PT_MEMBER(MedPhase, HomogeneusMedium, std::shared_ptr<PhaseFunction>, phaseFunction);
PT_MEMBER(HgG, HenyeyGreenstein, float, g);
PT_MEMBER(SphCenter, SphereShape, glm::vec3, center);
PT_MEMBER(SphRadius, SphereShape, float, radius);
PT_MEMBER(QuadQ, QuadShape, glm::vec3, Q);
PT_MEMBER(QuadU, QuadShape, glm::vec3, u);
PT_MEMBER(QuadV, QuadShape, glm::vec3, v);
PT_MEMBER(QuadN, QuadShape, glm::vec3, normal);
PT_MEMBER(QuadD, QuadShape, float, D);
PT_MEMBER(QuadW, QuadShape, glm::vec3, w);
PT_MEMBER(DifTex, MicrofacetDiffuse, TexPtr, tex);
PT_MEMBER(DifNorm, MicrofacetDiffuse, TexPtr, norm);
PT_MEMBER(DifRough, MicrofacetDiffuse, TexPtr, roughnessTexture);
PT_MEMBER(DifMetal, MicrofacetDiffuse, TexPtr, metallicTexture);
PT_MEMBER(DifAlpha, MicrofacetDiffuse, TexPtr, alpha);
PT_MEMBER(DifTester, MicrofacetDiffuse, AlphaTester, alphaTester);
PT_MEMBER(DieRi, MicrofacetDielectric, float, ri);
PT_MEMBER(DieTex, MicrofacetDielectric, TexPtr, tex);
PT_MEMBER(DieNorm, MicrofacetDielectric, TexPtr, norm);
PT_MEMBER(DieRough, MicrofacetDielectric, TexPtr, roughnessTexture);
PT_MEMBER(DieAlpha, MicrofacetDielectric, TexPtr, alpha);
PT_MEMBER(DieTester, MicrofacetDielectric, AlphaTester, alphaTester);
PT_MEMBER(ThinRi, ThinDielectric, float, ri);
PT_MEMBER(ThinAlbedo, ThinDielectric, TexPtr, albedo);
PT_MEMBER(CondAlbedo, SpecularConductor, glm::vec3, albedo);
PT_MEMBER(TexScale, Texture, glm::vec3, colorScale);
PT_MEMBER(SolidAlbedo, SolidColor, glm::vec3, albedo);
PT_MEMBER(ImgTexImage, ImageTexture, Image, image);
PT_MEMBER(ImgData, Image, unsigned char*, data);
PT_MEMBER(ImgW, Image, int, width);
PT_MEMBER(ImgH, Image, int, height);
PT_MEMBER(ImgC, Image, int, channels);
PT_MEMBER(FImgTexImage, FloatImageTexture, FloatImage, image);
PT_MEMBER(FImgData, FloatImage, float*, data);
PT_MEMBER(FImgW, FloatImage, int, width);
PT_MEMBER(FImgH, FloatImage, int, height);
PT_MEMBER(FImgC, FloatImage, int, channels);
PT_MEMBER(TexInfTex, TextureInfiniteLight, TexPtr, tex);
PT_MEMBER(TexInfScale, TextureInfiniteLight, float, LeScale);
PT_MEMBER(TexInfAcc, TextureInfiniteLight, std::vector<float>, accWeights);
PT_MEMBER(ChkA, CheckerTexture, TexPtr, tex1);
PT_MEMBER(ChkB, CheckerTexture, TexPtr, tex2);
PT_MEMBER(ChkInv, CheckerTexture, glm::vec2, invScale);
PT_MEMBER(AreaShape, AreaLight, std::shared_ptr<Shape>, shape);
PT_MEMBER(AreaTex, AreaLight, TexPtr, emissiveTexture);
PT_MEMBER(AreaOneSided, AreaLight, bool, oneSided);
PT_MEMBER(UniColor, UniformInfiniteLight, glm::vec3, color);
PT_MEMBER(FunFn, FunctionInfiniteLight, std::function<glm::vec3(const Ray&)>, lightFunction);
PT_MEMBER(DistDir, DistantLight, glm::vec3, dir);
PT_MEMBER(DistColor, DistantLight, glm::vec3, color);
PT_MEMBER(PointP, PointLight, glm::vec3, p);
PT_MEMBER(PointColor, PointLight, glm::vec3, color);
PT_MEMBER(UlsLights, UniformLightSampler, std::vector<std::shared_ptr<Light>>, lights);
PT_MEMBER(PlsLights, PowerLightSampler, std::vector<std::shared_ptr<Light>>, lights);
PT_MEMBER(CamFrom, Camera, glm::vec3, lookFrom);
PT_MEMBER(CamU, Camera, glm::vec3, u);
PT_MEMBER(CamV, Camera, glm::vec3, v);
PT_MEMBER(CamW, Camera, glm::vec3, w);
PT_MEMBER(CamHW, Camera, float, halfWidth);
PT_MEMBER(CamHH, Camera, float, halfHeight);
PT_MEMBER(CamDefocus, Camera, float, defocusRadius);
PT_MEMBER(CamFocusDist, Camera, float, FocusDistance);
PT_MEMBER(CamFocusAngle, Camera, float, FocusAngle);
PT_MEMBER(CamShutterStart, Camera, float, shutterStart);
PT_MEMBER(StratX, StratifiedSampler, unsigned int, xSamples);
PT_MEMBER(StratY, StratifiedSampler, unsigned int, ySamples);
PT_MEMBER(CamShutterEnd, Camera, float, shutterEnd);
PT_MEMBER(FilmFilter, Film, std::shared_ptr<Filter>, filter);
PT_MEMBER(MitB, MitchellFilter, double, b);
PT_MEMBER(MitC, MitchellFilter, double, c);
PT_MEMBER(GaussSigma, GaussianFilter, double, sigma);
PT_MEMBER(LanczosTau, LanczosFilter, double, tau);
#ifdef PT_WITH_MODEL
PT_MEMBER(ModelBvh, Model, std::shared_ptr<BLASBase>, model_bvh);
#endif
PT_MEMBER(TlLight, TransformedLight, std::shared_ptr<Light>, light);
PT_MEMBER(TlXf, TransformedLight, glm::mat4, transform);
PT_MEMBER(AlLight, AnimatedLight, std::shared_ptr<Light>, light);
PT_MEMBER(AlDir, AnimatedLight, glm::vec3, dir);
PT_MEMBER(AlTb, AnimatedLight, glm::vec2, timeBounds);
PT_MEMBER(TpPrim, TransformedPrimitive, std::shared_ptr<Primitive>, primitive);
PT_MEMBER(TpXf, TransformedPrimitive, glm::mat4, transform);
PT_MEMBER(TpInv, TransformedPrimitive, glm::mat4, invTransform);
PT_MEMBER(ApPrim, AnimatedPrimitive, std::shared_ptr<Primitive>, primitive);
PT_MEMBER(ApDir, AnimatedPrimitive, glm::vec3, dir);
PT_MEMBER(ApTb, AnimatedPrimitive, glm::vec2, timeBounds);

void check(pt_status st, const char* what, pt_ctx* c = nullptr) {
    if (st != PT_OK) throw std::runtime_error(std::string(what) + ": " + pt_last_error(c));
}

void put3(float* d, const glm::vec3& v) {
    d[0] = v.x;
    d[1] = v.y;
    d[2] = v.z;
}

// ---------------------------------------------------------------------------
// Flattened scene (owns every array a pt_scene_desc points at)
struct Flat {
    std::vector<float> positions, normals, uvs, tangents;
    std::vector<uint32_t> tri_vidx, tri_flags;
    std::vector<pt_quad> quads;
    std::vector<pt_sphere> spheres;
    std::vector<pt_prim> prims;
    std::vector<pt_bvh_desc> bvhs;
    std::vector<pt_material> materials;
    std::vector<pt_texture> textures;
    std::vector<pt_image> images;
    std::vector<uint8_t> texels;
    std::vector<pt_light> lights;
    std::vector<uint32_t> sampler_lights, infinite_lights;
    std::vector<float> light_dist;  // TextureInfiniteLight running sums
    uint32_t light_sampler = PT_LS_UNIFORM;
    std::vector<pt_medium> media;
    int32_t scene_medium = -1;
    std::unordered_map<const Medium*, int32_t> med_ids;
    std::vector<pt_instance> instances;
    // one-primitive BLASes of instanced GeometricPrimitives (own node storage)
    std::vector<std::vector<pt_ref_bvh4_cluster>> own_clusters;

    // HomogeneusMedium + HenyeyGreenstein (Medium.hpp:14-61, PhaseFunction.hpp:17-27)
    int32_t medium(const std::shared_ptr<Medium>& m) {
        if (!m) return -1;
        auto it = med_ids.find(m.get());
        if (it != med_ids.end()) return it->second;
        auto* h = dynamic_cast<const HomogeneusMedium*>(m.get());
        if (!h) throw std::runtime_error("HipVolPathIntegrator: unsupported medium type");
        auto* hg = dynamic_cast<const HenyeyGreenstein*>(PT_GET(*h, MedPhase).get());
        if (!hg) throw std::runtime_error("HipVolPathIntegrator: unsupported phase function");
        pt_medium r{};
        put3(r.sigma_a, PT_GET(*h, MedSigmaA));
        put3(r.sigma_s, PT_GET(*h, MedSigmaS));
        put3(r.sigma_t, PT_GET(*h, MedSigmaT));
        put3(r.Le, PT_GET(*h, MedLe));
        r.g = PT_GET(*hg, HgG);
        const int32_t id = (int32_t)media.size();
        media.push_back(r);
        med_ids[m.get()] = id;
        return id;
    }

    std::unordered_map<const Mesh*, uint32_t> mesh_vbase, mesh_tbase;
    std::unordered_map<const Texture*, int32_t> tex_ids;
    std::unordered_map<const Material*, int32_t> mat_ids;
    std::unordered_map<const Light*, int32_t> light_slot;  // AreaLight -> prim slot

    int32_t texture(const TexPtr& t) {
        if (!t) return -1;
        auto it = tex_ids.find(t.get());
        if (it != tex_ids.end()) return it->second;
        pt_texture r{};
        r.a = r.b = r.image = -1;
        put3(r.scale, PT_GET(*t, TexScale));
        if (auto* s = dynamic_cast<const SolidColor*>(t.get())) {
            r.kind = PT_TEX_SOLID;
            glm::vec3 v = PT_GET(*t, TexScale) * PT_GET(*s, SolidAlbedo);  // SolidColor::Evaluate
            put3(r.value, v);
        } else if (auto* c = dynamic_cast<const CheckerTexture*>(t.get())) {
            r.kind = PT_TEX_CHECKER;
            r.a = texture(PT_GET(*c, ChkA));
            r.b = texture(PT_GET(*c, ChkB));
            glm::vec2 inv = PT_GET(*c, ChkInv);
            r.inv_scale[0] = inv.x;
            r.inv_scale[1] = inv.y;
        } else if (auto* im = dynamic_cast<const ImageTexture*>(t.get())) {
            const Image& img = PT_GET(*im, ImgTexImage);
            pt_image pi{};
            pi.offset = texels.size();
            pi.width = PT_GET(img, ImgW);
            pi.height = PT_GET(img, ImgH);
            pi.channels = PT_GET(img, ImgC);
            const unsigned char* px = PT_GET(img, ImgData);
            texels.insert(texels.end(), px, px + (size_t)pi.width * pi.height * pi.channels);
            texels.resize((texels.size() + 15) & ~size_t(15));
            r.kind = PT_TEX_IMAGE;
            r.image = (int32_t)images.size();
            images.push_back(pi);
        } else if (auto* fm = dynamic_cast<const FloatImageTexture*>(t.get())) {
            // FloatImage texels (Texture.hpp:70-103): float bytes, 4-aligned
            const FloatImage& img = PT_GET(*fm, FImgTexImage);
            pt_image pi{};
            pi.offset = texels.size();
            pi.width = PT_GET(img, FImgW);
            pi.height = PT_GET(img, FImgH);
            pi.channels = PT_GET(img, FImgC);
            pi.format = PT_IMAGE_F32;
            const auto* px = reinterpret_cast<const uint8_t*>(PT_GET(img, FImgData));
            texels.insert(texels.end(), px, px + 4 * (size_t)pi.width * pi.height * pi.channels);
            texels.resize((texels.size() + 15) & ~size_t(15));
            r.kind = PT_TEX_IMAGE;
            r.image = (int32_t)images.size();
            images.push_back(pi);
        } else {
            throw std::runtime_error("HipPathIntegrator: unsupported texture type");
        }
        int32_t id = (int32_t)textures.size();
        textures.push_back(r);
        tex_ids[t.get()] = id;
        return id;
    }

    int32_t material(const std::shared_ptr<Material>& m) {
        if (!m) return -1;
        auto it = mat_ids.find(m.get());
        if (it != mat_ids.end()) return it->second;
        pt_material r{};
        r.tex = r.norm = r.rough = r.metal = r.alpha = -1;
        if (auto* d = dynamic_cast<const MicrofacetDiffuse*>(m.get())) {
            r.kind = PT_MAT_DIFFUSE;
            r.tex = texture(PT_GET(*d, DifTex));
            r.norm = texture(PT_GET(*d, DifNorm));
            r.rough = texture(PT_GET(*d, DifRough));
            r.metal = texture(PT_GET(*d, DifMetal));
            r.alpha = texture(PT_GET(*d, DifAlpha));
            const AlphaTester& at = PT_GET(*d, DifTester);
            r.alpha_mode = (uint32_t)at.mode;
            r.alpha_cutoff = at.cutoff;
        } else if (auto* e = dynamic_cast<const MicrofacetDielectric*>(m.get())) {
            r.kind = PT_MAT_DIELECTRIC;
            r.ri = PT_GET(*e, DieRi);
            r.tex = texture(PT_GET(*e, DieTex));
            r.norm = texture(PT_GET(*e, DieNorm));
            r.rough = texture(PT_GET(*e, DieRough));
            r.alpha = texture(PT_GET(*e, DieAlpha));
            const AlphaTester& at = PT_GET(*e, DieTester);
            r.alpha_mode = (uint32_t)at.mode;
            r.alpha_cutoff = at.cutoff;
        } else if (auto* t = dynamic_cast<const ThinDielectric*>(m.get())) {
            r.kind = PT_MAT_THIN;
            r.ri = PT_GET(*t, ThinRi);
            r.tex = texture(PT_GET(*t, ThinAlbedo));
        } else if (auto* c = dynamic_cast<const SpecularConductor*>(m.get())) {
            r.kind = PT_MAT_CONDUCTOR;
            put3(r.albedo, PT_GET(*c, CondAlbedo));
        } else {
            throw std::runtime_error("HipPathIntegrator: unsupported material type");
        }
        int32_t id = (int32_t)materials.size();
        materials.push_back(r);
        mat_ids[m.get()] = id;
        return id;
    }

    uint32_t triangle(const TriangleShape& ts) {
        const Mesh* mesh = TriangleShape::getMeshAt(ts.getMeshIndex());
        auto it = mesh_tbase.find(mesh);
        if (it == mesh_tbase.end()) {  // first triangle of this mesh: append the mesh
            const uint32_t vb = (uint32_t)(positions.size() / 3), tb = (uint32_t)tri_flags.size();
            auto v = mesh->GetVertices();
            auto n = mesh->GetNormals();
            auto uv = mesh->GetTexCoords();
            auto tg = mesh->GetTangents();
            auto idx = mesh->GetIndices();
            for (size_t i = 0; i < v.size(); i++) {
                positions.insert(positions.end(), {v[i].x, v[i].y, v[i].z});
                normals.insert(normals.end(), {n[i].x, n[i].y, n[i].z});
                uvs.insert(uvs.end(), {uv[i].x, uv[i].y});
                if (tg.empty()) tangents.insert(tangents.end(), {0.0f, 0.0f, 0.0f});
                else tangents.insert(tangents.end(), {tg[i].x, tg[i].y, tg[i].z});
            }
            for (uint32_t i : idx) tri_vidx.push_back(vb + i);
            tri_flags.insert(tri_flags.end(), idx.size() / 3, tg.empty() ? 0u : 1u);
            it = mesh_tbase.emplace(mesh, tb).first;
        }
        return it->second + ts.getTriIndex();
    }

    // One GeometricPrimitive into slot `slot`.
    void geometric(const GeometricPrimitive& gp, uint32_t slot) {
        pt_prim& p = prims[slot];
        const auto& shape = PT_GET(gp, GpShape);
        if (auto* t = dynamic_cast<const TriangleShape*>(shape.get())) {
            p.kind = PT_PRIM_TRIANGLE;
            p.index = triangle(*t);
        } else if (auto* q = dynamic_cast<const QuadShape*>(shape.get())) {
            pt_quad r{};
            put3(r.Q, PT_GET(*q, QuadQ));
            put3(r.u, PT_GET(*q, QuadU));
            put3(r.v, PT_GET(*q, QuadV));
            put3(r.normal, PT_GET(*q, QuadN));
            r.D = PT_GET(*q, QuadD);
            put3(r.w, PT_GET(*q, QuadW));
            p.kind = PT_PRIM_QUAD;
            p.index = (uint32_t)quads.size();
            quads.push_back(r);
        } else if (auto* s = dynamic_cast<const SphereShape*>(shape.get())) {
            pt_sphere r{};
            put3(r.center, PT_GET(*s, SphCenter));
            r.radius = PT_GET(*s, SphRadius);
            p.kind = PT_PRIM_SPHERE;
            p.index = (uint32_t)spheres.size();
            spheres.push_back(r);
        } else {
            throw std::runtime_error("HipPathIntegrator: unsupported shape type");
        }
        p.material = material(PT_GET(gp, GpMaterial));
        p.medium = medium(PT_GET(gp, GpMedium));
        p.light = -1;
        if (const auto& al = PT_GET(gp, GpArea)) light_slot[al.get()] = (int32_t)slot;
    }

    void build(const Scene& scene, const std::shared_ptr<LightSampler>& ls) {
        const auto& tb = PT_GET(scene, SceneBvh);
        auto* tlas = dynamic_cast<TLAS4*>(tb.get());
        if (!tlas) throw std::runtime_error("HipPathIntegrator: the scene must be built with BuildTlas<TLAS4>()");
        const auto& top = PT_GET(*static_cast<TLASBase*>(tlas), TlasPrims);
        const auto& tnodes = PT_GET(*tlas, TlasNodes);
        static_assert(sizeof(BVH4_CLUSTER) == sizeof(pt_ref_bvh4_cluster), "cluster layout");
        const uint32_t n_top = (uint32_t)top.size();
        scene_medium = medium(scene.GetMedium());
        // BLAS list: the Models of the TLAS slots and the instanced primitives
        // (TransformedPrimitive / AnimatedPrimitive), once each, in slot
        // order; an instanced GeometricPrimitive gets a one-primitive BLAS
        struct Blas {
            const BLAS4* b = nullptr;                // a Model's BLAS4
            const GeometricPrimitive* gp = nullptr;  // or one GeometricPrimitive
        };
        std::vector<Blas> blas;
        std::unordered_map<const void*, uint32_t> blas_index;
        auto blas_of = [&](const Primitive* p) -> uint32_t {
            const BLAS4* b = dynamic_cast<const BLAS4*>(p);
#ifdef PT_WITH_MODEL
            if (!b)
                if (auto* m = dynamic_cast<const Model*>(p)) b = dynamic_cast<const BLAS4*>(PT_GET(*m, ModelBvh).get());
#endif
            const GeometricPrimitive* gp = b ? nullptr : dynamic_cast<const GeometricPrimitive*>(p);
            if (!b && !gp) return UINT32_MAX;
            const void* key = b ? (const void*)b : (const void*)gp;
            auto it = blas_index.find(key);
            if (it != blas_index.end()) return it->second;
            blas.push_back(Blas{b, gp});
            return blas_index[key] = (uint32_t)blas.size() - 1;
        };
        // one wrapper level: TransformedPrimitive / AnimatedPrimitive
        struct Level {
            glm::mat4 xf, inv;
            bool animated = false;  // AnimatedPrimitive: translated per ray at its time
            glm::vec3 dir{0};
            glm::vec2 tb{0};
        };
        struct Inst {
            uint32_t blas;
            std::vector<Level> levels;  // nested wrappers, the outermost first (pt_instance.inner)
        };
        std::vector<Inst> inst;
        std::vector<uint32_t> blas_of_slot(n_top, UINT32_MAX), inst_of_slot(n_top, UINT32_MAX);
        auto mat_key = [](const glm::mat4& m) { return std::string((const char*)&m[0][0], sizeof(glm::mat4)); };
        // (inner AreaLight, the wrappers' matrices outermost first) -> instance
        std::map<std::pair<const Light*, std::string>, int32_t> inst_light;
        std::vector<std::shared_ptr<Light>> inner_lights;
        // a wrapper level, or false for anything else
        auto level_of = [&](const Primitive* p, Level& lv, const Primitive*& inner) {
            if (auto* tp = dynamic_cast<const TransformedPrimitive*>(p)) {
                inner = PT_GET(*tp, TpPrim).get();
                lv.xf = PT_GET(*tp, TpXf);
                lv.inv = PT_GET(*tp, TpInv);
                return true;
            }
            if (auto* ap = dynamic_cast<const AnimatedPrimitive*>(p)) {
                // AnimatedPrimitive::Intersect (Primitive.cpp:86-89): the
                // device translates by dir * t at each ray's time; the time-0
                // matrix keys its AnimatedLights below
                inner = PT_GET(*ap, ApPrim).get();
                const glm::vec2 tb = PT_GET(*ap, ApTb);
                const float t = glm::clamp(0.0f - tb.x, tb.x, tb.y) / (tb.y - tb.x);
                lv.xf = glm::translate(glm::mat4(1), PT_GET(*ap, ApDir) * t);
                lv.inv = glm::inverse(lv.xf);
                lv.animated = true;
                lv.dir = PT_GET(*ap, ApDir);
                lv.tb = tb;
                return true;
            }
            return false;
        };
        for (uint32_t i = 0; i < n_top; i++) {
            const Primitive* p = top[i].get();
            if (dynamic_cast<const GeometricPrimitive*>(p)) continue;
            Inst in{};
            const Primitive* inner = p;
            for (Level lv; level_of(inner, lv, inner); lv = Level{}) in.levels.push_back(lv);
            if (in.levels.empty()) {
                blas_of_slot[i] = blas_of(p);
                if (blas_of_slot[i] == UINT32_MAX) throw std::runtime_error("HipPathIntegrator: unsupported TLAS primitive");
                continue;
            }
            if (in.levels.size() > PT_MAX_INSTANCE_DEPTH)
                throw std::runtime_error("HipPathIntegrator: instances nested deeper than PT_MAX_INSTANCE_DEPTH");
            // emitters inside the instance: each wrapper's GetLights wraps its
            // inner primitive's lights with its own matrix (Primitive.cpp:66-73,
            // 91-96; Light.cpp:338-364), keyed here by the whole chain
            std::string key;
            for (const Level& lv : in.levels) key += mat_key(lv.xf);
            for (const auto& l : inner->GetLights()) {
                inst_light[{l.get(), key}] = (int32_t)inst.size();
                inner_lights.push_back(l);
            }
            in.blas = blas_of(inner);
            if (in.blas == UINT32_MAX) throw std::runtime_error("HipPathIntegrator: unsupported instanced primitive");
            inst_of_slot[i] = (uint32_t)inst.size();
            inst.push_back(std::move(in));
        }
        auto blas_count = [&](const Blas& b) -> uint32_t {
            return b.gp ? 1u : (uint32_t)PT_GET(*static_cast<const BLASBase*>(b.b), BlasPrims).size();
        };
        uint32_t total = n_top;
        std::vector<uint32_t> base(blas.size());
        for (size_t k = 0; k < blas.size(); k++) {
            base[k] = total;
            total += blas_count(blas[k]);
        }
        prims.assign(total, pt_prim{});
        pt_bvh_desc t{};
        t.clusters = reinterpret_cast<const pt_ref_bvh4_cluster*>(tnodes.data());
        t.n_clusters = (uint32_t)tnodes.size();
        std::memcpy(&t.root, &PT_GET(*tlas, TlasRoot), sizeof(t.root));
        t.prim_base = 0;
        t.n_prims = n_top;
        bvhs.push_back(t);
        uint32_t virt = total;  // virtual slots of the instances' primitives, ascending
        auto record = [&](const Level& lv, uint32_t b) {
            pt_instance r{};
            std::memcpy(r.transform, &lv.xf[0][0], sizeof(r.transform));
            std::memcpy(r.inv, &lv.inv[0][0], sizeof(r.inv));
            r.bvh = 1 + b;
            r.inner = -1;
            if (lv.animated) {
                r.animated = 1;
                put3(r.motion, lv.dir);
                r.time_bounds[0] = lv.tb.x;
                r.time_bounds[1] = lv.tb.y;
            }
            return r;
        };
        // the inner levels of nested wrappers follow every record a TLAS slot names
        uint32_t n_top_inst = 0;
        for (uint32_t i = 0; i < n_top; i++) n_top_inst += inst_of_slot[i] != UINT32_MAX;
        std::vector<pt_instance> level_records;
        for (uint32_t i = 0; i < n_top; i++) {
            if (inst_of_slot[i] != UINT32_MAX) {
                const Inst& in = inst[inst_of_slot[i]];
                pt_instance r = record(in.levels[0], in.blas);
                r.virt_base = virt;
                for (size_t k = 1; k < in.levels.size(); k++) {  // linked outermost first
                    const int32_t at = (int32_t)(n_top_inst + level_records.size());
                    (k == 1 ? r : level_records.back()).inner = at;
                    level_records.push_back(record(in.levels[k], in.blas));
                }
                virt += blas_count(blas[in.blas]);
                prims[i] = pt_prim{PT_PRIM_INSTANCE, (uint32_t)instances.size(), -1, -1, -1};
                instances.push_back(r);
            } else if (blas_of_slot[i] != UINT32_MAX) {
                prims[i] = pt_prim{PT_PRIM_BLAS, 1 + blas_of_slot[i], -1, -1, -1};
            } else {
                geometric(*static_cast<const GeometricPrimitive*>(top[i].get()), i);
            }
        }
        instances.insert(instances.end(), level_records.begin(), level_records.end());
        own_clusters.reserve(blas.size());
        for (size_t k = 0; k < blas.size(); k++) {
            pt_bvh_desc d{};
            if (blas[k].gp) {
                geometric(*blas[k].gp, base[k]);
                const AABB bb = PT_GET(*blas[k].gp, GpShape)->BoundingBox();
                const float box[6] = {bb.min.x, bb.min.y, bb.min.z, bb.max.x, bb.max.y, bb.max.z};
                own_clusters.emplace_back(1);
                uint32_t nc = 0, order = 0;
                float bbox[6];
                check(pt_bvh4_build(box, 1, own_clusters.back().data(), &nc, &d.root, &order, bbox), "pt_bvh4_build");
                d.clusters = own_clusters.back().data();
                d.n_clusters = nc;
                d.n_prims = 1;
            } else {
                const auto& bp = PT_GET(*static_cast<const BLASBase*>(blas[k].b), BlasPrims);
                for (size_t j = 0; j < bp.size(); j++) geometric(bp[j], base[k] + (uint32_t)j);
                const auto& bn = PT_GET(*blas[k].b, BlasNodes);
                d.clusters = reinterpret_cast<const pt_ref_bvh4_cluster*>(bn.data());
                d.n_clusters = (uint32_t)bn.size();
                std::memcpy(&d.root, &PT_GET(*blas[k].b, BlasRoot), sizeof(d.root));
                d.n_prims = (uint32_t)bp.size();
            }
            d.prim_base = base[k];
            bvhs.push_back(d);
        }
        // lights: Scene::GetLights() order, then lights only the sampler holds
        std::vector<std::shared_ptr<Light>> all = scene.GetLights();
        const std::vector<std::shared_ptr<Light>>* sl = nullptr;
        if (ls) {
            if (auto* u = dynamic_cast<UniformLightSampler*>(ls.get())) {
                sl = &PT_GET(*u, UlsLights);
                light_sampler = PT_LS_UNIFORM;
            } else if (auto* pw = dynamic_cast<PowerLightSampler*>(ls.get())) {
                sl = &PT_GET(*pw, PlsLights);
                light_sampler = PT_LS_POWER;
            } else {
                throw std::runtime_error("HipPathIntegrator: unsupported LightSampler");
            }
            for (const auto& l : *sl)
                if (std::find(all.begin(), all.end(), l) == all.end()) all.push_back(l);
        }
        std::unordered_map<const Light*, uint32_t> lid;
        auto area = [&](pt_light& r, const Light* inner, int32_t instance) {
            auto* a = dynamic_cast<const AreaLight*>(inner);
            if (!a) throw std::runtime_error("HipPathIntegrator: only area lights inside an instance");
            auto it = light_slot.find(a);
            if (it == light_slot.end()) throw std::runtime_error("HipPathIntegrator: area light without a primitive");
            r.kind = PT_LIGHT_AREA;
            r.prim = it->second;
            r.tex = texture(PT_GET(*a, AreaTex));
            r.one_sided = PT_GET(*a, AreaOneSided) ? 1u : 0u;
            r.instance = instance;
            return it->second;
        };
        // a TransformedLight / AnimatedLight, possibly wrapping another (a nested
        // wrapper's light): its AreaLight and the instance its chain of matrices names
        struct Unwrapped {
            const Light* area;
            int32_t instance;
        };
        auto unwrap = [&](const Light* l) {
            std::string key;
            for (;;) {
                if (auto* t = dynamic_cast<const TransformedLight*>(l)) {
                    key += mat_key(PT_GET(*t, TlXf));
                    l = PT_GET(*t, TlLight).get();
                } else if (auto* an = dynamic_cast<const AnimatedLight*>(l)) {
                    // AnimatedLight (Light.cpp:338-364): the light of the
                    // AnimatedPrimitive whose time-0 matrix this is; the device
                    // moves it with that instance at each ray's time
                    const glm::vec2 tb = PT_GET(*an, AlTb);
                    const float tt = glm::clamp(0.0f - tb.x, tb.x, tb.y) / (tb.y - tb.x);
                    key += mat_key(glm::translate(glm::mat4(1), PT_GET(*an, AlDir) * tt));
                    l = PT_GET(*an, AlLight).get();
                } else {
                    break;
                }
            }
            auto it = inst_light.find({l, key});
            if (it == inst_light.end()) throw std::runtime_error("HipPathIntegrator: light of an unknown instance");
            return Unwrapped{l, it->second};
        };
        for (const auto& l : all) {
            pt_light r{};
            r.prim = r.tex = -1;
            r.instance = -1;
            r.power = l->Power();
            r.pmf = ls ? ls->PMF(l) : 0.0f;
            if (dynamic_cast<const TransformedLight*>(l.get()) || dynamic_cast<const AnimatedLight*>(l.get())) {
                const Unwrapped u = unwrap(l.get());
                area(r, u.area, u.instance);
            } else if (auto* a = dynamic_cast<const AreaLight*>(l.get())) {
                auto it = light_slot.find(a);
                if (it == light_slot.end()) throw std::runtime_error("HipPathIntegrator: area light without a primitive");
                r.kind = PT_LIGHT_AREA;
                r.prim = it->second;
                r.tex = texture(PT_GET(*a, AreaTex));
                r.one_sided = PT_GET(*a, AreaOneSided) ? 1u : 0u;
                prims[it->second].light = (int32_t)lights.size();
            } else if (auto* u = dynamic_cast<const UniformInfiniteLight*>(l.get())) {
                r.kind = PT_LIGHT_UNIFORM_INF;
                put3(r.color, PT_GET(*u, UniColor));
            } else if (auto* f = dynamic_cast<const FunctionInfiniteLight*>(l.get())) {
                const auto* g = PT_GET(*f, FunFn).target<pt::SkyGradient>();
                if (!g) throw std::runtime_error("HipPathIntegrator: FunctionInfiniteLight needs a pt::SkyGradient");
                r.kind = PT_LIGHT_SKY_INF;
                put3(r.color, g->horizon);
                put3(r.vec, g->zenith);
                r.scale = g->scale;
            } else if (auto* ti = dynamic_cast<const TextureInfiniteLight*>(l.get())) {
                // the reference's own PreProcess result: its cell running sums
                const auto& acc = PT_GET(*ti, TexInfAcc);
                if (acc.size() != (size_t)PT_TEXINF_X * PT_TEXINF_Y)
                    throw std::runtime_error("HipPathIntegrator: TextureInfiniteLight before PreProcess");
                r.kind = PT_LIGHT_TEX_INF;
                r.tex = texture(PT_GET(*ti, TexInfTex));
                r.scale = PT_GET(*ti, TexInfScale);
                r.prim = (int32_t)light_dist.size();
                light_dist.insert(light_dist.end(), acc.begin(), acc.end());
            } else if (auto* d = dynamic_cast<const DistantLight*>(l.get())) {
                r.kind = PT_LIGHT_DISTANT;
                put3(r.color, PT_GET(*d, DistColor));
                put3(r.vec, PT_GET(*d, DistDir));
            } else if (auto* p = dynamic_cast<const PointLight*>(l.get())) {
                r.kind = PT_LIGHT_POINT;
                put3(r.color, PT_GET(*p, PointColor));
                put3(r.vec, PT_GET(*p, PointP));
            } else {
                throw std::runtime_error("HipPathIntegrator: unsupported light type");
            }
            lid[l.get()] = (uint32_t)lights.size();
            lights.push_back(r);
        }
        // the inner AreaLight of an emitter inside an instance: what a path
        // that hits it sees (interaction.AreaLight, Primitive.cpp:58)
        for (const auto& l : inner_lights) {
            if (lid.count(l.get())) continue;
            pt_light r{};
            r.power = l->Power();
            r.pmf = ls ? ls->PMF(l) : 0.0f;
            prims[area(r, l.get(), -1)].light = (int32_t)lights.size();
            lid[l.get()] = (uint32_t)lights.size();
            lights.push_back(r);
        }
        if (sl)
            for (const auto& l : *sl) sampler_lights.push_back(lid.at(l.get()));
        for (const auto& l : scene.infiniteLights) infinite_lights.push_back(lid.at(l.get()));
    }

    pt_scene_desc desc() const {
        pt_scene_desc d{};
        d.positions = positions.data();
        d.normals = normals.data();
        d.uvs = uvs.data();
        d.tangents = tangents.data();
        d.n_vertices = (uint32_t)(positions.size() / 3);
        d.tri_vidx = tri_vidx.data();
        d.tri_flags = tri_flags.data();
        d.n_triangles = (uint32_t)tri_flags.size();
        d.quads = quads.data();
        d.n_quads = (uint32_t)quads.size();
        d.spheres = spheres.data();
        d.n_spheres = (uint32_t)spheres.size();
        d.prims = prims.data();
        d.n_prims = (uint32_t)prims.size();
        d.bvhs = bvhs.data();
        d.n_bvhs = (uint32_t)bvhs.size();
        d.materials = materials.data();
        d.n_materials = (uint32_t)materials.size();
        d.textures = textures.data();
        d.n_textures = (uint32_t)textures.size();
        d.images = images.data();
        d.n_images = (uint32_t)images.size();
        d.texels = texels.data();
        d.n_texel_bytes = texels.size();
        d.lights = lights.data();
        d.n_lights = (uint32_t)lights.size();
        d.light_sampler = light_sampler;
        d.sampler_lights = sampler_lights.data();
        d.n_sampler_lights = (uint32_t)sampler_lights.size();
        d.infinite_lights = infinite_lights.data();
        d.n_infinite_lights = (uint32_t)infinite_lights.size();
        d.light_dist = light_dist.data();
        d.n_light_dist = light_dist.size();
        d.media = media.data();
        d.n_media = (uint32_t)media.size();
        d.scene_medium = scene_medium;
        d.instances = instances.data();
        d.n_instances = (uint32_t)instances.size();
        return d;
    }
};

pt_camera_desc camera_desc(const Camera& cam, const Flat& flat) {
    pt_camera_desc c{};
    put3(c.origin, PT_GET(cam, CamFrom));
    put3(c.u, PT_GET(cam, CamU));
    put3(c.v, PT_GET(cam, CamV));
    put3(c.w, PT_GET(cam, CamW));
    c.half_width = PT_GET(cam, CamHW);
    c.half_height = PT_GET(cam, CamHH);
    c.defocus_radius = PT_GET(cam, CamDefocus);
    c.focus_distance = PT_GET(cam, CamFocusDist);
    c.focus_angle = PT_GET(cam, CamFocusAngle);
    // rays carry time = glm::mix(shutterStart, shutterEnd, u) (Camera.hpp:25).
    // Only the shutter ctor (Camera.hpp:16-19) sets those bounds; the others
    // leave them uninitialised, and a ray's time matters only to
    // AnimatedPrimitive / AnimatedLight.  So a scene without them renders at
    // time 0, whatever the camera (the same images: no primitive or light
    // depends on it; the Python front end does the same), and a scene with
    // them takes the camera's bounds, which must then be finite.
    bool motion = false;
    for (const pt_instance& r : flat.instances) motion = motion || r.animated;
    c.has_shutter = motion ? 1 : 0;
    if (motion) {
        c.shutter[0] = PT_GET(cam, CamShutterStart);
        c.shutter[1] = PT_GET(cam, CamShutterEnd);
        if (!std::isfinite(c.shutter[0]) || !std::isfinite(c.shutter[1]))
            throw std::runtime_error("HipIntegrator: a scene with an AnimatedPrimitive needs a camera built with "
                                     "shutter bounds (Camera.hpp:16-19)");
    }
    glm::ivec2 res = cam.GetFilm()->Resolution();
    c.width = res.x;
    c.height = res.y;
    const auto m = cam.GetMedium();
    if (m && !flat.med_ids.count(m.get()))
        throw std::runtime_error("HipVolPathIntegrator: the camera's medium must be one the scene uses");
    c.medium = m ? flat.med_ids.at(m.get()) : -1;
    return c;
}

void filter_desc(const Film& film, pt_render_desc& rd) {
    const auto& f = PT_GET(film, FilmFilter);
    glm::vec2 r = f->Radius();
    rd.filter_radius[0] = r.x;
    rd.filter_radius[1] = r.y;
    if (auto* m = dynamic_cast<const MitchellFilter*>(f.get())) {
        rd.filter = PT_FILTER_MITCHELL;
        rd.filter_params[0] = PT_GET(*m, MitB);
        rd.filter_params[1] = PT_GET(*m, MitC);
    } else if (dynamic_cast<const BoxFilter*>(f.get())) {
        rd.filter = PT_FILTER_BOX;
    } else if (auto* g = dynamic_cast<const GaussianFilter*>(f.get())) {
        rd.filter = PT_FILTER_GAUSSIAN;
        rd.filter_params[0] = PT_GET(*g, GaussSigma);
    } else if (auto* l = dynamic_cast<const LanczosFilter*>(f.get())) {
        // WindowedSinc x WindowedSinc (Filter.hpp:114-144); the integral is the
        // object's own estimate (unseeded jitter: one value per call, as the
        // reference's FilmTile takes one per tile, Film.hpp:59)
        rd.filter = PT_FILTER_LANCZOS;
        rd.filter_params[0] = PT_GET(*l, LanczosTau);
        rd.filter_params[1] = f->Integral();
    } else {
        throw std::runtime_error("HipPathIntegrator: unsupported film filter");
    }
}

}  // namespace

namespace pt {

// ---------------------------------------------------------------------------
static inline uint32_t pcg_hash(uint32_t v) {
    uint32_t state = v * 747796405u + 2891336453u;
    uint32_t word = ((state >> ((state >> 28u) + 4u)) ^ state) * 277803737u;
    return (word >> 22u) ^ word;
}
void PCGSampler::StartPixelSample(const glm::ivec2& p, int index) {
    key_ = pcg_hash(pcg_hash(seed_ ^ pcg_hash((uint32_t)(p.y * width_ + p.x))) + (uint32_t)index);
    dim_ = 0;
}
float PCGSampler::next() { return (float)(pcg_hash(key_ + 0x9E3779B9u * dim_++) >> 8) * (1.0f / 16777216.0f); }
glm::dvec2 PCGSampler::get2D() {
    double a = next();
    double b = next();
    return {a, b};
}
std::array<glm::vec2, 4> PCGSampler::get2Dx4f() {
    std::array<glm::vec2, 4> r;
    for (auto& v : r) {
        float a = next();
        float b = next();
        v = {a, b};
    }
    return r;
}

// ---------------------------------------------------------------------------
class HipBackend {
public:
    Flat flat;
    pt_ctx* ctx = nullptr;  // one context over the frame's GPUs (pt_create(ctx, n, ids))
    // fallback when RCCL refuses the multi-device context (PT_ERR_COMM): one
    // context per GPU, the films summed on the host like Film::Merge
    std::vector<pt_ctx*> singles;
    RenderStats stats;
    std::vector<double> last;  // the reduced accumulation of the last frame
    std::vector<uint32_t> counts;  // samples per pixel of the last frame

    ~HipBackend() { release(); }

    void release() {
        pt_destroy(ctx);
        ctx = nullptr;
        for (pt_ctx* c : singles) pt_destroy(c);
        singles.clear();
    }
    int devices_in_use() const { return ctx ? pt_device_count(ctx) : (int)singles.size(); }

    // The scene is flattened once; the context (and its RCCL communicators)
    // is rebuilt when the requested GPU count changes.
    void ensure(const Scene& scene, const std::shared_ptr<LightSampler>& ls, unsigned n,
                const std::shared_ptr<Medium>& camera_medium = nullptr) {
        if (!flat_built) {
            flat.build(scene, ls);
            flat.medium(camera_medium);
            flat_built = true;
        }
        int devices = 0;
        if (hipcount(&devices) != 0 || devices <= 0) throw std::runtime_error("HipPathIntegrator: no HIP device");
        int want = (int)std::max(1u, std::min<unsigned>(n, (unsigned)devices));
        // PT_FORCE_HOST_MERGE=k (tests on a one-GPU box): the fallback below
        // with k contexts, on GPUs g % devices
        const char* fm = getenv("PT_FORCE_HOST_MERGE");
        const int force = fm ? atoi(fm) : 0;
        if (force > 0) want = force;
        if ((ctx || !singles.empty()) && devices_in_use() == want) return;
        release();
        const pt_scene_desc d = flat.desc();
        const pt_status st = force > 0 ? PT_ERR_COMM : pt_create(&ctx, want, nullptr);
        if (st == PT_ERR_COMM && (want > 1 || force > 0) && !getenv("PT_NO_HOST_MERGE")) {
            // RCCL could not join the GPUs: per-GPU contexts, host merge
            ctx = nullptr;
            for (int g = 0; g < want; g++) {
                pt_ctx* c = nullptr;
                const int id = g % devices;
                check(pt_create(&c, 1, &id), "pt_create");
                singles.push_back(c);
                check(pt_scene_upload(c, &d), "pt_scene_upload", c);
            }
            return;
        }
        check(st, "pt_create");
        check(pt_scene_upload(ctx, &d), "pt_scene_upload", ctx);
    }

    // One pt_render over the context's GPUs: the library shards the frame
    // (interleaved samples at fixed SPP, 32x32 tiles when adaptive), renders
    // one host thread per GPU and reduces the per-GPU films with ncclReduce
    // onto the first GPU; the result is merged into the Film once
    // (Film::Merge, Film.hpp:125-132).
    void render(const Camera& cam, uint32_t integrator, uint32_t spp, uint32_t depth, uint32_t seed, bool adaptive,
                std::array<uint32_t, 2> strata = {0u, 0u}) {
        const pt_camera_desc cd = camera_desc(cam, flat);
        const auto film = cam.GetFilm();
        const glm::ivec2 res = film->Resolution();
        const size_t npx = (size_t)res.x * res.y;
        pt_render_desc rd{};
        rd.integrator = integrator;
        rd.spp = spp;
        rd.max_depth = depth;
        rd.seed = seed;
        filter_desc(*film, rd);
        rd.shard_count = 1;
        rd.strata[0] = strata[0];
        rd.strata[1] = strata[1];
        last.assign(4 * npx, 0.0);
        pt_stats st{};
        auto t0 = std::chrono::steady_clock::now();
        if (!singles.empty()) {
            render_singles(cd, rd, npx, adaptive, st);
        } else if (adaptive) {
            counts.assign(npx, 0u);
            check(pt_render_adaptive(ctx, &cd, &rd, last.data(), counts.data(), &st), "pt_render_adaptive", ctx);
        } else {
            counts.assign(npx, spp);
            check(pt_render(ctx, &cd, &rd, last.data(), &st), "pt_render", ctx);
        }
        // {sum RGB*w, sum w} per pixel into the Film (Film.hpp:118-132)
        FilmTile tile = film->GetFilmTile(Bounds2i{{0, 0}, res});
        for (int y = 0; y < res.y; y++)
            for (int x = 0; x < res.x; x++) {
                FilmTilePixel& px = tile.At({x, y});
                const size_t i = 4 * ((size_t)y * res.x + x);
                px.RGB = glm::dvec3(last[i], last[i + 1], last[i + 2]);
                px.weight = last[i + 3];
            }
        film->Merge(tile);
        stats = RenderStats{};
        stats.paths = st.paths;
        stats.rays_closest = st.rays_closest;
        stats.rays_any = st.rays_any;
        stats.devices = st.n_devices;
        stats.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }

private:
    bool flat_built = false;
    static int hipcount(int* n);

    // The per-GPU fallback: GPU g renders shard g of n (interleaved samples at
    // fixed SPP, 32x32 tiles when adaptive) on its own host thread into its
    // own host film; the films and sample counts are summed here.
    void render_singles(const pt_camera_desc& cd, const pt_render_desc& rd0, size_t npx, bool adaptive,
                        pt_stats& total) {
        const uint32_t n = (uint32_t)singles.size();
        std::vector<std::vector<double>> films(n, std::vector<double>(4 * npx, 0.0));
        std::vector<std::vector<uint32_t>> cnts(n, std::vector<uint32_t>(adaptive ? npx : 0, 0u));
        std::vector<pt_stats> st(n);
        std::vector<pt_status> res(n, PT_OK);
        std::vector<std::thread> th;
        for (uint32_t g = 0; g < n; g++)
            th.emplace_back([&, g] {
                pt_render_desc rd = rd0;
                rd.shard_index = g;
                rd.shard_count = n;
                res[g] = adaptive ? pt_render_adaptive(singles[g], &cd, &rd, films[g].data(), cnts[g].data(), &st[g])
                                  : pt_render(singles[g], &cd, &rd, films[g].data(), &st[g]);
            });
        for (auto& t : th) t.join();
        for (uint32_t g = 0; g < n; g++) check(res[g], adaptive ? "pt_render_adaptive" : "pt_render", singles[g]);
        counts.assign(npx, adaptive ? 0u : rd0.spp);
        for (uint32_t g = 0; g < n; g++) {
            for (size_t i = 0; i < 4 * npx; i++) last[i] += films[g][i];
            if (adaptive)
                for (size_t i = 0; i < npx; i++) counts[i] += cnts[g][i];
            total.paths += st[g].paths;
            total.rays_closest += st[g].rays_closest;
            total.rays_any += st[g].rays_any;
        }
        total.n_devices = n;
    }
};

}  // namespace pt

#include <hip/hip_runtime_api.h>
int pt::HipBackend::hipcount(int* n) { return hipGetDeviceCount(n) == hipSuccess ? 0 : -1; }

namespace pt {

static uint32_t seed_of(const std::shared_ptr<Sampler>& s) {
    if (auto* p = dynamic_cast<const PCGSampler*>(s.get())) return p->Seed();
    return 0x5EED0001u;
}
// the camera strata of a StratifiedSampler host (Sampler.hpp:73-151), or of a
// PCGSampler given strata; {0, 0}: the plain stream
static std::array<uint32_t, 2> strata_of(const std::shared_ptr<Sampler>& s) {
    if (auto* st = dynamic_cast<const StratifiedSampler*>(s.get())) return {PT_GET(*st, StratX), PT_GET(*st, StratY)};
    if (auto* p = dynamic_cast<const PCGSampler*>(s.get())) return {p->StrataX(), p->StrataY()};
    return {0u, 0u};
}

HipPathIntegrator::HipPathIntegrator(const std::shared_ptr<Scene>& scene, const std::shared_ptr<Camera>& camera,
                                     const std::shared_ptr<Sampler>& sampler,
                                     const std::shared_ptr<LightSampler>& lightSampler, uint32_t maxDepth)
    : PathIntegrator(scene, camera, sampler, lightSampler, maxDepth), ls_(lightSampler), depth_(maxDepth) {}
HipPathIntegrator::~HipPathIntegrator() = default;

void HipPathIntegrator::Render(unsigned int n) const {
    std::lock_guard<std::mutex> lk(mu_);
    if (!be_) be_ = std::make_unique<HipBackend>();
    be_->ensure(*scene, ls_, n);
    be_->render(*camera, PT_INTEGRATOR_PATH, sampler->SamplesPerPixel(), depth_, seed_of(sampler),
                adaptive_, strata_of(sampler));
}
RenderStats HipPathIntegrator::LastStats() const { return be_ ? be_->stats : RenderStats{}; }
static const std::vector<double> kEmpty;
const std::vector<double>& HipPathIntegrator::LastAccumulation() const { return be_ ? be_->last : kEmpty; }

HipSimplePathIntegrator::HipSimplePathIntegrator(const std::shared_ptr<Scene>& scene,
                                                 const std::shared_ptr<Camera>& camera,
                                                 const std::shared_ptr<Sampler>& sampler, uint32_t maxDepth)
    : SimplePathIntegrator(scene, camera, sampler, maxDepth), depth_(maxDepth) {}
HipSimplePathIntegrator::~HipSimplePathIntegrator() = default;

void HipSimplePathIntegrator::Render(unsigned int n) const {
    std::lock_guard<std::mutex> lk(mu_);
    if (!be_) be_ = std::make_unique<HipBackend>();
    be_->ensure(*scene, nullptr, n);
    be_->render(*camera, PT_INTEGRATOR_SIMPLE, sampler->SamplesPerPixel(), depth_, seed_of(sampler),
                adaptive_, strata_of(sampler));
}
RenderStats HipSimplePathIntegrator::LastStats() const { return be_ ? be_->stats : RenderStats{}; }

HipVolPathIntegrator::HipVolPathIntegrator(const std::shared_ptr<Scene>& scene, const std::shared_ptr<Camera>& camera,
                                           const std::shared_ptr<Sampler>& sampler,
                                           const std::shared_ptr<LightSampler>& lightSampler, uint32_t maxDepth)
    : VolPathIntegrator(scene, camera, sampler, lightSampler, maxDepth), ls_(lightSampler), depth_(maxDepth) {}
HipVolPathIntegrator::~HipVolPathIntegrator() = default;

void HipVolPathIntegrator::Render(unsigned int n) const {
    std::lock_guard<std::mutex> lk(mu_);
    if (!be_) be_ = std::make_unique<HipBackend>();
    be_->ensure(*scene, ls_, n, camera->GetMedium());
    be_->render(*camera, PT_INTEGRATOR_VOLPATH, sampler->SamplesPerPixel(), depth_, seed_of(sampler),
                adaptive_, strata_of(sampler));
}
RenderStats HipVolPathIntegrator::LastStats() const { return be_ ? be_->stats : RenderStats{}; }
const std::vector<double>& HipVolPathIntegrator::LastAccumulation() const { return be_ ? be_->last : kEmpty; }
const std::vector<double>& HipSimplePathIntegrator::LastAccumulation() const { return be_ ? be_->last : kEmpty; }
static const std::vector<uint32_t> kNoCounts;
const std::vector<uint32_t>& HipPathIntegrator::LastSampleCounts() const { return be_ ? be_->counts : kNoCounts; }
const std::vector<uint32_t>& HipSimplePathIntegrator::LastSampleCounts() const { return be_ ? be_->counts : kNoCounts; }
const std::vector<uint32_t>& HipVolPathIntegrator::LastSampleCounts() const { return be_ ? be_->counts : kNoCounts; }

}  // namespace pt
