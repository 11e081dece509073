// TEST INFRASTRUCTURE ONLY — never part of the product path.
//
// The reference's own Model class (Model.hpp) without Assimp, so the
// harness's scenes can hold what every main.cpp scene holds: a
// ResourceManager::CacheModel<BLAS4>(...) result in the TLAS (main.cpp:290)
// or inside a TransformedPrimitive (main.cpp:376, 483).  Model.cpp -- its
// only non-inline code: the Assimp loader behind Model::Model(path) and
// GetMeshes -- is out of scope (the submodule is empty); this
// unit defines those two members loader-free: the "file" at `path` is a list
// of meshes the harness registered under that name.  Everything else runs as
// the reference wrote it: ResourceManager::CacheModel, Model::BuildBlas<BLAS4>
// (one GeometricPrimitive per triangle, an AreaLight per emissive one, culled
// at Power() <= FLT_EPSILON), BLAS4's build, Model::Intersect / IntersectPred
// / GetLights.  Compiled with the reference's flags by oracle/Makefile into
// ref_harness and hip_harness only.
#include "ref_model.hpp"

#include <cstdio>
#include <cstdlib>
#include <map>
#include <unordered_map>

#include "Model.hpp"
#include "ResourceManager.hpp"

namespace {
std::map<std::string, std::vector<std::shared_ptr<Mesh>>>& registry() {
    static std::map<std::string, std::vector<std::shared_ptr<Mesh>>> r;
    return r;
}
// private members reached through member pointers formed by explicit
// template instantiation (as the harness and the drop-in do)
template <class Tag, typename Tag::type M>
struct ModelMember {
    friend typename Tag::type get(Tag) { return M; }
};
#define M_MEMBER(NAME, CLASS, TYPE, FIELD) \
    struct NAME {                          \
        using type = TYPE CLASS::*;        \
        friend type get(NAME);             \
    };                                     \
    template struct ModelMember<NAME, &CLASS::FIELD>
M_MEMBER(MModelBvh, Model, std::shared_ptr<BVHBase<GeometricPrimitive>>, model_bvh);
M_MEMBER(MGeoShape, GeometricPrimitive, std::shared_ptr<Shape>, shape);
}  // namespace

// Model.cpp:16-20 loads `path` with Assimp into `meshes`; here the path names
// a registered mesh list
Model::Model(const std::string& path) {
    auto it = registry().find(path);
    if (it == registry().end()) {
        fprintf(stderr, "harness Model: no meshes registered as %s\n", path.c_str());
        exit(2);
    }
    meshes = it->second;
    model_path = path;
}

std::vector<std::shared_ptr<Mesh>> Model::GetMeshes() const { return meshes; }

HarnessModel pt_harness_model(const std::string& name, const std::vector<std::shared_ptr<Mesh>>& meshes,
                              bool override_mat, const std::shared_ptr<Material>& material,
                              const std::shared_ptr<Medium>& medium) {
    registry()[name] = meshes;
    std::shared_ptr<Model> m =
        override_mat ? ResourceManager::get_instance().CacheModel<BLAS4>(name, name, material, medium)
                     : ResourceManager::get_instance().CacheModel<BLAS4>(name, name);
    HarnessModel h;
    h.model = m;
    const std::shared_ptr<BVHBase<GeometricPrimitive>>& bvh = (*m).*get(MModelBvh{});
    auto* b4 = dynamic_cast<BLAS4*>(bvh.get());
    if (!b4) {
        fprintf(stderr, "harness Model %s: not a BLAS4\n", name.c_str());
        exit(2);
    }
    h.blas = std::shared_ptr<PeekBLAS>(bvh, static_cast<PeekBLAS*>(b4));  // (Peek adds no members)
    // the AreaLights BuildBlas made, named by their triangle: a primitive's
    // shape aliases mesh->GetShape(j) (Model.hpp:49)
    std::unordered_map<const Shape*, int> tri_of;
    int tri = 0;
    for (const auto& me : meshes)
        for (uint32_t j = 0; j < me->GetTriangleCount(); j++, tri++) tri_of[me->GetShape(j)] = tri;
    for (const GeometricPrimitive& p : h.blas->Prims()) {
        const auto lights = p.GetLights();
        if (lights.empty()) continue;
        const Shape* sh = (p.*get(MGeoShape{})).get();
        auto it = tri_of.find(sh);
        if (it == tri_of.end()) {
            fprintf(stderr, "harness Model %s: a light on an unknown triangle\n", name.c_str());
            exit(2);
        }
        h.lights.push_back({lights[0].get(), it->second});
    }
    return h;
}
