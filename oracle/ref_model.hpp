// TEST INFRASTRUCTURE ONLY — never part of the product path.
// The reference's own Model (Model.hpp) in the harness's "refmodels" recipes:
// see ref_model.cpp.
#pragma once
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "Light.hpp"
#include "Material.hpp"
#include "Medium.hpp"
#include "Mesh.hpp"
#include "ref_peek.hpp"

struct HarnessModel {
    std::shared_ptr<Primitive> model;  // the Model ResourceManager::CacheModel<BLAS4> returned
    std::shared_ptr<PeekBLAS> blas;    // its own BLAS4 (Model::model_bvh), read through Peek
    // its AreaLights (BuildBlas made them), each with its model-local
    // triangle index (meshes in order, triangles in mesh order)
    std::vector<std::pair<const Light*, int>> lights;
};

// ResourceManager::get_instance().CacheModel<BLAS4>(name, name) -- or, with
// override_mat, CacheModel<BLAS4>(name, name, material, medium), the
// BuildBlas(material, medium) form (Model.hpp:62-80, main.cpp:376) -- over a
// Model whose meshes are `meshes`.
HarnessModel pt_harness_model(const std::string& name, const std::vector<std::shared_ptr<Mesh>>& meshes,
                              bool override_mat, const std::shared_ptr<Material>& material,
                              const std::shared_ptr<Medium>& medium);
