// TEST INFRASTRUCTURE ONLY — never part of the product path.
// Expose protected BVH4 arrays (BVH.hpp:1214-1216, 392-394) — API use only.
#pragma once
#include <memory>
#include <vector>

#include "BVH.hpp"
#include "Primitive.hpp"

template <class T>
struct Peek : BVH4<T> {
    using BVH4<T>::BVH4;
    const std::vector<BVH4_CLUSTER>& Nodes() const { return this->nodes; }
    BVH4_NODE Root() const { return this->rootNode; }
    const std::vector<T>& Prims() const { return this->primitives; }
};
using PeekTLAS = Peek<std::shared_ptr<Primitive>>;
using PeekBLAS = Peek<GeometricPrimitive>;
