// Binary-tree node of the device BVH build (pt_bvh_gpu.hip).  Not part of the
// C ABI of include/pt_api.h.
#pragma once
#include <stdint.h>

#include "pt_api.h"

// One node of the binary SAH tree of BVHBase::BuildBaseThreaded
// (BVH.hpp:290-390): leaf iff count != 0 (then right = first primitive),
// else left/right are node indices and axis the split axis.
struct PtBvh2Node {
    float mn[3], mx[3];
    uint32_t left, right, count, axis;
};  // 40 bytes
