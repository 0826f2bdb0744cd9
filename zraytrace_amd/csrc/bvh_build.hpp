// bvh_build.hpp — host BVH build (bvh.zig:62-185 topology) for the HIP path.
#pragma once
#include <cstdint>
#include <vector>

#include "../../include/zrt.h"

namespace zrt {

// Pre-order (left first) node; child >= 0: node index, child < 0: primitive
// (-child - 1) in reference list order.
struct BuildNode {
  float mn[3];
  int32_t left;
  float mx[3];
  int32_t right;
};

struct BuiltBvh {
  std::vector<BuildNode> nodes;  // node 0 = root
  uint32_t max_depth = 0;        // Tracking.max_depth (root = 1)
};

BuiltBvh build_bvh(const zrt_prim* prims, uint32_t n);

}  // namespace zrt
