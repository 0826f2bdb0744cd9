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

// The device build of the same tree (bvh_gpu.hip): level by level, each
// segment's three stable axis sorts and the final re-sort as 64-bit (segment,
// key) radix sorts on `device`.  Returns false without touching *out when it
// does not apply (fewer than 3 primitives, NaN midpoints): use build_bvh.
bool build_bvh_device(const zrt_prim* prims, uint32_t n, int device, BuiltBvh* out);

// The build's arithmetic, shared by both builds (aabb.zig, sphere.zig:24-29,
// triangle.zig:33).
struct Box {
  float mn[3], mx[3], mid[3];
};
Box box_min_max(const float c1[3], const float c2[3]);  // aabb.zig:37-41 initMinMax
Box box_union(const Box& a, const Box& b);               // aabb.zig:68-71 initAabb
float pseudo_area(const Box& b);                         // aabb.zig:99-105
Box prim_box(const zrt_prim& p);
// Order-preserving u32 image of a midpoint (the comparator's `<`, -0 as +0);
// NaN has none (the builds check for it).
uint32_t mid_key(float f);

}  // namespace zrt
