// accel_build.hpp — wide SAH tree over the reference BVH's leaves (see accel_build.cpp).
#pragma once
#include <cstdint>
#include <vector>

namespace zrt {

struct float4v {  // host-side float4 (same layout as HIP's float4)
  float v[4];
};

// One reference leaf (bvh.zig:132-143): its exact box and its one or two
// primitives as render.hip primitive-slot refs (-(2*slot + kind) - 1).
struct RefLeaf {
  float mn[3], mx[3];
  int32_t prim_a, prim_b;
};

// The wide tree's encoding (WideBvh::layout), recorded by build_wide_bvh and
// compared with what the selected kernel decodes before any launch, on the host
// and again by the kernel itself (render.hip kKernelLayout): a kernel variant that
// did not decode biased sphere refs used them as primitive indices and faulted
// (VERDICT r03 #3).  A mismatch is ZRT_E_UNSUPPORTED, never a launch.
constexpr uint32_t kLayoutVersion = 1u << 8;      // 128-B nodes, inline leaves, refs as below
constexpr uint32_t kLayoutSphereSlots = 1u << 0;  // sphere leaf refs stored - kSphereSlotBias ...
constexpr uint32_t kLayoutSphereFirst = 1u << 1;  // ... in a node's first slots

struct WideBvh {
  std::vector<float4v> nodes;   // 8 per wide node, node 0 = root
  uint32_t n_nodes = 0, n_leaves = 0, depth = 0, max_stack = 0;
  uint32_t n_top = 0;           // nodes of the top levels, stored first (0 .. n_top-1)
  uint32_t layout = 0;          // kLayout* bits of this encoding
};

// A leaf slot holding a sphere stores its ref a minus kSphereSlotBias (below
// -2^30, where no other ref lies): render.hip opens such slots with the
// reference's loose test against t_max = +inf (DESIGN.md §3 "Spheres") and adds
// the bias back before testing the primitives.
constexpr int32_t kSphereSlotBias = int32_t(1) << 30;

// top_levels: how many levels (root = 1) are stored first, breadth-first.
// inflate: inner children's boxes are stored grown on every side by this much
// times their own largest |coordinate| (rounded outward); leaf children keep
// the reference leaf's box bit for bit.
// sphere_grow: inner children whose subtree holds a sphere are grown by this
// much more (absolute): the rounded sphere test's reach beyond the sphere.
// mark_spheres: leaf slots holding a sphere carry ref a - kSphereSlotBias (the
// kernel must then be built to decode them: render.hip ZRT_SPHERE_SLOTS).
WideBvh build_wide_bvh(const std::vector<RefLeaf>& leaves, uint32_t top_levels = 2, float inflate = 0.0f,
                       float sphere_grow = 0.0f, bool mark_spheres = false);

// primitive-slot ref of render.hip, -(2*slot + kind) - 1: kind 0 is a sphere
inline bool ref_is_sphere(int32_t ref) { return ref < 0 && ((-(int64_t(ref) + 1)) & 1) == 0; }

}  // namespace zrt
