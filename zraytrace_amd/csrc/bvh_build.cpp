// bvh_build.cpp — host BVH build for the HIP path.
//
// Produces the same tree as bvh.zig:62-185 (BVHNode.init -> divide ->
// optimal_axis_divide -> make_axis_divide):
//   * n == 1: a leaf with the primitive on both sides      (bvh.zig:132-136)
//   * n == 2: a leaf (left = s[1], right = s[0])            (bvh.zig:138-143)
//   * else: for axis 0..2, for split in {n/2} (n < 4) or {n/4, n/2, n/4+n/2}:
//       stable-sort the slice IN PLACE by AABB midpoint on that axis, score
//       (pseudoSA(right) + pseudoSA(left)) / pseudoSA(all), keep strictly
//       better; finally re-sort by the best axis starting from the order the
//       last trial left (bvh.zig:85-120).
//   pseudoSA(box) = 2 * (dx^2 + dy^2 + dz^2)                (aabb.zig:99-105)
//   node box = initAabb(left, right)                        (bvh.zig:164)
// std.sort.sort is a stable sort, so any stable sort with the same strict
// comparator yields the identical permutation.  Two consequences used here:
// re-sorting a slice on the axis it is already sorted on changes nothing, so
// each axis is sorted once (not once per split trial); and a stable LSD radix
// sort on order-preserving u32 images of the keys (-0 mapped to +0, which the
// comparator treats as equal) is the same permutation in O(n).  NaN keys (no
// strict weak order) fall back to std::stable_sort.
//
// Unlike the reference (one heap Surface per node, pointer chasing), nodes are
// emitted into a flat array in depth-first pre-order (left first), and the
// primitives are permuted into leaf order so that the device reads both
// arrays front-to-back as traversal descends.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "bvh_build.hpp"
#include "zrt.hpp"

namespace zrt {

inline float fmin_z(float x, float y) { return x < y ? x : y; }  // std.math.min
inline float fmax_z(float x, float y) { return x > y ? x : y; }  // std.math.max

// aabb.zig:37-41 initMinMax
Box box_min_max(const float c1[3], const float c2[3]) {
  Box b;
  for (int i = 0; i < 3; ++i) {
    b.mn[i] = fmin_z(c1[i], c2[i]);
    b.mx[i] = fmax_z(c1[i], c2[i]);
    b.mid[i] = (c1[i] + c2[i]) / 2.0f;
  }
  return b;
}
// aabb.zig:68-71 initAabb
Box box_union(const Box& a, const Box& b) {
  float mn[3], mx[3];
  for (int i = 0; i < 3; ++i) {
    mn[i] = fmin_z(a.mn[i], b.mn[i]);
    mx[i] = fmax_z(a.mx[i], b.mx[i]);
  }
  return box_min_max(mn, mx);
}
// aabb.zig:99-105
float pseudo_area(const Box& b) {
  const float dx = std::fabs(b.mn[0] - b.mx[0]);
  const float dy = std::fabs(b.mn[1] - b.mx[1]);
  const float dz = std::fabs(b.mn[2] - b.mx[2]);
  return 2.0f * (dx * dx + dy * dy + dz * dz);
}

Box prim_box(const zrt_prim& p) {
  if (p.kind == ZRT_PRIM_SPHERE) {  // sphere.zig:24-29
    const float r = p.radius;
    const float lo[3] = {p.center.x - r, p.center.y - r, p.center.z - r};
    const float hi[3] = {p.center.x + r, p.center.y + r, p.center.z + r};
    return box_min_max(lo, hi);
  }
  // triangle.zig:33 initAabb(initMinMax(a, b), initMinMax(a, c))
  const float a[3] = {p.a.x, p.a.y, p.a.z};
  const float b[3] = {p.b.x, p.b.y, p.b.z};
  const float c[3] = {p.c.x, p.c.y, p.c.z};
  return box_union(box_min_max(a, b), box_min_max(a, c));
}

uint32_t mid_key(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if (f == 0.0f) u = 0;  // -0 == +0 under `<`
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

namespace {

struct Builder {
  const std::vector<Box>& pbox;
  std::vector<uint32_t>& order;  // the slice being divided, permuted in place
  std::vector<BuildNode> nodes;
  uint32_t max_depth = 0;

  // bvh.zig:62-69 -> aabb.zig:73-81 (min/max over every box's min and max)
  Box range_box(size_t lo, size_t hi) const {
    float mn[3] = {INFINITY, INFINITY, INFINITY};
    float mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (size_t i = lo; i < hi; ++i) {
      const Box& b = pbox[order[i]];
      for (int k = 0; k < 3; ++k) {
        mn[k] = fmin_z(mn[k], b.mn[k]);
        mn[k] = fmin_z(mn[k], b.mx[k]);
        mx[k] = fmax_z(mx[k], b.mn[k]);
        mx[k] = fmax_z(mx[k], b.mx[k]);
      }
    }
    return box_min_max(mn, mx);
  }

  std::vector<uint32_t> key_a, key_b, idx_b;  // radix sort scratch

  void sort_axis(int axis, size_t lo, size_t hi) {
    const std::vector<Box>& pb = pbox;
    const size_t n = hi - lo;
    bool has_nan = false;
    for (size_t i = lo; i < hi && !has_nan; ++i) has_nan = std::isnan(pb[order[i]].mid[axis]);
    if (n < 64 || has_nan) {
      std::stable_sort(order.begin() + lo, order.begin() + hi,
                       [&pb, axis](uint32_t a, uint32_t b) { return pb[a].mid[axis] < pb[b].mid[axis]; });
      return;
    }
    key_a.resize(n);
    key_b.resize(n);
    idx_b.resize(n);
    uint32_t* idx_a = order.data() + lo;
    for (size_t i = 0; i < n; ++i) {
      key_a[i] = mid_key(pb[idx_a[i]].mid[axis]);
    }
    uint32_t *ka = key_a.data(), *kb = key_b.data(), *ia = idx_a, *ib = idx_b.data();
    for (int shift = 0; shift < 32; shift += 8) {
      size_t count[257] = {0};
      for (size_t i = 0; i < n; ++i) ++count[((ka[i] >> shift) & 0xffu) + 1];
      if (count[((ka[0] >> shift) & 0xffu) + 1] == n) continue;  // one digit value: pass is the identity
      for (int d = 0; d < 256; ++d) count[d + 1] += count[d];
      for (size_t i = 0; i < n; ++i) {
        const size_t at = count[(ka[i] >> shift) & 0xffu]++;
        kb[at] = ka[i];
        ib[at] = ia[i];
      }
      std::swap(ka, kb);
      std::swap(ia, ib);
    }
    if (ia != idx_a) std::memcpy(idx_a, ia, n * sizeof(uint32_t));
  }

  // bvh.zig:85-120
  size_t optimal_axis_divide(size_t lo, size_t hi) {
    const size_t n = hi - lo;
    int best_axis = 0;
    float best_ratio = INFINITY;
    size_t best_split = n / 2;
    const float total_area = pseudo_area(range_box(lo, hi));
    size_t splits[3] = {n / 2, 0, 0};
    int n_splits = 1;
    if (n >= 4) {
      splits[0] = n / 4;
      splits[1] = n / 2;
      splits[2] = n / 4 + n / 2;
      n_splits = 3;
    }
    for (int axis = 0; axis < 3; ++axis) {
      sort_axis(axis, lo, hi);  // (the reference sorts before every split; repeats are no-ops)
      for (int k = 0; k < n_splits; ++k) {
        const size_t split = splits[k];
        const float area = pseudo_area(range_box(lo + split, hi)) + pseudo_area(range_box(lo, lo + split));
        const float ratio = area / total_area;
        if (ratio < best_ratio) {
          best_ratio = ratio;
          best_axis = axis;
          best_split = split;
        }
      }
    }
    if (best_axis != 2) sort_axis(best_axis, lo, hi);  // from the z-sorted order, as the reference
    return best_split;
  }

  // bvh.zig:129-160, emitting pre-order; returns the node index and its box.
  int32_t divide(size_t lo, size_t hi, uint32_t depth, Box* out_box) {
    if (max_depth < depth) max_depth = depth;
    const size_t n = hi - lo;
    const int32_t me = int32_t(nodes.size());
    nodes.push_back(BuildNode{});
    Box lb, rb;
    int32_t l, r;
    if (n == 1) {
      l = r = -int32_t(order[lo]) - 1;
      lb = rb = pbox[order[lo]];
    } else if (n == 2) {
      l = -int32_t(order[lo + 1]) - 1;
      r = -int32_t(order[lo]) - 1;
      lb = pbox[order[lo + 1]];
      rb = pbox[order[lo]];
    } else {
      const size_t split = optimal_axis_divide(lo, hi);
      l = divide(lo, lo + split, depth + 1, &lb);
      r = divide(lo + split, hi, depth + 1, &rb);
    }
    const Box b = box_union(lb, rb);
    BuildNode& nd = nodes[size_t(me)];
    for (int k = 0; k < 3; ++k) {
      nd.mn[k] = b.mn[k];
      nd.mx[k] = b.mx[k];
    }
    nd.left = l;
    nd.right = r;
    *out_box = b;
    return me;
  }
};

}  // namespace

BuiltBvh build_bvh(const zrt_prim* prims, uint32_t n) {
  BuiltBvh out;
  if (n == 0) return out;
  std::vector<Box> pbox(n);
  for (uint32_t i = 0; i < n; ++i) pbox[i] = prim_box(prims[i]);
  std::vector<uint32_t> order(n);
  for (uint32_t i = 0; i < n; ++i) order[i] = i;
  Builder b{pbox, order, {}, 0};
  b.nodes.reserve(2 * size_t(n));
  Box root;
  b.divide(0, n, 1, &root);
  out.nodes = std::move(b.nodes);
  out.max_depth = b.max_depth;
  return out;
}

}  // namespace zrt

extern "C" int zrt_bvh_build(const zrt_scene* scene, zrt_bvh_node** out_nodes, uint32_t* n_nodes,
                             uint32_t* max_depth) {
  if (!scene || !out_nodes || !n_nodes) return zrt::fail(ZRT_E_INVALID, "null argument");
  *out_nodes = nullptr;
  *n_nodes = 0;
  if (scene->n_prims == 0 || !scene->prims) return zrt::fail(ZRT_E_INVALID, "empty scene");
  try {
    const zrt::BuiltBvh bvh = zrt::build_bvh(scene->prims, scene->n_prims);
    auto* nodes = static_cast<zrt_bvh_node*>(std::malloc(sizeof(zrt_bvh_node) * bvh.nodes.size()));
    if (!nodes) return zrt::fail(ZRT_E_NOMEM, "OutOfMemory");
    for (size_t i = 0; i < bvh.nodes.size(); ++i) {
      const zrt::BuildNode& s = bvh.nodes[i];
      nodes[i].min = {s.mn[0], s.mn[1], s.mn[2]};
      nodes[i].max = {s.mx[0], s.mx[1], s.mx[2]};
      nodes[i].left = s.left;
      nodes[i].right = s.right;
    }
    *out_nodes = nodes;
    *n_nodes = uint32_t(bvh.nodes.size());
    if (max_depth) *max_depth = bvh.max_depth;
    return ZRT_OK;
  } catch (const std::bad_alloc&) {
    return zrt::fail(ZRT_E_NOMEM, "OutOfMemory");
  }
}
