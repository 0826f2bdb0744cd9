// accel_build.cpp — a wide (4-ary) SAH tree over the reference's BVH leaves.
//
// Why this is exact.  The reference finds the closest hit by a left-first
// recursion (bvh.zig:187-205) whose node test is aabb.zig:109-127: every axis
// checked on its own against [t_min, t_max].  That test is monotone under box
// containment: node boxes are exact min/max unions of their children
// (bvh.zig:164), f32 rounding of (bound - origin) * (1/d) is monotone in the
// bound, so if a leaf's box passes, every ancestor's box passes for the same
// t_max (and the reference's t_max at an ancestor is never smaller than at the
// leaf).  Hence the primitives the reference can return are exactly those in
// leaves whose own box passes the loose test, and its answer is the minimum t
// with ties to the earliest leaf in its DFS order.
//
// So the device may reach the reference's leaves through ANY tree of boxes that
// contain them, culling with any test that never rejects a box containing a
// hit closer than the current best (the narrowed slab test with a 2^-16
// relative margin), as long as every leaf it opens is first put through the
// reference's own loose test and ties go to the lower DFS slot.  This file
// builds that tree: binned SAH (true surface area) over the reference leaves
// as items, then collapsed to 4 children per node.
//
// Device layout (filled here, read by render.hip):
//   wide node = 8 x float4 (128 B, one cache line):
//     {min.x of children 0..3}, {min.y}, {min.z}, {max.x}, {max.y}, {max.z},
//     {ref a of children 0..3}, {ref b of children 0..3}   (int bits)
//     inner child: ref a = wide node index (>= 0);
//     leaf child:  the box IS the reference leaf's box (bit for bit) and
//                  ref a / ref b are its one or two primitive-slot refs of
//                  render.hip (< 0; b == a for a one-primitive leaf);
//     empty slot:  an empty box (min = +inf, max = -inf), never entered.
//   An inner child's box is stored grown by `inflate` x its own largest
//   |coordinate| (render.hip passes 2^-19): a computed primitive hit lies outside
//   its box by a few ulps of the coordinates, and growing the box in space grows
//   each axis's t interval by that distance x |1/d_k| - the right slack for a
//   ray (nearly) parallel to a box face, at no cost per node (DESIGN.md §3
//   "Grazing rays").  An inner child whose subtree holds a sphere is grown by
//   `sphere_grow` more: the rounded sphere test accepts rays that pass outside
//   the sphere by up to ~sqrt(u) |oc| and errs by as much in t (DESIGN.md §3
//   "Spheres").  A leaf child holding a sphere stores ref a - kSphereSlotBias.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "accel_build.hpp"

namespace zrt {

namespace {

struct Aabb {
  float mn[3] = {INFINITY, INFINITY, INFINITY};
  float mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  void grow(const Aabb& b) {
    for (int k = 0; k < 3; ++k) {
      mn[k] = std::min(mn[k], b.mn[k]);
      mx[k] = std::max(mx[k], b.mx[k]);
    }
  }
  void grow(const float p[3]) {
    for (int k = 0; k < 3; ++k) {
      mn[k] = std::min(mn[k], p[k]);
      mx[k] = std::max(mx[k], p[k]);
    }
  }
  double area() const {
    if (mx[0] < mn[0]) return 0.0;
    const double dx = double(mx[0]) - mn[0], dy = double(mx[1]) - mn[1], dz = double(mx[2]) - mn[2];
    return 2.0 * (dx * dy + dy * dz + dz * dx);
  }
};

struct Item {
  Aabb box;
  float c[3];
  int32_t leaf;
  bool sphere;
};

struct Node2 {
  Aabb box;
  int32_t left = -1, right = -1;  // children (Node2 indices); -1 for a leaf
  int32_t leaf = -1;              // reference leaf index for a leaf
  bool sphere = false;            // the subtree holds a sphere
};

struct Builder2 {
  std::vector<Item>& items;
  std::vector<Node2> nodes;

  int32_t build(size_t lo, size_t hi) {
    const int32_t me = int32_t(nodes.size());
    nodes.emplace_back();
    Aabb box, cb;
    for (size_t i = lo; i < hi; ++i) {
      box.grow(items[i].box);
      cb.grow(items[i].c);
    }
    nodes[me].box = box;
    const size_t n = hi - lo;
    if (n == 1) {
      nodes[me].leaf = items[lo].leaf;
      nodes[me].sphere = items[lo].sphere;
      return me;
    }
    // binned SAH over centroids
    constexpr int kBins = 32;
    int best_axis = -1, best_bin = -1;
    double best_cost = INFINITY;
    for (int axis = 0; axis < 3; ++axis) {
      const float ext = cb.mx[axis] - cb.mn[axis];
      if (!(ext > 0.0f)) continue;
      Aabb bb[kBins];
      size_t cnt[kBins] = {0};
      const float scale = kBins / ext;
      for (size_t i = lo; i < hi; ++i) {
        int b = int((items[i].c[axis] - cb.mn[axis]) * scale);
        b = std::min(std::max(b, 0), kBins - 1);
        bb[b].grow(items[i].box);
        ++cnt[b];
      }
      double right_area[kBins];
      size_t right_cnt[kBins];
      Aabb acc;
      size_t c = 0;
      for (int b = kBins - 1; b > 0; --b) {
        acc.grow(bb[b]);
        c += cnt[b];
        right_area[b] = acc.area();
        right_cnt[b] = c;
      }
      Aabb lacc;
      size_t lc = 0;
      for (int b = 0; b < kBins - 1; ++b) {
        lacc.grow(bb[b]);
        lc += cnt[b];
        if (lc == 0 || right_cnt[b + 1] == 0) continue;
        const double cost = lacc.area() * double(lc) + right_area[b + 1] * double(right_cnt[b + 1]);
        if (cost < best_cost) {
          best_cost = cost;
          best_axis = axis;
          best_bin = b;
        }
      }
    }
    size_t mid;
    if (best_axis < 0) {  // coincident centroids: split by position in the list
      mid = lo + n / 2;
    } else {
      const float ext = cb.mx[best_axis] - cb.mn[best_axis];
      const float scale = kBins / ext;
      auto it = std::partition(items.begin() + lo, items.begin() + hi, [&](const Item& t) {
        int b = int((t.c[best_axis] - cb.mn[best_axis]) * scale);
        b = std::min(std::max(b, 0), kBins - 1);
        return b <= best_bin;
      });
      mid = size_t(it - items.begin());
      if (mid == lo || mid == hi) mid = lo + n / 2;
    }
    const int32_t l = build(lo, mid);
    const int32_t r = build(mid, hi);
    nodes[me].left = l;
    nodes[me].right = r;
    nodes[me].sphere = nodes[size_t(l)].sphere || nodes[size_t(r)].sphere;
    return me;
  }
};

void put4(float4v& q, int lane, float v) { q.v[lane] = v; }

}  // namespace

WideBvh build_wide_bvh(const std::vector<RefLeaf>& leaves, uint32_t top_levels, float inflate, float sphere_grow,
                       bool mark_spheres) {
  WideBvh out;
  out.layout = kLayoutVersion | (mark_spheres ? kLayoutSphereSlots | kLayoutSphereFirst : 0u);
  const size_t n = leaves.size();
  out.n_leaves = uint32_t(n);
  std::vector<Item> items(n);
  for (size_t i = 0; i < n; ++i) {
    const RefLeaf& L = leaves[i];
    for (int k = 0; k < 3; ++k) {
      items[i].box.mn[k] = L.mn[k];
      items[i].box.mx[k] = L.mx[k];
      items[i].c[k] = 0.5f * (L.mn[k] + L.mx[k]);
    }
    items[i].leaf = int32_t(i);
    items[i].sphere = ref_is_sphere(L.prim_a) || ref_is_sphere(L.prim_b);
  }
  if (n == 0) return out;
  Builder2 b{items, {}};
  b.nodes.reserve(2 * n);
  b.build(0, n);
  const std::vector<Node2>& N = b.nodes;

  // collapse to 4-wide: repeatedly open the child with the largest area
  struct Wide {
    int32_t child[4];
    int count;
  };
  std::vector<Wide> wide;
  std::vector<int32_t> wide_of(N.size(), -1);
  std::vector<uint32_t> depth_of;
  // BFS over binary nodes that become wide nodes
  std::vector<int32_t> queue;
  auto make_wide = [&](int32_t bn) {
    Wide w{};
    w.count = 0;
    if (N[bn].leaf >= 0) {  // a single-leaf tree
      w.child[w.count++] = bn;
    } else {
      w.child[w.count++] = N[bn].left;
      w.child[w.count++] = N[bn].right;
      while (w.count < 4) {
        int pick = -1;
        double best = -1.0;
        for (int k = 0; k < w.count; ++k) {
          const Node2& c = N[w.child[k]];
          if (c.leaf >= 0) continue;
          const double a = c.box.area();
          if (a > best) {
            best = a;
            pick = k;
          }
        }
        if (pick < 0) break;
        const int32_t opened = w.child[pick];
        w.child[pick] = N[opened].left;
        w.child[w.count++] = N[opened].right;
      }
    }
    // leaf children holding a sphere first (render.hip tests slot 0 alone for
    // a node with sphere slots); slot order never changes a result: hits are
    // ranked by t and primitive slot, children visited near-first
    if (mark_spheres)
      std::stable_partition(w.child, w.child + w.count,
                            [&](int32_t c) { return N[size_t(c)].leaf >= 0 && N[size_t(c)].sphere; });
    wide_of[bn] = int32_t(wide.size());
    wide.push_back(w);
    return wide_of[bn];
  };
  make_wide(0);
  depth_of.push_back(1);
  for (size_t wi = 0; wi < wide.size(); ++wi) {
    for (int k = 0; k < wide[wi].count; ++k) {
      const int32_t c = wide[wi].child[k];
      if (N[c].leaf < 0 && wide_of[c] < 0) {
        make_wide(c);
        depth_of.push_back(depth_of[wi] + 1);
      }
    }
  }
  out.n_nodes = uint32_t(wide.size());
  out.nodes.resize(8 * wide.size());
  // storage order: the top `top_levels` levels first, breadth-first (render.hip
  // serves them from LDS: nodes 0 .. n_top-1), then depth-first (pre-order,
  // children in slot order), so a subtree's nodes are adjacent (A/B against the
  // breadth-first construction order: equal on C4 / C5, +0.7 % on C3)
  std::vector<int32_t> pos(wide.size(), -1);
  {
    int32_t next_pos = 0;
    std::vector<int32_t> level{0}, roots;  // roots: first nodes below the top levels
    for (uint32_t l = 0; l < top_levels && !level.empty(); ++l) {
      std::vector<int32_t> below;
      for (const int32_t wi : level) {
        pos[size_t(wi)] = next_pos++;
        for (int k = 0; k < wide[size_t(wi)].count; ++k) {
          const int32_t c = wide[size_t(wi)].child[k];
          if (N[c].leaf < 0) below.push_back(wide_of[c]);
        }
      }
      level.swap(below);
      out.level_end.push_back(uint32_t(next_pos));
    }
    out.n_top = uint32_t(next_pos);
    for (const int32_t r : level) {
      std::vector<int32_t> todo{r};
      while (!todo.empty()) {
        const int32_t wi = todo.back();
        todo.pop_back();
        pos[size_t(wi)] = next_pos++;
        for (int k = wide[size_t(wi)].count - 1; k >= 0; --k) {
          const int32_t c = wide[size_t(wi)].child[k];
          if (N[c].leaf < 0) todo.push_back(wide_of[c]);
        }
      }
    }
  }
  uint32_t max_depth = 0;
  for (size_t wi = 0; wi < wide.size(); ++wi) {
    float4v q[8];
    for (int k = 0; k < 8; ++k) q[k] = float4v{};
    for (int k = 0; k < 4; ++k) {
      int32_t ref = -1, ref_b = -1;  // empty slot: never entered (empty box)
      Aabb box;                      // empty by default
      if (k < wide[wi].count) {
        const int32_t c = wide[wi].child[k];
        box = N[c].box;
        if (N[c].leaf >= 0) {
          ref = leaves[size_t(N[c].leaf)].prim_a;
          ref_b = leaves[size_t(N[c].leaf)].prim_b;
          if (N[c].sphere && mark_spheres) ref -= kSphereSlotBias;
        } else {
          ref = pos[size_t(wide_of[c])];
          ref_b = 0;
          double cmax = 0.0;
          for (int a = 0; a < 3; ++a) cmax = std::max({cmax, std::fabs(double(box.mn[a])), std::fabs(double(box.mx[a]))});
          const double g = double(inflate) * cmax + (N[c].sphere ? double(sphere_grow) : 0.0);
          for (int a = 0; a < 3 && g > 0.0; ++a) {  // grown outward, rounded outward
            float lo = float(double(box.mn[a]) - g), hi = float(double(box.mx[a]) + g);
            if (double(lo) > double(box.mn[a]) - g) lo = std::nextafter(lo, -INFINITY);
            if (double(hi) < double(box.mx[a]) + g) hi = std::nextafter(hi, INFINITY);
            box.mn[a] = lo;
            box.mx[a] = hi;
          }
        }
      }
      put4(q[0], k, box.mn[0]);
      put4(q[1], k, box.mn[1]);
      put4(q[2], k, box.mn[2]);
      put4(q[3], k, box.mx[0]);
      put4(q[4], k, box.mx[1]);
      put4(q[5], k, box.mx[2]);
      std::memcpy(&q[6].v[k], &ref, 4);
      std::memcpy(&q[7].v[k], &ref_b, 4);
    }
    for (int k = 0; k < 8; ++k) out.nodes[8 * size_t(pos[wi]) + k] = q[k];
    max_depth = std::max(max_depth, depth_of[wi]);
  }
  out.depth = max_depth;
  // near-first traversal pushes at most 3 inner children per wide level
  out.max_stack = 3 * max_depth + 2;
  return out;
}

}  // namespace zrt

namespace zrt {

namespace {
// One axis of a node: the step exponent and origin multiple with every plane of
// [lo, hi] an exact f32 origin + q * step, q in 0..255.  False if none exists.
bool quant_axis(double lo, double hi, int* e_out, double* m0_out) {
  if (!(std::isfinite(lo) && std::isfinite(hi) && lo <= hi)) return false;
  int e = -126;  // the smallest normal step
  if (hi > lo) e = std::max(e, int(std::floor(std::log2((hi - lo) / 255.0))) - 1);
  for (; e <= 127; ++e) {
    const double s = std::ldexp(1.0, e);
    const double m0 = std::floor(lo / s), m1 = std::ceil(hi / s);
    if (m1 - m0 <= 255.0 && std::fabs(m0) + 256.0 < 16777216.0) {
      *e_out = e;
      *m0_out = m0;
      return true;
    }
  }
  return false;
}
}  // namespace

QuantWide quantize_wide(const WideBvh& w) {
  QuantWide out;
  const uint32_t n = w.n_nodes;
  out.n_nodes = n;
  std::vector<float4v> base(size_t(n) * kQuantNodeF4);  // unswapped; bytes as min (near) / max (far)
  struct Planes {
    uint32_t qmin[3], qmax[3];  // bytes of slots 0..3, per axis
  };
  std::vector<Planes> planes(n);
  for (uint32_t i = 0; i < n; ++i) {
    const float4v* q = &w.nodes[8 * size_t(i)];
    int32_t ref[4], ref_b[4];
    std::memcpy(ref, q[6].v, 16);
    std::memcpy(ref_b, q[7].v, 16);
    bool empty[4];
    for (int k = 0; k < 4; ++k) empty[k] = q[0].v[k] > q[3].v[k];  // (min = +inf, max = -inf)
    uint32_t word[16] = {0};
    Planes& P = planes[i];
    for (int a = 0; a < 3; ++a) {
      double lo = INFINITY, hi = -INFINITY;
      for (int k = 0; k < 4; ++k)
        if (!empty[k]) {
          lo = std::min(lo, double(q[a].v[k]));
          hi = std::max(hi, double(q[3 + a].v[k]));
        }
      int e = 0;
      double m0 = 0.0;
      if (lo > hi) {  // no child
        lo = hi = 0.0;
      }
      if (!quant_axis(lo, hi, &e, &m0)) return out;  // (ok stays false)
      const double s = std::ldexp(1.0, e);
      const float origin = float(m0 * s);
      if (double(origin) != m0 * s) return out;
      std::memcpy(&word[a], &origin, 4);
      word[3] |= uint32_t(e + 127) << (8 * a);
      P.qmin[a] = P.qmax[a] = 0;
      for (int k = 0; k < 4; ++k) {
        uint32_t qn = 255, qf = 0;  // an empty slot: near above far (never opened: its ref is kEmptyRef)
        if (!empty[k]) {
          const double mn = q[a].v[k], mx = q[3 + a].v[k];
          qn = uint32_t(std::floor(mn / s) - m0);
          qf = uint32_t(std::ceil(mx / s) - m0);
          // decoded exactly, outward (the child's box within the quantized one)
          const float dn = float(double(origin) + double(qn) * s), df = float(double(origin) + double(qf) * s);
          if (qn > 255 || qf > 255 || !(double(dn) <= mn) || !(double(df) >= mx) ||
              double(dn) != double(origin) + double(qn) * s || double(df) != double(origin) + double(qf) * s)
            return out;
        }
        P.qmin[a] |= qn << (8 * k);
        P.qmax[a] |= qf << (8 * k);
      }
    }
    for (int k = 0; k < 4; ++k) {
      int32_t r = ref[k];
      if (empty[k]) {
        r = kEmptyRef;
      } else if (r < 0) {  // a leaf: its record
        const uint32_t L = out.n_leaves++;
        const bool sphere = r < -kSphereSlotBias;
        const int32_t a = sphere ? r + kSphereSlotBias : r;
        float4v rec[2];
        for (int j = 0; j < 3; ++j) {
          rec[0].v[j] = q[j].v[k];
          rec[1].v[j] = q[3 + j].v[k];
        }
        std::memcpy(&rec[0].v[3], &a, 4);
        std::memcpy(&rec[1].v[3], &ref_b[k], 4);
        out.leaves.push_back(rec[0]);
        out.leaves.push_back(rec[1]);
        r = -int32_t(L) - 1 - (sphere ? kSphereSlotBias : 0);
      }
      std::memcpy(&word[10 + k], &r, 4);
    }
    std::memcpy(&base[size_t(i) * kQuantNodeF4], word, sizeof(word));
  }
  // the octant copies: axis k's near / far bytes swapped where the direction is negative
  out.nodes.resize(8 * size_t(n) * kQuantNodeF4);
  for (uint32_t o = 0; o < 8; ++o) {
    float4v* dst = out.nodes.data() + size_t(o) * n * kQuantNodeF4;
    std::memcpy(dst, base.data(), base.size() * sizeof(float4v));
    for (uint32_t i = 0; i < n; ++i) {
      uint32_t word[16];
      std::memcpy(word, &dst[size_t(i) * kQuantNodeF4], sizeof(word));
      for (int a = 0; a < 3; ++a) {
        const bool neg = (o >> a) & 1u;
        word[4 + a] = neg ? planes[i].qmax[a] : planes[i].qmin[a];
        word[7 + a] = neg ? planes[i].qmin[a] : planes[i].qmax[a];
      }
      std::memcpy(&dst[size_t(i) * kQuantNodeF4], word, sizeof(word));
    }
  }
  out.ok = true;
  return out;
}

}  // namespace zrt
