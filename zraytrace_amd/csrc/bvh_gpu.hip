// bvh_gpu.hip — the reference BVH (bvh.zig:62-185) built on the GPU.
//
// Same tree as build_bvh (bvh_build.cpp), node for node, for the million-
// triangle meshes where the host build dominated the frame (C5 substitute:
// 1.6 M triangles, 5.6 s on the host).  divide() (bvh.zig:129-160) is run
// breadth-first: every level's segments (slices of the primitive order that
// still need a split, n >= 3) are divided together.
//
// The reference's optimal_axis_divide (bvh.zig:85-120) stable-sorts the slice
// on x, then (from that order) on y, then on z, scoring the splits n/4, n/2,
// 3n/4 after each sort, and finally stable-sorts the z-sorted slice on the best
// axis.  A stable sort of one segment is a stable sort of the whole order
// array by the 64-bit key (segment start << 32 | axis key), because segments
// are contiguous and their starts increase with position (positions outside
// every active segment carry their own position as the segment start, so they
// never move).  Each level is therefore four hipcub radix sorts (LSD radix
// sort is stable) of (key, primitive) pairs, three scoring launches (one wave
// per segment: the left / right range boxes of each split and the segment's
// box, min/max reduced with shuffles — min/max are exact, and the zero signs a
// different reduction order could give do not reach the pseudo surface area,
// which takes |min - max|), and one choice of the best (axis, split) per
// segment with the reference's strict `<` in its trial order.  The host keeps
// the segment list (one download of the splits per level), then numbers the
// nodes in depth-first pre-order and computes their boxes bottom-up with
// box_union exactly as the host build does.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "bvh_build.hpp"
#include "device_math.hpp"
#include "zrt.hpp"

namespace zrt {
namespace {

#define BVHCHK(expr)                                                                         \
  do {                                                                                       \
    const hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess)                                                                    \
      throw ::zrt::Error(ZRT_E_HIP, std::string("BVH device build: ") + #expr + ": " +      \
                                        hipGetErrorString(e_));                              \
  } while (0)

template <class T>
struct GBuf {
  T* p = nullptr;
  size_t n = 0;
  GBuf() = default;
  GBuf(const GBuf&) = delete;
  GBuf& operator=(const GBuf&) = delete;
  ~GBuf() {
    if (p) (void)hipFree(p);
  }
  void alloc(size_t count) {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    if (count == 0) return;
    BVHCHK(hipMalloc(&p, count * sizeof(T)));
    n = count;
  }
};

// ---- device side -----------------------------------------------------------

__global__ void iota_kernel(uint32_t* __restrict__ a, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) a[i] = i;
}

// every position its own segment start (positions of finished segments never
// move) and no segment index; then the level's active segments claim theirs
__global__ void unmark_kernel(uint32_t* __restrict__ pos_seg, uint32_t* __restrict__ pos_idx, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    pos_seg[i] = i;
    pos_idx[i] = 0xffffffffu;
  }
}

__global__ void mark_kernel(const uint32_t* __restrict__ seg_lo, const uint32_t* __restrict__ seg_n, uint32_t S,
                            uint32_t* __restrict__ pos_seg, uint32_t* __restrict__ pos_idx) {
  const uint32_t s = blockIdx.x;
  if (s >= S) return;
  const uint32_t lo = seg_lo[s], n = seg_n[s];
  for (uint32_t j = threadIdx.x; j < n; j += blockDim.x) {
    pos_seg[lo + j] = lo;
    pos_idx[lo + j] = s;
  }
}

// sort keys of one trial: (segment start, the primitive's midpoint key on `axis`)
__global__ void keys_kernel(const uint32_t* __restrict__ pos_seg, const uint32_t* __restrict__ order,
                            const uint32_t* __restrict__ axis_keys, uint64_t* __restrict__ out, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = ((uint64_t)pos_seg[i] << 32) | axis_keys[order[i]];
}

// the final re-sort: each active segment on its best axis (finished positions: key 0)
__global__ void best_keys_kernel(const uint32_t* __restrict__ pos_seg, const uint32_t* __restrict__ pos_idx,
                                 const uint32_t* __restrict__ order, const uint32_t* __restrict__ keys,
                                 const uint32_t* __restrict__ best_axis, uint32_t n, uint64_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t s = pos_idx[i];
  const uint32_t k = s == 0xffffffffu ? 0u : keys[(size_t)best_axis[s] * n + order[i]];
  out[i] = ((uint64_t)pos_seg[i] << 32) | k;
}

struct RBox {
  float mn[3], mx[3];
};

__device__ __forceinline__ void rbox_empty(RBox& b) {
  for (int k = 0; k < 3; ++k) {
    b.mn[k] = __builtin_inff();
    b.mx[k] = -__builtin_inff();
  }
}
// bvh.zig:62-69 -> aabb.zig:73-81: min / max over every box's min and max
__device__ __forceinline__ void rbox_add(RBox& b, const float4 lo, const float4 hi) {
  const float l[3] = {lo.x, lo.y, lo.z}, h[3] = {hi.x, hi.y, hi.z};
  for (int k = 0; k < 3; ++k) {
    b.mn[k] = dev::fmin_z(dev::fmin_z(b.mn[k], l[k]), h[k]);
    b.mx[k] = dev::fmax_z(dev::fmax_z(b.mx[k], l[k]), h[k]);
  }
}
__device__ __forceinline__ void rbox_wave_reduce(RBox& b) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    for (int k = 0; k < 3; ++k) {
      b.mn[k] = dev::fmin_z(b.mn[k], __shfl_xor(b.mn[k], off));
      b.mx[k] = dev::fmax_z(b.mx[k], __shfl_xor(b.mx[k], off));
    }
  }
}
// pseudoSA (aabb.zig:99-105) of initMinMax(min, max) (aabb.zig:37-41)
__device__ __forceinline__ float rbox_area(const RBox& b) {
  float d[3];
  for (int k = 0; k < 3; ++k) {
    const float lo = dev::fmin_z(b.mn[k], b.mx[k]), hi = dev::fmax_z(b.mn[k], b.mx[k]);
    d[k] = __builtin_fabsf(lo - hi);
  }
  return 2.0f * (d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
}

// One wave per active segment: the trial of `axis` on the segment as `order`
// now holds it (sorted on that axis).  scores[s * 9 + axis * 3 + k] = the
// ratio of split k (bvh.zig:104-106); the z trial also picks the best (axis,
// split) in the reference's trial order with its strict `<` (bvh.zig:107-113).
__global__ void __launch_bounds__(64) score_kernel(const uint32_t* __restrict__ seg_lo,
                                                   const uint32_t* __restrict__ seg_n, uint32_t S,
                                                   const uint32_t* __restrict__ order, const float4* __restrict__ plo,
                                                   const float4* __restrict__ phi, int axis, float* __restrict__ scores,
                                                   float* __restrict__ totals, uint32_t* __restrict__ best_axis,
                                                   uint32_t* __restrict__ best_split) {
  const uint32_t s = blockIdx.x;
  if (s >= S) return;
  const uint32_t lo = seg_lo[s], n = seg_n[s];
  uint32_t split[3] = {n / 2, 0, 0};
  int ns = 1;
  if (n >= 4) {
    split[0] = n / 4;
    split[1] = n / 2;
    split[2] = n / 4 + n / 2;
    ns = 3;
  }
  RBox left[3], right[3], all;
  rbox_empty(all);
  for (int k = 0; k < 3; ++k) {
    rbox_empty(left[k]);
    rbox_empty(right[k]);
  }
  for (uint32_t j = threadIdx.x; j < n; j += 64) {
    const uint32_t p = order[lo + j];
    const float4 bl = plo[p], bh = phi[p];
    if (axis == 0) rbox_add(all, bl, bh);
    for (int k = 0; k < ns; ++k) {
      if (j < split[k]) rbox_add(left[k], bl, bh);
      else rbox_add(right[k], bl, bh);
    }
  }
  if (axis == 0) rbox_wave_reduce(all);
  for (int k = 0; k < ns; ++k) {
    rbox_wave_reduce(left[k]);
    rbox_wave_reduce(right[k]);
  }
  if (threadIdx.x != 0) return;
  if (axis == 0) totals[s] = rbox_area(all);
  const float total = totals[s];
  for (int k = 0; k < ns; ++k) {
    const float area = rbox_area(right[k]) + rbox_area(left[k]);  // right + left, as bvh.zig:104
    scores[(size_t)s * 9 + axis * 3 + k] = area / total;
  }
  if (axis != 2) return;
  uint32_t ba = 0, bs = n / 2;
  float br = __builtin_inff();
  for (int a = 0; a < 3; ++a)
    for (int k = 0; k < ns; ++k) {
      const float ratio = scores[(size_t)s * 9 + a * 3 + k];
      if (ratio < br) {
        br = ratio;
        ba = (uint32_t)a;
        bs = split[k];
      }
    }
  best_axis[s] = ba;
  best_split[s] = bs;
}

// ---- host side ---------------------------------------------------------------

struct Seg {
  uint32_t lo, n, node, depth;
};
// A node in the order the levels create it: an inner node's children are node
// ids; a leaf (n <= 2) keeps its slice, resolved from the final order.
struct LNode {
  int32_t l = -1, r = -1;
  uint32_t lo = 0, n = 0, depth = 0;
};

inline uint32_t grid_of(uint32_t n, uint32_t b) { return (n + b - 1) / b; }

}  // namespace

bool build_bvh_device(const zrt_prim* prims, uint32_t n, int device, BuiltBvh* out) {
  if (n < 3 || n >= 0x80000000u) return false;
  std::vector<Box> pbox(n);
  std::vector<float4> lo4(n), hi4(n);
  std::vector<uint32_t> keys(3 * size_t(n));
  for (uint32_t i = 0; i < n; ++i) {
    pbox[i] = prim_box(prims[i]);
    const Box& b = pbox[i];
    for (int k = 0; k < 3; ++k) {
      if (std::isnan(b.mid[k])) return false;  // no strict weak order: the host build's stable_sort
      keys[size_t(k) * n + i] = mid_key(b.mid[k]);
    }
    lo4[i] = make_float4(b.mn[0], b.mn[1], b.mn[2], 0.0f);
    hi4[i] = make_float4(b.mx[0], b.mx[1], b.mx[2], 0.0f);
  }
  BVHCHK(hipSetDevice(device));
  // tests: a HIP failure inside the device build (flatten_scene must fall back to the host build)
  if (const char* e = std::getenv("ZRT_DEBUG_BVH_DEVICE_FAIL"))
    if (std::atoi(e) != 0) BVHCHK(hipErrorOutOfMemory);
  hipStream_t st = nullptr;
  BVHCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  struct StreamGuard {
    hipStream_t s;
    ~StreamGuard() { (void)hipStreamDestroy(s); }
  } sg{st};

  GBuf<float4> plo, phi;
  GBuf<uint32_t> dkeys, order_a, order_b, pos_seg, pos_idx, seg_lo, seg_n, best_axis, best_split;
  GBuf<uint64_t> key_a, key_b;
  GBuf<float> scores, totals;
  plo.alloc(n);
  phi.alloc(n);
  dkeys.alloc(3 * size_t(n));
  order_a.alloc(n);
  order_b.alloc(n);
  pos_seg.alloc(n);
  pos_idx.alloc(n);
  key_a.alloc(n);
  key_b.alloc(n);
  BVHCHK(hipMemcpyAsync(plo.p, lo4.data(), n * sizeof(float4), hipMemcpyHostToDevice, st));
  BVHCHK(hipMemcpyAsync(phi.p, hi4.data(), n * sizeof(float4), hipMemcpyHostToDevice, st));
  BVHCHK(hipMemcpyAsync(dkeys.p, keys.data(), keys.size() * sizeof(uint32_t), hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(iota_kernel, dim3(grid_of(n, 256)), dim3(256), 0, st, order_a.p, n);
  BVHCHK(hipGetLastError());
  int end_bit = 32;
  while ((1ull << (end_bit - 32)) < n) ++end_bit;  // segment starts < n
  size_t temp_bytes = 0;
  BVHCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, temp_bytes, key_a.p, key_b.p, order_a.p, order_b.p, int(n), 0,
                                            end_bit, st));
  GBuf<uint8_t> temp;
  temp.alloc(std::max<size_t>(temp_bytes, 1));
  uint32_t* order = order_a.p;  // the current primitive order
  uint32_t* spare = order_b.p;
  auto sort = [&](void) {
    size_t tb = temp_bytes;
    BVHCHK(hipcub::DeviceRadixSort::SortPairs(temp.p, tb, key_a.p, key_b.p, order, spare, int(n), 0, end_bit, st));
    std::swap(order, spare);
  };

  std::vector<LNode> nodes(1);
  nodes[0].depth = 1;
  std::vector<Seg> segs{{0, n, 0, 1}}, next;
  std::vector<uint32_t> h_lo, h_n, h_split;
  uint32_t max_depth = 1;
  while (!segs.empty()) {
    const uint32_t S = uint32_t(segs.size());
    h_lo.resize(S);
    h_n.resize(S);
    for (uint32_t s = 0; s < S; ++s) {
      h_lo[s] = segs[s].lo;
      h_n[s] = segs[s].n;
    }
    if (seg_lo.n < S) {
      const size_t cap = std::max<size_t>(S, seg_lo.n * 2);
      seg_lo.alloc(cap);
      seg_n.alloc(cap);
      best_axis.alloc(cap);
      best_split.alloc(cap);
      scores.alloc(cap * 9);
      totals.alloc(cap);
    }
    BVHCHK(hipMemcpyAsync(seg_lo.p, h_lo.data(), S * sizeof(uint32_t), hipMemcpyHostToDevice, st));
    BVHCHK(hipMemcpyAsync(seg_n.p, h_n.data(), S * sizeof(uint32_t), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(unmark_kernel, dim3(grid_of(n, 256)), dim3(256), 0, st, pos_seg.p, pos_idx.p, n);
    hipLaunchKernelGGL(mark_kernel, dim3(S), dim3(256), 0, st, seg_lo.p, seg_n.p, S, pos_seg.p, pos_idx.p);
    BVHCHK(hipGetLastError());
    for (int axis = 0; axis < 3; ++axis) {  // x, then y from the x order, then z from the y order
      hipLaunchKernelGGL(keys_kernel, dim3(grid_of(n, 256)), dim3(256), 0, st, pos_seg.p, order,
                         dkeys.p + size_t(axis) * n, key_a.p, n);
      BVHCHK(hipGetLastError());
      sort();
      hipLaunchKernelGGL(score_kernel, dim3(S), dim3(64), 0, st, seg_lo.p, seg_n.p, S, order, plo.p, phi.p, axis,
                         scores.p, totals.p, best_axis.p, best_split.p);
      BVHCHK(hipGetLastError());
    }
    // the best axis' stable re-sort of the z-sorted slice (identity when z won)
    hipLaunchKernelGGL(best_keys_kernel, dim3(grid_of(n, 256)), dim3(256), 0, st, pos_seg.p, pos_idx.p, order,
                       dkeys.p, best_axis.p, n, key_a.p);
    BVHCHK(hipGetLastError());
    sort();
    h_split.resize(S);
    BVHCHK(hipMemcpyAsync(h_split.data(), best_split.p, S * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    BVHCHK(hipStreamSynchronize(st));
    next.clear();
    for (uint32_t s = 0; s < S; ++s) {
      const Seg& g = segs[s];
      const uint32_t split = h_split[s];
      const uint32_t cl[2] = {g.lo, g.lo + split}, cn[2] = {split, g.n - split};
      for (int c = 0; c < 2; ++c) {
        const uint32_t id = uint32_t(nodes.size());
        LNode ln;
        ln.lo = cl[c];
        ln.n = cn[c];
        ln.depth = g.depth + 1;
        nodes.push_back(ln);
        (c == 0 ? nodes[g.node].l : nodes[g.node].r) = int32_t(id);
        max_depth = std::max(max_depth, g.depth + 1);
        if (cn[c] >= 3) next.push_back(Seg{cl[c], cn[c], id, g.depth + 1});
      }
    }
    segs.swap(next);
  }
  std::vector<uint32_t> fin(n);
  BVHCHK(hipMemcpyAsync(fin.data(), order, n * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  BVHCHK(hipStreamSynchronize(st));

  // depth-first pre-order (left first) numbering, then boxes bottom-up
  const size_t total = nodes.size();
  std::vector<uint32_t> pre(total);
  std::vector<uint32_t> by_pre(total);
  {
    std::vector<uint32_t> stack{0};
    uint32_t k = 0;
    while (!stack.empty()) {
      const uint32_t id = stack.back();
      stack.pop_back();
      pre[id] = k;
      by_pre[k++] = id;
      if (nodes[id].l >= 0) {  // inner: right pushed first so the left comes next
        stack.push_back(uint32_t(nodes[id].r));
        stack.push_back(uint32_t(nodes[id].l));
      }
    }
  }
  out->nodes.assign(total, BuildNode{});
  out->max_depth = max_depth;
  std::vector<Box> nbox(total);
  for (size_t k = total; k-- > 0;) {  // children have larger pre-order numbers than their parent
    const uint32_t id = by_pre[k];
    const LNode& ln = nodes[id];
    BuildNode& bn = out->nodes[k];
    Box lb, rb;
    if (ln.l >= 0) {
      bn.left = int32_t(pre[uint32_t(ln.l)]);
      bn.right = int32_t(pre[uint32_t(ln.r)]);
      lb = nbox[uint32_t(ln.l)];
      rb = nbox[uint32_t(ln.r)];
    } else if (ln.n == 1) {  // bvh.zig:132-136: the primitive on both sides
      const uint32_t p = fin[ln.lo];
      bn.left = bn.right = -int32_t(p) - 1;
      lb = rb = pbox[p];
    } else {  // bvh.zig:138-143: left = s[1], right = s[0]
      const uint32_t p0 = fin[ln.lo], p1 = fin[ln.lo + 1];
      bn.left = -int32_t(p1) - 1;
      bn.right = -int32_t(p0) - 1;
      lb = pbox[p1];
      rb = pbox[p0];
    }
    const Box b = box_union(lb, rb);  // bvh.zig:164
    nbox[id] = b;
    for (int c = 0; c < 3; ++c) {
      bn.mn[c] = b.mn[c];
      bn.mx[c] = b.mx[c];
    }
  }
  return true;
}

}  // namespace zrt

// The device build exported for parity tests (node-for-node against
// zrt_bvh_build and the oracle) and timing.
extern "C" int zrt_bvh_build_device(const zrt_scene* scene, uint32_t device, zrt_bvh_node** out_nodes,
                                    uint32_t* n_nodes, uint32_t* max_depth) {
  if (!scene || !out_nodes || !n_nodes) return zrt::fail(ZRT_E_INVALID, "null argument");
  *out_nodes = nullptr;
  *n_nodes = 0;
  if (scene->n_prims == 0 || !scene->prims) return zrt::fail(ZRT_E_INVALID, "empty scene");
  try {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || int(device) >= count)
      return zrt::fail(ZRT_E_NODEVICE, "no HIP device " + std::to_string(device));
    zrt::BuiltBvh bvh;
    if (!zrt::build_bvh_device(scene->prims, scene->n_prims, int(device), &bvh))
      return zrt::fail(ZRT_E_UNSUPPORTED, "the device build needs >= 3 primitives and no NaN midpoints");
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
  } catch (const zrt::Error& e) {
    return zrt::fail(e.code, e.what());
  } catch (const std::bad_alloc&) {
    return zrt::fail(ZRT_E_NOMEM, "OutOfMemory");
  }
}
