// render.hip — the MI355X path of the reference's per-pixel sampling loop.
//
// Replaces raytrace.render (raytrace.zig:136-203) + rayColor (:62-100) and
// everything they call per sample: Camera.getRay (camera.zig:46-52), BVH/AABB
// traversal (bvh.zig:187-205, aabb.zig:109-127), Sphere.hit / Triangle.hit
// (sphere.zig:31-71, triangle.zig:48-70), HitRecord.init (hit_record.zig:28-41),
// Material.scatter (material.zig:43-129), Sample.randomUnitVector
// (sample.zig:47-61), Texture.albedo (texture.zig:20-74).
//
// Kernel structure (gfx950, wave64):
//   * persistent grid (CUs x resident blocks), 256-thread blocks;
//   * each lane owns one pixel at a time and walks its samples in order, so
//     the per-pixel f32 sum is accumulated exactly as raytrace.zig:172-179
//     does; when a lane's path ends it immediately starts the next sample, and
//     when its pixel is done the wave refills its finished lanes from a global
//     work counter with ONE atomic per wave (__ballot + popcount + mbcnt rank);
//   * the recursion `attenuation * rayColor(...)` is unrolled into an
//     iterative loop; the attenuations are stacked per lane and multiplied in
//     reverse at path end so the product keeps the recursion's association;
//   * BVH traversal uses a per-lane stack in LDS laid out [depth][lane]
//     (conflict-free: every lane of a wave hits a distinct bank);
//   * RNG: one Xoroshiro128+ (or Xoshiro256++) stream per (pixel, sample),
//     seeded through SplitMix64 exactly as DefaultPrng.init seeds.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "accel_build.hpp"
#include "bvh_build.hpp"
#include "device_math.hpp"
#include "zrt.hpp"

namespace zrt {

// ---------------------------------------------------------------------------
// device data layout
// ---------------------------------------------------------------------------
// nodes: 2 x float4 per node {min.xyz, left}, {max.xyz, right}; child >= 0 is
//   a node index, child < 0 a primitive slot ref -(2*slot + kind) - 1.
// prims: 3 x float4 per slot (slots in DFS leaf order, or list order):
//   triangle {a.xyz, e1.x} {e1.yz, e2.xy} {e2.z, n.xyz}  (n = e1 x e2)
//   sphere   {center.xyz, radius^2} {0} {0}   (radius * radius rounded once, on the host)
// shade: 1 x float4 per slot: triangle {unit normal.xyz, tag},
//   sphere {1/radius, 0, 0, tag}; tag = material | kind << 31 (as u32 bits)
struct alignas(16) DevMaterial {
  float r, g, b, ior;          // texture color / index of refraction
  float u_off, v_off;          // image texture offsets
  uint32_t kind, tex_kind;     // ZRT_MAT_*, ZRT_TEX_*
  uint32_t img_w, img_h, img_off;  // image texture (img_off in texels of its store)
  uint32_t img_u8;                 // 1: the image is stored as 8-bit RGBX (exact k/255), 0: f32 RGB
};

struct KArgs {
  const float4* __restrict__ nodes;
  const float4* __restrict__ prims;
  const float4* __restrict__ shade;
  const float4* __restrict__ wnodes;   // FAST: 4-wide nodes (node_f4 float4 each: 8 full, 4 compressed)
  const float4* __restrict__ qleaves;  // compressed nodes' leaf records (kLeafRecF4 float4 each), else null
  uint32_t n_qnodes, n_qleaves;        // compressed nodes per octant copy and leaf records (bounds checks)
  const DevMaterial* __restrict__ mats;
  const float* __restrict__ texels;    // f32 RGB images
  const uint32_t* __restrict__ texels8;  // 8-bit RGBX images (every value exactly k/255)
  uint32_t* __restrict__ att;          // [row - att_lds_rows][lane or path]: attenuation codes (att_code)
  float4* __restrict__ partial;        // [chunk][tile slot] chunk sums
  uint32_t* __restrict__ work_counter;
  uint32_t* __restrict__ unit_cost;         // probe: loop iterations a wave spent on each tile, else null
  // lockstep render after a scheduling probe: the probe's counters, from which every
  // wave derives the same lockstep interval (render_loop, auto_sync); null: a.sync
  const unsigned long long* __restrict__ sync_probe;
  const uint32_t* __restrict__ tile_order;  // local tiles in the order units are handed out, or null
  unsigned long long* __restrict__ wave_times;  // ZRT_PROFILE builds: {start, end} realtime per wave
  unsigned long long* __restrict__ counters;  // kNumCounters x u64
  // ZRT_FLAG_SCANLINES: [row][3] recursion-limit hits, reflections, background
  // hits per frame row (raytrace.zig:184's printProgress deltas), else null
  unsigned long long* __restrict__ scanlines;
  uint32_t* __restrict__ error_flag;
  float org[3], llc[3], hor[3], ver[3];
  // jitter (raytrace.zig:173-174) divides by width / height: (x + r - 0.5) lies
  // in {+0} u [2^-23, 65536], so dev::div_core with inv_* = RN(1 / width) (IEEE on
  // the host) is the IEEE quotient with no range check
  float f_width, f_height, color_scale, inv_width, inv_height;
  uint32_t width, height, xbound, spp, max_depth;
  uint32_t tiles_x, rank, world, total_work;
  uint32_t n_list, stack_depth, n_lanes;
  uint32_t chunk, n_chunks, sync;  // a work unit = one chunk of one tile
  uint32_t n_slots;  // this launch's pixel slots (tiles x 64): the stride of a chunk in partial
  uint32_t wide_stride;  // float4s per octant copy of the wide tree
  uint32_t node_f4;      // float4s per wide node: 8 (full, wide_iter) or 4 (compressed, wide_iter_q)
  uint32_t lds_rows;     // FAST: stack rows in LDS; rows lds_rows.. stack_depth-1 in stack_ovf
  uint32_t ref_stack;    // rows the reference traversal needs (FAST's order-hazard replay)
  const uint32_t* __restrict__ leaf_of_slot;  // primitive slot -> its reference BVH leaf node
  void* stack_ovf;       // [row - lds_rows][lane] overflow rows of the FAST stack (StackT)
  unsigned long long seed_mix;
  // LDS beyond the stack rows (byte offsets into the block's dynamic LDS):
  uint32_t n_top;         // FAST: wide nodes 0 .. n_top-1 (the top levels) served from LDS
  uint32_t lds_top_off;   //   [copy][node][8] float4, copied in at kernel start
  uint32_t lds_att_off;   // attenuation rows 0 .. att_lds_rows-1: [row][lane] u32 codes (att_code)
  uint32_t att_lds_rows;  //   (rows att_lds_rows.. in `att`, [row - att_lds_rows][lane])
  uint32_t lds_mat_off;   // the material table (n_mats DevMaterial), when mats_in_lds
  uint32_t n_mats, mats_in_lds;
  uint32_t wf_thresh;  // wavefront loop: shade when ready lanes >= this / 64 of the unit's active lanes
                       // (path-pool loop: once the queue is empty and fewer than 64 - this lanes traverse)
  uint32_t lds_pool_off;  // path-pool loop: rays, hits and queues (kBlockPaths paths per block)
  uint32_t lds_state_off;  // lockstep FAST loop: lane state across the traversal, [word][lane] u32 (LaneState)
  uint32_t n_paths;       //   paths of the launch (grid x kBlockPaths): the stride of its global attenuation rows
  uint32_t tri_rcp_fast;  // every triangle |n| < 2^125: 1/det by dev::rcp_core (RayT::rcp_det)
  float scene_extent;     // the triangles' largest |coordinate| (ray_slack)
  float tri_c[3], tri_h[3];  // the triangles' bounding box: centre, half extents (paxis_grow)
  float paxis_m;             // per-axis margins in waves with a lane of max_k |1/d_k| above this (kPaxisM)
  // Spheres (DESIGN.md §3 "Spheres"): the reference BVH nodes whose subtree holds
  // a sphere (1 byte each), and the origins the wide tree's sphere growth was
  // sized for: max_k |o_k - root_c[k]| <= origin_bound (other rays are traced the
  // reference's way, ray_origin_ok)
  const uint8_t* __restrict__ ref_sph;
  float root_c[3], origin_bound;
  uint32_t check_origins;  // 0: every ray of the launch starts inside the bound (the camera does, checked
                           // on the host, and scattered rays start at hits), so ray_origin_ok is skipped
  uint32_t layout;         // the wide tree's encoding (accel_build.hpp kLayout*): must equal kKernelLayout
  float graze_m;           // the grazing margins' coefficient (RayT::gm; DESIGN.md §3 "Grazing rays")
  float graze_leaf;        // ... of leaf slots' relative margin (RayT::gl, >= graze_m)
  float guard;             // the grazing-triangle guard (RayT::gk, wide_iter; 0: off)
  uint64_t att_cap, ovf_cap;  // elements of `att` and of `stack_ovf` (StackT): row_ok's bounds
};


// error_flag bits (zrt_ctx_sync / zrt_ctx_stats / zrt_render report them as ZRT_E_UNSUPPORTED)
constexpr uint32_t kErrOverflow = 1u;  // a traversal stack deeper than it was sized for
constexpr uint32_t kErrLayout = 2u;    // the wide tree's encoding is not the one this kernel decodes
constexpr uint32_t kErrBounds = 4u;    // STATS flavour: a global row index past its buffer (row_ok)

// The STATS flavour's bounds check of a global row index (attenuation rows,
// stack overflow rows) against its buffer (KArgs::att_cap / ovf_cap, set from the
// allocations): past it, kErrBounds is raised and the access skipped, so a
// sizing mistake the host check (zrt::check_buffers) missed reports instead of
// faulting.  The timed flavour compiles it away.
#ifndef ZRT_DEBUG_BOUNDS
#define ZRT_DEBUG_BOUNDS 1
#endif
template <bool STATS>
__device__ __forceinline__ bool row_ok(const KArgs& a, uint64_t idx, uint64_t cap) {
  if (!STATS || !ZRT_DEBUG_BOUNDS || idx < cap) return true;
  atomicOr(a.error_flag, kErrBounds);
  return false;
}

// counters[]: progress counters of raytrace.zig:20-34 + traffic diagnostics
enum { kDepthHits, kReflections, kBackground, kRays, kNodes, kTriTests, kSphereTests, kShades, kTexels,
       kLeaves, kReplays, kExcessTri, kExcessSph, kExcessHits, kNumCounters };
constexpr int kWorkSlot = 14, kErrorSlot = 15, kProfSlot = 16, kScratchSlots = 48;
// STATS flavour, SIMD efficiency (zrt_ctx_debug_counters): traversal loop trips
// of the waves (per traced step, the most node visits of any lane: kNodes /
// (64 kTravTrips) is the lane efficiency of traversal), loop iterations in which
// some lane ran a rayColor step, and the lane-steps run in them
constexpr int kTravTrips = 21, kLoopTrips = 22, kLaneSteps = 23;
// STATS flavour, coherence of the FAST loop's vector-memory fetches (lane
// counts): wide nodes read from global memory, and those read while every
// active lane of the wave read the same node; primitive tests, and those in
// which every active lane tested the same primitive (a wave-uniform address
// could come through the scalar cache instead of the vector data return)
constexpr int kGlobalNodes = 24, kUniformNodes = 25, kPrimLaneTests = 26, kUniformPrims = 27;
// STATS: attenuation-stack rows written to / read from global memory (rows past
// the LDS ones): with the chunk sums, the loop's HBM writes
constexpr int kAttWrites = 28, kAttReads = 29;
// STATS: FAST traversal stack entries written to the global rows (deep trees:
// rows past the LDS ones, 32-bit entries)
constexpr int kStackOvfWrites = 30;
// scheduling probe: the loop iterations in which some lane of the wave ran a
// rayColor step, summed over the waves (with kReflections, kBackground and
// kDepthHits, the steps run: the probe's lane efficiency, auto_sync)
constexpr int kProbeTrips = 31;
// STATS: the FAST loops' vector-memory wave-instructions by shape (wave-level
// event counts, not lane counts): the inputs of bench.py's data-return model
// (DESIGN.md §4 "The data-return model"), priced per shape by
// tools/ubench_shapes.hip.  Wave trips that read a global wide node through the
// vector path (8 dwordx4 loads but for the last: 7) and the distinct nodes they
// read; trips that read one through the scalar cache; leaf trips that read a
// node's second refs (one flat dwordx4); wave trips of vector primitive tests and
// their distinct primitives; scalar primitive tests; shade records read through
// the vector path; attenuation rows written to / read from global memory.
// kVNodeCost / kVPrimCost: the same trips' sum of max(16, distinct records) - the
// data-return cycles of one of their dwordx4 loads (ubench_shapes: 16 per
// wave-instruction up to 16 distinct 64-B lines, one per line beyond)
constexpr int kVNodeTrips = 32, kVNodeLines = 33, kSNodeTrips = 34, kRbTrips = 35, kVPrimTrips = 36,
              kVPrimLines = 37, kSPrimTrips = 38, kVShadeTrips = 39, kAttWTrips = 40, kAttRTrips = 41,
              kVNodeCost = 42, kVPrimCost = 43;

// ZRT_PROFILE builds (diagnostic only, never the shipped library) add s_memtime
// cycle sums per loop section into counters[kProfSlot + section].
#ifndef ZRT_PROFILE
#define ZRT_PROFILE 0
#endif
__device__ __forceinline__ uint64_t prof_stamp() {
  uint64_t t = 0;
#if ZRT_PROFILE
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
#endif
  return t;
}

constexpr int kBlock = 256;
#ifndef ZRT_PROBE_SPP
#define ZRT_PROBE_SPP 1  // samples per pixel of the scheduling probe; A/B at N=8: 1, 2, 4, 8 give the same render launch
#endif
#ifndef ZRT_LIST_SCALAR
#define ZRT_LIST_SCALAR 1  // list mode reads its (wave-uniform) surfaces with scalar loads
#endif
#ifndef ZRT_OCT_COPIES
#define ZRT_OCT_COPIES 1  // the wide tree stored once per ray octant (0: one copy, planes selected per ray)
#endif
#ifndef ZRT_ORDER_EXACT
#define ZRT_ORDER_EXACT 1  // FAST / BINARY: re-trace order-hazard rays the reference's way (0: A/B only, not exact)
#endif
#ifndef ZRT_LEAF_LOOP
#define ZRT_LEAF_LOOP 1  // 16-bit stack too: opened leaves walked in one loop (one copy of the primitive tests)
#endif
#ifndef ZRT_HAZARD_ENTRY
#define ZRT_HAZARD_ENTRY 1  // also replay rays whose best hit lies below its own leaf's loose entry
#endif
#ifndef ZRT_LDS_TOP
#define ZRT_LDS_TOP 1  // FAST: the wide tree's top levels read from LDS (0: A/B, every node from global memory)
#endif
#ifndef ZRT_LANE_LDS
#define ZRT_LANE_LDS 1  // lockstep FAST loop: RNG state, chunk sums, sample and depth kept in LDS across the traversal
#endif
#ifndef ZRT_LANE_OD
#define ZRT_LANE_OD 0  // lockstep FAST loop: the ray's origin and direction parked with the lane state too
                       // (25 spills instead of 26; C4 53.6 vs 53.9 Gray/s, profiles/r06/r06c)
#endif
#ifndef ZRT_STACK_ROWS_LOCK
#define ZRT_STACK_ROWS_LOCK 16  // lockstep FAST loop: traversal stack rows in LDS (deeper rows in global memory)
#endif
#ifndef ZRT_SYNC_SAMPLES
#define ZRT_SYNC_SAMPLES 1  // the lanes of a wave wait for each other every this many samples
#endif

// ---------------------------------------------------------------------------
// RNG: std.rand DefaultPrng restated per (pixel, sample)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
__device__ __forceinline__ uint64_t splitmix_next(uint64_t& s) {
  s += 0x9e3779b97f4a7c15ULL;
  uint64_t z = s;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

template <int PRNG>
struct Rng;

template <>
struct Rng<ZRT_PRNG_XOROSHIRO128> {
  uint64_t s0, s1;
  __device__ __forceinline__ void init(uint64_t key) {
    uint64_t g = key;
    s0 = splitmix_next(g);
    s1 = splitmix_next(g);
  }
  __device__ __forceinline__ uint64_t next() {  // Xoroshiro128+
    const uint64_t a = s0;
    uint64_t b = s1;
    const uint64_t r = a + b;
    b ^= a;
    s0 = rotl64(a, 55) ^ b ^ (b << 14);
    s1 = rotl64(b, 36);
    return r;
  }
};

template <>
struct Rng<ZRT_PRNG_XOSHIRO256> {
  uint64_t s[4];
  __device__ __forceinline__ void init(uint64_t key) {
    uint64_t g = key;
    s[0] = splitmix_next(g);
    s[1] = splitmix_next(g);
    s[2] = splitmix_next(g);
    s[3] = splitmix_next(g);
  }
  __device__ __forceinline__ uint64_t next() {  // Xoshiro256++
    const uint64_t r = rotl64(s[0] + s[3], 23) + s[0];
    const uint64_t t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl64(s[3], 45);
    return r;
  }
};

// Random.float(f32) / Random.boolean()
template <class R>
__device__ __forceinline__ float rand_float(R& r) {
  const uint32_t s = (uint32_t)r.next();
  return __uint_as_float((0x7fu << 23) | (s >> 9)) - 1.0f;
}
template <class R>
__device__ __forceinline__ bool rand_bool(R& r) {
  return (r.next() & 1u) != 0;
}
// r = c ? t : r, word by word (a lane keeps the state it advanced only where it drew)
template <class R>
__device__ __forceinline__ void rng_keep(R& r, const R& t, bool c) {
  uint32_t a[sizeof(R) / 4], b[sizeof(R) / 4];
  __builtin_memcpy(a, &r, sizeof(a));
  __builtin_memcpy(b, &t, sizeof(b));
#pragma unroll
  for (uint32_t k = 0; k < sizeof(R) / 4; ++k) a[k] = c ? b[k] : a[k];
  __builtin_memcpy(&r, a, sizeof(a));
}

// ---------------------------------------------------------------------------
// small vector helpers (evaluation order as vector.zig)
// ---------------------------------------------------------------------------
struct V3 {
  float x, y, z;
};
__device__ __forceinline__ V3 mk(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ V3 cross(V3 u, V3 v) {
  return mk(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}
__device__ __forceinline__ V3 add(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 scale(V3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ V3 neg(V3 a) { return mk(-a.x, -a.y, -a.z); }
#ifndef ZRT_FD_UNIT  // per-site switches of the short divisions (A/B and register-pressure probes)
#define ZRT_FD_UNIT ZRT_FAST_DIV
#endif
#ifndef ZRT_FD_INV
#define ZRT_FD_INV ZRT_FAST_DIV
#endif
#ifndef ZRT_FD_TRI
#define ZRT_FD_TRI ZRT_FAST_DIV
#endif
__device__ __forceinline__ V3 unit(V3 v) {  // vector.zig:88-92
  const float l = dev::sqrt_rn(v.x * v.x + v.y * v.y + v.z * v.z);
  // v.k / l as dev::div_core over one reciprocal of l (12 VALU instead of 30):
  // bit-identical to the three IEEE divisions while l lies in [2^-50, 2^50] and
  // every quotient in [2^-51, 1]; a zero / tiny component or a degenerate l takes
  // the IEEE divisions (zero's sign, NaN of 0/0, inf)
  // (the range is checked on the operands, |v.k| >= l * 2^-50, before any quotient
  // exists, so each component's three steps need two registers at a time)
  const float vmin = __builtin_fminf(__builtin_fminf(__builtin_fabsf(v.x), __builtin_fabsf(v.y)), __builtin_fabsf(v.z));
  if (__builtin_expect(ZRT_FD_UNIT && l >= 0x1p-50f && l <= 0x1p50f && vmin >= l * 0x1p-50f, 1)) {
    const float y = dev::rcp_core(l);
    return mk(dev::div_core(v.x, l, y), dev::div_core(v.y, l, y), dev::div_core(v.z, l, y));
  }
  return mk(v.x / l, v.y / l, v.z / l);
}
// 1/d of aabb.zig:112 (one IEEE division per axis), bit for bit: dev::rcp_core
// while every |d.k| lies in [2^-126, 2^126), else the IEEE divisions
__device__ __forceinline__ void inv_dir(float dx, float dy, float dz, float& ix, float& iy, float& iz) {
  const float lo = __builtin_fminf(__builtin_fminf(__builtin_fabsf(dx), __builtin_fabsf(dy)), __builtin_fabsf(dz));
  const float hi = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(dx), __builtin_fabsf(dy)), __builtin_fabsf(dz));
  if (__builtin_expect(ZRT_FD_INV && lo >= 0x1p-126f && hi < 0x1p126f, 1)) {
    ix = dev::rcp_core(dx);
    iy = dev::rcp_core(dy);
    iz = dev::rcp_core(dz);
  } else {
    ix = 1.0f / dx;
    iy = 1.0f / dy;
    iz = 1.0f / dz;
  }
}
// 1/det of triangle.zig:63 for det >= 1e-6 (the only dets the hit test uses).
// `fast` (wave-uniform, RayT::rcp_det): the scene's triangles keep det below
// 2^126, so dev::rcp_core needs no per-lane guard (a per-lane branch here, in the
// leaf loop, cost the FAST kernel 4 spilled VGPRs)
__device__ __forceinline__ float inv_det_rn(float det, uint32_t fast) {
  if (ZRT_FD_TRI && fast) return dev::rcp_core(det);
  return 1.0f / det;
}
__device__ __forceinline__ V3 reflect(V3 v, V3 n) { return sub(v, scale(n, 2.0f * dot(v, n))); }
__device__ __forceinline__ V3 refract(V3 v, V3 n, float ratio) {  // vector.zig:132-137
  const float cos_theta = dev::fmin_z(dot(neg(v), n), 1.0f);
  const V3 perp = scale(add(v, scale(n, cos_theta)), ratio);
  const V3 par = scale(n, -dev::sqrt_rn(__builtin_fabsf(1.0f - (perp.x * perp.x + perp.y * perp.y + perp.z * perp.z))));
  return add(perp, par);
}

// ---------------------------------------------------------------------------
// traversal
// ---------------------------------------------------------------------------
struct RayT {
  float ox, oy, oz;
  float ix, iy, iz;  // 1/d per axis (aabb.zig:112 computes it per test; same bits)
  float dx, dy, dz;
  // 1 when every triangle of the scene has |n| < 2^125 (host check), so a det of
  // triangle.zig:61 that passes det >= 1e-6 lies in dev::rcp_core's range; a
  // wave-uniform value (from KArgs), so the choice below is a scalar branch
  uint32_t rcp_det;
  // the scene's grazing-margin coefficients (KArgs::graze_m / graze_leaf, 2^-18 by
  // default): inner slots / leaf slots; wave-uniform, so they stay in SGPRs
  float gm, gl;
  float gk;  // the grazing-triangle guard's coefficient (KArgs::guard; 0: off), wave-uniform
};

// A computed primitive hit lies outside its own box: a triangle's by a few ulps
// of the coordinates involved, about 2^-23 x (t + the triangle's largest
// |coordinate|) (|o| <= t + that, so the origin adds nothing); a sphere's only
// along the ray (its point is o + t d), i.e. by its error in t.  In t that is
// the distance times |1/d_k| on the axis it is measured along, unbounded for a
// ray (nearly) parallel to a box face: the relative margin alone culled boxes the
// reference opens and hits in (DESIGN.md §3 "Grazing rays").  So:
// * the t-proportional part: every narrowed cull's relative margin is
//   1 + 2^-16 + 2^-18 max_k |1/d_k| (ray_rel, per ray);
// * the coordinate part, inner wide slots: their boxes are stored grown by
//   2^-19 x their own largest |coordinate| (accel_build.cpp), which grows each
//   axis's t interval by exactly that distance x |1/d_k|, at no cost per node;
// * the coordinate part, reference boxes (leaf slots, the BINARY traversal, the
//   replay), which stay bit for bit: a uniform slack 2^-18 x the triangles'
//   largest |coordinate| x max_k |1/d_k| (ray_slack).  A leaf slot failing the
//   narrowed test by less is decided by loose_slot: the reference's own
//   per-axis test, and the narrowed test of the leaf's box grown by its own
//   coordinates.
// On the grazing rays no hit lies outside its box's t interval by more than 0.72
// of half these margins (tools/grazing_excess.py).
#ifndef ZRT_GRAZE_SLACK
#define ZRT_GRAZE_SLACK 1  // 0: A/B only (round-2 margins, not exact on grazing rays)
#endif
#ifndef ZRT_GROW
#define ZRT_GROW ZRT_GRAZE_SLACK  // A/B only: 0 stores inner boxes ungrown (not exact)
#endif
#ifndef ZRT_REL_M
#define ZRT_REL_M ZRT_GRAZE_SLACK  // A/B only: 0 keeps the constant relative margin (not exact)
#endif
#ifndef ZRT_LEAF_SLACK
#define ZRT_LEAF_SLACK ZRT_GRAZE_SLACK  // A/B only: 0 drops the leaf slots' slack (not exact)
#endif
// (recomputed where used from 1/d, 1 VALU each, rather than kept in VGPRs across
// the traversal: two more live registers cost the deep-tree loop spills)
__device__ __forceinline__ float ray_m(const RayT& r) {  // max_k |1/d_k|
  return __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(r.ix), __builtin_fabsf(r.iy)), __builtin_fabsf(r.iz));
}
// relative margin of every narrowed cull: 1 + 2^-16 + 2^-18 m
__device__ __forceinline__ float ray_rel(const RayT& r, float m) { return ZRT_REL_M ? 1.0000153f + r.gm * m : 1.0000153f; }
// the reference boxes' slack: 2^-18 x the triangles' largest |coordinate| x m
__device__ __forceinline__ float ray_slack(const RayT& r, float extent, float m) {
  return ZRT_LEAF_SLACK ? __builtin_fmaxf(extent, 0x1p-100f) * r.gm * m : 0.0f;
}

// Nearly axis-parallel rays (DESIGN.md §3 "Per-axis margins").  The margins
// above are t-space terms scaled by m = max_k |1/d_k| on every axis, but a hit's
// excess beyond its box is a distance in space: e (t + coordinates), on axis k
// e (t + coordinates) |1/d_k| in t.  Only an axis the ray runs (nearly) parallel
// to needs the large term; applied to all three it turns the narrowed cull off
// (m = 2^20: every exit x 5) and such a ray walks most of the tree.  A wave with
// a lane whose m exceeds kPaxisM (a wave-uniform branch) therefore widens each
// axis of every slot by its own term g |1/d_k|, g = 2^-18 (T + extent) (T: the
// ray's farthest distance to the triangles' box, which bounds the hit's t; extent:
// the triangles' largest |coordinate|, ray_slack's spatial term) - 6 more adds
// per slot, for waves with such a lane only; the other waves keep ray_rel with
// m <= kPaxisM.
#ifndef ZRT_GRAZE_LEAF
#define ZRT_GRAZE_LEAF 0  // leaf slots' relative margin from its own coefficient (KArgs::graze_leaf; A/B of a
                          // leaf-only guard: fixed none of the grazing-triangle misses, C4 -4 %, profiles/r04/r04c)
#endif
#ifndef ZRT_PAXIS
#define ZRT_PAXIS 1  // 0: A/B only (every wave on the t-space margins of ray_rel / ray_slack)
#endif
#ifndef ZRT_PAXIS_LOCK
#define ZRT_PAXIS_LOCK 0  // the lockstep loop too (its 96-VGPR budget spills 7 -> 28 registers with the branch: C4 -2.8 %)
#endif
#ifndef ZRT_PAXIS_LOG2M
#define ZRT_PAXIS_LOG2M 10
#endif
constexpr float kPaxisM = float(1u << ZRT_PAXIS_LOG2M);
__device__ __forceinline__ float paxis_grow(const KArgs& a, const RayT& r) {
  const float T = (__builtin_fabsf(r.ox - a.tri_c[0]) + a.tri_h[0]) + (__builtin_fabsf(r.oy - a.tri_c[1]) + a.tri_h[1]) +
                  (__builtin_fabsf(r.oz - a.tri_c[2]) + a.tri_h[2]);  // >= the L2 distance to any corner
  return (T + __builtin_fmaxf(a.scene_extent, 0x1p-100f)) * (r.gm * 1.0000153f);  // (rounding of T: the extra 2^-16)
}
// the per-axis term in t, finite (an infinite 1/d_k keeps the slab's exact +-inf:
// the reference's own test then rejects every leaf off the plane)
__device__ __forceinline__ float paxis_t(float g, float inv) {
  return __builtin_fminf(g * __builtin_fabsf(inv), 0x1p126f);
}
// The grazing-triangle guard's spatial widening for this ray: gk (T + extent)
// (T as in paxis_grow bounds |o - a| for every triangle vertex a): the reach of
// an accepted hit beyond its triangle, k |ao| + k_c (DESIGN.md §3 "Triangles").
#ifndef ZRT_GUARD
#define ZRT_GUARD 1
#endif
__device__ __forceinline__ float guard_grow(const KArgs& a, const RayT& r) {
  const float T = (__builtin_fabsf(r.ox - a.tri_c[0]) + a.tri_h[0]) + (__builtin_fabsf(r.oy - a.tri_c[1]) + a.tri_h[1]) +
                  (__builtin_fabsf(r.oz - a.tri_c[2]) + a.tri_h[2]);
  return (T + __builtin_fmaxf(a.scene_extent, 0x1p-100f)) * (r.gk * 1.0000153f);
}

// aabb.zig:109-127: each axis against [t_min, t_max] on its own.
// FAST additionally narrows the interval across axes (with a 2^-16 relative
// margin) and reports the entry distance for near-first ordering.
// gw: the grazing-triangle guard's spatial widening of the narrowed test (per
// axis gw |1/d_k|; 0: none) - the loose test stays the reference's own
template <bool FAST>
__device__ __forceinline__ bool box_test(const float4 lo, const float4 hi, const RayT& r, float t_max,
                                         float* entry, float slack = 0.0f, bool narrow = true, float gw = 0.0f) {
  const float t_min = 0.001f;
  float a0 = (lo.x - r.ox) * r.ix, a1 = (hi.x - r.ox) * r.ix;
  float b0 = (lo.y - r.oy) * r.iy, b1 = (hi.y - r.oy) * r.iy;
  float c0 = (lo.z - r.oz) * r.iz, c1 = (hi.z - r.oz) * r.iz;
  if (r.ix < 0.0f) { const float t = a0; a0 = a1; a1 = t; }
  if (r.iy < 0.0f) { const float t = b0; b0 = b1; b1 = t; }
  if (r.iz < 0.0f) { const float t = c0; c0 = c1; c1 = t; }
  // math.max(t0, t_min) / math.min(t1, t_max) are `x > y ? x : y` / `x < y ? x : y`.
  // With a non-NaN second operand (t_min, t_max never are) these equal IEEE
  // maxNum / minNum (v_max_f32 / v_min_f32) for every NaN first operand, and
  // differ only in the sign of a zero result, which no comparison below sees.
  const float an = __builtin_fmaxf(a0, t_min), ax = __builtin_fminf(a1, t_max);
  const float bn = __builtin_fmaxf(b0, t_min), bx = __builtin_fminf(b1, t_max);
  const float cn = __builtin_fmaxf(c0, t_min), cx = __builtin_fminf(c1, t_max);
  bool ok = (ax > an) && (bx > bn) && (cx > cn);  // !(tmax <= tmin) for every axis
  if (FAST) {
    const float en = __builtin_fmaxf(__builtin_fmaxf(an, bn), cn);
    const float ex = __builtin_fminf(__builtin_fminf(ax, bx), cx);
    if (__builtin_expect(gw > 0.0f, 0)) {  // (a scalar branch: gw is the scene's guard)
      const float wa = paxis_t(gw, r.ix), wb = paxis_t(gw, r.iy), wc = paxis_t(gw, r.iz);
      const float enw = __builtin_fmaxf(__builtin_fmaxf(a0 - wa, b0 - wb), __builtin_fmaxf(c0 - wc, t_min));
      const float exw = __builtin_fminf(__builtin_fminf(a1 + wa, b1 + wb), __builtin_fminf(c1 + wc, t_max));
      ok = ok && (!narrow || !(enw > __builtin_fmaf(exw, ray_rel(r, ray_m(r)), slack)));
    } else {
      ok = ok && (!narrow || !(en > __builtin_fmaf(ex, ray_rel(r, ray_m(r)), slack)));
    }
    *entry = en;
  }
  return ok;
}

__device__ __forceinline__ int as_int(float f) { return __float_as_int(f); }

// Order hazards.  The reference tests each leaf against the best
// hit of the leaves before it in its DFS order, so the hit FAST finds closest is
// one the reference never reaches when a hit of another leaf lies between it and
// its own leaf's loose entry (the two roundings disagree at shared vertices on a
// box face).  TRACK flags such near ties in the sign bit of best_t (a hit's t is
// > t_min > 0; every reader takes |best_t|, a free source modifier), so the
// flag costs no register: set when another hit lies within kNearTie of the best.
constexpr float kNearTie = 1.00006104f;  // 1 + 2^-14
// FAST opens every box whose entry lies below best * kOpen: 1 + 2^-12 (exact in
// f32).  With the near-tie band f = 2^-14 this is exact for any scene whose
// primitive hits lie in their leaf's box up to a relative m < 2^-12 - 2^-14
// ("Exactness"; the REFERENCE traversal's STATS flavour
// measures m: zrt_stats.box_excess_max_*).  Round 1 used 1 + 2^-16 here, which
// left the verdict's band (1 + 2^-15, 1 + 2^-14] unguarded.
#ifndef ZRT_OPEN_MARGIN
#define ZRT_OPEN_MARGIN 1.000244140625f  // A/B only: 1.0000153f reproduces round 1
#endif
constexpr float kOpen = ZRT_OPEN_MARGIN;

template <bool TIE, bool TRACK>
__device__ __forceinline__ void accept_hit(float t, int slot, float& best_t, int& best, const RayT& r,
                                           float entry) {
  if (!TRACK) {
    const bool in_range = TIE ? (t < best_t || (t == best_t && slot < best)) : (t < best_t);
    if (in_range) {
      best_t = t;
      best = slot;
    }
    return;
  }
  const float bt = __builtin_fabsf(best_t);
  if (t < bt || (t == bt && slot < best)) {
    bool near = t < bt ? bt <= t * kNearTie : best_t < 0.0f;  // an equal-t swap keeps the flag
    // FAST: the leaf's loose entry E (aabb.zig:109-127, >= t_min > 0; the slot's
    // `en` of wide_iter, bit for bit) above the hit by more than the band also
    // flags the ray; entry < 0: no leaf entry to check (the other traversals)
    near = near || entry > t * kNearTie;
    best_t = near ? -t : t;
    best = slot;
  } else if (t > bt && t <= bt * kNearTie) {
    best_t = -bt;
  }
}

// Triangle.hit (triangle.zig:48-70) for the candidate slot; accepts when the
// reference would (det >= 1e-6, t_min < t < t_max, u,v >= 0, u+v <= 1), with
// equal-t ties going to the lower slot (= earlier in the reference's DFS).
template <bool TIE, bool TRACK = false>
__device__ __forceinline__ void tri_test_v(const float4 p0, const float4 p1, const float4 p2, int slot,
                                           const RayT& r, float& best_t, int& best, float entry = -1.0f) {
  const V3 n = mk(p2.y, p2.z, p2.w);
  const V3 d = mk(r.dx, r.dy, r.dz);
  const float det = -dot(d, n);
  if (!(det >= 1e-6f)) return;
  const float inv_det = inv_det_rn(det, r.rcp_det);
  const V3 ao = mk(r.ox - p0.x, r.oy - p0.y, r.oz - p0.z);
  const V3 dao = cross(ao, d);
  const V3 e1 = mk(p0.w, p1.x, p1.y);
  const V3 e2 = mk(p1.z, p1.w, p2.x);
  const float u = dot(e2, dao) * inv_det;
  const float v = -dot(e1, dao) * inv_det;
  const float t = dot(ao, n) * inv_det;
  if (t > 0.001f && u >= 0.0f && v >= 0.0f && (u + v) <= 1.0f) accept_hit<TIE, TRACK>(t, slot, best_t, best, r, entry);
}

template <bool TIE, bool TRACK = false>
__device__ __forceinline__ void tri_test(const float4* __restrict__ prims, int slot, const RayT& r,
                                         float& best_t, int& best, float entry = -1.0f) {
  tri_test_v<TIE, TRACK>(prims[3 * slot + 0], prims[3 * slot + 1], prims[3 * slot + 2], slot, r, best_t, best,
                         entry);
}

// Sphere.hit (sphere.zig:31-41, 53-56): nearest root in (t_min, t_max).
template <bool TIE, bool TRACK = false>
__device__ __forceinline__ void sphere_test(const float4 c, int slot, const RayT& r, float& best_t,
                                            int& best, float entry = -1.0f) {
  const V3 oc = mk(r.ox - c.x, r.oy - c.y, r.oz - c.z);
  const V3 d = mk(r.dx, r.dy, r.dz);
  const float half_b = dot(oc, d);
  const float cc = (oc.x * oc.x + oc.y * oc.y + oc.z * oc.z) - c.w;  // c.w = RN(r * r)
  const float disc = half_b * half_b - cc;
  if (disc < 0.0f) return;
  const float root = dev::sqrt_rn(disc);
  const float t1 = -half_b - root;
  const float t = (t1 > 0.001f) ? t1 : (-half_b + root);
  if (t > 0.001f) accept_hit<TIE, TRACK>(t, slot, best_t, best, r, entry);
}

template <bool TIE, bool STATS, bool TRACK = false>
__device__ __forceinline__ void prim_test(const float4* __restrict__ prims, int ref, const RayT& r,
                                          float& best_t, int& best, uint32_t& c_tri, uint32_t& c_sph,
                                          float entry = -1.0f) {
  const int code = -ref - 1;
  const int slot = code >> 1;
  if (code & 1) {
    if (STATS) ++c_tri;
    tri_test<TIE, TRACK>(prims, slot, r, best_t, best, entry);
  } else {
    if (STATS) ++c_sph;
    sphere_test<TIE, TRACK>(prims[3 * slot], slot, r, best_t, best, entry);
  }
}

#ifndef ZRT_SORT_SKIP
#define ZRT_SORT_SKIP 1  // FAST: skip the inner-child sort when no lane of the wave has two children to order
#endif
#ifndef ZRT_Q_GLOBAL
#define ZRT_Q_GLOBAL 0  // lockstep FAST loop: the current node's pointer always its global copy (A/B: exact,
                        // C4 -0.5 %, C3 +-0, profiles/r06/r06q2)
#endif
#ifndef ZRT_MATS_LDS_ONLY
// the lockstep and list-lane loops read the material table from their LDS copy only,
// through LDS-typed pointers (ds_read), not a generic pointer chosen at run time (flat
// loads); the host plans the table into LDS first and falls back to the wavefront /
// wave-unit list loop when it does not fit (C4 +1.5 %, C2 +0.5 %: profiles/r06/r06l)
#define ZRT_MATS_LDS_ONLY 1
#endif
#ifndef ZRT_STACK_LDS_FAST
#define ZRT_STACK_LDS_FAST 2  // FAST, while every lane's stack is in its LDS rows: 2 the pops as ds_reads in the
                              // usual branches (C3 +1.6-2.4 %, C4 +0.3 %: profiles/r06/r06w), 1 push / pop as
                              // LDS selects (A/B: C3 +1.3 %, C4 ±0.3 %), 0 the generic pop only
#endif
#ifndef ZRT_SCALAR_NODES
#define ZRT_SCALAR_NODES 1  // FAST: a wide node every active lane reads next comes through the scalar cache
#endif
#ifndef ZRT_POOL_SCALAR
#define ZRT_POOL_SCALAR 0  // path-pool loop: a node every traversing lane reads next comes through the scalar cache
#endif
#ifndef ZRT_SCALAR_RB
#define ZRT_SCALAR_RB 0  // FAST: a wave-uniform node's second refs through the scalar cache (exact; C4 -2.4 %,
                         // C3 -1.9 %, profiles/r06/r06o: less data-return work, more issue)
#endif
#ifndef ZRT_LOCK_QN
#define ZRT_LOCK_QN 0  // A/B: the lockstep FAST loop over the compressed 64-B nodes (wide_iter_q)
#endif
#ifndef ZRT_SCALAR_PRIMS
#define ZRT_SCALAR_PRIMS 1  // FAST: a primitive every active lane tests is read through the scalar cache
#endif
// prim_test for a WAVE-UNIFORM ref: the record is read with scalar loads
// (s_load through the constant address space), so the 48 bytes do not cross
// the vector data return (TD), which is what the FAST loop saturates (DESIGN.md
// §4); on the bunny 89 % of the leaf trips test one primitive in every active
// lane (tools/simd_eff.py uniform_prim_frac).  Same arithmetic as prim_test.
template <bool TIE, bool STATS, bool TRACK = false>
__device__ __forceinline__ void prim_test_uniform(const float4* __restrict__ prims, int ref, const RayT& r,
                                                  float& best_t, int& best, uint32_t& c_tri, uint32_t& c_sph,
                                                  float entry = -1.0f) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef const __attribute__((address_space(4))) float4 cfloat4;
  cfloat4* cp = (cfloat4*)prims;
#else
  const float4* cp = prims;
#endif
  const int code = -ref - 1;
  const int slot = code >> 1;
  if (code & 1) {
    if (STATS) ++c_tri;
    tri_test_v<TIE, TRACK>(cp[3 * slot + 0], cp[3 * slot + 1], cp[3 * slot + 2], slot, r, best_t, best, entry);
  } else {
    if (STATS) ++c_sph;
    sphere_test<TIE, TRACK>(cp[3 * slot], slot, r, best_t, best, entry);
  }
}

// The reference's loose entry of a box (aabb.zig:109-127): the largest per-axis
// max(t0, t_min) after the swap of aabb.zig:116-118, the t_max a test of the box
// needs to exceed.
__device__ __forceinline__ float loose_entry(const float4 lo, const float4 hi, const RayT& r) {
  const float nx = ((r.ix < 0.0f ? hi.x : lo.x) - r.ox) * r.ix;
  const float ny = ((r.iy < 0.0f ? hi.y : lo.y) - r.oy) * r.iy;
  const float nz = ((r.iz < 0.0f ? hi.z : lo.z) - r.oz) * r.iz;
  return __builtin_fmaxf(__builtin_fmaxf(nx, ny), __builtin_fmaxf(nz, 0.001f));
}

// Order hazard of a hit found by a near-first traversal (best_t's sign cleared
// here): a near tie was flagged (the reference may reach the other hit first and
// then reject the best's leaf), or the loose entry E of the best's own reference
// leaf lies above the best hit by more than the near-tie band (hits in leaves
// culled against the best could then be below E).  Such rays are traced again
// the reference's way.
template <bool ENTRY>
__device__ __forceinline__ bool order_hazard(const KArgs& a, const RayT& r, float& best_t, int best) {
  const bool near = best_t < 0.0f;
  best_t = __builtin_fabsf(best_t);
  if (best < 0) return false;
  if (near || !ENTRY) return near;  // FAST folds the entry test into the flag (accept_hit)
#if ZRT_HAZARD_ENTRY
  const uint32_t leaf = a.leaf_of_slot[best];  // the reference BVH node holding slot `best`
  const float e = loose_entry(a.nodes[2 * leaf], a.nodes[2 * leaf + 1], r);
  return e > best_t * kNearTie;
#else
  (void)a; (void)r;
  return false;
#endif
}

// The geometry of a primitive hit alone (t_max = inf): its t, or +inf.  Used by
// the REFERENCE traversal's STATS flavour to measure how far the hits the
// reference computes lie outside their own leaf's box (box_excess_*).
__device__ __forceinline__ float prim_hit_t(const float4* __restrict__ prims, int ref, const RayT& r) {
  const int code = -ref - 1;
  const int slot = code >> 1;
  float t = __builtin_inff();
  int b = -1;
  if (code & 1) tri_test<false>(prims, slot, r, t, b);
  else sphere_test<false>(prims[3 * slot], slot, r, t, b);
  return t;
}

// max(E / t - 1, t / X - 1) for a hit t in a leaf whose loose entry is E and
// whose exit (min over axes of the far slab distance) is X: > 0 when the
// rounded hit lies before the box's entry or past its exit.
__device__ __forceinline__ float box_excess(const float4 lo, const float4 hi, const RayT& r, float t) {
  const float e = loose_entry(lo, hi, r);
  const float xx = ((r.ix < 0.0f ? lo.x : hi.x) - r.ox) * r.ix;
  const float xy = ((r.iy < 0.0f ? lo.y : hi.y) - r.oy) * r.iy;
  const float xz = ((r.iz < 0.0f ? lo.z : hi.z) - r.oz) * r.iz;
  const float x = __builtin_fminf(__builtin_fminf(xx, xy), xz);
  return __builtin_fmaxf(e / t - 1.0f, t / x - 1.0f);
}

struct ExcessAcc {
  float tri = 0.0f, sph = 0.0f;
  uint32_t over = 0;  // hits outside their box by more than 2^-14
  __device__ __forceinline__ void leaf(const float4* __restrict__ prims, const float4 lo, const float4 hi,
                                       const RayT& r, int ra, int rb) {
    for (int k = 0; k < 2; ++k) {
      const int ref = k == 0 ? ra : rb;
      if (k == 1 && rb == ra) break;
      const float t = prim_hit_t(prims, ref, r);
      if (t == __builtin_inff()) continue;
      const float ex = box_excess(lo, hi, r, t);
      if (!(ex > 0.0f)) continue;
      if ((-ref - 1) & 1) tri = __builtin_fmaxf(tri, ex);
      else sph = __builtin_fmaxf(sph, ex);
      over += ex > 6.1035156e-05f ? 1u : 0u;
    }
  }
};

#ifndef ZRT_REPLAY_NARROW
#define ZRT_REPLAY_NARROW 1  // the replay also culls boxes the ray does not cross (0: the reference's test alone)
#endif
#ifndef ZRT_REPLAY_INLINE
#define ZRT_REPLAY_INLINE 1
#endif
#if ZRT_REPLAY_INLINE
#define ZRT_REPLAY_ATTR __forceinline__
#else
#define ZRT_REPLAY_ATTR __noinline__
#endif
// A ray whose origin lies where the wide tree's sphere growth was sized for
// (KArgs::origin_bound, DESIGN.md §3 "Spheres"); other rays (none in a render of
// the reference's scenes: their cameras lie inside that region) are traced the
// reference's way alone.
#ifndef ZRT_ORIGIN_CHECK
#define ZRT_ORIGIN_CHECK 1  // A/B only: 0 drops the check (not exact for origins outside the bound)
#endif
__device__ __forceinline__ bool ray_origin_ok(const KArgs& a, const RayT& r) {
  if (!ZRT_ORIGIN_CHECK || !a.check_origins) return true;  // (wave-uniform: a scalar branch)
  const float m = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(r.ox - a.root_c[0]), __builtin_fabsf(r.oy - a.root_c[1])),
                                  __builtin_fabsf(r.oz - a.root_c[2]));
  return m <= a.origin_bound;
}

// The reference's traversal (bvh.zig:187-205) for a ray FAST flagged: left-first
// over the reference BVH, every box through the reference's loose test against the
// current best, so every leaf is accepted or rejected as the reference does.
// narrow: also cull boxes the ray does not cross (the narrowed test with the
// grazing slack) - except boxes holding a sphere, whose rounded
// test reaches beyond the sphere (KArgs::ref_sph); false: the reference's test alone.
template <class StackT>
__device__ ZRT_REPLAY_ATTR void reference_replay(const KArgs& a, const RayT& r, StackT* __restrict__ stk, uint32_t gl,
                                              float& best_t, int& best, bool narrow = true) {
  const uint32_t rows = a.lds_rows, cap = a.ref_stack;
  StackT* __restrict__ ovf = reinterpret_cast<StackT*>(a.stack_ovf) + gl;
  const float slack = ray_slack(r, a.scene_extent, ray_m(r));
  const float gw = ZRT_GUARD && r.gk > 0.0f ? guard_grow(a, r) : 0.0f;  // the grazing-triangle guard
  best_t = __builtin_inff();
  best = -1;
  uint32_t c_tri = 0, c_sph = 0;
  stk[0] = 0;
  uint32_t sp = 1;
  while (sp > 0) {
    --sp;
    const int idx = sp < rows ? (int)stk[sp * kBlock] : (int)ovf[(size_t)(sp - rows) * a.n_lanes];
    const float4 lo = a.nodes[2 * idx], hi = a.nodes[2 * idx + 1];
    float e;
    // the reference's loose test against the current best, and FAST's narrowed
    // emptiness test (a box the ray does not cross holds no hit):
    // left-first with the reference's t_max, so every leaf is accepted or
    // rejected exactly as the reference does it, in ~1 % of its node visits
    if (!box_test<ZRT_REPLAY_NARROW>(lo, hi, r, best_t, &e, slack, narrow && a.ref_sph[idx] == 0, gw)) continue;
    const int left = as_int(lo.w), right = as_int(hi.w);
    if (left < 0) {
      prim_test<false, false>(a.prims, left, r, best_t, best, c_tri, c_sph);
      if (right != left) prim_test<false, false>(a.prims, right, r, best_t, best, c_tri, c_sph);
    } else if (sp + 2 <= cap) {
      const StackT v[2] = {(StackT)right, (StackT)left};
#pragma unroll
      for (uint32_t j = 0; j < 2; ++j) {
        if (sp + j < rows) stk[(sp + j) * kBlock] = v[j];
        else ovf[(size_t)(sp + j - rows) * a.n_lanes] = v[j];
      }
      sp += 2;
    } else {
      atomicOr(a.error_flag, kErrOverflow);
    }
  }
}


// BINARY's node test: the narrowed test with the grazing slack against tb, or,
// for a node whose subtree holds a sphere (KArgs::ref_sph), the reference's loose
// test against t_max = +inf: the rounded sphere test reaches beyond the sphere
// and its box by ~sqrt(u) |oc| and errs by as much in t (DESIGN.md §3 "Spheres").
__device__ __forceinline__ bool binary_test(const KArgs& a, int idx, const float4 lo, const float4 hi, const RayT& r,
                                            float tb, float* e, float slack, float gw) {
  if (a.ref_sph[idx]) return box_test<true>(lo, hi, r, __builtin_inff(), e, 0.0f, false);
  return box_test<true>(lo, hi, r, tb, e, slack, true, gw);
}

// Closest hit over the BVH.  FAST: near-first order with the narrowed slab
// test; REFERENCE: left-first DFS with exactly bvh.zig:187-205's tests.
template <bool FAST, bool STATS, class StackT>
__device__ __forceinline__ void traverse_bvh(const KArgs& a, const RayT& r, StackT* __restrict__ stk,
                                             float& best_t, int& best, uint32_t& c_nodes,
                                             uint32_t& c_tri, uint32_t& c_sph, ExcessAcc* excess = nullptr) {
  const int stride = kBlock;
  uint32_t sp = 0;
  const uint32_t cap = a.stack_depth;
  if (FAST) {
    const float slack = ray_slack(r, a.scene_extent, ray_m(r));
    const float gw = ZRT_GUARD && r.gk > 0.0f ? guard_grow(a, r) : 0.0f;  // the grazing-triangle guard
    float e;
    float4 lo = a.nodes[0], hi = a.nodes[1];
    if (STATS) ++c_nodes;
    if (!binary_test(a, 0, lo, hi, r, __builtin_fabsf(best_t) * kOpen + slack, &e, slack, gw)) {
      if (!ray_origin_ok(a, r)) reference_replay<StackT>(a, r, stk, 0u, best_t, best, false);
      return;
    }
    int left = as_int(lo.w), right = as_int(hi.w);
    for (;;) {
      if (left < 0) {
        prim_test<true, STATS, ZRT_ORDER_EXACT>(a.prims, left, r, best_t, best, c_tri, c_sph);
        if (right != left) prim_test<true, STATS, ZRT_ORDER_EXACT>(a.prims, right, r, best_t, best, c_tri, c_sph);
      } else {
        const float4 l0 = a.nodes[2 * left], l1 = a.nodes[2 * left + 1];
        const float4 r0 = a.nodes[2 * right], r1 = a.nodes[2 * right + 1];
        if (STATS) c_nodes += 2;
        const float tb = __builtin_fabsf(best_t) * kOpen + slack;
        float el, er;
        const bool hl = binary_test(a, left, l0, l1, r, tb, &el, slack, gw);
        const bool hr = binary_test(a, right, r0, r1, r, tb, &er, slack, gw);
        if (hl && hr) {
          const bool rfirst = er < el;
          const int far_idx = rfirst ? left : right;
          if (sp < cap) stk[(sp++) * stride] = (StackT)far_idx;
          else atomicOr(a.error_flag, kErrOverflow);  // too deep for the stack: the subtree is dropped (flagged)
          left = rfirst ? as_int(r0.w) : as_int(l0.w);
          right = rfirst ? as_int(r1.w) : as_int(l1.w);
          continue;
        }
        if (hl) { left = as_int(l0.w); right = as_int(l1.w); continue; }
        if (hr) { left = as_int(r0.w); right = as_int(r1.w); continue; }
      }
      // pop: re-test the node's own box against the (possibly shrunk) best_t
      bool found = false;
      while (sp > 0) {
        --sp;
        const int idx = stk[sp * stride];
        const float4 p0 = a.nodes[2 * idx], p1 = a.nodes[2 * idx + 1];
        if (STATS) ++c_nodes;
        if (binary_test(a, idx, p0, p1, r, __builtin_fabsf(best_t) * kOpen + slack, &e, slack, gw)) {
          left = as_int(p0.w);
          right = as_int(p1.w);
          found = true;
          break;
        }
      }
      if (!found) break;
    }
    // the order hazard of DESIGN.md §3, as in traverse_wide (the stack is all in LDS here)
    if (__builtin_expect(ZRT_ORDER_EXACT && order_hazard<true>(a, r, best_t, best), 0))
      reference_replay<StackT>(a, r, stk, 0u, best_t, best);
    if (__builtin_expect(!ray_origin_ok(a, r), 0)) reference_replay<StackT>(a, r, stk, 0u, best_t, best, false);
  } else {
    stk[0] = 0;
    sp = 1;
    while (sp > 0) {
      --sp;
      const int idx = stk[sp * stride];
      const float4 lo = a.nodes[2 * idx], hi = a.nodes[2 * idx + 1];
      if (STATS) ++c_nodes;
      float e;
      if (!box_test<false>(lo, hi, r, best_t, &e)) continue;
      const int left = as_int(lo.w), right = as_int(hi.w);
      if (left < 0) {
        if (STATS && excess) excess->leaf(a.prims, lo, hi, r, left, right);
        prim_test<false, STATS>(a.prims, left, r, best_t, best, c_tri, c_sph);
        if (right != left) prim_test<false, STATS>(a.prims, right, r, best_t, best, c_tri, c_sph);
      } else {
        if (sp + 2 <= cap) {
          stk[sp * stride] = (StackT)right;
          stk[(sp + 1) * stride] = (StackT)left;
          sp += 2;
        } else {
          atomicOr(a.error_flag, kErrOverflow);
        }
      }
    }
  }
}

// Slab test of child slot k of a wide node: entry distance, or +inf on a miss.
// Every slot gets the narrowed test (entry > exit * (1 + 2^-16) culls; it never
// rejects a box holding a hit closer than best_t).  A leaf slot additionally
// gets the reference's own loose test (aabb.zig:109-127: each axis on its own
// against [t_min, t_max]) - its box is the reference leaf's box bit for bit.
__device__ __forceinline__ float wide_slot(float mnx, float mny, float mnz, float mxx, float mxy, float mxz,
                                           const RayT& r, float tb, bool leaf) {
  const float t_min = 0.001f;
  float a0 = (mnx - r.ox) * r.ix, a1 = (mxx - r.ox) * r.ix;
  float b0 = (mny - r.oy) * r.iy, b1 = (mxy - r.oy) * r.iy;
  float c0 = (mnz - r.oz) * r.iz, c1 = (mxz - r.oz) * r.iz;
  if (r.ix < 0.0f) { const float t = a0; a0 = a1; a1 = t; }
  if (r.iy < 0.0f) { const float t = b0; b0 = b1; b1 = t; }
  if (r.iz < 0.0f) { const float t = c0; c0 = c1; c1 = t; }
  // math.max(t0, t_min) / math.min(t1, t_max) are `x > y ? x : y` / `x < y ? x : y`;
  // with a non-NaN second operand these equal maxNum / minNum for every first
  // operand (a NaN slab bound, (bound - o) * inf with bound == o, then
  // constrains nothing, as in the reference) up to the sign of a zero result,
  // which no comparison below sees.
  const float an = __builtin_fmaxf(a0, t_min), ax = __builtin_fminf(a1, tb);
  const float bn = __builtin_fmaxf(b0, t_min), bx = __builtin_fminf(b1, tb);
  const float cn = __builtin_fmaxf(c0, t_min), cx = __builtin_fminf(c1, tb);
  const float en = __builtin_fmaxf(__builtin_fmaxf(an, bn), cn);
  const float ex = __builtin_fminf(__builtin_fminf(ax, bx), cx);
  bool ok = !(en > ex * ray_rel(r, ray_m(r)));
  if (leaf) ok = ok && (ax > an) && (bx > bn) && (cx > cn);  // !(tmax <= tmin) per axis
  return ok ? en : __builtin_inff();
}

__device__ __forceinline__ void cswap(float& ka, int& ra, float& kb, int& rb) {
  const bool s = kb < ka;
  const float tk = s ? kb : ka;
  const int tr = s ? rb : ra;
  kb = s ? ka : kb;
  rb = s ? ra : rb;
  ka = tk;
  ra = tr;
}

// Two slots' slab distances (bound - o) * inv.  (Written as packed f32,
// v_pk_add_f32 / v_pk_mul_f32 with the same roundings, this traversal ran
// 1.2-1.8x slower: packed f32 issues at half the rate of single f32 here.)
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 slab2(float b0, float b1, float o, float inv) {
  return (f2){(b0 - o) * inv, (b1 - o) * inv};
}

// The same distances as fma(plane, 1/d, -o/d) (ZRT_FMA_SLABS): one rounding
// after an exact product instead of (plane - o) * (1/d)'s two, 24 VALU fewer
// per wide node.  With p = RN(o_k / d_k) such a distance lies within
// 1.0002 u |p| + 3.0001 u |s| of the reference's RN(RN(plane - o) * (1/d))
// (u = 2^-24); wide_iter's culls carry kFmaE2 * max_k |p_k| more slack for it
// (both ends of an interval), the relative margin (>= 2^-16) covers the rest, and
// each decision that must be the reference's own - a leaf's loose test, a sphere
// slot's static test, the hazard entry - is taken from these values only when it
// is certain by that margin (kFmaSure), else from the exact distances recomputed
// from memory (loose_slot / static_ok_slot), as for intervals within the margin.
// A ray with |1/d_k| >= 2^100 or |p_k| >= 2^120 (a direction component ~0) is
// "degenerate": it culls everything here and is traced the reference's way
// (wide_finish, ray_degenerate).
#ifndef ZRT_FMA_SLABS
#define ZRT_FMA_SLABS 1  // 0: the reference's (plane - o) * (1/d) for every slot (A/B)
#endif
constexpr float kFmaE2 = 0x1.04p-23f;   // >= 2 x 1.0002 u (+ the rounding of this product)
constexpr float kFmaSure = 1.0000019f;  // 1 + 2^-19 > 1 + 6.0002 u: relative error of both ends
__device__ __forceinline__ f2 slab2f(float b0, float b1, float p, float inv) {
  return (f2){__builtin_fmaf(b0, inv, -p), __builtin_fmaf(b1, inv, -p)};
}
__device__ __forceinline__ bool ray_degenerate(const RayT& r) {
  if (!ZRT_FMA_SLABS) return false;
  const float pm = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(r.ox * r.ix), __builtin_fabsf(r.oy * r.iy)),
                                   __builtin_fabsf(r.oz * r.iz));
  return !(ray_m(r) < 0x1p100f) || !(pm < 0x1p120f);
}

struct SlotT {
  float en, ex;
};
__device__ __forceinline__ SlotT slot_interval(float nx, float ny, float nz, float fx, float fy, float fz,
                                               float tb) {
  const float t_min = 0.001f;
  SlotT s;
  s.en = __builtin_fmaxf(__builtin_fmaxf(nx, ny), __builtin_fmaxf(nz, t_min));
  s.ex = __builtin_fminf(__builtin_fminf(fx, fy), __builtin_fminf(fz, tb));
  return s;
}
#ifndef ZRT_SPHERE_FIRST
#define ZRT_SPHERE_FIRST 1  // A/B: 0 looks for sphere slots in all four slots of every node
#endif
#ifndef ZRT_SPHERE_SLOTS
#define ZRT_SPHERE_SLOTS 1  // A/B only: 0 culls sphere leaves like triangle leaves (not exact, DESIGN.md §3 "Spheres")
#endif
// The wide-tree encoding these kernels decode (accel_build.hpp kLayout*); the
// host refuses any other before launching, and a kernel handed one anyway sets
// kErrLayout and returns without reading the tree.
constexpr uint32_t kKernelLayout = kLayoutVersion | (ZRT_SPHERE_SLOTS ? kLayoutSphereSlots | kLayoutSphereFirst : 0u);
__device__ __forceinline__ bool layout_ok(const KArgs& a) {
  if (a.layout == kKernelLayout) return true;  // (block-uniform: every thread returns together)
  if (threadIdx.x == 0) atomicOr(a.error_flag, kErrLayout);
  return false;
}
// The reference's loose test (aabb.zig:109-127) with t_max = +inf: every axis's
// (post-swap) slab [n, f] reaches past t_min and is not empty.  max(n, t_min) /
// min(f, +inf) as maxNum / minNum: a NaN bound constrains nothing, as math.max /
// math.min with t_min / t_max leave it in the reference.
__device__ __forceinline__ bool static_ok(float nx, float ny, float nz, float fx, float fy, float fz) {
  const float t_min = 0.001f, inf = __builtin_inff();
  return (__builtin_fminf(fx, inf) > __builtin_fmaxf(nx, t_min)) && (__builtin_fminf(fy, inf) > __builtin_fmaxf(ny, t_min)) &&
         (__builtin_fminf(fz, inf) > __builtin_fmaxf(nz, t_min));
}

// The reference's own loose test (aabb.zig:109-127) of leaf slot k whose
// narrowed test passed with en >= ex (rare; with en < ex it passes outright:
// an <= en < ex <= ax on every axis): each axis on its own, its distances
// recomputed from the node in memory (the same two roundings as the packed
// form) so that none of them stays live across the node.
// gg: the grazing-triangle guard's spatial widening of this ray (0: off), added to
// the leaf's own slack in both tests; the entry stays the exact loose entry, so a
// best hit found below it (a leaf opened only by the widening) is replayed.
// (planes: the slot's near / far planes in the ray's octant, bx / by / bz near, cx / cy / cz far)
__device__ __forceinline__ bool loose_planes(float bx, float by, float bz, float cx, float cy, float cz, const RayT& r,
                                             float tb, float& entry, float gg = 0.0f) {
  const float t_min = 0.001f;
  const float nx = (bx - r.ox) * r.ix, fx = (cx - r.ox) * r.ix;
  const float ny = (by - r.oy) * r.iy, fy = (cy - r.oy) * r.iy;
  const float nz = (bz - r.oz) * r.iz, fz = (cz - r.oz) * r.iz;
  // the exact loose entry (the order-hazard test's E; wide_iter's en when its slabs are not widened)
  entry = __builtin_fmaxf(__builtin_fmaxf(nx, ny), __builtin_fmaxf(nz, t_min));
  if (!ZRT_GRAZE_SLACK)
    return (__builtin_fminf(fx, tb) > __builtin_fmaxf(nx, t_min)) &&
           (__builtin_fminf(fy, tb) > __builtin_fmaxf(ny, t_min)) &&
           (__builtin_fminf(fz, tb) > __builtin_fmaxf(nz, t_min));
  // the leaf's own coordinate slack (ray_slack): g = 2 x 2^-19 x its largest |coordinate|,
  // g |1/d_k| on axis k; a hit below the leaf's entry by that still counts against tb
  const float cl = __builtin_fmaxf(
      __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(bx), __builtin_fabsf(cx)),
                      __builtin_fmaxf(__builtin_fabsf(by), __builtin_fabsf(cy))),
      __builtin_fmaxf(__builtin_fabsf(bz), __builtin_fabsf(cz)));
  const float g = __builtin_fmaf(cl, r.gm, gg);
  const float gx = paxis_t(g, r.ix), gy = paxis_t(g, r.iy), gz = paxis_t(g, r.iz);
  const float tl = tb + __builtin_fmaxf(__builtin_fmaxf(gx, gy), gz);
  const bool loose = (__builtin_fminf(fx, tl) > __builtin_fmaxf(nx, t_min)) &&
                     (__builtin_fminf(fy, tl) > __builtin_fmaxf(ny, t_min)) &&
                     (__builtin_fminf(fz, tl) > __builtin_fmaxf(nz, t_min));
  // the narrowed test of the box grown by g (NaN bounds constrain nothing)
  const float en = __builtin_fmaxf(__builtin_fmaxf(nx - gx, ny - gy), __builtin_fmaxf(nz - gz, t_min));
  const float ex = __builtin_fminf(__builtin_fminf(fx + gx, fy + gy), __builtin_fminf(fz + gz, tl));
  return loose && !(en > ex * (ZRT_GRAZE_LEAF ? 1.0000153f + r.gl * ray_m(r) : ray_rel(r, ray_m(r))));
}
__device__ __forceinline__ bool loose_slot(const float4* __restrict__ q, int k, const RayT& r, float tb,
                                           bool sx, bool sy, bool sz, float& entry, float gg = 0.0f) {
  const float* f = reinterpret_cast<const float*>(q) + k;
#if ZRT_OCT_COPIES
  (void)sx; (void)sy; (void)sz;
  const int px = 0, py = 4, pz = 8, qx = 12, qy = 16, qz = 20;
#else
  const int px = sx ? 12 : 0, py = sy ? 16 : 4, pz = sz ? 20 : 8;
  const int qx = sx ? 0 : 12, qy = sy ? 4 : 16, qz = sz ? 8 : 20;
#endif
  return loose_planes(f[px], f[py], f[pz], f[qx], f[qy], f[qz], r, tb, entry, gg);
}

// static_ok of leaf slot k, its slab distances recomputed from the node in memory
// (the same two roundings as wide_iter's) so that none stays live across the node
template <class FP>
__device__ __forceinline__ bool static_ok_at(FP f, const RayT& r, bool sx, bool sy, bool sz, float& entry) {
#if ZRT_OCT_COPIES
  (void)sx; (void)sy; (void)sz;
  const int px = 0, py = 4, pz = 8, qx = 12, qy = 16, qz = 20;
#else
  const int px = sx ? 12 : 0, py = sy ? 16 : 4, pz = sz ? 20 : 8;
  const int qx = sx ? 0 : 12, qy = sy ? 4 : 16, qz = sz ? 8 : 20;
#endif
  const float nx = (f[px] - r.ox) * r.ix, ny = (f[py] - r.oy) * r.iy, nz = (f[pz] - r.oz) * r.iz;
  entry = __builtin_fmaxf(__builtin_fmaxf(nx, ny), __builtin_fmaxf(nz, 0.001f));  // the exact loose entry
  return static_ok(nx, ny, nz, (f[qx] - r.ox) * r.ix, (f[qy] - r.oy) * r.iy, (f[qz] - r.oz) * r.iz);
}
// (q is a generic pointer: a node of the top levels lives in LDS - the root,
// which holds the ground sphere's leaf in every reference scene - and is read
// with ds_read, not a flat load through the vector memory path)
__device__ __forceinline__ bool static_ok_slot(const float4* __restrict__ q, int k, const RayT& r, bool sx, bool sy,
                                               bool sz, float& entry) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (__builtin_amdgcn_is_shared(reinterpret_cast<const void*>(q)))
    return static_ok_at((const __attribute__((address_space(3))) float*)(reinterpret_cast<const float*>(q)) + k, r,
                        sx, sy, sz, entry);
#endif
  return static_ok_at(reinterpret_cast<const float*>(q) + k, r, sx, sy, sz, entry);
}

constexpr uint32_t kOctCopies = ZRT_OCT_COPIES ? 8u : 1u;

// The wide tree's top levels (accel_build.cpp stores them first: nodes 0 ..
// n_top-1), every octant copy, copied into the block's LDS once at kernel
// start.  Every ray begins at the root and most go on to a level-1 node, and
// vector-memory data return (TD) is what the FAST loop saturates:
// these node reads come from LDS instead.  All threads of the block call this.
__device__ __forceinline__ void fill_lds_top(const KArgs& a, float4* __restrict__ top) {
  const uint32_t per = a.n_top * a.node_f4;  // float4 per octant copy
  for (uint32_t i = threadIdx.x; i < per * kOctCopies; i += kBlock) {
    const uint32_t o = i / per, j = i - o * per;
    top[i] = a.wnodes[o * a.wide_stride + j];
  }
  __syncthreads();
}

// The material table (a few records in every reference scene) copied into
// LDS at kernel start: the shading of a hit reads its material right after its
// shade record, a dependent chain of loads.
__device__ __forceinline__ void fill_lds_mats(const KArgs& a, float4* __restrict__ m) {
  const float4* src = reinterpret_cast<const float4*>(a.mats);
  for (uint32_t i = threadIdx.x; i < a.n_mats * 3u; i += kBlock) m[i] = src[i];
  __syncthreads();
}

// FAST: near-first over the 4-wide tree (accel_build.cpp), stored once per
// ray octant with each axis' min / max planes swapped where the octant's
// direction is negative, so a node's first three float4 are the four slots'
// near planes and the next three their far planes: the reference's swap
// (aabb.zig:116-118) is done by the layout, not per slot.  All four slots are
// tested against the t_max at node entry (a leaf passing with a t_max >= the
// current one is a superset of what the reference opens, and every primitive
// test still uses the current best with lower-slot tie-breaking); leaf slots
// are intersected in place, inner slots are sorted by entry distance and the
// farther ones pushed, branch-free.
// STATS: coherence of the FAST loop's fetches (kGlobalNodes .. kUniformPrims)
struct Coh {
  uint32_t gnodes = 0, unodes = 0, ptests = 0, uprims = 0, attw = 0, attr = 0, ovfw = 0;
  // wave-level events (kVNodeTrips ..), counted in the wave's first active lane
  uint32_t vn_trips = 0, vn_lines = 0, sn_trips = 0, rb_trips = 0, vp_trips = 0, vp_lines = 0, sp_trips = 0;
  uint32_t vsh_trips = 0, attw_trips = 0, attr_trips = 0, vn_cost = 0, vp_cost = 0;
  __device__ __forceinline__ void flush(unsigned long long* counters);
};

// STATS helpers: 1 in the first active lane of the wave (a wave-level event is
// counted once), and the number of distinct values of x among the active lanes
__device__ __forceinline__ uint32_t wave_once() {
  return __lane_id() == (uint32_t)__builtin_ctzll(__ballot(1)) ? 1u : 0u;
}
__device__ __forceinline__ uint32_t wave_distinct(uint32_t x) {
  uint64_t m = __ballot(1);
  uint32_t n = 0;
  while (m != 0ull) {
    const uint32_t f = (uint32_t)__builtin_amdgcn_readlane((int)x, (int)__builtin_ctzll(m));
    m &= ~__ballot(x == f);
    ++n;
  }
  return n;
}

// One wide node's record in registers: the four slots' near planes, far planes
// (per axis, pre-swapped in the ray's octant copy) and primitive/child refs.
struct WideNode {
  float4 nx, ny, nz, fx, fy, fz, ra;
};

__device__ __forceinline__ void wide_load(const float4* __restrict__ q, bool sx, bool sy, bool sz, WideNode& w) {
#if ZRT_OCT_COPIES
  (void)sx; (void)sy; (void)sz;
  w.nx = q[0]; w.ny = q[1]; w.nz = q[2]; w.fx = q[3]; w.fy = q[4]; w.fz = q[5]; w.ra = q[6];
#else
  const float4 m0 = q[0], m1 = q[1], m2 = q[2], m3 = q[3], m4 = q[4], m5 = q[5];
  w.nx = sx ? m3 : m0; w.fx = sx ? m0 : m3;
  w.ny = sy ? m4 : m1; w.fy = sy ? m1 : m4;
  w.nz = sz ? m5 : m2; w.fz = sz ? m2 : m5;
  w.ra = q[6];
#endif
}

// Where a ray reads the wide tree: its octant's copy (global memory) and that
// copy's top levels in LDS.
struct WideView {
  const float4* __restrict__ top;  // this octant's copy of the top nodes in LDS
  uint32_t base;                   // float4 offset of this octant's copy (< 2^32)
  uint32_t n_top;
  bool sx, sy, sz;
};

__device__ __forceinline__ WideView wide_view(const KArgs& a, const RayT& r, const float4* __restrict__ lds_top) {
  WideView v;
  v.sx = r.ix < 0.0f;
  v.sy = r.iy < 0.0f;
  v.sz = r.iz < 0.0f;
#if ZRT_OCT_COPIES
  const uint32_t oct = (v.sx ? 1u : 0u) | (v.sy ? 2u : 0u) | (v.sz ? 4u : 0u);
  v.base = oct * a.wide_stride;
#else
  const uint32_t oct = 0;
  v.base = 0;
#endif
  v.top = lds_top + (ZRT_OCT_COPIES ? oct : 0u) * (a.n_top * a.node_f4);
  v.n_top = ZRT_LDS_TOP ? a.n_top : 0u;
  return v;
}

// The address of wide node `i` for this ray: LDS for a top-level node, else
// its octant copy in global memory.
__device__ __forceinline__ const float4* wide_node_ptr(const KArgs& a, const WideView& v, uint32_t i) {
  return i < v.n_top ? v.top + 8u * i : a.wnodes + (v.base + 8u * i);
}

// FAST: near-first over the 4-wide tree (accel_build.cpp), stored once per
// ray octant with each axis' min / max planes swapped where the octant's
// direction is negative, so a node's first three float4 are the four slots'
// near planes and the next three their far planes: the reference's swap
// (aabb.zig:116-118) is done by the layout, not per slot.  All four slots are
// tested against the t_max at node entry (a leaf passing with a t_max >= the
// current one is a superset of what the reference opens, and every primitive
// test still uses the current best with lower-slot tie-breaking); leaf slots
// are intersected in place, inner slots are sorted by entry distance and the
// farther ones pushed, branch-free.
//
// wide_iter processes the node in `w` (read from q), picks the next node
// (pushing the farther inner children), intersects the opened leaves and loads
// the next node into `w` / q.  Returns false when the traversal is over (then
// the order-hazard test of wide_finish follows).  Its state between calls is
// (w, q, sp, best_t, best) and the lane's stack column, so a traversal can be
// suspended between nodes (the wavefront loop, render_loop_wf).
template <bool STATS, class StackT, bool SCALAR_NODES = ZRT_SCALAR_NODES, bool PAXIS = ZRT_PAXIS_LOCK, bool GUARD = true,
          bool QG = false>
__device__ __forceinline__ bool wide_iter(const KArgs& a, const RayT& r, const WideView& v,
                                          StackT* __restrict__ stk, uint32_t gl, WideNode& w,
                                          const float4*& q, uint32_t& sp, float& best_t, int& best,
                                          uint32_t& c_nodes, uint32_t& c_leaves, uint32_t& c_tri, uint32_t& c_sph,
                                          Coh& coh) {
  const int stride = kBlock;
  const uint32_t cap = a.stack_depth;  // rows allocated: the deepest push + 3
  // the first rows in LDS, the rest in global memory (a.lds_rows: zrt::plan_lds)
  constexpr bool kOvf = true;
  const uint32_t rows = a.lds_rows;
  StackT* __restrict__ ovf = reinterpret_cast<StackT*>(a.stack_ovf) + gl;
  const float inf = __builtin_inff();
  const bool sx = v.sx, sy = v.sy, sz = v.sz;
  int r0 = as_int(w.ra.x), r1 = as_int(w.ra.y), r2 = as_int(w.ra.z), r3 = as_int(w.ra.w);
  const float tb = __builtin_fabsf(best_t) * kOpen;
  const float m = ray_m(r), rel = ray_rel(r, m), slk = ray_slack(r, a.scene_extent, m);
#if ZRT_FMA_SLABS
  // slab distances fma(plane, 1/d, -p), p = o / d (see slab2f): E2 covers their error
  const float px = r.ox * r.ix, py = r.oy * r.iy, pz = r.oz * r.iz;
  const float pm = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(px), __builtin_fabsf(py)), __builtin_fabsf(pz));
  const bool deg = !(m < 0x1p100f) || !(pm < 0x1p120f);  // ray_degenerate: nothing opens, wide_finish replays
  float E2 = pm * kFmaE2;
  // The grazing-triangle guard (DESIGN.md §3 "Triangles"): every box widened on
  // every axis by the reach g of the rounded triangle test, as w_k = g |1/d_k| in
  // t, through the offsets of the FMA form (near planes - (p + w), far planes
  // - (p - w)): no instruction per plane.  The exact interval then lies within
  // [en, en + wm] .. [ex - wm, ex], so certain decisions need 2 wm more (Eg).
  // (Two copies of the 24 distances under a scene-uniform branch: the offsets
  // held across one copy cost the lockstep kernel 11 more spilled VGPRs.)
  float Eg = E2, gg = 0.0f;  // gg: the guard's spatial widening (loose_slot), 0 when off
  f2 nx01, nx23, ny01, ny23, nz01, nz23, fx01, fx23, fy01, fy23, fz01, fz23;
#define ZRT_SLABS(PNX, PNY, PNZ, PFX, PFY, PFZ)                                                         \
  nx01 = slab2f(w.nx.x, w.nx.y, PNX, r.ix); nx23 = slab2f(w.nx.z, w.nx.w, PNX, r.ix);                   \
  ny01 = slab2f(w.ny.x, w.ny.y, PNY, r.iy); ny23 = slab2f(w.ny.z, w.ny.w, PNY, r.iy);                   \
  nz01 = slab2f(w.nz.x, w.nz.y, PNZ, r.iz); nz23 = slab2f(w.nz.z, w.nz.w, PNZ, r.iz);                   \
  fx01 = slab2f(w.fx.x, w.fx.y, PFX, r.ix); fx23 = slab2f(w.fx.z, w.fx.w, PFX, r.ix);                   \
  fy01 = slab2f(w.fy.x, w.fy.y, PFY, r.iy); fy23 = slab2f(w.fy.z, w.fy.w, PFY, r.iy);                   \
  fz01 = slab2f(w.fz.x, w.fz.y, PFZ, r.iz); fz23 = slab2f(w.fz.z, w.fz.w, PFZ, r.iz);
  // (the wavefront, path-pool and trace loops only: in the lockstep kernel the branch
  // alone cost 4 more spilled VGPRs, C4 -4 %, profiles/r04/r04d)
  if (ZRT_GUARD && GUARD && PAXIS && __builtin_expect(r.gk > 0.0f, 0)) {  // scene-uniform: a scalar branch
    const float g = guard_grow(a, r);
    gg = g;
    const float wx = paxis_t(g, r.ix), wy = paxis_t(g, r.iy), wz = paxis_t(g, r.iz);
    const float wm = __builtin_fmaxf(__builtin_fmaxf(wx, wy), wz);
    E2 = (pm + wm) * kFmaE2;  // (the offsets p -+ w are rounded too)
    Eg = __builtin_fmaf(wm, 2.0f, E2);
    ZRT_SLABS(px + wx, py + wy, pz + wz, px - wx, py - wy, pz - wz)
  } else {
    ZRT_SLABS(px, py, pz, px, py, pz)
  }
#undef ZRT_SLABS
#else
  constexpr bool deg = false;
  constexpr float E2 = 0.0f, Eg = 0.0f, gg = 0.0f;
#define ZRT_SLAB_X(V, A, B) slab2(V.A, V.B, r.ox, r.ix)
#define ZRT_SLAB_Y(V, A, B) slab2(V.A, V.B, r.oy, r.iy)
#define ZRT_SLAB_Z(V, A, B) slab2(V.A, V.B, r.oz, r.iz)
  f2 nx01 = ZRT_SLAB_X(w.nx, x, y), nx23 = ZRT_SLAB_X(w.nx, z, w);
  f2 ny01 = ZRT_SLAB_Y(w.ny, x, y), ny23 = ZRT_SLAB_Y(w.ny, z, w);
  f2 nz01 = ZRT_SLAB_Z(w.nz, x, y), nz23 = ZRT_SLAB_Z(w.nz, z, w);
  f2 fx01 = ZRT_SLAB_X(w.fx, x, y), fx23 = ZRT_SLAB_X(w.fx, z, w);
  f2 fy01 = ZRT_SLAB_Y(w.fy, x, y), fy23 = ZRT_SLAB_Y(w.fy, z, w);
  f2 fz01 = ZRT_SLAB_Z(w.fz, x, y), fz23 = ZRT_SLAB_Z(w.fz, z, w);
#undef ZRT_SLAB_X
#undef ZRT_SLAB_Y
#undef ZRT_SLAB_Z
#endif
  // a lane of the wave runs nearly parallel to an axis (paxis_grow): every slab
  // widened in place by its axis's own term; the leaf slots' exact intervals (the
  // reference's loose test, the hazard entry) are then recomputed by loose_slot
  bool pw = false;
  if (ZRT_PAXIS && PAXIS && __builtin_expect(__ballot(m > a.paxis_m) != 0ull, 0)) {
    pw = true;
    const float g = paxis_grow(a, r);
    const float gx = paxis_t(g, r.ix), gy = paxis_t(g, r.iy), gz = paxis_t(g, r.iz);
    nx01.x -= gx; nx01.y -= gx; nx23.x -= gx; nx23.y -= gx;
    ny01.x -= gy; ny01.y -= gy; ny23.x -= gy; ny23.y -= gy;
    nz01.x -= gz; nz01.y -= gz; nz23.x -= gz; nz23.y -= gz;
    fx01.x += gx; fx01.y += gx; fx23.x += gx; fx23.y += gx;
    fy01.x += gy; fy01.y += gy; fy23.x += gy; fy23.y += gy;
    fz01.x += gz; fz01.y += gz; fz23.x += gz; fz23.y += gz;
  }
  SlotT s0 = slot_interval(nx01.x, ny01.x, nz01.x, fx01.x, fy01.x, fz01.x, tb);
  SlotT s1 = slot_interval(nx01.y, ny01.y, nz01.y, fx01.y, fy01.y, fz01.y, tb);
  SlotT s2 = slot_interval(nx23.x, ny23.x, nz23.x, fx23.x, fy23.x, fz23.x, tb);
  SlotT s3 = slot_interval(nx23.y, ny23.y, nz23.y, fx23.y, fy23.y, fz23.y, tb);
  // narrowed test: entry > exit * rel (+ slack for a leaf slot) culls (ray_slack:
  // inner slots' boxes are stored grown, leaf slots' are the reference leaves');
  // widened slabs carry their margins already (rounding: 2^-16)
  const float rl = pw ? 1.0000153f : rel, sl = (pw ? 0.0f : slk) + E2;
#if ZRT_GRAZE_LEAF
  const float rll = pw ? 1.0000153f : 1.0000153f + r.gl * m;  // leaf slots (KArgs::graze_leaf)
#else
  const float rll = rl;
#endif
  const bool h0 = !deg && !(s0.en > __builtin_fmaf(s0.ex, r0 < 0 ? rll : rl, r0 < 0 ? sl : E2));
  const bool h1 = !deg && !(s1.en > __builtin_fmaf(s1.ex, r1 < 0 ? rll : rl, r1 < 0 ? sl : E2));
  const bool h2 = !deg && !(s2.en > __builtin_fmaf(s2.ex, r2 < 0 ? rll : rl, r2 < 0 ? sl : E2));
  const bool h3 = !deg && !(s3.en > __builtin_fmaf(s3.ex, r3 < 0 ? rll : rl, r3 < 0 ? sl : E2));
  if (STATS) {
    ++c_nodes;
    c_leaves += (r0 < 0) + (r1 < 0) + (r2 < 0) + (r3 < 0);
  }
  // leaf slots that pass both tests: their primitive refs (a in r_k, b in the node's last float4)
  bool o0 = r0 < 0 && h0, o1 = r1 < 0 && h1, o2 = r2 < 0 && h2, o3 = r3 < 0 && h3;
  // (certain: en < ex by the FMA distances' error; ZRT_FMA_SLABS = 0: kFmaSure is exact enough)
#define ZRT_SURE(S) (__builtin_fmaf(S.en, ZRT_FMA_SLABS ? kFmaSure : 1.0f, Eg) < S.ex)
  // (guarded: the slabs are widened, so every opened leaf takes its exact loose entry - the
  // hazard test's E - and its widened per-axis tests from memory)
  const bool pg = pw || gg > 0.0f;
  const bool w0 = o0 && (pg || !ZRT_SURE(s0)), w1 = o1 && (pg || !ZRT_SURE(s1));
  const bool w2 = o2 && (pg || !ZRT_SURE(s2)), w3 = o3 && (pg || !ZRT_SURE(s3));
  if (w0 || w1 || w2 || w3) {  // rare: an interval within the margin, decide per axis
    if (w0) o0 = loose_slot(q, 0, r, tb, sx, sy, sz, s0.en, gg);
    if (w1) o1 = loose_slot(q, 1, r, tb, sx, sy, sz, s1.en, gg);
    if (w2) o2 = loose_slot(q, 2, r, tb, sx, sy, sz, s2.en, gg);
    if (w3) o3 = loose_slot(q, 3, r, tb, sx, sy, sz, s3.en, gg);
  }
#if ZRT_SPHERE_SLOTS
  // leaf slots holding a sphere (ref a - 2^30, accel_build.hpp): opened when the
  // reference's loose test passes against t_max = +inf.  The rounded sphere test
  // accepts rays that pass outside the sphere - and its box - by up to ~sqrt(u)|oc|
  // and errs by as much in t (DESIGN.md §3 "Spheres"), so neither the narrowed
  // test nor the current best may cull them; every sphere hit of a static-ok
  // leaf is then seen, and the order-hazard tests see it too.  (A wave-uniform
  // branch: nodes with sphere leaves are few.)
  // The slot's interval in registers settles most: en < ex (the narrowed interval
  // is not empty: every axis passes) opens it, ex <= t_min (an axis's far plane
  // at or behind t_min: that axis fails; tb > t_min) keeps it shut; the rest, and
  // every slot of a widened wave (pw), take the per-axis test from memory.
#if ZRT_SPHERE_FIRST  // accel_build puts a node's sphere leaves in its first slots
  if (__builtin_expect(__ballot(r0 < -kSphereSlotBias) != 0ull, 0)) {
#else
  if (__builtin_expect(__ballot(min(min(r0, r1), min(r2, r3)) < -kSphereSlotBias) != 0ull, 0)) {
#endif
#define ZRT_SPHERE_SLOT(K)                                                                                   \
  if (r##K < -kSphereSlotBias) {                                                                             \
    o##K = !pw && !deg && ZRT_SURE(s##K);                                                                    \
    if (!o##K && !deg && s##K.ex + __builtin_fmaf(__builtin_fabsf(s##K.ex), 0x1p-19f, Eg) > 0.001f)          \
      o##K = static_ok_slot(q, K, r, sx, sy, sz, s##K.en);                                                   \
    r##K += kSphereSlotBias;                                                                                 \
  }
    ZRT_SPHERE_SLOT(0)
    ZRT_SPHERE_SLOT(1)
    ZRT_SPHERE_SLOT(2)
    ZRT_SPHERE_SLOT(3)
#undef ZRT_SPHERE_SLOT
  }
#endif
#undef ZRT_SURE
  const int l0 = o0 ? r0 : 0, l1 = o1 ? r1 : 0, l2 = o2 ? r2 : 0, l3 = o3 ? r3 : 0;
  const float4* leaf_q = q;  // (the leaves are intersected after the next node is chosen)
  int32_t next = -1;
  // inner slots that pass, keyed by entry distance
  float k0 = r0 >= 0 && h0 ? s0.en : inf, k1 = r1 >= 0 && h1 ? s1.en : inf;
  float k2 = r2 >= 0 && h2 ? s2.en : inf, k3 = r3 >= 0 && h3 ? s3.en : inf;
  const uint32_t n = (k0 != inf) + (k1 != inf) + (k2 != inf) + (k3 != inf);
#if ZRT_STACK_LDS_FAST
  // every active lane's stack top and its next three pushes inside the LDS rows (a
  // wave-uniform test, true throughout for trees whose stack fits the LDS plan): the
  // pop is a ds_read of the lane's LDS column - not a generic load that could also
  // reach the global rows - and push, pop and the choice between them are selects,
  // not exec-mask regions (the same stack contents and the same next node)
  if (ZRT_STACK_LDS_FAST == 2 && __ballot(sp + 3u > rows) == 0ull) {
    // (A/B form 2: the same branches as below, the pop a ds_read of the LDS column)
    if (ZRT_SORT_SKIP && __ballot(n > 1u) == 0ull) {
      if (n != 0) {
        next = k0 != inf ? r0 : k1 != inf ? r1 : k2 != inf ? r2 : r3;
      } else if (sp != 0) {
        --sp;
        next = (int32_t)stk[sp * stride];
      }
    } else {
      cswap(k0, r0, k1, r1);
      cswap(k2, r2, k3, r3);
      cswap(k0, r0, k2, r2);
      cswap(k1, r1, k3, r3);
      cswap(k1, r1, k2, r2);
      if (n != 0) {
        stk[sp * stride] = (StackT)(n == 4 ? r3 : n == 3 ? r2 : r1);
        stk[(sp + 1) * stride] = (StackT)(n == 4 ? r2 : r1);
        stk[(sp + 2) * stride] = (StackT)r1;
        const uint32_t nsp = sp + n - 1;
        if (__builtin_expect(nsp > cap - 3, 0)) atomicOr(a.error_flag, kErrOverflow);
        sp = min(nsp, cap - 3);
        next = r0;
      } else if (sp != 0) {
        --sp;
        next = (int32_t)stk[sp * stride];
      }
    }
  } else if (ZRT_STACK_LDS_FAST == 1 && __ballot(sp + 3u > rows) == 0ull) {
    const uint32_t psp = sp != 0 ? sp - 1u : 0u;
    const int32_t top = (int32_t)stk[psp * stride];
    if (ZRT_SORT_SKIP && __ballot(n > 1u) == 0ull) {
      next = n != 0 ? (k0 != inf ? r0 : k1 != inf ? r1 : k2 != inf ? r2 : r3) : sp != 0 ? top : -1;
      sp = n != 0 ? sp : psp;
    } else {
      cswap(k0, r0, k1, r1);
      cswap(k2, r2, k3, r3);
      cswap(k0, r0, k2, r2);
      cswap(k1, r1, k3, r3);
      cswap(k1, r1, k2, r2);
      // (a lane with no inner child writes above its top: dead entries)
      stk[sp * stride] = (StackT)(n == 4 ? r3 : n == 3 ? r2 : r1);
      stk[(sp + 1) * stride] = (StackT)(n == 4 ? r2 : r1);
      stk[(sp + 2) * stride] = (StackT)r1;
      const uint32_t nsp = sp + n - 1;
      if (__builtin_expect(__ballot(n != 0 && nsp > cap - 3) != 0ull, 0)) {
        if (n != 0 && nsp > cap - 3) atomicOr(a.error_flag, kErrOverflow);
      }
      next = n != 0 ? r0 : sp != 0 ? top : -1;
      sp = n != 0 ? min(nsp, cap - 3) : psp;
    }
  } else {
#endif
#if ZRT_SORT_SKIP
  if (__ballot(n > 1u) == 0ull) {
    // every active lane follows at most one inner child: no sort, nothing to push
    // (a wave-uniform branch around the 5 compare-exchanges and the 3 stores)
    if (n != 0) {
      next = k0 != inf ? r0 : k1 != inf ? r1 : k2 != inf ? r2 : r3;
    } else if (sp != 0) {
      --sp;
      next = kOvf && sp >= rows ? (row_ok<STATS>(a, (uint64_t)(sp - rows) * a.n_lanes + gl, a.ovf_cap) ? (int32_t)ovf[(size_t)(sp - rows) * a.n_lanes] : -1)
                                  : (int32_t)stk[sp * stride];
    }
  } else {
#endif
  // sort (entry, ref) ascending: 5 compare-exchanges
  cswap(k0, r0, k1, r1);
  cswap(k2, r2, k3, r3);
  cswap(k0, r0, k2, r2);
  cswap(k1, r1, k3, r3);
  cswap(k1, r1, k2, r2);
  if (n != 0) {
    // push r_{n-1} .. r_1 (farthest first) and continue with the nearest; the
    // three stores are unconditional (entries above the new top are dead)
    const StackT e0 = (StackT)(n == 4 ? r3 : n == 3 ? r2 : r1), e1 = (StackT)(n == 4 ? r2 : r1);
    const StackT e2 = (StackT)r1;
    // sp <= cap - 3 always holds (the clamp below), so the three stores stay in the rows
    if (sp + 3 <= rows) {
      stk[sp * stride] = e0;
      stk[(sp + 1) * stride] = e1;
      stk[(sp + 2) * stride] = e2;
    } else if (kOvf) {  // deep trees: rows past the LDS part live in global memory
      const StackT e[3] = {e0, e1, e2};
#pragma unroll
      for (uint32_t j = 0; j < 3; ++j) {
        if (sp + j < rows) {
          stk[(sp + j) * stride] = e[j];
        } else {
          if (row_ok<STATS>(a, (uint64_t)(sp + j - rows) * a.n_lanes + gl, a.ovf_cap))
            ovf[(size_t)(sp + j - rows) * a.n_lanes] = e[j];
          if (STATS) ++coh.ovfw;
        }
      }
    }
    const uint32_t nsp = sp + n - 1;
    // the host sizes cap = the tree's deepest stack + 3, so this never fires
    // unless the stack was sized too small: then entries would be lost
    if (__builtin_expect(nsp > cap - 3, 0)) atomicOr(a.error_flag, kErrOverflow);
    sp = min(nsp, cap - 3);
    next = r0;
  } else if (sp != 0) {
    --sp;
    next = kOvf && sp >= rows ? (row_ok<STATS>(a, (uint64_t)(sp - rows) * a.n_lanes + gl, a.ovf_cap) ? (int32_t)ovf[(size_t)(sp - rows) * a.n_lanes] : -1)
                                  : (int32_t)stk[sp * stride];
  }
#if ZRT_SORT_SKIP
  }
#endif
#if ZRT_STACK_LDS_FAST
  }
#endif
  // each lane walks ITS opened leaves in slot order, so lanes that opened
  // different slots share loop trips (the result is the closest t, ties to
  // the lower slot, order hazards flagged).  A/B against four unrolled slot
  // blocks: C5 +2.9 %, C3 +3.2 %, C4 -0.2 % (and one copy of the tests).
  if constexpr (sizeof(StackT) == 4 || ZRT_LEAF_LOOP) {
    uint32_t open = (l0 != 0 ? 1u : 0u) | (l1 != 0 ? 2u : 0u) | (l2 != 0 ? 4u : 0u) | (l3 != 0 ? 8u : 0u);
    if (open != 0) {
      float4 rb;
#if ZRT_SCALAR_RB && defined(__HIP_DEVICE_COMPILE__)
      // a node every active lane reads (loaded through the scalar cache, or wave-uniform
      // anyway): its second refs through the scalar cache too - a vector dwordx4 costs
      // the data-return path 16 cycles however few lanes or addresses it has
      // (tools/ubench_shapes.hip)
      const uint64_t qa = reinterpret_cast<uint64_t>(leaf_q);
      const uint64_t fq = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(qa >> 32)) << 32) |
                          (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)qa);
      if (__ballot(qa != fq) == 0ull && !__builtin_amdgcn_is_shared((const void*)fq)) {
        typedef const __attribute__((address_space(4))) float4 cfloat4;
        rb = ((cfloat4*)fq)[7];
      } else {
        rb = leaf_q[7];
        if (STATS) coh.rb_trips += wave_once();
      }
#else
      rb = leaf_q[7];
      if (STATS) coh.rb_trips += wave_once();
#endif
      do {
        const uint32_t k = (uint32_t)__builtin_ctz(open);
        open &= open - 1u;
        const int L = k == 0 ? l0 : k == 1 ? l1 : k == 2 ? l2 : l3;
        const int pb = as_int(k == 0 ? rb.x : k == 1 ? rb.y : k == 2 ? rb.z : rb.w);
        // the leaf's loose entry, or (FMA distances) an upper bound of it: flags a superset
        // (a guarded leaf's entry is exact: it went through loose_slot)
        const float lp = ZRT_HAZARD_ENTRY ? (ZRT_FMA_SLABS ? __builtin_fmaf(k == 0 ? s0.en : k == 1 ? s1.en : k == 2 ? s2.en : s3.en, kFmaSure, E2)
                                                           : (k == 0 ? s0.en : k == 1 ? s1.en : k == 2 ? s2.en : s3.en))
                                        : -1.0f;
        if (STATS) {
          const int f = __builtin_amdgcn_readfirstlane(L);
          coh.ptests += 1u;
          coh.uprims += __ballot(L != f) == 0ull ? 1u : 0u;
        }
        const int fl = __builtin_amdgcn_readfirstlane(L), fb = __builtin_amdgcn_readfirstlane(pb);
        if (ZRT_SCALAR_PRIMS && __ballot(L != fl || pb != fb) == 0ull) {  // one leaf in every active lane
          if (STATS) coh.sp_trips += wave_once() * (fb != fl ? 2u : 1u);
          prim_test_uniform<true, STATS, ZRT_ORDER_EXACT>(a.prims, fl, r, best_t, best, c_tri, c_sph, lp);
          if (fb != fl) prim_test_uniform<true, STATS, ZRT_ORDER_EXACT>(a.prims, fb, r, best_t, best, c_tri, c_sph, lp);
        } else {
          if (STATS) {
            const uint32_t dl = wave_distinct((uint32_t)L);
            if (wave_once()) { ++coh.vp_trips; coh.vp_lines += dl; coh.vp_cost += max(16u, dl); }
          }
          prim_test<true, STATS, ZRT_ORDER_EXACT>(a.prims, L, r, best_t, best, c_tri, c_sph, lp);
          if (pb != L) {
            if (STATS) {
              const uint32_t db = wave_distinct((uint32_t)pb);
              if (wave_once()) { ++coh.vp_trips; coh.vp_lines += db; coh.vp_cost += max(16u, db); }
            }
            prim_test<true, STATS, ZRT_ORDER_EXACT>(a.prims, pb, r, best_t, best, c_tri, c_sph, lp);
          }
        }
      } while (open != 0);
    }
  } else if ((l0 | l1 | l2 | l3) != 0) {
    const float4 rb = leaf_q[7];  // (loaded with the node instead: 3.6 % slower, 2 spills)
#define ZRT_WIDE_LEAF(L, RB, K)                                                                     \
  if (L != 0) {                                                                                     \
    const int pb = as_int(RB);                                                                      \
    const float lp = ZRT_HAZARD_ENTRY ? (ZRT_FMA_SLABS ? __builtin_fmaf(s##K.en, kFmaSure, E2) : s##K.en) : -1.0f; \
    prim_test<true, STATS, ZRT_ORDER_EXACT>(a.prims, L, r, best_t, best, c_tri, c_sph, lp);              \
    if (pb != L) prim_test<true, STATS, ZRT_ORDER_EXACT>(a.prims, pb, r, best_t, best, c_tri, c_sph, lp); \
  }
    ZRT_WIDE_LEAF(l0, rb.x, 0)
    ZRT_WIDE_LEAF(l1, rb.y, 1)
    ZRT_WIDE_LEAF(l2, rb.z, 2)
    ZRT_WIDE_LEAF(l3, rb.w, 3)
#undef ZRT_WIDE_LEAF
  }
  if (STATS && next >= 0 && (uint32_t)next >= v.n_top) {
    const int32_t f = __builtin_amdgcn_readfirstlane(next);
    const bool uni = __ballot(next != f || (uint32_t)next < v.n_top) == 0ull;  // (among the lanes here)
    ++coh.gnodes;
    coh.unodes += uni ? 1u : 0u;
  }
  if (next < 0) return false;
  if ((uint32_t)next < v.n_top) {  // a top-level node: from LDS (ds_read)
    const float4* __restrict__ t = v.top + 8u * (uint32_t)next;
    // QG: q names the node's global copy even here (the leaf refs and the rare plane
    // re-reads then load from global memory, never through a generic pointer)
    q = QG ? a.wnodes + (v.base + 8u * (uint32_t)next) : t;
    wide_load(t, sx, sy, sz, w);
  } else {
    const uint32_t at = v.base + 8u * (uint32_t)next;  // this ray's octant copy
    const float4* __restrict__ g = a.wnodes + at;
    q = g;
    const uint32_t fa = __builtin_amdgcn_readfirstlane(at);
    if (SCALAR_NODES && __ballot(at != fa) == 0ull) {  // one node in every active lane: scalar loads
      if (STATS) coh.sn_trips += wave_once();
#if defined(__HIP_DEVICE_COMPILE__)
      typedef const __attribute__((address_space(4))) float4 cfloat4;
      wide_load(reinterpret_cast<const float4*>((cfloat4*)a.wnodes + fa), sx, sy, sz, w);
#else
      wide_load(a.wnodes + fa, sx, sy, sz, w);
#endif
    } else {
      if (STATS) {
        const uint32_t dn = wave_distinct(at);
        if (wave_once()) { ++coh.vn_trips; coh.vn_lines += dn; coh.vn_cost += max(16u, dn); }
      }
      wide_load(g, sx, sy, sz, w);
#if ZRT_AB_DOUBLE_NODE  // A/B probe only (never shipped): the same node read again from another octant copy
      {
        WideNode w2;
        const uint32_t o2 = (v.base + a.wide_stride * (ZRT_AB_DOUBLE_NODE)) % (a.wide_stride * 8u);
        wide_load(a.wnodes + o2 + 8u * (uint32_t)next, sx, sy, sz, w2);
        const uint32_t x = __float_as_uint(w2.nx.x) ^ __float_as_uint(w2.ny.y) ^ __float_as_uint(w2.nz.z) ^
                           __float_as_uint(w2.fx.w) ^ __float_as_uint(w2.fy.x) ^ __float_as_uint(w2.fz.y) ^
                           __float_as_uint(w2.ra.z);
        if (x == 0x7fc01234u) w.ra.x = w.ra.y;  // never true for the scenes measured
      }
#endif
    }
  }
  return true;
}

// The end of a FAST traversal: the order hazard of DESIGN.md §3 (1e-8..1e-5
// of rays) re-traced the reference's way.
template <bool STATS, class StackT>
__device__ __forceinline__ void wide_finish(const KArgs& a, const RayT& r, StackT* __restrict__ stk, uint32_t gl,
                                            float& best_t, int& best, uint32_t& c_replays) {
  // an origin farther out than the sphere growth was sized for: the reference's
  // way alone (narrow = false).  One call site for both cases: the replay is
  // inlined, and a second copy cost the lockstep loop 2.8 % on C4 (registers).
  const bool far = __builtin_expect(!ray_origin_ok(a, r) || ray_degenerate(r), 0);
  if (__builtin_expect((ZRT_ORDER_EXACT && order_hazard<false>(a, r, best_t, best)) || far, 0)) {
    if (STATS) ++c_replays;
#if ZRT_REPLAY_OFF
    if (!far) best_t = -best_t;  // A/B only: the replay's cost without its code (results not exact)
    else
#endif
    reference_replay<StackT>(a, r, stk, gl, best_t, best, !far);
  }
}

// ---------------------------------------------------------------------------
// Compressed wide nodes (accel_build.hpp quantize_wide; DESIGN.md §3
// "Compressed nodes"): 64 B per node - the origin and per-axis power-of-two
// step, the 24 planes as bytes, the refs - instead of 128 B, for trees past the
// caches (the C5 mesh: 475 MB of octant copies become 238 MB).  A plane decodes
// exactly (origin + q * step is an f32 by construction), so the slab distances
// and every margin are wide_iter's; the quantized boxes contain the full nodes'
// boxes, so the culls are supersets.  A leaf slot's exact box (the reference's,
// bit for bit) and its primitive refs come from its leaf record, read when the
// quantized box passes: every decision wide_iter takes from the leaf's planes -
// the narrowed and loose tests, a sphere slot's static test, the hazard entry -
// is taken from the record's planes with wide_iter's formulas.
struct WideNodeQ {
  float4 f0, f1, f2, f3;  // {origin.xyz, steps}, {near x/y/z, far x}, {far y/z, ref 0/1}, {ref 2/3, 0, 0}
};
template <class P>
__device__ __forceinline__ void qnode_load(P q, WideNodeQ& w) {
  w.f0 = q[0];
  w.f1 = q[1];
  w.f2 = q[2];
  w.f3 = q[3];
}
// plane byte k of `word`: origin + q * step (exact: a product of a byte and a
// power of two, then a sum the encoder made representable)
__device__ __forceinline__ float qplane(uint32_t word, int k, float step, float origin) {
  return __builtin_fmaf((float)((word >> (8 * k)) & 0xffu), step, origin);
}
__device__ __forceinline__ float qstep(uint32_t e8) { return __uint_as_float(e8 << 23); }

// static_ok (aabb.zig:109-127 against t_max = +inf) of a box given by its planes in
// the ray's octant, and its exact loose entry
__device__ __forceinline__ bool static_ok_planes(float bx, float by, float bz, float cx, float cy, float cz,
                                                 const RayT& r, float& entry) {
  const float nx = (bx - r.ox) * r.ix, ny = (by - r.oy) * r.iy, nz = (bz - r.oz) * r.iz;
  entry = __builtin_fmaxf(__builtin_fmaxf(nx, ny), __builtin_fmaxf(nz, 0.001f));
  return static_ok(nx, ny, nz, (cx - r.ox) * r.ix, (cy - r.oy) * r.iy, (cz - r.oz) * r.iz);
}

template <bool STATS, class StackT, bool PAXIS = true, bool GUARD = true, bool SCALAR = false>
__device__ __forceinline__ bool wide_iter_q(const KArgs& a, const RayT& r, const WideView& v,
                                            StackT* __restrict__ stk, uint32_t gl, WideNodeQ& w,
                                            const float4*& q, uint32_t& sp, float& best_t, int& best,
                                            uint32_t& c_nodes, uint32_t& c_leaves, uint32_t& c_tri, uint32_t& c_sph,
                                            Coh& coh) {
  (void)q;
  const int stride = kBlock;
  const uint32_t cap = a.stack_depth;
  const uint32_t rows = a.lds_rows;  // the first rows in LDS, the rest in global memory (either stack width)
  StackT* __restrict__ ovf = reinterpret_cast<StackT*>(a.stack_ovf) + gl;
  const float inf = __builtin_inff();
  const bool sx = v.sx, sy = v.sy, sz = v.sz;
  int r0 = as_int(w.f2.z), r1 = as_int(w.f2.w), r2 = as_int(w.f3.x), r3 = as_int(w.f3.y);
  const float ox = w.f0.x, oy = w.f0.y, oz = w.f0.z;
  const uint32_t ee = __float_as_uint(w.f0.w);
  const float stx = qstep(ee & 0xffu), sty = qstep((ee >> 8) & 0xffu), stz = qstep((ee >> 16) & 0xffu);
  const uint32_t bnx = __float_as_uint(w.f1.x), bny = __float_as_uint(w.f1.y), bnz = __float_as_uint(w.f1.z);
  const uint32_t bfx = __float_as_uint(w.f1.w), bfy = __float_as_uint(w.f2.x), bfz = __float_as_uint(w.f2.y);
  const float tb = __builtin_fabsf(best_t) * kOpen;
  const float m = ray_m(r), rel = ray_rel(r, m), slk = ray_slack(r, a.scene_extent, m);
  const float px = r.ox * r.ix, py = r.oy * r.iy, pz = r.oz * r.iz;
  const float pm = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(px), __builtin_fabsf(py)), __builtin_fabsf(pz));
  const bool deg = !(m < 0x1p100f) || !(pm < 0x1p120f);  // ray_degenerate: nothing opens, wide_finish replays
  float E2 = pm * kFmaE2;
  float Eg = E2, gg = 0.0f;
  // the slab offsets of the near / far planes (wide_iter: p -+ the guard's w)
  float onx = px, ony = py, onz = pz, ofx = px, ofy = py, ofz = pz;
  if (ZRT_GUARD && GUARD && PAXIS && __builtin_expect(r.gk > 0.0f, 0)) {  // scene-uniform: a scalar branch
    const float g = guard_grow(a, r);
    gg = g;
    const float wx = paxis_t(g, r.ix), wy = paxis_t(g, r.iy), wz = paxis_t(g, r.iz);
    const float wm = __builtin_fmaxf(__builtin_fmaxf(wx, wy), wz);
    E2 = (pm + wm) * kFmaE2;
    Eg = __builtin_fmaf(wm, 2.0f, E2);
    onx = px + wx; ony = py + wy; onz = pz + wz;
    ofx = px - wx; ofy = py - wy; ofz = pz - wz;
  }
#define ZRT_QSLAB(BW, K, ST, OR, OFF, INV) __builtin_fmaf(qplane(BW, K, ST, OR), INV, -(OFF))
  f2 nx01 = {ZRT_QSLAB(bnx, 0, stx, ox, onx, r.ix), ZRT_QSLAB(bnx, 1, stx, ox, onx, r.ix)};
  f2 nx23 = {ZRT_QSLAB(bnx, 2, stx, ox, onx, r.ix), ZRT_QSLAB(bnx, 3, stx, ox, onx, r.ix)};
  f2 ny01 = {ZRT_QSLAB(bny, 0, sty, oy, ony, r.iy), ZRT_QSLAB(bny, 1, sty, oy, ony, r.iy)};
  f2 ny23 = {ZRT_QSLAB(bny, 2, sty, oy, ony, r.iy), ZRT_QSLAB(bny, 3, sty, oy, ony, r.iy)};
  f2 nz01 = {ZRT_QSLAB(bnz, 0, stz, oz, onz, r.iz), ZRT_QSLAB(bnz, 1, stz, oz, onz, r.iz)};
  f2 nz23 = {ZRT_QSLAB(bnz, 2, stz, oz, onz, r.iz), ZRT_QSLAB(bnz, 3, stz, oz, onz, r.iz)};
  f2 fx01 = {ZRT_QSLAB(bfx, 0, stx, ox, ofx, r.ix), ZRT_QSLAB(bfx, 1, stx, ox, ofx, r.ix)};
  f2 fx23 = {ZRT_QSLAB(bfx, 2, stx, ox, ofx, r.ix), ZRT_QSLAB(bfx, 3, stx, ox, ofx, r.ix)};
  f2 fy01 = {ZRT_QSLAB(bfy, 0, sty, oy, ofy, r.iy), ZRT_QSLAB(bfy, 1, sty, oy, ofy, r.iy)};
  f2 fy23 = {ZRT_QSLAB(bfy, 2, sty, oy, ofy, r.iy), ZRT_QSLAB(bfy, 3, sty, oy, ofy, r.iy)};
  f2 fz01 = {ZRT_QSLAB(bfz, 0, stz, oz, ofz, r.iz), ZRT_QSLAB(bfz, 1, stz, oz, ofz, r.iz)};
  f2 fz23 = {ZRT_QSLAB(bfz, 2, stz, oz, ofz, r.iz), ZRT_QSLAB(bfz, 3, stz, oz, ofz, r.iz)};
#undef ZRT_QSLAB
  // per-axis widening (wide_iter, paxis_grow): the same terms, kept for the leaf records
  bool pw = false;
  float gx = 0.0f, gy = 0.0f, gz = 0.0f;
  if (ZRT_PAXIS && PAXIS && __builtin_expect(__ballot(m > a.paxis_m) != 0ull, 0)) {
    pw = true;
    const float g = paxis_grow(a, r);
    gx = paxis_t(g, r.ix); gy = paxis_t(g, r.iy); gz = paxis_t(g, r.iz);
    nx01.x -= gx; nx01.y -= gx; nx23.x -= gx; nx23.y -= gx;
    ny01.x -= gy; ny01.y -= gy; ny23.x -= gy; ny23.y -= gy;
    nz01.x -= gz; nz01.y -= gz; nz23.x -= gz; nz23.y -= gz;
    fx01.x += gx; fx01.y += gx; fx23.x += gx; fx23.y += gx;
    fy01.x += gy; fy01.y += gy; fy23.x += gy; fy23.y += gy;
    fz01.x += gz; fz01.y += gz; fz23.x += gz; fz23.y += gz;
  }
  const SlotT s0 = slot_interval(nx01.x, ny01.x, nz01.x, fx01.x, fy01.x, fz01.x, tb);
  const SlotT s1 = slot_interval(nx01.y, ny01.y, nz01.y, fx01.y, fy01.y, fz01.y, tb);
  const SlotT s2 = slot_interval(nx23.x, ny23.x, nz23.x, fx23.x, fy23.x, fz23.x, tb);
  const SlotT s3 = slot_interval(nx23.y, ny23.y, nz23.y, fx23.y, fy23.y, fz23.y, tb);
  const float rl = pw ? 1.0000153f : rel, sl = (pw ? 0.0f : slk) + E2;
#if ZRT_GRAZE_LEAF
  const float rll = pw ? 1.0000153f : 1.0000153f + r.gl * m;
#else
  const float rll = rl;
#endif
  // the quantized boxes' narrowed test (a superset of the full node's, with its margins)
  const bool h0 = !deg && !(s0.en > __builtin_fmaf(s0.ex, r0 < 0 ? rll : rl, r0 < 0 ? sl : E2));
  const bool h1 = !deg && !(s1.en > __builtin_fmaf(s1.ex, r1 < 0 ? rll : rl, r1 < 0 ? sl : E2));
  const bool h2 = !deg && !(s2.en > __builtin_fmaf(s2.ex, r2 < 0 ? rll : rl, r2 < 0 ? sl : E2));
  const bool h3 = !deg && !(s3.en > __builtin_fmaf(s3.ex, r3 < 0 ? rll : rl, r3 < 0 ? sl : E2));
  if (STATS) {
    ++c_nodes;
    c_leaves += (r0 < 0) + (r1 < 0) + (r2 < 0) + (r3 < 0);
  }
  // candidate leaf slots, decided against their records below: a triangle leaf whose
  // quantized box passes the narrowed test; a sphere leaf (wide_iter: opened by the
  // static test against t_max = +inf, never culled by the best) whose quantized exit
  // can lie past t_min (its exact exit is not larger)
#define ZRT_QCAND(K) \
  (r##K < 0 && r##K != kEmptyRef && \
   (r##K < -kSphereSlotBias ? !deg && s##K.ex + __builtin_fmaf(__builtin_fabsf(s##K.ex), 0x1p-19f, Eg) > 0.001f : h##K))
  uint32_t open = (ZRT_QCAND(0) ? 1u : 0u) | (ZRT_QCAND(1) ? 2u : 0u) | (ZRT_QCAND(2) ? 4u : 0u) |
                  (ZRT_QCAND(3) ? 8u : 0u);
#undef ZRT_QCAND
  const int l0 = r0, l1 = r1, l2 = r2, l3 = r3;
  int32_t next = -1;
  float k0 = r0 >= 0 && h0 ? s0.en : inf, k1 = r1 >= 0 && h1 ? s1.en : inf;
  float k2 = r2 >= 0 && h2 ? s2.en : inf, k3 = r3 >= 0 && h3 ? s3.en : inf;
  const uint32_t n = (k0 != inf) + (k1 != inf) + (k2 != inf) + (k3 != inf);
  if (__ballot(n > 1u) == 0ull) {
    if (n != 0) {
      next = k0 != inf ? r0 : k1 != inf ? r1 : k2 != inf ? r2 : r3;
    } else if (sp != 0) {
      --sp;
      next = sp >= rows ? (row_ok<STATS>(a, (uint64_t)(sp - rows) * a.n_lanes + gl, a.ovf_cap) ? (int32_t)ovf[(size_t)(sp - rows) * a.n_lanes] : -1)
                        : (int32_t)stk[sp * stride];
    }
  } else {
    cswap(k0, r0, k1, r1);
    cswap(k2, r2, k3, r3);
    cswap(k0, r0, k2, r2);
    cswap(k1, r1, k3, r3);
    cswap(k1, r1, k2, r2);
    if (n != 0) {
      const StackT e0 = (StackT)(n == 4 ? r3 : n == 3 ? r2 : r1), e1 = (StackT)(n == 4 ? r2 : r1);
      const StackT e2 = (StackT)r1;
      if (sp + 3 <= rows) {
        stk[sp * stride] = e0;
        stk[(sp + 1) * stride] = e1;
        stk[(sp + 2) * stride] = e2;
      } else {
        const StackT e[3] = {e0, e1, e2};
#pragma unroll
        for (uint32_t j = 0; j < 3; ++j) {
          if (sp + j < rows) {
            stk[(sp + j) * stride] = e[j];
          } else {
            if (row_ok<STATS>(a, (uint64_t)(sp + j - rows) * a.n_lanes + gl, a.ovf_cap))
              ovf[(size_t)(sp + j - rows) * a.n_lanes] = e[j];
            if (STATS) ++coh.ovfw;
          }
        }
      }
      const uint32_t nsp = sp + n - 1;
      if (__builtin_expect(nsp > cap - 3, 0)) atomicOr(a.error_flag, kErrOverflow);
      sp = min(nsp, cap - 3);
      next = r0;
    } else if (sp != 0) {
      --sp;
      next = sp >= rows ? (row_ok<STATS>(a, (uint64_t)(sp - rows) * a.n_lanes + gl, a.ovf_cap) ? (int32_t)ovf[(size_t)(sp - rows) * a.n_lanes] : -1)
                        : (int32_t)stk[sp * stride];
    }
  }
  // each lane walks its candidate leaves in slot order: the record's exact box
  // through wide_iter's leaf decisions, then the primitives
  while (open != 0) {
    const uint32_t k = (uint32_t)__builtin_ctz(open);
    open &= open - 1u;
    const int ref = k == 0 ? l0 : k == 1 ? l1 : k == 2 ? l2 : l3;
    const bool sph = ref < -kSphereSlotBias;
    const uint32_t L = (uint32_t)(-(sph ? ref + kSphereSlotBias : ref) - 1);
    if (__builtin_expect(L >= a.n_qleaves, 0)) {  // a corrupt ref: report, never read past the records
      atomicOr(a.error_flag, kErrLayout);
      continue;
    }
    const float4 mn = a.qleaves[2 * L], mx = a.qleaves[2 * L + 1];
    const float bx = sx ? mx.x : mn.x, cx = sx ? mn.x : mx.x;
    const float by = sy ? mx.y : mn.y, cy = sy ? mn.y : mx.y;
    const float bz = sz ? mx.z : mn.z, cz = sz ? mn.z : mx.z;
    // wide_iter's distances of this slot: the same planes, offsets and widening
    SlotT s = slot_interval(__builtin_fmaf(bx, r.ix, -onx) - gx, __builtin_fmaf(by, r.iy, -ony) - gy,
                            __builtin_fmaf(bz, r.iz, -onz) - gz, __builtin_fmaf(cx, r.ix, -ofx) + gx,
                            __builtin_fmaf(cy, r.iy, -ofy) + gy, __builtin_fmaf(cz, r.iz, -ofz) + gz, tb);
#define ZRT_SURE(S) (__builtin_fmaf(S.en, ZRT_FMA_SLABS ? kFmaSure : 1.0f, Eg) < S.ex)
    // (in wide_iter's order: the narrowed test, the per-axis test within the margin,
    // then a sphere slot's static test, which decides it)
    bool o = !deg && !(s.en > __builtin_fmaf(s.ex, rll, sl));
    if (o && (pw || gg > 0.0f || !ZRT_SURE(s))) o = loose_planes(bx, by, bz, cx, cy, cz, r, tb, s.en, gg);
    if (sph) {
      o = !pw && !deg && ZRT_SURE(s);
      if (!o && !deg && s.ex + __builtin_fmaf(__builtin_fabsf(s.ex), 0x1p-19f, Eg) > 0.001f)
        o = static_ok_planes(bx, by, bz, cx, cy, cz, r, s.en);
    }
#undef ZRT_SURE
    if (!o) continue;
    const int La = as_int(mn.w), pb = as_int(mx.w);
    const float lp = ZRT_HAZARD_ENTRY ? (ZRT_FMA_SLABS ? __builtin_fmaf(s.en, kFmaSure, E2) : s.en) : -1.0f;
    if (STATS) {
      const int f = __builtin_amdgcn_readfirstlane(La);
      coh.ptests += 1u;
      coh.uprims += __ballot(La != f) == 0ull ? 1u : 0u;
    }
    prim_test<true, STATS, ZRT_ORDER_EXACT>(a.prims, La, r, best_t, best, c_tri, c_sph, lp);
    if (pb != La) prim_test<true, STATS, ZRT_ORDER_EXACT>(a.prims, pb, r, best_t, best, c_tri, c_sph, lp);
  }
  if (STATS && next >= 0 && (uint32_t)next >= v.n_top) {
    const int32_t f = __builtin_amdgcn_readfirstlane(next);
    const bool uni = __ballot(next != f || (uint32_t)next < v.n_top) == 0ull;
    ++coh.gnodes;
    coh.unodes += uni ? 1u : 0u;
  }
  if (next < 0) return false;
  if (__builtin_expect((uint32_t)next >= a.n_qnodes, 0)) {  // a corrupt node index: report, never read past the tree
    atomicOr(a.error_flag, kErrLayout);
    return false;
  }
  if ((uint32_t)next < v.n_top) {  // a top-level node: from LDS
    const float4* __restrict__ t = v.top + kQuantNodeF4 * (uint32_t)next;
    q = t;
    qnode_load(t, w);
  } else {
    const uint32_t at = v.base + kQuantNodeF4 * (uint32_t)next;
    const float4* __restrict__ g = a.wnodes + at;
    q = g;
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (SCALAR) {  // one node in every active lane (the lockstep loop): scalar loads
      const uint32_t fa = __builtin_amdgcn_readfirstlane(at);
      if (__ballot(at != fa) == 0ull) {
        typedef const __attribute__((address_space(4))) float4 cfloat4;
        qnode_load((cfloat4*)a.wnodes + fa, w);
        return true;
      }
    }
#endif
    qnode_load(g, w);
  }
  return true;
}

// the suspended node of a wavefront / pool lane (re)loaded, in either format
template <bool QN, class W>
__device__ __forceinline__ void node_load(const float4* q, const WideView& v, W& w) {
  if constexpr (QN) qnode_load(q, w);
  else wide_load(q, v.sx, v.sy, v.sz, w);
}

// zrt_trace over compressed nodes (MODE 8): traverse_wide with wide_iter_q; LOCK: the
// lockstep loop's A/B build (ZRT_LOCK_QN: its margins, wave-uniform nodes from the scalar cache)
template <bool STATS, class StackT, bool LOCK = false>
__device__ __forceinline__ void traverse_wide_q(const KArgs& a, const RayT& r, StackT* __restrict__ stk,
                                                const float4* __restrict__ lds_top, uint32_t gl, float& best_t,
                                                int& best, uint32_t& c_nodes, uint32_t& c_leaves, uint32_t& c_tri,
                                                uint32_t& c_sph, uint32_t& c_replays, Coh& coh) {
  const WideView v = wide_view(a, r, lds_top);
  uint32_t sp = 0;
  const float4* q = ZRT_LDS_TOP ? v.top : a.wnodes + v.base;
  WideNodeQ w;
  qnode_load(q, w);
  while (wide_iter_q<STATS, StackT, LOCK ? ZRT_PAXIS_LOCK != 0 : true, true, LOCK>(
      a, r, v, stk, gl, w, q, sp, best_t, best, c_nodes, c_leaves, c_tri, c_sph, coh)) {
  }
  wide_finish<STATS, StackT>(a, r, stk, gl, best_t, best, c_replays);
}

template <bool STATS, class StackT, bool PAXIS = ZRT_PAXIS_LOCK>
__device__ __forceinline__ void traverse_wide(const KArgs& a, const RayT& r, StackT* __restrict__ stk,
                                              const float4* __restrict__ lds_top, uint32_t gl, float& best_t,
                                              int& best, uint32_t& c_nodes, uint32_t& c_leaves, uint32_t& c_tri,
                                              uint32_t& c_sph, uint32_t& c_replays, Coh& coh) {
  const WideView v = wide_view(a, r, lds_top);
  uint32_t sp = 0;
  // the root is node 0 of this octant's copy (in LDS when the top levels are)
  const float4* q = ZRT_LDS_TOP && !ZRT_Q_GLOBAL ? v.top : a.wnodes + v.base;
  WideNode w;
  wide_load(ZRT_LDS_TOP ? v.top : a.wnodes + v.base, v.sx, v.sy, v.sz, w);
  while (wide_iter<STATS, StackT, ZRT_SCALAR_NODES, PAXIS, true, ZRT_Q_GLOBAL != 0>(
      a, r, v, stk, gl, w, q, sp, best_t, best, c_nodes, c_leaves, c_tri, c_sph, coh)) {
  }
  wide_finish<STATS, StackT>(a, r, stk, gl, best_t, best, c_replays);
}

// ---------------------------------------------------------------------------
// shading
// ---------------------------------------------------------------------------
// @floatToInt(u64, f) then clamp(.., 0, n-1) as it executes on x86-64.
__device__ __forceinline__ uint32_t texel_index(float f, uint32_t n) {
  if (f >= 0.0f && f < 18446744073709551616.0f) {
    const float lim = (float)(n - 1);
    return f >= lim ? n - 1 : (uint32_t)f;
  }
  if (f < 0.0f && f > -1.0f) return 0;
  return n - 1;
}

// A material: the {u_off, v_off, kind, tex_kind} quad is read at the hit;
// color / image descriptor are read where the albedo is needed (keeping the
// whole 48-B record live across scatter spilled it to scratch).
struct MatReg {
  const float4* q;
  float4 m1;  // {u_off, v_off, kind, tex_kind}
  __device__ __forceinline__ uint32_t kind() const { return __float_as_uint(m1.z); }
  __device__ __forceinline__ uint32_t tex_kind() const { return __float_as_uint(m1.w); }
  __device__ __forceinline__ float ior() const { return q[0].w; }
};
__device__ __forceinline__ MatReg load_material(const DevMaterial* __restrict__ mats, uint32_t i) {
  const float4* q = reinterpret_cast<const float4*>(mats + i);
  return MatReg{q, q[1]};
}

// Attenuation codes.  What Material.scatter returns as the attenuation
// (material.zig:43-129) is one of: the (1,1,1) of a dielectric, a solid
// texture's color (a material's), or one texel of an image texture
// (texture.zig:20-74) - so a path stacks a 4-B code per scatter instead of
// three floats, and an image texel is fetched only when the product is taken
// (paths that end black never fetch theirs).  The values are the same f32s, so
// the product (att_product) is bit for bit the recursion's.
//   0xffffffff            dielectric (1, 1, 1)
//   1 << 31 | material    the material's solid color
//   1 << 30 | t           texel t of the f32 RGB store (a.texels)
//   t                     texel t of the 8-bit store (a.texels8, values k / 255)
// (t < 2^30: flatten_scene refuses larger stores)
constexpr uint32_t kAttOne = 0xffffffffu;

// texture.zig:20-74: the texel an image texture's albedo reads, as an att code
__device__ __forceinline__ uint32_t image_texel_code(const MatReg& mr, float u, float v) {
  const float4 m2 = mr.q[2];
  struct { float u_off, v_off; uint32_t img_w, img_h, img_off, img_u8; } m = {
      mr.m1.x, mr.m1.y, __float_as_uint(m2.x), __float_as_uint(m2.y), __float_as_uint(m2.z), __float_as_uint(m2.w)};
  const float uu_first = 1.0f - u + m.u_off;
  float uu = uu_first;
  if (uu_first > 1.0f) uu = uu_first - 1.0f;
  else if (uu_first < 0.0f) uu = uu_first + 1.0f;
  const float vv_first = v + m.v_off;
  float vv = vv_first;
  if (vv_first > 1.0f) vv = vv_first - 1.0f;
  else if (uu_first < 0.0f) vv = vv_first + 1.0f;  // texture.zig:66 tests uu_first
  const uint32_t x = texel_index(uu * (float)m.img_w, m.img_w);
  const uint32_t y = texel_index(vv * (float)m.img_h, m.img_h);
  const uint32_t t = m.img_off + y * m.img_w + x;  // < 2^30
  return m.img_u8 ? t : (1u << 30) | t;
}

// The albedo of a lambertian / metal hit (texture.zig:20-74) as an att code
__device__ __forceinline__ uint32_t albedo_code(const MatReg& mr, uint32_t mat, float u, float v) {
  if (mr.tex_kind() == ZRT_TEX_COLOR) return (1u << 31) | mat;
  return image_texel_code(mr, u, v);
}

// The attenuation an att code stands for
__device__ __forceinline__ V3 att_value(const KArgs& a, const DevMaterial* __restrict__ mats, uint32_t code) {
  if (code == kAttOne) return mk(1.0f, 1.0f, 1.0f);
  if (code >> 31) {
    const float4 c = reinterpret_cast<const float4*>(mats + (code & 0x7fffffffu))[0];
    return mk(c.x, c.y, c.z);
  }
  if (code >> 30) {
    const float* p = a.texels + 3ull * (code & 0x3fffffffu);
    return mk(p[0], p[1], p[2]);
  }
  // 4 B instead of 12 B per texel.  Its values are k / 255 (png_image.zig:88): the
  // correctly rounded quotient, which dev::div_known gives bit for bit for every
  // k in 0..255 (checked exactly: tests/test_host.py) - no dependent table loads
  const uint32_t px = a.texels8[code];
  constexpr float kInv255 = 1.0f / 255.0f;  // RN(1/255)
  return mk(dev::div_known(float(px & 0xffu), 255.0f, kInv255), dev::div_known(float((px >> 8) & 0xffu), 255.0f, kInv255),
            dev::div_known(float((px >> 16) & 0xffu), 255.0f, kInv255));
}

// raytrace.zig:53-58
// unit(d).y alone (vector.zig:88-92 for the one component backgroundColor reads)
__device__ __forceinline__ float unit_y(V3 v) {
  const float l = dev::sqrt_rn(v.x * v.x + v.y * v.y + v.z * v.z);
  if (__builtin_expect(ZRT_FAST_DIV && l >= 0x1p-50f && l <= 0x1p50f && __builtin_fabsf(v.y) >= l * 0x1p-50f, 1))
    return dev::div_core(v.y, l, dev::rcp_core(l));
  return v.y / l;
}

__device__ __forceinline__ V3 background(V3 d) {  // raytrace.zig:53-58
  const float t = 0.5f * (unit_y(d) + 1.0f);
  const float w = 1.0f - t;
  return mk(w + 0.5f * t, w + 0.7f * t, w + 1.0f * t);
}


// ---------------------------------------------------------------------------
// per-wave counter reduction: one 64-bit atomic per wave per counter
// ---------------------------------------------------------------------------
__device__ __forceinline__ void wave_add_u64(unsigned long long* dst, uint32_t v) {
  uint32_t lo = v, hi = 0;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const uint32_t olo = __shfl_xor(lo, off);
    const uint32_t ohi = __shfl_xor(hi, off);
    const uint32_t nlo = lo + olo;
    hi = hi + ohi + (nlo < lo ? 1u : 0u);
    lo = nlo;
  }
  if (__lane_id() == 0 && (lo | hi)) atomicAdd(dst, ((unsigned long long)hi << 32) | lo);
}

__device__ __forceinline__ void Coh::flush(unsigned long long* counters) {
  wave_add_u64(&counters[kGlobalNodes], gnodes);
  wave_add_u64(&counters[kUniformNodes], unodes);
  wave_add_u64(&counters[kPrimLaneTests], ptests);
  wave_add_u64(&counters[kUniformPrims], uprims);
  wave_add_u64(&counters[kAttWrites], attw);
  wave_add_u64(&counters[kAttReads], attr);
  wave_add_u64(&counters[kStackOvfWrites], ovfw);
  wave_add_u64(&counters[kVNodeTrips], vn_trips);
  wave_add_u64(&counters[kVNodeLines], vn_lines);
  wave_add_u64(&counters[kSNodeTrips], sn_trips);
  wave_add_u64(&counters[kRbTrips], rb_trips);
  wave_add_u64(&counters[kVPrimTrips], vp_trips);
  wave_add_u64(&counters[kVPrimLines], vp_lines);
  wave_add_u64(&counters[kSPrimTrips], sp_trips);
  wave_add_u64(&counters[kVShadeTrips], vsh_trips);
  wave_add_u64(&counters[kAttWTrips], attw_trips);
  wave_add_u64(&counters[kAttRTrips], attr_trips);
  wave_add_u64(&counters[kVNodeCost], vn_cost);
  wave_add_u64(&counters[kVPrimCost], vp_cost);
}

// ZRT_FLAG_SCANLINES: a finished unit's counters added to its frame rows.  The
// 8 lanes of a tile row (lanes 8k .. 8k+7) are summed with shuffles, then one
// lane per row adds them.  Called with the whole wave converged.
__device__ __forceinline__ void flush_scanline(unsigned long long* __restrict__ rows, uint32_t py, uint32_t height,
                                               int lane, uint32_t d, uint32_t r, uint32_t b) {
#pragma unroll
  for (int off = 1; off <= 4; off <<= 1) {
    d += __shfl_xor(d, off);
    r += __shfl_xor(r, off);
    b += __shfl_xor(b, off);
  }
  if ((lane & 7) == 0 && py < height) {
    if (d) atomicAdd(&rows[3 * py + 0], (unsigned long long)d);
    if (r) atomicAdd(&rows[3 * py + 1], (unsigned long long)r);
    if (b) atomicAdd(&rows[3 * py + 2], (unsigned long long)b);
  }
}

// ---------------------------------------------------------------------------
// the sampling loop
// ---------------------------------------------------------------------------
// LDS-typed pointers are 32-bit: a generic (flat) float* into LDS costs a 64-bit
// register pair across the whole loop (it was among the values the FAST kernel
// spilled to scratch)
#if defined(__HIP_DEVICE_COMPILE__)
typedef __attribute__((address_space(3))) float lds_float;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
#else
typedef float lds_float;
typedef uint32_t lds_u32;
#endif
constexpr float kPi = 3.14159274101257324f;     // std.math.pi as f32
constexpr float kTwoPi = 6.28318548202514648f;  // comptime 2*pi as f32
constexpr float kInvPi = 1.0f / kPi;              // RN(1/pi), RN(1/(2pi)): dev::div_core's y
constexpr float kInvTwoPi = 1.0f / kTwoPi;

#ifndef ZRT_WAVES_PER_SIMD
#define ZRT_WAVES_PER_SIMD 8  // binary/reference; A/B (tools/ab.sh): w5 11.2, w6 12.1, w7 12.4, w8 12.6 Gray/s
#endif
#ifndef ZRT_WAVES_LIST
#define ZRT_WAVES_LIST 6      // list mode (C2); A/B: w5 27.8, w6 30.3, w8 28.7 Gray/s
#endif
#ifndef ZRT_WAVES_WIDE
#define ZRT_WAVES_WIDE 6      // FAST (wide tree) kernel, 80 VGPRs.  A/B, round 2 (96 VGPRs at w5): w4 46.0, w5 50.6,
                              // w6 48.2 (spills); round 4 (4-B att codes): C4 w5 52.5, w6 55.1, w7 44.8; C3 15.1 / 15.1 / 13.4
#endif

// The rest of one rayColor step after its closest-hit query (raytrace.zig:
// 71-100): a miss is the sky (backgroundColor); a hit is HitRecord.init
// (hit_record.zig:28-41) + Material.scatter (material.zig:43-129): absorbed
// ends the path black, a scatter pushes its attenuation (the product is taken
// in the recursion's order when the path ends) and moves the ray on.
// Where a path's attenuation rows (att codes) live: rows 0 .. a.att_lds_rows-1
// in LDS at lds[row * lds_stride], the rest in global memory at
// a.att[(row - a.att_lds_rows) * g_stride + g_index].  The lockstep, wavefront and
// list loops index them by lane (stride kBlock / a.n_lanes), the path-pool loop by path.
struct AttRows {
  lds_u32* __restrict__ lds;
  uint32_t lds_stride;
  uint64_t g_index;
  uint32_t g_stride;
};

// attenuation_1 * (attenuation_2 * (... * L)): the recursion's association
// (raytrace.zig:99), over the n rows a path pushed, read back in reverse
template <bool STATS>
__device__ __forceinline__ uint32_t att_row(const KArgs& a, const AttRows& ar, uint32_t i, Coh& coh) {
  if (i < a.att_lds_rows) return ar.lds[i * ar.lds_stride];
  if (STATS) {
    ++coh.attr;
    coh.attr_trips += wave_once();
  }
  const uint64_t k = (uint64_t)(i - a.att_lds_rows) * ar.g_stride + ar.g_index;
  return row_ok<STATS>(a, k, a.att_cap) ? a.att[k] : kAttOne;
}
#ifndef ZRT_SHADE_CONVERGE
#define ZRT_SHADE_CONVERGE 0  // BVH loops' shade_step: the operations materials share in Material.scatter issued
                              // once (1, 2: exact at 5 waves per SIMD, a wrong frame from the 6-wave lockstep
                              // kernel's timed flavour - DESIGN.md §3 "The lockstep kernel's spills"; A/B only)
#endif
#ifndef ZRT_ATT_PAIRS
#define ZRT_ATT_PAIRS 1  // att_product decodes two rows at a time (their texel loads in flight together)
#endif
template <bool STATS>
__device__ __forceinline__ V3 att_product(const KArgs& a, const DevMaterial* __restrict__ mats, const AttRows& ar,
                                          uint32_t n, V3 col, Coh& coh) {
  uint32_t i = n;
  // two rows per trip: both texel loads are issued before either product, so a
  // textured path's chain of dependent fetches is half as long (the values and
  // the order of the multiplications are the recursion's, as below)
  if (ZRT_ATT_PAIRS) {
    for (; i >= 2; i -= 2) {
      const V3 hi = att_value(a, mats, att_row<STATS>(a, ar, i - 1, coh));
      const V3 lo = att_value(a, mats, att_row<STATS>(a, ar, i - 2, coh));
      col = mk(hi.x * col.x, hi.y * col.y, hi.z * col.z);
      col = mk(lo.x * col.x, lo.y * col.y, lo.z * col.z);
    }
  }
  for (; i-- > 0;) {
    const V3 at = att_value(a, mats, att_row<STATS>(a, ar, i, coh));
    col = mk(at.x * col.x, at.y * col.y, at.z * col.z);
  }
  return col;
}

template <bool STATS, class R>
__device__ __forceinline__ void shade_step(const KArgs& a, const DevMaterial* __restrict__ mats,
                                           const AttRows& ar, R& rng, int best, float best_t,
                                           V3& o, V3& d, uint32_t& depth_left, bool& path_end, bool& sky, V3& L,
                                           uint32_t& c_bg, uint32_t& c_refl, uint32_t& c_shade, uint32_t& c_tex,
                                           Coh& coh) {
  if (best < 0) {
    ++c_bg;
    L = background(d);
    path_end = true;
    sky = true;
  } else {
    // ---- HitRecord.init (hit_record.zig:28-41)
    float4 sh;
    const int fb = __builtin_amdgcn_readfirstlane(best);
    if (ZRT_SCALAR_PRIMS && __ballot(best != fb) == 0ull) {  // one hit surface in every lane here
#if defined(__HIP_DEVICE_COMPILE__)
      typedef const __attribute__((address_space(4))) float4 cfloat4;
      sh = ((cfloat4*)a.shade)[fb];
#else
      sh = a.shade[fb];
#endif
    } else {
      if (STATS) coh.vsh_trips += wave_once();
      sh = a.shade[best];
    }
    const uint32_t tag = __float_as_uint(sh.w);
    const MatReg mat = load_material(mats, tag & 0x7fffffffu);
    const uint32_t mkind = mat.kind();
    const bool need_uv = mkind != ZRT_MAT_DIELECTRIC && mat.tex_kind() == ZRT_TEX_IMAGE;
    if (STATS) {
      ++c_shade;
      c_tex += need_uv ? 1u : 0u;
    }
    const V3 loc = add(o, scale(d, best_t));
    V3 outward;
    float tu = 0.0f, tv = 0.0f;
    if (tag >> 31) {
      outward = mk(sh.x, sh.y, sh.z);  // face_unit_normal
      if (need_uv) {  // barycentric (u, v), same arithmetic as the hit test
        const float4 p0 = a.prims[3 * best + 0];
        const float4 p1 = a.prims[3 * best + 1];
        const float4 p2 = a.prims[3 * best + 2];
        const V3 n = mk(p2.y, p2.z, p2.w);
        const float det = -dot(d, n);
        const float inv_det = inv_det_rn(det, a.tri_rcp_fast);
        const V3 ao = mk(o.x - p0.x, o.y - p0.y, o.z - p0.z);
        const V3 dao = cross(ao, d);
        tu = dot(mk(p1.z, p1.w, p2.x), dao) * inv_det;
        tv = -dot(mk(p0.w, p1.x, p1.y), dao) * inv_det;
      }
    } else {
      const float4 c = a.prims[3 * best];
      outward = scale(sub(loc, mk(c.x, c.y, c.z)), sh.x);  // (p - c) * (1/r)
      if (need_uv) {  // sphere.zig:47-51
        const float theta = dev::acos_z(-outward.y);
        const float phi = dev::atan2_z(-outward.z, -outward.x) + kPi;
        // phi in {+0} u [2^-23, 2pi], theta in {+0} u [2^-12, pi]: dev::div_core's
        // range, and +0 stays +0 (q = +0, r = +0, q + r*y = +0)
        tu = dev::div_known(phi, kTwoPi, kInvTwoPi);
        tv = dev::div_known(theta, kPi, kInvPi);
      }
    }
    bool front = true;
    V3 normal = outward;
    if (dot(d, outward) > 0.0f) {
      normal = neg(outward);
      front = false;
    }
    // ---- Material.scatter (material.zig:43-129)
    bool absorbed = false;
    uint32_t att = kAttOne;  // the attenuation as an att code (dielectric: (1, 1, 1))
    V3 nd;
#if ZRT_SHADE_CONVERGE == 2
    // as below, every shared piece under a wave-uniform branch (taken when some lane
    // of the wave needs it) that all the wave's lanes run, each lane keeping its own
    // result by a select: no divergent branch around the scatter (the divergent form
    // miscompiled in the 80-VGPR lockstep kernel's timed flavour)
    {
      const bool lamb = mkind == ZRT_MAT_LAMBERTIAN, metal = mkind == ZRT_MAT_METAL;
      const bool diel = !lamb && !metal;
      V3 ud = d;
      if (__ballot(!lamb) != 0ull) {
        const V3 u = unit(d);
        if (!lamb) ud = u;
      }
      float r1 = 0.0f;
      if (__ballot(lamb) != 0ull) {
        R t = rng;
        const float v = rand_float(t);
        rng_keep(rng, t, lamb);
        r1 = lamb ? v : 0.0f;
      }
      float ratio = 1.0f, cos_theta = 0.0f;
      if (__ballot(diel) != 0ull) {
        const float rt = front ? dev::rcp_rn(mat.ior()) : mat.ior();
        const float ct = dev::fmin_z(dot(neg(ud), normal), 1.0f);
        ratio = diel ? rt : 1.0f;
        cos_theta = diel ? ct : 0.0f;
      }
      const float qv = lamb ? r1 : cos_theta;
      const float root = dev::sqrt_rn(1.0f - qv * qv);  // Lambertian rr, dielectric sin_theta
      bool refl = diel && ratio * root > 1.0f;
      const bool schlick = diel && !refl;
      float reflectance = 0.0f;
      if (__ballot(schlick) != 0ull) {
        const float r0 = dev::div_rn(1.0f - ratio, 1.0f + ratio);
        reflectance = r0 + (1.0f - r0) * dev::pow5_z(1.0f - cos_theta);
      }
      const bool draw2 = lamb || schlick;
      float r2 = 0.0f;
      if (__ballot(draw2) != 0ull) {
        R t = rng;
        const float v = rand_float(t);
        rng_keep(rng, t, draw2);
        r2 = draw2 ? v : 0.0f;
      }
      refl = schlick ? reflectance > r2 : refl;
      V3 x = mk(0.0f, 0.0f, 0.0f);
      if (__ballot(lamb) != 0ull) {
        float sn, cs;
        dev::sincos_z(kTwoPi * r2, &sn, &cs);
        V3 hv = mk(cs * root, sn * root, r1);
        R t = rng;
        const bool b = rand_bool(t);
        rng_keep(rng, t, lamb);
        if (!b) hv.z = hv.z * -1.0f;
        const V3 xl = add(normal, hv);
        if (lamb) x = xl;
      }
      const bool rfl = metal || refl, rfr = diel && !refl;
      if (__ballot(rfl) != 0ull) {
        const V3 xr = reflect(ud, normal);
        if (rfl) x = xr;
      }
      if (__ballot(rfr) != 0ull) {
        const V3 xf = refract(ud, normal, ratio);
        if (rfr) x = xf;
      }
      nd = unit(x);
      if (!diel) att = albedo_code(mat, tag & 0x7fffffffu, tu, tv);
      if (metal && !(dot(nd, normal) > 0.0f)) absorbed = true;
    }
#elif ZRT_SHADE_CONVERGE
    // the operations the materials share issued once for the lanes of all of them
    // (shade_hit_a's ZRT_LIST_CONVERGE for the BVH loops): unit(d) of metal and
    // dielectric, sqrt(1 - q^2) and the second draw of Lambertian and dielectric, the
    // reflection of metal and reflected dielectric rays, the final unit() of every
    // scatter and the albedo of Lambertian and metal.  Per lane the same operations on
    // the same values in the same order: bit-identical.
    {
      const bool lamb = mkind == ZRT_MAT_LAMBERTIAN, metal = mkind == ZRT_MAT_METAL;
      const bool diel = !lamb && !metal;
      V3 ud = d;
      if (!lamb) ud = unit(d);
      float r1 = 0.0f;
      if (lamb) r1 = rand_float(rng);
      float ratio = 1.0f, cos_theta = 0.0f;
      if (diel) {
        ratio = front ? dev::rcp_rn(mat.ior()) : mat.ior();
        cos_theta = dev::fmin_z(dot(neg(ud), normal), 1.0f);
      }
      const float qv = lamb ? r1 : cos_theta;
      const float root = dev::sqrt_rn(1.0f - qv * qv);  // Lambertian rr, dielectric sin_theta
      bool refl = diel && ratio * root > 1.0f;
      float reflectance = 0.0f;
      const bool schlick = diel && !refl;
      if (schlick) {
        const float r0 = dev::div_rn(1.0f - ratio, 1.0f + ratio);
        reflectance = r0 + (1.0f - r0) * dev::pow5_z(1.0f - cos_theta);
      }
      float r2 = 0.0f;
      if (lamb || schlick) r2 = rand_float(rng);
      if (schlick) refl = reflectance > r2;
      V3 x;
      if (lamb) {
        float sn, cs;
        dev::sincos_z(kTwoPi * r2, &sn, &cs);
        V3 hv = mk(cs * root, sn * root, r1);
        if (!rand_bool(rng)) hv.z = hv.z * -1.0f;
        x = add(normal, hv);
      } else if (metal || refl) {
        x = reflect(ud, normal);
      } else {
        x = refract(ud, normal, ratio);
      }
      nd = unit(x);
      if (!diel) att = albedo_code(mat, tag & 0x7fffffffu, tu, tv);
      if (metal && !(dot(nd, normal) > 0.0f)) absorbed = true;
    }
#else
    if (mkind == ZRT_MAT_LAMBERTIAN) {
      const float r1 = rand_float(rng);
      const float r2 = rand_float(rng);
      const float rr = dev::sqrt_rn(1.0f - r1 * r1);
      float sn, cs;
      dev::sincos_z(kTwoPi * r2, &sn, &cs);
      V3 hv = mk(cs * rr, sn * rr, r1);
      if (!rand_bool(rng)) hv.z = hv.z * -1.0f;
      nd = unit(add(normal, hv));
      att = albedo_code(mat, tag & 0x7fffffffu, tu, tv);
    } else if (mkind == ZRT_MAT_METAL) {
      nd = unit(reflect(unit(d), normal));
      if (dot(nd, normal) > 0.0f) att = albedo_code(mat, tag & 0x7fffffffu, tu, tv);
      else absorbed = true;
    } else {
      const float ratio = front ? dev::rcp_rn(mat.ior()) : mat.ior();
      const V3 ud = unit(d);
      const float cos_theta = dev::fmin_z(dot(neg(ud), normal), 1.0f);
      const float sin_theta = dev::sqrt_rn(1.0f - cos_theta * cos_theta);
      bool refl = ratio * sin_theta > 1.0f;
      if (!refl) {
        const float r0 = dev::div_rn(1.0f - ratio, 1.0f + ratio);
        const float reflectance = r0 + (1.0f - r0) * dev::pow5_z(1.0f - cos_theta);
        refl = reflectance > rand_float(rng);
      }
      nd = unit(refl ? reflect(ud, normal) : refract(ud, normal, ratio));
    }
#endif
    if (absorbed) {
      path_end = true;  // black
    } else {
      ++c_refl;
      if (depth_left > 1) {  // an attenuation pushed at depth 1 is never read
        // every earlier scatter was at a depth > this one, so all were pushed;
        // the first rows live in LDS, deeper ones in global memory
        const uint32_t i = a.max_depth - depth_left;
        if (i < a.att_lds_rows) {
          ar.lds[i * ar.lds_stride] = att;
        } else {
          const uint64_t k = (uint64_t)(i - a.att_lds_rows) * ar.g_stride + ar.g_index;
          if (row_ok<STATS>(a, k, a.att_cap)) a.att[k] = att;
          if (STATS) {
            ++coh.attw;
            coh.attw_trips += wave_once();
          }
        }
      }
      o = loc;
      d = nd;
      --depth_left;
    }
  }
}

// The lockstep loop's lane state parked in LDS across a traversal: the RNG
// state's words, then the chunk sums (r, g, b), the sample and the depth left,
// each a [word][lane] row of u32 (consecutive lanes, consecutive banks).  The
// traversal writes the stack rows of the same LDS, so the compiler cannot keep
// the values in registers past the traversal: they are stored and re-read.
template <int PRNG>
struct LaneState {
  static constexpr uint32_t kRngWords = sizeof(Rng<PRNG>) / 4;
  static constexpr uint32_t kOdWords = ZRT_LANE_OD ? 6 : 0;  // the ray's origin and direction (park_od)
  static constexpr uint32_t kWords = kRngWords + 5 + kOdWords;
  __device__ __forceinline__ static void park_od(lds_u32* p, V3 o, V3 d) {
    const float v[6] = {o.x, o.y, o.z, d.x, d.y, d.z};
#pragma unroll
    for (uint32_t k = 0; k < kOdWords; ++k) p[(kRngWords + 5 + k) * kBlock] = __float_as_uint(v[k]);
  }
  __device__ __forceinline__ static void unpark_od(const lds_u32* p, V3& o, V3& d) {
    if (!kOdWords) return;
    float v[6];
#pragma unroll
    for (uint32_t k = 0; k < 6; ++k) v[k] = __uint_as_float(p[(kRngWords + 5 + k) * kBlock]);
    o = mk(v[0], v[1], v[2]);
    d = mk(v[3], v[4], v[5]);
  }
  __device__ __forceinline__ static void park(lds_u32* p, const Rng<PRNG>& rng, float r, float g, float b,
                                              uint32_t sample, uint32_t depth) {
    uint32_t w[kRngWords];
    __builtin_memcpy(w, &rng, sizeof(w));
#pragma unroll
    for (uint32_t k = 0; k < kRngWords; ++k) p[k * kBlock] = w[k];
    p[(kRngWords + 0) * kBlock] = __float_as_uint(r);
    p[(kRngWords + 1) * kBlock] = __float_as_uint(g);
    p[(kRngWords + 2) * kBlock] = __float_as_uint(b);
    p[(kRngWords + 3) * kBlock] = sample;
    p[(kRngWords + 4) * kBlock] = depth;
  }
  __device__ __forceinline__ static void unpark(const lds_u32* p, Rng<PRNG>& rng, float& r, float& g, float& b,
                                                uint32_t& sample, uint32_t& depth) {
    uint32_t w[kRngWords];
#pragma unroll
    for (uint32_t k = 0; k < kRngWords; ++k) w[k] = p[k * kBlock];
    __builtin_memcpy(&rng, w, sizeof(w));
    r = __uint_as_float(p[(kRngWords + 0) * kBlock]);
    g = __uint_as_float(p[(kRngWords + 1) * kBlock]);
    b = __uint_as_float(p[(kRngWords + 2) * kBlock]);
    sample = p[(kRngWords + 3) * kBlock];
    depth = p[(kRngWords + 4) * kBlock];
  }
};

// The lockstep interval of a render launch after a scheduling probe (ZRT_AUTO_SYNC):
// the probe ran the same loop over every tile at one sample with the lanes in step,
// and its counters give the share of lane slots that ran a rayColor step (steps =
// reflections + sky hits + depth ends; absorbed metal paths, rare, are not counted).
// Where most lanes wait for a wave's longest path (the teapot, C3: 0.61 of the lane
// slots step, against 0.96 on the bunny, C4) the lanes run the unit's chunk freely
// instead of sample by sample: C3 +3.7 %, C4 -2.8 % with it (profiles/r05/r05l).
// Every wave reads the same counters, so every wave takes the same interval; the
// interval changes no result (each lane still renders its own samples in order).
#ifndef ZRT_AUTO_SYNC_UTIL
#define ZRT_AUTO_SYNC_UTIL 0.8  // lane-step share below which the lanes run free
#endif
__device__ __forceinline__ uint32_t auto_sync(const KArgs& a) {
  if (!a.sync_probe) return a.sync;
  const unsigned long long* p = a.sync_probe;
  const unsigned long long steps = p[kReflections] + p[kBackground] + p[kDepthHits];
  const unsigned long long slots = 64ull * p[kProbeTrips];
  return slots != 0 && double(steps) < ZRT_AUTO_SYNC_UTIL * double(slots) ? a.chunk : a.sync;
}

// StackT: uint16_t when the BVH has < 65536 nodes (halves the LDS stack, so
// more blocks fit per CU), uint32_t otherwise.
// PROBE: the scheduling probe's instance (schedule_probe_kernel): its one-sample
// units - one per tile, 65 536 on C4 - are dealt to the waves round-robin instead of
// through the global counter, whose one atomic per unit serialised the probe
// (ZRT_PROBE_STATIC; the render launch's units are 32 samples and keep the counter)
#ifndef ZRT_PROBE_STATIC
#define ZRT_PROBE_STATIC 1
#endif
template <int MODE /*0 list, 1 BVH binary, 2 BVH reference, 3 wide (FAST)*/, int PRNG, bool STATS, class StackT,
          bool PROBE = false>
__device__ __forceinline__ void render_loop(const KArgs& a) {
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  StackT* stk = reinterpret_cast<StackT*>(lds_raw) + threadIdx.x;  // LDS: the traversal stack
  float4* lds_top = reinterpret_cast<float4*>(lds_raw + a.lds_top_off);
  lds_u32* att_l = (lds_u32*)(lds_raw + a.lds_att_off) + threadIdx.x;  // [row][lane] att codes
  if (MODE == 3 && !layout_ok(a)) return;
  if (MODE == 3 && ZRT_LDS_TOP) fill_lds_top(a, lds_top);
  const DevMaterial* mats = a.mats;
  if (ZRT_MATS_LDS_ONLY && MODE == 3) {  // the host planned the table into LDS: LDS-typed reads
    float4* m = reinterpret_cast<float4*>(lds_raw + a.lds_mat_off);
    fill_lds_mats(a, m);
    mats = reinterpret_cast<const DevMaterial*>(m);
  } else if (a.mats_in_lds) {  // block-uniform
    float4* m = reinterpret_cast<float4*>(lds_raw + a.lds_mat_off);
    fill_lds_mats(a, m);
    mats = reinterpret_cast<const DevMaterial*>(m);
  }
  const int lane = (int)__lane_id();
  const uint32_t gl = blockIdx.x * kBlock + threadIdx.x;  // n_lanes < 2^32
  // FAST: what a lane carries across its traversal - RNG state, chunk sums, sample,
  // depth - is parked in LDS ([word][lane], LaneState) while it traverses: the
  // traversal needs every VGPR of the 6-wave budget, and these values otherwise
  // went to scratch (9 stores + 9 loads per step through the vector-memory path)
  constexpr bool kLaneLds = MODE == 3 && ZRT_LANE_LDS;
  lds_u32* st_l = (lds_u32*)(lds_raw + a.lds_state_off) + threadIdx.x;

  bool active = false, in_sample = false;  // active: this lane still has samples in the wave's unit
  uint32_t sample = 0;
  // wave-uniform unit state (SGPRs): lanes run samples < gate; the unit (one
  // chunk of one tile) ends at unit_end; its tile lt has its corner at (x0, y0)
  uint32_t gate = 0, unit_end = 0, chunk_j = 0, x0 = 0, y0 = 0;
  uint32_t cur_lt = 0xffffffffu, iters = 0;  // the unit's tile, loop iterations spent on it
  const uint32_t sync = MODE == 3 ? auto_sync(a) : a.sync;  // lanes run samples < gate, `sync` at a time
  const uint64_t t_begin = ZRT_PROFILE ? __builtin_amdgcn_s_memrealtime() : 0;
  float acc_r = 0.0f, acc_g = 0.0f, acc_b = 0.0f;
  V3 o = mk(0.0f, 0.0f, 0.0f), d = mk(0.0f, 0.0f, 1.0f);
  uint32_t depth_left = 0;  // attenuations stacked so far: max_depth - depth_left
  Rng<PRNG> rng;
  rng.init(0);
  uint32_t c_rays = 0, c_refl = 0, c_bg = 0, c_depth = 0, c_nodes = 0, c_tri = 0, c_sph = 0;
  uint32_t c_shade = 0, c_tex = 0, c_leaves = 0, c_replays = 0;
  Coh coh;  // STATS
  ExcessAcc excess;  // REFERENCE traversal, STATS flavour only

  uint64_t pf[5] = {0, 0, 0, 0, 0};  // refill, sample start, traversal, shading, path end
  // (PROBE: this wave's next unit; the waves of the grid take units w, w + W, w + 2W ..)
  uint32_t probe_u = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  uint32_t c_trips = 0, c_loops = 0, c_lsteps = 0, nodes_prev = 0;  // STATS: SIMD efficiency
  for (;;) {
    ++iters;
    if (STATS) {  // the wave is converged here: the previous step's traversal trips
      uint32_t m = c_nodes - nodes_prev;
      nodes_prev = c_nodes;
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, off));
      if (lane == 0) c_trips += m;
    }
    uint64_t t0 = prof_stamp();
    // ---- work: the WAVE takes units (local tile lt, a group of unit_chunks
    // chunks) from the global counter, one atomic per unit; lane p renders
    // pixel p of the unit's 8x8 tile.  The lanes run their paths on their own
    // but wait for each other every sync samples (gate), so the wave keeps
    // entering traversal and shading together and its camera rays stay
    // coherent: divergence, not memory, bounds this loop.
    const bool runnable = active && sample < gate;
    if (__ballot(runnable) == 0ull) {
      if (__ballot(active) != 0ull) {
        gate = min(gate + sync, unit_end);
      } else {
        if (cur_lt != 0xffffffffu)  // the finished unit's chunk sums, [chunk][pixel slot]: one 1 KiB store per wave
          a.partial[chunk_j * a.n_slots + cur_lt * 64u + (uint32_t)lane] = make_float4(acc_r, acc_g, acc_b, 0.0f);
        if (a.unit_cost && cur_lt != 0xffffffffu && lane == 0) {
          a.unit_cost[cur_lt] = iters;
          // (the probe's units are one sample: one of the unit's iterations ran no step)
          atomicAdd(&a.counters[kProbeTrips], (unsigned long long)(iters - 1u));
        }
        if (a.scanlines && cur_lt != 0xffffffffu) {  // the finished unit's counters, per frame row
          flush_scanline(a.scanlines, y0 + ((uint32_t)lane >> 3), a.height, lane, c_depth, c_refl, c_bg);
          c_depth = c_refl = c_bg = 0;  // (so the launch totals are the rows' sums)
        }
        uint32_t u = 0;
        if (PROBE && ZRT_PROBE_STATIC) {
          u = probe_u;
          probe_u += gridDim.x * (kBlock / 64);
        } else {
          if (lane == 0) u = atomicAdd(a.work_counter, 1u);
          u = __builtin_amdgcn_readfirstlane(u);
        }
        if (u >= a.total_work) break;  // the counter is exhausted
        const uint32_t ord = u / a.n_chunks, g = u - ord * a.n_chunks;
        const uint32_t lt = a.tile_order ? a.tile_order[ord] : ord;  // costliest tiles first
        cur_lt = lt;
        iters = 0;
        const uint32_t t = lt * a.world + a.rank;  // local tile lt = global tile lt*world + rank
        x0 = (t % a.tiles_x) * 8u;
        y0 = (t / a.tiles_x) * 8u;
        chunk_j = g;
        sample = g * a.chunk;
        unit_end = min(sample + a.chunk, a.spp);
        gate = min(sample + sync, unit_end);
        // lane p renders pixel p of the 8x8 tile; off-frame lanes stay idle (finalize writes black)
        active = x0 + ((uint32_t)lane & 7u) < a.xbound && y0 + ((uint32_t)lane >> 3) < a.height;
        acc_r = acc_g = acc_b = 0.0f;
        in_sample = false;
      }
      if (ZRT_PROFILE) { const uint64_t t = prof_stamp(); pf[0] += t - t0; }
      continue;
    }
    if (ZRT_PROFILE) { const uint64_t t = prof_stamp(); pf[0] += t - t0; t0 = t; }
    if (STATS) {
      c_loops += lane == 0 ? 1u : 0u;
      c_lsteps += runnable ? 1u : 0u;
    }
    if (!runnable) continue;

    // ---- a new sample: jitter + Camera.getRay (raytrace.zig:173-175)
    if (!in_sample) {
      const uint32_t px = x0 + ((uint32_t)lane & 7u), py = y0 + ((uint32_t)lane >> 3);
      const uint64_t offset = (uint64_t)py * a.width + px;
      rng.init(((offset << 16) | (uint64_t)sample) + a.seed_mix);
      const float u = dev::div_known((float)px + rand_float(rng) - 0.5f, a.f_width, a.inv_width);
      const float v = dev::div_known((float)py + rand_float(rng) - 0.5f, a.f_height, a.inv_height);
      const V3 llc = mk(a.llc[0], a.llc[1], a.llc[2]);
      const V3 hor = mk(a.hor[0], a.hor[1], a.hor[2]);
      const V3 ver = mk(a.ver[0], a.ver[1], a.ver[2]);
      o = mk(a.org[0], a.org[1], a.org[2]);
      d = unit(sub(add(add(llc, scale(hor, u)), scale(ver, v)), o));
      depth_left = a.max_depth;
      in_sample = true;
    }
    if (ZRT_PROFILE) { const uint64_t t = prof_stamp(); pf[1] += t - t0; t0 = t; }

    // ---- one rayColor step (raytrace.zig:62-100)
    bool path_end = false, sky = false;
    V3 L = mk(0.0f, 0.0f, 0.0f);
    if (depth_left == 0) {
      ++c_depth;
      path_end = true;
    } else {
      if (STATS) ++c_rays;
      RayT r;
      r.ox = o.x; r.oy = o.y; r.oz = o.z;
      r.dx = d.x; r.dy = d.y; r.dz = d.z;
      r.rcp_det = a.tri_rcp_fast;
      r.gm = a.graze_m;
      r.gl = a.graze_leaf;
      r.gk = a.guard;
      inv_dir(d.x, d.y, d.z, r.ix, r.iy, r.iz);
            float best_t = __builtin_inff();
      int best = -1;
      if (MODE == 0) {
#if ZRT_LIST_SCALAR && defined(__HIP_DEVICE_COMPILE__)
        // the list is wave-uniform: read it through the scalar cache (s_load)
        typedef const __attribute__((address_space(4))) float4 cfloat4;
        cfloat4* cprims = (cfloat4*)a.prims;
        cfloat4* cshade = (cfloat4*)a.shade;
#else
        const float4* cprims = a.prims;
        const float4* cshade = a.shade;
#endif
        for (uint32_t i = 0; i < a.n_list; ++i) {  // surfaces in list order, t_max shrinking
          const uint32_t tag = __float_as_uint(cshade[i].w);
          if (tag >> 31) {
            if (STATS) ++c_tri;
            tri_test_v<false>(cprims[3 * i], cprims[3 * i + 1], cprims[3 * i + 2], (int)i, r, best_t, best);
          } else {
            if (STATS) ++c_sph;
            sphere_test<false>(cprims[3 * i], (int)i, r, best_t, best);
          }
        }
      } else if (MODE == 3) {
        if (kLaneLds) {
          LaneState<PRNG>::park(st_l, rng, acc_r, acc_g, acc_b, sample, depth_left);
          if (ZRT_LANE_OD) LaneState<PRNG>::park_od(st_l, o, d);
        }
        if constexpr (ZRT_LOCK_QN && !PROBE)
          traverse_wide_q<STATS, StackT, true>(a, r, stk, lds_top, gl, best_t, best, c_nodes, c_leaves, c_tri, c_sph,
                                               c_replays, coh);
        else
          traverse_wide<STATS>(a, r, stk, lds_top, gl, best_t, best, c_nodes, c_leaves, c_tri, c_sph, c_replays, coh);
        if (kLaneLds) {
          LaneState<PRNG>::unpark(st_l, rng, acc_r, acc_g, acc_b, sample, depth_left);
          if (ZRT_LANE_OD) LaneState<PRNG>::unpark_od(st_l, o, d);
        }
      } else {
        traverse_bvh<MODE == 1, STATS>(a, r, stk, best_t, best, c_nodes, c_tri, c_sph, &excess);
      }
      if (ZRT_PROFILE) { const uint64_t t = prof_stamp(); pf[2] += t - t0; t0 = t; }
      shade_step<STATS>(a, mats, AttRows{att_l, kBlock, gl, a.n_lanes}, rng, best, best_t, o, d, depth_left, path_end,
                        sky, L, c_bg, c_refl, c_shade, c_tex, coh);
    }

    if (ZRT_PROFILE) { const uint64_t t = prof_stamp(); pf[3] += t - t0; t0 = t; }
    if (path_end) {
      // a path that reached the sky traced at depth_left >= 1: all of its
      // max_depth - depth_left scatters were pushed
      const V3 col = sky ? att_product<STATS>(a, mats, AttRows{att_l, kBlock, gl, a.n_lanes}, a.max_depth - depth_left, L, coh) : L;
      acc_r += col.x;
      acc_g += col.y;
      acc_b += col.z;
      in_sample = false;
      if (++sample == unit_end) active = false;  // chunk done: its sequential sum, stored when the unit ends
    }
    if (ZRT_PROFILE) { const uint64_t t = prof_stamp(); pf[4] += t - t0; }
  }
  if (ZRT_PROFILE && lane == 0) {
    for (int k = 0; k < 5; ++k) atomicAdd(&a.counters[kProfSlot + k], (unsigned long long)pf[k]);
    if (a.wave_times) {
      const uint32_t w = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
      a.wave_times[2 * w] = t_begin;
      a.wave_times[2 * w + 1] = __builtin_amdgcn_s_memrealtime();
    }
  }

  wave_add_u64(&a.counters[kDepthHits], c_depth);
  wave_add_u64(&a.counters[kReflections], c_refl);
  wave_add_u64(&a.counters[kBackground], c_bg);
  if (STATS) {
    wave_add_u64(&a.counters[kRays], c_rays);
    wave_add_u64(&a.counters[kNodes], c_nodes);
    wave_add_u64(&a.counters[kTriTests], c_tri);
    wave_add_u64(&a.counters[kSphereTests], c_sph);
    wave_add_u64(&a.counters[kShades], c_shade);
    wave_add_u64(&a.counters[kTexels], c_tex);
    wave_add_u64(&a.counters[kLeaves], c_leaves);
    wave_add_u64(&a.counters[kReplays], c_replays);
    wave_add_u64(&a.counters[kTravTrips], c_trips);
    wave_add_u64(&a.counters[kLoopTrips], c_loops);
    wave_add_u64(&a.counters[kLaneSteps], c_lsteps);
    coh.flush(a.counters);
    if (MODE == 2) {
      // maxima of non-negative floats: their bit patterns order like unsigned ints
      uint32_t mt = __float_as_uint(excess.tri), ms = __float_as_uint(excess.sph);
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) {
        mt = max(mt, (uint32_t)__shfl_xor((int)mt, off));
        ms = max(ms, (uint32_t)__shfl_xor((int)ms, off));
      }
      if (lane == 0) {
        atomicMax(&a.counters[kExcessTri], (unsigned long long)mt);
        atomicMax(&a.counters[kExcessSph], (unsigned long long)ms);
      }
      wave_add_u64(&a.counters[kExcessHits], excess.over);
    }
  }
}

// ---------------------------------------------------------------------------
// The wavefront loop (FAST traversal, MODE 4).  render_loop keeps a wave's 64
// lanes in lockstep: every lane traces one ray per loop step and the wave
// waits for its slowest traversal.  Where traversal lengths vary a lot between
// lanes (a large mesh filling the frame: teapot, C5) most lanes idle most of
// the time (tools/simd_eff.py: 22-29 % traversal lane efficiency on C3/C5 vs
// 74 % on the bunny).  Here a lane's traversal is suspended between nodes
// (wide_iter), and the wave alternates two phases, chosen with __ballot:
//   traverse: node steps for the lanes with a ray in flight, until at least
//             wf_thresh/64 of the unit's active lanes have finished theirs
//             (the others stay suspended: node, stack, best hit kept);
//   shade:    the finished lanes, together, run the rest of their rayColor
//             step (shade_step) and set up their next ray - the scattered one,
//             or the camera ray of their pixel's next sample - so they rejoin
//             the traversal while the suspended lanes go on.
// The active-ray set is compacted by the ballot counts (no lane waits for the
// whole wave's traversal), the stacks stay in LDS per lane, and every lane
// still renders its own pixel's samples in order (sequential chunk sums, the
// attenuation stack in the recursion's order): images are bit-identical to
// render_loop's.
// ---------------------------------------------------------------------------
template <int PRNG, bool STATS, class StackT>
__device__ __forceinline__ void render_loop_wf(const KArgs& a) {
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  StackT* stk = reinterpret_cast<StackT*>(lds_raw) + threadIdx.x;  // LDS: the traversal stack
  float4* lds_top = reinterpret_cast<float4*>(lds_raw + a.lds_top_off);
  lds_u32* att_l = (lds_u32*)(lds_raw + a.lds_att_off) + threadIdx.x;  // [row][lane] att codes
  if (!layout_ok(a)) return;
  if (ZRT_LDS_TOP) fill_lds_top(a, lds_top);
  const DevMaterial* mats = a.mats;
  if (a.mats_in_lds) {  // block-uniform
    float4* m = reinterpret_cast<float4*>(lds_raw + a.lds_mat_off);
    fill_lds_mats(a, m);
    mats = reinterpret_cast<const DevMaterial*>(m);
  }
  const int lane = (int)__lane_id();
  const uint32_t gl = blockIdx.x * kBlock + threadIdx.x;

  bool active = false;     // this lane has samples left in the wave's unit
  bool in_sample = false;  // ... and one of them is under way
  bool trav = false;       // ... whose current ray is being traversed
  uint32_t sample = 0;
  uint32_t unit_end = 0, chunk_j = 0, x0 = 0, y0 = 0, cur_lt = 0xffffffffu;  // wave-uniform
  float acc_r = 0.0f, acc_g = 0.0f, acc_b = 0.0f;
  V3 o = mk(0.0f, 0.0f, 0.0f), d = mk(0.0f, 0.0f, 1.0f);
  uint32_t depth_left = 0;
  Rng<PRNG> rng;
  rng.init(0);
  // the ray in flight and its suspended traversal
  RayT r{};
  r.rcp_det = a.tri_rcp_fast;
  r.gm = a.graze_m;
  r.gl = a.graze_leaf;
  r.gk = a.guard;
  float best_t = __builtin_inff();
  int best = -1;
  uint32_t sp = 0;
  const float4* q = nullptr;  // the lane's current node (LDS or global)
  uint32_t c_rays = 0, c_refl = 0, c_bg = 0, c_depth = 0, c_nodes = 0, c_tri = 0, c_sph = 0;
  uint32_t c_shade = 0, c_tex = 0, c_leaves = 0, c_replays = 0;
  Coh coh;  // STATS
  uint32_t c_trips = 0, c_loops = 0, c_lsteps = 0;  // STATS: SIMD efficiency

  for (;;) {
    // ---- traverse: node steps while enough lanes still have a ray in flight
    {
      const uint32_t n_act = (uint32_t)__builtin_popcountll(__ballot(active));
      const uint32_t thresh = max(1u, (n_act * a.wf_thresh) >> 6);
      WideView v{};
      WideNode w;
      if (trav) {
        v = wide_view(a, r, lds_top);
        wide_load(q, v.sx, v.sy, v.sz, w);  // the suspended node (re)loaded
      }
      for (;;) {
        if (trav) {
          // (its lanes' nodes are rarely one: no scalar-load test, C5 -1.4 % with it)
          if (!wide_iter<STATS, StackT, false, true, false>(a, r, v, stk, gl, w, q, sp, best_t, best, c_nodes, c_leaves, c_tri,
                                               c_sph, coh)) {
            wide_finish<STATS, StackT>(a, r, stk, gl, best_t, best, c_replays);
            trav = false;
          }
        }
        if (STATS) c_trips += lane == 0 ? 1u : 0u;
        if (__ballot(trav) == 0ull) break;
        if ((uint32_t)__builtin_popcountll(__ballot(active && !trav)) >= thresh) break;
      }
    }
    // ---- refill: the wave's unit is done (lanes wait at unit ends only)
    if (__ballot(active) == 0ull) {
      // the finished unit's chunk sums, [chunk][pixel slot], all 64 lanes at once: one
      // 1 KiB store per wave (stored by each lane as it finished, the lines went out
      // to memory in 32-B pieces: twice the bytes, profiles/r03 write budget)
      if (cur_lt != 0xffffffffu)
        a.partial[chunk_j * a.n_slots + cur_lt * 64u + (uint32_t)lane] = make_float4(acc_r, acc_g, acc_b, 0.0f);
      if (a.scanlines && cur_lt != 0xffffffffu) {
        flush_scanline(a.scanlines, y0 + ((uint32_t)lane >> 3), a.height, lane, c_depth, c_refl, c_bg);
        c_depth = c_refl = c_bg = 0;
      }
      uint32_t u = 0;
      if (lane == 0) u = atomicAdd(a.work_counter, 1u);
      u = __builtin_amdgcn_readfirstlane(u);
      if (u >= a.total_work) break;  // the counter is exhausted
      const uint32_t ord = u / a.n_chunks, g = u - ord * a.n_chunks;
      const uint32_t lt = a.tile_order ? a.tile_order[ord] : ord;  // costliest tiles first
      cur_lt = lt;
      const uint32_t t = lt * a.world + a.rank;
      x0 = (t % a.tiles_x) * 8u;
      y0 = (t / a.tiles_x) * 8u;
      chunk_j = g;
      sample = g * a.chunk;
      unit_end = min(sample + a.chunk, a.spp);
      active = x0 + ((uint32_t)lane & 7u) < a.xbound && y0 + ((uint32_t)lane >> 3) < a.height;
      acc_r = acc_g = acc_b = 0.0f;
      in_sample = false;
      trav = false;
    }
    // ---- shade: the lanes whose ray is done, together
    if (STATS) {
      c_loops += lane == 0 ? 1u : 0u;
      c_lsteps += active && !trav ? 1u : 0u;
    }
    if (!active || trav) continue;
    bool path_end = false, sky = false;
    V3 L = mk(0.0f, 0.0f, 0.0f);
    if (in_sample) {
      shade_step<STATS>(a, mats, AttRows{att_l, kBlock, gl, a.n_lanes}, rng, best, best_t, o, d, depth_left, path_end,
                        sky, L, c_bg, c_refl, c_shade, c_tex, coh);
      if (!path_end && depth_left == 0) {  // the next rayColor is at depth 0: black (raytrace.zig:64-67)
        ++c_depth;
        path_end = true;
      }
    }
    if (path_end) {
      const V3 col = sky ? att_product<STATS>(a, mats, AttRows{att_l, kBlock, gl, a.n_lanes}, a.max_depth - depth_left, L, coh) : L;
      acc_r += col.x;
      acc_g += col.y;
      acc_b += col.z;
      in_sample = false;
      if (++sample == unit_end) {  // chunk done: its sequential sum (stored at the unit's end)
        active = false;
        continue;
      }
    }
    if (!in_sample) {  // a new sample: jitter + Camera.getRay (raytrace.zig:173-175); max_depth >= 1 here
      const uint32_t px = x0 + ((uint32_t)lane & 7u), py = y0 + ((uint32_t)lane >> 3);
      const uint64_t offset = (uint64_t)py * a.width + px;
      rng.init(((offset << 16) | (uint64_t)sample) + a.seed_mix);
      const float u = dev::div_known((float)px + rand_float(rng) - 0.5f, a.f_width, a.inv_width);
      const float vv = dev::div_known((float)py + rand_float(rng) - 0.5f, a.f_height, a.inv_height);
      const V3 llc = mk(a.llc[0], a.llc[1], a.llc[2]);
      const V3 hor = mk(a.hor[0], a.hor[1], a.hor[2]);
      const V3 ver = mk(a.ver[0], a.ver[1], a.ver[2]);
      o = mk(a.org[0], a.org[1], a.org[2]);
      d = unit(sub(add(add(llc, scale(hor, u)), scale(ver, vv)), o));
      depth_left = a.max_depth;
      in_sample = true;
    }
    // ---- the next closest-hit query (raytrace.zig:71-81): suspended at the root
    if (STATS) ++c_rays;
    r.ox = o.x; r.oy = o.y; r.oz = o.z;
    r.dx = d.x; r.dy = d.y; r.dz = d.z;
    inv_dir(d.x, d.y, d.z, r.ix, r.iy, r.iz);
        best_t = __builtin_inff();
    best = -1;
    sp = 0;
    {
      const WideView v = wide_view(a, r, lds_top);
      q = ZRT_LDS_TOP ? v.top : a.wnodes + v.base;
    }
    trav = true;
  }

  wave_add_u64(&a.counters[kDepthHits], c_depth);
  wave_add_u64(&a.counters[kReflections], c_refl);
  wave_add_u64(&a.counters[kBackground], c_bg);
  if (STATS) {
    wave_add_u64(&a.counters[kRays], c_rays);
    wave_add_u64(&a.counters[kNodes], c_nodes);
    wave_add_u64(&a.counters[kTriTests], c_tri);
    wave_add_u64(&a.counters[kSphereTests], c_sph);
    wave_add_u64(&a.counters[kShades], c_shade);
    wave_add_u64(&a.counters[kTexels], c_tex);
    wave_add_u64(&a.counters[kLeaves], c_leaves);
    wave_add_u64(&a.counters[kReplays], c_replays);
    wave_add_u64(&a.counters[kTravTrips], c_trips);
    wave_add_u64(&a.counters[kLoopTrips], c_loops);
    wave_add_u64(&a.counters[kLaneSteps], c_lsteps);
    coh.flush(a.counters);
  }
}

// ---------------------------------------------------------------------------
// The path-pool loop (FAST traversal, MODE 5): the wavefront loop with its rays
// decoupled from lanes.  A wave holds two 64-pixel units at a time (unit slots
// 0 and 1) - 128 paths, each one pixel's current sample - and a queue of the
// paths whose next ray waits for traversal, in LDS.  Two phases alternate,
// chosen with __ballot:
//   traverse: every lane without a ray takes the next queued one - lane k of
//             the idle lanes (mbcnt rank over the ballot of idle lanes) takes
//             queue entry head + k, so the queue is compacted onto the idle
//             lanes - and takes node steps; a finished traversal writes its
//             hit to the path's LDS record and the lane takes the next ray.
//             The phase ends when the queue is empty and fewer than
//             wf_thresh / 64 of the lanes still traverse (the others stay
//             suspended: node, stack, best hit kept in registers).
//   shade:    lane q owns paths q and 64 + q (pixel q of each unit) and shades
//             those whose hit is in (shade_step): the scattered ray, or its
//             pixel's next camera ray, is appended to the queue (ballot +
//             mbcnt again); a unit whose 64 paths have finished their chunk
//             stores its chunk sums and takes the next unit from the global
//             counter.
// A pixel's samples still run one after another on one path, summed in order
// by its owner lane, and every path's attenuations are stacked per path in the
// recursion's order: images are bit-identical to render_loop's.  Rays move
// between lanes, traversals never do (a lane keeps its ray, stack column and
// node until the traversal ends).
// ---------------------------------------------------------------------------
constexpr uint32_t kPoolPaths = 128;                           // per wave: two unit slots of 64 paths
constexpr uint32_t kBlockPaths = kPoolPaths * (kBlock / 64);   // per block
constexpr int32_t kHitPending = -2;                            // a path's hit record before its traversal ends

// One path's state, held by its owner lane: its pixel's sample under way (a path
// whose sample reached its unit's end is done) and the depth left, packed
// (both u16: RenderParams, raytrace.zig:102-108), the chunk's running sum.
template <int PRNG>
struct PathReg {
  Rng<PRNG> rng;
  uint32_t ds;  // depth_left << 16 | sample
  float acc_r, acc_g, acc_b;
  __device__ __forceinline__ uint32_t sample() const { return ds & 0xffffu; }
  __device__ __forceinline__ uint32_t depth_left() const { return ds >> 16; }
};

// ZRT_FLAG_SCANLINES: a path's counter events go straight to its frame row
// (paths of one unit finish at different times here); raytrace.zig:184
__device__ __forceinline__ void scanline_add(const KArgs& a, uint32_t py, uint32_t k, uint32_t n) {
  if (n != 0u && py < a.height) atomicAdd(&a.scanlines[3 * py + k], (unsigned long long)n);
}

// The pool's LDS: rays [6][kBlockPaths] (o.xyz, d.xyz), hits t / slot
// [kBlockPaths], the per-wave queues [waves][kPoolPaths] of path ids.
struct PoolLds {
  lds_float* ray;
  lds_float* hit_t;
  __attribute__((address_space(3))) int32_t* hit_p;
  __attribute__((address_space(3))) uint8_t* queue;  // this wave's
};

// Where a path's attenuation rows past LDS go: [path][row] keeps one path's rows in
// one or two 32-B sectors, so its pushes of one sample (and the next samples') merge
// in L2 before they are written back; [row][path] (0) spreads them, every 4-B code a
// sector of its own (the pool's lanes shade paths at unrelated depths).
#ifndef ZRT_POOL_ATT_PATH
#define ZRT_POOL_ATT_PATH 1
#endif
template <int PRNG, bool STATS, class StackT, bool GUARD, bool QN = false>
__device__ __forceinline__ void render_loop_pool(const KArgs& a) {
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  StackT* stk = reinterpret_cast<StackT*>(lds_raw) + threadIdx.x;  // LDS: the lane's traversal stack column
  float4* lds_top = reinterpret_cast<float4*>(lds_raw + a.lds_top_off);
  if (!layout_ok(a)) return;
  if (ZRT_LDS_TOP) fill_lds_top(a, lds_top);
  const DevMaterial* mats = a.mats;
  if (a.mats_in_lds) {  // block-uniform
    float4* m = reinterpret_cast<float4*>(lds_raw + a.lds_mat_off);
    fill_lds_mats(a, m);
    mats = reinterpret_cast<const DevMaterial*>(m);
  }
  const int lane = (int)__lane_id();
  const uint32_t gl = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t wave_paths = (threadIdx.x >> 6) * kPoolPaths;  // this wave's first path in the block
  const uint64_t g_paths = (uint64_t)blockIdx.x * kBlockPaths;  // the block's first path in the launch
  PoolLds pl;
  {
    lds_float* base = (lds_float*)(lds_raw + a.lds_pool_off);
    pl.ray = base;
    pl.hit_t = base + 6 * kBlockPaths;
    pl.hit_p = (__attribute__((address_space(3))) int32_t*)(base + 7 * kBlockPaths);
    pl.queue = (__attribute__((address_space(3))) uint8_t*)(base + 8 * kBlockPaths) + wave_paths;
  }
  lds_u32* att_base = (lds_u32*)(lds_raw + a.lds_att_off);  // [row][path of the block] att codes
  // global rows past the LDS ones: [path][row] (ZRT_POOL_ATT_PATH), g_rows per path
  const uint32_t g_rows = a.max_depth > a.att_lds_rows ? a.max_depth - a.att_lds_rows : 1u;

  // unit slots (wave-uniform): tile, chunk, the samples [.., unit_end) of the chunk
  bool slot_on[2] = {false, false};
  uint32_t s_lt[2] = {0xffffffffu, 0xffffffffu}, s_chunk[2] = {0, 0}, s_end[2] = {0, 0}, s_x0[2] = {0, 0},
           s_y0[2] = {0, 0};
  bool exhausted = false;  // the global unit counter ran out
  PathReg<PRNG> pA, pB;    // paths lane and 64 + lane (done: sample >= the slot's unit end, 0 while it is off)
  pA.acc_r = pA.acc_g = pA.acc_b = pB.acc_r = pB.acc_g = pB.acc_b = 0.0f;
  pA.ds = pB.ds = 0;
  pA.rng.init(0);
  pB.rng.init(0);
  uint32_t c_depth = 0, c_refl = 0, c_bg = 0;  // Progress counters (raytrace.zig:20-34) of this lane's paths
  uint32_t q_head = 0, q_tail = 0;  // wave-uniform queue positions (mod kPoolPaths)

  // the ray in flight on this lane and its suspended traversal
  bool trav = false;
  uint32_t cp = 0;  // its path (0 .. kPoolPaths-1 of this wave)
  RayT r{};
  r.rcp_det = a.tri_rcp_fast;
  r.gm = a.graze_m;
  r.gl = a.graze_leaf;
  r.gk = GUARD ? a.guard : 0.0f;
  float best_t = __builtin_inff();
  int best = -1;
  uint32_t sp = 0;
  const float4* q = nullptr;
  uint32_t c_rays = 0, c_nodes = 0, c_tri = 0, c_sph = 0, c_shade = 0, c_tex = 0, c_leaves = 0, c_replays = 0;
  Coh coh;  // STATS
  uint32_t c_trips = 0, c_loops = 0, c_lsteps = 0;

  for (;;) {
    // ---- traverse: idle lanes take queued rays; node steps
    {
      // shade once the queue is empty and fewer than 64 - wf_thresh lanes still traverse
      const uint32_t thresh = 64u - a.wf_thresh;
      WideView v{};
      std::conditional_t<QN, WideNodeQ, WideNode> w;
      if (trav) {
        v = wide_view(a, r, lds_top);
        node_load<QN>(q, v, w);  // the suspended node (re)loaded
      }
      for (;;) {
        const uint64_t idle = __ballot(!trav);
        const uint32_t avail = q_tail - q_head;
        if (idle != 0ull && avail != 0u) {
          const uint32_t rank = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32),
                                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
          if (!trav && rank < avail) {  // the rank-th idle lane takes queue entry head + rank
            cp = pl.queue[(q_head + rank) & (kPoolPaths - 1u)];
            const uint32_t P = wave_paths + cp;
            const V3 o = mk(pl.ray[0 * kBlockPaths + P], pl.ray[1 * kBlockPaths + P], pl.ray[2 * kBlockPaths + P]);
            const V3 d = mk(pl.ray[3 * kBlockPaths + P], pl.ray[4 * kBlockPaths + P], pl.ray[5 * kBlockPaths + P]);
            if (STATS) ++c_rays;
            r.ox = o.x; r.oy = o.y; r.oz = o.z;
            r.dx = d.x; r.dy = d.y; r.dz = d.z;
            inv_dir(d.x, d.y, d.z, r.ix, r.iy, r.iz);
            best_t = __builtin_inff();
            best = -1;
            sp = 0;
            v = wide_view(a, r, lds_top);
            q = ZRT_LDS_TOP ? v.top : a.wnodes + v.base;
            node_load<QN>(q, v, w);
            trav = true;
          }
          const uint32_t n_idle = (uint32_t)__builtin_popcountll(idle);
          q_head += n_idle < avail ? n_idle : avail;
        }
        if (trav) {
          bool more;
          if constexpr (QN)
            more = wide_iter_q<STATS, StackT, true, GUARD>(a, r, v, stk, gl, w, q, sp, best_t, best, c_nodes, c_leaves,
                                                          c_tri, c_sph, coh);
          else
            more = wide_iter<STATS, StackT, ZRT_POOL_SCALAR != 0, true, GUARD>(a, r, v, stk, gl, w, q, sp, best_t, best,
                                                                               c_nodes, c_leaves, c_tri, c_sph, coh);
          if (!more) {
            wide_finish<STATS, StackT>(a, r, stk, gl, best_t, best, c_replays);
            const uint32_t P = wave_paths + cp;
            pl.hit_t[P] = best_t;
            pl.hit_p[P] = best;
            trav = false;
          }
        }
        if (STATS) c_trips += lane == 0 ? 1u : 0u;
        const uint32_t n_trav = (uint32_t)__builtin_popcountll(__ballot(trav));
        if (n_trav == 0u) break;
        if (q_tail == q_head && n_trav < thresh) break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // hits written by other lanes of the wave
    // ---- shade: owners shade their paths whose hit is in; units end and refill
#pragma unroll 1
    for (uint32_t s = 0; s < 2; ++s) {
      const uint32_t p = s * 64u + (uint32_t)lane, P = wave_paths + p;
      const AttRows ar = ZRT_POOL_ATT_PATH ? AttRows{att_base + P, kBlockPaths, (g_paths + P) * g_rows, 1u}
                                           : AttRows{att_base + P, kBlockPaths, g_paths + P, a.n_paths};
      const uint32_t unit_end = s ? s_end[1] : s_end[0];
      const uint32_t x0 = s ? s_x0[1] : s_x0[0], y0 = s ? s_y0[1] : s_y0[0];
      bool push = false;
      const uint32_t py = y0 + ((uint32_t)lane >> 3);
      if (pA.sample() < unit_end && pl.hit_p[P] != kHitPending) {
        if (STATS) {
          c_lsteps += 1u;
        }
        V3 o = mk(pl.ray[0 * kBlockPaths + P], pl.ray[1 * kBlockPaths + P], pl.ray[2 * kBlockPaths + P]);
        V3 d = mk(pl.ray[3 * kBlockPaths + P], pl.ray[4 * kBlockPaths + P], pl.ray[5 * kBlockPaths + P]);
        const int hb = pl.hit_p[P];
        const float ht = pl.hit_t[P];
        bool path_end = false, sky = false;
        V3 L = mk(0.0f, 0.0f, 0.0f);
        uint32_t dl = pA.depth_left();
        const uint32_t bg0 = c_bg, rf0 = c_refl;
        shade_step<STATS>(a, mats, ar, pA.rng, hb, ht, o, d, dl, path_end, sky, L, c_bg, c_refl, c_shade, c_tex, coh);
        uint32_t dh = 0;
        if (!path_end && dl == 0) {  // the next rayColor is at depth 0: black (raytrace.zig:64-67)
          ++c_depth;
          dh = 1;
          path_end = true;
        }
        if (a.scanlines) {
          scanline_add(a, py, 0, dh);
          scanline_add(a, py, 1, c_refl - rf0);
          scanline_add(a, py, 2, c_bg - bg0);
        }
        uint32_t smp = pA.sample();
        if (path_end) {
          const V3 col = sky ? att_product<STATS>(a, mats, ar, a.max_depth - dl, L, coh) : L;
          pA.acc_r += col.x;
          pA.acc_g += col.y;
          pA.acc_b += col.z;
          if (++smp < unit_end) {  // the pixel's next sample: jitter + Camera.getRay (raytrace.zig:173-175)
            // (at the unit's end the path is done: its chunk's sequential sum is stored with the unit)
            const uint32_t px = x0 + ((uint32_t)lane & 7u);
            pA.rng.init((((uint64_t)py * a.width + px) << 16 | (uint64_t)smp) + a.seed_mix);
            const float u = dev::div_known((float)px + rand_float(pA.rng) - 0.5f, a.f_width, a.inv_width);
            const float vv = dev::div_known((float)py + rand_float(pA.rng) - 0.5f, a.f_height, a.inv_height);
            o = mk(a.org[0], a.org[1], a.org[2]);
            d = unit(sub(add(add(mk(a.llc[0], a.llc[1], a.llc[2]), scale(mk(a.hor[0], a.hor[1], a.hor[2]), u)),
                             scale(mk(a.ver[0], a.ver[1], a.ver[2]), vv)),
                         o));
            dl = a.max_depth;
            push = true;
          }
        } else {
          push = true;  // the scattered ray
        }
        pA.ds = dl << 16 | smp;
        if (push) {
          pl.ray[0 * kBlockPaths + P] = o.x; pl.ray[1 * kBlockPaths + P] = o.y; pl.ray[2 * kBlockPaths + P] = o.z;
          pl.ray[3 * kBlockPaths + P] = d.x; pl.ray[4 * kBlockPaths + P] = d.y; pl.ray[5 * kBlockPaths + P] = d.z;
          pl.hit_p[P] = kHitPending;
        }
      }
      // the unit in slot s is over: its chunk sums (one 1 KiB store), its rows' counters; the next unit
      const bool s_on = s ? slot_on[1] : slot_on[0];
      if (__ballot(pA.sample() < unit_end) == 0ull && (s_on || !exhausted)) {
        const uint32_t lt = s ? s_lt[1] : s_lt[0];
        if (s_on) {
          const uint32_t cj = s ? s_chunk[1] : s_chunk[0];
          a.partial[cj * a.n_slots + lt * 64u + (uint32_t)lane] = make_float4(pA.acc_r, pA.acc_g, pA.acc_b, 0.0f);
        }
        uint32_t u = a.total_work;
        if (!exhausted) {
          if (lane == 0) u = atomicAdd(a.work_counter, 1u);
          u = __builtin_amdgcn_readfirstlane(u);
        }
        bool on = false;
        uint32_t nlt = 0xffffffffu, g = 0, nx0 = 0, ny0 = 0;
        if (u < a.total_work) {
          const uint32_t ord = u / a.n_chunks;
          g = u - ord * a.n_chunks;
          nlt = a.tile_order ? a.tile_order[ord] : ord;  // costliest tiles first
          const uint32_t t = nlt * a.world + a.rank;
          nx0 = (t % a.tiles_x) * 8u;
          ny0 = (t / a.tiles_x) * 8u;
          on = true;
        } else {
          exhausted = true;
        }
        if (s) { slot_on[1] = on; s_lt[1] = nlt; s_chunk[1] = g; s_x0[1] = nx0; s_y0[1] = ny0; }
        else { slot_on[0] = on; s_lt[0] = nlt; s_chunk[0] = g; s_x0[0] = nx0; s_y0[0] = ny0; }
        pA.acc_r = pA.acc_g = pA.acc_b = 0.0f;
        const uint32_t first = g * a.chunk, end = on ? min(first + a.chunk, a.spp) : 0u;
        if (s) s_end[1] = end;
        else s_end[0] = end;
        pA.ds = end;  // done, unless its pixel is on the frame
        if (on) {
          const uint32_t px = nx0 + ((uint32_t)lane & 7u), ny = ny0 + ((uint32_t)lane >> 3);
          // pixel q of the tile; off-frame paths stay done (finalize writes black)
          if (px < a.xbound && ny < a.height) {
            pA.rng.init((((uint64_t)ny * a.width + px) << 16 | (uint64_t)first) + a.seed_mix);
            const float uu = dev::div_known((float)px + rand_float(pA.rng) - 0.5f, a.f_width, a.inv_width);
            const float vv = dev::div_known((float)ny + rand_float(pA.rng) - 0.5f, a.f_height, a.inv_height);
            const V3 o = mk(a.org[0], a.org[1], a.org[2]);
            const V3 d = unit(sub(add(add(mk(a.llc[0], a.llc[1], a.llc[2]), scale(mk(a.hor[0], a.hor[1], a.hor[2]), uu)),
                                      scale(mk(a.ver[0], a.ver[1], a.ver[2]), vv)),
                                  o));
            pA.ds = a.max_depth << 16 | first;
            pl.ray[0 * kBlockPaths + P] = o.x; pl.ray[1 * kBlockPaths + P] = o.y; pl.ray[2 * kBlockPaths + P] = o.z;
            pl.ray[3 * kBlockPaths + P] = d.x; pl.ray[4 * kBlockPaths + P] = d.y; pl.ray[5 * kBlockPaths + P] = d.z;
            pl.hit_p[P] = kHitPending;
            push = true;
          }
        }
      }
      // append the new rays to the queue: the rank-th pushing lane at tail + rank
      const uint64_t pm = __ballot(push);
      if (pm != 0ull) {
        const uint32_t rank = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(pm >> 32),
                                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)pm, 0u));
        if (push) pl.queue[(q_tail + rank) & (kPoolPaths - 1u)] = (uint8_t)p;
        q_tail += (uint32_t)__builtin_popcountll(pm);
      }
      // the other path's state to the front (both slots go through the same code)
      { PathReg<PRNG> t = pA; pA = pB; pB = t; }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // rays and queue entries written by other lanes
    if (STATS) c_loops += lane == 0 ? 1u : 0u;
    if (!slot_on[0] && !slot_on[1] && __ballot(trav) == 0ull) break;
  }

  if (!a.scanlines) {  // (with ZRT_FLAG_SCANLINES they went to the frame rows, whose sums are the totals)
    wave_add_u64(&a.counters[kDepthHits], c_depth);
    wave_add_u64(&a.counters[kReflections], c_refl);
    wave_add_u64(&a.counters[kBackground], c_bg);
  }
  if (STATS) {
    wave_add_u64(&a.counters[kRays], c_rays);
    wave_add_u64(&a.counters[kNodes], c_nodes);
    wave_add_u64(&a.counters[kTriTests], c_tri);
    wave_add_u64(&a.counters[kSphereTests], c_sph);
    wave_add_u64(&a.counters[kShades], c_shade);
    wave_add_u64(&a.counters[kTexels], c_tex);
    wave_add_u64(&a.counters[kLeaves], c_leaves);
    wave_add_u64(&a.counters[kReplays], c_replays);
    wave_add_u64(&a.counters[kTravTrips], c_trips);
    wave_add_u64(&a.counters[kLoopTrips], c_loops);
    wave_add_u64(&a.counters[kLaneSteps], c_lsteps);
    coh.flush(a.counters);
  }
}

#ifndef ZRT_LIST_MERGE
#define ZRT_LIST_MERGE 1  // list loop: one unit() per step for every new direction (scatters and camera rays)
#endif
#ifndef ZRT_LIST_CONVERGE
#define ZRT_LIST_CONVERGE 1  // list loop: the operations materials share in Material.scatter issued once per wave (C2 +2.9 %, profiles/r06/r06i)
#endif
// shade_step's first half for the list loop (ZRT_LIST_MERGE): a hit's scatter up
// to the direction it normalises.  Every material's new direction - and a new
// sample's camera ray - is normalised once per step for all lanes together
// (unit(), vector.zig:88-92, ~20 VALU: where the materials ran it in their own
// branches a wave paid for it up to six times per step), and a metal scatter's
// absorption test (material.zig:96-101) reads the normalised direction after it.
// Same operations on the same values as shade_step, in the same order per lane.
// pend: 0 nothing to normalise, 1 a scatter, 2 a metal scatter to be tested after.
template <bool STATS, class R>
__device__ __forceinline__ void shade_hit_a(const KArgs& a, const DevMaterial* __restrict__ mats, R& rng, int best,
                                            float best_t, const V3 o, const V3 d, bool& path_end, bool& sky, V3& L,
                                            uint32_t& c_bg, uint32_t& c_shade, uint32_t& c_tex, V3& x, V3& loc,
                                            V3& normal, uint32_t& att, uint32_t& pend) {
  pend = 0;
  if (best < 0) {
    ++c_bg;
    L = background(d);
    path_end = true;
    sky = true;
    return;
  }
  float4 sh;
  const int fb = __builtin_amdgcn_readfirstlane(best);
  if (ZRT_SCALAR_PRIMS && __ballot(best != fb) == 0ull) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef const __attribute__((address_space(4))) float4 cfloat4;
    sh = ((cfloat4*)a.shade)[fb];
#else
    sh = a.shade[fb];
#endif
  } else {
    sh = a.shade[best];
  }
  const uint32_t tag = __float_as_uint(sh.w);
  const MatReg mat = load_material(mats, tag & 0x7fffffffu);
  const uint32_t mkind = mat.kind();
  const bool need_uv = mkind != ZRT_MAT_DIELECTRIC && mat.tex_kind() == ZRT_TEX_IMAGE;
  if (STATS) {
    ++c_shade;
    c_tex += need_uv ? 1u : 0u;
  }
  loc = add(o, scale(d, best_t));
  V3 outward;
  float tu = 0.0f, tv = 0.0f;
  if (tag >> 31) {
    outward = mk(sh.x, sh.y, sh.z);
    if (need_uv) {
      const float4 p0 = a.prims[3 * best + 0];
      const float4 p1 = a.prims[3 * best + 1];
      const float4 p2 = a.prims[3 * best + 2];
      const V3 n = mk(p2.y, p2.z, p2.w);
      const float det = -dot(d, n);
      const float inv_det = inv_det_rn(det, a.tri_rcp_fast);
      const V3 ao = mk(o.x - p0.x, o.y - p0.y, o.z - p0.z);
      const V3 dao = cross(ao, d);
      tu = dot(mk(p1.z, p1.w, p2.x), dao) * inv_det;
      tv = -dot(mk(p0.w, p1.x, p1.y), dao) * inv_det;
    }
  } else {
    const float4 c = a.prims[3 * best];
    outward = scale(sub(loc, mk(c.x, c.y, c.z)), sh.x);
    if (need_uv) {
      const float theta = dev::acos_z(-outward.y);
      const float phi = dev::atan2_z(-outward.z, -outward.x) + kPi;
      tu = dev::div_known(phi, kTwoPi, kInvTwoPi);
      tv = dev::div_known(theta, kPi, kInvPi);
    }
  }
  bool front = true;
  normal = outward;
  if (dot(d, outward) > 0.0f) {
    normal = neg(outward);
    front = false;
  }
  // metal and dielectric both start from unit(d): one normalisation for the lanes of either
  V3 ud = d;
  if (mkind != ZRT_MAT_LAMBERTIAN) ud = unit(d);
#if ZRT_LIST_CONVERGE
  // Material.scatter (material.zig:43-129) with the operations the materials share
  // issued once for the lanes of all of them (a wave whose lanes hit two or three
  // materials otherwise runs each shared piece once per material): the correctly
  // rounded sqrt(1 - q^2) - Lambertian q = its first draw, dielectric q = cos_theta -,
  // the second uniform draw - Lambertian's r2, the dielectric's reflectance draw,
  // each lane's draws still in its own order (r1, r2, bool / one draw after its
  // Schlick term) -, reflect() for metal and reflected dielectric rays, and the
  // albedo lookup for Lambertian and metal.  The same operations on the same values
  // per lane as the branches below: bit-identical (test_list_loops_bit_exact).
  {
    const bool lamb = mkind == ZRT_MAT_LAMBERTIAN, metal = mkind == ZRT_MAT_METAL;
    const bool diel = !lamb && !metal;
    float r1 = 0.0f;
    if (lamb) r1 = rand_float(rng);
    float ratio = 1.0f, cos_theta = 0.0f;
    if (diel) {
      ratio = front ? dev::rcp_rn(mat.ior()) : mat.ior();
      cos_theta = dev::fmin_z(dot(neg(ud), normal), 1.0f);
    }
    const float qv = lamb ? r1 : cos_theta;
    const float root = dev::sqrt_rn(1.0f - qv * qv);  // Lambertian rr, dielectric sin_theta
    bool refl = diel && ratio * root > 1.0f;
    float reflectance = 0.0f;
    const bool schlick = diel && !refl;
    if (schlick) {
      const float r0 = dev::div_rn(1.0f - ratio, 1.0f + ratio);
      reflectance = r0 + (1.0f - r0) * dev::pow5_z(1.0f - cos_theta);
    }
    float r2 = 0.0f;
    if (lamb || schlick) r2 = rand_float(rng);
    if (schlick) refl = reflectance > r2;
    if (lamb) {
      float sn, cs;
      dev::sincos_z(kTwoPi * r2, &sn, &cs);
      V3 hv = mk(cs * root, sn * root, r1);
      if (!rand_bool(rng)) hv.z = hv.z * -1.0f;
      x = add(normal, hv);
    } else if (metal || refl) {
      x = reflect(ud, normal);
    } else {
      x = refract(ud, normal, ratio);
    }
    att = kAttOne;
    if (!diel) att = albedo_code(mat, tag & 0x7fffffffu, tu, tv);  // (metal: used only when not absorbed)
    pend = metal ? 2u : 1u;
    return;
  }
#endif
  if (mkind == ZRT_MAT_LAMBERTIAN) {
    const float r1 = rand_float(rng);
    const float r2 = rand_float(rng);
    const float rr = dev::sqrt_rn(1.0f - r1 * r1);
    float sn, cs;
    dev::sincos_z(kTwoPi * r2, &sn, &cs);
    V3 hv = mk(cs * rr, sn * rr, r1);
    if (!rand_bool(rng)) hv.z = hv.z * -1.0f;
    x = add(normal, hv);
    att = albedo_code(mat, tag & 0x7fffffffu, tu, tv);
    pend = 1;
  } else if (mkind == ZRT_MAT_METAL) {
    x = reflect(ud, normal);
    att = albedo_code(mat, tag & 0x7fffffffu, tu, tv);  // (used only when the scatter is not absorbed)
    pend = 2;
  } else {
    const float ratio = front ? dev::rcp_rn(mat.ior()) : mat.ior();
    const float cos_theta = dev::fmin_z(dot(neg(ud), normal), 1.0f);
    const float sin_theta = dev::sqrt_rn(1.0f - cos_theta * cos_theta);
    bool refl = ratio * sin_theta > 1.0f;
    if (!refl) {
      const float r0 = dev::div_rn(1.0f - ratio, 1.0f + ratio);
      const float reflectance = r0 + (1.0f - r0) * dev::pow5_z(1.0f - cos_theta);
      refl = reflectance > rand_float(rng);
    }
    x = refl ? reflect(ud, normal) : refract(ud, normal, ratio);
    att = kAttOne;
    pend = 1;
  }
}

// ---------------------------------------------------------------------------
// The surface-list loop with per-lane work items (MODE 6; raytrace.zig:71-81
// without a BVH, config C2).  Every ray of a list scene costs the same - all
// n_list surfaces, read through the scalar cache - so the coherence that makes
// the lockstep loop win on a BVH buys nothing here, while its waits cost most
// of the lanes: a wave that steps sample by sample waits for its longest path
// (C2: 2.14 rays per sample, glass paths up to depth 30; VALU lane utilisation
// 0.31).  Here a work item is one (pixel, chunk) - the 64 items of a unit are
// the 64 pixels of its tile - and each lane runs its own item's samples in
// order and takes the next item as soon as it is done: the wave claims a unit
// (one atomic) and hands its pixels to its lanes as they free up (ballot +
// mbcnt rank), so no lane waits for another.  The chunk's sum is the same
// sequential sum in the same slot, so images are bit-identical to the other
// loops'.
// ---------------------------------------------------------------------------
template <int PRNG, bool STATS>
__device__ __forceinline__ void render_loop_list(const KArgs& a) {
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  lds_u32* att_l = (lds_u32*)(lds_raw + a.lds_att_off) + threadIdx.x;  // [row][lane] att codes
  const DevMaterial* mats = a.mats;
  if (ZRT_MATS_LDS_ONLY) {  // the host planned the table into LDS: LDS-typed reads
    float4* m = reinterpret_cast<float4*>(lds_raw + a.lds_mat_off);
    fill_lds_mats(a, m);
    mats = reinterpret_cast<const DevMaterial*>(m);
  } else if (a.mats_in_lds) {  // block-uniform
    float4* m = reinterpret_cast<float4*>(lds_raw + a.lds_mat_off);
    fill_lds_mats(a, m);
    mats = reinterpret_cast<const DevMaterial*>(m);
  }
#if defined(__HIP_DEVICE_COMPILE__)
  typedef const __attribute__((address_space(4))) float4 cfloat4;  // the list is wave-uniform: scalar loads
  cfloat4* cprims = (cfloat4*)a.prims;
  cfloat4* cshade = (cfloat4*)a.shade;
#else
  const float4* cprims = a.prims;
  const float4* cshade = a.shade;
#endif
  const int lane = (int)__lane_id();
  const uint32_t gl = blockIdx.x * kBlock + threadIdx.x;

  bool has = false, in_sample = false;  // this lane holds an item / one of its samples is under way
  bool exhausted = false;               // wave-uniform: the unit counter ran out
  // the wave's current unit (wave-uniform): tile, chunk, corner, next pixel to hand out (64: none left)
  uint32_t u_lt = 0, u_chunk = 0, u_x0 = 0, u_y0 = 0, u_next = 64;
  uint32_t sample = 0, s_end = 0, slot = 0, px = 0, py = 0;
  float acc_r = 0.0f, acc_g = 0.0f, acc_b = 0.0f;
  V3 o = mk(0.0f, 0.0f, 0.0f), d = mk(0.0f, 0.0f, 1.0f);
  uint32_t depth_left = 0;
  Rng<PRNG> rng;
  rng.init(0);
  uint32_t c_rays = 0, c_refl = 0, c_bg = 0, c_depth = 0, c_tri = 0, c_sph = 0, c_shade = 0, c_tex = 0;
  uint32_t c_loops = 0, c_lsteps = 0;
  Coh coh;  // STATS
  for (;;) {
    // ---- refill: the lanes without an item take the next pixels of the wave's
    // current unit (ballot + mbcnt rank); a unit runs dry -> the next one, one
    // atomic per 64 items (an atomic per refill step ran the C2 frame at a
    // quarter of the rate: one global counter for every wave's every step)
    const uint64_t need = __ballot(!has);
    if (need != 0ull && !(exhausted && u_next >= 64u)) {
      const uint32_t rank =
          (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
      const uint32_t cnt = (uint32_t)__builtin_popcountll(need);
      uint32_t taken = 0;  // lanes served so far (by rank)
#pragma unroll 1
      for (int pass = 0; pass < 2 && taken < cnt; ++pass) {
        if (u_next >= 64u) {  // the wave's unit is handed out: claim the next one
          if (exhausted) break;
          uint32_t u = 0;
          if (lane == 0) u = atomicAdd(a.work_counter, 1u);
          u = __builtin_amdgcn_readfirstlane(u);
          if (u >= a.total_work) {
            exhausted = true;
            break;
          }
          const uint32_t ord = u / a.n_chunks;
          u_chunk = u - ord * a.n_chunks;
          u_lt = a.tile_order ? a.tile_order[ord] : ord;
          const uint32_t t = u_lt * a.world + a.rank;  // local tile lt = global tile lt*world + rank
          u_x0 = (t % a.tiles_x) * 8u;
          u_y0 = (t / a.tiles_x) * 8u;
          u_next = 0;
        }
        const uint32_t take = min(cnt - taken, 64u - u_next);
        if (!has && rank >= taken && rank < taken + take) {
          const uint32_t p = u_next + (rank - taken);
          px = u_x0 + (p & 7u);
          py = u_y0 + (p >> 3);
          if (px < a.xbound && py < a.height) {  // off-frame pixels: nothing (finalize writes black)
            has = true;
            in_sample = false;
            sample = u_chunk * a.chunk;
            s_end = min(sample + a.chunk, a.spp);
            slot = u_chunk * a.n_slots + u_lt * 64u + p;
            acc_r = acc_g = acc_b = 0.0f;
          }
        }
        taken += take;
        u_next += take;
      }
    }
    if (__ballot(has) == 0ull) {
      if (exhausted && u_next >= 64u) break;
      continue;  // (every lane drew an off-frame pixel)
    }
    if (STATS) {
      c_loops += lane == 0 ? 1u : 0u;
      c_lsteps += has ? 1u : 0u;
    }
    if (!has) continue;
    // ---- a new sample: jitter + Camera.getRay (raytrace.zig:173-175)
    if (!in_sample) {
      const uint64_t offset = (uint64_t)py * a.width + px;
      rng.init(((offset << 16) | (uint64_t)sample) + a.seed_mix);
      const float u = dev::div_known((float)px + rand_float(rng) - 0.5f, a.f_width, a.inv_width);
      const float v = dev::div_known((float)py + rand_float(rng) - 0.5f, a.f_height, a.inv_height);
      o = mk(a.org[0], a.org[1], a.org[2]);
      d = unit(sub(add(add(mk(a.llc[0], a.llc[1], a.llc[2]), scale(mk(a.hor[0], a.hor[1], a.hor[2]), u)),
                       scale(mk(a.ver[0], a.ver[1], a.ver[2]), v)),
                   o));
      depth_left = a.max_depth;
      in_sample = true;
    }
    // ---- one rayColor step (raytrace.zig:62-100)
    bool path_end = false, sky = false;
    V3 L = mk(0.0f, 0.0f, 0.0f);
    const uint32_t dh0 = c_depth, rf0 = c_refl, bg0 = c_bg;
    const AttRows ar{att_l, kBlock, gl, a.n_lanes};
    V3 x = mk(0.0f, 0.0f, 0.0f), loc = x, nrm = x;  // ZRT_LIST_MERGE: the direction to normalise, hit, normal
    uint32_t att = 0, pend = 0;
    if (depth_left == 0) {
      ++c_depth;
      path_end = true;
    } else {
      if (STATS) ++c_rays;
      RayT r;
      r.ox = o.x; r.oy = o.y; r.oz = o.z;
      r.dx = d.x; r.dy = d.y; r.dz = d.z;
      r.rcp_det = a.tri_rcp_fast;
      r.gm = a.graze_m;
      r.gl = a.graze_leaf;
      r.gk = a.guard;
      inv_dir(d.x, d.y, d.z, r.ix, r.iy, r.iz);
      float best_t = __builtin_inff();
      int best = -1;
      for (uint32_t i = 0; i < a.n_list; ++i) {  // surfaces in list order, t_max shrinking
        const uint32_t tag = __float_as_uint(cshade[i].w);
        if (tag >> 31) {
          if (STATS) ++c_tri;
          tri_test_v<false>(cprims[3 * i], cprims[3 * i + 1], cprims[3 * i + 2], (int)i, r, best_t, best);
        } else {
          if (STATS) ++c_sph;
          sphere_test<false>(cprims[3 * i], (int)i, r, best_t, best);
        }
      }
      if (ZRT_LIST_MERGE)
        shade_hit_a<STATS>(a, mats, rng, best, best_t, o, d, path_end, sky, L, c_bg, c_shade, c_tex, x, loc, nrm, att,
                           pend);
      else
        shade_step<STATS>(a, mats, ar, rng, best, best_t, o, d, depth_left, path_end, sky, L, c_bg, c_refl, c_shade,
                          c_tex, coh);
    }
    bool cam = false;  // ZRT_LIST_MERGE: the item's next sample starts in this step
    if (path_end) {
      const V3 col = sky ? att_product<STATS>(a, mats, ar, a.max_depth - depth_left, L, coh) : L;
      acc_r += col.x;
      acc_g += col.y;
      acc_b += col.z;
      in_sample = false;
      if (++sample == s_end) {  // the chunk's sequential sum, in its [chunk][pixel slot] place
        a.partial[slot] = make_float4(acc_r, acc_g, acc_b, 0.0f);
        has = false;
      } else if (ZRT_LIST_MERGE) {  // the next sample's jitter + Camera.getRay (raytrace.zig:173-175)
        const uint64_t offset = (uint64_t)py * a.width + px;
        rng.init(((offset << 16) | (uint64_t)sample) + a.seed_mix);
        const float u = dev::div_known((float)px + rand_float(rng) - 0.5f, a.f_width, a.inv_width);
        const float v = dev::div_known((float)py + rand_float(rng) - 0.5f, a.f_height, a.inv_height);
        x = sub(add(add(mk(a.llc[0], a.llc[1], a.llc[2]), scale(mk(a.hor[0], a.hor[1], a.hor[2]), u)),
                    scale(mk(a.ver[0], a.ver[1], a.ver[2]), v)),
                mk(a.org[0], a.org[1], a.org[2]));
        cam = true;
        in_sample = true;
      }
    }
    if (ZRT_LIST_MERGE && (pend != 0u || cam)) {  // every new direction of the step, normalised together
      const V3 nd = unit(x);
      if (cam) {
        o = mk(a.org[0], a.org[1], a.org[2]);
        d = nd;
        depth_left = a.max_depth;
      } else if (pend == 1u || dot(nd, nrm) > 0.0f) {  // scattered (material.zig:71-128)
        ++c_refl;
        if (depth_left > 1) {  // (shade_step: an attenuation pushed at depth 1 is never read)
          const uint32_t i = a.max_depth - depth_left;
          if (i < a.att_lds_rows) {
            ar.lds[i * ar.lds_stride] = att;
          } else {
            const uint64_t k = (uint64_t)(i - a.att_lds_rows) * ar.g_stride + ar.g_index;
            if (row_ok<STATS>(a, k, a.att_cap)) a.att[k] = att;
            if (STATS) ++coh.attw;
          }
        }
        o = loc;
        d = nd;
        --depth_left;
      } else {  // a metal scatter absorbed: the path ends black (its next sample starts next step)
        acc_r += 0.0f;
        acc_g += 0.0f;
        acc_b += 0.0f;
        in_sample = false;
        if (++sample == s_end) {
          a.partial[slot] = make_float4(acc_r, acc_g, acc_b, 0.0f);
          has = false;
        }
      }
    }
    if (a.scanlines) {  // this lane's item is one pixel: its events go to its row (raytrace.zig:184)
      scanline_add(a, py, 0, c_depth - dh0);
      scanline_add(a, py, 1, c_refl - rf0);
      scanline_add(a, py, 2, c_bg - bg0);
    }
  }
  if (!a.scanlines) {  // (with ZRT_FLAG_SCANLINES they went to the frame rows, whose sums are the totals)
    wave_add_u64(&a.counters[kDepthHits], c_depth);
    wave_add_u64(&a.counters[kReflections], c_refl);
    wave_add_u64(&a.counters[kBackground], c_bg);
  }
  if (STATS) {
    wave_add_u64(&a.counters[kRays], c_rays);
    wave_add_u64(&a.counters[kTriTests], c_tri);
    wave_add_u64(&a.counters[kSphereTests], c_sph);
    wave_add_u64(&a.counters[kShades], c_shade);
    wave_add_u64(&a.counters[kTexels], c_tex);
    wave_add_u64(&a.counters[kLoopTrips], c_loops);
    wave_add_u64(&a.counters[kLaneSteps], c_lsteps);
    coh.flush(a.counters);
  }
}

#ifndef ZRT_ATT_ROWS_LIST
#define ZRT_ATT_ROWS_LIST 24  // list loops (MODE 0 / 6): attenuation rows kept in LDS (as many as their 6-block share holds)
#endif
#ifndef ZRT_ATT_ROWS_LOCK
#define ZRT_ATT_ROWS_LOCK 4  // lockstep FAST loop: attenuation rows kept in LDS (4 KiB per block, beside its lane state)
#endif
#ifndef ZRT_ATT_ROWS_WF
#define ZRT_ATT_ROWS_WF 12  // wavefront loop: attenuation rows kept in LDS (12 KiB per block, as 4 rows of 3 floats were)
#endif
#ifndef ZRT_WAVES_WF
#define ZRT_WAVES_WF 4  // wavefront loop (MODE 4)
#endif

#ifndef ZRT_WAVES_POOL
#define ZRT_WAVES_POOL 4  // path-pool loop (MODE 5)
#endif
#ifndef ZRT_ATT_ROWS_POOL
#define ZRT_ATT_ROWS_POOL 3  // path-pool loop: attenuation rows kept in LDS per path (2 KiB per row per block)
#endif

template <int MODE, int PRNG, bool STATS, class StackT>
__global__ void __launch_bounds__(kBlock, MODE == 5 || MODE == 7 || MODE == 8 || MODE == 9 ? ZRT_WAVES_POOL
                                          : MODE == 4 ? ZRT_WAVES_WF
                                          : MODE == 3 ? ZRT_WAVES_WIDE
                                          : MODE == 0 || MODE == 6 ? ZRT_WAVES_LIST
                                                      : ZRT_WAVES_PER_SIMD)
    render_kernel(const KArgs a) {
  if constexpr (MODE == 6) render_loop_list<PRNG, STATS>(a);
  else if constexpr (MODE == 5) render_loop_pool<PRNG, STATS, StackT, false>(a);
  else if constexpr (MODE == 7) render_loop_pool<PRNG, STATS, StackT, true>(a);  // with the grazing-triangle guard
  else if constexpr (MODE == 8) render_loop_pool<PRNG, STATS, StackT, false, true>(a);  // compressed nodes
  else if constexpr (MODE == 9) render_loop_pool<PRNG, STATS, StackT, true, true>(a);   // compressed, guarded
  else if constexpr (MODE == 4) render_loop_wf<PRNG, STATS, StackT>(a);
  else render_loop<MODE, PRNG, STATS, StackT>(a);
}

// The scheduling probe (FAST traversal): the same loop over a few samples per
// pixel, one unit per tile, recording each tile's cost (a.unit_cost); its own
// symbol so profiles keep it apart from the render launches.
template <int PRNG, class StackT>
__global__ void __launch_bounds__(kBlock, ZRT_WAVES_WIDE) schedule_probe_kernel(const KArgs a) {
  render_loop<3, PRNG, false, StackT, true>(a);
}

// Closest hit of a batch of rays (zrt_trace): the top-level query of rayColor
// (raytrace.zig:71-81, t_min 0.001, t_max shrinking) through the same
// traversal code as the render loop, one lane per ray.  Ray.init normalises the
// direction (ray.zig:11-13).  Result: t (+inf on a miss) and the device slot.
template <int MODE, class StackT>
__global__ void __launch_bounds__(kBlock) trace_kernel(const KArgs a, const float* __restrict__ rays, uint32_t n,
                                                       float* __restrict__ out_t, int32_t* __restrict__ out_slot) {
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  StackT* stk = reinterpret_cast<StackT*>(lds_raw) + threadIdx.x;
  float4* lds_top = reinterpret_cast<float4*>(lds_raw + a.lds_top_off);
  if ((MODE == 3 || MODE == 8) && !layout_ok(a)) return;
  if ((MODE == 3 || MODE == 8) && ZRT_LDS_TOP) fill_lds_top(a, lds_top);
  const uint32_t gl = blockIdx.x * kBlock + threadIdx.x;
  if (gl >= n) return;
  const float* q = rays + 6ull * gl;
  const V3 d = unit(mk(q[3], q[4], q[5]));
  RayT r;
  r.ox = q[0]; r.oy = q[1]; r.oz = q[2];
  r.dx = d.x; r.dy = d.y; r.dz = d.z;
  r.rcp_det = a.tri_rcp_fast;
  r.gm = a.graze_m;
  r.gl = a.graze_leaf;
  r.gk = a.guard;
  inv_dir(d.x, d.y, d.z, r.ix, r.iy, r.iz);
    float best_t = __builtin_inff();
  int best = -1;
  uint32_t c_nodes = 0, c_leaves = 0, c_tri = 0, c_sph = 0;
  if (MODE == 0) {
    for (uint32_t i = 0; i < a.n_list; ++i) {  // surfaces in list order
      if (__float_as_uint(a.shade[i].w) >> 31) tri_test<false>(a.prims, (int)i, r, best_t, best);
      else sphere_test<false>(a.prims[3 * i], (int)i, r, best_t, best);
    }
  } else if (MODE == 3) {
    uint32_t c_replays = 0;
    Coh coh;
    traverse_wide<false, StackT, true>(a, r, stk, lds_top, gl, best_t, best, c_nodes, c_leaves, c_tri, c_sph, c_replays,
                                       coh);
  } else if (MODE == 8) {  // compressed nodes
    uint32_t c_replays = 0;
    Coh coh;
    traverse_wide_q<false, StackT>(a, r, stk, lds_top, gl, best_t, best, c_nodes, c_leaves, c_tri, c_sph, c_replays,
                                   coh);
  } else {
    traverse_bvh<MODE == 1, false>(a, r, stk, best_t, best, c_nodes, c_tri, c_sph);
  }
  out_t[gl] = best < 0 ? __builtin_inff() : best_t;
  out_slot[gl] = best;
}

// Per-pixel sum of the chunk sums in chunk order, times 1/spp
// (raytrace.zig:182), into the rank's tile-major output.  A launch that set the
// device error flag (a traversal stack overflow) leaves NaN in every pixel, so
// a caller that never asks for the status still cannot take the frame for a
// correct one (the status itself: zrt_ctx_sync / zrt_ctx_stats / zrt_render).
__global__ void finalize_kernel(const float4* __restrict__ partial, float* __restrict__ out,
                                uint32_t n_slots, uint32_t n_chunks, uint32_t world, uint32_t rank,
                                uint32_t tiles_x, uint32_t xbound, uint32_t height, float color_scale,
                                const unsigned long long* __restrict__ error_flag) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_slots) return;
  const uint32_t lt = i >> 6, p = i & 63u;
  const uint32_t t = lt * world + rank;
  const uint32_t px = (t % tiles_x) * 8u + (p & 7u);
  const uint32_t py = (t / tiles_x) * 8u + (p >> 3);
  float r = 0.0f, g = 0.0f, b = 0.0f;
  if (*error_flag != 0ull) {
    r = g = b = __builtin_nanf("");
  } else if (px < xbound && py < height) {
    for (uint32_t j = 0; j < n_chunks; ++j) {  // [chunk][slot]: a wave reads 1 KiB per chunk
      const float4 v = partial[(size_t)j * n_slots + i];
      r += v.x;
      g += v.y;
      b += v.z;
    }
    r *= color_scale;
    g *= color_scale;
    b *= color_scale;
  }
  out[3ull * i + 0] = r;
  out[3ull * i + 1] = g;
  out[3ull * i + 2] = b;
}

// Scatter gathered rank tiles into the framebuffer (raytrace.zig:182 layout).
// Packed (stride_px == 0): rank r's tiles start at rank_base[r].  Padded: rank r
// starts at r * stride_px, as a gather of equal per-rank counts leaves them.
__global__ void assemble_kernel(const float* __restrict__ gathered, float* __restrict__ frame,
                                const uint32_t* __restrict__ rank_base, uint32_t world,
                                uint32_t tiles_x, uint32_t xbound, uint32_t height, uint32_t width,
                                uint32_t total, uint32_t stride_px, uint32_t n_tiles) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  uint32_t r = 0, w = 0;
  if (stride_px) {
    r = i / stride_px;
    w = i - r * stride_px;
  } else {
    // find the rank owning gathered pixel i (world is small)
    while (r + 1 < world && rank_base[r + 1] <= i) ++r;
    w = i - rank_base[r];
  }
  const uint32_t lt = w >> 6, p = w & 63u;
  const uint32_t t = lt * world + r;
  if (t >= n_tiles) return;  // padding
  const uint32_t px = (t % tiles_x) * 8u + (p & 7u);
  const uint32_t py = (t / tiles_x) * 8u + (p >> 3);
  if (px >= xbound || py >= height) return;
  const size_t o = ((size_t)py * width + px) * 3;
  frame[o + 0] = gathered[3ull * i + 0];
  frame[o + 1] = gathered[3ull * i + 1];
  frame[o + 2] = gathered[3ull * i + 2];
}

// Device evaluation of the path's math (parity probes against the oracle).
__global__ void debug_math_kernel(int fn, const float* __restrict__ x, const float* __restrict__ y,
                                  float* __restrict__ out, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float a = x[i], b = y ? y[i] : 0.0f;
  float s, c, r;
  switch (fn) {
    case 0: dev::sincos_z(a, &s, &c); r = s; break;
    case 1: dev::sincos_z(a, &s, &c); r = c; break;
    case 2: r = dev::acos_z(a); break;
    case 3: r = dev::atan_z(a); break;
    case 4: r = dev::sqrt_rn(a); break;
    case 5: r = dev::atan2_z(a, b); break;
    case 6: r = dev::pow5_z(a); break;
    case 8: r = dev::rcp_rn(a); break;
    case 9: r = dev::div_rn(a, b); break;
    default: r = a / b; break;
  }
  out[i] = r;
}

// Self-check of the short correctly rounded divisions (device_math.hpp) against
// HIP's IEEE `/` and sqrtf on this device: counts[0] rcp_rn and sqrt_rn over all
// 2^32 inputs; [1] div_rn
// over n hashed pairs (every exponent, signed zeros, subnormals, inf, NaN, and
// dividends near short multiples of the divisor); [2] unit() over n vectors (wide
// exponents, zero / tiny components); [3] inv_dir over n triples; [4] the jitter
// quotient (x + r - 0.5) / width with y = RN(1/width) over n (width, x, r) draws.
__device__ __forceinline__ uint32_t mix32(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return uint32_t(x);
}
__device__ __forceinline__ bool same_f(float x, float y) {
  return __float_as_uint(x) == __float_as_uint(y) || (x != x && y != y);
}
__device__ __forceinline__ float wild_float(uint32_t h, uint32_t h2) {  // any class, biased to edges
  switch (h2 & 15) {
    case 0: return __uint_as_float(h & 0x807fffffu);                       // +-0, subnormal
    case 1: return __uint_as_float((h & 0x807fffffu) | 0x7f800000u);        // +-inf, NaN
    case 2: return __uint_as_float((h & 0x80ffffffu) | (((h2 >> 4) & 3u) << 23) | 0x3f000000u);  // near 1
    default: return __uint_as_float(h);                                     // any pattern
  }
}
__global__ void debug_division_kernel(uint64_t n, unsigned long long* __restrict__ counts) {
  const uint64_t tid = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0, c4 = 0;
  for (uint64_t i = tid; i < (1ull << 32); i += stride) {
    const float b = __uint_as_float(uint32_t(i));
    c0 += same_f(dev::rcp_rn(b), 1.0f / b) ? 0u : 1u;
    c0 += same_f(dev::sqrt_rn(b), __builtin_sqrtf(b)) ? 0u : 1u;
  }
  for (uint64_t i = tid; i < n; i += stride) {
    const uint32_t h0 = mix32(8 * i), h1 = mix32(8 * i + 1), h2 = mix32(8 * i + 2), h3 = mix32(8 * i + 3);
    const uint32_t h4 = mix32(8 * i + 4), h5 = mix32(8 * i + 5);
    // [1] div_rn
    float a = wild_float(h0, h2), b = wild_float(h1, h2 >> 8);
    if ((h3 & 3) == 0) {  // a close to a short multiple of b (quotients near rounding midpoints)
      const float k = float(int(h3 >> 20) + 1) * 0.0009765625f;
      a = __uint_as_float(__float_as_uint(b * k) + int((h3 >> 2) & 7) - 3);
    }
    c1 += same_f(dev::div_rn(a, b), a / b) ? 0u : 1u;
    // [2] unit(): components of one vector share an exponent window, some zero / tiny
    const int e0 = int(h4 & 255) - 128;
    V3 v;
    float* vp = &v.x;
    for (int k = 0; k < 3; ++k) {
      const uint32_t hk = mix32(8 * i + 6 + uint64_t(k) * 0x100000000ull);
      const int e = e0 + int((hk >> 24) & 31) - 16;
      const uint32_t bexp = uint32_t(e + 127 < 1 ? 0 : e + 127 > 254 ? 254 : e + 127);
      float x = __uint_as_float((hk & 0x807fffffu) | (bexp << 23));
      if (((h5 >> (4 * k)) & 15) == 0) x = (hk & 1) ? -0.0f : 0.0f;
      if (((h5 >> (4 * k)) & 15) == 1) x = __uint_as_float(hk & 0x800fffffu);  // subnormal
      vp[k] = x;
    }
    const float l = __builtin_sqrtf(v.x * v.x + v.y * v.y + v.z * v.z);
    const V3 u = unit(v);
    c2 += (same_f(u.x, v.x / l) && same_f(u.y, v.y / l) && same_f(u.z, v.z / l) && same_f(unit_y(v), v.y / l)) ? 0u : 1u;
    // [3] inv_dir over the same triples and over unit directions
    float ix, iy, iz;
    inv_dir(v.x, v.y, v.z, ix, iy, iz);
    c3 += (same_f(ix, 1.0f / v.x) && same_f(iy, 1.0f / v.y) && same_f(iz, 1.0f / v.z)) ? 0u : 1u;
    inv_dir(u.x, u.y, u.z, ix, iy, iz);
    c3 += (same_f(ix, 1.0f / u.x) && same_f(iy, 1.0f / u.y) && same_f(iz, 1.0f / u.z)) ? 0u : 1u;
    // [4] jitter (raytrace.zig:173): width in [1, 65535], x < 65536, r = Random.float
    const float w = float((h0 & 0xffffu) | 1u) + float((h1 >> 16) & 0xfffeu);
    const float fw = w > 65535.0f ? 65535.0f : w;
    const float px = float(h2 & 0xffffu) * ((h3 >> 30) ? 1.0f : 0.0f);  // many x = 0 (tiny quotients)
    const float r = __uint_as_float((0x7fu << 23) | (h4 >> 9)) - 1.0f;
    const float num = px + r - 0.5f;
    c4 += same_f(dev::div_core(num, fw, 1.0f / fw), num / fw) ? 0u : 1u;
  }
  if (c0) atomicAdd(&counts[0], (unsigned long long)c0);
  if (c1) atomicAdd(&counts[1], (unsigned long long)c1);
  if (c2) atomicAdd(&counts[2], (unsigned long long)c2);
  if (c3) atomicAdd(&counts[3], (unsigned long long)c3);
  if (c4) atomicAdd(&counts[4], (unsigned long long)c4);
}

template <int PRNG>
__global__ void debug_rng_kernel(uint64_t key, unsigned long long* out, uint32_t n) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  Rng<PRNG> r;
  r.init(key);
  for (uint32_t i = 0; i < n; ++i) out[i] = r.next();
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
namespace {

struct HipError {
  hipError_t err;
  std::string where;
};

#define HIPCHK(expr)                                                       \
  do {                                                                     \
    const hipError_t e_ = (expr);                                          \
    if (e_ != hipSuccess) throw ::zrt::HipError{e_, std::string(#expr)};          \
  } while (0)

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p(o.p), n(o.n) {
    o.p = nullptr;
    o.n = 0;
  }
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  void alloc(size_t count) {
    release();
    if (count == 0) count = 1;
    HIPCHK(hipMalloc(&p, count * sizeof(T)));
    n = count;
  }
  void upload(const std::vector<T>& v) {
    alloc(v.size());
    if (!v.empty()) HIPCHK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  }
};

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int check_device(int dev) {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
    return fail(ZRT_E_NODEVICE, "no HIP device visible (the HIP path needs an MI355X / gfx950)");
  if (dev < 0 || dev >= count) return fail(ZRT_E_NODEVICE, "device ordinal out of range");
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return fail(ZRT_E_NODEVICE, "hipGetDeviceProperties failed");
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(ZRT_E_NODEVICE, std::string("device is ") + prop.gcnArchName + ", libzrt is built for gfx950 only");
  return ZRT_OK;
}

int validate_scene(const zrt_scene* s) {
  if (!s) return fail(ZRT_E_INVALID, "scene is null");
  if (s->n_prims && !s->prims) return fail(ZRT_E_INVALID, "prims is null");
  if (s->n_materials && !s->materials) return fail(ZRT_E_INVALID, "materials is null");
  if (s->n_textures && !s->textures) return fail(ZRT_E_INVALID, "textures is null");
  if (s->n_images && !s->images) return fail(ZRT_E_INVALID, "images is null");
  if (s->n_prims >= (1u << 29)) return fail(ZRT_E_UNSUPPORTED, "more than 2^29 primitives");
  for (uint32_t i = 0; i < s->n_prims; ++i) {
    const zrt_prim& p = s->prims[i];
    if (p.kind != ZRT_PRIM_SPHERE && p.kind != ZRT_PRIM_TRIANGLE) return fail(ZRT_E_INVALID, "unknown primitive kind");
    if (p.material >= s->n_materials) return fail(ZRT_E_INVALID, "material index out of range");
  }
  for (uint32_t i = 0; i < s->n_materials; ++i) {
    const zrt_material& m = s->materials[i];
    if (m.kind > ZRT_MAT_DIELECTRIC) return fail(ZRT_E_INVALID, "unknown material kind");
    if (m.kind != ZRT_MAT_DIELECTRIC) {
      if (m.texture >= s->n_textures) return fail(ZRT_E_INVALID, "texture index out of range");
      const zrt_texture& t = s->textures[m.texture];
      if (t.kind > ZRT_TEX_IMAGE) return fail(ZRT_E_INVALID, "unknown texture kind");
      if (t.kind == ZRT_TEX_IMAGE) {
        if (t.image >= s->n_images) return fail(ZRT_E_INVALID, "image index out of range");
        const zrt_image& im = s->images[t.image];
        if (!im.pixels || im.width == 0 || im.height == 0) return fail(ZRT_E_INVALID, "empty image");
      }
    }
  }
  return ZRT_OK;
}

int validate_params(const zrt_params* p) {
  if (!p) return fail(ZRT_E_INVALID, "params is null");
  if (p->width == 0 || p->height == 0 || p->samples_per_pixel == 0)
    return fail(ZRT_E_INVALID, "width, height and samples_per_pixel must be > 0");
  if (p->width > 65535 || p->height > 65535 || p->samples_per_pixel > 65535 || p->max_depth > 65535)
    return fail(ZRT_E_INVALID, "RenderParams fields are u16 (raytrace.zig:102-108)");
  if (p->height > p->width)
    return fail(ZRT_E_INVALID,
                "height > width: raytrace.zig:168 iterates x over image.height and would write past the image");
  if (p->rng_mode != ZRT_RNG_COUNTER)
    return fail(ZRT_E_UNSUPPORTED,
                "the single sequential reference stream cannot be split across GPU lanes; use ZRT_RNG_COUNTER");
  if (p->prng > ZRT_PRNG_XOSHIRO256) return fail(ZRT_E_INVALID, "unknown prng");
  if (p->traversal > ZRT_TRAVERSAL_BINARY) return fail(ZRT_E_INVALID, "unknown traversal");
  if (p->world_size == 0 || p->rank >= p->world_size) return fail(ZRT_E_INVALID, "rank must be < world_size");
  if (p->sample_chunk > 65535) return fail(ZRT_E_INVALID, "sample_chunk must be <= 65535");
  return ZRT_OK;
}

struct Geometry {
  uint32_t xbound, tiles_x, tiles_y, n_tiles;
};
Geometry geometry(const zrt_params* p) {
  Geometry g;
  g.xbound = p->height;  // raytrace.zig:168: `while (x < image.height)`
  g.tiles_x = (g.xbound + 7) / 8;
  g.tiles_y = (p->height + 7) / 8;
  g.n_tiles = g.tiles_x * g.tiles_y;
  return g;
}
uint32_t rank_tiles(const Geometry& g, uint32_t rank, uint32_t world) {
  return g.n_tiles > rank ? (g.n_tiles - rank + world - 1) / world : 0;
}

}  // namespace
}  // namespace zrt

struct zrt_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool use_bvh = false;
  uint32_t n_prims = 0, n_nodes = 0, bvh_depth = 0, stack_depth = 0;
  uint32_t n_wide = 0, n_leaves = 0, wide_stack = 0, wide_stride = 0, n_top = 0, n_mats = 0;
  std::vector<uint32_t> slot_to_prim;  // device primitive slot -> reference list index
  zrt::DevBuf<float4> wnodes;
  zrt::DevBuf<float4> qnodes, qleaves;  // compressed wide nodes + leaf records (q_ok)
  bool q_ok = false;
  uint32_t q_stride = 0, q_top = 0, n_qleaves = 0;
  zrt::DevBuf<float4> nodes, prims, shade;
  zrt::DevBuf<zrt::DevMaterial> mats;
  zrt::DevBuf<float> texels;
  zrt::DevBuf<uint32_t> texels8;
  zrt::DevBuf<uint32_t> leaf_of_slot;
  zrt::DevBuf<uint8_t> ref_sph;
  float root_c[3] = {0.0f, 0.0f, 0.0f}, origin_bound = 0.0f;
  uint32_t layout = 0;  // the wide tree's encoding (KArgs::layout)
  float graze_m = 0x1p-18f, graze_leaf = 0x1p-18f;  // KArgs::graze_m / graze_leaf
  float guard = 0.0f;                                // KArgs::guard
  uint32_t texel_bytes = 0;
  uint32_t tri_rcp_fast = 1;
  float scene_extent = 1.0f;
  float tri_c[3] = {0.0f, 0.0f, 0.0f}, tri_h[3] = {0.0f, 0.0f, 0.0f};  // KArgs::tri_c / tri_h
  zrt::DevBuf<uint32_t> att;  // attenuation rows past the LDS ones (att codes)
  zrt::DevBuf<uint8_t> stack_ovf;  // FAST stack rows beyond the LDS part (deep trees)
  zrt::DevBuf<unsigned long long> scratch;  // counters, work counter, error flag (kScratchSlots)
  zrt::DevBuf<float4> partial;
  zrt::DevBuf<uint32_t> rank_base;
  // scheduling probe: its own partial sums + counters, per-tile costs, the sort
  zrt::DevBuf<float4> probe_partial;
  zrt::DevBuf<unsigned long long> probe_scratch;
  zrt::DevBuf<uint32_t> tile_cost, tile_ids, cost_sorted, tile_order;
  zrt::DevBuf<uint8_t> sort_temp;
  uint32_t tile_ids_n = 0;
  zrt::DevBuf<unsigned long long> wave_times;  // ZRT_PROFILE builds
  uint32_t n_waves = 0;
  zrt::DevBuf<unsigned long long> scanlines;  // ZRT_FLAG_SCANLINES: [row][3] of the last launch
  uint32_t scanline_rows = 0;                 // rows counted by the last launch (0: not flagged)
  bool scheduled = false;
  hipEvent_t ev_pre = nullptr, ev0 = nullptr, ev1 = nullptr, ev_done = nullptr;
  double preprocess_ms = 0, upload_ms = 0;
  // last launch: its device error flag, copied into pinned host memory behind
  // ev_done on the stream it was enqueued on (the caller's, or `stream`)
  unsigned long long* err_host = nullptr;
  bool err_reported = false;  // the last launch's device error was returned to the caller
  uint32_t last_pixels = 0, last_spp = 0, launched = 0;
  uint32_t last_tiles = 0, last_rank = 0, last_world = 1, last_tiles_x = 0, last_xbound = 0;
  bool last_stats = false;
  int last_mode = 0;
  bool last_qn = false;  // the last launch read compressed nodes
  int last_loop = 0;  // zrt_stats::sampling_loop
  float last_guard = 0.0f;  // zrt_stats::guard
  int cu_count = 0;
  ~zrt_ctx() {
    if (ev_pre) (void)hipEventDestroy(ev_pre);
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
    if (ev_done) (void)hipEventDestroy(ev_done);
    if (err_host) (void)hipHostFree(err_host);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

namespace zrt {
namespace {

// The scene flattened for the device (host arrays, built once, uploaded to
// every GPU that renders it).
struct HostScene {
  bool use_bvh = false;
  uint32_t n_prims = 0, n_nodes = 0, bvh_depth = 0;
  uint32_t n_wide = 0, n_leaves = 0, wide_stack = 0, wide_stride = 0, n_top = 0, n_mats = 0;
  uint32_t texel_bytes = 0;
  uint32_t tri_rcp_fast = 1;  // KArgs::tri_rcp_fast
  float scene_extent = 0.0f;  // KArgs::scene_extent
  float tri_c[3] = {0.0f, 0.0f, 0.0f}, tri_h[3] = {0.0f, 0.0f, 0.0f};  // KArgs::tri_c / tri_h
  float root_c[3] = {0.0f, 0.0f, 0.0f}, origin_bound = 0.0f;  // KArgs::root_c / origin_bound
  uint32_t layout = 0;           // KArgs::layout: the wide tree's encoding
  float graze_m = 0x1p-18f;      // KArgs::graze_m (the inner boxes are grown by half of it)
  float graze_leaf = 0x1p-18f;   // KArgs::graze_leaf
  float guard = 0.0f;            // KArgs::guard
  std::vector<uint8_t> ref_sph;  // KArgs::ref_sph
  std::vector<float4> nodes, wn, prims, shade;
  std::vector<float4> qn, ql;  // compressed wide nodes (8 octant copies) and leaf records, when q_ok
  bool q_ok = false;
  uint32_t q_stride = 0;       // float4s per octant copy of qn
  uint32_t q_top = 0;          // compressed nodes served from LDS (their top levels)
  std::vector<DevMaterial> mats;
  std::vector<float> tex;
  std::vector<uint32_t> tex8;
  std::vector<uint32_t> slot_to_prim;  // device primitive slot -> reference list index
  std::vector<uint32_t> leaf_of_slot;  // device primitive slot -> its reference BVH leaf node
  double preprocess_ms = 0;
};

// Meshes from this many primitives have their reference BVH built on the GPU
// (bvh_gpu.hip: same tree; 1.6 M triangles in a fraction of a second instead of
// 5.6 s on the host).  ZRT_BVH_DEVICE=0/1 forces the host / device build.
constexpr uint32_t kDeviceBvhMin = 1u << 16;
bool device_bvh(uint32_t n) {
  if (const char* e = std::getenv("ZRT_BVH_DEVICE")) return std::atoi(e) != 0;
  return n >= kDeviceBvhMin;
}

// The grazing margins' coefficient (DESIGN.md §3 "Grazing rays"): 2^-18;
// ZRT_GRAZE_M overrides it (A/B of larger margins)
float graze_margin() {
  if (const char* e = std::getenv("ZRT_GRAZE_M")) return std::max(0x1p-18f, float(std::atof(e)));
  return 0x1p-18f;
}

// The grazing-triangle guard's coefficient for a scene (DESIGN.md §3
// "Triangles"): an accepted hit of the rounded test (triangle.zig:48-70) lies
// outside its triangle by at most K u |ao| |e1||e2| / det, K = 2.6 the largest
// measured (tools/tri_reach.py; 1.3 on the reference scenes' own triangles,
// tools/tri_reach_bound.py gives the first-order worst case), and det >= 1e-6:
// K u max |e1||e2| / 1e-6 per unit of |ao| <= T + extent (guard_grow).  Capped at
// 2^-10 (above it the guard opens much of the tree; the teapot's model asks 0.024):
// the grazing-triangle rays of every reference scene are exact from 2^-12
// (profiles/r04/r04f).  ZRT_GUARD_K overrides it (A/B).
float guard_model(double max_p12) {
  if (const char* e = std::getenv("ZRT_GUARD_K")) return std::max(0.0f, float(std::atof(e)));
  const double k = 2.6 * 0x1p-24 * max_p12 / 1e-6;
  return float(std::min(k, double(0x1p-10)));
}
float graze_leaf_margin() {  // ZRT_GRAZE_LEAF: leaf slots' coefficient (A/B of a leaf-only guard)
  if (const char* e = std::getenv("ZRT_GRAZE_LEAF")) return std::max(0x1p-18f, float(std::atof(e)));
  return 0x1p-18f;
}

// Flatten the scene for the device: BVH (pre-order), slots in DFS leaf order.
// `device` >= 0: the GPU that may build the BVH (device_bvh).  `qnodes`: build
// the compressed nodes too (1), not (0), or as want_qnodes decides (-1, ZRT_QNODES).
bool want_qnodes(uint32_t n_wide);
uint32_t qtop_levels();
void flatten_scene(HostScene* c, const zrt_scene* s, bool use_bvh, int device, int qnodes = -1) {
  const double t0 = now_ms();
  const uint32_t n = s->n_prims;
  std::vector<uint32_t> slot_to_prim, leaf_of_slot;
  std::vector<float4> nodes;
  uint32_t depth = 0;
  if (use_bvh) {
    BuiltBvh bvh;
    bool built = false;
    if (device >= 0 && device_bvh(n)) {
      // the same tree on the GPU; any HIP failure there (hipMalloc on a busy GPU,
      // a hipcub error) falls back to the host build, which gives the same tree
      try {
        built = build_bvh_device(s->prims, n, device, &bvh);
      } catch (const Error& e) {
        if (std::getenv("ZRT_DEBUG_LAUNCH"))
          std::fprintf(stderr, "zrt preprocess: device BVH build failed (%s); host build\n", e.what());
        (void)hipGetLastError();  // clear a sticky runtime error of the failed build
      }
    }
    if (!built) bvh = build_bvh(s->prims, n);
    if (std::getenv("ZRT_DEBUG_LAUNCH"))
      std::fprintf(stderr, "zrt preprocess: reference BVH %zu nodes in %.1f ms\n", bvh.nodes.size(), now_ms() - t0);
    depth = bvh.max_depth;
    nodes.resize(2 * bvh.nodes.size());
    std::vector<int32_t> prim_slot(n, -1);
    auto ref_of = [&](int32_t child) -> int32_t {
      if (child >= 0) return child;
      const uint32_t prim = uint32_t(-child - 1);
      if (prim_slot[prim] < 0) {
        prim_slot[prim] = int32_t(slot_to_prim.size());
        slot_to_prim.push_back(prim);
      }
      const int32_t kind = s->prims[prim].kind == ZRT_PRIM_TRIANGLE ? 1 : 0;
      return -(2 * prim_slot[prim] + kind) - 1;
    };
    std::vector<RefLeaf> leaves;
    for (size_t i = 0; i < bvh.nodes.size(); ++i) {  // pre-order == reference DFS order
      const BuildNode& b = bvh.nodes[i];
      const int32_t l = ref_of(b.left);
      const int32_t r = ref_of(b.right);
      if (b.left < 0) {  // a reference leaf: its box and its primitive refs
        for (const int32_t ref : {l, r}) {
          const uint32_t slot = uint32_t(-ref - 1) >> 1;
          if (leaf_of_slot.size() <= slot) leaf_of_slot.resize(slot + 1);
          leaf_of_slot[slot] = uint32_t(i);
        }
        RefLeaf L;
        for (int k = 0; k < 3; ++k) {
          L.mn[k] = b.mn[k];
          L.mx[k] = b.mx[k];
        }
        L.prim_a = l;
        L.prim_b = r;
        leaves.push_back(L);
      }
      float4 lo, hi;
      lo.x = b.mn[0]; lo.y = b.mn[1]; lo.z = b.mn[2];
      hi.x = b.mx[0]; hi.y = b.mx[1]; hi.z = b.mx[2];
      std::memcpy(&lo.w, &l, 4);
      std::memcpy(&hi.w, &r, 4);
      nodes[2 * i] = lo;
      nodes[2 * i + 1] = hi;
    }
    c->n_nodes = uint32_t(bvh.nodes.size());
    // Spheres (DESIGN.md §3 "Spheres").  The rounded disc of sphere.zig:31-41 errs by
    // E <= 32 u (|oc|^2 + r^2) (u = 2^-24, three rounded dot products and two
    // subtractions), so an accepted ray passes within sqrt(r^2 + E) - r <= sqrt(E) of
    // the sphere and its hit errs by <= 1.5 sqrt(E) in t: subtrees holding a sphere
    // are grown by 2 sqrt(E) = 2^-8.5 R, R >= |oc| + r for every ray whose origin
    // lies within 2 H of the root box's center on every axis (H: its largest half
    // extent; |oc| <= 2 sqrt(3) H + sqrt(3) H, r <= H).  Rays from farther out are
    // traced the reference's way (render.hip ray_origin_ok).
    c->ref_sph.assign(bvh.nodes.size(), 0);
    bool any_sphere = false;
    for (size_t i = bvh.nodes.size(); i-- > 0;) {  // pre-order: children after their parent
      const BuildNode& b = bvh.nodes[i];
      uint8_t f = 0;
      for (const int32_t ch : {b.left, b.right}) {
        if (ch >= 0) f |= c->ref_sph[size_t(ch)];
        else f |= s->prims[uint32_t(-ch - 1)].kind == ZRT_PRIM_SPHERE ? 1 : 0;
      }
      c->ref_sph[i] = f;
      any_sphere = any_sphere || f;
    }
    // The region the bound is sized over: the root box united with every sphere's
    // centre -+ |radius|.  A negative radius (the reference scenes use them) makes
    // sphere.zig:25's box inverted, so the root box alone need not cover that
    // sphere's surface.
    float lo[3], hi[3];
    for (int k = 0; k < 3; ++k) {
      lo[k] = bvh.nodes[0].mn[k];
      hi[k] = bvh.nodes[0].mx[k];
    }
    for (uint32_t i = 0; i < n; ++i) {
      const zrt_prim& p = s->prims[i];
      if (p.kind != ZRT_PRIM_SPHERE) continue;
      const float r = std::fabs(p.radius), cc[3] = {p.center.x, p.center.y, p.center.z};
      for (int k = 0; k < 3; ++k) {  // (rounded outward: the f32 box contains the exact one)
        lo[k] = std::min(lo[k], std::nextafter(cc[k] - r, -HUGE_VALF));
        hi[k] = std::max(hi[k], std::nextafter(cc[k] + r, HUGE_VALF));
      }
    }
    float H = 0.0f;
    for (int k = 0; k < 3; ++k) {
      c->root_c[k] = 0.5f * lo[k] + 0.5f * hi[k];
      H = std::max(H, std::max(hi[k] - c->root_c[k], c->root_c[k] - lo[k]));
    }
    if (!(H < 0x1p100f)) H = 0x1p100f;  // NaN / huge extents: every origin fails ray_origin_ok's bound
    // Only sphere slots depend on where a ray starts (their growth is sized for
    // origins within 2 H); the triangle margins do not, so a scene without spheres
    // accepts every origin (a distant camera no longer replays every ray)
    c->origin_bound = any_sphere ? 2.0f * H : HUGE_VALF;
    const float sphere_grow = any_sphere ? float(std::ldexp(std::sqrt(2.0), -9) * (3.0 * std::sqrt(3.0) + 1.0) * double(H)) : 0.0f;
    const double tw = now_ms();
    c->graze_m = graze_margin();
    c->graze_leaf = std::max(c->graze_m, graze_leaf_margin());
    c->guard = 0.0f;  // (set below, once the triangles are known)
    // the top levels stored first (LDS): two for the full 128-B nodes; a tree that
    // also gets compressed nodes stores qtop_levels() (their 64-B nodes leave room
    // for a third level in the path pool's LDS), the full kernels reading the first two
    const uint32_t n_leaf_est = uint32_t(leaves.size());
    const bool want_q = qnodes >= 0 ? qnodes != 0 : want_qnodes((n_leaf_est + 2) / 3);  // (about leaves / 3 nodes)
    const uint32_t top_levels = want_q ? qtop_levels() : 2u;
    const WideBvh wide = build_wide_bvh(leaves, top_levels, ZRT_GROW ? 0.5f * c->graze_m : 0.0f,
                                        ZRT_SPHERE_SLOTS ? sphere_grow : 0.0f, ZRT_SPHERE_SLOTS != 0);
    if (std::getenv("ZRT_DEBUG_LAUNCH"))
      std::fprintf(stderr, "zrt preprocess: wide tree %u nodes in %.1f ms\n", wide.n_nodes, now_ms() - tw);
    const size_t nw = wide.nodes.size();
#if ZRT_OCT_COPIES
    // one copy per ray octant o (bit k set: direction k negative) with axis k's
    // min / max planes swapped, so float4 0-2 are the near planes, 3-5 the far
    std::vector<float4> wn(8 * nw);
    for (uint32_t o = 0; o < 8; ++o) {
      float4* dst = wn.data() + o * nw;
      std::memcpy(dst, wide.nodes.data(), nw * sizeof(float4));
      for (size_t i = 0; i < nw; i += 8)
        for (int k = 0; k < 3; ++k)
          if (o >> k & 1u) std::swap(dst[i + k], dst[i + 3 + k]);
    }
#else
    std::vector<float4> wn(nw);
    std::memcpy(wn.data(), wide.nodes.data(), nw * sizeof(float4));
#endif
    c->wide_stack = wide.max_stack + 3;  // + the dead entries of a branch-free push
    // compressed nodes for trees past the caches (want_qnodes): the same tree, 64-B nodes
    // (quantize_wide stores octant copies with pre-swapped planes, which wide_iter_q
    // reads as such: never built for a one-copy A/B build, ZRT_OCT_COPIES = 0)
    if (want_q && ZRT_OCT_COPIES) {
      const double tq = now_ms();
      QuantWide qw = quantize_wide(wide);
      if (qw.ok) {
        c->qn.resize(qw.nodes.size());
        std::memcpy(c->qn.data(), qw.nodes.data(), qw.nodes.size() * sizeof(float4));
        c->ql.resize(std::max<size_t>(1, qw.leaves.size()));
        std::memcpy(c->ql.data(), qw.leaves.data(), qw.leaves.size() * sizeof(float4));
        c->q_ok = true;
        c->q_stride = qw.n_nodes * kQuantNodeF4;
        c->q_top = wide.n_top;
      }
      if (std::getenv("ZRT_DEBUG_LAUNCH"))
        std::fprintf(stderr, "zrt preprocess: compressed nodes %s, %u leaf records, %.1f ms\n", qw.ok ? "built" : "refused",
                     qw.n_leaves, now_ms() - tq);
    }
    c->wn = std::move(wn);
    c->wide_stride = uint32_t(nw);
    c->n_wide = wide.n_nodes;
    c->n_leaves = wide.n_leaves;
    c->n_top = wide.level_end.empty() ? 0u : wide.level_end[std::min<size_t>(2, wide.level_end.size()) - 1];
    c->layout = wide.layout;
    if (const char* e = std::getenv("ZRT_DEBUG_TREE_LAYOUT"))  // tests: a tree another kernel would have to decode
      c->layout ^= uint32_t(std::strtoul(e, nullptr, 0));
    if (c->layout != kKernelLayout)
      throw Error(ZRT_E_UNSUPPORTED, "the wide tree's layout (" + std::to_string(c->layout) +
                                         ") is not the one this library's kernels decode (" +
                                         std::to_string(kKernelLayout) + "): accel_build and render.hip disagree");
  } else {
    for (uint32_t i = 0; i < n; ++i) slot_to_prim.push_back(i);
  }
  std::vector<float4> prims(3 * size_t(slot_to_prim.size()));
  std::vector<float4> shade(slot_to_prim.size());
  double tlo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, thi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
  double tri_p12 = 0.0;  // the largest |e1| |e2| (guard_model)
  for (size_t sl = 0; sl < slot_to_prim.size(); ++sl) {
    const zrt_prim& p = s->prims[slot_to_prim[sl]];
    if (p.kind == ZRT_PRIM_TRIANGLE)  // ray_slack: the triangles' largest |coordinate|
      for (const auto& v : {p.a, p.b, p.c}) {
        c->scene_extent = std::max({c->scene_extent, std::fabs(v.x), std::fabs(v.y), std::fabs(v.z)});
        const double vk[3] = {v.x, v.y, v.z};
        for (int k = 0; k < 3; ++k) {  // (NaN coordinates: the box becomes NaN, paxis_grow infinite)
          tlo[k] = vk[k] < tlo[k] || vk[k] != vk[k] ? vk[k] : tlo[k];
          thi[k] = vk[k] > thi[k] || vk[k] != vk[k] ? vk[k] : thi[k];
        }
      }
    float4* q = &prims[3 * sl];
    float4& sh = shade[sl];
    uint32_t tag = p.material;
    if (p.kind == ZRT_PRIM_TRIANGLE) {
      // triangle.zig:35-38: e1 = b-a, e2 = c-a, n = e1 x e2, unit n = n / |n|
      const float e1x = p.b.x - p.a.x, e1y = p.b.y - p.a.y, e1z = p.b.z - p.a.z;
      const float e2x = p.c.x - p.a.x, e2y = p.c.y - p.a.y, e2z = p.c.z - p.a.z;
      const float nx = e1y * e2z - e1z * e2y;
      const float ny = e1z * e2x - e1x * e2z;
      const float nz = e1x * e2y - e1y * e2x;
      const float len = std::sqrt(nx * nx + ny * ny + nz * nz);
      q[0] = make_float4(p.a.x, p.a.y, p.a.z, e1x);
      q[1] = make_float4(e1y, e1z, e2x, e2y);
      q[2] = make_float4(e2z, nx, ny, nz);
      tag |= 0x80000000u;
      sh = make_float4(nx / len, ny / len, nz / len, 0.0f);
      // |det| = |d . n| <= |d| |n| < (1 + 2^-22) sqrt(3) 2^124 < 2^126 (NaN fails too)
      const float mn = std::max(std::fabs(nx), std::max(std::fabs(ny), std::fabs(nz)));
      if (!(mn < 0x1p124f)) c->tri_rcp_fast = 0;
      // the grazing guard's model (guard_model): the largest |e1| |e2| of the scene
      const double p12 = std::sqrt((double(e1x) * e1x + double(e1y) * e1y + double(e1z) * e1z) *
                                   (double(e2x) * e2x + double(e2y) * e2y + double(e2z) * e2z));
      if (p12 == p12) tri_p12 = std::max(tri_p12, p12);
    } else {
      q[0] = make_float4(p.center.x, p.center.y, p.center.z, p.radius * p.radius);  // sphere.zig:35 r*r, once
      q[1] = make_float4(0, 0, 0, 0);
      q[2] = make_float4(0, 0, 0, 0);
      sh = make_float4(1.0f / p.radius, 0.0f, 0.0f, 0.0f);  // sphere.zig:46 scale(1.0/radius)
    }
    std::memcpy(&sh.w, &tag, 4);
  }
  if (use_bvh) c->guard = guard_model(tri_p12);
  // the triangles' bounding box as centre and half extents, rounded so that the
  // f32 box contains the exact one (paxis_grow); no triangle: an empty box at 0
  for (int k = 0; k < 3; ++k) {
    if (!(tlo[k] <= thi[k])) {
      if (tlo[k] == HUGE_VAL) tlo[k] = thi[k] = 0.0;  // no triangles
      else { c->tri_c[k] = 0.0f; c->tri_h[k] = HUGE_VALF; continue; }  // NaN
    }
    const double ctr = 0.5 * tlo[k] + 0.5 * thi[k];
    c->tri_c[k] = float(ctr);
    const double h = std::max(thi[k] - double(c->tri_c[k]), double(c->tri_c[k]) - tlo[k]);
    c->tri_h[k] = std::nextafter(float(h), HUGE_VALF);
  }
  // materials + textures.  An image whose every value is exactly k/255 (what
  // png_image.zig:76-89 produces) is stored as 8-bit RGBX and expanded through
  // a table of the same f32 values; any other image stays f32 RGB.
  float lut[256];
  for (int k = 0; k < 256; ++k) lut[k] = float(k) / 255.0f;
  std::vector<DevMaterial> mats(s->n_materials);
  std::vector<uint64_t> img_off(s->n_images);
  std::vector<uint32_t> img_u8(s->n_images, 0);
  uint64_t texel_count = 0, texel8_count = 0;
  for (uint32_t i = 0; i < s->n_images; ++i) {
    const zrt_image& im = s->images[i];
    const size_t nv = 3 * size_t(im.width) * im.height;
    bool exact = true;
    for (size_t j = 0; j < nv && exact; ++j) {
      const float v = im.pixels[j];
      const long k = std::lrint(double(v) * 255.0);
      exact = k >= 0 && k <= 255 && std::memcmp(&lut[k], &v, 4) == 0;
    }
    img_u8[i] = exact ? 1u : 0u;
    uint64_t& count = exact ? texel8_count : texel_count;
    img_off[i] = count;
    count += uint64_t(im.width) * im.height;
  }
  if (texel_count >= (1ull << 30) || texel8_count >= (1ull << 30))  // (att codes carry a 30-bit texel index)
    throw Error(ZRT_E_UNSUPPORTED, "more than 2^30 texels in one store");
  for (uint32_t i = 0; i < s->n_materials; ++i) {
    const zrt_material& m = s->materials[i];
    DevMaterial dm{};
    dm.kind = m.kind;
    dm.ior = m.index_of_refraction;
    dm.tex_kind = ZRT_TEX_COLOR;
    if (m.kind != ZRT_MAT_DIELECTRIC) {
      const zrt_texture& t = s->textures[m.texture];
      dm.tex_kind = t.kind;
      dm.r = t.color.x;
      dm.g = t.color.y;
      dm.b = t.color.z;
      dm.u_off = t.u_offset;
      dm.v_off = t.v_offset;
      if (t.kind == ZRT_TEX_IMAGE) {
        dm.img_w = s->images[t.image].width;
        dm.img_h = s->images[t.image].height;
        dm.img_off = uint32_t(img_off[t.image]);
        dm.img_u8 = img_u8[t.image];
      }
    }
    mats[i] = dm;
  }
  std::vector<float> tex(3 * texel_count);
  std::vector<uint32_t> tex8(texel8_count);
  for (uint32_t i = 0; i < s->n_images; ++i) {
    const zrt_image& im = s->images[i];
    const size_t np = size_t(im.width) * im.height;
    if (img_u8[i]) {
      for (size_t j = 0; j < np; ++j) {
        uint32_t px = 0;
        for (int ch = 0; ch < 3; ++ch)
          px |= uint32_t(std::lrint(double(im.pixels[3 * j + ch]) * 255.0)) << (8 * ch);
        tex8[img_off[i] + j] = px;
      }
    } else {
      std::memcpy(&tex[3 * img_off[i]], im.pixels, sizeof(float) * 3 * np);
    }
  }
  c->texel_bytes = s->n_images == 0 ? 0u : texel_count == 0 ? 4u : 12u;
  c->nodes = std::move(nodes);
  c->prims = std::move(prims);
  c->shade = std::move(shade);
  c->mats = std::move(mats);
  c->tex = std::move(tex);
  c->tex8 = std::move(tex8);
  c->slot_to_prim = std::move(slot_to_prim);
  c->leaf_of_slot = std::move(leaf_of_slot);
  c->preprocess_ms = now_ms() - t0;
  c->use_bvh = use_bvh;
  c->n_prims = n;
  c->bvh_depth = depth;
}

// Upload a flattened scene to the context's device.
void upload_scene(zrt_ctx* c, const HostScene& h) {
  const double t1 = now_ms();
  c->nodes.upload(h.nodes);
  c->wnodes.upload(h.wn);
  if (h.q_ok) {
    c->qnodes.upload(h.qn);
    c->qleaves.upload(h.ql);
  }
  c->q_ok = h.q_ok;
  c->q_stride = h.q_stride;
  c->q_top = h.q_top;
  c->n_qleaves = uint32_t(h.ql.size() / kLeafRecF4);
  c->prims.upload(h.prims);
  c->shade.upload(h.shade);
  c->mats.upload(h.mats);
  c->texels.upload(h.tex);
  c->texels8.upload(h.tex8);
  c->leaf_of_slot.upload(h.leaf_of_slot);
  c->ref_sph.upload(h.ref_sph);
  for (int k = 0; k < 3; ++k) c->root_c[k] = h.root_c[k];
  c->origin_bound = h.origin_bound;
  c->layout = h.layout;
  c->graze_m = h.graze_m;
  c->graze_leaf = h.graze_leaf;
  c->guard = h.guard;
  c->upload_ms = now_ms() - t1;
  c->preprocess_ms = h.preprocess_ms;
  c->use_bvh = h.use_bvh;
  c->n_prims = h.n_prims;
  c->n_nodes = h.n_nodes;
  c->bvh_depth = h.bvh_depth;
  c->stack_depth = h.use_bvh ? h.bvh_depth + 2 : 0;
  c->n_wide = h.n_wide;
  c->n_leaves = h.n_leaves;
  c->n_top = h.n_top;
  c->n_mats = uint32_t(h.mats.size());
  c->wide_stack = h.wide_stack;
  c->wide_stride = h.wide_stride;
  c->texel_bytes = h.texel_bytes;
  c->tri_rcp_fast = h.tri_rcp_fast;
  c->scene_extent = h.scene_extent;
  for (int k = 0; k < 3; ++k) {
    c->tri_c[k] = h.tri_c[k];
    c->tri_h[k] = h.tri_h[k];
  }
  c->slot_to_prim = h.slot_to_prim;
}

// The wavefront loop (render_loop_wf) for this scene?  ZRT_WF=0/1 forces it.
// It doubles the traversal lane efficiency where traversal lengths diverge
// (C3 0.29 -> 0.59, C5 0.22 -> 0.41), but the FAST loop is bound by its
// per-lane node fetches (vector memory), not by VALU lane slots, so that buys
// little time: C5 +2.6 %, C3 -3 .. +1 %, and on the bunny, whose lockstep
// camera rays share cache lines, it costs a third.  Default:
// trees too large for the 16-bit stack (million-triangle meshes, C5).
bool use_wavefront(const zrt_ctx* c, bool stk16) {
  if (const char* e = std::getenv("ZRT_WF")) return std::atoi(e) != 0;
  (void)c;
  return !stk16;
}
// Per-axis margins (wide_iter) in waves with a lane whose max_k |1/d_k| exceeds
// this; ZRT_PAXIS_M overrides (the tests set 0: every wave takes them)
float paxis_threshold() {
  if (const char* e = std::getenv("ZRT_PAXIS_M")) return float(std::atof(e));
  return kPaxisM;
}
// The path-pool loop (render_loop_pool, MODE 5) instead of the wavefront loop?
// ZRT_POOL=0/1 forces it.  Default: the wavefront loop's cases (trees past the
// 16-bit stack), where it is 4 % faster at C5's full size (8.30 -> 8.65 Gray/s,
// profiles/r03/ab5); on the teapot (C3) and the bunny (C4) the lockstep loop
// stays ahead (14.7 vs 14.3, 50.5 vs 29.4 Gray/s).
bool use_pool(const zrt_ctx* c, bool stk16) {
  if (const char* e = std::getenv("ZRT_POOL")) return std::atoi(e) != 0;
  (void)c;
  return !stk16;
}
// Compressed wide nodes (wide_iter_q, MODE 8 / 9) for this tree?  ZRT_QNODES=1
// builds them (for trees of the path-pool loop's size, >= 65536 wide nodes, past the
// 16-bit stack, or any tree when forced); off by default: on the C5 mesh the pool
// over compressed nodes ran 7.17 Gray/s against 8.57 over the full nodes - each
// opened leaf's record is one more dependent fetch (DESIGN.md §3 "Compressed nodes")
bool want_qnodes(uint32_t n_wide) {
  if (const char* e = std::getenv("ZRT_QNODES")) return std::atoi(e) != 0;
  (void)n_wide;
  return ZRT_LOCK_QN != 0;  // (the A/B build's lockstep loop reads nothing else)
}
// Top levels of a compressed tree served from LDS (ZRT_QTOP overrides): every ray
// reads the root and a level-1 node, most a level-2 node - with 64-B nodes the
// third level (<= 21 nodes, 10.5 KiB of octant copies) fits beside the pool's queues
uint32_t qtop_levels() {
  if (const char* e = std::getenv("ZRT_QTOP")) return uint32_t(std::max(1, std::min(4, std::atoi(e))));
  return 3;
}
// The list loop with per-lane work items (render_loop_list, MODE 6) for scenes
// without a BVH; ZRT_LIST_LANES=0 forces the wave-unit loop (render_loop MODE 0).
// C2: 34.1 (MODE 0, lanes in per-sample lockstep) -> 45.4 (MODE 0, free lanes
// within a unit) -> MODE 6.
bool use_list_lanes() {
  if (const char* e = std::getenv("ZRT_LIST_LANES")) return std::atoi(e) != 0;
  return true;
}
// LDS of the path-pool loop's rays, hits and queues per block (render_loop_pool)
constexpr size_t kPoolLdsBytes = ((8 * sizeof(float) + 1) * kBlockPaths + 15) & ~size_t(15);

template <int MODE, int PRNG, bool STATS, class StackT>
void* kernel_ptr() {
  return reinterpret_cast<void*>(&render_kernel<MODE, PRNG, STATS, StackT>);
}

template <int PRNG, bool STATS>
void* select_kernel_ps(int mode, bool stk16) {
  if (mode == 0) return kernel_ptr<0, PRNG, STATS, uint16_t>();  // list mode: no stack
  if (mode == 6) return kernel_ptr<6, PRNG, STATS, uint16_t>();  // list mode, per-lane work items
  if (mode == 1) return stk16 ? kernel_ptr<1, PRNG, STATS, uint16_t>() : kernel_ptr<1, PRNG, STATS, uint32_t>();
  if (mode == 3) return stk16 ? kernel_ptr<3, PRNG, STATS, uint16_t>() : kernel_ptr<3, PRNG, STATS, uint32_t>();
  if (mode == 4) return stk16 ? kernel_ptr<4, PRNG, STATS, uint16_t>() : kernel_ptr<4, PRNG, STATS, uint32_t>();
  if (mode == 5) return stk16 ? kernel_ptr<5, PRNG, STATS, uint16_t>() : kernel_ptr<5, PRNG, STATS, uint32_t>();
  if (mode == 7) return stk16 ? kernel_ptr<7, PRNG, STATS, uint16_t>() : kernel_ptr<7, PRNG, STATS, uint32_t>();
  if (mode == 8) return stk16 ? kernel_ptr<8, PRNG, STATS, uint16_t>() : kernel_ptr<8, PRNG, STATS, uint32_t>();
  if (mode == 9) return stk16 ? kernel_ptr<9, PRNG, STATS, uint16_t>() : kernel_ptr<9, PRNG, STATS, uint32_t>();
  return stk16 ? kernel_ptr<2, PRNG, STATS, uint16_t>() : kernel_ptr<2, PRNG, STATS, uint32_t>();
}
#ifdef ZRT_ISA_KERNEL
// tools/isa.sh: device assembly of ONE render kernel (register / spill probes in
// seconds instead of minutes); ZRT_ISA_KERNEL = MODE, PRNG, STATS, StackT
void* select_kernel(int, uint32_t, bool, bool) { return kernel_ptr<ZRT_ISA_KERNEL>(); }
#else
void* select_kernel(int mode, uint32_t prng, bool stats, bool stk16) {
  if (prng == ZRT_PRNG_XOSHIRO256)
    return stats ? select_kernel_ps<ZRT_PRNG_XOSHIRO256, true>(mode, stk16)
                 : select_kernel_ps<ZRT_PRNG_XOSHIRO256, false>(mode, stk16);
  return stats ? select_kernel_ps<ZRT_PRNG_XOROSHIRO128, true>(mode, stk16)
               : select_kernel_ps<ZRT_PRNG_XOROSHIRO128, false>(mode, stk16);
}
#endif

template <int PRNG>
void* probe_ptr(bool stk16) {
#ifdef ZRT_ISA_KERNEL
  (void)stk16;
  return nullptr;
#else
  return stk16 ? reinterpret_cast<void*>(&schedule_probe_kernel<PRNG, uint16_t>)
               : reinterpret_cast<void*>(&schedule_probe_kernel<PRNG, uint32_t>);
#endif
}

// The block's dynamic LDS: [stack rows][lane] (StackT), then (FAST) the top
// wide nodes of every octant copy, then the first attenuation rows
// [row][rgb][lane] f32.  Sized so the waves per SIMD the kernel is built for
// (its __launch_bounds__) still fit: 160 KiB / that many blocks per CU.
struct LdsPlan {
  uint32_t stack_rows = 0, top_off = 0, att_off = 0, att_rows = 0, mat_off = 0, mats_in_lds = 0, pool_off = 0;
  uint32_t state_off = 0;
  size_t bytes = 0, budget = 0;
  size_t stack_b = 0, top_b = 0, pool_b = 0, state_b = 0, att_b = 0, mats_b = 0;  // region sizes (check_plan)
};
constexpr size_t kLdsPerBlockMax = 160u << 10;  // gfx950: a work-group may use the CU's whole LDS
// Every region of a plan inside the block's share and disjoint from the others,
// float4 regions 16-B aligned (the kernels index them from lds_raw by these
// offsets, nothing else keeps them apart); a violation is a bug in plan_lds.
void check_plan(const LdsPlan& L) {
  struct Reg { size_t off, n; const char* name; bool f4; };
  const Reg regs[] = {{0, L.stack_b, "stack", false}, {L.top_off, L.top_b, "top nodes", true},
                      {L.pool_off, L.pool_b, "pool", true}, {L.state_off, L.state_b, "lane state", false},
                      {L.att_off, L.att_b, "attenuation rows", false}, {L.mat_off, L.mats_b, "materials", true}};
  if (L.bytes > kLdsPerBlockMax)
    throw Error(ZRT_E_UNSUPPORTED, "LDS plan: " + std::to_string(L.bytes) + " B, past a block's " +
                                       std::to_string(kLdsPerBlockMax) + " B");
  for (const Reg& x : regs) {
    if (!x.n) continue;
    if (x.off + x.n > L.bytes)
      throw Error(ZRT_E_UNSUPPORTED, std::string("LDS plan: ") + x.name + " past the plan's end");
    if (x.f4 && x.off % 16)
      throw Error(ZRT_E_UNSUPPORTED, std::string("LDS plan: ") + x.name + " not 16-B aligned");
    for (const Reg& y : regs)
      if (&x != &y && y.n && x.off < y.off + y.n && y.off < x.off + x.n)
        throw Error(ZRT_E_UNSUPPORTED, std::string("LDS plan: ") + x.name + " overlaps " + y.name);
  }
}
// 32-bit words of the lockstep loop's lane state (LaneState)
uint32_t lane_state_words(uint32_t prng) {
  return (prng == ZRT_PRNG_XOSHIRO256 ? LaneState<ZRT_PRNG_XOSHIRO256>::kWords
                                      : LaneState<ZRT_PRNG_XOROSHIRO128>::kWords);
}
// pool: the path-pool loop (MODE 5): its attenuation rows are per path
// (kBlockPaths per block), and its rays / hits / queues follow them.
// The lockstep FAST loop (mode 3, neither wf nor pool) also holds its lane state
// (ZRT_LANE_LDS) and keeps at most ZRT_STACK_ROWS_LOCK stack rows in LDS.
LdsPlan plan_lds(uint32_t n_top, uint32_t n_mats, int mode, bool stk16, uint32_t stack_depth, uint32_t max_depth,
                 bool wf, bool pool, uint32_t prng, uint32_t node_f4 = 8) {
  const uint32_t waves = mode == 3 ? (pool ? ZRT_WAVES_POOL : wf ? ZRT_WAVES_WF : ZRT_WAVES_WIDE)
                         : mode == 0 ? ZRT_WAVES_LIST : ZRT_WAVES_PER_SIMD;
  // 256-thread blocks: `waves` blocks per CU; 1 KiB below the even share (a
  // block of exactly 32 KiB ran 8 % slower at 5 blocks per CU)
  const size_t budget = (160u << 10) / waves - (1u << 10);
  const size_t entry = stk16 ? sizeof(uint16_t) : sizeof(uint32_t);
  const size_t row_att = sizeof(uint32_t) * (pool ? kBlockPaths : kBlock);  // one att code per lane / path
  const size_t top = mode == 3 && ZRT_LDS_TOP ? size_t(n_top) * node_f4 * sizeof(float4) * kOctCopies : 0;
  const size_t pool_b = pool ? kPoolLdsBytes : 0;
  const bool lock = mode == 3 && !wf && !pool;
  const size_t state = lock && ZRT_LANE_LDS ? size_t(lane_state_words(prng)) * sizeof(uint32_t) * kBlock : 0;
  // attenuation rows wanted: rows 0 .. max_depth-2 are ever pushed (raytrace.zig:99 at depth > 1).
  // A row is one 4-B att code per lane (att_code; round 3: three floats, 12 B), so
  // the same LDS holds three times the rows: the lockstep loop 6 (round 3, 2 rows
  // of floats - C4 A/B: none 50.35, 1 row 50.57, 2 rows 50.70 Gray/s; a 32 KiB
  // block 46.5), the wavefront loop 12 (its 4 blocks per CU have a larger share;
  // the textured C5 mesh scatters often), the path pool 3 per path, the list loops
  // 24 (no stack, no tree in LDS; C2 at depth 30 with glass: round 3 2 -> 4 -> 8
  // rows of floats 32.7 -> 33.3 -> 34.0 Gray/s, profiles/r03/ab12)
  const uint32_t att_cap = pool ? ZRT_ATT_ROWS_POOL : wf ? ZRT_ATT_ROWS_WF : mode == 0 ? ZRT_ATT_ROWS_LIST : ZRT_ATT_ROWS_LOCK;
  uint32_t want = att_cap;
  if (const char* e = std::getenv("ZRT_ATT_LDS_ROWS")) want = uint32_t(std::atoi(e));
  want = std::min<uint32_t>(want, max_depth > 1 ? max_depth - 1 : 0);
  LdsPlan L;
  L.budget = budget;
  if (mode == 3) {
    // the stack takes what the top nodes, the lane state and the wanted attenuation
    // rows leave (the lockstep loop: at most ZRT_STACK_ROWS_LOCK rows; it wants
    // ZRT_ATT_ROWS_LOCK att rows); deeper rows live in global memory (wide_iter and
    // wide_iter_q read them at either stack width, so no FAST plan holds a stack
    // the block's LDS cannot)
    want = std::min<uint32_t>(want, att_cap);
    const size_t fixed = top + pool_b + state + want * row_att;
    const size_t room = budget > fixed ? budget - fixed : 0;
    L.stack_rows = std::max<uint32_t>(1, std::min<uint32_t>(stack_depth, uint32_t(room / (kBlock * entry))));
    if (lock) L.stack_rows = std::min<uint32_t>(L.stack_rows, ZRT_STACK_ROWS_LOCK);
  } else {
    L.stack_rows = stack_depth;  // BINARY / REFERENCE: the whole stack in LDS (check_plan: within a block's LDS)
  }
  if (const char* f = std::getenv("ZRT_STACK_LDS_ROWS"))  // tests: force the overflow rows into use
    if (mode == 3) L.stack_rows = std::max<uint32_t>(1, std::min<uint32_t>(L.stack_rows, uint32_t(std::atoi(f))));
  const size_t stack = (size_t(L.stack_rows) * kBlock * entry + 15) & ~size_t(15);
  const size_t used = stack + top + pool_b + state;
  // loops that read the material table from LDS only (ZRT_MATS_LDS_ONLY): the table
  // before the attenuation rows, which live in global memory when LDS runs out
  const size_t mats = size_t(n_mats) * sizeof(DevMaterial);
  const bool mats_first = ZRT_MATS_LDS_ONLY && (lock || mode == 0);
  const size_t mats_res = mats_first && used + mats <= budget ? mats : 0;
  L.att_rows = std::min<uint32_t>(want, used + mats_res < budget ? uint32_t((budget - used - mats_res) / row_att) : 0u);
  L.top_off = uint32_t(stack);
  L.pool_off = uint32_t(stack + top);
  L.state_off = uint32_t(stack + top + pool_b);
  L.att_off = uint32_t(used);
  L.bytes = used + L.att_rows * row_att;
  L.stack_b = size_t(L.stack_rows) * kBlock * entry;
  L.top_b = top;
  L.pool_b = pool_b;
  L.state_b = state;
  L.att_b = L.att_rows * row_att;
  // the material table, if it fits what is left (ZRT_MATS_LDS=0: A/B, always global,
  // for the loops that can read it there)
  const char* me = std::getenv("ZRT_MATS_LDS");
  if (mats > 0 && L.bytes + mats <= budget && (mats_first || !(me && std::atoi(me) == 0))) {
    L.mat_off = uint32_t(L.bytes);
    L.mats_in_lds = 1;
    L.bytes += mats;
    L.mats_b = mats;
  }
  // the lockstep FAST kernel's waves per SIMD hold only within the share (the
  // other loops' plans may exceed it: their launch then fits fewer blocks per CU)
  if (lock && L.bytes > budget) throw Error(ZRT_E_UNSUPPORTED, "LDS plan: the lockstep loop's regions exceed its share");
  check_plan(L);
  return L;
}
LdsPlan plan_lds(const zrt_ctx* c, int mode, bool stk16, uint32_t stack_depth, uint32_t max_depth, bool wf, bool pool,
                 uint32_t prng, uint32_t node_f4 = 8) {
  return plan_lds(node_f4 == kQuantNodeF4 ? c->q_top : c->n_top, c->n_mats, mode, stk16, stack_depth, max_depth, wf,
                  pool, prng, node_f4);
}

// The context's global buffers that the launches of a frame share (the render
// launch and its scheduling probe) and that later frames reuse: attenuation rows
// past the plan's LDS rows ([row][lane], the path pool [row][path]: elements of
// c->att) and FAST stack rows past the plan's LDS rows ([row][lane]: bytes of
// c->stack_ovf).  A launch's need follows from its own plan; every launch is
// checked against the allocation before it is enqueued (check_buffers), so a
// sizing mistake - round 5's scheduling probe kept 4 LDS attenuation rows where
// the wavefront render it shared the buffer with kept 12 - is refused as
// ZRT_E_UNSUPPORTED on the host instead of faulting on the GPU.
struct BufNeed {
  uint64_t att_elems = 0;  // u32 attenuation codes
  uint64_t ovf_bytes = 0;  // stack entries (StackT) past the LDS rows
};
BufNeed buffer_need(const LdsPlan& lp, uint32_t max_depth, uint32_t stack_depth, uint64_t n_paths, uint64_t n_lanes,
                    bool stk16) {
  BufNeed n;
  n.att_elems = std::max<uint64_t>(1, max_depth - std::min(max_depth, lp.att_rows)) * n_paths;
  if (stack_depth > lp.stack_rows)
    n.ovf_bytes = uint64_t(stack_depth - lp.stack_rows) * n_lanes * (stk16 ? sizeof(uint16_t) : sizeof(uint32_t));
  return n;
}
void check_buffers(const char* launch, const BufNeed& need, uint64_t att_elems, uint64_t ovf_bytes) {
  if (need.att_elems > att_elems)
    throw Error(ZRT_E_UNSUPPORTED, std::string(launch) + ": needs " + std::to_string(need.att_elems) +
                                       " global attenuation-row entries, the context holds " + std::to_string(att_elems));
  if (need.ovf_bytes > ovf_bytes)
    throw Error(ZRT_E_UNSUPPORTED, std::string(launch) + ": needs " + std::to_string(need.ovf_bytes) +
                                       " B of global stack rows, the context holds " + std::to_string(ovf_bytes));
}
// The device side of the same check (KArgs::att_cap / ovf_cap: the allocations'
// elements), in the STATS flavour: a row index past its buffer sets kErrBounds and
// the access is skipped (tests/test_gpu_runtime.py shrinks the capacity it is told)
uint64_t ovf_cap_elems(uint64_t ovf_bytes, bool stk16) { return ovf_bytes / (stk16 ? 2u : 4u); }

// Longest-processing-time-first order of this rank's tiles (zrt.h,
// ZRT_FLAG_NO_SCHEDULE): the probe renders kProbeSpp samples of every tile as
// one unit each and records the loop iterations its wave spent (lockstep makes
// that the unit's time); a stable device radix sort orders the tiles by
// descending cost, ties in tile order.  Sets a.tile_order for the render launch.
bool schedule_tiles(zrt_ctx* c, KArgs& a, uint32_t prng, bool stk16, uint32_t my_tiles, uint32_t grid,
                    size_t lds, hipStream_t st) {
  constexpr uint32_t kProbeSpp = ZRT_PROBE_SPP;
  KArgs pa = a;
  pa.spp = kProbeSpp;
  pa.chunk = kProbeSpp;
  pa.n_chunks = 1;
  pa.total_work = my_tiles;
  if (c->probe_partial.n < uint64_t(my_tiles) * 64u) c->probe_partial.alloc(uint64_t(my_tiles) * 64u);
  if (c->probe_scratch.n < uint64_t(kScratchSlots)) c->probe_scratch.alloc(kScratchSlots);
  if (c->tile_cost.n < my_tiles) {
    c->tile_cost.alloc(my_tiles);
    c->cost_sorted.alloc(my_tiles);
    c->tile_order.alloc(my_tiles);
  }
  if (c->tile_ids_n != my_tiles) {
    std::vector<uint32_t> ids(my_tiles);
    for (uint32_t i = 0; i < my_tiles; ++i) ids[i] = i;
    c->tile_ids.upload(ids);
    c->tile_ids_n = my_tiles;
  }
  pa.partial = c->probe_partial.p;
  pa.counters = c->probe_scratch.p;
  pa.work_counter = reinterpret_cast<uint32_t*>(c->probe_scratch.p + kWorkSlot);
  // pa.error_flag stays the render launch's: a probe overflow fails the frame too
  pa.unit_cost = c->tile_cost.p;
  pa.tile_order = nullptr;
  const uint32_t pgrid = std::max(1u, std::min(grid, (my_tiles + kBlock / 64 - 1) / (kBlock / 64)));
  pa.n_lanes = pgrid * kBlock;
  // the probe is the lockstep loop over the full nodes, whatever loop and node
  // format the render launch uses: its own LDS plan (the render's may be the path
  // pool's, whose regions the lockstep loop would read as its lane state and rows)
  const LdsPlan pp = plan_lds(c, 3, stk16, a.stack_depth, a.max_depth, false, false, prng, 8);
  pa.wnodes = c->wnodes.p;
  pa.wide_stride = c->wide_stride;
  pa.node_f4 = 8;
  pa.n_top = c->n_top;  // (the full nodes' top levels: a compressed tree keeps more in LDS)
  pa.qleaves = nullptr;
  pa.n_qnodes = pa.n_qleaves = 0;
  pa.lds_rows = pp.stack_rows;
  pa.lds_top_off = pp.top_off;
  pa.lds_att_off = pp.att_off;
  pa.att_lds_rows = pp.att_rows;
  pa.lds_mat_off = pp.mat_off;
  pa.mats_in_lds = pp.mats_in_lds;
  // (the probe is the lockstep loop, which reads the table from LDS only: no schedule
  // for a table past its LDS share - the render then takes the tiles in order)
  if (ZRT_MATS_LDS_ONLY && !pp.mats_in_lds) return false;
  pa.lds_pool_off = pp.pool_off;
  pa.lds_state_off = pp.state_off;
  lds = pp.bytes;
  // its deep stack rows and global attenuation rows ([row][lane] past its LDS rows):
  // the render launch's buffers, grown if the probe's plan needs more (the wavefront
  // loop keeps 12 attenuation rows in LDS, the lockstep probe 4)
  const BufNeed need = buffer_need(pp, a.max_depth, a.stack_depth, pa.n_lanes, pa.n_lanes, stk16);
  if (need.ovf_bytes) {
    if (c->stack_ovf.n < need.ovf_bytes) {
      HIPCHK(hipStreamSynchronize(st));  // (the previous launch may still read the old buffer)
      c->stack_ovf.alloc(need.ovf_bytes);
    }
    a.stack_ovf = pa.stack_ovf = c->stack_ovf.p;
  }
  if (c->att.n < need.att_elems) {
    HIPCHK(hipStreamSynchronize(st));  // (the previous launch may still read the old buffer)
    c->att.alloc(need.att_elems);
  }
  a.att = pa.att = c->att.p;
  a.att_cap = pa.att_cap = c->att.n;
  a.ovf_cap = pa.ovf_cap = ovf_cap_elems(c->stack_ovf.n, stk16);
  check_buffers("scheduling probe", need, c->att.n, c->stack_ovf.n);
  HIPCHK(hipMemsetAsync(c->probe_scratch.p, 0, kScratchSlots * sizeof(unsigned long long), st));
  void* fn = prng == ZRT_PRNG_XOSHIRO256 ? probe_ptr<ZRT_PRNG_XOSHIRO256>(stk16)
                                         : probe_ptr<ZRT_PRNG_XOROSHIRO128>(stk16);
  void* args[] = {&pa};
  HIPCHK(hipLaunchKernel(fn, dim3(pgrid), dim3(kBlock), args, lds, st));
  size_t bytes = 0;
  HIPCHK(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, bytes, c->tile_cost.p, c->cost_sorted.p,
                                                      c->tile_ids.p, c->tile_order.p, int(my_tiles), 0, 32, st));
  if (c->sort_temp.n < bytes) c->sort_temp.alloc(bytes);
  HIPCHK(hipcub::DeviceRadixSort::SortPairsDescending(c->sort_temp.p, bytes, c->tile_cost.p, c->cost_sorted.p,
                                                      c->tile_ids.p, c->tile_order.p, int(my_tiles), 0, 32, st));
  a.tile_order = c->tile_order.p;
  return true;
}

int hip_fail(const HipError& e) {
  return fail(ZRT_E_HIP, e.where + ": " + hipGetErrorString(e.err));
}

// The catch clauses of every C entry point: no exception crosses the ABI.
#define ZRT_CATCH_ALL                                  \
  catch (const ::zrt::HipError& e) {                   \
    return ::zrt::hip_fail(e);                         \
  }                                                    \
  catch (const ::zrt::Error& e) {                      \
    return ::zrt::fail(e.code, e.what());              \
  }                                                    \
  catch (const std::bad_alloc&) {                      \
    return ::zrt::fail(ZRT_E_NOMEM, "OutOfMemory");    \
  }

constexpr const char* kOverflowMsg = "BVH traversal stack overflow (tree deeper than the stack was sized for)";
constexpr const char* kLayoutMsg = "the kernel refused the wide tree: its layout is not the one the kernel decodes";
constexpr const char* kBoundsMsg = "a global attenuation or stack row index past its buffer (STATS bounds check)";
const char* device_error_msg(unsigned long long flag) {
  return (flag & kErrLayout) ? kLayoutMsg : (flag & kErrBounds) ? kBoundsMsg : kOverflowMsg;
}

// The device error flag of the context's last launch, copied to pinned host
// memory behind ev_done.  wait: block until the launch is done and report its
// error (every such call does); else (render_tiles' sticky check) report it only
// if the launch has finished and no call has reported it yet.
int launch_status(zrt_ctx* c, bool wait) {
  if (!c->launched) return ZRT_OK;
  if (wait) {
    HIPCHK(hipEventSynchronize(c->ev_done));
  } else if (hipEventQuery(c->ev_done) != hipSuccess || c->err_reported) {
    return ZRT_OK;
  }
  if (*c->err_host == 0) return ZRT_OK;
  c->err_reported = true;
  return fail(ZRT_E_UNSUPPORTED, device_error_msg(*c->err_host));
}

// RCCL for zrt_render_multi, opened on first use so that single-GPU callers do
// not load it: the copy already in the process when torch brought one (same
// soname, librccl.so.1), else ROCm's.
struct Rccl {
  decltype(&ncclCommInitAll) comm_init_all = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclGather) gather = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
};
const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    r.comm_init_all = reinterpret_cast<decltype(r.comm_init_all)>(dlsym(h, "ncclCommInitAll"));
    r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
    r.gather = reinterpret_cast<decltype(r.gather)>(dlsym(h, "ncclGather"));
    r.group_start = reinterpret_cast<decltype(r.group_start)>(dlsym(h, "ncclGroupStart"));
    r.group_end = reinterpret_cast<decltype(r.group_end)>(dlsym(h, "ncclGroupEnd"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(h, "ncclGetErrorString"));
  });
  if (!r.comm_init_all || !r.comm_destroy || !r.gather || !r.group_start || !r.group_end || !r.error_string)
    throw Error(ZRT_E_UNSUPPORTED, "RCCL (librccl.so.1 with ncclGather) is not available");
  return r;
}

#define NCCLCHK(R, expr)                                                                     \
  do {                                                                                       \
    const ncclResult_t r_ = (expr);                                                          \
    if (r_ != ncclSuccess) throw ::zrt::Error(ZRT_E_HIP, std::string("RCCL ") + #expr + ": " + (R).error_string(r_)); \
  } while (0)

// A context on `device` holding an uploaded copy of a flattened scene.
std::unique_ptr<zrt_ctx> ctx_on_device(const HostScene& h, int device) {
  std::unique_ptr<zrt_ctx> c(new zrt_ctx);
  c->device = device;
  HIPCHK(hipSetDevice(c->device));
  // a blocking stream: work a caller enqueues on the legacy default stream (NULL,
  // e.g. torch's default stream) after a render on this one waits for it
  HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamDefault));
  HIPCHK(hipEventCreate(&c->ev_pre));
  HIPCHK(hipEventCreate(&c->ev0));
  HIPCHK(hipEventCreate(&c->ev1));
  HIPCHK(hipEventCreateWithFlags(&c->ev_done, hipEventDisableTiming));
  HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&c->err_host), sizeof(unsigned long long), hipHostMallocDefault));
  *c->err_host = 0;
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, c->device));
  c->cu_count = prop.multiProcessorCount;
  upload_scene(c.get(), h);
  c->scratch.alloc(kScratchSlots);
  return c;
}

// ncclCommInitAll communicators, one per device, destroyed with the call.
struct Comms {
  const Rccl* R = nullptr;
  std::vector<ncclComm_t> c;
  ~Comms() {
    for (ncclComm_t x : c)
      if (x) (void)R->comm_destroy(x);
  }
};

struct CtxDeleter {
  void operator()(zrt_ctx* c) const { zrt_ctx_destroy(c); }
};

}  // namespace
}  // namespace zrt

// One rank per entry of `devices`: its context (scene copy in that GPU's HBM),
// its padded tile buffer, and - one rank per distinct device - the RCCL
// communicators, all kept across frames.  Members are destroyed in reverse
// order: the communicators go before the contexts.
struct zrt_multi {
  std::vector<uint32_t> devices;
  uint32_t n_distinct = 0;
  bool use_rccl = false;
  std::vector<std::unique_ptr<zrt_ctx, zrt::CtxDeleter>> ctx;
  std::vector<zrt::DevBuf<float>> send;
  zrt::DevBuf<float> gathered, frame;  // on devices[0]
  size_t frame_n = 0;                  // floats of the last frame in `frame` (0: none rendered yet)
  std::vector<double> rank_ms;         // the last frame: each rank's render-kernel time (HIP events)
  zrt::Comms comms;
};

namespace zrt {
namespace {
int assemble(zrt_ctx* c, const zrt_params* p, const float* dev_gathered, uint32_t stride_tiles, float* dev_frame,
             void* hip_stream) {
  if (!c || !dev_gathered || !dev_frame) return fail(ZRT_E_INVALID, "null argument");
  const int rc = validate_params(p);
  if (rc) return rc;
  try {
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
    const Geometry g = geometry(p);
    uint32_t total = 0;
    if (stride_tiles) {
      for (uint32_t r = 0; r < p->world_size; ++r)
        if (rank_tiles(g, r, p->world_size) > stride_tiles)
          return fail(ZRT_E_INVALID, "stride_tiles is smaller than a rank's tile count");
      if (uint64_t(stride_tiles) * 64u * p->world_size >= (1ull << 32)) return fail(ZRT_E_UNSUPPORTED, "frame too large");
      total = stride_tiles * 64u * p->world_size;
    } else {
      std::vector<uint32_t> base(p->world_size + 1, 0);
      for (uint32_t r = 0; r < p->world_size; ++r) base[r + 1] = base[r] + rank_tiles(g, r, p->world_size) * 64u;
      c->rank_base.upload(base);
      total = base[p->world_size];
    }
    HIPCHK(hipMemsetAsync(dev_frame, 0, sizeof(float) * 3 * size_t(p->width) * p->height, st));
    if (total) {
      hipLaunchKernelGGL(assemble_kernel, dim3((total + 255) / 256), dim3(256), 0, st, dev_gathered, dev_frame,
                         stride_tiles ? nullptr : c->rank_base.p, p->world_size, g.tiles_x, g.xbound, p->height,
                         p->width, total, stride_tiles * 64u, g.n_tiles);
      HIPCHK(hipGetLastError());
    }
    return ZRT_OK;
  }
  ZRT_CATCH_ALL
}
}  // namespace
}  // namespace zrt

using zrt::fail;

extern "C" {

int zrt_abi_version(void) { return ZRT_ABI_VERSION; }

const char* zrt_build_info(void) {
  return "libzrt: HIP path for gfx950 (MI355X); persistent wave64 path-tracing kernel; -ffp-contract=off";
}

int zrt_ctx_create(const zrt_scene* scene, const zrt_params* params, zrt_ctx** out) {
  if (!out) return fail(ZRT_E_INVALID, "out is null");
  *out = nullptr;
  int rc = zrt::validate_scene(scene);
  if (rc) return rc;
  if (!params) return fail(ZRT_E_INVALID, "params is null");
  try {
    // raytrace.zig:124-133: BVH iff requested and more than 10 surfaces.  The
    // scene is flattened before the device is checked, so a tree whose layout
    // the kernels do not decode is refused on any machine (flatten_scene); the
    // GPU builds the reference BVH only when one is visible
    const bool use_bvh = params->bounded_volume_hierarchy != 0 && scene->n_prims > 10;
    int n_dev = 0;
    const bool gpus = hipGetDeviceCount(&n_dev) == hipSuccess && n_dev > 0;
    // with GPUs present, an unusable device is refused before the (seconds-long on a
    // million-triangle mesh) scene build; without any, the layout check still runs first
    if (gpus) {
      rc = zrt::check_device(int(params->device));
      if (rc) return rc;
    }
    const bool have_dev = gpus && int(params->device) < n_dev;
    zrt::HostScene h;
    zrt::flatten_scene(&h, scene, use_bvh, have_dev ? int(params->device) : -1);
    rc = zrt::check_device(int(params->device));
    if (rc) return rc;
    *out = zrt::ctx_on_device(h, int(params->device)).release();
    return ZRT_OK;
  } catch (const zrt::HipError& e) {
    return zrt::hip_fail(e);
  } catch (const zrt::Error& e) {
    return fail(e.code, e.what());
  } catch (const std::bad_alloc&) {
    return fail(ZRT_E_NOMEM, "OutOfMemory");
  }
}

int zrt_ctx_destroy(zrt_ctx* ctx) {
  if (!ctx) return ZRT_OK;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  delete ctx;
  return ZRT_OK;
}

int zrt_ctx_tile_count(const zrt_ctx* ctx, const zrt_params* params, uint32_t* n_tiles) {
  (void)ctx;  // the partition depends on the params only; ctx may be NULL
  if (!n_tiles) return fail(ZRT_E_INVALID, "null argument");
  const int rc = zrt::validate_params(params);
  if (rc) return rc;
  *n_tiles = zrt::rank_tiles(zrt::geometry(params), params->rank, params->world_size);
  return ZRT_OK;
}

int zrt_ctx_render_tiles(zrt_ctx* c, const zrt_camera* cam, const zrt_params* p, float* dev_tiles,
                         void* hip_stream) {
  if (!c || !cam || !dev_tiles) return fail(ZRT_E_INVALID, "null argument");
  int rc = zrt::validate_params(p);
  if (rc) return rc;
  if (int(p->device) != c->device)
    return fail(ZRT_E_INVALID, "params->device differs from the device the context was created on");
  if ((p->bounded_volume_hierarchy != 0 && c->n_prims > 10) != c->use_bvh)
    return fail(ZRT_E_INVALID,
                "params->bounded_volume_hierarchy implies another preprocessSufraces decision (raytrace.zig:124-133) "
                "than the one the context was built with");
  try {
    HIPCHK(hipSetDevice(c->device));
    // a device error of the previous launch that finished meanwhile is reported
    // here (sticky), so a caller that never synchronises through the ABI still sees it
    rc = zrt::launch_status(c, false);
    if (rc) return rc;
    hipStream_t st = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
    const zrt::Geometry g = zrt::geometry(p);
    const uint32_t my_tiles = zrt::rank_tiles(g, p->rank, p->world_size);
    const int mode = !c->use_bvh ? 0
                     : p->traversal == ZRT_TRAVERSAL_REFERENCE ? 2
                     : p->traversal == ZRT_TRAVERSAL_BINARY ? 1 : 3;
    const bool diag = (p->flags & ZRT_FLAG_STATS) != 0;
    // FAST: a 16-bit stack when node indices fit (either flavour keeps its first
    // rows in LDS and deeper ones in global memory, zrt::plan_lds)
    const char* force_rows = std::getenv("ZRT_STACK_LDS_ROWS");  // tests: force the overflow rows into use
    // (FAST also holds the reference traversal's rows for its order-hazard replay)
    uint32_t stack_depth = mode == 3 ? std::max(c->wide_stack, c->stack_depth) : c->stack_depth;
    if (const char* cap = std::getenv("ZRT_DEBUG_STACK_CAP"))  // tests: a stack too small for the tree
      stack_depth = std::max<uint32_t>(4, std::min<uint32_t>(stack_depth, uint32_t(std::atoi(cap))));
    bool stk16 = mode == 3 ? c->n_wide < 65536 && c->n_nodes < 65536 && !force_rows : c->n_nodes < 65536;
    // FAST: the wavefront loop (MODE 4) where lanes' traversal lengths diverge
    bool wf = mode == 3 && p->max_depth >= 1 && zrt::use_wavefront(c, stk16);
    // the path-pool loop (MODE 5) for the same cases, when asked for; a 16-bit stack
    // must fit beside its rays and queues in the block's LDS share, else the 32-bit
    // stack with overflow rows
    // the grazing-triangle guard (ZRT_FLAG_GUARD): carried by the path-pool loop's traversal
    const bool guard_on = mode == 3 && (p->flags & ZRT_FLAG_GUARD) != 0 && c->guard > 0.0f;
    const bool pool = mode == 3 && p->max_depth >= 1 && (zrt::use_pool(c, stk16) || guard_on);
    // the path pool over compressed nodes (MODE 8 / 9) where the context built them (and
    // the lockstep loop in the ZRT_LOCK_QN A/B build, which has no other traversal)
    const bool lock_qn = ZRT_LOCK_QN && mode == 3 && !pool && !wf;
    if (lock_qn && !c->q_ok) return fail(ZRT_E_UNSUPPORTED, "ZRT_LOCK_QN build: no compressed nodes for this tree");
    const bool qn = (pool || lock_qn) && c->q_ok;
    const uint32_t node_f4 = qn ? zrt::kQuantNodeF4 : 8u;
    if (pool && stk16) {
      const size_t budget = (160u << 10) / ZRT_WAVES_POOL - (1u << 10);
      const size_t top = ZRT_LDS_TOP ? size_t(qn ? c->q_top : c->n_top) * node_f4 * sizeof(float4) * zrt::kOctCopies : 0;
      if (size_t(stack_depth) * zrt::kBlock * sizeof(uint16_t) + top + zrt::kPoolLdsBytes > budget) stk16 = false;
    }
    const bool list_lanes = mode == 0 && zrt::use_list_lanes();
    // (the guard's branch costs the path pool 0.7 % on C5, so a guarded render has a
    // kernel of its own, MODE 7; profiles/r04/r04n)
    int kmode = pool ? (qn ? (guard_on ? 9 : 8) : (guard_on ? 7 : 5)) : wf ? 4 : list_lanes ? 6 : mode;
    // FAST: deep trees keep their last stack rows in global memory (rarely
    // touched) so the LDS never caps the occupancy the registers allow; the
    // other traversals keep the whole stack in LDS (zrt::plan_lds)
    zrt::LdsPlan lp = zrt::plan_lds(c, mode, stk16, stack_depth, p->max_depth, wf, pool, p->prng, node_f4);
    if (ZRT_MATS_LDS_ONLY && (kmode == 3 || kmode == 6) && !lp.mats_in_lds) {
      // a material table past the loop's LDS share: the loop that reads it from global
      // memory (the wavefront loop for FAST, the wave-unit list loop; same images)
      if (kmode == 6) {
        kmode = 0;
      } else {
        wf = true;
        kmode = 4;
      }
      lp = zrt::plan_lds(c, mode, stk16, stack_depth, p->max_depth, wf, pool, p->prng, node_f4);
    }
    void* kfn = zrt::select_kernel(kmode, p->prng, diag, stk16);
    const uint32_t lds_rows = lp.stack_rows;
    const size_t lds = lp.bytes;
    int per_cu = 0;
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, zrt::kBlock, lds));
    per_cu = std::max(1, std::min(per_cu, 8));
    uint32_t grid = uint32_t(c->cu_count) * uint32_t(per_cu);
    const uint32_t chunk = p->sample_chunk ? p->sample_chunk : ZRT_DEFAULT_SAMPLE_CHUNK;
    const uint32_t n_chunks = (p->samples_per_pixel + chunk - 1) / chunk;
    const uint64_t work64 = uint64_t(my_tiles) * n_chunks;  // units: (tile, chunk)
    if (uint64_t(my_tiles) * 64u * n_chunks >= (1ull << 32) - (1ull << 26))  // (+ one refill per lane of slack)
      return fail(ZRT_E_UNSUPPORTED, "more than 2^32 (pixel, chunk) work items");
    const uint32_t work = uint32_t(work64);
    // one wave per unit at the start; more waves than units would only idle
    grid = std::max(1u, std::min(grid, (work + (zrt::kBlock / 64) - 1) / (zrt::kBlock / 64)));
    const uint64_t n_partial = uint64_t(my_tiles) * 64u * n_chunks;
    if (c->partial.n < n_partial) c->partial.alloc(n_partial);
    const uint64_t n_lanes = uint64_t(grid) * zrt::kBlock;
    // global attenuation rows: [row][lane], or [path][row] for the path-pool loop
    const uint64_t n_paths = pool ? uint64_t(grid) * zrt::kBlockPaths : n_lanes;
    if (n_paths >= (1ull << 32)) return fail(ZRT_E_UNSUPPORTED, "too many paths");
    const zrt::BufNeed need = zrt::buffer_need(lp, p->max_depth, stack_depth, n_paths, n_lanes, stk16);
    if (need.att_elems * sizeof(uint32_t) > (16ull << 30))
      return fail(ZRT_E_UNSUPPORTED, "max_depth too large for the per-lane attenuation stack");
    if (c->att.n < need.att_elems) c->att.alloc(need.att_elems);
    HIPCHK(hipMemsetAsync(c->scratch.p, 0, zrt::kScratchSlots * sizeof(unsigned long long), st));

    zrt::KArgs a{};
    a.nodes = c->nodes.p;
    a.prims = c->prims.p;
    a.shade = c->shade.p;
    a.mats = c->mats.p;
    a.texels = c->texels.p;
    a.texels8 = c->texels8.p;
    a.att = c->att.p;
    a.partial = c->partial.p;
    a.counters = c->scratch.p;
    a.work_counter = reinterpret_cast<uint32_t*>(c->scratch.p + zrt::kWorkSlot);
    a.error_flag = reinterpret_cast<uint32_t*>(c->scratch.p + zrt::kErrorSlot);
    const zrt_vec3* v[4] = {&cam->origin, &cam->lower_left_corner, &cam->horizontal, &cam->vertical};
    float* dst[4] = {a.org, a.llc, a.hor, a.ver};
    for (int k = 0; k < 4; ++k) {
      dst[k][0] = v[k]->x;
      dst[k][1] = v[k]->y;
      dst[k][2] = v[k]->z;
    }
    a.f_width = float(p->width);
    a.f_height = float(p->height);
    a.inv_width = 1.0f / a.f_width;  // IEEE RN(1/width): dev::div_core's y
    a.inv_height = 1.0f / a.f_height;
    a.color_scale = 1.0f / float(p->samples_per_pixel);  // raytrace.zig:157
    a.width = p->width;
    a.height = p->height;
    a.xbound = g.xbound;
    a.spp = p->samples_per_pixel;
    a.max_depth = p->max_depth;
    a.tiles_x = g.tiles_x;
    a.rank = p->rank;
    a.world = p->world_size;
    a.total_work = work;
    a.n_list = c->use_bvh ? 0 : c->n_prims;
    a.tri_rcp_fast = c->tri_rcp_fast;
    a.scene_extent = c->scene_extent;
    a.paxis_m = zrt::paxis_threshold();
    for (int k = 0; k < 3; ++k) {
      a.tri_c[k] = c->tri_c[k];
      a.tri_h[k] = c->tri_h[k];
    }
    a.stack_depth = stack_depth;
    a.ref_stack = std::min(c->stack_depth, stack_depth);
    a.leaf_of_slot = c->leaf_of_slot.p;
    a.ref_sph = c->ref_sph.p;
    for (int k = 0; k < 3; ++k) a.root_c[k] = c->root_c[k];
    a.origin_bound = c->origin_bound;
    a.layout = c->layout;
    a.graze_m = c->graze_m;
    a.graze_leaf = c->graze_leaf;
    a.guard = guard_on ? c->guard : 0.0f;
    {  // the camera inside the bound: so is every ray of the launch (scattered rays start at hits)
      const float m = std::max({std::fabs(a.org[0] - a.root_c[0]), std::fabs(a.org[1] - a.root_c[1]),
                                std::fabs(a.org[2] - a.root_c[2])});
      a.check_origins = m <= a.origin_bound ? 0u : 1u;
    }
    a.wnodes = qn ? c->qnodes.p : c->wnodes.p;
    a.wide_stride = qn ? c->q_stride : c->wide_stride;
    a.node_f4 = node_f4;
    a.qleaves = qn ? c->qleaves.p : nullptr;
    a.n_qnodes = qn ? c->q_stride / zrt::kQuantNodeF4 : 0u;
    a.n_qleaves = qn ? c->n_qleaves : 0u;
    a.lds_rows = lds_rows;
    if (need.ovf_bytes) {
      if (c->stack_ovf.n < need.ovf_bytes) c->stack_ovf.alloc(need.ovf_bytes);
      a.stack_ovf = c->stack_ovf.p;
    }
    a.n_lanes = uint32_t(n_lanes);
    a.n_top = qn ? c->q_top : c->n_top;
    a.lds_top_off = lp.top_off;
    a.lds_att_off = lp.att_off;
    a.att_lds_rows = lp.att_rows;
    a.lds_mat_off = lp.mat_off;
    a.lds_pool_off = lp.pool_off;
    a.lds_state_off = lp.state_off;
    a.n_paths = uint32_t(n_paths);
    a.n_mats = c->n_mats;
    a.mats_in_lds = lp.mats_in_lds;
    a.seed_mix = p->seed * 0x9E3779B97F4A7C15ULL;
    if (std::getenv("ZRT_DEBUG_LAUNCH"))
      std::fprintf(stderr, "zrt launch: mode %d stk16 %d grid %u (%d blocks/CU x %d CUs) lds %zu B "
                   "(stack rows %u, top nodes %u @%u, att rows %u @%u, mats %u @%u)\n", mode, int(stk16), grid,
                   per_cu, c->cu_count, lds, lp.stack_rows, a.n_top, lp.top_off, lp.att_rows, lp.att_off,
                   lp.mats_in_lds ? c->n_mats : 0u, lp.mat_off);
    a.chunk = chunk;
    a.n_chunks = n_chunks;
    a.wf_thresh = 48;  // shade once 3/4 of the unit's active lanes are ready (C5: 32 -> 7.32, 48 -> 7.71, 56 -> 7.70 Gray/s)
    if (const char* e = std::getenv("ZRT_WF_THRESH")) a.wf_thresh = std::max(1, std::min(64, std::atoi(e)));
    // the lockstep interval: the BVH loops keep a wave's lanes on one sample (its
    // camera rays coherent); the list loop gains nothing from that (every ray reads
    // the same surfaces) and lets its lanes run through the unit's chunk
    // (C2: 34.1 -> 45.4 Gray/s, profiles/r04/s1)
    a.sync = mode == 0 ? chunk : ZRT_SYNC_SAMPLES;
    if (const char* e = std::getenv("ZRT_SYNC"))  // A/B: lockstep interval in samples (identical images)
      a.sync = std::max(1u, uint32_t(std::atoi(e)));
    a.n_slots = my_tiles * 64u;

    HIPCHK(hipEventRecord(c->ev_pre, st));
    bool schedule =
        mode == 3 && !(p->flags & ZRT_FLAG_NO_SCHEDULE) && p->samples_per_pixel >= 128 && my_tiles >= 2;
    if (schedule) schedule = zrt::schedule_tiles(c, a, p->prng, stk16, my_tiles, grid, lds, st);
    c->scheduled = schedule;
    // the lockstep loop takes its interval from the probe's lane efficiency (auto_sync;
    // ZRT_SYNC or ZRT_AUTO_SYNC=0: the fixed interval, A/B)
    {
      const char* as = std::getenv("ZRT_AUTO_SYNC");
      const bool auto_on = !std::getenv("ZRT_SYNC") && !(as && std::atoi(as) == 0);
      a.sync_probe = schedule && kmode == 3 && auto_on ? c->probe_scratch.p : nullptr;
    }
    c->scanline_rows = 0;
    if (p->flags & ZRT_FLAG_SCANLINES) {  // (not the probe's: set after it)
      if (c->scanlines.n < size_t(p->height) * 3) c->scanlines.alloc(size_t(p->height) * 3);
      HIPCHK(hipMemsetAsync(c->scanlines.p, 0, size_t(p->height) * 3 * sizeof(unsigned long long), st));
      a.scanlines = c->scanlines.p;
      c->scanline_rows = p->height;
    }
    if (ZRT_PROFILE) {
      c->n_waves = grid * (zrt::kBlock / 64);
      if (c->wave_times.n < 2ull * c->n_waves) c->wave_times.alloc(2ull * c->n_waves);
      a.wave_times = c->wave_times.p;
    }
    // every global row the render launch may touch lies inside its buffer (the probe
    // may have grown them): checked on the host, and handed to the STATS flavour's
    // device check
    zrt::check_buffers("render launch", need, c->att.n, c->stack_ovf.n);
    a.att = c->att.p;
    if (need.ovf_bytes) a.stack_ovf = c->stack_ovf.p;
    a.att_cap = c->att.n;
    a.ovf_cap = zrt::ovf_cap_elems(c->stack_ovf.n, stk16);
    if (diag)
      if (const char* e = std::getenv("ZRT_DEBUG_ROW_CAP")) {  // tests: the device check reports a smaller buffer
        const double f = std::atof(e);
        a.att_cap = uint64_t(double(a.att_cap) * f);
        a.ovf_cap = uint64_t(double(a.ovf_cap) * f);
      }
    HIPCHK(hipEventRecord(c->ev0, st));
    if (work > 0) {
      void* args[] = {&a};
      HIPCHK(hipLaunchKernel(kfn, dim3(grid), dim3(zrt::kBlock), args, lds, st));
    }
    HIPCHK(hipEventRecord(c->ev1, st));
    if (my_tiles > 0) {
      const uint32_t n_slots = my_tiles * 64u;
      hipLaunchKernelGGL(zrt::finalize_kernel, dim3((n_slots + 255) / 256), dim3(256), 0, st, c->partial.p,
                         dev_tiles, n_slots, n_chunks, p->world_size, p->rank, g.tiles_x, g.xbound, p->height,
                         a.color_scale, c->scratch.p + zrt::kErrorSlot);
      HIPCHK(hipGetLastError());
    }
    HIPCHK(hipMemcpyAsync(c->err_host, c->scratch.p + zrt::kErrorSlot, sizeof(unsigned long long),
                          hipMemcpyDeviceToHost, st));
    HIPCHK(hipEventRecord(c->ev_done, st));
    c->err_reported = false;
    // count the pixels this rank renders (for samples/pixels counters)
    uint64_t pixels = 0;
    for (uint32_t lt = 0; lt < my_tiles; ++lt) {
      const uint32_t t = lt * p->world_size + p->rank;
      const uint32_t tx = t % g.tiles_x, ty = t / g.tiles_x;
      const uint32_t w = std::min(8u, g.xbound - tx * 8u), h = std::min(8u, p->height - ty * 8u);
      pixels += uint64_t(w) * h;
    }
    c->last_pixels = uint32_t(pixels);
    c->last_spp = p->samples_per_pixel;
    c->last_tiles = my_tiles;
    c->last_rank = p->rank;
    c->last_world = p->world_size;
    c->last_tiles_x = g.tiles_x;
    c->last_xbound = g.xbound;
    c->last_stats = diag;
    c->last_mode = mode;
    c->last_loop = kmode == 7 || kmode == 8 || kmode == 9 ? 5 : kmode;
    c->last_qn = qn;
    c->last_guard = a.guard;
    c->launched = 1;
    return ZRT_OK;
  }
  ZRT_CATCH_ALL
}

int zrt_ctx_stats(zrt_ctx* c, zrt_stats* out) {
  if (!c || !out) return fail(ZRT_E_INVALID, "null argument");
  if (!c->launched) return fail(ZRT_E_INVALID, "zrt_ctx_stats before any zrt_ctx_render_tiles");
  try {
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipEventSynchronize(c->ev_done));
    unsigned long long h[zrt::kScratchSlots] = {0};
    HIPCHK(hipMemcpy(h, c->scratch.p, sizeof(h), hipMemcpyDeviceToHost));
    if (c->scanline_rows) {  // ZRT_FLAG_SCANLINES: the launch counted these three per row only
      std::vector<unsigned long long> rows(size_t(c->scanline_rows) * 3);
      HIPCHK(hipMemcpy(rows.data(), c->scanlines.p, rows.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
      for (size_t y = 0; y < c->scanline_rows; ++y) {
        h[zrt::kDepthHits] += rows[3 * y];
        h[zrt::kReflections] += rows[3 * y + 1];
        h[zrt::kBackground] += rows[3 * y + 2];
      }
    }
    std::memset(out, 0, sizeof(*out));
    out->recursion_depth_hits = h[zrt::kDepthHits];
    out->reflections = h[zrt::kReflections];
    out->background_hits = h[zrt::kBackground];
    // rayColor calls = samples + reflections = rays + depth-limit hits
    out->rays_processed = c->last_stats ? h[zrt::kRays]
                                        : uint64_t(c->last_pixels) * c->last_spp + h[zrt::kReflections] -
                                              h[zrt::kDepthHits];
    out->node_visits = h[zrt::kNodes];
    out->prim_tests = h[zrt::kTriTests] + h[zrt::kSphereTests];
    out->sphere_tests = h[zrt::kSphereTests];
    out->shade_fetches = h[zrt::kShades];
    out->texel_fetches = h[zrt::kTexels];
    out->leaf_visits = h[zrt::kLeaves];
    out->order_replays = h[zrt::kReplays];
    uint32_t bt = uint32_t(h[zrt::kExcessTri]), bs = uint32_t(h[zrt::kExcessSph]);
    std::memcpy(&out->box_excess_max_triangle, &bt, 4);
    std::memcpy(&out->box_excess_max_sphere, &bs, 4);
    out->box_excess_hits = h[zrt::kExcessHits];
    // FAST: leaf boxes ride in their parent's 128 B; compressed: 64-B nodes (+ 32-B leaf records)
    out->node_bytes = c->last_mode == 3 ? (c->last_qn ? 64 : 128) : 32;
    out->wide_nodes = c->n_wide;
    out->sampling_loop = uint32_t(c->last_loop);
    out->guard = c->last_guard;
    out->texel_bytes = c->texel_bytes;
    out->pixels_processed = c->last_pixels;
    out->samples_processed = uint64_t(c->last_pixels) * c->last_spp;
    out->preprocess_ms = c->preprocess_ms;
    out->upload_ms = c->upload_ms;
    float ms = 0.0f, sched = 0.0f;
    HIPCHK(hipEventElapsedTime(&ms, c->ev_pre, c->ev1));
    HIPCHK(hipEventElapsedTime(&sched, c->ev_pre, c->ev0));
    out->render_ms = ms;
    out->schedule_ms = c->scheduled ? sched : 0.0f;
    out->used_bvh = c->use_bvh ? 1 : 0;
    out->bvh_nodes = c->n_nodes;
    out->bvh_max_depth = c->bvh_depth;
    out->n_gpus = 1;
    return zrt::launch_status(c, true);
  }
  ZRT_CATCH_ALL
}

int zrt_ctx_sync(zrt_ctx* c) {
  if (!c) return fail(ZRT_E_INVALID, "null argument");
  try {
    HIPCHK(hipSetDevice(c->device));
    return zrt::launch_status(c, true);
  }
  ZRT_CATCH_ALL
}

namespace zrt {
namespace {
// The per-row Progress counters of c's last launch (ZRT_FLAG_SCANLINES) added
// into out[0 .. height): this rank's pixels, samples and rays of each row and
// the three counters the kernel counted per row.
int add_scanlines(zrt_ctx* c, zrt_scanline* out, uint32_t height) {
  if (!c->launched || c->scanline_rows == 0)
    return fail(ZRT_E_INVALID, "the last launch did not count scanlines (ZRT_FLAG_SCANLINES)");
  if (height != c->scanline_rows) return fail(ZRT_E_INVALID, "height differs from the last launch's");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipEventSynchronize(c->ev_done));
  std::vector<unsigned long long> rows(size_t(height) * 3);
  HIPCHK(hipMemcpy(rows.data(), c->scanlines.p, rows.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  for (uint32_t lt = 0; lt < c->last_tiles; ++lt) {  // pixels of this rank's tiles, per row
    const uint32_t t = lt * c->last_world + c->last_rank;
    const uint32_t tx = t % c->last_tiles_x, ty = t / c->last_tiles_x;
    const uint32_t w = std::min(8u, c->last_xbound - tx * 8u);
    for (uint32_t y = ty * 8u; y < std::min(height, ty * 8u + 8u); ++y) out[y].pixels += w;
  }
  for (uint32_t y = 0; y < height; ++y) {
    out[y].recursion_depth_hits += rows[3 * y];
    out[y].reflections += rows[3 * y + 1];
    out[y].background_hits += rows[3 * y + 2];
  }
  // samples and rays from the pixels (rays = rayColor calls - depth-limit hits)
  for (uint32_t y = 0; y < height; ++y) {
    out[y].samples = out[y].pixels * uint64_t(c->last_spp);
    out[y].rays = out[y].samples + out[y].reflections - out[y].recursion_depth_hits;
  }
  return ZRT_OK;
}
}  // namespace
}  // namespace zrt

int zrt_ctx_scanlines(zrt_ctx* c, zrt_scanline* out, uint32_t height) {
  if (!c || !out) return fail(ZRT_E_INVALID, "null argument");
  try {
    std::memset(out, 0, sizeof(zrt_scanline) * height);
    int rc = zrt::add_scanlines(c, out, height);
    if (rc) return rc;
    return zrt::launch_status(c, true);
  }
  ZRT_CATCH_ALL
}

int zrt_ctx_debug_counters(zrt_ctx* c, uint64_t* out, uint32_t n) {
  if (!c || !out) return fail(ZRT_E_INVALID, "null argument");
  if (!c->launched) return fail(ZRT_E_INVALID, "no kernel launched on this context yet");
  try {
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipEventSynchronize(c->ev_done));
    unsigned long long h[zrt::kScratchSlots] = {0};
    HIPCHK(hipMemcpy(h, c->scratch.p, sizeof(h), hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < n && i < uint32_t(zrt::kScratchSlots); ++i) out[i] = h[i];
    return ZRT_OK;
  }
  ZRT_CATCH_ALL
}

int zrt_ctx_debug_wave_times(zrt_ctx* c, uint64_t* out, uint32_t cap, uint32_t* n_waves) {
  if (!c || !n_waves) return fail(ZRT_E_INVALID, "null argument");
  try {
    HIPCHK(hipSetDevice(c->device));
    if (c->launched) HIPCHK(hipEventSynchronize(c->ev_done));
    *n_waves = ZRT_PROFILE ? c->n_waves : 0u;
    const size_t n = std::min<size_t>(cap / 2, *n_waves);
    if (n && out) HIPCHK(hipMemcpy(out, c->wave_times.p, 2 * n * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return ZRT_OK;
  }
  ZRT_CATCH_ALL
}

int zrt_ctx_debug_schedule(zrt_ctx* c, uint32_t* costs, uint32_t* order, uint32_t cap, uint32_t* n_tiles) {
  if (!c || !n_tiles) return fail(ZRT_E_INVALID, "null argument");
  if (!c->launched) return fail(ZRT_E_INVALID, "no kernel launched on this context yet");
  try {
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipEventSynchronize(c->ev_done));
    *n_tiles = c->scheduled ? c->tile_ids_n : 0u;
    const size_t n = std::min<size_t>(cap, *n_tiles);
    if (n && costs) HIPCHK(hipMemcpy(costs, c->tile_cost.p, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (n && order) HIPCHK(hipMemcpy(order, c->tile_order.p, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return ZRT_OK;
  }
  ZRT_CATCH_ALL
}

int zrt_ctx_last_kernel_ms(zrt_ctx* c, double* ms) {
  if (!c || !ms) return fail(ZRT_E_INVALID, "null argument");
  if (!c->launched) return fail(ZRT_E_INVALID, "no kernel launched on this context yet");
  try {
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipEventSynchronize(c->ev1));
    float f = 0.0f;
    HIPCHK(hipEventElapsedTime(&f, c->ev0, c->ev1));
    *ms = f;
    return zrt::launch_status(c, true);
  }
  ZRT_CATCH_ALL
}

int zrt_ctx_assemble(zrt_ctx* c, const zrt_params* p, const float* dev_gathered, float* dev_frame,
                     void* hip_stream) {
  return zrt::assemble(c, p, dev_gathered, 0, dev_frame, hip_stream);
}

int zrt_ctx_assemble_padded(zrt_ctx* c, const zrt_params* p, const float* dev_gathered, uint32_t stride_tiles,
                            float* dev_frame, void* hip_stream) {
  if (stride_tiles == 0) return fail(ZRT_E_INVALID, "stride_tiles must be > 0");
  return zrt::assemble(c, p, dev_gathered, stride_tiles, dev_frame, hip_stream);
}

namespace zrt {
namespace {
int render_one(const zrt_scene* scene, const zrt_camera* camera, const zrt_params* params, float* out_rgb,
               zrt_stats* stats, zrt_scanline* rows) {
  if (!camera || !out_rgb) return fail(ZRT_E_INVALID, "null argument");
  int rc = zrt::validate_params(params);
  if (rc) return rc;
  zrt_params p = *params;
  p.rank = 0;
  p.world_size = 1;
  if (rows) p.flags |= ZRT_FLAG_SCANLINES;
  zrt_ctx* c = nullptr;
  rc = zrt_ctx_create(scene, &p, &c);
  if (rc) return rc;
  std::unique_ptr<zrt_ctx, int (*)(zrt_ctx*)> guard(c, zrt_ctx_destroy);
  try {
    uint32_t n_tiles = 0;
    rc = zrt_ctx_tile_count(c, &p, &n_tiles);
    if (rc) return rc;
    zrt::DevBuf<float> tiles, frame;
    tiles.alloc(size_t(n_tiles) * 64 * 3);
    frame.alloc(size_t(p.width) * p.height * 3);
    rc = zrt_ctx_render_tiles(c, camera, &p, tiles.p, nullptr);
    if (rc) return rc;
    rc = zrt_ctx_assemble(c, &p, tiles.p, frame.p, nullptr);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipMemcpy(out_rgb, frame.p, sizeof(float) * 3 * size_t(p.width) * p.height, hipMemcpyDeviceToHost));
    zrt_stats s;
    rc = zrt_ctx_stats(c, &s);
    if (rc) return rc;
    if (rows) {
      std::memset(rows, 0, sizeof(zrt_scanline) * p.height);
      rc = add_scanlines(c, rows, p.height);
      if (rc) return rc;
    }
    if (stats) *stats = s;
    return ZRT_OK;
  }
  ZRT_CATCH_ALL
}
}  // namespace
}  // namespace zrt

int zrt_render(const zrt_scene* scene, const zrt_camera* camera, const zrt_params* params,
               float* out_rgb, zrt_stats* stats) {
  return zrt::render_one(scene, camera, params, out_rgb, stats, nullptr);
}

int zrt_render_progress(const zrt_scene* scene, const zrt_camera* camera, const zrt_params* params,
                        float* out_rgb, zrt_stats* stats, zrt_scanline* scanlines) {
  if (!scanlines) return fail(ZRT_E_INVALID, "null argument");
  return zrt::render_one(scene, camera, params, out_rgb, stats, scanlines);
}

// ---- several GPUs from one host thread (zrt_multi_*, zrt_render_multi) -------
int zrt_multi_create(const zrt_scene* scene, const zrt_params* params, const uint32_t* devices,
                     uint32_t n_devices, zrt_multi** out) {
  if (!out || !devices) return fail(ZRT_E_INVALID, "null argument");
  *out = nullptr;
  if (n_devices == 0 || n_devices > 1024) return fail(ZRT_E_INVALID, "n_devices must be in 1..1024");
  if (!params) return fail(ZRT_E_INVALID, "params is null");
  int rc = zrt::validate_scene(scene);
  if (rc) return rc;
  for (uint32_t r = 0; r < n_devices; ++r) {
    rc = zrt::check_device(int(devices[r]));
    if (rc) return rc;
  }
  try {
    std::unique_ptr<zrt_multi> m(new zrt_multi);
    m->devices.assign(devices, devices + n_devices);
    std::vector<uint32_t> distinct(m->devices);
    std::sort(distinct.begin(), distinct.end());
    distinct.erase(std::unique(distinct.begin(), distinct.end()), distinct.end());
    m->n_distinct = uint32_t(distinct.size());
    // RCCL only where there is something to move between GPUs: one rank per
    // device, at least two devices (a device listed twice gathers by copies)
    m->use_rccl = m->n_distinct == n_devices && n_devices > 1;
    // the scene flattened once (BVH build, raytrace.zig:124-133), a copy on every GPU
    const bool use_bvh = params->bounded_volume_hierarchy != 0 && scene->n_prims > 10;
    zrt::HostScene host;
    zrt::flatten_scene(&host, scene, use_bvh, int(devices[0]));
    for (uint32_t r = 0; r < n_devices; ++r) m->ctx.emplace_back(zrt::ctx_on_device(host, int(devices[r])).release());
    m->send.resize(n_devices);
    if (m->use_rccl) {
      // communicators live as long as the context (not per frame)
      const zrt::Rccl& R = zrt::rccl();
      m->comms.R = &R;
      m->comms.c.assign(n_devices, nullptr);
      std::vector<int> devs(devices, devices + n_devices);
      NCCLCHK(R, R.comm_init_all(m->comms.c.data(), int(n_devices), devs.data()));
    }
    *out = m.release();
    return ZRT_OK;
  }
  ZRT_CATCH_ALL
}

int zrt_multi_destroy(zrt_multi* m) {
  if (!m) return ZRT_OK;
  for (auto& c : m->ctx) {
    (void)hipSetDevice(c->device);
    (void)hipDeviceSynchronize();
  }
  delete m;
  return ZRT_OK;
}

int zrt_multi_render(zrt_multi* m, const zrt_camera* camera, const zrt_params* params, float* out_rgb,
                     zrt_stats* stats) {
  if (!m || !camera) return fail(ZRT_E_INVALID, "null argument");  // out_rgb NULL: the frame stays on devices[0]
  int rc = zrt::validate_params(params);
  if (rc) return rc;
  const uint32_t n = uint32_t(m->ctx.size());
  try {
    const zrt::Geometry g = zrt::geometry(params);
    std::vector<zrt_params> rp(n, *params);
    std::vector<uint32_t> count(n), base(n + 1, 0);
    uint32_t max_tiles = 0;
    for (uint32_t r = 0; r < n; ++r) {
      rp[r].rank = r;
      rp[r].world_size = n;
      rp[r].device = m->devices[r];
      count[r] = zrt::rank_tiles(g, r, n);
      base[r + 1] = base[r] + count[r];
      max_tiles = std::max(max_tiles, count[r]);
    }
    const size_t slot = 64 * 3;  // floats per tile
    // tile buffers padded to the largest rank's (ncclGather sends equal counts)
    for (uint32_t r = 0; r < n; ++r) {
      HIPCHK(hipSetDevice(m->ctx[r]->device));
      if (m->send[r].n < std::max<size_t>(1, max_tiles * slot)) m->send[r].alloc(std::max<size_t>(1, max_tiles * slot));
    }
    // the sampling loops, all enqueued before any is waited on
    for (uint32_t r = 0; r < n; ++r) {
      rc = zrt_ctx_render_tiles(m->ctx[r].get(), camera, &rp[r], m->send[r].p, nullptr);
      if (rc) return rc;
    }
    zrt_stats sum;
    std::memset(&sum, 0, sizeof(sum));
    int device_rc = ZRT_OK;
    std::string device_msg;
    m->frame_n = 0;
    m->rank_ms.assign(n, 0.0);
    for (uint32_t r = 0; r < n; ++r) {
      zrt_stats s;
      rc = zrt_ctx_stats(m->ctx[r].get(), &s);  // waits for rank r's launch
      if (rc == ZRT_E_UNSUPPORTED) {  // device error: finish the frame (NaN tiles), then report it
        device_rc = rc;
        device_msg = zrt_last_error();
      }
      else if (rc) return rc;
      {  // the render kernel alone (ev0 -> ev1; render_ms also holds the schedule probe)
        float ms = 0.0f;
        HIPCHK(hipSetDevice(m->ctx[r]->device));
        HIPCHK(hipEventElapsedTime(&ms, m->ctx[r]->ev0, m->ctx[r]->ev1));
        m->rank_ms[r] = ms;
      }
      if (r == 0) {
        sum = s;
        continue;
      }
      sum.recursion_depth_hits += s.recursion_depth_hits;
      sum.reflections += s.reflections;
      sum.background_hits += s.background_hits;
      sum.pixels_processed += s.pixels_processed;
      sum.samples_processed += s.samples_processed;
      sum.rays_processed += s.rays_processed;
      sum.node_visits += s.node_visits;
      sum.prim_tests += s.prim_tests;
      sum.sphere_tests += s.sphere_tests;
      sum.shade_fetches += s.shade_fetches;
      sum.texel_fetches += s.texel_fetches;
      sum.leaf_visits += s.leaf_visits;
      sum.order_replays += s.order_replays;
      sum.preprocess_ms = std::max(sum.preprocess_ms, s.preprocess_ms);
      sum.upload_ms = std::max(sum.upload_ms, s.upload_ms);
      sum.render_ms = std::max(sum.render_ms, s.render_ms);
      sum.schedule_ms = std::max(sum.schedule_ms, s.schedule_ms);
    }
    // the gather to devices[0] in the padded rank-major layout (rank r at
    // r * max_tiles tiles), which zrt_ctx_assemble_padded reads as it lies
    const double t0 = zrt::now_ms();
    zrt_ctx* root = m->ctx[0].get();
    HIPCHK(hipSetDevice(root->device));
    const size_t frame_n = size_t(params->width) * params->height * 3;
    if (m->frame.n < frame_n) m->frame.alloc(frame_n);
    const size_t gathered_n = std::max<size_t>(1, size_t(n) * max_tiles * slot);
    if (m->gathered.n < gathered_n) m->gathered.alloc(gathered_n);
    if (m->use_rccl) {
      const zrt::Rccl& R = *m->comms.R;
      NCCLCHK(R, R.group_start());
      for (uint32_t r = 0; r < n; ++r)
        NCCLCHK(R, R.gather(m->send[r].p, r == 0 ? m->gathered.p : nullptr, size_t(max_tiles) * slot, ncclFloat32, 0,
                            m->comms.c[r], m->ctx[r]->stream));
      NCCLCHK(R, R.group_end());
      // every rank's part of the gather is done before the next frame reuses its buffer
      for (uint32_t r = 1; r < n; ++r) {
        HIPCHK(hipSetDevice(m->ctx[r]->device));
        HIPCHK(hipStreamSynchronize(m->ctx[r]->stream));
      }
      HIPCHK(hipSetDevice(root->device));
    } else {
      // one device (or ranks sharing devices): copies; every rank's launch is done (stats above)
      for (uint32_t r = 0; r < n; ++r)
        if (count[r])
          HIPCHK(hipMemcpyPeerAsync(m->gathered.p + size_t(r) * max_tiles * slot, root->device, m->send[r].p,
                                    m->ctx[r]->device, size_t(count[r]) * slot * sizeof(float), root->stream));
    }
    rc = zrt_ctx_assemble_padded(root, &rp[0], m->gathered.p, std::max(1u, max_tiles), m->frame.p, nullptr);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(root->stream));
    sum.gather_ms = zrt::now_ms() - t0;
    m->frame_n = frame_n;
    if (out_rgb) HIPCHK(hipMemcpy(out_rgb, m->frame.p, sizeof(float) * frame_n, hipMemcpyDeviceToHost));
    sum.n_gpus = m->n_distinct;
    if (stats) *stats = sum;
    if (device_rc) return fail(device_rc, device_msg);
    return ZRT_OK;
  }
  ZRT_CATCH_ALL
}

int zrt_multi_frame(zrt_multi* m, float* out_rgb, uint64_t n_floats) {
  if (!m || !out_rgb) return fail(ZRT_E_INVALID, "null argument");
  if (m->frame_n == 0) return fail(ZRT_E_INVALID, "no frame: zrt_multi_frame before a successful zrt_multi_render");
  if (n_floats != m->frame_n) return fail(ZRT_E_INVALID, "n_floats differs from the last frame's width * height * 3");
  try {
    HIPCHK(hipSetDevice(m->ctx[0]->device));
    HIPCHK(hipMemcpy(out_rgb, m->frame.p, sizeof(float) * m->frame_n, hipMemcpyDeviceToHost));
    return ZRT_OK;
  }
  ZRT_CATCH_ALL
}

int zrt_multi_rank_ms(zrt_multi* m, double* kernel_ms, uint32_t n) {
  if (!m || !kernel_ms) return fail(ZRT_E_INVALID, "null argument");
  if (m->rank_ms.empty()) return fail(ZRT_E_INVALID, "no frame rendered yet");
  if (n != m->rank_ms.size()) return fail(ZRT_E_INVALID, "n differs from the context's rank count");
  for (uint32_t r = 0; r < n; ++r) kernel_ms[r] = m->rank_ms[r];
  return ZRT_OK;
}

int zrt_multi_scanlines(zrt_multi* m, zrt_scanline* out, uint32_t height) {
  if (!m || !out) return fail(ZRT_E_INVALID, "null argument");
  try {
    std::memset(out, 0, sizeof(zrt_scanline) * height);
    for (auto& c : m->ctx) {
      const int rc = zrt::add_scanlines(c.get(), out, height);
      if (rc) return rc;
    }
    return ZRT_OK;
  }
  ZRT_CATCH_ALL
}

int zrt_render_multi(const zrt_scene* scene, const zrt_camera* camera, const zrt_params* params,
                     const uint32_t* devices, uint32_t n_devices, float* out_rgb, zrt_stats* stats) {
  if (!camera || !out_rgb || !devices) return fail(ZRT_E_INVALID, "null argument");
  int rc = zrt::validate_params(params);
  if (rc) return rc;
  zrt_multi* m = nullptr;
  rc = zrt_multi_create(scene, params, devices, n_devices, &m);
  if (rc) return rc;
  rc = zrt_multi_render(m, camera, params, out_rgb, stats);
  const std::string msg = zrt_last_error();
  zrt_multi_destroy(m);
  if (rc) return fail(rc, msg);
  return ZRT_OK;
}

int zrt_trace(const zrt_scene* scene, const zrt_params* params, const float* rays, uint32_t n_rays, float* out_t,
              int32_t* out_prim) {
  if (!params || (n_rays && (!rays || !out_t || !out_prim))) return fail(ZRT_E_INVALID, "null argument");
  int rc = zrt::validate_scene(scene);
  if (rc) return rc;
  if (params->traversal > ZRT_TRAVERSAL_BINARY) return fail(ZRT_E_INVALID, "unknown traversal");
  rc = zrt::check_device(int(params->device));
  if (rc) return rc;
  if (n_rays == 0) return ZRT_OK;
  try {
    const bool use_bvh = params->bounded_volume_hierarchy != 0 && scene->n_prims > 10;
    zrt::HostScene h;
    zrt::flatten_scene(&h, scene, use_bvh, int(params->device));
    std::unique_ptr<zrt_ctx> c = zrt::ctx_on_device(h, int(params->device));
    const int mode = !c->use_bvh ? 0
                     : params->traversal == ZRT_TRAVERSAL_REFERENCE ? 2
                     : params->traversal == ZRT_TRAVERSAL_BINARY ? 1 : 3;
    const char* force_rows = std::getenv("ZRT_STACK_LDS_ROWS");  // tests: force the overflow rows into use
    const uint32_t stack_depth = mode == 3 ? std::max(c->wide_stack, c->stack_depth) : c->stack_depth;
    const bool stk16 = mode == 3 ? c->n_wide < 65536 && c->n_nodes < 65536 && !force_rows : c->n_nodes < 65536;
    // FAST over compressed nodes (wide_iter_q, MODE 8) where the context built them
    const bool qn = mode == 3 && c->q_ok;
    const uint32_t node_f4 = qn ? zrt::kQuantNodeF4 : 8u;
    const zrt::LdsPlan lp = zrt::plan_lds(c.get(), mode, stk16, stack_depth, 0, false, false, ZRT_PRNG_XOROSHIRO128,
                                          node_f4);
    const uint32_t lds_rows = lp.stack_rows;
    const uint32_t grid = (n_rays + zrt::kBlock - 1) / zrt::kBlock;
    const uint64_t n_lanes = uint64_t(grid) * zrt::kBlock;
    zrt::DevBuf<float> d_rays, d_t;
    zrt::DevBuf<int32_t> d_slot;
    d_rays.alloc(6ull * n_rays);
    d_t.alloc(n_rays);
    d_slot.alloc(n_rays);
    HIPCHK(hipMemcpy(d_rays.p, rays, sizeof(float) * 6ull * n_rays, hipMemcpyHostToDevice));
    HIPCHK(hipMemset(c->scratch.p, 0, zrt::kScratchSlots * sizeof(unsigned long long)));
    zrt::KArgs a{};
    a.nodes = c->nodes.p;
    a.prims = c->prims.p;
    a.shade = c->shade.p;
    a.wnodes = qn ? c->qnodes.p : c->wnodes.p;
    a.wide_stride = qn ? c->q_stride : c->wide_stride;
    a.node_f4 = node_f4;
    a.qleaves = qn ? c->qleaves.p : nullptr;
    a.n_qnodes = qn ? c->q_stride / zrt::kQuantNodeF4 : 0u;
    a.n_qleaves = qn ? c->n_qleaves : 0u;
    a.error_flag = reinterpret_cast<uint32_t*>(c->scratch.p + zrt::kErrorSlot);
    a.n_list = c->use_bvh ? 0 : c->n_prims;
    a.tri_rcp_fast = c->tri_rcp_fast;
    a.scene_extent = c->scene_extent;
    a.paxis_m = zrt::paxis_threshold();
    for (int k = 0; k < 3; ++k) {
      a.tri_c[k] = c->tri_c[k];
      a.tri_h[k] = c->tri_h[k];
    }
    a.stack_depth = stack_depth;
    a.ref_stack = c->stack_depth;
    a.leaf_of_slot = c->leaf_of_slot.p;
    a.ref_sph = c->ref_sph.p;
    for (int k = 0; k < 3; ++k) a.root_c[k] = c->root_c[k];
    a.origin_bound = c->origin_bound;
    a.check_origins = 1;  // arbitrary ray origins
    a.layout = c->layout;
    a.graze_m = c->graze_m;
    a.graze_leaf = c->graze_leaf;
    // tests: ZRT_DEBUG_NO_GUARD=1 traces without the grazing-triangle guard (the
    // default render kernels' traversal), to record what the guard is for
    a.guard = std::getenv("ZRT_DEBUG_NO_GUARD") ? 0.0f : c->guard;
    a.lds_rows = lds_rows;
    a.n_lanes = uint32_t(n_lanes);
    a.n_top = qn ? c->q_top : c->n_top;
    a.lds_top_off = lp.top_off;
    a.lds_att_off = lp.att_off;
    const zrt::BufNeed need = zrt::buffer_need(lp, 0, stack_depth, n_lanes, n_lanes, stk16);
    if (need.ovf_bytes) {
      c->stack_ovf.alloc(need.ovf_bytes);
      a.stack_ovf = c->stack_ovf.p;
    }
    zrt::check_buffers("trace launch", zrt::BufNeed{0, need.ovf_bytes}, c->att.n, c->stack_ovf.n);
    a.att_cap = c->att.n;
    a.ovf_cap = zrt::ovf_cap_elems(c->stack_ovf.n, stk16);
    void* fn = nullptr;
#define ZRT_TK(M) (stk16 ? reinterpret_cast<void*>(&zrt::trace_kernel<M, uint16_t>) \
                         : reinterpret_cast<void*>(&zrt::trace_kernel<M, uint32_t>))
#ifdef ZRT_ISA_KERNEL
    fn = nullptr;
#else
    fn = mode == 0 ? ZRT_TK(0) : mode == 1 ? ZRT_TK(1) : mode == 2 ? ZRT_TK(2) : qn ? ZRT_TK(8) : ZRT_TK(3);
#endif
#undef ZRT_TK
    const float* rp = d_rays.p;
    float* tp = d_t.p;
    int32_t* sp = d_slot.p;
    uint32_t nn = n_rays;
    void* args[] = {&a, &rp, &nn, &tp, &sp};
    HIPCHK(hipLaunchKernel(fn, dim3(grid), dim3(zrt::kBlock), args, lp.bytes, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    unsigned long long err = 0;
    HIPCHK(hipMemcpy(&err, c->scratch.p + zrt::kErrorSlot, sizeof(err), hipMemcpyDeviceToHost));
    if (err) return fail(ZRT_E_UNSUPPORTED, zrt::device_error_msg(err));
    std::vector<int32_t> slot(n_rays);
    HIPCHK(hipMemcpy(out_t, d_t.p, sizeof(float) * n_rays, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(slot.data(), d_slot.p, sizeof(int32_t) * n_rays, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < n_rays; ++i)
      out_prim[i] = slot[i] < 0 ? -1 : int32_t(c->slot_to_prim[size_t(slot[i])]);
    return ZRT_OK;
  } catch (const zrt::HipError& e) {
    return zrt::hip_fail(e);
  } catch (const zrt::Error& e) {
    return fail(e.code, e.what());
  } catch (const std::bad_alloc&) {
    return fail(ZRT_E_NOMEM, "OutOfMemory");
  }
}

int zrt_debug_math(int fn, const float* x, const float* y, float* out, uint32_t n, uint32_t device) {
  if (!x || !out) return fail(ZRT_E_INVALID, "null argument");
  int rc = zrt::check_device(int(device));
  if (rc) return rc;
  try {
    HIPCHK(hipSetDevice(int(device)));
    zrt::DevBuf<float> dx, dy, dout;
    dx.alloc(n);
    dout.alloc(n);
    HIPCHK(hipMemcpy(dx.p, x, n * sizeof(float), hipMemcpyHostToDevice));
    if (y) {
      dy.alloc(n);
      HIPCHK(hipMemcpy(dy.p, y, n * sizeof(float), hipMemcpyHostToDevice));
    }
    hipLaunchKernelGGL(zrt::debug_math_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, fn, dx.p,
                       y ? dy.p : nullptr, dout.p, n);
    HIPCHK(hipGetLastError());
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(out, dout.p, n * sizeof(float), hipMemcpyDeviceToHost));
    return ZRT_OK;
  }
  ZRT_CATCH_ALL
}

int zrt_debug_lds_plans(const zrt_scene* scene, uint32_t* n_checked) {
  if (!n_checked) return fail(ZRT_E_INVALID, "null argument");
  *n_checked = 0;
  int rc = zrt::validate_scene(scene);
  if (rc) return rc;
  try {
    zrt::HostScene h;
    // (the host BVH build: no device; the compressed nodes built too, so their
    // plans are checked with the top levels they really keep in LDS)
    zrt::flatten_scene(&h, scene, scene->n_prims > 10, -1, scene->n_prims > 10 ? 1 : 0);
    const uint32_t n_mats = uint32_t(h.mats.size());
    const uint32_t ref_depth = h.use_bvh ? h.bvh_depth + 2 : 0;
    std::string where;
    for (int mode : {0, 1, 2, 3}) {
      for (int loop = 0; loop < (mode == 3 ? 3 : 1); ++loop) {  // lockstep, wavefront, path pool
        for (bool stk16 : {true, false}) {
          for (uint32_t prng : {uint32_t(ZRT_PRNG_XOROSHIRO128), uint32_t(ZRT_PRNG_XOSHIRO256)}) {
            for (uint32_t depth : {0u, 1u, 2u, 5u, 20u, 50u}) {
              for (uint32_t nf4 : {8u, 4u}) {  // full / compressed wide nodes (the path pool only)
                if (nf4 == 4u && (loop != 2 || !h.q_ok)) continue;
                const uint32_t sd = mode == 3 ? std::max(h.wide_stack, ref_depth) : ref_depth;
                where = "mode " + std::to_string(mode) + " loop " + std::to_string(loop) + " stk16 " +
                        std::to_string(int(stk16)) + " prng " + std::to_string(prng) + " depth " +
                        std::to_string(depth) + " node_f4 " + std::to_string(nf4);
                try {
                  (void)zrt::plan_lds(nf4 == 4u ? h.q_top : h.n_top, n_mats, mode, stk16, sd, depth, loop == 1,
                                      loop == 2, prng, nf4);
                } catch (const zrt::Error& e) {
                  throw zrt::Error(e.code, std::string(e.what()) + " (" + where + ")");
                }
                ++*n_checked;
              }
            }
          }
        }
      }
    }
    return ZRT_OK;
  }
  ZRT_CATCH_ALL
}

int zrt_debug_buffer_plans(const zrt_scene* scene, uint32_t legacy, uint32_t* n_checked) {
  if (!n_checked) return fail(ZRT_E_INVALID, "null argument");
  *n_checked = 0;
  int rc = zrt::validate_scene(scene);
  if (rc) return rc;
  if (scene->n_prims <= 10) return ZRT_OK;  // no tree: no FAST launch, no probe
  try {
    zrt::HostScene h;
    zrt::flatten_scene(&h, scene, true, -1, 1);
    const uint32_t n_mats = uint32_t(h.mats.size());
    const uint32_t sd = std::max(h.wide_stack, h.bvh_depth + 2);  // zrt_render's FAST stack depth
    for (int loop = 0; loop < 3; ++loop) {  // the render launch: lockstep, wavefront, path pool
      for (bool stk16 : {true, false}) {
        for (uint32_t prng : {uint32_t(ZRT_PRNG_XOROSHIRO128), uint32_t(ZRT_PRNG_XOSHIRO256)}) {
          for (uint32_t depth : {0u, 1u, 2u, 4u, 5u, 6u, 13u, 20u, 50u}) {
            for (uint32_t nf4 : {8u, 4u}) {
              if (nf4 == 4u && (loop != 2 || !h.q_ok)) continue;
              for (uint32_t grid : {64u, 1536u, 2048u}) {  // blocks (the probe: at most the render's)
                const std::string where = "loop " + std::to_string(loop) + " stk16 " + std::to_string(int(stk16)) +
                                          " prng " + std::to_string(prng) + " depth " + std::to_string(depth) +
                                          " node_f4 " + std::to_string(nf4) + " grid " + std::to_string(grid);
                // zrt_render's sizing: the render launch's need, then (schedule_tiles) the
                // probe's, the buffers grown to the larger of the two
                const zrt::LdsPlan lp = zrt::plan_lds(nf4 == 4u ? h.q_top : h.n_top, n_mats, 3, stk16, sd, depth,
                                                      loop == 1, loop == 2, prng, nf4);
                const uint64_t n_lanes = uint64_t(grid) * zrt::kBlock;
                const uint64_t n_paths = loop == 2 ? uint64_t(grid) * zrt::kBlockPaths : n_lanes;
                const zrt::BufNeed rn = zrt::buffer_need(lp, depth, sd, n_paths, n_lanes, stk16);
                const zrt::LdsPlan pp = zrt::plan_lds(h.n_top, n_mats, 3, stk16, sd, depth, false, false, prng, 8);
                const zrt::BufNeed pn = zrt::buffer_need(pp, depth, sd, n_lanes, n_lanes, stk16);
                uint64_t att = rn.att_elems, ovf = std::max(rn.ovf_bytes, pn.ovf_bytes);
                // legacy = 1: the sizing before commit 4072f5f, where the probe shared the
                // render launch's attenuation rows without growing them
                if (!legacy) att = std::max(att, pn.att_elems);
                try {
                  zrt::check_buffers("scheduling probe", pn, att, ovf);
                  zrt::check_buffers("render launch", rn, att, ovf);
                } catch (const zrt::Error& e) {
                  throw zrt::Error(e.code, std::string(e.what()) + " (" + where + ")");
                }
                ++*n_checked;
              }
            }
          }
        }
      }
    }
    return ZRT_OK;
  }
  ZRT_CATCH_ALL
}

int zrt_debug_qnodes(const zrt_scene* scene, uint64_t* n_checked) {
  if (!n_checked) return fail(ZRT_E_INVALID, "null argument");
  *n_checked = 0;
  int rc = zrt::validate_scene(scene);
  if (rc) return rc;
  if (scene->n_prims <= 10) return fail(ZRT_E_INVALID, "no BVH for <= 10 surfaces (raytrace.zig:124-133)");
  try {
    zrt::HostScene h;
    zrt::flatten_scene(&h, scene, true, -1, 1);  // (the compressed nodes asked for explicitly)
    if (!h.q_ok) return fail(ZRT_E_UNSUPPORTED, "the encoder refused this tree (a non-finite plane)");
    const uint32_t nn = h.q_stride / zrt::kQuantNodeF4, nw = h.wide_stride / 8u;
    if (nn != nw) return fail(ZRT_E_UNSUPPORTED, "compressed and full trees differ in node count");
    auto bad = [](const std::string& what, uint32_t o, uint32_t i, int k) {
      return fail(ZRT_E_UNSUPPORTED, what + " (octant " + std::to_string(o) + ", node " + std::to_string(i) + ", slot " +
                                         std::to_string(k) + ")");
    };
    for (uint32_t o = 0; o < 8; ++o) {
      for (uint32_t i = 0; i < nn; ++i) {
        const float4* F = &h.wn[size_t(o) * h.wide_stride + 8u * i];  // full node, this octant's copy
        uint32_t W[16];
        std::memcpy(W, &h.qn[size_t(o) * h.q_stride + zrt::kQuantNodeF4 * i], sizeof(W));
        float org[3], step[3];
        std::memcpy(org, W, 12);
        for (int a = 0; a < 3; ++a) step[a] = std::ldexp(1.0f, int((W[3] >> (8 * a)) & 0xffu) - 127);
        int32_t fr[4], qr[4], fb[4];
        std::memcpy(fr, &F[6], 16);
        std::memcpy(fb, &F[7], 16);
        std::memcpy(qr, &W[10], 16);
        for (int k = 0; k < 4; ++k) {
          const float* fn = reinterpret_cast<const float*>(F);
          const bool empty = qr[k] == zrt::kEmptyRef;
          for (int a = 0; a < 3 && !empty; ++a) {
            const double qn = double((W[4 + a] >> (8 * k)) & 0xffu), qf = double((W[7 + a] >> (8 * k)) & 0xffu);
            const double dn = double(org[a]) + qn * double(step[a]), df = double(org[a]) + qf * double(step[a]);
            if (double(float(dn)) != dn || double(float(df)) != df) return bad("a plane does not decode exactly", o, i, k);
            const bool neg = (o >> a) & 1u;  // the near plane is the max one
            const double full_n = fn[4 * a + k], full_f = fn[4 * (3 + a) + k];
            if (neg ? !(dn >= full_n && df <= full_f) : !(dn <= full_n && df >= full_f))
              return bad("a decoded box does not contain the full node's", o, i, k);
          }
          if (!empty && qr[k] >= 0 && qr[k] != fr[k]) return bad("an inner child ref differs", o, i, k);
          if (!empty && qr[k] < 0) {
            const bool sph = qr[k] < -zrt::kSphereSlotBias;
            const uint32_t L = uint32_t(-(sph ? qr[k] + zrt::kSphereSlotBias : qr[k]) - 1);
            if (size_t(L) * zrt::kLeafRecF4 + 1 >= h.ql.size()) return bad("a leaf record index past the records", o, i, k);
            const float4 mn = h.ql[zrt::kLeafRecF4 * size_t(L)], mx = h.ql[zrt::kLeafRecF4 * size_t(L) + 1];
            const float m[3] = {mn.x, mn.y, mn.z}, M[3] = {mx.x, mx.y, mx.z};
            for (int a = 0; a < 3; ++a) {
              const bool neg = (o >> a) & 1u;
              const float full_n = fn[4 * a + k], full_f = fn[4 * (3 + a) + k];
              const float rn = neg ? M[a] : m[a], rf = neg ? m[a] : M[a];
              if (std::memcmp(&rn, &full_n, 4) || std::memcmp(&rf, &full_f, 4)) return bad("a leaf record's box differs", o, i, k);
            }
            int32_t ra, rb;
            std::memcpy(&ra, &mn.w, 4);
            std::memcpy(&rb, &mx.w, 4);
            const int32_t full_a = sph ? fr[k] + zrt::kSphereSlotBias : fr[k];
            if (ra != full_a || rb != fb[k] || sph != (fr[k] < -zrt::kSphereSlotBias))
              return bad("a leaf record's refs differ", o, i, k);
          }
          ++*n_checked;
        }
      }
    }
    return ZRT_OK;
  }
  ZRT_CATCH_ALL
}

int zrt_debug_division(uint64_t n, uint64_t* counts, uint32_t device) {
  if (!counts) return fail(ZRT_E_INVALID, "null argument");
  int rc = zrt::check_device(int(device));
  if (rc) return rc;
  try {
    HIPCHK(hipSetDevice(int(device)));
    zrt::DevBuf<unsigned long long> d;
    d.alloc(5);
    HIPCHK(hipMemset(d.p, 0, 5 * sizeof(unsigned long long)));
    hipLaunchKernelGGL(zrt::debug_division_kernel, dim3(8192), dim3(256), 0, 0, n, d.p);
    HIPCHK(hipGetLastError());
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(counts, d.p, 5 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return ZRT_OK;
  }
  ZRT_CATCH_ALL
}

int zrt_debug_rng(uint32_t prng, uint64_t key, uint64_t* out, uint32_t n, uint32_t device) {
  if (!out) return fail(ZRT_E_INVALID, "null argument");
  int rc = zrt::check_device(int(device));
  if (rc) return rc;
  try {
    HIPCHK(hipSetDevice(int(device)));
    zrt::DevBuf<unsigned long long> d;
    d.alloc(n);
    if (prng == ZRT_PRNG_XOSHIRO256)
      hipLaunchKernelGGL(zrt::debug_rng_kernel<ZRT_PRNG_XOSHIRO256>, dim3(1), dim3(64), 0, 0, key, d.p, n);
    else
      hipLaunchKernelGGL(zrt::debug_rng_kernel<ZRT_PRNG_XOROSHIRO128>, dim3(1), dim3(64), 0, 0, key, d.p, n);
    HIPCHK(hipGetLastError());
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(out, d.p, n * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return ZRT_OK;
  }
  ZRT_CATCH_ALL
}

}  // extern "C"
